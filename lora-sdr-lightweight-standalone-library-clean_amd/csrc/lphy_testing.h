// lphy_testing.h — comparison / test paths of lphy_hip_demod_batch, not part
// of the public C ABI (include/lphy_hip.h).  The flag bits are accepted only
// by the test-only build (Makefile `test`: lib/test/liblphy_hip.so, compiled
// with -DLPHY_TEST_PATHS and -DLPHY_DEBUG_BOUNDS); the product library
// rejects them with -EINVAL.  The kernels are the same code: the flags only
// select schedules the tests use as references.
//
// The same holds for the launch overrides below: only the test build reads
// them from the environment; the product library's dispatch depends on the
// call's arguments and lphy_hip_ctx_set_fused_min_frames alone.
#pragma once

#include <cstdlib>

enum lphy_test_flags {
    LPHY_F_EXACT_ROTATION = 64u,   // every symbol with the reference's per-sample
                                   // sincos rotation instead of the certified
                                   // per-frame table (tests/test_gpu_fast_rotation.py)
    LPHY_F_SCAN_FIRST = 256u,      // modes 1/2: whole-frame max-abs pre-scan
                                   // instead of the speculative normalisation
                                   // (tests/test_gpu_spec.py)
    LPHY_F_DEBUG_RECHECK = 512u,   // separate launches: every estimated frame
                                   // marked "has open symbols" first; fused
                                   // kernels: every symbol left to k_post's
                                   // exact re-run (tests/test_gpu_concurrency.py)
    LPHY_F_FRAMES_KERNEL = 1024u,  // SF 7-10: k_frames where k_wave would run
                                   // (the matrix-core symbol tiles' tests,
                                   // tests/test_gpu_certificate.py)
};
constexpr unsigned kTestFlags =
    LPHY_F_EXACT_ROTATION | 128u | LPHY_F_SCAN_FIRST | LPHY_F_DEBUG_RECHECK | LPHY_F_FRAMES_KERNEL;

// Test build only: LPHY_FUSED_MIN_FRAMES sets the process default of the
// smallest batch the fused kernels take (the lora_phy:: probes run once with
// it at 0 through this build).  -1: the measured per-SF crossover.
inline long lphy_test_fused_min_frames() {
#ifdef LPHY_TEST_PATHS
    static const long v = [] {
        const char* e = std::getenv("LPHY_FUSED_MIN_FRAMES");
        return e ? std::atol(e) : -1L;
    }();
    return v;
#else
    return -1L;
#endif
}
