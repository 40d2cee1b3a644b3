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
    LPHY_F_DEBUG_LOCKFAIL = 1024u, // k_wave2s: every third exchange-buffer
                                   // acquisition fails and the others try
                                   // once, so the fail-safe path (the unit left
                                   // to the exact re-run) runs
                                   // (tests/test_gpu_wave2s.py)
};
constexpr unsigned kTestFlags =
    LPHY_F_EXACT_ROTATION | 128u | LPHY_F_SCAN_FIRST | LPHY_F_DEBUG_RECHECK | LPHY_F_DEBUG_LOCKFAIL;

// Test build only: LPHY_WAVE=1 forces k_wave, LPHY_WAVE=2s k_wave2s (SF 9-10,
// frames of at least a unit) on the fused SF 9-10 path, for comparisons of
// the two kernels.  -1: the library's own choice.
inline int lphy_test_wave_kind() {
#ifdef LPHY_TEST_PATHS
    static const int v = [] {
        const char* e = std::getenv("LPHY_WAVE");
        if (!e) return -1;
        if (e[0] == '1') return 1;
        if (e[0] == '2' && e[1] == 's') return 2;
        return -1;
    }();
    return v;
#else
    return -1;
#endif
}

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
