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

// A context's device counters (lphy_hip_ctx::d_counters, kCounters slots),
// each with a slot of its own (the modulator's fallback count
// shared slot 8 with the phase clocks, and the modulator clocks slot 1 with
// the Parseval count):
constexpr int kCtrRecheck = 0;    // symbols re-run exactly (lphy_hip_recheck_count)
constexpr int kCtrParseval = 1;   // test build: symbols the wave kernel certified by Parseval
constexpr int kCtrModSerial = 2;  // frames k_mod_fast gave to its serial walk
constexpr int kCtrClocks = 8;     // timing builds only: 8 phase-clock sums (lphy_hip_phase_cycles)
constexpr int kCounters = 16;

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
