// Pins csrc/libm_exact.h against the host glibc libm (the library the
// reference links).  Usage:
//   libm_exact_check sincos <first_u32> <last_u32> [threads]   # float range
//   libm_exact_check atan2 <count> <seed> [threads]            # random pairs
//   libm_exact_check cabs <count> <seed> [threads]
//   libm_exact_check log10 <first_u32> <last_u32> [threads]    # float range
//   libm_exact_check logf <first_u32> <last_u32> [threads]
// Prints "mismatches=<k> checked=<n>" and exits non-zero on any mismatch.
#include "../../lora-sdr-lightweight-standalone-library-clean_amd/csrc/libm_exact.h"

#include <atomic>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

static uint32_t bits(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static float fromb(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }

static bool same(float a, float b) {
    if (a != a && b != b) return true;  // both NaN
    return bits(a) == bits(b);
}

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage\n"); return 2; }
    const char* what = argv[1];
    if (!strcmp(what, "pio4")) {  // the device's shift form of the Payne-Hanek windows == the table, every index
        int bad_w = 0;
        for (int i = 0; i < 24; ++i) bad_w += lphy_libm::inv_pio4_shift(i) != lphy_libm::inv_pio4_table(i);
        printf("mismatches=%d checked=24\n", bad_w);
        return bad_w ? 1 : 0;
    }
    int threads = argc > 4 ? atoi(argv[4]) : 8;
    std::atomic<uint64_t> bad{0}, checked{0};
    std::vector<std::thread> th;
    if (!strcmp(what, "log10") || !strcmp(what, "logf") || !strcmp(what, "log10c")) {
        uint64_t lo = strtoull(argv[2], 0, 0), hi = strtoull(argv[3], 0, 0);
        uint64_t span = hi - lo + 1, per = (span + threads - 1) / threads;
        int which = !strcmp(what, "logf") ? 0 : !strcmp(what, "log10") ? 1 : 2;
        for (int t = 0; t < threads; ++t) {
            th.emplace_back([&, t, which] {
                uint64_t a = lo + t * per, b = std::min(hi + 1, a + per);
                uint64_t nb = 0, n = 0;
                for (uint64_t u = a; u < b; ++u) {
                    float x = fromb((uint32_t)u), g, o;
                    if (which == 0) { g = logf(x); o = lphy_libm::logf_exact(x); }
                    else if (which == 1) { g = log10f(x); o = lphy_libm::log10f_exact(x); }
                    else { g = log10f(x); o = lphy_libm::log10f_exact_t<true>(x); }
                    ++n;
                    if (!same(g, o)) {
                        if (nb < 5) fprintf(stderr, "x=%a glibc=%a ours=%a\n", x, g, o);
                        ++nb;
                    }
                }
                bad += nb; checked += n;
            });
        }
    } else if (!strcmp(what, "sincos")) {
        uint64_t lo = strtoull(argv[2], 0, 0), hi = strtoull(argv[3], 0, 0);
        uint64_t span = hi - lo + 1, per = (span + threads - 1) / threads;
        for (int t = 0; t < threads; ++t) {
            th.emplace_back([&, t] {
                uint64_t a = lo + t * per, b = std::min(hi + 1, a + per);
                uint64_t nb = 0, n = 0;
                for (uint64_t u = a; u < b; ++u) {
                    float x = fromb((uint32_t)u), s0, c0, s1, c1;
                    sincosf(x, &s0, &c0);
                    lphy_libm::sincosf_exact(x, &s1, &c1);
                    ++n;
                    if (!same(s0, s1) || !same(c0, c1)) {
                        if (nb < 5)
                            fprintf(stderr, "x=%a glibc=(%a,%a) ours=(%a,%a)\n",
                                    x, s0, c0, s1, c1);
                        ++nb;
                    }
                }
                bad += nb; checked += n;
            });
        }
    } else {
        uint64_t count = strtoull(argv[2], 0, 0);
        uint64_t seed = strtoull(argv[3], 0, 0);
        bool is_atan = !strcmp(what, "atan2");
        for (int t = 0; t < threads; ++t) {
            th.emplace_back([&, t] {
                std::mt19937_64 rng(seed * 1000003ull + t);
                uint64_t nb = 0, n = 0;
                for (uint64_t i = t; i < count; i += threads) {
                    float y, x;
                    uint64_t r = rng();
                    switch (r & 3) {
                        case 0:  // arbitrary bit patterns
                            y = fromb((uint32_t)(r >> 32));
                            x = fromb((uint32_t)rng());
                            break;
                        default: {  // FFT-bin-like magnitudes
                            std::uniform_real_distribution<float> d(-1.0f, 1.0f);
                            std::uniform_int_distribution<int> e(-30, 30);
                            y = ldexpf(d(rng), e(rng));
                            x = ldexpf(d(rng), e(rng));
                            if ((r >> 8 & 7) == 0) y = 0.0f;
                            if ((r >> 11 & 7) == 0) x = -x;
                        }
                    }
                    float g, o;
                    if (is_atan) { g = atan2f(y, x); o = lphy_libm::atan2f_exact(y, x); }
                    else {
                        if (!std::isfinite(x) || !std::isfinite(y)) continue;
                        g = std::abs(std::complex<float>(y, x));  // glibc cabsf, as the reference's std::abs
                        o = lphy_libm::cabsf_exact(y, x);
                    }
                    ++n;
                    if (!same(g, o)) {
                        if (nb < 5)
                            fprintf(stderr, "y=%a x=%a glibc=%a ours=%a\n", y, x, g, o);
                        ++nb;
                    }
                }
                bad += nb; checked += n;
            });
        }
    }
    for (auto& t : th) t.join();
    printf("mismatches=%llu checked=%llu\n", (unsigned long long)bad.load(),
           (unsigned long long)checked.load());
    return bad.load() ? 1 : 0;
}
