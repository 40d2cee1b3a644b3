// libm_exact.h — device (and host) restatements of the three glibc 2.35 libm
// routines the LoRa demodulator's results depend on, written so that the
// GPU reproduces the reference CPU path bit for bit:
//
//   * sincosf  — the reference's per-sample CFO rotation
//                (/root/reference/src/phy/LoRaDemod.cpp:153-155,
//                 src/phy/phy.cpp:220-222; GCC merges the cos/sin pair into one
//                 sincosf call).  glibc 2.35 implements it in double
//                 precision (sysdeps/ieee754/flt-32/s_sincosf.{c,h}) and, on
//                 any x86-64 host with FMA/AVX2, dispatches to the *_fma
//                 variant in which every a + b*c of the polynomial and of the
//                 fast range reduction is a fused multiply-add.
//   * atan2f   — std::arg() of the strongest sync-symbol bin in the CFO
//                estimate (LoRaDemod.cpp:127, phy.cpp:136).  glibc 2.35 uses
//                the fdlibm single-precision algorithm (e_atan2f.c, s_atanf.c),
//                plain float arithmetic, no FMA.
//   * cabsf    — std::abs() of the bins adjacent to the peak in the
//                fractional-index interpolation (LoRaDetector.hpp:66-67):
//                glibc 2.35's hypotf is sqrt((double)x*x + (double)y*y)
//                rounded to float.
//
// The constants below are the published values of those algorithms; the
// sincosf tables were additionally read back from this image's libm.so.6
// .rodata.  tests/cpp/libm_exact_check.cpp compares every function against
// the host glibc over all 2^32 float inputs (sincosf) or >10^8 inputs
// (atan2f); see DESIGN.md §"Transcendentals".
//
// Everything here must be compiled with -ffp-contract=off: the only fused
// operations are the explicit fma() calls.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define LPHY_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#include <string.h>
#define LPHY_HD static inline
#endif

namespace lphy_libm {

LPHY_HD uint32_t f2u(float x) {
#if defined(__HIPCC__)
    return __builtin_bit_cast(uint32_t, x);
#else
    uint32_t u; memcpy(&u, &x, 4); return u;
#endif
}
LPHY_HD float u2f(uint32_t u) {
#if defined(__HIPCC__)
    return __builtin_bit_cast(float, u);
#else
    float x; memcpy(&x, &u, 4); return x;
#endif
}
LPHY_HD double dfma(double a, double b, double c) {
#if defined(__HIPCC__)
    return __builtin_fma(a, b, c);
#else
    return fma(a, b, c);
#endif
}

// ---------------------------------------------------------------------------
// sincosf
// ---------------------------------------------------------------------------
// Polynomial coefficient set; set 1 is set 0 with the cos/sin signs folded in
// for odd quadrant pairs.  Order of fields follows the glibc table layout.
struct SinCosCoef {
    double c0, c1, s1, c2, s2, c3, s3, c4;
};

LPHY_HD SinCosCoef sincos_coef(int set) {
    SinCosCoef p;
    const double C1 = -0x1.ffffffd0c621cp-2, S1 = -0x1.555545995a603p-3;
    const double C2 = 0x1.55553e1068f19p-5, S2 = 0x1.1107605230bc4p-7;
    const double C3 = -0x1.6c087e89a359dp-10, S3 = -0x1.994eb3774cf24p-13;
    const double C4 = 0x1.99343027bf8c3p-16;
    if (set == 0) {
        p.c0 = 1.0; p.c1 = C1; p.c2 = C2; p.c3 = C3; p.c4 = C4;
    } else {
        p.c0 = -1.0; p.c1 = -C1; p.c2 = -C2; p.c3 = -C3; p.c4 = -C4;
    }
    p.s1 = S1; p.s2 = S2; p.s3 = S3;
    return p;
}

// top 12 bits of |x| (sign stripped): exponent + 3 mantissa bits
LPHY_HD uint32_t top12(float x) { return (f2u(x) >> 20) & 0x7ff; }

// Both polynomials on the reduced argument; n&1 swaps the roles.
LPHY_HD void sincos_poly(double x, double x2, const SinCosCoef& p, int n,
                         float* sinp, float* cosp) {
    double x4 = x2 * x2;
    double x3 = x2 * x;
    double c2 = dfma(x2, p.c4, p.c3);
    double s1 = dfma(x2, p.s3, p.s2);
    double c1 = dfma(x2, p.c1, p.c0);
    double x5 = x3 * x2;
    double x6 = x4 * x2;
    double s = dfma(x3, p.s1, x);
    double c = dfma(x4, p.c2, c1);
    float sv = (float)dfma(x5, s1, s);
    float cv = (float)dfma(x6, c2, c);
    if (n & 1) { *sinp = cv; *cosp = sv; }
    else       { *sinp = sv; *cosp = cv; }
}

// 2/pi as 24 overlapping 32-bit windows (Payne-Hanek table).
LPHY_HD uint32_t inv_pio4_table(int i) {
    // static: one read-only table (constant memory on the device), not a
    // per-call private array (scratch) that every inlined copy would fill
    static constexpr uint32_t t[24] = {
        0xa2u,       0xa2f9u,     0xa2f983u,   0xa2f9836eu,
        0xf9836e4eu, 0x836e4e44u, 0x6e4e4415u, 0x4e441529u,
        0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u,
        0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u,
        0x34ddc0dbu, 0xddc0db62u, 0xc0db6295u, 0xdb629599u,
        0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u};
    return t[i];
}
// The same windows without a memory access: window i is the 32 bits of the
// 192-bit string W0:W1:W2 (the table's 24 bytes, big-endian) that end at
// byte i, i.e. the low word of (W0:W1:W2) >> 8 (23 - i).  On the device a
// table load is a global load whose wait (vmcnt) also waits for every
// older vector-memory operation of the wave - in the fused kernels the next
// unit's LDS-DMA - and at the low occupancy of k_post's exact re-runs each
// costs a memory round trip.  Checked against the table for every i
// (tests/test_cpu_checks.py via lphy_oracle / libm_exact_check).
LPHY_HD uint32_t inv_pio4_shift(int i) {
    const uint64_t W0 = 0xa2f9836e4e441529ull, W1 = 0xfc2757d1f534ddc0ull, W2 = 0xdb6295993c439041ull;
    const int s = 8 * (23 - i);  // 0 .. 184
    const int k = s >> 6, r = s & 63;
    const uint64_t lo = k == 0 ? W2 : (k == 1 ? W1 : W0);
    const uint64_t hi = k == 0 ? W1 : (k == 1 ? W0 : 0ull);
    const uint64_t v = r == 0 ? lo : ((lo >> r) | (hi << (64 - r)));
    return (uint32_t)v;
}
LPHY_HD uint32_t inv_pio4(int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    return inv_pio4_shift(i);
#else
    return inv_pio4_table(i);
#endif
}

// Large |y| (>= 120) and Inf/NaN: glibc's Payne-Hanek path (reduce_large).
LPHY_HD void sincosf_large(float y, float* sinp, float* cosp) {
    const uint32_t T_INF = 0x7f8;                  // top12(INFINITY)
    const double pi63 = 0x1.921FB54442D18p-62;     // 2pi * 2^-64
    if (top12(y) >= T_INF) {
        float nanv = y - y;
        *sinp = nanv; *cosp = nanv;
        return;
    }
    uint32_t xi = f2u(y);
    int sign = (int)(xi >> 31);
    int idx = (int)((xi >> 26) & 15);
    int shift = (int)((xi >> 23) & 7);
    uint32_t m = (xi & 0xffffffu) | 0x800000u;
    m <<= shift;
    uint64_t res0 = (uint64_t)(uint32_t)(m * inv_pio4(idx));
    uint64_t res1 = (uint64_t)m * inv_pio4(idx + 4);
    uint64_t res2 = (uint64_t)m * inv_pio4(idx + 8);
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    uint64_t nq = (res0 + (1ULL << 61)) >> 62;
    res0 -= nq << 62;
    double xr = (double)(int64_t)res0 * pi63;
    int n = (int)nq;
    int q = (n + sign) & 3;
    double s = (q == 1 || q == 2) ? -1.0 : 1.0;
    sincos_poly(xr * s, xr * xr, sincos_coef(((n + sign) & 2) ? 1 : 0), n, sinp, cosp);
}

// sincosf(y) exactly as glibc 2.35's FMA variant.  |y| < 120 (every CFO
// rotation angle in practice) runs one straight-line path:
//  * glibc's |y| < pi/4 branch is the n = 0 case of its fast reduction
//    (n = 0, x - 0*hpi = x exactly), so it needs no branch of its own;
//  * the second coefficient table is the first with the cos-polynomial
//    coefficients negated, i.e. an exact negation of the cos result;
//  * the quadrant sign s multiplies an odd polynomial: exact negation.
// |y| < 2^-12 returns (y, 1) as glibc does; |y| >= 120 takes sincosf_large.
// True when sincosf_fast is not valid for y (|y| >= 120, Inf, NaN).
LPHY_HD bool sincosf_needs_large(float y) { return top12(y) >= 0x42f; }

// The |y| < 120 path alone (result meaningless when sincosf_needs_large(y)).
// glibc's tiny-argument shortcut (|y| < 2^-12 -> (y, 1)) is not needed: the
// polynomial rounds to the same floats for every such input except y = -0,
// whose sine it returns as +0 (exhaustive check, tests/cpp/libm_exact_check);
// the y == 0 select restores that sign.
LPHY_HD void sincosf_fast(float y, float* sinp, float* cosp) {
    const double S1 = -0x1.555545995a603p-3, S2 = 0x1.1107605230bc4p-7,
                 S3 = -0x1.994eb3774cf24p-13;
    const double C1 = -0x1.ffffffd0c621cp-2, C2 = 0x1.55553e1068f19p-5,
                 C3 = -0x1.6c087e89a359dp-10, C4 = 0x1.99343027bf8c3p-16;
    const double x = (double)y;
    const double r = x * 0x1.45F306DC9C883p+23;            // x * 2^24 * 2/pi
    const int n = ((int32_t)r + 0x800000) >> 24;
    const double xr = dfma(-(double)n, 0x1.921FB54442D18p0, x);  // x - n*pi/2
    const double x2 = xr * xr;
    // sin polynomial
    const double x3 = x2 * xr;
    const double s1 = dfma(x2, S3, S2);
    const double s = dfma(x3, S1, xr);
    const double x5 = x3 * x2;
    const float sv0 = (float)dfma(x5, s1, s);
    // cos polynomial
    const double x4 = x2 * x2;
    const double c2 = dfma(x2, C4, C3);
    const double c1 = dfma(x2, C1, 1.0);
    const double x6 = x4 * x2;
    const double c = dfma(x4, C2, c1);
    const float cv0 = (float)dfma(x6, c2, c);
    // quadrant: sin sign flips for n&3 in {1,2} (bit 1 of n+1), the cos
    // table flips for n&3 in {2,3} (bit 1 of n); odd n swaps the pair
    const uint32_t sflip = ((uint32_t)(n + 1) & 2u) << 30;
    const uint32_t cflip = ((uint32_t)n & 2u) << 30;
    const float sv = u2f(f2u(sv0) ^ sflip);
    const float cv = u2f(f2u(cv0) ^ cflip);
    const bool swap = (n & 1) != 0;
    *sinp = y == 0.0f ? y : (swap ? cv : sv);
    *cosp = swap ? sv : cv;
}

LPHY_HD void sincosf_exact(float y, float* sinp, float* cosp) {
    if (sincosf_needs_large(y)) { sincosf_large(y, sinp, cosp); return; }
    sincosf_fast(y, sinp, cosp);
}

// ---------------------------------------------------------------------------
// atan2f (fdlibm single precision)
// ---------------------------------------------------------------------------
LPHY_HD float atanf_exact(float x) {
    // atanhi / atanlo of fdlibm as constants chosen in the argument reduction
    // (no table: on the GPU an indexed load from a constant table waits for
    // every load in flight, the fused kernel's prefetched samples included)
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f,
                aT2 = 1.4285714924e-01f, aT3 = -1.1111110449e-01f,
                aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f,
                aT8 = 4.9768779427e-02f, aT9 = -3.6531571299e-02f,
                aT10 = 1.6285819933e-02f;
    const float hi3 = 1.5707962513e+00f, lo3 = 7.5497894159e-08f;
    int32_t hx = (int32_t)f2u(x);
    int32_t ix = hx & 0x7fffffff;
    bool red;
    float hi = 0.0f, lo = 0.0f;
    if (ix >= 0x4c000000) {
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? hi3 + lo3 : -hi3 - lo3;
    }
    if (ix < 0x3ee00000) {
        if (ix < 0x31000000) return x;
        red = false;
    } else {
        red = true;
        x = u2f(f2u(x) & 0x7fffffffu);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) {
                hi = 4.6364760399e-01f; lo = 5.0121582440e-09f;
                x = (2.0f * x - 1.0f) / (2.0f + x);
            } else {
                hi = 7.8539812565e-01f; lo = 3.7748947079e-08f;
                x = (x - 1.0f) / (x + 1.0f);
            }
        } else {
            if (ix < 0x401c0000) {
                hi = 9.8279368877e-01f; lo = 3.4473217170e-08f;
                x = (x - 1.5f) / (1.0f + 1.5f * x);
            } else {
                hi = hi3; lo = lo3;
                x = -1.0f / x;
            }
        }
    }
    float z = x * x;
    float w = z * z;
    float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (!red) return x - x * (s1 + s2);
    z = hi - ((x * (s1 + s2) - lo) - x);
    return hx < 0 ? -z : z;
}

LPHY_HD float atan2f_exact(float y, float x) {
    const float tiny = 1.0e-30f;
    const float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    int32_t hx = (int32_t)f2u(x), ix = hx & 0x7fffffff;
    int32_t hy = (int32_t)f2u(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return atanf_exact(y);
    int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        switch (m) {
            case 0: case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    int k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = atanf_exact(u2f(f2u(y / x) & 0x7fffffffu));
    switch (m) {
        case 0: return z;
        case 1: return u2f(f2u(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// cabsf as glibc 2.35 computes it for finite inputs.
LPHY_HD float cabsf_exact(float re, float im) {
    double a = (double)re, b = (double)im;
#if defined(__HIPCC__)
    return (float)__builtin_sqrt(a * a + b * b);
#else
    return (float)sqrt(a * a + b * b);
#endif
}

// logf as glibc 2.35 computes it (the table-driven double-precision
// evaluation that replaced fdlibm's in glibc 2.28): x = 2^k * z with z in
// [0x3f330000, 2*0x3f330000), 16 sub-intervals each with a tabulated
// 1/c and log(c), then a degree-3 polynomial in r = z/c - 1.  Only normal
// positive inputs reach it from the detector; the special cases follow
// glibc for completeness.  CONTRACT selects whether the double-precision
// multiply-adds are fused (x86-64 glibc builds are not; see the host check).
template <bool CONTRACT>
LPHY_HD double logf_eval(uint32_t ix) {
    constexpr uint32_t OFF = 0x3f330000u;
    constexpr double Ln2 = 0x1.62e42fefa39efp-1;
    constexpr double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2,
                     A2 = -0x1.ffffef20a4123p-2;
    constexpr double invc_t[16] = {
        0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010b0p+0,
        0x1.3c995b0b80385p+0, 0x1.30d190c8864a5p+0, 0x1.25e227b0b8ea0p+0,
        0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0, 0x1.0953f419900a7p+0,
        0x1.0000000000000p+0, 0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aa0p-1,
        0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1,
        0x1.767dcf5534862p-1};
    constexpr double logc_t[16] = {
        -0x1.57bf7808caadep-2, -0x1.2bef0a7c06ddbp-2, -0x1.01eae7f513a67p-2,
        -0x1.b31d8a68224e9p-3, -0x1.6574f0ac07758p-3, -0x1.1aa2bc79c8100p-3,
        -0x1.a4e76ce8c0e5ep-4, -0x1.1973c5a611cccp-4, -0x1.252f438e10c1ep-5,
        0x0.0p+0,              0x1.aa5aa5df25984p-5,  0x1.c5e53aa362eb4p-4,
        0x1.526e57720db08p-3,  0x1.bc2860d224770p-3,  0x1.1058bc8a07ee1p-2,
        0x1.4043057b6ee09p-2};
    uint32_t tmp = ix - OFF;
    int i = (int)((tmp >> 19) % 16u);
    int k = (int32_t)tmp >> 23;
    uint32_t iz = ix - (tmp & 0xff800000u);
    double invc = invc_t[i], logc = logc_t[i];
    double z = (double)u2f(iz);
    double r, y0, y;
    if (CONTRACT) {
        r = dfma(z, invc, -1.0);
        y0 = dfma((double)k, Ln2, logc);
        double r2 = r * r;
        y = dfma(A1, r, A2);
        y = dfma(A0, r2, y);
        y = dfma(y, r2, y0 + r);
    } else {
        r = z * invc - 1.0;
        y0 = logc + (double)k * Ln2;
        double r2 = r * r;
        y = A1 * r + A2;
        y = A0 * r2 + y;
        y = y * r2 + (y0 + r);
    }
    return y;
}

template <bool CONTRACT>
LPHY_HD float logf_exact_t(float x) {
    uint32_t ix = f2u(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2u == 0u) return u2f(0xff800000u);             // -inf
        if (ix == 0x7f800000u) return x;                        // +inf
        if ((ix & 0x80000000u) || ix * 2u >= 0xff000000u) return u2f(0x7fc00000u);
        ix = f2u(x * 0x1p23f);
        ix -= 23u << 23;
    }
    return (float)logf_eval<CONTRACT>(ix);
}

LPHY_HD float logf_exact(float x) { return logf_exact_t<false>(x); }

// log10f as glibc 2.35 computes it: fdlibm's e_log10f.c, which splits
// x = 2^k * m (m in [1,2), or [0.5,1) when k < 0 so the 2^k term is
// exact), then z = k*log10_2lo + ivln10*logf(m); result z + k*log10_2hi
// (all single precision).  Used by the osr>1 estimator's detector power,
// LoRaDetector.hpp:64 (20*log10f(sqrtf(maxValue))).
template <bool CONTRACT>
LPHY_HD float log10f_exact_t(float x) {
    const float two25 = 3.3554432000e+07f;
    const float ivln10 = u2f(0x3ede5bd9u);
    const float log10_2hi = u2f(0x3e9a2080u);
    const float log10_2lo = u2f(0x355427dbu);
    int32_t hx = (int32_t)f2u(x);
    int32_t k = 0;
    if (hx < 0x00800000) {
        if ((hx & 0x7fffffff) == 0) return u2f(0xff800000u);
        if (hx < 0) return u2f(0x7fc00000u);
        k -= 25;
        x *= two25;
        hx = (int32_t)f2u(x);
    }
    if (hx >= 0x7f800000) return x + x;
    k += (hx >> 23) - 127;
    int32_t i = (int32_t)(((uint32_t)k & 0x80000000u) >> 31);
    hx = (hx & 0x007fffff) | ((0x7f - i) << 23);
    float y = (float)(k + i);
    x = u2f((uint32_t)hx);
    float lx = logf_exact_t<CONTRACT>(x);
    float z;
    if (CONTRACT) {
        z = __builtin_fmaf(y, log10_2lo, ivln10 * lx);
        return __builtin_fmaf(y, log10_2hi, z);
    }
    z = y * log10_2lo + ivln10 * lx;
    return z + y * log10_2hi;
}

LPHY_HD float log10f_exact(float x) { return log10f_exact_t<false>(x); }

}  // namespace lphy_libm
