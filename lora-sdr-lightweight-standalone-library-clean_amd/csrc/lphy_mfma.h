// Symbol-unit transform on the matrix cores (SF 7, modes 1/2, k_frames'
// symbol-only tiles).  Included by lphy_kernels.h after lphy_fft.h.
//
// A symbol unit only needs argmax |X|^2, and its winner is certified
// against KISS's exact result (lphy_kernels.h, "Certified fast rotation"),
// so its transform need not follow KISS's arithmetic: only its deviation
// from the exact DFT has to be bounded.  Here the 128-point DFT of a tile's
// 8 symbols is two matrix products in f16 with f32 accumulation,
// 128 = 16 x 8 (n = 8 n1 + n2, k = k1 + 16 k2):
//   stage 1  P[k1][n2] = sum_n1 y[8 n1 + n2] W16^(n1 k1)   (MFMA, y as A)
//   twiddle  P[k1][n2] *= W128^(n2 k1)                      (VALU, f32)
//   stage 2  X[k1 + 16 k2] = sum_n2 P[k1][n2] W8^(n2 k2)    (MFMA, P as B)
// v_mfma_f32_16x16x32_f16 on complex data made real (K = 32 = 16 complex
// inputs, one MFMA for the real and one for the imaginary part of the
// output), two symbols per MFMA tile (rows (s, n2); stage 2's A is
// block-diagonal over s).  Stage 1's accumulator has its column (k1) on the
// lane and its rows in the registers, so it is stage 2's B operand in place
// (MI355X guide, "An accumulator tile as the next MFMA's operand"); the
// k order of both operands is permuted to match (k = 8q + j <-> (row 4q +
// j/2, re/im j&1)).  Per 8-symbol tile and lane: 16 MFMA, 32 f16 packs and
// 4 twiddle products, against ~176 packed-f32 butterfly instructions of the
// KISS-order transform (fft_tile TRIV).  The samples enter from the lanes'
// KISS first-pass registers through the tile's LDS slots, and the bins go
// back to bin_of order the same way, so staging, the keyed top two and the
// certificate are unchanged.
//
// Error against the exact DFT of the staged samples y (RNE f16 conversion
// <= 2^-11 relative per component, twiddle constants in f16 <= 2^-12
// absolute, products exact in f32, f32 sums and the f32 twiddle product
// O(u)): stage 1 output |dC| <= (sqrt2 2^-11 + 2^-11) sum|y| over its 16
// inputs = 1.18e-3 of that sum; stage 2 adds the same factor of
// sum_n2 |C| <= |y|_1, so |dX_k| <= 2.36e-3 |y|_1 <= 2.36e-3 A (A of
// cert_bound).  kMfmaExtra charges 3 * 2^14 u = 2.93e-3 (slack 1.24).
// tools/ubench/mfma_dft.py measured max |dX| / |y|_1 = 3.1e-4.
#pragma once

#include <hip/hip_runtime.h>

namespace {

typedef _Float16 lphy_h8 __attribute__((ext_vector_type(8)));
typedef float lphy_f4 __attribute__((ext_vector_type(4)));

constexpr float kMfmaExtra = 49152.0f;  // u-multiples of A (see above)

// per-lane operand constants (96 B), one table per workgroup in LDS
struct MfmaLane {
    lphy_h8 b1r, b1i, a2r, a2i;  // stage-1 B (Re, Im output), stage-2 A (Re, Im output)
    cf32 t[4];                   // twiddles of the lane's four stage-1 rows
};
static_assert(sizeof(MfmaLane) == 96, "six 16-byte parts");

// The table in LDS as six planes of 16-byte parts, plane k holding part k of
// every lane (lane stride 16 B: the ds_read_b128 lane groups are
// conflict-free, where a 96-byte struct stride is not).
struct MfmaTable {
    uint4 part[6][64];
    __device__ void put(int lane, const MfmaLane& K) {
        uint4 u[6];
        __builtin_memcpy(u, &K, sizeof K);
#pragma unroll
        for (int k = 0; k < 6; ++k) part[k][lane] = u[k];
    }
    __device__ MfmaLane get(int lane) const {
        uint4 u[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) u[k] = part[k][lane];
        MfmaLane K;
        __builtin_memcpy(&K, u, sizeof K);
        return K;
    }
};

// SF 7 (128 = 16 x 8, two symbols per MFMA tile) and SF 8 (256 = 16 x 16,
// one symbol per tile); four MFMA tiles per wave either way.
template <int SF>
struct MfmaUse {
    static constexpr bool value = SF == 7 || SF == 8;
};

// lane l's constants from the KISS twiddle table tw[k] = e^{-2 pi i k / N}.
// n = N2 n1 + n2, N2 = N / 16; stage-1 rows r = (symbol r / N2, n2 = r % N2)
template <int SF>
__device__ __forceinline__ MfmaLane mfma_lane_consts(const cf32* tw, int l) {
    constexpr int N = 1 << SF, N2 = N / 16;
    MfmaLane K;
    const int col = l & 15, q = l >> 4, row = l & 15;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = j & 1;
        const cf32 w = tw[(N2 * (q + 4 * (j >> 1)) * col) & (N - 1)];  // W16^(n1 k1), n1 = q + 4 (j/2)
        K.b1r[j] = (_Float16)(c == 0 ? w.x : -w.y);
        K.b1i[j] = (_Float16)(c == 0 ? w.y : w.x);
        const int r = 4 * q + (j >> 1), s = r / N2, n2 = r % N2, sp = row / N2, k2 = row % N2;
        const cf32 v = tw[(16 * n2 * k2) & (N - 1)];  // W_N2^(n2 k2)
        const bool on = s == sp;                      // block-diagonal over the tile's symbols
        K.a2r[j] = (_Float16)(on ? (c == 0 ? v.x : -v.y) : 0.0f);
        K.a2i[j] = (_Float16)(on ? (c == 0 ? v.y : v.x) : 0.0f);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) K.t[i] = tw[(((4 * q + i) % N2) * col) & (N - 1)];  // W_N^(n2 k1)
    return K;
}

// LDS image of the wave's 8 symbols for the two transposes (the wave's own
// 1,024-entry slot region; Geo's swizzle is not used).  Address of sample /
// bin p of local symbol s, from the bits s0 s1 s2 and p0 .. p6:
//     bank bits   b0 = p0, b1 = p2, b2 = p1 ^ p3, b3 = s0 ^ p3
//     L(s, p) = b0 + 2 b1 + 4 b2 + 8 b3 + 16 p3 + 32 (p >> 4) + 256 (s >> 1)
// The merged ds_read2 / ds_write2 forms the compiler emits serve 16-lane
// groups on 16 complex banks (b0..b3).  The lanes of a group vary
// {s0, p0, p2, p3} in the first-pass stores, {s0, p0, p1, p2} in the MFMA
// operand reads and the bin_of reads, {p0, p1, p2, p3} in the bin stores,
// and each set maps onto b0..b3 with rank 4: no bank conflict anywhere.
// Every access is a per-lane base plus a compile-time offset (the
// instruction's immediate); where an XOR pairs a lane bit with a
// compile-time bit (p1 in the stores, p3 in the bin_of reads) there are two
// bases, one per value of that bit.
__host__ __device__ constexpr int mfma_lds(int s, int p) {
    const int p0 = p & 1, p1 = (p >> 1) & 1, p2 = (p >> 2) & 1, p3 = (p >> 3) & 1, s0 = s & 1;
    return p0 + 2 * p2 + 4 * (p1 ^ p3) + 8 * (s0 ^ p3) + 16 * p3 + 32 * (p >> 4) + 256 * (s >> 1);
}

template <int SF>
struct MfmaMap {
    // first_pass_index(e, lam) = lp(lam) | ep(e), lp on bits 0, 2, 3 and ep
    // on bits 1, 4, 5, 6 (checked below)
    static constexpr int lp(int lam) { return first_pass_index<SF>(0, lam); }
    static constexpr int ep(int e) { return first_pass_index<SF>(e, 0); }
    static constexpr bool layout_ok() {
        for (int lam = 0; lam < 8; ++lam) {
            if ((lp(lam) & ~0xD) != 0) return false;
            for (int e = 0; e < 16; ++e)
                if ((ep(e) & ~0x72) != 0 || first_pass_index<SF>(e, lam) != (lp(lam) | ep(e)) ||
                    bin_of<SF>(e, lam) != lam + 8 * e)
                    return false;
        }
        bool seen[1024] = {};
        for (int s = 0; s < 8; ++s)
            for (int p = 0; p < 128; ++p) {
                const int a = mfma_lds(s, p);
                if (a < 0 || a >= 1024 || seen[a]) return false;
                seen[a] = true;
            }
        return true;
    }
};

// The wave's 8 symbols (slots w0 .. w0+7 of `lds`), held in KISS first-pass
// order (element e of lane lam of slot w0 + lane/8 = sample
// first_pass_index(e, lam)), to their bins in bin_of order: v[e] =
// X[bin_of(e, lam)].  Every lane of the wave calls it (wave-uniform control
// flow: the MFMAs read all 64 lanes).
template <int SF>
__device__ __forceinline__ void mfma_symbols7(cf32 (&v)[16], cf32* lds, int w0, const MfmaTable& kt, int lane) {
    using G = Geo<SF>;
    using M = MfmaMap<SF>;
    static_assert(G::E == 16 && G::LPS == 8 && G::SSTRIDE == 128, "the 16 x 8 MFMA form is SF 7's");
    static_assert(M::layout_ok(), "index splits and the LDS image assumed below");
    cf32* wl = lds + w0 * G::SSTRIDE;  // the wave's 1,024 entries
    const int sl = lane >> 3, lam = lane & 7;
    {
        cf32* pa0 = wl + mfma_lds(sl, M::lp(lam));      // stores with ep bit 1 clear
        cf32* pa1 = wl + mfma_lds(sl, M::lp(lam) | 2);  // ... and set
#pragma unroll
        for (int e = 0; e < G::E; ++e) {
            cf32* pa = (M::ep(e) & 2) ? pa1 : pa0;
            pa[32 * (M::ep(e) >> 4)] = v[e];
        }
    }
    team_sync<SF>();
    const MfmaLane K = kt.get(lane);
    const int row = lane & 15, q = lane >> 4;
    const lphy_f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
    lphy_f4 xr[4], xi[4];
    // stage-1 A: lane (row = (r, n2), q) holds samples n1 = q + 4 jj, i.e.
    // p = 8 (q + 4 jj) + n2, of symbol 2t + r
    const cf32* pb = wl + mfma_lds(row >> 3, 8 * q + (row & 7));
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        lphy_h8 a;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const cf32 y = pb[256 * t + 64 * jj];
            a[2 * jj] = (_Float16)y.x;
            a[2 * jj + 1] = (_Float16)y.y;
        }
        const lphy_f4 cr = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, K.b1r, z, 0, 0, 0);
        const lphy_f4 ci = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, K.b1i, z, 0, 0, 0);
        lphy_h8 b;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float pr = fmaf(cr[i], K.t[i].x, -(ci[i] * K.t[i].y));
            const float pi = fmaf(cr[i], K.t[i].y, ci[i] * K.t[i].x);
            b[2 * i] = (_Float16)pr;
            b[2 * i + 1] = (_Float16)pi;
        }
        xr[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(K.a2r, b, z, 0, 0, 0);
        xi[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(K.a2i, b, z, 0, 0, 0);
    }
    team_sync<SF>();  // every lane's sample reads before the bins overwrite them
    {
        // lane (col, q) holds bins col + 64 (q & 1) + 16 i of symbol 2t + (q >> 1)
        cf32* pc = wl + mfma_lds(q >> 1, (lane & 15) + 64 * (q & 1));
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) pc[256 * t + 32 * i] = cf32{xr[t][i], xi[t][i]};
    }
    team_sync<SF>();
    const cf32* pd0 = wl + mfma_lds(sl, lam);      // bins lam + 8e, e even
    const cf32* pd1 = wl + mfma_lds(sl, lam + 8);  // ... e odd
#pragma unroll
    for (int e = 0; e < G::E; ++e) v[e] = ((e & 1) ? pd1 : pd0)[32 * (e >> 1)];
}


// SF 8: one symbol per MFMA tile (rows n2 = 0..15), stage 2's A full.  The
// plain image L(s, p) = 256 s + p is conflict-free for all four patterns:
// in every 16-lane group the lanes vary p's low four bits (first-pass lp,
// n2, the bin column, bin_of's lam).
template <int SF>
struct MfmaMap8 {
    static constexpr int lp(int lam) { return first_pass_index<SF>(0, lam); }
    static constexpr int ep(int e) { return first_pass_index<SF>(e, 0); }
    static constexpr bool layout_ok() {
        for (int lam = 0; lam < 16; ++lam) {
            if ((lp(lam) & ~0xF) != 0) return false;
            for (int e = 0; e < 16; ++e)
                if ((ep(e) & 0xF) != 0 || first_pass_index<SF>(e, lam) != (lp(lam) | ep(e)) ||
                    bin_of<SF>(e, lam) != lam + 16 * e)
                    return false;
        }
        return true;
    }
};

template <int SF>
__device__ __forceinline__ void mfma_symbols8(cf32 (&v)[16], cf32* lds, int w0, const MfmaTable& kt, int lane) {
    using G = Geo<SF>;
    using M = MfmaMap8<SF>;
    static_assert(G::E == 16 && G::LPS == 16 && G::SSTRIDE == 256, "the 16 x 16 MFMA form is SF 8's");
    static_assert(M::layout_ok(), "index splits assumed by the LDS image");
    cf32* wl = lds + w0 * G::SSTRIDE;  // the wave's 4 x 256 entries
    const int sl = lane >> 4, lam = lane & 15;
    {
        cf32* pa = wl + 256 * sl + M::lp(lam);
#pragma unroll
        for (int e = 0; e < G::E; ++e) pa[M::ep(e)] = v[e];
    }
    team_sync<SF>();
    const MfmaLane K = kt.get(lane);
    const int row = lane & 15, q = lane >> 4;
    const lphy_f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
    lphy_f4 xr[4], xi[4];
    // stage-1 A: lane (row = n2, q) holds samples n1 = q + 4 jj, p = 16 n1 + n2, of symbol t
    const cf32* pb = wl + 16 * q + row;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        lphy_h8 a;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const cf32 y = pb[256 * t + 64 * jj];
            a[2 * jj] = (_Float16)y.x;
            a[2 * jj + 1] = (_Float16)y.y;
        }
        const lphy_f4 cr = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, K.b1r, z, 0, 0, 0);
        const lphy_f4 ci = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, K.b1i, z, 0, 0, 0);
        lphy_h8 b;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float pr = fmaf(cr[i], K.t[i].x, -(ci[i] * K.t[i].y));
            const float pi = fmaf(cr[i], K.t[i].y, ci[i] * K.t[i].x);
            b[2 * i] = (_Float16)pr;
            b[2 * i + 1] = (_Float16)pi;
        }
        xr[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(K.a2r, b, z, 0, 0, 0);
        xi[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(K.a2i, b, z, 0, 0, 0);
    }
    team_sync<SF>();
    {
        // lane (col, q) holds bins col + 16 (4 q + i) of symbol t
        cf32* pc = wl + (lane & 15) + 64 * q;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) pc[256 * t + 16 * i] = cf32{xr[t][i], xi[t][i]};
    }
    team_sync<SF>();
    const cf32* pd = wl + 256 * sl + lam;
#pragma unroll
    for (int e = 0; e < G::E; ++e) v[e] = pd[16 * e];
}

// The wave's symbols (slots w0 .. of `lds`) in KISS first-pass order to their
// bins in bin_of order, on the matrix cores.
template <int SF>
__device__ __forceinline__ void mfma_symbols(cf32 (&v)[16], cf32* lds, int w0, const MfmaTable& kt, int lane) {
    if constexpr (SF == 7) mfma_symbols7<SF>(v, lds, w0, kt, lane);
    else mfma_symbols8<SF>(v, lds, w0, kt, lane);
}

}  // namespace
