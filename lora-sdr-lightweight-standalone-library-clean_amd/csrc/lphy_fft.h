// lphy_fft.h — register/LDS-tiled KISS-identical forward FFT for gfx950.
//
// The reference transform is KISS FFT's recursive mixed-radix decimation in
// time (/root/reference/include/lora_phy/kissfft.hh:71-185): for N = 2^SF the
// plan is radix 4 for every stage except a trailing radix 2 when SF is odd
// (:78-98), twiddles tw[i] = exp(-2*pi*i/N) from a table (:24-29), and the
// butterflies kf_bfly4 (:164-185) / kf_bfly2 (:155-162).  Bit-exact parity
// with the reference demands the SAME butterflies on the SAME operands, so
// this file re-expresses the recursion as an iterative in-place sweep over
// KISS's output positions and keeps the butterfly arithmetic as is; only the
// data movement is MI355X-shaped:
//
//   * stage l has radix R(l), sub-DFT length M(l) = N / (R(0)...R(l)) and
//     twiddle stride FS(l) = R(0)...R(l-1) = 4^l.  Output position
//     pos = sum_l q_l*M(l); KISS's leaf copies put input index
//     sum_l q_l*FS(l) at that position (a base-4 digit reversal).
//   * stages are grouped into "passes" (innermost first) whose combined
//     radix is <= 16 = E, the complex elements a lane keeps in VGPRs.  Within
//     a pass every butterfly is lane-local; between passes the symbol makes
//     one round trip through LDS (its N complex values, padded).
//   * a symbol is owned by LPS = N/16 consecutive lanes (8 lanes at SF7, one
//     wavefront at SF10, four wavefronts at SF12); a 256-thread workgroup
//     tile carries T = 256/LPS symbols and uses 32 KiB of LDS.
//
// Every floating-point operation below is a plain IEEE op compiled with
// -ffp-contract=off, in the reference's operand order.
#pragma once
#include <hip/hip_runtime.h>

namespace lphy {

constexpr int kTile = 256;  // threads per workgroup tile

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    // GCC's inline complex<float> product: (ac - bd, ad + bc)
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }

template <int SF>
struct Geo {
    static constexpr int N = 1 << SF;
    static constexpr int L = (SF + 1) / 2;          // KISS stages
    static constexpr int E = N < 16 ? N : 16;       // complex per lane
    static constexpr int LPS = N / E;               // lanes per symbol
    static constexpr int T = kTile / LPS;           // symbols per tile
    static constexpr int PAD = N >= 32 ? N / 32 : 0;  // LDS pad (complex) per symbol
    static constexpr int SSTRIDE = N + PAD;         // LDS stride per symbol
    __host__ __device__ static constexpr int R(int l) { return ((SF & 1) && l == L - 1) ? 2 : 4; }
    __host__ __device__ static constexpr int M(int l) {
        int p = 1;
        for (int j = 0; j <= l; ++j) p *= R(j);
        return N / p;
    }
    __host__ __device__ static constexpr int FS(int l) { return 1 << (2 * l); }
    // padded LDS offset of position p inside a symbol (one slot per 32)
    __device__ static __forceinline__ int lds(int p) { return N >= 32 ? p + (p >> 5) : p; }
};

// Pass partition: stages [lo, hi], innermost (largest l) first.
template <int SF>
struct Passes {
    int n = 0;
    int hi[8] = {};
    int lo[8] = {};
    constexpr Passes() {
        using G = Geo<SF>;
        int l = G::L - 1;
        while (l >= 0) {
            int h = l, prod = G::R(l);
            --l;
            while (l >= 0 && prod * G::R(l) <= G::E) { prod *= G::R(l); --l; }
            hi[n] = h;
            lo[n] = l + 1;
            ++n;
        }
    }
};

template <int SF, int HI, int LO>
struct PassGeo {
    using G = Geo<SF>;
    __host__ __device__ static constexpr int Gsz() {
        int p = 1;
        for (int l = LO; l <= HI; ++l) p *= G::R(l);
        return p;
    }
    static constexpr int GS = Gsz();                 // elements per group
    static constexpr int SLOTS = G::E / GS;          // groups per lane
    static constexpr int MH = G::M(HI);              // position weight of the pass's lowest digit
    static constexpr int SPAN = G::M(LO) * G::R(LO); // positions spanned by one group
    // weight of digit l inside a group index (digit HI fastest)
    __host__ __device__ static constexpr int W(int l) {
        int w = 1;
        for (int j = l + 1; j <= HI; ++j) w *= G::R(j);
        return w;
    }
    // digit l of group-local index a
    __host__ __device__ static constexpr int digit(int a, int l) { return (a / W(l)) % G::R(l); }
    // input-index contribution of group-local index a (first pass only)
    __host__ __device__ static constexpr int vidx(int a) {
        int s = 0;
        for (int l = LO; l <= HI; ++l) s += digit(a, l) * G::FS(l);
        return s;
    }
};

// Base-4 digit reversal of `high` over `ndig` digits (leaf permutation of the
// digits that precede the first pass).
__device__ __forceinline__ int rev4(int high, int ndig) {
    int r = 0;
    for (int d = 0; d < ndig; ++d) { r = (r << 2) | (high & 3); high >>= 2; }
    return r;
}

// Position bookkeeping for pass (HI, LO), group slot s of lane lam:
// group g = s*LPS + lam; fixed digits split into the part above the pass
// (g / MH, weight SPAN) and below it (g % MH).
template <int SF, int HI, int LO>
struct Group {
    using G = Geo<SF>;
    using P = PassGeo<SF, HI, LO>;
    __device__ static __forceinline__ int g(int s, int lam) { return s * G::LPS + lam; }
    __device__ static __forceinline__ int low(int s, int lam) { return g(s, lam) % P::MH; }
    __device__ static __forceinline__ int high(int s, int lam) { return g(s, lam) / P::MH; }
    __device__ static __forceinline__ int base(int s, int lam) {
        return high(s, lam) * P::SPAN + low(s, lam);
    }
    // position of element e (= s*GS + a) of the lane
    __device__ static __forceinline__ int pos(int e, int lam) {
        return base(e / P::GS, lam) + (e % P::GS) * P::MH;
    }
};

// All butterflies of one pass on the lane's registers.  v[s*GS + a] is group
// s, group-local index a.
template <int SF, int HI, int LO>
__device__ __forceinline__ void pass_butterflies(float2 (&v)[16], int lam,
                                                 const float2* __restrict__ tw) {
    using G = Geo<SF>;
    using P = PassGeo<SF, HI, LO>;
    using Gr = Group<SF, HI, LO>;
#pragma unroll
    for (int l = HI; l >= LO; --l) {
        const int R = G::R(l), w = P::W(l), fs = G::FS(l);
#pragma unroll
        for (int s = 0; s < P::SLOTS; ++s) {
            const int low = Gr::low(s, lam);
#pragma unroll
            for (int a = 0; a < P::GS; ++a) {
                if (P::digit(a, l) != 0) continue;
                const int k = low + (a % w) * P::MH;
                float2* x = &v[s * P::GS];
                if (R == 2) {
                    const float2 t = cmul(x[a + w], tw[k * fs]);
                    x[a + w] = csub(x[a], t);
                    x[a] = cadd(x[a], t);
                } else {
                    const float2 s0 = cmul(x[a + w], tw[k * fs]);
                    const float2 s1 = cmul(x[a + 2 * w], tw[k * fs * 2]);
                    const float2 s2 = cmul(x[a + 3 * w], tw[k * fs * 3]);
                    const float2 s5 = csub(x[a], s1);
                    const float2 a0 = cadd(x[a], s1);
                    const float2 s3 = cadd(s0, s2);
                    const float2 s4 = csub(s0, s2);
                    const float2 r4 = make_float2(s4.y, -s4.x);
                    x[a + 2 * w] = csub(a0, s3);
                    x[a] = cadd(a0, s3);
                    x[a + w] = cadd(s5, r4);
                    x[a + 3 * w] = csub(s5, r4);
                }
            }
        }
    }
}

// Pass PI of the transform.  `sym` points at the symbol's LDS slot.
//  first pass: read inputs from the natural-order staging copy at index
//              rev4(high) + vidx(a) (KISS's leaf permutation), barrier,
//              compute, write positions;
//  last pass:  leave results in registers for the detector.
template <int SF, int PI, bool LAST>
__device__ __forceinline__ void run_pass(float2 (&v)[16], float2* sym, int lam,
                                         const float2* __restrict__ tw) {
    using G = Geo<SF>;
    constexpr Passes<SF> PS{};
    constexpr int HI = PS.hi[PI], LO = PS.lo[PI];
    using P = PassGeo<SF, HI, LO>;
    using Gr = Group<SF, HI, LO>;
    if (PI == 0) {
#pragma unroll
        for (int s = 0; s < P::SLOTS; ++s) {
            const int ib = rev4(Gr::high(s, lam), LO);
#pragma unroll
            for (int a = 0; a < P::GS; ++a) v[s * P::GS + a] = sym[G::lds(ib + P::vidx(a))];
        }
        __syncthreads();
    } else {
#pragma unroll
        for (int e = 0; e < G::E; ++e) v[e] = sym[G::lds(Gr::pos(e, lam))];
    }
    pass_butterflies<SF, HI, LO>(v, lam, tw);
    if (!LAST) {
#pragma unroll
        for (int e = 0; e < G::E; ++e) sym[G::lds(Gr::pos(e, lam))] = v[e];
        __syncthreads();
    }
}

template <int SF, int PI>
__device__ __forceinline__ void run_passes(float2 (&v)[16], float2* sym, int lam,
                                           const float2* __restrict__ tw) {
    constexpr Passes<SF> PS{};
    if constexpr (PI < PS.n) {
        run_pass<SF, PI, PI == PS.n - 1>(v, sym, lam, tw);
        run_passes<SF, PI + 1>(v, sym, lam, tw);
    }
}

// Full transform of the staged symbol; on return v[e] holds bin
// bin_of<SF>(e, lam).  Must be called by every thread of the tile.
template <int SF>
__device__ __forceinline__ void fft_tile(float2 (&v)[16], float2* sym, int lam,
                                         const float2* __restrict__ tw) {
    run_passes<SF, 0>(v, sym, lam, tw);
}

template <int SF>
__device__ __forceinline__ int bin_of(int e, int lam) {
    constexpr Passes<SF> PS{};
    return Group<SF, PS.hi[PS.n - 1], PS.lo[PS.n - 1]>::pos(e, lam);
}

// Argmax with the detector's semantics (LoRaDetector.hpp:46-58): strict '>'
// from maxValue = 0 scanning upward, i.e. the lowest index among the maxima
// of |X|^2 = re*re + im*im (float, unfused); NaN never wins; all-zero -> 0.
struct ArgMax {
    float v;
    int i;
};

__device__ __forceinline__ ArgMax better(ArgMax a, ArgMax b) {
    const bool take = (b.v > a.v) | ((b.v == a.v) & (b.i < a.i));
    return ArgMax{take ? b.v : a.v, take ? b.i : a.i};
}

template <int SF>
__device__ __forceinline__ ArgMax local_argmax(const float2 (&v)[16], int lam) {
    using G = Geo<SF>;
    ArgMax best{0.0f, 0x7fffffff};
#pragma unroll
    for (int e = 0; e < G::E; ++e) {
        const float m2 = v[e].x * v[e].x + v[e].y * v[e].y;
        const int bi = bin_of<SF>(e, lam);
        const bool take = (m2 > best.v) | ((m2 == best.v) & (bi < best.i));
        best.v = take ? m2 : best.v;
        best.i = take ? bi : best.i;
    }
    return best;
}

// Reduce over the LPS lanes of a symbol.  For LPS <= 64 pure cross-lane;
// above that through `red` (LDS, >= kTile/64 entries).  Every thread of the
// tile must call it.  Returns the winner in every lane of the symbol.
template <int SF>
__device__ __forceinline__ ArgMax symbol_argmax(ArgMax a, ArgMax* red) {
    using G = Geo<SF>;
    constexpr int W = G::LPS < 64 ? G::LPS : 64;
#pragma unroll
    for (int off = W / 2; off >= 1; off >>= 1) {
        ArgMax o;
        o.v = __shfl_xor(a.v, off, 64);
        o.i = __shfl_xor(a.i, off, 64);
        a = better(a, o);
    }
    if constexpr (G::LPS > 64) {
        const int wave = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) red[wave] = a;
        __syncthreads();
        constexpr int WPS = G::LPS / 64;  // waves per symbol
        const int first = (wave / WPS) * WPS;
        ArgMax b = red[first];
#pragma unroll
        for (int w = 1; w < WPS; ++w) b = better(b, red[first + w]);
        __syncthreads();
        a = b;
    }
    if (!(a.v > 0.0f)) a.i = 0;  // nothing beat maxValue = 0
    return a;
}

}  // namespace lphy
