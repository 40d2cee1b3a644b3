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
//     one round trip through LDS (its N complex values, bank-swizzled).
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

// Complex float held as a native 2-vector: adds/subs/scales issue as one
// v_pk_*_f32 each (same IEEE ops per component), the complex product as two
// v_pk_mul_f32 + one sub + one add.  Memory layout = std::complex<float>.
typedef float cf32 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ cf32 cmul(cf32 a, cf32 b) {
    // GCC's inline complex<float> product (ac - bd, ad + bc), unfused, as
    // three packed ops: P = (ac, bc), Q = (bd, ad), P + (-Q.x, Q.y).
    // x - y == x + (-y) and bc + ad == ad + bc exactly in IEEE arithmetic.
    const cf32 P = a * b.xx;
    const cf32 Q = a.yx * b.yy;
    cf32 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(r) : "v"(P), "v"(Q));
    return r;
}
// The reference's std::complex<float> product is GCC's inline formula plus a
// call to __mulsc3 when BOTH parts come out NaN (built without
// -fcx-limited-range): C99 Annex G.5.1's recovery of infinities, which boxes
// an infinite factor to +-1 / +-0, zeroes NaNs of the other factor and
// recomputes times infinity.  cmul_x is that product.  Only the exact paths
// use it directly; the hot paths run cmul and detect the case afterwards
// (see fft_has_nan): a (NaN, NaN) product anywhere reaches at least one bin
// of the transform as NaN, and without one cmul == cmul_x bit for bit.
__device__ __attribute__((noinline)) cf32 cmul_recover(float a, float b, float c, float d) {
    const float ac = a * c, bd = b * d, ad = a * d, bc = b * c;
    cf32 r = cf32{ac - bd, ad + bc};
    bool recalc = false;
    if (__builtin_isinf(a) || __builtin_isinf(b)) {
        a = __builtin_copysignf(__builtin_isinf(a) ? 1.0f : 0.0f, a);
        b = __builtin_copysignf(__builtin_isinf(b) ? 1.0f : 0.0f, b);
        if (__builtin_isnan(c)) c = __builtin_copysignf(0.0f, c);
        if (__builtin_isnan(d)) d = __builtin_copysignf(0.0f, d);
        recalc = true;
    }
    if (__builtin_isinf(c) || __builtin_isinf(d)) {
        c = __builtin_copysignf(__builtin_isinf(c) ? 1.0f : 0.0f, c);
        d = __builtin_copysignf(__builtin_isinf(d) ? 1.0f : 0.0f, d);
        if (__builtin_isnan(a)) a = __builtin_copysignf(0.0f, a);
        if (__builtin_isnan(b)) b = __builtin_copysignf(0.0f, b);
        recalc = true;
    }
    if (!recalc && (__builtin_isinf(ac) || __builtin_isinf(bd) || __builtin_isinf(ad) ||
                    __builtin_isinf(bc))) {
        if (__builtin_isnan(a)) a = __builtin_copysignf(0.0f, a);
        if (__builtin_isnan(b)) b = __builtin_copysignf(0.0f, b);
        if (__builtin_isnan(c)) c = __builtin_copysignf(0.0f, c);
        if (__builtin_isnan(d)) d = __builtin_copysignf(0.0f, d);
        recalc = true;
    }
    if (recalc) {
        const float inf = __builtin_inff();
        r.x = inf * (a * c - b * d);
        r.y = inf * (a * d + b * c);
    }
    return r;
}
__device__ __forceinline__ cf32 cmul_x(cf32 a, cf32 b) {
    const cf32 r = cmul(a, b);
    if (__builtin_expect(__builtin_isnan(r.x) && __builtin_isnan(r.y), 0))
        return cmul_recover(a.x, a.y, b.x, b.y);
    return r;
}
template <bool AG>
__device__ __forceinline__ cf32 cmul_t(cf32 a, cf32 b) {
    if constexpr (AG) return cmul_x(a, b);
    else return cmul(a, b);
}
// KISS radix-4 cross terms with scratch[4] = (s4.y, -s4.x) folded into the
// operand modifiers (kissfft.hh:178-183): a + (b.y, -b.x) and a - (b.y, -b.x).
__device__ __forceinline__ cf32 cadd_rot(cf32 a, cf32 b) {
    cf32 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ cf32 csub_rot(cf32 a, cf32 b) {
    cf32 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// Fused complex product for the certified fast path only (symbol units
// whose result is the argmax of |X|^2, proven against the rounding bound of
// fast_certified): (ax bx - ay by, ax by + ay bx) as one v_pk_mul_f32 and one
// v_pk_fma_f32.  Each part rounds once after an exact product instead of
// three times, so its error is within the plain product's bound.  Never used
// where the reference's bits are reproduced.
__device__ __forceinline__ cf32 cmul_fma(cf32 a, cf32 b) {
    const cf32 t = a.yy * b.yx;  // (ay by, ay bx)
    cf32 r;                      // (ax bx - t.x, ax by + t.y): the sign as a modifier
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_lo:[0,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
    return r;
}
// The same with a wave-uniform b (a compile-time twiddle): b is an SGPR-pair
// operand of both instructions, no copy to a VGPR.
__device__ __forceinline__ cf32 cmul_fma_s(cf32 a, cf32 b) {
    const cf32 t = a.yy * b.yx;
    cf32 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_lo:[0,0,1]" : "=v"(r) : "v"(a), "s"(b), "v"(t));
    return r;
}
__device__ __forceinline__ cf32 cadd(cf32 a, cf32 b) { return a + b; }
__device__ __forceinline__ cf32 csub(cf32 a, cf32 b) { return a - b; }
__device__ __forceinline__ cf32 cscale(cf32 a, float s) { return a * s; }
__device__ __forceinline__ cf32 czero() { return cf32{0.0f, 0.0f}; }

// Debug index checks (the test build, -DLPHY_DEBUG_BOUNDS): a computed LDS /
// global index outside its array counts in this translation unit's device
// counter (read back through SfOps::violations, lphy_hip_bounds_violations)
// instead of trapping, so a bad index fails a test rather than faulting the
// GPU.  Compiled out of the product library.
#ifdef LPHY_DEBUG_BOUNDS
namespace {
__device__ unsigned long long g_bound_violations;
}
#endif
__host__ __device__ constexpr void bound_check(long long i, long long lim) {
#if defined(LPHY_DEBUG_BOUNDS) && defined(__HIP_DEVICE_COMPILE__)
    if (!__builtin_is_constant_evaluated() && !(i >= 0 && i < lim)) atomicAdd(&g_bound_violations, 1ull);
#else
    (void)i;
    (void)lim;
#endif
}

template <int SF>
struct Geo {
    static constexpr int N = 1 << SF;
    static constexpr int L = (SF + 1) / 2;          // KISS stages
    static constexpr int E = N < 16 ? N : 16;       // complex per lane
    static constexpr int LPS = N / E;               // lanes per symbol
    static constexpr int T = kTile / LPS;           // symbols per tile
    // LDS layout (bank model of every access pattern in this file, see
    // DESIGN.md): for SF >= 5 a symbol slot is N complex wide and a position
    // p lives at slot*N + (swz(p) ^ sx(slot)), where swz XORs higher position
    // bits into lower ones and sx(slot) = slot*SKX mod N shifts neighbouring
    // slots to other banks.  Both are GF(2)-linear, so for p = lanepart |
    // constpart (disjoint bits, always the case here) the address is
    // lbase(slot, lanepart) ^ cpart(constpart): one XOR per access.  SF <= 4
    // (one symbol per lane) uses a padded stride N + 1 instead.
    static constexpr bool XS = SF >= 5;
    static constexpr int SSTRIDE = XS ? N : N + 1;  // LDS stride per symbol
    static constexpr int SK1 = SF == 7 || SF == 8 ? 2 : SF <= 6 ? 3 : 4;
    static constexpr int SM1 = SF <= 4 ? 0 : SF == 5 ? 1 : SF == 6 ? 3 : SF == 7 ? 7 : SF == 8 ? 15 : 31;
    static constexpr int SK2 = SF == 8 ? 6 : 5;
    static constexpr int SM2 = SF == 6 || SF == 7 ? 1 : SF == 8 || SF >= 11 ? 3 : 0;
    static constexpr int SKX = SF == 5 ? 2 : SF == 6 ? 4 : SF == 7 ? 8 : SF == 8 ? 16 : 0;
    __host__ __device__ static constexpr int swz(int p) {
        return XS ? (p ^ ((p >> SK1) & SM1) ^ ((p >> SK2) & SM2)) : p;
    }
    __host__ __device__ static constexpr int sx(int slot) { return XS ? (slot * SKX) & (N - 1) : 0; }
    // general address of position p of the symbol in `slot`
    __host__ __device__ static constexpr int addr(int slot, int p) {
        bound_check(p, N);
        const int a = slot * SSTRIDE + (swz(p) ^ sx(slot));
        bound_check(a, T * SSTRIDE);
        return a;
    }
    // split form: per-lane base for the lane-dependent position bits ...
    __host__ __device__ static constexpr int lbase(int slot, int lanepart) {
        return XS ? ((slot * N) | (swz(lanepart) ^ sx(slot))) : slot * SSTRIDE + lanepart;
    }
    // ... and the compile-time part of each access
    __host__ __device__ static constexpr int cpart(int constpart) { return XS ? swz(constpart) : constpart; }
    __host__ __device__ static constexpr int at(int lb, int cp) { return XS ? (lb ^ cp) : (lb + cp); }
    // the same in bytes (complex = 8 B): lb8 = lbase << 3, cp8 = cpart << 3
    __host__ __device__ static constexpr int at8(int lb8, int cp8) {
        const int a = XS ? (lb8 ^ cp8) : (lb8 + cp8);
        bound_check(a, 8 * T * SSTRIDE);
        return a;
    }
    __host__ __device__ static constexpr int R(int l) { return ((SF & 1) && l == L - 1) ? 2 : 4; }
    __host__ __device__ static constexpr int M(int l) {
        int p = 1;
        for (int j = 0; j <= l; ++j) p *= R(j);
        return N / p;
    }
    __host__ __device__ static constexpr int FS(int l) { return 1 << (2 * l); }
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

// Synchronisation of the lanes that share a symbol ("team" of LPS lanes).
// Up to LPS = 64 a team lives inside one wavefront: its LDS exchanges only
// need no compiler motion across the point (a wave's LDS instructions
// execute in order, so a read issued after a write sees it).  Larger teams span
// wavefronts and need the workgroup barrier.
template <int SF>
__device__ __forceinline__ void team_sync() {
    if constexpr (Geo<SF>::LPS <= 64) {
#ifdef LPHY_TEAM_WAIT  // experiments: drain the wave's LDS queue (7 % slower)
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
#else
        // a wave's LDS operations execute in issue order, so a team inside
        // one wavefront only needs compiler motion across the point stopped
        asm volatile("" ::: "memory");
#endif
        __builtin_amdgcn_wave_barrier();
    } else {
        __syncthreads();
    }
}

// Base-4 digit reversal of `high` over `ndig` digits (leaf permutation of the
// digits that precede the first pass).
__host__ __device__ constexpr int rev4(int high, int ndig) {
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
    __host__ __device__ static constexpr int g(int s, int lam) { return s * G::LPS + lam; }
    __host__ __device__ static constexpr int low(int s, int lam) { return g(s, lam) % P::MH; }
    __host__ __device__ static constexpr int high(int s, int lam) { return g(s, lam) / P::MH; }
    __host__ __device__ static constexpr int base(int s, int lam) {
        return high(s, lam) * P::SPAN + low(s, lam);
    }
    // position of element e (= s*GS + a) of the lane; the lane bits and the
    // element bits are disjoint: pos(e, lam) = pos(0, lam) | pos(e, 0)
    __host__ __device__ static constexpr int pos(int e, int lam) {
        return base(e / P::GS, lam) + (e % P::GS) * P::MH;
    }
    // first-pass input index of element e (KISS leaf permutation), same split
    __host__ __device__ static constexpr int inidx(int e, int lam) {
        return rev4(high(e / P::GS, lam), LO) + P::vidx(e % P::GS);
    }
};

// All butterflies of one pass on the lane's registers.  v[s*GS + a] is group
// s, group-local index a.
//
// TRIV (symbol units of the certified fast path only): butterflies whose
// twiddle index is 0 at compile time skip the product with tw[0] = (1, 0).
// x * (1, 0) = (re - im*0, im + re*0) equals x up to the sign of an exact
// zero (and NaN from an infinite component, which the certificate rejects),
// so every |X|^2 - all a symbol unit keeps - is unchanged.  Estimate units
// keep the multiply: their bins feed atan2, where the sign of a zero counts.
template <int SF, int HI, int LO, bool TRIV = false, bool AG = false>
__device__ __forceinline__ void pass_butterflies(cf32 (&v)[16], int lam,
                                                 const cf32* __restrict__ tw) {
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
                // twiddle index 0 for every lane: MH == 1 makes low == 0
                const bool one = TRIV && P::MH == 1 && (a % w) == 0;
                cf32* x = &v[s * P::GS];
                // TRIV transforms only feed the certified |X|^2 argmax: fused products
                auto mul = [&](cf32 u, cf32 t) __attribute__((always_inline)) {
                    if constexpr (TRIV) return cmul_fma(u, t);
                    else return cmul_t<AG>(u, t);
                };
                if (R == 2) {
                    const cf32 t = one ? x[a + w] : mul(x[a + w], tw[k * fs]);
                    x[a + w] = csub(x[a], t);
                    x[a] = cadd(x[a], t);
                } else {
                    const cf32 s0 = one ? x[a + w] : mul(x[a + w], tw[k * fs]);
                    const cf32 s1 = one ? x[a + 2 * w] : mul(x[a + 2 * w], tw[k * fs * 2]);
                    const cf32 s2 = one ? x[a + 3 * w] : mul(x[a + 3 * w], tw[k * fs * 3]);
                    const cf32 s5 = csub(x[a], s1);
                    const cf32 a0 = cadd(x[a], s1);
                    const cf32 s3 = cadd(s0, s2);
                    const cf32 s4 = csub(s0, s2);
                    x[a + 2 * w] = csub(a0, s3);
                    x[a] = cadd(a0, s3);
                    x[a + w] = cadd_rot(s5, s4);
                    x[a + 3 * w] = csub_rot(s5, s4);
                }
            }
        }
    }
}

// Pass PI of the transform on the tile's LDS (`lds`), symbol in `slot`.
//  first pass: read inputs from the natural-order staging copy at KISS's
//              leaf-permuted index, barrier, compute, write positions;
//  last pass:  leave results in registers for the detector.
__device__ __forceinline__ cf32 lds_ld(const cf32* lds, int byte_off) {
    return *reinterpret_cast<const cf32*>(reinterpret_cast<const char*>(lds) + byte_off);
}
__device__ __forceinline__ void lds_st(cf32* lds, int byte_off, cf32 v) {
    *reinterpret_cast<cf32*>(reinterpret_cast<char*>(lds) + byte_off) = v;
}

template <int SF, int PI, bool LAST, bool TRIV, bool AG, bool REG0 = false>
__device__ __forceinline__ void run_pass(cf32 (&v)[16], cf32* lds, int slot, int lam,
                                         const cf32* __restrict__ tw) {
    using G = Geo<SF>;
    constexpr Passes<SF> PS{};
    constexpr int HI = PS.hi[PI], LO = PS.lo[PI];
    using Gr = Group<SF, HI, LO>;
    if (PI == 0 && REG0) {
        // inputs already in registers, in first-pass order (first_pass_index)
    } else if (PI == 0) {
        const int lb8 = G::lbase(slot, Gr::inidx(0, lam)) << 3;
#pragma unroll
        for (int e = 0; e < G::E; ++e) v[e] = lds_ld(lds, G::at8(lb8, G::cpart(Gr::inidx(e, 0)) << 3));
        team_sync<SF>();
    } else {
        const int lb8 = G::lbase(slot, Gr::pos(0, lam)) << 3;
#pragma unroll
        for (int e = 0; e < G::E; ++e) v[e] = lds_ld(lds, G::at8(lb8, G::cpart(Gr::pos(e, 0)) << 3));
    }
    pass_butterflies<SF, HI, LO, TRIV, AG>(v, lam, tw);
    if (!LAST) {
        const int lb8 = G::lbase(slot, Gr::pos(0, lam)) << 3;
#pragma unroll
        for (int e = 0; e < G::E; ++e) lds_st(lds, G::at8(lb8, G::cpart(Gr::pos(e, 0)) << 3), v[e]);
        team_sync<SF>();
    }
}

template <int SF, int PI, bool TRIV, bool AG, bool REG0 = false>
__device__ __forceinline__ void run_passes(cf32 (&v)[16], cf32* lds, int slot, int lam,
                                           const cf32* __restrict__ tw) {
    constexpr Passes<SF> PS{};
    if constexpr (PI < PS.n) {
        run_pass<SF, PI, PI == PS.n - 1, TRIV, AG, REG0>(v, lds, slot, lam, tw);
        run_passes<SF, PI + 1, TRIV, AG, false>(v, lds, slot, lam, tw);
    }
}

// Full transform of the symbol staged (natural order) in `slot` of the tile
// LDS; on return v[e] holds bin bin_of<SF>(e, lam).  Must be called by every
// thread of the tile (contains barriers).
// TRIV: see pass_butterflies (magnitude-only consumers).
// AG: every product with the reference's Annex G recovery (cmul_x).
// REG0: v already holds the symbol's samples in first-pass order (element e
// = sample first_pass_index<SF>(e, lam)), so the transform starts without the
// natural-order LDS staging round trip.
template <int SF, bool TRIV = false, bool AG = false, bool REG0 = false>
__device__ __forceinline__ void fft_tile(cf32 (&v)[16], cf32* lds, int slot, int lam,
                                         const cf32* __restrict__ tw) {
    run_passes<SF, 0, TRIV, AG, REG0>(v, lds, slot, lam, tw);
}

// Sample index that element e of lane lam holds at the start of the first
// pass (KISS leaf permutation): lane part | compile-time part.
template <int SF>
__host__ __device__ constexpr int first_pass_index(int e, int lam) {
    constexpr Passes<SF> PS{};
    return Group<SF, PS.hi[0], PS.lo[0]>::inidx(e, lam);
}

// Whether any of the lane's bins has a NaN part: the trigger for re-running
// a transform (and the products staged into it) with cmul_x.  Sums the
// detector's |X|^2 values (>= 0 or NaN, so the sum is NaN exactly when one
// of them is); written like local_argmax so the compiler shares them.
template <int SF>
__device__ __forceinline__ bool fft_has_nan(const cf32 (&v)[16]) {
    float s = 0.0f;
#pragma unroll
    for (int e = 0; e < Geo<SF>::E; ++e) {
        const cf32 sq = v[e] * v[e];
        s += sq.x + sq.y;
    }
    return s != s;
}

template <int SF>
__host__ __device__ constexpr int bin_of(int e, int lam) {
    constexpr Passes<SF> PS{};
    return Group<SF, PS.hi[PS.n - 1], PS.lo[PS.n - 1]>::pos(e, lam);
}

// Natural-order staging address of sample i = lam + e*LPS of the slot.
template <int SF>
struct Stage {
    using G = Geo<SF>;
    int lb8;
    __device__ __forceinline__ Stage(int slot, int lam) : lb8(G::lbase(slot, lam) << 3) {}
    __device__ __forceinline__ void put(cf32* lds, int e, cf32 x) const {
        lds_st(lds, G::at8(lb8, G::cpart(e * G::LPS) << 3), x);
    }
};

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

// Element order of the last pass sorted by increasing bin: bin_of(e, lam) =
// bin_of(0, lam) | bin_of(e, 0), so this order is increasing for every lane.
template <int SF>
struct BinOrder {
    int e[16] = {};
    constexpr BinOrder() {
        constexpr int E = Geo<SF>::E;
        for (int i = 0; i < E; ++i) e[i] = i;
        for (int i = 0; i < E; ++i)
            for (int j = i + 1; j < E; ++j)
                if (bin_of<SF>(e[j], 0) < bin_of<SF>(e[i], 0)) { int t = e[i]; e[i] = e[j]; e[j] = t; }
    }
};

// Lane-local part of the detector's scan: visiting the lane's bins in
// increasing order with a strict '>' keeps the first maximum, exactly like
// the reference loop restricted to these bins.
template <int SF>
__device__ __forceinline__ ArgMax local_argmax(const cf32 (&v)[16], int lam) {
    using G = Geo<SF>;
    constexpr BinOrder<SF> BO{};
    ArgMax best{0.0f, 0x7fffffff};
    const int lane_bin = bin_of<SF>(0, lam);
#pragma unroll
    for (int k = 0; k < G::E; ++k) {
        const int e = BO.e[k];
        const cf32 sq = v[e] * v[e];
        const float m2 = sq.x + sq.y;
        const bool take = m2 > best.v;
        best.v = take ? m2 : best.v;
        best.i = take ? (lane_bin | bin_of<SF>(e, 0)) : best.i;
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

// Argmax plus the runner-up value: v2 = max |X|^2 over every bin but the
// winner (ties give v2 == v).  NaN bins are ignored by both (v_min / v_max
// return the other operand), so an all-NaN symbol ends with v = v2 = 0.
// Used by the certified fast rotation (k_frames): a symbol whose winner
// clears the runner-up by more than the rounding bound has the reference's
// argmax, any other symbol is recomputed with the exact rotation.
struct ArgMax2 {
    float v;
    int i;
    float v2;
};

// The winning element index is tracked (an inline constant per select) and
// mapped to its bin once at the end: bin_of(e, 0) = (e % GS) * MH + (e / GS)
// * bin_of(GS, 0) with the last pass's group size GS (checked at compile
// time below).
template <int SF>
__device__ __forceinline__ ArgMax2 local_argmax2(const cf32 (&v)[16], int lam) {
    using G = Geo<SF>;
    constexpr BinOrder<SF> BO{};
    constexpr Passes<SF> PS{};
    using PG = PassGeo<SF, PS.hi[PS.n - 1], PS.lo[PS.n - 1]>;
    constexpr int GS = PG::GS < G::E ? PG::GS : G::E;
    constexpr int MH = bin_of<SF>(1, 0);
    constexpr int XS = GS < G::E ? bin_of<SF>(GS, 0) : 0;
    static_assert([] {
        for (int e = 0; e < G::E; ++e)
            if (bin_of<SF>(e, 0) != (e % GS) * MH + (e / GS) * XS) return false;
        return true;
    }(), "bin_of separable in the element's digits");
    ArgMax2 best{0.0f, 0x7fffffff, 0.0f};
    int best_e = -1;
#pragma unroll
    for (int k = 0; k < G::E; ++k) {
        const int e = BO.e[k];
        const cf32 sq = v[e] * v[e];
        const float m2 = sq.x + sq.y;
        // runner-up = max(v2, min(m2, v)) = med3(v, v2, m2) as v >= v2 (one
        // v_med3; a NaN m2 only arises with every bin NaN, where v stays 0)
        best.v2 = __builtin_amdgcn_fmed3f(best.v, best.v2, m2);
        const bool take = m2 > best.v;
        best.v = take ? m2 : best.v;
        best_e = take ? e : best_e;
    }
    if (best_e >= 0) best.i = bin_of<SF>(0, lam) | ((best_e % GS) * MH + (best_e / GS) * XS);
    return best;
}

// Team reduction (LPS <= 64 only: one wavefront per symbol).
template <int SF>
__device__ __forceinline__ ArgMax2 symbol_argmax2(ArgMax2 a) {
    using G = Geo<SF>;
    static_assert(G::LPS <= 64, "team inside one wavefront");
#pragma unroll
    for (int off = G::LPS / 2; off >= 1; off >>= 1) {
        ArgMax2 o;
        o.v = __shfl_xor(a.v, off, 64);
        o.i = __shfl_xor(a.i, off, 64);
        o.v2 = __shfl_xor(a.v2, off, 64);
        a.v2 = fmaxf(fmaxf(a.v2, o.v2), fminf(a.v, o.v));
        const bool take = (o.v > a.v) | ((o.v == a.v) & (o.i < a.i));
        a.v = take ? o.v : a.v;
        a.i = take ? o.i : a.i;
    }
    if (!(a.v > 0.0f)) a.i = 0;  // nothing beat maxValue = 0
    return a;
}

// DPP row shift (v_mov_b32_dpp row_shl:n): lane i receives lane i + n of
// its 16-lane row (lanes past the row keep `old`).
template <int N>
__device__ __forceinline__ int dpp_row_shl(int v) {
    static_assert(N >= 1 && N <= 15, "row_shl range");
    return __builtin_amdgcn_update_dpp(v, v, 0x100 | N, 0xF, 0xF, false);
}
template <int N>
__device__ __forceinline__ float dpp_row_shl(float v) {
    return __builtin_bit_cast(float, dpp_row_shl<N>(__builtin_bit_cast(int, v)));
}

// Team reduction toward the team's first lane (LPS <= 16: the team sits in
// one DPP row), no LDS traffic: the result is valid in lane lam == 0 only
// (the lanes above read across into the next team).
template <int SF, int OFF = Geo<SF>::LPS / 2>
__device__ __forceinline__ ArgMax2 team_argmax2_first(ArgMax2 a) {
    static_assert(Geo<SF>::LPS <= 16, "team inside one DPP row");
    if constexpr (OFF >= 1) {
        ArgMax2 o;
        o.v = dpp_row_shl<OFF>(a.v);
        o.i = dpp_row_shl<OFF>(a.i);
        o.v2 = dpp_row_shl<OFF>(a.v2);
        a.v2 = fmaxf(fmaxf(a.v2, o.v2), fminf(a.v, o.v));
        const bool take = (o.v > a.v) | ((o.v == a.v) & (o.i < a.i));
        a.v = take ? o.v : a.v;
        a.i = take ? o.i : a.i;
        return team_argmax2_first<SF, OFF / 2>(a);
    } else {
        if (!(a.v > 0.0f)) a.i = 0;  // nothing beat maxValue = 0
        return a;
    }
}
// Keyed top two for the certified symbol-only tiles (LPS <= 16).  A bin's
// key is its |X|^2 bit pattern (>= 0, so ordered like the value as an
// unsigned integer) with the KB low bits replaced by an id: the element e in
// bits 0-3, the team lane in the bits above.  Top two of the keys is one
// v_max_u32 and one v_med3_u32 per bin, the team merge two DPP moves, a max
// and a med3 per step.  The result is a bound, not the detector's argmax:
// with T(k) = k & ~MASK (the value truncated to its high bits), every step
// is monotone in T, so T(k1) is the largest truncated value and T(k2) the
// second largest (counted with multiplicity).  When T(k1) > T(k2) the bin of
// k1 is the unique maximum, v = T(k1) <= its |X|^2 and v2 = T(k2) | MASK >=
// every other bin's |X|^2; otherwise v <= v2 and the certificate fails (a
// tie or near-tie goes to the exact recheck, as before).  NaN bins key above
// every number (v = NaN fails the certificate).  Valid in lane lam == 0.
__device__ __forceinline__ unsigned med3_u32(unsigned a, unsigned b, unsigned c) {
    unsigned r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// (row shift with bound_ctrl: lanes past the row read 0, the keys' least
// value, and no copy of the old value is needed, so the compiler can fold
// the shift of k2 into the v_max_u32 that consumes it)
template <int N>
__device__ __forceinline__ unsigned dpp_row_shl_z(unsigned v) {
    static_assert(N >= 1 && N <= 15, "row_shl range");
#ifdef LPHY_AB_DPP_OLD  // A/B timing only: the old-value form
    return (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x100 | N, 0xF, 0xF, false);
#else
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x100 | N, 0xF, 0xF, true);
#endif
}
// Top two of {k1, k2, a, b} for distinct keys with k1 >= k2: the second
// largest is max(k2, med3(k1, a, b)) (if k1 leads {k1, a, b}, the middle is
// max(a, b); otherwise the middle is the larger of k1 and the other new
// key, and k1 >= k2).  One v_max3_u32, one v_med3_u32 and one v_max_u32
// per two keys, against a v_med3_u32 and a v_max_u32 per key.
__device__ __forceinline__ void top2_pair(unsigned& k1, unsigned& k2, unsigned a, unsigned b) {
#ifdef LPHY_AB_TOP2_SINGLE  // A/B timing only: one key at a time
    k2 = med3_u32(k1, k2, a);
    k1 = k1 > a ? k1 : a;
    k2 = med3_u32(k1, k2, b);
    k1 = k1 > b ? k1 : b;
#else
    const unsigned m = med3_u32(k1, a, b);
    const unsigned t = k1 > a ? k1 : a;
    k1 = t > b ? t : b;
    k2 = k2 > m ? k2 : m;
#endif
}
template <int SF, int OFF = Geo<SF>::LPS / 2>
__device__ __forceinline__ void team_top2_keys(unsigned& k1, unsigned& k2) {
    if constexpr (OFF >= 1) {
        const unsigned o1 = dpp_row_shl_z<OFF>(k1);
        const unsigned o2 = dpp_row_shl_z<OFF>(k2);
        k2 = med3_u32(k1, o1, k2 > o2 ? k2 : o2);
        k1 = k1 > o1 ? k1 : o1;
        team_top2_keys<SF, OFF / 2>(k1, k2);
    }
}
template <int SF>
__device__ __forceinline__ ArgMax2 team_argmax2_keyed_first(const cf32 (&v)[16], int lam) {
    using G = Geo<SF>;
    static_assert(G::LPS <= 16 && G::E <= 16, "team inside one DPP row, 4 element bits");
    constexpr Passes<SF> PS{};
    using PG = PassGeo<SF, PS.hi[PS.n - 1], PS.lo[PS.n - 1]>;
    constexpr int GS = PG::GS < G::E ? PG::GS : G::E;
    constexpr int MH = bin_of<SF>(1, 0);
    constexpr int XS = GS < G::E ? bin_of<SF>(GS, 0) : 0;
    constexpr int LB = G::LPS >= 16 ? 4 : G::LPS >= 8 ? 3 : G::LPS >= 4 ? 2 : G::LPS >= 2 ? 1 : 0;
    constexpr unsigned MASK = (1u << (4 + LB)) - 1u;
    // a lane's first bin (bin_of(0, lam)) as arithmetic on lam
    constexpr int LMH = PG::MH, LSPAN = PG::SPAN;
    static_assert([] {
        for (int l = 0; l < G::LPS; ++l)
            if (bin_of<SF>(0, l) != (l / LMH) * LSPAN + l % LMH) return false;
        for (int e = 0; e < G::E; ++e)
            if (bin_of<SF>(e, 0) != (e % GS) * MH + (e / GS) * XS) return false;
        return true;
    }(), "bin_of separable in the lane and element digits");
    static_assert(G::E % 2 == 0, "keys taken in pairs");
    auto key_of = [&](int e) __attribute__((always_inline)) {
#ifdef LPHY_KEY_FMA  // A/B: |X|^2 = fma(x, x, fl(y y)), scalar f32 (within cert_gap's 8 u)
        const float m2 = __builtin_fmaf(v[e].x, v[e].x, v[e].y * v[e].y);
#else
        const cf32 sq = v[e] * v[e];
        const float m2 = sq.x + sq.y;
#endif
        return (__float_as_uint(m2) & ~15u) | (unsigned)e;
    };
    unsigned k1 = 0u, k2 = 0u;
#pragma unroll
    for (int e = 0; e < G::E; e += 2) top2_pair(k1, k2, key_of(e), key_of(e + 1));
    if constexpr (LB > 0) {
        k1 = (k1 & ~(MASK & ~15u)) | ((unsigned)lam << 4);
        team_top2_keys<SF>(k1, k2);
    }
    ArgMax2 r;
    r.v = __uint_as_float(k1 & ~MASK);
    r.v2 = __uint_as_float(k2 | MASK);
    const int e = (int)(k1 & 15u), lw = (int)((k1 >> 4) & (MASK >> 4));
    r.i = ((lw / LMH) * LSPAN + lw % LMH) | ((e % GS) * MH + (e / GS) * XS);
    return r;
}

template <int SF, int OFF = Geo<SF>::LPS / 2>
__device__ __forceinline__ float team_max_first(float a) {
    if constexpr (OFF >= 1) return team_max_first<SF, OFF / 2>(fmaxf(a, dpp_row_shl<OFF>(a)));
    else return a;
}

// Workgroup form for teams spanning wavefronts (LPS > 64: SF 11-12): the
// waves reduce in registers, then combine through `red` (one entry per wave;
// contains barriers, every thread of the tile calls it).
// TAIL_SYNC = false: the caller alternates `red` / `redm` between tiles, so
// the trailing barrier that protects their reuse is not needed.
template <int SF, bool TAIL_SYNC = true>
__device__ __forceinline__ ArgMax2 symbol_argmax2_wg(ArgMax2 a, ArgMax2* red, float* m = nullptr,
                                                     float* redm = nullptr) {
    using G = Geo<SF>;
    static_assert(G::LPS > 64, "teams inside one wavefront use symbol_argmax2");
    auto comb = [](ArgMax2 x, ArgMax2 o) __attribute__((always_inline)) {
        x.v2 = fmaxf(fmaxf(x.v2, o.v2), fminf(x.v, o.v));
        const bool take = (o.v > x.v) | ((o.v == x.v) & (o.i < x.i));
        x.v = take ? o.v : x.v;
        x.i = take ? o.i : x.i;
        return x;
    };
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        ArgMax2 o;
        o.v = __shfl_xor(a.v, off, 64);
        o.i = __shfl_xor(a.i, off, 64);
        o.v2 = __shfl_xor(a.v2, off, 64);
        a = comb(a, o);
    }
    // m (optional): a per-lane max reduced over the team alongside
    if (m) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) *m = fmaxf(*m, __shfl_xor(*m, off, 64));
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[wave] = a;
        if (m) redm[wave] = *m;
    }
    __syncthreads();
    constexpr int WPS = G::LPS / 64;
    const int first = (wave / WPS) * WPS;
    ArgMax2 b = red[first];
#pragma unroll
    for (int w = 1; w < WPS; ++w) b = comb(b, red[first + w]);
    if (m) {
        float mm = redm[first];
#pragma unroll
        for (int w = 1; w < WPS; ++w) mm = fmaxf(mm, redm[first + w]);
        *m = mm;
    }
    if constexpr (TAIL_SYNC) __syncthreads();
    if (!(b.v > 0.0f)) b.i = 0;
    return b;
}

}  // namespace lphy
