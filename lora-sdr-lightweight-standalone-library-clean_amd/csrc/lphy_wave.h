// lphy_wave.h — fused single launch for SF 7-12 (N = 128 .. 4096): one
// wavefront per unit of 64 x 64 complex values, i.e. one symbol at SF 12,
// 2 / 4 / 8 / 16 / 32 symbols at SF 11 / 10 / 9 / 8 / 7 (SF 7-10: units
// spanning frames, WSchedSpan), no workgroup barrier in the loop.  Included by lphy_kernels.h inside its anonymous
// namespace, after k_frames (it reuses SymCtx, EstFold, the certificate and
// the speculative normalisation of the SF <= 10 path).
//
// The reference demodulates a frame in one pass at every SF
// (/root/reference/src/phy/LoRaDemod.cpp:142-176, phy.cpp:204-238) with
// KISS's recursive radix-4 DIT (kissfft.hh:106-185).  Here a lane holds 64
// complex values of one symbol (LPS = N/64 lanes per symbol: 64 at SF 12,
// 32 / 16 / 8 / 4 / 2 at SF 11 .. 7 where a wave carries SPW = 64 / LPS
// symbols):
//
//   staging  the unit's IQ was copied HBM -> LDS by LDS-DMA during the
//            previous unit (global_load_lds_dwordx4, 1 KiB per wave
//            instruction, natural sample order); lane (h, l) reads samples
//            i = l + LPS m of symbol h, m = 0..63, applies the [exact]
//            dechirp and the rotation, keeps them in registers;
//   pass 1   KISS stages L-1 .. 3 (the innermost) on the lane's registers:
//            the inputs with equal i mod 64 form one sub-transform of
//            length LPS (SPW groups per lane);
//   exchange the 64 x LPS transpose through the wave's own LDS buffer (the
//            one the IQ landed in: XOR-swizzled rows, conflict-free b64
//            writes and reads), then the next unit's LDS-DMA is issued into
//            it;
//   pass 2   KISS stages 2, 1, 0 on the lane's registers: lane l ends with
//            the bins l + LPS B', B' = 0..63;
//   argmax   lane-local top two and a cross-lane merge (the keyed bound of
//            the certified path, or the detector's exact first maximum for
//            the estimate units).
//
// Symbol units take the certified fast rotation: the frame's
// rotation is a per-lane table of 8 entries times a wave-uniform one of 8,
// and pass 2's last stage forms its per-lane twiddle tw[(l + LPS r) q] as
// tw[l q] tw[LPS r q].  Both deviations are charged to the certificate
// (kWaveExtra below); an uncertified symbol is left to k_post as in k_frames.
// Estimate units run KISS's own arithmetic: every twiddle from the table,
// unfused products, the detector's exact argmax, bit-identical bins.
//
// Per wave, frames w, w + W, ... (W waves); per frame the estimate units (2
// at SF 12, each folding its symbol's max-abs for the normalisation; SF 11
// one unit whose halves 0 and 1 hold symbols 0 and 1; SF 7-10 one unit for
// EPU frames), then the symbol units.  The next frame's estimate units run two
// symbol units before the current frame's end, so its time shift is known
// when its first symbol unit's LDS-DMA is issued:
//   E(0) | D(0)_0..D(0)_{p-1}, E(1), D(0)_p..D(0)_{ND-1} | D(1)_0 ...
// with ND symbol units per frame and p = max(0, ND - 2).
//
// LDS: 4 waves x 32 KiB buffers (below 32 lanes per symbol each symbol's
// rows padded by LPS entries) + the down-chirp (N entries): the whole
// 160 KiB of a CU at SF 12, one 256-thread workgroup per CU.  SF 12 with
// the Hann window (round 6, modes 0 / 2): 3 waves (192 threads) x 32 KiB +
// the down-chirp + the window's N floats, 144 KiB (wave_wpb).

// unroll of the LDS-DMA's run of shifted windows: 4 (the loop's counter,
// compare and branch per 1 KiB piece were a third of a piece's ~8
// instructions at SF 7, 32 pieces per unit; same-box A/B SF 7 fused
// 0.785-0.801 -> 0.767-0.771 ms, SF 8-9 within noise).  (-D for timing
// experiments only.)
#ifndef LPHY_DMA_UNROLL
#define LPHY_DMA_UNROLL 4
#endif

// cache policy of the IQ's LDS-DMA: nt (2), streaming. Every IQ line is
// read once (twice for the estimate symbols), so it should not push the
// twiddle table and the partly written output lines out of L2: same-box
// A/B (profiles/r5/ab_iq_nt.txt) C2 1.63-1.69 -> 1.57-1.60 ms, FETCH
// 1.044x -> 1.039x of the algorithmic bytes, WRITE 0.85 -> 0.66 MB (the
// results exactly); SF 9 -1..2 %; sc1 (16): no change.  (-D for timing
// experiments only.)
#ifndef LPHY_IQ_CPOL
#define LPHY_IQ_CPOL 2
#endif

template <int SF>
struct WGeo {
    static constexpr int N = 1 << SF;
    static constexpr int LPS = N / 64;    // lanes per symbol = pass-1 sub-transform length
    static constexpr int SPW = 64 / LPS;  // symbols per unit (1 | 2 | 4 | 8)
    static constexpr int NE = SPW == 1 ? 2 : 1;  // estimate units per frame (group)
    // frames per estimate unit: SF 7-10 put EPU frames' two estimate symbols
    // in one unit (halves 2j, 2j + 1: frame j), SF 11-12 one frame's
    static constexpr int EPU = SPW >= 4 ? SPW / 2 : 1;
    // frame records in the per-wave LDS ring (EPU > 1): the group in
    // demodulation and the next one
    static constexpr int RING = EPU > 1 ? (2 * EPU > 8 ? 2 * EPU : 8) : 1;
    static constexpr int L = (SF + 1) / 2;       // KISS stages (radix 4, a last radix 2 for odd SF)
    static constexpr int PPS = N / 128;   // LDS-DMA pieces (1 KiB) per symbol
    static_assert(PPS < 4 || PPS % 4 == 0, "LDS-DMA in groups of four pieces (SF 7-8: one, two)");
    // symbol stride in the wave's buffer: below 32 lanes per symbol a row of
    // LPS entries shifts the next symbol's banks (conflict-free exchange
    // reads and staging reads across the symbols of one lane group)
    static constexpr int SS = LPS >= 32 ? N : N + LPS;
    static constexpr int BUF = SPW * SS;  // complex per wave buffer
    static constexpr int WPB = 4;         // waves per workgroup
    // radix of KISS stage l, its butterfly span M(l) (product of the inner
    // radices) and the digit weight of stage l inside a pass-1 input index
    __host__ __device__ static constexpr int rad(int l) { return ((SF & 1) && l == L - 1) ? 2 : 4; }
    __host__ __device__ static constexpr int Mst(int l) {
        int m = 1;
        for (int k = l + 1; k < L; ++k) m *= rad(k);
        return m;
    }
    __host__ __device__ static constexpr int Wst(int l) {
        int w = 1;
        for (int k = 3; k < l; ++k) w *= rad(k);
        return w;
    }
    // block of pass-1 group c = i mod 64 in KISS's output order: base-4
    // reversal of its three digits (c = d0 + 4 d1 + 16 d2 -> 16 d0 + 4 d1 + d2)
    __host__ __device__ static constexpr int rev3(int c) {
        return ((c & 3) << 4) | (((c >> 2) & 3) << 2) | ((c >> 4) & 3);
    }
    // in-group index m (i = c + 64 m) of pass-1 position p: the mixed-radix
    // digit reversal of KISS's stages 3 .. L-1 (SF 12: m = d3 + 4 d4 + 16 d5,
    // p = d3 M3 + d4 M4 + d5)
    __host__ __device__ static constexpr int minv(int p) {
        int m = 0;
        for (int l = 3; l < L; ++l) m += ((p / Mst(l)) % rad(l)) * Wst(l);
        return m;
    }
    // register of pass-1 group g, position p (element m'' = SPW m + g holds
    // sample i = l + LPS m'')
    __host__ __device__ static constexpr int reg1(int g, int p) { return SPW * minv(p) + g; }
    // exchange row swizzle (complex units) of block B: distinct over the
    // lanes of one symbol that write together (B's digits d0, d1 follow the
    // lane), below LPS
    __host__ __device__ static constexpr int sw(int B) {
        return LPS >= 32 ? (B >> 2) & 15 : (((B >> 4) & 3) + 4 * ((B >> 2) & 3)) & (LPS - 1);
    }
};

// u-multiples the certificate charges beyond KISS's 12 L, each
// a bound on how far a twiddle (or rotation factor) of the symbol units'
// transform lies from the KISS value it replaces, charged once per stage on
// that stage's inputs like the stage's own 6 u:
//   * KISS's table entry std::exp(i fl(k phinc)) lies within 7.3 u of the
//     ideal root (phase rounding <= 2 pi u, phinc's rounding <= pi u, the
//     float cos / sin <= 1 u);
//   * pass 1's stages 4 and 3 use the correctly rounded ideal root (<= 1 u):
//     <= 8.3 u from the table, 9 each;
//   * pass 2's stages 1 and 0 use a table entry times a rounded root (the
//     fused product: <= 7.3 + 1 + 2 u from the ideal): <= 18 u from the
//     table, 18 each;
//   * the two-table rotation, 6 (as k_demod's).
// 9 + 9 + 18 + 18 + 6 = 60, rounded up.
constexpr float kWaveExtra = 64.0f;

// The KISS twiddle table as the constant address space: wave-uniform reads
// become scalar loads (counted on lgkmcnt, so they never wait for the
// LDS-DMA in flight on vmcnt).  The table is never written by a kernel.
typedef const __attribute__((address_space(4))) cf32 ctw_t;
__device__ __forceinline__ ctw_t* ctw(const cf32* p) { return (ctw_t*)p; }

// The kernel's own argument block in the kernarg segment (constant address
// space), for the functions k_wave calls out of line: a reference to its
// DemodArgs would make the compiler copy the whole block to scratch, whose
// reloads (vmcnt) then wait for the LDS-DMA in flight; through this pointer
// every field is a scalar load (lgkmcnt).  P is k_wave's only argument, at
// offset 0 of the segment.
typedef const __attribute__((address_space(4))) FrameArgs* KArgs;
typedef __attribute__((address_space(3))) cf32 lds_cf32;  // LDS pointers across calls
__device__ __forceinline__ const DemodArgs& kargs(KArgs k) { return ((const FrameArgs*)k)->A; }

// Compiler-only fence: memory operations are not moved across it, so the
// scheduler cannot hoist a whole loop's loads (and their registers) ahead.
__device__ __forceinline__ void cfence() { asm volatile("" ::: "memory"); }

// The wave-uniform twiddles of the symbol units' transform, all 64th roots
// of unity e^{-2 pi i j / 64} (every uniform index is a multiple of N/64),
// computed at compile time in double and rounded to float: literal operands
// (SGPRs set by s_mov), no table load.  They differ from KISS's float table
// (std::exp of a rounded phase, kissfft.hh:24-29) by a few u, which the
// certificate charges (kWaveExtra); estimate units use the table itself.
struct CTw {
    float re, im;
};
struct Roots64 {
    CTw t[64];
    constexpr Roots64() : t{} {
        constexpr double kPiD = 3.14159265358979323846;
        for (int j = 0; j < 64; ++j) {
            // angle 2 pi j / 64 = quadrant q (pi/2) + remainder r in [0, pi/2)
            const int q = j / 16;
            const double r = 2.0 * kPiD * (double)(j % 16) / 64.0;
            // cos / sin of r by their Taylor series (|r| < pi/2, 20 terms)
            double c = 0.0, sn = 0.0, tc = 1.0, ts = r;
            for (int n = 0; n < 20; ++n) {
                c += tc;
                sn += ts;
                tc *= -r * r / ((2.0 * n + 1.0) * (2.0 * n + 2.0));
                ts *= -r * r / ((2.0 * n + 2.0) * (2.0 * n + 3.0));
            }
            double cq = c, sq = sn;  // rotate by q quarter turns
            for (int k = 0; k < q; ++k) {
                const double tmp = cq;
                cq = -sq;
                sq = tmp;
            }
            t[j] = CTw{(float)cq, (float)-sq};  // e^{-i angle}
        }
    }
};
constexpr Roots64 kRoots64{};
__device__ __forceinline__ cf32 root64(int j) {
    const CTw c = kRoots64.t[j & 63];
    return cf32{c.re, c.im};
}

// x * root64(j) on the fast path from nine base constants: root64(j) =
// (-i)^q root64(r) (j = 16 q + r), and for r > 8 root64(r) = (-B.y, -B.x)
// with B = root64(16 - r); so w = (sx B[cx], sy B[1 - cx]) for B = root64(r'),
// r' <= 8, and the swap and signs go into the op_sel / neg modifiers of
// cmul_fma's two instructions (the constants then fit the SGPR budget; the
// roots are the same correctly rounded values).
// (two statements: hipcc pads the dependent pair itself, and may schedule
// other work between them)
#define LPHY_CMR(CX, CY, NX, NY)                                                                  \
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1," #CY "] op_sel_hi:[1," #CX "] neg_lo:[0," #NY          \
        "] neg_hi:[0," #NX "]"                                                                      \
        : "=v"(t)                                                                                   \
        : "v"(a), "s"(B));                                                                          \
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0," #CX ",0] op_sel_hi:[0," #CY ",1] neg_lo:[0," #NX \
        ",1] neg_hi:[0," #NY ",0]"                                                                  \
        : "=v"(r)                                                                                   \
        : "v"(a), "s"(B), "v"(t))
__device__ __forceinline__ cf32 cmul_root(cf32 a, int j) {
    j &= 63;
    if (j == 0) return a;
    const int q = j >> 4, r0 = j & 15;
    const int rb = r0 <= 8 ? r0 : 16 - r0;
    int cx = r0 <= 8 ? 0 : 1, cy = 1 - cx;
    int sx = r0 <= 8 ? 0 : 1, sy = sx;  // 1: negated
    for (int k = 0; k < q; ++k) {      // w <- -i w: (x, y) -> (y, -x)
        const int c = cx, n = sx;
        cx = cy;
        sx = sy;
        cy = c;
        sy = n ^ 1;
    }
    const cf32 B = root64(rb);
    cf32 r, t;
    const int code = cx * 4 + sx * 2 + sy;
    switch (code) {
        case 0: LPHY_CMR(0, 1, 0, 0); break;
        case 1: LPHY_CMR(0, 1, 0, 1); break;
        case 2: LPHY_CMR(0, 1, 1, 0); break;
        case 3: LPHY_CMR(0, 1, 1, 1); break;
        case 4: LPHY_CMR(1, 0, 0, 0); break;
        case 5: LPHY_CMR(1, 0, 0, 1); break;
        case 6: LPHY_CMR(1, 0, 1, 0); break;
        default: LPHY_CMR(1, 0, 1, 1); break;
    }
    return r;
}
#undef LPHY_CMR

template <bool FAST, bool UNI = false>
__device__ __forceinline__ cf32 wmul(cf32 x, cf32 t) {
    if constexpr (FAST && UNI) return cmul_fma_s(x, t);
    else if constexpr (FAST) return cmul_fma(x, t);
    else return cmul(x, t);
}

// kf_bfly4 / kf_bfly2 (kissfft.hh:155-185) on registers; `one` (constant
// after unrolling): every twiddle is tw[0] = (1, 0), skipped on the fast
// path (magnitudes unchanged, see pass_butterflies' TRIV).
template <bool FAST, bool UNI = false>
__device__ __forceinline__ void wbfly4(cf32& x0, cf32& x1, cf32& x2, cf32& x3, cf32 w1, cf32 w2, cf32 w3,
                                       bool one) {
    const cf32 s0 = (FAST && one) ? x1 : wmul<FAST, UNI>(x1, w1);
    const cf32 s1 = (FAST && one) ? x2 : wmul<FAST, UNI>(x2, w2);
    const cf32 s2 = (FAST && one) ? x3 : wmul<FAST, UNI>(x3, w3);
    const cf32 s5 = csub(x0, s1);
    const cf32 a0 = cadd(x0, s1);
    const cf32 s3 = cadd(s0, s2);
    const cf32 s4 = csub(s0, s2);
    x2 = csub(a0, s3);
    x0 = cadd(a0, s3);
    x1 = cadd_rot(s5, s4);
    x3 = csub_rot(s5, s4);
}
// wbfly4 on the fast path with twiddles root64(j1), root64(j2), root64(j3)
__device__ __forceinline__ void wbfly4r(cf32& x0, cf32& x1, cf32& x2, cf32& x3, int j1, int j2, int j3) {
    const cf32 s0 = cmul_root(x1, j1);
    const cf32 s1 = cmul_root(x2, j2);
    const cf32 s2 = cmul_root(x3, j3);
    const cf32 s5 = csub(x0, s1);
    const cf32 a0 = cadd(x0, s1);
    const cf32 s3 = cadd(s0, s2);
    const cf32 s4 = csub(s0, s2);
    x2 = csub(a0, s3);
    x0 = cadd(a0, s3);
    x1 = cadd_rot(s5, s4);
    x3 = csub_rot(s5, s4);
}
template <bool FAST, bool UNI = false>
__device__ __forceinline__ void wbfly2(cf32& x0, cf32& x1, cf32 w, bool one) {
    const cf32 t = (FAST && one) ? x1 : wmul<FAST, UNI>(x1, w);
    x1 = csub(x0, t);
    x0 = cadd(x0, t);
}

// Pass 1: KISS stages L-1 .. 3 (the innermost ones: sub-transforms of
// length N/64 = LPS) of every group of the lane.  Twiddle indices are
// compile-time: the root on the fast path, wave-uniform loads from the KISS
// table otherwise.
template <int SF, bool FAST, int LV>
__device__ __forceinline__ void wpass1_stage(cf32 (&v)[64], ctw_t* tab, int g) {
    using W = WGeo<SF>;
    if constexpr (LV >= 3) {
        constexpr int R = W::rad(LV), M = W::Mst(LV), SPAN = R * M, FS = W::N / SPAN;
        static_assert(W::LPS % SPAN == 0 && 64 % SPAN == 0, "pass-1 stage inside a group");
#pragma unroll
        for (int blk = 0; blk < W::LPS / SPAN; ++blk) {
#pragma unroll
            for (int k = 0; k < M; ++k) {
                const int b0 = blk * SPAN + k;
                if constexpr (R == 4) {
                    if constexpr (FAST) {
                        // tw[j k FS] = root64(j k FS / (N/64)) = root64(j k 64 / SPAN)
                        wbfly4r(v[W::reg1(g, b0)], v[W::reg1(g, b0 + M)], v[W::reg1(g, b0 + 2 * M)],
                                v[W::reg1(g, b0 + 3 * M)], k * 64 / SPAN, 2 * k * 64 / SPAN, 3 * k * 64 / SPAN);
                    } else {
                        wbfly4<false>(v[W::reg1(g, b0)], v[W::reg1(g, b0 + M)], v[W::reg1(g, b0 + 2 * M)],
                                      v[W::reg1(g, b0 + 3 * M)], cf32(tab[k * FS]), cf32(tab[2 * k * FS]),
                                      cf32(tab[3 * k * FS]), false);
                    }
                } else {
                    if constexpr (FAST) {
                        const cf32 t = cmul_root(v[W::reg1(g, b0 + M)], k * 64 / SPAN);
                        v[W::reg1(g, b0 + M)] = csub(v[W::reg1(g, b0)], t);
                        v[W::reg1(g, b0)] = cadd(v[W::reg1(g, b0)], t);
                    } else {
                        wbfly2<false>(v[W::reg1(g, b0)], v[W::reg1(g, b0 + M)], cf32(tab[k * FS]), false);
                    }
                }
            }
        }
        wpass1_stage<SF, FAST, LV - 1>(v, tab, g);
    }
}
template <int SF, bool FAST>
__device__ __forceinline__ void wpass1(cf32 (&v)[64], ctw_t* tab) {
    using W = WGeo<SF>;
#pragma unroll
    for (int g = 0; g < W::SPW; ++g) wpass1_stage<SF, FAST, W::L - 1>(v, tab, g);
}

// Per-lane twiddles of pass 2's fast form (lane l of its symbol), q = 1..3:
// stage 2 tw[16 l q]; the lane factors tw[4 l q] and tw[l q] of stages 1
// and 0, whose twiddles tw[4 (l + LPS r) q] and tw[(l + LPS r) q] are taken
// as products with the wave-uniform tw[4 LPS r q] / tw[LPS r q] (r > 0).
template <int SF>
struct WTw {
    cf32 t2[3], t1[3], t0[3];
    __device__ __forceinline__ void load(const cf32* __restrict__ tw, int l) {
#pragma unroll
        for (int q = 1; q <= 3; ++q) {
            t2[q - 1] = tw[16 * l * q];
            t1[q - 1] = tw[4 * l * q];
            t0[q - 1] = tw[l * q];
        }
    }
};

// Pass 2: KISS stages 2, 1, 0 on elements B' (bins l + LPS B').  FAST: the
// per-lane table above and products with wave-uniform twiddles; exact: every
// twiddle from the KISS table (per-lane loads, one butterfly group at a time).
template <int SF, bool FAST>
__device__ __forceinline__ void wpass2_s2(cf32 (&v)[64], const WTw<SF>& T, const cf32* __restrict__ tw, int l) {
    cf32 w2[3];
#pragma unroll
    for (int q = 1; q <= 3; ++q) w2[q - 1] = FAST ? T.t2[q - 1] : tw[16 * l * q];
#pragma unroll
    for (int b = 0; b < 16; ++b)
        wbfly4<FAST>(v[4 * b], v[4 * b + 1], v[4 * b + 2], v[4 * b + 3], w2[0], w2[1], w2[2], false);
}
template <int SF, bool FAST>
__device__ __forceinline__ void wpass2_s10(cf32 (&v)[64], const WTw<SF>& T, const cf32* __restrict__ tw, int l) {
    using W = WGeo<SF>;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        cfence();
        cf32 w[3];
#pragma unroll
        for (int q = 1; q <= 3; ++q) {
            if constexpr (FAST) w[q - 1] = r == 0 ? T.t1[q - 1] : cmul_root(T.t1[q - 1], 4 * r * q);
            else w[q - 1] = tw[4 * (l + W::LPS * r) * q];
        }
#pragma unroll
        for (int gm = 0; gm < 4; ++gm) {
            const int b0 = 16 * gm + r;
            wbfly4<FAST>(v[b0], v[b0 + 4], v[b0 + 8], v[b0 + 12], w[0], w[1], w[2], false);
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        cfence();  // twiddle loads (and products) one butterfly group at a time
        cf32 w[3];
#pragma unroll
        for (int q = 1; q <= 3; ++q) {
            if constexpr (FAST) w[q - 1] = r == 0 ? T.t0[q - 1] : cmul_root(T.t0[q - 1], r * q);
            else w[q - 1] = tw[(l + W::LPS * r) * q];
        }
        wbfly4<FAST>(v[r], v[r + 16], v[r + 32], v[r + 48], w[0], w[1], w[2], false);
    }
}
template <int SF, bool FAST>
__device__ __forceinline__ void wpass2(cf32 (&v)[64], const WTw<SF>& T, const cf32* __restrict__ tw, int l) {
    wpass2_s2<SF, FAST>(v, T, tw, l);
    wpass2_s10<SF, FAST>(v, T, tw, l);
}

// The 64 x LPS transpose between the passes through the wave's buffer.
// Pass-1 group g of lane (h, l) is sub-transform c = l + LPS g, whose block
// B = rev3(c) holds positions LPS B .. LPS B + LPS - 1; pass-2 lane (h, l')
// takes position l' of every block.  Row B at h N + LPS B, column
// swizzled by sw(B): b64 writes (16-lane groups) and reads (32-lane groups)
// meet every bank once.
template <int SF>
__device__ __forceinline__ void wexchange(cf32 (&v)[64], cf32* buf, int h, int l) {
    using W = WGeo<SF>;
    char* b8 = reinterpret_cast<char*>(buf);
#pragma unroll
    for (int g = 0; g < W::SPW; ++g) {
        const int B = W::rev3(l + W::LPS * g);
        const int lb = ((h * W::SS + B * W::LPS) << 3) | (W::sw(B) << 3);
#pragma unroll
        for (int p = 0; p < W::LPS; ++p) lds_st(buf, lb ^ (p << 3), v[W::reg1(g, p)]);
    }
    // a wave's LDS operations run in issue order: the reads see the writes
    asm volatile("" ::: "memory");
    (void)b8;
    const int rb = (h * W::SS) << 3;
#pragma unroll
    for (int Bp = 0; Bp < 64; ++Bp) v[Bp] = lds_ld(buf, rb + ((Bp * W::LPS) << 3) + ((l ^ W::sw(Bp)) << 3));
}

// One unit's LDS-DMA.  Symbol unit: frame f's symbols s0, s0 + 1, ... (time
// shift t_off) from half 0 up to the frame's end, then (units spanning
// frames, SF 7-10) n1 halves of frame f1's symbols 0, 1, ... (shift t1).
// Estimate unit (est): SF 12 symbol s0 of frame f; below, the EPU frames
// f + j fstride, j < nest, symbols 0 and 1 in halves 2j, 2j + 1.  on = 0:
// no unit.
struct WDma {
    unsigned f, s0;
    int t_off;
    int est, on;
    unsigned fstride, nest;
    unsigned f1;
    int t1;
    unsigned n1;
};

// LDS-DMA of one unit's windows into the wave's buffer: symbol h of the
// unit at h SS.  Halves without a symbol (an estimate unit's halves past the
// two estimate symbols, a frame's last unit's halves past its last symbol)
// load nothing: their lanes compute on whatever the buffer holds, and
// nothing of them is used (round 4 loaded a valid window for them: at SF 9
// 48 KiB per frame, 18 % more than the frame's 270 KiB).
template <int SF>
__device__ __forceinline__ void wdma(const DemodArgs& A, cf32* buf, const WDma& d, int lane) {
    using W = WGeo<SF>;
    typedef __attribute__((address_space(3))) void lds_void;
    typedef __attribute__((address_space(1))) const void g_void;
    const unsigned S = (unsigned)A.total_syms;
    // one symbol window (src: this lane's first sample of it) into the
    // buffer at dst
    auto piece = [&](const cf32* src, cf32* dst) __attribute__((always_inline)) {
        // four 1 KiB pieces per base: the instruction's immediate offset moves
        // the source and the LDS destination alike (tools/ubench/glds_align);
        // SF 7-8: one or two pieces per symbol
#pragma unroll
        for (int r = 0; r < W::PPS; r += 4) {
            g_void* g = (g_void*)(src + 128 * r);
            lds_void* ld = (lds_void*)(dst + 128 * r);
            __builtin_amdgcn_global_load_lds(g, ld, 16, 0, LPHY_IQ_CPOL);
            if constexpr (W::PPS >= 2) __builtin_amdgcn_global_load_lds(g, ld, 16, 1024, LPHY_IQ_CPOL);
            if constexpr (W::PPS >= 4) {
                __builtin_amdgcn_global_load_lds(g, ld, 16, 2048, LPHY_IQ_CPOL);
                __builtin_amdgcn_global_load_lds(g, ld, 16, 3072, LPHY_IQ_CPOL);
            }
        }
    };
    // (loops, not unrolled: the halves' wave-uniform addresses would
    // otherwise all be live at once and spill SGPRs.  The frame's address and
    // the time shift's range are hoisted and the windows of a run of shifted
    // symbols advance by N, so below 8 lanes per symbol, where a unit has 16
    // or 32 halves, a half costs a few instructions.)
    if (d.est) {
        // SF 12: symbol j; below: half h holds symbol h & 1 of the group's
        // frame h >> 1
        if constexpr (W::SPW == 1) {
            piece(A.iq + (unsigned long long)d.f * A.frame_samples + d.s0 * (unsigned)W::N + 2 * lane, buf);
        } else {
            const unsigned ne = d.nest < (unsigned)(W::SPW / 2) ? d.nest : (unsigned)(W::SPW / 2);
#pragma unroll 1
            for (unsigned jf = 0; jf < ne; ++jf) {
                const cf32* src = A.iq + (unsigned long long)(d.f + jf * d.fstride) * A.frame_samples + 2 * lane;
                piece(src, buf + 2 * jf * W::SS);
                piece(src + W::N, buf + (2 * jf + 1) * W::SS);
            }
        }
        return;
    }
    const unsigned N = (unsigned)W::N, count = (unsigned)A.frame_samples;
    if constexpr (W::SPW == 1) {  // SF 12: one window (wwin, LoRaDemod.cpp:144-150)
        if (d.s0 >= S) return;
        const int t = d.t_off;
        unsigned base = d.s0 * N;
        if (t > 0) {
            if (base + N <= count && (unsigned)t <= count - N - base) base += (unsigned)t;
        } else if (t < 0) {
            const unsigned off = 0u - (unsigned)t;
            if (off <= base) base -= off;
        }
        piece(A.iq + (unsigned long long)d.f * A.frame_samples + base + 2 * lane, buf);
        return;
    }
    // symbols sy0 .. sy0 + nh - 1 of frame f (shift t) into halves h0, h0 + 1, ...
    auto run = [&](unsigned f, int t, unsigned sy0, unsigned nh, unsigned h0) __attribute__((always_inline)) {
        // (debug build: the run's frame, its symbols and halves exist; each
        // window is checked against the frame below)
        bound_check(f, (long long)A.frames);
        if (nh) {
            bound_check(sy0 + nh - 1, (long long)S);
            bound_check(h0 + nh - 1, (long long)W::SPW);
        }
        const cf32* fsrc = A.iq + (unsigned long long)f * A.frame_samples + 2 * lane;
        // the shifted symbols (as above): s_lo .. s_hi
        unsigned s_lo = 0u, s_hi = 0xffffffffu;
        if (t > 0) {
            if (count >= N + (unsigned)t) s_hi = (count - N - (unsigned)t) / N;
            else s_lo = 1u, s_hi = 0u;  // (no shifted window fits)
        } else if (t < 0) {
            s_lo = ((0u - (unsigned)t) + N - 1u) / N;
        }
        // halves [0, ha) unshifted, [ha, hb) shifted, [hb, nh) unshifted
        const unsigned ha = s_lo > sy0 ? (s_lo - sy0 < nh ? s_lo - sy0 : nh) : 0u;
        const unsigned hb0 = s_hi >= sy0 ? (s_hi - sy0 < nh ? s_hi - sy0 + 1u : nh) : 0u;  // (s_hi may be ~0u)
        const unsigned hb = hb0 > ha ? hb0 : ha;
        cf32* const b0 = buf + h0 * W::SS;
        unsigned h = 0;
#pragma unroll 1
        for (; h < ha; ++h) piece(fsrc + (sy0 + h) * N, b0 + h * W::SS);
        {
            const cf32* src = fsrc + (sy0 + h) * N + t;
            cf32* dst = b0 + h * W::SS;
            if (hb > h) {  // (debug build: the shifted run's first and last windows lie in the frame)
                bound_check((long long)(sy0 + h) * N + t, (long long)count - N + 1);
                bound_check((long long)(sy0 + hb - 1) * N + t, (long long)count - N + 1);
            }
#pragma unroll LPHY_DMA_UNROLL
            for (; h < hb; ++h, src += N, dst += W::SS) piece(src, dst);
        }
#pragma unroll 1
        for (; h < nh; ++h) piece(fsrc + (sy0 + h) * N, b0 + h * W::SS);
    };
    const unsigned nh0 = d.s0 < S ? (S - d.s0 < (unsigned)W::SPW ? S - d.s0 : (unsigned)W::SPW) : 0u;
    run(d.f, d.t_off, d.s0, nh0, 0u);
    if (d.n1) run(d.f1, d.t1, 0u, d.n1, nh0);
}

// Keyed top two (see team_argmax2_keyed_first) merged over each symbol's
// LPS lanes without LDS traffic: DPP exchanges inside every 16-lane row
// (xor 1, xor 2, half mirror, mirror: each step pairs disjoint lane sets, so
// every lane ends with its 8- or 16-lane group's top two), then, for 32 or
// 64 lanes per symbol, the rows' results by v_readlane as wave-uniform
// values.  Every lane of symbol h gets its top two.
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u32(unsigned v) {
    // (permutations: every lane has a source; no old value, so the move can
    // fold into its consumer)
#ifdef LPHY_AB_DPP_OLD  // A/B timing only: the old-value form
    return (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false);
#else
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
#endif
}
__device__ __forceinline__ void top2_add(unsigned& K1, unsigned& K2, unsigned o1, unsigned o2) {
    K2 = med3_u32(K1, o1, K2 > o2 ? K2 : o2);
    K1 = K1 > o1 ? K1 : o1;
}
template <int LPS>
__device__ __forceinline__ void wave_top2_merge(unsigned k1, unsigned k2, int h, unsigned& K1, unsigned& K2) {
    static_assert(LPS >= 2 && LPS <= 64 && (LPS & (LPS - 1)) == 0, "2 to 64 lanes per symbol");
    top2_add(k1, k2, dpp_u32<0xB1>(k1), dpp_u32<0xB1>(k2));    // quad_perm [1,0,3,2]
    if constexpr (LPS == 2) {
        K1 = k1;
        K2 = k2;
        return;
    }
    top2_add(k1, k2, dpp_u32<0x4E>(k1), dpp_u32<0x4E>(k2));    // quad_perm [2,3,0,1]
    if constexpr (LPS == 4) {
        K1 = k1;
        K2 = k2;
        return;
    }
    top2_add(k1, k2, dpp_u32<0x141>(k1), dpp_u32<0x141>(k2));  // row_half_mirror
    if constexpr (LPS == 8) {  // every lane holds its 8-lane symbol's top two
        K1 = k1;
        K2 = k2;
        return;
    }
    top2_add(k1, k2, dpp_u32<0x140>(k1), dpp_u32<0x140>(k2));  // row_mirror
    if constexpr (LPS == 16) {
        K1 = k1;
        K2 = k2;
        return;
    }
    unsigned r1[4], r2[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        r1[r] = (unsigned)__builtin_amdgcn_readlane((int)k1, 16 * r);
        r2[r] = (unsigned)__builtin_amdgcn_readlane((int)k2, 16 * r);
    }
    top2_add(r1[0], r2[0], r1[1], r2[1]);
    top2_add(r1[2], r2[2], r1[3], r2[3]);
    if constexpr (LPS == 64) {
        top2_add(r1[0], r2[0], r1[2], r2[2]);
        K1 = r1[0];
        K2 = r2[0];
    } else {
        K1 = h ? r1[2] : r1[0];
        K2 = h ? r2[2] : r2[0];
    }
}

__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }   // vmcnt(0)

// LDS-DMA of the KISS twiddle table (N complex) into the wave's buffer.
template <int SF>
__device__ __forceinline__ void wdma_table(const cf32* tw, cf32* buf, int lane) {
    using W = WGeo<SF>;
    typedef __attribute__((address_space(3))) void lds_void;
    typedef __attribute__((address_space(1))) const void g_void;
#pragma unroll
    for (int r = 0; r < W::PPS; r += 4) {
        g_void* g = (g_void*)(tw + 128 * r + 2 * lane);
        lds_void* d = (lds_void*)(buf + 128 * r);
        __builtin_amdgcn_global_load_lds(g, d, 16, 0, 0);
        if constexpr (W::PPS >= 2) __builtin_amdgcn_global_load_lds(g, d, 16, 1024, 0);
        if constexpr (W::PPS >= 4) {
            __builtin_amdgcn_global_load_lds(g, d, 16, 2048, 0);
            __builtin_amdgcn_global_load_lds(g, d, 16, 3072, 0);
        }
    }
}
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); } // lgkmcnt(0)

// Element e (per-lane index, -1: none) of the lane's registers.
__device__ __forceinline__ cf32 wpick(const cf32 (&v)[64], int e) {
    cf32 r = czero();
#pragma unroll
    for (int k = 0; k < 64; ++k) r = e == k ? v[k] : r;
    return r;
}

// Detector outputs of an estimate unit (LoRaDetector.hpp:39-74; as
// unit_result): the exact first maximum of |X|^2 over the half's bins
// l + LPS B', its neighbours' magnitudes and its phase.  Every lane of the
// half gets the result.
template <int SF>
__device__ __forceinline__ UnitResult wunit_result(const cf32 (&v)[64], int h, int l, int lane) {
    using W = WGeo<SF>;
    constexpr int N = W::N;
    ArgMax best{0.0f, 0x7fffffff};
#pragma unroll
    for (int e = 0; e < 64; ++e) {  // bins l + LPS e increase with e
        const cf32 sq = v[e] * v[e];
        const float m2 = sq.x + sq.y;
        const bool take = m2 > best.v;
        best.v = take ? m2 : best.v;
        best.i = take ? l + W::LPS * e : best.i;
    }
#pragma unroll
    for (int off = W::LPS / 2; off >= 1; off >>= 1) {
        ArgMax o;
        o.v = __shfl_xor(best.v, off, 64);
        o.i = __shfl_xor(best.i, off, 64);
        best = better(best, o);
    }
    if (!(best.v > 0.0f)) best.i = 0;  // nothing beat maxValue = 0
    const int idx = best.i;
    const int il = idx > 0 ? idx - 1 : N - 1, ir = idx < N - 1 ? idx + 1 : 0;
    // the lanes holding bins il, idx, ir pick them; three broadcasts
    const int hb = h * W::LPS;
    cf32 lb, bn, rb;
    if constexpr (W::LPS >= 4) {  // three distinct lanes
        int e = -1;
        if (l == (il & (W::LPS - 1))) e = il / W::LPS;
        if (l == (idx & (W::LPS - 1))) e = idx / W::LPS;
        if (l == (ir & (W::LPS - 1))) e = ir / W::LPS;
        const cf32 mine = wpick(v, e);
        auto get = [&](int bin) {
            const int src = hb + (bin & (W::LPS - 1));
            return cf32{__shfl(mine.x, src, 64), __shfl(mine.y, src, 64)};
        };
        lb = get(il);
        bn = get(idx);
        rb = get(ir);
    } else {  // SF 7 (2 lanes per symbol): il and ir share a lane
        auto get = [&](int bin) {
            const cf32 mine = wpick(v, l == (bin & (W::LPS - 1)) ? bin / W::LPS : -1);
            const int src = hb + (bin & (W::LPS - 1));
            return cf32{__shfl(mine.x, src, 64), __shfl(mine.y, src, 64)};
        };
        lb = get(il);
        bn = get(idx);
        rb = get(ir);
    }
    (void)lane;
    UnitResult r;
    const float mv = best.v > 0.0f ? best.v : 0.0f;
    const float fund = sqrtf(mv);
    const float left = lphy_libm::cabsf_exact(lb.x, lb.y);
    const float right = lphy_libm::cabsf_exact(rb.x, rb.y);
    const double demon = (2.0 * (double)fund) - (double)right - (double)left;
    r.idx = idx;
    r.valid = mv > 0.0f;
    r.findex = demon == 0.0 ? 0.0f : (float)(0.5 * (double)(right - left) / demon);
    r.phase = lphy_libm::atan2f_exact(bn.y, bn.x);
    r.nan = 0;
    return r;
}

// ---------------------------------------------------------------------------
// Parseval certificate (round 5): a symbol unit proven without its FFT.
//
// The fast path above transforms every symbol and certifies the winner
// against the runner-up.  A clean symbol - one tone after the dechirp and the
// rotation - carries nearly all of its energy in one bin, and then the winner
// can be proven from that one bin alone: by Parseval, sum_j |Y_j|^2 =
// N sum_n |y_n|^2 = N E for the exact DFT Y of the staged samples y, so every
// other bin obeys |Y_j| <= sqrt(N E - |Y_k|^2).  With B the certificate's
// bound on | |X_ref_j| - |Y_j| | (the rotation's and KISS's roundings, as
// cert_bound charges them; our own FFT's roundings are not incurred here),
// KISS's argmax is k once
//     |Y_k| - sqrt(N E - |Y_k|^2) > 2 B
// (strict: k beats every other bin, so the detector's first-maximum rule,
// LoRaDetector.hpp:46-58, picks it); the kernels ask for 4 B like the
// runner-up certificate.  Per half (symbol) of a unit:
//   * a candidate k: the lag-1 autocorrelation across lanes (DPP row_shl:1,
//     samples 0 .. 8 LPS - 1) gives k coarsely, the lag-LPS one inside each
//     lane (samples i, i + LPS: arg = 2 pi k / 64) gives k mod 64; a wrong
//     candidate only fails the test;
//   * Y_k = sum_l W^{k l} sum_a W_8^{k a} sum_b y[l + LPS (8 a + b)] W_64^{k b}
//     (W_64 / W_8 powers: the correctly rounded 64th roots, read from a
//     register table by ds_bpermute; W^{k l} = W_64^{m / LPS} W_N^{m mod LPS}
//     for m = k l mod N, from that table and a second one of the KISS
//     entries W_N^s, s < LPS), and E, both with per-lane partial sums and a
//     tree over the symbol's lanes;
//   * the samples are taken before the frame's rotation, which is folded
//     into the twiddles (pv_lane_sums): the staging then skips the two
//     rotation products per sample, and only a failed unit applies them;
//   * |dY_k| <= kPvErr u A (A = N sqrt2 amax >= sum |y_n|): the folded
//     twiddle products (<= 3 u each, two), fused products and 8-term partial
//     sums (<= 16 u each, two stages), W^{k l} (the KISS entry W_N^s <= 7.3 u
//     from the ideal root, root64 <= 1 u, their fused product <= 2 u: <= 10.3
//     u) and its product (3 u), the tree (<= 6 u): < 58 u; E's relative error (8-term
//     partial sums, the tree, scale^2) < 26 u (charged 32 u);
//   * lead = Ylo - sqrt(max(0, N E (1 + 32 u) - Ylo^2)) (1 + 4 u) with
//     Ylo = sqrt(|Y_k|^2) (1 - 4 u) - kPvErr u A (v_sqrt within 2 u, the
//     square's rounding within 2 u), certified when lead > 4 B.
// A unit whose every live symbol passes skips pass 1, the exchange, pass 2
// and the top two (~3x fewer VALU instructions at SF 12); otherwise it runs
// them as before.  After a failed unit the frame's remaining units go
// straight to the transform (noisy frames pay one attempt per frame).  The
// speculative normalisation's lead ratio of a Parseval-certified symbol is
// lead / B: a lower bound of the exact winner's lead over every other bin,
// as the runner-up certificate's is.
// ---------------------------------------------------------------------------
constexpr float kPvErr = 64.0f;

// Test build: symbols certified by Parseval, summed in counters[kCtrParseval]
// (lphy_hip_test_counter; tests/test_gpu_parseval.py).
__device__ __forceinline__ void pv_count(const DemodArgs& A, bool mine) {
#ifdef LPHY_TEST_PATHS
    const unsigned long long m = __ballot(mine);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&A.counters[kCtrParseval], (unsigned long long)__popcll(m));
#else
    (void)A;
    (void)mine;
#endif
}

template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// Sum over the LPS lanes of each symbol (every lane gets its symbol's sum).
template <int LPS>
__device__ __forceinline__ float half_sum(float x) {
    static_assert(LPS >= 2 && LPS <= 64 && (LPS & (LPS - 1)) == 0, "2 to 64 lanes per symbol");
    x = x + dpp_f32<0xB1>(x);                             // quad_perm [1,0,3,2]
    if constexpr (LPS >= 4) x = x + dpp_f32<0x4E>(x);     // quad_perm [2,3,0,1]
    if constexpr (LPS >= 8) x = x + dpp_f32<0x141>(x);    // row_half_mirror: the 8-lane sum
    if constexpr (LPS >= 16) x = x + dpp_f32<0x140>(x);  // row_mirror: 16
    if constexpr (LPS >= 32) x = x + __shfl_xor(x, 16, 64);
    if constexpr (LPS >= 64) x = x + __shfl_xor(x, 32, 64);
    return x;
}
// Max over the LPS lanes of each symbol, by DPP as half_sum (mode 0's
// per-symbol amax: no LDS round trip of __shfl_xor in the unit's path).
template <int LPS>
__device__ __forceinline__ float half_max(float x) {
    static_assert(LPS >= 2 && LPS <= 64 && (LPS & (LPS - 1)) == 0, "2 to 64 lanes per symbol");
    x = fmaxf(x, dpp_f32<0xB1>(x));                             // quad_perm [1,0,3,2]
    if constexpr (LPS >= 4) x = fmaxf(x, dpp_f32<0x4E>(x));     // quad_perm [2,3,0,1]
    if constexpr (LPS >= 8) x = fmaxf(x, dpp_f32<0x141>(x));    // row_half_mirror
    if constexpr (LPS >= 16) x = fmaxf(x, dpp_f32<0x140>(x));  // row_mirror
    if constexpr (LPS >= 32) x = fmaxf(x, __shfl_xor(x, 16, 64));
    if constexpr (LPS >= 64) x = fmaxf(x, __shfl_xor(x, 32, 64));
    return x;
}
// root64(idx) for a per-lane idx from the register table rr = root64(lane)
__device__ __forceinline__ cf32 pv_root(cf32 rr, int idx) {
    return cf32{__int_as_float(__builtin_amdgcn_ds_bpermute((idx & 63) << 2, __float_as_int(rr.x))),
                __int_as_float(__builtin_amdgcn_ds_bpermute((idx & 63) << 2, __float_as_int(rr.y)))};
}
// acc + y * w (complex), two fused packed ops
__device__ __forceinline__ cf32 cmac(cf32 acc, cf32 y, cf32 w) {
    cf32 t, r;
    // t = (acc.x + y.x w.x, acc.y + y.x w.y)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(t) : "v"(y), "v"(w), "v"(acc));
    // r = (t.x - y.y w.y, t.y + y.y w.x)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r) : "v"(y), "v"(w), "v"(t));
    return r;
}

// acc + (y.x^2, y.y^2), one packed fma
__device__ __forceinline__ cf32 pk_fma_sq(cf32 acc, cf32 y) {
    cf32 r;
    asm("v_pk_fma_f32 %0, %1, %1, %2" : "=v"(r) : "v"(y), "v"(acc));
    return r;
}

// The candidate bin of each symbol of the unit (every lane of the symbol
// gets it).  v[e]: sample l + LPS e of the lane's symbol before the frame's
// rotation e^{j rate i} (which shifts every lag-d autocorrelation's phase by
// rate d).
template <int SF>
__device__ __forceinline__ int pv_candidate(const cf32 (&v)[64], int l, float rate) {
    constexpr int N = 1 << SF, LPS = WGeo<SF>::LPS;
    constexpr float kInv2Pi = 0.159154943f;
    // lag 1: sample i + 1 sits in lane l + 1 of the same row (DPP row_shl:1;
    // a row's last lane, and a symbol's last lane, have no partner)
    float zr = 0.0f, zi = 0.0f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float nx = dpp_f32<0x101>(v[e].x), ny = dpp_f32<0x101>(v[e].y);
        zr = fmaf(v[e].x, nx, zr);
        zr = fmaf(v[e].y, ny, zr);
        zi = fmaf(v[e].x, ny, zi);
        zi = fmaf(-v[e].y, nx, zi);
    }
    if ((l & 15) == 15 || (l % LPS) == LPS - 1) zr = zi = 0.0f;
    // lag LPS inside the lane: arg = 2 pi k / 64
    float wr = 0.0f, wi = 0.0f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        wr = fmaf(v[e].x, v[e + 1].x, wr);
        wr = fmaf(v[e].y, v[e + 1].y, wr);
        wi = fmaf(v[e].x, v[e + 1].y, wi);
        wi = fmaf(-v[e].y, v[e + 1].x, wi);
    }
    zr = half_sum<LPS>(zr);
    zi = half_sum<LPS>(zi);
    wr = half_sum<LPS>(wr);
    wi = half_sum<LPS>(wi);
    const int kc = (int)rintf((atan2f(zi, zr) + rate) * (kInv2Pi * (float)N));
    const int k64 = (int)rintf((atan2f(wi, wr) + rate * (float)LPS) * (kInv2Pi * 64.0f));
    int d = (k64 - kc) & 63;
    d = d >= 32 ? d - 64 : d;
    return (kc + d) & (N - 1);
}

// The lane's share of Y_k before its factor W^{k l} (the caller applies it:
// the table entry's load is issued early) and the lane's share of sum |p|^2.
// v[e] = p: the sample before the rotation, which is folded into the
// twiddles: y_i W^{k i} = p_i (Qr[b] W_64^{k b}) (Pr[a] W_8^{k a}) W^{k l}
// for i = l + LPS (8 a + b) (Qr carries the normalisation's scale; the
// caller multiplies E by scale^2).
template <int SF>
__device__ __forceinline__ void pv_lane_sums(const cf32 (&v)[64], int k, cf32 rr, const cf32 (&Qr)[8],
                                             const cf32 (&Pr)[8], cf32& yk, float& e) {
    cf32 q[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) q[b] = b == 0 ? Qr[0] : cmul_fma(pv_root(rr, k * b), Qr[b]);
    cf32 acc = czero();
    cf32 e2 = czero();  // (sum re^2, sum im^2), 8-term partial sums
#pragma unroll
    for (int a = 0; a < 8; ++a) {
        cf32 in = cmul_fma(v[8 * a], q[0]);
        cf32 ep = v[8 * a] * v[8 * a];
#pragma unroll
        for (int b = 1; b < 8; ++b) {
            in = cmac(in, v[8 * a + b], q[b]);
            ep = pk_fma_sq(ep, v[8 * a + b]);
        }
        e2 = e2 + ep;
        const cf32 t = a == 0 ? Pr[0] : cmul_fma(pv_root(rr, 8 * k * a), Pr[a]);
        acc = a == 0 ? cmul_fma(in, t) : cmac(acc, in, t);
    }
    yk = acc;
    e = e2.x + e2.y;
}

// The certificate's lead of a symbol from its lanes' shares (summed here).
template <int SF>
__device__ __forceinline__ float pv_lead(cf32 yk, float e, float scale2, float am) {
    constexpr int N = 1 << SF, LPS = WGeo<SF>::LPS;
    const float yr = half_sum<LPS>(yk.x), yi = half_sum<LPS>(yk.y);
    const float E = half_sum<LPS>(e) * scale2;  // sum |y|^2 = scale^2 sum |p|^2
    const float A = (float)N * 1.41421366f * am * 1.0001f;
    const float y2 = __builtin_fmaf(yr, yr, yi * yi);
    const float ylo = __builtin_amdgcn_sqrtf(y2) * (1.0f - 4.0f * kU) - kPvErr * kU * A;
    const float rest = fmaxf(0.0f, (float)N * E * (1.0f + 32.0f * kU) - ylo * ylo * (1.0f - 4.0f * kU));
    const float lead = ylo - __builtin_amdgcn_sqrtf(rest) * (1.0f + 4.0f * kU);
    // finite, normal and in range (a NaN fails every comparison)
    return (y2 >= 1e-30f && y2 < 1e30f && E < 1e30f && ylo > 0.0f) ? lead : -1.0f;
}

// The rare parts of k_wave live in functions of their own (not inlined):
// their registers then never compete with the symbol units' 64-value
// transform, and the few calls per frame cost a spill of the loop state.

// Another half's estimate unit result (lanes of half h: src = first lane of
// the half wanted).
__device__ __forceinline__ UnitResult wur_from(const UnitResult& u, int src) {
    UnitResult r;
    r.idx = __shfl(u.idx, src, 64);
    r.valid = __shfl(u.valid, src, 64);
    r.findex = __shfl(u.findex, src, 64);
    r.phase = __shfl(u.phase, src, 64);
    r.nan = __shfl(u.nan, src, 64);
    return r;
}

// An estimate unit from the wave's buffer (SF 12: one estimate symbol; SF
// 9-11: symbols 0 and 1 in halves 0 and 1): KISS's exact transform and the
// detector outputs; .nan when a bin is NaN (the frame then goes to the exact
// re-run, as in k_frames).  Modes 1/2 normalise with the max-abs `mx`, or
// with find_mx with the max-abs folded here from the unit's own samples, as
// the reference's normalisation scans them (LoRaDemod.cpp:60-78; NaN when one
// is not finite): SF 7-11 both estimate symbols' (both are in the unit), SF
// 12 this symbol's folded with `mx` (0, or symbol 0's for symbol 1).  No
// blocking pre-scan of the frame is then needed.  Returns the max-abs used.
struct WEstU {
    UnitResult ur;
    float mx;
};
template <int SF, int MODE>
__device__ __forceinline__ WEstU west_unit(KArgs ka, lds_cf32* lbuf, const lds_cf32* ldnl, float mx, bool find_mx,
                                        unsigned nlive) {
    using W = WGeo<SF>;
    constexpr int LPS = W::LPS, SPW = W::SPW;
    constexpr bool M0 = (MODE & 3) == LPHY_MODE_DEMODULATE;
    constexpr bool DECH = (MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE;
    const DemodArgs& A = kargs(ka);
    cf32* const buf = (cf32*)lbuf;  // LDS (the cast keeps the address space known)
    const cf32* const dnl = (const cf32*)ldnl;
    const int lane = threadIdx.x & 63, h = lane / LPS, l = lane % LPS;
    cf32 v[64];
    const int rb = (h * W::SS + l) << 3;
#pragma unroll
    for (int e = 0; e < 64; ++e) {
        if ((e & 7) == 0) cfence();
        cf32 x = lds_ld(buf, rb + ((LPS * e) << 3));
        if constexpr (DECH) x = cmul(x, dnl[l + LPS * e]);
        v[e] = x;
    }
    // (SF 7-11: halves 2j, 2j + 1 hold frame j's two estimate symbols, j <
    // nlive; the other halves hold nothing of use)
    const bool live_frame = SPW == 1 || (unsigned)(h >> 1) < nlive;
    if constexpr (!M0) {
        if (find_mx) {
            float fm = 0.0f;
            cf32 sum = czero();
            if (live_frame) {
#pragma unroll
                for (int e = 0; e < 64; ++e) {
                    fm = max3_abs(fm, v[e].x, v[e].y);
                    sum = sum + v[e];
                }
            }
            const bool bad = !(sum.x == sum.x && sum.y == sum.y) || !(fm <= 3.40282347e38f);
            // over the frame's two halves (2 LPS lanes; SF 12: the wave)
#pragma unroll
            for (int off = LPS < 32 ? LPS : 32; off >= 1; off >>= 1) fm = fmaxf(fm, __shfl_xor(fm, off, 64));
            constexpr unsigned long long PM = 2 * LPS >= 64 ? ~0ull : ((1ull << (2 * LPS)) - 1ull);
            const unsigned pair = SPW == 1 ? 0u : (unsigned)(lane / (2 * LPS));
            // (SF 12: folded with the max-abs `mx` of the frame's other estimate
            // symbol, NaN staying NaN)
            mx = (((__ballot(bad) >> (pair * 2 * LPS)) & PM) != 0 || !(mx == mx)) ? __builtin_nanf("")
                                                                                  : fmaxf(mx, fm);
        }
    }
    lphy_frame_meta nm{};
    nm.scale = 1.0f;
    if constexpr (!M0) nm = norm_meta_hot(mx, true, A.no_scratch);
    const bool live = live_frame && nm.status == 0;
    // (k_wave's windowed form: the Hann window's N floats right after the
    // down-chirp in LDS, ldnl + N; mode 1: at ldnl itself)
    constexpr bool WIN = (MODE & kWinBit) != 0;
    const float* const wl = reinterpret_cast<const float*>(dnl + ((MODE & 3) != LPHY_MODE_LORA_DEMODULATE ? W::N : 0));
#pragma unroll
    for (int e = 0; e < 64; ++e) {
        cf32 x = v[e];
        if constexpr (!M0) x = cscale(x, nm.scale);
        if constexpr (WIN) x = cscale(x, wl[l + LPS * e]);  // samp *= window[i] (LoRaDemod.cpp:97-98, phy.cpp:110-111)
        v[e] = live ? x : czero();
    }
    const WTw<SF> T{};  // unused by the exact pass
    wpass1<SF, false>(v, ctw(A.tw));
    wexchange<SF>(v, buf, h, l);
    // pass 2's per-lane twiddles from an LDS copy of the KISS table: one
    // LDS-DMA round trip instead of one global round trip per butterfly group
    wait_lgkm0();  // the exchange reads are done: the buffer is free
    wdma_table<SF>(A.tw, buf, lane);
    wait_vm0();
    wpass2<SF, false>(v, T, buf, l);
    float sumsq = 0.0f;
#pragma unroll
    for (int e = 0; e < 64; ++e) {
        const cf32 sq = v[e] * v[e];
        sumsq += sq.x + sq.y;
    }
    const unsigned long long nb = __ballot(!(sumsq == sumsq));
    WEstU r;
    r.ur = wunit_result<SF>(v, h, l, lane);
    r.ur.nan = (LPS == 64 ? nb : ((nb >> (LPS * h)) & ((1ull << (LPS & 63)) - 1))) != 0 ? 1 : 0;
    if (!live) r.ur = UnitResult{0, 0, 0.0f, 0.0f, 0};
    r.mx = mx;
    return r;
}

// The frame's rotation tables: q[b] = [scale] e^{j rate (l + LPS b)} for the
// lane, and p = e^{j rate 8 LPS (lane & 7)} (the caller takes p of lanes 0..7
// as the wave-uniform table).
struct WRot {
    cf32 q[8];
    cf32 p;
};
template <int SF, int MODE>
__device__ __forceinline__ WRot wrot(float rate, float scale) {
    constexpr int LPS = WGeo<SF>::LPS;
    const int lane = threadIdx.x & 63, l = lane % LPS;
    WRot r;
#pragma unroll 1
    for (int b = 0; b < 8; ++b) {
        float sn, cs;
        lphy_libm::sincosf_exact(rate * (float)(l + LPS * b), &sn, &cs);
        cf32 t = cf32{cs, sn};
        if constexpr ((MODE & 3) != LPHY_MODE_DEMODULATE) t = cscale(t, scale);
        // (a select per entry: r.q[b] with the loop's run-time b would put
        // r.q in scratch memory)
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (i == b) r.q[i] = t;
    }
    float sn, cs;
    lphy_libm::sincosf_exact(rate * (float)(8 * LPS * (lane & 7)), &sn, &cs);
    r.p = cf32{cs, sn};
    return r;
}

// Frame end under the speculative normalisation (as k_frames' close): the
// samples no symbol window covers are scanned, then the frame's true
// max-abs confirms the two-symbol normalisation, sends the frame to the
// exact re-run (NaN / inf), or settles it here.  Settling (the frame's
// normalisation differs from the two-symbol prediction): the estimate
// symbols are fetched again into the wave's buffer (once the next unit's
// LDS-DMA `nd` has landed; it is issued again at the end) and re-run with
// the exact scale
// (KISS's arithmetic, as the estimate units); the symbols are kept when the
// time shift is unchanged and every certified symbol's lead covers the
// larger sample bound and the rate difference (settle_frames' rule, with
// r the symbols' least certificate ratio), else the frame goes to k_post's
// exact re-run.
template <int SF, int MODE>
__device__ __forceinline__ void wclose(KArgs ka, lds_cf32* lbuf, const lds_cf32* ldnl, unsigned f, float rate,
                                    float scale, int t_off, float mx01, float m, float r, bool nan, bool open,
                                    const WDma& nd) {
    using W = WGeo<SF>;
    constexpr int N = W::N, LPS = W::LPS, SPW = W::SPW;
    constexpr bool DECH = (MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE;
    const DemodArgs& A = kargs(ka);
    cf32* const buf = (cf32*)lbuf;
    const cf32* const dnl = (const cf32*)ldnl;
    const int lane = threadIdx.x & 63;
    const unsigned S = (unsigned)A.total_syms;
    const unsigned cnt = DECH ? S * N : (unsigned)A.frame_samples;
    const unsigned end = covered_end(S, N, cnt, t_off);
    bool fbad = false;
    if (end < cnt) m = fmaxf(m, wave_range_maxabs<SF, MODE>(A, f, end, cnt, dnl, fbad));
    const float mt = fmaxf(m, mx01);
    const lphy_frame_meta mg = norm_meta(mx01, true, 0), me = norm_meta(mt, true, 0);
    if (nan || fbad || !(mt <= 3.40282347e38f)) {
        if (lane == 0) A.meta[f].status = kStatusFixup;
        return;
    }
    if (me.scale == mg.scale && me.normalised == mg.normalised) return;
    wait_vm0();  // the next unit's IQ has landed in the buffer
    UnitResult ua{0, 0, 0.0f, 0.0f, 0}, ub = ua;
#pragma unroll 1
    for (int j = 0; j < W::NE; ++j) {
        wdma<SF>(A, buf, WDma{f, (unsigned)j, 0, 1, 1, 0u, 1u}, lane);
        wait_vm0();
        const UnitResult ur = west_unit<SF, MODE>(ka, lbuf, ldnl, mt, false, 1u).ur;
        if constexpr (SPW == 1) {
            if (j == 0) ua = ur;
            else ub = ur;
        } else {
            ua.idx = __shfl(ur.idx, 0, 64);
            ua.valid = __shfl(ur.valid, 0, 64);
            ua.findex = __shfl(ur.findex, 0, 64);
            ua.phase = __shfl(ur.phase, 0, 64);
            ua.nan = __shfl(ur.nan, 0, 64);
            ub.idx = __shfl(ur.idx, LPS, 64);
            ub.valid = __shfl(ur.valid, LPS, 64);
            ub.findex = __shfl(ur.findex, LPS, 64);
            ub.phase = __shfl(ur.phase, LPS, 64);
            ub.nan = __shfl(ur.nan, LPS, 64);
        }
    }
    lphy_frame_meta e = me;
    EstFold fold;
    if (ua.valid) fold.add(ua.idx, ua.findex, 0, ua.phase);
    else fold.add(0, 0.0f, 0, 0.0f);
    if (ub.valid) fold.add(ub.idx, ub.findex, 0, ub.phase);
    else fold.add(0, 0.0f, 0, 0.0f);
    fold.finish(e, 2, N, 1);
    const float a = fmaxf(1.0f, mt * scale) * 1.0001f;
    const float b1 = cert_bound<SF>(rate, rate * (float)t_off, 1.0f);
    const float d = fabsf(e.rate - rate) * (1.0f + 4.0f * kU);
    const float A1 = (float)N * 1.41421366f * 1.0001f;
    const bool ok = !ua.nan && !ub.nan && e.t_off == t_off && t_off >= -N && t_off <= N &&
                    r > 4.0f * a + 4.0f * d * (float)N * A1 * a / b1;
    if (lane == 0) {
        e.status = !ok ? kStatusFixup : (open ? kStatusRecheck : 0);
        meta_put_est(&A.meta[f], e);
    }
    if (nd.on) wdma<SF>(A, buf, nd, lane);
}

// Units spanning frames (SF 7-10): a frame whose end overturns its
// speculative normalisation is not re-run at once (wclose would spend a unit
// on two of its halves and expose two DMA round trips per frame); it is
// queued, and EPU queued frames are settled together in one unit: their
// estimate symbols in halves 2j, 2j + 1, each pair transformed with its own
// frame's true max-abs (KISS's arithmetic, as wclose), folded, and the
// symbols kept or the frame sent to the exact re-run by wclose's rule.
// AWGN, tools/noise_ab.py, profiles/r5/noise_ab.txt.
struct WSettle {
    unsigned f;
    float mt, r, rate, scale;
    int t_off, open, pad;
};
typedef __attribute__((address_space(3))) WSettle lds_settle;
template <int SF, int MODE>
__device__ __forceinline__ void wsettle(KArgs ka, lds_cf32* lbuf, const lds_cf32* ldnl, const lds_settle* es,
                                        unsigned n, const WDma& nd, int lane) {
    using W = WGeo<SF>;
    constexpr int N = W::N, LPS = W::LPS;
    typedef __attribute__((address_space(3))) void lds_void;
    typedef __attribute__((address_space(1))) const void g_void;
    const DemodArgs& A = kargs(ka);
    cf32* const buf = (cf32*)lbuf;
    const int h = lane / LPS, l = lane % LPS;
    wait_vm0();  // the next unit's IQ has landed (it is fetched again at the end)
#pragma unroll 1
    for (unsigned j = 0; j < n; ++j) {
        const unsigned fj = es[j].f;
        bound_check(fj, (long long)A.frames);
        const cf32* src = A.iq + (unsigned long long)fj * A.frame_samples + 2 * lane;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
            for (int r = 0; r < W::PPS; r += 4) {
                g_void* g = (g_void*)(src + s * N + 128 * r);
                lds_void* ld = (lds_void*)(buf + (2 * j + s) * W::SS + 128 * r);
                __builtin_amdgcn_global_load_lds(g, ld, 16, 0, LPHY_IQ_CPOL);
                if constexpr (W::PPS >= 2) __builtin_amdgcn_global_load_lds(g, ld, 16, 1024, LPHY_IQ_CPOL);
                if constexpr (W::PPS >= 4) {
                    __builtin_amdgcn_global_load_lds(g, ld, 16, 2048, LPHY_IQ_CPOL);
                    __builtin_amdgcn_global_load_lds(g, ld, 16, 3072, LPHY_IQ_CPOL);
                }
            }
        }
    }
    wait_vm0();
    const unsigned jp = (unsigned)(h >> 1) < n ? (unsigned)(h >> 1) : 0u;
    const lds_settle& q = es[jp];
    const WSettle e{q.f, q.mt, q.r, q.rate, q.scale, q.t_off, q.open, 0};
    const WEstU eu = west_unit<SF, MODE>(ka, lbuf, ldnl, e.mt, false, n);
    const int hb = (h & ~1) * LPS;
    const UnitResult ua = wur_from(eu.ur, hb), ub = wur_from(eu.ur, hb + LPS);
    lphy_frame_meta em = norm_meta(e.mt, true, 0);
    EstFold fold;
    if (ua.valid) fold.add(ua.idx, ua.findex, 0, ua.phase);
    else fold.add(0, 0.0f, 0, 0.0f);
    if (ub.valid) fold.add(ub.idx, ub.findex, 0, ub.phase);
    else fold.add(0, 0.0f, 0, 0.0f);
    fold.finish(em, 2, N, 1);
    const float a = fmaxf(1.0f, e.mt * e.scale) * 1.0001f;
    const float b1 = cert_bound<SF>(e.rate, e.rate * (float)e.t_off, 1.0f);
    const float d = fabsf(em.rate - e.rate) * (1.0f + 4.0f * kU);
    const float A1 = (float)N * 1.41421366f * 1.0001f;
    const bool ok = !ua.nan && !ub.nan && em.t_off == e.t_off && e.t_off >= -N && e.t_off <= N &&
                    e.r > 4.0f * a + 4.0f * d * (float)N * A1 * a / b1;
    if ((h & 1) == 0 && l == 0 && (unsigned)(h >> 1) < n) {
        em.status = !ok ? kStatusFixup : (e.open ? kStatusRecheck : 0);
        meta_put_est(&A.meta[e.f], em);
    }
    if (nd.on) wdma<SF>(A, buf, nd, lane);
}

// A frame's symbol outputs, collected in registers and stored 128 at a time
// (lane t holds entries base + 2t and base + 2t + 1 as a u16 pair), the
// sync symbols (the frame record's sw0, sw1) at the frame's end.  Stored
// unit by unit, each 2-byte store (one to eight per unit) left a partly
// written line that the streaming IQ evicted before its neighbours came:
// ~32 B of HBM writes per 2-byte symbol (round 4's WRITE_SIZE, 13x the
// results at SF 12).  Entries are stored only where a unit put one (data
// symbols of frames whose estimate succeeded; store_symbol's rule).
template <int SF>
struct WOut {
    unsigned acc = 0u, msk = 0u;  // per lane: the pair, its valid bits
    unsigned sw = 0u, swm = 0u;   // wave-uniform: sw0 | sw1 << 16, valid bits
    unsigned f = 0xffffffffu;     // frame (global index) ...
    int base = 0;                 // ... and its data index of lane 0's first entry
    __device__ __forceinline__ void flush(const DemodArgs& A, int lane) {
        if (f != 0xffffffffu) {
            bound_check(f, (long long)A.frames);
            uint16_t* const row = A.syms + (unsigned long long)f * A.out_per_frame + (unsigned)base;
            if (msk & 1u) {
                bound_check(base + 2 * lane, (long long)A.out_per_frame);
                row[2 * lane] = (uint16_t)acc;
            }
            if (msk & 2u) {
                bound_check(base + 2 * lane + 1, (long long)A.out_per_frame);
                row[2 * lane + 1] = (uint16_t)(acc >> 16);
            }
            if (lane == 0 && swm != 0u) {
                if (swm == 3u) {
                    *reinterpret_cast<unsigned*>(&A.meta[f].sw0) = sw;
                } else {
                    if (swm & 1u) A.meta[f].sw0 = (uint16_t)sw;
                    if (swm & 2u) A.meta[f].sw1 = (uint16_t)(sw >> 16);
                }
            }
        }
        acc = msk = sw = swm = 0u;
        f = 0xffffffffu;
    }
    // a symbol unit whose half h holds symbol s0 + h of frame fr (s0 < 0:
    // the halves before -s0 hold another frame's, with pk 0); pk (lane
    // h LPS): 0x10000 | the output when it is stored, else 0
    __device__ __forceinline__ void put(const DemodArgs& A, unsigned fr, int s0, unsigned pk, int lane) {
        constexpr int LPS = WGeo<SF>::LPS, SPW = WGeo<SF>::SPW;
        const int o0 = s0 - 2;  // data index of half 0 (the frame has its sync symbols)
        if (fr != f || o0 + SPW > base + 128) {
            flush(A, lane);
            f = fr;
            base = (o0 > 0 ? o0 : 0) & ~63;
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // sync symbol i: half i - s0
            const int hs = i - s0;
            if (hs >= 0 && hs < SPW) {
                const unsigned v = (unsigned)__builtin_amdgcn_readlane((int)pk, hs * LPS);
                if (v != 0u) {
                    sw = (sw & ~(0xffffu << (16 * i))) | ((v & 0xffffu) << (16 * i));
                    swm |= 1u << i;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int hh = base + 2 * lane + q - o0;  // (>= 2 for the sync halves' data index < 0)
            const bool in = hh >= 0 && hh < SPW;
            const unsigned v = (unsigned)__shfl((int)pk, in ? hh * LPS : 0, 64);
            if (in && (v & 0x10000u)) {
                acc = (acc & ~(0xffffu << (16 * q))) | ((v & 0xffffu) << (16 * q));
                msk |= 1u << q;
            }
        }
    }
};

// Timing experiments only (-DLPHY_PROFILE_PHASES, tools/ubench): per-wave
// clock sums of the unit phases, added to the clock counters at the end.
#ifdef LPHY_PROFILE_PHASES
#define WPH_DECL unsigned long long wph[8] = {}, wpt = clock64();
#define WPH(i)                                  \
    do {                                        \
        const unsigned long long t_ = clock64(); \
        wph[i] += t_ - wpt;                     \
        wpt = t_;                               \
    } while (0)
#define WPH_FLUSH(A)                                                  \
    if ((threadIdx.x & 63) == 0)                                      \
        for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&(A).counters[kCtrClocks + i_], wph[i_]);
#else
#define WPH_DECL
#define WPH(i) \
    do {       \
    } while (0)
#define WPH_FLUSH(A)
#endif

// Unit kinds and the per-wave schedule cursor (see the header comment).
enum : int { kWDead = 0, kWEst = 1, kWSym = 2 };

struct WCursor {
    int phase;      // 0: E(0); 1: D(k) before E(k+1); 2: E(k+1) (frames k+1 .. k+EPU); 3: D(k) after; 4: done
    unsigned k, j;  // frame (wave-local) of the D units; unit index within the phase
    unsigned k0, s0;  // (units spanning frames: the unit's first frame and symbol)
};

template <int SF>
struct WSched {
    unsigned nk, ND, p;
    // first unit of a (possibly empty) phase
    __device__ __forceinline__ void settle(WCursor& c) const {
        for (;;) {
            // (an estimate unit before the end of D(k) when frame k + 1 starts a group)
            if (c.phase == 1 && c.j >= p) {
                c.phase = (c.k + 1 < nk && (c.k + 1) % (unsigned)WGeo<SF>::EPU == 0) ? 2 : 3;
                c.j = c.phase == 2 ? 0 : p;
                continue;
            }
            if (c.phase == 2 && c.j >= (unsigned)WGeo<SF>::NE) { c.phase = 3; c.j = p; continue; }
            if (c.phase == 3 && c.j >= ND) {
                if (++c.k >= nk) { c.phase = 4; return; }
                c.phase = 1; c.j = 0; continue;
            }
            if (c.phase == 0 && c.j >= (unsigned)WGeo<SF>::NE) { c.phase = 1; c.j = 0; continue; }
            return;
        }
    }
    __device__ __forceinline__ WCursor first() const { WCursor c{0, 0, 0}; settle(c); return c; }
    __device__ __forceinline__ WCursor next(WCursor c) const { ++c.j; settle(c); return c; }
    // kind, wave-local frame, unit index (estimate unit / first symbol s = SPW j)
    __device__ __forceinline__ int kind(const WCursor& c) const {
        return c.phase == 4 ? kWDead : (c.phase == 0 || c.phase == 2) ? kWEst : kWSym;
    }
    __device__ __forceinline__ unsigned frame(const WCursor& c) const { return c.phase == 2 ? c.k + 1 : c.k; }
};

// Units spanning frames (SF 7-10, S >= SPW symbols per frame): the wave's
// frames are one stream of nk S symbols, symbol unit j holds stream symbols
// SPW j .. SPW j + SPW - 1 (at most two frames: the end of frame k0 and the
// start of k0 + 1), so no half idles at a frame's end (SF 7: 66 symbols in
// 2.06 units instead of 3).  The estimate unit of group g (frames g EPU ..
// g EPU + EPU - 1) runs two symbol units before the first one that reaches
// the group, as in WSched.  Cursor: phase 2 estimate unit of group k, phase
// 1 symbol unit j (first frame k0, first symbol s0), phase 4 done.
template <int SF>
struct WSchedSpan {
    unsigned nk, S, NDT, NG;
    __device__ __forceinline__ unsigned jE(unsigned g) const {
        if (g == 0) return 0u;
        const unsigned jf = (unsigned)(((unsigned long long)g * (unsigned)WGeo<SF>::EPU * S) / (unsigned)WGeo<SF>::SPW);
        return jf >= 2u ? jf - 2u : 0u;
    }
    __device__ __forceinline__ void settle(WCursor& c) const {
        c.phase = (c.k < NG && c.j >= jE(c.k)) ? 2 : (c.j < NDT ? 1 : 4);
    }
    __device__ __forceinline__ WCursor first() const { WCursor c{0, 0, 0, 0, 0}; settle(c); return c; }
    __device__ __forceinline__ WCursor next(WCursor c) const {
        if (c.phase == 2) {
            ++c.k;
        } else {
            ++c.j;
            c.s0 += (unsigned)WGeo<SF>::SPW;
            if (c.s0 >= S) { c.s0 -= S; ++c.k0; }  // (SPW <= S)
        }
        settle(c);
        return c;
    }
    __device__ __forceinline__ int kind(const WCursor& c) const {
        return c.phase == 4 ? kWDead : c.phase == 2 ? kWEst : kWSym;
    }
    __device__ __forceinline__ unsigned frame(const WCursor& c) const {
        return c.phase == 2 ? c.k * (unsigned)WGeo<SF>::EPU : c.k0;
    }
};

// Frame record the symbol units read (wave-uniform), kept per wave-local
// frame parity: frame k's record is written by its fold, while frame k - 1's
// symbol units still run.
struct WFrame {
    float rate, scale, mx;  // mx: the two estimate symbols' max-abs (modes 1/2)
    int t_off;
    int ok;                 // estimate folded, status 0
};

// waves per workgroup of k_wave<SF, MODE>: 4, but 3 at SF 12 with the
// window (modes 0 / 2: the window's table does not fit beside four 32 KiB
// buffers and the down-chirp; SF 12 mode 1 with the window stays on the
// separate launches, wave_fit: its k_wave spilled 212 B per lane)
template <int SF, int MODE>
__host__ __device__ constexpr int wave_wpb() {
    return (SF == 12 && (MODE & kWinBit) != 0) ? 3 : WGeo<SF>::WPB;
}

template <int SF, int MODE, bool SPAN = false>
__global__ __launch_bounds__(256, 1) void k_wave(FrameArgs P) {
    using W = WGeo<SF>;
    constexpr int N = W::N, LPS = W::LPS, SPW = W::SPW;
    static_assert(!SPAN || (SPW >= 4 && W::RING >= W::EPU + 3), "units spanning frames: SF 7-10");
    constexpr bool M0 = (MODE & 3) == LPHY_MODE_DEMODULATE;
    constexpr bool DECH = (MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE;
    constexpr bool DN = (MODE & 3) != LPHY_MODE_LORA_DEMODULATE;  // down-chirp used
    const DemodArgs& A = P.A;
    const KArgs ka = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
    // one LDS block: the down-chirp at offset 0 (its wrapped index is then
    // the byte address itself), the waves' buffers after it
    // WIN (Hann window): the window's N floats after the down-chirp
    // (west_unit finds them there: wwin_of), the waves' buffers after that
    constexpr bool WIN = (MODE & kWinBit) != 0;
    constexpr int WPB = wave_wpb<SF, MODE>();  // (SF 12 windowed: 3, the LDS)
    constexpr int WOFS = (DN ? N : 0) + (WIN ? N / 2 : 0);  // (cf32 units)
    __shared__ cf32 lds_all[WOFS + WPB * W::BUF];
    __shared__ WFrame frings[WPB][W::RING];  // (EPU > 1: the frame records)
    // SPAN: the rotation tables of the (at most two) frames of a unit, by
    // frame parity: [scale] e^{j rate i}, i < 8 LPS, then e^{j rate 8 LPS a}
    constexpr int RT = 8 * LPS + 8;
    // SPAN mode 0 at SF 7-8 (LDS room): one table per frame instead, t_i =
    // down_i e^{j rate i} (k_frames' mode-0 table, build_rtab), so a sample's
    // dechirp and rotation are one fused product (k_frames' certificate:
    // no charge beyond cert_bound's own, kWaveExtra's two-table share unused)
    constexpr bool M0T = M0 && SPAN && SF <= 8;
    __shared__ cf32 rtabs[SPAN && !M0T ? WPB : 1][2][SPAN && !M0T ? RT : 1];
    __shared__ cf32 m0tabs[M0T ? WPB : 1][2][M0T ? N : 1];
    __shared__ WSettle settles[SPAN ? WPB : 1][SPAN ? W::EPU : 1];  // (SPAN: frames to settle)
    cf32* const dnl = lds_all;
    cf32 (*const sbuf)[W::BUF] = reinterpret_cast<cf32 (*)[W::BUF]>(lds_all + WOFS);
    float* const wtab = reinterpret_cast<float*>(lds_all + (DN ? N : 0));  // (WIN)

    const int tid = threadIdx.x;
    if constexpr (DN) {
        for (int i = tid; i < N; i += 64 * WPB) dnl[i] = A.down[i];
    }
    if constexpr (WIN) {
        for (int i = tid; i < N; i += 64 * WPB) wtab[i] = A.win[i];
    }
    __syncthreads();  // the only workgroup barrier: waves are independent below

    // wave index as a scalar: the schedule below is wave-uniform (SALU, no
    // exec-mask branches) and the LDS-DMA destination needs no readfirstlane
    const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane / LPS, l = lane % LPS;
    cf32* buf = sbuf[wv];
    const unsigned nframes = (unsigned)A.frames;
    const unsigned S = (unsigned)A.total_syms;
    const unsigned Wn = P.waves;
    const unsigned w = blockIdx.x * WPB + wv;
    if (w >= nframes) return;
    typename std::conditional<SPAN, WSchedSpan<SF>, WSched<SF>>::type sch;
    if constexpr (SPAN) {
        sch.nk = (nframes - 1 - w) / Wn + 1;
        sch.S = S;
        sch.NDT = (sch.nk * S + SPW - 1) / SPW;  // (nk S < 2^32: lphy_hip_demod_batch's limit)
        sch.NG = (sch.nk + W::EPU - 1) / W::EPU;
    } else {
        sch.nk = (nframes - 1 - w) / Wn + 1;
        sch.ND = (S + SPW - 1) / SPW;
        sch.p = sch.ND >= 2 ? sch.ND - 2 : 0;
    }
    const bool spec = !M0 && A.spec != 0;

    WTw<SF> T;
    T.load(A.tw, l);

    // frame records: EPU = 1, two in registers by frame parity (frame k + 1's
    // is written while frame k's units run); EPU > 1, a per-wave LDS ring
    // (an estimate unit writes EPU frames' records at once, lane by lane)
    WFrame rec0{0.0f, 1.0f, 0.0f, 0, 0}, rec1 = rec0;
    typedef __attribute__((address_space(3))) WFrame lds_frame;
    lds_frame* const ring = (lds_frame*)frings[wv];
    auto rec = [&](unsigned k) -> WFrame {
        if constexpr (W::EPU > 1) {
            const lds_frame& q = ring[k & (unsigned)(W::RING - 1)];
            return WFrame{q.rate, q.scale, q.mx, q.t_off, q.ok};
        } else {
            return (k & 1) ? rec1 : rec0;
        }
    };
    auto set_rec = [&](unsigned k, const WFrame& r) {
        if (k & 1) rec1 = r;
        else rec0 = r;
    };
    auto fglob = [&](unsigned k) { return w + k * Wn; };
    // the LDS-DMA of unit c: its frame, unit index and the frame's time shift
    auto dma_plan = [&](const WCursor& c) {
        WDma d{0u, 0u, 0, 0, 0, Wn, 1u, 0u, 0, 0u};
        const int kd = sch.kind(c);
        if (kd == kWDead) return d;
        const unsigned kf = sch.frame(c);
        d.f = fglob(kf);
        d.s0 = kd == kWEst || SPAN ? c.j : (unsigned)SPW * c.j;
        d.on = 1;
        d.est = kd == kWEst ? 1 : 0;
        d.nest = (sch.nk - kf) < (unsigned)W::EPU ? (sch.nk - kf) : (unsigned)W::EPU;
        if (kd != kWEst) d.t_off = rec(kf).t_off;
        if constexpr (SPAN) {
            if (kd == kWSym) {
                d.s0 = c.s0;
                const unsigned n0 = S - c.s0 < (unsigned)SPW ? S - c.s0 : (unsigned)SPW;
                if (n0 < (unsigned)SPW && kf + 1 < sch.nk) {
                    d.f1 = fglob(kf + 1);
                    d.t1 = rec(kf + 1).t_off;
                    d.n1 = (unsigned)SPW - n0;
                }
            }
        }
        return d;
    };
    auto dma_unit = [&](const WCursor& c) {
        const WDma d = dma_plan(c);
        if (d.on) wdma<SF>(A, buf, d, lane);
    };

    // rotation of the frame in demodulation: Qr[b] = [scale] e^{j rate (l + LPS b)}
    // per lane, Pr[a] = e^{j rate 8 LPS a} wave-uniform (sample i = l + LPS (8a + b))
    cf32 Qr[8], Pr[8];
    unsigned rot_frame = 0xffffffffu;
    // Parseval certificate: the 64th roots as a register table (lane j holds
    // root64(j)); tried while no unit of the frame has failed it
    const cf32 rr = root64(lane);
    // ... and lane s < LPS holds the KISS entry W_N^s: W^{k l} = root64(m / LPS)
    // W_N^{m mod LPS} (m = k l mod N) from two register tables, so no global
    // load sits between the next unit's LDS-DMA and the lead (its wait would
    // be vmcnt(0): the whole DMA)
    const cf32 rs = A.tw[lane & (LPS - 1)];
    bool pv_on = true;
    // Adaptive attempts (wave-uniform, speed only: the candidate never
    // decides what is stored): after a frame whose attempt failed, the next
    // 2^m - 1 frames skip it (m = consecutive failed frames, at most
    // kPvBackoff), so input that never certifies this way (mode 0's IQ, whose
    // offsets put every tone between two bins; noise) pays one attempt per
    // 2^kPvBackoff frames instead of one per frame; a success resets m.
#ifndef LPHY_PV_BACKOFF  // (-D0: an attempt on every frame, the round-5 rule; timing A/B)
#define LPHY_PV_BACKOFF 6
#endif
    constexpr unsigned kPvBackoff = LPHY_PV_BACKOFF;
    unsigned pv_miss = 0, pv_wait = 0;
    auto pv_frame = [&]() __attribute__((always_inline)) {
        if (pv_wait != 0) {
            --pv_wait;
            pv_on = false;
        } else {
            pv_on = true;
        }
    };
    // speculative normalisation of the frame in demodulation (lane state)
    constexpr float kBig = 3.0e38f;
    float sp_mx = 0.0f, sp_r = kBig;
    unsigned sp_fl = 0u;
    float sp_mx1 = 0.0f, sp_r1 = kBig;  // (SPAN: the odd frames')
    unsigned sp_fl1 = 0u;
    unsigned tab0 = 0xffffffffu, tab1 = 0xffffffffu;  // (SPAN: the frames in rtabs)
    unsigned nset = 0;  // (SPAN: frames queued in settles)
    UnitResult ur0{0, 0, 0.0f, 0.0f, 0};  // SF 12: the first estimate unit's result

    WOut<SF> wo;  // the frame's symbol outputs until they are stored

    WCursor cu = sch.first();
    WPH_DECL
    dma_unit(cu);
    while (sch.kind(cu) != kWDead) {
        const WCursor nx = sch.next(cu);
        const unsigned k = sch.frame(cu), f = fglob(k);
        cf32 v[64];
        WPH(7);
#ifndef LPHY_ABLATE_W_VMWAIT  // timing experiments only
        wait_vm0();  // this unit's IQ has landed
#endif
        WPH(0);
        if (sch.kind(cu) == kWSym) {
            const WFrame R0 = rec(k);
            WFrame R = R0;      // this lane's frame record (SPAN: frame k or k + 1)
            unsigned s, fh = f;  // this lane's symbol and frame (global)
            bool live;
            bool second = false;  // SPAN: the lane's half is in frame k + 1
            unsigned n0 = (unsigned)SPW;
            bool two = false;
            const lds_cf32* mt = nullptr;  // (M0T: the lane's frame's table)
            if constexpr (SPAN) {
                n0 = S - cu.s0 < (unsigned)SPW ? S - cu.s0 : (unsigned)SPW;
                two = n0 < (unsigned)SPW && k + 1 < sch.nk;
                const WFrame R1 = two ? rec(k + 1) : R0;
                if (k != rot_frame) {
                    rot_frame = k;
                    pv_frame();
                }
                // the rotation tables of frames k and k + 1, built once per
                // frame (by parity) by the whole wave: the wrot values
                auto ensure = [&](unsigned kk, const WFrame& Rk) __attribute__((always_inline)) {
                    if (((kk & 1u) ? tab1 : tab0) == kk) return;
                    if (kk & 1u) tab1 = kk;
                    else tab0 = kk;
                    if constexpr (M0T) {
                        lds_cf32* tm = (lds_cf32*)m0tabs[wv][kk & 1u];
#pragma unroll 1
                        for (int i = lane; i < N; i += 64) {
                            float sn, cs;
                            lphy_libm::sincosf_exact(Rk.rate * (float)i, &sn, &cs);
                            cf32 t = cmul(dnl[i], cf32{cs, sn});
                            if constexpr (WIN) t = cscale(t, wtab[i]);  // (build_rtab's order)
                            tm[i] = t;
                        }
                        return;
                    }
                    lds_cf32* tb = (lds_cf32*)rtabs[wv][kk & 1u];
#pragma unroll 1
                    for (int i = lane; i < RT; i += 64) {
                        const bool qp = i < 8 * LPS;
                        float sn, cs;
                        lphy_libm::sincosf_exact(Rk.rate * (float)(qp ? i : 8 * LPS * (i - 8 * LPS)), &sn, &cs);
                        cf32 t = cf32{cs, sn};
                        if constexpr (!M0) {
                            if (qp) t = cscale(t, Rk.scale);
                        }
                        tb[i] = t;
                    }
                };
                ensure(k, R0);
                if (two) ensure(k + 1, R1);
                second = (unsigned)h >= n0;
                s = second ? (unsigned)h - n0 : cu.s0 + (unsigned)h;
                live = !second || two;
                if (second && two) {
                    R = R1;
                    fh = fglob(k + 1);
                }
                if constexpr (M0T) {
                    mt = (const lds_cf32*)m0tabs[wv][(k + (second ? 1u : 0u)) & 1u];
#pragma unroll
                    for (int b = 0; b < 8; ++b) Qr[b] = Pr[b] = cf32{1.0f, 0.0f};  // (rotated in the staging)
                } else {
                    const lds_cf32* tb = (const lds_cf32*)rtabs[wv][(k + (second ? 1u : 0u)) & 1u];
#pragma unroll
                    for (int b = 0; b < 8; ++b) Qr[b] = tb[l + LPS * b];
#pragma unroll
                    for (int a = 0; a < 8; ++a) Pr[a] = tb[8 * LPS + a];
                }
            } else {
                if (k != rot_frame) {
                    rot_frame = k;
                    pv_frame();
                    const WRot rt = wrot<SF, MODE>(R.rate, R.scale);
#pragma unroll
                    for (int b = 0; b < 8; ++b) Qr[b] = rt.q[b];
#pragma unroll
                    for (int a = 0; a < 8; ++a)
                        Pr[a] = cf32{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(rt.p.x), a)),
                                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rt.p.y), a))};
                }
                s = SPW * cu.j + (unsigned)h;
                live = s < S;
            }
            lphy_frame_meta m{};
            m.rate = R.rate;
            m.scale = R.scale;
            m.t_off = R.t_off;
            m.status = R.ok ? 0 : -1;
            m.have_sync = 1;
            const SymCtx c = sym_ctx(A, fh, live ? s : 0u, live, N, m);
            // staging: [exact dechirp,] certified rotation, from the LDS copy
            float amax = 0.0f;
            const int rb = (h * W::SS + l) << 3;
            // software-pipelined in chunks of 8 samples: chunk q + 1's LDS reads
            // are issued before chunk q's arithmetic (sched barriers pin the
            // order; a single wave per SIMD has no other wave to hide them)
#ifndef LPHY_W_STAGE_DEPTH
#define LPHY_W_STAGE_DEPTH 1
#endif
            constexpr int SD = LPHY_W_STAGE_DEPTH, SB = SD + 1;  // chunks in flight, buffers
            cf32 xq[SB][8], dq[SB][8];
            constexpr bool WS = WIN && !M0T;  // the window's product in the staging (M0T: in the table)
            float wq[SB][WS ? 8 : 1];
            // byte address of the down-chirp entry of element 0; element e's
            // is (d0 + 8 LPS e) mod 8 N (mode 2: the window's own chirp indices)
            const unsigned d0 = ((c.base + (unsigned)l) & (unsigned)(N - 1)) << 3;
            auto ld_chunk = [&](int q, cf32 (&xs)[8], cf32 (&ds)[8], float* ws) __attribute__((always_inline)) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int e = 8 * q + i;
                    if constexpr (WS) ws[i] = wtab[l + LPS * e];
#ifndef LPHY_ABLATE_W_STAGE  // timing experiments only
                    xs[i] = lds_ld(buf, rb + ((LPS * e) << 3));
#else
                    xs[i] = cf32{(float)e, (float)l};
#endif
                    if constexpr (DECH) ds[i] = lds_ld(dnl, (int)((d0 + (unsigned)((LPS * e) << 3)) & (unsigned)(8 * N - 1)));
                    if constexpr (M0T) ds[i] = mt[l + LPS * e];
                    else if constexpr (M0) ds[i] = dnl[l + LPS * e];
                }
            };
#pragma unroll
            for (int q = 0; q < SD; ++q) ld_chunk(q, xq[q], dq[q], wq[q]);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                if (q + SD < 8) ld_chunk(q + SD, xq[(q + SD) % SB], dq[(q + SD) % SB], wq[(q + SD) % SB]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int e = 8 * q + i;
                    const cf32 x = xq[q % SB][i];
                    cf32 p = x;
                    if constexpr (DECH) p = cmul(x, dq[q % SB][i]);
                    amax = max3_abs(amax, p.x, p.y);
                    if constexpr (M0T) p = cmul_fma(p, dq[q % SB][i]);  // dechirp and rotation
                    else if constexpr (M0) p = cmul(p, dq[q % SB][i]);
                    // Hann window (after the max-abs: the normalisation scans
                    // the samples themselves, LoRaDemod.cpp:60-78, 154-160)
                    if constexpr (WS) p = cscale(p, wq[q % SB][i]);
                    // (a unit whose symbol is not demodulated transforms whatever
                    // its window holds; nothing of it is stored; the rotation
                    // is applied below, or folded into the Parseval sums)
                    v[e] = p;
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            WPH(1);
            float am = 1.0f;  // modes 1/2: normalised frame (see fast_certified)
            if constexpr (M0) {
                amax = half_max<LPS>(amax);
                am = amax;
            }
            // (WIN: + 2 u for the window's product taken in another order than
            // the reference's, (x [down]) w before the rotation)
            const float cb1 = cert_bound<SF>(c.rate, c.start, 1.0f, kWaveExtra + (WIN ? 2.0f : 0.0f));
            int sym = 0;         // the symbol's bin (certified) ...
            float cgap = -1.0f;  // ... and its certified lead (-1: not certified)
            bool pv = false;     // the whole unit certified by Parseval
            if (pv_on && !A.debug_recheck) {
                // Parseval certificate (above): the candidate, its DFT bin
                // and the energy; the buffer is free after the staging, so
                // the next unit's IQ is on its way meanwhile
                const int kc = pv_candidate<SF>(v, l, M0T ? 0.0f : c.rate);
                const unsigned mkl = (unsigned)(kc * l) & (unsigned)(N - 1);
                const cf32 wkl = cmul_fma(pv_root(rr, (int)(mkl / (unsigned)LPS)), pv_root(rs, (int)(mkl % (unsigned)LPS)));
                WPH(3);  // (timing builds: slots 3 / 4 time the Parseval candidate / DMA issue)
                wait_lgkm0();
                dma_unit(nx);
                WPH(4);
                cf32 ykl;
                float el;
                pv_lane_sums<SF>(v, kc, rr, Qr, Pr, ykl, el);
                const float lead = pv_lead<SF>(cmul_fma(ykl, wkl), el, M0 ? 1.0f : c.scale * c.scale, am);
                const bool ok = lead > 4.0f * (cb1 * am) && (float)N * 1.41421366f * am * 1.0001f < 1e18f &&
                                am >= 1e-20f;
                pv = __ballot(live && c.ok && !ok) == 0;
                if (pv) {
                    pv_count(A, live && c.ok && l == 0);
                    sym = kc;
                    cgap = lead;
                    pv_miss = 0;
                } else {
                    pv_on = false;  // the frame's other units: the transform
                    if (pv_miss < kPvBackoff) ++pv_miss;
                    pv_wait = (1u << pv_miss) - 1u;
                    wait_vm0();     // the early DMA has landed before the exchange reuses the buffer
                }
            }
            WPH(2);
            if (!pv) {
                // the certified rotation (staging left the samples unrotated;
                // M0T: rotated there)
                if constexpr (!M0T) {
#pragma unroll
                    for (int e = 0; e < 64; ++e) v[e] = cmul_fma(cmul_fma(v[e], Qr[e & 7]), Pr[e >> 3]);
                }
                wpass1<SF, true>(v, ctw(A.tw));
#ifndef LPHY_ABLATE_W_EXCH  // timing experiments only
                wexchange<SF>(v, buf, h, l);
#endif
#ifdef LPHY_W_LATE_DMA
                // pass 2's first stage consumes the exchange reads as they land;
                // then the buffer is free for the next unit's IQ
                wpass2_s2<SF, true>(v, T, A.tw, l);
                wait_lgkm0();
                dma_unit(nx);
                WPH(3);
                wpass2_s10<SF, true>(v, T, A.tw, l);
#else
                wait_lgkm0();  // the exchange reads are done: the buffer is free
#ifndef LPHY_ABLATE_W_DMA  // timing experiments only
                dma_unit(nx);  // the next unit's IQ lands during pass 2
#endif
                WPH(3);
                wpass2<SF, true>(v, T, A.tw, l);
#endif
                WPH(4);
                // keyed top two over the half's bins l + LPS e (key: |X|^2 bits,
                // low 6 bits the element; see team_argmax2_keyed_first)
                unsigned k1 = 0u, k2 = 0u;
#pragma unroll
                for (int e = 0; e < 64; e += 2) {
                    // |X|^2 = fma(x, x, fl(y y)): within 2 u, inside cert_gap's 8 u;
                    // scalar f32 ops (no packed-f32 dependency pad)
                    const float ma = __builtin_fmaf(v[e].x, v[e].x, v[e].y * v[e].y);
                    const float mb = __builtin_fmaf(v[e + 1].x, v[e + 1].x, v[e + 1].y * v[e + 1].y);
                    top2_pair(k1, k2, (__float_as_uint(ma) & ~63u) | (unsigned)e,
                              (__float_as_uint(mb) & ~63u) | (unsigned)(e + 1));
                }
                unsigned K1, K2;
                wave_top2_merge<LPS>(k1, k2, h, K1, K2);
                const unsigned long long bm = __ballot(k1 == K1);
                const unsigned long long hm = LPS == 64 ? bm : ((bm >> (LPS * h)) & ((1ull << (LPS & 63)) - 1));
                ArgMax2 b2;
                b2.v = __uint_as_float(K1 & ~63u);
                b2.v2 = __uint_as_float(K2 | 63u);
                b2.i = (__ffsll((long long)hm) - 1) + LPS * (int)(K1 & 63u);
                const float g = cert_gap(b2);
                const bool cert = g > 4.0f * (cb1 * am) && (float)N * 1.41421366f * am * 1.0001f < 1e18f &&
                                  am >= 1e-20f && b2.v >= 1e-30f;
                sym = b2.i;
                cgap = cert && !A.debug_recheck ? g : -1.0f;  // (DEBUG_RECHECK: tests)
            }
            const bool redo = c.ok && !(cgap >= 0.0f);
            {
                const uint16_t out = redo ? kSymRecheck : (uint16_t)sym;
                const bool sync_sym = c.s < 2;  // (have_sync: set above)
                const bool st = live && l == 0 && (sync_sym || c.ok);
                const unsigned pk = st ? (0x10000u | (c.ok ? out : 0u)) : 0u;
                if constexpr (SPAN) {
                    wo.put(A, f, (int)cu.s0, second ? 0u : pk, lane);
                    if (two) wo.put(A, fglob(k + 1), -(int)n0, second ? pk : 0u, lane);
                } else {
                    wo.put(A, f, (int)(SPW * cu.j), pk, lane);
                }
                if (live && l == 0 && redo) A.meta[c.f].status = kStatusRecheck;
                if constexpr (!SPAN) {
                    if (cu.phase == 3 && cu.j + 1 == sch.ND) wo.flush(A, lane);  // the frame's last unit
                }
            }
            if (spec && c.ok) {
                // (SPAN: the state of the lane's frame, by parity)
                const bool p1 = SPAN && (((k + (second ? 1u : 0u)) & 1u) != 0u);
                float smx = p1 ? sp_mx1 : sp_mx, sr = p1 ? sp_r1 : sp_r;
                unsigned sfl = p1 ? sp_fl1 : sp_fl;
                smx = fmaxf(smx, amax);
                const cf32 q = v[0] * v[0];
                const float q2 = q.x + q.y;
                if (!(q2 == q2)) sfl |= 1u;  // a NaN sample reaches every bin
                if (l == 0) {
                    if (redo) sfl |= 2u;
                    else sr = fminf(sr, cgap * __builtin_amdgcn_rcpf(cb1) * (1.0f - 4.0f * kU));
                }
                if (p1) {
                    sp_mx1 = smx;
                    sp_r1 = sr;
                    sp_fl1 = sfl;
                } else {
                    sp_mx = smx;
                    sp_r = sr;
                    sp_fl = sfl;
                }
            }
            WPH(5);
            // the frame's last symbol unit closes it (speculative normalisation)
            bool closes;
            if constexpr (SPAN) closes = cu.s0 + (unsigned)SPW >= S;  // (frame k ends in this unit)
            else closes = cu.phase == 3 && cu.j + 1 == sch.ND;
            if (spec && closes) {
                const bool p1 = SPAN && (k & 1u) != 0u;
                float mm = p1 ? sp_mx1 : sp_mx, rr = p1 ? sp_r1 : sp_r;
                const unsigned fl = p1 ? sp_fl1 : sp_fl;
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    mm = fmaxf(mm, __shfl_xor(mm, off, 64));
                    rr = fminf(rr, __shfl_xor(rr, off, 64));
                }
                const bool nan = __ballot(fl & 1u) != 0, open = __ballot(fl & 2u) != 0;
                if (p1) {
                    sp_mx1 = 0.0f;
                    sp_r1 = kBig;
                    sp_fl1 = 0u;
                } else {
                    sp_mx = 0.0f;
                    sp_r = kBig;
                    sp_fl = 0u;
                }
                if (R0.ok) {
                    if constexpr (SPAN) {
                        // wclose's frame-end check; a settle is queued (wsettle)
                        const unsigned cnt = DECH ? S * N : (unsigned)A.frame_samples;
                        const unsigned end = covered_end(S, N, cnt, R0.t_off);
                        bool fbad = false;
                        if (end < cnt) mm = fmaxf(mm, wave_range_maxabs<SF, MODE>(A, f, end, cnt, dnl, fbad));
                        const float mt = fmaxf(mm, R0.mx);
                        const lphy_frame_meta mg = norm_meta(R0.mx, true, 0), me = norm_meta(mt, true, 0);
                        if (nan || fbad || !(mt <= 3.40282347e38f)) {
                            if (lane == 0) A.meta[f].status = kStatusFixup;
                        } else if (me.scale != mg.scale || me.normalised != mg.normalised) {
                            if (lane == 0)
                                settles[wv][nset] = WSettle{f, mt, rr, R0.rate, R0.scale, R0.t_off, open ? 1 : 0, 0};
                            if (++nset == (unsigned)W::EPU) {
                                wsettle<SF, MODE>(ka, (lds_cf32*)buf, (const lds_cf32*)dnl,
                                                  (const lds_settle*)settles[wv], nset, dma_plan(nx), lane);
                                nset = 0;
                            }
                        }
                    } else {
                        const WDma nd = dma_plan(nx);
                        wclose<SF, MODE>(ka, (lds_cf32*)buf, (const lds_cf32*)dnl, f, R0.rate, R0.scale, R0.t_off,
                                         R0.mx, mm, rr, nan, open, nd);
                    }
                }
            }
            WPH(6);
        } else {
            // estimate unit(s): KISS's arithmetic, bit for bit (LoRaDemod.cpp:80-136,
            // phy.cpp:81-148); SF 12 symbol j, SF 11 symbol h of the pair,
            // SF 7-10 symbol h & 1 of frame k + (h >> 1) of the group
            // (SF 7-11: the unit folds the two estimate symbols' max-abs itself)
            if constexpr (W::EPU > 1) {
                const unsigned nest = (sch.nk - k) < (unsigned)W::EPU ? (sch.nk - k) : (unsigned)W::EPU;
                const WEstU eu = west_unit<SF, MODE>(ka, (lds_cf32*)buf, (const lds_cf32*)dnl, 0.0f, true, nest);
                // every lane folds its own pair's frame; the pair's first lane stores it
                const int hb = (h & ~1) * LPS;
                const UnitResult ua = wur_from(eu.ur, hb), ub = wur_from(eu.ur, hb + LPS);
                lphy_frame_meta m{};
                m.scale = 1.0f;
                m.have_sync = 1;
                if constexpr (!M0) m = norm_meta_hot(eu.mx, true, A.no_scratch);
                if (m.status == 0) {
                    EstFold fold;
                    if (ua.valid) fold.add(ua.idx, ua.findex, 0, ua.phase);
                    else fold.add(0, 0.0f, 0, 0.0f);
                    if (ub.valid) fold.add(ub.idx, ub.findex, 0, ub.phase);
                    else fold.add(0, 0.0f, 0, 0.0f);
                    fold.finish(m, 2, N, 1);
                    if (ua.nan || ub.nan) m.status = kStatusFixup;
                }
                const unsigned kj = k + (unsigned)(h >> 1);
                if ((h & 1) == 0 && l == 0 && (unsigned)(h >> 1) < nest) {
                    bound_check(fglob(kj), (long long)A.frames);
                    meta_put_est(&A.meta[fglob(kj)], m);
                    lds_frame& q = ring[kj & (unsigned)(W::RING - 1)];
                    q.rate = m.rate;
                    q.scale = m.scale;
                    q.mx = eu.mx;
                    q.t_off = m.t_off;
                    q.ok = m.status == 0 ? 1 : 0;
                }
            } else {
                WFrame R0 = rec(k);
                // SF 12: symbol 0's unit normalises with its own max-abs m0 (the
                // speculation that symbol 1 does not change the frame's scale:
                // max-abs <= 1, no scaling, for any signal within the reference's
                // [-1, 1] range), symbol 1's with max(m0, m1); a frame whose
                // symbol 1 changes the scale runs symbol 0's unit again below
                const float mx_in = (SPW > 1 || cu.j == 0) ? 0.0f : R0.mx;
                const WEstU eu = west_unit<SF, MODE>(ka, (lds_cf32*)buf, (const lds_cf32*)dnl, mx_in, true, 1u);
                const UnitResult ur = eu.ur;
                const float m_prev = R0.mx;
                R0.mx = eu.mx;
                lphy_frame_meta nm{};
                nm.scale = 1.0f;
                nm.have_sync = 1;
                if constexpr (!M0) nm = norm_meta_hot(R0.mx, true, A.no_scratch);
                bool fold_now = true;
                UnitResult ua = ur, ub = ur;
                if constexpr (SPW == 1) {
                    if (cu.j == 0) {
                        ur0 = ur;
                        fold_now = false;
                        set_rec(k, R0);  // m0, for symbol 1's unit
                    } else {
                        ua = ur0;
                        if constexpr (!M0) {
                            const lphy_frame_meta n0 = norm_meta_hot(m_prev, true, A.no_scratch);
                            if (nm.status == 0 && n0.status == 0 &&
                                (n0.scale != nm.scale || n0.normalised != nm.normalised)) {
                                wdma<SF>(A, buf, WDma{f, 0u, 0, 1, 1, 0u, 1u}, lane);
                                wait_vm0();
                                ua = west_unit<SF, MODE>(ka, (lds_cf32*)buf, (const lds_cf32*)dnl, R0.mx, false, 1u).ur;
                            }
                        }
                    }
                } else {  // the pair's second estimate unit from the upper half
                    ua = wur_from(ur, 0);
                    ub = wur_from(ur, LPS);
                }
                if (fold_now) {
                    lphy_frame_meta m = nm;
                    if (m.status == 0) {
                        EstFold fold;
                        if (ua.valid) fold.add(ua.idx, ua.findex, 0, ua.phase);
                        else fold.add(0, 0.0f, 0, 0.0f);
                        if (ub.valid) fold.add(ub.idx, ub.findex, 0, ub.phase);
                        else fold.add(0, 0.0f, 0, 0.0f);
                        fold.finish(m, 2, N, 1);
                        if (ua.nan || ub.nan) m.status = kStatusFixup;
                    }
                    if (lane == 0) meta_put_est(&A.meta[f], m);
                    WFrame r = R0;
                    r.rate = m.rate;
                    r.scale = m.scale;
                    r.t_off = m.t_off;
                    r.ok = m.status == 0 ? 1 : 0;
                    set_rec(k, r);
                }
            }
            dma_unit(nx);  // after the fold: a symbol unit's window needs the time shift
            WPH(6);
        }
        // (WPH slot 7 from here to the next unit: the cursor)
        cu = nx;
    }
    wo.flush(A, lane);  // (every frame's last unit has stored it already)
    if constexpr (SPAN) {
        if (nset) {
            const WDma none{0u, 0u, 0, 0, 0, 0u, 1u, 0u, 0, 0u};
            wsettle<SF, MODE>(ka, (lds_cf32*)buf, (const lds_cf32*)dnl, (const lds_settle*)settles[wv], nset, none,
                              lane);
        }
    }
    WPH(7);
    WPH_FLUSH(A)
}
