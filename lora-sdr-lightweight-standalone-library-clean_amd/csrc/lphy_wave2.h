// lphy_wave2.h — the SF 9-10 fused launch at two waves per SIMD with units
// spanning frames (k_wave2s).  Included by lphy_kernels.h after lphy_wave.h,
// whose unit geometry (WGeo: one wavefront per unit of 64 x 64 complex
// values), transform passes, exchange, keyed top two and estimate fold it
// reuses.
//
// k_wave (one 256-thread workgroup per CU, one wave per SIMD) keeps each
// unit's IQ in a per-wave 32 KiB LDS buffer filled by LDS-DMA.  Here:
//   * 512-thread workgroups, 8 independent waves per CU (2 per SIMD, at most
//     256 VGPR + AGPR each): one wave's loads and LDS waits run under its
//     partner's arithmetic;
//   * the unit's IQ goes from HBM straight into the lane's 64 registers
//     (64 coalesced 8-byte loads per lane: lane (h, l) reads samples
//     l + LPS m of its symbol's window), no LDS staging copy;
//   * the 64 x LPS exchange between the passes borrows one of NBUF shared
//     LDS buffers (4 per CU, an LDS compare-and-swap lock each) for the ~130
//     LDS operations it takes, so 8 waves fit beside the down-chirp;
//   * the estimate units fold the two estimate symbols' max-abs from their
//     own registers, with no separate two-symbol scan.
// Round 4 also had k_wave2, the same units one frame at a time: slower than
// k_wave at every SF and removed in round 5.
// Results are bit-identical to k_wave: the same arithmetic in the same
// order on the same values (tests/test_gpu_*: oracle, goldens, k_wave).
//
// Reference: the per-symbol loop of LoRaDemod.cpp:142-176 / phy.cpp:204-238,
// the estimate of LoRaDemod.cpp:80-136 / phy.cpp:81-148, the normalisation
// of LoRaDemod.cpp:60-78.

template <int SF, int MODE>
struct W2Lds {
    using W = WGeo<SF>;
    static constexpr bool DN = (MODE & 3) != LPHY_MODE_LORA_DEMODULATE;  // down-chirp in LDS
    static constexpr int DNC = DN ? W::N : 0;                              // its entries
    static constexpr int NBUF0 = (163840 - 64 - 8 * DNC) / (8 * W::BUF);
    static constexpr int NBUF = NBUF0 > 4 ? 4 : NBUF0;                     // exchange buffers
    static_assert(NBUF >= 2, "two exchange buffers at least");
    static constexpr int WPB = 8;                                          // waves per workgroup
};

typedef __attribute__((address_space(3))) unsigned lds_u32;

// Borrow one of the CU's exchange buffers: lane 0 takes the first free one
// from `start` on by an LDS compare-and-swap (acquire), the wave learns it
// by readfirstlane; with none free the wave sleeps and sweeps again.  A
// holder never waits for anything but its own LDS operations, so every
// wait ends; still, the sweeps are capped (2^20, ~0.1 s, far beyond any
// holder's ~1 us) so that a lost lock can never hang the GPU, and at the cap
// the wave gets -1: it then uses no buffer, and its caller leaves the unit
// to the exact re-run (a symbol: kSymRecheck; an estimate: the frame to
// kStatusFixup), so the outputs stay bit-exact.
// `salt` >= 0 (test build, LPHY_F_DEBUG_LOCKFAIL): one sweep only, and every
// third salt fails outright, so the tests reach the fail-safe path.
template <int NBUF>
__device__ __forceinline__ int wbuf_acquire(lds_u32* locks, int start, int salt) {
    unsigned cap = 1u << 20;
#ifdef LPHY_TEST_PATHS
    if (salt >= 0) {
        if (salt % 3 == 0) return -1;
        cap = 1;
    }
#else
    (void)salt;
#endif
    for (unsigned spin = 0; spin < cap; ++spin) {
        int got = -1;
        if ((threadIdx.x & 63) == 0) {
#pragma unroll
            for (int k = 0; k < NBUF; ++k) {
                int b = start + k;
                b = b >= NBUF ? b - NBUF : b;
                unsigned expected = 0u;
                if (__hip_atomic_compare_exchange_strong((unsigned*)&locks[b], &expected, 1u, __ATOMIC_ACQUIRE,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                    got = b;
                    break;
                }
            }
        }
        got = __builtin_amdgcn_readfirstlane(got);
        if (got >= 0) return got;
        __builtin_amdgcn_s_sleep(2);
    }
    return -1;
}
// Give the buffer back once this wave's reads of it are done (release: the
// compiler orders the store after them; the LDS serves one wave's requests
// in order, so the next holder's writes follow them).
__device__ __forceinline__ void wbuf_release(lds_u32* locks, int b) {
    if ((threadIdx.x & 63) == 0)
        __hip_atomic_store((unsigned*)&locks[b], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// wbuf_acquire's salt: the unit's own number (lane 0's: wave-uniform, as the
// acquisition is) under LPHY_F_DEBUG_LOCKFAIL, -1 otherwise
__device__ __forceinline__ int wlock_salt(const DemodArgs& A, unsigned unit) {
    return A.lock_fail ? (int)((unsigned)__builtin_amdgcn_readfirstlane((int)unit) & 0x3fffffffu) : -1;
}

struct WEst {
    UnitResult ur;  // the lane's half
    float mx;       // the frame's two estimate symbols' max-abs (when computed here)
};

// The settle re-run of a frame's estimate unit (KISS's arithmetic, bit for
// bit: LoRaDemod.cpp:80-136, phy.cpp:81-148): symbols 0 and 1 in halves 0
// and 1 (the other halves idle), normalised with the frame's true max-abs
// `mx`.  Without an exchange buffer (wbuf_acquire's cap) the unit reports
// NaN, which sends the frame to the exact re-run.
template <int SF, int MODE>
__device__ __noinline__ WEst west2(KArgs ka, lds_cf32* lpool, lds_u32* locks, const lds_cf32* ldnl, unsigned f,
                                   float mx) {
    using W = WGeo<SF>;
    using L = W2Lds<SF, MODE>;
    constexpr int N = W::N, LPS = W::LPS, SPW = W::SPW;
    static_assert(SPW >= 2, "both estimate symbols in one unit");
    constexpr bool M0 = (MODE & 3) == LPHY_MODE_DEMODULATE;
    constexpr bool DECH = (MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE;
    const DemodArgs& A = kargs(ka);
    const cf32* const dnl = (const cf32*)ldnl;
    const int lane = threadIdx.x & 63, h = lane / LPS, l = lane % LPS;
    const bool mine = h < 2;
    const unsigned s = (unsigned)(h < 2 ? h : 0);
    cf32 v[64];
    const cf32* src = A.iq + (unsigned long long)f * A.frame_samples + (unsigned long long)s * N + l;
    iq_check(A, f, (long long)s * N + l + LPS * 63);
    if (mine) {
#pragma unroll
        for (int e = 0; e < 64; ++e) v[e] = src[LPS * e];
    } else {
#pragma unroll
        for (int e = 0; e < 64; ++e) v[e] = czero();
    }
    if constexpr (DECH) {
#pragma unroll
        for (int e = 0; e < 64; ++e) v[e] = cmul(v[e], dnl[l + LPS * e]);
    }
    lphy_frame_meta nm{};
    nm.scale = 1.0f;
    if constexpr (!M0) nm = norm_meta_hot(mx, true, A.no_scratch);
    const bool live = nm.status == 0;
#pragma unroll
    for (int e = 0; e < 64; ++e) {
        cf32 x = v[e];
        if constexpr (!M0) x = cscale(x, nm.scale);
        v[e] = live ? x : czero();
    }
    const WTw<SF> T{};  // unused by the exact pass
    wpass1<SF, false>(v, ctw(A.tw));
    const int b = wbuf_acquire<L::NBUF>(locks, (threadIdx.x >> 6) & (L::NBUF - 1), wlock_salt(A, f + 1));
    if (b >= 0) {
        cf32* const buf = (cf32*)(lpool + b * W::BUF);
        wexchange<SF>(v, buf, h, l);
        // pass 2's per-lane twiddles from an LDS copy of the KISS table
        wait_lgkm0();  // the exchange reads are done
        wdma_table<SF>(A.tw, buf, lane);
        wait_vm0();
        wpass2<SF, false>(v, T, buf, l);
        wait_lgkm0();
        wbuf_release(locks, b);
    }
    float sumsq = 0.0f;
#pragma unroll
    for (int e = 0; e < 64; ++e) {
        const cf32 sq = v[e] * v[e];
        sumsq += sq.x + sq.y;
    }
    const unsigned long long nb = __ballot(!(sumsq == sumsq));
    WEst r;
    r.ur = wunit_result<SF>(v, h, l, lane);
    r.ur.nan = (b < 0 || ((nb >> (LPS * h)) & ((1ull << (LPS & 63)) - 1)) != 0) ? 1 : 0;
    if (!live) r.ur = UnitResult{0, 0, 0.0f, 0.0f, 0};
    r.mx = mx;
    return r;
}

// The pair's two results (halves 0 and 1).
__device__ __forceinline__ UnitResult wur_from(const UnitResult& u, int src) {
    UnitResult r;
    r.idx = __shfl(u.idx, src, 64);
    r.valid = __shfl(u.valid, src, 64);
    r.findex = __shfl(u.findex, src, 64);
    r.phase = __shfl(u.phase, src, 64);
    r.nan = __shfl(u.nan, src, 64);
    return r;
}

// Frame end under the speculative normalisation (wclose's rule): the
// samples no symbol window covers are scanned, then the frame's true max-abs
// confirms the two-symbol normalisation, sends the frame to the exact re-run
// (NaN / inf), or settles it here: both estimates again with the exact
// scale, and the symbols kept when the time shift is unchanged and every
// certified symbol's lead covers the larger sample bound and the rate
// difference (settle_frames' rule), else k_post's exact re-run.
template <int SF, int MODE>
__device__ __noinline__ void wclose2(KArgs ka, lds_cf32* lpool, lds_u32* locks, const lds_cf32* ldnl, unsigned f,
                                     float rate, float scale, int t_off, float mx01, float m, float r, bool nan,
                                     bool open) {
    using W = WGeo<SF>;
    constexpr int N = W::N, LPS = W::LPS;
    constexpr bool DECH = (MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE;
    const DemodArgs& A = kargs(ka);
    const cf32* const dnl = (const cf32*)ldnl;
    const int lane = threadIdx.x & 63;
    const unsigned S = (unsigned)A.total_syms;
    const unsigned cnt = DECH ? S * N : (unsigned)A.frame_samples;
    const unsigned end = covered_end(S, N, cnt, t_off);
    bool fbad = false;
    if (end < cnt) m = fmaxf(m, wave_range_maxabs<SF, MODE>(A, f, end, cnt, dnl, fbad));
    const float mt = fmaxf(m, mx01);
    const lphy_frame_meta mg = norm_meta(mx01, true, 0), me = norm_meta(mt, true, 0);
    bound_check(f, (long long)A.frames);
    if (nan || fbad || !(mt <= 3.40282347e38f)) {
        if (lane == 0) A.meta[f].status = kStatusFixup;
        return;
    }
    if (me.scale == mg.scale && me.normalised == mg.normalised) return;
    // settle: the estimate unit with the frame's true max-abs (norm_meta_hot
    // of it gives me.scale)
    const WEst est = west2<SF, MODE>(ka, lpool, locks, ldnl, f, mt);
    const UnitResult ua = wur_from(est.ur, 0), ub = wur_from(est.ur, LPS);
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
}

// ---------------------------------------------------------------------------
// k_wave2s: units spanning frames (SF 9-10: 8 / 4 symbols per unit).
// Whole units per frame (k_wave) give a frame's 66 symbols at SF 9 9 units,
// the last with 2 live halves of 8, and its estimate unit uses 2 halves of
// 8 - 10 units for 8.5 units of work.  Here a wave's
// frames w, w + W, ... form one stream of symbols (frame k's symbol s at
// position k S + s) cut into units of SPW consecutive symbols, whatever
// frames they belong to, and one estimate unit takes the two estimate
// symbols of EPU = SPW / 2 frames.  An estimate unit runs as soon as a
// symbol unit needs a frame not yet estimated.  Per-frame state lives in a
// per-wave LDS ring of RING records (the rotation, normalisation and time
// shift of the estimate, and the speculation's running max-abs, least
// certificate ratio and flags, which each unit's halves fold in with LDS
// atomics); the unit holding a frame's last symbol closes it (wclose2).
// Each lane rotates with its own frame's tables.
// Precondition (host, launch_wave_mode): frames of at least SPW symbols
// (S >= SPW).  Then a unit of SPW consecutive stream positions holds at most
// one frame end (ends are S apart), so it closes at most one frame, a lane's
// position advances past at most one frame end per unit, and a unit spans at
// most two frames, which the ring holds with the EPU frames of the estimate
// unit ahead.  Shorter frames take k_wave.
// ---------------------------------------------------------------------------
struct WRec {  // 32 B
    float rate, scale, mx;  // estimate: rotation rate, normalisation, estimate symbols' max-abs
    int t_off;
    unsigned ok;    // estimate folded, status 0
    unsigned mxs;   // symbol units' max-abs (float bits, LDS atomic max)
    unsigned rmin;  // least certificate ratio (float bits, LDS atomic min)
    unsigned fl;    // 1 a NaN, 2 a symbol left to the exact re-run (LDS atomic or)
};
typedef __attribute__((address_space(3))) WRec lds_rec;

template <int SF>
struct W2Span {
    static constexpr int SPW = WGeo<SF>::SPW;
    static constexpr int EPU = SPW / 2;  // frames per estimate unit
    static constexpr int RING = EPU + 2 <= 4 ? 4 : (EPU + 2 <= 8 ? 8 : (EPU + 2 <= 16 ? 16 : 32));
};

// Estimate unit of frames fb .. fb + EPU - 1 (wave-local k0 ..): half h
// holds symbol h % 2 of frame fb + h / 2 (fglob: the batch frame of a
// wave-local one).  Each frame's max-abs is folded over its two halves
// (modes 1/2), the frame normalised with it, the halves transformed with
// KISS's arithmetic; returns the half's detector outputs and its frame's
// max-abs.  Dead halves (frames past the wave's last) load nothing.
template <int SF, int MODE>
__device__ __noinline__ WEst west2s(KArgs ka, lds_cf32* lpool, lds_u32* locks, const lds_cf32* ldnl, unsigned fg,
                                    bool live_frame) {
    using W = WGeo<SF>;
    using L = W2Lds<SF, MODE>;
    constexpr int N = W::N, LPS = W::LPS;
    constexpr bool M0 = (MODE & 3) == LPHY_MODE_DEMODULATE;
    constexpr bool DECH = (MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE;
    const DemodArgs& A = kargs(ka);
    const cf32* const dnl = (const cf32*)ldnl;
    const int lane = threadIdx.x & 63, h = lane / LPS, l = lane % LPS;
    const unsigned s = (unsigned)(h & 1);
    cf32 v[64];
    if (live_frame) {
        iq_check(A, fg, (long long)s * N + l + LPS * 63);
        const cf32* src = A.iq + (unsigned long long)fg * A.frame_samples + (unsigned long long)s * N + l;
#pragma unroll
        for (int e = 0; e < 64; ++e) v[e] = src[LPS * e];
    } else {
#pragma unroll
        for (int e = 0; e < 64; ++e) v[e] = czero();
    }
    if constexpr (DECH) {
#pragma unroll
        for (int e = 0; e < 64; ++e) v[e] = cmul(v[e], dnl[l + LPS * e]);
    }
    float mx = 0.0f;
    if constexpr (!M0) {
        float fm = 0.0f;
        cf32 sum = czero();
#pragma unroll
        for (int e = 0; e < 64; ++e) {
            fm = max3_abs(fm, v[e].x, v[e].y);
            sum = sum + v[e];
        }
        const bool bad = !(sum.x == sum.x && sum.y == sum.y) || !(fm <= 3.40282347e38f);
        // over the frame's two halves (2 LPS lanes)
#pragma unroll
        for (int off = LPS; off >= 1; off >>= 1) fm = fmaxf(fm, __shfl_xor(fm, off, 64));
        const unsigned long long bm = __ballot(bad);
        const unsigned pair = (unsigned)(lane / (2 * LPS));
        constexpr unsigned long long PM = 2 * LPS >= 64 ? ~0ull : ((1ull << (2 * LPS)) - 1ull);
        mx = ((bm >> (pair * 2 * LPS)) & PM) != 0 ? __builtin_nanf("") : fm;
    }
    lphy_frame_meta nm{};
    nm.scale = 1.0f;
    if constexpr (!M0) nm = norm_meta_hot(mx, true, A.no_scratch);
    const bool live = live_frame && nm.status == 0;
#pragma unroll
    for (int e = 0; e < 64; ++e) {
        cf32 x = v[e];
        if constexpr (!M0) x = cscale(x, nm.scale);
        v[e] = live ? x : czero();
    }
    const WTw<SF> T{};  // unused by the exact pass
    wpass1<SF, false>(v, ctw(A.tw));
    // (no exchange buffer at wbuf_acquire's cap: the unit reports NaN, which
    // sends its frames to the exact re-run)
    const int b = wbuf_acquire<L::NBUF>(locks, (threadIdx.x >> 6) & (L::NBUF - 1), wlock_salt(A, fg + 2));
    if (b >= 0) {
        cf32* const buf = (cf32*)(lpool + b * W::BUF);
        wexchange<SF>(v, buf, h, l);
        wait_lgkm0();
        wdma_table<SF>(A.tw, buf, lane);
        wait_vm0();
        wpass2<SF, false>(v, T, buf, l);
        wait_lgkm0();
        wbuf_release(locks, b);
    }
    float sumsq = 0.0f;
#pragma unroll
    for (int e = 0; e < 64; ++e) {
        const cf32 sq = v[e] * v[e];
        sumsq += sq.x + sq.y;
    }
    const unsigned long long nb = __ballot(!(sumsq == sumsq));
    WEst r;
    r.ur = wunit_result<SF>(v, h, l, lane);
    r.ur.nan = (b < 0 || ((nb >> (LPS * h)) & ((1ull << (LPS & 63)) - 1)) != 0) ? 1 : 0;
    if (!live) r.ur = UnitResult{0, 0, 0.0f, 0.0f, 0};
    r.mx = mx;
    return r;
}

// The frame's rotation tables for lanes whose frames differ (k_wave2s):
// q[b] = [scale] e^{j rate (l + LPS b)} and p = e^{j rate 8 LPS (l & 7)} of
// the lane's own frame (LPS >= 8: every half's lanes 0..7 give its table).
template <int SF, int MODE>
__device__ __noinline__ WRot wrot_lane(float rate, float scale) {
    constexpr int LPS = WGeo<SF>::LPS;
    static_assert(LPS >= 8, "p from the half's own lanes");
    const int lane = threadIdx.x & 63, l = lane % LPS;
    WRot r;
#pragma unroll 1
    for (int b = 0; b < 8; ++b) {
        float sn, cs;
        lphy_libm::sincosf_exact(rate * (float)(l + LPS * b), &sn, &cs);
        cf32 t = cf32{cs, sn};
        if constexpr ((MODE & 3) != LPHY_MODE_DEMODULATE) t = cscale(t, scale);
        r.q[b] = t;
    }
    float sn, cs;
    lphy_libm::sincosf_exact(rate * (float)(8 * LPS * (l & 7)), &sn, &cs);
    r.p = cf32{cs, sn};
    return r;
}

template <int SF, int MODE>
__global__ __launch_bounds__(512) void k_wave2s(FrameArgs P) {
    using W = WGeo<SF>;
    using L = W2Lds<SF, MODE>;
    using SP = W2Span<SF>;
    constexpr int N = W::N, LPS = W::LPS, SPW = W::SPW, EPU = SP::EPU, RING = SP::RING;
    constexpr bool M0 = (MODE & 3) == LPHY_MODE_DEMODULATE;
    constexpr bool DECH = (MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE;
    static_assert(SPW >= 4 && LPS >= 8, "spanning units: SF 9-10");
    const DemodArgs& A = P.A;
    const KArgs ka = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ cf32 lds_all[L::DNC + L::NBUF * W::BUF];
    __shared__ unsigned locks_s[L::NBUF];
    __shared__ WRec rings[L::WPB][RING];
    cf32* const dnl = lds_all;
    lds_cf32* const pool = (lds_cf32*)(lds_all + L::DNC);
    lds_u32* const locks = (lds_u32*)locks_s;

    const int tid = threadIdx.x;
    if constexpr (L::DN) {
        for (int i = tid; i < N; i += 512) dnl[i] = A.down[i];
    }
    if (tid < L::NBUF) locks_s[tid] = 0u;
    __syncthreads();  // the only workgroup barrier: waves are independent below

    const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane / LPS, l = lane % LPS;
    const unsigned nframes = (unsigned)A.frames;
    const unsigned S = (unsigned)A.total_syms;
    const unsigned Wn = P.waves;
    const unsigned w = blockIdx.x * L::WPB + wv;
    if (w >= nframes) return;
    const unsigned nk = (nframes - 1 - w) / Wn + 1;
    const unsigned long long total = (unsigned long long)nk * S;
    const unsigned NU = (unsigned)((total + SPW - 1) / SPW);
    const bool spec = !M0 && A.spec != 0;
    const int bstart = wv & (L::NBUF - 1);
    WRec* const ring = rings[wv];
    constexpr float kBig = 3.0e38f;

    cf32 Qr[8], Pr[8];
    unsigned rot_k = 0xffffffffu;  // the lane's frame its tables are for
    const cf32 rroot = root64(lane);  // Parseval certificate's register table
    bool pv_on = true;
    // the lane's stream position for the next symbol unit: frame kh, symbol sh
    unsigned kh = 0, sh = (unsigned)h;
    unsigned est = 0;  // frames whose estimate is folded
    for (unsigned u = 0; u < NU;) {
        const unsigned kmax_raw = (unsigned)__builtin_amdgcn_readlane((int)kh, 63);
        const unsigned kmax = kmax_raw < nk ? kmax_raw : nk - 1;
        if (est <= kmax) {
            // estimate unit: frames est .. est + EPU - 1, half h symbol h % 2
            const unsigned ke = est + (unsigned)(h >> 1);
            const bool lf = ke < nk;
            const unsigned fe = w + (lf ? ke : 0u) * Wn;
            const WEst e = west2s<SF, MODE>(ka, pool, locks, (const lds_cf32*)dnl, fe, lf);
            // the frame's fold on the first lane of its even half
            const UnitResult ub = wur_from(e.ur, (lane + LPS) & 63);
            if ((h & 1) == 0 && l == 0 && lf) {
                lphy_frame_meta m{};
                m.scale = 1.0f;
                m.have_sync = 1;
                if constexpr (!M0) m = norm_meta_hot(e.mx, true, A.no_scratch);
                if (m.status == 0) {
                    EstFold fold;
                    if (e.ur.valid) fold.add(e.ur.idx, e.ur.findex, 0, e.ur.phase);
                    else fold.add(0, 0.0f, 0, 0.0f);
                    if (ub.valid) fold.add(ub.idx, ub.findex, 0, ub.phase);
                    else fold.add(0, 0.0f, 0, 0.0f);
                    fold.finish(m, 2, N, 1);
                    if (e.ur.nan || ub.nan) m.status = kStatusFixup;
                }
                bound_check(fe, (long long)A.frames);
                meta_put_est(&A.meta[fe], m);
                WRec r;
                r.rate = m.rate;
                r.scale = m.scale;
                r.mx = e.mx;
                r.t_off = m.t_off;
                r.ok = m.status == 0 ? 1u : 0u;
                r.mxs = 0u;
                r.rmin = __float_as_uint(kBig);
                r.fl = 0u;
                ring[ke % RING] = r;
            }
            est += EPU;
            continue;
        }
        // symbol unit u: half h is symbol sh of frame kh
        const bool live = kh < nk;
        const unsigned f = w + (live ? kh : 0u) * Wn;
        const WRec R = ring[(live ? kh : kmax) % RING];
        lphy_frame_meta m{};
        m.rate = R.rate;
        m.scale = R.scale;
        m.t_off = R.t_off;
        m.status = R.ok ? 0 : -1;
        m.have_sync = 1;
        const SymCtx c = sym_ctx(A, f, live ? sh : 0u, live, N, m);
        cf32 v[64];
        {
            const cf32* src = A.iq + (unsigned long long)f * A.frame_samples + c.base + (unsigned)l;
            if (live) {
                iq_check(A, f, (long long)c.base + l + LPS * 63);
#pragma unroll
                for (int e = 0; e < 64; ++e) v[e] = src[LPS * e];
            } else {
#pragma unroll
                for (int e = 0; e < 64; ++e) v[e] = czero();
            }
        }
        if (__ballot(live && kh != rot_k)) {
            pv_on = true;  // a new frame: try the Parseval certificate again
            const WRot rt = wrot_lane<SF, MODE>(R.rate, R.scale);
#pragma unroll
            for (int b = 0; b < 8; ++b) Qr[b] = rt.q[b];
#pragma unroll
            for (int a = 0; a < 8; ++a)
                Pr[a] = cf32{__shfl(rt.p.x, h * LPS + a, 64), __shfl(rt.p.y, h * LPS + a, 64)};
            rot_k = kh;
        }
        float amax = 0.0f;
        const unsigned d0 = ((c.base + (unsigned)l) & (unsigned)(N - 1)) << 3;
        cf32 dq[2][8];
        auto ld_chunk = [&](int q, cf32 (&ds)[8]) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int e = 8 * q + i;
                if constexpr (DECH) ds[i] = lds_ld(dnl, (int)((d0 + (unsigned)((LPS * e) << 3)) & (unsigned)(8 * N - 1)));
                if constexpr (M0) ds[i] = dnl[l + LPS * e];
            }
        };
        ld_chunk(0, dq[0]);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (q + 1 < 8) ld_chunk(q + 1, dq[(q + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int e = 8 * q + i;
                cf32 p = v[e];
                if constexpr (DECH) p = cmul(p, dq[q & 1][i]);
                amax = max3_abs(amax, p.x, p.y);
                if constexpr (M0) p = cmul(p, dq[q & 1][i]);
                v[e] = p;  // the rotation: below, or folded into the Parseval sums
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        float am = 1.0f;
        if constexpr (M0) {
#pragma unroll
            for (int off = 1; off < LPS; off <<= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 64));
            am = amax;
        }
        const float cb1 = cert_bound<SF>(c.rate, c.start, 1.0f, kWaveExtra);
        int sym = 0;         // the symbol's bin (certified) ...
        float cgap = -1.0f;  // ... and its certified lead (-1: not certified)
        bool pv = false;     // the whole unit certified by Parseval (lphy_wave.h)
        if (pv_on && !A.debug_recheck) {
            const int kc = pv_candidate<SF>(v, l, c.rate);
            const cf32 wkl = A.tw[(unsigned)(kc * l) & (unsigned)(N - 1)];
            cf32 ykl;
            float el;
            pv_lane_sums<SF>(v, kc, rroot, Qr, Pr, ykl, el);
            const float lead = pv_lead<SF>(cmul_fma(ykl, wkl), el, M0 ? 1.0f : c.scale * c.scale, am);
            const bool ok = lead > 4.0f * (cb1 * am) && (float)N * 1.41421366f * am * 1.0001f < 1e18f &&
                            am >= 1e-20f;
            pv = __ballot(live && c.ok && !ok) == 0;
            if (pv) {
                pv_count(A, live && c.ok && l == 0);
                sym = kc;
                cgap = lead;
            } else {
                pv_on = false;  // until a unit enters a new frame: the transform
            }
        }
        if (!pv) {
#pragma unroll
            for (int e = 0; e < 64; ++e) v[e] = cmul_fma(cmul_fma(v[e], Qr[e & 7]), Pr[e >> 3]);
            wpass1<SF, true>(v, ctw(A.tw));
            int hx = h, lx = l;
            asm volatile("" : "+v"(hx), "+v"(lx));
            WTw<SF> T;
            T.load(A.tw, lx);
            // (no exchange buffer at wbuf_acquire's cap: the unit's symbols go to
            // the exact re-run, `lost`)
            const int b = wbuf_acquire<L::NBUF>(locks, bstart, wlock_salt(A, u));
            const bool lost = b < 0;
            if (!lost) {
                wexchange<SF>(v, (cf32*)(pool + b * W::BUF), hx, lx);
                wait_lgkm0();
                wbuf_release(locks, b);
            } else {
#pragma unroll
                for (int e = 0; e < 64; ++e) v[e] = czero();
            }
            wpass2<SF, true>(v, T, A.tw, l);
            unsigned k1 = 0u, k2 = 0u;
#pragma unroll
            for (int e = 0; e < 64; e += 2) {
                const float ma = __builtin_fmaf(v[e].x, v[e].x, v[e].y * v[e].y);
                const float mb = __builtin_fmaf(v[e + 1].x, v[e + 1].x, v[e + 1].y * v[e + 1].y);
                top2_pair(k1, k2, (__float_as_uint(ma) & ~63u) | (unsigned)e,
                          (__float_as_uint(mb) & ~63u) | (unsigned)(e + 1));
            }
            unsigned K1, K2;
            wave_top2_merge<LPS>(k1, k2, h, K1, K2);
            const unsigned long long bm = __ballot(k1 == K1);
            const unsigned long long hm = (bm >> (LPS * h)) & ((1ull << (LPS & 63)) - 1);
            ArgMax2 b2;
            b2.v = __uint_as_float(K1 & ~63u);
            b2.v2 = __uint_as_float(K2 | 63u);
            b2.i = (__ffsll((long long)hm) - 1) + LPS * (int)(K1 & 63u);
            const float g = cert_gap(b2);
            const bool cert = g > 4.0f * (cb1 * am) && (float)N * 1.41421366f * am * 1.0001f < 1e18f &&
                              am >= 1e-20f && b2.v >= 1e-30f;
            sym = b2.i;
            cgap = cert && !A.debug_recheck && !lost ? g : -1.0f;
        }
        const bool redo = c.ok && !(cgap >= 0.0f);
        if (live && l == 0) {
            const uint16_t out = redo ? kSymRecheck : (uint16_t)sym;
            if (c.have_sync && c.s < 2) store_symbol(A, c, c.ok ? out : (uint16_t)0);
            else if (c.ok) store_symbol(A, c, out);
            if (redo) A.meta[c.f].status = kStatusRecheck;
        }
        if (spec) {
            // the half's share of its frame's speculation state: max-abs of its
            // samples (NaN dropped as fmaxf does: the NaN flag carries it), the
            // certificate ratio, the flags; folded into the frame's record
            float mm = c.ok ? amax : 0.0f;
            const cf32 q0 = v[0] * v[0];
            const float q2 = q0.x + q0.y;
            unsigned fl = (c.ok && !(q2 == q2)) ? 1u : 0u;
            float rr = kBig;
            if (c.ok && l == 0) {
                if (redo) fl |= 2u;
                else rr = cgap * __builtin_amdgcn_rcpf(cb1) * (1.0f - 4.0f * kU);
            }
#pragma unroll
            for (int off = LPS / 2; off >= 1; off >>= 1) {
                mm = fmaxf(mm, __shfl_xor(mm, off, 64));
                rr = fminf(rr, __shfl_xor(rr, off, 64));
                fl |= (unsigned)__shfl_xor((int)fl, off, 64);
            }
            if (live && l == 0 && R.ok) {
                WRec* rp = &ring[kh % RING];
                atomicMax(&rp->mxs, __float_as_uint(mm));
                atomicMin(&rp->rmin, __float_as_uint(rr));
                if (fl) atomicOr(&rp->fl, fl);
            }
            // the half holding a frame's last symbol closes that frame
            const unsigned long long cm = __ballot(live && sh == S - 1 && l == 0);
            if (cm) {
                const int src = __ffsll((long long)cm) - 1;
                const unsigned kc = (unsigned)__builtin_amdgcn_readlane((int)kh, src);
                wait_lgkm0();  // this wave's atomics above are done
                const WRec Rc = ring[kc % RING];
                if (Rc.ok)
                    wclose2<SF, MODE>(ka, pool, locks, (const lds_cf32*)dnl, w + kc * Wn, Rc.rate, Rc.scale,
                                      Rc.t_off, Rc.mx, __uint_as_float(Rc.mxs), __uint_as_float(Rc.rmin),
                                      (Rc.fl & 1u) != 0, (Rc.fl & 2u) != 0);
            }
        }
        sh += SPW;
        if (sh >= S) {
            sh -= S;
            ++kh;
        }
        ++u;
    }
}
