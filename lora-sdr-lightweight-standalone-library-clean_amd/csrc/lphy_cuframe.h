// lphy_cuframe.h — single-read fused demodulation of short frames (SF 7,
// 56..70 symbols per frame): included inside the anonymous namespace of
// lphy_kernels.h.
//
// Why: lora_demodulate normalises by the whole frame's max(|I|,|Q|)
// (LoRaDemod.cpp:60-78) before its two-symbol estimate (:80-140), and every
// symbol's rotation depends on that estimate (:142-176).  k_frames reads a
// frame twice (max-abs scan, then the symbols); on MI355X the second read
// costs full HBM bandwidth (profiles/r2/reread_microbench.txt: 1.41 ms for
// two passes over 4.4 GB against 0.71 ms for one).  Here each frame crosses
// HBM once and stays on the CU until its symbols are done:
//
//   HBM --(2 register slots, 9 x 16 B per thread)--> scan + estimate staging
//       --> LDS frame buffer (2 per CU) --> symbol transforms (in place)
//
// One 512-thread workgroup per CU (8 waves).  Frames of the workgroup are
// f = blockIdx.x + k * gridDim.x, k = 0, 1, ...  Waves 0..6 are workers: they
// hold the register slots (10 x 16 B per thread) and per round their 56
// teams (8 lanes each) take the next 56 symbol units of the stream D(0),
// D(1), ... (frame k's S symbols, in order).  Wave 7 runs the estimates: per
// frame the two estimate units (the same KISS transforms as k_frames' E
// units), the fold into the frame's offsets and the certified fast rotation
// table (the header comment of k_frames).  The two roles run separate loops
// with the same barrier sequence, so the estimate code (libm restatements,
// full transform) never shares registers with the in-flight slots.
//
// Events, all at round boundaries and executed by every thread:
//   event k (round E_k = max(k, round(last unit of D(k-2)) + 1)):
//     scan frame k+1 from its register slot (wait for the loads, max-abs,
//     workgroup reduction, estimate staging of symbols 0 and 1); write frame
//     k from its slot into buffer k % 2 (free: D(k-2) is done); issue the
//     loads of frame k+2 into that slot.
//   Frame k+1's estimate runs in round E_k, D(k+1) starts >= 2 rounds later
//   (133 units of stream lie between); its loads were issued at event k-1,
//   about one frame (66 / 56 rounds) earlier.
//
// A symbol unit transforms in place: the first pass reads its window of the
// frame buffer (natural order, shifted by t_off, times the frame's table),
// a workgroup barrier, then writes its intermediate values into buffer slot
// s (slot s + 2 holds symbol s; slots 0, 1 are spare), which no later unit
// reads.
// ---------------------------------------------------------------------------
template <int SF>
struct CuCfg {
    using G = Geo<SF>;
    static constexpr int N = G::N;
    static constexpr int WAVES = 8, WORKERS = 7, THREADS = 64 * WAVES;
    static constexpr int WTHREADS = 64 * WORKERS;   // threads holding register slots
    static constexpr int TPW = 64 / G::LPS;        // teams per wave
    static constexpr int TEAMS = WORKERS * TPW;    // symbol units per round
    static constexpr int SMAX = 70;                // symbols per frame (LDS)
    static constexpr int SMIN = TEAMS;             // a round spans <= 2 frames
    static constexpr int FSLOTS = SMAX + 2;        // slots per frame buffer
    static constexpr int PF = 10;                  // 16-B loads per worker thread per frame
    static_assert(PF * WTHREADS * 2 >= SMAX * N, "register slot holds a frame");
    static_assert(WTHREADS >= N, "symbols 0 and 1 sit in the first pass of the slot");
    static constexpr int ESLOTS = 4;               // estimate staging slots
};

template <int SF>
struct CuShared {
    using C = CuCfg<SF>;
    cf32 fb[2][C::FSLOTS * C::N];  // frame buffers, Geo layout per slot
    cf32 ea[C::ESLOTS * C::N];     // estimate staging, Geo layout
    cf32 twl[C::N];
    cf32 dnl[C::N];
    float wnl[C::N];
    cf32 rtab[3][C::N];            // fast rotation tables of frames k % 3
    float4 rec[3];                 // rate, scale, t_off, flags (bit0 ok, bit1 have_sync)
    UnitResult ures[C::ESLOTS];
    float red[C::WAVES];
    unsigned redbad[C::WAVES];
    float ejmx[2];                 // max-abs of the frames staged for estimate
    unsigned ejk[2];               // their workgroup-local frame indices
    unsigned nej;                  // estimate jobs this round
};

template <int SF, int MODE>
__global__ __launch_bounds__(512, 1) void k_cuframe(DemodArgs A) {
    using C = CuCfg<SF>;
    using G = Geo<SF>;
    constexpr int N = C::N;
    constexpr Passes<SF> PS{};
    static_assert(PS.n == 2, "two-pass transform");
    constexpr int HI0 = PS.hi[0], LO0 = PS.lo[0];
    using Gr0 = Group<SF, HI0, LO0>;
    constexpr bool DECH = (MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE;
    constexpr bool NORM = (MODE & 3) != LPHY_MODE_DEMODULATE;
    __shared__ CuShared<SF> sh;

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int team = lane / G::LPS, lam = lane % G::LPS;
    const unsigned nframes = (unsigned)A.frames;
    const unsigned GS = gridDim.x;
    const unsigned nk = blockIdx.x < nframes ? (nframes - 1 - blockIdx.x) / GS + 1 : 0;
    const unsigned S = (unsigned)A.total_syms;
    const unsigned n4 = S * (unsigned)N / 2;  // 16-B pairs per frame
    const bool exact_only = A.exact_rotation != 0;

    for (int i = tid; i < N; i += C::THREADS) {
        sh.twl[i] = A.tw[i];
        sh.dnl[i] = A.down[i];
        if (A.win) sh.wnl[i] = A.win[i];
    }
    if (tid == 0) sh.nej = 0;
    if (lane == 0) {
        sh.red[wv] = 0.0f;
        sh.redbad[wv] = 0;
    }
    __syncthreads();
    const float* win = A.win ? sh.wnl : nullptr;

    auto last_round = [&](unsigned k) -> unsigned {  // round of the last unit of D(k)
        return 1u + (unsigned)(((unsigned long long)S * (k + 1ull) - 1ull) / (unsigned)C::TEAMS);
    };
    const unsigned rounds = nk ? last_round(nk - 1) + 1u : 0u;
    auto event_round = [&](unsigned k) -> unsigned { return k < 2 ? k : last_round(k - 2) + 1u; };

    // The event / round skeleton, identical for both roles (same barriers):
    // scanf(slot, k) scans frame k from register slot `slot`; evf(slot, k)
    // writes frame k from that slot to its buffer and refills the slot with
    // frame k + 2; roundf(r) runs round r.  Slot roles are fixed in the code
    // (even events read slot 1 and refill slot 0, odd events the reverse), so
    // a slot whose loads are in flight is never copied.
#ifdef LPHY_PROFILE_PHASES  // timing experiments only: [1] events, [2] round, [3] barriers
    unsigned long long ph_ev = 0, ph_round = 0, ph_bar = 0, ph_t = 0;
#define CU_T0() ph_t = clock64()
#define CU_ACC(x) x += clock64() - ph_t
#else
#define CU_T0()
#define CU_ACC(x)
#endif
    auto skeleton = [&](auto&& scanf, auto&& evf, auto&& roundf) __attribute__((always_inline)) {
        unsigned r = 0;
        auto rounds_to = [&](unsigned rend) __attribute__((always_inline)) {
            for (; r < rend; ++r) {
                CU_T0();
                __syncthreads();  // event stores visible; previous round done
                CU_ACC(ph_bar);
                CU_T0();
                roundf(r);
                CU_ACC(ph_round);
                CU_T0();
                __syncthreads();
                CU_ACC(ph_bar);
            }
        };
        if (nk) scanf(std::integral_constant<int, 0>{}, 0u);
        for (unsigned k = 0; k < nk; k += 2) {
            rounds_to(event_round(k));
            CU_T0();
            if (k + 1 < nk) scanf(std::integral_constant<int, 1>{}, k + 1);
            evf(std::integral_constant<int, 0>{}, k);
            CU_ACC(ph_ev);
            if (k + 1 >= nk) break;
            rounds_to(event_round(k + 1));
            CU_T0();
            if (k + 2 < nk) scanf(std::integral_constant<int, 0>{}, k + 2);
            evf(std::integral_constant<int, 1>{}, k + 1);
            CU_ACC(ph_ev);
        }
        rounds_to(rounds);
#ifdef LPHY_PROFILE_PHASES
        if (lane == 0 && (wv == 0 || wv == C::WORKERS)) {
            const int o = wv == 0 ? 0 : 3;  // worker wave 0: [1..3] (+ [4] events of estimate wave)
            if (o == 0) {
                atomicAdd(&A.counters[1], ph_ev);
                atomicAdd(&A.counters[2], ph_round);
                atomicAdd(&A.counters[3], ph_bar);
            } else {
                atomicAdd(&A.counters[4], ph_round);
            }
        }
#endif
    };
    // workgroup max-abs reduction of a scan (modes 1, 2); every thread calls
    // it, the estimate wave with mx = 0
    auto reduce_max = [&](float mx, bool bad) -> float {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const float o = __shfl_xor(mx, off, 64);
            mx = o > mx ? o : mx;
        }
        const bool wbad = __ballot(bad) != 0;
        if (lane == 0) {
            sh.red[wv] = mx;
            sh.redbad[wv] = wbad;
        }
        __syncthreads();
        mx = sh.red[0];
        bool nf = sh.redbad[0] != 0;
#pragma unroll
        for (int w = 1; w < C::WAVES; ++w) {
            nf |= sh.redbad[w] != 0;
            mx = sh.red[w] > mx ? sh.red[w] : mx;
        }
        __syncthreads();  // red[] read by all before the next scan rewrites it
        return nf ? __builtin_nanf("") : mx;  // norm_meta_hot -> exact re-run
    };

    if (wv == C::WORKERS) {
        // ================================================= estimate wave
        auto scan_e = [&](auto, unsigned) __attribute__((always_inline)) {
            if constexpr (NORM) (void)reduce_max(0.0f, false);
        };
        auto ev_e = [&](auto, unsigned) __attribute__((always_inline)) {};
        auto round_e = [&](unsigned) __attribute__((always_inline)) {
            const unsigned nej = sh.nej;
            const unsigned es = (unsigned)team;  // estimate slot of this team
            const unsigned job = es >> 1;
            const bool act = job < nej;
            const unsigned kj = act ? sh.ejk[job] : 0u;
            const bool jok = act && [&] {
                if constexpr (NORM) return norm_meta_hot(sh.ejmx[job], true, A.no_scratch).status == 0;
                else return true;
            }();
            const unsigned slot = 2u * (kj & 1u) + (es & 1u);
#ifdef LPHY_ABLATE_CU_EFFT  // timing experiments only
            if (false) {
#else
            if (act) {  // whole teams: the transform's exchanges stay in the team's slot
#endif
                cf32 v[16];
                fft_tile<SF>(v, sh.ea, (int)slot, lam, sh.twl);
                const ArgMax2 b2 = symbol_argmax2<SF>(local_argmax2<SF>(v, lam));
                const ArgMax best{b2.v, b2.i};
#pragma unroll
                for (int e = 0; e < G::E; ++e) sh.ea[G::addr((int)slot, bin_of<SF>(e, lam))] = v[e];
                team_sync<SF>();
                // a NaN bin may hide an Annex G product: exact re-run (k_post)
                const unsigned long long nanm = __ballot(jok && fft_has_nan<SF>(v));
                if (lam == 0) {
#ifdef LPHY_ABLATE_CU_UR  // timing experiments only
                    UnitResult ur = UnitResult{best.i, 1, 0.0f, 0.0f, 0};
#else
                    UnitResult ur = jok ? unit_result<SF>(sh.ea, (int)slot, best) : UnitResult{0, 0, 0.0f, 0.0f, 0};
#endif
                    ur.nan = ((nanm >> (team * G::LPS)) & ((1ull << G::LPS) - 1)) != 0;
                    sh.ures[slot] = ur;
                }
                team_sync<SF>();
            }
            __syncthreads();  // (the workers' in-place barrier)
            // fold (lane j for job j), then the job's rotation table
            if (lane < (int)nej) {
                const unsigned k = sh.ejk[lane];
                lphy_frame_meta m{};
                m.scale = 1.0f;
                m.have_sync = 1;
                if constexpr (NORM) m = norm_meta_hot(sh.ejmx[lane], true, A.no_scratch);
                if (m.status == 0) {
                    EstFold fold;
                    bool nan = false;
                    const unsigned p0 = 2u * (k & 1u);
#pragma unroll
                    for (unsigned u = 0; u < 2; ++u) {
                        const UnitResult ur = sh.ures[p0 + u];
                        nan |= ur.nan != 0;
                        if (ur.valid) fold.add(ur.idx, ur.findex, 0, ur.phase);
                        else fold.add(0, 0.0f, 0, 0.0f);
                    }
                    fold.finish(m, 2, N, 1);
                    if (nan) m.status = kStatusFixup;
                }
                sh.rec[k % 3] = float4{m.rate, m.scale, __int_as_float(m.t_off),
                                       __uint_as_float((m.status == 0 ? 1u : 0u) | 2u)};
                meta_put_est(&A.meta[blockIdx.x + k * GS], m);
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            for (unsigned j = 0; j < nej; ++j) {
                const unsigned k = sh.ejk[j];
                const float4 rc = sh.rec[k % 3];
#ifndef LPHY_ABLATE_CU_RTAB  // timing experiments only
                if (__float_as_uint(rc.w) & 1u)
                    build_rtab<SF, MODE>(sh.rtab[k % 3], rc.x, rc.y, __float_as_int(rc.z), sh.dnl, win, lane);
#endif
            }
            if (lane == 0) sh.nej = 0;
        };
        skeleton(scan_e, ev_e, round_e);
        return;
    }

    // ===================================================== worker waves
    float4 P0[C::PF], P1[C::PF];
    auto fetch = [&](float4 (&P)[C::PF], unsigned k) __attribute__((always_inline)) {
        if (k >= nk) return;
        const float4* fr = reinterpret_cast<const float4*>(A.iq + (unsigned long long)(blockIdx.x + k * GS) * A.frame_samples);
#pragma unroll
        for (int j = 0; j < C::PF; ++j) {
            // unconditional (clamped) loads: a per-element condition would
            // make hipcc wait for each load in turn
            const unsigned q = (unsigned)tid + (unsigned)(j * C::WTHREADS);
            P[j] = fr[q < n4 ? q : n4 - 1];
        }
    };
    // scan of frame k (modes 1, 2: max-abs of the [dechirped] frame, with the
    // NaN / overflow sentinel of wave_maxabs) and its estimate staging
    auto scan = [&](float4 (&P)[C::PF], unsigned k) __attribute__((always_inline)) {
        float mx = 0.0f;
        if constexpr (NORM) {
            float fm = 0.0f;
            cf32 sum = czero();
#pragma unroll
            for (int j = 0; j < C::PF; ++j) {
                const unsigned q = (unsigned)tid + (unsigned)(j * C::WTHREADS);
                cf32 a = cf32{P[j].x, P[j].y}, b = cf32{P[j].z, P[j].w};
                if (q >= n4) a = b = czero();
                if constexpr (DECH) {
                    a = cmul(a, sh.dnl[(2u * q) & (N - 1)]);
                    b = cmul(b, sh.dnl[(2u * q + 1u) & (N - 1)]);
                }
                fm = max3_abs(fm, a.x, a.y);
                fm = max3_abs(fm, b.x, b.y);
                sum = sum + a;
                sum = sum + b;
            }
            const bool bad = !(sum.x == sum.x && sum.y == sum.y) || !(fm <= 3.40282347e38f);
            mx = reduce_max(fm, bad);
        }
        lphy_frame_meta m{};
        m.scale = 1.0f;
        if constexpr (NORM) m = norm_meta_hot(mx, true, A.no_scratch);
        const bool ok = m.status == 0;
        const unsigned slot0 = 2u * (k & 1u);  // estimate pair of this frame
        // symbols 0 and 1 are the frame's first N pairs: threads 0..N-1, j = 0
        if (tid < N) {
            const unsigned i0 = (2u * (unsigned)tid) & (N - 1);
            const unsigned u = (2u * (unsigned)tid) >> SF;
            const cf32 x[2] = {cf32{P[0].x, P[0].y}, cf32{P[0].z, P[0].w}};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const unsigned i = i0 + (unsigned)h;
                cf32 p = x[h];
                if constexpr (NORM) {
                    if constexpr (DECH) p = cmul(p, sh.dnl[i]);
                    p = cscale(p, m.scale);
                }
                cf32 y = ok ? p : czero();
                if constexpr ((MODE & kWinBit) != 0) y = cscale(y, win[i]);
                sh.ea[G::addr((int)(slot0 + u), (int)i)] = y;
            }
        }
        if (tid == 0) {
            const unsigned j = sh.nej;
            sh.ejmx[j] = mx;
            sh.ejk[j] = k;
            sh.nej = j + 1;
        }
    };
    // frame k from its register slot into buffer k % 2 (symbol s in slot s + 2)
    auto store_frame = [&](float4 (&P)[C::PF], unsigned k) __attribute__((always_inline)) {
        cf32* F = sh.fb[k & 1u];
#pragma unroll
        for (int j = 0; j < C::PF; ++j) {
            const unsigned q = (unsigned)tid + (unsigned)(j * C::WTHREADS);
            if (q < n4) {
                const unsigned smp = 2u * q;
                const int a0 = G::addr((int)(smp >> SF) + 2, (int)(smp & (N - 1)));
                // the swizzle keeps an even/odd pair in one 16-byte cell,
                // possibly swapped
                float4* cell = reinterpret_cast<float4*>(F + (a0 & ~1));
                *cell = (a0 & 1) ? float4{P[j].z, P[j].w, P[j].x, P[j].y} : P[j];
            }
        }
    };
    auto scan_w = [&](auto slot, unsigned k) __attribute__((always_inline)) {
        if constexpr (decltype(slot)::value == 0) scan(P0, k);
        else scan(P1, k);
    };
    auto ev_w = [&](auto slot, unsigned k) __attribute__((always_inline)) {
        if constexpr (decltype(slot)::value == 0) {
            store_frame(P0, k);
            fetch(P0, k + 2);
        } else {
            store_frame(P1, k);
            fetch(P1, k + 2);
        }
    };

    // stream position of this team: unit p = TEAMS*(r-1) + TPW*wv + team
    unsigned dk = 0, ds = (unsigned)(C::TPW * wv + team);
    while (ds >= S) { ds -= S; ++dk; }
    auto round_w = [&](unsigned r) __attribute__((always_inline)) {
        const bool act = r >= 1 && dk < nk;
        const unsigned f = blockIdx.x + dk * GS;
        lphy_frame_meta m{};
        if (act) {
            const float4 rc = sh.rec[dk % 3];
            m.rate = rc.x;
            m.scale = rc.y;
            m.t_off = __float_as_int(rc.z);
            const unsigned fl = __float_as_uint(rc.w);
            m.status = (fl & 1u) ? 0 : -1;
            m.have_sync = (fl & 2u) ? 1 : 0;
        }
        const SymCtx c = sym_ctx(A, act ? f : 0u, act ? ds : 0u, act, N, m);
        cf32* F = sh.fb[dk & 1u];
        const cf32* rt = sh.rtab[dk % 3];
        cf32 v[16];
#pragma unroll
        for (int e = 0; e < G::E; ++e) v[e] = czero();
        float amax = 0.0f;
        if (c.ok) {
            // first pass: window samples (KISS leaf order) times the table
            const unsigned base = c.base;
            if ((base & (N - 1)) == 0) {
                const int lb8 = G::lbase((int)(base >> SF) + 2, Gr0::inidx(0, lam)) << 3;
#pragma unroll
                for (int e = 0; e < G::E; ++e) v[e] = lds_ld(F, G::at8(lb8, G::cpart(Gr0::inidx(e, 0)) << 3));
            } else {
#pragma unroll
                for (int e = 0; e < G::E; ++e) {
                    const unsigned q = base + (unsigned)Gr0::inidx(e, lam);
                    v[e] = F[G::addr((int)(q >> SF) + 2, (int)(q & (N - 1)))];
                }
            }
#pragma unroll
            for (int e = 0; e < G::E; ++e) {
                cf32 x = v[e];
                if constexpr ((MODE & 3) == LPHY_MODE_DEMODULATE)
                    amax = fmaxf(amax, fmaxf(fabsf(x.x), fabsf(x.y)));
                // mode 2: the exact dechirp at the sample's chirp index (the
                // table holds the rotation and scale only, build_rtab)
                if constexpr ((MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE)
                    x = cmul(x, sh.dnl[(base + (unsigned)Gr0::inidx(e, lam)) & (N - 1)]);
                v[e] = cmul(x, rt[Gr0::inidx(e, lam)]);
            }
#ifndef LPHY_ABLATE_CU_DFFT  // timing experiments only
            pass_butterflies<SF, HI0, LO0, true>(v, lam, sh.twl);
#endif
        }
        __syncthreads();  // every unit's window read before any in-place write
        if (c.ok) {
            const int lb8 = G::lbase((int)ds, Gr0::pos(0, lam)) << 3;
#pragma unroll
            for (int e = 0; e < G::E; ++e) lds_st(F, G::at8(lb8, G::cpart(Gr0::pos(e, 0)) << 3), v[e]);
        }
        team_sync<SF>();
#ifndef LPHY_ABLATE_CU_DFFT
        if (c.ok) run_pass<SF, 1, true, true, false>(v, F, (int)ds, lam, sh.twl);
#endif
        const ArgMax2 b2 = symbol_argmax2<SF>(local_argmax2<SF>(v, lam));
        if constexpr ((MODE & 3) == LPHY_MODE_DEMODULATE) {
#pragma unroll
            for (int off = G::LPS / 2; off >= 1; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 64));
        } else {
            amax = 1.0f;  // normalised frame (see fast_certified)
        }
        if (act && lam == 0) {
            const bool redo = c.ok && (exact_only || !fast_applies<SF, MODE>(c, c.toff) ||
                                       !fast_certified<SF>(b2, c, amax));
            const uint16_t out = redo ? kSymRecheck : (uint16_t)b2.i;
            // (no status store: the estimate wave writes this record; the
            // sentinel itself tells k_post to recompute the symbol)
            if (c.have_sync && c.s < 2) store_symbol(A, c, c.ok ? out : (uint16_t)0);
            else if (c.ok) store_symbol(A, c, out);
        }
        if (r >= 1) {
            ds += C::TEAMS;
            while (ds >= S) { ds -= S; ++dk; }
        }
    };
    fetch(P0, 0);
    fetch(P1, 1);
    skeleton(scan_w, ev_w, round_w);
}
