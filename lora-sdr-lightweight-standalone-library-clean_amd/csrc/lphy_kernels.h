// lphy_kernels.h — device code of the MI355X LoRa PHY demodulator and the
// per-SF launch templates.  Included by lphy_sf.hip, which is compiled once
// per spreading factor (-DLPHY_SF=n) so the kernel instantiations build in
// parallel; lphy_hip.hip (host side, C ABI) reaches them through the
// per-SF SfOps tables declared below.
//
// Hot path: per frame a prologue (whole-frame max|I|,|Q| for
// lora_demodulate's normalisation, LoRaDemod.cpp:60-78, and the two-symbol
// CFO/timing estimate, LoRaDemod.cpp:80-136 / phy.cpp:81-148), then per
// symbol CFO rotation -> KISS-identical FFT -> |X|^2 argmax
// (LoRaDemod.cpp:142-176 / phy.cpp:204-238), then per frame Hamming(8,4)
// decode + sx1272 CRC (LoRaDecoder.cpp:7-21, phy.cpp:245-261).
//
// Kernels:
//   k_prologue   one 256-thread workgroup per frame: max-abs reduction,
//                estimate FFTs (tile machinery of lphy_fft.h), offsets.
//   k_demod<SF>  256-thread tiles of T = 256/(N/16) symbols; each symbol is
//                staged to LDS with coalesced cf32 loads while the rotation
//                (glibc-exact sincosf in FP64) is applied, transformed by
//                LPS = N/16 lanes holding 16 complex each, and reduced by
//                cross-lane argmax.  No MFMA: the path is HBM/VALU bound.
//   k_finalize   one thread per frame: sync word, decode, CRC.
//   k_modulate*  bit-exact lora_modulate (producer for synthetic IQ).
//
// All device arithmetic is built with -ffp-contract=off (see
// __graft_entry__.build); every product/sum is evaluated in the reference's
// operand order so that symbol indices, sync words and decoded bytes are
// bit-identical to the reference's CPU path.
#pragma once
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "lphy_testing.h"  // (the device counter slots)

#include "../../include/lphy_hip.h"
#include "libm_exact.h"
#include "lphy_testing.h"
#include "lphy_fft.h"


using namespace lphy;

namespace lphy {
// ---------------------------------------------------------------------------
// Per-launch parameters (shared by every translation unit)
// ---------------------------------------------------------------------------
struct DemodArgs {
    const cf32* iq;        // frames * frame_samples
    const cf32* tw;        // N twiddles (KISS, forward)
    const cf32* down;      // N down-chirp samples (genChirp, down=true)
    const float* win;        // N window coefficients or nullptr
    uint16_t* syms;          // output symbols
    lphy_frame_meta* meta;   // per-frame meta (prologue -> demod hand-off)
    unsigned long long frames;
    unsigned long long frame_samples;
    unsigned long long total_syms;  // symbols per frame = frame_samples / step
    unsigned long long out_per_frame;
    int osr;
    int mode;
    int no_scratch;
    int est_units;           // estimate units per frame (est_syms * osr)
    int exact_rotation;      // LPHY_F_EXACT_ROTATION: no certified fast path
    float power_scale;       // LoRaDetector.hpp:29, (float)(20*log10((double)N))
    unsigned long long* counters;  // ctx counters: [0] rechecks, [1..4] phase clocks
    int spec;                // k_frames modes 1/2: speculative normalisation (no whole-frame pre-scan)
    // separate launches, SF 11-12 fast path, modes 1/2: the same speculation
    // across workgroups, per frame {max-abs of the two estimate symbols,
    // max-abs of the symbol windows, least certificate ratio (float bits,
    // atomic max / min), flags (1 NaN, 2 symbol left open)}; nullptr = off
    uint4* spec_big;
    int debug_recheck;       // LPHY_F_DEBUG_RECHECK: mark estimated frames kStatusRecheck before k_demod
    int wave;                // the fused k_wave launch ran (it settles its frames itself)
    // persistent demod workers: symbol stride per step split into whole
    // frames + symbols (host-computed, so the kernel never divides)
    unsigned stride_f, stride_s;
};

struct FinalArgs {
    const uint16_t* syms;
    uint8_t* bytes;
    lphy_frame_meta* meta;
    unsigned long long frames;
    unsigned long long nsyms;     // symbols per frame to decode
    unsigned long long sym_stride;
    int shift;                    // sf > 4 ? sf - 4 : 0
    int decode;
    int set_sync;
};

// Per-SF launch entry points (one table per lphy_sf.hip instance)
struct SfOps {
    int (*demod)(const DemodArgs&, hipStream_t, bool prologue, bool symbols, int per_cu);
    int (*frames)(const DemodArgs&, hipStream_t);
    int (*post)(int mode, const DemodArgs&, const FinalArgs&, bool fix, bool fin, hipStream_t);
    int (*estimate)(const DemodArgs&, hipStream_t);
    // debug build: read (and reset) this SF's failed index checks (else null)
    int (*violations)(unsigned long long* out, int reset);
};
extern const SfOps sf_ops_1, sf_ops_2, sf_ops_3, sf_ops_4, sf_ops_5, sf_ops_6,
    sf_ops_7, sf_ops_8, sf_ops_9, sf_ops_10, sf_ops_11, sf_ops_12;
}  // namespace lphy

namespace {

constexpr float kPi = 3.14159265358979323846f;  // lora_phy::PI (phy.hpp:20)
// Kernel MODE template argument: the lphy_mode in bits 0-1, plus kWinBit when
// a window is applied, so the per-sample window multiply is compile-time
// (a runtime branch per sample would split the staging block and serialise
// the 16 independent sincos chains of a lane).
constexpr int kWinBit = 4;
// ... and kOsrBit when osr > 1: k_demod then reads every osr-th sample
// (LoRaDemod.cpp:155, phy.cpp:225); the osr == 1 kernels keep unit-stride
// addressing.
constexpr int kOsrBit = 8;

#ifdef LPHY_PROFILE_PHASES
#endif

// Experiments only: -DLPHY_ONLY_SF=n instantiates the kernels of one SF
// (the launch switches below); the default build has every SF.

// ---------------------------------------------------------------------------
// Per-launch parameters
// ---------------------------------------------------------------------------


// (int)std::round(x) as the x86-64 reference evaluates it: cvttss2si on the
// rounded value, INT_MIN for NaN / out of range.
__device__ __forceinline__ int round_to_int(float x) {
    const float r = roundf(x);
    if (!(r >= -2147483648.0f && r < 2147483648.0f)) return (int)0x80000000u;
    return (int)r;
}

// Input sample for the estimate (no rotation): raw (mode 0) or
// [dechirped,] [normalised] (modes 1, 2).  idx is the absolute sample index
// in the frame, i the index inside the symbol (window / mode-0 chirp).
__device__ __forceinline__ cf32 est_sample(const DemodArgs& A, const cf32* fr,
                                             unsigned long long idx, int i, int N,
                                             const lphy_frame_meta& m) {
    cf32 x = fr[idx];
    if (A.mode == LPHY_MODE_DECHIRP_LORA_DEMODULATE)
        x = idx < A.total_syms * (unsigned long long)N ? cmul_x(x, A.down[idx & (N - 1)])
                                                       : czero();
    if (A.mode != LPHY_MODE_DEMODULATE && m.normalised) x = cscale(x, m.scale);
    if (A.win) x = cscale(x, A.win[i]);
    return x;
}

// max(|I|,|Q|) accumulation of LoRaDemod.cpp:62-66 for one sample:
// std::max(r, im) keeps r when im is NaN and yields NaN (never > mx) when r
// is NaN, so a NaN real part hides the whole sample.
__device__ __forceinline__ void maxabs_acc(float& mx, cf32 x) {
    const float r = fabsf(x.x), im = fabsf(x.y);
    const float m = (r < im) ? im : r;
    if (m > mx) mx = m;
}

// Internal frame status between the launches of one lphy_hip_demod_batch:
// the frame holds a non-finite value where the reference's Annex G complex
// product (cmul_x) could differ from the hot kernels' plain one, and is
// re-run exactly by k_post.  Never left in a record after the call.
constexpr int kStatusFixup = 0x7f5a0001;
// ... and: some symbols were left uncertified by the fused kernel's fast
// rotation (value kSymRecheck in the output; k_post recomputes exactly those)
constexpr int kStatusRecheck = 0x7f5a0002;
constexpr uint16_t kSymRecheck = 0xffff;  // never a bin index (N <= 4096)
// ... and: k_frames demodulated the frame with the normalisation of its
// first two symbols, but a later sample raised the frame's max-abs, so the
// estimate must be redone with the exact scale and the symbols' certificates
// re-checked against the exact rate (k_post settle_frames).  The record then
// holds {cfo: the frame's max-abs, time_offset: the symbols' least
// certificate ratio}; the second code also has symbols left open.
constexpr int kStatusSettle = 0x7f5a0003;
constexpr int kStatusSettleRecheck = 0x7f5a0004;

// Normalisation decision of LoRaDemod.cpp:60-78 from the frame's max-abs.
__device__ __forceinline__ lphy_frame_meta norm_meta(float mx, bool have_sync, int no_scratch) {
    lphy_frame_meta m{};
    m.scale = 1.0f;
    m.have_sync = have_sync;
    if (mx > 1.0f) {
        if (no_scratch) m.status = -ERANGE;  // LoRaDemod.cpp:69-71
        m.normalised = 1;
        m.scale = 1.0f / mx;
    }
    return m;
}
// The same in the hot kernels, whose scans return NaN for a frame with a
// non-finite sample: that frame goes to the exact re-run.
__device__ __forceinline__ lphy_frame_meta norm_meta_hot(float mx, bool have_sync, int no_scratch) {
    lphy_frame_meta m = norm_meta(mx, have_sync, no_scratch);
    if (!(mx <= 3.40282347e38f)) m.status = kStatusFixup;
    return m;
}

// ---------------------------------------------------------------------------
// Stage 1a (modes 1, 2): per-frame max(|I|,|Q|) of the [dechirped] frame and
// the normalisation decision (LoRaDemod.cpp:60-78).  A pure streaming
// reduction: one workgroup per frame, 16-byte loads, 8 in flight per lane.
// ---------------------------------------------------------------------------
template <int SF>
__global__ __launch_bounds__(kTile) void k_maxabs(DemodArgs A) {
    constexpr int N = 1 << SF;
    __shared__ float wmax[kTile / 64];
    const unsigned long long f = blockIdx.x;
    const int tid = threadIdx.x;
    const cf32* fr = A.iq + f * A.frame_samples;
    // spec_big: the two estimate symbols only (the symbols fold the rest)
    const unsigned long long count = A.spec_big ? 2ull * N : A.frame_samples;
    const unsigned long long dech_end = A.total_syms * N;  // whole symbols
    const bool dech = A.mode == LPHY_MODE_DECHIRP_LORA_DEMODULATE;
    float mx = 0.0f;
    bool bad = false;  // a non-finite [dechirped] sample: exact re-run (k_post)
    auto acc = [&](cf32 x, unsigned long long i) {
        if (dech) x = i < dech_end ? cmul(x, A.down[i & (N - 1)]) : czero();
        bad |= !(__builtin_isfinite(x.x) && __builtin_isfinite(x.y));
        maxabs_acc(mx, x);
    };
    if ((reinterpret_cast<uintptr_t>(fr) & 15) == 0) {
        const float4* f4 = reinterpret_cast<const float4*>(fr);
        const unsigned long long n4 = count / 2;
        constexpr int U = 8;
        unsigned long long j = tid;
        for (; j + (U - 1) * kTile < n4; j += U * kTile) {
            float4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = f4[j + u * kTile];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const unsigned long long i = 2 * (j + u * kTile);
                acc(cf32{v[u].x, v[u].y}, i);
                acc(cf32{v[u].z, v[u].w}, i + 1);
            }
        }
        for (; j < n4; j += kTile) {
            const float4 v = f4[j];
            acc(cf32{v.x, v.y}, 2 * j);
            acc(cf32{v.z, v.w}, 2 * j + 1);
        }
        if ((count & 1) && tid == 0) acc(fr[count - 1], count - 1);
    } else {
        for (unsigned long long i = tid; i < count; i += kTile) acc(fr[i], i);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float o = __shfl_xor(mx, off, 64);
        mx = o > mx ? o : mx;
    }
    if (__ballot(bad)) mx = __builtin_nanf("");
    if ((tid & 63) == 0) wmax[tid >> 6] = mx;
    __syncthreads();
    if (tid == 0) {
        mx = wmax[0];
        bool nf = !(mx == mx);
#pragma unroll
        for (int w = 1; w < kTile / 64; ++w) {
            nf |= !(wmax[w] == wmax[w]);
            mx = wmax[w] > mx ? wmax[w] : mx;
        }
        A.meta[f] = norm_meta_hot(nf ? __builtin_nanf("") : mx, A.total_syms >= 2, A.no_scratch);
        if (A.spec_big) A.spec_big[f] = make_uint4(__float_as_uint(nf ? 0.0f : mx), 0u, 0x7f7fffffu, nf ? 1u : 0u);
    }
}

// ---------------------------------------------------------------------------
// Stage 1b: offset estimate (LoRaDemod.cpp:80-140 / phy.cpp:81-148).
// Units = (symbol, osr phase) FFTs; a 256-thread tile packs T units, i.e.
// T/U whole frames when a frame has U <= T units (8 frames per workgroup at
// SF7), otherwise loops over one frame's units.  Per frame, one thread folds
// the unit results in symbol order exactly like the reference loop.
// ---------------------------------------------------------------------------
struct UnitResult {
    int idx;
    int valid;   // p > best_p reachable (maxValue > 0)
    float findex;
    float phase;
    int nan;     // a NaN bin (k_frames: the frame goes to the exact re-run)
};

// Detector outputs of one estimate unit from its FFT bins, which the team
// has written back to its LDS slot (LoRaDetector.hpp:60-71).
template <int SF>
__device__ __forceinline__ UnitResult unit_result(const cf32* lds, int slot, ArgMax best) {
    using G = Geo<SF>;
    constexpr int N = G::N;
    UnitResult r;
    const int idx = best.i;
    const float mv = best.v > 0.0f ? best.v : 0.0f;
    const float fund = sqrtf(mv);
    const cf32 lb = lds[G::addr(slot, idx > 0 ? idx - 1 : N - 1)];
    const cf32 rb = lds[G::addr(slot, idx < N - 1 ? idx + 1 : 0)];
    const float left = lphy_libm::cabsf_exact(lb.x, lb.y);
    const float right = lphy_libm::cabsf_exact(rb.x, rb.y);
    const double demon = (2.0 * (double)fund) - (double)right - (double)left;
    const float fi = demon == 0.0 ? 0.0f : (float)(0.5 * (double)(right - left) / demon);
    const cf32 bin = lds[G::addr(slot, idx)];
    r.idx = idx;
    r.valid = mv > 0.0f;  // osr == 1: p > -1e30 <=> maxValue > 0
    r.findex = fi;
    r.phase = lphy_libm::atan2f_exact(bin.y, bin.x);
    r.nan = 0;
    return r;
}

// Detector power of LoRaDetector.hpp:64, 20*log10(sqrt(maxValue)) - scale in
// single precision with glibc's log10f.  Only the osr > 1 estimate compares
// powers (with one phase, p > -1e30 <=> maxValue > 0).
__device__ __forceinline__ float detector_power(float max_value, float power_scale) {
    const float fund = sqrtf(max_value);
    const float db = 20.0f * lphy_libm::log10f_exact(fund);
    return db - power_scale;
}

// Running fold of the per-symbol estimates in symbol order
// (LoRaDemod.cpp:95-128 / phy.cpp:95-135).
struct EstFold {
    float sum_index = 0.0f, phase_diff = 0.0f, prev_phase = 0.0f;
    bool have_prev = false;
    unsigned sum_t = 0;
    __device__ __forceinline__ void add(int best_idx, float best_f, int best_t, float best_phase) {
        sum_t += (unsigned)best_t;
        sum_index += (float)best_idx + best_f;
        if (have_prev) {
            float d = best_phase - prev_phase;
            while (d > kPi) d -= 2.0f * kPi;
            while (d < -kPi) d += 2.0f * kPi;
            phase_diff += d;
        }
        prev_phase = best_phase;
        have_prev = true;
    }
    // per-phase selection over the osr phases of one symbol
    // (LoRaDemod.cpp:93-113 with the lowest-index tie-break, phy.cpp:106-121
    // without it); units arrive in (symbol, phase) order
    float best_p = -1e30f, best_f = 0.0f, best_phase = 0.0f;
    int best_idx = 0, best_t = 0, t = 0;
    __device__ __forceinline__ void unit(const UnitResult& r, float p, int osr, bool tie_low) {
        if (r.valid && (p > best_p || (tie_low && p == best_p && r.idx < best_idx))) {
            best_p = p; best_idx = r.idx; best_f = r.findex; best_t = t; best_phase = r.phase;
        }
        if (++t == osr) {
            add(best_idx, best_f, best_t, best_phase);
            best_p = -1e30f; best_f = 0.0f; best_phase = 0.0f;
            best_idx = 0; best_t = 0; t = 0;
        }
    }
    // offsets of LoRaDemod.cpp:130-140 / phy.cpp:137-147 into m
    __device__ __forceinline__ void finish(lphy_frame_meta& m, int est_syms, int N, int osr) const {
        const float avg_index = sum_index / (float)est_syms;
        const float cfo_coarse = avg_index / (float)N;
        float cfo_fine = 0.0f;
        if (est_syms > 1)
            cfo_fine = (phase_diff / (float)(est_syms - 1)) / (2.0f * kPi * (float)N);
        m.cfo = cfo_coarse + cfo_fine;
        const float frac = avg_index - floorf(avg_index + 0.5f);
        const float avg_t = (float)sum_t / (float)est_syms;
        m.time_offset = avg_t - frac * (float)N * (float)osr;
        m.t_off = round_to_int(m.time_offset);
        m.rate = -2.0f * kPi * m.cfo / (float)N;
    }
};

template <int SF>
__global__ __launch_bounds__(kTile) void k_estimate(DemodArgs A) {
    using G = Geo<SF>;
    constexpr int N = G::N, T = G::T;
    __shared__ cf32 lds[T * G::SSTRIDE];
    __shared__ cf32 twl[N];
    __shared__ ArgMax red[kTile / 64];
    __shared__ UnitResult units[T];
    __shared__ float upow[T];

    const int tid = threadIdx.x;
    const int U = A.est_units;
    const bool packed = U <= T;
    const int FPT = packed ? T / U : 1;
    const unsigned long long fbase = (unsigned long long)blockIdx.x * FPT;
    const unsigned long long step = (unsigned long long)N * A.osr;
    for (int i = tid; i < N; i += kTile) twl[i] = A.tw[i];

    // fold state of frame (fbase + tid), held by thread tid < FPT
    EstFold fold;
    lphy_frame_meta mine{};
    const bool folder = tid < FPT && fbase + tid < A.frames;
    if (folder) {
        if (A.mode == LPHY_MODE_DEMODULATE) {
            mine.scale = 1.0f;
            mine.have_sync = A.total_syms >= 2;
        } else {
            mine = A.meta[fbase + tid];
        }
    }

    const int slot = tid / G::LPS, lam = tid % G::LPS;
    const int chunks = packed ? 1 : (U + T - 1) / T;
    for (int c = 0; c < chunks; ++c) {
        int fl, u;
        if (packed) { fl = slot / U; u = slot % U; }
        else        { fl = 0; u = c * T + slot; }
        const unsigned long long f = fbase + fl;
        bool live = (packed ? fl < FPT : u < U) && f < A.frames;
        lphy_frame_meta m{};
        if (live) {
            if (A.mode == LPHY_MODE_DEMODULATE) m.scale = 1.0f;
            else m = A.meta[f];
            live = m.status == 0;
        }
        const int s = live ? u / A.osr : 0, t = live ? u % A.osr : 0;
        const cf32* fr = A.iq + f * A.frame_samples;
        __syncthreads();  // previous chunk's readers are done with lds / units
        // stage natural-order samples sym[t + i*osr] (LoRaDemod.cpp:86-92)
        const Stage<SF> st(slot, lam);
#pragma unroll
        for (int e = 0; e < G::E; ++e) {
            const int i = lam + e * G::LPS;
            cf32 x = czero();
            if (live) x = est_sample(A, fr, (unsigned long long)s * step + t + (unsigned long long)i * A.osr, i, N, m);
            st.put(lds, e, x);
        }
        __syncthreads();
        cf32 v[16];
        fft_tile<SF, false, true>(v, lds, slot, lam, twl);
        // keep the bins for the interpolation and the phase
#pragma unroll
        for (int e = 0; e < G::E; ++e) lds[G::addr(slot, bin_of<SF>(e, lam))] = v[e];
        ArgMax best = symbol_argmax<SF>(local_argmax<SF>(v, lam), red);
        __syncthreads();
        if (lam == 0) {
            units[slot] = live ? unit_result<SF>(lds, slot, best) : UnitResult{0, 0, 0.0f, 0.0f};
            if (A.osr > 1)
                upow[slot] = live ? detector_power(best.v > 0.0f ? best.v : 0.0f, A.power_scale) : 0.0f;
        }
        __syncthreads();
        if (folder) {
            const int first = packed ? tid * U : 0;
            const int nu = packed ? U : ((U - c * T) < T ? (U - c * T) : T);
            const bool tie_low = A.mode != LPHY_MODE_DEMODULATE;
            // an unset best bin is (0, 0), whose atan2 is 0
            for (int k = 0; k < nu; ++k)
                fold.unit(units[first + k], A.osr > 1 ? upow[first + k] : 0.0f, A.osr, tie_low);
        }
    }

    if (folder && mine.status == 0) {
        lphy_frame_meta m = mine;
        fold.finish(m, U / A.osr, N, A.osr);
        A.meta[fbase + tid] = m;
    }
}

// LPHY_F_DEBUG_RECHECK (tests): every frame the prologue estimated (status
// 0) is marked as if another workgroup had already left a sentinel in it, the
// state a symbol of the separate launches may observe at any time
// (sym_ctx); k_post's recheck then finds no sentinel and clears the mark.
__global__ void k_mark_recheck(lphy_frame_meta* meta, unsigned long long frames) {
    const unsigned long long f = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (f < frames && meta[f].status == 0) meta[f].status = kStatusRecheck;
}

// ---------------------------------------------------------------------------
// Stage 2: per-symbol demodulation.  Persistent grid; each 256-thread
// workgroup stages the twiddles (and, up to N = 1024, the down-chirp and the
// window) in LDS once, then loops over tiles of T symbols.
// ---------------------------------------------------------------------------
// Per-tile context of the symbol a team (LPS lanes) works on.  Frame and
// symbol indices are 32-bit (lphy_hip_demod_batch checks frames*symbols and
// frame_samples fit) and advance incrementally: no division per tile.
struct SymCtx {
    unsigned f, s;            // frame, symbol within the frame
    unsigned base;            // first sample of the (shifted) window in the frame
    float start, rate, scale;
    int toff;                 // the frame's t_off (fast-rotation table offset)
    bool ok, have_sync, live;
};

template <bool OSR = false>
__device__ __forceinline__ SymCtx sym_ctx(const DemodArgs& A, unsigned f, unsigned s, bool live,
                                          int N, const lphy_frame_meta& m) {
    SymCtx c;
    c.f = f;
    c.s = s;
    // kStatusRecheck only marks that some symbol of the frame left a
    // sentinel for k_post (another team or workgroup may set it while this
    // symbol's record is read): its estimate stands, and k_post recomputes
    // the sentinels only, so every other symbol must still be demodulated
    c.ok = live && (m.status == 0 || m.status == kStatusRecheck);
    c.live = live;
    c.have_sync = m.have_sync != 0;
    // LoRaDemod.cpp:144-151 / phy.cpp:208-216, in 32 bits
    const unsigned osr = OSR ? (unsigned)A.osr : 1u;
    const unsigned step = (unsigned)N * osr, count = (unsigned)A.frame_samples;
    unsigned base = s * step;
    const int t = m.t_off;
    // all in 32 bits without overflow: count < 2^31 (lphy_hip_demod_batch),
    // base + step <= count for a symbol of the frame, |INT_MIN| = 2^31
    if (t > 0) {
        if (base + step <= count && (unsigned)t <= count - step - base) base += (unsigned)t;
    } else if (t < 0) {
        const unsigned off = 0u - (unsigned)t;
        if (off <= base) base -= off;
    }
    c.base = base;
    c.rate = m.rate;
    c.scale = m.scale;
    c.toff = m.t_off;
    // LoRaDemod.cpp:152-153 / phy.cpp:217-218; (float) of the size_t product
    // equals (float) of the same value held in 32 bits; x / 1.0f == x
    const float toff = OSR ? (float)m.t_off / (float)osr : (float)m.t_off;
    c.start = m.rate * ((float)(s * (unsigned)N) + toff);
    return c;
}

// One rotated input sample (LoRaDemod.cpp:152-163, phy.cpp:217-229).
template <int SF, int MODE, bool AG = false>
__device__ __forceinline__ cf32 rotate_sample(cf32 x, int i, const SymCtx& c,
                                              const cf32* down, const float* win, bool large) {
    constexpr int N = 1 << SF;
    if constexpr ((MODE & 3) == LPHY_MODE_DEMODULATE) {
        x = cmul_t<AG>(x, down[i]);  // phy.cpp:219-220: down-chirp of the window
    } else {
        if constexpr ((MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE) {
            // the external dechirp ran on the unshifted buffer
            // (e2e_chain_test.cpp:88-93): chirp index of the absolute sample
            // (frames hold whole symbols in this mode)
            x = cmul_t<AG>(x, down[((unsigned)c.base + (unsigned)i) & (N - 1)]);
        }
        // LoRaDemod.cpp:74-76; scale == 1.0f exactly when no rescale was
        // needed and x * 1.0f == x, so the multiply is unconditional
        x = cscale(x, c.scale);
    }
    const float ph = c.start + c.rate * (float)i;
    float sn, cs;
#ifdef LPHY_ABLATE_SINCOS  // timing experiments only (tools/ubench/demod_ablate)
    sn = ph; cs = 1.0f - ph;
    (void)large;
#else
    if (large) lphy_libm::sincosf_large(ph, &sn, &cs);
    else lphy_libm::sincosf_fast(ph, &sn, &cs);
#endif
    x = cmul_t<AG>(x, cf32{cs, sn});
    if constexpr ((MODE & kWinBit) != 0) x = cscale(x, win[i]);
    return x;
}

// Exact restaging of the team's symbol from its IQ in memory, one sample at
// a time (rare paths: the certificate's re-check, and the Annex G re-run of
// a transform that produced a NaN bin).
template <int SF, int MODE, bool AG>
__device__ __forceinline__ void restage_symbol(cf32* lds, const Stage<SF>& stg, const cf32* src,
                                               const SymCtx& c, int lam, const cf32* down,
                                               const float* win, unsigned osr = 1) {
    using G = Geo<SF>;
    // the lane's samples loaded first, all in flight together (one memory
    // round trip for the symbol: k_post re-runs run at low occupancy, where
    // a load per sincos cost a round trip each - mode A's ~6,600 re-runs at
    // SF 7 took 43 us)
    cf32 raw[G::E];
#pragma unroll
    for (int e = 0; e < G::E; ++e) raw[e] = src[(unsigned)(lam + e * G::LPS) * osr];
#pragma unroll
    for (int e = 0; e < G::E; ++e) {
        const int i = lam + e * G::LPS;
        const float ph = c.start + c.rate * (float)i;
        stg.put(lds, e, rotate_sample<SF, MODE, AG>(raw[e], i, c, down, win, lphy_libm::sincosf_needs_large(ph)));
    }
}

// Stage the team's symbol (rotated, natural order) into its LDS slot.
template <int SF, int MODE>
__device__ __forceinline__ void stage_symbol(cf32* lds, const Stage<SF>& stg, const cf32 (&raw)[16],
                                             const cf32* src, const SymCtx& c, int lam,
                                             const cf32* down, const float* win, int osr = 1) {
    using G = Geo<SF>;
#pragma unroll
    for (int e = 0; e < G::E; ++e)
        stg.put(lds, e, rotate_sample<SF, MODE>(raw[e], lam + e * G::LPS, c, down, win, false));
    // rare: |phase| >= 120 rad (large CFO x long frame).  The angle is
    // monotone in i, so the lane's first and last samples bound it.
    if (lphy_libm::sincosf_needs_large(c.start + c.rate * (float)lam) ||
        lphy_libm::sincosf_needs_large(c.start + c.rate * (float)(lam + (G::E - 1) * G::LPS))) {
        for (int e = 0; e < G::E; ++e) {
            const int i = lam + e * G::LPS;
            if (lphy_libm::sincosf_needs_large(c.start + c.rate * (float)i))
                stg.put(lds, e, rotate_sample<SF, MODE>(src[(unsigned)i * (unsigned)osr], i, c, down, win, true));
        }
    }
}

// debug build: sample `off` of frame `f` lies inside the batch (bound_check)
__device__ __forceinline__ void iq_check(const DemodArgs& A, unsigned long long f, long long off) {
    bound_check((long long)f, (long long)A.frames);
    bound_check(off, (long long)A.frame_samples);
}

// k_frames' IQ loads (each sample read once, the estimate symbols twice):
// non-temporal, so the stream does not evict the partly written output
// lines and the tables from L2 (as k_wave's IQ DMA, lphy_wave.h
// LPHY_IQ_CPOL).  Same-box A/B (profiles/r5/ab_iq_nt.txt): SF 8 fused
// 0.999-1.012 -> 0.977-0.979 ms, SF 7 within noise; C1 WRITE_SIZE 33.0 ->
// 12.6 MB per launch.  (-DLPHY_IQ_NT=0 for timing experiments only.)
#ifndef LPHY_IQ_NT
#define LPHY_IQ_NT 1
#endif
__device__ __forceinline__ cf32 ld_iq(const cf32* p) {
#if LPHY_IQ_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

__device__ __forceinline__ void store_symbol(const DemodArgs& A, const SymCtx& c, uint16_t idx) {
    bound_check(c.f, (long long)A.frames);
    if (c.have_sync && c.s < 2) {
        if (c.s == 0) A.meta[c.f].sw0 = idx;
        else A.meta[c.f].sw1 = idx;
    } else {
        const unsigned o = c.have_sync ? c.s - 2 : c.s;
        bound_check(o, (long long)A.out_per_frame);
        A.syms[(unsigned long long)c.f * A.out_per_frame + o] = idx;
    }
}

// (shared by k_demod's fast path and k_frames; see the certified fast
// rotation comment below k_frames' max-abs scan)
__device__ __forceinline__ float max3_abs(float m, float a, float b) {
    float r;
    asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}

constexpr float kU = 5.9604645e-8f;  // 2^-24

// Table of frame `rec` (rate, scale, t_off): t_i for i = lane, lane+64, ...
template <int SF, int MODE>
__device__ __forceinline__ void build_rtab(cf32* tab, float rate, float scale, int t_off,
                                           const cf32* down, const float* win, int lane) {
    constexpr int N = 1 << SF;
    (void)t_off;
    for (int i = lane; i < N; i += 64) {
        float sn, cs;
        lphy_libm::sincosf_exact(rate * (float)i, &sn, &cs);
        cf32 t = cf32{cs, sn};
        if constexpr ((MODE & 3) == LPHY_MODE_DEMODULATE) t = cmul(down[i], t);
        if constexpr ((MODE & 3) != LPHY_MODE_DEMODULATE) t = cscale(t, scale);
        if constexpr ((MODE & kWinBit) != 0) t = cscale(t, win[i]);
        tab[i] = t;
    }
}

// Whether the fast path may take this symbol unit: every window (mode 2
// dechirps each sample exactly at its own chirp index before the table).
template <int SF, int MODE>
__device__ __forceinline__ bool fast_applies(const SymCtx& c, int t_off) {
    (void)c;
    (void)t_off;
    return true;
}

// The certificate of the header comment.  amax bounds max(|Re y|, |Im y|)
// over the symbol's samples before rotation (modes 1/2: <= 1 after the
// frame's normalisation; mode 0: measured).
//
// Range guards keep every rounding relative: amax >= 1e-20 (denormal
// arithmetic stays negligible against B), b.v >= 1e-30 (a normal |X|^2), and
// a runner-up below 1e-30 is taken as 1e-30.
// extra: further u-multiples of a sample's rotation error (the two-table
// rotation of k_demod's fast path)
template <int SF>
__device__ __forceinline__ float cert_bound(float rate, float start, float amax, float extra = 0.0f) {
    constexpr int N = 1 << SF, L = (SF + 1) / 2;
    const float A = (float)N * 1.41421366f * amax * 1.0001f;
    const float ar = fabsf(rate) * (float)N;
    const float P = fabsf(start) + ar;
    return kU * A * ((24.0f + 12.0f * L + extra) + 2.0f * ar + P) * 1.001f;
}
// winner's lead over the runner-up, less the |X|^2 roundings.  The square
// roots are the hardware v_sqrt_f32 (within 1 ulp, i.e. 2u relative, for the
// normal inputs the certificate admits: b.v >= 1e-30, runner-up clamped to
// 1e-30), charged as 2 ulp = 4u on each side on top of the 8u: the
// correctly rounded sqrtf's Newton fix-up cost ~20 VALU per symbol tile.
// A NaN winner stays NaN and fails the comparison.
__device__ __forceinline__ float cert_gap(const ArgMax2& b) {
#ifdef LPHY_AB_SQRT_EXACT  // A/B timing only: the correctly rounded sqrtf
    return sqrtf(b.v) * (1.0f - 8.0f * kU) - sqrtf(fmaxf(b.v2, 1e-30f)) * (1.0f + 8.0f * kU);
#else
    return __builtin_amdgcn_sqrtf(b.v) * (1.0f - 12.0f * kU) -
           __builtin_amdgcn_sqrtf(fmaxf(b.v2, 1e-30f)) * (1.0f + 12.0f * kU);
#endif
}
template <int SF>
__device__ __forceinline__ bool fast_certified(const ArgMax2& b, const SymCtx& c, float amax,
                                               float extra = 0.0f) {
    constexpr int N = 1 << SF;
    const float A = (float)N * 1.41421366f * amax * 1.0001f;
    const float B = cert_bound<SF>(c.rate, c.start, amax, extra);
    return cert_gap(b) > 4.0f * B && A < 1e18f && amax >= 1e-20f && b.v >= 1e-30f;
}

// Stage 2: per-symbol demodulation, persistent grid.  The workgroup stages
// the twiddles (and, up to N = 1024, the down-chirp and window) in LDS once.
//  * SF <= 10 (a symbol's LPS <= 64 lanes sit in one wavefront): every
//    wavefront is an independent worker with its own LDS slots and no
//    workgroup barrier in its loop; it software-pipelines the next tile's
//    frame record (during staging) and IQ (during the FFT).
//  * SF 11-12: workgroup tiles with barriers (a symbol spans wavefronts).
//    Symbols take the certified fast rotation (as k_frames) with
//    a two-table rotation: e^{j rate i} = e^{j rate 64h} e^{j rate l} for
//    i = 64h + l, whose 64 + N/64 entries the team computes per tile (exact
//    sincos) instead of one sincos per sample; uncertified symbols are left
//    to k_post (kSymRecheck, kStatusRecheck).  LPHY_F_EXACT_ROTATION and
//    osr > 1 keep the per-sample rotation.
template <int SF, int MODE, int OCC>
__global__ __launch_bounds__(kTile, OCC) void k_demod(DemodArgs A) {
    using G = Geo<SF>;
    constexpr int N = G::N;
    constexpr bool TAB = N <= 1024;  // chirp + window tables in LDS
    constexpr bool WAVE = G::LPS <= 64;
    constexpr int WT = WAVE ? 64 / G::LPS : G::T;  // symbols per worker tile
    constexpr bool FASTB = !WAVE && (MODE & kOsrBit) == 0;  // two-table fast path
    constexpr int NH = N / 64;                               // high-part entries
    __shared__ cf32 lds[G::T * G::SSTRIDE];
    __shared__ cf32 twl[N];
    __shared__ cf32 dnl[TAB ? N : 1];
    __shared__ float wnl[TAB ? N : 1];
    __shared__ ArgMax red[kTile / 64];
    // double-buffered by tile parity: the next tile's tables are built at the
    // end of this one, and the reductions need no trailing barrier
    __shared__ ArgMax2 red2[2][FASTB ? kTile / 64 : 1];
    __shared__ float redm[2][FASTB ? kTile / 64 : 1];
    __shared__ cf32 thi[2][FASTB ? G::T : 1][FASTB ? NH : 1];
    __shared__ cf32 tlo[2][FASTB ? G::T : 1][FASTB ? 64 : 1];
    const bool fastb = FASTB && !A.exact_rotation;
    unsigned tp = 0;  // tile parity

    const int tid = threadIdx.x;
    for (int i = tid; i < N; i += kTile) {
        twl[i] = A.tw[i];
        if constexpr (TAB) {
            if ((MODE & 3) != LPHY_MODE_LORA_DEMODULATE) dnl[i] = A.down[i];
            if (A.win) wnl[i] = A.win[i];
        }
    }
    __syncthreads();
    const cf32* down = TAB ? dnl : A.down;
    const float* win = A.win ? (TAB ? wnl : A.win) : nullptr;

    const int slot = tid / G::LPS, lam = tid % G::LPS;
    const unsigned S = (unsigned)A.total_syms;
    const unsigned nframes = (unsigned)A.frames;
    const int wslot = WAVE ? slot % WT : slot;  // symbol slot inside the worker tile
    unsigned worker;
    if constexpr (WAVE) worker = blockIdx.x * (kTile / 64) + (tid >> 6);
    else worker = blockIdx.x;
    const Stage<SF> stg(slot, lam);

    // this team's first symbol and its (frame, symbol) coordinates
    const unsigned g0 = worker * WT + wslot;
    unsigned f = g0 / S, s = g0 - f * S;
    auto step = [&](unsigned& ff, unsigned& ss) {
        ss += A.stride_s;
        ff += A.stride_f;
        if (ss >= S) { ss -= S; ++ff; }
    };
    // the worker's tile loop ends when its first team passes the last frame
    const unsigned fw0 = (worker * WT) / S;
    unsigned fw = fw0, sw = worker * WT - fw0 * S;

    // prologue of the software pipeline
    constexpr bool OSR = (MODE & kOsrBit) != 0;
    const unsigned osr = OSR ? (unsigned)A.osr : 1u;  // sample stride of a symbol
    lphy_frame_meta m = A.meta[f < nframes ? f : 0];
    SymCtx c = sym_ctx<OSR>(A, f < nframes ? f : 0, f < nframes ? s : 0, f < nframes, N, m);
    // the two rotation tables of a tile's symbol (scale folded into the low
    // one), written by the team's first NH + 64 lanes
    auto build_tables = [&](const SymCtx& cc, unsigned b) __attribute__((always_inline)) {
        if constexpr (FASTB) {
            if (cc.ok) {
                float sn, cs;
                if (lam < NH) {
                    lphy_libm::sincosf_exact(cc.rate * (float)(64 * lam), &sn, &cs);
                    thi[b][slot][lam] = cf32{cs, sn};
                } else if (lam < NH + 64) {
                    const int l = lam - NH;
                    lphy_libm::sincosf_exact(cc.rate * (float)l, &sn, &cs);
                    cf32 t = cf32{cs, sn};
                    if constexpr ((MODE & 3) != LPHY_MODE_DEMODULATE) t = cscale(t, cc.scale);
                    tlo[b][slot][l] = t;
                }
            }
        }
    };
    if (FASTB && fastb) build_tables(c, 0);  // visible after the loop's first barrier
    cf32 raw[16];
    {
        const cf32* src = A.iq + (unsigned long long)c.f * A.frame_samples + c.base;
#pragma unroll
        for (int e = 0; e < G::E; ++e) raw[e] = src[(unsigned)(lam + e * G::LPS) * osr];
    }

#ifdef LPHY_PROFILE_PHASES  // timing experiments only: per-phase clock sums
    unsigned long long ph_stage = 0, ph_fft = 0, ph_tail = 0;
#endif
    while (fw < nframes) {
#ifdef LPHY_PROFILE_PHASES
        const unsigned long long p0 = clock64();
#endif
        // next tile: coordinates and frame record (in flight during staging)
        unsigned nf = f, ns = s, nfw = fw, nsw = sw;
        step(nf, ns);
        step(nfw, nsw);
        const bool nlive = nf < nframes;
        const lphy_frame_meta nm = A.meta[nlive ? nf : 0];

        if constexpr (!WAVE) __syncthreads();  // previous tile's readers done
        float amax = 0.0f;  // fast path, mode 0: the team's max(|Re x|, |Im x|)
        if (FASTB && fastb) {
            // this tile's tables were built at the end of the previous one
            const cf32 tl = tlo[tp][slot][lam & 63];
#pragma unroll
            for (int e = 0; e < G::E; ++e) {
                const int i = lam + e * G::LPS;
                cf32 p = raw[e];
                if constexpr ((MODE & 3) == LPHY_MODE_DEMODULATE) {
                    amax = max3_abs(amax, p.x, p.y);
                    p = cmul(p, down[i]);
                }
                if constexpr ((MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE)
                    p = cmul(p, down[(c.base + (unsigned)i) & (N - 1)]);
                // modes 1/2 (spec_big): the [dechirped] samples' max-abs
                if constexpr ((MODE & 3) != LPHY_MODE_DEMODULATE) amax = max3_abs(amax, p.x, p.y);
                cf32 q = cmul_fma(cmul_fma(p, tl), thi[tp][slot][(lam >> 6) + e * (G::LPS / 64)]);
                if constexpr ((MODE & kWinBit) != 0) q = cscale(q, win[i]);
                stg.put(lds, e, c.ok ? q : czero());
            }
        } else {
            stage_symbol<SF, MODE>(lds, stg, raw, A.iq + (unsigned long long)c.f * A.frame_samples + c.base,
                                   c, lam, down, win, (int)osr);
        }
        team_sync<SF>();
#ifdef LPHY_PROFILE_PHASES
        const unsigned long long p1 = clock64();
#endif

        // next tile's IQ: in flight during this tile's FFT
        const SymCtx nc = sym_ctx<OSR>(A, nlive ? nf : 0, nlive ? ns : 0, nlive, N, nm);
        if (nfw < nframes) {
            const cf32* nsrc = A.iq + (unsigned long long)nc.f * A.frame_samples + nc.base;
#ifdef LPHY_ABLATE_LOAD  // timing experiments only
            (void)nsrc;
#pragma unroll
            for (int e = 0; e < G::E; ++e) raw[e] = raw[e] * 0.999f + cf32{(float)e, (float)lam};
#else
#pragma unroll
            for (int e = 0; e < G::E; ++e) raw[e] = nsrc[(unsigned)(lam + e * G::LPS) * osr];
#endif
        }

        cf32 v[16];
#ifdef LPHY_ABLATE_FFT  // timing experiments only
        {
            const Stage<SF> st2(slot, lam);
#pragma unroll
            for (int e = 0; e < G::E; ++e) v[e] = lds_ld(lds, G::at8(st2.lb8, G::cpart(e * G::LPS) << 3));
        }
#else
        if (FASTB && fastb) fft_tile<SF, true>(v, lds, slot, lam, twl);
        else fft_tile<SF>(v, lds, slot, lam, twl);
#endif
        if constexpr (FASTB) {
            if (fastb) {
#ifdef LPHY_PROFILE_PHASES
                const unsigned long long q2 = clock64();
#endif
                // certificate (fast_certified, with the two-table rotation's
                // further 6u); a NaN or near-tie leaves the symbol to k_post
                // the team's top two and its samples' max-abs in one exchange
                const bool tm = (MODE & 3) == LPHY_MODE_DEMODULATE || A.spec_big != nullptr;
                const ArgMax2 b2 = symbol_argmax2_wg<SF, false>(local_argmax2<SF>(v, lam), red2[tp],
                                                                tm ? &amax : nullptr, redm[tp]);
                // modes 1/2: normalised frame (under spec_big, k_post's close
                // confirms the normalisation or settles the frame)
                const float am = (MODE & 3) == LPHY_MODE_DEMODULATE ? amax : 1.0f;
                const bool redo = !fast_certified<SF>(b2, c, am, 6.0f);
                if (c.ok && lam == 0) {
                    store_symbol(A, c, redo ? kSymRecheck : (uint16_t)b2.i);
                    if (redo) A.meta[c.f].status = kStatusRecheck;
                }
                if constexpr ((MODE & 3) != LPHY_MODE_DEMODULATE) {
                    if (A.spec_big && c.ok) {
                        uint4* r = &A.spec_big[c.f];
                        const cf32 q = v[0] * v[0];
                        const float q2 = q.x + q.y;
                        if (!(q2 == q2)) atomicOr(&r->w, 1u);  // a NaN sample reaches every bin
                        if (lam == 0) {
                            atomicMax(&r->y, __float_as_uint(amax));
                            if (redo) atomicOr(&r->w, 2u);
                            else atomicMin(&r->z, __float_as_uint(cert_gap(b2) / cert_bound<SF>(c.rate, c.start, 1.0f, 6.0f)));
                        }
                    }
                }
                build_tables(nc, tp ^ 1u);  // the next tile's, behind its first barrier
                tp ^= 1u;
                c = nc;
                f = nf; s = ns; fw = nfw; sw = nsw;
#ifdef LPHY_PROFILE_PHASES
                const unsigned long long q3 = clock64();
                ph_stage += p1 - p0; ph_fft += q2 - p1; ph_tail += q3 - q2;
#endif
                continue;
            }
        }
        // a NaN bin may hide a (NaN, NaN) product, where the reference's
        // Annex G product differs: the frame goes to the exact re-run
        if (fft_has_nan<SF>(v) && c.ok) A.meta[c.f].status = kStatusFixup;
#ifdef LPHY_PROFILE_PHASES
        const unsigned long long p2 = clock64();
#endif
        const ArgMax best = symbol_argmax<SF>(local_argmax<SF>(v, lam), red);
        if (c.ok && lam == 0) store_symbol(A, c, (uint16_t)best.i);
        if constexpr (WAVE) team_sync<SF>();  // slot reads done before restaging
        c = nc;
        f = nf; s = ns; fw = nfw; sw = nsw;
#ifdef LPHY_PROFILE_PHASES
        const unsigned long long p3 = clock64();
        ph_stage += p1 - p0; ph_fft += p2 - p1; ph_tail += p3 - p2;
#endif
    }
#ifdef LPHY_PROFILE_PHASES
    if ((tid & 63) == 0) {
        atomicAdd(&A.counters[kCtrClocks + 0], ph_stage);
        atomicAdd(&A.counters[kCtrClocks + 1], ph_fft);
        atomicAdd(&A.counters[kCtrClocks + 2], ph_tail);
    }
#endif
}

// ---------------------------------------------------------------------------
// Fused single launch (LPS <= 64 i.e. SF <= 10, two estimate symbols, osr 1).
// Every wavefront owns the frames f = w, w + W, w + 2W, ... (W waves in the
// grid) and runs their whole chain itself, so no data crosses wavefronts:
//   M  max(|I|,|Q|) scan of the frame (LoRaDemod.cpp:60-78), wave-wide
//   E  the two estimate FFTs (LoRaDemod.cpp:80-140 / phy.cpp:81-148) and the
//      fold into the frame's offsets
//   D  the frame's symbols (rotation, FFT, argmax)
// The wave works through a stream of "units" in tiles of WT = 64/LPS, one
// unit per team of LPS lanes.  Its frames go in groups of F = WT/2 (at
// least 1), whose 2F estimate units fill EBT whole tiles (EB):
//   [EB(0), one spacer tile] then per group g:
//   [D(g): DBT - 1 tiles, EB(g+1), D(g): its last tile]
// where D(g) is the F S symbol units of the group (the last tile padded
// with dead units).  No tile mixes estimate units with symbol units: a
// mixed tile runs the estimate staging, the exact transform and the exact
// top two for the whole wave (measured at SF7: one mixed tile per frame
// cost 1.8x a symbol tile, 20 % of the wave's clocks; a whole EB tile for
// four frames costs 2.1x, 6 %).  The F frames of an EB tile fold on the
// first lanes of their teams at once.  EB(g+1) folds two tiles before
// D(g+1) starts (what the one-tile-ahead context and IQ prefetch need).
// M of group g+1's frames runs right before the EB tile.  Measured
// alternatives, all slower at SF7 than this blocking 8-deep scan: M
// streamed in row chunks held in registers across the FFT (spills, 1.35x),
// M streamed by LDS-DMA into a per-wave ring (1.15x), scan-only workgroups
// beside the symbol waves (1.3-5x: they need ~25 % of the slots to stay
// ahead), the group's F scans with all their loads in flight at once (2 %
// slower in mode 2).
// Frame records pass between teams through a 2F-slot ring per wave in LDS
// (the group in demodulation and the next one).  Compared with separate launches this
// removes a whole-batch pass (the prologue kernels) and overlaps the
// HBM-bound max-abs scans of some waves with the VALU-bound transforms of
// the others.
// ---------------------------------------------------------------------------
struct FrameArgs {
    DemodArgs A;
    unsigned waves;  // wavefronts in the grid
};

// Per-frame record of the public meta array written by E: every field but
// sw0 / sw1, which the D tasks of symbols 0 and 1 write (disjoint bytes, so
// the two L2 write-backs cannot clobber each other).
__device__ __forceinline__ void meta_put_est(lphy_frame_meta* dst, const lphy_frame_meta& m) {
    float4* d16 = reinterpret_cast<float4*>(dst);
    d16[0] = float4{m.cfo, m.time_offset, m.rate, m.scale};
    int* d8 = reinterpret_cast<int*>(dst);
    d8[4] = m.t_off;
    d8[5] = m.status;
    uint8_t* b = reinterpret_cast<uint8_t*>(dst);
    b[28] = m.sync_word;
    b[29] = m.crc_ok;
    b[30] = m.normalised;
    b[31] = m.have_sync;
}

// Max-abs of frame f by one wavefront (16-byte loads, 8 in flight per
// lane), same arithmetic as k_maxabs; the result is in every lane.
//
// Fast form of the aligned bulk (one v_max3 per sample): max(mx, |re|, |im|)
// equals the reference's fold for samples without NaN, and the frame's
// samples are summed alongside (one packed add per sample) so that any NaN
// - or an overflow to inf, which could make one - sends the whole frame to
// the per-sample fold above, whose NaN rules (a NaN real part hides the
// sample) v_max3 does not have.  In mode 2 only the whole symbols are
// scanned: the zeros the reference's dechirp leaves past them never raise
// the maximum.

template <int SF, int MODE>
__device__ __forceinline__ float wave_maxabs(const DemodArgs& A, unsigned f, const cf32* down,
                                             unsigned limit = 0) {
    constexpr int N = 1 << SF;
    constexpr bool DECH = (MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE;
    const int lane = threadIdx.x & 63;
    const cf32* fr = A.iq + (unsigned long long)f * A.frame_samples;
    // limit: the first `limit` samples only (speculative normalisation)
    const unsigned count = limit ? limit : (DECH ? (unsigned)A.total_syms * N : (unsigned)A.frame_samples);
    iq_check(A, f, (long long)count - 1);
    float mx = 0.0f;
    bool bad = false;  // non-finite [dechirped] sample
    auto acc = [&](cf32 x, unsigned i) {
        if constexpr (DECH) x = cmul(x, down[i & (N - 1)]);
        bad |= !(__builtin_isfinite(x.x) && __builtin_isfinite(x.y));
        maxabs_acc(mx, x);
    };
    // loads in flight per lane (round 1, whole-frame scan at SF7: 16, 24,
    // 32 and 33 within 1 %; round 2, with the samples staged in registers:
    // 8 spills 6 VGPRs where 16 spills 15, 4 % faster under speculation and
    // 1 % with the whole-frame scan)
#ifdef LPHY_MAXABS_U
    constexpr int U = LPHY_MAXABS_U;
#else
    constexpr int U = 8;
#endif
    // chirp index of sample 2 (b + 64 u + lane) for a round base b = 64 U r:
    // the 128 U r term vanishes mod N
    static_assert((128 * U) % N == 0, "chirp phase of the unrolled scan");
    bool exact = (reinterpret_cast<uintptr_t>(fr) & 15) != 0;
    if (!exact) {
        const float4* f4 = reinterpret_cast<const float4*>(fr);
        const unsigned n4 = count / 2;
        float fm = 0.0f;
        cf32 sum = czero();
        auto round = [&](const float4 (&v)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                cf32 a = cf32{v[u].x, v[u].y}, b = cf32{v[u].z, v[u].w};
                if constexpr (DECH) {
                    const unsigned ci = (2u * (unsigned)lane + 128u * (unsigned)u) & (N - 1);
                    a = cmul(a, down[ci]);
                    b = cmul(b, down[(ci + 1) & (N - 1)]);
                }
                fm = max3_abs(fm, a.x, a.y);
                fm = max3_abs(fm, b.x, b.y);
                sum = sum + a;
                sum = sum + b;
            }
        };
        unsigned base = 0;
        for (; base + U * 64 <= n4; base += U * 64) {
            float4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = f4[base + u * 64 + lane];
            round(v);
        }
        if (base < n4) {  // last partial round, zero-filled (zeros never raise the max)
            float4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const unsigned j = base + u * 64 + lane;
                v[u] = j < n4 ? f4[j] : float4{0.0f, 0.0f, 0.0f, 0.0f};
            }
            round(v);
        }
        // a NaN or inf sample (or an inf - inf) ends in the sum as NaN, or
        // in the maximum as inf: the frame goes to the exact re-run
        bad = !(sum.x == sum.x && sum.y == sum.y) || !(fm <= 3.40282347e38f);
        mx = fm;
        if ((count & 1) && lane == 0) acc(fr[count - 1], count - 1);
    } else {
        for (unsigned i = lane; i < count; i += 64) acc(fr[i], i);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float o = __shfl_xor(mx, off, 64);
        mx = o > mx ? o : mx;
    }
    // NaN: the caller's norm_meta_hot routes the frame to k_post
    return __ballot(bad) ? __builtin_nanf("") : mx;
}

// Max-abs of samples [lo, hi) of frame f by one wavefront, per-sample fold
// with the reference's NaN rules; `bad` when one is non-finite.  Used for
// the few samples no symbol window of a speculatively normalised frame
// covers (a negative time shift's last samples, mode 1's partial symbol).
template <int SF, int MODE>
__device__ float wave_range_maxabs(const DemodArgs& A, unsigned f, unsigned lo, unsigned hi,
                                   const cf32* down, bool& bad) {
    constexpr int N = 1 << SF;
    const int lane = threadIdx.x & 63;
    const cf32* fr = A.iq + (unsigned long long)f * A.frame_samples;
    float mx = 0.0f;
    bool b = false;
    if (hi > lo) iq_check(A, f, (long long)hi - 1);
    for (unsigned i = lo + (unsigned)lane; i < hi; i += 64) {
        cf32 x = fr[i];
        if constexpr ((MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE) x = cmul(x, down[i & (N - 1)]);
        b |= !(__builtin_isfinite(x.x) && __builtin_isfinite(x.y));
        maxabs_acc(mx, x);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float o = __shfl_xor(mx, off, 64);
        mx = o > mx ? o : mx;
    }
    bad = __ballot(b) != 0;
    return mx;
}

// End of the samples the frame's symbol windows (shifted by t_off as
// LoRaDemod.cpp:144-150 does) and its two estimate symbols cover together,
// a contiguous run from sample 0; the frame's max-abs needs [end, count) too.
__device__ __forceinline__ unsigned covered_end(unsigned S, unsigned N, unsigned count, int t) {
    unsigned end = S * N;
    if (t > 0) {
        // windows s with s N + t + N <= count are shifted
        if ((unsigned long long)t + N <= count) {
            const unsigned long long smax = ((unsigned long long)count - (unsigned)t - N) / N;
            const unsigned long long last = smax < S - 1 ? smax : S - 1;
            const unsigned long long e = (last + 1) * N + (unsigned)t;
            if (e > end) end = (unsigned)e;
        }
    } else if (t < 0) {
        const unsigned long long off = (unsigned long long)(-(long long)t);
        if (off <= (unsigned long long)(S - 1) * N) end = (unsigned)(S * N - off);
    }
    return end > 2 * N ? end : 2 * N;
}

enum : int { kUnitDead = 0, kUnitEst = 1, kUnitSym = 2 };

// ---------------------------------------------------------------------------
// Certified fast rotation (k_frames symbol units).
//
// The reference rotates sample i of symbol s by the glibc sincosf of
// ph_i = fl(start_s + fl(rate * i)), start_s = rate * (s*N + t_off)
// (LoRaDemod.cpp:152-158, phy.cpp:217-222): one double-precision sincos per
// sample, half of the path's arithmetic.  A symbol's output is only the
// argmax of |FFT|^2, and |FFT(y * e^{j start})| = |FFT(y)|: the common phase
// start_s drops out of every magnitude.  So symbols are transformed as
//     q_i = x_i * t_i,   t_i = [down] * e^{j rate i} * [scale] * [win]
// with t a per-FRAME table (N entries, built once per frame from exact
// sincos of fl(rate*i)), i.e. one complex multiply per sample instead of a
// dechirp, a rescale, a sincos and a rotation.
//
// Exactness is certified per symbol, not assumed.  With u = 2^-24, A an
// upper bound of sum_i |y_i| (the symbol's L1 norm), P = |start| + |rate| N,
// L the number of KISS stages, the reference's bins X and ours X' satisfy
//   | |X_k| - |X'_k| | <= B = u A (24 + 12 L + 2 |rate| N + P) (1 + 1e-3):
//   * rotation inputs: the reference's sample differs from the ideal
//     y_i e^{j(start + rate i)} by <= u(10 + |rate| N + P)|y_i| (dechirp
//     3u, rescale u, sincos sqrt(2)u, phase roundings u(|rate| i + |ph|),
//     rotation 3u, window u); ours from e^{j start}-times-ideal by
//     <= u(10 + |rate| N)|y_i|;
//   * transform: each KISS stage adds <= 6u (sum of its butterfly's input
//     magnitudes) to an output; an output depends on one value of every
//     sub-transform of a level, whose inputs partition the symbol, so both
//     FFTs are within 6 L u A of the exact map (same float twiddles), and
//     the input difference passes with gain (1+u)^L.
// The reference's winner is ours when |X'_best| - 2B > |X'_second| (plus
// the 2u rounding of |X|^2 on both sides and of the check itself); any
// symbol that fails it - ties, near-ties, NaN, overflow risk, frames whose
// time shift is not applied to every symbol - is recomputed with the exact
// per-sample path.  The check below uses 4B (a factor 2 of slack).
// ---------------------------------------------------------------------------

// Fast staging of one tile: symbol units q_i = y_i * t_i from the frame's
// rotation table t (LDS ring for SF <= 8, the lane's registers above) with a
// fused product, where y is the sample, or in mode 2 its exact dechirp at
// its own chirp index (down: the doubled table); estimate units exactly as
// stage_mixed (no rotation).  Returns the lane's max(|Re y|, |Im y|) over its
// symbol samples: mode 0's certificate amplitude, and for modes 1/2 the
// samples' share of the frame's max-abs (speculative normalisation).
//
// The samples are held in first-pass order (element e of lane lam is sample
// fl + first_pass_index<SF>(e, 0), fl = the lane part): the staged values
// stay in registers and the transform starts there (fft_tile REG0).
template <int SF, int MODE, bool MIXED, bool EARLY>
__device__ __forceinline__ float stage_fast(cf32 (&v)[16], cf32 (&raw)[16], const SymCtx& c, int fl,
                                            const cf32* down, const float* win, const cf32* rt,
                                            const cf32* thl, bool est, const cf32* nsrc) {
    using G = Geo<SF>;
    constexpr int N = G::N;
    constexpr bool RLDS = SF <= 8;
    float amax = 0.0f;
    const cf32* dl = down + (c.base & (N - 1)) + fl;  // doubled table: no wrap
    const cf32* rtl = rt + fl;
    const float* wl = win + fl;
    // one branch per tile, not per element (per-element branches serialise
    // the table reads behind their own waits)
    if (MIXED && est) {
#pragma unroll
        for (int e = 0; e < G::E; ++e) {
            const int ce = first_pass_index<SF>(e, 0);
            bound_check((c.base & (N - 1)) + fl + ce, 2 * N);
            cf32 p = raw[e];
            if constexpr (EARLY) raw[e] = ld_iq(nsrc + ce);  // the next tile's sample, as this one is consumed
            if constexpr ((MODE & 3) != LPHY_MODE_DEMODULATE) {
                if constexpr ((MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE) p = cmul(p, dl[ce]);
                p = cscale(p, c.scale);
            }
            cf32 y = c.ok ? p : czero();
            if constexpr ((MODE & kWinBit) != 0) y = cscale(y, wl[ce]);
            v[e] = y;
        }
    } else {
#pragma unroll
        for (int e = 0; e < G::E; ++e) {
            const int ce = first_pass_index<SF>(e, 0);
            bound_check((c.base & (N - 1)) + fl + ce, 2 * N);
            bound_check(fl + ce, N);
            cf32 p = raw[e];
            if constexpr (EARLY) raw[e] = ld_iq(nsrc + ce);
            if constexpr ((MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE) p = cmul(p, dl[ce]);
            amax = max3_abs(amax, p.x, p.y);
            if constexpr (RLDS) {
                v[e] = cmul_fma(p, rtl[ce]);
            } else {
                // SF 9-10: two-table rotation (build_rtab2): thl[0..63] the low
                // part e^{j rate l} [* scale], thl[64..] the high part
                const int i = fl + ce;
                if constexpr ((MODE & 3) == LPHY_MODE_DEMODULATE) p = cmul(p, down[i]);
                cf32 q = cmul_fma(cmul_fma(p, thl[i & 63]), thl[64 + (i >> 6)]);
                if constexpr ((MODE & kWinBit) != 0) q = cscale(q, win[i]);
                v[e] = q;
            }
        }
    }
    return amax;
}

template <int SF, int MODE, int OCC>
__global__ __launch_bounds__(kTile, OCC) void k_frames(FrameArgs P) {
    using G = Geo<SF>;
    static_assert(G::LPS <= 64, "fused path needs a symbol inside one wavefront");
    constexpr int N = G::N;
    constexpr bool TAB = N <= 1024;
    static_assert(TAB, "LDS tables (the doubled down-chirp) for every fused SF");
    constexpr int WT = 64 / G::LPS;               // units per tile
    constexpr unsigned U = 2;                      // estimate units per frame
    // frames per group: the estimate units of F frames fill whole tiles
    // (EBT estimate-only tiles), so no tile mixes estimates with symbols
    constexpr unsigned F = WT >= (int)U ? (unsigned)WT / U : 1u;
    constexpr unsigned EBU = U * F, EBT = (EBU + WT - 1) / WT;
    // prefix tiles: EB(0), then one tile that keeps group 0's symbols two
    // tiles behind it like every later group's
    constexpr unsigned PT = EBT + 1;
    constexpr unsigned NSLOT = 2 * F;  // frame slots: the group in demodulation, the next one
    constexpr int WPB = kTile / 64;
    // rotation tables: per-wave LDS ring of two frames up to SF 8, per-lane
    // registers (built when a team reaches a new frame) for SF 9-10
    constexpr bool RLDS = SF <= 8;
    const DemodArgs& A = P.A;
    __shared__ cf32 lds[G::T * G::SSTRIDE];
    __shared__ cf32 twl[N];
    // down-chirp twice over (entry i = down[i mod N]): a symbol window's
    // chirp indices t0 + i, i < N, need no wrap
    __shared__ cf32 dnl[TAB ? 2 * N : 1];
    __shared__ float wnl[TAB ? N : 1];
    __shared__ UnitResult ures[WPB][F][U];
    __shared__ float4 ring[WPB][NSLOT];  // frame records: rate, scale, t_off, flags
    __shared__ float ringmx[WPB][NSLOT];  // ... and the max-abs their normalisation used
    __shared__ cf32 rtab[RLDS ? WPB : 1][RLDS ? NSLOT : 1][RLDS ? N : 1];
    // SF 9-10: two-table rotation per frame (64 low + N/64 high entries): a
    // whole-symbol table per lane cost 32 VGPRs and spilled
    __shared__ cf32 rtab2[RLDS ? 1 : WPB][RLDS ? 1 : NSLOT][RLDS ? 1 : 64 + N / 64];

    const int tid = threadIdx.x;
    for (int i = tid; i < N; i += kTile) {
        twl[i] = A.tw[i];
        if constexpr (TAB) {
            if ((MODE & 3) != LPHY_MODE_LORA_DEMODULATE) dnl[i] = dnl[i + N] = A.down[i];
            if (A.win) wnl[i] = A.win[i];
        }
    }
    __syncthreads();  // the last workgroup barrier: waves are independent below
    const cf32* down = TAB ? dnl : A.down;
    const float* win = A.win ? (TAB ? wnl : A.win) : nullptr;

    const int lane = tid & 63, wv = tid >> 6;
    const int slot = tid / G::LPS, lam = tid % G::LPS;
    const unsigned wslot = (unsigned)(slot % WT);
    const int fl = first_pass_index<SF>(0, lam);  // lane part of the sample index
    const unsigned nframes = (unsigned)A.frames;
    const unsigned S = (unsigned)A.total_syms;
    const unsigned W = P.waves;
    const unsigned w = blockIdx.x * WPB + wv;
    if (w >= nframes) return;
    const unsigned nk = (nframes - 1 - w) / W + 1;  // frames of this wave
    // group g: D(g) = the F S symbol units of frames gF..gF+F-1 in DBT tiles
    // (the last one padded with dead units), and EB(g+1) = the next group's
    // estimate units in EBT tiles after D(g)'s first PB = DBT - 1 tiles, so
    // that the last EB tile folds two tiles before D(g+1) starts (what the
    // one-tile-ahead context and IQ prefetch need; frames_fit: S >= WT, so
    // DBT >= 2 and the scan ahead of EB(g+1) runs in a D(g) tile)
    const unsigned DBT = (F * S + WT - 1) / WT, GT = DBT + EBT, PB = DBT - 1;
    const unsigned ng = (nk + F - 1) / F;
    const unsigned dt_last = ((nk - (ng - 1) * F) * S + WT - 1) / WT;  // live D tiles of the last group
    const unsigned ntiles = PT + (ng - 1) * GT + (dt_last <= PB ? dt_last : dt_last + EBT);
    auto slot_of = [](unsigned kf) -> unsigned {
        const unsigned sl = ((kf / F) & 1u) * F + kf % F;
        bound_check(sl, NSLOT);
        return sl;
    };
    // no certified outputs: LPHY_F_EXACT_ROTATION, or LPHY_F_DEBUG_RECHECK
    // (tests: every symbol left to k_post's exact re-run)
    const bool exact_only = A.exact_rotation != 0 || A.debug_recheck != 0;
    constexpr bool DECH = (MODE & 3) == LPHY_MODE_DECHIRP_LORA_DEMODULATE;
    // Speculative normalisation (modes 1/2).  The reference scales the whole
    // frame by 1 / max(|I|,|Q|) before it estimates (LoRaDemod.cpp:60-78), so
    // the exact estimate needs every sample first: a blocking pre-scan that
    // re-reads the frame.  Instead M scans only the two estimate symbols, the
    // frame is estimated and demodulated with that normalisation, and each
    // symbol unit folds its own samples' max-abs while they are in registers.
    // When the symbol that ends the frame is done, the frame's true max-abs
    // is known: the same normalisation means every output stands; otherwise
    // the frame goes to k_post's settle_frames (exact estimate, certificates
    // re-checked against the exact rate, else the whole-frame re-run).
    const bool spec = (MODE & 3) != LPHY_MODE_DEMODULATE && A.spec != 0;
    constexpr bool EARLY = (MODE & 3) == LPHY_MODE_DEMODULATE && (SF == 7 || SF == 8);

    // unit of this team in tile t; for t >= PT: group g, tile tg of the
    // group, and the team's symbol unit (frame dj of the group, symbol ds)
    // when tg is a D tile
    auto unit_of = [&](unsigned t, unsigned g, unsigned tg, unsigned dj, unsigned ds, unsigned& kind,
                       unsigned& fk, unsigned& s) {
        if (t < PT) {
            const unsigned q = t * WT + wslot;
            const bool e = t < EBT && q < EBU;
            fk = e ? q / U : 0u;
            s = e ? q % U : 0u;
            kind = e && fk < nk ? kUnitEst : kUnitDead;
        } else if (tg >= PB && tg < PB + EBT) {
            const unsigned q = (tg - PB) * WT + wslot;
            fk = (g + 1) * F + q / U;
            s = q % U;
            kind = q < EBU && fk < nk ? kUnitEst : kUnitDead;
        } else {
            fk = g * F + dj;
            s = ds;
            kind = dj < F && fk < nk ? kUnitSym : kUnitDead;
        }
    };
    // context of a unit; symbol units read their frame record from the ring
    auto ctx_of = [&](unsigned kind, unsigned fk, unsigned s) -> SymCtx {
        const unsigned f = w + fk * W;
        if (kind == kUnitSym) {
            const float4 r = ring[wv][slot_of(fk)];
            lphy_frame_meta m{};
            m.rate = r.x;
            m.scale = r.y;
            m.t_off = __float_as_int(r.z);
            const unsigned fl = __float_as_uint(r.w);
            m.status = (fl & 1u) ? 0 : -1;
            m.have_sync = (fl & 2u) ? 1 : 0;
            return sym_ctx(A, f, s, true, N, m);
        }
        SymCtx c{};
        c.f = kind == kUnitEst ? f : w;
        c.s = s;
        c.base = kind == kUnitEst ? s * N : 0;
        c.scale = 1.0f;
        c.live = kind == kUnitEst;
        return c;
    };

    unsigned g = 0, tg = 0, dj = 0, ds = wslot;  // position of tile t (t >= PT)
    unsigned kind, fk, su;
    unit_of(0, g, tg, dj, ds, kind, fk, su);
    SymCtx c = ctx_of(kind, fk, su);
    // M (modes 1/2): the max-abs scans of a group's frames run in the tile
    // before its first EB tile, between that tile's staging and its IQ
    // prefetch, when no tile data is held in registers; tile 0 holds EB(0),
    // scanned here.  Each frame's maximum goes to its slot of ringmx.
    // (Measured alternative, 1.4x slower at SF7: the scan streamed one
    // chunk per tile through a per-wave LDS buffer by LDS-DMA, issued after
    // staging and folded a tile later.)
    unsigned m_seq = 0xffffffffu;  // group whose frames are scanned
    // Under speculation (modes 1/2 with scratch) the EB tile takes its
    // frames' two-symbol max-abs from its own staged samples instead
    // (EST_MAX below), so the scans run only for the pre-scan schedule.
    // That needs both estimate units of a frame in one tile (teams 2j and
    // 2j + 1): 2 LPS <= 64 lanes, i.e. SF <= 9.  At SF 10 a team is the
    // whole wave (EBT = 2 tiles per frame), so the scans stay.
#ifdef LPHY_AB_EB_SCAN  // A/B timing only: the round-2 scans under speculation too
    constexpr bool kEbMax = false;
#else
    constexpr bool kEbMax = 2 * G::LPS <= 64;
#endif
    auto scan_ahead = [&](unsigned nkind_, unsigned nfk_) {
        if constexpr ((MODE & 3) != LPHY_MODE_DEMODULATE) {
            if (kEbMax && spec) return;
            const unsigned long long nem = __ballot(nkind_ == kUnitEst);
            if (nem) {
                const unsigned grp = (unsigned)__shfl((int)nfk_, __ffsll((long long)nem) - 1, 64) / F;
                if (grp != m_seq) {
                    for (unsigned j = 0; j < F && grp * F + j < nk; ++j) {
                        const unsigned kk = grp * F + j;
#ifdef LPHY_ABLATE_FRAME_SCAN  // timing experiments only
                        const float m = 1.0f;
#else
                        const float m = wave_maxabs<SF, MODE>(A, w + kk * W, down, spec ? 2u * N : 0u);
#endif
                        if (lane == 0) ringmx[wv][slot_of(kk)] = m;
                    }
                    m_seq = grp;
                }
            }
        }
    };
    scan_ahead(kind, fk);
    cf32 raw[16];  // the next unit's samples, first-pass order
    {
        const cf32* src = A.iq + (unsigned long long)c.f * A.frame_samples + c.base + fl;
#pragma unroll
        for (int e = 0; e < G::E; ++e) {
            iq_check(A, c.f, (long long)c.base + fl + first_pass_index<SF>(e, 0));
            raw[e] = ld_iq(src + first_pass_index<SF>(e, 0));
        }
    }
    // speculative normalisation: the lane's running state for the two frames
    // whose symbols can be in flight (by parity of the frame): max-abs of the
    // symbol samples, least certificate ratio, flags (1 NaN, 2 symbol open)
    constexpr float kBig = 3.0e38f;
    float sp_mx0 = 0.0f, sp_mx1 = 0.0f, sp_r0 = kBig, sp_r1 = kBig;
    unsigned sp_fl0 = 0u, sp_fl1 = 0u;
#ifdef LPHY_PROFILE_PHASES  // timing experiments only: mixed / symbol-only tile clocks
    unsigned long long ph_mix = 0, ph_sym = 0, ph_fold = 0, n_mix = 0;
#endif

    for (unsigned t = 0; t < ntiles; ++t) {
#ifdef LPHY_PROFILE_PHASES
        const unsigned long long p0 = clock64();
        unsigned long long pf = 0;
#endif
        cf32 v[16];  // this tile's unit: staged samples, then its bins
        const cf32* rt = rtab[RLDS ? wv : 0][RLDS ? slot_of(fk) : 0];
        const cf32* thl = rtab2[RLDS ? 0 : wv][RLDS ? 0 : slot_of(fk)];
        // next tile's unit and context
        unsigned ng_ = g, ntg = tg, ndj = dj, nds = ds;
        unsigned nkind, nfk, nsu;
        SymCtx nc;
        auto next_pos = [&] {
            if (t + 1 == PT) {
                ng_ = 0; ntg = 0; ndj = 0; nds = wslot;
            } else if (t + 1 > PT) {
                if (tg < PB || tg >= PB + EBT) {  // tile t was a D tile
                    nds += WT;
                    if (nds >= S) { nds -= S; ++ndj; }
                }
                if (++ntg == GT) { ntg = 0; ++ng_; ndj = 0; nds = wslot; }
            }
            unit_of(t + 1, ng_, ntg, ndj, nds, nkind, nfk, nsu);
        };
        auto next_ctx = [&] {
            if (t + 1 < ntiles) scan_ahead(nkind, nfk);
            nc = ctx_of(nkind, nfk, nsu);
        };
        // EARLY (mode 0 at SF 7-8, measured): the next tile's IQ is loaded as
        // this tile's staging consumes the registers, so it is in flight
        // during staging and the FFT.  (Mode 2: 13 % slower at SF7, mode 0
        // at SF9: 6 % slower.)  The last tile reloads a valid window: a
        // dead unit's is frame w's first.
        const cf32* nsrc = nullptr;
        next_pos();
        // (measured alternative: early in modes 1/2 too, except in the tile
        // before an EB tile, whose scans need the registers: 4-5x slower,
        // the two staging variants of one loop spilled)
        constexpr bool early = EARLY;
        if (early) {
            next_ctx();
            nsrc = A.iq + (unsigned long long)nc.f * A.frame_samples + nc.base + fl;
            iq_check(A, nc.f, (long long)nc.base);
            iq_check(A, nc.f, (long long)nc.base + N - 1);
        }
        // an EB tile (estimate units of one group, and dead units): each
        // unit's frame max-abs, scanned ahead, first
        const unsigned long long emask = __ballot(kind == kUnitEst);
        float amax;
        if (kEbMax && spec && emask) {
            // EST_MAX: an EB tile holds both estimate units of each of its
            // frames, in teams 2j and 2j + 1 (2 LPS lanes).  The samples are
            // staged [dechirped], the frame's max(|I|,|Q|) over them folded
            // (v_max3, and NaN when one is non-finite, like wave_maxabs: such
            // a frame goes to k_post's exact re-run), then the normalisation
            // applied: the same operations on the same operands as staging
            // with the scanned maximum, without reading the two symbols
            // twice or blocking on a scan.  (Modes 1/2 only, so never with
            // EARLY, the mode-0 in-staging reload of `raw`, which this
            // staging does not do.)
            static_assert(!EARLY || (MODE & 3) == LPHY_MODE_DEMODULATE, "EST_MAX staging has no EARLY reload");
            const cf32* dl = down + (c.base & (N - 1)) + fl;
            float fm = 0.0f;
            cf32 sum = czero();
#pragma unroll
            for (int e = 0; e < G::E; ++e) {
                const int ce = first_pass_index<SF>(e, 0);
                cf32 p = raw[e];
                if constexpr (DECH) p = cmul(p, dl[ce]);
                fm = max3_abs(fm, p.x, p.y);
                sum = sum + p;
                v[e] = p;
            }
            bool bad = !(sum.x == sum.x && sum.y == sum.y) || !(fm <= 3.40282347e38f);
#pragma unroll
            for (int off = G::LPS; off >= 1; off >>= 1) {
                const float o = __shfl_xor(fm, off, 64);
                fm = o > fm ? o : fm;
            }
            const unsigned long long bm = __ballot(bad);
            const unsigned pair = (unsigned)(lane / (2 * G::LPS));
            constexpr unsigned long long PM = 2 * G::LPS >= 64 ? ~0ull : ((1ull << (2 * G::LPS)) - 1ull);
            bad = ((bm >> (pair * 2 * G::LPS)) & PM) != 0;
            const float mx = bad ? __builtin_nanf("") : fm;
            if (kind == kUnitEst) {
                const lphy_frame_meta nm = norm_meta_hot(mx, true, A.no_scratch);
                c.scale = nm.scale;
                c.live = nm.status == 0;
                if (su == 0 && lam == 0) ringmx[wv][slot_of(fk)] = mx;
            }
            c.ok = kind == kUnitEst && c.live;
            const float* wl = win + fl;
#pragma unroll
            for (int e = 0; e < G::E; ++e) {
                cf32 y = c.ok ? cscale(v[e], c.scale) : czero();
                if constexpr ((MODE & kWinBit) != 0) y = cscale(y, wl[first_pass_index<SF>(e, 0)]);
                v[e] = y;
            }
            amax = 0.0f;
        } else if (emask) {
            if (kind == kUnitEst) {
                if ((MODE & 3) != LPHY_MODE_DEMODULATE) {
                    const lphy_frame_meta nm = norm_meta_hot(ringmx[wv][slot_of(fk)], true, A.no_scratch);
                    c.scale = nm.scale;
                    c.live = nm.status == 0;
                }
                c.ok = c.live;  // estimate this unit (else stage zeros)
            }
            amax = early ? stage_fast<SF, MODE, true, true>(v, raw, c, fl, down, win, rt, thl, kind != kUnitSym, nsrc)
                         : stage_fast<SF, MODE, true, false>(v, raw, c, fl, down, win, rt, thl, kind != kUnitSym, nsrc);
        } else {
            amax = early ? stage_fast<SF, MODE, false, true>(v, raw, c, fl, down, win, rt, thl, false, nsrc)
                         : stage_fast<SF, MODE, false, false>(v, raw, c, fl, down, win, rt, thl, false, nsrc);
        }
        if constexpr ((MODE & 3) == LPHY_MODE_DEMODULATE) {
            if constexpr (G::LPS <= 16) {
                amax = team_max_first<SF>(amax);  // the certificate reads lane lam == 0
            } else {
#pragma unroll
                for (int off = G::LPS / 2; off >= 1; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 64));
            }
        } else {
            // normalised frame: max(|I|,|Q|) <= 1 (see fast_certified); under
            // speculation the frame end confirms it or settles the frame
            if (spec) {
                // the symbol's [dechirped] samples, as the pre-scan folds them
                const float lm = kind == kUnitSym && c.ok ? amax : 0.0f;
                if (fk & 1) sp_mx1 = fmaxf(sp_mx1, lm);
                else sp_mx0 = fmaxf(sp_mx0, lm);
            }
            amax = 1.0f;
        }
        team_sync<SF>();

        if (!early) {
            // next tile's context and IQ (in flight during the FFT)
            next_ctx();
            if (t + 1 < ntiles) {
                const cf32* lsrc = A.iq + (unsigned long long)nc.f * A.frame_samples + nc.base + fl;
#pragma unroll
                for (int e = 0; e < G::E; ++e) {
                    iq_check(A, nc.f, (long long)nc.base + fl + first_pass_index<SF>(e, 0));
                    raw[e] = ld_iq(lsrc + first_pass_index<SF>(e, 0));
                }
            }
        }

        // tiles of symbol units only: magnitude-only transform (fft_tile TRIV)
        // (measured alternative: a packed-key max/min tournament for the top
        // two, 3 % slower than this ordered scan)
        // the transform and the top two at issue priority 1: of the two
        // waves on a SIMD, the one in its arithmetic segment issues first
        // (the other is mostly in staging, bookkeeping or waiting on loads),
        // so each wave's compute segment ends, and its next loads go out,
        // sooner.  Same-box A/B: fused 1.037 -> 1.016 ms (three rounds;
        // priority over the transform alone: 1.021)
#ifndef LPHY_AB_NO_PRIO  // A/B timing only
        __builtin_amdgcn_s_setprio(1);
#endif
        if (emask) fft_tile<SF, false, false, true>(v, lds, slot, lam, twl);
        else fft_tile<SF, true, false, true>(v, lds, slot, lam, twl);

        // (SF <= 8: reduced toward lane lam == 0 by DPP, the only lane that
        // reads it; above, every lane of the team holds it)
        // (symbol-only tiles: keyed top two, a bound that only certified
        // symbols use; estimate units need the detector's exact argmax)
        ArgMax2 b2;
        if constexpr (G::LPS <= 16) {
#ifdef LPHY_EXACT_TOP2  // A/B experiments: the exact top two everywhere
            b2 = team_argmax2_first<SF>(local_argmax2<SF>(v, lam));
#else
            if (emask) b2 = team_argmax2_first<SF>(local_argmax2<SF>(v, lam));
            else b2 = team_argmax2_keyed_first<SF>(v, lam);
#endif
        } else {
            b2 = symbol_argmax2<SF>(local_argmax2<SF>(v, lam));
        }
#ifndef LPHY_AB_NO_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
        ArgMax best{b2.v, b2.i};
        if (emask) {
            // detector outputs of the estimate units (LoRaDetector.hpp:60-71)
            if (kind == kUnitEst) {
#pragma unroll
                for (int e = 0; e < G::E; ++e) lds[G::addr(slot, bin_of<SF>(e, lam))] = v[e];
            }
            team_sync<SF>();
            // a NaN bin may hide an Annex G product: exact re-run (k_post)
            const unsigned long long nanm = __ballot(kind == kUnitEst && c.ok && fft_has_nan<SF>(v));
            if (kind == kUnitEst && lam == 0) {
                UnitResult& ur = ures[wv][fk % F][su];
                ur = c.ok ? unit_result<SF>(lds, slot, best) : UnitResult{0, 0, 0.0f, 0.0f};
                ur.nan = ((nanm >> (slot * G::LPS)) & ((G::LPS == 64) ? ~0ull : ((1ull << G::LPS) - 1))) != 0;
            }
            team_sync<SF>();  // slot reads done before a re-check restages
        }
        // symbols the certificate does not cover: exact per-sample rotation
        // certificate (fast_certified, written out so that the speculation
        // below reuses its lead and bound): B is linear in amax
        const float cb1 = cert_bound<SF>(c.rate, c.start, 1.0f, RLDS ? 0.0f : 6.0f);
        const float cgap = cert_gap(b2);
        const bool cert = cgap > 4.0f * (cb1 * amax) && (float)N * 1.41421366f * amax * 1.0001f < 1e18f &&
                          amax >= 1e-20f && b2.v >= 1e-30f && b2.v < 1e30f;
        const bool redo = kind == kUnitSym && c.ok &&
                          (exact_only || !fast_applies<SF, MODE>(c, c.toff) || !cert);
        // (no exact re-run here: it would keep a second transform's state
        // live beside the prefetch.  The symbol is left as kSymRecheck and
        // its frame as kStatusRecheck; k_post recomputes it exactly.)
        if (spec && kind == kUnitSym && c.ok) {
            // a NaN sample reaches every bin (fft_has_nan); the certificate's
            // lead over its bound, for the frame end's rate check (from the
            // team's first lane, which holds the team's top two)
            const cf32 q = v[0] * v[0];
            const float q2 = q.x + q.y;
            unsigned fl = q2 == q2 ? 0u : 1u;
            float r = kBig;
            if (lam == 0) {
                // a lower bound of the lead / bound ratio (v_rcp within 1 ulp)
                if (redo) fl |= 2u;
                else r = cgap * __builtin_amdgcn_rcpf(cb1) * (1.0f - 4.0f * kU);
            }
            if (fk & 1) {
                sp_fl1 |= fl;
                sp_r1 = fminf(sp_r1, r);
            } else {
                sp_fl0 |= fl;
                sp_r0 = fminf(sp_r0, r);
            }
        }
        if (kind == kUnitSym && lam == 0) {
            // sw0 / sw1 also for frames that are not demodulated (0, as the
            // separate-launch path leaves them)
            const uint16_t out = redo ? kSymRecheck : (uint16_t)best.i;
            if (c.have_sync && c.s < 2) store_symbol(A, c, c.ok ? out : (uint16_t)0);
            else if (c.ok) store_symbol(A, c, out);
            if (redo) A.meta[c.f].status = kStatusRecheck;
        }
        team_sync<SF>();  // slot reads (and ures) done
#ifdef LPHY_PROFILE_PHASES
        pf = clock64();
#endif
        // the frames whose last estimate unit was in this tile: each folds on
        // the first lane of the team holding that unit (F lanes at once)
        const bool my_fold = kind == kUnitEst && su == U - 1 && lam == 0;
        const unsigned long long fmask = __ballot(my_fold);
        if (my_fold) {
            const unsigned sl = slot_of(fk);
            lphy_frame_meta m{};
            m.scale = 1.0f;
            m.have_sync = 1;
            if ((MODE & 3) != LPHY_MODE_DEMODULATE) m = norm_meta_hot(ringmx[wv][sl], true, A.no_scratch);
            if (m.status == 0) {
                EstFold fold;
                bool nan = false;
#pragma unroll
                for (unsigned u = 0; u < U; ++u) {
                    const UnitResult r = ures[wv][fk % F][u];
                    nan |= r.nan != 0;
                    if (r.valid) fold.add(r.idx, r.findex, 0, r.phase);
                    else fold.add(0, 0.0f, 0, 0.0f);
                }
                fold.finish(m, (int)U, N, 1);
                if (nan) m.status = kStatusFixup;
            }
            ring[wv][sl] = float4{m.rate, m.scale, __int_as_float(m.t_off),
                                  __uint_as_float((m.status == 0 ? 1u : 0u) | 2u)};
            bound_check(w + fk * W, (long long)A.frames);
            meta_put_est(&A.meta[w + fk * W], m);
        }
        team_sync<SF>();
        // the folded frames' rotation tables, first read two tiles later
        // (their slots' previous frames, of group g - 1, have no units left)
        for (unsigned long long fm = fmask; fm; fm &= fm - 1) {
            const unsigned kf = (unsigned)__shfl((int)fk, __ffsll((long long)fm) - 1, 64);
            const unsigned sl = slot_of(kf);
            const float4 r = ring[wv][sl];
            if (__float_as_uint(r.w) & 1u) {
                if constexpr (RLDS) {
                    build_rtab<SF, MODE>(rtab[wv][sl], r.x, r.y, __float_as_int(r.z), down, win, lane);
                } else {
                    cf32* tb = rtab2[wv][sl];
                    for (int j = lane; j < 64 + N / 64; j += 64) {
                        const int ph = j < 64 ? j : 64 * (j - 64);
                        float sn, cs;
                        lphy_libm::sincosf_exact(r.x * (float)ph, &sn, &cs);
                        cf32 t = cf32{cs, sn};
                        if constexpr ((MODE & 3) != LPHY_MODE_DEMODULATE)
                            if (j < 64) t = cscale(t, r.y);
                        tb[j] = t;
                    }
                }
            }
        }
        // speculative normalisation: the tile holding a frame's last symbol
        // unit closes the frame (its other symbols are in earlier tiles)
        if (spec) {
            const unsigned long long fe = __ballot(kind == kUnitSym && su == S - 1);
            if (fe) {
                const unsigned kf = (unsigned)__shfl((int)fk, __ffsll((long long)fe) - 1, 64);
                const bool p1 = (kf & 1) != 0;
                float m = p1 ? sp_mx1 : sp_mx0, r = p1 ? sp_r1 : sp_r0;
                const unsigned fl = p1 ? sp_fl1 : sp_fl0;
                if (p1) { sp_mx1 = 0.0f; sp_r1 = kBig; sp_fl1 = 0u; }
                else { sp_mx0 = 0.0f; sp_r0 = kBig; sp_fl0 = 0u; }
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    m = fmaxf(m, __shfl_xor(m, off, 64));
                    r = fminf(r, __shfl_xor(r, off, 64));
                }
                const bool nan = __ballot(fl & 1u) != 0, open = __ballot(fl & 2u) != 0;
                const float4 rr = ring[wv][slot_of(kf)];
                if (__float_as_uint(rr.w) & 1u) {
                    const unsigned f = w + kf * W;
                    bound_check(f, (long long)A.frames);
                    const unsigned cnt = DECH ? S * N : (unsigned)A.frame_samples;
                    const unsigned end = covered_end(S, N, cnt, __float_as_int(rr.z));
                    bool fbad = false;
                    if (end < cnt) m = fmaxf(m, wave_range_maxabs<SF, MODE>(A, f, end, cnt, down, fbad));
                    if (lane == 0) {
                        const float mx01 = ringmx[wv][slot_of(kf)];
                        const float mt = fmaxf(m, mx01);
                        const lphy_frame_meta mg = norm_meta(mx01, true, 0), me = norm_meta(mt, true, 0);
                        if (nan || fbad || !(mt <= 3.40282347e38f)) {
                            A.meta[f].status = kStatusFixup;
                        } else if (me.scale != mg.scale || me.normalised != mg.normalised) {
                            A.meta[f].cfo = mt;
                            A.meta[f].time_offset = r;
                            A.meta[f].status = open ? kStatusSettleRecheck : kStatusSettle;
                        }
                    }
                }
            }
        }
        g = ng_;
        tg = ntg;
        dj = ndj;
        ds = nds;
        kind = nkind;
        fk = nfk;
        su = nsu;
        c = nc;
#ifdef LPHY_PROFILE_PHASES
        const unsigned long long p9 = clock64();
        if (emask) { ph_mix += p9 - p0; ph_fold += p9 - pf; ++n_mix; }
        else ph_sym += p9 - p0;
#endif
    }
#ifdef LPHY_PROFILE_PHASES
    if (lane == 0) {
        atomicAdd(&A.counters[kCtrClocks + 0], ph_mix);
        atomicAdd(&A.counters[kCtrClocks + 1], ph_sym);
        atomicAdd(&A.counters[kCtrClocks + 2], ph_fold);
        atomicAdd(&A.counters[kCtrClocks + 3], n_mix);
    }
#endif
}

// ---------------------------------------------------------------------------
// Per-frame finalisation: sync word, decode, CRC
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint8_t hamming84_decode(uint8_t b) {
    // LoRaCodes.hpp:250-281 (decodeHamming84sx): syndrome bits are the
    // parities of b & 0x17, 0x2E, 0x4B, 0x8D (b0^b1^b2^b4, b1^b2^b3^b5,
    // b0^b1^b3^b6, b0^b2^b3^b7); syndromes 0xD / 0x7 / 0xB / 0xE flip data
    // bit 0 / 1 / 2 / 3, read from a nibble table (all 256 inputs checked
    // against the switch form on the host)
    const unsigned x = b;
    const unsigned syn = (__builtin_popcount(x & 0x17u) & 1u) | ((__builtin_popcount(x & 0x2Eu) & 1u) << 1) |
                         ((__builtin_popcount(x & 0x4Bu) & 1u) << 2) | ((__builtin_popcount(x & 0x8Du) & 1u) << 3);
    constexpr unsigned long long kFlip = (1ull << 52) | (2ull << 28) | (4ull << 44) | (8ull << 56);
    return (uint8_t)((x ^ (unsigned)(kFlip >> (4 * syn))) & 0xfu);
}

// LoRaCodes.hpp:69-105
// The reference shifts the register 8 times through poly 0x1021 with a
// zero input bit per byte; that equals the byte-wise CCITT step with a
// zero input byte below (all 65,536 registers checked on the host), and
// the whitening register's feedback is the parity of v & 0xB8.
__device__ __forceinline__ unsigned sx_shift8(unsigned c) {
    unsigned x = c >> 8;
    x ^= x >> 4;
    return ((c << 8) ^ (x << 12) ^ (x << 5) ^ x) & 0xffffu;
}
__device__ __forceinline__ unsigned sx_lfsr(unsigned v) {
    return ((__builtin_popcount(v & 0xB8u) & 1u) | (v << 1)) & 0xffu;
}
__device__ __forceinline__ uint16_t sx1272_checksum(const uint8_t* data, int len) {
    auto shift8 = [](unsigned c) -> unsigned { return sx_shift8(c); };
    auto lfsr = [](unsigned v) -> unsigned { return sx_lfsr(v); };
    unsigned res = 0, v = 0xff;
    for (int i = 0; i < len; ++i) {
        const unsigned crc = shift8(res);
        v = lfsr(v);
        res = crc ^ data[i];
    }
    res ^= v;
    v = lfsr(v);
    res ^= v << 8;
    return (uint16_t)res;
}



// Register form of the finalisation for rows of up to 64 symbols (32
// bytes) that are 16-byte aligned with 4-aligned output: the record and all
// the symbols are loaded before the status test (one memory round trip, not
// two), and the checksum runs over the decoded words held in registers
// instead of re-reading the bytes just stored (a third round trip and 28
// byte loads per frame).  Same bytes, same checksum steps as below.
__device__ __forceinline__ bool finalize_frame_regs(const FinalArgs& A, unsigned long long f) {
    const unsigned long long nb = A.nsyms / 2;
    const uint16_t* s = A.syms + f * A.sym_stride;
    uint8_t* out = A.bytes + f * nb;
    if (!A.decode || (A.nsyms & 1) || nb > 32 || (nb & 3) || (reinterpret_cast<uintptr_t>(s) & 15) ||
        (reinterpret_cast<uintptr_t>(out) & 3))
        return false;
    const unsigned nw = (unsigned)(nb / 4);  // wave-uniform
    const uint4* s4 = reinterpret_cast<const uint4*>(s);
    uint4 q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if ((unsigned)j < nw) q[j] = s4[j];
    lphy_frame_meta m = A.meta[f];
    if (m.status != 0) return true;
    if (A.set_sync && m.have_sync)
        m.sync_word = (uint8_t)((((m.sw0 >> A.shift) & 0x0f) << 4) | ((m.sw1 >> A.shift) & 0x0f));
    unsigned wd[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        wd[j] = 0u;
        if ((unsigned)j < nw) {
            const unsigned qs[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const unsigned hi = hamming84_decode((uint8_t)qs[b]) & 0x0fu;
                const unsigned lo = hamming84_decode((uint8_t)(qs[b] >> 16)) & 0x0fu;
                wd[j] |= ((hi << 4) | lo) << (8 * b);
            }
            *reinterpret_cast<unsigned*>(out + 4 * j) = wd[j];
        }
    }
    if (nb >= 4) {  // phy.cpp:252-259, over bytes 2 .. nb-3
        const int len = (int)nb - 4;
        unsigned res = 0, v = 0xff;
#pragma unroll
        for (int i = 0; i < 28; ++i) {
            if (i >= len) break;  // wave-uniform
            const unsigned byte = (wd[(i + 2) >> 2] >> (8 * ((i + 2) & 3))) & 0xffu;
            const unsigned crc = sx_shift8(res);
            v = sx_lfsr(v);
            res = crc ^ byte;
        }
        res ^= v;
        v = sx_lfsr(v);
        res ^= v << 8;
        const unsigned pw = wd[(nb - 2) >> 2] >> (8 * ((nb - 2) & 3));  // bytes nb-2, nb-1 (same word)
        m.crc_ok = (uint16_t)(pw & 0xffffu) == (uint16_t)res;
    } else {
        m.crc_ok = 0;
    }
    A.meta[f] = m;
    return true;
}

__device__ __forceinline__ void finalize_frame(const FinalArgs& A, unsigned long long f) {
#ifndef LPHY_AB_FINAL_MEM  // A/B timing only: the memory form for every row
    if (finalize_frame_regs(A, f)) return;
#endif
    lphy_frame_meta m = A.meta[f];
    if (m.status != 0) return;
    if (A.set_sync && m.have_sync)
        m.sync_word = (uint8_t)((((m.sw0 >> A.shift) & 0x0f) << 4) | ((m.sw1 >> A.shift) & 0x0f));
    if (A.decode) {
        if (A.nsyms & 1) {
            m.status = -EINVAL;  // LoRaDecoder.cpp:10
        } else {
            const unsigned long long nb = A.nsyms / 2;
            const uint16_t* s = A.syms + f * A.sym_stride;
            uint8_t* out = A.bytes + f * nb;
            unsigned long long k0 = 0;
            // 8 symbols per 16-byte load and 4 bytes per store where aligned
            // (the bench rows: 64 symbols in, 32 bytes out)
            if ((reinterpret_cast<uintptr_t>(s) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 3) == 0) {
                const uint4* s4 = reinterpret_cast<const uint4*>(s);
                for (; k0 + 4 <= nb; k0 += 4) {
                    const uint4 q = s4[k0 / 4];
                    const unsigned qs[4] = {q.x, q.y, q.z, q.w};
                    unsigned wd = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const unsigned hi = hamming84_decode((uint8_t)qs[j]) & 0x0fu;
                        const unsigned lo = hamming84_decode((uint8_t)(qs[j] >> 16)) & 0x0fu;
                        wd |= ((hi << 4) | lo) << (8 * j);
                    }
                    *reinterpret_cast<unsigned*>(out + k0) = wd;
                }
            }
            for (unsigned long long k = k0; k < nb; ++k) {
                const uint8_t hi = hamming84_decode((uint8_t)s[2 * k]) & 0x0f;
                const uint8_t lo = hamming84_decode((uint8_t)s[2 * k + 1]) & 0x0f;
                out[k] = (uint8_t)((hi << 4) | lo);
            }
            if (nb >= 4) {  // phy.cpp:252-259
                const uint16_t provided = (uint16_t)(out[nb - 2] | (out[nb - 1] << 8));
                m.crc_ok = provided == sx1272_checksum(out + 2, (int)(nb - 4));
            } else {
                m.crc_ok = 0;
            }
        }
    }
    A.meta[f] = m;
}

// A workgroup's 256 rows at once (the register form's rows: 8 to 64
// symbols, a multiple of 8, 16-byte aligned): the symbols come in and the
// bytes go out as whole contiguous rows across the workgroup, staged in LDS,
// instead of each thread's 128-byte row at a 128-byte lane stride; each
// thread then decodes its frame as finalize_frame_regs does (same bytes,
// same checksum steps).  Rows of a non-zero status are left as they are.
struct FinStage {
    uint4 in[kTile * 9];      // 9 x 16 B per row (8 used): conflict-free 16-byte reads
    unsigned out[kTile * 9];  // the decoded words
    unsigned char ok[kTile];  // the row was decoded
};
__device__ __forceinline__ bool finalize_block(const FinalArgs& A, unsigned long long f0, FinStage& st) {
    const unsigned long long nb = A.nsyms / 2;
    if (!A.decode || (A.nsyms & 1) || nb < 4 || nb > 32 || (nb & 3) || (A.sym_stride & 7) ||
        (reinterpret_cast<uintptr_t>(A.syms) & 15) || (reinterpret_cast<uintptr_t>(A.bytes) & 3) ||
        f0 >= A.frames)
        return false;  // (uniform over the workgroup)
    const unsigned nw = (unsigned)(nb / 4);
    const unsigned nf = A.frames - f0 < (unsigned long long)kTile ? (unsigned)(A.frames - f0) : (unsigned)kTile;
    const unsigned t = threadIdx.x;
    for (unsigned i = t; i < nf * nw; i += kTile) {
        const unsigned fr = i / nw, k = i - fr * nw;
        st.in[fr * 9 + k] = reinterpret_cast<const uint4*>(A.syms + (f0 + fr) * A.sym_stride)[k];
    }
    __syncthreads();
    if (t < nf) {
        const unsigned long long f = f0 + t;
        lphy_frame_meta m = A.meta[f];
        const bool ok = m.status == 0;
        st.ok[t] = ok ? 1 : 0;
        if (ok) {
            if (A.set_sync && m.have_sync)
                m.sync_word = (uint8_t)((((m.sw0 >> A.shift) & 0x0f) << 4) | ((m.sw1 >> A.shift) & 0x0f));
            unsigned wd[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                wd[j] = 0u;
                if ((unsigned)j < nw) {
                    const uint4 q = st.in[t * 9 + j];
                    const unsigned qs[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const unsigned hi = hamming84_decode((uint8_t)qs[b]) & 0x0fu;
                        const unsigned lo = hamming84_decode((uint8_t)(qs[b] >> 16)) & 0x0fu;
                        wd[j] |= ((hi << 4) | lo) << (8 * b);
                    }
                    st.out[t * 9 + j] = wd[j];
                }
            }
            // phy.cpp:252-259, over bytes 2 .. nb-3 (finalize_frame_regs)
            const int len = (int)nb - 4;
            unsigned res = 0, v = 0xff;
#pragma unroll
            for (int i = 0; i < 28; ++i) {
                if (i >= len) break;  // uniform
                const unsigned byte = (wd[(i + 2) >> 2] >> (8 * ((i + 2) & 3))) & 0xffu;
                const unsigned crc = sx_shift8(res);
                v = sx_lfsr(v);
                res = crc ^ byte;
            }
            res ^= v;
            v = sx_lfsr(v);
            res ^= v << 8;
            const unsigned pw = st.out[t * 9 + (unsigned)((nb - 2) >> 2)] >> (8 * ((nb - 2) & 3));
            m.crc_ok = (uint16_t)(pw & 0xffffu) == (uint16_t)res;
            A.meta[f] = m;
        }
    }
    __syncthreads();
    for (unsigned i = t; i < nf * nw; i += kTile) {
        const unsigned fr = i / nw, k = i - fr * nw;
        if (st.ok[fr]) reinterpret_cast<unsigned*>(A.bytes + (f0 + fr) * nb)[k] = st.out[fr * 9 + k];
    }
    return true;
}

__global__ __launch_bounds__(kTile) void k_finalize(FinalArgs A) {
    __shared__ FinStage st;
#ifndef LPHY_AB_FINAL_THREAD  // A/B timing only: a row per thread straight from memory
    if (blockDim.x == kTile && finalize_block(A, (unsigned long long)blockIdx.x * kTile, st)) return;
#endif
    const unsigned long long f = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (f < A.frames) finalize_frame(A, f);
}

// ---------------------------------------------------------------------------
// Exact re-run of one frame by a whole 256-thread workgroup (k_post): the
// reference's arithmetic with its Annex G complex products (cmul_x)
// everywhere - max-abs (LoRaDemod.cpp:60-78), estimate (LoRaDemod.cpp:80-140
// / phy.cpp:81-148), every symbol (LoRaDemod.cpp:142-176 / phy.cpp:204-238).
// Frames get here only when a hot kernel met a non-finite value (status
// kStatusFixup), so this path favours plainness over speed.
// ---------------------------------------------------------------------------
template <int SF>
struct PostShared {
    cf32 lds[Geo<SF>::T * Geo<SF>::SSTRIDE];
    ArgMax red[kTile / 64];
    UnitResult units[Geo<SF>::T];
    float upow[Geo<SF>::T];
    float wmax[kTile / 64];
    lphy_frame_meta m;
    uint16_t sw[2];
    unsigned list[kTile];
    unsigned listf[kTile];
    unsigned count;
    UnitResult ures2[kTile][2];  // settle_frames: both estimate units of each frame
};

template <int SF, int MODE>
__device__ void exact_frame(const DemodArgs& A, unsigned f, PostShared<SF>& sh) {
    using G = Geo<SF>;
    constexpr int N = G::N, T = G::T;
    const int tid = threadIdx.x;
    const int slot = tid / G::LPS, lam = tid % G::LPS;
    const cf32* fr = A.iq + (unsigned long long)f * A.frame_samples;
    const unsigned long long step = (unsigned long long)N * A.osr;
    const bool have_sync = A.total_syms >= 2;
    // (1) normalisation (modes 1, 2)
    if (MODE != LPHY_MODE_DEMODULATE) {
        const unsigned long long count = MODE == LPHY_MODE_DECHIRP_LORA_DEMODULATE
                                             ? A.total_syms * N : A.frame_samples;
        float mx = 0.0f;
        for (unsigned long long i = tid; i < count; i += kTile) {
            cf32 x = fr[i];
            if (MODE == LPHY_MODE_DECHIRP_LORA_DEMODULATE) x = cmul_x(x, A.down[i & (N - 1)]);
            maxabs_acc(mx, x);
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const float o = __shfl_xor(mx, off, 64);
            mx = o > mx ? o : mx;
        }
        if ((tid & 63) == 0) sh.wmax[tid >> 6] = mx;
    }
    __syncthreads();
    if (tid == 0) {
        lphy_frame_meta m{};
        m.scale = 1.0f;
        m.have_sync = have_sync;
        if (MODE != LPHY_MODE_DEMODULATE) {
            float mx = sh.wmax[0];
            for (int w = 1; w < kTile / 64; ++w) mx = sh.wmax[w] > mx ? sh.wmax[w] : mx;
            m = norm_meta(mx, have_sync, A.no_scratch);
        }
        sh.m = m;
        sh.sw[0] = sh.sw[1] = 0;
    }
    __syncthreads();
    // (2) estimate: units (symbol, osr phase) in chunks of T, folded in
    // order by thread 0 (the separate k_estimate's unpacked path)
    EstFold fold;
    const int U = A.est_units;
    const bool tie_low = MODE != LPHY_MODE_DEMODULATE;
    for (int c0 = 0; c0 < U && sh.m.status == 0; c0 += T) {
        const lphy_frame_meta m = sh.m;
        const int u = c0 + slot;
        const bool live = u < U;
        const int s = live ? u / A.osr : 0, t = live ? u % A.osr : 0;
        const Stage<SF> st(slot, lam);
#pragma unroll
        for (int e = 0; e < G::E; ++e) {
            const int i = lam + e * G::LPS;
            cf32 x = czero();
            if (live) x = est_sample(A, fr, (unsigned long long)s * step + t + (unsigned long long)i * A.osr, i, N, m);
            st.put(sh.lds, e, x);
        }
        __syncthreads();
        cf32 v[16];
        fft_tile<SF, false, true>(v, sh.lds, slot, lam, A.tw);
#pragma unroll
        for (int e = 0; e < G::E; ++e) sh.lds[G::addr(slot, bin_of<SF>(e, lam))] = v[e];
        const ArgMax best = symbol_argmax<SF>(local_argmax<SF>(v, lam), sh.red);
        __syncthreads();
        if (lam == 0) {
            sh.units[slot] = live ? unit_result<SF>(sh.lds, slot, best) : UnitResult{0, 0, 0.0f, 0.0f, 0};
            sh.upow[slot] = live && A.osr > 1 ? detector_power(best.v > 0.0f ? best.v : 0.0f, A.power_scale) : 0.0f;
        }
        __syncthreads();
        if (tid == 0) {
            const int nu = U - c0 < T ? U - c0 : T;
            for (int k = 0; k < nu; ++k) fold.unit(sh.units[k], A.osr > 1 ? sh.upow[k] : 0.0f, A.osr, tie_low);
        }
        __syncthreads();
    }
    if (tid == 0 && sh.m.status == 0) fold.finish(sh.m, U / A.osr, N, A.osr);
    __syncthreads();
    // (3) symbols, T per tile, exact per-sample rotation
    const lphy_frame_meta m = sh.m;
    const unsigned S = (unsigned)A.total_syms;
    for (unsigned s0 = 0; s0 < S; s0 += T) {
        const unsigned s = s0 + slot;
        const bool live = s < S;
        const SymCtx c = sym_ctx<true>(A, f, live ? s : 0, live, N, m);
        if (A.win)
            restage_symbol<SF, MODE | kWinBit, true>(sh.lds, Stage<SF>(slot, lam), fr + c.base, c, lam,
                                                     A.down, A.win, (unsigned)A.osr);
        else
            restage_symbol<SF, MODE, true>(sh.lds, Stage<SF>(slot, lam), fr + c.base, c, lam,
                                           A.down, nullptr, (unsigned)A.osr);
        __syncthreads();
        cf32 v[16];
        fft_tile<SF, false, true>(v, sh.lds, slot, lam, A.tw);
        const ArgMax best = symbol_argmax<SF>(local_argmax<SF>(v, lam), sh.red);
        if (lam == 0 && live) {
            if (c.have_sync && s < 2) sh.sw[s] = c.ok ? (uint16_t)best.i : (uint16_t)0;
            else if (c.ok) A.syms[(unsigned long long)f * A.out_per_frame + (c.have_sync ? s - 2 : s)] = (uint16_t)best.i;
        }
        __syncthreads();
    }
    if (tid == 0) {
        lphy_frame_meta r = sh.m;
        r.sw0 = sh.sw[0];
        r.sw1 = sh.sw[1];
        A.meta[f] = r;
    }
    __syncthreads();
}

// Symbols the fused kernel's certificate left open (kSymRecheck in the
// output, frame status kStatusRecheck) among the workgroup's frames fb ..
// fb + kTile - 1: the reference's per-sample rotation with its Annex G
// products, T (frame, symbol) pairs per tile; the frames' offsets from the
// hot kernel stand (only symbol units were uncertified).  Thread t scans
// frame fb + t when `mine` (its status is kStatusRecheck).
template <int SF, int MODE>
__device__ void recheck_frames(const DemodArgs& A, unsigned long long fb, bool mine, PostShared<SF>& sh) {
    using G = Geo<SF>;
    constexpr int N = G::N, T = G::T;
    const int tid = threadIdx.x;
    const int slot = tid / G::LPS, lam = tid % G::LPS;
    const unsigned S = (unsigned)A.total_syms;
    unsigned cur = mine ? 0u : S;  // this thread's scan position in its frame
    unsigned long long done = 0;
    lphy_frame_meta mm{};
    if (mine) mm = A.meta[fb + tid];
    // Rows of up to 64 aligned data symbols (every bench shape): the row's
    // sentinels as a bit mask from its words loaded at once (one memory round
    // trip per frame; a load per symbol, then per 8, made the scan k_post's
    // longest part at mode A's ~6,600 re-runs per SF 7 launch)
    const bool hs0 = mm.have_sync != 0;
    const uint16_t* const out0 = A.syms + (fb + (unsigned)tid) * A.out_per_frame;
    const unsigned ofs0 = hs0 ? 2u : 0u;
    const bool fastscan = A.out_per_frame <= 64 && (A.out_per_frame & 7) == 0 && ((unsigned long long)out0 & 15ull) == 0ull &&
                          S == A.out_per_frame + ofs0;
    unsigned long long smask = 0;  // bit b: data symbol b is a sentinel; bits 62/63: sw0/sw1 (shifted below)
    unsigned smask_sync = 0;
    if (mine && fastscan) {
        uint4 q[8];
#pragma unroll
        for (int w = 0; w < 8; ++w)
            if (w * 8 < (int)A.out_per_frame) q[w] = reinterpret_cast<const uint4*>(out0)[w];
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            if (w * 8 >= (int)A.out_per_frame) break;
            const unsigned x[4] = {q[w].x, q[w].y, q[w].z, q[w].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if ((x[k] & 0xffffu) == kSymRecheck) smask |= 1ull << (8 * w + 2 * k);
                if ((x[k] >> 16) == kSymRecheck) smask |= 1ull << (8 * w + 2 * k + 1);
            }
        }
        if (hs0) smask_sync = (mm.sw0 == kSymRecheck ? 1u : 0u) | (mm.sw1 == kSymRecheck ? 2u : 0u);
    }
    for (;;) {
        __syncthreads();
        if (tid == 0) sh.count = 0;
        __syncthreads();
        // collect up to kTile open symbols
        if (cur < S && fastscan) {
            for (;;) {
                // the next sentinel at or after cur
                unsigned next = S;
                if (cur < ofs0) {
                    const unsigned sm = smask_sync >> cur;
                    if (sm) next = cur + (unsigned)(__ffs(sm) - 1);
                }
                if (next == S) {
                    const unsigned d = cur > ofs0 ? cur - ofs0 : 0u;
                    const unsigned long long m = d < 64 ? (smask >> d) << d : 0ull;
                    if (m) next = ofs0 + (unsigned)(__ffsll((long long)m) - 1);
                }
                cur = next;
                if (cur >= S) break;
                const unsigned k = atomicAdd(&sh.count, 1u);
                if (k >= kTile) break;  // full: this symbol goes in the next round
                sh.list[k] = cur;
                sh.listf[k] = (unsigned)tid;
                ++cur;
            }
        } else if (cur < S) {
            const unsigned long long f = fb + tid;
            const bool hs = mm.have_sync != 0;
            const uint16_t* out = A.syms + f * A.out_per_frame;
            for (; cur < S; ++cur) {
                const uint16_t v = (hs && cur < 2) ? (cur == 0 ? mm.sw0 : mm.sw1) : out[hs ? cur - 2 : cur];
                if (v != kSymRecheck) continue;
                const unsigned k = atomicAdd(&sh.count, 1u);
                if (k >= kTile) break;  // full: this symbol goes in the next round
                sh.list[k] = cur;
                sh.listf[k] = (unsigned)tid;
            }
        }
        __syncthreads();
        const unsigned n = sh.count < kTile ? sh.count : kTile;
        if (n == 0) break;
        done += n;
        for (unsigned k0 = 0; k0 < n; k0 += T) {
            const unsigned k = k0 + (unsigned)slot;
            const bool live = k < n;
            const unsigned sy = live ? sh.list[k] : 0;
            const unsigned long long f = fb + (live ? sh.listf[k] : 0);
            lphy_frame_meta m = A.meta[f];
            m.status = 0;
            const SymCtx c = sym_ctx<true>(A, (unsigned)f, sy, live, N, m);
            const cf32* fr = A.iq + f * A.frame_samples;
            if (A.win)
                restage_symbol<SF, MODE | kWinBit, true>(sh.lds, Stage<SF>(slot, lam), fr + c.base, c, lam,
                                                         A.down, A.win, (unsigned)A.osr);
            else
                restage_symbol<SF, MODE, true>(sh.lds, Stage<SF>(slot, lam), fr + c.base, c, lam,
                                               A.down, nullptr, (unsigned)A.osr);
            __syncthreads();
            cf32 v[16];
            fft_tile<SF, false, true>(v, sh.lds, slot, lam, A.tw);
            const ArgMax best = symbol_argmax<SF>(local_argmax<SF>(v, lam), sh.red);
            if (lam == 0 && live) store_symbol(A, c, (uint16_t)best.i);
            __syncthreads();
        }
    }
    if (tid == 0 && done) atomicAdd(&A.counters[kCtrRecheck], done);
}

// Frames k_frames demodulated under a speculative normalisation that the
// frame's later samples overturned (status kStatusSettle[Recheck]), among the
// workgroup's frames fb .. fb + kTile - 1 (thread t: frame fb + t, `mine`).
// Their two estimate symbols are transformed again, T/2 frames per tile, with
// the exact normalisation (the reference's arithmetic, as exact_frame), and
// folded into the exact offsets.  The symbols stand when the time shift is
// unchanged and every certified symbol's lead still covers the larger sample
// bound and the rate difference: a rate error d moves every bin by at most
// |d| N sum|y_i| <= |d| N A (the phase error of sample i is |d| i), charged
// twice on both sides of the comparison as fast_certified charges its B.
// Otherwise the frame is re-run whole (kStatusFixup).
template <int SF, int MODE>
__device__ void settle_frames(const DemodArgs& A, unsigned long long fb, bool mine, PostShared<SF>& sh) {
    using G = Geo<SF>;
    constexpr int N = G::N, T = G::T;
    const int tid = threadIdx.x;
    const int slot = tid / G::LPS, lam = tid % G::LPS;
    if (tid == 0) sh.count = 0;
    __syncthreads();
    if (mine) sh.list[atomicAdd(&sh.count, 1u)] = (unsigned)tid;
    __syncthreads();
    const unsigned n = sh.count;
    // units (frame k, estimate symbol s) = 2k + s, T per tile pass
    for (unsigned u0 = 0; u0 < 2 * n; u0 += T) {
        const unsigned u = u0 + (unsigned)slot;
        const bool live = u < 2 * n;
        const unsigned k = live ? u / 2 : 0u, s = u & 1u;
        const unsigned long long f = fb + (live ? sh.list[k] : 0u);
        const lphy_frame_meta m = norm_meta(A.meta[f].cfo, true, 0);  // cfo holds the max-abs
        const cf32* fr = A.iq + f * A.frame_samples;
        const Stage<SF> st(slot, lam);
#pragma unroll
        for (int e = 0; e < G::E; ++e) {
            const int i = lam + e * G::LPS;
            st.put(sh.lds, e, live ? est_sample(A, fr, (unsigned long long)s * N + (unsigned)i, i, N, m) : czero());
        }
        __syncthreads();
        cf32 v[16];
        fft_tile<SF, false, true>(v, sh.lds, slot, lam, A.tw);
#pragma unroll
        for (int e = 0; e < G::E; ++e) sh.lds[G::addr(slot, bin_of<SF>(e, lam))] = v[e];
        const ArgMax best = symbol_argmax<SF>(local_argmax<SF>(v, lam), sh.red);
        __syncthreads();
        if (lam == 0 && live) sh.ures2[k][s] = unit_result<SF>(sh.lds, slot, best);
        __syncthreads();
    }
    if ((unsigned)tid < n) {
        const unsigned long long g = fb + sh.list[tid];
        const lphy_frame_meta sm = A.meta[g];
        lphy_frame_meta e = norm_meta(sm.cfo, true, 0);
        EstFold fold;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const UnitResult r = sh.ures2[tid][u];
            if (r.valid) fold.add(r.idx, r.findex, 0, r.phase);
            else fold.add(0, 0.0f, 0, 0.0f);
        }
        fold.finish(e, 2, N, 1);
        // amplitude bound of the speculatively scaled samples, and the
        // smallest bound of any symbol (|start| grows with the symbol)
        const float a = fmaxf(1.0f, sm.cfo * sm.scale) * 1.0001f;
        const float b1 = cert_bound<SF>(sm.rate, sm.rate * (float)sm.t_off, 1.0f);
        const float d = fabsf(e.rate - sm.rate) * (1.0f + 4.0f * kU);
        const float A1 = (float)N * 1.41421366f * 1.0001f;
        const bool ok = e.t_off == sm.t_off && sm.t_off >= -N && sm.t_off <= N &&
                        sm.time_offset > 4.0f * a + 4.0f * d * (float)N * A1 * a / b1;
        lphy_frame_meta r = e;
        r.sw0 = sm.sw0;
        r.sw1 = sm.sw1;
        r.status = !ok ? kStatusFixup : (sm.status == kStatusSettleRecheck ? kStatusRecheck : 0);
        A.meta[g] = r;
    }
    __syncthreads();
}

// Separate launches with spec_big (SF 11-12, modes 1/2): the frame-end
// check k_frames makes in-kernel, one workgroup per frame (so the exact
// estimates of settled frames run in parallel).  The samples no symbol
// window covers are scanned; the frame's true max-abs then confirms the
// two-symbol normalisation, or - NaN / inf - sends the frame to k_post's
// exact re-run, or settles it here: both estimate FFTs again with the exact
// scale (the reference's arithmetic, as exact_frame) and the certificate
// check of settle_frames against the exact rate, else the exact re-run.
template <int SF, int MODE>
__global__ __launch_bounds__(kTile) void k_spec_settle(DemodArgs A) {
    using G = Geo<SF>;
    constexpr int N = G::N, T = G::T;
    constexpr bool DECH = MODE == LPHY_MODE_DECHIRP_LORA_DEMODULATE;
    __shared__ PostShared<SF> sh;
    const unsigned long long f = blockIdx.x;
    const int tid = threadIdx.x;
    const lphy_frame_meta m = A.meta[f];
    if (!(m.status == 0 || m.status == kStatusRecheck)) return;  // uniform
    const unsigned S = (unsigned)A.total_syms;
    const unsigned cnt = DECH ? S * N : (unsigned)A.frame_samples;
    const unsigned end = covered_end(S, N, cnt, m.t_off);
    const cf32* fr = A.iq + f * A.frame_samples;
    float frag = 0.0f;
    bool fbad = false;
    if (end < cnt) {
        float mx = 0.0f;
        bool bad = false;
        for (unsigned i = end + (unsigned)tid; i < cnt; i += kTile) {
            cf32 x = fr[i];
            if constexpr (DECH) x = cmul(x, A.down[i & (N - 1)]);
            bad |= !(__builtin_isfinite(x.x) && __builtin_isfinite(x.y));
            maxabs_acc(mx, x);
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const float o = __shfl_xor(mx, off, 64);
            mx = o > mx ? o : mx;
        }
        fbad = __syncthreads_or(bad);
        if ((tid & 63) == 0) sh.wmax[tid >> 6] = mx;
        __syncthreads();
        frag = sh.wmax[0];
        for (int w = 1; w < kTile / 64; ++w) frag = sh.wmax[w] > frag ? sh.wmax[w] : frag;
    }
    const uint4 r = A.spec_big[f];
    const float mx01 = __uint_as_float(r.x);
    const float mt = fmaxf(fmaxf(mx01, __uint_as_float(r.y)), frag);
    const lphy_frame_meta mg = norm_meta(mx01, true, 0), me = norm_meta(mt, true, 0);
    if ((r.w & 1u) || fbad || !(mt <= 3.40282347e38f)) {
        if (tid == 0) A.meta[f].status = kStatusFixup;
        return;
    }
    if (me.scale == mg.scale && me.normalised == mg.normalised) return;  // confirmed
    // settle: the two estimate units, T per pass
    const int slot = tid / G::LPS, lam = tid % G::LPS;
    for (unsigned u0 = 0; u0 < 2; u0 += T) {
        const unsigned s = u0 + (unsigned)slot;
        const bool live = s < 2;
        const Stage<SF> st(slot, lam);
#pragma unroll
        for (int e = 0; e < G::E; ++e) {
            const int i = lam + e * G::LPS;
            st.put(sh.lds, e, live ? est_sample(A, fr, (unsigned long long)s * N + (unsigned)i, i, N, me) : czero());
        }
        __syncthreads();
        cf32 v[16];
        fft_tile<SF, false, true>(v, sh.lds, slot, lam, A.tw);
#pragma unroll
        for (int e = 0; e < G::E; ++e) sh.lds[G::addr(slot, bin_of<SF>(e, lam))] = v[e];
        const ArgMax best = symbol_argmax<SF>(local_argmax<SF>(v, lam), sh.red);
        __syncthreads();
        if (lam == 0 && live) sh.ures2[0][s] = unit_result<SF>(sh.lds, slot, best);
        __syncthreads();
    }
    if (tid == 0) {
        lphy_frame_meta e = me;
        EstFold fold;
        for (int u = 0; u < 2; ++u) {
            const UnitResult ur = sh.ures2[0][u];
            if (ur.valid) fold.add(ur.idx, ur.findex, 0, ur.phase);
            else fold.add(0, 0.0f, 0, 0.0f);
        }
        fold.finish(e, 2, N, 1);
        const float a = fmaxf(1.0f, mt * m.scale) * 1.0001f;
        const float b1 = cert_bound<SF>(m.rate, m.rate * (float)m.t_off, 1.0f);
        const float d = fabsf(e.rate - m.rate) * (1.0f + 4.0f * kU);
        const float A1 = (float)N * 1.41421366f * 1.0001f;
        const float R = __uint_as_float(r.z);
        const bool ok = e.t_off == m.t_off && m.t_off >= -N && m.t_off <= N &&
                        R > 4.0f * a + 4.0f * d * (float)N * A1 * a / b1;
        lphy_frame_meta out = e;
        out.sw0 = m.sw0;
        out.sw1 = m.sw1;
        out.status = !ok ? kStatusFixup : (((r.w & 2u) || m.status == kStatusRecheck) ? kStatusRecheck : 0);
        A.meta[f] = out;
    }
}

// After the symbol kernels: the exact re-run of the frames they flagged
// (kStatusFixup: whole frame; kStatusRecheck: the open symbols), then (fin)
// the per-frame finalisation, one thread per frame.
template <int SF>
union PostLds {  // the exact re-runs' workspace, then the finalisation's staging
    PostShared<SF> sh;
    FinStage fs;
};
template <int SF, int MODE>
__global__ __launch_bounds__(kTile) void k_post(DemodArgs A, FinalArgs F, int fix, int fin) {
    __shared__ PostLds<SF> L;
    PostShared<SF>& sh = L.sh;
    __shared__ unsigned flist[kTile];
    __shared__ unsigned fcount;
    const unsigned long long f = (unsigned long long)blockIdx.x * kTile + threadIdx.x;
    if (fix) {
        int st = f < A.frames ? A.meta[f].status : 0;
        const bool settle = st == kStatusSettle || st == kStatusSettleRecheck;
        if (__syncthreads_or(settle)) {
            settle_frames<SF, MODE>(A, (unsigned long long)blockIdx.x * kTile, settle, sh);
            __syncthreads();
            if (f < A.frames) st = A.meta[f].status;
        }
        const bool fixup = st == kStatusFixup;
        const bool recheck = st == kStatusRecheck;
        if (__syncthreads_or(fixup)) {
            if (threadIdx.x == 0) fcount = 0;
            __syncthreads();
            if (fixup) flist[atomicAdd(&fcount, 1u)] = (unsigned)f;
            __syncthreads();
            const unsigned n = fcount;
            for (unsigned k = 0; k < n; ++k) exact_frame<SF, MODE>(A, flist[k], sh);
        }
        if (__syncthreads_or(recheck)) {
            recheck_frames<SF, MODE>(A, (unsigned long long)blockIdx.x * kTile, recheck, sh);
            __syncthreads();
            if (recheck) A.meta[f].status = 0;
        }
    }
    if (!fin) return;
#ifndef LPHY_AB_FINAL_THREAD  // A/B timing only: a row per thread straight from memory
    if (fix) __syncthreads();  // the re-runs are done with the shared workspace
    if (finalize_block(F, (unsigned long long)blockIdx.x * kTile, L.fs)) return;
#endif
    if (f < A.frames) finalize_frame(F, f);
}

#include "lphy_wave.h"

// ---------------------------------------------------------------------------
// lora_modulate (LoRaMod.cpp:8-43 + ChirpGenerator.hpp:24-51), bit-exact.
// The phase accumulator is one float recurrence through the whole frame
// (phase += f, f += fStep with one wrap per symbol), so some thread has to
// walk it in order.  Batches (many symbols): pass 1, one thread per frame,
// walks it and records the phase at each symbol start; pass 2, one thread
// per symbol, regenerates its samples from there.  Few symbols (a single
// frame, the reference's per-packet loop): pass 2 would be a handful of
// threads each walking N samples with a sincos per step, so instead each
// symbol's frequency sequence is built in parallel (k_mod_freq), one thread
// per frame adds them up in order (k_mod_accumulate, one dependent add per
// sample, loads a block ahead) and a sample-parallel pass turns the phases into IQ
// (k_mod_sincos).
// ---------------------------------------------------------------------------
struct ModArgs {
    const uint16_t* syms;
    cf32* iq;
    float* phase0;           // frames * (nsyms + 2) phase at symbol start
    float* phases;           // (walk) frames * (nsyms + 2) * N * osr phases
    unsigned long long frames, nsyms;
    int N, osr;
    float bws, ampl;
    uint8_t sync;
    unsigned long long* slow;  // (k_mod_fast) frames that took the serial walk
    int force_serial;          // (test build) k_mod_fast takes its serial walk for every frame
    struct ModFastG* mfg;      // (k_mod_fast GROWS, split) per frame: windows, pivots, chain start
    unsigned char* mft;        // (ditto) per frame: T, kModFastSyms x kModFastWin
    int blk;                   // 0: phases row after row; else (split form) rows interleaved by
                               // 16-byte groups, blk = rows per frame (k_mod_fast GROWS)
};

__device__ __forceinline__ float mod_f0(const ModArgs& A, unsigned long long f, unsigned long long s) {
    uint16_t v;
    if (s < 2) {
        int sf = 0;
        while ((1 << sf) < A.N) ++sf;
        const unsigned sh = sf > 4 ? sf - 4 : 0;
        v = s == 0 ? (uint16_t)((A.sync >> 4) << sh) : (uint16_t)((A.sync & 0x0f) << sh);
    } else {
        v = A.syms[f * A.nsyms + (s - 2)];
    }
    return (2.0f * kPi * (float)v * A.bws) / ((float)A.N * (float)A.osr);
}

// Eight steps of the chirp recurrence (ChirpGenerator.hpp:39-43): f += fStep,
// wrap once past fMax, phase += f; every rounding as the reference's loop.
// f only grows between wraps, so when the eighth f is not past fMax none of
// the eight is and the wrap test is skipped.
struct ChirpWalk {
    float fmin, fmax, fstep;
    __device__ __forceinline__ void step8(float& fr, float& phase, float p[8]) const {
        float g[8];
        float x = fr;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            x += fstep;
            g[k] = x;
        }
        if (g[7] > fmax) {
            x = fr;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                x += fstep;
                if (x > fmax) x -= (fmax - fmin);
                g[k] = x;
            }
        }
        fr = g[7];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            phase += g[k];
            p[k] = phase;
        }
    }
    __device__ __forceinline__ void step1(float& fr, float& phase) const {
        fr += fstep;
        if (fr > fmax) fr -= (fmax - fmin);
        phase += fr;
    }
};

__device__ __forceinline__ ChirpWalk chirp_walk(const ModArgs& A) {
    ChirpWalk w;
    w.fmin = -kPi * A.bws / (float)A.osr;
    w.fmax = kPi * A.bws / (float)A.osr;
    w.fstep = (2.0f * kPi * A.bws) / (float)(A.N * A.osr * A.osr);
    return w;
}

// the symbol-end wrap (ChirpGenerator.hpp:49, evaluated in double there)
__device__ __forceinline__ float wrap_phase(float phase) {
    const double w = floor((double)(phase / (2.0f * kPi))) * 2 * (double)kPi;
    return (float)((double)phase - w);
}

// Batch pass 1: the phase at every symbol start.
__global__ void k_mod_walk(ModArgs A) {
    const unsigned long long f = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= A.frames) return;
    const ChirpWalk W = chirp_walk(A);
    const int step = A.N * A.osr;
    float phase = 0.0f;
    const unsigned long long ns = A.nsyms + 2;
    for (unsigned long long s = 0; s < ns; ++s) {
        A.phase0[f * ns + s] = phase;
        float fr = W.fmin + mod_f0(A, f, s);
        int i = 0;
        for (; i + 8 <= step; i += 8) {
            float p[8];
            W.step8(fr, phase, p);
        }
        for (; i < step; ++i) W.step1(fr, phase);
        phase = wrap_phase(phase);
    }
}

// Few-symbol pass 1a: each symbol's frequency sequence (ChirpGenerator.hpp:
// 39-40; it restarts at fMin + f0 every symbol, so symbols run in parallel),
// one thread per symbol, into phases[].
__global__ void k_mod_freq(ModArgs A) {
    const unsigned long long g = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long ns = A.nsyms + 2;
    if (g >= A.frames * ns) return;
    const ChirpWalk W = chirp_walk(A);
    const int step = A.N * A.osr;
    float fr = W.fmin + mod_f0(A, g / ns, g % ns);
    float* out = A.phases + g * (unsigned long long)step;
    int i = 0;
    for (; (step & 3) == 0 && i + 4 <= step; i += 4) {  // 16-B aligned rows
        float q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            fr += W.fstep;
            if (fr > W.fmax) fr -= (W.fmax - W.fmin);
            q[k] = fr;
        }
        *reinterpret_cast<float4*>(out + i) = make_float4(q[0], q[1], q[2], q[3]);
    }
    for (; i < step; ++i) {
        fr += W.fstep;
        if (fr > W.fmax) fr -= (W.fmax - W.fmin);
        out[i] = fr;
    }
}

// Few-symbol pass 1b: the phase accumulator through the frame, in order
// (ChirpGenerator.hpp:41, 49), one thread per frame: phases[] holds each
// sample's f on entry and its phase on return.  The chain is one dependent
// add per sample, so the loads must never be what it waits for: blocks of
// 64 samples in registers, the next block's 16 loads issued before the
// current block's adds (ping-pong).  Loads and stores share vmcnt, so when
// a block starts, the 16 stores of the previous block and the 16 loads of
// the next are younger than its own loads: the explicit vmcnt(32) says so
// (the compiler's own analysis of the loop falls back to a near-full
// drain).  Rows of a multiple of 64 samples (SF >= 6 at osr 1); the rest
// take the plain loop.
constexpr int kAccBlock = 64;

__device__ __forceinline__ void acc_load(float4 (&b)[kAccBlock / 4], const float* p) {
#pragma unroll
    for (int k = 0; k < kAccBlock / 4; ++k) b[k] = *reinterpret_cast<const float4*>(p + 4 * k);
}

__device__ __forceinline__ void acc_run(float4 (&b)[kAccBlock / 4], float& phase, float* p) {
    __builtin_amdgcn_s_waitcnt(0x8F70);  // vmcnt(32): this block's loads have landed
#pragma unroll
    for (int k = 0; k < kAccBlock / 4; ++k) {
        float4 o;
        phase += b[k].x;
        o.x = phase;
        phase += b[k].y;
        o.y = phase;
        phase += b[k].z;
        o.z = phase;
        phase += b[k].w;
        o.w = phase;
        *reinterpret_cast<float4*>(p + 4 * k) = o;
    }
}

__global__ __launch_bounds__(64) void k_mod_accumulate(ModArgs A) {
    const unsigned long long f = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= A.frames) return;
    const unsigned long long step = (unsigned long long)A.N * A.osr;
    const unsigned long long ns = A.nsyms + 2;
    float* io = A.phases + f * ns * step;
    float phase = 0.0f;
    if (step % kAccBlock == 0) {
        const unsigned long long nb = ns * step / kAccBlock, per = step / kAccBlock;
        float4 b0[kAccBlock / 4], b1[kAccBlock / 4];
        acc_load(b0, io);
        // (the look-ahead loads are unconditional - past the end they
        // re-read the last block - so every path has the same VMEM count
        // and the compiler's waits stay relaxed)
        for (unsigned long long k = 0; k < nb; k += 2) {
            acc_load(b1, io + (k + 1 < nb ? k + 1 : nb - 1) * kAccBlock);
            acc_run(b0, phase, io + k * kAccBlock);
            if ((k + 1) % per == 0) phase = wrap_phase(phase);
            if (k + 1 >= nb) break;
            acc_load(b0, io + (k + 2 < nb ? k + 2 : nb - 1) * kAccBlock);
            acc_run(b1, phase, io + (k + 1) * kAccBlock);
            if ((k + 2) % per == 0) phase = wrap_phase(phase);
        }
        return;
    }
    for (unsigned long long s = 0; s < ns; ++s) {
        float* row = io + s * step;
        for (unsigned long long i = 0; i < step; ++i) {
            phase += row[i];
            row[i] = phase;
        }
        phase = wrap_phase(phase);
    }
}

// A packet's walk without walking it in order, one
// workgroup per frame, everything in LDS.  Symbol s's walk from its pivot
// sample k_s (where |phase| is largest, so consecutive floats are furthest
// apart) to the next symbol's pivot depends only on the float at k_s.  So:
// estimate every symbol's start in double (exact sums of its f row, then
// once more with each symbol's own rounding error, measured by walking every
// symbol from the first estimate in parallel), take the 64 consecutive
// floats around each pivot's estimate as candidates, walk every candidate in
// parallel to the next pivot (tail, symbol-end wrap, head of the next
// symbol) and record where it lands among that symbol's candidates.  The
// serial part is then a chain of ns table lookups from symbol 0's pivot,
// which is walked exactly from phase 0.  Every step is the reference's
// arithmetic on floats (ChirpGenerator.hpp:39-49), so a chain that stays
// inside the windows is the serial walk; one that leaves them (an estimate
// off by more than 32 floats, measured ≤ 19 at SF 7-8: tools/walk_lattice.py)
// falls back to the serial walk of the whole frame.  Rows `stride` floats
// apart in LDS, then T (dynamic LDS: up to SF 9 at 66 symbols); at most
// kModFastSyms symbols; the phases go to A.phases for k_mod_sincos.
// GROWS (round 6, frames whose rows do not fit the LDS: SF 10-12): the rows
// live in A.phases itself (stride = step, where k_mod_sincos reads the
// phases anyway), only T in dynamic LDS; the walks read them through L1/L2
// (one frame's rows: 66 x 16 KiB at SF 12), 16 candidates per thread in the
// candidate walks (one load per 16 chains).  The drift of the corrected
// estimates stays inside the window there too: <= 27 floats at SF 10-12
// after one correction (tools/walk_lattice.py 10 11 12, host).
constexpr int kModFastThreads = 1024;
constexpr int kModFastSyms = 256;
constexpr int kModFastWin = 64;
constexpr size_t kModFastLds = size_t(144) << 10;  // the f rows and T (dynamic)

__device__ __forceinline__ int f_ord(float x) {
    const int i = __float_as_int(x);
    return i >= 0 ? i : (int)(0x80000000u - (unsigned)i);
}
__device__ __forceinline__ float f_unord(int o) {
    return __int_as_float(o >= 0 ? o : (int)(0x80000000u - (unsigned)o));
}

// The split GROWS form's hand-over between its launches (per frame).
struct ModFastG {
    int base[kModFastSyms];
    int kp[kModFastSyms];
    int j0, ok;
};

struct ModFastShared {
    double est[kModFastSyms + 1];  // start estimates
    double tot[kModFastSyms];      // exact sum of each f row
    double err[kModFastSyms];      // each row's rounding error from est
    double piv[kModFastSyms];      // exact partial sum up to the pivot
    int kp[kModFastSyms];          // pivot sample
    int base[kModFastSyms];        // f_ord of the window's first candidate
    int J[kModFastSyms];           // the chain's candidate per symbol
    float xs[kModFastSyms];        // exact symbol starts
    int ok;
};

// f rows read 8 at a time: one LDS round trip per 8 steps of a walk, the
// loads of a block issued before its adds (and stores)
// (PF, rows in global memory, 16-byte aligned: chunks of 16 floats, NB of
// them in flight - a walk waits for one cache round trip per NB x 16 steps
// instead of one per 8; round 6: at SF 12 the round trips were most of the
// split modulator's 390 us per packet)
// PF: element i of the row at row[(i / 4) bs + i % 4] (bs = 4: contiguous;
// the split modulator's interleaved rows: 4 x rows per frame)
template <bool PF = false, int NB = 4, class Fn>
__device__ __forceinline__ void row_blocks(const float* row, int bs, int i0, int i1, Fn fn) {
    int i = i0;
    if constexpr (PF) {
        for (; i < i1 && (i & 3); ++i) fn(i, row[(i >> 2) * bs + (i & 3)]);
        const int nc = i < i1 ? (i1 - i) >> 4 : 0;
        if (nc > 0) {
            // float4 j of chunk c: group (i / 4) + j
            auto src = [&](int j) __attribute__((always_inline)) {
                return reinterpret_cast<const float4*>(row + (size_t)((i >> 2) + j) * (unsigned)bs);
            };
            float4 b[NB][4];
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                const int c = k < nc ? k : nc - 1;
#pragma unroll
                for (int q = 0; q < 4; ++q) b[k][q] = *src(4 * c + q);
            }
            auto eat = [&](int c, const float4 (&ch)[4]) __attribute__((always_inline)) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int ii = i + 16 * c + 4 * q;
                    fn(ii, ch[q].x);
                    fn(ii + 1, ch[q].y);
                    fn(ii + 2, ch[q].z);
                    fn(ii + 3, ch[q].w);
                }
            };
            // (whole rounds without branches, so the load counter's waits
            // stay partial across the loop's back edge; then the rest)
            int c0 = 0;
            for (; c0 + NB <= nc; c0 += NB) {
#pragma unroll
                for (int k = 0; k < NB; ++k) {
                    eat(c0 + k, b[k]);
                    const int cn = c0 + k + NB < nc ? c0 + k + NB : nc - 1;  // (past the end: a harmless re-read)
#pragma unroll
                    for (int q = 0; q < 4; ++q) b[k][q] = *src(4 * cn + q);
                }
            }
#pragma unroll
            for (int k = 0; k < NB - 1; ++k)
                if (c0 + k < nc) eat(c0 + k, b[k]);
            i += 16 * nc;
        }
        for (; i < i1; ++i) fn(i, row[(i >> 2) * bs + (i & 3)]);
    } else {
        (void)bs;  // (rows in LDS: contiguous)
        for (; i + 8 <= i1; i += 8) {
            float b[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) b[k] = row[i + k];
#pragma unroll
            for (int k = 0; k < 8; ++k) fn(i + k, b[k]);
        }
        for (; i < i1; ++i) fn(i, row[i]);
    }
}

// The in-place running sum of a global row over [i0, i1) from p (row[i] =
// p += row[i]), the loads pipelined as row_blocks<true, NB> and each chunk
// of 16 stored as four 16-byte stores; returns p.
template <int NB = 4>
__device__ __forceinline__ float walk_store(float* row, int bs, int i0, int i1, float p) {
    int i = i0;
    auto at = [&](int k) -> float& { return row[(k >> 2) * bs + (k & 3)]; };
    for (; i < i1 && (i & 3); ++i) at(i) = p += at(i);
    const int nc = i < i1 ? (i1 - i) >> 4 : 0;
    if (nc > 0) {
        auto io = [&](int j) __attribute__((always_inline)) {
            return reinterpret_cast<float4*>(row + (size_t)((i >> 2) + j) * (unsigned)bs);
        };
        float4 b[NB][4];
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int c = k < nc ? k : nc - 1;
#pragma unroll
            for (int q = 0; q < 4; ++q) b[k][q] = *io(4 * c + q);
        }
        auto eat = [&](int c, const float4 (&ch)[4]) __attribute__((always_inline)) {
            float4 o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                o[q].x = p += ch[q].x;
                o[q].y = p += ch[q].y;
                o[q].z = p += ch[q].z;
                o[q].w = p += ch[q].w;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) *io(4 * c + q) = o[q];
        };
        int c0 = 0;
        for (; c0 + NB <= nc; c0 += NB) {
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                eat(c0 + k, b[k]);
                const int cn = c0 + k + NB < nc ? c0 + k + NB : nc - 1;  // (a chunk not yet stored, or a re-read)
#pragma unroll
                for (int q = 0; q < 4; ++q) b[k][q] = *io(4 * cn + q);
            }
        }
#pragma unroll
        for (int k = 0; k < NB - 1; ++k)
            if (c0 + k < nc) eat(c0 + k, b[k]);
        i += 16 * nc;
    }
    for (; i < i1; ++i) at(i) = p += at(i);
    return p;
}

// sum of row s's samples [0, i1[s]) in double, a wave per row (GROWS: the
// rows are in global memory, interleaved by 16-byte groups, and every thread
// of the workgroup helps; the sums are estimates, exact to far below a
// float step)
template <class I1>
__device__ __forceinline__ void mf_row_sums(double* out, const float* rows, int ns, int tid, I1 i1) {
    const int wave = tid >> 6, lane = tid & 63, nw = kModFastThreads / 64;
    for (int s = wave; s < ns; s += nw) {
        const float* row = rows + 4 * s;
        const int n = i1(s);
        auto at = [&](int i) { return row[(i >> 2) * 4 * ns + (i & 3)]; };
        double t = 0.0;
        int i = lane;
        // (16 loads in flight per lane before their adds: one cache round
        // trip per 1,024 samples, not per 64)
        for (; i + 64 * 15 < n; i += 64 * 16) {
            float x[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) x[k] = at(i + 64 * k);
#pragma unroll
            for (int k = 0; k < 16; ++k) t += (double)x[k];
        }
        for (; i < n; i += 64) t += (double)at(i);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) t += __shfl_xor(t, off, 64);
        if (lane == 0) out[s] = t;
    }
}

// est[s] = sum over r < s of (a[r] + b[r]) (exclusive prefix, unwrapped),
// one wave, 64 symbols per pass
__device__ __forceinline__ void mf_scan(double* est, const double* a, const double* b, int ns, int lane) {
    double carry = 0.0;
    for (int s0 = 0; s0 < ns; s0 += 64) {
        const int s = s0 + lane;
        const double v = s < ns ? a[s] + (b ? b[s] : 0.0) : 0.0;
        double x = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const double y = __shfl_up(x, off, 64);
            if (lane >= off) x += y;
        }
        if (s < ns) est[s] = carry + (x - v);
        carry += __shfl(x, 63, 64);
    }
}

#ifdef LPHY_MODFAST_CLOCKS  // timing aid only: per-phase wall clock sums into the clock counters
#define MF_T(k)                                                                   \
    if (tid == 0) {                                                               \
        const unsigned long long now = wall_clock64();                            \
        if (k > 0) atomicAdd(A.slow - kCtrModSerial + kCtrClocks + k - 1, now - mf_t); \
        mf_t = now;                                                               \
    }
#else
#define MF_T(k)
#endif
// PART (GROWS only): 0 the whole walk in this launch; 1 steps 1-5, handing
// the windows, pivots and chain start to A.mfg; 3 steps 7-8 from A.mfg and
// the T that k_mod_cand (step 6, spread over the GPU) wrote to A.mft.
template <bool GROWS, int PART = 0>
__global__ __launch_bounds__(kModFastThreads) void k_mod_fast(ModArgs A, int stride) {
    extern __shared__ float4 mod_lds[];
    __shared__ ModFastShared M;
    const unsigned long long f = blockIdx.x;
    const int step = A.N * A.osr;
    const int ns = (int)(A.nsyms + 2);
    const int tid = threadIdx.x;
    float* rows = GROWS ? A.phases + f * (unsigned long long)ns * step : reinterpret_cast<float*>(mod_lds);
    // GROWS (round 6): the frame's rows interleaved by 16-byte groups,
    // element i of row s at ((i / 4) ns + s) 4 + i % 4, so the walks of one
    // row per lane read and write 1 KiB contiguous per instruction (row
    // after row, each lane's 16 bytes were a cache line of their own); rowp
    // and the group stride bs (LDS rows: contiguous, bs = 4)
    const int bs = GROWS ? 4 * ns : 4;
    auto rowp = [&](int s) __attribute__((always_inline)) { return GROWS ? rows + 4 * s : rows + (size_t)s * stride; };
    // T[s][j]: where candidate j of symbol s lands among symbol s+1's, 255 outside
    unsigned char* T = PART != 0 ? A.mft + f * (unsigned long long)(kModFastSyms * kModFastWin)
                       : GROWS   ? reinterpret_cast<unsigned char*>(mod_lds)
                                 : reinterpret_cast<unsigned char*>(rows + (size_t)ns * stride);
    const ChirpWalk W = chirp_walk(A);
    const double two_pi = 2.0 * (double)kPi;
#ifdef LPHY_MODFAST_CLOCKS
    unsigned long long mf_t = 0;
#endif
    if constexpr (PART == 3) {
        // the hand-over of PART 1 (the rows are in A.phases already)
        const ModFastG& G = A.mfg[f];
        for (int s = tid; s < ns; s += blockDim.x) {
            M.base[s] = G.base[s];
            M.kp[s] = G.kp[s];
        }
        if (tid == 0) {
            M.J[0] = G.j0;
            M.ok = G.ok;
        }
#ifdef LPHY_MODFAST_CLOCKS
        if (tid == 0) mf_t = wall_clock64();
#endif
        __syncthreads();
    } else {
    MF_T(0)
    // 1. f rows (ChirpGenerator.hpp:39-40) and their exact sums
    for (int s = tid; s < ns; s += blockDim.x) {
        float fr = W.fmin + mod_f0(A, f, (unsigned long long)s);
        float* row = rowp(s);
        double t = 0.0;
        int i = 0;
        for (; i + 8 <= step; i += 8) {
            float g[8];
            float x = fr;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                x += W.fstep;
                g[k] = x;
            }
            if (g[7] > W.fmax) {  // (f only grows between wraps: ChirpWalk::step8)
                x = fr;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    x += W.fstep;
                    if (x > W.fmax) x -= (W.fmax - W.fmin);
                    g[k] = x;
                }
            }
            fr = g[7];
            if constexpr (GROWS) {  // (two 16-byte groups)
                *reinterpret_cast<float4*>(row + (size_t)(i >> 2) * bs) = float4{g[0], g[1], g[2], g[3]};
                *reinterpret_cast<float4*>(row + (size_t)((i >> 2) + 1) * bs) = float4{g[4], g[5], g[6], g[7]};
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) row[i + k] = g[k];
            }
            if constexpr (!GROWS)
                t += (((double)g[0] + (double)g[1]) + ((double)g[2] + (double)g[3])) +
                     (((double)g[4] + (double)g[5]) + ((double)g[6] + (double)g[7]));  // (an estimate)
        }
        for (; i < step; ++i) {
            fr += W.fstep;
            if (fr > W.fmax) fr -= (W.fmax - W.fmin);
            row[(i >> 2) * bs + (i & 3)] = fr;
            t += (double)fr;
        }
        if constexpr (!GROWS) M.tot[s] = t;
    }
    __syncthreads();
    if constexpr (GROWS) {  // (the exact sums by the whole workgroup, off the walks' chains)
        mf_row_sums(M.tot, rows, ns, tid, [&](int) { return step; });
        __syncthreads();
    }
    MF_T(1)
    // 2. first estimates of the starts: unwrapped running sums (one add per
    //    symbol in order), wrapped per symbol in parallel
    if (tid < 64) mf_scan(M.est, M.tot, nullptr, ns, tid);
    if (tid == 0) M.ok = A.force_serial ? 0 : 1;  // (force_serial: test build, the fallback's tests)
    __syncthreads();
    MF_T(2)
    // 3. each row walked in float from its estimate: its rounding error, and
    //    the pivot (largest |phase| among every 8th sample) with the exact
    //    partial sum up to it
    for (int s = tid; s < ns; s += blockDim.x) {
        const float* row = rowp(s);
        const double e = M.est[s];
        const float x0 = (float)(e - floor(e * (1.0 / two_pi)) * two_pi);
        float p = x0;
        double q = 0.0, qb = 0.0;
        float best = -1.0f;
        int kb = 0;
        int i = 0;
        if constexpr (GROWS) {
            // the walk alone (the pivot's partial sum: mf_row_sums below)
            row_blocks<true>(row, bs, 0, step, [&](int k, float x) {
                p += x;
                if ((k & 7) == 7) {
                    const float a = fabsf(p);
                    if (a > best) {
                        best = a;
                        kb = k;
                    }
                }
            });
            i = step;
        }
        for (; i + 8 <= step; i += 8) {
            float b[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) b[k] = row[i + k];
#pragma unroll
            for (int k = 0; k < 8; ++k) p += b[k];
            q += (((double)b[0] + (double)b[1]) + ((double)b[2] + (double)b[3])) +
                 (((double)b[4] + (double)b[5]) + ((double)b[6] + (double)b[7]));
            const float a = fabsf(p);
            if (a > best) {
                best = a;
                kb = i + 7;
                qb = q;
            }
        }
        for (; i < step; ++i) {
            p += row[i];
            q += (double)row[i];
            if (fabsf(p) > best) {
                best = fabsf(p);
                kb = i;
                qb = q;
            }
        }
        M.err[s] = (double)p - ((double)x0 + M.tot[s]);
        M.kp[s] = kb;
        M.piv[s] = qb;
    }
    __syncthreads();
    if constexpr (GROWS) {
        mf_row_sums(M.piv, rows, ns, tid, [&](int s) { return M.kp[s] + 1; });
        __syncthreads();
    }
    MF_T(3)
    // 4. corrected estimates (unwrapped, in order); 5. the windows, and
    //    symbol 0's pivot walked exactly from 0
    if (tid < 64) mf_scan(M.est, M.tot, M.err, ns, tid);
    __syncthreads();
    for (int s = tid; s < ns; s += blockDim.x) {
        const double e = M.est[s];
        M.base[s] = f_ord((float)(e - floor(e * (1.0 / two_pi)) * two_pi + M.piv[s])) - kModFastWin / 2;
    }
    __syncthreads();
    if (tid == 0) {
        float p = 0.0f;
        row_blocks<GROWS>(rowp(0), bs, 0, M.kp[0] + 1, [&](int, float x) { p += x; });
        const int j = f_ord(p) - M.base[0];
        M.J[0] = j;
        if (j < 0 || j >= kModFastWin) M.ok = 0;
    }
    MF_T(4)
    if constexpr (PART == 1) {
        __syncthreads();
        ModFastG& G = A.mfg[f];
        for (int s = tid; s < ns; s += blockDim.x) {
            G.base[s] = M.base[s];
            G.kp[s] = M.kp[s];
        }
        if (tid == 0) {
            G.j0 = M.J[0];
            G.ok = M.ok;
        }
        return;
    }
    // 6. every candidate of every symbol walked to the next symbol's pivot,
    //    kPer candidates (j = g, g + kGroups, ...) per thread: one read of
    //    the row feeds kPer independent chains (8 from LDS, 16 from GROWS)
    constexpr int kPer = GROWS ? 16 : 8, kGroups = kModFastWin / kPer;
    for (int idx = tid; idx < (PART == 0 ? (ns - 1) * kGroups : 0); idx += blockDim.x) {
        const int s = idx / kGroups, g = idx - s * kGroups;
        const float* row = rowp(s);
        float p[kPer];
#pragma unroll
        for (int m = 0; m < kPer; ++m) p[m] = f_unord(M.base[s] + g + kGroups * m);
        row_blocks<GROWS>(row, bs, M.kp[s] + 1, step, [&](int, float x) {
#pragma unroll
            for (int m = 0; m < kPer; ++m) p[m] += x;
        });
#pragma unroll
        for (int m = 0; m < kPer; ++m) p[m] = wrap_phase(p[m]);
        const float* nrow = rowp(s + 1);
        const int kn = M.kp[s + 1];
        row_blocks<GROWS>(nrow, bs, 0, kn + 1, [&](int, float x) {
#pragma unroll
            for (int m = 0; m < kPer; ++m) p[m] += x;
        });
        const int b1 = M.base[s + 1];
#pragma unroll
        for (int m = 0; m < kPer; ++m) {
            const int jj = f_ord(p[m]) - b1;
            T[s * kModFastWin + g + kGroups * m] = (jj >= 0 && jj < kModFastWin) ? (unsigned char)jj : (unsigned char)255;
        }
    }
    __syncthreads();
    MF_T(5)
    }  // (PART != 3)
    // 7. the chain, one wave: lane j holds T[s][j], the next candidate is a
    //    lane read at the current one (uniform); T rows read 16 at a time
    if (tid < 64 && M.ok) {
        int j = M.J[0];
        int bad = 0;
        for (int s0 = 0; s0 + 1 < ns; s0 += 16) {
            int t[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) t[k] = s0 + k + 1 < ns ? T[(s0 + k) * kModFastWin + tid] : 0;
            int jv = 0;  // lane k: the candidate of symbol s0 + k + 1
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (s0 + k + 1 < ns) {
                    j = __builtin_amdgcn_readlane(t[k], j & 63);
                    bad |= j == 255;
                    jv = tid == k ? j : jv;
                }
            }
            if (tid < 16 && s0 + tid + 1 < ns) M.J[s0 + tid + 1] = jv;
        }
        if (bad && tid == 0) M.ok = 0;
    }
    __syncthreads();
    MF_T(6)
    if (M.ok) {
        // 8. the rows from their exact pivots: each symbol's tail (after the
        //    pivot) and, from the start that tail's wrap gives the next
        //    symbol, each symbol's head (up to its pivot)
        for (int s = tid; s < ns; s += blockDim.x) {
            float* row = rowp(s);
            float p = f_unord(M.base[s] + M.J[s]);
            if constexpr (GROWS) {
                p = walk_store(row, bs, M.kp[s] + 1, step, p);
            } else {
                row_blocks(row, bs, M.kp[s] + 1, step, [&](int i, float x) {
                    p += x;
                    row[i] = p;
                });
            }
            M.xs[s + 1 < ns ? s + 1 : 0] = s + 1 < ns ? wrap_phase(p) : 0.0f;
        }
        __syncthreads();
        for (int s = tid; s < ns; s += blockDim.x) {
            float* row = rowp(s);
            float p = M.xs[s];
            if constexpr (GROWS) {
                walk_store(row, bs, 0, M.kp[s] + 1, p);
            } else {
                row_blocks(row, bs, 0, M.kp[s] + 1, [&](int i, float x) {
                    p += x;
                    row[i] = p;
                });
            }
        }
    } else if (tid == 0) {
        // the serial walk (k_mod_accumulate's order)
        if (A.slow) atomicAdd(A.slow, 1ull);
        float phase = 0.0f;
        for (int s = 0; s < ns; ++s) {
            float* row = rowp(s);
            for (int i = 0; i < step; ++i) {
                float& x = row[(i >> 2) * bs + (i & 3)];
                phase += x;
                x = phase;
            }
            phase = wrap_phase(phase);
        }
    }
    __syncthreads();
    // 9. the phases out, row after row (k_mod_sincos, GPU-wide, turns them
    //    into IQ: one CU's sincos would be the longest phase); GROWS: they
    //    are there already
    if constexpr (GROWS) {
        MF_T(7)
        return;
    }
    const int count = ns * step;
    float* out = A.phases + f * (unsigned long long)count;
    for (int g = tid; g < count; g += blockDim.x) {
        const int s = g / step;
        out[g] = rows[(size_t)s * stride + (g - s * step)];
    }
    MF_T(7)
}
#undef MF_T

// Step 6 of the split GROWS form across the GPU: one thread per candidate
// (frame f, symbol s < ns - 1, candidate j), a wave per symbol, so the row
// reads are wave-uniform (scalar loads) and the 64 walks of a symbol run
// side by side; each walks its candidate from symbol s's pivot through the
// symbol-end wrap to symbol s + 1's pivot in the reference's float order and
// records where it lands (T).  Four symbols per 256-thread workgroup; 8
// chunks of 16 floats in flight per walk (row_blocks).
__global__ __launch_bounds__(256) void k_mod_cand(ModArgs A) {
    const int ns = (int)(A.nsyms + 2);
    const int per = (ns - 1 + 3) / 4;  // workgroups per frame
    const unsigned long long f = blockIdx.x / (unsigned)per;
    const int s = (int)(blockIdx.x % (unsigned)per) * 4 + (int)(threadIdx.x >> 6);
    const int j = (int)(threadIdx.x & 63);
    if (s >= ns - 1) return;  // (wave-uniform)
    const int step = A.N * A.osr;
    const ModFastG& G = A.mfg[f];
    // (the frame's rows interleaved by 16-byte groups, as k_mod_fast<true> writes them)
    const float* rows = A.phases + f * (unsigned long long)ns * (unsigned)step;
    float p = f_unord(G.base[s] + j);
    row_blocks<true, 8>(rows + 4 * s, 4 * ns, G.kp[s] + 1, step, [&](int, float x) { p += x; });
    p = wrap_phase(p);
    row_blocks<true, 8>(rows + 4 * (s + 1), 4 * ns, 0, G.kp[s + 1] + 1, [&](int, float x) { p += x; });
    const int jj = f_ord(p) - G.base[s + 1];
    A.mft[f * (unsigned long long)(kModFastSyms * kModFastWin) + (unsigned)(s * kModFastWin + j)] =
        (jj >= 0 && jj < kModFastWin) ? (unsigned char)jj : (unsigned char)255;
}

__global__ void k_mod_samples(ModArgs A) {
    const unsigned long long g = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long ns = A.nsyms + 2;
    if (g >= A.frames * ns) return;
    const unsigned long long f = g / ns, s = g % ns;
    const ChirpWalk W = chirp_walk(A);
    const int step = A.N * A.osr;
    float phase = A.phase0[g];
    float fr = W.fmin + mod_f0(A, f, s);
    cf32* out = A.iq + (f * ns + s) * (unsigned long long)step;
    for (int i = 0; i < step; ++i) {
        W.step1(fr, phase);
        float sn, cs;
        lphy_libm::sincosf_exact(phase, &sn, &cs);
        out[i] = cf32{A.ampl * cs, A.ampl * sn};  // std::polar(ampl, phase)
    }
}

__global__ void k_mod_sincos(ModArgs A, unsigned long long count) {
    const unsigned long long g = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= count) return;
    unsigned long long src = g;
    if (A.blk) {  // (the split form's interleaved rows: k_mod_fast<true>)
        const unsigned long long step = (unsigned long long)A.N * A.osr, fs = step * (unsigned)A.blk;
        const unsigned long long fb = g / fs * fs, r = g - fb, s = r / step, i = r - s * step;
        src = fb + ((i >> 2) * (unsigned)A.blk + s) * 4 + (i & 3);
    }
    float sn, cs;
    lphy_libm::sincosf_exact(A.phases[src], &sn, &cs);
    A.iq[g] = cf32{A.ampl * cs, A.ampl * sn};
}

// compensate_offsets (phy.cpp:150-180): rotation then integer time shift.
__global__ void k_comp_rotate(cf32* out, const cf32* in, unsigned long long count,
                              float rate) {
    const unsigned long long n = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= count) return;
    const float ph = rate * (float)n;
    float sn, cs;
    lphy_libm::sincosf_exact(ph, &sn, &cs);
    out[n] = cmul_x(in[n], cf32{cs, sn});  // samples[n] *= complex (phy.cpp:163)
}

__global__ void k_comp_shift(cf32* out, const cf32* in, unsigned long long count,
                             long long offset) {
    const unsigned long long n = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= count) return;
    const long long src = (long long)n - offset;
    out[n] = (src >= 0 && src < (long long)count) ? in[src] : czero();
}

}  // namespace

#ifdef LPHY_SF  // per-SF translation unit: launch templates
namespace {
#define HIP_OK(x)                                                         \
    do {                                                                  \
        hipError_t e_ = (x);                                              \
        if (e_ != hipSuccess) {                                           \
            fprintf(stderr, "lphy_hip: %s failed: %s (%s:%d)\n", #x,      \
                    hipGetErrorString(e_), __FILE__, __LINE__);           \
            return -EIO;                                                  \
        }                                                                 \
    } while (0)

// Waves per SIMD the demod kernel is register-budgeted for (launch bound):
// 3 (<= 168 VGPRs) or 2 (<= 256).  LPHY_DEMOD_OCC overrides for experiments.
constexpr int demod_occ(int sf) { return sf <= 8 ? 3 : 2; }

template <int SF, int MODE, int OCC>
int demod_grid() {
    static int grid = 0;
    if (grid == 0) {
        int dev = 0, cus = 0, per = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_demod<SF, MODE, OCC>, kTile, 0);
        grid = (cus > 0 ? cus : 256) * (per > 0 ? per : 1);
    }
    return grid;
}

inline int cu_count() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (cus <= 0) cus = 256;
    }
    return cus;
}

// per_cu > 0 caps the persistent grid at per_cu workgroups per CU (room
// for a concurrent kernel on another stream)
template <int SF, int MODE, int OCC>
void launch_symbols_occ(const DemodArgs& A0, unsigned long long tiles, hipStream_t st, int per_cu) {
    using G = Geo<SF>;
    constexpr bool WAVE = G::LPS <= 64;
    constexpr int WT = WAVE ? 64 / G::LPS : G::T;      // symbols per worker tile
    constexpr int WPB = WAVE ? kTile / 64 : 1;         // workers per workgroup
    unsigned long long g = (unsigned long long)demod_grid<SF, MODE, OCC>();
    if (per_cu > 0 && g > (unsigned long long)per_cu * cu_count()) g = (unsigned long long)per_cu * cu_count();
    const unsigned long long wtiles = (A0.frames * A0.total_syms + WT - 1) / WT;
    unsigned long long grid = (wtiles + WPB - 1) / WPB;
    if (grid > g) grid = g;
    DemodArgs A = A0;
    const unsigned long long stride = grid * WPB * WT;  // symbols per worker step
    A.stride_f = (unsigned)(stride / A0.total_syms);
    A.stride_s = (unsigned)(stride % A0.total_syms);
    (void)tiles;
    hipLaunchKernelGGL((k_demod<SF, MODE, OCC>), dim3((unsigned)grid), dim3(kTile), 0, st, A);
}

template <int SF, int MODE>
void launch_symbols(const DemodArgs& A, unsigned long long tiles, hipStream_t st, int per_cu) {
    launch_symbols_occ<SF, MODE, demod_occ(SF)>(A, tiles, st, per_cu);
}

// Fused path (k_frames).
template <int SF, int MODE, int OCC>
int frames_grid() {
    static int grid = 0;
    if (grid == 0) {
        int dev = 0, cus = 0, per = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_frames<SF, MODE, OCC>, kTile, 0);
        grid = (cus > 0 ? cus : 256) * (per > 0 ? per : 1);
    }
    return grid;
}

template <int SF, int MODE, int OCC>
int launch_frames_occ(const DemodArgs& A, hipStream_t st) {
    FrameArgs P{};
    P.A = A;
    constexpr unsigned WPB = kTile / 64;
    unsigned long long blocks = (unsigned long long)frames_grid<SF, MODE, OCC>();
    const unsigned long long need = (A.frames + WPB - 1) / WPB;
    if (blocks > need) blocks = need;
    P.waves = (unsigned)(blocks * WPB);
    hipLaunchKernelGGL((k_frames<SF, MODE, OCC>), dim3((unsigned)blocks), dim3(kTile), 0, st, P);
    HIP_OK(hipGetLastError());
    return 0;
}

// Waves per SIMD of k_frames: 2 (<= 256 VGPRs; its loop carries more state
// than k_demod's and spills at 3).
#ifndef LPHY_FRAMES_OCC  // experiments: -DLPHY_FRAMES_OCC=3
#define LPHY_FRAMES_OCC 2
#endif
template <int SF, int MODE>
int launch_frames_mode(const DemodArgs& A, hipStream_t st) {
    return launch_frames_occ<SF, MODE, LPHY_FRAMES_OCC>(A, st);
}

template <int SF, int MODE>
void launch_symbols_w(const DemodArgs& A, unsigned long long tiles, hipStream_t st, int per_cu) {
    if (A.osr > 1) {
        // oversampled input: strided symbol loads (no dechirp mode here)
        if constexpr ((MODE & 3) != LPHY_MODE_DECHIRP_LORA_DEMODULATE) {
            if (A.win) launch_symbols_occ<SF, MODE | kWinBit | kOsrBit, 2>(A, tiles, st, per_cu);
            else launch_symbols_occ<SF, MODE | kOsrBit, 2>(A, tiles, st, per_cu);
        }
        return;
    }
    if (A.win) launch_symbols<SF, MODE | kWinBit>(A, tiles, st, per_cu);
    else launch_symbols<SF, MODE>(A, tiles, st, per_cu);
}

template <int SF>
int launch_demod_sf(const DemodArgs& A, hipStream_t st, bool prologue, bool symbols, int per_cu) {
    using G = Geo<SF>;
    if (prologue) {
        if (A.mode != LPHY_MODE_DEMODULATE)
            hipLaunchKernelGGL(k_maxabs<SF>, dim3((unsigned)A.frames), dim3(kTile), 0, st, A);
        const int fpt = A.est_units <= G::T ? G::T / A.est_units : 1;
        const unsigned long long blocks = (A.frames + fpt - 1) / fpt;
        hipLaunchKernelGGL(k_estimate<SF>, dim3((unsigned)blocks), dim3(kTile), 0, st, A);
    }
    if (A.debug_recheck && symbols)
        hipLaunchKernelGGL(k_mark_recheck, dim3((unsigned)((A.frames + kTile - 1) / kTile)), dim3(kTile), 0, st,
                           A.meta, A.frames);
    if (symbols) {
        const unsigned long long nsym = A.frames * A.total_syms;
        const unsigned long long tiles = (nsym + G::T - 1) / G::T;
        if (tiles) {
            switch (A.mode) {
                case LPHY_MODE_DEMODULATE: launch_symbols_w<SF, LPHY_MODE_DEMODULATE>(A, tiles, st, per_cu); break;
                case LPHY_MODE_LORA_DEMODULATE: launch_symbols_w<SF, LPHY_MODE_LORA_DEMODULATE>(A, tiles, st, per_cu); break;
                default: launch_symbols_w<SF, LPHY_MODE_DECHIRP_LORA_DEMODULATE>(A, tiles, st, per_cu); break;
            }
        }
    }
    HIP_OK(hipGetLastError());
    return 0;
}

// Fused wave-per-symbol path, SF 7-12: k_wave (lphy_wave.h): one wave per
// SIMD, 256-thread workgroups, the next unit staged through LDS by DMA while
// a unit computes.  (Round 4's k_wave2 / k_wave2s, two waves per SIMD with
// shared exchange buffers, were removed in round 5: with the Parseval
// certificate and the grouped estimate units k_wave was faster at every SF,
// DESIGN §4.9.)
#ifndef LPHY_SPAN_MIN_SPW  // (-D for timing experiments only)
#define LPHY_SPAN_MIN_SPW 4
#endif
// SF 7-10 with at least SPW symbols per frame: units spanning frames
// (WSchedSpan); SF 7-8 take k_wave only then (wave_fit).
template <int SF, int MODE>
int launch_wave_mode(const DemodArgs& A, hipStream_t st) {
    FrameArgs P{};
    P.A = A;
    constexpr int WPB = wave_wpb<SF, MODE>();
    unsigned long long blocks = (unsigned long long)cu_count();
    const unsigned long long need = (A.frames + WPB - 1) / WPB;
    if (blocks > need) blocks = need;
    P.waves = (unsigned)(blocks * WPB);
    if constexpr (WGeo<SF>::SPW >= LPHY_SPAN_MIN_SPW) {
        if (A.total_syms >= (unsigned long long)WGeo<SF>::SPW) {
            hipLaunchKernelGGL((k_wave<SF, MODE, true>), dim3((unsigned)blocks), dim3(64 * WPB), 0, st, P);
            HIP_OK(hipGetLastError());
            return 0;
        }
    }
    if constexpr (SF >= 9) {
        hipLaunchKernelGGL((k_wave<SF, MODE, false>), dim3((unsigned)blocks), dim3(64 * WPB), 0, st, P);
        HIP_OK(hipGetLastError());
        return 0;
    } else {
        return -ENOTSUP;  // (wave_fit: S >= SPW below SF 9)
    }
}

// k_wave by mode, windowed (Hann) or not
template <int SF>
int launch_wave_sf(const DemodArgs& A, hipStream_t st) {
    if (A.win) {
        switch (A.mode) {
            case LPHY_MODE_DEMODULATE: return launch_wave_mode<SF, LPHY_MODE_DEMODULATE | kWinBit>(A, st);
            case LPHY_MODE_LORA_DEMODULATE:
                if constexpr (SF == 12) return -ENOTSUP;  // (wave_fit: the separate launches)
                else return launch_wave_mode<SF, LPHY_MODE_LORA_DEMODULATE | kWinBit>(A, st);
            default: return launch_wave_mode<SF, LPHY_MODE_DECHIRP_LORA_DEMODULATE | kWinBit>(A, st);
        }
    }
    switch (A.mode) {
        case LPHY_MODE_DEMODULATE: return launch_wave_mode<SF, LPHY_MODE_DEMODULATE>(A, st);
        case LPHY_MODE_LORA_DEMODULATE: return launch_wave_mode<SF, LPHY_MODE_LORA_DEMODULATE>(A, st);
        default: return launch_wave_mode<SF, LPHY_MODE_DECHIRP_LORA_DEMODULATE>(A, st);
    }
}

template <int SF>
int launch_frames_sf(const DemodArgs& A, hipStream_t st) {
    if constexpr (Geo<SF>::LPS > 64) {
        if constexpr (SF == 11 || SF == 12) return launch_wave_sf<SF>(A, st);
        (void)A; (void)st;
        return -ENOTSUP;
    } else {
        if constexpr (SF >= 7) {  // the wave-per-symbol geometry down to 2 lanes per symbol
            if (A.wave) return launch_wave_sf<SF>(A, st);
        }
        switch (A.mode) {
            case LPHY_MODE_DEMODULATE:
                return A.win ? launch_frames_mode<SF, LPHY_MODE_DEMODULATE | kWinBit>(A, st)
                             : launch_frames_mode<SF, LPHY_MODE_DEMODULATE>(A, st);
            case LPHY_MODE_LORA_DEMODULATE:
                return A.win ? launch_frames_mode<SF, LPHY_MODE_LORA_DEMODULATE | kWinBit>(A, st)
                             : launch_frames_mode<SF, LPHY_MODE_LORA_DEMODULATE>(A, st);
            default:
                return A.win ? launch_frames_mode<SF, LPHY_MODE_DECHIRP_LORA_DEMODULATE | kWinBit>(A, st)
                             : launch_frames_mode<SF, LPHY_MODE_DECHIRP_LORA_DEMODULATE>(A, st);
        }
    }
}

template <int SF>
int launch_post_sf(int mode, const DemodArgs& A, const FinalArgs& F, bool fix, bool fin, hipStream_t st) {
    const dim3 grid((unsigned)((A.frames + kTile - 1) / kTile));
    if (fix && A.spec_big) {
        if (mode == LPHY_MODE_LORA_DEMODULATE)
            hipLaunchKernelGGL((k_spec_settle<SF, LPHY_MODE_LORA_DEMODULATE>), dim3((unsigned)A.frames), dim3(kTile), 0,
                               st, A);
        else if (mode == LPHY_MODE_DECHIRP_LORA_DEMODULATE)
            hipLaunchKernelGGL((k_spec_settle<SF, LPHY_MODE_DECHIRP_LORA_DEMODULATE>), dim3((unsigned)A.frames),
                               dim3(kTile), 0, st, A);
    }
    switch (mode) {
        case LPHY_MODE_DEMODULATE:
            hipLaunchKernelGGL((k_post<SF, LPHY_MODE_DEMODULATE>), grid, dim3(kTile), 0, st, A, F, (int)fix, (int)fin);
            break;
        case LPHY_MODE_LORA_DEMODULATE:
            hipLaunchKernelGGL((k_post<SF, LPHY_MODE_LORA_DEMODULATE>), grid, dim3(kTile), 0, st, A, F, (int)fix, (int)fin);
            break;
        default:
            hipLaunchKernelGGL((k_post<SF, LPHY_MODE_DECHIRP_LORA_DEMODULATE>), grid, dim3(kTile), 0, st, A, F, (int)fix,
                               (int)fin);
            break;
    }
    HIP_OK(hipGetLastError());
    return 0;
}

template <int SF>
int launch_estimate_sf(const DemodArgs& A, hipStream_t st) {
    const int fpt = A.est_units <= Geo<SF>::T ? Geo<SF>::T / A.est_units : 1;
    hipLaunchKernelGGL(k_estimate<SF>, dim3((unsigned)((A.frames + fpt - 1) / fpt)), dim3(kTile), 0, st, A);
    HIP_OK(hipGetLastError());
    return 0;
}
}  // namespace
#endif
