// lphy_hip.hip — MI355X (gfx950) LoRa PHY demodulation kernels + C ABI.
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
#include "lphy_kernels.h"
#include "lphy_testing.h"

#include <cstring>
#include <memory>
#include <atomic>
#include <mutex>
#include <vector>

// ===========================================================================
// Host side
// ===========================================================================
#ifndef __HIP_DEVICE_COMPILE__
// Empty launch tables, overridden by every lphy_sf.hip object linked in
// (experiment builds may link only the SF they time: tools/ubench/variants.py)
namespace lphy {
__attribute__((weak)) extern const SfOps sf_ops_1 = {};
__attribute__((weak)) extern const SfOps sf_ops_2 = {};
__attribute__((weak)) extern const SfOps sf_ops_3 = {};
__attribute__((weak)) extern const SfOps sf_ops_4 = {};
__attribute__((weak)) extern const SfOps sf_ops_5 = {};
__attribute__((weak)) extern const SfOps sf_ops_6 = {};
__attribute__((weak)) extern const SfOps sf_ops_7 = {};
__attribute__((weak)) extern const SfOps sf_ops_8 = {};
__attribute__((weak)) extern const SfOps sf_ops_9 = {};
__attribute__((weak)) extern const SfOps sf_ops_10 = {};
__attribute__((weak)) extern const SfOps sf_ops_11 = {};
__attribute__((weak)) extern const SfOps sf_ops_12 = {};
}  // namespace lphy
#endif
// Constant device tables of one (sf, bw, window): KISS twiddles, down-chirp,
// Hann window.  Read-only after creation, so contexts made by
// lphy_hip_ctx_share hold the same tables.
struct lphy_tables {
    int device = 0;
    cf32* d_tw = nullptr;
    cf32* d_down = nullptr;
    float* d_win = nullptr;
    ~lphy_tables() {
        (void)hipSetDevice(device);
        if (d_tw) (void)hipFree(d_tw);
        if (d_down) (void)hipFree(d_down);
        if (d_win) (void)hipFree(d_win);
    }
};

struct lphy_hip_ctx {
    int device = 0;
    unsigned sf = 0, N = 0, bw_hz = 0, osr = 1;
    int window = 0;
    float power_scale = 0.0f;
    std::shared_ptr<lphy_tables> tab;
    cf32* d_tw = nullptr;   // tab's
    cf32* d_down = nullptr;
    float* d_win = nullptr;
    // the host convenience entry points (*_host): their own stream, so a
    // call waits for its own work only (hipStreamSynchronize), and staging
    // sized by lphy_hip_ctx_reserve up front; the mutex only orders calls
    // that share this context (one context per workspace / thread: never
    // contended)
    std::mutex mu;
    hipStream_t stream = nullptr;
    void* d_stage = nullptr;
    // pinned mirror of the staging's first h_stage_bytes (up to kPinnedMax):
    // a call whose buffers fit moves them with one DMA copy each way instead
    // of the runtime's pageable path (per-packet latency)
    void* h_stage = nullptr;
    size_t h_stage_bytes = 0;
    unsigned long long* d_counters = nullptr;  // kCounters slots (lphy_testing.h: kCtr*)
    size_t stage_bytes = 0;
    // the streaming entry point's pinned slots and streams (lphy_stream.hip),
    // made by its first call, kept for the next ones, freed with the context
    void* stream_ext = nullptr;
    void (*stream_ext_free)(void*) = nullptr;
    // smallest batch the fused kernels take on this context (-1: the measured
    // per-SF crossover, fused_min_frames; lphy_hip_ctx_set_fused_min_frames)
    std::atomic<long> fused_min{-1};
    std::atomic<int> mod_force_serial{0};  // (test build: lphy_hip_test_mod_force_serial)
    // (per-call scratch of the device entry points - the SF 11-12 speculation
    // records, the producer's phases, the compensation's shift buffer - comes
    // from the stream-ordered allocator on the caller's stream, so concurrent
    // calls on different streams or threads of one context never share it)
};


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

// Host-side constant tables with the reference's own libm calls.
void make_twiddles(std::vector<std::complex<float>>& tw, int nfft) {
    // kissfft.hh:24-29: exp(i * (i*phinc)), phinc = -2*acos(-1)/nfft in float
    tw.resize(nfft);
    const float phinc = (-2 * std::acos((float)-1)) / nfft;
    for (int i = 0; i < nfft; ++i) tw[i] = std::exp(std::complex<float>(0, i * phinc));
}

void make_downchirp(std::vector<std::complex<float>>& d, int N, float bw_scale) {
    // genChirp(out, N, 1, N, 0, down=true, 1, phase=0, bw_scale)
    // (ChirpGenerator.hpp:24-51)
    d.resize(N);
    const float fMin = -kPi * bw_scale / 1;
    const float fMax = kPi * bw_scale / 1;
    const float fStep = (2 * kPi * bw_scale) / (N * 1 * 1);
    float f = fMin + 0.0f;
    float phase = 0.0f;
    for (int i = 0; i < N; ++i) {
        f += fStep;
        if (f > fMax) f -= (fMax - fMin);
        phase -= f;
        d[i] = std::polar(1.0f, phase);
    }
}

void make_hann(std::vector<float>& w, int N) {
    // LoRaDemod.cpp:17-21 / phy.cpp:37-42
    w.resize(N);
    for (int i = 0; i < N; ++i)
        w[i] = 0.5f - 0.5f * std::cos(2.0f * kPi * static_cast<float>(i) /
                                      (static_cast<float>(N) - 1.0f));
}

// Whether k_frames can take this batch: a symbol within one wavefront, the
// two-symbol estimate, and frames long enough that a frame's estimate tile
// precedes its first symbol tile by two tiles (S + 3 >= 2 * units/tile).
inline bool frames_fit(unsigned sf, unsigned osr, int est_units, size_t total) {
    if (sf > 10 || osr != 1 || est_units != 2 || total < 2) return false;
    const size_t E = sf >= 4 ? 16 : ((size_t)1 << sf);
    const size_t lps = ((size_t)1 << sf) / E;
    const size_t wt = 64 / lps;
    return total + 1 >= 2 * wt;
}

// Whether the fused kernel k_wave (64 x 64 values per wavefront unit)
// takes this batch: SF 7-12, osr 1, the two-symbol estimate, the certified
// rotation, in modes 1/2 the speculative normalisation, and below SF 9 at
// least one unit of symbols per frame (4096 / N: its units span frames
// there); with or without the Hann window (round 6: its N floats beside the
// down-chirp in LDS; SF 12 with three waves per workgroup, wave_wpb, and not
// in mode 1, whose windowed k_wave spilled).
// LPHY_F_EXACT_ROTATION, the pre-scan schedule and shorter frames stay on
// k_frames (SF <= 10) or the separate launches (SF 11-12).
#ifndef LPHY_WAVE_MIN_SF  // smallest SF on k_wave (-D for timing experiments only)
#define LPHY_WAVE_MIN_SF 7
#endif
inline bool wave_fit(unsigned sf, unsigned osr, int est_units, size_t total, int mode, const DemodArgs& A) {
    return sf >= LPHY_WAVE_MIN_SF && sf <= 12 && (sf >= 9 || total >= (size_t)(4096u >> sf)) && osr == 1 &&
           !(sf == 12 && A.win && mode == LPHY_MODE_LORA_DEMODULATE) && est_units == 2 && total >= 2 &&
           !A.exact_rotation &&
           (mode == LPHY_MODE_DEMODULATE || A.spec);
}

const SfOps* sf_ops(unsigned sf) {
    static const SfOps* const t[13] = {nullptr,    &sf_ops_1, &sf_ops_2, &sf_ops_3,  &sf_ops_4,
                                       &sf_ops_5,  &sf_ops_6, &sf_ops_7, &sf_ops_8,  &sf_ops_9,
                                       &sf_ops_10, &sf_ops_11, &sf_ops_12};
    return sf >= 1 && sf <= 12 && t[sf]->demod ? t[sf] : nullptr;
}

int launch_demod(unsigned sf, const DemodArgs& A, hipStream_t st, bool pro, bool sym, int per_cu = 0) {
    const SfOps* o = sf_ops(sf);
    return o ? o->demod(A, st, pro, sym, per_cu) : -EINVAL;
}

int launch_frames(unsigned sf, const DemodArgs& A, hipStream_t st) {
    const SfOps* o = sf_ops(sf);
    return o ? o->frames(A, st) : -ENOTSUP;
}

int launch_post(unsigned sf, int mode, const DemodArgs& A, const FinalArgs& F, bool fix, bool fin,
                hipStream_t st) {
    const SfOps* o = sf_ops(sf);
    return o ? o->post(mode, A, F, fix, fin, st) : -EINVAL;
}


// Smallest batch the fused kernels take.  They give each frame one
// wavefront that walks its symbols in order, so a small batch leaves most
// of the GPU idle and the separate launches (symbol-parallel k_demod) finish
// first.  Crossovers measured per SF, mode 2 with decode, device time per
// call (tools/fused_crossover.py, profiles/r5/fused_crossover.json: with
// k_wave at SF 7-12 the fused kernel wins from 256 frames at SF 7-10, from
// 512 at SF 11-12, where 256 is a tie); the per-packet latency of the
// lora_phy:: API rides on the small end.  A context's own setting
// (lphy_hip_ctx_set_fused_min_frames) wins; the test build also reads a
// process default from LPHY_FUSED_MIN_FRAMES.
size_t fused_min_frames(const lphy_hip_ctx* c) {
    const long own = c->fused_min.load(std::memory_order_relaxed);
    if (own >= 0) return (size_t)own;
    const long test = lphy_test_fused_min_frames();
    if (test >= 0) return (size_t)test;
    static const size_t t[13] = {256, 256, 256, 256, 256, 256, 256, 256, 256, 256, 256, 384, 384};
    return t[c->sf <= 12 ? c->sf : 12];
}

constexpr size_t kPinnedMax = size_t(32) << 20;

int ensure_stage(lphy_hip_ctx* c, size_t bytes) {
    if (c->stage_bytes >= bytes) return 0;
    void* old = c->d_stage;
    c->d_stage = nullptr;
    c->stage_bytes = 0;
    if (old) HIP_OK(hipFree(old));
    HIP_OK(hipMalloc(&c->d_stage, bytes));
    c->stage_bytes = bytes;
    const size_t hb = std::min(bytes, kPinnedMax);
    if (hb > c->h_stage_bytes) {
        if (c->h_stage) HIP_OK(hipHostFree(c->h_stage));
        c->h_stage = nullptr;
        c->h_stage_bytes = 0;
        if (hipHostMalloc(&c->h_stage, hb, hipHostMallocDefault) == hipSuccess) c->h_stage_bytes = hb;
        else c->h_stage = nullptr;  // no pinned mirror: the calls take the pageable path
    }
    return 0;
}

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// Per-call device scratch of the device-buffer entry points, one policy for
// all of them (demod_batch's SF 11-12 speculation records, the producer's
// phases, the compensation's shift buffer): allocated and released in the
// caller's stream order (hipMallocAsync / hipFreeAsync from the stream-
// ordered pool, the null stream included), so its lifetime is exactly the
// call's kernels and no caller synchronises.  (Round 2-3 kept a plain
// hipMalloc plus a stream sync for the producers on the null stream, over a
// transcript that read a recycled block once and was never reproduced;
// round 3 removed the scratch-lowered table that was its likely cause,
// DESIGN §8.)  The *_host entry points lend a slice of their reserved
// staging instead (they run on the context's own stream and synchronise it
// before returning).
struct StreamScratch {
    void* p = nullptr;
    hipStream_t st;
    bool owned = false, pooled = false, pool_null = false;
    explicit StreamScratch(hipStream_t s, void* lent = nullptr, bool pool_on_null = true)
        : p(lent), st(s), pool_null(pool_on_null) {}
    int get(size_t bytes) {
        if (p) return 0;  // lent by the caller
        pooled = st != nullptr || pool_null;
        const hipError_t e = pooled ? hipMallocAsync(&p, bytes, st) : hipMalloc(&p, bytes);
        if (e != hipSuccess) {
            p = nullptr;
            return -ENOMEM;
        }
        owned = true;
        return 0;
    }
    ~StreamScratch() {
        if (!owned) return;
        if (pooled) {
            (void)hipFreeAsync(p, st);
        } else {
            (void)hipStreamSynchronize(st);
            (void)hipFree(p);
        }
    }
};


}  // namespace

extern "C" {

const char* lphy_hip_version(void) {
#if defined(LPHY_TEST_PATHS) && defined(LPHY_DEBUG_BOUNDS)
    return "lphy_hip 0.2 gfx950 test+bounds";
#elif defined(LPHY_TEST_PATHS)
    return "lphy_hip 0.2 gfx950 test";
#else
    return "lphy_hip 0.2 gfx950";
#endif
}

// Internal (not in include/lphy_hip.h): the context's HIP device, for the
// streaming ingestion in lphy_stream.hip.
int lphy_hip_ctx_device(const lphy_hip_ctx* c) { return c ? c->device : -1; }

// Internal: the streaming ingestion's state kept with the context (made by
// `make` on first use, released by `destroy` with the context).
void* lphy_hip_ctx_stream_ext(lphy_hip_ctx* c, void* (*make)(), void (*destroy)(void*)) {
    if (!c) return nullptr;
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->stream_ext) {
        c->stream_ext = make();
        c->stream_ext_free = destroy;
    }
    return c->stream_ext;
}

namespace {
// A context's own state: the host entry points' stream and the counters
// (the tables are set by the caller).
int ctx_own_state(lphy_hip_ctx* c) {
    if (hipMalloc(&c->d_counters, kCounters * sizeof(unsigned long long)) != hipSuccess) return -ENOMEM;
    HIP_OK(hipMemset(c->d_counters, 0, kCounters * sizeof(unsigned long long)));
    HIP_OK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    return 0;
}
}  // namespace

int lphy_hip_ctx_create(lphy_hip_ctx** out, int device, unsigned sf, unsigned bw_hz,
                        unsigned osr, int window) {
    if (!out) return -EINVAL;
    *out = nullptr;
    if (sf < 1 || sf > 12) return -EINVAL;
    if (bw_hz != 125000 && bw_hz != 250000 && bw_hz != 500000) return -EINVAL;
    if (osr == 0) osr = 1;
    if (osr > 64) return -EINVAL;
    if (window != LPHY_WINDOW_NONE && window != LPHY_WINDOW_HANN) return -EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return -ENODEV;
    HIP_OK(hipSetDevice(device));
    auto* c = new lphy_hip_ctx;
    c->device = device;
    c->sf = sf;
    c->N = 1u << sf;
    c->bw_hz = bw_hz;
    c->osr = osr;
    c->window = window;
    c->power_scale = (float)(20.0 * std::log10((double)c->N));  // LoRaDetector.hpp:29
    c->tab = std::make_shared<lphy_tables>();
    lphy_tables& t = *c->tab;
    t.device = device;
    std::vector<std::complex<float>> tw, down;
    make_twiddles(tw, (int)c->N);
    make_downchirp(down, (int)c->N, (float)bw_hz / 125000.0f);
    if (hipMalloc(&t.d_tw, c->N * sizeof(cf32)) != hipSuccess ||
        hipMalloc(&t.d_down, c->N * sizeof(cf32)) != hipSuccess ||
        (window == LPHY_WINDOW_HANN && hipMalloc(&t.d_win, c->N * sizeof(float)) != hipSuccess)) {
        lphy_hip_ctx_destroy(c);
        return -ENOMEM;
    }
    c->d_tw = t.d_tw;
    c->d_down = t.d_down;
    c->d_win = t.d_win;
    if (int rc = ctx_own_state(c)) {
        lphy_hip_ctx_destroy(c);
        return rc;
    }
    HIP_OK(hipMemcpy(t.d_tw, tw.data(), c->N * sizeof(cf32), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(t.d_down, down.data(), c->N * sizeof(cf32), hipMemcpyHostToDevice));
    if (window == LPHY_WINDOW_HANN) {
        std::vector<float> w;
        make_hann(w, (int)c->N);
        HIP_OK(hipMemcpy(t.d_win, w.data(), c->N * sizeof(float), hipMemcpyHostToDevice));
    }
    *out = c;
    return 0;
}

int lphy_hip_ctx_share(lphy_hip_ctx** out, const lphy_hip_ctx* base, unsigned osr) {
    if (!out || !base) return -EINVAL;
    *out = nullptr;
    if (osr == 0) osr = base->osr;
    if (osr > 64) return -EINVAL;
    HIP_OK(hipSetDevice(base->device));
    auto* c = new lphy_hip_ctx;
    c->device = base->device;
    c->sf = base->sf;
    c->N = base->N;
    c->bw_hz = base->bw_hz;
    c->osr = osr;  // the tables depend on N only
    c->window = base->window;
    c->power_scale = base->power_scale;
    c->tab = base->tab;
    c->d_tw = base->d_tw;
    c->d_down = base->d_down;
    c->d_win = base->d_win;
    if (int rc = ctx_own_state(c)) {
        lphy_hip_ctx_destroy(c);
        return rc;
    }
    *out = c;
    return 0;
}

// Internal (not in include/lphy_hip.h): the oversampling ratio of a context
// the caller owns alone (the C++ shim's per-workspace contexts; the
// reference's lora_demodulate takes osr per call).  The tables depend on N
// only.
int lphy_hip_ctx_set_osr(lphy_hip_ctx* c, unsigned osr) {
    if (!c || osr == 0 || osr > 64) return -EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    c->osr = osr;
    return 0;
}

void lphy_hip_ctx_destroy(lphy_hip_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamDestroy(c->stream);
    }
    if (c->stream_ext && c->stream_ext_free) c->stream_ext_free(c->stream_ext);
    if (c->d_stage) (void)hipFree(c->d_stage);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->d_counters) (void)hipFree(c->d_counters);
    c->tab.reset();  // the tables go with the last context holding them
    delete c;
}

int lphy_hip_ctx_set_fused_min_frames(lphy_hip_ctx* c, long frames) {
    if (!c) return -EINVAL;
    c->fused_min.store(frames < 0 ? -1L : frames, std::memory_order_relaxed);
    return 0;
}

size_t lphy_hip_syms_per_frame(const lphy_hip_ctx* c, size_t frame_samples, int mode) {
    if (!c) return 0;
    const size_t total = frame_samples / ((size_t)c->N * c->osr);
    if (mode == LPHY_MODE_DEMODULATE) return total >= 2 ? total - 2 : 0;
    return total >= 2 ? total - 2 : total;
}

namespace {
int demod_batch_impl(lphy_hip_ctx* c, const float* d_iq, size_t frames, size_t frame_samples,
                     uint16_t* d_syms, uint8_t* d_bytes, lphy_frame_meta* d_meta, int mode,
                     unsigned flags, hipStream_t st, void* lent_spec);
}

int lphy_hip_demod_batch(lphy_hip_ctx* c, const float* d_iq, size_t frames,
                         size_t frame_samples, uint16_t* d_syms, uint8_t* d_bytes,
                         lphy_frame_meta* d_meta, int mode, unsigned flags, void* stream) {
    return demod_batch_impl(c, d_iq, frames, frame_samples, d_syms, d_bytes, d_meta, mode, flags,
                            (hipStream_t)stream, nullptr);
}

namespace {
// lent_spec: frames * 16 bytes of speculation records the caller owns
// (the *_host entry point's staging), else per-call pooled scratch.
int demod_batch_impl(lphy_hip_ctx* c, const float* d_iq, size_t frames, size_t frame_samples,
                     uint16_t* d_syms, uint8_t* d_bytes, lphy_frame_meta* d_meta, int mode,
                     unsigned flags, hipStream_t st, void* lent_spec) {
    if (!c || !d_iq || !d_meta || !d_syms) return -EINVAL;
    if (mode < 0 || mode > 2) return -EINVAL;
#ifndef LPHY_TEST_PATHS
    if (flags & kTestFlags) return -EINVAL;  // comparison paths: test build only
#endif
    if ((flags & LPHY_F_DECODE) && !d_bytes) return -EINVAL;
    if (frames == 0) return 0;
    const size_t step = (size_t)c->N * c->osr;
    const size_t total = frame_samples / step;
    if (mode == LPHY_MODE_DEMODULATE) {
        // phy.cpp:190-194
        if (frame_samples % step != 0) return -EINVAL;
        if (total < 2) return -ERANGE;
    }
    if (mode == LPHY_MODE_DECHIRP_LORA_DEMODULATE && (c->osr != 1 || frame_samples % c->N)) return -EINVAL;
    HIP_OK(hipSetDevice(c->device));
    DemodArgs A{};
    A.iq = reinterpret_cast<const cf32*>(d_iq);
    A.tw = c->d_tw;
    A.down = c->d_down;
    A.win = c->window == LPHY_WINDOW_HANN ? c->d_win : nullptr;
    A.syms = d_syms;
    A.meta = d_meta;
    A.frames = frames;
    A.frame_samples = frame_samples;
    A.total_syms = total;
    A.out_per_frame = lphy_hip_syms_per_frame(c, frame_samples, mode);
    A.osr = (int)c->osr;
    A.power_scale = c->power_scale;
    A.mode = mode;
    A.no_scratch = (flags & LPHY_F_NO_SCRATCH) ? 1 : 0;
    A.exact_rotation = (flags & LPHY_F_EXACT_ROTATION) ? 1 : 0;
    A.counters = c->d_counters;
    A.spec = (mode != LPHY_MODE_DEMODULATE && !A.no_scratch && !(flags & LPHY_F_SCAN_FIRST)) ? 1 : 0;
    A.debug_recheck = (flags & LPHY_F_DEBUG_RECHECK) ? 1 : 0;
    const size_t est_syms = mode == LPHY_MODE_DEMODULATE ? 2 : (total < 2 ? total : 2);
    A.est_units = (int)(est_syms * c->osr);
    // 32-bit symbol / sample bookkeeping in the kernels
    if (frames > 0x7fffffffULL || frames * (total ? total : 1) >= 0xffffffffULL ||
        frame_samples >= 0x7fffffffULL)
        return -ERANGE;
    const unsigned stages = flags & (LPHY_F_STAGE_PROLOGUE | LPHY_F_STAGE_SYMBOLS | LPHY_F_STAGE_FINAL);
    const bool all = stages == 0;
    // one fused launch for prologue + symbols when the frame shape allows it
    // (see k_frames); selecting exactly those two stages runs it alone
    const unsigned both = LPHY_F_STAGE_PROLOGUE | LPHY_F_STAGE_SYMBOLS;
    // (Measured alternative: the separate kernels pipelined over chunks on
    // two streams, prologue of chunk c+1 beside the symbol kernel of chunk
    // c: the co-running kernels slowed each other ~2x, 1.1x slower overall.)
    // (LPHY_F_FRAMES_KERNEL, test build: k_frames where k_wave would run -
    // SF 7-10; the certificate tests on k_frames)
    const bool wfit = wave_fit(c->sf, c->osr, A.est_units, total, mode, A) &&
                      !(flags & LPHY_F_FRAMES_KERNEL);
    const bool fused = (all || (stages & both) == both) && !(flags & LPHY_F_UNFUSED) &&
                       frames >= fused_min_frames(c) && (frames_fit(c->sf, c->osr, A.est_units, total) || wfit);
    A.wave = fused && (c->sf >= 11 || wfit) ? 1 : 0;
    // SF 11-12 separate launches, modes 1/2: the speculative normalisation
    // of k_frames across workgroups (k_maxabs scans the two estimate
    // symbols, k_demod folds the rest, k_post closes each frame); needs the
    // prologue, the symbols and the fix-up in this one call
    // (per call, in the caller's stream order: released after this call's
    // last kernel, k_post, which is launched below while `spec` is in scope)
    StreamScratch spec(st, lent_spec);
    if (!fused && A.spec && c->sf >= 11 && c->osr == 1 && !A.exact_rotation && total >= 2 &&
        (all || (stages & both) == both)) {
        if (int rc = spec.get(frames * sizeof(uint4))) return rc;
        A.spec_big = static_cast<uint4*>(spec.p);
    }
    int rc = fused ? launch_frames(c->sf, A, st)
                   : launch_demod(c->sf, A, st, all || (stages & LPHY_F_STAGE_PROLOGUE),
                                  all || (stages & LPHY_F_STAGE_SYMBOLS));
    if (rc) return rc;
    // exact re-run of flagged frames (part of the symbols stage) and the
    // per-frame finalisation, in one launch
    const bool fix = all || (stages & LPHY_F_STAGE_SYMBOLS);
    const bool fin = all || (stages & LPHY_F_STAGE_FINAL);
    if (!fix && !fin) return 0;
    FinalArgs F{};
    F.syms = d_syms;
    F.bytes = d_bytes;
    F.meta = d_meta;
    F.frames = frames;
    F.nsyms = A.out_per_frame;
    F.sym_stride = A.out_per_frame;
    F.shift = c->sf > 4 ? (int)c->sf - 4 : 0;
    F.decode = (flags & LPHY_F_DECODE) ? 1 : 0;
    F.set_sync = 1;
    return launch_post(c->sf, mode, A, F, fix, fin, st);
}
}  // namespace

#ifdef LPHY_PROFILE_PHASES
// experiments only: read and clear the kernels' per-phase clock sums (8)
int lphy_hip_phase_cycles(lphy_hip_ctx* c, unsigned long long* out8) {
    if (!c || !out8) return -EINVAL;
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(out8, c->d_counters + kCtrClocks, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    HIP_OK(hipMemset(c->d_counters + kCtrClocks, 0, 8 * sizeof(unsigned long long)));
    return 0;
}
#endif

int lphy_hip_decode_batch(lphy_hip_ctx* c, const uint16_t* d_syms, size_t frames,
                          size_t syms_per_frame, uint8_t* d_bytes, lphy_frame_meta* d_meta,
                          void* stream) {
    if (!c || !d_syms || !d_bytes || !d_meta) return -EINVAL;
    if (syms_per_frame & 1) return -EINVAL;
    if (frames == 0) return 0;
    HIP_OK(hipSetDevice(c->device));
    FinalArgs F{};
    F.syms = d_syms;
    F.bytes = d_bytes;
    F.meta = d_meta;
    F.frames = frames;
    F.nsyms = syms_per_frame;
    F.sym_stride = syms_per_frame;
    F.shift = 0;
    F.decode = 1;
    F.set_sync = 0;
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)((frames + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, F);
    HIP_OK(hipGetLastError());
    return 0;
}

int lphy_hip_estimate_batch(lphy_hip_ctx* c, const float* d_iq, size_t frames,
                            size_t frame_samples, size_t est_samples,
                            lphy_frame_meta* d_meta, void* stream) {
    if (!c || !d_iq || !d_meta) return -EINVAL;
    const size_t step = (size_t)c->N * c->osr;
    const size_t syms = est_samples / step;
    if (syms == 0 || frames == 0) return 0;  // phy.cpp:87,91: nothing written
    if (syms * c->osr > 0x7fffffffULL) return -ERANGE;
    HIP_OK(hipSetDevice(c->device));
    DemodArgs A{};
    A.iq = reinterpret_cast<const cf32*>(d_iq);
    A.tw = c->d_tw;
    A.down = c->d_down;
    A.win = c->window == LPHY_WINDOW_HANN ? c->d_win : nullptr;
    A.meta = d_meta;
    A.frames = frames;
    A.frame_samples = frame_samples;
    A.total_syms = frame_samples / step;
    A.osr = (int)c->osr;
    A.power_scale = c->power_scale;
    A.mode = LPHY_MODE_DEMODULATE;
    A.est_units = (int)(syms * c->osr);
    A.counters = c->d_counters;
    const SfOps* o = sf_ops(c->sf);
    return o ? o->estimate(A, (hipStream_t)stream) : -EINVAL;
}

namespace {
// compensate_offsets (phy.cpp:150-180) on device samples.  The rotation is
// elementwise and runs in place; only a time shift needs scratch (`lent`,
// when given, is count complex values the caller owns).
int compensate_impl(lphy_hip_ctx* c, float* d_iq, size_t count, float cfo, float time_offset,
                    hipStream_t st, void* lent) {
    // phy.cpp:159-160
    const float rate = -2.0f * kPi * cfo / (static_cast<float>(c->N) * static_cast<float>(c->osr));
    const unsigned blocks = (unsigned)((count + 255) / 256);
    cf32* x = reinterpret_cast<cf32*>(d_iq);
    const float r = std::round(time_offset);  // phy.cpp:167, x86 cvttss2si
    const long long off = (r >= -2147483648.0f && r < 2147483648.0f) ? (long long)(int)r
                                                                     : (long long)(int)0x80000000u;
    if (off == 0 || (unsigned long long)(off > 0 ? off : -off) >= count) {
        hipLaunchKernelGGL(k_comp_rotate, dim3(blocks), dim3(256), 0, st, x, x,
                           (unsigned long long)count, rate);
        HIP_OK(hipGetLastError());
        return 0;
    }
    StreamScratch scratch(st, lent);
    if (int rc = scratch.get(count * sizeof(cf32))) return rc;
    cf32* tmp = static_cast<cf32*>(scratch.p);
    hipLaunchKernelGGL(k_comp_rotate, dim3(blocks), dim3(256), 0, st, tmp, x, (unsigned long long)count, rate);
    hipLaunchKernelGGL(k_comp_shift, dim3(blocks), dim3(256), 0, st, x, tmp, (unsigned long long)count, off);
    HIP_OK(hipGetLastError());
    return 0;
}

// lora_modulate (LoRaMod.cpp:8-43) for `frames` frames; `lent` (optional)
// holds mod_scratch_bytes(): the per-symbol start phases, and below
// mod_walk_all_below symbols every sample's phase too.
constexpr size_t mod_walk_all_below = 4096;
#ifndef LPHY_MOD_FAST  // 0: the three-kernel few-symbol form only (A/B builds)
#define LPHY_MOD_FAST 1
#endif

struct ModFastLimits {
    size_t lds = 0;
};
const ModFastLimits& mod_fast_limits(int device);

// Which modulator form a call takes (modulate_impl): 0 the three-kernel or
// batch forms, 1 k_mod_fast with the f rows in LDS, 2 k_mod_fast's split
// form with the f rows in the phase buffer (GROWS: k_mod_fast<true, 1>,
// k_mod_cand, k_mod_fast<true, 3>).
int mod_form(const lphy_hip_ctx* c, size_t frames, size_t nsyms) {
    const size_t ns = nsyms + 2, nph = frames * ns;
    if (!LPHY_MOD_FAST || nph >= mod_walk_all_below || ns > (size_t)kModFastSyms) return 0;
    const size_t lds = ns * (((size_t)c->N * c->osr + 4) * sizeof(float) + kModFastWin);
    return lds <= mod_fast_limits(c->device).lds ? 1 : 2;
}

size_t mod_scratch_bytes(const lphy_hip_ctx* c, size_t frames, size_t nsyms) {
    const size_t nph = frames * (nsyms + 2);
    return align_up(nph * sizeof(float)) +
           (nph < mod_walk_all_below ? align_up(nph * (size_t)c->N * c->osr * sizeof(float)) : 0) +
           (mod_form(c, frames, nsyms) == 2
                ? align_up(frames * sizeof(ModFastG)) + align_up(frames * (size_t)kModFastSyms * kModFastWin)
                : 0);
}

// k_mod_fast's dynamic LDS limit on the context's device, found once per
// device: the device's LDS per workgroup less the kernel's static LDS
// (ModFastShared), and the kernel's attribute raised to it once, outside the
// per-packet path (the limit was a gfx950 constant, set per call).
const ModFastLimits& mod_fast_limits(int device) {
    static ModFastLimits lim[64];
    static std::once_flag once[64];
    const int d = device >= 0 && device < 64 ? device : 0;
    std::call_once(once[d], [d] {
        int cur = 0, per_block = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(d);
        (void)hipDeviceGetAttribute(&per_block, hipDeviceAttributeMaxSharedMemoryPerBlock, d);
        size_t stat = 0;
        hipFuncAttributes fa{};
        if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k_mod_fast<false>)) == hipSuccess)
            stat = fa.sharedSizeBytes;
        size_t avail = per_block > 0 && (size_t)per_block > stat ? (size_t)per_block - stat : 0;
        if (avail > kModFastLds) avail = kModFastLds;
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_mod_fast<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)avail) != hipSuccess)
            avail = std::min<size_t>(avail, size_t(64) << 10);  // the default limit stands
        lim[d].lds = avail;
        (void)hipSetDevice(cur);
    });
    return lim[d];
}

int modulate_impl(lphy_hip_ctx* c, const uint16_t* d_syms, size_t frames, size_t nsyms,
                  float* d_iq, float amplitude, uint8_t sync, hipStream_t st, void* lent) {
    ModArgs A{};
    A.syms = d_syms;
    A.iq = reinterpret_cast<cf32*>(d_iq);
    A.frames = frames;
    A.nsyms = nsyms;
    A.N = (int)c->N;
    A.osr = (int)c->osr;
    A.bws = (float)c->bw_hz / 125000.0f;
    A.ampl = std::max(-1.0f, std::min(1.0f, amplitude));  // LoRaMod.cpp:18
    A.sync = sync;
    A.slow = c->d_counters + kCtrModSerial;  // lphy_hip_test_counter(kCtrModSerial)
#ifdef LPHY_TEST_PATHS
    A.force_serial = c->mod_force_serial.load(std::memory_order_relaxed);
#endif
    const size_t nph = frames * (nsyms + 2);
    const size_t samples = nph * (size_t)c->N * c->osr;
    // few symbols: every sample's phase from the walk, then sample-parallel
    // sincos (a per-symbol pass would run a handful of threads N steps each)
    const bool walk_all = nph < mod_walk_all_below;
    const int form = mod_form(c, frames, nsyms);
    StreamScratch scratch(st, lent);
    if (int rc = scratch.get(mod_scratch_bytes(c, frames, nsyms))) return rc;
    A.phase0 = static_cast<float*>(scratch.p);
    A.phases = walk_all ? reinterpret_cast<float*>(static_cast<char*>(scratch.p) + align_up(nph * sizeof(float)))
                        : nullptr;
    if (form == 2) {
        char* g = static_cast<char*>(scratch.p) + align_up(nph * sizeof(float)) + align_up(samples * sizeof(float));
        A.mfg = reinterpret_cast<ModFastG*>(g);
        A.mft = reinterpret_cast<unsigned char*>(g + align_up(frames * sizeof(ModFastG)));
        A.blk = (int)(nsyms + 2);  // (k_mod_fast<true>'s interleaved rows, read so by k_mod_sincos)
    }
    // ... then the walk by candidate windows and a chain of lookups
    // (k_mod_fast): with the f rows in LDS when they fit there beside the
    // kernel's static LDS (up to SF 9 at 66 symbols), else in A.phases
    // (k_mod_fast<true, 1> / k_mod_cand / k_mod_fast<true, 3>), then the sincos
    const int stride = (int)(c->N * c->osr) + 4;
    const size_t ns = nsyms + 2;
    const size_t lds = ns * ((size_t)stride * sizeof(float) + kModFastWin);
    if (form == 1 || form == 2) {
        if (form == 1) {
            hipLaunchKernelGGL((k_mod_fast<false>), dim3((unsigned)frames), dim3(kModFastThreads), lds, st, A, stride);
        } else {
            // (the candidate walks, 64 per symbol boundary, are 64x the work of
            // a row walk: across the GPU, between the two halves)
            const int step = (int)(c->N * c->osr);
            hipLaunchKernelGGL((k_mod_fast<true, 1>), dim3((unsigned)frames), dim3(kModFastThreads), 0, st, A, step);
            hipLaunchKernelGGL(k_mod_cand, dim3((unsigned)(frames * ((ns - 1 + 3) / 4))), dim3(256), 0, st, A);
            hipLaunchKernelGGL((k_mod_fast<true, 3>), dim3((unsigned)frames), dim3(kModFastThreads), 0, st, A, step);
        }
        hipLaunchKernelGGL(k_mod_sincos, dim3((unsigned)((samples + 255) / 256)), dim3(256), 0, st, A,
                           (unsigned long long)samples);
    } else if (walk_all) {
        hipLaunchKernelGGL(k_mod_freq, dim3((unsigned)((nph + 63) / 64)), dim3(64), 0, st, A);
        hipLaunchKernelGGL(k_mod_accumulate, dim3((unsigned)((frames + 63) / 64)), dim3(64), 0, st, A);
        hipLaunchKernelGGL(k_mod_sincos, dim3((unsigned)((samples + 255) / 256)), dim3(256), 0, st, A,
                           (unsigned long long)samples);
    } else {
        hipLaunchKernelGGL(k_mod_walk, dim3((unsigned)((frames + 63) / 64)), dim3(64), 0, st, A);
        hipLaunchKernelGGL(k_mod_samples, dim3((unsigned)((nph + 63) / 64)), dim3(64), 0, st, A);
    }
    HIP_OK(hipGetLastError());
    return 0;
}
}  // namespace

int lphy_hip_compensate(lphy_hip_ctx* c, float* d_iq, size_t count, float cfo,
                        float time_offset, void* stream) {
    if (!c || !d_iq) return -EINVAL;
    if (count == 0) return 0;
    HIP_OK(hipSetDevice(c->device));
    return compensate_impl(c, d_iq, count, cfo, time_offset, (hipStream_t)stream, nullptr);
}

int lphy_hip_modulate_batch(lphy_hip_ctx* c, const uint16_t* d_syms, size_t frames,
                            size_t nsyms, float* d_iq, float amplitude, uint8_t sync,
                            void* stream) {
    if (!c || !d_iq || (nsyms && !d_syms)) return -EINVAL;
    if (frames == 0) return 0;
    HIP_OK(hipSetDevice(c->device));
    return modulate_impl(c, d_syms, frames, nsyms, d_iq, amplitude, sync, (hipStream_t)stream,
                         nullptr);
}

int lphy_hip_sync(void* stream) {
    HIP_OK(hipStreamSynchronize((hipStream_t)stream));
    return 0;
}

int lphy_hip_recheck_count(lphy_hip_ctx* c, unsigned long long* out, int reset) {
    if (!c || !out) return -EINVAL;
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(out, c->d_counters + kCtrRecheck, sizeof(*out), hipMemcpyDeviceToHost));
    if (reset) HIP_OK(hipMemset(c->d_counters + kCtrRecheck, 0, sizeof(*out)));
    return 0;
}

#ifdef LPHY_TEST_PATHS
// Test build only (csrc/lphy_testing.h): the context's device counter `idx`
// (kCtrParseval: symbols the wave kernels certified by Parseval; kCtrModSerial:
// frames k_mod_fast walked serially).  Synchronises.
// Test build only: every k_mod_fast frame takes the serial walk (its
// fallback, otherwise reached only when a candidate chain leaves its windows).
int lphy_hip_test_mod_force_serial(lphy_hip_ctx* c, int on) {
    if (!c) return -EINVAL;
    c->mod_force_serial.store(on ? 1 : 0, std::memory_order_relaxed);
    return 0;
}

int lphy_hip_test_counter(lphy_hip_ctx* c, int idx, unsigned long long* out, int reset) {
    if (!c || !out || idx < 0 || idx >= kCounters) return -EINVAL;
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(out, c->d_counters + idx, sizeof(*out), hipMemcpyDeviceToHost));
    if (reset) HIP_OK(hipMemset(c->d_counters + idx, 0, sizeof(*out)));
    return 0;
}
#endif

int lphy_hip_bounds_violations(lphy_hip_ctx* c, unsigned long long* out, int reset) {
    if (!c || !out) return -EINVAL;
#ifdef LPHY_DEBUG_BOUNDS
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipDeviceSynchronize());
    unsigned long long total = 0;
    for (unsigned sf = 1; sf <= 12; ++sf) {
        const SfOps* o = sf_ops(sf);
        unsigned long long n = 0;
        if (o && o->violations) {
            if (int rc = o->violations(&n, reset)) return rc;
        }
        total += n;
    }
    *out = total;
    return 0;
#else
    *out = 0;
    return -ENOTSUP;
#endif
}

// ---- host-buffer convenience (synchronous) --------------------------------
// Each call runs on the context's own stream and waits for that stream only:
// host copies in (async, ordered on the stream), the kernels, host copies
// out, hipStreamSynchronize.  Staging comes from lphy_hip_ctx_reserve; a
// call larger than the reservation grows it (the only allocation after it).
namespace {
struct HostLayout {  // byte offsets in the staging buffer of one *_host call
    size_t iq = 0, syms = 0, bytes = 0, meta = 0, spec = 0, end = 0;
};

HostLayout demod_layout(const lphy_hip_ctx* c, size_t frames, size_t frame_samples, int mode) {
    const size_t per = lphy_hip_syms_per_frame(c, frame_samples, mode);
    HostLayout L;
    L.syms = align_up(frames * frame_samples * sizeof(cf32));
    L.bytes = L.syms + align_up(std::max<size_t>(1, frames * per) * sizeof(uint16_t));
    L.meta = L.bytes + align_up(std::max<size_t>(1, frames * (per / 2)));
    L.spec = L.meta + align_up(frames * sizeof(lphy_frame_meta));
    L.end = L.spec + align_up(frames * sizeof(uint4));
    return L;
}

// staging every *_host entry point needs for calls of up to `frames`
// frames of `frame_samples` samples (or one buffer of frames * frame_samples)
size_t host_stage_bytes(const lphy_hip_ctx* c, size_t frames, size_t frame_samples) {
    const size_t n = frames * frame_samples;
    const size_t syms = frame_samples / ((size_t)c->N * c->osr) + 2;
    size_t b = std::max(demod_layout(c, frames, frame_samples, LPHY_MODE_LORA_DEMODULATE).end,
                        demod_layout(c, frames, frame_samples, LPHY_MODE_DEMODULATE).end);
    b = std::max(b, 2 * align_up(n * sizeof(cf32)));                                      // compensate
    b = std::max(b, align_up(syms * sizeof(uint16_t)) + align_up(n * sizeof(cf32)) +
                        mod_scratch_bytes(c, 1, syms - 2));                               // modulate
    b = std::max(b, 3 * align_up(std::max<size_t>(1, frames * syms) * sizeof(uint16_t)));  // decode
    return b;
}

int ensure_host_stage(lphy_hip_ctx* c, size_t bytes) {
    if (c->stage_bytes >= bytes) return 0;
    // the old staging may still be read by this context's stream
    if (c->d_stage) HIP_OK(hipStreamSynchronize(c->stream));
    return ensure_stage(c, bytes);
}
}  // namespace

int lphy_hip_ctx_reserve(lphy_hip_ctx* c, size_t frames, size_t frame_samples) {
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_OK(hipSetDevice(c->device));
    return ensure_host_stage(c, host_stage_bytes(c, std::max<size_t>(frames, 1), frame_samples));
}

int lphy_hip_demod_host(lphy_hip_ctx* c, const float* h_iq, size_t frames,
                        size_t frame_samples, uint16_t* h_syms, uint8_t* h_bytes,
                        lphy_frame_meta* h_meta, int mode, unsigned flags) {
    if (!c || !h_iq || !h_meta) return -EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_OK(hipSetDevice(c->device));
    const size_t per = lphy_hip_syms_per_frame(c, frame_samples, mode);
    const HostLayout L = demod_layout(c, frames, frame_samples, mode);
    int rc = ensure_host_stage(c, L.end);
    if (rc) return rc;
    char* base = (char*)c->d_stage;
    float* d_iq = (float*)(base + L.iq);
    uint16_t* d_syms = (uint16_t*)(base + L.syms);
    uint8_t* d_bytes = (uint8_t*)(base + L.bytes);
    lphy_frame_meta* d_meta = (lphy_frame_meta*)(base + L.meta);
    hipStream_t st = c->stream;
    const size_t iq_n = frames * frame_samples * sizeof(cf32), meta_n = frames * sizeof(lphy_frame_meta);
    const size_t syms_n = frames * per * sizeof(uint16_t), bytes_n = frames * (per / 2);
    const bool decode = (flags & LPHY_F_DECODE) != 0;
    // pinned: IQ and the zeroed records in with one copy, symbols / bytes /
    // records out with one
    char* h = L.spec <= c->h_stage_bytes ? (char*)c->h_stage : nullptr;
    if (h) {
        std::memcpy(h + L.iq, h_iq, iq_n);
        std::memset(h + L.meta, 0, meta_n);
        HIP_OK(hipMemcpyAsync(base, h, L.spec, hipMemcpyHostToDevice, st));
    } else {
        HIP_OK(hipMemcpyAsync(d_iq, h_iq, iq_n, hipMemcpyHostToDevice, st));
        HIP_OK(hipMemsetAsync(d_meta, 0, meta_n, st));
    }
    rc = demod_batch_impl(c, d_iq, frames, frame_samples, d_syms, decode ? d_bytes : nullptr, d_meta, mode, flags,
                          st, base + L.spec);
    if (rc) {
        (void)hipStreamSynchronize(st);
        return rc;
    }
    if (h) {
        HIP_OK(hipMemcpyAsync(h + L.syms, base + L.syms, L.spec - L.syms, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        std::memcpy(h_meta, h + L.meta, meta_n);
        if (h_syms && per) std::memcpy(h_syms, h + L.syms, syms_n);
        if (h_bytes && decode && per / 2) std::memcpy(h_bytes, h + L.bytes, bytes_n);
        return 0;
    }
    HIP_OK(hipMemcpyAsync(h_meta, d_meta, meta_n, hipMemcpyDeviceToHost, st));
    if (h_syms && per) HIP_OK(hipMemcpyAsync(h_syms, d_syms, syms_n, hipMemcpyDeviceToHost, st));
    if (h_bytes && decode && per / 2) HIP_OK(hipMemcpyAsync(h_bytes, d_bytes, bytes_n, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    return 0;
}

int lphy_hip_decode_host(lphy_hip_ctx* c, const uint16_t* h_syms, size_t count,
                         uint8_t* h_bytes, lphy_frame_meta* h_meta) {
    if (!c || !h_syms || !h_bytes || !h_meta) return -EINVAL;
    if (count & 1) return -EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_OK(hipSetDevice(c->device));
    const size_t sym_b = align_up(std::max<size_t>(1, count) * sizeof(uint16_t));
    const size_t byte_b = align_up(std::max<size_t>(1, count / 2));
    const size_t meta_b = align_up(sizeof(lphy_frame_meta));
    int rc = ensure_host_stage(c, sym_b + byte_b + meta_b);
    if (rc) return rc;
    char* base = (char*)c->d_stage;
    uint16_t* d_syms = (uint16_t*)base;
    uint8_t* d_bytes = (uint8_t*)(base + sym_b);
    lphy_frame_meta* d_meta = (lphy_frame_meta*)(base + sym_b + byte_b);
    hipStream_t st = c->stream;
    const size_t end = sym_b + byte_b + meta_b;
    char* h = end <= c->h_stage_bytes ? (char*)c->h_stage : nullptr;
    if (h) {  // pinned: symbols and the zeroed record in, bytes and record out
        if (count) std::memcpy(h, h_syms, count * sizeof(uint16_t));
        std::memset(h + sym_b + byte_b, 0, sizeof(lphy_frame_meta));
        HIP_OK(hipMemcpyAsync(base, h, end, hipMemcpyHostToDevice, st));
    } else {
        if (count) HIP_OK(hipMemcpyAsync(d_syms, h_syms, count * sizeof(uint16_t), hipMemcpyHostToDevice, st));
        HIP_OK(hipMemsetAsync(d_meta, 0, sizeof(lphy_frame_meta), st));
    }
    rc = lphy_hip_decode_batch(c, d_syms, 1, count, d_bytes, d_meta, st);
    if (rc) {
        (void)hipStreamSynchronize(st);
        return rc;
    }
    if (h) {
        HIP_OK(hipMemcpyAsync(h + sym_b, base + sym_b, byte_b + meta_b, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        std::memcpy(h_meta, h + sym_b + byte_b, sizeof(lphy_frame_meta));
        if (count / 2) std::memcpy(h_bytes, h + sym_b, count / 2);
        return 0;
    }
    HIP_OK(hipMemcpyAsync(h_meta, d_meta, sizeof(lphy_frame_meta), hipMemcpyDeviceToHost, st));
    if (count / 2) HIP_OK(hipMemcpyAsync(h_bytes, d_bytes, count / 2, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    return 0;
}

int lphy_hip_estimate_host(lphy_hip_ctx* c, const float* h_iq, size_t count,
                           lphy_frame_meta* h_meta) {
    if (!c || !h_iq || !h_meta) return -EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_OK(hipSetDevice(c->device));
    const size_t iq_b = align_up(std::max<size_t>(1, count) * sizeof(cf32));
    const size_t meta_b = align_up(sizeof(lphy_frame_meta));
    int rc = ensure_host_stage(c, iq_b + meta_b);
    if (rc) return rc;
    char* base = (char*)c->d_stage;
    float* d_iq = (float*)base;
    lphy_frame_meta* d_meta = (lphy_frame_meta*)(base + iq_b);
    hipStream_t st = c->stream;
    HIP_OK(hipMemcpyAsync(d_iq, h_iq, count * sizeof(cf32), hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(d_meta, h_meta, sizeof(lphy_frame_meta), hipMemcpyHostToDevice, st));
    rc = lphy_hip_estimate_batch(c, d_iq, 1, count, count, d_meta, st);
    if (rc) {
        (void)hipStreamSynchronize(st);
        return rc;
    }
    HIP_OK(hipMemcpyAsync(h_meta, d_meta, sizeof(lphy_frame_meta), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    return 0;
}

int lphy_hip_compensate_host(lphy_hip_ctx* c, float* h_iq, size_t count, float cfo,
                             float time_offset) {
    if (!c || !h_iq) return -EINVAL;
    if (count == 0) return 0;
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_OK(hipSetDevice(c->device));
    const size_t iq_b = align_up(count * sizeof(cf32));
    int rc = ensure_host_stage(c, 2 * iq_b);
    if (rc) return rc;
    float* d = (float*)c->d_stage;
    hipStream_t st = c->stream;
    HIP_OK(hipMemcpyAsync(d, h_iq, count * sizeof(cf32), hipMemcpyHostToDevice, st));
    rc = compensate_impl(c, d, count, cfo, time_offset, st, (char*)c->d_stage + iq_b);
    if (rc) {
        (void)hipStreamSynchronize(st);
        return rc;
    }
    HIP_OK(hipMemcpyAsync(h_iq, d, count * sizeof(cf32), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    return 0;
}

int lphy_hip_modulate_host(lphy_hip_ctx* c, const uint16_t* h_syms, size_t nsyms,
                           float* h_iq, float amplitude, uint8_t sync) {
    if (!c || !h_iq || (nsyms && !h_syms)) return -EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_OK(hipSetDevice(c->device));
    const size_t samples = (nsyms + 2) * (size_t)c->N * c->osr;
    const size_t sym_b = align_up(std::max<size_t>(1, nsyms) * sizeof(uint16_t));
    const size_t iq_b = align_up(samples * sizeof(cf32));
    int rc = ensure_host_stage(c, sym_b + iq_b + mod_scratch_bytes(c, 1, nsyms));
    if (rc) return rc;
    char* base = (char*)c->d_stage;
    uint16_t* d_syms = (uint16_t*)base;
    float* d_iq = (float*)(base + sym_b);
    hipStream_t st = c->stream;
    char* h = sym_b + iq_b <= c->h_stage_bytes ? (char*)c->h_stage : nullptr;
    if (nsyms) {
        if (h) std::memcpy(h, h_syms, nsyms * sizeof(uint16_t));
        HIP_OK(hipMemcpyAsync(d_syms, h ? (const void*)h : (const void*)h_syms, nsyms * sizeof(uint16_t),
                              hipMemcpyHostToDevice, st));
    }
    rc = modulate_impl(c, d_syms, 1, nsyms, d_iq, amplitude, sync, st, base + sym_b + iq_b);
    if (rc) {
        (void)hipStreamSynchronize(st);
        return rc;
    }
    HIP_OK(hipMemcpyAsync(h ? (void*)(h + sym_b) : (void*)h_iq, d_iq, samples * sizeof(cf32), hipMemcpyDeviceToHost,
                          st));
    HIP_OK(hipStreamSynchronize(st));
    if (h) std::memcpy(h_iq, h + sym_b, samples * sizeof(cf32));
    return 0;
}

}  // extern "C"
