// lora_phy:: C++17 API (include/lora_phy/phy.hpp) on top of the MI355X C ABI
// (include/lphy_hip.h).  Argument validation, return codes and workspace side
// effects follow the reference (file:line on each function); the numerical
// work — offset estimation, rotation, FFT, argmax, decode, modulation — runs
// on the GPU.  There is no CPU fallback: if no HIP device is usable the
// demodulation entry points fail with -ENODEV.
//
// GPU state follows the reference's ownership (API_SPEC.md:9-14,136-140):
//   * every workspace gets a context of its own at init() / lora_demod_init()
//     - its own stream and host-call staging, sized there, over constant
//     tables (twiddles, down-chirp, window) shared per sf/bw/window - so
//     workspaces used from different threads never wait for each other and
//     a call allocates nothing (unless it exceeds what init reserved);
//   * the reference's stateless free functions (lora_decode, lora_modulate)
//     use a context per calling thread, created by that thread's first
//     init() / lora_demod_init() (or its first call);
//   * the shared tables are the one process-wide cache (read-only); a freed
//     workspace's context goes back to a per-configuration pool for the
//     next init() (no device allocation on workspace churn).
#include <lora_phy/phy.hpp>
#include <lphy_hip.h>

#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <tuple>
#include <unordered_map>
#include <vector>

extern "C" int lphy_hip_ctx_set_osr(lphy_hip_ctx* c, unsigned osr);  // internal (lphy_hip.hip)

namespace lora_phy {
namespace {

using cf = std::complex<float>;

int device_index() {
    const char* e = std::getenv("LPHY_DEVICE");
    return e ? std::atoi(e) : 0;
}

// Symbols per call the high-level API's staging is sized for at init()
// (a 127-byte payload and its 2 sync symbols); larger calls grow it once.
constexpr size_t kReserveSymbols = 256 + 2;

// The shared constant tables: one base context per (sf, bw, window), never
// used for calls itself.
lphy_hip_ctx* base_ctx(unsigned sf, unsigned bw_hz, int window, int* err) {
    static std::mutex mu;
    static std::map<std::tuple<unsigned, unsigned, int>, lphy_hip_ctx*> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_tuple(sf, bw_hz, window);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    lphy_hip_ctx* c = nullptr;
    int rc = lphy_hip_ctx_create(&c, device_index(), sf, bw_hz, 1, window);
    if (rc) {
        if (err) *err = rc;
        return nullptr;
    }
    cache[key] = c;
    return c;
}

// Contexts of freed workspaces (and of ended threads) wait here, per
// (sf, bw, window), for the next init() / lora_demod_init() of that
// configuration: a workspace churn costs no device allocation after the
// first, and the device memory is held until the process exits (at most
// the peak number of live workspaces' contexts).  Never destroyed, like
// the table cache, so no HIP call runs during static teardown.
using CtxKey = std::tuple<unsigned, unsigned, int>;
struct CtxPool {
    std::mutex mu;
    std::map<CtxKey, std::vector<lphy_hip_ctx*>> idle;
    std::unordered_map<const lphy_hip_ctx*, CtxKey> key_of;
};
CtxPool& ctx_pool() {
    static CtxPool* p = new CtxPool;
    return *p;
}

void release_ctx(lphy_hip_ctx* c) {
    if (!c) return;
    CtxPool& p = ctx_pool();
    std::lock_guard<std::mutex> lk(p.mu);
    auto it = p.key_of.find(c);
    if (it == p.key_of.end()) return;  // not ours
    p.idle[it->second].push_back(c);
}

// A context of one's own over the shared tables, staging reserved for
// `samples` samples per call.
lphy_hip_ctx* own_ctx(unsigned sf, unsigned bw_hz, unsigned osr, int window, size_t samples, int* err) {
    const CtxKey key = std::make_tuple(sf, bw_hz, window);
    lphy_hip_ctx* c = nullptr;
    {
        CtxPool& p = ctx_pool();
        std::lock_guard<std::mutex> lk(p.mu);
        auto it = p.idle.find(key);
        if (it != p.idle.end() && !it->second.empty()) {
            c = it->second.back();
            it->second.pop_back();
        }
    }
    int rc = 0;
    if (c) {
        rc = lphy_hip_ctx_set_osr(c, osr ? osr : 1u);
    } else {
        lphy_hip_ctx* b = base_ctx(sf, bw_hz, window, err);
        if (!b) return nullptr;
        rc = lphy_hip_ctx_share(&c, b, osr ? osr : 1u);
        if (!rc) {
            CtxPool& p = ctx_pool();
            std::lock_guard<std::mutex> lk(p.mu);
            p.key_of.emplace(c, key);
        }
    }
    if (!rc) rc = lphy_hip_ctx_reserve(c, 1, samples);
    if (rc) {
        release_ctx(c);
        if (err) *err = rc;
        return nullptr;
    }
    return c;
}

// Per-thread contexts of the stateless free functions, keyed by
// (sf, bw, osr); freed when the thread ends.
struct ThreadCtx {
    std::map<std::tuple<unsigned, unsigned, unsigned>, lphy_hip_ctx*> m;
    ~ThreadCtx() {
        for (auto& kv : m) release_ctx(kv.second);
    }
};
thread_local ThreadCtx t_ctx;

lphy_hip_ctx* thread_ctx(unsigned sf, unsigned bw_hz, unsigned osr, int* err) {
    auto key = std::make_tuple(sf, bw_hz, osr);
    auto it = t_ctx.m.find(key);
    if (it != t_ctx.m.end()) return it->second;
    lphy_hip_ctx* c = own_ctx(sf, bw_hz, osr, LPHY_WINDOW_NONE, kReserveSymbols * (size_t(1) << sf) * osr, err);
    if (c) t_ctx.m[key] = c;
    return c;
}

// the decoder's context (any SF: decode only reads symbols)
lphy_hip_ctx* decode_ctx(int* err) { return thread_ctx(7, 125000, 1, err); }

// lora_workspace -> its context (the reference struct has no room for it).
// Lookups take a shared lock only; init() replaces the entry.
// The reference has no free function for lora_workspace, so an application
// that heap-allocates a workspace per session would otherwise leave a
// context (stream, staging, pinned mirror) behind for every address it ever
// passed to init().  So at most kMaxWsContexts workspaces get a context of
// their own; the workspaces beyond them are not remembered and share one
// context per (sf, bw, osr, window) (shared_ctx: calls on it are serialised
// by the context's mutex, so they are correct, just not concurrent).  Both
// the map and the number of contexts stay bounded.
constexpr size_t kMaxWsContexts = 64;
std::shared_mutex ws_mu;
std::unordered_map<const lora_workspace*, lphy_hip_ctx*> ws_map;

int window_flag(window_type k, const void* buf);

// The shared context of a configuration (made once, never released).
lphy_hip_ctx* shared_ctx(unsigned sf, unsigned bw_hz, unsigned osr, int window, int* err) {
    static std::mutex mu;
    static std::map<std::tuple<unsigned, unsigned, unsigned, int>, lphy_hip_ctx*> m;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_tuple(sf, bw_hz, osr, window);
    auto it = m.find(key);
    if (it != m.end()) return it->second;
    lphy_hip_ctx* c = own_ctx(sf, bw_hz, osr, window, kReserveSymbols * (size_t(1) << sf) * osr, err);
    if (c) m.emplace(key, c);
    return c;
}

bool ws_has_room(const lora_workspace* ws) {
    std::shared_lock<std::shared_mutex> lk(ws_mu);
    return ws_map.count(ws) != 0 || ws_map.size() < kMaxWsContexts;
}

lphy_hip_ctx* ws_ctx(const lora_workspace* ws, unsigned sf, unsigned osr, int* err) {
    {
        std::shared_lock<std::shared_mutex> lk(ws_mu);
        auto it = ws_map.find(ws);
        if (it != ws_map.end()) return it->second;
    }
    const unsigned bw = static_cast<unsigned>(ws->bw);
    const int win = window_flag(ws->window_kind, ws->window);
    if (!ws_has_room(ws)) return shared_ctx(sf, bw, osr, win, err);
    // a workspace init() did not set up here (e.g. a copy): make its context now
    lphy_hip_ctx* c = own_ctx(sf, bw, osr, win, kReserveSymbols * (size_t(1) << sf) * osr, err);
    if (!c) return nullptr;
    std::unique_lock<std::shared_mutex> lk(ws_mu);
    auto it = ws_map.find(ws);
    if (it != ws_map.end()) {  // another thread got there first
        release_ctx(c);
        return it->second;
    }
    if (ws_map.size() >= kMaxWsContexts) {  // the last place went meanwhile
        release_ctx(c);
        lk.unlock();
        return shared_ctx(sf, bw, osr, win, err);
    }
    ws_map.emplace(ws, c);
    return c;
}

lphy_hip_ctx* ws_ctx_if_any(const lora_workspace* ws) {
    std::shared_lock<std::shared_mutex> lk(ws_mu);
    auto it = ws_map.find(ws);
    return it != ws_map.end() ? it->second : nullptr;
}

// lora_demod_workspace keeps its context pointer in the reference layout's
// fft_buf (8 bytes, the storage the reference placement-constructs its FFT
// object into); ws->fft == ws->fft_buf marks it valid.
lphy_hip_ctx* demod_ws_ctx(const lora_demod_workspace* ws) {
    if (ws->fft != static_cast<const void*>(ws->fft_buf)) return nullptr;
    lphy_hip_ctx* c = nullptr;
    std::memcpy(&c, ws->fft_buf, sizeof c);
    return c;
}

unsigned deduce_sf(const lora_workspace* ws) {  // phy.cpp:14-19
    unsigned sf = 0;
    size_t n = static_cast<size_t>(ws->plan_fwd.nfft);
    while ((size_t(1) << sf) < n) ++sf;
    return sf;
}

unsigned get_osr(const lora_workspace* ws) { return ws->osr ? ws->osr : 1u; }  // phy.cpp:21-23

// kissfft.hh:71-98 — the plan record callers can inspect.
void fill_plan(kissfft_plan<float>& plan, int nfft, bool inverse) {
    plan.nfft = nfft;
    plan.inverse = inverse;
    const float phinc = (inverse ? 2 : -2) * std::acos((float)-1) / nfft;
    for (int i = 0; i < nfft && i < (int)kissfft_utils::KISSFFT_MAX_N; ++i)
        plan.twiddles[i] = std::exp(std::complex<float>(0, i * phinc));
    int n = nfft, p = 4;
    plan.stages = 0;
    do {
        while (n % p) {
            p = p == 4 ? 2 : (p == 2 ? 3 : p + 2);
            if (p * p > n) p = n;
        }
        n /= p;
        plan.stageRadix[plan.stages] = p;
        plan.stageRemainder[plan.stages] = n;
        ++plan.stages;
    } while (n > 1);
}

void fill_window(float* w, size_t N, window_type kind) {  // LoRaDemod.cpp:16-24
    for (size_t i = 0; i < N; ++i)
        w[i] = kind == window_type::window_hann
                   ? 0.5f - 0.5f * std::cos(2.0f * PI * static_cast<float>(i) /
                                            (static_cast<float>(N) - 1.0f))
                   : 1.0f;
}

int window_flag(window_type k, const void* buf) {
    return (k != window_type::window_none && buf) ? LPHY_WINDOW_HANN : LPHY_WINDOW_NONE;
}

}  // namespace

// ---------------------------------------------------------------------------
// High-level API
// ---------------------------------------------------------------------------
int init(lora_workspace* ws, const lora_params* cfg) {  // phy.cpp:27-52
    if (!ws || !cfg) return -EINVAL;
    if (cfg->sf < 1 || cfg->sf > 12) return -EINVAL;  // reference overflows its 4096 plan
    const int N = 1 << cfg->sf;
    fill_plan(ws->plan_fwd, N, false);
    fill_plan(ws->plan_inv, N, true);
    ws->metrics = {};
    ws->osr = cfg->osr ? cfg->osr : 1u;
    ws->bw = cfg->bw;
    ws->sync_word = cfg->sync_word;
    ws->window_kind = cfg->window;
    if (ws->window_kind != window_type::window_none && !ws->window) return -ENOMEM;
    if (ws->window) fill_window(ws->window, (size_t)N, ws->window_kind);
    // the workspace's GPU context and staging, so later calls allocate
    // nothing (the reference allocates nothing after init, API_SPEC.md:9-14)
    // (beyond kMaxWsContexts workspaces: the configuration's shared context,
    // made here so that calls still allocate nothing)
    int err = 0;
    const unsigned bw = static_cast<unsigned>(ws->bw);
    const int win = window_flag(ws->window_kind, ws->window);
    lphy_hip_ctx* c = ws_has_room(ws) ? own_ctx(cfg->sf, bw, ws->osr, win, kReserveSymbols * size_t(N) * ws->osr, &err)
                                      : nullptr;
    if (c) {
        std::unique_lock<std::shared_mutex> lk(ws_mu);
        auto it = ws_map.find(ws);
        if (it != ws_map.end()) {
            release_ctx(it->second);  // re-init: the new configuration wins
            it->second = c;
        } else if (ws_map.size() < kMaxWsContexts) {
            ws_map.emplace(ws, c);
        } else {
            release_ctx(c);
            c = nullptr;
        }
    }
    if (!c) (void)shared_ctx(cfg->sf, bw, ws->osr, win, &err);
    (void)decode_ctx(&err);  // this thread's decoder context
    return 0;
}

void reset(lora_workspace* ws) {  // phy.cpp:54-56
    if (ws) ws->metrics = {};
}

ssize_t encode(lora_workspace* ws, const uint8_t* payload, size_t payload_len,
               uint16_t* symbols, size_t symbol_cap) {  // phy.cpp:58-66
    if (!ws || !payload || !symbols) return -EINVAL;
    if (2 * payload_len > symbol_cap) return -ERANGE;  // checked before writing
    return static_cast<ssize_t>(lora_encode(payload, payload_len, symbols, deduce_sf(ws)));
}

ssize_t decode(lora_workspace* ws, const uint16_t* symbols, size_t symbol_count,
               uint8_t* payload, size_t payload_cap) {  // phy.cpp:245-261
    if (!ws || !symbols || !payload) return -EINVAL;
    if (symbol_count % 2) return -EINVAL;  // LoRaDecoder.cpp:10
    if (symbol_count / 2 > payload_cap) return -ERANGE;  // checked before writing
    // decode reads symbols only, so a workspace init() never saw (the
    // reference's decode needs none of its fields) takes this thread's
    // decoder context rather than one made for its unset SF
    int err = -ENODEV;
    lphy_hip_ctx* c = ws_ctx_if_any(ws);
    if (!c) c = decode_ctx(&err);
    if (!c) return err;
    lphy_frame_meta m{};
    int rc = lphy_hip_decode_host(c, symbols, symbol_count, payload, &m);
    if (rc) return rc;
    ws->metrics.crc_ok = m.crc_ok != 0;
    return static_cast<ssize_t>(symbol_count / 2);
}

ssize_t modulate(lora_workspace* ws, const uint16_t* symbols, size_t symbol_count,
                 std::complex<float>* iq, size_t iq_cap) {  // phy.cpp:68-79
    if (!ws || !symbols || !iq) return -EINVAL;
    const unsigned sf = deduce_sf(ws), osr = get_osr(ws);
    const size_t produced = (symbol_count + 2) * (size_t(1) << sf) * osr;
    if (produced > iq_cap) return -ERANGE;  // checked before writing
    size_t r = lora_modulate(symbols, symbol_count, iq, sf, osr, ws->bw, 1.0f, ws->sync_word);
    return r == produced ? static_cast<ssize_t>(r) : -EIO;
}

void estimate_offsets(lora_workspace* ws, const std::complex<float>* samples,
                      size_t sample_count) {  // phy.cpp:81-148
    if (!ws || !samples || sample_count == 0) return;
    const unsigned sf = deduce_sf(ws), osr = get_osr(ws);
    const size_t step = (size_t(1) << sf) * osr;
    if (sample_count / step == 0) return;
    lphy_hip_ctx* c = ws_ctx(ws, sf, osr, nullptr);
    if (!c) return;
    lphy_frame_meta m{};
    if (lphy_hip_estimate_host(c, reinterpret_cast<const float*>(samples), sample_count, &m)) return;
    ws->metrics.cfo = m.cfo;
    ws->metrics.time_offset = m.time_offset;
}

void compensate_offsets(const lora_workspace* ws, std::complex<float>* samples,
                        size_t sample_count) {  // phy.cpp:150-180
    if (!ws || !samples || sample_count == 0) return;
    const unsigned sf = deduce_sf(ws), osr = get_osr(ws);
    lphy_hip_ctx* c = ws_ctx(ws, sf, osr, nullptr);
    if (!c) return;
    (void)lphy_hip_compensate_host(c, reinterpret_cast<float*>(samples), sample_count,
                                   ws->metrics.cfo, ws->metrics.time_offset);
}

ssize_t demodulate(lora_workspace* ws, const std::complex<float>* iq, size_t sample_count,
                   uint16_t* symbols, size_t symbol_cap) {  // phy.cpp:182-243
    if (!ws || !iq || !symbols) return -EINVAL;
    const unsigned sf = deduce_sf(ws), osr = get_osr(ws);
    const size_t step = (size_t(1) << sf) * osr;
    if (sample_count % step != 0) return -EINVAL;
    const size_t total = sample_count / step;
    if (total < 2) return -ERANGE;
    const size_t num = total - 2;
    if (num > symbol_cap) return -ERANGE;
    int err = -ENODEV;
    lphy_hip_ctx* c = ws_ctx(ws, sf, osr, &err);
    if (!c) return err;
    lphy_frame_meta m{};
    int rc = lphy_hip_demod_host(c, reinterpret_cast<const float*>(iq), 1, sample_count,
                                 symbols, nullptr, &m, LPHY_MODE_DEMODULATE, 0);
    if (rc) return rc;
    ws->metrics.cfo = m.cfo;
    ws->metrics.time_offset = m.time_offset;
    ws->sync_word = m.sync_word;  // phy.cpp:239-241
    return static_cast<ssize_t>(num);
}

const lora_metrics* get_last_metrics(const lora_workspace* ws) {  // phy.cpp:263-266
    if (!ws) return nullptr;
    return &ws->metrics;
}

int demodulate_batch(const lora_workspace* ws, const std::complex<float>* iq, size_t frames,
                     size_t frame_samples, uint16_t* symbols, uint8_t* payloads,
                     uint8_t* sync_words, int32_t* status) {
    if (!ws || !iq || !symbols) return -EINVAL;
    const unsigned sf = deduce_sf(ws), osr = get_osr(ws);
    int err = -ENODEV;
    lphy_hip_ctx* c = ws_ctx(ws, sf, osr, &err);
    if (!c) return err;
    std::vector<lphy_frame_meta> m(frames);
    int rc = lphy_hip_demod_host(c, reinterpret_cast<const float*>(iq), frames, frame_samples,
                                 symbols, payloads, m.data(), LPHY_MODE_DEMODULATE,
                                 payloads ? static_cast<unsigned>(LPHY_F_DECODE) : 0u);
    if (rc) return rc;
    for (size_t f = 0; f < frames; ++f) {
        if (sync_words) sync_words[f] = m[f].sync_word;
        if (status) status[f] = m[f].status;
    }
    return 0;
}

// ---------------------------------------------------------------------------
// Legacy API
// ---------------------------------------------------------------------------
void lora_demod_init(lora_demod_workspace* ws, unsigned sf, window_type win,
                     std::complex<float>* scratch, size_t max_samples) {  // LoRaDemod.cpp:11-33
    if (lphy_hip_ctx* old = demod_ws_ctx(ws)) release_ctx(old);  // re-init without free
    ws->N = size_t(1) << sf;
    ws->window_kind = win;
    fill_window(ws->window, ws->N, win);
    fill_plan(ws->fft_plan, (int)ws->N, false);
    // the workspace's GPU context, its staging sized for max_samples (the
    // scratch length the reference is given for the calls to come; without
    // one, kReserveSymbols symbols), kept where the reference constructs its
    // FFT object; no context (no device) leaves nullptr there and the calls
    // return -ENODEV
    int err = 0;
    lphy_hip_ctx* c = sf >= 1 && sf <= 12
                          ? own_ctx(sf, 125000, 1,
                                    win != window_type::window_none ? LPHY_WINDOW_HANN : LPHY_WINDOW_NONE,
                                    max_samples ? max_samples : kReserveSymbols * ws->N, &err)
                          : nullptr;
    std::memcpy(ws->fft_buf, &c, sizeof c);
    ws->fft = ws->fft_buf;          // non-null "constructed" markers
    ws->detector = ws->detector_buf;
    ws->scratch = scratch;
    ws->scratch_len = max_samples;
    (void)decode_ctx(&err);  // this thread's lora_decode context
}

void lora_demod_free(lora_demod_workspace* ws) {  // LoRaDemod.cpp:35-48
    if (lphy_hip_ctx* c = demod_ws_ctx(ws)) release_ctx(c);
    std::memset(ws->fft_buf, 0, sizeof ws->fft_buf);
    ws->detector = nullptr;
    ws->fft = nullptr;
    ws->N = 0;
    ws->scratch = nullptr;
    ws->scratch_len = 0;
}

size_t lora_modulate(const uint16_t* symbols, size_t symbol_count, std::complex<float>* out,
                     unsigned sf, unsigned osr, bandwidth bw, float amplitude,
                     uint8_t sync) {  // LoRaMod.cpp:8-43
    const size_t produced = (symbol_count + 2) * (size_t(1) << sf) * osr;
    if (osr == 0 || sf < 1 || sf > 12) return 0;
    lphy_hip_ctx* c = thread_ctx(sf, static_cast<unsigned>(bw), osr, nullptr);
    if (!c) return 0;
    if (lphy_hip_modulate_host(c, symbols, symbol_count, reinterpret_cast<float*>(out),
                               amplitude, sync))
        return 0;
    return produced;
}

ssize_t lora_demodulate(lora_demod_workspace* ws, const std::complex<float>* samples,
                        size_t sample_count, uint16_t* out_symbols, unsigned osr,
                        uint8_t* out_sync) {  // LoRaDemod.cpp:50-197
    if (!ws || ws->N == 0 || osr == 0) return -EINVAL;
    lphy_hip_ctx* c = demod_ws_ctx(ws);
    if (!c) return -ENODEV;
    if (int rc = lphy_hip_ctx_set_osr(c, osr)) return rc;  // the workspace's own context
    const bool scratch_ok = ws->scratch && ws->scratch_len >= sample_count;
    const size_t total = sample_count / (ws->N * osr);
    lphy_frame_meta m{};
    int rc = lphy_hip_demod_host(c, reinterpret_cast<const float*>(samples), 1, sample_count,
                                 out_symbols, nullptr, &m, LPHY_MODE_LORA_DEMODULATE,
                                 scratch_ok ? 0u : static_cast<unsigned>(LPHY_F_NO_SCRATCH));
    if (rc) return rc;
    if (m.status) return m.status;  // -ERANGE: rescale needed, no scratch (:69-71)
    ws->metrics.cfo = m.cfo;
    ws->metrics.time_offset = m.time_offset;
    if (out_sync) *out_sync = m.have_sync ? m.sync_word : 0;
    return total >= 2 ? static_cast<ssize_t>(total - 2) : static_cast<ssize_t>(total);
}

size_t lora_encode(const uint8_t* bytes, size_t byte_count, uint16_t* out_symbols,
                   unsigned /*sf*/) {  // LoRaEncoder.cpp:6-18 (producer, host)
    auto h84 = [](unsigned x) -> uint16_t {  // LoRaCodes.hpp:229-242
        const unsigned d0 = x & 1, d1 = (x >> 1) & 1, d2 = (x >> 2) & 1, d3 = (x >> 3) & 1;
        return static_cast<uint16_t>((x & 0xf) | (d0 ^ d1 ^ d2) << 4 | (d1 ^ d2 ^ d3) << 5 |
                                     (d0 ^ d1 ^ d3) << 6 | (d0 ^ d2 ^ d3) << 7);
    };
    size_t k = 0;
    for (size_t i = 0; i < byte_count; ++i) {
        out_symbols[k++] = h84(bytes[i] >> 4);
        out_symbols[k++] = h84(bytes[i] & 0x0f);
    }
    return k;
}

ssize_t lora_decode(const uint16_t* symbols, size_t symbol_count,
                    uint8_t* out_bytes) {  // LoRaDecoder.cpp:7-21
    if (symbol_count % 2 != 0) return -EINVAL;
    if (symbol_count == 0) return 0;
    int err = -ENODEV;
    lphy_hip_ctx* c = decode_ctx(&err);
    if (!c) return err;
    lphy_frame_meta m{};
    int rc = lphy_hip_decode_host(c, symbols, symbol_count, out_bytes, &m);
    if (rc) return rc;
    return static_cast<ssize_t>(symbol_count / 2);
}

}  // namespace lora_phy
