// lora_phy:: API transcript probe (TEST INFRASTRUCTURE).
//
// One source, two builds:
//   * against the drop-in (include/ + liblora_phy_amd.so, GPU behind the
//     C ABI) — built by tests/test_gpu_cxx_api.py on the GPU box;
//   * against the reference library compiled from /root/reference's own
//     sources (oracle/Makefile target `probe`, CPU) — prebuilt here, travels
//     as oracle/_ref/lora_phy_api_probe_ref.
// Each build prints a transcript of return codes, symbols, sync words,
// metrics (float bits) and payload bytes over the scenarios the reference's
// own tests cover (error_code, roundtrip, no_alloc, e2e_chain, bit_exact,
// equal_power_bin, scratch_buffer_error, odd_symbol_count, sync_word) plus
// impaired frames; the test asserts the two transcripts are identical.
// Buffers are always large enough that the reference's write-before-check
// paths stay in bounds.
#include <lora_phy/ChirpGenerator.hpp>
#include <lora_phy/phy.hpp>

#include <cerrno>
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using namespace lora_phy;
using cf = std::complex<float>;

namespace {

uint32_t fbits(float x) { uint32_t u; std::memcpy(&u, &x, 4); return u; }

uint64_t fnv(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ull; }
    return h;
}

void line(const char* name, const std::string& s) { std::printf("%s: %s\n", name, s.c_str()); }

std::string syms_str(const uint16_t* s, ssize_t n) {
    std::string o;
    char buf[16];
    for (ssize_t i = 0; i < n; ++i) { std::snprintf(buf, sizeof buf, "%s%u", i ? "," : "", s[i]); o += buf; }
    return o;
}

std::string hex(const uint8_t* b, ssize_t n) {
    std::string o;
    char buf[4];
    for (ssize_t i = 0; i < n; ++i) { std::snprintf(buf, sizeof buf, "%02x", b[i]); o += buf; }
    return o;
}

// deterministic impairments (same arithmetic in both builds)
struct Lcg {
    uint64_t s;
    float uni() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (float)((s >> 40) & 0xffffff) / 16777216.0f; }
    float gauss() {
        float u1 = uni(), u2 = uni();
        if (u1 < 1e-7f) u1 = 1e-7f;
        return std::sqrt(-2.0f * std::log(u1)) * std::cos(6.2831853f * u2);
    }
};

void impair(std::vector<cf>& x, unsigned N, float cfo_bins, int delay, float sigma, uint64_t seed) {
    Lcg g{seed};
    std::vector<cf> y(x.size());
    for (size_t i = 0; i < x.size(); ++i) {
        const long src = (long)i - delay;
        cf v = (src >= 0 && src < (long)x.size()) ? x[(size_t)src] : cf(0, 0);
        const float ph = 6.2831853f * cfo_bins / (float)N * (float)i;
        v *= cf(std::cos(ph), std::sin(ph));
        v += cf(sigma * g.gauss(), sigma * g.gauss());
        y[i] = v;
    }
    x.swap(y);
}

struct Ws {
    std::vector<cf> in, out;
    std::vector<float> win;
    lora_workspace ws{};
    int rc;
    Ws(unsigned sf, bandwidth bw, window_type w = window_type::window_none, uint8_t sync = 0x12,
       unsigned osr = 1) {
        const size_t N = size_t(1) << sf;
        in.resize(N); out.resize(N); win.resize(N);
        ws.fft_in = in.data(); ws.fft_out = out.data(); ws.window = win.data();
        lora_params p{};
        p.sf = sf; p.bw = bw; p.cr = 1; p.osr = osr; p.window = w; p.sync_word = sync;
        rc = init(&ws, &p);
    }
};

std::vector<uint8_t> ramp32() {
    std::vector<uint8_t> p(32);
    for (int i = 0; i < 32; ++i) p[i] = (uint8_t)i;
    return p;
}

void chain(const char* tag, unsigned sf, bandwidth bw, const std::vector<uint8_t>& payload,
           float cfo, int delay, float sigma, window_type w = window_type::window_none,
           uint8_t sync = 0x12, unsigned osr = 1) {
    Ws s(sf, bw, w, sync, osr);
    const size_t N = (size_t(1) << sf) * osr;  // samples per symbol
    std::vector<uint16_t> syms(2 * payload.size() + 8);
    const ssize_t ns = encode(&s.ws, payload.data(), payload.size(), syms.data(), syms.size());
    std::vector<cf> iq((ns + 2) * N + 64);
    const ssize_t nm = modulate(&s.ws, syms.data(), (size_t)ns, iq.data(), iq.size());
    iq.resize(nm > 0 ? (size_t)nm : 0);  // (a failed call: no samples)
    if (cfo != 0.0f || delay || sigma > 0.0f) impair(iq, (unsigned)N, cfo, delay, sigma, sf * 131 + delay);
    std::vector<uint16_t> got(ns + 8);
    const ssize_t nd = demodulate(&s.ws, iq.data(), iq.size(), got.data(), got.size());
    const lora_metrics* m = get_last_metrics(&s.ws);
    std::vector<uint8_t> pay(payload.size() + 8);
    const ssize_t nb = nd > 0 ? decode(&s.ws, got.data(), (size_t)(nd & ~1), pay.data(), pay.size()) : -1;
    char buf[256];
    std::snprintf(buf, sizeof buf, "init=%d enc=%zd mod=%zd dem=%zd sync=%02x cfo=%08x toff=%08x dec=%zd crc=%d",
                  s.rc, ns, nm, nd, s.ws.sync_word, fbits(m->cfo), fbits(m->time_offset), nb, (int)m->crc_ok);
    line(tag, std::string(buf) + " syms=" + syms_str(got.data(), nd) + " bytes=" + hex(pay.data(), nb));
}

void legacy(const char* tag, unsigned sf, bandwidth bw, const std::vector<uint8_t>& payload,
            float cfo, int delay, float sigma, float gain, bool scratch,
            window_type w = window_type::window_none, unsigned osr = 1) {
    const size_t N = size_t(1) << sf;
    std::vector<uint16_t> syms(2 * payload.size() + 8);
    const size_t ns = lora_encode(payload.data(), payload.size(), syms.data(), sf);
    std::vector<cf> iq((ns + 2) * N * osr);
    const size_t nm = lora_modulate(syms.data(), ns, iq.data(), sf, osr, bw, 1.0f, 0x12);
    iq.resize(nm);
    if (cfo != 0.0f || delay || sigma > 0.0f) impair(iq, (unsigned)(N * osr), cfo, delay, sigma, sf * 977 + delay);
    for (auto& v : iq) v *= gain;
    // external dechirp (e2e_chain_test.cpp:80-93 / bit_exact_test.cpp:145-155),
    // at the chip rate only
    if (osr == 1) {
        std::vector<cf> down(N);
        float ph = 0.0f;
        genChirp<float>(down.data(), (int)N, 1, (int)N, 0.0f, true, 1.0f, ph, bw_scale(bw));
        for (size_t i = 0; i < iq.size(); ++i) iq[i] *= down[i % N];
    }
    static lora_demod_workspace ws;  // ~115 KB: keep off the stack
    std::vector<cf> scr(iq.size());
    lora_demod_init(&ws, sf, w, scratch ? scr.data() : nullptr, scratch ? scr.size() : 0);
    std::vector<uint16_t> got(iq.size() / N + 2);
    uint8_t sw = 0xEE;
    const ssize_t nd = lora_demodulate(&ws, iq.data(), iq.size(), got.data(), osr, &sw);
    std::vector<uint8_t> pay(got.size());
    const ssize_t nb = nd >= 0 ? lora_decode(got.data(), (size_t)(nd & ~1), pay.data()) : -1;
    char buf[256];
    std::snprintf(buf, sizeof buf, "dem=%zd sync=%02x cfo=%08x toff=%08x dec=%zd", nd, sw,
                  fbits(ws.metrics.cfo), fbits(ws.metrics.time_offset), nb);
    line(tag, std::string(buf) + " syms=" + syms_str(got.data(), nd) + " bytes=" + hex(pay.data(), nb));
    lora_demod_free(&ws);
}

void errors() {
    lora_params cfg{};
    cfg.sf = 7; cfg.bw = bandwidth::bw_125; cfg.cr = 1; cfg.osr = 1; cfg.sync_word = 0x12;
    char buf[512];
    lora_workspace tmp{};
    const int e1 = init(nullptr, &cfg), e2 = init(&tmp, nullptr);
    cfg.window = window_type::window_hann;
    const int e3 = init(&tmp, &cfg);
    cfg.window = window_type::window_none;
    Ws s(7, bandwidth::bw_125);
    uint8_t payload[4] = {1, 2, 3, 4};
    std::vector<uint16_t> sy(64, 0);
    std::vector<cf> iq(4096);
    std::vector<uint8_t> out(64);
    const ssize_t a = encode(nullptr, payload, 4, sy.data(), 8);
    const ssize_t b = encode(&s.ws, payload, 4, sy.data(), 1);
    const ssize_t c = modulate(nullptr, sy.data(), 1, iq.data(), 8);
    const ssize_t d = modulate(&s.ws, sy.data(), 1, iq.data(), 1);
    const ssize_t e = demodulate(nullptr, iq.data(), 10, sy.data(), 8);
    const ssize_t f = demodulate(&s.ws, iq.data(), 10, sy.data(), 8);
    const ssize_t g = demodulate(&s.ws, iq.data(), 128, sy.data(), 8);
    const ssize_t h = demodulate(&s.ws, iq.data(), 512, sy.data(), 1);
    const ssize_t i = decode(nullptr, sy.data(), 1, out.data(), 4);
    const ssize_t j = decode(&s.ws, sy.data(), 1, out.data(), 0);
    const ssize_t k = decode(&s.ws, sy.data(), 2, out.data(), 0);
    const ssize_t l = lora_decode(sy.data(), 3, out.data());
    std::snprintf(buf, sizeof buf,
                  "init_null_ws=%d init_null_cfg=%d init_no_window=%d init_ok=%d enc_null=%zd enc_cap=%zd "
                  "mod_null=%zd mod_cap=%zd dem_null=%zd dem_misaligned=%zd dem_short=%zd dem_cap=%zd "
                  "dec_null=%zd dec_odd=%zd dec_cap=%zd lora_decode_odd=%zd",
                  e1, e2, e3, s.rc, a, b, c, d, e, f, g, h, i, j, k, l);
    line("errors", buf);
}

void roundtrip() {
    Ws s(7, bandwidth::bw_125);
    const uint8_t p[4] = {0xDE, 0xAD, 0xBE, 0xEF};  // roundtrip_test.cpp:30-31
    uint16_t sy[16];
    uint8_t out[8];
    const ssize_t n = encode(&s.ws, p, 4, sy, 16);
    const ssize_t m = decode(&s.ws, sy, (size_t)n, out, 8);
    line("roundtrip", syms_str(sy, n) + " -> " + hex(out, m));
}

void no_alloc() {
    // no_alloc_test.cpp:35: symbols [0,1,12,34,56] at SF7
    Ws s(7, bandwidth::bw_125);
    const uint16_t sy[5] = {0, 1, 12, 34, 56};
    std::vector<cf> iq(7 * 128);
    const ssize_t nm = modulate(&s.ws, sy, 5, iq.data(), iq.size());
    uint16_t got[8] = {};
    const ssize_t nd = demodulate(&s.ws, iq.data(), (size_t)nm, got, 8);
    char buf[64];
    std::snprintf(buf, sizeof buf, "mod=%zd dem=%zd sync=%02x samples=%016llx ", nm, nd, s.ws.sync_word,
                  (unsigned long long)(nm > 0 ? fnv(iq.data(), (size_t)nm * sizeof(cf)) : 0));
    line("no_alloc", buf + syms_str(got, nd));
}

void equal_power(const char* dir) {
    std::string path = std::string(dir) + "/equal_power_iq.bin";
    FILE* fp = std::fopen(path.c_str(), "rb");
    if (!fp) { line("equal_power", "missing fixture"); return; }
    cf x[4];
    const size_t n = std::fread(x, sizeof(cf), 4, fp);
    std::fclose(fp);
    static lora_demod_workspace ws;
    lora_demod_init(&ws, 2);
    uint16_t o[4] = {};
    uint8_t sw = 0xEE;
    const ssize_t r = lora_demodulate(&ws, x, n, o, 1, &sw);
    char buf[128];
    std::snprintf(buf, sizeof buf, "n=%zu dem=%zd sync=%02x", n, r, sw);
    line("equal_power", std::string(buf) + " syms=" + syms_str(o, r));
    lora_demod_free(&ws);
}

void scratch_error() {
    // scratch_buffer_error_test.cpp:16-21: amplitude 2, no scratch
    std::vector<cf> x(128, cf(2.0f, 0.0f));
    static lora_demod_workspace ws;
    lora_demod_init(&ws, 7);
    uint16_t o[4] = {};
    const ssize_t r = lora_demodulate(&ws, x.data(), x.size(), o, 1);
    std::vector<cf> scr(x.size());
    lora_demod_init(&ws, 7, window_type::window_none, scr.data(), scr.size());
    const ssize_t r2 = lora_demodulate(&ws, x.data(), x.size(), o, 1);
    char buf[128];
    std::snprintf(buf, sizeof buf, "no_scratch=%zd with_scratch=%zd sym=%u", r, r2, o[0]);
    line("scratch_error", buf);
    lora_demod_free(&ws);
}

void bit_exact(const char* dir) {
    // vectors/golden/modulation_tests.bin record format (bit_exact_test.cpp)
    std::string path = std::string(dir) + "/modulation_tests.bin";
    FILE* fp = std::fopen(path.c_str(), "rb");
    if (!fp) { line("bit_exact", "missing fixture"); return; }
    uint32_t count = 0;
    if (std::fread(&count, 4, 1, fp) != 1) count = 0;
    for (uint32_t r = 0; r < count; ++r) {
        uint8_t kind = 0;
        uint32_t hdr[5];
        if (std::fread(&kind, 1, 1, fp) != 1 || std::fread(hdr, 4, 5, fp) != 5) break;
        std::vector<uint8_t> payload(hdr[4]);
        if (std::fread(payload.data(), 1, payload.size(), fp) != payload.size()) break;
        uint32_t ns = 0;
        if (std::fread(&ns, 4, 1, fp) != 1) break;
        std::vector<double> ri(2 * (size_t)ns);
        if (std::fread(ri.data(), 8, ri.size(), fp) != ri.size()) break;
        const unsigned sf = hdr[0];
        const size_t N = size_t(1) << sf;
        std::vector<cf> iq(ns);
        for (size_t i = 0; i < ns; ++i) iq[i] = cf((float)ri[2 * i], (float)ri[2 * i + 1]);
        // our own modulation of the record's payload must match the stored IQ
        std::vector<uint16_t> sy(2 * payload.size());
        const size_t n = lora_encode(payload.data(), payload.size(), sy.data(), sf);
        std::vector<cf> mod((n + 2) * N);
        const size_t nm = lora_modulate(sy.data(), n, mod.data(), sf, 1, bandwidth::bw_125, 1.0f, 0x12);
        const bool same = nm == ns && std::memcmp(mod.data(), iq.data(), ns * sizeof(cf)) == 0;
        std::vector<cf> down(N);
        float ph = 0.0f;
        genChirp<float>(down.data(), (int)N, 1, (int)N, 0.0f, true, 1.0f, ph, 1.0f);
        for (size_t i = 0; i < iq.size(); ++i) iq[i] *= down[i % N];
        static lora_demod_workspace ws;
        std::vector<cf> scr(iq.size());
        lora_demod_init(&ws, sf, window_type::window_none, scr.data(), scr.size());
        std::vector<uint16_t> got(ns / N);
        uint8_t sw = 0;
        const ssize_t nd = lora_demodulate(&ws, iq.data(), iq.size(), got.data(), 1, &sw);
        std::vector<uint8_t> out(got.size());
        const ssize_t nb = lora_decode(got.data(), (size_t)(nd & ~1), out.data());
        char buf[128];
        std::snprintf(buf, sizeof buf, "rec=%u sf=%u cr=%u mod_equal=%d dem=%zd sync=%02x match=%d ", r, sf,
                      hdr[2], (int)same, nd, sw, (int)(nb == (ssize_t)payload.size() &&
                                                       std::memcmp(out.data(), payload.data(), payload.size()) == 0));
        line("bit_exact", buf + hex(out.data(), nb));
        lora_demod_free(&ws);
    }
    std::fclose(fp);
}

void offsets() {
    // estimate_offsets / compensate_offsets on an impaired frame
    Ws s(8, bandwidth::bw_125);
    std::vector<uint8_t> p = ramp32();
    std::vector<uint16_t> sy(64);
    const ssize_t ns = encode(&s.ws, p.data(), p.size(), sy.data(), sy.size());
    std::vector<cf> iq((ns + 2) * 256);
    const ssize_t nm = modulate(&s.ws, sy.data(), (size_t)ns, iq.data(), iq.size());
    iq.resize(nm > 0 ? (size_t)nm : 0);  // (a failed call: no samples)
    impair(iq, 256, 0.37f, 5, 0.1f, 4242);
    estimate_offsets(&s.ws, iq.data(), iq.size());
    const lora_metrics m = *get_last_metrics(&s.ws);
    compensate_offsets(&s.ws, iq.data(), iq.size());
    char buf[160];
    std::snprintf(buf, sizeof buf, "cfo=%08x toff=%08x compensated=%016llx", fbits(m.cfo),
                  fbits(m.time_offset), (unsigned long long)fnv(iq.data(), iq.size() * sizeof(cf)));
    line("offsets", buf);
}

}  // namespace

int main(int argc, char** argv) {
    const char* dir = argc > 1 ? argv[1] : "tests/golden";
    errors();
    roundtrip();
    no_alloc();
    equal_power(dir);
    scratch_error();
    bit_exact(dir);
    offsets();
    const std::vector<uint8_t> r32 = ramp32();
    // tests/profiles.yaml profiles with the e2e 32-byte ramp (e2e_chain_test.cpp:63-66)
    chain("chain_sf7_bw125", 7, bandwidth::bw_125, r32, 0, 0, 0);
    chain("chain_sf8_bw125", 8, bandwidth::bw_125, r32, 0, 0, 0);
    chain("chain_sf9_bw250", 9, bandwidth::bw_250, r32, 0, 0, 0);
    chain("chain_sf10_bw250", 10, bandwidth::bw_250, r32, 0, 0, 0);
    chain("chain_sf11_bw500", 11, bandwidth::bw_500, r32, 0, 0, 0);
    chain("chain_sf12_bw500", 12, bandwidth::bw_500, r32, 0, 0, 0);
    chain("chain_sf7_impaired", 7, bandwidth::bw_125, r32, 0.3f, 3, 0.5f);
    chain("chain_sf9_noisy", 9, bandwidth::bw_125, r32, -0.2f, 0, 2.0f);
    chain("chain_sf8_hann", 8, bandwidth::bw_125, r32, 0.1f, 7, 0.3f, window_type::window_hann);
    chain("chain_sync34", 8, bandwidth::bw_125, r32, 0, 0, 0, window_type::window_none, 0x34);
    chain("chain_syncab", 7, bandwidth::bw_125, r32, 0, 0, 0, window_type::window_none, 0xAB);
    legacy("legacy_sf7", 7, bandwidth::bw_125, r32, 0, 0, 0, 1.0f, true);
    legacy("legacy_sf7_impaired", 7, bandwidth::bw_125, r32, 0.25f, 2, 0.7f, 1.0f, true);
    legacy("legacy_sf9_gain3", 9, bandwidth::bw_250, r32, 0, 0, 0.2f, 3.0f, true);
    legacy("legacy_sf9_gain3_noscratch", 9, bandwidth::bw_250, r32, 0, 0, 0.2f, 3.0f, false);
    legacy("legacy_sf12", 12, bandwidth::bw_125, r32, 0, 0, 0, 1.0f, true);
    legacy("legacy_sf8_hann", 8, bandwidth::bw_125, r32, -0.15f, 1, 0.4f, 0.5f, true, window_type::window_hann);
    // oversampled input (lora_params::osr, lora_demodulate's osr argument)
    chain("chain_sf7_osr2", 7, bandwidth::bw_125, r32, 0, 0, 0, window_type::window_none, 0x12, 2);
    chain("chain_sf8_osr4_impaired", 8, bandwidth::bw_125, r32, 0.2f, 37, 0.4f,
          window_type::window_none, 0x12, 4);
    chain("chain_sf9_osr2_hann", 9, bandwidth::bw_250, r32, -0.1f, 5, 0.2f,
          window_type::window_hann, 0x34, 2);
    legacy("legacy_sf7_osr2", 7, bandwidth::bw_125, r32, 0.1f, 9, 0.3f, 1.0f, true,
           window_type::window_none, 2);
    legacy("legacy_sf10_osr3_gain2", 10, bandwidth::bw_125, r32, 0, 100, 0.2f, 2.0f, true,
           window_type::window_none, 3);
    return 0;
}
