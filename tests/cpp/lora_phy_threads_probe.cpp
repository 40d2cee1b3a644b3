// Re-entrancy probe of the lora_phy:: API (TEST INFRASTRUCTURE).
//
// The reference is re-entrant with one workspace per thread and no global
// state (API_SPEC.md:136-140).  Two (or more) threads each own a
// lora_demod_workspace and a lora_workspace at the SAME spreading factor
// and run interleaved receive chains concurrently: dechirp +
// lora_demodulate + lora_decode on the legacy workspace, demodulate +
// decode + get_last_metrics on the high-level one, over frames with
// per-thread CFO, gain and payloads.  Each thread records its transcript;
// after the join they are printed in thread order.  Built against the
// drop-in (tests/test_gpu_cxx_api.py) and against the reference's sources
// (oracle/Makefile `tprobe`); the two transcripts must be identical.
#include <lora_phy/ChirpGenerator.hpp>
#include <lora_phy/phy.hpp>

#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

using namespace lora_phy;
using cf = std::complex<float>;

namespace {

uint32_t fbits(float x) {
    uint32_t u;
    std::memcpy(&u, &x, 4);
    return u;
}

std::string worker(int id, unsigned sf, int frames) {
    const size_t N = size_t(1) << sf;
    std::string out;
    char buf[256];
    lora_demod_workspace* dws = new lora_demod_workspace{};
    const size_t nsym = 2 * 24, count = (nsym + 2) * N;
    std::vector<cf> samples(count), dech(count), scratch(count), down(N), fin(N), fout(N);
    lora_demod_init(dws, sf, window_type::window_none, scratch.data(), scratch.size());
    lora_workspace* ws = new lora_workspace{};
    ws->fft_in = fin.data();
    ws->fft_out = fout.data();
    lora_params prm{};
    prm.sf = sf;
    if (init(ws, &prm) != 0) return "init failed\n";
    float ph = 0.0f;
    genChirp(down.data(), (int)N, 1, (int)N, 0.0f, true, 1.0f, ph, 1.0f);
    std::vector<uint8_t> payload(24), bytes(24);
    std::vector<uint16_t> syms(nsym), demod(nsym);
    for (int f = 0; f < frames; ++f) {
        for (size_t i = 0; i < payload.size(); ++i) payload[i] = (uint8_t)(37 * f + 11 * id + 5 * i);
        lora_encode(payload.data(), payload.size(), syms.data(), sf);
        lora_modulate(syms.data(), nsym, samples.data(), sf, 1, bandwidth::bw_125, 1.0f, 0x12);
        const float cfo = 0.07f * (float)((f + id) % 5) - 0.14f, gain = 1.0f + 0.5f * (float)((f * 3 + id) % 4);
        for (size_t i = 0; i < count; ++i) {
            const float a = 2.0f * PI * cfo * (float)i / (float)N;
            samples[i] = samples[i] * cf(std::cos(a), std::sin(a)) * gain;
        }
        for (size_t i = 0; i < count; ++i) dech[i] = samples[i] * down[i % N];
        uint8_t sync = 0;
        const ssize_t r = lora_demodulate(dws, dech.data(), count, demod.data(), 1, &sync);
        const ssize_t b = r > 0 ? lora_decode(demod.data(), (size_t)r, bytes.data()) : r;
        std::snprintf(buf, sizeof buf, "t%d f%d B r=%zd b=%zd sync=%02x cfo=%08x to=%08x", id, f, r, b, sync,
                      fbits(dws->metrics.cfo), fbits(dws->metrics.time_offset));
        out += buf;
        for (ssize_t i = 0; i < b; ++i) {
            std::snprintf(buf, sizeof buf, "%s%02x", i ? "" : " bytes=", bytes[i]);
            out += buf;
        }
        out += "\n";
        const ssize_t ra = demodulate(ws, samples.data(), count, demod.data(), demod.size());
        const ssize_t ba = ra > 0 ? decode(ws, demod.data(), (size_t)ra, bytes.data(), bytes.size()) : ra;
        const lora_metrics* m = get_last_metrics(ws);
        std::snprintf(buf, sizeof buf, "t%d f%d A r=%zd b=%zd sync=%02x cfo=%08x to=%08x crc=%d s0=%u s7=%u", id, f,
                      ra, ba, ws->sync_word, fbits(m->cfo), fbits(m->time_offset), (int)m->crc_ok,
                      ra > 0 ? demod[0] : 0u, ra > 7 ? demod[7] : 0u);
        out += buf;
        out += "\n";
    }
    lora_demod_free(dws);
    delete dws;
    delete ws;
    return out;
}

}  // namespace

int main(int argc, char** argv) {
    const int threads = argc > 1 ? std::atoi(argv[1]) : 2;
    const unsigned sf = argc > 2 ? (unsigned)std::atoi(argv[2]) : 9;
    const int frames = argc > 3 ? std::atoi(argv[3]) : 12;
    std::vector<std::string> res(threads);
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back([&, t] { res[t] = worker(t, sf, frames); });
    for (auto& t : ts) t.join();
    for (auto& r : res) std::fputs(r.c_str(), stdout);
    return 0;
}
