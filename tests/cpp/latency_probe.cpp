// Single-frame latency of the lora_phy:: API (TEST / MEASUREMENT TOOL).
//
// One source, two builds (as lora_phy_api_probe.cpp): against the drop-in
// (liblora_phy_amd.so, GPU behind the C ABI) and against the reference
// library compiled from /root/reference's sources (oracle/Makefile
// `latprobe`, CPU).  It times what the reference's own perf harness times,
// one call per packet (tests/performance_test.cpp:98-123 of the reference:
// lora_demod_init once, then per packet lora_modulate + external dechirp +
// lora_demodulate), and the receive chain of runners/rx_runner.cpp:107-116
// (init once, then demodulate + decode per input), plus the legacy receive
// chain dechirp + lora_demodulate + lora_decode.  32-byte payload (66
// symbols), BW125, osr 1.  Prints one JSON line per (SF, chain): median and
// p99 microseconds per call over `packets` calls after a warm-up, and that
// every call returned the expected count.
#include <lora_phy/ChirpGenerator.hpp>
#include <lora_phy/phy.hpp>

#include <algorithm>
#include <chrono>
#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace lora_phy;
using cf = std::complex<float>;
using clk = std::chrono::steady_clock;

namespace {

struct Stat {
    double med, p99;
};

Stat stats(std::vector<double>& us) {
    std::sort(us.begin(), us.end());
    return {us[us.size() / 2], us[std::min(us.size() - 1, (size_t)(0.99 * (double)us.size()))]};
}

void report(const char* chain, unsigned sf, std::vector<double>& us, bool ok, int packets) {
    const Stat s = stats(us);
    std::printf("{\"chain\": \"%s\", \"sf\": %u, \"packets\": %d, \"median_us\": %.2f, \"p99_us\": %.2f, "
                "\"data_symbols_per_s\": %.1f, \"ok\": %s}\n",
                chain, sf, packets, s.med, s.p99, 64.0 / (s.med * 1e-6), ok ? "true" : "false");
    std::fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
    const int sf_lo = argc > 1 ? std::atoi(argv[1]) : 7;
    const int sf_hi = argc > 2 ? std::atoi(argv[2]) : 12;
    const int budget = argc > 3 ? std::atoi(argv[3]) : 400;  // packets at SF7, fewer above
    for (int sf = sf_lo; sf <= sf_hi; ++sf) {
        const int packets = std::max(20, budget >> (sf - 7));
        const size_t N = size_t(1) << sf;
        std::vector<uint8_t> payload(32);
        for (size_t i = 0; i < payload.size(); ++i) payload[i] = static_cast<uint8_t>(i & 0xFF);
        std::vector<uint16_t> symbols(64);
        const size_t nsym = lora_encode(payload.data(), payload.size(), symbols.data(), sf);
        const size_t count = (nsym + 2) * N;
        std::vector<cf> samples(count), dechirped(count), scratch(count), down(N);
        std::vector<uint16_t> demod(nsym);
        std::vector<uint8_t> bytes(nsym / 2);
        float phase = 0.0f;
        genChirp(down.data(), (int)N, 1, (int)N, 0.0f, true, 1.0f, phase, 1.0f);
        lora_modulate(symbols.data(), nsym, samples.data(), sf, 1, bandwidth::bw_125, 1.0f, 0x12);
        auto dechirp = [&] {
            for (size_t s = 0; s < nsym + 2; ++s)
                for (size_t i = 0; i < N; ++i) dechirped[s * N + i] = samples[s * N + i] * down[i];
        };

        // (1) the reference perf harness loop (performance_test.cpp:112-123)
        {
            lora_demod_workspace* ws = new lora_demod_workspace{};
            lora_demod_init(ws, sf, window_type::window_none, scratch.data(), scratch.size());
            std::vector<double> us;
            bool ok = true;
            for (int p = -3; p < packets; ++p) {
                const auto t0 = clk::now();
                lora_modulate(symbols.data(), nsym, samples.data(), sf, 1, bandwidth::bw_125, 1.0f, 0x12);
                dechirp();
                const ssize_t r = lora_demodulate(ws, dechirped.data(), count, demod.data(), 1, nullptr);
                const auto t1 = clk::now();
                ok &= r == (ssize_t)nsym;
                if (p >= 0) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            }
            report("perf_test: lora_modulate + dechirp + lora_demodulate", sf, us, ok, packets);
            // (2) the legacy receive chain
            us.clear();
            for (int p = -3; p < packets; ++p) {
                const auto t0 = clk::now();
                dechirp();
                const ssize_t r = lora_demodulate(ws, dechirped.data(), count, demod.data(), 1, nullptr);
                const ssize_t b = lora_decode(demod.data(), nsym, bytes.data());
                const auto t1 = clk::now();
                ok &= r == (ssize_t)nsym && b == (ssize_t)(nsym / 2) &&
                      std::equal(bytes.begin(), bytes.end(), payload.begin());
                if (p >= 0) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            }
            report("dechirp + lora_demodulate + lora_decode", sf, us, ok, packets);
            lora_demod_free(ws);
            delete ws;
        }
        // (3) rx_runner's chain (rx_runner.cpp:107-116): demodulate + decode
        {
            lora_workspace* ws = new lora_workspace{};
            std::vector<cf> fin(N), fout(N);
            ws->fft_in = fin.data();
            ws->fft_out = fout.data();
            lora_params prm{};
            prm.sf = (unsigned)sf;
            prm.bw = bandwidth::bw_125;
            const bool init_ok = init(ws, &prm) == 0;
            std::vector<double> us;
            bool ok = init_ok;
            for (int p = -3; p < packets; ++p) {
                const auto t0 = clk::now();
                const ssize_t r = demodulate(ws, samples.data(), count, demod.data(), demod.size());
                const ssize_t b = decode(ws, demod.data(), nsym, bytes.data(), bytes.size());
                const auto t1 = clk::now();
                ok &= r == (ssize_t)nsym && b == (ssize_t)(nsym / 2);
                if (p >= 0) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            }
            report("rx_runner: demodulate + decode", sf, us, ok, packets);
            delete ws;
        }
    }
    return 0;
}
