// TEST INFRASTRUCTURE ONLY — never linked into the product library.
//
// extern "C" shims around the *reference* implementation
// (/root/reference/src/phy/*.cpp, compiled from its own sources by
// oracle/Makefile into oracle/_ref/libloraref.so).  Only tests/, the golden
// generator (tests/golden/make_golden.py) and bench.py's cpu_baseline leg use
// this library: it is the checker, not the product.
//
// Every shim forwards straight to the reference function named in its comment;
// no arithmetic happens here.
#include <lora_phy/phy.hpp>
#include <lora_phy/ChirpGenerator.hpp>
#include <lora_phy/LoRaCodes.hpp>
#include <lorawan/lorawan.hpp>
extern "C" {
#include <lorawan/aes.h>
}

#include <chrono>
#include <complex>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

using cf = std::complex<float>;
using namespace lora_phy;

extern "C" {

size_t ref_sizeof_workspace() { return sizeof(lora_workspace); }
size_t ref_sizeof_demod_workspace() { return sizeof(lora_demod_workspace); }
size_t ref_sizeof_params() { return sizeof(lora_params); }
size_t ref_sizeof_metrics() { return sizeof(lora_metrics); }

// kissfft.hh:71-103 — one forward transform with a fresh plan.
void ref_fft(const float* in, float* out, int nfft) {
    auto* plan = new kissfft_plan<float>{};
    kissfft<float>::init(*plan, nfft, false);
    kissfft<float> f(*plan);
    f.transform(reinterpret_cast<const cf*>(in), reinterpret_cast<cf*>(out));
    delete plan;
}

// LoRaDetector.hpp:39-74
size_t ref_detect(const float* in, float* out, int nfft, float* power,
                  float* power_avg, float* findex) {
    auto* plan = new kissfft_plan<float>{};
    kissfft<float>::init(*plan, nfft, false);
    kissfft<float> f(*plan);
    std::vector<cf> fin(reinterpret_cast<const cf*>(in),
                        reinterpret_cast<const cf*>(in) + nfft);
    LoRaDetector<float> det(size_t(nfft), fin.data(),
                            reinterpret_cast<cf*>(out), f);
    size_t idx = det.detect(*power, *power_avg, *findex);
    delete plan;
    return idx;
}

// ChirpGenerator.hpp:24-51
int ref_genchirp(float* out, int N, int osr, int NN, float f0, int down,
                 float ampl, float* phase, float bw_scale) {
    float ph = *phase;
    int r = genChirp(reinterpret_cast<cf*>(out), N, osr, NN, f0, down != 0,
                     ampl, ph, bw_scale);
    *phase = ph;
    return r;
}

// Test-side dechirp exactly as tests/e2e_chain_test.cpp:80-93 writes it:
// down = genChirp(N, down=true, phase 0); out[s*N+i] = in[s*N+i] * down[i]
// for every whole symbol; samples past the last whole symbol stay zero.
void ref_dechirp(const float* in, float* out, size_t count, unsigned sf,
                 unsigned bw_hz) {
    const size_t N = size_t(1) << sf;
    std::vector<cf> down(N);
    float phase = 0.0f;
    genChirp(down.data(), int(N), 1, int(N), 0.0f, true, 1.0f, phase,
             bw_scale(static_cast<bandwidth>(bw_hz)));
    const cf* x = reinterpret_cast<const cf*>(in);
    cf* y = reinterpret_cast<cf*>(out);
    for (size_t i = 0; i < count; ++i) y[i] = cf(0.0f, 0.0f);
    for (size_t s = 0; s < count / N; ++s)
        for (size_t i = 0; i < N; ++i) y[s * N + i] = x[s * N + i] * down[i];
}

// LoRaMod.cpp:8-43
size_t ref_lora_modulate(const uint16_t* syms, size_t n, float* out,
                         unsigned sf, unsigned osr, unsigned bw_hz,
                         float ampl, uint8_t sync) {
    return lora_modulate(syms, n, reinterpret_cast<cf*>(out), sf, osr,
                         static_cast<bandwidth>(bw_hz), ampl, sync);
}

// LoRaEncoder.cpp:6-18
size_t ref_lora_encode(const uint8_t* bytes, size_t n, uint16_t* out,
                       unsigned sf) {
    return lora_encode(bytes, n, out, sf);
}

// LoRaDecoder.cpp:7-21
ssize_t ref_lora_decode(const uint16_t* syms, size_t n, uint8_t* out) {
    return lora_decode(syms, n, out);
}

// LoRaCodes.hpp:92-105
uint16_t ref_sx1272_checksum(const uint8_t* data, int len) {
    return sx1272DataChecksum(data, len);
}

// LoRaCodes.hpp:250-281
uint8_t ref_decode_hamming84(uint8_t b) {
    bool e = false, bad = false;
    return decodeHamming84sx(b, e, bad);
}

// LoRaCodes.hpp helpers, forwarded one to one.
uint16_t ref_gray(uint16_t v, int to_binary) { return to_binary ? grayToBinary16(v) : binaryToGray16(v); }
void ref_interleave(const uint8_t* cw, size_t ncw, uint16_t* syms, size_t ppm, size_t rdd) {
    diagonalInterleaveSx(cw, ncw, syms, ppm, rdd);
}
void ref_deinterleave(const uint16_t* syms, size_t nsyms, uint8_t* cw, size_t ppm, size_t rdd) {
    diagonalDeterleaveSx(syms, nsyms, cw, ppm, rdd);
}
void ref_whiten(uint8_t* buf, size_t len, int kind, int bit_ofs, unsigned rdd) {
    if (kind == 0) SX1232RadioComputeWhitening(buf, (uint16_t)len);
    else if (kind == 1) Sx1272ComputeWhitening(buf, (uint16_t)len, bit_ofs, (int)rdd);
    else Sx1272ComputeWhiteningLfsr(buf, (uint16_t)len, bit_ofs, rdd);
}
uint8_t ref_hamming(uint8_t x, int op, uint8_t* flags) {
    bool e = false, b = false;
    uint8_t out;
    switch (op) {
        case 0: out = encodeHamming84sx(x); break;
        case 1: out = decodeHamming84sx(x, e, b); break;
        case 2: out = encodeHamming74sx(x); break;
        case 3: out = decodeHamming74sx(x, e); break;
        case 4: out = encodeParity54(x); break;
        case 5: out = checkParity54(x, e); break;
        case 6: out = encodeParity64(x); break;
        default: out = checkParity64(x, e); break;
    }
    if (flags) *flags = (uint8_t)((e ? 1 : 0) | (b ? 2 : 0));
    return out;
}
uint16_t ref_checksum(const uint8_t* buf, size_t len, int kind) {
    if (kind == 0) return sx1272DataChecksum(buf, (int)len);
    if (kind == 1) return headerChecksum(buf);
    return checksum8(buf, len);
}

// LoRaDemod.cpp:11-197 (init + demodulate + free).  metrics_out gets
// {cfo, time_offset} as stored in ws->metrics.
ssize_t ref_lora_demodulate(unsigned sf, int window, const float* samples,
                            size_t count, uint16_t* out, unsigned osr,
                            uint8_t* out_sync, int with_scratch,
                            float* metrics_out) {
    auto* ws = new lora_demod_workspace{};
    std::vector<cf> scratch(with_scratch ? count : 0);
    lora_demod_init(ws, sf, window ? window_type::window_hann
                                   : window_type::window_none,
                    with_scratch ? scratch.data() : nullptr,
                    with_scratch ? count : 0);
    ssize_t r = lora_demodulate(ws, reinterpret_cast<const cf*>(samples),
                                count, out, osr, out_sync);
    if (metrics_out) {
        metrics_out[0] = ws->metrics.cfo;
        metrics_out[1] = ws->metrics.time_offset;
    }
    lora_demod_free(ws);
    delete ws;
    return r;
}

// Workspace helpers for phy.cpp entry points.
struct ref_ws {
    lora_workspace ws{};
    std::vector<cf> fin, fout;
    std::vector<float> win;
    std::vector<uint16_t> sb;
};

static int ref_ws_init(ref_ws& r, unsigned sf, unsigned bw_hz, unsigned osr,
                       int window, uint8_t sync) {
    size_t N = size_t(1) << sf;
    r.fin.resize(N * (osr ? osr : 1));
    r.fout.resize(N * (osr ? osr : 1));
    r.win.resize(N);
    r.sb.resize(N);
    r.ws.fft_in = r.fin.data();
    r.ws.fft_out = r.fout.data();
    r.ws.window = r.win.data();
    r.ws.symbol_buf = r.sb.data();
    lora_params p{};
    p.sf = sf;
    p.bw = static_cast<bandwidth>(bw_hz);
    p.osr = osr;
    p.window = window ? window_type::window_hann : window_type::window_none;
    p.sync_word = sync;
    return init(&r.ws, &p);
}

// phy.cpp:182-243.  meta_out = {cfo, time_offset}; sync_out = ws->sync_word.
ssize_t ref_demodulate(unsigned sf, unsigned bw_hz, unsigned osr, int window,
                       uint8_t sync, const float* iq, size_t count,
                       uint16_t* syms, size_t cap, float* meta_out,
                       uint8_t* sync_out) {
    auto* r = new ref_ws;
    ref_ws_init(*r, sf, bw_hz, osr, window, sync);
    ssize_t n = demodulate(&r->ws, reinterpret_cast<const cf*>(iq), count,
                           syms, cap);
    if (meta_out) {
        meta_out[0] = r->ws.metrics.cfo;
        meta_out[1] = r->ws.metrics.time_offset;
    }
    if (sync_out) *sync_out = r->ws.sync_word;
    delete r;
    return n;
}

// phy.cpp:81-148
void ref_estimate_offsets(unsigned sf, unsigned bw_hz, unsigned osr,
                          int window, const float* iq, size_t count,
                          float* meta_out) {
    auto* r = new ref_ws;
    ref_ws_init(*r, sf, bw_hz, osr, window, 0x12);
    estimate_offsets(&r->ws, reinterpret_cast<const cf*>(iq), count);
    meta_out[0] = r->ws.metrics.cfo;
    meta_out[1] = r->ws.metrics.time_offset;
    delete r;
}

// phy.cpp:150-180 with ws->metrics = {cfo, time_offset}; samples in place.
void ref_compensate_offsets(unsigned sf, unsigned osr, float cfo,
                            float time_offset, float* iq, size_t count) {
    auto* r = new ref_ws;
    ref_ws_init(*r, sf, 125000, osr, 0, 0x12);
    r->ws.metrics.cfo = cfo;
    r->ws.metrics.time_offset = time_offset;
    compensate_offsets(&r->ws, reinterpret_cast<cf*>(iq), count);
    delete r;
}

// phy.cpp:245-261.  crc_out = ws->metrics.crc_ok.
ssize_t ref_decode(unsigned sf, const uint16_t* syms, size_t n, uint8_t* out,
                   size_t cap, uint8_t* crc_out) {
    auto* r = new ref_ws;
    ref_ws_init(*r, sf, 125000, 1, 0, 0x12);
    ssize_t k = decode(&r->ws, syms, n, out, cap);
    if (crc_out) *crc_out = r->ws.metrics.crc_ok ? 1 : 0;
    delete r;
    return k;
}

// CPU baseline harness (bench.py cpu_baseline leg, BASELINE.md §2 "mode B"):
// `frames` pre-modulated frames of `frame_samples` samples each in `iq`;
// T threads, one lora_demod_workspace each, dechirp + lora_demodulate +
// lora_decode per frame.  Returns wall seconds; writes the decoded bytes.
double ref_bench_modeB(unsigned sf, unsigned bw_hz, const float* iq,
                       size_t frames, size_t frame_samples, uint8_t* bytes_out,
                       int threads) {
    const size_t N = size_t(1) << sf;
    const size_t nsym = frame_samples / N;
    const size_t ndata = nsym >= 2 ? nsym - 2 : 0;
    std::vector<cf> down(N);
    float phase = 0.0f;
    genChirp(down.data(), int(N), 1, int(N), 0.0f, true, 1.0f, phase,
             bw_scale(static_cast<bandwidth>(bw_hz)));
    auto worker = [&](size_t f0, size_t f1) {
        auto* ws = new lora_demod_workspace{};
        std::vector<cf> scratch(frame_samples), dech(frame_samples);
        std::vector<uint16_t> syms(ndata + 2);
        lora_demod_init(ws, sf, window_type::window_none, scratch.data(),
                        scratch.size());
        for (size_t f = f0; f < f1; ++f) {
            const cf* x = reinterpret_cast<const cf*>(iq) + f * frame_samples;
            for (size_t s = 0; s < nsym; ++s)
                for (size_t i = 0; i < N; ++i)
                    dech[s * N + i] = x[s * N + i] * down[i];
            lora_demodulate(ws, dech.data(), frame_samples, syms.data(), 1,
                            nullptr);
            lora_decode(syms.data(), ndata & ~size_t(1),
                        bytes_out + f * (ndata / 2));
        }
        lora_demod_free(ws);
        delete ws;
    };
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    size_t per = (frames + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        size_t a = t * per, b = std::min(frames, a + per);
        if (a < b) th.emplace_back(worker, a, b);
    }
    for (auto& t : th) t.join();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// Same for the high-level API ("mode A": demodulate + decode, phy.cpp).
double ref_bench_modeA(unsigned sf, unsigned bw_hz, const float* iq,
                       size_t frames, size_t frame_samples, uint8_t* bytes_out,
                       int threads) {
    const size_t N = size_t(1) << sf;
    const size_t nsym = frame_samples / N;
    const size_t ndata = nsym >= 2 ? nsym - 2 : 0;
    auto worker = [&](size_t f0, size_t f1) {
        auto* r = new ref_ws;
        ref_ws_init(*r, sf, bw_hz, 1, 0, 0x12);
        std::vector<uint16_t> syms(ndata + 2);
        for (size_t f = f0; f < f1; ++f) {
            const cf* x = reinterpret_cast<const cf*>(iq) + f * frame_samples;
            demodulate(&r->ws, x, frame_samples, syms.data(), syms.size());
            decode(&r->ws, syms.data(), ndata & ~size_t(1),
                   bytes_out + f * (ndata / 2), ndata / 2);
        }
        delete r;
    };
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    size_t per = (frames + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        size_t a = t * per, b = std::min(frames, a + per);
        if (a < b) th.emplace_back(worker, a, b);
    }
    for (auto& t : th) t.join();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// ---- LoRaWAN (lorawan.cpp + tiny-AES aes.c), SURVEY §8f rank 4
void ref_aes128(const uint8_t key[16], uint8_t blk[16]) {
    AES_ctx ctx;
    AES_init_ctx(&ctx, key);
    AES_ECB_encrypt(&ctx, blk);
}

uint32_t ref_lorawan_mic(const uint8_t key[16], int uplink, uint32_t devaddr, uint32_t fcnt,
                         const uint8_t* data, size_t len) {
    return lorawan::compute_mic(key, uplink != 0, devaddr, fcnt, data, len);
}

// build_frame: hdr = {mtype, major, devaddr, fctrl, fcnt}; returns its value,
// symbols in `syms` (capacity cap), tmp bytes in `tmp` (capacity tmp_cap).
long ref_lorawan_build(const uint8_t key[16], const uint32_t* hdr, const uint8_t* fopts, size_t nfopts,
                       const uint8_t* payload, size_t npay, uint16_t* syms, size_t cap, uint8_t* tmp,
                       size_t tmp_cap) {
    lora_workspace ws{};
    lorawan::Frame f;
    f.mhdr.mtype = static_cast<lorawan::MType>(hdr[0]);
    f.mhdr.major = static_cast<uint8_t>(hdr[1]);
    f.fhdr.devaddr = hdr[2];
    f.fhdr.fctrl = static_cast<uint8_t>(hdr[3]);
    f.fhdr.fcnt = static_cast<uint16_t>(hdr[4]);
    f.fhdr.fopts.assign(fopts, fopts + nfopts);
    f.payload.assign(payload, payload + npay);
    return lorawan::build_frame(&ws, key, f, syms, cap, tmp, tmp_cap);
}

// parse_frame: out = {mtype, major, devaddr, fctrl, fcnt, nfopts, npay} of the
// Frame after the call (pre-set to all-ones markers), fopts / payload bytes
// copied to the given buffers (capacity 256 / 65536).  `tmp` must hold
// symbol_count / 2 bytes whatever tmp_cap says (the reference decodes before
// checking the capacity).
long ref_lorawan_parse(const uint8_t key[16], const uint16_t* syms, size_t n, uint8_t* tmp, size_t tmp_cap,
                       uint32_t* out, uint8_t* fopts, uint8_t* payload) {
    lora_workspace ws{};
    lorawan::Frame f;
    f.mhdr.mtype = static_cast<lorawan::MType>(7);
    f.mhdr.major = 3;
    f.fhdr.devaddr = 0xFFFFFFFFu;
    f.fhdr.fctrl = 0xFF;
    f.fhdr.fcnt = 0xFFFF;
    long r = lorawan::parse_frame(&ws, key, syms, n, f, tmp, tmp_cap);
    out[0] = static_cast<uint32_t>(f.mhdr.mtype);
    out[1] = f.mhdr.major;
    out[2] = f.fhdr.devaddr;
    out[3] = f.fhdr.fctrl;
    out[4] = f.fhdr.fcnt;
    out[5] = static_cast<uint32_t>(f.fhdr.fopts.size());
    out[6] = static_cast<uint32_t>(f.payload.size());
    std::memcpy(fopts, f.fhdr.fopts.data(), f.fhdr.fopts.size());
    std::memcpy(payload, f.payload.data(), f.payload.size());
    return r;
}

}  // extern "C"
