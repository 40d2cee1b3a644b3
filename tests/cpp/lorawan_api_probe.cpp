// lorawan:: API transcript probe (TEST INFRASTRUCTURE).
//
// One source, two builds, as lora_phy_api_probe.cpp: against the drop-in
// (include/lorawan/lorawan.hpp + liblora_phy_amd.so, MIC and decode on the
// GPU), built by tests/test_gpu_cxx_api.py on the GPU box; and against the
// reference's src/lorawan/lorawan.cpp + aes.c + src/phy compiled from
// /root/reference (oracle/Makefile target `lwprobe`, travels prebuilt as
// oracle/_ref/lorawan_api_probe_ref).  Prints return codes, MICs, symbols,
// temporary bytes and every Frame field after each call; the test asserts
// the transcripts are identical.  Scenarios: the MIC known answer
// (lorawan_mic_test.cpp:10-11), seeded MICs over lengths 0..300, seeded
// build_frame -> parse_frame round trips over every MType, FOpts 0..17
// bytes and payloads up to 222 bytes, tampered symbols (MIC nibble, a
// correctable bit), odd / short / truncated symbol runs, capacity errors,
// null arguments and an FOpts length that runs into the MIC.  Buffers are
// always large enough for the reference's decode-before-check path.
#include <lorawan/lorawan.hpp>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <vector>

namespace {

uint64_t rng_state = 0x9E3779B97F4A7C15ull;
uint32_t next() {
    rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
    return static_cast<uint32_t>(rng_state >> 32);
}
std::vector<uint8_t> bytes(size_t n) {
    std::vector<uint8_t> v(n);
    for (auto& b : v) b = static_cast<uint8_t>(next());
    return v;
}

void hex(const char* tag, const uint8_t* p, size_t n) {
    std::printf(" %s=", tag);
    for (size_t i = 0; i < n; ++i) std::printf("%02x", p[i]);
}

void frame(const lorawan::Frame& f) {
    std::printf(" mtype=%u major=%u devaddr=%08x fctrl=%02x fcnt=%04x", unsigned(f.mhdr.mtype), f.mhdr.major,
                f.fhdr.devaddr, f.fhdr.fctrl, f.fhdr.fcnt);
    hex("fopts", f.fhdr.fopts.data(), f.fhdr.fopts.size());
    hex("payload", f.payload.data(), f.payload.size());
}

lorawan::Frame marker() {
    lorawan::Frame f;
    f.mhdr.mtype = lorawan::MType::Proprietary;
    f.mhdr.major = 3;
    f.fhdr.devaddr = 0xDEADBEEF;
    f.fhdr.fctrl = 0xAA;
    f.fhdr.fcnt = 0x5555;
    f.fhdr.fopts = {1, 2, 3};
    f.payload = {9};
    return f;
}

void parse(const char* tag, lora_phy::lora_workspace* ws, const uint8_t* key, const uint16_t* syms, size_t n,
           size_t tmp_cap) {
    std::vector<uint8_t> tmp(n / 2 + 16, 0);
    lorawan::Frame f = marker();
    const ssize_t r = lorawan::parse_frame(ws, key, syms, n, f, tmp.data(), tmp_cap);
    std::printf("parse %s n=%zu cap=%zu ret=%zd", tag, n, tmp_cap, r);
    frame(f);
    std::printf("\n");
}

}  // namespace

int main() {
    static lora_phy::lora_workspace ws{};
    // known answer (lorawan_mic_test.cpp:8-11)
    uint8_t k2[16];
    for (auto& b : k2) b = 2;
    const uint8_t msg[] = {0x40, 0x04, 0x03, 0x02, 0x01, 0x80, 0x01, 0x00, 0x01, 0xA6, 0x94, 0x64, 0x26, 0x15};
    std::printf("mic kat %08x\n", lorawan::compute_mic(k2, true, 0x01020304, 1, msg, sizeof msg));
    for (size_t n = 0; n <= 300; n += (n < 40 ? 1 : 13)) {
        auto key = bytes(16), d = bytes(n);
        const bool up = next() & 1;
        const uint32_t da = next(), fc = next();
        std::printf("mic n=%zu up=%d %08x\n", n, int(up), lorawan::compute_mic(key.data(), up, da, fc, d.data(), n));
    }
    const size_t pays[] = {0, 1, 5, 12, 13, 31, 51, 115, 222};
    for (int i = 0; i < 36; ++i) {
        auto key = bytes(16);
        lorawan::Frame f;
        f.mhdr.mtype = static_cast<lorawan::MType>(i % 8);
        f.mhdr.major = static_cast<uint8_t>(next() & 3);
        f.fhdr.devaddr = next();
        f.fhdr.fctrl = static_cast<uint8_t>(next());
        f.fhdr.fcnt = static_cast<uint16_t>(next());
        f.fhdr.fopts = bytes(i % 18);
        f.payload = bytes(pays[i % 9]);
        const size_t need = 12 + f.fhdr.fopts.size() + f.payload.size();
        std::vector<uint16_t> syms(2 * need + 8, 0);
        std::vector<uint8_t> tmp(need + 8, 0);
        const ssize_t r = lorawan::build_frame(&ws, key.data(), f, syms.data(), syms.size(), tmp.data(), tmp.size());
        std::printf("build %d ret=%zd", i, r);
        hex("tmp", tmp.data(), need);
        std::printf(" syms=");
        for (ssize_t j = 0; j < r; ++j) std::printf("%02x", syms[j]);
        std::printf("\n");
        if (r <= 0) continue;
        parse("clean", &ws, key.data(), syms.data(), r, r / 2);
        auto t = syms;
        t[r - 1] ^= 0x0F;
        parse("mic", &ws, key.data(), t.data(), r, r / 2);
        t = syms;
        t[next() % r] ^= static_cast<uint16_t>(1u << (next() % 8));
        parse("bit", &ws, key.data(), t.data(), r, r / 2);
        parse("odd", &ws, key.data(), syms.data(), r - 1, r);
        parse("short", &ws, key.data(), syms.data(), 22, 11);
        parse("trunc", &ws, key.data(), syms.data(), r - 2, r / 2);
        parse("cap", &ws, key.data(), syms.data(), r, r / 2 - 1);
        parse("nullws", nullptr, key.data(), syms.data(), r, r / 2);
        // capacity and null-argument errors of build_frame
        std::printf("build-errs %d %zd %zd %zd %zd\n", i,
                    lorawan::build_frame(&ws, key.data(), f, syms.data(), syms.size(), tmp.data(), need - 1),
                    lorawan::build_frame(&ws, key.data(), f, syms.data(), 2 * need - 1, tmp.data(), tmp.size()),
                    lorawan::build_frame(nullptr, key.data(), f, syms.data(), syms.size(), tmp.data(), tmp.size()),
                    lorawan::build_frame(&ws, key.data(), f, syms.data(), syms.size(), nullptr, tmp.size()));
    }
    // FOpts length running into the MIC, with a valid MIC (lorawan.cpp:172)
    {
        uint8_t key[16];
        for (int i = 0; i < 16; ++i) key[i] = static_cast<uint8_t>(16 + i);
        std::vector<uint8_t> b = {0x40, 1, 2, 3, 4, 0x0F, 9, 0, 1, 2};
        const uint32_t mic = lorawan::compute_mic(key, true, 0x04030201, 9, b.data(), b.size());
        for (int i = 0; i < 4; ++i) b.push_back(static_cast<uint8_t>(mic >> (8 * i)));
        std::vector<uint16_t> syms(2 * b.size());
        const ssize_t r = lora_phy::encode(&ws, b.data(), b.size(), syms.data(), syms.size());
        parse("fopts-overrun", &ws, key, syms.data(), static_cast<size_t>(r), b.size());
    }
    return 0;
}
