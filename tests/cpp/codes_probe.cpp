// Transcript of every LoRaCodes.hpp helper over exhaustive 8/16-bit inputs
// and seeded buffers.  tests/test_codes_cpu.py builds it twice - against
// include/lora_phy/LoRaCodes.hpp (this tree) and against the reference's
// header of the same name - and requires identical transcripts.
#include <cstdio>
#include <cstring>
#include <vector>

#include "LoRaCodes.hpp"

static unsigned long long g_state = 0x9E3779B97F4A7C15ull;
static unsigned rnd() {
    g_state ^= g_state << 13;
    g_state ^= g_state >> 7;
    g_state ^= g_state << 17;
    return (unsigned)(g_state >> 11);
}

static void put(const char* tag, unsigned long long v) { printf("%s %llx\n", tag, v); }

int main() {
    for (unsigned x = 0; x < 256; ++x) {
        bool e = false, b = false;
        put("h84e", encodeHamming84sx((unsigned char)x));
        const unsigned d84 = decodeHamming84sx((unsigned char)x, e, b);
        put("h84d", d84 | (e << 8) | (b << 9));
        put("h74e", encodeHamming74sx((unsigned char)x));
        e = false;
        const unsigned d74 = decodeHamming74sx((unsigned char)x, e);
        put("h74d", d74 | (e << 8));
        e = false;
        const unsigned p54 = checkParity54((unsigned char)x, e);
        put("p54c", p54 | (e << 8));
        put("p54e", encodeParity54((unsigned char)x));
        e = false;
        const unsigned p64 = checkParity64((unsigned char)x, e);
        put("p64c", p64 | (e << 8));
        put("p64e", encodeParity64((unsigned char)x));
        put("xs8", xsum8((uint8_t)x));
        for (unsigned y = 0; y < 16; ++y) {
            const uint8_t h[2] = {(uint8_t)x, (uint8_t)(y | (rnd() & 0xF0))};
            put("hdr", headerChecksum(h));
        }
    }
    for (unsigned x = 0; x < 65536; ++x) {
        put("g2b", grayToBinary16((unsigned short)x));
        put("b2g", binaryToGray16((unsigned short)x));
        put("crc", crc16sx((uint16_t)x, 0x1021));
    }
    for (unsigned n = 0; n < 300; n += 7) put("rup", roundUp(n, 1 + n % 13));
    // checksums and whitening over seeded buffers
    for (int len = 0; len < 80; ++len) {
        std::vector<uint8_t> buf(len + 1);
        for (auto& v : buf) v = (uint8_t)rnd();
        put("ck8", checksum8(buf.data(), len));
        put("sxcrc", sx1272DataChecksum(buf.data(), len));
        std::vector<uint8_t> w = buf;
        SX1232RadioComputeWhitening(w.data(), (uint16_t)len);
        for (int i = 0; i < len; ++i) put("w1232", w[i]);
        for (int rdd = 1; rdd <= 4; ++rdd) {
            for (int ofs = 0; ofs < 12; ofs += 5) {
                w = buf;
                Sx1272ComputeWhitening(w.data(), (uint16_t)len, ofs, rdd);
                for (int i = 0; i < len; ++i) put("w1272", w[i]);
                w = buf;
                Sx1272ComputeWhiteningLfsr(w.data(), (uint16_t)len, ofs, (size_t)rdd);
                for (int i = 0; i < len; ++i) put("wlfsr", w[i]);
            }
        }
    }
    // the whitening_test.cpp known answer (DE AD BE EF 70 0D -> 21 52 90 10 2C F2)
    {
        uint8_t p[6] = {0xDE, 0xAD, 0xBE, 0xEF, 0x70, 0x0D};
        Sx1272ComputeWhiteningLfsr(p, 6, 0, 4);
        for (int i = 0; i < 6; ++i) put("wkat", p[i]);
    }
    // diagonal interleaver round trips, PPM = SF 7..12, RDD 1..4
    for (size_t ppm = 5; ppm <= 12; ++ppm) {
        for (size_t rdd = 1; rdd <= 4; ++rdd) {
            const size_t blocks = 3;
            std::vector<uint8_t> cw(blocks * ppm);
            for (auto& v : cw) v = (uint8_t)(rnd() & ((1u << (4 + rdd)) - 1));
            std::vector<uint16_t> sym(blocks * (4 + rdd) + ppm, 0);
            diagonalInterleaveSx(cw.data(), cw.size(), sym.data(), ppm, rdd);
            for (size_t i = 0; i < blocks * (4 + rdd); ++i) put("ilv", sym[i]);
            std::vector<uint8_t> back(cw.size(), 0);
            diagonalDeterleaveSx(sym.data(), blocks * (4 + rdd), back.data(), ppm, rdd);
            for (auto v : back) put("dil", v);
            for (auto& v : sym) v = (uint16_t)rnd();
            std::vector<uint8_t> b2(cw.size(), 0);
            diagonalDeterleaveSx2(sym.data(), blocks * (4 + rdd), b2.data(), ppm, rdd);
            for (auto v : b2) put("dil2", v);
        }
    }
    return 0;
}
