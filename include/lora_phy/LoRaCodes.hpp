/**
 * @file lora_phy/LoRaCodes.hpp
 * Codec helpers of the LoRa PHY: checksums, whitening, Gray mapping,
 * Hamming / parity codes and the SX127x diagonal interleaver.
 *
 * Drop-in for the reference's header of the same name
 * (/root/reference/include/lora_phy/LoRaCodes.hpp): same names, signatures
 * and results for every helper, so reference consumers such as its
 * whitening_test.cpp and lora_phy_vector_dump.cpp build unchanged against
 * this tree.  Written from the algorithms, not from the reference text:
 * parity-check bits are masks over the codeword, the LFSRs are a single
 * state word.  tests/test_codes_cpu.py compares every function with the
 * reference header exhaustively (all 8-bit inputs, seeded buffers).
 * Host-only; the batch forms of the decode-side helpers run on the GPU.
 */
#pragma once

#include <cstddef>
#include <cstdint>

// Explicit-header geometry of the SX127x (reference LoRaCodes.hpp:17-19).
#define HEADER_RDD 4
#define N_HEADER_SYMBOLS (HEADER_RDD + 4)
#define N_HEADER_CODEWORDS 5

namespace lora_codes_detail {

// parity of the set bits of v
static inline unsigned par(unsigned v) { return (unsigned)__builtin_parity(v); }

// One step of the 8-bit LFSR that masks the SX1272 payload CRC: shift left,
// feed back the parity of taps 0xB8.
static inline uint8_t crc_mask_step(uint8_t v) {
    return (uint8_t)((v << 1) | par(v & 0xB8u));
}

// Whitening sequence of the SX1272 (510 bits as reverse engineered from the
// modem; reference LoRaCodes.hpp:147-152) and the per-bit offsets into it:
// coding rates 2-4, and 1 (single parity).
static const uint64_t kWhitenSeq[8] = {
    0x0102291EA751AAFFull, 0xD24B050A8D643A17ull, 0x5B279B671120B8F4ull, 0x032B37B9F6FB55A2ull,
    0x994E0F87E95E2D16ull, 0x7CBCFC7631984C26ull, 0x281C8E4F0DAEF7F9ull, 0x1741886EB7733B15ull};
static const int kWhitenLen = 510;
static const int kWhitenOfs[8] = {6, 4, 2, 0, -112, -114, -302, -34};
static const int kWhitenOfsCr1[5] = {6, 4, 2, 0, -360};

// Interleaved byte LFSRs of the SX1272 whitening (polynomial 0x1D); start
// values per coding-rate class (reference LoRaCodes.hpp:183-184).
static const uint64_t kLfsrSeed[2] = {0x6572D100E85C2EFFull, 0xE85C2EFFFFFFFFFFull};
static const uint64_t kLfsrSeedCr1[2] = {0x05121100F8ECFEEFull, 0xF8ECFEEFEFEFEFEFull};
static inline uint64_t lfsr64_step(uint64_t r) {
    const uint64_t fb = (r >> 32) ^ (r >> 24) ^ (r >> 16) ^ r;
    return (r >> 8) | (fb << 56);
}

}  // namespace lora_codes_detail

static inline unsigned roundUp(unsigned num, unsigned factor) {
    return (num + factor - 1) / factor * factor;
}

/// 8-bit rotate-and-add checksum.
static inline uint8_t checksum8(const uint8_t* p, const size_t len) {
    uint8_t acc = 0;
    for (size_t i = 0; i < len; ++i) acc = (uint8_t)((uint8_t)((acc >> 1) | (acc << 7)) + p[i]);
    return acc;
}

/// Explicit-header checksum: five parity bits over the 12 header bits
/// h[0] (8) and the low nibble of h[1].
static inline uint8_t headerChecksum(const uint8_t* h) {
    using lora_codes_detail::par;
    const unsigned w = (unsigned)h[0] | ((unsigned)(h[1] & 0x0F) << 8);
    return (uint8_t)((par(w & 0x0F0u) << 4) | (par(w & 0x18Eu) << 3) | (par(w & 0xA49u) << 2) |
                     (par(w & 0x725u) << 1) | par(w & 0xF12u));
}

/// Eight steps of a CCITT-style CRC register with polynomial `poly`.
static inline uint16_t crc16sx(uint16_t crc, const uint16_t poly) {
    for (int k = 0; k < 8; ++k) crc = (uint16_t)((crc & 0x8000u) ? ((crc << 1) ^ poly) : (crc << 1));
    return crc;
}

/// Parity of an 8-bit value.
static inline uint8_t xsum8(uint8_t t) { return (uint8_t)lora_codes_detail::par(t); }

/// SX1272 payload CRC: CRC-16/CCITT (0x1021) over the bytes, masked with
/// the output of an 8-bit LFSR (two steps past the data).
static inline uint16_t sx1272DataChecksum(const uint8_t* data, int length) {
    using lora_codes_detail::crc_mask_step;
    uint16_t res = 0;
    uint8_t v = 0xff;
    for (int i = 0; i < length; ++i) {
        v = crc_mask_step(v);
        res = (uint16_t)(crc16sx(res, 0x1021) ^ data[i]);
    }
    res ^= v;
    v = crc_mask_step(v);
    return (uint16_t)(res ^ (uint16_t)(v << 8));
}

/// SX1232 whitening (Semtech AN1200.18): x^9 + x^5 + 1 LFSR seeded with
/// 0x1FF, its low byte XORed into each data byte, 8 shifts per byte.
static inline void SX1232RadioComputeWhitening(uint8_t* buffer, uint16_t bufferSize) {
    unsigned s = 0x1FF;  // 9-bit state
    for (uint16_t j = 0; j < bufferSize; ++j) {
        buffer[j] ^= (uint8_t)s;
        for (int k = 0; k < 8; ++k) s = (s >> 1) | (((s ^ (s >> 5)) & 1u) << 8);
    }
}

/// SX1272 whitening from the stored sequence: bit i of codeword j takes
/// sequence bit (ofs[i] + j + bitOfs) mod 510, for the 4 + RDD codeword bits.
static inline void Sx1272ComputeWhitening(uint8_t* buffer, uint16_t bufferSize, const int bitOfs,
                                          const int RDD) {
    using namespace lora_codes_detail;
    const int* ofs = RDD == 1 ? kWhitenOfsCr1 : kWhitenOfs;
    for (int j = 0; j < bufferSize; ++j) {
        unsigned mask = 0;
        for (int i = 0; i < 4 + RDD; ++i) {
            const int t = (ofs[i] + j + bitOfs + kWhitenLen) % kWhitenLen;
            mask |= (unsigned)((kWhitenSeq[t >> 6] >> (t & 63)) & 1u) << i;
        }
        buffer[j] ^= (uint8_t)mask;
    }
}

/// SX1272 whitening with the modem's two interleaved 64-bit LFSR states
/// (even / odd codewords), advanced bitOfs codewords before the buffer.
static inline void Sx1272ComputeWhiteningLfsr(uint8_t* buffer, uint16_t bufferSize, const int bitOfs,
                                              const size_t RDD) {
    using namespace lora_codes_detail;
    const uint64_t* seed = RDD == 1 ? kLfsrSeedCr1 : kLfsrSeed;
    uint64_t r[2] = {seed[0], seed[1]};
    const uint8_t m = (uint8_t)(0xff >> (4 - RDD));
    int i = 0;
    for (; i < bitOfs; ++i) r[i & 1] = lfsr64_step(r[i & 1]);
    for (int j = 0; j < bufferSize; ++j, ++i) {
        buffer[j] ^= (uint8_t)(r[i & 1] & m);
        r[i & 1] = lfsr64_step(r[i & 1]);
    }
}

/// Binary -> reflected Gray code.
static inline unsigned short binaryToGray16(unsigned short num) {
    return (unsigned short)(num ^ (num >> 1));
}

/// Reflected Gray code -> binary (prefix XOR over 16 bits).
static inline unsigned short grayToBinary16(unsigned short num) {
    unsigned v = num;
    for (int sh = 8; sh >= 1; sh >>= 1) v ^= v >> sh;
    return (unsigned short)v;
}

/// Hamming(8,4), SX127x bit order: data in bits 0-3, parity bits 4-7 over
/// data masks 0x7, 0xE, 0xB, 0xD.
static inline unsigned char encodeHamming84sx(const unsigned char x) {
    using lora_codes_detail::par;
    return (unsigned char)((x & 0x0F) | (par(x & 0x7u) << 4) | (par(x & 0xEu) << 5) |
                           (par(x & 0xBu) << 6) | (par(x & 0xDu) << 7));
}

/// Hamming(8,4) decode with single-bit correction of the data bits.  The
/// 4-bit syndrome flags `error` when non-zero; syndromes of one flipped
/// data bit correct it, those of one flipped parity bit leave the data, any
/// other sets `bad`.
static inline unsigned char decodeHamming84sx(const unsigned char b, bool& error, bool& bad) {
    using lora_codes_detail::par;
    const unsigned syn = par(b & 0x17u) | (par(b & 0x2Eu) << 1) | (par(b & 0x4Bu) << 2) |
                         (par(b & 0x8Du) << 3);
    if (syn) error = true;
    unsigned flip = 0;
    switch (syn) {
        case 0xD: flip = 1; break;
        case 0x7: flip = 2; break;
        case 0xB: flip = 4; break;
        case 0xE: flip = 8; break;
        case 0x0: case 0x1: case 0x2: case 0x4: case 0x8: break;
        default: bad = true; break;
    }
    return (unsigned char)((b ^ flip) & 0x0F);
}

/// Hamming(7,4), SX127x bit order (the first three parity bits of 8,4).
static inline unsigned char encodeHamming74sx(const unsigned char x) {
    using lora_codes_detail::par;
    return (unsigned char)((x & 0x0F) | (par(x & 0x7u) << 4) | (par(x & 0xEu) << 5) |
                           (par(x & 0xBu) << 6));
}

/// Hamming(7,4) decode: 3-bit syndrome, single data-bit correction.
static inline unsigned char decodeHamming74sx(const unsigned char b, bool& error) {
    using lora_codes_detail::par;
    const unsigned syn = par(b & 0x17u) | (par(b & 0x2Eu) << 1) | (par(b & 0x4Bu) << 2);
    if (syn) error = true;
    unsigned flip = 0;
    switch (syn) {
        case 0x5: flip = 1; break;
        case 0x7: flip = 2; break;
        case 0x3: flip = 4; break;
        case 0x6: flip = 8; break;
        default: break;
    }
    return (unsigned char)((b ^ flip) & 0x0F);
}

/// 5/4 single parity code: `error` when bits 0-4 have odd parity.
static inline unsigned char checkParity54(const unsigned char b, bool& error) {
    if (lora_codes_detail::par(b & 0x1Fu)) error = true;
    return (unsigned char)(b & 0x0F);
}
static inline unsigned char encodeParity54(const unsigned char b) {
    return (unsigned char)((b & 0x0F) | (lora_codes_detail::par(b & 0x0Fu) << 4));
}

/// 6/4 double parity code: parity bits 4 and 5 over data masks 0x7, 0xE.
static inline unsigned char checkParity64(const unsigned char b, bool& error) {
    using lora_codes_detail::par;
    if (par(b & 0x17u) | par(b & 0x2Eu)) error = true;
    return (unsigned char)(b & 0x0F);
}
static inline unsigned char encodeParity64(const unsigned char b) {
    using lora_codes_detail::par;
    return (unsigned char)((par(b & 0x7u) << 4) | (par(b & 0xEu) << 5) | (b & 0x0F));
}

/// SX127x diagonal interleaver: per block of PPM codewords, symbol `bit`
/// gathers bit `bit` of codewords (cw + bit) mod PPM into its bit cw.
static inline void diagonalInterleaveSx(const uint8_t* codewords, const size_t numCodewords,
                                        uint16_t* symbols, const size_t PPM, const size_t RDD) {
    const size_t nb = 4 + RDD;
    for (size_t k = 0; k < numCodewords / PPM; ++k) {
        const uint8_t* cw = codewords + k * PPM;
        for (size_t bit = 0; bit < nb; ++bit) {
            unsigned s = 0;
            for (size_t c = 0; c < PPM; ++c) s |= (unsigned)((cw[(c + bit) % PPM] >> bit) & 1u) << c;
            symbols[k * nb + bit] = (uint16_t)s;
        }
    }
}

/// Its inverse: OR-accumulates into codewords (zeroed by the caller).
static inline void diagonalDeterleaveSx(const uint16_t* symbols, const size_t numSymbols,
                                        uint8_t* codewords, const size_t PPM, const size_t RDD) {
    const size_t nb = 4 + RDD;
    for (size_t k = 0; k < numSymbols / nb; ++k) {
        uint8_t* cw = codewords + k * PPM;
        for (size_t bit = 0; bit < nb; ++bit) {
            const unsigned s = symbols[k * nb + bit];
            for (size_t c = 0; c < PPM; ++c) cw[(c + bit) % PPM] |= (uint8_t)(((s >> c) & 1u) << bit);
        }
    }
}

/// The reference's second deinterleaver form, kept with its exact indexing:
/// per block it walks m over PPM symbols starting at the block's first
/// symbol and places bit k of symbol m into bit m of codeword (m + k) mod PPM.
static inline void diagonalDeterleaveSx2(const uint16_t* symbols, const size_t numSymbols,
                                         uint8_t* codewords, const size_t PPM, const size_t RDD) {
    const size_t nb = RDD + 4;
    for (size_t x = 0; x < numSymbols / nb; ++x) {
        uint8_t* cw = codewords + x * PPM;
        const uint16_t* sy = symbols + x * nb;
        for (size_t m = 0; m < PPM; ++m) {
            const unsigned s = sy[m];
            for (size_t k = 0; k < PPM; ++k) cw[(m + k) % PPM] |= (uint8_t)(((s >> k) & 1u) << m);
        }
    }
}
