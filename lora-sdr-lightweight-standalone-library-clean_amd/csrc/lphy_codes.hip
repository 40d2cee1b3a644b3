// lphy_codes.hip — batch forms of the reference's LoRaCodes.hpp helpers on
// the GPU: Gray mapping, the SX127x diagonal
// (de)interleaver, the three whitening generators, the Hamming / parity
// codes and the checksums, over `frames` rows of a fixed stride in device
// memory.  Each kernel cites the helper whose results it reproduces bit for
// bit (tests/test_gpu_codes.py against the oracle, which
// tests/test_oracle_vs_reference.py pins to the reference header).
//
// All of these are byte/halfword streams: one thread per output element,
// coalesced along the row; they run at memory speed and need no LDS.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>

#include "../../include/lphy_hip.h"

namespace {

#define CODES_OK(x)                                                        \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            fprintf(stderr, "lphy_codes: %s failed: %s (%s:%d)\n", #x,     \
                    hipGetErrorString(e_), __FILE__, __LINE__);            \
            return -EIO;                                                   \
        }                                                                  \
    } while (0)

__device__ __forceinline__ unsigned par(unsigned v) { return __popc(v) & 1u; }

constexpr unsigned kThreads = 256;

unsigned blocks_for(unsigned long long n) { return (unsigned)((n + kThreads - 1) / kThreads); }

// --------------------------------------------------------------- Gray map
// binaryToGray16 / grayToBinary16 (LoRaCodes.hpp:201-222)
__global__ void k_gray(uint16_t* s, unsigned long long n, int to_binary) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned v = s[i];
    if (to_binary) {
        v ^= v >> 8;
        v ^= v >> 4;
        v ^= v >> 2;
        v ^= v >> 1;
    } else {
        v ^= v >> 1;
    }
    s[i] = (uint16_t)v;
}

// --------------------------------------------------- diagonal interleaver
// diagonalInterleaveSx (LoRaCodes.hpp:376-393): per block of PPM codewords,
// symbol `bit` holds in its bit c bit `bit` of codeword (c + bit) mod PPM.
// One thread per output symbol.
__global__ void k_interleave(const uint8_t* cw, unsigned long long cw_stride, uint16_t* sy,
                             unsigned long long sy_stride, unsigned long long frames, unsigned blocks,
                             unsigned ppm, unsigned nb) {
    const unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long per = (unsigned long long)blocks * nb;
    if (t >= frames * per) return;
    const unsigned long long f = t / per;
    const unsigned o = (unsigned)(t - f * per);
    const unsigned blk = o / nb, bit = o - blk * nb;
    const uint8_t* c = cw + f * cw_stride + (unsigned long long)blk * ppm;
    unsigned s = 0, src = bit % ppm;
    for (unsigned k = 0; k < ppm; ++k) {
        s |= ((unsigned)(c[src] >> bit) & 1u) << k;
        if (++src == ppm) src = 0;
    }
    sy[f * sy_stride + o] = (uint16_t)s;
}

// diagonalDeterleaveSx (LoRaCodes.hpp:396-412), writing what the reference
// leaves in a zeroed codeword buffer: codeword d gets, in bit `bit`, bit
// (d - bit) mod PPM of symbol `bit`.  One thread per output codeword.
__global__ void k_deinterleave(const uint16_t* sy, unsigned long long sy_stride, uint8_t* cw,
                               unsigned long long cw_stride, unsigned long long frames, unsigned blocks,
                               unsigned ppm, unsigned nb) {
    const unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long per = (unsigned long long)blocks * ppm;
    if (t >= frames * per) return;
    const unsigned long long f = t / per;
    const unsigned o = (unsigned)(t - f * per);
    const unsigned blk = o / ppm, d = o - blk * ppm;
    const uint16_t* s = sy + f * sy_stride + (unsigned long long)blk * nb;
    unsigned v = 0;
    for (unsigned bit = 0; bit < nb; ++bit) {
        const unsigned sh = (d + ppm - bit % ppm) % ppm;
        v |= (((unsigned)s[bit] >> sh) & 1u) << bit;
    }
    cw[f * cw_stride + o] = (uint8_t)v;
}

// -------------------------------------------------------------- whitening
// The masks do not depend on the data: byte j of every row is XORed with
// the generator's output for position j, computed by the thread itself.
//   LPHY_WHITEN_SX1232       SX1232RadioComputeWhitening (LoRaCodes.hpp:111-137):
//                            9-bit x^9 + x^5 + 1 LFSR from 0x1FF, 8 steps a byte
//   LPHY_WHITEN_SX1272       Sx1272ComputeWhitening (:147-167): stored 510-bit sequence
//   LPHY_WHITEN_SX1272_LFSR  Sx1272ComputeWhiteningLfsr (:176-189): two interleaved
//                            64-bit LFSR states, one step per codeword
__constant__ unsigned long long c_whiten_seq[8] = {
    0x0102291EA751AAFFull, 0xD24B050A8D643A17ull, 0x5B279B671120B8F4ull, 0x032B37B9F6FB55A2ull,
    0x994E0F87E95E2D16ull, 0x7CBCFC7631984C26ull, 0x281C8E4F0DAEF7F9ull, 0x1741886EB7733B15ull};
__constant__ int c_whiten_ofs[8] = {6, 4, 2, 0, -112, -114, -302, -34};
__constant__ int c_whiten_ofs1[5] = {6, 4, 2, 0, -360};

__device__ __forceinline__ unsigned long long lfsr64_step(unsigned long long r) {
    return (r >> 8) | (((r >> 32) ^ (r >> 24) ^ (r >> 16) ^ r) << 56);  // poly 0x1D
}

__global__ void k_whiten(uint8_t* b, unsigned long long stride, unsigned long long frames, unsigned len,
                         int kind, int bit_ofs, unsigned rdd) {
    const unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= frames * len) return;
    const unsigned long long f = t / len;
    const unsigned j = (unsigned)(t - f * len);
    unsigned mask = 0;
    if (kind == LPHY_WHITEN_SX1232) {
        unsigned s = 0x1FF;
        for (unsigned k = 0; k < 8u * j; ++k) s = (s >> 1) | (((s ^ (s >> 5)) & 1u) << 8);
        mask = s & 0xFF;
    } else if (kind == LPHY_WHITEN_SX1272) {
        const int* ofs = rdd == 1 ? c_whiten_ofs1 : c_whiten_ofs;
        for (unsigned i = 0; i < 4 + rdd; ++i) {
            const int q = (ofs[i] + (int)j + bit_ofs + 510) % 510;
            mask |= (unsigned)((c_whiten_seq[q >> 6] >> (q & 63)) & 1ull) << i;
        }
        mask &= 0xFF;
    } else {
        // codeword position p = bit_ofs + j uses state p & 1 after p >> 1 steps
        const bool one = rdd == 1;
        const unsigned p = (unsigned)bit_ofs + j;
        unsigned long long r = (p & 1u) ? (one ? 0xF8ECFEEFEFEFEFEFull : 0xE85C2EFFFFFFFFFFull)
                                        : (one ? 0x05121100F8ECFEEFull : 0x6572D100E85C2EFFull);
        for (unsigned k = 0; k < (p >> 1); ++k) r = lfsr64_step(r);
        mask = (unsigned)(r & (0xffu >> (4 - rdd)));
    }
    b[f * stride + j] ^= (uint8_t)mask;
}

// -------------------------------------------------- Hamming / parity codes
// LoRaCodes.hpp:229-371, one byte per thread; decoders write their flags
// (bit 0 error, bit 1 bad) to `flags` when given.
__global__ void k_hamming(uint8_t* b, unsigned long long n, int op, uint8_t* flags) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned x = b[i];
    unsigned out = 0, fl = 0;
    switch (op) {
        case LPHY_CODE_ENC84:  // encodeHamming84sx :229-242
            out = (x & 0xF) | (par(x & 0x7) << 4) | (par(x & 0xE) << 5) | (par(x & 0xB) << 6) |
                  (par(x & 0xD) << 7);
            break;
        case LPHY_CODE_DEC84: {  // decodeHamming84sx :250-281
            const unsigned syn = par(x & 0x17) | (par(x & 0x2E) << 1) | (par(x & 0x4B) << 2) |
                                 (par(x & 0x8D) << 3);
            unsigned flip = 0;
            if (syn) fl |= 1;
            switch (syn) {
                case 0xD: flip = 1; break;
                case 0x7: flip = 2; break;
                case 0xB: flip = 4; break;
                case 0xE: flip = 8; break;
                case 0x0: case 0x1: case 0x2: case 0x4: case 0x8: break;
                default: fl |= 2; break;
            }
            out = (x ^ flip) & 0xF;
            break;
        }
        case LPHY_CODE_ENC74:  // encodeHamming74sx :287-297
            out = (x & 0xF) | (par(x & 0x7) << 4) | (par(x & 0xE) << 5) | (par(x & 0xB) << 6);
            break;
        case LPHY_CODE_DEC74: {  // decodeHamming74sx :306-334
            const unsigned syn = par(x & 0x17) | (par(x & 0x2E) << 1) | (par(x & 0x4B) << 2);
            unsigned flip = 0;
            if (syn) fl |= 1;
            switch (syn) {
                case 0x5: flip = 1; break;
                case 0x7: flip = 2; break;
                case 0x3: flip = 4; break;
                case 0x6: flip = 8; break;
                default: break;
            }
            out = (x ^ flip) & 0xF;
            break;
        }
        case LPHY_CODE_ENCP54:  // encodeParity54 :347-350
            out = (x & 0xF) | (par(x & 0xF) << 4);
            break;
        case LPHY_CODE_CHKP54:  // checkParity54 :340-345
            if (par(x & 0x1F)) fl |= 1;
            out = x & 0xF;
            break;
        case LPHY_CODE_ENCP64:  // encodeParity64 :367-371
            out = (par(x & 0x7) << 4) | (par(x & 0xE) << 5) | (x & 0xF);
            break;
        default:  // LPHY_CODE_CHKP64, checkParity64 :357-365
            if (par(x & 0x17) | par(x & 0x2E)) fl |= 1;
            out = x & 0xF;
            break;
    }
    b[i] = (uint8_t)out;
    if (flags) flags[i] = (uint8_t)fl;
}

// -------------------------------------------------------------- checksums
// One thread per row:
//   LPHY_SUM_SX1272_CRC  sx1272DataChecksum (LoRaCodes.hpp:69-105)
//   LPHY_SUM_HEADER      headerChecksum (:43-67) of the row's first 2 bytes
//   LPHY_SUM_CHECKSUM8   checksum8 (:32-41)
__device__ __forceinline__ unsigned crc_step8(unsigned crc) {
    for (int b = 0; b < 8; ++b) crc = (crc & 0x8000) ? ((crc << 1) ^ 0x1021) : (crc << 1);
    return crc & 0xFFFF;
}

__global__ void k_checksum(const uint8_t* b, unsigned long long stride, unsigned long long frames,
                           unsigned len, int kind, uint16_t* out) {
    const unsigned long long f = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= frames) return;
    const uint8_t* p = b + f * stride;
    unsigned r = 0;
    if (kind == LPHY_SUM_SX1272_CRC) {
        unsigned v = 0xFF;
        for (unsigned i = 0; i < len; ++i) {
            r = crc_step8(r) ^ p[i];
            v = (par(v & 0xB8) | (v << 1)) & 0xFF;
        }
        r ^= v;
        v = (par(v & 0xB8) | (v << 1)) & 0xFF;
        r = (r ^ (v << 8)) & 0xFFFF;
    } else if (kind == LPHY_SUM_HEADER) {
        // five parity bits over h[0] (a: bits 4-7, b: bits 0-3) and the low
        // nibble c of h[1], the reference's expressions
        const unsigned a0 = (p[0] >> 4) & 1, a1 = (p[0] >> 5) & 1, a2 = (p[0] >> 6) & 1,
                       a3 = (p[0] >> 7) & 1;
        const unsigned b0 = (p[0] >> 0) & 1, b1 = (p[0] >> 1) & 1, b2 = (p[0] >> 2) & 1,
                       b3 = (p[0] >> 3) & 1;
        const unsigned c0 = (p[1] >> 0) & 1, c1 = (p[1] >> 1) & 1, c2 = (p[1] >> 2) & 1,
                       c3 = (p[1] >> 3) & 1;
        const unsigned x0 = a3 ^ a2 ^ a1 ^ a0;
        const unsigned x1 = a3 ^ b3 ^ b2 ^ b1 ^ c0;
        const unsigned x2 = a2 ^ b3 ^ b0 ^ c3 ^ c1;
        const unsigned x3 = a1 ^ b0 ^ b2 ^ c0 ^ c1 ^ c2;
        const unsigned x4 = a0 ^ b1 ^ c3 ^ c2 ^ c1 ^ c0;
        r = (x0 << 4) | (x1 << 3) | (x2 << 2) | (x3 << 1) | x4;
    } else {
        unsigned x = 0;
        for (unsigned i = 0; i < len; ++i) {
            x = (((x & 1) << 7) | (x >> 1)) & 0xFF;
            x = (x + p[i]) & 0xFF;
        }
        r = x;
    }
    out[f] = (uint16_t)r;
}

// lora_encode (LoRaEncoder.cpp:6-18): one thread per byte, two Hamming(8,4)
// codewords out, high nibble first.
__device__ __forceinline__ unsigned enc84(unsigned x) {
    return (x & 0xF) | (par(x & 0x7) << 4) | (par(x & 0xE) << 5) | (par(x & 0xB) << 6) | (par(x & 0xD) << 7);
}

__global__ void k_lora_encode(const uint8_t* b, unsigned long long stride, unsigned long long frames, unsigned len,
                              uint16_t* sy, unsigned long long sy_stride) {
    const unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= frames * len) return;
    const unsigned long long f = t / len;
    const unsigned j = (unsigned)(t - f * len);
    const unsigned x = b[f * stride + j];
    uint16_t* o = sy + f * sy_stride + 2ull * j;
    o[0] = (uint16_t)enc84(x >> 4);
    o[1] = (uint16_t)enc84(x & 0xF);
}

}  // namespace

extern "C" {

int lphy_hip_lora_encode_batch(const uint8_t* d_bytes, size_t frames, size_t stride, size_t len,
                               uint16_t* d_syms, size_t sym_stride, void* stream) {
    if (len > stride || len > 0x7fffffff || (frames && len && (!d_bytes || !d_syms))) return -EINVAL;
    if (2 * len > sym_stride) return -ERANGE;
    if (!frames || !len) return 0;
    hipLaunchKernelGGL(k_lora_encode, dim3(blocks_for(frames * len)), dim3(kThreads), 0, (hipStream_t)stream,
                       d_bytes, (unsigned long long)stride, (unsigned long long)frames, (unsigned)len, d_syms,
                       (unsigned long long)sym_stride);
    CODES_OK(hipGetLastError());
    return 0;
}

int lphy_hip_gray_batch(uint16_t* d_syms, size_t count, int to_binary, void* stream) {
    if (!d_syms && count) return -EINVAL;
    if (!count) return 0;
    hipLaunchKernelGGL(k_gray, dim3(blocks_for(count)), dim3(kThreads), 0, (hipStream_t)stream, d_syms,
                       (unsigned long long)count, to_binary ? 1 : 0);
    CODES_OK(hipGetLastError());
    return 0;
}

int lphy_hip_interleave_batch(const uint8_t* d_cw, size_t frames, size_t cw_stride, size_t cw_per_frame,
                              uint16_t* d_syms, size_t sym_stride, unsigned ppm, unsigned rdd,
                              void* stream) {
    if (ppm < 1 || ppm > 16 || rdd > 4 || (frames && (!d_cw || !d_syms))) return -EINVAL;
    const unsigned long long blocks = cw_per_frame / ppm, nb = 4 + rdd;
    if (blocks * nb > sym_stride || cw_per_frame > cw_stride) return -ERANGE;
    if (!frames || !blocks) return 0;
    hipLaunchKernelGGL(k_interleave, dim3(blocks_for(frames * blocks * nb)), dim3(kThreads), 0,
                       (hipStream_t)stream, d_cw, (unsigned long long)cw_stride, d_syms,
                       (unsigned long long)sym_stride, (unsigned long long)frames, (unsigned)blocks, ppm,
                       (unsigned)nb);
    CODES_OK(hipGetLastError());
    return 0;
}

int lphy_hip_deinterleave_batch(const uint16_t* d_syms, size_t frames, size_t sym_stride,
                                size_t syms_per_frame, uint8_t* d_cw, size_t cw_stride, unsigned ppm,
                                unsigned rdd, void* stream) {
    if (ppm < 1 || ppm > 16 || rdd > 4 || (frames && (!d_cw || !d_syms))) return -EINVAL;
    const unsigned long long nb = 4 + rdd, blocks = syms_per_frame / nb;
    if (blocks * ppm > cw_stride || syms_per_frame > sym_stride) return -ERANGE;
    if (!frames || !blocks) return 0;
    hipLaunchKernelGGL(k_deinterleave, dim3(blocks_for(frames * blocks * ppm)), dim3(kThreads), 0,
                       (hipStream_t)stream, d_syms, (unsigned long long)sym_stride, d_cw,
                       (unsigned long long)cw_stride, (unsigned long long)frames, (unsigned)blocks, ppm,
                       (unsigned)nb);
    CODES_OK(hipGetLastError());
    return 0;
}

int lphy_hip_whiten_batch(uint8_t* d_bytes, size_t frames, size_t stride, size_t len, int kind,
                          int bit_ofs, unsigned rdd, void* stream) {
    if (kind != LPHY_WHITEN_SX1232 && kind != LPHY_WHITEN_SX1272 && kind != LPHY_WHITEN_SX1272_LFSR)
        return -EINVAL;
    if (kind != LPHY_WHITEN_SX1232 && rdd > 4) return -EINVAL;
    if (bit_ofs < 0 || len > 65535 || len > stride || (frames && len && !d_bytes)) return -EINVAL;
    if (!frames || !len) return 0;
    hipLaunchKernelGGL(k_whiten, dim3(blocks_for(frames * len)), dim3(kThreads), 0, (hipStream_t)stream,
                       d_bytes, (unsigned long long)stride, (unsigned long long)frames, (unsigned)len, kind,
                       bit_ofs, rdd);
    CODES_OK(hipGetLastError());
    return 0;
}

int lphy_hip_hamming_batch(uint8_t* d_bytes, size_t count, int op, uint8_t* d_flags, void* stream) {
    if (op < LPHY_CODE_ENC84 || op > LPHY_CODE_CHKP64 || (count && !d_bytes)) return -EINVAL;
    if (!count) return 0;
    hipLaunchKernelGGL(k_hamming, dim3(blocks_for(count)), dim3(kThreads), 0, (hipStream_t)stream, d_bytes,
                       (unsigned long long)count, op, d_flags);
    CODES_OK(hipGetLastError());
    return 0;
}

int lphy_hip_checksum_batch(const uint8_t* d_bytes, size_t frames, size_t stride, size_t len, int kind,
                            uint16_t* d_out, void* stream) {
    if (kind != LPHY_SUM_SX1272_CRC && kind != LPHY_SUM_HEADER && kind != LPHY_SUM_CHECKSUM8) return -EINVAL;
    if (kind == LPHY_SUM_HEADER) len = 2;
    if (len > stride || len > 0x7fffffff || (frames && (!d_bytes || !d_out))) return -EINVAL;
    if (!frames) return 0;
    hipLaunchKernelGGL(k_checksum, dim3(blocks_for(frames)), dim3(kThreads), 0, (hipStream_t)stream, d_bytes,
                       (unsigned long long)stride, (unsigned long long)frames, (unsigned)len, kind, d_out);
    CODES_OK(hipGetLastError());
    return 0;
}

}  // extern "C"
