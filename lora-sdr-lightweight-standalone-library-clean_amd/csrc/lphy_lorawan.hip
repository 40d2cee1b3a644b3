// lphy_lorawan.hip — the LoRaWAN MAC helpers of the reference
// (src/lorawan/lorawan.cpp) batched on the GPU:
// compute_mic (lorawan.cpp:35-98: AES-128 CMAC over B0 || data) for many
// frames, and parse_frame's checks (lorawan.cpp:150-176) on the decoded
// bytes the demodulator leaves in HBM.  Bit-exact to the reference
// (tests/test_gpu_lorawan.py against the oracle, which
// tests/test_oracle_vs_reference.py pins to lorawan.cpp + tiny-AES).
//
// One thread per frame: a CMAC is a chain of AES blocks, so the parallelism
// is across frames.  AES-128 runs from one 1 KiB "T-table" (SubBytes and
// MixColumns of one input byte, LoRa-independent FIPS-197 algebra) held in
// LDS as 32 replicas, entry x of replica c at dword 32x + c: lane l reads
// replica l & 31, so the 32 lanes of a ds_read_b32 group always hit 32
// different banks whatever bytes they look up (no conflicts).  The other
// three tables are byte rotations of the first (v_alignbit).  The table is
// derived in the prologue from the field inverse, not loaded.  Round keys
// (44 dwords) live in VGPRs.  Each workgroup loops over frames
// (grid-stride), so the 32 KiB table build is paid once per workgroup.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>

#include "../../include/lphy_hip.h"

namespace {

#define LW_OK(x)                                                           \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            fprintf(stderr, "lphy_lorawan: %s failed: %s (%s:%d)\n", #x,   \
                    hipGetErrorString(e_), __FILE__, __LINE__);            \
            return -EIO;                                                   \
        }                                                                  \
    } while (0)

constexpr unsigned kThreads = 256;
constexpr unsigned kCopies = 32;
constexpr unsigned kMaxBlocks = 2048;  // 8 workgroups per CU, grid-stride beyond

// ---------------------------------------------------------------- AES-128
__device__ __forceinline__ unsigned gmul2(unsigned a) { return ((a << 1) ^ ((a & 0x80) ? 0x1B : 0)) & 0xFF; }

__device__ unsigned gmul(unsigned a, unsigned b) {
    unsigned r = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) r ^= a;
        a = gmul2(a);
        b >>= 1;
    }
    return r;
}

// S-box entry by definition: affine map of the inverse in GF(2^8).
__device__ unsigned sbox_entry(unsigned x) {
    unsigned inv = 1, p = x;
    for (int e = 254; e; e >>= 1) {
        if (e & 1) inv = gmul(inv, p);
        p = gmul(p, p);
    }
    if (!x) inv = 0;
    unsigned y = 0x63;
    for (int k = 0; k < 5; ++k) y ^= ((inv << k) | (inv >> ((8 - k) & 7))) & 0xFF;
    return y;
}

// T[x] for byte row 0 of a column, little-endian packed: (2s, s, s, 3s).
__device__ void build_table(uint32_t* lds) {
    for (unsigned x = threadIdx.x; x < 256; x += blockDim.x) {
        const unsigned s = sbox_entry(x), s2 = gmul2(s);
        const uint32_t t = s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
        for (unsigned c = 0; c < kCopies; ++c) lds[x * kCopies + c] = t;
    }
    __syncthreads();
}

struct Tab {
    const uint32_t* t;  // this lane's replica
    __device__ __forceinline__ uint32_t T(uint32_t x) const { return t[x * kCopies]; }
    __device__ __forceinline__ uint32_t S(uint32_t x) const { return (t[x * kCopies] >> 8) & 0xFF; }
};

__device__ __forceinline__ uint32_t rotl(uint32_t v, unsigned r) { return __builtin_amdgcn_alignbit(v, v, 32 - r); }
__device__ __forceinline__ uint32_t byte_of(uint32_t v, unsigned k) { return (v >> (8 * k)) & 0xFF; }

// FIPS-197 5.2 key expansion; words little-endian (key byte 4i in bits 0-7).
__device__ __forceinline__ void expand_key(const Tab& tb, const uint32_t k[4], uint32_t rk[44]) {
    constexpr uint32_t rcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1B, 0x36};
#pragma unroll
    for (int i = 0; i < 4; ++i) rk[i] = k[i];
#pragma unroll
    for (int i = 4; i < 44; ++i) {
        uint32_t t = rk[i - 1];
        if (i % 4 == 0)  // SubWord(RotWord(t)) ^ Rcon
            t = (tb.S(byte_of(t, 1)) | tb.S(byte_of(t, 2)) << 8 | tb.S(byte_of(t, 3)) << 16 |
                 tb.S(byte_of(t, 0)) << 24) ^ rcon[i / 4 - 1];
        rk[i] = rk[i - 4] ^ t;
    }
}

// FIPS-197 5.1 cipher: new column c takes row r from old column c + r
// (ShiftRows); rows 1-3 of the MixColumns contribution are the row-0 table
// rotated by 8r bits.
__device__ __forceinline__ void encrypt(const Tab& tb, const uint32_t rk[44], uint32_t s[4]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) s[c] ^= rk[c];
#pragma unroll
    for (int r = 1; r < 10; ++r) {
        uint32_t t[4];
#pragma unroll
        for (int c = 0; c < 4; ++c)
            t[c] = tb.T(byte_of(s[c], 0)) ^ rotl(tb.T(byte_of(s[(c + 1) & 3], 1)), 8) ^
                   rotl(tb.T(byte_of(s[(c + 2) & 3], 2)), 16) ^ rotl(tb.T(byte_of(s[(c + 3) & 3], 3)), 24) ^
                   rk[4 * r + c];
#pragma unroll
        for (int c = 0; c < 4; ++c) s[c] = t[c];
    }
    uint32_t t[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
        t[c] = (tb.S(byte_of(s[c], 0)) | tb.S(byte_of(s[(c + 1) & 3], 1)) << 8 |
                tb.S(byte_of(s[(c + 2) & 3], 2)) << 16 | tb.S(byte_of(s[(c + 3) & 3], 3)) << 24) ^
               rk[40 + c];
#pragma unroll
    for (int c = 0; c < 4; ++c) s[c] = t[c];
}

// CMAC doubling of a little-endian-packed block read as one big-endian
// 128-bit number (lorawan.cpp:15-31).
__device__ __forceinline__ void cmac_double(const uint32_t in[4], uint32_t out[4]) {
    uint32_t b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = __builtin_bswap32(in[i]);
    const uint32_t msb = b[0] >> 31;
    uint32_t o[4];
    o[0] = (b[0] << 1) | (b[1] >> 31);
    o[1] = (b[1] << 1) | (b[2] >> 31);
    o[2] = (b[2] << 1) | (b[3] >> 31);
    o[3] = (b[3] << 1) ^ (msb ? 0x87u : 0u);
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = __builtin_bswap32(o[i]);
}

// Up to 16 bytes at p (n >= 1 of them valid) as 4 little-endian words, the
// bytes past n zero.  Only 4-byte-aligned dwords holding at least one valid
// byte are read: such a dword never leaves the page its valid byte is on.
__device__ __forceinline__ void load16(const uint8_t* p, unsigned n, uint32_t w[4]) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    const unsigned sh = (unsigned)(a & 3) * 8;
    const unsigned last = ((unsigned)(a & 3) + n - 1) >> 2;
    uint32_t d[5];
#pragma unroll
    for (unsigned k = 0; k < 5; ++k) d[k] = q[k < last ? k : last];
#pragma unroll
    for (unsigned k = 0; k < 4; ++k) {
        const uint32_t v = __builtin_amdgcn_alignbit(d[k + 1], d[k], sh);
        const int vb = (int)n - 4 * (int)k;
        w[k] = vb >= 4 ? v : (vb <= 0 ? 0u : v & ((1u << (8 * vb)) - 1u));
    }
}

// lorawan.cpp:35-98 for one frame.
__device__ uint32_t frame_mic(const Tab& tb, const uint32_t key[4], bool uplink, uint32_t devaddr, uint32_t fcnt,
                              const uint8_t* data, uint32_t len) {
    uint32_t rk[44];
    expand_key(tb, key, rk);
    uint32_t K1[4] = {0, 0, 0, 0}, K2[4];
    encrypt(tb, rk, K1);  // L = E_K(0)
    cmac_double(K1, K1);
    cmac_double(K1, K2);
    // B0 (lorawan.cpp:46-58), bytes 4j..4j+3 of the block in word j
    uint32_t X[4] = {0x49u, (uplink ? 0u : 1u) << 8 | (devaddr & 0xFFFFu) << 16,
                     (devaddr >> 16) | (fcnt & 0xFFFFu) << 16,
                     (fcnt >> 16) | ((len >> 8) & 0xFFu) << 16 | (len & 0xFFu) << 24};
    const uint32_t total = len + 16, nblk = (total + 15) / 16;
    if (nblk == 1) {  // B0 is also the last block (len == 0)
#pragma unroll
        for (int j = 0; j < 4; ++j) X[j] ^= K1[j];
        encrypt(tb, rk, X);
        return X[0];
    }
    encrypt(tb, rk, X);
    for (uint32_t b = 1; b < nblk; ++b) {
        const uint32_t have = total - 16 * b < 16 ? total - 16 * b : 16;
        uint32_t m[4];
        load16(data + 16 * (b - 1), have, m);
        if (b + 1 == nblk) {
            if (have < 16) m[have >> 2] |= 0x80u << (8 * (have & 3));
            const uint32_t* K = have == 16 ? K1 : K2;
#pragma unroll
            for (int j = 0; j < 4; ++j) m[j] ^= K[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) X[j] ^= m[j];
        encrypt(tb, rk, X);
    }
    return X[0];  // tag bytes 0-3, little-endian (lorawan.cpp:94-97)
}

__device__ __forceinline__ void load_key(const uint8_t* keys, uint32_t idx, uint32_t k[4]) {
    const uint4 v = *reinterpret_cast<const uint4*>(keys + 16ull * idx);
    k[0] = v.x, k[1] = v.y, k[2] = v.z, k[3] = v.w;
}

__device__ __forceinline__ Tab lane_tab(const uint32_t* lds) { return Tab{lds + (threadIdx.x & (kCopies - 1))}; }

__global__ void __launch_bounds__(kThreads) k_lw_mic(uint8_t* bytes, const lphy_lorawan_desc* desc,
                                                     unsigned long long frames, const uint8_t* keys,
                                                     unsigned long long nkeys, uint32_t* mic, unsigned flags) {
    extern __shared__ uint32_t lds[];
    build_table(lds);
    const Tab tb = lane_tab(lds);
    for (unsigned long long f = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; f < frames;
         f += (unsigned long long)gridDim.x * blockDim.x) {
        const lphy_lorawan_desc d = desc[f];
        if (d.key >= nkeys) {  // no such key: MIC 0, nothing appended
            if (mic) mic[f] = 0;
            continue;
        }
        uint32_t k[4];
        load_key(keys, d.key, k);
        uint8_t* data = bytes + d.offset;
        const uint32_t m = frame_mic(tb, k, d.uplink != 0, d.devaddr, d.fcnt, data, d.len);
        if (mic) mic[f] = m;
        if (flags & LPHY_LW_APPEND) {
#pragma unroll
            for (int j = 0; j < 4; ++j) data[d.len + j] = (uint8_t)(m >> (8 * j));
        }
    }
}

// lorawan.cpp:150-176 on one row of decoded bytes.
__global__ void __launch_bounds__(kThreads) k_lw_parse(const uint8_t* bytes, unsigned long long frames,
                                                       unsigned long long stride, const uint32_t* lens,
                                                       uint32_t len0, const uint8_t* keys,
                                                       unsigned long long nkeys, const uint32_t* key_index,
                                                       lphy_lorawan_frame* out) {
    extern __shared__ uint32_t lds[];
    build_table(lds);
    const Tab tb = lane_tab(lds);
    for (unsigned long long f = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; f < frames;
         f += (unsigned long long)gridDim.x * blockDim.x) {
        const uint32_t len = lens ? lens[f] : len0;
        const uint8_t* row = bytes + f * stride;
        uint32_t rec[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const uint32_t kidx = key_index ? key_index[f] : 0u;
        // a row length past the row (or past the 16-bit record fields) would
        // read beyond the row: -ERANGE, nothing read
        if (len < 12 || len > stride || len > 65535u) {
            rec[0] = (uint32_t)-ERANGE;
        } else if (kidx >= nkeys) {
            rec[0] = (uint32_t)-ENOKEY;
        } else {
            uint32_t h[4], t[4];
            load16(row, 8, h);
            load16(row + len - 4, 4, t);
            const uint32_t mhdr = h[0] & 0xFF, devaddr = (h[0] >> 8) | (h[1] << 24);
            const uint32_t fctrl = (h[1] >> 8) & 0xFF, fcnt = h[1] >> 16, fol = fctrl & 0x0F;
            uint32_t k[4];
            load_key(keys, kidx, k);
            const uint32_t calc = frame_mic(tb, k, ((mhdr >> 5) & 1) == 0, devaddr, fcnt, row, len - 4);
            rec[1] = devaddr, rec[2] = t[0], rec[3] = calc;
            rec[6] = fcnt | mhdr << 16 | fctrl << 24;
            rec[7] = fol;
            if (t[0] != calc) {
                rec[0] = (uint32_t)-EINVAL;
            } else if (8 + fol > len - 4) {
                rec[0] = (uint32_t)-ERANGE;
            } else {
                rec[4] = 8 + fol;
                rec[5] = len - 12 - fol;
                rec[0] = rec[5];
            }
        }
        uint4* o = reinterpret_cast<uint4*>(out + f);
        o[0] = make_uint4(rec[0], rec[1], rec[2], rec[3]);
        o[1] = make_uint4(rec[4], rec[5], rec[6], rec[7]);
    }
}

unsigned grid_for(unsigned long long frames) {
    const unsigned long long b = (frames + kThreads - 1) / kThreads;
    return (unsigned)(b < kMaxBlocks ? b : kMaxBlocks);
}

constexpr size_t kLds = 256 * kCopies * sizeof(uint32_t);  // 32 KiB

}  // namespace

static_assert(sizeof(lphy_lorawan_desc) == 32, "descriptor layout");
static_assert(sizeof(lphy_lorawan_frame) == 32, "record layout");

extern "C" {

int lphy_hip_lorawan_mic_batch(uint8_t* d_bytes, const lphy_lorawan_desc* d_desc, size_t frames,
                               const uint8_t* d_keys, size_t nkeys, uint32_t* d_mic, unsigned flags,
                               void* stream) {
    if (!frames) return 0;
    if (!d_bytes || !d_desc || !d_keys || !nkeys || (!d_mic && !(flags & LPHY_LW_APPEND))) return -EINVAL;
    if (flags & ~LPHY_LW_APPEND) return -EINVAL;
    if (reinterpret_cast<uintptr_t>(d_keys) & 15 || reinterpret_cast<uintptr_t>(d_desc) & 15) return -EINVAL;
    hipLaunchKernelGGL(k_lw_mic, dim3(grid_for(frames)), dim3(kThreads), kLds, (hipStream_t)stream, d_bytes,
                       d_desc, (unsigned long long)frames, d_keys, (unsigned long long)nkeys, d_mic, flags);
    LW_OK(hipGetLastError());
    return 0;
}

int lphy_hip_lorawan_parse_batch(const uint8_t* d_bytes, size_t frames, size_t stride,
                                 const uint32_t* d_lens, size_t len, const uint8_t* d_keys, size_t nkeys,
                                 const uint32_t* d_key_index, lphy_lorawan_frame* d_out, void* stream) {
    if (!frames) return 0;
    if (!d_bytes || !d_keys || !nkeys || !d_out) return -EINVAL;
    if (!d_lens && (len > stride || len > 65535)) return -EINVAL;
    if (reinterpret_cast<uintptr_t>(d_keys) & 15 || reinterpret_cast<uintptr_t>(d_out) & 15) return -EINVAL;
    hipLaunchKernelGGL(k_lw_parse, dim3(grid_for(frames)), dim3(kThreads), kLds, (hipStream_t)stream, d_bytes,
                       (unsigned long long)frames, (unsigned long long)stride, d_lens, (uint32_t)len, d_keys,
                       (unsigned long long)nkeys, d_key_index, d_out);
    LW_OK(hipGetLastError());
    return 0;
}

int lphy_hip_lorawan_mic_host(int device, const uint8_t key[16], int uplink, uint32_t devaddr, uint32_t fcnt,
                              const uint8_t* data, size_t len, uint32_t* mic) {
    if (!key || !mic || (len && !data) || len > 0xFFFFFFFFull - 64) return -EINVAL;
    struct Stage {
        void* p = nullptr;
        size_t bytes = 0;
    };
    static std::mutex mu;
    static std::map<int, Stage> stages;
    std::lock_guard<std::mutex> lk(mu);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return -ENODEV;
    LW_OK(hipSetDevice(device));
    // [key 16 | desc 32 | mic 4 .. pad to 64 | data]
    const size_t need = 64 + len + 4;
    Stage& s = stages[device];
    if (s.bytes < need) {
        if (s.p) (void)hipFree(s.p);
        s.p = nullptr;
        s.bytes = 0;
        LW_OK(hipMalloc(&s.p, need < 4096 ? 4096 : need));
        s.bytes = need < 4096 ? 4096 : need;
    }
    uint8_t* base = static_cast<uint8_t*>(s.p);
    lphy_lorawan_desc d{};
    d.offset = 64;
    d.len = (uint32_t)len;
    d.devaddr = devaddr;
    d.fcnt = fcnt;
    d.key = 0;
    d.uplink = uplink ? 1u : 0u;
    LW_OK(hipMemcpy(base, key, 16, hipMemcpyHostToDevice));
    LW_OK(hipMemcpy(base + 16, &d, sizeof d, hipMemcpyHostToDevice));
    if (len) LW_OK(hipMemcpy(base + 64, data, len, hipMemcpyHostToDevice));
    const int rc = lphy_hip_lorawan_mic_batch(base, reinterpret_cast<const lphy_lorawan_desc*>(base + 16), 1,
                                              base, 1, reinterpret_cast<uint32_t*>(base + 48), 0, nullptr);
    if (rc) return rc;
    LW_OK(hipDeviceSynchronize());
    LW_OK(hipMemcpy(mic, base + 48, 4, hipMemcpyDeviceToHost));
    return 0;
}

}  // extern "C"
