// lphy_stream.hip — streaming IQ ingestion for the demodulator (SURVEY §8f
// rank 2).
//
// The reference's receive runner reads float32 (I, Q) pairs back to back
// from a file or stdin (runners/rx_runner.cpp:61-79) and demodulates them
// in one call (:105-116).  Here the same byte format arrives on a file
// descriptor and is demodulated as a stream of whole frames:
//
//   host   read(fd) -> pinned slot s                 (blocking, short reads ok;
//                                                     a file: 8 parallel preads)
//   copy   hipMemcpyAsync H2D slot s                 (copy stream)
//   comp   wait(H2D s); lphy_hip_demod_batch(slot s);
//          D2H results -> pinned result slot s       (compute stream)
//
// with NSLOT slots in flight, so the read of chunk i+1 and the copy of
// chunk i overlap the demodulation of chunk i-1.  Results are copied to the
// caller's arrays when their slot is reused or at the end.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
#include <unistd.h>

#include "../../include/lphy_hip.h"

extern "C" int lphy_hip_ctx_device(const lphy_hip_ctx* c);  // lphy_hip.hip

namespace {

#define ST_OK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "lphy_stream: %s failed: %s (%s:%d)\n", #x,       \
                    hipGetErrorString(e_), __FILE__, __LINE__);               \
            rc = -EIO;                                                        \
            goto done;                                                        \
        }                                                                     \
    } while (0)

constexpr int NSLOT = 3;

// Fill buf with up to `want` bytes from fd; stops early only at EOF.
// Returns the byte count, or -errno.
long long read_full(int fd, char* buf, size_t want) {
    size_t got = 0;
    while (got < want) {
        const ssize_t r = ::read(fd, buf + got, want - got);
        if (r == 0) break;
        if (r < 0) {
            if (errno == EINTR) continue;
            return -(long long)errno;
        }
        got += (size_t)r;
    }
    return (long long)got;
}

// A seekable fd (a file) is read by kReaders threads with pread, each a
// contiguous part of the chunk (one thread's memcpy out of the page cache
// runs at ~5 GB/s, a tenth of PCIe); a pipe or a socket is read in order.
// The fd's offset is left after the bytes consumed, as read() would.
constexpr int kReaders = 8;
constexpr size_t kParMin = size_t(4) << 20;  // below this one read() suffices

long long read_chunk(int fd, bool seekable, char* buf, size_t want) {
    if (!seekable || want < kParMin) return read_full(fd, buf, want);
    const off_t base = ::lseek(fd, 0, SEEK_CUR);
    if (base < 0) return read_full(fd, buf, want);
    const size_t part = (want + kReaders - 1) / kReaders;
    std::vector<long long> got(kReaders, 0);
    std::vector<std::thread> th;
    int parts = 0;
    for (int k = 0; k < kReaders; ++k) {
        const size_t o = (size_t)k * part;
        if (o >= want) break;
        const size_t n = want - o < part ? want - o : part;
        auto part_read = [&, k, o, n] {
            size_t g = 0;
            while (g < n) {
                const ssize_t r = ::pread(fd, buf + o + g, n - g, base + (off_t)(o + g));
                if (r == 0) break;
                if (r < 0) {
                    if (errno == EINTR) continue;
                    got[k] = -(long long)errno;
                    return;
                }
                g += (size_t)r;
            }
            got[k] = (long long)g;
        };
        // no exception may cross the C ABI: when a thread cannot be started
        // (std::system_error under a thread limit) this thread reads the part
        try {
            th.emplace_back(part_read);
        } catch (...) {
            part_read();
        }
        ++parts;
    }
    for (auto& t : th) t.join();
    // the bytes read are the contiguous prefix up to the first short part (EOF)
    size_t total = 0;
    for (int k = 0; k < parts; ++k) {
        if (got[k] < 0) return got[k];
        total += (size_t)got[k];
        const size_t o = (size_t)k * part;
        const size_t n = want - o < part ? want - o : part;
        if ((size_t)got[k] < n) break;
    }
    if (::lseek(fd, base + (off_t)total, SEEK_SET) < 0) return -(long long)errno;
    return (long long)total;
}

struct Slot {
    char* pin_iq = nullptr;         // pinned input chunk
    float* d_iq = nullptr;          // device input chunk
    uint16_t* d_syms = nullptr;
    uint8_t* d_bytes = nullptr;
    lphy_frame_meta* d_meta = nullptr;
    uint16_t* pin_syms = nullptr;   // pinned results
    uint8_t* pin_bytes = nullptr;
    lphy_frame_meta* pin_meta = nullptr;
    hipEvent_t h2d = nullptr, done = nullptr;
    size_t first = 0, frames = 0;   // stream frame range held by the slot
    bool busy = false;
};

}  // namespace

extern "C" int lphy_hip_demod_stream(lphy_hip_ctx* ctx, int fd, size_t frame_samples,
                                     size_t chunk_frames, int mode, unsigned flags,
                                     size_t max_frames, uint16_t* h_syms, uint8_t* h_bytes,
                                     lphy_frame_meta* h_meta, size_t* frames_out,
                                     size_t* tail_bytes) {
    // max_frames is the capacity of h_syms / h_bytes / h_meta in frames: the
    // C ABI takes no other size, so an unbounded read could overrun them
    if (!ctx || fd < 0 || frame_samples == 0 || chunk_frames == 0 || max_frames == 0 || !h_meta ||
        !frames_out)
        return -EINVAL;
    if (mode < 0 || mode > 2) return -EINVAL;
    if ((flags & LPHY_F_DECODE) && !h_bytes) return -EINVAL;
    const size_t per = lphy_hip_syms_per_frame(ctx, frame_samples, mode);
    if (per && !h_syms) return -EINVAL;
    const bool dec = (flags & LPHY_F_DECODE) != 0;
    const size_t frame_bytes = frame_samples * 2 * sizeof(float);
    const size_t chunk_bytes = chunk_frames * frame_bytes;
    *frames_out = 0;
    if (tail_bytes) *tail_bytes = 0;

    int rc = 0;
    Slot sl[NSLOT];
    hipStream_t copy_st = nullptr, comp_st = nullptr;
    size_t next = 0;  // stream frames read so far
    unsigned long long chunk = 0;
    int dev = 0;

    // results of a slot into the caller's arrays (after its event)
    auto harvest = [&](Slot& s) -> int {
        if (!s.busy) return 0;
        if (hipEventSynchronize(s.done) != hipSuccess) return -EIO;
        memcpy(h_meta + s.first, s.pin_meta, s.frames * sizeof(lphy_frame_meta));
        if (per) memcpy(h_syms + s.first * per, s.pin_syms, s.frames * per * sizeof(uint16_t));
        if (dec && per / 2) memcpy(h_bytes + s.first * (per / 2), s.pin_bytes, s.frames * (per / 2));
        s.busy = false;
        return 0;
    };

    const bool seekable = ::lseek(fd, 0, SEEK_CUR) >= 0;
    dev = lphy_hip_ctx_device(ctx);
    ST_OK(hipSetDevice(dev));
    ST_OK(hipStreamCreateWithFlags(&copy_st, hipStreamNonBlocking));
    ST_OK(hipStreamCreateWithFlags(&comp_st, hipStreamNonBlocking));
    for (Slot& s : sl) {
        ST_OK(hipHostMalloc((void**)&s.pin_iq, chunk_bytes, hipHostMallocDefault));
        ST_OK(hipMalloc((void**)&s.d_iq, chunk_bytes));
        ST_OK(hipMalloc((void**)&s.d_syms, (per ? per : 1) * chunk_frames * sizeof(uint16_t)));
        ST_OK(hipMalloc((void**)&s.d_bytes, (per / 2 ? per / 2 : 1) * chunk_frames));
        ST_OK(hipMalloc((void**)&s.d_meta, chunk_frames * sizeof(lphy_frame_meta)));
        ST_OK(hipHostMalloc((void**)&s.pin_syms, (per ? per : 1) * chunk_frames * sizeof(uint16_t),
                            hipHostMallocDefault));
        ST_OK(hipHostMalloc((void**)&s.pin_bytes, (per / 2 ? per / 2 : 1) * chunk_frames,
                            hipHostMallocDefault));
        ST_OK(hipHostMalloc((void**)&s.pin_meta, chunk_frames * sizeof(lphy_frame_meta),
                            hipHostMallocDefault));
        ST_OK(hipEventCreateWithFlags(&s.h2d, hipEventDisableTiming));
        ST_OK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    }

    for (;; ++chunk) {
        Slot& s = sl[chunk % NSLOT];
        if ((rc = harvest(s)) != 0) goto done;  // slot free (its H2D and demod are done)
        size_t want = chunk_bytes;
        if (max_frames - next < chunk_frames) want = (max_frames - next) * frame_bytes;
        if (want == 0) break;
        const long long got = read_chunk(fd, seekable, s.pin_iq, want);
        if (got < 0) { rc = -EIO; goto done; }
        const size_t nf = (size_t)got / frame_bytes;
        if ((size_t)got % frame_bytes) {
            // EOF inside a frame: the reference rejects a partial symbol
            // count (rx_runner.cpp:87-91); the whole frames before it run
            if (tail_bytes) *tail_bytes = (size_t)got % frame_bytes;
        }
        if (nf == 0) break;
        ST_OK(hipMemcpyAsync(s.d_iq, s.pin_iq, nf * frame_bytes, hipMemcpyHostToDevice, copy_st));
        ST_OK(hipEventRecord(s.h2d, copy_st));
        ST_OK(hipStreamWaitEvent(comp_st, s.h2d, 0));
        ST_OK(hipMemsetAsync(s.d_meta, 0, nf * sizeof(lphy_frame_meta), comp_st));
        rc = lphy_hip_demod_batch(ctx, s.d_iq, nf, frame_samples, s.d_syms, dec ? s.d_bytes : nullptr,
                                  s.d_meta, mode, flags, comp_st);
        if (rc) goto done;
        ST_OK(hipMemcpyAsync(s.pin_meta, s.d_meta, nf * sizeof(lphy_frame_meta), hipMemcpyDeviceToHost,
                             comp_st));
        if (per)
            ST_OK(hipMemcpyAsync(s.pin_syms, s.d_syms, nf * per * sizeof(uint16_t), hipMemcpyDeviceToHost,
                                 comp_st));
        if (dec && per / 2)
            ST_OK(hipMemcpyAsync(s.pin_bytes, s.d_bytes, nf * (per / 2), hipMemcpyDeviceToHost, comp_st));
        ST_OK(hipEventRecord(s.done, comp_st));
        s.first = next;
        s.frames = nf;
        s.busy = true;
        next += nf;
        if ((size_t)got < want) break;  // EOF
    }
    for (unsigned long long k = 1; k <= NSLOT; ++k)
        if ((rc = harvest(sl[(chunk + k) % NSLOT])) != 0) goto done;
    *frames_out = next;

done:
    if (comp_st) (void)hipStreamSynchronize(comp_st);
    if (copy_st) (void)hipStreamSynchronize(copy_st);
    for (Slot& s : sl) {
        if (s.pin_iq) (void)hipHostFree(s.pin_iq);
        if (s.d_iq) (void)hipFree(s.d_iq);
        if (s.d_syms) (void)hipFree(s.d_syms);
        if (s.d_bytes) (void)hipFree(s.d_bytes);
        if (s.d_meta) (void)hipFree(s.d_meta);
        if (s.pin_syms) (void)hipHostFree(s.pin_syms);
        if (s.pin_bytes) (void)hipHostFree(s.pin_bytes);
        if (s.pin_meta) (void)hipHostFree(s.pin_meta);
        if (s.h2d) (void)hipEventDestroy(s.h2d);
        if (s.done) (void)hipEventDestroy(s.done);
    }
    if (copy_st) (void)hipStreamDestroy(copy_st);
    if (comp_st) (void)hipStreamDestroy(comp_st);
    return rc;
}
