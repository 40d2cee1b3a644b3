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
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <immintrin.h>
#include <mutex>
#include <thread>
#include <vector>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/lphy_hip.h"

extern "C" int lphy_hip_ctx_device(const lphy_hip_ctx* c);  // lphy_hip.hip (internal)
extern "C" void* lphy_hip_ctx_stream_ext(lphy_hip_ctx* c, void* (*make)(), void (*destroy)(void*));

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
constexpr size_t kAutoChunkBytes = size_t(64) << 20;  // chunk_frames = 0: ~64 MiB chunks

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

// The CPUs this process may use: the affinity mask, capped by the cgroup
// CPU quota (a GPU box reports the whole host but grants a share of it).
int usable_cpus() {
    int n = (int)std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long long period = 0;
        if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
            const long long quota = atoll(q);
            const int c = (int)((quota + period - 1) / period);
            if (c > 0 && c < n) n = c;
        }
        fclose(f);
    }
    return n > 0 ? n : 1;
}

// A seekable fd (a file) is read by a pool of reader threads, each a
// contiguous part of the chunk (one thread's copy out of the page cache runs
// at ~3-5 GB/s, a tenth of PCIe); a pipe or a socket is read in order.  A
// regular file is mapped (read-only) and the readers copy from the mapping
// with non-temporal stores: the pinned slot is written without being read
// first, which pread's kernel copy does, and the syscall per part goes away
// (tools/stream_bench.py; LPHY_STREAM_COPY=pread selects the pread readers).
// The fd's offset is left after the bytes consumed, as read() would.
// Readers: LPHY_STREAM_READERS, default one per usable CPU but one (the
// calling thread drives the GPU), at most 32.
constexpr size_t kParMin = size_t(4) << 20;  // below this one read() suffices

// dst 32-byte aligned; streaming stores, then a fence so the copy engine
// (which reads the slot after the readers return) sees every byte
__attribute__((target("avx2"))) void copy_nt_avx2(char* dst, const char* src, size_t n) {
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 64));
        const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), a);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 96), d);
    }
    memcpy(dst + i, src + i, n - i);
    _mm_sfence();
}
void copy_part(char* dst, const char* src, size_t n) {
    static const bool avx2 = [] {
#ifndef __HIP_DEVICE_COMPILE__  // (host code; the device pass only parses it)
        __builtin_cpu_init();  // a library may run before the CPU model is filled in
#endif
        return __builtin_cpu_supports("avx2") != 0;
    }();
    if (avx2 && (reinterpret_cast<uintptr_t>(dst) & 31) == 0) copy_nt_avx2(dst, src, n);
    else memcpy(dst, src, n);
}

class ReaderPool {
  public:
    explicit ReaderPool(int n) {
        for (int k = 0; k < n; ++k) {
            try {
                th_.emplace_back([this, k] { run(k); });
            } catch (...) {  // no exception may cross the C ABI: fewer readers
                break;
            }
        }
    }
    ~ReaderPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return (int)th_.size(); }
    // the file bytes [off, off + len) mapped at `map` (nullptr: pread)
    void set_map(const char* map, off_t off, size_t len) {
        map_ = map;
        map_off_ = off;
        map_len_ = len;
    }
    // read [base, base + want) of fd into buf with all readers; returns the
    // bytes of the contiguous prefix read (short at EOF) or -errno
    long long read(int fd, off_t base, char* buf, size_t want) {
        const int n = size();
        if (n == 0) return -EAGAIN;
        std::unique_lock<std::mutex> lk(mu_);
        fd_ = fd;
        base_ = base;
        buf_ = buf;
        want_ = want;
        part_ = ((want + n - 1) / n + 4095) & ~size_t(4095);  // page-aligned parts
        got_.assign(n, 0);
        pending_ = n;
        ++gen_;
        cv_.notify_all();
        done_cv_.wait(lk, [this] { return pending_ == 0; });
        size_t total = 0;
        for (int k = 0; k < n; ++k) {
            if (got_[k] < 0) return got_[k];
            total += (size_t)got_[k];
            const size_t o = (size_t)k * part_;
            const size_t len = o >= want ? 0 : (want - o < part_ ? want - o : part_);
            if ((size_t)got_[k] < len) break;
        }
        return (long long)total;
    }

  private:
    void run(int k) {
        unsigned long long seen = 0;
        for (;;) {
            int fd;
            off_t base;
            char* buf;
            size_t o, len;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                fd = fd_;
                base = base_;
                buf = buf_;
                o = (size_t)k * part_;
                len = o >= want_ ? 0 : (want_ - o < part_ ? want_ - o : part_);
            }
            long long g = 0;
            const off_t at = base + (off_t)o;
            if (map_ && len && at >= map_off_ && (size_t)(at - map_off_) + len <= map_len_) {
                copy_part(buf + o, map_ + (at - map_off_), len);
                g = (long long)len;
            }
            while ((size_t)g < len) {
                const ssize_t r = ::pread(fd, buf + o + g, len - (size_t)g, base + (off_t)(o + (size_t)g));
                if (r == 0) break;
                if (r < 0) {
                    if (errno == EINTR) continue;
                    g = -(long long)errno;
                    break;
                }
                g += r;
            }
            {
                std::lock_guard<std::mutex> lk(mu_);
                got_[k] = g;
                if (--pending_ == 0) done_cv_.notify_one();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    bool stop_ = false;
    unsigned long long gen_ = 0;
    int fd_ = -1;
    off_t base_ = 0;
    const char* map_ = nullptr;
    off_t map_off_ = 0;
    size_t map_len_ = 0;
    char* buf_ = nullptr;
    size_t want_ = 0, part_ = 0;
    std::vector<long long> got_;
    int pending_ = 0;
};

long long read_chunk(ReaderPool* pool, int fd, bool seekable, char* buf, size_t want) {
    if (!seekable || want < kParMin || !pool || pool->size() == 0) return read_full(fd, buf, want);
    const off_t base = ::lseek(fd, 0, SEEK_CUR);
    if (base < 0) return read_full(fd, buf, want);
    const long long total = pool->read(fd, base, buf, want);
    if (total < 0) return total;
    if (::lseek(fd, base + (off_t)total, SEEK_SET) < 0) return -(long long)errno;
    return total;
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

// The slots and streams of a context's streaming calls, kept with the
// context (lphy_hip_ctx_stream_ext) so that repeated calls allocate nothing;
// regrown when a call needs larger chunks.
struct StreamState {
    // held for a whole lphy_hip_demod_stream call: the slots, buffers and
    // streams below are the call's own while it runs (a second thread's call
    // on the same context waits; ensure() never releases buffers in use)
    std::mutex mu;
    Slot sl[NSLOT];
    hipStream_t copy_st = nullptr, comp_st = nullptr;
    size_t chunk_bytes = 0, sym_cap = 0, byte_cap = 0, meta_cap = 0;
    void release() {
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
            s = Slot{};
        }
        chunk_bytes = sym_cap = byte_cap = meta_cap = 0;
    }
    ~StreamState() {
        release();
        if (copy_st) (void)hipStreamDestroy(copy_st);
        if (comp_st) (void)hipStreamDestroy(comp_st);
    }
    int ensure(size_t cbytes, size_t syms, size_t bytes, size_t metas) {
        if (!copy_st && hipStreamCreateWithFlags(&copy_st, hipStreamNonBlocking) != hipSuccess) return -EIO;
        if (!comp_st && hipStreamCreateWithFlags(&comp_st, hipStreamNonBlocking) != hipSuccess) return -EIO;
        if (cbytes <= chunk_bytes && syms <= sym_cap && bytes <= byte_cap && metas <= meta_cap) return 0;
        release();
        for (Slot& s : sl) {
            if (hipHostMalloc((void**)&s.pin_iq, cbytes, hipHostMallocDefault) != hipSuccess ||
                hipMalloc((void**)&s.d_iq, cbytes) != hipSuccess ||
                hipMalloc((void**)&s.d_syms, syms * sizeof(uint16_t)) != hipSuccess ||
                hipMalloc((void**)&s.d_bytes, bytes) != hipSuccess ||
                hipMalloc((void**)&s.d_meta, metas * sizeof(lphy_frame_meta)) != hipSuccess ||
                hipHostMalloc((void**)&s.pin_syms, syms * sizeof(uint16_t), hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void**)&s.pin_bytes, bytes, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void**)&s.pin_meta, metas * sizeof(lphy_frame_meta), hipHostMallocDefault) !=
                    hipSuccess ||
                hipEventCreateWithFlags(&s.h2d, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) {
                release();
                return -ENOMEM;
            }
        }
        chunk_bytes = cbytes;
        sym_cap = syms;
        byte_cap = bytes;
        meta_cap = metas;
        return 0;
    }
};

void free_stream_state(void* p) { delete static_cast<StreamState*>(p); }

}  // namespace

extern "C" int lphy_hip_demod_stream(lphy_hip_ctx* ctx, int fd, size_t frame_samples,
                                     size_t chunk_frames, int mode, unsigned flags,
                                     size_t max_frames, uint16_t* h_syms, uint8_t* h_bytes,
                                     lphy_frame_meta* h_meta, size_t* frames_out,
                                     size_t* tail_bytes) {
    // max_frames is the capacity of h_syms / h_bytes / h_meta in frames: the
    // C ABI takes no other size, so an unbounded read could overrun them
    if (!ctx || fd < 0 || frame_samples == 0 || max_frames == 0 || !h_meta || !frames_out) return -EINVAL;
    if (mode < 0 || mode > 2) return -EINVAL;
    if ((flags & LPHY_F_DECODE) && !h_bytes) return -EINVAL;
    const size_t per = lphy_hip_syms_per_frame(ctx, frame_samples, mode);
    if (per && !h_syms) return -EINVAL;
    const bool dec = (flags & LPHY_F_DECODE) != 0;
    const size_t frame_bytes = frame_samples * 2 * sizeof(float);
    if (chunk_frames == 0) {  // chunks of ~64 MiB, whole frames
        chunk_frames = kAutoChunkBytes / frame_bytes;
        if (chunk_frames == 0) chunk_frames = 1;
    }
    if (chunk_frames > max_frames) chunk_frames = max_frames;
    const size_t chunk_bytes = chunk_frames * frame_bytes;
    *frames_out = 0;
    if (tail_bytes) *tail_bytes = 0;

    if (hipSetDevice(lphy_hip_ctx_device(ctx)) != hipSuccess) return -EIO;
    int rc = 0;
    size_t next = 0;  // stream frames read so far
    unsigned long long chunk = 0;
    const bool seekable = ::lseek(fd, 0, SEEK_CUR) >= 0;
    int nreaders = usable_cpus() - 1;
    if (const char* e = getenv("LPHY_STREAM_READERS")) nreaders = atoi(e);
    nreaders = nreaders < 1 ? 1 : (nreaders > 32 ? 32 : nreaders);
    ReaderPool pool(seekable && chunk_bytes >= kParMin ? nreaders : 0);
    // the readers' source mapping (regular files; LPHY_STREAM_COPY=pread: none)
    char* rmap = nullptr;
    size_t rmap_len = 0;
    if (pool.size() > 0 && !(getenv("LPHY_STREAM_COPY") && strcmp(getenv("LPHY_STREAM_COPY"), "pread") == 0)) {
        struct stat stt;
        if (fstat(fd, &stt) == 0 && S_ISREG(stt.st_mode) && stt.st_size > 0) {
            rmap_len = (size_t)stt.st_size;
            void* m = mmap(nullptr, rmap_len, PROT_READ, MAP_SHARED, fd, 0);
            if (m != MAP_FAILED) {
                rmap = static_cast<char*>(m);
                (void)madvise(rmap, rmap_len, MADV_SEQUENTIAL);
                pool.set_map(rmap, 0, rmap_len);
            }
        }
    }
    StreamState* S = nullptr;
    std::unique_lock<std::mutex> call_lock;  // S->mu, from S's lookup to the return
    Slot* sl = nullptr;
    hipStream_t copy_st = nullptr, comp_st = nullptr;

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

    ST_OK(hipSetDevice(lphy_hip_ctx_device(ctx)));
    S = static_cast<StreamState*>(lphy_hip_ctx_stream_ext(
        ctx, [] { return static_cast<void*>(new StreamState); }, free_stream_state));
    if (!S) {
        rc = -ENOMEM;
        goto done;
    }
    call_lock = std::unique_lock<std::mutex>(S->mu);
    if ((rc = S->ensure(chunk_bytes, (per ? per : 1) * chunk_frames, (per / 2 ? per / 2 : 1) * chunk_frames,
                        chunk_frames)) != 0)
        goto done;
    sl = S->sl;
    copy_st = S->copy_st;
    comp_st = S->comp_st;

    for (;; ++chunk) {
        Slot& s = sl[chunk % NSLOT];
        if ((rc = harvest(s)) != 0) goto done;  // slot free (its H2D and demod are done)
        size_t want = chunk_bytes;
        if (max_frames - next < chunk_frames) want = (max_frames - next) * frame_bytes;
        if (want == 0) break;
        if (rmap) {  // a file shortened since the call began: its lost tail is pread (short), not copied
            struct stat stt;
            if (fstat(fd, &stt) == 0 && (size_t)stt.st_size < rmap_len) pool.set_map(rmap, 0, (size_t)stt.st_size);
        }
        const long long got = read_chunk(&pool, fd, seekable, s.pin_iq, want);
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
    if (sl)
        for (int k = 0; k < NSLOT; ++k) sl[k].busy = false;
    if (rmap) munmap(rmap, rmap_len);
    return rc;
}
