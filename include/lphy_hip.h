/*
 * lphy_hip.h — C ABI of the MI355X (gfx950) LoRa PHY demodulation layer.
 *
 * This is the drop-in boundary below the lora_phy:: C++ API
 * (include/lora_phy/phy.hpp, implemented by liblora_phy_amd.so on top of
 * these entry points).  Plain pointers and sizes only; device pointers are
 * hipMalloc'd (or torch) memory, `stream` is a hipStream_t (NULL = default).
 * Every function returns 0 or a negative errno, like the reference.
 *
 * Reference interfaces replaced (file:line under the reference tree):
 *   lphy_hip_ctx_create    lora_phy::init            src/phy/phy.cpp:27-52
 *                          lora_phy::lora_demod_init src/phy/LoRaDemod.cpp:11-33
 *   lphy_hip_ctx_destroy   lora_phy::lora_demod_free src/phy/LoRaDemod.cpp:35-48
 *   lphy_hip_demod_batch   mode LPHY_MODE_DEMODULATE:
 *                            lora_phy::demodulate        src/phy/phy.cpp:182-243
 *                            (+ estimate_offsets          src/phy/phy.cpp:81-148)
 *                          mode LPHY_MODE_LORA_DEMODULATE:
 *                            lora_phy::lora_demodulate   src/phy/LoRaDemod.cpp:50-197
 *                          mode LPHY_MODE_DECHIRP_LORA_DEMODULATE:
 *                            test-side dechirp (tests/e2e_chain_test.cpp:80-93)
 *                            fused in front of lora_demodulate
 *                          flag LPHY_F_DECODE adds, per frame:
 *                            lora_phy::decode / lora_decode src/phy/phy.cpp:245-261,
 *                            src/phy/LoRaDecoder.cpp:7-21
 *   lphy_hip_decode_batch  lora_phy::decode / lora_decode on device symbols
 *   lphy_hip_estimate_batch lora_phy::estimate_offsets src/phy/phy.cpp:81-148
 *   lphy_hip_modulate_batch lora_phy::lora_modulate  src/phy/LoRaMod.cpp:8-43
 *                            (producer; bit-exact, used for synthetic IQ)
 *   lphy_hip_compensate    lora_phy::compensate_offsets src/phy/phy.cpp:150-180
 *
 * Batch layout in HBM:
 *   IQ      interleaved float32 (I,Q) = std::complex<float>, frame f at
 *           d_iq + 2*f*frame_samples floats.
 *   symbols uint16, frame f at d_syms + f*lphy_hip_syms_per_frame(...)
 *           (data symbols only when the frame has >= 2 symbols — the two
 *           sync symbols go to lphy_frame_meta.sw0/sw1, as the reference
 *           routes them to ws->sync_word / *out_sync).
 *   bytes   uint8, frame f at d_bytes + f*(data_symbols/2) (LPHY_F_DECODE).
 *   meta    one lphy_frame_meta per frame (also the kernels' hand-off
 *           between the per-frame prologue and the per-symbol demodulator).
 */
#ifndef LPHY_HIP_H
#define LPHY_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lphy_hip_ctx lphy_hip_ctx;

/* Per-frame results (32 bytes). */
typedef struct lphy_frame_meta {
    float cfo;          /* ws->metrics.cfo after the call                    */
    float time_offset;  /* ws->metrics.time_offset                           */
    float rate;         /* -2*pi*cfo/N: per-sample CFO rotation              */
    float scale;        /* 1/max(|I|,|Q|) when normalised (modes 1,2), else 1 */
    int32_t t_off;      /* (int)round(time_offset)                           */
    int32_t status;     /* 0 | -ERANGE (needs scratch) | -EINVAL (odd count) */
    uint16_t sw0, sw1;  /* argmax bins of the two sync symbols               */
    uint8_t sync_word;  /* ((sw0>>(sf-4))&15)<<4 | ((sw1>>(sf-4))&15)        */
    uint8_t crc_ok;     /* lora_phy::decode's metrics.crc_ok (LPHY_F_DECODE) */
    uint8_t normalised; /* 1 when max(|I|,|Q|) > 1 forced the rescale        */
    uint8_t have_sync;  /* frame had >= 2 symbols                            */
} lphy_frame_meta;

enum lphy_mode {
    LPHY_MODE_DEMODULATE = 0,              /* lora_phy::demodulate (raw IQ)  */
    LPHY_MODE_LORA_DEMODULATE = 1,         /* lora_demodulate (dechirped IQ) */
    LPHY_MODE_DECHIRP_LORA_DEMODULATE = 2  /* raw IQ, dechirp fused, then 1  */
};

enum lphy_flags {
    LPHY_F_DECODE = 1u,      /* also Hamming-decode + CRC each frame        */
    LPHY_F_NO_SCRATCH = 2u,  /* modes 1/2: behave as lora_demodulate with no
                                scratch buffer (-ERANGE when rescale needed) */
    /* Stage selection (profiling / overlap): when any of these bits is set
     * only the selected stages are launched; none set = all three.  With
     * PROLOGUE | SYMBOLS both set, the fused kernel (when it applies) runs
     * both in one launch. */
    LPHY_F_STAGE_PROLOGUE = 4u,  /* per-frame max-abs + offset estimate   */
    LPHY_F_STAGE_SYMBOLS = 8u,   /* per-symbol rotate + FFT + argmax      */
    LPHY_F_STAGE_FINAL = 16u,    /* per-frame sync word, decode, CRC      */
    LPHY_F_UNFUSED = 32u         /* separate prologue / symbol launches
                                    instead of the fused single launch
                                    (same results; the shapes the fused
                                    kernels do not take run them anyway) */
    /* Bits 64..1024 are comparison / test paths of the test-only build
     * (lib/test/, csrc/lphy_testing.h); this library rejects them with
     * -EINVAL. */
};

enum lphy_window { LPHY_WINDOW_NONE = 0, LPHY_WINDOW_HANN = 1 };

/* Create a context for one (sf, bandwidth, osr, window) configuration on
 * HIP device `device`.  Precomputes the KISS twiddles, the down-chirp and
 * the window on the host with the same libm calls as the reference, and
 * uploads them.  sf in [1,12]; bw_hz in {125000,250000,500000}.
 * Returns 0, -EINVAL (bad arguments) or -ENODEV / -ENOMEM. */
int lphy_hip_ctx_create(lphy_hip_ctx** out, int device, unsigned sf,
                        unsigned bw_hz, unsigned osr, int window);
void lphy_hip_ctx_destroy(lphy_hip_ctx* ctx);

/* A context of its own over `base`'s constant tables (shared, read-only;
 * they are freed with the last context holding them), with `osr` (0: the
 * base's).  Each context has its own stream and staging for the *_host
 * entry points, so contexts made this way - one per workspace or thread, as
 * the C++ shim does (lora_demod_init, init) - never wait for each other.
 * Returns 0, -EINVAL, -ENOMEM or -EIO. */
int lphy_hip_ctx_share(lphy_hip_ctx** out, const lphy_hip_ctx* base, unsigned osr);

/* Size the context's host-call staging for calls of up to `frames` frames
 * of `frame_samples` samples (the *_host entry points below), so that those
 * calls allocate nothing: the reference allocates nothing after init
 * (API_SPEC.md:9-14; lora_demod_init's max_samples, LoRaDemod.cpp:11-33).
 * A larger call later grows the staging once.  Returns 0 or -ENOMEM/-EIO. */
int lphy_hip_ctx_reserve(lphy_hip_ctx* ctx, size_t frames, size_t frame_samples);

/* Smallest batch (frames per lphy_hip_demod_batch call) that takes the
 * fused single-launch kernels on this context; smaller batches take the
 * separate symbol-parallel launches, which finish a few frames sooner.
 * `frames` < 0 restores the measured per-SF crossover (the default); 0 sends
 * every batch whose shape fits to the fused kernels (throughput callers, the
 * test suite).  Results are identical either way.  Returns 0 or -EINVAL. */
int lphy_hip_ctx_set_fused_min_frames(lphy_hip_ctx* ctx, long frames);

/* Symbols written per frame for a frame of `frame_samples` samples. */
size_t lphy_hip_syms_per_frame(const lphy_hip_ctx* ctx, size_t frame_samples,
                               int mode);

/* Demodulate `frames` frames of device-resident IQ (asynchronous on
 * `stream`).  d_bytes may be NULL unless LPHY_F_DECODE.  d_meta is
 * required.  Returns 0 or -EINVAL/-ERANGE for shape errors (the per-frame
 * conditions the reference reports through its return value are in
 * lphy_frame_meta.status).
 * Limits: frames * (frame_samples / (N*osr)) < 2^32 symbols per call and
 * frame_samples < 2^31 (32-bit symbol bookkeeping in the kernels): larger
 * batches give -ERANGE; split them across calls.
 * Launch choice: the fused launches (k_wave at SF 7-12 for osr 1, no
 * window, modes 1/2 with the speculative normalisation or mode 0, and below
 * SF 9 at least 4096/N symbols per frame - SF 7-10 with units spanning
 * frames; k_frames otherwise up to SF 10, e.g. windowed or short frames)
 * for batches of at
 * least a per-SF crossover (256 frames at SF <= 7 ... 384 at SF 10-12,
 * DESIGN.md 4.7; lphy_hip_ctx_set_fused_min_frames overrides it per
 * context), the separate symbol-parallel launches below it (a packet at a
 * time).  The choice depends on the arguments and that setting only (no
 * environment variables).
 * Memory: the fused launches allocate nothing.  The SF 11-12 separate launches
 * (LPHY_F_UNFUSED, small batches, osr > 1, a window) take per-call speculation records
 * (16 B per frame) from the stream-ordered pool on `stream`, released in
 * stream order, so calls on different streams of one context never share
 * them; the *_host forms lend them from the reserved staging instead. */
int lphy_hip_demod_batch(lphy_hip_ctx* ctx, const float* d_iq, size_t frames,
                         size_t frame_samples, uint16_t* d_syms,
                         uint8_t* d_bytes, lphy_frame_meta* d_meta, int mode,
                         unsigned flags, void* stream);

/* Hamming(8,4)sx decode + sx1272 CRC of device symbols: frame f holds
 * syms_per_frame symbols at d_syms + f*syms_per_frame and yields
 * syms_per_frame/2 bytes; meta[f].crc_ok / .status updated.  An odd
 * syms_per_frame gives -EINVAL (LoRaDecoder.cpp:10). */
int lphy_hip_decode_batch(lphy_hip_ctx* ctx, const uint16_t* d_syms,
                          size_t frames, size_t syms_per_frame,
                          uint8_t* d_bytes, lphy_frame_meta* d_meta,
                          void* stream);

/* estimate_offsets (phy.cpp:81-148) over the first `est_samples` samples of
 * each frame: writes meta[f].cfo / .time_offset / .t_off / .rate. */
int lphy_hip_estimate_batch(lphy_hip_ctx* ctx, const float* d_iq,
                            size_t frames, size_t frame_samples,
                            size_t est_samples, lphy_frame_meta* d_meta,
                            void* stream);

/* compensate_offsets (phy.cpp:150-180), in place on one device buffer. */
int lphy_hip_compensate(lphy_hip_ctx* ctx, float* d_iq, size_t count,
                        float cfo, float time_offset, void* stream);

/* lora_modulate (LoRaMod.cpp:8-43) for `frames` frames of `nsyms` symbols
 * each (d_syms + f*nsyms) into d_iq + 2*f*(nsyms+2)*N*osr floats; bit-exact
 * with the reference.  Producer for synthetic input, not on the timed path. */
int lphy_hip_modulate_batch(lphy_hip_ctx* ctx, const uint16_t* d_syms,
                            size_t frames, size_t nsyms, float* d_iq,
                            float amplitude, uint8_t sync, void* stream);

/* Host-buffer convenience used by the C++ shim: uploads, runs
 * lphy_hip_demod_batch, downloads, on the context's own stream and staging
 * (lphy_hip_ctx_reserve); returns when that stream is done, without waiting
 * for other work on the device.  Calls on one context are serialised; use
 * one context per thread (lphy_hip_ctx_share) for concurrent calls. */
int lphy_hip_demod_host(lphy_hip_ctx* ctx, const float* h_iq, size_t frames,
                        size_t frame_samples, uint16_t* h_syms,
                        uint8_t* h_bytes, lphy_frame_meta* h_meta, int mode,
                        unsigned flags);
int lphy_hip_decode_host(lphy_hip_ctx* ctx, const uint16_t* h_syms,
                         size_t count, uint8_t* h_bytes, lphy_frame_meta* h_meta);
int lphy_hip_estimate_host(lphy_hip_ctx* ctx, const float* h_iq,
                           size_t count, lphy_frame_meta* h_meta);
int lphy_hip_compensate_host(lphy_hip_ctx* ctx, float* h_iq, size_t count,
                             float cfo, float time_offset);
int lphy_hip_modulate_host(lphy_hip_ctx* ctx, const uint16_t* h_syms,
                           size_t nsyms, float* h_iq, float amplitude,
                           uint8_t sync);

/* Streaming ingestion.  Reads the reference receive
 * runner's input format - float32 (I, Q) pairs back to back, from a file or
 * stdin (runners/rx_runner.cpp:61-79) - from file descriptor `fd` until EOF
 * or `max_frames` frames, whichever comes first, as consecutive frames of
 * `frame_samples` samples, and demodulates them (lphy_hip_demod_batch,
 * `mode`, `flags`) in chunks of `chunk_frames` (0: whole frames of about
 * 64 MiB): the read of one chunk into
 * pinned host memory and its H2D copy (copy stream) overlap the
 * demodulation of the previous one (compute stream).  Results land in the
 * caller's host arrays in stream order (frame f at h_syms +
 * f*lphy_hip_syms_per_frame, h_bytes + f*(syms/2) with LPHY_F_DECODE,
 * h_meta + f).  A seekable fd is read by a pool of reader threads
 * (LPHY_STREAM_READERS, default one per usable CPU but one); a regular file
 * is mapped read-only and the readers copy out of the mapping with
 * non-temporal stores (LPHY_STREAM_COPY=pread: pread instead; the file
 * size is re-read before each chunk, but as with any mapping, a truncation
 * racing a chunk's copy can raise SIGBUS); the pinned
 * slots and streams stay with the context for its next call, and calls on
 * one context are serialised (a second thread's call waits for the first);
 * use one context per thread (lphy_hip_ctx_share) for concurrent streams.
 * `max_frames` is their capacity in frames and is required
 * (0 gives -EINVAL): reading stops there and the rest of the stream is left
 * unread on `fd` for a later call.  Synchronous.
 * *frames_out = whole frames demodulated; *tail_bytes (optional) = bytes of
 * a trailing partial frame, which is not demodulated (the runner rejects a
 * partial symbol count, rx_runner.cpp:87-91).  Returns 0, -EINVAL, -EIO
 * (read or HIP error) or a lphy_hip_demod_batch shape error. */
int lphy_hip_demod_stream(lphy_hip_ctx* ctx, int fd, size_t frame_samples,
                          size_t chunk_frames, int mode, unsigned flags,
                          size_t max_frames, uint16_t* h_syms, uint8_t* h_bytes,
                          lphy_frame_meta* h_meta, size_t* frames_out,
                          size_t* tail_bytes);

/* Wait for all work queued on `stream`. */
int lphy_hip_sync(void* stream);

/* Version / build string (for tests that check the library loaded). */
const char* lphy_hip_version(void);

/* Symbols the fused kernel recomputed with the exact per-sample rotation
 * because the certified fast path could not prove its argmax (near-ties,
 * NaN, shifted windows; every symbol under LPHY_F_EXACT_ROTATION), summed
 * over launches on `ctx`'s device since the last reset.  Diagnostic only:
 * synchronises the device.  Returns 0 or -EIO. */
int lphy_hip_recheck_count(lphy_hip_ctx* ctx, unsigned long long* out, int reset);

/* Device index checks that failed (an LDS or global index outside its
 * array) since the last reset, summed over the kernels of every SF.  Only
 * the test build (lib/test/, -DLPHY_DEBUG_BOUNDS) counts them; this library
 * returns -ENOTSUP.  Synchronises the device. */
int lphy_hip_bounds_violations(lphy_hip_ctx* ctx, unsigned long long* out, int reset);

/* ------------------------------------------------------------------------
 * Batch forms of the codec helpers of the reference's LoRaCodes.hpp (SURVEY
 * §8f rank 3) on device buffers; `stream` is a hipStream_t (NULL = default).
 * Rows are `frames` records `stride` elements apart.  Results equal the
 * reference helper applied to each row (tests/test_gpu_codes.py).
 * --------------------------------------------------------------------- */
enum lphy_whiten_kind {
    LPHY_WHITEN_SX1232 = 0,      /* SX1232RadioComputeWhitening (LoRaCodes.hpp:111-137) */
    LPHY_WHITEN_SX1272 = 1,      /* Sx1272ComputeWhitening (LoRaCodes.hpp:147-167)      */
    LPHY_WHITEN_SX1272_LFSR = 2  /* Sx1272ComputeWhiteningLfsr (LoRaCodes.hpp:176-189)  */
};
enum lphy_code_op {
    LPHY_CODE_ENC84 = 0,   /* encodeHamming84sx (LoRaCodes.hpp:229-242)             */
    LPHY_CODE_DEC84 = 1,   /* decodeHamming84sx (:250-281); flags bit0 error, bit1 bad */
    LPHY_CODE_ENC74 = 2,   /* encodeHamming74sx (:287-297)                          */
    LPHY_CODE_DEC74 = 3,   /* decodeHamming74sx (:306-334); flags bit0 error         */
    LPHY_CODE_ENCP54 = 4,  /* encodeParity54 (:347-350)                             */
    LPHY_CODE_CHKP54 = 5,  /* checkParity54 (:340-345); flags bit0 error             */
    LPHY_CODE_ENCP64 = 6,  /* encodeParity64 (:367-371)                             */
    LPHY_CODE_CHKP64 = 7   /* checkParity64 (:357-365); flags bit0 error             */
};
enum lphy_sum_kind {
    LPHY_SUM_SX1272_CRC = 0, /* sx1272DataChecksum over `len` bytes (LoRaCodes.hpp:92-105) */
    LPHY_SUM_HEADER = 1,     /* headerChecksum of the row's first 2 bytes (:43-67)        */
    LPHY_SUM_CHECKSUM8 = 2   /* checksum8 over `len` bytes (:32-41)                       */
};

/* binaryToGray16 (to_binary = 0) / grayToBinary16 (1), in place
 * (LoRaCodes.hpp:201-222). */
int lphy_hip_gray_batch(uint16_t* d_syms, size_t count, int to_binary, void* stream);

/* diagonalInterleaveSx (LoRaCodes.hpp:376-393) per row: cw_per_frame / ppm
 * blocks of ppm codewords -> (4 + rdd) symbols each.  -ERANGE when a row's
 * symbols exceed sym_stride.  1 <= ppm <= 16, rdd <= 4. */
int lphy_hip_interleave_batch(const uint8_t* d_cw, size_t frames, size_t cw_stride, size_t cw_per_frame,
                              uint16_t* d_syms, size_t sym_stride, unsigned ppm, unsigned rdd,
                              void* stream);

/* diagonalDeterleaveSx (LoRaCodes.hpp:396-412) per row: syms_per_frame /
 * (4 + rdd) blocks -> ppm codewords each, written as the reference leaves a
 * zero-initialised codeword buffer. */
int lphy_hip_deinterleave_batch(const uint16_t* d_syms, size_t frames, size_t sym_stride,
                                size_t syms_per_frame, uint8_t* d_cw, size_t cw_stride, unsigned ppm,
                                unsigned rdd, void* stream);

/* Whitening / de-whitening of the first `len` bytes of every row in place
 * (the generators are involutions).  bit_ofs and rdd as the reference's
 * bitOfs / RDD (ignored by LPHY_WHITEN_SX1232). */
int lphy_hip_whiten_batch(uint8_t* d_bytes, size_t frames, size_t stride, size_t len, int kind,
                          int bit_ofs, unsigned rdd, void* stream);

/* Hamming / parity code `op` on `count` bytes in place; the decoders' error
 * flags go to d_flags[i] when it is not NULL. */
int lphy_hip_hamming_batch(uint8_t* d_bytes, size_t count, int op, uint8_t* d_flags, void* stream);

/* Checksum `kind` of every row -> d_out[frame] (uint16). */
int lphy_hip_checksum_batch(const uint8_t* d_bytes, size_t frames, size_t stride, size_t len, int kind,
                            uint16_t* d_out, void* stream);

/* lora_encode (LoRaEncoder.cpp:6-18) per row: byte j of the first `len`
 * bytes -> symbols 2j, 2j+1 (encodeHamming84sx of the high, low nibble),
 * the symbols modulate_batch takes.  -ERANGE when 2*len > sym_stride. */
int lphy_hip_lora_encode_batch(const uint8_t* d_bytes, size_t frames, size_t stride, size_t len,
                               uint16_t* d_syms, size_t sym_stride, void* stream);

/* ------------------------------------------------------------------------
 * LoRaWAN MAC helpers batched: lorawan::compute_mic
 * (lorawan.cpp:35-98, AES-128 CMAC over B0 || data) and parse_frame's
 * checks (lorawan.cpp:150-176) on the decoded bytes of many frames at once.
 * Keys are 16-byte records in device memory (d_keys, 16-byte aligned;
 * -EINVAL otherwise).
 * --------------------------------------------------------------------- */
typedef struct lphy_lorawan_desc { /* one MIC job */
    uint64_t offset;   /* byte offset of the frame's MHDR..FRMPayload in d_bytes */
    uint32_t len;      /* bytes the MIC covers (compute_mic's len)            */
    uint32_t devaddr;
    uint32_t fcnt;     /* 32-bit frame counter as compute_mic takes it        */
    uint32_t key;      /* index into d_keys                                   */
    uint32_t uplink;   /* nonzero: uplink (B0 byte 5 = 0)                     */
    uint32_t reserved;
} lphy_lorawan_desc;

typedef struct lphy_lorawan_frame { /* parse_frame's outcome for one row */
    int32_t  status;          /* parse_frame's return: FRMPayload length, or
                                 -EINVAL (MIC mismatch) / -ERANGE (short frame,
                                 FOpts past the MIC); -ENOKEY: key index
                                 >= nkeys (not a reference outcome)          */
    uint32_t devaddr;
    uint32_t mic;             /* MIC the frame carries (last 4 bytes)         */
    uint32_t calc_mic;        /* MIC computed over the rest                   */
    uint32_t payload_offset;  /* FRMPayload's offset in the row (status >= 0) */
    uint32_t payload_len;
    uint16_t fcnt;
    uint8_t  mhdr;            /* MType = mhdr >> 5, Major = mhdr & 3          */
    uint8_t  fctrl;           /* FOpts (at offset 8) length = fctrl & 0x0F    */
    uint8_t  fopts_len;
    uint8_t  reserved[3];
} lphy_lorawan_frame;         /* 32 bytes; all-zero but status when len < 12 */

#define LPHY_LW_APPEND 1u  /* mic_batch: also store the 4 MIC bytes (little
                              endian) right after each frame's data, as
                              build_frame does (lorawan.cpp:131-134) */

/* compute_mic for every descriptor -> d_mic[i] (NULL allowed with
 * LPHY_LW_APPEND).  d_bytes is written only with LPHY_LW_APPEND.  A
 * descriptor naming a key >= nkeys gets MIC 0 and nothing appended. */
int lphy_hip_lorawan_mic_batch(uint8_t* d_bytes, const lphy_lorawan_desc* d_desc, size_t frames,
                               const uint8_t* d_keys, size_t nkeys, uint32_t* d_mic, unsigned flags,
                               void* stream);

/* parse_frame's checks on `frames` rows of decoded bytes `stride` apart
 * (e.g. demod_batch's d_bytes): row i holds d_lens[i] bytes (d_lens NULL:
 * `len` each) and uses key d_key_index[i] (NULL: key 0).  Results in
 * d_out[i].  Lengths up to 65535 bytes and at most `stride`: a row whose
 * d_lens[i] exceeds either gets status -ERANGE and nothing of it is read
 * (a fixed `len` beyond them is -EINVAL for the whole call). */
int lphy_hip_lorawan_parse_batch(const uint8_t* d_bytes, size_t frames, size_t stride,
                                 const uint32_t* d_lens, size_t len, const uint8_t* d_keys, size_t nkeys,
                                 const uint32_t* d_key_index, lphy_lorawan_frame* d_out, void* stream);

/* One compute_mic through the batch kernel, host buffers (device `device`);
 * serialised process-wide.  Returns 0, -EINVAL, -ENODEV or -EIO. */
int lphy_hip_lorawan_mic_host(int device, const uint8_t key[16], int uplink, uint32_t devaddr, uint32_t fcnt,
                              const uint8_t* data, size_t len, uint32_t* mic);

#ifdef __cplusplus
}
#endif
#endif /* LPHY_HIP_H */
