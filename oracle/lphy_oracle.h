/* TEST INFRASTRUCTURE ONLY — the CPU oracle.
 *
 * Plain-C restatement of the reference LoRa PHY hot path
 * (/root/reference/src/phy, include/lora_phy).  Used only by tests/, by
 * __graft_entry__.smoke() as the checker and by bench.py's cpu_baseline leg.
 * The product (liblphy_hip.so / liblora_phy_amd.so) never links or calls it.
 *
 * Complex buffers are interleaved float32 (re, im) pairs, i.e. the memory
 * layout of std::complex<float>.
 *
 * Pinned against oracle/_ref (the reference compiled from its own sources)
 * and the committed fixtures under tests/golden/ — see tests/test_oracle.py.
 */
#ifndef LPHY_ORACLE_H
#define LPHY_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include <sys/types.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ChirpGenerator.hpp:24-51 */
int orc_genchirp(float* out, int N, int osr, int NN, float f0, int down,
                 float ampl, float* phase, float bw_scale);

/* kissfft.hh:71-185 — forward, unscaled, KISS-identical arithmetic */
void orc_fft(const float* in, float* out, int nfft);

/* LoRaDetector.hpp:39-74.  Returns argmax index; power/fIndex out. */
size_t orc_detect(const float* fft_in, float* fft_out, int N, float* power,
                  float* power_avg, float* findex);

/* LoRaMod.cpp:8-43 */
size_t orc_lora_modulate(const uint16_t* syms, size_t n, float* out,
                         unsigned sf, unsigned osr, unsigned bw_hz,
                         float ampl, uint8_t sync);

/* tests/e2e_chain_test.cpp:80-93 (whole symbols; tail zeroed) */
void orc_dechirp(const float* in, float* out, size_t count, unsigned sf,
                 unsigned bw_hz);

/* LoRaEncoder.cpp:6-18 / LoRaDecoder.cpp:7-21 */
size_t orc_lora_encode(const uint8_t* bytes, size_t n, uint16_t* out);
ssize_t orc_lora_decode(const uint16_t* syms, size_t n, uint8_t* out);

/* LoRaCodes.hpp:92-105, 229-281 */
uint16_t orc_sx1272_checksum(const uint8_t* data, int len);
uint8_t orc_encode_hamming84(uint8_t x);
uint8_t orc_decode_hamming84(uint8_t b);

/* LoRaDemod.cpp:50-197 ("mode B": pre-dechirped input).
 * scratch_len: capacity of the caller's scratch (0 = none).
 * metrics_out[0..1] = {cfo, time_offset} (may be NULL). */
ssize_t orc_lora_demodulate(unsigned sf, int hann, const float* samples,
                            size_t count, uint16_t* out, unsigned osr,
                            uint8_t* out_sync, size_t scratch_len,
                            float* metrics_out);

/* phy.cpp:182-243 ("mode A": lora_phy::demodulate).  Returns the reference
 * return value; metrics_out = {cfo, time_offset}; *sync_out = ws->sync_word
 * after the call (initial value sync_in). */
ssize_t orc_demodulate(unsigned sf, unsigned bw_hz, unsigned osr, int hann,
                       const float* iq, size_t count, uint16_t* syms,
                       size_t cap, float* metrics_out, uint8_t sync_in,
                       uint8_t* sync_out);

/* phy.cpp:81-148 */
void orc_estimate_offsets(unsigned sf, unsigned osr, int hann,
                          const float* iq, size_t count, float* metrics_out);

/* phy.cpp:150-180, in place, with ws->metrics = {cfo, time_offset} */
void orc_compensate_offsets(unsigned sf, unsigned osr, float cfo,
                            float time_offset, float* iq, size_t count);

/* phy.cpp:245-261 (crc_ok written to *crc_out when the call gets that far) */
ssize_t orc_decode(const uint16_t* syms, size_t n, uint8_t* out, size_t cap,
                   uint8_t* crc_out);

/* LoRaCodes.hpp helpers, restated for the GPU batch
 * kernels' parity tests.  kind / op numbering as include/lphy_hip.h. */
uint16_t orc_gray(uint16_t v, int to_binary);                         /* :201-222 */
void orc_interleave(const uint8_t* cw, size_t ncw, uint16_t* syms,
                    size_t ppm, size_t rdd);                          /* :376-393 */
void orc_deinterleave(const uint16_t* syms, size_t nsyms, uint8_t* cw,
                      size_t ppm, size_t rdd);                        /* :396-412 */
void orc_whiten(uint8_t* buf, size_t len, int kind, int bit_ofs,
                unsigned rdd);                                        /* :111-189 */
uint8_t orc_hamming(uint8_t x, int op, uint8_t* flags);               /* :229-371 */
uint16_t orc_checksum(const uint8_t* buf, size_t len, int kind);      /* :32-105  */

/* LoRaWAN: FIPS-197 AES-128 encryption of one block in
 * place; compute_mic (lorawan.cpp:35-98); parse_frame's checks on decoded
 * bytes (lorawan.cpp:150-176), rec[10] as documented in lphy_oracle.c. */
void orc_aes128(const uint8_t key[16], uint8_t blk[16]);
uint32_t orc_lorawan_mic(const uint8_t key[16], int uplink, uint32_t devaddr,
                         uint32_t fcnt, const uint8_t* data, size_t len);
void orc_lorawan_parse(const uint8_t key[16], const uint8_t* bytes, size_t len,
                       int64_t* rec);

/* Multi-threaded timing harness for bench.py's cpu_baseline ("port" kind):
 * mode 1 = dechirp + lora_demodulate + lora_decode per frame,
 * mode 0 = demodulate + decode.  Returns wall seconds. */
double orc_bench(int mode, unsigned sf, unsigned bw_hz, const float* iq,
                 size_t frames, size_t frame_samples, uint8_t* bytes_out,
                 int threads);

#ifdef __cplusplus
}
#endif
#endif
