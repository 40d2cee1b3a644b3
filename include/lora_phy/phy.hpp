/**
 * @file lora_phy/phy.hpp
 * lora_phy:: C++17 API of the MI355X LoRa PHY (liblora_phy_amd.so).
 *
 * Replacement for the reference header /root/reference/include/lora_phy/
 * phy.hpp, source- and ABI/layout-compatible for its public API:
 *   - the same free functions with the same signatures and negative-errno
 *     returns (reference phy.hpp:104-161, 195-224);
 *   - the same caller-owned structs with the same field sets, sizes and
 *     offsets (lora_workspace 66,136 B, lora_demod_workspace 115,064 B on
 *     x86-64; tests/test_abi_cpu.py compares them against the reference
 *     build).
 * Not carried over: the reference's internal FFT / detector classes
 * (kissfft.hh, LoRaDetector.hpp).  lora_demod_workspace keeps their storage
 * as opaque bytes (fft / detector are void*), so code that reaches into
 * those objects does not compile against this header.  The codec helpers
 * (LoRaCodes.hpp) and the chirp generator (ChirpGenerator.hpp) are shipped
 * beside it.
 * Demodulation, offset estimation, compensation, decoding and modulation run
 * on the GPU through the C ABI in lphy_hip.h; the structs here only carry
 * configuration and results between calls, as in the reference.
 */
#pragma once

#include <cstddef>
#include <cstdint>
#include <complex>
#include <sys/types.h>

namespace kissfft_utils {
constexpr std::size_t KISSFFT_MAX_N = 4096;       // largest N (SF12)
constexpr std::size_t KISSFFT_MAX_FACTORS = 32;
constexpr std::size_t KISSFFT_MAX_FFT_RADIX = 32;
}  // namespace kissfft_utils

/// FFT plan record embedded by value in the workspaces (layout of the
/// reference's kissfft_plan<T>, kissfft.hh:43-55).  init() fills it exactly
/// as the reference does so callers that inspect it see the same values.
template <typename T_scalar>
struct kissfft_plan {
    using scalar_type = T_scalar;
    using cpx_type = std::complex<scalar_type>;
    int nfft{};
    bool inverse{};
    int stages{};
    cpx_type twiddles[kissfft_utils::KISSFFT_MAX_N];
    int stageRadix[kissfft_utils::KISSFFT_MAX_FACTORS];
    int stageRemainder[kissfft_utils::KISSFFT_MAX_FACTORS];
};

namespace lora_phy {

constexpr float PI = 3.14159265358979323846f;

enum class window_type {
    window_none,
    window_hann,
};

enum class bandwidth : unsigned {
    bw_125 = 125000,
    bw_250 = 250000,
    bw_500 = 500000,
};

constexpr float bw_to_hz(bandwidth bw) { return static_cast<float>(static_cast<unsigned>(bw)); }
constexpr float bw_scale(bandwidth bw) { return bw_to_hz(bw) / 125000.0f; }

struct lora_params {
    unsigned sf{};
    bandwidth bw{bandwidth::bw_125};
    unsigned cr{};
    unsigned osr{1};
    window_type window{window_type::window_none};
    uint8_t sync_word{0x12};
};

struct lora_metrics {
    bool crc_ok{};
    float cfo{};
    float time_offset{};
};

struct lora_workspace {
    uint16_t* symbol_buf{};
    std::complex<float>* fft_in{};
    std::complex<float>* fft_out{};
    float* window{};
    window_type window_kind{window_type::window_none};
    kissfft_plan<float> plan_fwd{};
    kissfft_plan<float> plan_inv{};
    lora_metrics metrics{};
    unsigned osr{1};
    bandwidth bw{bandwidth::bw_125};
    uint8_t sync_word{0x12};
};

// High level API (reference phy.hpp:104-161)
int init(lora_workspace* ws, const lora_params* cfg);
void reset(lora_workspace* ws);
ssize_t encode(lora_workspace* ws, const uint8_t* payload, size_t payload_len,
               uint16_t* symbols, size_t symbol_cap);
ssize_t decode(lora_workspace* ws, const uint16_t* symbols, size_t symbol_count,
               uint8_t* payload, size_t payload_cap);
ssize_t modulate(lora_workspace* ws, const uint16_t* symbols, size_t symbol_count,
                 std::complex<float>* iq, size_t iq_cap);
ssize_t demodulate(lora_workspace* ws, const std::complex<float>* iq, size_t sample_count,
                   uint16_t* symbols, size_t symbol_cap);
void estimate_offsets(lora_workspace* ws, const std::complex<float>* samples,
                      size_t sample_count);
void compensate_offsets(const lora_workspace* ws, std::complex<float>* samples,
                        size_t sample_count);
const lora_metrics* get_last_metrics(const lora_workspace* ws);

/// Legacy demodulator workspace (reference phy.hpp:175-190).  The two
/// opaque buffers and pointers keep the reference layout; this
/// implementation stores no C++ objects in them.
struct lora_demod_workspace {
    static const size_t MAX_N = kissfft_utils::KISSFFT_MAX_N;
    size_t N{};
    std::complex<float> fft_in[MAX_N];
    std::complex<float> fft_out[MAX_N];
    float window[MAX_N];
    window_type window_kind{window_type::window_none};
    kissfft_plan<float> fft_plan{};
    alignas(8) unsigned char fft_buf[8];
    alignas(8) unsigned char detector_buf[40];
    void* fft{};
    void* detector{};
    lora_metrics metrics{};
    std::complex<float>* scratch{};
    size_t scratch_len{};
};

void lora_demod_init(lora_demod_workspace* ws, unsigned sf,
                     window_type win = window_type::window_none,
                     std::complex<float>* scratch = nullptr, size_t max_samples = 0);
void lora_demod_free(lora_demod_workspace* ws);
size_t lora_modulate(const uint16_t* symbols, size_t symbol_count,
                     std::complex<float>* out_samples, unsigned sf, unsigned osr,
                     bandwidth bw, float amplitude = 1.0f, uint8_t sync = 0x12);
ssize_t lora_demodulate(lora_demod_workspace* ws, const std::complex<float>* samples,
                        size_t sample_count, uint16_t* out_symbols, unsigned osr,
                        uint8_t* out_sync = nullptr);
size_t lora_encode(const uint8_t* bytes, size_t byte_count, uint16_t* out_symbols, unsigned sf);
ssize_t lora_decode(const uint16_t* symbols, size_t symbol_count, uint8_t* out_bytes);

// Batch extension (no reference counterpart): many frames in one call,
// host buffers; frames are consecutive in `iq`, frame_samples each.
// Returns 0 or a negative errno; per-frame status lands in `status`
// (may be null), per-frame sync words in `sync_words` (may be null).
int demodulate_batch(const lora_workspace* ws, const std::complex<float>* iq,
                     size_t frames, size_t frame_samples, uint16_t* symbols,
                     uint8_t* payloads, uint8_t* sync_words, int32_t* status);

}  // namespace lora_phy
