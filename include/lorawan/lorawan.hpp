// lorawan:: — the LoRaWAN MAC helpers of the reference
// (include/lorawan/lorawan.hpp:8-77 there), same names, types and return
// codes, implemented by liblora_phy_amd.so on top of the MI355X C ABI
// (include/lphy_hip.h): the MIC is computed by the GPU CMAC kernel
// (csrc/lphy_lorawan.hip) and parse_frame decodes through lora_phy::decode
// (GPU).  For many frames at once use lphy_hip_lorawan_mic_batch /
// lphy_hip_lorawan_parse_batch directly.
#pragma once

#include <cstdint>
#include <vector>

#include <lora_phy/phy.hpp>

namespace lorawan {

// MHDR message types (3 bits, MHDR bits 7..5).
enum class MType : uint8_t {
    JoinRequest = 0,
    JoinAccept = 1,
    UnconfirmedDataUp = 2,
    UnconfirmedDataDown = 3,
    ConfirmedDataUp = 4,
    ConfirmedDataDown = 5,
    RFU = 6,
    Proprietary = 7,
};

struct MHDR {
    MType mtype{MType::UnconfirmedDataUp};
    uint8_t major{0};
};

struct MACCommand {
    uint8_t cid{};
    std::vector<uint8_t> payload;
};

struct FHDR {
    uint32_t devaddr{};
    uint8_t fctrl{};              // bits 3..0: FOpts length
    uint16_t fcnt{};
    std::vector<uint8_t> fopts;   // MAC commands, raw
};

struct Frame {
    MHDR mhdr;
    FHDR fhdr;
    std::vector<uint8_t> payload;  // FRMPayload
};

// AES-128 CMAC MIC over B0 || data (little-endian first four tag bytes).
// There is no error return in this signature: if the GPU path fails the
// reason goes to stderr and the result is 0.
uint32_t compute_mic(const uint8_t nwk_skey[16], bool uplink, uint32_t devaddr, uint32_t fcnt,
                     const uint8_t* data, size_t len);

// MHDR | DevAddr | FCtrl | FCnt | FOpts | payload | MIC into tmp_bytes, then
// lora_phy::encode into symbols.  Returns the symbol count, -EINVAL for a
// null argument, -ERANGE when tmp_cap or symbol_cap is too small.
ssize_t build_frame(lora_phy::lora_workspace* ws, const uint8_t nwk_skey[16], const Frame& frame,
                    uint16_t* symbols, size_t symbol_cap, uint8_t* tmp_bytes, size_t tmp_cap);

// lora_phy::decode into tmp_bytes, MIC check, then the fields into `out`.
// Returns the FRMPayload length, a decode error, -ERANGE (fewer than 12
// bytes, FOpts running into the MIC) or -EINVAL (MIC mismatch).
ssize_t parse_frame(lora_phy::lora_workspace* ws, const uint8_t nwk_skey[16], const uint16_t* symbols,
                    size_t symbol_count, Frame& out, uint8_t* tmp_bytes, size_t tmp_cap);

}  // namespace lorawan
