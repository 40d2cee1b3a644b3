// lorawan:: (include/lorawan/lorawan.hpp) over the MI355X C ABI.  Argument
// checks, byte layout and return codes follow the reference's
// src/lorawan/lorawan.cpp (file:line on each function); the MIC runs in the
// GPU CMAC kernel and the symbol decode in the GPU decoder.  No CPU
// fallback: without a usable HIP device compute_mic reports the failure and
// parse_frame returns the decoder's -ENODEV.
#include <lorawan/lorawan.hpp>
#include <lphy_hip.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>

namespace lorawan {
namespace {

int device_index() {
    const char* e = std::getenv("LPHY_DEVICE");
    return e ? std::atoi(e) : 0;
}

uint32_t le32(const uint8_t* p) {
    return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

// The MIC through the GPU CMAC, or the device error (-ENODEV, -EIO, ...):
// build_frame / parse_frame return that error rather than a frame built or
// accepted against a MIC of 0.
int gpu_mic(const uint8_t nwk_skey[16], bool uplink, uint32_t devaddr, uint32_t fcnt, const uint8_t* data,
            size_t len, uint32_t* mic) {
    *mic = 0;
    return lphy_hip_lorawan_mic_host(device_index(), nwk_skey, uplink ? 1 : 0, devaddr, fcnt, data, len, mic);
}

}  // namespace

// compute_mic has no error channel in the reference's signature: a device
// failure is reported on stderr and yields MIC 0 (the frame helpers below do
// not rely on it).
uint32_t compute_mic(const uint8_t nwk_skey[16], bool uplink, uint32_t devaddr, uint32_t fcnt,
                     const uint8_t* data, size_t len) {  // lorawan.cpp:35-98
    uint32_t mic = 0;
    if (const int rc = gpu_mic(nwk_skey, uplink, devaddr, fcnt, data, len, &mic)) {
        std::fprintf(stderr, "lorawan::compute_mic: GPU MIC failed (%d)\n", rc);
        return 0;
    }
    return mic;
}

ssize_t build_frame(lora_phy::lora_workspace* ws, const uint8_t nwk_skey[16], const Frame& frame,
                    uint16_t* symbols, size_t symbol_cap, uint8_t* tmp_bytes,
                    size_t tmp_cap) {  // lorawan.cpp:100-136
    if (!ws || !symbols || !tmp_bytes) return -EINVAL;
    const size_t nfo = frame.fhdr.fopts.size(), npay = frame.payload.size();
    if (12 + nfo + npay > tmp_cap) return -ERANGE;
    uint8_t* p = tmp_bytes;
    *p++ = static_cast<uint8_t>(static_cast<uint8_t>(frame.mhdr.mtype) << 5 | (frame.mhdr.major & 0x3));
    for (int i = 0; i < 4; ++i) *p++ = static_cast<uint8_t>(frame.fhdr.devaddr >> (8 * i));
    *p++ = static_cast<uint8_t>((frame.fhdr.fctrl & 0xF0) | (nfo & 0x0F));
    *p++ = static_cast<uint8_t>(frame.fhdr.fcnt);
    *p++ = static_cast<uint8_t>(frame.fhdr.fcnt >> 8);
    for (uint8_t b : frame.fhdr.fopts) *p++ = b;
    for (uint8_t b : frame.payload) *p++ = b;
    const size_t n = static_cast<size_t>(p - tmp_bytes);
    const bool uplink = (static_cast<uint8_t>(frame.mhdr.mtype) & 1) == 0;
    uint32_t mic = 0;
    if (const int rc = gpu_mic(nwk_skey, uplink, frame.fhdr.devaddr, frame.fhdr.fcnt, tmp_bytes, n, &mic))
        return rc;
    for (int i = 0; i < 4; ++i) *p++ = static_cast<uint8_t>(mic >> (8 * i));
    return lora_phy::encode(ws, tmp_bytes, n + 4, symbols, symbol_cap);
}

ssize_t parse_frame(lora_phy::lora_workspace* ws, const uint8_t nwk_skey[16], const uint16_t* symbols,
                    size_t symbol_count, Frame& out, uint8_t* tmp_bytes,
                    size_t tmp_cap) {  // lorawan.cpp:138-177
    if (!ws || !symbols || !tmp_bytes) return -EINVAL;
    const ssize_t got = lora_phy::decode(ws, symbols, symbol_count, tmp_bytes, tmp_cap);
    if (got < 0) return got;
    const size_t len = static_cast<size_t>(got);
    if (len < 12) return -ERANGE;
    const uint8_t mhdr = tmp_bytes[0];
    const uint32_t devaddr = le32(tmp_bytes + 1);
    const uint16_t fcnt = static_cast<uint16_t>(tmp_bytes[6] | tmp_bytes[7] << 8);
    const uint32_t carried = le32(tmp_bytes + len - 4);
    uint32_t calc = 0;
    if (const int rc = gpu_mic(nwk_skey, ((mhdr >> 5) & 1) == 0, devaddr, fcnt, tmp_bytes, len - 4, &calc))
        return rc;
    if (carried != calc) return -EINVAL;
    // fields land in `out` in the reference's order, so an FOpts overrun
    // leaves the same partial update (:163-172)
    out.mhdr.mtype = static_cast<MType>(mhdr >> 5);
    out.mhdr.major = mhdr & 0x3;
    out.fhdr.devaddr = devaddr;
    out.fhdr.fctrl = tmp_bytes[5];
    out.fhdr.fcnt = fcnt;
    const size_t fol = out.fhdr.fctrl & 0x0F;
    if (8 + fol > len - 4) return -ERANGE;
    out.fhdr.fopts.assign(tmp_bytes + 8, tmp_bytes + 8 + fol);
    out.payload.assign(tmp_bytes + 8 + fol, tmp_bytes + len - 4);
    return static_cast<ssize_t>(out.payload.size());
}

}  // namespace lorawan
