// lphy_sf.hip — the kernels of one spreading factor (built once per SF with
// -DLPHY_SF=n, see ../Makefile) and their launch table for lphy_hip.hip.
#include "lphy_kernels.h"

#ifndef LPHY_SF
#error "build with -DLPHY_SF=<1..12>"
#endif
#define LPHY_CAT2(a, b) a##b
#define LPHY_CAT(a, b) LPHY_CAT2(a, b)

// Explicit instantiations (both compilation passes: the device pass emits
// the kernels these launchers reference)
namespace {
template int launch_demod_sf<LPHY_SF>(const DemodArgs&, hipStream_t, bool, bool, int);
template int launch_frames_sf<LPHY_SF>(const DemodArgs&, hipStream_t);
template int launch_post_sf<LPHY_SF>(int, const DemodArgs&, const FinalArgs&, bool, bool, hipStream_t);
template int launch_estimate_sf<LPHY_SF>(const DemodArgs&, hipStream_t);
}  // namespace

#ifdef LPHY_DEBUG_BOUNDS
// this translation unit's failed index checks (lphy_fft.h bound_check)
namespace {
int read_violations(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bound_violations), sizeof(*out)) != hipSuccess) return -EIO;
    if (reset) {
        const unsigned long long z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_bound_violations), &z, sizeof(z)) != hipSuccess) return -EIO;
    }
    return 0;
}
}  // namespace
#endif

// host-side table (the device pass would otherwise emit it as a constant
// referencing host functions)
#ifndef __HIP_DEVICE_COMPILE__
namespace lphy {
const SfOps LPHY_CAT(sf_ops_, LPHY_SF) = {
    &launch_demod_sf<LPHY_SF>,
    &launch_frames_sf<LPHY_SF>,
    &launch_post_sf<LPHY_SF>,
    &launch_estimate_sf<LPHY_SF>,
#ifdef LPHY_DEBUG_BOUNDS
    &read_violations,
#else
    nullptr,
#endif
};
}  // namespace lphy
#endif
