"""Drop-in boundary checks that need no GPU:
* liblphy_hip.so (the HIP product) loads and exports every function
  include/lphy_hip.h declares;
* liblora_phy_amd.so exports the lora_phy:: C++ API of include/lora_phy/phy.hpp
  (the reference's mangled names, phy.hpp:104-161,195-224 of the reference);
* the public structs keep the reference's sizes (callers size them at compile
  time) and lphy_frame_meta its 32-byte layout;
* without a GPU the entry points fail with an error code, never fall back."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "lora-sdr-lightweight-standalone-library-clean_amd"
HIP_SO = PKG / "lib" / "liblphy_hip.so"
CXX_SO = PKG / "lib" / "liblora_phy_amd.so"


def _declared_c_functions():
    text = (ROOT / "include" / "lphy_hip.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(lphy_hip_\w+)\s*\(", text, re.M)))


def _exports(so: Path):
    out = subprocess.run(["nm", "-D", "--defined-only", str(so)], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


@pytest.fixture(scope="module")
def built():
    if not HIP_SO.exists() or not CXX_SO.exists():
        subprocess.run(["make", "-s", "-C", str(PKG)], check=True)
    return True


def test_c_abi_exports_every_declared_function(built):
    decl = _declared_c_functions()
    assert len(decl) >= 15
    missing = [f for f in decl if f not in _exports(HIP_SO)]
    assert not missing, missing


def test_c_abi_loads_and_reports_version(built):
    lib = C.CDLL(str(HIP_SO))
    lib.lphy_hip_version.restype = C.c_char_p
    assert b"gfx950" in lib.lphy_hip_version()


def test_c_abi_argument_errors_without_device(built):
    lib = C.CDLL(str(HIP_SO))
    h = C.c_void_p()
    # argument validation precedes any device call
    assert lib.lphy_hip_ctx_create(None, 0, 7, 125000, 1, 0) == -22          # -EINVAL
    assert lib.lphy_hip_ctx_create(C.byref(h), 0, 13, 125000, 1, 0) == -22   # sf > 12
    assert lib.lphy_hip_ctx_create(C.byref(h), 0, 7, 100000, 1, 0) == -22    # bandwidth
    assert lib.lphy_hip_ctx_create(C.byref(h), 0, 7, 125000, 1, 9) == -22    # window
    assert lib.lphy_hip_demod_batch(None, None, 1, 128, None, None, None, 0, 0, None) == -22


def test_c_abi_no_silent_cpu_fallback(built):
    """On a host without a HIP device, creating a context fails loudly."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = C.CDLL(str(HIP_SO))
    h = C.c_void_p()
    assert lib.lphy_hip_ctx_create(C.byref(h), 0, 7, 125000, 1, 0) == -19    # -ENODEV


CXX_API = [
    "lora_phy::init(lora_phy::lora_workspace*, lora_phy::lora_params const*)",
    "lora_phy::reset(lora_phy::lora_workspace*)",
    "lora_phy::encode(lora_phy::lora_workspace*, unsigned char const*, unsigned long, unsigned short*, unsigned long)",
    "lora_phy::decode(lora_phy::lora_workspace*, unsigned short const*, unsigned long, unsigned char*, unsigned long)",
    "lora_phy::modulate(lora_phy::lora_workspace*, unsigned short const*, unsigned long, std::complex<float>*, unsigned long)",
    "lora_phy::demodulate(lora_phy::lora_workspace*, std::complex<float> const*, unsigned long, unsigned short*, unsigned long)",
    "lora_phy::estimate_offsets(lora_phy::lora_workspace*, std::complex<float> const*, unsigned long)",
    "lora_phy::compensate_offsets(lora_phy::lora_workspace const*, std::complex<float>*, unsigned long)",
    "lora_phy::get_last_metrics(lora_phy::lora_workspace const*)",
    "lora_phy::lora_demod_free(lora_phy::lora_demod_workspace*)",
    "lora_phy::lora_encode(unsigned char const*, unsigned long, unsigned short*, unsigned int)",
    "lora_phy::lora_decode(unsigned short const*, unsigned long, unsigned char*)",
]


def test_cxx_api_exports(built):
    out = subprocess.run(["nm", "-DC", "--defined-only", str(CXX_SO)], capture_output=True, text=True,
                         check=True).stdout
    missing = [f for f in CXX_API if f not in out]
    assert not missing, missing
    for name in ("lora_phy::lora_demod_init(", "lora_phy::lora_modulate(", "lora_phy::lora_demodulate("):
        assert name in out, name


def _sizes_of_our_headers():
    src = r'''
#include <cstdio>
#include <cstddef>
#include "lora_phy/phy.hpp"
#include "lphy_hip.h"
int main() {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(lora_phy::lora_workspace),
         sizeof(lora_phy::lora_demod_workspace), sizeof(lora_phy::lora_params),
         sizeof(lora_phy::lora_metrics), sizeof(lphy_frame_meta),
         offsetof(lphy_frame_meta, t_off), offsetof(lphy_frame_meta, sw0),
         offsetof(lphy_frame_meta, have_sync));
}
'''
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        (Path(d) / "s.cpp").write_text(src)
        subprocess.run(["g++", "-std=c++17", f"-I{ROOT / 'include'}", "-o", f"{d}/s", f"{d}/s.cpp"],
                       check=True)
        return [int(x) for x in subprocess.run([f"{d}/s"], capture_output=True, text=True,
                                                check=True).stdout.split()]


def test_struct_layouts():
    ws, dws, params, metrics, meta, t_off, sw0, have_sync = _sizes_of_our_headers()
    # lora_workspace 66,136 B, lora_demod_workspace 115,064 B
    assert (ws, dws) == (66136, 115064)
    assert (meta, t_off, sw0, have_sync) == (32, 16, 24, 31)
    from checkers import Reference, reference_available
    if reference_available():
        r = Reference().lib
        for n in ("ref_sizeof_workspace", "ref_sizeof_demod_workspace", "ref_sizeof_params",
                  "ref_sizeof_metrics"):
            getattr(r, n).restype = C.c_size_t
        assert (ws, dws, params, metrics) == (r.ref_sizeof_workspace(), r.ref_sizeof_demod_workspace(),
                                              r.ref_sizeof_params(), r.ref_sizeof_metrics())
