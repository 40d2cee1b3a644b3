"""Build-flag / source variants of liblphy_hip.so restricted to one SF (the
host TU plus that SF's kernel TU) and time their kernels on the bench workload.
  python tools/ubench/variants.py build <sf> name:"flags" ...   (dev container)
  python tools/ubench/variants.py run <sf> name ...             (GPU box)
Timing aid only."""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
PKG = ROOT / "lora-sdr-lightweight-standalone-library-clean_amd"
HERE = Path(__file__).resolve().parent


def build(sf, specs):
    procs = []
    for spec in specs:
        name, _, flags = spec.partition(":")
        so = HERE / f"var_{name}.so"
        cmd = (f"/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off "
               f"-fno-slp-vectorize -fPIC -shared -DLPHY_SF={sf} {flags} -I{ROOT}/include "
               f"-I{PKG}/csrc -o {so} {PKG}/csrc/lphy_hip.hip {PKG}/csrc/lphy_sf.hip "
               f"{PKG}/csrc/lphy_stream.hip {PKG}/csrc/lphy_codes.hip {PKG}/csrc/lphy_lorawan.hip")
        procs.append((name, subprocess.Popen(cmd, shell=True)))
    for name, p in procs:
        assert p.wait() == 0, name
        print("built", name)


def run(sf, names):
    sys.path.insert(0, str(ROOT))
    import torch
    import bench
    lphy = bench.lphy
    for name in names:
        lphy.use(HERE / f"var_{name}.so")
        wl = bench.Workload(sf, 125000, bench.DEFAULT_FRAMES[sf], 0, torch.device("cuda:0"))
        mode = lphy.MODE_DECHIRP_LORA_DEMODULATE
        D = lphy.F_DECODE
        both = lphy.F_STAGE_PROLOGUE | lphy.F_STAGE_SYMBOLS
        full = wl._event_ms(mode, D, 10)
        fused = wl._event_ms(mode, D | both, 10)
        sym = wl._event_ms(mode, D | lphy.F_UNFUSED | lphy.F_STAGE_SYMBOLS, 10)
        fin = wl._event_ms(mode, D | lphy.F_STAGE_FINAL, 10)
        extra = ""
        lib = lphy.load()
        if hasattr(lib, "lphy_hip_phase_cycles"):
            import ctypes as C
            out = (C.c_ulonglong * 8)()
            lib.lphy_hip_phase_cycles.argtypes = [C.c_void_p, C.c_void_p]
            lib.lphy_hip_phase_cycles(wl.dem.ctx, out)  # clear
            wl._event_ms(mode, D | lphy.F_UNFUSED | lphy.F_STAGE_SYMBOLS, 1)
            lib.lphy_hip_phase_cycles(wl.dem.ctx, out)
            tot = sum(out[:3]) or 1
            extra = " phases stage/fft/tail = " + "/".join(f"{out[i] / tot:.2f}" for i in range(3))
        wl.run(mode)
        chk = wl.check(mode)
        print(f"{name:14s} SF{sf}: full {full:.3f} ms  fused {fused:.3f} ms  k_demod {sym:.3f} ms  final {fin * 1e3:.1f} us  "
              f"ok={chk['payloads_recovered']}/{chk['frames']} oracle={chk['oracle_frames_bit_exact']}{extra}",
              flush=True)
        del wl
        torch.cuda.empty_cache()


if __name__ == "__main__":
    what, sf = sys.argv[1], int(sys.argv[2])
    (build if what == "build" else run)(sf, sys.argv[3:])
