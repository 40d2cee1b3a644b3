"""Per-phase wall-clock split of k_mod_fast (one-launch modulator) for one
66-symbol packet at a time, from a -DLPHY_PROFILE_PHASES
-DLPHY_MODFAST_CLOCKS build of the library (tools/ubench/mfclk).  Timing aid
only.    python tools/modfast_phases.py <lib.so> [sf ...]   (GPU box)"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "lora-sdr-lightweight-standalone-library-clean_amd"))
import lphy  # noqa: E402

NAMES = ["f rows + sums", "estimates", "row walks + pivots", "corrected + windows + sym 0",
         "candidate walks", "chain", "starts + rows + sincos"]


def main():
    lib = lphy.use(sys.argv[1])
    lib.lphy_hip_phase_cycles.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    for sf in [int(a) for a in sys.argv[2:]] or [7, 8]:
        d = lphy.Demodulator(sf)
        rng = np.random.default_rng(sf)
        out = (C.c_ulonglong * 8)()
        for _ in range(20):
            d.modulate_host(rng.integers(0, 1 << sf, 64, dtype=np.uint16), 1.0, 0x12)
        lib.lphy_hip_phase_cycles(d.ctx, out)
        n = 200
        for _ in range(n):
            d.modulate_host(rng.integers(0, 1 << sf, 64, dtype=np.uint16), 1.0, 0x12)
        lib.lphy_hip_phase_cycles(d.ctx, out)
        us = [out[k] / n / 100.0 for k in range(7)]  # wall_clock64: 100 MHz
        print(f"SF{sf}: total {sum(us):.1f} us: " + ", ".join(f"{a} {b:.1f}" for a, b in zip(NAMES, us)),
              flush=True)
        d.close()


if __name__ == "__main__":
    main()
