"""Per-phase clock shares of the fused SF 9-12 wave kernel (timing aid).
Build: python tools/ubench/variants.py build <sf> ph<sf>:"-DLPHY_PROFILE_PHASES"
Run:   python tools/ubench/wave_phases.py <sf> [mode] [variant]   (GPU box; mode default 2,
       variant default ph<sf>: var_<variant>.so)
Phases (k_wave, lphy_wave.h WPH): 0 wait for the unit's IQ, 1 staging,
2 pass 1, 3 exchange + next DMA, 4 pass 2, 5 top two / certificate / stores,
6 estimate units and frame close, 7 the next frame's two-symbol
max-abs scan and the schedule cursor."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402

lphy = bench.lphy
sf = int(sys.argv[1]) if len(sys.argv) > 1 else 12
var = sys.argv[3] if len(sys.argv) > 3 else f"ph{sf}"
lphy.use(Path(__file__).resolve().parent / f"var_{var}.so")
wl = bench.Workload(sf, 125000, bench.DEFAULT_FRAMES[sf], 0, torch.device("cuda:0"))
mode = int(sys.argv[2]) if len(sys.argv) > 2 else lphy.MODE_DECHIRP_LORA_DEMODULATE
flags = lphy.F_DECODE | lphy.F_STAGE_PROLOGUE | lphy.F_STAGE_SYMBOLS
lib = lphy.load()
lib.lphy_hip_phase_cycles.argtypes = [C.c_void_p, C.c_void_p]
out = (C.c_ulonglong * 8)()
wl._event_ms(mode, flags, 3)
lib.lphy_hip_phase_cycles(wl.dem.ctx, out)  # clear
ms = wl._event_ms(mode, flags, 1)
lib.lphy_hip_phase_cycles(wl.dem.ctx, out)
tot = sum(out) or 1
names = ["iq_wait", "staging", "parseval_sums+lead | transform: -", "pv_candidate | rot+pass1+exch+dma", "pv_dma_issue | pass2", "top2+cert+stores", "estimate+close", "scan+cursor"]
print(f"{var} SF{sf} mode {mode} fused {ms:.3f} ms; phase shares: " + ", ".join(f"{n} {out[i] / tot:.3f}" for i, n in enumerate(names)))
