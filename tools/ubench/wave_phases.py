"""k_wave phase clocks (timing aid only): per-wave clock sums of the unit
phases (DMA wait, staging, pass 1, exchange + DMA issue, pass 2, argmax +
store, estimate units, other) on the bench workload of one SF.
Needs a variant built with -DLPHY_PROFILE_PHASES (variants.py build).
  python tools/ubench/wave_phases.py <sf> <variant> [mode]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
import bench  # noqa: E402

sf, name = int(sys.argv[1]), sys.argv[2]
mode = int(sys.argv[3]) if len(sys.argv) > 3 else 2
lphy = bench.lphy
lphy.use(Path(__file__).resolve().parent / f"var_{name}.so")
wl = bench.Workload(sf, 125000, bench.DEFAULT_FRAMES[sf], 0, torch.device("cuda:0"))
flags = lphy.F_DECODE | lphy.F_STAGE_PROLOGUE | lphy.F_STAGE_SYMBOLS
ms = wl._event_ms(mode, flags, 10)
lib = lphy.load()
out = (C.c_ulonglong * 8)()
lib.lphy_hip_phase_cycles.argtypes = [C.c_void_p, C.c_void_p]
lib.lphy_hip_phase_cycles(wl.dem.ctx, out)
wl._event_ms(mode, flags, 1, warmup=0)
lib.lphy_hip_phase_cycles(wl.dem.ctx, out)
names = ["dma_wait", "staging", "pass1", "exch+dma", "pass2", "argmax+out", "estimate", "other"]
tot = sum(out) or 1
waves = min(256, (wl.frames + 3) // 4) * 4
units = wl.frames * (66 + 2) / (64 // max((1 << sf) // 64, 1))
print(f"SF{sf} mode {mode} {name}: {ms:.3f} ms/launch (phase-clock build), per-wave cycles {tot / waves:.0f}, "
      f"per unit {tot / units:.0f}", flush=True)
for n, v in zip(names, out):
    print(f"  {n:11s} {v / tot:6.3f}  {v / units:8.0f} cycles/unit", flush=True)
