"""k_frames tile clocks (timing aid only): mixed (estimate-bearing) tiles vs
symbol-only tiles, and the fold/rotation-table tail of the mixed tiles.
Needs a variant built with -DLPHY_PROFILE_PHASES (variants.py build).
  python tools/ubench/frame_phases.py <sf> <variant> [mode]"""
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
mix, sym, fold, nmix = out[0], out[1], out[2], out[3]
N = 1 << sf
wt = 64 // max(N // 16, 1)
nsym = wl.frames * 68 // wt - nmix  # approximate: prefix tiles ignored
tot = mix + sym
print(f"SF{sf} mode {mode} {name}: {ms:.3f} ms; mixed tiles {mix / tot:.3f} of wave clocks "
      f"(fold+rtab+close tail {fold / tot:.3f}); mixed tiles {nmix}, "
      f"cycles per mixed tile {mix / max(nmix, 1):.0f}, per symbol-only tile {sym / max(nsym, 1):.0f}", flush=True)
