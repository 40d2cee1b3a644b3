"""Timing aid: the per-step finalisation on the C1 workload - k_post with
fix-up and finalisation (the default step's second launch), k_post with the
finalisation only (LPHY_F_STAGE_FINAL), and k_finalize (lphy_hip_decode_batch)
on the same symbols.  python tools/ubench/final_cost.py [sf] [mode]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402

lphy = bench.lphy
sf = int(sys.argv[1]) if len(sys.argv) > 1 else 7
wl = bench.Workload(sf, 125000, bench.DEFAULT_FRAMES[sf], 0, torch.device("cuda:0"))
mode = int(sys.argv[2]) if len(sys.argv) > 2 else lphy.MODE_DECHIRP_LORA_DEMODULATE
D = lphy.F_DECODE
both = lphy.F_STAGE_PROLOGUE | lphy.F_STAGE_SYMBOLS
st = torch.cuda.current_stream().cuda_stream
per = wl.syms.numel() // wl.frames


def ev(fn, reps=50):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


full = ev(lambda: wl.run(mode, D))
fused = ev(lambda: wl.run(mode, D | both))
fin = ev(lambda: wl.run(mode, D | lphy.F_STAGE_FINAL))
kfin = ev(lambda: wl.dem.decode_batch(wl.syms, wl.frames, per, wl.pay, wl.meta, st))
print(f"SF{sf} mode {mode}: step {full:.1f} us, fused launch {fused:.1f} us (step - fused {full - fused:.1f}), "
      f"k_post finalisation only {fin:.1f} us, k_finalize {kfin:.1f} us")
for nf in (256, 1024, 4096, 16384, wl.frames):
    t = ev(lambda: wl.dem.decode_batch(wl.syms, nf, per, wl.pay, wl.meta, st))
    print(f"  k_finalize over {nf} frames: {t:.1f} us")
