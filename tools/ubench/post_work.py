"""Timing/diagnosis aid: after the fused launch alone (no k_post), how many
frames of the bench workload are left to k_post (status fix-up / recheck /
settle) and how many symbols carry the recheck sentinel, per mode.
python tools/ubench/post_work.py [sf]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

lphy = bench.lphy
sf = int(sys.argv[1]) if len(sys.argv) > 1 else 7
wl = bench.Workload(sf, 125000, bench.DEFAULT_FRAMES[sf], 0, torch.device("cuda:0"))
both = lphy.F_STAGE_PROLOGUE | lphy.F_STAGE_SYMBOLS
for mode in (lphy.MODE_DEMODULATE, lphy.MODE_DECHIRP_LORA_DEMODULATE):
    wl.run(mode, lphy.F_DECODE | both)
    torch.cuda.synchronize()
    meta = wl.meta.cpu().numpy().view(lphy.META_DTYPE)
    st = meta["status"]
    syms = wl.syms.cpu().numpy().view(np.uint16)
    names = {0x7f5a0001: "fixup", 0x7f5a0002: "recheck", 0x7f5a0003: "settle", 0x7f5a0004: "settle+recheck"}
    counts = {names.get(int(v), str(int(v))): int((st == v).sum()) for v in np.unique(st)}
    print(f"SF{sf} mode {mode}: frames {wl.frames}, statuses {counts}, recheck symbols {(syms == 0xffff).sum()}")
