#!/usr/bin/env python3
"""Share of symbols proven without their transform (the Parseval / bin-set
certificates of k_wave), per SF and mode, on the bench's IQ (lora_modulate
of random payloads): the test build's counter (lphy_hip_test_counter) and
the exact re-runs, over one fused launch.  Diagnostic aid (GPU box).

  python tools/pv_count.py [frames] [sf ...]
"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "lora-sdr-lightweight-standalone-library-clean_amd"))
import lphy  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
sfs = [int(a) for a in sys.argv[2:]] or [7, 8, 9, 10, 11, 12]
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
for sf in sfs:
    N = 1 << sf
    fs = 66 * N
    rng = np.random.default_rng(0x5EED + sf)
    pay = rng.integers(0, 256, (frames, 32), dtype=np.uint8)
    syms_in = torch.from_numpy(lphy.encode_payloads(pay).view(np.int16).reshape(-1).copy()).to(dev)
    iq = torch.empty(frames * fs * 2, dtype=torch.float32, device=dev)
    d = lphy.Demodulator(sf, test_build=True)
    d.set_fused_min_frames(0)
    d.modulate_batch(syms_in, frames, 64, iq, 1.0, 0x12, st)
    out = torch.zeros(frames * 64, dtype=torch.int16, device=dev)
    meta = torch.zeros(frames * 32, dtype=torch.uint8, device=dev)
    pl = torch.zeros(frames * 32, dtype=torch.uint8, device=dev)
    for mode in (0, 2):
        d.parseval_count(reset=True)
        d.recheck_count(reset=True)
        d.demod_batch(iq, frames, fs, out, meta, mode, lphy.F_DECODE, payload=pl, stream=st)
        torch.cuda.synchronize()
        pv, rc = d.parseval_count(reset=True), d.recheck_count(reset=True)
        print(f"SF{sf} mode {mode}: proven without transform {pv}/{frames * 66} "
              f"({pv / (frames * 66):.4f}), exact re-runs {rc}", flush=True)
    d.close()
