"""Fused (k_frames / k_wave*) against the separate launches (LPHY_F_UNFUSED:
k_maxabs / k_estimate + symbol-parallel k_demod + k_post) by batch size:
device time per demod_batch call (HIP events, the bench's Workload), mode 2
with decode, for the frame counts below which the fused kernels cannot fill
the GPU (one frame per wavefront).  Feeds the library's fused_min_frames.
  python tools/fused_crossover.py [out.json [sf ...]]"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

lphy = bench.lphy


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else ""
    sfs = [int(a) for a in sys.argv[2:]] or [7, 8, 9, 10, 11, 12]
    dev = torch.device("cuda:0")
    lphy.FUSED_MIN_FRAMES = 0  # every batch to the fused kernels unless LPHY_F_UNFUSED
    mode = lphy.MODE_DECHIRP_LORA_DEMODULATE
    rows = []
    for sf in sfs:
        for frames in (1, 2, 4, 16, 64, 256, 512, 1024, 2048):
            wl = bench.Workload(sf, 125000, frames, 0, dev)
            fused = wl._event_ms(mode, lphy.F_DECODE, 20, warmup=5)
            sep = wl._event_ms(mode, lphy.F_DECODE | lphy.F_UNFUSED, 20, warmup=5)
            rows.append({"sf": sf, "frames": frames, "fused_ms": fused, "unfused_ms": sep})
            print(json.dumps(rows[-1]), flush=True)
            del wl
            torch.cuda.empty_cache()
    if out:
        Path(out).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
