"""A/B timing of the fused single launch (k_frames) against the separate
launches on one GPU, for the bench workload of a given SF.  Tuning aid.
Usage: python tools/stream_tune.py [sf] [frames] [mode]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

lphy = bench.lphy


def main():
    sf = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else bench.DEFAULT_FRAMES[sf]
    mode = int(sys.argv[3]) if len(sys.argv) > 3 else lphy.MODE_DECHIRP_LORA_DEMODULATE
    wl = bench.Workload(sf, 125000, frames, 0, torch.device("cuda:0"))

    def run(flags, reps=10):
        wl.run(mode, flags)
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            wl.run(mode, flags)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    for name, fl in (("unfused", lphy.F_DECODE | lphy.F_UNFUSED), ("fused", lphy.F_DECODE)):
        ms = run(fl)
        chk = wl.check(mode)
        nsym = frames * bench.DATA_SYMS
        print(f"sf={sf} frames={frames} mode={mode} {name}: {ms:.3f} ms  {nsym / ms / 1e6:.3f} Gsym/s "
              f"ok={chk['payloads_recovered']}/{chk['frames']} oracle={chk['oracle_frames_bit_exact']}",
              flush=True)


if __name__ == "__main__":
    main()
