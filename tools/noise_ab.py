"""Fused-kernel time under noise: k_wave (the product's choice from SF 7) vs
k_frames (the test build's LPHY_F_FRAMES_KERNEL) on the bench's frame shape
with AWGN added on the device (per-sample SNR; noisy symbols fail the
Parseval certificate and take k_wave's transform).  Timing aid only.
    python tools/noise_ab.py [sf ...]        (GPU box)"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

lphy = bench.lphy


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--lib=")]
    libs = [a[6:] for a in sys.argv[1:] if a.startswith("--lib=")]
    if libs:  # --lib=<variant .so>: time that build's default launch only
        lphy.use(libs[0])
    sfs = [int(a) for a in args] or [7, 8, 9, 10]
    dev = torch.device("cuda:0")
    mode = lphy.MODE_DECHIRP_LORA_DEMODULATE
    flags = lphy.F_DECODE | lphy.F_STAGE_PROLOGUE | lphy.F_STAGE_SYMBOLS
    for sf in sfs:
        wl = bench.Workload(sf, 125000, bench.DEFAULT_FRAMES[sf], 0, dev)
        clean = wl.iq.clone()
        test = lphy.Demodulator(sf, 125000, 1, lphy.WINDOW_NONE, device=0, test_build=True)
        test.set_fused_min_frames(0)
        for snr in (None, 10.0, 0.0, -10.0):
            wl.iq.copy_(clean)
            if snr is not None:
                g = torch.Generator(device=dev)
                g.manual_seed(1234 + sf)
                wl.iq.add_(torch.randn(wl.iq.shape, generator=g, device=dev) * float(np.sqrt(10 ** (-snr / 10) / 2)))
            t_wave = wl._event_ms(mode, flags, 10)
            if libs:
                print(f"SF{sf} snr {'clean' if snr is None else f'{snr:+.0f} dB'}: {Path(libs[0]).name} "
                      f"{t_wave:.3f} ms", flush=True)
                continue
            syms, pay, meta = wl.outs[0]
            st = torch.cuda.current_stream().cuda_stream

            def run_frames():
                test.demod_batch(wl.iq, wl.frames, wl.fs, syms, meta, mode, flags | lphy.F_FRAMES_KERNEL,
                                 payload=pay, stream=st)
            for _ in range(5):
                run_frames()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                run_frames()
            b.record()
            torch.cuda.synchronize()
            t_frames = a.elapsed_time(b) / 10
            print(f"SF{sf} snr {'clean' if snr is None else f'{snr:+.0f} dB'}: k_wave {t_wave:.3f} ms, "
                  f"k_frames {t_frames:.3f} ms", flush=True)
        test.close()
        del wl
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
