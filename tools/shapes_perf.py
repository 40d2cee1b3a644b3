#!/usr/bin/env python3
"""Throughput of the shapes the headline bench does not run (VERDICT r5
missing 2-3): per SF and shape, the device time of one whole demod_batch
call (every launch of the product path, HIP events on its stream) over a
resident synthetic batch, as data symbols/s and as a fraction of the 8 TB/s
HBM roofline of the call's algorithmic bytes (the IQ once + 2 B per output
symbol + the 32 B frame record).  Shapes:

  mode_A      lora_phy::demodulate (LPHY_MODE_DEMODULATE + decode), osr 1 -
              phy.cpp:182-243; the bench's IQ (lora_modulate of random payloads)
  hann        the bench's mode (dechirp -> lora_demodulate -> decode) with the
              Hann window context (LoRaDemod.cpp:16-24, phy.cpp:218-229)
  osr2/osr4   lora_phy::demodulate on oversampled IQ (lora_modulate at osr
              2 / 4; phy.cpp:107-113's best-of-osr estimate, strided symbols)
  short16     the bench's mode on frames of 16 data symbols (18 in all: below
              one k_wave unit at SF 7, 32 symbols)
  short8      ... 8 data symbols (10 in all: below one unit at SF 8, 16)

Writes a CSV (shape,sf,osr,mode,frames,symbols_per_frame,ms,symbols_per_s,
hbm_gbps,roofline_frac) and prints it.  Timing aid; the numbers are the
product library's (lib/liblphy_hip.so).
  python tools/shapes_perf.py out.csv [sf ...] [--shapes mode_A,hann,...]   (GPU box)"""
import csv
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "lora-sdr-lightweight-standalone-library-clean_amd"))
import lphy  # noqa: E402

BYTES_TARGET = 4.4e9  # IQ bytes per call (about the bench's C1 batch)
SHAPES = [("mode_A", 1, lphy.WINDOW_NONE, lphy.MODE_DEMODULATE, 64),
          ("hann", 1, lphy.WINDOW_HANN, lphy.MODE_DECHIRP_LORA_DEMODULATE, 64),
          ("osr2", 2, lphy.WINDOW_NONE, lphy.MODE_DEMODULATE, 64),
          ("osr4", 4, lphy.WINDOW_NONE, lphy.MODE_DEMODULATE, 64),
          ("short16", 1, lphy.WINDOW_NONE, lphy.MODE_DECHIRP_LORA_DEMODULATE, 16),
          ("short8", 1, lphy.WINDOW_NONE, lphy.MODE_DECHIRP_LORA_DEMODULATE, 8)]


def run_shape(dev, sf, name, osr, window, mode, nsyms, reps=20, warmup=10):
    N = 1 << sf
    fs = (nsyms + 2) * N * osr
    frames = int(BYTES_TARGET // (fs * 8))
    frames = max(256, min(frames, 1 << 17))
    d = lphy.Demodulator(sf, 125000, osr, window, device=dev.index)
    rng = np.random.default_rng(sf * 101 + osr)
    pay = rng.integers(0, 256, (frames, nsyms // 2), dtype=np.uint8)
    syms = lphy.encode_payloads(pay)
    st = torch.cuda.current_stream().cuda_stream
    t_in = torch.from_numpy(syms.view(np.int16).reshape(-1).copy()).to(dev)
    iq = torch.empty(frames * fs * 2, dtype=torch.float32, device=dev)
    d.modulate_batch(t_in, frames, nsyms, iq, 1.0, 0x12, st)
    per = d.syms_per_frame(fs, mode)
    out = torch.zeros(frames * per, dtype=torch.int16, device=dev)
    meta = torch.zeros(frames * 32, dtype=torch.uint8, device=dev)
    paybuf = torch.zeros(frames * max(per // 2, 1), dtype=torch.uint8, device=dev)
    run = lambda: d.demod_batch(iq, frames, fs, out, meta, mode, lphy.F_DECODE, payload=paybuf, stream=st)
    for _ in range(warmup):
        run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        run()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    ok = None
    if mode == lphy.MODE_DECHIRP_LORA_DEMODULATE:
        got = paybuf.cpu().numpy().reshape(frames, -1)[:, : nsyms // 2]
        ok = int((got == pay).all(axis=1).sum())
    nbytes = frames * (fs * 8 + per * 2 + 32)
    row = {"shape": name, "sf": sf, "osr": osr, "mode": mode, "frames": frames,
           "symbols_per_frame": nsyms + 2, "ms": round(ms, 5),
           "symbols_per_s": f"{frames * nsyms / (ms * 1e-3):.4g}",
           "hbm_gbps": round(nbytes / (ms * 1e-3) / 1e9, 1),
           "roofline_frac": round(nbytes / (ms * 1e-3) / 8e12, 3),
           "payloads_recovered": "" if ok is None else f"{ok}/{frames}"}
    d.close()
    del iq, out, meta, paybuf, t_in
    torch.cuda.empty_cache()
    return row


def main():
    args = sys.argv[1:]
    only = None
    if "--shapes" in args:
        i = args.index("--shapes")
        only = set(args[i + 1].split(","))
        args = args[:i] + args[i + 2:]
    dst = args[0] if args else "shapes.csv"
    sfs = [int(a) for a in args[1:]] or [7, 8, 9, 10, 11, 12]
    dev = torch.device("cuda", 0)
    rows = []
    for sf in sfs:
        for name, osr, window, mode, nsyms in SHAPES:
            if only is not None and name not in only:
                continue
            if name.startswith("short") and not ((name == "short16" and sf == 7) or (name == "short8" and sf == 8)):
                continue
            r = run_shape(dev, sf, name, osr, window, mode, nsyms)
            rows.append(r)
            print(",".join(str(v) for v in r.values()), flush=True)
    with open(dst, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)


if __name__ == "__main__":
    main()
