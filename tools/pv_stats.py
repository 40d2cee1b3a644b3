"""Parseval / re-run statistics of the bench's synthetic workload (test
build counters): how many symbol units the Parseval certificate proves and
how many symbols k_post re-runs, per SF.  GPU box:
    python tools/pv_stats.py [frames]"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "lora-sdr-lightweight-standalone-library-clean_amd"))
import lphy  # noqa: E402

PAYLOAD, DATA_SYMS = 32, 64
TOTAL = DATA_SYMS + 2


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    dev = torch.device("cuda:0")
    for sf in (9, 10, 11, 12):
        N = 1 << sf
        d = lphy.Demodulator(sf, 125000, 1, lphy.WINDOW_NONE, device=0, test_build=True)
        rng = np.random.default_rng(0x5EED + sf)
        pay = rng.integers(0, 256, (frames, PAYLOAD), dtype=np.uint8)
        syms = lphy.encode_payloads(pay)
        t_in = torch.from_numpy(syms.view(np.int16).reshape(-1).copy()).to(dev)
        iq = torch.empty(frames * TOTAL * N * 2, dtype=torch.float32, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        d.modulate_batch(t_in, frames, DATA_SYMS, iq, 1.0, 0x12, st)
        out = torch.zeros(frames * DATA_SYMS, dtype=torch.int16, device=dev)
        meta = torch.zeros(frames * 32, dtype=torch.uint8, device=dev)
        pay_out = torch.zeros(frames * PAYLOAD, dtype=torch.uint8, device=dev)
        d.parseval_count(reset=True)
        d.recheck_count(reset=True)
        d.demod_batch(iq, frames, TOTAL * N, out, meta, 2, lphy.F_DECODE, payload=pay_out, stream=st)
        torch.cuda.synchronize()
        pv, rc = d.parseval_count(reset=True), d.recheck_count(reset=True)
        ok = bool((out.cpu().numpy().view(np.uint16).reshape(frames, -1) == syms).all())
        print(f"sf{sf}: frames {frames} symbols {frames * TOTAL} parseval {pv} ({pv / (frames * TOTAL):.4f}) "
              f"rechecked {rc} symbols_exact {ok}", flush=True)


if __name__ == "__main__":
    main()
