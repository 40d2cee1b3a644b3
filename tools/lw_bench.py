"""Throughput of the LoRaWAN batch kernels (csrc/lphy_lorawan.hip) and the
codes kernels on one MI355X: frames/s for compute_mic (MIC append) and for
parse_frame's checks over decoded rows, HIP-event timed on one stream.
usage: python tools/lw_bench.py [frames] [row_bytes]"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "lora-sdr-lightweight-standalone-library-clean_amd"))
import lphy  # noqa: E402


def timed(fn, reps=20):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps / 1e3


def main():
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(1)
    rows = torch.from_numpy(rng.integers(0, 256, nf * L, dtype=np.uint8)).to(dev)
    keys = torch.from_numpy(rng.integers(0, 256, 16 * 1024, dtype=np.uint8)).to(dev)
    d = np.zeros(nf, lphy.LORAWAN_DESC_DTYPE)
    d["offset"] = np.arange(nf) * L
    d["len"] = L - 4
    d["devaddr"] = rng.integers(0, 2**32, nf, dtype=np.uint64).astype(np.uint32)
    d["fcnt"] = np.arange(nf)
    d["key"] = rng.integers(0, 1024, nf)
    d["uplink"] = 1
    desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    st = torch.cuda.current_stream().cuda_stream
    t_mic = timed(lambda: lphy.lorawan_mic_batch(rows, desc, keys, None, lphy.LW_APPEND, stream=st))
    out = torch.empty(nf * 32, dtype=torch.uint8, device=dev)
    kidx = torch.from_numpy(d["key"].astype(np.int32)).to(dev)
    t_parse = timed(lambda: lphy.lorawan_parse_batch(rows, nf, L, L, keys, out, key_index=kidx, stream=st))
    blocks = (L - 4 + 16 + 15) // 16 + 1  # CMAC blocks + the subkey block
    res = {"frames": nf, "row_bytes": L, "mic_ms": t_mic * 1e3, "mic_frames_per_s": nf / t_mic,
           "parse_ms": t_parse * 1e3, "parse_frames_per_s": nf / t_parse,
           "aes_blocks_per_s": nf * blocks / t_mic}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
