"""Streaming-ingestion throughput (lphy_hip_demod_stream): the
rx_runner input format (float32 I/Q pairs back to back) read from a file
descriptor in chunks into pinned memory, copied H2D on one stream and
demodulated on another, against the plain pinned H2D copy rate of the same
bytes (the PCIe bound of any host-fed path).  The frames are the bench's
synthetic SF frames (device lora_modulate), written once to a file whose
pages are then cached, so the read is a memory copy.
  python tools/stream_bench.py [sf] [frames] [chunk_frames] [out.json]"""
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

lphy = bench.lphy


def main():
    sf = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # 0: the binding's ~32 MiB chunks
    out = sys.argv[4] if len(sys.argv) > 4 else ""
    dev = torch.device("cuda:0")
    wl = bench.Workload(sf, 125000, frames, 0, dev)
    mode = lphy.MODE_DECHIRP_LORA_DEMODULATE
    host = wl.iq.cpu().numpy()
    nbytes = host.nbytes
    fd_dir = os.environ.get("TMPDIR", "/tmp")
    with tempfile.NamedTemporaryFile(dir=fd_dir, suffix=".iq", delete=False) as f:
        path = f.name
        host.tofile(f)
    try:
        # plain pinned H2D of the same bytes: the PCIe rate
        pinned = torch.from_numpy(host).pin_memory()
        dst = torch.empty_like(wl.iq)
        dst.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            dst.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
        h2d = 3 * nbytes / (time.perf_counter() - t0) / 1e9
        del pinned, dst
        # device-resident demodulation of the same frames (no PCIe)
        resident_ms = wl._event_ms(mode, lphy.F_DECODE, 5, warmup=3)
        # streamed: file -> pinned chunks -> H2D (copy stream) || demod (compute stream)
        res = None
        times = []
        for _ in range(3):
            fd = os.open(path, os.O_RDONLY)
            t0 = time.perf_counter()
            res = wl.dem.demod_stream(fd, wl.fs, mode, lphy.F_DECODE, chunk_frames=chunk, max_frames=frames)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            os.close(fd)
        dt = float(np.median(times))
        syms, pay, meta, tail = res
        ok = int((pay.reshape(frames, -1)[:, : bench.PAYLOAD] == wl.payloads).all(axis=1).sum())
        line = {
            "metric": "streaming ingestion (lphy_hip_demod_stream): IQ GB/s and data symbols/s",
            "sf": sf, "frames": frames, "chunk_frames": chunk, "iq_bytes": nbytes,
            "stream_gbps": nbytes / dt / 1e9, "stream_syms_per_s": frames * bench.DATA_SYMS / dt,
            "stream_s_median_of_3": dt, "pinned_h2d_gbps": h2d,
            "stream_vs_pcie": nbytes / dt / 1e9 / h2d,
            "resident_demod_ms": resident_ms, "resident_gbps": nbytes / (resident_ms * 1e-3) / 1e9,
            "payloads_recovered": ok, "tail_bytes": int(tail),
            "note": "file pages cached after the write: the read is a memory copy; value bound = PCIe",
        }
        print(json.dumps(line), flush=True)
        if out:
            Path(out).write_text(json.dumps(line) + "\n")
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
