"""Phase clock split of k_cuframe (build with -DLPHY_PROFILE_PHASES via
variants.py): worker wave 0's cycles in events / round bodies / barriers and
the estimate wave's round-body cycles, per workgroup.  Timing aid only.
  python tools/ubench/cu_phases.py tools/ubench/var_phases.so"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "lora-sdr-lightweight-standalone-library-clean_amd"))
import lphy  # noqa: E402

so = Path(sys.argv[1])
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
lphy.load(so)
lib = lphy._LIB
lib.lphy_hip_phase_cycles.argtypes = [C.c_void_p, C.c_void_p]
d = lphy.Demodulator(7)
dev = torch.device("cuda:0")
rng = np.random.default_rng(1)
pay = rng.integers(0, 256, (nf, 32), dtype=np.uint8)
syms_in = torch.from_numpy(lphy.encode_payloads(pay).view(np.int16).reshape(-1).copy()).to(dev)
fs = 66 * 128
iq = torch.empty(nf * fs * 2, dtype=torch.float32, device=dev)
st = torch.cuda.current_stream().cuda_stream
d.modulate_batch(syms_in, nf, 64, iq, 1.0, 0x12, st)
s = torch.zeros(nf * 64, dtype=torch.int16, device=dev)
m = torch.zeros(nf * 32, dtype=torch.uint8, device=dev)
p = torch.zeros(nf * 32, dtype=torch.uint8, device=dev)
out = (C.c_ulonglong * 4)()
flags = lphy.F_DECODE | lphy.F_STAGE_PROLOGUE | lphy.F_STAGE_SYMBOLS
for mode in (2, 0):
    for _ in range(3):
        d.demod_batch(iq, nf, fs, s, m, mode, flags, payload=p, stream=st)
    torch.cuda.synchronize()
    lib.lphy_hip_phase_cycles(d.ctx, out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    d.demod_batch(iq, nf, fs, s, m, mode, flags, payload=p, stream=st)
    e1.record()
    torch.cuda.synchronize()
    lib.lphy_hip_phase_cycles(d.ctx, out)
    wg = min(256, nf)
    print(f"mode {mode}: {e0.elapsed_time(e1):.3f} ms; per workgroup (Mcycles): worker events {out[0] / wg / 1e6:.3f} "
          f"round bodies {out[1] / wg / 1e6:.3f} barriers {out[2] / wg / 1e6:.3f}; estimate wave round bodies "
          f"{out[3] / wg / 1e6:.3f}")
