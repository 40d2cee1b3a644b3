"""Layout/precision check and rough timing of tools/ubench/mfma_dft.hip (an
experiment, not the library): 128-point DFTs on the matrix cores against
numpy's float64 FFT.
  python tools/ubench/mfma_dft.py            (GPU box, after building the .so)"""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent


def main():
    lib = ctypes.CDLL(str(HERE / "mfma_dft.so"))
    lib.mfma_dft128.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    rng = np.random.default_rng(1)
    S = 4096
    n = np.arange(128)
    tones = rng.integers(0, 128, S)
    x = np.exp(2j * np.pi * (tones[:, None] + rng.uniform(-0.3, 0.3, (S, 1))) * n / 128)
    x = x + 0.3 * (rng.standard_normal((S, 128)) + 1j * rng.standard_normal((S, 128)))
    x = (x / np.abs(x).max()).astype(np.complex64)
    ref = np.fft.fft(x.astype(np.complex128), axis=1)
    dev = torch.device("cuda:0")
    xt = torch.from_numpy(x.view(np.float32).copy()).to(dev)
    ot = torch.zeros_like(xt)
    rc = lib.mfma_dft128(xt.data_ptr(), ot.data_ptr(), S, None)
    torch.cuda.synchronize()
    assert rc == 0, rc
    out = ot.cpu().numpy().view(np.complex64).reshape(S, 128)
    err = np.abs(out - ref).max(axis=1)
    l1 = np.abs(x).sum(axis=1)
    print(f"max |X - ref| / L1 = {np.max(err / l1):.3e}  (2^-9 = {2**-9:.3e})")
    agree = (np.argmax(np.abs(out), axis=1) == np.argmax(np.abs(ref), axis=1)).mean()
    print(f"argmax agreement {agree:.4f}")
    # rough timing: many symbols
    S2 = 1 << 22
    xb = torch.randn(S2 * 256, device=dev)
    ob = torch.empty_like(xb)
    for _ in range(3):
        lib.mfma_dft128(xb.data_ptr(), ob.data_ptr(), S2, None)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        lib.mfma_dft128(xb.data_ptr(), ob.data_ptr(), S2, None)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    print(f"{S2} symbols: {ms:.3f} ms, {2 * S2 * 1024 / ms / 1e6:.0f} GB/s in+out")
    return 0 if np.max(err / l1) < 2 ** -8 and agree > 0.999 else 1


if __name__ == "__main__":
    sys.exit(main())
