"""Time k_demod<SF> variants built with phases stubbed out (sincos / FFT /
global loads) to see where the kernel's time goes.  Builds one .so per
variant from the real source with -DLPHY_ABLATE_*; timing only."""
import ctypes, os, subprocess, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "lora-sdr-lightweight-standalone-library-clean_amd")
sys.path.insert(0, PKG)
import lphy
import torch
sf = int(sys.argv[1]) if len(sys.argv) > 1 else 7
variants = {"full": "", "no_sincos": "-DLPHY_ABLATE_SINCOS", "no_fft": "-DLPHY_ABLATE_FFT",
            "no_load": "-DLPHY_ABLATE_LOAD", "no_sincos_fft": "-DLPHY_ABLATE_SINCOS -DLPHY_ABLATE_FFT"}
frames = 65536 if sf == 7 else 8192
N = 1 << sf; fs = 66 * N
dev = torch.device("cuda:0")
for name, flags in variants.items():
    so = os.path.join(ROOT, "tools", "ubench", f"ablate_{name}.so")
    if not os.path.exists(so):
        subprocess.run(f"/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -shared {flags} -I{ROOT}/include -I{PKG}/csrc -o {so} {PKG}/csrc/lphy_hip.hip", shell=True, check=True)
    lib = lphy.use(__import__("pathlib").Path(so))
    d = lphy.Demodulator(sf)
    rng = np.random.default_rng(1)
    pay = rng.integers(0, 256, (frames, 32), dtype=np.uint8)
    syms_in = torch.from_numpy(lphy.encode_payloads(pay).view(np.int16).reshape(-1).copy()).to(dev)
    iq = torch.empty(frames * fs * 2, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    d.modulate_batch(syms_in, frames, 64, iq, 1.0, 0x12, st)
    out = torch.zeros(frames * 64, dtype=torch.int16, device=dev)
    meta = torch.zeros(frames * 32, dtype=torch.uint8, device=dev)
    pl = torch.zeros(frames * 32, dtype=torch.uint8, device=dev)
    d.demod_batch(iq, frames, fs, out, meta, 2, lphy.F_DECODE, payload=pl, stream=st)
    ts = []
    for rep in range(6):
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record(); d.demod_batch(iq, frames, fs, out, meta, 2, lphy.F_DECODE | lphy.F_STAGE_SYMBOLS, payload=pl, stream=st); b.record()
        torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
    ok = (pl.cpu().numpy().reshape(frames, 32) == pay).all(axis=1).mean()
    print(f"SF{sf} {name:14s} symbols kernel {np.median(ts):.3f} ms  (payload ok frac {ok:.3f})", flush=True)
    d.close(); del iq, out, meta, pl
    torch.cuda.empty_cache()
