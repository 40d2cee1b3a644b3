"""How far an exact-arithmetic estimate of each symbol's start phase drifts
from lora_modulate's float phase walk (ChirpGenerator.hpp:31-49): the float
chain in numpy float32, one rounding per step in the reference's order,
against the same recurrence in float64; prints the drift in float32 ulps
(bit-pattern distance) of the symbol starts.  DESIGN §4.7.
    python tools/walk_drift.py 7 9"""
import numpy as np, sys
PI = np.float32(3.14159265358979323846)
def sim(sf, syms, osr=1, bws=np.float32(1.0)):
    N = 1 << sf
    fmin = np.float32(-PI * bws / np.float32(osr)); fmax = np.float32(PI * bws / np.float32(osr))
    fstep = np.float32((np.float32(2.0) * PI * bws) / np.float32(N * osr * osr))
    ph = np.float32(0.0); phd = 0.0
    p0f = []; p0d = []
    for v in syms:
        f0 = np.float32((np.float32(2.0) * PI * np.float32(v) * bws) / (np.float32(N) * np.float32(osr)))
        # float f sequence (exact) - same for both chains
        f = np.float32(fmin + f0)
        fs = np.empty(N, np.float32)
        for i in range(N):
            f = np.float32(f + fstep)
            if f > fmax: f = np.float32(f - np.float32(fmax - fmin))
            fs[i] = f
        p0f.append(ph); p0d.append(phd)
        for i in range(N):
            ph = np.float32(ph + fs[i])
        phd = phd + float(np.sum(fs.astype(np.float64)))
        w = np.floor(float(np.float32(ph / np.float32(2.0 * PI)))) * 2 * float(PI)
        ph = np.float32(float(ph) - w)
        wd = np.floor(phd / (2 * float(PI))) * 2 * float(PI)
        phd = phd - wd
    p0f = np.array(p0f, np.float32); 
    dev = [int(np.float32(a).view(np.int32)) - int(np.float32(b).view(np.int32)) for a, b in zip(p0f, np.array(p0d, np.float32))]
    return dev
rng = np.random.default_rng(1)
for sf in [int(a) for a in sys.argv[1:]]:
    worst = 0
    for t in range(3):
        syms = [0x12 >> 4 << (sf-4), (0x12 & 15) << (sf-4)] + list(rng.integers(0, 1 << sf, 64))
        dev = sim(sf, syms)
        worst = max(worst, max(abs(d) for d in dev))
        print(sf, t, 'max |dev| ulps', max(abs(d) for d in dev), 'last', dev[-5:])
