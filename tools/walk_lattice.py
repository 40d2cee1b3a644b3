"""Feasibility of a parallel, exact form of lora_modulate's phase walk
(ChirpGenerator.hpp:31-49), measured on the host in
numpy float32 with the reference's rounding order:

* estimate each symbol's start in float64 (the exact sums of its f
  sequence), then correct it by each symbol's own rounding error, measured
  by walking every symbol in parallel from the estimate (`rounds` times);
* the walk of a symbol is determined by its partial sum at the pivot, the
  sample where |phase| is largest: that value lies on the float grid of
  its magnitude (the coarsest grid of the walk), so a window of candidates
  for it, each walked in parallel to the next symbol's pivot, and an exact
  lookup chaining the windows would reproduce the serial walk;
* printed: the distance of the corrected estimate from the true pivot value,
  in grid steps (the window a candidate set must cover), per symbol.
Timing aid / analysis only.   python tools/walk_lattice.py 7 8 9"""
import sys

import numpy as np

PI = np.float32(3.14159265358979323846)


def fseq(sf, v):
    N = 1 << sf
    fmin, fmax = np.float32(-PI), np.float32(PI)
    fstep = np.float32((np.float32(2.0) * PI) / np.float32(N))
    f = np.float32(fmin + np.float32((np.float32(2.0) * PI * np.float32(v)) / np.float32(N)))
    fs = np.empty(N, np.float32)
    for i in range(N):
        f = np.float32(f + fstep)
        if f > fmax:
            f = np.float32(f - np.float32(fmax - fmin))
        fs[i] = f
    return fs


def walk(start, fs):
    out = np.empty(fs.size, np.float32)
    ph = np.float32(start)
    for i, x in enumerate(fs):
        ph = np.float32(ph + x)
        out[i] = ph
    return out


def wrap(ph):
    w = np.floor(float(np.float32(ph / np.float32(2.0 * PI)))) * 2 * float(PI)
    return np.float32(float(ph) - w)


def main():
    rng = np.random.default_rng(1)
    for sf in [int(a) for a in sys.argv[1:]] or [7]:
        for t in range(3):
            syms = [0x12 >> 4 << (sf - 4), (0x12 & 15) << (sf - 4)] + list(rng.integers(0, 1 << sf, 64))
            F = [fseq(sf, v) for v in syms]
            S = [np.cumsum(f.astype(np.float64)) for f in F]
            x = [np.float32(0)]
            tw = []
            for f in F:  # the serial walk (truth)
                p = walk(x[-1], f)
                tw.append(p)
                x.append(wrap(p[-1]))
            est = [0.0]
            for s in S:
                est.append((est[-1] + s[-1]) % (2 * np.pi))
            res = []
            for r in range(3):
                # distance at the pivot, in steps of the pivot's grid
                d = []
                for k in range(1, len(F)):
                    piv = int(np.argmax(np.abs(est[k] + S[k])))
                    true = float(tw[k][piv])
                    grid = float(np.spacing(np.float32(abs(true))))
                    e = est[k] + S[k][piv]
                    dd = (e - true + np.pi) % (2 * np.pi) - np.pi
                    d.append(abs(dd) / grid)
                res.append((max(d), float(np.mean(d))))
                # one correction round: each symbol walked from its estimate
                err = []
                for k, f in enumerate(F):
                    p = walk(np.float32(est[k]), f)
                    err.append(float(p[-1]) - (float(np.float32(est[k])) + S[k][-1]))
                new = [0.0]
                for k in range(len(F)):
                    new.append((new[-1] + S[k][-1] + err[k]) % (2 * np.pi))
                est = new
            print(f"SF{sf} packet {t}: pivot-grid steps max/mean after 0/1/2 corrections: " +
                  ", ".join(f"{a:.1f}/{b:.1f}" for a, b in res), flush=True)


if __name__ == "__main__":
    main()
