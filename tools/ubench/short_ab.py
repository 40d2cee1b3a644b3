"""A/B of one-SF library variants on the frames shorter than a wave unit
(tools/shapes_perf.py's short16 / short8 rows), e.g. the f16 matrix-core
symbol tiles of k_frames against -DLPHY_NO_MFMA.  Timing aid only.
  python tools/ubench/short_ab.py <sf> <variant> ...   (GPU box; var_<variant>.so)"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tools"))
import shapes_perf  # noqa: E402

lphy = shapes_perf.lphy
sf = int(sys.argv[1])
nsyms = 16 if sf == 7 else 8
dev = torch.device("cuda", 0)
for rnd in range(2):
    for v in sys.argv[2:]:
        lphy.use(Path(__file__).resolve().parent / f"var_{v}.so")
        r = shapes_perf.run_shape(dev, sf, f"short{nsyms}", 1, lphy.WINDOW_NONE,
                                  lphy.MODE_DECHIRP_LORA_DEMODULATE, nsyms)
        print(v, rnd, r["ms"], r["symbols_per_s"], r["roofline_frac"], r["payloads_recovered"], flush=True)
