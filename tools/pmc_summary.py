"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) into profiles/pmc_<tag>.json:
per kernel, HBM bytes per launch = FETCH_SIZE x 2 (gfx950 reports half of a
wide streaming read, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both in KiB
in rocprofv3's output; plus the SQ counters when those passes ran.
Usage: python tools/pmc_summary.py <pmc dir> <tag> <frames> <sf> [dest dir] [mode]
(mode: the lphy mode the passes ran, default 2 = the bench's)"""
import csv
import json
import re
import sys
import time
from collections import defaultdict
from pathlib import Path


def norm(name: str) -> str:
    m = re.search(r"(k_\w+)<(\d+)", name)
    return f"{m.group(1)}<{m.group(2)}>" if m else name.split("(")[0].strip()


def load(d: Path):
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(lambda: defaultdict(int))
    for f in d.glob("*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = norm(r["Kernel_Name"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k][r["Counter_Name"]] += 1
    return acc, n


def main():
    d, tag, frames, sf = Path(sys.argv[1]), sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    acc, n = load(d)
    mode = int(sys.argv[6]) if len(sys.argv) > 6 else 2
    # "written": bench.py's measured_traffic takes the newest summary of a
    # configuration by this stamp
    out = {"tag": tag, "frames": frames, "sf": sf, "mode": mode, "source": str(d),
           "written": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()), "kernels": {}}
    for k, c in acc.items():
        if not k.startswith("k_"):
            continue
        e = {name: c[name] / n[k][name] for name in c}
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["fetch_bytes_corrected"] = e["FETCH_SIZE"] * 1024 * 2
            e["write_bytes"] = e["WRITE_SIZE"] * 1024
            e["hbm_bytes_per_launch"] = e["fetch_bytes_corrected"] + e["write_bytes"]
        e["launches"] = max(n[k].values())
        out["kernels"][k] = e
    root = Path(__file__).resolve().parents[1]
    dest = Path(sys.argv[5]) if len(sys.argv) > 5 else root / "profiles"
    dest.mkdir(parents=True, exist_ok=True)
    (dest / f"pmc_{tag}.json").write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
