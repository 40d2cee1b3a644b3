#!/usr/bin/env python3
"""Perf regression gate over two CSVs written by `bench.py --csv` (the
reference's schema run_id,profile,sf,N,pps,cycles_per_symbol plus
hbm_gbps,roofline_frac).  Same rule as the reference's
scripts/compare_perf.py:18-43: a profile regresses when its pps drops or its
cycles per symbol rise; here also when hbm_gbps / roofline_frac drop.
`--tolerance` (relative, default 0) absorbs run-to-run noise.

usage: compare_perf.py <baseline.csv> <new.csv> [--tolerance 0.03]
exit 0: no regression, 2: regression, 1: usage error."""
from __future__ import annotations

import argparse
import csv

HIGHER = ("pps", "hbm_gbps", "roofline_frac")
LOWER = ("cycles_per_symbol",)


def load(path: str) -> dict:
    out = {}
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            out[row["profile"]] = {k: float(row[k]) for k in HIGHER + LOWER if row.get(k) not in (None, "", "N/A")}
    return out


def compare(base: dict, new: dict, tol: float = 0.0) -> list:
    reg = []
    for prof, m in new.items():
        b = base.get(prof)
        if b is None:
            continue
        for k in HIGHER:
            if k in m and k in b and m[k] < b[k] * (1.0 - tol):
                reg.append((prof, k, b[k], m[k]))
        for k in LOWER:
            if k in m and k in b and m[k] > b[k] * (1.0 + tol):
                reg.append((prof, k, b[k], m[k]))
    return reg


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("baseline")
    ap.add_argument("new")
    ap.add_argument("--tolerance", type=float, default=0.0)
    a = ap.parse_args()
    reg = compare(load(a.baseline), load(a.new), a.tolerance)
    if reg:
        print("REGRESSION DETECTED")
        for prof, k, b, n in reg:
            print(f"{prof}: {k} {b:.6g} -> {n:.6g}")
        return 2
    print("No regressions detected.")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
