#!/usr/bin/env python3
"""Per-kernel-name table of averaged PMC counters from tools/pmc_k.sh output."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

acc = defaultdict(lambda: defaultdict(list))
for f in Path(sys.argv[1]).glob("*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in acc.items():
    if "k_" not in k:
        continue
    print(k)
    for n, v in sorted(c.items()):
        print(f"   {n:24s} {sum(v) / len(v):16.4g}  (x{len(v)})")
