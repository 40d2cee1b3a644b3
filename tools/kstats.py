#!/usr/bin/env python3
"""Per-kernel VGPR / spill / LDS summary of a -save-temps gfx950 assembly file."""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in s.split("- .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if pat not in name:
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, None])[1]
    print(f"{name[:64]:64s} vgpr {g('vgpr_count'):>4} spill {g('vgpr_spill_count'):>3} "
          f"lds {g('group_segment_fixed_size'):>6} sgpr {g('sgpr_count')}")
