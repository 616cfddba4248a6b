#!/usr/bin/env python3
"""VGPR / occupancy per kernel from hipcc -Rpass-analysis=kernel-resource-usage
(stdin); optional substring filter.  usage:
  hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/vgprs.py sell_small"""
import re
import subprocess
import sys

sub = sys.argv[1] if len(sys.argv) > 1 else ""
name = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        try:
            name = subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        rows[name] = {}
        continue
    for key in ("VGPRs", "AGPRs", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]", "ScratchSize [bytes/lane]"):
        m = re.search(re.escape(key) + r": (\d+)", line)
        if m and name:
            rows[name][key] = int(m.group(1))
for n, r in rows.items():
    if sub in n:
        short = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        print(f"{r.get('VGPRs', '?'):>4} vgpr  occ {r.get('Occupancy [waves/SIMD]', '?')}  "
              f"scratch {r.get('ScratchSize [bytes/lane]', '?')}  {short}")
