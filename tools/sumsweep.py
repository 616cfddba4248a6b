#!/usr/bin/env python3
"""Print a compact table from tools/sweep.py logs: python tools/sumsweep.py LOG..."""
import json
import sys

for path in sys.argv[1:]:
    print(f"== {path}")
    for line in open(path):
        if not line.startswith('{"fmt"'):
            continue
        d = json.loads(line)
        k = {a: b for a, b in d.items() if a not in ("ms", "GBs_alg", "GBs_stored", "frac", "spread")}
        print(f"  {str(k):58s} {d['ms']:.4f} ms  {d['frac'] * 100:5.1f}%  stored {d['GBs_stored']:7.1f} GB/s")
