#!/usr/bin/env python3
"""Median / min duration (us) and dispatch count per kernel name in a
rocprofv3 kernel-trace CSV (template arguments kept, arguments dropped).
    python tools/trace_medians.py DIR_OR_CSV [substring]"""
from __future__ import annotations

import csv
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np


def main():
    p = Path(sys.argv[1])
    if p.is_dir():
        p = sorted(p.rglob("*kernel_trace.csv"))[-1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    by = defaultdict(list)
    for r in csv.DictReader(open(p, newline="")):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        if sub in name:
            by[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    for name, d in sorted(by.items(), key=lambda kv: np.median(kv[1])):
        print(f"{np.median(d):9.2f} us  min {min(d):8.2f}  n={len(d):5d}  {name}")


if __name__ == "__main__":
    main()
