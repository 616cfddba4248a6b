#!/usr/bin/env python3
"""inproc_noise — where bench.py's in-process cold figure varies (lab only).

For one format on one cant-like matrix: the in-process cold SpMV time
(bench.cold_fn_ms: graph of K x (read flush + SpMV) minus graph of K
flushes) measured R times on the SAME device arrays, then R times with the
matrix re-uploaded (new allocations, other physical pages) before each
measurement.  Prints the spread of each series (us).
    python tools/inproc_noise.py [--format sell] [--reps 6] [--steps 100]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "opencl-spmv-algorithms_amd"), str(REPO), str(REPO / "tools")]
import spmv_amd as sa  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--format", default="sell")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--steps", type=int, default=100)
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda:0")
    m = sa.gen_cantlike(0, 1)
    x = torch.from_numpy(sa.ramp_x(m.n_cols)).to(dev)
    y = torch.empty(m.n_rows, dtype=torch.float64, device=dev)
    out = {"format": a.format, "steps": a.steps}
    dm = sa.to_device(m, a.format, dev)
    same = [bench.cold_fn_ms(torch, lambda: dm.run(x, y), a.steps) * 1e3 for _ in range(a.reps)]
    del dm
    fresh = []
    keep = []  # hold earlier copies so each upload lands on new pages
    for _ in range(a.reps):
        d2 = sa.to_device(m, a.format, dev)
        keep.append(d2)
        fresh.append(bench.cold_fn_ms(torch, lambda: d2.run(x, y), a.steps) * 1e3)
    for k, v in (("same_arrays_us", same), ("fresh_arrays_us", fresh)):
        out[k] = [round(t, 3) for t in v]
        out[k.replace("_us", "_median")] = round(float(np.median(v)), 3)
        out[k.replace("_us", "_range")] = round(float(max(v) - min(v)), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
