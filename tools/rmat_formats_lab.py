#!/usr/bin/env python3
"""rmat_formats_lab — the formats on bench.py's R-MAT layout (1e7 / 1e8,
columns relabelled with first-row ties, rows sorted), each with variant
keyword sets, warm, HIP-graph timed as bench.py's per_format leg; every
output checked against the host rule.  Lab only (A/B of format settings on
configs[3]).

usage: rmat_formats_lab.py 'coo@{}' 'coo@{"hot": 2}' ...
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "opencl-spmv-algorithms_amd"), str(REPO)]
import spmv_amd as sa  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("specs", nargs="+", help="fmt@{json kwargs}")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda:0")
    argv, sys.argv = sys.argv, [sys.argv[0], "--workload", "rmat"]
    bargs = bench.parse()
    sys.argv = argv
    full = bench.rmat_matrix(bargs)
    ptr, col, val = sa.csr_from_coo(full)
    n, z = full.n_rows, full.nnz
    del full
    col, xh, _, _, _ = bench.rmat_layout(bargs, n, ptr, col, val)
    m = sa.Coo(n, n, np.repeat(np.arange(n, dtype=np.int32), np.diff(ptr)), col, val)
    x = torch.from_numpy(xh).to(dev)
    y = torch.empty(n, dtype=torch.float64, device=dev)
    b = sa.bytes_alg(n, n, z)
    for r in range(a.rounds):
        for spec in a.specs:
            fmt, _, kw = spec.partition("@")
            kw = json.loads(kw or "{}")
            dm = sa.to_device(m, fmt, dev, **kw)
            _, k = bench.time_steps(torch, dm, x, y, a.steps, 5)
            km = float(np.mean(k))
            bad, _ = sa.check(m, xh, y.cpu().numpy())
            print(json.dumps({"round": r, "spec": spec, "kernel_ms": round(km, 5),
                              "frac": round(b / (km * 1e-3) * 1e-9 / sa.HBM_PEAK_GBS, 4),
                              "params": {k2: v for k2, v in dm.params.items() if isinstance(v, (int, float, str))},
                              "parity_ok": bad == 0}), flush=True)
            del dm
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
