#!/usr/bin/env python3
"""Mean kernel time of every format on one workload, each format built once
(the library picked by SPMV_HIP_LIB, so two libraries can be compared by
alternating processes: tools/gpu_job.sh abformats).

    python tools/time_formats.py [--matrix cantlike|rmat] [--formats coo,cmrs] [--rounds 3]

Prints one JSON line per format: median over rounds of the mean of
`--reps` back-to-back launches (HIP events on the launch stream), and the
host check_result verdict of the last launch.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "opencl-spmv-algorithms_amd"), str(REPO)]
import spmv_amd as sa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--matrix", default="cantlike", choices=["cantlike", "rmat"])
    ap.add_argument("--copies", type=int, default=32)
    ap.add_argument("--formats", default="coo,cmrs,ell,sell,csr,hyb")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda:0")
    m = sa.gen_cantlike(0, a.copies) if a.matrix == "cantlike" else sa.gen_rmat()
    b = sa.bytes_alg(m.n_rows, m.n_cols, m.nnz)
    xh = sa.ramp_x(m.n_cols)
    x = torch.from_numpy(xh).to(dev)
    y = torch.empty(m.n_rows, dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream()
    for fmt in a.formats.split(","):
        kw = {"sigma": 1 << 24} if fmt == "sell" and a.matrix == "rmat" else {}
        try:
            dm = sa.to_device(m, fmt, dev, **kw)
        except sa.SpmvError as e:
            print(json.dumps({"fmt": fmt, "na": str(e)}), flush=True)
            continue
        res = []
        for _ in range(a.rounds):
            for _ in range(3):
                dm.run(x, y, s)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            ev[0].record(s)
            for k in range(a.reps):
                dm.run(x, y, s)
                ev[k + 1].record(s)
            torch.cuda.synchronize()
            res.append(float(np.mean([ev[k].elapsed_time(ev[k + 1]) for k in range(a.reps)])))
        bad, _ = sa.check(m, xh, y.cpu().numpy())
        ms = float(np.median(res))
        print(json.dumps({"fmt": fmt, "lib": os.environ.get("SPMV_HIP_LIB", "in-tree"), "ms": round(ms, 5),
                          "GBs_alg": round(b / ms * 1e-6, 1), "frac": round(b / ms * 1e-6 / sa.HBM_PEAK_GBS, 4),
                          "parity_ok": bad == 0, "params": {k: v for k, v in dm.params.items()
                                                            if isinstance(v, (int, float, str))}}), flush=True)
        del dm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
