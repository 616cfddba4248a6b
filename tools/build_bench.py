#!/usr/bin/env python3
"""Format construction time: host builders vs device builders.

For each matrix and format, times (a) the host path of spmv_amd.to_device
(host CSR/ELL/SELL/CMRS builders + upload of the built arrays) and (b)
spmv_amd.device_build (upload of the raw COO + spmv_dev_* builders), both
from the same in-memory COO, and checks that the two produce the same y.
    python tools/build_bench.py [--matrix rmat|cantlike|both]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "opencl-spmv-algorithms_amd"), str(REPO)]
import spmv_amd as sa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--matrix", default="both", choices=["rmat", "cantlike", "both"])
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda:0")
    mats = []
    if a.matrix in ("cantlike", "both"):
        mats.append(("cantlike x32", sa.gen_cantlike(0, 32)))
    if a.matrix in ("rmat", "both"):
        mats.append(("rmat 1e7/1e8", sa.gen_rmat()))
    for name, m in mats:
        x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, m.n_cols)).to(dev)
        for fmt in ("csr", "sell", "cmrs", "ell"):
            if fmt == "ell" and name.startswith("rmat"):
                continue
            kw = dict(xwin=False)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dh = sa.to_device(m, fmt, dev, **kw) if fmt != "csr" else sa.to_device(m, fmt, dev, variant=3, **kw)
            torch.cuda.synchronize()
            t_host = time.perf_counter() - t0
            y1 = torch.empty(m.n_rows, dtype=torch.float64, device=dev)
            dh.run(x, y1)
            del dh
            torch.cuda.empty_cache()
            t0 = time.perf_counter()
            dd = sa.device_build(m, fmt, dev, **kw)
            torch.cuda.synchronize()
            t_dev = time.perf_counter() - t0
            y2 = torch.empty(m.n_rows, dtype=torch.float64, device=dev)
            dd.run(x, y2)
            torch.cuda.synchronize()
            same = bool(torch.equal(y1.view(torch.int64), y2.view(torch.int64)))
            del dd
            torch.cuda.empty_cache()
            print(json.dumps({"matrix": name, "format": fmt, "nnz": m.nnz, "host_build_upload_s": round(t_host, 3),
                              "device_build_s": round(t_dev, 3), "speedup": round(t_host / t_dev, 2),
                              "same_y_bits": same}), flush=True)


if __name__ == "__main__":
    main()
