#!/usr/bin/env python3
"""R-MAT x-gather experiments (GPU box): tools/rmat_exp.hip variants.

    python tools/rmat_exp.py [--reps 20]
Prints one JSON line per variant: R (stage rounds), NT, mode (0 plain
gathers, 1 hot-column table of H columns, 2 stream-only bound), ms.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import subprocess
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "opencl-spmv-algorithms_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="300,310,600,610,312,612,302,312")
    ap.add_argument("--hot", default="65536,262144,524288")
    a = ap.parse_args()
    import torch  # before the tool's .so: torch's HIP runtime must be the one loaded

    so = REPO / "tools" / "rmat_exp.so"
    if not so.exists():
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", str(REPO / "tools" / "rmat_exp.hip"),
                        "-o", str(so)], check=True)
    lib = ctypes.CDLL(str(so))
    lib.rmat_exp_run.restype = ctypes.c_int
    lib.rmat_exp_ws.restype = ctypes.c_int64

    import spmv_amd as sa

    m = sa.gen_rmat()
    ptr, col, val = sa.csr_from_coo(m)
    n, M, nnz = m.n_rows, m.n_cols, m.nnz
    del m
    cnt = np.bincount(col, minlength=M)
    order = np.argsort(-cnt, kind="stable").astype(np.int32)
    dev = torch.device("cuda:0")
    d_ptr = torch.from_numpy(ptr).to(dev)
    d_col = torch.from_numpy(col).to(dev)
    d_val = torch.from_numpy(val).to(dev)
    x = torch.from_numpy(np.arange(M, dtype=np.float64)).to(dev)
    y = torch.empty(n, dtype=torch.float64, device=dev)
    ws = lib.rmat_exp_ws(2, nnz)
    own = torch.empty(ws + 1, dtype=torch.int32, device=dev)
    crow = torch.empty(ws, dtype=torch.int32, device=dev)
    cval = torch.empty(ws, dtype=torch.float64, device=dev)
    xh = torch.zeros(1 << 20, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    P = ctypes.c_void_p

    def launch(variant, dcol, hot, H):
        rc = lib.rmat_exp_run(variant, ctypes.c_int64(n), ctypes.c_int64(nnz), ctypes.c_int64(M), P(d_ptr.data_ptr()),
                              P(dcol.data_ptr()), P(d_val.data_ptr()), P(x.data_ptr()),
                              P(hot.data_ptr() if hot is not None else 0), ctypes.c_int64(H), P(xh.data_ptr()),
                              P(y.data_ptr()), P(own.data_ptr()), P(crow.data_ptr()), P(cval.data_ptr()), P(st))
        assert rc == 0, (variant, rc)

    def timeit(variant, dcol, hot, H):
        for _ in range(3):
            launch(variant, dcol, hot, H)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        for e0, e1 in ev:
            e0.record()
            launch(variant, dcol, hot, H)
            e1.record()
        torch.cuda.synchronize()
        return float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))

    b_alg = 12 * nnz + 4 * (n + 1) + 16 * n
    launch(300, d_col, None, 0)
    torch.cuda.synchronize()
    y_ref = y.clone()
    cols = {0: (d_col, None)}
    for H in [int(h) for h in a.hot.split(",") if h]:
        rank = np.full(M, -1, np.int64)
        rank[order[:H]] = np.arange(H)
        c2 = np.where(rank[col] >= 0, M + rank[col], col).astype(np.int32)
        cols[H] = (torch.from_numpy(c2).to(dev), torch.from_numpy(order[:H].copy()).to(dev))
        print(json.dumps({"H": H, "hot_mass": float(cnt[order[:H]].sum() / nnz)}), flush=True)
    for v in [int(s) for s in a.variants.split(",")]:
        for H, (dcol, hot) in cols.items():
            if (v % 10 == 1) != (H > 0):
                continue
            ms = timeit(v, dcol, hot, H)
            same = bool(torch.equal(y, y_ref)) if v % 10 != 2 else None
            print(json.dumps({"R": v // 100, "nt": (v // 10) % 10, "mode": v % 10, "H": H, "ms": round(ms, 4),
                              "GBs_alg": round(b_alg / ms * 1e-6, 1), "bit_equal": same}), flush=True)


if __name__ == "__main__":
    main()
