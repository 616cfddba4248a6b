#!/usr/bin/env python3
"""R-MAT column-split experiment (GPU box; diagnostic, not product).

Question: does splitting the R-MAT's columns into P groups of whole 128-B x
lines, and running the entries group after group, let each XCD's 4 MiB L2
hold the x lines the in-flight tiles gather from, so that the cold-column
gathers stop filling a line each (profiles/traffic_rmat.json: 3.46x
bytes_alg)?  The split matrix is the library's column-grouped CSR (format
"csrg": one pair per (row, column group) with entries, group-major; the
tiled kernel over the pairs, then the per-row sum of the pair sums).

    python tools/rmat_split_exp.py [--parts 8,16,32,64] [--reps 20]
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


def time_run(torch, dm, x, y, reps, cold, sa):
    st = torch.cuda.current_stream()
    ts = []
    for r in range(reps + 2):
        if cold:
            sa.flush_cache(st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        dm.run(x, y)
        e1.record(st)
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", default="8,16,32,64")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--sorts", default="",
                    help="also time the product path with each row's entries reordered: col (ascending "
                         "column) or hot (ascending hot-table id: cold columns by id, then hot ones by rank)")
    ap.add_argument("--colmaps", default="",
                    help="also time the product kernel (no hot table) with the columns replaced: "
                         "zero, mod<k>, rand<k> (uniform over k columns), comma-separated")
    a = ap.parse_args()
    import torch
    import spmv_amd as sa

    dev = torch.device("cuda:0")
    t = time.time()
    m = sa.gen_rmat()
    xh = np.random.default_rng(7).uniform(-1, 1, m.n_cols)
    x = torch.from_numpy(xh).to(dev)
    b = sa.bytes_alg(m.n_rows, m.n_cols, m.nnz)
    print(json.dumps({"setup_s": round(time.time() - t, 1)}), flush=True)
    # baseline: the product path (tiled CSR + hot table, library rule)
    dm = sa.to_device(m, "csr", dev)
    y = torch.empty(m.n_rows, dtype=torch.float64, device=dev)
    for cold in (0, 1):
        ms = time_run(torch, dm, x, y, a.reps, cold, sa)
        print(json.dumps({"variant": "product", "params": dm.params, "cold": cold, "ms": round(ms, 4),
                          "GBs": round(b / ms * 1e-6, 1)}), flush=True)
    y_ref = y.cpu().numpy()
    import hashlib
    print(json.dumps({"product_y_sha1": hashlib.sha1(y_ref.tobytes()).hexdigest()}), flush=True)
    del dm
    torch.cuda.empty_cache()
    # within-row entry orders (same rows, same tiles; sums reordered inside rows)
    for so in [c for c in a.sorts.split(",") if c]:
        if so == "col":
            key = m.col.astype(np.int64)
        else:
            _, _, col_hot = sa.hot_columns(m.n_cols, m.col, 0)
            key = col_hot.astype(np.int64)
        o = np.lexsort((key, m.row))
        m2 = sa.Coo(m.n_rows, m.n_cols, m.row[o], m.col[o], m.val[o], False, so)
        del o, key
        dm = sa.to_device(m2, "csr", dev)
        for cold in (0, 1):
            ms = time_run(torch, dm, x, y, a.reps, cold, sa)
            print(json.dumps({"variant": "sorted", "order": so, "cold": cold, "ms": round(ms, 4),
                              "GBs": round(b / ms * 1e-6, 1)}), flush=True)
        bad, first = sa.check(m2, xh, y.cpu().numpy())
        print(json.dumps({"variant": "sorted", "order": so, "parity_bad_rows": int(bad)}), flush=True)
        del dm, m2
        torch.cuda.empty_cache()
    # gather-cost probes: same rows, same tiles, columns replaced
    for cm in [c for c in a.colmaps.split(",") if c]:
        if cm == "zero":
            c2 = np.zeros_like(m.col)
        elif cm.startswith("mod"):
            c2 = (np.arange(m.nnz, dtype=np.int64) * 7919 % int(cm[3:])).astype(np.int32)
        else:
            c2 = np.random.default_rng(3).integers(0, int(cm[4:]), m.nnz).astype(np.int32)
        m2 = sa.Coo(m.n_rows, m.n_cols, m.row, c2, m.val, False, cm)
        dm = sa.to_device(m2, "csr", dev, variant=4, hot=0)
        for cold in (0, 1):
            ms = time_run(torch, dm, x, y, a.reps, cold, sa)
            print(json.dumps({"variant": "colmap", "map": cm, "cold": cold, "ms": round(ms, 4),
                              "GBs": round(b / ms * 1e-6, 1)}), flush=True)
        del dm, m2, c2
        torch.cuda.empty_cache()
    for P in [int(p) for p in a.parts.split(",") if p]:
        t = time.time()
        dm = sa.to_device(m, "csrg", dev, groups=P)
        setup = time.time() - t
        yg = torch.empty(m.n_rows, dtype=torch.float64, device=dev)
        res = {}
        for cold in (0, 1):
            res["cold" if cold else "warm"] = round(time_run(torch, dm, x, yg, a.reps, cold, sa), 4)
        yy = yg.cpu().numpy()
        err = float(np.max(np.abs(yy - y_ref) / np.maximum(np.abs(y_ref), 1e-300)))
        print(json.dumps({"variant": "csrg", "groups": P, "pairs": dm.params["n_pairs"], "ms": res,
                          "GBs_warm": round(b / res["warm"] * 1e-6, 1), "GBs_cold": round(b / res["cold"] * 1e-6, 1),
                          "max_rel_vs_product": err, "setup_s": round(setup, 1)}), flush=True)
        del dm, yg
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
