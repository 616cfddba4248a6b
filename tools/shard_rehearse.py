#!/usr/bin/env python3
"""Strong-scaling rehearsal of the row-sharded R-MAT on ONE GPU.

bench.py --workload rmat --gpus G cuts the 1e7 x 1e7 / 1e8-entry R-MAT
(BASELINE.json configs[3], the north-star scaling matrix) into G
nnz-balanced row shards (spmv_partition_rows, aligned to 1024 rows), one
per GPU, x replicated, and reports bytes_alg(whole) / max over ranks of the
step time.  Here every shard of every G is built and timed ALONE on cuda:0
(HIP events over back-to-back launches, as bench.py), so

    aggregate_GBs(G) = bytes_alg(whole matrix) / max_g t_g

is the SpMV-only figure a G-GPU run reports when every GPU runs its shard
concurrently (the GPUs share nothing on the SpMV path).  Back-to-back
launches keep part of a small shard and of x in the 256 MiB Infinity Cache,
on every GPU alike, so the figure is labelled warm.  --flush also times
every shard cold (a 512 MiB flush before each SpMV, bench.cold_step_ms:
a graph of flush + SpMV minus a graph of flushes) and reports the cold
aggregate beside the warm one.  The y all-gather over
RCCL is not included (bench.py times it separately).  A rehearsal on one
card, not a substitute for the driver's 8-GPU run.

    python tools/shard_rehearse.py [--gpus 1,2,4,8] [--format csr] [--reps 20]
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "opencl-spmv-algorithms_amd"), str(REPO)]
import spmv_amd as sa  # noqa: E402


def time_shard(torch, dm, x, y, reps, graph=False):
    """Mean ms per SpMV over back-to-back launches; graph=True captures the
    `reps` SpMVs (3-4 kernels each) into one HIP graph and times its replay
    as one span (as bench.py times its steps)."""
    s = torch.cuda.current_stream()
    for _ in range(3):
        dm.run(x, y, s)
    if graph:
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                dm.run(x, y)
        torch.cuda.synchronize()
        g.replay()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(s)
        g.replay()
        b.record(s)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(s)
    for k in range(reps):
        dm.run(x, y, s)
        ev[k + 1].record(s)
    torch.cuda.synchronize()
    return float(np.mean([ev[k].elapsed_time(ev[k + 1]) for k in range(reps)]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--format", default="csr")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--row-weights", default="2", help="spmv_partition_rows_weighted weights to try")
    ap.add_argument("--hot", default="-1", help="CSR hot-column table(s), comma-separated: -1 library rule, 0 off, H")
    ap.add_argument("--graph", action="store_true", help="time the reps as one captured HIP graph replay (bench.py's timing)")
    ap.add_argument("--env", action="append", default=[],
                    help="KEY=v1,v2: library knobs timed interleaved on every shard (several: cartesian product)")
    ap.add_argument("--rounds", type=int, default=1, help="interleaved rounds per shard (median of rounds)")
    ap.add_argument("--flush", action="store_true", help="also time every shard cold (512 MiB flush first)")
    ap.add_argument("--damp", type=float, default=0.5,
                    help="each re-cut moves the cut points this fraction of the way (bench.py's RMAT_DAMP)")
    ap.add_argument("--sort-rows", action="store_true",
                    help="after the relabel: every row's entries by increasing column (spmv_csr_sort_rows)")
    ap.add_argument("--ties", default="first", choices=["id", "first"],
                    help="relabel ties: column id, or first appearance (the first row using the column)")
    ap.add_argument("--relabel", action="store_true",
                    help="columns relabelled by decreasing degree (spmv_column_relabel), x permuted to match; "
                         "no hot-column table")
    ap.add_argument("--calibrate", type=int, default=0,
                    help="profile-guided re-cuts after the weighted cut (spmv_partition_rows_calibrated, "
                         "from the first --env config's shard times), each timed again")
    a = ap.parse_args()
    keys, vals = [], []
    for e in a.env:
        k, v = e.split("=", 1)
        keys.append(k)
        vals.append(v.split(","))
    envs = [dict(zip(keys, c)) for c in itertools.product(*vals)] or [{}]
    import torch

    dev = torch.device("cuda:0")
    full = sa.gen_rmat()
    ptr, col, val = sa.csr_from_coo(full)
    n, z = full.n_rows, full.nnz
    del full
    xh = sa.ramp_x(n)
    if a.relabel:  # the replicated x arrives in the relabelled layout (outside the timed step)
        order, _, col = sa.column_relabel(n, col, a.ties)
        xh = np.ascontiguousarray(xh[order])
        a.hot = "0"
    if a.sort_rows:
        sa.csr_sort_rows(n, ptr, col, val)
    x = torch.from_numpy(xh).to(dev)
    b_total = sa.bytes_alg(n, n, z)
    base = None
    for G, w, hot in [(int(g), float(w), int(h)) for h in a.hot.split(",") for w in a.row_weights.split(",")
                      for g in a.gpus.split(",")]:
        kw = {"hot": None if hot < 0 else hot} if a.format in ("csr", "coo", "cmrs", "sell") else {}
        if a.format == "sell":
            kw["sigma"] = 1 << 24  # whole-matrix sort on R-MAT (bench.py's R-MAT default)
        bounds = sa.partition_rows(n, ptr, G, align=1024, row_weight=w)
        for cpass in range(a.calibrate + 1):
            if cpass:  # re-cut on the cold shard times with --flush (bench.py's rule), else warm
                cost = cold if a.flush and cold and min(cold) > 0 else times[0]
                nb = sa.partition_rows_calibrated(n, ptr, G, bounds, cost, align=1024, row_weight=w)
                bounds = sa.partition_rows_damped(n, bounds, nb, a.damp) if a.damp < 1 else nb
            times, base, cold = run_split(a, torch, sa, dev, ptr, col, val, n, x, xh, b_total, envs, kw, G, w,
                                          hot, bounds, cpass, base)


def run_split(a, torch, sa, dev, ptr, col, val, n, x, xh, b_total, envs, kw, G, w, hot, bounds, cpass, base):
    times, nnzs, params, cold = [[] for _ in envs], [], None, []
    for r in range(G):
        lo, hi = int(bounds[r]), int(bounds[r + 1])
        lptr = ptr[lo:hi + 1] - ptr[lo]
        loc = sa.Coo(hi - lo, n, np.repeat(np.arange(hi - lo, dtype=np.int32), np.diff(lptr)),
                     col[ptr[lo]:ptr[hi]], val[ptr[lo]:ptr[hi]])
        dm = sa.to_device(loc, a.format, dev, **kw)
        params = params or {k: v for k, v in dm.params.items() if isinstance(v, (int, float, str))}
        y = torch.empty(max(loc.n_rows, 1), dtype=torch.float64, device=dev)
        per = [[] for _ in envs]
        for _ in range(a.rounds):
            for i, env in enumerate(envs):
                os.environ.update(env)
                per[i].append(time_shard(torch, dm, x, y, a.reps, a.graph))
                bad, first = sa.check(loc, xh, y[:loc.n_rows].cpu().numpy())
                if bad:
                    raise SystemExit(f"G={G} shard {r} env {env}: parity failure at row {first}")
        for i in range(len(envs)):
            times[i].append(float(np.median(per[i])))
        if a.flush:
            from bench import cold_step_ms

            cold.append(cold_step_ms(torch, dm, x, y, a.reps))
        nnzs.append(loc.nnz)
        del dm, y, loc
        torch.cuda.empty_cache()
    for i, env in enumerate(envs):
        tmax = max(times[i])
        agg = b_total / (tmax * 1e-3) * 1e-9
        base = base or agg
        extra = {}
        if cold:
            extra = {"shard_ms_cold": [round(t, 4) for t in cold], "max_ms_cold": round(max(cold), 4),
                     "aggregate_GBs_cold": round(b_total / (max(cold) * 1e-3) * 1e-9, 1)}
        print(json.dumps({"workload": "rmat 1e7/1e8", "format": a.format, "relabel": a.relabel, "ties": a.ties, "sort_rows": a.sort_rows, "env": env,
                          "params_shard0": params,
                          "gpus": G, "row_weight": w, "hot": hot, "graph": a.graph, "calibration_pass": cpass,
                          "shard_rows": np.diff(bounds).tolist(), "shard_nnz": nnzs,
                          "shard_ms": [round(t, 4) for t in times[i]], "max_ms": round(tmax, 4),
                          "aggregate_GBs_warm": round(agg, 1), "speedup_vs_first": round(agg / base, 2), **extra}),
              flush=True)
    return times, base, cold


if __name__ == "__main__":
    main()
