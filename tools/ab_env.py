#!/usr/bin/env python3
"""Interleaved A/B of the library's switches (spmv_set_option: xwin_remap,
xcd_remap, stream_nt; placement and load policy, never a result bit) on
ONE device matrix built once, and of to_device keywords (one matrix each).

    python tools/ab_env.py --format csr --opt xwin_remap=0,1 [--kw JSON ...] [--rounds 5]

Every configuration runs `--reps` back-to-back launches per round (HIP events
on the launch stream), configurations interleaved round by round in one
process; prints the median of the per-round means and whether y is
bit-identical to the first configuration's.
"""
from __future__ import annotations

import argparse
import itertools
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "opencl-spmv-algorithms_amd"), str(REPO)]
import spmv_amd as sa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--format", default="csr")
    ap.add_argument("--matrix", default="cantlike", choices=["cantlike", "rmat", "banded"])
    ap.add_argument("--banded-rows", type=int, default=20_000_000, help="banded: rows (16 entries each)")
    ap.add_argument("--copies", type=int, default=32)
    ap.add_argument("--opt", action="append", default=[],
                    help="NAME=v1,v2 of spmv_amd.OPTIONS, -1 = default (several: cartesian product)")
    ap.add_argument("--kw", action="append", default=[],
                    help="to_device keyword arguments (JSON; several: one device matrix each, crossed with --env)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--total", action="store_true",
                    help="time the reps as one span (two events) instead of an event after every launch")
    ap.add_argument("--graph", action="store_true",
                    help="with --total: capture the reps launches into one HIP graph and time its replay")
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda:0")
    if a.matrix == "banded":  # generated in HBM (BASELINE.json configs[4] structure)
        nb = a.banded_rows
        m = sa.Coo(nb, nb, np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0))  # sizes only
        b = sa.bytes_alg(nb, nb, 16 * nb)
    else:
        m = sa.gen_cantlike(0, a.copies) if a.matrix == "cantlike" else sa.gen_rmat()
        b = sa.bytes_alg(m.n_rows, m.n_cols, m.nnz)
    keys, vals = [], []
    for e in a.opt:
        k, v = e.split("=", 1)
        keys.append(k)
        vals.append(v.split(","))
    envs = [dict(zip(keys, c)) for c in itertools.product(*vals)] or [{}]
    kws = a.kw or ["{}"]
    x = torch.from_numpy(np.random.default_rng(7).uniform(-1, 1, m.n_cols)).to(dev)
    y = torch.empty(m.n_rows, dtype=torch.float64, device=dev)
    dms = []
    for kw in kws:
        if a.matrix == "banded":
            dms.append(sa.banded_to_device(m.n_rows, a.format, dev, **json.loads(kw)))
        else:
            dms.append(sa.to_device(m, a.format, dev, **json.loads(kw)))
    configs = [(i, env) for i in range(len(kws)) for env in envs]
    s = torch.cuda.current_stream()
    res = [[] for _ in configs]
    same = [True for _ in configs]
    y0 = None
    for _ in range(a.rounds):
        for i, (di, env) in enumerate(configs):
            dm = dms[di]
            for k, v in env.items():
                sa.set_option(k, int(v))
            for _ in range(5):
                dm.run(x, y, s)
            if a.total and a.graph:
                torch.cuda.synchronize()
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr):
                    for k in range(a.reps):
                        dm.run(x, y)
                torch.cuda.synchronize()
                gr.replay()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record(s)
                gr.replay()
                ev[1].record(s)
                torch.cuda.synchronize()
                res[i].append(ev[0].elapsed_time(ev[1]) / a.reps)
                del gr
            elif a.total:
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record(s)
                for k in range(a.reps):
                    dm.run(x, y, s)
                ev[1].record(s)
                torch.cuda.synchronize()
                res[i].append(ev[0].elapsed_time(ev[1]) / a.reps)
            else:
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
                ev[0].record(s)
                for k in range(a.reps):
                    dm.run(x, y, s)
                    ev[k + 1].record(s)
                torch.cuda.synchronize()
                res[i].append(float(np.mean([ev[k].elapsed_time(ev[k + 1]) for k in range(a.reps)])))
            if y0 is None:
                y0 = y.clone()
            elif not torch.equal(y.view(torch.int64), y0.view(torch.int64)):
                same[i] = False
            for k in env:
                sa.set_option(k, None)
    for i, (di, env) in enumerate(configs):
        ms = float(np.median(res[i]))
        print(json.dumps(dict(fmt=a.format, kw=kws[di], env=env, ms=round(ms, 5), GBs_alg=round(b / ms * 1e-6, 1),
                              frac=round(b / ms * 1e-6 / sa.HBM_PEAK_GBS, 4),
                              spread=round((max(res[i]) - min(res[i])) / ms, 4), bit_identical=same[i])),
              flush=True)
    print(json.dumps({"matrix": a.matrix, "copies": a.copies, "bytes_alg": b, "params": [d.params for d in dms]},
                     default=str))


if __name__ == "__main__":
    main()
