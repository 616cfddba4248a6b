#!/usr/bin/env python3
"""Iterated SpMV on MI355X: power iteration / CG.

One process per GPU (torch.distributed.run; backend nccl = RCCL), or a
single process.  Each rank owns an nnz-balanced row range of the matrix in
the gathered layout (opencl-spmv-algorithms_amd/iterate.py); every
iteration is SpMV + deterministic dots + vector update + an in-place
all-reduce of the scalars + an all-gather of the new x.

    python tools/iterate_bench.py --what power --matrix cantlike --iters 200
    python tools/iterate_bench.py --what cg --matrix laplacian --k 2000
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        tools/iterate_bench.py --backend gloo --share-gpu --out gpurun_out/it.json

Prints one JSON line (rank 0): ms per iteration (max over ranks), the
share of it spent in the SpMV launch alone, effective GB/s of the SpMV's
algorithmic bytes per iteration, and the result (eigenvalue estimate or
CG residual).  --out also stores each rank's local result vector summary
for the multi-rank test.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "opencl-spmv-algorithms_amd"), str(REPO)]
import iterate as it  # noqa: E402
import spmv_amd as sa  # noqa: E402


def laplacian_2d(k: int, shift: float = 0.0) -> sa.Coo:
    n = k * k
    idx = np.arange(n, dtype=np.int64).reshape(k, k)
    rows, cols, vals = [idx.ravel()], [idx.ravel()], [np.full(n, 4.0 + shift)]
    for a, b in ((idx[:, :-1], idx[:, 1:]), (idx[:-1, :], idx[1:, :])):
        rows += [a.ravel(), b.ravel()]
        cols += [b.ravel(), a.ravel()]
        vals += [np.full(a.size, -1.0), np.full(a.size, -1.0)]
    r = np.concatenate(rows).astype(np.int32)
    c = np.concatenate(cols).astype(np.int32)
    v = np.concatenate(vals)
    o = np.lexsort((c, r))
    return sa.Coo(n, n, r[o], c[o], v[o], False, f"2-D Laplacian {k}x{k}")


def sym_random(n: int, seed: int = 4) -> sa.Coo:
    b = sa.gen_random(n, n, 0, 12, seed=seed)
    d = np.arange(n, dtype=np.int32)
    return sa.Coo(n, n, np.concatenate([b.row, b.col, d]), np.concatenate([b.col, b.row, d]),
                  np.concatenate([b.val, b.val, np.full(n, 8.0)]), False, f"symmetric random n={n}")


def make_matrix(a) -> sa.Coo:
    if a.matrix == "cantlike":
        return sa.gen_cantlike(0, a.copies)
    if a.matrix == "laplacian":
        return laplacian_2d(a.k)
    if a.matrix == "sym":
        return sym_random(a.n)
    raise SystemExit(f"unknown matrix {a.matrix}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", choices=["power", "cg"], default="power")
    ap.add_argument("--matrix", choices=["cantlike", "laplacian", "sym"], default="cantlike")
    ap.add_argument("--copies", type=int, default=32)
    ap.add_argument("--k", type=int, default=1000, help="Laplacian grid side")
    ap.add_argument("--n", type=int, default=3000, help="rows of the symmetric random matrix")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--format", default="csr")
    ap.add_argument("--graph", action="store_true", help="HIP-graph replay (one rank)")
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--share-gpu", action="store_true", help="all ranks on cuda:0 (rehearsal)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dev_idx = 0 if a.share_gpu else local
        torch.cuda.set_device(dev_idx)
        dist.init_process_group(a.backend, rank=rank, world_size=world)
    dev = torch.device(f"cuda:{0 if a.share_gpu else local}")
    comm = it.Comm(dist)

    m = make_matrix(a)
    op = it.build_operator(m, rank, world, a.format, dev, align=64)
    loc_nnz = int(np.count_nonzero((m.row >= op.lo) & (m.row < op.lo + op.rows)))
    bytes_iter = sa.bytes_alg(op.rows, m.n_cols, loc_nnz)

    def barrier():
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()

    # SpMV alone on this shard, for the share of the iteration it takes
    x = torch.ones(op.world * op.pad, dtype=torch.float64, device=dev)
    y = torch.empty(max(op.rows, 1), dtype=torch.float64, device=dev)
    for _ in range(5):
        op.kernels.spmv(x, y)
    barrier()
    t0 = time.perf_counter()
    for _ in range(50):
        op.kernels.spmv(x, y)
    barrier()
    spmv_ms = (time.perf_counter() - t0) / 50 * 1e3

    result = {}
    if a.what == "power":
        it.power_iteration(op, 3, comm, graph=False)  # warm-up
        barrier()
        t0 = time.perf_counter()
        hist, x_loc = it.power_iteration(op, a.iters, comm, graph=a.graph)
        barrier()
        el = time.perf_counter() - t0
        result = {"lambda": float(hist[-1, 0]), "lambda_prev": float(hist[-2, 0]) if a.iters > 1 else None,
                  "hist_tail": hist[-3:].tolist()}
        vec = x_loc
        n_it = a.iters
    else:
        b = torch.ones(op.rows, dtype=torch.float64, device=dev)
        it.cg(op, b, comm, maxit=3, check_every=3)  # warm-up
        barrier()
        t0 = time.perf_counter()
        vec, n_it, rel = it.cg(op, b, comm, tol=1e-10, maxit=a.iters, check_every=10)
        barrier()
        el = time.perf_counter() - t0
        result = {"iterations": n_it, "rel_residual": rel}
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms_it = float(t.item()) / max(n_it, 1) * 1e3
    total_bytes = bytes_iter
    bt = torch.tensor([float(bytes_iter)], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(bt)
        total_bytes = float(bt.item())
    line = {"what": a.what, "matrix": m.label, "n": m.n_rows, "nnz": m.nnz, "ranks": world,
            "backend": a.backend if world > 1 else None, "format": a.format, "graph": a.graph,
            "iterations": n_it, "ms_per_iter": round(ms_it, 5), "spmv_ms_rank": round(spmv_ms, 5),
            "spmv_share": round(spmv_ms / ms_it, 4) if ms_it else None,
            "GBs_spmv_alg_per_iter": round(total_bytes / (ms_it * 1e-3) * 1e-9, 1), **result}
    if a.out:
        rec = {"rank": rank, "lo": op.lo, "rows": op.rows,
               "x_head": vec[: min(8, op.rows)].cpu().tolist(), "x_sum": float(vec.sum().item()),
               "x_sq": float((vec * vec).sum().item()), **line}
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        with open(f"{a.out}.rank{rank}", "w") as f:
            json.dump(rec, f)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
