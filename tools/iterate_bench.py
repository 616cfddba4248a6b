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

--mode split / overlap: the shard split into local / remote column parts
(iterate.split_local_remote); overlap runs the local part while the x
all-gather is in flight.

--rehearse W (one process, one GPU): the overlap rehearsal.  For every
rank r of a W-way cut, the shard's SpMV is timed unsplit, as its local and
remote parts, and against an exchange stand-in: a device-to-device copy of
the bytes rank r receives in the all-gather ((W-1) blocks of x), issued on
a second stream.  Sequential = copy, then local + remote; overlapped = copy
on the second stream while the local part runs, then the remote part.  On
one GPU the copy moves HBM to HBM, so it competes with the SpMV for the
same bandwidth; over xGMI the received bytes arrive over the links.
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
import launch  # noqa: E402
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
        return sym_random(a.sym_rows)
    if a.matrix == "rmat":
        return sa.gen_rmat()
    raise SystemExit(f"unknown matrix {a.matrix}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", choices=["power", "cg"], default="power")
    ap.add_argument("--matrix", choices=["cantlike", "laplacian", "sym", "rmat"], default="cantlike")
    ap.add_argument("--copies", type=int, default=32)
    ap.add_argument("--k", type=int, default=1000, help="Laplacian grid side")
    ap.add_argument("--sym-rows", type=int, default=3000, help="rows of the symmetric random matrix")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--format", default="csr")
    ap.add_argument("--graph", action="store_true", help="HIP-graph replay (one rank)")
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks; without torch.distributed.run, N > 1 starts N ranks in a child job")
    ap.add_argument("--share-gpu", action="store_true", help="all ranks on cuda:0 (rehearsal)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--mode", choices=["plain", "split", "overlap"], default="plain",
                    help="split: local / remote column parts; overlap: local part during the all-gather")
    ap.add_argument("--rehearse", type=int, default=0, metavar="W",
                    help="one-GPU overlap rehearsal of a W-way cut (no torch.distributed)")
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    if launch.needs_spawn(a.gpus):  # N ranks in a child torch.distributed.run job
        sys.exit(launch.spawn_ranks(__file__, a.gpus))
    if a.rehearse:
        return rehearse(a)

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
    op = it.build_operator(m, rank, world, a.format, dev, align=64, split=a.mode != "plain",
                           overlap=a.mode == "overlap")
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
            "backend": a.backend if world > 1 else None, "format": a.format, "graph": a.graph, "mode": a.mode,
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


def rehearse(a):
    """One-GPU overlap rehearsal (see the module docstring)."""
    import torch

    dev = torch.device("cuda:0")
    W = a.rehearse
    m = make_matrix(a)
    counts = np.bincount(m.row, minlength=m.n_rows).astype(np.int64)
    layout = it.layout_for(m.n_rows, counts, W, 1024)
    xg = torch.from_numpy(layout.to_gathered(sa.ramp_x(m.n_rows) / m.n_rows + 0.5)).to(dev)
    main, side = torch.cuda.current_stream(dev), torch.cuda.Stream(dev)
    lib = sa.hip_lib()
    one = torch.ones(1, dtype=torch.float64, device=dev)
    out = []
    for r in range(W):
        loc = it.local_shard(m, layout, r)
        local, remote = it.split_local_remote(loc, layout, r)
        d_all = sa.to_device(loc, a.format, dev)
        d_loc = sa.to_device(local, a.format, dev)
        d_rem = sa.to_device(remote, a.format, dev)
        rows = loc.n_rows
        full = xg.clone()
        send = full[r * layout.pad:(r + 1) * layout.pad]
        src = xg.clone()  # what the other ranks would send
        recv = [(k * layout.pad, (k + 1) * layout.pad) for k in range(W) if k != r]
        y, y2, yp = (torch.zeros(max(rows, 1), dtype=torch.float64, device=dev) for _ in range(3))

        def add():
            sa._check(lib.spmv_axpy_ratio(rows, sa._ptr(one), sa._ptr(one), 1.0, sa._ptr(y2), sa._ptr(y), 0,
                                          main.cuda_stream), "axpy")

        def exchange(st):
            with torch.cuda.stream(st):
                for lo, hi in recv:
                    full[lo:hi].copy_(src[lo:hi], non_blocking=True)

        def seq():
            exchange(main)
            d_loc.run(send, y)
            d_rem.run(full, y2)
            add()

        def ovl():
            side.wait_stream(main)
            exchange(side)
            d_loc.run(send, y)
            main.wait_stream(side)
            d_rem.run(full, y2)
            add()

        legs = {"plain_spmv": lambda: d_all.run(full, yp), "local": lambda: d_loc.run(send, y),
                "remote_add": lambda: (d_rem.run(full, y2), add()), "exchange_copy": lambda: exchange(main),
                "sequential": seq, "overlapped": ovl}
        t = {}
        for name, fn in legs.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main)
            for _ in range(a.reps):
                fn()
            e1.record(main)
            torch.cuda.synchronize()
            t[name] = round(e0.elapsed_time(e1) / a.reps, 5)
        seq()
        torch.cuda.synchronize()
        y_seq = y.clone()
        ovl()
        torch.cuda.synchronize()
        same = bool(torch.equal(y_seq.view(torch.int64), y.view(torch.int64)))
        bad, first = sa.check(loc, xg.cpu().numpy(), y[:rows].cpu().numpy())
        out.append({"rank": r, "rows": rows, "nnz_local": local.nnz, "nnz_remote": remote.nnz,
                    "recv_bytes": 8 * layout.pad * (W - 1), "ms": t, "overlap_same_bits": same,
                    "parity_ok": bad == 0})
        del d_all, d_loc, d_rem
        torch.cuda.empty_cache()
    worst = {k: max(o["ms"][k] for o in out) for k in out[0]["ms"]}
    print(json.dumps({"rehearsal": f"overlap, {W}-way cut on one GPU", "matrix": m.label, "format": a.format,
                      "max_over_ranks_ms": worst, "ranks": out}), flush=True)


if __name__ == "__main__":
    main()
