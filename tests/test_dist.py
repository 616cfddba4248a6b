"""Multi-process row sharding on CPU with gloo, world 2.

Each rank takes its contiguous row range from spmv_partition_rows, builds
its shard, computes y_shard with the product's CPU loop (the device
kernel reads the same arrays; on the GPU box bench.py runs the same
split over RCCL), and the shards are concatenated with an all-gather
padded to the largest shard — the exchange step of the path.  The
gathered y must equal the oracle's y for the whole matrix.
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

import spmv_amd as sa
from conftest import GOLDEN, PKG, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, fmt, q):
    sys.path[:0] = [str(PKG), str(REPO)]
    import torch
    import torch.distributed as dist

    import spmv_amd as sa
    from oracle import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if case == "cantlike":
            m = sa.gen_cantlike(0)
        elif case == "rmat":
            m = sa.gen_rmat(200_000, 2_000_000, scale=18, seed=3)
        else:
            m = sa.read_mtx(GOLDEN / f"{case}.mtx")
        ptr, _, _ = sa.csr_from_coo(m)
        bounds = sa.partition_rows(m.n_rows, ptr, world, align=64)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        loc = sa.shard(m, lo, hi)
        x = sa.ramp_x(m.n_cols)  # replicated
        y = np.zeros(max(loc.n_rows, 1))
        L = sa.host_lib()
        lptr, lcol, lval = sa.csr_from_coo(loc)
        if fmt == "csr":
            L.spmv_cpu_csr(loc.n_rows, sa._ptr(lptr), sa._ptr(lcol), sa._ptr(lval), sa._ptr(x), sa._ptr(y), 1)
        else:
            s = sa.sell_build(loc.n_rows, lptr, lcol, lval, C=64, sigma=1024 if loc.n_rows >= 1024 else 64, ki=2)
            L.spmv_cpu_sell(loc.n_rows, 64, 2, s["n_slices"], sa._ptr(s["slice_ptr"]), sa._ptr(s["perm"]),
                            sa._ptr(s["col"]), sa._ptr(s["val"]), sa._ptr(x), sa._ptr(y), 1)
        # all-gather of y shards, padded to the largest shard
        sizes = np.diff(bounds)
        pad = int(sizes.max()) if sizes.size else 0
        buf = torch.zeros(max(pad, 1), dtype=torch.float64)
        buf[: loc.n_rows] = torch.from_numpy(y[: loc.n_rows])
        out = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(out, buf)
        y_full = np.concatenate([out[r][: sizes[r]].numpy() for r in range(world)])
        y_ref = oracle.file_order_spmv(m.n_rows, m.row, m.col, m.val, x)
        bad = oracle.parity(y_full, y_ref, m.row, m.col, m.val, x, m.n_rows)
        q.put((rank, int(bad.size), lo, hi, int(loc.nnz)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,fmt", [("cantlike", "csr"), ("cantlike", "sell"), ("rmat", "csr"),
                                      ("empty_rows", "csr"), ("n67", "sell"), ("all_empty", "csr")])
def test_two_rank_shard_allgather(case, fmt):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, fmt, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(2))
    assert all(bad == 0 for _, bad, *_ in res)
    assert res[0][3] == res[1][2]  # contiguous ranges


def test_partition_balances_entries():
    m = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=2)
    ptr, _, _ = sa.csr_from_coo(m)
    for parts in (1, 2, 4, 8):
        b = sa.partition_rows(m.n_rows, ptr, parts, align=1024)
        assert b[0] == 0 and b[-1] == m.n_rows and np.all(np.diff(b) >= 0)
        assert np.all(b[1:-1] % 1024 == 0)
        nnz = np.diff(ptr[b])
        assert nnz.max() <= 1.1 * m.nnz / parts + 1024 * 200
    b = sa.partition_rows(10, np.zeros(11, np.int64), 4, align=1)
    assert b.tolist() == [0, 2, 5, 7, 10]


@pytest.mark.parametrize("w", [0.0, 0.5, 2.0, 8.0])
def test_weighted_partition_balances_cost(w):
    """spmv_partition_rows_weighted: contiguous aligned ranges whose
    entries + w * rows are balanced (w = 0 is the plain nnz partition)."""
    m = sa.gen_rmat(200_000, 2_000_000, scale=18, seed=3)
    ptr, _, _ = sa.csr_from_coo(m)
    parts = 8
    b = sa.partition_rows(m.n_rows, ptr, parts, align=64, row_weight=w)
    assert b[0] == 0 and b[-1] == m.n_rows and np.all(np.diff(b) >= 0)
    assert np.all(b[1:-1] % 64 == 0)
    if w == 0.0:
        assert np.array_equal(b, sa.partition_rows(m.n_rows, ptr, parts, align=64))
    cost = ptr[b[1:]] - ptr[b[:-1]] + w * np.diff(b)
    total = ptr[-1] + w * m.n_rows
    # every cut is within one aligned block (+ its longest row) of its target
    slack = 64 * (w + 1) + np.diff(ptr).max()
    assert np.all(np.abs(cost - total / parts) <= 2 * slack)


def _recut_worker(rank, world, port, q):
    """bench.py's profile-guided cut on CPU: time the weighted cut's shard,
    all-gather the times, re-cut (every rank alike), compute again, gather y."""
    sys.path[:0] = [str(PKG), str(REPO)]
    import time

    import torch
    import torch.distributed as dist

    import spmv_amd as sa
    from oracle import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = sa.gen_rmat(200_000, 2_000_000, scale=18, seed=3)
        ptr, col, val = sa.csr_from_coo(m)
        x = sa.ramp_x(m.n_cols)
        L = sa.host_lib()

        def shard_y(b):
            lo, hi = int(b[rank]), int(b[rank + 1])
            lptr = np.ascontiguousarray(ptr[lo:hi + 1] - ptr[lo])
            lcol = np.ascontiguousarray(col[ptr[lo]:ptr[hi]])
            lval = np.ascontiguousarray(val[ptr[lo]:ptr[hi]])
            y = np.zeros(max(hi - lo, 1))
            t0 = time.perf_counter()
            for _ in range(3):
                L.spmv_cpu_csr(hi - lo, sa._ptr(lptr), sa._ptr(lcol), sa._ptr(lval), sa._ptr(x), sa._ptr(y), 1)
            return y[:hi - lo], (time.perf_counter() - t0) / 3 * 1e3

        b0 = sa.partition_rows(m.n_rows, ptr, world, align=1024, row_weight=2.0)
        _, ms = shard_y(b0)
        g = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(g, torch.tensor([ms], dtype=torch.float64))
        b1 = sa.partition_rows_calibrated(m.n_rows, ptr, world, b0, [float(v.item()) for v in g],
                                          align=1024, row_weight=2.0)
        bs = [torch.zeros(world + 1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(bs, torch.from_numpy(b1))
        agree = all(torch.equal(bs[0], v) for v in bs)
        y, _ = shard_y(b1)
        sizes = np.diff(b1)
        pad = max(int(sizes.max()), 1)
        buf = torch.zeros(pad, dtype=torch.float64)
        buf[:y.size] = torch.from_numpy(y)
        out = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(out, buf)
        y_full = np.concatenate([out[r][:sizes[r]].numpy() for r in range(world)])
        y_ref = oracle.file_order_spmv(m.n_rows, m.row, m.col, m.val, x)
        bad = oracle.parity(y_full, y_ref, m.row, m.col, m.val, x, m.n_rows)
        q.put((rank, int(bad.size), bool(agree), b1.tolist()))
    finally:
        dist.destroy_process_group()


def _allgatherv_worker(rank, world, port, case, q):
    """bench.py's exchange step (rmat_strong / banded_strong): every rank
    writes its shard of y into a full-length vector, iterate.Comm.allgatherv
    fills in the other shards with their REAL sizes (no padding)."""
    sys.path[:0] = [str(PKG), str(REPO)]
    import torch
    import torch.distributed as dist

    import iterate
    import spmv_amd as sa
    from oracle import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = sa.gen_rmat(200_000, 2_000_000, scale=18, seed=3) if case == "rmat" else sa.read_mtx(GOLDEN / f"{case}.mtx")
        ptr, col, val = sa.csr_from_coo(m)
        x = sa.ramp_x(m.n_cols)
        if case == "rmat":
            bounds = sa.partition_rows(m.n_rows, ptr, world, align=1024, row_weight=2.0)
        else:  # golden file: rank 1 owns the last 3 rows
            cut = max(m.n_rows - 3, 0)
            bounds = np.array([0, cut, m.n_rows] if world == 2 else [0, m.n_rows], np.int64)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        y_full = torch.full((m.n_rows,), float("nan"), dtype=torch.float64)
        lptr = np.ascontiguousarray(ptr[lo:hi + 1] - ptr[lo])
        lcol, lval = np.ascontiguousarray(col[ptr[lo]:ptr[hi]]), np.ascontiguousarray(val[ptr[lo]:ptr[hi]])
        ys = np.zeros(max(hi - lo, 1))
        sa.host_lib().spmv_cpu_csr(hi - lo, sa._ptr(lptr), sa._ptr(lcol), sa._ptr(lval), sa._ptr(x), sa._ptr(ys), 1)
        y_full[lo:hi] = torch.from_numpy(ys[:hi - lo])
        how = iterate.Comm(dist).allgatherv(y_full, bounds)
        y_ref = oracle.file_order_spmv(m.n_rows, m.row, m.col, m.val, x)
        bad = oracle.parity(y_full.numpy(), y_ref, m.row, m.col, m.val, x, m.n_rows)
        q.put((rank, int(bad.size), bool(torch.isnan(y_full).any()), how))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["rmat", "ragged_shuffled", "all_empty"])
def test_two_rank_allgatherv_real_sizes(case):
    """World 2 over gloo: the unequal-shard all-gather of bench.py's strong-
    scaling legs assembles the whole y (oracle parity, no NaN left) from
    shards of their real sizes; the golden files give rank 1 the last three rows."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_allgatherv_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(2))
    assert all(bad == 0 and not nan for _, bad, nan, _ in res), res
    assert all(how == "gloo broadcast per shard" for *_, how in res)


def test_two_rank_calibrated_recut():
    """World 2 over gloo: the measured-cost re-cut is the same on both ranks
    (times all-gathered first), covers every row once, and the re-sharded
    product still equals the oracle's whole y."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_recut_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(2))
    assert all(bad == 0 and agree for _, bad, agree, _ in res)
    b = res[0][3]
    assert b == res[1][3] and b[0] == 0 and b[-1] == 200_000 and b[1] % 1024 == 0
