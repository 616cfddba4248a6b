"""Iterated SpMV over row shards — CPU tests.

The gathered-layout renumbering and the multi-rank orchestration of
iterate.power_iteration / iterate.cg run here on gloo ranks with the numpy
kernel double (tests/iterate_double.py); tests/test_iterate_gpu.py runs the
same solvers through libspmv_hip on the MI355X.
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import scipy.sparse as sp

import iterate as it
import spmv_amd as sa
from conftest import PKG, REPO
from iterate_double import NumpyKernels, laplacian_2d, numpy_power


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sym_random(n=3000, seed=4):
    """B + B^T + 8 I: symmetric with a clear dominant eigenvalue."""
    b = sa.gen_random(n, n, 0, 12, seed=seed)
    r = np.concatenate([b.row, b.col, np.arange(n, dtype=np.int32)])
    c = np.concatenate([b.col, b.row, np.arange(n, dtype=np.int32)])
    v = np.concatenate([b.val, b.val, np.full(n, 8.0)])
    return sa.Coo(n, n, r.astype(np.int32), c.astype(np.int32), v, False, "sym random")


def _np_operator(m, rank, world, align=64, mode="plain"):
    """mode: plain (one SpMV on the gathered x), split (local / remote
    column parts, all-gather first), overlap (local part while the
    all-gather is in flight)."""
    counts = np.bincount(m.row, minlength=m.n_rows).astype(np.int64)
    layout = it.layout_for(m.n_rows, counts, world, align)
    loc = it.local_shard(m, layout, rank)
    if mode == "plain":
        return it.DistOperator(layout, rank, m.n_rows, NumpyKernels(loc), "cpu")
    local, remote = it.split_local_remote(loc, layout, rank)
    return it.DistOperator(layout, rank, m.n_rows, NumpyKernels(local), "cpu", NumpyKernels(remote),
                           mode == "overlap")


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_gathered_layout_renumbering(world):
    m = sa.gen_random(5000, 5000, 0, 40, seed=7)
    counts = np.bincount(m.row, minlength=m.n_rows).astype(np.int64)
    lay = it.layout_for(m.n_rows, counts, world, align=64)
    pos = lay.positions(np.arange(m.n_rows))
    assert len(np.unique(pos)) == m.n_rows and pos.max() < world * lay.pad
    v = np.random.default_rng(1).uniform(-1, 1, m.n_rows)
    assert np.array_equal(lay.from_gathered(lay.to_gathered(v), m.n_rows), v)
    # each shard times the gathered x equals its rows of A x
    A = sp.csr_matrix((m.val, (m.row, m.col)), shape=(m.n_rows, m.n_cols))
    y = A @ v
    xg = lay.to_gathered(v)
    for r in range(world):
        loc = it.local_shard(m, lay, r)
        Al = sp.csr_matrix((loc.val, (loc.row, loc.col)), shape=(loc.n_rows, loc.n_cols))
        lo, hi = lay.bounds[r], lay.bounds[r + 1]
        assert np.allclose(Al @ xg, y[lo:hi], rtol=1e-13, atol=1e-13)


def test_local_shard_rejects_rectangular():
    m = sa.gen_random(100, 120, 1, 5, seed=2)
    lay = it.layout_for(100, np.bincount(m.row, minlength=100).astype(np.int64), 1, 64)
    with pytest.raises(sa.SpmvError):
        it.local_shard(m, lay, 0)


def test_power_iteration_single_rank_matches_numpy():
    m = _sym_random()
    op = _np_operator(m, 0, 1)
    hist, x = it.power_iteration(op, 60)
    x0 = 1.0 + (np.arange(m.n_rows) % 7) / 7.0
    ref, xr = numpy_power(m, 60, x0)
    assert np.allclose(hist, ref, rtol=1e-12)
    assert np.allclose(x.numpy(), xr, rtol=1e-10, atol=1e-14)


def test_cg_single_rank_solves_laplacian():
    m = laplacian_2d(40)
    op = _np_operator(m, 0, 1)
    import torch

    b = torch.ones(m.n_rows, dtype=torch.float64)
    x, its, rel = it.cg(op, b, tol=1e-10, maxit=500, check_every=5)
    A = sp.csr_matrix((m.val, (m.row, m.col)), shape=(m.n_rows, m.n_cols))
    assert rel <= 1e-10 and its < 500
    assert np.linalg.norm(A @ x.numpy() - 1.0) <= 1e-9 * np.sqrt(m.n_rows)


def test_split_local_remote_parts():
    """The local part holds exactly the own-block columns (renumbered to the
    send block), the remote part the rest; together they are the shard."""
    m = sa.gen_random(4000, 4000, 0, 30, seed=5)
    counts = np.bincount(m.row, minlength=m.n_rows).astype(np.int64)
    lay = it.layout_for(m.n_rows, counts, 3, align=64)
    v = np.random.default_rng(2).uniform(-1, 1, m.n_rows)
    xg = lay.to_gathered(v)
    for r in range(3):
        loc = it.local_shard(m, lay, r)
        local, remote = it.split_local_remote(loc, lay, r)
        assert local.nnz + remote.nnz == loc.nnz and local.n_cols == lay.pad
        assert local.col.size == 0 or (local.col.min() >= 0 and local.col.max() < lay.pad)
        own = (remote.col >= r * lay.pad) & (remote.col < (r + 1) * lay.pad)
        assert not own.any()
        A = lambda c: sp.csr_matrix((c.val, (c.row, c.col)), shape=(c.n_rows, c.n_cols))  # noqa: E731
        send = xg[r * lay.pad:(r + 1) * lay.pad]
        assert np.allclose(A(local) @ send + A(remote) @ xg, A(loc) @ xg, rtol=1e-13, atol=1e-13)


def _worker(rank, world, port, what, q, mode="plain"):
    sys.path[:0] = [str(PKG), str(REPO), str(REPO / "tests")]
    import torch
    import torch.distributed as dist

    import iterate as it2

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = it2.Comm(dist)
        if what == "power":
            m = _sym_random()
            op = _np_operator(m, rank, world, mode=mode)
            hist, x = it2.power_iteration(op, 60, comm)
            q.put((rank, hist, op.lo, x.numpy().copy()))
        else:
            m = laplacian_2d(40)
            op = _np_operator(m, rank, world, mode=mode)
            b = torch.ones(op.rows, dtype=torch.float64)
            x, its, rel = it2.cg(op, b, comm, tol=1e-10, maxit=500, check_every=5)
            q.put((rank, (its, rel), op.lo, x.numpy().copy()))
    finally:
        dist.destroy_process_group()


def _run_ranks(world, what, mode="plain"):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, what, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_power_iteration_multi_rank(world):
    res = _run_ranks(world, "power")
    m = _sym_random()
    x0 = 1.0 + (np.arange(m.n_rows) % 7) / 7.0
    ref, xr = numpy_power(m, 60, x0)
    for _, hist, lo, x in res:
        assert np.allclose(hist, ref, rtol=1e-12)  # every rank sees the all-reduced scalars
    x = np.concatenate([r[3] for r in res])
    assert np.allclose(x, xr, rtol=1e-10, atol=1e-14)


def test_cg_two_ranks():
    res = _run_ranks(2, "cg")
    m = laplacian_2d(40)
    A = sp.csr_matrix((m.val, (m.row, m.col)), shape=(m.n_rows, m.n_cols))
    x = np.concatenate([r[3] for r in res])
    (its0, rel0), (its1, rel1) = res[0][1], res[1][1]
    assert its0 == its1 and rel0 == rel1 and rel0 <= 1e-10
    assert np.linalg.norm(A @ x - 1.0) <= 1e-9 * np.sqrt(m.n_rows)


@pytest.mark.parametrize("what,world", [("power", 2), ("power", 3), ("cg", 2)])
def test_overlap_same_bits_as_sequential(what, world):
    """§8f row 3: the overlapped loop (local-column SpMV while the x
    all-gather is in flight) gives the same bits as the same split run
    sequentially, on every rank, and the answer of the unsplit loop within
    the parity rule."""
    seq = _run_ranks(world, what, "split")
    ovl = _run_ranks(world, what, "overlap")
    plain = _run_ranks(world, what, "plain")
    for a, b, c in zip(seq, ovl, plain):
        assert np.array_equal(a[3], b[3])  # x: bit-identical
        if what == "power":
            assert np.array_equal(a[1], b[1])  # the all-reduced scalars too
            assert np.allclose(a[1], c[1], rtol=1e-12)
        else:
            assert a[1] == b[1]  # iterations and residual
        assert np.allclose(a[3], c[3], rtol=1e-9, atol=1e-12)
