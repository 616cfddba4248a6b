"""Iterated SpMV on the MI355X through libspmv_hip.

The vector kernels against fp64 torch references, the dot product's
determinism, power iteration against the numpy restatement of the same
algorithm, CG against the oracle's residual, HIP-graph replay bit-identical
to eager launches, and two ranks (gloo, sharing cuda:0) against one.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

import iterate as it
import spmv_amd as sa
from conftest import REPO
from iterate_double import laplacian_2d, numpy_power
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    return torch, torch.device("cuda:0")


def _sym_random(n=3000, seed=4):
    b = sa.gen_random(n, n, 0, 12, seed=seed)
    d = np.arange(n, dtype=np.int32)
    return sa.Coo(n, n, np.concatenate([b.row, b.col, d]), np.concatenate([b.col, b.row, d]),
                  np.concatenate([b.val, b.val, np.full(n, 8.0)]), False, "sym random")


@pytest.mark.parametrize("n", [0, 1, 255, 4097, 1_000_003])
def test_dot_matches_fp64_and_is_deterministic(torch_dev, n):
    torch, dev = torch_dev
    g = torch.Generator(device=dev)
    g.manual_seed(n)
    a = torch.rand(max(n, 1), dtype=torch.float64, device=dev, generator=g) - 0.5
    b = torch.rand(max(n, 1), dtype=torch.float64, device=dev, generator=g) - 0.5
    lib = sa.hip_lib()
    ws = torch.empty(lib.spmv_dot_ws_bytes(n), dtype=torch.uint8, device=dev)
    out = torch.full((2,), float("nan"), dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    for k in range(2):
        assert lib.spmv_dot(n, sa._ptr(a), sa._ptr(b), sa._ptr(out[k:]), sa._ptr(ws), ws.numel(), 0, s) == 0
    torch.cuda.synchronize()
    ref = float(np.dot(a[:n].cpu().numpy(), b[:n].cpu().numpy())) if n else 0.0
    assert abs(float(out[0]) - ref) <= 1e-12 * max(1.0, float((a[:n].abs() * b[:n].abs()).sum()))
    assert torch.equal(out[0:1].view(torch.int64), out[1:2].view(torch.int64))


def test_dot_rejects_small_workspace(torch_dev):
    torch, dev = torch_dev
    lib = sa.hip_lib()
    a = torch.ones(1 << 20, dtype=torch.float64, device=dev)
    out = torch.empty(1, dtype=torch.float64, device=dev)
    ws = torch.empty(8, dtype=torch.uint8, device=dev)
    rc = lib.spmv_dot(a.numel(), sa._ptr(a), sa._ptr(a), sa._ptr(out), sa._ptr(ws), 8, 0, None)
    assert rc == sa.OTHER_ERROR


def test_vector_updates(torch_dev):
    torch, dev = torch_dev
    lib = sa.hip_lib()
    n = 300_001
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    x = torch.rand(n, dtype=torch.float64, device=dev, generator=g)
    y0 = torch.rand(n, dtype=torch.float64, device=dev, generator=g)
    num = torch.tensor([3.0], dtype=torch.float64, device=dev)
    den = torch.tensor([7.0], dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    y = y0.clone()
    assert lib.spmv_axpy_ratio(n, sa._ptr(num), sa._ptr(den), -1.0, sa._ptr(x), sa._ptr(y), 0, s) == 0
    torch.testing.assert_close(y, y0 - (3.0 / 7.0) * x, rtol=1e-15, atol=1e-15)
    y = y0.clone()
    assert lib.spmv_xpay_ratio(n, sa._ptr(num), sa._ptr(den), sa._ptr(x), sa._ptr(y), 0, s) == 0
    torch.testing.assert_close(y, x + (3.0 / 7.0) * y0, rtol=1e-15, atol=1e-15)
    y = torch.empty_like(x)
    assert lib.spmv_scale_rsqrt(n, sa._ptr(den), sa._ptr(x), sa._ptr(y), 0, s) == 0
    torch.testing.assert_close(y, x / np.sqrt(7.0), rtol=1e-15, atol=0.0)


@pytest.mark.parametrize("fmt", ["csr", "sell", "cmrs", "coo"])
def test_power_iteration_matches_numpy(torch_dev, fmt):
    torch, dev = torch_dev
    m = _sym_random()
    op = it.build_operator(m, 0, 1, fmt, dev, align=64)
    hist, x = it.power_iteration(op, 60)
    x0 = 1.0 + (np.arange(m.n_rows) % 7) / 7.0
    ref, xr = numpy_power(m, 60, x0)
    assert np.allclose(hist, ref, rtol=1e-11)
    assert np.allclose(x.cpu().numpy(), xr, rtol=1e-9, atol=1e-13)


@pytest.mark.parametrize("split", [False, True])
def test_side_stream_same_bits(torch_dev, split):
    """kernels on a non-default stream (HipKernels(stream=s)):
    the solve runs on that stream end to end (copies, dots, the exchange and
    the host reads ordered with the SpMVs), same bits as the default."""
    torch, dev = torch_dev
    m = _sym_random()
    ref = it.build_operator(m, 0, 1, "csr", dev, align=64, split=split)
    h1, x1 = it.power_iteration(ref, 30)
    x1 = x1.clone()
    op = it.build_operator(m, 0, 1, "csr", dev, align=64, split=split)
    s = torch.cuda.Stream(dev)
    op.kernels.stream = s
    if op.remote is not None:
        op.remote.stream = s
    h2, x2 = it.power_iteration(op, 30)
    torch.cuda.synchronize()
    assert np.array_equal(h1.view(np.int64), h2.view(np.int64))
    assert torch.equal(x1.view(torch.int64), x2.view(torch.int64))
    xs, iters, res = it.cg(op, torch.ones(op.rows, dtype=torch.float64, device=dev), maxit=50)
    torch.cuda.synchronize()
    assert iters > 0 and np.isfinite(res)


def test_power_iteration_graph_replay_same_bits(torch_dev):
    torch, dev = torch_dev
    m = sa.gen_cantlike(0, copies=2)
    op = it.build_operator(m, 0, 1, "csr", dev, align=64)
    h1, x1 = it.power_iteration(op, 40, graph=False)
    x1 = x1.clone()
    h2, x2 = it.power_iteration(op, 40, graph=True, block=8)
    assert np.array_equal(h1.view(np.int64), h2.view(np.int64))
    assert torch.equal(x1.view(torch.int64), x2.view(torch.int64))


@pytest.mark.parametrize("fmt", ["csr", "sell"])
def test_cg_laplacian_residual(torch_dev, fmt):
    torch, dev = torch_dev
    m = laplacian_2d(150)
    op = it.build_operator(m, 0, 1, fmt, dev, align=64)
    b = torch.ones(m.n_rows, dtype=torch.float64, device=dev)
    x, its, rel = it.cg(op, b, tol=1e-10, maxit=2000, check_every=10)
    assert rel <= 1e-10 and its < 2000
    xh = x.cpu().numpy()
    r = 1.0 - oracle.file_order_spmv(m.n_rows, m.row, m.col, m.val, xh)
    assert np.linalg.norm(r) <= 2e-10 * np.sqrt(m.n_rows)


@pytest.mark.parametrize("what", ["power", "cg"])
def test_two_ranks_sharing_the_gpu(tmp_path, what):
    """Two processes (gloo, both on cuda:0) give the single-rank answer:
    the all-reduced scalars make every rank's history identical."""
    out = tmp_path / "r"
    base = [sys.executable, str(REPO / "tools" / "iterate_bench.py"), "--what", what, "--iters",
            "60" if what == "power" else "1000"]
    base += ["--matrix", "sym"] if what == "power" else ["--matrix", "laplacian", "--k", "120"]
    env = dict(os.environ)
    one = subprocess.run(base + ["--out", str(out) + "1"], capture_output=True, text=True, timeout=600, env=env)
    assert one.returncode == 0, one.stdout + one.stderr
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", "29561"] + base[1:] +
                         ["--backend", "gloo", "--share-gpu", "--out", str(out) + "2"],
                         capture_output=True, text=True, timeout=600, env=env)
    assert two.returncode == 0, two.stdout + two.stderr
    r1 = json.loads((tmp_path / "r1.rank0").read_text())
    r2 = [json.loads((tmp_path / f"r2.rank{k}").read_text()) for k in range(2)]
    assert r2[0]["lo"] == 0 and r2[1]["lo"] == r2[0]["rows"]
    if what == "power":
        assert r2[0]["lambda"] == r2[1]["lambda"]
        assert abs(r2[0]["lambda"] - r1["lambda"]) <= 1e-10 * abs(r1["lambda"])
    else:
        assert r2[0]["iterations"] == r2[1]["iterations"]
        assert r2[0]["rel_residual"] <= 1e-10 and r1["rel_residual"] <= 1e-10
    sq = r2[0]["x_sq"] + r2[1]["x_sq"]
    assert abs(sq - r1["x_sq"]) <= 1e-9 * r1["x_sq"]


def test_two_ranks_overlap_same_bits_as_split(tmp_path):
    """§8f row 3 on the device: two ranks (gloo, sharing cuda:0) run power
    iteration with the shard split into local / remote column parts, once
    sequentially and once with the local part launched while the x
    all-gather is in flight: the same bits on every rank, and the unsplit
    answer within the parity rule."""
    base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
            "--master-addr", "127.0.0.1", "--master-port", "29563", str(REPO / "tools" / "iterate_bench.py"),
            "--what", "power", "--iters", "40", "--matrix", "sym", "--sym-rows", "20000", "--backend", "gloo", "--share-gpu"]
    res = {}
    for mode in ("plain", "split", "overlap"):
        p = subprocess.run(base + ["--mode", mode, "--out", str(tmp_path / mode)], capture_output=True, text=True,
                           timeout=600, env=dict(os.environ))
        assert p.returncode == 0, p.stdout + p.stderr
        res[mode] = [json.loads((tmp_path / f"{mode}.rank{k}").read_text()) for k in range(2)]
    for k in range(2):
        s, o, pl = res["split"][k], res["overlap"][k], res["plain"][k]
        assert s["x_head"] == o["x_head"] and s["x_sum"] == o["x_sum"] and s["x_sq"] == o["x_sq"]
        assert s["lambda"] == o["lambda"] and s["hist_tail"] == o["hist_tail"]
        assert abs(s["lambda"] - pl["lambda"]) <= 1e-10 * abs(pl["lambda"])


def test_overlap_rehearsal_runs(tmp_path):
    """The one-GPU rehearsal: overlapped and sequential launches give the
    same bits, and the split SpMV passes the parity rule on every rank."""
    p = subprocess.run([sys.executable, str(REPO / "tools" / "iterate_bench.py"), "--rehearse", "2", "--matrix",
                        "laplacian", "--k", "300", "--reps", "5"], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ))
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert all(r["overlap_same_bits"] and r["parity_ok"] for r in line["ranks"])
