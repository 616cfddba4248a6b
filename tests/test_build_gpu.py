"""Device format builders against the host builders.

spmv_dev_* build CSR / ELL / SELL-C-sigma / CMRS from a COO in HBM; every
array must equal the host builder's (host/formats.c) element for element,
and the SpMV of a device-built matrix must pass the oracle parity check.
"""
from __future__ import annotations

import numpy as np
import pytest

import spmv_amd as sa
from conftest import GOLDEN, golden_cases
from oracle import oracle

pytestmark = pytest.mark.gpu

CASES = [c["name"] for c in golden_cases()]


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    return torch, torch.device("cuda:0")


def _mats():
    out = [(c, sa.read_mtx(GOLDEN / f"{c}.mtx")) for c in CASES]
    out += [("cantlike1", sa.gen_cantlike(1)), ("ragged", sa.gen_random(20_000, 30_000, 0, 400, seed=3)),
            ("rmat", sa.gen_rmat(200_000, 2_000_000, scale=18, seed=2))]
    return out


MATS = _mats()
IDS = [n for n, _ in MATS]


def _eq(dev_t, host_a, n=None):
    d = dev_t.cpu().numpy()
    h = np.asarray(host_a)
    n = h.shape[0] if n is None else n
    return np.array_equal(d[:n], h[:n])


@pytest.mark.parametrize("name,m", MATS, ids=IDS)
def test_csr_matches_host(torch_dev, name, m):
    torch, dev = torch_dev
    dm = sa.device_build(m, "csr", dev, xwin=False)
    ptr, col, val = sa.csr_from_coo(m)
    assert _eq(dm.arrays["row_ptr"], ptr)
    assert _eq(dm.arrays["col"], col, m.nnz) and _eq(dm.arrays["val"], val, m.nnz)


@pytest.mark.parametrize("ki", [1, 2])
@pytest.mark.parametrize("name,m", [t for t in MATS if t[0] != "rmat"], ids=[n for n in IDS if n != "rmat"])
def test_ell_matches_host(torch_dev, name, m, ki):
    torch, dev = torch_dev
    dm = sa.device_build(m, "ell", dev, ki=ki, xwin=False)
    ptr, col, val = sa.csr_from_coo(m)
    e = sa.ell_build(m.n_rows, ptr, col, val, ki=ki)
    assert (dm.params["K"], dm.params["ld"]) == (e["K"], e["ld"])
    assert _eq(dm.arrays["col"], e["col"], e["stored"]) and _eq(dm.arrays["val"], e["val"], e["stored"])


@pytest.mark.parametrize("C,sigma,ki", [(64, 1024, 1), (64, 1, 2), (32, 64, 2), (64, 4096, 1)])
@pytest.mark.parametrize("name,m", MATS, ids=IDS)
def test_sell_matches_host(torch_dev, name, m, C, sigma, ki):
    torch, dev = torch_dev
    dm = sa.device_build(m, "sell", dev, C=C, sigma=sigma, ki=ki, xwin=False)
    ptr, col, val = sa.csr_from_coo(m)
    s = sa.sell_build(m.n_rows, ptr, col, val, C=C, sigma=sigma, ki=ki)
    assert dm.params["stored"] == s["stored"] and dm.params["n_slices"] == s["n_slices"]
    assert _eq(dm.arrays["perm"], s["perm"], s["n_slices"] * C)
    assert _eq(dm.arrays["slice_ptr"], s["slice_ptr"])
    assert _eq(dm.arrays["col"], s["col"], s["stored"]) and _eq(dm.arrays["val"], s["val"], s["stored"])


@pytest.mark.parametrize("h", [1, 8, 64])
@pytest.mark.parametrize("name,m", MATS, ids=IDS)
def test_cmrs_matches_host(torch_dev, name, m, h):
    torch, dev = torch_dev
    dm = sa.device_build(m, "cmrs", dev, h=h)
    ptr, _, _ = sa.csr_from_coo(m)
    c = sa.cmrs_build(m.n_rows, ptr, h=h)
    assert _eq(dm.arrays["strip_ptr"], c["strip_ptr"])
    assert _eq(dm.arrays["row_in_strip"], c["row_in_strip"], m.nnz)


@pytest.mark.parametrize("fmt", ["csr", "ell", "sell", "cmrs"])
def test_device_built_spmv_parity(torch_dev, fmt):
    torch, dev = torch_dev
    m = sa.gen_cantlike(2, copies=2)
    dm = sa.device_build(m, fmt, dev)
    x = np.random.default_rng(5).uniform(-1, 1, m.n_cols)
    y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    dm.run(torch.from_numpy(x).to(dev), y)
    torch.cuda.synchronize()
    y_ref = oracle.file_order_spmv(m.n_rows, m.row, m.col, m.val, x)
    bad = oracle.parity(y.cpu().numpy(), y_ref, m.row, m.col, m.val, x, m.n_rows)
    assert bad.size == 0


def test_bad_row_index_rejected(torch_dev):
    torch, dev = torch_dev
    m = sa.gen_random(100, 100, 1, 5, seed=1)
    bad = sa.Coo(m.n_rows, m.n_cols, m.row.copy(), m.col, m.val)
    bad.row[3] = 100  # == n_rows
    with pytest.raises(sa.SpmvError):
        sa.device_build(bad, "csr", dev)


def test_sigma_above_device_sort_limit_rejected(torch_dev):
    torch, dev = torch_dev
    m = sa.gen_random(10_000, 10_000, 1, 5, seed=1)
    with pytest.raises(sa.SpmvError):
        sa.device_build(m, "sell", dev, sigma=8192)
