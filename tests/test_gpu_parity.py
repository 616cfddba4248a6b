"""Parity of the HIP path (libspmv_hip.so through the C-ABI) with the oracle.

Criterion (BASELINE.json north_star): per row
    |y - y_ref| <= 1e-6 * max(|y_ref|, sum_j |a_ij x_j|)
against the file-order sum of check_result (oracle/oracle.c), plus the
committed scipy fixtures.  Every output buffer is pre-filled with NaN so a
row the kernel forgets to write fails.  Full-size configs (R-MAT 1e8
entries, banded shards) are checked against the oracle directly (it is C
and finishes in seconds) or through size-independent identities.
"""
from __future__ import annotations

import numpy as np
import pytest

import spmv_amd as sa
from conftest import GOLDEN, golden_cases
from oracle import oracle

pytestmark = pytest.mark.gpu

CASES = [c["name"] for c in golden_cases()]

FMT_PARAMS = [
    ("coo", {}),
    ("csr", {}),
    ("csr", {"lanes": 2}),
    ("csr", {"lanes": 8}),
    ("csr", {"lanes": 32}),
    ("csr", {"lanes": 64}),
    ("csr", {"variant": 2}),
    ("csr", {"lanes": 2, "variant": 2}),
    ("csr", {"lanes": 64, "variant": 2}),
    ("csr", {"variant": 3}),
    ("csr", {"variant": 4}),
    ("csr", {"variant": 1}),
    ("csr", {"lanes": 2, "variant": 1}),
    ("csr", {"lanes": 64, "variant": 1}),
    ("csr16", {}),
    ("csrf32", {}),
    ("csrf32", {"lanes": 2}),
    ("csr16", {"lanes": 2}),
    ("csr16", {"lanes": 64}),
    ("ell", {"ki": 1}),
    ("ell", {"ki": 2}),
    ("sell", {"C": 64, "sigma": 1024, "ki": 2}),
    ("sell", {"C": 64, "sigma": 1024, "ki": 1, "xwin": True}),
    ("sell", {"C": 32, "sigma": 64, "ki": 2, "xwin": True}),
    ("ell", {"ki": 2, "xwin": True}),
    ("hyb", {}),
    ("hyb", {"ki": 1}),
    # ELL part + tail forced (the rule picks one part on small matrices: a
    # second kernel's fixed cost outweighs the bytes the split saves)
    ("hyb", {"hyb_k": 2}),
    ("hyb", {"hyb_k": 3, "ki": 1}),
    ("csr", {"xwin": True}),
    ("csr", {"lanes": 2, "xwin": True}),
    ("sell", {"C": 64, "sigma": 1, "ki": 1}),
    ("sell", {"C": 32, "sigma": 1, "ki": 1}),
    ("sell", {"C": 128, "sigma": 256, "ki": 2}),
    ("cmrs", {"h": 8}),
    ("cmrs", {"h": 1}),
    ("cmrs", {"h": 64}),
    # wide-slice split / entry-balanced CMRS forced on ordinary matrices
    # (tiny T: every slice wider than T is split; tiles cut strips anywhere)
    ("sell", {"C": 64, "sigma": 1024, "ki": 2, "split": 2}),
    ("sell", {"C": 32, "sigma": 64, "ki": 1, "split": 1, "xwin": True}),
    ("sell", {"C": 64, "sigma": 1, "ki": 1, "split": 3, "xwin": False}),
    ("cmrs", {"h": 8, "cmrs_variant": 1}),
    ("cmrs", {"h": 1, "cmrs_variant": 1}),
    ("cmrs", {"h": 64, "cmrs_variant": 1}),
    # COO with x windows in LDS (opt-in), CMRS with global x gathers
    ("coo", {"xwin": True}),
    ("coo", {"coo_tail": False}),  # the carry pass (default: single pass where rows allow)
    ("hyb", {"coo_tail": False, "hyb_k": 2}),  # HYB tail through the carry pass
    ("cmrs", {"h": 8, "xwin": False}),
    # SELL16: 16-bit column offsets from each workgroup's window base
    ("sell16", {"C": 64, "sigma": 1024, "ki": 2}),
    ("sell16", {"C": 64, "sigma": 1024, "ki": 1}),
    ("sell16", {"C": 64, "sigma": 1, "ki": 1}),
    # column-grouped CSR (gather-bound power-law matrices)
    ("csrg", {"groups": 1}),
    ("csrg", {"groups": 5}),
    ("csrg", {"groups": 32}),
]
IDS = [f"{f}-{'-'.join(f'{k}{v}' for k, v in kw.items()) or 'default'}" for f, kw in FMT_PARAMS]


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    return torch, torch.device("cuda:0")


def run_fmt(torch, dev, m, fmt, x=None, **kw):
    if fmt == "ell":
        kw.setdefault("ell_max_padding", None)  # tiny fixtures pad to 64 rows
    dm = sa.to_device(m, fmt, dev, **kw)
    xh = sa.ramp_x(m.n_cols) if x is None else x
    xd = torch.from_numpy(xh).to(dev)
    y = torch.full((max(m.n_rows, 1),), float("nan"), dtype=torch.float64, device=dev)
    dm.run(xd, y)
    torch.cuda.synchronize()
    return y.cpu().numpy()[: m.n_rows], xh, dm


def assert_parity(m, y, x, y_ref=None, rel=1e-6):
    if y_ref is None:
        y_ref = oracle.file_order_spmv(m.n_rows, m.row, m.col, m.val, x)
    bad = oracle.parity(y, y_ref, m.row, m.col, m.val, x, m.n_rows, rel=rel)
    assert bad.size == 0, f"{bad.size} bad rows, first {bad[:5]}: got {y[bad[:5]]} want {y_ref[bad[:5]]}"


@pytest.mark.parametrize("fmt,kw", FMT_PARAMS, ids=IDS)
@pytest.mark.parametrize("name", CASES)
def test_golden_fixtures(torch_dev, name, fmt, kw):
    torch, dev = torch_dev
    m = sa.read_mtx(GOLDEN / f"{name}.mtx")
    y, x, _ = run_fmt(torch, dev, m, fmt, **kw)
    assert_parity(m, y, x)
    assert_parity(m, y, x, y_ref=np.load(GOLDEN / f"{name}.y.npy"))


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("fmt,kw", FMT_PARAMS, ids=IDS)
def test_cantlike(torch_dev, fmt, kw, mode):
    """The cant-like stand-in (real cant.mtx is an LFS pointer): row-sorted,
    column-major and symmetric-lower (literal) entry orders."""
    torch, dev = torch_dev
    m = sa.gen_cantlike(mode)
    y, x, _ = run_fmt(torch, dev, m, fmt, **kw)
    assert_parity(m, y, x)


@pytest.mark.parametrize("fmt", ["coo", "csr", "sell", "cmrs", "ell", "sell16"])
def test_cantlike_batch_random_x(torch_dev, fmt):
    """The bench workload (block-diagonal batch of cant-like copies) with a
    random x instead of the ramp."""
    torch, dev = torch_dev
    m = sa.gen_cantlike(0, copies=4)
    x = np.random.default_rng(1).uniform(-1, 1, m.n_cols)
    y, x, _ = run_fmt(torch, dev, m, fmt, x=x)
    assert_parity(m, y, x)


@pytest.mark.parametrize("fmt,kw", [("coo", {}), ("csr", {}), ("csr", {"variant": 2}), ("csr", {"variant": 4}),
                                    ("csr", {"variant": 1}), ("sell", {}), ("cmrs", {}), ("hyb", {}),
                                    ("sell", {"split": 0}), ("sell", {"split": 256, "ki": 2}),
                                    ("sell", {"split": 64, "ki": 1, "xwin": False}),
                                    ("sell", {"sigma": 65536, "ki": 2}),
                                    ("csr", {"variant": 4, "hot": 4096}), ("csr", {"variant": 4, "hot": 0}),
                                    ("cmrs", {"cmrs_variant": 0}), ("cmrs", {"cmrs_variant": 1, "h": 1}),
                                    ("cmrs", {"cmrs_variant": 1, "h": 64})])
def test_rmat_skewed(torch_dev, fmt, kw):
    """R-MAT 1e6 rows / 1e7 entries: empty rows, rows of thousands of entries."""
    torch, dev = torch_dev
    m = sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=1)
    y, x, _ = run_fmt(torch, dev, m, fmt, **kw)
    assert_parity(m, y, x)


def test_ell_refuses_rmat_padding(torch_dev):
    torch, dev = torch_dev
    m = sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=1)
    with pytest.raises(sa.SpmvError):
        sa.to_device(m, "ell", dev)


@pytest.mark.parametrize("fmt,kw", [("coo", {}), ("csr", {}), ("sell", {}), ("cmrs", {"h": 8}),
                                    ("cmrs", {"h": 32}), ("csr", {"lanes": 64}), ("csr", {"variant": 2}),
                                    ("csr", {"lanes": 2, "variant": 2}), ("csr", {"variant": 1}),
                                    ("csr", {"lanes": 2, "variant": 1})])
def test_ragged_long_rows(torch_dev, fmt, kw):
    torch, dev = torch_dev
    m = sa.gen_random(20_000, 50_000, 0, 2_000, seed=21)
    y, x, _ = run_fmt(torch, dev, m, fmt, **kw)
    assert_parity(m, y, x)


@pytest.mark.parametrize("fmt,kw", [(f, {}) for f in sa.ALL_FORMATS] + [("csr", {"variant": 4}), ("csr", {"variant": 1}),
                                                                     ("sell", {"split": 2}), ("cmrs", {"cmrs_variant": 1})])
def test_bitwise_reproducible(torch_dev, fmt, kw):
    """No atomics anywhere: two launches give identical bits (the reference
    COO's CAS-atomic order is nondeterministic)."""
    torch, dev = torch_dev
    m = sa.gen_random(30_000, 30_000, 0, 300, seed=5)
    dm = sa.to_device(m, fmt, dev, **kw)
    x = torch.from_numpy(np.random.default_rng(2).uniform(-1, 1, m.n_cols)).to(dev)
    y1 = torch.empty(m.n_rows, dtype=torch.float64, device=dev)
    y2 = torch.full_like(y1, float("nan"))
    dm.run(x, y1)
    dm.run(x, y2)
    torch.cuda.synchronize()
    assert torch.equal(y1.view(torch.int64), y2.view(torch.int64))


@pytest.mark.parametrize("lanes", [2, 4, 16])
def test_csr_staged_variants_bit_identical(torch_dev, lanes):
    """Variants 2 and 3 and the x-window kernel form the same products and
    sum each row in the same order, so their y agree bit for bit."""
    torch, dev = torch_dev
    m = sa.gen_random(40_000, 40_000, 0, 700, seed=9)
    x = torch.from_numpy(np.random.default_rng(4).uniform(-1, 1, m.n_cols)).to(dev)
    ys = []
    for v, xw in ((2, False), (3, False), (3, True)):
        dm = sa.to_device(m, "csr", dev, lanes=lanes, variant=v, xwin=xw)
        y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
        dm.run(x, y)
        ys.append(y)
    torch.cuda.synchronize()
    assert torch.equal(ys[0].view(torch.int64), ys[1].view(torch.int64))
    assert torch.equal(ys[0].view(torch.int64), ys[2].view(torch.int64))


@pytest.mark.parametrize("case", ["cantlike", "rmat", "ragged"])
def test_csr16_bit_identical_to_csr(torch_dev, case):
    """Compressed 16-bit column indices decode to CSR's columns, so the
    staged kernel gives CSR variant 3's bits (escaped blocks included)."""
    torch, dev = torch_dev
    if case == "cantlike":
        m = sa.gen_cantlike(1, copies=2)
    elif case == "rmat":
        m = sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=1)
    else:
        m = sa.gen_random(20_000, 300_000, 0, 2_000, seed=21)
    x = torch.from_numpy(np.random.default_rng(6).uniform(-1, 1, m.n_cols)).to(dev)
    ys = []
    for fmt, kw in (("csr", {"variant": 3, "lanes": 4}), ("csr16", {"lanes": 4, "csr16_max_escape": None})):
        dm = sa.to_device(m, fmt, dev, **kw)
        y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
        dm.run(x, y)
        ys.append(y)
    torch.cuda.synchronize()
    assert torch.equal(ys[0].view(torch.int64), ys[1].view(torch.int64))
    assert_parity(m, ys[1].cpu().numpy(), x.cpu().numpy())


@pytest.mark.parametrize("fmt,kw", [("csr", {"variant": 3}), ("csr", {"variant": 3, "xwin": True}), ("csr", {"variant": 2}),
                                    ("sell", {"ki": 1}), ("sell", {"ki": 2}), ("ell", {"ki": 1}), ("ell", {"ki": 2})])
def test_stream_load_policy_same_bits(torch_dev, fmt, kw):
    """The stream_nt switch (spmv_set_option) only changes the cache policy
    of the matrix loads."""
    torch, dev = torch_dev
    m = sa.gen_cantlike(0, copies=2)
    x = torch.from_numpy(np.random.default_rng(3).uniform(-1, 1, m.n_cols)).to(dev)
    dm = sa.to_device(m, fmt, dev, **kw)
    out = []
    try:
        for nt in (0, 1):
            sa.set_option("stream_nt", nt)
            y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
            dm.run(x, y)
            torch.cuda.synchronize()
            out.append(y)
    finally:
        sa.set_option("stream_nt", None)
    assert torch.equal(out[0].view(torch.int64), out[1].view(torch.int64))
    assert_parity(m, out[1].cpu().numpy(), x.cpu().numpy())


@pytest.fixture(scope="module")
def rmat_full():
    m = sa.gen_rmat()
    x = sa.ramp_x(m.n_cols)
    return m, x, oracle.file_order_spmv(m.n_rows, m.row, m.col, m.val, x)


@pytest.mark.parametrize("fmt", sa.FORMATS + ("csrg",))
def test_linearity_and_checksum_full_rmat(torch_dev, rmat_full, fmt):
    """BASELINE.json configs[3] at full size (1e7 rows, 1e8 entries):
    A(2u - 3v) == 2Au - 3Av, and with x = ones sum(y) == sum(values).
    ELL is skipped (padding factor ~1e4, reported N/A by the builders)."""
    if fmt == "ell":
        pytest.skip("ELL not applicable to R-MAT (padding)")
    torch, dev = torch_dev
    m, x, y_ref = rmat_full
    dm = sa.to_device(m, fmt, dev)
    n = m.n_cols
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    u = torch.rand(n, dtype=torch.float64, device=dev, generator=g)
    v = torch.rand(n, dtype=torch.float64, device=dev, generator=g)
    yu, yv, yw = (torch.empty(m.n_rows, dtype=torch.float64, device=dev) for _ in range(3))
    dm.run(u, yu)
    dm.run(v, yv)
    dm.run(2 * u - 3 * v, yw)
    ones = torch.ones(n, dtype=torch.float64, device=dev)
    ys = torch.empty(m.n_rows, dtype=torch.float64, device=dev)
    dm.run(ones, ys)
    torch.cuda.synchronize()
    atol = 1e-10 * float((yu.abs() + yv.abs()).max()) * 3 + 1e-12
    assert float((yw - (2 * yu - 3 * yv)).abs().max()) <= atol
    total = float(np.sum(m.val))
    assert abs(float(ys.sum()) - total) <= 1e-8 * float(np.abs(m.val).sum())
    # and against the oracle at full size, x = ramp
    y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    dm.run(torch.from_numpy(x).to(dev), y)
    assert_parity(m, y.cpu().numpy(), x, y_ref=y_ref)


@pytest.fixture(scope="module")
def rmat_bench_layout(rmat_full):
    """bench.py's configs[3] layout, built by bench's own code
    (bench.rmat_layout: columns relabelled by degree, ties by first row,
    rows in new-column order, x' = x[order]) as the whole-matrix shard
    bench.rmat_strong / rmat_per_format run (rows in CSR order)."""
    import argparse

    import bench

    m, x, y_ref = rmat_full
    ptr, col, val = sa.csr_from_coo(m)
    args = argparse.Namespace(relabel="yes", relabel_ties="first", format="csr", lanes=0, variant=0, ki=0, C=64,
                              sigma=0, h=8, workload="cant")
    col2, xh, hot, _, order = bench.rmat_layout(args, m.n_rows, ptr, col, val)
    loc = sa.Coo(m.n_rows, m.n_cols, np.repeat(np.arange(m.n_rows, dtype=np.int32), np.diff(ptr)), col2, val)
    return args, loc, xh, hot, order


@pytest.mark.parametrize("fmt", sa.ALL_FORMATS)
def test_rmat_bench_layout_every_format(torch_dev, rmat_full, rmat_bench_layout, fmt):
    """configs[3] at full size (1e7 rows, 1e8 entries) in
    exactly the layout and with exactly the to_device keywords bench.py
    times (bench.rmat_fmt_kwargs), every format, against the oracle's
    file-order sum of the ORIGINAL matrix on the ORIGINAL x (the relabel and
    the row sort change the summation order: the parity rule, not bits).
    ELL, CSR16 and SELL16 are refused (padding / 16-bit windows), as the
    bench reports them N/A; csrf32 is checked against the oracle on its
    fp32-rounded values."""
    import bench

    torch, dev = torch_dev
    m, x, y_ref = rmat_full
    args, loc, xh, hot, order = rmat_bench_layout
    assert np.array_equal(xh, x[order])
    kw = bench.rmat_fmt_kwargs(args, fmt, hot)
    if fmt in ("ell", "csr16", "sell16"):
        with pytest.raises(sa.SpmvError):
            sa.to_device(loc, fmt, dev, **kw)
        return
    dm = sa.to_device(loc, fmt, dev, **kw)
    y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    dm.run(torch.from_numpy(xh).to(dev), y)
    torch.cuda.synchronize()
    if fmt == "csrf32":
        v32 = m.val.astype(np.float32).astype(np.float64)
        assert_parity(sa.Coo(m.n_rows, m.n_cols, m.row, m.col, v32), y.cpu().numpy(), x,
                      y_ref=oracle.file_order_spmv(m.n_rows, m.row, m.col, v32, x))
    else:
        assert_parity(m, y.cpu().numpy(), x, y_ref=y_ref)
    if fmt == "csr":  # the kernel bench's rmat_strong reports
        assert dm.kernel == "csr_tiled_kernel" and dm.params["H"] == 0 and dm.params["big_tiles"] > 0


def test_banded_shard_full_parity(torch_dev):
    """BASELINE.json configs[4]: one of 8 row shards of the 1e8-row banded
    matrix (1.25e7 rows, 2e8 entries) in CSR and SELL, every row checked by
    the parity rule against the host generator's entries, with x[j] = j and
    with a random x (a wrong column index changes y; with x = 1 it would
    not)."""
    torch, dev = torch_dev
    n = 100_000_000
    lo, hi = 3 * n // 8, 4 * n // 8
    ptr, col, val = sa.gen_banded_csr(n, lo, hi)
    rows = hi - lo
    m = sa.Coo(rows, n, np.repeat(np.arange(rows, dtype=np.int32), 16), col, val)
    c2, v2 = col.reshape(-1, 16), val.reshape(-1, 16)
    xs = {"ramp": sa.ramp_x(n), "random": np.random.default_rng(11).uniform(-1.0, 1.0, n)}
    for name, xh in xs.items():
        g = xh[c2]
        ref = np.zeros(rows)
        for e in range(16):  # file order
            ref += v2[:, e] * g[:, e]
        scale = np.maximum(np.abs(ref), np.sum(np.abs(v2 * g), axis=1))
        del g
        x = torch.from_numpy(xh).to(dev)
        for fmt in ("csr", "sell"):
            dm = sa.to_device(m, fmt, dev)
            y = torch.full((rows,), float("nan"), dtype=torch.float64, device=dev)
            dm.run(x, y)
            torch.cuda.synchronize()
            bad = np.abs(y.cpu().numpy() - ref) > 1e-6 * scale
            assert not bad.any(), (name, fmt, np.nonzero(bad)[0][:5])
            del dm


@pytest.mark.parametrize("fmt", ["csr", "sell"])
def test_banded_full_matrix_sampled_rows(torch_dev, fmt):
    """The whole 1e8-row / 1.6e9-entry banded matrix generated in HBM (as
    bench.py's banded_strong at one GPU): value offsets run to 12.8 GB, past
    2^31 and 2^32 bytes.  Sampled rows (first / last 512, around the 2-, 4-
    and 8-way cuts, past the 2^31..2^33-byte offsets, 4,096 spread) checked
    against the host generator with x[j] = j (bench.banded_check)."""
    torch, dev = torch_dev
    from bench import banded_check

    n = 100_000_000
    dm = sa.banded_to_device(n, fmt, dev, 0, n, **({"ki": 1} if fmt == "sell" else {}))
    x = torch.from_numpy(sa.ramp_x(n)).to(dev)
    y = torch.full((n,), float("nan"), dtype=torch.float64, device=dev)
    dm.run(x, y)
    torch.cuda.synchronize()
    k, bad = banded_check(n, 0, n, y)
    assert k > 6000 and bad is None, (k, bad)
    del dm, x, y
    torch.cuda.empty_cache()


def test_nondefault_stream(torch_dev):
    torch, dev = torch_dev
    m = sa.gen_cantlike(0)
    dm = sa.to_device(m, "sell", dev)
    x = torch.from_numpy(sa.ramp_x(m.n_cols)).to(dev)
    y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        dm.run(x, y, stream=s)
    s.synchronize()
    assert_parity(m, y.cpu().numpy(), x.cpu().numpy())


def test_bad_arguments_rejected(torch_dev):
    """Invalid configurations return the reference's OtherError (4) and
    launch nothing."""
    torch, dev = torch_dev
    L = sa.hip_lib()
    d = sa.Dims(10, 10, 5, 0, None)
    assert L.spmv_csr_run(d, None, None, None, None, None, 3) == sa.OTHER_ERROR
    assert L.spmv_ell_run(d, 4, 63, 1, None, None, None, None) == sa.OTHER_ERROR
    assert L.spmv_sell_run(d, 0, 1, 1, 1, None, None, None, None, None, None) == sa.OTHER_ERROR
    assert L.spmv_sell_run(d, 64, 1, 3, 1, None, None, None, None, None, None) == sa.OTHER_ERROR
    assert L.spmv_sell_run(d, 64, 100, 1, 1, None, None, None, None, None, None) == sa.OTHER_ERROR
    assert L.spmv_cmrs_run(d, 8, 7, None, None, None, None, None, None) == sa.OTHER_ERROR
    assert L.spmv_cmrs_run(d, 65, 1, None, None, None, None, None, None) == sa.OTHER_ERROR
    assert L.spmv_coo_run(d, None, None, None, None, None, None, 0) == sa.OTHER_ERROR
    assert b"workspace" in L.spmv_last_error()
    # zero rows: a successful no-op
    assert L.spmv_csr_run(sa.Dims(0, 0, 0, 0, None), None, None, None, None, None, 0) == 0


def test_flush_and_event_timer(torch_dev):
    torch, dev = torch_dev
    sa.flush_cache()
    torch.cuda.synchronize()
    assert "gfx950" in sa.device_name(0)


@pytest.mark.parametrize("layout", ["csr", "sell"])
def test_device_banded_generator_matches_host(torch_dev, layout):
    """spmv_gen_banded_device writes bit-identical entries to the host
    generator (configs[4] shards are generated on the GPU)."""
    torch, dev = torch_dev
    n, lo, hi = 1_000_003, 123_457, 456_789
    ptr, col, val = sa.gen_banded_csr(n, lo, hi)
    dm = sa.banded_to_device(n, layout, dev, lo, hi, C=64, ki=2)
    if layout == "csr":
        assert np.array_equal(dm.arrays["row_ptr"].cpu().numpy(), ptr)
        assert np.array_equal(dm.arrays["col"].cpu().numpy(), col)
        assert np.array_equal(dm.arrays["val"].cpu().numpy().view(np.uint64), val.view(np.uint64))
    else:
        m = sa.Coo(hi - lo, n, np.repeat(np.arange(hi - lo, dtype=np.int32), 16), col, val)
        s = sa.sell_build(m.n_rows, ptr, col, val, C=64, sigma=1024, ki=2)
        assert np.array_equal(dm.arrays["slice_ptr"].cpu().numpy(), s["slice_ptr"])
        assert np.array_equal(dm.arrays["perm"].cpu().numpy(), s["perm"])
        assert np.array_equal(dm.arrays["val"].cpu().numpy().view(np.uint64), s["val"].view(np.uint64))
        got_col = dm.arrays["col"].cpu().numpy()
        real = s["val"] != 0  # padding columns may differ (both are valid reads)
        assert np.array_equal(got_col[real], s["col"][real])
    x = torch.arange(n, dtype=torch.float64, device=dev)
    y = torch.full((hi - lo,), float("nan"), dtype=torch.float64, device=dev)
    dm.run(x, y)
    torch.cuda.synchronize()
    m = sa.Coo(hi - lo, n, np.repeat(np.arange(hi - lo, dtype=np.int32), 16), col, val)
    assert_parity(m, y.cpu().numpy(), np.arange(n, dtype=np.float64))


@pytest.mark.parametrize("case", ["cantlike", "rmat", "ragged", "banded"])
@pytest.mark.parametrize("ki", [1, 2])
def test_sell_xwin_bit_identical(torch_dev, case, ki):
    """The LDS x-window kernel reads the same x values in the same order as
    the global-gather kernel; workgroups whose window does not fit fall back
    to global gathers (R-MAT: all of them)."""
    torch, dev = torch_dev
    if case == "cantlike":
        m = sa.gen_cantlike(0, copies=16)  # >= 512 windows: 1024-slot workgroups
    elif case == "rmat":
        m = sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=1)
    elif case == "ragged":
        m = sa.gen_random(20_000, 20_000, 0, 700, seed=21)
    else:
        n = 600_000
        ptr, col, val = sa.gen_banded_csr(n, 0, n)
        row = np.repeat(np.arange(n, dtype=np.int32), np.diff(ptr))
        m = sa.Coo(n, n, row, col, val, False, "banded")
    x = torch.from_numpy(np.random.default_rng(8).uniform(-1, 1, m.n_cols)).to(dev)
    ys = []
    for xw in (False, True):
        dm = sa.to_device(m, "sell", dev, C=64, sigma=1024, ki=ki, xwin=xw)
        y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
        dm.run(x, y)
        ys.append(y)
        if xw and case in ("cantlike", "banded"):
            assert dm.params["xcap"] > 0
    torch.cuda.synchronize()
    assert torch.equal(ys[0].view(torch.int64), ys[1].view(torch.int64))
    assert_parity(m, ys[1].cpu().numpy(), x.cpu().numpy())


@pytest.mark.parametrize("case", ["cantlike", "cantlike16", "ragged", "ragged_wide"])
@pytest.mark.parametrize("ki", [1, 2])
def test_sell16_bit_identical_to_sell(torch_dev, case, ki):
    """SELL16 decodes the same columns and sums in the same order as the
    x-window SELL kernel of the same geometry (one cant-like copy: the
    small-matrix kernel; 16 copies: one sigma-window per workgroup)."""
    torch, dev = torch_dev
    if case == "cantlike":
        m = sa.gen_cantlike(0)
    elif case == "cantlike16":
        m = sa.gen_cantlike(1, copies=16)
    elif case == "ragged":
        m = sa.gen_random(20_000, 20_000, 0, 700, seed=21)
    else:  # columns up to 65,000 apart inside a workgroup: offsets near the 16-bit limit
        m = sa.gen_random(30_000, 65_000, 1, 40, seed=22)
    x = torch.from_numpy(np.random.default_rng(9).uniform(-1, 1, m.n_cols)).to(dev)
    ys = []
    for fmt in ("sell", "sell16"):
        dm = sa.to_device(m, fmt, dev, C=64, sigma=1024, ki=ki, xwin=True)
        y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
        dm.run(x, y)
        ys.append(y)
        if fmt == "sell16":
            assert "col" not in dm.arrays and dm.params["index16"] == 1
            assert dm.stored_bytes < 12 * dm.params["stored"]
    torch.cuda.synchronize()
    assert torch.equal(ys[0].view(torch.int64), ys[1].view(torch.int64))
    assert_parity(m, ys[1].cpu().numpy(), x.cpu().numpy())


@pytest.mark.parametrize("groups", [8, 32, 64])
def test_csrg_rmat(torch_dev, groups):
    """Column-grouped CSR on a skewed R-MAT (hub rows over many tiles, empty
    rows): parity with the oracle, same bits on a second run."""
    torch, dev = torch_dev
    m = sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=5)
    x = np.random.default_rng(12).uniform(-1, 1, m.n_cols)
    y, _, dm = run_fmt(torch, dev, m, "csrg", x=x, groups=groups)
    assert dm.params["n_pairs"] > m.n_rows // 4
    assert_parity(m, y, x)
    y2 = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    dm.run(torch.from_numpy(x).to(dev), y2)
    torch.cuda.synchronize()
    assert np.array_equal(y.view(np.int64), y2.cpu().numpy().view(np.int64))


def test_sell16_refuses_wide_windows(torch_dev):
    """A workgroup whose columns span more than 65,536 cannot hold 16-bit
    offsets: the fill refuses and writes nothing (the caller keeps SELL)."""
    torch, dev = torch_dev
    m = sa.gen_rmat(200_000, 2_000_000, scale=18, seed=3)
    with pytest.raises(sa.SpmvError, match="65,536"):
        sa.to_device(m, "sell16", dev, C=64, sigma=1024)
    with pytest.raises(sa.SpmvError, match="needs C = 64"):
        sa.to_device(sa.gen_cantlike(0), "sell16", dev, C=32, sigma=1024)


@pytest.mark.parametrize("case", ["cantlike", "rmat", "ragged", "fixtures"])
@pytest.mark.parametrize("lanes", [0, 2, 16])
def test_csr_xwin_bit_identical(torch_dev, case, lanes):
    """The LDS x-window CSR kernel gives variant 3's bits (row groups whose
    window does not fit gather from global memory)."""
    torch, dev = torch_dev
    if case == "cantlike":
        ms = [sa.gen_cantlike(2, copies=4)]
    elif case == "rmat":
        ms = [sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=1)]
    elif case == "ragged":
        ms = [sa.gen_random(20_000, 20_000, 0, 700, seed=21)]
    else:
        ms = [sa.read_mtx(GOLDEN / f"{c}.mtx") for c in CASES]
    for m in ms:
        if m.n_rows == 0:
            continue
        x = torch.from_numpy(np.random.default_rng(8).uniform(-1, 1, max(m.n_cols, 1))).to(dev)
        ys = []
        for xw in (False, True):
            dm = sa.to_device(m, "csr", dev, lanes=lanes, variant=3, xwin=xw)
            y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
            dm.run(x, y)
            ys.append(y)
            if xw and case == "cantlike":
                assert dm.params["xcap"] > 0
        torch.cuda.synchronize()
        assert torch.equal(ys[0].view(torch.int64), ys[1].view(torch.int64)), m.label
        assert_parity(m, ys[1].cpu().numpy(), x.cpu().numpy()[: m.n_cols])


@pytest.mark.parametrize("ki", [1, 2])
def test_ell_xwin_bit_identical(torch_dev, ki):
    torch, dev = torch_dev
    for m in (sa.gen_cantlike(0, copies=2), sa.gen_random(20_000, 20_000, 0, 70, seed=21)):
        x = torch.from_numpy(np.random.default_rng(8).uniform(-1, 1, m.n_cols)).to(dev)
        ys = []
        for xw in (False, True):
            dm = sa.to_device(m, "ell", dev, ki=ki, xwin=xw, ell_max_padding=None)
            y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
            dm.run(x, y)
            ys.append(y)
        torch.cuda.synchronize()
        assert torch.equal(ys[0].view(torch.int64), ys[1].view(torch.int64))
        assert_parity(m, ys[1].cpu().numpy(), x.cpu().numpy())


@pytest.mark.parametrize("case", ["cantlike", "rmat", "ragged", "fixtures"])
@pytest.mark.parametrize("fmt,kw", [("coo", {}), ("cmrs", {"h": 8, "cmrs_variant": 0}),
                                    ("cmrs", {"h": 1, "cmrs_variant": 0}), ("cmrs", {"h": 64, "cmrs_variant": 0})])
def test_coo_cmrs_xwin_bit_identical(torch_dev, case, fmt, kw):
    """COO / CMRS x windows in LDS: same products, same order as the global
    gathers, so y is bit-identical (windows too wide fall back per tile)."""
    torch, dev = torch_dev
    if case == "cantlike":
        ms = [sa.gen_cantlike(0, copies=2)]
    elif case == "rmat":
        ms = [sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=1)]
    elif case == "ragged":
        ms = [sa.gen_random(20_000, 50_000, 0, 2_000, seed=21)]
    else:
        ms = [sa.read_mtx(GOLDEN / f"{n}.mtx") for n in CASES]
    for m in ms:
        a = sa.to_device(m, fmt, dev, xwin=True, **kw)
        extra = {"coo_tail": False} if fmt == "coo" else {}  # the carry path: the same tiles and sums
        b = sa.to_device(m, fmt, dev, xwin=False, **kw, **extra)
        assert a.params["xwin"] and not b.params["xwin"]
        if case == "cantlike":
            assert a.params["xcap"] > 0
        x = torch.from_numpy(np.random.default_rng(4).uniform(-1, 1, m.n_cols)).to(dev)
        ya = torch.full((max(m.n_rows, 1),), float("nan"), dtype=torch.float64, device=dev)
        yb = torch.full_like(ya, float("nan"))
        a.run(x, ya)
        b.run(x, yb)
        torch.cuda.synchronize()
        assert torch.equal(ya.view(torch.int64), yb.view(torch.int64))
        assert_parity(m, ya.cpu().numpy()[: m.n_rows], x.cpu().numpy())


@pytest.mark.parametrize("H", [1, 4096, 1 << 16])
def test_csr_hot_bit_identical(torch_dev, H):
    """Hot-column table (spmv_csr_run_tiled_hot): the same products in the
    same order as the tiled kernel on the original columns."""
    torch, dev = torch_dev
    m = sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=1)
    a = sa.to_device(m, "csr", dev, variant=4, hot=H)
    b = sa.to_device(m, "csr", dev, variant=4, hot=0)
    assert a.params["H"] == H and b.params["H"] == 0
    x = torch.from_numpy(np.random.default_rng(6).uniform(-1, 1, m.n_cols)).to(dev)
    ya = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    yb = torch.full_like(ya, float("nan"))
    yc = torch.full_like(ya, float("nan"))
    a.run(x, ya)
    b.run(x, yb)
    # and without the build-once tile plan (the per-run pre-pass)
    bb = b.arrays
    ws = torch.empty(sa.hip_lib().spmv_csr_tiled_ws_bytes(m.n_rows, m.nnz), dtype=torch.uint8, device=dev)
    rc = sa.hip_lib().spmv_csr_run_tiled(b.dims(), sa._ptr(bb["row_ptr"]), sa._ptr(bb["col"]), sa._ptr(bb["val"]),
                                         sa._ptr(x), sa._ptr(yc), sa._ptr(ws), ws.numel())
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.equal(ya.view(torch.int64), yb.view(torch.int64))
    assert torch.equal(yc.view(torch.int64), yb.view(torch.int64))
    assert_parity(m, ya.cpu().numpy(), x.cpu().numpy())


@pytest.mark.parametrize("case", ["rmat_odd", "empty_runs", "one_row"])
def test_csr_tiled_edge_tiles(torch_dev, case):
    """The tiled kernel's carry and offset staging at the edges: an odd entry
    count (the array's last entry loaded singly), tiles owning more rows than
    the LDS offset table, a single row over every tile; the tiled kernel,
    with and without the hot table, against the oracle."""
    torch, dev = torch_dev
    if case == "rmat_odd":
        m = sa.gen_rmat(300_000, 2_999_999, scale=19, seed=4)
    elif case == "empty_runs":
        m, _ = _empty_run_matrix()
    else:
        rng = np.random.default_rng(5)
        m = sa.Coo(3, 5_000, np.full(20_001, 1, np.int32), rng.integers(0, 5_000, 20_001).astype(np.int32),
                   rng.uniform(-1, 1, 20_001))
    x = np.random.default_rng(13).uniform(-1, 1, m.n_cols)
    for H in (0, 4096):
        y, _, dm = run_fmt(torch, dev, m, "csr", x=x, variant=4, hot=H)
        assert dm.params["variant"] == 4
        assert_parity(m, y, x)


def _empty_run_matrix(seed=11):
    """Nonempty rows scattered among long runs of empty rows (a tile of the
    tiled CSR kernel then owns thousands of rows), one 20000-entry row that
    runs over several tiles right after an empty run, trailing empty rows."""
    rng = np.random.default_rng(seed)
    n, nc = 400_000, 50_000
    rows = np.sort(rng.choice(np.arange(1, n - 5000), 4000, replace=False))
    lens = rng.integers(2, 20, rows.size)
    lens[rows.size // 2] = 20_000
    r = np.repeat(rows, lens).astype(np.int32)
    c = rng.integers(0, nc, r.size).astype(np.int32)
    v = rng.uniform(-1, 1, r.size)
    return sa.Coo(n, nc, r, c, v), rows


@pytest.mark.parametrize("bigplan", [True, False])
@pytest.mark.parametrize("H", [0, 1024])
def test_csr_tiled_empty_row_runs(torch_dev, H, bigplan):
    """Rows a tile owns past its 1024-entry LDS offset table: with the
    big-tile plan (default) the tile sums only its listed rows and writes
    zeros from a bitmap, without it reads row_ptr from global memory
    (csr_tiled_kernel, rp_lds false); either way the same bits as the
    compacted matrix (3 empty rows after each nonempty one, so the same
    lanes per row and every row staged by its tile: the same entries in the
    same tiles), zeros for empty rows."""
    torch, dev = torch_dev
    m, rows = _empty_run_matrix()
    inv = np.zeros(m.n_rows, np.int32)
    inv[rows] = 4 * np.arange(rows.size, dtype=np.int32)
    mc = sa.Coo(4 * rows.size, m.n_cols, inv[m.row], m.col, m.val)
    x = torch.from_numpy(np.random.default_rng(3).uniform(-1, 1, m.n_cols)).to(dev)
    a = sa.to_device(m, "csr", dev, variant=4, hot=H, bigplan=bigplan)
    assert (a.params["big_tiles"] > 0) == bigplan and (not bigplan or a.params["big_tiles"] > 10)
    c = sa.to_device(mc, "csr", dev, variant=4, hot=H)
    ya = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    yc = torch.full((mc.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    a.run(x, ya)
    c.run(x, yc)
    yp = torch.full_like(ya, float("nan"))
    if H == 0:  # and without the build-once tile plan
        aa = a.arrays
        ws = torch.empty(sa.hip_lib().spmv_csr_tiled_ws_bytes(m.n_rows, m.nnz), dtype=torch.uint8, device=dev)
        rc = sa.hip_lib().spmv_csr_run_tiled(a.dims(), sa._ptr(aa["row_ptr"]), sa._ptr(aa["col"]),
                                             sa._ptr(aa["val"]), sa._ptr(x), sa._ptr(yp), sa._ptr(ws), ws.numel())
        assert rc == 0
    torch.cuda.synchronize()
    idx = torch.from_numpy(rows.astype(np.int64)).to(dev)
    assert torch.equal(ya[idx].view(torch.int64), yc[::4].view(torch.int64))
    mask = torch.ones(m.n_rows, dtype=torch.bool, device=dev)
    mask[idx] = False
    assert bool((ya[mask] == 0).all())
    if H == 0:
        assert torch.equal(yp.view(torch.int64), ya.view(torch.int64))
    assert_parity(m, ya.cpu().numpy(), x.cpu().numpy())


@pytest.mark.parametrize("fmt,kw", [("coo", {}), ("cmrs", {"cmrs_variant": 1}), ("cmrs", {"cmrs_variant": 1, "h": 32}),
                                    ("sell", {"xwin": False}), ("sell", {"sigma": 1 << 24, "ki": 2, "xwin": False}),
                                    ("sell", {"split": 0, "xwin": False}), ("hyb", {}), ("hyb", {"ki": 1})])
@pytest.mark.parametrize("H", [1, 4096])
def test_coo_cmrs_hot_bit_identical(torch_dev, fmt, kw, H):
    """COO / tiled CMRS / SELL / HYB over the hot-column table: the same
    products in the same order as over the original columns.  COO is also
    compared bitwise with a one-column table, and with the plain carry pass
    (spmv_coo_run: the same 512-entry tiles below a mean row of 96)."""
    torch, dev = torch_dev
    m = sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=1)
    a = sa.to_device(m, fmt, dev, hot=H, **kw)
    H_ref = (2 if H == 1 else 1) if fmt == "coo" else 0
    b = sa.to_device(m, fmt, dev, hot=H_ref, **kw)
    assert a.params["H"] == H and b.params["H"] == H_ref
    x = torch.from_numpy(np.random.default_rng(7).uniform(-1, 1, m.n_cols)).to(dev)
    ya = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    yb = torch.full_like(ya, float("nan"))
    a.run(x, ya)
    b.run(x, yb)
    torch.cuda.synchronize()
    assert torch.equal(ya.view(torch.int64), yb.view(torch.int64))
    assert_parity(m, ya.cpu().numpy(), x.cpu().numpy())
    if fmt == "coo":  # and the plain COO's carry pass: same tiles, same bits
        c = sa.to_device(m, fmt, dev, hot=0, **kw)
        assert not c.params["single_pass"]  # R-MAT rows run past 80 entries: the carry pass
        yc = torch.full_like(ya, float("nan"))
        c.run(x, yc)
        torch.cuda.synchronize()
        assert torch.equal(ya.view(torch.int64), yc.view(torch.int64))


def test_csr16_refuses_escape_heavy_matrix(torch_dev):
    """R-MAT columns spread over 1e6 ids: most 64-entry blocks need 32-bit
    escapes, so CSR16 is reported not applicable (like ELL's padding cap)."""
    torch, dev = torch_dev
    m = sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=1)
    with pytest.raises(sa.SpmvError):
        sa.to_device(m, "csr16", dev)


@pytest.mark.parametrize("case", ["cantlike", "ragged", "fixtures"])
def test_csrf32_equals_csr_on_rounded_values(torch_dev, case):
    """CSR with fp32 values widens each value before the fp64 product: y is
    bit-identical to the fp64 CSR x-window kernel on the fp32-rounded
    matrix, and within the 1e-6 criterion of the exact one."""
    torch, dev = torch_dev
    if case == "cantlike":
        ms = [sa.gen_cantlike(0, copies=2)]
    elif case == "ragged":
        ms = [sa.gen_random(20_000, 50_000, 0, 2_000, seed=21)]
    else:
        ms = [sa.read_mtx(GOLDEN / f"{n}.mtx") for n in CASES]
    for m in ms:
        m32 = sa.Coo(m.n_rows, m.n_cols, m.row, m.col, m.val.astype(np.float32).astype(np.float64))
        a = sa.to_device(m, "csrf32", dev)
        b = sa.to_device(m32, "csr", dev, variant=3, xwin=True)
        assert a.stored_bytes < b.stored_bytes or m.nnz == 0
        x = torch.from_numpy(np.random.default_rng(9).uniform(-1, 1, m.n_cols)).to(dev)
        ya = torch.full((max(m.n_rows, 1),), float("nan"), dtype=torch.float64, device=dev)
        yb = torch.full_like(ya, float("nan"))
        a.run(x, ya)
        b.run(x, yb)
        torch.cuda.synchronize()
        assert torch.equal(ya.view(torch.int64), yb.view(torch.int64))
        assert_parity(m, ya.cpu().numpy()[: m.n_rows], x.cpu().numpy())


@pytest.mark.parametrize("H", [0, 4096])
def test_csrf32_tiled_on_skewed_rows(torch_dev, H):
    """Skewed rows: the fp32-value CSR runs the entry-balanced kernel (with
    or without the hot table) and equals the fp64 tiled CSR on the rounded
    values bit for bit."""
    torch, dev = torch_dev
    m = sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=1)
    m32 = sa.Coo(m.n_rows, m.n_cols, m.row, m.col, m.val.astype(np.float32).astype(np.float64))
    a = sa.to_device(m, "csrf32", dev, hot=H)
    b = sa.to_device(m32, "csr", dev, variant=4, hot=H)
    assert a.params["variant"] == 4 and a.params["H"] == H
    x = torch.from_numpy(np.random.default_rng(10).uniform(-1, 1, m.n_cols)).to(dev)
    ya = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    yb = torch.full_like(ya, float("nan"))
    a.run(x, ya)
    b.run(x, yb)
    torch.cuda.synchronize()
    assert torch.equal(ya.view(torch.int64), yb.view(torch.int64))
    assert_parity(m, ya.cpu().numpy(), x.cpu().numpy())


def _xstream_cases(case):
    if case == "cantlike":
        return [sa.gen_cantlike(0, copies=2)]
    if case == "ragged":  # random columns: most row groups span more than the ring
        return [sa.gen_random(20_000, 50_000, 0, 2_000, seed=21)]
    if case == "empty_runs":
        return [_empty_run_matrix()[0]]
    if case == "shuffled_bands":
        # banded blocks in shuffled order: column ranges jump up and down
        # between neighbouring row groups (both ends of the ring update), and
        # some jumps leave no overlap at all
        n, blk = 40_000, 500
        rng = np.random.default_rng(5)
        perm = rng.permutation(n // blk)
        rows, cols = [], []
        for b, pb in enumerate(perm):
            r = np.repeat(np.arange(b * blk, (b + 1) * blk), 9)
            c = (np.repeat(np.arange(pb * blk, (pb + 1) * blk), 9) + np.tile(np.arange(-4, 5), blk)) % n
            rows.append(r)
            cols.append(c)
        r, c = np.concatenate(rows), np.concatenate(cols)
        return [sa.Coo(n, n, r.astype(np.int32), c.astype(np.int32), rng.uniform(-1, 1, r.size))]
    return [sa.read_mtx(GOLDEN / f"{n}.mtx") for n in CASES]


@pytest.mark.parametrize("case", ["cantlike", "ragged", "fixtures", "empty_runs", "shuffled_bands"])
def test_csr_xwin_window_sizes(torch_dev, case):
    """x windows of 1 row group up to 1024 rows (the MODE 0 / MODE 3 load
    schedules, windows that fit LDS and windows that gather globally) form
    staged_group's chunks and sums: the same bits as variant 3 at every lane
    width, also where column ranges jump between neighbouring groups."""
    torch, dev = torch_dev
    for m in _xstream_cases(case):
        if m.n_rows == 0:
            continue
        x = torch.from_numpy(np.random.default_rng(12).uniform(-1, 1, max(m.n_cols, 1))).to(dev)
        for lanes in (2, 4, 16, 64):
            ref = sa.to_device(m, "csr", dev, lanes=lanes, variant=3, xwin=False)
            y0 = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
            ref.run(x, y0)
            for rows in (1, 128, 1024):
                dm = sa.to_device(m, "csr", dev, lanes=lanes, variant=3, xwin=True, xwin_rows=rows)
                y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
                dm.run(x, y)
                dm.run(x, y)  # twice: nothing carried between runs
                torch.cuda.synchronize()
                assert torch.equal(y.view(torch.int64), y0.view(torch.int64)), (m.label, lanes, rows)
        assert_parity(m, y0.cpu().numpy(), x.cpu().numpy()[: m.n_cols])


@pytest.mark.parametrize("n_rows", [1, 64, 65, 3 * 64 + 5, 5 * 64, 17 * 64 + 1, 1000 * 64 - 7])
@pytest.mark.parametrize("sigma", [1, 64, 128, 1024])
@pytest.mark.parametrize("ki", [1, 2])
def test_sell_small_kernel_shapes(torch_dev, n_rows, sigma, ki):
    """The small-matrix SELL kernel (4 slices x 2 waves per workgroup, one
    shared x window): slice counts that are not multiples of 4, σ windows
    of 1..16 slices (a workgroup's 4 slices may span two σ windows), rows
    of 0..300 entries; the x-window run must give the same bits as the
    global-gather run and pass the parity rule."""
    torch, dev = torch_dev
    m = sa.gen_random(n_rows, 3 * n_rows + 50, 0, 300 if n_rows < 2000 else 90, seed=n_rows + sigma)
    x = torch.from_numpy(np.random.default_rng(n_rows).uniform(-1, 1, m.n_cols)).to(dev)
    ys = []
    for xw in (False, True):
        dm = sa.to_device(m, "sell", dev, C=64, sigma=sigma, ki=ki, xwin=xw)
        y = torch.full((max(m.n_rows, 1),), float("nan"), dtype=torch.float64, device=dev)
        dm.run(x, y)
        ys.append(y)
    torch.cuda.synchronize()
    assert torch.equal(ys[0].view(torch.int64), ys[1].view(torch.int64))
    assert_parity(m, ys[1].cpu().numpy()[: m.n_rows], x.cpu().numpy())


def test_sell_small_kernel_window_fallback(torch_dev):
    """Slices whose shared window exceeds the LDS cap gather from global
    memory; same bits either way."""
    torch, dev = torch_dev
    m = sa.gen_random(900 * 64, 20_000_000, 10, 60, seed=5)  # columns spread over 2e7: no window fits
    x = torch.from_numpy(np.random.default_rng(3).uniform(-1, 1, m.n_cols)).to(dev)
    ys = []
    for xw in (False, True):
        dm = sa.to_device(m, "sell", dev, xwin=xw)
        y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
        dm.run(x, y)
        ys.append(y)
        if xw:
            assert dm.params["xcap"] == 0
    torch.cuda.synchronize()
    assert torch.equal(ys[0].view(torch.int64), ys[1].view(torch.int64))
    assert_parity(m, ys[1].cpu().numpy(), x.cpu().numpy())


def test_sell_auto_ki_rule(torch_dev):
    """spmv_sell_auto_ki: k-interleave 2 for matrices the small-matrix kernel
    runs (one cant-like copy), 1 for the σ-window kernel (the 32-copy batch)."""
    lib = sa.hip_lib()
    assert lib.spmv_sell_auto_ki(62_451, 64) == 2
    assert lib.spmv_sell_auto_ki(32 * 62_451, 64) == 1
    assert lib.spmv_sell_auto_ki(62_451, 32) == 1  # C != 64: no small kernel
    assert sa.to_device(sa.gen_cantlike(0), "sell", torch_dev[1]).params["ki"] == 2


@pytest.mark.parametrize("ki", [1, 2])
@pytest.mark.parametrize("case", ["cantlike", "ragged", "few_slices"])
def test_sell16_head_same_bits(torch_dev, ki, case):
    """SELL16's head copy (small matrices: every wave's first slot groups at
    computed addresses, spmv_sell16_head_fill) gives the bits of the run
    without it; waves with fewer groups than the head holds read padding
    they never add."""
    torch, dev = torch_dev
    if case == "cantlike":
        m = sa.gen_cantlike(2)
    elif case == "ragged":
        m = sa.gen_random(30_000, 20_000, 0, 150, seed=23)
    else:  # 3 slices, rows of 0-5 entries: most waves have no groups or one
        m = sa.gen_random(150, 400, 0, 5, seed=24)
    x = torch.from_numpy(np.random.default_rng(19).uniform(-1, 1, m.n_cols)).to(dev)
    ys = []
    for head in (False, True):
        dm = sa.to_device(m, "sell16", dev, C=64, sigma=1024, ki=ki, head=head)
        assert bool(dm.params["head"]) == head
        y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
        dm.run(x, y)
        torch.cuda.synchronize()
        ys.append(y)
    assert torch.equal(ys[0].view(torch.int64), ys[1].view(torch.int64))
    assert_parity(m, ys[1].cpu().numpy(), x.cpu().numpy())

@pytest.mark.parametrize("ki", [1, 2])
@pytest.mark.parametrize("case", ["cantlike", "ragged", "few_slices", "inf_x"])
def test_sell_int32_head_same_bits(torch_dev, ki, case):
    """The head for int32 SELL (sell_head=True, small matrices) gives the
    bits of the x-window run without it, also for an x holding Inf."""
    torch, dev = torch_dev
    if case == "cantlike":
        m = sa.gen_cantlike(2)
    elif case == "ragged":
        m = sa.gen_random(30_000, 20_000, 0, 150, seed=23)
    else:
        m = sa.gen_random(150, 400, 0, 5, seed=24)
    xh = np.random.default_rng(19).uniform(-1, 1, m.n_cols)
    if case == "inf_x":
        xh[::37] = np.inf
    x = torch.from_numpy(xh).to(dev)
    ys = []
    for head in (False, True):
        dm = sa.to_device(m, "sell", dev, C=64, sigma=1024, ki=ki, sell_head=head)
        assert bool(dm.params["head"]) == head
        y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
        dm.run(x, y)
        torch.cuda.synchronize()
        ys.append(y)
    assert torch.equal(ys[0].view(torch.int64), ys[1].view(torch.int64))
    if case != "inf_x":
        assert_parity(m, ys[1].cpu().numpy(), x.cpu().numpy())


@pytest.mark.parametrize("ki", [1, 2])
def test_sell16_head_same_bits_nonfinite_x(torch_dev, ki):
    """The head pads a wave's unused groups with its own first group (as the
    run without a head re-reads it), so even an x holding Inf gives the same
    bits (NaN where 0·Inf enters a row) with and without the head
    (padding with offset 0 read an unrelated x entry)."""
    torch, dev = torch_dev
    m = sa.gen_random(150, 400, 0, 5, seed=24)  # most waves have no groups or one
    xh = np.random.default_rng(7).uniform(-1, 1, m.n_cols)
    xh[::37] = np.inf
    x = torch.from_numpy(xh).to(dev)
    ys = []
    for head in (False, True):
        dm = sa.to_device(m, "sell16", dev, C=64, sigma=1024, ki=ki, head=head)
        y = torch.full((m.n_rows,), 7.0, dtype=torch.float64, device=dev)
        dm.run(x, y)
        torch.cuda.synchronize()
        ys.append(y)
    assert torch.equal(ys[0].view(torch.int64), ys[1].view(torch.int64))


# --------------------------------------------------------------------------
# single-pass COO (spmv_coo_run_tail): the owning tile finishes its last row

COO_TAIL_CAP = 80  # csrc/staged.hip kCooTailCap


@pytest.mark.parametrize("case", ["cantlike", "ragged_tails", "aligned", "odd_tail", "fixtures", "batch", "tail52"])
def test_coo_single_pass(torch_dev, case):
    """The single-pass COO (the default where the plan allows) matches the oracle
    (parity rule) and the carry path within it wherever every row ends
    within COO_TAIL_CAP entries of its tile, reproducible run to run; y pre-filled
    with NaN."""
    torch, dev = torch_dev
    rng = np.random.default_rng(41)
    if case == "cantlike":
        ms = [sa.gen_cantlike(0)]
    elif case == "batch":
        ms = [sa.gen_cantlike(1, copies=3)]
    elif case == "tail52":
        # the cant-like rows' entries past 52 (HYB's tail as a COO matrix):
        # two 1,536-entry tiles span more than 250 rows, the row-first
        # bitmap path of coo_staged_kernel (profiles/round6/ab_coo_first.md)
        c = sa.gen_cantlike(0)
        ptr, col, val = sa.csr_from_coo(c)
        h = sa.hyb_build(c.n_rows, ptr, col, val, ki=2, K=52)
        t = h["tail_nnz"]
        ms = [sa.Coo(c.n_rows, c.n_cols, h["tail_row"][:t].copy(), h["tail_col"][:t].copy(),
                     h["tail_val"][:t].copy(), False, "cant-like tail past 52")]
    elif case == "ragged_tails":
        lens = rng.integers(0, COO_TAIL_CAP + 1, 4000)
        lens[::53] = 0
        row = np.repeat(np.arange(lens.size, dtype=np.int32), lens)
        ms = [sa.Coo(lens.size, 3000, row, rng.integers(0, 3000, row.size).astype(np.int32),
                     rng.uniform(-1, 1, row.size), False, "ragged")]
    elif case == "aligned":  # rows of 82 entries: tails up to exactly the cap (80, tile 26)
        lens = np.full(600, COO_TAIL_CAP + 2)
        row = np.repeat(np.arange(lens.size, dtype=np.int32), lens)
        ms = [sa.Coo(lens.size, 3000, row, rng.integers(0, 3000, row.size).astype(np.int32),
                     rng.uniform(-1, 1, row.size), False, "aligned")]
    elif case == "odd_tail":
        # odd nnz, the last row 30 entries before a tile end and 31 past it:
        # its tail ends on the lone entry nnz - 1 (once loaded as
        # the odd pair (nnz - 2, nnz - 1)).  One matrix per candidate tile size.
        ms = []
        for ch in (1024, 1536, 2048, 3072, 4096):
            lead = rng.integers(1, 40, ch)
            lead = lead[np.cumsum(lead) <= ch - 30]
            lead[-1] += ch - 30 - int(lead.sum())
            lens = np.append(lead, 61)
            row = np.repeat(np.arange(lens.size, dtype=np.int32), lens)
            assert row.size % 2 == 1
            ms.append(sa.Coo(lens.size, 500, row, rng.integers(0, 500, row.size).astype(np.int32),
                             rng.uniform(-1, 1, row.size), False, f"odd_tail_{ch}"))
    else:
        ms = [sa.read_mtx(GOLDEN / f"{c}.mtx") for c in CASES]
    for m in ms:
        if m.n_rows == 0:
            continue
        longest = int(np.bincount(m.row, minlength=m.n_rows).max()) if m.nnz else 0
        # a row of k entries runs at most k - 1 past a tile end (rows of 82:
        # tile ends are even, so a tail of 81 never occurs)
        fits = 0 < longest <= COO_TAIL_CAP + 1 or case == "aligned"
        a = sa.to_device(m, "coo", dev)  # default: single pass where the plan allows
        if fits:
            assert a.params["single_pass"], m.label
        b = sa.to_device(m, "coo", dev, coo_tail=False)  # the carry pass
        assert not b.params["single_pass"]
        x = torch.from_numpy(rng.uniform(-1, 1, max(m.n_cols, 1))).to(dev)
        ya = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
        ya2, yb = torch.full_like(ya, float("nan")), torch.full_like(ya, float("nan"))
        a.run(x, ya)
        a.run(x, ya2)
        b.run(x, yb)
        torch.cuda.synchronize()
        assert torch.equal(ya.view(torch.int64), ya2.view(torch.int64))
        assert_parity(m, ya.cpu().numpy(), x.cpu().numpy()[: m.n_cols])
        assert_parity(m, yb.cpu().numpy(), x.cpu().numpy()[: m.n_cols])


@pytest.mark.parametrize("case", ["cantlike", "cantlike_k72", "fixtures", "batch"])
def test_hyb_single_pass_tail(torch_dev, case):
    """HYB's COO tail in one pass (spmv_hyb_run_tail, the default where the
    tail plan allows) against the oracle and the carry pass; y pre-filled
    with NaN, reproducible run to run.  cantlike_k72: tails on scattered
    rows, tiles spanning thousands of rows (the accumulate path that finds
    rows at their first entry)."""
    torch, dev = torch_dev
    if case.startswith("cantlike"):
        ms = [sa.gen_cantlike(0)]
    elif case == "batch":
        ms = [sa.gen_cantlike(1, copies=3)]
    else:
        ms = [sa.read_mtx(GOLDEN / f"{c}.mtx") for c in CASES]
    rng = np.random.default_rng(43)
    for m in ms:
        if m.n_rows == 0:
            continue
        # K = 52 on the cant-like matrices (the stored-bytes optimum; the
        # rule, which also prices the tail's kernel, picks the longest row
        # there); fixtures: K = 2, a tail wherever a row is longer
        K = {"fixtures": 2, "cantlike_k72": 72}.get(case, 52)
        a = sa.to_device(m, "hyb", dev, hyb_k=K)
        b = sa.to_device(m, "hyb", dev, coo_tail=False, hyb_k=K)
        c = sa.to_device(m, "hyb", dev, xwin=False, hyb_k=K)  # the ELL part without x windows
        assert "tails" not in b.arrays and "win" not in c.arrays
        if case != "fixtures":
            assert a.params["tail_nnz"] > 0 and "tails" in a.arrays and "win" in a.arrays, m.label
        x = torch.from_numpy(rng.uniform(-1, 1, max(m.n_cols, 1))).to(dev)
        ya = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
        ya2, yb, yc = (torch.full_like(ya, float("nan")) for _ in range(3))
        a.run(x, ya)
        a.run(x, ya2)
        b.run(x, yb)
        c.run(x, yc)
        torch.cuda.synchronize()
        assert torch.equal(ya.view(torch.int64), ya2.view(torch.int64))
        assert torch.equal(ya.view(torch.int64), yc.view(torch.int64))  # x windows: same bits
        assert_parity(m, ya.cpu().numpy(), x.cpu().numpy()[: m.n_cols])
        assert_parity(m, yb.cpu().numpy(), x.cpu().numpy()[: m.n_cols])


@pytest.mark.parametrize("hot", [0, 4096])
def test_hyb_k0_runs_as_coo(torch_dev, hot):
    """HYB whose plan picks K = 0 (R-MAT: most rows empty or short) has no
    ELL part: it runs as COO over the same entries (spmv_coo_run /
    spmv_coo_run_hot), so y has COO's bits, NaN-prefilled y fully written."""
    torch, dev = torch_dev
    m = sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=3)
    a = sa.to_device(m, "hyb", dev, hot=hot)
    b = sa.to_device(m, "coo", dev, hot=hot)
    assert a.params["K"] == 0 and a.params["tail_nnz"] == m.nnz and a.params["H"] == b.params["H"]
    x = torch.from_numpy(np.random.default_rng(11).uniform(-1, 1, m.n_cols)).to(dev)
    ya = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    yb = torch.full_like(ya, float("nan"))
    a.run(x, ya)
    b.run(x, yb)
    torch.cuda.synchronize()
    assert torch.equal(ya.view(torch.int64), yb.view(torch.int64))
    assert_parity(m, ya.cpu().numpy(), x.cpu().numpy())


def test_coo_single_pass_empty_row_run_search_path(torch_dev):
    """the single pass with mean rows >= 12 (the 250-row start
    table) where one tile spans more rows than the table (a run of 400 empty
    rows), so the row phase searches the staged keys including the tail
    entries, and that tile's last row runs 64 entries past its end.
    Against the carry pass (same tiles) and the oracle."""
    torch, dev = torch_dev
    lens = np.concatenate([np.full(70, 20), np.zeros(400, np.int64), [200], np.full(1000, 40)])
    rng = np.random.default_rng(12)
    row = np.repeat(np.arange(lens.size, dtype=np.int32), lens)
    m = sa.Coo(lens.size, 3000, row, rng.integers(0, 3000, row.size).astype(np.int32), rng.uniform(-1, 1, row.size),
               False, "empty-row run")
    assert m.nnz / m.n_rows >= 12
    a = sa.to_device(m, "coo", dev, coo_tail=True, hot=0)
    b = sa.to_device(m, "coo", dev, coo_tail=False, hot=0)
    assert a.params["single_pass"] and not b.params["single_pass"]
    x = torch.from_numpy(rng.uniform(-1, 1, m.n_cols)).to(dev)
    ya, yb = (torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev) for _ in range(2))
    a.run(x, ya)
    b.run(x, yb)
    torch.cuda.synchronize()
    assert_parity(m, ya.cpu().numpy(), x.cpu().numpy())
    assert_parity(m, yb.cpu().numpy(), x.cpu().numpy())
    assert np.all(ya.cpu().numpy()[70:470] == 0.0)


def test_coo_tail_conflicting_options_raise(torch_dev):
    """coo_tail=True with the x-window or hot-table COO path (which
    use the carry pass) raises instead of being ignored."""
    _, dev = torch_dev
    m = sa.gen_random(2000, 2000, 1, 20, seed=3)
    with pytest.raises(sa.SpmvError):
        sa.to_device(m, "coo", dev, coo_tail=True, xwin=True)
    with pytest.raises(sa.SpmvError):
        sa.to_device(m, "coo", dev, coo_tail=True, hot=64)


def test_coo_single_pass_refuses_long_rows(torch_dev):
    """A row running more than COO_TAIL_CAP entries past its tile refuses the single
    pass (coo_tail=True raises); the default falls back to the carry pass."""
    torch, dev = torch_dev
    lens = np.concatenate([np.full(10, 100), [3000], np.full(10, 100)])
    rng = np.random.default_rng(5)
    row = np.repeat(np.arange(lens.size, dtype=np.int32), lens)
    m = sa.Coo(lens.size, 2000, row, rng.integers(0, 2000, row.size).astype(np.int32), rng.uniform(-1, 1, row.size),
               False, "long")
    dm = sa.to_device(m, "coo", dev)
    assert not dm.params["single_pass"]
    with pytest.raises(sa.SpmvError):
        sa.to_device(m, "coo", dev, coo_tail=True)
    x = torch.from_numpy(rng.uniform(-1, 1, m.n_cols)).to(dev)
    y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    dm.run(x, y)
    torch.cuda.synchronize()
    assert_parity(m, y.cpu().numpy(), x.cpu().numpy())


@pytest.mark.parametrize("fmt,kw", [("csr", {"variant": 4}), ("coo", {}), ("cmrs", {"cmrs_variant": 1}),
                                    ("sell", {"sigma": 1 << 24, "ki": 2, "xwin": False}), ("csrf32", {})])
def test_column_relabel_same_bits(torch_dev, fmt, kw):
    """Columns relabelled by degree (spmv_column_relabel) with x gathered
    into that layout on the device (spmv_gather): the same products in the
    same order, so y is bit-identical to the original matrix on x (no hot
    table on either side), and passes the oracle on the ORIGINAL matrix."""
    torch, dev = torch_dev
    m = sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=6)
    m2, order = sa.relabel_columns(m)
    xh = np.random.default_rng(21).uniform(-1, 1, m.n_cols)
    x = torch.from_numpy(xh).to(dev)
    x2 = sa.gather_x(torch.from_numpy(order).to(dev), x)
    assert torch.equal(x2.cpu(), torch.from_numpy(xh[order]))
    a = sa.to_device(m, fmt, dev, hot=0, **kw)
    b = sa.to_device(m2, fmt, dev, hot=0, **kw)
    ya, yb = (torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev) for _ in range(2))
    a.run(x, ya)
    b.run(x2, yb)
    torch.cuda.synchronize()
    assert torch.equal(ya.view(torch.int64), yb.view(torch.int64))
    if fmt != "csrf32":
        assert_parity(m, yb.cpu().numpy(), xh)


def test_csr_tiled_bigplan_rmat_same_bits(torch_dev):
    """The R-MAT's big tiles (runs of empty rows) through the big-tile plan:
    bit-identical to the global-offset row phase (bigplan=False), with and
    without the relabel, and the oracle's y."""
    torch, dev = torch_dev
    m = sa.gen_rmat(2_000_000, 6_000_000, scale=21, seed=7)
    xh = np.random.default_rng(22).uniform(-1, 1, m.n_cols)
    x = torch.from_numpy(xh).to(dev)
    a = sa.to_device(m, "csr", dev, variant=4, hot=0)
    b = sa.to_device(m, "csr", dev, variant=4, hot=0, bigplan=False)
    assert a.params["big_tiles"] > 0 and b.params["big_tiles"] == 0
    ya, yb = (torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev) for _ in range(2))
    a.run(x, ya)
    b.run(x, yb)
    torch.cuda.synchronize()
    assert torch.equal(ya.view(torch.int64), yb.view(torch.int64))
    assert_parity(m, ya.cpu().numpy(), xh)
