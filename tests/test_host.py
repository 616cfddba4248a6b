"""Host side of the product (libspmv_host.so) on a CPU-only machine.

The reader must accept/reject exactly like the oracle (the reference's
rules), every builder must lay the matrix out so that its CPU loop gives
the oracle's y, and the generators must be deterministic with the
documented sizes.  The HIP kernels read the same arrays (tests/test_gpu_*).
"""
from __future__ import annotations

import numpy as np
import pytest

import spmv_amd as sa
from conftest import GOLDEN, golden_cases
from oracle import oracle

CASES = [c["name"] for c in golden_cases()]


def _both(name):
    m = sa.read_mtx(GOLDEN / f"{name}.mtx")
    n, mc, r, c, v, sym = oracle.read_mtx(GOLDEN / f"{name}.mtx")
    return m, (n, mc, r, c, v, sym)


@pytest.mark.parametrize("name", CASES)
def test_reader_matches_oracle_bit_exact(name):
    m, (n, mc, r, c, v, sym) = _both(name)
    assert (m.n_rows, m.n_cols, m.symmetric) == (n, mc, sym)
    assert np.array_equal(m.row, r) and np.array_equal(m.col, c)
    assert np.array_equal(m.val.view(np.uint64), v.view(np.uint64))  # same strtod rounding


def test_reader_rejections(tmp_path):
    bad = {
        "complex.mtx": "%%MatrixMarket matrix coordinate complex general\n2 2 1\n1 1 1.0 0.0\n",
        "array.mtx": "%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n",
        "nobanner.mtx": "2 2 1\n1 1 1.0\n",
        "short.mtx": "%%MatrixMarket matrix coordinate real general\n2 2 3\n1 1 1.0\n",
        "range.mtx": "%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1.0\n",
        "zero_index.mtx": "%%MatrixMarket matrix coordinate real general\n2 2 1\n0 1 1.0\n",
        "badtype.mtx": "%%MatrixMarket matrix coordinate quaternion general\n2 2 1\n1 1 1.0\n",
    }
    for name, text in bad.items():
        p = tmp_path / name
        p.write_text(text)
        with pytest.raises(sa.SpmvError) as e:
            sa.read_mtx(p)
        assert e.value.rc == sa.FILE_ERROR, name
    with pytest.raises(sa.SpmvError) as e:
        sa.read_mtx(tmp_path / "missing.mtx")
    assert e.value.rc == sa.FILE_ERROR


def test_reader_case_insensitive_banner(tmp_path):
    p = tmp_path / "upper.mtx"
    p.write_text("%%MatrixMarket MATRIX Coordinate REAL General\n2 2 2\n1 1 1.5\n2 2 -2e3\n")
    m = sa.read_mtx(p)
    assert m.val.tolist() == [1.5, -2000.0]


def test_write_read_roundtrip(tmp_path):
    m = sa.gen_random(300, 200, 0, 9, seed=11)
    sa.write_mtx(tmp_path / "rt.mtx", m)
    m2 = sa.read_mtx(tmp_path / "rt.mtx")
    assert np.array_equal(m.row, m2.row) and np.array_equal(m.col, m2.col)
    assert np.array_equal(m.val, m2.val)  # %.17g is exact


def _y_gold(name):
    return np.load(GOLDEN / f"{name}.y.npy")


def _cpu_fmt(m, fmt, **kw):
    """Build `fmt` with the product builders and run the product CPU loop."""
    L = sa.host_lib()
    x = sa.ramp_x(m.n_cols)
    y = np.full(max(m.n_rows, 1), np.nan)
    ptr, col, val = sa.csr_from_coo(m)
    if fmt == "coo":
        r, c, v = sa.coo_sort_by_row(m)
        L.spmv_cpu_coo(m.n_rows, m.nnz, sa._ptr(r), sa._ptr(c), sa._ptr(v), sa._ptr(x), sa._ptr(y), 2)
    elif fmt == "csr":
        L.spmv_cpu_csr(m.n_rows, sa._ptr(ptr), sa._ptr(col), sa._ptr(val), sa._ptr(x), sa._ptr(y), 2)
    elif fmt == "ell":
        e = sa.ell_build(m.n_rows, ptr, col, val, ki=kw.get("ki", 2))
        L.spmv_cpu_ell(m.n_rows, e["K"], e["ld"], e["ki"], sa._ptr(e["col"]), sa._ptr(e["val"]), sa._ptr(x),
                       sa._ptr(y), 2)
    elif fmt == "sell":
        s = sa.sell_build(m.n_rows, ptr, col, val, C=kw.get("C", 64), sigma=kw.get("sigma", 1024),
                          ki=kw.get("ki", 2))
        L.spmv_cpu_sell(m.n_rows, s["C"], s["ki"], s["n_slices"], sa._ptr(s["slice_ptr"]), sa._ptr(s["perm"]),
                        sa._ptr(s["col"]), sa._ptr(s["val"]), sa._ptr(x), sa._ptr(y), 2)
    elif fmt == "cmrs":
        c = sa.cmrs_build(m.n_rows, ptr, h=kw.get("h", 8))
        L.spmv_cpu_cmrs(m.n_rows, c["h"], c["n_strips"], sa._ptr(c["strip_ptr"]), sa._ptr(c["row_in_strip"]),
                        sa._ptr(col), sa._ptr(val), sa._ptr(x), sa._ptr(y), 2)
    return y[: m.n_rows], x


FMT_PARAMS = [
    ("coo", {}),
    ("csr", {}),
    ("ell", {"ki": 1}),
    ("ell", {"ki": 2}),
    ("sell", {"C": 64, "sigma": 1024, "ki": 2}),
    ("sell", {"C": 64, "sigma": 1, "ki": 1}),
    ("sell", {"C": 32, "sigma": 1, "ki": 1}),  # the reference's configuration
    ("sell", {"C": 128, "sigma": 256, "ki": 2}),
    ("cmrs", {"h": 8}),
    ("cmrs", {"h": 1}),
    ("cmrs", {"h": 64}),
]


@pytest.mark.parametrize("fmt,kw", FMT_PARAMS, ids=[f"{f}-{'-'.join(f'{k}{v}' for k, v in kw.items())}" for f, kw in FMT_PARAMS])
@pytest.mark.parametrize("name", CASES)
def test_builders_cpu_loops_match_oracle(name, fmt, kw):
    m = sa.read_mtx(GOLDEN / f"{name}.mtx")
    y, x = _cpu_fmt(m, fmt, **kw)
    y_ref = oracle.file_order_spmv(m.n_rows, m.row, m.col, m.val, x)
    assert oracle.parity(y, y_ref, m.row, m.col, m.val, x, m.n_rows).size == 0
    assert oracle.parity(y, _y_gold(name), m.row, m.col, m.val, x, m.n_rows).size == 0


def test_sell_layout_properties():
    m = sa.gen_random(1000, 1000, 0, 40, seed=5)
    ptr, col, val = sa.csr_from_coo(m)
    s = sa.sell_build(m.n_rows, ptr, col, val, C=64, sigma=256, ki=2)
    perm = s["perm"][: s["n_slices"] * 64]
    real = perm[perm >= 0]
    assert np.array_equal(np.sort(real), np.arange(m.n_rows))  # a permutation
    lens = np.diff(ptr)
    for w in range(0, m.n_rows, 256):  # sorted by length, descending, per window
        win = perm[w: w + 256]
        win = win[win >= 0]
        assert np.all(np.diff(lens[win]) <= 0)
        assert set(win.tolist()) == set(range(w, min(w + 256, m.n_rows)))
    widths = np.diff(s["slice_ptr"]) // 64
    assert np.all(widths % 2 == 0)
    assert s["slice_ptr"][-1] == s["stored"]


def test_padding_reuses_row_column():
    m = sa.gen_random(200, 500, 1, 20, seed=9)
    ptr, col, val = sa.csr_from_coo(m)
    e = sa.ell_build(m.n_rows, ptr, col, val, ki=2)
    K, ld = e["K"], e["ld"]
    for i in range(m.n_rows):
        cols_i = set(col[ptr[i]:ptr[i + 1]].tolist())
        for k in range(K):
            pos = (k // 2) * ld * 2 + i * 2 + (k % 2)
            if k >= ptr[i + 1] - ptr[i]:
                assert e["val"][pos] == 0.0
                assert e["col"][pos] in cols_i


def test_cmrs_row_in_strip():
    m = sa.gen_random(103, 50, 0, 7, seed=4)
    ptr, col, val = sa.csr_from_coo(m)
    c = sa.cmrs_build(m.n_rows, ptr, h=8)
    assert c["n_strips"] == 13
    for s in range(c["n_strips"]):
        b, e = c["strip_ptr"][s], c["strip_ptr"][s + 1]
        rin = c["row_in_strip"][b:e]
        assert np.all(np.diff(rin.astype(int)) >= 0) and (rin.size == 0 or rin.max() < 8)


def test_coo_sort_is_stable():
    m = sa.read_mtx(GOLDEN / "colmajor.mtx")
    r, c, v = sa.coo_sort_by_row(m)
    order = np.argsort(m.row, kind="stable")
    assert np.array_equal(r, m.row[order]) and np.array_equal(c, m.col[order])
    assert np.array_equal(v, m.val[order])


def test_cantlike_counts_and_symmetry():
    m = sa.gen_cantlike(0)
    assert (m.n_rows, m.nnz) == (62451, 4007383)  # SuiteSparse cant's N and nnz
    assert np.all(np.diff(m.row) >= 0)
    lo = sa.gen_cantlike(2)
    assert lo.nnz == 2034917 and lo.symmetric and np.all(lo.row >= lo.col)
    t = sa.gen_cantlike(1)
    assert np.all(np.diff(t.col) >= 0)  # column-major order
    # symmetric pattern + values: A == A^T
    import scipy.sparse as sp

    A = sp.coo_matrix((m.val, (m.row, m.col)), shape=(m.n_rows, m.n_rows)).tocsr()
    assert abs(A - A.T).max() == 0.0
    two = sa.gen_cantlike(0, copies=2)
    assert two.n_rows == 2 * 62451 and two.nnz == 2 * 4007383
    assert np.array_equal(two.row[m.nnz:] - 62451, m.row)


def test_generators_deterministic():
    a = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=1)
    b = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=1)
    assert np.array_equal(a.row, b.row) and np.array_equal(a.col, b.col) and np.array_equal(a.val, b.val)
    assert a.row.max() < 100_000 and a.col.max() < 100_000 and a.row.min() >= 0
    deg = np.bincount(a.row, minlength=100_000)
    assert deg.max() > 20 * deg.mean()  # R-MAT skew
    assert np.all((a.val >= -1) & (a.val < 1))
    ptr, col, val = sa.gen_banded_csr(1000, 10, 20)
    assert ptr.tolist() == list(range(0, 161, 16))
    assert col[:16].tolist() == [(10 + o) % 1000 for o in range(-8, 8)]
    p2, c2, v2 = sa.gen_banded_csr(1000)
    assert np.array_equal(v2[160:320], val)  # row-range generation = slice of the whole


def test_check_function():
    m = sa.read_mtx(GOLDEN / "hand3.mtx")
    x = sa.ramp_x(3)
    assert sa.check(m, x, np.array([4.0, 3.0, 17.0])) == (0, -1)
    bad, first = sa.check(m, x, np.array([4.0, 3.1, 17.0]))
    assert bad == 1 and first == 1
    assert sa.check(m, x, np.array([4.0, 3.0, np.nan]))[0] == 1


def test_binary_cache_roundtrip(tmp_path):
    m = sa.gen_random(500, 300, 0, 30, seed=17)
    sa.write_bin(tmp_path / "m.bin", m)
    b = sa.read_bin(tmp_path / "m.bin")
    assert (b.n_rows, b.n_cols, b.nnz) == (m.n_rows, m.n_cols, m.nnz)
    assert np.array_equal(b.row, m.row) and np.array_equal(b.col, m.col) and np.array_equal(b.val, m.val)
    (tmp_path / "bad.bin").write_bytes(b"NOTABIN" + bytes(100))
    with pytest.raises(sa.SpmvError):
        sa.read_bin(tmp_path / "bad.bin")


def test_parallel_parse_matches_serial_semantics(tmp_path):
    """Files > 4 MiB are parsed by all threads; the result must equal the
    oracle's fscanf reader entry for entry (file order kept)."""
    m = sa.gen_rmat(200_000, 400_000, scale=18, seed=9)
    p = tmp_path / "big.mtx"
    sa.write_mtx(p, m)
    assert p.stat().st_size > (4 << 20)
    r = sa.read_mtx(p)
    n, mc, orow, ocol, oval, _ = oracle.read_mtx(p)
    assert np.array_equal(r.row, orow) and np.array_equal(r.col, ocol)
    assert np.array_equal(r.val.view(np.uint64), oval.view(np.uint64))
    # an extra trailing entry beyond nz: the reference reads nz and ignores the rest
    with open(p, "a") as f:
        f.write("1 1 5.0\n")
    r2 = sa.read_mtx(p)
    assert r2.nnz == m.nnz and np.array_equal(r2.val, r.val)


@pytest.mark.parametrize("kind", ["cantlike", "rmat", "mixed", "tiny"])
def test_csr16_round_trip(kind):
    """Compressed 16-bit column offsets decode to the
    CSR columns exactly; wide blocks go through the escape array."""
    if kind == "cantlike":
        m = sa.gen_cantlike(0)
    elif kind == "rmat":
        m = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=2)
    elif kind == "mixed":
        m = sa.gen_random(70_000, 200_000, 0, 40, seed=11)
    else:
        m = sa.read_mtx(GOLDEN / "n67.mtx")
    ptr, col, val = sa.csr_from_coo(m)
    c = sa.csr16_build(col)
    nnz = len(col)
    assert c["n_blocks"] == (nnz + 63) // 64
    p = np.arange(nnz)
    base = c["blk_base"][p // 64].astype(np.int64)
    esc_slot = -1 - base
    esc = np.concatenate([c["col_esc"], np.zeros(64, np.int32)])  # np.where evaluates both sides
    dec = np.where(base >= 0, base + c["col_off"][:nnz].astype(np.int64),
                   esc[np.maximum(esc_slot, 0) * 64 + (p % 64)])
    assert np.array_equal(dec, col.astype(np.int64))
    assert c["n_esc"] == int(np.sum(c["blk_base"][: c["n_blocks"]] < 0))
    if kind == "cantlike":
        assert c["n_esc"] == 0
    if kind == "rmat":
        assert c["n_esc"] > 0.9 * c["n_blocks"]


def _hyb_plan(lens, ki=2):
    import ctypes
    ptr = np.concatenate([[0], np.cumsum(np.asarray(lens, np.int64))]).astype(np.int64)
    K, ld, tail = ctypes.c_int32(0), ctypes.c_int64(0), ctypes.c_int64(0)
    assert sa.host_lib().spmv_hyb_plan(len(lens), sa._ptr(ptr), ki, 0, ctypes.byref(K), ctypes.byref(ld),
                                       ctypes.byref(tail)) == 0
    return K.value, ld.value, tail.value


def test_hyb_rule_prices_the_second_kernel():
    """spmv_hyb_plan's K rule: stored bytes (12 per ELL slot, 16 per tail
    entry) plus 32 MB when both parts are non-empty.  A small matrix gets ONE
    part: the cant-like rows (64.2 mean, 81 longest) all in the ELL part (the
    bytes-only optimum, K = 52, ran 22.2 vs 15.1 us, profiles/round6/ab_hyb_k.md);
    an R-MAT all in the tail (K = 0).  A large matrix with a few long rows
    still splits."""
    m = sa.gen_cantlike(0)
    lens = np.diff(sa.csr_from_coo(m)[0])
    assert _hyb_plan(lens) == (82, 62464, 0)
    r = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=2)
    K, _, tail = _hyb_plan(np.diff(sa.csr_from_coo(r)[0]))
    assert K == 0 and tail == r.nnz
    big = np.full(2_000_000, 10, np.int64)
    big[::2000] = 5000  # 1,000 long rows: 80 MB of tail against 120 GB of ELL padding
    K, ld, tail = _hyb_plan(big)
    assert K == 10 and ld == 2_000_000 and tail == 1000 * 4990


@pytest.mark.parametrize("kind,K", [("rmat", 0), ("rmat", 3), ("ragged", 0), ("cantlike", 0), ("tiny", 0)])
def test_hyb_split_round_trip(kind, K):
    """HYB (§8f row 4): ELL part + COO tail hold exactly the CSR entries,
    each row's first K in the ELL slots, the rest row-sorted in the tail."""
    if kind == "rmat":
        m = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=2)
    elif kind == "ragged":
        m = sa.gen_random(5_000, 5_000, 0, 300, seed=4)
    elif kind == "cantlike":
        m = sa.gen_cantlike(0)
    else:
        m = sa.read_mtx(GOLDEN / "empty_rows.mtx")
    ptr, col, val = sa.csr_from_coo(m)
    h = sa.hyb_build(m.n_rows, ptr, col, val, ki=2, K=K)
    Kh, ld = h["K"], h["ld"]
    if K:
        assert Kh == K + (K % 2)
    lens = np.diff(ptr)
    assert h["tail_nnz"] == int(np.maximum(lens - Kh, 0).sum())
    for i in range(0, m.n_rows, max(1, m.n_rows // 500)):
        n_e = min(int(lens[i]), Kh)
        for k in range(n_e):
            pos = (k // 2) * ld * 2 + i * 2 + (k % 2)
            assert h["ell_col"][pos] == col[ptr[i] + k] and h["ell_val"][pos] == val[ptr[i] + k]
    t = h["tail_nnz"]
    assert np.all(np.diff(h["tail_row"][:t].astype(np.int64)) >= 0)
    if t:
        # the tail is the CSR entries past K, in order
        exp = np.concatenate([col[ptr[r] + Kh:ptr[r + 1]] for r in range(m.n_rows) if lens[r] > Kh])
        assert np.array_equal(h["tail_col"][:t], exp)


def _sell_split_model(s, T, cs, ck, x):
    """numpy model of spmv_sell_run_split: main part = first T slot columns
    of every slice, chunks add the rest; y scattered through perm."""
    C, ki = s["C"], s["ki"]
    sp, perm, col, val = s["slice_ptr"], s["perm"], s["col"], s["val"]
    acc = np.zeros(s["n_slices"] * C)
    for sl in range(s["n_slices"]):
        w = (sp[sl + 1] - sp[sl]) // C
        blk_v = val[sp[sl]:sp[sl + 1]].reshape(w // ki, C, ki)
        blk_c = col[sp[sl]:sp[sl + 1]].reshape(w // ki, C, ki)
        n = min(w, T) if T else w
        acc[sl * C:(sl + 1) * C] = (blk_v[: n // ki] * x[blk_c[: n // ki]]).sum(axis=(0, 2))
    for c, k0 in zip(cs, ck):
        sl = int(c)
        w = (sp[sl + 1] - sp[sl]) // C
        blk_v = val[sp[sl]:sp[sl + 1]].reshape(w // ki, C, ki)
        blk_c = col[sp[sl]:sp[sl + 1]].reshape(w // ki, C, ki)
        g0, g1 = k0 // ki, min(k0 + T, w) // ki
        acc[sl * C:(sl + 1) * C] += (blk_v[g0:g1] * x[blk_c[g0:g1]]).sum(axis=(0, 2))
    y = np.full(max(perm.max() + 1, 0) if perm.size else 0, np.nan)
    ok = perm[: s["n_slices"] * C] >= 0
    y[perm[: s["n_slices"] * C][ok]] = acc[ok]
    return y


@pytest.mark.parametrize("kind,T,ki", [("rmat", None, 1), ("rmat", None, 2), ("rmat", 64, 2), ("cantlike", 2, 1),
                                       ("cantlike", None, 1), ("tiny", 1, 1)])
def test_sell_split_plan_covers_every_slot(kind, T, ki):
    """The split plan (§8 A6 on power-law rows): main kernel's first T slot
    columns + chunks [k0, k0+T) tile every slice exactly once, so the model
    of spmv_sell_run_split gives the oracle's y."""
    if kind == "rmat":
        m = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=2)
    elif kind == "cantlike":
        m = sa.gen_cantlike(0)
    else:
        m = sa.read_mtx(GOLDEN / "empty_rows.mtx")
    ptr, col, val = sa.csr_from_coo(m)
    s = sa.sell_build(m.n_rows, ptr, col, val, C=64, sigma=1024, ki=ki)
    Tp, cs, ck = sa.sell_split_plan(s, T)
    if kind == "rmat" and T is None:
        assert Tp >= 256 and Tp % ki == 0 and len(cs) > 0  # the rule fires on hubs
    if kind == "cantlike" and T is None:
        assert Tp == 0  # and stays off for ordinary matrices
    widths = np.diff(s["slice_ptr"]) // 64
    if Tp:
        exp = sum(max(0, -(-int(w) // Tp) - 1) for w in widths)
        assert len(cs) == exp and np.all(np.diff(cs) >= 0) and np.all(ck % Tp == 0) and np.all(ck > 0)
        assert np.all(ck < widths[cs])
    x = np.random.default_rng(3).uniform(-1, 1, m.n_cols)
    y = _sell_split_model(s, Tp, cs, ck, x)[: m.n_rows]
    y_ref = oracle.file_order_spmv(m.n_rows, m.row, m.col, m.val, x)
    assert len(oracle.parity(y, y_ref, m.row, m.col, m.val, x, m.n_rows)) == 0


@pytest.mark.parametrize("kind,exp", [("rmat", 1), ("cantlike", 0), ("ragged", 0)])
def test_cmrs_pick_variant(kind, exp):
    if kind == "rmat":
        m = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=2)
    elif kind == "cantlike":
        m = sa.gen_cantlike(0)
    else:
        m = sa.gen_random(5_000, 5_000, 0, 300, seed=4)
    ptr, _, _ = sa.csr_from_coo(m)
    c = sa.cmrs_build(m.n_rows, ptr, h=8)
    assert sa.host_lib().spmv_cmrs_pick_variant(c["n_strips"], sa._ptr(c["strip_ptr"])) == exp


@pytest.mark.parametrize("H", [0, 1, 100, 5000])
def test_hot_columns_selection_and_renumbering(H):
    """spmv_hot_columns: the H most frequent columns in decreasing count,
    renumbered n_cols + rank; every other column untouched (the inverse
    map restores col exactly, so the hot-column CSR is the same matrix)."""
    m = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=2)
    _, col, _ = sa.csr_from_coo(m)
    n, hot, ch = sa.hot_columns(m.n_cols, col, H)
    cnt = np.bincount(col, minlength=m.n_cols)
    if H == 0:  # the rule: 1e5 columns (0.8 MB of x) need no table
        assert n == 0 and np.array_equal(ch, col)
        return
    assert n == min(H, np.count_nonzero(cnt))
    assert len(set(hot.tolist())) == n and np.all(np.diff(cnt[hot]) <= 0)
    rest = np.delete(cnt, hot)
    assert cnt[hot].min() >= rest.max()
    is_hot = ch >= m.n_cols
    back = ch.copy()
    back[is_hot] = hot[ch[is_hot] - m.n_cols]
    assert np.array_equal(back, col)
    assert not np.isin(col[~is_hot], hot).any()


@pytest.mark.parametrize("skewed", [True, False])
def test_hot_columns_rule(skewed):
    """H = 0 picks 2^19 columns, halved while above nnz / 32 (5.6e6
    entries: 2^17), when they hold at least half the entries of a matrix
    with more than 2^21 columns, 8 or more each on average; a uniform
    column spread (little reuse) gets none."""
    rng = np.random.default_rng(9)
    n_cols = 3_000_000
    if skewed:
        col = np.concatenate([rng.integers(0, 1000, 5_000_000), rng.integers(0, n_cols, 600_000)])
    else:
        col = rng.integers(0, n_cols, 2_000_000)
    col = col.astype(np.int32)
    n, hot, ch = sa.hot_columns(n_cols, col, 0)
    if skewed:
        assert n == 1 << 17 and np.all(hot[:1000] < 1000)
    else:
        assert n == 0 and np.array_equal(ch, col)


@pytest.mark.parametrize("kind", ["rmat", "tiny", "empty_cols"])
def test_column_relabel(kind):
    """spmv_column_relabel: a permutation ranking columns by decreasing
    count (ties by id, empty columns last in id order); col' = newid[col];
    the relabelled matrix on x[order] gives the oracle's y bit for bit
    (same rows, same entry order, same products)."""
    if kind == "rmat":
        m = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=2)
    elif kind == "tiny":
        m = sa.Coo(3, 4, np.array([0, 1, 2, 2], np.int32), np.array([3, 1, 3, 1], np.int32),
                   np.array([1.0, 2.0, 3.0, 4.0]))
    else:
        m = sa.gen_random(500, 5000, 0, 9, seed=4)
    order, newid, c2 = sa.column_relabel(m.n_cols, m.col)
    cnt = np.bincount(m.col, minlength=m.n_cols)
    assert np.array_equal(np.sort(order), np.arange(m.n_cols))
    assert np.array_equal(newid[order], np.arange(m.n_cols))
    assert np.all(np.diff(cnt[order]) <= 0)
    ties = np.diff(cnt[order]) == 0
    assert np.all(np.diff(order)[ties] > 0)  # ties in increasing column id
    assert np.array_equal(c2, newid[m.col])
    m2, order2 = sa.relabel_columns(m)
    assert np.array_equal(order2, order) and np.array_equal(m2.row, m.row) and np.array_equal(m2.col, c2)
    x = np.random.default_rng(1).uniform(-1, 1, m.n_cols)
    assert np.array_equal(oracle.file_order_spmv(m.n_rows, m.row, m.col, m.val, x), oracle.file_order_spmv(m2.n_rows, m2.row, m2.col, m2.val, np.ascontiguousarray(x[order])))
    if kind == "tiny":
        assert order.tolist() == [1, 3, 0, 2]


@pytest.mark.parametrize("tile,cap", [(512, 1024), (512, 16), (1536, 100)])
def test_csr_tiled_bigplan(tile, cap):
    """spmv_csr_tiled_bigplan lists, for every tile owning more than `cap`
    rows (at most 65,536), exactly its owned rows with entries in it and
    their [a, b) relative to the tile start; other tiles get -1."""
    m = sa.gen_rmat(200_000, 600_000, scale=18, seed=3)
    ptr, _, _ = sa.csr_from_coo(m)
    lib = sa.host_lib()
    n = lib.spmv_csr_tiled_bigplan(m.n_rows, ptr.ctypes.data, tile, cap, None)
    plan = np.empty(n, np.int32)
    assert lib.spmv_csr_tiled_bigplan(m.n_rows, ptr.ctypes.data, tile, cap, plan.ctypes.data) == n
    z = int(ptr[-1])
    tiles = (z + tile - 1) // tile
    seen = 0
    for t in range(tiles):
        t0, t1 = t * tile, min(t * tile + tile, z)
        r_lo = int(np.searchsorted(ptr, t0, side="left"))
        r_hi = m.n_rows - 1 if t1 == z else int(np.searchsorted(ptr, t1, side="left")) - 1
        nr = r_hi - r_lo + 1
        if nr <= cap or nr > 65536:
            assert plan[t] == -1
            continue
        assert plan[t] == seen
        st, en = plan[tiles + seen], plan[tiles + seen + 1]
        assert st % 2 == 0
        want = [(r - r_lo, int(ptr[r] - t0), int(min(ptr[r + 1], t1) - t0)) for r in range(r_lo, r_hi + 1)
                if ptr[r] < min(ptr[r + 1], t1)]
        got = [(int(plan[i]), int(plan[i + 1]) & 0xFFFF, (int(plan[i + 1]) >> 16) & 0xFFFF) for i in range(st, en, 2)]
        assert got == want
        seen += 1
    assert (seen > 0) == (cap == 16 or seen > 0)
    assert lib.spmv_csr_tiled_bigplan(m.n_rows, ptr.ctypes.data, 1, cap, None) == -1


@pytest.mark.parametrize("kind", ["random", "rmat", "tiny"])
def test_column_relabel_ties_first(kind):
    """spmv_column_relabel_ex(ties = 1): the same count ranking, equal
    counts in order of first appearance in col (unused columns last by
    id); the relabelled matrix gives the oracle's y bit for bit."""
    if kind == "rmat":
        m = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=2)
    elif kind == "tiny":
        m = sa.Coo(3, 6, np.array([0, 0, 1, 1, 1, 2, 2, 2], np.int32), np.array([3, 1, 3, 2, 1, 0, 5, 3], np.int32),
                   np.arange(1.0, 9.0))
    else:
        m = sa.gen_random(500, 5000, 0, 9, seed=4)
    order, newid, c2 = sa.column_relabel(m.n_cols, m.col, "first")
    cnt = np.bincount(m.col, minlength=m.n_cols)
    assert np.array_equal(np.sort(order), np.arange(m.n_cols))
    assert np.array_equal(newid[order], np.arange(m.n_cols))
    assert np.all(np.diff(cnt[order]) <= 0)
    first = np.full(m.n_cols, np.iinfo(np.int64).max)
    np.minimum.at(first, m.col, np.arange(m.col.size))
    key = np.where(cnt[order] > 0, first[order], m.col.size + order)  # unused: after, by id
    ties = np.diff(cnt[order]) == 0
    assert np.all(np.diff(key)[ties] > 0)
    assert np.array_equal(c2, newid[m.col])
    x = np.random.default_rng(1).uniform(-1, 1, m.n_cols)
    assert np.array_equal(oracle.file_order_spmv(m.n_rows, m.row, m.col, m.val, x),
                          oracle.file_order_spmv(m.n_rows, m.row, c2, m.val, np.ascontiguousarray(x[order])))
    if kind == "tiny":
        assert order.tolist() == [3, 1, 2, 0, 5, 4]


def test_column_relabel_bad_input():
    lib = sa.host_lib()
    col = np.array([0, 5], np.int32)
    buf = np.empty(8, np.int32)
    assert lib.spmv_column_relabel(5, 2, col.ctypes.data, buf.ctypes.data, buf.ctypes.data, buf.ctypes.data) == -1
    assert lib.spmv_column_relabel(0, 0, None, buf.ctypes.data, buf.ctypes.data, None) == -1
    assert lib.spmv_column_relabel_ex(5, 2, col.ctypes.data, buf.ctypes.data, buf.ctypes.data, buf.ctypes.data, 1) == -1
    ok = np.array([0, 1], np.int32)
    assert lib.spmv_column_relabel_ex(5, 2, ok.ctypes.data, buf.ctypes.data, buf.ctypes.data, buf.ctypes.data, 2) == -1
    with pytest.raises(sa.SpmvError):
        sa.column_relabel(5, ok, "degree")


def _ref_sort_rows(ptr, col, val):
    """numpy model of spmv_csr_sort_rows: each row's entries by column,
    equal columns in their original order (a stable sort)."""
    c2, v2 = col.copy(), val.copy()
    for r in range(ptr.size - 1):
        a, b = int(ptr[r]), int(ptr[r + 1])
        o = np.argsort(col[a:b], kind="stable")
        c2[a:b], v2[a:b] = col[a:b][o], val[a:b][o]
    return c2, v2


@pytest.mark.parametrize("kind", ["duplicates", "empty_rows", "long_rows", "rmat_small"])
def test_csr_sort_rows(kind):
    """spmv_csr_sort_rows (bench.py's R-MAT layout): every
    row's entries by increasing column, in place; the (col, val) pairs stay
    together; equal columns (duplicate entries) keep their file order, which
    the merge path (rows >= 32 entries) must preserve as well as the
    insertion path; empty rows and row_ptr are untouched."""
    rng = np.random.default_rng(17)
    if kind == "duplicates":  # short rows, many equal columns: insertion sort path
        lens = rng.integers(0, 20, 300)
        cols = [rng.integers(0, 6, n) for n in lens]
    elif kind == "empty_rows":
        lens = np.where(rng.random(500) < 0.6, 0, rng.integers(1, 50, 500))
        cols = [rng.integers(0, 1000, n) for n in lens]
    elif kind == "long_rows":  # merge sort path, with duplicates across the halves
        lens = np.array([0, 31, 32, 33, 64, 1000, 4097, 1])
        cols = [rng.integers(0, max(n // 3, 1), n) for n in lens]
    else:
        m = sa.gen_rmat(50_000, 500_000, scale=16, seed=8)
        ptr, col, val = sa.csr_from_coo(m)
        lens, cols = None, None
    if lens is not None:
        ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        col = np.concatenate([np.asarray(c, np.int32) for c in cols] + [np.zeros(0, np.int32)]).astype(np.int32)
        val = rng.uniform(-1, 1, col.size)  # distinct values: the pairing and the stability are visible
    want_c, want_v = _ref_sort_rows(ptr, col, val)
    ptr0 = ptr.copy()
    c, v = col.copy(), val.copy()
    sa.csr_sort_rows(ptr.size - 1, ptr, c, v)
    assert np.array_equal(ptr, ptr0)
    assert np.array_equal(c, want_c)
    assert np.array_equal(v.view(np.int64), want_v.view(np.int64))
    # every row now ascending, and the multiset of (col, val) pairs per row kept
    for r in rng.integers(0, ptr.size - 1, 50):
        a, b = int(ptr[r]), int(ptr[r + 1])
        assert np.all(np.diff(c[a:b]) >= 0)
        assert sorted(zip(col[a:b].tolist(), val[a:b].tolist())) == sorted(zip(c[a:b].tolist(), v[a:b].tolist()))


def test_csr_sort_rows_bad_arguments():
    lib = sa.host_lib()
    ptr = np.array([0, 2, 3], np.int64)
    col = np.array([1, 0, 2], np.int32)
    val = np.ones(3)
    assert lib.spmv_csr_sort_rows(-1, ptr.ctypes.data, col.ctypes.data, val.ctypes.data) == sa.OTHER_ERROR
    assert lib.spmv_csr_sort_rows(2, None, col.ctypes.data, val.ctypes.data) == sa.OTHER_ERROR
    assert lib.spmv_csr_sort_rows(2, ptr.ctypes.data, None, val.ctypes.data) == sa.OTHER_ERROR
    assert lib.spmv_csr_sort_rows(2, ptr.ctypes.data, col.ctypes.data, None) == sa.OTHER_ERROR
    dec = np.array([0, 3, 2], np.int64)  # decreasing offsets: a negative row length
    assert lib.spmv_csr_sort_rows(2, dec.ctypes.data, col.ctypes.data, val.ctypes.data) == sa.OTHER_ERROR
    assert np.array_equal(col, [1, 0, 2])  # refused calls write nothing
    empty = np.zeros(1, np.int64)
    assert lib.spmv_csr_sort_rows(0, empty.ctypes.data, None, None) == sa.SUCCESS
    with pytest.raises(sa.SpmvError):
        sa.csr_sort_rows(2, dec, col, val)


@pytest.mark.parametrize("h", [0, -1, 65])
def test_cpu_cmrs_refuses_strip_heights(h):
    """spmv_cpu_cmrs keeps per-strip sums in a fixed array: a strip height
    outside 1..64 (the builder's range) is refused, y untouched."""
    lib = sa.host_lib()
    sp = np.array([0, 1], np.int64)
    tag = np.zeros(1, np.uint8)
    col = np.zeros(1, np.int32)
    val = np.ones(1)
    x = np.ones(1)
    y = np.full(1, 7.0)
    rc = lib.spmv_cpu_cmrs(1, h, 1, sp.ctypes.data, tag.ctypes.data, col.ctypes.data, val.ctypes.data,
                           x.ctypes.data, y.ctypes.data, 1)
    assert rc == sa.OTHER_ERROR and y[0] == 7.0


@pytest.mark.parametrize("ties", ["first", "id"])
def test_rmat_bench_layout_same_y(ties):
    """bench.py's R-MAT layout (column_relabel + csr_sort_rows, rmat_layout)
    on a small R-MAT: the relabelled, row-sorted CSR on x[order] gives the
    original matrix's y within the parity rule (the sort changes each row's
    summation order, so not bit for bit), and the CPU CSR loop over it too."""
    import bench

    m = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=2)
    ptr, col, val = sa.csr_from_coo(m)
    args = type("A", (), {"relabel": "yes", "relabel_ties": ties})()
    col2, xh, hot, layout, order2 = bench.rmat_layout(args, m.n_rows, ptr, col, val)
    assert hot == 0 and "relabelled" in layout
    order, newid, _ = sa.column_relabel(m.n_cols, sa.csr_from_coo(m)[1], ties)
    assert np.array_equal(order2, order) and np.array_equal(xh, sa.ramp_x(m.n_cols)[order])
    for r in range(0, m.n_rows, 997):
        a, b = int(ptr[r]), int(ptr[r + 1])
        assert np.all(np.diff(col2[a:b]) >= 0)
    rows = np.repeat(np.arange(m.n_rows, dtype=np.int32), np.diff(ptr))
    x0 = sa.ramp_x(m.n_cols)
    y_ref = oracle.file_order_spmv(m.n_rows, m.row, m.col, m.val, x0)
    y = oracle.file_order_spmv(m.n_rows, rows, col2, val, xh)
    assert oracle.parity(y, y_ref, m.row, m.col, m.val, x0, m.n_rows).size == 0
    yc = np.empty(m.n_rows)
    assert sa.host_lib().spmv_cpu_csr(m.n_rows, ptr.ctypes.data, col2.ctypes.data, val.ctypes.data,
                                      xh.ctypes.data, yc.ctypes.data, 0) == sa.SUCCESS
    assert oracle.parity(yc, y_ref, m.row, m.col, m.val, x0, m.n_rows).size == 0


def _rmat_like_ptr(n=200_000, seed=3):
    rng = np.random.default_rng(seed)
    lens = (rng.pareto(1.2, n) * 3).astype(np.int64)
    return np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)


@pytest.mark.parametrize("w", [0.0, 2.0])
def test_partition_calibrated_uniform_rate_is_weighted(w):
    """Times proportional to each old shard's weighted cost (one rate for
    all) give exactly the weighted partition back."""
    ptr = _rmat_like_ptr()
    n = ptr.size - 1
    old = sa.partition_rows(n, ptr, 8, align=1024, row_weight=w or 1e-300)
    W = np.diff(ptr[old]) + w * np.diff(old)
    new = sa.partition_rows_calibrated(n, ptr, 8, old, 1e-6 * W, align=1024, row_weight=w)
    assert np.array_equal(new, sa.partition_rows(n, ptr, 8, align=1024, row_weight=w or 1e-300))


def test_partition_calibrated_balances_measured_cost():
    """A shard measured 3x slower per unit gives rows away; every new range
    then holds 1/parts of the calibrated cost (within one aligned block)."""
    ptr = _rmat_like_ptr()
    n, w, parts = ptr.size - 1, 2.0, 4
    old = sa.partition_rows(n, ptr, parts, align=1024, row_weight=w)
    W = np.diff(ptr[old]) + w * np.diff(old)
    ms = W * np.array([3.0, 1.0, 1.0, 1.0]) * 1e-6
    new = sa.partition_rows_calibrated(n, ptr, parts, old, ms, align=1024, row_weight=w)
    assert new[0] == 0 and new[-1] == n and np.all(np.diff(new) >= 0) and np.all(new[1:-1] % 1024 == 0)
    assert new[1] < old[1]

    def prefix(r):  # restatement of the cost model
        c = 0.0
        for g in range(parts):
            lo, hi = old[g], old[g + 1]
            if r >= hi:
                c += ms[g]
                continue
            if r > lo:
                c += ms[g] * ((ptr[r] - ptr[lo]) + w * (r - lo)) / W[g]
            break
        return c

    tot = ms.sum()
    blk = max(ms[g] / W[g] * (ptr[min(r + 1024, n)] - ptr[r] + w * 1024)
              for g in range(parts) for r in range(int(old[g]), int(old[g + 1]), 1024))
    for p in range(1, parts):
        assert abs(prefix(int(new[p])) - tot * p / parts) <= blk


def test_partition_calibrated_bad_input():
    ptr = _rmat_like_ptr(10_000)
    n = ptr.size - 1
    with pytest.raises(sa.SpmvError):
        sa.partition_rows_calibrated(n, ptr, 4, np.array([0, 5000, n - 1]), [1.0, 1.0])  # does not end at n
    with pytest.raises(sa.SpmvError):
        sa.partition_rows_calibrated(n, ptr, 4, np.array([0, 5000, n]), [1.0, -1.0])


@pytest.mark.parametrize("parts", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("kind", ["ragged", "empty_rows", "rmat"])
def test_row_shards_reassemble(parts, kind):
    """The drivers' --gpus N path on the host: spmv_partition_rows cuts the
    rows, spmv_coo_row_shard hands each shard its entries in file order with
    local row ids, each shard's CSR loop writes y[lo:hi] — the concatenation
    is bit-identical to the unsharded loop (rows never straddle shards),
    every entry lands in exactly one shard."""
    L = sa.host_lib()
    if kind == "ragged":
        m = sa.gen_random(3001, 2500, 0, 90, seed=4)
    elif kind == "empty_rows":
        m = sa.read_mtx(GOLDEN / "empty_rows.mtx")
    else:
        m = sa.gen_rmat(20_000, 200_000, scale=15, seed=3)
    x = np.random.default_rng(5).uniform(-1, 1, m.n_cols)
    ptr, col, val = sa.csr_from_coo(m)
    full = np.empty(m.n_rows)
    assert L.spmv_cpu_csr(m.n_rows, sa._ptr(ptr), sa._ptr(col), sa._ptr(val), sa._ptr(x), sa._ptr(full), 1) == 0
    bounds = np.empty(parts + 1, np.int64)
    assert L.spmv_partition_rows(m.n_rows, sa._ptr(ptr), parts, 1024, sa._ptr(bounds)) == 0
    y = np.full(m.n_rows, np.nan)
    total = 0
    for g in range(parts):
        lo, hi = int(bounds[g]), int(bounds[g + 1])
        n = L.spmv_coo_row_shard(m.nnz, sa._ptr(m.row), sa._ptr(m.col), sa._ptr(m.val), lo, hi, None, None, None)
        r, c, v = np.empty(max(n, 1), np.int32), np.empty(max(n, 1), np.int32), np.empty(max(n, 1))
        assert L.spmv_coo_row_shard(m.nnz, sa._ptr(m.row), sa._ptr(m.col), sa._ptr(m.val), lo, hi, sa._ptr(r),
                                    sa._ptr(c), sa._ptr(v)) == n
        total += n
        keep = (m.row >= lo) & (m.row < hi)  # file order kept
        assert np.array_equal(r[:n], m.row[keep] - lo) and np.array_equal(c[:n], m.col[keep])
        s = sa.Coo(hi - lo, m.n_cols, r[:n], c[:n], v[:n])
        sp, sc, sv = sa.csr_from_coo(s)
        if hi > lo:
            assert L.spmv_cpu_csr(hi - lo, sa._ptr(sp), sa._ptr(sc), sa._ptr(sv), sa._ptr(x),
                                  sa._ptr(y[lo:hi]), 1) == 0
    assert total == m.nnz
    assert np.array_equal(y.view(np.int64), full.view(np.int64))


def test_row_shard_bad_arguments():
    L = sa.host_lib()
    assert L.spmv_coo_row_shard(-1, None, None, None, 0, 1, None, None, None) == -1
    assert L.spmv_coo_row_shard(0, None, None, None, 5, 3, None, None, None) == -1
    assert L.spmv_coo_row_shard(0, None, None, None, 0, 0, None, None, None) == 0


@pytest.mark.parametrize("kind,groups", [("rmat", 32), ("rmat", 64), ("random", 7), ("empty_rows", 3), ("one", 1),
                                         ("tall", 5)])
def test_csrg_layout(kind, groups):
    """Column-grouped CSR: entries group after group (groups of whole 16-column
    x lines), each pair one (row, group) with its entries in CSR order, rows
    ascending in a group; blk_off / pair_row name every pair's row block and
    row; the pair sums added per row in group order give the CSR product."""
    if kind == "rmat":
        m = sa.gen_rmat(100_000, 1_000_000, scale=17, seed=2)
    elif kind == "random":
        m = sa.gen_random(5_000, 3_000, 0, 50, seed=3)
    elif kind == "empty_rows":
        m = sa.read_mtx(GOLDEN / "empty_rows.mtx")
    elif kind == "tall":  # several row blocks, trailing empty block
        m = sa.gen_random(20_000, 900, 0, 4, seed=5)
    else:
        m = sa.gen_random(100, 100, 0, 3, seed=1)
    ptr, col, val = sa.csr_from_coo(m)
    g = sa.csrg_build(m.n_rows, ptr, col, val, groups)
    n, pp, nnz, nb, B = g["n_pairs"], g["pair_ptr"], m.nnz, g["nb"], int(sa.host_lib().spmv_csrg_block_rows())
    assert nb == (m.n_rows + B - 1) // B
    assert pp[0] == 0 and pp[n] == nnz and (np.diff(pp) > 0).all()
    grp = np.array([sa.host_lib().spmv_csrg_group(int(c), groups) for c in g["col_g"][:nnz]])
    assert (np.diff(grp) >= 0).all()  # group-major
    assert all(sa.host_lib().spmv_csrg_group(c, groups) == sa.host_lib().spmv_csrg_group(c | 15, groups)
               for c in range(0, 4096, 16))  # a 128-B line is in one group
    off = g["blk_off"].reshape(groups, nb + 1).astype(np.int64)
    assert off[0, 0] == 0 and off[-1, -1] == n and (np.diff(off.ravel()) >= 0).all()
    pair_row = np.empty(n, np.int64)
    pair_grp = np.empty(n, np.int64)
    for gg in range(groups):
        for b in range(nb):
            pair_row[off[gg, b]:off[gg, b + 1]] = b * B + g["pair_row"][off[gg, b]:off[gg, b + 1]].astype(np.int64)
            pair_grp[off[gg, b]:off[gg, b + 1]] = gg
    for gg in range(groups):  # rows ascending and distinct inside a group
        rows = pair_row[pair_grp == gg]
        assert (np.diff(rows) > 0).all()
    for k in range(0, n, max(1, n // 500)):  # a pair = that row's entries of that group, CSR order
        e0, e1 = pp[k], pp[k + 1]
        assert (grp[e0:e1] == pair_grp[k]).all()
        r = pair_row[k]
        row_cols = col[ptr[r]:ptr[r + 1]]
        row_grp = np.array([sa.host_lib().spmv_csrg_group(int(c), groups) for c in row_cols])
        assert np.array_equal(g["col_g"][e0:e1], row_cols[row_grp == pair_grp[k]])
    x = np.random.default_rng(1).uniform(-1, 1, m.n_cols)
    prod = g["val_g"][:nnz] * x[g["col_g"][:nnz]]
    yp = np.add.reduceat(prod, pp[:-1]) if n else np.zeros(0)
    y = np.zeros(m.n_rows)
    np.add.at(y, pair_row, yp)
    y_ref = np.zeros(m.n_rows)
    np.add.at(y_ref, m.row, m.val * x[m.col])
    assert np.allclose(y, y_ref, rtol=1e-12, atol=1e-12)
