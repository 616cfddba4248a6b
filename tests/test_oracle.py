"""The oracle (oracle/oracle.c) against the committed fixtures.

The reference has no tests or golden vectors of its own,
so the oracle is pinned here against independently computed expected
vectors (scipy.sparse, tests/golden/make_golden.py) and a hand-computed
case; parity with the reference's own outputs stays UNPINNED (no output of
the reference exists).
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import GOLDEN, golden_cases
from oracle import oracle

CASES = [c["name"] for c in golden_cases()]


def _load(name):
    n, m, r, c, v, sym = oracle.read_mtx(GOLDEN / f"{name}.mtx")
    return n, m, r, c, v, sym, np.load(GOLDEN / f"{name}.y.npy")


@pytest.mark.parametrize("name", CASES)
def test_file_order_sum_matches_golden(name):
    n, m, r, c, v, _, y_gold = _load(name)
    x = np.arange(m, dtype=np.float64)
    y = oracle.file_order_spmv(n, r, c, v, x)
    assert y.shape == y_gold.shape
    assert oracle.parity(y, y_gold, r, c, v, x, n, rel=1e-12).size == 0


@pytest.mark.parametrize("fmt", ["csr", "ell", "sell", "cmrs", "coo"])
@pytest.mark.parametrize("name", CASES)
def test_reference_kernel_replay_matches_golden(name, fmt):
    """Each replayed reference kernel (its summation order) gives check_result's y."""
    n, m, r, c, v, _, y_gold = _load(name)
    x = np.arange(m, dtype=np.float64)
    y = oracle.ref_kernel(fmt, n, r, c, v, x)
    assert oracle.parity(y, y_gold, r, c, v, x, n, rel=1e-12).size == 0


def test_hand_computed():
    n, m, r, c, v, _, y_gold = _load("hand3")
    y = oracle.file_order_spmv(n, r, c, v, np.arange(m, dtype=np.float64))
    assert y.tolist() == [4.0, 3.0, 17.0]
    assert y_gold.tolist() == [4.0, 3.0, 17.0]


def test_symmetric_banner_is_not_mirrored():
    n, m, r, c, v, sym, _ = _load("symmetric_lower")
    assert sym
    assert np.all(r >= c)  # only the stored lower triangle is multiplied


def test_rejections(tmp_path):
    bad = {
        "complex.mtx": "%%MatrixMarket matrix coordinate complex general\n2 2 1\n1 1 1.0 0.0\n",
        "array.mtx": "%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n",
        "nobanner.mtx": "2 2 1\n1 1 1.0\n",
        "short.mtx": "%%MatrixMarket matrix coordinate real general\n2 2 3\n1 1 1.0\n",
        "range.mtx": "%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1.0\n",
    }
    for name, text in bad.items():
        p = tmp_path / name
        p.write_text(text)
        with pytest.raises(OSError):
            oracle.read_mtx(p)
    with pytest.raises(OSError):
        oracle.read_mtx(tmp_path / "missing.mtx")


def test_absolute_epsilon_rule():
    """check_result's |y - y_ref| <= 1e-6 (reference helper_functions.h:11,221-231)."""
    import ctypes

    L = oracle.lib()
    ref = np.array([1.0, 2.0, 3.0])
    ok = ref + np.array([0.0, 9e-7, -9e-7])
    bad = ref + np.array([0.0, 0.0, 2e-6])
    assert L.oracle_check(3, ref.ctypes.data, ok.ctypes.data, ctypes.c_double(1e-6)) == -1
    assert L.oracle_check(3, ref.ctypes.data, bad.ctypes.data, ctypes.c_double(1e-6)) == 2
