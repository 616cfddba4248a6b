"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker or the timed CPU baseline.
The product path never imports it.  See oracle.c for what each function
restates (reference file:line) and why parity is UNPINNED against the
reference's own outputs (no fixtures exist; building/running the
reference was denied).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"

_i64 = ctypes.c_longlong


class OracleFileError(OSError):
    """The reference's FileError (code 3): missing or rejected .mtx."""

    rc = 3


_vp = ctypes.c_void_p
_lib = None


def build() -> Path:
    """Compile liboracle.so with gcc (no reference code is compiled)."""
    src = HERE / "oracle.c"
    if not LIB.exists() or LIB.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["gcc", "-O2", "-std=c11", "-fPIC", "-fopenmp", "-shared", str(src),
                        "-o", str(LIB), "-lm"], check=True)
    return LIB


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        path = os.environ.get("SPMV_ORACLE_LIB")  # `make test-san`: the sanitizer build
        if not path:
            build()
        L = ctypes.CDLL(str(path or LIB))
        L.oracle_read_info.argtypes = [ctypes.c_char_p, ctypes.POINTER(_i64), ctypes.POINTER(_i64),
                                       ctypes.POINTER(_i64), ctypes.POINTER(ctypes.c_int)]
        L.oracle_read_mtx.argtypes = [ctypes.c_char_p, _vp, _vp, _vp]
        for name in ("oracle_file_order_spmv", "oracle_ref_csr", "oracle_ref_ell", "oracle_ref_sell",
                     "oracle_ref_cmrs"):
            getattr(L, name).argtypes = [_i64, _i64, _vp, _vp, _vp, _vp, _vp]
            getattr(L, name).restype = None
        L.oracle_check.argtypes = [_i64, _vp, _vp, ctypes.c_double]
        L.oracle_check.restype = _i64
        L.oracle_cpu_csr_omp.argtypes = [_i64, _vp, _vp, _vp, _vp, _vp, ctypes.c_int]
        L.oracle_cpu_csr_omp.restype = ctypes.c_double
        L.oracle_max_threads.restype = ctypes.c_int
        L.oracle_sweep.argtypes = [_vp, _i64, ctypes.c_int]
        L.oracle_sweep.restype = None
        _lib = L
    return _lib


def read_mtx(path):
    """-> (n_rows, n_cols, row, col, val, symmetric) in file order, or
    raises OracleFileError (the reference's FileError, code 3)."""
    L = lib()
    m, n, z, flags = _i64(), _i64(), _i64(), ctypes.c_int()
    p = str(path).encode()
    if L.oracle_read_info(p, ctypes.byref(m), ctypes.byref(n), ctypes.byref(z), ctypes.byref(flags)):
        raise OracleFileError(f"oracle: cannot read {path}")
    row = np.empty(z.value, np.int32)
    col = np.empty(z.value, np.int32)
    val = np.empty(z.value, np.float64)
    if L.oracle_read_mtx(p, row.ctypes.data, col.ctypes.data, val.ctypes.data):
        raise OracleFileError(f"oracle: cannot read entries of {path}")
    return m.value, n.value, row, col, val, bool(flags.value & 1)


def _run(name, n_rows, row, col, val, x):
    y = np.empty(max(n_rows, 1), np.float64)
    row = np.ascontiguousarray(row, np.int32)
    col = np.ascontiguousarray(col, np.int32)
    val = np.ascontiguousarray(val, np.float64)
    x = np.ascontiguousarray(x, np.float64)
    getattr(lib(), name)(n_rows, row.shape[0], row.ctypes.data, col.ctypes.data, val.ctypes.data,
                         x.ctypes.data, y.ctypes.data)
    return y[:n_rows]


def file_order_spmv(n_rows, row, col, val, x):
    """check_result's expected y (reference inc/helper_functions.h:184-236)."""
    return _run("oracle_file_order_spmv", n_rows, row, col, val, x)


def _row_sorted(row, col, val):
    order = np.argsort(row, kind="stable")
    return row[order], col[order], val[order]


def ref_kernel(fmt, n_rows, row, col, val, x):
    """Replay the reference OpenCL kernel of `fmt` (its summation order)
    on a row-sorted copy of the entries.  fmt in csr/ell/sell/cmrs; the
    reference COO kernel's order is nondeterministic (CAS atomics), so
    'coo' returns the file-order sum its CPU path would give."""
    if fmt == "coo":
        return file_order_spmv(n_rows, row, col, val, x)
    r, c, v = _row_sorted(row, col, val)
    name = {"csr": "oracle_ref_csr", "ell": "oracle_ref_ell", "sell": "oracle_ref_sell",
            "cmrs": "oracle_ref_cmrs"}[fmt]
    return _run(name, n_rows, r, c, v, x)


def parity(y, y_ref, row, col, val, x, n_rows, rel=1e-6):
    """SURVEY.md §8d criterion, per row:
    |y - y_ref| <= rel * max(|y_ref|, sum_j |a_ij x_j|).  -> bad row ids."""
    mag = np.bincount(row, weights=np.abs(val * x[col]), minlength=n_rows)[:n_rows]
    scale = np.maximum(np.abs(y_ref), mag)
    diff = np.abs(np.asarray(y) - y_ref)
    return np.nonzero(~(diff <= rel * scale))[0]


def cpu_csr_omp(n_rows, row_ptr, col, val, x, y, threads=0) -> float:
    """csr.c:285-309 compute_using_cpu (OpenMP); returns seconds."""
    return lib().oracle_cpu_csr_omp(n_rows, row_ptr.ctypes.data, col.ctypes.data, val.ctypes.data,
                                    x.ctypes.data, y.ctypes.data, threads)


def sweep(buf: np.ndarray, threads=0) -> None:
    """Write every 64th byte of buf from all threads (host cache eviction
    between cold CPU passes)."""
    lib().oracle_sweep(buf.ctypes.data, buf.nbytes, threads)


def max_threads() -> int:
    return lib().oracle_max_threads()
