"""Numpy/scipy stand-in for iterate.HipKernels: TEST INFRASTRUCTURE ONLY.

Used by the CPU tests to run the multi-rank orchestration of iterate.py
(partition, column renumbering, in-place all-reduce / all-gather over gloo)
without a GPU; the product path only ever uses HipKernels, and the GPU
tests run the same solvers through libspmv_hip.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch


class NumpyKernels:
    def __init__(self, loc):
        self.A = sp.csr_matrix((loc.val, (loc.row, loc.col)), shape=(loc.n_rows, loc.n_cols))

    def spmv(self, x_full, y):
        r = self.A.shape[0]
        y[:r] = torch.from_numpy(self.A @ x_full.numpy())

    def dot(self, n, a, b, out, ws):
        out[0] = float(np.dot(a[:n].numpy(), b[:n].numpy()))

    def axpy_ratio(self, n, num, den, sign, x, y):
        y[:n] += sign * (float(num[0]) / float(den[0])) * x[:n]

    def xpay_ratio(self, n, num, den, x, y):
        y[:n] = x[:n] + (float(num[0]) / float(den[0])) * y[:n]

    def scale_rsqrt(self, n, s, x, y):
        y[:n] = x[:n] / np.sqrt(float(s[0]))

    def dot_ws(self, n):
        return torch.empty(8, dtype=torch.uint8)


def laplacian_2d(k: int, shift: float = 0.0):
    """5-point Laplacian on a k x k grid (+ shift I): SPD, symmetric."""
    import spmv_amd as sa

    n = k * k
    idx = np.arange(n).reshape(k, k)
    rows, cols, vals = [idx.ravel()], [idx.ravel()], [np.full(n, 4.0 + shift)]
    for a, b in ((idx[:, :-1], idx[:, 1:]), (idx[:-1, :], idx[1:, :])):
        rows += [a.ravel(), b.ravel()]
        cols += [b.ravel(), a.ravel()]
        vals += [np.full(a.size, -1.0), np.full(a.size, -1.0)]
    r = np.concatenate(rows).astype(np.int32)
    c = np.concatenate(cols).astype(np.int32)
    v = np.concatenate(vals)
    o = np.lexsort((c, r))
    return sa.Coo(n, n, r[o], c[o], v[o], False, f"laplacian {k}x{k}")


def numpy_power(m, iters, x0):
    A = sp.csr_matrix((m.val, (m.row, m.col)), shape=(m.n_rows, m.n_cols))
    x = x0 / np.linalg.norm(x0)
    hist = np.empty((iters, 2))
    for i in range(iters):
        y = A @ x
        hist[i] = (x @ y, y @ y)
        x = y / np.sqrt(y @ y)
    return hist, x
