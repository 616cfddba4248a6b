"""Generate the committed parity fixtures in tests/golden/.

The reference ships no fixtures and its only inputs,
databases/cant*.mtx, are Git-LFS pointers; running it was denied
(SURVEY.md §8c).  These small Matrix Market files therefore come from this
script, and their expected y = A·x with x[j] = j (the reference's input
vector, reference csr.c:95-99) is computed with scipy.sparse — an
implementation independent of both the oracle and the product.  Each case
targets one hidden assumption of the reference.

    python tests/golden/make_golden.py      # rewrites *.mtx, *.y.npy, manifest.json
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import scipy.sparse as sp

HERE = Path(__file__).resolve().parent


def write(name, n_rows, n_cols, r, c, v, *, banner="real general", header_extra="", desc=""):
    r = np.asarray(r, np.int64)
    c = np.asarray(c, np.int64)
    v = np.asarray(v, np.float64)
    lines = [f"%%MatrixMarket matrix coordinate {banner}\n"]
    lines.append(header_extra)
    lines.append(f"{n_rows} {n_cols} {len(r)}\n")
    pattern = "pattern" in banner
    integer = "integer" in banner
    for ri, ci, vi in zip(r, c, v):
        if pattern:
            lines.append(f"{ri + 1} {ci + 1}\n")
        elif integer:
            lines.append(f"{ri + 1} {ci + 1} {int(vi)}\n")
        else:
            lines.append(f"{ri + 1} {ci + 1} {float(vi)!r}\n")
    (HERE / f"{name}.mtx").write_text("".join(lines))
    vals = np.ones(len(r)) if pattern else v
    A = sp.coo_matrix((vals, (r, c)), shape=(n_rows, n_cols)).tocsr()  # duplicates summed
    x = np.arange(n_cols, dtype=np.float64)
    y = A @ x if len(r) else np.zeros(n_rows)
    np.save(HERE / f"{name}.y.npy", np.asarray(y, np.float64))
    return dict(name=name, n_rows=n_rows, n_cols=n_cols, nnz=int(len(r)), banner=banner, desc=desc)


def main():
    rng = np.random.default_rng(20261015)
    cases = []

    # 1. hand-computed: y = [1*0 + 2*2, 3*1, 4*0 + 5*1 + 6*2] = [4, 3, 17]
    cases.append(write("hand3", 3, 3, [0, 0, 1, 2, 2, 2], [0, 2, 1, 0, 1, 2], [1, 2, 3, 4, 5, 6],
                       desc="hand-computed y = [4, 3, 17]"))

    # 2. empty rows, including the first and the last (reference A3/A7/A9)
    n, m = 100, 90
    rows = [i for i in range(n) if i not in (0, 1, 17, 50, 51, 52, 99)]
    r, c, v = [], [], []
    for i in rows:
        k = rng.integers(1, 9)
        r += [i] * k
        c += list(rng.integers(0, m, k))
        v += list(rng.uniform(-1, 1, k))
    cases.append(write("empty_rows", n, m, r, c, v, desc="empty rows incl. first and last"))

    # 3. N % 8, % 32, % 64 != 0 (CMRS tail strip, SELL tail slice, ELL ld)
    n = 67
    r, c, v = [], [], []
    for i in range(n):
        k = 1 + (i * 7) % 11
        r += [i] * k
        c += list(rng.integers(0, n, k))
        v += list(rng.uniform(-2, 2, k))
    cases.append(write("n67", n, n, r, c, v, desc="N=67: N%8, N%32, N%64 != 0"))

    # 4. duplicate entries (summed, like the reference's += )
    cases.append(write("duplicates", 4, 4, [0, 0, 0, 2, 2, 3, 3, 3], [1, 1, 1, 0, 0, 3, 3, 2],
                       [1.5, 2.5, -1.0, 0.25, 0.75, 1, 1, 1], desc="repeated (row,col) entries"))

    # 5. unsorted (column-major, the shape of cant.mtx, reference coo.c:43)
    n = 200
    A = sp.random(n, n, density=0.05, random_state=7, format="coo")
    order = np.lexsort((A.row, A.col))
    cases.append(write("colmajor", n, n, A.row[order], A.col[order], A.data[order] * 10 - 5,
                       desc="entries in column-major (unsorted) order"))

    # 6. symmetric banner: only the listed (lower) entries are used (A12)
    n = 50
    L = sp.tril(sp.random(n, n, density=0.1, random_state=3, format="coo")).tocoo()
    d = np.arange(n)
    rr = np.concatenate([L.row, d])
    cc = np.concatenate([L.col, d])
    vv = np.concatenate([L.data, np.full(n, 4.0)])
    o = np.lexsort((rr, cc))
    cases.append(write("symmetric_lower", n, n, rr[o], cc[o], vv[o], banner="real symmetric",
                       desc="symmetric banner, lower triangle, NOT mirrored"))

    # 7. the longest row is the last row (reference ell.c:73-101 misses it)
    n = 40
    r, c, v = [], [], []
    for i in range(n):
        k = 3 if i < n - 1 else 35
        r += [i] * k
        c += list(rng.choice(n, k, replace=False))
        v += list(rng.uniform(-1, 1, k))
    cases.append(write("longest_last", n, n, r, c, v, desc="longest row is the last row"))

    # 8. integer and pattern banners
    cases.append(write("integer", 5, 6, [0, 1, 2, 3, 4, 4], [5, 4, 3, 2, 1, 0], [3, -2, 7, 1, 9, -4],
                       banner="integer general", desc="integer values"))
    cases.append(write("pattern", 5, 5, [0, 0, 1, 3, 4], [0, 4, 2, 3, 1], [1] * 5,
                       banner="pattern general", desc="pattern: every value 1.0 (documented)"))

    # 9. one long row spanning several COO tiles (1024 entries) + short rows
    n = 30
    r = [0] * 3 + [7] * 5000 + [8] * 2 + [29] * 1500
    c = list(rng.integers(0, 4000, len(r)))
    v = list(rng.uniform(-1, 1, len(r)))
    cases.append(write("long_rows", n, 4000, r, c, v, desc="rows of 5000 and 1500 entries"))

    # 10. no entries at all
    cases.append(write("all_empty", 10, 10, [], [], [], desc="nz = 0"))

    # 11. wide (M >> N) and tall (N >> M)
    cases.append(write("wide", 5, 1000, [0, 1, 2, 3, 4, 4], [999, 500, 0, 1, 998, 2],
                       [1, 2, 3, 4, 5, 6], desc="5 x 1000"))
    n = 300
    cases.append(write("tall", n, 3, np.arange(n), np.arange(n) % 3, rng.uniform(-1, 1, n),
                       desc="300 x 3"))

    # 12. comment lines and a blank line before the size line
    cases.append(write("comments", 3, 3, [0, 1, 2], [0, 1, 2], [1.0, 2.0, 3.0],
                       header_extra="% a comment\n%another\n\n", desc="comments + blank line"))

    # 13. ragged random (row lengths 0..60) in random entry order
    n = 500
    lens = rng.integers(0, 61, n)
    r = np.repeat(np.arange(n), lens)
    c = rng.integers(0, n, r.size)
    v = rng.uniform(-1, 1, r.size)
    perm = rng.permutation(r.size)
    cases.append(write("ragged_shuffled", n, n, r[perm], c[perm], v[perm],
                       desc="ragged rows 0..60, shuffled entry order"))

    # 14. a 1x1 matrix
    cases.append(write("one", 1, 1, [0], [0], [2.5], desc="1 x 1"))

    (HERE / "manifest.json").write_text(json.dumps(cases, indent=1) + "\n")
    print(f"wrote {len(cases)} fixtures to {HERE}")


if __name__ == "__main__":
    main()
