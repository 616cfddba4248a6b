#!/usr/bin/env python3
"""Diagnostic: tiled CSR with the hot table (H) vs without, both with a plan,
on the 1e6-row R-MAT of test_csr_hot_bit_identical; prints the rows that
differ (bitwise) and whether they are rows spanning tiles."""
from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "opencl-spmv-algorithms_amd"), str(REPO)]
import spmv_amd as sa  # noqa: E402


def main():
    import torch

    dev = torch.device("cuda:0")
    m = sa.gen_rmat(1_000_000, 10_000_000, scale=20, seed=1)
    ptr, _, _ = sa.csr_from_coo(m)
    span = (ptr[1:] - 1) // 1536 > ptr[:-1] // 1536
    x = torch.from_numpy(np.random.default_rng(6).uniform(-1, 1, m.n_cols)).to(dev)
    outs = {}
    for H, fused in ((0, "0"), (0, "1"), (1, "1"), (4096, "1"), (4096, "0")):
        os.environ["SPMV_TILED_FUSED_CARRY"] = fused
        dm = sa.to_device(m, "csr", dev, variant=4, hot=H)
        for rep in range(2):
            y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
            dm.run(x, y)
            torch.cuda.synchronize()
            outs[(H, fused, rep)] = y.cpu().numpy()
    ref0 = outs[(0, "0", 0)]
    ref = ref0.view(np.int64)
    for k, v in outs.items():
        d = np.nonzero(v.view(np.int64) != ref)[0]
        print(f"H={k[0]} fused={k[1]} rep={k[2]} lib={os.environ.get('SPMV_HIP_LIB', 'tree')}: {d.size} rows differ, "
              f"{int(span[d].sum()) if d.size else 0} of them span tiles; first {d[:5].tolist()}", flush=True)
        if d.size:
            r = d[0]
            print(f"   row {r}: len {ptr[r + 1] - ptr[r]}, {v[r]!r} vs {ref0[r]!r}", flush=True)


if __name__ == "__main__":
    main()
