#!/usr/bin/env python3
"""Kernel-variant sweep on the bench workload (B cant-like copies).

Prints one line per variant: mean kernel ms over back-to-back launches
(HIP events on the launch stream), effective GB/s of algorithmic bytes,
and GB/s of stored bytes.  Variants are interleaved over rounds in ONE
process (cdna_hip_programming.md §5.4 rule 24).
    python tools/sweep.py [--copies 32] [--rounds 3] [--matrix cantlike|rmat]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "opencl-spmv-algorithms_amd"), str(REPO)]
import spmv_amd as sa  # noqa: E402

VARIANTS = [
    ("csr", {"lanes": 8, "variant": 1}), ("csr", {"lanes": 16, "variant": 1}),
    ("csr", {"lanes": 2, "variant": 2}), ("csr", {"lanes": 4, "variant": 2}), ("csr", {"lanes": 8, "variant": 2}),
    ("csr", {"lanes": 2, "variant": 3}), ("csr", {"lanes": 4, "variant": 3}), ("csr", {"lanes": 8, "variant": 3}),
    ("csr", {"variant": 4}),
    ("ell", {"ki": 1}), ("ell", {"ki": 2}),
    ("sell", {"C": 64, "sigma": 1, "ki": 2}), ("sell", {"C": 64, "sigma": 256, "ki": 2}),
    ("sell", {"C": 64, "sigma": 1024, "ki": 2}), ("sell", {"C": 64, "sigma": 1024, "ki": 1}),
    ("sell", {"C": 64, "sigma": 512, "ki": 1}), ("sell", {"C": 64, "sigma": 256, "ki": 1}),
    ("sell", {"C": 64, "sigma": 512, "ki": 2}),
    ("cmrs", {"h": 8}), ("cmrs", {"h": 16}), ("cmrs", {"h": 32}),
    ("coo", {}),
    ("csr16", {"lanes": 4}), ("csr16", {"lanes": 2}), ("csr16", {"lanes": 8}),
    # skewed matrices (--matrix rmat): HYB vs tiled CSR
    ("hyb", {"env": {}}),
    ("hyb", {"ki": 1, "env": {}}),
    ("csr", {"variant": 4, "env": {}}),
    ("csr", {"variant": 4, "hot": 0, "env": {}}),
    ("csr", {"variant": 4, "hot": 1 << 18, "env": {}}),
    ("csr", {"variant": 4, "hot": 1 << 20, "env": {}}),
    ("csr", {"variant": 4, "env": {"stream_nt": 0}}),
    ("coo", {"xwin": True, "env": {}}),
    ("csr", {"env": {"xwin_remap": 1}}),
    ("csr", {"env": {"xwin_remap": 0}}),
    ("sell", {"env": {"xwin_remap": 1}}),
    ("sell", {"env": {"xwin_remap": 0}}),
    ("sell", {"C": 64, "sigma": 65536, "ki": 1, "env": {}}),
    ("sell", {"C": 64, "sigma": 1 << 20, "ki": 1, "env": {}}),
    ("sell", {"C": 64, "sigma": 1 << 24, "ki": 1, "env": {}}),
    ("sell", {"C": 64, "sigma": 1 << 24, "ki": 2, "env": {}}),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--copies", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--matrix", default="cantlike")
    ap.add_argument("--only", default="", help="comma list of formats")
    ap.add_argument("--env-only", action="store_true", help="only the variants that set env knobs")
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda:0")
    m = sa.gen_cantlike(0, a.copies) if a.matrix == "cantlike" else sa.gen_rmat()
    b = sa.bytes_alg(m.n_rows, m.n_cols, m.nnz)
    x = torch.from_numpy(sa.ramp_x(m.n_cols)).to(dev)
    y = torch.empty(m.n_rows, dtype=torch.float64, device=dev)
    variants = [v for v in VARIANTS if not a.only or v[0] in a.only.split(",")]
    if a.env_only:
        variants = [v for v in variants if "env" in v[1] or v[1].get("xwin")]
    if a.matrix != "cantlike":
        variants = [v for v in variants if v[0] != "ell"]
    res = {i: [] for i in range(len(variants))}
    stored = {}
    for r in range(a.rounds):
        for i, (fmt, kw) in enumerate(variants):
            kw = dict(kw)
            env = kw.pop("env", {})  # spmv_set_option switches for this variant
            for k, v in env.items():
                sa.set_option(k, v)
            dm = sa.to_device(m, fmt, dev, **kw)
            stored[i] = dm.stored_bytes
            s = torch.cuda.current_stream()
            for _ in range(5):
                dm.run(x, y, s)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
            ev[0].record(s)
            for k in range(a.reps):
                dm.run(x, y, s)
                ev[k + 1].record(s)
            torch.cuda.synchronize()
            res[i].append(float(np.mean([ev[k].elapsed_time(ev[k + 1]) for k in range(a.reps)])))
            del dm
            torch.cuda.empty_cache()
            for k in env:
                sa.set_option(k, None)
    out = []
    for i, (fmt, kw) in enumerate(variants):
        ms = float(np.median(res[i]))
        row = dict(fmt=fmt, **kw, ms=round(ms, 5), GBs_alg=round(b / ms * 1e-6, 1),
                   GBs_stored=round(stored[i] / ms * 1e-6, 1), frac=round(b / ms * 1e-6 / 8000, 4),
                   spread=round((max(res[i]) - min(res[i])) / ms, 4))
        out.append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps({"matrix": a.matrix, "copies": a.copies, "bytes_alg": b,
                      "xcd_remap": sa.get_option("xcd_remap")}))


if __name__ == "__main__":
    main()
