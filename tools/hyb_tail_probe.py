"""Diagnostic: a HYB tail (the entries past K of every cant-like row) timed
as HYB (ELL part + accumulate-mode COO tail) and, on its own, as a plain COO
matrix (the single-pass, non-accumulating COO kernel), cold (512 MiB read
before every launch).  Run under rocprofv3 --kernel-trace; the kernel
durations per phase come from the trace (tools/trace_segments.py).

    rocprofv3 --kernel-trace --output-format csv -d D -o run -- \\
        python3 tools/hyb_tail_probe.py --k 72 52
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "opencl-spmv-algorithms_amd"))
sys.path.insert(0, str(ROOT / "tools"))
import spmv_amd as sa  # noqa: E402
from cant_single import FLUSH_BYTES, probe_lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, nargs="+", default=[72, 52])
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda:0")
    sp = torch.cuda.current_stream(dev).cuda_stream
    P = probe_lib()
    scratch = torch.empty(FLUSH_BYTES, dtype=torch.uint8, device=dev)
    fsink = torch.zeros(16, dtype=torch.int32, device=dev)
    m = sa.gen_cantlike(0, 1)
    ptr, col, val = sa.csr_from_coo(m)
    x = torch.from_numpy(sa.ramp_x(m.n_cols)).to(dev)
    out = {}
    phase = 0
    for K in a.k:
        h = sa.hyb_build(m.n_rows, ptr, col, val, ki=2, K=K)
        t = h["tail_nnz"]
        tail = sa.Coo(m.n_rows, m.n_cols, h["tail_row"][:t].copy(), h["tail_col"][:t].copy(),
                      h["tail_val"][:t].copy(), False, f"tail K={K}")
        for label, mm, fmt, kw in ((f"hyb K={K}", m, "hyb", {"hyb_k": K}),
                                   (f"tail K={K} as coo", tail, "coo", {}),
                                   (f"tail K={K} as coo, carry pass", tail, "coo", {"coo_tail": False})):
            dm = sa.to_device(mm, fmt, dev, **kw)
            y = torch.zeros(mm.n_rows, dtype=torch.float64, device=dev)
            dm.run(x, y)
            torch.cuda.synchronize()
            assert P.spmv_probe_tag(phase, sp) == 0
            for _ in range(a.reps):
                assert P.spmv_probe_flush_read(scratch.data_ptr(), FLUSH_BYTES, fsink.data_ptr(), sp) == 0
                dm.run(x, y)
            torch.cuda.synchronize()
            out[label] = {"phase": phase, "tail_nnz": t, "params": {k: v for k, v in dm.params.items()
                                                                    if isinstance(v, (int, float, str))}}
            phase += 1
            del dm
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
