"""Diagnostic: the COO single pass (1,536-entry tiles, no carry kernel) against
the carry pass (512-entry tiles below a mean row of 96, then
coo_carry_kernel) as the grid shrinks: row prefixes of the cant-like matrix
and the HYB tails of it (entries past K per row), cold (512 MiB read before
every launch).  Run under rocprofv3 --kernel-trace; spans per phase come
from the trace (tools/trace_segments.py).

    rocprofv3 --kernel-trace --output-format csv -d D -o run -- \\
        python3 tools/coo_grid_probe.py
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


def matrices():
    m = sa.gen_cantlike(0, 1)
    ptr, col, val = sa.csr_from_coo(m)
    out = []
    for frac in (1.0, 0.5, 0.35, 0.25, 0.125):
        n = int(m.n_rows * frac)
        z = int(ptr[n])
        rows = np.repeat(np.arange(n, dtype=np.int32), np.diff(ptr[: n + 1]))
        out.append((f"cant rows<{n}", sa.Coo(n, m.n_cols, rows, col[:z].copy(), val[:z].copy(), False, "")))
    for K in (52, 64, 72):
        h = sa.hyb_build(m.n_rows, ptr, col, val, ki=2, K=K)
        t = h["tail_nnz"]
        out.append((f"tail K={K}", sa.Coo(m.n_rows, m.n_cols, h["tail_row"][:t].copy(), h["tail_col"][:t].copy(),
                                          h["tail_val"][:t].copy(), False, "")))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda:0")
    sp = torch.cuda.current_stream(dev).cuda_stream
    P = probe_lib()
    scratch = torch.empty(FLUSH_BYTES, dtype=torch.uint8, device=dev)
    fsink = torch.zeros(16, dtype=torch.int32, device=dev)
    out = {}
    phase = 0
    for label, mm in matrices():
        x = torch.from_numpy(sa.ramp_x(mm.n_cols)).to(dev)
        for mode, kw in (("single", {"coo_tail": True}), ("carry", {"coo_tail": False})):
            try:
                dm = sa.to_device(mm, "coo", dev, hot=0, **kw)
            except sa.SpmvError as e:
                out[f"{label} {mode}"] = {"na": str(e)}
                continue
            y = torch.zeros(mm.n_rows, dtype=torch.float64, device=dev)
            dm.run(x, y)
            torch.cuda.synchronize()
            assert P.spmv_probe_tag(phase, sp) == 0
            for _ in range(a.reps):
                assert P.spmv_probe_flush_read(scratch.data_ptr(), FLUSH_BYTES, fsink.data_ptr(), sp) == 0
                dm.run(x, y)
            assert P.spmv_probe_tag(999, sp) == 0  # the next setup lands in an ignored phase
            torch.cuda.synchronize()
            bad, _ = sa.check(mm, sa.ramp_x(mm.n_cols), y.cpu().numpy())
            out[f"{label} {mode}"] = {"phase": phase, "nnz": mm.nnz, "rows": mm.n_rows, "parity_ok": bad == 0}
            phase += 1
            del dm
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
