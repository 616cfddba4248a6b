#!/usr/bin/env python3
"""coo_stamps — where the single-pass COO kernel's time goes, per tile.

Lab only.  Runs the single-pass COO (coo_tail=True, no hot table) on the
matrices of tools/coo_grid_probe.py with the stamps_coo lab build of
libspmv_hip.so (tools/build_variant.sh stamps_coo; SPMV_HIP_LIB points at
it), cold (512 MiB read before each launch), and reads thread 0's
s_memrealtime stamps (100 MHz) per tile: 0 start, 1 products and keys in
LDS, 2 row starts in LDS, 3 end (after a barrier).  Prints, per matrix, the
kernel span (first start to last end) and per path (0 row starts, 1 bitmap,
2 searches) the tile count and the p50 / max of stage (0-1), heads (1-2),
rows (2-3) and the start offset (0 relative to the first tile's start), us.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "opencl-spmv-algorithms_amd"), str(REPO / "tools")]
import spmv_amd as sa  # noqa: E402
from cant_single import FLUSH_BYTES, probe_lib  # noqa: E402
from coo_grid_probe import matrices  # noqa: E402

NT, NS = 16384, 8


def main():
    import torch

    lib = ctypes.CDLL(os.environ["SPMV_HIP_LIB"])
    lib.spmv_lab_coo_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.spmv_lab_coo_stamps.restype = ctypes.c_int
    lib.spmv_lab_coo_stamps_clear.argtypes = []
    lib.spmv_lab_coo_stamps_clear.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    sp = torch.cuda.current_stream(dev).cuda_stream
    P = probe_lib()
    scratch = torch.empty(FLUSH_BYTES, dtype=torch.uint8, device=dev)
    fsink = torch.zeros(16, dtype=torch.int32, device=dev)
    buf = np.zeros(NT * NS, np.uint64)
    out = {}
    for label, m in matrices():
        if "rows<" in label and "62451" not in label:
            continue
        dm = sa.to_device(m, "coo", dev, coo_tail=True, hot=0)
        x = torch.from_numpy(sa.ramp_x(m.n_cols)).to(dev)
        y = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
        tiles = -(-m.nnz // 1536)
        spans, per = [], {}
        for rep in range(6):
            assert lib.spmv_lab_coo_stamps_clear() == 0
            assert P.spmv_probe_flush_read(scratch.data_ptr(), FLUSH_BYTES, fsink.data_ptr(), sp) == 0
            dm.run(x, y)
            torch.cuda.synchronize()
            assert lib.spmv_lab_coo_stamps(buf.ctypes.data, buf.nbytes) == 0
            if rep == 0:
                continue  # first launch: warm-up
            s = buf.reshape(NT, NS)[: min(tiles, NT)].astype(np.int64)
            t0 = s[:, 0].min()
            spans.append((s[:, 3].max() - t0) / 100.0)
            for path in (0, 1, 2):
                sel = s[:, 5] == path
                if not sel.any():
                    continue
                d = per.setdefault(path, {"tiles": int(sel.sum()), "stage": [], "heads": [], "rows": [],
                                          "start": [], "end": [], "span_rows_max": int(s[sel, 4].max())})
                d["stage"] += list((s[sel, 1] - s[sel, 0]) / 100.0)
                d["heads"] += list((s[sel, 2] - s[sel, 1]) / 100.0)
                d["rows"] += list((s[sel, 3] - s[sel, 2]) / 100.0)
                d["start"] += list((s[sel, 0] - t0) / 100.0)
                d["end"] += list((s[sel, 3] - t0) / 100.0)
        q = lambda v: [round(float(np.percentile(v, 50)), 2), round(float(np.max(v)), 2)]  # noqa: E731
        out[label] = {"kernel_span_us_median": round(float(np.median(spans)), 2), "tiles": tiles,
                      "paths": {p: {"tiles": d["tiles"], "span_rows_max": d["span_rows_max"],
                                    **{k: q(d[k]) for k in ("start", "stage", "heads", "rows", "end")}}
                                for p, d in per.items()}}
        print(label, json.dumps(out[label]), flush=True)
        del dm


if __name__ == "__main__":
    main()
