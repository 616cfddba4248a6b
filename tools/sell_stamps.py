#!/usr/bin/env python3
"""sell_stamps — where the small-matrix SELL (or the CSR x-window) kernel's time goes, per wave.

Lab only.  Runs the library's SELL (int32, head copy) and SELL16 on one
cant-like matrix with the stamps_sell lab build of libspmv_hip.so
(tools/build_variant.sh stamps_sell, which injects tools/lab_stamps_sell.h;
SPMV_HIP_LIB points at it), cold (512 MiB read before each launch) and warm,
and reads the per-wave s_memrealtime stamps (100 MHz, 10 ns) that build
writes at: 0 start, 1 x window published (barrier), 2 first batch summed,
3 all batches summed, 4 partial sums published (barrier), 5 y stored.
Prints medians over launches of the kernel span and of each phase's
distribution over the waves (p10 / p50 / p90 / max, us).  --kernel csr: the
CSR x-window kernel of the stamps_csr lab build (tools/build_variant.sh
stamps_csr) (0 start, 1 window and
offsets published, 2 chunk 0's products in LDS, 3 its barrier, 4 its row
sums read, 5 its second barrier, 6 / 7 chunks 1 / 2's products in LDS)."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "opencl-spmv-algorithms_amd"), str(REPO), str(REPO / "tools")]
import spmv_amd as sa  # noqa: E402
from cant_single import FLUSH_BYTES, probe_lib  # noqa: E402

NSTAMP, NWAVES = 8, 8192
PHASES = [("window", 0, 1), ("first_batch", 1, 2), ("batches", 2, 3), ("part_barrier", 3, 4), ("store", 4, 5),
          ("wave_total", 0, 5)]


def q(v):
    return [round(float(np.nanpercentile(v, p)), 3) for p in (10, 50, 90)] + [round(float(np.nanmax(v)), 3)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--formats", default="sell,sell16")
    ap.add_argument("--kernel", default="sell", choices=["sell", "csr"])
    a = ap.parse_args()
    if a.kernel == "csr":
        return csr_main(a)
    if not os.environ.get("SPMV_HIP_LIB"):
        sys.exit("set SPMV_HIP_LIB to a stamps_sell lab build")
    import torch

    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    sp = st.cuda_stream
    P = probe_lib()
    lib = sa.hip_lib()
    fn = lib.spmv_lab_sell_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    fn.restype = ctypes.c_int
    scratch = torch.empty(FLUSH_BYTES, dtype=torch.uint8, device=dev)
    fsink = torch.zeros(16, dtype=torch.int32, device=dev)
    m = sa.gen_cantlike(0, 1)
    xh = sa.ramp_x(m.n_cols)
    x = torch.from_numpy(xh).to(dev)
    host = np.zeros(NWAVES * NSTAMP, dtype=np.uint64)
    for fmt in a.formats.split(","):
        dm = sa.to_device(m, fmt, dev)
        y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
        n_slices = int(dm.params["n_slices"])
        nw = (n_slices + 3) // 4 * 8
        # groups per wave (P = 4 slices, S = 2 waves per slice, KI = ki)
        sp_h = dm.arrays["slice_ptr"].cpu().numpy()
        ki = int(dm.params["ki"])
        widths = np.diff(sp_h) // 64 // ki
        per = (widths + 1) // 2
        gw = np.zeros(nw, dtype=np.int64)
        for s in range(n_slices):
            gw[(s // 4) * 8 + (s % 4) * 2] = per[s]
            gw[(s // 4) * 8 + (s % 4) * 2 + 1] = max(0, min(per[s], widths[s] - per[s]))
        for state in ("cold", "warm"):
            spans, phases, late = [], {k: [] for k, _, _ in PHASES}, []
            last_groups, start_skew = [], []
            for _ in range(a.reps):
                if state == "cold":
                    assert P.spmv_probe_flush_read(scratch.data_ptr(), FLUSH_BYTES, fsink.data_ptr(), sp) == 0
                dm.run(x, y)
                torch.cuda.synchronize()
                assert fn(host.ctypes.data, host.nbytes) == 0
                t = host[: nw * NSTAMP].reshape(nw, NSTAMP)[:, :6].astype(np.int64)
                t0 = t[:, 0].min()
                us = (t - t0) * 0.01
                spans.append(float(us[:, 5].max()))
                start_skew.append(q(us[:, 0]))
                for k, i, j in PHASES:
                    phases[k].append(q(us[:, j] - us[:, i]))
                lw = int(np.argmax(us[:, 5]))
                last_groups.append(int(gw[lw]))
                late.append([round(float(v), 3) for v in us[lw]])
            bad, _ = sa.check(m, xh, y.cpu().numpy())
            out = {"format": fmt, "state": state, "waves": nw, "parity_ok": bad == 0,
                   "span_us_median": round(float(np.median(spans)), 3),
                   "span_us_range": [round(min(spans), 3), round(max(spans), 3)],
                   "start_us_p10_p50_p90_max": np.median(np.array(start_skew), axis=0).round(3).tolist(),
                   "phases_us_p10_p50_p90_max": {k: np.median(np.array(v), axis=0).round(3).tolist()
                                                  for k, v in phases.items()},
                   "last_wave_stamps_us_median": np.median(np.array(late), axis=0).round(3).tolist(),
                   "last_wave_groups": last_groups[:10],
                   "groups_per_wave_p10_p50_p90_max": [int(np.percentile(gw, p)) for p in (10, 50, 90, 100)]}
            print(json.dumps(out), flush=True)
        del dm


def csr_main(a):
    import torch

    dev = torch.device("cuda:0")
    sp = torch.cuda.current_stream(dev).cuda_stream
    P = probe_lib()
    fn = sa.hip_lib().spmv_lab_csr_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    fn.restype = ctypes.c_int
    scratch = torch.empty(FLUSH_BYTES, dtype=torch.uint8, device=dev)
    fsink = torch.zeros(16, dtype=torch.int32, device=dev)
    m = sa.gen_cantlike(0, 1)
    xh = sa.ramp_x(m.n_cols)
    x = torch.from_numpy(xh).to(dev)
    host = np.zeros(NWAVES * NSTAMP, dtype=np.uint64)
    dm = sa.to_device(m, "csr", dev)
    y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    nw = ((m.n_rows + 127) // 128) * 4
    for state in ("cold", "warm"):
        rows = []
        for _ in range(a.reps):
            host[:] = 0
            if state == "cold":
                assert P.spmv_probe_flush_read(scratch.data_ptr(), FLUSH_BYTES, fsink.data_ptr(), sp) == 0
            dm.run(x, y)
            torch.cuda.synchronize()
            assert fn(host.ctypes.data, host.nbytes) == 0
            t = host[: nw * NSTAMP].reshape(nw, NSTAMP).astype(np.int64)
            t0 = t[:, 0].min()
            us = np.where(t > 0, (t - t0) * 0.01, np.nan)
            last = np.nanmax(us, axis=1)
            rows.append({"span": float(np.nanmax(last)),
                         "start": q(us[:, 0]), "window": q(us[:, 1] - us[:, 0]),
                         "chunks": [q(us[:, k + 1] - us[:, k]) for k in range(1, NSTAMP - 1)
                                    if not np.all(np.isnan(us[:, k + 1]))]})
        bad, _ = sa.check(m, xh, y.cpu().numpy())
        out = {"format": "csr", "state": state, "waves": nw, "parity_ok": bad == 0,
               "span_us_median": round(float(np.median([r["span"] for r in rows])), 3),
               "start_us": np.median(np.array([r["start"] for r in rows]), axis=0).round(3).tolist(),
               "window_us": np.median(np.array([r["window"] for r in rows]), axis=0).round(3).tolist(),
               "chunk_us": [np.median(np.array([r["chunks"][k] for r in rows if len(r["chunks"]) > k]), axis=0)
                            .round(3).tolist() for k in range(max(len(r["chunks"]) for r in rows))]}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
