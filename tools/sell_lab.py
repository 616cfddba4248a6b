#!/usr/bin/env python3
"""sell_lab — where the time of the small-matrix SELL kernel goes.

Runs diagnostic copies of the waves-per-slice SELL kernel (tools/sell_lab.hip,
lib/libspmv_lab.so) on the library's own SELL-64-1024 arrays of one cant-like
matrix, cold (512 MiB flush first) and warm, and reads per-wave timestamps
(s_memrealtime, 10 ns): kernel span (first wave start to last wave end),
wave durations, and how late the last wave started.  Diagnostic only."""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "opencl-spmv-algorithms_amd"), str(REPO), str(REPO / "tools")]
import spmv_amd as sa  # noqa: E402
from cant_single import FLUSH_BYTES, probe_lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--codes", default="M22408,B22408,M12408,B12408,M22406,B22406,B22404,B12412,M22408,B22408")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    sp = st.cuda_stream
    lab = ctypes.CDLL(str(sa.LIB_DIR / "libspmv_lab.so"))
    vp = ctypes.c_void_p
    lab.lab_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int32, vp,
                            vp]
    lab.lab_windows.argtypes = [ctypes.c_int64, vp, vp, vp, vp]
    lab.lab_chunk.argtypes = [ctypes.c_int, ctypes.c_int64] + [vp] * 14
    lab.lab_multi.argtypes = [ctypes.c_int, ctypes.c_int64] + [vp] * 7 + [ctypes.c_int32, vp, vp]
    lab.lab_flat.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, vp, vp, vp, vp, vp, vp]
    P = probe_lib()
    scratch = torch.empty(FLUSH_BYTES, dtype=torch.uint8, device=dev)
    m = sa.gen_cantlike(0, 1)
    xh = sa.ramp_x(m.n_cols)
    x = torch.from_numpy(xh).to(dev)
    b = sa.bytes_alg(m.n_rows, m.n_cols, m.nnz)
    mats = {}
    for ki in (1, 2):
        dm = sa.to_device(m, "sell", dev, ki=ki, xwin=False)
        A = dm.arrays
        n = dm.params["n_slices"]
        win = torch.empty(2 * n, dtype=torch.int32, device=dev)
        assert lab.lab_windows(n, A["slice_ptr"].data_ptr(), A["col"].data_ptr(), win.data_ptr(), sp) == 0
        torch.cuda.synchronize()
        w = win.view(-1, 2).cpu().numpy()
        xcap = int((w[:, 1] - w[:, 0] + 1).max())
        mats[ki] = (dm, n, win, xcap)
    # the stream ceiling of the same bytes in this process (cold / warm)
    nb = (b + 15) // 16 * 16
    buf = torch.ones(nb // 8, dtype=torch.float64, device=dev)
    sink = torch.zeros(1 << 16, dtype=torch.float64, device=dev)
    for mode in ("warm", "cold"):
        ts = []
        for r in range(a.reps):
            if mode == "cold":
                P.spmv_probe_flush(scratch.data_ptr(), FLUSH_BYTES, sp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            P.spmv_probe_stream(buf.data_ptr(), nb, sink.data_ptr(), sp)
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        print(json.dumps({"probe": mode, "event_us": round(float(np.median(ts)), 2)}), flush=True)
    for code in a.codes.split(","):
        if code.startswith("M") or code.startswith("B"):  # multi-slice workgroups: M|B + KI*10000 + S*1000 + P*100 + G
            c = int(code[1:])
            ki, S, P2, G = c // 10000, (c // 1000) % 10, (c // 100) % 10, c % 100
            if code.startswith("B"):  # balanced slice choice inside 16-slice sigma windows
                c += 100000
            dm, n, win, xcap = mats[ki]
            A = dm.arrays
            nb = (n + P2 - 1) // P2
            stamps = torch.zeros(nb * S * P2 * 3, dtype=torch.int64, device=dev)
            y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
            # the union window of P slices can exceed the per-slice xcap: give the lab its own cap
            cap = 2048 if P2 > 1 else xcap

            def run_m():
                rc = lab.lab_multi(c, n, A["slice_ptr"].data_ptr(), A["perm"].data_ptr(), A["col"].data_ptr(),
                                   A["val"].data_ptr(), x.data_ptr(), y.data_ptr(), win.data_ptr(), cap,
                                   stamps.data_ptr(), sp)
                assert rc == 0, rc

            res = {}
            for mode in ("warm", "cold"):
                spans, durs, late = [], [], []
                for r in range(a.reps):
                    if mode == "cold":
                        P.spmv_probe_flush(scratch.data_ptr(), FLUSH_BYTES, sp)
                    run_m()
                    torch.cuda.synchronize()
                    st_ = stamps.view(-1, 3).cpu().numpy().astype(np.int64)
                    t0, t1 = st_[:, 0], st_[:, 1]
                    spans.append((t1.max() - t0.min()) * 10e-3)
                    durs.append(np.median(t1 - t0) * 10e-3)
                    late.append((t0.max() - t0.min()) * 10e-3)
                res[mode] = {"span_us": round(float(np.median(spans)), 2),
                             "wave_us_med": round(float(np.median(durs)), 2),
                             "last_start_us": round(float(np.median(late)), 2)}
            bad, _ = sa.check(m, xh, y.cpu().numpy())
            print(json.dumps({"code": code, "ki": ki, "S": S, "P": P2, "G": G, "cap": cap, **res,
                              "cold_GBs_span": round(b / (res["cold"]["span_us"] * 1e-6) * 1e-9, 1),
                              "parity_ok": bad == 0}), flush=True)
            continue
        if code.startswith("C"):  # chunked: C + KI*1000 + G*10 + SYNC*2 + PREF, e.g. C1082 = ki 1, G 8, sync 1
            c = int(code[1:])
            ki, G, sy = c // 1000, (c // 10) % 100, c % 10
            chunked(a, torch, lab, P, scratch, sp, mats[ki], m, x, xh, b, ki, G, c, code)
            continue
        if code.startswith("F"):  # flat one-shot read of the ki = 2 arrays: F<U><gather>
            flat(a, torch, lab, P, scratch, st, sp, mats[2][0], x, b, int(code[1:-1]), int(code[-1]), code)
            continue
        xw = code.endswith("x")
        c = int(code.rstrip("x"))
        if c >= 200000:  # diagnostic modes of the one-shot variant: (2+MODE)KSSGG
            ki, S, U = (c // 10000) % 10, (c // 100) % 100, c % 100
        elif c >= 100000:  # one-shot variant: 1KSSGG
            ki, S, U = (c // 10000) % 10, (c // 100) % 100, c % 100
        else:
            ki, S, U = c // 1000, (c % 1000) // 10, c % 10
        dm, n, win, xcap = mats[ki]
        A = dm.arrays
        stamps = torch.zeros(n * S * 3, dtype=torch.int64, device=dev)
        y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)

        def run():
            rc = lab.lab_run(c, int(xw), n, A["slice_ptr"].data_ptr(), A["perm"].data_ptr(), A["col"].data_ptr(),
                             A["val"].data_ptr(), x.data_ptr(), y.data_ptr(), win.data_ptr(), xcap,
                             stamps.data_ptr(), sp)
            assert rc == 0, rc

        res = {}
        for mode in ("warm", "cold"):
            spans, durs, late = [], [], []
            for r in range(a.reps):
                if mode == "cold":
                    P.spmv_probe_flush(scratch.data_ptr(), FLUSH_BYTES, sp)
                run()
                torch.cuda.synchronize()
                s = stamps.view(-1, 3).cpu().numpy().astype(np.int64)
                t0, t1 = s[:, 0], s[:, 1]
                spans.append((t1.max() - t0.min()) * 10e-3)  # us
                durs.append(np.median(t1 - t0) * 10e-3)
                late.append((t0.max() - t0.min()) * 10e-3)
            res[mode] = {"span_us": round(float(np.median(spans)), 2), "wave_us_med": round(float(np.median(durs)), 2),
                         "last_start_us": round(float(np.median(late)), 2)}
        bad, _ = sa.check(m, xh, y.cpu().numpy())
        span = res["cold"]["span_us"]
        print(json.dumps({"code": code, "ki": ki, "S": S, "U": U, "xwin": xw, "xcap": xcap, **res,
                          "cold_GBs_span": round(b / (span * 1e-6) * 1e-9, 1), "parity_ok": bad == 0}), flush=True)


def chunked(a, torch, lab, P, scratch, sp, mat, m, x, xh, b, ki, G, c, code):
    dm, n, win, xcap = mat
    A = dm.arrays
    spt = A["slice_ptr"].cpu().numpy()
    ng = np.diff(spt) // (64 * ki)
    nch = np.maximum((ng + G - 1) // G, 1)
    sf = np.zeros(n + 1, np.int32)
    np.cumsum(nch, out=sf[1:])
    cs = np.repeat(np.arange(n, dtype=np.int32), nch)
    cg = (np.arange(sf[-1]) - np.repeat(sf[:-1], nch)).astype(np.int32) * G
    dev = x.device
    t = lambda v: torch.from_numpy(np.ascontiguousarray(v)).to(dev)  # noqa: E731
    cs_d, cg_d, sf_d = t(cs), t(cg), t(sf)
    nchunks = int(sf[-1])
    part = torch.zeros(nchunks * 64, dtype=torch.float64, device=dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    blocks = ((nchunks + 3) // 4 + 7) // 8 * 8
    stamps = torch.zeros(blocks * 4 * 3, dtype=torch.int64, device=dev)
    y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    res = {}
    for mode in ("warm", "cold"):
        spans, durs, late = [], [], []
        for r in range(a.reps):
            if mode == "cold":
                P.spmv_probe_flush(scratch.data_ptr(), FLUSH_BYTES, sp)
            rc = lab.lab_chunk(c, nchunks, cs_d.data_ptr(), cg_d.data_ptr(), sf_d.data_ptr(), A["slice_ptr"].data_ptr(),
                               A["perm"].data_ptr(), A["col"].data_ptr(), A["val"].data_ptr(), x.data_ptr(),
                               y.data_ptr(), part.data_ptr(), cnt.data_ptr(), win.data_ptr(), stamps.data_ptr(), sp)
            assert rc == 0, rc
            torch.cuda.synchronize()
            st = stamps.view(-1, 3).cpu().numpy().astype(np.int64)
            t0, t1 = st[:, 0], st[:, 1]
            spans.append((t1.max() - t0.min()) * 10e-3)
            durs.append(np.median(t1 - t0) * 10e-3)
            late.append((t0.max() - t0.min()) * 10e-3)
        res[mode] = {"span_us": round(float(np.median(spans)), 2), "wave_us_med": round(float(np.median(durs)), 2),
                     "last_start_us": round(float(np.median(late)), 2)}
    bad, _ = sa.check(m, xh, y.cpu().numpy())
    y1 = y.clone()
    lab.lab_chunk(c, nchunks, cs_d.data_ptr(), cg_d.data_ptr(), sf_d.data_ptr(), A["slice_ptr"].data_ptr(),
                  A["perm"].data_ptr(), A["col"].data_ptr(), A["val"].data_ptr(), x.data_ptr(), y.data_ptr(),
                  part.data_ptr(), cnt.data_ptr(), win.data_ptr(), stamps.data_ptr(), sp)
    torch.cuda.synchronize()
    same = bool(torch.equal(y1.view(torch.int64), y.view(torch.int64)))
    print(json.dumps({"code": code, "ki": ki, "G": G, "chunks": nchunks, "blocks": blocks, **res,
                      "cold_GBs_span": round(b / (res["cold"]["span_us"] * 1e-6) * 1e-9, 1), "parity_ok": bad == 0,
                      "repeat_same_bits": same, "counters_reset": bool((cnt == 0).all().item())}), flush=True)


def flat(a, torch, lab, P, scratch, st, sp, dm, x, b, U, gather, code):
    A = dm.arrays
    n2 = A["val"].numel() // 2
    blocks = (n2 + 256 * U - 1) // (256 * U)
    stamps = torch.zeros(blocks * 4 * 3, dtype=torch.int64, device=x.device)
    out_all = torch.zeros(blocks + 1, dtype=torch.float64, device=x.device)
    out_all[0] = float(x.numel())  # the kernel reads n_x from out[-1]
    out = out_all[1:]
    res = {}
    for mode in ("warm", "cold"):
        spans, durs, late = [], [], []
        for r in range(a.reps):
            if mode == "cold":
                P.spmv_probe_flush(scratch.data_ptr(), FLUSH_BYTES, sp)
            assert lab.lab_flat(U, gather, n2, A["val"].data_ptr(), A["col"].data_ptr(), x.data_ptr(),
                                out.data_ptr(), stamps.data_ptr(), sp) == 0
            torch.cuda.synchronize()
            s = stamps.view(-1, 3).cpu().numpy().astype(np.int64)
            t0, t1 = s[:, 0], s[:, 1]
            spans.append((t1.max() - t0.min()) * 10e-3)
            durs.append(np.median(t1 - t0) * 10e-3)
            late.append((t0.max() - t0.min()) * 10e-3)
        res[mode] = {"span_us": round(float(np.median(spans)), 2), "wave_us_med": round(float(np.median(durs)), 2),
                     "last_start_us": round(float(np.median(late)), 2)}
    nbytes = 24 * n2
    print(json.dumps({"code": code, "flat_U": U, "gather": gather, "bytes": nbytes, "blocks": blocks, **res,
                      "cold_GBs_span": round(nbytes / (res["cold"]["span_us"] * 1e-6) * 1e-9, 1)}), flush=True)


if __name__ == "__main__":
    main()
