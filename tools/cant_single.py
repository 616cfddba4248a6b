#!/usr/bin/env python3
"""cant_single — BASELINE.json configs[1] (CSR-vector) and configs[2]
(SELL-C-σ, C = 64, σ = 1024) on ONE cant-like matrix (62,451 rows,
4,007,383 entries, 49.3 MB bytes_alg), the configuration the metric is
quoted on, every format, cold and warm:

  cold  a 512 MiB scratch write (probe_flush_kernel) before every launch
        evicts the 256 MiB Infinity Cache and the L2s, so the matrix is read
        from HBM;
  warm  launches back to back: the 49 MB matrix stays in the Infinity Cache
        (cache-resident, NOT an HBM figure).

Beside them, the pure-stream ceiling of the same bytes: spmv_probe_stream
reads bytes_alg once with 16-byte non-temporal loads, cold and warm.

Phases are marked with spmv_probe_tag (tools/probe.hip) so that, run under
`rocprofv3 --kernel-trace`, the kernel durations of every phase can be read
from the trace (tools/trace_segments.py; bench.py does that and reports the
trace figures).  Without a profiler the HIP-event figures are reported.

    python tools/cant_single.py --json out.json
    rocprofv3 --kernel-trace --output-format csv -d D -o run -- \\
        python3 tools/cant_single.py --json out.json
    python tools/cant_single.py --json out.json --attach D
"""
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

FLUSH_BYTES = 512 << 20
PROBE_TAG = 1000  # stream-probe phases: tags 1000 (cold) and 1001 (warm)
SETUP_TAG = 1500  # ignored phases: builds and first runs
END_TAG = 2000


def probe_lib():
    lib = ctypes.CDLL(str(sa.LIB_DIR / "libspmv_probe.so"))
    vp = ctypes.c_void_p
    lib.spmv_probe_stream.argtypes = [vp, ctypes.c_size_t, vp, vp]
    lib.spmv_probe_flush.argtypes = [vp, ctypes.c_size_t, vp]
    lib.spmv_probe_tag.argtypes = [ctypes.c_int, vp]
    lib.spmv_probe_csr_stream.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int, vp, vp]
    lib.spmv_probe_flush_read.argtypes = [vp, ctypes.c_size_t, vp, vp]
    lib.spmv_probe_gather_stream.argtypes = [vp, vp, ctypes.c_int64, vp, vp, vp]
    for f in (lib.spmv_probe_stream, lib.spmv_probe_flush, lib.spmv_probe_tag, lib.spmv_probe_csr_stream,
              lib.spmv_probe_flush_read, lib.spmv_probe_gather_stream):
        f.restype = ctypes.c_int
    return lib


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--json", default=None, help="write the result here (also printed)")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--formats", default=",".join(sa.ALL_FORMATS))
    ap.add_argument("--extra", action="append", default=[], metavar='FMT@JSON',
                    help='another run of FMT with to_device kwargs, e.g. csr@{"xwin_rows": 64}; '
                         '"_opt" sets library switches (spmv_set_option) for that run only, e.g. '
                         'sell@{"_opt": {"xwin_remap": 0}}')
    ap.add_argument("--flush-mode", default="write", choices=["write", "read"],
                    help="cold state: 512 MiB WRITTEN before each launch (default; the caches hold dirty lines) "
                         "or READ (clean lines)")
    ap.add_argument("--warm-x", action="store_true",
                    help="diagnostic: read x once after every flush (matrix cold, x cache-resident)")
    ap.add_argument("--csr-probes", default="", help="also time the CSR-shaped stream probe (val + col pairs, "
                    "no x) on the matrix's CSR arrays with these R values, e.g. 1,3,8")
    ap.add_argument("--attach", default=None, metavar="TRACE_DIR",
                    help="no GPU run: add the kernel-trace figures of a finished rocprofv3 run in TRACE_DIR "
                         "to the --json file it wrote")
    a = ap.parse_args()
    if a.attach:
        out = json.loads(Path(a.json).read_text())
        attach_trace(out, a.attach)
        Path(a.json).write_text(json.dumps(out))
        print(json.dumps(out), flush=True)
        return
    import torch

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    st = torch.cuda.current_stream(dev)
    sp = st.cuda_stream
    P = probe_lib()
    scratch = torch.empty(FLUSH_BYTES, dtype=torch.uint8, device=dev)

    fsink = torch.zeros(16, dtype=torch.int32, device=dev)

    def flush():
        if a.flush_mode == "read":
            assert P.spmv_probe_flush_read(scratch.data_ptr(), FLUSH_BYTES, fsink.data_ptr(), sp) == 0
        else:
            assert P.spmv_probe_flush(scratch.data_ptr(), FLUSH_BYTES, sp) == 0

    def tag(i):
        assert P.spmv_probe_tag(i, sp) == 0

    m = sa.gen_cantlike(0, 1)
    b = sa.bytes_alg(m.n_rows, m.n_cols, m.nnz)
    xh = sa.ramp_x(m.n_cols)
    x = torch.from_numpy(xh).to(dev)
    if a.warm_x:
        xsink = torch.zeros(1 << 12, dtype=torch.float64, device=dev)
        plain_flush = flush

        def flush():  # noqa: F811 — diagnostic: x read back into the caches after the flush
            plain_flush()
            assert P.spmv_probe_stream(x.data_ptr(), (m.n_cols * 8) // 16 * 16, xsink.data_ptr(), sp) == 0
    reps = a.reps
    out = {"matrix": "cant-like (62,451 rows, 4,007,383 entries), x[j] = j", "bytes_alg": b, "reps": reps,
           "flush": f"512 MiB {'read' if a.flush_mode == 'read' else 'written'} before every cold launch",
           "formats": {}, "phases": {}}
    formats = [(f, f, {}) for f in a.formats.split(",") if f]
    for e in a.extra:
        f, kw = e.split("@", 1)
        formats.append((f"{f}@{kw}", f, json.loads(kw)))
    for i, (label, fmt, kw) in enumerate(formats):
        tag(SETUP_TAG + i)  # builds, fills and the first run land in an ignored phase
        kw = dict(kw)
        # "_opt": the library's A/B switches for this run only (spmv_set_option:
        # placement / load policy, never a result bit), e.g. {"xwin_remap": 0}
        opt = kw.pop("_opt", {})
        for k, v in opt.items():
            sa.set_option(k, v)
        dm = sa.to_device(m, fmt, dev, **kw)
        y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
        dm.run(x, y)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
        tag(2 * i)
        for r in range(reps):
            flush()
            ev[2 * r].record(st)
            dm.run(x, y)
            ev[2 * r + 1].record(st)
        tag(SETUP_TAG + 100 + i)  # the check's copy lands in an ignored phase
        torch.cuda.synchronize()
        cold = [ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(reps)]
        bad, first = sa.check(m, xh, y.cpu().numpy())
        wev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        tag(2 * i + 1)
        wev[0].record(st)
        for r in range(reps):
            dm.run(x, y)
            wev[r + 1].record(st)
        tag(SETUP_TAG + 200 + i)
        torch.cuda.synchronize()
        warm = [wev[r].elapsed_time(wev[r + 1]) for r in range(reps)]
        bad2, _ = sa.check(m, xh, y.cpu().numpy())
        c, w = float(np.median(cold)), float(np.median(warm))
        out["formats"][label] = {"kernel_params": {k: v for k, v in dm.params.items() if isinstance(v, (int, float, str))},
                               "event_cold_ms": round(c, 5), "event_warm_ms": round(w, 5),
                               "event_cold_GBs": round(b / (c * 1e-3) * 1e-9, 1),
                               "parity_ok": bad == 0 and bad2 == 0}
        if fmt == "csrf32":
            out["formats"][label]["parity"] = "within fp32-value tolerance (values rounded to fp32)"
        out["phases"][label] = [2 * i, 2 * i + 1]
        del dm
        for k in opt:
            sa.set_option(k, None)
    # the CSR arrays streamed without the kernels' structure (val + col pairs)
    if a.csr_probes:
        _, ccol, cval = sa.csr_from_coo(m)
        dval = torch.from_numpy(cval).to(dev)
        dcol = torch.from_numpy(ccol).to(dev)
        npairs = m.nnz // 2
        sink2 = torch.zeros(1 << 16, dtype=torch.float64, device=dev)
        for j, r in enumerate(int(v) for v in a.csr_probes.split(",")):
            label = f"csr_stream_probe_R{r}"
            ph = PROBE_TAG + 10 + 2 * j
            tag(ph)
            for _ in range(reps):
                flush()
                assert P.spmv_probe_csr_stream(dval.data_ptr(), dcol.data_ptr(), npairs, r, sink2.data_ptr(), sp) == 0
            tag(ph + 1)
            for _ in range(reps):
                assert P.spmv_probe_csr_stream(dval.data_ptr(), dcol.data_ptr(), npairs, r, sink2.data_ptr(), sp) == 0
            out["formats"][label] = {"bytes": 12 * 2 * npairs}
            out["phases"][label] = [ph, ph + 1]
        # the same probe on other placements of the same bytes: fresh copies,
        # and val + col inside ONE allocation; and the plain probe on val alone
        one = torch.empty(12 * 2 * npairs + 256, dtype=torch.uint8, device=dev)
        v1 = one[: 16 * npairs].view(torch.float64)
        c1 = one[16 * npairs: 24 * npairs].view(torch.int32)
        v1.copy_(dval[: 2 * npairs])
        c1.copy_(dcol[: 2 * npairs])
        dval2, dcol2 = dval.clone(), dcol.clone()
        extra = [("csr_stream_probe_R3_copies", lambda: P.spmv_probe_csr_stream(dval2.data_ptr(), dcol2.data_ptr(), npairs,
                                                                                  3, sink2.data_ptr(), sp), 24 * npairs),
                 ("csr_stream_probe_R3_one_alloc", lambda: P.spmv_probe_csr_stream(v1.data_ptr(), c1.data_ptr(), npairs, 3,
                                                                                     sink2.data_ptr(), sp), 24 * npairs),
                 ("stream_probe_val_only", lambda: P.spmv_probe_stream(dval.data_ptr(), 16 * npairs, sink2.data_ptr(), sp),
                  16 * npairs)]
        for j, (label, fn, nbytes) in enumerate(extra):
            ph = PROBE_TAG + 40 + 2 * j
            tag(ph)
            for _ in range(reps):
                flush()
                assert fn() == 0
            tag(ph + 1)
            for _ in range(reps):
                assert fn() == 0
            out["formats"][label] = {"bytes": nbytes}
            out["phases"][label] = [ph, ph + 1]
        tag(SETUP_TAG + len(formats) + 1)
        torch.cuda.synchronize()
    # the stream ceiling of the same bytes
    nb = (b + 15) // 16 * 16
    tag(SETUP_TAG + len(formats))
    buf = torch.ones(nb // 8, dtype=torch.float64, device=dev)
    sink = torch.zeros(1 << 16, dtype=torch.float64, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    tag(PROBE_TAG)
    for r in range(reps):
        flush()
        ev[2 * r].record(st)
        assert P.spmv_probe_stream(buf.data_ptr(), nb, sink.data_ptr(), sp) == 0
        ev[2 * r + 1].record(st)
    tag(PROBE_TAG + 1)
    for r in range(reps):
        assert P.spmv_probe_stream(buf.data_ptr(), nb, sink.data_ptr(), sp) == 0
    tag(END_TAG)
    torch.cuda.synchronize()
    c = float(np.median([ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(reps)]))
    out["stream_probe"] = {"bytes": nb, "event_cold_ms": round(c, 5), "event_cold_GBs": round(nb / (c * 1e-3) * 1e-9, 1)}
    out["phases"]["stream_probe"] = [PROBE_TAG, PROBE_TAG + 1]
    text = json.dumps(out)
    if a.json:
        Path(a.json).write_text(text)
    print(text, flush=True)


def attach_trace(out, trace_dir):
    """Add rocprofv3 kernel-trace medians (cold / warm ms per format and for
    the stream probe) to `out`; the trace file is written when the profiled
    process exits, so this is called by the PARENT (bench.py) on a finished
    trace directory."""
    import trace_segments as ts

    paths = sorted(Path(trace_dir).rglob("*kernel_trace.csv"))
    if not paths:
        out["trace"] = "no kernel trace found"
        return
    seg = ts.segments(paths[-1])
    b, reps = out["bytes_alg"], out["reps"]
    for fmt, (tc, tw) in out["phases"].items():
        cold = ts.cold_ms(seg.get(tc, []))
        warm = ts.warm_ms(seg.get(tw, []), reps)
        rec = out["formats"][fmt] if fmt in out["formats"] else out["stream_probe"]
        nbytes = rec.get("bytes", b)
        if cold:
            cm = round(float(np.median(cold)), 5)  # every figure from the rounded median (bench.py reuses it)
            rec.update(cold_ms=cm, cold_ms_mean=round(float(np.mean(cold)), 5), cold_reps=len(cold),
                       cold_GBs=round(nbytes / (cm * 1e-3) * 1e-9, 1),
                       cold_frac=round(nbytes / (cm * 1e-3) * 1e-9 / sa.HBM_PEAK_GBS, 4),
                       cold_ms_range=[round(min(cold), 5), round(max(cold), 5)])
        if warm:
            wm = float(np.median(warm))
            rec.update(warm_ms=round(wm, 5), warm_GBs_cache_resident=round(nbytes / (wm * 1e-3) * 1e-9, 1))
        rec["kernels"] = ts.kernel_names(seg.get(tc, []))
    out["timing"] = "rocprofv3 kernel trace (GPU timestamps), median over reps"
    probe = out["stream_probe"].get("cold_ms")
    if probe:
        for rec in out["formats"].values():
            if rec.get("cold_ms"):
                rec["cold_vs_stream_probe"] = round(probe / rec["cold_ms"], 3)


if __name__ == "__main__":
    main()
