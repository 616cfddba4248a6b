#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X SpMV suite.

Metric (BASELINE.json): effective HBM GB/s (+ GFLOP/s) of fp64 y = A·x per
format on cant.mtx.  The real cant.mtx is a Git-LFS pointer in the
reference, so the matrix is the cant-like stand-in
(spmv_gen_cantlike: N = 62,451, Z = 4,007,383, the real cant's counts).

Headline (default `--workload cant`, BASELINE.json configs[1]): CSR-vector
on ONE cant-like matrix per GPU, COLD.  A step is a 512 MiB flush (evicts
the 256 MiB Infinity Cache and the L2s) followed by ONE SpMV launch, so the
49.3 MB matrix is read from HBM every step.  W untimed warm-up steps, then
exactly K steps captured in one HIP graph and replayed between a barrier +
synchronize on both sides; a graph of K flushes alone is timed the same
way, and the SpMV's share of a step is (span of K x (flush + SpMV) - span
of K x flush) / K, HIP events on the launch stream, max over ranks.  A
rocprofv3 kernel trace of the same kernel, cold (tools/cant_single.py, a
child process started before this process touches the GPU: every format
at N=1, the headline format on every rank's GPU at N>1, beside the
stream-probe ceiling of the same bytes), is reported beside it as
corroboration (roofline.kernel_ms_trace).  value = N x bytes_alg / (that
in-process cold SpMV time) = the whole job's throughput of replicated
configs[1] steps (weak scaling: one matrix per GPU, no collective);
ms_per_step = that SpMV time; the timed region's wall clock (flushes
included) is `timed_region`.

At N=1 also `batch`: ONE launch over 32 cant-like matrices stacked
block-diagonally (1.58 GB, 6x the Infinity Cache, streamed from HBM; the
round 1-3 headline) with its own roofline and every format on it
(`per_format`).  `rmat_strong` (configs[3]) and `banded_strong`
(configs[4]) cut ONE matrix into N row shards (strong scaling, x
replicated) and report SpMV-only, the y all-gather of the real shard sizes
over RCCL (an allgatherv), SpMV + all-gather, and cold shards.

`python3 bench.py --gpus N` without a launcher starts itself as N ranks
under torch.distributed.run in a CHILD process (launch.spawn_ranks) and
exits with its code; under torch.distributed.run (WORLD_SIZE set) it is a
rank.

bytes_alg = 12·Z + 4·(N+1) + 8·M + 8·N per matrix:
values, columns, row offsets, x and y once each.  roofline.achieved uses
the same bytes over the dominant kernel's cold duration; roofline.traffic
comes from the rocprofv3 PMC passes committed in profiles/
(tools/pmc_traffic.py).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "opencl-spmv-algorithms_amd"))
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tools"))

import iterate  # noqa: E402
import launch  # noqa: E402
import spmv_amd as sa  # noqa: E402

METRIC = "effective HBM GB/s + GFLOP/s per format on cant.mtx, 1/2/4/8 MI355X"
# R-MAT shards balance entries + RMAT_ROW_WEIGHT * rows: with 512-entry
# tiles the slowest of 8 shards took 0.1421 / 0.1411 / 0.1464 / 0.1549 ms
# with weights 1 / 2 / 3 / 4 (profiles/round2/shard_rehearse_tiled_w.log)
RMAT_ROW_WEIGHT = 2.0
# profile-guided re-cuts of the R-MAT shards (on cold shard times with --flush yes),
# each moving the cut points RMAT_DAMP of the way (full cold re-cuts overshot:
# profiles/round4/shard_rehearse_cold_calibrated.log)
RMAT_RECUTS = 4
RMAT_DAMP = 0.5
CSR_DEFAULT_VARIANT = 3  # spmv_csr_run_variant's default (csrc/csr.hip)
# untimed replays of a freshly captured graph before the timed replay, at
# least this much GPU time: the first replays of a new graph ran ~4 % slower
# than later ones (headline 0.2659 vs per-format 0.2557 ms
# for the same kernel in the same process)
WARM_REPLAY_MS = 100.0
INPROC_REPS = 5  # timed regions per in-process cold figure (their median is reported)


def parse():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--format", default="csr", choices=sa.ALL_FORMATS)
    p.add_argument("--copies", type=int, default=32, help="cant-like copies per GPU (batch)")
    p.add_argument("--workload", default="cant", choices=["cant", "batch", "cantlike", "rmat", "banded"],
                   help="cant (default: ONE cant-like matrix per GPU, cold, configs[1]/[2]); batch (= cantlike: "
                        "the 32-copy block-diagonal batch); rmat (configs[3]); banded (configs[4])")
    p.add_argument("--batch", default="auto", choices=["auto", "yes", "no"],
                   help="with --workload cant, also time the 32-copy batch and every format on it (auto: N=1)")
    p.add_argument("--banded-rows", type=int, default=100_000_000)
    p.add_argument("--per-format", default="auto", choices=["auto", "yes", "no"],
                   help="also measure the other formats (default: at N=1 only)")
    p.add_argument("--single", default="auto", choices=["auto", "yes", "no"],
                   help="cant_single: ONE cant-like matrix, cold and warm, from a rocprofv3 kernel trace of a "
                        "child process (auto, with --workload cant: every format at N=1, the headline format "
                        "on every rank at N>1)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0: skip)")
    p.add_argument("--lanes", type=int, default=0)
    p.add_argument("--variant", type=int, default=0, help="CSR kernel variant (0 auto, 1 direct, 2 staged)")
    p.add_argument("--ki", type=int, default=0, help="k-interleave (0: format default, ELL 2, SELL 1)")
    p.add_argument("--C", type=int, default=64)
    p.add_argument("--sigma", type=int, default=0,
                   help="SELL sigma (0: 1024 = configs[2]; whole-matrix sort, 2^24, on R-MAT)")
    p.add_argument("--h", type=int, default=8)
    p.add_argument("--profile", action="store_true", help="only the timed loop (for rocprofv3 passes)")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="collective backend for N>1 (nccl = RCCL; gloo only to rehearse on one GPU)")
    p.add_argument("--share-gpu", action="store_true", help="all ranks on cuda:0 (rehearsal only)")
    p.add_argument("--rmat-strong", default="auto", choices=["auto", "yes", "no"],
                   help="also time CSR on the R-MAT 1e7/1e8 row-sharded over all ranks (strong scaling, "
                        "north-star sweep; auto: with the default workload)")
    p.add_argument("--banded-strong", default="auto", choices=["auto", "yes", "no"],
                   help="also time CSR and SELL on the banded 1e8-row / 1.6e9-entry matrix row-sharded over all "
                        "ranks (configs[4], generated on device; auto: with the default workload)")
    p.add_argument("--cold-flush", default="read", choices=["read", "write"],
                   help="headline cold state: 512 MiB READ (clean lines, default) or WRITTEN before every SpMV; "
                        "the other is timed beside it")
    p.add_argument("--relabel-ties", default="first", choices=["first", "id"],
                   help="R-MAT relabel: equal-degree columns in order of their first row (default: neighbouring "
                        "rows' low-degree columns share x lines; whole R-MAT 0.715 -> 0.680 ms, "
                        "profiles/round5/ab_rmat_ties.md) or by column id")
    p.add_argument("--relabel", default="auto", choices=["auto", "yes", "no"],
                   help="R-MAT: columns relabelled by decreasing degree at build time (spmv_column_relabel), x "
                        "replicated in that layout (auto: yes); no = the per-run hot-column table instead")
    p.add_argument("--rmat-per-format", default="auto", choices=["auto", "yes", "no"],
                   help="with rmat_strong at N = 1: every format on the whole R-MAT (configs[3]), cold and warm, "
                        "beside the gather ceiling of its column sequence")
    p.add_argument("--sell-single", default="auto", choices=["auto", "yes", "no"],
                   help="with --workload cant: also SELL-C-sigma on the single matrix (configs[2]) by the "
                        "headline's in-process method (auto: yes)")
    p.add_argument("--rmat-rows", type=int, default=10_000_000, help="R-MAT rows (configs[3]: 1e7)")
    p.add_argument("--rmat-nnz", type=int, default=100_000_000, help="R-MAT entries (configs[3]: 1e8)")
    p.add_argument("--recuts", type=int, default=None, help="profile-guided R-MAT re-cuts (default RMAT_RECUTS)")
    p.add_argument("--flush", default="yes", choices=["yes", "no"],
                   help="strong-scaling legs: also time every shard cold (512 MiB flush before each step)")
    p.add_argument("--graph", default="yes", choices=["yes", "no"],
                   help="replay the timed launches from one HIP graph (yes) or launch them eagerly")
    return p.parse_args()


def kernel_name(args, dm=None):
    """The dominant kernel as rocprofv3 names it (for profiles/): the C
    plan's own answer (spmv_plan_info) where the format has one."""
    if dm is not None and getattr(dm, "kernel", ""):
        return dm.kernel
    params = (getattr(dm, "params", {}) or {}) if dm is not None else {}
    if args.format == "cmrs" and params.get("variant") == 1:
        return "cmrs_tiled_kernel"
    if dm is not None and "win" in getattr(dm, "arrays", {}):
        if args.format in ("csr16", "csrf32"):  # the CSR x-window kernel with another column / value source
            return "csr_xwin_kernel"
        if args.format == "sell16":  # the SELL kernels with 16-bit column offsets
            return "sell_small_kernel" if params.get("n_slices", 1 << 30) < 14 * 256 else "sell_xwin_kernel"
        return f"{args.format}_xwin_kernel"
    if args.format == "csr":
        v = params.get("variant", 0) or args.variant or CSR_DEFAULT_VARIANT
        return {2: "csr_staged_kernel", 3: "csr_staged_persistent_kernel",
                4: "csr_tiled_kernel"}.get(v, "csr_vector_kernel")
    if args.format == "csr16":
        return "csr_staged_persistent_kernel"
    if args.format in ("coo", "cmrs"):
        return f"{args.format}_staged_kernel"
    return {"sell": "sell_kernel", "ell": "ell_kernel"}.get(args.format, args.format)


def fmt_kwargs(args, fmt):
    if fmt == "csr":
        return {"lanes": args.lanes, "variant": args.variant}
    if fmt == "csr16":
        return {"lanes": args.lanes}
    if fmt == "ell":
        return {"ki": args.ki}
    if fmt == "sell":
        sigma = args.sigma or (1 << 24 if args.workload == "rmat" else 1024)
        return {"C": args.C, "sigma": sigma, "ki": args.ki}
    if fmt == "sell16":
        return {"C": args.C, "sigma": args.sigma or 1024, "ki": args.ki}
    if fmt == "cmrs":
        return {"h": args.h}
    return {}


GRAPH = {"on": True}  # --graph: the timed launches replayed from one HIP graph


def capture(torch, fn, steps):
    """`steps` calls of fn() captured into one HIP graph (None if the capture
    fails: then the launches are timed eagerly)."""
    try:
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(steps):
                fn()
        torch.cuda.synchronize()
        return g
    except Exception as e:  # noqa: BLE001 — fall back to eager launches, say so
        print(f"warning: HIP graph capture failed ({e}); timing eager launches", file=sys.stderr)
        return None


def warm_replays(torch, g, steps, est_ms):
    """Untimed replays of a fresh graph: at least WARM_REPLAY_MS of GPU work
    (est_ms = one launch's time from the eager warm-up), at most 50."""
    n = int(np.ceil(WARM_REPLAY_MS / max(est_ms * steps, 1e-3)))
    for _ in range(min(max(n, 1), 50)):
        g.replay()
    torch.cuda.synchronize()


def time_steps(torch, dm, x, y, steps, warmup, dist=None):
    """W warm-up launches, then exactly `steps` launches bracketed by a
    barrier + synchronize.  Default: the `steps` launches are captured into
    one HIP graph (one SpMV kernel per step, as eager; the graph removes the
    host launch path between them: 0.2473 vs 0.2537 ms per step,
    profiles/round2/ab_graph.log), replayed untimed for >= WARM_REPLAY_MS,
    then replayed once between two HIP events on the launch stream: the
    per-launch time is the span / steps.  --graph no: eager launches with
    one HIP event after each."""
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(warmup):
        dm.run(x, y, stream)
    torch.cuda.synchronize()
    est_ms = (time.perf_counter() - t0) * 1e3 / max(warmup, 1)
    g = capture(torch, lambda: dm.run(x, y), steps) if GRAPH["on"] else None
    if g is not None:
        warm_replays(torch, g, steps, est_ms)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.record(stream)
        g.replay()
        b.record(stream)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        per = a.elapsed_time(b) / steps
        del g
        GRAPH["last"] = "hip-graph"
        return wall, [per] * steps
    GRAPH["last"] = "eager"
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record(stream)
    for i in range(steps):
        dm.run(x, y, stream)
        ev[i + 1].record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern = [ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]  # ms, back-to-back launches
    return wall, kern


def cold_step_ms(torch, dm, x, y, steps):
    """Mean time of an SpMV that starts from cold caches (cold_fn_ms)."""
    return cold_fn_ms(torch, lambda: dm.run(x, y), steps)


def cold_fn_ms(torch, run, steps):
    """Mean time of run() started from cold caches: one graph of `steps` x
    (512 MiB flush + run) minus one graph of `steps` flushes, each replayed
    once untimed and once between HIP events on the stream (the flush is
    ~80 us; the difference of the two spans is run()'s)."""
    stream = torch.cuda.current_stream()
    sa.flush_cache(stream)  # allocates the scratch outside the capture
    torch.cuda.synchronize()
    spans = {}
    for key, fn in (("both", lambda: (sa.flush_cache(), run())), ("flush", lambda: sa.flush_cache())):
        g = capture(torch, fn, steps)
        if g is None:
            return None
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        g.replay()
        b.record(stream)
        torch.cuda.synchronize()
        spans[key] = a.elapsed_time(b)
        del g
    return (spans["both"] - spans["flush"]) / steps


def warm_fn_ms(torch, run, steps):
    """Mean time of run() back to back (cache-resident operands): `steps`
    calls captured in one HIP graph, replayed untimed, then once between HIP
    events on the stream (span / steps)."""
    stream = torch.cuda.current_stream()
    run()
    torch.cuda.synchronize()
    g = capture(torch, run, steps)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if g is None:
        a.record(stream)
        for _ in range(steps):
            run()
        b.record(stream)
    else:
        g.replay()
        torch.cuda.synchronize()
        a.record(stream)
        g.replay()
        b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def traffic_for(fmt, workload_bytes, kernel=None, cold=False):
    """HBM bytes per launch from the committed PMC passes, if they were
    measured on this workload and this kernel (cold: the single-matrix
    passes with a flush before every launch, profiles/traffic_single.json)."""
    for name in (("traffic_single.json",) if cold else ("traffic.json", "traffic_rmat.json")):
        f = REPO / "profiles" / name
        if not f.exists():
            continue
        try:
            t = json.loads(f.read_text()).get(fmt)
        except (ValueError, AttributeError):
            continue
        if not t or int(t.get("bytes_alg", -1)) != int(workload_bytes):
            continue
        if kernel is not None and str(t.get("kernel")) not in str(kernel):  # a name substring of the kernel
            continue
        return t.get("hbm_bytes_per_launch")
    return None


def all_ok(dist, cdev, torch, ok: bool, what: str, rank: int):
    """Parity gate shared by all ranks: the failure flags are all-reduced
    first, so every rank exits non-zero together instead of the healthy ones
    blocking in the next collective."""
    if dist is not None:
        t = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if float(t.item()) != 0.0:
            where = "this rank" if not ok else "another rank"
            raise SystemExit(f"rank {rank}: parity failure on {where} ({what})")
    elif not ok:
        raise SystemExit(f"parity failure ({what})")


def banded_bounds(n, world):
    """Equal 1024-aligned row ranges of the banded matrix."""
    step = (n // world + 1023) // 1024 * 1024
    return [min(r * step, n) for r in range(world)] + [n]


def banded_sample_rows(n, lo, hi):
    """Rows of shard [lo, hi) checked at full size: the first and last 512,
    128 around every 2-, 4- and 8-way cut point, 4096 spread evenly, and
    rows whose CSR entries lie past 2^31 and 2^32 bytes of values (entry
    2^28 = row 2^24 onward: the int64-offset path)."""
    cand = [np.arange(lo, min(lo + 512, hi)), np.arange(max(hi - 512, lo), hi),
            np.linspace(lo, hi - 1, 4096).astype(np.int64)]
    for parts in (2, 4, 8):
        for cut in banded_bounds(n, parts)[1:-1]:
            cand.append(np.arange(max(cut - 64, lo), min(cut + 64, hi)))
    for r0 in (1 << 24, 1 << 25, 3 << 24, 1 << 26):  # value bytes 2^31, 2^32, 3*2^31, 2^33
        cand.append(np.arange(max(r0 - 32, lo), min(r0 + 32, hi)))
    cand = [c for c in cand if c.size]
    rows = np.unique(np.concatenate(cand)) if cand else np.zeros(0, np.int64)
    return rows[(rows >= lo) & (rows < hi)]


def banded_check(n, lo, hi, y_shard):
    """Full-range banded parity with x[j] = j (a wrong column index changes
    y, unlike with x = 1): every sampled row (banded_sample_rows) recomputed
    from the host generator in file order (the check_result rule, reference
    csr.c:225-233), relative 1e-6 of sum |a_ij x_j|.  Returns (rows checked,
    first bad rows or None)."""
    rows = banded_sample_rows(n, lo, hi)
    if rows.size == 0:
        return 0, None
    got = y_shard.cpu().numpy()[rows - lo]
    runs = np.split(rows, np.nonzero(np.diff(rows) != 1)[0] + 1)
    bad, k = [], 0
    for run in runs:
        _, c, v = sa.gen_banded_csr(n, int(run[0]), int(run[-1]) + 1)
        c, v = c.reshape(-1, 16), v.reshape(-1, 16)
        xv = c.astype(np.float64)  # x[j] = j
        ref = np.zeros(run.size)
        for e in range(16):  # file order
            ref = ref + v[:, e] * xv[:, e]
        scale = np.sum(np.abs(v * xv), axis=1)
        err = np.abs(got[k:k + run.size] - ref) > 1e-6 * scale
        bad.extend(run[err].tolist())
        k += run.size
    return int(rows.size), (bad[:5] if bad else None)


def build_workload(args, torch, dev, rank, world):
    """This rank's share of the workload, resident in HBM.

    cantlike (default, weak scaling): rank r owns copies [r·B, (r+1)·B) of
        a block-diagonal stack of cant-like matrices; its x block is local.
    rmat (strong scaling, BASELINE.json configs[3] / north-star sweep): the
        1e7 x 1e7 / 1e8-entry R-MAT, rows cut by spmv_partition_rows into
        nnz-balanced ranges aligned to 1024; x replicated.
    banded (strong scaling, configs[4]): the 1e8-row / 1.6e9-entry banded
        matrix, equal row ranges, each shard generated on its GPU.
    """
    fk = fmt_kwargs(args, args.format)
    if args.workload == "batch":
        B = args.copies
        m = sa.gen_cantlike(0, B)
        x = torch.from_numpy(sa.ramp_x(m.n_cols) + rank * m.n_cols).to(dev)  # this shard's x block
        y = torch.empty(m.n_rows, dtype=torch.float64, device=dev)
        dm = sa.to_device(m, args.format, dev, **fk)
        b = sa.bytes_alg(m.n_rows, m.n_cols, m.nnz)

        def check():  # the whole batch, all B copies (host check_result rule)
            bad, first = sa.check(m, x.cpu().numpy(), y.cpu().numpy())
            return f"row {first}" if bad else None

        return dict(dm=dm, x=x, y=y, m=m, rows=m.n_rows, nnz=m.nnz, bytes_rank=b, bytes_total=b * world,
                    nnz_total=m.nnz * world, check=check, scaling="weak",
                    data="synthetic: cant-like stand-in (62,451 rows, 4,007,383 entries = SuiteSparse cant's "
                         "counts; the reference's cant.mtx is an unfetched Git-LFS pointer), x[j] = j",
                    config={"workload": f"{args.format} SpMV over a batch: {B} independent cant-like matrices "
                                        "(BASELINE.json configs[1]'s matrix) per GPU stacked block-diagonally, "
                                        "one launch per step, 1.58 GB per GPU streamed from HBM; the single "
                                        "49 MB matrix (Infinity-Cache resident when warm) is cant_single",
                            "copies_per_gpu": B})
    if args.workload == "rmat":
        full = rmat_matrix(args)  # deterministic: every rank builds the same matrix
        ptr, col, val = sa.csr_from_coo(full)
        n, z = full.n_rows, full.nnz
        del full
        col, xh, hot, layout, _ = rmat_layout(args, n, ptr, col, val)
        bounds = sa.partition_rows(n, ptr, world, align=1024, row_weight=RMAT_ROW_WEIGHT)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        lptr = ptr[lo:hi + 1] - ptr[lo]
        loc = sa.Coo(hi - lo, n, np.repeat(np.arange(hi - lo, dtype=np.int32), np.diff(lptr)),
                     col[ptr[lo]:ptr[hi]], val[ptr[lo]:ptr[hi]])
        x = torch.from_numpy(xh).to(dev)
        y = torch.empty(max(loc.n_rows, 1), dtype=torch.float64, device=dev)
        if hot is not None:
            fk = dict(fk, hot=hot)
        dm = sa.to_device(loc, args.format, dev, **fk)

        def check():
            bad, first = sa.check(loc, xh, y[:loc.n_rows].cpu().numpy())
            return f"row {first}" if bad else None

        return dict(dm=dm, x=x, y=y, loc=loc, rows=loc.n_rows, nnz=loc.nnz, hot=hot,
                    bytes_rank=sa.bytes_alg(loc.n_rows, loc.n_cols, loc.nnz), bytes_total=sa.bytes_alg(n, n, z),
                    nnz_total=z, check=check, scaling="strong",
                    data=f"synthetic: R-MAT (a,b,c,d)=(.57,.19,.19,.05), {n:.0e} rows, {z:.0e} entries, seed 1, "
                         "x[j] = j",
                    config={"workload": f"{args.format} SpMV on R-MAT {n:.0e}/{z:.0e} row-sharded over {world} "
                                        "GPU(s) (BASELINE.json configs[3])", "layout": layout})
    # banded
    n = args.banded_rows
    lo, hi = banded_bounds(n, world)[rank:rank + 2]
    if args.format == "sell":
        dm = sa.banded_to_device(n, "sell", dev, lo, hi, C=args.C, sigma=1024, ki=args.ki or 1)
    elif args.format == "csr":
        dm = sa.banded_to_device(n, "csr", dev, lo, hi, lanes=args.lanes, variant=args.variant)
    else:
        raise SystemExit("--workload banded supports --format csr or sell")
    x = torch.from_numpy(sa.ramp_x(n)).to(dev)
    y = torch.empty(max(hi - lo, 1), dtype=torch.float64, device=dev)

    def check():
        k, bad = banded_check(n, lo, hi, y)
        return f"banded rows {bad} ({k} rows sampled)" if bad else None

    return dict(dm=dm, x=x, y=y, rows=hi - lo, nnz=16 * (hi - lo), lo=lo, hi=hi, bounds=banded_bounds(n, world),
                bytes_rank=sa.bytes_alg(hi - lo, n, 16 * (hi - lo)) - 8 * n + 8 * (hi - lo),
                bytes_total=sa.bytes_alg(n, n, 16 * n), nnz_total=16 * n, check=check, scaling="strong",
                data=f"synthetic: banded, {n} rows x 16 entries at offsets -8..7 (mod n), generated on device, "
                     "x[j] = j",
                config={"workload": f"{args.format} SpMV on the banded {n}-row / {16 * n}-entry matrix "
                                    f"row-sharded over {world} GPU(s) (BASELINE.json configs[4])"})


CPU_SWEEP_BYTES = 2 << 30  # > every host's last-level caches together (cold CPU passes)


def cpu_baseline(m_single_csr, copies, budget_s, cold=False):
    """The oracle's restatement of the reference's OpenMP CSR loop
    (reference csr.c:285-309) on the same batch, bounded to ~budget_s.
    cold: before every timed pass all threads sweep a 2 GiB buffer
    (oracle_sweep), so the pass reads the matrix from DRAM, as the cold GPU
    step reads it from HBM; the sweep is not timed."""
    from oracle import oracle

    ptr, col, val, n_rows, n_cols = m_single_csr
    # the batch is `copies` identical block-diagonal copies: time whole
    # passes over a host batch built the same way as the device one
    B = copies
    bptr = np.concatenate([ptr[:-1] + k * ptr[-1] for k in range(B)] + [np.array([B * ptr[-1]], np.int64)])
    bcol = np.concatenate([col + k * n_cols for k in range(B)]).astype(np.int32)
    bval = np.tile(val, B)
    x = np.arange(B * n_cols, dtype=np.float64)
    y = np.empty(B * n_rows, np.float64)
    threads = oracle.max_threads()
    scratch = np.zeros(CPU_SWEEP_BYTES, np.uint8) if cold else None
    times = []
    t_end = time.perf_counter() + budget_s
    while time.perf_counter() < t_end or len(times) < 3:
        if cold:
            oracle.sweep(scratch, threads)
        times.append(oracle.cpu_csr_omp(B * n_rows, bptr, bcol, bval, x, y, threads))
        if len(times) >= 200_000:  # ~10 s of passes on one cant-like matrix (~0.1 ms each)
            break
    t = float(np.median(times))
    b = sa.bytes_alg(B * n_rows, B * n_cols, B * int(ptr[-1]))
    state = ("cold: a 2 GiB all-thread sweep before every pass evicts the host caches (not timed)" if cold
             else "warm: every pass re-reads what the last one left in the host caches")
    return {"value": round(b / t * 1e-9, 2), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"oracle OpenMP CSR loop (reference csr.c:285-309) over the same {B}-copy batch, "
                      f"{len(times)} passes in ~{sum(times):.1f} s of timed passes, median {t * 1e3:.3f} ms/pass; "
                      + state,
            "state": "cold" if cold else "warm",
            "gflops": round(2 * B * int(ptr[-1]) / t * 1e-9, 2)}


def child_device_env(local: int) -> dict:
    """Environment of a per-rank child that must see only this rank's GPU
    (as its cuda:0): HIP_VISIBLE_DEVICES = the rank's entry of any visible
    list the launcher already set, else the local rank."""
    env = dict(os.environ)
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if env.get(var):
            ids = [t for t in env[var].split(",") if t.strip()]
            if local < len(ids):
                env["HIP_VISIBLE_DEVICES"] = ids[local].strip()
                env.pop("CUDA_VISIBLE_DEVICES", None)
                return env
    env["HIP_VISIBLE_DEVICES"] = str(local)
    env.pop("CUDA_VISIBLE_DEVICES", None)
    return env


def cant_single_rocprof(formats=None, local=None, flush_mode="read"):
    """tools/cant_single.py under `rocprofv3 --kernel-trace` as a child
    process, run before this process touches the GPU: formats (default
    every format) on ONE cant-like matrix, cold and warm, kernel durations
    from the trace, beside the stream ceiling of the same bytes.  `local`
    (a rank's local GPU): the child sees only that GPU.  Without rocprofv3
    (or if the profiled run fails) the child runs unprofiled and its
    HIP-event figures are reported, labelled so."""
    tool = REPO / "tools" / "cant_single.py"
    rocprof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    env = child_device_env(local) if local is not None else None
    with tempfile.TemporaryDirectory(prefix="cant_single_") as tmp:
        out = Path(tmp) / "cant_single.json"
        plain = [sys.executable, str(tool), "--json", str(out), "--flush-mode", flush_mode]
        if formats:
            plain += ["--formats", ",".join(formats)]
        traced = Path(rocprof).exists()
        cmd = ([rocprof, "--kernel-trace", "--stats", "--output-format", "csv", "-d", tmp, "-o", "run", "--"] + plain
               if traced else plain)
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=420, cwd=str(REPO), env=env)
            if traced and (r.returncode != 0 or not out.exists()):
                traced = False
                r = subprocess.run(plain, capture_output=True, text=True, timeout=300, cwd=str(REPO), env=env)
        except subprocess.TimeoutExpired:
            return {"error": "cant_single timed out"}
        if r.returncode != 0 or not out.exists():
            return {"error": f"cant_single failed (rc {r.returncode}): {r.stderr[-400:]}"}
        res = json.loads(out.read_text())
        if traced:
            from cant_single import attach_trace

            attach_trace(res, tmp)
            # the profiler's own --stats summary of the same run (every launch
            # of a kernel, cold and warm together)
            stats = sorted(Path(tmp).rglob("*kernel_stats.csv"))
            if stats:
                import csv

                res["rocprof_kernel_stats"] = [
                    {"kernel": r["Name"].replace("void ", "").split("(")[0], "calls": int(r["Calls"]),
                     "avg_ns": round(float(r["AverageNs"]), 1), "min_ns": int(float(r["MinNs"])),
                     "max_ns": int(float(r["MaxNs"]))}
                    for r in csv.DictReader(open(stats[-1], newline="")) if "spmv::" in r["Name"]]
        else:
            res["timing"] = "HIP events around each launch (no rocprofv3 trace): includes event overhead"
    res.pop("phases", None)
    return res


def single_cold(args, torch, dev, rank, world, dist, cdev, prof, fmt=None):
    """The headline (BASELINE.json configs[1]; configs[2] with --format
    sell): ONE cant-like matrix on this rank's GPU, cold.  A step = 512 MiB
    flush + one SpMV launch.  W untimed warm-up steps; then the K steps are
    captured in one HIP graph, replayed once untimed, and replayed once
    between barrier + synchronize on both sides (the timed region); a graph
    of K flushes alone is timed the same way right before and right after it,
    so the in-process cold SpMV time is
    (span(K x (flush + SpMV)) - mean span(K x flush)) / K; the region is
    replayed INPROC_REPS times (F B F B ... F) and the median taken, max over
    ranks: the headline.  The rocprofv3 trace median and mean of the same
    kernel cold (`prof`, this rank's cant_single child) go beside it.
    fmt: the format (default --format; "sell" for the sell_single record,
    BASELINE.json configs[2])."""
    fmt = fmt or args.format
    m = sa.gen_cantlike(0, 1)
    b = sa.bytes_alg(m.n_rows, m.n_cols, m.nnz)
    fk = fmt_kwargs(args, fmt)
    xh = sa.ramp_x(m.n_cols)
    x = torch.from_numpy(xh).to(dev)
    y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
    dm = sa.to_device(m, fmt, dev, **fk)
    stream = torch.cuda.current_stream()
    # the same flush as the traced child (tools/cant_single.py): a 512 MiB
    # scratch written by probe_flush_kernel, so both measure one cold state
    from cant_single import FLUSH_BYTES, probe_lib

    probe = probe_lib()
    scratch = torch.empty(FLUSH_BYTES, dtype=torch.uint8, device=dev)
    sink = torch.zeros(64, dtype=torch.int32, device=dev)

    def flush_write():
        assert probe.spmv_probe_flush(scratch.data_ptr(), FLUSH_BYTES, torch.cuda.current_stream().cuda_stream) == 0

    def flush_read():  # the same eviction by READING 512 MiB: clean lines, nothing to write back
        assert probe.spmv_probe_flush_read(scratch.data_ptr(), FLUSH_BYTES, sink.data_ptr(),
                                           torch.cuda.current_stream().cuda_stream) == 0

    modes = {"write": flush_write, "read": flush_read}
    flush = modes[args.cold_flush]
    other = modes["read" if args.cold_flush == "write" else "write"]
    flush_write()
    torch.cuda.synchronize()

    def step():
        flush()
        dm.run(x, y)

    def timed(fn, k):
        """fn's k calls as one graph (None: eager) and a timer: each call of the
        timer replays it once between barrier + synchronize, returning (wall s,
        GPU span ms on the launch stream)."""
        g = capture(torch, fn, k) if GRAPH["on"] else None
        if g is not None:
            g.replay()
            torch.cuda.synchronize()

        def run():
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a.record(stream)
            if g is not None:
                g.replay()
            else:
                for _ in range(k):
                    fn()
            e.record(stream)
            torch.cuda.synchronize()
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            return time.perf_counter() - t0, a.elapsed_time(e)
        return run

    def inprocess(both_fn, flush_fn, k, reps):
        """Cold SpMV time from `reps` timed regions of k x (flush + SpMV), each
        between two replays of k flushes alone (F B F B ... F): per region
        (span_B - mean of its two F spans) / k, and the median of those.  One
        difference alone moved +-0.5 us between repeats on the same arrays
        (1 % of the ~95 us flush is ~1 us; tools/inproc_noise.py,
        profiles/round6/inproc_noise.md); the median of 5 interleaved ones is
        what the line reports, every difference beside it."""
        tb, tf = timed(both_fn, k), timed(flush_fn, k)
        f = [tf()[1]]
        walls, diffs = [], []
        for _ in range(reps):
            w, b_ = tb()
            f.append(tf()[1])
            walls.append(w)
            diffs.append((b_ - 0.5 * (f[-2] + f[-1])) / k)
        return walls[0], max(float(np.median(diffs)), 1e-6), diffs, [v / k for v in f]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    K = args.steps
    reps = 1 if args.profile else INPROC_REPS
    wall, inproc, diffs, flush_spans = inprocess(step, flush, K, reps)
    # the other cold state beside it (not the headline; not in --profile runs,
    # whose PMC passes average every launch of the kernel)
    inproc_other = None
    node_ms = None
    if not args.profile:
        _, inproc_other, _, _ = inprocess(lambda: (other(), dm.run(x, y)), other, K, reps)
        # what the estimator charges ANY kernel node: the same F B F ... F
        # measurement of an empty one-workgroup kernel (tools/probe.hip
        # spmv_probe_tag) — the graph's launch gap plus an empty dispatch,
        # which the rocprofv3 kernel time does not contain
        _, node_ms, _, _ = inprocess(lambda: (flush(), probe.spmv_probe_tag(1, torch.cuda.current_stream().cuda_stream)),
                                     flush, K, reps)
    bad, first = sa.check(m, xh, y.cpu().numpy())
    all_ok(dist, cdev, torch, bad == 0, f"cant-like single matrix, row {first}", rank)

    # the headline is the in-process figure: the timed region's
    # own span difference; the child's rocprofv3 trace of the same kernel
    # cold (median and mean of 50 launches) is reported beside it
    rec = (prof or {}).get("formats", {}).get(fmt, {}) if isinstance(prof, dict) else {}
    traced, traced_mean = rec.get("cold_ms"), rec.get("cold_ms_mean")
    t = torch.tensor([inproc, wall * 1e3 / K], dtype=torch.float64, device=cdev)
    per_rank = [float(t[0].item())]
    if dist is not None:
        g = [torch.zeros(2, dtype=torch.float64, device=cdev) for _ in range(world)]
        dist.all_gather(g, t)
        per_rank = [float(v[0].item()) for v in g]
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    cold_ms, wall_step = (float(v) for v in t.tolist())
    kernels = rec.get("kernels") or [kernel_name(argparse.Namespace(**dict(vars(args), format=fmt)), dm)]
    params = {k: v for k, v in dm.params.items() if isinstance(v, (int, float, str))}
    del dm
    torch.cuda.empty_cache()
    corr = None
    if traced:
        corr = {"kernel_ms_median": traced, "kernel_ms_mean": traced_mean,
                "in_process_over_trace_mean": round(cold_ms / traced_mean, 4) if traced_mean else None,
                "in_process_over_trace_median": round(cold_ms / traced, 4),
                "source": "rocprofv3 kernel trace of tools/cant_single.py, 50 cold launches" +
                          (" (rank 0's GPU)" if world > 1 else ""),
                "note": "the in-process span difference also holds the gap between the flush and the SpMV "
                        "kernel inside the graph (~1 us); the trace times the kernel alone"}
    return {"format": fmt, "cold_ms": cold_ms, "bytes": b, "nnz": m.nnz, "rows": m.n_rows, "kernels": kernels,
            "params": params,
            "source": "in-process: (span of K x (flush + SpMV) - span of K x flush) / K, HIP events on the launch "
                      "stream, max over ranks",
            "trace": corr,
            "timed_region": {"what": f"{K} x (512 MiB flush + one SpMV), "
                                     + ("one HIP graph replay" if GRAPH["on"] else "eager launches")
                                     + " between barrier + synchronize"
                                     + (f"; {reps} such regions, interleaved with flush-only ones" if reps > 1 else ""),
                             "wall_ms": round(wall * 1e3, 4), "wall_ms_per_step_incl_flush": round(wall_step, 5),
                             "cold_spmv_ms_in_process": round(cold_ms, 5),
                             "in_process_estimator": f"median of {reps} timed regions, each minus the mean of "
                                                     "the flush-only spans before and after it",
                             "cold_spmv_ms_each_region": [round(v, 5) for v in diffs],
                             "empty_kernel_node_ms": round(node_ms, 5) if node_ms is not None else None,
                             "empty_kernel_node_note": "the same estimator applied to an empty one-workgroup kernel: "
                                                       "the per-node launch gap any kernel is charged here and the "
                                                       "rocprofv3 kernel time leaves out (a diagnostic; value keeps it)",
                             "flush_only_ms_per_step": [round(v, 5) for v in flush_spans],
                             "cold_flush": f"{args.cold_flush}: 512 MiB " +
                                           ("written" if args.cold_flush == "write" else "read") +
                                           " before every SpMV (evicts the Infinity Cache and the L2s)",
                             "cold_spmv_ms_in_process_other_flush": {
                                 ("read" if args.cold_flush == "write" else "write"):
                                     round(inproc_other, 5) if inproc_other else None},
                             "cold_spmv_ms_rocprof_rank0": traced,
                             "cold_ms_per_rank": [round(v, 5) for v in per_rank]},
            "parity_ok": True,
            "check": "all 62,451 rows of y against the host check_result rule (1e-6 relative), every rank"}


def strong_exchange(torch, comm, cdev, dm, x, y_full, lo, hi, bounds, steps, flush):
    """The exchange step of a row-sharded SpMV: y all-gathered with the REAL
    shard sizes (iterate.Comm.allgatherv), timed alone and after the SpMV,
    per step, max over ranks; with `flush` also the shard's cold SpMV time
    (cold_step_ms), all ranks' values gathered.  y_full holds this rank's
    rows [lo, hi); the all-gather fills the rest in place."""
    dist = comm.dist
    yv = y_full[lo:hi]

    def spmv():
        if hi > lo:
            dm.run(x, yv)

    how = comm.allgatherv(y_full, bounds)

    def timed(fn, k):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        return (time.perf_counter() - t0) * 1e3 / k

    ag_ms = timed(lambda: comm.allgatherv(y_full, bounds), steps)
    both_ms = timed(lambda: (spmv(), comm.allgatherv(y_full, bounds)), steps)
    t = torch.tensor([ag_ms, both_ms], dtype=torch.float64, device=cdev)
    cold = None
    if flush:
        c = cold_step_ms(torch, dm, x, yv, max(5, steps // 2)) if hi > lo else 0.0
        cold = [c if c is not None else -1.0]
        if dist is not None:
            g = [torch.zeros(1, dtype=torch.float64, device=cdev) for _ in range(comm.world)]
            dist.all_gather(g, torch.tensor(cold, dtype=torch.float64, device=cdev))
            cold = [float(v.item()) for v in g]
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return how, float(t[0].item()), float(t[1].item()), cold


def rmat_matrix(args):
    """The R-MAT of configs[3] (default 1e7 rows / 1e8 entries; smaller with
    --rmat-rows / --rmat-nnz for tests), deterministic on every rank."""
    n, z = args.rmat_rows, args.rmat_nnz
    return sa.gen_rmat(n, z, scale=max(1, (n - 1).bit_length()))


def rmat_layout(args, n, ptr, col, val):
    """(col, x host, hot kwarg, label, order): with the relabel (default) the CSR's
    columns are renumbered by decreasing degree once at build time and x is
    replicated in that layout (x'[k] = x[order[k]]: the replication step,
    SURVEY.md §8e, delivers it; outside the timed SpMV), so no per-run
    hot-table fill runs and the touched part of x is one dense prefix; then
    every row's entries are ordered by the new column (spmv_csr_sort_rows,
    in place on col and val), so a long row reads that prefix in address
    order (whole R-MAT cold 0.762 -> 0.734 ms, profiles/round5/ab_rmat_sort_rows.md);
    y keeps the original row order.  Otherwise the per-run hot-column
    table on the file-order rows.  order: x'[k] = x[order[k]] (None
    without the relabel)."""
    xh = sa.ramp_x(n)
    if args.relabel == "no":
        return col, xh, None, "hot-column table (per-run fill of the 2^19 hottest x entries)", None
    order, _, col2 = sa.column_relabel(n, col, args.relabel_ties)
    sa.csr_sort_rows(n, ptr, col2, val)
    ties = "first row" if args.relabel_ties == "first" else "column id"
    return col2, np.ascontiguousarray(xh[order]), 0, (f"columns relabelled by decreasing degree at build time, "
                                                     f"ties by {ties} (spmv_column_relabel_ex), each row's entries "
                                                     "in new-column order (spmv_csr_sort_rows); x replicated in "
                                                     "that layout"), order


RMAT_HOT_FORMATS = ("coo", "csr", "csrf32", "cmrs", "sell", "hyb")  # formats with a hot-column table option


def rmat_fmt_kwargs(args, fmt, hot):
    """to_device keywords of `fmt` on the R-MAT (configs[3]): the format's
    defaults, SELL sorted over the whole matrix (sigma 2^24), and hot = 0
    (no per-run table) on the relabelled layout."""
    kw = fmt_kwargs(argparse.Namespace(**dict(vars(args), workload="rmat")), fmt)
    if hot is not None and fmt in RMAT_HOT_FORMATS:
        kw = dict(kw, hot=hot)
    return kw


def rmat_strong(args, torch, dev, rank, world, dist, cdev):
    """North-star sweep (BASELINE.json north_star, configs[3]): CSR on the
    1e7 x 1e7 / 1e8-entry R-MAT, rows cut into `world` shards, one per
    rank, x replicated; aggregate GB/s = bytes_alg(whole matrix) / max over
    ranks of the per-step time (HIP-graph replay between barriers).

    The cut is profile-guided: the weighted cut (entries + RMAT_ROW_WEIGHT
    x rows, 1024-aligned) is timed (20 steps), every rank's shard time is
    all-gathered, and spmv_partition_rows_calibrated re-cuts the rows into
    equal shares of the measured cost (`calibration`, on cold times with
    --flush yes); the measured cut with the lowest max shard time is kept
    (the same on every rank).  Setup only: the timed steps are the same
    SpMV on the final shards.  At N > 1, rank 0 first times the WHOLE
    matrix alone (warm and cold) in the same job, so the line carries its
    own strong-scaling speed-ups (speedup_warm / speedup_cold = whole /
    max shard).  Then the exchange on the final cut (strong_exchange): y
    all-gathered with the real shard sizes, SpMV + all-gather, cold
    shards.  Every rank checks its shard; rank 0 checks the whole gathered
    y against the ORIGINAL (un-relabelled) matrix and x."""
    t0 = time.perf_counter()
    full = rmat_matrix(args)  # deterministic: every rank builds the same matrix
    ptr, col, val = sa.csr_from_coo(full)
    n, z = full.n_rows, full.nnz
    if rank != 0:
        del full
    col, xh, hot, layout, order = rmat_layout(args, n, ptr, col, val)
    x = torch.from_numpy(xh).to(dev)
    b_total = sa.bytes_alg(n, n, z)
    steps = max(20, args.steps // 2)
    calib = args.flush == "yes"  # cut on COLD shard times (each shard flushed first), else warm
    recuts = RMAT_RECUTS if args.recuts is None else args.recuts

    def rows_of(lo, hi):
        lptr = ptr[lo:hi + 1] - ptr[lo]
        return sa.Coo(hi - lo, n, np.repeat(np.arange(hi - lo, dtype=np.int32), np.diff(lptr)),
                      col[ptr[lo]:ptr[hi]], val[ptr[lo]:ptr[hi]])

    def shard(bounds):
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        loc = rows_of(lo, hi)
        return loc, sa.to_device(loc, "csr", dev, hot=hot), lo, hi

    # the whole matrix alone on rank 0 (N > 1): the 1-GPU reference of the
    # speed-ups, measured in the same job as the shards
    whole = None
    if world > 1:
        if rank == 0:
            loc = rows_of(0, n)
            dm = sa.to_device(loc, "csr", dev, hot=hot)
            y = torch.empty(n, dtype=torch.float64, device=dev)
            _, kern = time_steps(torch, dm, x, y, 20, 5)
            bad, first = sa.check(loc, xh, y.cpu().numpy())
            c = cold_step_ms(torch, dm, x, y, 10) if calib else None
            whole = {"ms": float(np.mean(kern)), "cold_ms": c, "parity_ok": bad == 0}
            del dm, y, loc
            torch.cuda.empty_cache()
            if bad:
                print(f"rank 0: whole R-MAT parity failure at row {first}", file=sys.stderr)
        all_ok(dist, cdev, torch, whole is None or whole["parity_ok"], "whole R-MAT (rank 0 alone)", rank)

    def run(bounds, k, cold=False):
        """Warm steps of the cut (and with `cold`, each shard's cold time,
        bench.cold_step_ms); every rank's shard times gathered."""
        loc, dm, _, _ = shard(bounds)
        y = torch.empty(max(loc.n_rows, 1), dtype=torch.float64, device=dev)
        wall, kern = time_steps(torch, dm, x, y, k, 5, dist)
        bad, first = sa.check(loc, xh, y[:loc.n_rows].cpu().numpy())
        all_ok(dist, cdev, torch, bad == 0, f"R-MAT shard row {first}", rank)
        params = {kk: v for kk, v in dm.params.items() if isinstance(v, (int, float, str))}
        t = torch.tensor([wall / k * 1e3, float(np.mean(kern))], dtype=torch.float64, device=cdev)
        c = (cold_step_ms(torch, dm, x, y, 10) or -1.0) if cold else -1.0
        mine = torch.tensor([float(np.mean(kern)), c], dtype=torch.float64, device=cdev)
        shard_ms, shard_cold = [float(mine[0].item())], [c]
        if dist is not None:
            g = [torch.zeros(2, dtype=torch.float64, device=cdev) for _ in range(world)]
            dist.all_gather(g, mine)
            shard_ms = [float(v[0].item()) for v in g]
            shard_cold = [float(v[1].item()) for v in g]
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        del dm, y
        torch.cuda.empty_cache()
        return float(t[0].item()), float(t[1].item()), shard_ms, params, shard_cold

    bounds0 = sa.partition_rows(n, ptr, world, align=1024, row_weight=RMAT_ROW_WEIGHT)
    step0, _, shard0, _, cold0 = run(bounds0, 20, cold=calib and world > 1)
    bounds, passes = bounds0, []
    if world > 1:  # re-cuts, each from the previous cut's measured (cold) times;
        key0 = cold0 if calib and min(cold0) > 0 else shard0
        b, t, best = bounds0, key0, (max(key0), bounds0)  # the measured cut with the lowest max is kept
        for _ in range(recuts):
            nb = sa.partition_rows_calibrated(n, ptr, world, b, t, align=1024, row_weight=RMAT_ROW_WEIGHT)
            b = sa.partition_rows_damped(n, b, nb, RMAT_DAMP)
            _, _, tw, _, tc = run(b, 20, cold=calib)
            t = tc if calib and min(tc) > 0 else tw
            passes.append({"shard_rows": np.diff(b).tolist(), "shard_ms": [round(v, 5) for v in tw],
                           "shard_ms_cold": [round(v, 5) for v in tc] if calib else None})
            best = min(best, (max(t), b), key=lambda cc: cc[0])
        bounds = best[1]
    step_ms, kern_ms, shard_ms, params, _ = run(bounds, steps)

    # the exchange on the final cut
    comm = iterate.Comm(dist)
    _, dm, lo, hi = shard(bounds)
    y_full = torch.full((n,), float("nan"), dtype=torch.float64, device=dev)
    how, ag_ms, both_ms, cold = strong_exchange(torch, comm, cdev, dm, x, y_full, lo, hi, bounds, steps,
                                                args.flush == "yes")
    bad_whole = None
    if rank == 0:  # the gathered y against the ORIGINAL matrix and x (host rule)
        bad, first = sa.check(full, sa.ramp_x(n), y_full.cpu().numpy())
        bad_whole = None if bad == 0 else f"gathered R-MAT y, row {first}"
    all_ok(dist, cdev, torch, bad_whole is None, str(bad_whole), rank)
    del dm, y_full
    torch.cuda.empty_cache()
    # the relabelled layout takes x' = x[order]: what a new x pays before the
    # SpMV (spmv_gather, 1e7 x (4 + 8 + 8) B), timed beside it, not inside it
    permute = None
    if order is not None:
        od = torch.from_numpy(order).to(dev)
        x0 = torch.from_numpy(sa.ramp_x(n)).to(dev)
        xp = torch.empty_like(x0)
        sa.gather_x(od, x0, xp)
        torch.cuda.synchronize()
        assert torch.equal(xp, x), "spmv_gather x' differs from the host permutation"
        pw = warm_fn_ms(torch, lambda: sa.gather_x(od, x0, xp), 20)
        pc = cold_fn_ms(torch, lambda: sa.gather_x(od, x0, xp), 10)
        permute = {"what": "x' = x[order] on the device (spmv_gather): the relabelled layout's input, paid once per "
                           "new x; NOT inside ms_per_step (an iterated solver keeps its vectors in that layout)",
                   "warm_ms": round(pw, 5), "cold_ms": round(pc, 5) if pc else None,
                   "bytes": 20 * n}
        del od, x0, xp
    per_format = gather_ceiling = None
    if rank == 0 and world == 1 and args.rmat_per_format != "no":
        loc = rows_of(0, n)
        gather_ceiling = rmat_gather_ceiling(torch, dev, loc, x, b_total)
        per_format = rmat_per_format(args, torch, dev, loc, x, full, hot, b_total, gather_ceiling)
        del loc
    if rank == 0:
        del full
    torch.cuda.empty_cache()

    def gbs(ms):
        return round(b_total / (ms * 1e-3) * 1e-9, 1) if ms and ms > 0 else None

    out = {"workload": f"csr SpMV on R-MAT {n:.0e}/{z:.0e} (configs[3]) row-sharded over all ranks, x replicated",
           "layout": layout, "scaling": "strong", "steps": steps,
           "aggregate_GBs": gbs(step_ms),
           "GFLOPs": round(2 * z / (step_ms * 1e-3) * 1e-9, 1),
           "frac_of_one_gpu_peak": round(b_total / (step_ms * 1e-3) * 1e-9 / sa.HBM_PEAK_GBS, 4),
           "ms_per_step": round(step_ms, 5), "max_shard_kernel_ms": round(kern_ms, 5),
           "shard_ms": [round(v, 5) for v in shard_ms], "shard_rows": np.diff(bounds).tolist(),
           "bytes_alg_whole": b_total, "params_rank0": params, "parity_ok": True,
           "allgather": {"how": how, "bytes_received_rank0": 8 * (n - (hi - lo)) if rank == 0 else None,
                         "ms": round(ag_ms, 5), "spmv_plus_allgather_ms": round(both_ms, 5),
                         "aggregate_GBs_with_allgather": gbs(both_ms),
                         "gathered_y_parity": "rank 0 checks all rows of the gathered y against the original "
                                              "matrix and x"},
           "partition": ("profile-guided: weighted cut (row weight %g) and %d re-cuts by measured %s cost "
                         "(each moving the cut points %g of the way) timed, the one with the lowest max %s "
                         "shard time kept" % (RMAT_ROW_WEIGHT, recuts, "cold" if calib else "warm", RMAT_DAMP,
                                               "cold" if calib else "warm"))
                        if world > 1 else "whole matrix",
           "calibration": {"weighted_cut": {"shard_rows": np.diff(bounds0).tolist(),
                                            "shard_ms": [round(v, 5) for v in shard0],
                                            "shard_ms_cold": [round(v, 5) for v in cold0] if calib and world > 1
                                            else None,
                                            "aggregate_GBs": gbs(step0)},
                           "recuts": passes},
           "setup_s": round(time.perf_counter() - t0, 1)}
    if cold is not None:
        cm = max(cold)
        out["cold"] = {"how": "per rank: graph of K x (512 MiB flush + SpMV) minus a graph of K flushes",
                       "shard_ms": [round(v, 5) for v in cold], "max_shard_ms": round(cm, 5),
                       "aggregate_GBs": gbs(cm)}
    # strong-scaling speed-ups from this job's own 1-GPU figure (rank 0 alone)
    w_ms = whole["ms"] if whole else kern_ms
    w_cold = (whole or {}).get("cold_ms") if world > 1 else (min(cold) if cold else None)
    out["whole_matrix_one_gpu"] = {"ms": round(w_ms, 5), "cold_ms": round(w_cold, 5) if w_cold else None,
                                   "how": "rank 0 alone, before the shards, same job" if world > 1
                                          else "N = 1: the one shard is the whole matrix"}
    out["speedup_warm"] = round(w_ms / kern_ms, 3) if kern_ms > 0 else None
    out["speedup_cold"] = round(w_cold / max(cold), 3) if w_cold and cold and max(cold) > 0 else None
    if permute is not None:
        permute["spmv_plus_permute_ms"] = round(step_ms + permute["warm_ms"], 5)
        permute["aggregate_GBs_with_permute"] = gbs(step_ms + permute["warm_ms"])
        if cold and permute.get("cold_ms"):
            permute["spmv_plus_permute_cold_ms"] = round(max(cold) + permute["cold_ms"], 5)
        # one step of an iterated solver in this layout: SpMV, y all-gather,
        # then x' = P y on every rank (the relabel is columns-only)
        permute["spmv_allgather_permute_ms"] = round(both_ms + permute["warm_ms"], 5)
        permute["aggregate_GBs_iterated_step"] = gbs(both_ms + permute["warm_ms"])
    out["x_permute"] = permute
    out["gather_ceiling"] = gather_ceiling
    out["per_format"] = per_format
    return out


def rmat_gather_ceiling(torch, dev, loc, x, b_total):
    """The gather ceiling of the R-MAT's own access pattern
    (spmv_probe_gather_stream, tools/probe.hip): its value / column arrays
    streamed in entry order (the relabelled, row-sorted layout) with every
    entry's x' gather, no row structure — warm and cold (the cold one reads
    the 1.2 GB stream and the touched x' lines from HBM)."""
    from cant_single import probe_lib

    P = probe_lib()
    val = torch.from_numpy(np.ascontiguousarray(loc.val)).to(dev)
    col = torch.from_numpy(np.ascontiguousarray(loc.col)).to(dev)
    sink = torch.zeros(1 << 20, dtype=torch.float64, device=dev)
    npairs = loc.nnz // 2
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731

    def run():
        assert P.spmv_probe_gather_stream(val.data_ptr(), col.data_ptr(), npairs, x.data_ptr(), sink.data_ptr(),
                                          st()) == 0

    w = warm_fn_ms(torch, run, 20)
    c = cold_fn_ms(torch, run, 10)
    del val, col, sink
    torch.cuda.empty_cache()

    def frac(ms):
        return round(b_total / (ms * 1e-3) * 1e-9 / sa.HBM_PEAK_GBS, 4) if ms and ms > 0 else None

    return {"what": "spmv_probe_gather_stream (tools/probe.hip): the R-MAT's val/col streamed in entry order "
                    "(16-B value pairs, 8-B column pairs, non-temporal) with every entry's x' gather, no row "
                    "structure, no y: the access pattern's own time, the denominator of frac_of_gather_ceiling",
            "warm_ms": round(w, 5), "cold_ms": round(c, 5) if c else None,
            "frac_of_hbm_peak_warm": frac(w), "frac_of_hbm_peak_cold": frac(c)}


def rmat_per_format(args, torch, dev, loc, x, full, hot, b_total, ceiling):
    """BASELINE.json configs[3]: every format on the whole R-MAT (1e7 rows,
    1e8 entries) in bench's layout (rmat_layout: the relabelled, row-sorted
    CSR order; x' = x[order]), each through its C plan: warm (graph replay)
    and cold (flush span difference) ms, GB/s and fraction of the 8 TB/s
    HBM peak by bytes_alg, and the fraction of the gather ceiling (ceiling
    ms / format ms).  Every y is checked against the ORIGINAL matrix and x
    (host check_result rule).  ELL is N/A with its padding factor."""
    per = {}
    y = torch.empty(loc.n_rows, dtype=torch.float64, device=dev)
    x_orig = sa.ramp_x(loc.n_cols)
    lens = np.bincount(loc.row, minlength=loc.n_rows)
    for fmt in sa.ALL_FORMATS:
        t0 = time.perf_counter()
        if fmt == "ell":
            K = int(lens.max()) + (int(lens.max()) & 1)
            pad = (K * ((loc.n_rows + 63) // 64 * 64)) / max(loc.nnz, 1)
            per[fmt] = {"na": f"padding factor {pad:.0f} (K = {K} slots per row for a mean row of "
                              f"{loc.nnz / loc.n_rows:.1f}): refused above 64"}
            continue
        try:
            d2 = sa.to_device(loc, fmt, dev, **rmat_fmt_kwargs(args, fmt, hot))
        except sa.SpmvError as e:
            per[fmt] = {"na": str(e)}
            continue
        build_s = time.perf_counter() - t0
        wm = warm_fn_ms(torch, lambda: d2.run(x, y), 10)
        cm = cold_fn_ms(torch, lambda: d2.run(x, y), 5)
        bad, first = sa.check(full, x_orig, y.cpu().numpy())

        def gbs(ms):
            return round(b_total / (ms * 1e-3) * 1e-9, 1) if ms and ms > 0 else None

        rec = {"warm_ms": round(wm, 5), "cold_ms": round(cm, 5) if cm else None, "GBs_warm": gbs(wm),
               "GBs_cold": gbs(cm), "frac_warm": round(gbs(wm) / sa.HBM_PEAK_GBS, 4),
               "frac_cold": round(gbs(cm) / sa.HBM_PEAK_GBS, 4) if cm else None,
               "frac_of_gather_ceiling_warm": round(ceiling["warm_ms"] / wm, 4) if ceiling else None,
               "frac_of_gather_ceiling_cold": (round(ceiling["cold_ms"] / cm, 4)
                                               if ceiling and ceiling.get("cold_ms") and cm else None),
               "stored_MB": round(d2.stored_bytes * 1e-6, 1), "kernel": kernel_name(argparse.Namespace(
                   **dict(vars(args), format=fmt)), d2), "plan": d2.params.get("plan"),
               "parity_ok": bad == 0, "build_s": round(build_s, 1)}
        if bad:
            rec["first_bad_row"] = first
        stored = d2.stored_bytes + 8 * loc.n_cols + 8 * loc.n_rows
        if stored < b_total:
            rec["frac_cold_vs_stored"] = round(stored / (cm * 1e-3) * 1e-9 / sa.HBM_PEAK_GBS, 4) if cm else None
        if fmt == "csrf32":
            rec["parity"] = "within fp32-value tolerance (values rounded to fp32)"
        per[fmt] = rec
        del d2
        torch.cuda.empty_cache()
    return {"workload": "every format on the whole R-MAT 1e7 x 1e7 / 1e8 entries (configs[3]), bench's relabelled "
                        "layout, one GPU", "gather_ceiling": ceiling, "formats": per,
            "check": "each format's y against the ORIGINAL (un-relabelled) matrix and x[j] = j"}


def banded_strong(args, torch, dev, rank, world, dist, cdev):
    """BASELINE.json configs[4]: CSR and SELL-C-sigma on the banded
    --banded-rows x 16-entry matrix, equal 1024-aligned row ranges, each
    rank's shard generated in its HBM (spmv_gen_banded_device), x[j] = j
    replicated; aggregate GB/s = bytes_alg(whole matrix) / max over ranks of
    the per-step time (HIP-graph replay between barriers).  Every rank
    checks sampled rows across its whole shard (banded_check); then the
    exchange (strong_exchange): the y all-gather of the real shard sizes
    (800 MB of y in all), SpMV + all-gather, cold shards."""
    out = {}
    n = args.banded_rows
    comm = iterate.Comm(dist)
    for fmt in ("csr", "sell"):
        a = argparse.Namespace(**vars(args))
        a.workload, a.format, a.variant, a.lanes, a.ki, a.sigma = "banded", fmt, 0, 0, 0, 0
        t0 = time.perf_counter()
        w = build_workload(a, torch, dev, rank, world)
        torch.cuda.synchronize()  # the shard is generated on the device
        build_s = time.perf_counter() - t0
        steps = 20
        wall, kern = time_steps(torch, w["dm"], w["x"], w["y"], steps, 3, dist)
        bad = w["check"]()
        all_ok(dist, cdev, torch, bad is None, f"banded {fmt}: {bad}", rank)
        t = torch.tensor([wall / steps * 1e3, float(np.mean(kern))], dtype=torch.float64, device=cdev)
        if dist is not None:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        step_ms = float(t[0].item())
        tot = w["bytes_total"]

        def gbs(ms):
            return round(tot / (ms * 1e-3) * 1e-9, 1) if ms and ms > 0 else None

        rec = {"aggregate_GBs": gbs(step_ms),
               "GFLOPs": round(2 * w["nnz_total"] / (step_ms * 1e-3) * 1e-9, 1),
               "ms_per_step": round(step_ms, 5), "max_shard_kernel_ms": round(float(t[1].item()), 5),
               "rows_rank0": w["rows"], "bytes_alg_whole": tot, "parity_ok": True,
               "parity": f"{banded_sample_rows(n, w['lo'], w['hi']).size} rows of rank 0's shard (first/last 512, "
                         "around 2/4/8-way cuts, past 2^31..2^33 value bytes, 4096 spread) against the host "
                         "generator, x[j] = j; every rank checks its own",
               "build_s": round(build_s, 1)}
        w["y"] = None
        torch.cuda.empty_cache()
        y_full = torch.empty(n, dtype=torch.float64, device=dev)
        how, ag_ms, both_ms, cold = strong_exchange(torch, comm, cdev, w["dm"], w["x"], y_full, w["lo"], w["hi"],
                                                    w["bounds"], 10, args.flush == "yes")
        rec["allgather"] = {"how": how, "ms": round(ag_ms, 5),
                            "bytes_received_rank0": 8 * (n - w["rows"]) if rank == 0 else None,
                            "spmv_plus_allgather_ms": round(both_ms, 5),
                            "aggregate_GBs_with_allgather": gbs(both_ms)}
        if cold is not None:
            rec["cold"] = {"shard_ms": [round(v, 5) for v in cold], "max_shard_ms": round(max(cold), 5),
                           "aggregate_GBs": gbs(max(cold))}
        out[fmt] = rec
        del w, y_full
        torch.cuda.empty_cache()
    return {"workload": f"banded {args.banded_rows} rows x 16 entries (configs[4]), equal row shards over all "
                        "ranks, generated on device, x[j] = j replicated", "scaling": "strong", "steps": 20, **out}


def batch_leg(args, torch, dev, rank, world, dist, cdev):
    """The block-diagonal batch of `--copies` cant-like matrices per rank
    (rounds 1-3's headline): one launch per step streams 1.58 GB from HBM.
    Returns (the workload dict, per-step wall ms, kernel ms, roofline)."""
    a = argparse.Namespace(**vars(args))
    a.workload = "batch"
    w = build_workload(a, torch, dev, rank, world)
    wall, kern = time_steps(torch, w["dm"], w["x"], w["y"], args.steps, args.warmup, dist)
    bad = w["check"]()
    all_ok(dist, cdev, torch, bad is None, str(bad), rank)
    t = torch.tensor([wall, float(np.mean(kern))], dtype=torch.float64, device=cdev)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms_per_step = float(t[0].item()) / args.steps * 1e3
    kern_ms = float(t[1].item())
    achieved = w["bytes_rank"] / (kern_ms * 1e-3) * 1e-9
    kname = kernel_name(a, w["dm"])
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": sa.HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / sa.HBM_PEAK_GBS, 4), "traffic": traffic_for(a.format, w["bytes_rank"], kname),
            "kernel": kname, "kernel_ms": round(kern_ms, 5), "bytes_alg_per_launch": w["bytes_rank"]}
    return w, ms_per_step, kern_ms, roof


def per_format_leg(args, torch, dev, m, x, y, nnz, bytes_step, hot=None):
    """Every format on the same matrix (R-MAT: ELL is N/A, padding).  hot:
    the hot-column kwarg of a relabelled matrix (0: no per-run table)."""
    per_format = {}
    x_host = x.cpu().numpy()
    for fmt in sa.ALL_FORMATS:
        kw = fmt_kwargs(args, fmt)
        if hot is not None and fmt in ("coo", "csr", "csrf32", "cmrs", "sell", "hyb"):
            kw = dict(kw, hot=hot)
        try:
            d2 = sa.to_device(m, fmt, dev, **kw)
        except sa.SpmvError as e:
            per_format[fmt] = {"na": str(e)}
            continue
        _, k2 = time_steps(torch, d2, x, y, max(20, args.steps // 2), 5)
        km = float(np.mean(k2))
        # the output of every format is checked (host check_result rule,
        # 1e-6 relative); csrf32 rounds the values to fp32, so its check
        # shows fp32-value tolerance, not fp64 parity
        badf, _ = sa.check(m, x_host, y[:m.n_rows].cpu().numpy())
        per_format[fmt] = {"GBs": round(bytes_step / (km * 1e-3) * 1e-9, 1),
                           "GFLOPs": round(2 * nnz / (km * 1e-3) * 1e-9, 1),
                           "frac": round(bytes_step / (km * 1e-3) * 1e-9 / sa.HBM_PEAK_GBS, 4),
                           "kernel_ms": round(km, 5), "stored_MB": round(d2.stored_bytes * 1e-6, 1),
                           "params": dict(kw, **{k: v for k, v in d2.params.items()
                                                 if k in ("variant", "split_T", "n_chunks", "H")}) or None,
                           "parity_ok": badf == 0}
        # formats that store fewer bytes than bytes_alg credits (16-bit column
        # offsets, fp32 values): frac above is of the fp64/int32 bytes_alg and
        # can pass 1; frac_vs_stored prices the bytes they actually read
        stored = d2.stored_bytes + 8 * m.n_cols + 8 * m.n_rows
        if stored < bytes_step:
            per_format[fmt]["frac_vs_stored"] = round(stored / (km * 1e-3) * 1e-9 / sa.HBM_PEAK_GBS, 4)
            per_format[fmt]["frac_note"] = (f"frac is of bytes_alg ({bytes_step} B); this format stores "
                                            f"{stored} B with x and y: frac_vs_stored is the HBM figure")
        if fmt == "csrf32":
            per_format[fmt]["parity"] = "within fp32-value tolerance (values rounded to fp32)"
        del d2
        torch.cuda.empty_cache()
    return per_format


def main():
    args = parse()
    if args.workload == "cantlike":
        args.workload = "batch"
    if launch.needs_spawn(args.gpus):
        # `--gpus N` from a plain process: N ranks in a child
        # torch.distributed.run job; this process never touches the GPU
        sys.exit(launch.spawn_ranks(__file__, args.gpus))
    GRAPH["on"] = args.graph == "yes"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    # the single-matrix kernel trace comes from a profiled CHILD process,
    # run before this process initialises the GPU (every format at N=1; the
    # headline format on every rank's own GPU at N>1)
    prof = None
    if not args.profile and args.workload == "cant" and args.single != "no":
        if world == 1:
            prof = cant_single_rocprof(flush_mode=args.cold_flush)
        else:
            prof = cant_single_rocprof([args.format], 0 if args.share_gpu else local, args.cold_flush)
    elif rank == 0 and not args.profile and args.single == "yes" and world == 1:
        prof = cant_single_rocprof(flush_mode=args.cold_flush)

    import torch

    dist = None
    gpu = 0 if args.share_gpu else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    # collectives run on the GPU over RCCL (backend "nccl" on ROCm); the
    # gloo backend (CPU tensors) exists only to rehearse N>1 on one GPU
    cdev = dev if args.backend == "nccl" else torch.device("cpu")
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    if args.profile:  # only the timed loop, for rocprofv3 --pmc passes
        if args.workload == "cant":
            s = single_cold(args, torch, dev, rank, world, dist, cdev, None)
            ms = s["timed_region"]["cold_spmv_ms_in_process"]
        else:
            w = build_workload(args, torch, dev, rank, world)
            _, kern = time_steps(torch, w["dm"], w["x"], w["y"], args.steps, args.warmup, dist)
            ms = float(np.mean(kern))
        if rank == 0:
            print(json.dumps({"profile_run": args.format, "workload": args.workload, "ms_per_launch": ms}))
        return

    batch = per_format = cpu = allgather = sell_single = None
    if args.workload == "cant":
        s = single_cold(args, torch, dev, rank, world, dist, cdev, prof)
        if args.sell_single != "no" and args.format != "sell":
            # BASELINE.json configs[2] (the north star's >= 60 % target) by the
            # headline's own in-process method, its trace beside it
            sv = single_cold(args, torch, dev, rank, world, dist, cdev, prof, fmt="sell")
            sg = sv["bytes"] / (sv["cold_ms"] * 1e-3) * 1e-9
            sell_single = {"workload": "SELL-C-sigma (C = 64, sigma = 1024) on ONE cant-like matrix, cold "
                                       "(BASELINE.json configs[2])",
                           "value_GBs": round(sg, 1), "frac": round(sg / sa.HBM_PEAK_GBS, 4),
                           "ms": round(sv["cold_ms"], 5), "kernels": sv["kernels"], "params": sv["params"],
                           "source": sv["source"], "trace": sv["trace"], "timed_region": sv["timed_region"],
                           "parity_ok": sv["parity_ok"]}
            tr = (sv["trace"] or {}).get("kernel_ms_median")
            if tr:
                # the north star's own measure: "rocprof-reported achieved HBM GB/s
                # against the chip's HBM3E peak" (BASELINE.json north_star, target >= 0.60)
                sell_single["frac_rocprof"] = round(sv["bytes"] / (tr * 1e-3) * 1e-9 / sa.HBM_PEAK_GBS, 4)
                sell_single["north_star_target"] = ("SELL-C-sigma >= 0.60 of HBM3E peak on cant, 1 GPU, "
                                                    "rocprof-reported (frac_rocprof: median of 50 cold launches "
                                                    "in the kernel trace); frac is the in-process figure, which "
                                                    "also carries the graph node's launch gap "
                                                    "(timed_region.empty_kernel_node_ms)")
        ms_per_step = s["cold_ms"]
        bytes_step, total_bytes = s["bytes"], s["bytes"] * world
        value = total_bytes / (ms_per_step * 1e-3) * 1e-9
        gflops = 2.0 * s["nnz"] * world / (ms_per_step * 1e-3) * 1e-9
        kname = s["kernels"][0]
        roofline = {"bound": "hbm", "achieved": round(bytes_step / (ms_per_step * 1e-3) * 1e-9, 1),
                    "peak": sa.HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(bytes_step / (ms_per_step * 1e-3) * 1e-9 / sa.HBM_PEAK_GBS, 4),
                    "traffic": traffic_for(args.format, bytes_step, kname, cold=True),
                    "kernel": kname, "kernels": s["kernels"], "kernel_ms": round(ms_per_step, 5),
                    "kernel_ms_source": s["source"], "kernel_ms_trace": s["trace"],
                    "bytes_alg_per_launch": bytes_step,
                    "state": "cold: 512 MiB flush before every launch"}
        scaling, n_rows, nnz = "weak", s["rows"], s["nnz"]
        data = ("synthetic: cant-like stand-in (62,451 rows, 4,007,383 entries = SuiteSparse cant's counts; the "
                "reference's cant.mtx is an unfetched Git-LFS pointer), x[j] = j")
        config = {"workload": f"{args.format} SpMV on ONE cant-like matrix per GPU (BASELINE.json "
                              + ("configs[2]" if args.format == "sell" else "configs[1]")
                              + "), cold: 512 MiB flush before every step; N GPUs run N replicas, no collective",
                  "timed_region": s["timed_region"], "kernel_params": s["params"],
                  "ms_per_step_is": "the SpMV's share of one step (the step's 512 MiB flush excluded; the "
                                    "wall clock per step with it is timed_region.wall_ms_per_step_incl_flush)"}
        if world > 1:
            config["value_is"] = ("replica throughput: N independent copies of configs[1], one per GPU, no "
                                  "exchange (weak scaling); the strong-scaling evidence is rmat_strong."
                                  "speedup_cold / speedup_warm")
        launch_desc = s["timed_region"]["what"]
        do_batch = args.batch == "yes" or (args.batch == "auto" and world == 1)
        if do_batch:
            w, b_ms, b_kern, b_roof = batch_leg(args, torch, dev, rank, world, dist, cdev)
            batch = {"workload": w["config"]["workload"], "copies_per_gpu": args.copies,
                     "value_GBs": round(w["bytes_total"] / (b_ms * 1e-3) * 1e-9, 1), "ms_per_step": round(b_ms, 5),
                     "launch": "hip-graph replay (K launches, span / K)" if GRAPH.get("last") == "hip-graph"
                               else "eager", "roofline": b_roof, "parity_ok": True}
            if rank == 0 and world == 1 and args.per_format != "no":
                dm = w.pop("dm")
                del dm
                torch.cuda.empty_cache()
                batch["per_format"] = per_format_leg(args, torch, dev, w["m"], w["x"], w["y"], w["nnz"],
                                                     w["bytes_rank"])
            del w
            torch.cuda.empty_cache()
        if rank == 0 and world == 1 and args.cpu_seconds > 0:
            # cold, like the GPU headline (2/3 of the budget), and warm beside it
            sm = sa.gen_cantlike(0, 1)
            ptr, col, val = sa.csr_from_coo(sm)
            arrs = (ptr, col, val, sm.n_rows, sm.n_cols)
            cpu = cpu_baseline(arrs, 1, args.cpu_seconds * 2 / 3, cold=True)
            warm = cpu_baseline(arrs, 1, args.cpu_seconds / 3)
            for c in (cpu, warm):
                c["sample"] = c["sample"].replace("the same 1-copy batch", "the same single cant-like matrix")
            cpu["warm"] = {k: warm[k] for k in ("value", "unit", "cores", "sample", "gflops")}
    else:
        w = build_workload(args, torch, dev, rank, world)
        dm, x, y = w["dm"], w["x"], w["y"]
        n_rows, nnz, bytes_step = w["rows"], w["nnz"], w["bytes_rank"]
        wall, kern = time_steps(torch, dm, x, y, args.steps, args.warmup, dist)
        launch_desc = (f"hip-graph: the K launches captured once, replayed untimed for >= {WARM_REPLAY_MS:g} ms of "
                       "GPU work, then once timed; kernel_ms = span / K"
                       if GRAPH.get("last") == "hip-graph" else "eager launches, one HIP event after each")
        bad = w["check"]()
        all_ok(dist, cdev, torch, bad is None, str(bad), rank)
        wall_t = torch.tensor([wall], dtype=torch.float64, device=cdev)
        kern_t = torch.tensor([float(np.mean(kern))], dtype=torch.float64, device=cdev)
        if dist is not None:
            dist.all_reduce(wall_t, op=dist.ReduceOp.MAX)
            dist.all_reduce(kern_t, op=dist.ReduceOp.MAX)
        ms_per_step = float(wall_t.item()) / args.steps * 1e3
        total_bytes = w["bytes_total"]
        value = total_bytes / (ms_per_step * 1e-3) * 1e-9
        gflops = 2.0 * w["nnz_total"] / (ms_per_step * 1e-3) * 1e-9
        scaling, data, config = w["scaling"], w["data"], dict(w["config"])

        # weak-scaling batch: the y blocks (all the same size) all-gathered
        # over RCCL, timed separately, not in `value`
        if dist is not None and args.workload == "batch":
            y_loc = y if cdev.type == "cuda" else y.cpu()
            y_all = torch.empty(n_rows * world, dtype=torch.float64, device=cdev)
            for _ in range(3):
                dist.all_gather_into_tensor(y_all, y_loc)
            torch.cuda.synchronize()
            ok = bool(torch.equal(y_all[rank * n_rows:(rank + 1) * n_rows], y_loc))
            all_ok(dist, cdev, torch, ok, "all-gathered y block", rank)
            dist.barrier()
            t0 = time.perf_counter()
            reps = 20
            for _ in range(reps):
                dist.all_gather_into_tensor(y_all, y_loc)
            torch.cuda.synchronize()
            ag = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64, device=cdev)
            dist.all_reduce(ag, op=dist.ReduceOp.MAX)
            ag_ms = float(ag.item()) * 1e3
            allgather = {"ms": round(ag_ms, 4), "bytes_per_rank": 8 * n_rows, "backend": args.backend,
                         "value_with_allgather_GBs": round(total_bytes / ((ms_per_step + ag_ms) * 1e-3) * 1e-9, 1)}

        kern_ms = float(kern_t.item())
        achieved = bytes_step / (kern_ms * 1e-3) * 1e-9
        kname = kernel_name(args, dm)
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": sa.HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / sa.HBM_PEAK_GBS, 4),
                    "traffic": traffic_for(args.format, bytes_step, kname),
                    "kernel": kname, "kernel_ms": round(kern_ms, 5), "bytes_alg_per_launch": bytes_step}

        do_pf = rank == 0 and (args.per_format == "yes" or (args.per_format == "auto" and world == 1))
        if do_pf and args.workload in ("rmat", "batch"):
            m = w["loc"] if args.workload == "rmat" else w["m"]
            del dm, w["dm"]
            torch.cuda.empty_cache()
            per_format = per_format_leg(args, torch, dev, m, x, y, nnz, bytes_step, w.get("hot"))
            if args.cpu_seconds > 0:
                if args.workload == "rmat":
                    ptr, col, val = sa.csr_from_coo(m)
                    cpu = cpu_baseline((ptr, col, val, m.n_rows, m.n_cols), 1, args.cpu_seconds)
                    cpu["sample"] = cpu["sample"].replace("the same 1-copy batch", "the same R-MAT")
                else:
                    sm = sa.gen_cantlike(0, 1)
                    ptr, col, val = sa.csr_from_coo(sm)
                    cpu = cpu_baseline((ptr, col, val, sm.n_rows, sm.n_cols), args.copies, args.cpu_seconds)
        w.pop("dm", None)
        dm = None
        torch.cuda.empty_cache()

    rstrong = None
    default_wl = args.workload in ("cant", "batch")
    if args.rmat_strong == "yes" or (args.rmat_strong == "auto" and default_wl):
        torch.cuda.empty_cache()
        rstrong = rmat_strong(args, torch, dev, rank, world, dist, cdev)
    bstrong = None
    if args.banded_strong == "yes" or (args.banded_strong == "auto" and default_wl):
        bstrong = banded_strong(args, torch, dev, rank, world, dist, cdev)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": data,
            "config": dict(config, format=args.format, params=fmt_kwargs(args, args.format) or None,
                           rows_rank0=n_rows, nnz_rank0=nnz, bytes_alg_rank0_step=bytes_step,
                           bytes_alg_all_ranks_step=total_bytes, parallelism=f"row-shard x{world}"
                           if args.workload in ("rmat", "banded") else f"replicas x{world}",
                           launch=launch_desc),
            "gflops": round(gflops, 1),
            "roofline": roofline,
            "cpu_baseline": cpu,
            "sell_single": sell_single,
            "rmat_per_format": rstrong.pop("per_format", None) if rstrong else None,
            "cant_single": prof if world == 1 else ({"rank0": prof} if prof else None),
            "batch": batch,
            "per_format": per_format,
            "allgather": allgather,
            "rmat_strong": rstrong,
            "strong_scaling": ({"rmat_speedup_cold": rstrong.get("speedup_cold"),
                                "rmat_speedup_warm": rstrong.get("speedup_warm"),
                                "n_gpus": world, "layout": rstrong.get("layout")} if rstrong else None),
            "banded_strong": bstrong,
            "device": sa.device_name(gpu),
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
