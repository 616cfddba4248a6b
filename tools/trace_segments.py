"""Cut a rocprofv3 kernel trace into the phases that tools/cant_single.py
marks with spmv_probe_tag dispatches (tools/probe.hip: a tag of id k is an
empty grid of k + 1 workgroups), and time each SpMV from the trace.

A cold phase is [flush, SpMV kernels, flush, SpMV kernels, ...]: one rep is
the kernels between two probe_flush_kernel dispatches, timed from the first
one's start to the last one's end (gaps between a format's kernels count).
A warm phase is the SpMV kernels back to back: its dispatches are cut into
runs of equal kernel count.  Durations are the trace's own GPU timestamps,
not host-paired events.
"""
from __future__ import annotations

import csv
from collections import defaultdict

TAG = "probe_tag_kernel"
FLUSH = "probe_flush"  # probe_flush_kernel (write) or probe_flush_read_kernel


def _dispatches(path):
    rows = []
    for r in csv.DictReader(open(path, newline="")):
        gx, wx = int(r["Grid_Size_X"]), max(int(r.get("Workgroup_Size_X") or 1), 1)
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], gx // wx))
    rows.sort()
    return rows


def segments(path):
    """{tag id: [(start_ns, end_ns, kernel name), ...]} in dispatch order."""
    seg = defaultdict(list)
    cur = None
    for s, e, name, groups in _dispatches(path):
        if TAG in name:
            cur = groups - 1
            continue
        if cur is not None:
            seg[cur].append((s, e, name))
    return dict(seg)


def cold_ms(disp):
    """Per-rep span (ms) of the kernels between consecutive flushes."""
    reps, cur = [], []
    for s, e, name in disp + [(0, 0, FLUSH)]:
        if FLUSH in name:
            if cur:
                reps.append((max(x[1] for x in cur) - min(x[0] for x in cur)) * 1e-6)
            cur = []
        else:
            cur.append((s, e))
    return reps


def warm_ms(disp, runs):
    """Per-run span (ms) of `runs` back-to-back runs of equal kernel count."""
    if runs <= 0 or not disp or len(disp) % runs:
        return []
    k = len(disp) // runs
    return [(disp[i + k - 1][1] - disp[i][0]) * 1e-6 for i in range(0, len(disp), k)]


def kernel_names(disp):
    names = []
    for _, _, name in disp:
        short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        if FLUSH not in name and short not in names:
            names.append(short)
    return names
