#!/usr/bin/env python3
"""Per-format rocprofv3 summary of a default bench.py run (all formats on
the cant batch, then one copy cold/warm): for every SpMV kernel, the
dispatches of its LARGEST grid (the 32-copy batch; single-copy launches
have smaller grids) with their mean duration, and the algorithmic GB/s
that duration gives against the 8 TB/s HBM3E peak.

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fmt -o run -- \\
        python3 bench.py --steps 50 --rmat-strong no --cpu-seconds 0
    python tools/rocprof_formats.py gpurun_out/prof_fmt/run_kernel_trace.csv > profiles/round2/rocprof_formats.md
"""
from __future__ import annotations

import csv
import sys
from collections import defaultdict

BYTES_ALG = 1_578_803_716  # bench.py's 32-copy cant-like batch, bytes_alg per launch
PEAK = 8000.0


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    by = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if "spmv::" not in name or "window" in name or "carry" in name or "flush" in name:
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        by[name].append((grid, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3))
    print("| kernel (template arguments as rocprofv3 names them) | grid | dispatches | mean µs | GB/s (alg) | % of 8 TB/s |")
    print("|---|---|---|---|---|---|")
    out = []
    for name, v in by.items():
        g = max(x[0] for x in v)
        d = [t for gg, t in v if gg == g]
        mean = sum(d) / len(d)
        gbs = BYTES_ALG / (mean * 1e-6) * 1e-9
        out.append((mean, name, g, len(d), gbs))
    # HYB runs two kernels per SpMV: the ELL part (ell_kernel, no x window)
    # and the COO tail in accumulate mode (coo_staged_kernel<4, R, true, ...>)
    hyb = [o for o in out if "ell_kernel<" in o[1] and "xwin" not in o[1]
           or "coo_staged_kernel<4, 3, true" in o[1]]
    for mean, name, g, n, gbs in sorted(o for o in out if o not in hyb):
        short = name.split("(")[0].replace("void ", "")
        print(f"| `{short}` | {g} | {n} | {mean:.1f} | {gbs:,.0f} | {100 * gbs / PEAK:.1f} % |")
    if len(hyb) == 2:
        mean = sum(o[0] for o in hyb)
        gbs = BYTES_ALG / (mean * 1e-6) * 1e-9
        parts = " + ".join(f"`{o[1].split('(')[0].replace('void ', '')}` {o[0]:.1f}" for o in sorted(hyb))
        print(f"| HYB: {parts} | | {hyb[0][3]} | {mean:.1f} | {gbs:,.0f} | {100 * gbs / PEAK:.1f} % |")


if __name__ == "__main__":
    main()
