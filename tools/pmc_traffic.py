#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 PMC counters (GPU box only).

Follows MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7:
  * every counter group is collected in its OWN rocprofv3 pass, with
    --pmc only (no tracing domains), on `python3 bench.py --profile`;
  * FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts 128-B
    requests at 64 B (reads ~1/2 of a wide stream), so reads are priced
    from TCC_EA0_RDREQ_{32B,64B,128B} and CALIBRATED on tools/bw_probe,
    whose bytes per launch are known (2 GiB read);
  * the result (per format: HBM bytes per launch of the dominant kernel)
    goes to profiles/traffic.json, which bench.py reports as
    roofline.traffic when its workload (bytes_alg) matches.
    python tools/pmc_traffic.py [--formats csr,sell,ell,coo,cmrs] [--copies 32]
    python tools/pmc_traffic.py --workload cant --formats csr --out traffic_single.json
  (--workload cant: ONE cant-like matrix, COLD — bench.py's headline step,
  a 512 MiB flush before every launch — written for bench.py's cold
  roofline.traffic)
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
OUT = REPO / "gpurun_out" / "pmc"
KERNELS = {"csr": "csr_xwin_kernel", "sell": "sell_xwin_kernel", "ell": "ell_xwin_kernel",
           "coo": "coo_staged_kernel", "cmrs": "cmrs_staged_kernel", "csr16": "Col16"}
# one cant-like matrix: the small-matrix kernels
KERNELS_SINGLE = dict(KERNELS, sell="sell_small_kernel", sell16="sell_small_kernel")


def kernel_for(fmt, env, workload="batch"):
    """The dominant kernel's name (substring) for `fmt` under `env`."""
    del env  # placement / cache-policy knobs do not change the kernel
    return (KERNELS_SINGLE if workload == "cant" else KERNELS)[fmt]
PASSES = {
    "fetch": ["FETCH_SIZE"],
    "write": ["WRITE_SIZE"],
    "rdreq": ["TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_sum"],
    "l2": ["TCC_HIT_sum", "TCC_MISS_sum", "TA_BUSY_avr", "GRBM_GUI_ACTIVE"],
}
CANT_N, CANT_Z = 62451, 4007383


def run_pass(tag, counters, cmd, timeout=600):
    d = OUT / tag
    d.mkdir(parents=True, exist_ok=True)
    full = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", str(d), "-o", "run", "--", *cmd]
    env = dict(os.environ, TMPDIR="/tmp")
    print(f"pass {tag}: {' '.join(counters)}", flush=True)
    try:
        r = subprocess.run(full, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired as e:
        (d / "stdout.log").write_text(f"timed out after {timeout} s\n{e.stdout or ''}\n--- stderr ---\n{e.stderr or ''}")
        print(f"pass {tag} timed out after {timeout} s", file=sys.stderr, flush=True)
        return None
    (d / "stdout.log").write_text(r.stdout[-20000:] + "\n--- stderr ---\n" + r.stderr[-20000:])
    if r.returncode != 0:
        print(f"pass {tag} failed rc={r.returncode}", file=sys.stderr, flush=True)
        return None
    files = list(d.rglob("*counter_collection.csv"))
    if not files:
        print(f"pass {tag}: no counter_collection.csv", file=sys.stderr, flush=True)
        return None
    return files[0]


def mean_per_dispatch(path, kernel_substr):
    """{counter: mean value per dispatch} over dispatches of the kernel."""
    per = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel_substr not in row.get("Kernel_Name", ""):
                continue
            key = (row.get("Dispatch_Id"), row["Counter_Name"])
            per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
    sums, counts = {}, {}
    for (_, name), v in per.items():
        sums[name] = sums.get(name, 0.0) + v
        counts[name] = counts.get(name, 0) + 1
    return {k: sums[k] / counts[k] for k in sums}, max(counts.values()) if counts else 0


def bytes_from_rdreq(c):
    n32 = c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
    n64 = c.get("TCC_EA0_RDREQ_64B_sum", 0.0)
    n128 = c.get("TCC_EA0_RDREQ_128B_sum", 0.0)
    return 32 * n32 + 64 * n64 + 128 * n128


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--formats", default="csr,sell,ell,coo,cmrs")
    ap.add_argument("--copies", type=int, default=32)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--out", default=None, help="file name under profiles/ (default traffic.json)")
    ap.add_argument("--workload", default="batch", choices=["batch", "cantlike", "cant", "rmat"])
    ap.add_argument("--kernel", default=None, help="kernel name substring (default: the format's)")
    a = ap.parse_args()
    if a.workload == "cantlike":
        a.workload = "batch"
    probe = REPO / "tools" / "bw_probe"
    if not probe.exists():
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", str(REPO / "tools" / "bw_probe.hip"), "-o",
                        str(probe)], check=True)
    # ---- calibration on known bytes: read_kernel<double2,4> reads 2 GiB
    cal = {}
    for tag in ("fetch", "rdreq"):
        f = run_pass(f"probe_{tag}", PASSES[tag], [str(probe), str(2 << 30), "5"])
        if f:
            c, _ = mean_per_dispatch(f, "read_kernel<HIP_vector_type<double, 2u>")
            if not c:
                c, _ = mean_per_dispatch(f, "read_kernel")
            cal.update(c)
    known = float(2 << 30)
    cal_fetch = cal.get("FETCH_SIZE", 0.0) * 1024 / known if cal.get("FETCH_SIZE") else None
    cal_rdreq = bytes_from_rdreq(cal) / known if cal.get("TCC_EA0_RDREQ_sum") else None
    result = {"_calibration": {"probe": "tools/bw_probe read_dwordx4 of 2 GiB",
                               "FETCH_SIZE_bytes_over_known": cal_fetch,
                               "RDREQ_sized_bytes_over_known": cal_rdreq, "raw": cal}}
    print(json.dumps(result["_calibration"]), flush=True)

    for spec in a.formats.split(","):
        # spec: fmt[:key=val;key=val][@ENV=val]  e.g. sell:sigma=256  csr@SPMV_XCD_REMAP=1
        spec_main, *env_parts = spec.split("@")
        env_kv = dict(e.split("=", 1) for e in env_parts)
        fmt, _, params = spec_main.partition(":")
        cmd = ["python3", "bench.py", "--profile", "--format", fmt, "--steps", str(a.steps), "--warmup", "2",
               "--copies", str(a.copies), "--workload", a.workload]
        for kv in filter(None, params.split(";")):
            k, v = kv.split("=")
            cmd += [f"--{k}", v]
        os.environ.update(env_kv)
        tag0 = spec.replace(":", "_").replace(";", "_").replace("=", "").replace("@", "_")
        counters, n = {}, 0
        for tag, cs in PASSES.items():
            f = run_pass(f"{tag0}_{tag}", cs, cmd)
            if f:
                c, n = mean_per_dispatch(f, a.kernel or kernel_for(fmt, env_kv, a.workload))
                counters.update(c)
        if not counters:
            continue
        N, Z = {"batch": (CANT_N * a.copies, CANT_Z * a.copies), "cant": (CANT_N, CANT_Z)}.get(a.workload,
                                                                                               (10**7, 10**8))
        b_alg = 12 * Z + 4 * (N + 1) + 8 * N + 8 * N
        read_rdreq = bytes_from_rdreq(counters)
        if cal_rdreq and 0.8 < cal_rdreq < 1.25:
            read = read_rdreq / cal_rdreq
            how = "sized TCC_EA0_RDREQ (32/64/128 B) / probe calibration"
        elif cal_fetch:
            read = counters.get("FETCH_SIZE", 0.0) * 1024 / cal_fetch
            how = "FETCH_SIZE*1024 / probe calibration"
        else:
            read = counters.get("FETCH_SIZE", 0.0) * 1024 * 2
            how = "FETCH_SIZE*1024*2 (guide's gfx950 correction, uncalibrated)"
        write = counters.get("WRITE_SIZE", 0.0) * 1024
        hits, miss = counters.get("TCC_HIT_sum", 0.0), counters.get("TCC_MISS_sum", 0.0)
        for k in env_kv:
            os.environ.pop(k, None)
        result[spec] = {"kernel": a.kernel or kernel_for(fmt, env_kv, a.workload), "workload": a.workload,
                        "state": "cold: 512 MiB flush before every launch" if a.workload == "cant" else "streamed", "bytes_alg": b_alg, "dispatches": n, "cmd": " ".join(cmd[1:]),
                        "env": env_kv or None,
                       "hbm_read_bytes_per_launch": round(read), "hbm_write_bytes_per_launch": round(write),
                       "hbm_bytes_per_launch": round(read + write),
                       "traffic_over_alg": round((read + write) / b_alg, 4), "method": how,
                       "l2_hit_rate": round(hits / (hits + miss), 4) if hits + miss else None,
                       "counters": {k: round(v, 1) for k, v in counters.items()}}
        print(json.dumps({spec: result[spec]}), flush=True)
    dst = REPO / "profiles" / ("traffic.json" if a.out is None else a.out)
    dst.write_text(json.dumps(result, indent=1) + "\n")
    # only gpurun_out/ travels back from the GPU box
    (REPO / "gpurun_out" / dst.name).write_text(json.dumps(result, indent=1) + "\n")
    print(f"wrote {dst}")


if __name__ == "__main__":
    main()
