#!/usr/bin/env python3
"""Where a streaming SpMV kernel waits: TA / TD / TCP / TCC / SQ counters.

Runs `bench.py --profile` (and the bandwidth probe's non-temporal tile read
as the reference point) under separate `rocprofv3 --pmc` passes — never
combined with tracing — and prints, per kernel, each counter's mean per
dispatch plus the counters that are cycle counts as a fraction of
GRBM_GUI_ACTIVE (per XCD).  Written to gpurun_out/pmc_stalls.json.
    python tools/pmc_stalls.py [--formats csr,sell,ell]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))
from pmc_traffic import kernel_for, mean_per_dispatch, run_pass  # noqa: E402

PASSES = {
    "ta": ["TA_BUSY_avr", "GRBM_GUI_ACTIVE"],
    "ta2": ["TA_ADDR_STALLED_BY_TC_CYCLES_sum"],
    "ta3": ["TA_DATA_STALLED_BY_TC_CYCLES_sum"],
    "tcp": ["TCP_PENDING_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum", "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum",
            "TCP_TCC_READ_REQ_sum"],
    "td": ["TD_TD_BUSY_sum", "TD_TC_STALL_sum", "TD_SPI_STALL_sum", "TCP_TOTAL_CACHE_ACCESSES_sum"],
    "sq": ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VMEM"],
    "sq2": ["SQ_INSTS_VMEM_RD", "SQ_INST_CYCLES_VMEM_RD", "SQ_WAIT_ANY", "SQ_INSTS_LDS"],
    "tcc": ["TCC_EA0_RDREQ_DRAM_sum", "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "TCC_TAG_STALL_sum", "TCC_BUSY_avr"],
    "lat": ["TCP_TCC_READ_REQ_LATENCY_sum", "TA_FLAT_READ_WAVEFRONTS_sum", "TA_TOTAL_WAVEFRONTS_sum",
            "SQ_WAVES"],
    "lds": ["SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS"],
    "inst": ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY",
             "SQ_WAVES"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--formats", default="csr,sell,ell")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--passes", default="", help="comma list of pass names (default all)")
    ap.add_argument("--out", default="pmc_stalls.json")
    ap.add_argument("--workload", default="batch", choices=["batch", "cant"],
                    help="bench.py workload: the 32-copy batch, or ONE cant-like matrix cold")
    ap.add_argument("--no-probe", action="store_true", help="skip the bandwidth-probe reference passes")
    a = ap.parse_args()
    passes = {k: v for k, v in PASSES.items() if not a.passes or k in a.passes.split(",")}
    probe = REPO / "tools" / "bw_probe"
    jobs = [] if a.no_probe else [
        ("probe_tile_nt", [str(probe), str(2 << 30), "3"], "tile_read_kernel<true, 8>", {}),
        # the CSR access pattern without the LDS work (values + columns, R = 4)
        ("probe_csr_stream", [str(probe), str(2 << 30), "3"], "csr_stream_kernel<4>", {})]
    for spec in a.formats.split(","):
        spec_main, *env_parts = spec.split("@")
        env_kv = dict(e.split("=", 1) for e in env_parts)
        fmt = spec_main.partition(":")[0]
        cmd = ["python3", "bench.py", "--profile", "--format", fmt, "--steps", str(a.steps), "--warmup", "2",
               "--workload", a.workload]
        jobs.append((spec, cmd, kernel_for(fmt, env_kv, a.workload), env_kv))
    out = {}
    for name, cmd, kern, env_kv in jobs:
        counters = {}
        saved = {k: os.environ.get(k) for k in env_kv}
        os.environ.update(env_kv)  # run_pass hands os.environ to the profiled command
        for tag, cs in passes.items():
            tagdir = f"stall_{name}_{tag}".replace(":", "_").replace("=", "").replace("@", "_")
            f = run_pass(tagdir, cs, cmd, timeout=150)
            if f:
                c, _ = mean_per_dispatch(f, kern)
                counters.update(c)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        gui = counters.get("GRBM_GUI_ACTIVE")
        frac = {}
        if gui:
            for k, v in counters.items():
                if "CYCLES" in k or "STALL" in k or "BUSY" in k:
                    frac[k] = round(v / gui, 4)
        out[name] = {"kernel": kern, "counters": {k: round(v, 1) for k, v in counters.items()},
                     "per_gui_active": frac}
        print(json.dumps({name: out[name]}), flush=True)
    (REPO / "gpurun_out" / a.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
