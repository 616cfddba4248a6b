"""bench.py on a GPU: the driver's contract line, and `--gpus N` from a
plain process (no launcher) running N ranks (launch.spawn_ranks).

Two ranks share cuda:0 over gloo here (the rehearsal form); the driver's
multi-GPU run uses one GPU per rank over RCCL.  The legs that take minutes
(R-MAT / banded strong scaling, the 32-copy batch, the rocprofv3 child)
are switched off: the line, the timed region and the per-rank figures are
what is checked.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

QUICK = ["--steps", "5", "--warmup", "2", "--rmat-strong", "no", "--banded-strong", "no", "--batch", "no",
         "--single", "no", "--cpu-seconds", "0"]


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "SPMV_SPAWNED_RANKS")}
    env["OMP_NUM_THREADS"] = "4"
    return env


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


def test_bench_one_gpu_line():
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), *QUICK], capture_output=True, text=True,
                       timeout=600, env=_env(), cwd=str(REPO))
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and d["unit"] == "GB/s" and d["dtype"] == "f64" and d["scaling"] == "weak"
    assert "ONE cant-like matrix" in d["config"]["workload"]
    assert d["roofline"]["bound"] == "hbm" and 0 < d["roofline"]["frac"] < 1.2
    tr = d["config"]["timed_region"]
    assert d["ms_per_step"] * d["steps"] <= tr["wall_ms"]  # the SpMV share of the timed region
    expect = d["config"]["bytes_alg_all_ranks_step"] / (d["ms_per_step"] * 1e-3) * 1e-9
    assert abs(d["value"] - expect) <= 0.005 * expect  # ms_per_step is printed rounded to 10 ns


def test_bench_gpus_2_without_launcher():
    """`python3 bench.py --gpus 2` (the driver's form) measures TWO ranks, and
    the line carries its own strong-scaling evidence: rank 0 times the whole
    R-MAT alone in the same job, so rmat_strong has speedup_cold /
    speedup_warm (a 1e6 / 1e7 R-MAT here, one re-cut)."""
    args = [a for a in QUICK]
    i = args.index("--rmat-strong")
    args[i + 1] = "yes"
    args += ["--rmat-rows", "1000000", "--rmat-nnz", "10000000", "--recuts", "1"]
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--backend", "gloo", "--share-gpu",
                        *args], capture_output=True, text=True, timeout=900, env=_env(), cwd=str(REPO))
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2
    assert len(d["config"]["timed_region"]["cold_ms_per_rank"]) == 2
    assert d["config"]["bytes_alg_all_ranks_step"] == 2 * d["config"]["bytes_alg_rank0_step"]
    assert "replica throughput" in d["config"]["value_is"]
    rs = d["rmat_strong"]
    assert rs["whole_matrix_one_gpu"]["how"].startswith("rank 0 alone")
    assert rs["speedup_warm"] > 0 and rs["speedup_cold"] > 0
    assert d["strong_scaling"]["rmat_speedup_cold"] == rs["speedup_cold"]
    assert "relabelled" in rs["layout"]
    assert "[launch] --gpus 2 without a launcher" in r.stderr
