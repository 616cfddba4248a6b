"""`--gpus N` without a launcher (opencl-spmv-algorithms_amd/launch.py):
the parent spawns torch.distributed.run as a child, forwards its output and
exit code, and never touches the GPU.  CPU only (gloo-free: the ranks here
only print their environment)."""
from __future__ import annotations

import os
import re
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "opencl-spmv-algorithms_amd"))
import launch  # noqa: E402


def test_needs_spawn_rules():
    assert launch.needs_spawn(8, {})
    assert not launch.needs_spawn(1, {})
    assert not launch.needs_spawn(8, {"WORLD_SIZE": "8"})  # already a rank of a launcher
    assert not launch.needs_spawn(8, {launch.SPAWNED_ENV: "1"})  # never spawn twice


def test_spawn_command_and_env():
    cmd = launch.spawn_command("/r/bench.py", 4, ["--gpus", "4", "--steps", "7"], 29555, python="py")
    assert cmd == ["py", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
                   "--master-addr=127.0.0.1", "--master-port=29555", "/r/bench.py", "--gpus", "4", "--steps", "7"]
    env = launch.spawn_env({"PATH": "/bin"})
    assert env[launch.SPAWNED_ENV] == "1" and env["PATH"] == "/bin"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert launch.spawn_env({"HSA_ENABLE_IPC_MODE_LEGACY": "0"})["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    p = launch.free_port()
    assert 0 < p < 65536


SCRIPT = textwrap.dedent('''
    import os, sys
    sys.path.insert(0, {pkg!r})
    import launch
    n = int(sys.argv[1])
    if launch.needs_spawn(n):
        sys.exit(launch.spawn_ranks(__file__, n))
    r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.write(1, f"rank {{r}} of {{w}} local {{os.environ['LOCAL_RANK']}}\\n".encode())  # one write per line
    sys.exit(3 if (len(sys.argv) > 2 and r == 1) else 0)
''')


def _script(tmp_path):
    f = tmp_path / "ranks.py"
    f.write_text(SCRIPT.format(pkg=str(REPO / "opencl-spmv-algorithms_amd")))
    return f


def _clean_env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            launch.SPAWNED_ENV)}
    env["OMP_NUM_THREADS"] = "1"
    return env


def test_spawn_runs_n_ranks(tmp_path):
    r = subprocess.run([sys.executable, str(_script(tmp_path)), "3"], capture_output=True, text=True,
                       timeout=240, env=_clean_env())
    assert r.returncode == 0, r.stderr[-2000:]
    # (ranks share the pipe: match each record wherever a line break fell)
    lines = sorted(re.findall(r"rank \d+ of \d+ local \d+", r.stdout))
    assert lines == ["rank 0 of 3 local 0", "rank 1 of 3 local 1", "rank 2 of 3 local 2"]
    assert "[launch] --gpus 3" in r.stderr


def test_spawn_forwards_rank_failure(tmp_path):
    r = subprocess.run([sys.executable, str(_script(tmp_path)), "2", "fail"], capture_output=True, text=True,
                       timeout=240, env=_clean_env())
    assert r.returncode != 0
    assert "failed: exit" in r.stderr


@pytest.mark.parametrize("script,extra", [("bench.py", ["--single", "no"]), ("tools/iterate_bench.py", [])])
def test_bench_scripts_spawn_without_launcher(script, extra):
    """`python3 <script> --gpus 2` from a plain process starts two ranks in a
    child torch.distributed.run (here, with no GPU, the ranks fail at device
    setup and the parent must exit non-zero instead of measuring one rank)."""
    r = subprocess.run([sys.executable, str(REPO / script), "--gpus", "2", "--backend", "gloo", *extra],
                       capture_output=True, text=True, timeout=300, env=_clean_env(), cwd=str(REPO))
    assert "[launch] --gpus 2 without a launcher" in r.stderr, r.stderr[-2000:]
    assert "--nproc-per-node=2" in r.stderr
    assert r.returncode != 0
