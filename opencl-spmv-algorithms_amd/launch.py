"""launch — `--gpus N` without a launcher: run the same script as N ranks.

The driver (and a user) may start `python3 bench.py --gpus 8` as a plain
process.  Without `torch.distributed.run` that process sees no WORLD_SIZE
and would measure one GPU.  `spawn_ranks` makes such a process a parent
only: it starts `python -m torch.distributed.run --nproc-per-node N
<script> <same args>` as a CHILD process, lets the ranks write straight to
the inherited stdout / stderr (rank 0 prints the JSON line), waits, and
returns the child's exit code (torch.distributed.run exits non-zero when
any rank fails).

The parent never imports torch, never touches the GPU and never exec()s:
it spawns and waits (a process that initialised HIP must not replace
itself on this pool, and there is no reason to).  The reference has no
multi-GPU path at all: its context spans every device but only device 0
is used (reference csr.c:107,115) and its device loop breaks after the
first device (csr.c:30,279).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys

# set in every rank's environment by spawn_ranks; a rank never spawns again
SPAWNED_ENV = "SPMV_SPAWNED_RANKS"


def needs_spawn(gpus: int, env=None) -> bool:
    """True when `--gpus N` (N > 1) was asked for and this process is not
    already a rank of a torch.distributed.run job."""
    env = os.environ if env is None else env
    return gpus > 1 and "WORLD_SIZE" not in env and SPAWNED_ENV not in env


def free_port() -> int:
    """An unused TCP port on 127.0.0.1 for the rendezvous."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def spawn_command(script: str, gpus: int, argv: list[str], port: int, python: str | None = None) -> list[str]:
    """The child command line: torch.distributed.run, one node, `gpus`
    ranks, rendezvous on 127.0.0.1 (the container hostname may not
    resolve), then the script with the caller's own arguments unchanged."""
    return [python or sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
            script, *argv]


def spawn_env(env=None) -> dict:
    """The child environment: the parent's, plus the marker that stops a
    rank from spawning again; HSA_ENABLE_IPC_MODE_LEGACY=0 kept (RCCL over
    dmabuf IPC needs it on this pool)."""
    e = dict(os.environ if env is None else env)
    e[SPAWNED_ENV] = "1"
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return e


def spawn_ranks(script: str, gpus: int, argv: list[str] | None = None, timeout: float | None = None) -> int:
    """Run `script argv` as `gpus` ranks under torch.distributed.run in a
    child process; return its exit code (non-zero if any rank failed)."""
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = spawn_command(os.path.abspath(script), gpus, argv, free_port())
    print(f"[launch] --gpus {gpus} without a launcher: running {gpus} ranks: {' '.join(cmd)}",
          file=sys.stderr, flush=True)
    try:
        r = subprocess.run(cmd, env=spawn_env(), timeout=timeout)
    except subprocess.TimeoutExpired:
        print(f"[launch] {gpus}-rank job timed out after {timeout} s", file=sys.stderr, flush=True)
        return 124
    if r.returncode != 0:
        print(f"[launch] {gpus}-rank job failed: exit {r.returncode}", file=sys.stderr, flush=True)
    return 128 - r.returncode if r.returncode < 0 else r.returncode  # killed by signal s: 128 + s
