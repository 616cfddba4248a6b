"""The five drop-in programs ./bin/{coo,csr,ell,sigma_c,cmrs} on a GPU.

Each reads a Matrix Market file (the reference's only input path, reference
csr.c:43-91), prints the reference's lines (reference
inc/helper_functions.h:167-182, coo.c:201, ell.c:104, csr.c:229-255) and
checks its own result against the file-order sum; the parity verdict is
read from the output and double-checked with the oracle by re-running the
same file through the C-ABI in tests/test_gpu_parity.py.
"""
from __future__ import annotations

import re
import shutil
import subprocess

import pytest

from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu

PROGS = ["coo", "csr", "ell", "sigma_c", "cmrs"]


def run(prog, *args, cwd=None, timeout=300):
    exe = REPO / "bin" / prog
    if not exe.exists():
        subprocess.run(["make", "-C", str(REPO), prog], check=True, capture_output=True)
    return subprocess.run([str(exe), *args], cwd=cwd, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("prog", PROGS)
@pytest.mark.parametrize("case", ["ragged_shuffled", "empty_rows", "n67", "long_rows", "colmajor"])
def test_program_on_fixture(prog, case):
    r = run(prog, "--matrix", str(GOLDEN / f"{case}.mtx"), "--reps", "3", "--warmup", "1", "--strict",
            "--cpu")
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout
    assert re.search(r"^Your calculations took [0-9.]+ ms to run\.$", out, re.M)
    assert re.search(r"^Number of operations \d+, PERFORMANCE [0-9.]+ GFlops$", out, re.M)
    assert re.search(r"^GBytes transferred to processor [0-9.]+ - [0-9.]+, speed [0-9.]+ - [0-9.]+ GB/s$", out, re.M)
    assert "\nresult is ok\n" in "\n" + out
    assert "\ncpu result is ok\n" in out
    if prog == "coo":
        assert out.startswith("GPU calculations\n")
    if prog == "ell":
        assert out.startswith("average column length ")


def test_default_paths_and_file_error(tmp_path):
    """No arguments: the reference's default paths; missing file -> exit 3."""
    for prog in PROGS:
        r = run(prog, cwd=tmp_path)
        assert r.returncode == 3, (prog, r.stdout, r.stderr)
    # with databases/ present the programs read them (cant-like stand-in here)
    db = tmp_path / "databases"
    db.mkdir()
    shutil.copy(GOLDEN / "colmajor.mtx", db / "cant.mtx")
    shutil.copy(GOLDEN / "ragged_shuffled.mtx", db / "cant-sorted.mtx")
    for prog in PROGS:
        r = run(prog, "--reps", "2", cwd=tmp_path)
        assert r.returncode == 0 and "result is ok" in r.stdout, (prog, r.stdout, r.stderr)


def test_generated_cantlike_and_roundtrip(tmp_path):
    """--gen cantlike --write-mtx, then the written file read back."""
    path = tmp_path / "cantlike.mtx"
    r = run("csr", "--gen", "cantlike", "--write-mtx", str(path), "--reps", "5", "--strict")
    assert r.returncode == 0 and "result is ok" in r.stdout, r.stdout
    for prog in ("sigma_c", "ell", "cmrs"):
        r = run(prog, "--matrix", str(path), "--reps", "5", "--strict")
        assert r.returncode == 0 and "result is ok" in r.stdout, (prog, r.stdout)
    assert "Number of operations 8014766," in r.stdout  # 2 * 4,007,383


def test_bad_option_exit_code():
    r = run("csr", "--no-such-option")
    assert r.returncode == 4


@pytest.mark.parametrize("prog", ["csr", "sigma_c"])
def test_binary_cache(tmp_path, prog):
    """--cache writes PATH.bin on the first run and reads it on the next;
    the verdict is the same, and a newer text file invalidates it."""
    src = tmp_path / "m.mtx"
    shutil.copy(GOLDEN / "ragged_shuffled.mtx", src)
    args = ("--matrix", str(src), "--reps", "2", "--warmup", "0", "--strict", "--cache")
    r1 = run(prog, *args)
    assert r1.returncode == 0, r1.stdout + r1.stderr
    assert "[cache] wrote" in r1.stdout and (tmp_path / "m.mtx.bin").exists()
    r2 = run(prog, *args)
    assert r2.returncode == 0, r2.stdout + r2.stderr
    assert "[cache] read" in r2.stdout and "\nresult is ok\n" in "\n" + r2.stdout
    # a newer text file is parsed again
    import os
    st = (tmp_path / "m.mtx.bin").stat()
    os.utime(src, (st.st_atime + 10, st.st_mtime + 10))
    r3 = run(prog, *args)
    assert "[cache] wrote" in r3.stdout, r3.stdout


@pytest.mark.parametrize("prog", ["csr", "ell", "sigma_c"])
def test_xwin_and_global_paths_agree(prog):
    """Default (x window in LDS) and --no-xwin both pass the check."""
    for extra in ([], ["--no-xwin"]):
        r = run(prog, "--gen", "cantlike", "--copies", "2", "--reps", "3", "--warmup", "1", "--strict",
                "--no-cpu", *extra)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "\nresult is ok\n" in "\n" + r.stdout


@pytest.mark.parametrize("prog", ["csr", "sigma_c", "coo", "cmrs", "ell"])
def test_program_gpus_flag_rccl_path(prog):
    """--gpus 1: the single-process multi-GPU path (RCCL communicator over
    the devices, row shards, y completed by grouped RCCL broadcasts of the
    real shard sizes) on the box's one GPU; the check is the same."""
    r = run(prog, "--gen", "cantlike", "--gpus", "1", "--reps", "3", "--warmup", "1", "--strict", "--cpu")
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout
    assert re.search(r"^Your calculations took [0-9.]+ ms to run\.$", out, re.M)
    assert "\nresult is ok\n" in "\n" + out and "\ncpu result is ok\n" in out
    assert "[multi] y identical on all 1 GPUs: yes" in out
    assert re.search(r"\[multi\] y all-gather over RCCL .*: [0-9.]+ ms; SpMV \+ all-gather [0-9.]+ ms", out)


def test_program_gpus_flag_more_gpus_than_present():
    """Asking for more GPUs than the node has is the reference's device error (1)."""
    r = run("csr", "--gen", "cantlike", "--gpus", "64", "--reps", "1")
    assert r.returncode == 1, r.stdout + r.stderr


def test_sigma_c_index16():
    """./bin/sigma_c --index16: SELL16 (16-bit column offsets, head copy on a
    small matrix) through the C-ABI, checked like every run; refused for the
    other programs (the C-ABI refusal of wide windows:
    test_gpu_parity.test_sell16_refuses_wide_windows)."""
    r = run("sigma_c", "--gen", "cantlike", "--reps", "5", "--warmup", "1", "--strict", "--index16")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "kernel sell_small_kernel: SELL16" in r.stdout and "16-bit column offsets" in r.stdout
    assert "head copy" in r.stdout
    assert "\nresult is ok\n" in "\n" + r.stdout
    r = run("sigma_c", "--matrix", str(GOLDEN / "ragged_shuffled.mtx"), "--reps", "3", "--strict", "--index16")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "\nresult is ok\n" in "\n" + r.stdout
    r = run("csr", "--gen", "cantlike", "--index16")
    assert r.returncode == 4


def test_coo_single_pass_flag():
    """./bin/coo: the carry-free COO where rows allow (the cant-like matrix),
    the carry pass where one row is too long or with --carry-pass; all checked."""
    r = run("coo", "--gen", "cantlike", "--reps", "5", "--warmup", "1", "--strict")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "COO single pass: no carry kernel" in r.stderr
    assert "\nresult is ok\n" in "\n" + r.stdout
    r = run("coo", "--gen", "cantlike", "--reps", "5", "--warmup", "1", "--strict", "--carry-pass")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "COO single pass: off" in r.stderr and "\nresult is ok\n" in "\n" + r.stdout
    r = run("coo", "--matrix", str(GOLDEN / "long_rows.mtx"), "--reps", "2", "--warmup", "1", "--strict")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "COO single pass: refused" in r.stderr


def test_csr_program_big_tiles(tmp_path):
    """./bin/csr on a matrix whose rows run in long empty stretches (the
    tiled CSR path, tiles owning thousands of rows: the big-tile plan) —
    the reference's lines and a passing check."""
    import numpy as np

    import spmv_amd as sa

    rng = np.random.default_rng(11)
    n, nc = 400_000, 50_000
    rows = np.sort(rng.choice(np.arange(1, n - 5000), 4000, replace=False))
    lens = rng.integers(2, 20, rows.size)
    lens[rows.size // 2] = 20_000
    r = np.repeat(rows, lens).astype(np.int32)
    m = sa.Coo(n, nc, r, rng.integers(0, nc, r.size).astype(np.int32), rng.uniform(-1, 1, r.size))
    f = tmp_path / "big_tiles.mtx"
    sa.write_mtx(f, m)
    res = run("csr", "--matrix", str(f), "--reps", "3", "--warmup", "1", "--strict", "--cpu")
    assert res.returncode == 0, res.stdout + res.stderr
    assert "\nresult is ok\n" in "\n" + res.stdout


@pytest.mark.parametrize("prog,fmt", [("sigma_c", "sell"), ("csr", "csr"), ("coo", "coo"), ("cmrs", "cmrs"),
                                      ("ell", "ell")])
def test_program_runs_the_binding_plan(tmp_path, prog, fmt):
    """./bin/<fmt> and spmv_amd.to_device build the same C plan (spmv_plan_<fmt>,
    include/spmv.h) for the cant-like matrix (configs[1]/[2]): the program's
    "[plan]" line names the kernel and path the binding reports, and its y
    (--write-y) is bit-identical to the binding's on x[j] = j — the program
    runs what bench.py measures."""
    import numpy as np
    import torch

    import spmv_amd as sa

    yf = tmp_path / "y.bin"
    r = run(prog, "--gen", "cantlike", "--reps", "5", "--warmup", "1", "--strict", "--no-cpu", "--write-y", str(yf))
    assert r.returncode == 0, r.stdout + r.stderr
    got = re.search(r"^  \[plan\] kernel (\S+): (.*)$", r.stdout, re.M)
    assert got, r.stdout
    m = sa.gen_cantlike(1 if prog == "coo" else 0)  # the programs' --gen cantlike entry order
    dm = sa.to_device(m, fmt, "cuda:0")
    x = torch.from_numpy(sa.ramp_x(m.n_cols)).to("cuda:0")
    y = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device="cuda:0")
    dm.run(x, y)
    torch.cuda.synchronize()
    assert got.group(1) == dm.kernel and got.group(2) == dm.params["plan"], (got.groups(), dm.params)
    y_prog = np.fromfile(yf, dtype=np.float64)
    assert y_prog.size == m.n_rows
    assert np.array_equal(y.cpu().numpy().view(np.int64), y_prog.view(np.int64))
    if fmt == "sell":  # configs[2]: the small-matrix kernel with its head copy
        assert dm.kernel == "sell_small_kernel" and dm.params["head"] == 1


def test_csr_relabel_skewed_rows():
    """./bin/csr on an R-MAT (1e6 rows, 1e7 entries): --relabel auto (default)
    takes bench.py's configs[3] layout — degree-relabelled columns, rows in
    new-column order, x permuted on the host — and the plan's tiled kernel;
    the check is against the ORIGINAL matrix and x, for the GPU and the CPU
    loop; --relabel no and the one-process --gpus 1 path agree."""
    gen = "rmat:1000000:10000000"
    r = run("csr", "--gen", gen, "--reps", "3", "--warmup", "1", "--strict", "--cpu")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "[relabel]" in r.stdout and "kernel csr_tiled_kernel" in r.stdout, r.stdout
    assert "\nresult is ok\n" in "\n" + r.stdout and "\ncpu result is ok\n" in r.stdout
    r = run("csr", "--gen", gen, "--reps", "3", "--warmup", "1", "--strict", "--no-cpu", "--relabel", "no")
    assert r.returncode == 0 and "[relabel]" not in r.stdout and "\nresult is ok\n" in "\n" + r.stdout, r.stdout
    r = run("csr", "--gen", gen, "--reps", "3", "--warmup", "1", "--strict", "--cpu", "--gpus", "1")
    assert r.returncode == 0 and "[relabel]" in r.stdout, r.stdout + r.stderr
    assert "\nresult is ok\n" in "\n" + r.stdout and "\ncpu result is ok\n" in r.stdout
    for prog in ("coo", "sigma_c", "cmrs"):  # every format on the relabelled layout
        r = run(prog, "--gen", gen, "--reps", "2", "--warmup", "1", "--strict", "--no-cpu")
        assert r.returncode == 0 and "[relabel]" in r.stdout and "\nresult is ok\n" in "\n" + r.stdout, (prog, r.stdout)
    r = run("csr", "--gen", "cantlike", "--reps", "2", "--strict", "--relabel", "yes")  # forced on a FEM matrix
    assert r.returncode == 0 and "[relabel]" in r.stdout and "\nresult is ok\n" in "\n" + r.stdout, r.stdout
