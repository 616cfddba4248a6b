"""The C-ABI libraries load on a CPU-only host and export every function
that include/*.h declares (no compute calls without a GPU)."""
from __future__ import annotations

import ctypes
import re
import subprocess

import pytest

import spmv_amd as sa
from conftest import REPO

HEADERS = {"spmv.h": "libspmv_hip.so", "spmv_ext.h": "libspmv_hip.so", "spmv_host.h": "libspmv_host.so"}


def declared(header: str) -> set[str]:
    text = (REPO / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(spmv_[a-z0-9_]+)\s*\(", text)) - {"spmv_launch_fn"}


@pytest.mark.parametrize("header,lib", HEADERS.items())
def test_exports_every_declared_symbol(header, lib):
    names = declared(header)
    assert len(names) > 5
    so = ctypes.CDLL(str(sa.LIB_DIR / lib))
    missing = [n for n in sorted(names) if not hasattr(so, n)]
    assert not missing, f"{lib} lacks {missing}"
    # and they are C symbols (no C++ mangling)
    out = subprocess.run(["nm", "-D", "--defined-only", str(sa.LIB_DIR / lib)], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert names <= exported


def test_python_binding_covers_headers():
    assert declared("spmv.h") <= set(sa.HIP_SYMBOLS)
    assert declared("spmv_ext.h") <= set(sa.HIP_SYMBOLS)
    assert declared("spmv_host.h") <= set(sa.HOST_SYMBOLS)
    sa.hip_lib()  # binds every symbol; raises if one is missing
    sa.host_lib()


def test_no_device_is_reported_not_faked():
    """Without a GPU the library reports a device error — it never falls back."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    n = ctypes.c_int(-1)
    rc = sa.hip_lib().spmv_device_count(ctypes.byref(n))
    assert rc == sa.DEVICE_ERROR and n.value == 0
    assert sa.hip_lib().spmv_strerror(1) == b"device error"


def test_return_codes_match_reference_enum():
    text = (REPO / "include" / "spmv_rc.h").read_text()
    vals = dict(re.findall(r"(SPMV_[A-Z_]+)\s*=\s*(\d)", text))
    # reference inc/enums.h:4-11: Success, OpenCLDeviceError, OpenCLProgramError, FileError, OtherError
    assert vals == {"SPMV_SUCCESS": "0", "SPMV_DEVICE_ERROR": "1", "SPMV_PROGRAM_ERROR": "2",
                    "SPMV_FILE_ERROR": "3", "SPMV_OTHER_ERROR": "4"}


def test_gfx950_code_object_present(tmp_path):
    import shutil

    so = tmp_path / "libspmv_hip.so"  # objdump extracts bundles next to its input
    shutil.copy(sa.LIB_DIR / "libspmv_hip.so", so)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(so)],
                         capture_output=True, text=True, cwd=tmp_path)
    text = out.stdout + out.stderr
    if "unknown argument" in text or out.returncode != 0:
        data = (sa.LIB_DIR / "libspmv_hip.so").read_bytes()
        assert b"gfx950" in data
    else:
        assert "gfx950" in text


def test_drivers_exit_codes_without_gpu(tmp_path):
    """./bin/<fmt> on a GPU-less host exits with the reference's
    OpenCLDeviceError code (1), like get_device_ids failing (csr.c:25-28)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    for prog in ("coo", "csr", "ell", "sigma_c", "cmrs"):
        exe = REPO / "bin" / prog
        if not exe.exists():
            subprocess.run(["make", "-C", str(REPO), prog], check=True, capture_output=True)
        r = subprocess.run([str(exe)], cwd=tmp_path, capture_output=True, text=True)
        assert r.returncode == 1, (prog, r.stdout, r.stderr)


def test_plan_opts_defaults_and_options():
    """spmv_plan_opts_init: every switch at "the library's rule" (-1), lanes
    0 (rule), no SELL16; the A/B switches are set and read through the C-ABI
    (no environment reads on the launch path) and refuse unknown values."""
    o = sa.plan_opts()
    assert (o.variant, o.xwin, o.head, o.coo_pass, o.split, o.bigplan, o.H) == (-1,) * 7
    assert (o.lanes, o.index16, o.xwin_rows) == (0, 0, 0)
    lib = sa.hip_lib()
    for name in sa.OPTIONS:
        old = sa.get_option(name)
        for v in (0, 1, None):
            sa.set_option(name, v)
            assert sa.get_option(name) == (-1 if v is None else v)
        sa.set_option(name, old)
    assert lib.spmv_set_option(99, 0) == sa.OTHER_ERROR and lib.spmv_get_option(99) == -2
    assert lib.spmv_set_option(1, 2) == sa.OTHER_ERROR


def test_plan_without_gpu_is_a_device_error():
    """Creating a plan without a GPU reports the reference's device error
    (1) and returns no plan; it never falls back to the CPU."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = sa.hip_lib()
    ptr = (ctypes.c_int64 * 3)(0, 1, 2)
    d = sa.Dims(2, 2, 2, 0, None)
    plan = ctypes.c_void_p()
    o = sa.plan_opts()
    rc = lib.spmv_plan_csr(d, ctypes.addressof(ptr), ctypes.addressof(ptr), ctypes.addressof(ptr), ctypes.byref(o),
                           ctypes.byref(plan))
    assert rc == sa.DEVICE_ERROR and not plan.value
    assert lib.spmv_plan_csr(d, None, None, None, ctypes.byref(o), ctypes.byref(plan)) == sa.OTHER_ERROR
    assert lib.spmv_plan_run(None, None, None, None) == sa.OTHER_ERROR
    assert lib.spmv_plan_destroy(None) == sa.SUCCESS
