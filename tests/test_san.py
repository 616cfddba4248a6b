"""Host sanitizers: the host library's builders, reader,
CPU loops and partitioners compiled with ASan + UBSan and driven over the
fixtures, malformed files and the generators (tests/san/host_harness.c).
`make test-san` also runs the host/oracle pytest suites and the five
programs under the sanitizers; this CPU test runs the harness alone."""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc with libasan")
def test_host_harness_under_asan_ubsan(tmp_path):
    subprocess.run(["make", "-C", str(REPO), "build/san/host_harness"], check=True, capture_output=True)
    fixtures = sorted(str(p) for p in (REPO / "tests" / "golden").glob("*.mtx"))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:exitcode=99",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=99", OMP_NUM_THREADS="4")
    r = subprocess.run([str(REPO / "build" / "san" / "host_harness"), str(tmp_path), *fixtures], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "host_harness: ok" in r.stdout
