"""Shared pytest setup.

Markers:
  gpu  — needs an MI355X; the parity tests proper (HIP path vs oracle).
Everything else runs on a CPU-only host: oracle vs golden fixtures, host
reader/builders/CPU loops, C-ABI symbol exports, gloo multi-process logic.
"""
from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "opencl-spmv-algorithms_amd"
GOLDEN = REPO / "tests" / "golden"
for p in (str(PKG), str(REPO)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X GPU (HIP path parity)")


def _ensure_built():
    libs = [PKG / "lib" / "libspmv_hip.so", PKG / "lib" / "libspmv_host.so", REPO / "oracle" / "liboracle.so"]
    if not all(p.exists() for p in libs):
        subprocess.run(["make", "-C", str(REPO), "-j8", "lib", "oracle"], check=True)


_ensure_built()


def golden_cases():
    return json.loads((GOLDEN / "manifest.json").read_text())


@pytest.fixture(scope="session")
def golden():
    return golden_cases()
