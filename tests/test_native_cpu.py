"""Host-side native checks (CPU): the exact-integer MFMA tables built by
flyimg_amd/csrc/fi_plan.cpp reproduce sum(quant(w) * p) through the kernels'
integer algebra (tests/native/mfma_tables_check.cpp, compiled host-only)."""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_mfma_tables_exact():
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "mtc")
        subprocess.run([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests/native/mfma_tables_check.cpp"),
                        os.path.join(ROOT, "flyimg_amd/csrc/fi_plan.cpp"), "-o", exe],
                       check=True, capture_output=True, timeout=300)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "OK (0 failures)" in r.stdout
