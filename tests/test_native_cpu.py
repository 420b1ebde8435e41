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


def test_vr_two_limb_quantisation_bound():
    """k_rs_vr's two-limb weights (fi_plan.cpp vr_quant / quant_axis): every
    table of the BASELINE geometries and 200 random ones is rebuilt from its
    fragment bytes, its integer algebra re-derived (row sums 2^shift, the
    constant 128 * 2^shift bias, the Q16 hi/lo split), and the worst case over
    all 8-bit inputs of |kernel - ImageMagick f64| bounded per output: < 1 LSB
    (tests/native/vr_quant_bound.cpp).  The f64 weights the bound is taken
    against are checked first to be the oracle's own (or_im_axis_taps, bit for
    bit on every output of every geometry), so the bound chains to the
    oracle and not only to the planner's restatement."""
    import re

    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "vqb")
        # the oracle's tap restatement (or_im_axis_taps), with the oracle's own flags
        obj = os.path.join(d, "fi_oracle.o")
        subprocess.run(["gcc", "-O2", "-std=c99", "-D_GNU_SOURCE", "-ffp-contract=off", "-fno-fast-math", "-c",
                        os.path.join(ROOT, "oracle/fi_oracle.c"), "-o", obj], check=True, capture_output=True,
                       timeout=300)
        subprocess.run([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests/native/vr_quant_bound.cpp"),
                        os.path.join(ROOT, "flyimg_amd/csrc/fi_plan.cpp"), "-Xlinker", obj, "-o", exe, "-lm"],
                       check=True, capture_output=True, timeout=300)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK (0 failures)" in r.stdout
    worst = float(re.search(r"worst bound ([0-9.]+) LSB", r.stdout).group(1))
    # the bound is against the oracle's weights: the planner's tables equal them bit for bit
    m = re.search(r"planner tap tables == oracle's: (\d+) weights of (\d+) geometries", r.stdout)
    assert m and int(m.group(1)) > 100000 and int(m.group(2)) >= 100, r.stdout
    assert worst < 1.0
    for cfg in ("cfg1", "cfg2", "cfg3", "cfg5"):
        assert re.search(cfg + r" .*bound ([0-9.]+) LSB", r.stdout), cfg


@pytest.mark.parametrize("src,kernels", [
    ("fi_vr.hip", ["_ZN2fi7k_rs_vrILi0ELi2EE", "_ZN2fi7k_rs_vrILi0ELi4EE"]),
    ("fi_smartcrop.hip", ["_ZN2fi11k_sc_score2ILi1EE", "_ZN2fi11k_sc_score3E", ("_ZN2fi7k_sc_fdE", 12),
                          # k_sc_hx / k_sc_vx: the gray forms (cfg5's default) and the RGB two-k-step ones
                          "_ZN2fi7k_sc_hxILi2ELi1EE", "_ZN2fi7k_sc_vxILi2ELi1EE", "_ZN2fi7k_sc_hxILi1ELi1EE",
                          "_ZN2fi7k_sc_vxILi1ELi1EE", "_ZN2fi7k_sc_hxILi2ELi3EE", "_ZN2fi7k_sc_vxILi2ELi3EE",
                          "_ZN2fi7k_sc_hxILi1ELi3EE"]),
])
def test_hot_kernels_do_not_spill(src, kernels):
    """The production kernels of the hot path keep every value in registers: a
    VGPR spill (scratch) cost a 1.6x slowdown of k_rs_vr once (round 4).
    k_sc_fd spills 12 SGPRs into VGPR lanes (no scratch) outside its loops;
    the entry (name, n) caps that count so growth is caught."""
    import re

    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                            "-I", os.path.join(ROOT, "include"), "-c", os.path.join(ROOT, "flyimg_amd/csrc", src),
                            "-o", os.path.join(d, "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
    text = r.stderr
    for k in kernels:
        k, smax = k if isinstance(k, tuple) else (k, 0)
        i = text.find("Function Name: " + k)
        assert i >= 0, k
        block = text[i:i + 2000]
        scratch = int(re.search(r"ScratchSize \[bytes/lane\]: (\d+)", block).group(1))
        sspill = int(re.search(r"SGPRs Spill: (\d+)", block).group(1))
        vspill = int(re.search(r"VGPRs Spill: (\d+)", block).group(1))
        assert scratch == 0 and vspill == 0 and sspill <= smax, (k, scratch, vspill, sspill)


def test_vr_pair_class_list_layout():
    """k_rs_vr's pair-class copies of an uneven row list for 2 and 4 loader
    waves (fi_internal.h vr_pair_off): distinct slots inside each copy, a
    wave's own pairs at consecutive entries (tests/native/vr_pair_list_check.cpp)."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "vpl")
        subprocess.run([hipcc, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                        "-I", os.path.join(ROOT, "flyimg_amd/csrc"),
                        os.path.join(ROOT, "tests/native/vr_pair_list_check.cpp"), "-o", exe],
                       check=True, capture_output=True, timeout=300)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK (0 failures)" in r.stdout
