"""Host planner (flyimg_amd/csrc/fi_plan.cpp) and CPU oracle (oracle/fi_oracle.c)
under AddressSanitizer + UndefinedBehaviorSanitizer (the CPU
restatement under ASan/UBSan).  Host-only builds; any out-of-bounds access,
leak-free double free, signed overflow or other UB aborts the driver.

Inputs: the reference's 68 ImageProcessorTest geometry cases
(tests/golden/im_geometry_cases.json), the golden smartcrop shapes, and edge
geometries (1x1, tiny extents, extreme aspect ratios, rotations, gray,
monochrome, RGBA, convolutions) -- tests/native/plan_driver.cpp and
tests/native/oracle_driver.c."""
import json
import os
import shutil
import subprocess
import tempfile

import pytest

from flyimg_amd import _lib as L
from flyimg_amd.processor import ExecFailedException, ImageProcessor, OptionsBag

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _plan_lines():
    lines = []
    with open(os.path.join(ROOT, "tests/golden/im_geometry_cases.json")) as f:
        cases = json.load(f)
    for c in cases:
        C = 4 if c.get("mode") == "RGBA" else 3
        try:
            op = ImageProcessor(OptionsBag(c["options"]), c["src_w"], c["src_h"]).to_op()
        except ExecFailedException:
            continue
        lines.append((c["src_w"], c["src_h"], C, op.target_w, op.target_h, op.flags, op.gravity, op.rotate, 0, 0))
    with open(os.path.join(ROOT, "tests/golden/smartcrop_golden.json")) as f:
        sc = json.load(f)
    for c in sc["cases"]:
        lines.append((c["w"], c["h"], 3, 0, 0, L.FI_OP_THUMBNAIL | L.FI_OP_SMARTCROP, 5, 0, 100, 100))
    T, F, S, E, G, R = (L.FI_OP_THUMBNAIL, L.FI_GEOM_FILL, L.FI_GEOM_SHRINK_ONLY, L.FI_OP_EXTENT, L.FI_OP_GRAY,
                        L.FI_OP_ROTATE)
    edge = [
        (1, 1, 3, 1, 1, T, 5, 0), (2, 1, 3, 1, 1, T | F | E, 5, 0), (1, 5000, 3, 1, 0, T, 5, 0),
        (5000, 1, 3, 0, 1, T, 5, 0), (6000, 4000, 3, 400, 400, T | F | E | G | R, 5, 90),
        (3840, 2160, 3, 512, 512, T | F | E, 1, 0), (1920, 1080, 3, 500, 0, T | S, 5, 0),
        (120, 90, 3, 4000, 0, T, 5, 0), (640, 481, 3, 317, 0, L.FI_OP_RESIZE | S, 5, 0),
        (900, 600, 4, 250, 300, L.FI_OP_RESIZE | F | E | R, 9, 270), (800, 600, 3, 200, 0, T | L.FI_OP_MONOCHROME, 5, 0),
        (333, 222, 3, 200, 0, T | S | R | L.FI_SRC_PSEUDOCLASS, 5, 180), (16, 16, 3, 16, 16, T, 5, 0),
        (5657, 4243, 3, 300, 250, T | F | E, 5, 0), (530, 942, 3, 0, 300, T, 5, 0),
    ]
    for e in edge:
        lines.append(e + (0, 0))
        lines.append(e[:5] + (e[5] | L.FI_OP_SMARTCROP,) + e[6:] + (100, 56))
    return lines


def _compiler(name):
    path = shutil.which(name) or os.path.join("/opt/rocm/bin", name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not available")
    return path


def test_planner_under_asan_ubsan():
    hipcc = _compiler("hipcc")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "plan_driver")
        subprocess.run([hipcc, "-std=c++17", "-ffp-contract=off", "-fno-gpu-sanitize", *SAN, "-I",
                        os.path.join(ROOT, "include"), os.path.join(ROOT, "tests/native/plan_driver.cpp"),
                        os.path.join(ROOT, "flyimg_amd/csrc/fi_plan.cpp"), "-o", exe],
                       check=True, capture_output=True, timeout=300)
        lines = _plan_lines()
        stdin = "".join(" ".join(str(int(v)) for v in ln) + "\n" for ln in lines)
        r = subprocess.run([exe], input=stdin, capture_output=True, text=True, timeout=300, env=ENV)
        assert r.returncode == 0, r.stderr[-4000:]
        assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
        assert f"DONE {len(lines)} images" in r.stdout
        assert len(lines) > 68 + 15


def test_oracle_under_asan_ubsan():
    gcc = _compiler("gcc")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "oracle_driver")
        subprocess.run([gcc, "-std=c99", "-D_GNU_SOURCE", "-ffp-contract=off", *SAN,
                        os.path.join(ROOT, "tests/native/oracle_driver.c"), "-o", exe, "-lm"],
                       check=True, capture_output=True, timeout=300)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=ENV)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
        assert "0 unexpected errors" in r.stdout


def _jpeg_inputs(d):
    """Small JPEGs of every layout the GPU decoder's parser accepts, plus the
    progressive smart_crop.jpg fixture (rejected as unsupported)."""
    import io

    import numpy as np
    from PIL import Image
    rng = np.random.default_rng(5)
    px = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    cases = [("s420.jpg", dict(quality=90, subsampling=2)),
             ("s444r.jpg", dict(quality=75, subsampling=0, restart_marker_blocks=2)),
             ("s422o.jpg", dict(quality=95, subsampling=1, optimize=True))]
    paths = []
    for name, kw in cases:
        b = io.BytesIO()
        Image.fromarray(px).save(b, "JPEG", **kw)
        paths.append(os.path.join(d, name))
        open(paths[-1], "wb").write(b.getvalue())
    b = io.BytesIO()
    Image.fromarray(px[..., 0]).save(b, "JPEG", quality=80)
    paths.append(os.path.join(d, "gray.jpg"))
    open(paths[-1], "wb").write(b.getvalue())
    paths.append(os.path.join(ROOT, "tests/golden/smart_crop.jpg"))
    return paths


def test_jpeg_parser_under_asan_ubsan():
    """fi_jpeg_parse.cpp (the GPU decoder's host header parser and Huffman
    table builder) over every truncation and 3000 random mutations of each
    input, under ASan/UBSan."""
    hipcc = _compiler("hipcc")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "jpeg_fuzz")
        subprocess.run([hipcc, "-std=c++17", "-fno-gpu-sanitize", *SAN, "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests/native/jpeg_fuzz_driver.cpp"),
                        os.path.join(ROOT, "flyimg_amd/csrc/fi_jpeg_parse.cpp"), "-o", exe],
                       check=True, capture_output=True, timeout=300)
        files = _jpeg_inputs(d)
        r = subprocess.run([exe, *files], capture_output=True, text=True, timeout=300, env=ENV)
        assert r.returncode == 0, r.stderr[-4000:]
        assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
        assert "DONE" in r.stdout and int(r.stdout.split()[1]) > 5 * 3000
