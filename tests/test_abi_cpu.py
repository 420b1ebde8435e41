"""CPU: the C-ABI library loads, exports every declared symbol, and its host
planner (fi_plan, no GPU) reproduces the reference's geometry known answers
through the host-side mirror of OptionsBag / ImageProcessor."""
import ctypes
import subprocess

import pytest

from flyimg_amd import _lib as L
from flyimg_amd.processor import ExecFailedException, ImageProcessor, OptionsBag
from flyimg_amd.runtime import Op, plan
from tests import _golden as G


def test_library_exports_every_header_symbol():
    lib = L.lib()
    names = L.header_functions()
    assert len(names) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        assert hasattr(lib, n)
    assert lib.fi_abi_version() == 2


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", L.LIB_PATH], capture_output=True, text=True)
    # offload bundle carries gfx950; fall back to grepping the binary
    data = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_struct_sizes_match_header():
    # fi_image: 8 + 4*11 + 8 + 8 + 4*8 + 8 + 4*2 = 8+44+... checked against ctypes layout
    assert ctypes.sizeof(L.FiImage) % 8 == 0
    assert ctypes.sizeof(L.FiRecord) == 32
    assert ctypes.sizeof(L.FiCropScore) == 16 + 32 + 32 + 8


GEOM = G.load("im_geometry_cases.json")


@pytest.mark.parametrize("case", GEOM, ids=[f"{c['options']}@{c['fixture']}" for c in GEOM])
def test_fi_plan_geometry_known_answers(case):
    """ImageProcessorTest.php:74-261 through OptionsBag -> ImageProcessor -> fi_plan."""
    bag = OptionsBag(case["options"])
    op = ImageProcessor(bag, case["src_w"], case["src_h"]).to_op()
    w, h, c = plan(case["src_w"], case["src_h"], op)
    assert f"{w}x{h}" == case["expected"]


def test_options_bag_parse_known_answer():
    """OutputImageTest.php:18-67 (OPTION_URL of BaseTest.php:31)."""
    bag = OptionsBag("w_200,h_100,c_1,bg_#999999,rz_1,sc_50,r_-45,unsh_0.25x0.25+8+0.065,ett_100x80,fb_1,rf_1")
    a = bag.as_array()
    expect = {"width": "200", "height": "100", "crop": "1", "background": "#999999", "resize": "1",
              "scale": "50", "rotate": "-45", "unsharp": "0.25x0.25+8+0.065", "extent": "100x80",
              "face-blur": "1", "refresh": "1", "gravity": "Center", "filter": "Lanczos", "quality": 90,
              "colorspace": "sRGB", "preserve-natural-size": 1, "smart-crop": False}
    for k, v in expect.items():
        assert a[k] == v, k
    assert len(a) == 37


def test_generate_command_matches_reference_shape():
    bag = OptionsBag("w_300,h_250,c_1")
    cmd = ImageProcessor(bag, 3000, 2000).generate_command("in.jpg", "out.jpg")
    assert "-thumbnail '300'x'250'^ -gravity Center -extent '300'x'250'" in cmd
    assert "-colorspace sRGB" in cmd and "-filter Lanczos" in cmd and "-strip" in cmd
    bag = OptionsBag("w_500,smc_1")
    cmd = ImageProcessor(bag, 1920, 1080).generate_command()
    assert "-thumbnail '500''>'" in cmd


def test_baseline_configs_plan():
    cases = [
        ("w_300,h_250,c_1", 3000, 2000, (300, 250, 3)),
        ("w_500,smc_1", 1920, 1080, (500, 281, 3)),
        ("w_512,h_512,c_1", 3840, 2160, (512, 512, 3)),
        ("w_400,h_400,c_1,r_90,clsp_Gray,smc_1", 6000, 4000, (400, 400, 1)),
    ]
    for opts, w, h, exp in cases:
        op = ImageProcessor(OptionsBag(opts), w, h).to_op()
        assert plan(w, h, op) == exp, opts


def test_unsupported_ops_fail_loudly():
    with pytest.raises(ExecFailedException):
        ImageProcessor(OptionsBag("w_200,r_-45"), 400, 300).to_op()
    op = Op(100, 0, L.FI_OP_THUMBNAIL, rotate=45)
    op.flags |= L.FI_OP_ROTATE
    with pytest.raises(L.FiError):
        plan(400, 300, op)


def test_monochrome_plans_one_channel():
    """mnchr_1 (ImageProcessor.php:90-92): -monochrome converts to GRAY, so the
    output has one channel; rotation applies after it."""
    from flyimg_amd.processor import ImageProcessor, OptionsBag

    assert plan(400, 300, ImageProcessor(OptionsBag("w_100,mnchr_1"), 400, 300).to_op()) == (100, 75, 1)
    assert plan(400, 300, ImageProcessor(OptionsBag("w_100,h_50,c_1,r_90,mnchr_1"), 400, 300).to_op()) == (50, 100, 1)


def _norm_decls(text, struct="fi_image"):
    """Function prototypes and the fields of one struct of a C header, whitespace-normalised."""
    import re

    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][A-Za-z0-9_ \*]*?\b(fi_[a-z0-9_]+)\s*\([^;{]*\))\s*;", text):
        protos[m.group(2)] = re.sub(r"\s+", " ", m.group(1)).replace("( ", "(").strip()
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (struct, struct), text, flags=re.S).group(1)
    fields = []
    for decl in body.split(";"):
        decl = re.sub(r"\s+", " ", decl).strip()
        if not decl:
            continue
        m = re.match(r"(.*?)\s*(\**)([A-Za-z_][A-Za-z0-9_]*(?:\[\d+\])?)((?:\s*,\s*\**[A-Za-z_][A-Za-z0-9_]*)*)$", decl)
        base = m.group(1)
        names = [m.group(2) + m.group(3)] + [n.strip() for n in m.group(4).split(",") if n.strip()]
        fields += [(base.strip(), n) for n in names]
    return protos, fields


def test_php_ffi_cdef_matches_header():
    """php/flyimg_hip_ffi.h (FFI::cdef subset) declares the
    same prototypes and the same fi_image layout as include/flyimg_hip.h."""
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "include", "flyimg_hip.h")) as f:
        hp, hf = _norm_decls(f.read())
    with open(os.path.join(root, "php", "flyimg_hip_ffi.h")) as f:
        text = f.read()
    assert not any(l.lstrip().startswith("#") for l in text.splitlines())  # FFI::cdef: no preprocessor
    pp, pf = _norm_decls(text)
    assert pp and set(pp) <= set(hp)
    for name, proto in pp.items():
        assert proto == hp[name], (proto, hp[name])
    assert pf == hf
    with open(os.path.join(root, "include", "flyimg_hip.h")) as f:
        h2 = _norm_decls(f.read(), "fi_smartcrop_params")[1]
    assert _norm_decls(text, "fi_smartcrop_params")[1] == h2  # HipSmartCropProcessor passes it by pointer


def test_codec_decode_ex_flags_pseudoclass_modes():
    """codec.decode_ex: bilevel, 8-bit gray and palette sources are IM
    PseudoClass images (Mitchell); RGB / RGBA / 16-bit gray are not."""
    import io

    import numpy as np
    from PIL import Image

    from flyimg_amd.codec import decode_ex

    rgb = (np.arange(32 * 24 * 3) % 251).astype(np.uint8).reshape(24, 32, 3)
    im = Image.fromarray(rgb)
    cases = {"1": True, "L": True, "P": True, "RGB": False, "RGBA": False}
    for mode, want in cases.items():
        buf = io.BytesIO()
        im.convert(mode).save(buf, "PNG")
        px, pseudo = decode_ex(buf.getvalue())
        assert pseudo == want, mode
        assert px.shape[:2] == (24, 32) and px.shape[2] in (3, 4)
    buf = io.BytesIO()
    im.convert("L").save(buf, "JPEG")
    assert decode_ex(buf.getvalue())[1] is True
    buf = io.BytesIO()
    Image.fromarray((np.arange(24 * 32) * 60).astype(np.uint16).reshape(24, 32)).save(buf, "PNG")
    assert decode_ex(buf.getvalue())[1] is False  # 16-bit gray: DirectClass


def test_gravity_is_case_insensitive_and_unknown_rejected():
    """IM parses -gravity case-insensitively (g_north == North); an unknown
    gravity is an error, as convert's exit status would be."""
    import pytest

    from flyimg_amd import _lib as L
    from flyimg_amd.processor import ExecFailedException, ImageProcessor, OptionsBag

    for g in ("north", "NORTH", "North"):
        op = ImageProcessor(OptionsBag(f"w_200,h_200,c_1,g_{g}"), 800, 500).to_op()
        assert op.gravity == L.GRAVITY["North"]
    with pytest.raises(ExecFailedException):
        ImageProcessor(OptionsBag("w_200,h_200,c_1,g_Upwards"), 800, 500).to_op()


def test_jpeg_encoder_chroma_sampling_follows_im_quality_rule():
    """IM 6 jpeg.c: quality >= 90 -> 4:4:4, below -> 4:2:0 (no -sampling-factor)."""
    import io

    import numpy as np
    from PIL import Image, JpegImagePlugin

    from flyimg_amd.codec import encode

    px = (np.arange(64 * 48 * 3) % 253).astype(np.uint8).reshape(48, 64, 3)
    for q, want in ((90, 0), (95, 0), (89, 2), (75, 2)):
        im = Image.open(io.BytesIO(encode(px, q)))
        assert JpegImagePlugin.get_sampling(im) == want, q
