"""Generate the golden vectors that pin the CPU oracle (run in the build
container, where /root/reference exists; the GPU box never runs this).

Sources of truth, in order:
  * the reference module itself, /root/reference/python/smartcrop.py, imported
    with the one compatibility line PIL.Image.ANTIALIAS = LANCZOS (Pillow >= 10
    removed the alias the module uses at smartcrop.py:113,167) -- SURVEY.md 8(c);
  * Pillow 12.2.0 as installed here (the arithmetic smartcrop.py delegates to:
    convert("L", matrix), Kernel filter, reduce, LANCZOS resample, thumbnail);
  * the reference's own known answers: ImageProcessorTest.php:74-261 (output
    geometry) and SmartCropProcessorTest.php:16-24 with its 674x674 result.

Outputs (data only: inputs are regenerated from flyimg_amd/synth.py and checked
by sha256; the reference's own test image smart_crop.jpg is copied as data):
  smartcrop_golden.json, pillow_golden.json, im_geometry_cases.json,
  smart_crop.jpg, smartcrop_arrays.npz
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import shutil
import sys

import numpy as np
import PIL
import PIL.Image

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
from flyimg_amd.synth import SEED_BASE, synth_rgb  # noqa: E402

PIL.Image.ANTIALIAS = PIL.Image.Resampling.LANCZOS


def load_reference_smartcrop():
    spec = importlib.util.spec_from_file_location("ref_smartcrop", os.path.join(REF, "python", "smartcrop.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def fhex(v: float) -> str:
    return float(v).hex()


# (name, width, height, seed-or-kind)
SMARTCROP_CASES = [
    ("cfg2_500x281", 500, 281, SEED_BASE + 0),
    ("cfg2_500x281_b", 500, 281, SEED_BASE + 1),
    ("cfg5_400x400", 400, 400, SEED_BASE + 2),
    ("land_640x360", 640, 360, SEED_BASE + 3),
    ("port_281x500", 281, 500, SEED_BASE + 4),
    ("sq_300x300", 300, 300, SEED_BASE + 5),
    ("wide_900x200", 900, 200, SEED_BASE + 6),
    ("small_150x100", 150, 100, SEED_BASE + 7),
    ("exact_111x111", 111, 111, SEED_BASE + 8),
    ("tiny_100x100", 100, 100, SEED_BASE + 9),
    ("tiny_64x48", 64, 48, SEED_BASE + 10),
    ("reduce_1000x600", 1000, 600, SEED_BASE + 11),
    ("black_500x281", 500, 281, "black"),
    ("white_320x240", 320, 240, "white"),
    ("skin_300x200", 300, 200, "skin"),
    ("gray_ramp_256x160", 256, 160, "ramp"),
]


def make_input(w, h, kind):
    if kind == "black":
        return np.zeros((h, w, 3), np.uint8)
    if kind == "white":
        return np.full((h, w, 3), 255, np.uint8)
    if kind == "skin":
        a = np.empty((h, w, 3), np.uint8)
        a[:] = (199, 145, 112)
        return a
    if kind == "ramp":
        v = (np.arange(w, dtype=np.int64)[None, :] + 2 * np.arange(h, dtype=np.int64)[:, None]) % 256
        return np.repeat(v[:, :, None], 3, axis=2).astype(np.uint8)
    return synth_rgb(w, h, kind)


def run_reference(sc, arr, width=100, height=100):
    im = PIL.Image.fromarray(arr, "RGB")
    r = sc.SmartCrop().crop(im, width=width, height=height)
    crops = []
    for c in r["crops"]:
        s = c["score"]
        crops.append([c["x"], c["y"], c["width"], c["height"], fhex(s["detail"]), fhex(s["saturation"]),
                      fhex(s["skin"]), fhex(s["total"])])
    top = r["top_crop"]
    top_index = next(i for i, c in enumerate(r["crops"]) if c is top)
    geometry = "%sx%s+%s+%s" % (top["width"] + top["x"], top["height"] + top["y"], top["x"], top["y"])
    ana = np.asarray(r["analyse_image"])
    return {"crops": crops, "top_index": top_index, "geometry": geometry,
            "analyse_size": list(r["analyse_image"].size), "maps_sha256": sha(ana)}, ana


def reference_intermediates(sc, arr, width=100, height=100):
    """Re-derive the prescaled image and L map exactly as SmartCrop.crop()."""
    import math

    im = PIL.Image.fromarray(arr, "RGB")
    scale = min(im.size[0] / width, im.size[1] / height)
    min_scale = min(1, max(1 / scale, 0.9))
    pre = 1 / scale / min_scale
    if pre < 1:
        im = im.copy()
        im.thumbnail((int(im.size[0] * pre), int(im.size[1] * pre)), PIL.Image.ANTIALIAS)
    else:
        pre = 1
    L = np.asarray(im.convert("L", (0.2126, 0.7152, 0.0722, 0)))
    return np.asarray(im), L, pre


def geometry_cases():
    """ImageProcessorTest.php:74-261 -> (options, expected 'WxH', fixture)."""
    P = os.path.join(REF, "tests", "testImages")
    SQ, LAND, PORT = "square-opaque-600.png", "landscape-color-squares-900x600.png", "portrait-color-squares-600x900.png"
    SSQ, SLAND, SPORT = "square-opaque-200.png", "landscape-color-squares-300x200.png", "portrait-color-squares-200x300.png"
    shrink = [
        ("w_300", "300x300", SQ), ("w_300", "300x200", LAND), ("w_300", "300x451", PORT),
        ("h_300", "300x300", SQ), ("h_300", "450x300", LAND), ("h_300", "200x300", PORT),
        ("w_300,h_150", "150x150", SQ), ("w_300,h_150", "225x150", LAND), ("w_300,h_150", "100x150", PORT),
        ("w_150,h_300", "150x150", SQ), ("w_150,h_300", "150x100", LAND), ("w_150,h_300", "150x225", PORT),
        ("w_300,h_300,c_1", "300x300", SQ), ("w_300,h_300,c_1", "300x300", LAND), ("w_300,h_300,c_1", "300x300", PORT),
        ("w_250,h_300,c_1", "250x300", SQ), ("w_250,h_300,c_1", "250x300", LAND), ("w_250,h_300,c_1", "250x300", PORT),
        ("w_150,h_300,c_1", "150x300", SQ), ("w_150,h_300,c_1", "150x300", LAND), ("w_150,h_300,c_1", "150x300", PORT),
        ("w_300,h_250,c_1", "300x250", SQ), ("w_300,h_250,c_1", "300x250", LAND), ("w_300,h_250,c_1", "300x250", PORT),
        ("w_300,h_150,c_1", "300x150", SQ), ("w_300,h_150,c_1", "300x150", LAND), ("w_300,h_150,c_1", "300x150", PORT),
    ]
    expand = [
        ("w_400", "200x200", SSQ), ("w_400", "300x200", SLAND), ("w_400", "200x300", SPORT),
        ("h_400", "200x200", SSQ), ("h_400", "300x200", SLAND), ("h_400", "200x300", SPORT),
        ("w_400,h_300", "200x200", SSQ), ("w_400,h_300", "300x200", SLAND), ("w_400,h_350", "200x300", SPORT),
        ("w_320,h_400", "200x200", SSQ), ("w_320,h_400", "300x200", SLAND), ("w_320,h_400", "200x300", SPORT),
        ("w_400,h_400,c_1", "200x200", SSQ), ("w_400,h_400,c_1", "300x200", SLAND), ("w_400,h_400,c_1", "200x300", SPORT),
        ("w_310,h_600,c_1", "200x200", SSQ), ("w_310,h_600,c_1", "300x200", SLAND), ("w_310,h_600,c_1", "200x300", SPORT),
        ("w_320,h_640,c_1", "200x200", SSQ), ("w_320,h_640,c_1", "300x200", SLAND), ("w_320,h_400,c_1", "200x300", SPORT),
        ("w_380,h_320,c_1", "200x200", SSQ), ("w_380,h_320,c_1", "300x200", SLAND), ("w_380,h_320,c_1", "200x300", SPORT),
        ("w_600,h_300,c_1", "200x200", SSQ), ("w_600,h_300,c_1", "300x200", SLAND), ("w_600,h_300,c_1", "200x300", SPORT),
        ("w_250,h_250,c_1", "250x200", SLAND), ("w_250,h_250,c_1", "200x250", SPORT),
        ("w_190,h_220,c_1", "190x200", SSQ), ("w_210,h_300,c_1", "210x200", SLAND), ("w_210,h_290,c_1", "200x290", SPORT),
        ("w_190,h_300,c_1", "190x200", SSQ), ("w_190,h_350,c_1", "190x200", SLAND), ("w_190,h_350,c_1", "190x300", SPORT),
        ("w_250,h_190,c_1", "200x190", SSQ), ("w_290,h_210,c_1", "290x200", SLAND), ("w_290,h_210,c_1", "200x210", SPORT),
        ("w_320,h_190,c_1", "200x190", SSQ), ("w_320,h_190,c_1", "300x190", SLAND), ("w_320,h_190,c_1", "200x190", SPORT),
    ]
    out = []
    sizes = {}
    for fn in {c[2] for c in shrink + expand}:
        im = PIL.Image.open(os.path.join(P, fn))
        sizes[fn] = (im.size[0], im.size[1], im.mode)
    for opts, exp, fn in shrink + expand:
        w, h, mode = sizes[fn]
        out.append({"options": opts, "expected": exp, "fixture": fn, "src_w": w, "src_h": h, "mode": mode,
                    "ref": "tests/Core/Processor/ImageProcessorTest.php"})
    return out


def pillow_cases(rng_seed=1234):
    """Pillow primitives on synthetic inputs: reduce, resample(box), thumbnail."""
    cases = []
    base = synth_rgb(257, 193, rng_seed)
    for fx, fy in [(1, 2), (2, 1), (2, 2), (3, 3), (4, 4), (5, 5), (2, 3), (3, 2), (1, 5), (6, 1), (7, 3), (4, 6), (8, 8)]:
        out = np.asarray(PIL.Image.fromarray(base).reduce((fx, fy)))
        cases.append({"op": "reduce", "fx": fx, "fy": fy, "sha256": sha(out), "shape": list(out.shape)})
    for (ow, oh, box) in [(100, 70, None), (64, 64, None), (200, 150, None), (300, 250, None),
                          (90, 60, (0.0, 0.0, 128.5, 96.5)), (50, 40, (0.0, 0.0, 85.66666666666667, 64.33333333333333)),
                          (257, 100, None), (120, 193, None)]:
        out = np.asarray(PIL.Image.fromarray(base).resize((ow, oh), PIL.Image.Resampling.LANCZOS, box=box))
        cases.append({"op": "resample", "ow": ow, "oh": oh, "box": box, "sha256": sha(out), "shape": list(out.shape)})
    for (W, H, tx, ty, seed) in [(500, 281, 197, 111, 1), (1000, 750, 148, 111, 2), (400, 400, 111, 111, 3),
                                 (640, 360, 197, 111, 4), (3000, 2000, 166, 111, 5), (281, 500, 111, 197, 6),
                                 (123, 77, 100, 60, 7), (900, 200, 499, 111, 8), (1920, 1080, 197, 111, 9)]:
        src = synth_rgb(W, H, seed)
        im = PIL.Image.fromarray(src)
        im.thumbnail((tx, ty), PIL.Image.Resampling.LANCZOS)
        out = np.asarray(im)
        cases.append({"op": "thumbnail", "W": W, "H": H, "seed": seed, "tx": tx, "ty": ty,
                      "sha256": sha(out), "shape": list(out.shape)})
    return {"base_seed": rng_seed, "base_shape": [193, 257, 3], "base_sha256": sha(base), "cases": cases}


def luma_table_sha():
    """Exhaustive convert("L", Rec709 matrix) over all 2^24 RGB values."""
    v = np.arange(1 << 24, dtype=np.uint32)
    rgb = np.stack([(v >> 16) & 255, (v >> 8) & 255, v & 255], -1).astype(np.uint8).reshape(4096, 4096, 3)
    L = np.asarray(PIL.Image.fromarray(rgb, "RGB").convert("L", (0.2126, 0.7152, 0.0722, 0)))
    return sha(L)


def main():
    sc = load_reference_smartcrop()
    golden = {"generator": "tests/golden/make_golden.py", "pillow": PIL.__version__, "numpy": np.__version__,
              "reference": "python/smartcrop.py", "cases": []}
    arrays = {}
    for name, w, h, kind in SMARTCROP_CASES:
        arr = make_input(w, h, kind)
        res, ana = run_reference(sc, arr)
        pre_img, L, pre = reference_intermediates(sc, arr)
        case = {"name": name, "w": w, "h": h, "kind": kind if isinstance(kind, str) else "synth",
                "seed": kind if not isinstance(kind, str) else None, "input_sha256": sha(arr),
                "target": [100, 100], "prescale": fhex(pre), "prescaled_sha256": sha(pre_img),
                "L_sha256": sha(L), **res}
        golden["cases"].append(case)
        if name in ("cfg2_500x281", "tiny_64x48", "black_500x281"):
            arrays[name + "_prescaled"] = pre_img
            arrays[name + "_maps"] = ana
            arrays[name + "_L"] = L
        print(name, res["geometry"], len(res["crops"]), res["analyse_size"])
    # the reference's own smart-crop fixture (SmartCropProcessorTest.php:16-24)
    jpg = os.path.join(REF, "tests", "testImages", "smart_crop.jpg")
    shutil.copyfile(jpg, os.path.join(HERE, "smart_crop.jpg"))
    arr = np.asarray(PIL.Image.open(jpg).convert("RGB"))
    res, ana = run_reference(sc, arr)
    pre_img, L, pre = reference_intermediates(sc, arr)
    golden["fixture"] = {"name": "smart_crop.jpg", "w": arr.shape[1], "h": arr.shape[0], "input_sha256": sha(arr),
                         "expected_result_dims": "674x674", "prescale": fhex(pre),
                         "prescaled_sha256": sha(pre_img), "L_sha256": sha(L), **res}
    print("fixture", res["geometry"], len(res["crops"]))
    # portrait target (smartcrop.py main(): height = int(h / w * 100)) on one case
    arr = make_input(500, 281, SEED_BASE)
    res, _ = run_reference(sc, arr, width=100, height=56)
    golden["nonsquare_target"] = {"w": 500, "h": 281, "seed": SEED_BASE, "target": [100, 56], **res}
    with open(os.path.join(HERE, "smartcrop_golden.json"), "w") as f:
        json.dump(golden, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "smartcrop_arrays.npz"), **arrays)
    pil = pillow_cases()
    pil["luma_table_sha256"] = luma_table_sha()
    pil["pillow"] = PIL.__version__
    with open(os.path.join(HERE, "pillow_golden.json"), "w") as f:
        json.dump(pil, f, indent=1)
    with open(os.path.join(HERE, "im_geometry_cases.json"), "w") as f:
        json.dump(geometry_cases(), f, indent=1)
    print("done")


if __name__ == "__main__":
    main()
