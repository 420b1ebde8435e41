"""Helpers to load the committed golden vectors (tests/golden/)."""
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def case_input(case):
    """Regenerate a smartcrop golden case's input (checked by sha256)."""
    from flyimg_amd.synth import synth_rgb

    w, h, kind = case["w"], case["h"], case["kind"]
    if kind == "synth":
        arr = synth_rgb(w, h, case["seed"])
    elif kind == "black":
        arr = np.zeros((h, w, 3), np.uint8)
    elif kind == "white":
        arr = np.full((h, w, 3), 255, np.uint8)
    elif kind == "skin":
        arr = np.empty((h, w, 3), np.uint8)
        arr[:] = (199, 145, 112)
    elif kind == "ramp":
        v = (np.arange(w, dtype=np.int64)[None, :] + 2 * np.arange(h, dtype=np.int64)[:, None]) % 256
        arr = np.repeat(v[:, :, None], 3, axis=2).astype(np.uint8)
    else:
        raise ValueError(kind)
    assert sha(arr) == case["input_sha256"], "synthetic generator drifted from the golden input"
    return arr


def fixture_input():
    """smart_crop.jpg (reference tests/testImages) decoded by Pillow."""
    import PIL.Image

    g = load("smartcrop_golden.json")["fixture"]
    arr = np.asarray(PIL.Image.open(os.path.join(GOLDEN, "smart_crop.jpg")).convert("RGB"))
    assert sha(arr) == g["input_sha256"], "JPEG decode differs from the golden decode"
    return arr
