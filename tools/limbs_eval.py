#!/usr/bin/env python3
"""Model of the weight quantisation of k_rs_vr's two-limb tables (fi_plan.h
VrV): a Lanczos resample (IM's ResizeImage: vertical pass, Q16
ClampToQuantum, horizontal pass, ScaleQuantumToChar; optional Rec709 gray) in
f64, against the same with the weights quantised to W = rint(w * 2^shift):

  * a fixed shift (16 / 15), each tap rounded alone -- the exact-match rate
    falls to 98.5 % at a 1/10 factor: rounding each tap alone leaves every
    output row's weight sum off by a few units, a bias that repeats on every
    output at integral factors;
  * the shift fi_plan.cpp vr_quant picks (the largest whose W fit two signed
    bytes) with each row's sum kept (quant_axis): >= 99.95 % exact.

CPU only:  python tools/limbs_eval.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flyimg_amd.synth import synth_rgb  # noqa: E402


def lanczos(x):
    x = np.abs(x)
    return np.where(x < 3, np.sinc(x) * np.sinc(x / 3), 0.0)


def table(n_in, n_out):
    factor = n_out / n_in
    scale = max(1 / factor, 1.0)
    support = 3 * scale
    W = np.zeros((n_out, n_in))
    for o in range(n_out):
        bis = (o + 0.5) / factor
        s = int(max(bis - support + 0.5, 0))
        e = int(min(bis + support + 0.5, n_in))
        w = lanczos((np.arange(s, e) - bis + 0.5) / scale)
        W[o, s:e] = w / w.sum()
    return W


def q_each(W, s):
    return np.rint(W * 2.0 ** s) / 2.0 ** s


def q_sum(W, s):
    X = W * 2.0 ** s
    Q = np.rint(X)
    for o in range(W.shape[0]):
        d = int(np.rint(X[o].sum()) - Q[o].sum())
        if d:
            nz = np.nonzero(W[o])[0]
            r = (X[o, nz] - Q[o, nz]) * np.sign(d)
            Q[o, nz[np.argsort(-r, kind="stable")[:abs(d)]]] += np.sign(d)
    return Q / 2.0 ** s


def shift_of(W):
    for s in range(22, 14, -1):
        q = np.rint(W * 2.0 ** s)
        if q.min() >= -32896 and q.max() <= 32639:
            return s
    return 0


def resample(img, Wv, Wh, gray):
    v = np.einsum("ok,kwc->owc", Wv, img.astype(np.float64))
    Q = np.clip(np.floor(257.0 * v + 0.5), 0, 65535)
    Q2 = np.clip(np.floor(np.einsum("xk,okc->oxc", Wh, Q) + 0.5), 0, 65535)
    if gray:
        Q2 = np.clip(np.floor(0.212656 * Q2[..., 0] + 0.715158 * Q2[..., 1] + 0.072186 * Q2[..., 2] + 0.5), 0, 65535)
    return np.floor((Q2 + 128) / 257)


def main():
    for (W, H, ow, oh) in [(3000, 2000, 600, 400), (1920, 1080, 500, 281), (3840, 2160, 910, 512),
                           (1200, 900, 300, 225), (333, 517, 97, 151), (1000, 1000, 900, 900)]:
        img = synth_rgb(W, H, 7)
        Wv, Wh = table(H, oh), table(W, ow)
        for gray in (False, True):
            ref = resample(img, Wv, Wh, gray)
            row = [f"{W}x{H}->{ow}x{oh}{' gray' if gray else ''}"]
            for name, f, sv, sh in [("each@16", q_each, 16, 16), ("sum@vr_quant", q_sum, shift_of(Wv), shift_of(Wh))]:
                d = np.abs(resample(img, f(Wv, sv), f(Wh, sh), gray) - ref)
                row.append(f"{name}({sv},{sh}) exact {(d == 0).mean():.5f} max {int(d.max())}")
            print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
