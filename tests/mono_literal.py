"""Literal pure-Python restatement of ImageMagick 6's -monochrome for SMALL
images -- test infrastructure only (cross-checks oracle/fi_oracle.c's
or_im_monochrome, which reformulates the sums deterministically).

Follows IM 6 (Q16, non-HDRI) SetImageType(BilevelType) as the oracle header
describes it (reference call site
src/Core/Processor/ImageProcessor.php:90-92), statement by statement:
  * ContrastStretchImageChannel black/white search and stretch map (enhance.c);
  * ClassifyImageColors: raster order, runs of equal pixels (count), per-level
    midpoint bisection, quantize_error += count * sqrt(distance), the root's
    running-error sum, leaf totals count * QuantumScale * pixel (quantize.c);
  * ReduceImageColors: QuantizeErrorFlatten + qsort "rapid reduction", then
    Reduce / PruneChild passes;
  * DefineImageColormap, Riemersma (recursive Hilbert walk), RiemersmaDither
    with the CacheOffset cache and ClosestColor, the monochrome colormap
    threshold.
Parity with ImageMagick itself is unpinned (IM is absent here).
"""
from __future__ import annotations

import math
import sys

import numpy as np

QR = 65535.0
QSCALE = 1.0 / 65535.0


def q2c(q: int) -> int:
    return ((q + 128) - ((q + 128) >> 8)) >> 8


def clamp_pixel(v: float) -> int:
    if v < 0.0:
        return 0
    if v >= QR:
        return 65535
    return int(v + 0.5)


def clamp_to_quantum(v: float) -> int:
    if v <= 0.0:
        return 0
    if v >= QR:
        return 65535
    return int(v + 0.5)


class Node:
    __slots__ = ("child", "parent", "id", "level", "qerr", "nu", "tot", "color")

    def __init__(self, parent, id_, level):
        self.child = [None] * 8
        self.parent = parent if parent is not None else self
        self.id = id_
        self.level = level
        self.qerr = 0.0
        self.nu = 0
        self.tot = 0.0
        self.color = -1


def stretch(g: np.ndarray) -> np.ndarray:
    n = g.size
    hist = np.bincount(g.ravel(), minlength=65536)
    bp, wp = n * 0.0015, n * 0.9995
    acc = 0.0
    i = 0
    while i <= 65535:
        acc += float(hist[i])
        if acc > bp:
            break
        i += 1
    black = float(i)
    acc = 0.0
    i = 65535
    while i != 0:
        acc += float(hist[i])
        if acc > (n - wp):
            break
        i -= 1
    white = float(i)
    if black == white:
        return g.copy()
    out = np.empty_like(g)
    for idx, q in np.ndenumerate(g):
        q = int(q)
        if q < int(black):
            v = 0
        elif q > int(white):
            v = 65535
        else:
            m = 65535.0 * (q - black) / (white - black)
            v = 0 if m <= 0.0 else (65535 if m >= 65535.0 else int(m + 0.5))
        out[idx] = v
    return out


def monochrome(g: np.ndarray, exact_sums: bool = False) -> np.ndarray:
    """IM's -monochrome on a Q16 gray image -> 0/255.  exact_sums=True holds
    the leaf colour sums as exact integers (the oracle's reformulation);
    False accumulates count * QuantumScale * pixel in raster order as IM does."""
    g = np.asarray(g, dtype=np.uint16)
    h, w = g.shape
    if np.all((g == 0) | (g == 65535)):
        return np.where(g > 0, 255, 0).astype(np.uint8)
    s = stretch(g)
    root = Node(None, 0, 0)
    nodes = [1]
    colors = [0]
    # ClassifyImageColors
    for y in range(h):
        x = 0
        while x < w:
            count = 1
            while x + count < w and s[y, x + count] == s[y, x]:
                count += 1
            pix = float(s[y, x])
            c8 = q2c(int(s[y, x]))
            index = 7
            bisect = (QR + 1.0) / 2.0
            mid = QR / 2.0
            node = root
            for level in range(1, 9):
                bisect *= 0.5
                bit = (c8 >> index) & 1
                idn = 7 if bit else 0
                mid += bisect if bit else -bisect
                if node.child[idn] is None:
                    node.child[idn] = Node(node, idn, level)
                    nodes[0] += 1
                    if level == 8:
                        colors[0] += 1
                node = node.child[idn]
                e = QSCALE * (pix - mid)
                d = e * e + e * e
                d = d + e * e
                d = d + 0.0 * 0.0
                node.qerr += count * math.sqrt(d)
                root.qerr += node.qerr
                index -= 1
            node.nu += count
            if exact_sums:
                node.tot += count * clamp_pixel(pix)
            else:
                node.tot += count * QSCALE * float(clamp_pixel(pix))
            x += count
    # ReduceImageColors
    maxc = 2
    state = {"pruning": 0.0, "next": 0.0, "colors": colors[0], "nodes": nodes[0]}

    def flatten(node, out):
        out.append(node.qerr)
        for ch in node.child:
            if ch is not None:
                flatten(ch, out)

    def prune(node):
        for ch in node.child:
            if ch is not None:
                prune(ch)
        p = node.parent
        p.nu += node.nu
        p.tot += node.tot
        p.child[node.id] = None
        state["nodes"] -= 1

    def reduce(node):
        for ch in list(node.child):
            if ch is not None:
                reduce(ch)
        if node.qerr <= state["pruning"]:
            prune(node)
        else:
            if node.nu > 0:
                state["colors"] += 1
            if node.qerr < state["next"]:
                state["next"] = node.qerr

    if state["colors"] > maxc:
        errs = []
        flatten(root, errs)
        errs.sort()
        k = 110 * (maxc + 1) // 100
        if state["nodes"] > k:
            state["next"] = errs[state["nodes"] - k]
    while state["colors"] > maxc:
        state["pruning"] = state["next"]
        state["next"] = root.qerr - 1
        state["colors"] = 0
        reduce(root)
    # DefineImageColormap
    cmap = []

    def define(node):
        for ch in node.child:
            if ch is not None:
                define(ch)
        if node.nu != 0:
            alpha = 1.0 / float(node.nu)
            total = float(node.tot) * QSCALE if exact_sums else node.tot
            cmap.append(clamp_to_quantum(alpha * QR * total))
            node.color = len(cmap) - 1

    define(root)
    # Riemersma dither
    wts = [0.0] * 16
    weight = 1.0
    for i in range(16):
        wts[16 - i - 1] = 1.0 / weight
        weight *= math.exp(math.log(QR + 1.0) / (16 - 1.0))
    err = [0.0] * 16
    cache = [-1] * 64
    out = np.zeros((h, w), np.uint8)
    bilevel = [0 if (0.212656 * c + 0.715158 * c + 0.072186 * c) < QR / 2.0 else 65535 for c in cmap]
    cur = {"x": 0, "y": 0}

    def closest(node, target, best):
        for ch in node.child:
            if ch is not None:
                closest(ch, target, best)
        if node.nu != 0:
            px = 1.0 * cmap[node.color] - 1.0 * target
            d = px * px
            if d <= best[0]:
                d += px * px
                if d <= best[0]:
                    d += px * px
                    if d <= best[0] and d < best[0]:
                        best[0] = d
                        best[1] = node.color

    def dither(direction):
        x, y = cur["x"], cur["y"]
        if 0 <= x < w and 0 <= y < h:
            pv = float(s[y, x])
            for i in range(16):
                pv += wts[i] * err[i]
            pv = float(clamp_pixel(pv))
            c8 = q2c(int(pv))
            key = c8 >> 2
            if cache[key] < 0:
                node = root
                for index in range(7, 0, -1):
                    idn = 7 if (c8 >> index) & 1 else 0
                    if node.child[idn] is None:
                        break
                    node = node.child[idn]
                best = [4.0 * (QR + 1.0) * (QR + 1.0) + 1.0, 0]
                closest(node.parent, pv, best)
                cache[key] = best[1]
            idx = cache[key]
            out[y, x] = 255 if bilevel[idx] else 0
            del err[0]
            err.append(pv - float(cmap[idx]))
        if direction == "W":
            cur["x"] -= 1
        elif direction == "E":
            cur["x"] += 1
        elif direction == "N":
            cur["y"] -= 1
        elif direction == "S":
            cur["y"] += 1

    def riem(level, d):
        if level == 1:
            for m in {"W": "ESW", "E": "WNE", "N": "SEN", "S": "NWS"}[d]:
                dither(m)
            return
        seq = {
            "W": ("N", "E", "W", "S", "W", "W", "S"),
            "E": ("S", "W", "E", "N", "E", "E", "N"),
            "N": ("W", "S", "N", "E", "N", "N", "E"),
            "S": ("E", "N", "S", "W", "S", "S", "W"),
        }[d]
        riem(level - 1, seq[0])
        dither(seq[1])
        riem(level - 1, seq[2])
        dither(seq[3])
        riem(level - 1, seq[4])
        dither(seq[5])
        riem(level - 1, seq[6])

    i = max(w, h)
    depth = 1
    while i != 0:
        i >>= 1
        depth += 1
    if (1 << depth) < max(w, h):
        depth += 1
    old = sys.getrecursionlimit()
    sys.setrecursionlimit(max(old, 10000))
    if depth > 1:
        riem(depth - 1, "N")
    dither("F")
    return out


def curve_positions(level: int):
    """Cells visited by IM's Riemersma(level, NorthGravity) walk from (0, 0)
    plus the final ForgetGravity cell (the recursion above, moves only)."""
    seqs = {
        "W": ("N", "E", "W", "S", "W", "W", "S"),
        "E": ("S", "W", "E", "N", "E", "E", "N"),
        "N": ("W", "S", "N", "E", "N", "N", "E"),
        "S": ("E", "N", "S", "W", "S", "S", "W"),
    }
    moves = []

    def riem(lv, d):
        if lv == 1:
            moves.extend({"W": "ESW", "E": "WNE", "N": "SEN", "S": "NWS"}[d])
            return
        q = seqs[d]
        riem(lv - 1, q[0])
        moves.append(q[1])
        riem(lv - 1, q[2])
        moves.append(q[3])
        riem(lv - 1, q[4])
        moves.append(q[5])
        riem(lv - 1, q[6])

    riem(level, "N")
    x = y = 0
    pts = [(0, 0)]
    step = {"W": (-1, 0), "E": (1, 0), "N": (0, -1), "S": (0, 1)}
    for m in moves:
        dx, dy = step[m]
        x += dx
        y += dy
        pts.append((x, y))
    return pts
