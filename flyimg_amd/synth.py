"""Seeded synthetic RGB8 images (BASELINE.json configs use synthetic inputs).

The generator is pure 32-bit integer arithmetic so that the numpy version here
and the device version (``fi_fill_synthetic`` in csrc/fi_synth.hip) produce
identical bytes; tests/test_gpu_parity.py checks that.  Content: a smooth
coarse-grid field (bilinear between hashed 64-px grid nodes), uniform noise,
and skin-tone discs so that smartcrop's skin / saturation maps are non-empty
(seed = 0x5EED + image index).
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 0x5EED
GRID = 64  # px between smooth-field nodes
NOISE = 24  # peak-to-peak noise amplitude
SKIN_CELL = 96  # one potential skin disc per 96x96 cell


def _mix32(x):
    x = np.asarray(x, dtype=np.uint32)
    x = x ^ (x >> np.uint32(16))
    x = x * np.uint32(0x7FEB352D)
    x = x ^ (x >> np.uint32(15))
    x = x * np.uint32(0x846CA68B)
    x = x ^ (x >> np.uint32(16))
    return x


def _hash4(seed, a, b, c):
    s = np.uint32(seed) * np.uint32(0x9E3779B1)
    t = _mix32(np.asarray(b, np.uint32) * np.uint32(0xC2B2AE3D) ^ np.asarray(c, np.uint32))
    u = _mix32(np.asarray(a, np.uint32) * np.uint32(0x85EBCA77) ^ t)
    return _mix32(s ^ u)


def synth_rgb(width: int, height: int, seed: int) -> np.ndarray:
    """Return an (height, width, 3) uint8 image; identical to the HIP kernel."""
    with np.errstate(over="ignore"):
        y = np.arange(height, dtype=np.uint32)[:, None]
        x = np.arange(width, dtype=np.uint32)[None, :]
        gi, gj = x // GRID, y // GRID
        fx, fy = (x % GRID).astype(np.int64), (y % GRID).astype(np.int64)
        out = np.empty((height, width, 3), np.uint8)
        for c in range(3):
            g00 = (_hash4(seed, gi, gj, c) & 255).astype(np.int64)
            g10 = (_hash4(seed, gi + 1, gj, c) & 255).astype(np.int64)
            g01 = (_hash4(seed, gi, gj + 1, c) & 255).astype(np.int64)
            g11 = (_hash4(seed, gi + 1, gj + 1, c) & 255).astype(np.int64)
            smooth = (g00 * (GRID - fx) * (GRID - fy) + g10 * fx * (GRID - fy)
                      + g01 * (GRID - fx) * fy + g11 * fx * fy) >> 12
            noise = (_hash4(seed ^ 0xA5A5A5A5, x, y, c) % NOISE).astype(np.int64) - NOISE // 2
            out[:, :, c] = np.clip(smooth + noise, 0, 255).astype(np.uint8)
        # skin-tone discs: cell (ci, cj) holds a disc if its hash says so
        ci, cj = x // SKIN_CELL, y // SKIN_CELL
        h = _hash4(seed ^ 0x51D1, ci, cj, 7)
        has = (h & 3) == 0
        cx = (ci * SKIN_CELL + 24 + ((h >> 8) & 47)).astype(np.int64)
        cy = (cj * SKIN_CELL + 24 + ((h >> 16) & 47)).astype(np.int64)
        r = (12 + ((h >> 24) & 15)).astype(np.int64)
        dx, dy = x.astype(np.int64) - cx, y.astype(np.int64) - cy
        inside = has & (dx * dx + dy * dy <= r * r)
        shade = ((h >> 4) & 31).astype(np.int64)
        skin = np.stack([np.broadcast_to(np.clip(190 + shade, 0, 255), inside.shape),
                         np.broadcast_to(np.clip(135 + shade, 0, 255), inside.shape),
                         np.broadcast_to(np.clip(105 + shade, 0, 255), inside.shape)], -1)
        out = np.where(inside[:, :, None], skin.astype(np.uint8), out)
    return np.ascontiguousarray(out)
