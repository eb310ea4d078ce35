"""TEST INFRASTRUCTURE ONLY — numpy restatement of
utils/dmap_gen.py:53-81 `gaussian_filter_density_fixed` (and :14-51 adaptive).

The reference adds, per point, a full-frame scipy.ndimage.gaussian_filter of a
unit impulse (sigma=4, truncate=7/sigma -> radius int(7+0.5)=7, mode='constant').
That equals a 15x15 separable stamp clipped at the frame: scipy filters axis 0
then axis 1, each pass accumulating in float64 and storing float32, so the stamp
value is f32(f32(w_i) * w_j) with w = normalized exp(-x^2/(2 sigma^2)), and the
per-point maps are summed in float32 in point order.
"""
from __future__ import annotations

import numpy as np


def gauss1d(sigma: float, radius: int) -> np.ndarray:
    x = np.arange(-radius, radius + 1, dtype=np.float64)
    phi = np.exp(-0.5 / (sigma * sigma) * x * x)
    return phi / phi.sum()


def stamp(sigma: float = 4.0, radius: int = 7) -> np.ndarray:
    w = gauss1d(sigma, radius)
    col = w.astype(np.float32).astype(np.float64)
    return (col[:, None] * w[None, :]).astype(np.float32)


def dmap_fixed(points, H: int, W: int, sigma: float = 4.0, radius: int | None = None) -> np.ndarray:
    if radius is None:
        radius = int((7.0 / sigma) * sigma + 0.5)
    st = stamp(sigma, radius)
    den = np.zeros((H, W), dtype=np.float32)
    for x, y in np.asarray(points, dtype=np.float64).reshape(-1, 2):
        r, c = int(y), int(x)  # python int() truncation, as the reference
        if not (r < H and c < W):
            continue
        if r < 0:
            r += H  # numpy negative-index wrap (dmap_gen.py:74-75)
        if c < 0:
            c += W
        if r < 0 or c < 0:
            continue
        r0, r1 = max(0, r - radius), min(H, r + radius + 1)
        c0, c1 = max(0, c - radius), min(W, c + radius + 1)
        den[r0:r1, c0:c1] += st[r0 - r + radius:r1 - r + radius, c0 - c + radius:c1 - c + radius]
    return den
