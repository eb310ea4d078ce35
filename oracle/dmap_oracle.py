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


def dmap_adaptive(points, H: int, W: int) -> np.ndarray:
    """utils/dmap_gen.py:14-51: sigma = 0.1 * (sum of the 3 nearest-neighbour
    distances; brute force = the KDTree k=4 query incl. self), 15 for <= 3
    points; truncate 4 -> radius int(4 sigma + 0.5); same per-axis float32 rounding."""
    pts = np.asarray(points, dtype=np.float32).reshape(-1, 2)
    den = np.zeros((H, W), dtype=np.float32)
    n = len(pts)
    if n == 0:
        return den
    p64 = pts.astype(np.float64)
    for i in range(n):
        r, c = int(pts[i, 1]), int(pts[i, 0])
        if not (r < H and c < W):
            continue
        if n > 3:
            d = np.sort(np.sqrt(((p64 - p64[i]) ** 2).sum(1)))[:4]
            sigma = (d[1] + d[2] + d[3]) * 0.1
        else:
            sigma = 15.0
        rad = int(4.0 * sigma + 0.5)
        w = gauss1d(sigma, rad)
        st = (w.astype(np.float32).astype(np.float64)[:, None] * w[None, :]).astype(np.float32)
        if r < 0:
            r += H
        if c < 0:
            c += W
        r0, r1 = max(0, r - rad), min(H, r + rad + 1)
        c0, c1 = max(0, c - rad), min(W, c + rad + 1)
        den[r0:r1, c0:c1] += st[r0 - r + rad:r1 - r + rad, c0 - c + rad:c1 - c + rad]
    return den
