"""Gaussian density-map generation on the GPU — drop-in for reference
utils/dmap_gen.py.

The reference adds one full-frame scipy.ndimage.gaussian_filter per point
(O(N*H*W), ~15 ms/point at 768x1024, dmap_gen.py:72-79).  Here every point is a
15x15 stamp of scipy's two-pass float32 values, in one HIP launch per batch of images:

* default (`deterministic=True`, dg_dmap_fixed_tiled): one block per 64x64 tile walks its
  image's points in order and sums the stamps that reach it -- the reference's f32
  accumulation order, so the map is bit-identical to the reference and run to run (the
  reference runs under torch.use_deterministic_algorithms, utils/misc.py:131);
* `deterministic=False` (or DGVCC_DMAP_ATOMIC=1): one wave per point with f32 atomics
  (dg_dmap_fixed), order-dependent in the last ulp of overlapping stamps.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .. import kernels as K

SIGMA_FIXED = 4.0
RADIUS_FIXED = int((7.0 / SIGMA_FIXED) * SIGMA_FIXED + 0.5)  # truncate=7/sigma -> 7


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("dgvcc_amd.utils.dmap_gen needs the GPU (HIP kernel); no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


_ATOMIC = os.environ.get("DGVCC_DMAP_ATOMIC", "0") == "1"


def gaussian_filter_density_fixed_batch(points_list, H: int, W: int, sigma: float = SIGMA_FIXED,
                                        radius: int = RADIUS_FIXED, deterministic: bool | None = None) -> torch.Tensor:
    """points_list: N tensors [n_i, 2] (x=col, y=row).  Returns [N, H, W] f32 on device."""
    dev = points_list[0].device if len(points_list) and points_list[0].is_cuda else _device()
    counts = [int(p.shape[0]) for p in points_list]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(counts)]), dtype=torch.int64, device=dev)
    if sum(counts):
        pts = torch.cat([p.to(dev, torch.float32).reshape(-1, 2) for p in points_list]).contiguous()
    else:
        pts = torch.empty((0, 2), dtype=torch.float32, device=dev)
    det = (not _ATOMIC) if deterministic is None else deterministic
    return K.dmap_fixed(pts, offs, len(points_list), H, W, sigma, radius, deterministic=det)


def gaussian_filter_density_batch(points_list, H: int, W: int) -> torch.Tensor:
    """Adaptive-sigma maps (k-NN sigma, truncate 4) for N images -> [N, H, W] on device."""
    dev = points_list[0].device if len(points_list) and points_list[0].is_cuda else _device()
    counts = [int(p.shape[0]) for p in points_list]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(counts)]), dtype=torch.int64, device=dev)
    total = int(sum(counts))
    pts = torch.cat([p.to(dev, torch.float32).reshape(-1, 2) for p in points_list]).contiguous() \
        if total else torch.empty((0, 2), dtype=torch.float32, device=dev)
    sig = torch.empty(max(total, 1), dtype=torch.float64, device=dev)
    out = torch.empty((len(points_list), H, W), dtype=torch.float32, device=dev)
    K.call("dg_dmap_adaptive", K.ptr(pts) if total else None, K.ptr(offs), len(points_list), H, W,
           K.ptr(sig), K.ptr(out), K.stream())
    return out


def gaussian_filter_density(img, points):
    """reference dmap_gen.py:14-51 (k-nearest-neighbour adaptive sigma)."""
    H, W = int(img.shape[0]), int(img.shape[1])
    pts = torch.as_tensor(np.asarray(points, dtype=np.float32).reshape(-1, 2))
    return gaussian_filter_density_batch([pts.to(_device())], H, W)[0].cpu().numpy()


def gaussian_filter_density_fixed(img, points):
    """reference dmap_gen.py:53-81: `img` only supplies the shape (rows, cols)."""
    H, W = int(img.shape[0]), int(img.shape[1])
    pts = torch.as_tensor(np.asarray(points, dtype=np.float32).reshape(-1, 2))
    out = gaussian_filter_density_fixed_batch([pts.to(_device())], H, W)
    return out[0].cpu().numpy()


def run(img_fn):
    """File driver (dmap_gen.py:83-95): writes <name>_dmap.npy next to <name>.npy."""
    ext = os.path.splitext(img_fn)[1]
    base = os.path.basename(img_fn).replace(ext, "")
    gt_fn = img_fn.replace(ext, ".npy")
    dmap_fn = gt_fn.replace(base, base + "_dmap")
    if os.path.exists(dmap_fn):
        return
    from PIL import Image
    with Image.open(img_fn) as im:
        W, H = im.size
    gt = np.load(gt_fn)
    np.save(dmap_fn, gaussian_filter_density_fixed(np.empty((H, W), np.uint8), gt))
