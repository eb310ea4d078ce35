"""Device-side training augmentation of the reference's DenClsDataset
(datasets/den_cls_dataset.py:29-35, 77-158).

The reference applies grey-scale, horizontal flip, ToTensor/Normalize (view 1) and
`more_transform` = RandomApply(ColorJitter(0.5, 0.2, 0.2, 0.1), p=0.8),
RandomApply(GaussianBlur(3, sigma=1), p=0.5), RandomAdjustSharpness(5, p=0.5),
ToTensor/Normalize (view 2) to PIL images in host worker processes.  Here:

* the random decisions are drawn on the host with the same generators and in the
  same order as the reference (Python `random` for grey/crop/flip, torch's global RNG
  for the torchvision transforms: `draw_more_transform`), packed into a per-sample
  parameter record (`AUG_PARAMS`);
* the pixel work runs on the GPU (`dg_augment_den_cls`, augment.hip) on uint8 crops
  already in HBM, keeping PIL's integer semantics, and the block map (`dg_block_map`).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from .. import kernels as K
from .._capi import call, ptr, query, stream

AUG_PARAMS = ("grey", "flip", "jitter", "order0", "order1", "order2", "order3", "brightness", "contrast",
              "saturation", "hue_shift", "blur", "k0", "k1", "sharp", "sharp_factor")
P = {k: i for i, k in enumerate(AUG_PARAMS)}

# torchvision ColorJitter(brightness=0.5, contrast=0.2, saturation=0.2, hue=0.1) ranges
JITTER_RANGES = ((0.5, 1.5), (0.8, 1.2), (0.8, 1.2), (-0.1, 0.1))
BLUR_SIGMA = (1.0, 1.0)   # GaussianBlur(kernel_size=3, sigma=1)
SHARPNESS = 5.0


def hue_shift(hue_factor: float) -> int:
    """torchvision F_pil.adjust_hue: np.array(hue_factor * 255).astype(np.uint8)."""
    return int(np.array(hue_factor * 255).astype(np.uint8))


def gaussian_weights(sigma: float) -> tuple[float, float]:
    """torchvision _get_gaussian_kernel1d(3, sigma) in float32: (edge, centre)."""
    x = torch.linspace(-1.0, 1.0, steps=3, dtype=torch.float32)
    pdf = torch.exp(-0.5 * (x / sigma).pow(2))
    k = pdf / pdf.sum()
    return float(k[0]), float(k[1])


def draw_more_transform(rec: np.ndarray) -> None:
    """Consume torch's RNG exactly as `more_transform(img)` does and record the decisions:
    RandomApply (`p < torch.rand(1)` skips), ColorJitter.get_params (randperm(4), then one
    uniform_ per factor), GaussianBlur.get_params (uniform_), RandomAdjustSharpness (rand < p)."""
    if not (0.8 < torch.rand(1)):
        fn_idx = torch.randperm(4)
        b, c, s, h = (float(torch.empty(1).uniform_(lo, hi)) for lo, hi in JITTER_RANGES)
        rec[P["jitter"]] = 1.0
        rec[P["order0"]:P["order0"] + 4] = fn_idx.numpy().astype(np.float32)
        rec[P["brightness"]], rec[P["contrast"]], rec[P["saturation"]] = b, c, s
        rec[P["hue_shift"]] = hue_shift(h)
    if not (0.5 < torch.rand(1)):
        sigma = torch.empty(1).uniform_(BLUR_SIGMA[0], BLUR_SIGMA[1]).item()
        rec[P["blur"]] = 1.0
        rec[P["k0"]], rec[P["k1"]] = gaussian_weights(sigma)
    if torch.rand(1).item() < 0.5:
        rec[P["sharp"]] = 1.0
        rec[P["sharp_factor"]] = SHARPNESS


def new_record(grey: bool = False, flip: bool = False) -> np.ndarray:
    rec = np.zeros(len(AUG_PARAMS), dtype=np.float32)
    rec[P["grey"]] = float(grey)
    rec[P["flip"]] = float(flip)
    return rec


@dataclass
class RawDenClsBatch:
    """A collated training batch before its pixel augmentation: uint8 crops [B,H,W,3],
    parameter records [B,16], point sets, density maps [B,1,h,w] (already cropped,
    downsampled and flipped on the host, as in the reference)."""
    imgs: torch.Tensor
    params: torch.Tensor
    points: tuple
    dmaps: torch.Tensor | None = None


def augment_den_cls(imgs: torch.Tensor, params: torch.Tensor):
    """(img1, img2) NCHW f32 from uint8 crops [B,H,W,3] resident on the GPU."""
    if imgs.dtype != torch.uint8 or imgs.dim() != 4 or imgs.shape[3] != 3:
        raise ValueError("imgs must be uint8 [B, H, W, 3]")
    B, H, W, _ = imgs.shape
    dev = imgs.device
    imgs = imgs.contiguous()
    params = params.to(device=dev, dtype=torch.float32).contiguous()
    img1 = torch.empty((B, 3, H, W), dtype=torch.float32, device=dev)
    img2 = torch.empty_like(img1)
    ws = query("dg_augment_workspace", B, H, W)
    work = torch.empty(ws, dtype=torch.uint8, device=dev)
    call("dg_augment_den_cls", ptr(imgs), B, H, W, ptr(params), ptr(img1), ptr(img2), ptr(work), ws, stream())
    return img1, img2


def block_map(dmaps: torch.Tensor) -> torch.Tensor:
    """bmap = (16x16 block sums of dmap > 0) (datasets/den_cls_dataset.py:62-63)."""
    B, _, h, w = dmaps.shape
    d = dmaps.float().contiguous()
    out = torch.empty((B, 1, h // 16, w // 16), dtype=torch.float32, device=d.device)
    call("dg_block_map", ptr(d), B, h, w, ptr(out), stream())
    return out


class DeviceAugment:
    """RawDenClsBatch -> the reference's collated batch (img1, img2, (points, dmaps, bmaps))
    with all pixel work on `device`."""

    def __init__(self, device):
        self.device = torch.device(device)

    def __call__(self, raw: RawDenClsBatch):
        imgs = raw.imgs.to(self.device, non_blocking=True)
        img1, img2 = augment_den_cls(imgs, raw.params)
        dmaps = raw.dmaps.to(self.device, non_blocking=True)
        bmaps = block_map(dmaps)
        return img1, img2, (tuple(p.to(self.device) for p in raw.points), dmaps, bmaps)


__all__ = ["AUG_PARAMS", "RawDenClsBatch", "DeviceAugment", "augment_den_cls", "block_map", "draw_more_transform",
           "new_record", "hue_shift", "gaussian_weights"]
_ = K  # the kernels module loads the library (fails loudly when it is missing)
