"""TEST INFRASTRUCTURE ONLY (the product never imports this): CPU restatement of the
reference's DenClsDataset pixel pipeline (datasets/den_cls_dataset.py:29-35, 77-158) for
one parameter record of the product's datasets/augment.py.

Pinning: the PIL steps call PIL itself (installed here, the library the reference runs):
convert('L'), ImageEnhance.Brightness/Contrast/Color/Sharpness, convert('HSV').  The
torchvision steps are restated from torchvision's published source because torchvision is
absent here and unpinned in the reference (no requirements file): ColorJitter.forward's
op order, F_pil.adjust_hue (uint8 hue shift with wrap-around), F_t.gaussian_blur (float32
kernel from _get_gaussian_kernel1d, reflect padding, depthwise conv2d, round, uint8),
ToTensor (x / 255) and Normalize((x - 0.5) / 0.5).  Parity for those is "restated, version
unpinned".
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F
from PIL import Image, ImageEnhance

P = {k: i for i, k in enumerate(("grey", "flip", "jitter", "order0", "order1", "order2", "order3", "brightness",
                                 "contrast", "saturation", "hue_shift", "blur", "k0", "k1", "sharp",
                                 "sharp_factor"))}


def to_tensor_normalize(u8: np.ndarray) -> torch.Tensor:
    """T.ToTensor() + T.Normalize([.5]*3, [.5]*3) on an HWC uint8 array -> CHW float32."""
    t = torch.from_numpy(np.ascontiguousarray(u8)).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    return t.sub(0.5).div(0.5)


def base_image(u8: np.ndarray, rec) -> np.ndarray:
    img = Image.fromarray(u8)
    if rec[P["grey"]]:
        img = img.convert("L").convert("RGB")
    a = np.asarray(img)
    if rec[P["flip"]]:
        a = a[:, ::-1]
    return np.ascontiguousarray(a)


def adjust_hue(img: Image.Image, shift: int) -> Image.Image:
    h, s, v = img.convert("HSV").split()
    np_h = np.array(h, dtype=np.uint8)
    with np.errstate(over="ignore"):
        np_h += np.uint8(shift)
    return Image.merge("HSV", (Image.fromarray(np_h, "L"), s, v)).convert("RGB")


def gaussian_blur(img: Image.Image, k0: float, k1: float) -> Image.Image:
    k1d = torch.tensor([k0, k1, k0], dtype=torch.float32)
    k2d = torch.mm(k1d[:, None], k1d[None, :]).expand(3, 1, 3, 3)
    t = torch.from_numpy(np.array(img)).permute(2, 0, 1).unsqueeze(0).to(torch.float32)
    t = F.pad(t, [1, 1, 1, 1], mode="reflect")
    t = F.conv2d(t, k2d, groups=3)
    t = torch.round(t).to(torch.uint8)[0].permute(1, 2, 0).numpy()
    return Image.fromarray(np.ascontiguousarray(t))


def more_transform(base: np.ndarray, rec) -> np.ndarray:
    """uint8 result of more_transform before ToTensor/Normalize."""
    img = Image.fromarray(base)
    if rec[P["jitter"]]:
        for k in range(4):
            op = int(rec[P["order0"] + k])
            if op == 0:
                img = ImageEnhance.Brightness(img).enhance(float(rec[P["brightness"]]))
            elif op == 1:
                img = ImageEnhance.Contrast(img).enhance(float(rec[P["contrast"]]))
            elif op == 2:
                img = ImageEnhance.Color(img).enhance(float(rec[P["saturation"]]))
            else:
                img = adjust_hue(img, int(rec[P["hue_shift"]]))
    if rec[P["blur"]]:
        img = gaussian_blur(img, float(rec[P["k0"]]), float(rec[P["k1"]]))
    if rec[P["sharp"]]:
        img = ImageEnhance.Sharpness(img).enhance(float(rec[P["sharp_factor"]]))
    return np.asarray(img)


def augment(u8: np.ndarray, rec):
    """(img1, img2) CHW float32 tensors and the two uint8 images."""
    base = base_image(u8, rec)
    v2 = more_transform(base, rec)
    return to_tensor_normalize(base), to_tensor_normalize(v2), base, v2
