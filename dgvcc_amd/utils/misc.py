"""Utilities with the reference's semantics (utils/misc.py)."""
from __future__ import annotations

import math
import os
import random
import time

import numpy as np
import torch


def random_crop(im_h, im_w, crop_h, crop_w):
    """utils/misc.py:12-17: top-left corner of a uniform random crop."""
    return random.randint(0, im_h - crop_h), random.randint(0, im_w - crop_w)


def get_padding(h, w, new_h, new_w):
    """utils/misc.py:19-37: symmetric padding (extra pixel bottom/right) up to new size."""
    def split(cur, new):
        if cur >= new:
            return 0, 0, cur
        d = new - cur
        return d // 2, d // 2 + d % 2, new
    top, bottom, h2 = split(h, new_h)
    left, right, w2 = split(w, new_w)
    return (left, top, right, bottom), h2, w2


def cal_inner_area(c_left, c_up, c_right, c_down, bbox):
    """utils/misc.py:39-45."""
    il = np.maximum(c_left, bbox[:, 0])
    iu = np.maximum(c_up, bbox[:, 1])
    ir = np.minimum(c_right, bbox[:, 2])
    idn = np.minimum(c_down, bbox[:, 3])
    return np.maximum(ir - il, 0.0) * np.maximum(idn - iu, 0.0)


def divide_img_into_patches(img, patch_size):
    """utils/misc.py:47-67: non-overlapping tiles, the last row/col take the remainder."""
    h, w = img.shape[-2:]
    nh, nw = math.ceil(h / patch_size), math.ceil(w / patch_size)
    patches = []
    for i in range(nh):
        h0, h1 = i * patch_size, (h if i == nh - 1 else (i + 1) * patch_size)
        for j in range(nw):
            w0, w1 = j * patch_size, (w if j == nw - 1 else (j + 1) * patch_size)
            patches.append(img[..., h0:h1, w0:w1])
    return patches, nh, nw


def denormalize(img_tensor):
    """Undo Normalize(mean=0.5, std=0.5) (utils/misc.py:69-79)."""
    shape = (3, 1, 1) if img_tensor.dim() == 3 else (1, 3, 1, 1)
    half = torch.full(shape, 0.5, device=img_tensor.device, dtype=img_tensor.dtype)
    return img_tensor * half + half


class AverageMeter:
    def __init__(self):
        self.reset()

    def reset(self):
        self.val = self.avg = self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


class DictAvgMeter:
    def __init__(self):
        self.reset()

    def reset(self):
        self.val, self.avg, self.sum, self.count = {}, {}, {}, {}

    def update(self, val, n=1):
        for k, v in val.items():
            self.sum[k] = self.sum.get(k, 0) + v * n
            self.count[k] = self.count.get(k, 0) + n
            self.val[k] = v
            self.avg[k] = self.sum[k] / self.count[k]


def seed_everything(seed):
    """utils/misc.py:124-132 (deterministic algorithms with warn_only)."""
    random.seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.deterministic = False


def seed_worker(worker_id):
    s = torch.initial_seed() % 2 ** 32
    np.random.seed(s)
    random.seed(s)


def get_seeded_generator(seed):
    """Quirk kept: the seed argument is ignored, always 0."""
    g = torch.Generator()
    g.manual_seed(0)
    return g


def get_current_datetime():
    return time.strftime("%Y-%m-%d %H:%M:%S", time.localtime())


def easy_track(iterable, description=None):
    try:
        from rich.progress import track
        return track(iterable, description=description, complete_style="dim cyan", total=len(iterable))
    except Exception:  # no rich / no len(): plain iteration
        return iterable
