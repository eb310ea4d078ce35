"""Bayesian loss — drop-in for reference losses/bl.py (Post_Prob, Bay_Loss, BL).

`BL.forward(points, st_sizes, target_list, pre_density)` runs as four HIP passes
(dg_bl_loss): per-cell softmax statistics over the points (+ background), the
expected count of every point row, the trimmed per-image L1 (the reference's
variant: the smallest ceil(0.9*(n_rows-1)) residuals + the last row,
bl.py:75-78) and d loss / d density.  The [n+1, G^2] posterior is recomputed,
never stored.  `Post_Prob` materialises it (dg_bl_prob) for API parity.
"""
from __future__ import annotations

import numpy as np
import torch
from torch.nn import Module

from .._capi import call, ptr, query, stream


def _pack_points(points, device):
    counts = [int(p.shape[0]) for p in points]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(counts)]), dtype=torch.int64, device=device)
    total = int(sum(counts))
    if total:
        pts = torch.cat([p.to(device, torch.float32).reshape(-1, 2) for p in points]).contiguous()
    else:
        pts = torch.empty((0, 2), dtype=torch.float32, device=device)
    return pts, offs, total, counts


class _BLFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pre_density, pts, offs, total, st_sizes, targets, cfg):
        B = pre_density.shape[0]
        G = pre_density.shape[-1]
        dens = pre_density.float().contiguous()
        dev = dens.device
        ws = query("dg_bl_workspace", B, G, total)
        work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        ctx.save_for_backward(dens, pts, offs, st_sizes, targets)
        ctx.meta = (B, G, total, cfg)
        call("dg_bl_loss", ptr(pts) if total else None, ptr(offs), total, ptr(st_sizes),
             ptr(targets) if total else None, ptr(dens), B, G, cfg["stride"], cfg["sigma"], cfg["bg_ratio"],
             int(cfg["use_bg"]), ptr(loss), None, None, ptr(work), stream())
        return loss

    @staticmethod
    def backward(ctx, g):
        dens, pts, offs, st_sizes, targets = ctx.saved_tensors
        B, G, total, cfg = ctx.meta
        ws = query("dg_bl_workspace", B, G, total)
        work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=dens.device)
        loss = torch.empty((), dtype=torch.float32, device=dens.device)
        gd = torch.empty_like(dens)
        coef = g.float().reshape(1).contiguous()
        call("dg_bl_loss", ptr(pts) if total else None, ptr(offs), total, ptr(st_sizes),
             ptr(targets) if total else None, ptr(dens), B, G, cfg["stride"], cfg["sigma"], cfg["bg_ratio"],
             int(cfg["use_bg"]), ptr(loss), ptr(gd), ptr(coef), ptr(work), stream())
        return gd, None, None, None, None, None, None


class Post_Prob(Module):
    """Posterior of every grid cell over the annotated points (bl.py:5-52)."""

    def __init__(self, sigma, c_size, stride, background_ratio, use_background, device):
        super().__init__()
        assert c_size % stride == 0
        self.sigma = sigma
        self.bg_ratio = background_ratio
        self.device = device
        self.stride = stride
        self.G = c_size // stride
        self.use_bg = use_background

    def forward(self, points, st_sizes):
        dev = torch.device(self.device) if not isinstance(self.device, torch.device) else self.device
        pts, offs, total, counts = _pack_points(points, dev)
        B, G = len(points), self.G
        if total == 0:
            return [None] * B
        rows = [c + (1 if self.use_bg else 0) if c > 0 else 0 for c in counts]
        roff = torch.tensor(np.concatenate([[0], np.cumsum(rows)]), dtype=torch.int64, device=dev)
        prob = torch.empty((int(sum(rows)), G * G), dtype=torch.float32, device=dev)
        ws = query("dg_bl_workspace", B, G, total)
        work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=dev)
        st = torch.as_tensor(st_sizes, dtype=torch.float32, device=dev).contiguous()
        call("dg_bl_prob", ptr(pts), ptr(offs), total, ptr(st), B, G, float(self.stride), float(self.sigma),
             float(self.bg_ratio), int(self.use_bg), ptr(roff), ptr(prob), ptr(work), stream())
        out, r = [], 0
        for n in rows:
            out.append(prob[r:r + n] if n > 0 else None)
            r += n
        return out


class Bay_Loss(Module):
    """Trimmed expected-count L1 given explicit posteriors (bl.py:54-80)."""

    def __init__(self, use_background, device):
        super().__init__()
        self.device = device
        self.use_bg = use_background

    def forward(self, prob_list, target_list, pre_density):
        import math
        loss = 0
        for idx, prob in enumerate(prob_list):
            if prob is None or prob.shape[0] == 0:
                pre_count = torch.sum(pre_density[idx]).reshape(1)
                target = torch.zeros((1,), dtype=torch.float32, device=pre_density.device)
            else:
                N = len(prob)
                if self.use_bg:
                    target = torch.zeros((N,), dtype=torch.float32, device=pre_density.device)
                    target[:-1] = target_list[idx]
                else:
                    target = target_list[idx]
                pre_count = prob @ pre_density[idx].reshape(-1)
            res = torch.abs(target - pre_count)
            num = math.ceil(0.9 * (len(res) - 1))
            loss = loss + torch.sum(torch.topk(res[:-1], num, largest=False)[0]) + res[-1]
        return loss / len(prob_list)


class BL(Module):
    """Bayesian loss, fused on the GPU (bl.py:82-91)."""

    def __init__(self, sigma, c_size, stride, background_ratio, use_background, device):
        super().__init__()
        assert c_size % stride == 0
        self.post_prob = Post_Prob(sigma, c_size, stride, background_ratio, use_background, device)
        self.bay_loss = Bay_Loss(use_background, device)
        self.cfg = dict(stride=float(stride), sigma=float(sigma), bg_ratio=float(background_ratio),
                        use_bg=bool(use_background))
        self.G = c_size // stride

    def forward(self, points, st_sizes, target_list, pre_density):
        if pre_density.shape[-1] != self.G or pre_density.shape[-2] != self.G:
            raise ValueError(f"pre_density must be [B,1,{self.G},{self.G}] (square grid, bl.py:14-16)")
        if len(points) != pre_density.shape[0]:
            raise ValueError("one point set per image")
        dev = pre_density.device
        pts, offs, total, counts = _pack_points(points, dev)
        if total:
            tg = torch.cat([t.to(dev, torch.float32).reshape(-1) for t, c in zip(target_list, counts) if c > 0])
        else:
            tg = torch.empty((0,), dtype=torch.float32, device=dev)
        st = torch.as_tensor(st_sizes, dtype=torch.float32).to(dev).reshape(-1).contiguous()
        return _BLFn.apply(pre_density, pts, offs, total, st, tg.contiguous(), self.cfg)
