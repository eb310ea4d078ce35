"""TEST INFRASTRUCTURE ONLY — numpy restatement of losses/bl.py (Post_Prob
:5-52, Bay_Loss :54-80, BL :82-91) in float32 with the reference's formula
order; returns the loss and d loss / d pre_density."""
from __future__ import annotations

import math

import numpy as np


def bl_loss(points_list, st_sizes, targets_list, dens, c_size, stride, sigma, bg_ratio, use_bg):
    f32 = np.float32
    G = c_size // stride
    cood = (np.arange(0, c_size, stride, dtype=f32) + f32(stride / 2)).astype(f32)
    B = dens.shape[0]
    loss = 0.0
    grad = np.zeros_like(dens, dtype=np.float64)
    for b in range(B):
        d = dens[b].reshape(-1).astype(f32)
        pts = np.asarray(points_list[b], dtype=f32).reshape(-1, 2)
        if len(pts) == 0:
            s = d.sum(dtype=np.float64)
            loss += abs(s)
            grad[b] += np.sign(s)
            continue
        x, y = pts[:, :1], pts[:, 1:]
        xd = (f32(-2) * (x * cood[None, :]) + x * x + cood[None, :] * cood[None, :]).astype(f32)
        yd = (f32(-2) * (y * cood[None, :]) + y * y + cood[None, :] * cood[None, :]).astype(f32)
        dis = (yd[:, :, None] + xd[:, None, :]).reshape(len(pts), -1).astype(f32)
        if use_bg:
            mn = np.maximum(dis.min(axis=0, keepdims=True), 0).astype(f32)
            bg = ((f32(st_sizes[b] * bg_ratio) - np.sqrt(mn)) ** 2).astype(f32)
            dis = np.concatenate([dis, bg], 0)
        lg = (-dis / f32(2.0 * sigma ** 2)).astype(np.float64)
        lg -= lg.max(axis=0, keepdims=True)
        prob = np.exp(lg)
        prob /= prob.sum(axis=0, keepdims=True)
        n = len(prob)
        tg = np.zeros(n)
        tg[: len(pts)] = np.asarray(targets_list[b], dtype=np.float64)
        pre = prob @ d.astype(np.float64)
        res = np.abs(tg - pre)
        num = math.ceil(0.9 * (len(res) - 1))
        order = np.argsort(res[:-1], kind="stable")[:num]
        loss += res[order].sum() + res[-1]
        w = np.zeros(n)
        w[order] = np.sign(pre[order] - tg[order])
        w[-1] = np.sign(pre[-1] - tg[-1])
        grad[b] += (w @ prob).reshape(dens[b].shape)
    return loss / B, grad / B
