"""Fused AdamW over one flat fp32 buffer (torch.optim.AdamW semantics,
reference main.py:85-86), with the data-parallel gradient all-reduce folded in.

At construction every parameter's storage is moved into a flat buffer per
param group (`p.data` becomes a view), so one HIP launch updates the whole
model.  Gradients are gathered into a flat buffer by one launch
(`dg_gather_flat`); when torch.distributed is initialised that buffer is
all-reduced (RCCL over xGMI, one collective per step) and averaged before the
update — the only collective on the hot path.
"""
from __future__ import annotations

import torch

from . import kernels as K
from .dist import average_flat_
from ._capi import call, ptr, stream


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 amsgrad=False, allreduce=True):
        if amsgrad:
            raise ValueError("amsgrad is not supported by the fused AdamW")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.allreduce = allreduce
        for group in self.param_groups:
            ps = group["params"]
            dev = ps[0].device
            if any(p.dtype != torch.float32 or p.device != dev for p in ps):
                raise ValueError("fused AdamW needs fp32 params on one device")
            sizes = [p.numel() for p in ps]
            total = sum(sizes)
            flat = torch.empty(total, dtype=torch.float32, device=dev)
            offs = [0]
            for p, n in zip(ps, sizes):
                flat[offs[-1]:offs[-1] + n].copy_(p.detach().reshape(-1))
                offs.append(offs[-1] + n)
            for p, o, n in zip(ps, offs, sizes):
                p.data = flat[o:o + n].view_as(p)
            group["_flat"] = flat
            group["_offs"] = offs
            group["_m"] = torch.zeros_like(flat)
            group["_v"] = torch.zeros_like(flat)
            group["_g"] = torch.empty_like(flat)
            group["_step"] = 0
            group["_offs_dev"] = torch.tensor(offs, dtype=torch.int64, device=dev)

    def _gather(self, group):
        ps = group["params"]
        g = group["_g"]
        if all(p.grad is not None for p in ps):
            for p in ps:
                if not p.grad.is_contiguous() or p.grad.dtype != torch.float32:
                    p.grad = p.grad.contiguous().float()
            table = torch.tensor([p.grad.data_ptr() for p in ps], dtype=torch.int64).to(g.device)
            call("dg_gather_flat", ptr(table), ptr(group["_offs_dev"]), len(ps), g.numel(), ptr(g),
                 stream())
            group["_table"] = table  # keep alive until the launch retires
            return True
        for p, o in zip(ps, group["_offs"]):
            if p.grad is None:
                g[o:o + p.numel()].zero_()
            else:
                g[o:o + p.numel()].copy_(p.grad.reshape(-1))
        return True

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            if all(p.grad is None for p in group["params"]):
                continue
            self._gather(group)
            g = group["_g"]
            if self.allreduce:
                average_flat_(g)
            group["_step"] += 1
            b1, b2 = group["betas"]
            K.adamw_step(group["_flat"], g, group["_m"], group["_v"], group["lr"], b1, b2,
                         group["eps"], group["weight_decay"], group["_step"])
        return loss

    def zero_grad(self, set_to_none: bool = True):
        super().zero_grad(set_to_none=set_to_none)
