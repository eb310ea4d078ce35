"""F.binary_cross_entropy (mean) on one fused HIP pass (trainers/dgtrainer.py:178,188)."""
from __future__ import annotations

import torch

from .._capi import call, ptr, query, stream


class _BCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target):
        p = pred.float().contiguous()
        t = target.float().contiguous()
        n = p.numel()
        loss = torch.empty((), dtype=torch.float32, device=p.device)
        dp = torch.empty_like(p) if pred.requires_grad else None
        ws = query("dg_reduce_workspace", n)
        work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=p.device)
        call("dg_bce_loss", ptr(p), ptr(t), n, ptr(loss), ptr(dp), 1.0, ptr(work), stream())
        ctx.save_for_backward(dp if dp is not None else torch.empty(0))
        return loss

    @staticmethod
    def backward(ctx, g):
        (dp,) = ctx.saved_tensors
        return dp * g, None


def binary_cross_entropy(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    if pred.shape != target.shape:
        raise ValueError("pred/target shape mismatch")
    return _BCEFn.apply(pred, target)
