"""Losses of the DGVCC hot path on HIP kernels."""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import kernels as K


class _MSEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, gt, gt_scale):
        loss, dpred = K.mse_loss(pred.float().contiguous(), gt.float().contiguous(), gt_scale,
                                 want_grad=pred.requires_grad)
        ctx.save_for_backward(dpred if dpred is not None else torch.empty(0))
        return loss

    @staticmethod
    def backward(ctx, g):
        (dpred,) = ctx.saved_tensors
        return dpred * g, None, None


def mse_loss(pred: torch.Tensor, gt: torch.Tensor, gt_scale: float = 1.0) -> torch.Tensor:
    """mean((pred - gt*gt_scale)^2): nn.MSELoss()(pred, gt*log_para)
    (trainers/dgtrainer.py:57) in one fused HIP pass (loss + d/dpred)."""
    if pred.shape != gt.shape:
        raise ValueError(f"shape mismatch {tuple(pred.shape)} vs {tuple(gt.shape)}")
    return _MSEFn.apply(pred, gt, float(gt_scale))


class MSELoss(nn.Module):
    """nn.MSELoss(reduction='mean') replacement; class name kept so
    DGTrainer.compute_count_loss dispatches on it like the reference."""

    def forward(self, pred, target):
        return mse_loss(pred, target, 1.0)
