"""DGTrainer — drop-in for reference trainers/dgtrainer.py (the boundary named
by BASELINE.json north_star).

`train_step(model, loss, optimizer, batch, epoch) -> float` keeps the
reference's modes (simple/base/add/cls/final/isw, dgtrainer.py:143-209), batch
layout `(imgs1, imgs2, (points, dmaps, bmaps))` (datasets/den_cls_dataset.py:17-24)
and loss composition.  The MSE count loss runs as one fused HIP pass; the model
forward/backward run on the HIP plans; `optimizer` may be torch's AdamW or the
fused `dgvcc_amd.optim.AdamW` (which also all-reduces gradients under DDP).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn as nn

from ..losses import mse_loss
from ..losses.bce import binary_cross_entropy
from ..utils.misc import denormalize, divide_img_into_patches
from .trainer import Trainer


class DGTrainer(Trainer):
    def __init__(self, seed, version, device, log_para, patch_size, mode):
        super().__init__(seed, version, device)
        self.log_para = log_para
        self.patch_size = patch_size
        self.mode = mode

    # checkpoint I/O for a [generator, regressor] model pair (dgtrainer.py:35-48)
    def load_ckpt(self, model, path):
        if isinstance(model, list):
            if path is not None:
                super().load_ckpt(model[0], path[0])
                super().load_ckpt(model[1], path[1])
        else:
            super().load_ckpt(model, path)

    def save_ckpt(self, model, path):
        if isinstance(model, list):
            super().save_ckpt(model[0], path.replace(".pth", "_gen.pth"))
            super().save_ckpt(model[1], path.replace(".pth", "_reg.pth"))
        else:
            super().save_ckpt(model, path)

    def compute_count_loss(self, loss: nn.Module, pred_dmaps, gt_datas, weights=None):
        name = loss.__class__.__name__
        if name == "MSELoss":
            _, gt_dmaps, _ = gt_datas
            gt_dmaps = gt_dmaps.to(self.device, non_blocking=True)
            if weights is not None:
                pred_dmaps = pred_dmaps * weights
                gt_dmaps = gt_dmaps * weights
            return mse_loss(pred_dmaps, gt_dmaps, self.log_para)
        if name == "BL":
            gts, targs, st_sizes = gt_datas
            gts = [g.to(self.device) for g in gts]
            targs = [t.to(self.device) for t in targs]
            st_sizes = st_sizes.to(self.device)
            return loss(gts, st_sizes, targs, pred_dmaps)
        raise ValueError(f"Unknown loss: {loss}")

    def _pred(self, model, x):
        return model(x) if self.mode == "base" else model(x)[0]

    def predict(self, model, img):
        """Patch-tiled count prediction (dgtrainer.py:71-84)."""
        h, w = img.shape[2:]
        ps = self.patch_size
        if h >= ps or w >= ps:
            patches, _, _ = divide_img_into_patches(img, ps)
            return self._count([self._pred(model, p).sum() for p in patches])
        return self._pred(model, img).sum().item() / self.log_para

    def _count(self, sums):
        """The reference adds `torch.sum(pred).item() / log_para` per patch in Python
        floats; same arithmetic and order here, with one device->host copy instead of one
        synchronising .item() per patch."""
        total = 0
        for s in torch.stack(sums).cpu().tolist():
            total += s / self.log_para
        return total

    def predict2(self, model, img, img2):
        """predict + ISW covariance statistics pass (dgtrainer.py:86-102)."""
        h, w = img.shape[2:]
        ps = self.patch_size
        if h >= ps or w >= ps:
            p1, _, _ = divide_img_into_patches(img, ps)
            p2, _, _ = divide_img_into_patches(img2, ps)
            sums = []
            for a, b in zip(p1, p2):
                sums.append(self._pred(model, a).sum())
                model([a, b], cal_covstat=True)
            return self._count(sums)
        cnt = self._pred(model, img).sum().item() / self.log_para
        model([img, img2], cal_covstat=True)
        return cnt

    def prepare_batch(self, batch):
        """A `DenClsDataset.collate` RawDenClsBatch -> the reference's batch layout, with the
        pixel augmentation run on this trainer's device; reference-layout batches pass through."""
        from ..datasets.augment import DeviceAugment, RawDenClsBatch
        if isinstance(batch, RawDenClsBatch):
            return DeviceAugment(self.device)(batch)
        return batch

    def train_step(self, model, loss, optimizer, batch, epoch):
        imgs1, imgs2, gt_datas = self.prepare_batch(batch)
        imgs1 = imgs1.to(self.device, non_blocking=True)
        imgs2 = imgs2.to(self.device, non_blocking=True)
        gt_cmaps = gt_datas[-1].to(self.device, non_blocking=True)
        count_loss = self.compute_count_loss

        if self.mode == "simple":
            optimizer.zero_grad()
            loss_total = count_loss(loss, model(imgs1), gt_datas)
        elif self.mode == "base":
            optimizer.zero_grad()
            d1 = model(imgs1)
            d2 = model(imgs2)
            loss_total = count_loss(loss, d1, gt_datas) + count_loss(loss, d2, gt_datas)
        elif self.mode == "add":
            optimizer.zero_grad()
            d1, d2, loss_con = model.forward_train(imgs1, imgs2)
            loss_total = count_loss(loss, d1, gt_datas) + count_loss(loss, d2, gt_datas) + loss_con
        elif self.mode == "cls":
            optimizer.zero_grad()
            d1, c1 = model(imgs1, gt_cmaps)
            d2, c2 = model(imgs2, gt_cmaps)
            loss_den = count_loss(loss, d1, gt_datas) + count_loss(loss, d2, gt_datas)
            loss_cls = binary_cross_entropy(c1, gt_cmaps) + binary_cross_entropy(c2, gt_cmaps)
            loss_total = loss_den + 10 * loss_cls
        elif self.mode == "final":
            optimizer.zero_grad()
            d1, d2, c1, c2, _cerr, loss_con, _lerr = model.forward_train(imgs1, imgs2, gt_cmaps)
            loss_den = count_loss(loss, d1, gt_datas) + count_loss(loss, d2, gt_datas)
            loss_cls = binary_cross_entropy(c1, gt_cmaps) + binary_cross_entropy(c2, gt_cmaps)
            loss_total = loss_den + 10 * loss_cls + 10 * loss_con
        elif self.mode == "isw":
            optimizer.zero_grad()
            gts = gt_datas[1].to(self.device)
            losses = model(imgs1, gts=gts, apply_wtloss=(epoch > 5))
            loss_total = torch.zeros(1, device=self.device) + losses[0]
            if epoch > 5:
                loss_total = loss_total + 0.6 * losses[1]
        else:
            raise ValueError(f"Unknown mode: {self.mode}")
        scaler = self._scaler(model, optimizer)
        if scaler is None:
            loss_total.backward()
            optimizer.step()
        else:  # fp16 mode: scaled backward, unscaled (or skipped) update
            (loss_total * scaler.scale).backward()
            self._scaled_step(optimizer, scaler.scale)
            scaler.update(getattr(optimizer, "found_inf", False))
        return loss_total.detach().item()

    def _scaler(self, model, optimizer):
        models = model if isinstance(model, (list, tuple)) else [model]
        if not any(getattr(m, "precision", None) == "fp16" for m in models):
            return None
        if getattr(self, "loss_scaler", None) is None:
            from ..optim import LossScaler
            self.loss_scaler = LossScaler()
        return self.loss_scaler

    @staticmethod
    def _scaled_step(optimizer, scale):
        from ..optim import AdamW
        if isinstance(optimizer, AdamW):
            optimizer.grad_scale = scale
            optimizer.step()
            optimizer.grad_scale = None
            return
        grads = [p.grad for g in optimizer.param_groups for p in g["params"] if p.grad is not None]
        inf = any(not torch.isfinite(gr).all() for gr in grads)
        optimizer.found_inf = inf
        if not inf:
            for gr in grads:
                gr.div_(scale)
            optimizer.step()

    def _val_batch(self, batch):
        """DenClsDataset val/test samples collated with batch size 1 carry the uint8 image and
        the parameter record: run their pixel transforms on the device."""
        img = batch[0]
        if isinstance(img, torch.Tensor) and img.dtype == torch.uint8:
            from ..datasets.augment import augment_den_cls
            img1, img2 = augment_den_cls(img.to(self.device), batch[1])
            return (img1, img2, *batch[2:])
        return batch

    def val_step(self, model, batch):
        img1, img2, gt, _, _ = self._val_batch(batch)
        img1 = img1.to(self.device)
        img2 = img2.to(self.device)
        if self.mode == "isw":
            with torch.no_grad():
                pred = self.predict2(model, img1, img2)
        else:
            pred = self.predict(model, img1)
        n = gt.shape[1]
        return np.abs(pred - n), {"mse": (pred - n) ** 2}

    def test_step(self, model, batch):
        img1, _, gt, _, _ = self._val_batch(batch)
        pred = self.predict(model, img1.to(self.device))
        n = gt.shape[1]
        return {"mae": np.abs(pred - n), "mse": (pred - n) ** 2}

    def vis_step(self, model, batch):
        """Saves density (and class) maps next to the image (dgtrainer.py:239-299)."""
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        img1, img2, gt, name, _ = batch
        out_dir = os.path.join(self.log_dir, "vis")
        os.makedirs(out_dir, exist_ok=True)
        panels = []
        for img in (img1, img2):
            img = img.to(self.device)
            res = model(img)
            d = res if self.mode == "base" else res[0]
            dm = d[0, 0].float().cpu().numpy()
            panels.append((denormalize(img.detach())[0].cpu().permute(1, 2, 0).numpy(), dm))
        fig = plt.figure(figsize=(10, 6))
        titles = [name[0], f"Pred1: {panels[0][1].sum() / self.log_para}", f"GT: {gt.shape[1]}",
                  f"Pred2: {panels[1][1].sum() / self.log_para}"]
        for i, data in enumerate([panels[0][0], panels[0][1], panels[1][0], panels[1][1]]):
            ax = fig.add_subplot(2, 2, i + 1)
            ax.set_title(titles[i])
            ax.imshow(data)
        plt.savefig(os.path.join(out_dir, f"{name[0]}.png"))
        plt.close(fig)
