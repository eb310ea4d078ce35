"""Trainer base — contract of reference trainers/trainer.py:21-179 (seeding, log
dir `logs/<version>/`, checkpoint I/O with identical state_dict keys, the epoch
loop that calls `train_step` once per batch and the scheduler once per epoch)."""
from __future__ import annotations

import os
import time
from glob import glob

import torch
import torch.nn as nn

from ..utils.misc import AverageMeter, DictAvgMeter, easy_track, get_current_datetime, seed_everything


class Trainer:
    def __init__(self, seed, version, device):
        self.seed = seed
        self.version = version
        self.device = torch.device(device)
        seed_everything(self.seed)
        # seed_everything turns on deterministic algorithms (as the reference);
        # the HIP kernels overwrite every byte they allocate, so skip torch's
        # NaN-fill of torch.empty() (one extra HBM pass per allocation).
        torch.utils.deterministic.fill_uninitialized_memory = False
        self.log_dir = os.path.join("logs", self.version)
        os.makedirs(self.log_dir, exist_ok=True)

    @staticmethod
    def is_main() -> bool:
        """Rank 0 (or a single process): the one that prints, logs and writes checkpoints."""
        from ..dist import rank
        return rank() == 0

    def log(self, msg, verbose=True, **kwargs):
        if not self.is_main():
            return
        if verbose:
            print(msg, **kwargs)
        with open(os.path.join(self.log_dir, "log.txt"), "a") as f:
            f.write(msg + kwargs.get("end", "\n"))

    def load_ckpt(self, model, path):
        if path is not None:
            self.log(f"Loading checkpoint from {path}")
            sd = torch.load(path, map_location=self.device, weights_only=True)
            model.load_state_dict(sd, strict=False)

    def save_ckpt(self, model, path):
        if self.is_main():
            torch.save(model.state_dict(), path)

    def _remove(self, pattern):
        if self.is_main():
            for f in glob(os.path.join(self.log_dir, pattern)):
                os.remove(f)

    @staticmethod
    def _each(model):
        return [model] if isinstance(model, nn.Module) else list(model)

    def set_model_train(self, model):
        for m in self._each(model):
            m.train()

    def set_model_eval(self, model):
        for m in self._each(model):
            m.eval()

    def train_step(self, model, loss, optimizer, batch, epoch):
        raise NotImplementedError

    def val_step(self, model, batch):
        raise NotImplementedError

    def test_step(self, model, batch):
        raise NotImplementedError

    def vis_step(self, model, batch):
        raise NotImplementedError

    def train_epoch(self, model, loss, train_dataloader, val_dataloader, optimizer, scheduler, epoch,
                    best_criterion, best_epoch):
        t0 = time.time()
        self.set_model_train(model)
        sampler = getattr(train_dataloader, "sampler", None)
        if hasattr(sampler, "set_epoch"):  # DistributedSampler: a new shard order per epoch
            sampler.set_epoch(epoch)
        train_loss = float("nan")
        for batch in easy_track(train_dataloader, description=f"Epoch {epoch}: Training..."):
            train_loss = self.train_step(model, loss, optimizer, batch, epoch)
        for s in (scheduler if isinstance(scheduler, list) else [scheduler]):
            if s is not None:
                s.step()  # once per epoch, as the reference (trainers/trainer.py:82-87)
        self.log(f"Epoch {epoch}: Training loss: {train_loss:.4f} Version: {self.version}")

        self.set_model_eval(model)
        crit, extra = AverageMeter(), DictAvgMeter()
        for batch in easy_track(val_dataloader, description=f"Epoch {epoch}: Validating..."):
            with torch.no_grad():
                c, add = self.val_step(model, batch)
            crit.update(c, add["n"]) if "n" in add else crit.update(c)
            extra.update(add)
        cur = crit.avg
        self.log(f"Epoch {epoch}: Val criterion: {cur:.4f}", end=" ")
        for k, v in extra.avg.items():
            self.log(f"{k}: {v:.4f}", end=" ")
        self.log(f"best: {best_criterion:.4f}, time: {time.time() - t0:.4f}")

        self._remove("last*.pth")
        self.save_ckpt(model, os.path.join(self.log_dir, "last.pth"))
        if cur < best_criterion:
            best_criterion, best_epoch = cur, epoch
            self.log(f"Epoch {epoch}: saving best model...")
            self._remove("best*.pth")
            self.save_ckpt(model, os.path.join(self.log_dir, f"best_{best_epoch}_{best_criterion:.4f}.pth"))
        return best_criterion, best_epoch

    def train(self, model, loss, train_dataloader, val_dataloader, optimizer, scheduler, checkpoint=None,
              num_epochs=100):
        self.log(f"Start training at {get_current_datetime()}")
        self.load_ckpt(model, checkpoint)
        model = model.to(self.device) if isinstance(model, nn.Module) else [m.to(self.device) for m in model]
        from ..dist import broadcast_module_
        for m in self._each(model):
            broadcast_module_(m)  # identical initial weights on every rank (no-op for one process)
        loss = loss.to(self.device)
        best_criterion, best_epoch = 1e10, -1
        for epoch in range(num_epochs):
            best_criterion, best_epoch = self.train_epoch(model, loss, train_dataloader, val_dataloader,
                                                          optimizer, scheduler, epoch, best_criterion,
                                                          best_epoch)
        self.log(f"Best epoch: {best_epoch}, best criterion: {best_criterion}")
        self.log(f"Training results saved to {self.log_dir}")
        self.log(f"End training at {get_current_datetime()}")

    def test(self, model, test_dataloader, checkpoint=None):
        self.log(f"Start testing at {get_current_datetime()}")
        self.load_ckpt(model, checkpoint)
        model = model.to(self.device) if isinstance(model, nn.Module) else [m.to(self.device) for m in model]
        self.set_model_eval(model)
        res = DictAvgMeter()
        for batch in easy_track(test_dataloader, description="Testing..."):
            with torch.no_grad():
                res.update(self.test_step(model, batch))
        self.log("Testing results:", end=" ")
        for k, v in res.avg.items():
            self.log(f"{k}: {v:.4f}", end=" ")
        self.log("")
        mae = res.avg["mae"]
        thr = 15.5 if self.version.startswith("sta") else 105  # reference trainer.py:154-160
        if mae < thr:
            self.log("Saving test model...")
            self.save_ckpt(model, os.path.join(self.log_dir, f"test_{mae}.pth"))
        self.log(f"Testing results saved to {self.log_dir}")
        self.log(f"End testing at {get_current_datetime()}")

    def vis(self, model, test_dataloader, checkpoint=None):
        self.load_ckpt(model, checkpoint)
        os.makedirs(os.path.join(self.log_dir, "vis"), exist_ok=True)
        model = model.to(self.device) if isinstance(model, nn.Module) else [m.to(self.device) for m in model]
        self.set_model_eval(model)
        for batch in easy_track(test_dataloader, description="Visualizing..."):
            with torch.no_grad():
                self.vis_step(model, batch)
