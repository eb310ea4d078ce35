"""Fused AdamW over one flat fp32 buffer (torch.optim.AdamW semantics,
reference main.py:85-86), with the data-parallel gradient all-reduce folded in.

At the first step every parameter's storage is moved into a flat buffer per
param group (`p.data` becomes a view), so one HIP launch updates the whole
model.  Gradients are gathered into a flat buffer by one launch
(`dg_gather_flat`); when torch.distributed is initialised that buffer is
all-reduced (RCCL over xGMI, one collective per step) and averaged before the
update — the only collective on the hot path.
"""
from __future__ import annotations

import os

import torch

from . import engine as E
from . import kernels as K
from .dist import OverlapReducer, average_flat_, world
from .engine import invalidate_frozen
from ._capi import call, ptr, stream


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 amsgrad=False, allreduce=True, overlap=None, bucket_mb=32.0):
        if amsgrad:
            raise ValueError("amsgrad is not supported by the fused AdamW")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.allreduce = allreduce
        # overlap (default; DGVCC_DP_OVERLAP=0 or overlap=False: one blocking all-reduce of the flat
        # buffer after the backward): the FeaturePlan parameters' all-reduce runs in ~bucket_mb
        # buckets under the backward (dgvcc_amd.dist.OverlapReducer), from the second step on.  A
        # no-op on one rank.
        # One optimizer step per backward: with the overlap on, a second FeaturePlan backward before
        # step() (gradient accumulation over micro-batches) raises (dist.OverlapReducer: its buckets
        # are already in flight); accumulate with overlap=False / DGVCC_DP_OVERLAP=0.
        if overlap is None:
            overlap = os.environ.get("DGVCC_DP_OVERLAP", "1") == "1"
        self.reducer = OverlapReducer(bucket_mb) if (overlap and allreduce) else None
        # bench.py: a list receives per step and group two (start, end) HIP event pairs on the compute
        # stream around the gradient all-reduce's exposed parts -- the wait for the in-flight buckets,
        # and the blocking all-reduce of the remainder (the gather launch between them excluded);
        # None (default) records nothing
        self.comm_events = None
        # fp16 mode: the loss was multiplied by grad_scale before backward (LossScaler); the
        # step unscales the flat gradient and skips the update when it holds inf/NaN
        self.grad_scale = None
        self.found_inf = False
        for group in self.param_groups:
            ps = group["params"]
            if any(p.dtype != torch.float32 or p.device != ps[0].device for p in ps):
                raise ValueError("fused AdamW needs fp32 params on one device")

    @staticmethod
    def _is_flat(group):
        flat = group.get("_flat")
        if flat is None:
            return False
        base = flat.data_ptr()
        return all(p.device == flat.device and p.data_ptr() == base + 4 * o
                   for p, o in zip(group["params"], group["_offs"]))

    def _ensure_flat(self, group):
        """Move every parameter's storage into one flat buffer per group (`p.data` becomes a
        view).  Done at the first step, and again if the parameters were re-homed since
        (`model.to(device)` after the optimizer was built, as the reference's main.py
        does); the moments follow the parameters."""
        if self._is_flat(group):
            return
        ps = group["params"]
        dev = ps[0].device
        if any(p.dtype != torch.float32 or p.device != dev for p in ps):
            raise ValueError("fused AdamW needs fp32 params on one device")
        sizes = [p.numel() for p in ps]
        flat = torch.empty(sum(sizes), dtype=torch.float32, device=dev)
        offs = [0]
        for p, n in zip(ps, sizes):
            flat[offs[-1]:offs[-1] + n].copy_(p.detach().reshape(-1))
            offs.append(offs[-1] + n)
        for p, o, n in zip(ps, offs, sizes):
            p.data = flat[o:o + n].view_as(p)
        group["_flat"] = flat
        group["_offs"] = offs
        group["_m"] = group["_m"].to(dev) if "_m" in group else torch.zeros_like(flat)
        group["_v"] = group["_v"].to(dev) if "_v" in group else torch.zeros_like(flat)
        group["_g"] = torch.empty_like(flat)
        # per-parameter step counts, as torch.optim.AdamW's per-parameter state["step"]: a
        # parameter whose .grad is None on a step is skipped and its count does not advance
        steps = group.get("_steps")
        group["_steps"] = list(steps) if steps is not None and len(steps) == len(ps) else [0] * len(ps)
        group.pop("_live_cache", None)

    def _gather(self, group):
        """Gather live gradients into the flat buffer; returns the [i0, i1) parameter-index runs
        of parameters that have a gradient (torch.optim.AdamW skips params whose .grad
        is None: no decay, no moment update — e.g. the ISW counter's unused layer4)."""
        ps = group["params"]
        g = group["_g"]
        live = tuple(p.grad is not None for p in ps)
        for p in ps:
            if p.grad is not None and (not p.grad.is_contiguous() or p.grad.dtype != torch.float32):
                p.grad = p.grad.contiguous().float()
        cache = group.get("_live_cache")
        if cache is None or cache[0] != live:
            runs, start = [], None  # maximal runs [i0, i1) of consecutive live params
            for i, l in enumerate(live + (False,)):
                if l and start is None:
                    start = i
                elif not l and start is not None:
                    runs.append((start, i))
                    start = None
            offs = group["_offs"]
            dev_offs = [torch.tensor(offs[i0:i1] + [offs[i1 - 1] + ps[i1 - 1].numel()], dtype=torch.int64,
                                     device=g.device) for i0, i1 in runs]
            cache = (live, runs, dev_offs)
            group["_live_cache"] = cache
            offs = group["_offs"]
            for i, l in enumerate(live):  # dead regions stay zero (the all-reduce sums them harmlessly)
                if not l and ps[i].numel():
                    g[offs[i]:offs[i] + ps[i].numel()].zero_()
        _, runs, dev_offs = cache
        tables = []
        for (i0, i1), o in zip(runs, dev_offs):
            # pinned host table, copied on the stream without a host stall (kept alive with the launch)
            host = torch.tensor([ps[i].grad.data_ptr() for i in range(i0, i1)], dtype=torch.int64,
                                pin_memory=g.is_cuda)
            table = host.to(g.device, non_blocking=True)
            call("dg_gather_flat", ptr(table), ptr(o), i1 - i0, g.numel(), ptr(g), stream())
            tables.append((host, table))
        group["_table"] = tables  # keep alive until the launches retire
        return runs

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        invalidate_frozen()  # the update below writes parameters behind torch's version counters
        self.found_inf = False
        staged = []
        for group in self.param_groups:
            if all(p.grad is None for p in group["params"]):
                continue
            self._ensure_flat(group)
            ev = None
            if self.comm_events is not None and world() > 1 and group["_g"].is_cuda:
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                ev[0].record()
            if self.reducer is not None and self.reducer.flat is not None and self.reducer.flat is not group["_g"]:
                # the flat buffer was re-created (re-homed parameters): drain the reducer and
                # re-attach it to the new buffer after this step (its sinks keep pointing at it)
                self.reducer.detach()
            red = self.reducer if (self.reducer is not None and self.reducer.active
                                   and self.reducer.flat is group["_g"]) else None
            if red is not None and not red.finish():  # the FeaturePlan buckets, reduced under the backward
                red = None
            if ev is not None:
                ev[1].record()
            runs = self._gather(group)
            if ev is not None:
                ev[2].record()
            g = group["_g"]
            if red is not None:
                offs, ps = group["_offs"], group["params"]
                i = 0
                while i < len(ps):  # the maximal runs of parameters outside the buckets
                    if ps[i] in red.slot:
                        i += 1
                        continue
                    j = i
                    while j < len(ps) and ps[j] not in red.slot:
                        j += 1
                    average_flat_(g[offs[i]:offs[j - 1] + ps[j - 1].numel()])
                    i = j
            elif self.allreduce:
                average_flat_(g)
            if ev is not None:
                ev[3].record()
                self.comm_events.append(((ev[0], ev[1]), (ev[2], ev[3])))
            if self.grad_scale is not None and self.grad_scale != 1.0:
                flag = group.setdefault("_inf", torch.zeros(1, dtype=torch.int32, device=g.device))
                call("dg_grad_unscale", ptr(g), g.numel(), 1.0 / float(self.grad_scale), ptr(flag), stream())
                if int(flag.item()):  # one device->host flag per group (the trainer syncs per step anyway)
                    self.found_inf = True
            staged.append((group, runs))
        if self.found_inf:  # GradScaler semantics: no update, no step count, for any group
            return loss
        for group, runs in staged:
            g = group["_g"]
            b1, b2 = group["betas"]
            flat, m, v = group["_flat"], group["_m"], group["_v"]
            for a, b, step in self._step_runs(group, runs):
                K.adamw_step(flat[a:b], g[a:b], m[a:b], v[a:b], group["lr"], b1, b2,
                             group["eps"], group["weight_decay"], step)
        if self.reducer is not None and world() > 1 and len(self.param_groups) == 1 and self.reducer.flat is None:
            group = self.param_groups[0]
            if "_g" in group:  # from the next step on: the sink of the FeaturePlan backward
                plans = E.feature_plans_of(group["params"])
                self.reducer.attach(group["_g"], group["params"], group["_offs"],
                                    [p for plan in plans for p in plan.params()])
                if self.reducer.buckets:
                    for plan in plans:
                        plan.sink = self.reducer
                else:  # no FeaturePlan parameters (the ResNet trunks): the ordinary path
                    self.reducer = None
        return loss

    @staticmethod
    def _step_runs(group, runs):
        """Advance the step count of every live parameter and split the live runs (parameter
        index ranges [i0, i1)) into maximal sub-runs of equal count: one launch per (element
        range, bias-correction step); a single launch when every parameter has always had a
        gradient.  Walking indices, not element offsets, keeps zero-numel parameters (which
        share their offset with the next parameter) attributed correctly."""
        offs, steps = group["_offs"], group["_steps"]
        out = []
        for i0, i1 in runs:
            for i in range(i0, i1):
                steps[i] += 1
            j = i0
            while j < i1:
                k = j
                while k + 1 < i1 and steps[k + 1] == steps[j]:
                    k += 1
                if offs[k + 1] > offs[j]:
                    out.append((offs[j], offs[k + 1], steps[j]))
                j = k + 1
        return out

    def zero_grad(self, set_to_none: bool = True):
        super().zero_grad(set_to_none=set_to_none)


class LossScaler:
    """Dynamic loss scaling for the fp16 mode (torch.cuda.amp.GradScaler's defaults: init
    2^16, x2 after 2000 finite steps, x0.5 on an inf/NaN step).  Gradients of the density
    losses are ~1e-7 per element at 2048x2048 (MSE over 3.4e7 pixels): below fp16's normal
    range unless scaled."""

    def __init__(self, init_scale=65536.0, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000):
        self.scale = float(init_scale)
        self.growth_factor, self.backoff_factor = growth_factor, backoff_factor
        self.growth_interval = growth_interval
        self._good = 0

    def update(self, found_inf: bool):
        if found_inf:
            self.scale *= self.backoff_factor
            self._good = 0
        else:
            self._good += 1
            if self._good >= self.growth_interval:
                self.scale *= self.growth_factor
                self._good = 0
