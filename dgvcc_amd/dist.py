"""Data-parallel plumbing: frames shard over ranks; the only
exchange is one all-reduce of the flat fp32 gradient per step (RCCL over xGMI
with backend "nccl" on ROCm; gloo on CPU for tests)."""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def init_from_env(backend: str | None = None) -> int:
    """Initialise from torchrun's env (RANK/WORLD_SIZE/MASTER_*); returns local rank."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return local


def average_flat_(flat: torch.Tensor) -> torch.Tensor:
    """In-place mean over ranks of one flat gradient buffer (single collective)."""
    n = world()
    if n > 1:
        dist.all_reduce(flat)
        flat.div_(n)
    return flat


def broadcast_module_(module: torch.nn.Module, src: int = 0) -> None:
    """Identical initial weights/buffers on every rank."""
    if world() > 1:
        for t in module.state_dict().values():
            dist.broadcast(t, src)


def sum_moments(n_local: int):
    """Reducer for SyncSwitchWhiten2d (models/SW/ops/sync_switchwhiten.py:13-56):
    t -> (t summed over ranks, n_local * world).  Like the reference's SyncMeanCov it
    assumes every rank holds the same number of images."""
    def reduce(t: torch.Tensor):
        n = world()
        if n > 1:
            dist.all_reduce(t)
        return t, n_local * n
    return reduce


class OverlapReducer:
    """Bucketed data-parallel gradient all-reduce overlapped with the backward.

    The encoder/decoder FeaturePlan owns ~95% of a DGModel's parameters and runs its backward
    layer by layer (decoder first, then enc3 .. enc1).  With this reducer attached
    (dgvcc_amd.optim.AdamW(..., overlap=True), active from the optimizer's second step, once its
    flat gradient buffer exists), every FeaturePlan layer hands its parameter gradients to
    `emit` instead of returning them to autograd: they are summed straight into their slices of
    the optimizer's flat gradient buffer (p.grad becomes that slice), and as soon as the last
    FeaturePlan backward of the step (one per view: two in final mode) has delivered every
    parameter of a bucket, the bucket's contiguous slice is all-reduced asynchronously (RCCL on
    its own stream, so it runs under the remaining layers' backward kernels).  The optimizer step
    then waits for the buckets, averages them, and all-reduces only the parameters outside the
    FeaturePlan (the heads, the memory) as before.  Buckets are contiguous in the flat buffer
    and ~`bucket_mb` MB, so the all-reduces are few, large and ring-friendly over xGMI.

    One optimizer step = every taped FeaturePlan forward of the step followed by its backward:
    gradient accumulation over micro-batches (several backwards per step) is not supported with
    overlap=True, and a delivery into a bucket whose all-reduce is already in flight raises
    before anything is written (it would race RCCL on that slice)."""

    def __init__(self, bucket_mb: float = 32.0):
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.flat = None
        self.slot = {}       # param -> (start, end) element range in the flat buffer
        self.bucket_of = {}  # param -> bucket index
        self.buckets = []    # [start, end, n_params]
        self.handles = []
        self.reset()

    def attach(self, flat: torch.Tensor, params, offs, owned) -> None:
        """flat: the optimizer's flat gradient buffer; params / offs its layout; owned: the
        FeaturePlan parameters (their order in `params` defines the buckets)."""
        self.flat = flat
        owned = set(owned)
        self.slot = {p: (offs[i], offs[i] + p.numel()) for i, p in enumerate(params) if p in owned}
        self.buckets, self.bucket_of = [], {}
        cur = None
        for i, p in enumerate(params):
            if p not in owned:
                cur = None  # buckets never straddle a parameter outside the plan
                continue
            a, b = self.slot[p]
            if cur is None or 4 * (b - self.buckets[cur][0]) > self.bucket_bytes:
                self.buckets.append([a, b, 0])
                cur = len(self.buckets) - 1
            self.buckets[cur][1] = b
            self.buckets[cur][2] += 1
            self.bucket_of[p] = cur
        self.reset()

    def reset(self) -> None:
        self.nfwd = 0
        self.count = {}
        self.left = [bk[2] for bk in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.handles = []

    @property
    def active(self) -> bool:
        return self.flat is not None and world() > 1

    def forward_seen(self) -> None:
        self.nfwd += 1

    def emit(self, grads: dict) -> dict:
        """Take the owned parameters' gradients of one layer; return the rest for autograd."""
        if not self.active or self.nfwd == 0:
            return grads
        # every owned parameter is checked before any is written: a late failure must
        # not leave earlier parameters of this call summed into the buffer or a bucket in flight
        for p in grads:
            if p in self.slot and (self.launched[self.bucket_of[p]] or self.count.get(p, 0) >= self.nfwd):
                raise RuntimeError("OverlapReducer: more FeaturePlan backwards than taped forwards this step "
                                   "(gradient accumulation is not supported with overlap=True)")
        rest = {}
        for p, g in grads.items():
            sl = self.slot.get(p)
            if sl is None:
                rest[p] = g
                continue
            view = self.flat[sl[0]:sl[1]]
            k = self.count.get(p, 0)
            b = self.bucket_of[p]
            if k == 0:
                view.copy_(g.reshape(-1))
                if p.grad is None or p.grad.data_ptr() != view.data_ptr():
                    p.grad = view.view_as(p)
            else:
                view.add_(g.reshape(-1))
            self.count[p] = k + 1
            if k + 1 == self.nfwd:
                self.left[b] -= 1
                if self.left[b] == 0:
                    a, e, _ = self.buckets[b]
                    self.launched[b] = True
                    self.handles.append((a, e, dist.all_reduce(self.flat[a:e], async_op=True)))
        return rest

    def detach(self) -> None:
        """The optimizer re-created its flat buffer: settle what is in flight on the old one (its
        slices, which p.grad views, then hold rank averages) and forget it until re-attached."""
        for a, e, h in self.handles:
            h.wait()
            self.flat[a:e].div_(world())
        self.flat = None
        self.reset()

    def finish(self) -> bool:
        """Wait for the buckets and average them.  False when no FeaturePlan ran this step (its
        parameters' gradients then took the ordinary path and the caller reduces everything)."""
        used = self.nfwd > 0
        for a, e, h in self.handles:
            h.wait()
            self.flat[a:e].div_(world())
        complete = all(v == 0 for v in self.left)
        self.reset()
        if used and not complete:
            raise RuntimeError("OverlapReducer: a FeaturePlan backward did not deliver every parameter")
        return used
