"""Worker for test_dp_syncbn_strong_scaling (torch.distributed.run, 2 ranks sharing one GPU, gloo):
configs/jhu_fog2snow.yml's global batch strong-scaled over the ranks with SyncBatchNorm
(`nn.SyncBatchNorm.convert_sync_batchnorm`, dgvcc_amd/syncbn.py), so every BN layer normalises
with the statistics of the whole batch as the reference's single-device run does.  Each rank runs
the final-mode step on its half; the rank-averaged gradients, the loss average and the BN
running statistics must equal one process running the whole batch with plain BatchNorm.  Then
one real DGTrainer step with the fused AdamW (its flat-gradient all-reduce) leaves identical
parameters on both ranks.  Dropouts are off so both runs see the same masks."""
import os
import sys
import tempfile

import torch
import torch.distributed as dist
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import dg_oracle as O  # noqa: E402
from dgvcc_amd import dist as D  # noqa: E402
from dgvcc_amd.losses import MSELoss, mse_loss  # noqa: E402
from dgvcc_amd.losses.bce import binary_cross_entropy  # noqa: E402
from dgvcc_amd.models.models import DGModel_final  # noqa: E402
from dgvcc_amd.optim import AdamW  # noqa: E402
from dgvcc_amd.trainers.dgtrainer import DGTrainer  # noqa: E402

B, H, W = 4, 128, 128


def build(dev, sd0, sync):
    m = DGModel_final(pretrained=False, den_dropout=0.0, cls_dropout=0.0)
    m.load_state_dict(sd0)
    if sync:
        m = nn.SyncBatchNorm.convert_sync_batchnorm(m)
    return m.to(dev).set_precision("fp32").train()


def part(batch, r, world):
    i1, i2, (pts, dm, bm) = batch
    n = i1.shape[0] // world
    s = slice(r * n, (r + 1) * n)
    return i1[s], i2[s], (pts[s], dm[s], bm[s])


def step_grads(m, batch, dev):
    i1, i2, (pts, dm, bm) = batch
    i1, i2, dm, bm = i1.to(dev), i2.to(dev), dm.to(dev), bm.to(dev)
    for p in m.parameters():
        p.grad = None
    dc1, dc2, c1, c2, _, lcon, _ = m.forward_train(i1, i2, bm)
    loss = (mse_loss(dc1, dm, 1000.0) + mse_loss(dc2, dm, 1000.0)
            + 10 * (binary_cross_entropy(c1, bm) + binary_cross_entropy(c2, bm)) + 10 * lcon)
    loss.backward()
    return loss.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}


def main():
    D.init_from_env("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sd0 = O.seeded_state_dict(DGModel_final(pretrained=False).state_dict())
    batch = O.synthetic_batch(B, H, W, seed=2112)
    fails = []
    # strong-scaled data parallel with SyncBN: this rank's B / world samples
    m = build(dev, sd0, sync=True)
    assert sum(isinstance(x, nn.SyncBatchNorm) for x in m.modules()) == 21
    loss, grads = step_grads(m, part(batch, rank, world), dev)
    dist.all_reduce(loss)
    loss /= world
    for g in grads.values():
        dist.all_reduce(g)
        g /= world
    rstats = {k: v.detach().clone() for k, v in m.state_dict().items() if "running" in k}
    if rank == 0:
        ref = build(dev, sd0, sync=False)
        loss_ref, grads_ref = step_grads(ref, batch, dev)
        lr = abs(loss.item() - loss_ref.item()) / abs(loss_ref.item())
        if lr > 1e-5:
            fails.append(("loss", lr))
        worst = {}
        for k, r in grads_ref.items():
            if k.endswith(".bias") and (k.startswith("enc") or ".conv." in k):
                continue  # conv bias before BN: mathematically zero gradient
            if r.norm() == 0:
                continue
            worst[k] = ((grads[k].double() - r.double()).norm() / r.double().norm()).item()
        bad = {k: v for k, v in worst.items() if v > 1e-4}
        if bad:
            fails.append(("grads", bad))
        rs = max(((rstats[k].double() - v.double()).abs().max() / v.double().abs().max().clamp_min(1e-30)).item()
                 for k, v in ref.state_dict().items() if "running" in k)
        if rs > 1e-5:
            fails.append(("running stats", rs))
        print(f"RANK0 loss_rel={lr:.3e} worst_grad={max(worst.items(), key=lambda kv: kv[1])} running={rs:.3e}",
              flush=True)
    # one real trainer step (fused AdamW all-reduce) with SyncBN: parameters identical across ranks
    m2 = build(dev, sd0, sync=True)
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp())
    tr = DGTrainer(2112, f"sbn{rank}", dev, 1000, 10000, "final")
    i1, i2, (pts, dm, bm) = part(batch, rank, world)
    tr.train_step(m2, MSELoss(), AdamW(m2.parameters(), lr=1e-4, weight_decay=1e-4),
                  (i1.to(dev), i2.to(dev), (tuple(p.to(dev) for p in pts), dm.to(dev), bm.to(dev))), 0)
    os.chdir(cwd)
    chk = torch.stack([p.detach().double().sum() for p in m2.parameters()]).reshape(-1)
    hi, lo = chk.clone(), chk.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    if not torch.equal(hi, lo):
        fails.append("params differ across ranks")
    print(f"RANK{rank} {'OK' if not fails else 'FAIL ' + repr(fails)}", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if not fails else 1)


if __name__ == "__main__":
    main()
