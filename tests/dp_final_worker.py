"""Worker for test_dp_final_train_step (torch.distributed.run, 2 ranks sharing one GPU, gloo):
the configs/jhu_fog2snow.yml step — DGModel_final, DGTrainer 'final' mode, fused AdamW with
its flat-gradient all-reduce — run data-parallel over the ranks' halves of a 4-frame batch
must leave exactly the parameters of a single-process emulation: each half's gradients
computed separately (per-rank BatchNorm statistics, as DDP without SyncBN), averaged, then
one AdamW step.  Dropouts are off so both runs see the same masks.  Then the backward-overlapped
bucketed all-reduce equals the single collective bit for bit over three steps."""
import os
import sys
import tempfile

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import dg_oracle as O  # noqa: E402
from dgvcc_amd import dist as D  # noqa: E402
from dgvcc_amd.losses import MSELoss  # noqa: E402
from dgvcc_amd.models.models import DGModel_final  # noqa: E402
from dgvcc_amd.optim import AdamW  # noqa: E402
from dgvcc_amd.trainers.dgtrainer import DGTrainer  # noqa: E402


def build(dev, sd0):
    m = DGModel_final(pretrained=False, den_dropout=0.0, cls_dropout=0.0)
    m.load_state_dict(sd0)
    return m.to(dev).set_precision("fp32").train()


def half(batch, r, world):
    i1, i2, (pts, dm, bm) = batch
    n = i1.shape[0] // world
    s = slice(r * n, (r + 1) * n)
    return i1[s], i2[s], (pts[s], dm[s], bm[s])


def to_dev(batch, dev):
    i1, i2, (pts, dm, bm) = batch
    return i1.to(dev), i2.to(dev), (tuple(p.to(dev) for p in pts), dm.to(dev), bm.to(dev))


def main():
    D.init_from_env("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sd0 = O.seeded_state_dict(DGModel_final(pretrained=False).state_dict())
    batch = O.synthetic_batch(2 * world, 64, 64, seed=2112)
    cwd = os.getcwd()
    td = tempfile.mkdtemp()
    os.chdir(td)
    tr = DGTrainer(2112, f"dp{rank}", dev, 1000, 10000, "final")
    # data-parallel step: this rank's half, gradients averaged over RCCL/gloo inside AdamW
    model = build(dev, sd0)
    D.broadcast_module_(model)
    opt = AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    loss_dp = tr.train_step(model, MSELoss(), opt, to_dev(half(batch, rank, world), dev), 0)
    dp = {k: v.detach().clone() for k, v in model.named_parameters()}
    fails = []
    # parameters identical on every rank
    chk = torch.stack([p.detach().double().sum() for p in model.parameters()]).reshape(-1)
    hi, lo = chk.clone(), chk.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    if not torch.equal(hi, lo):
        fails.append("params differ across ranks")
    if rank == 0:
        # single-process emulation: per-half gradients (per-half BN), averaged, one AdamW step
        grads, losses = [], []
        for r in range(world):
            m = build(dev, sd0)
            for p in m.parameters():
                p.grad = None
            i1, i2, (pts, dm, bm) = to_dev(half(batch, r, world), dev)
            dc1, dc2, c1, c2, _, lcon, _ = m.forward_train(i1, i2, bm)
            from dgvcc_amd.losses import mse_loss
            from dgvcc_amd.losses.bce import binary_cross_entropy
            l = (mse_loss(dc1, dm, 1000.0) + mse_loss(dc2, dm, 1000.0)
                 + 10 * (binary_cross_entropy(c1, bm) + binary_cross_entropy(c2, bm)) + 10 * lcon)
            l.backward()
            grads.append({k: p.grad.detach().clone() for k, p in m.named_parameters()})
            losses.append(l.item())
        emu = build(dev, sd0)
        for k, p in emu.named_parameters():
            p.grad = (grads[0][k] + grads[1][k]) / world
        opt2 = AdamW(emu.parameters(), lr=1e-4, weight_decay=1e-4, allreduce=False)
        opt2.step()
        worst = 0.0
        for k, v in emu.named_parameters():
            d = (dp[k].double() - v.detach().double()).abs().max().item()
            worst = max(worst, d / max(v.detach().double().abs().max().item(), 1e-30))
        if worst > 1e-6:
            fails.append(("post-step params vs emulation", worst))
        print(f"RANK0 worst_rel={worst:.3e} loss_dp={loss_dp:.6f} loss_half0={losses[0]:.6f}", flush=True)
    # backward-overlapped bucketed all-reduce (dgvcc_amd.dist.OverlapReducer, active from the second
    # step): three steps leave exactly the parameters of the one-collective-after-backward path
    finals = []
    for overlap in (False, True):
        m = build(dev, sd0)
        opt = AdamW(m.parameters(), lr=1e-4, weight_decay=1e-4, overlap=overlap, bucket_mb=8.0)
        for _ in range(3):
            tr.train_step(m, MSELoss(), opt, to_dev(half(batch, rank, world), dev), 0)
        if overlap:
            red = opt.reducer
            if red is None or len(red.buckets) < 3 or m._get_plans()["fe"].sink is not red:
                fails.append("overlap reducer not attached")
        finals.append({k: v.detach().clone() for k, v in m.named_parameters()})
    diff = [k for k in finals[0] if not torch.equal(finals[0][k], finals[1][k])]
    if diff:
        fails.append(("overlapped all-reduce differs", diff[:5]))
    os.chdir(cwd)
    print(f"RANK{rank} {'OK' if not fails else 'FAIL ' + repr(fails)}", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if not fails else 1)


if __name__ == "__main__":
    main()
