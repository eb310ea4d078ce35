"""Worker for test_dp_syncbn_strong_scaling (torch.distributed.run, 2 ranks sharing one GPU, gloo):
configs/jhu_fog2snow.yml's global batch strong-scaled over the ranks with SyncBatchNorm
(`nn.SyncBatchNorm.convert_sync_batchnorm`, dgvcc_amd/syncbn.py), so every BN layer normalises
with the statistics of the whole batch as the reference's single-device run does
(models/ISW/mynn.py:8-14, models/SW/ops/sync_switchwhiten.py:9-56).

1. Layer level, every SyncBN route of the engine against the same layer with a plain BatchNorm2d
   on the whole batch (outputs, input gradients, parameter gradients, running statistics <= 1e-6):
   a plain ConvLayer, a max-pooled one, the decomposed CatConvLayer on CatParts (den_dec), and a
   ConvLayer whose BN backward consumes the next layer's dgrad-epilogue partial rows (decoder).
2. The whole final-mode step (whole_step): on a batch where the DP ranks and the single-process
   run take the same branches (every ReLU / max-pool decision compared; the thresholded e_mask and
   class maps of models/models.py:306-307, 324-325 injected from the single-process run with
   PairPlan.inject), the rank-averaged gradients, the loss and the BN running statistics must equal
   the single-process step's at 1e-5.
3. One real DGTrainer step with the fused AdamW (its flat-gradient all-reduce) leaves identical
   parameters on both ranks.
Every rank prints OK only when the verdict gathered from all ranks is clean."""
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

B, H, W = 4, 64, 64
SEEDS = 8
LAYER_TOL = 1e-6
STEP_TOL = 1e-5


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


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


def step_grads(m, batch, dev, inject=None, capture=None, backward=True):
    i1, i2, (pts, dm, bm) = batch
    i1, i2, dm, bm = i1.to(dev), i2.to(dev), dm.to(dev), bm.to(dev)
    plan = m._get_plans()["pair"]
    plan.inject, plan.capture = inject, capture
    for p in m.parameters():
        p.grad = None
    with torch.set_grad_enabled(backward):
        dc1, dc2, c1, c2, _, lcon, _ = m.forward_train(i1, i2, bm)
        loss = (mse_loss(dc1, dm, 1000.0) + mse_loss(dc2, dm, 1000.0)
                + 10 * (binary_cross_entropy(c1, bm) + binary_cross_entropy(c2, bm)) + 10 * lcon)
    plan.capture = None
    if not backward:
        return loss.detach(), None
    loss.backward()
    return loss.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}


# ----------------------------------------------------------------------------- layer level
def _bn(Co, sync, dev):
    bn = nn.BatchNorm2d(Co)
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.5, 1.5, Co))
        bn.bias.copy_(torch.linspace(-0.2, 0.2, Co))
    if sync:
        bn = nn.SyncBatchNorm.convert_sync_batchnorm(bn)
    return bn.to(dev)


def _conv(C, Co, R, seed, dev):
    g = torch.Generator().manual_seed(seed)
    cv = nn.Conv2d(C, Co, R, padding=R // 2)
    with torch.no_grad():
        cv.weight.copy_(torch.randn(cv.weight.shape, generator=g) * (2.0 / (C * R * R)) ** 0.5)
        cv.bias.copy_(torch.randn(Co, generator=g) * 0.1)
    return cv.to(dev)


def case_conv(pool, N=4, Hh=32, Ww=40, C=64, Co=128):
    """Conv3x3 C->Co + BN + ReLU (+ the fused MaxPool2d(2,2)) on N x Hh x Ww."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N, Hh, Ww, C, generator=g)
    gy = torch.randn(N, Hh // 2 if pool else Hh, Ww // 2 if pool else Ww, Co, generator=g)

    def run(sync, xs, gs, dev):
        from dgvcc_amd import engine as E
        from dgvcc_amd import kernels as K
        cv, bn = _conv(C, Co, 3, 7, dev), _bn(Co, sync, dev)
        L = E.ConvLayer(cv, bn, E.ACT_RELU)
        n, h, w = xs.shape[:3]
        tape = {}
        xa = K.Act(xs.to(dev).contiguous())
        if pool:
            out = K.Act(K.nhwc(n, h // 2, w // 2, Co, torch.float32, dev))
            L.forward(xa, None, True, tape, pool=out)
        else:
            out = K.Act(K.nhwc(n, h, w, Co, torch.float32, dev))
            L.forward(xa, out, True, tape)
        gx = K.Act(K.nhwc(n, h, w, C, torch.float32, dev))
        ga = K.Act(gs.to(dev).contiguous())
        grads = L.backward(tape, None, gx, g_pool=ga) if pool else L.backward(tape, ga, gx)
        names = {cv.weight: "w", cv.bias: "b", bn.weight: "gamma", bn.bias: "beta"}
        return ({"out": out.buf, "gx": gx.buf}, {names[p]: v for p, v in grads.items()},
                {"rm": bn.running_mean, "rv": bn.running_var})
    return x, gy, run


def case_cat():
    """den_dec: CatConvLayer (1x1 896->256 + BN + ReLU) on CatParts y1, y2 (1/2), y3 (1/4)."""
    N, h, w, Cs, Co = 4, 16, 16, (128, 256, 512), 256
    g = torch.Generator().manual_seed(11)
    xs = [torch.randn(N, h // s, w // s, c, generator=g) for c, s in zip(Cs, (1, 2, 4))]
    gy = torch.randn(N, h, w, Co, generator=g)

    def run(sync, parts, gs, dev):
        from dgvcc_amd import engine as E
        from dgvcc_amd import kernels as K
        cv, bn = _conv(sum(Cs), Co, 1, 13, dev), _bn(Co, sync, dev)
        L = E.CatConvLayer(cv, bn, E.ACT_RELU)
        cat = E.CatParts(*(K.Act(p.to(dev).contiguous()) for p in parts))
        n = parts[0].shape[0]
        out = K.Act(K.nhwc(n, h, w, Co, torch.float32, dev))
        tape = {}
        L.forward(cat, out, True, tape)
        gcat = cat.empty_like()
        grads = L.backward(tape, K.Act(gs.to(dev).contiguous()), gcat)
        names = {cv.weight: "w", cv.bias: "b", bn.weight: "gamma", bn.bias: "beta"}
        res = {"out": out.buf}
        res.update({f"gx{k}": t for k, t in enumerate(gcat.tensors())})
        return res, {names[p]: v for p, v in grads.items()}, {"rm": bn.running_mean, "rv": bn.running_var}
    return xs, gy, run


def case_bnpart():
    """Conv3x3 128->256 + BN + ReLU -> Conv3x3 256->128 + BN + ReLU (dec1's second layer), the
    second layer's dgrad epilogue emitting the first layer's BN-backward partial rows
    (ConvLayer.backward gx_bn; an opt-in route, kernels.conv_dgrad_bnpart, forced on for both
    runs; the f32 epilogue lives in the persistent pre-split kernel, which serves launches of more
    than 256 pixel tiles: 2 x 144 x 256 pixels per rank)."""
    N, Hh, Ww, C, C1, C2 = 4, 144, 256, 128, 256, 128
    g = torch.Generator().manual_seed(17)
    x = torch.randn(N, Hh, Ww, C, generator=g)
    gy = torch.randn(N, Hh, Ww, C2, generator=g)

    def run(sync, xs, gs, dev):
        from dgvcc_amd import engine as E
        from dgvcc_amd import kernels as K
        cva, bna = _conv(C, C1, 3, 19, dev), _bn(C1, sync, dev)
        cvb, bnb = _conv(C1, C2, 3, 23, dev), _bn(C2, sync, dev)
        A, Bl = E.ConvLayer(cva, bna, E.ACT_RELU), E.ConvLayer(cvb, bnb, E.ACT_RELU)
        n = xs.shape[0]
        tape = {}
        a = K.Act(K.nhwc(n, Hh, Ww, C1, torch.float32, dev))
        b = K.Act(K.nhwc(n, Hh, Ww, C2, torch.float32, dev))
        A.forward(K.Act(xs.to(dev).contiguous()), a, True, tape)
        Bl.forward(a, b, True, tape)
        ga = K.Act(K.nhwc(n, Hh, Ww, C1, torch.float32, dev))
        off = K._BNPART_F32_OFF
        K._BNPART_F32_OFF = False  # the route is opt-in (DGVCC_DGRAD_BNPART_F32=1): forced on here
        try:
            gb = Bl.backward(tape, K.Act(gs.to(dev).contiguous()), ga, gx_bn=A)
        finally:
            K._BNPART_F32_OFF = off
        if ("bnpart", A) not in tape:
            raise RuntimeError("case_bnpart: the dgrad-epilogue partial route was not taken")
        gx = K.Act(K.nhwc(n, Hh, Ww, C, torch.float32, dev))
        gA = A.backward(tape, ga, gx)
        names = {cva.weight: "wa", cva.bias: "ba", bna.weight: "gamma_a", bna.bias: "beta_a",
                 cvb.weight: "wb", cvb.bias: "bb", bnb.weight: "gamma_b", bnb.bias: "beta_b"}
        grads = {names[p]: v for p, v in list(gA.items()) + list(gb.items())}
        return ({"out": b.buf, "ga": ga.buf, "gx": gx.buf}, grads,
                {"rm_a": bna.running_mean, "rv_a": bna.running_var, "rm_b": bnb.running_mean,
                 "rv_b": bnb.running_var})
    return x, gy, run


def layer_check(name, case, dev, rank, world):
    x, gy, run = case
    n = gy.shape[0] // world
    sl = slice(rank * n, (rank + 1) * n)
    xs = [t[sl] for t in x] if isinstance(x, list) else x[sl]
    outs, grads, rs = run(True, xs, gy[sl], dev)
    full = {}
    for k, t in outs.items():
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t.contiguous())
        full[k] = torch.cat(parts)
    for v in grads.values():
        dist.all_reduce(v)  # the DP gradient sum (the average x world) of the per-rank sums
    fails = []
    if rank == 0:
        r_outs, r_grads, r_rs = run(False, x, gy, dev)
        errs = {k: rel(full[k], r_outs[k]) for k in r_outs}
        errs.update({k: rel(rs[k], r_rs[k]) for k in r_rs})
        errs.update({"grad_" + k: rel(grads[k], r_grads[k]) for k in r_grads
                     if k not in ("b", "ba", "bb")})  # pre-BN conv biases: zero in exact math
        print(f"RANK0 layer {name}: max {max(errs.values()):.2e} {errs}", flush=True)
        bad = {k: v for k, v in errs.items() if v > LAYER_TOL}
        if bad:
            fails.append((f"layer {name}", bad))
    return fails


# ----------------------------------------------------------------------------- whole step
def _skip(k):  # pre-BN conv biases: mathematically zero gradient (rounding noise on both sides)
    return k.endswith(".bias") and (k.startswith("enc") or ".conv." in k) and "cls_head.2" not in k


def decisions(m, batch, dev):
    """Every branch the final-mode forward takes on `batch`, from a no-grad forward with tapes on
    a fresh model: per ConvLayer of both views' FeaturePlan and of den_dec / cls_head the ReLU
    decisions (scale * z + shift > 0) and, for the max-pooled layers, each 2x2 window's argmax;
    the density-head ReLUs; and the thresholded e_mask / class maps (capture).  Batch-first
    uint8 tensors on the CPU, keyed by layer."""
    i1, i2, (_pts, _dm, bm) = batch
    plans = m._get_plans()
    fe, pair = plans["fe"], plans["pair"]
    tA, tB, tP = {}, {}, {}
    pair.capture = {}
    with torch.no_grad():
        oA = fe.forward(i1.to(dev), torch.float32, True, tA)
        oB = fe.forward(i2.to(dev), torch.float32, True, tB)
        pair.forward(oA[:3], oB[:3], oA[3], oB[3], bm.to(dev), 0.0, float(m.err_thrs), tP)
    cap, pair.capture = pair.capture, None
    out = {"emask": cap["emask"].cpu(), "c_pred1": cap["c_pred"][0].to(torch.uint8).cpu(),
           "c_pred2": cap["c_pred"][1].to(torch.uint8).cpu()}
    pooled = {fe.enc[i] for i in (1, 3, 6, 9)}

    def layer(key, L, ent):
        _x, z, st = ent[0], ent[1], ent[2]
        pre = z.view() * st[2] + st[3]
        if L.act == 1:  # ACT_RELU
            out[key + ".relu"] = (pre > 0).to(torch.uint8).cpu()
        if L in pooled:
            y = pre.clamp_min(0)
            n, h, w, c = y.shape
            win = y.view(n, h // 2, 2, w // 2, 2, c).permute(0, 1, 3, 5, 2, 4).reshape(n, h // 2, w // 2, c, 4)
            out[key + ".pool"] = win.argmax(-1).to(torch.uint8).cpu()

    for tag, t in (("A", tA), ("B", tB)):
        for i, L in enumerate(fe.layers):
            layer(f"{tag}{i}", L, t[L])
    st = tP[pair]
    for v in (1, 2):
        layer(f"den{v}", pair.den, st[f"s{v}"][pair.den])
        sub = st["sub"][f"c{v}"][0]
        layer(f"cls{v}", pair.cls, sub[pair.cls])
        out[f"head{v}"] = (st[f"yh{v}"] > 0).to(torch.uint8).cpu()
    return out


def _slice(dec, r, world):
    return {k: v[r * (v.shape[0] // world):(r + 1) * (v.shape[0] // world)].contiguous() for k, v in dec.items()}


def whole_step(dev, rank, world):
    """The strong-scaled SyncBN step against the single-process step, on a batch where both take
    the same branches.  The threshold decisions (e_mask, class maps) are injected from the
    single-process run; every other branch (ReLU, max-pool argmax, density-head ReLU) cannot be,
    so a seed is used only if all of them agree between the two runs (decisions()): a ReLU whose
    pre-activation is within rounding of zero flips with the last bit of the batch statistics, and
    one flip at a pixel that carries much of the density loss moves whole-layer gradients by
    percents (diagnosed in round 4: tools/diag_fwd_flips.py, tools/diag_step_glue.py).  Given equal
    branches the step must agree at 1e-5."""
    fails = []
    sd0 = O.seeded_state_dict(DGModel_final(pretrained=False).state_dict())
    batch = None
    for k in range(SEEDS):
        cand = O.synthetic_batch(B, H, W, seed=2112 + k)
        box = [None]
        if rank == 0:
            box[0] = decisions(build(dev, sd0, sync=False), cand, dev)
        dist.broadcast_object_list(box, src=0)
        ref_dec = _slice(box[0], rank, world)
        mine = decisions(build(dev, sd0, sync=True), part(cand, rank, world), dev)
        keys = sorted(ref_dec)
        diff = torch.tensor([int((mine[key] != ref_dec[key]).sum()) for key in keys], dtype=torch.int64)
        dist.all_reduce(diff)
        branch = {key: int(d) for key, d in zip(keys, diff) if d and key not in ("emask", "c_pred1", "c_pred2")}
        if rank == 0:
            thr = {key: int(d) for key, d in zip(keys, diff) if key in ("emask", "c_pred1", "c_pred2")}
            print(f"RANK0 seed {2112 + k}: differing decisions DP vs single-process: thresholds {thr} (injected), "
                  f"other branches {branch or 0}", flush=True)
        if not branch:
            batch = cand
            inj = {"emask": ref_dec["emask"].to(dev),
                   "c_pred": (ref_dec["c_pred1"].float().to(dev), ref_dec["c_pred2"].float().to(dev))}
            break
    if batch is None:
        return [f"no seed of {SEEDS} with identical branches in both runs"], sd0, cand
    # (a) the single-process whole-batch step with plain BatchNorm
    if rank == 0:
        ref = build(dev, sd0, sync=False)
        loss_ref, grads_ref = step_grads(ref, batch, dev)
        rstats_ref = {k: v.detach().cpu() for k, v in ref.state_dict().items() if "running" in k}
        del ref
    # (b) the strong-scaled SyncBN step on the single-process threshold decisions
    m = build(dev, sd0, sync=True)
    assert sum(isinstance(x, nn.SyncBatchNorm) for x in m.modules()) == 21
    loss, grads = step_grads(m, part(batch, rank, world), dev, inject=inj)
    dist.all_reduce(loss)
    loss /= world
    for g in grads.values():
        dist.all_reduce(g)
        g /= world
    rstats = {k: v.detach().cpu() for k, v in m.state_dict().items() if "running" in k}
    if rank == 0:
        lr = abs(loss.item() - loss_ref.item()) / abs(loss_ref.item())
        if lr > STEP_TOL:
            fails.append(("loss", lr))
        worst = {k: rel(grads[k], r) for k, r in grads_ref.items() if not _skip(k) and r.norm() > 0}
        top = sorted(worst.items(), key=lambda kv: -kv[1])[:6]
        bad = {k: v for k, v in worst.items() if v > STEP_TOL}
        if bad:
            fails.append(("grads", bad))
        rs = max(((rstats[k].double() - v.double()).abs().max() / v.double().abs().max().clamp_min(1e-30)).item()
                 for k, v in rstats_ref.items())
        if rs > STEP_TOL:
            fails.append(("running stats", rs))
        print(f"RANK0 step (same branches): loss_rel={lr:.3e} running={rs:.3e} worst grads {top}", flush=True)
    return fails, sd0, batch


def trainer_step(dev, rank, world, sd0, batch):
    """One real DGTrainer step with SyncBN and the fused AdamW: parameters identical across ranks."""
    m2 = build(dev, sd0, sync=True)
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp())
    try:
        tr = DGTrainer(2112, f"sbn{rank}", dev, 1000, 10000, "final")
        i1, i2, (pts, dm, bm) = part(batch, rank, world)
        tr.train_step(m2, MSELoss(), AdamW(m2.parameters(), lr=1e-4, weight_decay=1e-4),
                      (i1.to(dev), i2.to(dev), (tuple(p.to(dev) for p in pts), dm.to(dev), bm.to(dev))), 0)
    finally:
        os.chdir(cwd)
    chk = torch.stack([p.detach().double().sum() for p in m2.parameters()]).reshape(-1)
    hi, lo = chk.clone(), chk.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    return [] if torch.equal(hi, lo) else [f"rank {rank}: params differ across ranks"]


def main():
    D.init_from_env("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    fails = []
    for name, case in (("conv", case_conv(False)), ("conv+pool", case_conv(True)),
                       ("conv cls_head 8x8", case_conv(False, 4, 8, 8, 512, 256)),
                       ("conv dec3 8x8", case_conv(False, 4, 8, 8, 512, 1024)),
                       ("conv dec2 16x16", case_conv(False, 4, 16, 16, 1024, 512)),
                       ("cat", case_cat()), ("dgrad-bnpart", case_bnpart())):
        fails += layer_check(name, case, dev, rank, world)
    f, sd0, batch = whole_step(dev, rank, world)
    fails += f
    fails += trainer_step(dev, rank, world, sd0, batch)
    every = [None] * world
    dist.all_gather_object(every, fails)
    allf = [x for fl in every for x in fl]
    print(f"RANK{rank} {'OK' if not allf else 'FAIL ' + repr(allf)}", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if not allf else 1)


if __name__ == "__main__":
    main()
