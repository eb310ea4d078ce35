"""DGVCC MI355X benchmark: train-step frames/s at 768x1024 (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--mode simple|final]

Workload (BASELINE.json configs[1], configs/stb_reg_base.yml): DGModel_base
(VGG16-BN encoder + density decoder), DGTrainer 'simple' mode, MSE count loss
(log_para 1000), fused AdamW, bf16 storage/MFMA with f32 accumulation, batch 16
per GPU of synthetic 3x768x1024 frames resident in HBM (no dataset offline).
A step = DGTrainer.train_step (forward + loss + backward + optimizer step +
the reference's per-step `.item()` sync).  Multi-GPU: one process per GPU
(torchrun), per-GPU batch fixed (weak scaling), one RCCL all-reduce of the flat
fp32 gradient per step inside the fused optimizer.

Prints ONE JSON line on rank 0 with roofline (dominant kernel = the implicit-GEMM
conv, timed per launch with HIP events on the launch stream during the timed
region) and cpu_baseline (the oracle's CPU restatement of the same step, timed
on this host on a bounded sample, plus the fp32 density-map parity of the HIP
path against it on the same 768x1024 frame).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BF16_DENSE_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: ~2.5 PF dense bf16
F32_MFMA_PEAK_TFLOPS = 157.3
H0, W0 = 768, 1024


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16, help="frames per GPU")
    ap.add_argument("--mode", default="simple", choices=["simple", "final"])
    ap.add_argument("--trunk", default=None, choices=["ibn", "sw", "isw"],
                    help="secondary workload: ResNet-50 DG counter (IBN-b / SW / ISW) train step")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--height", type=int, default=H0)
    ap.add_argument("--width", type=int, default=W0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    return ap.parse_args()


def synthetic(B, H, W, device, seed):
    """SURVEY.md §8d synthetic frames (device-resident): images in [-1,1], view 2 =
    view 1 + 0.1 N(0,1), ~Poisson(500)-sized point sets, dmap by the HIP scatter,
    bmap = 16x16 block-sum > 0."""
    from dgvcc_amd.utils.dmap_gen import gaussian_filter_density_fixed_batch
    g = torch.Generator(device="cpu").manual_seed(seed)
    img1 = (torch.randn(B, 3, H, W, generator=g) * 0.5).clamp(-1, 1)
    img2 = (img1 + 0.1 * torch.randn(B, 3, H, W, generator=g)).clamp(-1, 1)
    n = torch.poisson(torch.full((B,), 500.0 * H * W / (H0 * W0)), generator=g).long().clamp_min(1)
    pts = [torch.rand(int(k), 2, generator=g) * torch.tensor([W, H], dtype=torch.float32) for k in n]
    dm = gaussian_filter_density_fixed_batch([p.to(device) for p in pts], H, W)
    dmaps = dm.view(B, 1, H, W)
    bmaps = (dmaps.reshape(B, 1, H // 16, 16, W // 16, 16).sum(dim=(3, 5)) > 0).float()
    return img1.to(device), img2.to(device), (tuple(p.to(device) for p in pts), dmaps, bmaps)


def conv_flops_per_step(B, H, W, mode):
    """Algorithmic conv FLOPs of one train step (fwd + dgrad + wgrad), SURVEY.md §8d."""
    views = 2 if mode == "final" else 1
    layers = []
    h, w, cin = H, W, 3
    for v in [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512]:
        if v == "M":
            h, w = h // 2, w // 2
            continue
        layers.append((h, w, cin, v, 9, cin != 3))
        cin = v
    s = H // 16, W // 16
    layers += [(s[0], s[1], 512, 1024, 9, True), (s[0], s[1], 1024, 512, 9, True),
               (2 * s[0], 2 * s[1], 1024, 512, 9, True), (2 * s[0], 2 * s[1], 512, 256, 9, True),
               (4 * s[0], 4 * s[1], 512, 256, 9, True), (4 * s[0], 4 * s[1], 256, 128, 9, True),
               (4 * s[0], 4 * s[1], 896, 256, 1, True)]
    tot = 0.0
    for (h, w, ci, co, k, dgrad) in layers:
        f = 2.0 * B * views * h * w * ci * co * k
        tot += f * (3 if dgrad else 2)
    return tot


class ConvTimer:
    """Per-launch HIP events around the implicit-GEMM conv launches, recorded on
    torch's current stream — the stream the C-ABI launches on.  Kinds: 'fwd' and
    'dgrad' run `conv_fwd_kernel`, 'wgrad' runs `conv_wgrad_kernel` (+ reduce)."""

    def __init__(self):
        self.ev = {}

    def __call__(self, kind, flops, launch, nbytes=0.0):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        launch()
        e.record()
        self.ev.setdefault(kind, []).append((s, e, flops, nbytes))

    def summary(self, kinds):
        torch.cuda.synchronize()
        ms = fl = nb = 0.0
        n = 0
        for k in kinds:
            for s, e, f, b in self.ev.get(k, []):
                ms += s.elapsed_time(e)
                fl += f
                nb += b
                n += 1
        self.nbytes = nb
        return ms, fl, n


def cpu_baseline(args, seconds):
    """The oracle's CPU restatement of the same train step (kind 'port'), batch 1."""
    from oracle import dg_oracle as O
    from dgvcc_amd.models.models import DGModel_base
    threads = max(1, min(os.cpu_count() or 1, 16))
    torch.set_num_threads(threads)
    tmpl = DGModel_base(pretrained=False, den_dropout=0.0).state_dict()
    sd = O.seeded_state_dict(tmpl)
    batch = O.synthetic_batch(1, args.height, args.width, seed=7)
    mode = "simple" if args.mode == "simple" else "final"
    loss_ref, outs, _, _ = O.train_step(sd, batch, mode)  # warm-up (and the parity reference below)
    parity = density_parity(sd, batch, loss_ref, outs[0]) if mode == "simple" else None
    n, t0 = 0, time.perf_counter()
    while True:
        O.train_step(sd, batch, mode)
        n += 1
        if time.perf_counter() - t0 >= seconds or n >= 8:
            break
    dt = time.perf_counter() - t0
    frames = n * (2 if mode == "final" else 1)
    out = {"value": frames / dt, "unit": "frames/s", "cores": threads, "kind": "port",
           "sample": f"{n} oracle train steps ({mode} mode, batch 1, {args.height}x{args.width}, fp32, "
                     f"torch CPU {threads} threads) after 1 warm-up"}
    if parity is not None:
        out["parity"] = parity
    return out


def density_parity(sd, batch, loss_ref, d_ref):
    """The metric's "MAE vs reference" on the warm-up frame: the HIP path (fp32 mode, the
    parity precision of BASELINE.json's north_star) against the oracle's density map and
    MSE loss for the same weights and frame.  The oracle is only the checker here."""
    from dgvcc_amd.models.models import DGModel_base
    from dgvcc_amd.losses import mse_loss
    dev = torch.device("cuda", torch.cuda.current_device())
    model = DGModel_base(pretrained=False, den_dropout=0.0)
    model.load_state_dict(sd)
    model = model.to(dev).set_precision("fp32").train()
    d = model(batch[0].to(dev))
    loss = mse_loss(d, batch[2][1].to(dev), 1000.0)
    loss.backward()
    torch.cuda.synchronize()
    d = d.detach().double().cpu()
    r = d_ref.detach().double()
    return {"precision": "fp32", "frame": "1x3x%dx%d" % tuple(r.shape[-2:]), "tolerance_rel": 1e-4,
            "density_map_mae": float((d - r).abs().mean()),
            "density_map_max_rel": float((d - r).abs().max() / r.abs().max()),
            "count_abs_err": float(abs(d.sum() - r.sum()) / 1000.0),
            "loss_rel": float(abs(loss.item() - loss_ref.item()) / abs(loss_ref.item()))}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DGVCC_BENCH_BACKEND=gloo: rehearsal of the multi-rank path with several ranks sharing one
    # GPU (local rank modulo the visible devices); the driver's runs use RCCL ("nccl").
    backend = os.environ.get("DGVCC_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from dgvcc_amd import kernels as K
    from dgvcc_amd.models import models as MM
    from dgvcc_amd.losses import MSELoss
    from dgvcc_amd.optim import AdamW
    from dgvcc_amd.trainers.dgtrainer import DGTrainer

    B, H, W = args.batch, args.height, args.width
    torch.manual_seed(2112)
    mode = args.mode
    if args.trunk:
        from dgvcc_amd.models import trunks as TM
        cls = {"ibn": TM.IBNCounter_ResNet, "sw": TM.SWCounter_ResNet, "isw": TM.ISWCounter_ResNet}
        model = cls[args.trunk](pretrained=False)
        mode = "isw" if args.trunk == "isw" else "simple"
    elif args.mode == "simple":
        model = MM.DGModel_base(pretrained=False, den_dropout=0.5)
    else:
        model = MM.DGModel_final(pretrained=False)
    model = model.to(dev).set_precision(args.precision)
    if world > 1:  # identical init on every rank
        import torch.distributed as dist
        for t in model.state_dict().values():
            dist.broadcast(t, 0)
    opt = AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    cwd = os.getcwd()
    os.makedirs("/tmp/dgvcc_bench", exist_ok=True)
    os.chdir("/tmp/dgvcc_bench")
    trainer = DGTrainer(2112 + rank, f"bench_r{rank}", dev, 1000, 10000, mode)
    os.chdir(cwd)
    batch = synthetic(B, H, W, dev, seed=1000 + rank)
    loss_fn = MSELoss()
    epoch = 0
    if args.trunk == "isw":  # cal_covstat pass (validation-time in the reference) -> masks; epoch > 5 -> wt loss on
        model.eval()
        with torch.no_grad():
            model([batch[0], batch[1]], cal_covstat=True)
        epoch = 6
    model.train()

    for _ in range(args.warmup):
        trainer.train_step(model, loss_fn, opt, batch, epoch)

    timer = ConvTimer()
    K.set_conv_timer(timer)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        last = trainer.train_step(model, loss_fn, opt, batch, epoch)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    K.set_conv_timer(None)
    conv_ms, conv_flops, conv_launches = timer.summary(("fwd", "dgrad"))
    conv_alg_bytes = timer.nbytes / max(conv_launches, 1)
    wg_ms, wg_flops, wg_launches = timer.summary(("wgrad",))
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        # data-parallel sanity check outside the timed region: identical parameters on every rank
        chk = torch.stack([p.detach().double().sum() for p in model.parameters()]).sum().reshape(1)
        hi, lo = chk.clone(), chk.clone()
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        params_in_sync = bool(hi.item() == lo.item())

    views = 2 if (args.mode == "final" and not args.trunk) else 1
    frames = B * views * world * args.steps
    value = frames / elapsed
    peak = BF16_DENSE_PEAK_TFLOPS if args.precision == "bf16" else F32_MFMA_PEAK_TFLOPS
    achieved = conv_flops / (conv_ms * 1e-3) / 1e12 if conv_ms > 0 else 0.0
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "conv_traffic.json")
    if os.path.exists(tpath):
        try:
            traffic = json.load(open(tpath)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    step_flops = conv_flops_per_step(B, H, W, args.mode) if not args.trunk else \
        (conv_flops + wg_flops) / args.steps
    out = {
        "metric": "train-step frames/sec at 768×1024, ShanghaiTech-A; MAE vs reference",
        "value": round(value, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic 3x768x1024 frames + Poisson(500) point sets (dmap via HIP scatter), HBM-resident",
        "config": {"workload": (f"{type(model).__name__} {mode}-mode DGTrainer.train_step "
                                f"(configs/baselines/sta_{args.trunk}.yml)") if args.trunk else
                   (f"DGModel_base {args.mode}-mode DGTrainer.train_step (configs/stb_reg_base.yml)"
                    if args.mode == "simple" else "DGModel_final final-mode DGTrainer.train_step (configs/sta_final.yml)"),
                   "global_batch": B * world, "frames_per_gpu_step": B * views,
                   "resolution": f"{H}x{W}", "parallelism": f"dp{world}", "last_loss": last},
        "roofline": {"bound": "mfma", "kernel": "conv_fwd_pers_kernel + conv_fwd_tap3p_kernel + conv_fwd_pipe_kernel + conv_fwd_tap3_kernel (implicit-GEMM conv: forward + dgrad launches)",
                     "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4), "traffic": traffic,
                     "algorithmic_bytes_per_launch": round(conv_alg_bytes),
                     "algorithmic_flop_per_launch": round(conv_flops / max(conv_launches, 1)),
                     "launches_per_step": conv_launches // args.steps,
                     "avg_launch_us": round(conv_ms * 1e3 / max(conv_launches, 1), 2),
                     "kernel_ms_per_step": round(conv_ms / args.steps, 3),
                     "wgrad_achieved": round(wg_flops / (wg_ms * 1e-3) / 1e12, 2) if wg_ms > 0 else None,
                     "wgrad_ms_per_step": round(wg_ms / args.steps, 3),
                     "model_conv_tflops_per_step_algorithmic": round(step_flops / 1e12, 4),
                     "whole_step_mfma_frac": round(step_flops / (elapsed / args.steps) / 1e12 / peak, 4)},
    }
    if world > 1:
        out["params_in_sync"] = params_in_sync
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
