"""DGVCC MI355X benchmark: train-step frames/s at 768x1024 (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--mode final|simple|base]
                    [--precision fp32|bf16] [--no-bf16] [--trunk ibn|sw|isw]

Default workload = the config BASELINE.json's metric is quoted on, configs/sta_final.yml
(ShanghaiTech-A "final"): DGModel_final, DGTrainer 'final' mode (two photometric views,
MSE count loss x log_para 1000 + 10 BCE class-map loss + 10 JSD-MSE consistency loss,
fused AdamW), batch 16 per GPU of synthetic 3x768x1024 frames resident in HBM (no dataset
offline), computed in fp32 like the reference: f32 storage, statistics and accumulation, the conv
GEMMs on the f16 matrix cores as "f16 x3" (default `--f32-math h16`): each f32 operand scaled by a
power of two (per filter row; per pixel-operand tensor in the forward / dgrad, per channel of both
operands in the weight gradient) and cut into two f16 parts by nearest rounding, three f16 MFMA
products per f32 product (hi*hi + hi*lo + lo*hi), f32 accumulation, exact rescale: f32-grade
(DESIGN.md §3.1).  `--f32-math split` selects the exact 3-way bf16 split (six bf16 products per f32
product), `--f32-math exact` v_mfma_f32_16x16x4_f32; the exact leg is reported beside the headline
as `f32_exact`.  A step is
DGTrainer.train_step: forward + loss + backward + optimizer step + the reference's per-step
`.item()`; a frame is one 3x768x1024 view through forward and backward (final mode counts
both views).  The same step in bf16 (bf16 storage/MFMA, f32 accumulation and
statistics) is reported beside it as `perf_bf16`, with its own roofline.

Multi-GPU: `--gpus N` without a torchrun environment starts
`python -m torch.distributed.run --nproc-per-node N` as a child process (before any GPU
call) and relays its rank-0 line; under torchrun one process per GPU, per-GPU batch fixed
(weak scaling), one RCCL all-reduce of the flat fp32 gradient per step inside the fused
optimizer, max-over-ranks timing.

Prints ONE JSON line on rank 0 with `roofline` (dominant kernel = the implicit-GEMM conv
forward/dgrad launches, each timed with HIP events on its launch stream over the timed
region; `traffic` = PMC HBM bytes per launch of the same workload from profiles/traffic/,
null when that workload has not been profiled) and `cpu_baseline` (the oracle's CPU
restatement of the same step on a bounded sample on this host's cores, plus the full-frame
fp32 parity of the HIP path against it).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BF16_DENSE_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: ~2.5 PF dense bf16 (no sparsity)
F32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: f32-input MFMA = the f32 vector peak
HBM_PEAK_GBPS = 8000.0
# f32 GEMMs through the 3-way bf16 split issue six bf16 MFMA products per f32 product: their
# f32-equivalent ceiling is the dense bf16 peak / 6
F32_SPLIT_PEAK_TFLOPS = BF16_DENSE_PEAK_TFLOPS / 6.0
# the f16 x3 arithmetic (default): three f16 MFMA products (same rate as bf16) per f32 product
F32_H16_PEAK_TFLOPS = BF16_DENSE_PEAK_TFLOPS / 3.0
PEAKS = {"fp32": F32_SPLIT_PEAK_TFLOPS, "fp32_exact": F32_MFMA_PEAK_TFLOPS, "bf16": BF16_DENSE_PEAK_TFLOPS,
         "fp16": BF16_DENSE_PEAK_TFLOPS}
H0, W0 = 768, 1024
F32_MATH_MODE = {"split": 1, "exact": 0, "h16": 2}  # dg_set_f32_math
METRIC = "train-step frames/sec at 768×1024, ShanghaiTech-A; MAE vs reference"
CONFIG_FILES = {"final": "configs/sta_final.yml", "simple": "configs/stb_reg_base.yml",
                "base": "configs/ablation (mode base)"}


def config_file(args):
    if args.model == "DensityRegressorBase" and args.height >= 2048:
        return "configs/qnrf_final.yml (dgnet, 2048-px crops)"
    if args.model == "DensityRegressorBase":
        return "configs/stb_reg_base.yml (dgnet)"
    return CONFIG_FILES.get(args.mode, "")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16, help="frames (samples) per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="strong scaling: this many samples per step over all ranks (per-rank batch = G / N)")
    ap.add_argument("--sync-bn", action="store_true",
                    help="nn.SyncBatchNorm.convert_sync_batchnorm: BN statistics over all ranks' samples")
    ap.add_argument("--mode", default="final", choices=["simple", "base", "final"])
    ap.add_argument("--model", default=None,
                    help="model class (default: DGModel_final for final mode, DGModel_base otherwise; "
                         "DensityRegressorBase = models2 'dgnet')")
    ap.add_argument("--trunk", default=None, choices=["ibn", "sw", "isw"],
                    help="secondary workload: ResNet-50 DG counter (IBN-b / SW / ISW) train step")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16", "fp16"])
    ap.add_argument("--no-bf16", action="store_true", help="skip the perf_bf16 leg")
    ap.add_argument("--f32-math", default="h16", choices=["split", "exact", "h16"],
                    help="f32 conv GEMM arithmetic: h16 (default: two scaled f16 parts per operand, three f16 MFMA "
                         "products, where the kernel has it; else the split), split (exact 3-way bf16 split, six "
                         "products) or exact (v_mfma_f32_16x16x4_f32)")
    ap.add_argument("--no-f32-exact", action="store_true", help="skip the f32_exact leg")
    ap.add_argument("--height", type=int, default=H0)
    ap.add_argument("--width", type=int, default=W0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the multi-rank plumbing (launcher, gloo ranks, per-rank timing "
                         "aggregation and the JSON line) with a toy step instead of the GPU workload")
    return ap.parse_args()


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`--gpus N` outside torchrun: one process per GPU via torch.distributed.run, started as
    a child (this process has not touched the GPU), whose rank 0 prints the JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__),
           *sys.argv[1:]]
    return subprocess.call(cmd)


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


def _vgg_layers(H, W):
    """(h, w, cin, cout, k, has_dgrad) of the encoder + decoder convs of DGModel_base."""
    layers, enc = [], []
    h, w, cin = H, W, 3
    for v in [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512]:
        if v == "M":
            h, w = h // 2, w // 2
            continue
        enc.append((h, w, cin, v, 9, cin != 3))
        cin = v
    s = H // 16, W // 16
    dec = [(s[0], s[1], 512, 1024, 9, True), (s[0], s[1], 1024, 512, 9, True),
           (2 * s[0], 2 * s[1], 1024, 512, 9, True), (2 * s[0], 2 * s[1], 512, 256, 9, True),
           (4 * s[0], 4 * s[1], 512, 256, 9, True), (4 * s[0], 4 * s[1], 256, 128, 9, True),
           (4 * s[0], 4 * s[1], 896, 256, 1, True)]
    return enc, dec


def step_flops(B, H, W, mode):
    """Algorithmic GEMM FLOPs of one train step (fwd + dgrad + wgrad), SURVEY.md §8d: the
    reference's op count (y_cat's 1x1 conv at H/4, the memory logits/readout bmm's)."""
    enc, dec = _vgg_layers(H, W)
    views = 2 if mode in ("final", "base") else 1
    tot = enc_tot = 0.0
    for i, (h, w, ci, co, k, dgrad) in enumerate(enc + dec):
        f = 2.0 * B * views * h * w * ci * co * k * (3 if dgrad else 2)
        tot += f
        if i < len(enc):
            enc_tot += f
    if mode == "final":
        hw = (H // 4) * (W // 4)
        tot += 2 * 3 * 2.0 * B * hw * 256 * 1024 * 2             # memory logits + readout, fwd/dgrad/wgrad
        tot += 2 * 3 * 2.0 * B * (H // 16) * (W // 16) * 512 * 256 * 9   # cls_head 3x3
    return tot, enc_tot


class ConvTimer:
    """Per-launch HIP events around the implicit-GEMM conv launches, recorded on torch's
    current stream — the stream the C-ABI launches on.  Kinds: 'fwd', 'dgrad' (forward GEMM
    kernels), 'wgrad', 'stem', 'stem_wgrad'; scope: 'enc' / 'dec' / 'head' (engine.py)."""

    def __init__(self):
        self.ev = []

    def __call__(self, kind, flops, launch, nbytes=0.0, scope="other"):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        launch()
        e.record()
        self.ev.append((kind, scope, s, e, flops, nbytes))

    def summary(self, kinds, scopes=None):
        torch.cuda.synchronize()
        ms = fl = nb = 0.0
        n = 0
        for k, sc, s, e, f, b in self.ev:
            if k in kinds and (scopes is None or sc in scopes):
                ms += s.elapsed_time(e)
                fl += f
                nb += b
                n += 1
        return ms, fl, n, nb

    def attainable(self, kinds, peak_tflops, peak_gbps=HBM_PEAK_GBPS):
        """Per-launch roofline: each launch's lower bound max(FLOP / MFMA peak, algorithmic bytes /
        HBM peak), summed over the launches, divided by their measured time.  For families that
        mix MFMA-bound and HBM-bound shapes (the ResNet trunks' 1x1 convs with K = 64..256 are
        at 25-60 FLOP/B, i.e. HBM-bound) this is the fraction of the attainable rate; the
        FLOP-only `frac` understates them.  Also the share of launches (by time) that are
        MFMA-bound."""
        torch.cuda.synchronize()
        tmin = tact = tmf = 0.0
        for k, _sc, s, e, f, b in self.ev:
            if k not in kinds:
                continue
            t = s.elapsed_time(e) * 1e-3
            tf, tb = f / (peak_tflops * 1e12), b / (peak_gbps * 1e9)
            tmin += max(tf, tb)
            tact += t
            if tf >= tb:
                tmf += t
        return (tmin / tact if tact else None), (tmf / tact if tact else None)


def build_model(args, precision, dev):
    from dgvcc_amd.models import models as MM
    if args.trunk:
        from dgvcc_amd.models import trunks as TM
        cls = {"ibn": TM.IBNCounter_ResNet, "sw": TM.SWCounter_ResNet, "isw": TM.ISWCounter_ResNet}
        return cls[args.trunk](pretrained=False).to(dev).set_precision(precision), \
            ("isw" if args.trunk == "isw" else "simple")
    name = args.model or ("DGModel_final" if args.mode == "final" else "DGModel_base")
    if name == "DensityRegressorBase":
        from dgvcc_amd.models import models2 as M2
        model = M2.DensityRegressorBase(pretrained=False)
    else:
        model = getattr(MM, name)(pretrained=False)
    return model.to(dev).set_precision(precision), args.mode


def traffic_key(args, precision):
    label = args.trunk or (args.model or args.mode)
    return f"{label}_{precision}_b{args.batch}_{args.height}x{args.width}"


def measured_traffic(args, precision):
    """PMC HBM bytes per conv forward/dgrad launch of THIS workload (tools/pmc_summary.py over a
    rocprofv3 FETCH_SIZE / WRITE_SIZE pass of the same bench command), or None."""
    path = os.path.join(ROOT, "profiles", "traffic", traffic_key(args, precision) + ".json")
    if not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
        return d.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    except (OSError, ValueError):
        return None, None


FWD_KERNEL_NAMES = {
    "fp32_split": "conv_fwd_psplit_kernel<256|128> + conv_fwd_rsplit3_kernel + conv_fwd_rsplit_kernel (implicit-GEMM "
            "conv, f32 operands split exactly into 3 bf16 parts, 6 x v_mfma_f32_16x16x32_bf16 per 32-deep block, "
            "f32 accumulation: forward + dgrad launches; peak = dense bf16 / 6)",
    "fp32_h16": "conv_fwd_psplit_kernel<256|128, HM> + conv_fwd_rsplit3w_kernel<HM> + split_x_h_kernel (the pixel "
                "operand's hi/lo pre-split pass of the dgrads, timed inside the same launch; the forwards read the "
                "pair image their BN apply wrote) (implicit-GEMM conv, each f32 "
                "operand scaled by a power of two and cut into two f16 parts, 3 x v_mfma_f32_16x16x32_f16 per "
                "32-deep block (hi*hi + hi*lo + lo*hi), f32 accumulation: forward + dgrad launches; peak = dense "
                "f16 / 3)",
    "fp32_exact": "conv_fwd_pers_kernel<float> (implicit-GEMM conv on v_mfma_f32_16x16x4_f32: forward + dgrad "
                  "launches)",
    "bf16": "conv_fwd_pers_kernel + conv_fwd_tap3p_kernel + conv_fwd_pipe_kernel + conv_fwd_tap3_kernel "
            "(implicit-GEMM conv on v_mfma_f32_16x16x32_bf16: forward + dgrad launches)",
    "fp16": "conv_fwd_pers_kernel + conv_fwd_tap3p_kernel + conv_fwd_pipe_kernel + conv_fwd_tap3_kernel "
            "(implicit-GEMM conv on v_mfma_f32_16x16x32_f16: forward + dgrad launches)",
}


def run_leg(args, precision, dev, world, rank):
    """Build, warm up and time one precision of the workload; returns the measurements.
    precision "fp32_exact" = fp32 with the conv GEMMs on v_mfma_f32_16x16x4_f32."""
    from dgvcc_amd import kernels as K
    K.call("dg_set_f32_math", 0 if precision == "fp32_exact" else F32_MATH_MODE[args.f32_math])
    precision = "fp32" if precision == "fp32_exact" else precision
    from dgvcc_amd.losses import MSELoss
    from dgvcc_amd.optim import AdamW
    from dgvcc_amd.trainers.dgtrainer import DGTrainer

    B, H, W = args.batch, args.height, args.width
    torch.manual_seed(2112)
    model, mode = build_model(args, precision, dev)
    if args.sync_bn:  # BN over the global batch (syncbn.py; a no-op for a single rank)
        model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
    if world > 1:  # identical init on every rank
        import torch.distributed as dist
        for t in model.state_dict().values():
            dist.broadcast(t, 0)
    opt = AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    dp = {"overlap": opt.reducer is not None,
          "bucket_mb": round(opt.reducer.bucket_bytes / (1 << 20), 3) if opt.reducer is not None else None}
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
        opt.comm_events = []  # the all-reduce's exposed parts, per step (optim.AdamW)
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = None
    for _ in range(args.steps):
        last = trainer.train_step(model, loss_fn, opt, batch, epoch)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    K.set_conv_timer(None)
    res = {"elapsed": elapsed, "last_loss": last, "mode": mode, "model": type(model).__name__}
    if world > 1:
        torch.cuda.synchronize()
        exposed = sum(a.elapsed_time(b) for pair in opt.comm_events for a, b in pair) / args.steps
        opt.comm_events = None
        res["allreduce"] = dict(dp, buckets=len(opt.reducer.buckets) if opt.reducer is not None else 1,
                                **dp_attribution(elapsed, exposed, args.steps, dev))
        res["elapsed"] = res["allreduce"]["step_ms_max"] * args.steps * 1e-3  # max over ranks
    else:  # the setting a --gpus N run of this command uses; one rank all-reduces nothing
        res["allreduce"] = dict(dp, buckets=None, exposed_ms=0.0, note="world size 1: no all-reduce runs")
    conv_ms, conv_flops, conv_n, conv_bytes = timer.summary(("fwd", "dgrad"))
    wg_ms, wg_flops, wg_n, _ = timer.summary(("wgrad",))
    enc_kinds = ("fwd", "dgrad", "wgrad", "stem", "stem_wgrad")
    enc_ms, enc_flops, _, _ = timer.summary(enc_kinds, scopes=("enc",))
    enc_gemm_ms, enc_gemm_flops, _, _ = timer.summary(("fwd", "dgrad", "wgrad"), scopes=("enc",))
    dump = os.environ.get("DGVCC_BENCH_LAUNCHES")
    if dump and rank == 0:  # per-launch (kind, scope, ms, GFLOP, MB) of the timed steps, for analysis
        torch.cuda.synchronize()
        with open(f"{dump}_{precision}.json", "w") as f:
            json.dump([(k, sc, s.elapsed_time(e), fl / 1e9, nb / 1e6) for k, sc, s, e, fl, nb in timer.ev], f)
    att, att_mf = timer.attainable(("fwd", "dgrad"), PEAKS[precision])
    watt, _ = timer.attainable(("wgrad",), PEAKS[precision])
    res.update(attainable_frac=att, mfma_bound_share=att_mf, wgrad_attainable_frac=watt)
    res.update(conv_ms=conv_ms, conv_flops=conv_flops, conv_n=conv_n, conv_bytes=conv_bytes,
               wg_ms=wg_ms, wg_flops=wg_flops, enc_ms=enc_ms, enc_flops=enc_flops,
               enc_gemm_ms=enc_gemm_ms, enc_gemm_flops=enc_gemm_flops)
    if world > 1:
        import torch.distributed as dist
        # data-parallel sanity check outside the timed region: identical parameters on every rank
        chk = torch.stack([p.detach().double().sum() for p in model.parameters()]).sum().reshape(1)
        hi, lo = chk.clone(), chk.clone()
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        res["params_in_sync"] = bool(hi.item() == lo.item())
    views = 2 if (mode in ("final", "base") and not args.trunk) else 1
    res["frames"] = B * views * world * args.steps
    del model, opt, trainer, batch
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


def dp_attribution(elapsed_s: float, exposed_ms: float, steps: int, device) -> dict:
    """Per-rank timing of a data-parallel run, gathered from every rank: step time
    (the timed region / steps) and the gradient all-reduce's exposed time per step (optim.AdamW
    comm_events: the compute stream's wait for the in-flight buckets + the blocking remainder).  The
    line's time is the max over ranks; the spread and the exposed share attribute a shortfall."""
    import torch.distributed as dist
    t = torch.tensor([elapsed_s / steps * 1e3, exposed_ms], dtype=torch.float64, device=device)
    rows = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(rows, t)
    step = [round(float(r[0]), 3) for r in rows]
    exp = [round(float(r[1]), 3) for r in rows]
    return {"step_ms_min": min(step), "step_ms_max": max(step), "step_ms_per_rank": step,
            "exposed_ms": max(exp), "exposed_ms_per_rank": exp,
            "exposed_note": "ms per step the compute stream waited on the gradient all-reduce (bucket waits + "
                            "the non-FeaturePlan remainder), HIP events; max over ranks"}


def dry_run(args, world, rank):
    """`--dry-run`: the multi-rank plumbing on CPU (gloo ranks from launch_ranks): a toy step
    (a matmul) and one blocking all-reduce of a flat 'gradient' per step, timed like run_leg, then
    dp_attribution and the JSON line.  tests/test_dist_cpu.py runs it at world 8."""
    import torch.distributed as dist
    from dgvcc_amd.dist import average_flat_
    a = torch.randn(256, 256)
    g = torch.randn(1 << 18)
    exposed = 0.0
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for _ in range(1 + rank % 2):  # an uneven load: the spread must show it
            a = torch.tanh(a @ a)
        t1 = time.perf_counter()
        average_flat_(g)
        exposed += (time.perf_counter() - t1) * 1e3
    dist.barrier()
    elapsed = time.perf_counter() - t0
    att = dp_attribution(elapsed, exposed / args.steps, args.steps, torch.device("cpu"))
    out = {"metric": METRIC, "value": round(world * args.steps / (att["step_ms_max"] * args.steps * 1e-3), 3),
           "unit": "toy steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "dry_run": True,
           "config": {"parallelism": f"dp{world}", "backend": "gloo", "allreduce": att}}
    if rank == 0:
        print(json.dumps(out), flush=True)


def roofline(args, precision, r):
    peak = PEAKS[precision]
    kkey = precision
    if precision == "fp32":
        kkey = {"h16": "fp32_h16", "split": "fp32_split", "exact": "fp32_exact"}[args.f32_math]
    kname = FWD_KERNEL_NAMES.get(kkey, "implicit-GEMM conv forward + dgrad")
    if args.trunk:  # ResNet-50 trunk: strided/non-"same" convs on conv_gen_kernel, 3x3/1x1 stride 1 as above
        kname = ("conv_gen_kernel (strided / 7x7 stem im2col / parity-class dgrad) + " + kname.split(" (")[0] +
                 " (ResNet-50 trunk convs: forward + dgrad launches)")
    precision = "fp32" if precision == "fp32_exact" else precision
    achieved = r["conv_flops"] / (r["conv_ms"] * 1e-3) / 1e12 if r["conv_ms"] > 0 else 0.0
    traffic, tsrc = measured_traffic(args, precision)
    steps = args.steps
    tot, enc_tot = step_flops(args.batch, args.height, args.width, r["mode"]) if not args.trunk else \
        ((r["conv_flops"] + r["wg_flops"]) / steps, None)
    step_s = r["elapsed"] / steps
    out = {"bound": "mfma", "kernel": kname,
           **({"f32_equivalent_frac_of_split6_ceiling": round(achieved / F32_SPLIT_PEAK_TFLOPS, 4)}
              if precision == "fp32" and args.f32_math == "h16" else {}),
           "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
           "traffic": traffic, "traffic_source": tsrc,
           "algorithmic_bytes_per_launch": round(r["conv_bytes"] / max(r["conv_n"], 1)),
           "algorithmic_flop_per_launch": round(r["conv_flops"] / max(r["conv_n"], 1)),
           "launches_per_step": r["conv_n"] // steps,
           "avg_launch_us": round(r["conv_ms"] * 1e3 / max(r["conv_n"], 1), 2),
           "kernel_ms_per_step": round(r["conv_ms"] / steps, 3),
           "wgrad_achieved": round(r["wg_flops"] / (r["wg_ms"] * 1e-3) / 1e12, 2) if r["wg_ms"] > 0 else None,
           "wgrad_frac": round(r["wg_flops"] / (r["wg_ms"] * 1e-3) / 1e12 / peak, 4) if r["wg_ms"] > 0 else None,
           "wgrad_ms_per_step": round(r["wg_ms"] / steps, 3),
           "attainable_frac": round(r["attainable_frac"], 4) if r.get("attainable_frac") else None,
           "mfma_bound_time_share": round(r["mfma_bound_share"], 4) if r.get("mfma_bound_share") else None,
           "wgrad_attainable_frac": round(r["wgrad_attainable_frac"], 4) if r.get("wgrad_attainable_frac") else None,
           "step_gemm_tflop_algorithmic": round(tot / 1e12, 4),
           "whole_step_mfma_frac": round(tot / step_s / 1e12 / peak, 4)}
    if r["enc_ms"] > 0:
        # encoder only (enc1-enc3 of vgg16_bn.features: fwd + dgrad + wgrad launches, measured
        # per launch; the fused bf16 stem's launches included in the first figure)
        out["encoder_achieved"] = round(r["enc_flops"] / (r["enc_ms"] * 1e-3) / 1e12, 2)
        out["encoder_frac"] = round(out["encoder_achieved"] / peak, 4)
        out["encoder_ms_per_step"] = round(r["enc_ms"] / steps, 3)
        if r["enc_gemm_ms"] > 0:
            out["encoder_gemm_frac"] = round(r["enc_gemm_flops"] / (r["enc_gemm_ms"] * 1e-3) / 1e12 / peak, 4)
    if enc_tot is not None:
        out["encoder_tflop_per_step_algorithmic"] = round(enc_tot / 1e12, 4)
    return out


def dmap_roofline(args, dev, reps=20):
    """The Gaussian density-map scatter (utils/dmap_gen.py:53-81) for one batch of the
    workload's synthetic frames: algorithmic bytes 4*H*W (the map, written once) + 8*N (the
    points) per frame over the launch time, HIP events on the launch stream."""
    from dgvcc_amd.utils.dmap_gen import gaussian_filter_density_fixed_batch
    B, H, W = args.batch, args.height, args.width
    g = torch.Generator(device="cpu").manual_seed(1000)
    n = torch.poisson(torch.full((B,), 500.0 * H * W / (H0 * W0)), generator=g).long().clamp_min(1)
    pts = [(torch.rand(int(k), 2, generator=g) * torch.tensor([W, H], dtype=torch.float32)).to(dev) for k in n]
    nbytes = 4.0 * B * H * W + 8.0 * int(n.sum())
    out = {"bound": "hbm", "peak": 8000.0, "unit": "GB/s", "frames": B, "points": int(n.sum()),
           "algorithmic_bytes_per_launch": nbytes}
    from dgvcc_amd import kernels as K
    flat = torch.cat(pts).contiguous()
    offs = torch.tensor([0] + torch.cumsum(n, 0).tolist(), dtype=torch.int64, device=dev)
    ref = gaussian_filter_density_fixed_batch(pts, H, W, deterministic=True)
    for det in (True, False):
        # the ABI launches alone (points and offsets already on the device, as the data path has them),
        # captured in a HIP graph so the events time the kernels, not the host's per-call overhead
        out_t = K.dmap_fixed(flat, offs, B, H, W, deterministic=det)
        if det:
            out["deterministic_equals_batch_api"] = bool(torch.equal(out_t, ref))
        graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            K.dmap_fixed(flat, offs, B, H, W, deterministic=det)  # warm the allocator on the capture stream
            with torch.cuda.graph(graph, stream=side):
                for _ in range(reps):
                    K.dmap_fixed(flat, offs, B, H, W, deterministic=det)
        torch.cuda.current_stream().wait_stream(side)
        graph.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        graph.replay()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / reps
        del graph
        key = "deterministic" if det else "atomic"
        out[key] = {"us_per_launch": round(us, 2), "achieved": round(nbytes / (us * 1e-6) / 1e9, 1),
                    "frac": round(nbytes / (us * 1e-6) / 1e9 / 8000.0, 4)}
    # the write floor of the same map: a plain fill of the [B][H][W] f32 tensor, timed the same way
    fill = torch.empty((B, H, W), dtype=torch.float32, device=dev)
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fill.fill_(1.0)
        with torch.cuda.graph(graph, stream=side):
            for _ in range(reps):
                fill.fill_(1.0)
    torch.cuda.current_stream().wait_stream(side)
    graph.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    graph.replay()
    e.record()
    torch.cuda.synchronize()
    us_fill = s.elapsed_time(e) * 1e3 / reps
    del graph
    out["fill_floor"] = {"us_per_launch": round(us_fill, 2), "achieved": round(4.0 * B * H * W / (us_fill * 1e-6) / 1e9, 1),
                         "note": "torch fill_ of the same map (write-only floor of this launch shape)"}
    out["deterministic"]["frac_of_fill_floor"] = round(us_fill / out["deterministic"]["us_per_launch"], 4)
    out["kernel"] = ("dmap_fixed_fused_kernel (default, 1 launch: one block per 64x64 tile "
                     "walks its image's points in order, bit-identical to the reference) / memset + dmap_fixed_kernel "
                     "(f32 atomics)")
    return out


def bl_timing(args, dev, reps=20):
    """sta_final's BL leg (SURVEY.md §8 config mapping): losses/bl.py BL(points, st_sizes,
    targets, pre_density) forward + backward on the workload's frames, with the synthetic BL
    parameters of SURVEY.md (sigma 8, background ratio 1, background row on, c_size 768,
    stride 8: the x8 avg-pooled density on a 96 x 96 grid of the frame's 768 x 768 crop).
    Work unit: one (row, cell) posterior term -- rows = points + one background row per image,
    cells = G^2 -- evaluated in each of the kernel's three exp passes (statistics, counts,
    gradient); VALU/transcendental-bound, so the line reports the rate, not an HBM fraction."""
    from dgvcc_amd.losses.bl import BL
    B, c_size, stride = args.batch, 768, 8
    G = c_size // stride
    g = torch.Generator(device="cpu").manual_seed(1001)
    n = torch.poisson(torch.full((B,), 500.0 * c_size * c_size / (H0 * W0)), generator=g).long().clamp_min(1)
    pts = [(torch.rand(int(k), 2, generator=g) * c_size).to(dev) for k in n]
    tg = [torch.ones(int(k), device=dev) for k in n]
    st = [float(c_size)] * B
    dens = torch.rand(B, 1, G, G, generator=g).to(dev).requires_grad_(True)
    crit = BL(8.0, c_size, stride, 1.0, True, dev)
    for _ in range(3):
        crit(pts, st, tg, dens).backward()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        dens.grad = None
        loss = crit(pts, st, tg, dens)
        loss.backward()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / reps
    terms = 3.0 * (int(n.sum()) + B) * G * G
    return {"us_per_step": round(us, 2), "frames": B, "points": int(n.sum()), "grid": f"{G}x{G}",
            "posterior_terms_per_s": round(terms / (us * 1e-6), 1), "bound": "valu (exp per posterior term)",
            "loss": round(float(loss.item()), 4),
            "note": "fwd + bwd through the autograd path (host packing of the point lists included)"}


def cpu_baseline(args, seconds):
    """The oracle's CPU restatement of the same train step (kind 'port'), batch 1, fp32, on this
    host's cores, plus the full-frame fp32 parity of the HIP path on the warm-up frame.

    The host's best stated configuration: torch CPU's conv / GEMM threading does
    not scale across sockets on batch-1 frames, so one step is timed at each thread count of a sweep
    (16, 32, 64, ..., the physical cores; DGVCC_CPU_THREADS pins one count), and `value` is the mean of
    >= 2 further timed steps at the fastest count (mean of >= 2 timed steps)."""
    from oracle import dg_oracle as O
    from dgvcc_amd.models.models import DGModel_base, DGModel_final
    nproc = os.cpu_count() or 1
    phys = _physical_cores()
    pinned = int(os.environ.get("DGVCC_CPU_THREADS", "0") or 0)
    sweep = [pinned] if pinned else sorted({t for t in (16, 32, 64, 128, 256) if t < phys} | {phys})
    prev = torch.get_num_threads()
    mode = args.mode if args.mode in ("simple", "final") else "simple"
    tmpl = (DGModel_final(pretrained=False) if mode == "final" else DGModel_base(pretrained=False)).state_dict()
    sd = O.seeded_state_dict(tmpl)
    batch = O.synthetic_batch(1, args.height, args.width, seed=7)
    torch.set_num_threads(sweep[0])
    t0 = time.perf_counter()
    loss_ref, outs, _, _ = O.train_step(sd, batch, mode)  # warm-up, and the parity reference below
    t_warm = time.perf_counter() - t0
    torch.set_num_threads(prev)
    parity = density_parity(sd, batch, loss_ref, outs, mode)
    frames_per_step = 2 if mode == "final" else 1
    probe = {}
    for t in sweep:  # one step per thread count (the pool resized before it)
        torch.set_num_threads(t)
        t0 = time.perf_counter()
        O.train_step(sd, batch, mode)
        probe[t] = time.perf_counter() - t0
    best = min(probe, key=probe.get)
    torch.set_num_threads(best)
    n, t0 = 0, time.perf_counter()
    while True:
        O.train_step(sd, batch, mode)
        n += 1
        if n >= 2 and (time.perf_counter() - t0 >= seconds / 2 or n >= 8):
            break
    dt = time.perf_counter() - t0
    torch.set_num_threads(prev)
    return {"value": n * frames_per_step / dt, "unit": "frames/s", "cores": best, "kind": "port",
            "threads_sweep": {str(t): round(frames_per_step / v, 4) for t, v in probe.items()},
            "threads_sweep_unit": "frames/s of one step at each torch CPU thread count",
            "host_nproc": nproc, "host_physical_cores": phys, "cpu_model": _cpu_model(),
            "warmup_step_s": round(t_warm, 2),
            "sample": f"{n} timed oracle train steps ({mode} mode, batch 1 = {frames_per_step} frame(s) of "
                      f"{args.height}x{args.width}, fp32, torch CPU {best} threads: the fastest of the sweep) after "
                      f"1 warm-up step and one step per swept thread count",
            "parity": parity}


def _physical_cores() -> int:
    """Physical cores this process may run on: distinct (package, core) pairs of /proc/cpuinfo
    among the CPUs of its affinity mask (SMT siblings counted once)."""
    try:
        allowed = os.sched_getaffinity(0)
    except (AttributeError, OSError):
        allowed = set(range(os.cpu_count() or 1))
    cores, cpu, pkg = set(), None, "0"
    try:
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "processor":
                cpu, pkg = int(v), "0"
            elif k == "physical id":
                pkg = v
            elif k == "core id" and cpu in allowed:
                cores.add((pkg, v))
    except OSError:
        pass
    return len(cores) or len(allowed) or 1


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def density_parity(sd, batch, loss_ref, outs_ref, mode):
    """The metric's "MAE vs reference" on the warm-up frame: the HIP path in fp32 (north_star's
    parity precision) against the oracle for the same weights and frame, for both f32 conv
    arithmetics (the headline 3-way split, and v_mfma_f32_16x16x4_f32 under `f32_exact`).  Final
    mode: the oracle is re-run on the HIP path's own threshold decisions (e_mask, class maps) and
    the number of decisions that differ is reported; the loss is compared as is."""
    from dgvcc_amd import kernels as K
    math_mode = int(K.lib_call_status("dg_get_f32_math"))
    try:
        res = _density_parity_once(sd, batch, loss_ref, outs_ref, mode, grads=True)
        K.call("dg_set_f32_math", 0)
        ex = _density_parity_once(sd, batch, loss_ref, outs_ref, mode)
    finally:
        K.call("dg_set_f32_math", math_mode)
    res["f32_math"] = {1: "split", 2: "h16"}.get(math_mode, str(math_mode))
    res["f32_exact"] = {k: v for k, v in ex.items() if k not in ("precision", "frame", "tolerance_rel", "note")}
    return res


def _density_parity_once(sd, batch, loss_ref, outs_ref, mode, grads=False):
    """grads (final mode): also the train step's backward, HIP against the oracle's step on the
    HIP decisions: per-parameter normwise gradient errors and each loss term's relative error
    (the whole loss is dominated by the MSE x 1000 term at random init, so it alone is no check)."""
    from oracle import dg_oracle as O
    from dgvcc_amd.models.models import DGModel_base, DGModel_final
    from dgvcc_amd.losses import mse_loss
    from dgvcc_amd.losses.bce import binary_cross_entropy
    dev = torch.device("cuda", torch.cuda.current_device())
    img1, img2, (pts, dmaps, bmaps) = batch
    if mode == "final":
        model = DGModel_final(pretrained=False, den_dropout=0.0, cls_dropout=0.0)
    else:
        model = DGModel_base(pretrained=False, den_dropout=0.0)
    model.load_state_dict(sd)
    model = model.to(dev).set_precision("fp32").train()
    res = {"precision": "fp32", "frame": "1x3x%dx%d" % tuple(img1.shape[-2:]), "tolerance_rel": 1e-4}
    with torch.set_grad_enabled(grads and mode == "final"):
        if mode == "final":
            plan = model._get_plans()["pair"]
            plan.capture = {}
            gb = bmaps.to(dev)
            dc1, dc2, c1, c2, _, loss_con, _ = model.forward_train(img1.to(dev), img2.to(dev), gb)
            gt = dmaps.to(dev)
            terms = (mse_loss(dc1, gt, 1000.0) + mse_loss(dc2, gt, 1000.0),
                     binary_cross_entropy(c1, gb) + binary_cross_entropy(c2, gb), loss_con)
            loss = terms[0] + 10 * terms[1] + 10 * terms[2]
            if grads:
                loss.backward()
            cap = plan.capture
            plan.capture = None
            em = cap["emask"].permute(0, 3, 1, 2).bool().cpu()
            cp = tuple(c.cpu() for c in cap["c_pred"])
            info = {}
            sd2 = {k: v.clone() for k, v in sd.items()}
            with torch.no_grad():
                r1, r2, rc1, rc2, _, rcon, _ = O.final_forward(sd2, img1, img2, bmaps, e_mask_in=em, c_pred_in=cp,
                                                               info=info)
            rt = (torch.nn.functional.mse_loss(r1, dmaps * 1000.0) + torch.nn.functional.mse_loss(r2, dmaps * 1000.0),
                  torch.nn.functional.binary_cross_entropy(rc1, bmaps)
                  + torch.nn.functional.binary_cross_entropy(rc2, bmaps), rcon)
            res["loss_terms_rel"] = {k: float(abs(a.item() - b.item()) / abs(b.item()))
                                     for k, a, b in zip(("mse", "bce", "jsd_mse"), terms, rt)}
            pairs = [(dc1, r1), (dc2, r2)]
            res.update({k: v for k, v in info.items()})
            res["note"] = ("oracle re-run on the HIP path's e_mask / class-map decisions; flips = decisions "
                           "within fp32 rounding of the threshold")
            res["loss_rel_uninjected"] = float(abs(loss.item() - loss_ref.item()) / abs(loss_ref.item()))
            if grads:
                _, _, g_ref, _ = O.train_step(sd, batch, "final", e_mask_in=em, c_pred_in=cp)
                err, num, den = {}, 0.0, 0.0
                for k, p in model.named_parameters():
                    if (k.endswith(".bias") and (k.startswith("enc") or ".conv." in k)) or g_ref[k].norm() == 0:
                        continue  # pre-BN conv biases: mathematically zero gradient
                    d = p.grad.detach().double().cpu() - g_ref[k].double()
                    err[k] = float(d.norm() / g_ref[k].double().norm())
                    num += float(d.norm() ** 2)
                    den += float(g_ref[k].double().norm() ** 2)
                worst = max(err.items(), key=lambda kv: kv[1])
                # both against the float64 oracle on the same decisions: the fp32 oracle's own spread
                # beside the HIP step's (tests/test_model_gpu.py test_step_grads_full_frame criterion)
                sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
                b64 = (img1.double(), img2.double(), (pts, dmaps.double(), bmaps.double()))
                _, _, g64, _ = O.train_step(sd64, b64, "final", e_mask_in=em, c_pred_in=cp)
                e64, e32, n64, n32, d64 = {}, {}, 0.0, 0.0, 0.0
                for k in err:
                    mine = dict(model.named_parameters())[k].grad.detach().double().cpu()
                    r = g64[k].double()
                    e64[k] = float((mine - r).norm() / r.norm())
                    e32[k] = float((g_ref[k].double() - r).norm() / r.norm())
                    n64 += float((mine - r).norm() ** 2)
                    n32 += float((g_ref[k].double() - r).norm() ** 2)
                    d64 += float(r.norm() ** 2)
                w64 = max(e64.items(), key=lambda kv: kv[1])
                g_hip, g_or = (n64 / d64) ** 0.5, (n32 / d64) ** 0.5
                ok = all(v <= max(2 * e32[k], 1.5e-2) for k, v in e64.items()) and g_hip <= max(2 * g_or, 1.2e-2)
                res["grad_parity"] = {"worst_param": worst[0], "worst_normwise_rel": worst[1],
                                      "global_normwise_rel": (num / den) ** 0.5, "params": len(err),
                                      "vs_float64": {"worst_param": w64[0], "worst_normwise_rel": w64[1],
                                                     "fp32_oracle_there": e32[w64[0]],
                                                     "fp32_oracle_worst": max(e32.values()),
                                                     "global_normwise_rel": g_hip,
                                                     "fp32_oracle_global": g_or,
                                                     "within_criterion": bool(ok),
                                                     "criterion": "per param <= max(2 x fp32 oracle, 1.5e-2); "
                                                                  "global <= max(2 x fp32 oracle, 1.2e-2)"},
                                      "note": "HIP fp32 step backward against the fp32 oracle's step on the HIP "
                                              "decisions; ReLU / max-pool branches are each side's own, so the "
                                              "residual is their fp32 spread (tests/test_model_gpu.py E2E_GRAD_TOL); "
                                              "vs_float64: both against the float64 oracle on the same decisions"}
        else:
            d = model(img1.to(dev))
            loss = mse_loss(d, dmaps.to(dev), 1000.0)
            pairs = [(d, outs_ref[0])]
            res["loss_rel"] = float(abs(loss.item() - loss_ref.item()) / abs(loss_ref.item()))
    torch.cuda.synchronize()
    mae = mx = cnt = 0.0
    for d, r in pairs:
        d = d.detach().double().cpu()
        r = r.detach().double()
        mae = max(mae, float((d - r).abs().mean()))
        mx = max(mx, float((d - r).abs().max() / r.abs().max()))
        cnt = max(cnt, float(abs(d.sum() - r.sum()) / 1000.0))
    res.update(density_map_mae=mae, density_map_max_rel=mx, count_abs_err=cnt)
    del model
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.f32_math == "h16":  # the fp32 legs' ceiling is that of the arithmetic they run
        PEAKS["fp32"] = F32_H16_PEAK_TFLOPS
    if args.global_batch is not None:  # strong scaling: the global batch is fixed, split over the ranks
        if args.global_batch % world:
            raise SystemExit(f"bench.py: --global-batch {args.global_batch} does not split over {world} ranks")
        args.batch = args.global_batch // world
    # DGVCC_BENCH_BACKEND=gloo: rehearsal of the multi-rank path with several ranks sharing one
    # GPU (local rank modulo the visible devices); the driver's runs use RCCL ("nccl").
    backend = os.environ.get("DGVCC_BENCH_BACKEND", "nccl")
    if args.dry_run:  # CPU ranks only: nothing below touches a GPU
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            dry_run(args, world, rank)
            dist.destroy_process_group()
        return
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    dist_world = 1
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        dist_world = dist.get_world_size()
        assert dist_world == args.gpus, (dist_world, args.gpus)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    prec = args.precision
    leg = "fp32_exact" if prec == "fp32" and args.f32_math == "exact" else prec
    r = run_leg(args, leg, dev, world, rank)
    value = r["frames"] / r["elapsed"]
    workload = (f"{r['model']} {r['mode']}-mode DGTrainer.train_step (configs/baselines/sta_{args.trunk}.yml)"
                if args.trunk else
                f"{r['model']} {r['mode']}-mode DGTrainer.train_step ({config_file(args)}: "
                + ("two views, MSE x log_para 1000 + 10 BCE(class maps) + 10 JSD-MSE, AdamW"
                   if r["mode"] == "final" else "MSE x log_para 1000, AdamW") + ")")
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(r["elapsed"] / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.global_batch is not None else "weak",
        "vs_baseline": None,
        "dtype": prec,
        "data": f"synthetic 3x{args.height}x{args.width} frames (view 2 = view 1 + 0.1 N(0,1)) + Poisson(500) "
                "point sets, dmap via the HIP scatter, HBM-resident; random-init weights",
        "config": {"workload": workload, "global_batch": args.batch * world,
                   "frames_per_gpu_step": r["frames"] // (world * args.steps),
                   "resolution": f"{args.height}x{args.width}", "parallelism": f"dp{world}",
                   "batch_per_gpu": args.batch, "sync_bn": bool(args.sync_bn),
                   "rccl_world_size": dist_world, "backend": backend if world > 1 else None,
                   "last_loss": r["last_loss"]},
        "roofline": roofline(args, leg, r),
    }
    if prec == "fp32":
        out["f32_math"] = ("v_mfma_f32_16x16x4_f32" if leg != "fp32" else
                           "f16 x3: each f32 operand scaled by a power of two into f16 range and cut into two f16 "
                           "parts by nearest rounding, 3 f16 MFMA products per f32 product (hi*hi + hi*lo + lo*hi), "
                           "f32 accumulation, exact rescale (DESIGN.md §3.1)" if args.f32_math == "h16" else
                           "exact 3-way bf16 split of both f32 operands, 6 bf16 MFMA products per f32 product, "
                           "f32 accumulation")
    if "params_in_sync" in r:
        out["params_in_sync"] = r["params_in_sync"]
    if "allreduce" in r:  # the gradient all-reduce: bucketed and overlapped with the backward
        out["config"]["allreduce"] = r["allreduce"]
    if leg == "fp32" and not args.no_f32_exact:
        re_ = run_leg(args, "fp32_exact", dev, world, rank)
        out["f32_exact"] = {"value": round(re_["frames"] / re_["elapsed"], 3), "unit": "frames/s", "dtype": "fp32",
                            "ms_per_step": round(re_["elapsed"] / args.steps * 1e3, 3),
                            "note": "same fp32 workload with the conv GEMMs on v_mfma_f32_16x16x4_f32",
                            "last_loss": re_["last_loss"], "roofline": roofline(args, "fp32_exact", re_)}
        K_ = __import__("dgvcc_amd.kernels", fromlist=["call"])
        K_.call("dg_set_f32_math", F32_MATH_MODE[args.f32_math])
    if prec == "fp32" and not args.no_bf16:
        rb = run_leg(args, "bf16", dev, world, rank)
        out["perf_bf16"] = {"value": round(rb["frames"] / rb["elapsed"], 3), "unit": "frames/s", "dtype": "bf16",
                            "ms_per_step": round(rb["elapsed"] / args.steps * 1e3, 3),
                            "note": "same workload in bf16 storage/MFMA with f32 accumulation, statistics and "
                                    "losses (a perf mode; not the headline value)",
                            "last_loss": rb["last_loss"], "roofline": roofline(args, "bf16", rb)}
        if "params_in_sync" in rb:
            out["perf_bf16"]["params_in_sync"] = rb["params_in_sync"]
    if rank == 0 and not args.trunk:
        out["dmap"] = dmap_roofline(args, dev)
        out["bl"] = bl_timing(args, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.trunk:
        out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
        __import__("dgvcc_amd.kernels", fromlist=["call"]).call("dg_set_f32_math", F32_MATH_MODE[args.f32_math])
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
