"""Per-shape conv launch times of one training step of a bench workload: every implicit-GEMM
launch (fwd / dgrad / wgrad / stem) timed with HIP events on the launch stream, grouped by
(kind, entry point, N, H, W, C, Cout, R, stride), with its algorithmic bytes and FLOP and the
fraction of the per-launch roofline max(FLOP / MFMA peak, bytes / HBM peak) it reaches.
usage: python tools/conv_shapes.py [--trunk sw] [--precision bf16] [--out file.json]"""
import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from dgvcc_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--trunk", default=None)
ap.add_argument("--precision", default="bf16")
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--out", default=None)
a = ap.parse_args()
sys.argv = ["bench.py", "--batch", str(a.batch), "--precision", a.precision] + (["--trunk", a.trunk] if a.trunk else [])
args = bench.parse()
dev = torch.device("cuda")
K.call("dg_set_f32_math", 2)
from dgvcc_amd.losses import MSELoss  # noqa: E402
from dgvcc_amd.optim import AdamW  # noqa: E402
from dgvcc_amd.trainers.dgtrainer import DGTrainer  # noqa: E402

torch.manual_seed(2112)
model, mode = bench.build_model(args, a.precision, dev)
opt = AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
os.makedirs("/tmp/dgvcc_bench", exist_ok=True)
cwd = os.getcwd()
os.chdir("/tmp/dgvcc_bench")
trainer = DGTrainer(2112, "shapes", dev, 1000, 10000, mode)
os.chdir(cwd)
batch = bench.synthetic(args.batch, args.height, args.width, dev, seed=1000)
epoch = 0
if a.trunk == "isw":
    model.eval()
    with torch.no_grad():
        model([batch[0], batch[1]], cal_covstat=True)
    epoch = 6
model.train()
for _ in range(2):
    trainer.train_step(model, MSELoss(), opt, batch, epoch)
torch.cuda.synchronize()

# entry -> argument indices of (N, H, W, C, Cout, R[, stride])
SHAPE_ARGS = {"dg_conv_fwd_ex": (3, 4, 5, 6, 8, 9), "dg_conv_fwd_bnbwd": (3, 4, 5, 6, 8, 9),
              "dg_conv_fwd_acc_relu": (3, 4, 5, 6, 8), "dg_conv_wgrad": (3, 4, 5, 6, 9, 10),
              "dg_conv2d_fwd": (3, 4, 5, 6, 8, 9, 11), "dg_conv2d_dgrad": (3, 4, 5, 6, 8, 11, 13),
              "dg_conv2d_wgrad": (3, 4, 5, 6, 9, 10, 12)}
peak_tf = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 2500.0 / 3}[a.precision]
rec = []
real_call, real_status = K.call, K.lib_call_status


class Timer:
    def __call__(self, kind, flops, launch, nbytes=0.0, scope="other"):
        seen = []

        def spy(fn):
            def f(name, *xs):
                seen.append((name, xs))
                return fn(name, *xs)
            return f
        K.call, K.lib_call_status = spy(real_call), spy(real_status)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        try:
            launch()
        finally:
            K.call, K.lib_call_status = real_call, real_status
        e.record()
        name, xs = seen[-1] if seen else ("?", ())
        idx = SHAPE_ARGS.get(name)
        shape = tuple(xs[i] for i in idx) if idx else ()
        rec.append((kind, name, shape, s, e, flops, nbytes))


K.set_conv_timer(Timer())
trainer.train_step(model, MSELoss(), opt, batch, epoch)
torch.cuda.synchronize()
K.set_conv_timer(None)
agg = collections.OrderedDict()
for kind, name, shape, s, e, fl, nb in rec:
    k = (kind, name, shape)
    g = agg.setdefault(k, [0, 0.0, 0.0, 0.0])
    g[0] += 1
    g[1] += s.elapsed_time(e)
    g[2] += fl
    g[3] += nb
rows = []
tot = sum(v[1] for v in agg.values())
for (kind, name, shape), (n, ms, fl, nb) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    t_min = max(fl / (peak_tf * 1e12), nb / 8e12) * 1e3
    rows.append({"kind": kind, "entry": name, "args": shape, "n": n, "ms": round(ms, 3), "share": round(ms / tot, 4),
                 "GBps": round(nb / (ms * 1e-3) / 1e9, 1), "TFps": round(fl / (ms * 1e-3) / 1e12, 1),
                 "roofline_frac": round(t_min / ms, 3), "bound": "hbm" if nb / 8e12 > fl / (peak_tf * 1e12) else "mfma"})
print(f"{len(rec)} conv launches, {tot:.3f} ms")
for r in rows:
    print(f"{r['ms']:8.3f} {r['share']:6.1%} n{r['n']:3d} {r['kind']:6s} {r['entry']:18s} {str(r['args']):44s} "
          f"{r['GBps']:7.1f} GB/s {r['TFps']:7.1f} TF/s  roof {r['roofline_frac']:.2f} ({r['bound']})")
if a.out:
    json.dump({"precision": a.precision, "trunk": a.trunk, "total_ms": tot, "rows": rows}, open(a.out, "w"), indent=1)
