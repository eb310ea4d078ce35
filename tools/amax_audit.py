"""Which f32 conv launches of one training step reach the library without an operand maximum
(so dgvcc computes it with its own amax pass): one warm-up step, then one audited step of the
bench workload, counting the conv entry points called with a NULL xamax / dyamax by caller.
usage: python tools/amax_audit.py [--trunk ibn|sw|isw] [--batch B] [--height H] [--width W]"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from dgvcc_amd import _capi, kernels as K  # noqa: E402

# entry -> argument indices (from the end, before the stream) of its operand maxima
AMAX_ARGS = {"dg_conv_fwd_ex": {"x": -2}, "dg_conv_fwd_bn_eval": {"x": -2}, "dg_conv_fwd_acc_relu": {"dy": -2},
             "dg_conv_fwd_bnbwd": {"dy": -2}, "dg_conv_wgrad": {"x": -3, "dy": -2},
             "dg_conv2d_wgrad": {"x": -3, "dy": -2}}
NO_AMAX = ()  # dg_conv2d_fwd / dg_conv2d_dgrad run exact f32 (conv_gen_kernel): no operand maxima

ap = argparse.ArgumentParser()
ap.add_argument("--trunk", default=None)
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--height", type=int, default=768)
ap.add_argument("--width", type=int, default=1024)
a = ap.parse_args()
sys.argv = ["bench.py", "--batch", str(a.batch), "--height", str(a.height), "--width", str(a.width)] + \
    (["--trunk", a.trunk] if a.trunk else [])
args = bench.parse()
dev = torch.device("cuda")
K.call("dg_set_f32_math", 2)
from dgvcc_amd.losses import MSELoss  # noqa: E402
from dgvcc_amd.optim import AdamW  # noqa: E402
from dgvcc_amd.trainers.dgtrainer import DGTrainer  # noqa: E402

torch.manual_seed(2112)
model, mode = bench.build_model(args, "fp32", dev)
opt = AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
os.makedirs("/tmp/dgvcc_bench", exist_ok=True)
cwd = os.getcwd()
os.chdir("/tmp/dgvcc_bench")
trainer = DGTrainer(2112, "audit", dev, 1000, 10000, mode)
os.chdir(cwd)
batch = bench.synthetic(a.batch, a.height, a.width, dev, seed=1000)
epoch = 0
if a.trunk == "isw":
    model.eval()
    with torch.no_grad():
        model([batch[0], batch[1]], cal_covstat=True)
    epoch = 6
model.train()
trainer.train_step(model, MSELoss(), opt, batch, epoch)
torch.cuda.synchronize()

miss = collections.Counter()
real_call, real_status = _capi.call, _capi.lib_call_status


def where():
    fr = [f for f in traceback.extract_stack()[:-3] if "dgvcc_amd" in f.filename and "kernels.py" not in f.filename]
    return " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in fr[-3:][::-1])


def audit(name, args):
    if name == "dg_amax":  # an explicit operand-max pass (kernels.amax)
        miss[(name, "pass", where())] += 1
    elif name in AMAX_ARGS:
        for op, i in AMAX_ARGS[name].items():
            if args[i] is None:
                miss[(name, op, where())] += 1
    elif name in NO_AMAX and args[0] == 0:
        miss[(name, "x+dy (no amax ABI)", where())] += 1


def call(name, *args):
    audit(name, args)
    return real_call(name, *args)


def status(name, *args):
    audit(name, args)
    return real_status(name, *args)


K.call, K.lib_call_status = call, status
trainer.train_step(model, MSELoss(), opt, batch, epoch)
torch.cuda.synchronize()
K.call, K.lib_call_status = real_call, real_status
tot = 0
for (name, op, w), n in sorted(miss.items(), key=lambda kv: -kv[1]):
    print(f"{n:4d}  {name:22s} {op:20s} {w}")
    tot += n
print(f"total: {tot} (conv launches without an operand maximum + explicit dg_amax passes)")
