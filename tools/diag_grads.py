"""Per-parameter gradient error of the HIP fp32 path vs a float64 oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from oracle import dg_oracle as O
from dgvcc_amd.models.models import DGModel_base
from dgvcc_amd.losses import mse_loss

dev = torch.device("cuda")
B, H, W = 2, 64, 64
m = DGModel_base(pretrained=False, den_dropout=0.0)
sd0 = O.seeded_state_dict(m.state_dict())
m.load_state_dict(sd0)
m = m.to(dev).set_precision("fp32").train()
batch = O.synthetic_batch(B, H, W, seed=2112)
i1, i2, (pts, dm, bm) = batch

# (a) feature net only, fixed upstream gradient on ycat
g = torch.Generator().manual_seed(1)
gy = torch.randn(B, 896, H // 4, W // 4, generator=g)
sd64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in sd0.items()}
keys = O.trainable_keys(sd64)
for k in keys: sd64[k].requires_grad_(True)
yc64, _ = O.forward_fe(sd64, i1.double(), True)
ref = torch.autograd.grad((yc64 * gy.double()).sum(), [sd64[k] for k in keys], allow_unused=True)
ref = dict(zip(keys, ref))
sd32 = {k: v.clone() for k, v in sd0.items()}
for k in keys: sd32[k].requires_grad_(True)
yc32, _ = O.forward_fe(sd32, i1, True)
r32 = dict(zip(keys, torch.autograd.grad((yc32 * gy).sum(), [sd32[k] for k in keys], allow_unused=True)))
ycat, x3 = m._forward_fe_nhwc(i1.to(dev))
(ycat.permute(0, 3, 1, 2).float() * gy.to(dev)).sum().backward()
print("== feature net, fixed g_ycat ==")
for k, p in m.named_parameters():
    if k not in ref or ref[k] is None or ref[k].norm() == 0: continue
    if p.grad is None: print("NOGRAD", k); continue
    e = ((p.grad.double().cpu() - ref[k]).norm() / ref[k].norm()).item()
    e32 = ((r32[k].double() - ref[k]).norm() / ref[k].norm()).item()
    flag = "  <<<" if e > max(2 * e32, 1e-4) else ""
    print(f"{k:28s} hip {e:.2e}  cpu32 {e32:.2e}{flag}")
