import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from oracle import dg_oracle as O
from dgvcc_amd.models import models as M
dev = torch.device("cuda")
g = torch.Generator().manual_seed(9)
m = M.DGModel_mem(pretrained=False, den_dropout=0.0)
sd0 = O.seeded_state_dict(m.state_dict()); m.load_state_dict(sd0)
m = m.to(dev).set_precision("fp32").train()
N, h, w = 2, 16, 16
ycat = torch.relu(torch.randn(N, h, w, 896, generator=g))
W = torch.randn(N, 1, 4 * h, 4 * w, generator=g)
plan = m._get_plans()["single"]
tape = {}
with torch.no_grad():
    d = plan.forward(ycat.to(dev), None, None, True, tape)
    (gin, grads) = plan.backward(tape, W.to(dev))
sd = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in sd0.items()}
keys = ["den_dec.0.conv.weight", "den_dec.0.bn.weight", "den_dec.0.bn.bias", "den_head.0.conv.weight", "mem"]
for k in keys: sd[k].requires_grad_(True)
yc = ycat.double().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
y = O._conv_bn_relu(yc, sd, "den_dec.0.conv", "den_dec.0.bn", True, pad=0)
yn, _ = O.forward_mem(sd, y)
dd = O._up(F.relu(F.conv2d(yn, sd["den_head.0.conv.weight"])), 4)
(dd * W.double()).sum().backward()
e = lambda a, r: ((a.double().cpu() - r.double()).norm() / r.double().norm()).item()
print("d", e(d, dd))
print("g_ycat", e(gin[0].permute(0, 3, 1, 2), yc.grad))
for c0, c1 in [(0, 128), (128, 384), (384, 896)]:
    print(f"  g_ycat[{c0}:{c1}]", e(gin[0].permute(0, 3, 1, 2)[:, c0:c1], yc.grad[:, c0:c1]))
P = dict(m.named_parameters())
for k in keys:
    print(k, e(grads[P[k]], sd[k].grad))
