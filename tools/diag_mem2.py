import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from oracle import dg_oracle as O
from dgvcc_amd.models import models as M
from dgvcc_amd import kernels as K
dev = torch.device("cuda")
batch = O.synthetic_batch(2, 64, 64, seed=2112)
i1 = batch[0]
m = M.DGModel_mem(pretrained=False, den_dropout=0.0)
sd0 = O.seeded_state_dict(m.state_dict()); m.load_state_dict(sd0)
m = m.to(dev).set_precision("fp32").train()
sd = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in sd0.items()}
e = lambda a, r: ((a.double().cpu() - r.double()).norm() / r.double().norm()).item()
with torch.no_grad():
    ycat, x3 = m._forward_fe_nhwc(i1.to(dev))
    y_cat, _ = O.forward_fe(sd, i1.double(), True)
    print("ycat", e(ycat.permute(0, 3, 1, 2), y_cat))
    plan = m._get_plans()["single"]
    tape = {}
    d = plan.forward(ycat, x3, None, True, tape)
    st = tape[plan]
    y = O._conv_bn_relu(y_cat, sd, "den_dec.0.conv", "den_dec.0.bn", True, pad=0)
    print("yden", e(st["yden"].buf.permute(0, 3, 1, 2), y))
    yn, lg = O.forward_mem(sd, y)
    print("P", e(st["P"].buf.view(2, -1, 1024).transpose(1, 2), F.softmax(lg, 1)))
    print("ynew", e(st["ynew"].buf.permute(0, 3, 1, 2), yn))
    dd = O._up(F.relu(F.conv2d(yn, sd["den_head.0.conv.weight"])), 4)
    print("d", e(d, dd))
    print("yden stats: frac zero", (y == 0).double().mean().item(), "max", y.max().item())
    print("logit range", lg.min().item(), lg.max().item())
