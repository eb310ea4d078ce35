import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from oracle import dg_oracle as O
from dgvcc_amd.models import models as M
dev = torch.device("cuda")
batch = O.synthetic_batch(2, 64, 64, seed=2112)
i1, i2, (pts, dm, bm) = batch
g = torch.Generator().manual_seed(9)

def run(name, fwd_ref, fwd_mine, **kw):
    m = getattr(M, name)(pretrained=False, **kw)
    sd0 = O.seeded_state_dict(m.state_dict()); m.load_state_dict(sd0)
    m = m.to(dev).set_precision("fp32").train()
    sd = {k: (v.double() if v.is_floating_point() else v) for k, v in sd0.items()}
    keys = O.trainable_keys(sd)
    for k in keys: sd[k].requires_grad_(True)
    Lr = fwd_ref(sd)
    ref = dict(zip(keys, torch.autograd.grad(Lr, [sd[k] for k in keys], allow_unused=True)))
    Lm = fwd_mine(m)
    Lm.backward()
    P = dict(m.named_parameters())
    errs = []
    for k, p in P.items():
        if k.endswith(".bias") and P[k[:-5] + ".weight"].dim() == 4: continue
        r = ref.get(k)
        if r is None or r.norm() == 0: continue
        errs.append((((p.grad.double().cpu() - r).norm() / r.norm()).item(), k))
    errs.sort(reverse=True)
    print(f"== {name}: L mine {Lm.item():.6g} ref {Lr.item():.6g}; worst:", [(f"{e:.1e}", k) for e, k in errs[:5]], flush=True)

W = torch.randn(2, 1, 64, 64, generator=g)
Wc = torch.randn(2, 1, 4, 4, generator=g)
def ref_single(sd, mem, cls):
    y_cat, x3 = O.forward_fe(sd, i1.double(), True)
    y = O._conv_bn_relu(y_cat, sd, "den_dec.0.conv", "den_dec.0.bn", True, pad=0)
    if mem: y, _ = O.forward_mem(sd, y)
    d = F.relu(F.conv2d(y, sd["den_head.0.conv.weight"]))
    if cls:
        c = O.cls_head(sd, x3, True)
        d = O._up(d * O._up(bm.double(), 4, "nearest"), 4)
        return (d * W.double()).sum() + (c * Wc.double()).sum()
    return (O._up(d, 4) * W.double()).sum()
def mine_single(m, cls):
    if cls:
        d, c = m(i1.to(dev), bm.to(dev))
        return (d * W.to(dev)).sum() + (c * Wc.to(dev)).sum()
    return (m(i1.to(dev)) * W.to(dev)).sum()
run("DGModel_mem", lambda sd: ref_single(sd, True, False), lambda m: mine_single(m, False), den_dropout=0.0)
run("DGModel_cls", lambda sd: ref_single(sd, False, True), lambda m: mine_single(m, True), den_dropout=0.0, cls_dropout=0.0)
run("DGModel_memcls", lambda sd: ref_single(sd, True, True), lambda m: mine_single(m, True), den_dropout=0.0, cls_dropout=0.0)
def ref_pair(sd):
    y_cat1, _ = O.forward_fe(sd, i1.double(), True); y_cat2, _ = O.forward_fe(sd, i2.double(), True)
    y1 = O._conv_bn_relu(y_cat1, sd, "den_dec.0.conv", "den_dec.0.bn", True, pad=0)
    y2 = O._conv_bn_relu(y_cat2, sd, "den_dec.0.conv", "den_dec.0.bn", True, pad=0)
    e = (torch.abs(F.instance_norm(y1, eps=1e-5) - F.instance_norm(y2, eps=1e-5)) < 0.5).detach()
    n1, l1 = O.forward_mem(sd, y1 * e); n2, l2 = O.forward_mem(sd, y2 * e)
    lc = F.mse_loss(F.softmax(l1, 1), F.softmax(l2, 1))
    d1 = O._up(F.relu(F.conv2d(n1, sd["den_head.0.conv.weight"])), 4)
    d2 = O._up(F.relu(F.conv2d(n2, sd["den_head.0.conv.weight"])), 4)
    return (d1 * W.double()).sum() + (d2 * W.double()).sum() + 1000 * lc
def mine_pair(m):
    d1, d2, lc = m.forward_train(i1.to(dev), i2.to(dev))
    return (d1 * W.to(dev)).sum() + (d2 * W.to(dev)).sum() + 1000 * lc
run("DGModel_memadd", ref_pair, mine_pair, den_dropout=0.0)
