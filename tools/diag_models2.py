"""Diagnostic: models2 classes on the HIP path vs a plain-torch float64 forward of the same
modules (GPU), per parameter gradient error, plus torch fp32 on the GPU as the calibration of
what fp32 arithmetic alone costs.  usage: python tools/diag_models2.py Generator [forward]"""
import copy
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import dg_oracle as O  # noqa: E402
from dgvcc_amd.models import models2 as M2  # noqa: E402
from dgvcc_amd.models.models import ConvBlock  # noqa: E402
from dgvcc_amd.kernels import Act  # noqa: E402


def torch_seq(mods, x):
    for m in mods:
        if isinstance(m, ConvBlock):
            x = m.conv(x)
            if m.bn is not None:
                x = F.batch_norm(x, None, None, m.bn.weight, m.bn.bias, True, 0.1, 1e-5)
            if m.relu is not None:
                x = F.relu(x)
        elif isinstance(m, nn.Dropout2d):
            continue
        else:
            x = m(x)
    return x


def torch_forward(name, m, x):
    if name == "Generator":
        return torch_seq(list(m.enc) + list(m.dec), x)
    if name == "Generator0":
        x1 = torch_seq(m.enc1, x)
        x2 = torch_seq(m.enc2, x1)
        x3 = torch_seq(m.enc3, x2)
        y = torch_seq(m.dec3, x3)
        y = torch.cat([F.interpolate(y, scale_factor=2, mode="bilinear", align_corners=False), x2], 1)
        y = torch_seq(m.dec2, y)
        y = torch.cat([F.interpolate(y, scale_factor=2, mode="bilinear", align_corners=False), x1], 1)
        y = torch_seq(m.dec1, y)
        y = F.interpolate(y, scale_factor=2, mode="bilinear", align_corners=False)
        return torch_seq(m.head, y)
    raise ValueError(name)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "Generator"
    dev = torch.device("cuda", 0)
    model = getattr(M2, name)()
    model.load_state_dict(O.seeded_state_dict(model.state_dict()))
    img = O.synthetic_batch(2, 64, 64, seed=2112)[0]
    ref = {}
    for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
        m = copy.deepcopy(model).to(dev).to(dt).train()
        out = torch_forward(name, m, img.to(dev).to(dt))
        r = torch.randn(out.shape, generator=torch.Generator().manual_seed(99), dtype=torch.float64).to(dev).to(dt)
        (out * r).sum().backward()
        ref[tag] = (out.detach().double(), {k: p.grad.double() for k, p in m.named_parameters()})
    mh = model.to(dev).set_precision("fp32").train()
    out = mh(img.to(dev))
    r = torch.randn(out.shape, generator=torch.Generator().manual_seed(99), dtype=torch.float64).to(dev).float()
    (out * r).sum().backward()
    o64, g64 = ref["f64"]
    print("out err hip", ((out.double() - o64).abs().max() / o64.abs().max()).item(),
          "torch32", ((ref["f32"][0] - o64).abs().max() / o64.abs().max()).item())
    for k, p in mh.named_parameters():
        g = p.grad.double()
        e_h = ((g - g64[k]).norm() / g64[k].norm().clamp_min(1e-30)).item()
        e_t = ((ref["f32"][1][k] - g64[k]).norm() / g64[k].norm().clamp_min(1e-30)).item()
        print(f"{k:28s} hip {e_h:9.2e}  torch32 {e_t:9.2e}  |g| {g64[k].norm().item():9.3e}")




def chain_trace(name="Generator"):
    """Per-op forward activations of the HIP chain vs torch float64 on the same weights."""
    from dgvcc_amd.models import plans2 as P2
    dev = torch.device("cuda", 0)
    model = getattr(M2, name)()
    model.load_state_dict(O.seeded_state_dict(model.state_dict()))
    img = O.synthetic_batch(2, 64, 64, seed=2112)[0].to(dev)
    model = model.to(dev).set_precision("fp32").train()
    plan = P2.ChainPlan(list(model.enc) + list(model.dec), image_input=True)
    tape = {}
    with torch.no_grad():
        plan.run(img, torch.float32, True, tape)
        rec = tape[plan]
        m64 = copy.deepcopy(model).double()
        mods = list(m64.enc) + list(m64.dec)
        x = img.double()
        k = 0
        for i, m in enumerate(mods):
            x = torch_seq([m], x)
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            if isinstance(m, (nn.ReLU, nn.Dropout2d, nn.Tanh)):
                continue
            if isinstance(m, nn.Conv2d) and isinstance(nxt, nn.ReLU):
                x = F.relu(x)
            op = plan.ops[k]
            r = rec[k]
            mine = r[1].buf.permute(0, 3, 1, 2) if op[0] != "head" else r[2]
            if op[0] == "head" and op[3]:
                x = torch.tanh(x)
            print(f"op {k:2d} {op[0]:5s} {type(m).__name__:10s} err {((mine.double() - x).norm() / x.norm()).item():.2e}"
                  f"  frac<=0 {(x <= 0).double().mean().item():.3f}")
            k += 1
            if op[0] == "head":
                break


def tail_check(name="Generator"):
    """The head and the last ConvBlock's BN backward of the HIP chain against float64 torch
    on the chain's own saved tensors."""
    from dgvcc_amd.models import plans2 as P2
    from dgvcc_amd import kernels as K
    dev = torch.device("cuda", 0)
    model = getattr(M2, name)()
    model.load_state_dict(O.seeded_state_dict(model.state_dict()))
    img = O.synthetic_batch(2, 64, 64, seed=2112)[0].to(dev)
    model = model.to(dev).set_precision("fp32").train()
    plan = P2.ChainPlan(list(model.enc) + list(model.dec), image_input=True)
    tape = {}
    out = plan.run(img, torch.float32, True, tape)
    rec = tape[plan]
    r = torch.randn(out.shape, generator=torch.Generator().manual_seed(99), dtype=torch.float64).to(dev)
    # float64 of the tail: x (head input) -> head conv -> tanh
    hx = rec[-1][0].buf.double().permute(0, 3, 1, 2).clone().requires_grad_(True)
    conv = plan.ops[-1][1]
    yt = torch.tanh(F.conv2d(hx, conv.weight.double()))
    yt.backward(r)
    g64 = hx.grad.permute(0, 2, 3, 1)
    grads, _ = None, None
    # HIP head backward alone (same code path as ChainPlan.back)
    tape2 = {plan: rec}
    layer = plan.ops[-2][1]
    x_l, z_l, st_l, wp_l, drop_l, tr_l = tape[layer]
    ghead = torch.empty_like(rec[-1][0].buf)
    gfin = r.float().contiguous()
    gpre = torch.empty_like(gfin)
    K.call("dg_tanh_bwd", K.ptr(rec[-1][2]), K.ptr(gfin), gfin.numel(), K.ptr(gpre), 0, K.stream())
    w = conv.weight.detach()
    for k in range(3):
        K.head_bwd(rec[-1][0], w[k].reshape(-1).contiguous(), K.ACT_NONE, rec[-1][1][k], gpre[:, k].contiguous(),
                   Act(ghead), torch.empty(64, device=dev), None, accumulate_gx=k > 0)
    torch.cuda.synchronize()
    print("head gx err", ((ghead.double() - g64).norm() / g64.norm()).item())
    # BN backward of the last ConvBlock with that (exact) gradient, f64 vs kernel
    zd = z_l.buf.double().permute(0, 3, 1, 2).clone().requires_grad_(True)
    bn = layer.bn
    gam = bn.weight.detach().double().requires_grad_(True)
    bet = bn.bias.detach().double().requires_grad_(True)
    yb = F.relu(F.batch_norm(zd, None, None, gam, bet, True, 0.1, 1e-5))
    yb.backward(g64.permute(0, 3, 1, 2))
    dz = Act(torch.empty_like(z_l.buf))
    dga, dbe = torch.empty(64, device=dev), torch.empty(64, device=dev)
    K.bn_bwd(Act(g64.float().contiguous()), z_l, bn.weight.detach(), st_l, 1, dz, dga, dbe, None)
    torch.cuda.synchronize()
    print("bn dz", ((dz.buf.double() - zd.grad.permute(0, 2, 3, 1)).norm() / zd.grad.norm()).item(),
          "dgamma", ((dga.double() - gam.grad).norm() / gam.grad.norm()).item(),
          "dbeta", ((dbe.double() - bet.grad).norm() / bet.grad.norm()).item())
    print("stats mean vs f64", ((st_l[0].double() - zd.detach().mean((0, 2, 3))).abs().max()).item(),
          "invstd", ((st_l[1].double() - 1 / (zd.detach().var((0, 2, 3), unbiased=False) + 1e-5).sqrt()).abs().max()
                     / st_l[1].double().abs().max()).item())


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "trace":
        chain_trace(sys.argv[1])
    elif len(sys.argv) > 2 and sys.argv[2] == "tail":
        tail_check(sys.argv[1])
    else:
        main()
