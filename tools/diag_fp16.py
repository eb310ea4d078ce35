"""Diagnostic: fp16 gradient quality at qnrf_final size (DensityRegressorBase, 1x2048x2048,
simple mode) vs this framework's fp32 path: per conv weight cosine and normwise error, for
several loss scales (is the gap f16 underflow of the scaled gradients, or rounding?), plus
the f32 gradient magnitudes per layer input.  usage: python tools/diag_fp16.py [H]"""
import os

os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import dg_oracle as O  # noqa: E402
from dgvcc_amd.models import models2 as M2  # noqa: E402
from dgvcc_amd.losses import MSELoss  # noqa: E402
from dgvcc_amd.trainers.dgtrainer import DGTrainer  # noqa: E402


def grads(sd0, batch, prec, scale, dev):
    m = M2.DensityRegressorBase(pretrained=False)
    m.load_state_dict(sd0)
    m.den_dropout = 0.0
    m = m.to(dev).set_precision(prec).train()
    os.makedirs("/tmp/diag_fp16", exist_ok=True)
    os.chdir("/tmp/diag_fp16")
    tr = DGTrainer(2112, "t", dev, 1000, 10000, "simple")
    lt = tr.compute_count_loss(MSELoss(), m(batch[0].to(dev)), batch[2])
    (lt * scale).backward()
    out = {k: p.grad.detach().double() / scale for k, p in m.named_parameters() if p.grad is not None}
    return lt.item(), out


def torch_grads(sd0, batch, dev, half):
    """plain torch on the GPU (MIOpen), fp32 or autocast fp16 with a 2^16 loss scale."""
    import torch.nn as nn
    import torch.nn.functional as F
    from dgvcc_amd.models.models import ConvBlock
    m = M2.DensityRegressorBase(pretrained=False)
    m.load_state_dict(sd0)
    m = m.to(dev).train()

    def seq(mods, x):
        for mod in mods:
            if isinstance(mod, ConvBlock):
                x = mod.conv(x)
                if mod.bn is not None:
                    x = F.batch_norm(x, None, None, mod.bn.weight, mod.bn.bias, True, 0.1, 1e-5)
                if mod.relu is not None:
                    x = F.relu(x)
            elif isinstance(mod, nn.Dropout2d):
                continue
            elif isinstance(mod, nn.BatchNorm2d):
                x = F.batch_norm(x, None, None, mod.weight, mod.bias, True, 0.1, 1e-5)
            else:
                x = mod(x)
        return x

    up = lambda t, s: F.interpolate(t, scale_factor=s, mode="bilinear", align_corners=False)  # noqa: E731
    img = batch[0].to(dev)
    with torch.autocast("cuda", dtype=torch.float16, enabled=half):
        x1 = seq(m.stage1, img)
        x2 = seq(m.stage2, x1)
        x3 = seq(m.stage3, x2)
        y3 = seq(m.dec3, x3)
        y2 = seq(m.dec2, torch.cat([up(y3, 2), x2], 1))
        y1 = seq(m.dec1, torch.cat([up(y2, 2), x1], 1))
        yc = torch.cat([y1, up(y2, 2), up(y3, 4)], 1)
        d = up(seq(m.den_head if isinstance(m.den_head, nn.Sequential) else [m.den_head], seq(m.den_dec, yc)), 4)
    gt = batch[2][1].to(dev) * 1000.0
    loss = F.mse_loss(d.float(), gt)
    sc = 65536.0 if half else 1.0
    (loss * sc).backward()
    return loss.item(), {k: p.grad.detach().double() / sc for k, p in m.named_parameters() if p.grad is not None}


def main():
    H = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    dev = torch.device("cuda", 0)
    sd0 = O.seeded_state_dict(M2.DensityRegressorBase(pretrained=False).state_dict())
    batch = O.synthetic_batch(1, H, H, seed=7)
    l32, g32 = grads(sd0, batch, "fp32", 1.0, dev)
    print("fp32 loss", l32, flush=True)
    res = {}
    for sc in (2.0 ** 16,):
        l16, g16 = grads(sd0, batch, "fp16", sc, dev)
        fin = all(torch.isfinite(g).all().item() for g in g16.values())
        print(f"scale 2^{int(torch.log2(torch.tensor(sc)).item())} loss {l16:.6g} finite {fin}", flush=True)
        res[sc] = g16
    print("torch legs ...", flush=True)
    lt32, gt32 = torch_grads(sd0, batch, dev, False)
    print("torch fp32 done", flush=True)
    lt16, gt16 = torch_grads(sd0, batch, dev, True)
    print("torch fp32 loss", lt32, "torch autocast-fp16 loss", lt16)
    res["torch32"] = gt32
    res["torch16"] = gt16
    for k, g in g32.items():
        if g.dim() != 4:
            continue
        line = f"{k:22s} |g|max {g.abs().max().item():9.2e}"
        for sc, g16 in res.items():
            h = g16[k]
            cos = ((g * h).sum() / (g.norm() * h.norm()).clamp_min(1e-300)).item()
            err = ((h - g).norm() / g.norm()).item()
            line += f" | cos {cos:.5f} err {err:.2e}"
        print(line)


if __name__ == "__main__":
    main()
