"""The final-mode forward of one view at B x 3 x H x W (default 4 x 128 x 128): the HIP FeaturePlan's
outputs against the float64 oracle's forward_fe, and per ConvLayer the ReLU / max-pool decisions
the HIP forward took against those of float64 evaluated at the HIP layer's own input (flips, and
the smallest float64 |pre-activation| among them).  A decision flip is invisible to the
exact-given-forward test (tests/exact_vjp.py evaluates the VJP at HIP's decisions).

    python tools/diag_fwd_flips.py [B H W]"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import dg_oracle as O  # noqa: E402
from dgvcc_amd.models.models import DGModel_final  # noqa: E402
import exact_vjp as X  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def main():
    B, H, W = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (4, 128, 128)
    dev = torch.device("cuda", 0)
    m = DGModel_final(pretrained=False, den_dropout=0.0, cls_dropout=0.0)
    sd0 = O.seeded_state_dict(m.state_dict())
    m.load_state_dict(sd0)
    m = m.to(dev).set_precision("fp32").train()
    i1 = O.synthetic_batch(B, H, W, seed=2112)[0]
    fe = m._get_plans()["fe"]
    tape = {}
    with torch.no_grad():
        y1, y2, y3, x3 = fe.forward(i1.to(dev), torch.float32, True, tape)
    torch.cuda.synchronize()
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd0.items()}
    ycat64, x364 = O.forward_fe(sd64, i1.double(), True)
    hy = [X.nchw64(t) for t in (y1, y2, y3)]
    print(f"B={B} {H}x{W}: y1 {rel(hy[0], ycat64[:, :128]):.2e}  x3 {rel(X.nchw64(x3), x364):.2e}")
    layers = fe.enc + fe.dec
    for i, L in enumerate(layers):
        x, z, stats, _wp, _drop, _tr = tape[L]
        if isinstance(x, torch.Tensor):  # the stem reads the image
            xin = x.double().cpu()
        else:
            xin = X.act64(x)
        w = L.conv.weight.detach().double().cpu()
        b = L.conv.bias.detach().double().cpu() if L.conv.bias is not None else None
        z64 = F.conv2d(xin, w, b, padding=L.pad)
        zh = X.act64(z)
        pre64 = F.batch_norm(z64, None, None, L.bn.weight.detach().double().cpu(),
                             L.bn.bias.detach().double().cpu(), True, 0.0, L.bn.eps)
        mh = X.relu_mask(zh, stats)
        m64 = pre64 > 0
        flips = mh != m64
        nf = int(flips.sum())
        mn = float(pre64.abs()[flips].min()) if nf else 0.0
        per_n = [int(flips[n].sum()) for n in range(B)] if nf else []
        print(f"layer {i:2d} {L.Cin:4d}->{L.Cout:4d} {z64.shape[2]}x{z64.shape[3]}: z rel {rel(zh, z64):.2e}, "
              f"relu flips {nf} of {flips.numel()} (min |pre| {mn:.2e}) per sample {per_n}", flush=True)


if __name__ == "__main__":
    main()
