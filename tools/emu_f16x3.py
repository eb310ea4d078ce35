"""CPU emulation of f32 convs on f16 matrix cores with two-part operands (hi = f16(x*s),
lo = f16(x*s - hi)) and three products hi*hi + hi*lo + lo*hi summed in f32, against float64
and beside the bf16 three-part / six-product split, through the oracle train step.
Scales are powers of two: per tensor for the pixel operand, per output channel for the filter.
usage: python tools/emu_f16x3.py simple|final H W [per_tensor|per_channel]"""
import math
import os
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import dg_oracle as O
from dgvcc_amd.models.models import DGModel_base, DGModel_final
torch.set_num_threads(8)
MODE = sys.argv[1]; H = int(sys.argv[2]); W = int(sys.argv[3])
SCALE = sys.argv[4] if len(sys.argv) > 4 else "per_tensor"
_conv = F.conv2d
ARITH = "f32"
HMAX_LOG2 = 14  # largest scaled magnitude 2^14 (f16 max 65504)
NP = int(os.environ.get("EMU_NP", "3"))  # 4: + lo*lo


def pow2_scale(amax):
    amax = torch.clamp(amax, min=1e-30)
    return torch.exp2(HMAX_LOG2 - torch.ceil(torch.log2(amax)))


def split_h(t, dims):  # dims: reduce dims for the amax (scale per remaining index)
    s = pow2_scale(t.abs().amax(dim=dims, keepdim=True)) if dims else pow2_scale(t.abs().max())
    ts = t * s
    hi = ts.to(torch.float16).to(torch.float32)
    lo = (ts - hi).to(torch.float16).to(torch.float32)
    return hi, lo, s


def split_b(t, n=3):
    parts = []; r = t
    for _ in range(n):
        h = r.to(torch.bfloat16).to(torch.float32); parts.append(h); r = r - h
    return parts


def prod(fn, xa, wa):
    """sum of the products of the operands' parts, as the matrix cores would form them"""
    if ARITH == "bf6":
        xs, ws = split_b(xa), split_b(wa)
        y = None
        for i in range(3):
            for j in range(3 - i):
                t = fn(xs[i], ws[j]); y = t if y is None else y + t
        return y
    # f16x3: per-tensor scale of the pixel-like operand, per-row (dim 0) scale of the filter
    xh, xl, sx = split_h(xa, None)
    wh, wl, sw = split_h(wa, tuple(range(1, wa.dim())) if SCALE == "per_channel" else None)
    y = fn(xh, wh) + fn(xh, wl) + fn(xl, wh)
    return (y + fn(xl, wl) if NP == 4 else y), sx, sw


class SC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, padding):
        ctx.save_for_backward(x, w); ctx.s = (stride, padding); ctx.hb = b is not None
        if ARITH == "bf6":
            y = prod(lambda p, q: _conv(p, q, None, stride, padding), x, w)
        else:
            y, sx, sw = prod(lambda p, q: _conv(p, q, None, stride, padding), x, w)
            y = y / (sx * sw.view(1, -1, 1, 1) if sw.dim() else sx * sw)
        return y if b is None else y + b.view(1, -1, 1, 1)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors; stride, padding = ctx.s
        if ARITH == "bf6":
            gx = prod(lambda p, q: torch.nn.grad.conv2d_input(x.shape, q, p, stride, padding), g, w)
            gw = prod(lambda p, q: torch.nn.grad.conv2d_weight(q, w.shape, p, stride, padding), g, x)
        else:
            # dgrad: pixel operand g (per tensor), filter w per input channel (dim 1 of w)
            wt = w.transpose(0, 1)
            gx, sg, swt = prod(lambda p, q: torch.nn.grad.conv2d_input(x.shape, q.transpose(0, 1), p, stride, padding), g, wt)
            gx = gx / (sg * swt.view(1, -1, 1, 1) if swt.dim() else sg * swt)
            # wgrad: both pixel-major operands per tensor
            gh, gl, s1 = split_h(g, None); xh, xl, s2 = split_h(x, None)
            f = lambda p, q: torch.nn.grad.conv2d_weight(q, w.shape, p, stride, padding)
            gw = (f(gh, xh) + f(gh, xl) + f(gl, xh)) / (s1 * s2)
        return gx, gw, (g.sum((0, 2, 3)) if ctx.hb else None), None, None


def conv_patch(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
    return SC.apply(x, w, b, stride, padding)


model = DGModel_base(pretrained=False, den_dropout=0.0) if MODE == "simple" else DGModel_final(pretrained=False)
sd = O.seeded_state_dict(model.state_dict())
batch = O.synthetic_batch(2, H, W, seed=2112)


def run(dt, patch):
    F.conv2d = conv_patch if patch else _conv
    s = {k: (v.to(dt) if v.is_floating_point() else v) for k, v in sd.items()}
    b = (batch[0].to(dt), batch[1].to(dt), (batch[2][0], batch[2][1].to(dt), batch[2][2].to(dt)))
    r = O.train_step(s, b, MODE)
    F.conv2d = _conv
    return r


l64, o64, g64, _ = run(torch.float64, False)
for name in ("fp32", "bf6", "f16x3"):
    ARITH = name
    l, o, g, _ = run(torch.float32, name != "fp32")
    oe = max(((a.double() - b).abs().max() / b.abs().max()).item() for a, b in zip(o, o64) if a.dim() > 0)
    big = max(v.norm() for v in g64.values())
    ge = max(((g[k].double() - g64[k]).norm() / (g64[k].norm() + 1e-30)).item() for k in g64 if g64[k].norm() > 1e-6 * big)
    gg = math.sqrt(sum(((g[k].double() - g64[k]).norm() ** 2).item() for k in g64)) / math.sqrt(sum((v.norm() ** 2).item() for v in g64.values()))
    print(f"{name:6s} scale {SCALE}: loss rel {abs(l.item() - l64.item()) / abs(l64.item()):.3e}  outs max rel {oe:.3e}  "
          f"grad worst {ge:.3e}  global {gg:.3e}", flush=True)
