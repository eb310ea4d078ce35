"""CPU emulation of the f32 split-math conv (bf16 parts, products i+j < NS, f32 sums) through the
oracle train step, against float64: usage python tools/emu_split.py simple|final H W NS"""
import sys, torch, math
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch.nn.functional as F
from oracle import dg_oracle as O
from dgvcc_amd.models.models import DGModel_base, DGModel_final
torch.set_num_threads(8)
MODE = sys.argv[1]; H = int(sys.argv[2]); W = int(sys.argv[3]); NS = int(sys.argv[4]) if len(sys.argv) > 4 else 2
_conv = F.conv2d
def split(t, n):
    parts = []; r = t
    for _ in range(n):
        h = r.to(torch.bfloat16).to(torch.float32); parts.append(h); r = r - h
    return parts
def sconv(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
    if x.dtype != torch.float32: return _conv(x, w, b, stride, padding, dilation, groups)
    xs, ws = split(x, NS), split(w, NS)
    y = None
    for i in range(NS):
        for j in range(NS - i):
            t = _conv(xs[i], ws[j], None, stride, padding, dilation, groups)
            y = t if y is None else y + t
    return y if b is None else y + b.view(1, -1, 1, 1)
class SC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, padding):
        ctx.save_for_backward(x, w); ctx.s = (stride, padding); ctx.hb = b is not None
        return sconv(x, w, b, stride, padding)
    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors; stride, padding = ctx.s
        gs, xs, ws = split(g, NS), split(x, NS), split(w, NS)
        gx = gw = None
        for i in range(NS):
            for j in range(NS - i):
                a = torch.nn.grad.conv2d_input(x.shape, ws[j], gs[i], stride, padding)
                c = torch.nn.grad.conv2d_weight(xs[j], w.shape, gs[i], stride, padding)
                gx = a if gx is None else gx + a; gw = c if gw is None else gw + c
        return gx, gw, (g.sum((0, 2, 3)) if ctx.hb else None), None, None
def conv_patch(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
    return SC.apply(x, w, b, stride, padding)
model = (DGModel_base if MODE == "simple" else DGModel_final)(pretrained=False, den_dropout=0.0) if MODE=="simple" else DGModel_final(pretrained=False)
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
for name, patch in (("fp32", False), ("split", True)):
    l, o, g, _ = run(torch.float32, patch)
    oe = max(((a.double() - b).abs().max() / b.abs().max()).item() for a, b in zip(o, o64) if a.dim() > 0)
    ge = max(((g[k].double() - g64[k]).norm() / (g64[k].norm() + 1e-30)).item() for k in g64 if g64[k].norm() > 1e-6 * max(v.norm() for v in g64.values()))
    print(name, "NS", NS, "loss rel", abs(l.item() - l64.item()) / abs(l64.item()), "outs max rel", oe, "grad worst normwise", ge, flush=True)
