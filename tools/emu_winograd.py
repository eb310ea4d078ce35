"""Feasibility of Winograd F(2x2, 3x3) for the fp32 3x3 stride-1 convolutions:
CPU emulation through the oracle's train step, every 3x3 / pad-1 conv replaced by
  U = B^T d B (input tiles, f32), V = G g G^T (filter, f32), M = sum_c U . V (f32 sums),
  Y = A^T M A (f32)
with autograd through the same transforms for the input / weight gradients, against float64
and beside the direct fp32 conv.  The parity bar is the density map within 1e-4 relative of
the fp32 CPU oracle (BASELINE.json north_star).

    python tools/emu_winograd.py simple|final H W [B]"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import dg_oracle as O  # noqa: E402
from dgvcc_amd.models.models import DGModel_base, DGModel_final  # noqa: E402

torch.set_num_threads(8)
_conv = F.conv2d
BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float64)
G = torch.tensor([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], dtype=torch.float64)
AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)


def wino(x, w, b=None, exact_transforms=False):
    """exact_transforms: U, V and the output transform formed in float64 (U, V then rounded to
    the f32 the GEMM consumes): isolates the error of the transforms from that of the sums."""
    N, C, H, W = x.shape
    Co = w.shape[0]
    dt = x.dtype
    tdt = torch.float64 if exact_transforms else dt
    bt, g, at = BT.to(tdt), G.to(tdt), AT.to(tdt)
    xp = F.pad(x, (1, 1, 1, 1))
    d = xp.unfold(2, 4, 2).unfold(3, 4, 2)                 # [N, C, H/2, W/2, 4, 4]
    U = torch.einsum("ai,nchwij,bj->nchwab", bt, d.to(tdt), bt).to(dt)   # B^T d B
    V = torch.einsum("ai,ocij,bj->ocab", g, w.to(tdt), g).to(dt)         # G g G^T
    M = torch.einsum("nchwab,ocab->nohwab", U, V)                        # per-position sums over C
    Y = torch.einsum("ia,nohwab,jb->nohwij", at, M.to(tdt), at).to(dt)   # A^T M A
    y = Y.permute(0, 1, 2, 4, 3, 5).reshape(N, Co, H, W)
    return y if b is None else y + b.view(1, -1, 1, 1)


def conv_patch(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
    if (x.dtype == torch.float32 and w.shape[-1] == 3 and w.shape[-2] == 3 and stride in (1, (1, 1))
            and padding in (1, (1, 1)) and groups == 1 and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0):
        return wino(x, w, b)
    return _conv(x, w, b, stride, padding, dilation, groups)


def main():
    mode = sys.argv[1]
    H, W = int(sys.argv[2]), int(sys.argv[3])
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    model = DGModel_base(pretrained=False, den_dropout=0.0) if mode == "simple" else DGModel_final(pretrained=False)
    sd = O.seeded_state_dict(model.state_dict())
    batch = O.synthetic_batch(B, H, W, seed=2112)
    # layer check: one 256 -> 256 conv on randn and on post-ReLU operands
    g = torch.Generator().manual_seed(1)
    for name, x in (("randn", torch.randn(2, 256, 32, 32, generator=g)),
                    ("relu", torch.relu(torch.randn(2, 256, 32, 32, generator=g)))):
        w = torch.randn(256, 256, 3, 3, generator=g) * 0.03
        r = _conv(x.double(), w.double(), padding=1)
        e_dir = ((_conv(x, w, padding=1).double() - r).norm() / r.norm()).item()
        e_win = ((wino(x, w).double() - r).norm() / r.norm()).item()
        e_wx = ((wino(x, w, exact_transforms=True).double() - r).norm() / r.norm()).item()
        print(f"layer {name}: direct f32 {e_dir:.2e}, winograd f32 {e_win:.2e}, winograd with float64 transforms "
              f"{e_wx:.2e}", flush=True)

    def run(dt, patch):
        F.conv2d = conv_patch if patch else _conv
        try:
            s = {k: (v.to(dt) if v.is_floating_point() else v) for k, v in sd.items()}
            b = (batch[0].to(dt), batch[1].to(dt), (batch[2][0], batch[2][1].to(dt), batch[2][2].to(dt)))
            return O.train_step(s, b, mode)
        finally:
            F.conv2d = _conv

    l64, o64, g64, _ = run(torch.float64, False)
    res = {}
    for name, patch in (("direct", False), ("winograd", True)):
        l, o, gr, _ = run(torch.float32, patch)
        res[name] = o
        oe = max(((a.double() - b).abs().max() / b.abs().max()).item() for a, b in zip(o, o64) if a.dim() > 0)
        ge = max(((gr[k].double() - g64[k]).norm() / (g64[k].norm() + 1e-30)).item() for k in g64
                 if g64[k].norm() > 1e-6 * max(v.norm() for v in g64.values()))
        print(f"{name}: loss rel {abs(l.item() - l64.item()) / abs(l64.item()):.2e}, density map max rel vs f64 "
              f"{oe:.2e}, grad worst normwise vs f64 {ge:.2e}", flush=True)
    d, wn = res["direct"][0].double(), res["winograd"][0].double()
    print(f"winograd vs direct fp32 density map max rel {((wn - d).abs().max() / d.abs().max()).item():.2e}")


if __name__ == "__main__":
    main()
