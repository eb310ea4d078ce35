"""Where does a final-mode step's gradient leave float64?  At B x 3 x H x W (default 4 x 128 x 128):
  A  the model's own step (forward_train + the trainer's loss + autograd), run twice (determinism);
  B  the plans driven by hand (FeaturePlan / PairPlan forward and backward, as
     tests/test_model_gpu.py::test_final_step_backward_exact_given_forward does), with the same
     float32 upstream gradients;
  64 the float64 oracle with A's e_mask / class decisions injected.
Prints per-parameter normwise errors A-vs-A', A-vs-B, A-vs-64, B-vs-64 for the worst parameters.

    python tools/diag_step_glue.py [B H W]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import dg_oracle as O  # noqa: E402
from dgvcc_amd.losses import mse_loss  # noqa: E402
from dgvcc_amd.losses.bce import binary_cross_entropy  # noqa: E402
from dgvcc_amd.models.models import DGModel_final  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def loss_of(dc1, dc2, c1, c2, lcon, dm, bm):
    return (mse_loss(dc1, dm, 1000.0) + mse_loss(dc2, dm, 1000.0)
            + 10 * (binary_cross_entropy(c1, bm) + binary_cross_entropy(c2, bm)) + 10 * lcon)


def main():
    B, H, W = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (4, 128, 128)
    dev = torch.device("cuda", 0)
    sd0 = O.seeded_state_dict(DGModel_final(pretrained=False).state_dict())
    batch = O.synthetic_batch(B, H, W, seed=2112)
    i1, i2, (pts, dm, bm) = batch

    def model():
        m = DGModel_final(pretrained=False, den_dropout=0.0, cls_dropout=0.0)
        m.load_state_dict(sd0)
        return m.to(dev).set_precision("fp32").train()

    def step_a(cap=None):
        m = model()
        m._get_plans()["pair"].capture = cap
        dc1, dc2, c1, c2, _, lcon, _ = m.forward_train(i1.to(dev), i2.to(dev), bm.to(dev))
        m._get_plans()["pair"].capture = None
        loss_of(dc1, dc2, c1, c2, lcon, dm.to(dev), bm.to(dev)).backward()
        return {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters()}

    cap = {}
    ga = step_a(cap)
    ga2 = step_a()
    # B: the plans by hand
    m = model()
    plans = m._get_plans()
    fe, pair = plans["fe"], plans["pair"]
    tA, tB, tP = {}, {}, {}
    with torch.no_grad():
        outA = fe.forward(i1.to(dev), torch.float32, True, tA)
        outB = fe.forward(i2.to(dev), torch.float32, True, tB)
        outs = pair.forward(outA[:3], outB[:3], outA[3], outB[3], bm.to(dev), 0.0, float(m.err_thrs), tP)
    leaves = [outs[i].detach().clone().requires_grad_(True) for i in (0, 1, 2, 3, 5)]
    g = torch.autograd.grad(loss_of(*leaves, dm.to(dev), bm.to(dev)), leaves)
    with torch.no_grad():
        gin, gp = pair.backward(tP, g[0], g[1], g[2], g[3], None, g[4])
        _, gfa = fe.backward(tA, *gin[0:3], gin[6])
        _, gfb = fe.backward(tB, *gin[3:6], gin[7])
    names = {p: n for n, p in m.named_parameters()}
    gb = {}
    for d in (gp, gfa, gfb):
        for p, t in d.items():
            n = names[p]
            gb[n] = gb[n] + t.double().cpu() if n in gb else t.double().cpu()
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd0.items()}
    b64 = (i1.double(), i2.double(), (pts, dm.double(), bm.double()))
    _, _, g64, _ = O.train_step(sd64, b64, "final", e_mask_in=cap["emask"].permute(0, 3, 1, 2).bool().cpu(),
                                c_pred_in=tuple(c.cpu() for c in cap["c_pred"]))
    skip = lambda k: k.endswith(".bias") and (k.startswith("enc") or ".conv." in k) and "cls_head.2" not in k  # noqa
    rows = []
    for k in g64:
        if skip(k) or g64[k].norm() == 0:
            continue
        rows.append((k, rel(ga[k], ga2[k]), rel(ga[k], gb[k].reshape(ga[k].shape)), rel(ga[k], g64[k]),
                     rel(gb[k].reshape(g64[k].shape), g64[k])))
    rows.sort(key=lambda r: -r[3])
    print(f"B={B} H={H} W={W}: param  A-vs-A'  A-vs-B  A-vs-f64  B-vs-f64")
    for r in rows[:25]:
        print(f"  {r[0]:28s} {r[1]:.2e} {r[2]:.2e} {r[3]:.2e} {r[4]:.2e}")


if __name__ == "__main__":
    main()
