"""Accuracy of the f32 conv arithmetics on real activations: per layer of the DGModel_final
forward (one view, 2 x 3 x H x W, train-mode BN), the conv output the HIP kernel wrote (z, taped)
against float64 conv of the same HIP input and weights (normwise and max relative), for the
3-way split (dg_set_f32_math(1)) and the exact f32 MFMA (0); then the end-to-end final-mode
gradient error at the same size against the float64 oracle with the step's thresholds injected.

    python tools/diag_split.py [H W]          -> one JSON line
Run it once per build (e.g. split rounding variants) on the same box for an A/B."""
import json
import os
import sys
import tempfile

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import dg_oracle as O  # noqa: E402
from dgvcc_amd import kernels as K  # noqa: E402
from dgvcc_amd.models.models import DGModel_final  # noqa: E402
from dgvcc_amd import _capi  # noqa: E402
import exact_vjp as X  # noqa: E402


def layer_errors(model, img, dev):
    fe = model._get_plans()["fe"]
    tape = {}
    with torch.no_grad():
        fe.forward(img.to(dev), torch.float32, True, tape)
    torch.cuda.synchronize()
    out = []
    for i, L in enumerate(fe.enc + fe.dec):
        x, z, *_ = tape[L]
        if i == 0:
            xin = img.double()
        else:
            xin = X.act64(x)
        ref = F.conv2d(xin, L.conv.weight.detach().double().cpu(),
                       None if L.conv.bias is None else L.conv.bias.detach().double().cpu(), padding=L.pad)
        got = X.act64(z)
        d = got - ref
        out.append({"layer": i, "cin": L.Cin, "cout": L.Cout, "norm_rel": (d.norm() / ref.norm()).item(),
                    "max_rel": (d.abs().max() / ref.abs().max()).item(), "mean_signed_rel": (d.sum() / ref.abs().sum()).item()})
    return out


def e2e(dev, H, W):
    model = DGModel_final(pretrained=False, den_dropout=0.0, cls_dropout=0.0)
    sd0 = O.seeded_state_dict(model.state_dict())
    model.load_state_dict(sd0)
    model = model.to(dev).set_precision("fp32").train()
    batch = O.synthetic_batch(2, H, W, seed=2112)
    plan = model._get_plans()["pair"]
    plan.capture = {}
    from dgvcc_amd.losses import MSELoss
    from dgvcc_amd.trainers.dgtrainer import DGTrainer
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        try:
            tr = DGTrainer(2112, "d", dev, 1000, 10000, "final")
            opt = torch.optim.SGD(model.parameters(), lr=0.0)
            tr.train_step(model, MSELoss(), opt, batch, 0)
        finally:
            os.chdir(cwd)
    cap = plan.capture
    plan.capture = None
    inject = dict(e_mask_in=cap["emask"].permute(0, 3, 1, 2).bool().cpu(), c_pred_in=tuple(c.cpu() for c in cap["c_pred"]))
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd0.items()}
    i1, i2, (pts, dm, bm) = batch
    _, _, g64, _ = O.train_step(sd64, (i1.double(), i2.double(), (pts, dm.double(), bm.double())), "final", **inject)
    keys = [k for k in g64 if not (k.endswith(".bias") and (k.startswith("enc") or ".conv." in k)) and g64[k].norm() > 0]
    mine = {k: p.grad.detach().double().cpu() for k, p in model.named_parameters()}
    per = {k: ((mine[k] - g64[k]).norm() / g64[k].norm()).item() for k in keys}
    cat = lambda d: torch.cat([d[k].reshape(-1) for k in keys])  # noqa: E731
    glob = ((cat(mine) - cat(g64)).norm() / cat(g64).norm()).item()
    return {"global": glob, "worst": max(per.items(), key=lambda kv: kv[1])}


def main():
    H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (256, 256)
    torch.set_num_threads(16)
    dev = torch.device("cuda", 0)
    res = {"lib_hash": _capi.library_hash(), "H": H, "W": W}
    img = O.synthetic_batch(2, H, W, seed=2112)[0]
    for mode, name in ((1, "split"), (0, "exact")):
        K.call("dg_set_f32_math", mode)
        model = DGModel_final(pretrained=False)
        model.load_state_dict(O.seeded_state_dict(model.state_dict()))
        model = model.to(dev).set_precision("fp32").train()
        res[name] = {"layers": layer_errors(model, img, dev), "e2e": e2e(dev, H, W)}
    K.call("dg_set_f32_math", 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
