"""Sensitivity of the HIP final-mode step gradients to a 1e-7-relative perturbation of the input
frames, next to the float64 oracle run on each HIP run's own e_mask / class-map decisions
(diagnosis of the 64x64 final-mode gradient check).  GPU; prints per-parameter
normwise differences for the decoder's BN parameters."""
import os, sys, tempfile, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from oracle import dg_oracle as O
from dgvcc_amd.models import models as MM
from dgvcc_amd.trainers.dgtrainer import DGTrainer
from dgvcc_amd.losses import MSELoss
dev = torch.device("cuda:0")
base = O.synthetic_batch(2, 64, 64, seed=2112)
runs = []
for eps in (0.0, 1e-7):
    g = torch.Generator().manual_seed(5)
    i1, i2, rest = base
    batch = (i1 * (1 + eps * torch.randn(i1.shape, generator=g)), i2 * (1 + eps * torch.randn(i2.shape, generator=g)), rest)
    m = MM.DGModel_final(pretrained=False, den_dropout=0.0, cls_dropout=0.0)
    sd0 = O.seeded_state_dict(m.state_dict()); m.load_state_dict(sd0)
    m = m.to(dev).set_precision("fp32").train()
    plan = m._get_plans()["pair"]
    plan.capture = {}
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        tr = DGTrainer(2112, "t", dev, 1000, 10000, "final")
        tr.train_step(m, MSELoss(), torch.optim.SGD(m.parameters(), lr=0.0), batch, 0)
    cap = plan.capture
    inj = dict(e_mask_in=cap["emask"].permute(0, 3, 1, 2).bool().cpu(), c_pred_in=tuple(c.cpu() for c in cap["c_pred"]))
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd0.items()}
    i1, i2, (pts, dm, bm) = batch
    _, _, g64, _ = O.train_step(sd64, (i1.double(), i2.double(), (pts, dm.double(), bm.double())), "final", **inj)
    hip = {n: p.grad.detach().double().cpu() for n, p in m.named_parameters() if p.grad is not None}
    runs.append((hip, g64, inj))
keys = [k for k in runs[0][0] if k.startswith("dec") and ".bn." in k]
rel = lambda a, b: ((a - b).norm() / b.norm()).item()
print("e_mask decisions differing between the two HIP runs:", int((runs[0][2]["e_mask_in"] != runs[1][2]["e_mask_in"]).sum()),
      " class decisions:", sum(int((a != b).sum()) for a, b in zip(runs[0][2]["c_pred_in"], runs[1][2]["c_pred_in"])))
for k in keys[:10]:
    print("%-22s hip0-vs-f64 %.2e  hip1-vs-f64 %.2e  hip0-vs-hip1 %.2e  f64_0-vs-f64_1 %.2e" % (
        k, rel(runs[0][0][k], runs[0][1][k]), rel(runs[1][0][k], runs[1][1][k]), rel(runs[0][0][k], runs[1][0][k]),
        rel(runs[0][1][k].double(), runs[1][1][k].double())))
