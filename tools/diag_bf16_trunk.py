"""Diagnostic: per-block relative difference of bf16 vs fp32 activations of a
ResNet counter (GPU), to locate bf16-specific divergence."""
import sys
import torch
sys.path.insert(0, ".")
from oracle import dg_oracle as O
from dgvcc_amd.models import trunks
from dgvcc_amd import trunk as TR

kind = sys.argv[1] if len(sys.argv) > 1 else "ibn"
dev = torch.device("cuda", 0)
cls = {"ibn": trunks.IBNCounter_ResNet, "sw": trunks.SWCounter_ResNet, "isw": trunks.ISWCounter_ResNet}[kind]
rec = {}
orig = TR.Block.forward


def fwd(self, x, training, tape, ws):
    out = orig(self, x, training, tape, ws)
    rec.setdefault(rec.get("_mode"), []).append(out.buf.float().clone())
    return out


TR.Block.forward = fwd
orig_feat = TR.CounterPlan.features


def feats(self, img, dt, training, tape):
    x, ws = orig_feat(self, img, dt, training, tape)
    return x, ws


img = O.synthetic_batch(2, 64, 64, seed=2112)[0].to(dev)
outs = {}
for prec in ("fp32", "bf16"):
    model = cls(pretrained=False)
    sd0 = O.seeded_state_dict(model.state_dict())
    model.load_state_dict(sd0)
    model = model.to(dev).set_precision(prec)
    model.train(kind != "isw")
    rec["_mode"] = prec
    with torch.no_grad():
        outs[prec] = model(img).float()
for i, (a, b) in enumerate(zip(rec["fp32"], rec["bf16"])):
    print(f"block {i:2d} C={a.shape[-1]:4d} HW={a.shape[1]}x{a.shape[2]} rel {((a - b).abs().max() / a.abs().max()).item():.4f}"
          f" normrel {((a - b).norm() / a.norm()).item():.4f}")
a, b = outs["fp32"], outs["bf16"]
print("out rel", ((a - b).abs().max() / a.abs().max()).item(), "sum", a.sum().item(), b.sum().item())
