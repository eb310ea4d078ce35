"""Diagnostic: per-parameter gradient norm ratio / cosine vs the float64 oracle
for the ResNet counters (GPU)."""
import sys
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from oracle import dg_oracle as O
from oracle import trunk_oracle as TO
from dgvcc_amd.models import trunks
from dgvcc_amd.losses import mse_loss

kind = sys.argv[1] if len(sys.argv) > 1 else "ibn"
dev = torch.device("cuda", 0)
cls = {"ibn": trunks.IBNCounter_ResNet, "sw": trunks.SWCounter_ResNet, "isw": trunks.ISWCounter_ResNet}[kind]
model = cls(pretrained=False)
sd0 = O.seeded_state_dict(model.state_dict())
model.load_state_dict(sd0)
model = model.to(dev).set_precision("fp32")
img, _, (_, dmaps, _) = O.synthetic_batch(2, 64, 64, seed=2112)
sd = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in sd0.items()}
sd = {k: v.requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
if kind == "isw":
    model.eval()
out64, _ = TO.counter_forward(kind, img.double(), sd, kind != "isw")
l = torch.nn.functional.mse_loss(out64, dmaps.double() * 1000)
l.backward()
model.train(kind != "isw")
out = model(img.to(dev))
loss = mse_loss(out, dmaps.to(dev), 1000.0)
loss.backward()
torch.cuda.synchronize()
print("loss", loss.item(), l.item())
for k, p in model.named_parameters():
    if k not in sd or sd[k].grad is None:
        continue
    g = p.grad.double().cpu().reshape(-1) if p.grad is not None else torch.zeros(p.numel(), dtype=torch.float64)
    r = sd[k].grad.reshape(-1)
    cos = (g @ r / (g.norm() * r.norm() + 1e-300)).item()
    print(f"{k:40s} ratio {(g.norm() / (r.norm() + 1e-300)).item():9.4f} cos {cos:8.5f}")
