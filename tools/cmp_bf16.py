import sys, os
sys.path.insert(0, os.getcwd())
import torch
from oracle import dg_oracle as O
from dgvcc_amd.models.models import DGModel_base
dev = torch.device("cuda")
for seed in (2112, 1, 2, 3):
    model = DGModel_base(pretrained=False, den_dropout=0.0)
    sd0 = O.seeded_state_dict(model.state_dict())
    model.load_state_dict(sd0)
    model = model.to(dev).set_precision("bf16")
    batch = O.synthetic_batch(2, int(os.environ.get("HW", "64")), int(os.environ.get("HW", "64")), seed=seed)
    _, outs, _, _ = O.train_step(sd0, batch, "simple")
    model.train()
    with torch.no_grad():
        d = model(batch[0].to(dev))
    c_ref, c = outs[0].sum().item(), d.sum().item()
    print(seed, "count rel err", abs(c - c_ref) / abs(c_ref), "map", ((d.cpu()-outs[0]).abs().max()/outs[0].abs().max()).item())
