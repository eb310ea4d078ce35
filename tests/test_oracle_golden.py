"""Pin the CPU oracle (oracle/) to fixtures produced by running the reference.

CPU-only: these run in the build container and on the GPU box alike (the
fixtures travel; the reference does not)."""
import os

import numpy as np
import pytest
import torch

from oracle import dg_oracle as O
from oracle.dmap_oracle import dmap_fixed

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLD, name)))


def check_summary(prefix, tensors, gold, rtol, atol=0.0):
    for k, v in tensors.items():
        key = prefix + k.replace(".", "__")
        v = v.detach().double().reshape(-1)
        if key in gold:
            ref = torch.from_numpy(gold[key]).double()
            err = (v - ref).abs().max().item()
            assert err <= atol + rtol * ref.abs().max().item(), (k, err)
        else:
            idx = torch.from_numpy(gold[key + "@idx"]).long()
            ref = torch.from_numpy(gold[key + "@val"]).double()
            s = gold[key + "@sum"]
            scale = max(ref.abs().max().item(), 1e-30)
            assert (v[idx] - ref).abs().max().item() <= atol + rtol * scale, k
            assert abs(v.sum().item() - s[0]) <= atol * v.numel() + rtol * s[1] + 1e-12, k


def test_dmap_oracle_bit_exact():
    g = load("dmap_fixed.npz")
    for name in ("edge", "empty", "full"):
        H, W = g[f"{name}__shape"]
        mine = dmap_fixed(g[f"{name}__points"], int(H), int(W))
        assert np.array_equal(mine, g[f"{name}__dmap"]), name


@pytest.mark.parametrize("name,mode", [("simple_base", "simple"), ("final", "final")])
def test_train_step_oracle(name, mode):
    g = load(f"train_{name}.npz")
    B, H, W = (int(v) for v in g["shape"])
    if mode == "simple":
        from dgvcc_amd.models.models import DGModel_base as M
        model = M(pretrained=False, den_dropout=0.0)
    else:
        from dgvcc_amd.models.models import DGModel_final as M
        model = M(pretrained=False, den_dropout=0.0, cls_dropout=0.0)
    sd0 = O.seeded_state_dict(model.state_dict())
    batch = O.synthetic_batch(B, H, W, seed=2112)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    loss, outs, grads, sd1 = O.train_step(sd0, batch, mode)
    assert abs(loss.item() - g["loss"][0]) <= 1e-5 * abs(g["loss"][0])
    if mode == "simple":
        assert np.allclose(outs[0].numpy(), g["out_d1"], rtol=1e-5, atol=1e-6)
    else:
        assert np.allclose(outs[0].numpy(), g["out_dc1"], rtol=1e-5, atol=1e-5)
        assert np.allclose(outs[2].numpy(), g["out_c1"], rtol=1e-5, atol=1e-6)
        assert abs(outs[4].item() - g["out_loss_con"][0]) <= 1e-5 * abs(g["out_loss_con"][0])
    check_summary("grad__", grads, g, rtol=1e-4, atol=1e-7)
    check_summary("post__", {k: v for k, v in sd1.items() if not k.endswith("num_batches_tracked")},
                  g, rtol=1e-5, atol=1e-7)
