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


MODE_CASES = [("simple_base", "simple", "DGModel_base"), ("final", "final", "DGModel_final"),
              ("base_base", "base", "DGModel_base"), ("mem_base", "base", "DGModel_mem"),
              ("memadd_add", "add", "DGModel_memadd"), ("cls_cls", "cls", "DGModel_cls"),
              ("memcls_cls", "cls", "DGModel_memcls")]


def state_template(cls_name):
    """The reference's state_dict key order and shapes (tests/golden/state_dict_keys.json)."""
    import json
    keys = json.load(open(os.path.join(GOLD, "state_dict_keys.json")))[cls_name]
    return {k: (torch.zeros(s, dtype=torch.int64) if k.endswith("num_batches_tracked") else torch.zeros(s))
            for k, s in keys}


@pytest.mark.parametrize("name,mode,cls_name", MODE_CASES)
def test_train_step_oracle(name, mode, cls_name):
    g = load(f"train_{name}.npz")
    B, H, W = (int(v) for v in g["shape"])
    sd0 = O.seeded_state_dict(state_template(cls_name))
    batch = O.synthetic_batch(B, H, W, seed=2112)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    loss, outs, grads, sd1 = O.train_step(sd0, batch, mode)
    assert abs(loss.item() - g["loss"][0]) <= 1e-5 * abs(g["loss"][0])
    if mode in ("simple", "base"):
        assert np.allclose(outs[0].numpy(), g["out_d1"], rtol=1e-5, atol=1e-6)
    elif mode == "add":
        assert np.allclose(outs[0].numpy(), g["out_d1"], rtol=1e-5, atol=1e-6)
        assert np.allclose(outs[1].numpy(), g["out_d2"], rtol=1e-5, atol=1e-6)
        assert abs(outs[2].item() - g["out_loss_con"][0]) <= 1e-5 * abs(g["out_loss_con"][0])
    elif mode == "cls":
        assert np.allclose(outs[0].numpy(), g["out_d1"], rtol=1e-5, atol=1e-6)
        assert np.allclose(outs[2].numpy(), g["out_c1"], rtol=1e-5, atol=1e-6)
    else:
        assert np.allclose(outs[0].numpy(), g["out_dc1"], rtol=1e-5, atol=1e-5)
        assert np.allclose(outs[2].numpy(), g["out_c1"], rtol=1e-5, atol=1e-6)
        assert abs(outs[4].item() - g["out_loss_con"][0]) <= 1e-5 * abs(g["out_loss_con"][0])
    # conv biases right before a BatchNorm (vgg16_bn's) have mathematically zero gradients: their
    # values are rounding noise of whichever CPU ran the reference, not a property of the oracle
    pre_bn = {f"{s}.{i}.bias" for s, idx in O.ENC_CONVS.items() for i in idx}
    check_summary("grad__", {k: v for k, v in grads.items() if k not in pre_bn}, g, rtol=1e-4, atol=1e-7)
    # (and AdamW's first step moves them by lr x the sign of that noise)
    check_summary("post__", {k: v for k, v in sd1.items() if not k.endswith("num_batches_tracked") and k not in pre_bn},
                  g, rtol=1e-5, atol=1e-7)


def test_final_err_loss_oracle():
    """DGModel_final(has_err_loss=True): loss_err = F.l1_loss(IN(y_den1), IN(y_den2)) and the
    gradients of loss_err alone (models/models.py:303-311) against train_final_err.npz, which
    tests/golden/make_golden.py (gen_final_err) produced by running the reference."""
    g = load("train_final_err.npz")
    B, H, W = (int(v) for v in g["shape"])
    sd0 = O.seeded_state_dict(state_template("DGModel_final"))
    batch = O.synthetic_batch(B, H, W, seed=2112)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    loss_err, grads = O.err_loss_grads(sd0, batch)
    assert abs(loss_err.item() - g["out_loss_err"][0]) <= 1e-6 * abs(g["out_loss_err"][0])
    pre_bn = {f"{s}.{i}.bias" for s, idx in O.ENC_CONVS.items() for i in idx}
    check_summary("grad__", {k: v for k, v in grads.items() if k not in pre_bn}, g, rtol=1e-4, atol=1e-7)
