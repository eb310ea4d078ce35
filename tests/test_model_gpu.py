"""Model-level parity on the GPU: the HIP DGModel_* path against the CPU oracle
(oracle/dg_oracle.py, itself pinned to the reference by tests/golden) on the
same seeded weights and synthetic frames.

Tolerance (north_star): density maps and losses within 1e-4 relative in fp32.
"""
import os
import tempfile

import pytest
import torch

from oracle import dg_oracle as O

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _model(name, **kw):
    from dgvcc_amd.models import models as M
    return getattr(M, name)(pretrained=False, **kw)


def _grads_normrel(model, ref_grads):
    """normwise relative error per parameter (conv biases followed by BN have
    mathematically-zero gradients: pure rounding noise in every implementation)."""
    worst = {}
    for k, p in model.named_parameters():
        if k.endswith(".bias") and (k.startswith("enc") or ".conv." in k):
            continue
        g = (p.grad if p.grad is not None else torch.zeros_like(p)).detach().double().cpu()
        r = ref_grads[k].double()
        if r.norm() == 0:
            continue
        worst[k] = ((g - r).norm() / r.norm()).item()
    return worst


def _f64(sd, batch):
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    i1, i2, (pts, dm, bm) = batch
    return sd64, (i1.double(), i2.double(), (pts, dm.double(), bm.double()))


@pytest.mark.parametrize("B,H,W", [(2, 64, 64), (1, 96, 128)])
def test_base_simple_step_fp32(dev, B, H, W):
    from dgvcc_amd.trainers.dgtrainer import DGTrainer
    from dgvcc_amd.losses import MSELoss
    model = _model("DGModel_base", den_dropout=0.0)
    sd0 = O.seeded_state_dict(model.state_dict())
    model.load_state_dict(sd0)
    model = model.to(dev).set_precision("fp32")
    batch = O.synthetic_batch(B, H, W, seed=2112)
    loss_ref, outs, grads_ref, sd1 = O.train_step(sd0, batch, "simple")

    model.train()
    with torch.no_grad():
        d = model(batch[0].to(dev))
    # the no-grad forward above also updated running stats: reload
    model.load_state_dict(sd0)
    assert rel(d, outs[0]) < 1e-4

    with tempfile.TemporaryDirectory() as td:
        cwd = os.getcwd()
        os.chdir(td)
        try:
            tr = DGTrainer(2112, "t", dev, 1000, 10000, "simple")
            opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
            loss = tr.train_step(model, MSELoss(), opt, batch, 0)
        finally:
            os.chdir(cwd)
    assert abs(loss - loss_ref.item()) <= 1e-4 * abs(loss_ref.item())
    # gradients: against the float64 oracle.  BN over few pixels makes some
    # parameter gradients ill-conditioned: the reference's own fp32 CPU path is
    # off by up to 4e-3 normwise (4% max-relative on dec3.0 at 64x64).  Criterion:
    # the HIP fp32 error is at most 2x the reference fp32 error (floor 1e-4).
    _, _, grads64, _ = O.train_step(*_f64(sd0, batch), "simple")
    mine = _grads_normrel(model, grads64)
    ref32 = {k: ((grads_ref[k].double() - grads64[k]).norm() / grads64[k].norm()).item() for k in mine}
    bad = {k: (v, ref32[k]) for k, v in mine.items() if v > max(2 * ref32[k], 1e-4)}
    assert not bad, bad
    sd = model.state_dict()
    for k in sd1:
        if "running" in k:
            assert rel(sd[k], sd1[k]) < 1e-4, k
        if k.endswith("num_batches_tracked"):
            assert int(sd[k]) == int(sd1[k]), k


def test_base_bf16_close(dev):
    model = _model("DGModel_base", den_dropout=0.0)
    sd0 = O.seeded_state_dict(model.state_dict())
    model.load_state_dict(sd0)
    model = model.to(dev).set_precision("bf16")
    batch = O.synthetic_batch(2, 64, 64, seed=2112)
    _, outs, _, _ = O.train_step(sd0, batch, "simple")
    model.train()
    with torch.no_grad():
        d = model(batch[0].to(dev))
    # bf16 storage/MFMA: compare the count (sum) and the map loosely
    c_ref, c = outs[0].sum().item(), d.sum().item()
    assert abs(c - c_ref) / abs(c_ref) < 5e-2
    assert rel(d, outs[0]) < 0.15


def test_fused_adamw_matches_torch(dev):
    from dgvcc_amd.optim import AdamW
    g = torch.Generator().manual_seed(0)
    ps = [torch.randn(s, generator=g) for s in [(3, 4), (7,), (2, 3, 5)]]
    a = [torch.nn.Parameter(p.clone().to(dev)) for p in ps]
    b = [torch.nn.Parameter(p.clone().to(dev)) for p in ps]
    oa = torch.optim.AdamW(a, lr=1e-3, weight_decay=1e-2)
    ob = AdamW(b, lr=1e-3, weight_decay=1e-2)
    for _ in range(3):
        for pa, pb in zip(a, b):
            gr = torch.randn(pa.shape, generator=g).to(dev)
            pa.grad = gr.clone()
            pb.grad = gr.clone()
        oa.step()
        ob.step()
    for pa, pb in zip(a, b):
        assert rel(pb, pa) < 1e-6
