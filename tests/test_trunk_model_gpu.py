"""ResNet-50 DG counters (IBN-b / SW / ISW) on the HIP trunk plans against the
CPU oracle (oracle/trunk_oracle.py, pinned to the reference by
tests/test_trunk_oracle.py) on the same seeded weights and synthetic frames.

Criteria: outputs/losses vs the float64 oracle within max(3 x the fp32 oracle's
own error, 1e-4) relative; gradients normwise per parameter within
max(2 x the fp32 oracle's error, 5e-3, 3 x the gradient's measured sensitivity to a
3e-5 relative input perturbation) (BN over a handful of pixels and ReLU-mask flips make
fp32 gradients differ at that level in any implementation, see
tests/test_model_gpu.py::_check_grads).
"""
import os
import tempfile

import pytest
import torch

from oracle import dg_oracle as O
from oracle import trunk_oracle as TO

pytestmark = pytest.mark.gpu

GRAD_TOL = 5e-3


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _cls(kind):
    from dgvcc_amd.models import trunks
    return {"ibn": trunks.IBNCounter_ResNet, "sw": trunks.SWCounter_ResNet,
            "isw": trunks.ISWCounter_ResNet}[kind]


def _setup(kind, dev, B=2, H=64, W=64, precision="fp32"):
    model = _cls(kind)(pretrained=False)
    sd0 = O.seeded_state_dict(model.state_dict())
    model.load_state_dict(sd0)
    model = model.to(dev).set_precision(precision)
    return model, sd0, O.synthetic_batch(B, H, W, seed=2112)


def _oracle(kind, sd0, img, dmaps, dtype, masks=None):
    # detached copies: requires_grad_ below must never reach the caller's sd0 (a later call's
    # .to() would then return non-leaf tensors whose .grad stays None)
    sd = {k: (v.detach().to(dtype).clone() if v.is_floating_point() else v.clone()) for k, v in sd0.items()}
    sd = {k: v.requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    if kind == "isw":
        l1, wt, out = TO.isw_train_forward(img.to(dtype), dmaps.to(dtype), sd,
                                           [(m.to(dtype), ns) for m, ns in masks])
        (l1 + 0.6 * wt).backward()
        loss = (l1.detach(), wt.detach())
    else:
        out, _ = TO.counter_forward(kind, img.to(dtype), sd, True)
        l1 = torch.nn.functional.mse_loss(out, dmaps.to(dtype) * 1000)
        l1.backward()
        loss = (l1.detach(),)
    grads = {k: (v.grad if v.grad is not None else torch.zeros_like(v)).double()
             for k, v in sd.items() if v.requires_grad}
    return out.detach().double(), loss, grads


def _sensitivity(kind, sd0, img, dmaps, g64, eps=3e-5, masks=None):
    """Normwise change of each float64 gradient when the frames move by eps (relative,
    seeded noise): the conditioning of that gradient against forward perturbations of the
    size fp32 arithmetic makes (see tests/test_model_gpu.py::grad_sensitivity).  masks: the
    ISW sensitive-covariance masks, held fixed."""
    noise = torch.randn(img.shape, generator=torch.Generator().manual_seed(77), dtype=torch.float64)
    _, _, g1 = _oracle(kind, sd0, img.double() * (1 + eps * noise), dmaps, torch.float64, masks)
    return {k: ((g1[k] - g64[k]).norm() / g64[k].norm().clamp_min(1e-300)).item() for k in g64}


def _check_grads(model, g64, g32, tol=GRAD_TOL, sens=None):
    bad = {}
    worst = (0.0, "", 0.0, 0.0)
    for k, p in model.named_parameters():
        if k not in g64 or g64[k].norm() == 0:
            continue
        g = (p.grad if p.grad is not None else torch.zeros_like(p)).detach().double().cpu()
        mine = ((g - g64[k]).norm() / g64[k].norm()).item()
        ref = ((g32[k] - g64[k]).norm() / g64[k].norm()).item()
        if ref > 0.5:  # structurally-zero gradient (e.g. a BN bias right before an IN): noise only
            continue
        if mine > max(2 * ref, tol, 3 * (sens or {}).get(k, 0.0)):
            bad[k] = (mine, ref, (sens or {}).get(k))
        worst = max(worst, (mine / max(2 * ref, tol), k, mine, ref))
    print("grad check worst (ratio to bound, param, err, fp32 ref err):", worst)
    assert not bad, bad


def _masks_from_model(model):
    return [(cm.mask_matrix.float().cpu(), float(cm.num_sensitive)) for cm in model.cov_matrix_layer]


@pytest.mark.parametrize("kind", ["ibn", "sw"])
def test_counter_train_fp32(dev, kind):
    from dgvcc_amd.losses import mse_loss
    model, sd0, batch = _setup(kind, dev)
    img, _, (_, dmaps, _) = batch
    out64, (l64,), g64 = _oracle(kind, sd0, img, dmaps, torch.float64)
    out32, (l32,), g32 = _oracle(kind, sd0, img, dmaps, torch.float32)
    model.train()
    out = model(img.to(dev))
    loss = mse_loss(out, dmaps.to(dev), 1000.0)
    loss.backward()
    torch.cuda.synchronize()
    assert rel(out, out64) < max(3 * rel(out32, out64), 1e-4)
    assert abs(loss.item() - l64.item()) <= max(3 * abs(l32.item() - l64.item()), 1e-4 * l64.item())
    _check_grads(model, g64, {k: v.double() for k, v in g32.items()}, sens=_sensitivity(kind, sd0, img, dmaps, g64))


def test_sw_running_stats(dev):
    """SwitchWhiten2d running_mean/running_cov updates (momentum 0.9) and the eval
    forward on the updated statistics (running stats start at zero, as the
    reference's reset_parameters, switchwhiten.py:64-67)."""
    model, sd0, batch = _setup("sw", dev)
    sd0 = {k: (torch.zeros_like(v) if k.endswith(("running_mean", "running_cov")) else v)
           for k, v in sd0.items()}
    model.load_state_dict(sd0)
    img = batch[0]
    sd = {k: v.double().clone() if v.is_floating_point() else v.clone() for k, v in sd0.items()}
    with torch.no_grad():
        TO.counter_forward("sw", img.double(), sd, True)
        model.train()
        model(img.to(dev))
    msd = model.state_dict()
    for k in sd:
        if k.endswith(("running_mean", "running_cov", "running_var")):
            assert rel(msd[k], sd[k]) < 1e-3, k
    with torch.no_grad():
        model.eval()
        out = model(img.to(dev))
        ref, _ = TO.counter_forward("sw", img.double(), sd, False)
    assert rel(out, ref) < 1e-3


def test_isw_covstat_and_train_fp32(dev):
    model, sd0, batch = _setup("isw", dev)
    img1, img2, (_, dmaps, _) = batch
    # cal_covstat in eval mode (dgtrainer.py:94-100) -> sensitive-covariance masks
    model.eval()
    with torch.no_grad():
        assert model([img1.to(dev), img2.to(dev)], cal_covstat=True) == 0
    model.set_mask_matrix()
    masks = _masks_from_model(model)
    with torch.no_grad():
        _, w = TO.counter_forward("isw", torch.cat([img1, img2]).double(),
                                  {k: v.double() if v.is_floating_point() else v for k, v in sd0.items()},
                                  False)
    for (m, ns), f in zip(masks, w):
        mref, kref = TO.sensitive_mask(TO.cov_variance(f), 1)
        assert ns == kref
        # top-k boundary ties can swap a few entries between fp32 and f64 variances
        assert (m != mref.float()).float().mean().item() < 1e-3
    model.train()
    losses = model(img1.to(dev), gts=dmaps.to(dev), apply_wtloss=True)
    (losses[0] + 0.6 * losses[1]).sum().backward()
    torch.cuda.synchronize()
    out64, (l64, wt64), g64 = _oracle("isw", sd0, img1, dmaps, torch.float64, masks)
    _, (l32, wt32), g32 = _oracle("isw", sd0, img1, dmaps, torch.float32, masks)
    print("isw covstat: loss err", abs(losses[0].item() - l64.item()), "fp32 ref", abs(l32.item() - l64.item()),
          "wt err", abs(losses[1].item() - wt64.item()), "fp32 ref", abs(wt32.item() - wt64.item()))
    assert abs(losses[0].item() - l64.item()) <= max(3 * abs(l32.item() - l64.item()), 1e-4 * l64.item())
    assert abs(losses[1].item() - wt64.item()) <= max(3 * abs(wt32.item() - wt64.item()), 1e-4 * wt64.item())
    sens = _sensitivity("isw", sd0, img1, dmaps, g64, masks=masks)
    print("isw sensitivity, largest:", sorted(sens.items(), key=lambda kv: -kv[1])[:3],
          "layer3.5.bn3.weight:", sens.get("layer3.5.bn3.weight"))
    _check_grads(model, g64, {k: v.double() for k, v in g32.items()}, sens=sens)


def test_isw_trainer_step(dev):
    """DGTrainer mode 'isw' (dgtrainer.py:194-204) against the oracle: at epoch 0 the step's
    loss is the counter's MSE alone, at epoch > 5 it adds 0.6 x the whitening loss
    (apply_wtloss); the returned loss values match the float64 oracle on the same masks,
    and the AdamW step leaves the torch-AdamW update of the oracle's gradients."""
    from dgvcc_amd.trainers.dgtrainer import DGTrainer
    model, sd0, batch = _setup("isw", dev)
    img1, img2, (_, dmaps, _) = batch
    model.eval()
    with torch.no_grad():
        model([img1.to(dev), img2.to(dev)], cal_covstat=True)
    model.set_mask_matrix()
    masks = _masks_from_model(model)
    out64, (l64, wt64), g64 = _oracle("isw", sd0, img1, dmaps, torch.float64, masks)
    _, (l32, wt32), _ = _oracle("isw", sd0, img1, dmaps, torch.float32, masks)
    tol_l = max(3 * abs(l32.item() - l64.item()), 1e-4 * l64.item())
    tol_w = max(3 * abs(wt32.item() - wt64.item()), 1e-4 * wt64.item())
    losses = {}
    for epoch in (0, 6):
        model.load_state_dict(sd0)
        with tempfile.TemporaryDirectory() as td:
            cwd = os.getcwd()
            os.chdir(td)
            try:
                tr = DGTrainer(2112, "t", dev, 1000, 10000, "isw")
                opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
                model.train()
                losses[epoch] = tr.train_step(model, torch.nn.MSELoss(), opt, batch, epoch)
            finally:
                os.chdir(cwd)
    assert abs(losses[0] - l64.item()) <= tol_l, (losses[0], l64.item())
    assert abs(losses[6] - (l64.item() + 0.6 * wt64.item())) <= tol_l + 0.6 * tol_w, (losses[6], l64, wt64)
    # the epoch-6 step's update: AdamW step 1 moves each live parameter by ~lr * sign(g)
    # (|m/sqrt(v)| = 1 at step 1), so the post-step parameters pin the gradient signs
    sd = model.state_dict()
    n_ok = n_all = moved = 0
    for k, g in g64.items():
        if g.abs().max() == 0 or k not in sd:
            continue
        delta = (sd[k].double().cpu() - sd0[k].double() * (1 - 1e-4 * 1e-4))
        big = g.abs() > 1e-2 * g.abs().max()  # fp32-noise-level gradients may flip sign
        n_ok += int((torch.sign(delta[big]) == -torch.sign(g[big])).sum())
        n_all += int(big.sum())
        moved += 1
    assert moved > 100 and n_ok >= 0.995 * n_all, (moved, n_ok, n_all)


@pytest.mark.parametrize("kind", ["ibn", "sw", "isw"])
def test_counter_bf16_close(dev, kind):
    """bf16 storage + bf16 MFMA (f32 statistics) vs the float64 oracle on the same
    bf16-rounded weights and input, in eval mode.  (Training mode with batch-2
    BatchNorm is chaotic for a random-init ResNet-50: rounding only the weights to
    bf16 moves the f64 output by 15-25%.)  The bar is the oracle's own bf16
    arithmetic (torch CPU, bfloat16 end to end): our cosine distance and count
    error (relative to the map's L1 mass) stay within a small multiple of it."""
    model, sd0, batch = _setup(kind, dev, precision="bf16")
    img = batch[0].bfloat16().float()
    if kind == "sw":  # valid (PSD) running covariances: one f64 training pass from zero
        sd0 = {k: (torch.zeros_like(v) if k.endswith(("running_mean", "running_cov")) else v.clone())
               for k, v in sd0.items()}
        sdt = {k: v.double() if v.is_floating_point() else v for k, v in sd0.items()}
        with torch.no_grad():
            TO.counter_forward("sw", img.double(), sdt, True)
        sd0 = {k: (sdt[k].float() if v.is_floating_point() else v) for k, v in sd0.items()}
        model.load_state_dict(sd0)
    with torch.no_grad():
        model.eval()
        out = model(img.to(dev)).double().cpu()
        sd = {k: (v.bfloat16().double() if v.dim() == 4 else v.double().clone()) if v.is_floating_point()
              else v.clone() for k, v in sd0.items()}
        ref, _ = TO.counter_forward(kind, img.double(), sd, False)
        sd16 = {k: (v.bfloat16() if v.is_floating_point() else v.clone()) for k, v in sd0.items()}
        t16, _ = TO.counter_forward(kind, img.bfloat16(), sd16, False)
        t16 = t16.double()

    mass = ref.abs().sum().item()

    def err(a):
        cosd = 1.0 - (a.flatten() @ ref.flatten() / (a.norm() * ref.norm())).item()
        return cosd, abs(a.sum().item() - ref.sum().item()) / mass

    ours, torch16 = err(out), err(t16)
    assert ours[0] <= 3 * torch16[0] + 1e-3 and ours[1] <= 3 * torch16[1] + 1e-2, (ours, torch16)


def _train_grads(model, kind, sd0, batch, dev):
    img1, img2, (_, dmaps, _) = batch
    model.load_state_dict(sd0)
    model.zero_grad(set_to_none=True)
    if kind == "isw":
        model.eval()
        with torch.no_grad():
            model([img1.to(dev), img2.to(dev)], cal_covstat=True)
        model.set_mask_matrix()
        model.train()
        losses = model(img1.to(dev), gts=dmaps.to(dev), apply_wtloss=True)
        (losses[0] + 0.6 * losses[1]).sum().backward()
    else:
        from dgvcc_amd.losses import mse_loss
        model.train()
        mse_loss(model(img1.to(dev)), dmaps.to(dev), 1000.0).backward()
    torch.cuda.synchronize()
    return {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("kind", ["ibn", "sw", "isw"])
def test_relu_fold_bit_identical(dev, kind, precision, monkeypatch):
    """The block-output ReLU backward folded into the next block's conv1 dgrad epilogue
    (dg_conv_fwd_acc_relu, trunk._RELU_FOLD) leaves every parameter gradient bit-identical to
    the separate relu_bwd pass (1x1 dgrad + accumulate, then the mask: the same rounding)."""
    from dgvcc_amd import trunk
    model, sd0, batch = _setup(kind, dev, B=2, H=96, W=128, precision=precision)
    monkeypatch.setattr(trunk, "_RELU_FOLD", False)
    ref = _train_grads(model, kind, sd0, batch, dev)
    monkeypatch.setattr(trunk, "_RELU_FOLD", True)
    got = _train_grads(model, kind, sd0, batch, dev)
    assert ref.keys() == got.keys() and len(ref) > 100
    bad = [k for k in ref if not torch.equal(ref[k], got[k])]
    assert not bad, bad[:5]
