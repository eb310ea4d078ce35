"""GPU parity of the evaluation path and the optimizer/scheduler step (SURVEY.md §8f ranks
2 and 4).

* `DGTrainer.predict` / `val_step` (trainers/dgtrainer.py:71-84,211-237) on the HIP
  DGModel_final in eval mode, patch-tiled with ragged edge patches, against the float64
  oracle forward of every patch (oracle/dg_oracle.py), count within 1e-4 relative (fp32
  north_star tolerance); bf16 within 1e-2.
* the fused AdamW under torch's OneCycleLR (the 47 'adamw' + 'onecycle' configs,
  main.py:85-100) against torch.optim.AdamW + OneCycleLR, built in main.py's order
  (optimizer before model.to(device)); parameters within 1e-6 relative.
"""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle import dg_oracle as O

pytestmark = pytest.mark.gpu


def _final_model(dev, precision="fp32"):
    from dgvcc_amd.models.models import DGModel_final
    model = DGModel_final(pretrained=False)
    sd0 = O.seeded_state_dict(model.state_dict())
    g = torch.Generator().manual_seed(3)
    for k in sd0:
        if k.endswith("running_mean"):
            sd0[k] = torch.randn(sd0[k].shape, generator=g) * 0.1
        elif k.endswith("running_var"):
            sd0[k] = torch.rand(sd0[k].shape, generator=g) + 0.5
    model.load_state_dict(sd0)
    return model.to(dev).set_precision(precision).eval(), sd0


def _oracle_density(sd, x):
    """DGModel_final.forward in eval mode (models/models.py:285-296) in float64."""
    sd = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    x = x.double()
    y_cat, x3 = O.forward_fe(sd, x, False)
    y = O._conv_bn_relu(y_cat, sd, "den_dec.0.conv", "den_dec.0.bn", False, pad=0)
    y, _ = O.forward_mem(sd, y)
    d = F.relu(F.conv2d(y, sd["den_head.0.conv.weight"]))
    c = O.cls_head(sd, x3, False)
    return O._up(d * O.cls_pred_map(c), 4)


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("bf16", 1e-2)])
def test_predict_patch_tiled_vs_oracle(dev, tmp_path, monkeypatch, precision, tol):
    from dgvcc_amd.trainers.dgtrainer import DGTrainer
    from dgvcc_amd.utils.misc import divide_img_into_patches
    monkeypatch.chdir(tmp_path)
    model, sd0 = _final_model(dev, precision)
    img = O.synthetic_batch(1, 160, 224, seed=11)[0]
    tr = DGTrainer(2112, "e", dev, 1000, 96, "final")  # patches 96/64 x 96/96/32
    with torch.no_grad():
        pred = tr.predict(model, img.to(dev))
    ref = sum(_oracle_density(sd0, p).sum().item() / 1000 for p in divide_img_into_patches(img, 96)[0])
    assert abs(pred - ref) <= tol * abs(ref)
    gt = torch.zeros(1, 3, 2)
    with torch.no_grad():
        mae, extra = tr.val_step(model, (img, img, gt, ["x"], [(0, 0, 0, 0)]))
    assert mae == abs(pred - 3) and extra["mse"] == (pred - 3) ** 2


def test_fused_adamw_onecycle_matches_torch(dev):
    from dgvcc_amd.optim import AdamW

    def build(cls):
        torch.manual_seed(0)
        m = nn.Sequential(nn.Conv2d(3, 8, 3), nn.BatchNorm2d(8), nn.Conv2d(8, 4, 1))
        opt = cls(m.parameters(), lr=1e-3, weight_decay=1e-4)  # main.py: optimizer first ...
        sch = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=1e-3, epochs=6, steps_per_epoch=15,
                                                  final_div_factor=1000)
        return m.to(dev), opt, sch  # ... then Trainer.train moves the model

    kw = dict(allreduce=False)
    m1, o1, s1 = build(lambda p, **a: AdamW(p, **a, **kw))
    m2, o2, s2 = build(torch.optim.AdamW)
    g = torch.Generator().manual_seed(5)
    for epoch in range(6):
        for _ in range(3):
            grads = [torch.randn(p.shape, generator=g) for p in m1.parameters()]
            for m, o in ((m1, o1), (m2, o2)):
                o.zero_grad()
                for p, gr in zip(m.parameters(), grads):
                    p.grad = gr.to(dev)
                o.step()
        s1.step(); s2.step()  # once per epoch (trainer.py:82-87)
    torch.cuda.synchronize()
    for p, q in zip(m1.parameters(), m2.parameters()):
        assert ((p - q).abs().max() / q.abs().max()).item() < 1e-6
    assert o1.param_groups[0]["lr"] == o2.param_groups[0]["lr"]
    assert o1.param_groups[0]["betas"] == o2.param_groups[0]["betas"]


def test_fused_adamw_late_gradient_matches_torch(dev):
    """A parameter whose .grad is None on the first steps: torch skips it and does not advance
    its step count, so its first update uses bias correction step 1 (per-parameter counts in
    the fused optimizer; a middle parameter splits the flat update into runs)."""
    from dgvcc_amd.optim import AdamW

    def build(cls):
        torch.manual_seed(0)
        m = nn.Sequential(nn.Conv2d(3, 8, 3), nn.Conv2d(8, 8, 1), nn.Conv2d(8, 4, 1)).to(dev)
        return m, cls(m.parameters(), lr=1e-2, weight_decay=1e-2)

    m1, o1 = build(lambda p, **a: AdamW(p, allreduce=False, **a))
    m2, o2 = build(torch.optim.AdamW)
    g = torch.Generator().manual_seed(3)
    for step in range(6):
        grads = [torch.randn(p.shape, generator=g) for p in m1.parameters()]
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad()
            for i, (p, gr) in enumerate(zip(m.parameters(), grads)):
                late = i in (2, 3) and step < 3   # conv #2 (weight, bias) joins at step 3
                p.grad = None if late else gr.to(dev)
            o.step()
    torch.cuda.synchronize()
    for p, q in zip(m1.parameters(), m2.parameters()):
        assert ((p - q).abs().max() / q.abs().max()).item() < 1e-6


def test_eval_weight_memo_follows_updates(dev):
    """Evaluation reuses packed filters / BN scale-shift across frames; they must follow a
    fused optimizer step (which writes parameters behind torch's version counters), a
    train()/eval() switch and load_state_dict."""
    from dgvcc_amd.models.models import DGModel_base
    from dgvcc_amd.optim import AdamW

    def fresh(sd):
        m = DGModel_base(pretrained=False)
        m.load_state_dict(sd)
        return m.to(dev).set_precision("fp32").eval()

    base = DGModel_base(pretrained=False)
    base.load_state_dict(O.seeded_state_dict(base.state_dict()))
    base = base.to(dev).set_precision("fp32").eval()
    x = O.synthetic_batch(1, 64, 64, seed=9)[0].to(dev)

    def run(m):  # decoder features (never all-zero) and the density map
        return torch.cat([m.forward_fe(x)[0].flatten(), m(x).flatten()]).clone()

    with torch.no_grad():
        y0 = run(base)
        assert torch.equal(run(base), y0)  # memo hit: same result
    opt = AdamW(base.parameters(), lr=1e-2, allreduce=False)
    for p in base.parameters():
        p.grad = torch.ones_like(p)
    opt.step()  # no train() switch: the optimizer itself invalidates
    with torch.no_grad():
        y1 = run(base)
        ref = run(fresh({k: v.detach().cpu() for k, v in base.state_dict().items()}))
    assert not torch.equal(y1, y0)
    assert torch.equal(y1, ref)
    sd = {k: v.detach().cpu().clone() for k, v in base.state_dict().items()}
    sd["enc1.0.weight"] = sd["enc1.0.weight"] * 0.5
    base.load_state_dict(sd)
    with torch.no_grad():
        assert torch.equal(run(base), run(fresh(sd)))
