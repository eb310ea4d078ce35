"""Host-side (no GPU) tests of the reference-facing entry points:
`dgvcc_amd.main` (reference main.py:30-160), `JHUDomainClsDataset`
(datasets/jhu_domain_cls_dataset.py), the patch-tiled count of `DGTrainer.predict` /
`predict2` (trainers/dgtrainer.py:71-102) against a restatement of the reference's loop,
checkpoint I/O (trainers/trainer.py:41-47) and the fused AdamW's host logic under torch's
OneCycleLR (main.py:85-100)."""
import os
import random

import numpy as np
import pytest
import torch
import torch.nn as nn
from PIL import Image

from test_augment import _write_dataset

CONFIG = """\
seed: 2112
version: {version}
device: 'cpu'
log_para: 1000
patch_size: 10000
mode: 'final'
num_epochs: &num_epochs 4
checkpoint: null
model:
  name: 'final'
  params:
    pretrained: False
    mem_size: 64
    mem_dim: 256
    cls_thrs: 0.5
    err_thrs: 0.5
    den_dropout: 0.5
    cls_dropout: 0.5
    has_err_loss: False
train_dataset: &train_dataset_params
  name: 'den_cls'
  params:
    root: '{root}'
    crop_size: 32
    downsample: 1
    is_grey: False
    unit_size: 16
    pre_resize: 1
val_dataset: *train_dataset_params
test_dataset: *train_dataset_params
train_loader:
  batch_size: 2
  num_workers: 0
  shuffle: True
  pin_memory: False
val_loader: &val_loader_params
  batch_size: 1
  num_workers: 0
  shuffle: False
  pin_memory: False
test_loader: *val_loader_params
loss:
  name: 'mse'
  params:
    reduction: 'mean'
optimizer:
  name: 'adamw'
  params:
    lr: &lr 0.001
    weight_decay: 0.0001
scheduler:
  name: 'onecycle'
  params:
    max_lr: *lr
    epochs: *num_epochs
    steps_per_epoch: 15
    final_div_factor: 1000
"""


def _dataset(root):
    _write_dataset(root)
    for split in ("val", "test"):
        os.makedirs(os.path.join(root, split))
        rng = np.random.default_rng(7)
        img = rng.integers(0, 256, (40, 56, 3), dtype=np.uint8)
        Image.fromarray(img).save(os.path.join(root, split, "v0.png"))
        np.save(os.path.join(root, split, "v0.npy"), np.stack([rng.uniform(0, 56, 5), rng.uniform(0, 40, 5)], 1))


def test_load_config_builds_the_reference_objects(tmp_path):
    from dgvcc_amd import main as Mn
    from dgvcc_amd.losses import MSELoss
    from dgvcc_amd.models.models import DGModel_final
    from dgvcc_amd.optim import AdamW
    root = str(tmp_path / "ds")
    _dataset(root)
    cfg = tmp_path / "c.yml"
    cfg.write_text(CONFIG.format(version="t", root=root))
    init, task = Mn.load_config(str(cfg), "train_test")
    assert init == dict(seed=2112, version="t", device="cpu", log_para=1000, patch_size=10000, mode="final")
    assert isinstance(task["model"], DGModel_final)
    assert isinstance(task["loss"], MSELoss)
    assert isinstance(task["optimizer"], AdamW)
    assert isinstance(task["scheduler"], torch.optim.lr_scheduler.OneCycleLR)
    assert task["num_epochs"] == 4 and task["checkpoint"] is None
    raw = next(iter(task["train_dataloader"]))
    assert raw.imgs.shape == (2, 32, 32, 3) and raw.imgs.dtype == torch.uint8
    val = next(iter(task["val_dataloader"]))
    assert val[0].dtype == torch.uint8 and val[0].shape == (1, 48, 64, 3)  # unit_size 16 padding
    assert len(task["test_dataloader"]) == 1
    _, task_t = Mn.load_config(str(cfg), "train")
    assert "test_dataloader" not in task_t
    _, task_e = Mn.load_config(str(cfg), "test")
    assert "optimizer" not in task_e and "test_dataloader" in task_e
    assert Mn.get_model("csrnet", {}) is None  # as main.py's get_model for unknown names
    # 'dgnet' (stb_reg_base / mall_base / qnrf_final) is main_base.py's get_basemodel()
    assert type(Mn.get_model("dgnet", {"pretrained": False})).__name__ == "DensityRegressorBase"
    with pytest.raises(NotImplementedError):
        Mn.get_dataset("bay", {}, "train")
    with pytest.raises(ValueError):
        Mn.get_loss("l1", {})


def test_jhu_domain_cls_dataset_matches_den_cls(tmp_path):
    """Same files listed in `domains/<label>_train.txt` -> the same samples as DenClsDataset
    (identical per-sample pipeline, jhu_domain_cls_dataset.py:66-126 vs den_cls_dataset.py:77-158)."""
    from dgvcc_amd.datasets import DenClsDataset, JHUDomainClsDataset
    root = str(tmp_path / "ds")
    _write_dataset(root)
    os.makedirs(os.path.join(root, "domains"))
    fns = sorted(os.path.join(root, "train", f) for f in os.listdir(os.path.join(root, "train"))
                 if f.endswith(".png"))
    with open(os.path.join(root, "domains", "fog_train.txt"), "w") as f:
        f.write("\n".join(fns) + "\n")
    with open(os.path.join(root, "domains", "fog_val.txt"), "w") as f:
        f.write(fns[0] + "\n")
    jd = JHUDomainClsDataset(root, "fog", 32, "weather", "fog", 2, "train")
    dc = DenClsDataset(root, 32, 2, "train", False, 16)
    dc.img_fns = fns
    assert len(jd) == 3
    for idx in range(3):
        random.seed(idx); torch.manual_seed(idx)
        a = jd[idx]
        random.seed(idx); torch.manual_seed(idx)
        b = dc[idx]
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    assert len(JHUDomainClsDataset(root, "fog", 32, "weather", "fog", 2, "test")) == 1  # test reads val


class _Mock(nn.Module):
    """Stand-in for a counting model: density = per-pixel function of the input."""

    def __init__(self):
        super().__init__()
        self.cov_calls = []

    def forward(self, x, cal_covstat=False):
        if cal_covstat:
            self.cov_calls.append(tuple(t.shape for t in x))
            return None
        d = (x.float() ** 2).mean(1, keepdim=True) * 37.0 + 0.1
        return d, None


def _ref_predict(model, img, ps, log_para):
    """trainers/dgtrainer.py:71-84 restated (per-patch .item() accumulation)."""
    from dgvcc_amd.utils.misc import divide_img_into_patches
    h, w = img.shape[2:]
    if h >= ps or w >= ps:
        cnt = 0
        for p in divide_img_into_patches(img, ps)[0]:
            cnt += torch.sum(model(p)[0]).cpu().item() / log_para
        return cnt
    return model(img)[0].sum().cpu().item() / log_para


@pytest.mark.parametrize("shape,ps", [((1, 3, 160, 224), 96), ((1, 3, 64, 80), 10000), ((1, 3, 50, 70), 16)])
def test_predict_count_matches_reference_loop(tmp_path, monkeypatch, shape, ps):
    from dgvcc_amd.trainers.dgtrainer import DGTrainer
    monkeypatch.chdir(tmp_path)
    tr = DGTrainer(1, "p", "cpu", 1000, ps, "final")
    g = torch.Generator().manual_seed(0)
    img = torch.randn(shape, generator=g)
    m = _Mock()
    assert tr.predict(m, img) == _ref_predict(m, img, ps, 1000)  # bit-identical Python float
    tr.mode = "isw"
    img2 = torch.randn(shape, generator=g)
    assert tr.predict2(m, img, img2) == _ref_predict(m, img, ps, 1000)
    from dgvcc_amd.utils.misc import divide_img_into_patches
    n = len(divide_img_into_patches(img, ps)[0]) if (shape[2] >= ps or shape[3] >= ps) else 1
    assert len(m.cov_calls) == n  # one covariance-statistics pass per patch pair


def test_val_and_test_step_metrics(tmp_path, monkeypatch):
    """val_step -> (|pred - n|, {'mse': (pred - n)^2}); test_step -> {'mae', 'mse'}
    (dgtrainer.py:211-237), with n = number of GT points."""
    from dgvcc_amd.trainers.dgtrainer import DGTrainer
    monkeypatch.chdir(tmp_path)
    tr = DGTrainer(1, "v", "cpu", 1000, 10000, "final")
    img = torch.randn(1, 3, 32, 48, generator=torch.Generator().manual_seed(1))
    gt = torch.zeros(1, 9, 2)
    m = _Mock()
    pred = _ref_predict(m, img, 10000, 1000)
    mae, extra = tr.val_step(m, (img, img, gt, ["x"], [(0, 0, 0, 0)]))
    assert mae == abs(pred - 9) and extra["mse"] == (pred - 9) ** 2
    out = tr.test_step(m, (img, img, gt, ["x"], [(0, 0, 0, 0)]))
    assert out == {"mae": abs(pred - 9), "mse": (pred - 9) ** 2}


def test_checkpoint_roundtrip(tmp_path, monkeypatch):
    """save_ckpt/load_ckpt keep the reference's state_dict keys and values
    (trainer.py:41-47; dgtrainer.py:35-48 for a [generator, regressor] pair)."""
    from dgvcc_amd.models.models import DGModel_final
    from dgvcc_amd.trainers.dgtrainer import DGTrainer
    monkeypatch.chdir(tmp_path)
    tr = DGTrainer(1, "c", "cpu", 1000, 10000, "final")
    torch.manual_seed(0)
    a = DGModel_final(pretrained=False)
    torch.manual_seed(1)
    b = DGModel_final(pretrained=False)
    path = str(tmp_path / "m.pth")
    tr.save_ckpt(a, path)
    tr.load_ckpt(b, path)
    sa, sb = a.state_dict(), b.state_dict()
    assert list(sa) == list(sb)
    assert all(torch.equal(sa[k], sb[k]) for k in sa)
    tr.save_ckpt([a, b], path)
    assert os.path.exists(str(tmp_path / "m_gen.pth")) and os.path.exists(str(tmp_path / "m_reg.pth"))


def test_adamw_flat_buffer_and_onecycle_host():
    """The fused AdamW flattens at the first step and again when the parameters were
    re-homed (model.to(device) after the optimizer was built, as main.py does); torch's
    OneCycleLR drives its lr and beta1 through param_groups."""
    from dgvcc_amd.optim import AdamW
    m = nn.Sequential(nn.Linear(4, 3), nn.Linear(3, 2))
    opt = AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
    g = opt.param_groups[0]
    before = [p.detach().clone() for p in m.parameters()]
    opt._ensure_flat(g)
    assert AdamW._is_flat(g)
    assert all(torch.equal(p, q) for p, q in zip(m.parameters(), before))
    flat = g["_flat"]
    m[0].weight.data = m[0].weight.data.clone()  # re-homed parameter
    assert not AdamW._is_flat(g)
    opt._ensure_flat(g)
    assert AdamW._is_flat(g) and g["_flat"] is not flat
    sch = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=1e-3, epochs=4, steps_per_epoch=15,
                                              final_div_factor=1000)
    ref_opt = torch.optim.AdamW(nn.Linear(1, 1).parameters(), lr=1e-3, weight_decay=1e-4)
    ref = torch.optim.lr_scheduler.OneCycleLR(ref_opt, max_lr=1e-3, epochs=4, steps_per_epoch=15,
                                              final_div_factor=1000)
    for _ in range(3):
        assert g["lr"] == ref_opt.param_groups[0]["lr"] and g["betas"] == ref_opt.param_groups[0]["betas"]
        sch.step(); ref.step()
