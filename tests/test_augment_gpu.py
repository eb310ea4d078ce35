"""GPU pixel pipeline of DenClsDataset (augment.hip) against the CPU oracle
(oracle/augment_oracle.py: PIL for the PIL steps, torchvision's blur restated)."""
import numpy as np
import pytest
import torch

from dgvcc_amd.datasets.augment import P, augment_den_cls, block_map, gaussian_weights, new_record
from oracle import augment_oracle as AO

pytestmark = pytest.mark.gpu


def _records(n, rng):
    recs = []
    for i in range(n):
        r = new_record(grey=bool(i % 5 == 1), flip=bool(i % 2))
        if i % 4 != 3:
            r[P["jitter"]] = 1
            r[3:7] = rng.permutation(4)
            r[P["brightness"]] = rng.uniform(0.5, 1.5)
            r[P["contrast"]] = rng.uniform(0.8, 1.2)
            r[P["saturation"]] = rng.uniform(0.8, 1.2)
            r[P["hue_shift"]] = int(np.array(rng.uniform(-0.1, 0.1) * 255).astype(np.uint8))
        if i % 3 != 2:
            r[P["blur"]] = 1
            r[P["k0"]], r[P["k1"]] = gaussian_weights(1.0)
        if i % 2 == 0:
            r[P["sharp"]], r[P["sharp_factor"]] = 1, 5.0
        recs.append(r)
    return np.stack(recs)


@pytest.mark.parametrize("B,H,W", [(8, 33, 47), (4, 64, 64)])
def test_augment_matches_pil_pipeline(dev, B, H, W):
    rng = np.random.default_rng(5)
    imgs = rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)
    imgs[0, :, : W // 2] = 200  # flat regions: ties and saturated blends
    recs = _records(B, rng)
    img1, img2 = augment_den_cls(torch.from_numpy(imgs).to(dev), torch.from_numpy(recs))
    img1, img2 = img1.cpu(), img2.cpu()
    blur_diff = 0
    for b in range(B):
        r1, r2, _, _ = AO.augment(imgs[b], recs[b])
        assert torch.equal(img1[b], r1), b
        if recs[b][P["blur"]]:  # float conv summation order: allow rare +-1 level at .5 boundaries
            d = (img2[b] - r2).abs()
            assert d.max() <= 2.0 / 255 + 1e-6, b
            blur_diff += int((d > 0).sum())
        else:
            assert torch.equal(img2[b], r2), b
    assert blur_diff <= 1e-3 * img2.numel(), blur_diff


def test_block_map(dev):
    g = torch.Generator().manual_seed(0)
    d = torch.rand(3, 1, 64, 48, generator=g)
    d[d < 0.995] = 0
    ref = (d.reshape(3, 1, 4, 16, 3, 16).sum(dim=(3, 5)) > 0).float()
    assert torch.equal(block_map(d.to(dev)).cpu(), ref)


def test_train_step_on_raw_batch(dev, tmp_path):
    """DenClsDataset -> collate -> DGTrainer.train_step (GPU augmentation inside) on DGModel_final."""
    import os
    import random
    from PIL import Image
    from dgvcc_amd.datasets import DenClsDataset
    from dgvcc_amd.losses import MSELoss
    from dgvcc_amd.models.models import DGModel_final
    from dgvcc_amd.optim import AdamW
    from dgvcc_amd.trainers.dgtrainer import DGTrainer
    rng = np.random.default_rng(2)
    root = tmp_path / "ds"
    (root / "train").mkdir(parents=True)
    for i in range(2):
        Image.fromarray(rng.integers(0, 256, (80, 96, 3), dtype=np.uint8)).save(root / "train" / f"a{i}.jpg")
        np.save(root / "train" / f"a{i}.npy", np.stack([rng.uniform(0, 96, 9), rng.uniform(0, 80, 9)], 1))
        np.save(root / "train" / f"a{i}_dmap.npy", rng.random((80, 96)).astype(np.float32) * 1e-3)
    random.seed(0)
    torch.manual_seed(0)
    ds = DenClsDataset(str(root), 64, 1, "train", False, 16)
    raw = DenClsDataset.collate([ds[0], ds[1]])
    model = DGModel_final(pretrained=False).to(dev).set_precision("bf16").train()
    opt = AdamW(model.parameters(), lr=1e-4)
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        tr = DGTrainer(2112, "t", dev, 1000, 10000, "final")
        loss = tr.train_step(model, MSELoss(), opt, raw, 0)
    finally:
        os.chdir(cwd)
    assert np.isfinite(loss)
    img1, img2, (pts, dmaps, bmaps) = tr.prepare_batch(raw)
    assert img1.shape == (2, 3, 64, 64) and bmaps.shape == (2, 1, 4, 4) and len(pts) == 2
