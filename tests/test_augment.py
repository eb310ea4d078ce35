"""Host side of the GPU data pipeline (dgvcc_amd/datasets): RNG consumption order of the
reference's transforms, DenClsDataset file conventions and geometric transform, and the CPU
oracle of the pixel pipeline (oracle/augment_oracle.py) against PIL on its own."""
import os

import numpy as np
import pytest
import torch
from PIL import Image, ImageEnhance

from dgvcc_amd.datasets.augment import AUG_PARAMS, P, draw_more_transform, gaussian_weights, hue_shift, new_record
from oracle import augment_oracle as AO


def test_more_transform_rng_order():
    """draw_more_transform consumes torch's RNG exactly as torchvision's more_transform:
    rand (RandomApply) -> randperm(4) + 4 uniform_ (ColorJitter.get_params) -> rand -> uniform_
    (GaussianBlur.get_params) -> rand (RandomAdjustSharpness)."""
    for seed in range(20):
        torch.manual_seed(seed)
        rec = new_record()
        draw_more_transform(rec)
        after = torch.rand(1).item()
        torch.manual_seed(seed)
        exp = new_record()
        if not (0.8 < torch.rand(1)):
            perm = torch.randperm(4)
            vals = [float(torch.empty(1).uniform_(lo, hi)) for lo, hi in
                    ((0.5, 1.5), (0.8, 1.2), (0.8, 1.2), (-0.1, 0.1))]
            exp[P["jitter"]] = 1
            exp[3:7] = perm.numpy()
            exp[7:10] = vals[:3]
            exp[P["hue_shift"]] = int(np.array(vals[3] * 255).astype(np.uint8))
        if not (0.5 < torch.rand(1)):
            sigma = torch.empty(1).uniform_(1.0, 1.0).item()
            exp[P["blur"]] = 1
            exp[P["k0"]], exp[P["k1"]] = gaussian_weights(sigma)
        if torch.rand(1).item() < 0.5:
            exp[P["sharp"]], exp[P["sharp_factor"]] = 1, 5.0
        assert np.array_equal(rec, exp), seed
        assert torch.rand(1).item() == after


def test_param_helpers():
    assert len(AUG_PARAMS) == 16
    assert hue_shift(-0.1) == 231 and hue_shift(0.1) == 25 and hue_shift(-0.0049) == 255
    k0, k1 = gaussian_weights(1.0)
    assert abs(2 * k0 + k1 - 1) < 1e-6 and abs(k0 / k1 - np.exp(-0.5)) < 1e-6


def test_oracle_hue_roundtrip_and_enhance():
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (9, 11, 3), dtype=np.uint8)
    assert np.array_equal(np.asarray(AO.adjust_hue(Image.fromarray(a), 0)),
                          np.asarray(Image.fromarray(a).convert("HSV").convert("RGB")))
    rec = new_record()
    rec[P["jitter"]] = 1
    rec[3:7] = [0, 3, 1, 2]
    rec[7:10] = [1.3, 0.9, 1.1]
    out = AO.more_transform(a, rec)
    ref = ImageEnhance.Brightness(Image.fromarray(a)).enhance(float(np.float32(1.3)))
    ref = AO.adjust_hue(ref, 0)
    ref = ImageEnhance.Contrast(ref).enhance(float(np.float32(0.9)))
    ref = ImageEnhance.Color(ref).enhance(float(np.float32(1.1)))
    assert np.array_equal(out, np.asarray(ref))


def _write_dataset(root, n=3, H=40, W=56):
    rng = np.random.default_rng(1)
    os.makedirs(os.path.join(root, "train"))
    for i in range(n):
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        Image.fromarray(img).save(os.path.join(root, "train", f"im{i}.png"))
        pts = np.stack([rng.uniform(0, W, 7), rng.uniform(0, H, 7)], 1)
        np.save(os.path.join(root, "train", f"im{i}.npy"), pts)
        np.save(os.path.join(root, "train", f"im{i}_dmap.npy"), rng.random((H, W)).astype(np.float32))
    return rng


def test_den_cls_dataset_host(tmp_path):
    """Crop/flip/downsample of the density map and the point set follow the reference
    (den_cls_dataset.py:96-151); the uint8 crop is the raw pixels of the crop window."""
    import random
    from dgvcc_amd.datasets import DenClsDataset
    root = str(tmp_path / "ds")
    _write_dataset(root)
    ds = DenClsDataset(root, 32, 2, "train", False, 16)
    assert len(ds) == 3
    for idx in range(3):
        random.seed(idx)
        torch.manual_seed(idx)
        img, rec, gt, dmap = ds[idx]
        fn = ds.img_fns[idx]
        src = np.asarray(Image.open(fn).convert("RGB"))
        full = np.load(fn.replace(".png", "_dmap.npy"))
        random.seed(idx)
        grey = random.random() > 0.88
        i, j = random.randint(0, 40 - 32), random.randint(0, 56 - 32)
        flip = random.random() > 0.5
        assert bool(rec[P["grey"]]) == grey and bool(rec[P["flip"]]) == flip
        assert img.shape == (32, 32, 3) and np.array_equal(img.numpy(), src[i:i + 32, j:j + 32])
        d = torch.from_numpy(full[i:i + 32, j:j + 32]).reshape(1, 16, 2, 16, 2).sum(dim=(2, 4))
        if flip:
            d = d.flip(-1)
        assert torch.equal(dmap, d.float())
        pts = np.load(fn.replace(".png", ".npy")) - [j, i]
        pts = pts[(pts[:, 0] >= 0) & (pts[:, 0] <= 32) & (pts[:, 1] >= 0) & (pts[:, 1] <= 32)] / 2
        if flip:
            pts[:, 0] = 32 - pts[:, 0]
        assert np.allclose(gt.numpy(), pts, atol=1e-5)
    raw = DenClsDataset.collate([ds[0], ds[1]])
    assert raw.imgs.shape == (2, 32, 32, 3) and raw.params.shape == (2, 16) and raw.dmaps.shape == (2, 1, 16, 16)
