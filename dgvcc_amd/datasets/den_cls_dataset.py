"""Drop-in `datasets.den_cls_dataset.DenClsDataset` (reference datasets/den_cls_dataset.py,
datasets/den_dataset.py, datasets/base_dataset.py) with the pixel augmentation moved to
the GPU (dgvcc_amd/datasets/augment.py, augment.hip).

File layout (preprocess_data.py / utils/dmap_gen.py): `<root>/<method>/<name>.jpg|png`,
points `<name>.npy` [n, 2] (x, y), density map `<name>_dmap.npy` [H, W] (or
`<gt_dir>/<name>.npy`).

Host work per sample is what needs the file or is O(points): decoding, the geometric
decisions (grey / pad / crop / flip with Python `random`, in the reference's order), the
crop itself, the density-map crop/downsample/flip and the point transform.  The sample
carries its uint8 crop and a parameter record; `collate` stacks them into a
`RawDenClsBatch`, which `DGTrainer.train_step` (or `DeviceAugment`) turns into the
reference's batch `(img1, img2, (points, dmaps, bmaps))` on the GPU.
"""
from __future__ import annotations

import os
import random
from glob import glob

import numpy as np
import torch
from PIL import Image

from ..utils.misc import get_padding, random_crop
from .augment import RawDenClsBatch, draw_more_transform, new_record


def _load_array(path: str) -> np.ndarray:
    return np.load(path, allow_pickle=False)


class DenClsDataset(torch.utils.data.Dataset):
    """reference datasets/den_cls_dataset.py:16-186 (constructor arguments as the reference)."""

    def __init__(self, root, crop_size, downsample, method, is_grey=False, unit_size=0, pre_resize=1,
                 roi_map_path=None, gt_dir=None, gen_root=None):
        self.root = root
        self.gen_root = gen_root
        self.crop_size = (crop_size, crop_size) if isinstance(crop_size, int) else tuple(crop_size)
        self.downsample = downsample
        self.method = method
        self.is_grey = is_grey
        self.unit_size = unit_size
        self.pre_resize = pre_resize
        self.gt_dir = gt_dir
        # the reference loads the ROI map with allow_pickle=True (base_dataset.py:31); here only
        # plain arrays are accepted
        self.roi_map = _load_array(roi_map_path) if roi_map_path is not None else None
        if method not in ("train", "val", "test"):
            raise ValueError("method must be train, val or test")
        self.img_fns = glob(os.path.join(root, method, "*.jpg")) + glob(os.path.join(root, method, "*.png"))
        if gen_root is not None and method == "train":
            self.img_fns += glob(os.path.join(gen_root, "*.jpg")) + glob(os.path.join(gen_root, "*.png"))
        if method in ("val", "test"):
            self.img_fns = sorted(self.img_fns)

    def __len__(self):
        return len(self.img_fns)

    # ---- loading (base_dataset.py:68-82, den_dataset.py:26-30) --------------------------
    def _load_img(self, img_fn):
        img = np.asarray(Image.open(img_fn).convert("RGB"))
        if self.roi_map is not None:
            img = img * np.expand_dims(self.roi_map, axis=2)
            img = img.astype(np.uint8)
        return img, os.path.splitext(img_fn)[1]

    def _load_gt(self, gt_fn):
        gt = _load_array(gt_fn)
        if self.roi_map is not None:
            gt = gt[np.where(self.roi_map[gt[:, 1].astype(int), gt[:, 0].astype(int)])]
        return gt

    def _load_dmap(self, dmap_fn):
        dmap = _load_array(dmap_fn)
        if self.roi_map is not None:
            dmap = dmap * self.roi_map.astype(np.float32)
        return dmap

    def _paths(self, img_fn, img_ext):
        basename = img_fn.split("/")[-1].split(".")[0]
        if img_fn.startswith(self.root):
            gt_fn = img_fn.replace(img_ext, ".npy")
            if basename.endswith("_aug"):
                gt_fn = gt_fn.replace("_aug", "")
            elif basename.endswith("_aug2"):
                gt_fn = gt_fn.replace("_aug2", "")
        else:
            basename = basename[:-2]
            gt_fn = os.path.join(self.root, "train", basename + ".npy")
        if self.gt_dir is None:
            dmap_fn = gt_fn.replace(basename, basename + "_dmap")
        else:
            dmap_fn = os.path.join(self.gt_dir, basename + ".npy")
        return basename, gt_fn, dmap_fn

    def __getitem__(self, index):
        img_fn = self.img_fns[index]
        img, img_ext = self._load_img(img_fn)
        basename, gt_fn, dmap_fn = self._paths(img_fn, img_ext)
        gt = self._load_gt(gt_fn)
        if self.method == "train":
            return self._train_transform(img, gt, self._load_dmap(dmap_fn))
        return self._val_transform(img, gt, basename)

    # ---- den_cls_dataset.py:77-158 ------------------------------------------------------
    def _train_transform(self, img, gt, dmap):
        """Host half of the reference's _train_transform (same Python-`random` calls, same
        order); the pixel half is recorded for the GPU."""
        h, w = img.shape[:2]
        dmap = torch.from_numpy(dmap).unsqueeze(0)
        grey = random.random() > 0.88
        st_size = 1.0 * min(w, h)
        if st_size < min(self.crop_size[0], self.crop_size[1]):
            (left, top, right, bottom), h, w = get_padding(h, w, self.crop_size[0], self.crop_size[1])
            img = np.pad(img, ((top, bottom), (left, right), (0, 0)))
            dmap = torch.nn.functional.pad(dmap, (left, right, top, bottom))
            if len(gt) > 0:
                gt = gt + [left, top]
        i, j = random_crop(h, w, self.crop_size[0], self.crop_size[1])
        h, w = self.crop_size
        img = np.ascontiguousarray(img[i:i + h, j:j + w])
        dmap = dmap[:, i:i + h, j:j + w]
        if len(gt) > 0:
            gt = gt - [j, i]
            idx_mask = (gt[:, 0] >= 0) * (gt[:, 0] <= w) * (gt[:, 1] >= 0) * (gt[:, 1] <= h)
            gt = gt[idx_mask]
        else:
            gt = np.empty([0, 2])
        ds = self.downsample
        dmap = dmap.reshape([1, h // ds, ds, w // ds, ds]).sum(dim=(2, 4))
        if len(gt) > 0:
            gt = gt / ds
        flip = random.random() > 0.5
        if flip:
            dmap = torch.flip(dmap, dims=[-1])
            if len(gt) > 0:
                gt[:, 0] = w - gt[:, 0]
        rec = new_record(grey=grey, flip=flip)
        draw_more_transform(rec)  # torch RNG, as more_transform(img) would consume it
        return (torch.from_numpy(img), torch.from_numpy(rec), torch.from_numpy(gt.copy()).float(),
                dmap.float())

    # ---- den_cls_dataset.py:159-185 -----------------------------------------------------
    def _val_transform(self, img, gt, name):
        if self.pre_resize != 1:
            pil = Image.fromarray(img)
            img = np.asarray(pil.resize((int(pil.size[0] * self.pre_resize), int(pil.size[1] * self.pre_resize))))
        if self.unit_size is not None and self.unit_size > 0:
            h, w = img.shape[:2]
            new_w = (w // self.unit_size + 1) * self.unit_size if w % self.unit_size != 0 else w
            new_h = (h // self.unit_size + 1) * self.unit_size if h % self.unit_size != 0 else h
            padding, h, w = get_padding(h, w, new_h, new_w)
            left, top, right, bottom = padding
            img = np.pad(img, ((top, bottom), (left, right), (0, 0)))
            if len(gt) > 0:
                gt = gt + [left, top]
        else:
            padding = (0, 0, 0, 0)
        gt = gt / self.downsample
        rec = new_record()
        draw_more_transform(rec)
        return (torch.from_numpy(np.ascontiguousarray(img)), torch.from_numpy(rec),
                torch.from_numpy(gt.copy()).float(), name, padding)

    @staticmethod
    def collate(batch):
        """Training samples -> RawDenClsBatch (the reference's collate after the GPU pass)."""
        imgs, recs, points, dmaps = zip(*batch)
        return RawDenClsBatch(torch.stack(imgs, 0), torch.stack(recs, 0), tuple(points), torch.stack(dmaps, 0))


def augment_val_sample(sample, device):
    """A `_val_transform` sample -> the reference's val tuple (img1, img2, gt, name, padding)
    with batch dimension 1, pixel work on `device`."""
    from .augment import augment_den_cls
    img, rec, gt, name, padding = sample
    img1, img2 = augment_den_cls(img.unsqueeze(0).to(device), rec.unsqueeze(0))
    return img1, img2, gt.unsqueeze(0), name, padding
