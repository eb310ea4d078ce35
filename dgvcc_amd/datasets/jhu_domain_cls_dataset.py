"""Drop-in `datasets.jhu_domain_cls_dataset.JHUDomainClsDataset` (reference
datasets/jhu_domain_cls_dataset.py:19-154 over datasets/jhu_domain_dataset.py:19-104), the
training set of the 16 JHU cross-domain configs.

Its per-sample pipeline is DenClsDataset's (grey, pad, crop, downsample, flip with Python
`random` in the same order; `more_transform` with the same torchvision parameters; bmap =
16x16 block sum > 0), so the host half and the GPU pixel half are shared with
`DenClsDataset`.  What differs is the file list, read from
`<root>/domains/<domain_label>_<train|val>.txt` (test reads the val list,
jhu_domain_dataset.py:44-48), and that there is no ROI map and no generated-image root.
"""
from __future__ import annotations

import os

from .den_cls_dataset import DenClsDataset


class JHUDomainClsDataset(DenClsDataset):
    """Constructor arguments as the reference; `domain_type`/`domain` are accepted and
    unused there too (the split comes from the domain list file)."""

    def __init__(self, root, domain_label, crop_size, domain_type, domain, downsample, method, is_grey=False,
                 unit_size=0, pre_resize=1):
        if method not in ("train", "val", "test"):
            raise ValueError("method must be train, val or test")
        self.root = root
        self.gen_root = None
        self.domain_label = domain_label
        self.domain_type = domain_type
        self.domain = domain
        self.crop_size = (crop_size, crop_size) if isinstance(crop_size, int) else tuple(crop_size)
        self.downsample = downsample
        self.method = method
        self.is_grey = is_grey
        self.unit_size = unit_size
        self.pre_resize = pre_resize
        self.gt_dir = None
        self.roi_map = None
        phase = {"train": "train", "val": "val", "test": "val"}[method]
        with open(os.path.join(root, "domains", f"{domain_label}_{phase}.txt")) as f:
            self.img_fns = [ln.strip() for ln in f.readlines()]
