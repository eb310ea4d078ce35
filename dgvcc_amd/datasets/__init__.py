"""Datasets with GPU-side augmentation."""
from .augment import DeviceAugment, RawDenClsBatch, augment_den_cls, block_map  # noqa: F401
from .den_cls_dataset import DenClsDataset, augment_val_sample  # noqa: F401
from .jhu_domain_cls_dataset import JHUDomainClsDataset  # noqa: F401
