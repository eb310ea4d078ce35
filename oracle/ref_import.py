"""TEST INFRASTRUCTURE ONLY — imports the read-only reference at /root/reference
(Python) so fixture scripts can run it as the parity oracle.  Never imported by
the product package.

The reference imports packages absent from this image; they are replaced by
*import placeholders* that provide only what the hot path touches:
  * torchvision.models.vgg16_bn(weights=None) — the standard cfg-D + BN
    `features` layout (the reference only slices `.features`), plus empty
    torchvision.transforms(.functional) modules (imported, never used by the step);
  * cv2 — imported by utils/dmap_gen.py, used only by its file driver `run`;
  * kmeans1d — imported by models/ISW/cov_settings.py, called only when
    relax_denom == 0 (never with the shipped defaults).
No reference source is copied; nothing here is shipped to the GPU box.
"""
from __future__ import annotations

import os
import sys
import types

REF = os.environ.get("DGVCC_REFERENCE", "/root/reference")


def available() -> bool:
    return os.path.isdir(os.path.join(REF, "models"))


# torchvision's published VGG "D" configuration (Simonyan & Zisserman 2014, table 1,
# column D); vgg16_bn inserts BatchNorm2d after every conv (torchvision/models/vgg.py
# `make_layers(cfgs["D"], batch_norm=True)`).  Restated here so the oracle's placeholder
# is independent of the product package.
_CFG_D = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]


def _vgg16_bn_features():
    """torchvision vgg16_bn().features: 44 children (13 x Conv3x3(pad 1)/BN/ReLU + 5 pools)
    with torchvision's initialisation (kaiming_normal fan_out on convs, zero bias, BN 1/0).
    Fixtures overwrite every weight with oracle.dg_oracle.seeded_state_dict, so only the
    layout matters for parity."""
    import torch.nn as nn
    layers, cin = [], 3
    for v in _CFG_D:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
            continue
        conv = nn.Conv2d(cin, v, kernel_size=3, padding=1)
        nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
        nn.init.zeros_(conv.bias)
        layers += [conv, nn.BatchNorm2d(v), nn.ReLU(inplace=True)]
        cin = v
    return nn.Sequential(*layers)


def _vgg19_features():
    """torchvision vgg19().features (cfg "E", no BN) for models2.Generator."""
    import torch.nn as nn
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
           512, 512, 512, 512, "M"]
    layers, cin = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
            continue
        layers += [nn.Conv2d(cin, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
        cin = v
    return nn.Sequential(*layers)


def _install_placeholders():
    import torch.nn as nn

    if "torchvision" not in sys.modules:
        tv = types.ModuleType("torchvision")
        tvm = types.ModuleType("torchvision.models")
        tvt = types.ModuleType("torchvision.transforms")
        tvtf = types.ModuleType("torchvision.transforms.functional")

        class _VGG(nn.Module):
            def __init__(self, features):
                super().__init__()
                self.features = features

        def vgg16_bn(weights=None, **kw):
            if weights is not None:
                raise RuntimeError("no pretrained weights offline")
            return _VGG(_vgg16_bn_features())

        class VGG16_BN_Weights:
            DEFAULT = "DEFAULT"

        def vgg19(weights=None, **kw):
            # models2.Generator/Generator0 always ask for VGG19_Weights.DEFAULT (a remote
            # download); the fixtures overwrite every weight with seeded values, so the
            # placeholder returns the cfg-E layout with random init whatever `weights` says.
            return _VGG(_vgg19_features())

        class VGG19_Weights:
            DEFAULT = "DEFAULT"

        tvm.vgg16_bn = vgg16_bn
        tvm.VGG16_BN_Weights = VGG16_BN_Weights
        tvm.vgg19 = vgg19
        tvm.VGG19_Weights = VGG19_Weights
        tv.models = tvm
        tv.transforms = tvt
        tvt.functional = tvtf
        sys.modules.update({"torchvision": tv, "torchvision.models": tvm,
                            "torchvision.transforms": tvt,
                            "torchvision.transforms.functional": tvtf})
    if "cv2" not in sys.modules:
        sys.modules["cv2"] = types.ModuleType("cv2")
    if "kmeans1d" not in sys.modules:
        km = types.ModuleType("kmeans1d")

        def cluster(*a, **k):
            raise RuntimeError("kmeans1d placeholder: relax_denom=0 path is parity-unpinned")

        km.cluster = cluster
        sys.modules["kmeans1d"] = km


def import_ref(modname: str):
    """Import `modname` (e.g. 'models.models') from the reference tree."""
    if not available():
        raise RuntimeError(f"reference not found at {REF}")
    _install_placeholders()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import importlib
    return importlib.import_module(modname)
