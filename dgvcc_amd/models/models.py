"""Drop-in MI355X implementation of `models.models` (reference models/models.py).

Same class names, constructor signatures, sub-module names and therefore the
same `state_dict` keys as the reference; the forward/backward math runs on
the HIP kernel plans of `dgvcc_amd.engine` (NHWC activations, implicit-GEMM
MFMA convolutions).  Precision: "fp32" (default; exact-f32 MFMA, parity with
the reference CPU path) or "bf16" (bf16 storage/MFMA, f32 accumulation and
statistics) — `model.set_precision(...)` or env DGVCC_PRECISION.
"""
from __future__ import annotations

import os
import warnings

import torch
import torch.nn as nn

from .. import engine as E

_VGG16_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
_PRECISIONS = {"fp32": torch.float32, "bf16": torch.bfloat16}


def vgg16_bn_features() -> nn.Sequential:
    """torchvision vgg16_bn().features layout (cfg "D" + BN), torchvision init."""
    layers, cin = [], 3
    for v in _VGG16_CFG:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            conv = nn.Conv2d(cin, v, kernel_size=3, padding=1)
            nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
            nn.init.constant_(conv.bias, 0)
            bn = nn.BatchNorm2d(v)
            layers += [conv, bn, nn.ReLU(inplace=True)]
            cin = v
    return nn.Sequential(*layers)


def _load_pretrained_vgg(features: nn.Sequential) -> None:
    """The reference downloads torchvision's VGG16_BN weights (models/models.py:35).
    There is no network here: use a local torchvision cache file if present."""
    home = os.environ.get("TORCH_HOME", os.path.expanduser("~/.cache/torch"))
    path = os.path.join(home, "hub", "checkpoints", "vgg16_bn-6c64b313.pth")
    if not os.path.exists(path):
        warnings.warn("pretrained VGG16-BN weights unavailable offline; using random init")
        return
    sd = torch.load(path, map_location="cpu", weights_only=True)
    feats = {k[len("features."):]: v for k, v in sd.items() if k.startswith("features.")}
    features.load_state_dict(feats, strict=False)


class ConvBlock(nn.Module):
    """reference models/models.py:8-21 (parameter container + standalone forward)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, dilation=1,
                 bias=False, bn=False, relu=True):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding,
                              dilation=dilation, bias=bias)
        self.bn = nn.BatchNorm2d(out_channels) if bn else None
        self.relu = nn.ReLU(inplace=True) if relu else None
        self._plan = None

    def forward(self, x):
        if self._plan is None:
            self._plan = _SingleConvPlan(self)
        return self._plan(x, self.training)


class _SingleConvPlan:
    """A lone ConvBlock on an NCHW tensor (not on the model hot path)."""

    def __init__(self, block):
        self.layer = E.ConvLayer(block.conv, block.bn,
                                 E.ACT_RELU if block.relu is not None else E.ACT_NONE)

    def params(self):
        return self.layer.params()

    def __call__(self, x, training):
        def fwd(xx, tape):
            xa = E.Act(xx.permute(0, 2, 3, 1).contiguous())
            out = E.Act(E.K.nhwc(xa.N, xa.H, xa.W, self.layer.Cout, xx.dtype, xx.device))
            self.layer.forward(xa, out, training, tape)
            if tape is not None:
                tape[self] = xa
            return out.buf.permute(0, 3, 1, 2)

        return E.run_plan(self, fwd, (x,), self.params())

    def backward(self, tape, g):
        xa = tape.pop(self)
        gx = E.Act(torch.empty_like(xa.buf))
        grads = self.layer.backward(tape, E.Act(g.permute(0, 2, 3, 1).contiguous().to(xa.buf.dtype)), gx)
        return (gx.buf.permute(0, 3, 1, 2),), grads


def upsample(x, scale_factor=2, mode="bilinear"):
    """reference models/models.py:23-27 on NCHW tensors (HIP resample kernel)."""
    from .. import kernels as K
    m = K.UP_NEAREST if mode == "nearest" else K.UP_BILINEAR
    s = int(scale_factor)
    N, C, H, W = x.shape
    xa = K.Act(x.permute(0, 2, 3, 1).contiguous())
    out = K.nhwc(N, H * s, W * s, C, x.dtype, x.device)
    K.upsample_fwd(xa, s, m, K.Act(out))
    return out.permute(0, 3, 1, 2)


class _DGBase(nn.Module):
    """Shared precision handling."""

    def _init_precision(self):
        self.precision = os.environ.get("DGVCC_PRECISION", "fp32")

    def set_precision(self, precision: str):
        if precision not in _PRECISIONS:
            raise ValueError(f"precision must be one of {list(_PRECISIONS)}")
        self.precision = precision
        return self

    @property
    def compute_dtype(self):
        return _PRECISIONS[self.precision]


class DGModel_base(_DGBase):
    """reference models/models.py:29-96."""

    def __init__(self, pretrained=True, den_dropout=0.5):
        super().__init__()
        self._init_precision()
        self.den_dropout = den_dropout

        features = vgg16_bn_features()
        if pretrained:
            _load_pretrained_vgg(features)
        self.enc1 = nn.Sequential(*list(features.children())[:23])
        self.enc2 = nn.Sequential(*list(features.children())[23:33])
        self.enc3 = nn.Sequential(*list(features.children())[33:43])

        self.dec3 = nn.Sequential(ConvBlock(512, 1024, bn=True), ConvBlock(1024, 512, bn=True))
        self.dec2 = nn.Sequential(ConvBlock(1024, 512, bn=True), ConvBlock(512, 256, bn=True))
        self.dec1 = nn.Sequential(ConvBlock(512, 256, bn=True), ConvBlock(256, 128, bn=True))

        self.den_dec = nn.Sequential(
            ConvBlock(512 + 256 + 128, 256, kernel_size=1, padding=0, bn=True),
            nn.Dropout2d(p=den_dropout))
        self.den_head = nn.Sequential(ConvBlock(256, 1, kernel_size=1, padding=0))
        self._plans = None

    # plans are plain objects bound to the sub-modules (rebuilt lazily)
    def _get_plans(self):
        if self._plans is None:
            self._plans = {"fe": E.FeaturePlan(self)}
            self._build_head_plans(self._plans)
        return self._plans

    def _build_head_plans(self, plans):
        plans["den"] = E.DensityPlan(self.den_dec[0], self.den_head[0], self.den_dropout)

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_plans"] = None
        return st

    def _forward_fe_nhwc(self, x):
        fe = self._get_plans()["fe"]
        dt = self.compute_dtype

        def fwd(img, tape):
            return fe.forward(img, dt, self.training, tape)

        return E.run_plan(fe, fwd, (x,), fe.params())

    def forward_fe(self, x):
        ycat, x3 = self._forward_fe_nhwc(x)
        return ycat.permute(0, 3, 1, 2), x3.permute(0, 3, 1, 2)

    def _density(self, ycat):
        den = self._get_plans()["den"]
        den.p = self.den_dropout

        def fwd(yc, tape):
            return den.forward(yc, self.training, tape)

        return E.run_plan(den, fwd, (ycat,), den.params())

    def forward(self, x):
        ycat, _ = self._forward_fe_nhwc(x)
        return self._density(ycat)
