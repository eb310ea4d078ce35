"""Drop-in MI355X implementation of `models.models` (reference models/models.py).

Same class names, constructor signatures, sub-module names and therefore the
same `state_dict` keys as the reference; the forward/backward math runs on
the HIP kernel plans of `dgvcc_amd.engine` (NHWC activations, implicit-GEMM
MFMA convolutions).  Precision: "fp32" (default; exact-f32 MFMA, parity with
the reference CPU path), "bf16" (bf16 storage/MFMA, f32 accumulation and
statistics) or "fp16" (fp16 storage + f16 MFMA, f32 accumulation and statistics:
configs/qnrf_final.yml) — `model.set_precision(...)` or env DGVCC_PRECISION.
"""
from __future__ import annotations

import os
import warnings

import torch
import torch.nn as nn

from .. import engine as E

_VGG16_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
_PRECISIONS = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}


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


class _CatPlan:
    """Materialise y_cat = cat[y1, up2(y2), up4(y3)] (NHWC) for forward_fe callers, with its
    backward (slice + bilinear U^T), on the HIP resample kernels."""

    def params(self):
        return []

    def __call__(self, y1, y2, y3):
        def fwd(a, b, c, tape):
            from .. import kernels as K
            N, h, w, c1 = a.shape
            out = K.nhwc(N, h, w, c1 + b.shape[3] + c.shape[3], a.dtype, a.device)
            out[..., :c1] = a
            K.upsample_fwd(K.Act(b.contiguous()), 2, K.UP_BILINEAR, K.Act(out, c1, b.shape[3]))
            K.upsample_fwd(K.Act(c.contiguous()), 4, K.UP_BILINEAR, K.Act(out, c1 + b.shape[3], c.shape[3]))
            if tape is not None:
                tape[self] = (a.shape, b.shape, c.shape)
            return out

        return E.run_plan(self, fwd, (y1, y2, y3), [])

    def backward(self, tape, g):
        from .. import kernels as K
        sa, sb, sc = tape.pop(self)
        g = g.contiguous()
        ga = g[..., :sa[3]].contiguous()
        gb = K.nhwc(*sb, g.dtype, g.device)
        gc = K.nhwc(*sc, g.dtype, g.device)
        K.upsample_bwd(K.Act(g, sa[3], sb[3]), 2, K.UP_BILINEAR, K.Act(gb))
        K.upsample_bwd(K.Act(g, sa[3] + sb[3], sc[3]), 4, K.UP_BILINEAR, K.Act(gc))
        return (ga, gb, gc), {}


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

    def train(self, mode: bool = True):
        from ..engine import invalidate_frozen
        invalidate_frozen()  # eval-mode packed weights are rebuilt after any mode switch
        return super().train(mode)


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
        """(y_cat, x3) NCHW as the reference returns them (models/models.py:64-87); y_cat is
        materialised here only — the model's own forward keeps it as its parts."""
        y1, y2, y3, x3 = self._forward_fe_nhwc(x)
        ycat = _CatPlan()(y1, y2, y3)
        return ycat.permute(0, 3, 1, 2), x3.permute(0, 3, 1, 2)

    def _density(self, cat):
        den = self._get_plans()["den"]
        den.p = self.den_dropout

        def fwd(y1, y2, y3, tape):
            return den.forward((y1, y2, y3), self.training, tape)

        return E.run_plan(den, fwd, tuple(cat), den.params())

    def forward(self, x):
        y1, y2, y3, _ = self._forward_fe_nhwc(x)
        return self._density((y1, y2, y3))


class DGModel_mem(DGModel_base):
    """reference models/models.py:98-136 (memory read after den_dec)."""

    def __init__(self, pretrained=True, mem_size=1024, mem_dim=256, den_dropout=0.5):
        super().__init__(pretrained, den_dropout)
        self.mem_size = mem_size
        self.mem_dim = mem_dim
        self.mem = nn.Parameter(torch.FloatTensor(1, self.mem_dim, self.mem_size).normal_(0.0, 1.0))
        self.den_dec = nn.Sequential(
            ConvBlock(512 + 256 + 128, self.mem_dim, kernel_size=1, padding=0, bn=True),
            nn.Dropout2d(p=den_dropout))
        self.den_head = nn.Sequential(ConvBlock(self.mem_dim, 1, kernel_size=1, padding=0))

    _USE_MEM, _USE_CLS = True, False

    def _build_head_plans(self, plans):
        plans["single"] = E.SinglePlan(self, mem=self._USE_MEM, cls=self._USE_CLS)
        if hasattr(self, "forward_train"):
            plans["pair"] = E.PairPlan(self, cls=self._USE_CLS)

    def forward_mem(self, y):
        """NCHW y -> (y_new NCHW, logits [b, mem_size, h*w]) (models/models.py:116-125)."""
        from .. import kernels as K
        b, k, h, w = y.shape
        plan = self._get_plans()["single"]
        dt = self.compute_dtype
        ya = K.Act(y.detach().permute(0, 2, 3, 1).contiguous().to(dt))
        memT_s, mem_p, _ = plan.memr.packs(dt, self.training)
        L = plan.memr.logits(ya, memT_s, dt)
        P = K.Act(torch.empty_like(L.buf))
        K.call("dg_softmax_fwd", L.dt, L.ptr, L.M, L.C, P.ptr, K.stream())
        yn = plan.memr.readout(P, mem_p, dt)
        return yn.buf.permute(0, 3, 1, 2), L.buf.view(b, h * w, -1).transpose(1, 2)

    def _single(self, cat, x3, c_gt=None):
        plan = self._get_plans()["single"]

        def fwd(y1, y2, y3, x, tape):
            return plan.forward((y1, y2, y3), x, c_gt, self.training, tape)

        return E.run_plan(plan, fwd, (*cat, x3), plan.params())

    def forward(self, x):
        y1, y2, y3, x3 = self._forward_fe_nhwc(x)
        return self._single((y1, y2, y3), x3)


class _PairMixin:
    def jsd(self, logits1, logits2):
        """mean((softmax(l1) - softmax(l2))^2) over the slot axis (models/models.py:147-157)."""
        import torch.nn.functional as F
        return F.mse_loss(F.softmax(logits1, dim=1), F.softmax(logits2, dim=1))

    def _pair(self, img1, img2, c_gt):
        *cat1, x3_1 = self._forward_fe_nhwc(img1)
        *cat2, x3_2 = self._forward_fe_nhwc(img2)
        plan = self._get_plans()["pair"]
        p = float(self.den_dropout)
        thr = float(self.err_thrs)

        def fwd(a1, a2, a3, b1, b2, b3, xa, xb, tape):
            return plan.forward((a1, a2, a3), (b1, b2, b3), xa, xb, c_gt, p, thr, tape)

        return E.run_plan(plan, fwd, (*cat1, *cat2, x3_1, x3_2), plan.params())


class DGModel_memadd(_PairMixin, DGModel_mem):
    """reference models/models.py:138-184."""

    def __init__(self, pretrained=True, mem_size=1024, mem_dim=256, den_dropout=0.5, err_thrs=0.5):
        super().__init__(pretrained, mem_size, mem_dim, den_dropout)
        self.err_thrs = err_thrs
        self.den_dec = nn.Sequential(ConvBlock(512 + 256 + 128, 256, kernel_size=1, padding=0, bn=True))

    def forward_train(self, img1, img2):
        d1, d2, loss_con = self._pair(img1, img2, None)
        return d1, d2, loss_con


def _cls_head(cls_dropout):
    return nn.Sequential(
        ConvBlock(512, 256, bn=True),
        nn.Dropout2d(p=cls_dropout),
        ConvBlock(256, 1, kernel_size=1, padding=0, relu=False),
        nn.Sigmoid())


class DGModel_cls(DGModel_base):
    """reference models/models.py:186-228."""

    def __init__(self, pretrained=True, den_dropout=0.5, cls_dropout=0.5, cls_thrs=0.5):
        super().__init__(pretrained, den_dropout)
        self.cls_dropout = cls_dropout
        self.cls_thrs = cls_thrs
        self.cls_head = _cls_head(self.cls_dropout)

    def _build_head_plans(self, plans):
        plans["single"] = E.SinglePlan(self, mem=False, cls=True)

    def transform_cls_map_gt(self, c_gt):
        return upsample(c_gt, scale_factor=4, mode="nearest")

    def transform_cls_map_pred(self, c):
        c_new = (c.detach() >= self.cls_thrs).to(c.dtype)
        return upsample(c_new, scale_factor=4, mode="nearest")

    def transform_cls_map(self, c, c_gt=None):
        return self.transform_cls_map_gt(c_gt) if c_gt is not None else self.transform_cls_map_pred(c)

    _single = DGModel_mem._single

    def forward(self, x, c_gt=None):
        y1, y2, y3, x3 = self._forward_fe_nhwc(x)
        return self._single((y1, y2, y3), x3, c_gt)


class DGModel_memcls(DGModel_mem):
    """reference models/models.py:230-273."""

    _USE_MEM, _USE_CLS = True, True

    def __init__(self, pretrained=True, mem_size=1024, mem_dim=256, den_dropout=0.5, cls_dropout=0.5,
                 cls_thrs=0.5):
        super().__init__(pretrained, mem_size, mem_dim, den_dropout)
        self.cls_dropout = cls_dropout
        self.cls_thrs = cls_thrs
        self.cls_head = _cls_head(self.cls_dropout)

    transform_cls_map_gt = DGModel_cls.transform_cls_map_gt
    transform_cls_map_pred = DGModel_cls.transform_cls_map_pred
    transform_cls_map = DGModel_cls.transform_cls_map

    def forward(self, x, c_gt=None):
        y1, y2, y3, x3 = self._forward_fe_nhwc(x)
        return self._single((y1, y2, y3), x3, c_gt)


class DGModel_final(_PairMixin, DGModel_memcls):
    """reference models/models.py:275-335."""

    def __init__(self, pretrained=True, mem_size=1024, mem_dim=256, cls_thrs=0.5, err_thrs=0.5, den_dropout=0.5,
                 cls_dropout=0.5, has_err_loss=False):
        super().__init__(pretrained, mem_size, mem_dim, den_dropout, cls_dropout, cls_thrs)
        self.err_thrs = err_thrs
        self.has_err_loss = has_err_loss
        self.den_dec = nn.Sequential(
            ConvBlock(512 + 256 + 128, self.mem_dim, kernel_size=1, padding=0, bn=True))

    def forward_train(self, img1, img2, c_gt=None):
        """(dc1, dc2, c1, c2, c_err, loss_con, loss_err); loss_err = F.l1_loss(IN(y_den1), IN(y_den2))
        when has_err_loss, else 0 (models/models.py:298-335)."""
        if c_gt is None:
            raise ValueError("DGModel_final.forward_train needs c_gt (the block map)")
        outs = self._pair(img1, img2, c_gt)
        if self.has_err_loss:
            return tuple(outs)
        dc1, dc2, c1, c2, c_err, loss_con = outs
        return dc1, dc2, c1, c2, c_err, loss_con, 0
