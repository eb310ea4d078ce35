"""Drop-in MI355X implementation of `models.models2` (reference models/models2.py).

Same class names, constructor signatures, sub-module names and therefore the same
`state_dict` keys as the reference (`tests/golden/state_dict_keys.json`); the forward and
backward math run on the HIP kernel plans of `dgvcc_amd.engine` (NHWC activations,
implicit-GEMM MFMA convolutions), exactly as `dgvcc_amd.models.models`.

  DensityRegressorBase     models2.py:375-432  (`get_basemodel`, the 'dgnet' of
                           configs/stb_reg_base.yml, mall_base.yml, qnrf_final.yml)
  DensityRegressor         models2.py:105-187  (instance-normalised stages, 3x3 heads)
  DensityRegressorM        models2.py:189-373  (memory read + class head, KL-JSD)
  DensityRegressorBaseCls  models2.py:434-511
  Generator / Generator0   models2.py:29-103   (VGG19 image generators)
  get_models / get_basemodel  models2.py:513-519
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import engine as E
from . import plans2 as P2
from .models import ConvBlock, DGModel_base, _DGBase, _load_pretrained_vgg, upsample, vgg16_bn_features  # noqa: F401

__all__ = ["ConvBlock", "upsample", "Generator", "Generator0", "DensityRegressor", "DensityRegressorM",
           "DensityRegressorBase", "DensityRegressorBaseCls", "get_models", "get_basemodel"]


def _vgg16_stages(module: nn.Module, pretrained: bool):
    features = vgg16_bn_features()
    if pretrained:
        _load_pretrained_vgg(features)
    ch = list(features.children())
    module.stage1 = nn.Sequential(*ch[:23])
    module.stage2 = nn.Sequential(*ch[23:33])
    module.stage3 = nn.Sequential(*ch[33:43])


def _vgg_decoder(module: nn.Module):
    module.dec3 = nn.Sequential(ConvBlock(512, 1024, bn=True), ConvBlock(1024, 512, bn=True))
    module.dec2 = nn.Sequential(ConvBlock(1024, 512, bn=True), ConvBlock(512, 256, bn=True))
    module.dec1 = nn.Sequential(ConvBlock(512, 256, bn=True), ConvBlock(256, 128, bn=True))


class DensityRegressorBase(DGModel_base):
    """reference models/models2.py:375-432: the DGModel_base network with stage1/2/3 keys, a
    BN-free den_dec (1x1 896->256 + ReLU + Dropout2d(0.5)) and a bare ConvBlock den_head.
    Runs on the same plans (FeaturePlan + decomposed-concat DensityPlan)."""

    _ENC_NAMES = ("stage1", "stage2", "stage3")

    def __init__(self, pretrained=True):
        _DGBase.__init__(self)
        self._init_precision()
        _vgg16_stages(self, pretrained)
        _vgg_decoder(self)
        self.den_dec = nn.Sequential(ConvBlock(512 + 256 + 128, 256, kernel_size=1, padding=0),
                                     nn.Dropout2d(p=0.5))
        self.den_head = ConvBlock(256, 1, kernel_size=1, padding=0)
        self._plans = None

    @property
    def den_dropout(self):
        return self.den_dec[1].p

    @den_dropout.setter
    def den_dropout(self, p):
        if "den_dec" in self._modules:
            self.den_dec[1].p = p

    def _build_head_plans(self, plans):
        plans["den"] = E.DensityPlan(self.den_dec[0], self.den_head, self.den_dropout)

    def forward_fe(self, x):
        raise AttributeError("DensityRegressorBase has no forward_fe (reference models2.py:375-432)")


class DensityRegressor(_DGBase):
    """reference models/models2.py:105-187: instance_norm after every VGG stage, 3x3 density and
    class heads without BatchNorm (Dropout2d 0.2 between blocks); returns (dc, d, c, x3)."""

    _ENC_NAMES = ("stage1", "stage2", "stage3")

    def __init__(self, pretrained=True):
        super().__init__()
        self._init_precision()
        _vgg16_stages(self, pretrained)
        _vgg_decoder(self)
        self.den_head = nn.Sequential(
            ConvBlock(512 + 256 + 128, 256, kernel_size=1, padding=0), nn.Dropout2d(p=0.2),
            ConvBlock(256, 256), nn.Dropout2d(p=0.2),
            ConvBlock(256, 256), nn.Dropout2d(p=0.2),
            ConvBlock(256, 1, kernel_size=1, padding=0))
        self.cls_head = nn.Sequential(
            ConvBlock(512, 256), nn.Dropout2d(p=0.2),
            ConvBlock(256, 256), nn.Dropout2d(p=0.2),
            ConvBlock(256, 256), nn.Dropout2d(p=0.2),
            ConvBlock(256, 1, kernel_size=1, padding=0, relu=False),
            nn.Sigmoid())
        self.thrs = 0.5
        self._plans = None

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_plans"] = None
        return st

    def _get_plans(self):
        if self._plans is None:
            self._plans = {"fe": E.FeaturePlan(self, inorm=True),
                           "den": P2.ChainPlan(self.den_head, cat_input=True),
                           "cls": P2.ChainPlan(self.cls_head)}
        return self._plans

    def forward(self, x, c_gt=None):
        plans = self._get_plans()
        fe, den, cls = plans["fe"], plans["den"], plans["cls"]
        dt = self.compute_dtype
        y1, y2, y3, x3 = E.run_plan(fe, lambda img, tape: fe.forward(img, dt, self.training, tape), (x,),
                                    fe.params())
        d = P2.run_chain(den, (y1, y2, y3), self.training, dt)      # [N,1,h,w] f32
        c = P2.run_chain(cls, (x3,), self.training, dt)             # [N,1,h/4,w/4] f32
        dc = P2.masked_up4(d, c, c_gt, self.thrs)
        return dc, d, c, x3.permute(0, 3, 1, 2)


class DensityRegressorBaseCls(_DGBase):
    """reference models/models2.py:434-511: DensityRegressorBase plus a class branch
    (cls_dec 3x3 512->256 + Dropout2d(0.5), cls_head 1x1 + Sigmoid); returns (dc, (d, c))."""

    _ENC_NAMES = ("stage1", "stage2", "stage3")

    def __init__(self, pretrained=True):
        super().__init__()
        self._init_precision()
        _vgg16_stages(self, pretrained)
        _vgg_decoder(self)
        self.den_dec = nn.Sequential(ConvBlock(512 + 256 + 128, 256, kernel_size=1, padding=0),
                                     nn.Dropout2d(p=0.5))
        self.cls_dec = nn.Sequential(ConvBlock(512, 256), nn.Dropout2d(p=0.5))
        self.den_head = ConvBlock(256, 1, kernel_size=1, padding=0)
        self.cls_head = nn.Sequential(ConvBlock(256, 1, kernel_size=1, padding=0, relu=False), nn.Sigmoid())
        self._plans = None

    __getstate__ = DensityRegressor.__getstate__

    def _get_plans(self):
        if self._plans is None:
            self._plans = {"fe": E.FeaturePlan(self),
                           "den": P2.ChainPlan(list(self.den_dec) + [self.den_head], cat_input=True),
                           "cls": P2.ChainPlan(list(self.cls_dec) + list(self.cls_head))}
        return self._plans

    def forward(self, x, c_gt=None):
        plans = self._get_plans()
        fe, den, cls = plans["fe"], plans["den"], plans["cls"]
        dt = self.compute_dtype
        y1, y2, y3, x3 = E.run_plan(fe, lambda img, tape: fe.forward(img, dt, self.training, tape), (x,),
                                    fe.params())
        d = P2.run_chain(den, (y1, y2, y3), self.training, dt)
        c = P2.run_chain(cls, (x3,), self.training, dt)
        dc = P2.masked_up4(d, c, c_gt, 0.5)
        return dc, (d, c)


class DensityRegressorM(_DGBase):
    """reference models/models2.py:189-373: den_dec (1x1 + BN) -> memory read (1024 slots) ->
    den_head; class head on x3.  forward(x, c_gt, raw) -> (dc, c); forward_train(img1, img2,
    c_gt) -> (dc1, dc2, c1, c2, loss_kl, loss_err) with the JSD of the two slot posteriors
    (KL to their mean, batchmean / HW) and the L1 distance of the instance-normalised features."""

    _ENC_NAMES = ("stage1", "stage2", "stage3")

    def __init__(self, pretrained=True):
        super().__init__()
        self._init_precision()
        self.thrs = 0.5
        self.train_dropout = 0.5  # the functional F.dropout2d(y_den, 0.5) of forward_train (models2.py:331-332)
        self.part_num = 1024
        self.final_dim = 256
        variance = 1.0
        _vgg16_stages(self, pretrained)
        _vgg_decoder(self)
        self.den_dec = nn.Sequential(ConvBlock(512 + 256 + 128, self.final_dim, kernel_size=1, padding=0, bn=True))
        self.mem = nn.Parameter(torch.FloatTensor(1, self.final_dim, self.part_num).normal_(0.0, variance))
        self.den_head = ConvBlock(self.final_dim, 1, kernel_size=1, padding=0)
        self.cls_head = nn.Sequential(
            ConvBlock(512, 256, bn=True), nn.Dropout2d(p=0.5),
            ConvBlock(256, 1, kernel_size=1, padding=0, relu=False), nn.Sigmoid())
        self._plans = None

    __getstate__ = DensityRegressor.__getstate__

    # attributes the shared engine heads read (DGModel_* names)
    @property
    def cls_thrs(self):
        return self.thrs

    def _get_plans(self):
        if self._plans is None:
            single = E.SinglePlan(self, mem=True, cls=True)
            pair = E.PairPlan(self, cls=True, variant="M")
            self._plans = {"fe": E.FeaturePlan(self), "single": single, "pair": pair}
        return self._plans

    def forward_fe(self, x):
        from .models import _CatPlan
        fe = self._get_plans()["fe"]
        dt = self.compute_dtype
        y1, y2, y3, x3 = E.run_plan(fe, lambda img, tape: fe.forward(img, dt, self.training, tape), (x,),
                                    fe.params())
        ycat = _CatPlan()(y1, y2, y3)
        return ycat.permute(0, 3, 1, 2), x3.permute(0, 3, 1, 2)

    def _fe(self, x):
        fe = self._get_plans()["fe"]
        dt = self.compute_dtype
        return E.run_plan(fe, lambda img, tape: fe.forward(img, dt, self.training, tape), (x,), fe.params())

    def forward(self, x, c_gt=None, raw=True):
        y1, y2, y3, x3 = self._fe(x)
        plan = self._get_plans()["single"]
        plan.raw = bool(raw)

        def fwd(a, b, c, xx, tape):
            return plan.forward((a, b, c), xx, c_gt, self.training, tape)

        return E.run_plan(plan, fwd, (y1, y2, y3, x3), plan.params())

    def forward_train(self, img1, img2, c_gt=None):
        *cat1, x3_1 = self._fe(img1)
        *cat2, x3_2 = self._fe(img2)
        plan = self._get_plans()["pair"]

        def fwd(a1, a2, a3, b1, b2, b3, xa, xb, tape):
            return plan.forward((a1, a2, a3), (b1, b2, b3), xa, xb, c_gt, float(self.train_dropout), 0.5, tape)

        return E.run_plan(plan, fwd, (*cat1, *cat2, x3_1, x3_2), plan.params())


class Generator(_DGBase):
    """reference models/models2.py:29-56: VGG19 features[:26] (conv1_1 .. conv4_4, no final ReLU)
    -> BN ConvBlock decoder with three bilinear x2 upsamplings -> 1x1 64->3 + Tanh."""

    def __init__(self):
        super().__init__()
        self._init_precision()
        self.enc = nn.Sequential(*list(_vgg19_features().children())[:26])
        self.dec = nn.Sequential(
            ConvBlock(512, 512, bn=True),
            ConvBlock(512, 256, bn=True),
            nn.Upsample(scale_factor=2, mode="bilinear", align_corners=False),
            ConvBlock(256, 256, bn=True),
            ConvBlock(256, 256, bn=True),
            ConvBlock(256, 256, bn=True),
            ConvBlock(256, 128, bn=True),
            nn.Upsample(scale_factor=2, mode="bilinear", align_corners=False),
            ConvBlock(128, 128, bn=True),
            ConvBlock(128, 64, bn=True),
            nn.Upsample(scale_factor=2, mode="bilinear", align_corners=False),
            ConvBlock(64, 64, bn=True),
            ConvBlock(64, 3, kernel_size=1, padding=0, relu=False),
            nn.Tanh())
        self._plans = None

    __getstate__ = DensityRegressor.__getstate__

    def forward(self, x):
        if self._plans is None:
            self._plans = {"g": P2.ChainPlan(list(self.enc) + list(self.dec), image_input=True)}
        return P2.run_chain(self._plans["g"], (x,), self.training, self.compute_dtype)


class Generator0(_DGBase):
    """reference models/models2.py:58-103: VGG19 enc1/enc2/enc3 (features[:9], [9:18], [18:26])
    with a U-Net decoder (upsample x2 + concat of the skip features) and a 64->3 Tanh head."""

    def __init__(self):
        super().__init__()
        self._init_precision()
        feats = list(_vgg19_features().children())
        self.enc1 = nn.Sequential(*feats[:9])
        self.enc2 = nn.Sequential(*feats[9:18])
        self.enc3 = nn.Sequential(*feats[18:26])
        self.dec3 = nn.Sequential(ConvBlock(512, 512, bn=True), ConvBlock(512, 256, bn=True))
        self.dec2 = nn.Sequential(ConvBlock(512, 256, bn=True), ConvBlock(256, 128, bn=True))
        self.dec1 = nn.Sequential(ConvBlock(256, 128, bn=True), ConvBlock(128, 64, bn=True))
        self.head = nn.Sequential(ConvBlock(64, 64, bn=True), ConvBlock(64, 3, kernel_size=1, padding=0, relu=False),
                                  nn.Tanh())
        self._plans = None

    __getstate__ = DensityRegressor.__getstate__

    def forward(self, x):
        if self._plans is None:
            self._plans = {"g": P2.UNetPlan(self)}
        return P2.run_unet(self._plans["g"], x, self.training, self.compute_dtype)


def _vgg19_features() -> nn.Sequential:
    """torchvision vgg19().features layout (cfg "E", no BN), torchvision init.  The reference
    loads VGG19_Weights.DEFAULT (models2.py:32,61), a remote download: random init offline."""
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
           512, 512, 512, 512, "M"]
    layers, cin = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
            continue
        conv = nn.Conv2d(cin, v, kernel_size=3, padding=1)
        nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
        nn.init.constant_(conv.bias, 0)
        layers += [conv, nn.ReLU(inplace=True)]
        cin = v
    return nn.Sequential(*layers)


def get_models():
    """reference models/models2.py:513-516."""
    return Generator(), DensityRegressorM()


def get_basemodel():
    """reference models/models2.py:518-519."""
    return DensityRegressorBase()
