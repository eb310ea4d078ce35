"""ResNet-50 domain-generalisation counters on the HIP trunk plans.

Drop-ins for the reference's
  * IBNCounter_ResNet  (models/ibnnet/__init__.py:11-29; resnet50_ibn_b,
                        models/ibnnet/resnet_ibn.py:65-183,285-297)
  * SWCounter_ResNet   (models/SW/__init__.py:4-10,24-42; SwitchWhiten2d,
                        models/SW/ops/switchwhiten.py:7-183; SW ResNet,
                        models/SW/backbones/resnet.py:75-212)
  * ISWCounter_ResNet  (models/ISW/__init__.py:21-122; ISW ResNet/Bottleneck,
                        models/ISW/Resnet.py:137-216,395-495; CovMatrix_ISW,
                        models/ISW/cov_settings.py:16-89)
with the same constructor arguments, forward signatures and state_dict keys
(tests/golden/trunk_state_dict_keys.json).  The modules only hold parameters and
buffers; forward/backward run as one kernel plan (dgvcc_amd.trunk.CounterPlan).

Pretrained ImageNet weights are remote downloads in the reference
(torch.hub / model_zoo); offline, `pretrained=True` loads a local state_dict
from $DGVCC_PRETRAINED_DIR/<name>.pth when present and otherwise keeps the
random initialisation with a warning.
"""
from __future__ import annotations

import math
import os
import warnings

import torch
import torch.nn as nn

from .. import engine as E
from .. import trunk as TR
from .models import _DGBase

LAYERS = [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]


def _load_local(module: nn.Module, name: str, pretrained: bool, strict=False):
    if not pretrained:
        return
    d = os.environ.get("DGVCC_PRETRAINED_DIR", os.path.expanduser("~/.cache/dgvcc"))
    f = os.path.join(d, name + ".pth")
    if os.path.isfile(f):
        sd = torch.load(f, map_location="cpu", weights_only=True)
        module.load_state_dict(sd, strict=strict)
    else:
        warnings.warn(f"pretrained weights for {name} not found at {f} (no network); "
                      "keeping random initialisation")


def _he_normal_fan_out(m: nn.Conv2d):
    n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
    m.weight.data.normal_(0, math.sqrt(2.0 / n))


def _downsample(cin, cout, stride):
    return nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride, bias=False), nn.BatchNorm2d(cout))


def _counter_head():
    return nn.Sequential(
        nn.Conv2d(1024, 512, kernel_size=3, padding=1), nn.ReLU(inplace=True),
        nn.Conv2d(512, 256, kernel_size=3, padding=1), nn.ReLU(inplace=True),
        nn.Conv2d(256, 1, kernel_size=1), nn.UpsamplingBilinear2d(scale_factor=16))


# ---------------------------------------------------------------------------
# IBN-Net b
# ---------------------------------------------------------------------------
class Bottleneck_IBN(nn.Module):
    """resnet_ibn.py:65-107 ('b': IN after the residual add)."""
    expansion = 4

    def __init__(self, inplanes, planes, ibn=None, stride=1, downsample=None):
        super().__init__()
        if ibn == "a":
            raise NotImplementedError("IBN-a blocks are not on the DGVCC path (resnet50_ibn_b only)")
        self.conv1 = nn.Conv2d(inplanes, planes, kernel_size=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.IN = nn.InstanceNorm2d(planes * 4, affine=True) if ibn == "b" else None
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def block(self):
        ds = self.downsample
        return TR.Block(self.conv1, self.bn1, self.conv2, TR.Norm("bn", self.bn2), self.conv3,
                        self.bn3, ds[0] if ds is not None else None, ds[1] if ds is not None else None,
                        TR.Norm("in", self.IN) if self.IN is not None else None)


def _ibn_b_backbone():
    """children()[:7] of resnet50_ibn_b: conv1, bn1 (IN affine), relu, maxpool, layer1-3."""
    inplanes = 64
    mods = [nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False),
            nn.InstanceNorm2d(64, affine=True), nn.ReLU(inplace=True),
            nn.MaxPool2d(kernel_size=3, stride=2, padding=1)]
    for li, (planes, nblk, stride) in enumerate(LAYERS[:3]):
        ibn = "b" if li < 2 else None
        ds = None
        if stride != 1 or inplanes != planes * 4:
            ds = _downsample(inplanes, planes * 4, stride)
        blocks = [Bottleneck_IBN(inplanes, planes, None, stride, ds)]
        inplanes = planes * 4
        for i in range(1, nblk):
            blocks.append(Bottleneck_IBN(inplanes, planes, None if (ibn == "b" and i < nblk - 1) else ibn))
        mods.append(nn.Sequential(*blocks))
    bb = nn.Sequential(*mods)
    for m in bb.modules():
        if isinstance(m, nn.Conv2d):
            _he_normal_fan_out(m)
        elif isinstance(m, (nn.BatchNorm2d, nn.InstanceNorm2d)) and m.weight is not None:
            m.weight.data.fill_(1)
            m.bias.data.zero_()
    return bb


class _CounterBase(_DGBase):
    def _stem_norm(self) -> TR.Norm:
        raise NotImplementedError

    def _blocks(self):
        return [blk.block() for layer in self._layers() for blk in layer]

    def _get_plan(self) -> TR.CounterPlan:
        if getattr(self, "_plan", None) is None:
            self._plan = TR.CounterPlan(self._conv1(), self._stem_norm(), self._blocks(), self.head)
        return self._plan

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_plan"] = None
        return st

    def _run(self, x, iw_masks=None):
        plan = self._get_plan()
        dt = self.compute_dtype
        training = self.training
        if iw_masks is None:
            fwd = lambda img, tape=None: plan.forward(img, training, None, tape, dt)  # noqa: E731
        else:
            fwd = lambda img, tape=None: plan.forward(img, training, iw_masks, tape, dt)  # noqa: E731
        return E.run_plan(plan, fwd, (x,), plan.params())


class IBNCounter_ResNet(_CounterBase):
    """models/ibnnet/__init__.py:11-29."""

    def __init__(self, pretrained=True):
        super().__init__()
        self._init_precision()
        self.backbone = _ibn_b_backbone()
        _load_local(self.backbone, "resnet50_ibn_b", pretrained)
        self.head = _counter_head()
        self._plan = None

    def _conv1(self):
        return self.backbone[0]

    def _stem_norm(self):
        return TR.Norm("in", self.backbone[1])

    def _layers(self):
        return [self.backbone[4], self.backbone[5], self.backbone[6]]

    def forward(self, x):
        return self._run(x)


# ---------------------------------------------------------------------------
# Switchable Whitening
# ---------------------------------------------------------------------------
class SwitchWhiten2d(nn.Module):
    """Parameters/buffers of models/SW/ops/switchwhiten.py:7-81 (sw_type 2 only on the
    HIP path); the computation is dg_sw_fwd / dg_sw_bwd inside the trunk plan."""

    def __init__(self, num_features, num_pergroup=16, sw_type=2, T=5, tie_weight=False, eps=1e-5,
                 momentum=0.99, affine=True):
        super().__init__()
        if sw_type not in [2, 3, 5]:
            raise ValueError("sw_type should be in [2, 3, 5], but got {}".format(sw_type))
        assert num_features % num_pergroup == 0
        if sw_type != 2 or num_pergroup != 16 or tie_weight or not affine:
            raise NotImplementedError("HIP SwitchWhiten2d: sw_type=2, num_pergroup=16, "
                                      "tie_weight=False, affine=True (the SW counter's sw_cfg)")
        self.num_features = num_features
        self.num_pergroup = num_pergroup
        self.num_groups = num_features // num_pergroup
        self.sw_type, self.T, self.tie_weight = sw_type, T, tie_weight
        self.eps, self.momentum, self.affine = eps, momentum, affine
        self.sw_mean_weight = nn.Parameter(torch.ones(sw_type))
        self.sw_var_weight = nn.Parameter(torch.ones(sw_type))
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(self.num_groups, num_pergroup, 1))
        self.register_buffer("running_cov",
                             torch.eye(num_pergroup).unsqueeze(0).repeat(self.num_groups, 1, 1))
        self.reset_parameters()

    def reset_parameters(self):
        self.running_mean.zero_()
        self.running_cov.zero_()  # as the reference (switchwhiten.py:66-67)
        nn.init.ones_(self.sw_mean_weight)
        nn.init.ones_(self.sw_var_weight)
        nn.init.ones_(self.weight)
        nn.init.zeros_(self.bias)


class SyncSwitchWhiten2d(SwitchWhiten2d):
    """models/SW/ops/sync_switchwhiten.py:59-183: the batch (BW) mean/covariance are
    synchronised over the data-parallel ranks (SyncMeanCov).  On the HIP path the
    statistics and whitening kernels are split and the [G][272] batch moments (and, in
    backward, their adjoints) are all-reduced over RCCL in between; with one rank it
    is SwitchWhiten2d."""
    sync = True

    def __init__(self, num_features, num_pergroup=16, sw_type=2, T=5, tie_weight=False, eps=1e-5,
                 momentum=0.99, affine=True):
        super().__init__(num_features, num_pergroup, sw_type, T, tie_weight, eps, momentum, affine)


SW_CFG = dict(type="SW", sw_type=2, num_pergroup=16, T=5, tie_weight=False, momentum=0.9, affine=True)


def _make_sw(sync=False):
    cls = SyncSwitchWhiten2d if sync else SwitchWhiten2d
    return lambda c: cls(c, num_pergroup=16, sw_type=2, T=5, tie_weight=False, eps=1e-5,
                         momentum=0.9, affine=True)


class Bottleneck_SW(nn.Module):
    """SW/backbones/resnet.py:75-118: norm2 is SwitchWhiten2d ('sw2') when with_sw."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, with_sw=False, sync=False):
        super().__init__()
        self.norm2_name = "sw2" if with_sw else "bn2"
        self.conv1 = nn.Conv2d(inplanes, planes, kernel_size=1, bias=False)
        self.add_module("bn1", nn.BatchNorm2d(planes))
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.add_module(self.norm2_name, _make_sw(sync)(planes) if with_sw else nn.BatchNorm2d(planes))
        self.conv3 = nn.Conv2d(planes, planes * 4, kernel_size=1, bias=False)
        self.add_module("bn3", nn.BatchNorm2d(planes * 4))
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def block(self):
        ds = self.downsample
        n2 = getattr(self, self.norm2_name)
        return TR.Block(self.conv1, self.bn1, self.conv2, TR.Norm("sw" if self.norm2_name == "sw2" else "bn", n2),
                        self.conv3, self.bn3, ds[0] if ds is not None else None,
                        ds[1] if ds is not None else None)


def _sw_backbone(sync=False):
    """children()[:7] of SW resnet50(sw_cfg): conv1, sw1, relu, maxpool, layer1-3."""
    conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
    mods = [conv1, _make_sw(sync)(64), nn.ReLU(inplace=True), nn.MaxPool2d(kernel_size=3, stride=2, padding=1)]
    inplanes = 64
    for planes, nblk, stride in LAYERS[:3]:
        ds = None
        if stride != 1 or inplanes != planes * 4:
            ds = _downsample(inplanes, planes * 4, stride)
        blocks = [Bottleneck_SW(inplanes, planes, stride, ds, with_sw=False)]
        inplanes = planes * 4
        for i in range(1, nblk):
            blocks.append(Bottleneck_SW(inplanes, planes, with_sw=(i % 2 == 1), sync=sync))
        mods.append(nn.Sequential(*blocks))
    bb = nn.Sequential(*mods)
    for m in bb.modules():
        if isinstance(m, nn.Conv2d):
            _he_normal_fan_out(m)
        elif isinstance(m, nn.BatchNorm2d):
            m.weight.data.fill_(1)
            m.bias.data.zero_()
    return bb


class SWCounter_ResNet(_CounterBase):
    """models/SW/__init__.py:24-42.  sync=True builds SyncSwitchWhiten2d layers (batch
    whitening statistics shared over the data-parallel ranks; an extension — the
    reference's SW counter uses SwitchWhiten2d)."""

    def __init__(self, pretrained=True, sync=False):
        super().__init__()
        self._init_precision()
        self.backbone = _sw_backbone(sync)
        _load_local(self.backbone, "resnet50", pretrained)
        self.head = _counter_head()
        self._plan = None

    def _conv1(self):
        return self.backbone[0]

    def _stem_norm(self):
        return TR.Norm("sw", self.backbone[1])

    def _layers(self):
        return [self.backbone[4], self.backbone[5], self.backbone[6]]

    def forward(self, x):
        return self._run(x)


# ---------------------------------------------------------------------------
# ISW
# ---------------------------------------------------------------------------
class InstanceWhitening(nn.Module):
    """models/ISW/instance_whitening.py:5-16 (IN affine=False; w = output)."""

    def __init__(self, dim):
        super().__init__()
        self.instance_standardization = nn.InstanceNorm2d(dim, affine=False)


class Bottleneck_ISW(nn.Module):
    """models/ISW/Resnet.py:137-216 (iw in {0, 2} on the counter's wt_layer)."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, iw=0):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, kernel_size=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.downsample = downsample
        self.stride = stride
        self.iw = iw
        if iw in (1, 2):
            self.instance_norm_layer = InstanceWhitening(planes * 4)
            self.relu = nn.ReLU(inplace=False)
        elif iw == 0:
            self.relu = nn.ReLU(inplace=True)
        else:
            raise NotImplementedError("ISW iw in {3,4,5} is not selected by ISWCounter_ResNet")

    def block(self):
        ds = self.downsample
        post = TR.Norm("iw", self.instance_norm_layer.instance_standardization) if self.iw else None
        return TR.Block(self.conv1, self.bn1, self.conv2, TR.Norm("bn", self.bn2), self.conv3, self.bn3,
                        ds[0] if ds is not None else None, ds[1] if ds is not None else None, post)


class CovMatrix_ISW:
    """models/ISW/cov_settings.py:16-89, device-resident (margin path, relax_denom > 0)."""

    def __init__(self, dim, relax_denom=0, clusters=50):
        self.dim = dim
        self.clusters = clusters
        self.num_off_diagonal = dim * (dim - 1) // 2
        self.relax_denom = relax_denom
        self.margin = 0 if relax_denom == 0 else float(self.num_off_diagonal // relax_denom)
        self.var_matrix = None
        self.count_var_cov = 0
        self.mask_matrix = None
        self.num_sensitive = None

    def reset_mask_matrix(self):
        self.mask_matrix = None

    def set_mask_matrix(self):
        if self.var_matrix is None:
            raise RuntimeError("no covariance statistics: run the model with cal_covstat=True first")
        if self.margin == 0:
            raise NotImplementedError("relax_denom=0 (kmeans1d clustering) is parity-unpinned: "
                                      "kmeans1d is not available offline")
        var = (self.var_matrix / self.count_var_cov).flatten()
        k = int(self.num_off_diagonal - self.margin)
        idx = torch.topk(var, k).indices  # device top-k over <= 512^2 entries, once per epoch
        m = torch.zeros(self.dim * self.dim, dtype=torch.float32, device=var.device)
        m[idx] = 1
        m = m.view(self.dim, self.dim)
        if self.mask_matrix is not None:
            m = (self.mask_matrix.int() & m.int()).float()
        self.mask_matrix = m
        self.num_sensitive = m.sum()
        self.var_matrix = None
        self.count_var_cov = 0

    def get_mask_matrix(self):
        if self.mask_matrix is None:
            self.set_mask_matrix()
        return self.mask_matrix, self.num_sensitive

    def accumulate(self, fraw: torch.Tensor, hw: int):
        from .. import kernels as K
        if self.var_matrix is None:
            self.var_matrix = torch.empty((self.dim, self.dim), dtype=torch.float32, device=fraw.device)
            K.iw_cov_var(fraw, hw, self.var_matrix, accumulate=False)
        else:
            K.iw_cov_var(fraw, hw, self.var_matrix, accumulate=True)
        self.count_var_cov += 1


class ISWCounter_ResNet(_CounterBase):
    """models/ISW/__init__.py:21-122."""

    def __init__(self, criterion=None, variant="D", skip="m1", skip_num=48, wt_layer=None,
                 use_wtloss=True, relax_denom=2.0, clusters=3, pretrained=True):
        super().__init__()
        self._init_precision()
        self.criterion = criterion if criterion is not None else nn.MSELoss()
        self.variant = variant
        self.wt_layer = list(wt_layer) if wt_layer is not None else [0, 0, 2, 2, 2, 0, 0]
        if self.wt_layer[0] or self.wt_layer[1] or self.wt_layer[6] or \
                any(v not in (0, 2) for v in self.wt_layer):
            raise NotImplementedError("HIP ISW counter supports wt_layer entries in {0, 2} at "
                                      "positions 2-5 (the reference default is [0,0,2,2,2,0,0])")
        self.use_wtloss = use_wtloss
        self.relax_denom = relax_denom
        self.clusters = clusters
        self.eps = 1e-5
        self.whitening = False

        conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        stem_norm = InstanceWhitening(64) if self.wt_layer[2] == 2 else nn.BatchNorm2d(64)
        self.layer0 = nn.Sequential(conv1, stem_norm, nn.ReLU(inplace=self.wt_layer[2] != 2),
                                    nn.MaxPool2d(kernel_size=3, stride=2, padding=1))
        inplanes = 64
        layers = []
        for li, (planes, nblk, stride) in enumerate(LAYERS):
            wl = self.wt_layer[3 + li]
            ds = None
            if stride != 1 or inplanes != planes * 4:
                ds = _downsample(inplanes, planes * 4, stride)
            blocks = [Bottleneck_ISW(inplanes, planes, stride, ds, iw=0)]
            inplanes = planes * 4
            for i in range(1, nblk):
                blocks.append(Bottleneck_ISW(inplanes, planes, iw=0 if (wl > 0 and i < nblk - 1) else wl))
            layers.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = layers
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        self.head = _counter_head()
        if pretrained:
            _load_local(self, "resnet50", pretrained)

        in_channel_list = [0, 0, 64, 256, 512, 1024, 2048]
        self.cov_matrix_layer = []
        self.cov_type = []
        for i, v in enumerate(self.wt_layer):
            if v == 2:
                self.whitening = True
                self.cov_matrix_layer.append(CovMatrix_ISW(dim=in_channel_list[i], relax_denom=relax_denom,
                                                           clusters=clusters))
                self.cov_type.append(v)
        self._plan = None

    def _conv1(self):
        return self.layer0[0]

    def _stem_norm(self):
        n = self.layer0[1]
        if isinstance(n, InstanceWhitening):
            return TR.Norm("iw", n.instance_standardization)
        return TR.Norm("bn", n)

    def _layers(self):
        return [self.layer1, self.layer2, self.layer3]

    def set_mask_matrix(self):
        for c in self.cov_matrix_layer:
            c.set_mask_matrix()

    def reset_mask_matrix(self):
        for c in self.cov_matrix_layer:
            c.reset_mask_matrix()

    def forward(self, x, gts=None, cal_covstat=False, apply_wtloss=True):
        if cal_covstat:
            x = torch.cat(list(x), dim=0)
            plan = self._get_plan()
            with torch.no_grad():
                _, ws = plan.features(x, self.compute_dtype, self.training, None)
                for w, cm in zip(ws, self.cov_matrix_layer):
                    cm.accumulate(TR.gram(w), w.H * w.W)
            return 0
        if not self.training:
            return self._run(x)
        masks = None
        if self.use_wtloss and apply_wtloss:
            masks = [cm.get_mask_matrix() for cm in self.cov_matrix_layer]
        if masks is None:
            main_out = self._run(x)
            wt_loss = torch.zeros(1, device=x.device)
        else:
            main_out, wt = self._run(x, masks)
            wt_loss = wt.reshape(1)
        if type(self.criterion).__name__ == "MSELoss":
            from ..losses import mse_loss
            loss1 = mse_loss(main_out, gts, 1000.0)
        else:
            loss1 = self.criterion(main_out, gts * 1000)
        if not self.use_wtloss:
            return [loss1, torch.zeros(1, device=x.device)]
        return [loss1, wt_loss]
