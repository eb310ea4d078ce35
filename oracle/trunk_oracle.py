"""TEST INFRASTRUCTURE ONLY — CPU restatement (torch ops, any float dtype) of
the ResNet-50 domain-generalisation trunks of the reference: IBN-Net-b, ISW
(instance selective whitening) and SW (switchable whitening), their counter
heads and the ISW whitening loss.  Used by tests/ and the fixture script as the
checker; never imported by the product package.

Pinned against the reference itself: tests/golden/make_golden.py runs the
reference modules (pretrained=False, seeded weights) and stores their outputs in
tests/golden/{sw_op,iw_loss,trunk_*}.npz; tests/test_trunk_oracle.py checks this
file against those fixtures.

Each function cites the reference code it restates.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


# ---------------------------------------------------------------------------
# norms
# ---------------------------------------------------------------------------
def batch_norm(x, sd, pre, training, momentum=0.1, eps=1e-5):
    """nn.BatchNorm2d / SyncBatchNorm without a process group (ISW mynn.Norm2d)."""
    rm, rv = sd[pre + "running_mean"], sd[pre + "running_var"]
    return F.batch_norm(x, rm, rv, sd[pre + "weight"], sd[pre + "bias"], training, momentum, eps)


def instance_norm(x, sd=None, pre=None, eps=1e-5):
    """nn.InstanceNorm2d(affine=sd is not None, track_running_stats=False)."""
    w = sd[pre + "weight"] if sd is not None else None
    b = sd[pre + "bias"] if sd is not None else None
    return F.instance_norm(x, weight=w, bias=b, eps=eps)


def switch_whiten(x, sd, pre, training, T=5, eps=1e-5, momentum=0.9, group=16):
    """SwitchWhiten2d sw_type=2 (BW + IW), models/SW/ops/switchwhiten.py:84-183.

    Batch statistics pool all N*H*W pixels of a 16-channel group; instance
    statistics pool one image's H*W pixels.  mean/cov are mixed with softmax
    weights, the whitening matrix is cov^{-1/2} by T Newton-Schulz steps on the
    trace-normalised covariance, then the affine map is applied."""
    N, C, H, W = x.shape
    c, g = group, C // group
    xt = x.transpose(0, 1).reshape(g, c, -1)
    if training:
        mean_bn = xt.mean(-1, keepdim=True)
        xc = xt - mean_bn
        cov_bn = xc @ xc.transpose(1, 2) / (N * H * W)
        with torch.no_grad():
            sd[pre + "running_mean"].mul_(momentum).add_((1 - momentum) * mean_bn)
            sd[pre + "running_cov"].mul_(momentum).add_((1 - momentum) * cov_bn)
    else:
        mean_bn = sd[pre + "running_mean"]
        cov_bn = sd[pre + "running_cov"]
    mean_bn = mean_bn.reshape(1, g, c, 1).expand(N, g, c, 1).reshape(N * g, c, 1)
    cov_bn = cov_bn.reshape(1, g, c, c).expand(N, g, c, c).reshape(N * g, c, c)
    xi = x.reshape(N * g, c, -1)
    mean_in = xi.mean(-1, keepdim=True)
    xic = xi - mean_in
    cov_in = xic @ xic.transpose(1, 2) / (H * W)
    a = torch.softmax(sd[pre + "sw_mean_weight"], 0)
    b = torch.softmax(sd[pre + "sw_var_weight"], 0)
    eye = torch.eye(c, dtype=x.dtype)
    mean = a[0] * mean_bn + a[1] * mean_in
    cov = b[0] * cov_bn + b[1] * cov_in + eps * eye
    r = 1.0 / torch.diagonal(cov, dim1=1, dim2=2).sum(-1).reshape(-1, 1, 1)
    covn = cov * r
    P = eye.expand(N * g, c, c)
    for _ in range(T):
        P = 1.5 * P - 0.5 * (P @ P @ P) @ covn
    wm = P * r.sqrt()
    y = (wm @ (xi - mean)).reshape(N, C, H, W)
    return y * sd[pre + "weight"].reshape(1, C, 1, 1) + sd[pre + "bias"].reshape(1, C, 1, 1)


# ---------------------------------------------------------------------------
# ISW whitening loss (models/ISW/instance_whitening.py:19-39, __init__.py:93-120,
# cov_settings.py:16-81)
# ---------------------------------------------------------------------------
def covariance(f_map, eps=1e-5):
    B, C, H, W = f_map.shape
    f = f_map.reshape(B, C, -1)
    return f @ f.transpose(1, 2) / (H * W - 1) + eps * torch.eye(C, dtype=f_map.dtype)


def whitening_loss(f_map, mask, num_sensitive):
    f_cor = covariance(f_map)
    s = (f_cor * mask).abs().sum(dim=(1, 2)) / num_sensitive
    return s.clamp(min=0).sum() / f_map.shape[0]


def cov_variance(f_map):
    """var over the batch of the strictly-upper off-diagonal covariance (cal_covstat)."""
    C = f_map.shape[1]
    upper = torch.ones(C, C, dtype=f_map.dtype).triu(diagonal=1)
    return torch.var(covariance(f_map) * upper, dim=0)


def sensitive_mask(var_sum, count, relax_denom=2.0):
    """CovMatrix_ISW.set_mask_matrix, margin path (relax_denom > 0)."""
    C = var_sum.shape[0]
    v = (var_sum / count).flatten()
    n_off = C * (C - 1) // 2
    k = n_off - int(n_off // relax_denom)
    idx = torch.topk(v, k).indices
    m = torch.zeros(C * C, dtype=var_sum.dtype)
    m[idx] = 1
    return m.view(C, C), float(k)


# ---------------------------------------------------------------------------
# ResNet-50 bottleneck trunks to layer3
# ---------------------------------------------------------------------------
LAYERS = [(64, 3, 1), (128, 4, 2), (256, 6, 2)]  # planes, blocks, stride


def _conv(x, sd, key, stride=1, pad=0):
    return F.conv2d(x, sd[key], sd.get(key[:-len("weight")] + "bias"), stride=stride, padding=pad)


def bottleneck(x, sd, pre, stride, training, norm2="bn", post=None, out_w=None):
    """Bottleneck.forward: resnet_ibn.py:84-107 / ISW Resnet.py:187-216 /
    SW backbones/resnet.py:100-118.  post: None | 'in' (IBN-b IN after the residual
    add) | 'iw' (ISW InstanceWhitening; the normalised map is appended to out_w)."""
    o = F.relu(batch_norm(_conv(x, sd, pre + "conv1.weight"), sd, pre + "bn1.", training))
    z2 = _conv(o, sd, pre + "conv2.weight", stride, 1)
    if norm2 == "sw":
        o = F.relu(switch_whiten(z2, sd, pre + "sw2.", training))
    else:
        o = F.relu(batch_norm(z2, sd, pre + "bn2.", training))
    o = batch_norm(_conv(o, sd, pre + "conv3.weight"), sd, pre + "bn3.", training)
    if pre + "downsample.0.weight" in sd:
        r = batch_norm(_conv(x, sd, pre + "downsample.0.weight", stride), sd, pre + "downsample.1.",
                       training)
    else:
        r = x
    o = o + r
    if post == "in":
        o = instance_norm(o, sd, pre + "IN.")
    elif post == "iw":
        o = instance_norm(o)
        out_w.append(o)
    return F.relu(o)


def trunk(kind, x, sd, training, out_w=None):
    """conv1 7x7/2 + stem norm + ReLU + maxpool 3x3/2/1 + layer1..3.
    kind: 'ibn' (resnet50_ibn_b, resnet_ibn.py:124-183,285-297), 'sw'
    (SW resnet50 with sw_cfg, SW/backbones/resnet.py:121-212, SW/__init__.py:4-10),
    'isw' (ISW resnet50 wt_layer [0,0,2,2,2,0,0], ISW/Resnet.py:395-495)."""
    if kind == "isw":
        stem, lay = "layer0.", ["layer1.", "layer2.", "layer3."]
        conv1 = "layer0.0.weight"
    else:
        stem, lay = "backbone.", ["backbone.4.", "backbone.5.", "backbone.6."]
        conv1 = "backbone.0.weight"
    x = F.conv2d(x, sd[conv1], stride=2, padding=3)
    if kind == "ibn":
        x = instance_norm(x, sd, stem + "1.")
    elif kind == "sw":
        x = switch_whiten(x, sd, stem + "1.", training)
    else:
        x = instance_norm(x)
        out_w.append(x)
    x = F.max_pool2d(F.relu(x), 3, 2, 1)
    for li, (planes, nblk, stride) in enumerate(LAYERS):
        for b in range(nblk):
            pre = f"{lay[li]}{b}."
            norm2 = "sw" if (kind == "sw" and b % 2 == 1) else "bn"
            post = None
            if b == nblk - 1 and li < 2:
                post = {"ibn": "in", "isw": "iw"}.get(kind)
            x = bottleneck(x, sd, pre, stride if b == 0 else 1, training, norm2, post, out_w)
    return x


def counter_head(x, sd):
    """head: 3x3 1024->512 +ReLU, 3x3 512->256 +ReLU, 1x1 256->1,
    UpsamplingBilinear2d(16) (align_corners=True) (ibnnet/__init__.py:17-24)."""
    x = F.relu(F.conv2d(x, sd["head.0.weight"], sd["head.0.bias"], padding=1))
    x = F.relu(F.conv2d(x, sd["head.2.weight"], sd["head.2.bias"], padding=1))
    x = F.conv2d(x, sd["head.4.weight"], sd["head.4.bias"])
    return F.interpolate(x, scale_factor=16, mode="bilinear", align_corners=True)


def counter_forward(kind, x, sd, training):
    w = []
    out = counter_head(trunk(kind, x, sd, training, w), sd)
    return out, w


def isw_train_forward(x, gts, sd, masks, apply_wtloss=True):
    """ISWCounter_ResNet.forward (training): [MSE(out, gts*1000), wt_loss]
    (ISW/__init__.py:106-120); masks = [(mask, num_sensitive)] per whitened layer."""
    out, w = counter_forward("isw", x, sd, True)
    loss1 = F.mse_loss(out, gts * 1000)
    wt = torch.zeros((), dtype=x.dtype)
    if apply_wtloss:
        for f_map, (mask, ns) in zip(w, masks):
            wt = wt + whitening_loss(f_map, mask, ns)
    return loss1, wt / len(w), out
