"""TEST INFRASTRUCTURE ONLY — CPU fp32 restatement of the reference's training
hot path, used by tests/, `__graft_entry__.smoke()` and bench.py's cpu_baseline
leg as the checker.  Never imported by the product package.

Functional torch-CPU code over a state_dict (same keys as the reference):
  base_forward      models/models.py:64-96  (DGModel_base.forward_fe/forward)
  final_forward     models/models.py:298-335 (DGModel_final.forward_train)
  single_forward    models/models.py:89-273 (DGModel_base/mem/cls/memcls .forward)
  memadd_forward_train models/models.py:159-184
  train_step        trainers/dgtrainer.py:143-192 (modes simple/base/add/cls/final)
  AdamW             torch.optim.AdamW (main.py:85-86)
Pinned against fixtures produced by running the reference itself
(tests/golden/make_golden.py -> tests/golden/*.npz).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

ENC_CONVS = {"enc1": [0, 3, 7, 10, 14, 17, 20], "enc2": [1, 4, 7], "enc3": [1, 4, 7]}
ENC_POOL_FIRST = {"enc1": False, "enc2": True, "enc3": True}
# enc1 also has pools after conv 3 (idx 6) and conv 10 (idx 13)
ENC1_POOL_AFTER = {3, 10}


def _bn(x, sd, pre, training, momentum=0.1, eps=1e-5):
    rm, rv = sd[pre + ".running_mean"], sd[pre + ".running_var"]
    y = F.batch_norm(x, rm, rv, sd[pre + ".weight"], sd[pre + ".bias"], training, momentum, eps)
    if training:
        sd[pre + ".num_batches_tracked"] += 1
    return y


def _conv_bn_relu(x, sd, conv, bn, training, pad=1, relu=True, drop=None):
    b = sd.get(conv + ".bias")
    y = F.conv2d(x, sd[conv + ".weight"], b, padding=pad)
    if bn is not None:
        y = _bn(y, sd, bn, training)
    if relu:
        y = F.relu(y)
    if drop is not None:
        y = y * drop[:, :, None, None]
    return y


def _up(x, s, mode="bilinear"):
    if mode == "nearest":
        return F.interpolate(x, scale_factor=s, mode="nearest")
    return F.interpolate(x, scale_factor=s, mode="bilinear", align_corners=False)


def forward_fe(sd, x, training):
    """VGG16-BN enc1/2/3 + dec3/2/1 (models/models.py:64-87)."""
    h = x
    for i in ENC_CONVS["enc1"]:
        h = _conv_bn_relu(h, sd, f"enc1.{i}", f"enc1.{i + 1}", training)
        if i in ENC1_POOL_AFTER:
            h = F.max_pool2d(h, 2, 2)
    x1 = h
    h = F.max_pool2d(x1, 2, 2)
    for i in ENC_CONVS["enc2"]:
        h = _conv_bn_relu(h, sd, f"enc2.{i}", f"enc2.{i + 1}", training)
    x2 = h
    h = F.max_pool2d(x2, 2, 2)
    for i in ENC_CONVS["enc3"]:
        h = _conv_bn_relu(h, sd, f"enc3.{i}", f"enc3.{i + 1}", training)
    x3 = h

    def cb(t, pre):
        return _conv_bn_relu(t, sd, pre + ".conv", pre + ".bn", training)

    h = cb(cb(x3, "dec3.0"), "dec3.1")
    y3 = h
    h = torch.cat([_up(h, 2), x2], 1)
    h = cb(cb(h, "dec2.0"), "dec2.1")
    y2 = h
    h = torch.cat([_up(h, 2), x1], 1)
    h = cb(cb(h, "dec1.0"), "dec1.1")
    y1 = h
    y_cat = torch.cat([y1, _up(y2, 2), _up(y3, 4)], 1)
    return y_cat, x3


def base_forward(sd, x, training, drop=None):
    """DGModel_base.forward (models/models.py:89-96); drop = Dropout2d keep mask/(1-p)."""
    y_cat, _ = forward_fe(sd, x, training)
    y_den = _conv_bn_relu(y_cat, sd, "den_dec.0.conv", "den_dec.0.bn", training, pad=0, drop=drop)
    d = F.relu(F.conv2d(y_den, sd["den_head.0.conv.weight"], sd.get("den_head.0.conv.bias")))
    return _up(d, 4)


def forward_mem(sd, y):
    """DGModel_mem.forward_mem (models/models.py:116-125)."""
    b, k, h, w = y.shape
    m = sd["mem"].repeat(b, 1, 1)
    m_key = m.transpose(1, 2)
    logits = torch.bmm(m_key, y.view(b, k, -1)) / math.sqrt(k)
    y_new = torch.bmm(m_key.transpose(1, 2), F.softmax(logits, dim=1))
    return y_new.view(b, k, h, w), logits


def cls_head(sd, x3, training, drop=None):
    """cls_head (models/models.py:238-243)."""
    c = _conv_bn_relu(x3, sd, "cls_head.0.conv", "cls_head.0.bn", training, drop=drop)
    c = F.conv2d(c, sd["cls_head.2.conv.weight"], sd.get("cls_head.2.conv.bias"))
    return torch.sigmoid(c)


def cls_pred_map(c, thrs=0.5):
    c_new = c.clone().detach()
    c_new[c < thrs] = 0
    c_new[c >= thrs] = 1
    return _up(c_new, 4, "nearest")


def final_forward(sd, img1, img2, c_gt, training=True, err_thrs=0.5, cls_thrs=0.5,
                  drop1=None, drop2=None, e_mask_in=None, c_pred_in=None, info=None, err=None):
    """DGModel_final.forward_train (models/models.py:298-335); drop* = dropout2d masks.

    Threshold injection for full-frame parity (SURVEY.md §7 "threshold discontinuities"):
    e_mask_in (bool [B,C,h,w]) replaces the |IN1-IN2| < err_thrs mask and c_pred_in
    ((c_r1, c_r2) 0/1 maps [B,1,h/4,w/4]) the thresholded class maps, so that a checked
    path whose fp32 rounding flips a few near-threshold decisions is compared on the same
    decisions; `info` (a dict) receives how many decisions the injection changed, `err` (a dict)
    the has_err_loss term loss_err (with its autograd graph)."""
    y_cat1, x3_1 = forward_fe(sd, img1, training)
    y_cat2, x3_2 = forward_fe(sd, img2, training)
    y_den1 = _conv_bn_relu(y_cat1, sd, "den_dec.0.conv", "den_dec.0.bn", training, pad=0)
    y_den2 = _conv_bn_relu(y_cat2, sd, "den_dec.0.conv", "den_dec.0.bn", training, pad=0)
    y_in1 = F.instance_norm(y_den1, eps=1e-5)
    y_in2 = F.instance_norm(y_den2, eps=1e-5)
    e_y = torch.abs(y_in1 - y_in2)
    e_mask = (e_y < err_thrs).clone().detach()
    if err is not None:  # has_err_loss=True: loss_err = F.l1_loss(y_in1, y_in2) (models/models.py:311)
        err["loss_err"] = F.l1_loss(y_in1, y_in2)
    if e_mask_in is not None:
        flip = e_mask_in.bool() != e_mask
        if info is not None:
            info["emask_elements"] = int(e_mask.numel())
            info["emask_flips"] = int(flip.sum())
            info["emask_flip_max_margin"] = float((e_y[flip] - err_thrs).abs().max()) if flip.any() else 0.0
        e_mask = e_mask_in.bool()
    m1 = y_den1 * e_mask
    m2 = y_den2 * e_mask
    if drop1 is not None:
        m1 = m1 * drop1[:, :, None, None]
    if drop2 is not None:
        m2 = m2 * drop2[:, :, None, None]
    y_new1, logits1 = forward_mem(sd, m1)
    y_new2, logits2 = forward_mem(sd, m2)
    loss_con = F.mse_loss(F.softmax(logits1, dim=1), F.softmax(logits2, dim=1))
    c1 = cls_head(sd, x3_1, training)
    c2 = cls_head(sd, x3_2, training)
    c_resized_gt = _up(c_gt, 4, "nearest")
    c_r1 = cls_pred_map(c1, cls_thrs)
    c_r2 = cls_pred_map(c2, cls_thrs)
    if c_pred_in is not None:
        r1, r2 = (_up(c.float(), 4, "nearest") for c in c_pred_in)
        if info is not None:
            info["cls_elements"] = int(c1.numel() + c2.numel())
            info["cls_flips"] = int(((c1 >= cls_thrs).float() != c_pred_in[0].float()).sum()
                                    + ((c2 >= cls_thrs).float() != c_pred_in[1].float()).sum())
        c_r1, c_r2 = r1, r2
    c_err = torch.abs(c_r1 - c_r2)
    c_resized = torch.clamp(c_resized_gt + c_err, 0, 1)
    d1 = F.relu(F.conv2d(y_new1, sd["den_head.0.conv.weight"]))
    d2 = F.relu(F.conv2d(y_new2, sd["den_head.0.conv.weight"]))
    dc1 = _up(d1 * c_resized, 4)
    dc2 = _up(d2 * c_resized, 4)
    return dc1, dc2, c1, c2, _up(c_err, 4), loss_con, e_mask


def single_forward(sd, x, training, c_gt=None, cls_thrs=0.5):
    """`.forward` of DGModel_base / mem / cls / memcls (models/models.py:89-96, 127-136,
    208-228, 262-273), chosen by the state_dict's keys (a 'mem' entry, cls_head.* entries)."""
    y_cat, x3 = forward_fe(sd, x, training)
    y = _conv_bn_relu(y_cat, sd, "den_dec.0.conv", "den_dec.0.bn", training, pad=0)
    if "mem" in sd:
        y, _ = forward_mem(sd, y)
    d = F.relu(F.conv2d(y, sd["den_head.0.conv.weight"], sd.get("den_head.0.conv.bias")))
    if "cls_head.0.conv.weight" not in sd:
        return _up(d, 4)
    c = cls_head(sd, x3, training)
    c_resized = _up(c_gt, 4, "nearest") if c_gt is not None else cls_pred_map(c, cls_thrs)
    return _up(d * c_resized, 4), c


def memadd_forward_train(sd, img1, img2, training=True, err_thrs=0.5, e_mask_in=None):
    """DGModel_memadd.forward_train (models/models.py:159-184) with dropout p = 0; e_mask_in
    (bool [B,C,h,w]) replaces the thresholded mask, as in final_forward."""
    y_cat1, _ = forward_fe(sd, img1, training)
    y_cat2, _ = forward_fe(sd, img2, training)
    y_den1 = _conv_bn_relu(y_cat1, sd, "den_dec.0.conv", "den_dec.0.bn", training, pad=0)
    y_den2 = _conv_bn_relu(y_cat2, sd, "den_dec.0.conv", "den_dec.0.bn", training, pad=0)
    e_mask = (torch.abs(F.instance_norm(y_den1, eps=1e-5) - F.instance_norm(y_den2, eps=1e-5)) < err_thrs).detach()
    if e_mask_in is not None:
        e_mask = e_mask_in.bool()
    y_new1, logits1 = forward_mem(sd, y_den1 * e_mask)
    y_new2, logits2 = forward_mem(sd, y_den2 * e_mask)
    loss_con = F.mse_loss(F.softmax(logits1, dim=1), F.softmax(logits2, dim=1))
    d1 = _up(F.relu(F.conv2d(y_new1, sd["den_head.0.conv.weight"])), 4)
    d2 = _up(F.relu(F.conv2d(y_new2, sd["den_head.0.conv.weight"])), 4)
    return d1, d2, loss_con


def err_loss_grads(sd, batch):
    """DGModel_final(has_err_loss=True).forward_train's loss_err (models/models.py:303-311) and
    the gradients of loss_err alone with respect to every trainable entry (dropouts off)."""
    sd = {k: v.clone() for k, v in sd.items()}
    keys = trainable_keys(sd)
    for k in keys:
        sd[k].requires_grad_(True)
    imgs1, imgs2, (_points, _dmaps, bmaps) = batch
    err = {}
    final_forward(sd, imgs1, imgs2, bmaps, err=err)
    loss_err = err["loss_err"]
    grads = torch.autograd.grad(loss_err, [sd[k] for k in keys], allow_unused=True)
    return loss_err.detach(), {k: (g if g is not None else torch.zeros_like(sd[k])) for k, g in zip(keys, grads)}


def trainable_keys(sd):
    return [k for k in sd if not (k.endswith("running_mean") or k.endswith("running_var")
                                 or k.endswith("num_batches_tracked"))]


def train_step(sd, batch, mode="simple", log_para=1000.0, lr=1e-4, weight_decay=1e-4, e_mask_in=None,
               c_pred_in=None):
    """One DGTrainer.train_step (trainers/dgtrainer.py:143-192, MSE loss, AdamW step 1).
    Returns (loss, outputs, grads, new_sd).  Final mode takes final_forward's threshold
    injection (e_mask_in, c_pred_in), add mode the e_mask one, so a checked path is compared on
    its own decisions."""
    sd = {k: v.clone() for k, v in sd.items()}
    keys = trainable_keys(sd)
    for k in keys:
        sd[k].requires_grad_(True)
    imgs1, imgs2, (points, dmaps, bmaps) = batch
    gt = dmaps * log_para
    if mode == "simple":
        d1 = base_forward(sd, imgs1, True)
        loss = F.mse_loss(d1, gt)
        outs = (d1,)
    elif mode == "base":  # DGModel_base / DGModel_mem (configs/ablation/*_base.yml, *_mem.yml)
        d1 = single_forward(sd, imgs1, True)
        d2 = single_forward(sd, imgs2, True)
        loss = F.mse_loss(d1, gt) + F.mse_loss(d2, gt)
        outs = (d1, d2)
    elif mode == "add":  # DGModel_memadd (trainers/dgtrainer.py:166-173)
        d1, d2, loss_con = memadd_forward_train(sd, imgs1, imgs2, e_mask_in=e_mask_in)
        loss = F.mse_loss(d1, gt) + F.mse_loss(d2, gt) + loss_con
        outs = (d1, d2, loss_con)
    elif mode == "cls":  # DGModel_cls / DGModel_memcls (trainers/dgtrainer.py:175-183)
        d1, c1 = single_forward(sd, imgs1, True, c_gt=bmaps)
        d2, c2 = single_forward(sd, imgs2, True, c_gt=bmaps)
        loss = (F.mse_loss(d1, gt) + F.mse_loss(d2, gt)
                + 10 * (F.binary_cross_entropy(c1, bmaps) + F.binary_cross_entropy(c2, bmaps)))
        outs = (d1, d2, c1, c2)
    elif mode == "final":
        dc1, dc2, c1, c2, c_err, loss_con, _ = final_forward(sd, imgs1, imgs2, bmaps, e_mask_in=e_mask_in,
                                                             c_pred_in=c_pred_in)
        loss_den = F.mse_loss(dc1, gt) + F.mse_loss(dc2, gt)
        loss_cls = F.binary_cross_entropy(c1, bmaps) + F.binary_cross_entropy(c2, bmaps)
        loss = loss_den + 10 * loss_cls + 10 * loss_con
        outs = (dc1, dc2, c1, c2, loss_con)
    else:
        raise ValueError(mode)
    params = [sd[k] for k in keys]
    grads = torch.autograd.grad(loss, params, allow_unused=True)
    grads = {k: (g if g is not None else torch.zeros_like(sd[k])) for k, g in zip(keys, grads)}
    new_sd = {k: v.detach().clone() for k, v in sd.items()}
    for k in keys:  # torch.optim.AdamW, step 1, betas (0.9, 0.999), eps 1e-8
        p, g = new_sd[k], grads[k]
        p.mul_(1 - lr * weight_decay)
        m = (1 - 0.9) * g
        v = (1 - 0.999) * g * g
        bc1, bc2 = 1 - 0.9, 1 - 0.999
        p.addcdiv_(m, v.sqrt() / math.sqrt(bc2) + 1e-8, value=-lr / bc1)
    return loss.detach(), tuple(o.detach() for o in outs), grads, new_sd


# ---------------------------------------------------------------------------
# deterministic weights shared by the fixture generator and the tests
# ---------------------------------------------------------------------------
def seeded_state_dict(template: dict, seed: int = 2112) -> dict:
    """Deterministic values for every state_dict entry (key order of `template`)."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k, v in template.items():
        if k.endswith("num_batches_tracked"):
            out[k] = torch.zeros_like(v)
        elif k.endswith("running_mean"):
            out[k] = torch.zeros_like(v)
        elif k.endswith("running_var"):
            out[k] = torch.ones_like(v)
        elif k == "mem":
            out[k] = torch.randn(v.shape, generator=g)
        elif v.dim() == 4:
            fan_in = v.shape[1] * v.shape[2] * v.shape[3]
            out[k] = torch.randn(v.shape, generator=g) * math.sqrt(2.0 / fan_in)
        elif k.endswith("bn.weight") or (k.split(".")[-1] == "weight" and v.dim() == 1):
            out[k] = torch.rand(v.shape, generator=g) + 0.5
        else:
            out[k] = (torch.rand(v.shape, generator=g) - 0.5) * 0.2
    return out


def synthetic_batch(B, H, W, seed=2112, n_points=None, with_dmap=True):
    """SURVEY.md §8d synthetic inputs: images in [-1,1], view2 = view1 + 0.1 N(0,1),
    points ~ U over the frame, dmap via the fixed Gaussian, bmap = 16x16 block-sum>0."""
    g = torch.Generator().manual_seed(seed)
    img1 = (torch.randn(B, 3, H, W, generator=g) * 0.5).clamp(-1, 1)
    img2 = (img1 + 0.1 * torch.randn(B, 3, H, W, generator=g)).clamp(-1, 1)
    pts = []
    for _ in range(B):
        n = n_points if n_points is not None else max(1, int(500 * H * W / (768 * 1024)))
        xy = torch.rand(n, 2, generator=g) * torch.tensor([W, H], dtype=torch.float32)
        pts.append(xy)
    dmaps = torch.zeros(B, 1, H, W)
    if with_dmap:
        from .dmap_oracle import dmap_fixed
        for i, p in enumerate(pts):
            dmaps[i, 0] = torch.from_numpy(dmap_fixed(p.numpy(), H, W))
    # datasets/den_cls_dataset.py:62-63: 16x16 block sum > 0
    bmaps = (dmaps.reshape(B, 1, H // 16, 16, W // 16, 16).sum(dim=(3, 5)) > 0).float()
    return img1, img2, (tuple(pts), dmaps, bmaps)
