"""Float64 vector-Jacobian products evaluated at the HIP plan's own saved fp32 activations
("exact given the forward"): a checker for the hand-scheduled backward of the DGModel plans
(dgvcc_amd/engine.py) that no fp32 rounding of the forward can move.

The reference graph is the reference's network (models/models.py:35-96, 116-125, 237-259,
298-335) rebuilt in float64 torch autograd, layer by layer, with two devices that pin it to
the HIP forward that actually ran:

  * every layer's input VALUE is the HIP activation that layer read, taken from the plan's tape
    (straight-through: `hip + (ref - ref.detach())` carries HIP's value forward and the float64
    gradient backward), so every Jacobian is evaluated at the HIP forward's own point;
  * every discrete decision is the HIP forward's: ReLU masks from the taped pre-BN z and the
    BN scale/shift exactly as the kernels decide them (fmaf(z, scale, shift) > 0, norm.hip),
    max-pool argmaxes as the first max of the rounded f32 activations (norm.hip first_max4),
    the density head's ReLU from its stored output, the e_mask and the class-map thresholds
    from the plan's saved masks.

What remains between the HIP backward and this one is fp32 rounding of the backward itself.
Test infrastructure only (imported by tests/test_model_gpu.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from dgvcc_amd import engine as E


def nchw64(t: torch.Tensor) -> torch.Tensor:
    """NHWC device tensor -> NCHW float64 on the CPU."""
    return t.detach().permute(0, 3, 1, 2).double().cpu().contiguous()


def act64(a) -> torch.Tensor:
    return nchw64(a.view())


def st(hip: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
    """HIP's value forward, the float64 gradient of `ref` backward."""
    return hip + (ref - ref.detach())


def _affine32(z: torch.Tensor, stats: torch.Tensor) -> torch.Tensor:
    """fmaf(z, scale, shift) as the kernels compute it, rounded to f32 (z*scale is exact in f64)."""
    sc = stats[2].double().cpu().view(1, -1, 1, 1)
    sf = stats[3].double().cpu().view(1, -1, 1, 1)
    return (z * sc + sf).float()


def relu_mask(z_hip64: torch.Tensor, stats: torch.Tensor) -> torch.Tensor:
    return _affine32(z_hip64, stats) > 0


def pool_argmax(z_hip64: torch.Tensor, stats: torch.Tensor, act: int) -> torch.Tensor:
    """Index (0..3, row-major in the 2x2 window) of the first max of the rounded activations."""
    y = _affine32(z_hip64, stats)
    if act == E.ACT_RELU:
        y = y.clamp_min(0.0)
    N, C, H, W = y.shape
    win = y.view(N, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(N, C, H // 2, W // 2, 4)
    return win.argmax(-1, keepdim=True)  # first occurrence of the max, as first_max4


def pool_gather(y: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    N, C, H, W = y.shape
    win = y.view(N, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(N, C, H // 2, W // 2, 4)
    return win.gather(-1, idx).squeeze(-1)


def bn_train64(z: torch.Tensor, gamma, beta, eps=1e-5) -> torch.Tensor:
    return F.batch_norm(z, None, None, gamma, beta, True, 0.0, eps)


class Params64:
    """float64 leaf copies of a model's parameters (requires_grad), keyed by the nn.Parameter."""

    def __init__(self, model):
        self.by_param = {}
        self.names = {}
        for n, p in model.named_parameters():
            q = p.detach().double().cpu().clone().requires_grad_(True)
            self.by_param[p] = q
            self.names[p] = n

    def __call__(self, p):
        return None if p is None else self.by_param[p]

    def grads(self):
        return {self.names[p]: (q.grad if q.grad is not None else torch.zeros_like(q))
                for p, q in self.by_param.items()}


def conv_layer(L: E.ConvLayer, tape: dict, x_in: torch.Tensor, P: Params64, pool: bool = False):
    """One ConvLayer (conv [+ BN(train)] [+ ReLU]) at its taped point; returns (y, pooled or None).
    x_in: the layer input carrying HIP's value (already straight-through)."""
    x, z, stats, _wp, drop, _tr = tape[L]
    assert drop is None, "the exact-given-forward checker runs with dropout p = 0"
    zr = F.conv2d(x_in, P(L.conv.weight), P(L.conv.bias), padding=L.pad)
    z_hip = act64(z)
    if L.bn is not None:
        zr = bn_train64(zr, P(L.bn.weight), P(L.bn.bias))
    y = zr
    if L.act == E.ACT_RELU:
        y = zr * relu_mask(z_hip, stats)
    pooled = None
    if pool:
        pooled = pool_gather(y, pool_argmax(z_hip, stats, L.act))
    return y, pooled


def up(x, s):
    return F.interpolate(x, scale_factor=s, mode="bilinear", align_corners=False)


def feature_ref(fe: E.FeaturePlan, tape: dict, img64: torch.Tensor, P: Params64, outs):
    """FeaturePlan.forward (forward_fe, models/models.py:64-87) at the taped point: returns
    (y1, y2, y3, x3) float64 NCHW graphs whose values are HIP's.  outs: the (y1, y2, y3, x3)
    NHWC tensors that forward returned."""
    assert not fe.inorm
    hy1, hy2, hy3, _ = outs
    Ee, D = fe.enc, fe.dec
    s = tape[fe]

    def xin(L, ref):
        return st(act64(tape[L][0]), ref)

    h, _ = conv_layer(Ee[0], tape, img64, P)
    _, p = conv_layer(Ee[1], tape, xin(Ee[1], h), P, pool=True)
    h, _ = conv_layer(Ee[2], tape, xin(Ee[2], p), P)
    _, p = conv_layer(Ee[3], tape, xin(Ee[3], h), P, pool=True)
    h, _ = conv_layer(Ee[4], tape, xin(Ee[4], p), P)
    h, _ = conv_layer(Ee[5], tape, xin(Ee[5], h), P)
    x1, p = conv_layer(Ee[6], tape, xin(Ee[6], h), P, pool=True)
    h, _ = conv_layer(Ee[7], tape, xin(Ee[7], p), P)
    h, _ = conv_layer(Ee[8], tape, xin(Ee[8], h), P)
    x2, p = conv_layer(Ee[9], tape, xin(Ee[9], h), P, pool=True)
    h, _ = conv_layer(Ee[10], tape, xin(Ee[10], p), P)
    h, _ = conv_layer(Ee[11], tape, xin(Ee[11], h), P)
    x3, _ = conv_layer(Ee[12], tape, xin(Ee[12], h), P)
    x3 = st(act64(s["x3"]), x3)
    h, _ = conv_layer(D[0], tape, x3, P)
    y3, _ = conv_layer(D[1], tape, xin(D[1], h), P)
    y3 = st(nchw64(hy3), y3)
    dec2 = torch.cat([up(y3, 2), x2], 1)
    h, _ = conv_layer(D[2], tape, xin(D[2], dec2), P)
    y2, _ = conv_layer(D[3], tape, xin(D[3], h), P)
    y2 = st(nchw64(hy2), y2)
    dec1 = torch.cat([up(y2, 2), x1], 1)
    h, _ = conv_layer(D[4], tape, xin(D[4], dec1), P)
    y1, _ = conv_layer(D[5], tape, xin(D[5], h), P)
    y1 = st(nchw64(hy1), y1)
    return y1, y2, y3, x3


def _den_dec(layer: E.CatConvLayer, sub: dict, parts, P: Params64):
    """den_dec (1x1 conv + BN + ReLU on cat[y1, up2 y2, up4 y3], models/models.py:55-58, 84)."""
    _x, z, stats, _wps, drop, _tr = sub[layer]
    assert drop is None
    y1, y2, y3 = parts
    ycat = torch.cat([y1, up(y2, 2), up(y3, 4)], 1)
    zr = F.conv2d(ycat, P(layer.conv.weight), P(layer.conv.bias))
    zr = bn_train64(zr, P(layer.bn.weight), P(layer.bn.bias))
    return zr * relu_mask(act64(z), stats)


def _cls_head(heads: E._Heads, sub: dict, key: str, x3: torch.Tensor, P: Params64):
    """cls_head (models/models.py:238-243): ConvBlock(512, 256, bn) + 1x1 -> 1 + sigmoid."""
    csub, _a, _c, _shape, _dt = sub[key]
    a, _ = conv_layer(heads.cls, csub, x3, P)
    return torch.sigmoid(F.conv2d(a, P(heads.cls_w), P(heads.cls_b)))


def pair_ref(pair: E.PairPlan, tp: dict, parts1, parts2, x31, x32, P: Params64):
    """PairPlan.forward (DGModel_final / memadd forward_train, models/models.py:147-184,
    298-335) at the taped point, with the HIP e_mask / class decisions; returns the outputs
    (dc1, dc2, c1, c2, loss_con) for final, (d1, d2, loss_con) for memadd."""
    s = tp[pair]
    assert pair.variant == "final" and s["d1"] is None and s["d2"] is None
    N, h, w = s["cat1"].N, s["cat1"].H, s["cat1"].W
    C = pair.den.Cout
    yd1 = _den_dec(pair.den, s["s1"], parts1, P)
    yd2 = _den_dec(pair.den, s["s2"], parts2, P)
    emask = s["mask"].view(N, h, w, C).permute(0, 3, 1, 2).bool().cpu()
    m1 = st(act64(s["m1"]), yd1 * emask)
    m2 = st(act64(s["m2"]), yd2 * emask)
    mem = P(pair.memr.mem)[0]  # [k, S]
    k = mem.shape[0]

    def read(m):
        logits = torch.einsum("ks,nkp->nsp", mem, m.reshape(N, k, h * w)) / k ** 0.5
        Pm = torch.softmax(logits, 1)
        return torch.einsum("ks,nsp->nkp", mem, Pm).reshape(N, k, h, w), Pm

    yn1, P1 = read(m1)
    yn2, P2 = read(m2)
    loss_con = F.mse_loss(P1, P2)

    def head(yn, yh_hip):
        d = F.conv2d(yn, P(pair.head_w), P(pair.head_b))
        if pair.head_act == E.ACT_RELU:
            d = d * (yh_hip.detach().double().cpu().view(N, 1, h, w) > 0)
        return d

    d1 = head(yn1, s["yh1"])
    d2 = head(yn2, s["yh2"])
    if pair.cls is None:
        return up(d1, 4), up(d2, 4), loss_con
    c1 = _cls_head(pair, s["sub"], "c1", x31, P)
    c2 = _cls_head(pair, s["sub"], "c2", x32, P)
    cres = s["cres"].double().cpu().view(N, 1, h, w)
    outs = (up(d1 * cres, 4), up(d2 * cres, 4), c1, c2, loss_con)
    if "y1" in s:  # has_err_loss: loss_err = F.l1_loss(IN(y_den1), IN(y_den2)) (models/models.py:303-311)
        outs = outs + (F.l1_loss(F.instance_norm(yd1, eps=1e-5), F.instance_norm(yd2, eps=1e-5)),)
    return outs


def final_loss_grads(outs, gt, bmaps, log_para=1000.0):
    """Upstream gradients of DGTrainer's final-mode loss (trainers/dgtrainer.py:184-192:
    MSE(dc, gt*log_para) x2 + 10 BCE(c, bmap) x2 + 10 loss_con) at the given outputs,
    float64, as torch's MSELoss / binary_cross_entropy define them (+ loss_err, weight 1, when
    the outputs carry it: the has_err_loss objective)."""
    leaves = [o.detach().double().cpu().requires_grad_(True) for o in outs]
    dc1, dc2, c1, c2, lc = leaves[:5]
    g = gt.double().cpu() * log_para
    b = bmaps.double().cpu()
    loss = (F.mse_loss(dc1, g) + F.mse_loss(dc2, g)
            + 10 * (F.binary_cross_entropy(c1, b) + F.binary_cross_entropy(c2, b)) + 10 * lc)
    if len(leaves) > 5:
        loss = loss + leaves[5]
    return torch.autograd.grad(loss, leaves)
