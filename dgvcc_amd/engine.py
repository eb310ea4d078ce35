"""Static kernel plans for the DGVCC encoder/decoder (the hot path of SURVEY.md §8a).

The reference runs `vgg16_bn.features` + ConvBlock decoders through eager
PyTorch/cuDNN (models/models.py:29-96).  Here the same computation is a fixed
sequence of HIP launches over NHWC activations:

  * each Conv+BN+ReLU is `ConvLayer`: implicit-GEMM conv (bias in the epilogue),
    BN batch statistics, one fused scale/shift/ReLU(/Dropout2d) pass;
  * torch.cat of the decoder is free: producers write into channel slices of
    the concatenation buffers (`dec2in`, `dec1in`, `ycat`);
  * backward is hand-scheduled in reverse (no autograd graph inside the net),
    with gradient sums (maxpool/upsample fan-in) done by accumulating kernels.

The nn.Modules only hold parameters/buffers, so state_dict keys are identical
to the reference's.  Each plan is wrapped in one torch.autograd.Function.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import kernels as K
from .kernels import Act

ACT_NONE, ACT_RELU = 0, 1


def _bn_momentum(bn: nn.BatchNorm2d) -> float:
    if bn.momentum is None:  # cumulative moving average (torch semantics)
        return 1.0 / float(bn.num_batches_tracked.item())
    return float(bn.momentum)


class ConvLayer:
    """Conv2d(k in {1,3}, stride 1, same pad) [+ BatchNorm2d] [+ ReLU] [+ channel mask]."""

    def __init__(self, conv: nn.Conv2d, bn: nn.BatchNorm2d | None, act: int = ACT_RELU,
                 first: bool = False):
        assert conv.stride == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1
        self.conv, self.bn, self.act, self.first = conv, bn, act, first
        self.R = conv.kernel_size[0]
        self.pad = conv.padding[0]
        self.Cin, self.Cout = conv.in_channels, conv.out_channels

    def params(self):
        ps = [self.conv.weight]
        if self.conv.bias is not None:
            ps.append(self.conv.bias)
        if self.bn is not None:
            ps += [self.bn.weight, self.bn.bias]
        return ps

    def _pack(self, dt):
        w = self.conv.weight.detach()
        if self.first:  # im2col filter [Cout][64], k = (r*3+s)*3+c
            return K.pack_weight(w, dt, cpad=self.Cin, row_len=64)
        return K.pack_weight(w, dt)

    def forward(self, x: Act, out: Act, training: bool, tape: dict | None,
                drop: torch.Tensor | None = None):
        dt = x.buf.dtype
        wp = self._pack(dt)
        bias = self.conv.bias.detach() if self.conv.bias is not None else None
        z = Act(K.nhwc(x.N, x.H, x.W, self.Cout, dt, x.buf.device))
        if self.first:
            K.conv_fwd(x, wp, self.Cout, 1, 0, z, bias=bias, k_alg=9 * self.Cin)
        else:
            K.conv_fwd(x, wp, self.Cout, self.R, self.pad, z, bias=bias)
        bn = self.bn
        if bn is not None:
            if training:
                bn.num_batches_tracked.add_(1)
                stats = K.bn_fwd_train(z, bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                                       bn.running_var, _bn_momentum(bn), bn.eps)
            else:
                stats = K.bn_eval_stats(bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                                        bn.running_var, bn.eps)
        else:
            C = self.Cout
            stats = torch.zeros((4, C), dtype=torch.float32, device=x.buf.device)
            stats[1].fill_(1.0)
            stats[2].fill_(1.0)
        K.bn_apply(z, stats, self.act, out, drop)
        if tape is not None:
            tape[self] = (x, z, stats, wp, drop, training)

    def backward(self, tape: dict, g: Act, gx: Act | None, accumulate_gx: bool = False) -> dict:
        x, z, stats, wp, drop, training = tape.pop(self)
        if self.bn is not None and not training:
            raise RuntimeError("backward through an eval-mode BatchNorm is not supported")
        dev = z.buf.device
        dz = Act(torch.empty_like(z.buf))
        dgamma = torch.empty(self.Cout, dtype=torch.float32, device=dev)
        dbeta = torch.empty(self.Cout, dtype=torch.float32, device=dev)
        dbias = torch.empty(self.Cout, dtype=torch.float32, device=dev) \
            if self.conv.bias is not None else None
        gamma = self.bn.weight.detach() if self.bn is not None else None
        K.bn_bwd(g, z, gamma, stats, self.act, dz, dgamma, dbeta, dbias, drop)
        dw = torch.empty_like(self.conv.weight, dtype=torch.float32)
        if self.first:
            dwcol = torch.empty((self.Cout, 64, 1, 1), dtype=torch.float32, device=dev)
            K.conv_wgrad(x, dz, 1, 0, dwcol, k_alg=9 * self.Cin)
            K.unpack_c3_grad(dwcol, dw)
        else:
            K.conv_wgrad(x, dz, self.R, self.pad, dw)
            if gx is not None:
                K.conv_dgrad(dz, wp, self.Cin, self.R, self.pad, gx, accumulate=accumulate_gx)
        grads = {self.conv.weight: dw}
        if self.conv.bias is not None:
            grads[self.conv.bias] = dbias if self.bn is not None else dbeta
        if self.bn is not None:
            grads[self.bn.weight] = dgamma
            grads[self.bn.bias] = dbeta
        return grads


# ---------------------------------------------------------------------------
# VGG16-BN encoder (features[0:43]) + density decoder (models/models.py:35-87)
# ---------------------------------------------------------------------------
class FeaturePlan:
    """forward_fe of DGModel_base: img [N,3,H,W] f32 -> (y_cat NHWC [N,H/4,W/4,896], x3 NHWC)."""

    def __init__(self, model):
        feats = list(model.enc1) + list(model.enc2) + list(model.enc3)
        conv_idx = [i for i, m in enumerate(feats) if isinstance(m, nn.Conv2d)]
        assert conv_idx == [0, 3, 7, 10, 14, 17, 20, 24, 27, 30, 34, 37, 40], conv_idx
        self.enc = [ConvLayer(feats[i], feats[i + 1], ACT_RELU, first=(i == 0)) for i in conv_idx]
        self.dec = [ConvLayer(cb.conv, cb.bn, ACT_RELU if cb.relu is not None else ACT_NONE)
                    for d in (model.dec3, model.dec2, model.dec1) for cb in d]
        self.layers = self.enc + self.dec

    def params(self):
        return [p for l in self.layers for p in l.params()]

    def forward(self, img: torch.Tensor, dt: torch.dtype, training: bool, tape: dict | None = None):
        N, _, H, W = img.shape
        if H % 16 or W % 16:
            raise ValueError(f"input H,W must be multiples of 16 (got {H}x{W})")
        dev = img.device
        E, D = self.enc, self.dec
        nh = lambda h, w, c: Act(K.nhwc(N, h, w, c, dt, dev))  # noqa: E731
        s = {}
        col = Act(K.im2col_c3(img.float(), dt))
        a = nh(H, W, 64); E[0].forward(col, a, training, tape)
        b = nh(H, W, 64); E[1].forward(a, b, training, tape)
        p1 = nh(H // 2, W // 2, 64); K.maxpool_fwd(b, p1)
        a2 = nh(H // 2, W // 2, 128); E[2].forward(p1, a2, training, tape)
        b2 = nh(H // 2, W // 2, 128); E[3].forward(a2, b2, training, tape)
        p2 = nh(H // 4, W // 4, 128); K.maxpool_fwd(b2, p2)
        a4 = nh(H // 4, W // 4, 256); E[4].forward(p2, a4, training, tape)
        a5 = nh(H // 4, W // 4, 256); E[5].forward(a4, a5, training, tape)
        dec1in = K.nhwc(N, H // 4, W // 4, 512, dt, dev)
        x1 = Act(dec1in, 256, 256); E[6].forward(a5, x1, training, tape)
        p3 = nh(H // 8, W // 8, 256); K.maxpool_fwd(x1, p3)
        a7 = nh(H // 8, W // 8, 512); E[7].forward(p3, a7, training, tape)
        a8 = nh(H // 8, W // 8, 512); E[8].forward(a7, a8, training, tape)
        dec2in = K.nhwc(N, H // 8, W // 8, 1024, dt, dev)
        x2 = Act(dec2in, 512, 512); E[9].forward(a8, x2, training, tape)
        p4 = nh(H // 16, W // 16, 512); K.maxpool_fwd(x2, p4)
        a10 = nh(H // 16, W // 16, 512); E[10].forward(p4, a10, training, tape)
        a11 = nh(H // 16, W // 16, 512); E[11].forward(a10, a11, training, tape)
        x3 = nh(H // 16, W // 16, 512); E[12].forward(a11, x3, training, tape)
        # decoder
        a13 = nh(H // 16, W // 16, 1024); D[0].forward(x3, a13, training, tape)
        y3 = nh(H // 16, W // 16, 512); D[1].forward(a13, y3, training, tape)
        ycat = K.nhwc(N, H // 4, W // 4, 896, dt, dev)
        K.upsample_fwd(y3, 2, K.UP_BILINEAR, Act(dec2in, 0, 512))
        K.upsample_fwd(y3, 4, K.UP_BILINEAR, Act(ycat, 384, 512))
        a15 = nh(H // 8, W // 8, 512); D[2].forward(Act(dec2in), a15, training, tape)
        y2 = nh(H // 8, W // 8, 256); D[3].forward(a15, y2, training, tape)
        K.upsample_fwd(y2, 2, K.UP_BILINEAR, Act(dec1in, 0, 256))
        K.upsample_fwd(y2, 2, K.UP_BILINEAR, Act(ycat, 128, 256))
        a17 = nh(H // 4, W // 4, 256); D[4].forward(Act(dec1in), a17, training, tape)
        D[5].forward(a17, Act(ycat, 0, 128), training, tape)
        if tape is not None:
            tape[self] = dict(b=b, b2=b2, x1=x1, x2=x2, dec1in=dec1in, dec2in=dec2in,
                              shape=(N, H, W), dt=dt)
        return ycat, x3.buf

    def backward(self, tape: dict, g_ycat: torch.Tensor, g_x3: torch.Tensor | None) -> dict:
        s = tape.pop(self)
        N, H, W = s["shape"]
        dt = s["dt"]
        dev = g_ycat.device
        E, D = self.enc, self.dec
        nh = lambda h, w, c: Act(K.nhwc(N, h, w, c, dt, dev))  # noqa: E731
        g_ycat = g_ycat.contiguous()
        grads = {}
        # decoder
        g_a17 = nh(H // 4, W // 4, 256)
        grads.update(D[5].backward(tape, Act(g_ycat, 0, 128), g_a17))
        g_dec1in = K.nhwc(N, H // 4, W // 4, 512, dt, dev)
        grads.update(D[4].backward(tape, g_a17, Act(g_dec1in)))
        g_y2 = nh(H // 8, W // 8, 256)
        K.upsample_bwd(Act(g_dec1in, 0, 256), 2, K.UP_BILINEAR, g_y2, gy2=Act(g_ycat, 128, 256))
        g_a15 = nh(H // 8, W // 8, 512)
        grads.update(D[3].backward(tape, g_y2, g_a15))
        g_dec2in = K.nhwc(N, H // 8, W // 8, 1024, dt, dev)
        grads.update(D[2].backward(tape, g_a15, Act(g_dec2in)))
        g_y3 = nh(H // 16, W // 16, 512)
        K.upsample_bwd(Act(g_dec2in, 0, 512), 2, K.UP_BILINEAR, g_y3)
        K.upsample_bwd(Act(g_ycat, 384, 512), 4, K.UP_BILINEAR, g_y3, accumulate=True)
        g_a13 = nh(H // 16, W // 16, 1024)
        grads.update(D[1].backward(tape, g_y3, g_a13))
        if g_x3 is not None:
            gx3 = Act(g_x3.to(dt).contiguous().clone())
            grads.update(D[0].backward(tape, g_a13, gx3, accumulate_gx=True))
        else:
            gx3 = nh(H // 16, W // 16, 512)
            grads.update(D[0].backward(tape, g_a13, gx3))
        # enc3
        g_a11 = nh(H // 16, W // 16, 512); grads.update(E[12].backward(tape, gx3, g_a11))
        g_a10 = nh(H // 16, W // 16, 512); grads.update(E[11].backward(tape, g_a11, g_a10))
        g_p4 = nh(H // 16, W // 16, 512); grads.update(E[10].backward(tape, g_a10, g_p4))
        K.maxpool_bwd(s["x2"], g_p4, Act(g_dec2in, 512, 512), accumulate=True)
        # enc2
        g_a8 = nh(H // 8, W // 8, 512); grads.update(E[9].backward(tape, Act(g_dec2in, 512, 512), g_a8))
        g_a7 = nh(H // 8, W // 8, 512); grads.update(E[8].backward(tape, g_a8, g_a7))
        g_p3 = nh(H // 8, W // 8, 256); grads.update(E[7].backward(tape, g_a7, g_p3))
        K.maxpool_bwd(s["x1"], g_p3, Act(g_dec1in, 256, 256), accumulate=True)
        # enc1
        g_a5 = nh(H // 4, W // 4, 256); grads.update(E[6].backward(tape, Act(g_dec1in, 256, 256), g_a5))
        g_a4 = nh(H // 4, W // 4, 256); grads.update(E[5].backward(tape, g_a5, g_a4))
        g_p2 = nh(H // 4, W // 4, 128); grads.update(E[4].backward(tape, g_a4, g_p2))
        g_b2 = nh(H // 2, W // 2, 128); K.maxpool_bwd(s["b2"], g_p2, g_b2)
        g_a2 = nh(H // 2, W // 2, 128); grads.update(E[3].backward(tape, g_b2, g_a2))
        g_p1 = nh(H // 2, W // 2, 64); grads.update(E[2].backward(tape, g_a2, g_p1))
        g_b = nh(H, W, 64); K.maxpool_bwd(s["b"], g_p1, g_b)
        g_a = nh(H, W, 64); grads.update(E[1].backward(tape, g_b, g_a))
        grads.update(E[0].backward(tape, g_a, None))
        return (), grads


class _PlanFn(torch.autograd.Function):
    """Bridges a plan's hand-scheduled backward into torch autograd.

    apply(plan, fwd, n_in, *inputs, *params): `fwd(*inputs, tape=...)` runs the
    forward launches; `plan.backward(tape, *grad_outputs)` returns
    (grads for the inputs, {param: grad}).  Params are Function arguments so
    autograd routes their gradients to `.grad` (AccumulateGrad)."""

    @staticmethod
    def forward(ctx, plan, fwd, n_in, *tensors):
        ctx.plan = plan
        ctx.n_in = n_in
        ctx.params = tensors[n_in:]
        ctx.tape = {}
        outs = fwd(*tensors[:n_in], tape=ctx.tape)
        return outs

    @staticmethod
    def backward(ctx, *gouts):
        gin, grads = ctx.plan.backward(ctx.tape, *gouts)
        gin = list(gin) + [None] * (ctx.n_in - len(gin))
        out = [grads.get(p) for p in ctx.params]
        ctx.plan = ctx.tape = None
        return (None, None, None, *gin, *out)


def run_plan(plan, fwd, inputs, params):
    """Run `fwd(*inputs, tape=...)` under autograd when gradients are needed."""
    need = torch.is_grad_enabled() and (any(p.requires_grad for p in params) or
                                        any(isinstance(t, torch.Tensor) and t.requires_grad
                                            for t in inputs))
    if need:
        return _PlanFn.apply(plan, fwd, len(inputs), *inputs, *params)
    with torch.no_grad():
        return fwd(*inputs, tape=None)


# ---------------------------------------------------------------------------
# density head of DGModel_base: den_dec (1x1 896->256 +BN+ReLU+Dropout2d),
# den_head (1x1 256->1 + ReLU), bilinear x4 (models/models.py:55-62, 89-96)
# ---------------------------------------------------------------------------
def dropout2d_mask(N: int, C: int, p: float, device) -> torch.Tensor | None:
    """Per-(sample, channel) keep mask scaled by 1/(1-p), as F.dropout2d (torch RNG)."""
    if p <= 0.0:
        return None
    if p >= 1.0:
        return torch.zeros((N, C), dtype=torch.float32, device=device)
    return torch.empty((N, C), dtype=torch.float32, device=device).bernoulli_(1.0 - p).div_(1.0 - p)


class DensityPlan:
    """ycat NHWC [N,h,w,896] -> d [N,1,4h,4w] f32."""

    def __init__(self, den_dec_block, den_head_block, dropout_p: float = 0.0):
        self.dec = ConvLayer(den_dec_block.conv, den_dec_block.bn, ACT_RELU)
        hc = den_head_block.conv
        self.head_w = hc.weight
        self.head_b = hc.bias
        self.head_act = K.ACT_RELU if den_head_block.relu is not None else K.ACT_NONE
        self.p = dropout_p

    def params(self):
        ps = self.dec.params() + [self.head_w]
        if self.head_b is not None:
            ps.append(self.head_b)
        return ps

    def forward(self, ycat: torch.Tensor, training: bool, tape: dict | None = None):
        N, h, w, C = ycat.shape
        dt = ycat.dtype
        dev = ycat.device
        drop = dropout2d_mask(N, self.dec.Cout, self.p, dev) if training else None
        yden = Act(K.nhwc(N, h, w, self.dec.Cout, dt, dev))
        self.dec.forward(Act(ycat), yden, training, tape, drop=drop)
        hb = self.head_b.detach() if self.head_b is not None else None
        yh = K.head_fwd(yden, self.head_w.detach().reshape(-1), hb, self.head_act)
        d = torch.empty((N, 4 * h, 4 * w, 1), dtype=torch.float32, device=dev)
        K.upsample_fwd(Act(yh.view(N, h, w, 1)), 4, K.UP_BILINEAR, Act(d))
        if tape is not None:
            tape[self] = (ycat.shape, dt, yden, yh)
        return d.view(N, 1, 4 * h, 4 * w)

    def backward(self, tape: dict, g_d: torch.Tensor):
        shape, dt, yden, yh = tape.pop(self)
        N, h, w, C = shape
        dev = g_d.device
        g_h = torch.empty((N, h, w, 1), dtype=torch.float32, device=dev)
        K.upsample_bwd(Act(g_d.contiguous().view(N, 4 * h, 4 * w, 1)), 4, K.UP_BILINEAR, Act(g_h))
        g_yden = Act(torch.empty_like(yden.buf))
        gw = torch.empty(self.dec.Cout, dtype=torch.float32, device=dev)
        gb = torch.empty(1, dtype=torch.float32, device=dev) if self.head_b is not None else None
        K.head_bwd(yden, self.head_w.detach().reshape(-1), self.head_act, yh, g_h.view(N, h, w),
                   g_yden, gw, gb)
        g_ycat = torch.empty(shape, dtype=dt, device=dev)
        grads = self.dec.backward(tape, g_yden, Act(g_ycat))
        grads[self.head_w] = gw.view_as(self.head_w)
        if gb is not None:
            grads[self.head_b] = gb
        return (g_ycat,), grads
