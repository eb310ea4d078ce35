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

import os

import torch
import torch.nn as nn

from . import kernels as K
from . import syncbn as SB
from .kernels import Act

# The memory readout y_new = mem P feeds only the 1x1 density head, so the head folds through it:
# d = act((mem^T w) . P + b), fused into the slot-softmax pass (dg_softmax_head_*; memread.hip).
# DGVCC_MEM_HEAD=0 restores the materialised readout GEMMs (A/B and cross-check).
MEM_HEAD_FUSED = os.environ.get("DGVCC_MEM_HEAD", "1") != "0"

ACT_NONE, ACT_RELU = 0, 1


_FROZEN_GEN = [0]
_EVAL_FUSE = __import__("os").environ.get("DGVCC_EVAL_FUSE", "1") != "0"
_STEM_RECOMP = __import__("os").environ.get("DGVCC_STEM_RECOMP", "1") != "0"
# fp32 first layer straight from the image (dg_stem_fwd_f32); 0 = im2col + GEMM + statistics pass
_STEM_F32 = __import__("os").environ.get("DGVCC_STEM_F32", "1") != "0"
# its backward: dz and the wgrad on f32 MFMA in one pass (dg_stem_bwd_f32); 0 = BN backward + im2col wgrad
_STEM_BWD_F32 = __import__("os").environ.get("DGVCC_STEM_BWD_F32", "1") != "0"
# fp32 training: the BN apply of a layer whose output feeds a 3x3 / 1x1 conv forward writes that
# conv's f16 x3 pair image too (dg_bn_apply_pair; DGVCC_BN_PAIR=0: the conv splits x itself)
_BN_PAIR = __import__("os").environ.get("DGVCC_BN_PAIR", "1") != "0"


def invalidate_frozen():
    """Weights may have changed behind torch's back (a train()/eval() switch, a fused
    optimizer step writing the flat parameter buffer through a raw pointer)."""
    _FROZEN_GEN[0] += 1


def frozen(owner, name, srcs, build):
    """Eval-mode memo of a weight-derived tensor (packed filters, BN scale/shift): rebuilt
    when a source tensor is replaced or modified in place, or after invalidate_frozen().
    Saves the per-frame repacking and the per-layer running-stat math of evaluation."""
    key = (_FROZEN_GEN[0],) + tuple((t.data_ptr(), t._version) for t in srcs)
    memo = owner.__dict__.setdefault("_frozen", {})
    ent = memo.get(name)
    if ent is None or ent[0] != key:
        ent = (key, build())
        memo[name] = ent
    return ent[1]


# training steps pack each filter and its dgrad flip in one launch (dg_pack_weight_flip); 0: two launches
_PACK_FLIP = os.environ.get("DGVCC_PACK_FLIP", "1") != "0"


def pack_flip(owner, w_param: torch.Tensor, dt) -> torch.Tensor:
    """Packed filter of w_param; its flip is kept beside it for the dgrad (flip_of)."""
    wp, wf = K.pack_weight_flip(w_param.detach(), dt)
    # the last two (several forwards of one step -- the views -- each pack; the tape holds each one's wp)
    owner.__dict__["_packflip"] = [(wp, wp._version, wf)] + owner.__dict__.get("_packflip", [])[:1]
    return wp


def flip_of(owner, w_param: torch.Tensor, wp: torch.Tensor, cout: int, cin: int, r: int) -> torch.Tensor:
    """The dgrad's flipped filter of the packed filter wp: the one pack_flip built with wp (a function of
    wp alone, so no generation check: a later forward's invalidate_frozen() must not discard it while
    the tape still holds wp), else flip_weight once per packed filter (frozen)."""
    for pw, ver, wf in owner.__dict__.get("_packflip", ()):
        if pw is wp and ver == wp._version:
            return wf
    return frozen(owner, ("flip", wp.dtype), (w_param, wp), lambda: K.flip_weight(wp, cout, cin, r))


def bn_eval_cached(owner, bn: nn.BatchNorm2d) -> torch.Tensor:
    return frozen(owner, "bn_eval", (bn.weight, bn.bias, bn.running_mean, bn.running_var),
                  lambda: K.bn_eval_stats(bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                                          bn.running_var, bn.eps))


def _bn_momentum(bn: nn.BatchNorm2d) -> float:
    if bn.momentum is None:  # cumulative moving average (torch semantics)
        SB.flush_batches()
        return 1.0 / float(bn.num_batches_tracked.item())
    return float(bn.momentum)


def _ident_stats(C, dev):
    st = torch.zeros((4, C), dtype=torch.float32, device=dev)
    st[1].fill_(1.0)
    st[2].fill_(1.0)
    return st


class ConvLayer:
    """Conv2d(k in {1,3}, stride 1, same pad) [+ BatchNorm2d] [+ ReLU] [+ channel mask]."""

    def __init__(self, conv: nn.Conv2d, bn: nn.BatchNorm2d | None, act: int = ACT_RELU,
                 first: bool = False):
        assert conv.stride == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1
        self.conv, self.bn, self.act, self.first = conv, bn, act, first
        self.scope = "head"  # FeaturePlan relabels its encoder / decoder layers (bench timing)
        self.R = conv.kernel_size[0]
        self.pad = conv.padding[0]
        self.Cin, self.Cout = conv.in_channels, conv.out_channels
        # the output (pooled output when pooling) is the input of a conv forward (FeaturePlan sets it):
        # the fp32 training BN apply then writes that conv's pair image (_BN_PAIR)
        self.pair_out = False

    def params(self):
        ps = [self.conv.weight]
        if self.conv.bias is not None:
            ps.append(self.conv.bias)
        if self.bn is not None:
            ps += [self.bn.weight, self.bn.bias]
        return ps

    def _pack(self, dt, training=False):
        w = self.conv.weight.detach()
        if self.first:  # im2col filter [Cout][64], k = (r*3+s)*3+c
            return K.pack_weight(w, dt, cpad=self.Cin, row_len=64)
        if training and _PACK_FLIP:  # the dgrad's flipped filter from the same launch
            return pack_flip(self, self.conv.weight, dt)
        return K.pack_weight(w, dt)

    def _flip(self, wp):
        """flip_weight(wp) for the dgrad, once per packed filter (both views of a step)."""
        return flip_of(self, self.conv.weight, wp, self.Cout, self.Cin, self.R)

    def stem_ok(self, dt) -> bool:
        """bf16 first layer with BN + ReLU: fused conv/statistics and BN-backward/wgrad kernels;
        fp32: conv + BN statistics from the image (the backward re-forms the im2col for its wgrad)."""
        ok_dt = dt == torch.bfloat16 or (dt == torch.float32 and _STEM_F32)
        return (self.first and ok_dt and self.bn is not None and self.act == ACT_RELU
                and self.Cin == 3 and self.Cout == 64 and self.R == 3)

    @staticmethod
    def stem_shape_ok(W: int) -> bool:  # row segments of 64 pixels (dg_stem_fwd)
        return W % 64 == 0

    def forward(self, x, out: Act | None, training: bool, tape: dict | None,
                drop: torch.Tensor | None = None, pool: Act | None = None):
        """x: NHWC Act, or for the fused bf16 stem the NCHW f32 image itself.
        pool: also apply the following MaxPool2d(2,2) into `pool` (BN/ReLU/pool in one pass);
        `out` (the un-pooled activation) may then be None when nothing else reads it."""
        K.set_scope(self.scope)
        stem = isinstance(x, torch.Tensor)
        dt = (out if out is not None else pool).buf.dtype
        # host-side shape guard: the kernels size their grids from x and write `out` blindly
        xs = (x.shape[0], x.shape[2], x.shape[3]) if stem else (x.N, x.H, x.W)
        if out is not None and ((out.N, out.H, out.W) != xs or out.C != self.Cout):
            raise ValueError(f"ConvLayer: output {(out.N, out.H, out.W, out.C)} != input {xs} x Cout {self.Cout}")
        if pool is not None and ((pool.N, pool.H * 2, pool.W * 2) != xs or pool.C != self.Cout):
            raise ValueError("ConvLayer: pooled output shape mismatch")
        bias = self.conv.bias.detach() if self.conv.bias is not None else None
        bn = self.bn
        # nn.SyncBatchNorm under a multi-rank process group: global batch statistics (syncbn.py)
        pg = SB.group_of(bn) if training else None
        if stem and dt == torch.float32:
            wk = (K.stem_weight_f32(self.conv.weight) if training else
                  frozen(self, ("stem32", dt), (self.conv.weight,), lambda: K.stem_weight_f32(self.conv.weight)))
            z = Act(K.nhwc(x.shape[0], x.shape[2], x.shape[3], self.Cout, dt, x.device))
            part, nblk = K.stem_fwd_f32(x, wk, bias, z)
            if pg is not None:
                stats = SB.fwd_stats(bn, pg, part=part, nblk=nblk, M=z.M)
            elif training:
                SB.bump_batches(bn)
                stats = K.bn_part_finalize(part, nblk, self.Cout, bn.weight.detach(), bn.bias.detach(),
                                           bn.running_mean, bn.running_var, _bn_momentum(bn), bn.eps)
            else:
                stats = bn_eval_cached(self, bn)
            self._apply(z, stats, out, drop, pool)
            if tape is not None:
                tape[self] = (x, z, stats, None, drop, training)
            return
        if stem:
            N, _, H, W = x.shape
            build = lambda: K.pack_weight(self.conv.weight.detach(), dt, cpad=3, row_len=32)  # noqa: E731
            wp = build() if training else frozen(self, ("stem", dt), (self.conv.weight,), build)
            if _STEM_RECOMP and pool is None and drop is None and out is not None and pg is None:
                # z-free stem: statistics pass, then conv recomputed with BN+ReLU applied; the
                # backward recomputes z again (27 MACs per output vs 128 B/px per HBM pass)
                if training:
                    part, nblk = K.stem_stats(x, wp, bias)
                    SB.bump_batches(bn)
                    stats = K.bn_part_finalize(part, nblk, self.Cout, bn.weight.detach(), bn.bias.detach(),
                                               bn.running_mean, bn.running_var, _bn_momentum(bn), bn.eps)
                else:
                    stats = bn_eval_cached(self, bn)
                K.stem_apply(x, wp, bias, stats, out)
                if tape is not None:
                    tape[self] = (x, None, stats, wp, drop, training)
                return
            z = Act(K.nhwc(N, H, W, self.Cout, dt, x.device))
            part, nblk = K.stem_fwd(x, wp, bias, z)
            if pg is not None:
                stats = SB.fwd_stats(bn, pg, part=part, nblk=nblk, M=z.M)
            elif training:
                SB.bump_batches(bn)
                stats = K.bn_part_finalize(part, nblk, self.Cout, bn.weight.detach(), bn.bias.detach(),
                                           bn.running_mean, bn.running_var, _bn_momentum(bn), bn.eps)
            else:
                stats = bn_eval_cached(self, bn)
            self._apply(z, stats, out, drop, pool)
            if tape is not None:
                tape[self] = (x, z, stats, wp, drop, training)
            return
        # packed once per weight version: in training the two views of a step share it (run_plan
        # starts each autograd forward on a fresh generation)
        wp = frozen(self, ("w", dt), (self.conv.weight,), lambda: self._pack(dt, training))
        if (_EVAL_FUSE and not training and bn is not None and pool is None and drop is None
                and out is not None and not self.first and tape is None):
            # evaluation: BN from the running statistics (+ReLU) in the conv epilogue, no z pass
            K.conv_fwd_bn_eval(x, wp, self.Cout, self.R, self.pad, out, bias, bn_eval_cached(self, bn), self.act)
            return
        z = Act(K.nhwc(x.N, x.H, x.W, self.Cout, dt, x.buf.device))
        epi = None
        if self.first:
            K.conv_fwd(x, wp, self.Cout, 1, 0, z, bias=bias, k_alg=9 * self.Cin)
        elif bn is not None and training:  # BN statistics from the conv epilogue where available
            epi = K.conv_fwd_stats(x, wp, self.Cout, self.R, self.pad, z, bias=bias)
            if epi is None:
                K.conv_fwd(x, wp, self.Cout, self.R, self.pad, z, bias=bias)
        else:
            K.conv_fwd(x, wp, self.Cout, self.R, self.pad, z, bias=bias)
        x.pair = None  # consumed (the image is not kept with the tape)
        if epi is not None and pg is not None:
            stats = SB.fwd_stats(bn, pg, part=epi[0], nblk=epi[1], M=z.M)
        elif epi is not None:
            SB.bump_batches(bn)
            stats = K.bn_part_finalize(epi[0], epi[1], self.Cout, bn.weight.detach(), bn.bias.detach(),
                                       bn.running_mean, bn.running_var, _bn_momentum(bn), bn.eps)
        elif pg is not None:
            stats = SB.fwd_stats(bn, pg, z=z)
        elif bn is not None:
            if training:
                SB.bump_batches(bn)
                stats = K.bn_fwd_train(z, bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                                       bn.running_var, _bn_momentum(bn), bn.eps)
            else:
                stats = bn_eval_cached(self, bn)
        else:
            stats = frozen(self, ("ident", x.buf.device), (), lambda: _ident_stats(self.Cout, x.buf.device))
        pair = _BN_PAIR and self.pair_out and training and bn is not None and pg is None
        self._apply(z, stats, out, drop, pool, pair)
        if tape is not None:
            tape[self] = (x, z, stats, wp, drop, training)

    def _dz_pair(self, gx) -> bool:
        """fp32 BN backward writes dz's pair image for the dgrad (_BN_PAIR): where a dgrad follows and
        takes the pre-split forward (its output, this layer's input, has >= 128 channels)."""
        return _BN_PAIR and gx is not None and not self.first and self.Cin >= 128

    def _apply(self, z: Act, stats, out: Act | None, drop, pool: Act | None, pair: bool = False):
        if pool is not None:
            K.bn_apply_pool(z, stats, self.act, out, pool, drop, pair=pair)
        else:
            K.bn_apply(z, stats, self.act, out, drop, pair=pair)

    def backward(self, tape: dict, g: Act | None, gx: Act | None, accumulate_gx: bool = False,
                 g_pool: Act | None = None, gx_bn: "ConvLayer | None" = None) -> dict:
        """g: gradient of the layer output (None if only the pooled output was used);
        g_pool: gradient of the pooled output when the forward ran with `pool`;
        gx_bn: the layer whose whole output gradient gx is (its BN-backward partial sums
        then come from this layer's dgrad epilogue)."""
        K.set_scope(self.scope)
        x, z, stats, wp, drop, training = tape.pop(self)
        pre = tape.pop(("bnpart", self), None)
        if self.bn is not None and not training:
            raise RuntimeError("backward through an eval-mode BatchNorm is not supported")
        dev = stats.device
        dz = Act(torch.empty_like(z.buf)) if z is not None else None
        dgamma = torch.empty(self.Cout, dtype=torch.float32, device=dev)
        dbeta = torch.empty(self.Cout, dtype=torch.float32, device=dev)
        dbias = torch.empty(self.Cout, dtype=torch.float32, device=dev) \
            if self.conv.bias is not None else None
        gamma = self.bn.weight.detach() if self.bn is not None else None
        pg = SB.group_of(self.bn)
        if isinstance(x, torch.Tensor) and z is not None and z.buf.dtype == torch.float32:
            if (_STEM_BWD_F32 and pg is None and drop is None and g is not None and g_pool is None
                    and pre is None and x.shape[3] % 32 == 0):
                # fp32 stem: BN-backward coefficients, then dz and the conv1_1 wgrad in one pass
                coef = K.bn_bwd_coef(g, z, gamma, stats, self.act, dgamma, dbeta, dbias, drop)
                dw = torch.empty_like(self.conv.weight, dtype=torch.float32)
                K.stem_bwd_f32(x, g, z, stats, coef, dw)
                grads = {self.conv.weight: dw, self.bn.weight: dgamma, self.bn.bias: dbeta}
                if self.conv.bias is not None:
                    grads[self.conv.bias] = dbias
                return grads
            x = Act(K.im2col_c3(x, torch.float32))  # the generic BN backward + im2col wgrad
        if isinstance(x, torch.Tensor):  # fused bf16 stem: coefficients, then BN-backward + wgrad in one pass
            dw = torch.empty_like(self.conv.weight, dtype=torch.float32)
            bias = self.conv.bias.detach() if self.conv.bias is not None else None
            if z is None:  # z-free stem: z recomputed from the image in both passes
                coef = K.stem_bwd_coef(x, wp, bias, g, gamma, stats, dgamma, dbeta, dbias)
                K.stem_bwd(x, g, None, stats, coef, dw, wp=wp, bias=bias)
            else:
                if pg is not None:
                    coef = SB.backward(self.bn, pg, g, z, stats, self.act, None, dgamma, dbeta, dbias, drop=drop)
                else:
                    coef = K.bn_bwd_coef(g, z, gamma, stats, self.act, dgamma, dbeta, dbias, drop)
                K.stem_bwd(x, g, z, stats, coef, dw)
            grads = {self.conv.weight: dw, self.bn.weight: dgamma, self.bn.bias: dbeta}
            if self.conv.bias is not None:
                grads[self.conv.bias] = dbias
            return grads
        if pg is not None:
            SB.backward(self.bn, pg, g, z, stats, self.act, dz, dgamma, dbeta, dbias, drop=drop, g_pool=g_pool,
                        part=pre[0] if pre is not None else None, nblk=pre[1] if pre is not None else 0)
        elif g_pool is not None:
            if self.bn is None:
                raise RuntimeError("pooled backward needs a BatchNorm layer")
            # fp32: the dgrad that follows reads dz's pair image (_BN_PAIR)
            K.bn_bwd_pool(g_pool, g, z, gamma, stats, self.act, dz, dgamma, dbeta, dbias, drop,
                          pair=self._dz_pair(gx))
        elif pre is not None:
            K.bn_bwd_from_part(pre, g, z, gamma, stats, self.act, dz, dgamma, dbeta, dbias, drop)
        else:
            K.bn_bwd(g, z, gamma, stats if self.bn is not None else None, self.act, dz, dgamma, dbeta,
                     dbias, drop, pair=self._dz_pair(gx) and self.bn is not None)
        dw = torch.empty_like(self.conv.weight, dtype=torch.float32)
        if self.first:
            dwcol = torch.empty((self.Cout, 64, 1, 1), dtype=torch.float32, device=dev)
            K.conv_wgrad(x, dz, 1, 0, dwcol, k_alg=9 * self.Cin)
            K.unpack_c3_grad(dwcol, dw)
        else:
            K.conv_wgrad(x, dz, self.R, self.pad, dw)
            if gx is not None:
                res = None
                if gx_bn is not None and not accumulate_gx and gx_bn.bn is not None:
                    xn, zn, stn, _, dropn, trn = tape[gx_bn]
                    if trn and not isinstance(xn, torch.Tensor) and zn.C == gx.C:
                        res = K.conv_dgrad_bnpart(dz, wp, self.Cin, self.R, self.pad, gx, zn, stn, gx_bn.act,
                                                  dropn, wflip=self._flip(wp))
                        if res is not None:
                            tape[("bnpart", gx_bn)] = res
                if res is None:
                    K.conv_dgrad(dz, wp, self.Cin, self.R, self.pad, gx, accumulate=accumulate_gx,
                                 wflip=self._flip(wp))
        if dz is not None:
            dz.pair = None
        grads = {self.conv.weight: dw}
        if self.conv.bias is not None:
            grads[self.conv.bias] = dbias if self.bn is not None else dbeta
        if self.bn is not None:
            grads[self.bn.weight] = dgamma
            grads[self.bn.bias] = dbeta
        return grads


class CatParts:
    """The decoder concatenation y_cat = cat[y1, up2(y2), up4(y3)] (models/models.py:84) kept
    as its parts (NHWC Acts at their own resolutions) instead of a materialised
    [N, H/4, W/4, 896] tensor."""
    SCALES = (1, 2, 4)

    def __init__(self, y1: Act, y2: Act, y3: Act):
        self.parts = (y1, y2, y3)
        for p, sc in zip(self.parts, self.SCALES):
            if (p.H * sc, p.W * sc) != (y1.H, y1.W):
                raise ValueError("CatParts: part resolutions must be y1, y1/2, y1/4")

    @property
    def N(self):
        return self.parts[0].N

    @property
    def H(self):
        return self.parts[0].H

    @property
    def W(self):
        return self.parts[0].W

    @property
    def C(self):
        return sum(p.C for p in self.parts)

    def empty_like(self) -> "CatParts":
        return CatParts(*(Act(torch.empty(p.N, p.H, p.W, p.C, dtype=p.buf.dtype, device=p.buf.device))
                          for p in self.parts))

    def tensors(self):
        return tuple(p.buf for p in self.parts)


def as_cat(x):
    """A head plan's concatenation input: a (y1, y2, y3) tuple of NHWC tensors -> CatParts,
    or a materialised NHWC y_cat tensor -> Act."""
    if isinstance(x, (tuple, list)):
        return CatParts(*(K.import_act(t) for t in x))
    return K.import_act(x)


def cat_empty_like(cat):
    return cat.empty_like() if isinstance(cat, CatParts) else Act(torch.empty_like(cat.buf))


def cat_grads(gcat) -> tuple:
    return gcat.tensors() if isinstance(gcat, CatParts) else (gcat.buf,)


class CatConvLayer(ConvLayer):
    """den_dec (1x1 Conv + BN + ReLU [+ Dropout2d], models/models.py:55-58) applied to the decoder
    concatenation.  On CatParts the 1x1 conv runs on each part at the part's own resolution
    and the bilinear upsampling moves behind it (both are linear):
        W . cat[y1, up2(y2), up4(y3)] = W1 y1 + up2(W2 y2) + up4(W3 y3),
    so neither y_cat (896 channels at H/4 x W/4) nor its gradient is ever materialised and the
    conv FLOPs drop 4x.  One pass (dg_cat_combine) sums the parts and emits the BN partials;
    the backward downsamples dz once per part (U^T) and runs the per-part dgrad/wgrad."""

    def forward(self, x, out, training, tape, drop=None, pool=None):
        if not isinstance(x, CatParts):
            return super().forward(x, out, training, tape, drop=drop, pool=pool)
        if self.R != 1 or pool is not None or x.C != self.Cin:
            raise ValueError("CatConvLayer: decomposed path needs an unpooled 1x1 conv")
        dt = out.buf.dtype
        dev = out.buf.device
        w = self.conv.weight.detach()
        zs, wps, lo = [], [], 0
        for part in x.parts:
            if dt == torch.float32 and training and part.amax is None:
                part.amax = K.amax(part)  # once for the forward and the backward's wgrad (f16 x3 scales)
            build = lambda lo=lo, c=part.C: K.pack_weight(w[:, lo:lo + c].contiguous(), dt)  # noqa: E731
            wp = build() if training else frozen(self, ("cat", dt, lo), (self.conv.weight,), build)
            zk = Act(K.nhwc(part.N, part.H, part.W, self.Cout, dt, dev))
            K.conv_fwd(part, wp, self.Cout, 1, 0, zk)
            zs.append(zk)
            wps.append(wp)
            lo += part.C
        z = zs[0]
        bias = self.conv.bias.detach() if self.conv.bias is not None else None
        rows = K.query("dg_cat_combine_part_rows", z.N, z.H, z.W)
        part = torch.empty((rows, 3, self.Cout), dtype=torch.float32, device=dev)
        K.call("dg_cat_combine", z.dt, z.ptr, z.ld, zs[1].ptr, zs[1].ld, zs[2].ptr, zs[2].ld, z.N, z.H, z.W,
               self.Cout, K.ptr(bias), z.ptr, z.ld, K.ptr(part), K.stream())
        bn = self.bn
        pg = SB.group_of(bn) if training else None
        if bn is None:  # models2 den_dec: ConvBlock without BatchNorm (bias-free conv + ReLU)
            stats = frozen(self, ("ident", dev), (), lambda: _ident_stats(self.Cout, dev))
        elif pg is not None:
            stats = SB.fwd_stats(bn, pg, part=part, nblk=rows, M=z.M)
        elif training:
            SB.bump_batches(bn)
            stats = K.bn_part_finalize(part, rows, self.Cout, bn.weight.detach(), bn.bias.detach(),
                                       bn.running_mean, bn.running_var, _bn_momentum(bn), bn.eps)
        else:
            stats = bn_eval_cached(self, bn)
        K.bn_apply(z, stats, self.act, out, drop,
                   pair=_BN_PAIR and self.pair_out and training and bn is not None and pg is None)
        if tape is not None:
            tape[self] = (x, z, stats, wps, drop, training)

    def backward(self, tape, g, gx, accumulate_gx=False, g_pool=None):
        if not isinstance(tape[self][0], CatParts):
            return super().backward(tape, g, gx, accumulate_gx=accumulate_gx, g_pool=g_pool)
        x, z, stats, wps, drop, training = tape.pop(self)
        if not training and self.bn is not None:
            raise RuntimeError("backward through an eval-mode BatchNorm is not supported")
        dev = z.buf.device
        dz = Act(torch.empty_like(z.buf))
        dgamma = torch.empty(self.Cout, dtype=torch.float32, device=dev)
        dbeta = torch.empty(self.Cout, dtype=torch.float32, device=dev)
        dbias = torch.empty(self.Cout, dtype=torch.float32, device=dev) \
            if (self.conv.bias is not None and self.bn is not None) else None
        gamma = self.bn.weight.detach() if self.bn is not None else None
        pg = SB.group_of(self.bn)
        if pg is not None:
            SB.backward(self.bn, pg, g, z, stats, self.act, dz, dgamma, dbeta, dbias, drop=drop)
        else:
            K.bn_bwd(g, z, gamma, stats if self.bn is not None else None, self.act, dz, dgamma, dbeta, dbias, drop,
                     pair=self._dz_pair(gx) and self.bn is not None)  # read by part 0's dgrad
        gzs = [dz]
        for part, sc in zip(x.parts[1:], CatParts.SCALES[1:]):  # U^T dz at the part's resolution
            gk = Act(K.nhwc(part.N, part.H, part.W, self.Cout, dz.buf.dtype, dev))
            K.upsample_bwd(dz, sc, K.UP_BILINEAR, gk)
            if gk.buf.dtype == torch.float32:
                gk.amax = K.amax(gk)  # once for the wgrad and the dgrad below
            gzs.append(gk)
        dw = torch.empty_like(self.conv.weight, dtype=torch.float32)
        lo = 0
        for k, part in enumerate(x.parts):
            dwk = torch.empty((self.Cout, part.C, 1, 1), dtype=torch.float32, device=dev)
            K.conv_wgrad(part, gzs[k], 1, 0, dwk)
            dw[:, lo:lo + part.C] = dwk
            if gx is not None:
                K.conv_dgrad(gzs[k], wps[k], part.C, 1, 0, gx.parts[k], accumulate=accumulate_gx)
            lo += part.C
        dz.pair = None
        grads = {self.conv.weight: dw}
        if self.bn is not None:
            grads.update({self.bn.weight: dgamma, self.bn.bias: dbeta})
        if self.conv.bias is not None:
            grads[self.conv.bias] = dbias if self.bn is not None else dbeta
        return grads


# ---------------------------------------------------------------------------
# VGG16-BN encoder (features[0:43]) + density decoder (models/models.py:35-87)
# ---------------------------------------------------------------------------
_FEATURE_PLANS = __import__("weakref").WeakSet()


def feature_plans_of(params) -> list:
    """The live FeaturePlans whose parameters are all in `params` (an optimizer's group)."""
    ps = set(params)
    return [plan for plan in list(_FEATURE_PLANS) if all(p in ps for p in plan.params())]


def _cat_act(buf: torch.Tensor, up_src: Act, skip: Act) -> Act:
    """The decoder concatenation [up2(up_src) | skip] as one Act; its amax (the f32 convs' operand
    scale) bounds both parts: bilinear upsampling does not exceed its source's max |.|."""
    a = Act(buf)
    if up_src.amax is not None and skip.amax is not None:
        cu, cs = up_src.C, skip.C
        if up_src.amax.numel() >= 1 + cu and skip.amax.numel() >= 1 + cs:  # per channel
            pad = K.amax_words(cu + cs) - (1 + cu + cs)
            a.amax = torch.cat([torch.maximum(up_src.amax[:1], skip.amax[:1]), up_src.amax[1:1 + cu],
                                skip.amax[1:1 + cs], up_src.amax.new_zeros(pad)])
        else:
            a.amax = torch.maximum(up_src.amax[:1], skip.amax[:1])
    return a


class FeaturePlan:
    """forward_fe of DGModel_base: img [N,3,H,W] f32 -> (y1, y2, y3, x3) NHWC, where the
    reference's y_cat = cat[y1, up2(y2), up4(y3)] (models/models.py:84) is left to the heads'
    CatConvLayer (never materialised on the hot path)."""

    def __init__(self, model, inorm: bool = False):
        # inorm: F.instance_norm (affine-free) on every stage output x1, x2, x3 before the next
        # stage and the decoder read it (models2.DensityRegressor, models/models2.py:149-155)
        self.inorm = inorm
        # DGModel_* name the VGG16-BN stages enc1/2/3, models2's DensityRegressor* stage1/2/3
        names = getattr(model, "_ENC_NAMES", ("enc1", "enc2", "enc3"))
        feats = [m for n in names for m in getattr(model, n)]
        conv_idx = [i for i, m in enumerate(feats) if isinstance(m, nn.Conv2d)]
        assert conv_idx == [0, 3, 7, 10, 14, 17, 20, 24, 27, 30, 34, 37, 40], conv_idx
        self.enc = [ConvLayer(feats[i], feats[i + 1], ACT_RELU, first=(i == 0)) for i in conv_idx]
        self.dec = [ConvLayer(cb.conv, cb.bn, ACT_RELU if cb.relu is not None else ACT_NONE)
                    for d in (model.dec3, model.dec2, model.dec1) for cb in d]
        self.layers = self.enc + self.dec
        self.sink = None
        _FEATURE_PLANS.add(self)
        for l in self.enc:
            l.scope = "enc"
        for l in self.dec:
            l.scope = "dec"
        # outputs read next by a conv forward (the pooled ones for E[1], E[3], E[6], E[9]); not the stem
        # output (its consumer is the Cout = 64 3-tap kernel), nor y3 / y2 / y1 (upsampled / heads)
        # (with inorm the stage outputs E[6], E[9], E[12] go to the InstanceNorm instead)
        for i in (1, 2, 3, 4, 5, 7, 8, 10, 11) + (() if inorm else (6, 9, 12)):
            self.enc[i].pair_out = True
        for i in (0, 2, 4):
            self.dec[i].pair_out = True

    def params(self):
        return [p for l in self.layers for p in l.params()]

    def forward(self, img: torch.Tensor, dt: torch.dtype, training: bool, tape: dict | None = None):
        N, _, H, W = img.shape
        if H % 16 or W % 16:
            raise ValueError(f"input H,W must be multiples of 16 (got {H}x{W})")
        # data-parallel gradient sink (dgvcc_amd.dist.OverlapReducer, attached by the optimizer):
        # the backward hands each layer's parameter gradients to it as soon as they exist
        if tape is not None and self.sink is not None and self.sink.active:
            self.sink.forward_seen()
        dev = img.device
        E, D = self.enc, self.dec
        nh = lambda h, w, c: Act(K.nhwc(N, h, w, c, dt, dev))  # noqa: E731
        s = {}
        a = nh(H, W, 64)
        if E[0].stem_ok(dt) and ConvLayer.stem_shape_ok(W):
            E[0].forward(img.float().contiguous(), a, training, tape)
        else:
            E[0].forward(Act(K.im2col_c3(img.float(), dt)), a, training, tape)
        # conv -> BN -> ReLU -> MaxPool run as conv + one BN/ReLU/pool pass (the un-pooled
        # activation is written only where the decoder also reads it: x1, x2)
        p1 = nh(H // 2, W // 2, 64); E[1].forward(a, None, training, tape, pool=p1)
        a2 = nh(H // 2, W // 2, 128); E[2].forward(p1, a2, training, tape)
        p2 = nh(H // 4, W // 4, 128); E[3].forward(a2, None, training, tape, pool=p2)
        a4 = nh(H // 4, W // 4, 256); E[4].forward(p2, a4, training, tape)
        a5 = nh(H // 4, W // 4, 256); E[5].forward(a4, a5, training, tape)
        dec1in = K.nhwc(N, H // 4, W // 4, 512, dt, dev)
        x1 = Act(dec1in, 256, 256)
        p3 = nh(H // 8, W // 8, 256)
        inst = {}
        if self.inorm:
            inst["x1"] = self._inorm_stage(E[6], a5, x1, p3, training, tape)
        else:
            E[6].forward(a5, x1, training, tape, pool=p3)
        a7 = nh(H // 8, W // 8, 512); E[7].forward(p3, a7, training, tape)
        a8 = nh(H // 8, W // 8, 512); E[8].forward(a7, a8, training, tape)
        dec2in = K.nhwc(N, H // 8, W // 8, 1024, dt, dev)
        x2 = Act(dec2in, 512, 512)
        p4 = nh(H // 16, W // 16, 512)
        if self.inorm:
            inst["x2"] = self._inorm_stage(E[9], a8, x2, p4, training, tape)
        else:
            E[9].forward(a8, x2, training, tape, pool=p4)
        a10 = nh(H // 16, W // 16, 512); E[10].forward(p4, a10, training, tape)
        a11 = nh(H // 16, W // 16, 512); E[11].forward(a10, a11, training, tape)
        x3 = nh(H // 16, W // 16, 512)
        if self.inorm:
            inst["x3"] = self._inorm_stage(E[12], a11, x3, None, training, tape)
        else:
            E[12].forward(a11, x3, training, tape)
        # decoder
        a13 = nh(H // 16, W // 16, 1024); D[0].forward(x3, a13, training, tape)
        y3 = nh(H // 16, W // 16, 512); D[1].forward(a13, y3, training, tape)
        K.upsample_fwd(y3, 2, K.UP_BILINEAR, Act(dec2in, 0, 512))
        a15 = nh(H // 8, W // 8, 512); D[2].forward(_cat_act(dec2in, y3, x2), a15, training, tape)
        y2 = nh(H // 8, W // 8, 256); D[3].forward(a15, y2, training, tape)
        K.upsample_fwd(y2, 2, K.UP_BILINEAR, Act(dec1in, 0, 256))
        a17 = nh(H // 4, W // 4, 256); D[4].forward(_cat_act(dec1in, y2, x1), a17, training, tape)
        y1 = nh(H // 4, W // 4, 128); D[5].forward(a17, y1, training, tape)
        if tape is not None:
            tape[self] = dict(dec1in=dec1in, dec2in=dec2in, shape=(N, H, W), dt=dt, inst=inst, x1=x1, x2=x2, x3=x3)
        # the plain tensors cross the autograd boundary; their f32 operand maxima go with them
        return K.export_amax(y1), K.export_amax(y2), K.export_amax(y3), K.export_amax(x3)

    @staticmethod
    def _inorm_stage(layer, x, out: Act, pool: Act | None, training, tape):
        """layer -> raw stage output, instance-normalised into `out`, then max-pooled into
        `pool` (the next stage's input).  Returns (raw output, IN statistics)."""
        raw = Act(K.nhwc(out.N, out.H, out.W, out.C, out.buf.dtype, out.buf.device))
        layer.forward(x, raw, training, tape)
        st = K.instnorm_stats(raw)
        K.instnorm_apply(raw, st, None, None, K.ACT_NONE, out)
        if pool is not None:
            K.maxpool_fwd(out, pool)
        return raw, st

    @staticmethod
    def _inorm_stage_bwd(layer, tape, g_out: Act, out: Act, g_pool: Act | None, inst, gx: Act, gx_bn=None):
        """Backward of _inorm_stage: g_out (the normalised output's direct gradient, written in
        place) += maxpool backward of g_pool; IN backward; the layer's backward."""
        raw, st = inst
        if g_pool is not None:
            K.maxpool_bwd(out, g_pool, g_out, accumulate=True)
        g_raw = Act(torch.empty_like(raw.buf))
        K.instnorm_bwd(g_out, raw, st, None, g_raw)
        return layer.backward(tape, g_raw, gx, gx_bn=gx_bn)

    def backward(self, tape: dict, g_y1, g_y2, g_y3, g_x3) -> dict:
        """Gradients of (y1, y2, y3, x3) from the heads (None = unused)."""
        s = tape.pop(self)
        N, H, W = s["shape"]
        dt = s["dt"]
        dev = s["dec1in"].device
        E, D = self.enc, self.dec
        nh = lambda h, w, c: Act(K.nhwc(N, h, w, c, dt, dev))  # noqa: E731

        def own(g, h, w, c):  # a writable NHWC gradient buffer (zeros when the output was unused)
            if g is None:
                return Act(K.nhwc(N, h, w, c, dt, dev, zero=True))
            return Act(g.to(dt).contiguous().clone())

        grads = _SinkDict(self.sink)
        # decoder
        g_a17 = nh(H // 4, W // 4, 256)
        grads.update(D[5].backward(tape, own(g_y1, H // 4, W // 4, 128), g_a17, gx_bn=D[4]))
        g_dec1in = K.nhwc(N, H // 4, W // 4, 512, dt, dev)
        grads.update(D[4].backward(tape, g_a17, Act(g_dec1in)))
        gy2 = own(g_y2, H // 8, W // 8, 256)
        K.upsample_bwd(Act(g_dec1in, 0, 256), 2, K.UP_BILINEAR, gy2, accumulate=True)
        g_a15 = nh(H // 8, W // 8, 512)
        grads.update(D[3].backward(tape, gy2, g_a15, gx_bn=D[2]))
        g_dec2in = K.nhwc(N, H // 8, W // 8, 1024, dt, dev)
        grads.update(D[2].backward(tape, g_a15, Act(g_dec2in)))
        g_y3 = own(g_y3, H // 16, W // 16, 512)
        K.upsample_bwd(Act(g_dec2in, 0, 512), 2, K.UP_BILINEAR, g_y3, accumulate=True)
        g_a13 = nh(H // 16, W // 16, 1024)
        grads.update(D[1].backward(tape, g_y3, g_a13, gx_bn=D[0]))
        inst = s["inst"]
        if g_x3 is not None:
            gx3 = Act(g_x3.to(dt).contiguous().clone())
            grads.update(D[0].backward(tape, g_a13, gx3, accumulate_gx=True))
        else:
            gx3 = nh(H // 16, W // 16, 512)
            grads.update(D[0].backward(tape, g_a13, gx3, gx_bn=None if inst else E[12]))
        # enc3
        g_a11 = nh(H // 16, W // 16, 512)
        if inst:
            grads.update(self._inorm_stage_bwd(E[12], tape, gx3, s["x3"], None, inst["x3"], g_a11, gx_bn=E[11]))
        else:
            grads.update(E[12].backward(tape, gx3, g_a11, gx_bn=E[11]))
        g_a10 = nh(H // 16, W // 16, 512); grads.update(E[11].backward(tape, g_a11, g_a10, gx_bn=E[10]))
        g_p4 = nh(H // 16, W // 16, 512); grads.update(E[10].backward(tape, g_a10, g_p4))
        # enc2 (the pooled gradients are routed inside the BN backward of the pooled layers)
        g_a8 = nh(H // 8, W // 8, 512)
        if inst:
            grads.update(self._inorm_stage_bwd(E[9], tape, Act(g_dec2in, 512, 512), s["x2"], g_p4, inst["x2"], g_a8))
        else:
            grads.update(E[9].backward(tape, Act(g_dec2in, 512, 512), g_a8, g_pool=g_p4))
        g_a7 = nh(H // 8, W // 8, 512); grads.update(E[8].backward(tape, g_a8, g_a7, gx_bn=E[7]))
        g_p3 = nh(H // 8, W // 8, 256); grads.update(E[7].backward(tape, g_a7, g_p3))
        # enc1
        g_a5 = nh(H // 4, W // 4, 256)
        if inst:
            grads.update(self._inorm_stage_bwd(E[6], tape, Act(g_dec1in, 256, 256), s["x1"], g_p3, inst["x1"], g_a5))
        else:
            grads.update(E[6].backward(tape, Act(g_dec1in, 256, 256), g_a5, g_pool=g_p3))
        g_a4 = nh(H // 4, W // 4, 256); grads.update(E[5].backward(tape, g_a5, g_a4, gx_bn=E[4]))
        g_p2 = nh(H // 4, W // 4, 128); grads.update(E[4].backward(tape, g_a4, g_p2))
        g_a2 = nh(H // 2, W // 2, 128); grads.update(E[3].backward(tape, None, g_a2, g_pool=g_p2, gx_bn=E[2]))
        g_p1 = nh(H // 2, W // 2, 64); grads.update(E[2].backward(tape, g_a2, g_p1))
        g_a = nh(H, W, 64); grads.update(E[1].backward(tape, None, g_a, g_pool=g_p1))
        grads.update(E[0].backward(tape, g_a, None))
        return (), grads


class _SinkDict(dict):
    """The FeaturePlan backward's {param: grad}: each layer's batch passes through the plan's
    data-parallel gradient sink first (if any), which keeps what it reduces itself."""

    def __init__(self, sink):
        super().__init__()
        self.sink = sink

    def update(self, grads):
        super().update(self.sink.emit(grads) if self.sink is not None else grads)


class _PlanFn(torch.autograd.Function):
    """Bridges a plan's hand-scheduled backward into torch autograd.

    apply(plan, fwd, n_in, *inputs, *params): `fwd(*inputs, tape=...)` runs the
    forward launches; `plan.backward(tape, *grad_outputs)` returns
    (grads for the inputs, {param: grad}).  Params are Function arguments so
    autograd routes their gradients to `.grad` (AccumulateGrad)."""

    @staticmethod
    def forward(ctx, plan, fwd, n_in, *tensors):
        ctx.set_materialize_grads(False)  # unused outputs -> None, not zero tensors
        ctx.plan = plan
        ctx.n_in = n_in
        ctx.params = tensors[n_in:]
        ctx.tape = {}
        outs = fwd(*tensors[:n_in], tape=ctx.tape)
        nd = getattr(plan, "nondiff", ())
        if nd:
            ctx.mark_non_differentiable(*[outs[i] for i in nd])
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
        invalidate_frozen()  # a training forward re-derives packed filters once (both views share them)
    try:
        if need:
            return _PlanFn.apply(plan, fwd, len(inputs), *inputs, *params)
        with torch.no_grad():
            return fwd(*inputs, tape=None)
    finally:
        SB.flush_batches()  # the BatchNorm batch counts the forward bumped, in one launch


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
        self.dec = CatConvLayer(den_dec_block.conv, den_dec_block.bn, ACT_RELU)
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

    def forward(self, ycat, training: bool, tape: dict | None = None):
        """ycat: (y1, y2, y3) NHWC parts (CatParts) or a materialised NHWC y_cat tensor."""
        cat = as_cat(ycat)
        N, h, w = cat.N, cat.H, cat.W
        dt = cat.parts[0].buf.dtype if isinstance(cat, CatParts) else cat.buf.dtype
        dev = cat.parts[0].buf.device if isinstance(cat, CatParts) else cat.buf.device
        drop = dropout2d_mask(N, self.dec.Cout, self.p, dev) if training else None
        yden = Act(K.nhwc(N, h, w, self.dec.Cout, dt, dev))
        self.dec.forward(cat, yden, training, tape, drop=drop)
        hb = self.head_b.detach() if self.head_b is not None else None
        yh = K.head_fwd(yden, self.head_w.detach().reshape(-1), hb, self.head_act)
        d = torch.empty((N, 4 * h, 4 * w, 1), dtype=torch.float32, device=dev)
        K.upsample_fwd(Act(yh.view(N, h, w, 1)), 4, K.UP_BILINEAR, Act(d))
        if tape is not None:
            tape[self] = (cat, dt, yden, yh)
        return d.view(N, 1, 4 * h, 4 * w)

    def backward(self, tape: dict, g_d: torch.Tensor):
        cat, dt, yden, yh = tape.pop(self)
        N, h, w = cat.N, cat.H, cat.W
        dev = g_d.device
        g_h = torch.empty((N, h, w, 1), dtype=torch.float32, device=dev)
        K.upsample_bwd(Act(g_d.contiguous().view(N, 4 * h, 4 * w, 1)), 4, K.UP_BILINEAR, Act(g_h))
        g_yden = Act(torch.empty_like(yden.buf))
        gw = torch.empty(self.dec.Cout, dtype=torch.float32, device=dev)
        gb = torch.empty(1, dtype=torch.float32, device=dev) if self.head_b is not None else None
        K.head_bwd(yden, self.head_w.detach().reshape(-1), self.head_act, yh, g_h.view(N, h, w),
                   g_yden, gw, gb)
        g_cat = cat_empty_like(cat)
        grads = self.dec.backward(tape, g_yden, g_cat)
        grads[self.head_w] = gw.view_as(self.head_w)
        if gb is not None:
            grads[self.head_b] = gb
        return cat_grads(g_cat), grads


# ---------------------------------------------------------------------------
# Memory read (DGModel_mem.forward_mem, models/models.py:116-125) on NHWC:
#   logits[px][slot] = y[px] . mem[:, slot] / sqrt(k)   (1x1 conv, Cout = 1024)
#   P = softmax over slots ; y_new[px][k] = sum_slot P[px][slot] mem[k][slot]
# ---------------------------------------------------------------------------
class MemRead:
    def __init__(self, mem: nn.Parameter):
        self.mem = mem  # [1, k, slots]

    def packs(self, dt, training=True):
        if not training:
            return frozen(self, ("packs", dt), (self.mem,), lambda: self.packs(dt))
        m = self.mem.detach()[0]  # [k, slots]
        k, S = m.shape
        scale = 1.0 / float(k) ** 0.5
        memT_s = K.pack_weight((m.t() * scale).contiguous().view(S, k, 1, 1), dt)  # logits GEMM
        mem_p = K.pack_weight(m.contiguous().view(k, S, 1, 1), dt)                 # y_new GEMM
        return memT_s, mem_p, scale

    def logits(self, y: Act, memT_s, dt):
        S = self.mem.shape[2]
        L = Act(K.nhwc(y.N, y.H, y.W, S, dt, y.buf.device))
        K.conv_fwd(y, memT_s, S, 1, 0, L)
        return L

    def readout(self, P: Act, mem_p, dt):
        k = self.mem.shape[1]
        yn = Act(K.nhwc(P.N, P.H, P.W, k, dt, P.buf.device))
        K.conv_fwd(P, mem_p, k, 1, 0, yn)
        return yn

    def bwd_readout(self, g_yn: Act, P: Act, dt):
        """g_P = g_yn . mem ; dmem_a[k][slot] = sum_px g_yn[px][k] P[px][slot]."""
        m = self.mem.detach()[0]
        k, S = m.shape
        memT = K.pack_weight(m.t().contiguous().view(S, k, 1, 1), dt)
        gP = Act(K.nhwc(P.N, P.H, P.W, S, dt, P.buf.device))
        K.conv_fwd(g_yn, memT, S, 1, 0, gP)
        dmem = torch.empty((k, S, 1, 1), dtype=torch.float32, device=P.buf.device)
        K.conv_wgrad(P, g_yn, 1, 0, dmem)
        return gP, dmem.view(k, S)

    # --- readout folded into the density head (MEM_HEAD_FUSED) -----------------
    def head_vec(self, head_w) -> torch.Tensor:
        """v = mem^T w [S] f32: den_head's weights pulled through the readout."""
        m = self.mem.detach()[0]
        k, S = m.shape
        v = torch.empty(S, dtype=torch.float32, device=m.device)
        K.call("dg_mem_head_vec", K.ptr(m), K.ptr(head_w.detach().reshape(-1)), k, S, K.ptr(v), K.stream())
        return v

    def head_grads(self, work, M: int, head_w, want_dmem: bool = True):
        """After dg_softmax_head_bwd: (dmem_readout [k][S] or None, gw [k], gb [1])."""
        m = self.mem.detach()[0]
        k, S = m.shape
        dmem = torch.empty((k, S), dtype=torch.float32, device=m.device) if want_dmem else None
        gw = torch.empty(k, dtype=torch.float32, device=m.device)
        gb = torch.empty(1, dtype=torch.float32, device=m.device)
        K.call("dg_mem_head_grads", K.ptr(work), M, S, K.ptr(m), K.ptr(head_w.detach().reshape(-1)), k,
               K.ptr(dmem), K.ptr(gw), K.ptr(gb), K.stream())
        return dmem, gw, gb

    def bwd_logits(self, gL: Act, y: Act, mem_p, scale, dt):
        """g_y = gL . mem^T * scale ; dmem_b[k][slot] = scale * sum_px y[px][k] gL[px][slot]."""
        k, S = self.mem.shape[1], self.mem.shape[2]
        gy = Act(K.nhwc(y.N, y.H, y.W, k, dt, y.buf.device))
        if dt == torch.float32:  # one operand-max pass each for the two convs below (f16 x3 scales)
            if gL.amax is None:
                gL.amax = K.amax(gL)
            if y.amax is None:
                y.amax = K.amax(y)
        m_s = K.pack_weight((self.mem.detach()[0] * scale).contiguous().view(k, S, 1, 1), dt)
        K.conv_fwd(gL, m_s, k, 1, 0, gy)
        dmem = torch.empty((k, S, 1, 1), dtype=torch.float32, device=y.buf.device)
        K.conv_wgrad(gL, y, 1, 0, dmem)
        return gy, dmem.view(k, S) * scale


class _Heads:
    """Shared pieces after forward_fe for the DGModel_* family (models/models.py:98-335)."""

    def __init__(self, model, mem: bool, cls: bool):
        dd = model.den_dec[0]
        self.den = CatConvLayer(dd.conv, dd.bn, ACT_RELU)
        self.den_drop_module = next((m for m in model.den_dec if isinstance(m, nn.Dropout2d)), None)
        # DGModel_*: den_head = Sequential(ConvBlock); models2.DensityRegressorM: a bare ConvBlock
        hb = model.den_head[0] if isinstance(model.den_head, nn.Sequential) else model.den_head
        hc = hb.conv
        self.head_w, self.head_b = hc.weight, hc.bias
        self.head_act = K.ACT_RELU if hb.relu is not None else K.ACT_NONE
        self.raw = True  # models2.DensityRegressorM.forward(raw=False): memory read under no_grad
        self.memr = MemRead(model.mem) if mem else None
        self.cls = None
        if cls:
            c0 = model.cls_head[0]
            self.cls = ConvLayer(c0.conv, c0.bn, ACT_RELU)
            self.cls_drop_module = model.cls_head[1]
            self.cls_w = model.cls_head[2].conv.weight
            self.cls_b = model.cls_head[2].conv.bias
        self.model = model

    def params(self):
        ps = self.den.params() + [self.head_w] + ([self.head_b] if self.head_b is not None else [])
        if self.memr is not None:
            ps.append(self.memr.mem)
        if self.cls is not None:
            ps += self.cls.params() + [self.cls_w] + ([self.cls_b] if self.cls_b is not None else [])
        return ps

    # --- pieces ---------------------------------------------------------------
    def head(self, y: Act):
        hb = self.head_b.detach() if self.head_b is not None else None
        return K.head_fwd(y, self.head_w.detach().reshape(-1), hb, self.head_act)

    def head_bwd(self, y: Act, yh, g_h, grads):
        g_y = Act(torch.empty_like(y.buf))
        gw = torch.empty(y.C, dtype=torch.float32, device=y.buf.device)
        gb = torch.empty(1, dtype=torch.float32, device=y.buf.device) if self.head_b is not None else None
        K.head_bwd(y, self.head_w.detach().reshape(-1), self.head_act, yh, g_h, g_y, gw, gb)
        _acc(grads, self.head_w, gw.view_as(self.head_w))
        if gb is not None:
            _acc(grads, self.head_b, gb)
        return g_y

    def head_acc(self, grads, gw, gb):
        _acc(grads, self.head_w, gw.view_as(self.head_w))
        if self.head_b is not None:
            _acc(grads, self.head_b, gb)

    def mem_head_fwd(self, Ls, dt, loss: int, keep_p: bool):
        """Slot softmax of 1 or 2 views' logits + the density head through the readout (+ loss):
        returns (Ps or None, yhs, v, loss tensor or None)."""
        L1 = Ls[0]
        N, h, w = L1.N, L1.H, L1.W
        dev = L1.buf.device
        v = self.memr.head_vec(self.head_w)
        Ps = [Act(torch.empty_like(L.buf)) for L in Ls] if keep_p else None
        yhs = [torch.empty((N, h, w), dtype=torch.float32, device=dev) for _ in Ls]
        loss_t = torch.empty((), dtype=torch.float32, device=dev) if loss else None
        work = torch.empty(K.query("dg_mem_head_workspace", L1.M, L1.C) // 4 + 1, dtype=torch.float32, device=dev)
        hb = self.head_b.detach() if self.head_b is not None else None
        two = len(Ls) == 2
        K.call("dg_softmax_head_fwd", L1.dt, len(Ls), loss, L1.ptr, Ls[1].ptr if two else None, L1.M, L1.C,
               K.ptr(v), K.ptr(hb), self.head_act, Ps[0].ptr if Ps else None,
               Ps[1].ptr if (Ps and two) else None, K.ptr(yhs[0]), K.ptr(yhs[1]) if two else None,
               K.ptr(loss_t), K.ptr(work), K.stream())
        return Ps, yhs, v, loss_t

    def mem_head_bwd(self, Ps, yhs, v, g_hs, loss: int, coef, grads, want_gl: bool = True):
        """Backward of mem_head_fwd: logit gradients (or None) and the head / readout-mem grads."""
        P1 = Ps[0]
        M, S = P1.M, P1.C
        dev = P1.buf.device
        two = len(Ps) == 2
        work = torch.empty(K.query("dg_mem_head_workspace", M, S) // 4 + 1, dtype=torch.float32, device=dev)
        gLs = [Act(torch.empty_like(P.buf)) for P in Ps] if want_gl else None
        # f32: the operand maxima with channels (slots) of gL_v from the same pass, for the logits GEMMs'
        # f16 x3 scales in bwd_logits (per slot in their weight gradient)
        nw = K.amax_words(S)
        am = torch.empty(2 * nw, dtype=torch.float32, device=dev) if (gLs and P1.buf.dtype == torch.float32) else None
        if am is not None:
            for i, gL in enumerate(gLs):
                gL.amax = am[i * nw:(i + 1) * nw]
        K.call("dg_softmax_head_bwd", P1.dt, len(Ps), loss, P1.ptr, Ps[1].ptr if two else None, M, S, K.ptr(v),
               self.head_act, K.ptr(yhs[0]), K.ptr(yhs[1]) if two else None, K.ptr(g_hs[0]),
               K.ptr(g_hs[1]) if two else None, K.ptr(coef), gLs[0].ptr if gLs else None,
               gLs[1].ptr if (gLs and two) else None, K.ptr(work), K.ptr(am), K.stream())
        dmem = None
        if any(g is not None for g in g_hs):
            dmem, gw, gb = self.memr.head_grads(work, M, self.head_w, want_dmem=want_gl)
            self.head_acc(grads, gw, gb)
        return gLs, dmem

    def cls_fwd(self, x3: torch.Tensor, training, tape, key):
        N, h, w, _ = x3.shape
        drop = dropout2d_mask(N, self.cls.Cout, self.cls_drop_module.p, x3.device) \
            if training and self.cls_drop_module.p > 0 else None
        a = Act(K.nhwc(N, h, w, self.cls.Cout, x3.dtype, x3.device))
        sub = {} if tape is not None else None
        self.cls.forward(K.import_act(x3), a, training, sub, drop=drop)
        cb = self.cls_b.detach() if self.cls_b is not None else None
        c = K.head_fwd(a, self.cls_w.detach().reshape(-1), cb, K.ACT_SIGMOID)
        if tape is not None:
            tape[key] = (sub, a, c, x3.shape, x3.dtype)
        return c  # [N, h, w] f32

    def cls_bwd(self, tape, key, g_c, grads):
        sub, a, c, shape, dt = tape.pop(key)
        g_a = Act(torch.empty_like(a.buf))
        gw = torch.empty(a.C, dtype=torch.float32, device=a.buf.device)
        gb = torch.empty(1, dtype=torch.float32, device=a.buf.device) if self.cls_b is not None else None
        K.head_bwd(a, self.cls_w.detach().reshape(-1), K.ACT_SIGMOID, c,
                   g_c.contiguous().view(c.shape).float(), g_a, gw, gb)
        _acc(grads, self.cls_w, gw.view_as(self.cls_w))
        if gb is not None:
            _acc(grads, self.cls_b, gb)
        g_x3 = torch.empty(shape, dtype=dt, device=a.buf.device)
        for p, g in self.cls.backward(sub, g_a, Act(g_x3)).items():
            _acc(grads, p, g)
        return g_x3


def _acc(grads, p, g):
    if p in grads:
        grads[p] = grads[p] + g
    else:
        grads[p] = g


def _up4(x_small: torch.Tensor, N, h, w):
    d = torch.empty((N, 4 * h, 4 * w, 1), dtype=torch.float32, device=x_small.device)
    K.upsample_fwd(Act(x_small.reshape(N, h, w, 1)), 4, K.UP_BILINEAR, Act(d))
    return d.view(N, 1, 4 * h, 4 * w)


def _up4_bwd(g: torch.Tensor, N, h, w):
    gs = torch.empty((N, h, w, 1), dtype=torch.float32, device=g.device)
    K.upsample_bwd(Act(g.contiguous().view(N, 4 * h, 4 * w, 1)), 4, K.UP_BILINEAR, Act(gs))
    return gs.view(N, h, w)


class SinglePlan(_Heads):
    """`.forward` of DGModel_mem / cls / memcls / final (and base via mem=cls=False):
    ycat, x3 (NHWC) [, c_gt] -> d  or  (dc, c)."""

    def forward(self, ycat, x3, c_gt, training, tape=None):
        """ycat: (y1, y2, y3) NHWC parts or a materialised NHWC y_cat tensor."""
        cat = as_cat(ycat)
        N, h, w = cat.N, cat.H, cat.W
        dt, dev = x3.dtype, x3.device
        p = self.den_drop_module.p if (self.den_drop_module is not None and training) else 0.0
        drop = dropout2d_mask(N, self.den.Cout, p, dev)
        sub = {} if tape is not None else None
        yden = Act(K.nhwc(N, h, w, self.den.Cout, dt, dev))
        self.den.forward(cat, yden, training, sub, drop=drop)
        st = {"sub": sub, "yden": yden, "cat": cat, "raw": self.raw}
        y = yden
        if self.memr is not None and MEM_HEAD_FUSED:
            memT_s, _, scale = self.memr.packs(dt, training)
            L = self.memr.logits(yden, memT_s, dt)
            Ps, yhs, v, _ = self.mem_head_fwd([L], dt, 0, keep_p=tape is not None)
            del L
            yh = yhs[0]
            st.update(P=Ps[0] if Ps else None, v=v, scale=scale)
        elif self.memr is not None:
            memT_s, mem_p, scale = self.memr.packs(dt, training)
            L = self.memr.logits(yden, memT_s, dt)
            P = Act(torch.empty_like(L.buf))
            K.call("dg_softmax_fwd", L.dt, L.ptr, L.M, L.C, P.ptr, K.stream())
            y = self.memr.readout(P, mem_p, dt)
            st.update(P=P, ynew=y, mem_p=mem_p, scale=scale)
            yh = self.head(y)
        else:
            yh = self.head(y)
        st["yh"] = yh
        if self.cls is None:
            out = _up4(yh, N, h, w)
            outs = out
        else:
            c = self.cls_fwd(x3, training, sub, "cls")
            cres = torch.empty((N, h, w), dtype=torch.float32, device=dev)
            cg = c_gt.float().contiguous() if c_gt is not None else None
            K.call("dg_cls_combine", K.ptr(c), None, K.ptr(cg), N, h // 4, w // 4, 4,
                   float(self.model.cls_thrs), K.ptr(cres), None, K.stream())
            prod = torch.empty_like(yh)
            K.call("dg_mul_f32", K.ptr(yh), K.ptr(cres), yh.numel(), K.ptr(prod), K.stream())
            st["cres"] = cres
            outs = (_up4(prod, N, h, w), c.view(N, 1, h // 4, w // 4))
        if tape is not None:
            tape[self] = st
        return outs

    def backward(self, tape, *gouts):
        st = tape.pop(self)
        sub = st["sub"]
        cat = st["cat"]
        N, h, w = cat.N, cat.H, cat.W
        grads = {}
        g_d = gouts[0]
        g_x3 = None
        if g_d is not None and not (self.memr is not None and not st["raw"]):
            g_h = _up4_bwd(g_d, N, h, w)
            if self.cls is not None:
                K.call("dg_mul_f32", K.ptr(g_h), K.ptr(st["cres"]), g_h.numel(), K.ptr(g_h), K.stream())
            if st.get("v") is not None:  # fused memory head
                (gL,), dmem_a = self.mem_head_bwd([st["P"]], [st["yh"]], st["v"], [g_h], 0, None, grads)
                g_y, dmem_b = self.memr.bwd_logits(gL, st["yden"], None, st["scale"], gL.buf.dtype)
                _acc(grads, self.memr.mem, (dmem_a + dmem_b).view_as(self.memr.mem))
            else:
                g_y = self.head_bwd(st.get("ynew", st["yden"]), st["yh"], g_h, grads)
            if self.memr is not None and st.get("v") is None:
                dt = st["ynew"].buf.dtype
                gP, dmem_a = self.memr.bwd_readout(g_y, st["P"], dt)
                gL = Act(torch.empty_like(gP.buf))
                K.call("dg_softmax_bwd", gP.dt, st["P"].ptr, gP.ptr, gP.M, gP.C, gL.ptr, K.stream())
                g_y, dmem_b = self.memr.bwd_logits(gL, st["yden"], st["mem_p"], st["scale"], dt)
                _acc(grads, self.memr.mem, (dmem_a + dmem_b).view_as(self.memr.mem))
            g_cat = cat_empty_like(cat)
            for p, g in self.den.backward(sub, g_y, g_cat).items():
                _acc(grads, p, g)
            g_cat = cat_grads(g_cat)
        else:
            g_cat = (None,) * (3 if isinstance(cat, CatParts) else 1)
            if g_d is not None:  # raw=False: only the density head sees the (constant) memory readout
                g_h = _up4_bwd(g_d, N, h, w)
                if self.cls is not None:
                    K.call("dg_mul_f32", K.ptr(g_h), K.ptr(st["cres"]), g_h.numel(), K.ptr(g_h), K.stream())
                if st.get("v") is not None:
                    self.mem_head_bwd([st["P"]], [st["yh"]], st["v"], [g_h], 0, None, grads, want_gl=False)
                else:
                    self.head_bwd(st["ynew"], st["yh"], g_h, grads)
        if self.cls is not None and len(gouts) > 1 and gouts[1] is not None:
            g_x3 = self.cls_bwd(sub, "cls", gouts[1], grads)
        return (*g_cat, g_x3), grads


class PairPlan(_Heads):
    """forward_train of DGModel_memadd (cls=False) and DGModel_final (cls=True)
    (models/models.py:147-184, 298-335): two views, e_mask from instance norms,
    functional Dropout2d (always on), memory read, JSD-MSE consistency loss."""

    def __init__(self, model, cls: bool, variant: str = "final"):
        super().__init__(model, mem=True, cls=cls)
        # variant "M" = models2.DensityRegressorM.forward_train (models/models2.py:321-373): KL-JSD
        # instead of the softmax MSE, per-view class maps (no c_err), plus loss_err =
        # L1(IN(y1), IN(y2)); outputs (dc1, dc2, c1, c2, loss_kl, loss_err)
        self.variant = variant
        # final: (dc1, dc2, c1, c2, c_err, loss_con); memadd: (d1, d2, loss_con)
        self.nondiff = (4,) if (cls and variant == "final") else ()
        # parity instrumentation: a dict here receives the threshold decisions of the next
        # forward (e_mask as uint8 NHWC [N,h,w,C]; the thresholded class maps), so a checker
        # can be run on the same decisions (bench.py's full-frame final-mode parity)
        self.capture = None
        # the converse: a dict {"emask": uint8 [N,h,w,C], "c_pred": (c1, c2) 0/1 [N,1,h/4,w/4]}
        # whose decisions the next forward uses instead of its own (a strong-scaled DP rank run on
        # a single-process run's decisions, tests/dp_syncbn_worker.py); consumed by that forward
        self.inject = None

    def forward(self, ycat1, ycat2, x3_1, x3_2, c_gt, p_drop, err_thrs, tape=None):
        """ycat1/2: (y1, y2, y3) NHWC parts or materialised NHWC y_cat tensors."""
        cat1, cat2 = as_cat(ycat1), as_cat(ycat2)
        N, h, w = cat1.N, cat1.H, cat1.W
        HW = h * w
        dt, dev = x3_1.dtype, x3_1.device
        training = True
        sub = {} if tape is not None else None
        C = self.den.Cout
        y1 = Act(K.nhwc(N, h, w, C, dt, dev))
        y2 = Act(K.nhwc(N, h, w, C, dt, dev))
        s1 = {} if tape is not None else None
        s2 = {} if tape is not None else None
        self.den.forward(cat1, y1, training, s1)
        self.den.forward(cat2, y2, training, s2)
        # instance-norm statistics -> e_mask (detached) -> masked, dropped features
        stats = torch.empty((4, N * C), dtype=torch.float32, device=dev)
        ws = K.query("dg_instnorm_workspace", N, HW, C)
        work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=dev)
        K.call("dg_instnorm_stats", y1.dt, y1.ptr, y1.ld, N, HW, C, 1e-5, K.ptr(stats[0]),
               K.ptr(stats[1]), K.ptr(work), K.stream())
        K.call("dg_instnorm_stats", y2.dt, y2.ptr, y2.ld, N, HW, C, 1e-5, K.ptr(stats[2]),
               K.ptr(stats[3]), K.ptr(work), K.stream())
        d1 = dropout2d_mask(N, C, p_drop, dev)
        d2 = dropout2d_mask(N, C, p_drop, dev)
        m1 = Act(K.nhwc(N, h, w, C, dt, dev))
        m2 = Act(K.nhwc(N, h, w, C, dt, dev))
        mask = torch.empty((N * HW * C,), dtype=torch.uint8, device=dev)
        K.call("dg_emask_fwd", y1.dt, y1.ptr, y2.ptr, y1.ld, N, HW, C, K.ptr(stats[0]), K.ptr(stats[1]),
               K.ptr(stats[2]), K.ptr(stats[3]), float(err_thrs), K.ptr(d1), K.ptr(d2), m1.ptr, m2.ptr,
               K.ptr(mask), K.stream())
        inject, self.inject = self.inject, None
        if self.capture is not None:
            self.capture["emask"] = mask.view(N, h, w, C).clone()
        if inject is not None and "emask" in inject:
            # injected decisions: m_v = y_v * e * drop_v is exactly dg_emask_bwd's product
            em = inject["emask"]
            if tuple(em.shape) != (N, h, w, C) or em.dtype != torch.uint8 or y1.ld != C:
                raise ValueError(f"PairPlan.inject: e_mask must be uint8 {(N, h, w, C)}, got {tuple(em.shape)}")
            mask.copy_(em.reshape(-1))
            K.call("dg_emask_bwd", y1.dt, y1.ptr, y2.ptr, N, HW, C, K.ptr(mask), K.ptr(d1), K.ptr(d2), m1.ptr,
                   m2.ptr, C, K.stream())
        if dt == torch.float32 and y1.amax is not None and y2.amax is not None:
            # m_v = y_v * e * drop_v with e in {0, 1} and one keep value per mask: fl(max|y_v| * max drop_v)
            # bounds every fl(|y| * drop) (rounding is monotone), the logits GEMMs' f16 x3 operand scale
            m1.amax = y1.amax if d1 is None else y1.amax * d1.max()
            m2.amax = y2.amax if d2 is None else y2.amax * d2.max()
        # memory read, both views, + consistency loss
        memT_s, mem_p, scale = self.memr.packs(dt)
        L1 = self.memr.logits(m1, memT_s, dt)
        L2 = self.memr.logits(m2, memT_s, dt)
        v = None
        if MEM_HEAD_FUSED:
            (P1, P2), (yh1, yh2), v, loss_con = self.mem_head_fwd([L1, L2], dt, 2 if self.variant == "M" else 1,
                                                                  keep_p=True)
            yn1 = yn2 = None
        else:
            P1, P2 = Act(torch.empty_like(L1.buf)), Act(torch.empty_like(L2.buf))
            loss_con = torch.empty((), dtype=torch.float32, device=dev)
            ws = K.query("dg_softmax_workspace", L1.M)
            work2 = torch.empty(ws // 4 + 1, dtype=torch.float32, device=dev)
            fn = "dg_softmax_jsd_fwd" if self.variant == "M" else "dg_softmax_pair_fwd"
            K.call(fn, L1.dt, L1.ptr, L2.ptr, L1.M, L1.C, P1.ptr, P2.ptr, K.ptr(loss_con), K.ptr(work2), K.stream())
            yn1 = self.memr.readout(P1, mem_p, dt)
            yn2 = self.memr.readout(P2, mem_p, dt)
            yh1, yh2 = self.head(yn1), self.head(yn2)
        del L1, L2
        st = dict(s1=s1, s2=s2, cat1=cat1, cat2=cat2, mask=mask, d1=d1, d2=d2, m1=m1, m2=m2, P1=P1,
                  P2=P2, yn1=yn1, yn2=yn2, yh1=yh1, yh2=yh2, mem_p=mem_p, scale=scale, v=v)
        if self.cls is None:
            outs = (_up4(yh1, N, h, w), _up4(yh2, N, h, w), loss_con)
        elif self.variant == "M":
            c1 = self.cls_fwd(x3_1, training, sub, "c1")
            c2 = self.cls_fwd(x3_2, training, sub, "c2")
            cg = c_gt.float().contiguous() if c_gt is not None else None
            thr = float(self.model.cls_thrs)
            cres1 = torch.empty((N, h, w), dtype=torch.float32, device=dev)
            cres2 = torch.empty((N, h, w), dtype=torch.float32, device=dev)
            K.call("dg_cls_combine", K.ptr(c1), None, K.ptr(cg), N, h // 4, w // 4, 4, thr, K.ptr(cres1), None,
                   K.stream())
            K.call("dg_cls_combine", K.ptr(c2), None, K.ptr(cg), N, h // 4, w // 4, 4, thr, K.ptr(cres2), None,
                   K.stream())
            p1, p2 = torch.empty_like(yh1), torch.empty_like(yh2)
            K.call("dg_mul_f32", K.ptr(yh1), K.ptr(cres1), yh1.numel(), K.ptr(p1), K.stream())
            K.call("dg_mul_f32", K.ptr(yh2), K.ptr(cres2), yh2.numel(), K.ptr(p2), K.stream())
            loss_err = self._in_l1(y1, y2, stats, N, HW, C)
            st.update(cres1=cres1, cres2=cres2, sub=sub, stats=stats, y1=y1, y2=y2)
            outs = (_up4(p1, N, h, w), _up4(p2, N, h, w), c1.view(N, 1, h // 4, w // 4),
                    c2.view(N, 1, h // 4, w // 4), loss_con, loss_err)
        else:
            c1 = self.cls_fwd(x3_1, training, sub, "c1")
            c2 = self.cls_fwd(x3_2, training, sub, "c2")
            cres = torch.empty((N, h, w), dtype=torch.float32, device=dev)
            cerr = torch.empty((N, h, w), dtype=torch.float32, device=dev)
            cg = c_gt.float().contiguous() if c_gt is not None else None
            thr = float(self.model.cls_thrs)
            cd1, cd2 = c1, c2
            if inject is not None and "c_pred" in inject:
                # injected class decisions as 0/1 maps: (1 >= thr) and (0 < thr) for thr in (0, 1]
                if not 0.0 < thr <= 1.0:
                    raise ValueError("PairPlan.inject: class decisions need 0 < cls_thrs <= 1")
                cd1, cd2 = (t.to(device=dev, dtype=torch.float32).reshape(c1.shape).contiguous()
                            for t in inject["c_pred"])
            K.call("dg_cls_combine", K.ptr(cd1), K.ptr(cd2), K.ptr(cg), N, h // 4, w // 4, 4,
                   thr, K.ptr(cres), K.ptr(cerr), K.stream())
            p1, p2 = torch.empty_like(yh1), torch.empty_like(yh2)
            K.call("dg_mul_f32", K.ptr(yh1), K.ptr(cres), yh1.numel(), K.ptr(p1), K.stream())
            K.call("dg_mul_f32", K.ptr(yh2), K.ptr(cres), yh2.numel(), K.ptr(p2), K.stream())
            st.update(cres=cres, sub=sub)
            outs = (_up4(p1, N, h, w), _up4(p2, N, h, w), c1.view(N, 1, h // 4, w // 4),
                    c2.view(N, 1, h // 4, w // 4), _up4(cerr, N, h, w), loss_con)
            if getattr(self.model, "has_err_loss", False):
                # loss_err = F.l1_loss(IN(y_den1), IN(y_den2)) (models/models.py:303-311)
                outs = outs + (self._in_l1(y1, y2, stats, N, HW, C),)
                st.update(stats=stats, y1=y1, y2=y2)
            if self.capture is not None:
                self.capture.update(c_pred=((c1 >= thr).float().view(N, 1, h // 4, w // 4),
                                            (c2 >= thr).float().view(N, 1, h // 4, w // 4)))
        if tape is not None:
            tape[self] = st
        return outs

    @staticmethod
    def _in_l1(y1: Act, y2: Act, stats, N, HW, C):
        """mean |IN(y1) - IN(y2)| from the instance-norm statistics already formed for e_mask."""
        dev = y1.buf.device
        loss_err = torch.empty((), dtype=torch.float32, device=dev)
        work = torch.empty(K.query("dg_in_l1_workspace", N, HW, C) // 4 + 1, dtype=torch.float32, device=dev)
        K.call("dg_in_l1_fwd", y1.dt, y1.ptr, y2.ptr, y1.ld, N, HW, C, K.ptr(stats[0]), K.ptr(stats[1]),
               K.ptr(stats[2]), K.ptr(stats[3]), K.ptr(loss_err), K.ptr(work), K.stream())
        return loss_err

    def backward(self, tape, *gouts):
        st = tape.pop(self)
        N, h, w = st["cat1"].N, st["cat1"].H, st["cat1"].W
        HW = h * w
        grads = {}
        g_err = None
        if self.cls is None:
            g_d1, g_d2, g_con = gouts
            g_c1 = g_c2 = None
        elif self.variant == "M":
            g_d1, g_d2, g_c1, g_c2, g_con, g_err = gouts
        else:  # (+ loss_err's gradient when the forward ran with has_err_loss)
            g_d1, g_d2, g_c1, g_c2, _g_cerr, g_con = gouts[:6]
            g_err = gouts[6] if len(gouts) > 6 else None
        dt = st["m1"].buf.dtype
        dev = st["m1"].buf.device
        C = self.den.Cout

        def head_path(g_d, yh, yn, cres):
            if g_d is None:
                return None
            g_h = _up4_bwd(g_d, N, h, w)
            if cres is not None:
                K.call("dg_mul_f32", K.ptr(g_h), K.ptr(cres), g_h.numel(), K.ptr(g_h), K.stream())
            return self.head_bwd(yn, yh, g_h, grads)

        P1, P2 = st["P1"], st["P2"]
        coef = g_con.float().reshape(1).contiguous() if g_con is not None else None
        dmem = torch.zeros((C, self.memr.mem.shape[2]), dtype=torch.float32, device=dev)
        if st["v"] is not None:  # fused memory head: gP = gpre v formed in registers
            def g_head(g_d, cres):
                if g_d is None:
                    return None
                g_h = _up4_bwd(g_d, N, h, w)
                if cres is not None:
                    K.call("dg_mul_f32", K.ptr(g_h), K.ptr(cres), g_h.numel(), K.ptr(g_h), K.stream())
                return g_h

            g_hs = [g_head(g_d1, st.get("cres1", st.get("cres"))), g_head(g_d2, st.get("cres2", st.get("cres")))]
            (gL1, gL2), da = self.mem_head_bwd([P1, P2], [st["yh1"], st["yh2"]], st["v"], g_hs,
                                               2 if self.variant == "M" else 1, coef, grads)
            if da is not None:
                dmem += da
        else:
            g_yn1 = head_path(g_d1, st["yh1"], st["yn1"], st.get("cres1", st.get("cres")))
            g_yn2 = head_path(g_d2, st["yh2"], st["yn2"], st.get("cres2", st.get("cres")))
            gP1 = gP2 = None
            if g_yn1 is not None:
                gP1, da = self.memr.bwd_readout(g_yn1, P1, dt)
                dmem += da
            if g_yn2 is not None:
                gP2, da = self.memr.bwd_readout(g_yn2, P2, dt)
                dmem += da
            gL1, gL2 = Act(torch.empty_like(P1.buf)), Act(torch.empty_like(P2.buf))
            fn = "dg_softmax_jsd_bwd" if self.variant == "M" else "dg_softmax_pair_bwd"
            K.call(fn, P1.dt, P1.ptr, P2.ptr, gP1.ptr if gP1 is not None else None,
                   gP2.ptr if gP2 is not None else None, P1.M, P1.C, K.ptr(coef), gL1.ptr, gL2.ptr, K.stream())
        g_m1, db1 = self.memr.bwd_logits(gL1, st["m1"], st["mem_p"], st["scale"], dt)
        g_m2, db2 = self.memr.bwd_logits(gL2, st["m2"], st["mem_p"], st["scale"], dt)
        dmem += db1 + db2
        _acc(grads, self.memr.mem, dmem.view_as(self.memr.mem))
        g_y1 = Act(K.nhwc(N, h, w, C, dt, dev))
        g_y2 = Act(K.nhwc(N, h, w, C, dt, dev))
        K.call("dg_emask_bwd", g_m1.dt, g_m1.ptr, g_m2.ptr, N, HW, C, K.ptr(st["mask"]), K.ptr(st["d1"]),
               K.ptr(st["d2"]), g_y1.ptr, g_y2.ptr, g_y1.ld, K.stream())
        if g_err is not None:  # loss_err = L1(IN(y1), IN(y2)) back through both instance norms
            stats, y1, y2 = st["stats"], st["y1"], st["y2"]
            gi1, gi2 = Act(torch.empty_like(y1.buf)), Act(torch.empty_like(y2.buf))
            ce = g_err.float().reshape(1).contiguous()
            K.call("dg_in_l1_bwd", y1.dt, y1.ptr, y2.ptr, y1.ld, N, HW, C, K.ptr(stats[0]), K.ptr(stats[1]),
                   K.ptr(stats[2]), K.ptr(stats[3]), K.ptr(ce), gi1.ptr, gi2.ptr, K.stream())
            K.instnorm_bwd(gi1, y1, stats[0:2], None, g_y1, accumulate=True)
            K.instnorm_bwd(gi2, y2, stats[2:4], None, g_y2, accumulate=True)
        g_cat1, g_cat2 = cat_empty_like(st["cat1"]), cat_empty_like(st["cat2"])
        for p, g in self.den.backward(st["s1"], g_y1, g_cat1).items():
            _acc(grads, p, g)
        for p, g in self.den.backward(st["s2"], g_y2, g_cat2).items():
            _acc(grads, p, g)
        g_x3_1 = g_x3_2 = None
        if self.cls is not None:
            if g_c1 is not None:
                g_x3_1 = self.cls_bwd(st["sub"], "c1", g_c1, grads)
            if g_c2 is not None:
                g_x3_2 = self.cls_bwd(st["sub"], "c2", g_c2, grads)
        return (*cat_grads(g_cat1), *cat_grads(g_cat2), g_x3_1, g_x3_2), grads
