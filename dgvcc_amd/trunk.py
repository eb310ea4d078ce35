"""Kernel plans for the ResNet-50 domain-generalisation counters (SURVEY.md §8a
rows a11-a16): IBN-Net-b, ISW (instance selective whitening) and SW
(switchable whitening) trunks to layer3, plus the shared counter head.

The reference runs these as eager nn.Modules (models/ibnnet/resnet_ibn.py,
models/ISW/Resnet.py, models/SW/backbones/resnet.py).  Here each Bottleneck is
a fixed launch sequence over NHWC activations:

  conv1 1x1 -> BN stats -> BN+ReLU apply
  conv2 3x3/s -> BN (or SwitchWhiten2d) + ReLU
  conv3 1x1 -> BN stats ; [downsample 1x1/s -> BN stats]
  join: act(bn3(z3) + bn_ds(zd) | x)  in one pass (dg_bn_add_apply)
        [IBN-b: IN(affine)+ReLU after the join; ISW: IN (the whitened map w) + ReLU]

and backward is hand-scheduled in reverse.  Strided convs use the general
implicit-GEMM kernel (dg_conv2d_*), stride-1 "same" convs the specialised one.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import dist as D
from . import kernels as K
from . import syncbn as SB
from .engine import _PACK_FLIP, ACT_NONE, ACT_RELU, ConvLayer, _acc, _bn_momentum, bn_eval_cached, flip_of, frozen, pack_flip
from .kernels import Act

STEM_KPAD = 192  # 7*7*3 = 147 taps, padded to a multiple of 64 for the MFMA K loop
# DGVCC_TRUNK_RELU_FOLD=0: the block output ReLU's backward as its own pass (relu_bwd) instead of
# in the next block's conv1 dgrad epilogue (A/B; bit-identical either way)
_RELU_FOLD = __import__("os").environ.get("DGVCC_TRUNK_RELU_FOLD", "1") != "0"


class TConv:
    """Weights of one bias-free nn.Conv2d of the trunk; fwd / dgrad / wgrad launches."""

    def __init__(self, conv: nn.Conv2d):
        assert conv.groups == 1 and conv.dilation == (1, 1) and conv.bias is None
        self.conv = conv
        self.R = conv.kernel_size[0]
        self.stride = conv.stride[0]
        self.pad = conv.padding[0]
        self.Cin, self.Cout = conv.in_channels, conv.out_channels
        self.same = self.stride == 1 and 2 * self.pad == self.R - 1

    def pack(self, dt, training=True):
        """Packed filter, once per weight version (engine.frozen; run_plan starts each training
        forward on a fresh generation)."""
        if training and self.same and _PACK_FLIP:  # the dgrad's flipped filter from the same launch
            return frozen(self, ("w", dt), (self.conv.weight,), lambda: pack_flip(self, self.conv.weight, dt))
        return frozen(self, ("w", dt), (self.conv.weight,), lambda: K.pack_weight(self.conv.weight.detach(), dt))

    def _flip(self, wp):
        return flip_of(self, self.conv.weight, wp, self.Cout, self.Cin, self.R)

    def out_hw(self, H, W):
        return K.conv_out(H, self.R, self.stride, self.pad), K.conv_out(W, self.R, self.stride, self.pad)

    def fwd(self, x: Act, wp, y: Act):
        if self.same:
            K.conv_fwd(x, wp, self.Cout, self.R, self.pad, y)
        else:
            K.conv2d_fwd(x, wp, self.Cout, self.R, self.stride, self.pad, y)

    def bwd(self, x: Act, dz: Act, wp, dx: Act | None, accumulate=False, relu_out: Act | None = None) -> torch.Tensor:
        """relu_out (with accumulate): dx also gets the backward of the ReLU whose output is
        relu_out, dx = (relu_out > 0) ? dx + dgrad : 0 -- in the dgrad epilogue for the 1x1
        convs (dg_conv_fwd_acc_relu), else a relu_bwd pass after the dgrad."""
        dw = torch.empty_like(self.conv.weight, dtype=torch.float32)
        if self.same:
            K.conv_wgrad(x, dz, self.R, self.pad, dw)
        else:
            K.conv2d_wgrad(x, dz, self.R, self.stride, self.pad, dw)
        if dx is None:
            return dw
        if relu_out is not None:
            assert accumulate
            if self.same and self.R == 1 and K.conv_dgrad_acc_relu(dz, wp, self.Cin, dx, relu_out,
                                                                   wflip=self._flip(wp)):
                return dw
        if self.same:
            K.conv_dgrad(dz, wp, self.Cin, self.R, self.pad, dx, accumulate=accumulate, wflip=self._flip(wp))
        else:
            wt = K.pack_weight_t(wp, self.Cout, self.Cin, self.R, self.R)
            K.conv2d_dgrad(dz, wt, self.R, self.stride, self.pad, dx, accumulate=accumulate)
        if relu_out is not None:
            K.relu_bwd(dx, relu_out, dx)
        return dw


def bn_stats(z: Act, bn: nn.BatchNorm2d, training: bool) -> torch.Tensor:
    """[4, C]: mean, invstd, scale, shift (train: batch stats + running update).  An
    nn.SyncBatchNorm under a multi-rank process group (the ISW trunk's Norm2d when cfg.MODEL.BNFUNC
    is SyncBatchNorm, models/ISW/mynn.py:8-14) normalises with the whole batch's statistics."""
    if training:
        pg = SB.group_of(bn)
        if pg is not None:
            return SB.fwd_stats(bn, pg, z=z)
        SB.bump_batches(bn)
        return K.bn_fwd_train(z, bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                              bn.running_var, _bn_momentum(bn), bn.eps)
    return bn_eval_cached(bn, bn)


_EPI_STATS_OFF = __import__("os").environ.get("DGVCC_TRUNK_EPI_STATS", "1") == "0"


def conv_bn_stats(tc: "TConv", x: Act, wp, z: Act, bn: nn.BatchNorm2d, training: bool) -> torch.Tensor:
    """z = conv(x) and bn_stats(z) in one: in training the statistics come from the conv
    epilogue where the kernel serving the shape writes them (stride-1 'same' convs, as
    engine.ConvLayer does for the VGG encoder), which saves the statistics pass's full read of z;
    else the conv, then bn_stats.  DGVCC_TRUNK_EPI_STATS=0: always the separate pass (A/B)."""
    if training and tc.same and not _EPI_STATS_OFF:
        epi = K.conv_fwd_stats(x, wp, tc.Cout, tc.R, tc.pad, z)
        if epi is not None:
            pg = SB.group_of(bn)
            if pg is not None:
                return SB.fwd_stats(bn, pg, part=epi[0], nblk=epi[1], M=z.M)
            SB.bump_batches(bn)
            return K.bn_part_finalize(epi[0], epi[1], tc.Cout, bn.weight.detach(), bn.bias.detach(),
                                      bn.running_mean, bn.running_var, _bn_momentum(bn), bn.eps)
    tc.fwd(x, wp, z)
    return bn_stats(z, bn, training)


def bn_backward(bn: nn.BatchNorm2d, g: Act, z: Act, st, act: int, dz: Act, grads: dict):
    """dz of a training-mode BatchNorm (+ ReLU) from g; dgamma / dbeta accumulated into grads
    (the synchronised backward under a process group, as bn_stats' forward)."""
    C, dev = z.C, z.buf.device
    dgam = torch.empty(C, dtype=torch.float32, device=dev)
    dbet = torch.empty(C, dtype=torch.float32, device=dev)
    pg = SB.group_of(bn)
    if pg is not None:
        SB.backward(bn, pg, g, z, st, act, dz, dgam, dbet)
    else:
        K.bn_bwd(g, z, bn.weight.detach(), st, act, dz, dgam, dbet)
    _acc(grads, bn.weight, dgam)
    _acc(grads, bn.bias, dbet)


def _identity_stats(C, dev):
    st = torch.zeros((4, C), dtype=torch.float32, device=dev)
    st[1].fill_(1.0)
    st[2].fill_(1.0)
    return st


class Norm:
    """Stem / conv2 normalisation: 'bn' (BatchNorm2d), 'in' (InstanceNorm2d affine),
    'iw' (ISW InstanceWhitening = InstanceNorm2d(affine=False)), 'sw' (SwitchWhiten2d)."""

    def __init__(self, kind: str, module: nn.Module | None):
        self.kind, self.m = kind, module

    def params(self):
        m = self.m
        if self.kind == "bn" or (self.kind == "in" and m is not None and m.affine):
            return [m.weight, m.bias]
        if self.kind == "sw":
            return [m.sw_mean_weight, m.sw_var_weight, m.weight, m.bias]
        return []

    def _in_affine(self):
        m = self.m
        return (m.weight.detach(), m.bias.detach()) if (m is not None and m.affine) else (None, None)

    def forward(self, z: Act, y: Act, training: bool, act: int):
        """y = act(norm(z)); returns the state needed by backward."""
        if self.kind == "bn":
            st = bn_stats(z, self.m, training)
            K.bn_apply(z, st, act, y)
            return st
        if self.kind in ("in", "iw"):
            st = K.instnorm_stats(z, self.m.eps if self.m is not None else 1e-5)
            g, b = self._in_affine()
            K.instnorm_apply(z, st, g, b, act, y)
            return st
        m = self.m  # sw
        if getattr(m, "sync", False) and D.world() > 1:  # SyncSwitchWhiten2d over RCCL
            save, work, _ = K.sw_fwd_sync(z, m.sw_mean_weight.detach(), m.sw_var_weight.detach(),
                                          m.weight.detach(), m.bias.detach(), m.running_mean,
                                          m.running_cov, training, act, y, D.sum_moments(z.N), T=m.T,
                                          eps=m.eps, momentum=m.momentum)
            return ("sync", save, work)
        return K.sw_fwd(z, m.sw_mean_weight.detach(), m.sw_var_weight.detach(), m.weight.detach(),
                        m.bias.detach(), m.running_mean, m.running_cov, training, act, y, T=m.T,
                        eps=m.eps, momentum=m.momentum)

    def backward(self, g: Act, z: Act, y: Act, st, act: int, dz: Act, grads: dict):
        """dz = d norm / dz given g = dL/dy (ReLU mask from y when act)."""
        dev = z.buf.device
        C = z.C
        if self.kind == "bn":
            bn_backward(self.m, g, z, st, act, dz, grads)
        elif self.kind in ("in", "iw"):
            if act:
                K.relu_bwd(g, y, g)
            gam, _ = self._in_affine()
            if gam is not None:
                dgam = torch.empty(C, dtype=torch.float32, device=dev)
                dbet = torch.empty(C, dtype=torch.float32, device=dev)
                K.instnorm_bwd(g, z, st, gam, dz, dgam, dbet)
                _acc(grads, self.m.weight, dgam)
                _acc(grads, self.m.bias, dbet)
            else:
                K.instnorm_bwd(g, z, st, None, dz)
        else:
            m = self.m
            d = {p: torch.empty(p.shape, dtype=torch.float32, device=dev)
                 for p in (m.weight, m.bias, m.sw_mean_weight, m.sw_var_weight)}
            if isinstance(st, tuple):  # synchronized statistics: all-reduce the batch adjoints
                _, save, work = st
                K.sw_bwd_sync(g, y, z, save, work, m.sw_mean_weight.detach(), m.sw_var_weight.detach(),
                              m.weight.detach(), act, dz, D.sum_moments(z.N), d[m.weight], d[m.bias],
                              d[m.sw_mean_weight], d[m.sw_var_weight], T=m.T, eps=m.eps)
            else:
                K.sw_bwd(g, y, z, st, m.sw_mean_weight.detach(), m.sw_var_weight.detach(),
                         m.weight.detach(), act, dz, d[m.weight], d[m.bias], d[m.sw_mean_weight],
                         d[m.sw_var_weight], T=m.T, eps=m.eps)
            for p, v in d.items():
                _acc(grads, p, v)


class Block:
    """One Bottleneck (expansion 4) with optional post-join IN / IW."""

    def __init__(self, conv1, bn1, conv2, norm2: Norm, conv3, bn3, ds_conv=None, ds_bn=None,
                 post: Norm | None = None):
        self.c1, self.bn1 = TConv(conv1), bn1
        self.c2, self.n2 = TConv(conv2), norm2
        self.c3, self.bn3 = TConv(conv3), bn3
        self.cd = TConv(ds_conv) if ds_conv is not None else None
        self.bnd = ds_bn
        self.post = post

    def params(self):
        ps = [self.c1.conv.weight, self.bn1.weight, self.bn1.bias, self.c2.conv.weight]
        ps += self.n2.params() + [self.c3.conv.weight, self.bn3.weight, self.bn3.bias]
        if self.cd is not None:
            ps += [self.cd.conv.weight, self.bnd.weight, self.bnd.bias]
        if self.post is not None:
            ps += self.post.params()
        return ps

    def forward(self, x: Act, training: bool, tape: dict | None, ws: list | None):
        dt, dev = x.buf.dtype, x.buf.device
        N = x.N
        nh = lambda h, w, c: Act(K.nhwc(N, h, w, c, dt, dev))  # noqa: E731
        wp1, wp2, wp3 = self.c1.pack(dt, training), self.c2.pack(dt, training), self.c3.pack(dt, training)
        z1 = nh(x.H, x.W, self.c1.Cout)
        st1 = conv_bn_stats(self.c1, x, wp1, z1, self.bn1, training)
        a1 = nh(x.H, x.W, self.c1.Cout); K.bn_apply(z1, st1, ACT_RELU, a1)
        P, Q = self.c2.out_hw(x.H, x.W)
        z2 = nh(P, Q, self.c2.Cout)
        a2 = nh(P, Q, self.c2.Cout)
        if self.n2.kind == "bn":  # Norm.forward's BN branch with the conv-epilogue statistics
            st2 = conv_bn_stats(self.c2, a1, wp2, z2, self.n2.m, training)
            K.bn_apply(z2, st2, ACT_RELU, a2)
        else:
            self.c2.fwd(a1, wp2, z2)
            st2 = self.n2.forward(z2, a2, training, ACT_RELU)
        z3 = nh(P, Q, self.c3.Cout)
        st3 = conv_bn_stats(self.c3, a2, wp3, z3, self.bn3, training)
        wpd = zd = std = None
        if self.cd is not None:
            wpd = self.cd.pack(dt, training)
            zd = nh(P, Q, self.cd.Cout)
            std = conv_bn_stats(self.cd, x, wpd, zd, self.bnd, training)
        out = nh(P, Q, self.c3.Cout)
        s = sst = w = None
        if self.post is None:
            K.bn_add_apply(z3, st3, zd if zd is not None else x, std, ACT_RELU, out)
        else:
            s = nh(P, Q, self.c3.Cout)
            K.bn_add_apply(z3, st3, zd if zd is not None else x, std, ACT_NONE, s)
            if self.post.kind == "iw":
                w = nh(P, Q, self.c3.Cout)
                sst = self.post.forward(s, w, training, ACT_NONE)
                K.bn_apply(w, _identity_stats(w.C, dev), ACT_RELU, out)
                ws.append(w)
            else:
                sst = self.post.forward(s, out, training, ACT_RELU)
        if tape is not None:
            tape[self] = dict(x=x, wp=(wp1, wp2, wp3, wpd), z1=z1, st1=st1, a1=a1, z2=z2, st2=st2,
                              a2=a2, z3=z3, st3=st3, zd=zd, std=std, s=s, sst=sst, w=w, out=out)
        return out

    def backward(self, tape: dict, g_out: Act, grads: dict, g_w=None, g_masked=False, relu_x=False) -> Act:
        """g_out: dL/d(block output) (consumed / overwritten).  g_w(gt) -> None: adds the
        whitening-loss gradient dL/dw into gt (ISW).  Returns dL/dx.
        g_masked: g_out already carries the output ReLU's backward (the next block folded it
        into its conv1 dgrad); relu_x: x is the previous block's ReLU output, whose backward
        this block folds into its conv1 dgrad epilogue (the returned dL/dx is then masked)."""
        t = tape.pop(self)
        x, out = t["x"], t["out"]
        wp1, wp2, wp3, wpd = t["wp"]
        dev, dt = x.buf.device, x.buf.dtype
        if self.post is None:
            if not g_masked:
                K.relu_bwd(g_out, out, g_out)
            g_s = g_out
        else:
            s = t["s"]
            if self.post.kind == "iw":
                if not g_masked:
                    K.relu_bwd(g_out, out, g_out)
                if g_w is not None:
                    g_w(g_out)
                g_s = Act(torch.empty_like(s.buf))
                self.post.backward(g_out, s, t["w"], t["sst"], ACT_NONE, g_s, grads)
            else:
                g_s = Act(torch.empty_like(s.buf))
                self.post.backward(g_out, s, out, t["sst"], ACT_RELU, g_s, grads)
        g_z3 = Act(torch.empty_like(t["z3"].buf))
        bn_backward(self.bn3, g_s, t["z3"], t["st3"], ACT_NONE, g_z3, grads)
        if self.cd is not None:
            g_zd = Act(torch.empty_like(t["zd"].buf))
            bn_backward(self.bnd, g_s, t["zd"], t["std"], ACT_NONE, g_zd, grads)
            gx = Act(K.nhwc(x.N, x.H, x.W, x.C, dt, dev))
            _acc(grads, self.cd.conv.weight, self.cd.bwd(x, g_zd, wpd, gx))
        else:
            gx = g_s  # identity shortcut: conv1's dgrad accumulates into it
        g_a2 = Act(torch.empty_like(t["a2"].buf))
        _acc(grads, self.c3.conv.weight, self.c3.bwd(t["a2"], g_z3, wp3, g_a2))
        g_z2 = Act(torch.empty_like(t["z2"].buf))
        self.n2.backward(g_a2, t["z2"], t["a2"], t["st2"], ACT_RELU, g_z2, grads)
        g_a1 = Act(torch.empty_like(t["a1"].buf))
        _acc(grads, self.c2.conv.weight, self.c2.bwd(t["a1"], g_z2, wp2, g_a1))
        g_z1 = Act(torch.empty_like(t["z1"].buf))
        bn_backward(self.bn1, g_a1, t["z1"], t["st1"], ACT_RELU, g_z1, grads)
        if relu_x:
            _acc(grads, self.c1.conv.weight, self.c1.bwd(x, g_z1, wp1, gx, accumulate=True, relu_out=x))
        else:
            _acc(grads, self.c1.conv.weight, self.c1.bwd(x, g_z1, wp1, gx, accumulate=True))
        return gx


class CounterPlan:
    """conv1 7x7/2 (im2col GEMM) + stem norm + ReLU + maxpool 3x3/2/1 + layer1..3 +
    counter head (3x3 1024->512 +ReLU, 3x3 512->256 +ReLU, 1x1 ->1, bilinear x16
    align_corners=True): img [N,3,H,W] -> [N,1,H,W] f32 (models/ibnnet/__init__.py:11-29,
    models/SW/__init__.py:24-42, models/ISW/__init__.py:21-91).

    ISW: `iw_masks` = [(mask [C,C], num_sensitive (device scalar))] per whitened map turns
    on the instance-whitening loss (ISW/__init__.py:112-118); it is the second output."""

    def __init__(self, conv1: nn.Conv2d, stem_norm: Norm, blocks: list[Block], head: nn.Sequential):
        self.conv1 = conv1
        self.stem = stem_norm
        self.blocks = blocks
        self.h0 = ConvLayer(head[0], None, ACT_RELU)
        self.h1 = ConvLayer(head[2], None, ACT_RELU)
        self.hw, self.hb = head[4].weight, head[4].bias
        self.nondiff = ()

    def params(self):
        ps = [self.conv1.weight] + self.stem.params()
        for b in self.blocks:
            ps += b.params()
        return ps + self.h0.params() + self.h1.params() + [self.hw, self.hb]

    # ---- forward -----------------------------------------------------------
    def features(self, img: torch.Tensor, dt, training: bool, tape: dict | None):
        """img [N,3,H,W] -> layer3 output (NHWC Act) and the whitened maps (ISW)."""
        N, _, H, W = img.shape
        if H % 16 or W % 16:
            raise ValueError(f"input H,W must be multiples of 16 (got {H}x{W})")
        dev = img.device
        imgf = img.float().contiguous()
        col = Act(K.im2col_c3_general(imgf, dt, 7, 2, 3, STEM_KPAD))
        if dt == torch.float32:  # the columns hold image values and zeros: the image channels' maxima bound them
            col.amax = _stem_col_amax(imgf, STEM_KPAD)
        build = lambda: K.pack_weight(self.conv1.weight.detach(), dt, cpad=3, row_len=STEM_KPAD)  # noqa: E731
        wp0 = build() if training else frozen(self, ("stem", dt), (self.conv1.weight,), build)
        P, Q = col.H, col.W
        z0 = Act(K.nhwc(N, P, Q, 64, dt, dev))
        K.conv_fwd(col, wp0, 64, 1, 0, z0, k_alg=147)
        ws = []
        y0 = Act(K.nhwc(N, P, Q, 64, dt, dev))
        if self.stem.kind == "iw":
            w0 = Act(K.nhwc(N, P, Q, 64, dt, dev))
            st0 = self.stem.forward(z0, w0, training, ACT_NONE)
            K.bn_apply(w0, _identity_stats(64, dev), ACT_RELU, y0)
            ws.append(w0)
        else:
            w0 = None
            st0 = self.stem.forward(z0, y0, training, ACT_RELU)
        Pm, Qm = K.conv_out(P, 3, 2, 1), K.conv_out(Q, 3, 2, 1)
        x = Act(K.nhwc(N, Pm, Qm, 64, dt, dev))
        pidx = K.maxpool_k_fwd_idx(y0, 3, 2, 1, x)
        for b in self.blocks:
            x = b.forward(x, training, tape, ws)
        if tape is not None:
            tape[self] = dict(col=col, z0=z0, st0=st0, y0=y0, w0=w0, pidx=pidx, shape=(N, H, W), dt=dt)
        return x, ws

    def head_fwd(self, x: Act, training: bool, tape: dict | None):
        N, h, w = x.N, x.H, x.W
        dt, dev = x.buf.dtype, x.buf.device
        a = Act(K.nhwc(N, h, w, 512, dt, dev)); self.h0.forward(x, a, training, tape)
        b = Act(K.nhwc(N, h, w, 256, dt, dev)); self.h1.forward(a, b, training, tape)
        yh = K.head_fwd(b, self.hw.detach().reshape(-1), self.hb.detach(), K.ACT_NONE)
        out = torch.empty((N, 16 * h, 16 * w, 1), dtype=torch.float32, device=dev)
        K.upsample_fwd(Act(yh.view(N, h, w, 1)), 16, K.UP_BILINEAR_AC, Act(out))
        if tape is not None:
            tape["head"] = (b, yh)
        return out.view(N, 1, 16 * h, 16 * w)

    def forward(self, img, training: bool, iw_masks=None, tape: dict | None = None, dt=None):
        x, ws = self.features(img, dt, training, tape)
        out = self.head_fwd(x, training, tape)
        if iw_masks is None:
            return out
        wt = torch.zeros((), dtype=torch.float32, device=img.device)
        frs = []
        for w, (mask, ns) in zip(ws, iw_masks):
            fr = gram(w)
            K.iw_loss(fr, w.H * w.W, mask, ns, 1.0 / len(ws), wt, accumulate=True, want_grad=False)
            frs.append(fr)
        if tape is not None:
            tape["iw"] = (ws, frs, iw_masks)
        return out, wt

    # ---- backward ----------------------------------------------------------
    def backward(self, tape: dict, g_out, g_wt=None):
        s = tape.pop(self)
        N, H, W = s["shape"]
        dt = s["dt"]
        grads = {}
        b, yh = tape.pop("head")
        h, w = b.H, b.W
        dev = yh.device
        g_h = torch.empty((N, h, w, 1), dtype=torch.float32, device=dev)
        K.upsample_bwd(Act(g_out.contiguous().view(N, 16 * h, 16 * w, 1)), 16, K.UP_BILINEAR_AC,
                       Act(g_h))
        g_b = Act(torch.empty_like(b.buf))
        gw = torch.empty(256, dtype=torch.float32, device=dev)
        gb = torch.empty(1, dtype=torch.float32, device=dev)
        K.head_bwd(b, self.hw.detach().reshape(-1), K.ACT_NONE, yh, g_h.view(N, h, w), g_b, gw, gb)
        grads[self.hw] = gw.view_as(self.hw)
        grads[self.hb] = gb
        g_a = Act(K.nhwc(N, h, w, 512, dt, dev))
        for p, g in self.h1.backward(tape, g_b, g_a).items():
            _acc(grads, p, g)
        g_x = Act(K.nhwc(N, h, w, 1024, dt, dev))
        for p, g in self.h0.backward(tape, g_a, g_x).items():
            _acc(grads, p, g)
        # whitening-loss gradients, applied where each w's gradient is formed
        iw = tape.pop("iw", None)
        hooks = {}
        if iw is not None and g_wt is not None:
            ws, frs, masks = iw
            for w_, fr, (mask, ns) in zip(ws, frs, masks):
                hooks[id(w_)] = _iw_grad_hook(w_, fr, mask, ns, 1.0 / len(ws), g_wt)
        masked = False
        for k in reversed(range(len(self.blocks))):
            blk = self.blocks[k]
            wkey = None
            if blk.post is not None and blk.post.kind == "iw":
                wkey = id(tape[blk]["w"])
            # the previous block's output ReLU backward folded into this block's conv1 dgrad
            # (its x is that output); IN-post blocks recompute the mask in their IN backward
            prev = self.blocks[k - 1] if k > 0 else None
            fold = _RELU_FOLD and prev is not None and (prev.post is None or prev.post.kind == "iw")
            g_x = blk.backward(tape, g_x, grads, hooks.get(wkey), g_masked=masked, relu_x=fold)
            masked = fold
        # maxpool, stem
        y0 = s["y0"]
        g_y0 = Act(torch.empty_like(y0.buf))
        K.maxpool_k_bwd_idx(s["pidx"], g_x, 3, 2, 1, g_y0)
        g_z0 = Act(torch.empty_like(s["z0"].buf))
        if self.stem.kind == "iw":
            w0 = s["w0"]
            K.relu_bwd(g_y0, y0, g_y0)
            if id(w0) in hooks:
                hooks[id(w0)](g_y0)
            self.stem.backward(g_y0, s["z0"], w0, s["st0"], ACT_NONE, g_z0, grads)
        else:
            self.stem.backward(g_y0, s["z0"], y0, s["st0"], ACT_RELU, g_z0, grads)
        dwcol = torch.empty((64, STEM_KPAD, 1, 1), dtype=torch.float32, device=dev)
        K.conv_wgrad(s["col"], g_z0, 1, 0, dwcol, k_alg=147)
        dw = torch.empty_like(self.conv1.weight, dtype=torch.float32)
        K.unpack_c3(dwcol.view(64, STEM_KPAD), dw)
        _acc(grads, self.conv1.weight, dw)
        return (None,), grads


def gram(w: Act) -> torch.Tensor:
    """Per-instance raw Gram matrices sum_p w_p w_p^T -> [N, C, C] f32 (one 1x1
    wgrad GEMM per instance: MFMA, K = H*W)."""
    N, C = w.N, w.C
    fr = torch.empty((N, C, C), dtype=torch.float32, device=w.buf.device)
    am = _whole_amax(w)
    for n in range(N):
        wn = Act(w.buf[n:n + 1], w.off, w.C, am)
        K.conv_wgrad(wn, wn, 1, 0, fr[n].view(C, C, 1, 1))
    return fr


def _stem_col_amax(imgf: torch.Tensor, kpad: int) -> torch.Tensor:
    """Operand maxima of the stem's im2col columns (dg_im2col_c3: column k < 3RS holds image channel
    k % 3, the rest zeros) from the image's per-channel maxima: [kernels.amax_words(kpad)] floats."""
    cm = imgf.abs().amax(dim=(0, 2, 3))  # [3]
    rs3 = 3 * 7 * 7
    out = torch.zeros(K.amax_words(kpad), dtype=torch.float32, device=imgf.device)
    out[0] = cm.max()
    out[1:1 + rs3] = cm.repeat(rs3 // 3)
    return out


def _whole_amax(w: Act):
    """f32: max |w| over the whole map (its producer's, else one pass), the f16 x3 operand bound
    every per-instance launch over w shares; None for 16-bit maps."""
    if w.buf.dtype != torch.float32:
        return None
    if w.amax is None:
        w.amax = K.amax(w)
    return w.amax


def _iw_grad_hook(w: Act, fr, mask, ns, scale, g_wt):
    """gt += dL_wt/dw: gsym = d loss/d fraw (symmetrised, / (HW-1)), then one 1x1
    conv per instance (w_n @ gsym_n) accumulated into gt."""
    def apply(gt: Act):
        gt.amax = None  # accumulated into below through per-instance views
        gsym = K.iw_loss(fr, w.H * w.W, mask, ns, scale, None, accumulate=False, want_grad=True,
                         grad_coef=g_wt)
        N, C = w.N, w.C
        wp = K.pack_weight(gsym.view(N * C, C, 1, 1), w.buf.dtype)
        am = _whole_amax(w)
        for n in range(N):
            K.conv_fwd(Act(w.buf[n:n + 1], w.off, C, am), wp[n * C:(n + 1) * C], C, 1, 0,
                       Act(gt.buf[n:n + 1], gt.off, C), accumulate=True, kind="iw")
    return apply
