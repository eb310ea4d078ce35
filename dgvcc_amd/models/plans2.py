"""HIP plans for the models2 classes whose heads are not the DGModel_* ones
(reference models/models2.py): sequential ConvBlock chains with Dropout2d / pooling /
upsampling and a small C->k terminal conv (+ Sigmoid / Tanh), and the VGG19 U-Net of
Generator0.  Every op is a HIP launch (engine.ConvLayer / CatConvLayer, the resample, head
and tanh kernels); NHWC activations; each chain is one torch.autograd.Function whose
backward is the reversed launch sequence.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import engine as E
from .. import kernels as K
from ..kernels import Act
from .models import ConvBlock


class ChainPlan:
    """A module sequence (nn.Sequential contents) run as NHWC HIP launches.

    Parsing: ConvBlock / (Conv2d [+ ReLU]) -> engine.ConvLayer, with a following Dropout2d
    as its channel mask (F.dropout2d order: act, then mask); MaxPool2d(2) and bilinear
    Upsample(x2); a final 1x1 ConvBlock with <= 4 output channels and no BN is the terminal
    head (one dg_head_fwd per output channel, ReLU / Sigmoid / none) and a trailing nn.Tanh
    runs dg_tanh_fwd on it.  cat_input: the first op is the 1x1 conv on the decoder
    concatenation parts (engine.CatConvLayer); image_input: the first conv reads the NCHW f32
    image through the Cin=3 im2col (engine.ConvLayer first=True)."""

    def __init__(self, modules, cat_input: bool = False, image_input: bool = False):
        mods = list(modules)
        self.cat_input, self.image_input = cat_input, image_input
        self.ops = []
        self._params = []
        for i, m in enumerate(mods):
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            rest_has_conv = any(isinstance(x, (ConvBlock, nn.Conv2d)) for x in mods[i + 1:])
            if isinstance(m, ConvBlock):
                conv, bn = m.conv, m.bn
                if (not rest_has_conv and conv.kernel_size == (1, 1) and conv.out_channels <= 4 and bn is None
                        and self.ops):
                    act = K.ACT_RELU if m.relu is not None else K.ACT_NONE
                    if isinstance(nxt, nn.Sigmoid):
                        if m.relu is not None:
                            raise ValueError("ChainPlan: ReLU followed by Sigmoid is not a supported head")
                        act = K.ACT_SIGMOID
                    self.ops.append(["head", conv, act, isinstance(nxt, nn.Tanh)])
                    self._params += [conv.weight] + ([conv.bias] if conv.bias is not None else [])
                    continue
                act = E.ACT_RELU if m.relu is not None else E.ACT_NONE
                self._conv(conv, bn, act, nxt)
            elif isinstance(m, nn.Conv2d):
                self._conv(m, None, E.ACT_RELU if isinstance(nxt, nn.ReLU) else E.ACT_NONE, None)
            elif isinstance(m, nn.MaxPool2d):
                if m.kernel_size not in (2, (2, 2)) or m.stride not in (2, (2, 2)):
                    raise ValueError("ChainPlan: only MaxPool2d(2, 2)")
                self.ops.append(["pool"])
            elif isinstance(m, nn.Upsample):
                if m.mode != "bilinear" or m.align_corners:
                    raise ValueError("ChainPlan: only bilinear align_corners=False upsampling")
                self.ops.append(["up", int(m.scale_factor)])
            elif isinstance(m, (nn.ReLU, nn.Dropout2d, nn.Sigmoid, nn.Tanh)):
                continue  # consumed by the op before (checked there)
            else:
                raise ValueError(f"ChainPlan: unsupported module {type(m).__name__}")
            if isinstance(m, (nn.Sigmoid, nn.Tanh)) and (not self.ops or self.ops[-1][0] != "head"):
                raise ValueError("ChainPlan: Sigmoid/Tanh only after the terminal head")

    def _conv(self, conv, bn, act, nxt):
        first = not self.ops
        if first and self.cat_input:
            layer = E.CatConvLayer(conv, bn, act)
        else:
            layer = E.ConvLayer(conv, bn, act, first=first and self.image_input)
        p = nxt.p if isinstance(nxt, nn.Dropout2d) else 0.0
        self.ops.append(["conv", layer, p])
        self._params += layer.params()

    def params(self):
        return self._params

    # ----------------------------------------------------------------- forward --
    def run(self, x, dt, training: bool, tape: dict | None, out: Act | None = None):
        """x: NCHW image (image_input), CatParts (cat_input) or an NHWC Act.  out: where the
        last conv op writes (a channel slice of a concatenation buffer), if given.
        Returns the last op's output: an Act, or the head's f32 [N,k,H,W] tensor."""
        if self.image_input:
            x = Act(K.im2col_c3(x.float().contiguous(), dt))
        rec = []
        nops = len(self.ops)
        for i, op in enumerate(self.ops):
            kind = op[0]
            if kind == "conv":
                layer, p = op[1], op[2]
                N, H, W = x.N, x.H, x.W
                dev = x.parts[0].buf.device if isinstance(x, E.CatParts) else x.buf.device
                y = out if (out is not None and i == nops - 1) else Act(K.nhwc(N, H, W, layer.Cout, dt, dev))
                drop = E.dropout2d_mask(N, layer.Cout, p, dev) if (training and p > 0) else None
                layer.forward(x, y, training, tape, drop=drop)
                rec.append((x, y))
            elif kind == "pool":
                y = Act(K.nhwc(x.N, x.H // 2, x.W // 2, x.C, x.buf.dtype, x.buf.device))
                K.maxpool_fwd(x, y)
                rec.append((x, y))
            elif kind == "up":
                s = op[1]
                y = Act(K.nhwc(x.N, x.H * s, x.W * s, x.C, x.buf.dtype, x.buf.device))
                K.upsample_fwd(x, s, K.UP_BILINEAR, y)
                rec.append((x, y))
            else:  # head
                conv, act, tanh = op[1], op[2], op[3]
                w = conv.weight.detach()
                ys = [K.head_fwd(x, w[k].reshape(-1).contiguous(),
                                 conv.bias.detach()[k:k + 1] if conv.bias is not None else None, act)
                      for k in range(conv.out_channels)]
                y = torch.stack(ys, 1)  # [N, k, H, W] f32 (plane per output channel)
                if tanh:
                    t = torch.empty_like(y)
                    K.call("dg_tanh_fwd", K.ptr(y), y.numel(), K.ptr(t), K.stream())
                    y = t
                rec.append((x, ys, y))
            x = y
        if tape is not None:
            tape[self] = rec
        return y

    # ---------------------------------------------------------------- backward --
    def back(self, tape: dict, g, gx=None, accumulate: bool = False) -> dict:
        """g: gradient of the last op's output (Act, or f32 [N,k,H,W] for a head).  gx: where
        the input gradient goes (Act / CatParts; allocated when None and the input needs
        one); returns ({param: grad}, input gradient)."""
        rec = tape.pop(self)
        grads = {}
        nops = len(self.ops)
        for i in range(nops - 1, -1, -1):
            op, r = self.ops[i], rec[i]
            x = r[0]
            last = i == 0
            if last and self.image_input:
                tgt = None
            elif last and gx is not None:
                tgt = gx
            elif isinstance(x, E.CatParts):
                tgt = x.empty_like()
            else:
                tgt = Act(torch.empty_like(x.buf))
            acc = accumulate and last and gx is not None
            kind = op[0]
            if kind == "conv":
                for p, gp in op[1].backward(tape, g, tgt, accumulate_gx=acc).items():
                    E._acc(grads, p, gp)
            elif kind == "pool":
                K.maxpool_bwd(x, g, tgt, accumulate=acc)
            elif kind == "up":
                K.upsample_bwd(g, op[1], K.UP_BILINEAR, tgt, accumulate=acc)
            else:
                conv, act, tanh = op[1], op[2], op[3]
                ys, y = r[1], r[2]
                g = g.float().contiguous()
                if tanh:
                    gpre = torch.empty_like(g)
                    K.call("dg_tanh_bwd", K.ptr(y), K.ptr(g), g.numel(), K.ptr(gpre), 0, K.stream())
                    g = gpre
                w = conv.weight.detach()
                gw = torch.empty((conv.out_channels, x.C), dtype=torch.float32, device=g.device)
                gb = torch.empty(conv.out_channels, dtype=torch.float32, device=g.device) \
                    if conv.bias is not None else None
                for k in range(conv.out_channels):
                    K.head_bwd(x, w[k].reshape(-1).contiguous(), act, ys[k], g[:, k].contiguous(), tgt, gw[k],
                               gb[k:k + 1] if gb is not None else None, accumulate_gx=(k > 0 or acc))
                E._acc(grads, conv.weight, gw.view_as(conv.weight))
                if gb is not None:
                    E._acc(grads, conv.bias, gb)
            g = tgt
        return grads, g

    # ---------------------------------------------- as a standalone autograd plan --
    def forward(self, inputs, dt, training, tape=None):
        if self.cat_input:
            x = E.as_cat(inputs)
        elif self.image_input:
            x = inputs[0]
        else:
            x = Act(inputs[0])
        y = self.run(x, dt, training, tape)
        return y.buf if isinstance(y, Act) else y

    def backward(self, tape, g):
        if not isinstance(g, Act) and self.ops[-1][0] != "head":
            g = Act(g.contiguous())
        grads, gin = self.back(tape, g)
        if gin is None:
            return (), grads
        if isinstance(gin, E.CatParts):
            return gin.tensors(), grads
        return (gin.buf,), grads


def run_chain(plan: ChainPlan, inputs, training: bool, dt: torch.dtype):
    """Run `plan` on NHWC tensors (or the NCHW image) under autograd."""
    return E.run_plan(plan, lambda *xs, tape: plan.forward(xs, dt, training, tape), tuple(inputs), plan.params())


class _MaskUp4(torch.autograd.Function):
    """dc = up4_bilinear(d * up4_nearest(c_gt if given else (c >= thr))) (models2.py:176-185,
    307-316, 500-509): the class map is a constant (thresholded copy / ground truth)."""

    @staticmethod
    def forward(ctx, d, c, c_gt, thr):
        N, _, h, w = d.shape
        cres = torch.empty((N, h, w), dtype=torch.float32, device=d.device)
        cg = c_gt.float().contiguous() if c_gt is not None else None
        K.call("dg_cls_combine", K.ptr(c.detach().contiguous()), None, K.ptr(cg), N, h // 4, w // 4, 4, float(thr),
               K.ptr(cres), None, K.stream())
        prod = torch.empty_like(cres)
        K.call("dg_mul_f32", K.ptr(d.detach().contiguous()), K.ptr(cres), cres.numel(), K.ptr(prod), K.stream())
        ctx.save_for_backward(cres)
        return E._up4(prod, N, h, w)

    @staticmethod
    def backward(ctx, g):
        (cres,) = ctx.saved_tensors
        N, h, w = cres.shape
        gs = E._up4_bwd(g, N, h, w)
        K.call("dg_mul_f32", K.ptr(gs), K.ptr(cres), gs.numel(), K.ptr(gs), K.stream())
        return gs.view(N, 1, h, w), None, None, None


def masked_up4(d, c, c_gt, thr):
    return _MaskUp4.apply(d, c, c_gt, thr)


class UNetPlan:
    """Generator0 (models/models2.py:58-103): VGG19 enc1/enc2/enc3, dec3 -> up2 -> cat[., x2]
    -> dec2 -> up2 -> cat[., x1] -> dec1 -> up2 -> head (64->64 BN, 64->3, Tanh).  The skip
    features are written by their producers into channel slices of the concatenation
    buffers (as engine.FeaturePlan)."""

    def __init__(self, model):
        self.enc1 = ChainPlan(model.enc1, image_input=True)
        self.enc2 = ChainPlan(model.enc2)
        self.enc3 = ChainPlan(model.enc3)
        self.dec3 = ChainPlan(model.dec3)
        self.dec2 = ChainPlan(model.dec2)
        self.dec1 = ChainPlan(model.dec1)
        self.head = ChainPlan(model.head)
        self.chains = [self.enc1, self.enc2, self.enc3, self.dec3, self.dec2, self.dec1, self.head]

    def params(self):
        return [p for c in self.chains for p in c.params()]

    def forward(self, img, dt, training, tape=None):
        N, _, H, W = img.shape
        if H % 8 or W % 8:
            raise ValueError(f"Generator0: H, W must be multiples of 8 (got {H}x{W})")
        dev = img.device
        dec1in = K.nhwc(N, H // 2, W // 2, 256, dt, dev)
        dec2in = K.nhwc(N, H // 4, W // 4, 512, dt, dev)
        x1 = Act(dec1in, 128, 128)
        x2 = Act(dec2in, 256, 256)
        self.enc1.run(img, dt, training, tape, out=x1)
        self.enc2.run(x1, dt, training, tape, out=x2)
        x3 = self.enc3.run(x2, dt, training, tape)
        y3 = self.dec3.run(x3, dt, training, tape)
        K.upsample_fwd(y3, 2, K.UP_BILINEAR, Act(dec2in, 0, 256))
        y2 = self.dec2.run(Act(dec2in), dt, training, tape)
        K.upsample_fwd(y2, 2, K.UP_BILINEAR, Act(dec1in, 0, 128))
        y1 = self.dec1.run(Act(dec1in), dt, training, tape)
        u = Act(K.nhwc(N, H, W, 64, dt, dev))
        K.upsample_fwd(y1, 2, K.UP_BILINEAR, u)
        out = self.head.run(u, dt, training, tape)
        if tape is not None:
            tape[self] = dict(dec1in=dec1in, dec2in=dec2in, y1=y1, y2=y2, y3=y3, u=u, x1=x1, x2=x2, x3=x3)
        return out

    def backward(self, tape, g):
        s = tape.pop(self)
        grads = {}

        def upd(gr):
            for p, gp in gr.items():
                E._acc(grads, p, gp)

        gr, g_u = self.head.back(tape, g)
        upd(gr)
        y1 = s["y1"]
        g_y1 = Act(torch.empty_like(y1.buf))
        K.upsample_bwd(g_u, 2, K.UP_BILINEAR, g_y1)
        g_dec1in = Act(torch.empty_like(s["dec1in"]))
        gr, _ = self.dec1.back(tape, g_y1, g_dec1in)
        upd(gr)
        y2 = s["y2"]
        g_y2 = Act(torch.empty_like(y2.buf))
        K.upsample_bwd(Act(g_dec1in.buf, 0, 128), 2, K.UP_BILINEAR, g_y2)
        g_dec2in = Act(torch.empty_like(s["dec2in"]))
        gr, _ = self.dec2.back(tape, g_y2, g_dec2in)
        upd(gr)
        y3 = s["y3"]
        g_y3 = Act(torch.empty_like(y3.buf))
        K.upsample_bwd(Act(g_dec2in.buf, 0, 256), 2, K.UP_BILINEAR, g_y3)
        gr, g_x3 = self.dec3.back(tape, g_y3)
        upd(gr)
        g_x2 = Act(g_dec2in.buf, 256, 256)             # skip gradient, plus enc3's input gradient
        gr, _ = self.enc3.back(tape, g_x3, g_x2, accumulate=True)
        upd(gr)
        g_x1 = Act(g_dec1in.buf, 128, 128)
        gr, _ = self.enc2.back(tape, g_x2, g_x1, accumulate=True)
        upd(gr)
        gr, _ = self.enc1.back(tape, g_x1)
        upd(gr)
        return (), grads


def run_unet(plan: UNetPlan, img, training: bool, dt: torch.dtype):
    return E.run_plan(plan, lambda x, tape: plan.forward(x, dt, training, tape), (img,), plan.params())
