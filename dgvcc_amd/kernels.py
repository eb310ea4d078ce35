"""Host wrappers over the C-ABI: torch tensors in, kernel launches out.

Activations are channel slices of NHWC buffers (`Act`): a pointer offset plus
the buffer's pixel stride, so the decoder's torch.cat (models/models.py:72,76,84)
becomes "write into a channel slice" with no copy.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ._capi import DGError, call, dtype_code, ptr, query, stream

F32, BF16 = 0, 1


@dataclass
class Act:
    """Channel slice [off, off+C) of an NHWC buffer `buf` [N,H,W,Ctot]."""
    buf: torch.Tensor
    off: int = 0
    C: int | None = None

    def __post_init__(self):
        if self.buf.dim() != 4:
            raise DGError("Act expects an NHWC 4-D buffer")
        if self.C is None:
            self.C = self.buf.shape[3] - self.off

    @property
    def N(self):
        return self.buf.shape[0]

    @property
    def H(self):
        return self.buf.shape[1]

    @property
    def W(self):
        return self.buf.shape[2]

    @property
    def ld(self):
        return self.buf.shape[3]

    @property
    def M(self):
        return self.N * self.H * self.W

    @property
    def ptr(self):
        return self.buf.data_ptr() + self.off * self.buf.element_size()

    @property
    def dt(self):
        return dtype_code(self.buf.dtype)

    def view(self) -> torch.Tensor:
        return self.buf[..., self.off:self.off + self.C]


def nhwc(N, H, W, C, dtype, device="cuda", zero=False) -> torch.Tensor:
    f = torch.zeros if zero else torch.empty
    return f((N, H, W, C), dtype=dtype, device=device)


# ---------------------------------------------------------------- conv -----
_CONV_TIMER = None


def set_conv_timer(timer):
    """Install a callable timer(kind, flops, launch_fn) around conv GEMM launches
    (bench.py roofline measurement); None disables."""
    global _CONV_TIMER
    _CONV_TIMER = timer


def _timed(kind, flops, fn, nbytes=0.0):
    if _CONV_TIMER is None:
        fn()
    else:
        _CONV_TIMER(kind, flops, fn, nbytes)

def pack_weight(w: torch.Tensor, dtype: torch.dtype, cpad: int | None = None,
                row_len: int | None = None) -> torch.Tensor:
    Cout, C, R, S = w.shape
    cpad = cpad or C
    row_len = row_len or R * S * cpad
    out = torch.empty((Cout, row_len), dtype=dtype, device=w.device)
    call("dg_pack_weight", dtype_code(dtype), ptr(w.contiguous()), Cout, C, R, S, cpad, row_len,
         ptr(out), stream())
    return out


def conv_fwd(x: Act, wp: torch.Tensor, Cout: int, R: int, pad: int, y: Act,
             bias: torch.Tensor | None = None, accumulate=False, kind="fwd", k_alg=None):
    """k_alg: algorithmic reduction length when the GEMM K is padded (im2col layer)."""
    flops = 2.0 * x.M * (k_alg if k_alg else x.C * R * R) * Cout
    es = x.buf.element_size()
    nbytes = es * (x.M * x.C + wp.numel() + x.M * Cout * (2 if accumulate else 1))  # x, w, y (+y read)
    _timed(kind, flops, lambda: call("dg_conv_fwd", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, ptr(wp),
                                     Cout, R, R, pad, ptr(bias), y.ptr, y.ld, int(accumulate),
                                     stream()), nbytes)


def flip_weight(wp: torch.Tensor, Cout: int, C: int, R: int) -> torch.Tensor:
    wflip = torch.empty_like(wp)
    call("dg_flip_weight", dtype_code(wp.dtype), ptr(wp), Cout, C, R, R, ptr(wflip), stream())
    return wflip


def conv_dgrad(dy: Act, wp: torch.Tensor, C: int, R: int, pad: int, dx: Act, accumulate=False):
    """dX = conv(dY, flipped W^T): the forward GEMM kernel on the flipped filter."""
    wflip = flip_weight(wp, dy.C, C, R)
    conv_fwd(dy, wflip, C, R, R - 1 - pad, dx, accumulate=accumulate, kind="dgrad")


def conv_wgrad(x: Act, dy: Act, R: int, pad: int, dw: torch.Tensor, accumulate=False, k_alg=None):
    ws = query("dg_conv_wgrad_workspace", x.dt, x.N, x.H, x.W, x.C, dy.C, R, R)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=x.buf.device)
    flops = 2.0 * x.M * (k_alg if k_alg else x.C * R * R) * dy.C
    nbytes = x.buf.element_size() * (x.M * x.C + dy.M * dy.C) + 4 * dw.numel()
    _timed("wgrad", flops, lambda: call("dg_conv_wgrad", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C,
                                        dy.ptr, dy.ld, dy.C, R, R, pad, ptr(dw), ptr(work), ws,
                                        int(accumulate), stream()), nbytes)


def im2col_c3(img: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    N, _, H, W = img.shape
    out = torch.empty((N, H, W, 64), dtype=dtype, device=img.device)
    call("dg_im2col3x3_c3", dtype_code(dtype), ptr(img.contiguous()), N, H, W, ptr(out), stream())
    return out


def unpack_c3_grad(dwcol: torch.Tensor, dw: torch.Tensor, accumulate=False):
    call("dg_unpack_c3_grad", ptr(dwcol), dw.shape[0], ptr(dw), int(accumulate), stream())


# ---------------------------------------------------------------- BN -------
def bn_fwd_train(z: Act, gamma, beta, running_mean, running_var, momentum, eps):
    C = z.C
    dev = z.buf.device
    stats = torch.empty((4, C), dtype=torch.float32, device=dev)  # mean, invstd, scale, shift
    ws = query("dg_bn_workspace", z.M, C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=dev)
    call("dg_bn_fwd_train", z.dt, z.ptr, z.ld, z.M, C, ptr(gamma), ptr(beta), ptr(running_mean),
         ptr(running_var), float(momentum), float(eps), ptr(stats[0]), ptr(stats[1]),
         ptr(stats[2]), ptr(stats[3]), ptr(work), stream())
    return stats


def bn_eval_stats(gamma, beta, running_mean, running_var, eps):
    """scale/shift from running statistics (eval mode) — tiny [C] host-side math."""
    invstd = torch.rsqrt(running_var + eps)
    scale = gamma * invstd
    shift = beta - running_mean * scale
    return torch.stack([running_mean, invstd, scale, shift])


def bn_apply(z: Act, stats, act: int, y: Act, drop: torch.Tensor | None = None):
    call("dg_bn_apply", z.dt, z.ptr, z.ld, z.M, z.C, ptr(stats[2]), ptr(stats[3]), act, ptr(drop),
         z.H * z.W, y.ptr, y.ld, stream())


def bn_bwd(g: Act, z: Act, gamma, stats, act: int, dz: Act, dgamma, dbeta, dbias=None,
           drop: torch.Tensor | None = None):
    ws = query("dg_bn_workspace", z.M, z.C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=z.buf.device)
    call("dg_bn_bwd", z.dt, g.ptr, g.ld, z.ptr, z.ld, z.M, z.C, ptr(gamma), ptr(stats[0]),
         ptr(stats[1]), ptr(stats[2]), ptr(stats[3]), act, ptr(drop), z.H * z.W, dz.ptr, dz.ld,
         ptr(dgamma), ptr(dbeta), ptr(dbias), ptr(work), stream())


# ---------------------------------------------------------------- resample -
def maxpool_fwd(x: Act, y: Act):
    call("dg_maxpool2_fwd", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, y.ptr, y.ld, stream())


def maxpool_bwd(x: Act, gy: Act, gx: Act, accumulate=False):
    call("dg_maxpool2_bwd", x.dt, x.ptr, x.ld, gy.ptr, gy.ld, x.N, x.H, x.W, x.C, gx.ptr, gx.ld,
         int(accumulate), stream())


UP_BILINEAR, UP_BILINEAR_AC, UP_NEAREST = 0, 1, 2


def upsample_fwd(x: Act, scale: int, mode: int, y: Act):
    call("dg_upsample_fwd", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, scale, mode, y.ptr, y.ld, stream())


def upsample_bwd(gy: Act, scale: int, mode: int, gx: Act, gy2: Act | None = None, accumulate=False):
    call("dg_upsample_bwd", gx.dt, gy.ptr, gy.ld, gy2.ptr if gy2 is not None else None,
         gy2.ld if gy2 is not None else 0, gx.N, gx.H, gx.W, gx.C, scale, mode, gx.ptr, gx.ld,
         int(accumulate), stream())


# ---------------------------------------------------------------- head -----
ACT_NONE, ACT_RELU, ACT_SIGMOID = 0, 1, 2


def head_fwd(x: Act, w: torch.Tensor, bias: torch.Tensor | None, act: int) -> torch.Tensor:
    y = torch.empty((x.N, x.H, x.W), dtype=torch.float32, device=x.buf.device)
    call("dg_head_fwd", x.dt, x.ptr, x.ld, x.M, x.C, ptr(w), ptr(bias), act, ptr(y), stream())
    return y


def head_bwd(x: Act, w, act, y, gy, gx: Act | None, gw, gbias=None, accumulate_gx=False):
    ws = query("dg_head_workspace", x.M, x.C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=x.buf.device)
    call("dg_head_bwd", x.dt, x.ptr, x.ld, x.M, x.C, ptr(w), act, ptr(y), ptr(gy),
         gx.ptr if gx is not None else None, gx.ld if gx is not None else 0, int(accumulate_gx),
         ptr(gw), ptr(gbias), ptr(work), stream())


# ---------------------------------------------------------------- loss/opt -
def mse_loss(pred: torch.Tensor, gt: torch.Tensor, gt_scale: float, want_grad=True, grad_coef=1.0):
    n = pred.numel()
    loss = torch.empty((), dtype=torch.float32, device=pred.device)
    dpred = torch.empty_like(pred) if want_grad else None
    ws = query("dg_reduce_workspace", n)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=pred.device)
    call("dg_mse_loss", ptr(pred.contiguous()), ptr(gt.contiguous()), float(gt_scale), n, ptr(loss),
         ptr(dpred), float(grad_coef), ptr(work), stream())
    return loss, dpred


def adamw_step(p, g, m, v, lr, beta1, beta2, eps, wd, step):
    call("dg_adamw_step", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), float(lr), float(beta1),
         float(beta2), float(eps), float(wd), int(step), stream())


def dmap_fixed(points: torch.Tensor, offsets: torch.Tensor, N: int, H: int, W: int,
               sigma: float = 4.0, radius: int = 7) -> torch.Tensor:
    out = torch.empty((N, H, W), dtype=torch.float32, device=offsets.device)
    call("dg_dmap_fixed", ptr(points) if points.numel() else None, ptr(offsets), N, H, W,
         float(sigma), int(radius), ptr(out), stream())
    return out
