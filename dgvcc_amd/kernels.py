"""Host wrappers over the C-ABI: torch tensors in, kernel launches out.

Activations are channel slices of NHWC buffers (`Act`): a pointer offset plus
the buffer's pixel stride, so the decoder's torch.cat (models/models.py:72,76,84)
becomes "write into a channel slice" with no copy.
"""
from __future__ import annotations

import weakref
from dataclasses import dataclass

import torch

from ._capi import DGError, call, dtype_code, lib_call_status, ptr, query, stream

F32, BF16, F16 = 0, 1, 2


@dataclass
class Act:
    """Channel slice [off, off+C) of an NHWC buffer `buf` [N,H,W,Ctot].  amax: None, or the operand
    maxima the kernel that wrote it produced (the f32 convs' f16 x3 scales): a device f32 [1 + C],
    [0] >= max |slice| and [1 + c] >= max |channel c| (a [1] tensor carries the tensor's word alone:
    the forward / dgrad read only that; the weight gradients, which scale per channel, then take a
    read pass of their own).  None makes the convs take one read pass over the slice."""
    buf: torch.Tensor
    off: int = 0
    C: int | None = None
    amax: torch.Tensor | None = None
    # f32: (image, bound) -- the f16 x3 pair image of the slice its producer wrote (bn_apply /
    # bn_apply_pool with pair=True) and the bound of its scale, for the next conv forward
    # (dg_conv_fwd_pair); cleared by writers that do not produce it
    pair: tuple | None = None

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
_SCOPE = ["other"]


def set_conv_timer(timer):
    """Install a callable timer(kind, flops, launch_fn, nbytes, scope) around conv GEMM
    launches (bench.py roofline measurement); None disables."""
    global _CONV_TIMER
    _CONV_TIMER = timer


def set_scope(scope: str):
    """Label the following conv launches ('enc' / 'dec' / 'head') for the timer."""
    _SCOPE[0] = scope


_CHECK_AMAX = __import__("os").environ.get("DGVCC_CHECK_AMAX", "0") == "1"


def check_amax(a: Act, what: str = ""):
    """DGVCC_CHECK_AMAX=1 (debug): the operand maxima attached to an f32 Act must bound the values
    (each word >= a fresh dg_amax of the slice); a smaller word would overflow the f16 x3 parts."""
    if a.amax is None or a.buf.dtype != torch.float32:
        return
    ref = amax(a)
    have = a.amax.float()
    n = min(have.numel(), ref.numel())
    bad = (have[:n] < ref[:n]).nonzero()
    if bad.numel():
        i = int(bad[0, 0])
        raise DGError(f"operand maxima below the values{' (' + what + ')' if what else ''}: word {i} holds "
                      f"{have[i].item()!r} < {ref[i].item()!r}")


def _timed(kind, flops, fn, nbytes=0.0):
    if _CONV_TIMER is None:
        fn()
    else:
        _CONV_TIMER(kind, flops, fn, nbytes, _SCOPE[0])

def pack_weight(w: torch.Tensor, dtype: torch.dtype, cpad: int | None = None,
                row_len: int | None = None) -> torch.Tensor:
    Cout, C, R, S = w.shape
    cpad = cpad or C
    row_len = row_len or R * S * cpad
    out = torch.empty((Cout, row_len), dtype=dtype, device=w.device)
    call("dg_pack_weight", dtype_code(dtype), ptr(w.contiguous()), Cout, C, R, S, cpad, row_len,
         ptr(out), stream())
    return out


def pack_weight_flip(w: torch.Tensor, dtype: torch.dtype) -> tuple[torch.Tensor, torch.Tensor]:
    """(pack_weight(w, dtype), flip_weight of it) from one launch (dg_pack_weight_flip)."""
    Cout, C, R, S = w.shape
    out = torch.empty((Cout, R * S * C), dtype=dtype, device=w.device)
    wflip = torch.empty_like(out)
    call("dg_pack_weight_flip", dtype_code(dtype), ptr(w.contiguous()), Cout, C, R, S, ptr(out), ptr(wflip),
         stream())
    return out, wflip


def conv_fwd(x: Act, wp: torch.Tensor, Cout: int, R: int, pad: int, y: Act,
             bias: torch.Tensor | None = None, accumulate=False, kind="fwd", k_alg=None):
    """k_alg: algorithmic reduction length when the GEMM K is padded (im2col layer)."""
    flops = 2.0 * x.M * (k_alg if k_alg else x.C * R * R) * Cout
    es = x.buf.element_size()
    nbytes = es * (x.M * x.C + wp.numel() + x.M * Cout * (2 if accumulate else 1))  # x, w, y (+y read)
    ws, work = _fwd_workspace(x, Cout, R)
    if _CHECK_AMAX:
        check_amax(x, kind)
    y.amax = None  # y is (re)written by a conv: no tracked maximum
    y.pair = None
    if x.pair is not None and x.dt == 0:
        xp, xb = x.pair
        _timed(kind, flops, lambda: call("dg_conv_fwd_pair", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, ptr(wp),
                                         Cout, R, R, pad, ptr(bias), y.ptr, y.ld, int(accumulate), None,
                                         ptr(work), ws, ptr(x.amax), ptr(xp), ptr(xb), stream()), nbytes)
        return
    _timed(kind, flops, lambda: call("dg_conv_fwd_ex", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, ptr(wp),
                                     Cout, R, R, pad, ptr(bias), y.ptr, y.ld, int(accumulate), None,
                                     ptr(work), ws, ptr(x.amax), stream()), nbytes)


def conv_fwd_bn_eval(x: Act, wp: torch.Tensor, Cout: int, R: int, pad: int, y: Act, bias, stats, act: int):
    """Eval-mode Conv + BN(running stats) [+ ReLU] in one launch: y = act((conv + bias)*scale + shift)."""
    flops = 2.0 * x.M * x.C * R * R * Cout
    nbytes = x.buf.element_size() * (x.M * x.C + wp.numel() + x.M * Cout)
    ws, work = _fwd_workspace(x, Cout, R)
    y.amax = None
    _timed("fwd", flops, lambda: call("dg_conv_fwd_bn_eval", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, ptr(wp), Cout,
                                      R, R, pad, ptr(bias), ptr(stats[2]), ptr(stats[3]), act, y.ptr, y.ld,
                                      ptr(work), ws, ptr(x.amax), stream()), nbytes)


_FWD_WS: dict = {}


def _fwd_workspace(x: Act, Cout: int, R: int):
    """Split-K partials for small-grid 16-bit forward/dgrad shapes (deep layers at small batch);
    f32: the pre-split filter planes of the split-math kernels (caller-owned, from torch's
    caching allocator, stream-ordered like every other buffer).  The size depends on
    DGVCC_PSPLIT_XS (pixel pre-split room), so the switch is part of the cache key."""
    key = (x.dt, x.N, x.H, x.W, x.C, Cout, R, __import__("os").environ.get("DGVCC_PSPLIT_XS"))
    ws = _FWD_WS.get(key)
    if ws is None:
        ws = _FWD_WS[key] = query("dg_conv_fwd_workspace", x.dt, x.N, x.H, x.W, x.C, Cout, R, R)
    if ws == 0:
        return 0, None
    return ws, torch.empty(ws, dtype=torch.uint8, device=x.buf.device)


_EXPORTED: dict = {}  # data_ptr -> (weakref to the buffer, its version, shape, amax)


def export_amax(a: Act) -> torch.Tensor:
    """a.buf, with a's operand maximum kept for a consumer that receives the plain tensor (plan
    outputs cross the autograd boundary as tensors; import_act finds the maximum again)."""
    if a.amax is not None and a.off == 0 and a.C == a.buf.shape[3]:
        if len(_EXPORTED) > 64:  # drop the entries whose buffers are gone
            for k in [k for k, e in _EXPORTED.items() if e[0]() is None]:
                del _EXPORTED[k]
        _EXPORTED[a.buf.data_ptr()] = (weakref.ref(a.buf), a.buf._version, tuple(a.buf.shape), a.amax)
    return a.buf


def import_act(t: torch.Tensor) -> Act:
    """Act(t) with the operand maximum export_amax kept for it: only while the exported buffer is
    alive (so the address is still its), unmodified (same version) and of the same shape."""
    a = Act(t)
    e = _EXPORTED.get(t.data_ptr())
    if e is not None:
        src = e[0]()
        if src is not None and src._version == e[1] and t._version == e[1] and tuple(t.shape) == e[2]:
            a.amax = e[3]
    return a


def amax(x: Act) -> torch.Tensor:
    """Operand maxima of the slice (f32): a device f32 [1 + C], [0] = max |x|, [1 + c] = max over
    channel c (dg_amax)."""
    out = torch.empty(amax_words(x.C), dtype=torch.float32, device=x.buf.device)
    call("dg_amax", x.dt, x.ptr, x.ld, x.M, x.C, ptr(out), stream())
    return out


def flip_weight(wp: torch.Tensor, Cout: int, C: int, R: int) -> torch.Tensor:
    wflip = torch.empty_like(wp)
    call("dg_flip_weight", dtype_code(wp.dtype), ptr(wp), Cout, C, R, R, ptr(wflip), stream())
    return wflip


def conv_dgrad(dy: Act, wp: torch.Tensor, C: int, R: int, pad: int, dx: Act, accumulate=False, wflip=None):
    """dX = conv(dY, flipped W^T): the forward GEMM kernel on the flipped filter (wflip: the caller's
    flip_weight(wp) when it holds one)."""
    if wflip is None:
        wflip = flip_weight(wp, dy.C, C, R)
    conv_fwd(dy, wflip, C, R, R - 1 - pad, dx, accumulate=accumulate, kind="dgrad")


def conv_dgrad_acc_relu(dy: Act, wp: torch.Tensor, C: int, dx: Act, relu_out: Act, wflip=None) -> bool:
    """dx = (relu_out > 0) ? dx + dgrad_1x1(dy) : 0 in one launch (the ReLU backward of relu_out
    folded into the accumulating dgrad's epilogue, dg_conv_fwd_acc_relu).  False (nothing
    launched) for the shapes that launch does not serve: the caller runs conv_dgrad + relu_bwd."""
    if wflip is None:
        wflip = flip_weight(wp, dy.C, C, 1)
    ws, work = _fwd_workspace(dy, C, 1)
    dx.amax = None
    flops = 2.0 * dy.M * dy.C * C
    nbytes = dy.buf.element_size() * (dy.M * dy.C + wflip.numel() + 3 * dy.M * C)
    res = []
    _timed("dgrad", flops, lambda: res.append(lib_call_status(
        "dg_conv_fwd_acc_relu", dy.dt, dy.ptr, dy.ld, dy.N, dy.H, dy.W, dy.C, ptr(wflip), C, relu_out.ptr,
        relu_out.ld, dx.ptr, dx.ld, ptr(work), ws, ptr(dy.amax), stream())), nbytes)
    if res[0] == -2:
        return False
    if res[0] != 0:
        raise DGError(f"dg_conv_fwd_acc_relu failed with status {res[0]}")
    return True


# Opt-in: measured slower on MI355X (the pipelined conv runs one 128-KB-LDS block per CU, so
# the epilogue's z loads and reductions are fully exposed: +1.3 ms of dgrad per step against
# the 0.75 ms partial pass it removes at 768x1024, A/B in DESIGN.md).
_BNPART_OFF = __import__("os").environ.get("DGVCC_DGRAD_BNPART", "0") != "1"
# fp32 (split math, conv_fwd_psplit_kernel EPI 2): opt-in as well; measured no faster on the fp32
# final step (415-417 ms either way, profiles/round2f/dgrad_bnpart_f32_ab.txt): the 8 KB-per-tile z
# reads and reductions in the persistent kernel's epilogue cost what the partial pass saved
_BNPART_F32_OFF = __import__("os").environ.get("DGVCC_DGRAD_BNPART_F32", "0") != "1"


def conv_dgrad_bnpart(dy: Act, wp: torch.Tensor, C: int, R: int, pad: int, dx: Act, z: Act, stats,
                      act: int, drop: torch.Tensor | None = None, wflip=None):
    """conv_dgrad (no accumulate) whose epilogue also emits the BatchNorm-backward partial
    sums of the layer whose output gradient dx is (z, stats, act, drop: that layer's);
    returns (part, rows) for bn_bwd_from_part, or None (nothing launched) when the shape is
    not served that way."""
    if stats is None or (dy.dt == 1 and _BNPART_OFF) or (dy.dt == 0 and _BNPART_F32_OFF) or dy.dt == 2:
        return None
    if wflip is None:
        wflip = flip_weight(wp, dy.C, C, R)
    rows = (query("dg_conv_bnpart_rows_ex", 0, dy.N, dy.H, dy.W, dy.C, dy.ld, C, R, R) if dy.dt == 0
            else query("dg_conv_stats_rows", dy.N, dy.H, dy.W))
    part = torch.empty((rows, 3, C), dtype=torch.float32, device=dy.buf.device)
    ws, work = _fwd_workspace(dy, C, R)
    dx.amax = None
    flops = 2.0 * dy.M * dy.C * R * R * C
    nbytes = dy.buf.element_size() * (dy.M * dy.C + wflip.numel() + 2 * dy.M * C)
    res = []

    def launch():
        res.append(lib_call_status("dg_conv_fwd_bnbwd", dy.dt, dy.ptr, dy.ld, dy.N, dy.H, dy.W, dy.C, ptr(wflip), C,
                                   R, R, R - 1 - pad, dx.ptr, dx.ld, z.ptr, z.ld, ptr(stats[2]), ptr(stats[3]),
                                   ptr(stats[0]), ptr(stats[1]), act, ptr(drop), z.H * z.W, ptr(part), ptr(work),
                                   ws, ptr(dy.amax), stream()))

    _timed("dgrad", flops, launch, nbytes)
    if res[0] == -2:
        return None
    if res[0] != 0:
        raise DGError(f"dg_conv_fwd_bnbwd failed with status {res[0]}")
    return part, rows


def bn_bwd_from_part(pre, g: Act, z: Act, gamma, stats, act: int, dz: Act, dgamma, dbeta, dbias=None,
                     drop: torch.Tensor | None = None):
    """bn_bwd with the partial sums from conv_dgrad_bnpart."""
    part, rows = pre
    coef = torch.empty((3, z.C), dtype=torch.float32, device=z.buf.device)
    am = _amax_out(dz)
    call("dg_bn_bwd_from_part", z.dt, ptr(part), rows, g.ptr, g.ld, z.ptr, z.ld, z.M, z.C, ptr(gamma),
         ptr(stats[0]), ptr(stats[1]), ptr(stats[2]), ptr(stats[3]), act, ptr(drop), z.H * z.W, dz.ptr, dz.ld,
         ptr(dgamma), ptr(dbeta), ptr(dbias), ptr(coef), ptr(am), stream())


def amax_words(C: int) -> int:
    """Floats of an operand-maxima buffer with channels: 1 + C, rounded up to a multiple of 4 (the
    library zeroes whole 16-byte words, include/dgvcc.h dg_amax)."""
    return (C + 4) & ~3


def chan_amax(a: Act):
    """a.amax when it carries per-channel words ([1 + C] and up: what the weight gradients' per-channel
    f16 x3 scales need), else None (the library then takes its own per-channel read pass)."""
    return a.amax if a.amax is not None and a.amax.numel() >= 1 + a.C else None


def conv_wgrad(x: Act, dy: Act, R: int, pad: int, dw: torch.Tensor, accumulate=False, k_alg=None):
    ws = query("dg_conv_wgrad_workspace", x.dt, x.N, x.H, x.W, x.C, dy.C, R, R)
    if _CHECK_AMAX:
        check_amax(x, "wgrad x")
        check_amax(dy, "wgrad dy")
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=x.buf.device)
    flops = 2.0 * x.M * (k_alg if k_alg else x.C * R * R) * dy.C
    nbytes = x.buf.element_size() * (x.M * x.C + dy.M * dy.C) + 4 * dw.numel()
    _timed("wgrad", flops, lambda: call("dg_conv_wgrad", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C,
                                        dy.ptr, dy.ld, dy.C, R, R, pad, ptr(dw), ptr(work), ws,
                                        int(accumulate), ptr(chan_amax(x)), ptr(chan_amax(dy)), stream()), nbytes)


def im2col_c3(img: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    N, _, H, W = img.shape
    out = torch.empty((N, H, W, 64), dtype=dtype, device=img.device)
    call("dg_im2col3x3_c3", dtype_code(dtype), ptr(img.contiguous()), N, H, W, ptr(out), stream())
    return out


def unpack_c3_grad(dwcol: torch.Tensor, dw: torch.Tensor, accumulate=False):
    call("dg_unpack_c3_grad", ptr(dwcol), dw.shape[0], ptr(dw), int(accumulate), stream())


def stem_fwd(img: torch.Tensor, wp: torch.Tensor, bias: torch.Tensor | None, z: Act) -> tuple:
    """Fused first layer (bf16): z = conv3x3(img NCHW f32, 3->64) + bias, plus BN partials."""
    N, _, H, W = img.shape
    rows = query("dg_stem_part_rows", N, H, W)
    part = torch.empty((rows, 3, 64), dtype=torch.float32, device=img.device)
    flops = 2.0 * N * H * W * 27 * 64
    nbytes = 4.0 * img.numel() + 2.0 * N * H * W * 64
    _timed("stem", flops, lambda: call("dg_stem_fwd", ptr(img), N, H, W, ptr(wp), ptr(bias), z.ptr, z.ld,
                                       ptr(part), stream()), nbytes)
    return part, rows


def stem_weight_f32(w: torch.Tensor) -> torch.Tensor:
    """[64][3][3][3] torch filter -> the f32 [27][64] layout of dg_stem_fwd_f32 (k = (c*3+r)*3+s)."""
    return w.detach().float().permute(1, 2, 3, 0).reshape(27, w.shape[0]).contiguous()


def stem_fwd_f32(img: torch.Tensor, wk: torch.Tensor, bias: torch.Tensor | None, z: Act) -> tuple:
    """fp32 first layer: z = conv3x3(img NCHW f32, 3->64) + bias (exact f32 FMAs), plus BN partials."""
    N, _, H, W = img.shape
    if wk.shape != (27, 64) or wk.dtype != torch.float32 or z.buf.dtype != torch.float32 or z.C != 64 \
            or (z.N, z.H, z.W) != (N, H, W):
        raise ValueError("stem_fwd_f32: operand shapes/dtypes")
    rows = query("dg_stem_part_rows", N, H, W)
    part = torch.empty((rows, 3, 64), dtype=torch.float32, device=img.device)
    flops = 2.0 * N * H * W * 27 * 64
    nbytes = 4.0 * img.numel() + 4.0 * N * H * W * 64
    _timed("stem", flops, lambda: call("dg_stem_fwd_f32", ptr(img), N, H, W, ptr(wk), ptr(bias), z.ptr, z.ld,
                                       ptr(part), stream()), nbytes)
    return part, rows


def stem_bwd_f32(img: torch.Tensor, g: Act, z: Act, stats, coef, dw: torch.Tensor, accumulate=False):
    """fp32 first-layer backward: conv1_1 weight gradient from (g, z) and the BN-backward coef."""
    N, _, H, W = img.shape
    if g.buf.dtype != torch.float32 or z.buf.dtype != torch.float32 or (z.N, z.H, z.W, z.C) != (N, H, W, 64) \
            or (g.N, g.H, g.W, g.C) != (N, H, W, 64) or dw.shape != (64, 3, 3, 3):
        raise ValueError("stem_bwd_f32: operand shapes/dtypes")
    ws = query("dg_stem_bwd_workspace", N, H, W)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=img.device)
    flops = 2.0 * N * H * W * 27 * 64
    nbytes = 4.0 * g.M * g.C * 2 + 4.0 * img.numel()
    _timed("stem_wgrad", flops, lambda: call("dg_stem_bwd_f32", ptr(img), N, H, W, g.ptr, g.ld, z.ptr, z.ld,
                                             ptr(stats[0]), ptr(stats[1]), ptr(stats[2]), ptr(stats[3]),
                                             ptr(coef), ptr(dw), ptr(work), ws, int(accumulate), stream()), nbytes)


def bn_part_finalize(part: torch.Tensor, nblk: int, C: int, gamma, beta, running_mean, running_var,
                     momentum, eps):
    stats = torch.empty((4, C), dtype=torch.float32, device=part.device)
    ws = query("dg_bn_part_workspace", nblk, C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=part.device)
    call("dg_bn_part_finalize", ptr(part), nblk, C, ptr(gamma), ptr(beta), ptr(running_mean),
         ptr(running_var), float(momentum), float(eps), ptr(stats[0]), ptr(stats[1]), ptr(stats[2]),
         ptr(stats[3]), ptr(work), stream())
    return stats


_EPI_STATS_OFF = __import__("os").environ.get("DGVCC_EPI_STATS", "1") == "0"


def conv_fwd_stats(x: Act, wp: torch.Tensor, Cout: int, R: int, pad: int, y: Act,
                   bias: torch.Tensor | None = None, k_alg=None):
    """conv_fwd with the BN statistics partials of y from the conv epilogue; returns
    (part, rows), or None (nothing launched) when the shape is served by a kernel without
    epilogue statistics.  k_alg: algorithmic reduction length when the GEMM K is padded."""
    rows = query("dg_conv_stats_rows_ex", x.dt, x.N, x.H, x.W, x.C, x.ld, Cout, R, R)
    part = torch.empty((rows, 3, Cout), dtype=torch.float32, device=x.buf.device)
    flops = 2.0 * x.M * (k_alg if k_alg else x.C * R * R) * Cout
    es = x.buf.element_size()
    nbytes = es * (x.M * x.C + wp.numel() + x.M * Cout)
    res = []

    if _EPI_STATS_OFF:
        return None
    ws, work = _fwd_workspace(x, Cout, R)
    y.amax = None
    y.pair = None

    def launch():
        if x.pair is not None and x.dt == 0:
            xp, xb = x.pair
            res.append(lib_call_status("dg_conv_fwd_pair", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, ptr(wp), Cout,
                                       R, R, pad, ptr(bias), y.ptr, y.ld, 0, ptr(part), ptr(work), ws,
                                       ptr(x.amax), ptr(xp), ptr(xb), stream()))
            return
        res.append(lib_call_status("dg_conv_fwd_ex", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, ptr(wp), Cout,
                                   R, R, pad, ptr(bias), y.ptr, y.ld, 0, ptr(part), ptr(work), ws, ptr(x.amax),
                                   stream()))

    _timed("fwd", flops, launch, nbytes)
    if res[0] == -2:  # DG_ERR_UNSUPPORTED: nothing was launched
        return None
    if res[0] != 0:
        raise DGError(f"dg_conv_fwd_ex failed with status {res[0]}")
    return part, rows


def bn_bwd_coef(g: Act, z: Act, gamma, stats, act: int, dgamma, dbeta, dbias=None,
                drop: torch.Tensor | None = None) -> torch.Tensor:
    ws = query("dg_bn_workspace", z.M, z.C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=z.buf.device)
    coef = torch.empty((3, z.C), dtype=torch.float32, device=z.buf.device)
    call("dg_bn_bwd_coef", z.dt, g.ptr, g.ld, z.ptr, z.ld, z.M, z.C, ptr(gamma), ptr(stats[0]),
         ptr(stats[1]), ptr(stats[2]), ptr(stats[3]), act, ptr(drop), z.H * z.W, ptr(coef),
         ptr(dgamma), ptr(dbeta), ptr(dbias), ptr(work), stream())
    return coef


def stem_bwd(img: torch.Tensor, g: Act, z: Act | None, stats, coef, dw: torch.Tensor, accumulate=False,
             wp: torch.Tensor | None = None, bias: torch.Tensor | None = None):
    """z = None: z recomputed from img with the packed filters wp (+ bias)."""
    N, _, H, W = img.shape
    ws = query("dg_stem_bwd_workspace", N, H, W)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=img.device)
    flops = 2.0 * N * H * W * 27 * 64
    nbytes = 2.0 * g.M * g.C * (2 if z is not None else 1) + 4.0 * img.numel()
    _timed("stem_wgrad", flops, lambda: call("dg_stem_bwd", ptr(img), N, H, W, g.ptr, g.ld,
                                             z.ptr if z is not None else None, z.ld if z is not None else 0,
                                             ptr(stats[0]), ptr(stats[1]), ptr(stats[2]), ptr(stats[3]),
                                             ptr(coef), ptr(dw), ptr(work), ws, int(accumulate), ptr(wp), ptr(bias),
                                             stream()), nbytes)


def stem_stats(img: torch.Tensor, wp: torch.Tensor, bias: torch.Tensor | None) -> tuple:
    """BN statistics partials of z = conv(img) + bias without storing z."""
    N, _, H, W = img.shape
    rows = query("dg_stem_part_rows", N, H, W)
    part = torch.empty((rows, 3, 64), dtype=torch.float32, device=img.device)
    _timed("stem", 2.0 * N * H * W * 27 * 64,
           lambda: call("dg_stem_stats", ptr(img), N, H, W, ptr(wp), ptr(bias), ptr(part), stream()),
           4.0 * img.numel())
    return part, rows


def stem_apply(img: torch.Tensor, wp: torch.Tensor, bias: torch.Tensor | None, stats, y: Act):
    """y = relu(BN(conv(img) + bias)) with z recomputed (stem_fwd + bn_apply, bit for bit)."""
    N, _, H, W = img.shape
    _timed("stem", 2.0 * N * H * W * 27 * 64,
           lambda: call("dg_stem_apply", ptr(img), N, H, W, ptr(wp), ptr(bias), ptr(stats[2]), ptr(stats[3]),
                        y.ptr, y.ld, stream()),
           4.0 * img.numel() + 2.0 * N * H * W * 64)


def stem_bwd_coef(img: torch.Tensor, wp: torch.Tensor, bias, g: Act, gamma, stats, dgamma, dbeta,
                  dbias=None) -> torch.Tensor:
    """bn_bwd_coef of the stem with z recomputed from the image."""
    N, _, H, W = img.shape
    rows = query("dg_stem_part_rows", N, H, W)
    part = torch.empty((rows, 3, 64), dtype=torch.float32, device=img.device)
    coef = torch.empty((3, 64), dtype=torch.float32, device=img.device)
    call("dg_stem_bwd_coef", ptr(img), N, H, W, ptr(wp), ptr(bias), g.ptr, g.ld, ptr(gamma), ptr(stats[0]),
         ptr(stats[1]), ptr(stats[2]), ptr(stats[3]), ptr(coef), ptr(dgamma), ptr(dbeta), ptr(dbias), ptr(part),
         stream())
    return coef


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


def _amax_out(a: Act | None, *more: Act | None) -> torch.Tensor | None:
    """A fresh device f32 [1 + C] that an f32 producer fills with its output's operand maxima (the
    tensor's, then each channel's), attached to the Acts it writes (same channels: the following f16
    x3 convs' scales); None for 16-bit outputs."""
    if a is None or a.buf.dtype != torch.float32:
        return None
    t = torch.empty(amax_words(a.C), dtype=torch.float32, device=a.buf.device)
    for o in (a, *more):
        if o is not None:
            o.amax = t
    return t


def _pair_bufs(M: int, C: int, dev):
    return torch.empty(M * C, dtype=torch.float32, device=dev), torch.empty(1, dtype=torch.float32, device=dev)


def bn_apply(z: Act, stats, act: int, y: Act, drop: torch.Tensor | None = None, pair: bool = False,
             count: int | None = None):
    """pair (f32, train-mode batch statistics over `count` pixels, default z.M; no dropout): also the
    f16 x3 pair image of y for the next conv forward (dg_bn_apply_pair), attached as y.pair."""
    am = _amax_out(y)
    y.pair = None
    if pair and z.dt == 0 and drop is None and z.C % 32 == 0:
        img, bound = _pair_bufs(z.M, z.C, z.buf.device)
        st = lib_call_status("dg_bn_apply_pair", z.ptr, z.ld, z.M, z.C, ptr(stats[2]), ptr(stats[3]),
                             ptr(stats[0]), ptr(stats[1]), float(count or z.M), act, y.ptr, y.ld, ptr(am),
                             ptr(img), ptr(bound), stream())
        if st == 0:
            y.pair = (img, bound)
            return
        if st != -2:
            raise DGError(f"dg_bn_apply_pair failed with status {st}")
    call("dg_bn_apply", z.dt, z.ptr, z.ld, z.M, z.C, ptr(stats[2]), ptr(stats[3]), act, ptr(drop),
         z.H * z.W, y.ptr, y.ld, ptr(am), stream())


def bn_bwd(g: Act, z: Act, gamma, stats, act: int, dz: Act, dgamma, dbeta, dbias=None,
           drop: torch.Tensor | None = None, pair: bool = False, count: int | None = None):
    """pair (f32, train-mode batch statistics over `count` pixels, default z.M; no dropout): also the
    f16 x3 pair image of dz for the dgrad (dg_bn_bwd_pair), attached as dz.pair."""
    ws = query("dg_bn_workspace", z.M, z.C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=z.buf.device)
    st = stats if stats is not None else (None, None, None, None)  # None: no normalisation
    am = _amax_out(dz)
    dz.pair = None
    if pair and stats is not None and z.dt == 0 and drop is None and z.C % 32 == 0:
        img, bound = _pair_bufs(z.M, z.C, z.buf.device)
        r = lib_call_status("dg_bn_bwd_pair", g.ptr, g.ld, z.ptr, z.ld, z.M, z.C, ptr(gamma), ptr(st[0]),
                            ptr(st[1]), ptr(st[2]), ptr(st[3]), act, float(count or z.M), dz.ptr, dz.ld,
                            ptr(dgamma), ptr(dbeta), ptr(dbias), ptr(work), ptr(am), ptr(img), ptr(bound), stream())
        if r == 0:
            dz.pair = (img, bound)
            return
        if r != -2:
            raise DGError(f"dg_bn_bwd_pair failed with status {r}")
    call("dg_bn_bwd", z.dt, g.ptr, g.ld, z.ptr, z.ld, z.M, z.C, ptr(gamma), ptr(st[0]),
         ptr(st[1]), ptr(st[2]), ptr(st[3]), act, ptr(drop), z.H * z.W, dz.ptr, dz.ld,
         ptr(dgamma), ptr(dbeta), ptr(dbias), ptr(work), ptr(am), stream())


def bn_apply_pool(z: Act, stats, act: int, y: Act | None, yp: Act, drop: torch.Tensor | None = None,
                  pair: bool = False, count: int | None = None):
    """y = act(BN(z)) [* drop] (only written when y is given) and yp = maxpool2x2(y).  pair: as
    bn_apply, the pair image of yp (dg_bn_apply_pool_pair)."""
    am = _amax_out(yp, y)  # max over the un-pooled values bounds both
    yp.pair = None
    if y is not None:
        y.pair = None
    if pair and z.dt == 0 and drop is None and z.C % 32 == 0:
        img, bound = _pair_bufs(yp.M, z.C, z.buf.device)
        st = lib_call_status("dg_bn_apply_pool_pair", z.ptr, z.ld, z.N, z.H, z.W, z.C, ptr(stats[2]),
                             ptr(stats[3]), ptr(stats[0]), ptr(stats[1]), float(count or z.M), act,
                             y.ptr if y is not None else None, y.ld if y is not None else 0, yp.ptr, yp.ld,
                             ptr(am), ptr(img), ptr(bound), stream())
        if st == 0:
            yp.pair = (img, bound)
            return
        if st != -2:
            raise DGError(f"dg_bn_apply_pool_pair failed with status {st}")
    call("dg_bn_apply_pool", z.dt, z.ptr, z.ld, z.N, z.H, z.W, z.C, ptr(stats[2]), ptr(stats[3]), act,
         ptr(drop), y.ptr if y is not None else None, y.ld if y is not None else 0, yp.ptr, yp.ld, ptr(am), stream())


def bn_bwd_pool(gp: Act, gd: Act | None, z: Act, gamma, stats, act: int, dz: Act, dgamma, dbeta,
                dbias=None, drop: torch.Tensor | None = None, pair: bool = False, count: int | None = None):
    """BN backward with the upstream gradient = maxpool2x2 backward of gp (argmax recomputed
    from z) [+ the direct gradient gd].  pair: as bn_bwd (dg_bn_bwd_pool_pair)."""
    ws = query("dg_bn_workspace", z.M, z.C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=z.buf.device)
    am = _amax_out(dz)
    dz.pair = None
    if pair and z.dt == 0 and drop is None and z.C % 32 == 0:
        img, bound = _pair_bufs(z.M, z.C, z.buf.device)
        r = lib_call_status("dg_bn_bwd_pool_pair", gp.ptr, gp.ld, gd.ptr if gd is not None else None,
                            gd.ld if gd is not None else 0, z.ptr, z.ld, z.N, z.H, z.W, z.C, ptr(gamma),
                            ptr(stats[0]), ptr(stats[1]), ptr(stats[2]), ptr(stats[3]), act, float(count or z.M),
                            dz.ptr, dz.ld, ptr(dgamma), ptr(dbeta), ptr(dbias), ptr(work), ptr(am), ptr(img),
                            ptr(bound), stream())
        if r == 0:
            dz.pair = (img, bound)
            return
        if r != -2:
            raise DGError(f"dg_bn_bwd_pool_pair failed with status {r}")
    call("dg_bn_bwd_pool", z.dt, gp.ptr, gp.ld, gd.ptr if gd is not None else None,
         gd.ld if gd is not None else 0, z.ptr, z.ld, z.N, z.H, z.W, z.C, ptr(gamma), ptr(stats[0]),
         ptr(stats[1]), ptr(stats[2]), ptr(stats[3]), act, ptr(drop), dz.ptr, dz.ld, ptr(dgamma),
         ptr(dbeta), ptr(dbias), ptr(work), ptr(am), stream())


# ---------------------------------------------------------------- resample -
def _expect(y: Act, N, H, W, C, what):
    if (y.N, y.H, y.W, y.C) != (N, H, W, C):
        raise DGError(f"{what}: output {(y.N, y.H, y.W, y.C)} != expected {(N, H, W, C)}")


def maxpool_fwd(x: Act, y: Act):
    _expect(y, x.N, x.H // 2, x.W // 2, x.C, "maxpool_fwd")
    call("dg_maxpool2_fwd", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, y.ptr, y.ld, stream())
    y.amax = x.amax  # a window maximum never exceeds its channel's max |x|


def maxpool_bwd(x: Act, gy: Act, gx: Act, accumulate=False):
    _expect(gy, x.N, x.H // 2, x.W // 2, x.C, "maxpool_bwd")
    _expect(gx, x.N, x.H, x.W, x.C, "maxpool_bwd")
    call("dg_maxpool2_bwd", x.dt, x.ptr, x.ld, gy.ptr, gy.ld, x.N, x.H, x.W, x.C, gx.ptr, gx.ld,
         int(accumulate), stream())
    gx.amax = None  # rewritten without a tracked maximum


UP_BILINEAR, UP_BILINEAR_AC, UP_NEAREST = 0, 1, 2


def upsample_fwd(x: Act, scale: int, mode: int, y: Act):
    _expect(y, x.N, x.H * scale, x.W * scale, x.C, "upsample_fwd")
    call("dg_upsample_fwd", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, scale, mode, y.ptr, y.ld, stream())
    y.amax = x.amax  # bilinear / nearest values are convex combinations of the source channel's


def upsample_bwd(gy: Act, scale: int, mode: int, gx: Act, gy2: Act | None = None, accumulate=False):
    _expect(gy, gx.N, gx.H * scale, gx.W * scale, gx.C, "upsample_bwd")
    call("dg_upsample_bwd", gx.dt, gy.ptr, gy.ld, gy2.ptr if gy2 is not None else None,
         gy2.ld if gy2 is not None else 0, gx.N, gx.H, gx.W, gx.C, scale, mode, gx.ptr, gx.ld,
         int(accumulate), stream())
    gx.amax = None


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
    if gx is not None:
        gx.amax = None


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
               sigma: float = 4.0, radius: int = 7, deterministic: bool = True) -> torch.Tensor:
    """deterministic: per-tile in-order sums (bit-identical to the reference); False: one
    wave per point with f32 atomics (order-dependent in the last ulp)."""
    out = torch.empty((N, H, W), dtype=torch.float32, device=offsets.device)
    pp = ptr(points) if points.numel() else None
    if not deterministic:
        call("dg_dmap_fixed", pp, ptr(offsets), N, H, W, float(sigma), int(radius), ptr(out), stream())
        return out
    npts = points.numel() // 2
    ws = query("dg_dmap_fixed_tiled_workspace", N, H, W, int(radius), npts)
    work = torch.empty(ws // 4, dtype=torch.int32, device=offsets.device) if ws else None
    call("dg_dmap_fixed_tiled", pp, ptr(offsets), N, H, W, float(sigma), int(radius), npts,
         ptr(work) if ws else None, ptr(out), stream())
    return out


# ---------------------------------------------------------------- ResNet trunks -
def conv_out(H: int, R: int, stride: int, pad: int) -> int:
    return (H + 2 * pad - R) // stride + 1


def pack_weight_t(wp: torch.Tensor, Cout: int, C: int, R: int, S: int) -> torch.Tensor:
    """packed [Cout][R][S][C] -> [C][R][S][Cout] (dgrad operand of strided convs)."""
    wt = torch.empty((C, R * S * Cout), dtype=wp.dtype, device=wp.device)
    call("dg_transpose_weight", dtype_code(wp.dtype), ptr(wp), Cout, C, R, S, ptr(wt), stream())
    return wt


def conv2d_fwd(x: Act, wp: torch.Tensor, Cout: int, R: int, stride: int, pad: int, y: Act,
               bias: torch.Tensor | None = None, accumulate=False, kind="fwd", k_alg=None):
    """General conv (any R, stride, pad): y [N,P,Q,Cout]."""
    P, Q = conv_out(x.H, R, stride, pad), conv_out(x.W, R, stride, pad)
    if (y.H, y.W, y.N, y.C) != (P, Q, x.N, Cout):
        raise DGError(f"conv2d_fwd: output {tuple(y.view().shape)} != {(x.N, P, Q, Cout)}")
    M = x.N * P * Q
    flops = 2.0 * M * (k_alg if k_alg else x.C * R * R) * Cout
    es = x.buf.element_size()
    nbytes = es * (x.M * x.C + wp.numel() + M * Cout * (2 if accumulate else 1))
    y.amax = None
    _timed(kind, flops, lambda: call("dg_conv2d_fwd", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, ptr(wp),
                                     Cout, R, R, stride, pad, ptr(bias), y.ptr, y.ld,
                                     int(accumulate), stream()), nbytes)


def conv2d_dgrad(dy: Act, wt: torch.Tensor, R: int, stride: int, pad: int, dx: Act, accumulate=False):
    """dX [N,H,W,C] of a general conv from dY [N,P,Q,Cout] and the transposed filter wt."""
    if conv_out(dx.H, R, stride, pad) != dy.H or conv_out(dx.W, R, stride, pad) != dy.W:
        raise DGError("conv2d_dgrad: dx/dy spatial sizes disagree with R/stride/pad")
    flops = 2.0 * dy.M * dx.C * R * R * dy.C
    es = dy.buf.element_size()
    nbytes = es * (dy.M * dy.C + wt.numel() + dx.M * dx.C * (2 if accumulate else 1))
    dx.amax = None
    _timed("dgrad", flops, lambda: call("dg_conv2d_dgrad", dy.dt, dy.ptr, dy.ld, dy.N, dy.H, dy.W,
                                        dy.C, ptr(wt), dx.C, dx.H, dx.W, R, R, stride, pad, dx.ptr,
                                        dx.ld, int(accumulate), stream()), nbytes)


def conv2d_wgrad(x: Act, dy: Act, R: int, stride: int, pad: int, dw: torch.Tensor,
                 accumulate=False, k_alg=None):
    ws = query("dg_conv2d_wgrad_workspace", x.dt, dy.N, dy.H, dy.W, x.C, dy.C, R, R)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=x.buf.device)
    flops = 2.0 * dy.M * (k_alg if k_alg else x.C * R * R) * dy.C
    nbytes = x.buf.element_size() * (x.M * x.C + dy.M * dy.C) + 4 * dw.numel()
    _timed("wgrad", flops, lambda: call("dg_conv2d_wgrad", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C,
                                        dy.ptr, dy.ld, dy.C, R, R, stride, pad, ptr(dw), ptr(work),
                                        ws, int(accumulate), ptr(chan_amax(x)), ptr(chan_amax(dy)), stream()), nbytes)


def im2col_c3_general(img: torch.Tensor, dtype: torch.dtype, R: int, stride: int, pad: int,
                      kpad: int) -> torch.Tensor:
    N, _, H, W = img.shape
    P, Q = conv_out(H, R, stride, pad), conv_out(W, R, stride, pad)
    out = torch.empty((N, P, Q, kpad), dtype=dtype, device=img.device)
    call("dg_im2col_c3", dtype_code(dtype), ptr(img.contiguous()), N, H, W, R, R, stride, pad, kpad,
         ptr(out), stream())
    return out


def unpack_c3(dwcol: torch.Tensor, dw: torch.Tensor, accumulate=False):
    Cout, _, R, S = dw.shape
    call("dg_unpack_c3", ptr(dwcol), Cout, R, S, dwcol.shape[1], ptr(dw), int(accumulate), stream())


def maxpool_k_fwd(x: Act, k: int, stride: int, pad: int, y: Act):
    call("dg_maxpool_fwd", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, k, stride, pad, y.ptr, y.ld,
         stream())
    y.amax = x.amax  # a window maximum never exceeds its channel's max |x|


def maxpool_k_bwd(x: Act, gy: Act, k: int, stride: int, pad: int, gx: Act, accumulate=False):
    call("dg_maxpool_bwd", x.dt, x.ptr, x.ld, gy.ptr, gy.ld, x.N, x.H, x.W, x.C, k, stride, pad,
         gx.ptr, gx.ld, int(accumulate), stream())
    gx.amax = None


def maxpool_k_fwd_idx(x: Act, k: int, stride: int, pad: int, y: Act) -> torch.Tensor:
    """maxpool_k_fwd that also records each window's argmax (uint8 [N,P,Q,C]) for maxpool_k_bwd_idx."""
    idx = torch.empty((y.N, y.H, y.W, x.C), dtype=torch.uint8, device=x.buf.device)
    call("dg_maxpool_fwd_idx", x.dt, x.ptr, x.ld, x.N, x.H, x.W, x.C, k, stride, pad, y.ptr, y.ld,
         ptr(idx), stream())
    y.amax = x.amax  # a window maximum never exceeds max |x|: x's bound serves the pooled map
    return idx


def maxpool_k_bwd_idx(idx: torch.Tensor, gy: Act, k: int, stride: int, pad: int, gx: Act, accumulate=False):
    call("dg_maxpool_bwd_idx", gx.dt, ptr(idx), gy.ptr, gy.ld, gx.N, gx.H, gx.W, gx.C, k, stride, pad,
         gx.ptr, gx.ld, int(accumulate), stream())
    gx.amax = None


def bn_add_apply(z1: Act, st1, z2: Act, st2, act: int, y: Act):
    """y = act(bn1(z1) + (bn2(z2) if st2 is not None else z2)) — Bottleneck join."""
    am = _amax_out(y)
    call("dg_bn_add_apply", z1.dt, z1.ptr, z1.ld, z1.M, z1.C, ptr(st1[2]), ptr(st1[3]), z2.ptr,
         z2.ld, ptr(st2[2]) if st2 is not None else None, ptr(st2[3]) if st2 is not None else None,
         act, y.ptr, y.ld, ptr(am), stream())


def relu_bwd(g: Act, y: Act, out: Act):
    call("dg_relu_bwd", g.dt, g.ptr, g.ld, y.ptr, y.ld, y.M, y.C, out.ptr, out.ld, stream())
    out.amax = g.amax  # |g * mask| <= |g| channel by channel


def instnorm_stats(x: Act, eps: float = 1e-5) -> torch.Tensor:
    """[2, N, C] f32: mean, invstd (biased variance) per (n, c)."""
    st = torch.empty((2, x.N, x.C), dtype=torch.float32, device=x.buf.device)
    ws = query("dg_instnorm_workspace", x.N, x.H * x.W, x.C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=x.buf.device)
    call("dg_instnorm_stats", x.dt, x.ptr, x.ld, x.N, x.H * x.W, x.C, float(eps), ptr(st[0]),
         ptr(st[1]), ptr(work), stream())
    return st


def instnorm_apply(x: Act, st, gamma, beta, act: int, y: Act):
    am = _amax_out(y)
    call("dg_instnorm_apply", x.dt, x.ptr, x.ld, x.N, x.H * x.W, x.C, ptr(st[0]), ptr(st[1]),
         ptr(gamma), ptr(beta), act, y.ptr, y.ld, ptr(am), stream())


def instnorm_bwd(g: Act, x: Act, st, gamma, dx: Act, dgamma=None, dbeta=None, accumulate=False):
    ws = query("dg_instnorm_bwd_workspace", x.N, x.H * x.W, x.C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=x.buf.device)
    am = _amax_out(dx)
    call("dg_instnorm_bwd", x.dt, g.ptr, g.ld, x.ptr, x.ld, x.N, x.H * x.W, x.C, ptr(st[0]),
         ptr(st[1]), ptr(gamma), dx.ptr, dx.ld, int(accumulate), ptr(dgamma), ptr(dbeta),
         ptr(work), ptr(am), stream())


# ---------------------------------------------------------------- whitening -
def iw_loss(fraw: torch.Tensor, hw: int, mask: torch.Tensor, num_sensitive: torch.Tensor,
            out_scale: float, loss: torch.Tensor | None, accumulate: bool,
            want_grad: bool, grad_coef: torch.Tensor | None = None, eps: float = 1e-5):
    """instance_whitening_loss over a batch of raw Gram matrices fraw [B,C,C]."""
    B, C, _ = fraw.shape
    ws = query("dg_iw_loss_workspace", B, C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=fraw.device)
    gsym = torch.empty_like(fraw) if want_grad else None
    call("dg_iw_loss", ptr(fraw), B, C, 1.0 / (hw - 1), float(eps), ptr(mask), ptr(num_sensitive),
         ptr(grad_coef), float(out_scale), int(accumulate), ptr(loss), ptr(gsym), ptr(work), stream())
    return gsym


def iw_cov_var(fraw: torch.Tensor, hw: int, var: torch.Tensor, accumulate=False):
    B, C, _ = fraw.shape
    call("dg_iw_cov_var", ptr(fraw), B, C, 1.0 / (hw - 1), ptr(var), int(accumulate), stream())


def sw_fwd(x: Act, mean_w, var_w, gamma, beta, running_mean, running_cov, training: bool,
           act: int, y: Act, T: int = 5, eps: float = 1e-5, momentum: float = 0.9) -> torch.Tensor:
    """SwitchWhiten2d (sw_type 2) forward; returns the `save` statistics buffer."""
    HW = x.H * x.W
    save = torch.empty(query("dg_sw_save_size", x.N, x.C) // 4, dtype=torch.float32,
                       device=x.buf.device)
    ws = query("dg_sw_workspace", x.N, HW, x.C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=x.buf.device)
    call("dg_sw_fwd", x.dt, x.ptr, x.ld, x.N, HW, x.C, int(T), float(eps), float(momentum),
         ptr(mean_w), ptr(var_w), ptr(gamma), ptr(beta), ptr(running_mean), ptr(running_cov),
         int(training), act, ptr(save), y.ptr, y.ld, ptr(work), stream())
    return save


def sw_fwd_sync(x: Act, mean_w, var_w, gamma, beta, running_mean, running_cov, training: bool,
                act: int, y: Act, reduce_fn, T: int = 5, eps: float = 1e-5, momentum: float = 0.9):
    """SyncSwitchWhiten2d forward: reduce_fn(moments f64 tensor) -> (moments summed over ranks,
    total image count) sits between the statistics and the whitening phases.
    Returns (save, workspace) for sw_bwd_sync."""
    HW = x.H * x.W
    dev = x.buf.device
    save = torch.empty(query("dg_sw_save_size", x.N, x.C) // 4, dtype=torch.float32, device=dev)
    ws = query("dg_sw_workspace", x.N, HW, x.C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=dev)
    mom = torch.empty(query("dg_sw_moments_size", x.C) // 8, dtype=torch.float64, device=dev)
    count = x.N
    if training:
        call("dg_sw_fwd_stats", x.dt, x.ptr, x.ld, x.N, HW, x.C, ptr(save), ptr(mom), ptr(work), stream())
        mom, count = reduce_fn(mom)
    else:
        call("dg_sw_fwd_stats", x.dt, x.ptr, x.ld, x.N, HW, x.C, ptr(save), ptr(mom), ptr(work), stream())
    call("dg_sw_fwd_finish", x.dt, x.ptr, x.ld, x.N, HW, x.C, int(T), float(eps), float(momentum),
         ptr(mean_w), ptr(var_w), ptr(gamma), ptr(beta), ptr(running_mean), ptr(running_cov),
         int(training), act, int(count), ptr(mom), ptr(save), y.ptr, y.ld, stream())
    return save, work, count


def sw_bwd_sync(gy: Act, y: Act | None, x: Act, save, work, mean_w, var_w, gamma, act: int, dx: Act,
                reduce_fn, dgamma=None, dbeta=None, dmean_w=None, dvar_w=None, accumulate=False,
                T: int = 5, eps: float = 1e-5):
    HW = x.H * x.W
    bm = torch.empty(query("dg_sw_moments_size", x.C) // 8, dtype=torch.float64, device=x.buf.device)
    call("dg_sw_bwd_stats", x.dt, gy.ptr, gy.ld, y.ptr if y is not None else None,
         y.ld if y is not None else 0, x.ptr, x.ld, x.N, HW, x.C, int(T), float(eps), ptr(mean_w),
         ptr(var_w), ptr(gamma), act, ptr(save), ptr(bm), ptr(dgamma), ptr(dbeta), ptr(work), stream())
    bm, count = reduce_fn(bm)
    call("dg_sw_bwd_finish", x.dt, gy.ptr, gy.ld, y.ptr if y is not None else None,
         y.ld if y is not None else 0, x.ptr, x.ld, x.N, HW, x.C, act, ptr(mean_w), ptr(var_w),
         ptr(save), int(count), ptr(bm), dx.ptr, dx.ld, int(accumulate), ptr(dmean_w), ptr(dvar_w),
         ptr(work), stream())


def sw_bwd(gy: Act, y: Act | None, x: Act, save, mean_w, var_w, gamma, act: int, dx: Act,
           dgamma=None, dbeta=None, dmean_w=None, dvar_w=None, accumulate=False, T: int = 5,
           eps: float = 1e-5):
    HW = x.H * x.W
    ws = query("dg_sw_workspace", x.N, HW, x.C)
    work = torch.empty(ws // 4 + 1, dtype=torch.float32, device=x.buf.device)
    call("dg_sw_bwd", x.dt, gy.ptr, gy.ld, y.ptr if y is not None else None,
         y.ld if y is not None else 0, x.ptr, x.ld, x.N, HW, x.C, int(T), float(eps), ptr(mean_w),
         ptr(var_w), ptr(gamma), act, ptr(save), dx.ptr, dx.ld, int(accumulate), ptr(dgamma),
         ptr(dbeta), ptr(dmean_w), ptr(dvar_w), ptr(work), stream())
