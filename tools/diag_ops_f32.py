"""Diagnostic: per-op fp32 accuracy of the HIP kernels against float64 torch on random data
(normwise relative error of each output / gradient), beside torch fp32 on the GPU."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgvcc_amd import kernels as K  # noqa: E402
from dgvcc_amd.kernels import Act  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)


def nerr(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def conv_case(N, H, W, C, Co, R):
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(Co, C, R, R, generator=g) / (C * R * R) ** 0.5
    b = torch.randn(Co, generator=g) * 0.1
    gy = torch.randn(N, Co, H, W, generator=g)
    xd, wd = x.double().requires_grad_(True), w.double().requires_grad_(True)
    y = F.conv2d(xd, wd, b.double(), padding=R // 2)
    y.backward(gy.double())
    X = Act(nhwc(x).to(dev))
    wp = K.pack_weight(w.to(dev), torch.float32)
    Y = Act(K.nhwc(N, H, W, Co, torch.float32, dev))
    K.conv_fwd(X, wp, Co, R, R // 2, Y, bias=b.to(dev))
    GY = Act(nhwc(gy).to(dev))
    GX = Act(K.nhwc(N, H, W, C, torch.float32, dev))
    K.conv_dgrad(GY, wp, C, R, R // 2, GX)
    DW = torch.empty(Co, C, R, R, device=dev)
    K.conv_wgrad(X, GY, R, R // 2, DW)
    torch.cuda.synchronize()
    print(f"conv {N}x{H}x{W} {C}->{Co} R{R}: fwd {nerr(Y.buf, nhwc(y.detach())):.2e} "
          f"dgrad {nerr(GX.buf, nhwc(xd.grad)):.2e} wgrad {nerr(DW, wd.grad):.2e}")


def bn_case(N, H, W, C, act, with_bn=True):
    z = torch.randn(N, C, H, W, generator=g) * 2 + 0.5
    gam = torch.rand(C, generator=g) + 0.5
    bet = torch.randn(C, generator=g) * 0.1
    gy = torch.randn(N, C, H, W, generator=g)
    zd = z.double().requires_grad_(True)
    gd, bd = gam.double().requires_grad_(True), bet.double().requires_grad_(True)
    if with_bn:
        y = F.batch_norm(zd, None, None, gd, bd, True, 0.1, 1e-5)
    else:
        y = zd
    if act:
        y = F.relu(y)
    y.backward(gy.double())
    Z = Act(nhwc(z).to(dev))
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    if with_bn:
        st = K.bn_fwd_train(Z, gam.to(dev), bet.to(dev), rm, rv, 0.1, 1e-5)
    else:
        st = None
    Y = Act(K.nhwc(N, H, W, C, torch.float32, dev))
    if with_bn:
        K.bn_apply(Z, st, act, Y)
    DZ = Act(K.nhwc(N, H, W, C, torch.float32, dev))
    dga, dbe = torch.empty(C, device=dev), torch.empty(C, device=dev)
    K.bn_bwd(Act(nhwc(gy).to(dev)), Z, gam.to(dev) if with_bn else None, st, act, DZ, dga, dbe, None)
    torch.cuda.synchronize()
    msg = f"bn {N}x{H}x{W}x{C} act{act} bn{int(with_bn)}: "
    if with_bn:
        msg += f"fwd {nerr(Y.buf, nhwc(y.detach())):.2e} dgamma {nerr(dga, gd.grad):.2e} "
    msg += f"dz {nerr(DZ.buf, nhwc(zd.grad)):.2e} dbeta {nerr(dbe, bd.grad if with_bn else gy.double().mul((zd > 0).double() if act else 1).sum((0, 2, 3))):.2e}"
    print(msg)


def resample_case(N, H, W, C):
    x = torch.randn(N, C, H, W, generator=g)
    gy = torch.randn(N, C, 2 * H, 2 * W, generator=g)
    xd = x.double().requires_grad_(True)
    F.interpolate(xd, scale_factor=2, mode="bilinear", align_corners=False).backward(gy.double())
    GX = Act(K.nhwc(N, H, W, C, torch.float32, dev))
    K.upsample_bwd(Act(nhwc(gy).to(dev)), 2, K.UP_BILINEAR, GX)
    gp = torch.randn(N, C, H // 2, W // 2, generator=g)
    xd2 = x.double().requires_grad_(True)
    F.max_pool2d(xd2, 2, 2).backward(gp.double())
    GP = Act(K.nhwc(N, H, W, C, torch.float32, dev))
    K.maxpool_bwd(Act(nhwc(x).to(dev)), Act(nhwc(gp).to(dev)), GP)
    torch.cuda.synchronize()
    print(f"resample {N}x{H}x{W}x{C}: upsample_bwd {nerr(GX.buf, nhwc(xd.grad)):.2e} maxpool_bwd "
          f"{nerr(GP.buf, nhwc(xd2.grad)):.2e}")


def head_case(N, H, W, C, act):
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, generator=g) / C ** 0.5
    gy = torch.randn(N, H, W, generator=g)
    xd, wd = x.double().requires_grad_(True), w.double().requires_grad_(True)
    y = torch.einsum("nchw,c->nhw", xd, wd)
    y = F.relu(y) if act == 1 else (torch.sigmoid(y) if act == 2 else y)
    y.backward(gy.double())
    X = Act(nhwc(x).to(dev))
    Y = K.head_fwd(X, w.to(dev), None, act)
    GX = Act(K.nhwc(N, H, W, C, torch.float32, dev))
    GW = torch.empty(C, device=dev)
    K.head_bwd(X, w.to(dev), act, Y, gy.to(dev), GX, GW)
    torch.cuda.synchronize()
    print(f"head {N}x{H}x{W}x{C} act{act}: fwd {nerr(Y, y.detach()):.2e} gx {nerr(GX.buf, nhwc(xd.grad)):.2e} "
          f"gw {nerr(GW, wd.grad):.2e}")


if __name__ == "__main__":
    for case in [(2, 64, 64, 64, 64, 3), (2, 32, 32, 128, 128, 3), (2, 16, 16, 256, 256, 3), (2, 8, 8, 512, 512, 3),
                 (2, 16, 16, 256, 512, 3), (2, 64, 64, 64, 64, 1), (2, 16, 16, 896, 256, 1)]:
        conv_case(*case)
    for case in [(2, 64, 64, 64, 1, True), (2, 8, 8, 512, 1, True), (2, 64, 64, 64, 1, False),
                 (2, 8, 8, 512, 0, True), (2, 4, 4, 512, 1, True)]:
        bn_case(*case)
    resample_case(2, 16, 16, 64)
    for act in (0, 1, 2):
        head_case(2, 64, 64, 64, act)
