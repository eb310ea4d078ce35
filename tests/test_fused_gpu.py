"""Fused bf16 kernels against their unfused HIP route and a float64 torch reference.

* stem (vgg16_bn.features[0:3], models/models.py:35-36): conv3x3(3->64) read
  straight from the NCHW image + BN partial statistics; BN/ReLU backward fused
  with the weight gradient.  The unfused route (im2col -> K=64 GEMM ->
  dg_bn_fwd_train / dg_bn_bwd -> wgrad) computes the same bf16 values, so z is
  compared bit-for-bit and dW to f32 summation-order tolerance.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _k():
    from dgvcc_amd import kernels as K
    return K


def to_nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def relerr(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("N,H,W", [(2, 32, 64), (2, 8, 128), (1, 16, 256), (3, 5, 64)])
def test_stem_fwd_bwd(dev, N, H, W):
    K = _k()
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(1)
    img = (torch.randn(N, 3, H, W, generator=g) * 0.5).clamp(-1, 1)
    w = torch.randn(64, 3, 3, 3, generator=g) / 27 ** 0.5
    b = torch.randn(64, generator=g) * 0.1 + 2.0  # |mean| >> std: exercises the shifted statistics
    gam = torch.rand(64, generator=g) + 0.5
    bet = torch.randn(64, generator=g) * 0.1
    gy = torch.randn(N, H, W, 64, generator=g)
    imgd, wd, bd = img.to(dev), w.to(dev), b.to(dev)

    # fused route
    wp = K.pack_weight(wd, bf, cpad=3, row_len=32)
    z = K.Act(K.nhwc(N, H, W, 64, bf, dev))
    part, nblk = K.stem_fwd(imgd, wp, bd, z)
    rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
    stats = K.bn_part_finalize(part, nblk, 64, gam.to(dev), bet.to(dev), rm, rv, 0.1, 1e-5)
    # unfused route
    col = K.Act(K.im2col_c3(imgd, bf))
    z0 = K.Act(K.nhwc(N, H, W, 64, bf, dev))
    K.conv_fwd(col, K.pack_weight(wd, bf, cpad=3, row_len=64), 64, 1, 0, z0, bias=bd)
    rm0, rv0 = torch.zeros(64, device=dev), torch.ones(64, device=dev)
    stats0 = K.bn_fwd_train(z0, gam.to(dev), bet.to(dev), rm0, rv0, 0.1, 1e-5)
    torch.cuda.synchronize()
    assert torch.equal(z.buf, z0.buf), "stem z differs from the im2col GEMM"
    # float64 conv on the bf16-rounded operands
    ref = F.conv2d(img.bfloat16().double(), w.bfloat16().double(), b.double(), padding=1)
    assert relerr(z.buf.permute(0, 3, 1, 2), ref) < 8e-3
    zf = z.buf.double().cpu().reshape(-1, 64)
    assert relerr(stats[0], zf.mean(0)) < 1e-6
    assert relerr(stats[1], 1.0 / (zf.var(0, unbiased=False) + 1e-5).sqrt()) < 1e-5
    assert relerr(rv, 0.9 + 0.1 * zf.var(0, unbiased=True)) < 1e-5
    assert relerr(stats, stats0) < 1e-5

    # backward
    g_act = K.Act(gy.to(dev, bf))
    dgam, dbet, dbias = (torch.empty(64, device=dev) for _ in range(3))
    coef = K.bn_bwd_coef(g_act, z, gam.to(dev), stats, 1, dgam, dbet, dbias)
    dw = torch.empty(64, 3, 3, 3, device=dev)
    K.stem_bwd(imgd, g_act, z, stats, coef, dw)
    dz0 = K.Act(K.nhwc(N, H, W, 64, bf, dev))
    dgam0, dbet0, dbias0 = (torch.empty(64, device=dev) for _ in range(3))
    K.bn_bwd(g_act, z, gam.to(dev), stats, 1, dz0, dgam0, dbet0, dbias0)
    dwcol = torch.empty(64, 64, 1, 1, device=dev)
    K.conv_wgrad(col, dz0, 1, 0, dwcol)
    dw0 = torch.empty(64, 3, 3, 3, device=dev)
    K.unpack_c3_grad(dwcol, dw0)
    torch.cuda.synchronize()
    assert torch.equal(dgam, dgam0) and torch.equal(dbet, dbet0) and torch.equal(dbias, dbias0)
    # float64 weight gradient of the (bf16) dz the unfused route materialised
    dz64 = dz0.buf.double().cpu().permute(0, 3, 1, 2)
    wref = torch.nn.grad.conv2d_weight(img.bfloat16().double(), (64, 3, 3, 3), dz64, padding=1)
    assert relerr(dw, wref) < 1e-4
    assert relerr(dw, dw0) < 1e-4
