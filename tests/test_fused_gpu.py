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


@pytest.mark.parametrize("N,H,W", [(2, 32, 64), (1, 16, 256), (3, 5, 64), (2, 128, 1024)])
def test_stem_fwd_f32(dev, N, H, W):
    """fp32 first layer (dg_stem_fwd_f32, exact f32 FMAs) vs the float64 conv, and its BN
    partials vs float64 statistics of the stored z; (2, 128, 1024): several segments per wave."""
    K = _k()
    g = torch.Generator().manual_seed(3)
    img = torch.randn(N, 3, H, W, generator=g)
    w = torch.randn(64, 3, 3, 3, generator=g) / 27 ** 0.5
    b = torch.randn(64, generator=g) * 0.1 + 2.0  # |mean| >> std: exercises the shifted statistics
    gam = torch.rand(64, generator=g) + 0.5
    bet = torch.randn(64, generator=g) * 0.1
    imgd, wd, bd = img.to(dev), w.to(dev), b.to(dev)
    z = K.Act(K.nhwc(N, H, W, 64, torch.float32, dev))
    z.buf.fill_(float("nan"))  # every output must be written
    part, nblk = K.stem_fwd_f32(imgd, K.stem_weight_f32(wd), bd, z)
    rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
    stats = K.bn_part_finalize(part, nblk, 64, gam.to(dev), bet.to(dev), rm, rv, 0.1, 1e-5)
    torch.cuda.synchronize()
    ref = F.conv2d(img.double(), w.double(), b.double(), padding=1)
    assert torch.isfinite(z.buf).all()
    assert relerr(z.buf.permute(0, 3, 1, 2), ref) < 2e-6
    zf = z.buf.double().cpu().reshape(-1, 64)
    assert relerr(stats[0], zf.mean(0)) < 1e-6
    assert relerr(stats[1], 1.0 / (zf.var(0, unbiased=False) + 1e-5).sqrt()) < 1e-5
    assert relerr(rv, 0.9 + 0.1 * zf.var(0, unbiased=True)) < 1e-5
    # the generic route (im2col + split-math GEMM + statistics pass) agrees to its own accuracy
    col = K.Act(K.im2col_c3(imgd, torch.float32))
    z0 = K.Act(K.nhwc(N, H, W, 64, torch.float32, dev))
    K.conv_fwd(col, K.pack_weight(wd, torch.float32, cpad=3, row_len=64), 64, 1, 0, z0, bias=bd)
    torch.cuda.synchronize()
    assert relerr(z.buf, z0.buf) < 1e-5

    # backward (dg_stem_bwd_f32): dz and the wgrad in one pass vs the materialised dz route
    gy = torch.randn(N, H, W, 64, generator=g)
    g_act = K.Act(gy.to(dev))
    dgam, dbet, dbias = (torch.empty(64, device=dev) for _ in range(3))
    coef = K.bn_bwd_coef(g_act, z, gam.to(dev), stats, 1, dgam, dbet, dbias)
    dw = torch.full((64, 3, 3, 3), float("nan"), device=dev)
    K.stem_bwd_f32(imgd, g_act, z, stats, coef, dw)
    dz0 = K.Act(K.nhwc(N, H, W, 64, torch.float32, dev))
    dgam0, dbet0, dbias0 = (torch.empty(64, device=dev) for _ in range(3))
    K.bn_bwd(g_act, z, gam.to(dev), stats, 1, dz0, dgam0, dbet0, dbias0)
    torch.cuda.synchronize()
    assert torch.equal(dgam, dgam0) and torch.equal(dbet, dbet0) and torch.equal(dbias, dbias0)
    dz64 = dz0.buf.double().cpu().permute(0, 3, 1, 2)
    wref = torch.nn.grad.conv2d_weight(img.double(), (64, 3, 3, 3), dz64, padding=1)
    assert torch.isfinite(dw).all()
    assert relerr(dw, wref) < 1e-5
    # accumulate = 1 adds into dw
    dw2 = dw.clone()
    K.stem_bwd_f32(imgd, g_act, z, stats, coef, dw2, accumulate=True)
    torch.cuda.synchronize()
    assert relerr(dw2, 2 * wref) < 1e-5


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

    # z-free route: statistics-only pass, recomputed z in the apply / coefficient / wgrad passes
    part1, nblk1 = K.stem_stats(imgd, wp, bd)
    rm1, rv1 = torch.zeros(64, device=dev), torch.ones(64, device=dev)
    stats1 = K.bn_part_finalize(part1, nblk1, 64, gam.to(dev), bet.to(dev), rm1, rv1, 0.1, 1e-5)
    y1 = K.Act(K.nhwc(N, H, W, 64, bf, dev))
    K.stem_apply(imgd, wp, bd, stats1, y1)
    y0 = K.Act(K.nhwc(N, H, W, 64, bf, dev))
    K.bn_apply(z, stats, 1, y0)
    dgam1, dbet1, dbias1 = (torch.empty(64, device=dev) for _ in range(3))
    coef1 = K.stem_bwd_coef(imgd, wp, bd, g_act, gam.to(dev), stats1, dgam1, dbet1, dbias1)
    dw1 = torch.empty(64, 3, 3, 3, device=dev)
    K.stem_bwd(imgd, g_act, None, stats1, coef1, dw1, wp=wp, bias=bd)
    torch.cuda.synchronize()
    assert torch.equal(part1, part) and torch.equal(stats1, stats)
    assert torch.equal(y1.buf, y0.buf)  # bit for bit: same z bits, same BN-apply arithmetic
    assert relerr(coef1, coef) < 1e-5 and relerr(dgam1, dgam) < 1e-5 and relerr(dbet1, dbet) < 1e-5
    assert relerr(dw1, dw) < 1e-4


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("with_y,with_gd", [(False, False), (True, True)])
@pytest.mark.parametrize("C,H,W", [(64, 8, 12), (256, 6, 4), (512, 4, 8)])
def test_bn_relu_pool_fused(dev, dtype, with_y, with_gd, C, H, W):
    """dg_bn_apply_pool / dg_bn_bwd_pool vs the unfused BN apply + maxpool (+ their backward),
    and vs float64 autograd of BatchNorm2d(train) -> ReLU -> MaxPool2d(2,2) in f32."""
    K = _k()
    N = 2
    g = torch.Generator().manual_seed(3)
    z = torch.randn(N, C, H, W, generator=g)
    z[:, :, :, 1::2] = z[:, :, :, 0::2]  # exact ties inside the pooling windows
    gam = torch.rand(C, generator=g) + 0.5
    bet = torch.randn(C, generator=g) * 0.2
    gp = torch.randn(N, C, H // 2, W // 2, generator=g)
    gd = torch.randn(N, C, H, W, generator=g) if with_gd else None
    if dtype != torch.float32:
        z, gp = z.to(dtype).float(), gp.to(dtype).float()
        gd = gd.to(dtype).float() if gd is not None else None
    zd = K.Act(to_nhwc(z).to(dev, dtype))
    stats = K.bn_fwd_train(zd, gam.to(dev), bet.to(dev), torch.zeros(C, device=dev),
                           torch.ones(C, device=dev), 0.1, 1e-5)
    # fused
    y = K.Act(K.nhwc(N, H, W, C, dtype, dev)) if with_y else None
    yp = K.Act(K.nhwc(N, H // 2, W // 2, C, dtype, dev))
    K.bn_apply_pool(zd, stats, 1, y, yp)
    gpd = K.Act(to_nhwc(gp).to(dev, dtype))
    gdd = K.Act(to_nhwc(gd).to(dev, dtype)) if gd is not None else None
    dz = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
    K.bn_bwd_pool(gpd, gdd, zd, gam.to(dev), stats, 1, dz, dg, db)
    # unfused
    y0 = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    K.bn_apply(zd, stats, 1, y0)
    yp0 = K.Act(K.nhwc(N, H // 2, W // 2, C, dtype, dev))
    K.maxpool_fwd(y0, yp0)
    gy0 = K.Act(gdd.buf.clone()) if gdd is not None else K.Act(K.nhwc(N, H, W, C, dtype, dev, zero=True))
    K.maxpool_bwd(y0, gpd, gy0, accumulate=True)
    dz0 = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    dg0, db0 = torch.empty(C, device=dev), torch.empty(C, device=dev)
    K.bn_bwd(gy0, zd, gam.to(dev), stats, 1, dz0, dg0, db0)
    torch.cuda.synchronize()
    assert torch.equal(yp.buf, yp0.buf)
    if with_y:
        assert torch.equal(y.buf, y0.buf)
    # bf16 with a direct gradient: the unfused route rounds gd + routed gp to bf16 before the BN
    # backward, the fused one adds them in f32
    tol = 1e-5 if (dtype == torch.float32 or not with_gd) else 1e-2
    assert relerr(dg, dg0) < tol and relerr(db, db0) < tol
    assert relerr(dz.buf, dz0.buf) < (1e-5 if dtype == torch.float32 else 1e-2)
    if dtype == torch.float32:  # float64 autograd reference
        zr = z.double().requires_grad_()
        gr, br = gam.double().requires_grad_(), bet.double().requires_grad_()
        a = F.relu(F.batch_norm(zr, None, None, gr, br, training=True, eps=1e-5))
        out = F.max_pool2d(a, 2)
        loss = (out * gp.double()).sum() + ((a * gd.double()).sum() if gd is not None else 0.0)
        loss.backward()
        assert relerr(yp.buf.permute(0, 3, 1, 2), out.detach()) < 1e-5
        assert relerr(dz.buf.permute(0, 3, 1, 2), zr.grad) < 1e-4
        assert relerr(dg, gr.grad) < 1e-4 and relerr(db, br.grad) < 1e-4


@pytest.mark.parametrize("N,H,W,C,Cout", [
    (2, 24, 40, 64, 256),     # pipelined 256-wide tiles, M % 256 != 0 (partial last tile)
    (2, 20, 24, 128, 128),    # pipelined 128-wide tiles
    (1, 8, 256, 64, 64),      # fused 3-tap kernel
    (3, 256, 512, 64, 64),    # fused 3-tap, 1536 partial rows: two-stage merge
    (1, 12, 12, 512, 1024),   # several co tiles
    (16, 48, 64, 256, 512),   # 384 256-channel tiles: persistent 384 x 128 tiles (DGVCC_PERS_WIDE_SMALL)
])
def test_conv_epilogue_bn_stats(dev, N, H, W, C, Cout):
    """dg_conv_fwd_stats (statistics in the conv epilogue) + dg_bn_part_finalize against
    dg_conv_fwd + dg_bn_fwd_train on the same inputs: z bit-identical, statistics ~1e-6."""
    K = _k()
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(4)
    x = torch.randn(N, H, W, C, generator=g).to(dev, bf)
    w = (torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** 0.5).to(dev)
    b = (torch.randn(Cout, generator=g) + 3.0).to(dev)  # |mean| >> std
    gam, bet = torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev)
    wp = K.pack_weight(w, bf)
    z = K.Act(K.nhwc(N, H, W, Cout, bf, dev))
    res = K.conv_fwd_stats(K.Act(x), wp, Cout, 3, 1, z, bias=b)
    assert res is not None
    rm, rv = torch.zeros(Cout, device=dev), torch.ones(Cout, device=dev)
    st = K.bn_part_finalize(res[0], res[1], Cout, gam, bet, rm, rv, 0.1, 1e-5)
    z0 = K.Act(K.nhwc(N, H, W, Cout, bf, dev))
    K.conv_fwd(K.Act(x), wp, Cout, 3, 1, z0, bias=b)
    rm0, rv0 = torch.zeros(Cout, device=dev), torch.ones(Cout, device=dev)
    st0 = K.bn_fwd_train(z0, gam, bet, rm0, rv0, 0.1, 1e-5)
    torch.cuda.synchronize()
    assert torch.equal(z.buf, z0.buf)
    zf = z.buf.double().reshape(-1, Cout)
    assert relerr(st[0], zf.mean(0)) < 1e-6
    assert relerr(st[1], 1.0 / (zf.var(0, unbiased=False) + 1e-5).sqrt()) < 2e-6
    assert relerr(st, st0) < 2e-6 and relerr(rv, rv0) < 2e-6 and relerr(rm, rm0) < 2e-6


@pytest.mark.parametrize("H,W", [(48, 112), (32, 80)])
def test_bf16_model_fallback_shapes(dev, H, W):
    """Shapes outside the fused kernels' tiling (W % 64 != 0: im2col stem; W % 256 != 0: no
    3-tap kernel) take the generic HIP routes: a bf16 DGModel_base train step stays finite and
    matches the fp32 HIP path's count to bf16 accuracy."""
    from oracle import dg_oracle as O
    from dgvcc_amd.models.models import DGModel_base
    from dgvcc_amd.losses import mse_loss
    batch = O.synthetic_batch(2, H, W, seed=3)
    outs = []
    for prec in ("fp32", "bf16"):
        model = DGModel_base(pretrained=False, den_dropout=0.0)
        model.load_state_dict(O.seeded_state_dict(model.state_dict()))
        model = model.to(dev).set_precision(prec).train()
        d = model(batch[0].to(dev))
        loss = mse_loss(d, batch[2][1].to(dev), 1000.0)
        loss.backward()
        assert torch.isfinite(d).all() and torch.isfinite(loss)
        assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in model.parameters())
        outs.append(d.sum().item())
    assert abs(outs[1] - outs[0]) / abs(outs[0]) < 0.1


@pytest.mark.parametrize("N,H,W,C,Cout,acc", [
    (1, 24, 32, 512, 512, False),   # conv5-like at batch 1: 6 tiles -> split 24
    (1, 48, 64, 256, 512, True),    # conv4-like, accumulate into y
    (2, 20, 24, 128, 128, False),   # 128-wide tiles
])
def test_conv_splitk_matches_unsplit(dev, monkeypatch, N, H, W, C, Cout, acc):
    """Small-grid bf16 forwards split their K loop over blocks (f32 partials + a reduce
    pass): same result as the unsplit kernel to f32 summation-order rounding, against a
    float64 reference, with bias, accumulate and the epilogue statistics."""
    K = _k()
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(6)
    x = torch.randn(N, H, W, C, generator=g).to(dev, bf)
    w = (torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** 0.5).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    y0 = torch.randn(N, H, W, Cout, generator=g).to(dev, bf)
    wp = K.pack_weight(w, bf)
    assert K.query("dg_conv_fwd_workspace", 1, N, H, W, C, Cout, 3, 3) > 0
    outs = []
    for split in ("1", "0"):
        monkeypatch.setenv("DGVCC_SPLITK", split)
        K._FWD_WS.clear()
        z = K.Act(y0.clone())
        K.conv_fwd(K.Act(x), wp, Cout, 3, 1, z, bias=b, accumulate=acc)
        zs = K.Act(K.nhwc(N, H, W, Cout, bf, dev))
        res = K.conv_fwd_stats(K.Act(x), wp, Cout, 3, 1, zs, bias=b)
        outs.append((z.buf.clone(), zs.buf.clone(), res))
    K._FWD_WS.clear()
    torch.cuda.synchronize()
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double(), padding=1).permute(0, 2, 3, 1)
    if acc:
        ref = ref + y0.double()
    for z, zs, _ in outs:
        assert relerr(z, ref) < 1e-2
    assert relerr(outs[0][0], outs[1][0]) < 1e-2
    part, rows = outs[0][2]
    rm, rv = torch.zeros(Cout, device=dev), torch.ones(Cout, device=dev)
    st = K.bn_part_finalize(part, rows, Cout, torch.ones(Cout, device=dev), torch.zeros(Cout, device=dev), rm, rv,
                            0.1, 1e-5)
    zf = outs[0][1].double().reshape(-1, Cout)
    assert relerr(st[0], zf.mean(0)) < 1e-6
    assert relerr(st[1], 1.0 / (zf.var(0, unbiased=False) + 1e-5).sqrt()) < 2e-6


@pytest.mark.parametrize("N,H,W,C,Cout", [
    (16, 40, 40, 256, 512),   # conv4 of a 320-px crop
    (16, 20, 20, 512, 512),   # conv5 of a 320-px crop
    (3, 7, 24, 64, 128),      # ragged: K-steps span rows and images, last step partial
    (2, 9, 40, 64, 64),       # Cout 64: the k-half wave split (two slab splits per block)
])
def test_wgrad9_padded_k(dev, monkeypatch, N, H, W, C, Cout):
    """Fused 9-tap bf16 wgrad over the zero-padded K index (W % 64 != 0) against float64
    and against the per-tap kernel it replaces."""
    K = _k()
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(8)
    x = torch.randn(N, H, W, C, generator=g).to(dev, bf)
    dy = torch.randn(N, H, W, Cout, generator=g).to(dev, bf)
    outs = []
    for pad in ("1", "0"):
        monkeypatch.setenv("DGVCC_WG9_PAD", pad)
        dw = torch.empty(Cout, C, 3, 3, device=dev)
        K.conv_wgrad(K.Act(x), K.Act(dy), 3, 1, dw)
        outs.append(dw)
    torch.cuda.synchronize()
    xr = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    wr = torch.zeros(Cout, C, 3, 3, dtype=torch.float64, device=dev, requires_grad=True)
    F.conv2d(xr, wr, padding=1).backward(dy.double().permute(0, 3, 1, 2))
    assert relerr(outs[0], wr.grad) < 1e-5
    assert relerr(outs[0], outs[1]) < 1e-5


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("N,H,W,C,Cin_next,act,use_drop", [
    (4, 128, 256, 256, 256, 1, False),   # 256-wide tiles (grids large enough not to split K / > 256 tiles)
    (4, 120, 300, 128, 256, 1, True),    # 128-wide tiles, ragged last tile, Dropout2d mask
    (2, 128, 256, 512, 512, 0, False),   # two channel tiles, no ReLU
])
def test_dgrad_epilogue_bn_partials(dev, monkeypatch, dtype, N, H, W, C, Cin_next, act, use_drop):
    """dg_conv_fwd_bnbwd (BN-backward partial sums in the dgrad epilogue: the bf16 pipe kernel,
    the fp32 pre-split kernel's EPI 2) + dg_bn_bwd_from_part against dg_conv_dgrad + dg_bn_bwd on
    the same inputs: gx bit-identical, dz/dgamma/dbeta to f32 summation-order rounding."""
    K = _k()
    monkeypatch.setattr(K, "_BNPART_OFF", False)
    monkeypatch.setattr(K, "_BNPART_F32_OFF", False)
    bf = dtype
    g = torch.Generator().manual_seed(9)
    dz_next = torch.randn(N, H, W, Cin_next, generator=g).to(dev, bf)
    w = (torch.randn(Cin_next, C, 3, 3, generator=g) / (9 * C) ** 0.5).to(dev)
    z = torch.randn(N, H, W, C, generator=g).to(dev, bf)
    gam, bet = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    st = K.bn_fwd_train(K.Act(z), gam, bet, rm, rv, 0.1, 1e-5)
    drop = ((torch.rand(N, C, generator=g) > 0.3).float() / 0.7).to(dev) if use_drop else None
    wp = K.pack_weight(w, bf)
    gx1 = K.Act(K.nhwc(N, H, W, C, bf, dev))
    pre = K.conv_dgrad_bnpart(K.Act(dz_next), wp, C, 3, 1, gx1, K.Act(z), st, act, drop)
    assert pre is not None
    dz1 = K.Act(K.nhwc(N, H, W, C, bf, dev))
    dg1, db1 = torch.empty(C, device=dev), torch.empty(C, device=dev)
    K.bn_bwd_from_part(pre, gx1, K.Act(z), gam, st, act, dz1, dg1, db1, None, drop)
    gx0 = K.Act(K.nhwc(N, H, W, C, bf, dev))
    K.conv_dgrad(K.Act(dz_next), wp, C, 3, 1, gx0)
    dz0 = K.Act(K.nhwc(N, H, W, C, bf, dev))
    dg0, db0 = torch.empty(C, device=dev), torch.empty(C, device=dev)
    K.bn_bwd(gx0, K.Act(z), gam, st, act, dz0, dg0, db0, None, drop)
    torch.cuda.synchronize()
    assert torch.equal(gx1.buf, gx0.buf)
    assert relerr(dg1, dg0) < 1e-5 and relerr(db1, db0) < 1e-5
    if dtype == torch.float32:
        assert relerr(dz1.buf, dz0.buf) < 1e-5
        return
    assert relerr(dz1.buf, dz0.buf) < 1e-2  # bf16 storage: rare 1-ulp flips from the coefficients
    assert (dz1.buf.float() - dz0.buf.float()).abs().max() <= 2 * dz0.buf.float().abs().max() * 2 ** -8


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W,C,Cout,act", [(1, 24, 32, 256, 512, 1), (2, 16, 256, 64, 64, 1), (1, 32, 48, 128, 128, 0)])
def test_conv_bn_eval_epilogue(dev, dtype, N, H, W, C, Cout, act):
    """dg_conv_fwd_bn_eval (eval BN + ReLU in the conv epilogue) against dg_conv_fwd +
    dg_bn_apply: f32 bit-identical; bf16 within one bf16 ulp (z is no longer rounded)."""
    K = _k()
    g = torch.Generator().manual_seed(10)
    x = torch.randn(N, H, W, C, generator=g).to(dev, dtype)
    w = (torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** 0.5).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    gam, bet = torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev)
    rm, rv = torch.randn(Cout, device=dev) * 0.1, torch.rand(Cout, device=dev) + 0.5
    st = K.bn_eval_stats(gam, bet, rm, rv, 1e-5)
    wp = K.pack_weight(w, dtype)
    y1 = K.Act(K.nhwc(N, H, W, Cout, dtype, dev))
    K.conv_fwd_bn_eval(K.Act(x), wp, Cout, 3, 1, y1, b, st, act)
    z = K.Act(K.nhwc(N, H, W, Cout, dtype, dev))
    K.conv_fwd(K.Act(x), wp, Cout, 3, 1, z, bias=b)
    y0 = K.Act(K.nhwc(N, H, W, Cout, dtype, dev))
    K.bn_apply(z, st, act, y0)
    torch.cuda.synchronize()
    if dtype == torch.float32:
        assert torch.equal(y1.buf, y0.buf)
    else:  # the unfused route rounds z to bf16 before scaling: error ~ |z * scale| * 2^-8
        d = (y1.buf.float() - y0.buf.float()).abs()
        zs = (z.buf.float() * st[2]).abs()
        assert (d <= zs * 2 ** -7 + y0.buf.float().abs() * 2 ** -7 + 1e-3).all()


@pytest.mark.parametrize("N,H,W,C,acc", [(2, 20, 40, 64, False), (3, 7, 24, 128, True), (1, 320, 320, 64, False)])
def test_tap3_padded_index(dev, monkeypatch, N, H, W, C, acc):
    """Cout = 64 bf16 3x3 forward with W % 256 != 0 on the 3-tap kernel over the padded pixel
    index (tiles spanning rows and images) against float64 and against the per-tap kernel;
    the epilogue-statistics entry point declines such shapes (the caller then runs the
    statistics pass)."""
    K = _k()
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(12)
    x = torch.randn(N, H, W, C, generator=g).to(dev, bf)
    w = (torch.randn(64, C, 3, 3, generator=g) / (9 * C) ** 0.5).to(dev)
    b = torch.randn(64, generator=g).to(dev)
    y0 = torch.randn(N, H, W, 64, generator=g).to(dev, bf)
    wp = K.pack_weight(w, bf)
    outs = []
    for pad in ("1", "0"):
        monkeypatch.setenv("DGVCC_TAP3_PAD", pad)
        y = K.Act(y0.clone())
        K.conv_fwd(K.Act(x), wp, 64, 3, 1, y, bias=b, accumulate=acc)
        outs.append(y.buf)
    zs = K.Act(K.nhwc(N, H, W, 64, bf, dev))
    monkeypatch.setenv("DGVCC_TAP3_PAD", "1")
    assert K.conv_fwd_stats(K.Act(x), wp, 64, 3, 1, zs, bias=b) is None
    torch.cuda.synchronize()
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double(), padding=1).permute(0, 2, 3, 1)
    if acc:
        ref = ref + y0.double()
    assert relerr(outs[0], ref) < 1e-2
    assert relerr(outs[0], outs[1]) < 1e-2


@pytest.mark.parametrize("N,H,W,C,Cout,stats", [(5, 128, 256, 64, 256, True), (3, 96, 320, 128, 128, True),
                                                (5, 128, 256, 128, 256, False), (2, 48, 64, 128, 1024, False),
                                                (2, 48, 64, 128, 1024, "eval"), (3, 64, 64, 64, 256, "eval"),
                                                (3, 64, 64, 128, 128, "eval")])
def test_persistent_conv_matches(dev, monkeypatch, N, H, W, C, Cout, stats):
    """The persistent pipelined forward (tiles walked by one block per CU, DMA ring running
    across tile boundaries) against the one-tile-per-block kernel: bit-identical outputs and
    statistics partials (same K order per tile); Cout = 1024 (two passes of the block's LDS
    bias fill); the eval-BN epilogue (bias, scale, shift staged in LDS, or read from global
    memory when 3 x Cout floats exceed the statistics scratch: the 1024-channel 128-wide case)."""
    K = _k()
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(13)
    x = torch.randn(N, H, W, C, generator=g).to(dev, bf)
    w = (torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** 0.5).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    wp = K.pack_weight(w, bf)
    outs = []
    for pers in ("0", "1"):
        monkeypatch.setenv("DGVCC_PERSIST", pers)
        K.call("dg_set_persist", int(pers))
        z = K.Act(K.nhwc(N, H, W, Cout, bf, dev))
        if stats == "eval":
            st = torch.stack([torch.zeros(Cout), torch.ones(Cout), torch.rand(Cout, generator=g) + 0.5,
                              torch.randn(Cout, generator=g) * 0.1]).to(dev) if pers == "0" else st
            K.conv_fwd_bn_eval(K.Act(x), wp, Cout, 3, 1, z, b, st, 1)
            outs.append((z.buf.clone(), None))
        elif stats:
            res = K.conv_fwd_stats(K.Act(x), wp, Cout, 3, 1, z, bias=b)
            outs.append((z.buf.clone(), res[0].clone()))
        else:
            K.conv_fwd(K.Act(x), wp, Cout, 3, 1, z, bias=b)
            outs.append((z.buf.clone(), None))
    K.call("dg_set_persist", -1)
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    if stats is True:
        assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("N,H,W,C,Cout", [(4, 192, 256, 64, 256), (8, 96, 128, 128, 512)])
def test_persistent_short_k_1x1(dev, monkeypatch, N, H, W, C, Cout):
    """bf16 1x1 convs of one or two 64-channel K-steps (the trunks' bottleneck expansions) on the
    persistent forward (DGVCC_PERS_SHORTK, default) against the one-tile-per-block pipe kernel
    they ran on before: bit-identical outputs and statistics partials (same K order per tile),
    and the outputs against float64."""
    K = _k()
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(17)
    x = torch.randn(N, H, W, C, generator=g).to(dev, bf)
    w = (torch.randn(Cout, C, 1, 1, generator=g) / C ** 0.5).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    wp = K.pack_weight(w, bf)
    outs = []
    for sk in ("1", "0"):
        monkeypatch.setenv("DGVCC_PERS_SHORTK", sk)
        z = K.Act(K.nhwc(N, H, W, Cout, bf, dev))
        res = K.conv_fwd_stats(K.Act(x), wp, Cout, 1, 0, z, bias=b)
        assert res is not None
        outs.append((z.buf.clone(), res[0].clone()))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double()).permute(0, 2, 3, 1)
    assert relerr(outs[0][0], ref) < 1e-2


@pytest.mark.parametrize("N,H,W,acc", [(2, 16, 256, False), (5, 128, 256, True), (3, 40, 512, False),
                                       (1, 15, 256, True), (3, 48, 256, False)])
def test_tap3_persistent_matches(dev, monkeypatch, N, H, W, acc):
    """C = Cout = 64 row-aligned 3x3 (enc1.3 and its dgrad): the persistent resident-filter
    kernel (conv_fwd_tap3p_kernel; grids below and above one block per CU) against the
    one-tile-per-block 3-tap kernel: bit-identical forward (+accumulate), BN statistics
    partials, eval-BN epilogue and dgrad (same K order per output row) with one, two or three
    output rows per tile (rows not dividing H fall back to fewer), and within bf16 rounding of
    float64."""
    K = _k()
    bf = torch.bfloat16
    g = torch.Generator().manual_seed(14)
    x = torch.randn(N, H, W, 64, generator=g).to(dev, bf)
    gy = torch.randn(N, H, W, 64, generator=g).to(dev, bf)
    w = (torch.randn(64, 64, 3, 3, generator=g) / 24.0).to(dev)
    b = torch.randn(64, generator=g).to(dev)
    y0 = torch.randn(N, H, W, 64, generator=g).to(dev, bf)
    gam, bet = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev)
    st = K.bn_eval_stats(gam, bet, torch.randn(64, device=dev) * 0.1, torch.rand(64, device=dev) + 0.5, 1e-5)
    wp = K.pack_weight(w, bf)
    outs = []
    for p, rows in (("0", "2"), ("1", "1"), ("1", "2"), ("1", "3")):  # ROWS rows per tile need H % ROWS == 0
        monkeypatch.setenv("DGVCC_TAP3P", p)
        monkeypatch.setenv("DGVCC_TAP3P_ROWS", rows)
        y = K.Act(y0.clone())
        K.conv_fwd(K.Act(x), wp, 64, 3, 1, y, bias=b, accumulate=acc)
        z = K.Act(K.nhwc(N, H, W, 64, bf, dev))
        res = K.conv_fwd_stats(K.Act(x), wp, 64, 3, 1, z, bias=b)
        ye = K.Act(K.nhwc(N, H, W, 64, bf, dev))
        K.conv_fwd_bn_eval(K.Act(x), wp, 64, 3, 1, ye, b, st, 1)
        dx = K.Act(K.nhwc(N, H, W, 64, bf, dev))
        K.conv_dgrad(K.Act(gy), wp, 64, 3, 1, dx)
        torch.cuda.synchronize()
        outs.append((y.buf.clone(), z.buf.clone(), res[0].clone(), ye.buf.clone(), dx.buf.clone()))
    for o in outs[1:]:
        for u, v in zip(outs[0], o):
            assert torch.equal(u, v)
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double(), padding=1).permute(0, 2, 3, 1)
    if acc:
        ref = ref + y0.double()
    assert relerr(outs[1][0], ref) < 1e-2
    refd = F.conv_transpose2d(gy.double().permute(0, 3, 1, 2), w.double(), padding=1).permute(0, 2, 3, 1)
    assert relerr(outs[1][4], refd) < 1e-2


# ---------------------------------------------------------------------------
# models2.DensityRegressorM pieces: KL-JSD of the slot posteriors, L1 of the instance norms,
# tanh (Generator heads) — against float64 torch autograd of the reference's formulas
# (models/models2.py:326-346, :334, :50)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("C", [1024, 512])
def test_softmax_jsd_matches_reference_formula(dev, C):
    import torch.nn.functional as F
    from dgvcc_amd import kernels as K
    B, HW = 2, 96
    g = torch.Generator().manual_seed(4)
    l1 = torch.randn(B * HW, C, generator=g) * 2
    l2 = l1 + 0.3 * torch.randn(B * HW, C, generator=g)
    gp1 = torch.randn(B * HW, C, generator=g) * 1e-3
    coef = 1.7
    # reference: logits [B, C, HW], softmax / log_softmax over the slot dim
    a = l1.double().view(B, HW, C).permute(0, 2, 1).requires_grad_(True)
    b = l2.double().view(B, HW, C).permute(0, 2, 1).requires_grad_(True)
    p1, p2 = F.softmax(a, 1), F.softmax(b, 1)
    pm = (p1 + p2) / 2
    loss = 0.5 / HW * (F.kl_div(F.log_softmax(a, 1), pm, reduction="batchmean")
                       + F.kl_div(F.log_softmax(b, 1), pm, reduction="batchmean"))
    (coef * loss + (p1 * gp1.double().view(B, HW, C).permute(0, 2, 1)).sum()).backward()
    P1 = torch.empty(B * HW, C, device=dev)
    P2 = torch.empty_like(P1)
    lk = torch.empty((), device=dev)
    ws = K.query("dg_softmax_workspace", B * HW)
    work = torch.empty(ws // 4 + 1, device=dev)
    L1, L2 = l1.to(dev), l2.to(dev)
    K.call("dg_softmax_jsd_fwd", 0, K.ptr(L1), K.ptr(L2), B * HW, C, K.ptr(P1), K.ptr(P2), K.ptr(lk), K.ptr(work),
           K.stream())
    G1 = gp1.to(dev)
    GL1, GL2 = torch.empty_like(P1), torch.empty_like(P1)
    cf = torch.tensor([coef], device=dev)
    K.call("dg_softmax_jsd_bwd", 0, K.ptr(P1), K.ptr(P2), K.ptr(G1), None, B * HW, C, K.ptr(cf), K.ptr(GL1),
           K.ptr(GL2), K.stream())
    torch.cuda.synchronize()
    assert abs(lk.item() - loss.item()) <= 1e-5 * abs(loss.item()), (lk.item(), loss.item())
    assert relerr(P1, p1.detach().permute(0, 2, 1).reshape(B * HW, C)) < 1e-5
    ga = a.grad.permute(0, 2, 1).reshape(B * HW, C)
    gb = b.grad.permute(0, 2, 1).reshape(B * HW, C)
    assert ((GL1.double().cpu() - ga).norm() / ga.norm()).item() < 1e-4
    assert ((GL2.double().cpu() - gb).norm() / gb.norm()).item() < 1e-4


def test_instance_norm_l1_loss_and_grad(dev):
    import torch.nn.functional as F
    from dgvcc_amd import kernels as K
    N, H, W, C = 2, 6, 5, 32
    g = torch.Generator().manual_seed(8)
    y1 = torch.randn(N, H, W, C, generator=g) * 1.5 + 0.3
    y2 = y1 + 0.4 * torch.randn(N, H, W, C, generator=g)
    a = y1.double().permute(0, 3, 1, 2).requires_grad_(True)
    b = y2.double().permute(0, 3, 1, 2).requires_grad_(True)
    loss = F.l1_loss(F.instance_norm(a, eps=1e-5), F.instance_norm(b, eps=1e-5))
    (0.7 * loss).backward()
    Y1, Y2 = K.Act(y1.to(dev)), K.Act(y2.to(dev))
    s1, s2 = K.instnorm_stats(Y1), K.instnorm_stats(Y2)
    out = torch.empty((), device=dev)
    ws = K.query("dg_in_l1_workspace", N, H * W, C)
    work = torch.empty(ws // 4 + 1, device=dev)
    K.call("dg_in_l1_fwd", 0, Y1.ptr, Y2.ptr, C, N, H * W, C, K.ptr(s1[0]), K.ptr(s1[1]), K.ptr(s2[0]),
           K.ptr(s2[1]), K.ptr(out), K.ptr(work), K.stream())
    gi1, gi2 = K.Act(torch.empty_like(Y1.buf)), K.Act(torch.empty_like(Y2.buf))
    cf = torch.tensor([0.7], device=dev)
    K.call("dg_in_l1_bwd", 0, Y1.ptr, Y2.ptr, C, N, H * W, C, K.ptr(s1[0]), K.ptr(s1[1]), K.ptr(s2[0]),
           K.ptr(s2[1]), K.ptr(cf), gi1.ptr, gi2.ptr, K.stream())
    g1, g2 = K.Act(torch.empty_like(Y1.buf)), K.Act(torch.empty_like(Y2.buf))
    K.instnorm_bwd(gi1, Y1, s1, None, g1)
    K.instnorm_bwd(gi2, Y2, s2, None, g2)
    torch.cuda.synchronize()
    assert abs(out.item() - loss.item()) <= 1e-5 * loss.item()
    assert relerr(g1.buf, a.grad.permute(0, 2, 3, 1)) < 1e-4
    assert relerr(g2.buf, b.grad.permute(0, 2, 3, 1)) < 1e-4


def test_tanh_fwd_bwd(dev):
    from dgvcc_amd import kernels as K
    x = torch.randn(3, 1000, generator=torch.Generator().manual_seed(2)) * 3
    gy = torch.randn(3, 1000, generator=torch.Generator().manual_seed(3))
    X, GY = x.to(dev), gy.to(dev)
    Y, GX = torch.empty_like(X), torch.empty_like(X)
    K.call("dg_tanh_fwd", K.ptr(X), X.numel(), K.ptr(Y), K.stream())
    K.call("dg_tanh_bwd", K.ptr(Y), K.ptr(GY), X.numel(), K.ptr(GX), 0, K.stream())
    torch.cuda.synchronize()
    xd = x.double().requires_grad_(True)
    torch.tanh(xd).backward(gy.double())
    assert relerr(Y, torch.tanh(x.double())) < 1e-6
    assert relerr(GX, xd.grad) < 1e-5


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W,C,Cout,acc,off", [(4, 96, 128, 64, 256, False, 0), (2, 48, 64, 128, 512, True, 0),
                                                  (2, 24, 32, 64, 256, False, 0), (16, 48, 64, 64, 256, False, 0),
                                                  (2, 37, 29, 64, 256, True, 0), (4, 96, 128, 64, 256, False, 4)])
def test_persistent_wide_stores(dev, monkeypatch, dtype, N, H, W, C, Cout, acc, off):
    """16-byte epilogue stores of the short-K 16-bit persistent forward (lane pairs exchange
    channel halves with v_permlane16_swap, DGVCC_PERS_WST) against the 8-byte stores:
    bit-identical outputs, accumulate and ragged pixel tails included; a y slice that is only
    8-byte aligned (off = 4 channels) takes the 8-byte stores."""
    K = _k()
    g = torch.Generator().manual_seed(23)
    x = torch.randn(N, H, W, C, generator=g).to(dev, dtype)
    wp = K.pack_weight((torch.randn(Cout, C, 1, 1, generator=g) / C ** 0.5).to(dev), dtype)
    b = torch.randn(Cout, generator=g).to(dev)
    base = torch.randn(N, H, W, Cout + 8, generator=g).to(dev, dtype)
    outs = []
    for wst in ("0", "1"):
        monkeypatch.setenv("DGVCC_PERS_WST", wst)
        yb = base.clone()
        y = K.Act(yb, off, Cout)
        K.conv_fwd(K.Act(x), wp, Cout, 1, 0, y, bias=None if acc else b, accumulate=acc)
        outs.append(yb)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert not torch.equal(outs[0], base)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W,C,Cout,R,acc,bias", [(1, 37, 41, 64, 256, 3, False, True), (2, 19, 23, 128, 128, 3, True, False),
                                                     (1, 33, 29, 64, 256, 1, False, False), (3, 11, 13, 192, 128, 3, False, True)])
def test_pipe_wide_stores(dev, monkeypatch, dtype, N, H, W, C, Cout, R, acc, bias):
    """16-byte epilogue stores of the one-tile-per-block pipe kernel (conv_fwd_pipe_kernel, forced by
    dg_set_persist(0); opt-in with DGVCC_PIPE_WST=1, 8-byte stores otherwise): bit-identical outputs on ragged pixel
    tails (N*H*W not a multiple of the 256-pixel tile), with and without bias, accumulating or not, both
    16-bit types, BN = 256 (2 stages) and 128 (3 stages)."""
    K = _k()
    g = torch.Generator().manual_seed(29)
    x = torch.randn(N, H, W, C, generator=g).to(dev, dtype)
    w = (torch.randn(Cout, C, R, R, generator=g) / (C * R * R) ** 0.5).to(dev)
    wp = K.pack_weight(w, dtype)
    b = torch.randn(Cout, generator=g).to(dev) if bias else None
    base = torch.randn(N, H, W, Cout, generator=g).to(dev, dtype)
    assert (N * H * W) % 256 != 0
    outs = []
    K.call("dg_set_persist", 0)
    try:
        for wst in ("0", "1"):
            monkeypatch.setenv("DGVCC_PIPE_WST", wst)
            yb = base.clone()
            K.conv_fwd(K.Act(x), wp, Cout, R, R // 2, K.Act(yb), bias=b, accumulate=acc)
            outs.append(yb)
        torch.cuda.synchronize()
    finally:
        K.call("dg_set_persist", -1)
    assert torch.equal(outs[0], outs[1])
    assert not torch.equal(outs[0], base)
    # and against torch on the rounded operands
    xr = x.float().permute(0, 3, 1, 2)
    ref = F.conv2d(xr, w.to(dtype).float(), bias=b, padding=R // 2).permute(0, 2, 3, 1)
    if acc:
        ref = ref + base.float()
    assert relerr(outs[1].float(), ref) < 2e-2
