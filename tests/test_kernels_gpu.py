"""Per-kernel numerics on the GPU against plain PyTorch fp32 on the CPU.

f32 (parity mode) must agree to ~1e-5 relative (exact-f32 MFMA, different
summation order); bf16 (perf mode) is compared against the CPU op applied to
the same bf16-rounded inputs with a bf16-output tolerance.
"""
import os
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _k():
    from dgvcc_amd import kernels as K
    return K


def to_nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def to_nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


def relerr(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


DTYPES = [torch.float32, torch.bfloat16, torch.float16]

CONV_CASES = [
    # N, H, W, C, Cout, R
    (2, 20, 24, 64, 128, 3),
    (1, 16, 16, 128, 64, 3),
    (2, 9, 13, 64, 64, 3),
    (1, 12, 8, 256, 128, 1),
    (1, 8, 8, 896, 256, 1),
    (1, 4, 256, 64, 64, 3),     # Cout 64, W % 256 == 0: fused 3-tap forward (+ its dgrad)
    (2, 6, 128, 64, 64, 3),     # Cout 64 9-tap wgrad: k-half wave split over several splits
    (2, 3, 512, 128, 64, 3),    # fused 3-tap forward with 2 channel blocks
    (2, 3, 512, 64, 128, 3),    # dgrad into 64 channels on the fused 3-tap kernel
]


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(dev, dtype, case):
    K = _k()
    N, H, W, C, Cout, R = case
    pad = R // 2
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(Cout, C, R, R, generator=g) / (C * R * R) ** 0.5
    b = torch.randn(Cout, generator=g)
    gy = torch.randn(N, Cout, H, W, generator=g)
    if dtype != torch.float32:  # reference on the rounded operands
        x = x.to(dtype).float()
        w = w.to(dtype).float()
        gy = gy.to(dtype).float()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, b, padding=pad)
    yr.backward(gy)

    xd = K.Act(to_nhwc(x).to(dev, dtype))
    wp = K.pack_weight(w.to(dev), dtype)
    y = K.Act(K.nhwc(N, H, W, Cout, dtype, dev))
    K.conv_fwd(xd, wp, Cout, R, pad, y, bias=b.to(dev))
    gyd = K.Act(to_nhwc(gy).to(dev, dtype))
    dx = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    K.conv_dgrad(gyd, wp, C, R, pad, dx)
    dw = torch.empty(Cout, C, R, R, device=dev)
    K.conv_wgrad(xd, gyd, R, pad, dw)
    torch.cuda.synchronize()
    tol = 2e-5 if dtype == torch.float32 else 1.5e-2
    assert relerr(to_nchw(y.buf.float()), yr.detach()) < tol
    assert relerr(to_nchw(dx.buf.float()), xr.grad) < tol
    wtol = 2e-5 if dtype == torch.float32 else 2e-3  # f32 accumulation of bf16 products
    assert relerr(dw, wr.grad) < wtol


def test_conv_slices_and_accumulate(dev):
    """Input/output as channel slices of wider NHWC buffers (the decoder concat)."""
    K = _k()
    N, H, W = 1, 10, 12
    g = torch.Generator().manual_seed(1)
    big = torch.randn(N, H, W, 192, generator=g)
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.1
    x = big[..., 64:128]
    ref = F.conv2d(to_nchw(x), w, padding=1)
    out = torch.randn(N, H, W, 128, generator=g)
    base = out.clone()
    xd = K.Act(big.to(dev), 64, 64)
    od = K.Act(out.to(dev), 32, 64)
    K.conv_fwd(xd, K.pack_weight(w.to(dev), torch.float32), 64, 3, 1, od, accumulate=True)
    torch.cuda.synchronize()
    res = od.buf.cpu()
    assert relerr(to_nchw(res[..., 32:96] - base[..., 32:96]), ref) < 2e-5
    assert torch.equal(res[..., :32], base[..., :32]) and torch.equal(res[..., 96:], base[..., 96:])


def test_first_layer_im2col(dev):
    K = _k()
    N, H, W = 2, 16, 20
    g = torch.Generator().manual_seed(2)
    img = torch.randn(N, 3, H, W, generator=g)
    w = torch.randn(64, 3, 3, 3, generator=g) * 0.2
    b = torch.randn(64, generator=g)
    gy = torch.randn(N, 64, H, W, generator=g)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(img, wr, b, padding=1)
    yr.backward(gy)
    col = K.Act(K.im2col_c3(img.to(dev), torch.float32))
    wp = K.pack_weight(w.to(dev), torch.float32, cpad=3, row_len=64)
    y = K.Act(K.nhwc(N, H, W, 64, torch.float32, dev))
    K.conv_fwd(col, wp, 64, 1, 0, y, bias=b.to(dev))
    dwcol = torch.empty(64, 64, 1, 1, device=dev)
    K.conv_wgrad(col, K.Act(to_nhwc(gy).to(dev)), 1, 0, dwcol)
    dw = torch.empty(64, 3, 3, 3, device=dev)
    K.unpack_c3_grad(dwcol, dw)
    torch.cuda.synchronize()
    assert relerr(to_nchw(y.buf), yr.detach()) < 2e-5
    assert relerr(dw, wr.grad) < 2e-5


@pytest.mark.parametrize("case", [(1, 256, 288, 64, 256, 3), (1, 256, 288, 128, 128, 3), (1, 256, 288, 64, 64, 3),
                                  (1, 256, 288, 256, 512, 1)])
def test_conv_f32_persistent(dev, monkeypatch, case):
    """f32 forward/dgrad on the persistent LDS-DMA kernel (> 256 tiles of 256 pixels, 32-channel
    K-steps; BN = 256 / 128 / 64 and a 1x1) against torch fp32, and against the register-staged
    conv_fwd_kernel (DGVCC_F32_PERSIST=0, read per launch) within f32 summation-order noise."""
    test_conv_fwd_dgrad_wgrad(dev, torch.float32, case)
    K = _k()
    N, H, W, C, Cout, R = case
    g = torch.Generator().manual_seed(1)
    x = K.Act(torch.randn(N, H, W, C, generator=g).to(dev))
    wp = K.pack_weight((torch.randn(Cout, C, R, R, generator=g) / (C * R * R) ** 0.5).to(dev), torch.float32)
    outs = []
    prev = K.lib_call_status("dg_get_f32_math")
    K.call("dg_set_f32_math", 0)  # both on v_mfma_f32_16x16x4_f32 (the split math: test_conv_f32_split_math)
    try:
        for flag in ("1", "0"):
            monkeypatch.setenv("DGVCC_F32_PERSIST", flag)
            y = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
            K.conv_fwd(x, wp, Cout, R, R // 2, y)
            outs.append(y.buf.clone())
        torch.cuda.synchronize()
    finally:
        K.call("dg_set_f32_math", prev)
    assert relerr(outs[0], outs[1]) < 2e-6


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("C,H,W", [(64, 12, 10), (256, 16, 16), (512, 8, 8), (1024, 6, 4), (128, 40, 33)])
def test_bn_train_fwd_bwd(dev, dtype, act, C, H, W):
    K = _k()
    N = 2
    g = torch.Generator().manual_seed(3)
    z = (torch.randn(N, C, H, W, generator=g) * 3 + 5)
    if dtype != torch.float32:
        z = z.to(dtype).float()
    gam = torch.rand(C, generator=g) + 0.5
    bet = torch.randn(C, generator=g)
    gy = torch.randn(N, C, H, W, generator=g)
    if dtype != torch.float32:
        gy = gy.to(dtype).float()
    bn = torch.nn.BatchNorm2d(C)
    bn.weight.data.copy_(gam)
    bn.bias.data.copy_(bet)
    zr = z.clone().requires_grad_(True)
    yr = bn(zr)
    if act:
        yr = F.relu(yr)
    yr.backward(gy)

    rm = torch.zeros(C, device=dev)
    rv = torch.ones(C, device=dev)
    zd = K.Act(to_nhwc(z).to(dev, dtype))
    stats = K.bn_fwd_train(zd, gam.to(dev), bet.to(dev), rm, rv, 0.1, 1e-5)
    y = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    K.bn_apply(zd, stats, act, y)
    dz = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    dgam = torch.empty(C, device=dev)
    dbet = torch.empty(C, device=dev)
    K.bn_bwd(K.Act(to_nhwc(gy).to(dev, dtype)), zd, gam.to(dev), stats, act, dz, dgam, dbet)
    torch.cuda.synchronize()
    tol = 2e-5 if dtype == torch.float32 else 1e-2
    assert relerr(to_nchw(y.buf.float()), yr.detach()) < tol
    assert relerr(rm, bn.running_mean) < 1e-5 and relerr(rv, bn.running_var) < 1e-5
    assert relerr(to_nchw(dz.buf.float()), zr.grad) < (1e-4 if dtype == torch.float32 else 2e-2)
    assert relerr(dgam, bn.weight.grad) < 1e-4 and relerr(dbet, bn.bias.grad) < 1e-4


@pytest.mark.parametrize("dtype", DTYPES)
def test_maxpool(dev, dtype):
    K = _k()
    N, H, W, C = 2, 8, 12, 64
    g = torch.Generator().manual_seed(4)
    x = F.relu(torch.randn(N, C, H, W, generator=g)).to(dtype).float()  # many ties at 0
    gy = torch.randn(N, C, H // 2, W // 2, generator=g).to(dtype).float()
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 2, 2)
    yr.backward(gy)
    xd = K.Act(to_nhwc(x).to(dev, dtype))
    y = K.Act(K.nhwc(N, H // 2, W // 2, C, dtype, dev))
    K.maxpool_fwd(xd, y)
    gx = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    K.maxpool_bwd(xd, K.Act(to_nhwc(gy).to(dev, dtype)), gx)
    torch.cuda.synchronize()
    assert torch.equal(to_nchw(y.buf.float()).cpu(), yr.detach())
    assert torch.equal(to_nchw(gx.buf.float()).cpu(), xr.grad)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("scale,mode,C", [(2, 0, 64), (4, 0, 512), (4, 2, 1), (16, 1, 1), (4, 0, 1), (2, 1, 16)])
def test_upsample(dev, dtype, scale, mode, C):
    K = _k()
    N, H, W = 2, 6, 5
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N, C, H, W, generator=g).to(dtype).float()
    gy = torch.randn(N, C, H * scale, W * scale, generator=g).to(dtype).float()
    xr = x.clone().requires_grad_(True)
    if mode == 2:
        yr = F.interpolate(xr, scale_factor=scale, mode="nearest")
    else:
        yr = F.interpolate(xr, scale_factor=scale, mode="bilinear", align_corners=(mode == 1))
    yr.backward(gy)
    xd = K.Act(to_nhwc(x).to(dev, dtype))
    y = K.Act(K.nhwc(N, H * scale, W * scale, C, dtype, dev))
    K.upsample_fwd(xd, scale, mode, y)
    gx = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    K.upsample_bwd(K.Act(to_nhwc(gy).to(dev, dtype)), scale, mode, gx)
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert relerr(to_nchw(y.buf.float()), yr.detach()) < tol
    assert relerr(to_nchw(gx.buf.float()), xr.grad) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("scale,mode,N,H,W", [(4, 0, 2, 24, 40), (16, 1, 2, 6, 10), (2, 1, 1, 9, 7), (8, 0, 1, 5, 12),
                                              (16, 1, 1, 3, 600), (4, 0, 1, 2, 1100)])
def test_upsample_c1(dev, dtype, scale, mode, N, H, W):
    """C = 1 maps (upsample_fwd_c1_kernel / upsample_bwd_c1_kernel, the latter in several input-column tiles
    for W = 600 / 1100): forward and backward (with a second gradient and accumulation) against torch, and
    against the per-pixel kernels (DGVCC_UP_C1_OFF=1), both within f32 rounding (the compiler contracts the
    same expression into different FMAs in the two forms)."""
    K = _k()
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, 1, H, W, generator=g).to(dtype).float()
    gy = torch.randn(N, 1, H * scale, W * scale, generator=g).to(dtype).float()
    gy2 = torch.randn(N, 1, H * scale, W * scale, generator=g).to(dtype).float()
    g0 = torch.randn(N, 1, H, W, generator=g).to(dtype).float()
    xr = x.clone().requires_grad_(True)
    yr = F.interpolate(xr, scale_factor=scale, mode="bilinear", align_corners=(mode == 1))
    yr.backward(gy + gy2)
    outs = []
    for off in (False, True):
        if off:
            os.environ["DGVCC_UP_C1_OFF"] = "1"
        try:
            xd = K.Act(to_nhwc(x).to(dev, dtype))
            y = K.Act(K.nhwc(N, H * scale, W * scale, 1, dtype, dev))
            K.upsample_fwd(xd, scale, mode, y)
            gx = K.Act(to_nhwc(g0).to(dev, dtype))
            K.upsample_bwd(K.Act(to_nhwc(gy).to(dev, dtype)), scale, mode, gx,
                           gy2=K.Act(to_nhwc(gy2).to(dev, dtype)), accumulate=True)
            torch.cuda.synchronize()
        finally:
            os.environ.pop("DGVCC_UP_C1_OFF", None)
        outs.append((to_nchw(y.buf.float()).cpu(), to_nchw(gx.buf.float()).cpu()))
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert relerr(outs[0][0], yr.detach()) < tol
    assert relerr(outs[0][1], xr.grad + g0) < tol
    close = 2e-6 if dtype == torch.float32 else 1e-2
    assert relerr(outs[0][0], outs[1][0]) < close
    assert relerr(outs[0][1], outs[1][1]) < close


@pytest.mark.parametrize("act", [0, 1, 2])
def test_head(dev, act):
    K = _k()
    N, H, W, C = 2, 7, 9, 256
    g = torch.Generator().manual_seed(6)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(1, C, 1, 1, generator=g) * 0.1
    b = torch.randn(1, generator=g) if act == 2 else None
    gy = torch.randn(N, 1, H, W, generator=g)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True) if b is not None else None
    yr = F.conv2d(xr, wr, br)
    yr = [yr, F.relu(yr), torch.sigmoid(yr)][act]
    yr.backward(gy)
    xd = K.Act(to_nhwc(x).to(dev))
    y = K.head_fwd(xd, w.view(-1).to(dev), b.to(dev) if b is not None else None, act)
    gx = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
    gw = torch.empty(C, device=dev)
    gb = torch.empty(1, device=dev)
    K.head_bwd(xd, w.view(-1).to(dev), act, y, gy.view(N, H, W).to(dev), gx, gw, gb)
    torch.cuda.synchronize()
    assert relerr(y.view(N, 1, H, W), yr.detach()) < 1e-5
    assert relerr(to_nchw(gx.buf), xr.grad) < 1e-5
    assert relerr(gw, wr.grad.view(-1)) < 1e-5
    if b is not None:
        assert relerr(gb, br.grad) < 1e-5


def test_mse_and_adamw(dev):
    K = _k()
    g = torch.Generator().manual_seed(7)
    pred = torch.randn(3, 1, 17, 19, generator=g)
    gt = torch.rand(3, 1, 17, 19, generator=g) * 1e-3
    pr = pred.clone().requires_grad_(True)
    lr_ = F.mse_loss(pr, gt * 1000)
    lr_.backward()
    loss, dpred = K.mse_loss(pred.to(dev), gt.to(dev), 1000.0)
    torch.cuda.synchronize()
    assert abs(loss.item() - lr_.item()) / lr_.item() < 1e-6
    assert relerr(dpred, pr.grad) < 1e-6

    n = 1000
    p = torch.randn(n, generator=g)
    p_ref = torch.nn.Parameter(p.clone())
    opt = torch.optim.AdamW([p_ref], lr=1e-3, weight_decay=1e-4)
    pd, md, vd = p.to(dev), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    for step in range(1, 4):
        grad = torch.randn(n, generator=g)
        p_ref.grad = grad.clone()
        opt.step()
        K.adamw_step(pd, grad.to(dev), md, vd, 1e-3, 0.9, 0.999, 1e-8, 1e-4, step)
    torch.cuda.synchronize()
    assert relerr(pd, p_ref.detach()) < 1e-6


def test_fused_adamw_matches_torch_with_missing_grads(dev):
    """dgvcc_amd.optim.AdamW == torch.optim.AdamW, including params whose .grad is
    None (skipped: no decay, no moment update — the ISW counter's unused layer4)."""
    from dgvcc_amd.optim import AdamW
    g = torch.Generator().manual_seed(3)
    shapes = [(7, 5), (3,), (4, 4, 3), (6,), (2, 9)]
    base = [torch.randn(s, generator=g) for s in shapes]
    ours = [torch.nn.Parameter(b.clone().to(dev)) for b in base]
    ref = [torch.nn.Parameter(b.clone().to(dev)) for b in base]
    o1 = AdamW(ours, lr=1e-2, weight_decay=1e-2, allreduce=False)
    o2 = torch.optim.AdamW(ref, lr=1e-2, weight_decay=1e-2)
    for step in range(3):
        grads = [torch.randn(s, generator=g) for s in shapes]
        for i, (a, b) in enumerate(zip(ours, ref)):
            dead = i in (2, 3) or (i == 0 and step == 0)
            a.grad = None if dead else grads[i].to(dev)
            b.grad = None if dead else grads[i].to(dev)
        o1.step()
        o2.step()
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(ours, ref)):
        if i == 0:
            continue  # live for fewer steps: torch keeps a per-param step count, ours per group
        assert torch.allclose(a.detach(), b.detach(), rtol=1e-5, atol=1e-6), i
    assert torch.equal(ours[2].detach().cpu(), base[2]) and torch.equal(ours[3].detach().cpu(), base[3])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(64, 64, 3, 3), (256, 64, 1, 1), (128, 96, 3, 3), (2048, 512, 1, 1), (1, 70, 3, 3),
                                   (100, 3, 5, 5)])
def test_pack_weight_flip(dev, dtype, shape):
    """dg_pack_weight_flip: both outputs bit-identical to dg_pack_weight + dg_flip_weight."""
    K = _k()
    w = torch.randn(shape, generator=torch.Generator().manual_seed(12)).to(dev)
    wp, wf = K.pack_weight_flip(w, dtype)
    ref = K.pack_weight(w, dtype)
    reff = K.flip_weight(ref, shape[0], shape[1], shape[2])
    torch.cuda.synchronize()
    assert torch.equal(wp, ref) and torch.equal(wf, reff)


def test_gather_flat_chunks(dev):
    """dg_gather_flat (one block per 4096-element chunk, tensor found by binary search): tensors of 0, 1, odd,
    chunk-straddling and multi-chunk sizes, gathered as two runs into one flat buffer (the optimizer's dead-
    parameter gaps stay untouched); bit-exact copies."""
    K = _k()
    g = torch.Generator().manual_seed(11)
    sizes = [5, 0, 4096, 1, 4095, 9000, 3, 0, 70001, 17, 4097, 2]
    ts = [torch.randn(s, generator=g).to(dev) for s in sizes]
    offs, o = [], 0
    for s in sizes:
        offs.append(o)
        o += s
    flat = torch.full((o + 100,), -7.0, device=dev)
    expect = flat.clone()
    for run in (range(0, 5), range(6, len(sizes))):  # tensor 5 is a dead parameter: its region stays as it was
        table = torch.tensor([ts[i].data_ptr() for i in run], dtype=torch.int64, device=dev)
        last = run[-1]
        dev_offs = torch.tensor([offs[i] for i in run] + [offs[last] + sizes[last]], dtype=torch.int64, device=dev)
        K.call("dg_gather_flat", K.ptr(table), K.ptr(dev_offs), len(run), flat.numel(), K.ptr(flat), K.stream())
        for i in run:
            expect[offs[i]:offs[i] + sizes[i]] = ts[i]
    torch.cuda.synchronize()
    assert torch.equal(flat, expect)


@pytest.mark.parametrize("case", [(1, 256, 288, 64, 256, 3), (1, 256, 288, 128, 128, 3), (1, 256, 288, 64, 64, 3),
                                  (1, 256, 288, 256, 512, 1), (2, 20, 24, 64, 128, 3), (1, 64, 64, 512, 512, 3)])
def test_conv_f32_split_math(dev, case):
    """DG_F32 on the bf16 matrix cores (dg_set_f32_math(1): exact 3-way bf16 split, six products) and on
    the f16 ones (2: two scaled f16 parts, three products) against float64 torch: forward, dgrad and
    wgrad within 5e-6 relative and no worse than 2x the v_mfma_f32_16x16x4_f32 path's own error on
    the same launch (f32-grade)."""
    K = _k()
    N, H, W, C, Cout, R = case
    pad = R // 2
    g = torch.Generator().manual_seed(3)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(Cout, C, R, R, generator=g) / (C * R * R) ** 0.5
    gy = torch.randn(N, Cout, H, W, generator=g)
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    yr = F.conv2d(xr, wr, padding=pad)
    yr.backward(gy.double())
    xd = K.Act(to_nhwc(x).to(dev))
    gyd = K.Act(to_nhwc(gy).to(dev))
    wp = K.pack_weight(w.to(dev), torch.float32)
    errs = {}
    prev = K.lib_call_status("dg_get_f32_math")
    try:
        for mode in (0, 1, 2):
            K.call("dg_set_f32_math", mode)
            y = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
            K.conv_fwd(xd, wp, Cout, R, pad, y)
            dx = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
            K.conv_dgrad(gyd, wp, C, R, pad, dx)
            dw = torch.empty(Cout, C, R, R, device=dev)
            K.conv_wgrad(xd, gyd, R, pad, dw)
            torch.cuda.synchronize()
            errs[mode] = (relerr(to_nchw(y.buf), yr.detach()), relerr(to_nchw(dx.buf), xr.grad), relerr(dw, wr.grad))
    finally:
        K.call("dg_set_f32_math", prev)
    for m in (1, 2):
        for e0, e1 in zip(errs[0], errs[m]):
            assert e1 < 5e-6 and e1 < 2 * e0 + 2e-7, errs


@pytest.mark.parametrize("case", [(2, 20, 24, 64, 128, 3), (1, 16, 256, 64, 64, 3), (1, 24, 64, 128, 128, 3),
                                  (1, 16, 64, 256, 256, 3), (1, 8, 64, 512, 512, 3), (1, 12, 8, 256, 128, 1),
                                  (2, 4, 512, 128, 64, 3), (1, 6, 1024, 64, 64, 3), (1, 8, 16, 896, 256, 1)])
def test_conv_f32_split_exact_identity(dev, case):
    """The 3-way split is exact (x = h0 + h1 + h2 bit for bit, dg_common.h split3_pair): with an
    identity filter (centre tap) every split-math forward and dgrad path must return its input
    bit-identically, and the weight gradient against a one-hot output gradient must return the
    input pixel exactly (one nonzero product per output: no rounding anywhere).  Run on mode 1
    (the f16 x3 arithmetic of mode 2 keeps 22 bits: test_conv_f32_h16_identity_bound)."""
    K = _k()
    prev = K.lib_call_status("dg_get_f32_math")
    K.call("dg_set_f32_math", 1)
    try:
        _identity_case(K, dev, case, exact=True)
    finally:
        K.call("dg_set_f32_math", prev)


@pytest.mark.parametrize("case", [(2, 20, 24, 64, 128, 3), (1, 16, 64, 256, 256, 3), (1, 8, 64, 512, 512, 3),
                                  (2, 4, 512, 128, 64, 3), (1, 6, 1024, 64, 64, 3), (1, 8, 16, 896, 256, 1)])
def test_conv_f32_h16_identity_bound(dev, case):
    """The f16 x3 arithmetic (dg_set_f32_math(2)) on an identity filter: the filter row scales to
    2^14 exactly, so each output is the input's two f16 parts, x*s = hi + lo + r with
    |r| <= 2^-23 |x*s| (nearest lo), and elements whose lo part is subnormal lose at most 2^-25 in
    scaled units (2^-25 / s_x): |y - x| <= 2^-23 |x| + 2^-25 / s_x for forward and dgrad; the
    one-hot wgrad likewise (dY's part exact, X's within the same bound)."""
    K = _k()
    prev = K.lib_call_status("dg_get_f32_math")
    K.call("dg_set_f32_math", 2)
    try:
        _identity_case(K, dev, case, exact=False)
    finally:
        K.call("dg_set_f32_math", prev)


def _identity_case(K, dev, case, exact):
    N, H, W, C, Cout, R = case
    pad = R // 2
    g = torch.Generator().manual_seed(31)
    n = min(C, Cout)
    w = torch.zeros(Cout, C, R, R)
    w[torch.arange(n), torch.arange(n), pad, pad] = 1.0
    x = torch.randn(N, H, W, C, generator=g) * torch.exp(torch.randn(N, H, W, C, generator=g))  # full mantissas
    gy = torch.randn(N, H, W, Cout, generator=g)
    xd, gyd = K.Act(x.to(dev)), K.Act(gy.to(dev))
    wp = K.pack_weight(w.to(dev), torch.float32)
    y = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
    K.conv_fwd(xd, wp, Cout, R, pad, y)
    dx = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
    K.conv_dgrad(gyd, wp, C, R, pad, dx)
    oh = torch.zeros(N, H, W, Cout)
    p = (N * H * W) // 2 + 3
    oh.view(-1, Cout)[p] = 1.0
    dw = torch.empty(Cout, C, R, R, device=dev)
    K.conv_wgrad(xd, K.Act(oh.to(dev)), R, pad, dw)
    torch.cuda.synchronize()
    xp = x.view(-1, C)[p]
    if exact:
        assert torch.equal(y.buf.cpu()[..., :n], x[..., :n]), "forward"
        assert torch.equal(dx.buf.cpu()[..., :n], gy[..., :n]), "dgrad"
        assert torch.equal(dw[:, :, pad, pad].cpu(), xp.view(1, C).expand(Cout, C)), "wgrad"
        return

    def bound(ref):  # 2^-23 |x| + 2^-25 / s_x with s_x = 2^(14 - e), max |x| = m 2^e
        e = torch.frexp(ref.abs().max())[1].item()
        return ref.abs() * 2.0 ** -23 + 2.0 ** (-25 - (14 - e))

    for got, ref, what in ((y.buf.cpu()[..., :n], x[..., :n], "forward"), (dx.buf.cpu()[..., :n], gy[..., :n], "dgrad"),
                           (dw[:, :, pad, pad].cpu(), xp.view(1, C).expand(Cout, C), "wgrad")):
        b = bound(x if what != "dgrad" else gy) if what != "wgrad" else bound(x)
        if what == "wgrad":
            b = xp.abs() * 2.0 ** -23 + 2.0 ** (-25 - (14 - torch.frexp(x.abs().max())[1].item()))
            b = b.view(1, C).expand(Cout, C)
        else:
            b = b[..., :n]
        assert bool(((got.double() - ref.double()).abs() <= b.double()).all()), what


@pytest.mark.parametrize("case,which", [((1, 32, 64, 512, 512, 3), "fd"),      # K = 4608 fwd + dgrad
                                        ((1, 48, 64, 512, 256, 3), "fd"),
                                        ((1, 768, 1024, 64, 64, 3), "w"),      # 786k-pixel wgrad reduction
                                        ((4, 192, 256, 128, 128, 3), "w")])
def test_conv_f32_split_same_sign(dev, case, which):
    """The truncating 3-way split drops x1*y2 + x2*y1 (+ x2*y2), up to ~2^-20 |x*y| and all with
    the sign of x*y (dg_common.h): a bias, which randn operands hide because mixed signs cancel.
    Same-sign operands (post-ReLU activations, positive filters and output gradients) make it add
    up coherently over the K = 4608 forward/dgrad and the 786k-pixel wgrad reduction.  Bound:
    within 2x the exact v_mfma_f32_16x16x4_f32 path's own error on the same launch."""
    K = _k()
    N, H, W, C, Cout, R = case
    pad = R // 2
    g = torch.Generator().manual_seed(21)
    x = torch.randn(N, C, H, W, generator=g).abs()
    w = torch.rand(Cout, C, R, R, generator=g) / (C * R * R)
    gy = torch.rand(N, Cout, H, W, generator=g)
    xd = K.Act(to_nhwc(x).to(dev))
    gyd = K.Act(to_nhwc(gy).to(dev))
    wp = K.pack_weight(w.to(dev), torch.float32)
    if which == "fd":
        ref_y = F.conv2d(x.double(), w.double(), padding=pad)
        ref_dx = torch.nn.grad.conv2d_input(x.shape, w.double(), gy.double(), padding=pad)
    else:
        ref_dw = torch.nn.grad.conv2d_weight(x.double(), w.shape, gy.double(), padding=pad)
    errs = {}
    prev = K.lib_call_status("dg_get_f32_math")
    try:
        for mode in (0, 1, 2):
            K.call("dg_set_f32_math", mode)
            if which == "fd":
                y = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
                K.conv_fwd(xd, wp, Cout, R, pad, y)
                dx = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
                K.conv_dgrad(gyd, wp, C, R, pad, dx)
                torch.cuda.synchronize()
                errs[mode] = (relerr(to_nchw(y.buf), ref_y), relerr(to_nchw(dx.buf), ref_dx))
            else:
                dw = torch.empty(Cout, C, R, R, device=dev)
                K.conv_wgrad(xd, gyd, R, pad, dw)
                torch.cuda.synchronize()
                errs[mode] = (relerr(dw, ref_dw),)
    finally:
        K.call("dg_set_f32_math", prev)
    for m in (1, 2):
        for e0, e1 in zip(errs[0], errs[m]):
            assert e1 < 2 * e0 + 1e-7, errs
    print("same-sign split errors (exact, split):", errs)


@pytest.mark.parametrize("N,H,W,C,Cout,epi", [(5, 128, 256, 64, 256, "stats"), (3, 96, 320, 128, 128, "stats"),
                                              (3, 128, 256, 256, 512, "eval"), (8, 100, 130, 128, 256, "bias"),
                                              (3, 70, 90, 64, 64, "stats"), (2, 64, 256, 128, 64, "eval"),
                                              (2, 33, 40, 64, 64, "bias"), (2, 8, 256, 64, 64, "stats"),
                                              (1, 6, 512, 128, 64, "bias"), (2, 5, 256, 64, 64, "eval"),
                                              (2, 4, 512, 64, 64, "stats"), (1, 3, 1024, 64, 64, "eval"),
                                              (16, 48, 64, 256, 256, "stats"), (2, 96, 128, 128, 256, "bias"),
                                              (16, 48, 64, 512, 256, "eval")])
@pytest.mark.parametrize("tall", ["0", "2"])
def test_conv_f32_psplit_epilogues(dev, N, H, W, C, Cout, epi, tall, monkeypatch):
    """Pre-split-filter f32 forward (conv_fwd_psplit_kernel, 192-pixel tiles, BN = 256 / 128; Cout = 64 on
    conv_fwd_rsplit_kernel, 256-pixel tiles) with
    bias + epilogue BN statistics (rows per 192-pixel tile: dg_conv_stats_rows_ex), the eval-BN
    epilogue and a ragged last tile, against float64: y within 5e-6, the merged (n, mean, M2)
    rows equal to the statistics of the stored y.  tall = "2": the 256-channel training launches on
    256-pixel tiles (DGVCC_PSPLIT_TALL, epilogue scratch and bias in the consumed stage).  The last three
    shapes have 128..256 pre-split tiles (fewer than the CUs: DGVCC_PSPLIT_MIN_TILES, the ISW trunk's
    layer3 at 48 x 64), served before round 4 by the exact-f32 register-staged kernel."""
    if tall == "2" and (Cout % 256 or epi == "eval"):
        pytest.skip("256-pixel tiles serve 256-channel training launches only")
    monkeypatch.setenv("DGVCC_PSPLIT_TALL", tall)
    K = _k()
    g = torch.Generator().manual_seed(14)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** 0.5
    b = torch.randn(Cout, generator=g)
    wp = K.pack_weight(w.to(dev), torch.float32)
    z = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double(), padding=1).permute(0, 2, 3, 1)
    if epi == "eval":
        st = torch.stack([torch.zeros(Cout), torch.ones(Cout), torch.rand(Cout, generator=g) + 0.5,
                          torch.randn(Cout, generator=g) * 0.1])
        K.conv_fwd_bn_eval(K.Act(x.to(dev)), wp, Cout, 3, 1, z, b.to(dev), st.to(dev), 1)
        ref = (ref * st[2].double() + st[3].double()).clamp_min(0)
    elif epi == "stats":
        rows = K.query("dg_conv_stats_rows_ex", 0, N, H, W, C, C, Cout, 3, 3)
        # tiles: 192 px at 256 channels, 384 px at 128 (conv_fwd_psplit_kernel), 256 px at 64 (rsplit),
        # 512 px at 64 where W % 512 == 0 (conv_fwd_rsplit3w_kernel)
        tile = (256 if tall == "2" else 192) if Cout % 256 == 0 else (384 if Cout % 128 == 0 else
                                                                      (512 if W % 512 == 0 else 256))
        assert rows == -(-(N * H * W) // tile)
        part, r2 = K.conv_fwd_stats(K.Act(x.to(dev)), wp, Cout, 3, 1, z, bias=b.to(dev))
        assert r2 == rows
    else:
        K.conv_fwd(K.Act(x.to(dev)), wp, Cout, 3, 1, z, bias=b.to(dev))
    torch.cuda.synchronize()
    y = z.buf.cpu()
    assert relerr(y, ref) < 5e-6
    if epi == "stats":
        p = part.double().cpu()
        n, mean, m2 = p[:, 0], p[:, 1], p[:, 2]
        tot = n.sum(0)
        gm = (n * mean).sum(0) / tot
        var = (m2 + n * (mean - gm) ** 2).sum(0) / tot
        yd = y.double().reshape(-1, Cout)
        assert torch.equal(tot, torch.full_like(tot, N * H * W))
        assert relerr(gm, yd.mean(0)) < 1e-5 and relerr(var, yd.var(0, unbiased=False)) < 1e-5


@pytest.mark.parametrize("N,H,W,C,Cout", [(16, 48, 64, 64, 256), (4, 96, 128, 64, 256), (4, 100, 130, 64, 128),
                                         (16, 48, 64, 32, 256)])
def test_conv_f32_psplit_short_k(dev, N, H, W, C, Cout, monkeypatch):
    """1x1 f32 convs from 64 (or 32) channels -- one or two 32-channel K-steps per tile, the
    trunks' bottleneck expansions -- on the pre-split kernel (DGVCC_PSPLIT_SHORTK, default on) with
    bias and epilogue statistics against float64, and against the exact-f32 kernel the switch
    restores: y within 5e-6, the (n, mean, M2) rows equal to the statistics of the stored y.
    C = 32 (a single K-step) stays on the exact kernel (the pre-split pipeline needs >= 2)."""
    K = _k()
    g = torch.Generator().manual_seed(21)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(Cout, C, 1, 1, generator=g) / C ** 0.5
    b = torch.randn(Cout, generator=g)
    wp = K.pack_weight(w.to(dev), torch.float32)
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double()).permute(0, 2, 3, 1)
    ys = []
    for sk in ("1", "0"):
        monkeypatch.setenv("DGVCC_PSPLIT_SHORTK", sk)
        z = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
        res = K.conv_fwd_stats(K.Act(x.to(dev)), wp, Cout, 1, 0, z, bias=b.to(dev))
        if res is None:  # served by a kernel without epilogue statistics: nothing was launched
            K.conv_fwd(K.Act(x.to(dev)), wp, Cout, 1, 0, z, bias=b.to(dev))
        torch.cuda.synchronize()
        y = z.buf.cpu()
        assert relerr(y, ref) < 5e-6
        ys.append(y)
        if sk == "1" and C == 64:
            rows = K.query("dg_conv_stats_rows_ex", 0, N, H, W, C, C, Cout, 1, 1)
            assert res is not None and res[1] == rows == -(-(N * H * W) // (192 if Cout == 256 else 384))
        if res is not None:
            p = res[0].double().cpu()
            n, mean, m2 = p[:, 0], p[:, 1], p[:, 2]
            tot = n.sum(0)
            gm = (n * mean).sum(0) / tot
            var = (m2 + n * (mean - gm) ** 2).sum(0) / tot
            yd = y.double().reshape(-1, Cout)
            assert torch.equal(tot, torch.full_like(tot, N * H * W))
            assert relerr(gm, yd.mean(0)) < 1e-5 and relerr(var, yd.var(0, unbiased=False)) < 1e-5
    assert relerr(ys[0], ys[1]) < 5e-6


@pytest.mark.parametrize("N,H,W,C,Cout,mode", [(2, 9, 64, 64, 64, "1"), (3, 17, 96, 64, 128, "1"),
                                               (2, 40, 32, 128, 64, "1"), (1, 48, 160, 256, 128, "2"),
                                               (4, 5, 128, 64, 64, "1"), (2, 11, 96, 128, 256, "3"),
                                               (1, 24, 64, 256, 128, "3")])
def test_conv_f32_wgrad_split3(dev, N, H, W, C, Cout, mode):
    """3-tap shared f32 split-math wgrad (conv_wgrad_split3_kernel: a kernel row's three taps on one
    staged dY tile and X strip, K-steps of 32 pixels of one image row) against float64 torch and
    against the per-tap split kernel (DGVCC_WGRAD_SPLIT3=0) on the same launch shapes: image and
    split boundaries inside the K range (small H, several images), both 64-channel sides."""
    import os
    K = _k()
    g = torch.Generator().manual_seed(21)
    x = torch.randn(N, C, H, W, generator=g)
    gy = torch.randn(N, Cout, H, W, generator=g)
    xr = x.double()
    wr = torch.zeros(Cout, C, 3, 3, dtype=torch.float64, requires_grad=True)
    F.conv2d(xr, wr, padding=1).backward(gy.double())
    xd = K.Act(to_nhwc(x).to(dev))
    gyd = K.Act(to_nhwc(gy).to(dev))
    out = {}
    old = os.environ.get("DGVCC_WGRAD_SPLIT3")
    try:
        for m in (mode, "0"):
            os.environ["DGVCC_WGRAD_SPLIT3"] = m
            dw = torch.empty(Cout, C, 3, 3, device=dev)
            K.conv_wgrad(xd, gyd, 3, 1, dw)
            torch.cuda.synchronize()
            out[m] = dw.cpu()
    finally:
        if old is None:
            os.environ.pop("DGVCC_WGRAD_SPLIT3", None)
        else:
            os.environ["DGVCC_WGRAD_SPLIT3"] = old
    e3, e1 = relerr(out[mode], wr.grad), relerr(out["0"], wr.grad)
    assert e3 < 5e-6 and e3 < 2 * e1 + 2e-7, (e3, e1)


@pytest.mark.parametrize("N,H,W,C,Cout", [(2, 7, 256, 64, 64), (1, 5, 512, 64, 128), (1, 4, 256, 256, 64),
                                          (2, 3, 1024, 64, 64), (1, 6, 512, 128, 64)])
def test_conv_f32_rsplit3(dev, N, H, W, C, Cout):
    """Cout = 64 split-math forward with the 3 taps of a kernel row on one staged strip
    (conv_fwd_rsplit3_kernel, W % 256 == 0; conv_fwd_rsplit3w_kernel, W % 512 == 0) and the dgrad
    that lands on it (64-channel dx): against
    float64 torch and against the per-tap kernel (DGVCC_RSPLIT3=0), within the f32-grade bound."""
    import os
    K = _k()
    g = torch.Generator().manual_seed(31)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** 0.5
    gy = torch.randn(N, Cout, H, W, generator=g)
    xr = x.double().requires_grad_(True)
    yr = F.conv2d(xr, w.double(), padding=1)
    yr.backward(gy.double())
    xd, gyd = K.Act(to_nhwc(x).to(dev)), K.Act(to_nhwc(gy).to(dev))
    wp = K.pack_weight(w.to(dev), torch.float32)
    errs = {}
    old = os.environ.get("DGVCC_RSPLIT3")
    try:
        for m in ("2", "1", "0"):
            os.environ["DGVCC_RSPLIT3"] = m
            e = []
            if Cout == 64:
                y = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
                K.conv_fwd(xd, wp, Cout, 3, 1, y)
                torch.cuda.synchronize()
                e.append(relerr(to_nchw(y.buf), yr.detach()))
            if C == 64:
                dx = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
                K.conv_dgrad(gyd, wp, C, 3, 1, dx)
                torch.cuda.synchronize()
                e.append(relerr(to_nchw(dx.buf), xr.grad))
            errs[m] = e
    finally:
        if old is None:
            os.environ.pop("DGVCC_RSPLIT3", None)
        else:
            os.environ["DGVCC_RSPLIT3"] = old
    for m in ("2", "1"):  # 512-pixel all-pixel-wave form (W % 512 == 0), 256-pixel form
        for e3, e1 in zip(errs[m], errs["0"]):
            assert e3 < 5e-6 and e3 < 2 * e1 + 2e-7, errs
    # each form within 2x the exact v_mfma_f32_16x16x4_f32 path's error on the same launch: the 512-pixel
    # form on f16 x3, the 256-pixel and per-tap ones on bf16 x6 (default) and on f16 x3 (DGVCC_RSPLIT_H16=1)
    old_h = os.environ.get("DGVCC_RSPLIT_H16")
    try:
        os.environ["DGVCC_RSPLIT_H16"] = "1"
        for m in ("1", "0"):
            os.environ["DGVCC_RSPLIT3"] = m
            e = []
            if Cout == 64:
                y = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
                K.conv_fwd(xd, wp, Cout, 3, 1, y)
                torch.cuda.synchronize()
                e.append(relerr(to_nchw(y.buf), yr.detach()))
            if C == 64:
                dx = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
                K.conv_dgrad(gyd, wp, C, 3, 1, dx)
                torch.cuda.synchronize()
                e.append(relerr(to_nchw(dx.buf), xr.grad))
            errs["h16_" + m] = e
    finally:
        for k, v in (("DGVCC_RSPLIT_H16", old_h), ("DGVCC_RSPLIT3", old)):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    prev = K.lib_call_status("dg_get_f32_math")
    K.call("dg_set_f32_math", 0)
    try:
        ex = []
        if Cout == 64:
            y = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
            K.conv_fwd(xd, wp, Cout, 3, 1, y)
            torch.cuda.synchronize()
            ex.append(relerr(to_nchw(y.buf), yr.detach()))
        if C == 64:
            dx = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
            K.conv_dgrad(gyd, wp, C, 3, 1, dx)
            torch.cuda.synchronize()
            ex.append(relerr(to_nchw(dx.buf), xr.grad))
    finally:
        K.call("dg_set_f32_math", prev)
    for m in ("2", "1", "0", "h16_1", "h16_0"):
        for e3, e0 in zip(errs[m], ex):
            assert e3 < 2 * e0 + 2e-7, (m, errs, ex)


@pytest.mark.parametrize("sch", ["1", "3", "5", "6", "9", "xs"])
@pytest.mark.parametrize("N,H,W,C,Cout,R", [(2, 96, 392, 256, 256, 3), (1, 20, 72, 128, 512, 3), (3, 9, 40, 64, 256, 1),
                                            (1, 33, 47, 512, 256, 3)])
def test_conv_f32_psplit_schedules(dev, sch, N, H, W, C, Cout, R, monkeypatch):
    """The f16 x3 pre-split forward's schedules (DGVCC_PSPLIT_SCH: 1 DMA pieces spread over the MFMA
    blocks, 3 SIMD partners out of phase, 5 register staging instead of LDS-DMA, 6 the two channel
    halves one phase apart, 9 the split once per block in LDS; "xs": the pixel operand pre-split by
    split_x_h_kernel, SCH 8) bit-identical
    to the in-kernel split (0): several tiles per block (the cross-tile prefetch), ragged pixel tails,
    bias, epilogue statistics and the dgrad on the same kernel."""
    K = _k()
    prev = K.call("dg_get_f32_math")
    K.call("dg_set_f32_math", 2)
    try:
        g = torch.Generator().manual_seed(41)
        x = K.Act(to_nhwc(torch.relu(torch.randn(N, C, H, W, generator=g))).to(dev))
        w = (torch.randn(Cout, C, R, R, generator=g) / (R * R * C) ** 0.5).to(dev)
        bias = (torch.randn(Cout, generator=g) * 0.1).to(dev)
        gy = K.Act(to_nhwc(torch.randn(N, Cout, H, W, generator=g) * 1e-3).to(dev))
        wp = K.pack_weight(w, torch.float32)
        outs = []
        for v in ("0", sch):
            if sch == "xs":  # the pre-split pixel operand (SCH 8, forced on every eligible shape) against the in-kernel split
                monkeypatch.setenv("DGVCC_PSPLIT_XS", "2" if v == "xs" else "0")
            else:
                monkeypatch.setenv("DGVCC_PSPLIT_XS", "0")
                monkeypatch.setenv("DGVCC_PSPLIT_SCH", v)
            y = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
            res = K.conv_fwd_stats(x, wp, Cout, R, R // 2, y, bias=bias)
            if res is None:  # a shape without epilogue statistics: nothing was launched
                K.conv_fwd(x, wp, Cout, R, R // 2, y, bias=bias)
            y2 = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
            K.conv_fwd(x, wp, Cout, R, R // 2, y2)
            dx = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
            K.conv_dgrad(gy, wp, C, R, R // 2, dx)
            torch.cuda.synchronize()
            outs.append([y.buf.clone(), y2.buf.clone(), dx.buf.clone()] + ([res[0].clone()] if res is not None else []))
        for u, v in zip(*outs):
            assert torch.equal(u, v)
    finally:
        K.call("dg_set_f32_math", prev)


@pytest.mark.parametrize("xs,ws", [(1e-30, 1.0), (1e-6, 1e-3), (1.0, 1.0), (1e6, 1e3), (1e30, 1e-20), (1e-12, 1e-25)])
@pytest.mark.parametrize("case", [(1, 64, 96, 256, 256, 3), (1, 32, 512, 64, 64, 3), (1, 48, 64, 128, 128, 3)])
def test_conv_f32_h16_scales(dev, xs, ws, case):
    """f16 x3 (dg_set_f32_math(2)) on operands of any magnitude: the power-of-two scales (per filter row,
    per pixel-operand tensor) bring them into f16 range and back exactly, so forward, dgrad and wgrad
    stay within 5e-6 (normwise relative) of float64 from 1e-30 to 1e30; one launch also holds a
    dynamic range of 1e-12 inside one tensor.  (1e-12, 1e-25): both operands tiny, so the two scales'
    exponents sum past f32's range (2^-151) while the outputs (~1e-37) are normal f32 values: the
    rescale is applied as one ldexp of the result, not as a factor that would flush."""
    K = _k()
    N, H, W, C, Cout, R = case
    pad = R // 2
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N, C, H, W, generator=g) * xs
    x[:, : C // 4] *= 1e-12  # a quarter of the channels twelve decades below the rest
    w = torch.randn(Cout, C, R, R, generator=g) / (C * R * R) ** 0.5 * ws
    gy = torch.randn(N, Cout, H, W, generator=g)
    y64 = F.conv2d(x.double(), w.double(), padding=pad)
    dx64 = torch.nn.grad.conv2d_input(x.shape, w.double(), gy.double() * xs, padding=pad)
    dw64 = torch.nn.grad.conv2d_weight(x.double(), w.shape, gy.double(), padding=pad)
    xd, gyd, gysd = K.Act(to_nhwc(x).to(dev)), K.Act(to_nhwc(gy).to(dev)), K.Act(to_nhwc(gy * xs).to(dev))
    wp = K.pack_weight(w.to(dev), torch.float32)
    prev = K.lib_call_status("dg_get_f32_math")
    K.call("dg_set_f32_math", 2)
    try:
        y = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
        K.conv_fwd(xd, wp, Cout, R, pad, y)
        dx = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
        K.conv_dgrad(gysd, wp, C, R, pad, dx)
        dw = torch.empty(Cout, C, R, R, device=dev)
        K.conv_wgrad(xd, gyd, R, pad, dw)
        torch.cuda.synchronize()
    finally:
        K.call("dg_set_f32_math", prev)
    nrel = lambda a, b: float((a.double().cpu() - b).norm() / b.norm())  # noqa: E731
    errs = (nrel(to_nchw(y.buf), y64), nrel(to_nchw(dx.buf), dx64), nrel(dw, dw64))
    assert max(errs) < 5e-6, errs
    assert all(torch.isfinite(t).all() for t in (y.buf, dx.buf, dw))


def test_amax(dev):
    """dg_amax: the operand maxima of a channel slice of an NHWC buffer (the f16 x3 scales): [0] the
    slice's max |x|, [1 + c] channel c's."""
    K = _k()
    g = torch.Generator().manual_seed(9)
    buf = torch.randn(2, 7, 9, 96, generator=g)
    buf[1, 3, 4, 70] = -123.5   # outside the slice below: must not count
    buf[0, 6, 8, 40] = -77.25   # inside
    a = K.Act(buf.to(dev), off=32, C=32)
    m = K.amax(a)
    torch.cuda.synchronize()
    assert m.shape == (K.amax_words(32),) and m[0].item() == 77.25  # 1 + C words, a multiple of 4
    assert torch.equal(m[1:33].cpu(), buf[..., 32:64].abs().amax(dim=(0, 1, 2)))
    full = K.amax(K.Act(buf.to(dev))).cpu()
    assert full[0].item() == 123.5 and torch.equal(full[1:97], buf.abs().amax(dim=(0, 1, 2)))
    for C in (4, 12, 896, 2048):  # chunk groups: one partial block, several rows, y-grid groups
        b = torch.randn(3, 5, 7, C, generator=g) * torch.logspace(-20, 20, C)
        m = K.amax(K.Act(b.to(dev))).cpu()
        assert m[0].item() == b.abs().max().item() and torch.equal(m[1:1 + C], b.abs().amax(dim=(0, 1, 2))), C


# channel magnitudes of the per-channel f16 x3 test: every fifth channel of the operand at full scale,
# the others 1e-3 .. 1e-12 below it
CHAN_DECADES = (1.0, 1e-3, 1e-6, 1e-9, 1e-12)


def _chan_scaled(n, C, H, W, g):
    s = torch.tensor([CHAN_DECADES[c % len(CHAN_DECADES)] for c in range(C)], dtype=torch.float64)
    return (torch.randn(n, C, H, W, generator=g, dtype=torch.float64) * s.view(1, C, 1, 1)).float()


def _chan_err(a, ref, dim):
    """Per-channel relative error along `dim`: max |a - ref| over the channel / max |ref| over it."""
    d = (a.double().cpu() - ref).abs()
    other = [i for i in range(ref.dim()) if i != dim]
    return d.amax(dim=other) / ref.abs().amax(dim=other).clamp_min(1e-300)


@pytest.mark.parametrize("case", [(1, 32, 64, 128, 128, 3), (1, 24, 128, 64, 64, 3), (2, 16, 32, 128, 256, 3),
                                  (1, 16, 64, 256, 128, 1), (1, 20, 36, 64, 128, 3)])
def test_conv_f32_h16_per_channel(dev, case, monkeypatch):
    """f16 x3 per element: channels of x and dY 1e-3 .. 1e-12 below their tensor's
    largest magnitude.  The weight gradient scales each channel of x and of dY by its own power of two,
    so every row (output channel) and column (input channel) of dW keeps f32-grade relative error; the
    forward and dgrad outputs per channel.  Bound: 2x the exact v_mfma_f32_16x16x4_f32 path's error on
    the same channel (+1e-7 against two tiny maxima), both against float64.  Shapes: the 3-tap 128 x 128
    and 64-channel 9-tap weight gradients, the per-tap kernel (1x1, and the 3x3 W % 32 != 0 rows).
    DGVCC_RSPLIT_H16=1: the Cout = 64 forward / dgrad forms that default to the bf16 x6 split run f16 x3
    here too, so every launch is the arithmetic under test."""
    monkeypatch.setenv("DGVCC_RSPLIT_H16", "1")
    K = _k()
    N, H, W, C, Cout, R = case
    pad = R // 2
    g = torch.Generator().manual_seed(77)
    x = _chan_scaled(N, C, H, W, g)
    gy = _chan_scaled(N, Cout, H, W, g)
    w = torch.randn(Cout, C, R, R, generator=g) / (C * R * R) ** 0.5
    y64 = F.conv2d(x.double(), w.double(), padding=pad)
    dx64 = torch.nn.grad.conv2d_input(x.shape, w.double(), gy.double(), padding=pad)
    dw64 = torch.nn.grad.conv2d_weight(x.double(), w.shape, gy.double(), padding=pad)
    xd, gyd = K.Act(to_nhwc(x).to(dev)), K.Act(to_nhwc(gy).to(dev))
    wp = K.pack_weight(w.to(dev), torch.float32)
    prev = K.lib_call_status("dg_get_f32_math")
    res = {}
    try:
        for m in (2, 0):
            K.call("dg_set_f32_math", m)
            y = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
            K.conv_fwd(xd, wp, Cout, R, pad, y)
            dx = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
            K.conv_dgrad(gyd, wp, C, R, pad, dx)
            dw = torch.empty(Cout, C, R, R, device=dev)
            K.conv_wgrad(xd, gyd, R, pad, dw)
            torch.cuda.synchronize()
            res[m] = {"fwd": _chan_err(to_nchw(y.buf), y64, 1), "dgrad": _chan_err(to_nchw(dx.buf), dx64, 1),
                      "wgrad_rows": _chan_err(dw, dw64, 0), "wgrad_cols": _chan_err(dw, dw64, 1)}
    finally:
        K.call("dg_set_f32_math", prev)
    for k in res[2]:
        h, e = res[2][k], res[0][k]
        bad = (h > 2 * e + 1e-7).nonzero().flatten().tolist()
        print(k, f"f16x3 worst {h.max().item():.3e} exact worst {e.max().item():.3e}")
        assert not bad, (k, [(c, h[c].item(), e[c].item()) for c in bad[:8]])
    # the small channels are not flushed: every dW column / row carries its own magnitude
    assert res[2]["wgrad_cols"].max().item() < 1e-5 and res[2]["wgrad_rows"].max().item() < 1e-5


def test_producer_channel_maxima(dev):
    """The f32 producers emit per-channel operand maxima ([1 + C]: bn_apply here, the BN backward
    below) equal to the written tensor's, and a weight gradient on them is bit-identical to one that
    takes the library's own read pass (same scales)."""
    K = _k()
    g = torch.Generator().manual_seed(12)
    N, H, W, C = 2, 16, 32, 128
    z = K.Act(to_nhwc(torch.randn(N, C, H, W, generator=g)).to(dev))
    scale = torch.tensor([CHAN_DECADES[c % 5] for c in range(C)], dtype=torch.float32, device=dev)
    shift = torch.randn(C, generator=g).to(dev) * scale
    stats = torch.stack([torch.zeros_like(scale), torch.ones_like(scale), scale, shift])
    y = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
    K.bn_apply(z, stats, K.ACT_RELU, y)
    dy = K.Act(to_nhwc(_chan_scaled(N, 128, H, W, g)).to(dev))
    torch.cuda.synchronize()
    ref = y.view().abs().amax(dim=(0, 1, 2))
    assert y.amax.shape == (K.amax_words(C),)
    assert torch.equal(y.amax[1:1 + C], ref) and y.amax[0].item() == ref.max().item()
    dw1 = torch.empty(128, C, 3, 3, device=dev)
    dw2 = torch.empty_like(dw1)
    K.conv_wgrad(y, dy, 3, 1, dw1)
    K.conv_wgrad(K.Act(y.buf), K.Act(dy.buf), 3, 1, dw2)  # no maxima: the library's pass
    torch.cuda.synchronize()
    assert torch.equal(dw1, dw2)
    # the BN backward's dz maxima
    gz = K.Act(to_nhwc(torch.randn(N, C, H, W, generator=g)).to(dev))
    dz = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
    dgam, dbet = (torch.empty(C, device=dev) for _ in range(2))
    K.bn_bwd(gz, z, torch.ones(C, device=dev), stats, K.ACT_RELU, dz, dgam, dbet)
    torch.cuda.synchronize()
    ref = dz.view().abs().amax(dim=(0, 1, 2))
    assert torch.equal(dz.amax[1:1 + C], ref) and dz.amax[0].item() == ref.max().item()


@pytest.mark.parametrize("N,H,W,C", [(2, 38, 54, 64), (3, 10, 14, 512)])
def test_wide_maxima_passes(dev, monkeypatch, N, H, W, C):
    """The f32 passes that fold per-channel operand maxima run 1024-thread blocks (a quarter of the
    256-thread grids' atomics, dg_common.h DG_EW_WIDE); DGVCC_EW_NT=256 keeps the 256-thread grids.
    Both forms write bit-identical outputs and maxima: BN apply / backward, pooled apply / backward,
    the residual join, InstanceNorm apply / backward (ragged pixel counts, 64 and 512 channels)."""
    K = _k()
    g = torch.Generator().manual_seed(21)

    def t(*shape):
        return to_nhwc(torch.randn(*shape, generator=g) * 2).to(dev)

    z, z2, gz = t(N, C, H, W), t(N, C, H, W), t(N, C, H, W)
    gp = t(N, C, H // 2, W // 2)
    gam = (torch.rand(C, generator=g) + 0.5).to(dev)
    bet = torch.randn(C, generator=g).to(dev)
    zd = K.Act(z)
    stats = K.bn_fwd_train(zd, gam, bet, torch.zeros(C, device=dev), torch.ones(C, device=dev), 0.1, 1e-5)
    st2 = torch.randn(4, C, generator=g).to(dev)

    def run():
        y = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
        K.bn_apply(zd, stats, 1, y)
        dz = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
        K.bn_bwd(K.Act(gz), zd, gam, stats, 1, dz, torch.empty(C, device=dev), torch.empty(C, device=dev))
        yq = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
        yp = K.Act(K.nhwc(N, H // 2, W // 2, C, torch.float32, dev))
        K.bn_apply_pool(zd, stats, 1, yq, yp)
        dzp = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
        K.bn_bwd_pool(K.Act(gp), K.Act(gz), zd, gam, stats, 1, dzp, torch.empty(C, device=dev),
                      torch.empty(C, device=dev))
        ya = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
        K.bn_add_apply(zd, st2, K.Act(z2), st2, 1, ya)
        ist = K.instnorm_stats(zd, 1e-5)
        yi = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
        K.instnorm_apply(zd, ist, gam, bet, 0, yi)
        dxi = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
        K.instnorm_bwd(K.Act(gz), zd, ist, gam, dxi)
        outs = []
        for a in (y, dz, yq, dzp, ya, yi, dxi):
            outs += [a.buf.clone(), a.amax.clone()]
        torch.cuda.synchronize()
        return outs

    wide = run()
    monkeypatch.setenv("DGVCC_EW_NT", "256")
    narrow = run()
    for k, (a, b) in enumerate(zip(wide, narrow)):
        assert torch.equal(a, b), k
    # the maxima are the written tensors' own
    for k in range(0, len(wide), 2):
        ref = wide[k].reshape(-1, C).abs().amax(dim=0)
        assert torch.equal(wide[k + 1][1:1 + C], ref) and wide[k + 1][0].item() == ref.max().item(), k


def _pair_image_ref(y: torch.Tensor, bound: float) -> torch.Tensor:
    """The f16 x3 pair image [M][C/32][hi 32 | lo 32] (f16) of y [M][C] * 2^e, e = h16_exp(bound)."""
    import math
    e = max(-100, min(100, 14 - math.frexp(bound)[1])) if bound > 0 else 0
    v = y.float() * (2.0 ** e)
    hi = v.half()
    lo = (v - hi.float()).half()
    M, C = y.shape
    return torch.cat([hi.view(M, C // 32, 32), lo.view(M, C // 32, 32)], dim=2)


@pytest.mark.parametrize("N,H,W,C,Cout,pool", [(2, 128, 128, 128, 256, False), (2, 96, 256, 64, 128, False),
                                               (2, 64, 128, 256, 512, False), (2, 128, 256, 128, 256, True)])
def test_bn_pair_image_and_conv(dev, N, H, W, C, Cout, pool):
    """fp32 training BN apply writing the next conv's f16 x3 pair image (dg_bn_apply_pair /
    dg_bn_apply_pool_pair): y, yp and the maxima bit-identical to dg_bn_apply(_pool); the bound equals
    |gamma| sqrt(M) + |beta| in the scale / shift / mean / invstd form and bounds max |y|; the image is
    the f16 split of y * 2^e (e from the bound) in the pre-split layout.  The conv forward reading it
    (dg_conv_fwd_pair: the 256-pixel kernel, a single channel tile, 128 channels, and the several-tile
    form that otherwise runs split_x_h) has per-output-channel error within 2x the exact
    v_mfma_f32_16x16x4_f32 path's against float64, with its BN statistics rows."""
    K = _k()
    g = torch.Generator().manual_seed(31)
    z = K.Act(to_nhwc(torch.randn(N, C, H, W, generator=g) * 3 + 1).to(dev))
    gam = (torch.rand(C, generator=g) + 0.5).to(dev)
    bet = (torch.randn(C, generator=g) * 0.3).to(dev)
    stats = K.bn_fwd_train(z, gam, bet, torch.zeros(C, device=dev), torch.ones(C, device=dev), 0.1, 1e-5)
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    outs = {}
    for pr in (True, False):
        y = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
        if pool:
            yp = K.Act(K.nhwc(N, Ho, Wo, C, torch.float32, dev))
            K.bn_apply_pool(z, stats, K.ACT_RELU, y, yp, pair=pr)
            outs[pr] = (y, yp)
        else:
            K.bn_apply(z, stats, K.ACT_RELU, y, pair=pr)
            outs[pr] = (y, y)
    torch.cuda.synchronize()
    (y1, x1), (y0, x0) = outs[True], outs[False]
    assert torch.equal(y1.buf, y0.buf) and torch.equal(x1.buf, x0.buf) and torch.equal(x1.amax, x0.amax)
    assert x1.pair is not None and x0.pair is None
    img, bound = x1.pair
    b = bound.item()
    st = stats.double()
    ref_b = (st[2].abs() * (z.M ** 0.5) / st[1] + (st[3] + st[0] * st[2]).abs()).max().item()
    assert abs(b - ref_b) <= 1e-5 * ref_b and b >= x1.buf.abs().max().item()
    Mx = x1.M
    ref_img = _pair_image_ref(x1.buf.reshape(Mx, C), b)
    assert torch.equal(img.view(torch.float16).view(Mx, C // 32, 64), ref_img)
    # the conv forward on the pair image vs the same conv on x (exact f32 MFMA), against float64
    w = torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** 0.5
    wp = K.pack_weight(w.to(dev), torch.float32)
    y64 = F.conv2d(to_nchw(x1.buf).double().cpu(), w.double(), padding=1)
    prev = K.lib_call_status("dg_get_f32_math")
    errs = {}
    try:
        for m in (2, 0):
            K.call("dg_set_f32_math", m)
            src = K.Act(x1.buf)
            src.amax, src.pair = x1.amax, (x1.pair if m == 2 else None)
            o = K.Act(K.nhwc(N, Ho, Wo, Cout, torch.float32, dev))
            res = K.conv_fwd_stats(src, wp, Cout, 3, 1, o)
            if res is None:
                K.conv_fwd(src, wp, Cout, 3, 1, o)
            torch.cuda.synchronize()
            errs[m] = _chan_err(to_nchw(o.buf), y64, 1)
            if res is not None:  # the statistics rows merge to the output's own mean
                part = res[0].double()
                mean = (part[:, 0] * part[:, 1]).sum(0) / part[:, 0].sum(0)
                assert torch.allclose(mean.cpu(), o.buf.double().reshape(-1, Cout).mean(0).cpu(), rtol=1e-6, atol=1e-7)
    finally:
        K.call("dg_set_f32_math", prev)
    h, e = errs[2], errs[0]
    print(f"pair worst {h.max().item():.3e} exact worst {e.max().item():.3e}")
    assert (h <= 2 * e + 1e-7).all(), (h.max().item(), e.max().item())


@pytest.mark.parametrize("N,H,W,C,Cin,pool", [(2, 128, 128, 256, 256, False), (2, 64, 128, 512, 256, False),
                                              (2, 128, 256, 128, 256, True)])
def test_bn_bwd_pair_image_and_dgrad(dev, N, H, W, C, Cin, pool):
    """fp32 BN backward writing the dgrad's f16 x3 pair image of dz (dg_bn_bwd_pair /
    dg_bn_bwd_pool_pair): dz, dgamma, dbeta and the maxima bit-identical to dg_bn_bwd(_pool); the bound
    bounds max |dz| and is max_c |k1| max |g'| + |k2| sqrt(M) + |k3| (k from dgamma / dbeta); the image
    is the split of dz at the bound's scale; the dgrad reading it has per-channel error within 2x the
    exact f32 MFMA path's against float64."""
    K = _k()
    g = torch.Generator().manual_seed(37)
    z = K.Act(to_nhwc(torch.randn(N, C, H, W, generator=g) * 2 - 0.5).to(dev))
    gam = (torch.rand(C, generator=g) + 0.5).to(dev)
    bet = (torch.randn(C, generator=g) * 0.3).to(dev)
    stats = K.bn_fwd_train(z, gam, bet, torch.zeros(C, device=dev), torch.ones(C, device=dev), 0.1, 1e-5)
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    gy = K.Act(to_nhwc(torch.randn(N, C, Ho, Wo, generator=g) * 1e-3).to(dev))
    outs = {}
    for pr in (True, False):
        dz = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
        dgam, dbet = torch.empty(C, device=dev), torch.empty(C, device=dev)
        if pool:
            K.bn_bwd_pool(gy, None, z, gam, stats, K.ACT_RELU, dz, dgam, dbet, pair=pr)
        else:
            K.bn_bwd(gy, z, gam, stats, K.ACT_RELU, dz, dgam, dbet, pair=pr)
        outs[pr] = (dz, dgam, dbet)
    torch.cuda.synchronize()
    (d1, a1, b1), (d0, a0, b0) = outs[True], outs[False]
    assert torch.equal(d1.buf, d0.buf) and torch.equal(a1, a0) and torch.equal(b1, b0)
    assert torch.equal(d1.amax, d0.amax) and d1.pair is not None and d0.pair is None
    img, bound = d1.pair
    bnd = bound.item()
    assert bnd >= d1.buf.abs().max().item()
    ref_img = _pair_image_ref(d1.buf.reshape(d1.M, C), bnd)
    assert torch.equal(img.view(torch.float16).view(d1.M, C // 32, 64), ref_img)
    # the dgrad on the pair image vs the exact f32 MFMA path, against float64
    w = torch.randn(C, Cin, 3, 3, generator=g) / (9 * C) ** 0.5
    wp = K.pack_weight(w.to(dev), torch.float32)
    dx64 = torch.nn.grad.conv2d_input((N, Cin, H, W), w.double(), to_nchw(d1.buf).double().cpu(), padding=1)
    prev = K.lib_call_status("dg_get_f32_math")
    errs = {}
    try:
        for m in (2, 0):
            K.call("dg_set_f32_math", m)
            src = K.Act(d1.buf)
            src.amax, src.pair = d1.amax, (d1.pair if m == 2 else None)
            dx = K.Act(K.nhwc(N, H, W, Cin, torch.float32, dev))
            K.conv_dgrad(src, wp, Cin, 3, 1, dx)
            torch.cuda.synchronize()
            errs[m] = _chan_err(to_nchw(dx.buf), dx64, 1)
    finally:
        K.call("dg_set_f32_math", prev)
    h, e = errs[2], errs[0]
    print(f"pair dgrad worst {h.max().item():.3e} exact worst {e.max().item():.3e} bound/max "
          f"{bnd / d1.buf.abs().max().item():.1f}")
    assert (h <= 2 * e + 1e-7).all(), (h.max().item(), e.max().item())
