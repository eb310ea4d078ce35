"""ResNet-trunk kernels (IBN-Net b / ISW / SW backbones) on the GPU against
plain PyTorch fp32 on the CPU: strided/any-R convolution (fwd, dgrad, wgrad),
the Cin=3 7x7/2 stem through im2col, MaxPool2d(3,2,1), the Bottleneck
residual join, InstanceNorm2d (affine / not) forward+backward.
"""
import pytest
import torch
import torch.nn.functional as F

from test_kernels_gpu import relerr, to_nchw, to_nhwc

pytestmark = pytest.mark.gpu


def _k():
    from dgvcc_amd import kernels as K
    return K


CONV2D_CASES = [
    # N, H, W, C, Cout, R, stride, pad
    (2, 17, 15, 64, 128, 3, 2, 1),   # layer2/3 conv2 (stride in the 3x3, odd sizes)
    (2, 16, 16, 128, 64, 1, 2, 0),   # downsample 1x1/2
    (2, 15, 13, 256, 128, 1, 2, 0),  # downsample on odd sizes
    (1, 9, 11, 64, 64, 3, 1, 1),     # stride-1 3x3 through the general kernel
    (1, 12, 10, 256, 64, 1, 1, 0),   # bottleneck conv1/conv3
    (2, 11, 9, 64, 128, 7, 2, 3),    # 7x7/2
    (1, 10, 10, 64, 64, 3, 2, 0),    # stride 2, no padding
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CONV2D_CASES)
def test_conv2d_general(dev, dtype, case):
    K = _k()
    N, H, W, C, Cout, R, s, p = case
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(Cout, C, R, R, generator=g) / (C * R * R) ** 0.5
    b = torch.randn(Cout, generator=g)
    P, Q = K.conv_out(H, R, s, p), K.conv_out(W, R, s, p)
    gy = torch.randn(N, Cout, P, Q, generator=g)
    if dtype != torch.float32:
        x, w, gy = x.to(dtype).float(), w.to(dtype).float(), gy.to(dtype).float()
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, b, stride=s, padding=p)
    yr.backward(gy)

    xd = K.Act(to_nhwc(x).to(dev, dtype))
    wp = K.pack_weight(w.to(dev), dtype)
    y = K.Act(K.nhwc(N, P, Q, Cout, dtype, dev))
    K.conv2d_fwd(xd, wp, Cout, R, s, p, y, bias=b.to(dev))
    gyd = K.Act(to_nhwc(gy).to(dev, dtype))
    wt = K.pack_weight_t(wp, Cout, C, R, R)
    dx = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    K.conv2d_dgrad(gyd, wt, R, s, p, dx)
    dw = torch.empty(Cout, C, R, R, device=dev)
    K.conv2d_wgrad(xd, gyd, R, s, p, dw)
    torch.cuda.synchronize()
    tol = 2e-5 if dtype == torch.float32 else 1.5e-2
    assert relerr(to_nchw(y.buf.float()), yr.detach()) < tol
    assert relerr(to_nchw(dx.buf.float()), xr.grad) < tol
    assert relerr(dw, wr.grad) < (2e-5 if dtype == torch.float32 else 2e-3)


def test_conv2d_slices_accumulate(dev):
    """Channel-slice inputs/outputs (pixel stride > C) and accumulate=True."""
    K = _k()
    N, H, W, C, Cout = 2, 14, 12, 64, 64
    g = torch.Generator().manual_seed(2)
    big = torch.randn(N, H, W, 3 * C, generator=g)
    w = torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** 0.5
    x = big[..., C:2 * C].permute(0, 3, 1, 2)
    ref = F.conv2d(x, w, stride=2, padding=1)
    P, Q = ref.shape[2:]
    base = torch.randn(N, P, Q, 2 * Cout, generator=g)
    xd = K.Act(big.to(dev), C, C)
    out = base.to(dev)
    y = K.Act(out, Cout, Cout)
    K.conv2d_fwd(xd, K.pack_weight(w.to(dev), torch.float32), Cout, 3, 2, 1, y, accumulate=True)
    torch.cuda.synchronize()
    exp = base.clone()
    exp[..., Cout:] += to_nhwc(ref)
    assert relerr(out, exp) < 2e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_stem_im2col_7x7(dev, dtype):
    """ResNet stem conv1 7x7/2 pad 3, Cin=3 -> 64 (resnet_ibn.py:158) as a 1x1 GEMM
    over im2col rows (K = 147 padded to 192)."""
    K = _k()
    N, H, W, Cout, R, s, p, kp = 2, 33, 31, 64, 7, 2, 3, 192
    g = torch.Generator().manual_seed(3)
    img = torch.randn(N, 3, H, W, generator=g)
    w = torch.randn(Cout, 3, R, R, generator=g) / 147 ** 0.5
    P, Q = K.conv_out(H, R, s, p), K.conv_out(W, R, s, p)
    gy = torch.randn(N, Cout, P, Q, generator=g)
    if dtype != torch.float32:
        img, w, gy = img.to(dtype).float(), w.to(dtype).float(), gy.to(dtype).float()
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(img, wr, stride=s, padding=p)
    yr.backward(gy)

    col = K.Act(K.im2col_c3_general(img.to(dev), dtype, R, s, p, kp))
    assert col.buf.shape == (N, P, Q, kp)
    wp = K.pack_weight(w.to(dev), dtype, cpad=3, row_len=kp)
    y = K.Act(K.nhwc(N, P, Q, Cout, dtype, dev))
    K.conv2d_fwd(col, wp, Cout, 1, 1, 0, y, k_alg=147)
    dwcol = torch.empty(Cout, kp, device=dev)
    K.conv2d_wgrad(col, K.Act(to_nhwc(gy).to(dev, dtype)), 1, 1, 0, dwcol)
    dw = torch.empty(Cout, 3, R, R, device=dev)
    K.unpack_c3(dwcol, dw)
    torch.cuda.synchronize()
    tol = 2e-5 if dtype == torch.float32 else 1.5e-2
    assert relerr(to_nchw(y.buf.float()), yr.detach()) < tol
    assert relerr(dw, wr.grad) < (2e-5 if dtype == torch.float32 else 2e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(2, 64, 17, 15), (1, 128, 16, 16), (1, 64, 2, 3)])
def test_maxpool_3x3_s2(dev, dtype, shape):
    """nn.MaxPool2d(3, 2, 1) with ties (first max wins, as ATen's CPU kernel)."""
    K = _k()
    N, C, H, W = shape
    g = torch.Generator().manual_seed(4)
    x = torch.randint(-3, 4, (N, C, H, W), generator=g).float()  # many ties
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    gy = torch.randn(yr.shape, generator=g)
    if dtype != torch.float32:
        gy = gy.to(dtype).float()
    yr.backward(gy)
    P, Q = yr.shape[2:]
    xd = K.Act(to_nhwc(x).to(dev, dtype))
    y = K.Act(K.nhwc(N, P, Q, C, dtype, dev))
    K.maxpool_k_fwd(xd, 3, 2, 1, y)
    gx = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    K.maxpool_k_bwd(xd, K.Act(to_nhwc(gy).to(dev, dtype)), 3, 2, 1, gx)
    torch.cuda.synchronize()
    assert torch.equal(to_nchw(y.buf.float()).cpu(), yr.detach())
    tol = 1e-6 if dtype == torch.float32 else 1e-2  # bf16: sums of up to 4 window grads
    assert relerr(to_nchw(gx.buf.float()), xr.grad) < tol
    # argmax-recording variant: identical pooled values and gradients (same summation order)
    y2 = K.Act(K.nhwc(N, P, Q, C, dtype, dev))
    idx = K.maxpool_k_fwd_idx(xd, 3, 2, 1, y2)
    gx2 = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    K.maxpool_k_bwd_idx(idx, K.Act(to_nhwc(gy).to(dev, dtype)), 3, 2, 1, gx2)
    torch.cuda.synchronize()
    assert torch.equal(y2.buf, y.buf) and torch.equal(gx2.buf, gx.buf)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("downsample", [False, True])
def test_bn_add_relu_join(dev, dtype, downsample):
    K = _k()
    N, H, W, C = 2, 7, 9, 256
    g = torch.Generator().manual_seed(5)
    z1 = torch.randn(N, H, W, C, generator=g)
    z2 = torch.randn(N, H, W, C, generator=g)
    st1 = torch.randn(4, C, generator=g)
    st2 = torch.randn(4, C, generator=g)
    if dtype != torch.float32:
        z1, z2 = z1.to(dtype).float(), z2.to(dtype).float()
    short = z2 * st2[2] + st2[3] if downsample else z2
    ref = torch.relu(z1 * st1[2] + st1[3] + short)
    y = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    K.bn_add_apply(K.Act(z1.to(dev, dtype)), st1.to(dev), K.Act(z2.to(dev, dtype)),
                   st2.to(dev) if downsample else None, 1, y)
    gg = torch.randn(N, H, W, C, generator=g)
    gout = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    K.relu_bwd(K.Act(gg.to(dev, dtype)), y, gout)
    torch.cuda.synchronize()
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    assert relerr(y.buf.float(), ref) < tol
    if dtype == torch.float32:  # the join's maxima (the next f16 x3 convs' operand bounds), exact: tensor, channels
        assert y.amax is not None and y.amax[0].item() == y.buf.abs().max().item()
        assert torch.equal(y.amax[1:1 + C], y.buf.abs().amax(dim=(0, 1, 2)))
    mask = (y.buf.float().cpu() > 0).float()
    assert torch.equal(gout.buf.float().cpu(), gg.to(dtype).float() * mask)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("affine", [True, False])
@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("shape", [(2, 64, 13, 11), (3, 128, 32, 20)])
def test_instance_norm(dev, dtype, affine, act, shape):
    """nn.InstanceNorm2d(C, affine) (+ReLU): IBN-b stem/layer ends, ISW InstanceWhitening."""
    K = _k()
    N, C, H, W = shape
    g = torch.Generator().manual_seed(6)
    x = torch.randn(N, C, H, W, generator=g) * 3 + 1
    gam = torch.randn(C, generator=g) if affine else None
    bet = torch.randn(C, generator=g) if affine else None
    gy = torch.randn(N, C, H, W, generator=g)
    if dtype != torch.float32:
        x, gy = x.to(dtype).float(), gy.to(dtype).float()
    xr = x.clone().requires_grad_(True)
    gr = gam.clone().requires_grad_(True) if affine else None
    br = bet.clone().requires_grad_(True) if affine else None
    yr = F.instance_norm(xr, weight=gr, bias=br, eps=1e-5)
    if act:
        yr = torch.relu(yr)
    yr.backward(gy)

    xd = K.Act(to_nhwc(x).to(dev, dtype))
    st = K.instnorm_stats(xd, 1e-5)
    gd, bd = (gam.to(dev), bet.to(dev)) if affine else (None, None)
    y = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    K.instnorm_apply(xd, st, gd, bd, act, y)
    gyd = K.Act(to_nhwc(gy).to(dev, dtype))
    if act:
        K.relu_bwd(gyd, y, gyd)
    dx = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    dgam = torch.empty(C, device=dev) if affine else None
    dbet = torch.empty(C, device=dev) if affine else None
    K.instnorm_bwd(gyd, xd, st, gd, dx, dgam, dbet)
    torch.cuda.synchronize()
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert relerr(to_nchw(y.buf.float()), yr.detach()) < tol
    assert relerr(to_nchw(dx.buf.float()), xr.grad) < (1e-4 if dtype == torch.float32 else 3e-2)
    if affine:
        assert relerr(dgam, gr.grad) < (2e-5 if dtype == torch.float32 else 1e-2)
        assert relerr(dbet, br.grad) < (2e-5 if dtype == torch.float32 else 1e-2)
    if dtype == torch.float32:  # max |y| and max |dx| from the apply passes, exact: tensor and channels
        for t in (y, dx):
            assert t.amax[0].item() == t.buf.abs().max().item()
            assert torch.equal(t.amax[1:1 + t.C], t.buf.abs().amax(dim=(0, 1, 2)))


def _sw_params(C, g):
    return dict(sw_mean_weight=torch.randn(2, generator=g), sw_var_weight=torch.randn(2, generator=g),
                weight=torch.rand(C, generator=g) + 0.5, bias=torch.randn(C, generator=g) * 0.1,
                running_mean=torch.randn(C // 16, 16, 1, generator=g) * 0.1,
                running_cov=torch.eye(16).repeat(C // 16, 1, 1))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(3, 64, 9, 7), (2, 256, 6, 5), (2, 32, 12, 10)])
@pytest.mark.parametrize("act", [0, 1])
def test_switch_whiten(dev, dtype, shape, act):
    """SwitchWhiten2d sw_type 2 forward/backward vs the float64 oracle restatement of
    models/SW/ops/switchwhiten.py:84-183 (itself pinned by tests/golden/sw_op.npz)."""
    from oracle import trunk_oracle as TO
    K = _k()
    N, C, H, W = shape
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, C, H, W, generator=g) * 1.5 + 0.3
    gy = torch.randn(N, C, H, W, generator=g)
    if dtype != torch.float32:
        x, gy = x.to(dtype).float(), gy.to(dtype).float()
    p = _sw_params(C, g)
    sd = {k: v.double().clone().requires_grad_(k in ("sw_mean_weight", "sw_var_weight", "weight", "bias"))
          for k, v in p.items()}
    xr = x.double().requires_grad_(True)
    yr = TO.switch_whiten(xr, sd, "", True, T=5, eps=1e-5, momentum=0.9)
    if act:
        yr = torch.relu(yr)
    yr.backward(gy.double())

    pd = {k: v.to(dev) for k, v in p.items()}
    xd = K.Act(to_nhwc(x).to(dev, dtype))
    y = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    save = K.sw_fwd(xd, pd["sw_mean_weight"], pd["sw_var_weight"], pd["weight"], pd["bias"],
                    pd["running_mean"], pd["running_cov"], True, act, y)
    dx = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    d = {k: torch.empty(p[k].shape, device=dev) for k in ("weight", "bias", "sw_mean_weight", "sw_var_weight")}
    K.sw_bwd(K.Act(to_nhwc(gy).to(dev, dtype)), y if act else None, xd, save, pd["sw_mean_weight"],
             pd["sw_var_weight"], pd["weight"], act, dx, d["weight"], d["bias"], d["sw_mean_weight"],
             d["sw_var_weight"])
    torch.cuda.synchronize()
    f32 = dtype == torch.float32
    assert relerr(to_nchw(y.buf.float()), yr.detach()) < (1e-4 if f32 else 3e-2)
    assert relerr(to_nchw(dx.buf.float()), xr.grad) < (1e-3 if f32 else 5e-2)
    for k in d:
        assert relerr(d[k], sd[k].grad) < (1e-3 if f32 else 5e-2), k
    assert relerr(pd["running_mean"], sd["running_mean"]) < (1e-4 if f32 else 1e-2)
    assert relerr(pd["running_cov"], sd["running_cov"]) < (1e-4 if f32 else 1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(3, 64, 9, 7), (2, 256, 24, 20), (16, 128, 12, 16)])
def test_switch_whiten_apply_mfma(dev, dtype, shape, monkeypatch):
    """The whitening applies on the matrix cores (sw_apply_mfma / sw_bwd_apply_mfma, default) against the
    thread-per-(pixel, group) FMA forms (DGVCC_SW_APPLY=0): same products, another summation order --
    f32 within 2e-6 relative, 16-bit within one rounding; ragged pixel tails, ReLU, accumulate."""
    K = _k()
    N, C, H, W = shape
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, C, H, W, generator=g) * 1.5 + 0.3
    gy = torch.randn(N, C, H, W, generator=g)
    p = {k: v.to(dev) for k, v in _sw_params(C, g).items()}
    dx0 = to_nhwc(torch.randn(N, C, H, W, generator=g)).to(dev, dtype)
    outs = []
    for mode in ("0", "1"):
        monkeypatch.setenv("DGVCC_SW_APPLY", mode)
        pm = {k: v.clone() for k, v in p.items()}
        xd = K.Act(to_nhwc(x).to(dev, dtype))
        y = K.Act(K.nhwc(N, H, W, C, dtype, dev))
        save = K.sw_fwd(xd, pm["sw_mean_weight"], pm["sw_var_weight"], pm["weight"], pm["bias"],
                        pm["running_mean"], pm["running_cov"], True, 1, y)
        dx = K.Act(dx0.clone())
        K.sw_bwd(K.Act(to_nhwc(gy).to(dev, dtype)), y, xd, save, pm["sw_mean_weight"], pm["sw_var_weight"],
                 pm["weight"], 1, dx, accumulate=True)
        torch.cuda.synchronize()
        outs.append((y.buf.float().cpu(), dx.buf.float().cpu()))
    tol = 2e-6 if dtype == torch.float32 else 1e-2
    assert relerr(outs[1][0], outs[0][0]) < tol
    assert relerr(outs[1][1], outs[0][1]) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C", [64, 256])
def test_iw_loss_and_grad(dev, dtype, C):
    """instance_whitening_loss (models/ISW/instance_whitening.py:19-39): per-instance
    Gram on the wgrad GEMM, masked L1 loss, and its gradient as a 1x1 conv."""
    from oracle import trunk_oracle as TO
    from dgvcc_amd import trunk as TR
    K = _k()
    N, H, W = 3, 9, 7
    g = torch.Generator().manual_seed(8)
    f = torch.randn(N, C, H, W, generator=g)
    f = f + 0.4 * f[:, :1]
    if dtype != torch.float32:
        f = f.to(dtype).float()
    var = TO.cov_variance(f.double())
    mask, ns = TO.sensitive_mask(var, 1)
    fr = f.double().requires_grad_(True)
    loss_ref = TO.whitening_loss(fr, mask, ns) / 3.0
    loss_ref.backward()
    w = K.Act(to_nhwc(f).to(dev, dtype))
    fraw = TR.gram(w)
    # cal_covstat variance on the device Grams
    vd = torch.empty(C, C, device=dev)
    K.iw_cov_var(fraw, H * W, vd)
    loss = torch.zeros((), device=dev)
    nsd = torch.tensor(ns, device=dev)
    K.iw_loss(fraw, H * W, mask.float().to(dev), nsd, 1.0 / 3.0, loss, accumulate=True, want_grad=False)
    gt = K.Act(K.nhwc(N, H, W, C, dtype, dev, zero=True))
    # fp16: the trainer's loss scale reaches this hook as its upstream coefficient (the unscaled
    # gradient, ~1e-5 here, would sit in f16's subnormal range)
    gscale = 1024.0 if dtype == torch.float16 else 1.0
    hook = TR._iw_grad_hook(w, fraw, mask.float().to(dev), nsd, 1.0 / 3.0, torch.full((), gscale, device=dev))
    hook(gt)
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert relerr(vd, var) < (1e-4 if dtype == torch.float32 else 3e-2)
    assert abs(loss.item() - loss_ref.item()) <= tol * abs(loss_ref.item())
    assert relerr(to_nchw(gt.buf.float()) / gscale, fr.grad) < (1e-5 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_bias_relu_bwd_no_norm(dev, dtype):
    """dg_bn_bwd without normalisation (counter-head Conv+bias+ReLU): dz = g*(z>0),
    dbias = sum dz."""
    K = _k()
    N, H, W, C = 2, 5, 7, 128
    g = torch.Generator().manual_seed(9)
    z = torch.randn(N, H, W, C, generator=g)
    gy = torch.randn(N, H, W, C, generator=g)
    if dtype != torch.float32:
        z, gy = z.to(dtype).float(), gy.to(dtype).float()
    dz = K.Act(K.nhwc(N, H, W, C, dtype, dev))
    db = torch.empty(C, device=dev)
    dbias = torch.empty(C, device=dev)
    K.bn_bwd(K.Act(gy.to(dev, dtype)), K.Act(z.to(dev, dtype)), None, None, 1, dz, None, db, dbias)
    torch.cuda.synchronize()
    ref = gy * (z > 0)
    assert torch.equal(dz.buf.float().cpu(), ref.to(dtype).float())
    assert relerr(db, ref.sum(dim=(0, 1, 2))) < 1e-5
    assert relerr(dbias, ref.sum(dim=(0, 1, 2))) < 1e-5


def test_sync_switch_whiten_two_ranks(dev):
    """SyncSwitchWhiten2d (a17): 2 ranks (gloo, one GPU) on half batches each reproduce
    the full-batch SwitchWhiten2d forward, running statistics, input and parameter
    gradients (batch moments and their adjoints all-reduced between kernel phases)."""
    import os
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={port}",
                        os.path.join(here, "sync_sw_worker.py")],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.count("OK") == 2, (r.stdout[-2000:], r.stderr[-3000:])


ACC_RELU_CASES = [
    # N, H, W, planes (dgrad input channels), C (dgrad output channels = the ReLU output's)
    (2, 48, 64, 64, 256),    # layer1 conv1 dgrad
    (2, 24, 32, 128, 512),   # layer2
    (2, 12, 16, 256, 1024),  # layer3 (16-bit split-K grid: the two-launch fallback)
    (4, 96, 128, 64, 256),   # persistent grids
    (2, 48, 64, 256, 64),    # 64 output channels
    (1, 5, 7, 64, 128),      # ragged pixel tail
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", ACC_RELU_CASES)
def test_conv_dgrad_acc_relu(dev, dtype, case):
    """dg_conv_fwd_acc_relu == accumulating 1x1 dgrad followed by relu_bwd, bit for bit (the
    mask applied to the same rounded sum), including exact zeros in the ReLU output."""
    K = _k()
    N, H, W, Cp, C = case
    g = torch.Generator().manual_seed(11)
    dy = K.Act(torch.randn(N, H, W, Cp, generator=g).to(dev, dtype))
    wp = K.pack_weight((torch.randn(Cp, C, 1, 1, generator=g) / Cp ** 0.5).to(dev), dtype)
    ro = K.Act(torch.relu(torch.randn(N, H, W, C, generator=g)).to(dev, dtype))
    base = torch.randn(N, H, W, C, generator=g).to(dev, dtype)
    d1 = K.Act(base.clone())
    K.conv_dgrad(dy, wp, C, 1, 0, d1, accumulate=True)
    K.relu_bwd(d1, ro, d1)
    d2 = K.Act(base.clone())
    fused = K.conv_dgrad_acc_relu(dy, wp, C, d2, ro)
    if not fused:
        K.conv_dgrad(dy, wp, C, 1, 0, d2, accumulate=True)
        K.relu_bwd(d2, ro, d2)
    torch.cuda.synchronize()
    if dtype == torch.float32:
        assert fused
    assert (d2.buf[ro.buf <= 0] == 0).all()
    assert torch.equal(d1.buf, d2.buf)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(2, 67, 131, 7, 2, 3, 192), (1, 33, 200, 3, 1, 1, 32), (3, 16, 16, 5, 2, 2, 80),
                                   (1, 9, 260, 7, 2, 3, 152)])
def test_im2col_lds_matches_gather(dev, dtype, shape, monkeypatch):
    """The LDS-staged stem im2col (one block per 64 output pixels of a row) writes exactly the
    one-thread-per-chunk gather kernel's rows: ragged row tails, padding on every edge, zero K tail."""
    K = _k()
    N, H, W, R, s, p, kp = shape
    img = torch.randn(N, 3, H, W, generator=torch.Generator().manual_seed(5)).to(dev)
    monkeypatch.setenv("DGVCC_IM2COL_LDS", "0")
    ref = K.im2col_c3_general(img, dtype, R, s, p, kp).clone()
    monkeypatch.setenv("DGVCC_IM2COL_LDS", "1")
    got = K.im2col_c3_general(img, dtype, R, s, p, kp)
    torch.cuda.synchronize()
    assert torch.equal(ref, got)
