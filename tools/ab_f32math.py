"""Same-process A/B of the f32 conv arithmetics on the headline's layer shapes (batch 16,
768x1024 frame): dg_set_f32_math 1 (3-way bf16 split, 6 products) vs 2 (f16 x3 where the
kernel has it), forward and dgrad, interleaved rounds; plus each arithmetic's error against
float64 (CPU) on a 1-image slice of the same launch.
usage: python tools/ab_f32math.py [rounds] [batch]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from dgvcc_amd import kernels as K

R_ = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
H0, W0 = 768, 1024
layers = [  # (H, W, C, Cout, R)
    (H0, W0, 64, 64, 3), (H0 // 2, W0 // 2, 64, 128, 3), (H0 // 2, W0 // 2, 128, 128, 3),
    (H0 // 4, W0 // 4, 128, 256, 3), (H0 // 4, W0 // 4, 256, 256, 3),
    (H0 // 8, W0 // 8, 256, 512, 3), (H0 // 8, W0 // 8, 512, 512, 3),
    (H0 // 16, W0 // 16, 512, 512, 3), (H0 // 16, W0 // 16, 512, 1024, 3), (H0 // 16, W0 // 16, 1024, 512, 3),
    (H0 // 8, W0 // 8, 1024, 512, 3), (H0 // 4, W0 // 4, 512, 256, 3),
]
dev = "cuda"


def timeit(fn, it=5):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


tot = {1: [0.0, 0.0, 0.0], 2: [0.0, 0.0, 0.0]}
for (H, W, C, Cout, R) in layers:
    g = torch.Generator(device="cpu").manual_seed(H * 7 + C)
    xc = torch.relu(torch.randn(B, H, W, C, generator=g))          # post-ReLU activations
    gyc = torch.randn(B, H, W, Cout, generator=g) * 1e-3              # gradients, small scale
    wc = torch.randn(Cout, C, R, R, generator=g) * (2.0 / (C * R * R)) ** 0.5
    x, gy = K.Act(xc.to(dev)), K.Act(gyc.to(dev))
    y, dx = K.Act(torch.empty(B, H, W, Cout, device=dev)), K.Act(torch.empty(B, H, W, C, device=dev))
    dw = torch.empty(Cout, C, R, R, device=dev)
    wp = K.pack_weight(wc.to(dev), torch.float32)
    fl = 2.0 * B * H * W * C * Cout * R * R
    res = {}
    for rnd in range(R_):
        for m in (1, 2):
            K.call("dg_set_f32_math", m)
            t1 = timeit(lambda: K.conv_fwd(x, wp, Cout, R, R // 2, y))
            t2 = timeit(lambda: K.conv_dgrad(gy, wp, C, R, R // 2, dx))
            t3 = timeit(lambda: K.conv_wgrad(x, gy, R, R // 2, dw))
            res.setdefault(m, []).append((t1, t2, t3))
    err = {}
    if H >= H0 // 2:  # float64 reference on the CPU too slow at full / half resolution
        err = {1: (float("nan"),) * 2, 2: (float("nan"),) * 2}
    x64 = xc[:1].permute(0, 3, 1, 2).double()
    g64 = gyc[:1].permute(0, 3, 1, 2).double()
    y64 = F.conv2d(x64, wc.double(), padding=R // 2) if not err else None
    dx64 = torch.nn.grad.conv2d_input(x64.shape, wc.double(), g64, padding=R // 2) if not err else None
    for m in ((1, 2) if not err else ()):
        K.call("dg_set_f32_math", m)
        K.conv_fwd(x, wp, Cout, R, R // 2, y)
        K.conv_dgrad(gy, wp, C, R, R // 2, dx)
        yh = y.buf[:1].permute(0, 3, 1, 2).double().cpu()
        dxh = dx.buf[:1].permute(0, 3, 1, 2).double().cpu()
        err[m] = (float((yh - y64).abs().max() / y64.abs().max()), float((dxh - dx64).abs().max() / dx64.abs().max()))
    K.call("dg_set_f32_math", 1)
    e32 = float("nan")
    if y64 is not None:
        y32 = F.conv2d(x64.float(), wc, padding=R // 2).double()
        e32 = float((y32 - y64).abs().max() / y64.abs().max())
    line = f"{H:4d}x{W:<4d} C{C:5d}->{Cout:5d}:"
    for m in (1, 2):
        t1 = sorted(t[0] for t in res[m])[len(res[m]) // 2]
        t2 = sorted(t[1] for t in res[m])[len(res[m]) // 2]
        t3 = sorted(t[2] for t in res[m])[len(res[m]) // 2]
        tot[m][0] += t1
        tot[m][1] += t2
        tot[m][2] += t3
        line += (f" | m{m} fwd {t1:7.3f} ms {fl / t1 / 1e9:6.1f} TF dgrad {t2:7.3f} ms {fl / t2 / 1e9:6.1f} TF"
                 f" wgrad {t3:7.3f} ms {fl / t3 / 1e9:6.1f} TF err {err[m][0]:.1e}/{err[m][1]:.1e}")
    print(line + f" | torch f32 fwd err {e32:.1e}", flush=True)
for m in (1, 2):
    print(f"TOTAL math {m}: fwd {tot[m][0]:.3f} ms  dgrad {tot[m][1]:.3f} ms  wgrad {tot[m][2]:.3f} ms")
