"""Micro-benchmark of the conv kernels on the VGG16/decoder layer shapes (bf16)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dgvcc_amd import kernels as K

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
dt = torch.bfloat16 if (len(sys.argv) < 3 or sys.argv[2] == "bf16") else torch.float32
H0 = int(sys.argv[3]) if len(sys.argv) > 3 else 768
W0 = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
layers = [  # (H, W, C, Cout, R)
    (H0, W0, 64, 64, 3), (H0 // 2, W0 // 2, 64, 128, 3), (H0 // 2, W0 // 2, 128, 128, 3),
    (H0 // 4, W0 // 4, 128, 256, 3), (H0 // 4, W0 // 4, 256, 256, 3),
    (H0 // 8, W0 // 8, 256, 512, 3), (H0 // 8, W0 // 8, 512, 512, 3),
    (H0 // 16, W0 // 16, 512, 512, 3), (H0 // 16, W0 // 16, 512, 1024, 3), (H0 // 16, W0 // 16, 1024, 512, 3),
    (H0 // 8, W0 // 8, 1024, 512, 3), (H0 // 4, W0 // 4, 512, 256, 3), (H0 // 4, W0 // 4, 896, 256, 1),
]
dev = "cuda"

def timeit(fn, it=10):
    fn(); torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it

tot = {"fwd": [0, 0], "dgrad": [0, 0], "wgrad": [0, 0]}
for (H, W, C, Cout, R) in layers:
    x = K.Act(torch.randn(B, H, W, C, device=dev).to(dt))
    gy = K.Act(torch.randn(B, H, W, Cout, device=dev).to(dt))
    y = K.Act(torch.empty(B, H, W, Cout, device=dev, dtype=dt))
    dx = K.Act(torch.empty(B, H, W, C, device=dev, dtype=dt))
    w = torch.randn(Cout, C, R, R, device=dev) * 0.05
    wp = K.pack_weight(w, dt)
    dw = torch.empty(Cout, C, R, R, device=dev)
    fl = 2.0 * B * H * W * C * Cout * R * R
    t1 = timeit(lambda: K.conv_fwd(x, wp, Cout, R, R // 2, y))
    t2 = timeit(lambda: K.conv_dgrad(gy, wp, C, R, R // 2, dx))
    t3 = timeit(lambda: K.conv_wgrad(x, gy, R, R // 2, dw))
    for k, t in zip(("fwd", "dgrad", "wgrad"), (t1, t2, t3)):
        tot[k][0] += t; tot[k][1] += fl
    print(f"{H:4d}x{W:<4d} C{C:5d}->{Cout:5d} R{R}: fwd {t1:7.3f} ms {fl/t1/1e9:7.1f} TF | dgrad {t2:7.3f} ms {fl/t2/1e9:7.1f} TF | wgrad {t3:7.3f} ms {fl/t3/1e9:7.1f} TF", flush=True)
for k, (t, f) in tot.items():
    print(f"TOTAL {k}: {t:.3f} ms  {f/t/1e9:.1f} TF")
