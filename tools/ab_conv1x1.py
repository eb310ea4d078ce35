"""Same-process A/B of the 16-bit 1x1 forward kernels on the ResNet trunks' shapes (batch 16 at
768x1024: layer1 192x256, layer2 96x128, layer3 48x64): the persistent forward (dg_set_persist(1),
the default) against the non-persistent pipe kernel (dg_set_persist(0)), interleaved rounds, best of
3; GB/s on the algorithmic x + w + y bytes.  Prints the max difference between the arms (0: same
arithmetic).  usage: python tools/ab_conv1x1.py [bf16|fp32]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dgvcc_amd import kernels as K  # noqa: E402

dt = torch.float32 if (len(sys.argv) > 1 and sys.argv[1] == "fp32") else torch.bfloat16
dev = "cuda"
B = 16
shapes = [(192, 256, 64, 256), (192, 256, 256, 64), (192, 256, 64, 64), (192, 256, 256, 128),
          (96, 128, 128, 512), (96, 128, 512, 128), (96, 128, 512, 256),
          (48, 64, 256, 1024), (48, 64, 1024, 256), (48, 64, 1024, 512)]


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


es = torch.tensor([], dtype=dt).element_size()
for H, W, C, Cout in shapes:
    g = torch.Generator(device="cpu").manual_seed(1)
    x = K.Act(torch.randn(B, H, W, C, generator=g).to(dev, dt))
    y = K.Act(torch.empty(B, H, W, Cout, device=dev, dtype=dt))
    wp = K.pack_weight((torch.randn(Cout, C, 1, 1, generator=g) * C ** -0.5).to(dev), dt)
    by = es * (B * H * W * (C + Cout) + Cout * C)
    res, ms = {}, {0: [], 1: []}
    for _ in range(3):
        for arm in (1, 0):
            K.call("dg_set_persist", arm)
            ms[arm].append(timed(lambda: K.conv_fwd(x, wp, Cout, 1, 0, y)))
            res[arm] = y.buf.float().clone()
    K.call("dg_set_persist", -1)
    d = (res[0] - res[1]).abs().max().item()
    b = {a: min(v) for a, v in ms.items()}
    print(f"{B}x{H}x{W} {C:4d}->{Cout:4d}: persistent {b[1] * 1e3:7.1f} us {by / b[1] / 1e6:6.0f} GB/s   "
          f"pipe {b[0] * 1e3:7.1f} us {by / b[0] / 1e6:6.0f} GB/s   diff {d:.1e}", flush=True)
