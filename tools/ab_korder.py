"""Same-process A/B of the conv forward K-step order (DGVCC_CONV_KORDER: 0 = tap-major, 1 =
channel-block-major) on the sta_final layer shapes: f32 split math (pre-split kernel) and bf16
(persistent kernel); forward and dgrad-shaped launches are the same kernels.  The two orders sum
the same products in a different order: outputs agree to rounding (max rel diff printed).
usage: ab_korder.py [reps]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dgvcc_amd import kernels as K

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
shapes = [(384, 512, 128, 128, 16), (192, 256, 128, 256, 16), (192, 256, 256, 256, 16), (96, 128, 256, 512, 16),
          (96, 128, 512, 512, 16), (48, 64, 512, 512, 16), (192, 256, 512, 256, 16)]
dev = "cuda"
K.call("dg_set_f32_math", 1)
for dt in (torch.float32, torch.bfloat16):
    tot = {"0": 0.0, "1": 0.0}
    for H, W, C, Cout, B in shapes:
        g = torch.Generator(device=dev).manual_seed(7)
        x = K.Act(torch.randn(B, H, W, C, device=dev, generator=g).to(dt))
        wp = K.pack_weight(torch.randn(Cout, C, 3, 3, device=dev, generator=g) * 0.05, dt)
        outs, ms = {}, {"0": [], "1": []}
        for rnd in range(3):
            for ko in ("0", "1"):
                os.environ["DGVCC_CONV_KORDER"] = ko
                y = K.Act(torch.empty(B, H, W, Cout, device=dev, dtype=dt))
                K.conv_fwd(x, wp, Cout, 3, 1, y)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(reps):
                    K.conv_fwd(x, wp, Cout, 3, 1, y)
                e.record()
                torch.cuda.synchronize()
                ms[ko].append(s.elapsed_time(e) / reps)
                outs[ko] = y.buf.float().clone()
        d = ((outs["0"] - outs["1"]).abs().max() / outs["0"].abs().max()).item()
        fl = 2.0 * B * H * W * C * 9 * Cout
        b0, b1 = min(ms["0"]), min(ms["1"])
        tot["0"] += b0
        tot["1"] += b1
        print(f"{str(dt)[6:]} {H}x{W} {C}->{Cout}: tap-major {b0:.3f} ms ({fl / b0 / 1e9:.1f} TF/s)  block-major {b1:.3f} ms"
              f" ({fl / b1 / 1e9:.1f} TF/s)  {b0 / b1:.3f}x  max rel diff {d:.2e}", flush=True)
    print(f"{str(dt)[6:]} total tap-major {tot['0']:.3f} ms  block-major {tot['1']:.3f} ms  {tot['0'] / tot['1']:.3f}x",
          flush=True)
os.environ["DGVCC_CONV_KORDER"] = "0"
