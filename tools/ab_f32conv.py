"""Time f32 conv forward launches of the sta_final layer shapes under the f32 GEMM modes
(exact f32 MFMA / per-wave split / pre-split filter), HIP events on the launch stream.
usage: ab_f32conv.py [reps]   (DGVCC_AB_SHAPES="H,W,C,Cout,B;..." overrides the shapes)"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dgvcc_amd import kernels as K

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
shapes = [(768, 1024, 64, 64, 16), (384, 512, 128, 128, 16), (192, 256, 256, 256, 16), (96, 128, 512, 512, 16),
          (192, 256, 512, 256, 16), (96, 128, 256, 512, 16)]
if os.environ.get("DGVCC_AB_SHAPES"):
    shapes = [tuple(int(v) for v in s.split(",")) for s in os.environ["DGVCC_AB_SHAPES"].split(";")]
modes = [("exact", 0, "1"), ("split_wave", 1, "0"), ("split_pre", 1, "1")]
kind = os.environ.get("DGVCC_AB_KIND", "fwd")
dev = "cuda"
for H, W, C, Cout, B in shapes:
    x = K.Act(torch.randn(B, H, W, C, device=dev))
    y = K.Act(torch.empty(B, H, W, Cout, device=dev))
    wp = K.pack_weight(torch.randn(Cout, C, 3, 3, device=dev) * 0.05, torch.float32)
    gy = K.Act(torch.randn(B, H, W, Cout, device=dev))
    dw = torch.empty(Cout, C, 3, 3, device=dev)
    run = (lambda: K.conv_fwd(x, wp, Cout, 3, 1, y)) if kind == "fwd" else (lambda: K.conv_wgrad(x, gy, 3, 1, dw))
    flops = 2.0 * B * H * W * C * 9 * Cout
    line = []
    for name, math, pre in modes:
        K.call("dg_set_f32_math", math)
        os.environ["DGVCC_PSPLIT"] = pre
        run()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            run()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / reps
        line.append(f"{name} {ms:7.3f} ms {flops / ms / 1e9:6.1f} TF")
    print(f"{H}x{W} C{C}->{Cout} B{B}: " + " | ".join(line), flush=True)
K.call("dg_set_f32_math", 1)
os.environ["DGVCC_PSPLIT"] = "1"
