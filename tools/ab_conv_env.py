"""Same-process A/B of a conv-forward environment switch read per launch (e.g. DGVCC_PSPLIT_INC,
DGVCC_CONV_KORDER) on the sta_final layer shapes, f32 split math (the pre-split kernel serves
forward- and dgrad-shaped launches alike), interleaved rounds, min over rounds.  Prints the max
abs difference between the two arms' outputs (0 when the switch only changes scheduling).
usage: ab_conv_env.py VAR A B [reps] [dtype] [fwd|wgrad] [sta|small|small16|shortk]
(small: launches of 96..256 pre-split tiles -- the ISW trunk's layer3 at 48 x 64 and the sta cls_head
-- for DGVCC_PSPLIT_MIN_TILES)"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dgvcc_amd import kernels as K

var, arms = sys.argv[1], sys.argv[2:4]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
dt = {"f32": torch.float32, "bf16": torch.bfloat16}[sys.argv[5] if len(sys.argv) > 5 else "f32"]
mode = sys.argv[6] if len(sys.argv) > 6 else "fwd"
# (H, W, C, Cout, N, R): the encoder / decoder 3x3 layers and the 1x1 den_dec / memory logits
shapes = [(768, 1024, 64, 64, 16, 3), (384, 512, 128, 128, 16, 3), (192, 256, 128, 256, 16, 3), (192, 256, 256, 256, 16, 3),
          (96, 128, 256, 512, 16, 3), (96, 128, 512, 512, 16, 3), (96, 128, 512, 1024, 16, 3),
          (96, 128, 1024, 512, 16, 3), (192, 256, 512, 256, 16, 3), (192, 256, 896, 256, 16, 1),
          (192, 256, 256, 1024, 16, 1)]
if len(sys.argv) > 7 and sys.argv[7] == "small":
    shapes = [(48, 64, 1024, 256, 16, 1), (48, 64, 256, 256, 16, 3), (48, 64, 512, 256, 16, 3),
              (48, 64, 256, 128, 16, 3), (40, 64, 256, 256, 16, 3), (32, 48, 512, 256, 16, 3),
              (24, 32, 1024, 512, 16, 3)]
if len(sys.argv) > 7 and sys.argv[7] == "small16":  # 256-channel grids of <= 2 rounds (DGVCC_PERS_WIDE_SMALL)
    shapes = [(48, 64, 512, 512, 16, 3), (48, 64, 256, 512, 16, 3), (48, 64, 512, 256, 16, 3), (48, 64, 1024, 256, 16, 1),
              (96, 128, 512, 256, 4, 3)]
if len(sys.argv) > 7 and sys.argv[7] == "shortk":  # 1x1 from 64 channels (two 32-channel K-steps)
    shapes = [(192, 256, 64, 256, 16, 1), (96, 128, 64, 256, 16, 1), (384, 512, 64, 128, 16, 1),
              (96, 128, 128, 512, 16, 1), (48, 64, 256, 1024, 16, 1)]
dev = "cuda"
K.call("dg_set_f32_math", 1)
tot = {a: 0.0 for a in arms}
for H, W, C, Cout, B, R in shapes:
    g = torch.Generator(device=dev).manual_seed(7)
    x = K.Act(torch.randn(B, H, W, C, device=dev, generator=g).to(dt))
    wp = K.pack_weight(torch.randn(Cout, C, R, R, device=dev, generator=g) * 0.05, dt)
    dz = K.Act(torch.randn(B, H, W, Cout, device=dev, generator=g).to(dt))
    dw = torch.empty(Cout, C, R, R, device=dev)

    def run(y):
        if mode == "wgrad":
            K.conv_wgrad(x, dz, R, R // 2, dw)
        else:
            K.conv_fwd(x, wp, Cout, R, R // 2, y)
    outs, ms = {}, {a: [] for a in arms}
    for rnd in range(3):
        for arm in arms:
            os.environ[var] = arm
            y = K.Act(torch.empty(B, H, W, Cout, device=dev, dtype=dt))
            run(y)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                run(y)
            e.record()
            torch.cuda.synchronize()
            ms[arm].append(s.elapsed_time(e) / reps)
            outs[arm] = (dw if mode == "wgrad" else y.buf).float().clone()
    d = (outs[arms[0]] - outs[arms[1]]).abs().max().item()
    fl = 2.0 * B * H * W * C * R * R * Cout
    b = {a: min(ms[a]) for a in arms}
    for a in arms:
        tot[a] += b[a]
    print(f"{H}x{W} {C}->{Cout} {R}x{R}: " + "  ".join(f"{var}={a} {b[a]:.3f} ms ({fl / b[a] / 1e9:.1f} TF/s)" for a in arms)
          + f"  {b[arms[0]] / b[arms[1]]:.3f}x  max abs diff {d:.3e}", flush=True)
print("total " + "  ".join(f"{var}={a} {tot[a]:.3f} ms" for a in arms) + f"  {tot[arms[0]] / tot[arms[1]]:.3f}x", flush=True)
os.environ.pop(var, None)
