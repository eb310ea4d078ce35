"""Run one conv layer's fwd/dgrad/wgrad a few times (for rocprofv3 counters).
usage: prof_conv_one.py H W C Cout R B [kinds]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dgvcc_amd import kernels as K

H, W, C, Cout, R, B = (int(v) for v in sys.argv[1:7])
kinds = sys.argv[7] if len(sys.argv) > 7 else "fwd,wgrad"
dt = torch.float32 if os.environ.get("DGVCC_PROF_DT", "bf16") == "f32" else torch.bfloat16
dev = "cuda"
x = K.Act(torch.randn(B, H, W, C, device=dev).to(dt))
gy = K.Act(torch.randn(B, H, W, Cout, device=dev).to(dt))
y = K.Act(torch.empty(B, H, W, Cout, device=dev, dtype=dt))
dx = K.Act(torch.empty(B, H, W, C, device=dev, dtype=dt))
wp = K.pack_weight(torch.randn(Cout, C, R, R, device=dev) * 0.05, dt)
dw = torch.empty(Cout, C, R, R, device=dev)
for _ in range(5):
    if "fwd" in kinds:
        K.conv_fwd(x, wp, Cout, R, R // 2, y)
    if "dgrad" in kinds:
        K.conv_dgrad(gy, wp, C, R, R // 2, dx)
    if "wgrad" in kinds:
        K.conv_wgrad(x, gy, R, R // 2, dw)
torch.cuda.synchronize()
print("done")
