"""Same-process A/B of the C = 1 upsample kernels (upsample_fwd_c1_kernel / upsample_bwd_c1_kernel) against
the per-pixel forms (DGVCC_UP_C1_OFF=1) on the step shapes: the density heads' x4 (16 x 192 x 256 -> 768 x
1024, align_corners=False) and the ResNet trunks' x16 (16 x 48 x 64, align_corners=True).  Interleaved
rounds, best of rounds, microseconds per launch."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dgvcc_amd import kernels as K

dev, reps = "cuda", 20


def timed(fn):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for (N, H, W, sc, mode) in [(16, 192, 256, 4, K.UP_BILINEAR), (16, 48, 64, 16, K.UP_BILINEAR_AC)]:
    x = K.Act(torch.randn(N, H, W, 1, device=dev))
    y = K.Act(torch.empty(N, H * sc, W * sc, 1, device=dev))
    gy = K.Act(torch.randn(N, H * sc, W * sc, 1, device=dev))
    gx = K.Act(torch.empty(N, H, W, 1, device=dev))
    ops = {"fwd": lambda: K.upsample_fwd(x, sc, mode, y), "bwd": lambda: K.upsample_bwd(gy, sc, mode, gx)}
    for name, fn in ops.items():
        best = {}
        for rnd in range(3):
            for arm in ("c1", "off"):
                if arm == "off":
                    os.environ["DGVCC_UP_C1_OFF"] = "1"
                else:
                    os.environ.pop("DGVCC_UP_C1_OFF", None)
                best[arm] = min(best.get(arm, 1e9), timed(fn))
        os.environ.pop("DGVCC_UP_C1_OFF", None)
        print(f"{N}x{H}x{W} x{sc} mode {mode} {name}: c1 {best['c1']:.1f} us  per-pixel {best['off']:.1f} us", flush=True)
