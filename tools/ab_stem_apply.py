"""Same-process A/B of the bf16 z-free stem's apply pass grid (DGVCC_STEM_APPLY_BPC, read per
launch): 16 x 3 x 768 x 1024 frames, interleaved rounds, min over rounds; checks that the output
is bit-identical across arms.   usage: python tools/ab_stem_apply.py [arms...]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dgvcc_amd import kernels as K

arms = sys.argv[1:] or ["2", "4", "8"]
dev = "cuda"
N, H, W = 16, 768, 1024
g = torch.Generator(device=dev).manual_seed(3)
img = torch.rand(N, 3, H, W, device=dev, generator=g)
w = torch.randn(64, 3, 3, 3, device=dev, generator=g) * 0.2
wp = K.pack_weight(w, torch.bfloat16, cpad=3, row_len=32)
bias = torch.randn(64, device=dev, generator=g) * 0.1
stats = torch.stack([torch.zeros(64, device=dev), torch.ones(64, device=dev), torch.rand(64, device=dev, generator=g) + 0.5,
                     torch.randn(64, device=dev, generator=g) * 0.1])
outs, best = {}, {a: 1e9 for a in arms}
for rnd in range(5):
    for a in arms:
        os.environ["DGVCC_STEM_APPLY_BPC"] = a
        y = K.Act(torch.empty(N, H, W, 64, device=dev, dtype=torch.bfloat16))
        K.stem_apply(img, wp, bias, stats, y)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            K.stem_apply(img, wp, bias, stats, y)
        e.record()
        torch.cuda.synchronize()
        best[a] = min(best[a], s.elapsed_time(e) / 10)
        outs[a] = y.buf
ref = outs[arms[0]]
for a in arms:
    print(f"DGVCC_STEM_APPLY_BPC={a}: {best[a]:.3f} ms per 16-frame apply, "
          f"{N * H * W * 64 * 2 / best[a] / 1e6:.0f} GB/s written, identical={torch.equal(outs[a], ref)}")
