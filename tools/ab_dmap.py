"""Same-process A/B of the deterministic dmap kernel's tile shapes (DGVCC_DMAP_TILE = 64, 64p,
32, 32p: tile rows, p = first point chunk loaded before the weights) at the bench shapes, each
checked bit-identical to the default.  usage: python tools/ab_dmap.py"""
import os
import sys
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dgvcc_amd import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
for B, H, W in ((16, 768, 1024), (8, 2048, 2048)):
    g = torch.Generator(device="cpu").manual_seed(1000)
    n = torch.poisson(torch.full((B,), 500.0 * H * W / (768 * 1024)), generator=g).long().clamp_min(1)
    flat = torch.cat([torch.rand(int(k), 2, generator=g) * torch.tensor([W, H], dtype=torch.float32) for k in n]).to(dev)
    offs = torch.tensor([0] + torch.cumsum(n, 0).tolist(), dtype=torch.int64, device=dev)
    os.environ["DGVCC_DMAP_TILE"] = "64"
    ref = K.dmap_fixed(flat, offs, B, H, W)
    for v in ("64", "w", "32p", "w", "64"):
        os.environ["DGVCC_DMAP_TILE"] = v
        same = torch.equal(K.dmap_fixed(flat, offs, B, H, W), ref)
        r = bench.dmap_roofline(SimpleNamespace(batch=B, height=H, width=W), dev)
        print(B, H, W, v, r["deterministic"]["us_per_launch"], "fill", r["fill_floor"]["us_per_launch"], "same", same,
              flush=True)
