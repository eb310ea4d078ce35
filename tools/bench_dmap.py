"""Time the density-map scatter (deterministic tiled vs atomic, and a plain fill of the map as the write floor) at the bench shapes:
768x1024 x16 frames (Poisson(500) points) and 2048x2048 x8 (qnrf scale).  usage:
python tools/bench_dmap.py"""
import os
import sys
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
for B, H, W in ((16, 768, 1024), (8, 2048, 2048)):
    r = bench.dmap_roofline(SimpleNamespace(batch=B, height=H, width=W), dev)
    print(B, H, W, r["points"], "det", r["deterministic"], "atomic", r["atomic"], "fill", r["fill_floor"], flush=True)
