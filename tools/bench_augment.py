"""Throughput of the GPU DenClsDataset pixel pipeline vs the PIL/torch CPU pipeline it replaces
(oracle/augment_oracle.py, one host thread), and the exact-match rate of the blur."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from dgvcc_amd.datasets.augment import P, augment_den_cls, draw_more_transform, new_record
from oracle import augment_oracle as AO

dev = torch.device("cuda")
for B, H, W in [(16, 320, 320), (16, 768, 1024)]:
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)
    torch.manual_seed(0)
    recs = []
    for i in range(B):
        r = new_record(grey=i % 8 == 0, flip=i % 2 == 1)
        draw_more_transform(r)
        recs.append(r)
    recs = np.stack(recs)
    x = torch.from_numpy(imgs).to(dev)
    p = torch.from_numpy(recs)
    augment_den_cls(x, p)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        a, b = augment_den_cls(x, p)
    torch.cuda.synchronize()
    gpu = (time.perf_counter() - t0) / 20
    t0 = time.perf_counter()
    n = min(B, 4)
    diff = 0
    for i in range(n):
        r1, r2, _, _ = AO.augment(imgs[i], recs[i])
        diff += int((b[i].cpu() != r2).sum()) + int((a[i].cpu() != r1).sum())
    cpu = (time.perf_counter() - t0) / n
    print(f"{B}x{H}x{W}: GPU {gpu*1e3:.3f} ms/batch = {B/gpu:.0f} frames/s; CPU oracle {cpu*1e3:.1f} ms/frame "
          f"= {1/cpu:.1f} frames/s/thread; differing elements in {n} frames: {diff}", flush=True)
