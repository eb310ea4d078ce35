"""Evaluation throughput: DGTrainer.test_step frames/s on synthetic
768x1024 frames resident in HBM, batch 1 as the reference's val/test loaders
(configs/*: val_loader batch_size 1), DGModel_final (or --model base) in eval mode,
patch_size 10000 (whole frame, as every shipped config) or --patch for tiled evaluation.

    python tools/bench_eval.py [--frames 50] [--warmup 5] [--precision bf16|fp32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--model", default="final", choices=["final", "base"])
    ap.add_argument("--height", type=int, default=768)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--patch", type=int, default=10000)
    args = ap.parse_args()
    from dgvcc_amd.models import models as M
    from dgvcc_amd.trainers.dgtrainer import DGTrainer
    dev = torch.device("cuda:0")
    model = (M.DGModel_final if args.model == "final" else M.DGModel_base)(pretrained=False)
    model = model.to(dev).set_precision(args.precision).eval()
    os.chdir(tempfile.mkdtemp())
    tr = DGTrainer(2112, "bench_eval", dev, 1000, args.patch, "final" if args.model == "final" else "base")
    g = torch.Generator(device=dev).manual_seed(0)
    frames = [torch.randn(1, 3, args.height, args.width, generator=g, device=dev) for _ in range(4)]
    gt = torch.zeros(1, 100, 2)
    batch = lambda i: (frames[i % 4], frames[i % 4], gt, ["x"], [(0, 0, 0, 0)])  # noqa: E731
    with torch.no_grad():
        for i in range(args.warmup):
            tr.test_step(model, batch(i))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.frames):
            tr.test_step(model, batch(i))  # ends in the reference's .item() sync per frame
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(json.dumps({"metric": "eval_frames_per_s", "value": args.frames / dt, "unit": "frames/s",
                      "ms_per_frame": 1e3 * dt / args.frames, "precision": args.precision,
                      "config": {"model": f"DGModel_{args.model}", "frame": [args.height, args.width],
                                 "patch_size": args.patch, "batch": 1}}))


if __name__ == "__main__":
    main()
