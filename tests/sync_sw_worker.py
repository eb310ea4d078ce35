"""Worker for test_sync_switch_whiten (launched by torch.distributed.run, 2 ranks on one
GPU, gloo): SyncSwitchWhiten2d on each rank's half batch must equal SwitchWhiten2d on
the full batch (models/SW/ops/sync_switchwhiten.py:9-56 semantics)."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgvcc_amd import dist as D  # noqa: E402
from dgvcc_amd import kernels as K  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    N, H, W, C = 4, 9, 7, 64
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, H, W, C, generator=g) * 1.3 + 0.2
    gy = torch.randn(N, H, W, C, generator=g)
    pr = dict(mw=torch.randn(2, generator=g), vw=torch.randn(2, generator=g),
              gam=torch.rand(C, generator=g) + 0.5, bet=torch.randn(C, generator=g) * 0.1)
    p = {k: v.to(dev) for k, v in pr.items()}
    fails = []
    for act in (0, 1):
        # full batch, one rank
        rm = torch.zeros(C // 16, 16, 1, device=dev)
        rc = torch.zeros(C // 16, 16, 16, device=dev)
        xf = K.Act(x.to(dev))
        yf = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
        save = K.sw_fwd(xf, p["mw"], p["vw"], p["gam"], p["bet"], rm, rc, True, act, yf)
        dxf = K.Act(K.nhwc(N, H, W, C, torch.float32, dev))
        dg = {k: torch.empty(C if k in ("g", "b") else 2, device=dev) for k in ("g", "b", "m", "v")}
        K.sw_bwd(K.Act(gy.to(dev)), yf, xf, save, p["mw"], p["vw"], p["gam"], act, dxf, dg["g"], dg["b"],
                 dg["m"], dg["v"])
        # this rank's half, synchronized
        h = slice(rank * N // world, (rank + 1) * N // world)
        rms = torch.zeros_like(rm)
        rcs = torch.zeros_like(rc)
        xs = K.Act(x[h].contiguous().to(dev))
        ys = K.Act(K.nhwc(N // world, H, W, C, torch.float32, dev))
        red = D.sum_moments(N // world)
        save_s, work, count = K.sw_fwd_sync(xs, p["mw"], p["vw"], p["gam"], p["bet"], rms, rcs, True, act, ys,
                                            red)
        dxs = K.Act(K.nhwc(N // world, H, W, C, torch.float32, dev))
        ds = {k: torch.empty(C if k in ("g", "b") else 2, device=dev) for k in ("g", "b", "m", "v")}
        K.sw_bwd_sync(K.Act(gy[h].contiguous().to(dev)), ys, xs, save_s, work, p["mw"], p["vw"], p["gam"], act,
                      dxs, red, ds["g"], ds["b"], ds["m"], ds["v"])
        for k in ds:
            dist.all_reduce(ds[k])  # parameter gradients: per-rank partial sums
        torch.cuda.synchronize()

        def rel(a, b):
            return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()

        checks = {"count": float(count == N), "y": rel(ys.buf, yf.buf[h]), "dx": rel(dxs.buf, dxf.buf[h]),
                  "rm": rel(rms, rm), "rc": rel(rcs, rc)}
        checks.update({"d" + k: rel(ds[k], dg[k]) for k in ds})
        for k, v in checks.items():
            bad = (v != 1.0) if k == "count" else (v > 1e-4)
            if bad:
                fails.append((act, k, v))
    print(f"RANK{rank} {'OK' if not fails else 'FAIL ' + repr(fails)}", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if not fails else 1)


if __name__ == "__main__":
    main()
