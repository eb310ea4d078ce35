import os, sys, torch
sys.path.insert(0, "/root/repo")
import torch.nn.functional as F
from dgvcc_amd import kernels as K
dev = "cuda"
for (N, H, W, C, Cout) in [(16, 48, 64, 64, 256), (4, 96, 128, 64, 256), (16, 96, 128, 64, 256), (32, 48, 64, 64, 256), (16, 48, 64, 96, 256)]:
    g = torch.Generator().manual_seed(21)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(Cout, C, 1, 1, generator=g) / C ** 0.5
    b = torch.randn(Cout, generator=g)
    wp = K.pack_weight(w.to(dev), torch.float32)
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double()).permute(0, 2, 3, 1)
    for stats in (False, True):
        for sk in ("1", "0"):
            os.environ["DGVCC_PSPLIT_SHORTK"] = sk
            z = K.Act(K.nhwc(N, H, W, Cout, torch.float32, dev))
            if stats:
                r = K.conv_fwd_stats(K.Act(x.to(dev)), wp, Cout, 1, 0, z, bias=b.to(dev))
            else:
                K.conv_fwd(K.Act(x.to(dev)), wp, Cout, 1, 0, z, bias=b.to(dev))
            torch.cuda.synchronize()
            y = z.buf.cpu().double()
            e = ((y - ref).norm() / ref.norm()).item()
            bad = ((y - ref).abs() > 1e-3).reshape(-1, Cout)
            rows = bad.any(1).nonzero().flatten()
            print(N, H, W, C, Cout, "stats" if stats else "plain", "sk", sk, f"rel {e:.2e}", "bad px", rows.numel(), rows[:5].tolist(), rows[-3:].tolist() if rows.numel() else "", flush=True)
