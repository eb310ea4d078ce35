"""Same-process A/B of the channel-stationary elementwise passes (BN backward apply, residual
join bn_add_apply, BN apply) under an environment switch read per launch (DGVCC_EW_UNROLL 1 / 2,
DGVCC_EW_GRID block caps), f32 and bf16, on the trunk / encoder activation shapes; interleaved
rounds, best of rounds, bytes = the algorithmic reads + writes.  Prints the max abs difference
between the first arm and each other (0: same arithmetic).
usage: bench_bn.py [VAR v1 v2 ...]   (default DGVCC_EW_UNROLL 1 2)"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dgvcc_amd import kernels as K

reps = 10
dev = "cuda"
var, arms = (sys.argv[1], sys.argv[2:]) if len(sys.argv) > 2 else ("DGVCC_EW_UNROLL", ["1", "2"])
# (pixels, channels): ResNet layer1 / layer2 / layer3 at 768x1024 b16, VGG enc1 / enc3
shapes = [(16 * 768 * 1024, 64), (16 * 192 * 256, 256), (16 * 96 * 128, 512), (16 * 48 * 64, 1024), (16 * 384 * 512, 128),
          (16 * 192 * 256, 64)]


def timed(fn):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for dt in (torch.bfloat16, torch.float32):
    es = torch.tensor([], dtype=dt).element_size()
    for M, C in shapes:
        g = torch.Generator(device=dev).manual_seed(3)
        a = torch.randn(M, C, device=dev, generator=g).to(dt)
        b = torch.randn(M, C, device=dev, generator=g).to(dt)
        out = torch.empty(M, C, device=dev, dtype=dt)
        st = torch.stack([torch.zeros(C, device=dev), torch.rand(C, device=dev) + 0.5,
                          torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1])
        coef = torch.randn(3, C, device=dev) * 0.1
        am = torch.zeros(K.amax_words(C), device=dev)  # ABI 6: [1 + C] words (rounded up to 4) for f32 outputs
        amp = K.ptr(am) if dt == torch.float32 else None  # the f32 passes' operand maxima (f16 x3 scales)
        dtc = K.DTYPES[dt] if hasattr(K, "DTYPES") else (0 if dt == torch.float32 else 1)
        ops = {
            "bn_bwd_apply": (3, lambda: K.call("dg_bn_bwd_apply_coef", dtc, K.ptr(a), C, K.ptr(b), C, M, C,
                                                K.ptr(st[0]), K.ptr(st[1]), K.ptr(st[2]), K.ptr(st[3]), 1, 0, 0,
                                                K.ptr(coef), K.ptr(out), C, None, K.stream())),
            "bn_add_apply": (3, lambda: K.call("dg_bn_add_apply", dtc, K.ptr(a), C, M, C, K.ptr(st[2]), K.ptr(st[3]),
                                                K.ptr(b), C, K.ptr(st[2]), K.ptr(st[3]), 1, K.ptr(out), C,
                                                None, K.stream())),
            "bn_apply": (2, lambda: K.call("dg_bn_apply", dtc, K.ptr(a), C, M, C, K.ptr(st[2]), K.ptr(st[3]), 1, 0, 0,
                                           K.ptr(out), C, None, K.stream())),
        }
        if amp is not None:
            ops["bn_apply+amax"] = (2, lambda: K.call("dg_bn_apply", dtc, K.ptr(a), C, M, C, K.ptr(st[2]),
                                                      K.ptr(st[3]), 1, 0, 0, K.ptr(out), C, amp, K.stream()))
            ops["bn_bwd_apply+amax"] = (3, lambda: K.call("dg_bn_bwd_apply_coef", dtc, K.ptr(a), C, K.ptr(b), C, M, C,
                                                          K.ptr(st[0]), K.ptr(st[1]), K.ptr(st[2]), K.ptr(st[3]), 1,
                                                          0, 0, K.ptr(coef), K.ptr(out), C, amp, K.stream()))
        for name, (nstream, fn) in ops.items():
            ms, res = {x: [] for x in arms}, {}
            for rnd in range(3):
                for arm in arms:
                    os.environ[var] = arm
                    ms[arm].append(timed(fn))
                    res[arm] = out.float().clone()
            d = max((res[arms[0]] - res[x]).abs().max().item() for x in arms)
            by = nstream * M * C * es
            best = {x: min(ms[x]) for x in arms}
            print(f"{name:13s} {str(dt)[6:]:8s} M={M:8d} C={C:5d}: " +
                  "  ".join(f"{x}: {best[x]:.3f} ms {by / best[x] / 1e6:6.0f} GB/s" for x in arms) +
                  f"  diff {d:.1e}", flush=True)
os.environ.pop(var, None)
