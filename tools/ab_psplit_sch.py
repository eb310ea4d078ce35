"""Same-process A/B of the f16 x3 256-pixel pre-split forward's schedules (DGVCC_PSPLIT_SCH, read per
launch) on the headline's 256-channel layers at batch 16 (forward of 192x256 256->256 and
96x128 512->512, dgrad of 192x256 512->256): interleaved rounds, best of 3, outputs compared
bitwise against schedule 0.  usage: python tools/ab_psplit_sch.py [schedules, default 0,5; "xs": the pre-split pixel operand]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dgvcc_amd import kernels as K  # noqa: E402

dev = "cuda"
K.call("dg_set_f32_math", 2)
schs = (sys.argv[1] if len(sys.argv) > 1 else "0,5").split(",")


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for (H, W, C, Cout, kind) in [(192, 256, 256, 256, "fwd"), (96, 128, 512, 512, "fwd"), (192, 256, 256, 512, "dgrad")]:
    B = 16
    g = torch.Generator(device="cpu").manual_seed(3)
    if kind == "fwd":
        x = K.Act(torch.relu(torch.randn(B, H, W, C, generator=g)).to(dev))
        wp = K.pack_weight((torch.randn(Cout, C, 3, 3, generator=g) * (2 / (9 * C)) ** 0.5).to(dev), torch.float32)
        out = K.Act(torch.empty(B, H, W, Cout, device=dev))
        fn = lambda: K.conv_fwd(x, wp, Cout, 3, 1, out)  # noqa: E731
        flops = 2.0 * B * H * W * 9 * C * Cout
    else:  # dgrad: dy has Cout channels, dx C
        dy = K.Act((torch.randn(B, H, W, Cout, generator=g) * 1e-3).to(dev))
        wp = K.pack_weight((torch.randn(Cout, C, 3, 3, generator=g) * (2 / (9 * C)) ** 0.5).to(dev), torch.float32)
        wfl = K.flip_weight(wp, Cout, C, 3)
        out = K.Act(torch.empty(B, H, W, C, device=dev))
        fn = lambda: K.conv_dgrad(dy, wp, C, 3, 1, out, wflip=wfl)  # noqa: E731
        flops = 2.0 * B * H * W * 9 * C * Cout
    ms, res = {v: [] for v in schs}, {}
    for _ in range(3):
        for v in schs:
            if v == "xs":  # the pre-split pixel operand (SCH 8)
                os.environ["DGVCC_PSPLIT_XS"] = "2"
                os.environ.pop("DGVCC_PSPLIT_SCH", None)
            else:
                os.environ["DGVCC_PSPLIT_XS"] = "0"
                os.environ["DGVCC_PSPLIT_SCH"] = v
            ms[v].append(timed(fn))
            res[v] = out.buf.clone()
    os.environ.pop("DGVCC_PSPLIT_SCH", None)
    os.environ.pop("DGVCC_PSPLIT_XS", None)
    line = f"{kind:5s} {B}x{H}x{W} {C}->{Cout}:"
    for v in schs:
        t = min(ms[v])
        line += f"  sch {v} {t:.3f} ms {flops / t / 1e9:.0f} TF/s" + ("" if v == schs[0] else f" ident {torch.equal(res[v], res[schs[0]])}")
    print(line, flush=True)
