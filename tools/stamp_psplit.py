"""Phase shares of the f16 x3 256-pixel pre-split forward (conv_fwd_psplit_kernel<256,..,TALL,HM>) from its
diagnostic stamp build (DGVCC_PSPLIT_STAMP + dg_debug_stamps): per K-step cycles in the DMA wait, the
barrier, the prologue (fragment reads, next DMA issue, B split), the MFMA block, and the epilogue per tile,
averaged over blocks for waves 0-3 and 4-7 (SIMD partners), for each schedule DGVCC_PSPLIT_SCH in
STAMP_SCHS (default 0,1,2), beside the real kernel's time per launch (same process, interleaved).
The stamp build's run time is not quoted (its fences forbid overlaps): read the shares.
usage: python tools/stamp_psplit.py [out.json]"""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dgvcc_amd import kernels as K

dev = "cuda"
B = 16
shapes = [(192, 256, 256, 256), (96, 128, 512, 512), (192, 256, 128, 256)]
SCHS = [int(v) for v in os.environ.get("STAMP_SCHS", "0,1,2").split(",")]
NAMES = ["dma_wait", "barrier", "prologue_reads_issue_split", "mfma_block"]
res = {}
buf = torch.zeros(256 * 8 * 8, dtype=torch.int64, device=dev)
K.call("dg_set_f32_math", 2)


def time_ms(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for (H, W, C, Cout) in shapes:
    g = torch.Generator(device="cpu").manual_seed(1)
    x = K.Act(torch.relu(torch.randn(B, H, W, C, generator=g)).to(dev))
    y = K.Act(torch.empty(B, H, W, Cout, device=dev))
    wp = K.pack_weight((torch.randn(Cout, C, 3, 3, generator=g) * (2.0 / (9 * C)) ** 0.5).to(dev), torch.float32)
    ref = None
    times = {sch: [] for sch in SCHS}
    for rnd in range(3):  # interleaved rounds of the real kernels
        for sch in SCHS:
            os.environ["DGVCC_PSPLIT_SCH"] = str(sch)
            times[sch].append(time_ms(lambda: K.conv_fwd(x, wp, Cout, 3, 1, y)))
            if ref is None:
                ref = y.buf.clone()
            elif not torch.equal(ref, y.buf):
                raise SystemExit(f"schedule {sch} changed the output")
    for sch in SCHS:
        os.environ["DGVCC_PSPLIT_SCH"] = str(sch)
        buf.zero_()
        K.call("dg_debug_stamps", K.ptr(buf), buf.numel() * 8)
        os.environ["DGVCC_PSPLIT_STAMP"] = "1"
        K.conv_fwd(x, wp, Cout, 3, 1, y)
        torch.cuda.synchronize()
        del os.environ["DGVCC_PSPLIT_STAMP"]
        K.call("dg_debug_stamps", None, 0)
        rows = buf.view(-1, 8, 8).cpu().double()
        rows = rows[rows[:, 0, 5] > 0]
        if rows.shape[0] == 0:
            print(f"{H}x{W} {C}->{Cout} sch {sch}: no stamp rows")
            continue
        out = {"shape": f"B{B} {H}x{W} {C}->{Cout}", "sch": sch,
               "ms_per_launch_real_kernel": sorted(times[sch])[1], "blocks": int(rows.shape[0])}
        for half, sl in (("waves0-3", slice(0, 4)), ("waves4-7", slice(4, 8))):
            r = rows[:, sl]
            nk = r[..., 5].sum()
            per = {n: round(float(r[..., i].sum() / nk), 1) for i, n in enumerate(NAMES)}
            tot = sum(per[n] for n in NAMES)
            per["kstep_total"] = round(tot, 1)
            per["epilogue_per_tile"] = round(float(r[..., 4].sum() / r[..., 6].sum()), 1)
            per["shares"] = {n: round(per[n] / tot, 4) for n in NAMES}
            out[half] = per
        out["kstep_mfma_cycles_ideal_per_simd"] = 2 * 96 * 16  # two waves x 96 16x16x32 MFMAs x 16 cycles
        res[f"{out['shape']} sch{sch}"] = out
        print(json.dumps(out), flush=True)
os.environ.pop("DGVCC_PSPLIT_SCH", None)
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
