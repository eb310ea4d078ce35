"""Summarise rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, KB per dispatch) per kernel.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per 128-B
request of wide coalesced reads, i.e. reports half the bytes -> x2.  WRITE_SIZE
is exact for 16-B-per-lane stores.  Writes profiles/<tag>/pmc_summary.json and
profiles/conv_traffic.json (read by bench.py for roofline.traffic)."""
import csv
import json
import os
import sys
from collections import defaultdict

src = sys.argv[1]          # gpurun_out/<tag>
dst = sys.argv[2]          # profiles/<tag>
os.makedirs(dst, exist_ok=True)


def load(path):
    acc = defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        acc[k][0] += float(r["Counter_Value"])
        acc[k][1] += 1
    return acc


fetch = load(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
write = load(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
out = {}
for k in sorted(set(fetch) | set(write), key=lambda k: -fetch.get(k, [0, 1])[0]):
    f, nf = fetch.get(k, [0.0, 0])
    w, nw = write.get(k, [0.0, 0])
    n = max(nf, nw, 1)
    out[k] = {"dispatches": n, "fetch_bytes_per_dispatch_corrected": 2 * f * 1024 / max(nf, 1),
              "write_bytes_per_dispatch": w * 1024 / max(nw, 1)}
json.dump(out, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
# the launches bench.py's roofline times (kinds fwd + dgrad): every forward-GEMM kernel variant
FWD_KERNELS = ("conv_fwd_pers_kernel", "conv_fwd_pipe_kernel", "conv_fwd_tap3_kernel", "conv_fwd_tap3p_kernel", "conv_fwd_kernel")
conv = [v for k, v in out.items() if any(f in k for f in FWD_KERNELS)]
if conv:
    n = sum(v["dispatches"] for v in conv)
    tot = sum((v["fetch_bytes_per_dispatch_corrected"] + v["write_bytes_per_dispatch"]) * v["dispatches"] for v in conv)
    json.dump({"kernel": "implicit-GEMM conv forward/dgrad (conv_fwd_pers_kernel, conv_fwd_pipe_kernel, conv_fwd_tap3_kernel, conv_fwd_tap3p_kernel)",
               "dispatches": n,
               "hbm_bytes_per_launch": tot / n,
               "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KB->bytes, averaged over dispatches of a 2-step bench run"},
              open(os.path.join(os.path.dirname(dst), "conv_traffic.json"), "w"), indent=1)
for k, v in list(out.items())[:12]:
    print(f"{v['fetch_bytes_per_dispatch_corrected']/1e6:10.2f} MB rd {v['write_bytes_per_dispatch']/1e6:10.2f} MB wr  n={v['dispatches']:4d} {k[:80]}")
