"""Join the PMC per-dispatch HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 corrections of
tools/pmc_summary.py) of the headline's conv forward/dgrad dispatches with bench.py's launch list
(DGVCC_BENCH_LAUNCHES: kind, scope, ms, GFLOP, algorithmic MB per launch, in launch order) and
print traffic / algorithmic per launch shape.  The timed step is the last one, so the last
len(list) fwd/dgrad dispatches of the pass are its launches.
usage: traffic_layers.py gpurun_out/tl [out.md]"""
import collections
import csv
import glob
import json
import sys

src = sys.argv[1]
FAM = ("conv_fwd_psplit_kernel", "conv_fwd_rsplit3w_kernel", "conv_fwd_rsplit_kernel", "conv_fwd_rsplit3_kernel",
       "conv_fwd_pers_kernel", "conv_fwd_kernel<float")


def per_dispatch(path):
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(glob.glob(f"{path}/**/*counter_collection.csv", recursive=True)[0])):
        if not any(f in r["Kernel_Name"] for f in FAM):
            continue
        k = int(r["Dispatch_Id"])
        if k not in rows:
            rows[k] = [r["Kernel_Name"].replace("void (anonymous namespace)::", "").split("(")[0], 0.0]
        rows[k][1] += float(r["Counter_Value"]) * 1024  # KB -> bytes
    return rows


fetch, write = per_dispatch(f"{src}/pmc_fetch"), per_dispatch(f"{src}/pmc_write")
launches = [l for l in json.load(open(glob.glob(f"{src}/launches_fp32.json")[0])) if l[0] in ("fwd", "dgrad")]
ids = sorted(fetch)[-len(launches):]
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, ""])
tot_m = tot_a = 0.0
for d, (kind, scope, ms, gf, mb) in zip(ids, launches):
    name, fb = fetch[d]
    wb = write.get(d, [name, 0.0])[1]
    meas = 2 * fb + wb
    key = (kind, round(gf, 1), round(mb, 1), name)
    a = agg[key]
    a[0] += 1; a[1] += meas; a[2] += mb * 1e6
    tot_m += meas; tot_a += mb * 1e6
out = ["| kind | GFLOP | algorithmic MB | kernel | n | HBM MB per launch | ratio |", "|---|---|---|---|---|---|---|"]
for (kind, gf, mb, name), (n, meas, alg, _) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    out.append(f"| {kind} | {gf} | {mb} | `{name}` | {n} | {meas / n / 1e6:.0f} | {meas / alg:.2f} |")
out.append(f"\nall fwd/dgrad launches of the step: {tot_m / 1e9:.2f} GB measured vs {tot_a / 1e9:.2f} GB algorithmic "
           f"= {tot_m / tot_a:.2f}x over {len(launches)} launches")
text = "\n".join(out)
print(text)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write("# Per-launch HBM traffic of the fp32 headline's conv fwd/dgrad (tools/traffic_layers.py)\n\n" + text + "\n")
