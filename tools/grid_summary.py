"""Per (kernel, grid) launch counts and mean durations from a rocprofv3 kernel trace, per step.
usage: grid_summary.py TRACE_DIR STEPS [filter]"""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
steps = int(sys.argv[2])
flt = sys.argv[3] if len(sys.argv) > 3 else ""
rows = list(csv.DictReader(open(f)))
c = collections.defaultdict(list)
for r in rows:
    if flt not in r["Kernel_Name"]:
        continue
    blocks = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    c[(r["Kernel_Name"][:90], blocks, int(r["Workgroup_Size_X"]))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
tot = sum(sum(v) for v in c.values()) / steps
print(f"{tot / 1000:.2f} ms per step over the selected kernels")
for k, v in sorted(c.items(), key=lambda kv: -sum(kv[1]))[:40]:
    print(f"{sum(v) / steps / 1000:7.3f} ms/step  n/step {len(v) / steps:5.1f}  mean {sum(v) / len(v):8.1f} us  blocks {k[1]:6d}x{k[2]:4d}  {k[0]}")
