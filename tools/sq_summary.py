"""Per-kernel SQ counter summary of a rocprofv3 --pmc csv (fractions of SQ_WAVE_CYCLES)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:90]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) == 0:
        continue
    n = cnt[(k, "SQ_WAVE_CYCLES")]
    wc = d["SQ_WAVE_CYCLES"]
    print(k, "dispatches", n)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v / n:14.4g}  {v / wc if wc else 0:6.3f} of wave-cycles")
