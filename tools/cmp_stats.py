"""Compare per-kernel average durations of two rocprofv3 kernel_stats csv files."""
import csv, re, sys
def load(p):
    return {re.sub(r'\(\(anonymous namespace\)::\w+\)', '', r['Name'])[:72]: (float(r['AverageNs']), int(r['Calls']), float(r['TotalDurationNs']))
            for r in csv.DictReader(open(p))}
a, b = load(sys.argv[1]), load(sys.argv[2])
for k in sorted(a, key=lambda k: -a[k][2])[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    if k in b:
        print(f"{a[k][0]/1e3:9.1f} -> {b[k][0]/1e3:9.1f} us  ({b[k][0]/a[k][0]-1:+6.1%})  {k}")
