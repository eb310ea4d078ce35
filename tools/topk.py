"""Print the top kernels of a rocprofv3 results database (kernel-trace --stats run)."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = 0.0
rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
for name, calls, dur, avg, pct in rows[:n]:
    print(f"{dur/1e3:9.2f} ms {calls:6d} x {avg:9.2f} us {pct:5.1f}%  {name[:110]}")
print("total ms", sum(r[2] for r in rows) / 1e3)
