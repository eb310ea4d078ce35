"""Per-launch-shape breakdown of a rocprofv3 results database: for kernels matching a
substring, average duration per (grid, workgroup) shape, in first-seen order."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 else ""
rows = c.execute("select name, grid_x, grid_y, grid_z, workgroup_x, duration, start from kernels "
                 "where name like ? order by start", (f"%{pat}%",))
agg = {}
for name, gx, gy, gz, wx, dur, _ in rows:
    k = (name[:60], gx, gy, gz, wx)
    a = agg.setdefault(k, [0, 0.0])
    a[0] += 1
    a[1] += dur
for (name, gx, gy, gz, wx), (n, tot) in agg.items():
    print(f"{n:5d} x {tot / n / 1e3:8.2f} us  grid=({gx},{gy},{gz}) wg={wx}  {name}")
