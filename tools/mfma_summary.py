"""Summarise a rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE pass (tools/prof_mfma.sh).

Per kernel: MFMA-busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GUI cycles), where
GUI cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs), and the effective clock
GRBM_GUI_ACTIVE / 8 / dispatch wall time (MI355X_MICROARCH.md, DVFS give-back).  Only the
last bench step's dispatches are used (after the last adamw_kernel of the warm-up step).
usage: python tools/mfma_summary.py gpurun_out/<tag>/pmc_mfma/run_counter_collection.csv profiles/<tag>/mfma_summary.json"""
import csv
import json
import re
import sys
from collections import defaultdict

rows = defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    d = rows[int(r["Dispatch_Id"])]
    d["name"] = r["Kernel_Name"]
    d["t"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    d[r["Counter_Name"]] = float(r["Counter_Value"])
ids = sorted(rows)
ad = [i for i in ids if "adamw_kernel" in rows[i]["name"]]
ids = [i for i in ids if i > ad[-2]] if len(ad) >= 2 else ids
SIMDS = 1024
agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for i in ids:
    d = rows[i]
    k = re.sub(r"\(\(anonymous namespace\)::\w+\)", "", d["name"]).replace("void (anonymous namespace)::", "")
    k = re.sub(r"\(.*", "", k)[:90]
    a = agg[k]
    a[0] += 1; a[1] += d["t"]; a[2] += d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0); a[3] += d.get("GRBM_GUI_ACTIVE", 0.0)
out = {}
tot_t = sum(a[1] for a in agg.values())
tot_busy = sum(a[2] for a in agg.values())
tot_gui = sum(a[3] for a in agg.values())
for k, (n, t, busy, gui) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    cyc = gui / 8
    out[k] = {"dispatches": n, "ms": round(t * 1e3, 3),
              "mfma_busy_frac": round(busy / (SIMDS * cyc), 4) if cyc else None,
              "clock_ghz": round(cyc / t / 1e9, 3) if t else None}
summary = {"note": __doc__.splitlines()[2].strip() + " ...",
           "step_kernel_ms": round(tot_t * 1e3, 3),
           "step_mfma_busy_frac": round(tot_busy / (SIMDS * tot_gui / 8), 4),
           "step_clock_ghz": round(tot_gui / 8 / tot_t / 1e9, 3),
           "kernels": out}
json.dump(summary, open(sys.argv[2], "w"), indent=1)
print(f"step: {summary['step_kernel_ms']} ms of kernels, MFMA busy {summary['step_mfma_busy_frac']:.1%}, "
      f"clock {summary['step_clock_ghz']} GHz")
for k, v in list(out.items())[:14]:
    print(f"{v['ms']:8.3f} ms  n={v['dispatches']:3d}  mfma {v['mfma_busy_frac'] or 0:6.1%}  {v['clock_ghz']} GHz  {k}")
