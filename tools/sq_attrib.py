"""Per-kernel SQ counter table from tools/prof_sq_headline.sh passes (p1..p4 run_counter_collection.csv):
per dispatch averages, the wave-state split of SQ_WAVE_CYCLES (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY,
disjoint per MI355X_MICROARCH.md), the issue mix (ACTIVE_INST_* / WAVE_CYCLES), MFMA-busy against
1024 SIMDs x GRBM_GUI_ACTIVE / 8 and the clock.  SQ wave/issue counters are in quad-cycles.
usage: python tools/sq_attrib.py gpurun_out/<tag>/sq [out.json]"""
import collections
import csv
import glob
import json
import re
import sys

src = sys.argv[1]
rows = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{src}/p*/run_counter_collection.csv")):
    seen = set()
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(\(anonymous namespace\)::\w+.*", "", r["Kernel_Name"]).replace("void (anonymous namespace)::", "")
        rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if (f, r["Dispatch_Id"]) not in seen:
            seen.add((f, r["Dispatch_Id"]))
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
out = {}
for k, c in rows.items():
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    wc = avg.get("SQ_WAVE_CYCLES")
    if not wc:
        continue
    t = sum(dur[k]) / len(dur[k])
    gui = avg.get("GRBM_GUI_ACTIVE", 0) / 8
    d = {"dispatches": len(c["SQ_WAVE_CYCLES"]), "us": round(t * 1e6, 1),
         "clock_ghz": round(gui / t / 1e9, 3) if t and gui else None,
         "mfma_busy": round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * gui), 4) if gui else None,
         "wave_state": {"wait_any (waitcnt/barrier)": round(avg["SQ_WAIT_ANY"] / wc, 4),
                        "wait_inst_any (issue stall)": round(avg["SQ_WAIT_INST_ANY"] / wc, 4),
                        "active_inst_any (issuing)": round(avg["SQ_ACTIVE_INST_ANY"] / wc, 4)},
         "issue_mix": {n.replace("SQ_ACTIVE_INST_", "").lower(): round(avg[n] / wc, 4)
                       for n in avg if n.startswith("SQ_ACTIVE_INST_") and n != "SQ_ACTIVE_INST_ANY"},
         "wait_inst_lds": round(avg.get("SQ_WAIT_INST_LDS", 0) / wc, 4),
         "per_wave_instructions": {n.replace("SQ_INSTS_", "").lower(): round(avg[n] / avg["SQ_WAVES"], 1)
                                   for n in avg if n.startswith("SQ_INSTS_")} if avg.get("SQ_WAVES") else {},
         "vmem_fifo_full_frac": {n.lower(): round(avg[n] / wc, 4) for n in avg if "FIFO_FULL" in n},
         "lds_bank_conflict_cycles": avg.get("SQ_LDS_BANK_CONFLICT"),
         "mfma_coexec_frac": round(avg.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0) / (1024 * gui), 4) if gui else None}
    out[k] = d
for k, d in sorted(out.items(), key=lambda kv: -kv[1]["us"] * kv[1]["dispatches"]):
    print(k, json.dumps(d))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
