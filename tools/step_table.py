"""Per-kernel table of ONE training step from a tools/r2_trunk.sh directory: durations from the
rocprofv3 kernel trace (last step: the dispatches after the second-to-last adamw_kernel),
HBM bytes from the FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE x2, the gfx950 wide-read
correction of MI355X_MICROARCH.md; KB -> bytes) and MFMA-busy from the
SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE pass (busy / (1024 SIMDs x GUI/8)), each taken
from that pass's own last step.  Kernels are grouped by the reference op they implement.

usage: python tools/step_table.py gpurun_out/r2t/ibn profiles/round2/trunk_ibn [title]
  writes <dst>.json and <dst>.md"""
import csv
import json
import re
import sys
from collections import defaultdict

GROUPS = [  # (group, regex on the short kernel name), first match wins
    ("conv fwd/dgrad (LDS-DMA pipeline)", r"conv_fwd_(pers|pipe|tap3|psplit|rsplit)|split_x_h"),
    ("split-weight prep", r"split_weight"),
    ("operand max (f16 x3 scales)", r"amax_kernel"),
    ("conv wgrad", r"conv_wgrad|wgrad_reduce|splitk_reduce"),
    ("conv strided/general", r"conv_gen|im2col"),
    ("conv (register-staged)", r"conv_fwd_kernel"),
    ("SwitchWhiten2d", r"^sw_"),
    ("ISW (cov/loss/mask)", r"^iw_|topk|cov"),
    ("InstanceNorm", r"^in_"),
    ("BatchNorm (+ReLU/pool)", r"^bn_|colsum"),
    ("residual join / ReLU bwd", r"bn_add|relu_bwd|join"),
    ("maxpool / resample", r"maxpool|upsample|cat_combine"),
    ("heads / losses / AdamW", r"head|mse|bce|adamw|gather_flat|reduce|grad_unscale"),
    ("pack / copies", r"pack|copy|fill|elementwise|vectorized|Memset|memset"),
]


def short(name):
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)(\w+)", name)
    if m:  # mangled template instance: base name + the mangled template arguments
        n = int(m.group(1))
        base, rest = m.group(2)[:n], m.group(2)[n:]
        return f"{base}<{rest[1:].split('EEv')[0]}>" if rest.startswith("I") else base
    k = name.replace("void ", "").replace("(anonymous namespace)::", "")
    k = re.sub(r"\(.*", "", k)
    return k[:100]


def group(k):
    base = k.split("<")[0]
    for g, rx in GROUPS:
        if re.search(rx, base):
            return g
    return "other"


def last_step(rows):
    """Dispatches of the last training step: after the second-to-last run of AdamW launches
    (one step may launch several, one per run of equal step counts), and before the dmap
    roofline's launches that bench.py makes after the timed legs."""
    ids = sorted(rows)
    ad = [i for i in ids if "adamw_kernel" in rows[i]["name"]]
    runs = []
    for j, i in enumerate(ad):
        if j == 0 or ids.index(i) - ids.index(ad[j - 1]) > 20:
            runs.append([i])
        else:
            runs[-1].append(i)
    if len(runs) < 2:
        return ids
    return [i for i in ids if runs[-2][-1] < i <= runs[-1][-1]]


def load_pmc(path):
    rows = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = rows[int(r["Dispatch_Id"])]
        d["name"] = r["Kernel_Name"]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return {i: rows[i] for i in last_step(rows)}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    title = sys.argv[3] if len(sys.argv) > 3 else src
    tr = {}
    for r in csv.DictReader(open(f"{src}/trace/run_kernel_trace.csv")):
        tr[int(r["Dispatch_Id"])] = {"name": r["Kernel_Name"],
                                     "t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9}
    tr = {i: tr[i] for i in last_step(tr)}
    per = defaultdict(lambda: {"n": 0, "t": 0.0, "bytes": 0.0, "busy": 0.0, "gui": 0.0, "npmc": 0})
    for d in tr.values():
        a = per[short(d["name"])]
        a["n"] += 1
        a["t"] += d["t"]
    fe, wr = load_pmc(f"{src}/pmc_fetch/run_counter_collection.csv"), load_pmc(f"{src}/pmc_write/run_counter_collection.csv")
    mf = load_pmc(f"{src}/pmc_mfma/run_counter_collection.csv")
    for d in fe.values():
        per[short(d["name"])]["bytes"] += 2 * 1024 * d.get("FETCH_SIZE", 0.0)
    for d in wr.values():
        per[short(d["name"])]["bytes"] += 1024 * d.get("WRITE_SIZE", 0.0)
    for d in mf.values():
        a = per[short(d["name"])]
        a["busy"] += d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        a["gui"] += d.get("GRBM_GUI_ACTIVE", 0.0)
    tot_t = sum(a["t"] for a in per.values())
    kern, groups = {}, defaultdict(lambda: {"ms": 0.0, "bytes": 0.0, "busy": 0.0, "gui": 0.0, "n": 0})
    for k, a in per.items():
        if a["n"] == 0:
            continue
        mfma = a["busy"] / (1024 * a["gui"] / 8) if a["gui"] else None
        kern[k] = {"group": group(k), "dispatches": a["n"], "ms": round(a["t"] * 1e3, 4),
                   "hbm_gb": round(a["bytes"] / 1e9, 4),
                   "hbm_gbps": round(a["bytes"] / a["t"] / 1e9, 1) if a["t"] else None,
                   "mfma_busy": round(mfma, 4) if mfma is not None else None}
        g = groups[group(k)]
        g["ms"] += a["t"] * 1e3; g["bytes"] += a["bytes"]; g["busy"] += a["busy"]; g["gui"] += a["gui"]; g["n"] += a["n"]
    gout = {g: {"dispatches": v["n"], "ms": round(v["ms"], 3), "share": round(v["ms"] / (tot_t * 1e3), 4),
                "hbm_gb": round(v["bytes"] / 1e9, 3),
                "hbm_gbps": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] else None,
                "mfma_busy": round(v["busy"] / (1024 * v["gui"] / 8), 4) if v["gui"] else None}
            for g, v in sorted(groups.items(), key=lambda kv: -kv[1]["ms"])}
    allbusy = sum(v["busy"] for v in groups.values())
    allgui = sum(v["gui"] for v in groups.values())
    out = {"title": title, "step_kernel_ms": round(tot_t * 1e3, 3),
           "step_mfma_busy": round(allbusy / (1024 * allgui / 8), 4) if allgui else None,
           "groups": gout, "kernels": dict(sorted(kern.items(), key=lambda kv: -kv[1]["ms"]))}
    json.dump(out, open(dst + ".json", "w"), indent=1)
    lines = [f"# {title}", "", f"One step: {out['step_kernel_ms']} ms of kernels, MFMA-busy "
             f"{out['step_mfma_busy']:.1%}" if out["step_mfma_busy"] is not None else "", "",
             "| group | dispatches | ms | share | HBM GB | GB/s | MFMA-busy |", "|---|---|---|---|---|---|---|"]
    for g, v in gout.items():
        mb = f"{v['mfma_busy']:.1%}" if v["mfma_busy"] is not None else "-"
        lines.append(f"| {g} | {v['dispatches']} | {v['ms']:.3f} | {v['share']:.1%} | {v['hbm_gb']:.3f} | {v['hbm_gbps']} | {mb} |")
    lines += ["", "| kernel | group | n | ms | HBM GB | GB/s | MFMA-busy |", "|---|---|---|---|---|---|---|"]
    for k, v in list(out["kernels"].items())[:40]:
        mb = f"{v['mfma_busy']:.1%}" if v["mfma_busy"] is not None else "-"
        lines.append(f"| `{k}` | {v['group']} | {v['dispatches']} | {v['ms']:.3f} | {v['hbm_gb']:.3f} | {v['hbm_gbps']} | {mb} |")
    open(dst + ".md", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:20 + len(gout)]))


if __name__ == "__main__":
    main()
