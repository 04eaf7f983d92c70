"""Summarise rocprofv3 PMC passes for the secondary kernels (k_prob_surf, k_cross_cov, k_predict_vsq):
per-dispatch averages of every collected counter, plus the kernel-trace duration of the same
dispatches. Usage: python scripts/pmc_secondary.py <out.json> <pass_dir> [<pass_dir> ...]"""
import csv
import glob
import json
import sys

KERNELS = ("k_prob_surf", "k_cross_cov", "k_predict_vsq")
out, dirs = sys.argv[1], sys.argv[2:]
res = {k: {"counters": {}, "dispatches": 0, "avg_ns": None} for k in KERNELS}
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = {}
        for row in csv.DictReader(open(f)):
            name = next((k for k in KERNELS if k in row.get("Kernel_Name", "")), None)
            if name is None:
                continue
            key = (name, row["Counter_Name"])
            disp = per.setdefault(key, {})
            disp[row["Dispatch_Id"]] = disp.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
        for (name, cn), disp in per.items():
            res[name]["counters"][cn] = sum(disp.values()) / len(disp)
            res[name]["dispatches"] = max(res[name]["dispatches"], len(disp))
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        dur = {k: [] for k in KERNELS}
        for row in csv.DictReader(open(f)):
            name = next((k for k in KERNELS if k in row.get("Kernel_Name", "")), None)
            if name:
                dur[name].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
        for k, v in dur.items():
            if v and res[k]["avg_ns"] is None:
                res[k]["avg_ns"] = sum(v) / len(v)
ps = res["k_prob_surf"]
c = ps["counters"]
if "SQ_INSTS_VALU_FLOPS_FP64" in c and ps["avg_ns"]:
    fl = c["SQ_INSTS_VALU_FLOPS_FP64"] + c.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0.0)
    ps["fp64_flops_per_dispatch"] = fl
    ps["fp64_tflops"] = fl / (ps["avg_ns"] * 1e-9) / 1e12
if "SQ_ACTIVE_INST_VALU" in c and "GRBM_GUI_ACTIVE" in c:
    # SQ counters are summed over the 8 XCDs' SEs; GRBM_GUI_ACTIVE over the 8 XCDs (quad-cycles /
    # cycles: see MI355X_MICROARCH.md "s_memtime tick vs SQ PMC units"); VALUBusy as in rocprof's
    # derived counter: 100 * SQ_ACTIVE_INST_VALU * 4 / CU_NUM / GRBM_GUI_ACTIVE (per XCD)
    ps["valu_busy_pct"] = 100.0 * c["SQ_ACTIVE_INST_VALU"] * 4 / 256 / (c["GRBM_GUI_ACTIVE"] / 8)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1)[:2500])
