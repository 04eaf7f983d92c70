#!/bin/bash
# Clock and MFMA-busy of k_step per library variant (VARIANTS): one PMC pass each.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-clk}; mkdir -p $O
for v in $VARIANTS; do
  GPFIT_LIB=$PWD/gaussian-process_amd/libgpfit_$v.so timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace -d $PWD/$O/$v -o c --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu --pso-steps 0 --no-profile --predict-points 0 --no-hull --psurf-rows 0 > $O/$v.log 2>&1 || exit $?
  python - "$O/$v" "$v" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "k_step" in r["Kernel_Name"]]
acc = collections.defaultdict(float); n = collections.Counter(); dur = {}
for r in rows:
    k = (r["Dispatch_Id"], r["Counter_Name"])
    acc[r["Counter_Name"]] += float(r["Counter_Value"])
    n[r["Counter_Name"]] += 1
    dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
nd = len(dur); T = sum(dur.values()) / nd
g = acc["GRBM_GUI_ACTIVE"] / nd
print(sys.argv[2], "dispatches", nd, "avg ns", round(T), "GRBM/dispatch", round(g), "clock GHz (GRBM/8/T)", round(g / 8 / T, 3),
      "mfma busy frac", round(acc["SQ_VALU_MFMA_BUSY_CYCLES"] / nd / (g / 8 * 1024), 3))
PY
done
