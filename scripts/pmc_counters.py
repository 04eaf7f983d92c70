"""Per-dispatch averages of every counter in rocprofv3 --pmc passes for one kernel.

usage: python scripts/pmc_counters.py <out.json> <note> <dir> [<dir> ...]
(KNAME: substring of the kernel name, default k_step)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out, note, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
tot, disp = defaultdict(float), defaultdict(set)
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if os.environ.get("KNAME", "k_step") in row.get("Kernel_Name", ""):
                tot[row["Counter_Name"]] += float(row["Counter_Value"])
                disp[row["Counter_Name"]].add(row.get("Dispatch_Id"))
res = {k: tot[k] / max(1, len(disp[k])) for k in sorted(tot)}
res["note"] = note
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
