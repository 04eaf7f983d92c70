"""Per-dispatch averages of rocprofv3 --pmc counters for one kernel: pmc_counters_k.py <kernel> <dir>..."""
import csv
import glob
import json
import sys
from collections import defaultdict

kern, dirs = sys.argv[1], sys.argv[2:]
tot, disp = defaultdict(float), defaultdict(set)
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kern in row.get("Kernel_Name", ""):
                tot[row["Counter_Name"]] += float(row["Counter_Value"])
                disp[row["Counter_Name"]].add(row.get("Dispatch_Id"))
print(json.dumps({k: tot[k] / max(1, len(disp[k])) for k in sorted(tot)}, indent=1))
