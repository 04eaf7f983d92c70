"""Summarise rocprofv3 PMC passes into HBM bytes per k_step launch.

Usage: python scripts/pmc_traffic.py <fetch_dir> <write_dir> <out.json> N d swarm
Each dir holds one `rocprofv3 --pmc ... --kernel-trace --output-format csv` pass
(FETCH_SIZE and WRITE_SIZE need separate passes on gfx950: TCC slots).
Per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reports 1/2 of the bytes of wide
coalesced streaming reads on gfx950, so it is doubled; WRITE_SIZE (KB) is exact
for 16-B-per-lane stores.
"""
import csv
import glob
import json
import sys


def counter_sum(d, name, kernel="k_step"):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    tot, disp = 0.0, set()
    for f in files:
        for row in csv.DictReader(open(f)):
            if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == name:
                tot += float(row["Counter_Value"])
                disp.add(row.get("Dispatch_Id"))
    return tot, len(disp)


def main():
    fdir, wdir, out, N, d, swarm = sys.argv[1:7]
    f, nf = counter_sum(fdir, "FETCH_SIZE")
    w, nw = counter_sum(wdir, "WRITE_SIZE")
    res = {"N": int(N), "d": int(d), "swarm": int(swarm), "kernel": "k_step",
           "launches_fetch_pass": nf, "launches_write_pass": nw,
           "fetch_kb_raw_per_launch": f / max(nf, 1), "write_kb_per_launch": w / max(nw, 1)}
    res["bytes_per_launch"] = (2.0 * res["fetch_kb_raw_per_launch"] + res["write_kb_per_launch"]) * 1024.0
    res["note"] = "FETCH_SIZE doubled (gfx950 reports half of wide streaming reads); KB -> bytes x1024"
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
