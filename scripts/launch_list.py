"""Kernel launches of a rocprofv3 kernel-trace CSV in time order: name, grid, duration, gap.

usage: python scripts/launch_list.py <kernel_trace.csv> [last_n]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows = rows[-n:]
prev = None
tot = 0.0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    tot += (e - s) / 1e3
    print(f"{name:28s} wg {grid:6d}  {(e - s) / 1e3:9.1f} us  gap {gap:7.1f} us")
    prev = e
print(f"sum of kernel time {tot:.1f} us over {len(rows)} launches")
