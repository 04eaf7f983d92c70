"""Per-launch spans of the last factorisation in a rocprofv3 kernel trace (k_step / k_diag /
k_build_cov), in start order: start offset, duration and gap to the previous launch on the same
queue. With one particle group (GPF_GROUPS=1) the launches are serial and the spans add up to the
factorisation's time.

usage: python scripts/launch_spans.py <kernel_trace.csv>"""
import csv
import sys

rows = sorted(([int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "?")]
               for r in csv.DictReader(open(sys.argv[1]))
               if any(n in r["Kernel_Name"] for n in ("k_build_cov", "k_diag", "k_step"))), key=lambda r: r[0])
starts = [i for i, r in enumerate(rows) if "k_build_cov" in r[2] and (i == 0 or "k_build_cov" not in rows[i - 1][2])]
sel = rows[starts[-1]:]
t0 = sel[0][0]
last = {}
tot = {}
for s, e, n, q in sel:
    kind = "build" if "k_build_cov" in n else "diag" if "k_diag" in n else "step"
    gap = (s - last[q]) / 1e3 if q in last else 0.0
    last[q] = e
    tot[kind] = tot.get(kind, 0) + (e - s)
    print(f"q{q} {kind:5s} start {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us  gap {gap:6.1f} us")
print("span", (sel[-1][1] - t0) / 1e3, "us;", {k: round(v / 1e3, 1) for k, v in tot.items()})
