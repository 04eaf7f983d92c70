"""Per-block-column k_step durations from a rocprofv3 kernel-trace CSV.

usage: python scripts/step_timeline.py <kernel_trace.csv> N
Prints, per J, the mean launch time and the algorithmic TF/s of the launch
(same flop formula as run_factor), and the gaps between consecutive launches. With concurrent
particle-group streams the launches of the groups overlap: the per-launch rate then counts one
group's share while the other group shares the GPU (see kernel_union.py for the whole phase)."""
import csv
import sys
from collections import defaultdict

f, N = sys.argv[1], int(sys.argv[2])
T = 128
nt = -(-N // T)
rows = [r for r in csv.DictReader(open(f)) if "k_step" in r["Kernel_Name"] or "k_diag" in r["Kernel_Name"]
        or "k_build_cov" in r["Kernel_Name"] or "k_points" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t3 = T ** 3


def flops(J):
    fl = 0.0
    for w in range(nt - 1):
        fl += (2 * t3 * J + 2 * t3) if w < nt - 1 - J else 2 * t3 * (J - (w - (nt - 1 - J)))
    return fl + (2 / 3 * t3 if J + 1 < nt else 0)


dur, gap = defaultdict(list), defaultdict(list)
P = None
k = 0
ngroups, builds, after_step = 1, 0, True
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"]
    if "k_build_cov" in name:  # the particle groups' K builds are adjacent: count them
        builds = 1 if after_step else builds + 1
        ngroups, k, after_step = builds, 0, False
    if "k_step" in name:
        after_step = True
        J = k // ngroups  # launches interleave the groups block column by block column
        P = ngroups * (int(r["Grid_Size_X"]) // (int(r["Workgroup_Size_X"]) * (nt - 1)))
        dur[J].append((e - s) * 1e-6)
        if prev_end is not None:
            gap[J].append((s - prev_end) * 1e-6)
        k += 1
    prev_end = e
tot_ms = tot_fl = 0.0
for j in sorted(dur):
    ms = sum(dur[j]) / len(dur[j])
    g = sum(gap[j]) / max(1, len(gap[j]))
    fl = flops(j) * P
    tot_ms += ms
    tot_fl += fl
    print(f"J={j:3d}  {ms:8.3f} ms  {fl / ms / 1e9:6.1f} TF/s  gap {g * 1e3:6.1f} us")
print(f"P={P} total {tot_ms:.2f} ms  {tot_fl / tot_ms / 1e9:.1f} TF/s")
