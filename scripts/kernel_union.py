"""Non-overlapping kernel time of the factorisation from a rocprofv3 kernel trace.

With concurrent particle-group streams the k_step launches of two groups overlap, so a per-launch
average duration does not measure one launch; the union of the factorisation kernels' busy
intervals (k_build_cov, k_diag, k_step) does. Prints, for the last `batches` factorisations of the
trace: the union time, the summed k_step launch time, and the algorithmic TFLOP/s on the union
(2/3 N^3 per particle, the formulation bench.py rates).

usage: python scripts/kernel_union.py <kernel_trace.csv> N particles_per_batch batches"""
import csv
import sys

f, N, P, nb = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
names = ("k_build_cov", "k_diag", "k_step")
rows = sorted(([int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]]
               for r in csv.DictReader(open(f)) if any(n in r["Kernel_Name"] for n in names)), key=lambda r: r[0])
T = 128
nt = -(-N // T)
# factorisations: a K build that follows a k_step starts a new one (the groups' builds are adjacent)
starts, prev_step = [], True
for i, r in enumerate(rows):
    if "k_build_cov" in r[2] and prev_step:
        starts.append(i)
    prev_step = "k_step" in r[2] if ("k_step" in r[2] or "k_build_cov" in r[2]) else prev_step
sel = rows[starts[-nb]:] if len(starts) >= nb else rows
ngroups = sum(1 for r in sel if "k_build_cov" in r[2]) // nb
union, cur_s, cur_e, step_sum = 0, None, None, 0
for s, e, n in sel:
    if "k_step" in n:
        step_sum += e - s
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
span = sel[-1][1] - sel[0][0]
flops = 2.0 / 3.0 * (nt * T) ** 3 * P * nb
print(f"{nb} factorisations of {P} particles (N={N}, {ngroups} group stream(s)): span {span / 1e6:.3f} ms, "
      f"union of kernel intervals {union / 1e6:.3f} ms, summed k_step launch time {step_sum / 1e6:.3f} ms; "
      f"{flops / (union * 1e-9) / 1e12:.1f} TFLOP/s on the union, {flops / (span * 1e-9) / 1e12:.1f} on the span")
