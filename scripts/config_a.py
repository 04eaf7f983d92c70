"""Config A: the reference's own workload — len_scale_opt on the bundled
Test files (N = 21, 15, 8, 13; d = 2; 40 particles; 500 iterations) through the drop-in, on the GPU.
Prints per-experiment wall time, evaluations, evals/s, and the per-batch latency."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import torch  # noqa: F401,E402
import find_len_scales as fls  # noqa: E402
import read_in  # noqa: E402
from gpfit import default_context  # noqa: E402

os.chdir(os.path.join(ROOT, "tests", "golden", "inputs"))
files = ["Test_file1.txt"] + sorted(os.path.join("Test_folder", f) for f in os.listdir("Test_folder"))
ctx = default_context()
# cold start (module load, first buffers, graph capture) reported apart from the timed runs
xs, pairs, _ = read_in.read_data(files[0], None, [0.01, 0.01])
t0 = time.perf_counter()
fls.len_scale_opt(xs[0], pairs[0][0], pairs[0][1], False, seed=1)
print(f"cold start ({files[0]}, untimed below): {time.perf_counter() - t0:.3f} s", flush=True)
tot_e = tot_t = 0.0
for fp in files:
    xs, pairs, _ = read_in.read_data(fp, None, [0.01, 0.01])
    for x, (y, e) in zip(xs, pairs):
        ctx.reset_profile()
        t0 = time.perf_counter()
        fls.len_scale_opt(x, y, e, False, seed=1)
        dt = time.perf_counter() - t0
        n = ctx.profile()["evals"]
        tot_e += n
        tot_t += dt
        print(f"{fp} N={x.shape[1]}: {dt:.3f} s, {n:.0f} GPU evals, {n / dt:.0f} evals/s", flush=True)
print(f"total {tot_t:.3f} s, {tot_e:.0f} GPU evals, {tot_e / tot_t:.0f} evals/s")

if "--cpu" in sys.argv:  # the reference path on the host: oracle restatement, serial map (1 core)
    from oracle import ref_cpu
    tot = 0.0
    for fp in files:
        xs, pairs, _ = read_in.read_data(fp, None, [0.01, 0.01])
        for x, (y, e) in zip(xs, pairs):
            np.random.seed(1)
            t0 = time.perf_counter()
            ref_cpu.len_scale_opt(np.ascontiguousarray(x), y, e, False, verbose=False)
            dt = time.perf_counter() - t0
            tot += dt
            print(f"CPU {fp} N={x.shape[1]}: {dt:.3f} s", flush=True)
    print(f"CPU total {tot:.3f} s")
