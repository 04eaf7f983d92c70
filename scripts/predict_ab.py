"""Same-box A/B of the single-particle prediction factorisation (the bench's predict line: N=4096,
d=3, M=10000): variants given as environment settings, interleaved over rounds in one process
(the library reads them per factorisation), profiled factor wall time and unprofiled call wall.
Usage: python scripts/predict_ab.py 'GPF_SPLIT_K_SLOTS=256' 'GPF_SPLIT_K_SLOTS=384' ..."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import gpfit  # noqa: E402

N, d, M = int(os.environ.get("N", 4096)), 3, 10000
variants = [dict(kv.split("=", 1) for kv in v.split(",") if kv) for v in (sys.argv[1:] or [""])]
rng = np.random.default_rng(1)
x = rng.uniform(size=(d, N))
y = np.sin(2 * np.pi * x).sum(0) + 0.1 * rng.standard_normal(N)
e = np.full(N, 0.1)
xf = np.random.default_rng(100).uniform(size=(d, M))
ls = np.full(d, 0.3)
ctx = gpfit.Context(0)
ctx.set_data(x, y, e)
res = {i: ([], []) for i in range(len(variants))}
ref = None


def apply(v):
    for vv in variants:
        for k in vv:
            os.environ.pop(k, None)
    os.environ.update(v)


for rnd in range(6):
    for i, v in enumerate(variants):
        apply(v)
        ctx.predict(ls, xf)  # warm
        ctx.synchronize()
        t0 = time.perf_counter()
        mu, sd = ctx.predict(ls, xf)
        ctx.synchronize()
        res[i][0].append((time.perf_counter() - t0) * 1e3)
        ctx.reset_profile()
        ctx.set_profiling(True)
        ctx.predict(ls, xf)
        ctx.synchronize()
        res[i][1].append(ctx.profile()["factor_wall_ms"])
        ctx.set_profiling(False)
        if ref is None:
            ref = (mu, sd)
        elif rnd == 0:
            dm = np.max(np.abs(mu - ref[0])) / np.max(np.abs(ref[0]))
            ds = np.max(np.abs(sd - ref[1])) / np.max(np.abs(ref[1]))
            print(f"variant {i} vs 0: max rel diff mu {dm:.2e} sd {ds:.2e}")
for i, v in enumerate(variants):
    w, f = res[i]
    print(f"{v or 'default'}: predict ms median {np.median(w):.3f} (min {min(w):.3f})  factor ms median {np.median(f):.3f} "
          f"(min {min(f):.3f})")
