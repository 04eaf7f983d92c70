"""GP prediction at N=4096 d=3, M=10000 query points (the bench's predict line), repeated: for
rocprofv3 kernel traces of the single-particle factorisation (launch_list.py)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import gpfit  # noqa: E402

N, d = int(os.environ.get("N", 4096)), 3
rng = np.random.default_rng(1)
x = rng.uniform(size=(d, N))
y = np.sin(2 * np.pi * x).sum(0) + 0.1 * rng.standard_normal(N)
e = np.full(N, 0.1)
ctx = gpfit.Context(0)
ctx.set_data(x, y, e)
xf = np.random.default_rng(100).uniform(size=(d, 10000))
for _ in range(3):
    ctx.predict(np.full(d, 0.3), xf)
ctx.synchronize()
ctx.close()
print("done")
