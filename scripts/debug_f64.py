"""Locate the first wrong column of the diagonal factor (GPU debug aid)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import torch  # noqa: F401,E402
import gpfit  # noqa: E402
from oracle import ref_cpu  # noqa: E402

ctx = gpfit.Context(0)
for N in (64, 128, 200):
    rng = np.random.default_rng(N)
    x = rng.uniform(size=(2, N))
    y = np.sin(3 * x[0]) + x[1]
    e = rng.uniform(0.05, 0.2, N)
    ctx.set_data(x, y, e)
    ls = np.array([0.3, 0.3])
    L, U, z, al = ctx.debug_factor(ls)
    npad = L.shape[0]
    K = np.eye(npad)
    K[:N, :N] = ref_cpu.kernel_func(x, x, ls) + np.diag(e ** 2)
    Lr = np.linalg.cholesky(K)
    Ur = np.linalg.inv(Lr)
    dl = np.abs(np.tril(L) - Lr)
    du = np.abs(np.tril(U) - Ur)
    badc = [c for c in range(npad) if not (dl[:, c].max() < 1e-8)]
    badu = [c for c in range(npad) if not (du[:, c].max() < 1e-6)]
    print(f"N={N}: first bad L col {badc[:6]} first bad U col {badu[:6]} upper-L max {np.abs(np.triu(L, 1)).max():.2e}")
    if badc:
        c = badc[0]
        print("   L[c:c+6, c] gpu", L[c:c + 6, c], "\n   ref", Lr[c:c + 6, c])
    if N == 64:
        np.set_printoptions(precision=3, linewidth=160)
        print("   U gpu [0:8,0:6]\n", U[0:8, 0:6], "\n   U ref\n", Ur[0:8, 0:6])
        bad_rows = [r for r in range(64) if not (du[r, :64].max() < 1e-6)]
        print("   bad U rows", bad_rows[:20])
    sys.stdout.flush()
ctx.close()
