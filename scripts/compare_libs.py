"""Bitwise A/B of two libgpfit builds on the same inputs (GPU).

usage: python scripts/compare_libs.py dump <lib.so> <out.npz>
       python scripts/compare_libs.py diff <a.npz> <b.npz>
dump: factor (L, U, z, alpha) and eval_batch (loss, mu, sd) for several N."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [(100, 2, 8), (128, 3, 8), (300, 2, 16), (1024, 2, 16), (2100, 3, 8)]

if sys.argv[1] == "dump":
    os.environ["GPFIT_LIB"] = os.path.abspath(sys.argv[2])
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
    import torch  # noqa: F401  (HIP runtime through torch first)
    import ctypes
    import gpfit
    from gpfit import _lib
    probe = ctypes.CDLL(os.environ["GPFIT_LIB"])  # an older build may lack newer measurement hooks
    for name in [n for n in _lib.SIGNATURES if not hasattr(probe, n)]:
        del _lib.SIGNATURES[name]
    ctx = gpfit.Context(0)
    out = {}
    for N, d, P in CASES:
        rng = np.random.default_rng(N)
        x = rng.uniform(size=(d, N))
        y = np.sin(3 * x[0]) + x[1]
        e = rng.uniform(0.05, 0.2, N)
        ctx.set_data(x, y, e)
        sig = np.linspace(0.1, 3, 30)
        ctx.set_grid(sig, 100 * (1 - 2 * (1 - 0.5 * (1 + np.tanh(sig / 1.4)))), np.zeros(d), np.ones(d))
        try:
            L, U, z, al = ctx.debug_factor(np.full(d, 0.3))
        except Exception as err:  # report and keep going
            print(f"N={N}: debug_factor failed: {err}", flush=True)
            L = U = np.zeros((1, 1))
            z = al = np.zeros(1)
        ls = rng.uniform(0.1, 0.6, size=(P, d))
        try:
            loss, mu, sd = ctx.eval_batch(ls, want_mu_sd=True)
        except Exception as err:
            print(f"N={N}: eval_batch failed: {err!r}", flush=True)
            loss, mu, sd = np.zeros(1), np.zeros(1), np.zeros(1)
        print(f"N={N} done: loss[:3]={loss[:3]}", flush=True)
        for k, v in dict(L=np.tril(L), U=np.tril(U), z=z, alpha=al, loss=loss, mu=mu, sd=sd).items():
            out[f"{N}_{k}"] = v
    np.savez(sys.argv[3], **out)
    ctx.close()
else:
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    worst = 0.0
    for k in a.files:
        x, y = a[k], b[k]
        same = np.array_equal(x, y)
        rel = float(np.max(np.abs(x - y) / np.maximum(np.abs(x), 1e-300))) if not same else 0.0
        nrm = float(np.max(np.abs(x - y)) / max(np.max(np.abs(x)), 1e-300)) if not same else 0.0
        worst = max(worst, nrm)
        print(f"{k:14s} {'bitwise' if same else f'max elementwise rel {rel:.3e}  max|d|/max|x| {nrm:.3e}'}")
    print("worst normwise", worst)
