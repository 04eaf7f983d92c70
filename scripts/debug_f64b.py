"""factor64 alone on the GPU (gpf_debug_factor64) vs numpy."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import torch  # noqa: F401,E402
import gpfit  # noqa: E402

ctx = gpfit.Context(0)
lib = ctx.lib
lib.gpf_debug_factor64.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_int)]
rng = np.random.default_rng(0)
B = rng.standard_normal((64, 64))
A1 = B @ B.T + 64 * np.eye(64)
An = A1.copy()
An[np.triu_indices(64, 1)] = np.nan
In = np.eye(64)
In[np.triu_indices(64, 1)] = np.nan
for name, A2 in [("identity", np.eye(64)), ("spd", A1.copy()), ("nan-upper", An), ("nan-upper-identity", In)]:
    inp = np.ascontiguousarray(np.stack([A1, A2]))
    out = np.zeros((4, 64, 64))
    bad = np.zeros(2, dtype=np.int32)
    lib.gpf_debug_factor64(ctx._h, inp.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                           out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                           bad.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    for k, A in enumerate([A1, A2]):
        Lr = np.linalg.cholesky(np.tril(A) + np.tril(A, -1).T)
        Xr = np.linalg.inv(Lr)
        dL = np.abs(out[2 * k] - Lr)
        dX = np.abs(out[2 * k + 1] - Xr)
        print(f"{name} call {k}: bad={bad[k]} |dL|={dL.max():.2e} |dX|={dX.max():.2e}")
        if not dL.max() < 1e-10 or not dX.max() < 1e-10:
            rows = sorted(set(np.argwhere(~(dL < 1e-10))[:, 0].tolist()))[:12]
            cols = sorted(set(np.argwhere(~(dL < 1e-10))[:, 1].tolist()))[:12]
            print("   bad L rows", rows, "cols", cols)
            rows = sorted(set(np.argwhere(~(dX < 1e-10))[:, 0].tolist()))[:12]
            cols = sorted(set(np.argwhere(~(dX < 1e-10))[:, 1].tolist()))[:12]
            print("   bad X rows", rows, "cols", cols)
ctx.close()
