"""Per-phase time of k_step workgroups (diagnostic build libgpfit_trace.so, -DGPF_WG_TRACE).

L tiles: GEMM (acc load + depth-128J stream + store C) | TRMM (C U_JJ^T + store) |
SYRK (load A_II, look-ahead update, store) | dot (y_I update) | rest (the fused diagonal, one
tile per particle). U tiles: GEMM (W = L U, store) | TRMM (-U_JJ W, store) | partials.
Mean over the workgroups of each kind, per block column J, in microseconds (wave-0 stamps)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GPFIT_LIB"] = os.path.join(ROOT, "gaussian-process_amd", "libgpfit_trace.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import torch  # noqa: F401,E402
import gpfit  # noqa: E402
from gpfit import _lib  # noqa: E402

probe = ctypes.CDLL(os.environ["GPFIT_LIB"])
for name in [n for n in _lib.SIGNATURES if not hasattr(probe, n)]:
    del _lib.SIGNATURES[name]
N, d, P = int(os.environ.get("N", 4096)), 3, int(os.environ.get("P", 64))
T = 128
nt = -(-N // T)
rng = np.random.default_rng(1)
x = rng.uniform(size=(d, N))
y = np.sin(2 * np.pi * x).sum(0) + 0.1 * rng.standard_normal(N)
e = np.full(N, 0.1)
from oracle import ref_cpu  # noqa: E402
lo, hi = ref_cpu.search_bounds(x)
s, ex = ref_cpu.sigma_grid()
ctx = gpfit.Context(0)
ctx.set_data(x, y, e)
ctx.set_grid(s, ex, lo, hi)
for _ in range(2):
    ctx.eval_batch(rng.uniform(0.05, 0.6, size=(P, d)))
W = P * (nt - 1)
tr = np.zeros((nt, W, 3), dtype=np.uint64)
ph = np.zeros((nt, W, 4), dtype=np.uint64)
u64p = ctypes.POINTER(ctypes.c_ulonglong)
assert probe.gpf_debug_wg_trace(tr.ctypes.data_as(u64p), nt, W) == 0
assert probe.gpf_debug_wg_phase(ph.ctypes.data_as(u64p), nt, W) == 0
tot = {}
print("J  |  L: n  gemm   trmm   syrk    dot   rest  |  U: n  gemm   trmm   part   (us, mean per workgroup)")
for J in range(nt):
    st, en = tr[J, :, 0].astype(np.int64), tr[J, :, 1].astype(np.int64)
    p = ph[J].astype(np.int64)
    w = np.arange(W) // P
    nL = nt - 1 - J
    isL = w < nL
    line = f"{J:2d} |"
    if isL.any():
        b = [st[isL], p[isL, 0], p[isL, 1], p[isL, 2], p[isL, 3], en[isL]]
        seg = [np.diff(np.stack(b), axis=0)[i] * 1e-2 for i in range(5)]
        for i, nm in enumerate(["Lgemm", "Ltrmm", "Lsyrk", "Ldot", "Lrest"]):
            tot[nm] = tot.get(nm, 0.0) + seg[i].sum()
        line += f" {isL.sum():5d} " + " ".join(f"{v.mean():6.1f}" for v in seg)
    else:
        line += " " * 42
    line += "  |"
    if (~isL).any():
        b = [st[~isL], p[~isL, 0], p[~isL, 1], en[~isL]]
        seg = [np.diff(np.stack(b), axis=0)[i] * 1e-2 for i in range(3)]
        for i, nm in enumerate(["Ugemm", "Utrmm", "Upart"]):
            tot[nm] = tot.get(nm, 0.0) + seg[i].sum()
        line += f" {(~isL).sum():5d} " + " ".join(f"{v.mean():6.1f}" for v in seg)
    print(line)
allt = sum(tot.values())
print("share of workgroup-slot time: " + ", ".join(f"{k} {v / allt * 100:.1f}%" for k, v in tot.items()))
print(f"slot-time / 512 slots: " + ", ".join(f"{k} {v / 512 / 1e3:.2f} ms" for k, v in tot.items()))
ctx.close()
