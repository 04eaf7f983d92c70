"""Per-phase time of k_step workgroups (diagnostic build libgpfit_trace.so, -DGPF_WG_TRACE), for
the round-3 schedule: one particle group (GPF_GROUPS=1 is forced: the trace buffer is indexed by
block column and workgroup id, which two concurrent group launches would share), SYRK workgroups
(deferred diagonal update) in front of the tiles in launches 1 .. nt-2.

L tiles: gemm (covariance seed + depth-128J stream) | trmm (U_JJ staged, L^T = U_JJ D, stores,
y update) | syrk (critical tile only: wait for the SYRK workgroup, rank-128 update) | rest (the
fused diagonal of the critical tile). U tiles: gemm | trmm (+ column partials). SYRK workgroups:
whole duration. Mean over the workgroups of each kind per block column J, in microseconds
(wave-0 stamps, s_memrealtime at 100 MHz)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GPFIT_LIB"] = os.path.join(ROOT, "gaussian-process_amd", os.environ.get("TRACE_LIB", "libgpfit_trace.so"))
os.environ["GPF_GROUPS"] = "1"
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import gpfit  # noqa: E402
from gpfit import _lib  # noqa: E402

probe = ctypes.CDLL(os.environ["GPFIT_LIB"])
for name in [n for n in _lib.SIGNATURES if not hasattr(probe, n)]:
    del _lib.SIGNATURES[name]
N, d, P = int(os.environ.get("N", 4096)), int(os.environ.get("D", 3)), int(os.environ.get("P", 64))
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
plan = gpfit.plan_check(P, nt)
ed = plan["diag_workgroups"] > 0
sy_on = plan["syrk_workgroups"] > 0
W = P * (nt - 1) + 2 * P
tr = np.zeros((nt, W, 3), dtype=np.uint64)
ph = np.zeros((nt, W, 4), dtype=np.uint64)
u64p = ctypes.POINTER(ctypes.c_ulonglong)
assert probe.gpf_debug_wg_trace(tr.ctypes.data_as(u64p), nt, W) == 0
assert probe.gpf_debug_wg_phase(ph.ctypes.data_as(u64p), nt, W) == 0
tot = {}
print(f"N={N} P={P} nt={nt} early_diag={ed} deferred_syrk={sy_on}")
print("J  | SYRK wg | L: n   gemm   trmm   syrk   rest |  U: n   gemm   trmm | launch span (us, mean per workgroup)")
for J in range(nt):
    off = (P if ed else 0) + (P if (sy_on and 1 <= J <= nt - 2) else 0)
    st, en = tr[J, :, 0].astype(np.int64), tr[J, :, 1].astype(np.int64)
    p = ph[J].astype(np.int64)
    line = f"{J:2d} |"
    if off > (P if ed else 0):
        sw = slice(off - P, off)
        dur = (en[sw] - st[sw]) * 1e-2
        tot["syrk_wg"] = tot.get("syrk_wg", 0.0) + dur.sum()
        line += f" {dur.mean():7.1f} |"
    else:
        line += "         |"
    n = P * (nt - 1)
    ids = np.arange(off, off + n)
    w = (ids - off) // P
    nL = nt - 1 - J
    isL = w < nL
    L = ids[isL]
    U = ids[~isL]
    if len(L):
        b = [st[L], p[L, 0], p[L, 1], p[L, 2], en[L]]
        seg = [np.diff(np.stack(b), axis=0)[i] * 1e-2 for i in range(4)]
        for i, nm in enumerate(["Lgemm", "Ltrmm", "Lsyrk", "Lrest"]):
            tot[nm] = tot.get(nm, 0.0) + seg[i].sum()
        line += f" {len(L):5d} " + " ".join(f"{v.mean():6.1f}" for v in seg)
    else:
        line += " " * 34
    line += " |"
    if len(U):
        b = [st[U], p[U, 0], en[U]]
        seg = [np.diff(np.stack(b), axis=0)[i] * 1e-2 for i in range(2)]
        for i, nm in enumerate(["Ugemm", "Utrmm"]):
            tot[nm] = tot.get(nm, 0.0) + seg[i].sum()
        line += f" {len(U):5d} " + " ".join(f"{v.mean():6.1f}" for v in seg)
    else:
        line += " " * 19
    allw = np.arange(0, off + n)
    line += f" | {(en[allw].max() - st[allw].min()) * 1e-2:8.1f}"
    print(line)
allt = sum(tot.values())
print("share of workgroup-slot time: " + ", ".join(f"{k} {v / allt * 100:.1f}%" for k, v in tot.items()))
print("slot-time / 512 slots: " + ", ".join(f"{k} {v / 512 / 1e3:.2f} ms" for k, v in tot.items()))
ctx.close()
