"""Per-phase time of k_step workgroups (diagnostic build libgpfit_trace.so, -DGPF_WG_TRACE), config C's
shape on one particle group (GPF_GROUPS=1, GPF_LA_ALL=0): per block column J the mean time per
workgroup of each phase, and the share of all workgroup-slot time.

L tiles: gemm (covariance seed + the depth-128J GEMM) | fin (U_JJ staging, the triangular multiply
from the accumulators, the L stores and the y update) | syrk (the critical tile's diagonal update) |
rest (the critical tile's fused factor128). U tiles: gemm | fin (staging, triangular multiply, the U
stores) | part (the column partials). SYRK workgroups (deferred diagonal update): their whole span.
Decode as gpf::step_decode for these launches: [P SYRK workgroups if 1 <= J <= nt-2][tiles, particle
fastest]. usage: build the trace library (scripts/build_variant.sh trace -DGPF_WG_TRACE), then
N=4096 P=64 python scripts/wg_phase.py"""
import ctypes
import os
import sys

os.environ.setdefault("GPF_GROUPS", "1")
os.environ.setdefault("GPF_LA_ALL", "0")
os.environ.setdefault("GPF_PERSIST", "0")
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GPFIT_LIB"] = os.path.join(ROOT, "gaussian-process_amd", "libgpfit_trace.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import gpfit  # noqa: E402
from gpfit import _lib  # noqa: E402
from oracle import ref_cpu  # noqa: E402

probe = ctypes.CDLL(os.environ["GPFIT_LIB"])
N, d, P = int(os.environ.get("N", 4096)), 3, int(os.environ.get("P", 64))
T = 128
nt = -(-N // T)
rng = np.random.default_rng(1)
x = rng.uniform(size=(d, N))
y = np.sin(2 * np.pi * x).sum(0) + 0.1 * rng.standard_normal(N)
e = np.full(N, 0.1)
lo, hi = ref_cpu.search_bounds(x)
s, ex = ref_cpu.sigma_grid()
ctx = gpfit.Context(0)
ctx.set_data(x, y, e)
ctx.set_grid(s, ex, lo, hi)
for _ in range(2):
    ctx.eval_batch(rng.uniform(0.05, 0.6, size=(P, d)))
W = P * nt  # (tiles + SYRK workgroups per launch)
tr = np.zeros((nt, W, 3), dtype=np.uint64)
ph = np.zeros((nt, W, 4), dtype=np.uint64)
u64p = ctypes.POINTER(ctypes.c_ulonglong)
assert probe.gpf_debug_wg_trace(tr.ctypes.data_as(u64p), nt, W) == 0
assert probe.gpf_debug_wg_phase(ph.ctypes.data_as(u64p), nt, W) == 0
tot = {}
fsplit, fsum = {}, {}
print("J  |  L: n   gemm    fin   syrk   rest |  U: n   gemm    fin   part | SYRK wg | span (us, mean per workgroup)")
for J in range(nt):
    sy = 1 if 1 <= J <= nt - 2 else 0
    n = P * (nt - 1) + sy * P
    st, en = tr[J, :n, 0].astype(np.int64), tr[J, :n, 1].astype(np.int64)
    p = ph[J, :n].astype(np.int64)
    b = np.arange(n)
    isS = b < sy * P
    w = (b - sy * P) // P
    nL = nt - 1 - J
    isL = (~isS) & (w < nL)
    isU = (~isS) & (w >= nL)
    line = f"{J:2d} |"
    if isL.any():
        crit = isL & (w == 0)
        segs = [p[isL, 0] - st[isL], p[isL, 1] - p[isL, 0], p[crit, 2] - p[crit, 1], en[crit] - p[crit, 2]]
        segs = [v * 1e-2 for v in segs]
        for nm, v in zip(["L gemm", "L fin", "crit syrk", "crit factor"], segs):
            tot[nm] = tot.get(nm, 0.0) + v.sum()
        noncrit = isL & (w > 0)
        if noncrit.any():
            tot["L tail"] = tot.get("L tail", 0.0) + ((en[noncrit] - p[noncrit, 1]) * 1e-2).sum()
        line += f" {isL.sum():5d} " + " ".join(f"{v.mean():6.1f}" for v in segs)
    else:
        line += " " * 34
    line += " |"
    if isU.any():
        segs = [(p[isU, 0] - st[isU]) * 1e-2, (p[isU, 1] - p[isU, 0]) * 1e-2, (en[isU] - p[isU, 1]) * 1e-2]
        for nm, v in zip(["U gemm", "U fin", "U part"], segs):
            tot[nm] = tot.get(nm, 0.0) + v.sum()
        line += f" {isU.sum():5d} " + " ".join(f"{v.mean():6.1f}" for v in segs)
    else:
        line += " " * 27
    line += " |"
    if isS.any():
        v = (en[isS] - st[isS]) * 1e-2
        tot["SYRK wg"] = tot.get("SYRK wg", 0.0) + v.sum()
        line += f" {v.mean():7.1f}"
    else:
        line += " " * 8
    line += f" | {(en.max() - st.min()) * 1e-2:7.1f}"
    print(line)
    for nm, m in (("L", isL), ("U", isU)):  # the finish split at U_JJ staged (phase 3)
        if m.any():
            stg, mul = (p[m, 3] - p[m, 0]) * 1e-2, (p[m, 1] - p[m, 3]) * 1e-2
            fsum[nm + " fin: stage U_JJ"] = fsum.get(nm + " fin: stage U_JJ", 0.0) + stg.sum()
            fsum[nm + " fin: multiply+store"] = fsum.get(nm + " fin: multiply+store", 0.0) + mul.sum()
            extra = ""
            if nm == "U" and (p[m, 2] > 0).all():  # trace builds: slot 2 of a U tile = its staging loads arrived
                extra = f" (loads {((p[m, 2] - p[m, 0]) * 1e-2).mean():5.1f} + writes/barrier {((p[m, 3] - p[m, 2]) * 1e-2).mean():5.1f})"
            fsplit.setdefault(J, []).append(f"{nm} stage {stg.mean():5.1f}{extra} mult {mul.mean():5.1f}")
allt = sum(tot.values())
print("share of workgroup-slot time: " + ", ".join(f"{k} {v / allt * 100:.1f}%" for k, v in tot.items()))
print("finish split (us, mean per workgroup: U_JJ staging | triangular multiply + stores):")
for J, v in fsplit.items():
    print(f"{J:2d}  " + "  ".join(v))
print("finish split, share of workgroup-slot time: " + ", ".join(f"{k} {v / allt * 100:.1f}%" for k, v in fsum.items()))
ctx.close()
