"""Does the early diagonal factor share its CU? (round-4 diagnostic, trace build libgpfit_trace.so,
-DGPF_WG_TRACE: every k_step workgroup's start / end (s_memrealtime, 100 MHz) and HW_ID / XCC_ID.)
Config B by default (N=1024 d=2, 32 particles). Per launch J: the diagonal workgroups' mean duration
when alone on their CU during their whole run vs when another workgroup of the launch overlapped
them on the same CU, and how many shared."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GPFIT_LIB"] = os.path.join(ROOT, "gaussian-process_amd", "libgpfit_trace.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import gpfit  # noqa: E402

probe = ctypes.CDLL(os.environ["GPFIT_LIB"])
N, d, P = int(os.environ.get("N", 1024)), int(os.environ.get("D", 2)), int(os.environ.get("P", 32))
nt = -(-N // 128)
rng = np.random.default_rng(1)
x = rng.uniform(size=(d, N))
y = np.sin(2 * np.pi * x).sum(0) + 0.1 * rng.standard_normal(N)
ctx = gpfit.Context(0)
ctx.set_data(x, y, np.full(N, 0.1))
s = np.linspace(0.001, 3, 1000)
ctx.set_grid(s, np.clip(s / 3, 0, 1), np.full(d, 1e-6), np.full(d, 2.0))
for _ in range(3):
    ctx.eval_batch(rng.uniform(0.05, 0.6, size=(P, d)))
ctx.synchronize()
W = 4096
tr = np.zeros((nt, W, 3), dtype=np.uint64)
assert probe.gpf_debug_wg_trace(tr.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), nt, W) == 0
print("J  wgs  diag end  | diag alone: n  mean us | diag shared: n  mean us | CUs with 2+ wgs")
for J in range(nt):
    st, en, hw = tr[J, :, 0].astype(np.int64), tr[J, :, 1].astype(np.int64), tr[J, :, 2]
    live = (st > 0) & (en >= st)
    if not live.any():
        continue
    t0 = st[live].min()
    live &= st >= t0
    ids = np.nonzero(live)[0]
    key = {}
    for b in ids:
        h = int(hw[b])
        xcc, hid = h >> 32, h & 0xFFFFFFFF
        key[b] = (xcc, (hid >> 8) & 0xF, (hid >> 12) & 1, (hid >> 13) & 7)
    cus = {}
    for b in ids:
        cus.setdefault(key[b], []).append(b)
    # diagonal workgroups: the first P of the launch, or the third P under the reordered dispatch
    # (launches 1 .. nt-2 with SYRK workgroups, GPF_REORDER on by default)
    ro = os.environ.get("GPF_REORDER", "1") != "0" and 1 <= J <= nt - 2
    dg = ids[(ids >= 2 * P) & (ids < 3 * P)] if ro else ids[ids < P]
    alone, shared = [], []
    for b in dg:
        others = [o for o in cus[key[b]] if o != b and st[o] < en[b] and en[o] > st[b]]
        (shared if others else alone).append((en[b] - st[b]) * 1e-2)
    multi = sum(1 for v in cus.values() if len(v) > 1)
    fmt = lambda v: f"{len(v):3d} {np.mean(v):7.1f}" if v else "  0     nan"  # noqa: E731
    print(f"{J:2d} {len(ids):4d} {(en[dg].max() - t0) * 1e-2 if len(dg) else float('nan'):8.1f}  |"
          f"   {fmt(alone)}     |    {fmt(shared)}      | {multi}")
ctx.close()
