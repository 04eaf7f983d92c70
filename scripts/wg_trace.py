"""Per-workgroup timeline of k_step launches (diagnostic build libgpfit_trace.so).

For each block column J: launch span, slot occupancy (sum of workgroup durations /
(512 slots x span)), and mean time per block of GEMM depth for L and U tiles."""
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
sys.path.insert(0, ROOT)
from oracle import ref_cpu  # noqa: E402
lo, hi = ref_cpu.search_bounds(x)
s, ex = ref_cpu.sigma_grid()
ctx = gpfit.Context(0)
ctx.set_data(x, y, e)
ctx.set_grid(s, ex, lo, hi)
for _ in range(2):
    ctx.eval_batch(rng.uniform(0.05, 0.6, size=(P, d)))
W = P * (nt - 1)
buf = np.zeros((nt, W, 3), dtype=np.uint64)
assert ctx.lib.gpf_debug_wg_trace(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), nt, W) == 0
tot_busy = tot_span = 0.0
for J in range(nt):
    st, en = buf[J, :, 0].astype(np.float64), buf[J, :, 1].astype(np.float64)
    dur = (en - st) * 10e-3  # us (100 MHz)
    span = (en.max() - st.min()) * 10e-3
    busy = dur.sum()
    b = np.arange(W)
    w = b // P
    nL = nt - 1 - J
    isL = w < nL
    units = np.where(isL, J + 2, np.maximum(J - (w - nL), 0) + 1).astype(np.float64)
    first_end = (en.min() - st.min()) * 10e-3
    last_start = (st.max() - st.min()) * 10e-3
    tail = span - last_start
    tot_busy += busy
    tot_span += span
    print(f"J={J:2d} span {span:8.1f} us  occ {busy / (512 * span):5.2f}  L {dur[isL].mean() if isL.any() else 0:7.1f} us "
          f"({(dur[isL] / units[isL]).mean() if isL.any() else 0:5.1f}/unit)  U {dur[~isL].mean() if (~isL).any() else 0:7.1f} us "
          f"({(dur[~isL] / units[~isL]).mean() if (~isL).any() else 0:5.1f}/unit)  last start {last_start:7.1f}  tail {tail:6.1f}")
print(f"total span {tot_span / 1e3:.2f} ms, mean occupancy {tot_busy / (512 * tot_span):.3f}")
ctx.close()
