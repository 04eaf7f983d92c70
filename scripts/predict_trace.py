"""Per-launch timeline of the single-particle prediction factorisation (diagnostic build
libgpfit_trace.so, -DGPF_WG_TRACE): for each k_step launch J, the launch span (first workgroup
start to last end), the diagonal workgroup's span (factor128 of block J, ending after its
partials), and over the pieces of the all-tile split (gpf::flat_piece) the latest wave-0 end of
each phase — A: partial stored, R: units summed, T: regions finished (triangular multiply), C: the
diagonal update blocks — all in microseconds from the launch start (s_memrealtime, 100 MHz).
Usage: python scripts/predict_trace.py [N] (default 4096, d = 3)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GPFIT_LIB"] = os.environ.get("TRACE_LIB", os.path.join(ROOT, "gaussian-process_amd", "libgpfit_trace.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import gpfit  # noqa: E402

probe = ctypes.CDLL(os.environ["GPFIT_LIB"])
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
d, T = 3, 128
nt = -(-N // T)
rng = np.random.default_rng(1)
x = rng.uniform(size=(d, N))
y = np.sin(2 * np.pi * x).sum(0) + 0.1 * rng.standard_normal(N)
e = np.full(N, 0.1)
ctx = gpfit.Context(0)
ctx.set_data(x, y, e)
xf = rng.uniform(size=(d, 2000))
for _ in range(2):
    ctx.predict(np.full(d, 0.3), xf)
ctx.synchronize()
W = 4096
tr = np.zeros((nt, W, 3), dtype=np.uint64)
ph = np.zeros((nt, W, 4), dtype=np.uint64)
u64p = ctypes.POINTER(ctypes.c_ulonglong)
assert probe.gpf_debug_wg_trace(tr.ctypes.data_as(u64p), nt, W) == 0
assert probe.gpf_debug_wg_phase(ph.ctypes.data_as(u64p), nt, W) == 0
print(f"N={N} nt={nt}: per launch J, us from the launch's first workgroup start")
print("  J  wgs   span | diag wg end | pieces: A max   R max   T max   C max |  last end")
tot = 0.0
prev_end = None
gaps = []
for J in range(nt):
    st, en = tr[J, :, 0].astype(np.int64), tr[J, :, 1].astype(np.int64)
    live = (st > 0) & (en >= st)
    if not live.any():
        continue
    t0 = st[live].min()
    live &= st >= t0
    span = (en[live].max() - t0) * 1e-2
    tot += span
    if prev_end is not None:
        gaps.append((t0 - prev_end) * 1e-2)
    prev_end = en[live].max()
    p = ph[J].astype(np.int64)
    ids = np.nonzero(live)[0]
    pieces = [b for b in ids if b > 0 and p[b, 3] >= t0]

    def mx(k):
        v = [p[b, k] for b in pieces if p[b, k] >= t0]
        return f"{(max(v) - t0) * 1e-2:7.1f}" if v else "      -"

    diag = (en[0] - t0) * 1e-2 if live[0] else float("nan")
    print(f"{J:3d} {len(ids):4d} {span:6.1f} | {diag:11.1f} | {mx(3)} {mx(0)} {mx(1)} {mx(2)} | {span:8.1f}")
print(f"sum of launch spans {tot / 1e3:.3f} ms; gaps between launches (last end -> next first start) "
      f"median {np.median(gaps):.1f} us, sum {sum(gaps) / 1e3:.3f} ms")
