"""Diagnostic: phase timing of the 128x128 diagonal factor (stamped build)."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GPFIT_LIB"] = os.path.join(ROOT, "gaussian-process_amd", os.environ.get("STAMPS_LIB", "libgpfit_stamps.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import gpfit
from oracle import ref_cpu
ctx = gpfit.Context(0)
names = ["factor64 #1", "store L11/U11, z1, partials", "L21 = A21 U11^T", "syrk, y2, T", "factor64 #2",
         "store L22/U22", "U21 = -U22 T", "z2", "partials + out"]
for N, P in [(int(a), int(b)) for a, b in (c.split("x") for c in os.environ.get("CFGS", "128x1,1024x32,4096x1").split(","))]:
    rng = np.random.default_rng(0)
    x = rng.uniform(size=(3, N)); y = np.sin(6 * x[0]); e = np.full(N, 0.1)
    lo, hi = ref_cpu.search_bounds(x); s, ex = ref_cpu.sigma_grid()
    ctx.set_data(x, y, e); ctx.set_grid(s, ex, lo, hi)
    for _ in range(3):
        ctx.eval_batch(rng.uniform(0.1, 0.5, size=(P, 3)))
    buf = (ctypes.c_ulonglong * 32)()
    assert ctx.lib.gpf_debug_diag_stamps(buf, 32) == 0
    st = np.array(buf[:10], dtype=np.float64)
    d = np.diff(st)
    print(f"N={N} P={P}: total {st[9]-st[0]:.0f} cycles; " + ", ".join(f"{n} {v:.0f}" for n, v in zip(names, d)))
    p = np.array(buf[10:14], dtype=np.float64)
    if p.any(): print(f"    iteration k=4 (last factor64, wave 0): barrier {p[1]-p[0]:.0f}, strip read+update {p[2]-p[1]:.0f}, "
          f"factor panel {p[3]-p[2]:.0f}")
    u = np.array(buf[20:26], dtype=np.float64)
    if u.any():
        print(f"    iteration k=4 update wave 1: work {u[1]-u[0]:.0f} (starts {u[0]-p[1]:+.0f} vs wave 0 after the barrier); "
              f"wave 7: work {u[5]-u[4]:.0f} (starts {u[4]-p[1]:+.0f})")
