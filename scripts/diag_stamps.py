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
        try:
            ctx.eval_batch(rng.uniform(0.1, 0.5, size=(P, 3)))
        except Exception as err:  # timing-experiment builds compute garbage
            print(f"    (eval_batch: {type(err).__name__})")
    NS = 32 + 16 * 16
    buf = (ctypes.c_ulonglong * NS)()
    assert ctx.lib.gpf_debug_diag_stamps(buf, NS) == 0
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
    # blocked factor64 (the last call): thread 0 leaving each of its 9 barriers (stamps 32..40, start 31),
    # wave 0's block-column factors ending (41..44)
    bs = np.array(buf[31:45], dtype=np.float64)
    if bs[0] and bs[10:14].all():
        ph = ["P1(0)", "P2(0)", "P1(1)", "P2(1)", "P1(2)", "P2(2)", "P1(3)", "T1", "T2"]
        print("    blocked factor64 phases (cycles): " + ", ".join(f"{n} {v:.0f}" for n, v in zip(ph, np.diff(bs[:10]))))
        print("    wave 0 column factors k=0..3 end after phase start: " +
              ", ".join(f"{bs[10 + k] - bs[2 * k]:.0f}" for k in range(4)))
    # per panel of the last factor64 call (build with the per-panel stamps)
    pk = np.array(buf[32:32 + 256], dtype=np.float64).reshape(16, 16)
    if pk[:, 8].any():
        print("    k | w0 work (apply, factor) | update waves: last arrival (wave), spread | barrier release after last arrival")
        for k in range(1, 16):
            t0 = pk[k - 1, 8]  # wave 0 left the barrier of panel k-1
            arr = pk[k, :8] - t0
            last = int(np.argmax(arr[1:])) + 1
            print(f"   {k:2d} | {arr[0]:6.0f} ({pk[k - 1, 9] - t0:5.0f}, {pk[k - 1, 10] - pk[k - 1, 9]:5.0f}) | "
                  f"{arr[last]:6.0f} (w{last}), {arr[1:].min():6.0f}..{arr[1:].max():6.0f} | {pk[k, 8] - pk[k, :8].max():6.0f}")
    uw = int(os.environ.get("DIAG_UW", 4))
    if pk[:, 14].any():
        print(f"    update wave {uw} per panel k (cycles after wave 0 leaves barrier k): leaves, after slot 0/1/2, arrives at k+1")
        for k in range(15):
            t0 = pk[k, 8]
            print(f"   {k:2d} | {pk[k, 14] - t0:6.0f} | {pk[k, 11] - t0:6.0f} {pk[k, 12] - t0:6.0f} {pk[k, 13] - t0:6.0f} | "
                  f"{pk[k + 1, uw] - t0:6.0f}")
