"""Critical-tile timeline per block column (diagnostic build libgpfit_trace.so, -DGPF_WG_TRACE).

For each k_step launch J of the last factorisation: the launch span (first workgroup start to
last end), and for particle 0's tile w = 0 (I = J+1: the GEMM, TRMM, SYRK, dot and the fused
diagonal factor of the next block) its workgroups' start and GEMM end, then the finisher's
phase ends (TRMM, SYRK, dot) and its end (after factor128), all relative to the launch start,
in microseconds. MODE=predict: GP prediction at N (single particle, all tiles split);
MODE=eval: a batch of P particles (config B: N=1024 P=32)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GPFIT_LIB"] = os.path.join(ROOT, "gaussian-process_amd", "libgpfit_trace.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
import gpfit  # noqa: E402
from gpfit import _lib  # noqa: E402

probe = ctypes.CDLL(os.environ["GPFIT_LIB"])
mode = os.environ.get("MODE", "predict")
N = int(os.environ.get("N", 4096 if mode == "predict" else 1024))
d = int(os.environ.get("D", 3 if mode == "predict" else 2))
P = int(os.environ.get("P", 1 if mode == "predict" else 32))
T = 128
nt = -(-N // T)
rng = np.random.default_rng(1)
x = rng.uniform(size=(d, N))
y = np.sin(2 * np.pi * x).sum(0) + 0.1 * rng.standard_normal(N)
e = np.full(N, 0.1)


def split_la_bits(J, nt):  # the r4 split look-ahead (09b4abc, removed after profiles/r4/ab_split_la.txt)
    if os.environ.get("GPF_SPLIT_LA", "0") == "0" or nt < 4:
        return 0
    return (1 if 1 <= J <= nt - 3 else 0) | (2 if 2 <= J <= nt - 2 else 0)


def split_all_chunks(J, w, nt, la=0):  # mirrors gpf::split_all_chunks / split_all_pieces / split_all_target
    if w == nt - 1:
        return J * 8 if la & 1 else 0
    if w == 0 and la & 2:
        return 8
    nL = nt - 1 - J
    return (J if w < nL else J - (w - nL)) * 8


def split_all_pieces(J, w, nt, tgt, la=0):
    if w == 0 and la & 2:
        return 1
    c = split_all_chunks(J, w, nt, la)
    return min(32, 1 if c <= 0 else -(-c // tgt))


def split_all_target(pc, nt, J, la=0):
    budget = max(1, int(os.environ.get("GPF_SPLIT_K_SLOTS", 256)) - pc)
    minch = int(os.environ.get("GPF_SPLIT_K_MINCH", 4))
    wl = nt if la & 1 else nt - 1
    tot = sum(split_all_chunks(J, w, nt, la) for w in range(wl))
    cap = max(1, J * 8)
    lo, hi = min(cap, max(minch, -(-pc * tot // budget))), cap
    while lo < hi:
        m = (lo + hi) // 2
        if pc * sum(split_all_pieces(J, w, nt, m, la) for w in range(wl)) <= budget:
            hi = m
        else:
            lo = m + 1
    return lo


ctx = gpfit.Context(0)
ctx.set_data(x, y, e)
if mode == "predict":
    xf = rng.uniform(size=(d, 2000))
    for _ in range(2):
        ctx.predict(np.full(d, 0.3), xf)
else:
    s = np.linspace(0.001, 3, 1000)
    lo, hi = np.full(d, 1e-6), np.full(d, 2.0)
    ctx.set_grid(s, np.clip(s / 3, 0, 1), lo, hi)
    for _ in range(2):
        ctx.eval_batch(rng.uniform(0.05, 0.6, size=(P, d)))
ctx.synchronize()
plan = gpfit.plan_check(P, nt)
W = 4096
tr = np.zeros((nt, W, 3), dtype=np.uint64)
ph = np.zeros((nt, W, 4), dtype=np.uint64)
u64p = ctypes.POINTER(ctypes.c_ulonglong)
assert probe.gpf_debug_wg_trace(tr.ctypes.data_as(u64p), nt, W) == 0
assert probe.gpf_debug_wg_phase(ph.ctypes.data_as(u64p), nt, W) == 0
tot = 0.0
print("J   span   | w0: pieces start..gemm-end (max)  gemm-only (max, finisher)  finisher: trmm   syrk    end   (us from launch start)")
for J in range(nt - 1):
    st, en = tr[J, :, 0].astype(np.int64), tr[J, :, 1].astype(np.int64)
    live = (st > 0) & (en >= st)
    # this launch's workgroups: those that started after the previous launch's first start
    if not live.any():
        continue
    t0 = st[live].min()
    # discard stale entries of an older, longer launch with the same J
    live &= st >= t0
    span = (en[live].max() - t0) * 1e-2
    tot += span
    # tile w = 0 of particle 0: block ids with (p, w) = (0, 0) in particle-fastest order, plus pieces;
    # the launch starts with P diagonal workgroups (early diagonal factor), then, in launches
    # 1 .. nt-2 without the all-tile split, P SYRK workgroups (deferred diagonal update)
    ed = P if plan["diag_workgroups"] > 0 else 0
    if mode == "predict":  # balanced all-tile split: tile w = 0's pieces right after the diagonal workgroup
        la = split_la_bits(J, nt)
        tgt = split_all_target(P, nt, J, la)
        np0 = split_all_pieces(J, 0, nt, tgt, la)
        ids = [b for b in range(ed, ed + np0 * P, P) if live[b]]
        if la & 1:  # the look-ahead pieces (virtual tile w = nt-1) after every real tile
            o = ed + P * sum(split_all_pieces(J, w, nt, tgt, la) for w in range(nt - 1))
            lids = [b for b in range(o, o + P * split_all_pieces(J, nt - 1, nt, tgt, la), P) if live[b]]
            if lids:
                p0 = ph[J].astype(np.int64)
                print(f"   la: {len(lids)} pieces, gemm-only max {(max(p0[b, 3] for b in lids) - t0) * 1e-2:6.1f}"
                      f"  end max {(max(en[b] for b in lids) - t0) * 1e-2:6.1f}  (target {tgt} chunks)")
                if os.environ.get("LA_DETAIL"):
                    r = lambda v: (v - t0) * 1e-2 if v >= t0 else float("nan")  # noqa: E731
                    print("      " + "  ".join(f"[{b}: {r(st[b]):.1f} {r(p0[b, 3]):.1f} {r(p0[b, 0]):.1f} {r(p0[b, 1]):.1f} "
                                              f"{r(en[b]):.1f} hw{int(tr[J, b, 2]):x}]" for b in lids))
    else:  # critical-tile split (csrc/gpfit_api.hip split_crit, off by default): pieces at b = off + s * P
        off = ed + (P if (plan["syrk_workgroups"] > 0 and 1 <= J <= nt - 2) else 0)
        # r4 reordered dispatch (GPF_REORDER, default on): light U tiles, SYRK, diagonal, then w = 0
        ro = (os.environ.get("GPF_REORDER", "1") != "0" and ed and plan["syrk_workgroups"] > 0 and 1 <= J <= nt - 2
              and 3 * P <= 256)
        if ro:
            off = 3 * P
        if os.environ.get("GPF_LOOKAHEAD", "0") != "0" and ed and 1 <= J <= nt - 3 and plan["syrk_workgroups"] == 0:
            off += P  # look-ahead workgroups of their own (gpf::la_item; with SYRK workgroups it rides on them)
        S = 1 if (J == 0 or J >= nt - 1 or nt < 4) else min(int(os.environ.get("GPF_SPLIT_CRIT", 1)), max(1, J * T // 16 // 16))
        while S > 1 and P * (nt - 1) + P * (S - 1) + off > 512:
            S -= 1
        ids = [off + s * P for s in range(S) if live[off + s * P]]
    last = int(np.argmax(np.where(live, en, 0)))
    d0 = 2 * P if (mode != "predict" and ed and plan["syrk_workgroups"] > 0 and 1 <= J <= nt - 2 and 3 * P <= 256
                   and os.environ.get("GPF_REORDER", "1") != "0") else 0
    dg = f" diag end {(en[d0] - t0) * 1e-2:6.1f}" if ed else ""
    if not ids:
        print(f"{J:2d} {span:7.1f}")
        continue
    p0 = ph[J].astype(np.int64)
    fin = max(ids, key=lambda b: en[b])
    g_end = max(p0[b, 0] for b in ids if p0[b, 0] >= t0) if any(p0[b, 0] >= t0 for b in ids) else 0
    rel = lambda v: (v - t0) * 1e-2 if v >= t0 else float("nan")  # noqa: E731
    g_only = max(p0[b, 3] for b in ids)
    print(f"{J:2d} {span:7.1f}   | {len(ids):2d} pieces {rel(min(st[b] for b in ids)):6.1f}..{rel(g_end):6.1f}"
          f"   {rel(g_only):6.1f} {rel(p0[fin, 3]):6.1f}"
          f"   {rel(p0[fin, 1]):6.1f} {rel(p0[fin, 2]):6.1f} {rel(en[fin]):6.1f}"
          f"  |{dg}  last wg {last} ends {(en[last] - t0) * 1e-2:6.1f}")
print(f"sum of launch spans {tot:.1f} us")
ctx.close()
