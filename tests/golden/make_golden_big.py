"""Reference-generated fixtures at the BASELINE sizes and for the KMeans subsample.

Run in the build container only (needs /root/reference, read-only), one fixture per call:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_big.py f8
    PYTHONDONTWRITEBYTECODE=1 OMP_NUM_THREADS=8 OPENBLAS_NUM_THREADS=8 \
        python tests/golden/make_golden_big.py f9
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_big.py f10
    PYTHONDONTWRITEBYTECODE=1 OMP_NUM_THREADS=1 OPENBLAS_NUM_THREADS=1 \
        python tests/golden/make_golden_big.py f11   # the reference pool policy: 1 BLAS thread
    PYTHONDONTWRITEBYTECODE=1 OMP_NUM_THREADS=8 OPENBLAS_NUM_THREADS=8 \
        python tests/golden/make_golden_big.py f9b

It reuses make_golden.py's loader: GP_func imported as shipped, find_len_scales executed with
only its `smt` import dropped. What runs is the reference's own code:

  * F8 (config C/D data, N=4096 d=3, seed 1) and F9 (config E data, N=16384 d=4
    heteroscedastic, seed 1): evaluate_loss (find_len_scales.py:181-182 -> wass_loss :154-177)
    for a few interior particles. The GP() call inside wass_loss (:159 -> GP_func.py:12-45) is
    wrapped to record the mean / sd it returned, so the fixture holds exactly the mu/sd the
    reference scored (one GP per particle instead of two). F9 is generated with 8 BLAS threads
    (single-threaded it takes ~25 min); threads change only the rounding of the LAPACK calls.
  * F11 (config B data, N=1024 d=2, seed 0 as SURVEY.md §8d prescribes for B): evaluate_loss
    and the recorded mean / sd for 8 interior particles, so config B's own timed schedule (a
    32-particle batch on the early-diagonal path) is pinned to the reference.
  * F9b: two more config E particles (particle seed 16384 + 8), same recording as F9, so the
    default 16-particle E batch holds 4 reference-scored particles.
  * F10: the KMeans subsample of len_scale_opt (find_len_scales.py:25-47) at N = 300..4096:
    the reference's Pool is replaced by a stub whose map() captures the (x, y, e, bounds) the
    first fan-out ships (:76) and stops the run; the kept indices are recovered by matching
    columns. The inputs are not stored (they are regenerated from the seed; a sha256 of their
    bytes is stored and checked by the tests).

Outputs are data only. The GPU box never sees /root/reference.
"""
from __future__ import annotations

import hashlib
import sys
import time
import types
from pathlib import Path

sys.dont_write_bytecode = True
sys.path.insert(0, str(Path(__file__).resolve().parent))

import numpy as np  # noqa: E402

import make_golden as mg  # noqa: E402  (imports the reference modules)

OUT = Path(__file__).resolve().parent


def data_hash(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    return h.hexdigest()


def bounds(x):
    lo = np.array([np.min(g[g > 0]) if np.any(g > 0) else 0 for g in [np.diff(np.unique(r)) for r in x]])
    return lo, np.max(x, axis=1) - np.min(x, axis=1)


class RecordingGP:
    """Stands in for the module-global GP that wass_loss calls; records what it returned."""

    def __init__(self, gp):
        self.gp, self.calls = gp, []

    def __call__(self, *a, **k):
        mu, sd = self.gp(*a, **k)
        self.calls.append((mu.copy(), sd.copy()))
        return mu, sd


def make_scored(name, N, d, hetero, seed, n_particles, pseed):
    x, y, e = mg.synth_data(N, d, hetero, seed)
    lo, hi = bounds(x)
    s = np.linspace(0.001, 3, 1000)
    ex = mg.ref_fls.sigma_to_percent(s)
    P = np.random.default_rng(pseed).uniform(0.05, 0.6, size=(n_particles, d))
    rec = RecordingGP(mg.ref_fls.GP)
    mg.ref_fls.GP = rec
    loss = []
    try:
        for p in P:
            t0 = time.time()
            loss.append(mg.ref_fls.evaluate_loss(p, x, y, e, s, ex, lo, hi))
            print(f"{name}: particle {p} loss {loss[-1]!r} ({time.time() - t0:.1f} s)", flush=True)
    finally:
        mg.ref_fls.GP = rec.gp
    assert len(rec.calls) == n_particles
    mu = np.array([c[0] for c in rec.calls])
    sd = np.array([c[1] for c in rec.calls])
    np.savez_compressed(OUT / f"{name}.npz", meta=np.array([N, d, int(hetero), seed]),
                        data_sha256=np.array(data_hash(x, y, e)), lo=lo, hi=hi, P=P, loss=np.array(loss),
                        mu=mu, sd=sd, sigma_vals=s, expected=ex)
    print(f"{name}: wrote {len(P)} particles")


class _Stop(Exception):
    pass


class _CapturePool:
    captured = None

    def __init__(self, *a, **k):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def map(self, fn, args):
        _CapturePool.captured = list(args)[0]
        raise _Stop


def make_f10():
    cases = [(300, 2, True, 5), (1024, 2, False, 0), (2000, 4, True, 9), (4096, 3, False, 1)]
    fake_mp = types.SimpleNamespace(get_context=lambda kind: types.SimpleNamespace(Pool=_CapturePool))
    real_mp = mg.ref_fls.multiprocessing
    mg.ref_fls.multiprocessing = fake_mp
    mg.InjectedLHS.positions = None
    arrays = {}
    try:
        for i, (N, d, het, seed) in enumerate(cases):
            x, y, e = mg.synth_data(N, d, het, seed)
            lo_b, hi_b = bounds(x)
            mg.InjectedLHS.positions = lo_b + 0.5 * (hi_b - lo_b) * np.ones((40, d))  # unused: stops first
            # LHS is called with the subsample's bounds; give it a shape-correct answer
            mg.ref_fls.LHS = lambda xlimits, criterion: (lambda n: np.tile(np.mean(xlimits, axis=1), (n, 1)))
            try:
                mg.ref_fls.len_scale_opt(x, y, e, False)
            except _Stop:
                pass
            p, xs, ys, es, sv, exv, lo, hi = _CapturePool.captured
            cols = {tuple(x[:, j]): j for j in range(N)}
            idx = np.array([cols[tuple(xs[:, j])] for j in range(xs.shape[1])], dtype=np.int64)
            assert np.array_equal(x[:, idx], xs) and np.array_equal(y[idx], ys) and np.array_equal(e[idx], es)
            arrays.update({f"c{i}_meta": np.array([N, d, int(het), seed]),
                           f"c{i}_data_sha256": np.array(data_hash(x, y, e)),
                           f"c{i}_idx": idx, f"c{i}_lo": lo, f"c{i}_hi": hi})
            print(f"F10 N={N} d={d}: kept {len(idx)} points, lo={lo}, hi={hi}")
    finally:
        mg.ref_fls.multiprocessing = real_mp
        mg.ref_fls.LHS = mg.InjectedLHS
    arrays["ncases"] = np.array(len(cases))
    np.savez_compressed(OUT / "f10_kmeans.npz", **arrays)


if __name__ == "__main__":
    what = sys.argv[1:] or ["f8", "f10"]
    if "f8" in what:
        make_scored("f8_configC", 4096, 3, False, 1, 4, 4096 + 7)
    if "f9" in what:
        make_scored("f9_configE", 16384, 4, True, 1, 2, 16384 + 7)
    if "f9b" in what:
        make_scored("f9b_configE", 16384, 4, True, 1, 2, 16384 + 8)
    if "f10" in what:
        make_f10()
    if "f11" in what:
        make_scored("f11_configB", 1024, 2, False, 0, 8, 1024 + 7)
