"""PSO length-scale search with the swarm as a batch axis.

Behaviour follows find_len_scales.py:22-150 line for line (same constants, same
RNG draws from the global ``np.random`` stream in the same order, same strict
``<`` comparisons and first-index ``argmin``, same progress strings); what
changes is the fan-out: instead of pickling one task per particle into a fork
pool (:73-77,102-104,133-135), every batch of particles is one call into the
HIP library (``gpf_eval_batch``), sharded across ranks when the launcher starts
several (one process per GPU; the library's own RCCL all-reduce per batch,
``gpf_eval_batch_sharded``).
"""
from __future__ import annotations

import numpy as np

from ._lib import default_comm, default_context

NUM_PARTICLES = 40      # find_len_scales.py:50
MAX_ITER = 500          # :51
PATIENCE = 100          # :52
INERTIA_DECAY = 0.002   # :53
MAX_POINTS = 100        # :25
SENTINEL = 1e13         # -wass_loss sentinel (:157) seen through evaluate_loss (:182)


def sigma_to_percent(x):
    """Two-sided normal coverage Phi(x) - Phi(-x) (find_len_scales.py:192-201)."""
    from scipy.stats import norm
    return norm.cdf(x) - norm.cdf(-x)


def sigma_grid():
    s = np.linspace(0.001, 3, 1000)          # :66
    return s, sigma_to_percent(s)            # :67


def search_bounds(x_known):
    """lower = smallest positive gap between sorted unique values, upper = range (:56-61)."""
    span = np.max(x_known, axis=1) - np.min(x_known, axis=1)
    lower = np.empty(x_known.shape[0])
    for k, row in enumerate(x_known):
        gaps = np.diff(np.unique(row))
        pos = gaps[gaps > 0]
        lower[k] = np.min(pos) if pos.size else 0
    return lower, span


def kmeans_representatives(x_known, y_known, e_known, max_points):
    """Nearest member to each KMeans centroid (:25-47); host-side, sklearn."""
    from sklearn.cluster import KMeans
    pts = x_known.T
    km = KMeans(n_clusters=max_points, n_init="auto", random_state=0)
    labels = km.fit_predict(pts)
    centres = km.cluster_centers_
    pick = []
    for k in range(max_points):
        members = np.where(labels == k)[0]
        if len(members) == 0:
            continue
        dist2 = np.sum((pts[members] - centres[k]) ** 2, axis=1)
        pick.append(members[np.argmin(dist2)])
    pick = np.array(pick)
    return x_known[:, pick], y_known[pick], e_known[pick]


def centred_lhs(lower, upper, n, seed=None):
    """Centred Latin hypercube (stands in for smt LHS(criterion='center'), :69-70).

    smt is not available here. Bin centres (k+1/2)/n per
    dimension with one permutation per dimension. Like smt's sampler it draws
    from a private RandomState, so the global np.random stream that feeds
    r1/r2 (:91-92) is consumed exactly as in the reference.
    """
    rs = np.random.RandomState(seed)
    d = lower.shape[0]
    u = np.empty((n, d))
    for k in range(d):
        u[:, k] = (rs.permutation(n) + 0.5) / n
    return lower + u * (upper - lower)


class ShardedScorer:
    """Scores a (P, d) batch of particles, sharded over the ranks of a gpfit.Comm.

    ``backend(positions) -> scores`` evaluates the local rows. With a GPU context the whole
    step is one library call, gpf_eval_batch_sharded: rank r scores rows [r*P//G, (r+1)*P//G)
    on its GPU and one all-reduce of a zero-initialised [P + G] vector (RCCL) gives every rank
    the full score vector (exact: one non-zero contributor per entry), so every rank takes the
    same argmin (find_len_scales.py:81,110). With an injected evaluator (tests) the local rows
    are scored in Python and the same C exchange runs (gpf_comm_exchange_scores). A failing
    particle on any rank raises the same error on every rank (the G status entries), instead
    of leaving the other ranks blocked in the collective. World size 1 is a plain call.
    """

    def __init__(self, backend, comm=None, ctx=None):
        self.backend = backend
        self.comm = comm if (comm is not None and comm.size > 1) else None
        self.ctx = ctx
        self.rank, self.world = (comm.rank, comm.size) if self.comm is not None else (0, 1)
        self.evals = 0

    def __call__(self, positions):
        P = positions.shape[0]
        if self.comm is None:
            self.evals += P
            return np.asarray(self.backend(positions), dtype=np.float64)
        lo, hi = self.comm.rows(P)
        self.evals += hi - lo
        if self.ctx is not None:
            return self.ctx.eval_batch_sharded(self.comm, positions)
        from ._lib import GPF_HIP_ERROR, GPF_NOT_PD, GPF_OK
        rc, local, failure, bad = GPF_OK, None, None, -1
        try:
            local = np.asarray(self.backend(positions[lo:hi]), dtype=np.float64) if hi > lo else np.zeros(0)
        except np.linalg.LinAlgError:
            rc = GPF_NOT_PD
            # the injected evaluator does not say which row failed: score the rows one at a time
            # (this path only runs on error), so the exchange reports the smallest failing row of
            # the whole swarm, the particle the reference's in-order map raises on
            bad = 0
            for i in range(hi - lo):
                try:
                    self.backend(positions[lo + i:lo + i + 1])
                except np.linalg.LinAlgError:
                    bad = i
                    break
        except Exception as exc:  # noqa: BLE001 - re-raised below, after the other ranks are told
            rc, failure = GPF_HIP_ERROR, exc
        try:
            return self.comm.exchange_scores(P, local, rc, bad)
        except Exception:
            if failure is not None:
                raise failure
            raise


def share_seed(seed, comm):
    """All ranks must draw identical r1/r2 (find_len_scales.py:91-92): rank 0's seed (picked
    from np.random when none is given) reaches every rank through one all-reduce."""
    if comm is None or comm.size == 1:
        return seed
    if seed is None:
        seed = int(np.random.randint(0, 2**31 - 1)) if comm.rank == 0 else 0
    mine = float(seed) if comm.rank == 0 else 0.0
    return int(comm.allreduce([mine])[0])


class Swarm:
    """PSO state machine of find_len_scales.py:22-150, one ``step`` per iteration.

    ``score(positions) -> scores`` is the (sharded) batch objective. The
    update order, constants, RNG draws and comparisons are the reference's:
    inertia w = max(0.4, 0.9 - 0.002 i) (:88), c1 = c2 = 1.4 (:89), r1/r2 from
    the global np.random stream (:91-92), clip to +-v_max and to the box
    (:98-100), strict ``<`` for personal bests (:106) and the global best
    (:113), first-index argmin (:81,110), soft restart after 100 stale
    iterations with +-10% jitter from np.random.uniform (:123-141).
    """

    def __init__(self, positions, lower, upper, score, progress=False, verbose=True):
        self.lower, self.upper = lower, upper
        self.v_max = 1.0 * (upper - lower)
        self.score = score
        self.progress = progress and verbose
        self.positions = np.array(positions, dtype=np.float64, copy=True)
        self.n, self.ndim = self.positions.shape
        self.velocities = np.zeros_like(self.positions)
        self.restarts = 0
        self.evals = 0
        self._rebest(self.positions.copy())

    def _rebest(self, pbest_pos):
        self.pbest_pos = pbest_pos
        self.pbest_scores = self.score(self.pbest_pos)
        self.evals += self.n
        g = np.argmin(self.pbest_scores)
        self.gbest_pos = self.pbest_pos[g].copy()
        self.gbest = self.pbest_scores[g]
        self.stale = 0

    def step(self, i):
        w = max(0.4, 0.9 - i * INERTIA_DECAY)
        c1 = c2 = 1.4
        r1 = np.random.rand(self.n, self.ndim)
        r2 = np.random.rand(self.n, self.ndim)
        v = (w * self.velocities + c1 * r1 * (self.pbest_pos - self.positions)
             + c2 * r2 * (self.gbest_pos - self.positions))
        self.velocities = np.clip(v, -self.v_max, self.v_max)
        self.positions += self.velocities
        self.positions = np.clip(self.positions, self.lower, self.upper)

        scores = self.score(self.positions)
        self.evals += self.n
        better = scores < self.pbest_scores
        self.pbest_pos[better] = self.positions[better]
        self.pbest_scores[better] = scores[better]
        c = np.argmin(self.pbest_scores)
        if self.pbest_scores[c] < self.gbest:
            self.gbest = self.pbest_scores[c]
            self.gbest_pos = self.pbest_pos[c].copy()
            self.stale = 0
        else:
            self.stale += 1

        if self.progress and i % 20 == 0:
            print(f"Iter {i}: Best Score = {self.gbest:.6f}, No Improve = {self.stale}")

        if self.stale >= PATIENCE:
            if self.progress:
                print(f"Stagnation at iter {i}, soft-restarting swarm...")
            noise = 0.1 * (self.upper - self.lower)
            jittered = self.pbest_pos + np.random.uniform(-noise, noise, self.pbest_pos.shape)
            jittered = np.clip(jittered, self.lower, self.upper)
            self.positions = jittered.copy()
            self.velocities = np.zeros_like(self.positions)
            self._rebest(jittered)
            self.restarts += 1


def prepare(x_known, y_known, e_known, *, max_points=MAX_POINTS, verbose=True, ctx=None):
    """KMeans subsample above max_points (:25-47), bounds (:56-61), sigma grid (:66-67). With a GPU
    context the KMeans fit's Lloyd iterations run on it (gpfit.kmeans, r4); without one (the
    injected-evaluator path of the CPU tests), or with more centres than the device step stages
    (max_points x (d + 1) > 8192), sklearn's fit runs on the host, as in the reference."""
    if x_known.shape[1] > max_points:
        if verbose:
            print(f"Dataset too large ({x_known.shape[1]} points). Subsampling to {max_points} for hyperparameter optimisation.")
        from .kmeans import fits_device, kmeans_representatives_gpu
        if ctx is not None and fits_device(max_points, x_known.shape[0]):
            x_known, y_known, e_known = kmeans_representatives_gpu(ctx, x_known, y_known, e_known, max_points)
        else:  # no device, or more centres than gpf_kmeans_step stages in LDS: sklearn's fit
            x_known, y_known, e_known = kmeans_representatives(x_known, y_known, e_known, max_points)
    lower, upper = search_bounds(x_known)
    sigma_vals, expected = sigma_grid()
    return x_known, y_known, e_known, lower, upper, sigma_vals, expected


def make_scorer(x_known, y_known, e_known, sigma_vals, expected, lower, upper, *, evaluator=None, ctx=None,
                comm=None):
    """Sharded batch objective: gpf_eval_batch(_sharded) on this GPU, or an injected per-particle
    evaluator. comm: a gpfit.Comm, or None for the launcher's group (WORLD_SIZE > 1) if any."""
    if evaluator is None:
        dev = ctx if ctx is not None else default_context()
        dev.set_data(x_known, y_known, e_known)
        dev.set_grid(sigma_vals, expected, lower, upper)
        comm = comm if comm is not None else default_comm(dev)
        return ShardedScorer(dev.eval_batch, comm, dev)

    def backend(pos):
        args = [(p, x_known, y_known, e_known, sigma_vals, expected, lower, upper) for p in pos]
        return np.array(list(evaluator(args)))
    comm = comm if comm is not None else default_comm()
    return ShardedScorer(backend, comm)


def particle_swarm(x_known, y_known, e_known, PSO_progress, *, num_particles=NUM_PARTICLES,
                   max_iter=MAX_ITER, max_points=MAX_POINTS, init_positions=None, seed=None,
                   evaluator=None, trace=None, ctx=None, comm=None, verbose=True):
    """len_scale_opt body (find_len_scales.py:22-150) with a batched evaluator.

    ``evaluator(args_list) -> scores`` (reference-style per-particle args, used
    by tests to inject a checker) replaces the default backend, gpf_eval_batch
    on this process's GPU. Either way batches are sharded over the ranks of ``comm`` (default:
    the launcher's group when WORLD_SIZE > 1, gpfit.default_comm).
    Returns (global_best_position, info) where info holds the final score,
    restart count and evaluation count.
    """
    if evaluator is None and ctx is None:  # the GPU path: this process's context, the KMeans fit included
        ctx = default_context()
    x_known, y_known, e_known, lower, upper, sigma_vals, expected = prepare(
        x_known, y_known, e_known, max_points=max_points, verbose=verbose, ctx=ctx if evaluator is None else None)

    score = make_scorer(x_known, y_known, e_known, sigma_vals, expected, lower, upper,
                        evaluator=evaluator, ctx=ctx, comm=comm)
    seed = share_seed(seed, score.comm)
    if seed is not None:
        np.random.seed(seed)
    if init_positions is None:
        init_positions = centred_lhs(lower, upper, num_particles, seed)

    sw = Swarm(init_positions, lower, upper, score, progress=PSO_progress, verbose=verbose)
    for i in range(max_iter):
        sw.step(i)
        if trace is not None:
            trace.append((float(sw.gbest), sw.gbest_pos.copy(), sw.stale, sw.restarts))

    if verbose:
        print("PSO completed.")
        print("Optimal length scale found:")
        print(sw.gbest_pos)
        print("Value of loss function:")
        print(sw.gbest)
        print(f"Total soft restarts: {sw.restarts}")
    comm = score.comm
    return sw.gbest_pos, {"score": sw.gbest, "restarts": sw.restarts, "evals": sw.evals,
                          "local_evals": score.evals, "transport": comm.transport if comm is not None else None,
                          "exchange": comm.stats() if comm is not None else None}
