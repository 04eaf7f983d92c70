"""Headline benchmark: PSO objective evals/s at N=4096, d=3 (BASELINE config C).

One "step" = the hot path of one PSO iteration (find_len_scales.py:102-104):
one batched objective evaluation of the whole swarm (gpf_eval_batch: K build,
Cholesky, L^-1 and the calibration loss for every particle) followed by the
all-reduce that gives every rank the full score vector. Every particle of the
timed steps is interior (SURVEY.md §8d fixed-work variant), so no evaluation
takes the sentinel short-cut. value = swarm x steps / wall time of the timed
region, max over ranks; at N GPUs the swarm is 64 particles per GPU (weak
scaling). The real PSO update loop, whose box-clipped particles are free
sentinels, is timed separately and reported under "pso_loop".

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 4096] [--d 3] [--swarm-per-gpu P]
                    [--no-cpu] [--plumbing]

N > 1: one process per GPU. Under a launcher (torchrun: RANK / WORLD_SIZE / LOCAL_RANK set)
this process is one rank; without one, `--gpus N` starts the N rank processes itself before
anything touches a GPU and exits with their status. The swarm exchange (one all-reduce per
batch) and the barrier / max-over-ranks timing go through libgpfit's own RCCL communicator
(gpf_comm_*). Default swarm: 64 particles on one GPU (config C); 32 per GPU at N > 1, which
is config D's 256-particle swarm at 8 GPUs (weak scaling, 32 per GPU).

Prints ONE JSON line on rank 0 (contract in the task statement), with a
"roofline" object for the dominant kernel (k_panel, the MFMA GEMM step) timed
with HIP events on the library's stream, and a "cpu_baseline" object: the
CPU oracle (a bit-exact NumPy restatement of the reference's evaluate_loss)
timed on this host's cores on a bounded sample of the same workload.
"""
from __future__ import annotations

import os

# BLAS pins must precede numpy (SURVEY.md §6 gotcha) — the CPU baseline runs one
# single-threaded evaluation per worker, exactly as the reference's pool (its modules assign
# these at import, GP_func.py:3-7, find_len_scales.py:3-7). Assigned, not defaulted: the GPU
# box presets OMP_NUM_THREADS=16.
for _k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS", "VECLIB_MAXIMUM_THREADS",
           "NUMEXPR_NUM_THREADS"):
    os.environ[_k] = "1"

import argparse  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402
from pathlib import Path  # noqa: E402

import numpy as np  # noqa: E402

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT), str(ROOT / "gaussian-process_amd")]

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X FP64 matrix (dense), spec; see DESIGN.md §Roofline
HBM_PEAK_GBS = 8000.0


def config_letter(N, d, swarm, hetero):
    """BASELINE.json configs: B = N1024 d2 P32, C/D = N4096 d3 (64 / 32 per GPU), E = N16384 d4 hetero."""
    if (N, d) == (1024, 2):
        return "B"
    if (N, d) == (4096, 3):
        return "C" if swarm == 64 else "D"
    if (N, d) == (16384, 4) and hetero:
        return "E"
    return "custom"


def _profile_order(f):
    """Sort key of a committed profile file: round directory (r1 < r3 < r3s2 < r4), then the
    evidence version of the file name (v5_ < v8_ < v12_), so the last match is the newest tree's."""
    import re
    rd = re.match(r"r(\d+)(?:s(\d+))?$", f.parent.name)
    vm = re.match(r"v(\d+)", f.name)
    return (int(rd.group(1)) if rd else -1, int(rd.group(2) or 0) if rd else 0, int(vm.group(1)) if vm else -1, f.name)


def pmc_traffic(N, d, swarm, kernel="k_step"):
    """HBM bytes per k_step launch from the newest committed rocprofv3 PMC passes
    (scripts/pmc_traffic.py writes profiles/<round>/[vK_]k_step_traffic.json), or None."""
    best = None
    for f in sorted((ROOT / "profiles").glob("*/*k_step_traffic.json"), key=_profile_order):
        try:
            t = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        if t.get("N") == N and t.get("d") == d and t.get("swarm") == swarm and t.get("kernel", "k_step") == kernel:
            best = {"bytes_per_launch": t["bytes_per_launch"], "source": str(f.relative_to(ROOT)),
                    "groups": t.get("particle_groups", 1), "per": t.get("per")}
    return best


def secondary_pmc():
    """rocprofv3 PMC summary of the secondary kernels from the latest committed
    profiles/<round>/secondary_pmc.json (scripts/gpu_secondary.sh + scripts/pmc_secondary.py,
    the bench's own secondary calls), or None."""
    best = None
    for f in sorted((ROOT / "profiles").glob("*/*secondary_pmc.json"), key=_profile_order):
        try:
            best = (json.loads(f.read_text()), str(f.relative_to(ROOT)))
        except (OSError, ValueError):
            continue
    return best


def synthetic(N, d, seed, hetero=False):
    """x ~ U[0,1)^d, y = sum_k sin(2 pi x_k) + 0.1 N(0,1), e = 0.1."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(0.0, 1.0, size=(d, N))
    y = np.sum(np.sin(2 * np.pi * x), axis=0) + 0.1 * rng.standard_normal(N)
    e = rng.uniform(0.05, 0.2, size=N) if hetero else np.full(N, 0.1)
    return x, y, e


def _cpu_eval(args):
    from oracle import ref_cpu
    return ref_cpu.evaluate_loss(*args)


def effective_cpus():
    """CPUs this process may actually use: affinity mask and cgroup quota (the GPU box shows
    the whole machine in os.cpu_count() but grants a 16-CPU share)."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def blas_threads():
    """Effective BLAS threading of this process (threadpoolctl), for the baseline record."""
    try:
        from threadpoolctl import threadpool_info
        return sorted({(i.get("internal_api"), i.get("num_threads")) for i in threadpool_info()})
    except Exception:  # noqa: BLE001 - diagnostic only
        return None


def cpu_baseline(x, y, e, positions, lo, hi, workers):
    """Reference-policy CPU path: a fork pool of single-BLAS-thread workers mapping
    evaluate_loss over the particles (find_len_scales.py:73-77)."""
    import multiprocessing as mp
    from oracle import ref_cpu
    s, ex = ref_cpu.sigma_grid()
    args = [(p, x, y, e, s, ex, lo, hi) for p in positions]
    ctx = mp.get_context("fork")
    with ctx.Pool(processes=workers) as pool:
        t0 = time.perf_counter()
        out = pool.map(_cpu_eval, args, chunksize=1)
        dt = time.perf_counter() - t0
    return len(args) / dt, np.array(out), dt


def cpu_baselines(x, y, e, lo, hi, N, d, seed):
    """Primary: the reference's own pool policy, Pool(max(1, os.cpu_count() // 4))
    (find_len_scales.py:73-75), every worker scoring one particle of the same workload.
    Secondary: one worker per CPU this process may use (cgroup quota / affinity)."""
    d_ = x.shape[0]
    rng = np.random.default_rng(seed + 7)
    eff = effective_cpus()
    policy = max(1, (os.cpu_count() or 1) // 4)
    out = {}
    for key, workers in (("primary", policy), ("all_cores", eff)):
        n = workers  # each worker scores (at least) one particle
        sample = lo + (hi - lo) * rng.uniform(0.2, 0.8, size=(n, d_))
        v, _, dt = cpu_baseline(x, y, e, sample, lo, hi, workers)
        out[key] = {"value": v, "unit": "evals/s", "workers": workers, "cores": min(workers, eff), "s": dt,
                    "evals": n}
    p = out["primary"]
    return {"value": p["value"], "unit": "evals/s", "cores": p["cores"], "kind": "port",
            "sample": f"{p['evals']} evaluate_loss calls (oracle/ref_cpu.py: the reference's NumPy/LAPACK calls, "
                      f"find_len_scales.py:154-182) at N={N} d={d} on the bench's synthetic data, in the reference's "
                      f"pool policy Pool(os.cpu_count()//4) = {p['workers']} fork workers on os.cpu_count() = "
                      f"{os.cpu_count()}, which this box's cgroup limits to {eff} CPUs; one BLAS thread per worker; "
                      f"{p['s']:.1f} s wall",
            "policy": "Pool(max(1, os.cpu_count() // 4)) (find_len_scales.py:73-75)",
            "workers": p["workers"], "host_cpu_count": os.cpu_count(), "effective_cpus": eff,
            "blas_env": {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS")},
            "blas_threads": blas_threads(),
            "all_cores": out["all_cores"]}


def predict_line(ctx, x, y, e, N, d, args):
    """Secondary measurement, SURVEY.md §8f row 1: GP(x, y, e, x_fit, l) at M query
    points (GP_fit.py:32 -> GP_func.py:12-45): one factorisation, then the
    cross-covariance build and V = U K_s reduced to column sums of squares."""
    M = args.predict_points
    rng = np.random.default_rng(args.seed + 99)
    xf = rng.uniform(size=(d, M))
    ls = np.full(d, 0.3)
    ctx.predict(ls, xf)  # warm-up (workspace, code objects)
    ctx.set_profiling(False)
    walls = []  # `ms`: five unprofiled calls (no HIP events in the stream), the median reported
    for _ in range(5):
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.predict(ls, xf)
        ctx.synchronize()
        walls.append(time.perf_counter() - t0)
    dt = sorted(walls)[2]
    runs = []  # the kernel breakdown: three more calls with an event pair around every launch
    for _ in range(3):
        ctx.reset_profile()
        ctx.set_profiling(True)
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.predict(ls, xf)
        ctx.synchronize()
        runs.append((time.perf_counter() - t0, ctx.profile()))
        ctx.set_profiling(False)
    pdt, prof = sorted(runs, key=lambda r: r[0])[1]
    out = {"N": N, "d": d, "M": M, "ms": dt * 1e3, "points_per_s": M / dt,
           "ms_runs": [round(w * 1e3, 3) for w in walls],
           "ms_profiled_pass": pdt * 1e3,
           "factor_flops": (2.0 / 3.0) * (-(-N // 128) * 128) ** 3,
           "factor_ms": prof["factor_wall_ms"],
           "k_predict_vsq_ms": prof["predict_ms"],
           "k_predict_vsq_tflops": prof["predict_flops"] / (prof["predict_ms"] * 1e-3) / 1e12
           if prof["predict_ms"] > 0 else None,
           "k_cross_cov_GBps": prof["predict_cov_bytes"] / (prof["predict_cov_ms"] * 1e-3) / 1e9
           if prof["predict_cov_ms"] > 0 else None,
           "k_cross_cov_hbm_frac": prof["predict_cov_bytes"] / (prof["predict_cov_ms"] * 1e-3) / 8e12
           if prof["predict_cov_ms"] > 0 else None,
           "other_ms_profiled": pdt * 1e3 - prof["factor_wall_ms"] - prof["predict_ms"] - prof["predict_cov_ms"],
           "note": "ms: wall time of unprofiled calls (median of 5) including the single-particle factorisation "
                   "and the host<->device copies; the kernel times come from a separate profiled pass"}
    if out["factor_ms"] > 0:
        out["factor_tflops"] = out["factor_flops"] / (out["factor_ms"] * 1e-3) / 1e12
    if not args.no_cpu and args.cpu_predict_points > 0:
        from oracle import ref_cpu  # CPU baseline leg only
        m = args.cpu_predict_points
        t1 = time.perf_counter()
        ref_cpu.GP(x, y, e, xf[:, :m], ls, batch_size=10000)
        cdt = time.perf_counter() - t1
        out["cpu_baseline"] = {"points_per_s": m / cdt, "sample": f"oracle GP (GP_func.py:12-45 restated) on {m} "
                               f"query points, 1 core", "cores": 1, "blas_threads": blas_threads(), "s": cdt}
    return out


def hull_line(ctx, args):
    """Secondary measurement, SURVEY.md §8f row 3: the prediction grid of GP_fit.py:31
    (convex_hull.fill_convex_hull) for 2-D and 3-D hulls; the facet rasterisation stays on
    the host, the d fill passes run on the GPU (gpf_hull_fill)."""
    sys.path.insert(0, str(ROOT / "gaussian-process_amd"))
    import convex_hull
    rng = np.random.default_rng(args.seed + 3)
    cases = [("2-D, 21 points, res 0.005", rng.uniform([1.2, -1.0], [2.0, 1.0], size=(21, 2)), [0.005, 0.005]),
             ("3-D, 12 points, res 0.02", rng.uniform(0.0, 1.0, size=(12, 3)), [0.02, 0.02, 0.02])]
    out = []
    for name, pts, res in cases:
        convex_hull.fill_convex_hull(pts, res)  # warm-up
        t0 = time.perf_counter()
        g = convex_hull.fill_convex_hull(pts, res)
        dt = time.perf_counter() - t0
        item = {"case": name, "grid_points": int(g.shape[0]), "ms": dt * 1e3, "points_per_s": g.shape[0] / dt}
        if not args.no_cpu:
            from oracle import ref_hull  # CPU baseline leg only
            t1 = time.perf_counter()
            ref = ref_hull.fill_convex_hull(pts, res)
            cdt = time.perf_counter() - t1
            item["cpu_baseline"] = {"ms": cdt * 1e3, "kind": "port", "cores": 1,
                                    "sample": "oracle/ref_hull.py (convex_hull.py restated, pure Python), full case"}
            item["identical"] = bool(np.array_equal(ref, g))
        out.append(item)
    return out


def kmeans_line(ctx, args):
    """Secondary measurement, SURVEY.md §8f row 2: the KMeans subsample of len_scale_opt
    (find_len_scales.py:25-47) at config E's size (N=16384, d=4 -> 100 points): the fit with its
    Lloyd E/M-steps on the GPU (gpfit.kmeans; sklearn's seeding on the host) beside sklearn's own
    KMeans.fit (the reference's call) on the host, both timed whole, labels compared."""
    from sklearn.cluster import KMeans
    from gpfit.kmeans import kmeans_fit
    rng = np.random.default_rng(args.seed + 5)
    X = rng.uniform(size=(16384, 4))
    kmeans_fit(ctx, X[:2048], 100)  # warm-up (first launches, sklearn import)
    t0 = time.perf_counter()
    labels, _ = kmeans_fit(ctx, X, 100)
    gdt = time.perf_counter() - t0
    out = {"N": 16384, "d": 4, "clusters": 100, "ms": gdt * 1e3,
           "note": "GPU: the Lloyd iterations' E/M-steps (gpf_kmeans_step); host: k-means++ seeding (sklearn) "
                   "and the O(k d) loop bookkeeping"}
    if not args.no_cpu:
        KMeans(n_clusters=100, n_init="auto", random_state=0).fit(X[:2048])
        t1 = time.perf_counter()
        km = KMeans(n_clusters=100, n_init="auto", random_state=0).fit(X)
        cdt = time.perf_counter() - t1
        out["cpu_baseline"] = {"ms": cdt * 1e3, "kind": "reference call", "threads": "sklearn/OpenMP default",
                               "sample": "sklearn KMeans(100, n_init='auto', random_state=0).fit, the full case"}
        out["labels_equal"] = bool(np.array_equal(labels, km.labels_))
        out["iterations_sklearn"] = int(km.n_iter_)
    return out


def psurf_line(ctx, args):
    """Secondary measurement, SURVEY.md §8f row 4: probability surface of a merged frame of
    `psurf_rows` grid rows x 4 experiments (calc_prob_surf.py:15-30,67-81), kernel time from
    HIP events; HBM roofline on its algorithmic bytes (tails read + 2 x 100 doubles written)."""
    M, E = args.psurf_rows, 8
    rng = np.random.default_rng(args.seed + 5)
    tails = np.empty((M, E))
    tails[:, 0::2] = rng.normal(size=(M, E // 2))
    tails[:, 1::2] = rng.uniform(0.05, 0.5, size=(M, E // 2))
    tails[rng.uniform(size=M) < 0.1, 6:] = np.inf  # some rows miss an experiment
    ctx.prob_surface(tails[:1000])
    ctx.reset_profile()
    ctx.set_profiling(True)
    t0 = time.perf_counter()
    _, p, ok = ctx.prob_surface(tails)
    dt = time.perf_counter() - t0
    prof = ctx.profile()
    ctx.set_profiling(False)
    kms = prof["psurf_ms"]
    out = {"rows": M, "experiments": E // 2, "wall_ms": dt * 1e3, "kernel_ms": kms,
           "rows_per_s_kernel": M / (kms * 1e-3) if kms > 0 else None, "rows_per_s_wall": M / dt,
           "kernel_GBps": prof["psurf_bytes"] / (kms * 1e-3) / 1e9 if kms > 0 else None,
           "hbm_peak_GBps": 8000.0,
           "note": "wall includes host<->device copies of the tails and of y, p (PCIe); kernel = row setup + "
                   "grid/probability kernel"}
    pmc = secondary_pmc()
    if pmc and pmc[0].get("k_prob_surf", {}).get("valu_busy_pct"):
        # VALU roofline: the kernels issue erf/erfc and division sequences, not HBM traffic; frac
        # = the fraction of cycles the vector ALUs were issuing (rocprofv3 PMC of the same call)
        k = pmc[0]["k_prob_surf"]
        out["roofline"] = {"bound": "valu", "frac": k["valu_busy_pct"] / 100.0,
                           "achieved_fp64_TFLOPs": k.get("fp64_tflops"), "valu_insts_per_simd": k.get("valu_insts_per_simd"),
                           "kernel_ns": k.get("avg_ns"), "source": pmc[1],
                           "note": "frac = SQ_ACTIVE_INST_VALU x 4 / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs)"}
    if not args.no_cpu:
        from oracle import ref_cpu  # CPU baseline leg only
        m = 2000
        vals = np.concatenate([np.zeros((m, 2)), tails[:m]], axis=1)
        t1 = time.perf_counter()
        ref_cpu.prob_surface(vals, 2)
        cdt = time.perf_counter() - t1
        out["cpu_baseline"] = {"rows_per_s": m / cdt, "sample": f"oracle prob_surface (calc_prob_surf.py "
                               f"restated: numpy + scipy.stats.norm) on {m} rows, 1 core", "s": cdt}
    return out


SECONDARY_CONFIGS = (
    # (letter, N, d, particles, seed, hetero, warmup, steps): the other single-GPU BASELINE configs
    # (BASELINE.json configs 1, 3 and 4 at one GPU's share, SURVEY.md §8d seeds), timed like the
    # headline (no HIP events in the stream, interior particles l ~ U[0.05, 0.6]^d)
    ("B", 1024, 2, 32, 0, False, 5, 200),
    ("D-share", 4096, 3, 32, 1, False, 2, 40),   # the per-GPU load of every rank of the N>1 runs
    ("E-share", 16384, 4, 16, 1, True, 1, 3),    # config E's 128 particles over 8 GPUs
)


def secondary_configs(ctx, args, peak):
    """Secondary lines: B, D's per-GPU share and E's per-GPU share on this GPU (find_len_scales.py:
    102-104 at each size). frac = evals/s x (2/3) Npad^3 / the FP64 MFMA peak (whole-step rate,
    everything in the step counted against the factorisation's flops)."""
    from gpfit.swarm import search_bounds, sigma_grid
    out = []
    for name, N, d, P, seed, hetero, warm, steps in SECONDARY_CONFIGS:
        if args.steps < 20:  # a short debug run keeps the secondary lines short too
            steps = max(1, min(steps, args.steps))
        x, y, e = synthetic(N, d, seed, hetero)
        lo, hi = search_bounds(x)
        s, ex = sigma_grid()
        ctx.set_data(x, y, e)
        ctx.set_grid(s, ex, lo, hi)
        rng = np.random.default_rng(seed + 2000)
        for _ in range(warm):
            ctx.eval_batch(rng.uniform(0.05, 0.6, size=(P, d)))
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            ctx.eval_batch(rng.uniform(0.05, 0.6, size=(P, d)))
        ctx.synchronize()
        dt = time.perf_counter() - t0
        v = P * steps / dt
        fl = (2.0 / 3.0) * float(-(-N // 128) * 128) ** 3
        out.append({"config": name, "N": N, "d": d, "particles": P, "hetero_noise": hetero, "seed": seed,
                    "steps": steps, "warmup": warm, "value": v, "unit": "evals/s", "ms_per_step": dt / steps * 1e3,
                    "achieved_tflops": v * fl / 1e12, "frac": v * fl / 1e12 / FP64_MFMA_PEAK_TFLOPS,
                    "frac_of_box_ceiling": (v * fl / 1e12 / peak) if peak else None,
                    "flops_per_eval": fl, "formulation": "potrf+trtri (2/3 Npad^3 per eval)"})
    return out


def launch_ranks(n):
    """`--gpus N` without a launcher: start the N rank processes (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set, one GPU each) before this process touches any GPU, and exit
    with their status. Only rank 0 prints the JSON line."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc != 0), 0)


def open_exchange(ctx, world, rank):
    """The measured run's swarm exchange: libgpfit's RCCL communicator on this rank's GPU.

    A host-transport side channel (TCP rendezvous, no device) first lets the ranks agree on
    whether every rank opened RCCL; if any could not, all ranks use the host transport for the
    (P + G)-double exchange and the JSON line says so (`exchange`), so a scaling run still
    measures the sharded factorisations. GPF_COMM_TRANSPORT=host skips RCCL."""
    import gpfit
    base = int(os.environ.get("GPF_COMM_PORT", int(os.environ.get("MASTER_PORT", "29599")) + 1))
    side = gpfit.Comm(rank, world, os.environ.get("MASTER_ADDR", "127.0.0.1"), base + 16, "host")
    if os.environ.get("GPF_COMM_TRANSPORT", "rccl") == "host":
        return side, {"transport": "host"}
    rccl, err = None, ""
    try:
        rccl = gpfit.Comm.from_env(ctx, transport="rccl")
    except gpfit.GPFitError as exc:  # reported below, on every rank's behalf by rank 0
        err = str(exc)[:400]
    if int(side.allreduce([1.0 if rccl is not None else 0.0])[0]) == world:
        side.close()
        return rccl, {"transport": "rccl"}
    if rccl is not None:
        rccl.close()
    why = err or "another rank could not open RCCL"
    if rank == 0:
        print(f"bench.py: RCCL unavailable on this node ({why}); the swarm exchange runs over the host "
              f"transport and the JSON line says so (rccl: false)", file=sys.stderr, flush=True)
    return side, {"transport": "host", "rccl_error": why}


def plumbing(args, world, rank):
    """CPU-only check of the multi-rank plumbing (`--plumbing`): the rank processes, the
    library's host-transport communicator, the barrier and the max-over-ranks timing, with a
    trivial stand-in score (no GP, no GPU). Prints n_gpus and the rank count; no measurement."""
    import gpfit
    comm = gpfit.Comm.from_env(transport="host") if world > 1 else None
    P = (args.swarm_per_gpu or (64 if world == 1 else 32)) * world
    pos = np.random.default_rng(args.seed).uniform(0.05, 0.6, size=(P, args.d))
    lo_r, hi_r = rank * P // world, (rank + 1) * P // world
    t0 = time.perf_counter()
    local = np.sum(pos[lo_r:hi_r] ** 2, axis=1)
    full = comm.exchange_scores(P, local) if comm else local
    dt = time.perf_counter() - t0
    xms = comm.stats()[0] if comm else 0.0
    ranks = int(comm.allreduce([1.0])[0]) if comm else 1
    dt = float(comm.allreduce([dt], op="max")[0]) if comm else dt
    xms = float(comm.allreduce([xms], op="max")[0]) if comm else 0.0
    if rank == 0:
        print(json.dumps({"metric": "plumbing check (no GPU work)", "value": None, "unit": None, "n_gpus": world,
                          "ranks_joined": ranks, "swarm": P, "scores_ok": bool(np.array_equal(full, np.sum(pos ** 2, axis=1))),
                          "ms": dt * 1e3, "rccl": False, "exchange": {"transport": "host"} if comm else None,
                          "exchange_ms_per_step": xms if comm else None}), flush=True)
    if comm:
        comm.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default: ~9 s of timed GPU work at config C, twice (the value pass and the profiled pass): the
    # round-2 default (60 steps, ~3 s) left the driver's ~5 s SMI sampler with no busy sample
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--d", type=int, default=3)
    ap.add_argument("--swarm-per-gpu", type=int, default=None,
                    help="particles per GPU (default 64 on one GPU = config C, 32 per GPU at N > 1 = config D)")
    ap.add_argument("--hetero", action="store_true")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="do not bracket launches with HIP events")
    ap.add_argument("--pso-steps", type=int, default=3, help="secondary: real PSO iterations timed")
    ap.add_argument("--predict-points", type=int, default=10000,
                    help="secondary (SURVEY.md §8f row 1): GP prediction at this many query points, 0 = skip")
    ap.add_argument("--cpu-predict-points", type=int, default=256, help="CPU GP sample for the prediction line")
    ap.add_argument("--no-hull", action="store_true", help="skip the convex-hull grid line (SURVEY.md §8f row 3)")
    ap.add_argument("--no-kmeans", action="store_true", help="skip the KMeans subsample line (SURVEY.md §8f row 2)")
    ap.add_argument("--psurf-rows", type=int, default=100000,
                    help="secondary (SURVEY.md §8f row 4): probability-surface rows, 0 = skip")
    ap.add_argument("--plumbing", action="store_true", help="CPU-only multi-rank plumbing check (no measurement)")
    ap.add_argument("--no-secondary", action="store_true", help="skip the B / D-share / E-share lines")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)", file=sys.stderr)
        sys.exit(2)
    if args.plumbing:
        plumbing(args, world, rank)
        return

    import gpfit
    from gpfit.swarm import Swarm, centred_lhs, make_scorer, search_bounds, sigma_grid  # noqa: F401

    N, d = args.n, args.d
    spg = args.swarm_per_gpu or (64 if world == 1 else 32)
    x, y, e = synthetic(N, d, args.seed, args.hetero)
    lo, hi = search_bounds(x)
    s, ex = sigma_grid()
    P = spg * world

    # one GPU per rank (LOCAL_RANK); GPFIT_DEVICE pins every rank to one device, for rehearsing
    # the multi-rank path on a one-GPU box with GPF_COMM_TRANSPORT=host (RCCL needs a GPU per rank)
    ctx = gpfit.Context(int(os.environ.get("GPFIT_DEVICE", local)))
    comm, exchange = open_exchange(ctx, world, rank) if world > 1 else (None, None)  # RCCL on this rank's GPU
    score = make_scorer(x, y, e, s, ex, lo, hi, ctx=ctx, comm=comm)
    rng = np.random.default_rng(args.seed + 1000)  # identical on every rank

    def batch():
        # SURVEY.md §8d fixed-work variant: interior particles l ~ U[0.05, 0.6]^d,
        # so every evaluation is a full factorise + score (no sentinel short-cuts)
        return rng.uniform(0.05, 0.6, size=(P, d))

    def fence():
        ctx.synchronize()  # device-wide (hipDeviceSynchronize): the torch.cuda.synchronize() role
        if comm is not None:
            comm.barrier()

    for _ in range(args.warmup):
        score(batch())

    # `value`: K steps with no HIP events in the stream (recording an event pair around every
    # launch costs the latency-bound configs real time: config B 31.8k vs 29.0k evals/s, C +0.8%;
    # profiles/r3/ab_profiling_overhead.txt); the roofline and the per-kernel breakdown come from
    # a second timed pass of the same K steps with an event pair around every launch
    ctx.set_profiling(False)
    fence()
    x0 = comm.stats()[0] if comm is not None else 0.0
    t0 = time.perf_counter()
    best = np.inf
    for _ in range(args.steps):
        sc = score(batch())
        best = min(best, float(sc[np.argmin(sc)]))
    fence()
    dt = time.perf_counter() - t0
    xch = (comm.stats()[0] - x0) / args.steps if comm is not None else None  # exchange ms per step, this rank
    dt_prof = None
    ctx.reset_profile()
    if not args.no_profile:
        ctx.set_profiling(True)
        ctx.reset_profile()
        fence()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            score(batch())
        fence()
        dt_prof = time.perf_counter() - t1
    prof = ctx.profile()
    ctx.set_profiling(False)
    if comm is not None:
        dt = float(comm.allreduce([dt], op="max")[0])  # max over ranks
        xch_max = float(comm.allreduce([xch], op="max")[0])
        xch_min = -float(comm.allreduce([-xch], op="max")[0])
        if dt_prof is not None:
            dt_prof = float(comm.allreduce([dt_prof], op="max")[0])
    evals = P * args.steps                # swarm x iterations, all of them full evaluations
    value = evals / dt

    # secondary: the real PSO update loop (find_len_scales.py:87-141) from a centred LHS;
    # particles clipped onto the box are sentinels (1e13, no GPU work), so its rate is higher
    pso = None
    if args.pso_steps > 0:
        np.random.seed(args.seed)
        sw = Swarm(centred_lhs(lo, hi, P, args.seed), lo, hi, score, progress=False, verbose=False)
        ctx.reset_profile()
        ctx.set_profiling(True)
        fence()
        t1 = time.perf_counter()
        e0 = sw.evals
        for i in range(args.pso_steps):
            sw.step(i)
        fence()
        pdt = time.perf_counter() - t1
        live = ctx.profile()["evals"]
        ctx.set_profiling(False)
        if comm is not None:
            pdt = float(comm.allreduce([pdt], op="max")[0])
        pso = {"iters": args.pso_steps, "evals_per_s": (sw.evals - e0) / pdt,
               "iters_per_s": args.pso_steps / pdt,
               "live_fraction_rank0": live / max(1, (sw.evals - e0) / world)}

    # roofline of the dominant kernel, from HIP events on the library's streams
    plan = gpfit.plan_check(spg, -(-N // 128))
    groups = plan["groups"]
    persistent = bool(plan["persistent"])
    if persistent:
        # one k_factor launch per batch covers every block column of every particle (block 0 is
        # k_diag's, the diagonal blocks' K entries k_build_cov's)
        achieved = prof["panel_flops"] / (prof["panel_ms"] * 1e-3) / 1e12 if prof["panel_ms"] > 0 else None
        timing = ("k_factor launch (the persistent factorisation: one launch per batch, every block column of "
                  "every particle), HIP events on the library stream")
    elif groups == 1:
        # one stream: the launches do not overlap, per-launch event time is exact
        achieved = prof["panel_flops"] / (prof["panel_ms"] * 1e-3) / 1e12 if prof["panel_ms"] > 0 else None
        timing = "k_step launch average (HIP events on the library stream)"
    else:
        # concurrent particle-group streams: per-launch windows overlap, so rate the whole
        # factorisation phase (its wall time, all groups) on the k_step + diagonal flops
        fl = prof["panel_flops"] + prof["diag_flops"]
        achieved = fl / (prof["factor_wall_ms"] * 1e-3) / 1e12 if prof["factor_wall_ms"] > 0 else None
        timing = f"factorisation-phase wall over {groups} concurrent group streams (non-overlapping)"
    # practical ceiling: the same GEMM core alone on L-tile-shaped operands (gpf_gemm_bench,
    # direct-to-LDS, N=4096-sized panels, depth 1920, 1024 workgroups = two whole rounds of the
    # 512 slots; r1-r5's 960 workgroups left 64 slots idle in the second round and read the core
    # ~6% low per clock, profiles/r5/core_geometry.txt), on non-zero operand data
    # (r4: the MFMA's power depends on its operand bits — on zero operands the chip held ~2.39 GHz,
    # on real data ~2.09 GHz, profiles/r4/clock_probe_*.json), sustained for ~0.3 s so the clock
    # has settled (a 3-launch run starts below it)
    core = ctx.gemm_bench(mode=2, npad=4096, particles=64, tiles=16, depth=1920, iters=300) \
        if (rank == 0 and N >= 2048) else None
    core_sclk = ctx.bench_clock() if core else None
    # this box's FP64 matrix ceiling: back-to-back independent v_mfma_f64_16x16x4 chains on every
    # SIMD (gpf_mfma_peak), at whatever clock the chip holds under that load; boxes of the pool
    # differ, so fractions against it are checkable per box
    box_peak = ctx.mfma_peak(blocks=1024, iters=8192) if rank == 0 else None
    peak_sclk = ctx.bench_clock() if box_peak else None
    traffic = pmc_traffic(N, d, spg, "k_factor" if persistent else "k_step")
    roof = {"kernel": "k_factor" if persistent else "k_step", "bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": (achieved / FP64_MFMA_PEAK_TFLOPS) if achieved else None,
            "traffic": traffic["bytes_per_launch"] if traffic else None,
            "traffic_source": traffic["source"] if traffic else None,
            # per k_step launch, like flops_per_launch: with particle groups a launch covers one
            # group's particles (the PMC pass ran the same schedule)
            "traffic_per": ("k_factor launch (one per batch)" if persistent else
                            f"k_step launch of one of {traffic['groups']} particle groups"
                            if traffic["groups"] > 1 else "k_step launch") if traffic else None,
            "timing": timing + "; measured over a second timed pass of the same steps with an event pair "
                               "around every launch (the `value` pass records no events)",
            "ms_per_step_profiled_pass": dt_prof / args.steps * 1e3 if dt_prof else None,
            "particle_groups": groups,
            "persistent": persistent,
            # this box: the shader clock the factor kernels held (in-kernel s_memtime / s_memrealtime
            # spans of every workgroup, profiled pass) and the FP64 matrix ceiling at that clock
            # (128 flop per CU per clock; 78.6 TF/s is the 2.4 GHz spec); and a dense MFMA loop's rate
            # (gpf_mfma_peak: power-bound, it throttles the clock well below what k_step runs at)
            "box_sclk_mhz": prof["factor_sclk_mhz"] or None,
            "box_fp64_ceiling_tflops": prof["fp64_ceiling_at_sclk_tflops"] or None,
            "frac_of_box_ceiling": (achieved / prof["fp64_ceiling_at_sclk_tflops"])
            if (achieved and prof["fp64_ceiling_at_sclk_tflops"]) else None,
            "box_dense_mfma_loop_tflops": box_peak,
            "box_dense_mfma_loop_sclk_mhz": peak_sclk or None,
            "gemm_core_tflops": core,
            "gemm_core_sclk_mhz": core_sclk or None,
            "frac_of_gemm_core": (achieved / core) if (achieved and core) else None,
            # per clock: achieved / (128 flop/CU/clock x CUs x the clock each one held)
            "gemm_core_frac_of_its_clock_ceiling": (core / (FP64_MFMA_PEAK_TFLOPS * core_sclk / 2400.0))
            if (core and core_sclk) else None,
            "dense_mfma_loop_frac_of_its_clock_ceiling": (box_peak / (FP64_MFMA_PEAK_TFLOPS * peak_sclk / 2400.0))
            if (box_peak and peak_sclk) else None,
            "launches": prof["panel_launches"], "avg_launch_ms": prof["panel_ms"] / max(prof["panel_launches"], 1),
            "flops_per_launch": prof["panel_flops"] / max(prof["panel_launches"], 1),
            "formulation": "potrf+trtri (2/3 N^3 per eval)",
            "factor_phase_tflops": (prof["factor_flops"] / (prof["factor_wall_ms"] * 1e-3) / 1e12)
            if prof["factor_wall_ms"] > 0 else None}
    # each rank's factorisation-phase rate (profiled pass), so a scaling line shows imbalance too
    ftf = roof["factor_phase_tflops"] or 0.0
    ftf_max = ftf_min = ftf
    if comm is not None:
        ftf_max = float(comm.allreduce([ftf], op="max")[0])
        ftf_min = -float(comm.allreduce([-ftf], op="max")[0])
    build_gbs = (prof["build_bytes"] / (prof["build_ms"] * 1e-3) / 1e9) if prof["build_ms"] > 0 else None
    breakdown = {k: prof[k] for k in ("panel_ms", "diag_ms", "build_ms", "loss_ms", "factor_wall_ms")}
    # k_build_cov writes only the 128-wide diagonal blocks (3 nt 64x64 tiles per particle): the
    # off-diagonal K tiles are generated inside k_step's accumulators (cov_tile_acc) and never
    # written, so this is not a whole-K build rate
    breakdown["k_build_cov_diag_blocks_GBps"] = build_gbs
    breakdown["k_build_cov_scope"] = "diagonal 128-blocks only; off-diagonal K tiles are built inside k_step"

    breakdown["evals_on_gpu"] = prof["evals"]

    cpu = None
    predict = None
    # secondary lines and the CPU baseline: single-GPU runs only (rank 0 at N=1); a multi-GPU
    # run reports the headline metric alone
    solo = world == 1
    if solo and args.predict_points > 0:
        predict = predict_line(ctx, x, y, e, N, d, args)
    psurf = None
    if solo and args.psurf_rows > 0:
        psurf = psurf_line(ctx, args)
    hull = None
    if solo and not args.no_hull:
        hull = hull_line(ctx, args)
    kmeans = None
    if solo and not args.no_kmeans:
        kmeans = kmeans_line(ctx, args)
    secondary = None
    if solo and not args.no_secondary:
        secondary = secondary_configs(ctx, args, prof["fp64_ceiling_at_sclk_tflops"] or None)
    if solo and not args.no_cpu:
        cpu = cpu_baselines(x, y, e, lo, hi, N, d, args.seed)

    if rank == 0:
        letter = config_letter(N, d, spg, args.hetero)
        line = {
            "metric": f"PSO objective evals/sec (swarm x iters) at N={N} d={d}",
            "value": value, "unit": "evals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": (value / cpu["value"]) if cpu else None,
            "vs_baseline_basis": "GPU value / CPU reference-policy baseline (cpu_baseline.value) on this box"
            if cpu else None,
            "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"PSO objective, BASELINE config {letter}: synthetic N={N} d={d}, "
                                   f"swarm {spg}/GPU x {world} GPU = {P}",
                       "N": N, "d": d, "swarm": P, "swarm_per_gpu": spg, "global_batch": P, "seq_len": N,
                       "parallelism": (f"swarm-shard x{world} (libgpfit {exchange['transport'].upper()} all-reduce)"
                                       if world > 1 else "single GPU"),
                       "hetero_noise": bool(args.hetero),
                       "pso_iters_per_s": args.steps / dt, "particles": "interior l~U[0.05,0.6]^d (full work)"},
            "configs": secondary,
            "pso_loop": pso,
            "predict": predict,
            "prob_surface": psurf,
            "hull_grid": hull,
            "kmeans": kmeans,
            "roofline": roof,
            "cpu_baseline": cpu,
            "gpu_vs_cpu": (value / cpu["value"]) if cpu else None,
            "gpu_vs_cpu_all_cores": (value / cpu["all_cores"]["value"]) if cpu else None,
            "breakdown_ms": breakdown,
            "build": gpfit.build_info(),
            "exchange": exchange,
            # the swarm exchange's own cost (time inside gpf_comm_exchange_scores per step: the
            # all-reduce of P + G doubles, including the wait for the slowest rank), max and min
            # over ranks; the min is the collective itself, the max adds the load imbalance
            "rccl": (exchange["transport"] == "rccl") if exchange else None,
            "exchange_ms_per_step": xch_max if comm is not None else None,
            "exchange_ms_per_step_min_rank": xch_min if comm is not None else None,
            "factor_tflops_rank_max": ftf_max if comm is not None else None,
            "factor_tflops_rank_min": ftf_min if comm is not None else None,
        }
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    ctx.close()


if __name__ == "__main__":
    main()
