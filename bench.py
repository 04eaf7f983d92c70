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

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 4096] [--d 3] [--swarm-per-gpu 64]
                    [--cpu-sample 8] [--cpu-workers 8] [--no-cpu]

Prints ONE JSON line on rank 0 (contract in the task statement), with a
"roofline" object for the dominant kernel (k_panel, the MFMA GEMM step) timed
with HIP events on the library's stream, and a "cpu_baseline" object: the
CPU oracle (a bit-exact NumPy restatement of the reference's evaluate_loss)
timed on this host's cores on a bounded sample of the same workload.
"""
from __future__ import annotations

import os

# BLAS pins must precede numpy (SURVEY.md §6 gotcha) — the CPU baseline runs
# one single-threaded evaluation per worker, exactly as the reference's pool.
os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")

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


def pmc_traffic(N, d, swarm):
    """HBM bytes per k_step launch from the committed rocprofv3 PMC passes
    (scripts/pmc_traffic.py writes profiles/<round>/k_step_traffic.json), or None."""
    best = None
    for f in sorted((ROOT / "profiles").glob("*/k_step_traffic.json")):
        try:
            t = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        if t.get("N") == N and t.get("d") == d and t.get("swarm") == swarm:
            best = {"bytes_per_launch": t["bytes_per_launch"], "source": str(f.relative_to(ROOT))}
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


def cpu_baseline(x, y, e, positions, lo, hi, workers):
    """Reference-policy CPU path: fork pool, one BLAS thread per worker."""
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


def predict_line(ctx, x, y, e, N, d, args):
    """Secondary measurement, SURVEY.md §8f row 1: GP(x, y, e, x_fit, l) at M query
    points (GP_fit.py:32 -> GP_func.py:12-45): one factorisation, then the
    cross-covariance build and V = U K_s reduced to column sums of squares."""
    M = args.predict_points
    rng = np.random.default_rng(args.seed + 99)
    xf = rng.uniform(size=(d, M))
    ls = np.full(d, 0.3)
    ctx.predict(ls, xf)  # warm-up (workspace, code objects)
    ctx.reset_profile()
    ctx.set_profiling(True)
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.predict(ls, xf)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    prof = ctx.profile()
    ctx.set_profiling(False)
    out = {"N": N, "d": d, "M": M, "ms": dt * 1e3, "points_per_s": M / dt,
           "factor_ms": prof["factor_wall_ms"],
           "k_predict_vsq_ms": prof["predict_ms"],
           "k_predict_vsq_tflops": prof["predict_flops"] / (prof["predict_ms"] * 1e-3) / 1e12
           if prof["predict_ms"] > 0 else None,
           "k_cross_cov_GBps": prof["predict_cov_bytes"] / (prof["predict_cov_ms"] * 1e-3) / 1e9
           if prof["predict_cov_ms"] > 0 else None,
           "note": "wall time includes the single-particle factorisation and host<->device copies"}
    if not args.no_cpu and args.cpu_predict_points > 0:
        from oracle import ref_cpu  # CPU baseline leg only
        m = args.cpu_predict_points
        t1 = time.perf_counter()
        ref_cpu.GP(x, y, e, xf[:, :m], ls, batch_size=10000)
        cdt = time.perf_counter() - t1
        out["cpu_baseline"] = {"points_per_s": m / cdt, "sample": f"oracle GP (GP_func.py:12-45 restated) on {m} "
                               f"query points, host BLAS threads={os.environ.get('OMP_NUM_THREADS')}", "s": cdt}
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
           "note": "wall includes host<->device copies of the tails and of y, p (PCIe)"}
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--d", type=int, default=3)
    ap.add_argument("--swarm-per-gpu", type=int, default=64)
    ap.add_argument("--hetero", action="store_true")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-sample", type=int, default=8)
    ap.add_argument("--cpu-workers", type=int, default=8)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="do not bracket launches with HIP events")
    ap.add_argument("--pso-steps", type=int, default=3, help="secondary: real PSO iterations timed")
    ap.add_argument("--predict-points", type=int, default=10000,
                    help="secondary (SURVEY.md §8f row 1): GP prediction at this many query points, 0 = skip")
    ap.add_argument("--cpu-predict-points", type=int, default=256, help="CPU GP sample for the prediction line")
    ap.add_argument("--no-hull", action="store_true", help="skip the convex-hull grid line (SURVEY.md §8f row 3)")
    ap.add_argument("--psurf-rows", type=int, default=100000,
                    help="secondary (SURVEY.md §8f row 4): probability-surface rows, 0 = skip")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import gpfit
    from gpfit.swarm import Swarm, centred_lhs, make_scorer, search_bounds, sigma_grid  # noqa: F401

    N, d = args.n, args.d
    x, y, e = synthetic(N, d, args.seed, args.hetero)
    lo, hi = search_bounds(x)
    s, ex = sigma_grid()
    P = args.swarm_per_gpu * world

    ctx = gpfit.Context(local)
    score = make_scorer(x, y, e, s, ex, lo, hi, ctx=ctx)
    rng = np.random.default_rng(args.seed + 1000)  # identical on every rank

    def batch():
        # SURVEY.md §8d fixed-work variant: interior particles l ~ U[0.05, 0.6]^d,
        # so every evaluation is a full factorise + score (no sentinel short-cuts)
        return rng.uniform(0.05, 0.6, size=(P, d))

    for _ in range(args.warmup):
        score(batch())

    if not args.no_profile:
        ctx.set_profiling(True)
    ctx.reset_profile()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    best = np.inf
    for _ in range(args.steps):
        sc = score(batch())
        best = min(best, float(sc[np.argmin(sc)]))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = ctx.profile()
    ctx.set_profiling(False)

    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
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
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        e0 = sw.evals
        for i in range(args.pso_steps):
            sw.step(i)
        if world > 1:
            dist.barrier()
        pdt = time.perf_counter() - t1
        live = ctx.profile()["evals"]
        ctx.set_profiling(False)
        pso = {"iters": args.pso_steps, "evals_per_s": (sw.evals - e0) / pdt,
               "iters_per_s": args.pso_steps / pdt,
               "live_fraction_rank0": live / max(1, (sw.evals - e0) / world)}

    # roofline of the dominant kernel, from HIP events on the library stream
    achieved = prof["panel_flops"] / (prof["panel_ms"] * 1e-3) / 1e12 if prof["panel_ms"] > 0 else None
    # practical ceiling: the same GEMM core alone on L-tile-shaped operands (gpf_gemm_bench,
    # direct-to-LDS, N=4096-sized panels, depth 2048, 960 workgroups)
    core = ctx.gemm_bench(mode=2, npad=4096, particles=64, tiles=15, depth=2048, iters=3) \
        if (rank == 0 and N >= 2048) else None
    traffic = pmc_traffic(N, d, args.swarm_per_gpu)
    roof = {"kernel": "k_step", "bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": (achieved / FP64_MFMA_PEAK_TFLOPS) if achieved else None,
            "traffic": traffic["bytes_per_launch"] if traffic else None,
            "traffic_source": traffic["source"] if traffic else None,
            "gemm_core_tflops": core,
            "frac_of_gemm_core": (achieved / core) if (achieved and core) else None,
            "launches": prof["panel_launches"], "avg_launch_ms": prof["panel_ms"] / max(prof["panel_launches"], 1),
            "flops_per_launch": prof["panel_flops"] / max(prof["panel_launches"], 1),
            "formulation": "potrf+trtri (2/3 N^3 per eval)",
            "factor_phase_tflops": (prof["factor_flops"] / (prof["factor_wall_ms"] * 1e-3) / 1e12)
            if prof["factor_wall_ms"] > 0 else None}
    build_gbs = (prof["build_bytes"] / (prof["build_ms"] * 1e-3) / 1e9) if prof["build_ms"] > 0 else None
    breakdown = {k: prof[k] for k in ("panel_ms", "diag_ms", "build_ms", "loss_ms")}
    breakdown["k_build_cov_GBps"] = build_gbs
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

    if solo and not args.no_cpu and args.cpu_sample > 0:
        rng = np.random.default_rng(args.seed + 7)
        sample = lo + (hi - lo) * rng.uniform(0.2, 0.8, size=(args.cpu_sample, d))
        workers = max(1, min(args.cpu_workers, args.cpu_sample))
        cv, _, cdt = cpu_baseline(x, y, e, sample, lo, hi, workers)
        cpu = {"value": cv, "unit": "evals/s", "cores": workers, "kind": "port",
               "sample": f"{args.cpu_sample} evaluate_loss calls (oracle/ref_cpu.py, same NumPy/LAPACK calls as "
                         f"find_len_scales.py:154-182) at N={N} d={d} on the same synthetic data, fork pool of "
                         f"{workers} single-BLAS-thread workers, {cdt:.1f} s wall",
               "host_cpu_count": os.cpu_count()}

    if rank == 0:
        line = {
            "metric": f"PSO objective evals/sec (swarm x iters) at N={N} d={d}",
            "value": value, "unit": "evals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"PSO objective, BASELINE config {config_letter(N, d, args.swarm_per_gpu, args.hetero)}: "
                                   f"synthetic N={N} d={d}, swarm {args.swarm_per_gpu}/GPU",
                       "N": N, "d": d, "swarm": P, "global_batch": P, "seq_len": N,
                       "parallelism": f"swarm-shard x{world}", "hetero_noise": bool(args.hetero),
                       "pso_iters_per_s": args.steps / dt, "particles": "interior l~U[0.05,0.6]^d (full work)"},
            "pso_loop": pso,
            "predict": predict,
            "prob_surface": psurf,
            "hull_grid": hull,
            "roofline": roof,
            "cpu_baseline": cpu,
            "gpu_vs_cpu": (value / cpu["value"]) if cpu else None,
            "breakdown_ms": breakdown,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
