"""The N>1 path: swarm rows sharded over ranks, one exchange per batch, inside libgpfit.

Ranks are processes (spawn) joined by the library's own communicator (gpf_comm_open,
include/gpfit.h). On CPU the host transport carries the exchange (the same C protocol the
RCCL transport runs on GPUs: gpf_comm_exchange_scores) and the objective is the injected
checker, so no GPU is needed. The sharded trajectory must equal the single-rank reference
trajectory (F4, produced by the reference's own len_scale_opt) bit for bit on every rank
(SURVEY.md §8e), with every particle scored exactly once across the ranks.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port, **extra):
    os.environ.update(MASTER_ADDR="127.0.0.1", GPF_COMM_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", GPF_COMM_TIMEOUT_S="120", **extra)
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]


def _worker(rank, world, port, path, k, q):
    _env(rank, world, port, GPF_COMM_TRANSPORT="host")
    import contextlib
    import io
    from gpfit.swarm import particle_swarm
    from oracle import ref_cpu
    f4 = np.load(path, allow_pickle=False)
    x = np.asfortranarray(f4[f"c{k}_x"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        best, info = particle_swarm(x, f4[f"c{k}_y"], f4[f"c{k}_e"], True, init_positions=f4[f"c{k}_init"],
                                    seed=int(f4[f"c{k}_seed"]),
                                    evaluator=lambda args: [ref_cpu.evaluate_loss_helper(a) for a in args])
    q.put((rank, best.tolist(), buf.getvalue(), info["local_evals"], info["evals"]))


def _spawn(target, world, *args, timeout=300):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=timeout) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return sorted(res)


@pytest.mark.parametrize("world,k", [(2, 0), (3, 1), (8, 0)])
def test_sharded_swarm_matches_single_rank(world, k):
    from conftest import GOLDEN
    f4 = np.load(GOLDEN / "f4_pso_trace.npz", allow_pickle=False)
    res = _spawn(_worker, world, str(GOLDEN / "f4_pso_trace.npz"), k)
    total_local = 0
    for rank, best, log, local, evals in res:
        assert np.array_equal(np.array(best), f4[f"c{k}_best"]), rank
        assert log == str(f4[f"c{k}_log"]), rank
        total_local += local
    assert total_local == res[0][4]  # every particle scored exactly once across ranks


def _exchange_worker(rank, world, port, q):
    """Protocol checks of gpf_comm_exchange_scores / gpf_comm_allreduce at `world` ranks."""
    _env(rank, world, port)
    import gpfit
    from gpfit._lib import GPF_HIP_ERROR, GPF_NOT_PD
    comm = gpfit.Comm.from_env()
    out = {}
    P = 11
    lo, hi = comm.rows(P)
    full = np.arange(P) * 1.5 + 0.25
    out["scores"] = comm.exchange_scores(P, full[lo:hi]).tolist()
    # a non-PD particle on the last rank (its 2nd row) and on rank 1 (1st row): every rank
    # raises LinAlgError; the smallest failing row is the one reported
    rc = GPF_NOT_PD if rank in (1, world - 1) else 0
    bad = 1 if rank == world - 1 else 0
    try:
        comm.exchange_scores(P, full[lo:hi], rc, bad)
        out["notpd"] = None
    except np.linalg.LinAlgError as e:
        out["notpd"] = e.bad_index
    # a device error on rank 0: every rank raises GPFitError
    try:
        comm.exchange_scores(P, full[lo:hi], GPF_HIP_ERROR if rank == 0 else 0, -1)
        out["hip"] = "no error"
    except gpfit.GPFitError as e:
        out["hip"] = "rank 0 failed" in str(e)
    out["max"] = comm.allreduce([rank, -rank], op="max").tolist()
    out["sum"] = comm.allreduce([1.0, rank]).tolist()
    comm.barrier()
    comm.close()
    q.put((rank, out))


@pytest.mark.parametrize("world", [1, 2, 5])
def test_exchange_protocol(world):
    res = _spawn(_exchange_worker, world, timeout=120)
    P = 11
    for rank, out in res:
        assert out["scores"] == (np.arange(P) * 1.5 + 0.25).tolist()
        rows = [(r * P // world, (r + 1) * P // world) for r in range(world)]
        failing = [rows[r][0] + (1 if r == world - 1 else 0) for r in range(world) if r in (1, world - 1)]
        assert out["notpd"] == min(failing)  # the smallest failing row of the swarm, on every rank
        assert out["hip"] is True
        assert out["max"] == [world - 1, 0]
        assert out["sum"] == [world, world * (world - 1) / 2]


def _injected_notpd_worker(rank, world, port, q):
    """ShardedScorer with an injected evaluator that raises LinAlgError (like numpy's cholesky)
    for particles 5 and 8 of a 10-particle swarm: every rank must report particle 5."""
    _env(rank, world, port)
    import gpfit
    from gpfit.swarm import ShardedScorer
    comm = gpfit.Comm.from_env()
    pos = np.arange(10.0)[:, None] * np.ones((1, 2))

    def backend(rows):
        if np.any(np.isin(rows[:, 0], (5.0, 8.0))):
            raise np.linalg.LinAlgError("Matrix is not positive definite")
        return rows[:, 0] * 2.0

    sc = ShardedScorer(backend, comm=comm)
    ok = sc(pos[[0, 1, 2, 3, 4, 6, 7, 9, 9, 9]]).tolist()
    try:
        sc(pos)
        bad = None
    except np.linalg.LinAlgError as e:
        bad = e.bad_index
    comm.close()
    q.put((rank, ok, bad))


def test_injected_evaluator_reports_the_failing_row():
    """with an injected evaluator the exchange used to report the failing rank's first
    row; the scorer now finds the failing row, so bad_index is the swarm's smallest failing row."""
    res = _spawn(_injected_notpd_worker, 3, timeout=120)
    for rank, ok, bad in res:
        assert ok == [0.0, 2.0, 4.0, 6.0, 8.0, 12.0, 14.0, 18.0, 18.0, 18.0]
        assert bad == 5, rank


def _gpu_worker(rank, world, port, path, k, q):
    """One rank; every rank scores its shard with gpf_eval_batch_sharded on GPU 0 (the host
    transport: RCCL needs one GPU per rank, the driver's 8-GPU run covers it)."""
    _env(rank, world, port, GPFIT_DEVICE="0", GPF_COMM_TRANSPORT="host")
    import contextlib
    import io
    from gpfit.swarm import particle_swarm
    f4 = np.load(path, allow_pickle=False)
    x = np.asfortranarray(f4[f"c{k}_x"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        best, info = particle_swarm(x, f4[f"c{k}_y"], f4[f"c{k}_e"], True, init_positions=f4[f"c{k}_init"],
                                    seed=int(f4[f"c{k}_seed"]), max_iter=150)
    q.put((rank, best.tolist(), buf.getvalue(), info["local_evals"], info["evals"]))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_gpu_swarm_matches_single_rank(world):
    """The multi-rank GPU path (ranks mapped onto the available device): each rank
    scores its rows with gpf_eval_batch_sharded, one exchange per batch; the trajectory on every
    rank equals the single-rank GPU trajectory bit for bit, every particle scored once."""
    from conftest import GOLDEN
    path = str(GOLDEN / "f4_pso_trace.npz")
    one = _spawn(_gpu_worker, 1, path, 0, timeout=600)[0]
    res = _spawn(_gpu_worker, world, path, 0, timeout=600)
    total_local = 0
    for rank, best, log, local, evals in res:
        assert best == one[1], rank
        assert log == one[2], rank
        total_local += local
    assert total_local == res[0][4] == one[4]


@pytest.mark.gpu
def test_rccl_exchange_single_rank():
    """The RCCL transport (ncclCommInitRank + ncclAllReduce on the context's device) at one
    rank, the most the one-GPU box allows: the sharded batch equals the plain batch bit for
    bit, and the all-reduce ops work on device."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process_amd")]
    import gpfit
    from conftest import load_golden
    f2 = load_golden("f2_loss_testfiles.npz")
    ctx = gpfit.Context(0)
    comm = gpfit.Comm(0, 1, transport="rccl", ctx=ctx)
    try:
        ctx.set_data(f2["c0_x"], f2["c0_y"], f2["c0_e"])
        ctx.set_grid(f2["sigma_vals"], f2["expected"], f2["c0_lo"], f2["c0_hi"])
        P = f2["c0_P"]
        np.testing.assert_array_equal(ctx.eval_batch_sharded(comm, P), ctx.eval_batch(P))
        assert comm.allreduce([2.5, -1.0], op="max").tolist() == [2.5, -1.0]
        assert comm.allreduce([2.5, -1.0]).tolist() == [2.5, -1.0]
    finally:
        comm.close()
        ctx.close()


def _rccl_worker(rank, world, port, path, k, q):
    """One rank per GPU over RCCL (the driver's N-GPU bench path): rank r on device r."""
    _env(rank, world, port, GPFIT_DEVICE=str(rank), GPF_COMM_TRANSPORT="rccl")
    import contextlib
    import io
    from gpfit.swarm import particle_swarm
    f4 = np.load(path, allow_pickle=False)
    x = np.asfortranarray(f4[f"c{k}_x"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        best, info = particle_swarm(x, f4[f"c{k}_y"], f4[f"c{k}_e"], True, init_positions=f4[f"c{k}_init"],
                                    seed=int(f4[f"c{k}_seed"]), max_iter=150)
    q.put((rank, best.tolist(), buf.getvalue(), info["local_evals"], info["evals"], info["transport"],
           list(info["exchange"])))


def _visible_gpus():
    """GPUs the ranks could use, counted without importing torch or initialising HIP in the pytest
    parent: the KFD topology's nodes with SIMDs (CPU nodes have none), narrowed by
    HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES when set."""
    import glob
    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            props = dict(line.split()[:2] for line in open(f) if line.strip())
        except (OSError, ValueError):
            continue
        n += int(props.get("simd_count", "0")) > 0
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([t for t in v.split(",") if t.strip()]))
    return n


@pytest.mark.gpu
def test_rccl_sharded_swarm_multi_gpu():
    """RCCL with more than one rank: on a box with G >= 2 GPUs, min(G, 8) ranks,
    one per GPU, each scoring its rows with gpf_eval_batch_sharded and exchanging over RCCL
    (ncclAllReduce over xGMI); every rank's trajectory equals the single-rank GPU run bit for bit,
    every particle scored once, and the exchange timing is recorded. Skipped on one-GPU boxes."""
    n = min(_visible_gpus(), 8)
    if n < 2:
        pytest.skip(f"{n} GPU visible: RCCL across ranks needs one GPU per rank")
    from conftest import GOLDEN
    path = str(GOLDEN / "f4_pso_trace.npz")
    one = _spawn(_gpu_worker, 1, path, 0, timeout=600)[0]
    res = _spawn(_rccl_worker, n, path, 0, timeout=600)
    total_local = 0
    for rank, best, log, local, evals, transport, (ms, count) in res:
        assert best == one[1], rank
        assert log == one[2], rank
        assert transport == "rccl" and count > 0 and ms >= 0.0, (rank, transport, ms, count)
        total_local += local
    assert total_local == res[0][4] == one[4]

