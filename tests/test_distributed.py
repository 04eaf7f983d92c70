"""The N>1 path: swarm rows sharded over ranks with one all-reduce per batch.

world_size 2 over gloo on CPU; the objective is the injected checker so no GPU
is needed. The sharded trajectory must equal the single-rank reference
trajectory bit for bit on every rank.
"""
import os
import socket
import sys

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, k, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "gaussian-process_amd")]
    import io
    import contextlib
    import torch.distributed as dist
    from gpfit.swarm import particle_swarm
    from oracle import ref_cpu
    dist.init_process_group("gloo", rank=rank, world_size=world)
    f4 = np.load(path, allow_pickle=False)
    x = np.asfortranarray(f4[f"c{k}_x"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        best, info = particle_swarm(x, f4[f"c{k}_y"], f4[f"c{k}_e"], True, init_positions=f4[f"c{k}_init"],
                                    seed=int(f4[f"c{k}_seed"]),
                                    evaluator=lambda args: [ref_cpu.evaluate_loss_helper(a) for a in args])
    q.put((rank, best.tolist(), buf.getvalue(), info["local_evals"], info["evals"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k", [(2, 0), (3, 1)])
def test_sharded_swarm_matches_single_rank(world, k):
    import torch.multiprocessing as mp
    from conftest import GOLDEN
    f4 = np.load(GOLDEN / "f4_pso_trace.npz", allow_pickle=False)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(GOLDEN / "f4_pso_trace.npz"), k, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    total_local = 0
    for rank, best, log, local, evals in res:
        assert np.array_equal(np.array(best), f4[f"c{k}_best"]), rank
        assert log == str(f4[f"c{k}_log"]), rank
        total_local += local
    assert total_local == res[0][4]  # every particle scored exactly once across ranks


def _gpu_worker(rank, world, port, path, k, q):
    """One rank of a gloo group; every rank scores its shard with gpf_eval_batch on GPU 0."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      GPFIT_DEVICE="0", OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "gaussian-process_amd")]
    import io
    import contextlib
    import torch  # noqa: F401  (HIP runtime through torch first)
    import torch.distributed as dist
    from gpfit.swarm import particle_swarm
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    f4 = np.load(path, allow_pickle=False)
    x = np.asfortranarray(f4[f"c{k}_x"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        best, info = particle_swarm(x, f4[f"c{k}_y"], f4[f"c{k}_e"], True, init_positions=f4[f"c{k}_init"],
                                    seed=int(f4[f"c{k}_seed"]), max_iter=150)
    q.put((rank, best.tolist(), buf.getvalue(), info["local_evals"], info["evals"]))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _run_ranks(world, k):
    import torch.multiprocessing as mp
    from conftest import GOLDEN
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, str(GOLDEN / "f4_pso_trace.npz"), k, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return sorted(res)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_gpu_swarm_matches_single_rank(world):
    """The multi-rank GPU path (ranks mapped onto the available device): each rank
    scores its rows of the swarm with gpf_eval_batch, one all-reduce per batch; the trajectory
    on every rank equals the single-rank GPU trajectory bit for bit, every particle scored once."""
    one = _run_ranks(1, 0)[0]
    res = _run_ranks(world, 0)
    total_local = 0
    for rank, best, log, local, evals in res:
        assert best == one[1], rank
        assert log == one[2], rank
        total_local += local
    assert total_local == res[0][4] == one[4]
