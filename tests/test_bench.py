"""bench.py's multi-rank launch path on CPU (missing item 3): `--gpus N` without a
launcher starts N rank processes itself, they join libgpfit's communicator (host transport in
the plumbing check; RCCL on GPUs), and rank 0 reports n_gpus = N. No GPU work runs here."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _run(args, env=None, timeout=180):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=str(ROOT))


@pytest.mark.parametrize("n", [2, 4, 8])
def test_gpus_flag_starts_that_many_ranks(n):
    r = _run(["--gpus", str(n), "--plumbing"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["ranks_joined"] == n and out["scores_ok"]
    assert out["swarm"] == 32 * n  # config D's 32 particles per GPU
    # the scaling line describes its exchange: transport, RCCL or not, its cost per step
    assert out["rccl"] is False and out["exchange"] == {"transport": "host"}
    assert out["exchange_ms_per_step"] >= 0.0


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "3", "--plumbing"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "--gpus 3" in r.stderr


@pytest.mark.gpu
def test_multi_rank_bench_on_one_gpu():
    """bench.py --gpus 2 end to end on the GPU box: the rank processes it starts, the library's
    communicator (host transport: RCCL needs one GPU per rank), gpf_eval_batch_sharded on the GPU,
    the barrier and the max-over-ranks timing. Both ranks share device 0 (GPFIT_DEVICE)."""
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--n", "1024", "--d", "2", "--no-cpu",
              "--pso-steps", "1", "--predict-points", "0", "--no-hull", "--psurf-rows", "0"],
             env={"GPFIT_DEVICE": "0", "GPF_COMM_TRANSPORT": "host"}, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["swarm"] == 64 and out["value"] > 0
    assert out["config"]["swarm_per_gpu"] == 32
    assert out["exchange"] == {"transport": "host"} and out["rccl"] is False
    assert 0.0 <= out["exchange_ms_per_step_min_rank"] <= out["exchange_ms_per_step"]
    # per-rank factorisation rates (imbalance of a scaling line)
    assert 0.0 < out["factor_tflops_rank_min"] <= out["factor_tflops_rank_max"]


@pytest.mark.gpu
def test_multi_rank_bench_rccl_agreement_on_one_gpu():
    """bench.py --gpus 2 with the default RCCL exchange, both ranks on device 0: RCCL refuses two
    ranks on one GPU, the ranks agree over the host side channel that RCCL is unavailable and
    all of them run the host-transport exchange; the JSON line records the RCCL error. (On a
    node with a GPU per rank the same agreement keeps RCCL.)"""
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--n", "1024", "--d", "2", "--no-cpu",
              "--pso-steps", "1", "--predict-points", "0", "--no-hull", "--psurf-rows", "0"],
             env={"GPFIT_DEVICE": "0", "GPF_COMM_TIMEOUT_S": "60"}, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 2 and out["value"] > 0
    ex = out["exchange"]
    assert ex["transport"] in ("rccl", "host")
    assert out["rccl"] == (ex["transport"] == "rccl") and out["exchange_ms_per_step"] >= 0.0
    if ex["transport"] == "host":
        assert ex["rccl_error"]
        assert "RCCL unavailable" in r.stderr  # one stderr line says the fallback triggered
