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


@pytest.mark.parametrize("n", [2, 4])
def test_gpus_flag_starts_that_many_ranks(n):
    r = _run(["--gpus", str(n), "--plumbing"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["ranks_joined"] == n and out["scores_ok"]
    assert out["swarm"] == 32 * n  # config D's 32 particles per GPU


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "3", "--plumbing"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "--gpus 3" in r.stderr
