import os
import sys
from pathlib import Path

# BLAS thread pins must precede the first numpy import (SURVEY.md §6 gotcha):
# multi-threaded dgesv rounds differently from the reference's 1-thread run.
os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")

import numpy as np  # noqa: E402
import pytest  # noqa: E402

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "gaussian-process_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = Path(__file__).resolve().parent / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def load_golden(name):
    return np.load(GOLDEN / name, allow_pickle=False)


@pytest.fixture(scope="session")
def f1():
    return load_golden("f1_gp_recovered.npz")


@pytest.fixture(scope="session")
def f2():
    return load_golden("f2_loss_testfiles.npz")


@pytest.fixture(scope="session")
def f3():
    return load_golden("f3_synthetic.npz")


@pytest.fixture(scope="session")
def f4():
    return load_golden("f4_pso_trace.npz")


def synth_data(N, d, hetero, seed):
    """SURVEY.md §8d synthetic set (the construction of bench.synthetic and of
    tests/golden/make_golden.py's synth_data): x~U[0,1)^d, y=sum sin(2 pi x)+0.1 N(0,1),
    e = 0.1 or U[0.05, 0.2] (heteroscedastic)."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(0.0, 1.0, size=(d, N))
    y = np.sum(np.sin(2 * np.pi * x), axis=0) + 0.1 * rng.standard_normal(N)
    e = rng.uniform(0.05, 0.2, size=N) if hetero else np.full(N, 0.1)
    return x, y, e


def data_sha256(*arrays):
    """Hash the reference-side fixture scripts store instead of the regenerated inputs."""
    import hashlib
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    return h.hexdigest()


def fixture_data(meta, sha):
    """Regenerate a fixture's synthetic inputs from its (N, d, hetero, seed) and check them."""
    N, d, het, seed = (int(v) for v in meta)
    x, y, e = synth_data(N, d, bool(het), seed)
    assert data_sha256(x, y, e) == str(sha), "regenerated inputs differ from the fixture's"
    return x, y, e
