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
