"""Shared test setup.

`-m "not gpu"` tests run in the build container (no GPU): the oracle against
the golden vectors, the host logic, and that libsbr loads and exports its
C ABI.  `-m gpu` tests run on an MI355X and compare the HIP path, called
through the C ABI, with the oracle.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
PKG = REPO / "replication-social-bank-runs_amd"
GOLDEN = REPO / "tests" / "golden"
for p in (str(PKG), str(REPO / "oracle"), str(REPO / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through libsbr)")
    config.addinivalue_line("markers", "slow: long CPU oracle runs")


def pytest_sessionstart(session):
    # the oracle is test infrastructure; build it in-tree if missing
    lib = REPO / "oracle" / "_build" / "libsbr_oracle.so"
    if not lib.exists():
        subprocess.run(["make", "-C", str(REPO / "oracle")], check=True, stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def golden():
    def load(name):
        p = GOLDEN / name
        if p.suffix == ".npz":
            return dict(np.load(p, allow_pickle=False))
        return json.loads(p.read_text())

    return load


@pytest.fixture(scope="session")
def oracle():
    import oracle as O

    O.lib()
    return O


@pytest.fixture(scope="session")
def engine():
    # PyTorch-ROCm bundles its own HIP runtime: let torch bring up the device first
    # (as bench.py does), so libsbr binds to the runtime already in the process.
    try:
        import torch

        if torch.cuda.is_available():
            torch.cuda.init()
    except ImportError:
        pass
    import sbr

    return sbr.Engine(int(os.environ.get("LOCAL_RANK", "0")))
