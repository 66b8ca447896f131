"""Shared test setup: markers, import paths, fixture helpers."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "sac-gat-her_transportationrl_amd")
os.environ["PYTHONPATH"] = os.pathsep.join([PKG_DIR, ROOT, os.environ.get("PYTHONPATH", "")])
for p in (ROOT, PKG_DIR, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- run with -m gpu")


def golden(name):
    return os.path.join(GOLDEN, name)


@pytest.fixture(scope="session")
def sf_graph_npz():
    import numpy as np
    return np.load(golden("sf_graph.npz"))


@pytest.fixture(scope="session")
def oracle_graph():
    import oracle as O
    return O.OracleGraph.from_npz(golden("sf_graph.npz"))
