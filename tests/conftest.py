import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "graph-embedding_amd")
GOLD = os.path.join(ROOT, "tests", "golden")
DATA = os.path.join(GOLD, "data")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def golden_index():
    with open(os.path.join(GOLD, "index.json")) as f:
        return json.load(f)


def load_golden(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


@pytest.fixture(scope="session")
def gindex():
    return golden_index()


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def gw():
    import gwamd
    gwamd.lib()
    return gwamd
