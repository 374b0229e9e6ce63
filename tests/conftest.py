import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def golden():
    with np.load(os.path.join(GOLDEN, "city_golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def folds():
    import json
    p = os.path.join(GOLDEN, "config_folds.json")
    if not os.path.exists(p):
        pytest.skip("config_folds.json not generated")
    with open(p) as f:
        return json.load(f)["configs"]


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


def pattern_a(n):
    return bytes(i & 0xFF for i in range(n))


def pattern_b(n):
    return bytes((i * 7 + 3) & 0xFF for i in range(n))
