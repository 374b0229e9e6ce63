import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_addoption(parser):
    parser.addoption("--tuning", action="store_true", default=False,
                     help="also run the tuning-build variant cases (marker 'tuning')")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "tuning: a case of a tuning-build kernel variant (A/B only, never "
                            "shipped); deselected unless --tuning is given")


def pytest_collection_modifyitems(config, items):
    """The tuning-build variant matrix (alternative shapes and thresholds the
    A/B tools select) stays out of the default runs: -m gpu checks what ships."""
    if config.getoption("--tuning"):
        return
    keep = [it for it in items if it.get_closest_marker("tuning") is None]
    if len(keep) != len(items):
        config.hook.pytest_deselected(items=[it for it in items if it.get_closest_marker("tuning")])
        items[:] = keep


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
