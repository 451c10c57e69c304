import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle"), GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine)")
    config.addinivalue_line("markers", "slow: full BASELINE.json sizes")
    config.addinivalue_line("markers", "latency: wall-clock bounds on a shared GPU (collected after every other test)")


def pytest_collection_modifyitems(session, config, items):
    """Wall-clock latency bounds run last: a timing outlier on a loaded GPU
    must not stop (-x) the run before the parity tests have reported."""
    items.sort(key=lambda it: it.get_closest_marker("latency") is not None)  # stable


@pytest.fixture(scope="session")
def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def vectors():
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def engine():
    """The HIP engine on cuda:0 — GPU tests only; fails loudly if the native
    library or the device is missing (no fallback)."""
    import torch  # noqa: F401  (one HIP runtime shared with torch)

    from netstack_amd import default_engine

    return default_engine(0)
