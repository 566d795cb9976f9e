import json
import os
import sys

import pytest

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
GOLDEN = os.path.join(TESTS, "golden")
for p in (os.path.join(ROOT, "plonk.c_amd"), os.path.join(ROOT, "oracle"), GOLDEN, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from pyoracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def hip():
    """libplonkhip on the GPU; fails loudly (no skip) if the library or device is missing."""
    import plonkhip
    plonkhip.init(0)
    return plonkhip
