import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "ns-3-dev-dnemu_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path through the C-ABI)")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(REPO, "tests", "golden", "reference_kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def bench_dist():
    import nsref
    return nsref.load_distribution(os.path.join(REPO, "tests", "golden", "bench_dist_u01_10k.txt"))
