import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "first: run before every other test of the session "
                                       "(the RCCL test initialises torch.distributed before any "
                                       "other GPU work of the process)")


def pytest_collection_modifyitems(config, items):
    items.sort(key=lambda it: 0 if it.get_closest_marker("first") else 1)


@pytest.fixture(scope="session")
def engine():
    from mythril_amd.engine import get_engine

    return get_engine(0)


def load_golden(name):
    import json

    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)
