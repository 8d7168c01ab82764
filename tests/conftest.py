import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (os.path.join(ROOT, "rs-pathplanning_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) — runs on the GPU box")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def built():
    import __graft_entry__ as g

    g.build()
    return g


@pytest.fixture(scope="session")
def oracle_mod(built):
    import oracle

    return oracle


@pytest.fixture(scope="session")
def pkg(built):
    import pathplanning_amd

    return pathplanning_amd
