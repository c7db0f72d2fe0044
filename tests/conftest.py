"""Test configuration: the `gpu` marker and shared helpers.

`-m "not gpu"` runs here (no GPU): oracle vs the reference's KATs, host logic,
and that libslime_rs.so loads and exports every symbol include/slime_rs.h
declares.  `-m gpu` runs on an MI355X: the HIP path against the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def kats():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "vectors.json")) as f:
        return json.load(f)
