import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs a real MI355X (gfx950); runs through the C ABI")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(TESTS, "golden", "kat.json")) as f:
        kat = json.load(f)
    with open(os.path.join(TESTS, "golden", "batches.json")) as f:
        batches = json.load(f)
    with open(os.path.join(TESTS, "golden", "survey_ref_sha2c.json")) as f:
        ref = json.load(f)
    return {"kat": kat, "batches": batches, "sha2c": ref}


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.lib()
    return oracle
