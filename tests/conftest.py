import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from srsgpu_testlib import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np
    z = np.load(os.path.join(HERE, "golden", "tdec_golden.npz"))
    manifest = json.loads(bytes(z["manifest"]).decode())
    return z, manifest


@pytest.fixture(autouse=True)
def _gc_after_each_test():
    """SRSGPU_GC_EACH=1: collect garbage after every test, so a failing native destructor shows up
    in the test that created the object (debugging aid)"""
    yield
    if os.environ.get("SRSGPU_GC_EACH") == "1":
        import gc
        gc.collect()
