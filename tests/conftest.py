import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size CPU oracle runs")


@pytest.fixture(scope="session")
def pkg():
    from __graft_entry__ import load_package
    return load_package()


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def _load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return _load


@pytest.fixture(scope="session")
def parity_report():
    """Measured errors of the GPU parity checks: tests add {check: value}; at the end of
    the session they are written to gpurun_out/parity_report.json (merged back by gpurun,
    then committed under profiles/)."""
    import json
    rep = {}
    yield rep
    if rep:
        d = os.path.join(ROOT, "gpurun_out")
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, "parity_report.json")
        old = json.load(open(path)) if os.path.exists(path) else {}
        old.update(rep)
        json.dump(old, open(path, "w"), indent=1, sort_keys=True)
