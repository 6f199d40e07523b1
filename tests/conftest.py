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


@pytest.fixture(autouse=True)
def _release_gpu_memory(request):
    """After each GPU test: drop the engines / graphs it left (reference cycles through the
    prepared calls keep them alive until a collection) and return the cached blocks, so one
    process can run the whole GPU suite.  The device's free memory before the release is
    appended to gpurun_out/gpu_mem.log."""
    yield
    if request.node.get_closest_marker("gpu") is None or "torch" not in sys.modules:
        return
    import gc
    import torch
    if not torch.cuda.is_available():
        return
    torch.cuda.synchronize()
    free, total = torch.cuda.mem_get_info()
    reserved = torch.cuda.memory_reserved()
    if os.environ.get("VQA_TEST_NO_GC") != "1":           # (A/B of the capture-time collector guard)
        gc.collect()
        torch.cuda.empty_cache()
    d = os.path.join(ROOT, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "gpu_mem.log"), "a") as f:
        f.write(f"{request.node.nodeid} free_gib={free / 2**30:.1f} total_gib={total / 2**30:.1f} "
                f"reserved_gib={reserved / 2**30:.2f} after_gc_free_gib={torch.cuda.mem_get_info()[0] / 2**30:.1f}\n")
