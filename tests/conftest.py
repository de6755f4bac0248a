import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


_EXIT = {"status": None}


def pytest_sessionfinish(session, exitstatus):
    _EXIT["status"] = int(exitstatus)


def pytest_unconfigure(config):
    """GPU sessions end with `os._exit` once pytest has reported: the DEFER tests
    leave aborted per-epoch gloo groups (host-staged links between GPU stages)
    whose backend threads are still parked in a cancelled recv, and the C++
    static teardown of the HIP runtime under them aborts the process
    ("terminate called without an active exception") after every test passed.
    The test verdict is already decided; skipping interpreter teardown keeps the
    exit code equal to it."""
    status = _EXIT["status"]
    if status is None or os.environ.get("ADAPT_TEST_NORMAL_EXIT") == "1":
        return
    try:
        import torch
        if not (torch.cuda.is_available() and torch.cuda.is_initialized()):
            return
        torch.cuda.synchronize()
    except Exception:  # noqa: BLE001
        pass
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(status)


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
