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
    """GPU sessions exit through normal interpreter teardown.  Until round 6 they
    ended with `os._exit`: aborted per-epoch groups from the DEFER tests left
    backend threads parked in native receives, and HIP's static teardown under
    them aborted the process after every test had passed.  With the RCCL
    async-error poll serialised and every communicator abort bounded
    (csrc/comm/rccl_p2p.cpp), the whole GPU suite exits cleanly
    (profiles/r6/pytest_gpu_normal_exit.log, rc 0).  ADAPT_TEST_FAST_EXIT=1
    restores the old exit for a box where teardown misbehaves."""
    status = _EXIT["status"]
    if status is None or os.environ.get("ADAPT_TEST_FAST_EXIT") != "1":
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
