"""Hardware-queue budget of a stage process.

HIP maps every stream of a process onto at most ``GPU_MAX_HW_QUEUES``
hardware (AQL) queues, 4 by default.  Streams beyond that share queues, and a
packet waits for the packets ahead of it in its queue even when they belong to
another stream.  A pipeline stage process owns more streams than 4: the
compute stream, the executor's capture stream, one stream per RCCL link plus
RCCL's internal streams, the codec side stream and the serving copy stream.
Measured on one MI355X (tests/test_stream_queues_gpu.py, `spin_flag`): with 4
queues, a ResNet-50 slice replay on the compute stream stalled behind a
spinning kernel as soon as 3 other streams were busy (a receive posted for a
later micro-batch is exactly such a kernel: it spins until the upstream peer
sends).  Stage processes therefore ask for 8 queues before their first HIP
call.  The reference has no device streams at all (Keras `model.predict`,
`src/node.py:177`).
"""
from __future__ import annotations

import logging
import os
import sys

STAGE_HW_QUEUES = 8
log = logging.getLogger(__name__)


def hip_initialised() -> bool:
    """Whether this process has already initialised HIP through torch (then the queue count is fixed)."""
    torch = sys.modules.get("torch")
    if torch is None:
        return False
    try:
        return bool(torch.cuda.is_initialized())
    except Exception:
        return False


def ensure_hw_queues(n: int = STAGE_HW_QUEUES) -> int:
    """Raise ``GPU_MAX_HW_QUEUES`` to at least `n` (never above 32) for this process and its children;
    effective only before the process's first HIP call.  ``ADAPT_HW_QUEUES`` overrides `n` (a user who
    wants fewer queues, e.g. 4, sets it; it is then applied as given, lower values included).  Returns the
    value in force and logs it when it differs from `n` or when HIP was already initialised."""
    want = os.environ.get("ADAPT_HW_QUEUES")
    explicit = want is not None
    try:
        n = int(want) if explicit else int(n)
    except ValueError:
        explicit, n = False, int(STAGE_HW_QUEUES)
    n = max(1, min(n, 32))
    try:
        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
    except ValueError:
        cur = 0
    if hip_initialised():
        log.warning("HIP is already initialised: GPU_MAX_HW_QUEUES stays %s for this process (stages want %d)",
                    cur or "the HIP default (4)", n)
        return cur
    if explicit or cur < n:
        os.environ["GPU_MAX_HW_QUEUES"] = str(n)
        cur = n
    return cur
