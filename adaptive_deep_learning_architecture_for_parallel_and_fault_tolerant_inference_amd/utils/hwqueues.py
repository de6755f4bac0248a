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

import os

STAGE_HW_QUEUES = 8


def ensure_hw_queues(n: int = STAGE_HW_QUEUES) -> int:
    """Raise ``GPU_MAX_HW_QUEUES`` to at least `n` (never above 32) for this
    process and its children; effective only before the process's first HIP
    call.  Returns the value in force."""
    n = max(1, min(int(n), 32))
    try:
        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
    except ValueError:
        cur = 0
    if cur < n:
        os.environ["GPU_MAX_HW_QUEUES"] = str(n)
        cur = n
    return cur
