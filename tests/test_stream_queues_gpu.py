"""A pipeline stage's compute stream must not queue behind its link streams.

A stage process owns more HIP streams than the default GPU_MAX_HW_QUEUES = 4
hardware queues: the compute stream (graph replays), the executor's private
capture stream, one stream per RCCL link (`parallel/rccl.py`), RCCL's own
internal streams, the codec's side stream and the serving copy stream.  Streams
beyond the queue count share queues, and a packet in a shared queue waits for
the packets ahead of it.  A receive posted for micro-batch t+2 that spins until
its upstream peer sends would then hold back compute(t+1), silently
serialising the pipeline.

`tools/queue_probe.py` (run here in a child process, so the queue count is
read fresh) builds that stream set in a stage process's creation order, parks a
spinning kernel (`spin_flag`: host-released flag, wall-clock bound, always
ends) on the busy streams and checks that a ResNet-50 slice's graph replay on
the compute stream still finishes.  With 4 queues it does not once 3 other
streams are busy (measured: the first GPU run of this test), so stage
processes (`node.py`, `bench.py`) ask for 8 (`utils/hwqueues.py`); the test
requires the stage set (links, codec side and copy streams all busy) to pass at
that setting, and records the sweep over k fresh busy streams and the 4-queue
behaviour.  The sweep is not monotonic in k at any queue count (measured at 4 /
8 / 16: `profiles/r4/queue_probe.txt`): which hardware queue a new stream lands
on depends on every stream the process created before it, so it is the stage
set, in its real creation order, that is asserted.

The reference's hop is a blocking TCP send from the worker's compute loop
(`src/node.py:163-179`), so its compute and transfer never overlap at all.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _probe(queues: int) -> dict:
    # ADAPT_HW_QUEUES: the package applies it as given at import (utils/hwqueues.py), lower counts included
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(queues), ADAPT_HW_QUEUES=str(queues))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "queue_probe.py")], env=env,
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


def test_stage_streams_do_not_block_compute_at_stage_queue_count():
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.utils.hwqueues import \
        STAGE_HW_QUEUES
    rec = _probe(STAGE_HW_QUEUES)
    print(json.dumps(rec))
    st = rec["stage"]
    assert st["links"]["released"] and st["links_side_copy"]["released"], "a spinner hit its time bound"
    assert st["links"]["ok"], f"compute waited for a spinning link stream: {st}"
    assert st["links_side_copy"]["ok"], f"compute waited for a spinning auxiliary stream: {st}"
    assert all(v["released"] for v in rec["sweep"].values())


def test_default_queue_count_blocks_compute():
    """The HIP default (4 queues): with the stage set busy, compute waits (the
    reason stage processes raise the count); every spinner is still released
    by its flag, never by its time bound."""
    rec = _probe(4)
    print(json.dumps(rec))
    assert all(v["released"] for v in rec["sweep"].values())
    assert not rec["stage"]["links_side_copy"]["ok"]
