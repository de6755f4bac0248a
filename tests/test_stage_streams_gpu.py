"""Concurrent buffer sets (runtime/executor.py private_sets, runtime/stage.py
per-set compute streams): two micro-batches replayed at the same time on two
streams must give exactly what each gives alone.  With a shared internal arena
(private_sets=False) the two replays would overwrite each other's activations."""
import numpy as np
import pytest
import torch

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models import resnet as R
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops._lib import private_stream
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.executor import \
    SliceExecutor
from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.runtime.stage import \
    StageCompute

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def r50():
    g = R.build_resnet("resnet50")
    return g, R.init_weights(g, seed=3)


def test_private_sets_replay_concurrently(r50):
    g, w = r50
    ex = SliceExecutor(g, w, batch=8, device="cuda:0", num_sets=2, private_sets=True, precision="bf16")
    ex.capture()
    rng = np.random.default_rng(0)
    xs = [torch.from_numpy(rng.standard_normal((8, 224, 224, 3)).astype(np.float32)).cuda() for _ in range(2)]
    want = []
    for j in range(2):                                   # each set alone, one after the other
        ex.input_buf(g.input, j).copy_(xs[j].to(ex.input_buf(g.input, j).dtype))
        want.append(ex.forward(j)[ex.outputs[0]].clone())
    torch.cuda.synchronize()
    streams = [private_stream("cuda:0") for _ in range(2)]
    for _ in range(20):                                  # both sets in flight at once
        for j in range(2):
            streams[j].wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(streams[j]):
                ex.forward(j)
        for j in range(2):
            torch.cuda.current_stream().wait_stream(streams[j])
        torch.cuda.synchronize()
        for j in range(2):
            assert torch.equal(ex.output_buf(ex.outputs[0], j), want[j])


def test_stage_submit_two_streams_in_order(r50):
    g, w = r50
    sc = StageCompute(g, w, batch=4, device="cuda:0", num_sets=2)
    assert sc.multi_stream and sc.ex.private_sets
    rng = np.random.default_rng(1)
    xs = [rng.standard_normal((4, 224, 224, 3)).astype(np.float32) for _ in range(6)]
    pending = [sc.submit([x], [False], 4) for x in xs]
    got = []
    for ev, res in pending:
        ev.synchronize()
        got.append(res[0][0].copy())
    ref = StageCompute(g, w, batch=4, device="cuda:0", num_sets=1)
    for x, y in zip(xs, got):
        outs, _ = ref.run_host([x], [False], 4)
        np.testing.assert_allclose(y, outs[0], rtol=0, atol=1e-6)
