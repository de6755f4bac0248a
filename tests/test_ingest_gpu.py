"""Serving ingest on the MI355X: the uint8 -> fp32 preprocess kernel
(csrc/kernels/ingest.hip) against the host reference of Keras
`preprocess_input`, and a DEFER GPU stage fed uint8 images through same-host
shared memory (registered for DMA) with caffe preprocessing
(`test/test.py:20-23`)."""
import queue
import threading

import numpy as np
import pytest
import torch

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import eltwise as E

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["none", "caffe", "tf", "torch"])
@pytest.mark.parametrize("shape", [(32, 224, 224, 3), (3, 17, 5, 3), (1, 1, 1, 3)])
def test_ingest_u8_matches_reference(mode, shape):
    x = np.random.default_rng(0).integers(0, 256, shape, dtype=np.uint8)
    out = torch.empty(shape, dtype=torch.float32, device="cuda")
    E.ingest_u8(torch.from_numpy(x).cuda(), out, mode)
    np.testing.assert_allclose(out.cpu().numpy(), E.preprocess_ref(x, mode), rtol=1e-6, atol=1e-5)


def test_defer_gpu_uint8_shm_ingest():
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.dispatcher import DEFER
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.models.model import resnet
    from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.node import Node
    m = resnet("resnet50", seed=0)
    d = DEFER(membership_port=0, result_port=0, worker_wait=20, batch=4, ordered=True, weight_codec="lz4",
              preprocess="caffe", replicas=1)
    assert d._shm is not None
    d.membership_server.start()
    node = Node(membership_port=d.membership_port, data_port=0, config_port=0, device="cuda:0", node_id="ing0")
    node.run(block=False)
    try:
        inq, outq = queue.Queue(), queue.Queue()
        threading.Thread(target=d.run_defer, args=(m, [], inq, outq), daemon=True).start()
        rng = np.random.default_rng(1)
        xs = [rng.integers(0, 256, (4, 224, 224, 3), dtype=np.uint8) for _ in range(4)]
        for x in xs:
            inq.put(x)
        got = np.concatenate([outq.get(timeout=120) for _ in xs])
        want = m.predict(E.preprocess_ref(np.concatenate(xs), "caffe"), device="cpu")
        assert np.abs(got - want).sum(-1).max() < 0.1
        assert (got.argmax(-1) == want.argmax(-1)).mean() >= 0.75
    finally:
        d.shutdown(stop_workers=True)
        node.stop()
