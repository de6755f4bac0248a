"""ADAPT on MI355X: layer-partitioned, fault-tolerant distributed inference.

A from-scratch MI355X-native rebuild of the ADAPT/DEFER reference
(Karthi-es/Adaptive-Deep-Learning-Architecture-for-Parallel-and-Fault-Tolerant-Inference):
named-layer model graphs are sliced into pipeline stages, each stage pinned to
one GPU, activations forwarded over RCCL point-to-point (xGMI), all hot ops
run as hand-written gfx950 HIP kernels, with an etcd-style membership
service driving repartition on worker join/leave.
"""
__version__ = "0.1.0"

# Stage processes own more HIP streams than the 4 default hardware queues (compute, capture, links, RCCL,
# codec, copy): ask for 8 at import, before anything initialises HIP, so `Node().run()` used as a library
# (the reference's entry point, `/root/reference/src/node.py:210-211`, and examples/test.py) gets them too
# (utils/hwqueues.py; a warning is logged if torch already initialised HIP).
from .utils.hwqueues import ensure_hw_queues as _ensure_hw_queues  # noqa: E402

_ensure_hw_queues()
