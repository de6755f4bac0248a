"""ADAPT on MI355X: layer-partitioned, fault-tolerant distributed inference.

A from-scratch MI355X-native rebuild of the ADAPT/DEFER reference
(Karthi-es/Adaptive-Deep-Learning-Architecture-for-Parallel-and-Fault-Tolerant-Inference):
named-layer model graphs are sliced into pipeline stages, each stage pinned to
one GPU, activations forwarded over RCCL point-to-point (xGMI), all hot ops
run as hand-written gfx950 HIP kernels, with an etcd-style membership
service driving repartition on worker join/leave.
"""
__version__ = "0.1.0"
