"""Distributed training: the native Cascade SVM (classical tree + modified two-layer star) with its
RCCL bootstraps, the distributed SMO over the GPUs of a node (one solve, candidates exchanged over
xGMI), and the rank transports of the one-vs-rest trainer."""
from .cascade import CascadeResult, CascadeSVM, partition_bounds
from .dsmo import DistributedSVC, DsmoGroup, DsmoRank
from .hostcomm import HostCommRank
from .transport import ThreadTransport, TorchDistTransport, Transport

__all__ = ["CascadeSVM", "CascadeResult", "partition_bounds", "DistributedSVC", "DsmoGroup", "DsmoRank",
           "HostCommRank", "Transport", "ThreadTransport", "TorchDistTransport"]
