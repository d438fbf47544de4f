"""Distributed training: the native Cascade SVM (classical tree + modified two-layer star) with its
RCCL bootstraps, and the rank transports of the one-vs-rest trainer."""
from .cascade import CascadeResult, CascadeSVM, partition_bounds
from .hostcomm import HostCommRank
from .transport import ThreadTransport, TorchDistTransport, Transport

__all__ = ["CascadeSVM", "CascadeResult", "partition_bounds", "HostCommRank", "Transport", "ThreadTransport",
           "TorchDistTransport"]
