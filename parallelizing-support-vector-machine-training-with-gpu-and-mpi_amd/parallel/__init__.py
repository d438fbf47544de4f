"""Distributed Cascade SVM (classical tree + modified two-layer star) and its transports."""
from .cascade import CascadeSVM, CascadeResult
from .transport import ThreadTransport, TorchDistTransport, Transport

__all__ = ["CascadeSVM", "CascadeResult", "Transport", "ThreadTransport", "TorchDistTransport"]
