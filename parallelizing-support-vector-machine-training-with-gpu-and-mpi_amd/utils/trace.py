"""roctx ranges from Python (rocprofv3 --marker-trace), e.g. cascade rounds and RCCL exchanges.

No-ops unless the HIP device library is already loaded (CPU-only runs never load it)."""
from __future__ import annotations

from contextlib import contextmanager

from .. import _native as N


@contextmanager
def trace_range(name: str):
    lib = N._hip
    if lib is None:
        yield
        return
    lib.svmd_trace_push(name.encode())
    try:
        yield
    finally:
        lib.svmd_trace_pop()
