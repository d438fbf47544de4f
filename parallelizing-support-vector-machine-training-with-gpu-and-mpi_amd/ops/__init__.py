"""Kernel-level ops: ``cpu`` (native C++ oracle) and ``device`` (gfx950 HIP kernels on torch tensors)."""
