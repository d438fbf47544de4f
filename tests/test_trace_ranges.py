"""roctx ranges from Python (svm355/utils/trace.py): no-ops without the device library, balanced
push / pop around the wrapped block (also when it raises), and the estimators' phases are wrapped
(parallel/decomp.py, parallel/cascade.py, models/multiclass.py)."""
import inspect

import pytest

from svm355 import _native as N
from svm355.utils.trace import trace_range


class _FakeLib:
    def __init__(self):
        self.calls = []

    def svmd_trace_push(self, name):
        self.calls.append(("push", name.decode()))

    def svmd_trace_pop(self):
        self.calls.append(("pop",))


def test_no_library_is_a_no_op(monkeypatch):
    monkeypatch.setattr(N, "_hip", None)
    with trace_range("x"):
        pass


def test_push_pop_balanced_and_nested(monkeypatch):
    lib = _FakeLib()
    monkeypatch.setattr(N, "_hip", lib)
    with trace_range("outer"):
        with trace_range("inner"):
            pass
    with pytest.raises(RuntimeError):
        with trace_range("raises"):
            raise RuntimeError("boom")
    assert lib.calls == [("push", "outer"), ("push", "inner"), ("pop",), ("pop",), ("push", "raises"), ("pop",)]


def test_phases_are_wrapped():
    from svm355.models import multiclass
    from svm355.parallel import cascade, decomp

    assert "svm355.decomp.solve" in inspect.getsource(decomp._fit_native)
    assert "svm355.decomp.model" in inspect.getsource(decomp.DistributedDecompSVC.fit)
    assert "svm355.cascade." in inspect.getsource(cascade.CascadeSVM.fit)
    src = inspect.getsource(multiclass.OneVsRestSVC._fit_cuda)
    assert "svm355.ovr.gram" in src and "svm355.ovr.solve" in src
    assert "svm355.ovr.decomp" in inspect.getsource(multiclass.OneVsRestSVC._fit_cuda_decomp)
