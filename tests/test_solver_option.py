"""SVC's solver option on the CPU: the decomposition solver (decomp.hip) is the GPU default ("auto"),
the pairwise SMO the CPU's (the oracle); an explicit decomp on the CPU says it is GPU-only; an unknown
solver is refused at construction."""
import numpy as np
import pytest

from svm355 import SVC
from svm355.utils.data import synthetic_mnist


def test_unknown_solver_is_refused():
    with pytest.raises(ValueError, match="solver"):
        SVC(solver="newton")


def test_decomp_on_the_cpu_is_refused():
    tr = synthetic_mnist(200, seed=1)
    with pytest.raises(ValueError, match="GPU"):
        SVC(device="cpu", solver="decomp").fit(tr.X, tr.y)


def test_default_solver_on_the_cpu_is_the_reference_smo():
    m = SVC(device="cpu")
    assert m.solver == "auto" and m.working_set == 1024
    tr = synthetic_mnist(300, seed=2)
    m.fit(tr.X, tr.y)
    assert m.stop_reason_ == "converged" and np.all(m.alpha_ >= 0)


def test_shrinking_option_codes():
    """SVC / SVMParams shrinking: off by default (profiles/shrinking.md), True = a pass every 2 outer
    iterations, an int k >= 0 = every k (0 off); anything else is rejected before any solve."""
    from svm355.utils.config import SVMParams

    assert SVMParams()._shrink_code() == 0 and SVC().params.shrinking is False
    assert SVMParams(shrinking=True)._shrink_code() == 2
    assert SVMParams(shrinking=False)._shrink_code() == 0
    assert SVMParams(shrinking=0)._shrink_code() == 0
    assert SVMParams(shrinking=5)._shrink_code() == 5
    assert SVMParams(shrinking=5).to_struct().shrink == 5
    for bad in (-1, 2.5, "yes"):
        with pytest.raises(ValueError, match="shrinking"):
            SVMParams(shrinking=bad)
