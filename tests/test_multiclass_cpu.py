"""Multi-class one-vs-rest over a shared kernel matrix (CPU oracle)."""
import numpy as np

from svm355 import SVC, OneVsRestSVC
from svm355.utils.data import synthetic_mnist


def test_ovr_cpu_matches_per_class_svc():
    tr = synthetic_mnist(500, seed=3)
    te = synthetic_mnist(200, seed=3, offset=500)
    m = OneVsRestSVC(device="cpu").fit(tr.X, tr.labels)
    assert list(m.classes_) == sorted(set(tr.labels.tolist()))
    assert all(s == "converged" for s in m.stop_reasons_)
    # class "1" equals the reference's single one-vs-rest classifier
    k = int(np.flatnonzero(m.classes_ == 1)[0])
    s = SVC(device="cpu").fit(tr.X, tr.y)
    assert abs(m.intercepts_b_[k] - s.b_) < 1e-12
    np.testing.assert_allclose(m.decision_function(te.X)[:, k], s.decision_function(te.X), rtol=0, atol=1e-12)
    acc = m.score(te.X, te.labels)
    assert acc > 0.8, acc
