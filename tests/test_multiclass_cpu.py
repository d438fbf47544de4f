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


def _ovr_rank(t, tr):
    m = OneVsRestSVC(device="cpu", n_threads=2).fit(tr.X, tr.labels, transport=t)
    return m.support_, m.dual_coef_, m.intercepts_b_, m.n_iter_, m.stop_reasons_


def test_ovr_distributed_over_threads_equals_single_rank():
    """Classes split over 3 ranks (k % world == rank), results all-reduced: every rank holds the
    same model as a single-rank fit, bit for bit (each class is solved by exactly one rank)."""
    from svm355.parallel.transport import run_threads

    tr = synthetic_mnist(400, seed=5)
    one = OneVsRestSVC(device="cpu", n_threads=2).fit(tr.X, tr.labels)
    for sup, coef, b, it, st in run_threads(3, lambda t: _ovr_rank(t, tr)):
        np.testing.assert_array_equal(sup, one.support_)
        np.testing.assert_array_equal(coef, one.dual_coef_)
        np.testing.assert_array_equal(b, one.intercepts_b_)
        np.testing.assert_array_equal(it, one.n_iter_)
        assert st == one.stop_reasons_


def _gloo_ovr_worker(rank, world, port, q):
    import os

    import torch
    import torch.distributed as dist

    from svm355.parallel.transport import TorchDistTransport

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = synthetic_mnist(400, seed=5)
        q.put((rank, *_ovr_rank(TorchDistTransport(torch.device("cpu")), tr)))
    finally:
        dist.destroy_process_group()


def test_ovr_distributed_gloo_two_processes():
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_ovr_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tr = synthetic_mnist(400, seed=5)
    one = OneVsRestSVC(device="cpu", n_threads=2).fit(tr.X, tr.labels)
    for _, sup, coef, b, it, st in res:
        np.testing.assert_array_equal(sup, one.support_)
        np.testing.assert_array_equal(coef, one.dual_coef_)
        np.testing.assert_array_equal(b, one.intercepts_b_)
        assert st == one.stop_reasons_


def test_ovr_save_load_roundtrip(tmp_path):
    """OneVsRestSVC.save writes the reference's four model files per class (pickle-free extras beside
    them); load gives back the same decision values and predictions."""
    tr = synthetic_mnist(700, seed=5)
    te = synthetic_mnist(200, seed=5, offset=700)
    m = OneVsRestSVC(device="cpu", n_threads=2).fit(tr.X, tr.labels)
    m.save(tmp_path / "ovr")
    for c in m.classes_:
        for f in ("final_sv_ids.txt", "final_sv_labels.txt", "final_sv_alphas.txt", "final_b.txt"):
            assert (tmp_path / "ovr" / f"class_{c}" / f).exists()
    r = OneVsRestSVC.load(tmp_path / "ovr")
    np.testing.assert_array_equal(r.classes_, m.classes_)
    np.testing.assert_array_equal(r.support_, m.support_)
    np.testing.assert_array_equal(r.dual_coef_, m.dual_coef_)
    np.testing.assert_array_equal(r.intercepts_b_, m.intercepts_b_)
    np.testing.assert_array_equal(r.decision_function(te.X), m.decision_function(te.X))
    np.testing.assert_array_equal(r.predict(te.X), m.predict(te.X))


def test_ovr_class_absent_from_the_labels_is_never_predicted():
    """An explicitly requested class with no training rows: its solve stops with no candidate (alpha = 0)
    and it becomes the constant predictor -1, so it never outranks the real classes."""
    tr = synthetic_mnist(400, seed=9)
    labels = np.where(tr.labels < 3, tr.labels, 2)  # classes 0, 1, 2 only
    m = OneVsRestSVC(device="cpu", n_threads=2).fit(tr.X, labels, classes=[0, 1, 2, 7])
    assert m.stop_reasons_[3] == "no_candidate" and m.intercepts_b_[3] == 1.0
    assert np.all(m.decision_function(tr.X)[:, 3] == -1.0)
    assert 7 not in set(m.predict(tr.X).tolist())


def test_device_empty_releases_the_ovr_pool_slabs_on_oom(monkeypatch):
    """an out-of-memory allocation hands back the library's own device memory -- including the
    one-vs-rest pool threads' column-cache slabs, which the calling thread's release cannot reach --
    before its one retry."""
    import torch

    from svm355.models import multiclass as MC
    from svm355.ops import device as D

    calls = []
    real_empty = torch.empty

    def empty(*a, **k):
        if not calls:
            calls.append("oom")
            raise torch.OutOfMemoryError("injected")
        return real_empty(*a, **{kk: v for kk, v in k.items() if kk != "device"})

    monkeypatch.setattr(torch, "empty", empty)
    monkeypatch.setattr(D, "release_gram_buffers", lambda: calls.append("gram"))
    monkeypatch.setattr(MC, "release_solver_caches", lambda timeout_s=5.0: calls.append("ovr") or True)
    monkeypatch.setattr(torch.cuda, "empty_cache", lambda: calls.append("empty_cache"))
    out = D.device_empty((4, 4), torch.float64, "cpu")
    assert out.shape == (4, 4) and calls == ["oom", "gram", "ovr", "empty_cache"]


def test_ovr_pool_is_replaced_not_piled_up():
    """One persistent class-solve pool at a time: a fit of another width replaces it (its threads first
    hand back their slabs), so threads and slabs stay bounded over a process's life."""
    from svm355.models import multiclass as MC

    p2 = MC._pool(2)
    assert MC._pool(2) is p2 and MC._POOL[1] == 2
    p3 = MC._pool(3)
    assert p3 is not p2 and MC._POOL[1] == 3 and p2._shutdown
    assert MC.release_solver_caches()
