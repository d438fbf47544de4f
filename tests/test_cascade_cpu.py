"""Cascade SVM on CPU ranks: thread-ranks (ThreadTransport) and a real
multi-process gloo group (TorchDistTransport), both topologies."""
import os
import socket

import numpy as np
import pytest
import torch

from svm355 import SVMParams
from svm355.ops import cpu as C
from svm355.parallel.cascade import CascadeSVM, SVSet, merge_unseen, partition_bounds, _CpuBackend
from svm355.parallel.transport import run_threads
from svm355.utils.data import MinMaxScaler, synthetic_mnist

N_TRAIN = 1500


@pytest.fixture(scope="module")
def data():
    return synthetic_mnist(N_TRAIN, seed=11), synthetic_mnist(500, seed=11, offset=N_TRAIN)


def _single(tr):
    p = SVMParams(n_threads=4)
    X = MinMaxScaler().fit_transform(tr.X)
    a, res, _ = C.smo_train(X, tr.y, p)
    return set(np.flatnonzero(a > p.sv_tol).tolist()), res.b


def _run(world, topology, tr, te, **kw):
    def fn(t):
        lo, hi = partition_bounds(tr.n, t.world, t.rank)
        c = CascadeSVM(t, SVMParams(n_threads=2), topology=topology, verbose=0, **kw)
        c.fit(tr.X[lo:hi], tr.y[lo:hi], np.arange(lo, hi), n_total=tr.n)
        return c.summary(), c.score(te.X, te.y), set(c.result.sv.ids.tolist())

    return run_threads(world, fn)


def test_partition_bounds():
    assert [partition_bounds(10, 4, r) for r in range(4)] == [(0, 3), (3, 6), (6, 9), (9, 10)]
    assert partition_bounds(2, 4, 3) == (2, 2)


def test_merge_unseen_keeps_warm_alpha_and_order():
    be = _CpuBackend(SVMParams(), 2)
    warm = SVSet(torch.tensor([[1.0, 1.0], [2.0, 2.0]]), np.array([1, -1], np.int32), np.array([0.5, 0.7]),
                 np.array([10, 20]))
    extra = SVSet(torch.tensor([[3.0, 3.0], [2.0, 2.0], [4.0, 4.0]]), np.array([1, -1, 1], np.int32),
                  np.array([9.0, 9.0, 9.0]), np.array([30, 20, 40]))
    m = merge_unseen(be, warm, extra)
    assert m.ids.tolist() == [10, 20, 30, 40]
    assert m.alpha.tolist() == [0.5, 0.7, 0.0, 0.0]
    assert m.X[:, 0].tolist() == [1, 2, 3, 4]


def test_svset_pack_roundtrip():
    s = SVSet(torch.arange(6, dtype=torch.float64).reshape(2, 3), np.array([1, -1], np.int32),
              np.array([0.25, 3.5]), np.array([7, 2 ** 40]))
    u = SVSet.unpack(s.pack(), 3)
    assert torch.equal(u.X, s.X) and u.y.tolist() == [1, -1] and u.alpha.tolist() == [0.25, 3.5]
    assert u.ids.tolist() == [7, 2 ** 40]


@pytest.mark.parametrize("topology,world", [("star", 1), ("star", 2), ("star", 3), ("tree", 2), ("tree", 4)])
def test_cascade_threads_converge_to_single_solve(data, topology, world):
    tr, te = data
    single_ids, single_b = _single(tr)
    out = _run(world, topology, tr, te)
    s0, acc0, ids0 = out[0]
    assert s0["converged"]
    assert s0["rounds"] <= 10
    # every rank holds the same final model
    for s, acc, ids in out[1:]:
        assert ids == ids0 and s["b"] == s0["b"] and acc == acc0
    # same optimum as one global SMO within the stopping tolerance
    assert len(ids0 ^ single_ids) <= max(3, len(single_ids) // 50)
    assert abs(s0["b"] - single_b) < 5e-3 * max(1.0, abs(single_b))
    assert acc0 > 0.95


def test_fit_and_score_do_not_mutate_inputs(data):
    tr, te = data
    X0, T0 = tr.X.copy(), te.X.copy()
    _run(2, "star", tr, te)
    np.testing.assert_array_equal(tr.X, X0)
    np.testing.assert_array_equal(te.X, T0)


def test_tree_rejects_non_power_of_two(data):
    tr, te = data
    with pytest.raises(ValueError, match="power-of-2"):
        _run(3, "tree", tr, te)


def test_checkpoint_resume(tmp_path, data):
    tr, te = data
    full = _run(2, "star", tr, te, checkpoint_dir=str(tmp_path))[0][0]
    assert (tmp_path / "cascade_state.npz").exists()
    # Resume from the final state: converges in one more round with the same model.
    res = _run(2, "star", tr, te, checkpoint_dir=str(tmp_path), resume=True)[0][0]
    assert res["converged"] and res["n_sv"] == full["n_sv"]
    assert abs(res["b"] - full["b"]) < 1e-9 * max(1, abs(full["b"]))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, topology, q):
    import torch.distributed as dist

    from svm355.parallel.transport import TorchDistTransport

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = synthetic_mnist(N_TRAIN, seed=11)
        te = synthetic_mnist(500, seed=11, offset=N_TRAIN)
        lo, hi = partition_bounds(tr.n, world, rank)
        t = TorchDistTransport(torch.device("cpu"))
        c = CascadeSVM(t, SVMParams(n_threads=2), topology=topology, verbose=0)
        c.fit(tr.X[lo:hi], tr.y[lo:hi], np.arange(lo, hi), n_total=tr.n)
        q.put((rank, c.summary(), c.score(te.X, te.y), sorted(c.result.sv.ids.tolist())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("topology", ["star", "tree"])
def test_cascade_gloo_two_processes_matches_threads(data, topology):
    import torch.multiprocessing as mp

    tr, te = data
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, topology, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    thr = _run(2, topology, tr, te)[0]
    for _, s, acc, ids in res:
        assert s["converged"] and s["rounds"] == thr[0]["rounds"]
        assert s["b"] == thr[0]["b"]  # identical arithmetic, identical transport payloads
        assert ids == sorted(thr[2])
        assert acc == thr[1]
