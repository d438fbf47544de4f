"""Cascade SVM on CPU thread-ranks: the ONE native driver (csrc/cascade) on the
C++ oracle backend with the loopback transport — the same round code the GPUs run.

Parity is pinned against an independent Python transcription of the reference round loops
(mpi_svm_main2.cpp:439-769 star, mpi_svm_main3.cpp:565-828 tree) on the same oracle SMO: rounds,
SV ids and b must be bit-identical."""
import time

import numpy as np
import pytest

from svm355 import SVMParams
from svm355._native import NativeError
from svm355.ops import cpu as C
from svm355.parallel.cascade import CascadeSVM, partition_bounds
from svm355.utils.data import MinMaxScaler, synthetic_mnist

N_TRAIN = 1500
P2 = SVMParams(n_threads=2)


@pytest.fixture(scope="module")
def data():
    return synthetic_mnist(N_TRAIN, seed=11), synthetic_mnist(500, seed=11, offset=N_TRAIN)


# ------------------------------------------------------------------ independent transcription
def _solve(X, y, a):
    a2, res, _ = C.smo_train(X, y, P2, alpha=a.copy(), warm=True)
    keep = np.flatnonzero(a2 > P2.sv_tol)
    return (X[keep], y[keep], a2[keep]), res.b, keep


def _merge_unseen(warm, extra):  # M3 :629-655 / M2 :474-502
    (Xw, yw, aw, iw), (Xe, ye, _, ie) = warm, extra
    keep = np.flatnonzero(~np.isin(ie, iw))
    return (np.concatenate([Xw, Xe[keep]]), np.concatenate([yw, ye[keep]]),
            np.concatenate([aw, np.zeros(len(keep))]), np.concatenate([iw, ie[keep]]))


def _py_cascade(tr, P, topology):
    Xs = MinMaxScaler().fit_transform(tr.X)  # global min/max (M3 :529-539)
    parts = []
    for r in range(P):
        lo, hi = partition_bounds(tr.n, P, r)
        parts.append((Xs[lo:hi], tr.y[lo:hi], np.zeros(hi - lo), np.arange(lo, hi)))
    G = (np.empty((0, tr.d)), np.empty(0, np.int32), np.empty(0), np.empty(0, np.int64))
    prev, b, rounds, hist = None, 0.0, 0, []
    while rounds < 50:
        rounds += 1
        if topology == "star":
            local = []
            for r in range(P):
                S = _merge_unseen(G, parts[r])
                (Xk, yk, ak), _, keep = _solve(*S[:3])
                local.append((Xk, yk, ak, S[3][keep]))
            merged = local[0]
            for w in local[1:]:  # worker alphas reset to 0 (M2 :600-601), source order (M2 :578)
                merged = _merge_unseen(merged, (w[0], w[1], np.zeros(len(w[1])), w[3]))
            (Xk, yk, ak), b, keep = _solve(*merged[:3])
            G = (Xk, yk, ak, merged[3][keep])
        else:
            cur = {}
            recv = {0: G}
            step = 1
            while step <= P:
                for r in range(0, P, step):
                    S = _merge_unseen(recv.get(r, G) if step > 1 else G, cur.get(r, parts[r]))
                    (Xk, yk, ak), bl, keep = _solve(*S[:3])
                    cur[r] = (Xk, yk, ak, S[3][keep])
                    if r == 0:
                        b = bl
                recv = {r: cur[r + step] for r in range(0, P, 2 * step) if r + step < P}
                step *= 2
            G = cur[0]
        hist.append(len(G[3]))
        ids = set(G[3].tolist())
        if ids == prev:
            break
        prev = ids
    return rounds, sorted(G[3].tolist()), b, hist


# ------------------------------------------------------------------------------------ tests
def test_partition_bounds():
    assert [partition_bounds(10, 4, r) for r in range(4)] == [(0, 3), (3, 6), (6, 9), (9, 10)]
    assert partition_bounds(2, 4, 3) == (2, 2)


@pytest.mark.parametrize("topology,world", [("star", 2), ("star", 3), ("tree", 2), ("tree", 4)])
def test_native_driver_bit_identical_to_transcription(data, topology, world):
    tr, _ = data
    nat = CascadeSVM(P2, topology=topology).fit(tr.X, tr.y, world=world).result
    rounds, ids, b, hist = _py_cascade(tr, world, topology)
    assert nat.rounds == rounds and nat.sv_history == hist
    assert sorted(nat.ids.tolist()) == ids
    assert nat.b == b


@pytest.mark.parametrize("topology,world", [("star", 1), ("star", 2), ("star", 3), ("tree", 2), ("tree", 4)])
def test_cascade_threads_converge_to_single_solve(data, topology, world):
    tr, te = data
    p = SVMParams(n_threads=4)
    a, res, _ = C.smo_train(MinMaxScaler().fit_transform(tr.X), tr.y, p)
    single = set(np.flatnonzero(a > p.sv_tol).tolist())
    c = CascadeSVM(P2, topology=topology).fit(tr.X, tr.y, world=world)
    r = c.result
    assert r.converged and r.rounds <= 10 and r.backend == "cpu" and r.transport == "loopback"
    assert len(set(r.ids.tolist()) ^ single) <= max(3, len(single) // 50)
    assert abs(r.b - res.b) < 5e-3 * max(1.0, abs(res.b))
    assert c.score(te.X, te.y) > 0.95
    # per-solve log: every rank's solves with rows / iterations
    assert {s["rank"] for s in r.solves} == set(range(world))
    assert all(s["iterations"] >= 1 and s["n"] > 0 for s in r.solves)


def test_fit_and_score_do_not_mutate_inputs(data):
    tr, te = data
    X0, T0 = tr.X.copy(), te.X.copy()
    CascadeSVM(P2).fit(tr.X, tr.y, world=2).score(te.X, te.y)
    np.testing.assert_array_equal(tr.X, X0)
    np.testing.assert_array_equal(te.X, T0)


def test_tree_rejects_non_power_of_two(data):
    tr, _ = data
    with pytest.raises(ValueError, match="power-of-2"):
        CascadeSVM(P2, topology="tree").fit(tr.X, tr.y, world=3)


def test_empty_data_is_an_error():
    with pytest.raises(NativeError, match="No data read"):
        CascadeSVM(P2).fit(np.empty((0, 4)), np.empty(0, np.int32), world=2)


@pytest.mark.parametrize("topology", ["star", "tree"])
def test_checkpoint_resume_bit_identical(tmp_path, data, topology):
    tr, _ = data
    full = CascadeSVM(P2, topology=topology).fit(tr.X, tr.y, world=2).result
    ck = str(tmp_path / topology)
    part = CascadeSVM(P2, topology=topology, max_rounds=1, checkpoint_dir=ck).fit(tr.X, tr.y, world=2).result
    assert part.rounds == 1 and not part.converged and (tmp_path / topology / "cascade_state.bin").exists()
    res = CascadeSVM(P2, topology=topology, checkpoint_dir=ck, resume=True).fit(tr.X, tr.y, world=2).result
    assert res.converged and res.rounds == full.rounds
    assert sorted(res.ids.tolist()) == sorted(full.ids.tolist()) and res.b == full.b


def test_checkpoint_of_other_topology_is_rejected(tmp_path, data):
    tr, _ = data
    CascadeSVM(P2, topology="star", max_rounds=1, checkpoint_dir=str(tmp_path)).fit(tr.X, tr.y, world=2)
    with pytest.raises(NativeError, match="does not match"):
        CascadeSVM(P2, topology="tree", checkpoint_dir=str(tmp_path), resume=True).fit(tr.X, tr.y, world=2)


def test_checkpoint_of_other_training_set_is_rejected(tmp_path, data):
    """A resume on other rows (another row count or other column ranges) is refused: the checkpoint
    carries a fingerprint of n and the global column bounds."""
    tr, _ = data
    CascadeSVM(P2, topology="star", max_rounds=1, checkpoint_dir=str(tmp_path)).fit(tr.X, tr.y, world=2)
    with pytest.raises(NativeError, match="another training set"):
        CascadeSVM(P2, topology="star", checkpoint_dir=str(tmp_path), resume=True).fit(tr.X[:-7], tr.y[:-7], world=2)
    X2 = tr.X.copy()
    X2[:, 300] = X2[:, 300] * 0.5  # one column's range changes
    with pytest.raises(NativeError, match="another training set"):
        CascadeSVM(P2, topology="star", checkpoint_dir=str(tmp_path), resume=True).fit(X2, tr.y, world=2)


def test_checkpoint_of_other_labels_or_rows_with_the_same_bounds_is_rejected(tmp_path, data):
    """the fingerprint also covers every rank's rows, labels and ids -- a resume of another
    one-vs-rest class on the same rows (other labels), or on other rows whose columns span the same
    ranges, is refused; the same data still resumes."""
    tr, _ = data
    ck = str(tmp_path)
    CascadeSVM(P2, topology="star", max_rounds=1, checkpoint_dir=ck).fit(tr.X, tr.y, world=2)
    y2 = tr.y.copy()
    y2[:5] = -y2[:5]  # another positive class on the same rows
    with pytest.raises(NativeError, match="another training set"):
        CascadeSVM(P2, topology="star", checkpoint_dir=ck, resume=True).fit(tr.X, y2, world=2)
    X3 = tr.X.copy()
    X3[[3, 4]] = X3[[4, 3]]  # two rows swapped: the same column bounds, other rows
    with pytest.raises(NativeError, match="another training set"):
        CascadeSVM(P2, topology="star", checkpoint_dir=ck, resume=True).fit(X3, tr.y, world=2)
    res = CascadeSVM(P2, topology="star", checkpoint_dir=ck, resume=True).fit(tr.X, tr.y, world=2).result
    assert res.converged


@pytest.mark.parametrize("world,fail_rank,fail_round", [(2, 1, 1), (3, 0, 0), (4, 2, 1)])
def test_failing_rank_ends_every_rank(data, world, fail_rank, fail_round):
    """One rank throws mid-run: the others leave their exchanges and the call reports that rank."""
    tr, _ = data
    t0 = time.perf_counter()
    with pytest.raises(NativeError, match=f"rank {fail_rank}: injected failure at round {fail_round}"):
        CascadeSVM(P2, comm_timeout_s=60, fail_rank=fail_rank, fail_round=fail_round).fit(tr.X, tr.y, world=world)
    assert time.perf_counter() - t0 < 30  # no deadline was needed: the abort token ended the waits


def test_stalled_rank_hits_the_deadline(data):
    """A rank that stops responding: its peers' exchanges time out instead of hanging."""
    tr, _ = data
    t0 = time.perf_counter()
    with pytest.raises(NativeError, match="no progress for 0.5 s"):
        CascadeSVM(P2, comm_timeout_s=0.5, fail_rank=1, fail_round=1, fail_stall_s=3.0).fit(tr.X, tr.y, world=2)
    assert time.perf_counter() - t0 < 30


@pytest.mark.parametrize("topology,world", [("star", 2), ("star", 3), ("tree", 2)])
def test_decomposition_solver_cascade(data, topology, world):
    """Every local / merge solve by the warm-started decomposition (its CPU oracle on the set's direct
    RBF Gram; decomp.hip on the GPUs): the same converged model as the pairwise cascade within the stop
    tolerance, every solve logged as decomp."""
    tr, te = data
    a = CascadeSVM(P2, topology=topology, solver="smo").fit(tr.X, tr.y, world=world)
    b = CascadeSVM(P2, topology=topology, solver="decomp").fit(tr.X, tr.y, world=world)
    ra, rb = a.result, b.result
    assert rb.converged and all(s["solver"] == "decomp" for s in rb.solves)
    assert all(s["solver"] == "smo" for s in ra.solves)
    assert abs(ra.b - rb.b) <= 10 * P2.tau
    assert len(set(ra.ids.tolist()) ^ set(rb.ids.tolist())) <= 2
    assert abs(a.score(te.X, te.y) - b.score(te.X, te.y)) <= 0.002


@pytest.mark.parametrize("topology", ["star", "tree"])
@pytest.mark.parametrize("solver", ["smo", "decomp"])
def test_partitions_of_one_class_each(topology, solver):
    """8 ranks on rows sorted by label: every partition holds one class, so no local solve finds a
    violating pair and no rank has a support vector (the gather of empty sets once faulted on rank 0).
    The cascade ends cleanly with an empty model, as the reference's rounds would."""
    rng = np.random.default_rng(11)
    X = rng.integers(0, 256, size=(24, 6)).astype(np.float64)
    y = np.where(np.arange(24) < 12, 1, -1).astype(np.int32)
    c = CascadeSVM(topology=topology, solver=solver).fit(X, y, world=8, device="cpu")
    assert c.result.converged and len(c.result.ids) == 0 and c.result.b == 0.0
