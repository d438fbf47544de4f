"""The strict loopback transport (csrc/cascade/loopback.cpp) and the transport exerciser / RCCL
preflight (csrc/cascade/exercise.cpp), on CPU thread-ranks.

Strict mode holds every call sequence to RCCL's contract -- matched collectives, rendezvous sends,
no wait-for cycles -- so a cascade sequence that would deadlock or corrupt over RCCL fails here with
both ranks named, well inside the deadline.  The exerciser checks every received byte."""
import time

import numpy as np
import pytest

from svm355 import SVMParams
from svm355._native import NativeError
from svm355.parallel.cascade import CascadeSVM, loopback_exercise, preflight_script
from svm355.utils.data import synthetic_mnist


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 8])
def test_preflight_script_passes_on_strict_loopback(world):
    """The op set the RCCL groups run before any fit (tree pairs per level included) is itself a
    valid RCCL sequence: no mismatch, no deadlock, every payload intact."""
    loopback_exercise(world, preflight_script(world, 1 << 16), strict=True, timeout_s=20)


def test_preflight_covers_every_driver_op():
    s = preflight_script(8, 64)
    ranks = s.split("|")
    assert len(ranks) == 8
    for op in ("bi@0", "ag", "mn:784", "mx:784", "bc:64@0", "ga:64@0", "ba"):
        assert all(op in r.split() for r in ranks), op
    # tree levels: 1 -> 0, 2 -> 0, 4 -> 0 (counts then payloads), 3 -> 2, ...
    r0 = ranks[0].split()
    assert ["ri<1", "r:64<1", "ri<2", "r:64<2", "ri<4", "r:64<4"] == [t for t in r0 if t.startswith(("ri", "r:"))]
    assert "si>0" in ranks[4].split() and "si>2" in ranks[3].split()


@pytest.mark.parametrize("script,words", [
    ("bi@0|ag", ["mismatch", "bcast_i64(root 0, 8 B)", "rank 1 called allgather_i64"]),
    ("bc:16@0|bc:32@0", ["mismatch", "16 B", "32 B"]),
    ("bi@0|bi@1", ["mismatch", "root 0", "root 1"]),
    ("s:8>1|s:8>0", ["deadlock", "rank 0 in send(to rank 1", "rank 1 in send(to rank 0"]),
    ("bi@0 s:8>1|r:8<0 bi@0", ["deadlock", "bcast_i64", "recv(from rank 0"]),
    ("ba|r:8<0", ["deadlock", "barrier", "recv(from rank 0"]),
    ("s:8>1|r:16<0", ["message of 8 bytes, expected 16"]),
])
def test_mismatched_sequences_fail_fast_naming_the_ranks(script, words):
    t0 = time.time()
    with pytest.raises(NativeError) as ei:
        loopback_exercise(2, script, strict=True, timeout_s=10)
    msg = str(ei.value)
    assert time.time() - t0 < 5, msg  # detected, not timed out
    for w in words:
        assert w in msg, msg


def test_three_rank_send_cycle_is_a_deadlock():
    with pytest.raises(NativeError, match="deadlock") as ei:
        loopback_exercise(3, "s:8>1|s:8>2|s:8>0", strict=True, timeout_s=10)
    for r, peer in ((0, 1), (1, 2), (2, 0)):  # whichever rank detects it names the whole cycle
        assert f"rank {r} in send(to rank {peer}" in str(ei.value), str(ei.value)


def test_rendezvous_send_waits_for_the_receiver():
    """A matched pair whose receiver arrives late completes (send blocks, no deadlock)."""
    loopback_exercise(2, "s:1024>1 ba|r:1024<0 ba", strict=True, timeout_s=10)
    loopback_exercise(3, "si>1 s:64>1 ba|ri<0 r:64<0 si>2 s:64>2 ba|ri<1 r:64<1 ba", strict=True, timeout_s=10)


def test_loose_mode_accepts_what_rccl_would_deadlock_on():
    """The old mailbox semantics (send returns after posting) hid exactly this class of bug."""
    loopback_exercise(2, "s:8>1 r:8<1|s:8>0 r:8<0", strict=False, timeout_s=5)
    with pytest.raises(NativeError, match="deadlock"):
        loopback_exercise(2, "s:8>1 r:8<1|s:8>0 r:8<0", strict=True, timeout_s=5)


def test_unanswered_recv_hits_the_deadline():
    """Without the strict checks a stuck wait ends at the deadline (the pre-strict behaviour)."""
    t0 = time.time()
    with pytest.raises(NativeError, match="no progress"):
        loopback_exercise(2, "ri<1|ba", strict=False, timeout_s=1.0)
    assert 0.9 < time.time() - t0 < 10


@pytest.mark.parametrize("topology,world", [("star", 2), ("star", 3), ("star", 8), ("tree", 2), ("tree", 4),
                                            ("tree", 8)])
def test_cascade_call_sequence_is_rccl_valid(topology, world):
    """The cascade driver's own call sequence passes the strict transport at the P the 8-GPU run uses
    (the default transport of every CPU / GPU-loopback cascade test is strict)."""
    tr = synthetic_mnist(1600, seed=5)
    r = CascadeSVM(SVMParams(), topology=topology, comm_timeout_s=60).fit(tr.X, tr.y, world=world).result
    assert r.converged and len(r.ids) > 0
    assert {s["rank"] for s in r.solves} == set(range(world))
