"""The model manager's theta queue through the C-ABI (run with -m gpu).

Reference: clib-multigpu/thetaqueue.c (slots FREE / BUSY / SKIP, round-robin
GetNext, CAS reserve / release), modelmanager.c:147-204 (acquireAccess,
upgradeAccess, GetNextOrWait, Release) and TaskProcessor.java:90-120 (the
caller).  The queue is host logic, but it lives in a context that needs the
GPU, hence the marker.
"""
from __future__ import annotations

import threading
import time

import pytest

from crossbow_amd import CbxError
from crossbow_amd import _abi
from tests.helpers import make_gpu

pytestmark = pytest.mark.gpu


def _task(g, rid):
    # execute (crossbowModelManagerGet, modelmanager.c:169-178) ... callback
    # (callbackhandler.c:154-155: updates++, Release).
    g.replica_lock(rid)
    g.replica_task_done(rid)
    g.replica_release(rid)


def test_acquire_round_robin_and_release():
    g = make_gpu(4096, 3, 0.1, 0.0)
    try:
        clock = [-1]
        got = [g.acquireAccess(clock) for _ in range(3)]
        assert got == [0, 1, 2] and clock == [0]  # GetNext starts at slot 0 (iter = -1)
        assert g.upgradeAccess(1, clock) == 1 and clock == [0]
        for rid in got:
            _task(g, rid)
        # Released slots come round again, in order.
        assert [g.acquireAccess(clock) for _ in range(3)] == [0, 1, 2]
        for rid in (0, 1, 2):
            _task(g, rid)
        assert g.acquireAccess(clock) == 0
        _task(g, 0)
        # A slot nobody reserved cannot be released (the reference would spin).
        with pytest.raises(CbxError, match="not reserved"):
            g.replica_release(1)
        # upgradeAccess(null) is null (TaskProcessor.java:112-114 re-acquires).
        assert g.upgradeAccess(None, clock) is None
    finally:
        g.free()


def test_acquire_waits_for_a_busy_slot():
    g = make_gpu(4096, 2, 0.1, 0.0)
    try:
        clock = [0]
        assert g.acquireAccess(clock) == 0
        assert g.acquireAccess(clock) == 1
        out = []
        t = threading.Thread(target=lambda: out.append(g.acquireAccess([0])), daemon=True)
        t.start()
        time.sleep(0.2)
        assert t.is_alive() and not out  # next in turn is slot 0, still busy
        _task(g, 0)
        t.join(10)
        assert out == [0]
        _task(g, 0)
        _task(g, 1)
    finally:
        g.free()


def test_disabled_slots_are_skipped_and_counted():
    g = make_gpu(4096, 3, 0.1, 0.0)
    try:
        assert g.set_replica_disabled(1, True)
        clock = [0]
        assert [g.acquireAccess(clock) for _ in range(2)] == [0, 2]
        # A reserved slot stays enabled (thetaqueue.c:199-201) ...
        assert not g.set_replica_disabled(0, True)
        # ... and cannot be re-enabled either (:182-184: invalid state).
        with pytest.raises(CbxError, match="reserved"):
            g.set_replica_disabled(0, False)
        _task(g, 0)
        _task(g, 2)
        # lockAny counts the disabled replica without locking it (modelmanager.c:217-222).
        assert g.lockAny() == 3
        g.synchronise(0, 1, 0, False)
        assert g.unlockAny() == 2
        assert g.replica_clock(1) == 0 and g.replica_clock(0) == 1
        # Every slot disabled: an error, where the reference spins forever.
        assert g.set_replica_disabled(0, True) and g.set_replica_disabled(2, True)
        with pytest.raises(CbxError) as e:
            g.acquireAccess(clock)
        assert e.value.code == _abi.CBX_ERR_STATE
        for rid in range(3):
            assert g.set_replica_disabled(rid, False)
        assert g.acquireAccess(clock) in (0, 1, 2)
    finally:
        g.free()


def test_deleted_replica_upgrades_to_null():
    # delModel removes the last replica of every device and disables its slot
    # (modelmanager.c:537); a task processor still holding it re-acquires.
    g = make_gpu(4096, 3, 0.1, 0.0)
    try:
        clock = [0]
        assert [g.acquireAccess(clock) for _ in range(3)] == [0, 1, 2]
        _task(g, 0)
        _task(g, 1)
        g.lockAny()
        g.synchronise(0, 1, -1, False)  # autotune -1: delModel
        g.unlockAny()
        assert g.num_replicas() == 2
        assert g.upgradeAccess(2, clock) is None
        got = {g.acquireAccess(clock) for _ in range(2)}
        assert got == {0, 1}
        for rid in got:
            _task(g, rid)
        # addModel brings id 2 back with a free slot.
        g.lockAny()
        g.synchronise(0, 2, 1, False)
        g.unlockAny()
        assert g.num_replicas() == 3
        assert sorted(g.acquireAccess(clock) for _ in range(3)) == [0, 1, 2]
    finally:
        g.free()


def test_get_next_or_wait_waits_for_the_clock():
    # modelmanager.c:147-167: reserve, wait for clock >= bound, lock.
    g = make_gpu(4096, 2, 0.1, 0.0)
    try:
        rid = g.get_next_or_wait(0)
        assert rid == 0
        with pytest.raises(CbxError):
            g.lockAny()  # BSP: replica 0 is locked by the task
        g.replica_task_done(rid)
        g.replica_release(rid)
        out = []
        t = threading.Thread(target=lambda: out.append(g.get_next_or_wait(1)), daemon=True)
        t.start()
        time.sleep(0.2)
        assert t.is_alive() and not out  # replica 1's clock is 0 < 1
        # The waiter holds the reservation, not the lock: the barrier runs
        # and advances every clock to 1.
        assert g.lockAny() == 2
        g.synchronise(0, 1, 0, False)
        g.unlockAny()
        t.join(10)
        assert out == [1] and g.replica_clock(1) == 1
        g.replica_release(1)
    finally:
        g.free()
