"""Host-side policy of the barrier caller (crossbow_amd.modelmanager), no GPU:
the Java ModelManager's trySynchronise call order, autotune decisions and
checkpoint step (ModelManager.java:73-88, 238-286, 293-353), against a
recording stand-in for TheGPU."""
from __future__ import annotations

import pytest

from crossbow_amd.modelmanager import ModelManager


class Recorder:
    def __init__(self):
        self.calls = []

    def __getattr__(self, name):
        def f(*args):
            self.calls.append((name,) + args)
            return 0
        return f


def test_try_synchronise_call_order():
    g = Recorder()
    mm = ModelManager(g, 4, 0)
    mm.GPURegister()
    assert mm.trySynchronise(7)
    assert g.calls == [("setModelManager", 4, 0), ("lockAny",), ("synchronise", 0, 7, 0, False), ("unlockAny",)]


def test_autotune_adds_while_throughput_improves_then_removes_once():
    # hasThroughputImproved: first reading always improves (delta := 1); then
    # relative gain > threshold adds a replica per GPU, anything else removes
    # one and stops autotuning (ModelManager.java:238-274).
    g = Recorder()
    readings = iter([100.0, 120.0, 125.0, 0.0, 0.0])
    mm = ModelManager(g, 2, 0, autotune_models=True, autotune_threshold=0.1, autotune_interval=2)
    mm.setPerformanceMonitor(lambda: next(readings))
    decisions = []
    for clock in range(1, 9):
        mm.trySynchronise(clock)
        decisions.append(g.calls[-2][3])
    # interval 2: decisions at barriers 2, 4, 6; +1 (first), +1 (+20 %), -1 (+4 %), then off
    assert decisions == [0, 1, 0, 1, 0, -1, 0, 0]
    assert not mm.autotuning


def test_autotune_off_by_default_and_needs_a_monitor():
    g = Recorder()
    mm = ModelManager(g, 2, 0)
    mm.trySynchronise(1)
    assert g.calls[-2] == ("synchronise", 0, 1, 0, False)
    mm = ModelManager(g, 2, 0, autotune_models=True)
    with pytest.raises(RuntimeError):
        mm.trySynchronise(1)


@pytest.mark.parametrize("interval,wpc,step", [(0, 4, 0), (8, 4, 2), (9, 4, 3), (10, 1, 10)])
def test_checkpoint_step_rounds_tasks_up_to_clocks(interval, wpc, step):
    g = Recorder()
    mm = ModelManager(g, 1, 0, wpc=wpc, checkpoint_interval=interval, checkpoint_directory="/tmp/ck")
    assert mm.checkpoint_step == step
    done = [c for c in range(1, 13) if mm.checkpoint(c)]
    assert done == ([] if step == 0 else list(range(step, 13, step)))
    assert all(call == ("checkpointModel", "/tmp/ck") for call in g.calls)
