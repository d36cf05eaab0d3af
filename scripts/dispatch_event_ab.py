#!/usr/bin/env python3
"""A/B of how the split pipeline signals its per-bucket events (ResNet-50,
R = 8, mu 0.9, one GPU, one-rank all-reduce, force split): a separate
hipEventRecord after kernel A(k) / B(k) (dispatch_events 0: a context made
with CBX_SEPARATE_EVENT_RECORDS=1) vs the event handed to the kernel's own
dispatch as its stop event (1, the library default).  Both contexts live in
one process; rounds interleave them.  ms per step from the host clock and
the library's device step span.
Writes gpurun_out/dispatch_event_ab.json."""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU, _lib
    from crossbow_amd.variables import MODELS, register
    R, steps, rounds = 8, 30, 5
    gpus, clock = {}, [0]
    for de in (0, 1):
        if de == 0:
            os.environ["CBX_SEPARATE_EVENT_RECORDS"] = "1"
        else:
            os.environ.pop("CBX_SEPARATE_EVENT_RECORDS", None)
        g = TheGPU()
        g.init([0])
        n = register(g, MODELS["resnet50"]())
        g.setUpdateModelType(UPDATE_SMA)
        g.setEamsgdAlpha(0.1)
        g.setMomentum(0.9, 0)
        g.setModelManager(R, SYNC_BSP)
        g.set_force_split(True)
        g.fill_synthetic(1)
        g.set_timing(True)
        gpus[de] = g

    def step(g):
        clock[0] += 1
        g.lockAny()
        g.synchronise(0, clock[0], 0, False)
        g.unlockAny()

    res = {}
    for _ in range(rounds):
        for nb in (4, 8, 16):
            for mode in (0, 1, 2):
                for de, g in gpus.items():
                    g.set_bucket_elements(-(-n // nb))
                    g.set_pipeline_mode(mode)
                    for _ in range(3):
                        step(g)
                    g.wait()
                    t0 = time.perf_counter()
                    for _ in range(steps):
                        step(g)
                    g.wait()
                    ms = (time.perf_counter() - t0) * 1e3 / steps
                    dev = statistics.median(g.timing_history(_lib.T_STEP)[-steps:])
                    res.setdefault((nb, mode, de), []).append((ms, dev))
    for g in gpus.values():
        g.free()
    out = []
    for (nb, mode, de), v in sorted(res.items()):
        row = dict(buckets=nb, mode=mode, dispatch_events=de,
                   wall_ms=round(statistics.median(x[0] for x in v), 4),
                   device_step_ms=round(statistics.median(x[1] for x in v), 4),
                   rounds_wall_ms=[round(x[0], 4) for x in v])
        out.append(row)
        print(json.dumps(row), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "dispatch_event_ab.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
