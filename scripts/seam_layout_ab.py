#!/usr/bin/env python3
"""Where the sma.c seam's step loses to the context's (bench.py field `seam`):
the seam's buffers are the caller's (one allocation per buffer, each starting
on a 2 MiB boundary) and a step covers a scalar tail (the elements past the
last whole kernel trip) on extra workgroups.  Interleaved A/B over C3 (ResNet-50, R = 8, mu 0.9):

  separate       one torch allocation per buffer (as bench.py's seam leg)
  staggered      one allocation carved into buffers 2 MiB + 4 KiB apart
                 (the context arena's slot stagger)
  *-no-tail      the same with n rounded down to whole kernel trips (no tail)

History (profiles/r02/seam_layout_ab*.json): with the tail as a second,
separate launch, `separate` cost ~20 us more per step than `separate-no-tail`
(0.480 vs 0.461 ms) while `staggered` did not; the tail now rides the bulk
launch on extra workgroups.

Prints one JSON line: ms per step (torch events around back-to-back steps)
per variant, median of 5 interleaved rounds.
"""
from __future__ import annotations

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from crossbow_amd.seam import SmaPlan  # noqa: E402

N = 25_557_032
R = 8
STEPS = 20
ROUNDS = 5


def buffers(n, staggered):
    dev = torch.device("cuda:0")
    count = 2 * R + 2
    if not staggered:
        return [torch.empty(n, device=dev).normal_(0, 0.01) for _ in range(count)], None
    slot = ((n * 4 + (2 << 20) - 1) // (2 << 20)) * (2 << 20) + 4096
    big = torch.empty(slot * count // 4 + 1024, device=dev)
    base = (big.data_ptr() + 4095) // 4096 * 4096
    off = (base - big.data_ptr()) // 4
    views = [big[off + k * slot // 4: off + k * slot // 4 + n].normal_(0, 0.01) for k in range(count)]
    return views, big


def run(variant):
    staggered = variant.startswith("staggered")
    n = N if not variant.endswith("no-tail") else (N // 4096) * 4096
    bufs, keep = buffers(n, staggered)
    z, last, s, w = bufs[0], bufs[1], bufs[2:2 + R], bufs[2 + R:]
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    with SmaPlan([0], n) as plan:
        reps = [(0, w[i].data_ptr(), s[i].data_ptr(), 1, 0) for i in range(R)]

        def one():
            plan.step([stream.cuda_stream], [z.data_ptr()], [last.data_ptr()], reps, 0.1, 0.9)
        for _ in range(3):
            one()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(STEPS):
            one()
        e1.record(stream)
        e1.synchronize()
    del bufs, keep
    torch.cuda.empty_cache()
    return e0.elapsed_time(e1) / STEPS


def main():
    variants = ["separate", "staggered", "separate-no-tail", "staggered-no-tail"]
    if len(sys.argv) > 1:  # --only V: one variant (e.g. under rocprofv3 --kernel-trace)
        variants = [sys.argv[sys.argv.index("--only") + 1]]
    res = {v: [] for v in variants}
    for _ in range(ROUNDS):
        for v in variants:
            res[v].append(run(v))
            print(f"{v}: {res[v][-1]:.4f} ms", file=sys.stderr, flush=True)
    print(json.dumps({"n": N, "R": R, "steps": STEPS, "rounds": ROUNDS,
                      "ms_per_step_median": {v: round(statistics.median(x), 4) for v, x in res.items()},
                      "ms_per_step_all": {v: [round(t, 4) for t in x] for v, x in res.items()}}))


if __name__ == "__main__":
    main()
