#!/usr/bin/env python3
"""Launch shapes for the small C2 step (LeNet, n = 1,111,946, R = 4, mu 0):
8 contexts used in rotation (720 MB, so HBM rather than the 256 MB Infinity
Cache), HIP-event kernel time per launch, interleaved over rounds.  A 62 MB
step is a ~10-20 us launch: ramp-up and drain, not bandwidth, set its time.
Writes gpurun_out/lenet_sweep.json."""
from __future__ import annotations

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

# (block, unroll, waves-per-CU cap, blocks per CU: 0 = one element group per
# lane, else a grid-stride loop over a grid of that many blocks per CU, so
# waves desynchronise and one iteration's stores overlap the next one's loads)
SHAPES = [(64, 2, -1, 0), (64, 1, -1, 0), (128, 1, -1, 0), (256, 1, -1, 0), (256, 2, -1, 0), (128, 2, -1, 0),
          (64, 4, -1, 0), (256, 4, -1, 0), (64, 2, 4, 0), (256, 1, 8, 0),
          (64, 1, 0, 16), (64, 1, 0, 8), (64, 1, 0, 4), (64, 2, 0, 8), (64, 2, 0, 4), (64, 2, 0, 2),
          (256, 1, 0, 4), (256, 1, 0, 2), (256, 1, 0, 1)]


def main():
    from configs import make, run
    from crossbow_amd import _lib
    n = 1_111_946
    nbytes = (12 * 4 + 8) * n
    gs = [make("lenet", 4, 0.0, False)[0] for _ in range(8)]
    steps, rounds = 20, int(os.environ.get("ROUNDS", "3"))
    shapes = SHAPES
    if os.environ.get("SHAPES"):  # e.g. "64,2,-1,0;64,1,0,8"
        shapes = [tuple(int(x) for x in t.split(",")) for t in os.environ["SHAPES"].split(";")]
    res = {s: [] for s in shapes}
    for _ in range(rounds):
        for shape in shapes:
            block, unroll, cap, bpc = shape
            for g in gs:
                g.set_kernel_config(block, bpc, 1, unroll)
                g.set_kernel_occupancy(cap)
            run(gs, 3)
            run(gs, steps)
            res[shape].append(statistics.median(
                statistics.median(g.timing_history(_lib.T_KERNEL)[-steps:]) for g in gs))
    rows = []
    for (block, unroll, cap, bpc), ms in res.items():
        med = statistics.median(ms)
        rows.append(dict(block=block, unroll=unroll, cap=cap, blocks_per_cu=bpc, us=round(med * 1e3, 2),
                         GBs=round(nbytes / (med * 1e-3) / 1e9, 1)))
        print(json.dumps(rows[-1]), flush=True)
    for g in gs:
        g.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "lenet_sweep.json"), "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
