#!/usr/bin/env python3
"""A/B of the small-launch shape (sma_internal.h, small_launch_shape) on the
C2 step (LeNet, R = 4, mu 0), interleaved over rounds on one box:
  A  occupancy 0    -- a launch under 16 waves per CU runs as before: two
                       float4 per lane, one element group per lane, uncapped;
  B  occupancy auto -- the same launch runs one float4 per lane in a
                       grid-stride loop over 8 one-wave blocks per CU.
Both cache-resident (one context) and HBM (8 contexts in rotation).
Prints one JSON line per case; writes gpurun_out/small_launch_ab.json."""
from __future__ import annotations

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    from configs import make, rate, run
    from crossbow_amd import _lib
    n = 1_111_946
    nbytes = (12 * 4 + 8) * n
    rot = [make("lenet", 4, 0.0, False)[0] for _ in range(8)]
    one = [make("lenet", 4, 0.0, False)[0]]
    steps, rounds = 20, int(os.environ.get("ROUNDS", "10"))
    res = {}
    for _ in range(rounds):
        for label, occ in (("A_old_shape", 0), ("B_small_launch_shape", -1)):
            for name, gs in (("cache_resident", one), ("8_rotated_contexts", rot)):
                for g in gs:
                    g.set_kernel_occupancy(occ)
                run(gs, 3)
                run(gs, steps)
                ms = statistics.median(statistics.median(g.timing_history(_lib.T_KERNEL)[-steps:]) for g in gs)
                res.setdefault((label, name), []).append(ms)
    out = {}
    for (label, name), v in sorted(res.items()):
        out[f"{name}/{label}"] = dict(rate(nbytes, statistics.median(v)), rounds=len(v))
        print(json.dumps({f"{name}/{label}": out[f"{name}/{label}"]}), flush=True)
    for g in rot + one:
        g.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "small_launch_ab.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
