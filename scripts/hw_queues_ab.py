#!/usr/bin/env python3
"""A/B of the bucket pipeline at GPU_MAX_HW_QUEUES 4 (HIP's default) against
16 (what bench.py and the Python package set), one MI355X, interleaved.

ROCclr reads GPU_MAX_HW_QUEUES once, when the HIP runtime starts, so every
sample is a fresh process: scripts/pipeline_sweep.py (the G > 1 pipeline
forced at G = 1, one-rank RCCL; ResNet-50, R = 8, momentum 0.9; ms per step,
best of its interleaved passes) alternately under 4 and 16 queues, `--rounds`
times.  Prints every sample and a summary (per configuration: the median of
each setting's samples and 4 / 16) as JSON lines.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--configs", default="1/0/1,8/0/1,8/1/1,8/1/2")
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--variants", default="spans,spans", help="pipeline_sweep.py variants (a repeat = 2nd context)")
    a = ap.parse_args()
    samples = {}
    for r in range(a.rounds):
        for q in (("4", "16") if r % 2 == 0 else ("16", "4")):
            env = dict(os.environ, GPU_MAX_HW_QUEUES=q)
            p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pipeline_sweep.py"), "--configs",
                                a.configs, "--passes", str(a.passes), "--variants", a.variants],
                               env=env, capture_output=True, text=True, timeout=400)
            if p.returncode != 0:
                print(json.dumps({"round": r, "hw_queues": int(q), "error": p.stderr[-1500:]}), flush=True)
                raise SystemExit(p.returncode)
            for line in p.stdout.splitlines():
                if not line.startswith("{"):  # native libraries' banners (RCCL's version line)
                    continue
                d = json.loads(line)
                d.update(round=r, hw_queues=int(q))
                print(json.dumps(d), flush=True)
                key = (d["buckets"], d["mode"], d["stride"], d["variant"])
                samples.setdefault(key, {}).setdefault(int(q), []).append(d["ms_per_step"])
    for key, by_q in sorted(samples.items()):
        m4, m16 = statistics.median(by_q[4]), statistics.median(by_q[16])
        print(json.dumps({"summary": True, "buckets": key[0], "mode": key[1], "stride": key[2], "variant": key[3],
                          "ms_4_queues": round(m4, 4), "ms_16_queues": round(m16, 4),
                          "ratio_4_over_16": round(m4 / m16, 4), "samples_4": by_q[4], "samples_16": by_q[16]}),
              flush=True)


if __name__ == "__main__":
    main()
