#!/usr/bin/env python3
"""The bucketed peer-read form against its one-bucket step, a fresh process
per sample (scripts/peer_sweep.py; one process over G "devices" that are all
device 0: a rehearsal, not an N-GPU measurement), `--rounds` times per G,
variants (library experiment toggles, scripts/peer_sweep.py) alternating.
Round 4 compared "default" with "norelay" ($CBX_EXP_PEER_NO_RELAY, since
removed with the relay it switched off) at GPU_MAX_HW_QUEUES = 4 x G
(profiles/r04/peer_ab.jsonl: 32 queues at G = 8 made every step ~5x slower,
the hardware scheduler oversubscribed); the default is now 16.  Every sample
and a summary (per G and configuration: the median of each variant's
samples, and each configuration against the variant's 1-bucket step) as
JSON lines."""
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
    ap.add_argument("--G", default="2,8")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--configs", default="1/0/1/1,4/0/1/1,8/0/1/1,4/1/1/1,8/1/1/1,8/1/2/1")
    ap.add_argument("--variants", default="default")
    ap.add_argument("--hw-queues", type=int, default=16)
    ap.add_argument("--passes", type=int, default=1)
    a = ap.parse_args()
    samples = {}
    variants = a.variants.split(",")
    for G in (int(x) for x in a.G.split(",")):
        for r in range(a.rounds):
            for v in (variants if r % 2 == 0 else variants[::-1]):
                env = dict(os.environ, GPU_MAX_HW_QUEUES=str(a.hw_queues))
                p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "peer_sweep.py"), "--G", str(G),
                                    "--configs", a.configs, "--variants", v, "--passes", str(a.passes)],
                                   env=env, capture_output=True, text=True, timeout=600)
                if p.returncode != 0:
                    print(json.dumps({"G": G, "round": r, "variant": v, "error": p.stderr[-1500:]}), flush=True)
                    raise SystemExit(p.returncode)
                for line in p.stdout.splitlines():
                    if not line.startswith('{"G"'):
                        continue
                    d = json.loads(line)
                    d["round"] = r
                    print(json.dumps(d), flush=True)
                    key = (G, d["buckets"], d["mode"], d["stride"], d["group"])
                    samples.setdefault(key, {}).setdefault(v, []).append(d["ms_per_step"])
    for key, by_v in sorted(samples.items()):
        G = key[0]
        one = samples.get((G, 1, 0, 1, 1), {})
        out = {"summary": True, "G": G, "buckets": key[1], "mode": key[2], "stride": key[3], "group": key[4]}
        for v, xs in by_v.items():
            m = statistics.median(xs)
            out[f"ms_{v}"] = round(m, 4)
            if one.get(v):
                out[f"vs_1_bucket_{v}"] = round(m / statistics.median(one[v]), 4)
            out[f"samples_{v}"] = xs
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
