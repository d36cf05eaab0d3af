#!/usr/bin/env python3
"""The peer-read form of the single-process step (cbx_set_allreduce_algorithm
PEER), bucketed: ms per step by bucket count, pipeline mode, wait stride,
all-reduce group and enqueue threads, ResNet-50, R = 8 per device, momentum
0.9, one process over G devices (`--distinct`: devices 0..G-1; default: G
copies of device 0, the one-GPU rehearsal, where every "peer" read is local
and all G devices' kernels share one GPU).  Wall clock over back-to-back
steps, interleaved passes, best pass kept; JSON lines on stdout.

Under `rocprofv3 --kernel-trace` run it with `--passes 1 --gap-ms 50`: the
configurations are then separated by idle gaps that
scripts/peer_trace_summary.py splits the trace at."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=2)
    ap.add_argument("--distinct", action="store_true")
    ap.add_argument("--configs", default="1/0/1/1,8/0/1/1,8/1/1/1,8/1/2/1,4/0/1/1,4/1/1/1",
                    help="buckets/mode/stride/group, comma-separated")
    ap.add_argument("--threads", default="0", help="enqueue threads to time, comma-separated (0, 1)")
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--timing", type=int, default=1)
    ap.add_argument("--gap-ms", type=float, default=0.0, help="host sleep between configurations (trace splitting)")
    ap.add_argument("--variants", default="default",
                    help="comma-separated contexts: 'default', or an experiment toggle of the library set in the "
                         "environment at the context's creation (none at present; round 4's 'norelay' was "
                         "CBX_EXP_PEER_NO_RELAY, profiles/r04/peer_ab.jsonl)")
    a = ap.parse_args()
    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU, _lib
    from crossbow_amd.variables import MODELS, register
    toggles = {"default": None}

    def make(variant):
        env = toggles[variant]
        if env:
            os.environ[env] = "1"
        g = TheGPU()
        g.init(list(range(a.G)) if a.distinct else [0] * a.G)
        if env:
            del os.environ[env]
        n = register(g, MODELS["resnet50"]())
        g.setUpdateModelType(UPDATE_SMA)
        g.setEamsgdAlpha(0.1)
        g.setMomentum(0.9, 0)
        g.setModelManager(8, SYNC_BSP)
        g.set_allreduce_algorithm(_lib.ALLREDUCE_PEER)
        g.fill_synthetic(1)
        g.set_timing(bool(a.timing))
        return g, n

    ctxs = {v: make(v) for v in a.variants.split(",")}
    clock = [0]
    g = None

    def step():
        clock[0] += 1
        g.lockAny()
        g.synchronise(0, clock[0], 0, False)
        g.unlockAny()

    configs = [tuple(int(x) for x in c.split("/")) for c in a.configs.split(",")]
    threads = [int(t) for t in a.threads.split(",")]
    best = {}
    order = []
    for _ in range(a.passes):
        for nb, mode, stride, group in configs:
            for t, variant in [(t, v) for t in threads for v in ctxs]:
                g, n = ctxs[variant]
                g.set_enqueue_threads(t)
                g.set_bucket_elements((1 << 62) if nb == 1 else -(-n // nb))
                g.set_pipeline_mode(mode)
                g.set_cross_wait_stride(stride)
                g.set_allreduce_group(group)
                for _ in range(a.warmup):
                    step()
                g.wait()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    step()
                g.wait()
                ms = (time.perf_counter() - t0) * 1e3 / a.steps
                key = (nb, mode, stride, group, t, variant)
                best[key] = min(ms, best.get(key, ms))
                order.append(key)
                if a.gap_ms > 0:
                    time.sleep(a.gap_ms / 1e3)
    for (nb, mode, stride, group, t, variant), ms in sorted(best.items()):
        print(json.dumps({"G": a.G, "distinct": a.distinct, "buckets": nb, "mode": mode, "stride": stride,
                          "group": group, "enqueue_threads": t, "variant": variant, "timing": a.timing, "steps": a.steps,
                          "warmup": a.warmup, "ms_per_step": round(ms, 4)}), flush=True)
    print(json.dumps({"order": [list(k) for k in order], "steps": a.steps, "warmup": a.warmup}), flush=True)
    for g, _ in ctxs.values():
        g.free()


if __name__ == "__main__":
    main()
