#!/usr/bin/env python3
"""CPU baseline (oracle/ OpenBLAS replay of the reference call sequence,
clib-multigpu/synch/sma.c:13-231) for the BASELINE configs C1-C3 on the GPU
box's host: 1 thread pinned to core 0 (BLAS.c:32, TheCPU.bind(0)) and 16
threads (the box's CPU share).  Test/measurement infrastructure only."""
from __future__ import annotations

import json
import os
import platform
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(O, n, R, mu, threads, seconds):
    O.blas_open()
    O.blas_set_threads(threads)
    st = O.make_state(n, 1, R, 0.1, mu)
    if threads == 1:
        O.bind_core(0)
    try:
        O.sma_step_blas(st)
        steps, t0 = 0, O.now()
        while True:
            O.sma_step_blas(st)
            steps += 1
            el = O.now() - t0
            if el >= seconds:
                break
    finally:
        if threads == 1:
            O.unbind()
        O.blas_set_threads(1)
    m = 1 if mu > 0 else 0
    return round((12 * R + 8 + 8 * m) * n * steps / el / 1e9, 2), steps, round(el, 2)


def main():
    from oracle import oracle as O
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    cfgs = [("C1 LeNet R=2 mu 0", 1_111_946, 2, 0.0, 1_111_946),
            ("C2 LeNet R=4 mu 0", 1_111_946, 4, 0.0, 1_111_946),
            ("C3 ResNet-50 R=8 mu 0.9 (sample: 4,194,304 elements)", 25_557_032, 8, 0.9, 1 << 22)]
    for name, n_full, R, mu, n in cfgs:
        for threads in (1, 16):
            gbs, steps, el = run(O, n, R, mu, threads, 4.0)
            print(json.dumps({"config": name, "threads": threads, "GBs": gbs, "steps": steps, "seconds": el,
                              "cpu": model, "blas": os.path.basename(O.openblas_path() or "")}), flush=True)


if __name__ == "__main__":
    main()
