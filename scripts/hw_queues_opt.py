#!/usr/bin/env python3
"""The replica optimiser step (sma_optimise_kernel) on
ResNet-50 / R = 8, launched the way bench.py launches it, under the
GPU_MAX_HW_QUEUES the caller exports (ROCclr reads it once, at HIP start).
Run it under rocprofv3 --kernel-trace --stats at several queue counts and
compare the kernel's own duration (VERDICT r04 Weak #2: 108 -> 145 us).

  --stream torch : every launch on one torch stream (bench.py's optimiser leg)
  --stream lib   : on the library's sync stream (stream = NULL)
  --extra-streams K : create K more torch streams first (more queues in use)

Prints one JSON line: wall ms per launch (launch gaps included) and the setting.
"""
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
    ap.add_argument("--stream", default="torch",
                    help="torch | torch-hi (priority -1) | hip (hipStreamCreate) | hip-nb (non-blocking) | "
                         "hip-prio<N> (hipStreamCreateWithPriority) | lib (the library's sync stream)")
    ap.add_argument("--extra-streams", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--sma-steps", type=int, default=5)
    ap.add_argument("--aux", default=None, help="block,unroll,waves_per_cu of the optimiser launch (cbx_set_aux_kernel_config)")
    a = ap.parse_args()
    import torch

    from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU
    from crossbow_amd.variables import MODELS, register
    torch.cuda.set_device(0)
    R = 8
    g = TheGPU()
    g.init([0])
    n = register(g, MODELS["resnet50"]())
    g.setUpdateModelType(UPDATE_SMA)
    g.setEamsgdAlpha(0.1)
    g.setMomentum(0.9, 0)
    g.setWeightDecay(1e-4)
    g.setLearningRateDecayPolicyMultiStep(0.1, 0.1, 0, [1 << 30])
    g.setModelManager(R, SYNC_BSP)
    g.fill_synthetic(20190701)
    if a.aux:
        g.set_aux_kernel_config(*[int(x) for x in a.aux.split(",")])
    extra = [torch.cuda.Stream() for _ in range(a.extra_streams)]
    for clock in range(1, a.sma_steps + 1):
        g.lockAny()
        g.synchronise(0, clock, 0, False)
        g.unlockAny()
    g.wait()
    handle = None
    if a.stream == "torch":
        stream = torch.cuda.Stream()
        handle = stream.cuda_stream
    elif a.stream == "torch-hi":
        stream = torch.cuda.Stream(priority=-1)
        handle = stream.cuda_stream
    elif a.stream.startswith("hip"):
        import ctypes
        hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        s = ctypes.c_void_p()
        if a.stream == "hip":
            rc = hip.hipStreamCreate(ctypes.byref(s))
        elif a.stream == "hip-nb":
            rc = hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
        else:
            rc = hip.hipStreamCreateWithPriority(ctypes.byref(s), 1, int(a.stream[len("hip-prio"):]))
        assert rc == 0, rc
        handle = s.value
        lo, hi = ctypes.c_int(), ctypes.c_int()
        hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi))
        prio_range = (lo.value, hi.value)
    task = 0
    for i in range(R):  # warm
        g.replica_optimise(i, task, handle)
        task += 1
    g.wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.rounds):
        for i in range(R):
            g.replica_optimise(i, task, handle)
            task += 1
    g.wait()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / (a.rounds * R)
    print(json.dumps({"stream": a.stream, "aux": a.aux, "priority_range": locals().get("prio_range"), "extra_streams": len(extra), "n": n,
                      "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "wall_ms_per_launch": round(ms, 4),
                      "alg_GBs_wall": round(28 * n / (ms * 1e-3) / 1e9, 1)}), flush=True)
    g.free()


if __name__ == "__main__":
    main()
