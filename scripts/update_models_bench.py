#!/usr/bin/env python3
"""Run the per-task and barrier kernels of every update model on ResNet-50
parameters (R = 8 replicas, momentum 0.9, weight decay 1e-4) so that
`rocprofv3 --kernel-trace --stats` reports their launch durations:

  SMA      sma_optimise_kernel (task)      + sma_fused_kernel (barrier)
  DEFAULT  default_optimise_kernel (task)  + broadcast_kernel (barrier)
  WORKER   ssgd_accumulate_kernel (task)   + ssgd_apply_kernel (barrier)

Usage: rocprofv3 --kernel-trace --stats -d gpurun_out/upd -o run --output-format csv -- python3 scripts/update_models_bench.py
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from crossbow_amd import SYNC_BSP, UPDATE_DEFAULT, UPDATE_SMA, UPDATE_WORKER, TheGPU
    from crossbow_amd.variables import MODELS, register
    R, clocks = 8, 6
    for utype in (UPDATE_SMA, UPDATE_DEFAULT, UPDATE_WORKER):
        g = TheGPU()
        g.init([0])
        register(g, MODELS["resnet50"]())
        g.setUpdateModelType(utype)
        g.setEamsgdAlpha(0.1)
        g.setMomentum(0.9, 0)
        g.setWeightDecay(1e-4)
        g.setLearningRateDecayPolicyFixed(0.01)
        g.setModelWorkPerClock(R)
        g.setModelManager(R, SYNC_BSP)
        g.fill_synthetic(1)
        task = 0
        for clock in range(1, clocks + 1):
            for i in range(R):
                g.replica_optimise(i, task)
                task += 1
            g.lockAny()
            g.synchronise(0, clock, 0, False)
            g.unlockAny()
        g.wait()
        g.free()
    print("update_models_bench: done", flush=True)


if __name__ == "__main__":
    main()
