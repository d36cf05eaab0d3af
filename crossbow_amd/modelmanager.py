"""Barrier-side caller of the SMA path, mirroring Crossbow's Java ModelManager.

``trySynchronise`` is ``src/main/java/uk/ac/imperial/lsds/crossbow/model/
ModelManager.java:293-353`` with its GPU-only body: lockAny -> synchronise(0,
clock, autotune(), false) -> unlockAny.  ``GPURegister`` is ``:355-358``.
"""
from __future__ import annotations

from .thegpu import TheGPU


class ModelManager:
    def __init__(self, gpu: TheGPU, replicas_per_gpu: int, sync_type: int = 0):
        self.gpu = gpu
        self.replicas_per_gpu = replicas_per_gpu
        self.sync_type = sync_type
        self.autotuning = False

    def GPURegister(self) -> None:
        self.gpu.setModelManager(self.replicas_per_gpu, self.sync_type)

    def autotune(self) -> int:
        # ModelManager.java:257-274; autotuning is off by default (SystemConf.java:228).
        return 0

    def trySynchronise(self, clock: int) -> bool:
        self.gpu.lockAny()
        self.gpu.synchronise(0, clock, self.autotune(), False)
        self.gpu.unlockAny()
        return True
