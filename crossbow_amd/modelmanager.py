"""Barrier-side caller of the SMA path, mirroring Crossbow's Java ModelManager.

``trySynchronise`` is ``src/main/java/uk/ac/imperial/lsds/crossbow/model/
ModelManager.java:293-353`` with its GPU-only body: lockAny -> synchronise(0,
clock, autotune(), false) -> unlockAny.  ``GPURegister`` is ``:355-358``.

Around it, the same host-side policy as the Java class:

* ``autotune`` (``:257-274``): every ``autotune_interval`` barriers, while
  autotuning is on, compare the performance monitor's throughput with the
  last reading (``hasThroughputImproved``, ``:238-255``); an improvement above
  ``autotune_threshold`` asks the library to add one replica per GPU (+1),
  anything else removes one (-1) and ends autotuning.  ``synchronise`` passes
  that value on, and the library adds / deletes the replicas after the step
  (executioncontext.c:2321-2328).
* the checkpoint step (``:73-80``, ``:276-286``): the checkpoint interval in
  tasks, rounded up to a multiple of the work per clock, then in clocks.  The
  Java barrier has the call commented out (``:340``); ``checkpoint`` is kept
  callable for hosts that want it.

Defaults follow ``SystemConf.java:209-231``: no checkpoints, autotuning off,
threshold 0.1, interval 1.
"""
from __future__ import annotations

from typing import Callable, Optional


class ModelManager:
    def __init__(self, gpu, replicas_per_gpu: int, sync_type: int = 0, *, wpc: int = 1,
                 checkpoint_interval: int = 0, checkpoint_directory: Optional[str] = None,
                 autotune_models: bool = False, autotune_threshold: float = 0.1, autotune_interval: int = 1):
        if wpc <= 0:
            raise ValueError("work per clock must be positive")
        if autotune_interval <= 0:
            raise ValueError("autotune interval must be positive")
        self.gpu = gpu
        self.replicas_per_gpu = replicas_per_gpu
        self.sync_type = sync_type
        # ModelManager.java:73-80: tasks -> clocks, rounded up to a whole clock
        step = checkpoint_interval
        while step % wpc != 0:
            step += 1
        self.checkpoint_step = step // wpc
        self.checkpoint_directory = checkpoint_directory
        self.autotune_models = autotune_models
        self.autotune_threshold = autotune_threshold
        self.autotune_interval = autotune_interval
        self.autotuning = autotune_models  # :84-85
        self.monitor: Optional[Callable[[], float]] = None
        self.throughput = 0.0
        self.step = 0

    def setPerformanceMonitor(self, monitor: Callable[[], float]) -> "ModelManager":
        """``monitor()`` returns the current throughput (PerformanceMonitor.getCurrentThroughput(0))."""
        self.monitor = monitor
        return self

    def GPURegister(self) -> None:
        self.gpu.setModelManager(self.replicas_per_gpu, self.sync_type)

    def hasThroughputImproved(self) -> bool:
        if self.monitor is None:
            raise RuntimeError("error: performance monitor is null")
        current = float(self.monitor())
        delta = 1.0 if self.throughput == 0 else (current - self.throughput) / self.throughput
        self.throughput = current
        return delta > self.autotune_threshold

    def autotune(self) -> int:
        if self.autotune_models and self.autotuning:
            self.step += 1
            if self.step % self.autotune_interval == 0:
                if self.hasThroughputImproved():
                    return 1
                self.autotuning = False
                return -1
        return 0

    def trySynchronise(self, clock: int) -> bool:
        self.gpu.lockAny()
        self.gpu.synchronise(0, clock, self.autotune(), False)
        self.gpu.unlockAny()
        return True

    def checkpoint(self, clock: int) -> bool:
        """ModelManager.java:276-286: checkpoint every ``checkpoint_step`` clocks."""
        if self.checkpoint_step > 0 and clock % self.checkpoint_step == 0:
            if self.checkpoint_directory is None:
                raise RuntimeError("checkpoint interval set without a checkpoint directory")
            self.gpu.checkpointModel(self.checkpoint_directory)
            return True
        return False
