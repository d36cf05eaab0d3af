"""Python mirror of Crossbow's ``TheGPU`` model-path natives.

Same method names, argument meaning and call order as
``src/main/java/uk/ac/imperial/lsds/crossbow/device/TheGPU.java:268-354``,
bound to ``libcrossbow_sma.so`` through its C-ABI (include/crossbow_sma.h)
instead of JNI.  Where the reference would print and ``exit(1)``
(clib-multigpu/debug.h:37-57) these methods raise :class:`CbxError`.

Extra helpers (snake_case) expose what the Java side reaches only through
other natives: buffer upload/download, pinned staging and timing.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import CbxError, check  # noqa: F401


def _ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)



def _java_int(what: str, v: int) -> None:
    # The natives take Java ints (TheGPU.java:268-271; model.h:35 `int bytes`):
    # a model is at most 2^31 - 1 bytes.  ctypes would wrap a larger value silently.
    if not -2**31 <= v < 2**31:
        raise CbxError(_lib.CBX_ERR_INVALID, f"{what} {v} does not fit a Java int (models are < 2 GiB)")

class TheGPU:
    """One execution context (the reference's process-global ``theGPU``)."""

    def __init__(self):
        self._L = _lib.load()
        self._ctx = ctypes.c_void_p()
        self._capacity = {}  # (op id, order) -> bytes setModelVariableBuffer copies

    # ---- lifecycle ------------------------------------------------------
    @staticmethod
    def device_count() -> int:
        n = ctypes.c_int(0)
        check(_lib.load().cbx_device_count(ctypes.byref(n)))
        return n.value

    def init(self, devices: Sequence[int]) -> int:
        """TheGPU.init (GPU.c:21-63): one process drives ``devices``."""
        arr = (ctypes.c_int * len(devices))(*devices)
        return check(self._L.cbx_init(ctypes.byref(self._ctx), arr, len(devices)))

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_ubyte * 128)()
        check(_lib.load().cbx_get_unique_id(buf))
        return bytes(buf)

    def init_rank(self, device: int, nranks: int, rank: int, unique_id: Optional[bytes]) -> int:
        """One process per GPU: rank ``rank`` of ``nranks`` drives ``device``."""
        uid = None
        if unique_id is not None:
            uid = (ctypes.c_ubyte * 128).from_buffer_copy(unique_id)
        return check(self._L.cbx_init_rank(ctypes.byref(self._ctx), device, nranks, rank, uid))

    def free(self) -> int:
        if self._ctx:
            rc = self._L.cbx_free(self._ctx)
            self._ctx = ctypes.c_void_p()
            return check(rc)
        return 0

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.free()

    @property
    def ctx(self):
        return self._ctx

    # ---- model registration (Model.GPURegister, Model.java:338-371) -------
    def setModel(self, variables: int, size: int) -> int:
        _java_int("setModel size", size)
        return check(self._L.cbx_set_model(self._ctx, variables, size))

    def setModelVariable(self, id: int, order: int, shape: Sequence[int], capacity: int) -> int:
        _java_int("setModelVariable capacity", capacity)
        arr = (ctypes.c_int * max(1, len(shape)))(*shape)
        rc = check(self._L.cbx_set_model_variable(self._ctx, id, order, len(shape), arr, capacity))
        self._capacity[(id, order)] = capacity
        return rc

    def setModelVariableBuffer(self, id: int, order: int, buffer) -> int:
        # The library copies the variable's whole capacity from the buffer
        # (executioncontext.c:1583-1590, a direct ByteBuffer of that size on the
        # Java side): a shorter Python buffer would be over-read, so refuse it.
        a = np.ascontiguousarray(np.frombuffer(memoryview(buffer).cast("B"), dtype=np.uint8))
        need = self._capacity.get((id, order))
        if need is not None and a.nbytes < need:
            raise CbxError(_lib.CBX_ERR_INVALID, f"variable ({id}, {order}) buffer of {a.nbytes} bytes is shorter "
                                                 f"than its capacity of {need} bytes")
        return check(self._L.cbx_set_model_variable_buffer(self._ctx, id, order, _ptr(a)))

    def setModelVariableLearningRateMultiplier(self, id: int, order: int, multiplier: float) -> int:
        return check(self._L.cbx_set_model_variable_learning_rate_multiplier(self._ctx, id, order, multiplier))

    def setModelWorkPerClock(self, wpc: int) -> int:
        return check(self._L.cbx_set_model_work_per_clock(self._ctx, wpc))

    def setUpdateModelType(self, type: int) -> int:
        return check(self._L.cbx_set_update_model_type(self._ctx, type))

    # ---- solver (SolverConf.GPURegister, SolverConf.java:355-409) ----------
    def setLearningRateDecayPolicyFixed(self, rate: float) -> int:
        return check(self._L.cbx_set_learning_rate_decay_policy_fixed(self._ctx, rate))

    def setLearningRateDecayPolicyInv(self, rate: float, gamma: float, power: float) -> int:
        return check(self._L.cbx_set_learning_rate_decay_policy_inv(self._ctx, rate, gamma, power))

    def setLearningRateDecayPolicyStep(self, rate: float, gamma: float, step: int) -> int:
        return check(self._L.cbx_set_learning_rate_decay_policy_step(self._ctx, rate, gamma, step))

    def setLearningRateDecayPolicyMultiStep(self, rate: float, gamma: float, warmup: int, steps: Sequence[int]) -> int:
        arr = (ctypes.c_int * max(1, len(steps)))(*steps)
        return check(self._L.cbx_set_learning_rate_decay_policy_multistep(self._ctx, rate, gamma, warmup,
                                                                           len(steps), arr))

    def setLearningRateDecayPolicyExp(self, rate: float, gamma: float) -> int:
        return check(self._L.cbx_set_learning_rate_decay_policy_exp(self._ctx, rate, gamma))

    def setLearningRateDecayPolicyCircular(self, rate: Sequence[float], superconvergence: int,
                                           momentum: Sequence[float], step: int) -> int:
        if len(rate) != 3 or len(momentum) != 3:
            raise CbxError(_lib.CBX_ERR_INVALID, "circular policy needs 3 rates and 3 momenta")  # GPU.c:810
        r = (ctypes.c_float * 3)(*rate)
        m = (ctypes.c_float * 3)(*momentum)
        return check(self._L.cbx_set_learning_rate_decay_policy_circular(self._ctx, r, superconvergence, m, step))

    def setBaseModelMomentum(self, momentum: float) -> int:
        return check(self._L.cbx_set_base_model_momentum(self._ctx, momentum))

    def setMomentum(self, momentum: float, method: int = 0) -> int:
        return check(self._L.cbx_set_momentum(self._ctx, momentum, method))

    def setWeightDecay(self, decay: float) -> int:
        return check(self._L.cbx_set_weight_decay(self._ctx, decay))

    def setEamsgdAlpha(self, alpha: float) -> int:
        return check(self._L.cbx_set_eamsgd_alpha(self._ctx, alpha))

    def setEamsgdTau(self, tau: int) -> int:
        return check(self._L.cbx_set_eamsgd_tau(self._ctx, tau))

    # ---- model manager / barrier path -------------------------------------
    def setModelManager(self, size: int, type: int) -> int:
        return check(self._L.cbx_set_model_manager(self._ctx, size, type))

    def lockAny(self) -> int:
        return check(self._L.cbx_lock_any(self._ctx))

    def merge(self, pull: bool) -> int:
        first = ctypes.c_int(-1)
        check(self._L.cbx_merge(self._ctx, 1 if pull else 0, ctypes.byref(first)))
        return first.value

    def synchronise(self, first: int, clock: int, autotune: int, push: bool) -> int:
        return check(self._L.cbx_synchronise(self._ctx, first, clock, autotune, 1 if push else 0))

    def synchronise_staged(self, first: int, clock: int, autotune: int = 0, buckets: int = 8) -> int:
        """stage_in + synchronise + stage_out in one call, pipelined over
        `buckets` so uploads, kernels and downloads overlap (host mirrors
        in, host mirrors out; include/crossbow_sma.h)."""
        return check(self._L.cbx_synchronise_staged(self._ctx, first, clock, autotune, buckets))

    def unlockAny(self) -> int:
        return check(self._L.cbx_unlock_any(self._ctx))

    def checkpointModel(self, directory: str) -> int:
        return check(self._L.cbx_checkpoint_model(self._ctx, directory.encode()))

    def overrideModelData(self, directory: Optional[str]) -> int:
        return check(self._L.cbx_override_model_data(self._ctx, directory.encode() if directory else None))

    def addModel(self) -> int:
        return check(self._L.cbx_add_model(self._ctx))

    def delModel(self) -> int:
        return check(self._L.cbx_del_model(self._ctx))

    # ---- batch-norm running statistics (cudnnbatchnormparams.c:102-222) ------
    def register_batchnorm_stats(self, op: int, elements: int, mean_ptrs: Sequence[int],
                                 var_ptrs: Sequence[int]) -> None:
        """Make BN operator ``op``'s running mean / variance part of the checkpoint.

        ``mean_ptrs[k]`` / ``var_ptrs[k]``: device pointers on local device k (both 0: that
        device holds no copy).  ``checkpointModel`` / ``overrideModelData`` then store / load
        ``gpu-%02d-bn-{avg,var}-%03d.dat`` beside the model files; ``elements == 0`` removes it.
        """
        ndev = check(self._L.cbx_num_local_devices(self._ctx))
        if len(mean_ptrs) != ndev or len(var_ptrs) != ndev:
            raise ValueError(f"one mean / variance pointer per local device ({ndev}) expected")
        mp = (ctypes.c_void_p * ndev)(*mean_ptrs)
        vp = (ctypes.c_void_p * ndev)(*var_ptrs)
        check(self._L.cbx_register_batchnorm_stats(self._ctx, op, elements, mp, vp))

    def average_batchnorm_stats(self, elements: Sequence[int], mean_ptrs: Sequence[int],
                                var_ptrs: Sequence[int], updated: Sequence[int]) -> None:
        """Average every BN layer's running mean/variance across devices.

        ``mean_ptrs[k * layers + l]`` / ``var_ptrs[...]``: device pointers of layer l on
        local device k; ``updated[...]``: that layer ran on that device since the last call.
        """
        L = len(elements)
        el = (ctypes.c_int * max(1, L))(*elements)
        mp = (ctypes.c_void_p * max(1, len(mean_ptrs)))(*mean_ptrs)
        vp = (ctypes.c_void_p * max(1, len(var_ptrs)))(*var_ptrs)
        up = (ctypes.c_int * max(1, len(updated)))(*[1 if u else 0 for u in updated])
        check(self._L.cbx_average_batchnorm_stats(self._ctx, L, el, mp, vp, up))

    # ---- task-side replica access -----------------------------------------
    def replica_lock(self, id: int) -> None:
        check(self._L.cbx_replica_lock(self._ctx, id))

    def replica_unlock(self, id: int) -> None:
        check(self._L.cbx_replica_unlock(self._ctx, id))

    def replica_task_done(self, id: int) -> None:
        check(self._L.cbx_replica_task_done(self._ctx, id))

    def replica_clock(self, id: int) -> int:
        return check(self._L.cbx_replica_clock(self._ctx, id))

    def replica_learning_rate(self, id: int, task: int) -> float:
        r = ctypes.c_float(0.0)
        check(self._L.cbx_replica_learning_rate(self._ctx, id, task, ctypes.byref(r)))
        return r.value

    def replica_optimise(self, id: int, task: int, stream: Optional[int] = None) -> None:
        """crossbowKernelOptimiserSMA (kernels/optimisers/sma.cu:3-100) for one task.

        ``stream`` is a raw hipStream_t handle (e.g. ``torch.cuda.current_stream().cuda_stream``);
        None enqueues on the replica device's synchronisation stream.
        """
        check(self._L.cbx_replica_optimise(self._ctx, id, task, ctypes.c_void_p(stream) if stream else None))

    def task_wait_count(self, local: int = 0) -> int:
        """Entries in the deferred task-stream wait table of a local device (cbx_task_wait_count; at most 64)."""
        return check(self._L.cbx_task_wait_count(self._ctx, local))

    def replica_copy(self, id: int) -> int:
        return check(self._L.cbx_replica_get_copy(self._ctx, id))

    def set_replica_copy(self, id: int, flag: bool) -> None:
        check(self._L.cbx_replica_set_copy(self._ctx, id, 1 if flag else 0))

    def set_replica_disabled(self, id: int, flag: bool) -> bool:
        """Theta-queue disable / enable (thetaqueue.c:182-206): counted, never locked.

        Returns False when a disable found the slot reserved by a task (it stays enabled).
        """
        return check(self._L.cbx_replica_set_disabled(self._ctx, id, 1 if flag else 0)) == 0

    # ---- the theta queue (TheGPU.java:297-299, modelmanager.c:147-204) ----------
    def acquireAccess(self, clock: list) -> Optional[int]:
        """Reserve the next replica (round robin, waits while it is busy); clock[0] := its clock."""
        c = ctypes.c_int(0)
        rid = check(self._L.cbx_acquire_access(self._ctx, ctypes.byref(c)))
        clock[0] = c.value
        return rid

    def upgradeAccess(self, replica_id: Optional[int], clock: list) -> Optional[int]:
        """Refresh clock[0] of a reserved replica; None once it is gone (delModel)."""
        if replica_id is None:
            return None
        c = ctypes.c_int(0)
        if not check(self._L.cbx_upgrade_access(self._ctx, replica_id, ctypes.byref(c))):
            return None
        clock[0] = c.value
        return replica_id

    def release(self, replica_id: int) -> int:
        # GPU.c:923-932: a GPU replica is released by the callback handler, not from Java.
        raise CbxError(_lib.CBX_ERR_STATE, "Cannot release a GPU model replica id object from the GPU")

    def replica_release(self, id: int) -> None:
        """The callback handler's release (modelmanager.c:200-204): unlock + free the slot."""
        check(self._L.cbx_replica_release(self._ctx, id))

    def get_next_or_wait(self, bound: int) -> int:
        """modelmanager.c:147-167: reserve the next replica, wait for clock >= bound, lock it."""
        return check(self._L.cbx_get_next_or_wait(self._ctx, bound))

    def replica_device(self, id: int) -> int:
        return check(self._L.cbx_replica_device(self._ctx, id))

    def replica_is_local(self, id: int) -> bool:
        return bool(check(self._L.cbx_replica_is_local(self._ctx, id)))

    def num_replicas(self) -> int:
        return check(self._L.cbx_num_replicas(self._ctx))

    def num_devices(self) -> int:
        return check(self._L.cbx_num_devices(self._ctx))

    def local_devices(self) -> Iterable[int]:
        k = check(self._L.cbx_num_local_devices(self._ctx))
        return [check(self._L.cbx_local_device_index(self._ctx, j)) for j in range(k)]

    def elements(self) -> int:
        return check(self._L.cbx_model_elements(self._ctx))

    def local_replicas(self) -> Sequence[int]:
        return [i for i in range(self.num_replicas()) if self.replica_is_local(i)]

    # ---- buffers -----------------------------------------------------------
    def replica_buffer(self, id: int, kind: int) -> int:
        """Device pointer of a replica buffer (what the task-side kernels use)."""
        p = ctypes.c_void_p()
        check(self._L.cbx_replica_buffer(self._ctx, id, kind, ctypes.byref(p)))
        return p.value

    def base_buffer(self, device: int, kind: int) -> int:
        p = ctypes.c_void_p()
        check(self._L.cbx_base_buffer(self._ctx, device, kind, ctypes.byref(p)))
        return p.value

    def step_event(self, local: int = 0) -> int:
        """The hipEvent_t (as an int) that marks the end of the last synchronise()."""
        p = ctypes.c_void_p()
        check(self._L.cbx_step_event(self._ctx, local, ctypes.byref(p)))
        return p.value

    def replica_write(self, id: int, kind: int, values: np.ndarray) -> None:
        a = np.ascontiguousarray(values, dtype=np.float32)
        check(self._L.cbx_replica_write(self._ctx, id, kind, _ptr(a), a.nbytes))

    def replica_read(self, id: int, kind: int) -> np.ndarray:
        a = np.empty(self.elements(), dtype=np.float32)
        check(self._L.cbx_replica_read(self._ctx, id, kind, _ptr(a), a.nbytes))
        return a

    def base_write(self, device: int, kind: int, values: np.ndarray) -> None:
        a = np.ascontiguousarray(values, dtype=np.float32)
        check(self._L.cbx_base_write(self._ctx, device, kind, _ptr(a), a.nbytes))

    def base_read(self, device: int, kind: int) -> np.ndarray:
        a = np.empty(self.elements(), dtype=np.float32)
        check(self._L.cbx_base_read(self._ctx, device, kind, _ptr(a), a.nbytes))
        return a

    def replica_host_view(self, id: int, kind: int) -> np.ndarray:
        p = ctypes.c_void_p()
        check(self._L.cbx_replica_host_buffer(self._ctx, id, kind, ctypes.byref(p)))
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_float)), shape=(self.elements(),))

    def base_host_view(self, device: int, kind: int) -> np.ndarray:
        p = ctypes.c_void_p()
        check(self._L.cbx_base_host_buffer(self._ctx, device, kind, ctypes.byref(p)))
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_float)), shape=(self.elements(),))

    def stage_in(self) -> None:
        check(self._L.cbx_stage_in(self._ctx))

    def stage_out(self) -> None:
        check(self._L.cbx_stage_out(self._ctx))

    def wait(self) -> None:
        check(self._L.cbx_wait(self._ctx))

    # ---- measurement -------------------------------------------------------
    def set_timing(self, enable: bool) -> None:
        check(self._L.cbx_set_timing(self._ctx, 1 if enable else 0))

    def last_timing(self, local: int = 0) -> np.ndarray:
        ms = (ctypes.c_float * _lib.T_COUNT)()
        check(self._L.cbx_last_timing(self._ctx, local, ms))
        return np.array(ms[:], dtype=np.float64)

    def timing_history(self, which: int = _lib.T_KERNEL, local: int = 0, max_steps: int = 1024) -> np.ndarray:
        ms = (ctypes.c_float * max_steps)()
        k = check(self._L.cbx_timing_history(self._ctx, local, which, ms, max_steps))
        return np.array(ms[:k], dtype=np.float64)

    def set_kernel_config(self, block: int = 64, blocks_per_cu: int = 0, policy: int = 1, unroll: int = 2) -> None:
        check(self._L.cbx_set_kernel_config(self._ctx, block, blocks_per_cu, policy, unroll))

    def set_kernel_occupancy(self, waves_per_cu: int) -> None:
        check(self._L.cbx_set_kernel_occupancy(self._ctx, waves_per_cu))

    def set_aux_kernel_config(self, block: int = 64, unroll: int = 1, waves_per_cu: int = -1) -> None:
        check(self._L.cbx_set_aux_kernel_config(self._ctx, block, unroll, waves_per_cu))

    def set_barrier_kernel_config(self, block: int, unroll: int, waves_per_cu: int) -> None:
        check(self._L.cbx_set_barrier_kernel_config(self._ctx, block, unroll, waves_per_cu))

    def set_apply_kernel_config(self, block: int, unroll: int, waves_per_cu: int) -> None:
        """Launch geometry of kernel B (Phase C) of the split SMA path."""
        check(self._L.cbx_set_apply_kernel_config(self._ctx, block, unroll, waves_per_cu))

    def set_pipeline_mode(self, mode: int) -> None:
        """0: buckets overlap within a step; 1: also across steps."""
        check(self._L.cbx_set_pipeline_mode(self._ctx, mode))

    def set_cross_wait_stride(self, stride: int) -> None:
        """Mode 1: buckets per cross-step wait of kernel A on last step's kernel B."""
        check(self._L.cbx_set_cross_wait_stride(self._ctx, stride))

    def set_allreduce_group(self, group: int) -> None:
        """Split path: buckets all-reduced behind one wait on the group's last kernel A."""
        check(self._L.cbx_set_allreduce_group(self._ctx, group))

    def set_order_check(self, enable: bool) -> None:
        """Record per-bucket timestamps of split steps (turns timing on); see check_order."""
        check(self._L.cbx_set_order_check(self._ctx, 1 if enable else 0))

    def check_order(self) -> int:
        """Verify the stream order of the last two split steps; returns the steps checked."""
        return check(self._L.cbx_check_order(self._ctx))

    def set_enqueue_threads(self, mode: int) -> None:
        """One process over several devices: 0 and -1 (the default) = one thread enqueues every
        device's step (the reference's), 1 = one thread per device."""
        check(self._L.cbx_set_enqueue_threads(self._ctx, mode))

    def set_allreduce_algorithm(self, algorithm: int) -> None:
        """ALLREDUCE_RCCL (default), ALLREDUCE_PEER (peer reads over xGMI, bucketed like the all-reduce: one
        process over every device, or one process per GPU after peer_export / peer_import) or ALLREDUCE_RSAG
        (reduce-scatter, momentum on the shard, all-gather)."""
        check(self._L.cbx_set_allreduce_algorithm(self._ctx, algorithm))

    def peer_export(self) -> bytes:
        """One process per GPU: this rank's IPC handles for the peer-read all-reduce (cbx_peer_export)."""
        buf = ctypes.create_string_buffer(_lib.PEER_BLOB_BYTES)
        n = ctypes.c_size_t(0)
        check(self._L.cbx_peer_export(self._ctx, buf, ctypes.byref(n)))
        return buf.raw[:n.value]

    def peer_import(self, blobs: Sequence[bytes]) -> None:
        """Every rank's peer_export() blob, in rank order (cbx_peer_import)."""
        if any(len(b) != _lib.PEER_BLOB_BYTES for b in blobs):
            raise CbxError(_lib.CBX_ERR_INVALID, "peer_import: every blob must be PEER_BLOB_BYTES long")
        joined = b"".join(blobs)
        check(self._L.cbx_peer_import(self._ctx, joined, len(blobs)))

    def resync_base(self, root: int = 0) -> None:
        """Every rank: broadcast z and last from `root` and clear the peer-read form's failure state
        (cbx_resync_base); after a failed step every collective step is refused until this runs."""
        check(self._L.cbx_resync_base(self._ctx, root))

    def set_staging_mode(self, mode: int) -> None:
        """synchronise_staged: STAGING_ZEROCOPY (kernels read / write the pinned mirror) or STAGING_DMA (copies)."""
        check(self._L.cbx_set_staging_mode(self._ctx, mode))

    def set_bucket_elements(self, elements: int) -> None:
        check(self._L.cbx_set_bucket_elements(self._ctx, elements))

    def set_force_split(self, force: bool) -> None:
        check(self._L.cbx_set_force_split(self._ctx, 1 if force else 0))

    def fill_synthetic(self, seed: int) -> None:
        check(self._L.cbx_fill_synthetic(self._ctx, seed))

    def bench_copy(self, nbytes: int, iters: int) -> float:
        g = ctypes.c_float(0.0)
        check(self._L.cbx_bench_copy(self._ctx, nbytes, iters, ctypes.byref(g)))
        return g.value
