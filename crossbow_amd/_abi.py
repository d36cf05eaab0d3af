"""The C-ABI of ``libcrossbow_sma.so`` as ctypes data: status codes, constants
and the signature of every function ``include/crossbow_sma.h`` declares.

Torch-free on purpose, so a process can bind a library build without loading
PyTorch's HIP runtime and RCCL (``tests/test_gpu_multirank.py`` loads a build
linked against a loopback collective).  ``crossbow_amd._lib`` is the binding
the package uses.
"""
from __future__ import annotations

import ctypes

CBX_OK = 0
CBX_ERR_INVALID = -1
CBX_ERR_STATE = -2
CBX_ERR_HIP = -3
CBX_ERR_RCCL = -4
CBX_ERR_IO = -5
CBX_ERR_NO_DEVICE = -6
CBX_ERR_BARRIER = -7
CBX_ERR_UNSUPPORTED = -8

ERROR_NAMES = {
    CBX_ERR_INVALID: "CBX_ERR_INVALID", CBX_ERR_STATE: "CBX_ERR_STATE", CBX_ERR_HIP: "CBX_ERR_HIP",
    CBX_ERR_RCCL: "CBX_ERR_RCCL", CBX_ERR_IO: "CBX_ERR_IO", CBX_ERR_NO_DEVICE: "CBX_ERR_NO_DEVICE",
    CBX_ERR_BARRIER: "CBX_ERR_BARRIER", CBX_ERR_UNSUPPORTED: "CBX_ERR_UNSUPPORTED",
}

BUF_DATA, BUF_GRADIENT, BUF_DIFF, BUF_LAST = 0, 1, 2, 3
T_KERNEL, T_ALLREDUCE, T_APPLY, T_STEP, T_H2D, T_D2H, T_COUNT = range(7)
SYNC_BSP, SYNC_SSP, SYNC_ASP = 0, 1, 2
UPDATE_DEFAULT, UPDATE_WORKER, UPDATE_SYNCHRONOUSEAMSGD, UPDATE_SMA = 0, 1, 3, 7
ALLREDUCE_RCCL, ALLREDUCE_PEER, ALLREDUCE_RSAG = 0, 1, 2
PEER_BLOB_BYTES = 256  # CBX_PEER_BLOB_BYTES
STAGING_ZEROCOPY, STAGING_DMA = 0, 1


class CbxError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {message}")
        self.code = code


_c = ctypes
_P = _c.c_void_p
_PP = _c.POINTER(_c.c_void_p)
_I = _c.c_int
_F = _c.c_float
_D = _c.c_double
_S = _c.c_size_t
_IP = _c.POINTER(_c.c_int)
_FP = _c.POINTER(_c.c_float)
_CP = _c.c_char_p
_UB = _c.POINTER(_c.c_ubyte)

# name -> (restype, argtypes); mirrors include/crossbow_sma.h one to one.
SIGNATURES = {
    "cbx_abi_version": (_I, []),
    "cbx_last_error": (_CP, []),
    "cbx_device_count": (_I, [_IP]),
    "cbx_init": (_I, [_PP, _IP, _I]),
    "cbx_get_unique_id": (_I, [_UB]),
    "cbx_init_rank": (_I, [_PP, _I, _I, _I, _UB]),
    "cbx_free": (_I, [_P]),
    "cbx_set_model": (_I, [_P, _I, _I]),
    "cbx_set_model_variable": (_I, [_P, _I, _I, _I, _IP, _I]),
    "cbx_set_model_variable_buffer": (_I, [_P, _I, _I, _P]),
    "cbx_set_model_variable_learning_rate_multiplier": (_I, [_P, _I, _I, _F]),
    "cbx_set_model_work_per_clock": (_I, [_P, _I]),
    "cbx_set_update_model_type": (_I, [_P, _I]),
    "cbx_set_learning_rate_decay_policy_fixed": (_I, [_P, _F]),
    "cbx_set_learning_rate_decay_policy_inv": (_I, [_P, _F, _D, _D]),
    "cbx_set_learning_rate_decay_policy_step": (_I, [_P, _F, _D, _I]),
    "cbx_set_learning_rate_decay_policy_multistep": (_I, [_P, _F, _D, _I, _I, _IP]),
    "cbx_set_learning_rate_decay_policy_exp": (_I, [_P, _F, _D]),
    "cbx_set_learning_rate_decay_policy_circular": (_I, [_P, _FP, _I, _FP, _I]),
    "cbx_set_base_model_momentum": (_I, [_P, _F]),
    "cbx_set_momentum": (_I, [_P, _F, _I]),
    "cbx_set_weight_decay": (_I, [_P, _F]),
    "cbx_set_eamsgd_alpha": (_I, [_P, _F]),
    "cbx_set_eamsgd_tau": (_I, [_P, _I]),
    "cbx_set_model_manager": (_I, [_P, _I, _I]),
    "cbx_lock_any": (_I, [_P]),
    "cbx_merge": (_I, [_P, _I, _IP]),
    "cbx_synchronise": (_I, [_P, _I, _I, _I, _I]),
    "cbx_synchronise_staged": (_I, [_P, _I, _I, _I, _I]),
    "cbx_unlock_any": (_I, [_P]),
    "cbx_checkpoint_model": (_I, [_P, _CP]),
    "cbx_override_model_data": (_I, [_P, _CP]),
    "cbx_register_batchnorm_stats": (_I, [_P, _I, _I, _PP, _PP]),
    "cbx_add_model": (_I, [_P]),
    "cbx_del_model": (_I, [_P]),
    "cbx_average_batchnorm_stats": (_I, [_P, _I, _IP, _PP, _PP, _IP]),
    "cbx_replica_lock": (_I, [_P, _I]),
    "cbx_replica_unlock": (_I, [_P, _I]),
    "cbx_replica_task_done": (_I, [_P, _I]),
    "cbx_replica_clock": (_I, [_P, _I]),
    "cbx_replica_learning_rate": (_I, [_P, _I, _I, _FP]),
    "cbx_replica_optimise": (_I, [_P, _I, _I, _P]),
    "cbx_replica_get_copy": (_I, [_P, _I]),
    "cbx_replica_set_copy": (_I, [_P, _I, _I]),
    "cbx_acquire_access": (_I, [_P, _IP]),
    "cbx_upgrade_access": (_I, [_P, _I, _IP]),
    "cbx_get_next_or_wait": (_I, [_P, _I]),
    "cbx_replica_release": (_I, [_P, _I]),
    "cbx_replica_set_disabled": (_I, [_P, _I, _I]),
    "cbx_replica_device": (_I, [_P, _I]),
    "cbx_replica_is_local": (_I, [_P, _I]),
    "cbx_num_replicas": (_I, [_P]),
    "cbx_num_devices": (_I, [_P]),
    "cbx_num_local_devices": (_I, [_P]),
    "cbx_local_device_index": (_I, [_P, _I]),
    "cbx_model_elements": (_c.c_longlong, [_P]),
    "cbx_replica_buffer": (_I, [_P, _I, _I, _PP]),
    "cbx_base_buffer": (_I, [_P, _I, _I, _PP]),
    "cbx_replica_write": (_I, [_P, _I, _I, _P, _S]),
    "cbx_replica_read": (_I, [_P, _I, _I, _P, _S]),
    "cbx_base_write": (_I, [_P, _I, _I, _P, _S]),
    "cbx_base_read": (_I, [_P, _I, _I, _P, _S]),
    "cbx_stage_in": (_I, [_P]),
    "cbx_stage_out": (_I, [_P]),
    "cbx_replica_host_buffer": (_I, [_P, _I, _I, _PP]),
    "cbx_base_host_buffer": (_I, [_P, _I, _I, _PP]),
    "cbx_wait": (_I, [_P]),
    "cbx_task_wait_count": (_I, [_P, _I]),
    "cbx_step_event": (_I, [_P, _I, _PP]),
    "cbx_set_timing": (_I, [_P, _I]),
    "cbx_last_timing": (_I, [_P, _I, _FP]),
    "cbx_timing_history": (_I, [_P, _I, _I, _FP, _I]),
    "cbx_set_kernel_config": (_I, [_P, _I, _I, _I, _I]),
    "cbx_set_kernel_occupancy": (_I, [_P, _I]),
    "cbx_set_aux_kernel_config": (_I, [_P, _I, _I, _I]),
    "cbx_set_barrier_kernel_config": (_I, [_P, _I, _I, _I]),
    "cbx_set_apply_kernel_config": (_I, [_P, _I, _I, _I]),
    "cbx_set_pipeline_mode": (_I, [_P, _I]),
    "cbx_set_cross_wait_stride": (_I, [_P, _I]),
    "cbx_set_allreduce_group": (_I, [_P, _I]),
    "cbx_set_allreduce_algorithm": (_I, [_P, _I]),
    "cbx_peer_export": (_I, [_P, _P, _c.POINTER(_S)]),
    "cbx_peer_import": (_I, [_P, _P, _I]),
    "cbx_resync_base": (_I, [_P, _I]),
    "cbx_set_staging_mode": (_I, [_P, _I]),
    "cbx_set_bucket_elements": (_I, [_P, _c.c_longlong]),
    "cbx_set_force_split": (_I, [_P, _I]),
    "cbx_set_enqueue_threads": (_I, [_P, _I]),
    "cbx_set_order_check": (_I, [_P, _I]),
    "cbx_check_order": (_I, [_P]),
    "cbx_fill_synthetic": (_I, [_P, _c.c_ulonglong]),
    "cbx_bench_copy": (_I, [_P, _S, _I, _FP]),
    "cbx_sma_plan_create": (_I, [_PP, _IP, _I, _c.c_longlong, _PP]),
    "cbx_sma_plan_free": (_I, [_P]),
    "cbx_sma_plan_set_buckets": (_I, [_P, _I]),
    "cbx_sma_plan_step": (_I, [_P, _PP, _PP, _PP, _I, _IP, _PP, _PP, _IP, _IP, _F, _F, _I]),
    "cbx_sma_optimise_buffers": (_I, [_P, _P, _P, _P, _P, _c.c_longlong, _F, _F, _F]),
    "cbx_sma_plan_average_batchnorm": (_I, [_P, _I, _IP, _PP, _PP, _IP]),
    "cbx_ssgd_plan_step": (_I, [_P, _PP, _PP, _PP, _PP, _I, _IP, _PP, _IP, _F, _I, _I]),
    "cbx_ssgd_accumulate_buffers": (_I, [_P, _P, _P, _P, _c.c_longlong, _F, _F]),
}


def bind(lib):
    """Set restype/argtypes of every declared function on a loaded CDLL."""
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib
