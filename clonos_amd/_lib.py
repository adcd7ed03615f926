"""ctypes binding of libclonos_engine.so (the C-ABI in include/clonos_engine.h).

The library is the only compute path: there is no CPU fallback.  If the library is
missing this module raises at import time; if no GPU is visible, engine creation fails
with CLG_E_DEVICE.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CLONOS_LIB") or os.path.join(HERE, "libclonos_engine.so")  # CLONOS_LIB: A/B builds

# ---- status codes (clonos_engine.h) ------------------------------------------------
CLG_OK = 0
CLG_E_INVALID_ARG = -1
CLG_E_CORRUPT_TAG = -2
CLG_E_TRUNCATED = -3
CLG_E_BAD_ENUM = -4
CLG_E_NEG_LEN = -5
CLG_E_BAD_SERIAL = -6
CLG_E_CONSUMER_BACKWARDS = -7
CLG_E_NO_CONSUMER = -8
CLG_E_GAP = -9
CLG_E_NOSPACE = -10
CLG_E_CAPACITY = -11
CLG_E_STATE = -12
CLG_E_DEVICE = -13
CLG_E_NO_LOG = -14
CLG_E_NOT_BUFFER_BUILT = -15
CLG_E_EPOCH_GAP = -16

STATUS_NAMES = {v: k for k, v in globals().items() if k.startswith("CLG_E_") or k == "CLG_OK"}

CLG_MEM_HOST = 0
CLG_MEM_DEVICE = 1
CLG_MEM_MAPPED = 2  # host memory registered with clg_host_register (the small decode writes it directly)
CLG_F_TIMING = 1
CLG_F_ROBUST_DECODE = 2
CLG_F_ASYNC_SLICE = 4
CLG_F_NO_SMALL_DECODE = 8
CLG_FULL_SHARING = -1
CLG_DECODE_MAX_INFLIGHT = 2  # asynchronous decodes queued before the first wait
CLG_IFL_IN_MEMORY = 0
CLG_IFL_SPILLABLE = 1
CLG_IFL_CONTINUE = 1        # IflReplayReq.flags
CLG_IFL_NULL_ITERATOR = 1   # IflReplayRes.flags
CLG_IFL_REPLAYING = 2       # IflReplayRes.flags

EXPORTED = [
    "clg_config_default", "clg_engine_create", "clg_engine_destroy", "clg_last_error", "clg_abi_version",
    "clg_engine_stream", "clg_gather_stream", "clg_sync", "clg_pool_stats", "clg_ifl_pool_stats", "clg_log_open", "clg_log_close", "clg_log_find", "clg_log_length_batch", "clg_log_get_id",
    "clg_job_open", "clg_job_close",
    "clg_append", "clg_append_batch", "clg_upstream_delta", "clg_log_length", "clg_has_delta",
    "clg_offset_from_epoch", "clg_get_delta", "clg_get_determinants", "clg_notify_checkpoint_complete",
    "clg_unregister_consumer", "clg_log_get_state", "clg_consumer_state", "clg_log_read_phys",
    "clg_slice_batch", "clg_consumer_seek", "clg_consumer_seek_batch", "clg_upstream_delta_batch", "clg_truncate_all", "clg_decode_host", "clg_decode_logs", "clg_decode_logs_async", "clg_decode_wait",
    "clg_replay_prep", "clg_kernel_stats", "clg_kernel_stats_reset",
    "clg_response_put", "clg_response_write", "clg_response_read", "clg_response_merge", "clg_causal_log_id_hash",
    "clg_replay_prepare", "clg_encode_batch", "clg_enrich_batch", "clg_process_delta",
    "clg_ifl_open", "clg_ifl_open_typed", "clg_ifl_close", "clg_ifl_log_batch", "clg_ifl_notify_checkpoint_complete", "clg_ifl_state",
    "clg_ifl_replay_batch", "clg_replay_prepare_device", "clg_get_determinants_batch", "clg_response_put_batch",
    "clg_host_register", "clg_host_unregister",
]


class ClonosError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class ChannelId(C.Structure):
    _fields_ = [("lo", C.c_uint64), ("hi", C.c_uint64)]


class CausalLogIdC(C.Structure):
    _fields_ = [
        ("vertex_id", C.c_int16),
        ("is_main", C.c_uint8),
        ("subpartition", C.c_int8),
        ("reserved", C.c_uint32),
        ("irp_lower", C.c_int64),
        ("irp_upper", C.c_int64),
    ]


class Config(C.Structure):
    _fields_ = [
        ("segment_bytes", C.c_uint32),
        ("pool_segments", C.c_uint32),
        ("device", C.c_int32),
        ("sharing_depth", C.c_int32),
        ("flags", C.c_uint32),
        ("host_tail_bytes", C.c_uint32),
        ("ifl_segment_bytes", C.c_uint32),
        ("ifl_pool_segments", C.c_uint32),
    ]


class LogState(C.Structure):
    _fields_ = [("writer", C.c_int32), ("capacity", C.c_int32), ("n_components", C.c_int32), ("n_epochs", C.c_int32)]


class SliceReq(C.Structure):
    _fields_ = [("log", C.c_uint32), ("reserved", C.c_uint32), ("consumer", ChannelId), ("epoch", C.c_int64)]


class DeltaReq(C.Structure):
    _fields_ = [
        ("log", C.c_uint32),
        ("offset_from_epoch", C.c_int32),
        ("epoch", C.c_int64),
        ("src_off", C.c_uint64),
        ("len", C.c_uint32),
        ("status", C.c_int32),
    ]


class SliceRes(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("has_delta", C.c_int32),
        ("offset_from_epoch", C.c_int32),
        ("len", C.c_int32),
        ("out_off", C.c_uint64),
    ]


class Decoded(C.Structure):
    _fields_ = [
        ("off", C.c_void_p),
        ("tag", C.c_void_p),
        ("v0", C.c_void_p),
        ("w_idx", C.c_void_p),
        ("w_rc", C.c_void_p),
        ("w_v1", C.c_void_p),
        ("w_var_off", C.c_void_p),
        ("w_var_len", C.c_void_p),
        ("w_sub", C.c_void_p),
        ("cap", C.c_uint64),
        ("wcap", C.c_uint64),
        ("out_kind", C.c_uint32),
        ("reserved", C.c_uint32),
        ("n_rec", C.c_uint64),
        ("n_wide", C.c_uint64),
        ("err_status", C.c_int32),
        ("err_span", C.c_uint32),
        ("err_off", C.c_int64),
        ("err_tag", C.c_int32),
        ("reserved2", C.c_uint32),
    ]


class ResponseEntry(C.Structure):
    _fields_ = [("id", CausalLogIdC), ("bytes", C.c_void_p), ("len", C.c_uint64)]


class Response(C.Structure):
    _fields_ = [
        ("found", C.c_int32),
        ("vertex_id", C.c_int16),
        ("reserved", C.c_int16),
        ("correlation_id", C.c_int64),
        ("n", C.c_uint32),
        ("cap", C.c_uint32),
        ("table_cap", C.c_uint32),
        ("reserved2", C.c_uint32),
        ("entries", C.POINTER(ResponseEntry)),
    ]


class ReplayVertex(C.Structure):
    _fields_ = [
        ("acc", C.POINTER(Response)),
        ("subpartitions", C.POINTER(CausalLogIdC)),
        ("n_subpartitions", C.c_uint32),
        ("vertex_id", C.c_int16),
        ("reserved", C.c_int16),
    ]


class ReplayOut(C.Structure):
    _fields_ = [
        ("main", C.POINTER(Decoded)),
        ("main_rec_base", C.c_void_p),
        ("buffer_sizes", C.c_void_p),
        ("sizes_cap", C.c_uint64),
        ("sizes_base", C.c_void_p),
        ("sub_count", C.c_void_p),
        ("sub_status", C.c_void_p),
        ("sub_err_off", C.c_void_p),
        ("sub_err_tag", C.c_void_p),
    ]


class EncodeIn(C.Structure):
    _fields_ = [
        ("tag", C.c_void_p), ("v0", C.c_void_p), ("n", C.c_uint64),
        ("w_idx", C.c_void_p), ("w_rc", C.c_void_p), ("w_v1", C.c_void_p), ("w_var_off", C.c_void_p),
        ("w_var_len", C.c_void_p), ("w_sub", C.c_void_p), ("n_wide", C.c_uint64),
        ("var", C.c_void_p), ("var_len", C.c_uint64), ("in_kind", C.c_uint32), ("reserved", C.c_uint32),
    ]


class EnrichReq(C.Structure):
    _fields_ = [
        ("consumer", ChannelId), ("epoch", C.c_int64), ("first", C.c_uint32), ("count", C.c_uint32),
        ("status", C.c_int32), ("header_bytes", C.c_uint32), ("out_off", C.c_uint64), ("out_len", C.c_uint64),
    ]


CLG_DELTA_FLAT = 0
CLG_DELTA_HIERARCHICAL = 1
CLG_DE_SEND = 1


class IflReplayReq(C.Structure):
    _fields_ = [("ifl", C.c_uint32), ("ignore_buffers", C.c_uint32), ("start_epoch", C.c_int64),
                ("max_buffers", C.c_uint32), ("flags", C.c_uint32)]


class IflReplayRes(C.Structure):
    _fields_ = [
        ("status", C.c_int32), ("n_buffers", C.c_uint32), ("remaining", C.c_uint32), ("flags", C.c_uint32),
        ("out_off", C.c_uint64), ("len", C.c_uint64), ("sizes_off", C.c_uint64), ("end_epoch", C.c_int64),
    ]


class KernelStat(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_uint64), ("total_ms", C.c_double), ("bytes", C.c_uint64)]


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -m clonos_amd.build` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    # One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 (same SONAME as
    # /opt/rocm's) and loads it by a different file name, so whichever of the two comes
    # second would be a second runtime in the process -- and torch's device init then
    # fails ("No HIP GPUs are available") once the engine's has initialised.  Importing
    # torch first makes its runtime the one the engine's NEEDED libamdhip64.so.7 resolves to.
    try:
        import torch  # noqa: F401
    except ImportError:  # a torch-less host: /opt/rocm's runtime
        pass
    lib = C.CDLL(LIB_PATH)
    P = C.c_void_p
    u32p, i32p, u64p, i64p = (C.POINTER(C.c_uint32), C.POINTER(C.c_int32), C.POINTER(C.c_uint64),
                              C.POINTER(C.c_int64))
    sig = {
        "clg_config_default": (None, [C.POINTER(Config)]),
        "clg_engine_create": (C.c_int, [C.POINTER(Config), C.POINTER(P)]),
        "clg_engine_destroy": (None, [P]),
        "clg_last_error": (C.c_char_p, []),
        "clg_abi_version": (C.c_int, []),
        "clg_engine_stream": (P, [P]),
        "clg_gather_stream": (P, [P]),
        "clg_sync": (C.c_int, [P]),
        "clg_pool_stats": (C.c_int, [P, u32p, u32p]),
        "clg_ifl_pool_stats": (C.c_int, [P, u32p, u32p]),
        "clg_log_open": (C.c_int, [P, C.c_uint32, C.POINTER(CausalLogIdC), u32p]),
        "clg_log_close": (C.c_int, [P, C.c_uint32]),
        "clg_log_find": (C.c_int, [P, C.c_uint32, C.POINTER(CausalLogIdC), u32p]),
        "clg_job_open": (C.c_int, [P, C.c_uint64, C.c_uint64, C.c_int32, u32p]),
        "clg_log_length_batch": (C.c_int, [P, P, C.c_uint32, P, u64p]),
        "clg_log_get_id": (C.c_int, [P, C.c_uint32, C.POINTER(CausalLogIdC), u32p]),
        "clg_job_close": (C.c_int, [P, C.c_uint32]),
        "clg_append": (C.c_int, [P, C.c_uint32, C.c_int64, C.c_char_p, C.c_uint32]),
        "clg_append_batch": (C.c_int, [P, P, P, P, P, C.c_uint32, P]),
        "clg_upstream_delta": (C.c_int, [P, C.c_uint32, C.c_int64, C.c_int32, C.c_char_p, C.c_uint32]),
        "clg_log_length": (C.c_int, [P, C.c_uint32, i32p]),
        "clg_has_delta": (C.c_int, [P, C.c_uint32, ChannelId, C.c_int64, i32p]),
        "clg_offset_from_epoch": (C.c_int, [P, C.c_uint32, ChannelId, i32p]),
        "clg_get_delta": (C.c_int, [P, C.c_uint32, ChannelId, C.c_int64, P, C.c_uint32, C.c_uint32, u32p]),
        "clg_get_determinants": (C.c_int, [P, C.c_uint32, C.c_int64, P, C.c_uint32, C.c_uint32, u32p]),
        "clg_notify_checkpoint_complete": (C.c_int, [P, C.c_uint32, C.c_int64]),
        "clg_unregister_consumer": (C.c_int, [P, C.c_uint32, ChannelId]),
        "clg_log_get_state": (C.c_int, [P, C.c_uint32, C.POINTER(LogState), P, P, C.c_int32]),
        "clg_consumer_state": (C.c_int, [P, C.c_uint32, ChannelId, i32p, i64p, i32p]),
        "clg_log_read_phys": (C.c_int, [P, C.c_uint32, C.c_int32, C.c_uint32, P]),
        "clg_slice_batch": (C.c_int, [P, P, C.c_uint32, P, P, C.c_uint64, C.c_uint32, u64p]),
        "clg_consumer_seek": (C.c_int, [P, C.c_uint32, ChannelId, C.c_int64, C.c_int32]),
        "clg_consumer_seek_batch": (C.c_int, [P, P, P, C.c_uint32]),
        "clg_upstream_delta_batch": (C.c_int, [P, P, C.c_uint32, P, C.c_uint32]),
        "clg_truncate_all": (C.c_int, [P, C.c_uint32, C.c_int64, i32p]),
        "clg_decode_host": (C.c_int, [P, P, P, P, C.c_uint32, C.POINTER(Decoded), P]),
        "clg_decode_logs": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(Decoded), P]),
        "clg_decode_logs_async": (C.c_int, [P, P, P, C.c_uint32, C.POINTER(Decoded), P]),
        "clg_decode_wait": (C.c_int, [P]),
        "clg_host_register": (C.c_int, [P, C.c_uint64]),
        "clg_host_unregister": (C.c_int, [P]),
        "clg_replay_prep": (C.c_int, [P, P, P, P, P, C.c_uint32, P, u32p, C.POINTER(Decoded), P]),
        "clg_kernel_stats": (C.c_int, [P, C.POINTER(KernelStat), C.c_uint32, u32p]),
        "clg_kernel_stats_reset": (C.c_int, [P]),
        "clg_response_put": (C.c_int, [C.POINTER(Response), C.POINTER(CausalLogIdC), P, C.c_uint64]),
        "clg_response_put_batch": (C.c_int, [C.POINTER(Response), P, P, P, C.c_uint32]),
        "clg_response_write": (C.c_int, [C.POINTER(Response), P, C.c_uint64, u64p]),
        "clg_response_read": (C.c_int, [P, C.c_uint64, C.POINTER(Response), u64p]),
        "clg_response_merge": (C.c_int, [C.POINTER(Response), C.POINTER(Response)]),
        "clg_causal_log_id_hash": (C.c_int32, [C.POINTER(CausalLogIdC)]),
        "clg_replay_prepare": (C.c_int, [P, C.POINTER(ReplayVertex), C.c_uint32, C.POINTER(ReplayOut)]),
        "clg_replay_prepare_device": (C.c_int, [P, C.POINTER(ReplayVertex), C.c_uint32, C.POINTER(ReplayOut)]),
        "clg_get_determinants_batch": (C.c_int, [P, P, P, C.c_uint32, P, C.c_uint64, C.c_uint32, P, P, u64p]),
        "clg_encode_batch": (C.c_int, [P, C.POINTER(EncodeIn), P, C.c_uint64, C.c_uint32, u64p, u64p]),
        "clg_enrich_batch": (C.c_int, [P, C.c_uint32, C.POINTER(EnrichReq), C.c_uint32, P, P, P, C.c_uint64,
                                       C.c_uint32, u64p]),
        "clg_process_delta": (C.c_int, [P, C.c_uint32, C.c_uint32, P, C.c_uint64, C.c_uint32, i64p, P, C.c_uint32, u32p,
                                        u64p]),
        "clg_ifl_open": (C.c_int, [P, u32p]),
        "clg_ifl_open_typed": (C.c_int, [P, C.c_uint32, u32p]),
        "clg_ifl_close": (C.c_int, [P, C.c_uint32]),
        "clg_ifl_log_batch": (C.c_int, [P, P, P, P, P, C.c_uint32, P, C.c_uint32]),
        "clg_ifl_notify_checkpoint_complete": (C.c_int, [P, C.c_uint32, C.c_int64]),
        "clg_ifl_state": (C.c_int, [P, C.c_uint32, P, P, C.c_uint32, u32p]),
        "clg_ifl_replay_batch": (C.c_int, [P, P, C.c_uint32, P, P, C.c_uint64, C.c_uint32, P, P, C.c_uint64,
                                           u64p, u64p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(status: int) -> int:
    if status != CLG_OK:
        raise ClonosError(status, lib.clg_last_error().decode(errors="replace"))
    return status
