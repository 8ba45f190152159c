"""uvhttp_amd — MI355X-native WebSocket frame decode / payload unmask for uvhttp.

The product is the C-ABI library ``uvhttp_amd/lib/libuvhttp_ws_amd.so`` (gfx950 HIP kernels
+ host C), declared in ``include/uvhttp_ws_amd.h``.  This package is a thin ctypes mirror of
that ABI so tests and ``bench.py`` can drive it from Python:

* the reference's decode surface (``src/uvhttp_websocket.c`` of adam-ikari/uvhttp v2.7.0):
  :func:`parse_frame_header`, :func:`apply_mask`, :class:`WsConnection` (``process_data``);
* the batched device surface: :class:`GpuEngine` (``decode_inplace`` / ``decode_compact``).

Nothing here computes a result in Python, and there is no CPU fallback: if the library is
missing, :func:`lib` raises; if no MI355X is present, :class:`GpuEngine` raises.
"""
from __future__ import annotations

import ctypes as C
import os

__all__ = [
    "lib", "LIB_PATH", "FrameHeader", "FrameDesc", "MessageDesc", "BatchSummary", "Batch",
    "WsConnectionStruct", "parse_frame_header", "apply_mask", "WsConnection", "GpuEngine",
    "GpuError", "OPCODES", "FRAME_STATUS", "gen_frame_stride", "GpuPipeline", "Stream",
    "StreamResult", "STREAM_DT", "STREAM_RESULT_DT", "STREAM_RESULT_BYTES", "Batcher",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libuvhttp_ws_amd.so")
# the same library built with -DUVWS_TEST_HOOKS (the batcher's fault injection); tests only
TESTHOOKS_LIB_PATH = os.path.join(_HERE, "lib", "libuvhttp_ws_amd_testhooks.so")

OPCODES = dict(CONTINUATION=0x0, TEXT=0x1, BINARY=0x2, CLOSE=0x8, PING=0x9, PONG=0xA)
FRAME_STATUS = {
    0: "OK", 1: "INCOMPLETE", 2: "SKIPPED", -1: "ERR_PARSE", -2: "ERR_RSV", -3: "ERR_CONTROL",
    -4: "ERR_UNMASKED", -5: "ERR_TOO_BIG", -6: "ERR_BUFFER", -7: "ERR_FRAGMENT",
    -8: "ERR_MESSAGE", -9: "ERR_LAYOUT", -10: "ERR_CAPACITY", -11: "ERR_DEVICE",
}
FLAG_FIN, FLAG_MASK, FLAG_MSG_END = 0x01, 0x02, 0x20


class GpuError(RuntimeError):
    pass


# ---- struct mirrors (include/uvhttp_ws_amd.h) ------------------------------------------

class FrameHeader(C.Structure):
    """uvhttp_ws_frame_header_t (16 B; bitfields in bytes 0-1, payload_length @8)."""
    _fields_ = [("fin", C.c_uint8, 1), ("rsv1", C.c_uint8, 1), ("rsv2", C.c_uint8, 1),
                ("rsv3", C.c_uint8, 1), ("opcode", C.c_uint8, 4), ("mask", C.c_uint8, 1),
                ("payload_len", C.c_uint8, 7), ("payload_length", C.c_uint64)]


class FrameDesc(C.Structure):
    _fields_ = [("payload_off", C.c_uint64), ("payload_len", C.c_uint64),
                ("masking_key", C.c_uint32), ("message", C.c_uint32), ("opcode", C.c_uint8),
                ("flags", C.c_uint8), ("header_size", C.c_uint8), ("status", C.c_int8),
                ("wire_len", C.c_uint32)]


class MessageDesc(C.Structure):
    _fields_ = [("arena_off", C.c_uint64), ("len", C.c_uint64), ("first_frame", C.c_uint32),
                ("last_frame", C.c_uint32), ("opcode", C.c_int32), ("reserved", C.c_uint32)]


class BatchSummary(C.Structure):
    _fields_ = [("n_frames", C.c_uint32), ("n_delivered", C.c_uint32), ("status", C.c_int32),
                ("first_status", C.c_int32), ("consumed_bytes", C.c_uint64),
                ("payload_bytes", C.c_uint64), ("n_messages", C.c_uint32),
                ("state_closed", C.c_uint32), ("arena_bytes", C.c_uint64),
                ("pending_bytes", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Stream(C.Structure):
    """uvhttp_ws_stream_t (64 B)."""
    _fields_ = [("begin", C.c_uint64), ("len", C.c_uint64), ("recv_buffer_size", C.c_uint64),
                ("pending_bytes", C.c_uint64), ("pending_opcode", C.c_int32),
                ("max_frame_size", C.c_int32), ("max_message_size", C.c_int32),
                ("is_server", C.c_int32), ("first_read", C.c_uint32), ("n_reads", C.c_uint32),
                ("reserved", C.c_uint64)]


class StreamResult(C.Structure):
    """uvhttp_ws_stream_result_t (64 B)."""
    _fields_ = [("first_frame", C.c_uint32), ("n_frames", C.c_uint32),
                ("n_delivered", C.c_uint32), ("status", C.c_int32), ("first_status", C.c_int32),
                ("calls", C.c_uint32), ("consumed_bytes", C.c_uint64),
                ("recv_buffer_size", C.c_uint64), ("pending_bytes", C.c_uint64),
                ("buffered_end", C.c_uint64), ("reserved", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def _np_dtype(struct):
    import numpy as np
    codes = {C.c_uint64: "<u8", C.c_int64: "<i8", C.c_uint32: "<u4", C.c_int32: "<i4"}
    dt = np.dtype([(name, codes[t]) for name, t in struct._fields_])
    assert dt.itemsize == C.sizeof(struct)
    return dt


STREAM_DT = _np_dtype(Stream)
STREAM_RESULT_DT = _np_dtype(StreamResult)
STREAM_RESULT_BYTES = C.sizeof(StreamResult)


class GpuStamp(C.Structure):
    """uvhttp_ws_gpu_stamp_t (24 B)."""
    _fields_ = [("call", C.c_uint32), ("kernel", C.c_uint32), ("begin_ns", C.c_uint64),
                ("end_ns", C.c_uint64)]


STAMP_KERNELS = {0: "walk", 1: "walk_scan", 2: "walk2", 3: "stream_desc", 4: "claims",
                 5: "payload", 6: "plan", 7: "fixup", 8: "finalize", 9: "build_size",
                 10: "build_scan", 11: "build_scan2", 12: "build_offsets", 13: "desc_emit",
                 14: "sum_scan", 15: "spec_plan"}


class Batch(C.Structure):
    _fields_ = [("wire", C.c_void_p), ("wire_len", C.c_uint64), ("frame_off", C.c_void_p),
                ("frame_stride", C.c_uint64), ("n_frames", C.c_uint32),
                ("max_frame_size", C.c_int32), ("max_message_size", C.c_int32),
                ("is_server", C.c_int32)]


ON_MESSAGE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_char), C.c_size_t, C.c_int)
ON_CLOSE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_char_p)
ON_ERROR = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_char_p)
CONTEXT_RESOLVER = C.CFUNCTYPE(C.c_void_p, C.c_void_p)
FAILURE_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_int)
READY_CB = C.CFUNCTYPE(None, C.c_void_p)
TLS_HANDBACK_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t,
                              C.c_uint64, C.c_int)
CONTROL_SINK = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_uint8),
                           C.c_size_t)


class WsConfig(C.Structure):
    _fields_ = [("max_frame_size", C.c_int), ("max_message_size", C.c_int),
                ("ping_interval", C.c_int), ("ping_timeout", C.c_int),
                ("enable_compression", C.c_int)]


class WsConnectionStruct(C.Structure):
    """uvhttp_ws_connection_t (248 B on x86-64)."""
    _fields_ = [("fd", C.c_int), ("state", C.c_int), ("config", WsConfig),
                ("ssl", C.c_void_p), ("is_server", C.c_int), ("client_key", C.c_char * 64),
                ("recv_buffer", C.c_void_p), ("recv_buffer_size", C.c_size_t),
                ("recv_buffer_pos", C.c_size_t), ("send_buffer", C.c_void_p),
                ("send_buffer_size", C.c_size_t), ("fragmented_message", C.c_void_p),
                ("fragmented_size", C.c_size_t), ("fragmented_capacity", C.c_size_t),
                ("fragmented_opcode", C.c_int), ("on_message", C.c_void_p),
                ("on_close", C.c_void_p), ("on_error", C.c_void_p), ("user_data", C.c_void_p),
                ("bytes_sent", C.c_uint64), ("bytes_received", C.c_uint64),
                ("frames_sent", C.c_uint64), ("frames_received", C.c_uint64)]


class UvhttpConfig(C.Structure):
    """uvhttp_config_t (include/uvhttp_config.h); websocket_* at offsets 64..79."""
    _fields_ = [("max_connections", C.c_int), ("read_buffer_size", C.c_int),
                ("backlog", C.c_int), ("keepalive_timeout", C.c_int),
                ("request_timeout", C.c_int), ("connection_timeout", C.c_int),
                ("max_body_size", C.c_size_t), ("max_header_size", C.c_size_t),
                ("max_url_size", C.c_size_t), ("max_file_size", C.c_size_t),
                ("max_requests_per_connection", C.c_int), ("rate_limit_window", C.c_int),
                ("websocket_max_frame_size", C.c_int), ("websocket_max_message_size", C.c_int),
                ("websocket_ping_interval", C.c_int), ("websocket_ping_timeout", C.c_int),
                ("tcp_keepalive_timeout", C.c_int), ("sendfile_timeout_ms", C.c_int),
                ("sendfile_max_retry", C.c_int), ("cache_default_max_entries", C.c_int),
                ("cache_default_ttl", C.c_int), ("lru_cache_batch_eviction_size", C.c_int),
                ("rate_limit_max_requests", C.c_int), ("rate_limit_max_window_seconds", C.c_int),
                ("rate_limit_min_timeout_seconds", C.c_int)]


class BatcherConfig(C.Structure):
    """uvhttp_ws_amd_batcher_config_t"""
    _fields_ = [("device", C.c_int), ("min_device_bytes", C.c_uint64), ("max_bytes", C.c_uint64),
                ("max_connections", C.c_uint32), ("max_reads", C.c_uint32),
                ("on_failure", FAILURE_CB), ("ctx", C.c_void_p),
                ("on_ready", READY_CB), ("ready_ctx", C.c_void_p),
                ("on_tls_handback", TLS_HANDBACK_CB)]


class BatcherStats(C.Structure):
    """uvhttp_ws_amd_batcher_stats_t"""
    _fields_ = [(k, C.c_uint64) for k in ("flushes", "device_flushes", "host_flushes", "host_reads",
                                          "device_reads", "device_frames", "device_bytes",
                                          "failures", "capacity_flushes")] + [("device_ms", C.c_double)] + \
        [(k, C.c_uint64) for k in ("async_flushes", "fallback_flushes", "device_errors",
                                   "direct_reads")] + \
        [(k, C.c_double) for k in ("blocked_ms", "max_blocked_ms", "wait_ms", "copy_ms",
                                   "upload_ms", "stage_ms", "deliver_ms")] + \
        [(k, C.c_uint64) for k in ("tls_records", "tls_bytes", "tls_handbacks", "desc_refetches",
                                   "blocked_calls")] + \
        [(k, C.c_double) for k in ("blocked_p50_ms", "blocked_p99_ms", "max_blocked_wait_ms",
                                   "max_blocked_stage_ms", "max_blocked_deliver_ms")] + \
        [("zero_copy_reads", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# ---- library ----------------------------------------------------------------------------

_LIB = None


def lib() -> C.CDLL:
    """Load the product library.  Raises if it has not been built (no fallback)."""
    global _LIB
    if _LIB is None:
        _LIB = load_library(LIB_PATH)
    return _LIB


_TESTHOOKS = None


def test_hooks_library() -> C.CDLL:
    """The test build (UVHTTP_WS_BATCHER_FAIL_EVERY honoured); the product library ignores the
    variable.  Tests pass it as Batcher(..., library=...)."""
    global _TESTHOOKS
    if _TESTHOOKS is None:
        _TESTHOOKS = load_library(TESTHOOKS_LIB_PATH)
    return _TESTHOOKS


# Environment switches only the experiment build (libuvhttp_ws_amd_testhooks.so, -DUVWS_EXPERIMENTS)
# reads; the product library reads no environment (ws_gpu.hip experiment_knobs).  Engines,
# batchers and pipelines created while one of these is set load the experiment build, so A/B
# tools and variant tests get the variant they name rather than a silently ignored switch.
EXPERIMENT_KNOBS = (
    "UVHTTP_WS_MAX_POLLS", "UVHTTP_WS_SCRATCH_POOL", "UVHTTP_WS_STORE_POLICY", "UVHTTP_WS_PLAN_FPT",
    "UVHTTP_WS_PLAN_TICKET", "UVHTTP_WS_EPOCH_START", "UVHTTP_WS_BUILD_SMALL", "UVHTTP_WS_FUSED",
    "UVHTTP_WS_FUSED_MAX", "UVHTTP_WS_PLAN_WIDE", "UVHTTP_WS_REC_SCAN", "UVHTTP_WS_BUILD_FRAMES",
    "UVHTTP_WS_COMPACT", "UVHTTP_WS_WALK_SINGLE", "UVHTTP_WS_WALK_FUSE", "UVHTTP_WS_STREAM_NT",
    "UVHTTP_WS_DESC_SCAN", "UVHTTP_WS_WALK_NT_LOAD", "UVHTTP_WS_WALK_REC", "UVHTTP_WS_WALK",
    "UVHTTP_WS_TIME_CHAIN", "UVHTTP_WS_COMPACT_RECS", "UVHTTP_WS_SPEC", "UVHTTP_WS_SPEC_MAX",
    "UVHTTP_WS_FUSED_AUX", "UVHTTP_WS_SUMMARY_FAST", "UVHTTP_WS_TILE", "UVHTTP_WS_FIXUP_BLOCKS",
    "UVHTTP_WS_FUSED_TILE", "UVHTTP_WS_TIMING_FENCE", "UVHTTP_WS_PIPE_IN_FLIGHT",
    "UVHTTP_TLS_CRYPT_GRID", "UVHTTP_WS_BATCHER_TRACE", "UVHTTP_WS_BATCHER_FAIL_EVERY",
    "UVHTTP_WS_COPY_SSE2", "UVHTTP_WS_DESC_EMIT", "UVHTTP_WS_STREAM_SPEC")


def experiment_knobs_set():
    return [k for k in EXPERIMENT_KNOBS if k in os.environ]


def default_library() -> C.CDLL:
    """the product library, or the experiment build while an experiment switch is set"""
    return test_hooks_library() if experiment_knobs_set() else lib()


def load_library(path: str) -> C.CDLL:
    """Load a build of libuvhttp_ws_amd.so from `path` and declare its entry points (lib()
    uses the in-tree build; tools/ab_lib.py loads a second build beside it for A/B runs)."""
    if not os.path.exists(path):
        raise ImportError(f"{path} missing: run `make` (or __graft_entry__.build())")
    try:  # share torch's HIP runtime (same SONAME) so torch device pointers are valid
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32
    sig = {
        "uvhttp_ws_amd_version": (C.c_char_p, []),
        "uvhttp_ws_parse_frame_header": (C.c_int, [vp, C.c_size_t, C.POINTER(FrameHeader),
                                                   C.POINTER(C.c_size_t)]),
        "uvhttp_ws_apply_mask": (None, [vp, C.c_size_t, vp]),
        "uvhttp_ws_connection_create": (C.POINTER(WsConnectionStruct),
                                        [C.c_int, vp, C.c_int, C.POINTER(UvhttpConfig)]),
        "uvhttp_ws_connection_free": (None, [C.POINTER(WsConnectionStruct)]),
        "uvhttp_ws_set_callbacks": (None, [C.POINTER(WsConnectionStruct), ON_MESSAGE, ON_CLOSE,
                                           ON_ERROR]),
        "uvhttp_ws_process_data": (C.c_int, [C.POINTER(WsConnectionStruct), vp, C.c_size_t]),
        "uvhttp_ws_amd_set_control_hooks": (None, [CONTEXT_RESOLVER, CONTROL_SINK]),
        "uvhttp_ws_gpu_engine_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "uvhttp_ws_gpu_engine_free": (None, [vp]),
        "uvhttp_ws_gpu_engine_reserve": (C.c_int, [vp, u32, u64, u64]),
        "uvhttp_ws_gpu_engine_set_timing": (C.c_int, [vp, C.c_int]),
        "uvhttp_ws_gpu_engine_set_tile": (C.c_int, [vp, C.c_int, C.c_int]),
        "uvhttp_ws_gpu_engine_kernel_time": (C.c_int, [vp, C.POINTER(C.c_double),
                                                       C.POINTER(u64)]),
        "uvhttp_ws_gpu_engine_last_error": (C.c_char_p, [vp]),
        "uvhttp_ws_gpu_engine_sync": (C.c_int, [vp, vp]),
        "uvhttp_ws_gpu_engine_set_stamps": (C.c_int, [vp, C.c_int]),
        "uvhttp_ws_gpu_engine_read_stamps": (C.c_int, [vp, vp, u32, C.POINTER(u32)]),
        "uvhttp_ws_gpu_stamp_ring_words": (u64, []),
        "uvhttp_ws_gpu_stamps_reduce": (C.c_int, [vp, u32, u32, vp, u32, C.POINTER(u32)]),
        "uvhttp_ws_gpu_stamp_simulate": (C.c_int, [vp, u32, u32, u64, u32, u32, u64, u64, u64]),
        "uvhttp_ws_gpu_decode_inplace": (C.c_int, [vp, C.POINTER(Batch), vp, vp, vp]),
        "uvhttp_ws_gpu_decode_compact": (C.c_int, [vp, C.POINTER(Batch), vp, u64, vp, vp, vp,
                                                   vp]),
        "uvhttp_ws_gpu_apply_mask": (C.c_int, [vp, vp, u64, vp, vp]),
        "uvhttp_ws_gen_frame_stride": (u64, [u64]),
        "uvhttp_ws_gpu_pipeline_create": (C.c_int, [C.c_int, C.c_int, u64, u32, C.POINTER(vp)]),
        "uvhttp_ws_gpu_pipeline_free": (None, [vp]),
        "uvhttp_ws_gpu_pipeline_slot_buffer": (vp, [vp, C.c_int]),
        "uvhttp_ws_gpu_pipeline_slot_offsets": (vp, [vp, C.c_int]),
        "uvhttp_ws_gpu_pipeline_submit": (C.c_int, [vp, C.c_int, u64, C.c_int, u64, u32, i32, i32,
                                                    i32]),
        "uvhttp_ws_gpu_pipeline_wait": (C.c_int, [vp, C.c_int, C.POINTER(vp), C.POINTER(vp)]),
        "uvhttp_ws_gpu_pipeline_submit_compact": (C.c_int, [vp, C.c_int, u64, C.c_int, u64, u32, i32,
                                                            i32, i32]),
        "uvhttp_ws_gpu_pipeline_wait_compact": (C.c_int, [vp, C.c_int, C.POINTER(vp), C.POINTER(vp),
                                                          C.POINTER(vp), C.POINTER(vp)]),
        "uvhttp_ws_deliver_batch": (C.c_int, [C.POINTER(WsConnectionStruct), vp, vp, vp]),
        "uvhttp_ws_deliver_messages": (C.c_int, [C.POINTER(WsConnectionStruct), vp, vp, vp, vp, vp,
                                                 u64]),
        "uvhttp_ws_gpu_decode_streams": (C.c_int, [vp, vp, u64, vp, u32, u32, vp, vp, vp]),
        "uvhttp_ws_gpu_decode_reads": (C.c_int, [vp, vp, u64, vp, u32, vp, u32, u32, vp, vp, vp]),
        "uvhttp_ws_gpu_build_frames": (C.c_int, [vp, vp, u64, vp, u32, vp, u64, vp, vp]),
        "uvhttp_ws_stream_init": (None, [C.POINTER(WsConnectionStruct), u64, u64,
                                         C.POINTER(Stream)]),
        "uvhttp_ws_deliver_stream": (C.c_int, [C.POINTER(WsConnectionStruct), vp, vp,
                                               C.POINTER(Stream), C.POINTER(StreamResult)]),
        "uvhttp_ws_gpu_gen_frames": (C.c_int, [vp, vp, u32, u64, u64, C.c_int, C.c_int, C.c_int,
                                               vp]),
        "uvhttp_ws_gpu_gen_frames_range": (C.c_int, [vp, vp, u32, u32, u32, u64, u64, C.c_int,
                                                     C.c_int, C.c_int, vp]),
        # batcher (include/uvhttp_ws_amd.h)
        "uvhttp_ws_amd_batcher_config_init": (None, [C.POINTER(BatcherConfig)]),
        "uvhttp_ws_amd_batcher_create": (C.c_int, [C.POINTER(BatcherConfig), C.POINTER(vp)]),
        "uvhttp_ws_amd_batcher_free": (None, [vp]),
        "uvhttp_ws_amd_batcher_submit_read": (C.c_int, [vp, C.POINTER(WsConnectionStruct), vp,
                                                        C.c_size_t]),
        "uvhttp_ws_amd_batcher_alloc_read": (C.c_int, [vp, C.POINTER(WsConnectionStruct), C.c_size_t,
                                                       C.POINTER(vp), C.POINTER(C.c_size_t)]),
        "uvhttp_ws_amd_batcher_commit_read": (C.c_int, [vp, C.POINTER(WsConnectionStruct), C.c_size_t]),
        "uvhttp_ws_amd_batcher_group_alloc_read": (C.c_int, [vp, C.POINTER(WsConnectionStruct), C.c_size_t,
                                                             C.POINTER(vp), C.POINTER(C.c_size_t)]),
        "uvhttp_ws_amd_batcher_group_commit_read": (C.c_int, [vp, C.POINTER(WsConnectionStruct),
                                                              C.c_size_t]),
        "uvhttp_ws_amd_batcher_flush": (C.c_int, [vp]),
        "uvhttp_ws_amd_batcher_flush_async": (C.c_int, [vp]),
        "uvhttp_ws_amd_batcher_poll": (C.c_int, [vp]),
        "uvhttp_ws_amd_batcher_in_flight": (C.c_int, [vp]),
        "uvhttp_ws_amd_batcher_set_tls": (C.c_int, [vp, C.POINTER(WsConnectionStruct), vp,
                                                   C.c_uint64]),
        "uvhttp_ws_amd_batcher_submit_tls_read": (C.c_int, [vp, C.POINTER(WsConnectionStruct),
                                                           vp, C.c_size_t]),
        "uvhttp_ws_amd_batcher_forget": (None, [vp, C.POINTER(WsConnectionStruct)]),
        "uvhttp_ws_amd_batcher_stats": (C.c_int, [vp, C.POINTER(BatcherStats)]),
        "uvhttp_ws_amd_batcher_reset_stats": (None, [vp]),
        "uvhttp_ws_amd_batcher_group_create": (C.c_int, [C.POINTER(BatcherConfig), vp, C.c_int,
                                                         C.POINTER(vp)]),
        "uvhttp_ws_amd_batcher_group_free": (None, [vp]),
        "uvhttp_ws_amd_batcher_group_size": (C.c_int, [vp]),
        "uvhttp_ws_amd_batcher_group_batcher": (vp, [vp, C.c_int]),
        "uvhttp_ws_amd_batcher_group_member": (C.c_int, [vp, C.POINTER(WsConnectionStruct)]),
        "uvhttp_ws_amd_batcher_group_submit_read": (C.c_int, [vp, C.POINTER(WsConnectionStruct),
                                                              vp, C.c_size_t]),
        "uvhttp_ws_amd_batcher_group_set_tls": (C.c_int, [vp, C.POINTER(WsConnectionStruct), vp,
                                                         C.c_uint64]),
        "uvhttp_ws_amd_batcher_group_submit_tls_read": (C.c_int, [vp, C.POINTER(WsConnectionStruct),
                                                                 vp, C.c_size_t]),
        "uvhttp_ws_amd_batcher_group_flush_async": (C.c_int, [vp]),
        "uvhttp_ws_amd_batcher_group_poll": (C.c_int, [vp]),
        "uvhttp_ws_amd_batcher_group_flush": (C.c_int, [vp]),
        "uvhttp_ws_amd_batcher_group_in_flight": (C.c_int, [vp]),
        "uvhttp_ws_amd_batcher_group_forget": (None, [vp, C.POINTER(WsConnectionStruct)]),
        "uvhttp_ws_amd_batcher_group_stats": (C.c_int, [vp, C.POINTER(BatcherStats)]),
        "uvhttp_ws_amd_batcher_group_reset_stats": (None, [vp]),
        "uvhttp_ws_amd_batcher_numa_node": (C.c_int, [vp]),
        # TLS record layer (include/uvhttp_tls_amd.h)
        "uvhttp_tls_gpu_engine_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "uvhttp_tls_gpu_engine_free": (None, [vp]),
        "uvhttp_tls_gpu_engine_last_error": (C.c_char_p, [vp]),
        "uvhttp_tls_gpu_engine_set_timing": (C.c_int, [vp, C.c_int]),
        "uvhttp_tls_gpu_engine_kernel_time": (C.c_int, [vp, C.POINTER(C.c_double),
                                                        C.POINTER(u64)]),
        "uvhttp_tls_gpu_open_records": (C.c_int, [vp, vp, u64, vp, u32, vp, u32, vp, u32, vp, vp,
                                                  u64, vp]),
        "uvhttp_tls_gpu_seal_records": (C.c_int, [vp, vp, u64, vp, u32, vp, u32, vp, u64, vp]),
        "uvhttp_tls_gpu_ws_streams": (C.c_int, [vp, vp, vp, u32, vp, vp, vp, vp, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        if path not in (LIB_PATH, TESTHOOKS_LIB_PATH) and not hasattr(L, name):
            continue  # an older build loaded beside the tree's for an A/B run (tools/ab_lib.py)
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def gen_frame_stride(payload_len: int) -> int:
    return int(lib().uvhttp_ws_gen_frame_stride(payload_len))


# ---- host drop-in surface ---------------------------------------------------------------

def parse_frame_header(data, length=None, null=None):
    """uvhttp_ws_parse_frame_header -> (rc, FrameHeader, header_size)."""
    L = lib()
    buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
    n = len(data) if length is None else length
    hdr, hs = FrameHeader(), C.c_size_t(0)
    rc = L.uvhttp_ws_parse_frame_header(None if null == "data" else buf, n,
                                        None if null == "header" else C.byref(hdr),
                                        None if null == "header_size" else C.byref(hs))
    return rc, hdr, hs.value


def apply_mask(data: bytearray, key, length=None, null=None):
    """uvhttp_ws_apply_mask in place on a bytearray."""
    L = lib()
    n = len(data) if length is None else length
    buf = (C.c_uint8 * max(1, len(data))).from_buffer(data) if len(data) else None
    kb = (C.c_uint8 * 4).from_buffer_copy(bytes(key)) if key else None
    L.uvhttp_ws_apply_mask(None if null == "data" else buf, n, None if null == "key" else kb)
    return data


class WsConnection:
    """One server-side connection of the drop-in stream decoder (records callbacks)."""

    def __init__(self, is_server=1, max_frame_size=None, max_message_size=None,
                 callbacks=True, user_data=False):
        L = lib()
        self._L = L
        cfg = None
        if max_frame_size is not None or max_message_size is not None:
            cfg = UvhttpConfig()
            cfg.websocket_max_frame_size = 16 * 1024 * 1024 if max_frame_size is None \
                else max_frame_size
            cfg.websocket_max_message_size = 64 * 1024 * 1024 if max_message_size is None \
                else max_message_size
            cfg.websocket_ping_interval = 30
            cfg.websocket_ping_timeout = 10
        self.ptr = L.uvhttp_ws_connection_create(0, None, is_server,
                                                 C.byref(cfg) if cfg is not None else None)
        if not self.ptr:
            raise MemoryError("uvhttp_ws_connection_create failed")
        self.events = []
        self.hook = None  # optional f(conn, event), run inside on_message (tests)
        if callbacks:
            self._cbs = (ON_MESSAGE(self._on_message), ON_CLOSE(self._on_close),
                         ON_ERROR(self._on_error))
            L.uvhttp_ws_set_callbacks(self.ptr, *self._cbs)
        if user_data:
            self.ptr.contents.user_data = 1

    def _on_message(self, conn, data, n, opcode):
        ev = ("message", opcode, C.string_at(data, n) if n else b"")
        self.events.append(ev)
        if self.hook is not None:
            self.hook(self, ev)
        return 0

    def _on_close(self, conn, code, reason):
        self.events.append(("close", code, None))
        return 0

    def _on_error(self, conn, code, msg):
        self.events.append(("error", code, None))
        return 0

    @property
    def struct(self) -> WsConnectionStruct:
        return self.ptr.contents

    def process_data(self, data: bytes, length=None, null=False) -> int:
        buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
        n = len(data) if length is None else length
        return self._L.uvhttp_ws_process_data(self.ptr, None if null else buf, n)

    def close(self):
        if getattr(self, "ptr", None):
            self._L.uvhttp_ws_connection_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _host_buf(x):
    """a ctypes buffer holding a host copy of x (bytes, numpy array, torch tensor) or None"""
    if x is None:
        return None
    if hasattr(x, "cpu"):
        x = x.cpu().numpy()
    raw = bytes(x.tobytes() if hasattr(x, "tobytes") else x)
    return (C.c_uint8 * max(1, len(raw))).from_buffer_copy(raw or b"\0")


def deliver_messages(conn, arena, msgs, summary, wire=None, desc=None, stride=0) -> int:
    """uvhttp_ws_deliver_messages (include/uvhttp_ws_amd.h): a compact decode's arena,
    message table (n_messages + 1 entries: the open message's too) and summary (a dict or its
    raw bytes) delivered to a WsConnection; wire / desc only for control frames."""
    if isinstance(summary, dict):
        sb = BatchSummary(**summary)
    else:
        sb = BatchSummary.from_buffer_copy(bytes(summary.cpu().numpy().tobytes()
                                                 if hasattr(summary, "cpu") else summary)[:C.sizeof(BatchSummary)])
    bufs = [_host_buf(x) for x in (arena, msgs, wire, desc)]
    ptrs = [C.cast(b, C.c_void_p) if b is not None else None for b in bufs]
    return lib().uvhttp_ws_deliver_messages(conn.ptr, ptrs[0], ptrs[1], C.byref(sb), ptrs[2],
                                            ptrs[3], stride)


# ---- batched device surface -------------------------------------------------------------

class GpuEngine:
    """Owns a uvhttp_ws_gpu_engine_t on one MI355X.  Device buffers are torch tensors
    (plumbing only); every decode runs the gfx950 kernels through the C-ABI."""

    DESC_BYTES = 32
    MSG_BYTES = 32

    def __init__(self, device: int = 0, library: C.CDLL = None):
        import torch
        self.torch = torch
        L = library or default_library()
        self._L = L
        self.device = device
        h = C.c_void_p()
        rc = L.uvhttp_ws_gpu_engine_create(device, C.byref(h))
        if rc != 0:
            raise GpuError(f"uvhttp_ws_gpu_engine_create({device}) failed rc={rc} "
                           "(needs an MI355X / gfx950 and the HIP runtime)")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self._L.uvhttp_ws_gpu_engine_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            err = self._L.uvhttp_ws_gpu_engine_last_error(self.h)
            raise GpuError(f"{what} rc={rc}: {err.decode() if err else ''}")

    def _stream(self, stream):
        if stream is None:
            stream = self.torch.cuda.current_stream(self.device)
        return C.c_void_p(stream.cuda_stream)

    def reserve(self, max_frames, max_wire, max_arena=0):
        self._check(self._L.uvhttp_ws_gpu_engine_reserve(self.h, max_frames, max_wire,
                                                         max_arena), "reserve")

    def set_tile(self, block: int, vectors_per_lane: int):
        self._check(self._L.uvhttp_ws_gpu_engine_set_tile(self.h, block, vectors_per_lane),
                    "set_tile")

    def set_timing(self, on, every=1):
        """HIP events around the payload kernel of every `every`-th call while on"""
        self._check(self._L.uvhttp_ws_gpu_engine_set_timing(self.h, every if on else 0), "timing")

    def kernel_time(self):
        ms, n = C.c_double(0), C.c_uint64(0)
        self._check(self._L.uvhttp_ws_gpu_engine_kernel_time(self.h, C.byref(ms), C.byref(n)),
                    "kernel_time")
        return ms.value, n.value

    def set_stamps(self, on=True):
        """device-side kernel stamps (include/uvhttp_ws_amd.h): on / off"""
        self._check(self._L.uvhttp_ws_gpu_engine_set_stamps(self.h, 1 if on else 0), "set_stamps")

    def read_stamps(self):
        """-> [(call, kernel name, begin_ns, end_ns)] of the calls the engine still holds
        (waits for the device; clears them)"""
        buf = (GpuStamp * 4096)()
        n = C.c_uint32(0)
        self._check(self._L.uvhttp_ws_gpu_engine_read_stamps(self.h, buf, 4096, C.byref(n)),
                    "read_stamps")
        return [(r.call, STAMP_KERNELS.get(r.kernel, str(r.kernel)), r.begin_ns, r.end_ns)
                for r in buf[:n.value]]

    def alloc_outputs(self, n_frames):
        t = self.torch
        dev = f"cuda:{self.device}"
        desc = t.empty(max(1, n_frames) * self.DESC_BYTES, dtype=t.uint8, device=dev)
        summ = t.zeros(C.sizeof(BatchSummary), dtype=t.uint8, device=dev)
        return desc, summ

    def _batch(self, wire, n_frames, stride, offsets, max_frame_size, max_message_size,
               is_server, wire_len):
        b = Batch()
        b.wire = wire.data_ptr()
        b.wire_len = wire.numel() if wire_len is None else wire_len
        b.frame_off = offsets.data_ptr() if offsets is not None else None
        b.frame_stride = stride or 0
        b.n_frames = n_frames
        b.max_frame_size = max_frame_size
        b.max_message_size = max_message_size
        b.is_server = is_server
        return b

    def decode_inplace(self, wire, n_frames, stride=None, offsets=None,
                       max_frame_size=16 * 1024 * 1024, max_message_size=64 * 1024 * 1024,
                       is_server=1, wire_len=None, desc=None, summary=None, stream=None,
                       no_desc=False):
        """no_desc=True: d_desc = NULL, a summary-only decode (include/uvhttp_ws_amd.h);
        returns (None, summary)"""
        if summary is None or (desc is None and not no_desc):
            d0, s0 = self.alloc_outputs(n_frames)
            desc = d0 if desc is None else desc
            summary = s0 if summary is None else summary
        if no_desc:
            desc = None
        b = self._batch(wire, n_frames, stride, offsets, max_frame_size, max_message_size,
                        is_server, wire_len)
        self._check(self._L.uvhttp_ws_gpu_decode_inplace(
            self.h, C.byref(b), C.c_void_p(desc.data_ptr() if desc is not None else None),
            C.c_void_p(summary.data_ptr()), self._stream(stream)), "decode_inplace")
        return desc, summary

    def decode_compact(self, wire, n_frames, arena, stride=None, offsets=None,
                       max_frame_size=16 * 1024 * 1024, max_message_size=64 * 1024 * 1024,
                       is_server=1, wire_len=None, desc=None, msgs=None, summary=None,
                       stream=None, no_desc=False):
        t = self.torch
        if summary is None or (desc is None and not no_desc):
            d0, s0 = self.alloc_outputs(n_frames)
            desc = d0 if desc is None else desc
            summary = s0 if summary is None else summary
        if no_desc:
            desc = None
        if msgs is None:
            msgs = t.empty(max(1, n_frames) * self.MSG_BYTES, dtype=t.uint8,
                           device=f"cuda:{self.device}")
        b = self._batch(wire, n_frames, stride, offsets, max_frame_size, max_message_size,
                        is_server, wire_len)
        self._check(self._L.uvhttp_ws_gpu_decode_compact(
            self.h, C.byref(b), C.c_void_p(arena.data_ptr()), arena.numel(),
            C.c_void_p(desc.data_ptr() if desc is not None else None), C.c_void_p(msgs.data_ptr()),
            C.c_void_p(summary.data_ptr()), self._stream(stream)), "decode_compact")
        return desc, msgs, summary

    def decode_streams(self, wire, streams_dev, n_streams, max_frames, desc=None, results=None,
                       wire_len=None, stream=None, read_end=None, n_reads=0):
        """uvhttp_ws_gpu_decode_streams (or _decode_reads when `read_end`, a device uint64
        tensor of read boundaries, is given); streams_dev = device uint8 tensor of n_streams
        uvhttp_ws_stream_t records.  Returns (desc, results) device tensors."""
        t = self.torch
        dev = f"cuda:{self.device}"
        if desc is None:
            desc = t.empty(max(1, max_frames) * 32, dtype=t.uint8, device=dev)
        if results is None:
            results = t.zeros(max(1, n_streams) * C.sizeof(StreamResult), dtype=t.uint8,
                              device=dev)
        wl = wire.numel() if wire_len is None else wire_len
        if read_end is None:
            rc = self._L.uvhttp_ws_gpu_decode_streams(
                self.h, C.c_void_p(wire.data_ptr()), wl, C.c_void_p(streams_dev.data_ptr()),
                n_streams, max_frames, C.c_void_p(desc.data_ptr()),
                C.c_void_p(results.data_ptr()), self._stream(stream))
        else:
            rc = self._L.uvhttp_ws_gpu_decode_reads(
                self.h, C.c_void_p(wire.data_ptr()), wl, C.c_void_p(streams_dev.data_ptr()),
                n_streams, C.c_void_p(read_end.data_ptr()), n_reads or read_end.numel(),
                max_frames, C.c_void_p(desc.data_ptr()), C.c_void_p(results.data_ptr()),
                self._stream(stream))
        self._check(rc, "decode_streams")
        return desc, results

    def sync(self, stream=None):
        """uvhttp_ws_gpu_engine_sync: raises GpuError if a call since the last sync gave up
        on the device (its outputs say ERR_DEVICE)."""
        self._check(self._L.uvhttp_ws_gpu_engine_sync(self.h, self._stream(stream)), "sync")

    def build_frames(self, src, frames_dev, n_frames, out, out_off=None, stream=None):
        """uvhttp_ws_gpu_build_frames; frames_dev = device uint8 tensor of n_frames
        uvhttp_ws_build_desc_t (32 B each).  Returns out_off (device int64[n+1])."""
        t = self.torch
        if out_off is None:
            out_off = t.zeros(n_frames + 1, dtype=t.int64, device=f"cuda:{self.device}")
        self._check(self._L.uvhttp_ws_gpu_build_frames(
            self.h, C.c_void_p(src.data_ptr()), src.numel(), C.c_void_p(frames_dev.data_ptr()),
            n_frames, C.c_void_p(out.data_ptr()), out.numel(), C.c_void_p(out_off.data_ptr()),
            self._stream(stream)), "build_frames")
        return out_off

    @staticmethod
    def read_stream_results(results, n):
        raw = bytes(results[: n * C.sizeof(StreamResult)].cpu().numpy().tobytes())
        sz = C.sizeof(StreamResult)
        return [StreamResult.from_buffer_copy(raw, k * sz) for k in range(n)]

    def apply_mask(self, data, key, length=None, offset=0, stream=None):
        kb = (C.c_uint8 * 4).from_buffer_copy(bytes(key))
        n = data.numel() - offset if length is None else length
        self._check(self._L.uvhttp_ws_gpu_apply_mask(
            self.h, C.c_void_p(data.data_ptr() + offset), n, kb, self._stream(stream)),
            "apply_mask")

    def gen_frames(self, wire, n_frames, payload_len, seed, opcode0=2, fragmented=False,
                   force_keys=False, stream=None, first=0, count=None, total=None):
        """frames [first, first + count) of a total-frame batch (default: all n_frames), as
        _oracle.gen_frames(..., first=, count=, total=) writes them"""
        if count is None and total is None and first == 0:
            self._check(self._L.uvhttp_ws_gpu_gen_frames(
                self.h, C.c_void_p(wire.data_ptr()), n_frames, payload_len, seed, opcode0,
                1 if fragmented else 0, 1 if force_keys else 0, self._stream(stream)), "gen_frames")
            return
        count = n_frames if count is None else count
        total = n_frames if total is None else total
        self._check(self._L.uvhttp_ws_gpu_gen_frames_range(
            self.h, C.c_void_p(wire.data_ptr()), first, count, total, payload_len, seed, opcode0,
            1 if fragmented else 0, 1 if force_keys else 0, self._stream(stream)), "gen_frames")

    # -- read-back helpers (host copies of device outputs) --
    @staticmethod
    def read_summary(summary) -> dict:
        raw = bytes(summary.cpu().numpy().tobytes())
        return BatchSummary.from_buffer_copy(raw).as_dict()

    @staticmethod
    def read_desc(desc, n_frames):
        import numpy as np
        dt = np.dtype([("payload_off", "<u8"), ("payload_len", "<u8"), ("masking_key", "<u4"),
                       ("message", "<u4"), ("opcode", "u1"), ("flags", "u1"),
                       ("header_size", "u1"), ("status", "i1"), ("wire_len", "<u4")])
        assert dt.itemsize == 32
        return desc[: n_frames * 32].cpu().numpy().view(dt)

    @staticmethod
    def read_msgs(msgs, n_msgs):
        import numpy as np
        dt = np.dtype([("arena_off", "<u8"), ("len", "<u8"), ("first_frame", "<u4"),
                       ("last_frame", "<u4"), ("opcode", "<i4"), ("reserved", "<u4")])
        return msgs[: n_msgs * 32].cpu().numpy().view(dt)


class GpuPipeline:
    """Host-memory pipeline (include/uvhttp_ws_amd.h): pinned staging slots, each decoded by
    H2D -> decode_inplace -> D2H on its own stream, so consecutive slots overlap."""

    def __init__(self, device=0, depth=3, slot_bytes=1 << 26, slot_frames=1 << 16):
        import numpy as np
        self.np = np
        L = default_library()
        self._L = L
        h = C.c_void_p()
        rc = L.uvhttp_ws_gpu_pipeline_create(device, depth, slot_bytes, slot_frames, C.byref(h))
        if rc != 0:
            raise GpuError(f"uvhttp_ws_gpu_pipeline_create rc={rc}")
        self.h = h
        self.depth, self.slot_bytes, self.slot_frames = depth, slot_bytes, slot_frames

    def buffer(self, slot):
        ptr = self._L.uvhttp_ws_gpu_pipeline_slot_buffer(self.h, slot)
        return self.np.ctypeslib.as_array((C.c_uint8 * self.slot_bytes).from_address(ptr))

    def offsets(self, slot):
        ptr = self._L.uvhttp_ws_gpu_pipeline_slot_offsets(self.h, slot)
        return self.np.ctypeslib.as_array((C.c_uint64 * self.slot_frames).from_address(ptr))

    def submit(self, slot, wire_len, n_frames, stride=0, use_offsets=False,
               max_frame_size=16 * 1024 * 1024, max_message_size=64 * 1024 * 1024, is_server=1):
        rc = self._L.uvhttp_ws_gpu_pipeline_submit(self.h, slot, wire_len, 1 if use_offsets else 0,
                                                   stride, n_frames, max_frame_size,
                                                   max_message_size, is_server)
        if rc != 0:
            raise GpuError(f"pipeline submit rc={rc}")

    def wait(self, slot):
        """-> (desc pointer, summary pointer, summary dict)"""
        dp, sp = C.c_void_p(), C.c_void_p()
        rc = self._L.uvhttp_ws_gpu_pipeline_wait(self.h, slot, C.byref(dp), C.byref(sp))
        if rc != 0:
            raise GpuError(f"pipeline wait rc={rc}")
        summ = BatchSummary.from_address(sp.value)
        return dp, sp, summ.as_dict()

    def desc_array(self, dp, n):
        raw = (C.c_uint8 * (32 * max(1, n))).from_address(dp.value)
        dt = self.np.dtype([("payload_off", "<u8"), ("payload_len", "<u8"),
                            ("masking_key", "<u4"), ("message", "<u4"), ("opcode", "u1"),
                            ("flags", "u1"), ("header_size", "u1"), ("status", "i1"),
                            ("wire_len", "<u4")])
        return self.np.frombuffer(raw, dtype=dt, count=n)

    def submit_compact(self, slot, wire_len, n_frames, stride=0, use_offsets=False,
                       max_frame_size=16 * 1024 * 1024, max_message_size=64 * 1024 * 1024,
                       is_server=1):
        rc = self._L.uvhttp_ws_gpu_pipeline_submit_compact(self.h, slot, wire_len,
                                                           1 if use_offsets else 0, stride, n_frames,
                                                           max_frame_size, max_message_size, is_server)
        if rc != 0:
            raise GpuError(f"pipeline submit_compact rc={rc}")

    def wait_compact(self, slot):
        """-> (arena ptr, msgs ptr, desc ptr (None: summary-only), summary ptr, summary dict)"""
        ap, mp, dp, sp = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        rc = self._L.uvhttp_ws_gpu_pipeline_wait_compact(self.h, slot, C.byref(ap), C.byref(mp),
                                                         C.byref(dp), C.byref(sp))
        if rc != 0:
            raise GpuError(f"pipeline wait_compact rc={rc}")
        return ap, mp, (dp if dp.value else None), sp, BatchSummary.from_address(sp.value).as_dict()

    def deliver_messages(self, conn, slot, ap, mp, dp, sp, stride=0):
        """uvhttp_ws_deliver_messages from this slot's compact results"""
        ptr = self._L.uvhttp_ws_gpu_pipeline_slot_buffer(self.h, slot)
        return self._L.uvhttp_ws_deliver_messages(conn.ptr, ap, mp, sp, C.c_void_p(ptr), dp, stride)

    def deliver(self, conn, slot, dp, sp):
        """uvhttp_ws_deliver_batch on a WsConnection from this slot's decoded bytes."""
        ptr = self._L.uvhttp_ws_gpu_pipeline_slot_buffer(self.h, slot)
        return self._L.uvhttp_ws_deliver_batch(conn.ptr, C.c_void_p(ptr), dp, sp)

    def close(self):
        if getattr(self, "h", None):
            self._L.uvhttp_ws_gpu_pipeline_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- TLS record layer (include/uvhttp_tls_amd.h) -----------------------------------------

TLS_RECORD_BYTES, TLS_RESULT_BYTES = 32, 64


class TlsEngine:
    """Owns a uvhttp_tls_gpu_engine_t.  Keys, streams, records, results and seal descriptors
    are device uint8 tensors holding the C structs of include/uvhttp_tls_amd.h."""

    def __init__(self, device: int = 0, library: C.CDLL = None):
        import torch
        self.torch = torch
        L = library or default_library()
        self._L = L
        self.device = device
        h = C.c_void_p()
        rc = L.uvhttp_tls_gpu_engine_create(device, C.byref(h))
        if rc != 0:
            raise GpuError(f"uvhttp_tls_gpu_engine_create({device}) failed rc={rc} "
                           "(needs an MI355X / gfx950 and the HIP runtime)")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self._L.uvhttp_tls_gpu_engine_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            err = self._L.uvhttp_tls_gpu_engine_last_error(self.h)
            raise GpuError(f"{what} rc={rc}: {err.decode() if err else ''}")

    def _stream(self, stream):
        if stream is None:
            stream = self.torch.cuda.current_stream(self.device)
        return C.c_void_p(stream.cuda_stream)

    def set_timing(self, on: bool):
        self._check(self._L.uvhttp_tls_gpu_engine_set_timing(self.h, 1 if on else 0), "timing")

    def kernel_time(self):
        ms, n = C.c_double(0), C.c_uint64(0)
        self._check(self._L.uvhttp_tls_gpu_engine_kernel_time(self.h, C.byref(ms), C.byref(n)),
                    "kernel_time")
        return ms.value, n.value

    def open_records(self, wire, keys, n_keys, streams, n_streams, max_records, out,
                     records=None, results=None, wire_len=None, stream=None):
        """uvhttp_tls_gpu_open_records -> (records, results) device tensors"""
        t = self.torch
        dev = f"cuda:{self.device}"
        if records is None:
            records = t.zeros(max(1, max_records) * TLS_RECORD_BYTES, dtype=t.uint8, device=dev)
        if results is None:
            results = t.zeros(max(1, n_streams) * TLS_RESULT_BYTES, dtype=t.uint8, device=dev)
        self._check(self._L.uvhttp_tls_gpu_open_records(
            self.h, C.c_void_p(wire.data_ptr()), wire.numel() if wire_len is None else wire_len,
            C.c_void_p(keys.data_ptr()), n_keys, C.c_void_p(streams.data_ptr()), n_streams,
            C.c_void_p(records.data_ptr()), max_records, C.c_void_p(results.data_ptr()),
            C.c_void_p(out.data_ptr()), out.numel(), self._stream(stream)), "open_records")
        return records, results

    def ws_streams(self, results, records, n_streams, streams, out, ws_streams, read_end,
                   prefix_src=None, prefix_off=None, stream=None):
        """uvhttp_tls_gpu_ws_streams: per-record WebSocket stream descriptors (+ prefixes)"""
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        self._check(self._L.uvhttp_tls_gpu_ws_streams(
            self.h, ptr(results), ptr(records), n_streams, ptr(streams), ptr(prefix_src),
            ptr(prefix_off), ptr(out), ptr(ws_streams), ptr(read_end), self._stream(stream)),
            "ws_streams")

    def seal_records(self, src, recs, n_records, keys, n_keys, out, stream=None):
        """uvhttp_tls_gpu_seal_records (recs: device tensor of uvhttp_tls_seal_t)"""
        self._check(self._L.uvhttp_tls_gpu_seal_records(
            self.h, C.c_void_p(src.data_ptr()), src.numel(), C.c_void_p(recs.data_ptr()),
            n_records, C.c_void_p(keys.data_ptr()), n_keys, C.c_void_p(out.data_ptr()),
            out.numel(), self._stream(stream)), "seal_records")


class Batcher:
    """uvhttp_ws_amd_batcher_t: queue live reads of WsConnection objects, decode at flush().
    device=-1 runs the host decoder only; failures arrive in self.failures {conn ptr: rc}."""

    def __init__(self, device=-1, min_device_bytes=0, max_bytes=32 << 20,
                 max_connections=16384, max_reads=1 << 18, library: C.CDLL = None):
        L = library or default_library()
        self._L = L
        cfg = BatcherConfig()
        L.uvhttp_ws_amd_batcher_config_init(C.byref(cfg))
        cfg.device, cfg.min_device_bytes, cfg.max_bytes = device, min_device_bytes, max_bytes
        cfg.max_connections, cfg.max_reads = max_connections, max_reads
        self.failures = {}
        self.handbacks = {}  # conn ptr -> (ciphertext bytes, next_seq, first_status)
        self._cb = FAILURE_CB(self._on_failure)
        cfg.on_failure = self._cb
        self._hb = TLS_HANDBACK_CB(self._on_handback)
        cfg.on_tls_handback = self._hb
        h = C.c_void_p()
        rc = L.uvhttp_ws_amd_batcher_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise GpuError(f"uvhttp_ws_amd_batcher_create rc={rc}")
        self.h = h

    def _on_failure(self, ctx, conn, rc):
        self.failures[conn] = rc

    def _on_handback(self, ctx, conn, data, n, next_seq, status):
        self.handbacks[conn] = (C.string_at(data, n) if n else b"", next_seq, status)

    def set_tls(self, conn: "WsConnection", key_bytes: bytes, read_seq: int) -> int:
        """key_bytes: one uvhttp_tls_key_t (64 bytes)"""
        kb = (C.c_uint8 * 64).from_buffer_copy(bytes(key_bytes))
        return self._L.uvhttp_ws_amd_batcher_set_tls(self.h, conn.ptr, kb, read_seq)

    def submit_tls(self, conn: "WsConnection", data: bytes) -> int:
        buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
        return self._L.uvhttp_ws_amd_batcher_submit_tls_read(self.h, conn.ptr, buf, len(data))

    def submit(self, conn: "WsConnection", data: bytes) -> int:
        buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
        return self._L.uvhttp_ws_amd_batcher_submit_read(self.h, conn.ptr, buf, len(data))

    _ZC = "uvhttp_ws_amd_batcher_"

    def alloc(self, conn: "WsConnection", suggested: int):
        """uvhttp_ws_amd_batcher_alloc_read -> (rc, address, length): space in the staging arena
        for conn's next read"""
        buf, n = C.c_void_p(), C.c_size_t()
        rc = getattr(self._L, self._ZC + "alloc_read")(self.h, conn.ptr, suggested, C.byref(buf),
                                                       C.byref(n))
        return rc, buf.value, n.value

    def commit(self, conn: "WsConnection", nread: int) -> int:
        return getattr(self._L, self._ZC + "commit_read")(self.h, conn.ptr, nread)

    def submit_zero_copy(self, conn: "WsConnection", data: bytes):
        """the libuv shape of one socket read of `data`: alloc_read, the read into the returned
        space (a memmove here), commit_read — in pieces when the space is shorter, as a socket
        would deliver them.  -> (rc, [lengths of the pieces committed]); a failing commit's piece
        is listed (a read no flush can hold is decoded at commit: rc is process_data's)"""
        pos, pieces = 0, []
        while pos < len(data):
            rc, addr, n = self.alloc(conn, len(data) - pos)
            if rc != 0:
                return rc, pieces
            k = min(n, len(data) - pos)
            C.memmove(addr, data[pos:pos + k], k)
            rc = self.commit(conn, k)
            pieces.append(k)  # (consumed even when commit fails: a direct decode's rc)
            if rc != 0:
                return rc, pieces
            pos += k
        return 0, pieces

    def flush(self) -> int:
        return self._L.uvhttp_ws_amd_batcher_flush(self.h)

    def flush_async(self) -> int:
        return self._L.uvhttp_ws_amd_batcher_flush_async(self.h)

    def poll(self) -> int:
        return self._L.uvhttp_ws_amd_batcher_poll(self.h)

    def in_flight(self) -> bool:
        return bool(self._L.uvhttp_ws_amd_batcher_in_flight(self.h))

    def forget(self, conn: "WsConnection"):
        self._L.uvhttp_ws_amd_batcher_forget(self.h, conn.ptr)

    def stats(self) -> dict:
        s = BatcherStats()
        self._L.uvhttp_ws_amd_batcher_stats(self.h, C.byref(s))
        return s.as_dict()

    def numa_node(self) -> int:
        """uvhttp_ws_amd_batcher_numa_node: the GPU's NUMA node (-1: host-only or unknown)"""
        return self._L.uvhttp_ws_amd_batcher_numa_node(self.h)

    def close(self):
        if getattr(self, "h", None):
            self._L.uvhttp_ws_amd_batcher_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BatcherGroup(Batcher):
    """uvhttp_ws_amd_batcher_group_t: one batcher per device (-1 = host decoder), each
    connection pinned to one member; the Batcher methods route / fan out."""

    _P = "uvhttp_ws_amd_batcher_group_"
    _ZC = _P

    def __init__(self, devices, min_device_bytes=0, max_bytes=32 << 20, max_connections=16384,
                 max_reads=1 << 18):
        L = default_library()
        self._L = L
        cfg = BatcherConfig()
        L.uvhttp_ws_amd_batcher_config_init(C.byref(cfg))
        cfg.min_device_bytes, cfg.max_bytes = min_device_bytes, max_bytes
        cfg.max_connections, cfg.max_reads = max_connections, max_reads
        self.failures, self.handbacks = {}, {}
        self._cb = FAILURE_CB(self._on_failure)
        cfg.on_failure = self._cb
        self._hb = TLS_HANDBACK_CB(self._on_handback)
        cfg.on_tls_handback = self._hb
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        rc = L.uvhttp_ws_amd_batcher_group_create(C.byref(cfg), devs, len(devices), C.byref(h))
        if rc != 0:
            raise GpuError(f"uvhttp_ws_amd_batcher_group_create rc={rc}")
        self.h = h

    def _fn(self, name):
        return getattr(self._L, self._P + name)

    def member(self, conn) -> int:
        return self._fn("member")(self.h, conn.ptr)

    def size(self) -> int:
        return self._fn("size")(self.h)

    def member_stats(self, i) -> dict:
        s = BatcherStats()
        self._L.uvhttp_ws_amd_batcher_stats(self._fn("batcher")(self.h, i), C.byref(s))
        return s.as_dict()

    def set_tls(self, conn, key_bytes, read_seq):
        kb = (C.c_uint8 * 64).from_buffer_copy(bytes(key_bytes))
        return self._fn("set_tls")(self.h, conn.ptr, kb, read_seq)

    def submit_tls(self, conn, data):
        buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
        return self._fn("submit_tls_read")(self.h, conn.ptr, buf, len(data))

    def submit(self, conn, data):
        buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
        return self._fn("submit_read")(self.h, conn.ptr, buf, len(data))

    def flush(self):
        return self._fn("flush")(self.h)

    def flush_async(self):
        return self._fn("flush_async")(self.h)

    def poll(self):
        return self._fn("poll")(self.h)

    def in_flight(self):
        return bool(self._fn("in_flight")(self.h))

    def forget(self, conn):
        self._fn("forget")(self.h, conn.ptr)

    def stats(self):
        s = BatcherStats()
        self._fn("stats")(self.h, C.byref(s))
        return s.as_dict()

    def numa_node(self):
        return -1

    def close(self):
        if getattr(self, "h", None):
            self._fn("free")(self.h)
            self.h = None
