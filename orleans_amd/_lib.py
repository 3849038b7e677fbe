"""ctypes binding of liborleans_route.so (include/orleans_route.h).

The library is built in-tree (``make`` / ``__graft_entry__.build()``) and loaded from this package
directory only.  There is deliberately no fallback: if the HIP library is missing, importing the
engine raises, so a GPU run can never silently route through Python or the CPU oracle.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

LIB_NAME = "liborleans_route.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

# ---- constants mirrored from include/orleans_route.h -------------------------------------------------
ABI_VERSION = 1
NULL_SILO = 0xFF
NO_ACT = 0xFFFFFFFF

OK, E_INVALID, E_NOMEM, E_DEVICE, E_CAPACITY, E_STATE, E_OVERFLOW = 0, -1, -2, -3, -4, -5, -6

CAT_NONE, CAT_SYSTEM_TARGET, CAT_SYSTEM_GRAIN, CAT_GRAIN, CAT_CLIENT, CAT_KEYEXT_GRAIN = 0, 1, 2, 3, 4, 6

HDR_ADDRESS_COMPLETE = 0x01
HDR_HASH_VALID = 0x02

ST_HIT = 0
ST_NEW_PLACEMENT = 1
ST_SYSTEM_TARGET = 2
ST_ADDRESS_COMPLETE = 3
ST_OWNER_NULL = 4
ST_NO_SEED = 5
ST_CLIENT_UNREGISTERED = 6
ST_KEYEXT_UNRESOLVED = 7
ST_REMOTE_OWNER = 8
ST_PAST_TOTAL = 9

RF_NEW_PLACEMENT = 0x01
RF_LOOPBACK = 0x02
RF_OWNER_IS_SEED = 0x04

POLICY_PREFER_LOCAL = 0
POLICY_HASH_SPREAD = 1

OPT_EXCLUDE_IF_STOPPING = 0x1
OPT_NO_BUCKETS = 0x2
OPT_TOTAL_GIVEN = 0x4
SPLIT_REMOVE = 0x1
RF_CACHED = 0x08
RF_CACHE_STALE = 0x10
RING_CONSISTENT, RING_VBUCKETS = 0, 1
OUTQ_LOOPBACK, OUTQ_PING, OUTQ_SYSTEM, OUTQ_REJECT, OUTQ_OVERFLOW, OUTQ_UNKNOWN_SILO = (
    0xFFFFFFF0, 0xFFFFFFF1, 0xFFFFFFF2, 0xFFFFFFF3, 0xFFFFFFF4, 0xFFFFFFF5)
DEC_OK, DEC_UNSUPPORTED, DEC_MALFORMED, DEC_UNKNOWN_SILO, DEC_NO_TARGET, DEC_NO_SENDER = 0, 1, 2, 3, 4, 5
SENDER_FROM_HEADER = 0xFF
STAMP_OK, STAMP_COMPLETE, STAMP_SKIPPED, STAMP_UNSUPPORTED, STAMP_MALFORMED, STAMP_OVERFLOW = 0, 1, 2, 3, 4, 5
STAMP_MAX_GROWTH = 72
MERGE_INSERTED, MERGE_KEPT, MERGE_REPLACED, MERGE_SAME, MERGE_DUPLICATE, MERGE_UNSUPPORTED = 0, 1, 2, 3, 4, 5

Q_PROBE_FORM, Q_FULL_UPLOADS, Q_SLOT_PATCHES, Q_DEVICE, Q_N_ACT, Q_MAX_BATCH, Q_RANK_MODE = 1, 2, 3, 4, 5, 6, 7
Q_WIRE_DIGEST = 8
Q_PART_ERROR = 9
PART_CACHED = 0x8
Q_HOT_KEY = 10
Q_HOT_BATCHES = 11
Q_STAGE4_ERROR = 12
MAX_WIRE_TYPES = 16
PART_LOOKBACK_FAILED = 0x4
PART_KEYEXT = 0x10
PART_EXT_FULL = 0x20

INS_INSERTED, INS_EXISTING, INS_INVALID_SILO, INS_REMOTE_OWNER, INS_OWNER_NULL, INS_UNSUPPORTED = 0, 1, 2, 3, 4, 5

# orl_grain_key / orl_msg_hdr as numpy structured dtypes (byte-identical to the C structs)
KEY_DTYPE = np.dtype([("tcd", "<u8"), ("n0", "<u8"), ("n1", "<u8")])
EXT_REF_DTYPE = np.dtype([("off", "<u4"), ("len", "<u4")])  # orl_ext_ref: a KeyExt string in a UTF-8 blob
MSG_DTYPE = np.dtype([("tcd", "<u8"), ("n0", "<u8"), ("n1", "<u8"), ("sending_silo", "u1"), ("category", "u1"),
                      ("flags", "u1"), ("target_silo", "u1"), ("aux", "<u4")])
assert KEY_DTYPE.itemsize == 24 and MSG_DTYPE.itemsize == 32


class orl_config(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("device", C.c_int32), ("dir_capacity", C.c_uint64),
                ("n_act", C.c_uint32), ("placement_policy", C.c_uint32), ("max_batch", C.c_uint64)]


NODE_ID_BYTES = 128
TRANSPORT_RCCL, TRANSPORT_LOCAL = 0, 1
NODE_WIDE_ONLY = 0x1
NODE_SPLIT_COMM = 0x2
NODE_MODE_SPLIT_COMM = 0x1
NODE_MODE_HEAD_STREAM = 0x2
NODE_MAX_RANKS = 8
NODE_MAX_CHUNKS = 16
NODE_HEAD_WORDS = 16


class orl_node_config(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("nranks", C.c_uint32), ("rank", C.c_uint32), ("transport", C.c_uint32),
                ("group_id", C.c_uint8 * NODE_ID_BYTES), ("rank_of_silo", C.c_uint8 * 256), ("max_batch", C.c_uint64),
                ("max_recv", C.c_uint64), ("chunks", C.c_uint32), ("flags", C.c_uint32)]


class orl_node_result(C.Structure):
    _fields_ = [("n_owned", C.c_uint64), ("n_hosted", C.c_uint64), ("n_forwarded", C.c_uint64),
                ("n_sent_remote", C.c_uint64), ("hop2", C.c_uint32), ("n_segments", C.c_uint32), ("route", C.c_void_p),
                ("act", C.c_void_p), ("order", C.c_void_p), ("bucket_offsets", C.c_void_p)]


class orl_node_stats(C.Structure):
    _fields_ = [("comm_count", C.c_uint32), ("chunks", C.c_uint32), ("bytes_sent", C.c_uint64 * NODE_MAX_RANKS),
                ("host_wait_us", C.c_uint64), ("host_waits", C.c_uint64), ("exchange_mode", C.c_uint32),
                ("reserved", C.c_uint32)]


class orl_node_chunk_plan(C.Structure):
    _fields_ = [("width", C.c_uint32), ("rewrite", C.c_uint32), ("send", C.c_uint64 * NODE_MAX_RANKS),
                ("recv", C.c_uint64 * NODE_MAX_RANKS), ("n_recv", C.c_uint64), ("act_lane", C.c_uint32),
                ("ext_lane", C.c_uint32)]


class orl_node_hop2_plan(C.Structure):
    _fields_ = [("forward", C.c_uint32), ("width", C.c_uint32), ("send", C.c_uint64 * NODE_MAX_RANKS),
                ("recv", C.c_uint64 * NODE_MAX_RANKS), ("n_hosted", C.c_uint64), ("n_forwarded", C.c_uint64)]


# Every symbol include/orleans_route.h declares, with its ctypes signature.
_P = C.c_void_p
_u8p = C.POINTER(C.c_uint8)
_SIGS = {
    "orl_abi_version": (C.c_uint32, []),
    "orl_ctx_create": (C.c_int, [C.POINTER(orl_config), C.POINTER(_P)]),
    "orl_ctx_destroy": (C.c_int, [_P]),
    "orl_last_error": (C.c_char_p, [_P]),
    "orl_silos_set": (C.c_int, [_P, C.c_uint32, _P, _P, _P, C.c_uint32]),
    "orl_ring_add_server": (C.c_int, [_P, C.c_uint32, C.c_int32]),
    "orl_ring_remove_server": (C.c_int, [_P, C.c_uint32]),
    "orl_ring_get": (C.c_int, [_P, _P, _P, C.c_uint32, C.POINTER(C.c_uint32)]),
    "orl_calc_id_hash": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.c_int32)]),
    "orl_silo_consistent_hash": (C.c_int, [C.c_char_p, C.c_int32, C.POINTER(C.c_int32)]),
    "orl_jenkins_bytes": (C.c_uint32, [C.c_char_p, C.c_size_t]),
    "orl_keyext_uniform_hash": (C.c_uint32, [_P, C.c_char_p, C.c_size_t]),
    "orl_dir_insert_single": (C.c_int, [_P, _P, _P, _P, C.c_size_t, _P, _P, _P]),
    "orl_dir_remove": (C.c_int, [_P, _P, C.c_size_t, _P]),
    "orl_dir_insert_keyext": (C.c_int, [_P, _P, _P, _P, C.c_uint64, _P, _P, C.c_size_t, _P, _P, _P]),
    "orl_dir_remove_keyext": (C.c_int, [_P, _P, _P, _P, C.c_uint64, C.c_size_t, _P]),
    "orl_dir_lookup_keyext_host": (C.c_int, [_P, _P, _P, _P, C.c_uint64, C.c_size_t, _P, _P]),
    "orl_dir_keyext_count": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "orl_dir_insert_keyext_device": (C.c_int, [_P, _P, _P, _P, C.c_uint64, _P, _P, C.c_size_t, _P, _P, _P, _P]),
    "orl_route_keyext_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, _P, C.c_uint64, _P, _P, _P, _P, _P]),
    "orl_dir_count": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "orl_dir_lookup_host": (C.c_int, [_P, _P, C.c_size_t, _P, _P]),
    "orl_hash_batch": (C.c_int, [_P, _P, C.c_size_t, _P]),
    "orl_route_batch": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, _P, _P, _P]),
    "orl_route_batch_narrow": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, _P, _P, _P]),
    "orl_route_batch_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, _P, _P, _P, _P]),
    "orl_fanout_route_device": (C.c_int, [_P, _P, _P, _P, _P, C.c_size_t, C.c_uint64, C.c_uint32, _P, _P, _P, _P, _P,
                                          C.POINTER(C.c_uint64), _P]),
    "orl_fanout_route_keys_device": (C.c_int, [_P, _P, _P, _P, _P, _P, C.c_size_t, C.c_uint32, _P, _P, _P, _P, _P,
                                               C.POINTER(C.c_uint64), _P]),
    "orl_fanout_route_mixed_device": (C.c_int, [_P, _P, C.c_size_t, _P, _P, _P, C.c_uint64, _P, _P, C.c_size_t, C.c_uint32,
                                                _P, _P, _P, _P, _P, C.POINTER(C.c_uint64), _P]),
    "orl_partition_by_owner_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, C.c_uint32, C.c_uint32, _P, _P, _P,
                                                _P]),
    "orl_partition_by_owner_padded_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, C.c_uint32, C.c_uint32,
                                                       C.c_size_t, _P, _P, _P, _P]),
    "orl_partition_compact_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, C.c_uint32, C.c_uint32, C.c_size_t,
                                               _P, _P, _P, _P, _P]),
    "orl_route_compact_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, _P, _P, _P, _P]),
    "orl_wire_types_set": (C.c_int, [_P, C.c_uint32, _P]),
    "orl_partition_narrow_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, C.c_uint32, C.c_uint32, C.c_size_t,
                                              _P, _P, _P, _P, _P]),
    "orl_route_narrow_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, _P, _P, _P, _P]),
    "orl_partition_cached_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, C.c_uint32, C.c_uint32, C.c_size_t, _P,
                                              C.c_uint32, _P, _P, _P, _P]),
    "orl_route_received_device": (C.c_int, [_P, _P, C.c_uint32, C.c_size_t, C.c_uint32, _P, _P, _P, _P]),
    "orl_dir_insert_single_device": (C.c_int, [_P, _P, _P, _P, C.c_size_t, _P, _P, _P, _P]),
    "orl_dir_remove_device": (C.c_int, [_P, _P, C.c_size_t, _P, _P]),
    "orl_dir_compact": (C.c_int, [_P]),
    "orl_dir_split_device": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _P, _P, C.c_uint64, _P, _P]),
    "orl_vring_set_buckets": (C.c_int, [_P, C.c_uint32]),
    "orl_vring_add_server": (C.c_int, [_P, C.c_uint32, _P, C.c_int32, C.c_int32]),
    "orl_vring_remove_server": (C.c_int, [_P, C.c_uint32]),
    "orl_vring_get": (C.c_int, [_P, _P, _P, C.c_uint32, C.POINTER(C.c_uint32)]),
    "orl_ring_owner_batch_device": (C.c_int, [_P, C.c_uint32, _P, C.c_size_t, C.c_uint32, C.c_uint32, _P, _P]),
    "orl_stream_queue_batch_device": (C.c_int, [_P, C.c_uint32, _P, C.c_size_t, C.c_uint32, C.c_uint32, C.c_uint32, _P,
                                                _P, _P]),
    "orl_silo_hash_set": (C.c_int, [_P, C.c_uint32, C.c_int32]),
    "orl_outbound_queues_device": (C.c_int, [_P, _P, _P, C.c_size_t, C.c_uint32, _P, _P]),
    "orl_client_buckets_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, _P]),
    "orl_silo_address_set": (C.c_int, [_P, C.c_uint32, _P, C.c_int32, C.c_int32]),
    "orl_decode_frames_device": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_size_t, C.c_uint32, _P, _P, _P, _P]),
    "orl_grain_type_set": (C.c_int, [_P, C.c_int32, C.c_char_p, C.c_size_t]),
    "orl_dir_merge_device": (C.c_int, [_P, _P, _P, _P, C.c_size_t, _P, C.c_uint32, _P, _P, _P, _P]),
    "orl_stamp_frames_device": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_size_t, _P, _P, _P, C.c_uint32, _P, _P, C.c_uint64,
                                          _P, _P, _P, _P]),
    "orl_cache_config": (C.c_int, [_P, C.c_uint64]),
    "orl_cache_clear": (C.c_int, [_P]),
    "orl_cache_add_or_update_device": (C.c_int, [_P, _P, _P, _P, C.c_size_t, _P]),
    "orl_cache_remove_device": (C.c_int, [_P, _P, C.c_size_t, _P, _P]),
    "orl_cache_count": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "orl_sync": (C.c_int, [_P]),
    "orl_ctx_query": (C.c_int, [_P, C.c_uint32, C.POINTER(C.c_uint64)]),
    "orl_bucket_device": (C.c_int, [_P, _P, C.c_size_t, _P, _P, _P]),
    "orl_ctx_set_rank_mode": (C.c_int, [_P, C.c_uint32]),
    "orl_device_alloc": (C.c_int, [_P, C.c_size_t, C.POINTER(_P)]),
    "orl_device_free": (C.c_int, [_P, _P]),
    "orl_copy_to_device": (C.c_int, [_P, _P, _P, C.c_size_t, _P]),
    "orl_copy_to_host": (C.c_int, [_P, _P, _P, C.c_size_t, _P]),
    "orl_copy_on_device": (C.c_int, [_P, _P, _P, C.c_size_t, _P]),
    "orl_stream_sync": (C.c_int, [_P, _P]),
    "orl_host_register": (C.c_int, [_P, _P, C.c_size_t]),
    "orl_host_unregister": (C.c_int, [_P, _P]),
    "orl_csr_set": (C.c_int, [_P, _P, C.c_size_t, _P, C.c_size_t]),
    "orl_fanout_batch": (C.c_int, [_P, _P, _P, C.c_size_t, C.c_uint64, C.c_uint32, _P, _P, _P, _P, _P, C.c_size_t,
                                   C.POINTER(C.c_uint64)]),
    "orl_node_unique_id": (C.c_int, [_P]),
    "orl_node_create": (C.c_int, [_P, C.POINTER(orl_node_config), C.POINTER(_P)]),
    "orl_node_destroy": (C.c_int, [_P]),
    "orl_node_last_error": (C.c_char_p, [_P]),
    "orl_node_set_timeout": (C.c_int, [_P, C.c_uint32]),
    "orl_node_plan_chunk": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, _P,
                                      C.POINTER(orl_node_chunk_plan)]),
    "orl_node_plan_hop2": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint64,
                                     C.POINTER(orl_node_hop2_plan)]),
    "orl_node_route_batch_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, C.POINTER(orl_node_result), _P]),
    "orl_node_route_batch_keyext_device": (C.c_int, [_P, _P, C.c_size_t, C.c_uint32, _P, _P, C.c_uint64,
                                                     C.POINTER(orl_node_result), _P]),
    "orl_node_segment": (C.c_int, [_P, C.c_uint32, C.POINTER(_P), C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]),
    "orl_node_get_stats": (C.c_int, [_P, C.POINTER(orl_node_stats)]),
    "orl_node_fanout_batch_device": (C.c_int, [_P, _P, _P, _P, C.c_uint64, _P, _P, C.c_size_t, C.c_uint32, _P,
                                               C.POINTER(C.c_uint64), C.POINTER(orl_node_result), _P]),
    "orl_fanout_expand_device": (C.c_int, [_P, _P, _P, _P, C.c_uint64, _P, _P, C.c_size_t, C.c_uint32, _P, _P, C.c_uint64,
                                           C.POINTER(C.c_uint64), _P]),
    "orl_set_timing": (C.c_int, [_P, C.c_int]),
    "orl_timing_summary": (C.c_int, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                     C.POINTER(C.c_float)]),
}

EXPORTED = tuple(_SIGS)

_lib = None


def load() -> C.CDLL:
    """Load the in-tree HIP library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build()); "
                           "the routing engine has no non-HIP fallback")
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.orl_abi_version() != ABI_VERSION:
        raise RuntimeError("liborleans_route.so ABI version mismatch")
    _lib = lib
    return lib


def ptr(a) -> C.c_void_p:
    """Raw pointer of a numpy array (C-contiguous) or a torch tensor (data_ptr), or None."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
        return C.c_void_p(a.ctypes.data)
    if hasattr(a, "data_ptr"):
        return C.c_void_p(a.data_ptr())
    if isinstance(a, int):
        return C.c_void_p(a)
    raise TypeError(f"cannot take a pointer of {type(a)}")


class OrleansRouteError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"orleans_route error {code}: {msg}")
        self.code = code
