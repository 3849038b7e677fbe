"""ctypes binding of oracle/liborleans_cpu_ref.so (the C++ restatement in cpu_ref.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liborleans_cpu_ref.so")

KEY_DTYPE = np.dtype([("tcd", "<u8"), ("n0", "<u8"), ("n1", "<u8")])
MSG_DTYPE = np.dtype([("tcd", "<u8"), ("n0", "<u8"), ("n1", "<u8"), ("sending_silo", "u1"), ("category", "u1"),
                      ("flags", "u1"), ("target_silo", "u1"), ("aux", "<u4")])


class RefCluster(C.Structure):
    _fields_ = [("n_silos", C.c_uint32), ("ring_n", C.c_uint32), ("ring_hash", C.c_int32 * 256),
                ("ring_silo", C.c_uint8 * 256), ("running", C.c_uint8 * 256), ("functional", C.c_uint8 * 256),
                ("local", C.c_uint8 * 256), ("seed", C.c_uint32), ("policy", C.c_uint32)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    P = C.c_void_p
    sigs = {
        "ref_jenkins_u64": (C.c_uint32, [C.c_uint64, C.c_uint64, C.c_uint64]),
        "ref_jenkins_bytes": (C.c_uint32, [C.c_char_p, C.c_size_t]),
        "ref_ring_add": (C.c_int, [P, C.c_uint32, C.c_int32]),
        "ref_ring_remove": (C.c_int, [P, C.c_uint32]),
        "ref_dir_new": (P, []),
        "ref_dir_free": (None, [P]),
        "ref_dir_size": (C.c_uint64, [P]),
        "ref_register": (C.c_int, [P, P, P, P, P, C.c_size_t, P, P, P]),
        "ref_unregister": (C.c_int, [P, P, C.c_size_t, P]),
        "ref_route": (C.c_int, [P, P, P, C.c_size_t, C.c_uint32, P, P]),
        "ref_bucket": (C.c_int, [P, C.c_size_t, C.c_uint32, P, P]),
        "ref_route_bucket_mt": (C.c_int, [P, P, P, C.c_size_t, C.c_uint32, C.c_uint32, P, P, P, P, C.c_int]),
        "ref_fanout_expand": (C.c_size_t, [P, P, P, P, C.c_size_t, C.c_uint64, P, C.c_size_t, P]),
        "ref_partition": (C.c_int, [P, P, C.c_size_t, C.c_uint32, P, C.c_uint32, C.c_uint32, P, P]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


class Oracle:
    """One cluster view + one directory partition, restated on the CPU."""

    def __init__(self, n_silos: int, running: Optional[Sequence[int]] = None, functional: Optional[Sequence[int]] = None,
                 local: Optional[Sequence[int]] = None, seed: int = 0xFF, policy: int = 0):
        self.lib = load()
        cl = RefCluster()
        cl.n_silos = n_silos
        cl.ring_n = 0
        for i in range(256):
            cl.running[i] = 1 if (running is None or (i < n_silos and running[i])) else 0
            cl.functional[i] = 1 if (functional is None or (i < n_silos and functional[i])) else 0
            cl.local[i] = 1 if (local is None or (i < n_silos and local[i])) else 0
        for i in range(n_silos, 256):
            cl.running[i] = cl.functional[i] = cl.local[i] = 0
        cl.seed = seed
        cl.policy = policy
        self.cl = cl
        self.dir = self.lib.ref_dir_new()

    def __del__(self):
        try:
            self.lib.ref_dir_free(self.dir)
        except Exception:
            pass

    def add_server(self, silo: int, h: int) -> None:
        assert self.lib.ref_ring_add(C.byref(self.cl), silo, h) == 0

    def remove_server(self, silo: int) -> None:
        self.lib.ref_ring_remove(C.byref(self.cl), silo)

    def ring(self):
        return [(self.cl.ring_hash[i], self.cl.ring_silo[i]) for i in range(self.cl.ring_n)]

    def register(self, keys: np.ndarray, acts: np.ndarray, silos: np.ndarray):
        keys = np.ascontiguousarray(keys, KEY_DTYPE)
        acts = np.ascontiguousarray(acts, np.uint32)
        silos = np.ascontiguousarray(silos, np.uint8)
        n = len(keys)
        st = np.zeros(n, np.uint8)
        wa = np.zeros(n, np.uint32)
        ws = np.zeros(n, np.uint8)
        self.lib.ref_register(C.byref(self.cl), self.dir, _p(keys), _p(acts), _p(silos), n, _p(st), _p(wa), _p(ws))
        return st, wa, ws

    def unregister(self, keys: np.ndarray) -> np.ndarray:
        keys = np.ascontiguousarray(keys, KEY_DTYPE)
        out = np.zeros(len(keys), np.uint8)
        self.lib.ref_unregister(self.dir, _p(keys), len(keys), _p(out))
        return out

    def size(self) -> int:
        return self.lib.ref_dir_size(self.dir)

    def route(self, msgs: np.ndarray, opts: int = 0):
        msgs = np.ascontiguousarray(msgs, MSG_DTYPE)
        n = len(msgs)
        route = np.zeros(n, np.uint32)
        act = np.zeros(n, np.uint32)
        self.lib.ref_route(C.byref(self.cl), self.dir, _p(msgs), n, opts, _p(route), _p(act))
        return route, act

    def bucket(self, act: np.ndarray, n_act: int):
        act = np.ascontiguousarray(act, np.uint32)
        order = np.zeros(len(act), np.uint32)
        off = np.zeros(n_act + 2, np.uint32)
        self.lib.ref_bucket(_p(act), len(act), n_act, _p(order), _p(off))
        return order, off

    def route_bucket_mt(self, msgs: np.ndarray, n_act: int, nthreads: int, opts: int = 0):
        msgs = np.ascontiguousarray(msgs, MSG_DTYPE)
        n = len(msgs)
        route = np.zeros(n, np.uint32)
        act = np.zeros(n, np.uint32)
        order = np.zeros(n, np.uint32)
        off = np.zeros(n_act + 2, np.uint32)
        self.lib.ref_route_bucket_mt(C.byref(self.cl), self.dir, _p(msgs), n, opts, n_act, _p(route), _p(act),
                                     _p(order), _p(off), nthreads)
        return route, act, order, off

    def partition(self, msgs: np.ndarray, rank_of_silo: Sequence[int], nranks: int, my_rank: int, opts: int = 0):
        msgs = np.ascontiguousarray(msgs, MSG_DTYPE)
        ros = np.zeros(256, np.uint8)
        ros[:len(rank_of_silo)] = rank_of_silo
        src = np.zeros(len(msgs), np.uint32)
        counts = np.zeros(nranks, np.uint64)
        self.lib.ref_partition(C.byref(self.cl), _p(msgs), len(msgs), opts, _p(ros), nranks, my_rank, _p(src),
                               _p(counts))
        return src, counts


def jenkins_u64(u1: int, u2: int, u3: int) -> int:
    return load().ref_jenkins_u64(u1, u2, u3)


def jenkins_bytes(b: bytes) -> int:
    return load().ref_jenkins_bytes(b, len(b))


def fanout_expand(csr_off: np.ndarray, csr_tgt: np.ndarray, pubs: np.ndarray, pub_silo: np.ndarray, follower_tcd: int):
    lib = load()
    csr_off = np.ascontiguousarray(csr_off, np.uint64)
    csr_tgt = np.ascontiguousarray(csr_tgt, np.uint32)
    pubs = np.ascontiguousarray(pubs, np.uint32)
    pub_silo = np.ascontiguousarray(pub_silo, np.uint8)
    n = lib.ref_fanout_expand(_p(csr_off), _p(csr_tgt), _p(pubs), _p(pub_silo), len(pubs), follower_tcd, None, 0, None)
    out = np.zeros(n, MSG_DTYPE)
    poff = np.zeros(len(pubs) + 1, np.uint64)
    lib.ref_fanout_expand(_p(csr_off), _p(csr_tgt), _p(pubs), _p(pub_silo), len(pubs), follower_tcd, _p(out), n,
                          _p(poff))
    return out, poff


# ---- compact exchange record (orl_wire_msg, include/orleans_route.h) --------------------------------------
# Independent numpy restatement of the 16-byte wire codec, used to check the GPU encoder / decoder.
# Compact form exists iff N0 == 0 and TypeCodeData = (category << 56) + sign-extended int type code
# (UniqueKey.NewKey, UniqueKey.cs:131-152), message category < 4, flags < 64 without HASH_VALID.
WIRE_DTYPE = np.dtype([("n1", "<u8"), ("type_code_lo", "<u4"), ("meta", "<u4")])
_LOW56 = np.uint64(0x00FFFFFFFFFFFFFF)


def wire_encode(msgs: np.ndarray):
    """-> (records, compactable mask)."""
    tcd = msgs["tcd"].astype(np.uint64)
    lo = (tcd & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    sext = lo.view(np.int32).astype(np.int64).view(np.uint64) & _LOW56
    ok = (msgs["n0"] == 0) & ((tcd & _LOW56) == sext) & (msgs["category"] < 4) & (msgs["flags"] < 64) & \
         ((msgs["flags"] & 0x02) == 0)
    r = np.zeros(len(msgs), WIRE_DTYPE)
    r["n1"] = msgs["n1"]
    r["type_code_lo"] = lo
    r["meta"] = (msgs["sending_silo"].astype(np.uint32) | (msgs["category"].astype(np.uint32) << 8) |
                 (msgs["flags"].astype(np.uint32) << 10) | ((tcd >> np.uint64(56)).astype(np.uint32) << 16) |
                 (msgs["target_silo"].astype(np.uint32) << 24))
    return r, ok


# ---- narrow exchange record (orl_wire8, include/orleans_route.h) ------------------------------------------
# 8-byte form: N1 < 2^32, N0 == 0, TypeCodeData one of the node's wire types (its index is carried), message
# category < 4, flags < 64 without HASH_VALID.  Same restatement role as wire_encode.
WIRE8_DTYPE = np.dtype([("n1", "<u4"), ("meta", "<u4")])


def narrow_encode(msgs: np.ndarray, wire_types):
    """-> (records, narrow-able mask) for the wire-type list `wire_types` (<= 16 TypeCodeData values)."""
    tcd = msgs["tcd"].astype(np.uint64)
    types = np.asarray(list(wire_types), np.uint64)
    idx = np.full(len(msgs), 16, np.uint32)
    for i, t in enumerate(types):
        idx[tcd == t] = i
    ok = (msgs["n0"] == 0) & (msgs["n1"] < np.uint64(1 << 32)) & (idx < 16) & (msgs["category"] < 4) & \
         (msgs["flags"] < 64) & ((msgs["flags"] & 0x02) == 0)
    r = np.zeros(len(msgs), WIRE8_DTYPE)
    r["n1"] = (msgs["n1"] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    r["meta"] = (msgs["sending_silo"].astype(np.uint32) | ((msgs["category"].astype(np.uint32) & 0xFF) << 8) |
                 ((msgs["flags"].astype(np.uint32) & 0xFF) << 10) | ((idx & 0xF) << 16) |
                 (msgs["target_silo"].astype(np.uint32) << 24))
    return r, ok


def wire_decode(recs: np.ndarray) -> np.ndarray:
    m = np.zeros(len(recs), MSG_DTYPE)
    meta = recs["meta"].astype(np.uint32)
    sext = recs["type_code_lo"].view(np.int32).astype(np.int64).view(np.uint64) & _LOW56
    m["tcd"] = (((meta >> 16) & 0xFF).astype(np.uint64) << np.uint64(56)) | sext
    m["n1"] = recs["n1"]
    m["sending_silo"] = (meta & 0xFF).astype(np.uint8)
    m["category"] = ((meta >> 8) & 0x3).astype(np.uint8)
    m["flags"] = ((meta >> 10) & 0x3F).astype(np.uint8)
    m["target_silo"] = (meta >> 24).astype(np.uint8)
    return m
