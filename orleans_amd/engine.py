"""Host-side mirror of the reference's routing interfaces over the C ABI.

``GrainDirectoryEngine`` is the batched stand-in for one GPU's worth of silos.  Its methods keep the
names and argument meaning of the reference calls they replace (paths relative to randa1/orleans):

=============================  ==================================================================
engine method                  reference
=============================  ==================================================================
set_silos / add_server /       LocalGrainDirectory.SiloStatusChangeNotification → AddServer /
remove_server                  RemoveServer (src/OrleansRuntime/GrainDirectory/LocalGrainDirectory.cs:243-304,390-419)
calculate_target_silo          LocalGrainDirectory.CalculateTargetSilo (:439-497)
register_single_activation     LocalGrainDirectory.RegisterSingleActivationAsync (:510-544) →
                               GrainDirectoryPartition.AddSingleActivation (GrainDirectoryPartition.cs:270-287)
unregister                     LocalGrainDirectory.UnregisterAsync (:587-612) → RemoveActivation(force)
address_messages               Dispatcher.AddressMessage (src/OrleansRuntime/Core/Dispatcher.cs:555-579) for a
                               batch, + per-activation FIFO grouping (ActivationData.cs:483-514)
hash_batch                     GrainId.GetUniformHashCode (src/Orleans/IDs/GrainId.cs:211-214)
=============================  ==================================================================

Error behaviour: API errors raise ``OrleansRouteError`` (the reference throws ArgumentException /
InvalidOperationException); per-message outcomes are status codes in the route word, which
``decode_route`` unpacks, and ``raise_for_status`` maps to the reference's exception types.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib as L
from ._lib import OrleansRouteError, ptr


def _check(lib, ctx, rc: int) -> None:
    if rc != L.OK:
        msg = lib.orl_last_error(ctx) if ctx else b""
        raise OrleansRouteError(rc, (msg or b"").decode(errors="replace"))


# ---- identity helpers (no context, host only) ---------------------------------------------------------
def calc_id_hash(text: str) -> int:
    """Utils.CalculateIdHash (src/Orleans/Utils/Utils.cs:201-220)."""
    lib = L.load()
    b = text.encode("utf-8")
    out = C.c_int32()
    _check(lib, None, lib.orl_calc_id_hash(b, len(b), C.byref(out)))
    return out.value


def silo_consistent_hash(endpoint: str, generation: int) -> int:
    """SiloAddress.GetConsistentHashCode (src/Orleans/IDs/SiloAddress.cs:197-206)."""
    lib = L.load()
    out = C.c_int32()
    _check(lib, None, lib.orl_silo_consistent_hash(endpoint.encode("utf-8"), int(generation), C.byref(out)))
    return out.value


def jenkins_bytes(data: bytes) -> int:
    """JenkinsHash.ComputeHash(byte[]) (src/Orleans/IDs/JenkinsHash.cs:68-115)."""
    return L.load().orl_jenkins_bytes(data, len(data))


def keyext_uniform_hash(tcd: int, n0: int, n1: int, key_ext: str) -> int:
    """UniqueKey.GetUniformHashCode, KeyExt branch (src/Orleans/IDs/UniqueKey.cs:288-294)."""
    k = np.zeros(1, L.KEY_DTYPE)
    k["tcd"], k["n0"], k["n1"] = tcd, n0, n1
    b = key_ext.encode("utf-8")
    return L.load().orl_keyext_uniform_hash(ptr(k), b, len(b))


def type_code_data(category: int, type_code: int) -> int:
    """UniqueKey.NewKey: TypeCodeData = (category << 56) + (typeData & 0x00FFFFFFFFFFFFFF) (UniqueKey.cs:141);
    an int type code is sign-extended to long first (GrainInterfaceMap.cs:437)."""
    return ((category & 0xFF) << 56) + (type_code & 0xFFFFFFFFFFFFFFFF & 0x00FFFFFFFFFFFFFF)


def grain_keys_from_longs(type_code: int, keys: np.ndarray, category: int = L.CAT_GRAIN) -> np.ndarray:
    """GrainId.GetGrainId(typeCode, long) for an array of long keys (GrainId.cs:90-95, UniqueKey.cs:146-152)."""
    out = np.zeros(len(keys), L.KEY_DTYPE)
    out["tcd"] = np.uint64(type_code_data(category, type_code))
    out["n1"] = np.asarray(keys).astype(np.int64).view(np.uint64)
    return out


def grain_keys_from_guid_bytes(type_code: int, guid_bytes: np.ndarray, category: int = L.CAT_GRAIN) -> np.ndarray:
    """GrainId.GetGrainId(typeCode, Guid) with Guid.ToByteArray() rows (UniqueKey.cs:159-167)."""
    gb = np.ascontiguousarray(guid_bytes, dtype=np.uint8).reshape(-1, 16)
    out = np.zeros(len(gb), L.KEY_DTYPE)
    out["tcd"] = np.uint64(type_code_data(category, type_code))
    out["n0"] = gb[:, 0:8].copy().view("<u8").ravel()
    out["n1"] = gb[:, 8:16].copy().view("<u8").ravel()
    return out


# ---- route word -------------------------------------------------------------------------------------
@dataclass
class RouteView:
    owner: np.ndarray
    host: np.ndarray
    status: np.ndarray
    flags: np.ndarray


def decode_route(route: np.ndarray) -> RouteView:
    r = np.asarray(route, dtype=np.uint32)
    return RouteView((r & 0xFF).astype(np.uint8), ((r >> 8) & 0xFF).astype(np.uint8),
                     ((r >> 16) & 0xFF).astype(np.uint8), ((r >> 24) & 0xFF).astype(np.uint8))


class GrainDirectoryStopping(RuntimeError):
    """InvalidOperationException("Grain directory is stopping") (LocalGrainDirectory.cs:514-518)."""


class UnregisteredClient(KeyError):
    """KeyNotFoundException for a client pseudo-grain (PlacementDirectorsManager.cs:75-81)."""


class NoSeed(ValueError):
    """ArgumentException: membership table grain without a Seed (LocalGrainDirectory.cs:449-460)."""


def raise_for_status(route_word: int) -> None:
    st = (int(route_word) >> 16) & 0xFF
    if st == L.ST_OWNER_NULL:
        raise GrainDirectoryStopping("Grain directory is stopping")
    if st == L.ST_CLIENT_UNREGISTERED:
        raise UnregisteredClient("No activation for client")
    if st == L.ST_NO_SEED:
        raise NoSeed("MembershipTableGrain cannot run without Seed node")


@dataclass
class RouteResult:
    route: np.ndarray      # uint32[n]
    act: np.ndarray        # uint32[n]
    order: Optional[np.ndarray]    # uint32[n]: message indices grouped per activation (FIFO)
    offsets: Optional[np.ndarray]  # uint32[n_act+2]

    def bucket(self, act: int) -> np.ndarray:
        return self.order[self.offsets[act]:self.offsets[act + 1]]


class GrainDirectoryEngine:
    """One context of liborleans_route.so (one GPU, one or more logical silos)."""

    def __init__(self, n_act: int, dir_capacity: int, max_batch: int = 1 << 20, device: int = 0,
                 placement: int = L.POLICY_PREFER_LOCAL):
        self._lib = L.load()
        cfg = L.orl_config(L.ABI_VERSION, int(device), int(dir_capacity), int(n_act), int(placement), int(max_batch))
        h = C.c_void_p()
        rc = self._lib.orl_ctx_create(C.byref(cfg), C.byref(h))
        if rc != L.OK:
            raise OrleansRouteError(rc, "orl_ctx_create failed (device=%d)" % device)
        self._ctx = h
        self.n_act = int(n_act)
        self.max_batch = int(max_batch)
        self.device = int(device)
        self.n_silos = 0

    # -- lifecycle
    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.orl_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _ck(self, rc: int) -> None:
        _check(self._lib, self._ctx, rc)

    @property
    def handle(self) -> C.c_void_p:
        return self._ctx

    # -- membership view
    def set_silos(self, n_silos: int, running: Optional[Sequence[bool]] = None,
                  functional: Optional[Sequence[bool]] = None, local: Optional[Sequence[bool]] = None,
                  seed: int = L.NULL_SILO) -> None:
        def arr(v):
            return None if v is None else np.ascontiguousarray(np.asarray(v, dtype=np.uint8))
        r, f, lo = arr(running), arr(functional), arr(local)
        self._ck(self._lib.orl_silos_set(self._ctx, int(n_silos), ptr(r), ptr(f), ptr(lo), int(seed)))
        self.n_silos = int(n_silos)

    def add_server(self, silo: int, consistent_hash: int) -> None:
        self._ck(self._lib.orl_ring_add_server(self._ctx, int(silo), int(consistent_hash)))

    def remove_server(self, silo: int) -> None:
        self._ck(self._lib.orl_ring_remove_server(self._ctx, int(silo)))

    def membership_ring(self):
        n = C.c_uint32()
        hs = np.zeros(256, np.int32)
        ss = np.zeros(256, np.uint8)
        self._ck(self._lib.orl_ring_get(self._ctx, ptr(hs), ptr(ss), 256, C.byref(n)))
        return [(int(hs[i]), int(ss[i])) for i in range(n.value)]

    # -- directory partition
    def register_single_activation(self, keys: np.ndarray, acts: np.ndarray, silos: np.ndarray):
        keys = np.ascontiguousarray(keys, dtype=L.KEY_DTYPE)
        acts = np.ascontiguousarray(acts, dtype=np.uint32)
        silos = np.ascontiguousarray(silos, dtype=np.uint8)
        n = len(keys)
        assert len(acts) == n and len(silos) == n
        st = np.zeros(n, np.uint8)
        wa = np.zeros(n, np.uint32)
        ws = np.zeros(n, np.uint8)
        self._ck(self._lib.orl_dir_insert_single(self._ctx, ptr(keys), ptr(acts), ptr(silos), n, ptr(wa), ptr(ws),
                                                 ptr(st)))
        return st, wa, ws

    # -- KeyExt (string-key) grains: their own device table (orl_dir_*_keyext)
    @staticmethod
    def ext_blob(strings):
        """(orl_ext_ref array, UTF-8 blob) for a sequence of str / bytes."""
        bs = [x.encode("utf-8") if isinstance(x, str) else bytes(x) for x in strings]
        ref = np.zeros(len(bs), L.EXT_REF_DTYPE)
        off = 0
        for i, b in enumerate(bs):
            ref[i] = (off, len(b))
            off += len(b)
        blob = np.frombuffer(b"".join(bs) or b"\0", np.uint8).copy()
        return ref, blob

    def register_keyext(self, keys: np.ndarray, strings, acts: np.ndarray, silos: np.ndarray):
        """RegisterSingleActivation of KeyExt grains (orl_dir_insert_keyext): (status, winner act, winner silo)."""
        keys = np.ascontiguousarray(keys, dtype=L.KEY_DTYPE)
        ref, blob = self.ext_blob(strings)
        acts = np.ascontiguousarray(acts, dtype=np.uint32)
        silos = np.ascontiguousarray(silos, dtype=np.uint8)
        n = len(keys)
        st, wa, ws = np.zeros(n, np.uint8), np.zeros(n, np.uint32), np.zeros(n, np.uint8)
        self._ck(self._lib.orl_dir_insert_keyext(self._ctx, ptr(keys), ptr(ref), ptr(blob), int(ref["len"].sum()), ptr(acts),
                                                 ptr(silos), n, ptr(wa), ptr(ws), ptr(st)))
        return st, wa, ws

    def register_keyext_device(self, d_keys, d_ext, d_blob, blob_bytes: int, d_acts, d_silos, n: int, d_status,
                               d_winner_act=None, d_winner_silo=None, stream=None):
        """RegisterSingleActivation of KeyExt grains on the device (orl_dir_insert_keyext_device): device arrays, async on
        `stream`; statuses / winners written to the device buffers."""
        self._ck(self._lib.orl_dir_insert_keyext_device(self._ctx, ptr(d_keys), ptr(d_ext), ptr(d_blob), int(blob_bytes),
                                                        ptr(d_acts), ptr(d_silos), int(n), ptr(d_winner_act),
                                                        ptr(d_winner_silo), ptr(d_status), ptr(stream)))

    def unregister_keyext(self, keys: np.ndarray, strings) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=L.KEY_DTYPE)
        ref, blob = self.ext_blob(strings)
        out = np.zeros(len(keys), np.uint8)
        self._ck(self._lib.orl_dir_remove_keyext(self._ctx, ptr(keys), ptr(ref), ptr(blob), int(ref["len"].sum()), len(keys),
                                                 ptr(out)))
        return out

    def lookup_keyext_host(self, keys: np.ndarray, strings):
        keys = np.ascontiguousarray(keys, dtype=L.KEY_DTYPE)
        ref, blob = self.ext_blob(strings)
        a, s = np.zeros(len(keys), np.uint32), np.zeros(len(keys), np.uint8)
        self._ck(self._lib.orl_dir_lookup_keyext_host(self._ctx, ptr(keys), ptr(ref), ptr(blob), int(ref["len"].sum()),
                                                      len(keys), ptr(a), ptr(s)))
        return a, s

    def keyext_count(self) -> int:
        n = C.c_uint64()
        self._ck(self._lib.orl_dir_keyext_count(self._ctx, C.byref(n)))
        return n.value

    def address_keyext_device(self, d_msgs, n: int, d_ext, d_blob, blob_bytes: int, d_route, d_act, d_order=None,
                              d_offsets=None, stream=None, opts: int = 0) -> None:
        """orl_route_keyext_device: the batch routed with its KeyExt strings (d_ext: orl_ext_ref per message into d_blob)."""
        self._ck(self._lib.orl_route_keyext_device(self._ctx, ptr(d_msgs), int(n), int(opts), ptr(d_ext), ptr(d_blob),
                                                   int(blob_bytes), ptr(d_route), ptr(d_act), ptr(d_order), ptr(d_offsets),
                                                   ptr(stream)))

    def unregister(self, keys: np.ndarray) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=L.KEY_DTYPE)
        out = np.zeros(len(keys), np.uint8)
        self._ck(self._lib.orl_dir_remove(self._ctx, ptr(keys), len(keys), ptr(out)))
        return out

    def directory_count(self) -> int:
        n = C.c_uint64()
        self._ck(self._lib.orl_dir_count(self._ctx, C.byref(n)))
        return n.value

    def lookup_host(self, keys: np.ndarray):
        keys = np.ascontiguousarray(keys, dtype=L.KEY_DTYPE)
        a = np.zeros(len(keys), np.uint32)
        s = np.zeros(len(keys), np.uint8)
        self._ck(self._lib.orl_dir_lookup_host(self._ctx, ptr(keys), len(keys), ptr(a), ptr(s)))
        return a, s

    # -- hot path (host buffers)
    def hash_batch(self, keys: np.ndarray) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=L.KEY_DTYPE)
        out = np.zeros(len(keys), np.uint32)
        self._ck(self._lib.orl_hash_batch(self._ctx, ptr(keys), len(keys), ptr(out)))
        return out

    def address_messages(self, msgs: np.ndarray, opts: int = 0) -> RouteResult:
        msgs = np.ascontiguousarray(msgs, dtype=L.MSG_DTYPE)
        n = len(msgs)
        route = np.zeros(n, np.uint32)
        act = np.zeros(n, np.uint32)
        buckets = not (opts & L.OPT_NO_BUCKETS)
        order = np.zeros(n, np.uint32) if buckets else None
        offsets = np.zeros(self.n_act + 2, np.uint32) if buckets else None
        self._ck(self._lib.orl_route_batch(self._ctx, ptr(msgs), n, int(opts), ptr(route), ptr(act), ptr(order),
                                           ptr(offsets)))
        return RouteResult(route, act, order, offsets)

    def route_batch_host(self, msgs: np.ndarray, route: np.ndarray, act: np.ndarray, order: np.ndarray,
                         offsets: np.ndarray, opts: int = 0) -> None:
        """orl_route_batch into caller-owned host arrays (the P/Invoke call shape; pin them with host_register)."""
        self._ck(self._lib.orl_route_batch(self._ctx, ptr(msgs), len(msgs), int(opts), ptr(route), ptr(act), ptr(order),
                                           ptr(offsets)))

    def route_batch_narrow_host(self, recs: np.ndarray, route: np.ndarray, act: np.ndarray, order: Optional[np.ndarray],
                                offsets: Optional[np.ndarray], opts: int = 0) -> None:
        """orl_route_batch_narrow: 8-B orl_wire8 records (uint32 pairs {n1, meta}) in host memory, outputs into caller
        arrays (order / offsets None: ORL_OPT_NO_BUCKETS)."""
        if order is None:
            opts |= L.OPT_NO_BUCKETS
        n = recs.size * recs.itemsize // 8
        self._ck(self._lib.orl_route_batch_narrow(self._ctx, ptr(recs), n, int(opts), ptr(route), ptr(act), ptr(order),
                                                  ptr(offsets)))

    def host_register(self, a: np.ndarray) -> None:
        """Page-lock a host array for asynchronous full-rate copies (a pinned GCHandle buffer on the C# side)."""
        self._ck(self._lib.orl_host_register(self._ctx, ptr(a), a.nbytes))

    def host_unregister(self, a: np.ndarray) -> None:
        self._ck(self._lib.orl_host_unregister(self._ctx, ptr(a)))

    def calculate_target_silo(self, keys: np.ndarray, me: int, exclude_if_stopping: bool = True) -> np.ndarray:
        """Owner silo per key as silo `me` computes it (0xFF = null)."""
        keys = np.ascontiguousarray(keys, dtype=L.KEY_DTYPE)
        m = np.zeros(len(keys), L.MSG_DTYPE)
        m["tcd"], m["n0"], m["n1"] = keys["tcd"], keys["n0"], keys["n1"]
        m["sending_silo"] = me
        r = self.address_messages(m, L.OPT_NO_BUCKETS | (L.OPT_EXCLUDE_IF_STOPPING if exclude_if_stopping else 0))
        return decode_route(r.route).owner

    # -- hot path (device-resident; torch tensors or raw device pointers)
    def address_messages_device(self, d_msgs, n: int, d_route, d_act, d_order=None, d_offsets=None, stream=None,
                                opts: int = 0) -> None:
        self._ck(self._lib.orl_route_batch_device(self._ctx, ptr(d_msgs), int(n), int(opts), ptr(d_route),
                                                  ptr(d_act), ptr(d_order), ptr(d_offsets), ptr(stream)))

    def fanout_device(self, d_csr_off, d_csr_tgt, d_pubs, d_pub_silo, n_pub: int, follower_tcd: int,
                      d_pub_offsets, d_route, d_act, d_order=None, d_offsets=None, stream=None, opts: int = 0,
                      total: Optional[int] = None) -> int:
        """ChirperAccount.PublishMessage fan-out (Samples/Chirper/ChirperGrains/ChirperAccount.cs:154-157) + stages 1-4.
        `total` (exact emitted count) makes the call sync-free and hipGraph-capturable."""
        if total is not None:
            opts |= L.OPT_TOTAL_GIVEN
        n_out = C.c_uint64(int(total or 0))
        self._ck(self._lib.orl_fanout_route_device(self._ctx, ptr(d_csr_off), ptr(d_csr_tgt), ptr(d_pubs),
                                                   ptr(d_pub_silo), int(n_pub), int(follower_tcd), int(opts),
                                                   ptr(d_pub_offsets), ptr(d_route), ptr(d_act), ptr(d_order),
                                                   ptr(d_offsets), C.byref(n_out), ptr(stream)))
        return n_out.value

    def fanout_keys_device(self, d_csr_off, d_csr_tgt, d_follower_keys, d_pubs, d_pub_silo, n_pub: int, d_pub_offsets,
                           d_route, d_act, d_order=None, d_offsets=None, stream=None, opts: int = 0,
                           total: Optional[int] = None) -> int:
        """Fan-out to followers named by a device key table (GameGrain.UpdateGameStatus players,
        Samples/Presence/PresenceGrains/GameGrain.cs:62-113)."""
        if total is not None:
            opts |= L.OPT_TOTAL_GIVEN
        n_out = C.c_uint64(int(total or 0))
        self._ck(self._lib.orl_fanout_route_keys_device(self._ctx, ptr(d_csr_off), ptr(d_csr_tgt), ptr(d_follower_keys),
                                                        ptr(d_pubs), ptr(d_pub_silo), int(n_pub), int(opts),
                                                        ptr(d_pub_offsets), ptr(d_route), ptr(d_act), ptr(d_order),
                                                        ptr(d_offsets), C.byref(n_out), ptr(stream)))
        return n_out.value

    def fanout_mixed_device(self, d_direct, n_direct: int, d_csr_off, d_csr_tgt, d_follower_keys, follower_tcd: int,
                            d_pubs, d_pub_silo, n_pub: int, d_pub_offsets, d_route, d_act, d_order=None, d_offsets=None,
                            stream=None, opts: int = 0, total: Optional[int] = None) -> int:
        """n_direct direct messages + a CSR fan-out routed and bucketed as ONE batch (output [0, n_direct) = the direct
        messages, then the fan-out; pub_offsets absolute).  d_follower_keys None = GrainId(follower_tcd, long id).
        `total` = n_direct + emitted makes the call sync-free.  Returns that total."""
        if total is not None:
            opts |= L.OPT_TOTAL_GIVEN
        n_out = C.c_uint64(int(total or 0))
        self._ck(self._lib.orl_fanout_route_mixed_device(self._ctx, ptr(d_direct), int(n_direct), ptr(d_csr_off),
                                                         ptr(d_csr_tgt), ptr(d_follower_keys), int(follower_tcd),
                                                         ptr(d_pubs), ptr(d_pub_silo), int(n_pub), int(opts),
                                                         ptr(d_pub_offsets), ptr(d_route), ptr(d_act), ptr(d_order),
                                                         ptr(d_offsets), C.byref(n_out), ptr(stream)))
        return n_out.value

    def fanout_expand_device(self, d_csr_off, d_csr_tgt, d_follower_keys, follower_tcd: int, d_pubs, d_pub_silo, n_pub: int,
                             d_pub_offsets, d_out, cap: int, stream=None, opts: int = 0, total: Optional[int] = None) -> int:
        """Stage 5 alone: the emitted messages as orl_msg_hdr records (ChirperAccount.cs:154-157). Returns the count."""
        if total is not None:
            opts |= L.OPT_TOTAL_GIVEN
        n_out = C.c_uint64(int(total or 0))
        self._ck(self._lib.orl_fanout_expand_device(self._ctx, ptr(d_csr_off), ptr(d_csr_tgt), ptr(d_follower_keys),
                                                    int(follower_tcd), ptr(d_pubs), ptr(d_pub_silo), int(n_pub), int(opts),
                                                    ptr(d_pub_offsets), ptr(d_out), int(cap), C.byref(n_out), ptr(stream)))
        return n_out.value

    def partition_by_owner_device(self, d_msgs, n: int, rank_of_silo: Sequence[int], nranks: int, my_rank: int,
                                  d_out, d_src_index, d_counts, stream=None, opts: int = 0) -> None:
        ros = np.zeros(256, np.uint8)
        ros[:len(rank_of_silo)] = np.asarray(rank_of_silo, dtype=np.uint8)
        self._ck(self._lib.orl_partition_by_owner_device(self._ctx, ptr(d_msgs), int(n), int(opts), ptr(ros),
                                                         int(nranks), int(my_rank), ptr(d_out), ptr(d_src_index),
                                                         ptr(d_counts), ptr(stream)))

    def partition_by_owner_padded_device(self, d_msgs, n: int, rank_of_silo: Sequence[int], nranks: int,
                                         my_rank: int, stride: int, d_out, d_counts, d_src_index=None, stream=None,
                                         opts: int = 0) -> None:
        """One-pass owner partition into padded per-rank send regions d_out[r * stride:] (the per-target-silo
        queues of OutboundMessageQueue.SendMessage, OutboundMessageQueue.cs:137-145)."""
        ros = np.zeros(256, np.uint8)
        ros[:len(rank_of_silo)] = np.asarray(rank_of_silo, dtype=np.uint8)
        self._ck(self._lib.orl_partition_by_owner_padded_device(self._ctx, ptr(d_msgs), int(n), int(opts), ptr(ros),
                                                                int(nranks), int(my_rank), int(stride), ptr(d_out),
                                                                ptr(d_src_index), ptr(d_counts), ptr(stream)))

    def partition_compact_device(self, d_msgs, n: int, rank_of_silo: Sequence[int], nranks: int, my_rank: int,
                                 stride: int, d_out, d_counts, d_status, d_src_index=None, stream=None,
                                 opts: int = 0) -> None:
        """partition_by_owner_padded_device writing 16-B orl_wire_msg records; d_status[0] = 1 if a message
        of the batch has no compact form (the caller then uses the 32-B form for this batch)."""
        ros = np.zeros(256, np.uint8)
        ros[:len(rank_of_silo)] = np.asarray(rank_of_silo, dtype=np.uint8)
        self._ck(self._lib.orl_partition_compact_device(self._ctx, ptr(d_msgs), int(n), int(opts), ptr(ros), int(nranks),
                                                        int(my_rank), int(stride), ptr(d_out), ptr(d_src_index),
                                                        ptr(d_counts), ptr(d_status), ptr(stream)))

    def set_wire_types(self, type_code_data: Sequence[int]) -> None:
        """The TypeCodeData values of the 8-B exchange form (orl_wire_types_set; the same list on every rank)."""
        arr = np.asarray([int(t) & 0xFFFFFFFFFFFFFFFF for t in type_code_data], dtype=np.uint64)
        self._ck(self._lib.orl_wire_types_set(self._ctx, len(arr), arr.ctypes.data if len(arr) else None))
        self.wire_types = arr

    def partition_narrow_device(self, d_msgs, n: int, rank_of_silo: Sequence[int], nranks: int, my_rank: int,
                                stride: int, d_out, d_counts, d_status, d_src_index=None, stream=None,
                                opts: int = 0) -> None:
        """partition_by_owner_padded_device writing 8-B orl_wire8 records; d_status[0] bit 0 = a message has no 16-B
        form, bit 1 = a message has no 8-B form (the records are then invalid)."""
        ros = np.zeros(256, np.uint8)
        ros[:len(rank_of_silo)] = np.asarray(rank_of_silo, dtype=np.uint8)
        self._ck(self._lib.orl_partition_narrow_device(self._ctx, ptr(d_msgs), int(n), int(opts), ptr(ros), int(nranks),
                                                       int(my_rank), int(stride), ptr(d_out), ptr(d_src_index),
                                                       ptr(d_counts), ptr(d_status), ptr(stream)))

    def partition_cached_device(self, d_msgs, n: int, rank_of_silo: Sequence[int], nranks: int, my_rank: int,
                                stride: int, d_out, fmt: int, d_act_out, d_counts, d_status, stream=None, opts: int = 0) -> None:
        """The node's hop-1 partition with this context's directory cache (orl_partition_cached_device): messages with a
        remote owner and a cached grain go to the cached activation's rank, addressed, with the handle in d_act_out."""
        ros = np.zeros(256, np.uint8)
        ros[:len(rank_of_silo)] = np.asarray(rank_of_silo, dtype=np.uint8)
        self._ck(self._lib.orl_partition_cached_device(self._ctx, ptr(d_msgs), int(n), int(opts), ptr(ros), int(nranks),
                                                       int(my_rank), int(stride), ptr(d_out), int(fmt), ptr(d_act_out),
                                                       ptr(d_counts), ptr(d_status), ptr(stream)))

    def route_received_device(self, d_recs, fmt: int, n: int, d_in_act, d_route, d_act, stream=None, opts: int = 0) -> None:
        """Stages 1-3 of received hop-1 records with their act lane (orl_route_received_device): records addressed by the
        sender's cache become HIT | CACHED without a probe."""
        self._ck(self._lib.orl_route_received_device(self._ctx, ptr(d_recs), int(fmt), int(n), int(opts), ptr(d_in_act),
                                                     ptr(d_route), ptr(d_act), ptr(stream)))

    def address_narrow_device(self, d_recs, n: int, d_route, d_act, d_order=None, d_offsets=None, stream=None,
                              opts: int = 0) -> None:
        """address_messages_device over 8-B exchange records (orl_wire8, this context's wire types)."""
        self._ck(self._lib.orl_route_narrow_device(self._ctx, ptr(d_recs), int(n), int(opts), ptr(d_route), ptr(d_act),
                                                   ptr(d_order), ptr(d_offsets), ptr(stream)))

    def address_compact_device(self, d_recs, n: int, d_route, d_act, d_order=None, d_offsets=None, stream=None,
                               opts: int = 0) -> None:
        """address_messages_device over compact exchange records (orl_wire_msg)."""
        self._ck(self._lib.orl_route_compact_device(self._ctx, ptr(d_recs), int(n), int(opts), ptr(d_route), ptr(d_act),
                                                    ptr(d_order), ptr(d_offsets), ptr(stream)))

    def register_single_activation_device(self, d_keys, d_acts, d_silos, n: int, d_status, d_winner_act=None,
                                          d_winner_silo=None, stream=None) -> None:
        """Batched RegisterSingleActivation on the device table (GrainDirectoryPartition.AddSingleActivation,
        GrainDirectoryPartition.cs:270-287), sequential batch-order semantics."""
        self._ck(self._lib.orl_dir_insert_single_device(self._ctx, ptr(d_keys), ptr(d_acts), ptr(d_silos), int(n),
                                                        ptr(d_winner_act), ptr(d_winner_silo), ptr(d_status), ptr(stream)))

    def unregister_device(self, d_keys, n: int, d_removed, stream=None) -> None:
        """Batched Unregister on the device table (GrainDirectoryPartition.RemoveActivation, :290-318)."""
        self._ck(self._lib.orl_dir_remove_device(self._ctx, ptr(d_keys), int(n), ptr(d_removed), ptr(stream)))

    def split_directory_device(self, me: int, d_keys, d_acts, d_silos, cap: int, d_n_out, remove: bool = True,
                               stream=None) -> None:
        """Hand-off split after a ring change (GrainDirectoryHandoffManager.ProcessSiloAddEvent): entries now owned
        by another silo → (d_keys, d_acts, d_silos)[: *d_n_out], tombstoned here with `remove`."""
        self._ck(self._lib.orl_dir_split_device(self._ctx, int(me), L.SPLIT_REMOVE if remove else 0, ptr(d_keys),
                                                ptr(d_acts), ptr(d_silos), int(cap), ptr(d_n_out), ptr(stream)))

    # ---- stream / reminder rings ----
    def vring_set_buckets(self, buckets_per_silo: int) -> None:
        self._ck(self._lib.orl_vring_set_buckets(self._ctx, int(buckets_per_silo)))

    def vring_add_server(self, silo: int, ip16: bytes, port: int, generation: int) -> None:
        """VirtualBucketsRingProvider.AddServer (VirtualBucketsRingProvider.cs:142-169)."""
        b = np.frombuffer(bytes(ip16), np.uint8).copy()
        assert len(b) == 16
        self._ck(self._lib.orl_vring_add_server(self._ctx, int(silo), ptr(b), int(port), int(generation)))

    def vring_remove_server(self, silo: int) -> None:
        self._ck(self._lib.orl_vring_remove_server(self._ctx, int(silo)))

    def vring(self):
        n = C.c_uint32()
        self._ck(self._lib.orl_vring_get(self._ctx, None, None, 0, C.byref(n)))
        hs = np.zeros(max(n.value, 1), np.uint32)
        ss = np.zeros(max(n.value, 1), np.uint8)
        self._ck(self._lib.orl_vring_get(self._ctx, ptr(hs), ptr(ss), n.value, C.byref(n)))
        return hs[:n.value], ss[:n.value]

    def ring_owner_device(self, kind: int, d_keys, n: int, me: int, d_owner, opts: int = 0, stream=None) -> None:
        """CalculateTargetSilo(uint hash) of ConsistentRingProvider / VirtualBucketsRingProvider per key."""
        self._ck(self._lib.orl_ring_owner_batch_device(self._ctx, int(kind), ptr(d_keys), int(n), int(me), int(opts),
                                                       ptr(d_owner), ptr(stream)))

    def stream_queue_device(self, kind: int, d_guids, n: int, n_queues: int, me: int, d_queue, d_silo=None,
                            opts: int = 0, stream=None) -> None:
        """HashRingBasedStreamQueueMapper.GetQueueForStream per stream Guid (+ the silo whose range holds it)."""
        self._ck(self._lib.orl_stream_queue_batch_device(self._ctx, int(kind), ptr(d_guids), int(n), int(n_queues),
                                                         int(me), int(opts), ptr(d_queue), ptr(d_silo), ptr(stream)))

    # ---- directory cache ----
    def cache_config(self, capacity: int) -> None:
        """Allocate the device directory cache (AdaptiveGrainDirectoryCache) for `capacity` remote grains."""
        self._ck(self._lib.orl_cache_config(self._ctx, int(capacity)))

    def cache_clear(self) -> None:
        self._ck(self._lib.orl_cache_clear(self._ctx))

    def cache_add_or_update_device(self, d_keys, d_acts, d_silos, n: int, stream=None) -> None:
        self._ck(self._lib.orl_cache_add_or_update_device(self._ctx, ptr(d_keys), ptr(d_acts), ptr(d_silos), int(n),
                                                          ptr(stream)))

    def cache_remove_device(self, d_keys, n: int, d_removed, stream=None) -> None:
        """Cache invalidation (CACHE_INVALIDATION_HEADER, InsideGrainClient.cs:298-308)."""
        self._ck(self._lib.orl_cache_remove_device(self._ctx, ptr(d_keys), int(n), ptr(d_removed), ptr(stream)))

    def cache_count(self) -> int:
        n = C.c_uint64()
        self._ck(self._lib.orl_cache_count(self._ctx, C.byref(n)))
        return n.value

    # ---- outbound queues / client buckets ----
    def set_silo_hash(self, silo: int, consistent_hash: int) -> None:
        self._ck(self._lib.orl_silo_hash_set(self._ctx, int(silo), int(consistent_hash)))

    def outbound_queues_device(self, d_msgs, d_route, n: int, n_senders: int, d_queue, stream=None) -> None:
        """OutboundMessageQueue.SendMessage's queue per routed message (OutboundMessageQueue.cs:75-150)."""
        self._ck(self._lib.orl_outbound_queues_device(self._ctx, ptr(d_msgs), ptr(d_route), int(n), int(n_senders),
                                                      ptr(d_queue), ptr(stream)))

    def client_buckets_device(self, d_msgs, n: int, n_buckets: int, d_bucket, stream=None) -> None:
        """ProxiedMessageCenter's gateway bucket per message: TargetGrain.GetHashCode_Modulo(n_buckets)."""
        self._ck(self._lib.orl_client_buckets_device(self._ctx, ptr(d_msgs), int(n), int(n_buckets), ptr(d_bucket),
                                                     ptr(stream)))

    def set_silo_address(self, silo: int, ip16: Optional[bytes], port: int = 0, generation: int = 0) -> None:
        """Silo address table of the wire decoder: serialized SiloAddress (16 IP bytes, port, generation) of
        silo index `silo`; ip16 None removes it."""
        if ip16 is None:
            self._ck(self._lib.orl_silo_address_set(self._ctx, int(silo), None, 0, 0))
            return
        b = bytes(ip16)
        if len(b) != 16:
            raise ValueError("ip16 must be 16 bytes")
        buf = (C.c_uint8 * 16).from_buffer_copy(b)
        self._ck(self._lib.orl_silo_address_set(self._ctx, int(silo), buf, int(port), int(generation)))

    def decode_frames_device(self, d_bytes, nbytes: int, d_offsets, n: int, d_out, d_status, d_n_bad=None,
                             sender_override: int = L.SENDER_FROM_HEADER, stream=None) -> None:
        """Received frames -> orl_msg_hdr records + one ORL_DEC_* status byte per frame (device buffers;
        d_bytes 4-byte aligned).  Reference: Message.Serialize_Impl framing + DeserializeMessageHeaders."""
        self._ck(self._lib.orl_decode_frames_device(self._ctx, ptr(d_bytes), int(nbytes), ptr(d_offsets), int(n),
                                                    int(sender_override), ptr(d_out), ptr(d_status), ptr(d_n_bad),
                                                    ptr(stream)))

    def merge_directory_device(self, d_keys, d_acts, d_silos, n: int, d_act_keys, n_act_keys: int, d_status,
                               d_dropped_act=None, d_dropped_silo=None, stream=None) -> None:
        """GrainDirectoryPartition.Merge of a partition copy (ProcessSiloRemoveEvent): absent grains added, present
        ones keep the smaller ActivationId (d_act_keys[handle]); the dropped activation is reported per entry."""
        self._ck(self._lib.orl_dir_merge_device(self._ctx, ptr(d_keys), ptr(d_acts), ptr(d_silos), int(n), ptr(d_act_keys),
                                                int(n_act_keys), ptr(d_status), ptr(d_dropped_act), ptr(d_dropped_silo),
                                                ptr(stream)))

    def set_grain_type(self, type_code: int, class_name: Optional[str]) -> None:
        """Grain class name of a type code (PlacementResult.GrainType of new placements); None removes it."""
        b = b"" if class_name is None else class_name.encode("utf-8")
        self._ck(self._lib.orl_grain_type_set(self._ctx, C.c_int32(int(type_code) & 0xFFFFFFFF).value, b, len(b)))

    def stamp_frames_device(self, d_bytes, nbytes: int, d_offsets, n: int, d_route, d_act, d_act_keys, n_act_keys: int,
                            d_new_act_keys, d_out, out_cap: int, d_out_offsets, d_out_total, d_status,
                            stream=None) -> None:
        """Routed frames re-serialized with Message.SetTargetPlacement applied (device buffers; one ORL_STAMP_*
        status byte per frame; output frame i at d_out_offsets[i], 4-byte aligned)."""
        self._ck(self._lib.orl_stamp_frames_device(self._ctx, ptr(d_bytes), int(nbytes), ptr(d_offsets), int(n), ptr(d_route),
                                                   ptr(d_act), ptr(d_act_keys), int(n_act_keys), ptr(d_new_act_keys),
                                                   ptr(d_out), int(out_cap), ptr(d_out_offsets), ptr(d_out_total),
                                                   ptr(d_status), ptr(stream)))

    def compact_directory(self) -> None:
        """Rebuild the partition without tombstones."""
        self._ck(self._lib.orl_dir_compact(self._ctx))

    def sync(self) -> None:
        self._ck(self._lib.orl_sync(self._ctx))

    def bucket_device(self, d_act, n: int, d_order, d_offsets, stream=None) -> None:
        """Stage 4 alone over routed activation handles (the receiving silo's side of hop 2)."""
        self._ck(self._lib.orl_bucket_device(self._ctx, ptr(d_act), int(n), ptr(d_order), ptr(d_offsets), ptr(stream)))

    def copy_to_host(self, h_dst: np.ndarray, d_src, nbytes: Optional[int] = None, stream=None) -> np.ndarray:
        """orl_copy_to_host + orl_stream_sync (the P/Invoke caller's way to read device outputs)."""
        nb = h_dst.nbytes if nbytes is None else int(nbytes)
        self._ck(self._lib.orl_copy_to_host(self._ctx, ptr(h_dst), ptr(d_src), nb, ptr(stream)))
        self._ck(self._lib.orl_stream_sync(self._ctx, ptr(stream)))
        return h_dst

    def copy_on_device(self, d_dst, d_src, nbytes: int, stream=None) -> None:
        """orl_copy_on_device: device-to-device copy on `stream` (d_dst / d_src: tensors or device pointers)."""
        self._ck(self._lib.orl_copy_on_device(self._ctx, ptr(d_dst), ptr(d_src), int(nbytes), ptr(stream)))

    def csr_set(self, csr_off: np.ndarray, csr_tgt: np.ndarray) -> None:
        """Upload the follower graph once (host-array fan-out, orl_fanout_batch)."""
        off = np.ascontiguousarray(csr_off, dtype=np.uint64)
        tgt = np.ascontiguousarray(csr_tgt, dtype=np.uint32)
        self._ck(self._lib.orl_csr_set(self._ctx, ptr(off), len(off) - 1, ptr(tgt), len(tgt)))

    def fanout_batch(self, pubs: np.ndarray, pub_silo: np.ndarray, follower_tcd: int, cap: int, opts: int = 0):
        """ChirperAccount.PublishMessage for host publisher arrays against the context's follower graph: host outputs
        (route, act, order, bucket offsets, publish offsets)."""
        pubs = np.ascontiguousarray(pubs, dtype=np.uint32)
        ps = np.ascontiguousarray(pub_silo, dtype=np.uint8)
        route, act, order = (np.zeros(cap, np.uint32) for _ in range(3))
        off = np.zeros(self.n_act + 2, np.uint32)
        poff = np.zeros(len(pubs) + 1, np.uint64)
        n_out = C.c_uint64()
        self._ck(self._lib.orl_fanout_batch(self._ctx, ptr(pubs), ptr(ps), len(pubs), int(follower_tcd), int(opts), ptr(poff),
                                            ptr(route), ptr(act), ptr(order), ptr(off), int(cap), C.byref(n_out)))
        n = n_out.value
        return route[:n], act[:n], order[:n], off, poff

    def set_rank_mode(self, mode: int) -> None:
        """Stage-4 ranking: 0 = LDS atomics (self-checked), 1 = ballot match (process-wide on this device)."""
        self._ck(self._lib.orl_ctx_set_rank_mode(self._ctx, int(mode)))

    def query(self, what: int) -> int:
        """orl_ctx_query: L.Q_PROBE_FORM (8 / 16 / 17 / 32), L.Q_FULL_UPLOADS, L.Q_SLOT_PATCHES."""
        v = C.c_uint64()
        self._ck(self._lib.orl_ctx_query(self._ctx, int(what), C.byref(v)))
        return v.value

    def set_timing(self, enable: bool) -> None:
        self._ck(self._lib.orl_set_timing(self._ctx, 1 if enable else 0))

    def timing_summary(self):
        """(batches, avg route-kernel ms, avg bucketing ms, avg call ms) over batches since set_timing(True)."""
        n, a, b, t = C.c_uint32(), C.c_float(), C.c_float(), C.c_float()
        self._ck(self._lib.orl_timing_summary(self._ctx, C.byref(n), C.byref(a), C.byref(b), C.byref(t)))
        return n.value, a.value, b.value, t.value
