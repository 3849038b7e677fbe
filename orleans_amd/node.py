"""Multi-GPU silo node: one process per GPU, the directory sharded by ring range.

The exchange lives behind the C ABI (``orl_node_*``, orleans_amd/csrc/orl_node.cpp): per batch, every rank partitions its
local messages by the rank of their directory owner, all-gathers the per-rank counts, exchanges the records with a grouped
RCCL send/recv (or, ORL_TRANSPORT_LOCAL, device copies between the ranks of one process), routes what it owns, forwards
messages whose activation lives on another rank (hop 2) and buckets what it hosts.  ``GrainNode`` is a thin ctypes wrapper
of that; there is no Python collective on the data path.

``plan_chunk`` / ``plan_hop2`` bind the protocol's host decisions (``orl_node_plan_chunk`` / ``orl_node_plan_hop2``: the
record width of a chunk, the send / receive sizes, the collective capacity errors, whether hop 2 forwards) — the same
functions orl_node_route_batch_device calls after each all-gather.  They are plain host code, so the multi-process CPU
tests (tests/test_distributed.py) run the protocol over gloo with them and check every rank's result against the
single-process replay.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _lib as L

HEAD_WORDS = L.NODE_HEAD_WORDS


@dataclass
class ChunkPlan:
    width: int          # record width every rank exchanges the chunk in (8 / 16 / 32)
    rewrite: bool       # this rank wrote another width: partition again in `width`
    send: List[int]     # records to each rank
    recv: List[int]     # records from each rank (back to back, rank order)
    n_recv: int
    act_lane: bool = False  # a sender's directory cache addressed records: a u32 handle per record travels beside them


@dataclass
class Hop2Plan:
    forward: bool
    width: int
    send: List[int]
    recv: List[int]
    n_hosted: int
    n_forwarded: int


def plan_chunk(heads: np.ndarray, me: int, written: int, max_recv: int, owned_total: np.ndarray) -> ChunkPlan:
    """orl_node_plan_chunk over all-gathered head words (uint64 [nranks, HEAD_WORDS]); owned_total (uint64 [nranks]) is
    updated in place.  Raises OrleansRouteError with the code every rank gets (E_CAPACITY, E_DEVICE)."""
    import ctypes as C
    h = np.ascontiguousarray(heads, np.uint64)
    nr = h.shape[0]
    assert h.shape == (nr, HEAD_WORDS) and owned_total.dtype == np.uint64 and owned_total.flags["C_CONTIGUOUS"]
    out = L.orl_node_chunk_plan()
    rc = L.load().orl_node_plan_chunk(L.ptr(h), nr, int(me), int(written), int(max_recv), L.ptr(owned_total), C.byref(out))
    if rc != L.OK:
        raise L.OrleansRouteError(rc, "orl_node_plan_chunk")
    return ChunkPlan(out.width, bool(out.rewrite), list(out.send)[:nr], list(out.recv)[:nr], out.n_recv, bool(out.act_lane))


def plan_hop2(heads: np.ndarray, me: int, n_owned: int, width_mask: int, max_recv: int) -> Hop2Plan:
    """orl_node_plan_hop2 over the all-gathered hop-2 words (uint64 [nranks, HEAD_WORDS])."""
    import ctypes as C
    h = np.ascontiguousarray(heads, np.uint64)
    nr = h.shape[0]
    out = L.orl_node_hop2_plan()
    rc = L.load().orl_node_plan_hop2(L.ptr(h), nr, int(me), int(n_owned), int(width_mask), int(max_recv), C.byref(out))
    if rc != L.OK:
        raise L.OrleansRouteError(rc, "orl_node_plan_hop2")
    return Hop2Plan(bool(out.forward), out.width, list(out.send)[:nr], list(out.recv)[:nr], out.n_hosted, out.n_forwarded)


def narrow_records_to_headers(raw: np.ndarray, wire_types) -> np.ndarray:
    """8-B orl_wire8 records → orl_msg_hdr with the wire types they were written with (include/orleans_route.h)."""
    w = np.ascontiguousarray(raw).view(np.uint32).reshape(-1, 2)
    meta = w[:, 1]
    types = np.zeros(L.MAX_WIRE_TYPES, np.uint64)
    types[:len(wire_types)] = np.asarray(wire_types, np.uint64)
    out = np.zeros(len(w), L.MSG_DTYPE)
    out["tcd"] = types[(meta >> 16) & 0xF]
    out["n1"] = w[:, 0].astype(np.uint64)
    out["sending_silo"] = (meta & 0xFF).astype(np.uint8)
    out["category"] = ((meta >> 8) & 0x3).astype(np.uint8)
    out["flags"] = ((meta >> 10) & 0x3F).astype(np.uint8)
    out["target_silo"] = (meta >> 24).astype(np.uint8)
    return out


def wire_records_to_headers(raw: np.ndarray) -> np.ndarray:
    """16-B orl_wire_msg records → orl_msg_hdr (the layout include/orleans_route.h documents; aux = 0)."""
    w = np.ascontiguousarray(raw).view(np.uint32).reshape(-1, 4)
    meta = w[:, 3]
    out = np.zeros(len(w), L.MSG_DTYPE)
    low56 = np.uint64(0x00FFFFFFFFFFFFFF)
    out["tcd"] = (((meta >> 16) & 0xFF).astype(np.uint64) << np.uint64(56)) | \
        (w[:, 2].view(np.int32).astype(np.int64).view(np.uint64) & low56)
    out["n1"] = w[:, 0].astype(np.uint64) | (w[:, 1].astype(np.uint64) << np.uint64(32))
    out["sending_silo"] = (meta & 0xFF).astype(np.uint8)
    out["category"] = ((meta >> 8) & 0x3).astype(np.uint8)
    out["flags"] = ((meta >> 10) & 0x3F).astype(np.uint8)
    out["target_silo"] = (meta >> 24).astype(np.uint8)
    return out


@dataclass
class NodeResult:
    n_owned: int
    n_hosted: int
    n_forwarded: int
    n_sent_remote: int
    hop2: bool
    route: int    # device pointers, valid until the next batch of the node
    act: int
    order: int
    offsets: int
    segments: List[tuple]  # (device pointer, count, record width)
    emitted: int = 0       # fanout_batch_device: messages this rank's publishes emitted


class GrainNode:
    """orl_node (include/orleans_route.h): this GPU's silos in a multi-GPU node — owner partition, counts all-gather,
    grouped send/recv (RCCL over xGMI, or the in-process LOCAL rehearsal), routing at the directory owner, hop 2 to the
    activation's host, and stage 4 at the host, all behind the C ABI (no Python collective on the path).  Reference:
    OutboundMessageQueue.SendMessage (OutboundMessageQueue.cs:113-145), Dispatcher.TransportMessage (Dispatcher.cs:618-622)."""

    def __init__(self, eng, nranks: int, rank: int, rank_of_silo: Sequence[int], max_batch: int, max_recv: int,
                 transport: int = L.TRANSPORT_RCCL, group_id: Optional[bytes] = None, chunks: int = 4,
                 wide_only: bool = False, split_comm: Optional[bool] = None):
        import ctypes as C
        import os
        self._C = C
        self._lib = L.load()
        self.eng = eng
        cfg = L.orl_node_config()
        cfg.abi_version = L.ABI_VERSION
        cfg.nranks, cfg.rank, cfg.transport = int(nranks), int(rank), int(transport)
        gid = bytes(group_id or b"")[:L.NODE_ID_BYTES].ljust(L.NODE_ID_BYTES, b"\0")
        C.memmove(cfg.group_id, gid, L.NODE_ID_BYTES)
        ros = np.zeros(256, np.uint8)
        ros[:len(rank_of_silo)] = np.asarray(rank_of_silo, dtype=np.uint8)
        C.memmove(cfg.rank_of_silo, ros.tobytes(), 256)
        cfg.max_batch, cfg.max_recv, cfg.chunks = int(max_batch), int(max_recv), int(chunks)
        if split_comm is None:  # opt-in: every rank must agree, which orl_node_create checks
            split_comm = os.environ.get("ORL_NODE_SPLIT_COMM", "0") == "1"
        cfg.flags = (L.NODE_WIDE_ONLY if wide_only else 0) | (L.NODE_SPLIT_COMM if split_comm else 0)
        h = C.c_void_p()
        rc = self._lib.orl_node_create(eng.handle, C.byref(cfg), C.byref(h))
        if rc != L.OK:
            raise L.OrleansRouteError(rc, "orl_node_create failed (rank %d of %d, transport %d)" % (rank, nranks, transport))
        self._node = h
        self.nranks, self.rank = int(nranks), int(rank)

    @staticmethod
    def unique_id() -> bytes:
        """A fresh RCCL group id (rank 0 creates it and shares it, e.g. by a torch.distributed broadcast)."""
        import ctypes as C
        buf = (C.c_uint8 * L.NODE_ID_BYTES)()
        rc = L.load().orl_node_unique_id(buf)
        if rc != L.OK:
            raise L.OrleansRouteError(rc, "orl_node_unique_id failed")
        return bytes(buf)

    def set_timeout(self, ms: int) -> None:
        """Deadline of every host wait of the exchange (orl_node_set_timeout)."""
        rc = self._lib.orl_node_set_timeout(self._node, int(ms))
        if rc != L.OK:
            raise L.OrleansRouteError(rc, "orl_node_set_timeout")

    def route_batch_device(self, d_msgs, n: int, stream=None, opts: int = 0) -> NodeResult:
        C = self._C
        r = L.orl_node_result()
        rc = self._lib.orl_node_route_batch_device(self._node, L.ptr(d_msgs), int(n), int(opts), C.byref(r), L.ptr(stream))
        return self._result(rc, r)

    def route_batch_keyext_device(self, d_msgs, n: int, d_ext, d_blob, blob_bytes: int, stream=None, opts: int = 0) -> NodeResult:
        """orl_node_route_batch_keyext_device: the batch with its KeyExt strings (d_ext: orl_ext_ref per message into d_blob)."""
        C = self._C
        r = L.orl_node_result()
        rc = self._lib.orl_node_route_batch_keyext_device(self._node, L.ptr(d_msgs), int(n), int(opts), L.ptr(d_ext), L.ptr(d_blob),
                                                          int(blob_bytes), C.byref(r), L.ptr(stream))
        return self._result(rc, r)

    def fanout_batch_device(self, d_csr_off, d_csr_tgt, d_follower_keys, follower_tcd: int, d_pubs, d_pub_silo, n_pub: int,
                            d_pub_offsets, total=None, stream=None, opts: int = 0) -> NodeResult:
        """This rank's publishes expanded (orl_fanout_expand_device) and routed across the node
        (orl_node_fanout_batch_device): ChirperAccount.PublishMessage sharded by publisher (config 4)."""
        C = self._C
        if total is not None:
            opts |= L.OPT_TOTAL_GIVEN
        t = C.c_uint64(int(total or 0))
        r = L.orl_node_result()
        rc = self._lib.orl_node_fanout_batch_device(self._node, L.ptr(d_csr_off), L.ptr(d_csr_tgt), L.ptr(d_follower_keys),
                                                    int(follower_tcd), L.ptr(d_pubs), L.ptr(d_pub_silo), int(n_pub), int(opts),
                                                    L.ptr(d_pub_offsets), C.byref(t), C.byref(r), L.ptr(stream))
        res = self._result(rc, r)
        res.emitted = t.value
        return res

    def _result(self, rc, r) -> NodeResult:
        C = self._C
        if rc != L.OK:
            raise L.OrleansRouteError(rc, (self._lib.orl_node_last_error(self._node) or b"").decode(errors="replace"))
        segs = []
        for i in range(r.n_segments):
            p, cnt, w = C.c_void_p(), C.c_uint64(), C.c_uint32()
            assert self._lib.orl_node_segment(self._node, i, C.byref(p), C.byref(cnt), C.byref(w)) == L.OK
            segs.append((p.value or 0, cnt.value, w.value))
        return NodeResult(r.n_owned, r.n_hosted, r.n_forwarded, r.n_sent_remote, bool(r.hop2), r.route or 0, r.act or 0,
                          r.order or 0, r.bucket_offsets or 0, segs)

    def fetch(self, res: NodeResult, stream=None):
        """Host copies of a result: (route, act, order, offsets, hosted message headers as MSG_DTYPE)."""
        e = self.eng
        u32 = lambda k: np.zeros(k, np.uint32)  # noqa: E731
        route = e.copy_to_host(u32(res.n_hosted), res.route, stream=stream) if res.n_hosted else u32(0)
        act = e.copy_to_host(u32(res.n_hosted), res.act, stream=stream) if res.n_hosted else u32(0)
        order = e.copy_to_host(u32(res.n_hosted), res.order, stream=stream) if res.n_hosted else u32(0)
        off = e.copy_to_host(u32(e.n_act + 2), res.offsets, stream=stream)
        parts = []
        for p, cnt, w in res.segments:
            raw = np.zeros(cnt * w, np.uint8)
            if cnt:
                e.copy_to_host(raw, p, stream=stream)
            parts.append(raw.view(L.MSG_DTYPE) if w == 32 else wire_records_to_headers(raw) if w == 16 else
                         narrow_records_to_headers(raw, getattr(e, "wire_types", ())))
        hdrs = np.concatenate(parts) if parts else np.zeros(0, L.MSG_DTYPE)
        return route, act, order, off, hdrs

    def stats(self) -> dict:
        """orl_node_get_stats: the last batch's communicator size, bytes sent per peer and host waits."""
        st = L.orl_node_stats()
        rc = self._lib.orl_node_get_stats(self._node, self._C.byref(st))
        if rc != L.OK:
            raise L.OrleansRouteError(rc, "orl_node_get_stats")
        return {"comm_count": st.comm_count, "chunks": st.chunks, "bytes_sent": list(st.bytes_sent)[:self.nranks],
                "host_wait_us": st.host_wait_us, "host_waits": st.host_waits, "exchange_mode": exchange_mode_name(st.exchange_mode)}

    def close(self) -> None:
        if getattr(self, "_node", None):
            self._lib.orl_node_destroy(self._node)
            self._node = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def exchange_mode_name(mode: int) -> str:
    """orl_node_stats.exchange_mode as the bench JSON records it."""
    if mode & L.NODE_MODE_SPLIT_COMM:
        return "split communicator: counts all-gathers on their own RCCL communicator and stream"
    if mode & L.NODE_MODE_HEAD_STREAM:
        return "counts all-gathers on their own stream (LOCAL transport)"
    return "one communicator: counts all-gathers queued on the exchange stream behind the previous chunk's send/recv"


def rank_of_silo(n_silos: int, world: int) -> np.ndarray:
    """Silo s lives on GPU s * world // n_silos (contiguous blocks of logical silos per GPU)."""
    return np.array([s * world // n_silos for s in range(n_silos)], np.uint8)


def local_silos(n_silos: int, world: int, rank: int) -> np.ndarray:
    return np.nonzero(rank_of_silo(n_silos, world) == rank)[0]
