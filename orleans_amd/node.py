"""Multi-GPU silo node: one process per GPU, the directory sharded by ring range.

Per batch (messages originate on the rank that hosts their sending silo):
  1. stages 1-2 + stable partition of the local batch by the rank holding each message's directory owner,
     in one pass into padded per-rank send regions (``orl_partition_by_owner_padded_device``);
  2. all-to-all of the per-rank counts, then grouped send/recv of the 32-B headers (torch.distributed
     batch_isend_irecv: RCCL over xGMI on GPUs, gloo on CPU) — the reference's per-target-silo sender
     queues + TCP (OutboundMessageQueue.cs:113-145) collapsed into one grouped exchange;
  3. on the owner rank: stages 1-4 over the received messages (``orl_route_batch_device``).
Received messages are concatenated in source-rank order and each source's block keeps its arrival
order, so the per-activation FIFO order is the stable order by (source rank, source index): per-sender
order holds because a sender's messages all originate on one rank.

PipelinedRouter keeps two batches in flight so the exchange of one overlaps the routing of the previous.
The exchange logic is independent of what computes the two local steps: ``HipExecutor`` drives the HIP
library; tests substitute a CPU executor built on the oracle to run the same protocol over gloo.
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass
from typing import List, Optional, Protocol, Sequence

import numpy as np

from . import _lib as L

HDR_WORDS = 8   # orl_msg_hdr as 8 int32 words
WIRE_WORDS = 4  # orl_wire_msg (compact exchange record) as 4 int32 words


HEAD_LEN = 9     # partition head: per-rank counts at [0, nranks), wire status at [8]


class Executor(Protocol):
    def partition(self, msgs, n: int, rank_of_silo: Sequence[int], nranks: int, my_rank: int, slot: int = 0,
                  stream=None, compact: bool = True):
        """-> (per-rank send regions: list of [>= count_r, W] int32 tensors (W = 8: orl_msg_hdr, 4: orl_wire_msg),
               head: int64 [HEAD_LEN] = per-rank counts, then at [8] 1 if the batch has no compact form)"""

    def route(self, msgs, n: int, slot: int = 0, stream=None):
        """-> (route [n], act [n], order [n], offsets [n_act+2]) for the received records ([n, W] int32)"""


@dataclass
class StepResult:
    recv_splits: List[int]   # messages received from each source rank
    send_splits: List[int]   # messages sent to each destination rank
    route: object
    act: object
    order: object
    offsets: object
    n_recv: int


class HipExecutor:
    """Drives liborleans_route.so on this rank's GPU with preallocated device buffers.

    `part_eng` (default: `eng`) runs the owner partition; giving it its own context (ring only) lets a partition
    and a route run concurrently on two streams without sharing scratch.  `slots` output sets let the
    pipelined router keep two batches in flight.  Send regions: `nranks` x `part_capacity` records per slot
    (the largest local batch; HBM is plentiful, so the one-pass partition needs no totals first).  `compact`
    sends 16-B orl_wire_msg records (half the exchange bytes) whenever the batch has that form."""

    def __init__(self, eng, capacity: int, torch_mod, device: str = "cuda", opts: int = 0, part_eng=None,
                 slots: int = 1, nranks: int = 1, part_capacity: Optional[int] = None, compact: bool = True):
        t = torch_mod
        self.t = t
        self.eng = eng
        self.part_eng = part_eng or eng
        self.opts = opts
        self.cap = capacity
        self.pcap = part_capacity or capacity
        self.nranks = nranks
        self.compact = compact
        mk = lambda *shape, dt=t.int32: t.empty(shape, dtype=dt, device=device)  # noqa: E731
        self.part = [mk(nranks * self.pcap * HDR_WORDS) for _ in range(slots)]  # flat: either record width
        self.head = [mk(HEAD_LEN, dt=t.int64) for _ in range(slots)]
        self.route_buf = [mk(capacity) for _ in range(slots)]
        self.act = [mk(capacity) for _ in range(slots)]
        self.order = [mk(capacity) for _ in range(slots)]
        self.offsets = [mk(eng.n_act + 2) for _ in range(slots)]

    def _stream(self, stream):
        return (stream or self.t.cuda.current_stream()).cuda_stream

    def partition(self, msgs, n, rank_of_silo, nranks, my_rank, slot: int = 0, stream=None, compact: bool = True):
        assert n <= self.pcap and nranks <= self.nranks
        head = self.head[slot]
        st = self._stream(stream)
        wide = not (compact and self.compact)
        width = HDR_WORDS if wide else WIRE_WORDS
        out = self.part[slot][:nranks * self.pcap * width].view(-1, width)
        if wide:
            self.part_eng.partition_by_owner_padded_device(msgs, n, rank_of_silo, nranks, my_rank, self.pcap, out,
                                                           head, stream=st, opts=self.opts)
            head[8:].zero_()
        else:
            head[8:].zero_()  # the kernel sets the low word of [8]
            self.part_eng.partition_compact_device(msgs, n, rank_of_silo, nranks, my_rank, self.pcap, out, head,
                                                   head[8:], stream=st, opts=self.opts)
        regions = [out[r * self.pcap:(r + 1) * self.pcap] for r in range(nranks)]
        return regions, head

    def route(self, msgs, n, slot: int = 0, stream=None):
        assert n <= self.cap
        fn = self.eng.address_compact_device if msgs.shape[1] == WIRE_WORDS else self.eng.address_messages_device
        fn(msgs, n, self.route_buf[slot], self.act[slot], self.order[slot], self.offsets[slot],
           stream=self._stream(stream), opts=self.opts)
        return self.route_buf[slot][:n], self.act[slot][:n], self.order[slot][:n], self.offsets[slot]


class PipelinedRouter:
    """The exchange protocol of one rank, with two batches in flight (overlap the exchange
    with stages 1-4).

    submit(batch k) enqueues, in this order:
      1. route(k-1) on stream R, after the exchange of batch k-1 (its Works' wait() on R);
      2. owner partition(k) on stream P, after route(k-2) released slot k % 2;
      3. an all-gather of every rank's per-rank counts and wire status (the host reads them: the exchange
         sizes, and whether the batch travels as 16-B compact records or, if any rank cannot, as 32-B headers);
      4. the grouped send/recv of batch k's records (async; RCCL's stream, after P).
    So on a GPU the RCCL exchange of batch k overlaps the routing of batch k-1, and the partition of batch
    k+1 overlaps the exchange of batch k.  submit returns batch k-1's StepResult (None for the first batch);
    flush() routes the last one; step() = submit + flush (one batch, nothing in flight).  Batch k's outputs
    live in slot k % 2 and stay valid until submit(k + 2); on a GPU they are complete once stream R is
    (flush() makes the current stream wait for it).  The executor needs 2 slots and, on a GPU, separate
    contexts for partition and route (HipExecutor(part_eng=...)).  On the CPU (gloo) it all runs in order."""

    def __init__(self, executor, rank: int, world: int, rank_of_silo: Sequence[int], capacity: int, torch_mod,
                 device: str = "cuda", group=None):
        t = torch_mod
        self.ex = executor
        self.rank = rank
        self.world = world
        self.ros = list(rank_of_silo)
        self.t = t
        self.group = group
        self.cap = capacity
        self.gpu = device != "cpu"
        self.recv_flat = [t.empty(capacity * HDR_WORDS, dtype=t.int32, device=device) for _ in range(2)]
        self.recv = [None, None]  # [n_recv, W] view of the received records of each slot
        self.heads = [t.empty((world, HEAD_LEN), dtype=t.int64, device=device) for _ in range(2)]
        if self.gpu:
            self.sp, self.sr = t.cuda.Stream(), t.cuda.Stream()
        self.route_done = [None, None]
        self.pending = None  # (slot, works, exchanged event, n_recv, send_splits, recv_splits)
        self.k = 0

    def _on(self, stream):
        return self.t.cuda.stream(stream) if self.gpu else contextlib.nullcontext()

    def _route_pending(self) -> Optional[StepResult]:
        if self.pending is None:
            return None
        slot, works, exchanged, n_recv, send_splits, recv_splits = self.pending
        self.pending = None
        with self._on(self.sr if self.gpu else None):
            for w in works:
                w.wait()
            if exchanged is not None:
                self.sr.wait_event(exchanged)
            r = self.ex.route(self.recv[slot], n_recv, slot=slot, stream=self.sr if self.gpu else None)
            if self.gpu:
                ev = self.t.cuda.Event()
                ev.record(self.sr)
                self.route_done[slot] = ev
        return StepResult(recv_splits, send_splits, *r, n_recv=n_recv)

    def _exchange(self, slot, regions, send_splits, recv_splits):
        """Grouped send/recv of every rank's region (self: a device copy).  Returns the Works to wait on."""
        dist = self.t.distributed
        recv_views, o = [], 0
        for c in recv_splits:
            recv_views.append(self.recv[slot][o:o + c])
            o += c
        ops = []
        for r in range(self.world):
            if r == self.rank:
                if send_splits[r]:
                    recv_views[r].copy_(regions[r][:send_splits[r]])
                continue
            if send_splits[r]:
                ops.append(dist.P2POp(dist.isend, regions[r][:send_splits[r]], r, self.group))
            if recv_splits[r]:
                ops.append(dist.P2POp(dist.irecv, recv_views[r], r, self.group))
        return dist.batch_isend_irecv(ops) if ops else []

    def submit(self, msgs, n: int) -> Optional[StepResult]:
        dist = self.t.distributed
        slot = self.k % 2
        self.k += 1
        prev = self._route_pending()
        exchanged = None
        with self._on(self.sp if self.gpu else None):
            if self.gpu:
                self.sp.wait_stream(self.t.cuda.current_stream())  # the caller's batch is ready
                if self.route_done[slot] is not None:
                    self.sp.wait_event(self.route_done[slot])
            st = self.sp if self.gpu else None
            regions, head = self.ex.partition(msgs, n, self.ros, self.world, self.rank, slot=slot, stream=st)
            # every rank's counts + wire status in one collective: the exchange sizes, and whether all ranks
            # can send compact records this batch (if one cannot, everyone re-partitions in the 32-B form)
            if self.world == 1:
                heads = [[int(x) for x in head.tolist()]]
            else:
                dist.all_gather_into_tensor(self.heads[slot], head.contiguous().view(1, -1), group=self.group)
                heads = self.heads[slot].tolist()
            if any(h[8] for h in heads):
                regions, head = self.ex.partition(msgs, n, self.ros, self.world, self.rank, slot=slot, stream=st,
                                                  compact=False)
            send_splits = [int(x) for x in heads[self.rank][:self.world]]
            recv_splits = [int(h[self.rank]) for h in heads]
            n_recv = sum(recv_splits)
            if n_recv > self.cap:
                raise RuntimeError(f"rank {self.rank}: received {n_recv} messages > capacity {self.cap}")
            width = regions[0].shape[1]
            self.recv[slot] = self.recv_flat[slot][:n_recv * width].view(n_recv, width)
            works = self._exchange(slot, regions, send_splits, recv_splits)
            if self.gpu:
                exchanged = self.t.cuda.Event()
                exchanged.record(self.sp)
        self.pending = (slot, works, exchanged, n_recv, send_splits, recv_splits)
        return prev

    def flush(self) -> Optional[StepResult]:
        r = self._route_pending()
        if self.gpu:
            self.t.cuda.current_stream().wait_stream(self.sr)
        return r

    def step(self, msgs, n: int) -> StepResult:
        """One batch with nothing in flight (submit + flush)."""
        assert self.pending is None, "step() with a batch in flight: flush() first"
        self.submit(msgs, n)
        return self.flush()


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
                 wide_only: bool = False):
        import ctypes as C
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
        cfg.flags = L.NODE_WIDE_ONLY if wide_only else 0
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

    def route_batch_device(self, d_msgs, n: int, stream=None, opts: int = 0) -> NodeResult:
        C = self._C
        r = L.orl_node_result()
        rc = self._lib.orl_node_route_batch_device(self._node, L.ptr(d_msgs), int(n), int(opts), C.byref(r), L.ptr(stream))
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

    def close(self) -> None:
        if getattr(self, "_node", None):
            self._lib.orl_node_destroy(self._node)
            self._node = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rank_of_silo(n_silos: int, world: int) -> np.ndarray:
    """Silo s lives on GPU s * world // n_silos (contiguous blocks of logical silos per GPU)."""
    return np.array([s * world // n_silos for s in range(n_silos)], np.uint8)


def local_silos(n_silos: int, world: int, rank: int) -> np.ndarray:
    return np.nonzero(rank_of_silo(n_silos, world) == rank)[0]
