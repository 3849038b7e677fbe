"""Multi-GPU silo node: one process per GPU, the directory sharded by ring range.

Per batch (messages originate on the rank that hosts their sending silo):
  1. stages 1-2 + stable partition of the local batch by the rank holding each message's directory owner
     (``orl_partition_by_owner_device``);
  2. all-to-all of the per-rank counts, then all-to-all of the 32-B headers (torch.distributed: RCCL over
     xGMI on GPUs, gloo on CPU) — the reference's per-target-silo sender queues + TCP
     (OutboundMessageQueue.cs:113-145) collapsed into one collective;
  3. on the owner rank: stages 1-4 over the received messages (``orl_route_batch_device``).
Received messages are concatenated in source-rank order and each source's block keeps its arrival
order, so the per-activation FIFO order is the stable order by (source rank, source index): per-sender
order holds because a sender's messages all originate on one rank.

The exchange logic is independent of what computes the two local steps: ``HipExecutor`` drives the HIP
library; tests substitute a CPU executor built on the oracle to run the same protocol over gloo.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Protocol, Sequence

import numpy as np

from . import _lib as L

HDR_WORDS = 8  # orl_msg_hdr as 8 int32 words (exchange unit)


class Executor(Protocol):
    def partition(self, msgs, n: int, rank_of_silo: Sequence[int], nranks: int, my_rank: int):
        """-> (partitioned headers [n, 8] int32, source index [n] int32, counts [nranks] int64)"""

    def route(self, msgs, n: int):
        """-> (route [n], act [n], order [n], offsets [n_act+2]) for the received batch"""


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
    """Drives liborleans_route.so on this rank's GPU with preallocated device buffers."""

    def __init__(self, eng, capacity: int, torch_mod, device: str = "cuda", opts: int = 0):
        t = torch_mod
        self.t = t
        self.eng = eng
        self.opts = opts
        self.cap = capacity
        self.part = t.empty((capacity, HDR_WORDS), dtype=t.int32, device=device)
        self.src = t.empty(capacity, dtype=t.int32, device=device)
        self.counts = t.empty(8, dtype=t.int64, device=device)
        self.route_buf = t.empty(capacity, dtype=t.int32, device=device)
        self.act = t.empty(capacity, dtype=t.int32, device=device)
        self.order = t.empty(capacity, dtype=t.int32, device=device)
        self.offsets = t.empty(eng.n_act + 2, dtype=t.int32, device=device)

    def _stream(self):
        return self.t.cuda.current_stream().cuda_stream

    def partition(self, msgs, n, rank_of_silo, nranks, my_rank):
        assert n <= self.cap
        self.eng.partition_by_owner_device(msgs, n, rank_of_silo, nranks, my_rank, self.part, self.src,
                                           self.counts, stream=self._stream(), opts=self.opts)
        return self.part[:n], self.src[:n], self.counts[:nranks]

    def route(self, msgs, n):
        assert n <= self.cap
        self.eng.address_messages_device(msgs, n, self.route_buf, self.act, self.order, self.offsets,
                                         stream=self._stream(), opts=self.opts)
        return self.route_buf[:n], self.act[:n], self.order[:n], self.offsets


class ShardedRouter:
    """The exchange protocol of one rank."""

    def __init__(self, executor: Executor, rank: int, world: int, rank_of_silo: Sequence[int], capacity: int,
                 torch_mod, device: str = "cuda", group=None):
        self.ex = executor
        self.rank = rank
        self.world = world
        self.ros = list(rank_of_silo)
        self.t = torch_mod
        self.group = group
        self.recv = torch_mod.empty((capacity, HDR_WORDS), dtype=torch_mod.int32, device=device)
        self.recv_counts = torch_mod.empty(world, dtype=torch_mod.int64, device=device)
        self.cap = capacity

    def step(self, msgs, n: int) -> StepResult:
        dist = self.t.distributed
        part, _src, counts = self.ex.partition(msgs, n, self.ros, self.world, self.rank)
        if self.world == 1:
            r = self.ex.route(part, n)
            return StepResult([n], [n], *r, n_recv=n)
        dist.all_to_all_single(self.recv_counts, counts.contiguous(), group=self.group)
        send_splits = [int(x) for x in counts.tolist()]
        recv_splits = [int(x) for x in self.recv_counts.tolist()]
        n_recv = sum(recv_splits)
        if n_recv > self.cap:
            raise RuntimeError(f"rank {self.rank}: received {n_recv} messages > capacity {self.cap}")
        dist.all_to_all_single(self.recv[:n_recv], part, recv_splits, send_splits, group=self.group)
        r = self.ex.route(self.recv[:n_recv], n_recv)
        return StepResult(recv_splits, send_splits, *r, n_recv=n_recv)


def rank_of_silo(n_silos: int, world: int) -> np.ndarray:
    """Silo s lives on GPU s * world // n_silos (contiguous blocks of logical silos per GPU)."""
    return np.array([s * world // n_silos for s in range(n_silos)], np.uint8)


def local_silos(n_silos: int, world: int, rank: int) -> np.ndarray:
    return np.nonzero(rank_of_silo(n_silos, world) == rank)[0]
