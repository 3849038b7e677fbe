"""The multi-rank exchange protocol (orleans_amd/node.py) over gloo on the CPU, world size 2 and 4.

The two local steps run on the oracle here (a CPU executor), the exchange is the real torch.distributed
counts all-to-all + grouped send/recv; on GPUs the same PipelinedRouter drives the HIP library over RCCL.  Checked: every message is
routed by its directory owner's rank, the routing decision equals the single-process oracle's, and each
rank's per-activation buckets keep the (source rank, source index) order.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import cpu_ref
from orleans_amd import _lib as L
from orleans_amd import workloads as W
from orleans_amd.node import HEAD_LEN, PipelinedRouter, local_silos, rank_of_silo

N_GRAINS = 3000
N_MSGS = 5000


class OracleExecutor:
    """CPU stand-in for HipExecutor: same contract, computed by the oracle (test only).  With compact=True the
    regions are 16-B wire records (oracle restatement of the codec) whenever the whole batch has that form."""

    def __init__(self, oracle, n_act, compact=False):
        self.o = oracle
        self.n_act = n_act
        self.compact = compact

    def partition(self, msgs, n, ros, nranks, my_rank, slot=0, stream=None, compact=True):
        m = msgs[:n].numpy().reshape(-1).view(L.MSG_DTYPE)
        src, counts = self.o.partition(m, ros, nranks, my_rank)
        head = torch.zeros(HEAD_LEN, dtype=torch.int64)
        head[:nranks] = torch.from_numpy(counts.astype(np.int64))
        rec = m[src]
        width = 8
        if self.compact and compact:
            w, ok = cpu_ref.wire_encode(rec)
            head[8] = int(not ok.all())
            rec, width = w, 4
        part = torch.from_numpy(rec.view(np.int32).reshape(-1, width).copy())
        return list(torch.split(part, [int(c) for c in counts])), head

    def route(self, msgs, n, slot=0, stream=None):
        rec = msgs[:n].numpy().reshape(-1)
        m = cpu_ref.wire_decode(rec.view(cpu_ref.WIRE_DTYPE)) if msgs.shape[1] == 4 else rec.view(L.MSG_DTYPE)
        r, a = self.o.route(m)
        order, off = self.o.bucket(a, self.n_act)
        return r, a, order, off


def _received(router, slot, n_recv):
    rec = router.recv[slot][:n_recv].numpy().reshape(-1)
    if router.recv[slot].shape[1] == 4:
        return cpu_ref.wire_decode(rec.view(cpu_ref.WIRE_DTYPE))
    return rec.view(L.MSG_DTYPE).copy()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup_rank(rank, world):
    cl = W.default_cluster()
    ros = rank_of_silo(cl.n_silos, world)
    mine = local_silos(cl.n_silos, world, rank)
    local = np.zeros(cl.n_silos, np.uint8)
    local[mine] = 1
    o = cpu_ref.Oracle(cl.n_silos, local=list(local))
    for s in range(cl.n_silos):
        o.add_server(s, int(cl.hashes[s]))
    keys, uni, owner, reg = W.grain_population(cl, N_GRAINS, 0.9)
    sel = reg & local[owner].astype(bool)
    idx = np.nonzero(sel)[0]
    st, _, _ = o.register(keys[idx], idx.astype(np.uint32), owner[idx])
    assert (st == L.INS_INSERTED).all()
    return cl, ros, mine, o


def _result_tuple(msgs, res, recv):
    return (msgs, res.send_splits, res.recv_splits, recv, np.asarray(res.route), np.asarray(res.act),
            np.asarray(res.order), np.asarray(res.offsets))


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cl, ros, mine, o = _setup_rank(rank, world)
        msgs = W.uniform_messages(cl, N_GRAINS + 200, N_MSGS, seed=99, start=rank * N_MSGS, sender_silos=mine)
        router = PipelinedRouter(OracleExecutor(o, N_GRAINS), rank, world, ros, 4 * N_MSGS, torch, device="cpu")
        res = router.step(torch.from_numpy(msgs.view(np.int32).reshape(-1, 8).copy()), N_MSGS)
        recv = _received(router, 0, res.n_recv)
        q.put((rank, [_result_tuple(msgs, res, recv)]))
    finally:
        dist.destroy_process_group()


def _worker_pipelined(rank, world, port, q, n_batches=3, compact=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cl, ros, mine, o = _setup_rank(rank, world)
        router = PipelinedRouter(OracleExecutor(o, N_GRAINS, compact=compact), rank, world, ros, 4 * N_MSGS, torch,
                                 device="cpu")
        batches = [W.uniform_messages(cl, N_GRAINS + 200, N_MSGS - 97 * b, seed=99 + b, start=(rank * 7 + b) * N_MSGS,
                                      sender_silos=mine) for b in range(n_batches)]
        if rank == 1:  # batch 1 of rank 1 has a Guid-keyed (N0 != 0) message: every rank sends 32-B headers
            batches[1]["n0"][17] = 5
        widths = []
        outs = []
        for b, m in enumerate(batches + [None]):
            res = router.submit(torch.from_numpy(m.view(np.int32).reshape(-1, 8).copy()), len(m)) if m is not None \
                else router.flush()
            if b > 0:  # result of batch b-1; its received records are still in slot (b-1) % 2
                widths.append(router.recv[(b - 1) % 2].shape[1])
                outs.append(_result_tuple(batches[b - 1], res, _received(router, (b - 1) % 2, res.n_recv)))
            else:
                assert res is None
        assert widths == ([4, 8, 4] if compact else [8, 8, 8]), widths
        q.put((rank, outs))
    finally:
        dist.destroy_process_group()


def _run(world, target):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        item = q.get(timeout=120)
        out[item[0]] = item[1]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def _verify(world, out):
    """out[rank] = (msgs, send_splits, recv_splits, recv, route, act, order, offsets) of one batch."""
    cl = W.default_cluster()
    o = cpu_ref.Oracle(cl.n_silos)
    for s in range(cl.n_silos):
        o.add_server(s, int(cl.hashes[s]))
    keys, uni, owner, reg = W.grain_population(cl, N_GRAINS, 0.9)
    idx = np.nonzero(reg)[0]
    o.register(keys[idx], idx.astype(np.uint32), owner[idx])
    ros = rank_of_silo(cl.n_silos, world)
    total_recv = 0
    for r in range(world):
        msgs_r, send, recv_splits, recv, route, act, order, off = out[r]
        # what rank r received = rank-major concatenation of every source's messages owned by r, in order
        expect = []
        for src in range(world):
            m = out[src][0]
            rr, _ = o.route(m)
            own = (rr & 0xFF).astype(np.int64)
            dest = np.where(own < 0xFF, ros[np.minimum(own, cl.n_silos - 1)], src)
            expect.append(m[dest == r])
            assert recv_splits[src] == int((dest == r).sum())
        expect = np.concatenate(expect)
        np.testing.assert_array_equal(recv, expect)
        # routing decision on the owner rank == single-process decision
        r_ref, a_ref = o.route(recv)
        np.testing.assert_array_equal(route, r_ref)
        np.testing.assert_array_equal(act, a_ref)
        o_ref, f_ref = o.bucket(a_ref, N_GRAINS)
        np.testing.assert_array_equal(order, o_ref)
        np.testing.assert_array_equal(off, f_ref)
        assert (decode := (route >> 16) & 0xFF).max() <= L.ST_NEW_PLACEMENT, np.unique(decode)
        total_recv += len(recv)
    assert total_recv == sum(len(out[r][0]) for r in range(world))


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_exchange_gloo(world):
    out = _run(world, _worker)
    _verify(world, {r: out[r][0] for r in range(world)})


def test_pipelined_exchange_gloo():
    """Two batches in flight: every batch's exchange and routing equal the single-process oracle's."""
    world = 2
    out = _run(world, _worker_pipelined)
    for b in range(3):
        _verify(world, {r: out[r][b] for r in range(world)})
