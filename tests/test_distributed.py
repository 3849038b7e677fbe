"""The node exchange protocol with several processes over gloo on the CPU (world sizes 2, 3, 4, and 8 as the SCALE run uses).

Every rank runs the steps orl_node_route_batch_device takes (orleans_amd/csrc/orl_node.cpp), in the same order, with the
product's own host decisions — orl_node_plan_chunk after each chunk's counts all-gather (record width, re-partition,
send / receive sizes, the collective capacity error) and orl_node_plan_hop2 after the hop-2 counts all-gather (whether
anything is forwarded, the forwarded record width, the hosted count) — called from liborleans_route.so, which loads and
runs these on a machine without a GPU.  The device steps (partition, record encoding, routing, bucketing) are the oracle
restatements here; the exchanges are real gloo all-gathers and grouped isend/irecv between processes.  Every rank's hosted
route words, activation handles, order, offsets and headers must equal the single-process oracle replay
(tests/node_replay.py), which tests/test_gpu_node.py also checks the GPU node against.
Reference: OutboundMessageQueue.SendMessage (OutboundMessageQueue.cs:113-145), Dispatcher.TransportMessage
(Dispatcher.cs:618-622).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import node_replay as R
from oracle import cpu_ref
from orleans_amd import _lib as L
from orleans_amd.node import HEAD_WORDS, narrow_records_to_headers, plan_chunk, plan_hop2, wire_records_to_headers

N_GRAINS = 6000
DIGEST_MASK = (1 << 56) - 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _digest(types):
    """The wire-type digest the product computes (ORL_Q_WIRE_DIGEST) of a host-only context."""
    from orleans_amd.engine import GrainDirectoryEngine
    if not types:
        return 0
    e = GrainDirectoryEngine(n_act=8, dir_capacity=16, max_batch=1024, device=-1)
    try:
        e.set_silos(8)
        e.set_wire_types(types)
        return e.query(L.Q_WIRE_DIGEST)
    finally:
        e.close()


def _encode(recs, width, types):
    """Records of `width` bytes for headers `recs` (the oracle restatements of the device encoders) -> uint8 [n, width]."""
    if width == 32:
        return np.ascontiguousarray(recs).view(np.uint8).reshape(-1, 32)
    if width == 16:
        w, ok = cpu_ref.wire_encode(recs)
        assert ok.all()
        return w.view(np.uint8).reshape(-1, 16)
    w, ok = cpu_ref.narrow_encode(recs, types)
    assert ok.all()
    return w.view(np.uint8).reshape(-1, 8)


def _decode(raw, width, types):
    if width == 32:
        return raw.reshape(-1).view(L.MSG_DTYPE).copy()
    if width == 16:
        return wire_records_to_headers(raw.reshape(-1))
    return narrow_records_to_headers(raw.reshape(-1), types)


def _allgather(words):
    world = dist.get_world_size()
    t = torch.from_numpy(words.view(np.int64).copy())
    out = [torch.zeros(HEAD_WORDS, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(out, t)
    return torch.stack(out).numpy().view(np.uint64).reshape(world, HEAD_WORDS)


def _exchange(parts, send, recv):
    """parts[r] = uint8 array to rank r (send[r] records of equal width); returns what each rank sent here, rank order."""
    me, world = dist.get_rank(), dist.get_world_size()
    outs = [None] * world
    ops = []
    for r in range(world):
        if r == me:
            outs[r] = parts[r].copy()
            continue
        if send[r]:
            ops.append(dist.P2POp(dist.isend, torch.from_numpy(np.ascontiguousarray(parts[r])), r))
        outs[r] = np.zeros((int(recv[r]),) + parts[r].shape[1:], parts[r].dtype)
        if recv[r]:
            ops.append(dist.P2POp(dist.irecv, torch.from_numpy(outs[r]), r))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return outs


def node_step(o, p, me, batch, chunks, types, max_recv, wide_only=False):
    """One batch of orl_node_route_batch_device, step for step, over gloo.  Returns (route, act, order, offsets, hosted
    headers, chunk widths, forward) or raises OrleansRouteError with the code the plan returned."""
    world = dist.get_world_size()
    ros = p.ros
    digest = _digest(types)
    written = 32 if wide_only else (8 if digest else 16)
    owned_total = np.zeros(world, np.uint64)
    owned, widths, width_mask = [], [], 0
    for c in range(chunks):
        lo, hi = R.chunk_bounds(len(batch), chunks, c)
        ch = batch[lo:hi]
        src, counts = o.partition(ch, ros, world, me)  # k_part_lb: stable partition by the owner's rank
        recs = ch[src]
        status = 0
        if written != 32:  # the partition kernel's status word over every message of the chunk
            status |= 0 if cpu_ref.wire_encode(ch)[1].all() else 1
            if written == 8:
                status |= 0 if cpu_ref.narrow_encode(ch, types)[1].all() else 2
        head = np.zeros(HEAD_WORDS, np.uint64)
        head[:world] = counts
        head[8] = status
        head[9] = (written << 56) | (digest & DIGEST_MASK)
        heads = _allgather(head)
        plan = plan_chunk(heads, me, written, max_recv, owned_total)
        enc = _encode(recs, plan.width, types)
        bounds = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        parts = [enc[bounds[r]:bounds[r + 1]] for r in range(world)]
        assert [len(x) for x in parts] == plan.send
        got = _exchange(parts, plan.send, plan.recv)
        owned.append(_decode(np.concatenate(got), plan.width, types))
        widths.append(plan.width)
        width_mask |= {8: 1, 16: 2, 32: 4}[plan.width]
    owned = np.concatenate(owned)
    route, act = o.route(owned)  # stages 1-3 at the owner
    hr = R.host_rank(route, ros, me)
    h2 = np.zeros(HEAD_WORDS, np.uint64)
    h2[:world] = np.bincount(hr, minlength=world)
    p2 = plan_hop2(_allgather(h2), me, len(owned), width_mask, max_recv)
    if not p2.forward:
        order, off = o.bucket(act, p.n_act)
        return route, act, order, off, owned, widths, False
    sel = np.argsort(hr, kind="stable")  # k_part_routed: stable partition of {record, route, act} by host rank
    cnt = np.bincount(hr, minlength=world)
    assert list(cnt) == p2.send
    bounds = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    lanes = [_encode(owned[sel], p2.width, types), route[sel].view(np.uint8).reshape(-1, 4),
             act[sel].view(np.uint8).reshape(-1, 4)]
    got = [_exchange([ln[bounds[r]:bounds[r + 1]] for r in range(world)], p2.send, p2.recv) for ln in lanes]
    hosted = _decode(np.concatenate(got[0]), p2.width, types)
    route = np.concatenate(got[1]).reshape(-1).view(np.uint32)
    act = np.concatenate(got[2]).reshape(-1).view(np.uint32)
    assert len(hosted) == p2.n_hosted
    order, off = o.bucket(act, p.n_act)
    return route, act, order, off, hosted, widths, True


def _worker(rank, world, port, q, case):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = R.population(world, N_GRAINS, seed=11, host_mix=case["host_mix"])
        o = R.rank_oracle(p, rank)
        types = R.wire_types(p, case["wire"])[rank]
        outs = []
        for b in range(case["batches"]):
            m = R.messages(p, rank, case["n"] - 97 * b + 13 * rank, seed=1000 * b + rank,
                           wide_at=case["wide_at"] if (b == 1 and rank == world - 1) else None)
            try:
                outs.append(("ok", node_step(o, p, rank, m, case["chunks"], types, case["max_recv"])))
            except L.OrleansRouteError as e:
                outs.append(("err", e.code))
        q.put((rank, outs))
    finally:
        dist.destroy_process_group()


def _run(world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, case)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = {}
    for _ in range(world):
        item = q.get(timeout=240)
        out[item[0]] = item[1]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    return out


def _expected(world, case, b):
    p = R.population(world, N_GRAINS, seed=11, host_mix=case["host_mix"])
    oracles = [R.rank_oracle(p, r) for r in range(world)]
    batches = [R.messages(p, r, case["n"] - 97 * b + 13 * r, seed=1000 * b + r,
                          wide_at=case["wide_at"] if (b == 1 and r == world - 1) else None) for r in range(world)]
    return R.expected(oracles, p.ros, batches, case["chunks"], p.n_act)


CASES = {
    # 8-B records, 30 % of activations off their owner (hop 2); batch 1 has a Guid-keyed target in the last rank's
    # chunk 1: that chunk goes as 32-B headers on every rank, and the forwarded set (a width mix) as headers too
    "narrow_hop2": dict(wire="both", host_mix=0.3, n=9000, chunks=3, batches=2, wide_at=4000, max_recv=1 << 20,
                        widths=[[8, 8, 8], [8, 32, 8]]),
    # no wire types: 16-B records; activations on their owners (no hop 2)
    "wire16": dict(wire=None, host_mix=0.0, n=8000, chunks=2, batches=2, wide_at=1000, max_recv=1 << 20,
                   widths=[[16, 16], [32, 16]]),
    # system-target messages lack the 8-B form (not in the list): every chunk falls back to 16 B
    "grain_only": dict(wire="grain_only", host_mix=0.3, n=7000, chunks=2, batches=1, wide_at=None, max_recv=1 << 20,
                       widths=[[16, 16]]),
    # the ranks' wire-type lists differ (digests): 16 B
    "mismatch": dict(wire="mismatch", host_mix=0.0, n=7000, chunks=2, batches=1, wide_at=None, max_recv=1 << 20,
                     widths=[[16, 16]]),
}


@pytest.mark.parametrize("world,name", [(2, "narrow_hop2"), (4, "narrow_hop2"), (8, "narrow_hop2"), (2, "wire16"), (3, "grain_only"),
                                        (2, "mismatch")])
def test_node_protocol_gloo(world, name):
    case = CASES[name]
    out = _run(world, case)
    for b in range(case["batches"]):
        exp, forward = _expected(world, case, b)
        for r in range(world):
            status, res = out[r][b]
            assert status == "ok", (r, b, res)
            route, act, order, off, hosted, widths, fwd = res
            assert widths == case["widths"][b], (r, b, widths)
            assert fwd == forward
            er, ea, eo, ef, eh = exp[r]
            np.testing.assert_array_equal(hosted, eh, err_msg=f"rank {r} batch {b} headers")
            np.testing.assert_array_equal(route, er, err_msg=f"rank {r} batch {b} route")
            np.testing.assert_array_equal(act, ea, err_msg=f"rank {r} batch {b} act")
            np.testing.assert_array_equal(order, eo, err_msg=f"rank {r} batch {b} order")
            np.testing.assert_array_equal(off, ef, err_msg=f"rank {r} batch {b} offsets")


def test_node_protocol_gloo_capacity_is_collective():
    """A receive capacity one rank exceeds: every rank's plan returns ORL_E_CAPACITY at the same chunk (none waits)."""
    case = dict(wire="both", host_mix=0.0, n=9000, chunks=3, batches=1, wide_at=None, max_recv=5000, widths=None)
    out = _run(2, case)
    assert [out[r][0] for r in range(2)] == [("err", L.E_CAPACITY)] * 2


def test_plan_chunk_rules():
    """orl_node_plan_chunk's width rules and collective errors on hand-made head words (no processes)."""
    def heads(nr, forms, status=None, digests=None):
        h = np.zeros((nr, HEAD_WORDS), np.uint64)
        for r in range(nr):
            h[r, :nr] = np.arange(nr) + 10 * r
            h[r, 8] = (status or [0] * nr)[r]
            h[r, 9] = (forms[r] << 56) | (digests or [77] * nr)[r]
        return h
    z = lambda n: np.zeros(n, np.uint64)  # noqa: E731
    assert plan_chunk(heads(2, [8, 8]), 0, 8, 100, z(2)).width == 8
    assert plan_chunk(heads(2, [8, 8], status=[0, 2]), 0, 8, 100, z(2)).width == 16      # a message lacks the 8-B form
    assert plan_chunk(heads(2, [8, 8], status=[1, 0]), 1, 8, 100, z(2)).width == 32      # ... or the 16-B form
    assert plan_chunk(heads(2, [8, 8], digests=[1, 2]), 0, 8, 100, z(2)).width == 16     # different wire-type lists
    assert plan_chunk(heads(2, [8, 16]), 0, 8, 100, z(2)).rewrite                        # one rank has no wire types
    assert plan_chunk(heads(2, [8, 32]), 0, 8, 100, z(2)).width == 32                    # a wide-only rank
    p = plan_chunk(heads(3, [16, 16, 16]), 1, 16, 100, z(3))
    assert p.send == [10, 11, 12] and p.recv == [1, 11, 21] and p.n_recv == 33 and not p.rewrite
    tot = z(3)
    plan_chunk(heads(3, [16] * 3), 0, 16, 40, tot)
    assert list(tot) == [30, 33, 36]
    for me in range(3):  # the second chunk pushes rank 2 past 40 on every rank
        with pytest.raises(L.OrleansRouteError) as e:
            plan_chunk(heads(3, [16] * 3), me, 16, 40, tot.copy())
        assert e.value.code == L.E_CAPACITY
    with pytest.raises(L.OrleansRouteError) as e:
        plan_chunk(heads(2, [8, 8], status=[0, L.PART_LOOKBACK_FAILED]), 0, 8, 100, z(2))
    assert e.value.code == L.E_DEVICE
    h2 = np.zeros((2, HEAD_WORDS), np.uint64)
    h2[0, :2] = [5, 0]
    h2[1, :2] = [0, 3]
    q = plan_hop2(h2, 1, 3, 1, 100)
    assert not q.forward and q.n_hosted == 3 and q.width == 8
    h2[0, 1] = 2
    q = plan_hop2(h2, 1, 3, 1 | 2, 100)
    assert q.forward and q.width == 32 and q.n_hosted == 5 and q.recv == [2, 3] and q.send == [0, 3]
    assert plan_hop2(h2, 0, 7, 2, 100).n_forwarded == 2
    with pytest.raises(L.OrleansRouteError):
        plan_hop2(h2, 0, 7, 2, 4)
