"""GPU parity of the node exchange behind the C ABI (orl_node_*).

World sizes 1-4 run as nodes of ONE process on one GPU (ORL_TRANSPORT_LOCAL: the same partition / all-gather / grouped
send-recv / hop-2 / bucketing protocol, with device copies instead of RCCL), one host thread per rank.  Every rank's
hosted output (route words, activation handles, per-activation order, bucket offsets, hosted headers) is compared with
the oracle replaying the protocol: each rank's chunks partitioned by owner rank (oracle partition), the owned set in
(chunk, source rank) order routed by the owner's oracle directory, forwarded to the host rank in owner order, bucketed.
An RCCL communicator of one rank checks the RCCL transport plumbing (all-gather, grouped self send) on the box.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import cpu_ref
from orleans_amd import _lib as L
from orleans_amd import workloads as W
from orleans_amd.engine import GrainDirectoryEngine, decode_route
from orleans_amd.node import GrainNode

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


class World:
    """W ranks: directory partitions by owner rank, activations on a host silo (owner or another), dense handles per
    host rank (each rank's catalog numbers its own activations)."""

    def __init__(self, nranks, n_grains=40_000, seed=3, host_mix=0.3, ros=None):
        cl = W.default_cluster()
        self.cl = cl
        self.nr = nranks
        self.ros = cl.rank_of_silo(nranks) if ros is None else np.asarray(ros, np.uint8)
        keys, uni, owner, reg = W.grain_population(cl, n_grains, 0.9, seed)
        rng = np.random.default_rng(seed)
        host = np.where(rng.random(n_grains) < 1.0 - host_mix, owner, rng.integers(0, 8, n_grains)).astype(np.uint8)
        hrank = self.ros[host]
        act = np.zeros(n_grains, np.uint32)
        cnt = []
        for r in range(nranks):
            idx = np.nonzero((hrank == r) & reg)[0]
            act[idx] = np.arange(len(idx), dtype=np.uint32)
            cnt.append(len(idx))
        self.n_act = max(cnt) + 8
        self.n_grains = n_grains
        self.engs, self.oracles = [], []
        for r in range(nranks):
            local = (self.ros == r).astype(np.uint8)
            e = GrainDirectoryEngine(n_act=self.n_act, dir_capacity=n_grains, max_batch=1 << 20, device=0)
            e.set_silos(8, local=local)
            o = cpu_ref.Oracle(8, local=list(local))
            for s in range(8):
                e.add_server(s, int(cl.hashes[s]))
                o.add_server(s, int(cl.hashes[s]))
            sel = np.nonzero(reg & (self.ros[owner] == r))[0]
            st, _, _ = e.register_single_activation(keys[sel], act[sel], host[sel])
            assert (st == L.INS_INSERTED).all()
            o.register(keys[sel], act[sel], host[sel])
            self.engs.append(e)
            self.oracles.append(o)

    def set_wire_types(self, mode):
        """8-B exchange form: None (off), "both" (grain + system-target types on every rank), "grain_only" (system-target
        messages lack the form), "mismatch" (the last rank's list differs: the digests disagree)."""
        if mode is None:
            return
        grain_t = (L.CAT_GRAIN << 56) + (self.cl.type_code & 0x00FFFFFFFFFFFFFF)
        sys_t = (L.CAT_SYSTEM_TARGET << 56) | 12
        for r, e in enumerate(self.engs):
            types = [grain_t] if mode == "grain_only" else [grain_t, sys_t]
            if mode == "mismatch" and r == self.nr - 1:
                types = [sys_t, grain_t]
            e.set_wire_types(types)

    def messages(self, rank, n, seed, wide_at=None):
        silos = np.nonzero(self.ros == rank)[0].astype(np.uint8)
        m = W.uniform_messages(self.cl, self.n_grains + 3000, n, seed=seed, sender_silos=silos)
        rng = np.random.default_rng(seed)
        c = rng.random(n)
        m["flags"][c < 0.03] = L.HDR_ADDRESS_COMPLETE  # responses: complete addresses, routed to the target silo
        m["target_silo"][c < 0.03] = rng.integers(0, 8, int((c < 0.03).sum()))
        st = (c >= 0.03) & (c < 0.05)
        m["tcd"][st] = (np.uint64(L.CAT_SYSTEM_TARGET) << np.uint64(56)) | np.uint64(12)
        if wide_at is not None:  # a Guid-keyed target: this chunk has no compact form
            m["n0"][wide_at] = 0x1234
        return m

    def expected(self, batches, chunks):
        """The oracle's replay of one batch per rank: per-rank (route, act, order, offsets, hosted headers)."""
        nr, ros = self.nr, self.ros
        owned = [[] for _ in range(nr)]
        for c in range(chunks):
            for s in range(nr):
                ms = batches[s]
                cs = -(-len(ms) // chunks)
                lo = min(c * cs, len(ms))
                ch = ms[lo:min(lo + cs, len(ms))]
                src, cnt = self.oracles[0].partition(ch, ros, nr, s)
                o0 = 0
                for d in range(nr):
                    owned[d].append(ch[src[o0:o0 + int(cnt[d])]])
                    o0 += int(cnt[d])
        owned = [np.concatenate(x) if x else np.zeros(0, L.MSG_DTYPE) for x in owned]
        routed = [self.oracles[d].route(owned[d]) for d in range(nr)]
        hostr = []
        for d in range(nr):
            h = decode_route(routed[d][0]).host
            hostr.append(np.where(h == 0xFF, d, ros[np.minimum(h, 7).astype(np.int64)]))
        forward = any((hostr[d] != d).any() for d in range(nr))
        out = []
        for hr in range(nr):
            if forward:
                sel = [hostr[o] == hr for o in range(nr)]
                hdr = np.concatenate([owned[o][sel[o]] for o in range(nr)])
                route = np.concatenate([routed[o][0][sel[o]] for o in range(nr)])
                act = np.concatenate([routed[o][1][sel[o]] for o in range(nr)])
            else:
                hdr, (route, act) = owned[hr], routed[hr]
            order, off = self.oracles[hr].bucket(act, self.n_act)
            out.append((route, act, order, off, hdr))
        return out, forward

    def close(self):
        for e in self.engs:
            e.close()


def _run(t, world, nodes, batches, streams):
    d_in = [t.from_numpy(b.view(np.int32).reshape(-1, 8)).cuda() for b in batches]
    t.cuda.synchronize()

    def one(r):
        res = nodes[r].route_batch_device(d_in[r], len(batches[r]), stream=streams[r].cuda_stream)
        streams[r].synchronize()
        return res, nodes[r].fetch(res, stream=streams[r].cuda_stream)

    with ThreadPoolExecutor(len(nodes)) as ex:
        return list(ex.map(one, range(len(nodes))))


@pytest.mark.parametrize("nranks,chunks,host_mix,wire", [(1, 1, 0.0, None), (2, 3, 0.0, None), (2, 2, 0.3, None),
                                                         (3, 4, 0.3, None), (4, 1, 0.3, None), (4, 4, 0.0, None),
                                                         (1, 2, 0.0, "both"), (2, 2, 0.3, "both"), (3, 4, 0.3, "both"),
                                                         (4, 4, 0.0, "both"), (2, 3, 0.3, "grain_only"),
                                                         (3, 2, 0.0, "mismatch")])
def test_node_local_transport_vs_oracle(torch, nranks, chunks, host_mix, wire):
    """Every rank's hosted output == the oracle's replay of the protocol, with each record form: 16-B (no wire types),
    8-B (wire types set; a Guid-keyed chunk in batch 1 drops that chunk to 32-B headers, so hop 2 forwards a mix), and the
    16-B fallbacks when a message lacks the 8-B form or the ranks' wire types differ."""
    t = torch
    ros = None if nranks != 3 else [s % 3 for s in range(8)]
    world = World(nranks, host_mix=host_mix, ros=ros)
    world.set_wire_types(wire)
    gid = b"node-test-%d-%d-%d-%s" % (nranks, chunks, int(host_mix * 10), str(wire).encode())
    nodes = [GrainNode(world.engs[r], nranks, r, world.ros, max_batch=200_000, max_recv=400_000,
                       transport=L.TRANSPORT_LOCAL, group_id=gid, chunks=chunks) for r in range(nranks)]
    streams = [t.cuda.Stream() for _ in range(nranks)]
    for b in range(2):  # two batches: buffers and send slots are reused
        batches = [world.messages(r, 150_000 - 7000 * r - 1000 * b, seed=100 * b + r,
                                  wide_at=(60_000 if (b == 1 and r == nranks - 1) else None)) for r in range(nranks)]
        got = _run(t, world, nodes, batches, streams)
        exp, forward = world.expected(batches, chunks)
        for r in range(nranks):
            res, (route, act, order, off, hdrs) = got[r]
            er, ea, eo, ef, eh = exp[r]
            widths = {w for _, c, w in res.segments if c}
            if wire == "both" and b == 0:  # every chunk in the 8-B form (a forwarded set keeps it)
                assert widths <= {8}, widths
            elif wire in ("grain_only", "mismatch") or (wire is None and b == 0):
                assert 8 not in widths, widths
            assert res.hop2 == forward
            assert res.n_hosted == len(er)
            np.testing.assert_array_equal(hdrs, eh, err_msg=f"rank {r} batch {b} headers")
            np.testing.assert_array_equal(route, er, err_msg=f"rank {r} batch {b} route")
            np.testing.assert_array_equal(act, ea, err_msg=f"rank {r} batch {b} act")
            np.testing.assert_array_equal(order, eo, err_msg=f"rank {r} batch {b} order")
            np.testing.assert_array_equal(off, ef, err_msg=f"rank {r} batch {b} offsets")
        if host_mix > 0 and nranks > 1:
            assert forward and sum(g[0].n_forwarded for g in got) > 1000
    for nd in nodes:
        nd.close()
    world.close()


@pytest.mark.parametrize("nranks", [2, 3])
def test_node_fanout_batch_vs_oracle(torch, nranks):
    """Config 4 sharded by publisher: every rank expands its own publishes (orl_node_fanout_batch_device) and the
    emitted messages are routed across the node; each rank's hosted output == the oracle's replay of the protocol over
    the expanded batches (cpu_ref.fanout_expand per rank)."""
    t = torch
    world = World(nranks, n_grains=40_000, host_mix=0.2, ros=None if nranks != 3 else [s % 3 for s in range(8)])
    cl = world.cl
    off, tgt = W.powerlaw_csr(world.n_grains + 3000, dmax=2000)  # some followers are never registered
    tcd = (3 << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)
    keys, uni, owner, reg = W.grain_population(cl, world.n_grains + 3000, 0.9, 3)
    pubs_all = (W.stream(21, 0, 6000) % np.uint64(world.n_grains)).astype(np.uint32)
    nodes = [GrainNode(world.engs[r], nranks, r, world.ros, max_batch=200_000, max_recv=400_000,
                       transport=L.TRANSPORT_LOCAL, group_id=b"node-fan-%d" % nranks, chunks=2) for r in range(nranks)]
    d_off = t.from_numpy(off.view(np.int64)).cuda()
    d_tgt = t.from_numpy(tgt.view(np.int32)).cuda()
    batches, args = [], []
    for r in range(nranks):  # a rank publishes for the accounts its silos own (sharded by publisher owner)
        pubs = pubs_all[world.ros[owner[pubs_all.astype(np.int64)]] == r]
        psilo = owner[pubs.astype(np.int64)].astype(np.uint8)
        exp, _ = cpu_ref.fanout_expand(off, tgt, pubs, psilo, tcd)
        batches.append(exp)
        args.append((t.from_numpy(pubs.view(np.int32)).cuda(), t.from_numpy(psilo).cuda(), len(pubs),
                     t.empty(len(pubs) + 1, dtype=t.int64, device="cuda")))
    streams = [t.cuda.Stream() for _ in range(nranks)]
    t.cuda.synchronize()

    def one(r):
        d_pubs, d_psilo, n_pub, poff = args[r]
        res = nodes[r].fanout_batch_device(d_off, d_tgt, None, tcd, d_pubs, d_psilo, n_pub, poff, stream=streams[r].cuda_stream)
        streams[r].synchronize()
        return res, nodes[r].fetch(res, stream=streams[r].cuda_stream)

    with ThreadPoolExecutor(nranks) as ex:
        got = list(ex.map(one, range(nranks)))
    exp, forward = world.expected(batches, 2)
    for r in range(nranks):
        res, (route, act, order, off_, hdrs) = got[r]
        assert res.emitted == len(batches[r])
        er, ea, eo, ef, eh = exp[r]
        np.testing.assert_array_equal(hdrs, eh, err_msg=f"rank {r} headers")
        np.testing.assert_array_equal(route, er, err_msg=f"rank {r} route")
        np.testing.assert_array_equal(act, ea, err_msg=f"rank {r} act")
        np.testing.assert_array_equal(order, eo, err_msg=f"rank {r} order")
        np.testing.assert_array_equal(off_, ef, err_msg=f"rank {r} offsets")
    for nd in nodes:
        nd.close()
    world.close()


def test_node_capacity_error_is_consistent(torch):
    """A batch that would overflow one rank's max_recv fails on EVERY rank with ORL_E_CAPACITY (no rank waits)."""
    t = torch
    world = World(2, n_grains=20_000, host_mix=0.0)
    nodes = [GrainNode(world.engs[r], 2, r, world.ros, max_batch=100_000, max_recv=60_000, transport=L.TRANSPORT_LOCAL,
                       group_id=b"node-cap", chunks=2) for r in range(2)]
    batches = [world.messages(r, 100_000, seed=r) for r in range(2)]
    d_in = [t.from_numpy(b.view(np.int32).reshape(-1, 8)).cuda() for b in batches]

    def one(r):
        try:
            nodes[r].route_batch_device(d_in[r], len(batches[r]))
            return 0
        except L.OrleansRouteError as e:
            return e.code

    with ThreadPoolExecutor(2) as ex:
        codes = list(ex.map(one, range(2)))
    assert codes == [L.E_CAPACITY, L.E_CAPACITY]
    for nd in nodes:
        nd.close()
    world.close()


def test_node_rccl_single_rank(torch):
    """The RCCL transport with a communicator of one rank: init from orl_node_unique_id, counts all-gather, grouped
    self send; results == the direct route + bucket of the context."""
    t = torch
    world = World(1, n_grains=30_000, host_mix=0.0)
    node = GrainNode(world.engs[0], 1, 0, world.ros, max_batch=300_000, max_recv=300_000, transport=L.TRANSPORT_RCCL,
                     group_id=GrainNode.unique_id(), chunks=3)
    s = t.cuda.Stream()
    batches = [world.messages(0, 250_000, seed=9)]
    (res, (route, act, order, off, hdrs)), = _run(t, world, [node], batches, [s])
    exp, forward = world.expected(batches, 3)
    er, ea, eo, ef, eh = exp[0]
    assert not forward and not res.hop2
    np.testing.assert_array_equal(hdrs, eh)
    np.testing.assert_array_equal(route, er)
    np.testing.assert_array_equal(act, ea)
    np.testing.assert_array_equal(order, eo)
    np.testing.assert_array_equal(off, ef)
    node.close()
    world.close()
