"""The node exchange protocol replayed by the oracle in ONE process (test infrastructure).

Used by tests/test_gpu_node.py (checks orl_node on the GPU) and tests/test_distributed.py (checks the protocol's host
decisions, orl_node_plan_chunk / orl_node_plan_hop2, over gloo with several processes).  What every rank must end with,
for one batch per rank: each rank's chunks partitioned by the rank of the message's directory owner (the oracle
partition, OutboundMessageQueue.SendMessage's per-target-silo queues, OutboundMessageQueue.cs:113-145); the owned set in
(chunk, source rank) order routed by the owner's directory (LocalGrainDirectory.cs:439-497); when any rank hosts an
activation another rank owns, every routed message forwarded to its host rank in owner order (Dispatcher.TransportMessage,
Dispatcher.cs:618-622); the hosted set bucketed per activation, FIFO (ActivationData.cs:483-514).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from oracle import cpu_ref
from orleans_amd import _lib as L
from orleans_amd import workloads as W
from orleans_amd.engine import decode_route


@dataclass
class Population:
    cl: W.Cluster
    ros: np.ndarray       # rank of each silo
    keys: np.ndarray      # KEY_DTYPE[n_grains]
    owner: np.ndarray     # directory owner silo of each grain
    reg: np.ndarray       # registered grains
    host: np.ndarray      # activation silo of each grain (the owner, or another silo for host_mix of them)
    act: np.ndarray       # activation handle: dense per host rank (each rank's catalog numbers its activations)
    n_act: int
    n_grains: int


def population(nranks, n_grains=40_000, seed=3, host_mix=0.3, ros=None, cl=None, reg_frac=0.9) -> Population:
    cl = cl or W.default_cluster()
    ros = cl.rank_of_silo(nranks) if ros is None else np.asarray(ros, np.uint8)
    keys, uni, owner, reg = W.grain_population(cl, n_grains, reg_frac, seed)
    rng = np.random.default_rng(seed)
    host = np.where(rng.random(n_grains) < 1.0 - host_mix, owner, rng.integers(0, 8, n_grains)).astype(np.uint8)
    hrank = ros[host]
    act = np.zeros(n_grains, np.uint32)
    cnt = []
    for r in range(nranks):
        idx = np.nonzero((hrank == r) & reg)[0]
        act[idx] = np.arange(len(idx), dtype=np.uint32)
        cnt.append(len(idx))
    return Population(cl, ros, keys, owner, reg, host, act, max(cnt) + 8, n_grains)


def rank_selection(p: Population, r: int) -> np.ndarray:
    """Grains whose directory entry rank r holds (registered, owner silo on rank r)."""
    return np.nonzero(p.reg & (p.ros[p.owner] == r))[0]


def rank_oracle(p: Population, r: int) -> cpu_ref.Oracle:
    local = (p.ros == r).astype(np.uint8)
    o = cpu_ref.Oracle(8, local=list(local))
    for s in range(8):
        o.add_server(s, int(p.cl.hashes[s]))
    sel = rank_selection(p, r)
    st, _, _ = o.register(p.keys[sel], p.act[sel], p.host[sel])
    assert (st == L.INS_INSERTED).all()
    return o


def chunk_bounds(n: int, chunks: int, c: int):
    cs = -(-n // chunks)
    lo = min(c * cs, n)
    return lo, min(lo + cs, n)


def host_rank(route: np.ndarray, ros: np.ndarray, me: int) -> np.ndarray:
    """Rank hosting each routed message's activation (no host silo: stays on the owner)."""
    h = decode_route(route).host
    return np.where(h == 0xFF, me, ros[np.minimum(h, 7).astype(np.int64)])


def expected(oracles, ros, batches, chunks, n_act, caches=None, functional=None, keyext=None):
    """The oracle's replay of one batch per rank -> ([per rank (route, act, order, offsets, hosted headers)], forward).

    caches[s] (optional): rank s's directory cache {(tcd, n0, n1): (act, silo)}.  A message whose owner is on another rank
    and whose grain rank s caches on a functional silo is addressed at the sender (LocalLookup's cache branch,
    LocalGrainDirectory.cs:690-717; pyref.apply_directory_cache: HIT | CACHED, TargetSilo = the cached silo) and sent to
    the rank hosting that silo instead of the owner's; the others follow the oracle partition by owner rank.  The receiver
    checks a cached record against its directory when it holds the grain's partition (stale entries are
    re-addressed and flagged ORL_RF_CACHE_STALE).  keyext(d, headers) -> (route, act) (optional): rank d's KeyExt lookups
    of the KeyExt messages it owns (strings beside the records: orl_node_route_batch_keyext_device)."""
    from oracle import pyref as P
    nr = len(batches)
    functional = functional if functional is not None else [1] * 8
    owned = [[] for _ in range(nr)]
    pre = [[] for _ in range(nr)]  # per owned record: (route, act) the sender's cache decided, or None
    for c in range(chunks):
        for s in range(nr):
            lo, hi = chunk_bounds(len(batches[s]), chunks, c)
            ch = batches[s][lo:hi].copy()
            src, cnt = oracles[0].partition(ch, ros, nr, s)
            dest = np.zeros(len(ch), np.int64)
            o0 = 0
            for d in range(nr):
                dest[src[o0:o0 + int(cnt[d])]] = d
                o0 += int(cnt[d])
            croute = np.full(len(ch), -1, np.int64)
            cact = np.zeros(len(ch), np.uint32)
            if caches is not None and caches[s] and len(ch):
                r0, a0 = oracles[s].route(ch)  # rank s's view: REMOTE_OWNER for grains owned elsewhere
                kt = list(zip(ch["tcd"].tolist(), ch["n0"].tolist(), ch["n1"].tolist()))
                r1, a1 = P.apply_directory_cache(r0.tolist(), a0.tolist(), ch["sending_silo"].tolist(), kt, caches[s],
                                                 functional)
                r1 = np.array(r1, np.uint32)
                hit = (r1 >> 24) & 0x08 != 0
                hit &= ((r0 >> 16) & 0xFF) == L.ST_REMOTE_OWNER
                hs = ((r1 >> 8) & 0xFF).astype(np.int64)
                dest[hit] = ros[hs[hit]]
                croute[hit] = r1[hit]
                cact[hit] = np.array(a1, np.uint32)[hit]
                ch["target_silo"][hit] = hs[hit].astype(np.uint8)  # the addressed record's TargetSilo
            order = np.argsort(dest, kind="stable")
            for d in range(nr):
                sel = order[dest[order] == d]
                owned[d].append(ch[sel])
                pre[d].append((croute[sel], cact[sel]))
    owned = [np.concatenate(x) if x else np.zeros(0, L.MSG_DTYPE) for x in owned]
    routed = []
    for d in range(nr):
        r, a = oracles[d].route(owned[d])
        if keyext is not None:  # KeyExt messages with their strings: the owner's KeyExt table (keyext(d, headers))
            kx = ((r >> 16) & 0xFF) == L.ST_KEYEXT_UNRESOLVED
            if kx.any():
                r, a = r.copy(), a.copy()
                r[kx], a[kx] = keyext(d, owned[d][kx])
        if pre[d]:
            cr = np.concatenate([x[0] for x in pre[d]])
            ca = np.concatenate([x[1] for x in pre[d]])
            m = cr >= 0
            r = r.copy()
            a = a.copy()
            # a record the sender addressed from its cache: where rank d holds the grain's directory partition (its own
            # route is not REMOTE_OWNER) the directory decides — HIT | CACHED kept only when it holds that handle on that
            # silo, else the directory's word | CACHE_STALE (NonExistentActivation → forward, Dispatcher.cs:138-182);
            # elsewhere the record is taken as addressed
            own_dir = ((r >> 16) & 0xFF) != L.ST_REMOTE_OWNER
            crw = cr.astype(np.uint32)
            same = (((r >> 16) & 0xFF) == L.ST_HIT) & (a == ca) & (((r >> 8) & 0xFF) == ((crw >> 8) & 0xFF))
            keep = m & (~own_dir | same)
            stale = m & own_dir & ~same
            r[keep] = crw[keep]
            a[keep] = ca[keep]
            r[stale] |= np.uint32(L.RF_CACHE_STALE << 24)
        routed.append((r, a))
    hostr = [host_rank(routed[d][0], ros, d) for d in range(nr)]
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
        order, off = oracles[hr].bucket(act, n_act)
        out.append((route, act, order, off, hdr))
    return out, forward


def messages(p: Population, rank: int, n: int, seed: int, wide_at=None) -> np.ndarray:
    """One rank's batch: targets uniform over the population (+3000 never-registered grains), senders = the rank's silos;
    3 % responses with complete addresses, 2 % system-target messages, optionally one Guid-keyed target at `wide_at`
    (its chunk has no compact exchange form)."""
    silos = np.nonzero(p.ros == rank)[0].astype(np.uint8)
    m = W.uniform_messages(p.cl, p.n_grains + 3000, n, seed=seed, sender_silos=silos)
    rng = np.random.default_rng(seed)
    c = rng.random(n)
    m["flags"][c < 0.03] = L.HDR_ADDRESS_COMPLETE  # responses: complete addresses, routed to the target silo
    m["target_silo"][c < 0.03] = rng.integers(0, 8, int((c < 0.03).sum()))
    st = (c >= 0.03) & (c < 0.05)
    m["tcd"][st] = (np.uint64(L.CAT_SYSTEM_TARGET) << np.uint64(56)) | np.uint64(12)
    if wide_at is not None:
        m["n0"][wide_at] = 0x1234
    return m


def wire_types(p: Population, mode):
    """Each rank's wire-type list for `mode`: None (8-B form off), "both" (grain + system-target types), "grain_only"
    (system-target messages lack the form), "mismatch" (the last rank lists them in another order: digests differ)."""
    nr = int(p.ros.max()) + 1
    if mode is None:
        return [[] for _ in range(nr)]
    grain_t = (L.CAT_GRAIN << 56) + (p.cl.type_code & 0x00FFFFFFFFFFFFFF)
    sys_t = (L.CAT_SYSTEM_TARGET << 56) | 12
    out = []
    for r in range(nr):
        types = [grain_t] if mode == "grain_only" else [grain_t, sys_t]
        if mode == "mismatch" and r == nr - 1:
            types = [sys_t, grain_t]
        out.append(types)
    return out
