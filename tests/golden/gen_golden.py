"""Generate the committed golden fixtures in tests/golden/ from the pure-Python restatement (oracle/pyref.py).

The reference (randa1/orleans, C#/.NET 4.5) cannot be compiled or run in this container (no dotnet / mono),
so these vectors come from the independent restatement, and are cross-checked in tests against the C++
restatement (oracle/cpu_ref.cpp) and the HIP library.  Hash-family anchors:
  * JenkinsHash: byte path == u64 path (the reference's own ID_HashCorrectness property,
    src/TesterInternal/General/Identifiertests.cs:284-301);
  * SHA-256 (CalculateIdHash) via Python hashlib (FIPS 180-4), checked against the FIPS "abc" vector.
The Chirper fixture is derived from the reference's shipped sample data
(Samples/Chirper/NetworkLoader/GraphData/Network-1000nodes-27000edges.graphml): only its edge list is kept.

Run:  python tests/golden/gen_golden.py [--graphml PATH]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

from oracle import pyref as P  # noqa: E402

GRAPHML = "/root/reference/Samples/Chirper/NetworkLoader/GraphData/Network-1000nodes-27000edges.graphml"

MSG_DTYPE = np.dtype([("tcd", "<u8"), ("n0", "<u8"), ("n1", "<u8"), ("sending_silo", "u1"), ("category", "u1"),
                      ("flags", "u1"), ("target_silo", "u1"), ("aux", "<u4")])
KEY_DTYPE = np.dtype([("tcd", "<u8"), ("n0", "<u8"), ("n1", "<u8")])


def rng_u64(seed: int, n: int):
    out, x = [], seed
    for _ in range(n):
        x = (x + 1) & P.M64
        out.append(P.splitmix64(x))
    return out


def gen_jenkins():
    r = rng_u64(0xB00B5, 4000)
    byte_cases = []
    for ln in range(0, 41):
        data = b"".join(v.to_bytes(8, "little") for v in r[ln * 6: ln * 6 + 6])[:ln]
        byte_cases.append({"hex": data.hex(), "hash": P.jenkins_bytes(data)})
    for s in ["", "a", "Orleans", "Four score and seven years ago", "x" * 400]:
        b = s.encode()
        byte_cases.append({"hex": b.hex(), "hash": P.jenkins_bytes(b)})
    u64_cases = []
    for i in range(256):
        u1, u2, u3 = r[1000 + 3 * i: 1003 + 3 * i]
        h = P.jenkins_u64(u1, u2, u3)
        assert h == P.jenkins_bytes(u1.to_bytes(8, "little") + u2.to_bytes(8, "little") + u3.to_bytes(8, "little"))
        u64_cases.append({"u": [hex(u1), hex(u2), hex(u3)], "hash": h})
    for u in [(0, 0, 0), (P.M64, P.M64, P.M64), (1, 2, 3), (1 << 63, 0, 1)]:
        u64_cases.append({"u": [hex(x) for x in u], "hash": P.jenkins_u64(*u)})
    tc_chirper = P.calc_id_hash(P.CHIRPER_ACCOUNT_CLASS)
    key_cases = []
    type_codes = [tc_chirper, 0, 1, -1, -(1 << 31), (1 << 31) - 1, 0xFABCCBAF - (1 << 32)]  # (int)0xfabccbaf
    long_keys = [0, 1, -1, (1 << 31) - 1, -(1 << 63), (1 << 63) - 1, 44444841, 12345]
    for tc in type_codes:
        for k in long_keys:
            key = P.key_from_long(k, tc)
            key_cases.append({"kind": "long", "type_code": tc, "key": k, "tcd": hex(key.tcd), "n0": hex(key.n0),
                              "n1": hex(key.n1), "uniform": P.uniform_hash(key)})
    guids = ["01145FEC-C21E-11E0-9105-D0FB4724019B", "00000000-0000-0000-0000-000000000000",
             "ffffffff-ffff-ffff-ffff-ffffffffffff", "3f2504e0-4f89-11d3-9a0c-0305e82c3301"]
    for tc in type_codes[:3]:
        for g in guids:
            key = P.key_from_guid(g, tc)
            key_cases.append({"kind": "guid", "type_code": tc, "guid": g, "tcd": hex(key.tcd), "n0": hex(key.n0),
                              "n1": hex(key.n1), "uniform": P.uniform_hash(key)})
    for sid in [10, 11, 14, 15, 17, -1]:
        key = P.key_system_target(sid)
        key_cases.append({"kind": "system_target", "system_id": sid, "tcd": hex(key.tcd), "n0": hex(key.n0),
                          "n1": hex(key.n1), "uniform": P.uniform_hash(key)})
    mk = P.MEMBERSHIP_TABLE_KEY
    key_cases.append({"kind": "membership_table", "tcd": hex(mk.tcd), "n0": hex(mk.n0), "n1": hex(mk.n1),
                      "uniform": P.uniform_hash(mk)})
    keyext_cases = []
    for ext in ["1", "2", "case 3", "case 5", "Guid-ExtKey-1", "12345" + "*" * 400, "é中\U0001F600"]:
        for base in [P.key_from_long(7, tc_chirper, ext), P.key_from_guid(guids[3], tc_chirper, ext)]:
            keyext_cases.append({"tcd": hex(base.tcd), "n0": hex(base.n0), "n1": hex(base.n1), "ext": ext,
                                 "serialized": P.serialize_unique_key(base).hex(), "uniform": P.uniform_hash(base)})
    return {"bytes": byte_cases, "u64": u64_cases, "keys": key_cases, "keyext": keyext_cases,
            "chirper_type_code": tc_chirper}


def gen_idhash():
    strings = ["", "a", "abc", P.CHIRPER_ACCOUNT_CLASS, "Orleans.Samples.Chirper.GrainInterfaces.IChirperAccount",
               "UnitTests.GrainInterfaces.ITestGrain", "été", "中文", "\U0001F600 emoji"]
    ids = [{"text": s, "hash": P.calc_id_hash(s)} for s in strings]
    silos = []
    for ep, gen in [(f"10.0.0.{i}:11111", 1) for i in range(1, 9)] + [
            ("127.0.0.1:22222", 0), ("127.0.0.1:22223", 123456789), ("[::1]:11111", -1),
            ("[fe80::1%3]:40000", -2147483648), ("192.168.1.254:65535", 2147483647)]:
        silos.append({"endpoint": ep, "generation": gen, "hash": P.silo_consistent_hash(ep, gen)})
    ip16 = bytes(12) + bytes([10, 0, 0, 1])
    uni = [{"ip16": ip16.hex(), "port": 11111, "generation": 1, "extra": e,
            "hash": P.silo_uniform_hash(ip16, 11111, 1, e)} for e in range(30)]
    return {"id_hash": ids, "silo_consistent": silos, "silo_uniform": uni}


def gen_ring():
    cases = []
    r = rng_u64(0x121A6, 5000)
    k = 0
    ring_specs = []
    ring8, _ = P.default_cluster()
    ring_specs.append(("cluster8", [(s, h) for h, s in sorted(ring8.entries, key=lambda e: e[1])]))
    for n in range(1, 9):
        adds = []
        for s in range(n):
            adds.append((s, P._to_int32(r[k])))
            k += 1
        ring_specs.append((f"rand{n}", adds))
    # ties: equal hashes inserted in silo order (AddServer inserts before existing equals)
    ring_specs.append(("ties", [(0, 100), (1, 100), (2, -5), (3, 100), (4, (1 << 31) - 1), (5, -(1 << 31))]))
    ring_specs.append(("extremes", [(0, -(1 << 31)), (1, (1 << 31) - 1)]))
    for name, adds in ring_specs:
        ring = P.Ring()
        for s, h in adds:
            ring.add_server(s, h)
        n_silos = max(s for s, _ in adds) + 1
        queries = []
        hashes = [h for h, _ in ring.entries]
        probe = set()
        for h in hashes:
            probe.update({h, (h - 1) & P.M32, (h + 1) & P.M32})
        probe.update({0, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF})
        for i in range(24):
            probe.add(r[k] & P.M32)
            k += 1
        for hv in sorted(probe):
            hv &= P.M32
            for me in range(n_silos):
                for running in (True, False):
                    for excl in (False, True):
                        view = P.SiloView(running=[running if s == me else True for s in range(n_silos)],
                                          functional=[True] * n_silos)
                        key = P.Key((P.CAT_GRAIN << 56), 0, 0)
                        owner, code = P.calculate_target_silo(ring, key, hv, me, view, excl)
                        queries.append([hv, me, int(running), int(excl), owner, code])
        cases.append({"name": name, "adds": adds, "ring": ring.entries, "queries": queries})
    # empty ring
    ring = P.Ring()
    q = []
    for running in (True, False):
        for excl in (False, True):
            view = P.SiloView(running=[running], functional=[True])
            owner, code = P.calculate_target_silo(ring, P.Key(3 << 56, 0, 0), 12345, 0, view, excl)
            q.append([12345, 0, int(running), int(excl), owner, code])
    cases.append({"name": "empty", "adds": [], "ring": [], "queries": q})
    return cases


def msgs_to_np(msgs):
    a = np.zeros(len(msgs), MSG_DTYPE)
    for i, m in enumerate(msgs):
        a[i] = (m.key.tcd, m.key.n0, m.key.n1, m.sending_silo, 2, m.flags, m.target_silo_hint, m.aux)
    return a


def gen_routing(name, n_grains, n_msgs, n_act, running, functional, seed_silo, opts, policy, seed):
    ring, hashes = P.default_cluster()
    n_silos = len(hashes)
    view = P.SiloView(running=running, functional=functional, seed=seed_silo)
    tc = P.calc_id_hash(P.CHIRPER_ACCOUNT_CLASS)
    part = P.Partition()
    r = rng_u64(seed, 4 * n_msgs + 4 * n_grains)
    k = 0
    reg_keys, reg_acts, reg_silos, reg_status, reg_wact, reg_wsilo = [], [], [], [], [], []
    grains = []
    for g in range(n_grains):
        kind = r[k] % 100
        k += 1
        if kind < 80:
            key = P.key_from_long(g, tc)
        elif kind < 90:
            gb = (r[k] ^ g).to_bytes(8, "little") + r[k + 1].to_bytes(8, "little")
            k += 2
            key = P.Key(P.type_code_data(P.CAT_GRAIN, tc), int.from_bytes(gb[:8], "little"),
                        int.from_bytes(gb[8:], "little"))
        elif kind < 95:
            key = P.Key(P.type_code_data(P.CAT_CLIENT, 0), r[k], r[k + 1])
            k += 2
        else:
            key = P.Key(P.type_code_data(P.CAT_SYSTEM_GRAIN, 77), 0, g)
        grains.append(key)
    # register 90%: activation silo = owner (70%) or another silo; some duplicate registrations (first writer wins)
    order = list(range(n_grains))
    for g in order:
        if r[k] % 10 == 0:
            k += 1
            continue
        k += 1
        key = grains[g]
        hv = P.uniform_hash(key)
        owner, code = P.calculate_target_silo(ring, key, hv, 0, P.SiloView([True] * n_silos, [True] * n_silos,
                                                                           seed_silo), True)
        silo = owner if r[k] % 10 < 7 else r[k] % n_silos
        k += 1
        act = g
        for rep in range(2 if g % 97 == 0 else 1):  # a second writer for a few grains loses
            # RegisterSingleActivation on the activation's silo; exclusion uses that silo's Running flag
            me = silo if rep == 0 else (silo + 1) % n_silos
            a = act if rep == 0 else (act + n_grains) % n_act
            st, wa, ws = P.register_single_activation(ring, part, view, key, a, me)
            reg_keys.append((key.tcd, key.n0, key.n1))
            reg_acts.append(a)
            reg_silos.append(me)
            reg_status.append(st)
            reg_wact.append(wa)
            reg_wsilo.append(ws)
    msgs = []
    for i in range(n_msgs):
        sel = r[k] % 1000
        k += 1
        me = r[k] % n_silos
        k += 1
        if sel < 900:
            key = grains[r[k] % n_grains]
            k += 1
            msgs.append(P.Msg(key, me))
        elif sel < 930:
            msgs.append(P.Msg(P.key_from_long(n_grains + (r[k] % 1000), tc), me))  # never registered
            k += 1
        elif sel < 945:
            msgs.append(P.Msg(P.key_system_target(int(r[k] % 30)), me))
            k += 1
        elif sel < 955:
            msgs.append(P.Msg(P.MEMBERSHIP_TABLE_KEY, me))
        elif sel < 975:
            ext = "ext-%d" % (r[k] % 50)
            k += 1
            key = P.key_from_long(int(r[k] % 100), tc, ext)
            k += 1
            msgs.append(P.Msg(key, me, P.HDR_HASH_VALID, P.NULL_SILO, P.uniform_hash(key)))
        else:
            key = grains[r[k] % n_grains]
            k += 1
            msgs.append(P.Msg(key, me, P.HDR_ADDRESS_COMPLETE, int(r[k] % n_silos)))
            k += 1
    routes, acts = P.route_batch(msgs, ring, part, view, bool(opts & 1), policy)
    offsets, bucket_order = P.bucket_stable(acts, n_act)
    np.savez_compressed(
        os.path.join(HERE, name + ".npz"),
        silo_hashes=np.array(hashes, np.int32), running=np.array(running, np.uint8),
        functional=np.array(functional, np.uint8), seed=np.uint32(seed_silo), opts=np.uint32(opts),
        policy=np.uint32(policy), n_act=np.uint32(n_act),
        reg_keys=np.array(reg_keys, np.uint64).reshape(-1, 3), reg_acts=np.array(reg_acts, np.uint32),
        reg_silos=np.array(reg_silos, np.uint8), reg_status=np.array(reg_status, np.uint8),
        reg_wact=np.array(reg_wact, np.uint32), reg_wsilo=np.array(reg_wsilo, np.uint8),
        msgs=msgs_to_np(msgs).view(np.uint8).reshape(-1, 32), route=np.array(routes, np.uint32),
        act=np.array(acts, np.uint32), order=np.array(bucket_order, np.uint32), offsets=np.array(offsets, np.uint32))


def gen_chirper(graphml: str):
    text = open(graphml, encoding="utf-8-sig").read()
    nodes = [int(x) for x in re.findall(r'<node id="(\d+)"', text)]
    edges = [(int(a), int(b)) for a, b in re.findall(r'<edge id="[^"]*" source="(\d+)" target="(\d+)"', text)]
    ids = {v: i for i, v in enumerate(nodes)}
    src = np.array([ids[a] for a, _ in edges], np.int64)
    tgt = np.array([ids[b] for _, b in edges], np.int64)
    # `source follows target` (ChirperNetworkLoader.cs:231-242 → FollowUserId): target's followers get its chirps
    pub = tgt
    fol = src
    order = np.argsort(pub, kind="stable")
    counts = np.bincount(pub, minlength=len(nodes))
    off = np.zeros(len(nodes) + 1, np.uint64)
    off[1:] = np.cumsum(counts)
    ftgt = np.array(nodes, np.uint64)[fol[order]].astype(np.uint32)  # follower account id (long key)
    ring, hashes = P.default_cluster()
    view = P.SiloView([True] * 8, [True] * 8)
    tc = P.calc_id_hash(P.CHIRPER_ACCOUNT_CLASS)
    part = P.Partition()
    # every account registered on its owner silo, activation handle = dense node index
    for i, v in enumerate(nodes):
        key = P.key_from_long(v, tc)
        own, _ = P.calculate_target_silo(ring, key, P.uniform_hash(key), 0, view, True)
        part.add_single_activation(key, i, own, view)
    # each account publishes once, from its owner silo; the CSR is indexed by dense node index
    pubs = np.arange(len(nodes), dtype=np.uint32)
    pub_silo = np.array([P.calculate_target_silo(ring, P.key_from_long(v, tc), P.uniform_hash(P.key_from_long(v, tc)),
                                                 0, view, True)[0] for v in nodes], np.uint8)
    follower_tcd = P.type_code_data(P.CAT_GRAIN, tc)
    msgs = []
    for p in range(len(nodes)):
        for e in range(int(off[p]), int(off[p + 1])):
            msgs.append(P.Msg(P.Key(follower_tcd, 0, int(ftgt[e])), int(pub_silo[p])))
    routes, acts = P.route_batch(msgs, ring, part, view)
    offsets, bucket_order = P.bucket_stable(acts, len(nodes))
    np.savez_compressed(os.path.join(HERE, "chirper_fanout.npz"), node_ids=np.array(nodes, np.int64),
                        edge_src=np.array([a for a, _ in edges], np.int64), edge_tgt=np.array([b for _, b in edges], np.int64),
                        csr_off=off, csr_tgt=ftgt, pubs=pubs, pub_silo=pub_silo, follower_tcd=np.uint64(follower_tcd),
                        route=np.array(routes, np.uint32), act=np.array(acts, np.uint32),
                        order=np.array(bucket_order, np.uint32), offsets=np.array(offsets, np.uint32))


def gen_chirper_generated(n_accounts: int = 1000, followers: int = 10):
    """BASELINE config 1: the ChirperNetworkGenerator graph in its deterministic mode
    (Samples/Chirper/NetworkGenerator/ChirperNetworkGenerator.cs:306-345, node / edge / edge-node ids start at 1:
    source = rel / k + 1, target = (rel / k + 1 + rel % k) % n + 1; source != target always, so the random
    replacement never runs) on ONE silo (10.0.0.1:11111, generation 1).  Every account publishes once: 10k routed
    messages.  Activation handle of account id v = v - 1."""
    e = np.arange(n_accounts * followers, dtype=np.int64)
    rel_src = e // followers
    src = rel_src + 1
    tgt = (rel_src + 1 + e % followers) % n_accounts + 1
    assert (src != tgt).all()
    pub, fol = tgt - 1, src  # `source follows target`: the target publishes to its followers
    order = np.argsort(pub, kind="stable")
    counts = np.bincount(pub, minlength=n_accounts)
    off = np.zeros(n_accounts + 1, np.uint64)
    off[1:] = np.cumsum(counts)
    ftgt = fol[order].astype(np.uint32)  # follower account id (long key)
    ring = P.Ring()
    ring.add_server(0, P.silo_consistent_hash("10.0.0.1:11111", 1))
    view = P.SiloView([True], [True])
    tc = P.calc_id_hash(P.CHIRPER_ACCOUNT_CLASS)
    part = P.Partition()
    for v in range(1, n_accounts + 1):
        part.add_single_activation(P.key_from_long(v, tc), v - 1, 0, view)
    follower_tcd = P.type_code_data(P.CAT_GRAIN, tc)
    msgs = [P.Msg(P.Key(follower_tcd, 0, int(ftgt[j])), 0) for p in range(n_accounts)
            for j in range(int(off[p]), int(off[p + 1]))]
    routes, acts = P.route_batch(msgs, ring, part, view)
    offsets, bucket_order = P.bucket_stable(acts, n_accounts)
    np.savez_compressed(os.path.join(HERE, "chirper_generated.npz"), csr_off=off, csr_tgt=ftgt,
                        pubs=np.arange(n_accounts, dtype=np.uint32), pub_silo=np.zeros(n_accounts, np.uint8),
                        follower_tcd=np.uint64(follower_tcd), silo_hash=np.int32(ring.entries[0][0]),
                        route=np.array(routes, np.uint32), act=np.array(acts, np.uint32),
                        order=np.array(bucket_order, np.uint32), offsets=np.array(offsets, np.uint32))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphml", default=GRAPHML)
    args = ap.parse_args()
    with open(os.path.join(HERE, "jenkins.json"), "w") as f:
        json.dump(gen_jenkins(), f, indent=0)
    with open(os.path.join(HERE, "idhash.json"), "w") as f:
        json.dump(gen_idhash(), f, indent=0)
    with open(os.path.join(HERE, "ring.json"), "w") as f:
        json.dump(gen_ring(), f, separators=(",", ":"))
    n_silos = 8
    gen_routing("routing_basic", 4096, 16384, 8192, [1] * n_silos, [1] * n_silos, 0, 0, P.POLICY_PREFER_LOCAL, 0xC0FFEE)
    running = [1] * n_silos
    running[3] = 0
    functional = [1] * n_silos
    functional[5] = 0
    gen_routing("routing_membership", 4096, 16384, 8192, running, functional, P.NULL_SILO, 1, P.POLICY_HASH_SPREAD,
                0xBEEF)
    gen_chirper_generated()
    if os.path.exists(args.graphml):
        gen_chirper(args.graphml)
    else:
        print("graphml not found; chirper_fanout.npz not regenerated", file=sys.stderr)


if __name__ == "__main__":
    main()
