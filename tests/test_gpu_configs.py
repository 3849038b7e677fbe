"""GPU parity at the BASELINE workloads (configs 1, 3, 4, 5 of SURVEY §8(d)) and the host-mutation contract.

Each full-size config runs the HIP path (through the C ABI) at its BASELINE size, asserts the size-independent
properties of the outputs (a permutation grouped by activation, arrival order inside each bucket, offsets = the
histogram prefix, route words consistent with the directory) and checks a >= 1M-message oracle sample bit for bit
(config 5's 590k messages per step are checked in full).  All integer work: exact equality, no tolerance.
"""
import numpy as np
import pytest

from oracle import cpu_ref
from orleans_amd import _lib as L
from orleans_amd import workloads as W
from orleans_amd.engine import GrainDirectoryEngine, decode_route

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def _u32(x):
    return x.cpu().numpy().view(np.uint32)


def check_buckets(a, od, of, n_act):
    """Stage-4 properties for activation handles a[n] (ORL_NO_ACT = unresolved bucket n_act)."""
    n = len(a)
    key = np.minimum(a.astype(np.int64), n_act)
    cnt = np.bincount(key, minlength=n_act + 1)
    exp_off = np.zeros(n_act + 2, np.int64)
    exp_off[1:] = np.cumsum(cnt)
    np.testing.assert_array_equal(of.astype(np.int64), exp_off)
    assert (np.bincount(od, minlength=n) == 1).all()             # a permutation
    srt = key[od]
    assert (np.diff(srt) >= 0).all()                             # grouped by activation
    same = np.diff(srt) == 0
    assert (np.diff(od.astype(np.int64))[same] > 0).all()        # arrival order inside a bucket


def _oracle_for(cl, keys, acts, silos, n_silos=None):
    o = cpu_ref.Oracle(n_silos or cl.n_silos)
    for s in range(n_silos or cl.n_silos):
        o.add_server(s, int(cl.hashes[s]))
    o.register(keys, acts, silos)
    return o


# ---- config 1 -----------------------------------------------------------------------------------------------
def test_config1_chirper_generated_golden(torch, golden_dir):
    """Config 1: ChirperNetworkGenerator's deterministic graph (ChirperNetworkGenerator.cs:306-345), 1k accounts x 10
    followers on ONE silo, every account publishes once: 10k fan-out messages == the committed golden."""
    import os
    t = torch
    d = np.load(os.path.join(golden_dir, "chirper_generated.npz"))
    eng = GrainDirectoryEngine(n_act=1000, dir_capacity=1000, max_batch=1 << 15, device=0)
    eng.set_silos(1)
    eng.add_server(0, int(d["silo_hash"]))
    keys = np.zeros(1000, L.KEY_DTYPE)
    keys["tcd"] = int(d["follower_tcd"])
    keys["n1"] = np.arange(1, 1001, dtype=np.uint64)
    st, _, _ = eng.register_single_activation(keys, np.arange(1000, dtype=np.uint32), np.zeros(1000, np.uint8))
    assert (st == L.INS_INSERTED).all()
    dv = "cuda"
    n = len(d["route"])
    outs = [t.empty(n, dtype=t.int32, device=dv) for _ in range(3)]
    off = t.empty(1002, dtype=t.int32, device=dv)
    poff = t.empty(1001, dtype=t.int64, device=dv)
    got = eng.fanout_device(t.from_numpy(d["csr_off"].astype(np.int64)).to(dv),
                            t.from_numpy(d["csr_tgt"].astype(np.int32)).to(dv),
                            t.from_numpy(d["pubs"].astype(np.int32)).to(dv), t.from_numpy(d["pub_silo"]).to(dv), 1000,
                            int(d["follower_tcd"]), poff, *outs, off, stream=t.cuda.current_stream().cuda_stream)
    t.cuda.synchronize()
    assert got == n == 10_000
    for x, k in zip(outs + [off], ("route", "act", "order", "offsets")):
        np.testing.assert_array_equal(_u32(x), d[k], err_msg=k)
    eng.close()


# ---- host-side directory changes vs batches in flight ----------------------------------
def test_host_mutation_waits_for_inflight_batch(torch):
    """A host registration / unregistration issued while a routed batch is still running on a side stream must not
    change that batch's decisions (the upload waits for the device); the next batch sees the change."""
    t = torch
    cl = W.default_cluster()
    n_grains, n = 1_000_000, 32 << 20
    eng = GrainDirectoryEngine(n_act=2 * n_grains, dir_capacity=2 * n_grains, max_batch=n, device=0)
    W.setup_engine(eng, cl)
    keys, uni, owner, reg = W.grain_population(cl, 2 * n_grains)
    o = _oracle_for(cl, keys[:n_grains], np.arange(n_grains, dtype=np.uint32), owner[:n_grains])
    eng.register_single_activation(keys[:n_grains], np.arange(n_grains, dtype=np.uint32), owner[:n_grains])
    msgs = W.uniform_messages(cl, 2 * n_grains, n, seed=4)  # half the targets unregistered yet
    d_in = t.from_numpy(msgs.view(np.int32).reshape(-1, 8)).cuda()
    s = t.cuda.Stream()
    outs = [[t.empty(n, dtype=t.int32, device="cuda") for _ in range(3)] + [t.empty(2 * n_grains + 2, dtype=t.int32,
                                                                                      device="cuda")] for _ in range(3)]
    samp = np.random.default_rng(1).choice(n, 1_000_000, replace=False)
    refs = [o.route(msgs[samp])]
    # (1) a small unregistration (slot patch) right behind batch 0; (2) a bulk registration (full upload) behind batch 1
    eng.address_messages_device(d_in, n, *outs[0], stream=s.cuda_stream)
    rm = keys[:100_000]
    eng.unregister(rm)
    o.unregister(rm)
    refs.append(o.route(msgs[samp]))
    eng.address_messages_device(d_in, n, *outs[1], stream=s.cuda_stream)
    new = np.arange(n_grains, 2 * n_grains)
    eng.register_single_activation(keys[new], new.astype(np.uint32), owner[new])
    o.register(keys[new], new.astype(np.uint32), owner[new])
    refs.append(o.route(msgs[samp]))
    eng.address_messages_device(d_in, n, *outs[2], stream=s.cuda_stream)
    s.synchronize()
    assert eng.query(L.Q_SLOT_PATCHES) >= 1 and eng.query(L.Q_FULL_UPLOADS) >= 2
    for b in range(3):
        r = _u32(outs[b][0])
        np.testing.assert_array_equal(r[samp], refs[b][0], err_msg=f"batch {b}")
        np.testing.assert_array_equal(_u32(outs[b][1])[samp], refs[b][1], err_msg=f"batch {b}")
    eng.close()


# ---- incremental slot uploads and the probe-table forms -----------------------------------
def test_incremental_slot_patches_vs_oracle(torch):
    """Small host registration batches are uploaded as slot patches (no whole-table upload), and the compact
    probe forms follow them: 8-B while one type with 32-bit ids fits, 16-B after an id >= 2^32 - 2 or a second
    type, the 32-B table after a Guid key; routing == the oracle after every step."""
    cl = W.default_cluster()
    n_grains = 30_000
    eng = GrainDirectoryEngine(n_act=1 << 16, dir_capacity=4 * n_grains, max_batch=1 << 18, device=0)
    W.setup_engine(eng, cl)
    o = cpu_ref.Oracle(cl.n_silos)
    for s in range(cl.n_silos):
        o.add_server(s, int(cl.hashes[s]))
    keys, uni, owner, reg = W.grain_population(cl, n_grains)

    def register(k, a, s):
        st_e, wa_e, _ = eng.register_single_activation(k, a, s)
        st_o, wa_o, _ = o.register(k, a, s)
        np.testing.assert_array_equal(st_e, st_o)
        np.testing.assert_array_equal(wa_e, wa_o)

    def route_check(seed, extra=None):
        m = W.uniform_messages(cl, n_grains + 1000, 200_000, seed=seed)
        if extra is not None:
            m = np.concatenate([m, extra])
        res = eng.address_messages(m)
        r, a = o.route(m)
        np.testing.assert_array_equal(res.route, r)
        np.testing.assert_array_equal(res.act, a)
        order, off = o.bucket(a, 1 << 16)
        np.testing.assert_array_equal(res.order, order)
        np.testing.assert_array_equal(res.offsets, off)

    register(keys[:20_000], np.arange(20_000, dtype=np.uint32), owner[:20_000])
    route_check(0)
    assert eng.query(L.Q_PROBE_FORM) == 8
    full0, p0 = eng.query(L.Q_FULL_UPLOADS), eng.query(L.Q_SLOT_PATCHES)
    for b in range(5):  # small batches: patches
        lo = 20_000 + 2000 * b
        register(keys[lo:lo + 2000], np.arange(lo, lo + 2000, dtype=np.uint32), owner[lo:lo + 2000])
        o.unregister(keys[b * 700:(b + 1) * 700])
        eng.unregister(keys[b * 700:(b + 1) * 700])
        route_check(b + 1)
    assert eng.query(L.Q_FULL_UPLOADS) == full0 and eng.query(L.Q_SLOT_PATCHES) == p0 + 5
    assert eng.query(L.Q_PROBE_FORM) == 8
    # an id that does not fit the 8-B form (N1 >= 2^32 - 2) and messages sharing its low 32 bits
    from orleans_amd.engine import grain_keys_from_longs, grain_keys_from_guid_bytes
    kb = grain_keys_from_longs(cl.type_code, np.array([(1 << 33) + 5, 0xFFFFFFFE], np.int64))
    ob = cl.owner_of(W.jenkins3_np(kb["tcd"], kb["n0"], kb["n1"]))
    register(kb, np.array([60_001, 60_002], np.uint32), ob)
    assert eng.query(L.Q_PROBE_FORM) == 16
    ex = np.zeros(4, L.MSG_DTYPE)
    ex["tcd"] = kb["tcd"][0]
    ex["n1"] = [(1 << 33) + 5, 5, 0xFFFFFFFE, (1 << 32) + 0xFFFFFFFE]
    ex["category"] = 2
    route_check(10, ex)
    # a second grain type: still 16-B (two types listed)
    k2 = grain_keys_from_longs(cl.type_code ^ 0x5A5A, np.arange(100, dtype=np.int64))
    o2 = cl.owner_of(W.jenkins3_np(k2["tcd"], k2["n0"], k2["n1"]))
    register(k2, np.arange(61_000, 61_100, dtype=np.uint32), o2)
    assert eng.query(L.Q_PROBE_FORM) == 16
    ex2 = np.zeros(100, L.MSG_DTYPE)
    ex2["tcd"], ex2["n1"], ex2["category"] = k2["tcd"], k2["n1"], 2
    route_check(11, ex2)
    # a Guid key (N0 != 0): the full 32-B table
    kg = grain_keys_from_guid_bytes(cl.type_code, np.arange(32, dtype=np.uint8).reshape(2, 16))
    og = cl.owner_of(W.jenkins3_np(kg["tcd"], kg["n0"], kg["n1"]))
    register(kg, np.array([62_000, 62_001], np.uint32), og)
    assert eng.query(L.Q_PROBE_FORM) == 32
    exg = np.zeros(2, L.MSG_DTYPE)
    exg["tcd"], exg["n0"], exg["n1"], exg["category"] = kg["tcd"], kg["n0"], kg["n1"], 2
    route_check(12, exg)
    eng.close()


def test_probe8_sentinel_edges(torch):
    """The 8-B probe form at its edges: a registered N1 = 0xFFFFFFFD with handle 2^24 - 1 keeps the 8-B form; messages
    with N1 = 0xFFFFFFFE / 0xFFFFFFFF (the empty / tombstone keys) and N1 sharing the low 32 bits of a registered id
    route as the oracle does."""
    from orleans_amd.engine import grain_keys_from_longs
    cl = W.default_cluster()
    n_act = 1 << 24
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=4096, max_batch=1 << 16, device=0)
    W.setup_engine(eng, cl)
    ids = np.array(list(range(1000)) + [0xFFFFFFFD, 0xFFFFFFFC], np.int64)
    k = grain_keys_from_longs(cl.type_code, ids)
    own = cl.owner_of(W.jenkins3_np(k["tcd"], k["n0"], k["n1"]))
    acts = np.arange(len(ids), dtype=np.uint32)
    acts[-2] = n_act - 1
    eng.register_single_activation(k, acts, own)
    o = _oracle_for(cl, k, acts, own)
    assert eng.query(L.Q_PROBE_FORM) == 8
    eng.unregister(k[5:10])  # tombstones on some chains
    o.unregister(k[5:10])
    m = np.zeros(20_000, L.MSG_DTYPE)
    m["tcd"] = k["tcd"][0]
    m["category"] = 2
    m["sending_silo"] = np.arange(20_000) % 8
    cand = np.array([0xFFFFFFFE, 0xFFFFFFFF, 0xFFFFFFFD, 0xFFFFFFFC, (1 << 32) + 0xFFFFFFFD, (1 << 32) + 3, 3, 7, 1001,
                     (1 << 40) | 0xFFFFFFFF], np.uint64)
    m["n1"] = cand[np.arange(20_000) % len(cand)]
    res = eng.address_messages(m)
    r, a = o.route(m)
    np.testing.assert_array_equal(res.route, r)
    np.testing.assert_array_equal(res.act, a)
    assert (res.act == n_act - 1).sum() == 2000  # the 2^24 - 1 handle is found
    assert eng.query(L.Q_PROBE_FORM) == 8
    eng.close()


def test_fanout_overstated_total(torch):
    """ORL_OPT_TOTAL_GIVEN with a total larger than the CSR emits: indices past the real total get ORL_ST_PAST_TOTAL
    and the unresolved bucket (no CSR / publisher access past the end); the real messages are unchanged."""
    t = torch
    cl = W.default_cluster()
    n_acc = 50_000
    off, tgt = W.powerlaw_csr(n_acc)
    from orleans_amd.engine import grain_keys_from_longs
    keys = grain_keys_from_longs(cl.type_code, np.arange(n_acc, dtype=np.int64))
    owner = cl.owner_of(W.jenkins3_np(keys["tcd"], keys["n0"], keys["n1"]))
    pubs = (W.stream(7, 0, 3000) % np.uint64(n_acc)).astype(np.uint32)
    real = int(np.diff(off.astype(np.int64))[pubs].sum())
    extra = 5000
    eng = GrainDirectoryEngine(n_act=n_acc, dir_capacity=n_acc, max_batch=real + extra + 1, device=0)
    W.setup_engine(eng, cl)
    W.register_population(eng, keys, owner, np.ones(n_acc, bool))
    dv = "cuda"
    args = [t.from_numpy(off.view(np.int64)).to(dv), t.from_numpy(tgt.view(np.int32)).to(dv),
            t.from_numpy(pubs.view(np.int32)).to(dv), t.from_numpy(owner[pubs]).to(dv), len(pubs),
            (3 << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)]
    res = []
    for total in (None, real + extra):
        m = real + extra
        poff = t.empty(len(pubs) + 1, dtype=t.int64, device=dv)
        outs = [t.full((m,), -3, dtype=t.int32, device=dv) for _ in range(3)]
        of = t.empty(n_acc + 2, dtype=t.int32, device=dv)
        eng.fanout_device(*args, poff, *outs, of, stream=t.cuda.current_stream().cuda_stream, total=total)
        t.cuda.synchronize()
        res.append([_u32(x) for x in outs] + [_u32(of)])
    (r0, a0, o0, f0), (r1, a1, o1, f1) = res
    np.testing.assert_array_equal(r1[:real], r0[:real])
    np.testing.assert_array_equal(a1[:real], a0[:real])
    assert (decode_route(r1[real:]).status == L.ST_PAST_TOTAL).all()
    assert (a1[real:] == L.NO_ACT).all()
    check_buckets(a1, o1, f1, n_acc)
    np.testing.assert_array_equal(f1[:n_acc + 1], f0[:n_acc + 1])
    eng.close()


# ---- config 3: Zipf(1.1) over 16M grains, 24-bit handles (LSD stage 4) ---------------------------------------
def test_config3_full_size_zipf(torch):
    """BASELINE config 3 on one GPU: 16M long-key grains, 64M messages, targets Zipf(1.1) through a seeded
    permutation (hot activations), activation handles up to 2^24 (the LSD bucketing path)."""
    t = torch
    n_grains, n = 16_000_000, 64 << 20
    cl = W.balanced_cluster()
    keys, uni, owner, reg = W.grain_population(cl, n_grains)
    eng = GrainDirectoryEngine(n_act=n_grains, dir_capacity=n_grains, max_batch=n, device=0)
    W.setup_engine(eng, cl)
    W.register_population(eng, keys, owner, reg)
    msgs = W.zipf_messages(cl, n_grains, n)
    d_in = t.from_numpy(msgs.view(np.int32).reshape(-1, 8)).cuda()
    outs = [t.empty(n, dtype=t.int32, device="cuda") for _ in range(3)]
    off = t.empty(n_grains + 2, dtype=t.int32, device="cuda")
    eng.address_messages_device(d_in, n, *outs, off, stream=t.cuda.current_stream().cuda_stream)
    t.cuda.synchronize()
    del d_in
    r, a, od, of = (_u32(x) for x in outs + [off])
    tg = msgs["n1"].astype(np.int64)
    np.testing.assert_array_equal(a, tg.astype(np.uint32))  # handle of grain i is i
    v = decode_route(r)
    assert (v.status == L.ST_HIT).all()
    np.testing.assert_array_equal(v.owner, owner[tg])
    hot = np.bincount(tg, minlength=n_grains).max()
    assert hot > 1_000_000  # Zipf(1.1): the hottest activation gets > 1M of the 64M messages
    check_buckets(a, od, of, n_grains)
    samp = np.random.default_rng(3).choice(n, 1_000_000, replace=False)
    o = _oracle_for(cl, keys, np.arange(n_grains, dtype=np.uint32), owner)
    ro, ao = o.route(msgs[samp])
    np.testing.assert_array_equal(r[samp], ro)
    np.testing.assert_array_equal(a[samp], ao)
    eng.close()


@pytest.mark.timeout(900)
def test_config3_256M_one_gpu(torch):
    """BASELINE config 3's whole batch on one GPU, as `bench.py --config 3` runs it: 256M messages (8 GiB of headers: every
    byte offset past 2^32, the size no smaller test reaches), Zipf(1.1) over 16M grains, generated on the device.  Every
    message is checked on the device by the size-independent properties (orleans_amd/selfcheck.py: owner, host, status
    and handle per message; a permutation grouped by activation, FIFO inside buckets, offsets = the count prefix), and a
    1M-message sample spread over the whole batch (the last 64M included) is bit-exact vs the oracle
    (LocalGrainDirectory.cs:439-497, GrainDirectoryPartition.cs:326-344, ActivationData.cs:483-514)."""
    import time
    from orleans_amd import selfcheck as SC
    t = torch
    t0 = time.perf_counter()
    log = lambda *a: print(f"[c3 256M {time.perf_counter() - t0:6.1f}s]", *a, flush=True)  # noqa: E731
    n_grains, n = 16_000_000, 256 << 20
    cl = W.balanced_cluster()
    keys, uni, owner, reg = W.grain_population(cl, n_grains)
    eng = GrainDirectoryEngine(n_act=n_grains, dir_capacity=n_grains, max_batch=n, device=0)
    W.setup_engine(eng, cl)
    W.register_population(eng, keys, owner, reg)
    d_in = W.device_messages(t, cl, n_grains, n, W.SEED_C3, zipf=W.zipf_tables(t, n_grains, W.SEED_C3))
    log("engine + 256M messages on the device")
    outs = [t.empty(n, dtype=t.int32, device="cuda") for _ in range(3)]
    off = t.empty(n_grains + 2, dtype=t.int32, device="cuda")
    eng.address_messages_device(d_in, n, *outs, off, stream=t.cuda.current_stream().cuda_stream)
    t.cuda.synchronize()
    log("routed")
    m32 = 0xFFFFFFFF
    route, act, order = (x.to(t.int64) & m32 for x in outs)
    offs = off.to(t.int64) & m32
    n1 = d_in.view(t.int64).view(-1, 4)[:, 2]
    owner_t = t.as_tensor(owner.astype(np.int64), device="cuda")
    handle_t = t.arange(n_grains, dtype=t.int64, device="cuda")  # handle of grain i is i
    errs = SC.check_routes(t, route, act, n1, owner_t, handle_t, True)
    errs += SC.check_stage4(t, act, order, offs, n_grains)
    assert not errs, errs
    log("properties of all 256M messages hold")
    samp = np.sort(np.random.default_rng(5).choice(n, 1_000_000, replace=False))
    samp_t = t.as_tensor(samp, device="cuda")
    hdr = d_in.view(-1, 8)[samp_t].cpu().numpy().reshape(-1).view(L.MSG_DTYPE)
    o = _oracle_for(cl, keys, np.arange(n_grains, dtype=np.uint32), owner)
    ro, ao = o.route(hdr)
    np.testing.assert_array_equal(route[samp_t].cpu().numpy().astype(np.uint32), ro)
    np.testing.assert_array_equal(act[samp_t].cpu().numpy().astype(np.uint32), ao)
    assert samp.max() > (192 << 20)
    log("1M-message oracle sample bit-exact")
    eng.close()


@pytest.mark.timeout(900)
def test_config3_8ranks_bench_size_rehearsal(torch):
    """Config 3's 8-GPU split at the size `bench.py --gpus 8` runs it, rehearsed on one GPU (orl_node LOCAL transport, the
    protocol code RCCL runs): 256M messages, 32M originated per rank, 4 chunks of 8-B records, Zipf(1.1) over 16M grains
    (the hot rank owns and hosts ~55M messages, and its second batch takes stage 4's hot-key path).  After the timed batch
    bench.py's checker (node_self_check) verifies every rank's hosted output: the owned count against the workload's own
    per-destination count, owner / host / status / handle of every hosted message, a permutation grouped by activation,
    FIFO inside buckets, offsets = the count prefix, and a 1M-message oracle sample per rank bit for bit
    (OutboundMessageQueue.cs:113-145, LocalGrainDirectory.cs:439-497, ActivationData.cs:483-514)."""
    import argparse
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    args = argparse.Namespace(local_ranks=8, config=3, grains=None, msgs=None, chunks=4, steps=1, warmup=1, wire16=False,
                              unregistered=0.0, check_sample=1 << 20, sender_cache=0)
    res = bench.run_rehearsal(args, torch)
    print({k: res[k] for k in ("ms_per_step", "owned_per_rank", "max_over_mean_owned", "exchange")}, flush=True)
    assert res["check"] == "ok", res["check"]
    assert max(res["owned_per_rank"]) > 50_000_000  # the Zipf-hot grain's owner, at the bench's size
    assert res["exchange"]["ncclCommCount"] == 8


# ---- config 4: 10M-account power-law CSR fan-out --------------------------------------------------------------
@pytest.mark.parametrize("fan_u", [None, "2", "4"])
def test_config4_full_size_fanout(torch, monkeypatch, fan_u):
    """BASELINE config 4: 10M accounts, power-law followers (exponent 2.1, 1..1e5), 1M publishers: the fan-out +
    stages 1-4 on the device; the first >= 1M emitted messages (whole publishers) bit-exact vs the oracle's CSR
    expansion + routing, the rest by properties.  fan_u: the fan-out kernel's messages per thread and step (ORL_FAN_U,
    an A/B knob: 4 messages per thread and step at this size's 1024-message tiles)."""
    t = torch
    if fan_u is not None:
        monkeypatch.setenv("ORL_FAN_U", fan_u)
    n_acc, n_pub = 10_000_000, 1_000_000
    cl = W.default_cluster()
    off, tgt = W.powerlaw_csr(n_acc)
    from orleans_amd.engine import grain_keys_from_longs
    keys = grain_keys_from_longs(cl.type_code, np.arange(n_acc, dtype=np.int64))
    owner = cl.owner_of(W.jenkins3_np(keys["tcd"], keys["n0"], keys["n1"]))
    pubs = (W.stream(W.SEED_C4 ^ 0xB0B, 0, n_pub) % np.uint64(n_acc)).astype(np.uint32)
    deg = np.diff(off.astype(np.int64))
    total = int(deg[pubs].sum())
    eng = GrainDirectoryEngine(n_act=n_acc, dir_capacity=n_acc, max_batch=total + 1, device=0)
    W.setup_engine(eng, cl)
    W.register_population(eng, keys, owner, np.ones(n_acc, bool))
    dv = "cuda"
    poff = t.empty(n_pub + 1, dtype=t.int64, device=dv)
    outs = [t.empty(total, dtype=t.int32, device=dv) for _ in range(3)]
    of = t.empty(n_acc + 2, dtype=t.int32, device=dv)
    tcd = (3 << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)
    got = eng.fanout_device(t.from_numpy(off.view(np.int64)).to(dv), t.from_numpy(tgt.view(np.int32)).to(dv),
                            t.from_numpy(pubs.view(np.int32)).to(dv), t.from_numpy(owner[pubs]).to(dv), n_pub, tcd, poff,
                            *outs, of, stream=t.cuda.current_stream().cuda_stream)
    t.cuda.synchronize()
    assert got == total > 5_000_000
    r, a, od, f = (_u32(x) for x in outs + [of])
    pf = poff.cpu().numpy()
    exp_poff = np.zeros(n_pub + 1, np.int64)
    exp_poff[1:] = np.cumsum(deg[pubs])
    np.testing.assert_array_equal(pf, exp_poff)
    # every emitted follower is a registered account: handle = follower id, host = owner
    fol = np.concatenate([tgt[int(off[p]):int(off[p + 1])] for p in pubs[:1]])  # shape check of the first publisher
    np.testing.assert_array_equal(a[:len(fol)], fol)
    v = decode_route(r)
    assert (v.status == L.ST_HIT).all()
    np.testing.assert_array_equal(v.owner, owner[a.astype(np.int64)])
    check_buckets(a, od, f, n_acc)
    # oracle: whole publishers until >= 1M emitted messages
    k = int(np.searchsorted(exp_poff, 1_000_000)) + 1
    exp, _ = cpu_ref.fanout_expand(off, tgt, pubs[:k], owner[pubs[:k]], tcd)
    o = _oracle_for(cl, keys, np.arange(n_acc, dtype=np.uint32), owner)
    ro, ao = o.route(exp)
    m = len(exp)
    assert m >= 1_000_000
    np.testing.assert_array_equal(r[:m], ro)
    np.testing.assert_array_equal(a[:m], ao)
    eng.close()


# ---- config 5: Presence heartbeats, 64k batches, eager and hipGraph --------------------------------------------
def test_config5_full_size_presence(torch):
    """BASELINE config 5: 100k Guid-keyed games x 8 players, one 64k-heartbeat batch = 64k game messages + 512k
    player messages (fan-out through the player key table), checked in full vs the oracle, eagerly and replayed from a
    captured hipGraph."""
    t = torch
    cl = W.default_cluster()
    n_games, per_game, n_hb = 100_000, 8, 64 * 1024
    pr = W.presence_population(n_games, per_game)
    all_keys = np.concatenate([pr.game_keys, pr.player_keys])
    n_keys = len(all_keys)
    owner = cl.owner_of(W.jenkins3_np(all_keys["tcd"], all_keys["n0"], all_keys["n1"]))
    eng = GrainDirectoryEngine(n_act=n_keys, dir_capacity=n_keys, max_batch=n_hb * per_game, device=0)
    W.setup_engine(eng, cl)
    W.register_population(eng, all_keys, owner, np.ones(n_keys, bool))
    o = _oracle_for(cl, all_keys, np.arange(n_keys, dtype=np.uint32), owner)
    games, gm = W.heartbeat_batch(pr, cl, n_hb, 0)
    gsilo = owner[games.astype(np.int64)]
    exp, poff_ref = cpu_ref.fanout_expand(pr.csr_off, pr.csr_tgt, games, gsilo, 0)
    kk = pr.player_keys[exp["n1"].astype(np.int64)]
    exp["tcd"], exp["n0"], exp["n1"] = kk["tcd"], kk["n0"], kk["n1"]
    r1, a1 = o.route(gm)
    o1, f1 = o.bucket(a1, n_keys)
    r2, a2 = o.route(exp)
    o2, f2 = o.bucket(a2, n_keys)
    dv = "cuda"
    d_gm = t.from_numpy(gm.view(np.int32).reshape(-1, 8)).to(dv)
    d_off = t.from_numpy(pr.csr_off.view(np.int64)).to(dv)
    d_tgt = t.from_numpy(pr.csr_tgt.view(np.int32)).to(dv)
    d_keys = t.from_numpy(pr.player_keys.view(np.uint8).reshape(-1, 24)).to(dv)
    d_g = t.from_numpy(games.view(np.int32)).to(dv)
    d_s = t.from_numpy(gsilo).to(dv)
    n_fan = n_hb * per_game
    g1 = [t.empty(n_hb, dtype=t.int32, device=dv) for _ in range(3)] + [t.empty(n_keys + 2, dtype=t.int32, device=dv)]
    g2 = [t.empty(n_fan, dtype=t.int32, device=dv) for _ in range(3)] + [t.empty(n_keys + 2, dtype=t.int32, device=dv)]
    poff = t.empty(n_hb + 1, dtype=t.int64, device=dv)
    s = t.cuda.Stream()

    def step():
        eng.address_messages_device(d_gm, n_hb, *g1, stream=s.cuda_stream)
        eng.fanout_keys_device(d_off, d_tgt, d_keys, d_g, d_s, n_hb, poff, *g2[:3], g2[3], stream=s.cuda_stream,
                               total=n_fan)

    def check():
        for x, e in zip(g1, (r1, a1, o1, f1)):
            np.testing.assert_array_equal(_u32(x), e)
        for x, e in zip(g2, (r2, a2, o2, f2)):
            np.testing.assert_array_equal(_u32(x), e)
        np.testing.assert_array_equal(poff.cpu().numpy().view(np.uint64), poff_ref)

    with t.cuda.stream(s):
        step()
    s.synchronize()
    check()
    g = t.cuda.CUDAGraph()
    with t.cuda.graph(g, stream=s):
        step()
    for x in g1 + g2:
        x.fill_(-1)
    t.cuda.synchronize()
    with t.cuda.stream(s):
        g.replay()
    s.synchronize()
    check()
    eng.close()


@pytest.mark.parametrize("over", [None, 0, 777])
def test_config5_mixed_batch(torch, over):
    """Config 5 as ONE batch (orl_fanout_route_mixed_device): the 64k game messages then their 512k-message player
    fan-out, routed and bucketed together == the oracle's route + bucket of the concatenated batch; publish offsets
    absolute.  over None: emitted count read back; 0: exact total given (eager + hipGraph replay); 777: total
    overstated, the tail is ORL_ST_PAST_TOTAL in the unresolved bucket."""
    t = torch
    cl = W.default_cluster()
    n_games, per_game, n_hb = 100_000, 8, 64 * 1024
    pr = W.presence_population(n_games, per_game)
    all_keys = np.concatenate([pr.game_keys, pr.player_keys])
    n_keys = len(all_keys)
    owner = cl.owner_of(W.jenkins3_np(all_keys["tcd"], all_keys["n0"], all_keys["n1"]))
    n_fan = n_hb * per_game
    n_tot = n_hb + n_fan
    cap = n_tot + 1024
    eng = GrainDirectoryEngine(n_act=n_keys, dir_capacity=n_keys, max_batch=cap, device=0)
    W.setup_engine(eng, cl)
    W.register_population(eng, all_keys, owner, np.ones(n_keys, bool))
    o = _oracle_for(cl, all_keys, np.arange(n_keys, dtype=np.uint32), owner)
    games, gm = W.heartbeat_batch(pr, cl, n_hb, 1)
    gsilo = owner[games.astype(np.int64)]
    exp, poff_ref = cpu_ref.fanout_expand(pr.csr_off, pr.csr_tgt, games, gsilo, 0)
    kk = pr.player_keys[exp["n1"].astype(np.int64)]
    exp["tcd"], exp["n0"], exp["n1"] = kk["tcd"], kk["n0"], kk["n1"]
    batch = np.concatenate([gm, exp])
    re, ae = o.route(batch)
    n_out = n_tot + (over or 0)
    if over:  # the overstated tail: no message, unresolved bucket
        re = np.concatenate([re, np.full(over, (L.ST_PAST_TOTAL << 16) | 0xFFFF, np.uint32)])
        ae = np.concatenate([ae, np.full(over, L.NO_ACT, np.uint32)])
    oe, fe = o.bucket(ae, n_keys)
    dv = "cuda"
    d_gm = t.from_numpy(gm.view(np.int32).reshape(-1, 8)).to(dv)
    d_off = t.from_numpy(pr.csr_off.view(np.int64)).to(dv)
    d_tgt = t.from_numpy(pr.csr_tgt.view(np.int32)).to(dv)
    d_keys = t.from_numpy(pr.player_keys.view(np.uint8).reshape(-1, 24)).to(dv)
    d_g = t.from_numpy(games.view(np.int32)).to(dv)
    d_s = t.from_numpy(gsilo).to(dv)
    outs = [t.empty(cap, dtype=t.int32, device=dv) for _ in range(3)] + [t.empty(n_keys + 2, dtype=t.int32, device=dv)]
    poff = t.empty(n_hb + 1, dtype=t.int64, device=dv)
    s = t.cuda.Stream()
    total = None if over is None else n_out

    def step():
        return eng.fanout_mixed_device(d_gm, n_hb, d_off, d_tgt, d_keys, 0, d_g, d_s, n_hb, poff, *outs[:3], outs[3],
                                       stream=s.cuda_stream, total=total)

    def check():
        for x, e, m in zip(outs, (re, ae, oe, fe), (n_out, n_out, n_out, n_keys + 2)):
            np.testing.assert_array_equal(_u32(x)[:m], e)
        np.testing.assert_array_equal(poff.cpu().numpy().view(np.uint64), poff_ref + np.uint64(n_hb))

    with t.cuda.stream(s):
        got = step()
    s.synchronize()
    assert got == n_out
    check()
    if over == 0:
        g = t.cuda.CUDAGraph()
        with t.cuda.graph(g, stream=s):
            step()
        for x in outs:
            x.fill_(-1)
        t.cuda.synchronize()
        with t.cuda.stream(s):
            g.replay()
        s.synchronize()
        check()
    eng.close()


@pytest.mark.parametrize("keyed,over", [(False, None), (False, 1000), (True, None)])
def test_fanout_expand_vs_oracle(torch, keyed, over):
    """orl_fanout_expand_device: the emitted headers (publisher-major, CSR order, the publisher's silo, category
    Application) == cpu_ref.fanout_expand, for long-key followers and for a follower key table (Guid players);
    with an overstated total the tail is null, address-complete headers (target silo 0xFF)."""
    t = torch
    cl = W.default_cluster()
    n_acc = 200_000
    off, tgt = W.powerlaw_csr(n_acc, dmax=5000)
    pubs = (W.stream(11, 0, 20_000) % np.uint64(n_acc)).astype(np.uint32)
    psilo = (pubs % 8).astype(np.uint8)
    tcd = (3 << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)
    exp, poff_ref = cpu_ref.fanout_expand(off, tgt, pubs, psilo, tcd)
    fkeys = None
    if keyed:  # Guid-keyed followers: the key table replaces (tcd, 0, id)
        fk = np.zeros(n_acc, L.KEY_DTYPE)
        fk["tcd"] = np.uint64(tcd ^ (1 << 40))
        fk["n0"] = W.stream(12, 0, n_acc)
        fk["n1"] = W.stream(13, 0, n_acc)
        kk = fk[exp["n1"].astype(np.int64)]
        exp["tcd"], exp["n0"], exp["n1"] = kk["tcd"], kk["n0"], kk["n1"]
        fkeys = t.from_numpy(fk.view(np.uint8).reshape(-1, 24)).cuda()
    n = len(exp) + (over or 0)
    eng = GrainDirectoryEngine(n_act=16, dir_capacity=64, max_batch=1 << 20, device=0)
    W.setup_engine(eng, cl)
    dv = "cuda"
    d_out = t.full((n + 64, 8), -1, dtype=t.int32, device=dv)
    poff = t.empty(len(pubs) + 1, dtype=t.int64, device=dv)
    got = eng.fanout_expand_device(t.from_numpy(off.view(np.int64)).to(dv), t.from_numpy(tgt.view(np.int32)).to(dv), fkeys,
                                   tcd, t.from_numpy(pubs.view(np.int32)).to(dv), t.from_numpy(psilo).to(dv), len(pubs), poff,
                                   d_out, n + 64, total=None if over is None else n)
    t.cuda.synchronize()
    assert got == n
    out = d_out.cpu().numpy().view(L.MSG_DTYPE).reshape(-1)
    np.testing.assert_array_equal(out[:len(exp)], exp)
    np.testing.assert_array_equal(poff.cpu().numpy().view(np.uint64), poff_ref)
    if over:
        tail = out[len(exp):n]
        assert (tail["tcd"] == 0).all() and (tail["flags"] == L.HDR_ADDRESS_COMPLETE).all()
        assert (tail["target_silo"] == 0xFF).all() and (tail["sending_silo"] == 0xFF).all()
    assert (out[n:]["tcd"] == np.uint64(0xFFFFFFFFFFFFFFFF)).all()  # nothing written past the total
    with pytest.raises(L.OrleansRouteError):  # more emitted than cap
        eng.fanout_expand_device(t.from_numpy(off.view(np.int64)).to(dv), t.from_numpy(tgt.view(np.int32)).to(dv), fkeys, tcd,
                                 t.from_numpy(pubs.view(np.int32)).to(dv), t.from_numpy(psilo).to(dv), len(pubs), poff, d_out,
                                 len(exp) - 1)
    eng.close()


# ---- stage-4 ranking: the LDS lane-order self-check and the ballot fallback ---------------
@pytest.mark.parametrize("n_act", [5000, 1_000_000, 12_000_000])
def test_stage4_rank_modes_vs_oracle(torch, n_act):
    """The self-check passed on this device (LDS-atomic ranking in use); with the ballot fallback forced, and back,
    stage 4 is bit-exact vs the oracle on uniform, Zipf-hot and single-activation batches (both stage-4 plans)."""
    cl = W.default_cluster()
    n_grains = 50_000
    keys, uni, owner, reg = W.grain_population(cl, n_grains)
    acts = (np.arange(n_grains, dtype=np.uint64) * np.uint64(2654435761) % np.uint64(n_act)).astype(np.uint32)
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=n_grains, max_batch=1 << 21, device=0)
    W.setup_engine(eng, cl)
    eng.register_single_activation(keys, acts, owner)
    o = _oracle_for(cl, keys, acts, owner)
    assert eng.query(L.Q_RANK_MODE) == 0, "the LDS lane-order self-check failed on this device"
    batches = [W.uniform_messages(cl, n_grains + 500, 1_500_000, seed=1),
               W.zipf_messages(cl, n_grains, 1_500_000, seed=2)]
    one = W.uniform_messages(cl, n_grains, 600_000, seed=3)
    one["n1"] = 7  # every message to one activation: whole waves of one digit
    batches.append(one)
    try:
        for mode in (1, 0):
            eng.set_rank_mode(mode)
            assert eng.query(L.Q_RANK_MODE) == mode
            for m in batches:
                res = eng.address_messages(m)
                r, a = o.route(m)
                np.testing.assert_array_equal(res.act, a)
                order, off = o.bucket(a, n_act)
                np.testing.assert_array_equal(res.offsets, off)
                np.testing.assert_array_equal(res.order, order)
    finally:
        eng.set_rank_mode(0)
    eng.close()


@pytest.mark.parametrize("n_act", [5000, 1_000_000])
def test_stage4_skew_hint_vs_oracle(torch, n_act):
    """Unskewed and skewed level-2 plans alternating through the route path (synchronous calls): the fused kernel takes
    the per-bucket form or, on the device's skew flag, the chunked look-back form in the same launch (round 5; until round
    4 a host hint from the previous plan chose the launches).  Every batch of the sequence is bit-exact vs the oracle's
    stable bucketing (ActivationData.cs:483-514)."""
    cl = W.default_cluster()
    n_grains = 50_000
    keys, uni, owner, reg = W.grain_population(cl, n_grains)
    acts = (np.arange(n_grains, dtype=np.uint64) * np.uint64(2654435761) % np.uint64(n_act)).astype(np.uint32)
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=n_grains, max_batch=1 << 21, device=0)
    W.setup_engine(eng, cl)
    eng.register_single_activation(keys, acts, owner)
    o = _oracle_for(cl, keys, acts, owner)
    uni_b = W.uniform_messages(cl, n_grains + 500, 600_000, seed=11)
    one = W.uniform_messages(cl, n_grains, 600_000, seed=12)
    one["n1"] = 9  # one activation: a bucket of ~147 segments (> 64: the skewed plan)
    big = W.uniform_messages(cl, n_grains, 1_200_000, seed=13)
    big["n1"][: 900_000] = 9  # >= 2^20 messages (the hot-key path's pick: counts, then the offsets scan) and skewed
    # hint after each: 0, then solo + direct on a skewed batch, then the chunked form, then solo on a big skewed batch
    for m in (uni_b, one, one, uni_b, uni_b, big, big, uni_b):
        res = eng.address_messages(m)
        r, a = o.route(m)
        np.testing.assert_array_equal(res.act, a)
        order, off = o.bucket(a, n_act)
        np.testing.assert_array_equal(res.offsets, off)
        np.testing.assert_array_equal(res.order, order)
    eng.close()


@pytest.mark.parametrize("n_act", [3_000, 1_000_000, 2_000_000])
def test_stage4_skewed_plans_async_vs_oracle(torch, n_act):
    """stage 4 alone (orl_bucket_device) over a sequence enqueued on ONE stream with no host sync in between,
    alternating small unskewed batches with large skewed ones — several hot activations (buckets of hundreds of segments
    that continue across many look-back chunks), one activation only, a Zipf stream, the unresolved bucket — so no launch
    decision can rely on an earlier batch's result.  n_act 3000: one bucket (no MSD pass; skewed iff the batch has > 64
    segments); 1M: 10 + 10-bit plan; 2M: 11 + 10.  Outputs of every batch bit-exact vs the oracle's stable bucketing
    (ActivationData.EnqueueMessage FIFO, ActivationData.cs:483-514)."""
    t = torch
    rng = np.random.default_rng(n_act + 5)
    o = cpu_ref.Oracle(8)
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=1024, max_batch=3_000_000, device=0)
    W.setup_engine(eng, W.default_cluster())

    def uniform(n):
        return rng.integers(0, n_act, n, dtype=np.int64).astype(np.uint32)

    def hot_mix(n, shares):
        a = uniform(n)
        u = rng.random(n)
        lo = 0.0
        for k, sh in shares:
            a[(u >= lo) & (u < lo + sh)] = k
            lo += sh
        return a

    def zipf(n):
        r = np.minimum(rng.zipf(1.1, n), n_act) - 1
        return ((r.astype(np.uint64) * np.uint64(2654435761)) % np.uint64(n_act)).astype(np.uint32)

    keys = [int(x) for x in rng.integers(0, n_act, 6)]
    batches = [uniform(200_000),
               hot_mix(2_500_000, [(keys[0], 0.30), (keys[1], 0.15), (keys[2], 0.10), (keys[3], 0.05), (keys[4], 0.03)]),
               uniform(150_001),
               np.full(1_100_000, keys[5], np.uint32),                      # one activation: one bucket of ~270 segments
               uniform(300_000),
               zipf(2_000_000),
               hot_mix(700_000, [(L.NO_ACT, 0.5), (keys[0], 0.2)]),        # the unresolved bucket skewed, below 2^20
               uniform(64),
               hot_mix(1_300_000, [(keys[1], 0.6)])]
    s = t.cuda.Stream()
    outs = []
    with t.cuda.stream(s):
        for a in batches:
            d_a = t.from_numpy(a.view(np.int32)).to("cuda", non_blocking=False)
            order = t.empty(len(a), dtype=t.int32, device="cuda")
            off = t.empty(n_act + 2, dtype=t.int32, device="cuda")
            eng.bucket_device(d_a, len(a), order, off, stream=s.cuda_stream)
            outs.append((d_a, order, off))
    s.synchronize()
    for a, (_, order, off) in zip(batches, outs):
        eo, ef = o.bucket(a, n_act)
        np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), ef)
        np.testing.assert_array_equal(order.cpu().numpy().view(np.uint32), eo)
    assert eng.query(L.Q_STAGE4_ERROR) == 0  # no look-back gave up (the fused level 2's error word)
    eng.close()


@pytest.mark.parametrize("n_act", [1_000_000, 2_000_000])
def test_stage4_hot_key_path_vs_oracle(torch, n_act):
    """Stage 4's hot-key path (route_kernels.hip kNoHotKey): a batch of >= 2^20 messages picks its most frequent key when
    it holds >= 1/32 of the batch; the next batch places that key's messages without sorting them.  Every batch, with
    the hot key right, wrong, absent or the unresolved bucket, is bit-exact vs the oracle's stable bucketing
    (ActivationData.EnqueueMessage FIFO, ActivationData.cs:483-514).  n_act 1M: 10 + 10-bit plan; 2M: 11 + 10 (the hot
    rank of config 3 at 8 ranks)."""
    t = torch
    rng = np.random.default_rng(n_act)
    o = cpu_ref.Oracle(8)
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=1024, max_batch=5_000_000, device=0)
    W.setup_engine(eng, W.default_cluster())

    def batch(n, hot=None, share=0.0, unresolved=0.0):
        a = rng.integers(0, n_act, n, dtype=np.int64).astype(np.uint32)
        u = rng.random(n)
        if hot is not None:
            a[u < share] = hot
        a[(u >= share) & (u < share + unresolved)] = L.NO_ACT
        return a

    hot1, hot2 = 123_457 % n_act, n_act - 3
    plan = [(batch(4_000_003, hot1, 0.30), hot1),          # picks hot1
            (batch(3_000_001, hot1, 0.55), hot1),          # uses hot1 (the hot rank's share), picks it again
            (batch(2_500_000, hot2, 0.20), hot2),          # uses hot1 (now rare), picks hot2
            (batch(2_000_000), None),                       # uses hot2 (absent), picks none
            (batch(2_000_000, unresolved=0.10), n_act),     # no hot key; picks the unresolved bucket (misses)
            (batch(1_500_000, unresolved=0.10), n_act),     # uses the unresolved bucket
            (batch(900_000, hot1, 0.9), n_act)]             # below 2^20 messages: no hot path, pick unchanged
    off = t.empty(n_act + 2, dtype=t.int32, device="cuda")
    for k, (a, expect_next) in enumerate(plan):
        d_act = t.from_numpy(a.view(np.int32)).cuda()
        order = t.empty(len(a), dtype=t.int32, device="cuda")
        eng.bucket_device(d_act, len(a), order, off)
        t.cuda.synchronize()
        eo, ef = o.bucket(a, n_act)
        np.testing.assert_array_equal(order.cpu().numpy().view(np.uint32), eo, err_msg=f"batch {k} order")
        np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), ef, err_msg=f"batch {k} offsets")
        nxt = eng.query(L.Q_HOT_KEY)
        assert nxt == (0xFFFFFFFF if expect_next is None else expect_next), (k, nxt)
    # with a sync after every batch the launcher's hint is current: batches 1, 2, 3 and 5 ran the path
    assert eng.query(L.Q_HOT_BATCHES) == 4
    # the same batches enqueued back to back: the launcher's host copy of the pick lags the device (it decides whether a
    # batch runs the path from an earlier batch's pick), which may cost time but never changes a result
    d_acts = [t.from_numpy(a.view(np.int32)).cuda() for a, _ in plan]
    outs = [(t.empty(len(a), dtype=t.int32, device="cuda"), t.empty(n_act + 2, dtype=t.int32, device="cuda"))
            for a, _ in plan]
    for k, (a, _) in enumerate(plan):
        eng.bucket_device(d_acts[k], len(a), outs[k][0], outs[k][1])
    t.cuda.synchronize()
    for k, (a, _) in enumerate(plan):
        eo, ef = o.bucket(a, n_act)
        np.testing.assert_array_equal(outs[k][0].cpu().numpy().view(np.uint32), eo, err_msg=f"queued batch {k} order")
        np.testing.assert_array_equal(outs[k][1].cpu().numpy().view(np.uint32), ef, err_msg=f"queued batch {k} offsets")
    # the route path (stage 4 after k_route's histogram) with misses: 10 % unregistered targets, two batches
    cl = W.default_cluster()
    n_grains = 200_000
    keys, uni, owner, reg = W.grain_population(cl, n_grains, 0.9)
    eng2 = GrainDirectoryEngine(n_act=n_grains, dir_capacity=n_grains, max_batch=3_000_000, device=0)
    W.setup_engine(eng2, cl)
    W.register_population(eng2, keys, owner, reg)
    o2 = _oracle_for(cl, keys[reg], np.nonzero(reg)[0].astype(np.uint32), owner[reg])
    for b in range(2):
        m = W.uniform_messages(cl, n_grains, 2_100_000 + b, seed=77 + b)
        d_in = t.from_numpy(m.view(np.uint8).reshape(-1, 32)).cuda()
        outs = [t.empty(len(m), dtype=t.int32, device="cuda") for _ in range(3)]
        off2 = t.empty(n_grains + 2, dtype=t.int32, device="cuda")
        eng2.address_messages_device(d_in, len(m), *outs, off2)
        t.cuda.synchronize()
        r, a = o2.route(m)
        eo, ef = o2.bucket(a, n_grains)
        np.testing.assert_array_equal(outs[0].cpu().numpy().view(np.uint32), r)
        np.testing.assert_array_equal(outs[1].cpu().numpy().view(np.uint32), a)
        np.testing.assert_array_equal(outs[2].cpu().numpy().view(np.uint32), eo, err_msg=f"route batch {b} order")
        np.testing.assert_array_equal(off2.cpu().numpy().view(np.uint32), ef)
        assert eng2.query(L.Q_HOT_KEY) == n_grains  # the unresolved bucket (PreferLocal placements) is hot
    eng2.close()
    eng.close()


@pytest.mark.parametrize("rank_mode", ["hot", "plain", "ballot"])
def test_stage4_level2_edges_vs_oracle(torch, monkeypatch, rank_mode):
    """Stage 4's two-level plan (MSD pass + segmented level 2) in every ranking variant, on the shapes its level-2 records
    depend on: uniform buckets; one digit with tens of thousands of messages in a bucket; a bucket of 100k messages next to
    small ones; a sparse bucket whose messages are five million positions apart (its level-2 records span many
    super-tiles); the hot-key path with its key in a small and in a large bucket; n_act + 1 == 2^20 (the key past the last
    bucket); tiny and all-unresolved batches.  Order and offsets == the oracle's stable bucketing
    (ActivationData.EnqueueMessage, ActivationData.cs:483-514)."""
    t = torch
    if rank_mode == "plain":
        monkeypatch.setenv("ORL_RANK_UNIFORM", "0")
    o = cpu_ref.Oracle(8)
    for n_act in (1_000_000, (1 << 20) - 1):
        rng = np.random.default_rng(n_act + len(rank_mode))
        eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=1024, max_batch=7_000_000, device=0)
        W.setup_engine(eng, W.default_cluster())
        eng.set_rank_mode(1 if rank_mode == "ballot" else 0)

        def uni(n, lo=0, hi=n_act):
            return rng.integers(lo, hi, n, dtype=np.int64).astype(np.uint32)

        def put(a, key, count):  # `count` messages of `key` at random positions
            a[rng.choice(len(a), count, replace=False)] = key
            return a

        sparse = uni(6_000_000, 0, 500_000)
        sparse[:100] = n_act - 5                   # the bucket of n_act - 5: 100 messages at the start ...
        sparse[5_000_000:5_000_100] = n_act - 5    # ... and 100 five million positions later
        big_bucket = put(uni(4_000_000), 77, 100_000)   # bucket 0: ~100k messages, many segments
        hot_seg = put(put(uni(4_000_000), 5 * 1024 + 9, 1_300_000), 5 * 1024 + 3, 100_000)
        plan = [uni(3_000_000),
                put(put(uni(4_000_000), 5 * 1024 + 7, 15_000), 6 * 1024 + 1, 30_000),  # heavy digits
                big_bucket,
                sparse,
                put(uni(4_000_000), 123_457, 1_300_000),   # picks 123457 (a small bucket's digit)
                put(uni(4_000_000), 123_457, 1_200_000),   # ... and uses it
                hot_seg,                                   # picks 5*1024+9 (its bucket: > 1.4M messages)
                put(hot_seg.copy(), 5 * 1024 + 3, 1),      # uses it; its bucket holds 100k more of 5*1024+3
                uni(1000),
                np.full(1_100_000, L.NO_ACT, np.uint32),
                np.array([n_act - 1], np.uint32)]
        off = t.empty(n_act + 2, dtype=t.int32, device="cuda")
        for k, a in enumerate(plan):
            d_act = t.from_numpy(a.view(np.int32)).cuda()
            order = t.empty(len(a), dtype=t.int32, device="cuda")
            off.fill_(-1)
            eng.bucket_device(d_act, len(a), order, off)
            t.cuda.synchronize()
            eo, ef = o.bucket(a, n_act)
            np.testing.assert_array_equal(_u32(order), eo, err_msg=f"n_act {n_act} batch {k} order")
            np.testing.assert_array_equal(_u32(off), ef, err_msg=f"n_act {n_act} batch {k} offsets")
            if k in (4, 5):
                assert eng.query(L.Q_HOT_KEY) == 123_457
            if k in (6, 7):
                assert eng.query(L.Q_HOT_KEY) == 5 * 1024 + 9
        assert eng.query(L.Q_HOT_BATCHES) >= 2
        eng.set_rank_mode(0)
        eng.close()


# ---- stage 4, LSD plan (keys > 22 bits): bucket offsets from the gaps between sorted keys -----------------------
@pytest.mark.parametrize("cap", [None, "3"])
def test_lsd_offsets_long_gaps_vs_oracle(torch, monkeypatch, cap):
    """The LSD plan's bucket offsets (k_offsets_gaps / k_offsets_long): every empty bucket gets lower_bound(sorted, b).
    Batches over 20M handles with short gaps only (uniform), gaps the whole wave writes (sparse keys), gaps queued in
    32768-bucket pieces (a few keys: millions of empty buckets between them, before the first and after the last) and, with
    the queue capped at 3 pieces (ORL_GAP_CAP), the full-queue fallback where the wave writes what did not fit; the
    offsets-only form (no messages) and a batch whose keys are all unresolved.  Order and offsets == the oracle's stable
    bucketing (ActivationData.cs:483-514)."""
    t = torch
    if cap is not None:
        monkeypatch.setenv("ORL_GAP_CAP", cap)
    n_act = 20_000_000
    rng = np.random.default_rng(11)
    o = cpu_ref.Oracle(8)
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=1024, max_batch=1 << 21, device=0)
    W.setup_engine(eng, W.default_cluster())
    batches = [rng.integers(0, n_act, 1_500_000, dtype=np.int64).astype(np.uint32),          # gaps of ~13
               rng.integers(0, n_act // 40, 300_000, dtype=np.int64).astype(np.uint32) * 40,  # gaps of 39 and more
               rng.choice(np.array([5, 6, 9_000_123, 9_000_124, 12_345_678], np.uint32), 700_001),
               np.full(1000, n_act - 1, np.uint32),
               np.full(5000, L.NO_ACT, np.uint32),
               np.array([n_act // 2], np.uint32)]
    off = t.empty(n_act + 2, dtype=t.int32, device="cuda")
    for k, a in enumerate(batches):
        d_act = t.from_numpy(a.view(np.int32)).cuda()
        order = t.empty(len(a), dtype=t.int32, device="cuda")
        off.fill_(-1)
        eng.bucket_device(d_act, len(a), order, off)
        t.cuda.synchronize()
        eo, ef = o.bucket(a, n_act)
        np.testing.assert_array_equal(_u32(order), eo, err_msg=f"batch {k} order")
        np.testing.assert_array_equal(_u32(off), ef, err_msg=f"batch {k} offsets")
    eng.close()


@pytest.mark.parametrize("lsd_hot", ["0", "1"])
def test_lsd_fused_offsets_dense_vs_oracle(torch, monkeypatch, lsd_hot):
    """The LSD plan's last pass writing the bucket offsets itself (round 6: OUT_FINAL_GAPS + k_bound_last / k_bound_scan /
    k_bound_apply + k_sweep_tail), taken when a batch has >= 2 messages per bucket (config 3's shape; sparser batches keep
    k_offsets_gaps).  n_act 8.5M (24-bit keys: 8 + 8 + 8-bit digits), batches of 18-20M messages: uniform, Zipf-hot (one key
    with millions of messages), a few keys with millions of empty buckets between and around them, the unresolved bucket,
    keys only in the low half, and the digit stream (OUT_PAIR_DIG) feeding each later histogram.  Order and offsets == the
    oracle's stable bucketing (ActivationData.cs:483-514).  (The sparse form: test_lsd_offsets_long_gaps_vs_oracle.)  Batches
    of one shape come in pairs: with the LSD hot-key path on (ORL_LSD_HOT=1 at context creation: opt-in) the
    second takes it on the key the first picked (ORL_Q_HOT_BATCHES)."""
    t = torch
    n_act = 8_500_000
    n = 2 * (n_act + 2) + 1000
    rng = np.random.default_rng(17)
    o = cpu_ref.Oracle(8)

    def zipf(k):
        r = np.minimum(rng.zipf(1.1, k), n_act) - 1
        return ((r.astype(np.uint64) * np.uint64(2654435761)) % np.uint64(n_act)).astype(np.uint32)

    few = np.array([3, 4, 4_000_000, 4_000_001, 8_400_000], np.uint32)
    unres = lambda: np.where(rng.random(n) < 0.3, np.uint32(L.NO_ACT), zipf(n)).astype(np.uint32)  # noqa: E731
    # consecutive batches of one shape: the second runs the hot-key path (round 6) on the key the first one picked —
    # Zipf's top key (keys above and below it), one of a few keys, the unresolved bucket (the largest key)
    batches = [rng.integers(0, n_act, n, dtype=np.int64).astype(np.uint32),
               zipf(n), zipf(n),
               rng.choice(few, n), rng.choice(few, n),
               unres(), unres(),
               rng.integers(0, n_act // 2, n, dtype=np.int64).astype(np.uint32)]
    monkeypatch.setenv("ORL_LSD_HOT", lsd_hot)  # read at context creation
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=1024, max_batch=n, device=0)
    monkeypatch.delenv("ORL_LSD_HOT")
    W.setup_engine(eng, W.default_cluster())
    off = t.empty(n_act + 2, dtype=t.int32, device="cuda")
    order = t.empty(n, dtype=t.int32, device="cuda")
    for k, a in enumerate(batches):
        d_act = t.from_numpy(a.view(np.int32)).cuda()
        off.fill_(-1)
        order.fill_(-1)
        eng.bucket_device(d_act, len(a), order, off)
        t.cuda.synchronize()
        eo, ef = o.bucket(a, n_act)
        np.testing.assert_array_equal(_u32(order), eo, err_msg=f"batch {k} order")
        np.testing.assert_array_equal(_u32(off), ef, err_msg=f"batch {k} offsets")
    if lsd_hot == "1":
        assert eng.query(L.Q_HOT_BATCHES) >= 3  # the second batch of each pair ran the hot-key path
    else:
        assert eng.query(L.Q_HOT_BATCHES) == 0
    eng.close()


@pytest.mark.parametrize("n_act", [12_000_000, 40_000_000])
def test_lsd_sweep_async_vs_oracle(torch, monkeypatch, n_act):
    """The LSD plan's single-sweep passes (round 6: k_digit_hist, one k_sweep per digit with a decoupled look-back, the
    final pass writing the bucket offsets itself, k_sweep_tail).  A sequence of batches enqueued on ONE stream with no host
    sync in between, so the look-back ring and its ticket words are reused launch after launch at every size: large and
    small, Zipf-hot (a digit with millions of messages), one activation, the unresolved bucket, sparse keys (long empty
    gaps, digits with no message), one message.  Each batch bit-exact vs the oracle's stable bucketing
    (ActivationData.EnqueueMessage FIFO, ActivationData.cs:483-514) and equal to the default k_hist_pairs form (the sweep
    is opt-in, ORL_LSD_SWEEP=1: slower on MI355X); then the same stage 4 captured in a hipGraph and replayed (the launch base lives on the device,
    so a replay needs no host state).  n_act 12M: 8 + 8 + 8-bit digits; 40M: 9 + 9 + 8."""
    t = torch
    rng = np.random.default_rng(n_act + 1)
    o = cpu_ref.Oracle(8)

    def zipf(n):
        r = np.minimum(rng.zipf(1.1, n), n_act) - 1
        return ((r.astype(np.uint64) * np.uint64(2654435761)) % np.uint64(n_act)).astype(np.uint32)

    batches = [rng.integers(0, n_act, 2_500_000, dtype=np.int64).astype(np.uint32),
               zipf(3_000_001),
               rng.integers(0, n_act, 4097, dtype=np.int64).astype(np.uint32),
               np.full(700_000, n_act // 3, np.uint32),
               rng.integers(0, 300, 200_000, dtype=np.int64).astype(np.uint32) * np.uint32(n_act // 301),  # sparse
               np.where(rng.random(1_000_000) < 0.4, np.uint32(L.NO_ACT), zipf(1_000_000)).astype(np.uint32),
               np.array([n_act - 1], np.uint32),
               zipf(2_000_000)]
    monkeypatch.setenv("ORL_LSD_SWEEP", "1")  # opt-in (slower on MI355X: DESIGN §4)
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=1024, max_batch=3_100_000, device=0)
    monkeypatch.delenv("ORL_LSD_SWEEP")
    W.setup_engine(eng, W.default_cluster())
    ref = GrainDirectoryEngine(n_act=n_act, dir_capacity=1024, max_batch=3_100_000, device=0)
    W.setup_engine(ref, W.default_cluster())
    s = t.cuda.Stream()
    d_acts = [t.from_numpy(a.view(np.int32)).cuda() for a in batches]
    outs, routs = [], []
    with t.cuda.stream(s):
        for d_a in d_acts:
            for e, acc in ((eng, outs), (ref, routs)):
                order = t.full((len(d_a),), -1, dtype=t.int32, device="cuda")
                off = t.full((n_act + 2,), -1, dtype=t.int32, device="cuda")
                e.bucket_device(d_a, len(d_a), order, off, stream=s.cuda_stream)
                acc.append((order, off))
    s.synchronize()
    for k, a in enumerate(batches):
        eo, ef = o.bucket(a, n_act)
        np.testing.assert_array_equal(_u32(outs[k][1]), ef, err_msg=f"batch {k} offsets")
        np.testing.assert_array_equal(_u32(outs[k][0]), eo, err_msg=f"batch {k} order")
        np.testing.assert_array_equal(_u32(routs[k][1]), ef, err_msg=f"batch {k} offsets (k_hist_pairs form)")
        np.testing.assert_array_equal(_u32(routs[k][0]), eo, err_msg=f"batch {k} order (k_hist_pairs form)")
    assert eng.query(L.Q_STAGE4_ERROR) == 0
    # the Zipf batch captured once, replayed three times (zeroed outputs between), then an eager batch of another size
    order, off = outs[1]
    g = t.cuda.CUDAGraph()
    with t.cuda.graph(g, stream=s):
        eng.bucket_device(d_acts[1], len(batches[1]), order, off, stream=s.cuda_stream)
    eo, ef = o.bucket(batches[1], n_act)
    for _ in range(3):
        order.fill_(0)
        off.fill_(0)
        g.replay()
        t.cuda.synchronize()
        np.testing.assert_array_equal(_u32(off), ef, err_msg="graph replay offsets")
        np.testing.assert_array_equal(_u32(order), eo, err_msg="graph replay order")
    order2, off2 = outs[0]
    eng.bucket_device(d_acts[0], len(batches[0]), order2, off2)
    t.cuda.synchronize()
    eo, ef = o.bucket(batches[0], n_act)
    np.testing.assert_array_equal(_u32(off2), ef, err_msg="eager after replays: offsets")
    np.testing.assert_array_equal(_u32(order2), eo, err_msg="eager after replays: order")
    assert eng.query(L.Q_STAGE4_ERROR) == 0
    ref.close()
    eng.close()
