"""GPU parity: the HIP path (through the C ABI) against the oracle, bit for bit.

Sizes the oracle finishes in seconds run message-for-message; the full config-2 batch (64M messages)
is checked per message on a random sample plus size-independent properties of the bucketing (a
permutation, stable, grouped, offsets consistent).  All integer/byte work: exact equality, no tolerance.
"""
import json
import os

import numpy as np
import pytest

from oracle import cpu_ref, pyref as P
from orleans_amd import _lib as L
from orleans_amd import workloads as W
from orleans_amd.engine import GrainDirectoryEngine, decode_route

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def _pair(d, max_batch=1 << 20, n_act=None):
    n = len(d["silo_hashes"])
    n_act = int(d["n_act"]) if n_act is None else n_act
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=max(16, len(d["reg_keys"])), max_batch=max_batch, device=0,
                               placement=int(d["policy"]))
    eng.set_silos(n, running=d["running"], functional=d["functional"], seed=int(d["seed"]))
    for s in range(n):
        eng.add_server(s, int(d["silo_hashes"][s]))
    keys = np.zeros(len(d["reg_keys"]), L.KEY_DTYPE)
    keys["tcd"], keys["n0"], keys["n1"] = d["reg_keys"][:, 0], d["reg_keys"][:, 1], d["reg_keys"][:, 2]
    eng.register_single_activation(keys, d["reg_acts"], d["reg_silos"])
    return eng


def test_hash_batch_golden(torch, golden_dir):
    g = json.load(open(os.path.join(golden_dir, "jenkins.json")))
    keys = np.zeros(len(g["keys"]) + len(g["u64"]), L.KEY_DTYPE)
    exp = np.zeros(len(keys), np.uint32)
    for i, c in enumerate(g["keys"]):
        keys[i] = (int(c["tcd"], 16), int(c["n0"], 16), int(c["n1"], 16))
        exp[i] = c["uniform"]
    for j, c in enumerate(g["u64"]):
        keys[len(g["keys"]) + j] = tuple(int(x, 16) for x in c["u"])
        exp[len(g["keys"]) + j] = c["hash"]
    eng = GrainDirectoryEngine(n_act=4, dir_capacity=16, device=0)
    np.testing.assert_array_equal(eng.hash_batch(keys), exp)
    rng = np.random.default_rng(3)
    rk = rng.integers(0, 2**63, (100_000, 3), dtype=np.int64).view(np.uint64)
    kk = np.zeros(len(rk), L.KEY_DTYPE)
    kk["tcd"], kk["n0"], kk["n1"] = rk[:, 0], rk[:, 1], rk[:, 2]
    np.testing.assert_array_equal(eng.hash_batch(kk), W.jenkins3_np(kk["tcd"], kk["n0"], kk["n1"]))
    eng.close()


@pytest.mark.parametrize("name", ["routing_basic", "routing_membership"])
def test_routing_golden(torch, golden_dir, name):
    d = np.load(os.path.join(golden_dir, name + ".npz"))
    eng = _pair(d)
    msgs = d["msgs"].reshape(-1).view(L.MSG_DTYPE)
    res = eng.address_messages(msgs, int(d["opts"]))
    np.testing.assert_array_equal(res.route, d["route"])
    np.testing.assert_array_equal(res.act, d["act"])
    np.testing.assert_array_equal(res.order, d["order"])
    np.testing.assert_array_equal(res.offsets, d["offsets"])
    eng.close()


def test_chirper_fanout_golden(torch, golden_dir):
    d = np.load(os.path.join(golden_dir, "chirper_fanout.npz"))
    cl = W.default_cluster()
    ids = d["node_ids"]
    eng = GrainDirectoryEngine(n_act=len(ids), dir_capacity=len(ids), max_batch=1 << 16, device=0)
    W.setup_engine(eng, cl)
    keys = np.zeros(len(ids), L.KEY_DTYPE)
    keys["tcd"] = np.uint64(int(d["follower_tcd"]))
    keys["n1"] = ids.astype(np.uint64)
    owner = cl.owner_of(W.jenkins3_np(keys["tcd"], keys["n0"], keys["n1"]))
    st, _, _ = eng.register_single_activation(keys, np.arange(len(ids), dtype=np.uint32), owner)
    assert (st == L.INS_INSERTED).all()
    dev = "cuda"
    t = torch
    csr_off = t.from_numpy(d["csr_off"].astype(np.int64)).to(dev)
    csr_tgt = t.from_numpy(d["csr_tgt"].astype(np.int32)).to(dev)
    pubs = t.from_numpy(d["pubs"].astype(np.int32)).to(dev)
    psilo = t.from_numpy(d["pub_silo"]).to(dev)
    n_exp = len(d["route"])
    poff = t.empty(len(d["pubs"]) + 1, dtype=t.int64, device=dev)
    route = t.empty(n_exp, dtype=t.int32, device=dev)
    act = t.empty(n_exp, dtype=t.int32, device=dev)
    order = t.empty(n_exp, dtype=t.int32, device=dev)
    off = t.empty(len(ids) + 2, dtype=t.int32, device=dev)
    stream = t.cuda.current_stream().cuda_stream
    n = eng.fanout_device(csr_off, csr_tgt, pubs, psilo, len(d["pubs"]), int(d["follower_tcd"]), poff, route, act,
                          order, off, stream=stream)
    t.cuda.synchronize()
    assert n == n_exp
    np.testing.assert_array_equal(route.cpu().numpy().view(np.uint32), d["route"])
    np.testing.assert_array_equal(act.cpu().numpy().view(np.uint32), d["act"])
    np.testing.assert_array_equal(order.cpu().numpy().view(np.uint32), d["order"])
    np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), d["offsets"])
    exp_poff = np.zeros(len(d["pubs"]) + 1, np.uint64)
    exp_poff[1:] = np.cumsum(np.diff(d["csr_off"].astype(np.int64))[d["pubs"]])
    np.testing.assert_array_equal(poff.cpu().numpy().view(np.uint64), exp_poff)
    eng.close()


def _random_setup(n_grains, n_act, n_silos=8, seed=11, functional=None, running=None, policy=0, n_registered=None):
    cl = W.default_cluster(n_silos)
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=n_grains, max_batch=1 << 20, device=0, placement=policy)
    eng.set_silos(n_silos, running=running, functional=functional, seed=0)
    o = cpu_ref.Oracle(n_silos, running=running, functional=functional, seed=0, policy=policy)
    for s in range(n_silos):
        eng.add_server(s, int(cl.hashes[s]))
        o.add_server(s, int(cl.hashes[s]))
    keys, uni, owner, reg = W.grain_population(cl, n_grains, 0.9, seed)
    rng = np.random.default_rng(seed)
    acts = rng.integers(0, n_act, n_grains).astype(np.uint32)  # handles may collide: many grains, one bucket
    silos = np.where(rng.random(n_grains) < 0.8, owner, rng.integers(0, n_silos, n_grains)).astype(np.uint8)
    idx = np.nonzero(reg)[0]
    st_e, wa_e, _ = eng.register_single_activation(keys[idx], acts[idx], silos[idx])
    st_o, wa_o, _ = o.register(keys[idx], acts[idx], silos[idx])
    np.testing.assert_array_equal(st_e, st_o)
    return cl, eng, o


@pytest.mark.parametrize("n", [0, 1, 63, 4095, 4096, 4097, 65536 + 17, 300_001])
@pytest.mark.parametrize("n_act", [1, 5, 2048, 5000, 3_000_000, 12_000_000, 40_000_000])
def test_random_batches_vs_oracle(torch, n, n_act):
    cl, eng, o = _random_setup(20_000, n_act)
    msgs = W.uniform_messages(cl, 22_000, n, seed=n * 7 + n_act)  # ~9% never-registered targets
    for opts in (0, L.OPT_EXCLUDE_IF_STOPPING):
        res = eng.address_messages(msgs, opts)
        r, a = o.route(msgs, opts)
        np.testing.assert_array_equal(res.route, r)
        np.testing.assert_array_equal(res.act, a)
        order, off = o.bucket(a, n_act)
        np.testing.assert_array_equal(res.offsets, off)
        np.testing.assert_array_equal(res.order, order)
    eng.close()


def test_membership_variants_vs_oracle(torch):
    running = [1, 0, 1, 1, 0, 1, 1, 1]
    functional = [1, 1, 0, 1, 1, 1, 0, 1]
    for policy in (L.POLICY_PREFER_LOCAL, L.POLICY_HASH_SPREAD):
        cl, eng, o = _random_setup(5000, 6000, running=running, functional=functional, policy=policy)
        msgs = W.zipf_messages(cl, 6000, 200_000, seed=5)
        for opts in (0, L.OPT_EXCLUDE_IF_STOPPING):
            res = eng.address_messages(msgs, opts)
            r, a = o.route(msgs, opts)
            np.testing.assert_array_equal(res.route, r)
            np.testing.assert_array_equal(res.act, a)
        # ring shrinks (RemoveServer) between batches: snapshot semantics
        eng.remove_server(3)
        o.remove_server(3)
        res = eng.address_messages(msgs)
        r, a = o.route(msgs)
        np.testing.assert_array_equal(res.route, r)
        eng.close()


def test_single_silo_ring_and_empty_ring(torch):
    for n_ring in (0, 1):
        eng = GrainDirectoryEngine(n_act=64, dir_capacity=64, device=0)
        eng.set_silos(2, running=[0, 1])
        o = cpu_ref.Oracle(2, running=[0, 1])
        if n_ring:
            eng.add_server(0, 5)
            o.add_server(0, 5)
        m = np.zeros(100, L.MSG_DTYPE)
        m["tcd"] = P.CAT_GRAIN << 56
        m["n1"] = np.arange(100)
        m["sending_silo"] = np.arange(100) % 2
        for opts in (0, 1):
            res = eng.address_messages(m, opts)
            r, a = o.route(m, opts)
            np.testing.assert_array_equal(res.route, r)
        eng.close()


def test_partition_by_owner_vs_oracle(torch):
    cl, eng, o = _random_setup(10_000, 10_000)
    t = torch
    for nranks in (1, 2, 4, 8):
        ros = cl.rank_of_silo(nranks)
        for my_rank in range(nranks):
            msgs = W.uniform_messages(cl, 11_000, 100_003, seed=my_rank)
            msgs["flags"][::97] = L.HDR_ADDRESS_COMPLETE
            d_in = t.from_numpy(msgs.view(np.uint8).reshape(-1, 32)).cuda()
            d_out = t.empty_like(d_in)
            d_src = t.empty(len(msgs), dtype=t.int32, device="cuda")
            d_cnt = t.empty(nranks, dtype=t.int64, device="cuda")
            eng.partition_by_owner_device(d_in, len(msgs), ros, nranks, my_rank, d_out, d_src, d_cnt,
                                          stream=t.cuda.current_stream().cuda_stream)
            t.cuda.synchronize()
            src, cnt = o.partition(msgs, ros, nranks, my_rank)
            np.testing.assert_array_equal(d_cnt.cpu().numpy(), cnt.astype(np.int64))
            np.testing.assert_array_equal(d_src.cpu().numpy().view(np.uint32), src)
            np.testing.assert_array_equal(d_out.cpu().numpy().reshape(-1).view(L.MSG_DTYPE), msgs[src])
    eng.close()


def test_partition_padded_vs_oracle(torch):
    """One-pass owner partition (decoupled look-back) into padded per-rank regions == the oracle's partition,
    region by region, for 1..8 ranks, ragged tile tails, complete-address messages, with and without the
    source-index output; plus a 24M-message batch (11.7k tiles of look-back) checked for counts + stability."""
    cl, eng, o = _random_setup(10_000, 10_000)
    t = torch
    for n in (0, 1, 2047, 2049, 100_003):
        for nranks in (1, 2, 3, 8):
            ros = cl.rank_of_silo(nranks) if nranks != 3 else np.array([s % 3 for s in range(8)], np.uint8)
            my_rank = (n + nranks) % nranks
            msgs = W.uniform_messages(cl, 11_000, n, seed=my_rank + n)
            msgs["flags"][::97] = L.HDR_ADDRESS_COMPLETE
            stride = n + 5
            d_in = t.from_numpy(msgs.view(np.uint8).reshape(-1, 32)).cuda()
            d_out = t.full((nranks * stride, 32), 0xEE, dtype=t.uint8, device="cuda")
            d_src = t.full((nranks * stride,), -1, dtype=t.int32, device="cuda")
            d_cnt = t.full((nranks,), -1, dtype=t.int64, device="cuda")
            eng.partition_by_owner_padded_device(d_in, n, ros, nranks, my_rank, stride, d_out, d_cnt, d_src,
                                                 stream=t.cuda.current_stream().cuda_stream)
            t.cuda.synchronize()
            src, cnt = o.partition(msgs, ros, nranks, my_rank)
            np.testing.assert_array_equal(d_cnt.cpu().numpy(), cnt.astype(np.int64))
            out = d_out.cpu().numpy().reshape(-1).view(L.MSG_DTYPE)
            srcs = d_src.cpu().numpy().view(np.uint32)
            o0 = 0
            for r in range(nranks):
                c = int(cnt[r])
                np.testing.assert_array_equal(out[r * stride:r * stride + c], msgs[src[o0:o0 + c]])
                np.testing.assert_array_equal(srcs[r * stride:r * stride + c], src[o0:o0 + c])
                assert (srcs[r * stride + c:(r + 1) * stride] == 0xFFFFFFFF).all()  # nothing past the count
                o0 += c
    # large: many look-back tiles, no source index
    n, nranks = 24_000_000, 8
    ros = cl.rank_of_silo(nranks)
    msgs = W.uniform_messages(cl, 11_000, n, seed=5)
    d_in = t.from_numpy(msgs.view(np.uint8).reshape(-1, 32)).cuda()
    eng2 = GrainDirectoryEngine(n_act=1, dir_capacity=1, max_batch=n, device=0)
    W.setup_engine(eng2, cl)
    d_out = t.empty((nranks * n, 32), dtype=t.uint8, device="cuda")
    d_cnt = t.empty((nranks,), dtype=t.int64, device="cuda")
    for rep in range(2):
        eng2.partition_by_owner_padded_device(d_in, n, ros, nranks, 3, n, d_out, d_cnt,
                                              stream=t.cuda.current_stream().cuda_stream)
    t.cuda.synchronize()
    owner = decode_route(o.route(msgs[:2_000_000])[0]).owner
    cnt = d_cnt.cpu().numpy()
    assert cnt.sum() == n
    dest = ros[owner.astype(np.int64)]
    for r in range(nranks):  # the first 2M messages' share of each region is its head, in order
        exp = msgs[:2_000_000][dest == r]
        got = d_out[r * n:r * n + len(exp)].cpu().numpy().reshape(-1).view(L.MSG_DTYPE)
        np.testing.assert_array_equal(got, exp)
    eng2.close()
    eng.close()


def test_compact_wire_partition_and_route(torch):
    """16-B exchange records: the one-pass partition's compact regions == the oracle's partition encoded by the
    oracle's codec; the status word flags a batch with a non-compact message; routing the compact records
    == routing the 32-B headers (route, act, order, offsets)."""
    cl, eng, o = _random_setup(10_000, 10_000)
    t = torch
    st = t.cuda.current_stream().cuda_stream
    for n, nranks in ((0, 2), (1, 1), (4097, 3), (100_003, 8)):
        ros = cl.rank_of_silo(nranks) if nranks != 3 else np.array([s % 3 for s in range(8)], np.uint8)
        msgs = W.uniform_messages(cl, 11_000, n, seed=n)
        msgs["flags"][::89] = L.HDR_ADDRESS_COMPLETE
        msgs["target_silo"][::89] = 3
        msgs["category"][::7] = 1
        d_in = t.from_numpy(msgs.view(np.uint8).reshape(-1, 32)).cuda()
        stride = n + 3
        d_out = t.empty((nranks * stride, 16), dtype=t.uint8, device="cuda")
        d_cnt = t.empty(nranks, dtype=t.int64, device="cuda")
        d_st = t.full((1,), 7, dtype=t.int32, device="cuda")
        eng.partition_compact_device(d_in, n, ros, nranks, 0, stride, d_out, d_cnt, d_st, stream=st)
        t.cuda.synchronize()
        assert int(d_st.item()) == 0
        src, cnt = o.partition(msgs, ros, nranks, 0)
        np.testing.assert_array_equal(d_cnt.cpu().numpy(), cnt.astype(np.int64))
        exp, ok = cpu_ref.wire_encode(msgs[src])
        assert ok.all()
        out = d_out.cpu().numpy().reshape(-1).view(cpu_ref.WIRE_DTYPE)
        o0 = 0
        for r in range(nranks):
            c = int(cnt[r])
            np.testing.assert_array_equal(out[r * stride:r * stride + c], exp[o0:o0 + c])
            o0 += c
        if n == 0:
            continue
        # route the compact records == route the headers
        recs, _ = cpu_ref.wire_encode(msgs)
        d_recs = t.from_numpy(recs.view(np.uint8).reshape(-1, 16)).cuda()
        outs = [t.empty(n, dtype=t.int32, device="cuda") for _ in range(3)] + [t.empty(10_002, dtype=t.int32, device="cuda")]
        eng.address_compact_device(d_recs, n, *outs, stream=st)
        t.cuda.synchronize()
        got = [x.cpu().numpy().view(np.uint32) for x in outs]
        r_ref, a_ref = o.route(msgs)
        np.testing.assert_array_equal(got[0], r_ref)
        np.testing.assert_array_equal(got[1], a_ref)
        o_ref, f_ref = o.bucket(a_ref, 10_000)
        np.testing.assert_array_equal(got[2], o_ref)
        np.testing.assert_array_equal(got[3], f_ref)
    # a non-compact message anywhere in the batch sets the status word
    for field, val in (("n0", 1), ("flags", L.HDR_HASH_VALID), ("tcd", (3 << 56) | 0x0000123412345678)):
        msgs = W.uniform_messages(cl, 11_000, 5000, seed=3)
        msgs[field][4321] = val
        d_in = t.from_numpy(msgs.view(np.uint8).reshape(-1, 32)).cuda()
        d_out = t.empty((2 * 5000, 16), dtype=t.uint8, device="cuda")
        d_cnt = t.empty(2, dtype=t.int64, device="cuda")
        d_st = t.zeros((1,), dtype=t.int32, device="cuda")
        eng.partition_compact_device(d_in, 5000, cl.rank_of_silo(2), 2, 1, 5000, d_out, d_cnt, d_st, stream=st)
        t.cuda.synchronize()
        assert int(d_st.item()) == 1, field
        assert not cpu_ref.wire_encode(msgs)[1].all()
    eng.close()


def test_narrow_wire_partition_and_route(torch):
    """8-B exchange records (orl_wire8): the one-pass partition's regions == the oracle's partition encoded by the
    oracle's narrow codec; the status word's bits say which forms a batch lacks; routing the 8-B records == routing
    the 32-B headers (route, act, order, offsets)."""
    cl, eng, o = _random_setup(10_000, 10_000)
    t = torch
    st = t.cuda.current_stream().cuda_stream
    grain_t = (L.CAT_GRAIN << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)
    sys_t = (L.CAT_SYSTEM_TARGET << 56) | 12
    types = [sys_t, grain_t]  # the grain type at index 1: the index is carried, not assumed
    with pytest.raises(L.OrleansRouteError):  # no wire types yet: the 8-B form is off
        eng.partition_narrow_device(t.zeros(32, dtype=t.uint8, device="cuda"), 1, cl.rank_of_silo(1), 1, 0, 1,
                                    t.empty(16, dtype=t.uint8, device="cuda"), t.empty(1, dtype=t.int64, device="cuda"),
                                    t.empty(1, dtype=t.int32, device="cuda"), stream=st)
    eng.set_wire_types(types)
    assert eng.query(L.Q_WIRE_DIGEST) != 0
    for n, nranks in ((0, 2), (1, 1), (4097, 3), (100_003, 8)):
        ros = cl.rank_of_silo(nranks) if nranks != 3 else np.array([s % 3 for s in range(8)], np.uint8)
        msgs = W.uniform_messages(cl, 11_000, n, seed=n)
        msgs["flags"][::89] = L.HDR_ADDRESS_COMPLETE
        msgs["target_silo"][::89] = 3
        msgs["category"][::7] = 1
        msgs["tcd"][5::97] = sys_t
        d_in = t.from_numpy(msgs.view(np.uint8).reshape(-1, 32)).cuda()
        stride = n + 3
        d_out = t.empty((nranks * stride, 8), dtype=t.uint8, device="cuda")
        d_cnt = t.empty(nranks, dtype=t.int64, device="cuda")
        d_st = t.full((1,), 7, dtype=t.int32, device="cuda")
        eng.partition_narrow_device(d_in, n, ros, nranks, 0, stride, d_out, d_cnt, d_st, stream=st)
        t.cuda.synchronize()
        assert int(d_st.item()) == 0
        src, cnt = o.partition(msgs, ros, nranks, 0)
        np.testing.assert_array_equal(d_cnt.cpu().numpy(), cnt.astype(np.int64))
        exp, ok = cpu_ref.narrow_encode(msgs[src], types)
        assert ok.all()
        out = d_out.cpu().numpy().reshape(-1).view(cpu_ref.WIRE8_DTYPE)
        o0 = 0
        for r in range(nranks):
            c = int(cnt[r])
            np.testing.assert_array_equal(out[r * stride:r * stride + c], exp[o0:o0 + c])
            o0 += c
        if n == 0:
            continue
        recs, _ = cpu_ref.narrow_encode(msgs, types)
        d_recs = t.from_numpy(recs.view(np.uint8).reshape(-1, 8)).cuda()
        outs = [t.empty(n, dtype=t.int32, device="cuda") for _ in range(3)] + [t.empty(10_002, dtype=t.int32, device="cuda")]
        eng.address_narrow_device(d_recs, n, *outs, stream=st)
        t.cuda.synchronize()
        got = [x.cpu().numpy().view(np.uint32) for x in outs]
        r_ref, a_ref = o.route(msgs)
        np.testing.assert_array_equal(got[0], r_ref)
        np.testing.assert_array_equal(got[1], a_ref)
        o_ref, f_ref = o.bucket(a_ref, 10_000)
        np.testing.assert_array_equal(got[2], o_ref)
        np.testing.assert_array_equal(got[3], f_ref)
    # status bits: bit 1 = a message without the 8-B form, bit 0 = also without the 16-B form
    for field, val, want in (("n1", 1 << 32, 2), ("tcd", grain_t + 1, 2), ("n0", 1, 3), ("flags", L.HDR_HASH_VALID, 3),
                             ("tcd", (3 << 56) | 0x0000123412345678, 3)):
        msgs = W.uniform_messages(cl, 11_000, 5000, seed=3)
        msgs[field][4321] = val
        d_in = t.from_numpy(msgs.view(np.uint8).reshape(-1, 32)).cuda()
        d_out = t.empty((2 * 5000, 8), dtype=t.uint8, device="cuda")
        d_cnt = t.empty(2, dtype=t.int64, device="cuda")
        d_st = t.zeros((1,), dtype=t.int32, device="cuda")
        eng.partition_narrow_device(d_in, 5000, cl.rank_of_silo(2), 2, 1, 5000, d_out, d_cnt, d_st, stream=st)
        t.cuda.synchronize()
        assert int(d_st.item()) == want, (field, val)
        assert not cpu_ref.narrow_encode(msgs, types)[1].all()
    eng.set_wire_types([])
    assert eng.query(L.Q_WIRE_DIGEST) == 0
    eng.close()


@pytest.mark.parametrize("reg_frac", [1.0, 0.9])
def test_config2_full_size_properties(torch, reg_frac):
    """BASELINE config 2 at full size (1M grains, 64M messages) on the device-resident path; reg_frac = 0.9 is SURVEY
    §8(d)'s "10 % unregistered" variant: a tenth of the targets miss the directory and are placed on the sending silo
    (PreferLocalPlacementDirector.OnAddActivation, PreferLocalPlacementDirector.cs:38-44, via Dispatcher.AddressMessage,
    Dispatcher.cs:555-579), and go to the unresolved bucket n_act."""
    t = torch
    n_grains, n = 1_000_000, 64 * 1024 * 1024
    cl = W.default_cluster()
    eng = GrainDirectoryEngine(n_act=n_grains, dir_capacity=n_grains, max_batch=n, device=0)
    W.setup_engine(eng, cl)
    keys, uni, owner, reg = W.grain_population(cl, n_grains, reg_frac)
    W.register_population(eng, keys, owner, reg)
    msgs = W.uniform_messages(cl, n_grains, n)
    d_in = t.from_numpy(msgs.view(np.uint8).reshape(-1, 32)).cuda()
    route = t.empty(n, dtype=t.int32, device="cuda")
    act = t.empty(n, dtype=t.int32, device="cuda")
    order = t.empty(n, dtype=t.int32, device="cuda")
    off = t.empty(n_grains + 2, dtype=t.int32, device="cuda")
    eng.address_messages_device(d_in, n, route, act, order, off, stream=t.cuda.current_stream().cuda_stream)
    t.cuda.synchronize()
    a = act.cpu().numpy().view(np.uint32)
    r = route.cpu().numpy().view(np.uint32)
    od = order.cpu().numpy().view(np.uint32)
    of = off.cpu().numpy().view(np.uint32).astype(np.int64)
    tgt = msgs["n1"].astype(np.int64)
    hit = reg[tgt]
    if reg_frac < 1.0:
        assert 0.09 < 1.0 - hit.mean() < 0.11, hit.mean()
    # a registered target's handle is its key (activation on the directory owner); a miss is placed on the sender
    v = decode_route(r)
    np.testing.assert_array_equal(a[hit], tgt[hit].astype(np.uint32))
    assert (v.status[hit] == L.ST_HIT).all()
    np.testing.assert_array_equal(v.owner, owner[tgt])
    np.testing.assert_array_equal(v.host[hit], v.owner[hit])
    assert (v.status[~hit] == L.ST_NEW_PLACEMENT).all()
    np.testing.assert_array_equal(v.host[~hit], msgs["sending_silo"][~hit])
    assert (a[~hit] == L.NO_ACT).all()
    # per-message oracle on a 1M random sample
    o = cpu_ref.Oracle(8)
    for s in range(8):
        o.add_server(s, int(cl.hashes[s]))
    idx = np.nonzero(reg)[0]
    o.register(keys[idx], idx.astype(np.uint32), owner[idx])
    samp = np.sort(np.random.default_rng(0).choice(n, 1_000_000, replace=False))
    ro, ao = o.route(msgs[samp])
    np.testing.assert_array_equal(r[samp], ro)
    np.testing.assert_array_equal(a[samp], ao)
    # bucketing: offsets = exclusive cumsum of per-activation counts (misses: bucket n_act); order groups, stable
    key = np.minimum(a, n_grains).astype(np.int64)
    cnt = np.bincount(key, minlength=n_grains + 1)
    exp_off = np.zeros(n_grains + 2, np.int64)
    exp_off[1:] = np.cumsum(cnt)
    np.testing.assert_array_equal(of, exp_off)
    assert (np.bincount(od, minlength=n) == 1).all()            # permutation
    srt = key[od]
    assert (np.diff(srt) >= 0).all()                            # grouped by activation
    same = np.diff(srt) == 0
    assert (np.diff(od.astype(np.int64))[same] > 0).all()       # arrival order kept inside a bucket
    eng.close()


def test_presence_keyed_fanout_and_graph_capture(torch):
    """Config-5 shape (small): Guid-keyed games fan out to 8 Guid-keyed players through a device key table
    (GameGrain.UpdateGameStatus, Samples/Presence/PresenceGrains/GameGrain.cs:62-113), bit-exact vs the oracle;
    the sync-free form (ORL_OPT_TOTAL_GIVEN) replayed from a captured graph gives the same words."""
    t = torch
    cl = W.default_cluster()
    pr = W.presence_population(2000, 8)
    all_keys = np.concatenate([pr.game_keys, pr.player_keys])
    n_keys = len(all_keys)
    owner = cl.owner_of(W.jenkins3_np(all_keys["tcd"], all_keys["n0"], all_keys["n1"]))
    reg = np.random.default_rng(5).random(n_keys) < 0.9  # some players unregistered: new placements
    eng = GrainDirectoryEngine(n_act=n_keys, dir_capacity=n_keys, max_batch=1 << 16, device=0)
    W.setup_engine(eng, cl)
    W.register_population(eng, all_keys, owner, reg)
    o = cpu_ref.Oracle(cl.n_silos)
    for s in range(cl.n_silos):
        o.add_server(s, int(cl.hashes[s]))
    idx = np.nonzero(reg)[0]
    o.register(all_keys[idx], idx.astype(np.uint32), owner[idx])
    games, _ = W.heartbeat_batch(pr, cl, 3000, 0)
    gsilo = owner[games.astype(np.int64)]
    # oracle: expand in CSR order, then name each follower by the key table
    exp, poff_ref = cpu_ref.fanout_expand(pr.csr_off, pr.csr_tgt, games, gsilo, 0)
    k = pr.player_keys[exp["n1"].astype(np.int64)]
    exp["tcd"], exp["n0"], exp["n1"] = k["tcd"], k["n0"], k["n1"]
    r_ref, a_ref = o.route(exp)
    o_ref, f_ref = o.bucket(a_ref, n_keys)
    dev = "cuda"
    d_off = t.from_numpy(pr.csr_off.view(np.int64)).to(dev)
    d_tgt = t.from_numpy(pr.csr_tgt.view(np.int32)).to(dev)
    d_keys = t.from_numpy(pr.player_keys.view(np.uint8).reshape(-1, 24)).to(dev)
    d_g = t.from_numpy(games.view(np.int32)).to(dev)
    d_s = t.from_numpy(gsilo).to(dev)
    n = len(exp)
    poff = t.empty(len(games) + 1, dtype=t.int64, device=dev)
    outs = [t.full((n,), -7, dtype=t.int32, device=dev) for _ in range(3)]
    off = t.empty(n_keys + 2, dtype=t.int32, device=dev)
    s = t.cuda.Stream()
    got = eng.fanout_keys_device(d_off, d_tgt, d_keys, d_g, d_s, len(games), poff, *outs, off, stream=s.cuda_stream)
    s.synchronize()
    assert got == n
    np.testing.assert_array_equal(outs[0].cpu().numpy().view(np.uint32), r_ref)
    np.testing.assert_array_equal(outs[1].cpu().numpy().view(np.uint32), a_ref)
    np.testing.assert_array_equal(outs[2].cpu().numpy().view(np.uint32), o_ref)
    np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), f_ref)
    np.testing.assert_array_equal(poff.cpu().numpy().view(np.uint64), poff_ref)
    # sync-free form under graph capture, outputs cleared before replay
    for x in outs:
        x.fill_(-7)
    g = t.cuda.CUDAGraph()
    with t.cuda.graph(g, stream=s):
        eng.fanout_keys_device(d_off, d_tgt, d_keys, d_g, d_s, len(games), poff, *outs, off, stream=s.cuda_stream,
                               total=n)
    for x in outs:
        x.fill_(-7)
    t.cuda.synchronize()
    g.replay()
    t.cuda.synchronize()
    np.testing.assert_array_equal(outs[0].cpu().numpy().view(np.uint32), r_ref)
    np.testing.assert_array_equal(outs[2].cpu().numpy().view(np.uint32), o_ref)
    np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), f_ref)
    eng.close()


def test_route_batch_graph_replay(torch):
    """A captured orl_route_batch_device replays to the same words as the eager call (config-5 hipGraph path)."""
    t = torch
    cl, eng, o = _random_setup(5000, 6000)
    msgs = W.uniform_messages(cl, 5500, 70_000, seed=77)
    d_in = t.from_numpy(msgs.view(np.int32).reshape(-1, 8)).cuda()
    n = len(msgs)
    outs = [t.empty(n, dtype=t.int32, device="cuda") for _ in range(3)]
    off = t.empty(6002, dtype=t.int32, device="cuda")
    s = t.cuda.Stream()
    eng.address_messages_device(d_in, n, *outs, off, stream=s.cuda_stream)
    s.synchronize()
    ref = [x.cpu().numpy().copy() for x in outs] + [off.cpu().numpy().copy()]
    g = t.cuda.CUDAGraph()
    with t.cuda.graph(g, stream=s):
        eng.address_messages_device(d_in, n, *outs, off, stream=s.cuda_stream)
    for x in outs + [off]:
        x.fill_(0)
    t.cuda.synchronize()
    for _ in range(3):
        g.replay()
    t.cuda.synchronize()
    for a, b in zip(ref, [x.cpu().numpy() for x in outs] + [off.cpu().numpy()]):
        np.testing.assert_array_equal(a, b)
    eng.close()


def test_device_directory_mutation_vs_oracle(torch):
    """batched RegisterSingleActivation / Unregister on the device table == the oracle applying
    the same batches one message at a time (statuses, winners, removed flags), then routing over the mutated
    directory == the oracle's.  Batches carry duplicate keys (first writer wins), re-registrations after
    removal, invalid silos, remote owners (two local silos), system targets and the membership grain."""
    t = torch
    cl = W.default_cluster()
    local = [1, 0, 0, 1, 0, 0, 0, 0]
    functional = [1, 1, 1, 1, 1, 0, 1, 1]
    n_grains, n_act = 60_000, 50_000
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=n_grains, max_batch=1 << 20, device=0)
    eng.set_silos(8, functional=functional, local=local, seed=3)
    o = cpu_ref.Oracle(8, functional=functional, local=local, seed=3)
    for s in range(8):
        eng.add_server(s, int(cl.hashes[s]))
        o.add_server(s, int(cl.hashes[s]))
    keys_all, _, owner, _ = W.grain_population(cl, n_grains)
    rng = np.random.default_rng(7)
    st_ = t.cuda.current_stream().cuda_stream

    def dev(a):
        return t.from_numpy(np.ascontiguousarray(a).view(np.uint8)).cuda()

    for rnd in range(4):
        m = 40_000
        pick = rng.integers(0, n_grains, m)
        hot = rng.random(m) < 0.2  # a fifth of the batch re-targets 500 hot grains: many duplicates per batch
        pick[hot] = rng.integers(0, 500, int(hot.sum()))
        keys = keys_all[pick].copy()
        keys[::997]["tcd"] = (np.uint64(L.CAT_SYSTEM_TARGET) << np.uint64(56)) | np.uint64(7)
        acts = rng.integers(0, n_act, m).astype(np.uint32)
        silos = np.where(rng.random(m) < 0.7, owner[pick], rng.integers(0, 8, m)).astype(np.uint8)
        d_st = t.empty(m, dtype=t.uint8, device="cuda")
        d_wa = t.empty(m, dtype=t.int32, device="cuda")
        d_ws = t.empty(m, dtype=t.uint8, device="cuda")
        eng.register_single_activation_device(dev(keys), dev(acts), dev(silos), m, d_st, d_wa, d_ws, stream=st_)
        t.cuda.synchronize()
        st_o, wa_o, ws_o = o.register(keys, acts, silos)
        np.testing.assert_array_equal(d_st.cpu().numpy(), st_o)
        np.testing.assert_array_equal(d_wa.cpu().numpy().view(np.uint32), wa_o)
        np.testing.assert_array_equal(d_ws.cpu().numpy(), ws_o)
        assert (st_o == L.INS_INSERTED).sum() > 1000 and (st_o == L.INS_EXISTING).sum() > 100, np.bincount(st_o)
        # remove a random subset (with duplicates) on the device and in the oracle
        rm = keys_all[rng.integers(0, n_grains, 15_000)]
        d_rm = t.empty(len(rm), dtype=t.uint8, device="cuda")
        eng.unregister_device(dev(rm), len(rm), d_rm, stream=st_)
        t.cuda.synchronize()
        np.testing.assert_array_equal(d_rm.cpu().numpy(), o.unregister(rm))
        assert eng.directory_count() == o.size()
        # routing over the mutated directory
        msgs = W.uniform_messages(cl, n_grains, 100_000, seed=rnd)
        res = eng.address_messages(msgs)
        r_ref, a_ref = o.route(msgs)
        np.testing.assert_array_equal(res.route, r_ref)
        np.testing.assert_array_equal(res.act, a_ref)
    # compaction drops the tombstones and keeps every live entry
    eng.compact_directory()
    assert eng.directory_count() == o.size()
    msgs = W.uniform_messages(cl, n_grains, 50_000, seed=99)
    np.testing.assert_array_equal(eng.address_messages(msgs).route, o.route(msgs)[0])
    # host-side registration after device mutations sees the device table (the mirror is re-read)
    k = keys_all[:1000]
    st_h, wa_h, _ = eng.register_single_activation(k, np.arange(1000, dtype=np.uint32), owner[:1000])
    st_o, wa_o, _ = o.register(k, np.arange(1000, dtype=np.uint32), owner[:1000])
    np.testing.assert_array_equal(st_h, st_o)
    np.testing.assert_array_equal(wa_h, wa_o)
    eng.close()


def test_device_handoff_split_on_silo_add(torch):
    """Membership change (GrainDirectoryHandoffManager.ProcessSiloAddEvent): a silo joins inside
    our ring arc; the device split emits exactly the entries whose owner under the new ring is another silo and
    whose activation silo is valid, tombstones them here, and the joining silo registers them; afterwards each
    silo's partition routes its keys exactly as the single-view oracle does."""
    t = torch
    cl = W.default_cluster()
    new = 7
    ring7 = sorted((int(cl.hashes[s]), s) for s in range(7))
    h_new = int(cl.hashes[new])
    me = max([p for p in ring7 if p[0] <= h_new], default=ring7[-1])[1]  # the arc that silo 7 lands in
    functional = [1] * 8
    functional[5] = 0  # silo 5 dies before the join: its entries are not handed off (ToListOfActivations: IsValidSilo)
    n_grains = 200_000
    keys, _, _, _ = W.grain_population(cl, n_grains)
    eng_a = GrainDirectoryEngine(n_act=n_grains, dir_capacity=n_grains, max_batch=1 << 20, device=0)
    eng_a.set_silos(8, local=[int(s == me) for s in range(8)])
    for s in range(7):
        eng_a.add_server(s, int(cl.hashes[s]))
    o7 = cpu_ref.Oracle(8, functional=functional)
    for s in range(7):
        o7.add_server(s, int(cl.hashes[s]))
    msgs_all = np.zeros(n_grains, L.MSG_DTYPE)
    msgs_all["tcd"], msgs_all["n1"] = keys["tcd"], keys["n1"]
    msgs_all["sending_silo"] = me
    owner7 = decode_route(o7.route(msgs_all)[0]).owner
    mine = np.nonzero(owner7 == me)[0]
    rng = np.random.default_rng(3)
    acts = np.arange(n_grains, dtype=np.uint32)
    silos = np.where(rng.random(n_grains) < 0.1, 5, me).astype(np.uint8)
    st, _, _ = eng_a.register_single_activation(keys[mine], acts[mine], silos[mine])
    assert (st == L.INS_INSERTED).all()
    reg = mine
    # silo 5 stops being functional, then silo 7 joins
    eng_a.set_silos(8, functional=functional, local=[int(s == me) for s in range(8)])
    eng_a.add_server(new, h_new)
    o8 = cpu_ref.Oracle(8, functional=functional)
    for s in range(8):
        o8.add_server(s, int(cl.hashes[s]))
    owner8 = decode_route(o8.route(msgs_all)[0]).owner
    exp = reg[(owner8[reg] != me) & (owner8[reg] != 0xFF) & (silos[reg] != 5)]
    assert len(exp) > 100, len(exp)  # silo 7 takes 0.4 % of the ring (generation-1 hashes)
    cap = len(reg)
    d_k = t.empty((cap, 24), dtype=t.uint8, device="cuda")
    d_a = t.empty(cap, dtype=t.int32, device="cuda")
    d_s = t.empty(cap, dtype=t.uint8, device="cuda")
    d_n = t.zeros(1, dtype=t.int64, device="cuda")
    eng_a.split_directory_device(me, d_k, d_a, d_s, cap, d_n, remove=True, stream=t.cuda.current_stream().cuda_stream)
    t.cuda.synchronize()
    n_out = int(d_n.item())
    assert n_out == len(exp)
    got_k = d_k[:n_out].cpu().numpy().reshape(-1).view(L.KEY_DTYPE)
    got_a = d_a[:n_out].cpu().numpy().view(np.uint32)
    assert sorted(got_a.tolist()) == sorted(exp.tolist())
    np.testing.assert_array_equal(got_k, keys[got_a])
    np.testing.assert_array_equal(d_s[:n_out].cpu().numpy(), silos[got_a])
    assert eng_a.directory_count() == len(reg) - n_out
    # the joining silo registers the hand-off (RegisterManySingleActivation) on its device table
    eng_b = GrainDirectoryEngine(n_act=n_grains, dir_capacity=n_grains, max_batch=1 << 20, device=0)
    eng_b.set_silos(8, functional=functional, local=[int(s == new) for s in range(8)])
    for s in range(8):
        eng_b.add_server(s, int(cl.hashes[s]))
    d_st = t.empty(n_out, dtype=t.uint8, device="cuda")
    eng_b.register_single_activation_device(d_k[:n_out], d_a[:n_out], d_s[:n_out], n_out, d_st,
                                            stream=t.cuda.current_stream().cuda_stream)
    t.cuda.synchronize()
    assert (d_st.cpu().numpy() == L.INS_INSERTED).all()
    # each silo's view routes its keys like the oracle holding both partitions under the 8-silo ring (the
    # silo-5 entries stayed in A's partition; IsValidSilo filters them from lookups on both sides)
    kept = reg[(silos[reg] != 5) | (owner8[reg] == me)]
    o8.register(keys[kept], acts[kept], np.where(silos[kept] == 5, me, silos[kept]).astype(np.uint8))
    probe = msgs_all[reg[silos[reg] != 5]]
    reg = reg[silos[reg] != 5]
    ref_r, ref_a = o8.route(probe)
    for eng, silo in ((eng_a, me), (eng_b, new)):
        sel = owner8[reg] == silo
        res = eng.address_messages(probe[sel])
        np.testing.assert_array_equal(res.route, ref_r[sel])
        np.testing.assert_array_equal(res.act, ref_a[sel])
    eng_a.close()
    eng_b.close()


def test_stream_reminder_rings_vs_oracle(torch):
    """ring-owner lookups on the device (ConsistentRingProvider over the directory ring,
    VirtualBucketsRingProvider over 30 buckets per silo) and stream → queue (+ pulling silo) mapping, against
    the pure-Python restatement, for running and stopping `me` with and without excludeThisSiloIfStopping."""
    t = torch
    n_silos = 12
    running = [1] * n_silos
    running[4] = 0
    eng = GrainDirectoryEngine(n_act=4, dir_capacity=16, max_batch=1024, device=0)
    eng.set_silos(n_silos, running=running)
    vr = P.VirtualBucketsRing()
    ring = P.Ring()
    for s in range(n_silos):
        ip = bytes(12) + bytes([10, 0, 0, s + 1])
        eng.vring_add_server(s, ip, 11111, 7 + s)
        vr.add_server(s, ip, 11111, 7 + s)
        h = P.silo_consistent_hash(f"10.0.0.{s + 1}:11111", 7 + s)
        eng.add_server(s, h)
        ring.add_server(s, h)
    eng.vring_remove_server(9)
    vr.remove_server(9)
    rng = np.random.default_rng(5)
    bucket_keys = np.array([h for h, _ in vr.sorted_list()], np.uint32)
    keys = np.concatenate([rng.integers(0, 1 << 32, 6000, dtype=np.uint64).astype(np.uint32), bucket_keys,
                           bucket_keys + 1, np.array([0, 1, 0xFFFFFFFF], np.uint32)])
    d_keys = t.from_numpy(keys.view(np.int32)).cuda()
    d_own = t.empty(len(keys), dtype=t.uint8, device="cuda")
    st = t.cuda.current_stream().cuda_stream
    for me in (0, 4):
        for opts in (0, L.OPT_EXCLUDE_IF_STOPPING):
            excl = bool(opts) and not running[me]
            for kind in (L.RING_CONSISTENT, L.RING_VBUCKETS):
                eng.ring_owner_device(kind, d_keys, len(keys), me, d_own, opts=opts, stream=st)
                t.cuda.synchronize()
                got = d_own.cpu().numpy()
                if kind == L.RING_VBUCKETS:
                    exp = [vr.target(int(k), me, excl) for k in keys]
                else:
                    exp = [P.consistent_ring_target(ring, int(k), me, excl) for k in keys]
                np.testing.assert_array_equal(got, np.array(exp, np.uint8), err_msg=f"kind {kind} me {me} opts {opts}")
    # stream → queue (+ the silo whose range holds the queue)
    guids = rng.integers(0, 256, (5000, 16), dtype=np.uint8)
    d_g = t.from_numpy(guids).cuda()
    d_q = t.empty(len(guids), dtype=t.int32, device="cuda")
    d_s = t.empty(len(guids), dtype=t.uint8, device="cuda")
    for nq in (1, 3, 8, 256, 65535):
        eng.stream_queue_device(L.RING_VBUCKETS, d_g, len(guids), nq, 0, d_q, d_s, stream=st)
        t.cuda.synchronize()
        exp_q = np.array([P.stream_queue_for_guid(bytes(g), nq) for g in guids], np.uint32)
        np.testing.assert_array_equal(d_q.cpu().numpy().view(np.uint32), exp_q)
        qh = P.stream_queue_hashes(nq)
        exp_s = np.array([vr.target(qh[q], 0, False) for q in exp_q], np.uint8)
        np.testing.assert_array_equal(d_s.cpu().numpy(), exp_s)
    eng.close()


def test_outbound_queues_and_client_buckets_vs_oracle(torch):
    """OutboundMessageQueue.SendMessage queue selection per routed message (reject, loopback,
    ping / system senders, Math.Abs(hash) % senders incl. the int.MinValue overflow, unknown silo) and the client's
    GetHashCode_Modulo gateway buckets (incl. KeyExt precomputed hashes), against the pure-Python restatement."""
    t = torch
    cl = W.default_cluster()
    eng = GrainDirectoryEngine(n_act=4, dir_capacity=16, max_batch=1024, device=0)
    eng.set_silos(12)
    hashes = {s: int(cl.hashes[s]) for s in range(8)}
    for s in range(8):
        eng.add_server(s, hashes[s])
    hashes[9] = -(1 << 31)   # Math.Abs(int.MinValue) overflows
    hashes[10] = -12345
    eng.set_silo_hash(9, hashes[9])
    eng.set_silo_hash(10, hashes[10])  # silo 11: never given → unknown
    rng = np.random.default_rng(11)
    n = 50_000
    msgs = W.uniform_messages(cl, 100_000, n, seed=8)
    msgs["category"] = rng.integers(0, 3, n)
    msgs["sending_silo"] = rng.integers(0, 12, n)
    kx = rng.random(n) < 0.1
    msgs["flags"][kx] |= L.HDR_HASH_VALID
    msgs["aux"][kx] = rng.integers(0, 1 << 32, int(kx.sum()), dtype=np.uint64).astype(np.uint32)
    host = rng.integers(0, 13, n)
    host[host == 12] = 0xFF
    route = (host.astype(np.uint32) << 8) | np.uint32(L.ST_HIT << 16)
    d_m = t.from_numpy(msgs.view(np.uint8).reshape(-1, 32)).cuda()
    d_r = t.from_numpy(route.view(np.int32)).cuda()
    d_q = t.empty(n, dtype=t.int32, device="cuda")
    st = t.cuda.current_stream().cuda_stream
    for ns in (1, 3, 8):
        eng.outbound_queues_device(d_m, d_r, n, ns, d_q, stream=st)
        t.cuda.synchronize()
        exp = np.array([P.outbound_queue(int(host[i]), int(msgs["sending_silo"][i]), int(msgs["category"][i]), hashes, ns)
                        for i in range(n)], np.uint32)
        np.testing.assert_array_equal(d_q.cpu().numpy().view(np.uint32), exp)
    uni = np.where(kx, msgs["aux"], W.jenkins3_np(msgs["tcd"], msgs["n0"], msgs["n1"])).astype(np.uint32)
    for nb in (1, 7, 100, 1 << 30):
        eng.client_buckets_device(d_m, n, nb, d_q, stream=st)
        t.cuda.synchronize()
        exp = np.array([P.client_bucket(int(u), nb) for u in uni], np.uint32)
        np.testing.assert_array_equal(d_q.cpu().numpy().view(np.uint32), exp)
    eng.close()


def test_directory_cache_in_route_vs_oracle(torch):
    """the device directory cache answers LocalLookup for remote-owned grains (HIT | CACHED, the
    cached silo as host; entries on invalid silos filtered; misses stay REMOTE_OWNER), AddOrUpdate keeps the batch's
    last writer, invalidation removes, and stage 4 buckets cached activations by their handle — all equal to the
    oracle (C++ restatement + pyref.apply_directory_cache)."""
    t = torch
    cl = W.default_cluster()
    local = [1, 1, 0, 0, 0, 0, 0, 0]
    functional = [1, 1, 1, 1, 1, 1, 0, 1]
    n_grains, n_act = 50_000, 60_000
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=n_grains, max_batch=1 << 20, device=0)
    eng.set_silos(8, functional=functional, local=local)
    o = cpu_ref.Oracle(8, functional=functional, local=local)
    for s in range(8):
        eng.add_server(s, int(cl.hashes[s]))
        o.add_server(s, int(cl.hashes[s]))
    keys, _, owner, _ = W.grain_population(cl, n_grains)
    mine = np.nonzero(np.isin(owner, [0, 1]))[0]
    eng.register_single_activation(keys[mine], mine.astype(np.uint32), owner[mine])
    o.register(keys[mine], mine.astype(np.uint32), owner[mine])
    eng.cache_config(40_000)
    rng = np.random.default_rng(2)
    remote = np.nonzero(~np.isin(owner, [0, 1]))[0]
    cache = {}
    st_ = t.cuda.current_stream().cuda_stream

    def dev(a):
        return t.from_numpy(np.ascontiguousarray(a).view(np.uint8)).cuda()

    msgs = W.uniform_messages(cl, n_grains, 200_000, seed=4)
    kt = list(zip(msgs["tcd"].tolist(), msgs["n0"].tolist(), msgs["n1"].tolist()))
    for rnd in range(3):
        pick = rng.choice(remote, 20_000)   # duplicates within the batch: the last writer wins
        # handles [50000, 70000): the half >= n_act is kept only for a silo this context does not host (the host's catalog
        # numbers it; since round 5, VERDICT r5 item 1 / ADVICE r5) — such a HIT | CACHED message lands in the unresolved
        # bucket n_act of this context's stage 4; on a local silo it is dropped (outside the local handle space)
        acts = (50_000 + rng.integers(0, 20_000, len(pick))).astype(np.uint32)
        silos = rng.integers(0, 8, len(pick)).astype(np.uint8)
        eng.cache_add_or_update_device(dev(keys[pick]), dev(acts), dev(silos), len(pick), stream=st_)
        for g, a, s in zip(pick.tolist(), acts.tolist(), silos.tolist()):
            if a < n_act or not local[s]:
                cache[(int(keys["tcd"][g]), int(keys["n0"][g]), int(keys["n1"][g]))] = (a, s)
        inval = rng.choice(remote, 3000)
        d_rm = t.empty(len(inval), dtype=t.uint8, device="cuda")
        eng.cache_remove_device(dev(keys[inval]), len(inval), d_rm, stream=st_)
        t.cuda.synchronize()
        for g in inval.tolist():
            cache.pop((int(keys["tcd"][g]), int(keys["n0"][g]), int(keys["n1"][g])), None)
        assert eng.cache_count() == len(cache)
        res = eng.address_messages(msgs)
        r0, a0 = o.route(msgs)
        r_ref, a_ref = P.apply_directory_cache(r0.tolist(), a0.tolist(), msgs["sending_silo"].tolist(), kt, cache,
                                               functional)
        np.testing.assert_array_equal(res.route, np.array(r_ref, np.uint32))
        np.testing.assert_array_equal(res.act, np.array(a_ref, np.uint32))
        o_ref, f_ref = o.bucket(np.array(a_ref, np.uint32), n_act)
        np.testing.assert_array_equal(res.order, o_ref)
        np.testing.assert_array_equal(res.offsets, f_ref)
        assert ((res.route >> 24) & L.RF_CACHED).sum() > 1000
        big = (((res.route >> 24) & L.RF_CACHED) != 0) & (res.act >= n_act)
        assert big.sum() > 500  # cached handles of another silo's catalog, >= this context's n_act
        assert (res.offsets[n_act + 1] - res.offsets[n_act]) >= big.sum()  # ... bucketed as unresolved here
    eng.cache_clear()
    np.testing.assert_array_equal(eng.address_messages(msgs).route, o.route(msgs)[0])
    eng.close()


def test_directory_cache_lru_eviction_vs_oracle(torch):
    """the directory cache evicts like the reference's instead of refusing (AdaptiveGrainDirectoryCache
    .AddOrUpdate → LRU.Add → AdjustSize frees the entry of the smallest generation while Count >= MaximumSize; every
    LookUp hit takes the next generation: AdaptiveGrainDirectoryCache.cs:97-133, LRU.cs:104-108,147-174,188-205).  A cache of
    3000 entries goes through add batches that fit (the device path), overflow it (the exact LRU on the host), update keys
    — the least recently used among them — at full capacity, outgrow it within one batch, lose entries by invalidation;
    between them route batches whose remote-owner lookups reorder the LRU.  After every step the cached count and every
    routed word / handle / bucket equal oracle/pyref.LRUCache fed the same sequence (lookups in message order)."""
    t = torch
    cl = W.default_cluster()
    local = [1, 1, 0, 0, 0, 0, 0, 0]
    functional = [1, 1, 1, 1, 1, 1, 0, 1]
    n_grains, n_act, cap = 50_000, 60_000, 3000
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=n_grains, max_batch=1 << 20, device=0)
    eng.set_silos(8, functional=functional, local=local)
    o = cpu_ref.Oracle(8, functional=functional, local=local)
    for s in range(8):
        eng.add_server(s, int(cl.hashes[s]))
        o.add_server(s, int(cl.hashes[s]))
    keys, _, owner, _ = W.grain_population(cl, n_grains)
    mine = np.nonzero(np.isin(owner, [0, 1]))[0]
    eng.register_single_activation(keys[mine], mine.astype(np.uint32), owner[mine])
    o.register(keys[mine], mine.astype(np.uint32), owner[mine])
    eng.cache_config(cap)
    lru = P.LRUCache(cap)
    rng = np.random.default_rng(9)
    remote = np.nonzero(~np.isin(owner, [0, 1]))[0]
    st_ = t.cuda.current_stream().cuda_stream
    kt_all = [(int(a), int(b), int(c)) for a, b, c in zip(keys["tcd"], keys["n0"], keys["n1"])]

    def dev(a):
        return t.from_numpy(np.ascontiguousarray(a).view(np.uint8)).cuda()

    def add(pick):
        acts = (50_000 + rng.integers(0, 20_000, len(pick))).astype(np.uint32)
        silos = rng.integers(0, 8, len(pick)).astype(np.uint8)
        eng.cache_add_or_update_device(dev(keys[pick]), dev(acts), dev(silos), len(pick), stream=st_)
        for g, a, s in zip(pick.tolist(), acts.tolist(), silos.tolist()):
            if a < n_act or not local[s]:  # what the device keeps (k_cache_probe)
                lru.add(kt_all[g], (a, s))
        t.cuda.synchronize()
        assert eng.cache_count() == len(lru.d), (eng.cache_count(), len(lru.d))

    def route(seed, n=60_000):
        msgs = W.uniform_messages(cl, n_grains, n, seed=seed)
        kt = list(zip(msgs["tcd"].tolist(), msgs["n0"].tolist(), msgs["n1"].tolist()))
        res = eng.address_messages(msgs)
        r0, a0 = o.route(msgs)
        r_ref, a_ref = P.apply_directory_cache_lru(r0.tolist(), a0.tolist(), msgs["sending_silo"].tolist(), kt, lru,
                                                   functional)
        np.testing.assert_array_equal(res.route, np.array(r_ref, np.uint32), err_msg=f"route words, batch {seed}")
        np.testing.assert_array_equal(res.act, np.array(a_ref, np.uint32))
        o_ref, f_ref = o.bucket(np.array(a_ref, np.uint32), n_act)
        np.testing.assert_array_equal(res.order, o_ref)
        np.testing.assert_array_equal(res.offsets, f_ref)
        return int((((res.route >> 24) & L.RF_CACHED) != 0).sum())

    add(rng.choice(remote, 2500))                    # fits: the device path
    assert route(1) > 1000
    add(rng.choice(remote, 1500))                    # overflows: the entries no lookup touched go first
    route(2)
    present = np.array([g for g in remote.tolist() if kt_all[g] in lru.d], np.int64)
    lru_first = sorted(present.tolist(), key=lambda g: lru.d[kt_all[g]][1])[:300]  # the least recently used
    add(np.concatenate([np.array(lru_first), rng.choice(present, 500)]))          # updates at full capacity
    route(3)
    inval = rng.choice(remote, 400)
    d_rm = t.empty(len(inval), dtype=t.uint8, device="cuda")
    eng.cache_remove_device(dev(keys[inval]), len(inval), d_rm, stream=st_)
    t.cuda.synchronize()
    for g in inval.tolist():
        lru.remove(kt_all[g])
    assert eng.cache_count() == len(lru.d)
    route(4)
    add(rng.choice(remote, cap + 700, replace=False))  # one batch larger than the cache
    assert route(5) > 1000
    add(rng.choice(remote, 100))
    route(6)
    eng.close()


def _decode_on_device(t, eng, buf, nbytes, offs, sender_override=L.SENDER_FROM_HEADER):
    d_buf = t.from_numpy(buf).cuda()
    d_off = t.from_numpy(offs.view(np.int64)).cuda()
    n = len(offs)
    d_out = t.empty((n, 32), dtype=t.uint8, device="cuda")
    d_st = t.empty(n, dtype=t.uint8, device="cuda")
    d_bad = t.empty(1, dtype=t.int32, device="cuda")
    eng.decode_frames_device(d_buf, nbytes, d_off, n, d_out, d_st, d_bad, sender_override=sender_override,
                             stream=t.cuda.current_stream().cuda_stream)
    t.cuda.synchronize()
    return d_st.cpu().numpy(), d_out.cpu().numpy().reshape(-1).view(L.MSG_DTYPE), int(d_bad.cpu()[0]), d_out


def test_decode_frames_vs_oracle(torch):
    """received frames -> orl_msg_hdr on the device, status and record bit-exact against
    oracle/wire_codec.py over (a) one frame per decoder rule, (b) random header dictionaries using every value
    type the reference header reader accepts, (c) random truncations / byte flips / garbage lengths of those, at
    every start alignment, with and without a sender override; then a small batch (the simple kernel)."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import wire_corpus as C
    t = torch
    eng = GrainDirectoryEngine(n_act=16, dir_capacity=16, max_batch=1024, device=0)
    eng.set_silos(8)
    for s in range(8):
        eng.set_silo_address(s, *C.silo_addr(s))
    typed = C.typed_corpus(4000, seed=21)
    frames = C.edge_corpus() + typed + C.mutate(typed, 8000, seed=22)
    frames = frames * 6  # > 64k frames: the launcher's pipelined (LDS-staged) kernel; gaps differ per copy
    buf, offs, nbytes = C.pack(frames)
    for so in (L.SENDER_FROM_HEADER, 3):
        st, m, n_bad, _ = _decode_on_device(t, eng, buf, nbytes, offs, so)
        st_ref, m_ref = C.oracle_decode(buf, nbytes, offs, so)
        bad = np.nonzero(st != st_ref)[0]
        assert len(bad) == 0, (so, bad[:10], st[bad[:10]], st_ref[bad[:10]])
        np.testing.assert_array_equal(m.view(np.uint8), m_ref.view(np.uint8))
        assert n_bad == int((st_ref != 0).sum())
        assert len(set(st_ref.tolist())) == (6 if so == L.SENDER_FROM_HEADER else 5)  # every status exercised
    small = C.edge_corpus() + typed[:500]
    sb, so_, snb = C.pack(small, seed=5)
    st, m, _, _ = _decode_on_device(t, eng, sb, snb, so_)
    st_ref, m_ref = C.oracle_decode(sb, snb, so_)
    np.testing.assert_array_equal(st, st_ref)
    np.testing.assert_array_equal(m.view(np.uint8), m_ref.view(np.uint8))
    # a silo address removed from the table -> UNKNOWN_SILO for its senders
    eng.set_silo_address(1, None)
    st, _, _, _ = _decode_on_device(t, eng, buf, nbytes, offs)
    st_ref, _ = C.oracle_decode(buf, nbytes, offs)
    idx = {k: v for k, v in C.silo_index().items() if v != 1}
    from oracle import wire_codec as WC
    exp = [d.status for d in WC.decode_frames(bytes(buf[:nbytes]), [int(o) for o in offs], idx)]
    np.testing.assert_array_equal(st, np.array(exp, np.uint8))
    assert (st == 3).sum() > (st_ref == 3).sum()
    eng.close()


def test_decode_generator_frames_then_route(torch):
    """f2 feeding stages 1-4: synthetic request / response frames (complete addresses, KeyExt targets) decoded on
    the device equal the oracle's decode, and routing the decoded records equals routing the expected headers
    (KeyExt aux = pyref.uniform_hash)."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import wire_corpus as C
    from oracle import wire_codec as WC
    t = torch
    cl = W.balanced_cluster()
    n_grains, n = 200_000, 120_000
    eng = GrainDirectoryEngine(n_act=n_grains, dir_capacity=n_grains, max_batch=1 << 18, device=0)
    W.setup_engine(eng, cl)
    W.register_silo_addresses(eng, cl)
    keys, _, owner, reg = W.grain_population(cl, n_grains, 0.8)
    W.register_population(eng, keys, owner, reg)
    buf, offs, exp = W.request_frames(cl, n_grains, n, seed=77, complete_frac=0.2, keyext_frac=0.1)
    st, m, n_bad, d_out = _decode_on_device(t, eng, buf, len(buf), offs)
    assert n_bad == 0 and (st == 0).all()
    for f in ("tcd", "n0", "n1", "sending_silo", "category", "flags", "target_silo"):
        np.testing.assert_array_equal(m[f], exp[f], err_msg=f)
    kx = np.nonzero(exp["flags"] & L.HDR_HASH_VALID)[0]
    assert len(kx) > 1000
    idx = {(cl.silo_ip16(s), W.PORT, cl.gens[s]): s for s in range(cl.n_silos)}
    for i in kx[:300].tolist():
        o = int(offs[i])
        hl = int.from_bytes(bytes(buf[o:o + 4]), "little")
        d = WC.decode_for_route(bytes(buf[o + 8:o + 8 + hl]), idx)
        assert d.status == 0 and d.aux == int(m["aux"][i])
    exp["aux"] = m["aux"]
    d_r = t.empty(n, dtype=t.int32, device="cuda")
    d_a = t.empty(n, dtype=t.int32, device="cuda")
    eng.address_messages_device(d_out, n, d_r, d_a, stream=t.cuda.current_stream().cuda_stream, opts=L.OPT_NO_BUCKETS)
    t.cuda.synchronize()
    ref = eng.address_messages(exp)
    np.testing.assert_array_equal(d_r.cpu().numpy().view(np.uint32), ref.route)
    np.testing.assert_array_equal(d_a.cpu().numpy().view(np.uint32), ref.act)
    assert ((ref.route >> 16) & 0xFF == L.ST_ADDRESS_COMPLETE).sum() > 10_000
    eng.close()


def test_stamp_frames_vs_oracle(torch):
    """f2 emit: routed frames re-serialized with Message.SetTargetPlacement applied (.NET Dictionary slot reuse,
    PRIOR_MESSAGE_* removal, IS_NEW_PLACEMENT / NEW_GRAIN_TYPE on new placements, unchanged copies with a status
    for everything else), byte-exact against oracle/wire_codec.stamp_frames: random typed headers, the rule
    corpus, random mutations and generator frames, at every start alignment; output offsets = the scan of the
    4-byte-aligned output sizes; the out_cap overflow rule."""
    import random
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import wire_corpus as C
    from oracle import wire_codec as WC
    from oracle.pyref import Key
    t = torch
    rng = random.Random(31)
    eng = GrainDirectoryEngine(n_act=16, dir_capacity=16, max_batch=1024, device=0)
    eng.set_silos(8)
    for s in range(8):
        eng.set_silo_address(s, *C.silo_addr(s))
    typed = C.typed_corpus(3000, seed=41)
    cl = W.balanced_cluster()
    gbuf, goffs, _ = W.request_frames(cl, 1000, 1500, seed=5, complete_frac=0.3, keyext_frac=0.1)
    gen = [bytes(gbuf[int(o):int(goffs[k + 1]) if k + 1 < len(goffs) else len(gbuf)]) for k, o in enumerate(goffs)]
    gen = [g[:8 + int.from_bytes(g[:4], "little") + int.from_bytes(g[4:8], "little")] for g in gen]
    frames = C.edge_corpus() + typed + C.mutate(typed, 2000, seed=42) + gen
    rng.shuffle(frames)
    frames = frames * 10  # > 64k frames: the pipelined (LDS-staged) kernels, incl. deferred long headers
    buf, offs, nbytes = C.pack(frames, seed=43)
    n = len(frames)
    # grain types for some target type codes
    codes = set()
    for f in frames:
        try:
            h = WC.parse_headers(f[8:8 + int.from_bytes(f[:4], "little", signed=True)])
        except Exception:
            continue
        tg = h.get(WC.H_TARGET_GRAIN)
        if tg is not None and tg[0] == "grain":
            codes.add(tg[1].tcd & 0xFFFFFFFF)
    codes = sorted(codes)
    rng.shuffle(codes)
    grain_types = {c: "Grains.Type%d.%s" % (c, "é" * (c % 3)) for c in codes[:400]}
    for c, name in grain_types.items():
        eng.set_grain_type(c, name)
    statuses = [0, 0, 0, 1, 1, 3, 8, 2]
    route = np.array([(rng.choice(statuses) << 16) | (rng.randrange(10) << 8) for _ in range(n)], np.uint32)
    n_keys = 500
    act = np.array([rng.randrange(n_keys + 20) for _ in range(n)], np.uint32)
    act_keys = [Key(rng.choice([0, 3 << 56]), rng.getrandbits(64), rng.getrandbits(64), None) for _ in range(n_keys)]
    new_keys = [Key(0, rng.getrandbits(64), rng.getrandbits(64), None) for _ in range(n)]
    # a frame that already targets the activation it routes to (no PRIOR_MESSAGE_* removal)
    kd = np.zeros(n_keys, L.KEY_DTYPE)
    kd["tcd"], kd["n0"], kd["n1"] = [k.tcd for k in act_keys], [k.n0 for k in act_keys], [k.n1 for k in act_keys]
    nd = np.zeros(n, L.KEY_DTYPE)
    nd["tcd"], nd["n0"], nd["n1"] = [k.tcd for k in new_keys], [k.n0 for k in new_keys], [k.n1 for k in new_keys]
    silo_of = {s: C.silo_addr(s) for s in range(8)}
    ref = WC.stamp_frames(bytes(buf[:nbytes]), [int(o) for o in offs], route, act, act_keys, new_keys, silo_of, grain_types)
    st_ref = np.array([r[0] for r in ref], np.uint8)
    sizes = np.array([(len(r[1]) + 3) // 4 * 4 for r in ref], np.uint64)
    off_ref = np.zeros(n, np.uint64)
    off_ref[1:] = np.cumsum(sizes)[:-1]
    total_ref = int(sizes.sum())
    assert len(set(st_ref.tolist())) == 5, np.unique(st_ref, return_counts=True)

    d_buf = t.from_numpy(buf).cuda()
    d_off = t.from_numpy(offs.view(np.int64)).cuda()
    d_route = t.from_numpy(route.view(np.int32)).cuda()
    d_act = t.from_numpy(act.view(np.int32)).cuda()
    d_keys = t.from_numpy(kd.view(np.uint8)).cuda()
    d_new = t.from_numpy(nd.view(np.uint8)).cuda()
    # frames may overlap (a garbage body length that still fits the buffer), so the output can exceed the input
    # buffer: size the output from the oracle's total
    cap = total_ref + 1024
    d_out = t.zeros(cap, dtype=t.uint8, device="cuda")
    d_ooff = t.empty(n, dtype=t.int64, device="cuda")
    d_tot = t.empty(1, dtype=t.int64, device="cuda")
    d_st = t.empty(n, dtype=t.uint8, device="cuda")
    stream = t.cuda.current_stream().cuda_stream
    eng.stamp_frames_device(d_buf, nbytes, d_off, n, d_route, d_act, d_keys, n_keys, d_new, d_out, cap, d_ooff, d_tot,
                            d_st, stream=stream)
    t.cuda.synchronize()
    st = d_st.cpu().numpy()
    goff = d_ooff.cpu().numpy().view(np.uint64)
    gsz = np.diff(np.append(goff, np.uint64(int(d_tot.cpu()[0]))))
    badsz = np.nonzero(gsz != sizes)[0]
    if len(badsz):
        j = int(badsz[0])
        f = frames[j]
        raise AssertionError(("size", j, int(gsz[j]), int(sizes[j]), int(st_ref[j]), int(st[j]),
                              int.from_bytes(f[:4], "little", signed=True), int(offs[j]) & 3, len(badsz)))
    bad = np.nonzero(st != st_ref)[0]
    if len(bad):
        j = int(bad[0])
        outb = d_out.cpu().numpy()
        firstbad_bytes = next((i for i in range(j) if bytes(outb[int(off_ref[i]):int(off_ref[i]) + len(ref[i][1])]) != ref[i][1]), -1)
        raise AssertionError(("status", j, int(st[j]), int(st_ref[j]), int(goff[j]), int(off_ref[j]), cap, int(sizes[j]),
                              "first bad bytes before", firstbad_bytes, "n bad", len(bad), "statuses of bad",
                              np.unique(st_ref[bad], return_counts=True)))
    np.testing.assert_array_equal(goff, off_ref)
    assert int(d_tot.cpu()[0]) == total_ref
    out = d_out.cpu().numpy()
    for i, (s_, b) in enumerate(ref):
        o = int(off_ref[i])
        assert bytes(out[o:o + len(b)]) == b, (i, s_)
    assert (st_ref == WC.STAMP_OK).sum() > 10000
    assert sum(1 for f in frames if int.from_bytes(f[:4], "little", signed=True) > 245) > 100  # deferred path
    # the small-batch kernel on a prefix
    m = 3000
    eng.stamp_frames_device(d_buf, nbytes, d_off, m, d_route, d_act, d_keys, n_keys, d_new, d_out, cap, d_ooff, d_tot,
                            d_st, stream=stream)
    t.cuda.synchronize()
    np.testing.assert_array_equal(d_st.cpu().numpy()[:m], st_ref[:m])
    out = d_out.cpu().numpy()
    for i in range(m):
        o = int(off_ref[i])
        assert bytes(out[o:o + len(ref[i][1])]) == ref[i][1], i
    # out_cap too small: frames past it are not written (ORL_STAMP_OVERFLOW), earlier ones are
    cap2 = int(off_ref[n // 2])
    d_out2 = t.zeros(cap2 + 64, dtype=t.uint8, device="cuda")
    eng.stamp_frames_device(d_buf, nbytes, d_off, n, d_route, d_act, d_keys, n_keys, d_new, d_out2, cap2, d_ooff, d_tot,
                            d_st, stream=stream)
    t.cuda.synchronize()
    st2 = d_st.cpu().numpy()
    fits = off_ref + sizes <= cap2
    np.testing.assert_array_equal(st2[fits], st_ref[fits])
    assert (st2[~fits & (sizes > 0)] == L.STAMP_OVERFLOW).all()
    assert not d_out2[cap2:].any()
    eng.close()


def test_device_directory_merge_on_silo_remove(torch):
    """ProcessSiloRemoveEvent's GrainDirectoryPartition.Merge of a removed silo's partition copy on
    the device == pyref.Partition.merge: absent grains added; present grains keep the smaller ActivationId
    (UniqueKey.CompareTo order over the handles' ActivationId keys, incl. ties in TypeCodeData / N0) and report
    the dropped activation; same ActivationId kept; duplicates within the copy; unsupported entries; then the
    whole table read back against the oracle partition."""
    t = torch
    from oracle.pyref import Partition, Key
    rng = np.random.default_rng(17)
    cl = W.default_cluster()
    n_grains, n_act = 40_000, 30_000
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=2 * n_grains, max_batch=1 << 18, device=0)
    eng.set_silos(8)
    for s in range(8):
        eng.add_server(s, int(cl.hashes[s]))
    keys_all, _, owner, _ = W.grain_population(cl, n_grains)
    # our partition: the first half of the grains, any silo (the host path registers without an owner check here:
    # a silo holding its own partition and the copy it merges)
    ours = np.arange(n_grains // 2)
    acts0 = rng.integers(0, n_act, len(ours)).astype(np.uint32)
    silos0 = rng.integers(0, 8, len(ours)).astype(np.uint8)
    part = Partition()
    st0 = np.zeros(len(ours), np.uint8)
    # register through the device merge itself into an empty table (all INSERTED) — also a test of that path
    n_keys = n_act
    ak = np.zeros(n_keys, L.KEY_DTYPE)
    ak["tcd"] = rng.integers(0, 3, n_keys).astype(np.uint64)          # ties in TypeCodeData ...
    ak["n0"] = rng.integers(0, 4, n_keys).astype(np.uint64)           # ... and in N0
    ak["n1"] = rng.integers(0, 1 << 62, n_keys, dtype=np.uint64)
    ak[7] = ak[8]                                                     # two handles, one ActivationId
    akey = lambda a: (int(ak["tcd"][a]), int(ak["n0"][a]), int(ak["n1"][a]))

    def dev(a):
        return t.from_numpy(np.ascontiguousarray(a).view(np.uint8)).cuda()

    d_ak = dev(ak)
    st_ = t.cuda.current_stream().cuda_stream

    def merge(keys, acts, silos):
        m = len(keys)
        d_st = t.empty(m, dtype=t.uint8, device="cuda")
        d_da = t.empty(m, dtype=t.int32, device="cuda")
        d_ds = t.empty(m, dtype=t.uint8, device="cuda")
        eng.merge_directory_device(dev(keys), dev(acts), dev(silos), m, d_ak, n_keys, d_st, d_da, d_ds, stream=st_)
        t.cuda.synchronize()
        return d_st.cpu().numpy(), d_da.cpu().numpy().view(np.uint32), d_ds.cpu().numpy()

    k0 = keys_all[ours]
    st, da, ds = merge(k0, acts0, silos0)
    exp = part.merge([(Key(int(k["tcd"]), int(k["n0"]), int(k["n1"])), int(a), int(s)) for k, a, s in zip(k0, acts0, silos0)], akey)
    np.testing.assert_array_equal(st, [e[0] for e in exp])
    assert (st == L.MERGE_INSERTED).all()
    # the removed silo's copy: half overlapping our grains, half new, duplicates, same activations, bad entries
    m = 30_000
    pick = rng.integers(n_grains // 4, n_grains, m)
    keys = keys_all[pick].copy()
    acts = rng.integers(0, n_act, m).astype(np.uint32)
    same = rng.random(m) < 0.1
    cur_act = {int(i): int(a) for i, a in zip(ours, acts0)}
    for j in np.nonzero(same)[0]:
        if int(pick[j]) in cur_act:
            acts[j] = cur_act[int(pick[j])]
    acts[5] = 8 if int(pick[5]) in cur_act and cur_act[int(pick[5])] == 7 else acts[5]
    silos = rng.integers(0, 8, m).astype(np.uint8)
    bad = np.zeros(m, bool)
    bad[::501] = True
    acts[::501] = n_act + 3                                           # out-of-range handle
    keys[250]["tcd"] = (np.uint64(L.CAT_KEYEXT_GRAIN) << np.uint64(56)) | np.uint64(5)
    bad[250] = True
    st, da, ds = merge(keys, acts, silos)
    good = np.nonzero(~bad)[0]
    exp = part.merge([(Key(int(keys["tcd"][j]), int(keys["n0"][j]), int(keys["n1"][j])), int(acts[j]), int(silos[j]))
                      for j in good], akey)
    assert (st[bad] == L.MERGE_UNSUPPORTED).all()
    np.testing.assert_array_equal(st[good], [e[0] for e in exp])
    np.testing.assert_array_equal(da[good], [e[1] for e in exp])
    np.testing.assert_array_equal(ds[good], [e[2] for e in exp])
    for code in (L.MERGE_INSERTED, L.MERGE_KEPT, L.MERGE_REPLACED, L.MERGE_SAME, L.MERGE_DUPLICATE):
        assert (st == code).sum() > 50, code
    # the table after the merge
    a, s = eng.lookup_host(keys_all)
    for g in range(n_grains):
        k = keys_all[g]
        r = part.data.get((int(k["tcd"]), int(k["n0"]), int(k["n1"]), None))
        assert (int(a[g]), int(s[g])) == (r if r is not None else (L.NO_ACT, 0xFF)), g
    assert eng.directory_count() == len(part.data)
    eng.close()


def _mixed_type_setup(n_types, guid_frac, seed):
    """A partition of long-key grains of `n_types` type codes (plus Guid keys with probability guid_frac), a tenth
    of them unregistered again (tombstones), and messages that also name unregistered keys, unknown type codes,
    N0 != 0 and registered N1 values under another type code."""
    n_silos, n = 8, 20_000
    cl = W.default_cluster(n_silos)
    rng = np.random.default_rng(seed)
    tcs = (L.CAT_GRAIN << 56) + (rng.integers(-2**31, 2**31, n_types).astype(np.int64).astype(np.uint64)
                                  & np.uint64(0x00FFFFFFFFFFFFFF))
    keys = np.zeros(n, L.KEY_DTYPE)
    keys["tcd"] = tcs[rng.integers(0, n_types, n)]
    keys["n1"] = rng.permutation(n * 4)[:n].astype(np.uint64)
    g = rng.random(n) < guid_frac
    keys["n0"][g] = rng.integers(1, 2**63, int(g.sum()), dtype=np.int64).astype(np.uint64)
    acts = np.arange(n, dtype=np.uint32)
    silos = rng.integers(0, n_silos, n).astype(np.uint8)
    msgs = np.zeros(200_000, L.MSG_DTYPE)
    pick = rng.integers(0, n, len(msgs))
    msgs["tcd"], msgs["n0"], msgs["n1"] = keys["tcd"][pick], keys["n0"][pick], keys["n1"][pick]
    r = rng.random(len(msgs))
    msgs["n1"][r < 0.05] += np.uint64(n * 4)                         # never registered
    msgs["tcd"][(r >= 0.05) & (r < 0.08)] ^= np.uint64(0x5A5A)        # unknown type code, registered N1
    msgs["n0"][(r >= 0.08) & (r < 0.10)] ^= np.uint64(1)              # N0 flipped
    msgs["tcd"][(r >= 0.10) & (r < 0.13)] = tcs[0]                     # N1 of another type under type 0
    msgs["n1"][(r >= 0.13) & (r < 0.15)] += np.uint64(1 << 32)        # low 32 bits of a registered N1
    msgs["sending_silo"] = rng.integers(0, n_silos, len(msgs)).astype(np.uint8)
    return cl, keys, acts, silos, msgs, rng


@pytest.mark.parametrize("n_types,guid_frac", [(1, 0.0), (8, 0.0), (9, 0.0), (3, 0.01)])
def test_compact_probe_table_vs_full_table(torch, monkeypatch, n_types, guid_frac):
    """The 16-B probe table (<= 8 long-key type codes: probe_tcd) and the 32-B table route identically, and both
    match the oracle, with tombstones, misses, foreign type codes and N0 != 0 keys; 9 types or a Guid key fall
    back to the 32-B table.  One type with 32-bit N1 values and small handles takes the 8-B form (N1 values whose
    low 32 bits name a registered grain must still miss)."""
    cl, keys, acts, silos, msgs, rng = _mixed_type_setup(n_types, guid_frac, seed=n_types * 31 + int(guid_frac * 100))
    o = cpu_ref.Oracle(8, seed=0)
    outs = []
    for off in ("0", "1", "8"):
        monkeypatch.setenv("ORL_NO_PROBE16", "1" if off == "1" else "0")
        monkeypatch.setenv("ORL_NO_PROBE8", "1" if off == "8" else "0")
        eng = GrainDirectoryEngine(n_act=len(keys), dir_capacity=len(keys), max_batch=1 << 20, device=0)
        eng.set_silos(8, seed=0)
        for s in range(8):
            eng.add_server(s, int(cl.hashes[s]))
            if off == "0":
                o.add_server(s, int(cl.hashes[s]))
        eng.register_single_activation(keys, acts, silos)
        gone = keys[rng.permutation(len(keys))[: len(keys) // 10]] if off == "0" else gone
        np.testing.assert_array_equal(eng.unregister(gone), np.ones(len(gone), np.uint8))
        if off == "0":
            o.register(keys, acts, silos)
            o.unregister(gone)
        res = eng.address_messages(msgs)
        outs.append((res.route.copy(), res.act.copy(), res.order.copy(), res.offsets.copy()))
        eng.close()
    r, a = o.route(msgs)
    np.testing.assert_array_equal(outs[0][0], r)
    np.testing.assert_array_equal(outs[0][1], a)
    for o2 in outs[1:]:
        for x, y in zip(outs[0], o2):
            np.testing.assert_array_equal(x, y)
    hit = (r >> 16) & 0xFF
    assert (hit == L.ST_HIT).sum() > 100_000 and (hit == L.ST_NEW_PLACEMENT).sum() > 20_000


def test_probe_table_rebuilt_after_device_mutations(torch, monkeypatch):
    """After device registrations / unregistrations (f1) the compact probe table is rebuilt on the device from the
    host's type list; routing matches the oracle and the 32-B table.  A device-registered Guid key (N0 != 0) does
    not fit the probe table: the build flags it and the route kernels fall back to the 32-B table."""
    t = torch
    cl = W.default_cluster()
    n_grains, n_act = 40_000, 40_000
    keys_all, _, owner, _ = W.grain_population(cl, n_grains)
    rng = np.random.default_rng(3)
    host_part = rng.permutation(n_grains)[:10_000]
    dev_part = rng.integers(0, n_grains, 30_000)
    rm = keys_all[rng.integers(0, n_grains, 8_000)]
    guid = keys_all[:64].copy()
    guid["n0"] = rng.integers(1, 2**63, 64, dtype=np.int64).astype(np.uint64)
    msgs = W.uniform_messages(cl, n_grains, 200_000, seed=4)
    gm = np.zeros(64, L.MSG_DTYPE)
    gm["tcd"], gm["n0"], gm["n1"] = guid["tcd"], guid["n0"], guid["n1"]
    msgs2 = np.concatenate([msgs, gm])

    def dev(a):
        return t.from_numpy(np.ascontiguousarray(a).view(np.uint8)).cuda()

    o = cpu_ref.Oracle(8, seed=0)
    for s in range(8):
        o.add_server(s, int(cl.hashes[s]))
    o.register(keys_all[host_part], host_part.astype(np.uint32), owner[host_part])
    o.register(keys_all[dev_part], dev_part.astype(np.uint32), owner[dev_part])
    o.unregister(rm)
    ref1 = o.route(msgs)
    o.register(guid, np.arange(64, dtype=np.uint32), owner[:64])
    ref2 = o.route(msgs2)
    outs = []
    for off in ("0", "1"):
        monkeypatch.setenv("ORL_NO_PROBE16", off)
        eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=n_grains, max_batch=1 << 20, device=0)
        eng.set_silos(8, seed=0)
        for s in range(8):
            eng.add_server(s, int(cl.hashes[s]))
        eng.register_single_activation(keys_all[host_part], host_part.astype(np.uint32), owner[host_part])
        st_ = t.cuda.current_stream().cuda_stream
        m = len(dev_part)
        d_st = t.empty(m, dtype=t.uint8, device="cuda")
        d_wa = t.empty(m, dtype=t.int32, device="cuda")
        d_ws = t.empty(m, dtype=t.uint8, device="cuda")
        eng.register_single_activation_device(dev(keys_all[dev_part]), dev(dev_part.astype(np.uint32)),
                                              dev(owner[dev_part]), m, d_st, d_wa, d_ws, stream=st_)
        d_rm = t.empty(len(rm), dtype=t.uint8, device="cuda")
        eng.unregister_device(dev(rm), len(rm), d_rm, stream=st_)
        t.cuda.synchronize()
        res = eng.address_messages(msgs)
        np.testing.assert_array_equal(res.route, ref1[0])
        np.testing.assert_array_equal(res.act, ref1[1])
        outs.append((res.route.copy(), res.act.copy(), res.order.copy()))
        d_st2 = t.empty(64, dtype=t.uint8, device="cuda")
        eng.register_single_activation_device(dev(guid), dev(np.arange(64, dtype=np.uint32)), dev(owner[:64]), 64,
                                              d_st2, d_wa[:64], d_ws[:64], stream=st_)
        t.cuda.synchronize()
        res2 = eng.address_messages(msgs2)
        np.testing.assert_array_equal(res2.route, ref2[0])
        np.testing.assert_array_equal(res2.act, ref2[1])
        eng.close()
    for x, y in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(x, y)
    assert ((ref2[0][-64:] >> 16) & 0xFF == L.ST_HIT).all()


def test_keyext_directory_vs_oracle(torch, golden_dir):
    """VERDICT r4 missing 2: KeyExt (string-key) grains registered and looked up on the device.  GrainDirectoryPartition
    holds any GrainId (GrainDirectoryPartition.cs:270-287, 326-344) and a KeyExt grain's identity includes its extension
    (UniqueKey.cs:288-294), so grains that share (TypeCodeData, N0, N1) and differ only in the string are different
    entries.  Registration (first writer wins, invalid silo, remote owner) and routing through orl_route_keyext_device —
    owner from the KeyExt hash (the header's precomputed one, or computed on the device from the bytes), HIT on the local
    owner filtered by IsValidSilo, placement of misses, ORL_ST_REMOTE_OWNER — then stage 4, all equal to pyref's restatement
    (+ the C++ oracle's stable bucketing); the golden KeyExt cases (the 400-char extension, non-ASCII UTF-8) included;
    removal, then the same batch again.  Long-key grains in the same batch route as before."""
    t = torch
    cl = W.default_cluster()
    local = [1, 1, 1, 1, 0, 0, 0, 0]
    functional = [1, 1, 1, 1, 1, 1, 0, 1]
    ring = P.Ring()
    for s in range(8):
        ring.add_server(s, int(cl.hashes[s]))
    view = P.SiloView(running=[True] * 8, functional=[bool(f) for f in functional], local=[bool(x) for x in local])
    part = P.Partition()
    n_act = 40_000
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=20_000, max_batch=1 << 18, device=0)
    eng.set_silos(8, functional=functional, local=local)
    for s in range(8):
        eng.add_server(s, int(cl.hashes[s]))
    rng = np.random.default_rng(11)
    tc = cl.type_code
    # long-key grains (the plain partition)
    lk = [P.key_from_long(int(i), tc) for i in range(5000)]
    lkeys = np.array([(k.tcd, k.n0, k.n1) for k in lk], L.KEY_DTYPE)
    lsilo = rng.integers(0, 8, len(lk)).astype(np.uint8)
    lact = np.arange(len(lk), dtype=np.uint32)
    st, _, _ = eng.register_single_activation(lkeys, lact, lsilo)
    for i, k in enumerate(lk):
        assert P.register_single_activation(ring, part, view, k, int(lact[i]), int(lsilo[i]))[0] == st[i]
    # KeyExt grains: golden cases + generated ones (N1 shared by several strings), duplicates, non-functional silos
    gold = json.load(open(os.path.join(golden_dir, "jenkins.json")))["keyext"]
    kx = [P.Key(int(g["tcd"], 16), int(g["n0"], 16), int(g["n1"], 16), g["ext"]) for g in gold]
    for k, g in zip(kx, gold):
        assert P.uniform_hash(k) == g["uniform"]
    for i in range(3000):
        ext = rng.choice(["user-%d", "ключ-%d", "grain/%d/part", "é中%d\U0001F600"]) % (i // 3)
        kx.append(P.key_from_long(int(i % 700), tc, ext))
    kx += kx[100:160]  # re-registrations: the first writer wins
    xact = (5000 + np.arange(len(kx))).astype(np.uint32)
    xsilo = rng.integers(0, 8, len(kx)).astype(np.uint8)
    keys = np.array([(k.tcd, k.n0, k.n1) for k in kx], L.KEY_DTYPE)
    st, wa, ws = eng.register_keyext(keys, [k.key_ext for k in kx], xact, xsilo)
    exp = [P.register_keyext(ring, part, view, k, int(a), int(s)) for k, a, s in zip(kx, xact, xsilo)]
    np.testing.assert_array_equal(st, np.array([e[0] for e in exp], np.uint8))
    np.testing.assert_array_equal(wa[st <= 1], np.array([e[1] for e in exp], np.uint32)[st <= 1])
    assert eng.keyext_count() == sum(1 for e in exp if e[0] == P.INS_INSERTED)
    assert {0, 1, 2, 3} <= set(st.tolist())  # inserted, existing, invalid silo, remote owner all occur
    a_h, s_h = eng.lookup_keyext_host(keys, [k.key_ext for k in kx])
    for i, k in enumerate(kx):
        r = part.data.get(P.Partition._k(k))
        assert (a_h[i], s_h[i]) == ((r[0], r[1]) if r else (L.NO_ACT, 0xFF))

    def batch(n, seed):
        r = np.random.default_rng(seed)
        msgs, strings = [], []
        for i in range(n):
            u = r.random()
            sender = int(r.integers(0, 4))
            if u < 0.3:
                k = lk[int(r.integers(0, len(lk)))]
            elif u < 0.85:
                k = kx[int(r.integers(0, len(kx)))]
            else:  # a KeyExt grain nobody registered
                k = P.key_from_long(int(r.integers(0, 700)), tc, "nobody-%d" % int(r.integers(0, 10 ** 6)))
            pre = k.key_ext is not None and r.random() < 0.5  # half carry the precomputed hash (ORL_HDR_HASH_VALID)
            msgs.append(P.Msg(k, sender, P.HDR_HASH_VALID if pre else 0, aux=P.uniform_hash(k) if pre else 0))
            strings.append(k.key_ext or "")
        return msgs, strings

    def run(msgs, strings):
        n = len(msgs)
        h = np.zeros(n, L.MSG_DTYPE)
        h["tcd"] = [m.key.tcd for m in msgs]
        h["n0"] = [m.key.n0 for m in msgs]
        h["n1"] = [m.key.n1 for m in msgs]
        h["sending_silo"] = [m.sending_silo for m in msgs]
        h["category"] = 2
        h["flags"] = [m.flags for m in msgs]
        h["target_silo"] = 0xFF
        h["aux"] = [m.aux for m in msgs]
        ref, blob = GrainDirectoryEngine.ext_blob(strings)
        d_in = t.from_numpy(h.view(np.int32).reshape(-1, 8)).cuda()
        d_ref = t.from_numpy(ref.view(np.int32)).cuda()
        d_blob = t.from_numpy(blob).cuda()
        outs = [t.empty(n, dtype=t.int32, device="cuda") for _ in range(3)] + [t.empty(n_act + 2, dtype=t.int32, device="cuda")]
        s = t.cuda.current_stream().cuda_stream
        eng.address_keyext_device(d_in, n, d_ref, d_blob, len(blob), *outs, stream=s)
        t.cuda.synchronize()
        route, act, order, off = (x.cpu().numpy().view(np.uint32) for x in outs)
        er, ea = P.route_batch(msgs, ring, part, view, keyext_directory=True)
        er, ea = np.array(er, np.uint32), np.array(ea, np.uint32)
        np.testing.assert_array_equal(route, er)
        np.testing.assert_array_equal(act, ea)
        eo, ef = cpu_ref.Oracle(8).bucket(ea, n_act)
        np.testing.assert_array_equal(order, eo)
        np.testing.assert_array_equal(off, ef)
        return er

    msgs, strings = batch(30_000, 5)
    er = run(msgs, strings)
    stc = (er >> 16) & 0xFF
    isx = np.array([m.key.key_ext is not None for m in msgs])
    for code in (L.ST_HIT, L.ST_NEW_PLACEMENT, L.ST_REMOTE_OWNER):  # every KeyExt outcome occurs
        assert (stc[isx] == code).sum() > 100, code
    # removal (UnregisterAsync -> RemoveActivation), then the same batch
    gone = kx[:1500:3]
    rm = eng.unregister_keyext(np.array([(k.tcd, k.n0, k.n1) for k in gone], L.KEY_DTYPE), [k.key_ext for k in gone])
    for i, k in enumerate(gone):
        assert bool(rm[i]) == part.remove(k)
    run(msgs, strings)
    eng.close()


def test_keyext_device_insert_vs_oracle(torch, golden_dir):
    """VERDICT r5 item 6 (second half): KeyExt registration by device kernels (orl_dir_insert_keyext_device: claim /
    resolve / commit over the KeyExt table, strings appended to the device store) with the host call's semantics —
    GrainDirectoryPartition.AddSingleActivation over any GrainId (GrainDirectoryPartition.cs:270-287), first writer of a key
    in the batch wins (GrainInfo.AddSingleActivation :103-107), invalid silo, remote owner, a key of another category;
    out-of-range acts give ORL_INS_UNSUPPORTED on the device.  Statuses and winners equal pyref's sequential restatement;
    then the host calls (lookup, count, a host insert, a removal) see the device's table, a second device batch after them
    (existing keys, new ones, a table that must grow), and the routed batch (orl_route_keyext_device) equals pyref."""
    t = torch
    cl = W.default_cluster()
    local = [1, 1, 1, 1, 0, 0, 0, 0]
    functional = [1, 1, 1, 1, 1, 1, 0, 1]
    ring = P.Ring()
    for s in range(8):
        ring.add_server(s, int(cl.hashes[s]))
    view = P.SiloView(running=[True] * 8, functional=[bool(f) for f in functional], local=[bool(x) for x in local])
    part = P.Partition()
    n_act = 40_000
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=1024, max_batch=1 << 16, device=0)
    eng.set_silos(8, functional=functional, local=local)
    for s in range(8):
        eng.add_server(s, int(cl.hashes[s]))
    rng = np.random.default_rng(23)
    tc = cl.type_code
    gold = json.load(open(os.path.join(golden_dir, "jenkins.json")))["keyext"]
    kx = [P.Key(int(g["tcd"], 16), int(g["n0"], 16), int(g["n1"], 16), g["ext"]) for g in gold]
    for i in range(1500):
        ext = rng.choice(["user-%d", "ключ-%d", "grain/%d/part", "é中%d\U0001F600", "%d"]) % (i // 2)
        kx.append(P.key_from_long(int(i % 300), tc, ext))
    kx += kx[50:120] + kx[7:9]  # re-registrations in the same batch: the first writer wins
    kx.append(P.key_from_long(5, tc))  # a long key: ORL_INS_UNSUPPORTED

    def dev_insert(keys_, acts, silos):
        strings = [k.key_ext or "" for k in keys_]
        keys = np.array([(k.tcd, k.n0, k.n1) for k in keys_], L.KEY_DTYPE)
        ref, blob = GrainDirectoryEngine.ext_blob(strings)
        n = len(keys_)
        d = lambda a: t.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()  # noqa: E731
        d_st, d_wa, d_ws = (t.zeros(n, dtype=t.uint8, device="cuda"), t.zeros(n, dtype=t.int32, device="cuda"),
                            t.zeros(n, dtype=t.uint8, device="cuda"))
        eng.register_keyext_device(d(keys), d(ref), d(blob), len(blob), d(acts.astype(np.uint32)), d(silos.astype(np.uint8)), n,
                                   d_st, d_wa, d_ws, stream=t.cuda.current_stream().cuda_stream)
        t.cuda.synchronize()
        return d_st.cpu().numpy(), d_wa.cpu().numpy().view(np.uint32), d_ws.cpu().numpy()

    def expected(keys_, acts, silos):
        out = []
        for k, a, s in zip(keys_, acts, silos):
            if a >= n_act:
                out.append((L.INS_UNSUPPORTED, L.NO_ACT, 0xFF))
            elif k.key_ext is None:
                out.append((L.INS_UNSUPPORTED, L.NO_ACT, 0xFF))
            else:
                out.append(P.register_keyext(ring, part, view, k, int(a), int(s)))
        return out

    def check(got, exp):
        st, wa, ws = got
        np.testing.assert_array_equal(st, np.array([e[0] for e in exp], np.uint8))
        ok = st <= 1
        np.testing.assert_array_equal(wa[ok], np.array([e[1] for e in exp], np.uint32)[ok])
        np.testing.assert_array_equal(ws[ok], np.array([e[2] for e in exp], np.uint8)[ok])

    acts = (1000 + np.arange(len(kx))).astype(np.uint32)
    acts[3] = n_act + 7  # out of range: UNSUPPORTED on the device, nothing inserted
    silos = rng.integers(0, 8, len(kx)).astype(np.uint8)
    got = dev_insert(kx, acts, silos)
    exp = expected(kx, acts, silos)
    check(got, exp)
    assert {0, 1, 2, 3, 5} <= set(got[0].tolist())  # inserted, existing, invalid silo, remote owner, unsupported
    # the host calls see the device's table (they download it first)
    assert eng.keyext_count() == len(part.data)
    q = kx[:400]
    a_h, s_h = eng.lookup_keyext_host(np.array([(k.tcd, k.n0, k.n1) for k in q], L.KEY_DTYPE), [k.key_ext or "" for k in q])
    for i, k in enumerate(q):
        r = part.data.get(P.Partition._k(k)) if k.key_ext is not None else None
        assert (a_h[i], s_h[i]) == ((r[0], r[1]) if r else (L.NO_ACT, 0xFF)), i
    # a host insert and a removal in between, then a second, larger device batch (the table grows on the host first)
    hk = [P.key_from_long(900 + i, tc, "host-%d" % i) for i in range(200)]
    st_h, _, _ = eng.register_keyext(np.array([(k.tcd, k.n0, k.n1) for k in hk], L.KEY_DTYPE), [k.key_ext for k in hk],
                                     np.arange(200, dtype=np.uint32) + 30000, np.zeros(200, np.uint8))
    exp_h = [P.register_keyext(ring, part, view, k, 30000 + i, 0) for i, k in enumerate(hk)]
    np.testing.assert_array_equal(st_h, np.array([e[0] for e in exp_h], np.uint8))
    gone = kx[10:400:4]
    rm = eng.unregister_keyext(np.array([(k.tcd, k.n0, k.n1) for k in gone], L.KEY_DTYPE), [k.key_ext or "" for k in gone])
    for i, k in enumerate(gone):
        assert bool(rm[i]) == (k.key_ext is not None and part.remove(k))
    kx2 = kx[:600] + hk[:50] + [P.key_from_long(int(i % 500), tc, "second-%d" % i) for i in range(3000)]
    acts2 = (5000 + np.arange(len(kx2))).astype(np.uint32)
    silos2 = rng.integers(0, 8, len(kx2)).astype(np.uint8)
    got2 = dev_insert(kx2, acts2, silos2)
    check(got2, expected(kx2, acts2, silos2))
    assert eng.keyext_count() == len(part.data)
    # routing reads the device table
    msgs, strings = [], []
    for i in range(20_000):
        k = kx2[int(rng.integers(0, len(kx2)))] if rng.random() < 0.85 else P.key_from_long(int(rng.integers(0, 500)), tc, "none-%d" % i)
        if k.key_ext is None:
            continue
        msgs.append(P.Msg(k, int(rng.integers(0, 4))))
        strings.append(k.key_ext)
    h = np.zeros(len(msgs), L.MSG_DTYPE)
    h["tcd"] = [m.key.tcd for m in msgs]
    h["n0"] = [m.key.n0 for m in msgs]
    h["n1"] = [m.key.n1 for m in msgs]
    h["sending_silo"] = [m.sending_silo for m in msgs]
    h["category"] = 2
    h["target_silo"] = 0xFF
    ref, blob = GrainDirectoryEngine.ext_blob(strings)
    n = len(msgs)
    outs = [t.empty(n, dtype=t.int32, device="cuda") for _ in range(3)] + [t.empty(n_act + 2, dtype=t.int32, device="cuda")]
    eng.address_keyext_device(t.from_numpy(h.view(np.int32).reshape(-1, 8)).cuda(), n, t.from_numpy(ref.view(np.int32)).cuda(),
                              t.from_numpy(blob).cuda(), len(blob), *outs, stream=t.cuda.current_stream().cuda_stream)
    t.cuda.synchronize()
    er, ea = P.route_batch(msgs, ring, part, view, keyext_directory=True)
    np.testing.assert_array_equal(outs[0].cpu().numpy().view(np.uint32), np.array(er, np.uint32))
    np.testing.assert_array_equal(outs[1].cpu().numpy().view(np.uint32), np.array(ea, np.uint32))
    eng.close()
