"""CPU tests of the C-ABI library: it loads, exports exactly what include/orleans_route.h declares, and its
host-side control plane (identity hashes, ring, directory registration) matches the oracle.  No GPU compute
is called here: contexts are created host-only (device = -1)."""
import json
import os
import re

import numpy as np
import pytest

from oracle import cpu_ref, pyref as P
from orleans_amd import _lib as L
from orleans_amd.engine import (GrainDirectoryEngine, OrleansRouteError, calc_id_hash, jenkins_bytes,
                                keyext_uniform_hash, silo_consistent_hash)

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def header_symbols():
    text = open(os.path.join(ROOT, "include", "orleans_route.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(orl_[a-z0-9_]+)\s*\(", text)) - {"orl_ctx"}


def test_library_exports_every_declared_symbol():
    lib = L.load()
    declared = header_symbols()
    assert declared == set(L.EXPORTED), declared ^ set(L.EXPORTED)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.orl_abi_version() == L.ABI_VERSION


def test_header_struct_layouts_match_oracle():
    assert L.MSG_DTYPE == cpu_ref.MSG_DTYPE
    assert L.KEY_DTYPE == cpu_ref.KEY_DTYPE


def test_calc_id_hash_golden(golden_dir):
    g = json.load(open(os.path.join(golden_dir, "idhash.json")))
    for c in g["id_hash"]:
        assert calc_id_hash(c["text"]) == c["hash"], c["text"]
    for c in g["silo_consistent"]:
        assert silo_consistent_hash(c["endpoint"], c["generation"]) == c["hash"], c


def test_jenkins_bytes_and_keyext_golden(golden_dir):
    g = json.load(open(os.path.join(golden_dir, "jenkins.json")))
    for c in g["bytes"]:
        assert jenkins_bytes(bytes.fromhex(c["hex"])) == c["hash"]
    for c in g["keyext"]:
        assert keyext_uniform_hash(int(c["tcd"], 16), int(c["n0"], 16), int(c["n1"], 16), c["ext"]) == c["uniform"]
    for c in json.load(open(os.path.join(golden_dir, "idhash.json")))["silo_uniform"]:
        b = bytes.fromhex(c["ip16"]) + c["port"].to_bytes(4, "little", signed=True) + \
            c["generation"].to_bytes(4, "little", signed=True) + c["extra"].to_bytes(4, "little", signed=True)
        assert jenkins_bytes(b) == c["hash"]


def test_ctx_create_validation():
    with pytest.raises(OrleansRouteError):
        GrainDirectoryEngine(n_act=0, dir_capacity=16, device=-1)
    with pytest.raises(OrleansRouteError):
        GrainDirectoryEngine(n_act=16, dir_capacity=16, device=-1, placement=7)


def test_host_only_ctx_refuses_device_work():
    eng = GrainDirectoryEngine(n_act=16, dir_capacity=16, device=-1)
    eng.set_silos(2)
    with pytest.raises(OrleansRouteError) as e:
        eng.address_messages(np.zeros(4, L.MSG_DTYPE))
    assert e.value.code == L.E_STATE
    eng.close()


def test_ring_golden(golden_dir):
    for c in json.load(open(os.path.join(golden_dir, "ring.json"))):
        if not c["adds"]:
            continue
        n_silos = max(s for s, _ in c["adds"]) + 1
        eng = GrainDirectoryEngine(n_act=16, dir_capacity=16, device=-1)
        eng.set_silos(n_silos)
        for s, h in c["adds"]:
            eng.add_server(s, h)
        eng.add_server(c["adds"][0][0], 12345)  # re-adding a cached silo is a no-op (:247-251)
        assert [list(e) for e in eng.membership_ring()] == [list(e) for e in c["ring"]], c["name"]
        eng.remove_server(c["adds"][0][0])
        assert [list(e) for e in eng.membership_ring()] == [list(e) for e in c["ring"] if e[1] != c["adds"][0][0]]
        eng.close()


@pytest.mark.parametrize("name", ["routing_basic", "routing_membership"])
def test_registration_golden(golden_dir, name):
    """RegisterSingleActivation → AddSingleActivation semantics of the library's partition mirror."""
    d = np.load(os.path.join(golden_dir, name + ".npz"))
    n = len(d["silo_hashes"])
    eng = GrainDirectoryEngine(n_act=int(d["n_act"]), dir_capacity=len(d["reg_keys"]), device=-1,
                               placement=int(d["policy"]))
    eng.set_silos(n, running=d["running"], functional=d["functional"], seed=int(d["seed"]))
    for s in range(n):
        eng.add_server(s, int(d["silo_hashes"][s]))
    keys = np.zeros(len(d["reg_keys"]), L.KEY_DTYPE)
    keys["tcd"], keys["n0"], keys["n1"] = d["reg_keys"][:, 0], d["reg_keys"][:, 1], d["reg_keys"][:, 2]
    st, wa, ws = eng.register_single_activation(keys, d["reg_acts"], d["reg_silos"])
    np.testing.assert_array_equal(st, d["reg_status"])
    np.testing.assert_array_equal(wa, d["reg_wact"])
    np.testing.assert_array_equal(ws, d["reg_wsilo"])
    assert eng.directory_count() == int((d["reg_status"] == L.INS_INSERTED).sum())
    a, s = eng.lookup_host(keys)
    ins = d["reg_status"] <= L.INS_EXISTING
    np.testing.assert_array_equal(a[ins], d["reg_wact"][ins])
    # unregister half, re-register: tombstones are reused and lookups stay exact
    half = keys[: len(keys) // 2]
    removed = eng.unregister(half)
    assert removed.sum() == len(np.unique(half[ins[: len(half)]]))
    a2, _ = eng.lookup_host(half)
    assert (a2 == L.NO_ACT).all()
    st2, _, _ = eng.register_single_activation(half, d["reg_acts"][: len(half)], d["reg_silos"][: len(half)])
    o = cpu_ref.Oracle(n, running=list(d["running"]), functional=list(d["functional"]), seed=int(d["seed"]))
    for s_ in range(n):
        o.add_server(s_, int(d["silo_hashes"][s_]))
    o.register(keys, d["reg_acts"], d["reg_silos"])
    o.unregister(half)
    st_o, _, _ = o.register(half, d["reg_acts"][: len(half)], d["reg_silos"][: len(half)])
    np.testing.assert_array_equal(st2, st_o)
    eng.close()


def test_registration_capacity_and_validation():
    eng = GrainDirectoryEngine(n_act=8, dir_capacity=4, device=-1)
    eng.set_silos(1)
    eng.add_server(0, 0)
    keys = np.zeros(20, L.KEY_DTYPE)
    keys["tcd"] = P.CAT_GRAIN << 56
    keys["n1"] = np.arange(20)
    with pytest.raises(OrleansRouteError):  # act >= n_act
        eng.register_single_activation(keys[:1], np.array([9], np.uint32), np.zeros(1, np.uint8))
    with pytest.raises(OrleansRouteError) as e:  # slots = 16, load capped at 1/2
        eng.register_single_activation(keys, np.arange(20, dtype=np.uint32) % 8, np.zeros(20, np.uint8))
    assert e.value.code == L.E_CAPACITY
    eng.close()
