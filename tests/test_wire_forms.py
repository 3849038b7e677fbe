"""Exchange record forms on the CPU: the oracle's 8-B (orl_wire8) and 16-B (orl_wire_msg) encoders against the host
decoders the node result uses (orleans_amd.node), and the conditions under which each form exists.  No GPU."""
import numpy as np

from oracle import cpu_ref
from orleans_amd import _lib as L
from orleans_amd import workloads as W
from orleans_amd.node import narrow_records_to_headers, wire_records_to_headers


def _msgs(n=20_000, seed=5):
    cl = W.default_cluster()
    m = W.uniform_messages(cl, 50_000, n, seed=seed)
    rng = np.random.default_rng(seed)
    c = rng.random(n)
    m["flags"][c < 0.05] = L.HDR_ADDRESS_COMPLETE
    m["target_silo"][c < 0.05] = rng.integers(0, 8, int((c < 0.05).sum()))
    m["category"][(c > 0.5) & (c < 0.6)] = 1
    sys_t = (np.uint64(L.CAT_SYSTEM_TARGET) << np.uint64(56)) | np.uint64(12)
    m["tcd"][(c > 0.9)] = sys_t
    return cl, m, sys_t


def test_narrow_roundtrip_and_conditions():
    cl, m, sys_t = _msgs()
    grain_t = int(m["tcd"][0])
    types = [grain_t, int(sys_t)]
    rec, ok = cpu_ref.narrow_encode(m, types)
    assert rec.itemsize == 8 and ok.all()
    back = narrow_records_to_headers(rec.view(np.uint8), types)
    np.testing.assert_array_equal(back, m)
    # each condition that removes the 8-B form
    bad = m.copy()
    bad["n1"][1] = 1 << 32            # N1 needs 64 bits
    bad["n0"][2] = 7                  # a Guid-shaped key
    bad["tcd"][3] = grain_t + 1       # a type that is not in the table
    bad["flags"][4] = L.HDR_HASH_VALID
    bad["category"][5] = 4
    _, ok2 = cpu_ref.narrow_encode(bad, types)
    assert list(np.nonzero(~ok2)[0]) == [1, 2, 3, 4, 5]
    # without the system-target type those messages lose the 8-B form but keep the 16-B one
    _, ok3 = cpu_ref.narrow_encode(m, types[:1])
    is_sys = m["tcd"] == sys_t
    np.testing.assert_array_equal(ok3, ~is_sys)
    assert cpu_ref.wire_encode(m)[1].all()


def test_compact_roundtrip():
    _, m, _ = _msgs(seed=9)
    rec, ok = cpu_ref.wire_encode(m)
    assert ok.all()
    np.testing.assert_array_equal(wire_records_to_headers(rec.view(np.uint8)), m)
    np.testing.assert_array_equal(cpu_ref.wire_decode(rec), m)
