"""one named fixture per bit-exactness gotcha.

The reference holds no known-answer vectors for ring ownership, key composition or silo hashes, so each fixture
here states its expected value as derived BY HAND from the .NET semantics the cited reference line relies on (byte
layouts, signed compares, list insertion order), independently of both restatements. The restatements
(`oracle/pyref.py`, `oracle/cpu_ref.cpp`), the C ABI's host functions and, under `-m gpu`, the HIP route kernel
must all produce it. Interpretations both restatements had to make are written next to the fixture that pins them.
"""
import hashlib
import struct

import numpy as np
import pytest

from oracle import cpu_ref, pyref
from orleans_amd import _lib as L
from orleans_amd import engine as E

TCD = pyref.type_code_data(pyref.CAT_GRAIN, 0x1524FEF4)  # ChirperAccount's type code (SURVEY sample)


# ---- 1. Jenkins argument order (UniqueKey.cs:297; BinaryTokenStreamWriter.cs:488-494) ----------------------------
def test_g01_jenkins_argument_order():
    """The u64 path hashes (TypeCodeData, N0, N1) in that order; the KeyExt byte path serializes N0, N1,
    TypeCodeData (LE8 each), then the string as int32 length + UTF-8."""
    k = pyref.Key(TCD, 0x0102030405060708, 0x1112131415161718)
    assert pyref.uniform_hash(k) == pyref.jenkins_u64(k.tcd, k.n0, k.n1)
    assert pyref.uniform_hash(k) != pyref.jenkins_u64(k.n0, k.n1, k.tcd)  # the order matters
    assert cpu_ref.jenkins_u64(k.tcd, k.n0, k.n1) == pyref.uniform_hash(k)
    kx = pyref.Key(pyref.type_code_data(pyref.CAT_KEYEXT_GRAIN, 7), 1, 2, "ab")
    by_hand = (bytes([1, 0, 0, 0, 0, 0, 0, 0]) + bytes([2, 0, 0, 0, 0, 0, 0, 0]) +
               struct.pack("<Q", kx.tcd) + bytes([2, 0, 0, 0]) + b"ab")
    assert pyref.serialize_unique_key(kx) == by_hand
    assert pyref.uniform_hash(kx) == pyref.jenkins_bytes(by_hand) == cpu_ref.jenkins_bytes(by_hand)
    assert E.keyext_uniform_hash(kx.tcd, 1, 2, "ab") == pyref.uniform_hash(kx)
    # `hi(u) = (uint)((u ^ (uint)u) >> 32)` (JenkinsHash.cs:133) is u >> 32: (u ^ low32) clears the low word only
    for u in (0, 1, 0xFFFFFFFF, 0x1_0000_0000, 0xDEADBEEF_CAFEBABE, (1 << 64) - 1):
        assert ((u ^ (u & 0xFFFFFFFF)) >> 32) == u >> 32


# ---- 2. Byte-path tail (JenkinsHash.cs:90-112) ---------------------------------------------------------------
def test_g02_byte_path_tail():
    """Lengths 9, 10, 11 put bytes 8, 9, 10 into c at shifts 8, 16, 24 (the low byte of c carries the length):
    appending a byte changes the hash, and a tail byte's position matters."""
    base = bytes(range(1, 9))
    hs = {n: pyref.jenkins_bytes(base + bytes([0xAA] * n)) for n in range(0, 4)}
    assert len(set(hs.values())) == 4
    assert pyref.jenkins_bytes(base + b"\x01\x02\x03") != pyref.jenkins_bytes(base + b"\x03\x02\x01")
    for n in range(0, 30):
        b = bytes((i * 37 + 11) & 0xFF for i in range(n))
        assert pyref.jenkins_bytes(b) == cpu_ref.jenkins_bytes(b) == E.jenkins_bytes(b)


# ---- 3. uniformHashCache == 0 sentinel (UniqueKey.cs:284) -----------------------------------------------------
def test_g03_hash_cache_sentinel_has_no_effect():
    """A cached 0 is recomputed by the reference; the GPU always recomputes. Either way the value is a pure function
    of the key: recomputation is idempotent."""
    k = pyref.Key(TCD, 0, 12345)
    assert pyref.uniform_hash(k) == pyref.uniform_hash(k) == cpu_ref.jenkins_u64(k.tcd, k.n0, k.n1)


# ---- 4. TypeCodeData sign extension (GrainInterfaceMap.cs:431-437, UniqueKey.cs:141) ---------------------------
def test_g04_type_code_sign_extension():
    """int type code widened to long, masked to 56 bits, category in the top byte."""
    assert pyref.type_code_data(3, -1) == 0x03FF_FFFF_FFFF_FFFF
    assert pyref.type_code_data(3, -2 ** 31) == 0x03FF_FFFF_8000_0000
    assert pyref.type_code_data(3, 2 ** 31 - 1) == 0x0300_0000_7FFF_FFFF
    assert pyref.type_code_data(3, 0x1524FEF4) == 0x0300_0000_1524_FEF4
    # generic grains: (hash & 0x00FFFFFF) << 32 added to the type code before the mask
    assert pyref.type_code_data(3, 0x1524FEF4 + ((0xABCDEF12 & 0x00FFFFFF) << 32)) == 0x03CD_EF12_1524_FEF4
    for cat, tc in ((3, -1), (3, 5), (6, -7)):
        assert E.type_code_data(cat, tc) == pyref.type_code_data(cat, tc)


# ---- 5. Guid byte order (UniqueKey.cs:163-165) -----------------------------------------------------------------
def test_g05_guid_byte_order():
    """Guid.ToByteArray() = Data1 LE4, Data2 LE2, Data3 LE2, 8 raw bytes; N0/N1 = LE u64 of bytes [0:8] / [8:16]."""
    g = "00112233-4455-6677-8899-aabbccddeeff"
    assert pyref.guid_to_bytearray(g) == bytes.fromhex("33221100554477668899aabbccddeeff")
    k = pyref.key_from_guid(g, 0x1234)
    assert (k.n0, k.n1) == (0x6677445500112233, 0xFFEEDDCCBBAA9988)
    rows = np.frombuffer(pyref.guid_to_bytearray(g), np.uint8).reshape(1, 16)
    ek = E.grain_keys_from_guid_bytes(0x1234, rows)
    assert (int(ek["n0"][0]), int(ek["n1"][0]), int(ek["tcd"][0])) == (k.n0, k.n1, k.tcd)


# ---- 6. CalculateIdHash (Utils.cs:207-213, SiloAddress.cs:202-203) ---------------------------------------------
def _id_hash_by_hand(text: str) -> int:
    d = hashlib.sha256(text.encode("utf-16-le")).digest()
    h = 0
    for i in range(0, 32, 4):
        h ^= int.from_bytes(d[i:i + 4], "big")
    return h - (1 << 32) if h >= 1 << 31 else h


@pytest.mark.parametrize("ep,gen", [("10.0.0.1:11111", 1), ("10.0.0.8:11111", 1), ("127.0.0.1:30000", -5),
                                    ("[::1]:11111", 123456789)])
def test_g06_calc_id_hash_utf16le_bigendian(ep, gen):
    """SHA-256 over the UTF-16LE string Endpoint.ToString() + Generation.ToString(InvariantCulture) (a negative
    generation keeps its '-'), folded by XOR of 8 big-endian int32 words (hashlib here: a third SHA-256)."""
    exp = _id_hash_by_hand(ep + str(gen))
    assert pyref.silo_consistent_hash(ep, gen) == exp
    assert E.silo_consistent_hash(ep, gen) == exp


# ---- 7. signed ring compare, insert before equals (LocalGrainDirectory.cs:261, 467, 481) ------------------------
# Ring by hand: A (silo 0) hash -100, B (silo 1) hash 5, then C (silo 2) hash 5 is inserted BEFORE B (FindLastIndex of
# h < 5 is A's index, +1), D (silo 3) hash 2^31 - 1.  List order [A, C, B, D].  Owner = FindLast(h <= (int)u), else the
# last silo.  Unsigned compares would give other owners for the negative hashes.
RING = [(0, -100), (1, 5), (2, 5), (3, 2 ** 31 - 1)]
RING_CASES = [  # uniform hash (uint32) -> owner, by hand
    (0xFFFFFF00, 3),  # (int) -256: nothing <= -256 -> wrap to the last silo, D
    (0xFFFFFF9C, 0),  # -100: A
    (0x00000004, 0),  # 4: A (C and B are 5)
    (0x00000005, 1),  # 5: the LAST of [A, C, B] with h <= 5 is B (C sits before B)
    (0x00000006, 1),  # 6: B
    (0x7FFFFFFF, 3),  # int.MaxValue: D
    (0x80000000, 3),  # int.MinValue: wrap to D
]
# excludeMySelf (me = D not running, excludeThisSiloIfStopping): FindLast skips D; the wrap picks ring[n-2] = B
RING_EXCL_CASES = [(0x7FFFFFFF, 1), (0xFFFFFF00, 1), (0x00000005, 1), (0xFFFFFF9C, 0)]


def _pyref_ring():
    r = pyref.Ring()
    for s, h in RING:
        r.add_server(s, h)
    return r


def test_g07_ring_order_and_signed_compare():
    r = _pyref_ring()
    assert [s for _, s in r.entries] == [0, 2, 1, 3]
    o = cpu_ref.Oracle(4)
    for s, h in RING:
        o.add_server(s, h)
    assert [s for _, s in o.ring()] == [0, 2, 1, 3]
    view = pyref.SiloView(running=[True] * 4, functional=[True] * 4)
    key = pyref.Key(TCD, 0, 1)
    for u, exp in RING_CASES:
        assert pyref.calculate_target_silo(r, key, u, 0, view, True) == (exp, pyref.OWN_OK), hex(u)
    stop = pyref.SiloView(running=[True, True, True, False], functional=[True] * 4)
    for u, exp in RING_EXCL_CASES:
        assert pyref.calculate_target_silo(r, key, u, 3, stop, True)[0] == exp, hex(u)
    msgs = _ring_msgs(RING_CASES, sender=0)
    assert list(np.asarray(o.route(msgs)[0]) & 0xFF) == [e for _, e in RING_CASES]
    os_ = cpu_ref.Oracle(4, running=[1, 1, 1, 0])
    for s, h in RING:
        os_.add_server(s, h)
    msgs = _ring_msgs(RING_EXCL_CASES, sender=3)
    assert list(np.asarray(os_.route(msgs, 1)[0]) & 0xFF) == [e for _, e in RING_EXCL_CASES]


def _ring_msgs(cases, sender):
    m = np.zeros(len(cases), L.MSG_DTYPE)
    m["tcd"], m["n1"] = TCD, np.arange(1, len(cases) + 1)
    m["sending_silo"], m["category"] = sender, 2
    m["flags"] = L.HDR_HASH_VALID  # aux carries the uniform hash: the fixture chooses it
    m["aux"] = [u for u, _ in cases]
    return m


# ---- 8. special owners (LocalGrainDirectory.cs:442-493) ---------------------------------------------------------
def test_g08_special_owners():
    """SystemTarget -> the routing silo; the membership-table grain -> the seed (no seed: ArgumentException);
    empty ring -> MyAddress, or null when stopping with excludeThisSiloIfStopping."""
    r = _pyref_ring()
    view = pyref.SiloView(running=[True] * 4, functional=[True] * 4, seed=2)
    assert pyref.calculate_target_silo(r, pyref.key_system_target(12), 0x5, 1, view, True) == (1, pyref.OWN_OK)
    assert pyref.calculate_target_silo(r, pyref.MEMBERSHIP_TABLE_KEY, 0x5, 1, view, True) == (2, pyref.OWN_OK)
    noseed = pyref.SiloView(running=[True] * 4, functional=[True] * 4)
    assert pyref.calculate_target_silo(r, pyref.MEMBERSHIP_TABLE_KEY, 0x5, 1, noseed, True)[1] == pyref.OWN_NO_SEED
    empty = pyref.Ring()
    stopping = pyref.SiloView(running=[False] * 4, functional=[True] * 4)
    assert pyref.calculate_target_silo(empty, pyref.Key(TCD, 0, 1), 0x5, 1, view, True) == (1, pyref.OWN_OK)
    assert pyref.calculate_target_silo(empty, pyref.Key(TCD, 0, 1), 0x5, 1, stopping, True)[1] == pyref.OWN_NULL
    assert pyref.calculate_target_silo(empty, pyref.Key(TCD, 0, 1), 0x5, 1, stopping, False) == (1, pyref.OWN_OK)
    # the membership-table grain's key: Guid 01145FEC-C21E-11E0-9105-D0FB4724019B as a system grain (Constants.cs:66)
    k = pyref.MEMBERSHIP_TABLE_KEY
    assert (k.n0, k.n1) == (0x11E0C21E01145FEC, 0x9B012447FBD00591)
    assert k.category == pyref.CAT_SYSTEM_GRAIN


# ---- 9. Math.Abs(int.MinValue) (OutboundMessageQueue.cs:141) ----------------------------------------------------
def test_g09_abs_int_min_is_an_error():
    """|int.MinValue| overflows in C# (OverflowException): flagged, not wrapped to a queue index."""
    hashes = {0: -2 ** 31, 1: -7}
    assert pyref.outbound_queue(0, 1, 2, hashes, 4) == pyref.OUTQ_OVERFLOW
    assert pyref.outbound_queue(1, 0, 2, hashes, 4) == 7 % 4  # Math.Abs(-7) % 4


# ---- 10. silo uniform hash layout (BinaryTokenStreamWriter.cs:448-486, SiloAddress.cs:223-230) -----------------
def test_g10_silo_uniform_hash_layout():
    """IPv4 = 12 zero bytes + the 4 address bytes (not ::ffff:-mapped), port / generation / extraBit LE4: 28 B."""
    ip16 = bytes(12) + bytes([10, 0, 0, 1])
    by_hand = ip16 + struct.pack("<iii", 11111, 1, 3)
    assert len(by_hand) == 28
    assert pyref.silo_uniform_hash(ip16, 11111, 1, 3) == pyref.jenkins_bytes(by_hand) == E.jenkins_bytes(by_hand)
    mapped = bytes(10) + b"\xff\xff" + bytes([10, 0, 0, 1])
    assert pyref.silo_uniform_hash(mapped, 11111, 1, 3) != pyref.silo_uniform_hash(ip16, 11111, 1, 3)


# ---- 11. nondeterministic reference choices (RandomPlacementDirector.cs:32-65 ...) -------------------------------
def test_g11_deterministic_placement_policies():
    """Random placement is replaced by documented deterministic policies: PreferLocal = the sending silo; hash-spread
    = (uniform hash) mod the number of active silos, in silo-index order."""
    view = pyref.SiloView(running=[True] * 4, functional=[True, False, True, True])
    assert pyref.placement_silo(L.POLICY_PREFER_LOCAL, 2, 0xDEADBEEF, view) == 2
    active = [s for s in range(4) if view.functional[s]]
    assert pyref.placement_silo(L.POLICY_HASH_SPREAD, 2, 0xDEADBEEF, view) == active[0xDEADBEEF % len(active)]


# ---- 12. CalculateGuidHash fold (Utils.cs:227-246, ActivationId.cs:72-83) ---------------------------------------
def test_g12_calc_guid_hash_fold():
    """SHA-256 over UTF-16LE folded into 16 bytes by hash[i % 16] ^= sha[i]; the bytes are the Guid's ToByteArray."""
    text = "10.0.0.1:11111@1"
    d = hashlib.sha256(text.encode("utf-16-le")).digest()
    by_hand = bytes(d[i] ^ d[i + 16] for i in range(16))
    assert pyref.calc_guid_hash(text) == by_hand


# ---- the HIP path on the hand-derived ring fixtures -----------------------------------------------------------
@pytest.mark.gpu
def test_g07_ring_fixtures_on_gpu():
    import torch
    assert torch.cuda.is_available()
    for cases, sender, running, opts in ((RING_CASES, 0, None, 0), (RING_EXCL_CASES, 3, [1, 1, 1, 0], 1)):
        eng = E.GrainDirectoryEngine(n_act=16, dir_capacity=64, max_batch=1024, device=0)
        eng.set_silos(4, running=running)
        for s, h in RING:
            eng.add_server(s, h)
        res = eng.address_messages(_ring_msgs(cases, sender), opts)
        assert list(E.decode_route(res.route).owner) == [e for _, e in cases]
        eng.close()
