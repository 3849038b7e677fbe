"""CPU tests of the f2 wire-codec oracle (oracle/wire_codec.py) and the synthetic frame generator.

The reference's test suite holds no serialized-header fixtures, so the oracle is pinned by
(1) writer/reader round trips over every header value type, (2) the rule table below — one frame per rule, the
expected status written next to it — and (3) the KeyExt uniform hash, which must equal pyref.uniform_hash
(pinned by the golden vectors of tests/golden/).
"""
import random
import struct
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent))
import wire_corpus as C  # noqa: E402

from oracle import wire_codec as W  # noqa: E402
from oracle import pyref as P  # noqa: E402


def _writer_form(v):
    """A parsed value in HeaderWriter's input form."""
    k = v[0]
    if k == "grain":
        return ("grain", v[1])
    if k == "list":
        return ("list", [_writer_form(x) for x in v[1]])
    if k == "actaddr":
        return ("actaddr", v[1], v[2], v[3])
    return v


def test_roundtrip_every_value_type():
    rng = random.Random(5)
    for _ in range(1500):
        items = C.random_headers(rng)
        hdr = W.serialize_headers(items)
        parsed = W.parse_headers(hdr)
        assert list(parsed) == [k for k, _ in items]
        again = W.serialize_headers([(k, _writer_form(v)) for k, v in parsed.items()])
        assert again == hdr


# (frame index in C.edge_corpus(), expected status) — the rules of oracle/wire_codec.py, one by one
EDGE_EXPECT = [
    W.DEC_OK, W.DEC_OK, W.DEC_UNKNOWN_SILO, W.DEC_OK, W.DEC_OK, W.DEC_OK, W.DEC_OK, W.DEC_OK,
    W.DEC_NO_SENDER, W.DEC_NO_TARGET, W.DEC_NO_SENDER, W.DEC_MALFORMED, W.DEC_MALFORMED, W.DEC_MALFORMED,
    W.DEC_OK, W.DEC_MALFORMED, W.DEC_MALFORMED, W.DEC_OK, W.DEC_UNSUPPORTED, W.DEC_UNSUPPORTED, W.DEC_OK,
    W.DEC_UNSUPPORTED, W.DEC_UNSUPPORTED, W.DEC_OK, W.DEC_MALFORMED, W.DEC_OK, W.DEC_OK, W.DEC_MALFORMED,
    W.DEC_OK, W.DEC_MALFORMED, W.DEC_MALFORMED, W.DEC_OK, W.DEC_MALFORMED, W.DEC_MALFORMED, W.DEC_OK,
    W.DEC_MALFORMED, W.DEC_MALFORMED, W.DEC_MALFORMED, W.DEC_MALFORMED, W.DEC_MALFORMED, W.DEC_MALFORMED,
    W.DEC_MALFORMED, W.DEC_MALFORMED, W.DEC_OK, W.DEC_MALFORMED, W.DEC_OK, W.DEC_OK, W.DEC_MALFORMED,
    W.DEC_NO_SENDER, W.DEC_MALFORMED, W.DEC_MALFORMED, W.DEC_OK, W.DEC_OK, W.DEC_UNSUPPORTED, W.DEC_OK,
    W.DEC_MALFORMED, W.DEC_MALFORMED, W.DEC_OK, W.DEC_OK, W.DEC_OK,
]


def test_edge_rules():
    frames = C.edge_corpus()
    assert len(frames) == len(EDGE_EXPECT)
    buf, offs, nb = C.pack(frames)
    st, m = C.oracle_decode(buf, nb, offs)
    assert list(st) == EDGE_EXPECT
    # non-OK records are all zero
    assert (m[st != 0].view(np.uint8) == 0).all()
    # the complete-address frame
    assert m[1]["flags"] == P.HDR_ADDRESS_COMPLETE and m[1]["target_silo"] == 4 and m[1]["sending_silo"] == 1
    assert m[7]["category"] == 0  # absent CATEGORY -> default(Categories) = Ping


def test_keyext_hash_is_uniform_hash():
    for ext in ["a", "acct-42", "été", "中文-key", "x" * 37, " y"]:
        k = P.key_from_long(991, -12345, ext)
        hdr = W.serialize_headers([(W.H_SENDING_SILO, ("silo", C.silo_addr(0))), (W.H_TARGET_GRAIN, ("grain", k))])
        d = W.decode_for_route(hdr, C.silo_index())
        assert d.status == W.DEC_OK and d.flags == P.HDR_HASH_VALID
        assert d.aux == P.uniform_hash(k)


def test_sender_override():
    k = P.key_from_long(5, 1)
    hdr = W.serialize_headers([(W.H_TARGET_GRAIN, ("grain", k))])
    assert W.decode_for_route(hdr, C.silo_index()).status == W.DEC_NO_SENDER
    d = W.decode_for_route(hdr, C.silo_index(), sender_override=6)
    assert d.status == W.DEC_OK and d.sending_silo == 6


def test_framing_bounds():
    f = W.frame(W.serialize_headers([(W.H_TARGET_GRAIN, ("grain", P.key_from_long(5, 1)))]), b"xyz")
    assert W.decode_frames(f, [0], {}, 1)[0].status == W.DEC_OK
    assert W.decode_frames(f[:-1], [0], {}, 1)[0].status == W.DEC_MALFORMED   # body past the buffer
    assert W.decode_frames(f, [len(f) - 4], {}, 1)[0].status == W.DEC_MALFORMED
    neg = struct.pack("<ii", -1, 0) + f[8:]
    assert W.decode_frames(neg, [0], {}, 1)[0].status == W.DEC_MALFORMED


def test_mutations_never_crash_the_oracle():
    frames = C.typed_corpus(300, seed=9)
    mut = C.mutate(frames, 3000, seed=4)
    buf, offs, nb = C.pack(mut)
    st, _ = C.oracle_decode(buf, nb, offs)
    assert set(np.unique(st)) <= {0, 1, 2, 3, 4, 5}
    assert (st == W.DEC_MALFORMED).sum() > 500


@pytest.mark.parametrize("complete_frac,keyext_frac", [(0.0, 0.0), (0.3, 0.2)])
def test_generator_frames_decode_to_the_expected_headers(complete_frac, keyext_frac):
    from orleans_amd import workloads as WL
    cl = WL.balanced_cluster()
    buf, offs, exp = WL.request_frames(cl, 100_000, 3000, complete_frac=complete_frac, keyext_frac=keyext_frac)
    assert len(buf) % 4 == 0
    idx = {(cl.silo_ip16(s), WL.PORT, cl.gens[s]): s for s in range(cl.n_silos)}
    dec = W.decode_frames(bytes(buf), [int(o) for o in offs], idx)
    assert all(d.status == W.DEC_OK for d in dec)
    for d, e in zip(dec, exp):
        assert (d.tcd, d.n0, d.n1, d.sending_silo, d.category, d.flags, d.target_silo) == \
               (int(e["tcd"]), int(e["n0"]), int(e["n1"]), int(e["sending_silo"]), 2, int(e["flags"]),
                int(e["target_silo"]))
    if keyext_frac:
        assert any(d.flags & P.HDR_HASH_VALID for d in dec)
        assert any(d.flags & P.HDR_ADDRESS_COMPLETE for d in dec)


# ---- emit: SetTargetPlacement + .NET Dictionary order --------------------------------------------------------
def _route(status, host=4):
    return (status << 16) | (host << 8)


def _stamp_items(items, status, act_key, new_key=None, grain_types=None):
    hdr = W.serialize_headers(items)
    st, fr = W.stamp_frame(hdr, b"BODY", _route(status), act_key, new_key,
                           {s: C.silo_addr(s) for s in range(8)}, grain_types or {})
    if st != W.STAMP_OK:
        return st, None
    hl = struct.unpack("<i", fr[:4])[0]
    assert fr[8 + hl:] == b"BODY"
    return st, list(W.parse_headers(fr[8:8 + hl]).items())


def test_stamp_new_placement_reuses_freed_slots_lifo():
    tg = P.key_from_long(77, 1234)
    items = [(W.H_CATEGORY, ("int", 2)), (W.H_PRIOR_MESSAGE_ID, ("corr", 5)), (W.H_TARGET_GRAIN, ("grain", tg)),
             (W.H_PRIOR_MESSAGE_TIMES, ("int", 3)), (W.H_SENDING_SILO, ("silo", C.silo_addr(1)))]
    new_act = P.Key(0, 11, 22, None)
    st, out = _stamp_items(items, 1, None, new_act, {1234: "My.Grain"})
    assert st == W.STAMP_OK
    # removed PRIOR_ID (index 1) then PRIOR_TIMES (index 3): TARGET_ACTIVATION takes 3, TARGET_SILO takes 1
    assert [k for k, _ in out] == [W.H_CATEGORY, W.H_TARGET_SILO, W.H_TARGET_GRAIN, W.H_TARGET_ACTIVATION,
                                   W.H_SENDING_SILO, W.H_IS_NEW_PLACEMENT, W.H_NEW_GRAIN_TYPE]
    d = dict(out)
    assert d[W.H_TARGET_ACTIVATION] == ("act", new_act) and d[W.H_TARGET_SILO] == ("silo", C.silo_addr(4))
    assert d[W.H_IS_NEW_PLACEMENT] == ("bool", True) and d[W.H_NEW_GRAIN_TYPE] == ("string", "My.Grain")


def test_stamp_hit_same_activation_keeps_prior_headers():
    tg = P.key_from_long(77, 1234)
    act = P.Key(0, 5, 6, None)
    items = [(W.H_TARGET_ACTIVATION, ("act", act)), (W.H_PRIOR_MESSAGE_ID, ("corr", 5)), (W.H_TARGET_GRAIN, ("grain", tg))]
    st, out = _stamp_items(items, 0, act)
    assert st == W.STAMP_OK
    assert [k for k, _ in out] == [W.H_TARGET_ACTIVATION, W.H_PRIOR_MESSAGE_ID, W.H_TARGET_GRAIN, W.H_TARGET_SILO]
    # a different activation drops PRIOR_MESSAGE_ID; TARGET_SILO then takes its slot
    st, out = _stamp_items(items, 0, P.Key(0, 5, 7, None))
    assert [k for k, _ in out] == [W.H_TARGET_ACTIVATION, W.H_TARGET_SILO, W.H_TARGET_GRAIN]


def test_stamp_statuses():
    tg = P.key_from_long(77, 1234)
    base = [(W.H_TARGET_GRAIN, ("grain", tg))]
    act = P.Key(0, 5, 6, None)
    assert _stamp_items(base, 3, act)[0] == W.STAMP_COMPLETE
    assert _stamp_items(base, 8, act)[0] == W.STAMP_SKIPPED
    assert _stamp_items(base, 1, None, act, {})[0] == W.STAMP_UNSUPPORTED          # no grain type
    assert _stamp_items(base + [(W.H_TARGET_ACTIVATION, ("null",))], 0, act)[0] == W.STAMP_MALFORMED
    assert _stamp_items(base + [(5, ("specified", b"x"))], 0, act)[0] == W.STAMP_UNSUPPORTED
    # a string that is not strict UTF-8 would not re-serialize to its bytes
    hdr = bytearray(W.serialize_headers(base + [(5, ("string", "abcd"))]))
    hdr[hdr.index(b"abcd")] = 0xC3
    st, fr = W.stamp_frame(bytes(hdr), b"", _route(0), act, None, {4: C.silo_addr(4)}, {})
    assert st == W.STAMP_UNSUPPORTED and fr[8:] == bytes(hdr)
    # unknown host silo
    st, _ = W.stamp_frame(W.serialize_headers(base), b"", _route(0, host=9), act, None, {4: C.silo_addr(4)}, {})
    assert st == W.STAMP_UNSUPPORTED


def test_stamped_frame_decodes_as_complete_address():
    tg = P.key_from_long(77, 1234)
    items = [(W.H_CATEGORY, ("int", 2)), (W.H_SENDING_SILO, ("silo", C.silo_addr(1))), (W.H_TARGET_GRAIN, ("grain", tg))]
    st, fr = W.stamp_frame(W.serialize_headers(items), b"", _route(0, host=6), P.Key(0, 1, 2, None), None,
                           {s: C.silo_addr(s) for s in range(8)}, {})
    assert st == W.STAMP_OK
    d = W.decode_frames(fr, [0], C.silo_index())[0]
    assert d.status == W.DEC_OK and d.flags == P.HDR_ADDRESS_COMPLETE and d.target_silo == 6
