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
