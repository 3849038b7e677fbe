"""Header-frame corpora for the f2 wire codec tests (test infrastructure; builds frames with the oracle's writer).

* ``typed_corpus``   every token type the header reader accepts, in random header dictionaries, plus the
                     routing headers in their valid / null / wrong-typed forms;
* ``edge_corpus``    hand-written edge cases: each MALFORMED / UNSUPPORTED rule of oracle/wire_codec.py;
* ``mutate``         random truncations / byte flips of valid frames (the decoder must agree with the oracle on
                     whatever the bytes say, including the status precedence).
"""
from __future__ import annotations

import random
import struct
from typing import Dict, List, Sequence, Tuple

import numpy as np

from oracle import wire_codec as W
from oracle.pyref import Key, key_from_long, key_from_guid, type_code_data, CAT_GRAIN, CAT_KEYEXT_GRAIN, \
    CAT_SYSTEM_TARGET, CAT_CLIENT, NULL_SILO

N_SILOS = 8
PORT = 11111


def silo_addr(s: int, gen: int = 1) -> W.SiloAddr:
    return (W.ip16_v4(f"10.0.0.{s + 1}"), PORT, gen)


def silo_index(n: int = N_SILOS) -> Dict[W.SiloAddr, int]:
    return {silo_addr(s): s for s in range(n)}


def _rand_key(rng: random.Random, keyext: bool = False) -> Key:
    tc = rng.randrange(-2**31, 2**31)
    if keyext:
        ext = rng.choice(["a", "acct-42", "  x ", "été", "中文-key", "k" * rng.randrange(1, 40)])
        return key_from_long(rng.getrandbits(63), tc, ext)
    if rng.random() < 0.5:
        return key_from_long(rng.getrandbits(64) - 2**63, tc)
    g = "%08x-%04x-%04x-%04x-%012x" % (rng.getrandbits(32), rng.getrandbits(16), rng.getrandbits(16),
                                       rng.getrandbits(16), rng.getrandbits(48))
    return key_from_guid(g, tc)


def _rand_simple(rng: random.Random, depth: int = 0):
    k = rng.randrange(24 if depth < 3 else 23)
    if k == 0: return ("null",)
    if k == 1: return ("bool", rng.random() < 0.5)
    if k == 2: return ("int", rng.randrange(-2**31, 2**31))
    if k == 3: return ("uint", rng.getrandbits(32))
    if k == 4: return ("short", rng.randrange(-2**15, 2**15))
    if k == 5: return ("ushort", rng.getrandbits(16))
    if k == 6: return ("long", rng.getrandbits(64) - 2**63)
    if k == 7: return ("ulong", rng.getrandbits(64))
    if k == 8: return ("byte", rng.getrandbits(8))
    if k == 9: return ("sbyte", rng.randrange(-128, 128))
    if k == 10: return ("double", rng.random())
    if k == 11: return ("decimal", struct.pack("<iiiI", 5, 0, 0, (rng.randrange(29) << 16) | (rng.getrandbits(1) << 31)))
    if k == 12: return ("string", rng.choice([None, "", "hello", "über", "x" * rng.randrange(60)]))
    if k == 13: return ("char", rng.randrange(0, 0x8000))
    if k == 14: return ("guid", rng.randbytes(16))
    if k == 15: return ("date", (rng.getrandbits(1) << 62) | rng.randrange(0, W.DATETIME_MAX_TICKS + 1))
    if k == 16: return ("timespan", rng.getrandbits(64) - 2**63)
    if k == 17: return ("ip", rng.randbytes(16))
    if k == 18: return ("ipep", rng.randbytes(16), rng.randrange(65536))
    if k == 19: return ("object",)
    if k == 20: return ("act", _rand_key(rng))
    if k == 21: return ("corr", rng.getrandbits(64) - 2**63)
    if k == 22: return ("actaddr", rng.choice([None, silo_addr(rng.randrange(N_SILOS))]), _rand_key(rng),
                        rng.choice([None, _rand_key(rng)]))
    return ("list", [_rand_simple(rng, depth + 1) for _ in range(rng.randrange(4))])


def random_headers(rng: random.Random) -> List[Tuple[int, tuple]]:
    """A header dictionary: routing headers in valid / null / wrong-typed / absent forms plus filler headers."""
    items: Dict[int, tuple] = {}
    r = rng.random
    if r() < 0.9:
        items[W.H_CATEGORY] = ("int", rng.choice([0, 1, 2, 2, 2])) if r() < 0.95 else rng.choice(
            [("null",), ("long", 2), ("int", 300), ("int", -1)])
    if r() < 0.95:
        items[W.H_SENDING_SILO] = ("silo", silo_addr(rng.randrange(N_SILOS))) if r() < 0.93 else rng.choice(
            [("null",), ("silo", silo_addr(3, gen=99)), ("int", 5)])
    if r() < 0.95:
        items[W.H_TARGET_GRAIN] = ("grain", _rand_key(rng, keyext=r() < 0.25)) if r() < 0.95 else rng.choice(
            [("null",), ("act", _rand_key(rng)), ("int", 1)])
    if r() < 0.35:
        items[W.H_TARGET_SILO] = ("silo", silo_addr(rng.randrange(N_SILOS))) if r() < 0.93 else rng.choice(
            [("null",), ("silo", silo_addr(2, gen=7)), ("string", "x")])
    if r() < 0.35:
        items[W.H_TARGET_ACTIVATION] = ("act", _rand_key(rng)) if r() < 0.93 else rng.choice(
            [("null",), ("grain", _rand_key(rng))])
    for _ in range(rng.randrange(8)):
        k = rng.choice([1, 2, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 21, 25, 26, 27, 28, 29, 30,
                        77, 200, 255])
        if k not in items:
            items[k] = _rand_simple(rng)
    keys = list(items)
    rng.shuffle(keys)
    return [(k, items[k]) for k in keys]


def typed_corpus(n: int, seed: int = 7) -> List[bytes]:
    rng = random.Random(seed)
    return [W.frame(W.serialize_headers(random_headers(rng)), rng.randbytes(rng.randrange(0, 40))) for _ in range(n)]


def _hdr(items, extra: bytes = b"") -> bytes:
    return W.serialize_headers(items) + extra


def edge_corpus() -> List[bytes]:
    """One frame per rule of the oracle (and the boundary on each side of it)."""
    k = key_from_long(12345, 77)
    kx = key_from_long(9, 77, "ext")
    base = [(W.H_CATEGORY, ("int", 2)), (W.H_SENDING_SILO, ("silo", silo_addr(1))), (W.H_TARGET_GRAIN, ("grain", k))]
    F = W.frame
    out = [
        F(_hdr(base)),                                                              # OK
        F(_hdr(base + [(W.H_TARGET_SILO, ("silo", silo_addr(4))), (W.H_TARGET_ACTIVATION, ("act", k))])),  # complete
        F(_hdr(base + [(W.H_TARGET_SILO, ("silo", silo_addr(4, 5))), (W.H_TARGET_ACTIVATION, ("act", k))])),  # unknown ts
        F(_hdr(base + [(W.H_TARGET_SILO, ("silo", silo_addr(4, 5)))])),             # unknown ts, not complete: OK
        F(_hdr(base + [(W.H_TARGET_ACTIVATION, ("act", k))])),                      # no target silo: not complete
        F(_hdr(base[:2] + [(W.H_TARGET_GRAIN, ("grain", kx))])),                     # KeyExt hash
        F(_hdr(base[:2] + [(W.H_TARGET_GRAIN, ("grain", key_from_long(9, 77, "é中")))])),
        F(_hdr(base[1:])),                                                          # no category: Ping
        F(_hdr(base[:1] + base[2:])),                                               # no sender
        F(_hdr(base[:2])),                                                          # no target
        F(_hdr(base[:1] + [(W.H_SENDING_SILO, ("null",))] + base[2:])),
        F(_hdr(base[:1] + [(W.H_SENDING_SILO, ("int", 3))] + base[2:])),            # sender cast fails
        F(_hdr([(W.H_CATEGORY, ("null",))] + base[1:])),                            # category cast fails
        F(_hdr([(W.H_CATEGORY, ("long", 2))] + base[1:])),
        F(_hdr([(W.H_CATEGORY, ("int", 255))] + base[1:])),
        F(_hdr([(W.H_CATEGORY, ("int", 256))] + base[1:])),
        F(_hdr(base + [(W.H_TARGET_SILO, ("int", 1))])),                            # target silo cast fails
        F(_hdr(base + [(W.H_TARGET_SILO, ("null",)), (W.H_TARGET_ACTIVATION, ("act", k))])),
        F(_hdr(base + [(5, ("specified", b"\x01\x02"))])),                          # SpecifiedType -> host
        F(_hdr(base + [(5, ("dict", [(1, ("int", 1))]))])),                         # nested dict -> host
        F(_hdr(base + [(5, ("list", [("list", [("list", [("int", 1)] * 3)] * 2), ("string", "s")]))])),
        F(_hdr(base + [(5, ("list", [("specified", b"")]))])),
        F(_hdr(base + [(5, ("date", 1 << 63))])),                                   # local DateTime -> host
        F(_hdr(base + [(5, ("date", W.DATETIME_MAX_TICKS))])),
        F(_hdr(base + [(5, ("date", W.DATETIME_MAX_TICKS + 1))])),
        F(_hdr(base + [(5, ("date", (1 << 62) | W.DATETIME_MAX_TICKS))])),
        F(_hdr(base + [(5, ("char", 0x7FFF))])),
        F(_hdr(base + [(5, ("raw", bytes([W.T_CHAR, 0x00, 0x80])))])),              # negative char
        F(_hdr(base + [(5, ("decimal", struct.pack("<iiiI", 1, 2, 3, 28 << 16)))])),
        F(_hdr(base + [(5, ("decimal", struct.pack("<iiiI", 1, 2, 3, 29 << 16)))])),
        F(_hdr(base + [(5, ("decimal", struct.pack("<iiiI", 1, 2, 3, 1)))])),
        F(_hdr(base + [(5, ("ipep", bytes(16), 65535))])),
        F(_hdr(base + [(5, ("raw", bytes([W.T_IPEP]) + bytes(16) + struct.pack("<i", 65536)))])),
        F(_hdr(base + [(5, ("raw", bytes([W.T_SILO]) + bytes(16) + struct.pack("<ii", -1, 0)))])),
        F(_hdr(base + [(5, ("string", None))])),
        F(_hdr(base + [(5, ("raw", bytes([W.T_STRING]) + struct.pack("<i", -2)))])),
        F(_hdr(base + [(5, ("raw", bytes([W.T_LIST]) + struct.pack("<i", -1)))])),
        F(_hdr(base + [(5, ("raw", bytes([1, 0, 0, 0, 0])))])),                     # Reference token: rejected
        F(_hdr(base + [(5, ("raw", bytes([2])))])),                                 # Fallback token
        F(_hdr(base + [(5, ("raw", bytes([45]) + bytes(28)))])),                    # RequestId: not a header type
        F(_hdr(base + [(W.H_CATEGORY, ("int", 2))])),                               # duplicate key
        F(_hdr(base + [(5, ("act", Key(type_code_data(CAT_KEYEXT_GRAIN, 1), 0, 5, None)))])),   # KeyExt w/o ext
        F(_hdr(base + [(5, ("act", Key(type_code_data(CAT_KEYEXT_GRAIN, 1), 0, 5, " \t　")))])),  # blank ext
        F(_hdr(base + [(5, ("act", Key(type_code_data(CAT_KEYEXT_GRAIN, 1), 0, 5, " \t　x")))])),
        F(_hdr(base + [(5, ("act", Key(type_code_data(CAT_GRAIN, 1), 0, 5, "")))])),  # ext on non-KeyExt
        F(_hdr(base + [(5, ("actaddr", None, k, None))])),
        F(_hdr(base + [(5, ("actaddr", silo_addr(2), kx, k))])),
        F(b"\x33" + _hdr(base)[1:]),                                                # bad intro token
        F(_hdr([]) ),                                                               # empty dict: no target
        F(b"\x32" + struct.pack("<i", -1)),                                         # negative count
        F(_hdr(base)[:-3]),                                                         # truncated header
        F(_hdr(base), b"body"),
        F(_hdr(base) + b"\x00\x00trailing"),                                        # trailing bytes ignored
    ]
    # invalid UTF-8 KeyExt on the target grain (hash path -> host) and on another header (fine)
    bad = bytearray(_hdr(base[:2] + [(W.H_TARGET_GRAIN, ("grain", key_from_long(9, 77, "abcd")))]))
    i = bytes(bad).index(b"abcd")
    bad[i + 1] = 0xC0
    out.append(F(bytes(bad)))
    bad2 = bytearray(_hdr(base + [(5, ("act", key_from_long(9, 77, "abcd")))]))
    i = bytes(bad2).index(b"abcd")
    bad2[i + 2] = 0xFF
    out.append(F(bytes(bad2)))
    for ext in ["   ", "\u0085", "᠎", "퟿", "\U0001f600"]:
        out.append(F(_hdr(base[:2] + [(W.H_TARGET_GRAIN, ("grain", key_from_long(3, 77, ext)))])))
    return out


def mutate(frames: Sequence[bytes], n: int, seed: int = 11) -> List[bytes]:
    """Random damage: truncate the header (keeping the length prefix consistent or not), flip a byte, or set a
    length field to garbage."""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        f = bytearray(rng.choice(frames))
        hl = struct.unpack("<i", f[:4])[0]
        m = rng.randrange(5)
        if m == 0 and hl > 1:       # consistent truncation
            cut = rng.randrange(1, hl)
            f = bytearray(struct.pack("<ii", cut, 0)) + f[8:8 + cut]
        elif m == 1 and hl > 0:     # byte flip inside the header
            j = 8 + rng.randrange(hl)
            f[j] = rng.getrandbits(8)
        elif m == 2 and hl > 0:     # several flips
            for _ in range(rng.randrange(2, 6)):
                j = 8 + rng.randrange(hl)
                f[j] ^= 1 << rng.randrange(8)
        elif m == 3:                # garbage header length
            f[0:4] = struct.pack("<i", rng.choice([-1, hl + 1, hl - 1, 2**31 - 1, 0]))
        else:                       # garbage body length
            f[4:8] = struct.pack("<i", rng.choice([-5, 1 << 20, 3]))
        out.append(bytes(f))
    return out


def pack(frames: Sequence[bytes], align_gap: bool = True, seed: int = 3):
    """Frames back to back in one buffer (random 0-3 byte gaps so frames start at any alignment); offsets u64.
    The last frame's lengths may point past the buffer (the decoder must say MALFORMED, not read past it)."""
    rng = random.Random(seed)
    buf = bytearray()
    offs = []
    for f in frames:
        if align_gap:
            buf += bytes(rng.randrange(4))
        offs.append(len(buf))
        buf += f
    nbytes = len(buf)
    buf += bytes((-len(buf)) % 4)
    return np.frombuffer(bytes(buf), np.uint8).copy(), np.array(offs, np.uint64), nbytes


def oracle_decode(buf: np.ndarray, nbytes: int, offs: np.ndarray, sender_override: int = W.SENDER_FROM_HEADER,
                  n_silos: int = N_SILOS):
    """oracle/wire_codec.decode_frames -> (status u8[n], MSG_DTYPE records)."""
    from orleans_amd import _lib as L
    dec = W.decode_frames(bytes(buf[:nbytes]), [int(o) for o in offs], silo_index(n_silos), sender_override)
    st = np.array([d.status for d in dec], np.uint8)
    m = np.zeros(len(dec), L.MSG_DTYPE)
    for i, d in enumerate(dec):
        m[i] = (d.tcd, d.n0, d.n1, d.sending_silo, d.category, d.flags, d.target_silo, d.aux)
    return st, m
