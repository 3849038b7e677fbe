"""Oracle for SURVEY §8(f) f2: the message header wire codec — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the product path
(orleans_amd/) never does.

Two halves, both CPU restatements of the reference (src/Orleans/Serialization, src/Orleans/Messaging):

* ``HeaderWriter`` / ``serialize_headers`` / ``frame`` — the sender side: Message.Serialize_Impl
  (Message.cs:915-951: int32 header length, int32 body length, header bytes, body bytes) over
  SerializationManager.SerializeMessageHeaders (SerializationManager.cs:1692-1770: token StringObjDict, int32
  count, then per header a byte key and the value: enums as Int, simple objects through
  BinaryTokenStreamWriter's token writers, nested dictionaries / lists as StringObjDict / ObjList, anything else
  as SpecifiedType + its serializer).  Used to build test frames.

* ``parse_headers`` / ``decode_for_route`` — the receiver side the GPU decoder is checked against:
  DeserializeMessageHeaders (SerializationManager.cs:1773-1853) over BinaryTokenStreamReader.TryReadSimpleType
  (BinaryTokenStreamReader.cs:489-582) and the readers it calls (ReadString :270-289, ReadIPAddress :357-390,
  ReadIPEndPoint :392-397, ReadSiloAddress :401-406, ReadUniqueKey :424-431 with UniqueKey.ValidateKeyExt
  UniqueKey.cs:328-350, ReadActivationAddress :441-454, ReadDecimal :254-266, ReadChar :331-335), then the
  Message getters the routing path calls: Category (Message.cs:149, GetScalarHeader :650-658 — an unboxing cast),
  TargetSilo / SendingSilo (:199-203, :251-255 — a reference cast), TargetGrain / TargetActivation (:211, :221,
  GetSimpleHeader :660-666 — wrong types read as null) and TargetAddress.IsComplete (:229-231).

Where the reference throws, the decoder reports MALFORMED; where the reference would hand the bytes to a
registered serializer (SpecifiedType) or the result depends on the host (local-kind DateTime: the host time
zone), it reports UNSUPPORTED — the host decodes those messages with the full serializer.  Documented
restrictions of the device decoder (also UNSUPPORTED, never a silent difference): a StringObjDict nested inside
a header value, and a TARGET_GRAIN KeyExt that is not strict
UTF-8 (its uniform hash re-encodes the decoded .NET string, UniqueKey.cs:288-294, so the wire bytes are not
the hashed bytes).

Parity anchoring: the reference's own tests hold no serialized header fixtures; the writer is pinned
by the token table (SerializationTokenType.cs:30-109) and by round-trip property tests (tests/test_wire_codec.py).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from .pyref import Key, NULL_SILO, HDR_ADDRESS_COMPLETE, HDR_HASH_VALID, CAT_KEYEXT_GRAIN, jenkins_bytes, \
    serialize_unique_key

# SerializationTokenType (SerializationTokenType.cs:30-109)
T_NULL, T_REFERENCE, T_FALLBACK, T_TRUE, T_FALSE = 0, 1, 2, 3, 4
T_INT, T_SHORT, T_LONG, T_SBYTE, T_UINT, T_USHORT, T_ULONG, T_BYTE = 11, 12, 13, 14, 15, 16, 17, 18
T_FLOAT, T_DOUBLE, T_DECIMAL, T_STRING, T_CHAR, T_GUID, T_DATE, T_TIMESPAN = 19, 20, 21, 22, 23, 24, 25, 26
T_IPADDR, T_IPEP, T_OBJECT = 27, 28, 29
T_GRAIN, T_ACT, T_SILO, T_ACTADDR, T_CORR, T_REQID = 40, 41, 42, 43, 44, 45
T_DICT, T_LIST = 50, 51
T_SPECIFIED = 97

# Message.Header (Message.cs:29-70) — the ones the routing path reads
H_CATEGORY = 3
H_SENDING_SILO = 20
H_TARGET_ACTIVATION = 22
H_TARGET_GRAIN = 23
H_TARGET_SILO = 24

# per-message decode status (include/orleans_route.h ORL_DEC_*)
DEC_OK = 0
DEC_UNSUPPORTED = 1
DEC_MALFORMED = 2
DEC_UNKNOWN_SILO = 3
DEC_NO_TARGET = 4
DEC_NO_SENDER = 5

LENGTH_HEADER_SIZE = 8                    # Message.LENGTH_HEADER_SIZE, Message.cs:87
DATETIME_MAX_TICKS = 3155378975999999999  # DateTime.MaxValue.Ticks
SENDER_FROM_HEADER = 0xFF

# ---------------------------------------------------------------------------------------
# values: ("null",) ("bool", b) ("int", v) ("uint", v) ("short", v) ("ushort", v) ("long", v) ("ulong", v)
# ("byte", v) ("sbyte", v) ("float", f) ("double", f) ("floatbits", u32) ("doublebits", u64) ("decimal", bytes16) ("string", s|None) ("char", u16)
# ("guid", bytes16) ("date", i64 binary) ("timespan", i64) ("ip", bytes16) ("ipep", bytes16, port)
# ("object",) ("grain", Key) ("act", Key) ("silo", SiloAddr) ("actaddr", SiloAddr|None, Key, Key|None)
# ("corr", i64) ("list", [values]) ("dict", [(key, value)]) ("specified", raw bytes after the token)
# ("raw", bytes) — arbitrary bytes, for malformed-stream tests
# ---------------------------------------------------------------------------------------
SiloAddr = Tuple[bytes, int, int]  # (16-byte serialized IP, port, generation)
SILO_ZERO: SiloAddr = (bytes(16), 0, 0)   # SiloAddress.Zero = New(IPEndPoint(IPAddress.Any, 0), 0)
ACT_ZERO = Key(0, 0, 0, None)              # ActivationId.Zero = GetActivationId(UniqueKey.Empty)


def ip16_v4(dotted: str) -> bytes:
    """BinaryTokenStreamWriter.Write(IPAddress) for IPv4: 12 zero bytes + the 4 address bytes (:455-469)."""
    return bytes(12) + bytes(int(x) for x in dotted.split("."))


class HeaderWriter:
    """The token writers SerializeMessageHeaders uses (BinaryTokenStreamWriter.cs; SerializationManager.cs:1711-1770)."""

    def __init__(self):
        self.out = bytearray()

    def tok(self, t: int):
        self.out.append(t & 0xFF)

    def i32(self, v: int):
        self.out += struct.pack("<i", v)

    def string(self, s: Optional[str]):
        """Write(string): int32 length (null -> -1) + UTF-8 (BinaryTokenStreamWriter.cs:237-250)."""
        if s is None:
            self.i32(-1)
        else:
            b = s.encode("utf-8")
            self.i32(len(b))
            self.out += b

    def silo(self, s: Optional[SiloAddr]):
        ip, port, gen = s if s is not None else SILO_ZERO
        self.out += ip + struct.pack("<ii", port, gen)   # Write(SiloAddress) :482-486

    def value(self, v):
        kind = v[0]
        fixed = {"int": (T_INT, "<i"), "uint": (T_UINT, "<I"), "short": (T_SHORT, "<h"), "ushort": (T_USHORT, "<H"),
                 "long": (T_LONG, "<q"), "ulong": (T_ULONG, "<Q"), "byte": (T_BYTE, "<B"), "sbyte": (T_SBYTE, "<b"),
                 "float": (T_FLOAT, "<f"), "double": (T_DOUBLE, "<d"), "char": (T_CHAR, "<H"),
                 "floatbits": (T_FLOAT, "<I"), "doublebits": (T_DOUBLE, "<Q"),
                 "date": (T_DATE, "<Q"), "timespan": (T_TIMESPAN, "<q"), "corr": (T_CORR, "<q")}
        if kind in fixed:
            t, f = fixed[kind]
            self.tok(t)
            self.out += struct.pack(f, v[1] & 0xFFFFFFFFFFFFFFFF if kind == "date" else v[1])
        elif kind == "null":
            self.tok(T_NULL)
        elif kind == "bool":
            self.tok(T_TRUE if v[1] else T_FALSE)
        elif kind == "object":
            self.tok(T_OBJECT)
        elif kind in ("decimal", "guid", "ip"):
            self.tok({"decimal": T_DECIMAL, "guid": T_GUID, "ip": T_IPADDR}[kind])
            assert len(v[1]) == 16
            self.out += v[1]
        elif kind == "ipep":
            self.tok(T_IPEP)
            self.out += v[1] + struct.pack("<i", v[2])
        elif kind == "string":
            self.tok(T_STRING)
            self.string(v[1])
        elif kind in ("grain", "act"):
            self.tok(T_GRAIN if kind == "grain" else T_ACT)
            self.out += serialize_unique_key(v[1])
        elif kind == "silo":
            self.tok(T_SILO)
            self.silo(v[1])
        elif kind == "actaddr":     # Write(ActivationAddress) :472-479: silo ?? Zero, grain, activation ?? Zero
            self.tok(T_ACTADDR)
            self.silo(v[1])
            self.out += serialize_unique_key(v[2])
            self.out += serialize_unique_key(v[3] if v[3] is not None else ACT_ZERO)
        elif kind == "list":        # SerializeMessageHeaderListHelper :1722-1728
            self.tok(T_LIST)
            self.i32(len(v[1]))
            for x in v[1]:
                self.value(x)
        elif kind == "dict":        # SerializeMessageHeaderDictHelper :1711-1720
            self.dict(v[1])
        elif kind == "specified":
            self.tok(T_SPECIFIED)
            self.out += v[1]
        elif kind == "raw":
            self.out += v[1]
        else:
            raise ValueError(kind)

    def dict(self, items: Sequence[Tuple[int, tuple]]):
        self.tok(T_DICT)
        self.i32(len(items))
        for k, v in items:
            self.out.append(k & 0xFF)
            self.value(v)


def serialize_headers(items: Sequence[Tuple[int, tuple]]) -> bytes:
    """SerializeMessageHeaders(headers): Dictionary enumeration order = insertion order (no removals)."""
    w = HeaderWriter()
    w.dict(items)
    return bytes(w.out)


def frame(header: bytes, body: bytes = b"") -> bytes:
    """Message.Serialize_Impl, non-batching (Message.cs:941-948)."""
    return struct.pack("<ii", len(header), len(body)) + header + body


# ---------------------------------------------------------------------------------------
# receiver side
# ---------------------------------------------------------------------------------------
class DecodeError(Exception):
    def __init__(self, status: int, why: str):
        super().__init__(why)
        self.status = status


_WS_SINGLE = {0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20, 0x85, 0xA0, 0x1680, 0x2028, 0x2029, 0x202F, 0x205F, 0x3000}


def _is_null_or_whitespace(s: Optional[str]) -> bool:
    """string.IsNullOrWhiteSpace with Char.IsWhiteSpace's set (U+0009-000D, 0020, 0085, 00A0, 1680, 2000-200A,
    2028, 2029, 202F, 205F, 3000)."""
    if s is None:
        return True
    return all(ord(ch) in _WS_SINGLE or 0x2000 <= ord(ch) <= 0x200A for ch in s)


def _strict_utf8(b: bytes) -> Optional[str]:
    try:
        return b.decode("utf-8", errors="strict")
    except UnicodeDecodeError:
        return None


class _Reader:
    """BinaryTokenStreamReader over one message's header bytes (reads past the end throw, CheckLength :115-131)."""

    def __init__(self, buf: bytes):
        self.b = buf
        self.p = 0

    def take(self, n: int) -> bytes:
        if n < 0 or self.p + n > len(self.b):
            raise DecodeError(DEC_MALFORMED, "read past end of header")
        r = self.b[self.p:self.p + n]
        self.p += n
        return r

    def u8(self) -> int:
        return self.take(1)[0]

    def i32(self) -> int:
        return struct.unpack("<i", self.take(4))[0]

    def string_bytes(self) -> Optional[bytes]:
        n = self.i32()
        if n == -1:
            return None
        if n < 0:
            raise DecodeError(DEC_MALFORMED, "negative string length")
        return self.take(n)

    def unique_key(self):
        """ReadUniqueKey :424-431 + ValidateKeyExt (UniqueKey.cs:328-350); returns (Key, serialized bytes, utf8_ok)."""
        start = self.p
        n0, n1, tcd = struct.unpack("<QQQ", self.take(24))
        ext = self.string_bytes()
        text = None if ext is None else ext.decode("utf-8", errors="replace")
        cat = (tcd >> 56) & 0xFF
        if cat == CAT_KEYEXT_GRAIN:
            if _is_null_or_whitespace(text):
                raise DecodeError(DEC_MALFORMED, "KeyExt grain with null/blank extension")
        elif ext is not None:
            raise DecodeError(DEC_MALFORMED, "extension on a non-KeyExt key")
        utf8_ok = ext is None or _strict_utf8(ext) is not None
        return Key(tcd, n0, n1, text), self.b[start:self.p], utf8_ok

    def silo(self) -> SiloAddr:
        ip = self.take(16)
        port, gen = struct.unpack("<ii", self.take(8))
        if port < 0 or port > 65535:   # new IPEndPoint(addr, port) range check
            raise DecodeError(DEC_MALFORMED, "port out of range")
        return ip, port, gen


def _read_value(r: _Reader, depth: int = 0):
    """DeserializeMessageHeaderHelper (:1833-1853) -> a tagged value as in HeaderWriter."""
    t = r.u8()
    if t == T_NULL:
        return ("null",)
    if t in (T_TRUE, T_FALSE):
        return ("bool", t == T_TRUE)
    if t == T_OBJECT:
        return ("object",)
    # floats keep their bits (BitConverter.ToSingle / GetBytes round-trip every pattern, signalling NaNs too;
    # Python's float32 unpack would quiet them)
    fixed = {T_INT: ("int", "<i"), T_UINT: ("uint", "<I"), T_SHORT: ("short", "<h"), T_USHORT: ("ushort", "<H"),
             T_LONG: ("long", "<q"), T_ULONG: ("ulong", "<Q"), T_BYTE: ("byte", "<B"), T_SBYTE: ("sbyte", "<b"),
             T_FLOAT: ("floatbits", "<I"), T_DOUBLE: ("doublebits", "<Q"), T_TIMESPAN: ("timespan", "<q"),
             T_CORR: ("corr", "<q")}
    if t in fixed:
        kind, f = fixed[t]
        return (kind, struct.unpack(f, r.take(struct.calcsize(f)))[0])
    if t == T_CHAR:        # Convert.ToChar(short) throws for negative values
        v = struct.unpack("<h", r.take(2))[0]
        if v < 0:
            raise DecodeError(DEC_MALFORMED, "negative char")
        return ("char", v)
    if t == T_DECIMAL:     # new decimal(int[]): flags must be sign|scale with scale <= 28
        raw = r.take(16)
        flags = struct.unpack("<I", raw[12:16])[0]
        if flags & 0x7F00FFFF or ((flags >> 16) & 0xFF) > 28:
            raise DecodeError(DEC_MALFORMED, "invalid decimal")
        return ("decimal", raw)
    if t == T_DATE:        # DateTime.FromBinary
        v = struct.unpack("<q", r.take(8))[0]
        if v & (1 << 63):
            raise DecodeError(DEC_UNSUPPORTED, "local-kind DateTime depends on the host time zone")
        if (v & 0x3FFFFFFFFFFFFFFF) > DATETIME_MAX_TICKS:
            raise DecodeError(DEC_MALFORMED, "DateTime ticks out of range")
        return ("date", v)
    if t in (T_GUID, T_IPADDR):
        return ("guid" if t == T_GUID else "ip", r.take(16))
    if t == T_IPEP:
        ip = r.take(16)
        port = r.i32()
        if port < 0 or port > 65535:
            raise DecodeError(DEC_MALFORMED, "port out of range")
        return ("ipep", ip, port)
    if t == T_STRING:
        b = r.string_bytes()
        return ("string", None if b is None else b.decode("utf-8", errors="replace"))
    if t == T_GRAIN:
        k, raw, ok = r.unique_key()
        return ("grain", k, raw, ok)
    if t == T_ACT:
        return ("act", r.unique_key()[0])
    if t == T_SILO:
        return ("silo", r.silo())
    if t == T_ACTADDR:
        s = r.silo()
        g = r.unique_key()[0]
        a = r.unique_key()[0]
        return ("actaddr", None if s == SILO_ZERO else s, g, None if a == ACT_ZERO else a)
    if t == T_LIST:
        n = r.i32()
        if n < 0:
            raise DecodeError(DEC_MALFORMED, "negative list count")
        return ("list", [_read_value(r, depth + 1) for _ in range(n)])
    if t == T_DICT:
        raise DecodeError(DEC_UNSUPPORTED, "nested header dictionary")
    if t == T_SPECIFIED:
        raise DecodeError(DEC_UNSUPPORTED, "SpecifiedType value (registered serializer)")
    raise DecodeError(DEC_MALFORMED, f"unexpected token {t}")


def parse_headers(hdr: bytes) -> Dict[int, tuple]:
    """DeserializeMessageHeaders (:1773-1831): intro token, int32 count, count x (byte key, value);
    Dictionary.Add throws on a duplicate key.  Bytes after the dictionary are not read."""
    return parse_headers_end(hdr)[0]


def parse_headers_end(hdr: bytes):
    """parse_headers + the offset one past the dictionary's last byte."""
    r = _Reader(hdr)
    if r.u8() != T_DICT:
        raise DecodeError(DEC_MALFORMED, "introductory token is not StringObjDict")
    n = r.i32()
    if n < 0:
        raise DecodeError(DEC_MALFORMED, "negative header count")
    out: Dict[int, tuple] = {}
    for _ in range(n):
        k = r.u8()
        v = _read_value(r)
        if k in out:
            raise DecodeError(DEC_MALFORMED, "duplicate header key")
        out[k] = v
    return out, r.p


@dataclass
class Decoded:
    status: int
    tcd: int = 0
    n0: int = 0
    n1: int = 0
    sending_silo: int = 0
    category: int = 0
    flags: int = 0
    target_silo: int = 0
    aux: int = 0


def decode_for_route(hdr: bytes, silo_index: Dict[SiloAddr, int], sender_override: int = SENDER_FROM_HEADER) -> Decoded:
    """One header -> the orl_msg_hdr the routing path reads, or a status.  Semantic checks in this order (the
    getters Dispatcher.AddressMessage / the outbound queue call): Category cast, TargetSilo cast, SendingSilo
    (cast, null, unknown), TargetGrain null, complete address with an unknown TargetSilo.  A non-OK message's
    record is all zero."""
    try:
        h = parse_headers(hdr)
    except DecodeError as e:
        return Decoded(e.status)
    cat = h.get(H_CATEGORY)
    if cat is None:
        category = 0                              # default(Categories) = Ping
    elif cat[0] != "int" or not 0 <= cat[1] <= 255:
        return Decoded(DEC_MALFORMED)             # unboxing cast of a non-int / null; > 255 not representable
    else:
        category = cat[1]
    ts = h.get(H_TARGET_SILO)
    if ts is not None and ts[0] not in ("silo", "null"):
        return Decoded(DEC_MALFORMED)             # (SiloAddress)GetHeader(TARGET_SILO)
    if sender_override == SENDER_FROM_HEADER:
        ss = h.get(H_SENDING_SILO)
        if ss is not None and ss[0] not in ("silo", "null"):
            return Decoded(DEC_MALFORMED)
        if ss is None or ss[0] == "null":
            return Decoded(DEC_NO_SENDER)
        if ss[1] not in silo_index:
            return Decoded(DEC_UNKNOWN_SILO)
        sending = silo_index[ss[1]]
    else:
        sending = sender_override
    tg = h.get(H_TARGET_GRAIN)
    if tg is None or tg[0] != "grain":
        return Decoded(DEC_NO_TARGET)             # GetSimpleHeader<GrainId>: null / wrong type -> null
    key, raw, utf8_ok = tg[1], tg[2], tg[3]
    d = Decoded(DEC_OK, key.tcd, key.n0, key.n1, sending, category)
    if key.category == CAT_KEYEXT_GRAIN:
        if not utf8_ok:
            return Decoded(DEC_UNSUPPORTED)
        d.aux = jenkins_bytes(raw)                # GetUniformHashCode KeyExt branch over Write(UniqueKey)
        d.flags |= HDR_HASH_VALID
    ta = h.get(H_TARGET_ACTIVATION)
    if ta is not None and ta[0] == "act" and ts is not None and ts[0] == "silo":
        if ts[1] not in silo_index:
            return Decoded(DEC_UNKNOWN_SILO)
        d.flags |= HDR_ADDRESS_COMPLETE
        d.target_silo = silo_index[ts[1]]
    return d


def decode_frames(buf: bytes, offsets: Sequence[int], silo_index: Dict[SiloAddr, int],
                  sender_override: int = SENDER_FROM_HEADER) -> List[Decoded]:
    """IncomingMessageBuffer.TryDecodeMessage framing (IncomingMessageBuffer.cs:94-135): at each frame offset,
    int32 header length + int32 body length; the frame must fit the buffer (negative lengths are malformed)."""
    out = []
    for off in offsets:
        if off + LENGTH_HEADER_SIZE > len(buf):
            out.append(Decoded(DEC_MALFORMED))
            continue
        hl, bl = struct.unpack("<ii", buf[off:off + 8])
        if hl < 0 or bl < 0 or off + 8 + hl + bl > len(buf):
            out.append(Decoded(DEC_MALFORMED))
            continue
        out.append(decode_for_route(buf[off + 8:off + 8 + hl], silo_index, sender_override))
    return out


# ---------------------------------------------------------------------------------------
# emit: SetTargetPlacement on a received header dictionary, re-serialized
# ---------------------------------------------------------------------------------------
H_NEW_GRAIN_TYPE = 11
H_IS_NEW_PLACEMENT = 21
H_PRIOR_MESSAGE_ID = 28
H_PRIOR_MESSAGE_TIMES = 29

STAMP_OK = 0          # SetTargetPlacement applied
STAMP_COMPLETE = 1    # TargetAddress already complete: frame copied unchanged (Dispatcher.cs:557-558)
STAMP_SKIPPED = 2     # route status other than HIT / NEW_PLACEMENT: copied unchanged, host path
STAMP_UNSUPPORTED = 3 # header not decodable on the device, or not byte-canonical (a non-UTF-8 string), or no grain type
STAMP_MALFORMED = 4   # the reference throws (undecodable header, or a present non-ActivationId TARGET_ACTIVATION)


class NetDictionary:
    """System.Collections.Generic.Dictionary<K,V> insertion / removal order as .NET Framework 4.5 keeps it:
    entries array in insertion order; Remove pushes the entry on a LIFO free list; Add takes the free list head
    (or appends); enumeration walks the entries array skipping free entries."""

    def __init__(self, items):
        self.entries = [[k, v] for k, v in items]
        self.free = []                 # stack of free entry indices

    def index(self, k):
        for i, e in enumerate(self.entries):
            if e is not None and e[0] == k:
                return i
        return -1

    def contains(self, k):
        return self.index(k) >= 0

    def get(self, k):
        i = self.index(k)
        return None if i < 0 else self.entries[i][1]

    def remove(self, k):
        i = self.index(k)
        if i >= 0:
            self.entries[i] = None
            self.free.append(i)

    def set(self, k, v):               # headers[tag] = value
        i = self.index(k)
        if i >= 0:
            self.entries[i][1] = v
        elif self.free:
            self.entries[self.free.pop()] = [k, v]
        else:
            self.entries.append([k, v])

    def items(self):
        return [(e[0], e[1]) for e in self.entries if e is not None]


def _strict_canonical(dict_bytes: bytes, parsed) -> bool:
    """Byte-exact canonicality of the dictionary: re-serializing the parsed values gives its bytes back (false
    for a string or KeyExt that is not strict UTF-8: .NET decodes it with U+FFFD and re-encodes that)."""
    return serialize_headers([(k, _writer_form(v)) for k, v in parsed.items()]) == dict_bytes


def _writer_form(v):
    if v[0] == "grain":
        return ("grain", v[1])
    if v[0] == "list":
        return ("list", [_writer_form(x) for x in v[1]])
    return v


def stamp_frame(frame_hdr: bytes, body: bytes, route: int, act_key: Optional[Key], new_act_key: Optional[Key],
                silo_addr_of: Dict[int, SiloAddr], grain_type_of: Dict[int, str]):
    """One outgoing frame after routing -> (status, frame bytes).  Message.SetTargetPlacement
    (Message.cs:1079-1096) with PlacementResult (Orleans/Placement/PlacementResult.cs:45-72): HIT ->
    IdentifySelection(activation, host silo); NEW_PLACEMENT -> SpecifyCreation(host silo, grain type of the
    target's type code) with the caller's new ActivationId.  Every other status leaves the frame unchanged."""
    st_route = (route >> 16) & 0xFF
    host = (route >> 8) & 0xFF
    unchanged = struct.pack("<ii", len(frame_hdr), len(body)) + frame_hdr + body
    try:
        parsed, dict_end = parse_headers_end(frame_hdr)
    except DecodeError as e:
        return (STAMP_UNSUPPORTED if e.status == DEC_UNSUPPORTED else STAMP_MALFORMED), unchanged
    if st_route == 3:  # ST_ADDRESS_COMPLETE
        return STAMP_COMPLETE, unchanged
    if st_route not in (0, 1):
        return STAMP_SKIPPED, unchanged
    if not _strict_canonical(frame_hdr[:dict_end], parsed):  # bytes after the dictionary are dropped, as
        return STAMP_UNSUPPORTED, unchanged                   # SerializeMessageHeaders writes the dictionary only
    new_placement = st_route == 1
    if host not in silo_addr_of:
        return STAMP_UNSUPPORTED, unchanged
    activation = new_act_key if new_placement else act_key
    d = NetDictionary(parsed.items())
    grain_type = None
    if new_placement:
        tg = d.get(H_TARGET_GRAIN)
        type_code = (tg[1].tcd & 0xFFFFFFFF) if tg is not None and tg[0] == "grain" else None
        if type_code is None or type_code not in grain_type_of:
            return STAMP_UNSUPPORTED, unchanged
        grain_type = grain_type_of[type_code]
        if new_act_key is None:
            return STAMP_UNSUPPORTED, unchanged
    elif act_key is None:
        return STAMP_UNSUPPORTED, unchanged
    if d.contains(H_TARGET_ACTIVATION):
        cur = d.get(H_TARGET_ACTIVATION)
        if cur[0] != "act":
            return STAMP_MALFORMED, unchanged  # null.Equals(...) in SetTargetPlacement
        differs = cur[1] != activation
    else:
        differs = False
    if new_placement or differs:
        d.remove(H_PRIOR_MESSAGE_ID)
        d.remove(H_PRIOR_MESSAGE_TIMES)
    d.set(H_TARGET_ACTIVATION, ("act", activation))
    d.set(H_TARGET_SILO, ("silo", silo_addr_of[host]))
    if new_placement:
        d.set(H_IS_NEW_PLACEMENT, ("bool", True))
        d.set(H_NEW_GRAIN_TYPE, ("string", grain_type))
    hdr = serialize_headers([(k, _writer_form(v)) for k, v in d.items()])
    return STAMP_OK, struct.pack("<ii", len(hdr), len(body)) + hdr + body


def stamp_frames(buf: bytes, offsets: Sequence[int], routes, acts, act_keys: Sequence[Key], new_act_keys,
                 silo_addr_of: Dict[int, SiloAddr], grain_type_of: Dict[int, str]):
    """orl_stamp_frames_device: per frame (status, output bytes); an invalid prefix emits nothing (MALFORMED)."""
    out = []
    for i, off in enumerate(offsets):
        if off + LENGTH_HEADER_SIZE > len(buf):
            out.append((STAMP_MALFORMED, b""))
            continue
        hl, bl = struct.unpack("<ii", buf[off:off + 8])
        if hl < 0 or bl < 0 or off + 8 + hl + bl > len(buf):
            out.append((STAMP_MALFORMED, b""))
            continue
        hdr = buf[off + 8:off + 8 + hl]
        body = buf[off + 8 + hl:off + 8 + hl + bl]
        a = int(acts[i])
        ak = act_keys[a] if a < len(act_keys) else None
        nk = new_act_keys[i] if new_act_keys is not None else None
        out.append(stamp_frame(hdr, body, int(routes[i]), ak, nk, silo_addr_of, grain_type_of))
    return out
