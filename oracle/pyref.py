"""Independent pure-Python restatement of the Orleans 1.1 grain-message routing path.

TEST INFRASTRUCTURE ONLY.  This module is one of the two oracles (the other is the C++
restatement in ``oracle/cpu_ref.cpp``).  It is imported only by ``tests/``,
``tests/golden/gen_golden.py`` and nothing else: the product path (``orleans_amd``,
``liborleans_route.so``) never imports, links or executes anything under ``oracle/``.

Every function cites the reference file:line it restates (paths relative to the
reference checkout, ``randa1/orleans`` @ 1.1.0.0).  The reference is C#/.NET 4.5 and
cannot run here (no dotnet/mono); its own tests pin only one property on this path
(``Identifiertests.ID_HashCorrectness``: byte-path Jenkins == u64-path Jenkins,
src/TesterInternal/General/Identifiertests.cs:284-301).  Ring ownership, directory
lookup, bucketing and fan-out are therefore "parity unpinned" by the reference tests and
pinned only by two independent restatements (this file and cpu_ref.cpp) plus the
committed golden fixtures generated from this file.

Pure-Python loops: use for small cases (<= ~1e5 messages).
"""
from __future__ import annotations

import hashlib
import struct
import uuid
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

M32 = 0xFFFFFFFF
M64 = 0xFFFFFFFFFFFFFFFF

# ---------------------------------------------------------------------------------------
# UniqueKey categories  (src/Orleans/IDs/UniqueKey.cs:41-49)
# ---------------------------------------------------------------------------------------
CAT_NONE = 0
CAT_SYSTEM_TARGET = 1
CAT_SYSTEM_GRAIN = 2
CAT_GRAIN = 3
CAT_CLIENT = 4
CAT_KEYEXT_GRAIN = 6


# ---------------------------------------------------------------------------------------
# Stage 1: Jenkins lookup2 (src/Orleans/IDs/JenkinsHash.cs)
# ---------------------------------------------------------------------------------------
def _mix(a: int, b: int, c: int) -> Tuple[int, int, int]:
    """JenkinsHash.Mix, JenkinsHash.cs:54-65 (all arithmetic mod 2^32)."""
    a = (a - b) & M32; a = (a - c) & M32; a ^= (c >> 13)
    b = (b - c) & M32; b = (b - a) & M32; b ^= (a << 8) & M32
    c = (c - a) & M32; c = (c - b) & M32; c ^= (b >> 13)
    a = (a - b) & M32; a = (a - c) & M32; a ^= (c >> 12)
    b = (b - c) & M32; b = (b - a) & M32; b ^= (a << 16) & M32
    c = (c - a) & M32; c = (c - b) & M32; c ^= (b >> 5)
    a = (a - b) & M32; a = (a - c) & M32; a ^= (c >> 3)
    b = (b - c) & M32; b = (b - a) & M32; b ^= (a << 10) & M32
    c = (c - a) & M32; c = (c - b) & M32; c ^= (b >> 15)
    return a, b, c


def jenkins_bytes(data: bytes) -> int:
    """JenkinsHash.ComputeHash(byte[]), JenkinsHash.cs:68-115 (the "reference implementation")."""
    n = len(data)
    a = b = 0x9E3779B9
    c = 0
    i = 0
    while i + 12 <= n:
        a = (a + int.from_bytes(data[i:i + 4], "little")) & M32
        b = (b + int.from_bytes(data[i + 4:i + 8], "little")) & M32
        c = (c + int.from_bytes(data[i + 8:i + 12], "little")) & M32
        i += 12
        a, b, c = _mix(a, b, c)
    c = (c + n) & M32
    tail = data[i:]
    # bytes 0..3 -> a, 4..7 -> b, 8..10 -> c at shifts 8/16/24 (JenkinsHash.cs:90-112)
    for j, byte in enumerate(tail):
        if j < 4:
            a = (a + (byte << (8 * j))) & M32
        elif j < 8:
            b = (b + (byte << (8 * (j - 4)))) & M32
        else:
            c = (c + (byte << (8 * (j - 7)))) & M32
    a, b, c = _mix(a, b, c)
    return c


def jenkins_u64(u1: int, u2: int, u3: int) -> int:
    """JenkinsHash.ComputeHash(ulong,ulong,ulong), JenkinsHash.cs:126-144.

    ``(uint)((u ^ (uint)u) >> 32)`` is the high word of ``u``.
    """
    a = b = 0x9E3779B9
    c = 0
    a = (a + (u1 & M32)) & M32
    b = (b + (u1 >> 32)) & M32
    c = (c + (u2 & M32)) & M32
    a, b, c = _mix(a, b, c)
    a = (a + (u2 >> 32)) & M32
    b = (b + (u3 & M32)) & M32
    c = (c + (u3 >> 32)) & M32
    a, b, c = _mix(a, b, c)
    c = (c + 24) & M32
    a, b, c = _mix(a, b, c)
    return c


# ---------------------------------------------------------------------------------------
# SHA-256 identity hashes (src/Orleans/Utils/Utils.cs:201-246); BCL SHA256 == FIPS 180-4
# ---------------------------------------------------------------------------------------
def _to_int32(x: int) -> int:
    x &= M32
    return x - (1 << 32) if x & 0x80000000 else x


def calc_id_hash(text: str) -> int:
    """Utils.CalculateIdHash, Utils.cs:201-220: SHA-256 over UTF-16LE, XOR of 8 big-endian int32."""
    digest = hashlib.sha256(text.encode("utf-16-le")).digest()
    h = 0
    for i in range(0, 32, 4):
        h ^= int.from_bytes(digest[i:i + 4], "big")
    return _to_int32(h)


def calc_guid_hash(text: str) -> bytes:
    """Utils.CalculateGuidHash, Utils.cs:227-246: 16-byte fold hash[i%16] ^= sha[i]; returns Guid bytes."""
    digest = hashlib.sha256(text.encode("utf-16-le")).digest()
    out = bytearray(16)
    for i, v in enumerate(digest):
        out[i % 16] ^= v
    return bytes(out)


# ---------------------------------------------------------------------------------------
# UniqueKey / GrainId composition (src/Orleans/IDs/UniqueKey.cs, GrainId.cs)
# ---------------------------------------------------------------------------------------
def guid_to_bytearray(guid_text: str) -> bytes:
    """.NET Guid.ToByteArray(): Data1 LE4, Data2 LE2, Data3 LE2, then 8 raw bytes (= uuid.bytes_le)."""
    return uuid.UUID(guid_text).bytes_le


def type_code_data(category: int, type_data: int) -> int:
    """UniqueKey.NewKey(n0,n1,category,typeData,keyExt), UniqueKey.cs:141.

    ``typeData`` is a C# ``long``: a negative int type code arrives sign-extended
    (GrainInterfaceMap.cs:437 returns int widened to long).
    """
    return (((category & 0xFF) << 56) + ((type_data & M64) & 0x00FFFFFFFFFFFFFF)) & M64


@dataclass(frozen=True)
class Key:
    """UniqueKey fields N0, N1, TypeCodeData, KeyExt (UniqueKey.cs:51-54)."""
    tcd: int
    n0: int
    n1: int
    key_ext: Optional[str] = None

    @property
    def category(self) -> int:
        return (self.tcd >> 56) & 0xFF  # UniqueKey.GetCategory


def key_from_long(long_key: int, type_code: int, key_ext: Optional[str] = None) -> Key:
    """GrainId.GetGrainId(typeCode, long, keyExt) -> UniqueKey.NewKey(long,...), GrainId.cs:90-95, UniqueKey.cs:146-152."""
    cat = CAT_GRAIN if key_ext is None else CAT_KEYEXT_GRAIN
    return Key(type_code_data(cat, type_code), 0, long_key & M64, key_ext)


def key_from_guid(guid_text: str, type_code: int, key_ext: Optional[str] = None,
               category: Optional[int] = None) -> Key:
    """UniqueKey.NewKey(Guid,...), UniqueKey.cs:159-167 (N0/N1 = LE u64 of Guid.ToByteArray())."""
    if category is None:
        category = CAT_GRAIN if key_ext is None else CAT_KEYEXT_GRAIN
    gb = guid_to_bytearray(guid_text)
    n0 = int.from_bytes(gb[0:8], "little")
    n1 = int.from_bytes(gb[8:16], "little")
    return Key(type_code_data(category, type_code), n0, n1, key_ext)


def key_system_target(system_id: int) -> Key:
    """UniqueKey.NewSystemTargetKey(short), UniqueKey.cs:177-181 (short sign-extended to ulong)."""
    return Key(type_code_data(CAT_SYSTEM_TARGET, 0), 0, system_id & M64, None)


# Constants.SystemMembershipTableId = GetSystemGrainId(Guid "01145FEC-C21E-11E0-9105-D0FB4724019B")
# (src/Orleans/Runtime/Constants.cs:66, GrainId.cs:70-73)
MEMBERSHIP_TABLE_KEY = key_from_guid("01145FEC-C21E-11E0-9105-D0FB4724019B", 0, category=CAT_SYSTEM_GRAIN)


def serialize_unique_key(k: Key) -> bytes:
    """BinaryTokenStreamWriter.Write(UniqueKey) = N0, N1, TypeCodeData (LE8) + Write(string)
    (BinaryTokenStreamWriter.cs:488-494, 237-250: int32 length + UTF-8, null -> -1)."""
    out = struct.pack("<QQQ", k.n0, k.n1, k.tcd)
    if k.key_ext is None:
        out += struct.pack("<i", -1)
    else:
        b = k.key_ext.encode("utf-8")
        out += struct.pack("<i", len(b)) + b
    return out


def uniform_hash(k: Key) -> int:
    """UniqueKey.GetUniformHashCode, UniqueKey.cs:280-305 (u64 path hashes (TCD, N0, N1))."""
    if k.category == CAT_KEYEXT_GRAIN and k.key_ext is not None:
        return jenkins_bytes(serialize_unique_key(k))
    return jenkins_u64(k.tcd, k.n0, k.n1)


# ---------------------------------------------------------------------------------------
# Silo hashes (src/Orleans/IDs/SiloAddress.cs:197-230)
# ---------------------------------------------------------------------------------------
def silo_consistent_hash(endpoint: str, generation: int) -> int:
    """SiloAddress.GetConsistentHashCode: CalculateIdHash(Endpoint.ToString() + Generation.ToString(Invariant))."""
    return calc_id_hash(endpoint + str(int(generation)))


def silo_uniform_hash(ip16: bytes, port: int, generation: int, extra_bit: int) -> int:
    """SiloAddress.GetUniformHashCode(jenkins, extraBit), SiloAddress.cs:223-230: 28-byte layout
    16-B IP (IPv4 = 12 zero bytes + 4), port LE4, generation LE4, extraBit LE4 (BinaryTokenStreamWriter.cs:448-486)."""
    assert len(ip16) == 16
    return jenkins_bytes(ip16 + struct.pack("<iii", port, generation, extra_bit))


# ---------------------------------------------------------------------------------------
# Stage 2: directory ring (src/OrleansRuntime/GrainDirectory/LocalGrainDirectory.cs)
# ---------------------------------------------------------------------------------------
NULL_SILO = 0xFF


@dataclass
class Ring:
    """membershipRingList: silos sorted ascending by signed consistent hash."""
    entries: List[Tuple[int, int]] = field(default_factory=list)  # (int32 hash, silo index)

    def add_server(self, silo: int, hash32: int) -> None:
        """LocalGrainDirectory.AddServer, :243-268: insert at FindLastIndex(h < hash)+1
        (i.e. before existing equal hashes); duplicates (membershipCache.Contains) ignored."""
        if any(s == silo for _, s in self.entries):
            return
        idx = -1
        for i, (h, _) in enumerate(self.entries):
            if h < hash32:
                idx = i
        self.entries.insert(idx + 1, (hash32, silo))

    def remove_server(self, silo: int) -> None:
        """LocalGrainDirectory.RemoveServer, :270-304 (list removal only)."""
        self.entries = [e for e in self.entries if e[1] != silo]


@dataclass
class SiloView:
    """Per-silo state the routing decision depends on."""
    running: Sequence[bool]      # LocalGrainDirectory.Running of that silo (as routing silo)
    functional: Sequence[bool]   # Membership.IsFunctionalDirectory(silo) (IsValidSilo)
    seed: int = NULL_SILO        # LocalGrainDirectory.Seed (NULL_SILO = none)
    local: Optional[Sequence[bool]] = None  # silos whose directory partition this engine holds (None = all)

    def is_local(self, silo: int) -> bool:
        return True if self.local is None else bool(self.local[silo])


OWN_OK = 0
OWN_NULL = 1      # owner null (stopping, :471-475 / :483-493)
OWN_NO_SEED = 2   # ArgumentException for membership table grain without seed (:449-460)


def calculate_target_silo(ring: Ring, key: Key, hash32: int, me: int, view: SiloView,
                          exclude_if_stopping: bool) -> Tuple[int, int]:
    """LocalGrainDirectory.CalculateTargetSilo, LocalGrainDirectory.cs:439-497.

    Returns (silo index or NULL_SILO, OWN_* code)."""
    if key.category == CAT_SYSTEM_TARGET:                      # :442-447
        return me, OWN_OK
    if key == MEMBERSHIP_TABLE_KEY or (key.tcd, key.n0, key.n1) == (
            MEMBERSHIP_TABLE_KEY.tcd, MEMBERSHIP_TABLE_KEY.n0, MEMBERSHIP_TABLE_KEY.n1):  # :449-464
        if view.seed == NULL_SILO:
            return NULL_SILO, OWN_NO_SEED
        return view.seed, OWN_OK
    h = _to_int32(hash32)                                        # :467
    ents = ring.entries
    running = bool(view.running[me])
    if len(ents) == 0:                                           # :471-475
        return (NULL_SILO, OWN_NULL) if (exclude_if_stopping and not running) else (me, OWN_OK)
    exclude_me = (not running) and exclude_if_stopping          # :478
    found = None
    for sh, s in ents:                                           # FindLast, :481-482
        if sh <= h and (s != me or not exclude_me):
            found = s
    if found is None:                                            # :483-493
        found = ents[-1][1]
        if found == me and exclude_me:
            if len(ents) > 1:
                found = ents[-2][1]
            else:
                return NULL_SILO, OWN_NULL
    return found, OWN_OK


# ---------------------------------------------------------------------------------------
# Stage 3: GrainDirectoryPartition (single activation) (GrainDirectoryPartition.cs)
# ---------------------------------------------------------------------------------------
INS_INSERTED = 0
INS_EXISTING = 1
INS_INVALID_SILO = 2
INS_REMOTE_OWNER = 3
INS_OWNER_NULL = 4
INS_UNSUPPORTED = 5

MERGE_INSERTED, MERGE_KEPT, MERGE_REPLACED, MERGE_SAME, MERGE_DUPLICATE, MERGE_UNSUPPORTED = 0, 1, 2, 3, 4, 5


class Partition:
    """Dictionary<GrainId, GrainInfo> restricted to single-activation grains
    (GrainDirectoryPartition.cs:186-344; GrainInfo.AddSingleActivation :100-114)."""

    def __init__(self) -> None:
        self.data: Dict[Tuple[int, int, int, Optional[str]], Tuple[int, int]] = {}

    @staticmethod
    def _k(key: Key):
        return (key.tcd, key.n0, key.n1, key.key_ext if key.category == CAT_KEYEXT_GRAIN else None)

    def add_single_activation(self, key: Key, act: int, silo: int, view: SiloView) -> Tuple[int, int, int]:
        """AddSingleActivation :270-287: null if !IsValidSilo(silo); first writer wins.
        Returns (status, winner act, winner silo)."""
        if not view.functional[silo]:
            return INS_INVALID_SILO, 0xFFFFFFFF, NULL_SILO
        k = self._k(key)
        if k in self.data:
            a, s = self.data[k]
            return INS_EXISTING, a, s
        self.data[k] = (act, silo)
        return INS_INSERTED, act, silo

    def remove(self, key: Key) -> bool:
        """RemoveGrain :310-318 / RemoveActivation(force) for a single-activation grain."""
        return self.data.pop(self._k(key), None) is not None

    def merge(self, entries, act_key_of) -> List[Tuple[int, int, int]]:
        """GrainDirectoryPartition.Merge(other) (GrainDirectoryPartition.cs:366-383) with `other` given as
        (Key, act, silo) entries in its enumeration order: an absent grain is added; a present one goes through
        GrainInfo.Merge (:158-183): the other's activation is added unless the same ActivationId is present, then
        the single-activation grain keeps the smallest ActivationId (OrderBy key: UniqueKey.CompareTo =
        (TypeCodeData, N0, N1)) and drops the rest.  act_key_of(handle) -> (tcd, n0, n1).  A grain repeated in
        `entries` is not a dictionary: MERGE_DUPLICATE after the first.  Returns per entry (status, dropped act,
        dropped silo)."""
        out, seen = [], set()
        for key, act, silo in entries:
            k = self._k(key)
            if key.category == CAT_KEYEXT_GRAIN:
                out.append((MERGE_UNSUPPORTED, NO_ACT, NULL_SILO))
                continue
            if k in seen:
                out.append((MERGE_DUPLICATE, NO_ACT, NULL_SILO))
                continue
            seen.add(k)
            if k not in self.data:
                self.data[k] = (act, silo)
                out.append((MERGE_INSERTED, NO_ACT, NULL_SILO))
                continue
            a_old, s_old = self.data[k]
            ko, kn = act_key_of(a_old), act_key_of(act)
            if ko == kn:
                out.append((MERGE_SAME, NO_ACT, NULL_SILO))
            elif kn < ko:
                self.data[k] = (act, silo)
                out.append((MERGE_REPLACED, a_old, s_old))
            else:
                out.append((MERGE_KEPT, act, silo))
        return out

    def lookup(self, key: Key, view: SiloView) -> Optional[Tuple[int, int]]:
        """LookUpGrain :326-344 filtered by IsValidSilo (:337-340): returns (act, silo) or None."""
        r = self.data.get(self._k(key))
        if r is None or not view.functional[r[1]]:
            return None
        return r


def register_single_activation(ring: "Ring", part: "Partition", view: "SiloView", key: Key, act: int,
                               silo: int) -> Tuple[int, int, int]:
    """LocalGrainDirectory.RegisterSingleActivationAsync (LocalGrainDirectory.cs:510-544) executed on the
    activation's silo: owner = CalculateTargetSilo(grain) (excludeThisSiloIfStopping = true); null ->
    "Grain directory is stopping"; remote owner -> forwarded (not applied here); local owner ->
    GrainDirectoryPartition.AddSingleActivation.  KeyExt / SystemTarget keys are not held by the engine's
    partition (INS_UNSUPPORTED).  Returns (status, winner act, winner silo)."""
    if key.category in (CAT_KEYEXT_GRAIN, CAT_SYSTEM_TARGET):
        return INS_UNSUPPORTED, NO_ACT, NULL_SILO
    owner, code = calculate_target_silo(ring, key, uniform_hash(key), silo, view, True)
    if code != OWN_OK:
        return INS_OWNER_NULL, NO_ACT, NULL_SILO
    if not view.is_local(owner):
        return INS_REMOTE_OWNER, NO_ACT, NULL_SILO
    return part.add_single_activation(key, act, silo, view)


def register_keyext(ring: "Ring", part: "Partition", view: "SiloView", key: Key, act: int, silo: int) -> Tuple[int, int, int]:
    """RegisterSingleActivationAsync for a KeyExt grain (the engine's KeyExt table, round 5): the same steps as
    register_single_activation with the owner of the KeyExt uniform hash (UniqueKey.cs:288-294); GrainDirectoryPartition
    keys it by the whole UniqueKey, extension included (Partition._k).  Non-KeyExt keys: INS_UNSUPPORTED."""
    if key.category != CAT_KEYEXT_GRAIN or key.key_ext is None:
        return INS_UNSUPPORTED, NO_ACT, NULL_SILO
    owner, code = calculate_target_silo(ring, key, uniform_hash(key), silo, view, True)
    if code != OWN_OK:
        return INS_OWNER_NULL, NO_ACT, NULL_SILO
    if not view.is_local(owner):
        return INS_REMOTE_OWNER, NO_ACT, NULL_SILO
    return part.add_single_activation(key, act, silo, view)


# ---------------------------------------------------------------------------------------
# Full per-message routing decision (Dispatcher.AddressMessage + placement)
# ---------------------------------------------------------------------------------------
ST_HIT = 0
ST_NEW_PLACEMENT = 1
ST_SYSTEM_TARGET = 2
ST_ADDRESS_COMPLETE = 3
ST_OWNER_NULL = 4
ST_NO_SEED = 5
ST_CLIENT_UNREGISTERED = 6
ST_KEYEXT_UNRESOLVED = 7
ST_REMOTE_OWNER = 8

FL_NEW_PLACEMENT = 0x01
FL_LOOPBACK = 0x02
FL_OWNER_IS_SEED = 0x04

POLICY_PREFER_LOCAL = 0
POLICY_HASH_SPREAD = 1

HDR_ADDRESS_COMPLETE = 0x01
HDR_HASH_VALID = 0x02

NO_ACT = 0xFFFFFFFF


@dataclass
class Msg:
    key: Key
    sending_silo: int
    flags: int = 0
    target_silo_hint: int = NULL_SILO
    aux: int = 0


def pack_route(owner: int, host: int, status: int, flags: int) -> int:
    return (owner & 0xFF) | ((host & 0xFF) << 8) | ((status & 0xFF) << 16) | ((flags & 0xFF) << 24)


def placement_silo(policy: int, me: int, hash32: int, view: SiloView) -> int:
    """OnAddActivation. PREFER_LOCAL = PreferLocalPlacementDirector.cs:38-44 (context.LocalSilo).
    HASH_SPREAD = deterministic stand-in for RandomPlacementDirector.cs:59-66: the active silo list
    (ascending silo index) indexed by hash % count instead of SafeRandom."""
    if policy == POLICY_PREFER_LOCAL:
        return me
    active = [i for i, f in enumerate(view.functional) if f]
    if not active:
        return NULL_SILO
    return active[hash32 % len(active)]


def route_one(m: Msg, ring: Ring, part: Partition, view: SiloView, exclude_if_stopping: bool = False,
              policy: int = POLICY_PREFER_LOCAL, keyext_directory: bool = False) -> Tuple[int, int]:
    """One message: returns (route word, activation handle).

    Dispatcher.AddressMessage (Dispatcher.cs:555-579): complete TargetAddress -> untouched;
    SelectOrAddActivation (PlacementDirectorsManager.cs:70-91) -> RandomPlacementDirector.OnSelectActivation
    (RandomPlacementDirector.cs:34-57, the single-activation case: 0 entries -> add, 1 -> that entry)
    -> context.Lookup -> LocalGrainDirectory.LocalLookup/FullLookup (LocalGrainDirectory.cs:663-765)
    -> CalculateTargetSilo(grain, false) + GrainDirectoryPartition.LookUpGrain on the owner."""
    me = m.sending_silo
    if m.flags & HDR_ADDRESS_COMPLETE:                                   # Dispatcher.cs:557-558
        host = m.target_silo_hint
        fl = FL_LOOPBACK if host == me else 0
        return pack_route(NULL_SILO, host, ST_ADDRESS_COMPLETE, fl), NO_ACT
    key = m.key
    h = (m.aux & M32) if (m.flags & HDR_HASH_VALID) else uniform_hash(key)
    owner, code = calculate_target_silo(ring, key, h, me, view, exclude_if_stopping)
    fl = FL_OWNER_IS_SEED if (code == OWN_OK and key.category == CAT_SYSTEM_GRAIN
                              and (key.tcd, key.n0, key.n1) == (MEMBERSHIP_TABLE_KEY.tcd, MEMBERSHIP_TABLE_KEY.n0,
                                                                MEMBERSHIP_TABLE_KEY.n1)) else 0
    if code == OWN_NO_SEED:
        return pack_route(NULL_SILO, NULL_SILO, ST_NO_SEED, 0), NO_ACT
    if code == OWN_NULL:
        return pack_route(NULL_SILO, NULL_SILO, ST_OWNER_NULL, 0), NO_ACT
    if key.category == CAT_SYSTEM_TARGET:                                # InsideGrainClient.cs:174-181
        return pack_route(owner, me, ST_SYSTEM_TARGET, FL_LOOPBACK), NO_ACT
    if key.category == CAT_KEYEXT_GRAIN and not keyext_directory:  # the plain route entry points leave them to the host
        return pack_route(owner, NULL_SILO, ST_KEYEXT_UNRESOLVED, fl), NO_ACT
    if not view.is_local(owner):              # LocalLookup non-owner branch -> cache / remote FullLookup (:711-754)
        return pack_route(owner, NULL_SILO, ST_REMOTE_OWNER, fl), NO_ACT
    r = part.lookup(key, view)
    if r is not None:
        act, host = r
        fl |= FL_LOOPBACK if host == me else 0
        return pack_route(owner, host, ST_HIT, fl), act
    if key.category == CAT_CLIENT:                                       # PlacementDirectorsManager.cs:75-81
        return pack_route(owner, NULL_SILO, ST_CLIENT_UNREGISTERED, fl), NO_ACT
    host = placement_silo(policy, me, h, view)
    fl |= FL_NEW_PLACEMENT | (FL_LOOPBACK if host == me else 0)
    return pack_route(owner, host, ST_NEW_PLACEMENT, fl), NO_ACT


def route_batch(msgs: Sequence[Msg], ring: Ring, part: Partition, view: SiloView,
                exclude_if_stopping: bool = False, policy: int = POLICY_PREFER_LOCAL, keyext_directory: bool = False):
    routes, acts = [], []
    for m in msgs:
        r, a = route_one(m, ring, part, view, exclude_if_stopping, policy, keyext_directory)
        routes.append(r)
        acts.append(a)
    return routes, acts


# ---------------------------------------------------------------------------------------
# Stage 4: stable bucketing by target activation (ActivationData.EnqueueMessage FIFO)
# ---------------------------------------------------------------------------------------
def bucket_stable(acts: Sequence[int], n_act: int):
    """Per-activation FIFO in arrival order (ActivationData.cs:483-514, "Insert in a FIFO order";
    IncomingMessageAgent.cs:147). Bucket of a message = its activation handle, or n_act (the
    'unresolved' bucket) for every message without a resident activation.

    Returns (offsets[n_act+2], order[n]) with order = message indices grouped by bucket, stable."""
    lists: List[List[int]] = [[] for _ in range(n_act + 1)]
    for i, a in enumerate(acts):
        b = a if a < n_act else n_act
        lists[b].append(i)
    offsets = [0]
    order: List[int] = []
    for lst in lists:
        order.extend(lst)
        offsets.append(len(order))
    return offsets, order


# ---------------------------------------------------------------------------------------
# Stage 5: multicast fan-out (ChirperAccount.PublishMessage :154-157, ObserverSubscriptionManager.Notify)
# ---------------------------------------------------------------------------------------
def fanout_expand(csr_off: Sequence[int], csr_tgt: Sequence[int], pubs: Sequence[int],
                  pub_silo: Sequence[int], follower_tcd: int) -> List[Msg]:
    """Expand each publish p (publisher account pubs[p] sending from silo pub_silo[p]) into one
    single-target send per follower, in CSR order (the reference's Dictionary enumeration order is
    not pinned; parity is defined on the CSR order given as input). Follower grain =
    GrainId(typeCode, long follower id) -> key (tcd, 0, id)."""
    out: List[Msg] = []
    for p, src in enumerate(pubs):
        for e in range(csr_off[src], csr_off[src + 1]):
            out.append(Msg(Key(follower_tcd, 0, csr_tgt[e] & M64), pub_silo[p]))
    return out


# ---------------------------------------------------------------------------------------
# Deterministic synthetic inputs shared by tests/bench
# ---------------------------------------------------------------------------------------
def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def default_cluster(n_silos: int = 8, port: int = 11111, generation: int = 1):
    """Fixed synthetic cluster: silos 10.0.0.{1..n}:port, generation 1; ring built by AddServer."""
    ring = Ring()
    hashes = []
    for s in range(n_silos):
        h = silo_consistent_hash(f"10.0.0.{s + 1}:{port}", generation)
        hashes.append(h)
        ring.add_server(s, h)
    return ring, hashes


CHIRPER_ACCOUNT_CLASS = "Orleans.Samples.Chirper.Grains.ChirperAccount"


# ---------------------------------------------------------------------------------------
# f3: stream / reminder rings
# ---------------------------------------------------------------------------------------
class VirtualBucketsRing:
    """VirtualBucketsRingProvider (src/OrleansRuntime/ConsistentRing/VirtualBucketsRingProvider.cs).

    bucketsMap: SortedDictionary<uint, SiloAddress> (:41,58).  AddServer (:142-169): the silo's
    GetUniformHashCodes(numBucketsPerSilo) (SiloAddress.cs:208-230); on an equal bucket hash the silo with the
    lesser generation keeps it (SiloAddress.CompareTo compares Generation only, SiloAddress.cs:254-257;
    `if (silo.CompareTo(other) > 0) continue`).  RemoveServer (:170-193): if the silo owns no bucket, nothing;
    else every one of ITS hashes is removed from the map, whoever holds it."""

    def __init__(self, buckets_per_silo: int = 30) -> None:
        self.nb = buckets_per_silo
        self.map: Dict[int, int] = {}
        self.silo_hashes: Dict[int, List[int]] = {}
        self.gen: Dict[int, int] = {}

    def add_server(self, silo: int, ip16: bytes, port: int, generation: int) -> None:
        hashes = [silo_uniform_hash(ip16, port, generation, i) for i in range(self.nb)]
        self.silo_hashes[silo] = hashes
        self.gen[silo] = generation
        for h in hashes:
            if h in self.map and generation > self.gen[self.map[h]]:
                continue
            self.map[h] = silo

    def remove_server(self, silo: int) -> None:
        if silo not in self.map.values():
            return
        for h in self.silo_hashes[silo]:
            self.map.pop(h, None)

    def sorted_list(self) -> List[Tuple[int, int]]:
        return sorted(self.map.items())

    def target(self, key: int, me: int, exclude_me: bool) -> int:
        """CalculateTargetSilo(uint hash) (:277-313): first bucket >= hash (clockwise) that is not me while
        excluding; none → bucket [0], or [1] if [0] is me and excluding (even if [1] is me too)."""
        lst = self.sorted_list()
        if not lst:
            return NULL_SILO if exclude_me else me
        for h, s in lst:
            if h >= key and (s != me or not exclude_me):
                return s
        s = lst[0][1]
        if s == me and exclude_me:
            return lst[1][1] if len(lst) > 1 else NULL_SILO
        return s


def consistent_ring_target(ring: Ring, key: int, me: int, exclude_me: bool) -> int:
    """ConsistentRingProvider.CalculateTargetSilo(uint hash) (ConsistentRingProvider.cs:342-379) over
    membershipRingList (ascending signed consistent hash, inserted as in :116-135): first silo with
    GetConsistentHashCode() >= hash — an int against a uint, so C# compares as long and a negative silo hash
    never matches; none → [0], or [1] if [0] is me and excluding."""
    lst = ring.entries
    if not lst:
        return NULL_SILO if exclude_me else me
    for h, s in lst:
        if h >= key and (s != me or not exclude_me):  # Python ints: the long promotion exactly
            return s
    s = lst[0][1]
    if s == me and exclude_me:
        return lst[1][1] if len(lst) > 1 else NULL_SILO
    return s


def stream_queue_hashes(n_queues: int) -> List[int]:
    """HashRingBasedStreamQueueMapper ctor (src/Orleans/Streams/QueueAdapters/HashRingBasedStreamQueueMapper.cs:
    36-53): one queue at hash 0, else queue i at portion * i, portion = (uint)(RING_SIZE / n + 1), RING_SIZE = 2^32
    (RangeFactory)."""
    if n_queues == 1:
        return [0]
    portion = (1 << 32) // n_queues + 1
    return [(portion * i) & M32 for i in range(n_queues)]


def stream_queue_for_guid(guid_bytes: bytes, n_queues: int) -> int:
    """GetQueueForStream(streamGuid, ns) = HashRing.CalculateResponsible(Guid) (src/Orleans/Runtime/HashRing.cs:
    95-126): Jenkins over Guid.ToByteArray(), then the first queue (ring sorted by uniform hash) with hash >= key,
    else the first queue.  Returns the queue index."""
    key = jenkins_bytes(guid_bytes)
    hs = stream_queue_hashes(n_queues)
    order = sorted(range(n_queues), key=lambda i: hs[i])
    for i in order:
        if hs[i] >= key:
            return i
    return order[0]


# ---------------------------------------------------------------------------------------
# f4: outbound queues and client gateway buckets
# ---------------------------------------------------------------------------------------
OUTQ_LOOPBACK, OUTQ_PING, OUTQ_SYSTEM, OUTQ_REJECT, OUTQ_OVERFLOW, OUTQ_UNKNOWN_SILO = (
    0xFFFFFFF0, 0xFFFFFFF1, 0xFFFFFFF2, 0xFFFFFFF3, 0xFFFFFFF4, 0xFFFFFFF5)


def cs_mod(a: int, b: int) -> int:
    """C#'s % on ints: truncating division, the remainder takes the dividend's sign."""
    r = abs(a) % abs(b)
    return -r if a < 0 else r


def outbound_queue(target_silo: int, sending_silo: int, category: int, silo_hash: Dict[int, int],
                   n_senders: int) -> int:
    """OutboundMessageQueue.SendMessage (src/OrleansRuntime/Messaging/OutboundMessageQueue.cs:75-150): no target
    silo → SendRejection (:100-105); target == MyAddress → InboundQueue (:113-119); Ping / System senders;
    else senders[Math.Abs(TargetSilo.GetConsistentHashCode()) % senders.Length] (:141; Math.Abs(int.MinValue)
    throws OverflowException)."""
    if target_silo == NULL_SILO:
        return OUTQ_REJECT
    if target_silo == sending_silo:
        return OUTQ_LOOPBACK
    if category == 0:
        return OUTQ_PING
    if category == 1:
        return OUTQ_SYSTEM
    if target_silo not in silo_hash:
        return OUTQ_UNKNOWN_SILO
    h = silo_hash[target_silo]
    if h == -(1 << 31):
        return OUTQ_OVERFLOW
    return abs(h) % n_senders


def client_bucket(uniform_hash32: int, n_buckets: int) -> int:
    """UniqueIdentifier.GetHashCode_Modulo (src/Orleans/IDs/UniqueIdentifier.cs:60-66) with
    GetHashCode() = unchecked((int)GetUniformHashCode()) (UniqueKey.cs:275-278)."""
    key = _to_int32(uniform_hash32)
    mod = _to_int32(n_buckets)
    return cs_mod(cs_mod(key, mod) + mod, mod)


def apply_directory_cache(route: Sequence[int], act: Sequence[int], sending_silos: Sequence[int],
                          keys: Sequence[Tuple[int, int, int]], cache: Dict[Tuple[int, int, int], Tuple[int, int]],
                          functional: Sequence[int]):
    """LocalGrainDirectory.LocalLookup's cache branch (LocalGrainDirectory.cs:691-702) + GetLocalCacheData
    (:711-717): a grain whose owner is remote (REMOTE_OWNER without a cache) resolves to its cached activation
    when that activation's silo is valid; the route becomes HIT | CACHED (+ LOOPBACK when it is the sender)."""
    r_out, a_out = list(route), list(act)
    for i, (r, k) in enumerate(zip(route, keys)):
        if (r >> 16) & 0xFF != ST_REMOTE_OWNER or k not in cache:
            continue
        a, silo = cache[k]
        if not functional[silo]:
            continue
        fl = ((r >> 24) & 0xFF) | 0x08 | (FL_LOOPBACK if silo == sending_silos[i] else 0)
        r_out[i] = pack_route(r & 0xFF, silo, ST_HIT, fl)
        a_out[i] = a
    return r_out, a_out


class LRUCache:
    """AdaptiveGrainDirectoryCache over LRU<GrainId, entry> (AdaptiveGrainDirectoryCache.cs:97-133, src/Orleans/Utils/LRU.cs),
    restated sequentially as the reference runs it (maxAge = TimeSpan.MaxValue: nothing expires):
      add       LRU.Add (:104-108): AdjustSize, then AddOrUpdate with the next generation;
      adjust    LRU.AdjustSize (:188-205): while Count >= MaximumSize, generationToFree += 1 and the entry whose generation
                equals it (if any) is removed;
      try_get   LRU.TryGetValue (:147-174): a hit takes the next generation;
      remove    LRU.RemoveKey (:118-125)."""

    def __init__(self, max_size: int):
        self.max = max_size
        self.next_gen = 0
        self.gen_free = 0
        self.d: Dict[Tuple[int, int, int], list] = {}   # key -> [(act, silo), generation]
        self.by_gen: Dict[int, Tuple[int, int, int]] = {}

    def _stamp(self, key):
        self.next_gen += 1
        old = self.d[key][1]
        self.by_gen.pop(old, None)
        self.d[key][1] = self.next_gen
        self.by_gen[self.next_gen] = key

    def add(self, key, value):
        while len(self.d) >= self.max:  # AdjustSize
            self.gen_free += 1
            victim = self.by_gen.pop(self.gen_free, None)
            if victim is not None:
                del self.d[victim]
        if key in self.d:
            self.d[key][0] = value
        else:
            self.d[key] = [value, 0]
        self._stamp(key)

    def try_get(self, key):
        if key not in self.d:
            return None
        self._stamp(key)
        return self.d[key][0]

    def remove(self, key) -> bool:
        e = self.d.pop(key, None)
        if e is None:
            return False
        self.by_gen.pop(e[1], None)
        return True

    def items(self):
        return {k: v[0] for k, v in self.d.items()}


def apply_directory_cache_lru(route: Sequence[int], act: Sequence[int], sending_silos: Sequence[int],
                              keys: Sequence[Tuple[int, int, int]], cache: LRUCache, functional: Sequence[int]):
    """apply_directory_cache with the LRU's side effect: every message of the batch whose owner is remote looks the cache
    up in batch order (LocalGrainDirectory.LocalLookup's cache branch, LocalGrainDirectory.cs:691-702 — TryGetValue stamps
    a found entry before GetLocalCacheData's IsValidSilo filter, :711-717)."""
    r_out, a_out = list(route), list(act)
    for i, (r, k) in enumerate(zip(route, keys)):
        if (r >> 16) & 0xFF != ST_REMOTE_OWNER:
            continue
        v = cache.try_get(k)
        if v is None:
            continue
        a, silo = v
        if not functional[silo]:
            continue
        fl = ((r >> 24) & 0xFF) | 0x08 | (FL_LOOPBACK if silo == sending_silos[i] else 0)
        r_out[i] = pack_route(r & 0xFF, silo, ST_HIT, fl)
        a_out[i] = a
    return r_out, a_out
