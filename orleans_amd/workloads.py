"""Deterministic synthetic workloads of BASELINE.json's configs.

Fixed synthetic cluster for every config: silos ``10.0.0.{1..8}:11111`` generation 1; ring hashes are
``SiloAddress.GetConsistentHashCode`` (SHA-256, computed by the library); silo s lives on GPU
``s * k // 8`` when k GPUs run, so the routing decisions are identical at 1/2/4/8 GPUs.

The grain population is ChirperAccount long-key grains (type code =
CalculateIdHash("Orleans.Samples.Chirper.Grains.ChirperAccount")); activation handle of grain i = i;
each activation lives on its directory owner silo (host silo = directory owner).

Vectorised numpy helpers here are workload plumbing (they decide which silo registers which grain);
routing decisions themselves come only from the HIP library, and parity is checked against oracle/.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

from . import _lib as L
from .engine import calc_id_hash, grain_keys_from_longs, silo_consistent_hash

CHIRPER_ACCOUNT_CLASS = "Orleans.Samples.Chirper.Grains.ChirperAccount"
N_SILOS = 8
PORT = 11111
GENERATION = 1

SEED_C2 = 0x5EED0002
SEED_C3 = 0x5EED0003
SEED_C4 = 0x5EED0004
SEED_C5 = 0x5EED0005

_M32 = np.uint32(0xFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser over a uint64 array (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = (np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)).astype(np.uint64)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def stream(seed: int, start: int, n: int) -> np.ndarray:
    """n pseudo-random u64 values for indices [start, start+n) of the stream `seed`."""
    idx = np.arange(start, start + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return splitmix64(idx * np.uint64(0x2545F4914F6CDD1D) + np.uint64(seed & 0xFFFFFFFFFFFFFFFF))


def jenkins3_np(u1: np.ndarray, u2: np.ndarray, u3: np.ndarray) -> np.ndarray:
    """Vectorised JenkinsHash.ComputeHash(ulong,ulong,ulong) (JenkinsHash.cs:126-144) for workload setup."""
    def lo(u):
        return (u & np.uint64(0xFFFFFFFF)).astype(np.uint32)

    def hi(u):
        return (u >> np.uint64(32)).astype(np.uint32)

    a = np.full(len(u1), 0x9E3779B9, np.uint32)
    b = a.copy()
    c = np.zeros(len(u1), np.uint32)

    def mix(a, b, c):
        a -= b; a -= c; a ^= (c >> 13)
        b -= c; b -= a; b ^= (a << 8)
        c -= a; c -= b; c ^= (b >> 13)
        a -= b; a -= c; a ^= (c >> 12)
        b -= c; b -= a; b ^= (a << 16)
        c -= a; c -= b; c ^= (b >> 5)
        a -= b; a -= c; a ^= (c >> 3)
        b -= c; b -= a; b ^= (a << 10)
        c -= a; c -= b; c ^= (b >> 15)

    with np.errstate(over="ignore"):
        a += lo(u1); b += hi(u1); c += lo(u2)
        mix(a, b, c)
        a += hi(u2); b += lo(u3); c += hi(u3)
        mix(a, b, c)
        c += np.uint32(24)
        mix(a, b, c)
    return c


@dataclass
class Cluster:
    n_silos: int
    hashes: np.ndarray        # int32 consistent hash per silo index
    ring_hash: np.ndarray     # int32, membershipRingList order
    ring_silo: np.ndarray     # uint8
    type_code: int
    gens: Tuple[int, ...] = ()  # generation per silo index (SiloAddress 10.0.0.{s+1}:PORT@gen)

    def silo_ip16(self, s: int) -> bytes:
        """Serialized IPv4 address of silo s (12 zero bytes + 4, BinaryTokenStreamWriter.cs:455-469)."""
        return bytes(12) + bytes([10, 0, 0, s + 1])

    def owner_of(self, uniform: np.ndarray) -> np.ndarray:
        """CalculateTargetSilo for running silos (no exclusion): predecessor-or-equal in signed order, wrap."""
        h = uniform.astype(np.uint32).view(np.int32)
        idx = np.searchsorted(self.ring_hash, h, side="right") - 1
        idx = np.where(idx < 0, len(self.ring_hash) - 1, idx)
        return self.ring_silo[idx]

    def rank_of_silo(self, nranks: int) -> np.ndarray:
        return np.array([s * nranks // self.n_silos for s in range(self.n_silos)], np.uint8)


def default_cluster(n_silos: int = N_SILOS, generations=None) -> Cluster:
    gens = [GENERATION] * n_silos if generations is None else list(generations)
    hashes = np.array([silo_consistent_hash(f"10.0.0.{s + 1}:{PORT}", gens[s]) for s in range(n_silos)], np.int32)
    # replay AddServer in silo-index order: insert at FindLastIndex(h < hash) + 1 (LocalGrainDirectory.cs:259-261)
    ring = []
    for s in range(n_silos):
        h = int(hashes[s])
        idx = max([i for i, (rh, _) in enumerate(ring) if rh < h], default=-1)
        ring.insert(idx + 1, (h, s))
    return Cluster(n_silos, hashes, np.array([h for h, _ in ring], np.int32), np.array([s for _, s in ring], np.uint8),
                   calc_id_hash(CHIRPER_ACCOUNT_CLASS), tuple(gens))


def grain_tcd(cl: Cluster, category: int = L.CAT_GRAIN) -> int:
    """TypeCodeData of the workload's long-key grain class: (category << 56) + sign-extended type code."""
    return ((category << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)) & 0xFFFFFFFFFFFFFFFF


def setup_engine(eng, cl: Cluster, local_silos: Optional[np.ndarray] = None, seed: int = 0) -> None:
    local = None
    if local_silos is not None:
        local = np.zeros(cl.n_silos, np.uint8)
        local[np.asarray(local_silos, dtype=np.int64)] = 1
    eng.set_silos(cl.n_silos, local=local, seed=seed)
    for s in range(cl.n_silos):
        eng.add_server(s, int(cl.hashes[s]))


def grain_population(cl: Cluster, n_grains: int, registered_frac: float = 1.0, seed: int = SEED_C2):
    """Keys of grains 0..n-1, their uniform hashes, owner silos, and which ones are registered."""
    keys = grain_keys_from_longs(cl.type_code, np.arange(n_grains, dtype=np.int64))
    uni = jenkins3_np(keys["tcd"], keys["n0"], keys["n1"])
    owner = cl.owner_of(uni)
    if registered_frac >= 1.0:
        reg = np.ones(n_grains, bool)
    else:
        r = stream(seed ^ 0xA11CE, 0, n_grains)
        reg = (r % np.uint64(1_000_000)) < np.uint64(int(registered_frac * 1_000_000))
    return keys, uni, owner, reg


def register_population(eng, keys: np.ndarray, owner: np.ndarray, reg: np.ndarray,
                        local_mask: Optional[np.ndarray] = None, dense_local: bool = False) -> int:
    """RegisterSingleActivation of grain i on its owner silo, activation handle i (or, with dense_local, the
    grain's rank among the registered grains of the local silos: a silo catalog numbers its own activations)."""
    sel = reg.copy()
    if local_mask is not None:
        sel &= local_mask[owner].astype(bool)
    idx = np.nonzero(sel)[0]
    acts = np.arange(len(idx), dtype=np.uint32) if dense_local else idx.astype(np.uint32)
    st, _, _ = eng.register_single_activation(keys[idx], acts, owner[idx])
    assert (st == L.INS_INSERTED).all(), np.unique(st, return_counts=True)
    return len(idx)


def uniform_messages(cl: Cluster, n_grains: int, n_msgs: int, seed: int = SEED_C2, start: int = 0,
                     sender_silos: Optional[np.ndarray] = None) -> np.ndarray:
    """Config 2 messages: targets Uniform[0, n_grains), sending silo from `sender_silos` (default all)."""
    t = stream(seed, start, n_msgs) % np.uint64(n_grains)
    s = stream(seed ^ 0x5E4D, start, n_msgs)
    silos = np.arange(cl.n_silos, dtype=np.uint8) if sender_silos is None else np.asarray(sender_silos, np.uint8)
    m = np.zeros(n_msgs, L.MSG_DTYPE)
    m["tcd"] = np.uint64(((L.CAT_GRAIN << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)) & 0xFFFFFFFFFFFFFFFF)
    m["n1"] = t
    m["sending_silo"] = silos[(s % np.uint64(len(silos))).astype(np.int64)]
    m["category"] = 2  # Application
    return m


def zipf_messages(cl: Cluster, n_grains: int, n_msgs: int, s_exp: float = 1.1, seed: int = SEED_C3, start: int = 0,
                  sender_silos: Optional[np.ndarray] = None) -> np.ndarray:
    """Config 3 messages: rank ~ Zipf(s) over [1, n_grains] mapped through a seeded permutation."""
    ranks = np.arange(1, n_grains + 1, dtype=np.float64)
    cdf = np.cumsum(ranks ** -s_exp)
    cdf /= cdf[-1]
    u = (stream(seed, start, n_msgs) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    r = np.searchsorted(cdf, u, side="right")
    r = np.minimum(r, n_grains - 1)
    perm = np.random.default_rng(seed).permutation(n_grains)
    m = uniform_messages(cl, n_grains, n_msgs, seed, start, sender_silos)
    m["n1"] = perm[r].astype(np.uint64)
    return m


# ---- the same generators as torch int64 arithmetic (on the device: 256M-message batches in milliseconds) ----------
def _s64(c: int) -> int:
    c &= 0xFFFFFFFFFFFFFFFF
    return c - (1 << 64) if c >= (1 << 63) else c


def _lsr(t, z, k: int):
    """Logical right shift of int64 tensors holding uint64 bits."""
    return (z >> k) & ((1 << (64 - k)) - 1)


def _t_stream(t, seed: int, start: int, n: int, device):
    idx = t.arange(start, start + n, dtype=t.int64, device=device)
    z = idx * _s64(0x2545F4914F6CDD1D) + _s64(seed)
    z = z + _s64(0x9E3779B97F4A7C15)
    z = (z ^ _lsr(t, z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ _lsr(t, z, 27)) * _s64(0x94D049BB133111EB)
    return z ^ _lsr(t, z, 31)


def _t_umod(t, z, m: int):
    """uint64 z mod m for int64 tensors holding uint64 bits (m < 2^62)."""
    return ((_lsr(t, z, 1) % m) * 2 + (z & 1)) % m


def zipf_cdf(n_grains: int, s_exp: float = 1.1) -> np.ndarray:
    ranks = np.arange(1, n_grains + 1, dtype=np.float64)
    cdf = np.cumsum(ranks ** -s_exp)
    cdf /= cdf[-1]
    return cdf


def device_messages(t, cl: Cluster, n_grains: int, n_msgs: int, seed: int, start: int = 0, sender_silos=None,
                    zipf: Optional[tuple] = None, device="cuda", chunk: int = 1 << 25):
    """uniform_messages / zipf_messages generated on `device` as an int32 [n, 8] tensor (orl_msg_hdr rows), bit-identical
    to the numpy generators.  zipf = (cdf tensor (float64, zipf_cdf), permutation tensor (int64)) for config 3."""
    out = t.zeros((n_msgs, 4), dtype=t.int64, device=device)
    silos = np.arange(cl.n_silos) if sender_silos is None else np.asarray(sender_silos)
    silos_t = t.as_tensor(silos.astype(np.int64), device=device)
    out[:, 0] = _s64(((L.CAT_GRAIN << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)) & 0xFFFFFFFFFFFFFFFF)
    for lo in range(0, n_msgs, chunk):
        k = min(chunk, n_msgs - lo)
        r = _t_stream(t, seed, start + lo, k, device)
        if zipf is None:
            tgt = _t_umod(t, r, n_grains)
        else:
            cdf, perm = zipf
            u = _lsr(t, r, 11).to(t.float64) * (1.0 / (1 << 53))
            rk = t.clamp(t.searchsorted(cdf, u, right=True), max=n_grains - 1)
            tgt = perm[rk]
        s = _t_stream(t, seed ^ 0x5E4D, start + lo, k, device)
        out[lo:lo + k, 2] = tgt
        out[lo:lo + k, 3] = silos_t[_t_umod(t, s, len(silos))] | (2 << 8)  # sending silo | Application category
    return out.view(t.int32)


def zipf_tables(t, n_grains: int, seed: int = SEED_C3, device="cuda"):
    """(cdf, permutation) device tensors of zipf_messages."""
    cdf = t.as_tensor(zipf_cdf(n_grains), device=device)
    perm = t.as_tensor(np.random.default_rng(seed).permutation(n_grains).astype(np.int64), device=device)
    return cdf, perm


def chirper_graph_deterministic(n_accounts: int = 1000, followers: int = 10, first_id: int = 1):
    """ChirperNetworkGenerator deterministic edges (NetworkGenerator/ChirperNetworkGenerator.cs:336-342):
    edge e: source = e // k, target = (source + 1 + e % k) % n (relative ids); `source follows target`,
    so target's followers include source (ChirperNetworkLoader.cs:231-242, 294-299)."""
    e = np.arange(n_accounts * followers, dtype=np.int64)
    src = e // followers
    tgt = (src + 1 + e % followers) % n_accounts
    return src + first_id, tgt + first_id


def csr_from_edges(publisher: np.ndarray, follower: np.ndarray, n_nodes: int):
    """Followers of each publisher in edge order (stable), as CSR offsets[n+1] (u64) / targets[E] (u32)."""
    order = np.argsort(publisher, kind="stable")
    counts = np.bincount(publisher, minlength=n_nodes)
    off = np.zeros(n_nodes + 1, np.uint64)
    off[1:] = np.cumsum(counts)
    return off, follower[order].astype(np.uint32)


def powerlaw_csr(n_nodes: int, exponent: float = 2.1, dmin: int = 1, dmax: int = 100_000, seed: int = SEED_C4):
    """Config 4 CSR: follower counts ~ discrete power law, follower ids uniform."""
    u = (stream(seed, 0, n_nodes) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    # inverse-CDF of continuous power law on [dmin, dmax], floored
    a = 1.0 - exponent
    d = ((dmax ** a - dmin ** a) * u + dmin ** a) ** (1.0 / a)
    deg = np.clip(np.floor(d).astype(np.int64), dmin, dmax)
    off = np.zeros(n_nodes + 1, np.uint64)
    off[1:] = np.cumsum(deg)
    e = int(off[-1])
    tgt = (stream(seed ^ 0xF011, 0, e) % np.uint64(n_nodes)).astype(np.uint32)
    return off, tgt


def balanced_generations(n_silos: int = N_SILOS, tol: float = 0.004) -> list:
    """Smallest silo generations >= 1 that put silo s's ring point within +-tol of s/n of the hash ring.

    The reference's directory ring has ONE point per silo (LocalGrainDirectory.AddServer, :243-268), so with
    generation-1 silos the 8 arcs are 0.4 % .. 35.7 % of the ring (a GPU hosting one silo would receive up to
    2.85x the average share at 8 GPUs).  Silo generations are deployment timestamps (SiloAddress.Generation),
    so choosing them is a deployment choice: the multi-GPU bench uses this balanced ring so weak scaling
    measures the engine, not the accident of 8 random ring points."""
    out = []
    span = 1 << 32
    for s in range(n_silos):
        target = -(1 << 31) + s * span // n_silos + span // (2 * n_silos)
        g = 1
        while abs(silo_consistent_hash(f"10.0.0.{s + 1}:{PORT}", g) - target) > tol * span:
            g += 1
        out.append(g)
    return out


def balanced_cluster(n_silos: int = N_SILOS) -> Cluster:
    return default_cluster(n_silos, balanced_generations(n_silos))


# ---- config 5: Presence heartbeats (Samples/Presence) ------------------------------------------------------
GAME_GRAIN_CLASS = "PresenceGrains.GameGrain"      # Samples/Presence/PresenceGrains/GameGrain.cs:32,39
PLAYER_GRAIN_CLASS = "PresenceGrains.PlayerGrain"  # Samples/Presence/PresenceGrains/PlayerGrain.cs:32,37
# LoadGenerator.GetPlayerId base Guid {2349992C-860A-4EDA-9590-000000000000} (Samples/Presence/LoadGenerator/
# Program.cs:86-91) as Guid.ToByteArray(): Data1/2/3 little-endian, then the 8 trailing bytes.
PLAYER_GUID_BASE = bytes([0x2C, 0x99, 0x49, 0x23, 0x0A, 0x86, 0xDA, 0x4E, 0x95, 0x90, 0, 0, 0, 0, 0, 0])


def player_guid_bytes(n_players: int) -> np.ndarray:
    """Player Guids.  The reference adds the player index to byte 15 only (wrapping at 256); for 800k distinct
    players the index is written big-endian into bytes 10..15, which equals the reference for index < 256."""
    g = np.tile(np.frombuffer(PLAYER_GUID_BASE, np.uint8), (n_players, 1))
    idx = np.arange(n_players, dtype=np.uint64)
    for b in range(6):
        g[:, 15 - b] = ((idx >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.uint8)
    return g


def game_guid_bytes(n_games: int, seed: int = SEED_C5) -> np.ndarray:
    """Game Guids: the reference uses Guid.NewGuid() (random); here 16 seeded splitmix64 bytes per game."""
    r = stream(seed, 0, 2 * n_games).reshape(n_games, 2)
    return r.view(np.uint8).reshape(n_games, 16).copy()


@dataclass
class Presence:
    game_keys: np.ndarray     # KEY_DTYPE[n_games]
    player_keys: np.ndarray   # KEY_DTYPE[n_games * per_game]
    csr_off: np.ndarray       # u64[n_games + 1]: game g -> players [g*k, g*k+k)
    csr_tgt: np.ndarray       # u32[n_games * k]
    per_game: int


def presence_population(n_games: int = 100_000, per_game: int = 8, seed: int = SEED_C5) -> Presence:
    from .engine import grain_keys_from_guid_bytes
    gtc = calc_id_hash(GAME_GRAIN_CLASS)
    ptc = calc_id_hash(PLAYER_GRAIN_CLASS)
    games = grain_keys_from_guid_bytes(gtc, game_guid_bytes(n_games, seed))
    players = grain_keys_from_guid_bytes(ptc, player_guid_bytes(n_games * per_game))
    off = (np.arange(n_games + 1, dtype=np.uint64) * np.uint64(per_game)).astype(np.uint64)
    tgt = np.arange(n_games * per_game, dtype=np.uint32)
    return Presence(games, players, off, tgt, per_game)


def heartbeat_batch(pr: Presence, cl: Cluster, n_hb: int, batch: int, seed: int = SEED_C5):
    """One batch of heartbeats: game index per heartbeat (uniform) and the game-message headers, sent from the
    PresenceGrain's silo (a StatelessWorker, local to the receiving silo: uniform over silos)."""
    g = (stream(seed ^ 0xB0B, batch * n_hb, n_hb) % np.uint64(len(pr.game_keys))).astype(np.int64)
    s = stream(seed ^ 0x5E4D, batch * n_hb, n_hb)
    m = np.zeros(n_hb, L.MSG_DTYPE)
    k = pr.game_keys[g]
    m["tcd"], m["n0"], m["n1"] = k["tcd"], k["n0"], k["n1"]
    m["sending_silo"] = (s % np.uint64(cl.n_silos)).astype(np.uint8)
    m["category"] = 2
    return g.astype(np.uint32), m


# ---- f2: received frames (Message.Serialize_Impl layout) --------------------------------------------------
# A typical request's header dictionary as InsideRuntimeClient.SendRequestMessage / Message.CreateMessage fill it
# (src/Orleans/Runtime/InsideRuntimeClient.cs, src/Orleans/Messaging/Message.cs): category, direction,
# correlation id, interface / method ids, sending silo / grain / activation, target grain, expiration; a
# response-style frame also carries TARGET_SILO + TARGET_ACTIVATION (a complete address).  Serialized per
# SerializationManager.SerializeMessageHeaders (token StringObjDict, count, byte key + token + value).
_H = dict(CATEGORY=3, CORRELATION_ID=4, DIRECTION=6, EXPIRATION=7, INTERFACE_ID=9, METHOD_ID=10,
          SENDING_ACTIVATION=18, SENDING_GRAIN=19, SENDING_SILO=20, TARGET_ACTIVATION=22, TARGET_GRAIN=23,
          TARGET_SILO=24)
_T_INT, _T_DATE, _T_STRDICT, _T_GRAIN, _T_ACT, _T_SILO, _T_CORR = 11, 25, 50, 40, 41, 42, 44


class _FrameTemplate:
    """One header shape: frame bytes with placeholders, and the offsets of the per-message fields."""

    def __init__(self, complete: bool, ext_len: int):
        b = bytearray(8)  # int32 header length, int32 body length
        at = {}

        def entry(key, tok):
            b.append(_H[key])
            b.append(tok)

        def field(name, n):
            at[name] = len(b)
            b.extend(bytes(n))

        def i32(v):
            b.extend(int(v).to_bytes(4, "little", signed=True))

        b.append(_T_STRDICT)
        i32(12 if complete else 10)
        entry("CATEGORY", _T_INT); i32(2)                       # Categories.Application
        entry("DIRECTION", _T_INT); i32(0)                      # Directions.Request
        entry("CORRELATION_ID", _T_CORR); field("corr", 8)
        entry("INTERFACE_ID", _T_INT); field("iface", 4)
        entry("METHOD_ID", _T_INT); field("method", 4)
        entry("SENDING_SILO", _T_SILO); field("ss", 24)
        entry("SENDING_GRAIN", _T_GRAIN); field("sg", 24); i32(-1)
        entry("SENDING_ACTIVATION", _T_ACT); field("sa", 24); i32(-1)
        entry("TARGET_GRAIN", _T_GRAIN); field("tg", 24)
        if ext_len:
            i32(ext_len); field("ext", ext_len)
        else:
            i32(-1)
        entry("EXPIRATION", _T_DATE); field("exp", 8)
        if complete:
            entry("TARGET_SILO", _T_SILO); field("ts", 24)
            entry("TARGET_ACTIVATION", _T_ACT); field("ta", 24); i32(-1)
        self.hl = len(b) - 8
        b[0:4] = self.hl.to_bytes(4, "little")
        self.bytes = np.frombuffer(bytes(b), np.uint8)
        self.at = at


def _put(rows: np.ndarray, pos: int, vals: np.ndarray, dtype: str) -> None:
    v = np.ascontiguousarray(vals.astype(dtype))
    rows[:, pos:pos + v.dtype.itemsize] = v.view(np.uint8).reshape(len(v), v.dtype.itemsize)


def _silo_words(cl: Cluster, silo: np.ndarray) -> np.ndarray:
    tab = np.zeros((cl.n_silos, 24), np.uint8)
    for s in range(cl.n_silos):
        tab[s] = np.frombuffer(cl.silo_ip16(s) + PORT.to_bytes(4, "little") +
                               int(cl.gens[s] if cl.gens else GENERATION).to_bytes(4, "little", signed=True), np.uint8)
    return tab[silo]


def request_frames(cl: Cluster, n_grains: int, n_frames: int, seed: int = SEED_C2, complete_frac: float = 0.0,
                   keyext_frac: float = 0.0, ext_lens=(11, 29), max_body: int = 48, chunk: int = 1 << 16):
    """n_frames back-to-back frames (one receive buffer) addressed like config 2 (target ~ Uniform[0, n_grains),
    sender ~ uniform silo) with `complete_frac` response-style complete addresses and `keyext_frac` KeyExt target
    grains (ASCII extensions of the given lengths).  Returns (buffer u8 padded to 4 bytes, frame offsets u64,
    expected headers MSG_DTYPE — aux left 0: the KeyExt hash is the decoder's to compute)."""
    r = [stream(seed ^ k, 0, n_frames) for k in (0x11, 0x22, 0x33, 0x44, 0x55, 0x66)]
    tgt = r[0] % np.uint64(n_grains)
    sender = (r[1] % np.uint64(cl.n_silos)).astype(np.int64)
    u = (r[2] >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    complete = u < complete_frac
    u2 = (r[3] >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    ext_cls = np.where(u2 < keyext_frac, 1 + (r[3] % np.uint64(len(ext_lens))).astype(np.int64), 0)
    body = ((r[4] % np.uint64(max_body // 8 + 1)) * np.uint64(8)).astype(np.int64) if max_body else np.zeros(n_frames, np.int64)
    tsilo = (r[5] % np.uint64(cl.n_silos)).astype(np.int64)
    shapes = {}
    for c in (False, True):
        for e in range(len(ext_lens) + 1):
            shapes[(c, e)] = _FrameTemplate(c, ext_lens[e - 1] if e else 0)
    shape_id = complete.astype(np.int64) * (len(ext_lens) + 1) + ext_cls
    hl = np.array([shapes[(c, e)].hl for c in (False, True) for e in range(len(ext_lens) + 1)], np.int64)[shape_id]
    size = 8 + hl + body
    offs = np.zeros(n_frames, np.uint64)
    offs[1:] = np.cumsum(size[:-1]).astype(np.uint64)
    total = int(size.sum())
    buf = np.zeros((total + 3) // 4 * 4, np.uint8)
    grain_tcd = np.uint64(((L.CAT_GRAIN << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)) & 0xFFFFFFFFFFFFFFFF)
    keyext_tcd = np.uint64(((6 << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)) & 0xFFFFFFFFFFFFFFFF)
    act_tcd = np.uint64(((L.CAT_GRAIN << 56)) & 0xFFFFFFFFFFFFFFFF)
    exp = np.full(n_frames, (1 << 62) | 638000000000000000, np.int64)  # a UTC DateTime.ToBinary
    exp = exp + (r[2] % np.uint64(10_000_000)).astype(np.int64)
    sw = _silo_words(cl, sender)
    tw = _silo_words(cl, tsilo)
    for (c, e), tpl in shapes.items():
        sel = np.nonzero(shape_id == (int(c) * (len(ext_lens) + 1) + e))[0]
        for lo in range(0, len(sel), chunk):
            idx = sel[lo:lo + chunk]
            k = len(idx)
            rows = np.tile(tpl.bytes, (k, 1))
            _put(rows, 4, body[idx], "<i4")
            _put(rows, tpl.at["corr"], r[4][idx] >> np.uint64(1), "<u8")
            _put(rows, tpl.at["iface"], np.full(k, cl.type_code, np.int64), "<i4")
            _put(rows, tpl.at["method"], (r[5][idx] >> np.uint64(40)) % np.uint64(7), "<i4")
            rows[:, tpl.at["ss"]:tpl.at["ss"] + 24] = sw[idx]
            sg = np.zeros((k, 3), np.uint64)
            sg[:, 1] = r[1][idx] >> np.uint64(8)
            sg[:, 2] = grain_tcd
            rows[:, tpl.at["sg"]:tpl.at["sg"] + 24] = sg.view(np.uint8).reshape(k, 24)
            sa = np.zeros((k, 3), np.uint64)
            sa[:, 0] = r[2][idx]
            sa[:, 1] = r[3][idx]
            sa[:, 2] = act_tcd
            rows[:, tpl.at["sa"]:tpl.at["sa"] + 24] = sa.view(np.uint8).reshape(k, 24)
            tg = np.zeros((k, 3), np.uint64)
            tg[:, 1] = tgt[idx]
            tg[:, 2] = keyext_tcd if e else grain_tcd
            rows[:, tpl.at["tg"]:tpl.at["tg"] + 24] = tg.view(np.uint8).reshape(k, 24)
            if e:
                n_ext = ext_lens[e - 1]
                letters = stream(seed ^ 0x77, int(lo), k * n_ext).reshape(k, n_ext) % np.uint64(26) + np.uint64(97)
                rows[:, tpl.at["ext"]:tpl.at["ext"] + n_ext] = letters.astype(np.uint8)
            _put(rows, tpl.at["exp"], exp[idx], "<i8")
            if c:
                rows[:, tpl.at["ts"]:tpl.at["ts"] + 24] = tw[idx]
                ta = np.zeros((k, 3), np.uint64)
                ta[:, 0] = r[0][idx]
                ta[:, 1] = r[5][idx]
                ta[:, 2] = act_tcd
                rows[:, tpl.at["ta"]:tpl.at["ta"] + 24] = ta.view(np.uint8).reshape(k, 24)
            L_ = rows.shape[1]
            buf[(offs[idx].astype(np.int64)[:, None] + np.arange(L_)[None, :]).ravel()] = rows.ravel()
    exp_m = np.zeros(n_frames, L.MSG_DTYPE)
    exp_m["tcd"] = np.where(ext_cls > 0, keyext_tcd, grain_tcd)
    exp_m["n1"] = tgt
    exp_m["sending_silo"] = sender.astype(np.uint8)
    exp_m["category"] = 2
    exp_m["flags"] = np.where(complete, L.HDR_ADDRESS_COMPLETE, 0) | np.where(ext_cls > 0, L.HDR_HASH_VALID, 0)
    exp_m["target_silo"] = np.where(complete, tsilo, 0).astype(np.uint8)
    return buf, offs, exp_m


def register_silo_addresses(eng, cl: Cluster) -> None:
    """The decoder's silo address table for the synthetic cluster."""
    for s in range(cl.n_silos):
        eng.set_silo_address(s, cl.silo_ip16(s), PORT, int(cl.gens[s] if cl.gens else GENERATION))
