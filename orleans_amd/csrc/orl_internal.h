// orl_internal.h — layouts shared by the host side (orl_api.cpp) and the CDNA4 kernels (route_kernels.hip).
//
// Nothing here is part of the public ABI (include/orleans_route.h is).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "../../include/orleans_route.h"

namespace orl {

// ---- directory partition table (GrainDirectoryPartition, single-activation grains) -----------------
// Open addressing, linear probing, power-of-two slot count, load <= 0.5.  One 32-B slot per grain:
// the full 24-B GrainId key (UniqueKey.Equals compares N0,N1,TCD: UniqueKey.cs:248-255), the dense
// activation handle, the activation's silo (ActivationInfo.SiloAddress) and a state byte.  Two slots
// share a 64-B line, so a probe that steps once usually stays in the line it already fetched.
enum : uint8_t { SLOT_EMPTY = 0, SLOT_FULL = 1, SLOT_TOMB = 2,
                 SLOT_CLAIMING = 3,  // device insert: slot won by CAS, key being written (never outlives an insert call)
                 SLOT_CLAIMED = 4 }; // device insert: key written, activation not yet committed

struct alignas(32) DirSlot {
    uint64_t tcd;
    uint64_t n0;
    uint64_t n1;
    uint32_t act;
    uint8_t silo;
    uint8_t state;
    uint16_t pad;
};
static_assert(sizeof(DirSlot) == 32, "slot must be 32 bytes");

// Compact probe table: a 16-B copy of every slot of the partition at the same index (same chains), kept when
// every FULL slot holds a long-key grain (N0 = 0) whose TypeCodeData is one of <= kProbeTypes values listed in
// RouteParams.probe_tcd.  The key is then exactly (probe_tcd[tidx], 0, n1), so a probe compares n1 and the
// type index: half the bytes per probe and half the table footprint (32 MB instead of 64 MB at config 2),
// which is what the route kernel's random-probe rate depends on.  w = state | silo << 8 | tidx << 16.
constexpr uint32_t kProbeTypes = 8;
struct alignas(16) ProbeSlot {
    uint64_t n1;
    uint32_t act;
    uint32_t w;
};
static_assert(sizeof(ProbeSlot) == 16, "probe slot must be 16 bytes");
// 8-B form of the probe table ({key, value} u32 pairs) when additionally there is ONE type, every FULL N1 is below
// kProbe8Tomb and every FULL activation handle is below 2^24: key = (uint32_t)N1 (kProbe8Empty / kProbe8Tomb mark
// empty slots and tombstones), value = act | silo << 24.  16 MB at config 2.
constexpr uint32_t kProbe8Empty = 0xFFFFFFFFu;
constexpr uint32_t kProbe8Tomb = 0xFFFFFFFEu;

// Probe start: murmur3 fmix32 of the Jenkins uniform hash.  The uniform hash alone would do for one
// silo, but a GPU that holds only some ring ranges sees hashes confined to those ranges; fmix32 is a
// bijection that spreads any range over the whole table.
__host__ __device__ inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

// Start slot of a key in a directory table of mask + 1 (a power of two, <= 2^32) slots: the HIGH bits of fmix32(uniform
// hash) (multiply-shift), so the table's eighths are fmix32(h) >> 29 whatever its size — the slice a node rank can name
// for a message without knowing the owner's table size.
__host__ __device__ inline uint64_t dir_slot(uint32_t h, uint64_t mask) {
    return ((uint64_t)fmix32(h) * (mask + 1)) >> 32;
}

// ---- Jenkins lookup2, 24-byte form (JenkinsHash.cs:54-65, 126-144) ---------------------------------
#define ORL_MIX(a, b, c)                 \
    do {                                 \
        a -= b; a -= c; a ^= (c >> 13);  \
        b -= c; b -= a; b ^= (a << 8);   \
        c -= a; c -= b; c ^= (b >> 13);  \
        a -= b; a -= c; a ^= (c >> 12);  \
        b -= c; b -= a; b ^= (a << 16);  \
        c -= a; c -= b; c ^= (b >> 5);   \
        a -= b; a -= c; a ^= (c >> 3);   \
        b -= c; b -= a; b ^= (a << 10);  \
        c -= a; c -= b; c ^= (b >> 15);  \
    } while (0)

__host__ __device__ inline uint32_t jenkins3(uint64_t u1, uint64_t u2, uint64_t u3) {
    uint32_t a = 0x9e3779b9u, b = 0x9e3779b9u, c = 0u;
    a += (uint32_t)u1;
    b += (uint32_t)(u1 >> 32);
    c += (uint32_t)u2;
    ORL_MIX(a, b, c);
    a += (uint32_t)(u2 >> 32);
    b += (uint32_t)u3;
    c += (uint32_t)(u3 >> 32);
    ORL_MIX(a, b, c);
    c += 24u;
    ORL_MIX(a, b, c);
    return c;
}

// ---- f2: SiloAddress -> silo index (wire decoder) ----------------------------------------------------
// The serialized form of a SiloAddress (BinaryTokenStreamWriter.Write(SiloAddress), :482-486): 16 IP bytes,
// int32 port, int32 generation = six LE words.  SiloAddress.Equals compares endpoint + generation
// (SiloAddress.cs:246-250) and the writer is canonical, so equal addresses have equal words.  Open addressing,
// linear probing, 512 entries for at most 255 silos (load <= 1/2); silo 0xFF marks an empty entry.
constexpr uint32_t kSiloAddrSlots = 512;
struct alignas(32) SiloAddrEntry {
    uint32_t w[6];
    uint32_t silo;
    uint32_t pad;
};
__host__ __device__ inline uint32_t silo_addr_slot(const uint32_t w[6]) {
    uint32_t h = 0x811C9DC5u;
    for (int i = 0; i < 6; ++i) h = fmix32(h ^ w[i]) * 0x9E3779B1u;
    return fmix32(h) & (kSiloAddrSlots - 1u);
}

// ---- f2 emit: grain class name per type code (PlacementResult.GrainType for new placements) ---------------
constexpr uint32_t kGrainTypeSlots = 1024;
constexpr uint32_t kGrainTypeBlob = 1u << 16;
struct GrainTypeEntry {
    int32_t code;
    uint32_t off, len, used;
};

// ---- everything a route launch needs besides the messages (device copy, staged into LDS) ------------
struct alignas(16) RouteParams {
    int32_t ring_hash[ORL_MAX_RING];   // membershipRingList, ascending signed hash
    uint8_t ring_silo[ORL_MAX_RING];
    uint8_t active_list[256];          // functional silos ascending (HASH_SPREAD placement)
    uint32_t running[8];               // 256-bit masks
    uint32_t functional[8];
    uint32_t local[8];
    uint32_t ring_n;
    uint32_t seed;
    uint32_t policy;
    uint32_t n_active;
    uint32_t n_act;
    uint32_t cache_on;                 // directory cache populated: probe it for remote owners
    uint32_t n_probe_types;            // entries of probe_tcd (compact probe table)
    uint32_t n_wire_types;             // entries of wire_tcd (8-B exchange records; 0 = no 8-B form)
    uint64_t mem_tcd, mem_n0, mem_n1;  // Constants.SystemMembershipTableId
    uint64_t wire_digest;              // FNV-1a of wire_tcd[0, n_wire_types): ranks compare it before using the 8-B form
    uint64_t probe_tcd[kProbeTypes];   // TypeCodeData of type index i in ProbeSlot.w
    uint64_t wire_tcd[ORL_MAX_WIRE_TYPES];  // TypeCodeData of wire type index i in orl_wire8.meta bits 16-19
};
static_assert(sizeof(RouteParams) % 16 == 0, "params must be 16-B granular");

constexpr uint32_t kRouteThreads = 256;
constexpr uint32_t kItems = 16;                               // messages per thread per tile
constexpr uint32_t kTile = kRouteThreads * kItems;            // 4096 messages per tile
constexpr uint32_t kMaxRouteRows = 8192;  // route tiles (= stage-4 histogram rows) of a small batch's finer grid
constexpr uint32_t kMaxDigitBits = 11;                        // radix digit width cap (2048 bins)

// Radix plan for keys in [0, n_buckets): passes of <= kMaxDigitBits bits, low digit first (LSD).
struct RadixPlan {
    int passes;
    int shift[4];
    int bits[4];
};

inline RadixPlan make_plan(uint32_t max_key) {
    int total = 0;
    while ((max_key >> total) != 0 && total < 32) ++total;
    if (total == 0) total = 1;
    RadixPlan p{};
    p.passes = (total + (int)kMaxDigitBits - 1) / (int)kMaxDigitBits;
    int base = total / p.passes, extra = total % p.passes, s = 0;
    for (int i = 0; i < p.passes; ++i) {
        p.bits[i] = base + (i < extra ? 1 : 0);
        p.shift[i] = s;
        s += p.bits[i];
    }
    return p;
}

// Stage-4 plan for keys in [0, n_act] (n_act = the unresolved bucket).  Keys of up to 2 x kMaxDigitBits bits
// take the two-level path: one stable MSD pass by the high `hb` bits (skipped when hb == 0) groups the
// messages into 2^hb buckets, then each bucket is counting-sorted by its low `lb` bits in segments of at
// most seg_elems() messages; the per-key counts of that second level ARE the bucket offsets (one scan).
// Wider keys fall back to LSD passes (`lsd`) + offsets from the sorted keys.
constexpr uint32_t kSegChunk = kTile;  // messages per LDS round inside a segment
// LSD path's bucket offsets: queue of long empty-bucket gaps (k_offsets_gaps / k_offsets_long), 4096 pieces
constexpr size_t kGapQueueWords = 2 + 3 * 4096;

struct BucketPlan {
    bool two_level;
    int hb, lb;
    RadixPlan lsd;
};

inline BucketPlan make_bucket_plan(uint32_t max_key) {
    int total = 0;
    while ((max_key >> total) != 0 && total < 32) ++total;
    if (total == 0) total = 1;
    BucketPlan p{};
    p.two_level = total <= 2 * (int)kMaxDigitBits;
    // an odd width gives the extra bit to the MSD digit (21 bits: 11 + 10): the hot rank of config 3 at 8 ranks buckets in
    // 0.84 vs 0.89 ms and the median rank in 0.51 vs 0.55 ms (scripts/rank_cost_lab.py, two repeats); 20 bits stays 10 + 10
    // (9 + 11: 0.89 ms, 11 + 9: 0.78 ms vs 0.69 ms at config 2).  ORL_LB_CEIL=1: the extra bit to level 2 (A/B).
    static const bool lb_ceil = [] { const char* e = getenv("ORL_LB_CEIL"); return e && e[0] == '1'; }();
    p.lb = total <= (int)kMaxDigitBits ? total : lb_ceil ? (total + 1) / 2 : total / 2;  // 20 bits: 10 + 10
    // (23-24-bit keys as 12 + 12 measured 2.82 ms vs 1.57 ms for 3 LSD passes at config 3: Zipf-hot digits
    // serialise the rank atomics and 4096 bins per 4096-message segment make the column work dominate)
    p.hb = total - p.lb;
    p.lsd = make_plan(max_key);
    return p;
}

// Segment size of the two-level path: one LDS round per segment.  (Four rounds per segment cut the segment
// histogram traffic but left each key's output lines partially written for a whole segment lifetime: 3.5x
// write amplification at config 2, profiles/r01c_config2_pmc.txt.)  The segment count is bounded by
// ceil(n / seg) + min(2^hb, n) (each nonempty bucket adds at most one partial segment).
inline uint32_t seg_elems(uint64_t) { return kSegChunk; }
inline uint64_t max_segments(uint64_t n, int hb) {
    const uint64_t s = seg_elems(n);
    return (n + s - 1) / s + std::min<uint64_t>(1ull << hb, n);
}

// The directory partition table and the directory cache (AdaptiveGrainDirectoryCache) a route launch probes.
// cache == nullptr / RouteParams.cache_on == 0: remote owners give ORL_ST_REMOTE_OWNER without a probe.
// probe != nullptr: the compact probe table of `dir` is current and the route kernel probes it instead.
struct DirView {
    const DirSlot* dir;
    uint64_t mask;
    const DirSlot* cache;
    uint64_t cmask;
    const ProbeSlot* probe = nullptr;
    const uint32_t* probe_bad = nullptr;  // device-built probe table: nonzero = a key did not fit, probe `dir`
    const void* probe8 = nullptr;         // 8-B form of `probe` ({u32 key, u32 value} pairs) when the keys fit it
    bool lru = false;                     // the cache is populated: lookups stamp its LRU generations (k_route<..., LRU>)
};

// ---- kernel launchers (route_kernels.hip) ---------------------------------------------------------
// All return hipError_t as int; they only enqueue on `stream`.
// KeyExt (string-key) directory slot, 48 B (round 5): the UniqueKey's 24 B, its KeyExt uniform hash, the activation
// handle, where the KeyExt bytes lie in the context's KeyExt blob, the silo and the slot state (SLOT_*).  Open addressing
// from dir_slot(hash) like the main partition.
struct ExtSlot {
    uint64_t tcd, n0, n1;
    uint32_t hash, act, off, len;
    uint8_t silo, state, pad[6];
};
static_assert(sizeof(ExtSlot) == 48, "KeyExt slot layout");

// Fused level 2 on skewed plans: segments per look-back chunk (k_seg_count_scan's kLbRows, ORL_SEG_LB_ROWS for lab builds)
// is at least this; the look-back buffers are sized for it.
constexpr uint32_t kSegLbMinRows = 8;

struct Scratch {
    uint2* pairs_a;         // [max_batch] {key, index} between radix passes
    uint2* pairs_b;         // [max_batch]
    uint32_t* idx_a;        // [max_batch + 1] fan-out publish offsets
    uint32_t* sorted_keys;  // [max_batch] (LSD fallback only)
    uint32_t* tile_hist;    // [2048 * rows] per-(tile, digit) output bases (col_scan's output; also a u32 scan buffer)
    uint16_t* tile_cnt;     // [2048 * rows] per-(tile, digit) counts written by the histogram passes (col_scan's input)
    uint32_t* scan_sums;    // [scan blocks]
    uint32_t* col_sums;     // [ceil(max_tiles/64) * 2048] column-scan chunk sums
    uint32_t* col_tot;      // [2048 + 1] column totals (+ the hot key's at [bins])
    uint8_t* digits;        // [max_batch] (partition by owner)
    uint32_t* seg_hist;     // [max segments][2^lb] two-level path: per-segment low-digit counts → bases
    uint32_t* seg_carry;    // [seg_lb_cap][2^lb] skewed plans: each segment chunk's carry-in (legacy scan: chunk sums first)
    uint32_t* seg_meta;     // [seg_lb_cap] skewed plans: each chunk's first bucket (+ shape bits in the legacy scan)
    uint32_t* seg_lb = nullptr;     // [2][seg_lb_cap][2^lb] fused level 2, skewed plans: chunk aggregate rows, inclusive rows
    uint32_t* seg_lbctl = nullptr;  // [4 + seg_lb_cap] ticket, done count, -, -, then one look-back flag per chunk (zeroed once)
    uint32_t seg_lb_cap = 0;        // chunks of kSegLbMinRows segments the look-back buffers hold
    mutable uint32_t seg_epoch = 0; // fused level-2 launches so far (the flags' epoch)
    uint32_t* bstart;       // [4097] bucket starts (two-level path; k_seg_plan handles up to 4096)
    uint32_t* sstart;       // [4098] first segment of each bucket; [4097] = a bucket has > 64 segments (skew flag)
    uint32_t* gap_q;        // [kGapQueueWords] LSD offsets: long-gap queue (zeroed once; k_offsets_long empties it)
    // one-pass exchange partition's look-back state, one set per stream that partitions (round 6: the node partitions
    // alternate chunks on two streams, so one chunk's tail overlaps the next chunk's start); a set taken over by another
    // stream is first waited for (its event), so launches that share a set never overlap
    struct LbSet {
        uint32_t* state = nullptr;  // ticket, error, 8 granules per 2048-message tile (zeroed once)
        uint32_t ticket = 0;        // host mirror of the ticket counter after the launches so far (tile = ticket - base)
        uint32_t epoch = 0;         // launches so far: the granules of launch k carry epoch k (earlier ones read as unpublished)
        hipStream_t stream = nullptr;
        hipEvent_t ev = nullptr;    // recorded after each launch on the set
        uint64_t last = 0;          // lb_clock at the last use (least recently used set is taken over)
    };
    static constexpr int kLbSets = 2;
    LbSet lb[kLbSets];
    uint64_t lb_clock = 0;
    uint64_t max_batch;
    uint64_t max_tiles;
    int device = -1;        // the context's HIP device: picks the ranking variant of its stage-4 launches (host_rm)
    uint32_t* hot = nullptr;  // stage 4's hot-key slots: [parity] the key in use (0xFFFFFFFF none), [parity ^ 1] the next pick
    mutable uint32_t hot_parity = 0;   // flips with every batch that picks (scan_offsets_pick)
    unsigned long long* hot_bmax = nullptr;  // [offset-scan chunks] per-chunk max of (count << 32 | key)
    unsigned long long* pick_word = nullptr; // the fused level-2 pick's max of (count << 32 | key), zero between batches
    uint32_t* hot_rows = nullptr;      // [rows + chunks] the hot key's count per histogram row, then its exclusive prefix
    uint32_t* lsd_hot = nullptr;       // [4] the LSD plan's hot-key path: {hot key, its messages hc, n - hc, -}
    uint32_t* hot_host = nullptr;      // mapped pinned host words: [0] the last pick's key (the launcher's hot-key hint), [1]
                                       // the last two-level plan's skew flag (k_seg_count_scan writes it): it picks the fused
                                       // level-2 kernel's solo form (no segment-scan launches) in launch_seg_bits
    uint32_t* hot_host_dev = nullptr;  // its device address
    mutable uint64_t hot_batches = 0;  // batches launched on the hot-key path (ORL_Q_HOT_BATCHES)
    uint32_t* fan_blk = nullptr;   // [fan_blk_cap] fan-out: the publisher of every 256th emitted message (k_scan_down WIDEN)
    uint32_t fan_blk_cap = 0;
    uint32_t gap_cap = 4096;  // LSD offsets' long-gap queue capacity (env_gap_cap() at context creation)
    int fan_u = 1;            // fan-out messages per thread and step (env_fan_u() at context creation)
    // LSD plan in single-sweep passes (round 6, k_sweep): look-back ring [1 << sw_rbits][1 << sw_row_bits] u64 (zeroed once),
    // control words {next ticket, launch base, done, -} (zeroed once), digit totals [3][2^kMaxDigitBits], each final digit's
    // largest key's low bits [2^kMaxDigitBits].  sw_ring == nullptr: the context's plan is two-level, or the ring would not
    // fit its budget — the LSD plan then takes the k_hist_pairs passes.
    unsigned long long* sw_ring = nullptr;
    uint32_t sw_rbits = 0, sw_row_bits = 0;
    uint32_t* sw_ctl = nullptr;
    uint32_t* sw_gtot = nullptr;
    uint32_t* sw_gmax = nullptr;
    // stage 4's look-back error word (the fused level-2 kernel's skewed form, k_sweep): |= 1 when a look-back gave up (a
    // device fault); read and cleared by ORL_Q_STAGE4_ERROR, checked by the node after every host-side stage 4.
    uint32_t* s4_err = nullptr;
};

// Knobs read from the environment once per context (orl_ctx_create): ORL_GAP_CAP, ORL_FAN_U.
uint32_t env_gap_cap();
int env_fan_u();

int launch_hash(const orl_grain_key* d_keys, size_t n, uint32_t* d_out, void* stream);
// Stage-4 ranking self-check on `device` (the current device; k_rank_selfcheck): selects the LDS-atomic rank (0) or the
// ballot fallback (1) for every kernel of this process on that device; mode 1 forces the fallback.  *ballot_out = mode | err << 1.
int launch_rank_selfcheck(int device, int mode, uint32_t* ballot_out);
// Sets `device`'s mode (the current device must be `device`): its kernels' flag word and the host mirror that picks the
// ranking-kernel variants of launches on contexts of that device.
int set_rank_mode(int device, uint32_t ballot);
// Host-changed slots of the partition: dir[idx[k]] = slots[k]; probe / probe8 (when non-null) patched alike.
int launch_dir_patch(const uint32_t* d_idx, const DirSlot* d_slots, const ProbeSlot* d_p16, const uint2* d_p8, uint32_t n,
                     DirSlot* d_dir, ProbeSlot* d_probe, uint2* d_probe8, void* stream);
// Compact probe table from the device partition (after device mutations), with the type list in d_params;
// *d_bad = 1 when a FULL slot is not a long key of a listed type.
int launch_probe_build(const DirSlot* d_dir, uint64_t slots, const RouteParams* d_params, ProbeSlot* d_probe,
                       uint32_t* d_bad, void* stream);
int launch_route_bucket(const RouteParams* d_params, const DirView& dv,
                        const void* d_in, int fmt, size_t n, uint32_t opts, uint32_t n_act, uint32_t* d_route,
                        uint32_t* d_act, uint32_t* d_order, uint32_t* d_offsets, const Scratch& s, void* stream,
                        void* ev_route_begin, void* ev_route_end, const uint32_t* d_in_act = nullptr);
int launch_fanout_route_bucket(const RouteParams* d_params, const DirView& dv, const orl_msg_hdr* d_direct, size_t n_direct,
                               const uint64_t* d_csr_off, const uint32_t* d_csr_tgt, const orl_grain_key* d_follower_keys,
                               const uint32_t* d_pubs, const uint8_t* d_pub_silo, size_t n_pub, uint64_t follower_tcd,
                               uint32_t opts, uint32_t n_act, uint64_t* d_pub_offsets, uint32_t* d_route, uint32_t* d_act,
                               uint32_t* d_order, uint32_t* d_offsets, uint64_t* n_out, uint64_t max_out,
                               const Scratch& s, void* stream, void* ev_route_begin, void* ev_route_end);
// Stage 5 alone: emitted messages as headers into d_out (cap records); -1 when the emitted count exceeds cap.
int launch_fanout_expand(const uint64_t* d_csr_off, const uint32_t* d_csr_tgt, const orl_grain_key* d_follower_keys,
                         const uint32_t* d_pubs, const uint8_t* d_pub_silo, size_t n_pub, uint64_t follower_tcd, uint32_t opts,
                         uint64_t* d_pub_offsets, orl_msg_hdr* d_out, uint64_t* n_out, uint64_t cap, const Scratch& s,
                         void* stream);
// Directory mutation on the device (dir kernels in route_kernels.hip).  d_claim: one u32 per table slot, all
// 0xFFFFFFFF between calls; d_cnt: {entries, tombstones} device counters; d_slot: one u32 per batch message.
int launch_dir_insert(const RouteParams* d_params, DirSlot* d_dir, uint64_t dir_mask, uint32_t* d_claim, uint64_t* d_cnt,
                      const orl_grain_key* d_keys, const uint32_t* d_acts, const uint8_t* d_silos, size_t n, uint32_t n_act,
                      uint32_t n_silos, uint32_t* d_slot, uint32_t* d_wact, uint8_t* d_wsilo, uint8_t* d_status, uint32_t* d_err,
                      void* stream);
int launch_cache_update(DirSlot* d_cache, uint64_t mask, uint32_t* d_claim, uint64_t* d_cnt, const orl_grain_key* d_keys,
                        const uint32_t* d_acts, const uint8_t* d_silos, size_t n, uint32_t n_act, uint32_t n_silos, uint32_t* d_slot,
                        uint8_t* d_flag, uint32_t* d_err, void* stream, const RouteParams* d_params);
// The directory cache's LRU generation base (after the cache table and its per-slot generations): += n, on `stream`.
int launch_cache_gen_advance(const DirSlot* d_cache, uint64_t mask, uint64_t n, void* stream);
int launch_dir_merge(DirSlot* d_dir, uint64_t dir_mask, uint32_t* d_claim, uint64_t* d_cnt, const orl_grain_key* d_keys,
                     const uint32_t* d_acts, const uint8_t* d_silos, size_t n, uint32_t n_act, uint32_t n_silos,
                     const orl_grain_key* d_act_keys, uint32_t n_act_keys, uint32_t* d_slot, uint8_t* d_status,
                     uint32_t* d_dropped_act, uint8_t* d_dropped_silo, uint32_t* d_err, void* stream);
int launch_dir_remove(DirSlot* d_dir, uint64_t dir_mask, uint32_t* d_claim, uint64_t* d_cnt, const orl_grain_key* d_keys,
                      size_t n, uint32_t* d_slot, uint8_t* d_removed, void* stream);
int launch_dir_split(const RouteParams* d_params, DirSlot* d_dir, uint64_t slots, uint32_t me, bool remove, uint64_t* d_cnt,
                     orl_grain_key* d_keys, uint32_t* d_acts, uint8_t* d_silos, uint64_t cap, uint64_t* d_n_out,
                     const Scratch& s, void* stream);
// Stream / reminder rings (f3).  kind: ORL_RING_CONSISTENT (the directory ring in RouteParams, clockwise, long
// compare) or ORL_RING_VBUCKETS (vr_hash/vr_silo: ascending bucket hashes).  excl_me: excludeMySelf.
int launch_ring_owner(uint32_t kind, const RouteParams* d_params, const uint32_t* d_vr_hash, const uint8_t* d_vr_silo,
                      uint32_t vr_n, const uint32_t* d_keys, size_t n, uint32_t me, bool excl_me, uint8_t* d_owner,
                      void* stream);
int launch_stream_queue(uint32_t kind, const RouteParams* d_params, const uint32_t* d_vr_hash, const uint8_t* d_vr_silo,
                        uint32_t vr_n, const uint8_t* d_guids, size_t n, uint32_t n_queues, uint32_t me, bool excl_me,
                        uint32_t* d_queue, uint8_t* d_silo, void* stream);
// f4: outbound queue per routed message; client gateway bucket per message.
int launch_outbound_queues(const orl_msg_hdr* d_msgs, const uint32_t* d_route, size_t n, uint32_t n_senders,
                           const int32_t* d_silo_hash, const uint8_t* d_silo_known, uint32_t* d_queue, void* stream);
int launch_client_buckets(const orl_msg_hdr* d_msgs, size_t n, uint32_t n_buckets, uint32_t* d_bucket, void* stream);
// f2: received frames -> orl_msg_hdr (wire_codec.hip).  d_bytes 4-byte aligned; d_flag: one device word of scratch.
int launch_decode_frames(const uint8_t* d_bytes, uint64_t nbytes, const uint64_t* d_offsets, size_t n,
                         uint32_t sender_override, const SiloAddrEntry* d_silo_tab, orl_msg_hdr* d_out,
                         uint8_t* d_status, uint32_t* d_n_bad, uint32_t* d_flag, void* stream);
// f2 emit (wire_codec.hip): SetTargetPlacement on routed frames.  d_sizes: n u64 of scratch; d_temp: the scan's
// temporary storage of stamp_scan_temp_bytes(n) bytes.
int launch_stamp_frames(const uint8_t* d_bytes, uint64_t nbytes, const uint64_t* d_offsets, size_t n, const uint32_t* d_route,
                        const uint32_t* d_act, const orl_grain_key* d_act_keys, uint32_t n_act_keys,
                        const orl_grain_key* d_new_act_keys, const GrainTypeEntry* d_gt, const uint8_t* d_gt_blob,
                        const uint32_t* d_silo_words, uint64_t* d_sizes, void* d_temp, size_t temp_bytes, uint8_t* d_out,
                        uint64_t out_cap, uint64_t* d_out_offsets, uint64_t* d_out_total, uint8_t* d_status, void* stream);
size_t stamp_scan_temp_bytes(size_t n);
// A node batch's KeyExt strings for the hop-1 partition (k_part_lb KX): the caller's references and blob, and the lanes
// they are written to (ext_out: one orl_ext_ref per record in the padded regions; blob_out: blob_cap bytes per destination,
// appended at cur[destination], u32 each).
struct KxLanes {
    const orl_ext_ref* ext;
    const uint8_t* blob;
    uint64_t blob_bytes;
    orl_ext_ref* ext_out;
    uint8_t* blob_out;
    uint64_t blob_cap;
    uint32_t* cur;
};
int launch_partition_padded(const RouteParams* d_params, const orl_msg_hdr* d_in, size_t n, uint32_t opts,
                            const uint8_t* d_rank_of_silo, uint32_t nranks, uint32_t my_rank, uint64_t stride,
                            void* d_out, int fmt, uint32_t* d_src_index, uint64_t* d_counts, uint32_t* d_wire_status,
                            Scratch& s, void* stream, const DirSlot* d_cache = nullptr, uint64_t cmask = 0,
                            uint32_t* d_act_out = nullptr, const KxLanes* kxl = nullptr);
// The received ext-ref lane of a chunk: source s's references (cnt[s] records, in rank order) += base[s].
int launch_ext_rebase(orl_ext_ref* d_refs, uint64_t n, uint32_t nranks, const uint64_t* cnt, const uint64_t* base, void* stream);
// Stage 4 alone over already-routed messages (activation handles): histogram + bucket_after_route.
int launch_bucket_acts(const uint32_t* d_act, size_t n, uint32_t n_act, uint32_t* d_order, uint32_t* d_offsets, const Scratch& s,
                       void* stream);
// Node hop 2: per-rank counts of routed messages by their host silo's rank (d_counts[8] u64, zeroed here), and the
// stable partition of {record, route, act} by host rank into padded regions (d_state: part_state_bytes(n) bytes).
int launch_host_rank_count(const uint32_t* d_route, size_t n, const uint8_t* d_ros, uint32_t my_rank, uint64_t* d_counts,
                           void* stream);
size_t part_state_bytes(size_t n);
// Node fault injection: a one-lane kernel on `stream` that waits (bounded, seconds) until the host-visible *flag != 0.
int launch_node_stall(const uint32_t* flag, void* stream);
// d_base_in (optional, device u64[nranks]): positions continue after an earlier partition into the same regions
// (its totals); d_counts receives base + this input's counts.  d_err (optional): |= ORL_PART_LOOKBACK_FAILED when a
// tile's look-back gave up (accumulates over launches; the caller zeroes it).
int launch_part_routed(const uint8_t* d_ros, const void* d_in, int win, int wout, const uint32_t* d_route, const uint32_t* d_act,
                       size_t n, uint32_t my_rank, uint32_t nranks, uint64_t stride, void* d_out, uint32_t* d_route_out,
                       uint32_t* d_act_out, uint32_t* d_state, const uint64_t* d_base_in, uint64_t* d_counts,
                       const uint64_t* d_wire_tcd, uint32_t* d_err, void* stream);
// Device address of a context's wire types (RouteParams::wire_tcd), current once a route or partition call synced state.
const uint64_t* ctx_wire_tcd(const orl_ctx* c);
// The node's hop-1 partition (orl_api.cpp): records of `fmt` bytes (8 / 16 / 32) into padded per-rank regions, per-rank
// counts into d_counts, and the status word (no 16-B form | no 8-B form | ORL_PART_LOOKBACK_FAILED) for every width.
// d_act_out (optional): the context's directory cache, when populated, addresses messages with a remote owner at the
// sender (their records go to the cached activation's rank; d_act_out, an act lane in the same padded regions, gets
// their cached handles, ORL_NO_ACT for every other record; the status word gets ORL_PART_CACHED).
int ctx_partition_padded(orl_ctx* c, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const uint8_t* rank_of_silo,
                         uint32_t nranks, uint32_t my_rank, size_t stride, void* d_out, int fmt, uint64_t* d_counts,
                         uint32_t* d_status, void* stream, uint32_t* d_act_out = nullptr, const KxLanes* kxl = nullptr);
// The KeyExt lookups of received 32-B records (k_keyext_route over messages the route kernel left ORL_ST_KEYEXT_UNRESOLVED)
// with their ext-ref lane into d_blob; ctx_keyext_prepare uploads a changed KeyExt table first (call it before a batch).
int ctx_route_keyext_received(orl_ctx* c, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const orl_ext_ref* d_ext,
                              const uint8_t* d_blob, uint64_t blob_bytes, uint32_t* d_route, uint32_t* d_act, void* stream);
int ctx_keyext_prepare(orl_ctx* c);
// Whether the context's directory cache is configured and holds entries (the partition's cached destinations).
bool ctx_cache_on(orl_ctx* c);
// Device address of the context's stage-4 look-back error word (Scratch::s4_err).
const uint32_t* ctx_stage4_err(const orl_ctx* c);
// Stages 1-3 of received exchange records (fmt 8 / 16 / 32, no stage 4) with an optional act lane d_in_act: records the
// sender addressed from its directory cache (act != ORL_NO_ACT) get HIT | CACHED without a probe.
int ctx_route_received(orl_ctx* c, const void* d_in, int fmt, size_t n, uint32_t opts, uint32_t* d_route, uint32_t* d_act,
                       const uint32_t* d_in_act, void* stream);
// KeyExt grains of a routed batch (orl_route_keyext_device): each message k_route left ORL_ST_KEYEXT_UNRESOLVED gets
// its owner's lookup in the KeyExt table when the owner is local (HIT, or placement on a miss) or ORL_ST_REMOTE_OWNER.
// KeyExt registration on the device (k_kx_ins_probe / resolve / commit); d_state = {string bytes used, entries, tombstones,
// error}; d_slot: n words of scratch.
int launch_keyext_insert(const RouteParams* d_params, ExtSlot* d_table, uint64_t mask, uint32_t* d_claim, uint8_t* d_tblob,
                         uint64_t tblob_cap, const orl_grain_key* d_keys, const orl_ext_ref* d_ext, const uint8_t* d_blob,
                         uint64_t blob_bytes, const uint32_t* d_acts, const uint8_t* d_silos, size_t n, uint32_t n_act,
                         uint32_t n_silos, uint32_t* d_slot, uint32_t* d_wact, uint8_t* d_wsilo, uint8_t* d_status,
                         uint64_t* d_state, void* stream);
int launch_keyext_route(const RouteParams* d_params, const orl_msg_hdr* d_in, size_t n, const orl_ext_ref* d_ext,
                        const uint8_t* d_blob, uint64_t blob_bytes, const ExtSlot* d_table, uint64_t mask,
                        const uint8_t* d_tblob, uint32_t excl, uint32_t* d_route, uint32_t* d_act, void* stream);
int launch_partition_by_owner(const RouteParams* d_params, const orl_msg_hdr* d_in, size_t n, uint32_t opts,
                              const uint8_t* d_rank_of_silo, uint32_t nranks, uint32_t my_rank, orl_msg_hdr* d_out,
                              uint32_t* d_src_index, uint64_t* d_counts, const Scratch& s, void* stream);

}  // namespace orl
