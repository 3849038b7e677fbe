// orl_api.cpp — host side of liborleans_route.so: context, silo table + ring (membership events),
// directory partition mirror (registration), identity hashes, and the C ABI entry points.
//
// The host side is the control plane of the path: everything here runs once per membership change or
// registration, never per message.  Per-message work is in route_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <tuple>
#include <vector>

#include "orl_internal.h"

using namespace orl;

namespace {

// ---- SHA-256 (FIPS 180-4), for Utils.CalculateIdHash (Utils.cs:201-220) ---------------------------------
struct Sha256 {
    uint32_t h[8];
    uint8_t buf[64];
    uint64_t len = 0;
    size_t fill = 0;
    static constexpr uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    Sha256() {
        static const uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                       0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
        std::memcpy(h, H0, sizeof h);
    }
    static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
    void block(const uint8_t* p) {
        uint32_t w[64];
        for (int i = 0; i < 16; ++i) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; ++i) {
            const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
            const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int i = 0; i < 64; ++i) {
            const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
            const uint32_t ch = (e & f) ^ (~e & g);
            const uint32_t t1 = hh + S1 + ch + K[i] + w[i];
            const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
            const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
            const uint32_t t2 = S0 + mj;
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }
    void update(const uint8_t* p, size_t n) {
        len += n;
        while (n) {
            const size_t take = std::min(n, 64 - fill);
            std::memcpy(buf + fill, p, take);
            fill += take; p += take; n -= take;
            if (fill == 64) { block(buf); fill = 0; }
        }
    }
    void final(uint8_t out[32]) {
        const uint64_t bits = len * 8;
        const uint8_t one = 0x80, zero = 0;
        update(&one, 1);
        while (fill != 56) update(&zero, 1);
        uint8_t lb[8];
        for (int i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
        update(lb, 8);
        for (int i = 0; i < 8; ++i) {
            out[4 * i] = (uint8_t)(h[i] >> 24); out[4 * i + 1] = (uint8_t)(h[i] >> 16);
            out[4 * i + 2] = (uint8_t)(h[i] >> 8); out[4 * i + 3] = (uint8_t)h[i];
        }
    }
};
constexpr uint32_t Sha256::K[64];

// UTF-8 → UTF-16LE (.NET Encoding.Unicode).  Returns false on malformed input.
bool utf8_to_utf16le(const char* s, size_t n, std::vector<uint8_t>& out) {
    out.clear();
    size_t i = 0;
    auto put = [&](uint32_t u) { out.push_back((uint8_t)u); out.push_back((uint8_t)(u >> 8)); };
    while (i < n) {
        const uint8_t c = (uint8_t)s[i];
        uint32_t cp;
        int extra;
        if (c < 0x80) { cp = c; extra = 0; }
        else if ((c >> 5) == 6) { cp = c & 0x1F; extra = 1; }
        else if ((c >> 4) == 14) { cp = c & 0x0F; extra = 2; }
        else if ((c >> 3) == 30) { cp = c & 0x07; extra = 3; }
        else return false;
        if (i + (size_t)extra >= n && extra) return false;  // truncated sequence
        for (int k = 1; k <= extra; ++k) {
            const uint8_t cc = (uint8_t)s[i + k];
            if ((cc >> 6) != 2) return false;
            cp = (cp << 6) | (cc & 0x3F);
        }
        i += 1 + extra;
        if (cp >= 0x10000) {
            cp -= 0x10000;
            put(0xD800 + (cp >> 10));
            put(0xDC00 + (cp & 0x3FF));
        } else {
            put(cp);
        }
    }
    return true;
}

int32_t calc_id_hash_utf16(const std::vector<uint8_t>& u16) {
    Sha256 sh;
    sh.update(u16.data(), u16.size());
    uint8_t d[32];
    sh.final(d);
    uint32_t h = 0;
    for (int i = 0; i < 32; i += 4) h ^= (uint32_t)d[i] << 24 | (uint32_t)d[i + 1] << 16 | (uint32_t)d[i + 2] << 8 | d[i + 3];
    return (int32_t)h;
}

// JenkinsHash.ComputeHash(byte[]) (JenkinsHash.cs:68-115)
uint32_t jenkins_bytes(const uint8_t* d, size_t len) {
    uint32_t a = 0x9e3779b9u, b = 0x9e3779b9u, c = 0;
    size_t i = 0;
    auto rd = [&](size_t k) { return (uint32_t)d[k] | (uint32_t)d[k + 1] << 8 | (uint32_t)d[k + 2] << 16 | (uint32_t)d[k + 3] << 24; };
    while (i + 12 <= len) {
        a += rd(i); b += rd(i + 4); c += rd(i + 8);
        i += 12;
        ORL_MIX(a, b, c);
    }
    c += (uint32_t)len;
    const size_t rem = len - i;
    for (size_t k = 0; k < rem; ++k) {
        const uint32_t v = d[i + k];
        if (k < 4) a += v << (8 * k);
        else if (k < 8) b += v << (8 * (k - 4));
        else c += v << (8 * (k - 7));
    }
    ORL_MIX(a, b, c);
    return c;
}

// Stage-4 rank mode per device (launch_rank_selfcheck): -1 = not checked yet; else ballot | self-check error << 1.
std::mutex g_rank_mu;
int g_rank_state[64];
bool g_rank_init = false;

int ensure_rank_mode(int device) {
    std::lock_guard<std::mutex> lk(g_rank_mu);
    if (!g_rank_init) {
        for (int& x : g_rank_state) x = -1;
        g_rank_init = true;
    }
    if (device < 0 || device >= 64) return (int)hipErrorInvalidDevice;
    if (g_rank_state[device] >= 0) return 0;
    const char* m = getenv("ORL_RANK_MODE");
    uint32_t st = 0;
    int e = launch_rank_selfcheck(device, m && std::strcmp(m, "ballot") == 0 ? 1 : 0, &st);
    if (e) return e;
    g_rank_state[device] = (int)st;
    return 0;
}

// orl_route_batch: chunks per host-array batch (and the smallest chunk)
constexpr size_t kHostChunks = 8;
constexpr size_t kHostChunk = 1u << 20;

uint64_t next_pow2(uint64_t v) {
    uint64_t p = 16;
    while (p < v) p <<= 1;
    return p;
}

}  // namespace

// ---------------------------------------------------------------------------------------------------
struct orl_ctx {
    orl_config cfg{};
    bool device_mode = false;
    std::string err;
    // silos (LocalGrainDirectory membership view)
    uint32_t n_silos = 0;
    std::vector<uint8_t> running, functional, local;
    uint32_t seed = ORL_NULL_SILO;
    std::vector<std::pair<int32_t, uint8_t>> ring;  // membershipRingList (signed hash, silo)
    // directory partition mirror
    std::vector<DirSlot> table;
    uint64_t mask = 0, count = 0, tombs = 0;
    bool dir_dirty = true;           // the whole table must be uploaded (and the probe tables rebuilt)
    std::vector<uint32_t> dirty_slots;  // else: host-changed slots since the last upload, patched in place
    std::vector<uint8_t> slot_marked;   // dirty_slots membership (one byte per slot, allocated on first use)
    void* d_patch_data = nullptr;       // device staging of a slot patch (grows to the largest patch)
    size_t patch_cap = 0;
    uint64_t n_full_uploads = 0, n_patches = 0;
    // follower graph of orl_csr_set (host-array fan-out)
    uint64_t* d_csr_off = nullptr;
    uint32_t* d_csr_tgt = nullptr;
    size_t csr_nodes = 0;
    std::vector<uint64_t> h_csr_off;
    bool mirror_stale = false;       // device mutations since the mirror was last downloaded
    uint64_t count_ub = 0, tombs_ub = 0;  // upper bounds while the mirror is stale (capacity checks without a sync)
    // device state
    DirSlot* d_table = nullptr;
    ProbeSlot* d_probe = nullptr;    // compact probe table of d_table (ProbeSlot, orl_internal.h)
    bool probe_valid = false;        // d_probe mirrors d_table (set by the host upload, cleared by device mutations)
    bool probe_off = false;          // ORL_NO_PROBE16=1: always probe the 32-B table (A/B measurements)
    bool probe_dev = false;          // d_probe was built on the device: validity in *d_probe_bad
    uint2* d_probe8 = nullptr;       // 8-B form of the probe table (one type, 32-bit N1, 24-bit handles)
    bool probe8_valid = false;       // d_probe8 mirrors d_table (host upload only)
    bool probe8_off = false;         // ORL_NO_PROBE8=1: never the 8-B form (A/B measurements)
    bool probe_dev_stale = false;    // device mutations since: rebuild before the next route launch
    uint32_t* d_probe_bad = nullptr;
    uint32_t* d_claim = nullptr;     // per-slot claim word of the device insert/remove kernels (0xFFFFFFFF at rest)
    uint64_t* d_dirstate = nullptr;  // {entries, tombstones, error flag}
    uint32_t* d_dslot = nullptr;     // per-message slot of a device directory batch
    uint8_t* d_dflag = nullptr;      // per-message flag of a device cache batch
    // KeyExt grains (round 5): host table + extension blob, uploaded whole when changed.  Round 6: registrations on the
    // device (orl_dir_insert_keyext_device) make the device table the newer one (ext_dev_newer): the host functions first
    // download it (ext_sync_host).  ext_dirty (host newer) and ext_dev_newer never hold together.
    std::vector<ExtSlot> ext_table;
    std::vector<uint8_t> ext_blob;
    uint64_t ext_count = 0, ext_tombs = 0;
    bool ext_dirty = false;
    bool ext_dev_newer = false;
    uint64_t ext_count_ub = 0, ext_tombs_ub = 0, ext_blob_ub = 0;  // upper bounds while the device is newer
    uint64_t ext_blob_min_cap = 0;   // the device string store's capacity at the next upload (room for a device batch)
    ExtSlot* d_ext_table = nullptr;
    uint8_t* d_ext_blob = nullptr;
    size_t d_ext_table_cap = 0, d_ext_blob_cap = 0;
    uint32_t* d_ext_claim = nullptr;  // per-slot claim words of the device registration (0xFFFFFFFF at rest)
    size_t d_ext_claim_cap = 0;
    uint64_t* d_ext_state = nullptr;  // {string bytes used, entries, tombstones, error}
    // directory cache (AdaptiveGrainDirectoryCache, f4): device table of remote-owned grains
    DirSlot* d_cache = nullptr;
    uint32_t* d_cclaim = nullptr;
    uint64_t* d_cstate = nullptr;    // {entries, tombstones, error flag}
    uint64_t cache_slots = 0, cache_ub = 0, cache_tombs_ub = 0;
    uint64_t cache_cap = 0;       // LRU.MaximumSize (orl_cache_config's capacity)
    uint64_t cache_gen_free = 0;  // LRU.generationToFree: the generation of the last entry evicted
    RouteParams hp{};
    RouteParams* d_params = nullptr;
    bool params_dirty = true;
    uint8_t* d_rank_of_silo = nullptr;
    uint8_t h_rank_of_silo[256] = {};  // last uploaded rank_of_silo (uploads only on change: no per-batch sync)
    bool ros_valid = false;
    Scratch s{};
    hipStream_t stream = nullptr;
    // host-buffer staging (orl_route_batch / orl_hash_batch) and its copy streams / per-chunk events
    uint8_t* st_in = nullptr; size_t st_in_cap = 0;
    hipStream_t hstream[2] = {nullptr, nullptr};
    hipEvent_t hev[2 * (kHostChunks + 1)] = {};
    uint32_t* st_out = nullptr; size_t st_out_cap = 0;
    uint32_t* st_off = nullptr;
    // silo consistent hashes (SiloAddress.GetConsistentHashCode) for outbound sender queues
    int32_t silo_hash[256] = {};
    uint8_t silo_known[256] = {};
    bool silo_hash_dirty = true;
    int32_t* d_silo_hash = nullptr;
    uint8_t* d_silo_known = nullptr;
    // stream / reminder virtual-bucket ring (VirtualBucketsRingProvider.bucketsMap)
    uint32_t vr_nb = 30;
    std::map<uint32_t, uint8_t> vr_map;                // bucket hash → silo
    std::map<uint8_t, std::vector<uint32_t>> vr_hashes;  // silo → its GetUniformHashCodes
    std::map<uint8_t, int32_t> vr_gen;
    bool vr_dirty = false;
    uint32_t vr_n_dev = 0;
    uint32_t* d_vr_hash = nullptr;
    uint8_t* d_vr_silo = nullptr;
    // f2: serialized SiloAddress -> silo index for the wire decoder
    uint32_t silo_addr[256][6] = {};
    uint8_t silo_addr_known[256] = {};
    bool silo_addr_dirty = true;
    SiloAddrEntry* d_silo_tab = nullptr;
    uint32_t* d_decode_flag = nullptr;
    uint32_t* d_silo_words = nullptr;  // [256][6] serialized SiloAddress by silo index (stamp)
    // f2 emit: grain class names by type code, and the stamp's scratch
    std::map<int32_t, std::string> grain_types;
    bool gt_dirty = true;
    GrainTypeEntry* d_gt = nullptr;
    uint8_t* d_gt_blob = nullptr;
    uint64_t* d_stamp_sizes = nullptr;
    void* d_stamp_temp = nullptr;
    size_t stamp_cap = 0, stamp_temp_bytes = 0;
    // timing: 4 events per recorded batch (call begin, route begin, route end, call end)
    bool timing = false;
    std::vector<hipEvent_t> tev;
    uint32_t tcount = 0;
};

const uint64_t* orl::ctx_wire_tcd(const orl_ctx* c) {
    if (!c || !c->d_params) return nullptr;
    return reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint8_t*>(c->d_params) + offsetof(RouteParams, wire_tcd));
}

namespace {

int fail(orl_ctx* c, int code, const char* fmt, ...) {
    if (c) {
        char b[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(b, sizeof b, fmt, ap);
        va_end(ap);
        c->err = b;
    }
    return code;
}

int hipfail(orl_ctx* c, hipError_t e, const char* what) {
    return fail(c, ORL_E_DEVICE, "%s: %s", what, hipGetErrorString(e));
}

#define ORL_HIP(c, call)                                           \
    do {                                                           \
        hipError_t _e = (call);                                    \
        if (_e != hipSuccess) return hipfail((c), _e, #call);      \
    } while (0)

bool silo_ok(const orl_ctx* c, uint32_t s) { return s < c->n_silos; }

// CalculateTargetSilo on the host (LocalGrainDirectory.cs:439-497) for registrations.
uint32_t host_owner(const orl_ctx* c, const orl_grain_key& k, uint32_t me, bool excl) {
    const uint32_t cat = (uint32_t)(k.type_code_data >> 56);
    if (cat == ORL_CAT_SYSTEM_TARGET) return me;
    if (k.type_code_data == c->hp.mem_tcd && k.n0 == c->hp.mem_n0 && k.n1 == c->hp.mem_n1) return c->seed;
    const int32_t h = (int32_t)jenkins3(k.type_code_data, k.n0, k.n1);
    const bool running = me < c->n_silos && c->running[me];
    const int n = (int)c->ring.size();
    if (n == 0) return (excl && !running) ? ORL_NULL_SILO : me;
    const bool ex = excl && !running;
    int found = -1;
    for (int i = 0; i < n; ++i)
        if (c->ring[i].first <= h && !(c->ring[i].second == me && ex)) found = i;
    if (found < 0) {
        found = n - 1;
        if (c->ring[found].second == me && ex) {
            if (n > 1) found = n - 2; else return ORL_NULL_SILO;
        }
    }
    return c->ring[found].second;
}

void rebuild_params(orl_ctx* c) {
    RouteParams& P = c->hp;
    const uint64_t mt = P.mem_tcd, m0 = P.mem_n0, m1 = P.mem_n1;
    const uint32_t cache_on = P.cache_on, npt = P.n_probe_types, nwt = P.n_wire_types;
    const uint64_t wdig = P.wire_digest;
    uint64_t ptcd[kProbeTypes], wtcd[ORL_MAX_WIRE_TYPES];
    std::memcpy(ptcd, P.probe_tcd, sizeof ptcd);
    std::memcpy(wtcd, P.wire_tcd, sizeof wtcd);
    std::memset(&P, 0, sizeof P);
    P.mem_tcd = mt; P.mem_n0 = m0; P.mem_n1 = m1;
    P.cache_on = cache_on;
    P.n_probe_types = npt;
    std::memcpy(P.probe_tcd, ptcd, sizeof ptcd);
    P.n_wire_types = nwt;
    P.wire_digest = wdig;
    std::memcpy(P.wire_tcd, wtcd, sizeof wtcd);
    P.ring_n = (uint32_t)c->ring.size();
    for (size_t i = 0; i < c->ring.size(); ++i) {
        P.ring_hash[i] = c->ring[i].first;
        P.ring_silo[i] = c->ring[i].second;
    }
    uint32_t na = 0;
    for (uint32_t s = 0; s < c->n_silos; ++s) {
        if (c->running[s]) P.running[s >> 5] |= 1u << (s & 31);
        if (c->functional[s]) { P.functional[s >> 5] |= 1u << (s & 31); P.active_list[na++] = (uint8_t)s; }
        if (c->local[s]) P.local[s >> 5] |= 1u << (s & 31);
    }
    P.n_active = na;
    P.seed = c->seed;
    P.policy = c->cfg.placement_policy;
    P.n_act = c->cfg.n_act;
    c->params_dirty = true;
}

// Probe-table forms of one directory slot (ProbeSlot, orl_internal.h).  t = the slot's type index.
ProbeSlot probe16_of(const DirSlot& d, uint32_t t) {
    // EMPTY ends a chain, FULL is compared, every other state (tombstone) is stepped over
    const uint32_t state = d.state == SLOT_EMPTY ? SLOT_EMPTY : d.state == SLOT_FULL ? SLOT_FULL : SLOT_TOMB;
    if (d.state != SLOT_FULL) return ProbeSlot{0, 0, state};
    return ProbeSlot{d.n1, d.act, state | ((uint32_t)d.silo << 8) | (t << 16)};
}
uint2 probe8_of(const DirSlot& d) {  // {(uint32_t)N1, act | silo << 24}, EMPTY / TOMB as reserved keys
    if (d.state == SLOT_FULL) return make_uint2((uint32_t)d.n1, d.act | ((uint32_t)d.silo << 24));
    return make_uint2(d.state == SLOT_EMPTY ? kProbe8Empty : kProbe8Tomb, 0u);
}
bool fits8(const DirSlot& d) { return d.state != SLOT_FULL || (d.n1 < kProbe8Tomb && d.act < (1u << 24)); }

// Compact probe table from the host mirror: valid when every FULL slot is a long-key grain (N0 = 0) of at most
// kProbeTypes TypeCodeData values.  Slot i of d_probe describes slot i of d_table, so chains are identical.
int upload_probe(orl_ctx* c) {
    c->probe_valid = c->probe_dev = c->probe_dev_stale = c->probe8_valid = false;
    if (c->probe_off) return ORL_OK;
    uint64_t types[kProbeTypes];
    uint32_t nt = 0;
    if (c->count == 0 && c->tombs == 0) {  // empty partition: every probe slot EMPTY
        ORL_HIP(c, hipMemset(c->d_probe, 0, c->table.size() * sizeof(ProbeSlot)));
        c->hp.n_probe_types = 0;
        c->params_dirty = true;
        c->probe_valid = true;
        return ORL_OK;
    }
    for (const DirSlot& d : c->table) {
        if (d.state != SLOT_FULL) continue;
        if (d.n0 != 0) return ORL_OK;
        uint32_t t = 0;
        while (t < nt && types[t] != d.tcd) ++t;
        if (t == nt) {
            if (nt == kProbeTypes) return ORL_OK;
            types[nt++] = d.tcd;
        }
    }
    bool fit8 = nt == 1 && !c->probe8_off;
    for (size_t i = 0; fit8 && i < c->table.size(); ++i) fit8 = fits8(c->table[i]);
    if (fit8) {
        std::vector<uint2> p8(c->table.size());
        for (size_t i = 0; i < c->table.size(); ++i) p8[i] = probe8_of(c->table[i]);
        ORL_HIP(c, hipMemcpy(c->d_probe8, p8.data(), p8.size() * 8, hipMemcpyHostToDevice));
        c->probe8_valid = true;  // the 16-B form below is built too (the fan-out kernel reads it)
    }
    std::vector<ProbeSlot> pt(c->table.size());
    for (size_t i = 0; i < c->table.size(); ++i) {
        const DirSlot& d = c->table[i];
        uint32_t t = 0;
        if (d.state == SLOT_FULL)
            while (types[t] != d.tcd) ++t;
        pt[i] = probe16_of(d, t);
    }
    ORL_HIP(c, hipMemcpy(c->d_probe, pt.data(), pt.size() * sizeof(ProbeSlot), hipMemcpyHostToDevice));
    c->hp.n_probe_types = nt;
    std::memcpy(c->hp.probe_tcd, types, nt * sizeof(uint64_t));
    c->params_dirty = true;
    c->probe_valid = true;
    return ORL_OK;
}

// A host-side change of directory slot i (registration / unregistration through the host mirror).
void mark_slot(orl_ctx* c, uint64_t i) {
    if (c->dir_dirty) return;  // the whole table goes up anyway
    if (c->slot_marked.size() != c->table.size()) c->slot_marked.assign(c->table.size(), 0);
    if (c->slot_marked[i]) return;
    c->slot_marked[i] = 1;
    c->dirty_slots.push_back((uint32_t)i);
    if (c->dirty_slots.size() > c->table.size() / 16 + 64) c->dir_dirty = true;  // a bulk load: one full upload
}

void clear_dirty_slots(orl_ctx* c) {
    for (uint32_t i : c->dirty_slots) c->slot_marked[i] = 0;
    c->dirty_slots.clear();
}

// Upload only the host-changed slots of the partition and patch the probe forms in place (k_dir_patch), instead of
// re-uploading the whole table and rebuilding the probe tables on the host after every small registration batch.
// A changed slot that no longer fits the 16-B form (an N0 != 0 key, a ninth type) makes the probe table rebuild
// (upload_probe); one that does not fit the 8-B form retires that form.
int patch_dirty_slots(orl_ctx* c) {
    const size_t m = c->dirty_slots.size();
    bool p16 = c->probe_valid, p8 = c->probe8_valid;
    const bool dev_probe = c->probe_dev || c->probe_dev_stale;  // device-built probe table: rebuilt on the device
    bool rebuild16 = false;
    for (uint32_t i : c->dirty_slots) {
        const DirSlot& d = c->table[i];
        if (d.state != SLOT_FULL) continue;
        if (p16 || dev_probe) {
            uint32_t t = 0;
            while (t < c->hp.n_probe_types && c->hp.probe_tcd[t] != d.tcd) ++t;
            if (d.n0 != 0) {
                rebuild16 = p16;
            } else if (t == c->hp.n_probe_types) {
                if (t < kProbeTypes) {  // a new long-key type: append it to the list
                    c->hp.probe_tcd[t] = d.tcd;
                    c->hp.n_probe_types = t + 1;
                    c->params_dirty = true;
                } else {
                    rebuild16 = p16;
                }
            }
        }
        if (p8 && (c->hp.n_probe_types != 1 || !fits8(d))) p8 = false;
    }
    if (c->hp.n_probe_types != 1) p8 = false;
    c->probe8_valid = p8;
    if (rebuild16) p16 = false;
    const size_t bytes = m * (sizeof(DirSlot) + sizeof(ProbeSlot) + sizeof(uint2) + 4);
    if (bytes > c->patch_cap) {
        if (c->d_patch_data) (void)hipFree(c->d_patch_data);
        c->d_patch_data = nullptr;
        c->patch_cap = 0;
        ORL_HIP(c, hipMalloc(&c->d_patch_data, bytes));
        c->patch_cap = bytes;
    }
    std::vector<uint8_t> h(bytes);
    DirSlot* hs = reinterpret_cast<DirSlot*>(h.data());
    ProbeSlot* h16 = reinterpret_cast<ProbeSlot*>(h.data() + m * sizeof(DirSlot));
    uint2* h8 = reinterpret_cast<uint2*>(h.data() + m * (sizeof(DirSlot) + sizeof(ProbeSlot)));
    uint32_t* hi = reinterpret_cast<uint32_t*>(h.data() + m * (sizeof(DirSlot) + sizeof(ProbeSlot) + sizeof(uint2)));
    for (size_t k = 0; k < m; ++k) {
        const DirSlot& d = c->table[c->dirty_slots[k]];
        uint32_t t = 0;
        if (d.state == SLOT_FULL)
            while (t + 1 < c->hp.n_probe_types && c->hp.probe_tcd[t] != d.tcd) ++t;
        hs[k] = d;
        h16[k] = probe16_of(d, t);
        h8[k] = probe8_of(d);
        hi[k] = c->dirty_slots[k];
    }
    uint8_t* dd = static_cast<uint8_t*>(c->d_patch_data);
    ORL_HIP(c, hipMemcpy(dd, h.data(), bytes, hipMemcpyHostToDevice));
    int e = launch_dir_patch(reinterpret_cast<const uint32_t*>(dd + m * (sizeof(DirSlot) + sizeof(ProbeSlot) + sizeof(uint2))),
                             reinterpret_cast<const DirSlot*>(dd), reinterpret_cast<const ProbeSlot*>(dd + m * sizeof(DirSlot)),
                             reinterpret_cast<const uint2*>(dd + m * (sizeof(DirSlot) + sizeof(ProbeSlot))), (uint32_t)m,
                             c->d_table, p16 ? c->d_probe : nullptr, p8 ? c->d_probe8 : nullptr, c->stream);
    if (e) return hipfail(c, (hipError_t)e, "directory patch launch");
    ORL_HIP(c, hipStreamSynchronize(c->stream));
    const uint64_t st[3] = {c->count, c->tombs, 0};
    ORL_HIP(c, hipMemcpy(c->d_dirstate, st, sizeof st, hipMemcpyHostToDevice));
    c->count_ub = c->count;
    c->tombs_ub = c->tombs;
    clear_dirty_slots(c);
    ++c->n_patches;
    if (dev_probe) {  // the device rebuild (next route launch) reads the patched table with the updated type list
        c->probe_dev = false;
        c->probe_dev_stale = true;
    } else if (rebuild16) {
        if (int r = upload_probe(c)) return r;
    }
    return ORL_OK;
}

bool state_dirty(const orl_ctx* c) {
    return c->silo_hash_dirty || c->vr_dirty || c->silo_addr_dirty || c->gt_dirty || c->dir_dirty || c->params_dirty ||
           !c->dirty_slots.empty();
}

int sync_device_state(orl_ctx* c) {
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    if (!state_dirty(c)) return ORL_OK;
    // A batch launched earlier on any stream may still be reading the tables and params below: wait for the device
    // before overwriting them, so membership / registration changes take effect between batches.
    // Uploads happen only after host-side changes, never per batch.
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    ORL_HIP(c, hipDeviceSynchronize());
    if (c->silo_hash_dirty) {
        ORL_HIP(c, hipMemcpy(c->d_silo_hash, c->silo_hash, sizeof c->silo_hash, hipMemcpyHostToDevice));
        ORL_HIP(c, hipMemcpy(c->d_silo_known, c->silo_known, sizeof c->silo_known, hipMemcpyHostToDevice));
        c->silo_hash_dirty = false;
    }
    if (c->vr_dirty) {
        std::vector<uint32_t> h;
        std::vector<uint8_t> sl;
        for (const auto& e : c->vr_map) {  // SortedDictionary order: ascending bucket hash
            h.push_back(e.first);
            sl.push_back(e.second);
        }
        if (!h.empty()) {
            ORL_HIP(c, hipMemcpy(c->d_vr_hash, h.data(), h.size() * 4, hipMemcpyHostToDevice));
            ORL_HIP(c, hipMemcpy(c->d_vr_silo, sl.data(), sl.size(), hipMemcpyHostToDevice));
        }
        c->vr_n_dev = (uint32_t)h.size();
        c->vr_dirty = false;
    }
    if (c->silo_addr_dirty) {
        SiloAddrEntry tab[kSiloAddrSlots];
        for (auto& e : tab) { std::memset(&e, 0, sizeof e); e.silo = 0xFFu; }
        for (uint32_t s = 0; s < 255; ++s) {
            if (!c->silo_addr_known[s]) continue;
            uint32_t i = silo_addr_slot(c->silo_addr[s]);
            while (tab[i].silo != 0xFFu) i = (i + 1) & (kSiloAddrSlots - 1);
            std::memcpy(tab[i].w, c->silo_addr[s], sizeof tab[i].w);
            tab[i].silo = s;
        }
        ORL_HIP(c, hipMemcpy(c->d_silo_tab, tab, sizeof tab, hipMemcpyHostToDevice));
        ORL_HIP(c, hipMemcpy(c->d_silo_words, c->silo_addr, sizeof c->silo_addr, hipMemcpyHostToDevice));
        c->silo_addr_dirty = false;
    }
    if (c->gt_dirty) {
        std::vector<GrainTypeEntry> tab(kGrainTypeSlots, GrainTypeEntry{0, 0, 0, 0});
        std::vector<uint8_t> blob;
        for (const auto& kv : c->grain_types) {
            uint32_t i = fmix32((uint32_t)kv.first) & (kGrainTypeSlots - 1);
            while (tab[i].used) i = (i + 1) & (kGrainTypeSlots - 1);
            tab[i] = GrainTypeEntry{kv.first, (uint32_t)blob.size(), (uint32_t)kv.second.size(), 1};
            blob.insert(blob.end(), kv.second.begin(), kv.second.end());
        }
        ORL_HIP(c, hipMemcpy(c->d_gt, tab.data(), tab.size() * sizeof(GrainTypeEntry), hipMemcpyHostToDevice));
        if (!blob.empty()) ORL_HIP(c, hipMemcpy(c->d_gt_blob, blob.data(), blob.size(), hipMemcpyHostToDevice));
        c->gt_dirty = false;
    }
    if (c->dir_dirty) {
        if (c->count == 0 && c->tombs == 0)  // an empty partition: no 32 B/slot upload
            ORL_HIP(c, hipMemset(c->d_table, 0, c->table.size() * sizeof(DirSlot)));
        else
            ORL_HIP(c, hipMemcpy(c->d_table, c->table.data(), c->table.size() * sizeof(DirSlot), hipMemcpyHostToDevice));
        const uint64_t st[3] = {c->count, c->tombs, 0};
        ORL_HIP(c, hipMemcpy(c->d_dirstate, st, sizeof st, hipMemcpyHostToDevice));
        c->dir_dirty = false;
        ++c->n_full_uploads;
        if (!c->slot_marked.empty()) clear_dirty_slots(c);
        c->count_ub = c->count;
        c->tombs_ub = c->tombs;
        if (int r = upload_probe(c)) return r;
    } else if (!c->dirty_slots.empty()) {
        if (int r = patch_dirty_slots(c)) return r;
    }
    if (c->params_dirty) {  // last: upload_probe sets the probe type list
        ORL_HIP(c, hipMemcpy(c->d_params, &c->hp, sizeof(RouteParams), hipMemcpyHostToDevice));
        c->params_dirty = false;
    }
    return ORL_OK;
}

DirView dir_view(const orl_ctx* c) {
    return DirView{c->d_table, c->mask, c->d_cache, c->cache_slots ? c->cache_slots - 1 : 0,
                   (c->probe_valid || c->probe_dev) ? c->d_probe : nullptr, c->probe_dev ? c->d_probe_bad : nullptr,
                   c->probe8_valid ? c->d_probe8 : nullptr, c->d_cache != nullptr && c->hp.cache_on != 0};
}

// After a device mutation of the partition: the probe table no longer mirrors it.  When it held a type list,
// the next route launch rebuilds it on the device (prepare_probe); the route kernels check the build's flag.
void probe_after_device_mutation(orl_ctx* c) {
    if ((c->probe_valid || c->probe_dev) && c->hp.n_probe_types > 0) c->probe_dev_stale = true;
    c->probe_valid = c->probe_dev = c->probe8_valid = false;
}

int prepare_probe(orl_ctx* c, hipStream_t st) {
    if (!c->probe_dev_stale) return ORL_OK;
    int e = launch_probe_build(c->d_table, c->table.size(), c->d_params, c->d_probe, c->d_probe_bad, st);
    if (e) return hipfail(c, (hipError_t)e, "probe table build launch");
    c->probe_dev_stale = false;
    c->probe_dev = true;
    return ORL_OK;
}

void set_cache_on(orl_ctx* c, bool on) {
    if (c->hp.cache_on != (on ? 1u : 0u)) {
        c->hp.cache_on = on ? 1u : 0u;
        c->params_dirty = true;
    }
}

// Exact device-table counters after device mutations (synchronises the device; 24 bytes, no table download).
int refresh_counts(orl_ctx* c) {
    if (!c->mirror_stale) return ORL_OK;
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    ORL_HIP(c, hipDeviceSynchronize());
    uint64_t st[3];
    ORL_HIP(c, hipMemcpy(st, c->d_dirstate, sizeof st, hipMemcpyDeviceToHost));
    c->count_ub = st[0];
    c->tombs_ub = st[1];
    if (st[2]) return fail(c, ORL_E_CAPACITY, "a device registration found no free slot (directory overrun)");
    return ORL_OK;
}

// The host mirror after device mutations: download the table (synchronises the device) and recount.
int ensure_mirror(orl_ctx* c) {
    if (!c->mirror_stale) return ORL_OK;
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    ORL_HIP(c, hipDeviceSynchronize());
    ORL_HIP(c, hipMemcpy(c->table.data(), c->d_table, c->table.size() * sizeof(DirSlot), hipMemcpyDeviceToHost));
    uint64_t full = 0, tomb = 0;
    for (const DirSlot& d : c->table) {
        full += d.state == SLOT_FULL;
        tomb += d.state == SLOT_TOMB;
    }
    c->count = c->count_ub = full;
    c->tombs = c->tombs_ub = tomb;
    c->mirror_stale = false;
    return ORL_OK;
}

bool keys_equal(const DirSlot& s, const orl_grain_key& k) {
    return s.tcd == k.type_code_data && s.n0 == k.n0 && s.n1 == k.n1;
}

// Probe the mirror: returns slot index of the key, or -1; *free_slot = first reusable slot on the chain.
int64_t dir_find(const orl_ctx* c, const orl_grain_key& k, int64_t* free_slot) {
    const uint32_t h = jenkins3(k.type_code_data, k.n0, k.n1);
    uint64_t i = dir_slot(h, c->mask);
    int64_t fr = -1;
    for (uint64_t step = 0; step <= c->mask; ++step) {
        const DirSlot& s = c->table[i];
        if (s.state == SLOT_EMPTY) { if (fr < 0) fr = (int64_t)i; break; }
        if (s.state == SLOT_TOMB) { if (fr < 0) fr = (int64_t)i; }
        else if (keys_equal(s, k)) { if (free_slot) *free_slot = fr; return (int64_t)i; }
        i = (i + 1) & c->mask;
    }
    if (free_slot) *free_slot = fr;
    return -1;
}

int ensure_staging(orl_ctx* c, size_t in_bytes, size_t out_words) {
    if (in_bytes > c->st_in_cap) {
        if (c->st_in) (void)hipFree(c->st_in);
        c->st_in = nullptr; c->st_in_cap = 0;
        ORL_HIP(c, hipMalloc((void**)&c->st_in, in_bytes));
        c->st_in_cap = in_bytes;
    }
    if (out_words > c->st_out_cap) {
        if (c->st_out) (void)hipFree(c->st_out);
        c->st_out = nullptr; c->st_out_cap = 0;
        ORL_HIP(c, hipMalloc(&c->st_out, out_words * sizeof(uint32_t)));
        c->st_out_cap = out_words;
    }
    return ORL_OK;
}

void free_device(orl_ctx* c) {
    auto f = [](void* p) { if (p) (void)hipFree(p); };
    f(c->d_table); f(c->d_probe); f(c->d_probe8); f(c->d_probe_bad); f(c->d_params); f(c->d_rank_of_silo); f(c->d_claim); f(c->d_dirstate); f(c->d_dslot); f(c->d_vr_hash); f(c->d_vr_silo); f(c->d_silo_hash); f(c->d_silo_known); f(c->d_dflag); f(c->d_cache); f(c->d_cclaim); f(c->d_cstate); f(c->d_silo_tab); f(c->d_decode_flag); f(c->d_silo_words); f(c->d_gt); f(c->d_gt_blob); f(c->d_stamp_sizes); f(c->d_stamp_temp); f(c->d_patch_data); f(c->d_csr_off); f(c->d_csr_tgt); f(c->d_ext_table); f(c->d_ext_blob); f(c->d_ext_claim); f(c->d_ext_state);
    f(c->s.pairs_a); f(c->s.pairs_b); f(c->s.idx_a); f(c->s.sorted_keys); f(c->s.tile_hist); f(c->s.tile_cnt); f(c->s.scan_sums); f(c->s.digits); f(c->s.col_sums); f(c->s.col_tot); f(c->s.seg_hist); f(c->s.seg_carry); f(c->s.seg_meta); f(c->s.seg_lb); f(c->s.seg_lbctl); f(c->s.bstart); f(c->s.sstart); f(c->s.gap_q); f(c->s.hot); f(c->s.hot_rows); f(c->s.hot_bmax); f(c->s.pick_word); f(c->s.fan_blk); f(c->s.lsd_hot);
    for (auto& L : c->s.lb) {
        f(L.state);
        if (L.ev) (void)hipEventDestroy(L.ev);
        L = Scratch::LbSet{};
    }
    f(c->s.sw_ring); f(c->s.sw_ctl); f(c->s.sw_gtot); f(c->s.sw_gmax); f(c->s.s4_err);
    if (c->s.hot_host) (void)hipHostFree(c->s.hot_host);
    f(c->st_in); f(c->st_out); f(c->st_off);
    for (auto& e : c->tev) if (e) (void)hipEventDestroy(e);
    for (auto& e : c->hev) if (e) (void)hipEventDestroy(e);
    for (auto& st : c->hstream) if (st) (void)hipStreamDestroy(st);
    if (c->stream) (void)hipStreamDestroy(c->stream);
}

}  // namespace

// =====================================================================================================
extern "C" {

uint32_t orl_abi_version(void) { return ORL_ABI_VERSION; }

int orl_ctx_create(const orl_config* cfg, orl_ctx** out) {
    if (!cfg || !out) return ORL_E_INVALID;
    *out = nullptr;
    if (cfg->abi_version != ORL_ABI_VERSION) return ORL_E_INVALID;
    if (cfg->n_act == 0 || cfg->n_act >= 0x7FFFFFFFu) return ORL_E_INVALID;
    if (cfg->placement_policy > ORL_POLICY_HASH_SPREAD) return ORL_E_INVALID;
    if (cfg->max_batch >= (1ull << 31)) return ORL_E_INVALID;
    orl_ctx* c = new (std::nothrow) orl_ctx();
    if (!c) return ORL_E_NOMEM;
    c->cfg = *cfg;
    // Constants.SystemMembershipTableId = SystemGrain Guid 01145FEC-C21E-11E0-9105-D0FB4724019B (Constants.cs:66):
    // Guid.ToByteArray = EC 5F 14 01 | 1E C2 | E0 11 | 91 05 D0 FB 47 24 01 9B
    c->hp.mem_tcd = (uint64_t)ORL_CAT_SYSTEM_GRAIN << 56;
    c->hp.mem_n0 = 0x11E0C21E01145FECull;
    c->hp.mem_n1 = 0x9B012447FBD00591ull;
    const uint64_t slots = next_pow2(std::max<uint64_t>(cfg->dir_capacity, 1) * 2);
    try {
        c->table.assign(slots, DirSlot{});
    } catch (...) {
        delete c;
        return ORL_E_NOMEM;
    }
    c->mask = slots - 1;
    rebuild_params(c);
    if (cfg->device >= 0) {
        c->device_mode = true;
        auto bail = [&](hipError_t e, const char* what) {
            int r = hipfail(c, e, what);
            free_device(c);
            delete c;
            return r;
        };
        hipError_t e;
        if ((e = hipSetDevice(cfg->device)) != hipSuccess) return bail(e, "hipSetDevice");
        if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return bail(e, "hipStreamCreate");
        if ((e = (hipError_t)ensure_rank_mode(cfg->device)) != hipSuccess) return bail(e, "stage-4 rank self-check");
        if ((e = hipMalloc((void**)&c->d_table, slots * sizeof(DirSlot))) != hipSuccess) return bail(e, "hipMalloc(directory)");
        if ((e = hipMalloc((void**)&c->d_probe, slots * sizeof(ProbeSlot))) != hipSuccess) return bail(e, "hipMalloc(probe table)");
        if ((e = hipMalloc((void**)&c->d_probe_bad, 4)) != hipSuccess) return bail(e, "hipMalloc(probe flag)");
        if ((e = hipMalloc((void**)&c->d_probe8, slots * 8)) != hipSuccess) return bail(e, "hipMalloc(probe table 8)");
        const char* np = getenv("ORL_NO_PROBE16");
        c->probe_off = np && np[0] == '1';
        const char* np8 = getenv("ORL_NO_PROBE8");
        c->probe8_off = np8 && np8[0] == '1';
        if ((e = hipMalloc((void**)&c->d_claim, slots * 4)) != hipSuccess) return bail(e, "hipMalloc(claim)");
        if ((e = hipMemset(c->d_claim, 0xFF, slots * 4)) != hipSuccess) return bail(e, "hipMemset(claim)");
        if ((e = hipMalloc((void**)&c->d_vr_hash, ORL_MAX_SILOS * ORL_MAX_VBUCKETS_PER_SILO * 4)) != hipSuccess)
            return bail(e, "hipMalloc(vring)");
        if ((e = hipMalloc((void**)&c->d_vr_silo, ORL_MAX_SILOS * ORL_MAX_VBUCKETS_PER_SILO)) != hipSuccess)
            return bail(e, "hipMalloc(vring silos)");
        if ((e = hipMalloc((void**)&c->d_silo_hash, 1024)) != hipSuccess) return bail(e, "hipMalloc(silo hashes)");
        if ((e = hipMalloc((void**)&c->d_silo_known, 256)) != hipSuccess) return bail(e, "hipMalloc(silo known)");
        if ((e = hipMalloc((void**)&c->d_silo_tab, kSiloAddrSlots * sizeof(SiloAddrEntry))) != hipSuccess)
            return bail(e, "hipMalloc(silo addresses)");
        if ((e = hipMalloc((void**)&c->d_decode_flag, 4)) != hipSuccess) return bail(e, "hipMalloc(decode flag)");
        if ((e = hipMalloc((void**)&c->d_silo_words, 256 * 24)) != hipSuccess) return bail(e, "hipMalloc(silo words)");
        if ((e = hipMalloc((void**)&c->d_gt, kGrainTypeSlots * sizeof(GrainTypeEntry))) != hipSuccess)
            return bail(e, "hipMalloc(grain types)");
        if ((e = hipMalloc((void**)&c->d_gt_blob, kGrainTypeBlob)) != hipSuccess) return bail(e, "hipMalloc(grain type names)");
        if ((e = hipMalloc((void**)&c->d_dirstate, 32)) != hipSuccess) return bail(e, "hipMalloc(dirstate)");
        if ((e = hipMemset(c->d_dirstate, 0, 32)) != hipSuccess) return bail(e, "hipMemset(dirstate)");
        if ((e = hipMalloc((void**)&c->d_params, sizeof(RouteParams))) != hipSuccess) return bail(e, "hipMalloc(params)");
        if ((e = hipMalloc((void**)&c->d_rank_of_silo, 256)) != hipSuccess) return bail(e, "hipMalloc(rank map)");
        const uint64_t mb = std::max<uint64_t>(cfg->max_batch, kTile);
        const uint64_t tiles = (mb + kTile - 1) / kTile;
        c->s.max_batch = mb;
        c->s.max_tiles = tiles;
        c->s.device = cfg->device;
        c->s.gap_cap = env_gap_cap();
        c->s.fan_u = env_fan_u();
        // histogram rows: one per 4096-element radix tile, or one per route workgroup for small batches (route
        // tiles shrink towards 256 messages for a finer grid, never past kMaxRouteRows rows: route_items)
        const uint64_t rows = std::max<uint64_t>(tiles, std::min<uint64_t>(kMaxRouteRows, (mb + 255) / 256));
        const uint64_t hist_words = (1ull << kMaxDigitBits) * rows;
        if ((e = hipMalloc((void**)&c->s.pairs_a, mb * 8)) != hipSuccess) return bail(e, "hipMalloc(pairs_a)");
        if ((e = hipMalloc((void**)&c->s.pairs_b, mb * 8)) != hipSuccess) return bail(e, "hipMalloc(pairs_b)");
        if ((e = hipMalloc((void**)&c->s.idx_a, (mb + 1) * 4)) != hipSuccess) return bail(e, "hipMalloc(idx)");
        if ((e = hipMalloc((void**)&c->s.sorted_keys, mb * 4)) != hipSuccess) return bail(e, "hipMalloc(sorted)");
        if ((e = hipMalloc((void**)&c->s.tile_hist, hist_words * 4)) != hipSuccess) return bail(e, "hipMalloc(tile_hist)");
        if ((e = hipMalloc((void**)&c->s.tile_cnt, hist_words * 2)) != hipSuccess) return bail(e, "hipMalloc(tile_cnt)");
        // device-wide scans: tile histograms, fan-out degrees (mb + 1), bucket offsets (n_act + 2)
        const uint64_t scan_words = std::max<uint64_t>(std::max<uint64_t>(hist_words, mb + 1), (uint64_t)cfg->n_act + 2);
        if ((e = hipMalloc((void**)&c->s.scan_sums, ((scan_words + 4095) / 4096 + 2) * 4)) != hipSuccess) return bail(e, "hipMalloc(scan)");
        // two-level stage 4: per-segment low-digit rows (segment size drops to kSegChunk below 16M messages)
        const BucketPlan bp = make_bucket_plan(cfg->n_act);
        const uint64_t seg_rows = std::max<uint64_t>(max_segments(mb, bp.hb), max_segments(std::min<uint64_t>(mb, (16u << 20) - 1), bp.hb));
        const uint64_t seg_words = bp.two_level ? seg_rows << bp.lb : 1;
        if ((e = hipMalloc((void**)&c->s.seg_hist, seg_words * 4)) != hipSuccess) return bail(e, "hipMalloc(seg_hist)");
        // skewed plans: per chunk of >= kSegLbMinRows segments a carry-in row and a first bucket; the fused kernel's
        // look-back also keeps an aggregate and an inclusive row per chunk, and one flag (zeroed once: epoch-tagged)
        const uint64_t lb_cap = bp.two_level ? (seg_rows + kSegLbMinRows - 1) / kSegLbMinRows + 1 : 1;
        c->s.seg_lb_cap = (uint32_t)lb_cap;
        const uint64_t carry_words = bp.two_level ? lb_cap << bp.lb : 1;
        if ((e = hipMalloc((void**)&c->s.seg_carry, carry_words * 4)) != hipSuccess) return bail(e, "hipMalloc(seg_carry)");
        if ((e = hipMalloc((void**)&c->s.seg_meta, (lb_cap + 1) * 4)) != hipSuccess) return bail(e, "hipMalloc(seg_meta)");
        if ((e = hipMalloc((void**)&c->s.seg_lb, 2 * carry_words * 4)) != hipSuccess) return bail(e, "hipMalloc(seg_lb)");
        if ((e = hipMalloc((void**)&c->s.seg_lbctl, (4 + lb_cap) * 4)) != hipSuccess) return bail(e, "hipMalloc(seg_lbctl)");
        if ((e = hipMemset(c->s.seg_lbctl, 0, (4 + lb_cap) * 4)) != hipSuccess) return bail(e, "hipMemset(seg_lbctl)");
        if ((e = hipMalloc((void**)&c->s.bstart, 4097 * 4)) != hipSuccess) return bail(e, "hipMalloc(bstart)");
        c->s.fan_blk_cap = (uint32_t)((mb + 255) / 256 + 2);
        if ((e = hipMalloc((void**)&c->s.fan_blk, (size_t)c->s.fan_blk_cap * 4)) != hipSuccess) return bail(e, "hipMalloc(fan_blk)");
        if ((e = hipMalloc((void**)&c->s.sstart, 4098 * 4)) != hipSuccess) return bail(e, "hipMalloc(sstart)");
        if ((e = hipMalloc((void**)&c->d_dslot, mb * 4)) != hipSuccess) return bail(e, "hipMalloc(dslot)");
        if ((e = hipMalloc((void**)&c->d_dflag, mb)) != hipSuccess) return bail(e, "hipMalloc(dflag)");
        for (auto& L : c->s.lb) {
            if ((e = hipMalloc((void**)&L.state, 16 + ((mb + 2047) / 2048) * 64)) != hipSuccess) return bail(e, "hipMalloc(lb_state)");
            if ((e = hipMemset(L.state, 0, 16 + ((mb + 2047) / 2048) * 64)) != hipSuccess) return bail(e, "hipMemset(lb_state)");
            if ((e = hipEventCreateWithFlags(&L.ev, hipEventDisableTiming)) != hipSuccess) return bail(e, "hipEventCreate(lb)");
        }
        // (zeroed once: later launches tag their granules with an epoch and number tiles from a host-mirrored ticket)
        if (const char* lh = getenv("ORL_LSD_HOT"); lh && lh[0] == '1')  // the LSD plan's hot-key path: opt-in
            if ((e = hipMalloc((void**)&c->s.lsd_hot, 16)) != hipSuccess) return bail(e, "hipMalloc(lsd_hot)");
        if ((e = hipMalloc((void**)&c->s.s4_err, 4)) != hipSuccess) return bail(e, "hipMalloc(s4_err)");
        if ((e = hipMemset(c->s.s4_err, 0, 4)) != hipSuccess) return bail(e, "hipMemset(s4_err)");
        // the LSD plan's single-sweep passes (opt-in, ORL_LSD_SWEEP=1 at context creation: measured 8x slower than the
        // k_hist_pairs passes on MI355X): a look-back ring of >= `tiles` rows, zeroed once
        const char* sweep_env = getenv("ORL_LSD_SWEEP");
        if (!bp.two_level && sweep_env && sweep_env[0] == '1') {
            uint32_t row_bits = 0, rbits = 0;
            for (int p = 0; p < bp.lsd.passes; ++p) row_bits = std::max<uint32_t>(row_bits, (uint32_t)bp.lsd.bits[p]);
            while ((1ull << rbits) < tiles) ++rbits;
            const uint64_t ring_bytes = (8ull << rbits) << row_bits;
            if (ring_bytes <= (4ull << 30) && bp.lsd.passes <= 3) {  // else the k_hist_pairs passes (no ring)
                if ((e = hipMalloc((void**)&c->s.sw_ring, ring_bytes)) != hipSuccess) return bail(e, "hipMalloc(sweep ring)");
                if ((e = hipMemset(c->s.sw_ring, 0, ring_bytes)) != hipSuccess) return bail(e, "hipMemset(sweep ring)");
                if ((e = hipMalloc((void**)&c->s.sw_ctl, 16)) != hipSuccess) return bail(e, "hipMalloc(sweep ctl)");
                if ((e = hipMemset(c->s.sw_ctl, 0, 16)) != hipSuccess) return bail(e, "hipMemset(sweep ctl)");
                if ((e = hipMalloc((void**)&c->s.sw_gtot, (3ull << kMaxDigitBits) * 4)) != hipSuccess) return bail(e, "hipMalloc(sweep totals)");
                if ((e = hipMemset(c->s.sw_gtot, 0, (3ull << kMaxDigitBits) * 4)) != hipSuccess) return bail(e, "hipMemset(sweep totals)");
                if ((e = hipMalloc((void**)&c->s.sw_gmax, (1ull << kMaxDigitBits) * 4)) != hipSuccess) return bail(e, "hipMalloc(sweep max)");
                c->s.sw_rbits = rbits;
                c->s.sw_row_bits = row_bits;
            }
        }
        if ((e = hipMalloc((void**)&c->s.gap_q, kGapQueueWords * 4)) != hipSuccess) return bail(e, "hipMalloc(gap_q)");
        if ((e = hipMemset(c->s.gap_q, 0, kGapQueueWords * 4)) != hipSuccess) return bail(e, "hipMemset(gap_q)");
        if ((e = hipMalloc((void**)&c->s.digits, mb)) != hipSuccess) return bail(e, "hipMalloc(digits)");
        if ((e = hipMalloc((void**)&c->s.col_sums, ((rows + 63) / 64) * (1ull << kMaxDigitBits) * 4)) != hipSuccess)
            return bail(e, "hipMalloc(col_sums)");
        if ((e = hipMalloc((void**)&c->s.col_tot, ((1ull << kMaxDigitBits) + 1) * 4)) != hipSuccess) return bail(e, "hipMalloc(col_tot)");
        if ((e = hipMalloc((void**)&c->s.hot, 16)) != hipSuccess) return bail(e, "hipMalloc(hot)");
        {
            const uint32_t init[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u};  // no hot key in either slot
            if ((e = hipMemcpy(c->s.hot, init, 16, hipMemcpyHostToDevice)) != hipSuccess) return bail(e, "hipMemcpy(hot)");
        }
        // the hot column's rows, then its 64-row chunk sums
        if ((e = hipMalloc((void**)&c->s.hot_bmax, (((uint64_t)cfg->n_act + 2 + 4095) / 4096 + 1) * 8)) != hipSuccess)
            return bail(e, "hipMalloc(hot_bmax)");
        if ((e = hipMalloc((void**)&c->s.pick_word, 8)) != hipSuccess) return bail(e, "hipMalloc(pick_word)");
        if ((e = hipMemset(c->s.pick_word, 0, 8)) != hipSuccess) return bail(e, "hipMemset(pick_word)");
        if ((e = hipMalloc((void**)&c->s.hot_rows, (rows + (rows + 63) / 64 + 1) * 4)) != hipSuccess) return bail(e, "hipMalloc(hot_rows)");
        if ((e = hipHostMalloc((void**)&c->s.hot_host, 8, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
            return bail(e, "hipHostMalloc(hot_host)");
        c->s.hot_host[0] = 0xFFFFFFFFu;
        c->s.hot_host[1] = 1u;  // stage 4's skew hint: the first plan launches the chunked segment scan too
        if ((e = hipHostGetDevicePointer((void**)&c->s.hot_host_dev, c->s.hot_host, 0)) != hipSuccess)
            return bail(e, "hipHostGetDevicePointer(hot_host)");
        if ((e = hipMalloc((void**)&c->st_off, ((size_t)cfg->n_act + 2) * 4)) != hipSuccess) return bail(e, "hipMalloc(offsets)");
    }
    *out = c;
    return ORL_OK;
}

int orl_ctx_destroy(orl_ctx* c) {
    if (!c) return ORL_E_INVALID;
    if (c->device_mode) {
        (void)hipSetDevice(c->cfg.device);
        (void)hipStreamSynchronize(c->stream);
        free_device(c);
    }
    delete c;
    return ORL_OK;
}

const char* orl_last_error(const orl_ctx* c) { return c ? c->err.c_str() : "null context"; }

int orl_silos_set(orl_ctx* c, uint32_t n, const uint8_t* running, const uint8_t* functional, const uint8_t* local,
                  uint32_t seed) {
    if (!c) return ORL_E_INVALID;
    if (n == 0 || n > ORL_MAX_SILOS) return fail(c, ORL_E_INVALID, "n_silos must be in [1, %u]", ORL_MAX_SILOS);
    if (seed != ORL_NULL_SILO && seed >= n) return fail(c, ORL_E_INVALID, "seed %u out of range", seed);
    for (auto& e : c->ring)
        if (e.second >= n) return fail(c, ORL_E_STATE, "ring holds silo %u >= n_silos", e.second);
    c->n_silos = n;
    c->running.assign(n, 1); c->functional.assign(n, 1); c->local.assign(n, 1);
    for (uint32_t i = 0; i < n; ++i) {
        if (running) c->running[i] = running[i] ? 1 : 0;
        if (functional) c->functional[i] = functional[i] ? 1 : 0;
        if (local) c->local[i] = local[i] ? 1 : 0;
    }
    c->seed = seed;
    rebuild_params(c);
    return ORL_OK;
}

int orl_ring_add_server(orl_ctx* c, uint32_t silo, int32_t hash) {
    if (!c) return ORL_E_INVALID;
    if (!silo_ok(c, silo)) return fail(c, ORL_E_INVALID, "silo %u not in the silo table (call orl_silos_set first)", silo);
    for (auto& e : c->ring)
        if (e.second == silo) return ORL_OK;  // membershipCache.Contains → already cached (:247-251)
    if (c->ring.size() >= ORL_MAX_RING) return fail(c, ORL_E_CAPACITY, "ring full");
    // FindLastIndex(s => s.hash < hash) + 1: before existing equal hashes (:259-261)
    int idx = -1;
    for (int i = 0; i < (int)c->ring.size(); ++i)
        if (c->ring[i].first < hash) idx = i;
    c->ring.insert(c->ring.begin() + (idx + 1), std::make_pair(hash, (uint8_t)silo));
    c->silo_hash[silo] = hash;
    c->silo_known[silo] = 1;
    c->silo_hash_dirty = true;
    rebuild_params(c);
    return ORL_OK;
}

int orl_silo_hash_set(orl_ctx* c, uint32_t silo, int32_t hash) {
    if (!c) return ORL_E_INVALID;
    if (silo >= 256) return fail(c, ORL_E_INVALID, "silo %u out of range", silo);
    c->silo_hash[silo] = hash;
    c->silo_known[silo] = 1;
    c->silo_hash_dirty = true;
    return ORL_OK;
}

int orl_ring_remove_server(orl_ctx* c, uint32_t silo) {
    if (!c) return ORL_E_INVALID;
    auto it = std::find_if(c->ring.begin(), c->ring.end(), [&](const std::pair<int32_t, uint8_t>& e) { return e.second == silo; });
    if (it != c->ring.end()) c->ring.erase(it);
    rebuild_params(c);
    return ORL_OK;
}

int orl_ring_get(const orl_ctx* c, int32_t* hashes, uint8_t* silos, uint32_t cap, uint32_t* n_out) {
    if (!c || !n_out) return ORL_E_INVALID;
    *n_out = (uint32_t)c->ring.size();
    for (uint32_t i = 0; i < c->ring.size() && i < cap; ++i) {
        if (hashes) hashes[i] = c->ring[i].first;
        if (silos) silos[i] = c->ring[i].second;
    }
    return ORL_OK;
}

int orl_calc_id_hash(const char* utf8, size_t len, int32_t* out) {
    if (!out || (!utf8 && len)) return ORL_E_INVALID;
    std::vector<uint8_t> u16;
    if (!utf8_to_utf16le(utf8, len, u16)) return ORL_E_INVALID;
    *out = calc_id_hash_utf16(u16);
    return ORL_OK;
}

int orl_silo_consistent_hash(const char* endpoint, int32_t generation, int32_t* out) {
    if (!endpoint || !out) return ORL_E_INVALID;
    std::string s(endpoint);
    s += std::to_string(generation);  // Generation.ToString(CultureInfo.InvariantCulture)
    return orl_calc_id_hash(s.data(), s.size(), out);
}

uint32_t orl_jenkins_bytes(const uint8_t* data, size_t len) { return jenkins_bytes(data, len); }

uint32_t orl_keyext_uniform_hash(const orl_grain_key* k, const char* ext, size_t len) {
    // BinaryTokenStreamWriter.Write(UniqueKey): N0, N1, TypeCodeData (LE8), Write(string) = int32 len + UTF-8
    std::vector<uint8_t> b(28 + len);
    auto put64 = [&](size_t o, uint64_t v) { for (int i = 0; i < 8; ++i) b[o + i] = (uint8_t)(v >> (8 * i)); };
    put64(0, k->n0);
    put64(8, k->n1);
    put64(16, k->type_code_data);
    const uint32_t l = (uint32_t)len;
    for (int i = 0; i < 4; ++i) b[24 + i] = (uint8_t)(l >> (8 * i));
    if (len) std::memcpy(b.data() + 28, ext, len);
    return jenkins_bytes(b.data(), b.size());
}

}  // extern "C"
namespace {
// ---- KeyExt grains (round 5): the host table, first writer wins, tombstones, rebuilt (and the blob compacted) when full
uint32_t keyext_hash(const orl_grain_key& k, const uint8_t* ext, uint32_t len) {
    return orl_keyext_uniform_hash(&k, reinterpret_cast<const char*>(ext), len);
}

bool ext_equal(const orl_ctx* c, const ExtSlot& e, const orl_grain_key& k, uint32_t h, const uint8_t* ext, uint32_t len) {
    return e.state == SLOT_FULL && e.hash == h && e.tcd == k.type_code_data && e.n0 == k.n0 && e.n1 == k.n1 && e.len == len &&
           (len == 0 || std::memcmp(c->ext_blob.data() + e.off, ext, len) == 0);
}

// Slot of the key (or -1); *free_slot = the first tombstone / empty slot of its chain.
int64_t ext_find(const orl_ctx* c, const orl_grain_key& k, uint32_t h, const uint8_t* ext, uint32_t len, int64_t* free_slot) {
    if (free_slot) *free_slot = -1;
    if (c->ext_table.empty()) return -1;
    const uint64_t mask = c->ext_table.size() - 1;
    uint64_t i = dir_slot(h, mask);
    for (uint64_t step = 0; step <= mask; ++step, i = (i + 1) & mask) {
        const ExtSlot& e = c->ext_table[i];
        if (e.state == SLOT_EMPTY) {
            if (free_slot && *free_slot < 0) *free_slot = (int64_t)i;
            return -1;
        }
        if (e.state == SLOT_TOMB) {
            if (free_slot && *free_slot < 0) *free_slot = (int64_t)i;
            continue;
        }
        if (ext_equal(c, e, k, h, ext, len)) return (int64_t)i;
    }
    return -1;
}

// Rebuild with room for `need` entries at load <= 1/2, without tombstones, the blob compacted.
void ext_rebuild(orl_ctx* c, uint64_t need) {
    uint64_t size = 1024;
    while (size < 2 * need) size <<= 1;
    std::vector<ExtSlot> old;
    old.swap(c->ext_table);
    std::vector<uint8_t> oblob;
    oblob.swap(c->ext_blob);
    c->ext_table.assign(size, ExtSlot{});
    for (auto& e : c->ext_table) e.state = SLOT_EMPTY;
    for (const ExtSlot& e : old) {
        if (e.state != SLOT_FULL) continue;
        ExtSlot n = e;
        n.off = (uint32_t)c->ext_blob.size();
        c->ext_blob.insert(c->ext_blob.end(), oblob.begin() + e.off, oblob.begin() + e.off + e.len);
        uint64_t i = dir_slot(e.hash, size - 1);
        while (c->ext_table[i].state != SLOT_EMPTY) i = (i + 1) & (size - 1);
        c->ext_table[i] = n;
    }
    c->ext_tombs = 0;
    c->ext_dirty = true;
}

// The ring owner of a KeyExt hash (CalculateTargetSilo :466-494), as host_owner computes it for the u64 path.
uint32_t host_owner_hash(const orl_ctx* c, int32_t h, uint32_t me, bool excl) {
    const bool running = me < c->n_silos && c->running[me];
    const int n = (int)c->ring.size();
    if (n == 0) return (excl && !running) ? ORL_NULL_SILO : me;
    const bool ex = excl && !running;
    int found = -1;
    for (int i = 0; i < n; ++i)
        if (c->ring[i].first <= h && !(c->ring[i].second == me && ex)) found = i;
    if (found < 0) {
        found = n - 1;
        if (c->ring[found].second == me && ex) {
            if (n > 1) found = n - 2; else return ORL_NULL_SILO;
        }
    }
    return c->ring[found].second;
}

// Every reference of a host KeyExt call inside the caller's blob (the entry points used to read past it).
int check_ext_refs(orl_ctx* c, const orl_ext_ref* ext, size_t n, uint64_t blob_bytes) {
    for (size_t i = 0; i < n; ++i)
        if ((uint64_t)ext[i].off + ext[i].len > blob_bytes)
            return fail(c, ORL_E_INVALID, "KeyExt reference %zu (%u + %u bytes) outside the %llu-byte blob", i, ext[i].off,
                        ext[i].len, (unsigned long long)blob_bytes);
    return ORL_OK;
}

// The host mirror after device registrations: the table, the used string store and the exact counters (synchronises).
int ext_sync_host(orl_ctx* c) {
    if (!c->ext_dev_newer) return ORL_OK;
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    ORL_HIP(c, hipDeviceSynchronize());
    uint64_t st[4];
    ORL_HIP(c, hipMemcpy(st, c->d_ext_state, sizeof st, hipMemcpyDeviceToHost));
    c->ext_blob.resize(st[0]);
    if (st[0]) ORL_HIP(c, hipMemcpy(c->ext_blob.data(), c->d_ext_blob, st[0], hipMemcpyDeviceToHost));
    if (!c->ext_table.empty())
        ORL_HIP(c, hipMemcpy(c->ext_table.data(), c->d_ext_table, c->ext_table.size() * sizeof(ExtSlot), hipMemcpyDeviceToHost));
    c->ext_count = c->ext_count_ub = st[1];
    c->ext_tombs = c->ext_tombs_ub = st[2];
    c->ext_blob_ub = st[0];
    c->ext_dev_newer = false;
    if (st[3]) {
        ORL_HIP(c, hipMemset(c->d_ext_state + 3, 0, 8));
        return fail(c, ORL_E_CAPACITY, "a device KeyExt registration found no free slot or no string-store room (%llu)",
                    (unsigned long long)st[3]);
    }
    return ORL_OK;
}

int upload_keyext(orl_ctx* c) {
    if (!c->ext_dirty) return ORL_OK;
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    ORL_HIP(c, hipDeviceSynchronize());  // batches in flight may read the old table (snapshot semantics, as the partition)
    const size_t tb = c->ext_table.size() * sizeof(ExtSlot);
    const size_t bb = std::max<size_t>(std::max<size_t>(c->ext_blob.size(), 4), c->ext_blob_min_cap);
    if (tb > c->d_ext_table_cap) {
        (void)hipFree(c->d_ext_table);
        c->d_ext_table = nullptr;
        ORL_HIP(c, hipMalloc((void**)&c->d_ext_table, tb));
        c->d_ext_table_cap = tb;
    }
    if (bb > c->d_ext_blob_cap) {
        (void)hipFree(c->d_ext_blob);
        c->d_ext_blob = nullptr;
        ORL_HIP(c, hipMalloc((void**)&c->d_ext_blob, bb + bb / 2));
        c->d_ext_blob_cap = bb + bb / 2;
    }
    if (tb) ORL_HIP(c, hipMemcpy(c->d_ext_table, c->ext_table.data(), tb, hipMemcpyHostToDevice));
    if (!c->ext_blob.empty()) ORL_HIP(c, hipMemcpy(c->d_ext_blob, c->ext_blob.data(), c->ext_blob.size(), hipMemcpyHostToDevice));
    // the device registration's state: claim words at rest, the string cursor 4-B aligned, the counters
    const size_t slots = c->ext_table.size();
    if (slots > c->d_ext_claim_cap) {
        (void)hipFree(c->d_ext_claim);
        c->d_ext_claim = nullptr;
        ORL_HIP(c, hipMalloc((void**)&c->d_ext_claim, slots * 4));
        c->d_ext_claim_cap = slots;
    }
    if (slots) ORL_HIP(c, hipMemset(c->d_ext_claim, 0xFF, slots * 4));
    if (!c->d_ext_state) ORL_HIP(c, hipMalloc((void**)&c->d_ext_state, 4 * sizeof(uint64_t)));
    const uint64_t st[4] = {(c->ext_blob.size() + 3) & ~uint64_t(3), c->ext_count, c->ext_tombs, 0};
    ORL_HIP(c, hipMemcpy(c->d_ext_state, st, sizeof st, hipMemcpyHostToDevice));
    c->ext_count_ub = c->ext_count;
    c->ext_tombs_ub = c->ext_tombs;
    c->ext_blob_ub = st[0];
    c->ext_dirty = false;
    return ORL_OK;
}
}  // namespace
extern "C" {

int orl_dir_insert_keyext(orl_ctx* c, const orl_grain_key* keys, const orl_ext_ref* ext, const uint8_t* blob,
                          uint64_t blob_bytes, const uint32_t* acts, const uint8_t* silos, size_t n, uint32_t* wact,
                          uint8_t* wsilo, uint8_t* status) {
    if (!c || (n && (!keys || !ext || !blob || !acts || !silos))) return ORL_E_INVALID;
    if (int r = check_ext_refs(c, ext, n, blob_bytes)) return r;
    if (int r = ext_sync_host(c)) return r;
    for (size_t i = 0; i < n; ++i) {
        uint8_t st;
        uint32_t a = ORL_NO_ACT;
        uint8_t s = ORL_NULL_SILO;
        const orl_grain_key& k = keys[i];
        if (acts[i] >= c->cfg.n_act) return fail(c, ORL_E_INVALID, "act %u >= n_act %u at %zu", acts[i], c->cfg.n_act, i);
        if (!silo_ok(c, silos[i])) return fail(c, ORL_E_INVALID, "silo %u out of range at %zu", silos[i], i);
        if ((uint32_t)(k.type_code_data >> 56) != ORL_CAT_KEYEXT_GRAIN) {
            st = ORL_INS_UNSUPPORTED;
        } else {
            const uint8_t* x = blob + ext[i].off;
            const uint32_t len = ext[i].len;
            const uint32_t h = keyext_hash(k, x, len);
            const uint32_t owner = host_owner_hash(c, (int32_t)h, silos[i], true);
            if (owner == ORL_NULL_SILO) st = ORL_INS_OWNER_NULL;
            else if (!c->local[owner]) st = ORL_INS_REMOTE_OWNER;
            else if (!c->functional[silos[i]]) st = ORL_INS_INVALID_SILO;  // AddSingleActivation :277-279
            else {
                if ((c->ext_count + c->ext_tombs + 1) * 2 > c->ext_table.size()) ext_rebuild(c, c->ext_count + 1);
                int64_t fr = -1;
                const int64_t at = ext_find(c, k, h, x, len, &fr);
                if (at >= 0) {  // GrainInfo.AddSingleActivation: an instance exists → return it (:103-107)
                    st = ORL_INS_EXISTING;
                    a = c->ext_table[at].act;
                    s = c->ext_table[at].silo;
                } else {
                    if (c->ext_blob.size() + len > UINT32_MAX)  // ExtSlot.off is 32-bit: the store never wraps
                        return fail(c, ORL_E_CAPACITY, "KeyExt extension store full (4 GiB) at %zu", i);
                    ExtSlot& e = c->ext_table[fr];
                    if (e.state == SLOT_TOMB) --c->ext_tombs;
                    e.tcd = k.type_code_data; e.n0 = k.n0; e.n1 = k.n1;
                    e.hash = h; e.act = acts[i]; e.silo = silos[i]; e.state = SLOT_FULL;
                    e.off = (uint32_t)c->ext_blob.size();
                    e.len = len;
                    c->ext_blob.insert(c->ext_blob.end(), x, x + len);
                    ++c->ext_count;
                    c->ext_dirty = true;
                    st = ORL_INS_INSERTED;
                    a = acts[i];
                    s = silos[i];
                }
            }
        }
        if (status) status[i] = st;
        if (wact) wact[i] = a;
        if (wsilo) wsilo[i] = s;
    }
    return ORL_OK;
}

int orl_dir_remove_keyext(orl_ctx* c, const orl_grain_key* keys, const orl_ext_ref* ext, const uint8_t* blob,
                          uint64_t blob_bytes, size_t n, uint8_t* removed) {
    if (!c || (n && (!keys || !ext || !blob))) return ORL_E_INVALID;
    if (int r = check_ext_refs(c, ext, n, blob_bytes)) return r;
    if (int r = ext_sync_host(c)) return r;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t* x = blob + ext[i].off;
        const int64_t at = ext_find(c, keys[i], keyext_hash(keys[i], x, ext[i].len), x, ext[i].len, nullptr);
        if (at >= 0) {
            c->ext_table[at].state = SLOT_TOMB;
            --c->ext_count;
            ++c->ext_tombs;
            c->ext_dirty = true;
        }
        if (removed) removed[i] = at >= 0 ? 1 : 0;
    }
    return ORL_OK;
}

int orl_dir_lookup_keyext_host(orl_ctx* c, const orl_grain_key* keys, const orl_ext_ref* ext, const uint8_t* blob,
                               uint64_t blob_bytes, size_t n, uint32_t* act, uint8_t* silo) {
    if (!c || (n && (!keys || !ext || !blob))) return ORL_E_INVALID;
    if (int r = check_ext_refs(c, ext, n, blob_bytes)) return r;
    if (int r = ext_sync_host(c)) return r;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t* x = blob + ext[i].off;
        const int64_t at = ext_find(c, keys[i], keyext_hash(keys[i], x, ext[i].len), x, ext[i].len, nullptr);
        if (act) act[i] = at >= 0 ? c->ext_table[at].act : ORL_NO_ACT;
        if (silo) silo[i] = at >= 0 ? c->ext_table[at].silo : (uint8_t)ORL_NULL_SILO;
    }
    return ORL_OK;
}

int orl_dir_keyext_count(const orl_ctx* c, uint64_t* n) {
    if (!c || !n) return ORL_E_INVALID;
    if (int r = ext_sync_host(const_cast<orl_ctx*>(c))) return r;  // after device registrations: the exact count
    *n = c->ext_count;
    return ORL_OK;
}

int orl_dir_insert_keyext_device(orl_ctx* c, const orl_grain_key* d_keys, const orl_ext_ref* d_ext, const uint8_t* d_blob,
                                 uint64_t blob_bytes, const uint32_t* d_acts, const uint8_t* d_silos, size_t n,
                                 uint32_t* d_wact, uint8_t* d_wsilo, uint8_t* d_status, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "no device");
    if (n && (!d_keys || !d_ext || !d_blob || !d_acts || !d_silos || !d_status)) return fail(c, ORL_E_INVALID, "null device buffer");
    if (n > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "batch %zu > max_batch %llu", n, (unsigned long long)c->s.max_batch);
    if (c->n_silos == 0) return fail(c, ORL_E_STATE, "silo table not set");
    if (blob_bytes > UINT32_MAX) return fail(c, ORL_E_INVALID, "KeyExt blob of %llu bytes (<= 4 GiB)", (unsigned long long)blob_bytes);
    if (n == 0) return ORL_OK;
    int r = sync_device_state(c);
    if (r) return r;
    if ((r = upload_keyext(c))) return r;  // host changes first: the device table is the authority from here
    // every message might insert (load <= 1/2) and append its string (4-B aligned)
    const uint64_t add = blob_bytes + 3 * (uint64_t)n;
    auto fits = [&]() {
        return (c->ext_count_ub + c->ext_tombs_ub + n) * 2 <= c->ext_table.size() && c->ext_blob_ub + add <= c->d_ext_blob_cap &&
               c->ext_blob_ub + add <= UINT32_MAX;
    };
    if (!fits()) {
        if ((r = ext_sync_host(c))) return r;
        if (c->ext_blob.size() + add > UINT32_MAX)
            return fail(c, ORL_E_CAPACITY, "KeyExt extension store full (4 GiB)");
        if ((c->ext_count + c->ext_tombs + n) * 2 > c->ext_table.size()) ext_rebuild(c, c->ext_count + n);
        c->ext_blob_min_cap = std::max<uint64_t>(c->ext_blob_min_cap, c->ext_blob.size() + add + 64);
        c->ext_dirty = true;
        if (c->ext_blob_min_cap > c->d_ext_blob_cap) {  // a new store is allocated at the upload
            (void)hipFree(c->d_ext_blob);
            c->d_ext_blob = nullptr;
            c->d_ext_blob_cap = 0;
        }
        if ((r = upload_keyext(c))) return r;
        if (!fits()) return fail(c, ORL_E_CAPACITY, "KeyExt table: no room for a batch of %zu", n);
    }
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    int e = launch_keyext_insert(c->d_params, c->d_ext_table, c->ext_table.size() - 1, c->d_ext_claim, c->d_ext_blob,
                                 c->d_ext_blob_cap, d_keys, d_ext, d_blob, blob_bytes, d_acts, d_silos, n, c->cfg.n_act,
                                 c->n_silos, c->d_dslot, d_wact, d_wsilo, d_status, c->d_ext_state, st);
    if (e) return hipfail(c, (hipError_t)e, "KeyExt insert launch");
    c->ext_count_ub += n;
    c->ext_blob_ub += add;
    c->ext_dev_newer = true;
    return ORL_OK;
}

int orl_dir_insert_single(orl_ctx* c, const orl_grain_key* keys, const uint32_t* acts, const uint8_t* silos, size_t n,
                          uint32_t* wact, uint8_t* wsilo, uint8_t* status) {
    if (!c || (n && (!keys || !acts || !silos))) return ORL_E_INVALID;
    if (int r = ensure_mirror(c)) return r;
    for (size_t i = 0; i < n; ++i) {
        uint8_t st;
        uint32_t a = ORL_NO_ACT;
        uint8_t s = ORL_NULL_SILO;
        const orl_grain_key& k = keys[i];
        const uint32_t cat = (uint32_t)(k.type_code_data >> 56);
        if (acts[i] >= c->cfg.n_act) return fail(c, ORL_E_INVALID, "act %u >= n_act %u at %zu", acts[i], c->cfg.n_act, i);
        if (!silo_ok(c, silos[i])) return fail(c, ORL_E_INVALID, "silo %u out of range at %zu", silos[i], i);
        if (cat == ORL_CAT_KEYEXT_GRAIN || cat == ORL_CAT_SYSTEM_TARGET) {
            st = ORL_INS_UNSUPPORTED;
        } else {
            const uint32_t owner = host_owner(c, k, silos[i], true);
            if (owner == ORL_NULL_SILO) st = ORL_INS_OWNER_NULL;
            else if (!c->local[owner]) st = ORL_INS_REMOTE_OWNER;
            else if (!c->functional[silos[i]]) st = ORL_INS_INVALID_SILO;  // AddSingleActivation :277-279
            else {
                int64_t fr = -1;
                const int64_t at = dir_find(c, k, &fr);
                if (at >= 0) {  // GrainInfo.AddSingleActivation: an instance exists → return it (:103-107)
                    st = ORL_INS_EXISTING;
                    a = c->table[at].act;
                    s = c->table[at].silo;
                } else {
                    if (fr < 0 || (c->count + c->tombs + 1) * 2 > c->table.size())
                        return fail(c, ORL_E_CAPACITY, "directory full (%llu entries)", (unsigned long long)c->count);
                    DirSlot& d = c->table[fr];
                    if (d.state == SLOT_TOMB) --c->tombs;
                    d.tcd = k.type_code_data; d.n0 = k.n0; d.n1 = k.n1;
                    d.act = acts[i]; d.silo = silos[i]; d.state = SLOT_FULL; d.pad = 0;
                    ++c->count;
                    mark_slot(c, (uint64_t)fr);
                    st = ORL_INS_INSERTED;
                    a = acts[i];
                    s = silos[i];
                }
            }
        }
        if (status) status[i] = st;
        if (wact) wact[i] = a;
        if (wsilo) wsilo[i] = s;
    }
    return ORL_OK;
}

int orl_dir_remove(orl_ctx* c, const orl_grain_key* keys, size_t n, uint8_t* removed) {
    if (!c || (n && !keys)) return ORL_E_INVALID;
    if (int r = ensure_mirror(c)) return r;
    for (size_t i = 0; i < n; ++i) {
        const int64_t at = dir_find(c, keys[i], nullptr);
        if (at >= 0) {
            c->table[at].state = SLOT_TOMB;
            --c->count;
            ++c->tombs;
            mark_slot(c, (uint64_t)at);
        }
        if (removed) removed[i] = at >= 0 ? 1 : 0;
    }
    return ORL_OK;
}

int orl_dir_count(const orl_ctx* c, uint64_t* n) {
    if (!c || !n) return ORL_E_INVALID;
    if (c->mirror_stale) {  // device mutations since the mirror was read: the device counters are exact
        if (int r = refresh_counts(const_cast<orl_ctx*>(c))) return r;
        *n = c->count_ub;
        return ORL_OK;
    }
    *n = c->count;
    return ORL_OK;
}

int orl_dir_lookup_host(const orl_ctx* c, const orl_grain_key* keys, size_t n, uint32_t* act, uint8_t* silo) {
    if (!c || (n && !keys)) return ORL_E_INVALID;
    if (int r = ensure_mirror(const_cast<orl_ctx*>(c))) return r;
    for (size_t i = 0; i < n; ++i) {
        const int64_t at = dir_find(c, keys[i], nullptr);
        if (act) act[i] = at >= 0 ? c->table[at].act : ORL_NO_ACT;
        if (silo) silo[i] = at >= 0 ? c->table[at].silo : (uint8_t)ORL_NULL_SILO;
    }
    return ORL_OK;
}

int orl_hash_batch(orl_ctx* c, const orl_grain_key* keys, size_t n, uint32_t* out) {
    if (!c || (n && (!keys || !out))) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    if (n == 0) return ORL_OK;
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    int r = ensure_staging(c, n * sizeof(orl_grain_key), n);
    if (r) return r;
    ORL_HIP(c, hipMemcpyAsync(c->st_in, keys, n * sizeof(orl_grain_key), hipMemcpyHostToDevice, c->stream));
    int e = launch_hash((const orl_grain_key*)c->st_in, n, c->st_out, c->stream);
    if (e) return hipfail(c, (hipError_t)e, "k_hash");
    ORL_HIP(c, hipMemcpyAsync(out, c->st_out, n * 4, hipMemcpyDeviceToHost, c->stream));
    ORL_HIP(c, hipStreamSynchronize(c->stream));
    return ORL_OK;
}

namespace {
int route_impl(orl_ctx* c, const void* d_in, int fmt, size_t n, uint32_t opts, uint32_t* d_route, uint32_t* d_act,
               uint32_t* d_order, uint32_t* d_off, void* stream, const uint32_t* d_in_act = nullptr) {
    if (!c) return ORL_E_INVALID;
    if (fmt != 8 && fmt != 16 && fmt != 32) return fail(c, ORL_E_INVALID, "record width %d (8, 16 or 32)", fmt);
    if (n && (!d_in || !d_route || !d_act)) return fail(c, ORL_E_INVALID, "null device buffer");
    const bool buckets = !(opts & ORL_OPT_NO_BUCKETS);
    if (buckets && (!d_off || (n && !d_order))) return fail(c, ORL_E_INVALID, "null order/offsets buffer");
    if (n > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "batch %zu > max_batch %llu", n, (unsigned long long)c->s.max_batch);
    if (c->n_silos == 0) return fail(c, ORL_E_STATE, "silo table not set");
    int r = sync_device_state(c);
    if (r) return r;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    hipEvent_t* ev = nullptr;
    if (c->timing && n > 0 && c->tcount < ORL_TIMING_SLOTS) ev = &c->tev[4 * (size_t)c->tcount++];
    if ((r = prepare_probe(c, st))) return r;
    if (ev) ORL_HIP(c, hipEventRecord(ev[0], st));
    if (fmt == 8 && c->hp.n_wire_types == 0) return fail(c, ORL_E_STATE, "8-byte records need the wire types (orl_wire_types_set)");
    int e = launch_route_bucket(c->d_params, dir_view(c), d_in, fmt, n, opts, c->cfg.n_act, d_route, d_act, d_order,
                                d_off, c->s, st, ev ? ev[1] : nullptr, ev ? ev[2] : nullptr, d_in_act);
    if (!e && ctx_cache_on(c)) e = launch_cache_gen_advance(c->d_cache, c->cache_slots - 1, n, st);  // the lookups' LRU stamps
    if (e) return hipfail(c, (hipError_t)e, "route launch");
    if (ev) ORL_HIP(c, hipEventRecord(ev[3], st));
    return ORL_OK;
}
}  // namespace

}  // extern "C"
namespace orl {
int ctx_route_received(orl_ctx* c, const void* d_in, int fmt, size_t n, uint32_t opts, uint32_t* d_route, uint32_t* d_act,
                       const uint32_t* d_in_act, void* stream) {
    return route_impl(c, d_in, fmt, n, opts | ORL_OPT_NO_BUCKETS, d_route, d_act, nullptr, nullptr, stream, d_in_act);
}

bool ctx_cache_on(orl_ctx* c) { return c && c->d_cache && c->hp.cache_on; }

int ctx_keyext_prepare(orl_ctx* c) { return upload_keyext(c); }

int ctx_route_keyext_received(orl_ctx* c, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const orl_ext_ref* d_ext,
                              const uint8_t* d_blob, uint64_t blob_bytes, uint32_t* d_route, uint32_t* d_act, void* stream) {
    if (n == 0) return ORL_OK;
    const uint32_t excl = (opts & ORL_OPT_EXCLUDE_IF_STOPPING) ? 1u : 0u;
    int e = launch_keyext_route(c->d_params, d_in, n, d_ext, d_blob, blob_bytes, c->d_ext_table,
                                c->ext_table.empty() ? 0 : c->ext_table.size() - 1, c->d_ext_blob, excl, d_route, d_act,
                                stream ? stream : c->stream);
    if (e) return hipfail(c, (hipError_t)e, "KeyExt route launch (node)");
    return ORL_OK;
}
const uint32_t* ctx_stage4_err(const orl_ctx* c) { return c->s.s4_err; }
}  // namespace orl
extern "C" {

int orl_route_batch_device(orl_ctx* c, const orl_msg_hdr* d_in, size_t n, uint32_t opts, uint32_t* d_route, uint32_t* d_act,
                           uint32_t* d_order, uint32_t* d_off, void* stream) {
    return route_impl(c, d_in, 32, n, opts, d_route, d_act, d_order, d_off, stream);
}

int orl_route_compact_device(orl_ctx* c, const orl_wire_msg* d_in, size_t n, uint32_t opts, uint32_t* d_route, uint32_t* d_act,
                             uint32_t* d_order, uint32_t* d_off, void* stream) {
    return route_impl(c, d_in, 16, n, opts, d_route, d_act, d_order, d_off, stream);
}

int orl_route_narrow_device(orl_ctx* c, const orl_wire8* d_in, size_t n, uint32_t opts, uint32_t* d_route, uint32_t* d_act,
                            uint32_t* d_order, uint32_t* d_off, void* stream) {
    return route_impl(c, d_in, 8, n, opts, d_route, d_act, d_order, d_off, stream);
}

// Stages 1-3 (k_route leaves KeyExt messages ORL_ST_KEYEXT_UNRESOLVED with their owner), the KeyExt lookups
// (k_keyext_route), then stage 4 over the final handles (orl_bucket_device's path: its own histogram pass).
int orl_route_keyext_device(orl_ctx* c, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const orl_ext_ref* d_ext,
                            const uint8_t* d_blob, uint64_t blob_bytes, uint32_t* d_route, uint32_t* d_act, uint32_t* d_order,
                            uint32_t* d_off, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (n && (!d_ext || !d_blob)) return fail(c, ORL_E_INVALID, "null KeyExt references or blob");
    const bool buckets = !(opts & ORL_OPT_NO_BUCKETS);
    if (buckets && (!d_off || (n && !d_order))) return fail(c, ORL_E_INVALID, "null order/offsets buffer");
    if (int r = upload_keyext(c)) return r;
    if (int r = route_impl(c, d_in, 32, n, opts | ORL_OPT_NO_BUCKETS, d_route, d_act, nullptr, nullptr, stream)) return r;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    if (n) {
        const uint32_t excl = (opts & ORL_OPT_EXCLUDE_IF_STOPPING) ? 1u : 0u;
        int e = launch_keyext_route(c->d_params, d_in, n, d_ext, d_blob, blob_bytes, c->d_ext_table,
                                    c->ext_table.empty() ? 0 : c->ext_table.size() - 1, c->d_ext_blob, excl, d_route, d_act, st);
        if (e) return hipfail(c, (hipError_t)e, "KeyExt route launch");
    }
    if (!buckets) return ORL_OK;
    int e = launch_bucket_acts(d_act, n, c->cfg.n_act, d_order, d_off, c->s, st);
    if (e) return hipfail(c, (hipError_t)e, "bucket launch");
    return ORL_OK;
}

// Host-array form (the P/Invoke call): the batch is cut into chunks; chunk k's upload (copy stream), its stages 1-3
// (the context's stream) and the download of its route words / handles (second copy stream) overlap with the
// neighbouring chunks', and stage 4 runs once over the whole batch at the end.  Caller arrays registered with
// orl_host_register (pinned) are copied asynchronously at full PCIe rate; pageable ones go through the runtime's
// staging (correct, slower).  fmt = the input record width (32 = orl_msg_hdr, 8 = orl_wire8).
namespace {
int route_batch_host(orl_ctx* c, const void* in, int fmt, size_t n, uint32_t opts, uint32_t* route, uint32_t* act,
                     uint32_t* order, uint32_t* offsets) {
    if (!c) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    const bool buckets = !(opts & ORL_OPT_NO_BUCKETS);
    if (n && (!in || !route || !act)) return fail(c, ORL_E_INVALID, "null host buffer");
    if (buckets && (!offsets || (n && !order))) return fail(c, ORL_E_INVALID, "null order/offsets buffer");
    if (n > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "batch %zu > max_batch %llu", n, (unsigned long long)c->s.max_batch);
    if (fmt == 8 && c->hp.n_wire_types == 0) return fail(c, ORL_E_STATE, "8-byte records need the wire types (orl_wire_types_set)");
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    int r = ensure_staging(c, std::max<size_t>(n, 1) * sizeof(orl_msg_hdr), std::max<size_t>(n, 1) * 3);
    if (r) return r;
    if (!c->hstream[0]) {
        for (auto& st : c->hstream) ORL_HIP(c, hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        for (auto& ev : c->hev) ORL_HIP(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    uint32_t* d_route = c->st_out;
    uint32_t* d_act = d_route + n;
    uint32_t* d_order = d_act + n;
    const uint8_t* h_in = static_cast<const uint8_t*>(in);
    const size_t esz = (size_t)fmt;
    const size_t chunk = std::max<size_t>(kHostChunk, (n + kHostChunks - 1) / kHostChunks);
    hipStream_t up = c->hstream[0], down = c->hstream[1];
    size_t k = 0;
    for (size_t lo = 0; lo < n; lo += chunk, ++k) {
        const size_t len = std::min(chunk, n - lo);
        hipEvent_t ev_up = c->hev[2 * (k % (kHostChunks + 1))], ev_rt = c->hev[2 * (k % (kHostChunks + 1)) + 1];
        ORL_HIP(c, hipMemcpyAsync(c->st_in + lo * esz, h_in + lo * esz, len * esz, hipMemcpyHostToDevice, up));
        ORL_HIP(c, hipEventRecord(ev_up, up));
        ORL_HIP(c, hipStreamWaitEvent(c->stream, ev_up, 0));
        if ((r = route_impl(c, c->st_in + lo * esz, fmt, len, opts | ORL_OPT_NO_BUCKETS, d_route + lo, d_act + lo, nullptr, nullptr,
                            c->stream)))
            return r;
        ORL_HIP(c, hipEventRecord(ev_rt, c->stream));
        ORL_HIP(c, hipStreamWaitEvent(down, ev_rt, 0));
        ORL_HIP(c, hipMemcpyAsync(route + lo, d_route + lo, len * 4, hipMemcpyDeviceToHost, down));
        ORL_HIP(c, hipMemcpyAsync(act + lo, d_act + lo, len * 4, hipMemcpyDeviceToHost, down));
    }
    if (buckets) {
        int e = launch_bucket_acts(d_act, n, c->cfg.n_act, d_order, c->st_off, c->s, c->stream);
        if (e) return hipfail(c, (hipError_t)e, "bucket launch");
        if (n) ORL_HIP(c, hipMemcpyAsync(order, d_order, n * 4, hipMemcpyDeviceToHost, c->stream));
        ORL_HIP(c, hipMemcpyAsync(offsets, c->st_off, ((size_t)c->cfg.n_act + 2) * 4, hipMemcpyDeviceToHost, c->stream));
    }
    ORL_HIP(c, hipStreamSynchronize(c->stream));
    ORL_HIP(c, hipStreamSynchronize(down));
    ORL_HIP(c, hipStreamSynchronize(up));
    return ORL_OK;
}
}  // namespace

int orl_route_batch(orl_ctx* c, const orl_msg_hdr* in, size_t n, uint32_t opts, uint32_t* route, uint32_t* act,
                    uint32_t* order, uint32_t* offsets) {
    return route_batch_host(c, in, 32, n, opts, route, act, order, offsets);
}

int orl_route_batch_narrow(orl_ctx* c, const orl_wire8* in, size_t n, uint32_t opts, uint32_t* route, uint32_t* act,
                           uint32_t* order, uint32_t* offsets) {
    return route_batch_host(c, in, 8, n, opts, route, act, order, offsets);
}

namespace {
int fanout_impl(orl_ctx* c, const orl_msg_hdr* d_direct, size_t n_direct, const uint64_t* d_csr_off, const uint32_t* d_csr_tgt,
                const orl_grain_key* d_keys, const uint32_t* d_pubs, const uint8_t* d_pub_silo, size_t n_pub,
                uint64_t follower_tcd, uint32_t opts, uint64_t* d_pub_offsets, uint32_t* d_route, uint32_t* d_act,
                uint32_t* d_order, uint32_t* d_off, uint64_t* n_out, void* stream) {
    if (!c || !n_out) return ORL_E_INVALID;
    if (!d_csr_off || !d_csr_tgt || !d_pub_offsets || !d_route || !d_act) return fail(c, ORL_E_INVALID, "null device buffer");
    if (n_pub && (!d_pubs || !d_pub_silo)) return fail(c, ORL_E_INVALID, "null publisher buffer");
    if (n_direct && !d_direct) return fail(c, ORL_E_INVALID, "null direct message buffer");
    if (!(opts & ORL_OPT_NO_BUCKETS) && (!d_order || !d_off)) return fail(c, ORL_E_INVALID, "null order/offsets buffer");
    if (n_pub + 1 > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "too many publishers");
    if (n_direct > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "%zu direct messages > max_batch", n_direct);
    if ((opts & ORL_OPT_TOTAL_GIVEN) && *n_out > c->s.max_batch)
        return fail(c, ORL_E_CAPACITY, "given fan-out total %llu > max_batch", (unsigned long long)*n_out);
    if ((opts & ORL_OPT_TOTAL_GIVEN) && *n_out < n_direct)
        return fail(c, ORL_E_INVALID, "given total %llu < %zu direct messages", (unsigned long long)*n_out, n_direct);
    if (c->n_silos == 0) return fail(c, ORL_E_STATE, "silo table not set");
    int r = sync_device_state(c);
    if (r) return r;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    hipEvent_t* ev = nullptr;
    if (c->timing && c->tcount < ORL_TIMING_SLOTS) ev = &c->tev[4 * (size_t)c->tcount++];
    if ((r = prepare_probe(c, st))) return r;
    if (ev) ORL_HIP(c, hipEventRecord(ev[0], st));
    int e = launch_fanout_route_bucket(c->d_params, dir_view(c), d_direct, n_direct, d_csr_off, d_csr_tgt, d_keys, d_pubs,
                                       d_pub_silo, n_pub,
                                       follower_tcd, opts, c->cfg.n_act, d_pub_offsets, d_route, d_act, d_order, d_off, n_out,
                                       c->s.max_batch, c->s, st, ev ? ev[1] : nullptr, ev ? ev[2] : nullptr);
    if (e == -1) return fail(c, ORL_E_CAPACITY, "fan-out emits %llu > max_batch", (unsigned long long)*n_out);
    if (!e && ctx_cache_on(c)) e = launch_cache_gen_advance(c->d_cache, c->cache_slots - 1, c->s.max_batch, st);  // LRU stamps
    if (e) return hipfail(c, (hipError_t)e, "fanout launch");
    if (ev) {
        if (*n_out == 0) {  // no route kernel ran: mark it empty
            ORL_HIP(c, hipEventRecord(ev[1], st));
            ORL_HIP(c, hipEventRecord(ev[2], st));
        }
        ORL_HIP(c, hipEventRecord(ev[3], st));
    }
    return ORL_OK;
}
}  // namespace

int orl_fanout_route_device(orl_ctx* c, const uint64_t* d_csr_off, const uint32_t* d_csr_tgt, const uint32_t* d_pubs,
                            const uint8_t* d_pub_silo, size_t n_pub, uint64_t follower_tcd, uint32_t opts,
                            uint64_t* d_pub_offsets, uint32_t* d_route, uint32_t* d_act, uint32_t* d_order,
                            uint32_t* d_off, uint64_t* n_out, void* stream) {
    return fanout_impl(c, nullptr, 0, d_csr_off, d_csr_tgt, nullptr, d_pubs, d_pub_silo, n_pub, follower_tcd, opts, d_pub_offsets,
                       d_route, d_act, d_order, d_off, n_out, stream);
}

int orl_fanout_route_keys_device(orl_ctx* c, const uint64_t* d_csr_off, const uint32_t* d_csr_tgt,
                                 const orl_grain_key* d_keys, const uint32_t* d_pubs, const uint8_t* d_pub_silo, size_t n_pub,
                                 uint32_t opts, uint64_t* d_pub_offsets, uint32_t* d_route, uint32_t* d_act, uint32_t* d_order,
                                 uint32_t* d_off, uint64_t* n_out, void* stream) {
    if (c && !d_keys) return fail(c, ORL_E_INVALID, "null follower key table");
    return fanout_impl(c, nullptr, 0, d_csr_off, d_csr_tgt, d_keys, d_pubs, d_pub_silo, n_pub, 0, opts, d_pub_offsets, d_route,
                       d_act, d_order, d_off, n_out, stream);
}

int orl_fanout_route_mixed_device(orl_ctx* c, const orl_msg_hdr* d_direct, size_t n_direct, const uint64_t* d_csr_off,
                                  const uint32_t* d_csr_tgt, const orl_grain_key* d_keys, uint64_t follower_tcd,
                                  const uint32_t* d_pubs, const uint8_t* d_pub_silo, size_t n_pub, uint32_t opts,
                                  uint64_t* d_pub_offsets, uint32_t* d_route, uint32_t* d_act, uint32_t* d_order,
                                  uint32_t* d_off, uint64_t* n_out, void* stream) {
    return fanout_impl(c, d_direct, n_direct, d_csr_off, d_csr_tgt, d_keys, d_pubs, d_pub_silo, n_pub, d_keys ? 0 : follower_tcd,
                       opts, d_pub_offsets, d_route, d_act, d_order, d_off, n_out, stream);
}

int orl_fanout_expand_device(orl_ctx* c, const uint64_t* d_csr_off, const uint32_t* d_csr_tgt, const orl_grain_key* d_keys,
                             uint64_t follower_tcd, const uint32_t* d_pubs, const uint8_t* d_pub_silo, size_t n_pub, uint32_t opts,
                             uint64_t* d_pub_offsets, orl_msg_hdr* d_out, uint64_t cap, uint64_t* n_out, void* stream) {
    if (!c || !n_out) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    if (!d_csr_off || !d_csr_tgt || !d_pub_offsets || (cap && !d_out)) return fail(c, ORL_E_INVALID, "null device buffer");
    if (n_pub && (!d_pubs || !d_pub_silo)) return fail(c, ORL_E_INVALID, "null publisher buffer");
    if (n_pub + 1 > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "too many publishers");
    if ((opts & ORL_OPT_TOTAL_GIVEN) && *n_out > cap)
        return fail(c, ORL_E_CAPACITY, "given fan-out total %llu > cap %llu", (unsigned long long)*n_out, (unsigned long long)cap);
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    const int e = launch_fanout_expand(d_csr_off, d_csr_tgt, d_keys, d_pubs, d_pub_silo, n_pub, d_keys ? 0 : follower_tcd, opts,
                                       d_pub_offsets, d_out, n_out, cap, c->s, st);
    if (e == -1) return fail(c, ORL_E_CAPACITY, "fan-out emits %llu > cap %llu", (unsigned long long)*n_out, (unsigned long long)cap);
    if (e) return hipfail(c, (hipError_t)e, "fan-out expand launch");
    return ORL_OK;
}

namespace {
// Shared checks of the two partition entry points + the rank_of_silo upload (only when it changes).
int partition_prologue(orl_ctx* c, const orl_msg_hdr* d_in, size_t n, const uint8_t* rank_of_silo, uint32_t nranks,
                       uint32_t my_rank, const void* d_out, uint64_t* d_counts, hipStream_t st) {
    if (nranks == 0 || nranks > 8 || my_rank >= nranks) return fail(c, ORL_E_INVALID, "nranks must be 1..8 and my_rank < nranks");
    if (n && (!d_in || !d_out)) return fail(c, ORL_E_INVALID, "null device buffer");
    if (!d_counts) return fail(c, ORL_E_INVALID, "null counts buffer");
    if (n > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "batch too large");
    int r = sync_device_state(c);
    if (r) return r;
    uint8_t ros[256];
    std::memset(ros, 0, sizeof ros);
    for (uint32_t s = 0; s < c->n_silos; ++s) {
        if (rank_of_silo[s] >= nranks) return fail(c, ORL_E_INVALID, "rank_of_silo[%u] = %u >= nranks", s, rank_of_silo[s]);
        ros[s] = rank_of_silo[s];
    }
    if (!c->ros_valid || std::memcmp(ros, c->h_rank_of_silo, sizeof ros) != 0) {  // a membership change: rare
        ORL_HIP(c, hipStreamSynchronize(st));
        ORL_HIP(c, hipMemcpy(c->d_rank_of_silo, ros, 256, hipMemcpyHostToDevice));
        std::memcpy(c->h_rank_of_silo, ros, sizeof ros);
        c->ros_valid = true;
    }
    return ORL_OK;
}
}  // namespace

int orl_partition_by_owner_device(orl_ctx* c, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const uint8_t* rank_of_silo,
                                  uint32_t nranks, uint32_t my_rank, orl_msg_hdr* d_out, uint32_t* d_src, uint64_t* d_counts,
                                  void* stream) {
    if (!c || !rank_of_silo) return ORL_E_INVALID;
    if (n && !d_src) return fail(c, ORL_E_INVALID, "null device buffer");
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    int r = partition_prologue(c, d_in, n, rank_of_silo, nranks, my_rank, d_out, d_counts, st);
    if (r) return r;
    int e = launch_partition_by_owner(c->d_params, d_in, n, opts, c->d_rank_of_silo, nranks, my_rank, d_out, d_src, d_counts,
                                      c->s, st);
    if (e) return hipfail(c, (hipError_t)e, "partition launch");
    return ORL_OK;
}

int orl_partition_by_owner_padded_device(orl_ctx* c, const orl_msg_hdr* d_in, size_t n, uint32_t opts,
                                         const uint8_t* rank_of_silo, uint32_t nranks, uint32_t my_rank, size_t stride,
                                         orl_msg_hdr* d_out, uint32_t* d_src, uint64_t* d_counts, void* stream) {
    if (!c || !rank_of_silo) return ORL_E_INVALID;
    if (stride < n) return fail(c, ORL_E_INVALID, "stride %zu < batch %zu", stride, n);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    int r = partition_prologue(c, d_in, n, rank_of_silo, nranks, my_rank, d_out, d_counts, st);
    if (r) return r;
    int e = launch_partition_padded(c->d_params, d_in, n, opts, c->d_rank_of_silo, nranks, my_rank, stride, d_out, 32, d_src,
                                    d_counts, nullptr, c->s, st);
    if (e) return hipfail(c, (hipError_t)e, "padded partition launch");
    return ORL_OK;
}

}  // extern "C"
namespace orl {
// The node's hop-1 partition: any record width, with the status word (look-back failures included) for every width.
int ctx_partition_padded(orl_ctx* c, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const uint8_t* rank_of_silo,
                         uint32_t nranks, uint32_t my_rank, size_t stride, void* d_out, int fmt, uint64_t* d_counts,
                         uint32_t* d_status, void* stream, uint32_t* d_act_out, const KxLanes* kxl) {
    if (!c || !rank_of_silo || !d_status) return ORL_E_INVALID;
    if (fmt != 8 && fmt != 16 && fmt != 32) return fail(c, ORL_E_INVALID, "record width %d", fmt);
    if (stride < n) return fail(c, ORL_E_INVALID, "stride %zu < batch %zu", stride, n);
    if (fmt == 8 && c->hp.n_wire_types == 0) return fail(c, ORL_E_STATE, "8-byte records need the wire types (orl_wire_types_set)");
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    int r = partition_prologue(c, d_in, n, rank_of_silo, nranks, my_rank, d_out, d_counts, st);
    if (r) return r;
    const bool cached = d_act_out && ctx_cache_on(c);
    int e = launch_partition_padded(c->d_params, d_in, n, opts, c->d_rank_of_silo, nranks, my_rank, stride, d_out, fmt, nullptr,
                                    d_counts, d_status, c->s, st, cached ? c->d_cache : nullptr,
                                    cached ? c->cache_slots - 1 : 0, cached ? d_act_out : nullptr, kxl);
    if (!e && cached) e = launch_cache_gen_advance(c->d_cache, c->cache_slots - 1, n, st);  // the sender's lookups' LRU stamps
    if (e) return hipfail(c, (hipError_t)e, "node partition launch");
    return ORL_OK;
}
}  // namespace orl
extern "C" {

int orl_partition_compact_device(orl_ctx* c, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const uint8_t* rank_of_silo,
                                 uint32_t nranks, uint32_t my_rank, size_t stride, orl_wire_msg* d_out, uint32_t* d_src,
                                 uint64_t* d_counts, uint32_t* d_status, void* stream) {
    if (!c || !rank_of_silo) return ORL_E_INVALID;
    if (stride < n) return fail(c, ORL_E_INVALID, "stride %zu < batch %zu", stride, n);
    if (!d_status) return fail(c, ORL_E_INVALID, "null status word");
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    int r = partition_prologue(c, d_in, n, rank_of_silo, nranks, my_rank, d_out, d_counts, st);
    if (r) return r;
    int e = launch_partition_padded(c->d_params, d_in, n, opts, c->d_rank_of_silo, nranks, my_rank, stride, d_out, 16, d_src,
                                    d_counts, d_status, c->s, st);
    if (e) return hipfail(c, (hipError_t)e, "compact partition launch");
    return ORL_OK;
}

int orl_partition_narrow_device(orl_ctx* c, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const uint8_t* rank_of_silo,
                                uint32_t nranks, uint32_t my_rank, size_t stride, orl_wire8* d_out, uint32_t* d_src,
                                uint64_t* d_counts, uint32_t* d_status, void* stream) {
    if (!c || !rank_of_silo) return ORL_E_INVALID;
    if (stride < n) return fail(c, ORL_E_INVALID, "stride %zu < batch %zu", stride, n);
    if (!d_status) return fail(c, ORL_E_INVALID, "null status word");
    if (c->hp.n_wire_types == 0) return fail(c, ORL_E_STATE, "8-byte records need the wire types (orl_wire_types_set)");
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    int r = partition_prologue(c, d_in, n, rank_of_silo, nranks, my_rank, d_out, d_counts, st);
    if (r) return r;
    int e = launch_partition_padded(c->d_params, d_in, n, opts, c->d_rank_of_silo, nranks, my_rank, stride, d_out, 8, d_src,
                                    d_counts, d_status, c->s, st);
    if (e) return hipfail(c, (hipError_t)e, "narrow partition launch");
    return ORL_OK;
}

int orl_partition_cached_device(orl_ctx* c, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const uint8_t* rank_of_silo,
                                uint32_t nranks, uint32_t my_rank, size_t stride, void* d_out, uint32_t fmt,
                                uint32_t* d_act_out, uint64_t* d_counts, uint32_t* d_status, void* stream) {
    if (!c || !rank_of_silo) return ORL_E_INVALID;
    if (n && !d_act_out) return fail(c, ORL_E_INVALID, "null act lane");
    if (!ctx_cache_on(c) && n) {  // no cache: every record unaddressed
        hipStream_t st = stream ? (hipStream_t)stream : c->stream;
        for (uint32_t r = 0; r < nranks && r < 8; ++r)
            ORL_HIP(c, hipMemsetAsync(d_act_out + (size_t)r * stride, 0xFF, n * 4, st));
    }
    return ctx_partition_padded(c, d_in, n, opts, rank_of_silo, nranks, my_rank, stride, d_out, (int)fmt, d_counts, d_status,
                                stream, d_act_out);
}

int orl_route_received_device(orl_ctx* c, const void* d_in, uint32_t fmt, size_t n, uint32_t opts, const uint32_t* d_in_act,
                              uint32_t* d_route, uint32_t* d_act, void* stream) {
    return ctx_route_received(c, d_in, (int)fmt, n, opts, d_route, d_act, d_in_act, stream);
}

int orl_wire_types_set(orl_ctx* c, uint32_t n, const uint64_t* tcd) {
    if (!c) return ORL_E_INVALID;
    if (n > ORL_MAX_WIRE_TYPES || (n && !tcd)) return fail(c, ORL_E_INVALID, "wire types: n = %u (at most %u)", n, ORL_MAX_WIRE_TYPES);
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t j = 0; j < i; ++j)
            if (tcd[i] == tcd[j]) return fail(c, ORL_E_INVALID, "wire types: entry %u repeats entry %u", i, j);
    RouteParams& P = c->hp;
    std::memset(P.wire_tcd, 0, sizeof P.wire_tcd);
    if (n) std::memcpy(P.wire_tcd, tcd, n * sizeof(uint64_t));
    P.n_wire_types = n;
    uint64_t h = 0xCBF29CE484222325ull;  // FNV-1a over the count and the values, little-endian bytes
    auto mix = [&](uint64_t v) {
        for (int b = 0; b < 8; ++b) { h ^= (v >> (8 * b)) & 0xFFu; h *= 0x100000001B3ull; }
    };
    mix(n);
    for (uint32_t i = 0; i < n; ++i) mix(tcd[i]);
    P.wire_digest = n ? h : 0;
    c->params_dirty = true;
    return ORL_OK;
}

int orl_dir_insert_single_device(orl_ctx* c, const orl_grain_key* d_keys, const uint32_t* d_acts, const uint8_t* d_silos,
                                 size_t n, uint32_t* d_wact, uint8_t* d_wsilo, uint8_t* d_status, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (n && (!d_keys || !d_acts || !d_silos || !d_status)) return fail(c, ORL_E_INVALID, "null device buffer");
    if (n > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "batch %zu > max_batch %llu", n, (unsigned long long)c->s.max_batch);
    if (c->n_silos == 0) return fail(c, ORL_E_STATE, "silo table not set");
    int r = sync_device_state(c);
    if (r) return r;
    // every message might insert: live entries stay <= 1/2 of the slots, entries + tombstones <= 7/8
    auto fits = [&](uint64_t cnt, uint64_t tombs) {
        return (cnt + n) * 2 <= c->table.size() && (cnt + tombs + n) * 8 <= c->table.size() * 7;
    };
    if (!fits(c->count_ub, c->tombs_ub)) {
        if ((r = refresh_counts(c))) return r;
        if (!fits(c->count_ub, c->tombs_ub))
            return fail(c, ORL_E_CAPACITY, "directory full (%llu entries + %llu tombstones + batch %zu; orl_dir_compact "
                        "drops tombstones)", (unsigned long long)c->count_ub, (unsigned long long)c->tombs_ub, n);
    }
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    int e = launch_dir_insert(c->d_params, c->d_table, c->mask, c->d_claim, c->d_dirstate, d_keys, d_acts, d_silos, n,
                              c->cfg.n_act, c->n_silos, c->d_dslot, d_wact, d_wsilo, d_status,
                              reinterpret_cast<uint32_t*>(c->d_dirstate + 2), st);
    if (e) return hipfail(c, (hipError_t)e, "directory insert launch");
    c->count_ub += n;
    c->mirror_stale = true;
    probe_after_device_mutation(c);
    return ORL_OK;
}

int orl_dir_merge_device(orl_ctx* c, const orl_grain_key* d_keys, const uint32_t* d_acts, const uint8_t* d_silos, size_t n,
                         const orl_grain_key* d_act_keys, uint32_t n_act_keys, uint8_t* d_status, uint32_t* d_dropped_act,
                         uint8_t* d_dropped_silo, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (n && (!d_keys || !d_acts || !d_silos || !d_status || !d_act_keys)) return fail(c, ORL_E_INVALID, "null device buffer");
    if (n > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "batch %zu > max_batch %llu", n, (unsigned long long)c->s.max_batch);
    if (c->n_silos == 0) return fail(c, ORL_E_STATE, "silo table not set");
    int r = sync_device_state(c);
    if (r) return r;
    auto fits = [&](uint64_t cnt, uint64_t tombs) {
        return (cnt + n) * 2 <= c->table.size() && (cnt + tombs + n) * 8 <= c->table.size() * 7;
    };
    if (!fits(c->count_ub, c->tombs_ub)) {
        if ((r = refresh_counts(c))) return r;
        if (!fits(c->count_ub, c->tombs_ub))
            return fail(c, ORL_E_CAPACITY, "directory full (%llu entries + %llu tombstones + batch %zu)",
                        (unsigned long long)c->count_ub, (unsigned long long)c->tombs_ub, n);
    }
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    int e = launch_dir_merge(c->d_table, c->mask, c->d_claim, c->d_dirstate, d_keys, d_acts, d_silos, n, c->cfg.n_act, c->n_silos,
                             d_act_keys, n_act_keys, c->d_dslot, d_status, d_dropped_act, d_dropped_silo,
                             reinterpret_cast<uint32_t*>(c->d_dirstate + 2), st);
    if (e) return hipfail(c, (hipError_t)e, "directory merge launch");
    c->count_ub += n;
    c->mirror_stale = true;
    probe_after_device_mutation(c);
    return ORL_OK;
}

int orl_dir_remove_device(orl_ctx* c, const orl_grain_key* d_keys, size_t n, uint8_t* d_removed, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (n && (!d_keys || !d_removed)) return fail(c, ORL_E_INVALID, "null device buffer");
    if (n > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "batch %zu > max_batch %llu", n, (unsigned long long)c->s.max_batch);
    int r = sync_device_state(c);
    if (r) return r;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    int e = launch_dir_remove(c->d_table, c->mask, c->d_claim, c->d_dirstate, d_keys, n, c->d_dslot, d_removed, st);
    if (e) return hipfail(c, (hipError_t)e, "directory remove launch");
    c->tombs_ub += n;
    c->mirror_stale = true;
    probe_after_device_mutation(c);
    return ORL_OK;
}

int orl_dir_split_device(orl_ctx* c, uint32_t me, uint32_t flags, orl_grain_key* d_keys, uint32_t* d_acts, uint8_t* d_silos,
                         uint64_t cap, uint64_t* d_n_out, void* stream) {
    if (!c || !d_n_out) return ORL_E_INVALID;
    if (cap && (!d_keys || !d_acts || !d_silos)) return fail(c, ORL_E_INVALID, "null device buffer");
    if (!silo_ok(c, me)) return fail(c, ORL_E_INVALID, "silo %u out of range", me);
    int r = sync_device_state(c);
    if (r) return r;
    // the tile counts live in the scratch histogram: a table of more slots than the scan scratch is split by the host
    if ((c->table.size() + kTile - 1) / kTile > c->s.max_tiles * (1ull << kMaxDigitBits))
        return fail(c, ORL_E_CAPACITY, "table too large for the split scratch");
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    const bool remove = flags & ORL_SPLIT_REMOVE;
    int e = launch_dir_split(c->d_params, c->d_table, c->table.size(), me, remove, c->d_dirstate, d_keys, d_acts, d_silos, cap,
                             d_n_out, c->s, st);
    if (e) return hipfail(c, (hipError_t)e, "directory split launch");
    if (remove) {
        c->mirror_stale = true;
        probe_after_device_mutation(c);
    }  // tombstones: the upper bounds stay valid (entries + tombstones unchanged)
    return ORL_OK;
}

int orl_dir_compact(orl_ctx* c) {
    if (!c) return ORL_E_INVALID;
    if (!c->device_mode) return ORL_OK;
    if (int r = ensure_mirror(c)) return r;
    if (c->tombs == 0) return ORL_OK;
    std::vector<DirSlot> old;
    old.swap(c->table);
    c->table.assign(old.size(), DirSlot{});
    c->count = c->tombs = 0;
    for (const DirSlot& d : old) {  // re-insert every live entry in slot order (lookups are layout-independent)
        if (d.state != SLOT_FULL) continue;
        uint64_t i = dir_slot(jenkins3(d.tcd, d.n0, d.n1), c->mask);
        while (c->table[i].state != SLOT_EMPTY) i = (i + 1) & c->mask;
        c->table[i] = d;
        ++c->count;
    }
    c->dir_dirty = true;
    return sync_device_state(c);
}

// ---- f3: stream / reminder rings -----------------------------------------------------------------
int orl_vring_set_buckets(orl_ctx* c, uint32_t nb) {
    if (!c) return ORL_E_INVALID;
    if (nb == 0 || nb > ORL_MAX_VBUCKETS_PER_SILO) return fail(c, ORL_E_INVALID, "buckets per silo must be 1..%u", ORL_MAX_VBUCKETS_PER_SILO);
    if (!c->vr_hashes.empty()) return fail(c, ORL_E_STATE, "virtual-bucket ring not empty");
    c->vr_nb = nb;
    return ORL_OK;
}

int orl_vring_add_server(orl_ctx* c, uint32_t silo, const uint8_t* ip16, int32_t port, int32_t gen) {
    if (!c || !ip16) return ORL_E_INVALID;
    if (!silo_ok(c, silo)) return fail(c, ORL_E_INVALID, "silo %u not in the silo table", silo);
    // SiloAddress.GetUniformHashCodes (SiloAddress.cs:208-230): Jenkins over Write(SiloAddress) + Write(int i):
    // 16-B IP (IPv4 as 12 zero bytes + 4), port LE4, generation LE4, i LE4 (BinaryTokenStreamWriter.cs:448-486)
    std::vector<uint32_t> hs(c->vr_nb);
    uint8_t b[28];
    std::memcpy(b, ip16, 16);
    for (int k = 0; k < 4; ++k) {
        b[16 + k] = (uint8_t)((uint32_t)port >> (8 * k));
        b[20 + k] = (uint8_t)((uint32_t)gen >> (8 * k));
    }
    for (uint32_t i = 0; i < c->vr_nb; ++i) {
        for (int k = 0; k < 4; ++k) b[24 + k] = (uint8_t)(i >> (8 * k));
        hs[i] = jenkins_bytes(b, 28);
    }
    c->vr_hashes[(uint8_t)silo] = hs;
    c->vr_gen[(uint8_t)silo] = gen;
    for (uint32_t h : hs) {  // AddServer (VirtualBucketsRingProvider.cs:142-169)
        auto it = c->vr_map.find(h);
        if (it != c->vr_map.end() && gen > c->vr_gen[it->second]) continue;  // lesser generation keeps the bucket
        c->vr_map[h] = (uint8_t)silo;
    }
    c->vr_dirty = true;
    return ORL_OK;
}

int orl_vring_remove_server(orl_ctx* c, uint32_t silo) {
    if (!c) return ORL_E_INVALID;
    bool owns = false;  // bucketsMap.ContainsValue(silo) (:174)
    for (const auto& e : c->vr_map) owns |= e.second == silo;
    if (!owns) return ORL_OK;
    for (uint32_t h : c->vr_hashes[(uint8_t)silo]) c->vr_map.erase(h);  // every one of ITS hashes (:176-180)
    c->vr_dirty = true;
    return ORL_OK;
}

int orl_vring_get(const orl_ctx* c, uint32_t* hashes, uint8_t* silos, uint32_t cap, uint32_t* n_out) {
    if (!c || !n_out) return ORL_E_INVALID;
    uint32_t i = 0;
    for (const auto& e : c->vr_map) {
        if (i < cap) {
            if (hashes) hashes[i] = e.first;
            if (silos) silos[i] = e.second;
        }
        ++i;
    }
    *n_out = i;
    return ORL_OK;
}

namespace {
int ring_prologue(orl_ctx* c, uint32_t kind, uint32_t me, uint32_t opts, bool* excl) {
    if (kind != ORL_RING_CONSISTENT && kind != ORL_RING_VBUCKETS) return fail(c, ORL_E_INVALID, "unknown ring kind %u", kind);
    if (!silo_ok(c, me)) return fail(c, ORL_E_INVALID, "silo %u out of range", me);
    *excl = (opts & ORL_OPT_EXCLUDE_IF_STOPPING) && !c->running[me];  // excludeMySelf
    return sync_device_state(c);
}
}  // namespace

int orl_ring_owner_batch_device(orl_ctx* c, uint32_t kind, const uint32_t* d_keys, size_t n, uint32_t me, uint32_t opts,
                                uint8_t* d_owner, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (n && (!d_keys || !d_owner)) return fail(c, ORL_E_INVALID, "null device buffer");
    if (n > 0xFFFFFFFFull) return fail(c, ORL_E_CAPACITY, "batch too large");
    bool excl;
    if (int r = ring_prologue(c, kind, me, opts, &excl)) return r;
    int e = launch_ring_owner(kind, c->d_params, c->d_vr_hash, c->d_vr_silo, c->vr_n_dev, d_keys, n, me, excl, d_owner,
                              stream ? stream : c->stream);
    if (e) return hipfail(c, (hipError_t)e, "ring owner launch");
    return ORL_OK;
}

int orl_stream_queue_batch_device(orl_ctx* c, uint32_t kind, const uint8_t* d_guids, size_t n, uint32_t n_queues, uint32_t me,
                                  uint32_t opts, uint32_t* d_queue, uint8_t* d_silo, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (n && (!d_guids || !d_queue)) return fail(c, ORL_E_INVALID, "null device buffer");
    if (n_queues == 0 || n_queues >= 65536) return fail(c, ORL_E_INVALID, "n_queues must be 1..65535");
    if (n > 0xFFFFFFFFull) return fail(c, ORL_E_CAPACITY, "batch too large");
    bool excl;
    if (int r = ring_prologue(c, kind, me, opts, &excl)) return r;
    int e = launch_stream_queue(kind, c->d_params, c->d_vr_hash, c->d_vr_silo, c->vr_n_dev, d_guids, n, n_queues, me, excl,
                                d_queue, d_silo, stream ? stream : c->stream);
    if (e) return hipfail(c, (hipError_t)e, "stream queue launch");
    return ORL_OK;
}

// ---- f4: directory cache ---------------------------------------------------------------------------
int orl_cache_config(orl_ctx* c, uint64_t capacity) {
    if (!c) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    if (capacity == 0) return fail(c, ORL_E_INVALID, "capacity must be >= 1");
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    ORL_HIP(c, hipDeviceSynchronize());
    (void)hipFree(c->d_cache); (void)hipFree(c->d_cclaim); (void)hipFree(c->d_cstate);
    c->d_cache = nullptr; c->d_cclaim = nullptr; c->d_cstate = nullptr;
    const uint64_t slots = next_pow2(2 * capacity);
    // the table, then one u64 LRU generation per slot and the generation base (route_kernels.hip cache_gens)
    const size_t bytes = slots * sizeof(DirSlot) + (slots + 1) * 8;
    ORL_HIP(c, hipMalloc((void**)&c->d_cache, bytes));
    ORL_HIP(c, hipMalloc((void**)&c->d_cclaim, slots * 4));
    ORL_HIP(c, hipMalloc((void**)&c->d_cstate, 32));
    ORL_HIP(c, hipMemset(c->d_cache, 0, bytes));
    ORL_HIP(c, hipMemset(c->d_cclaim, 0xFF, slots * 4));
    ORL_HIP(c, hipMemset(c->d_cstate, 0, 32));
    c->cache_slots = slots;
    c->cache_cap = capacity;
    c->cache_gen_free = 0;
    c->cache_ub = c->cache_tombs_ub = 0;
    set_cache_on(c, false);
    return ORL_OK;
}

int orl_cache_clear(orl_ctx* c) {  // LRU.Clear: the entries go, the generation counters run on
    if (!c) return ORL_E_INVALID;
    if (!c->cache_slots) return ORL_OK;
    ORL_HIP(c, hipDeviceSynchronize());
    ORL_HIP(c, hipMemset(c->d_cache, 0, c->cache_slots * sizeof(DirSlot)));
    ORL_HIP(c, hipMemset(c->d_cstate, 0, 32));
    c->cache_ub = c->cache_tombs_ub = 0;
    set_cache_on(c, false);
    return ORL_OK;
}

namespace {
// AddOrUpdate of a batch that can overflow the capacity: the reference's sequential LRU on the host, exactly
// (AdaptiveGrainDirectoryCache.AddOrUpdate → LRU.Add: AdjustSize — while Count >= MaximumSize free the entry of the next
// generation, LRU.cs:188-205 — then AddOrUpdate with the next generation, :104-108), over the device table read back, then
// the table rebuilt and uploaded (no tombstones).  Entries the device path would not keep (an invalid silo, a handle
// outside this context's space on a local silo: k_cache_probe) are skipped as there.  Generations stay the device's
// sparse stamps (only their order matters); G advances by n as on the fast path.
int cache_add_host_lru(orl_ctx* c, const orl_grain_key* d_keys, const uint32_t* d_acts, const uint8_t* d_silos, size_t n) {
    const uint64_t slots = c->cache_slots, mask = slots - 1;
    ORL_HIP(c, hipDeviceSynchronize());
    std::vector<DirSlot> tab(slots);
    std::vector<uint64_t> gen(slots + 1);
    ORL_HIP(c, hipMemcpy(tab.data(), c->d_cache, slots * sizeof(DirSlot), hipMemcpyDeviceToHost));
    ORL_HIP(c, hipMemcpy(gen.data(), reinterpret_cast<uint8_t*>(c->d_cache) + slots * sizeof(DirSlot), (slots + 1) * 8,
                         hipMemcpyDeviceToHost));
    std::vector<orl_grain_key> keys(n);
    std::vector<uint32_t> acts(n);
    std::vector<uint8_t> silos(n);
    if (n) {
        ORL_HIP(c, hipMemcpy(keys.data(), d_keys, n * sizeof(orl_grain_key), hipMemcpyDeviceToHost));
        ORL_HIP(c, hipMemcpy(acts.data(), d_acts, n * 4, hipMemcpyDeviceToHost));
        ORL_HIP(c, hipMemcpy(silos.data(), d_silos, n, hipMemcpyDeviceToHost));
    }
    struct Ent {
        orl_grain_key k;
        uint32_t act;
        uint8_t silo;
        uint64_t gen;
    };
    auto kk = [](const orl_grain_key& k) { return std::make_tuple(k.type_code_data, k.n0, k.n1); };
    std::map<std::tuple<uint64_t, uint64_t, uint64_t>, Ent> ents;  // the cache
    std::map<uint64_t, std::tuple<uint64_t, uint64_t, uint64_t>> by_gen;  // LRU order
    for (uint64_t i = 0; i < slots; ++i)
        if (tab[i].state == SLOT_FULL) {
            const orl_grain_key k{tab[i].tcd, tab[i].n0, tab[i].n1};
            ents[kk(k)] = Ent{k, tab[i].act, tab[i].silo, gen[i]};
            by_gen[gen[i]] = kk(k);
        }
    const uint64_t G = gen[slots];
    for (size_t i = 0; i < n; ++i) {
        const uint32_t sl = silos[i];
        if (!(sl < c->n_silos && (acts[i] < c->cfg.n_act || (acts[i] != ORL_NO_ACT && !c->local[sl])))) continue;
        while (ents.size() >= c->cache_cap && !by_gen.empty()) {  // AdjustSize
            auto v = by_gen.begin();
            c->cache_gen_free = v->first;
            ents.erase(v->second);
            by_gen.erase(v);
        }
        const auto key = kk(keys[i]);
        const uint64_t g = G + i + 1;
        auto it = ents.find(key);
        if (it != ents.end()) {
            by_gen.erase(it->second.gen);
            it->second = Ent{keys[i], acts[i], (uint8_t)sl, g};
        } else {
            ents[key] = Ent{keys[i], acts[i], (uint8_t)sl, g};
        }
        by_gen[g] = key;
    }
    std::fill(tab.begin(), tab.end(), DirSlot{});
    std::fill(gen.begin(), gen.end() - 1, 0ull);
    gen[slots] = G + n;
    for (const auto& kv : ents) {
        const Ent& e = kv.second;
        uint64_t i = dir_slot(jenkins3(e.k.type_code_data, e.k.n0, e.k.n1), mask);
        while (tab[i].state != SLOT_EMPTY) i = (i + 1) & mask;
        tab[i].tcd = e.k.type_code_data; tab[i].n0 = e.k.n0; tab[i].n1 = e.k.n1;
        tab[i].act = e.act; tab[i].silo = e.silo; tab[i].state = SLOT_FULL;
        gen[i] = e.gen;
    }
    ORL_HIP(c, hipMemcpy(c->d_cache, tab.data(), slots * sizeof(DirSlot), hipMemcpyHostToDevice));
    ORL_HIP(c, hipMemcpy(reinterpret_cast<uint8_t*>(c->d_cache) + slots * sizeof(DirSlot), gen.data(), (slots + 1) * 8,
                         hipMemcpyHostToDevice));
    const uint64_t stw[3] = {ents.size(), 0, 0};
    ORL_HIP(c, hipMemcpy(c->d_cstate, stw, sizeof stw, hipMemcpyHostToDevice));
    c->cache_ub = ents.size();
    c->cache_tombs_ub = 0;
    return ORL_OK;
}
}  // namespace

// LRU.Add per entry in batch order.  No entry can be evicted while the cache holds <= capacity - n entries before the batch
// (every add then finds Count < MaximumSize): the device path (the batch's last writer of a key wins, its generation
// stamped).  Otherwise the exact sequential LRU on the host (cache_add_host_lru).
int orl_cache_add_or_update_device(orl_ctx* c, const orl_grain_key* d_keys, const uint32_t* d_acts, const uint8_t* d_silos,
                                   size_t n, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (!c->cache_slots) return fail(c, ORL_E_STATE, "directory cache not configured (orl_cache_config)");
    if (n && (!d_keys || !d_acts || !d_silos)) return fail(c, ORL_E_INVALID, "null device buffer");
    if (n > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "batch %zu > max_batch %llu", n, (unsigned long long)c->s.max_batch);
    auto fits = [&](uint64_t cnt, uint64_t tombs) {  // no eviction possible, and the table's load stays <= 7/8
        return cnt + n <= c->cache_cap && (cnt + tombs + n) * 8 <= c->cache_slots * 7;
    };
    int r = sync_device_state(c);
    if (r) return r;
    set_cache_on(c, true);
    if ((r = sync_device_state(c))) return r;
    if (!fits(c->cache_ub, c->cache_tombs_ub)) {  // exact counters (a sync)
        ORL_HIP(c, hipDeviceSynchronize());
        uint64_t stw[3];
        ORL_HIP(c, hipMemcpy(stw, c->d_cstate, sizeof stw, hipMemcpyDeviceToHost));
        c->cache_ub = stw[0];
        c->cache_tombs_ub = stw[1];
        if (!fits(c->cache_ub, c->cache_tombs_ub)) return cache_add_host_lru(c, d_keys, d_acts, d_silos, n);
    }
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    int e = launch_cache_update(c->d_cache, c->cache_slots - 1, c->d_cclaim, c->d_cstate, d_keys, d_acts, d_silos, n, c->cfg.n_act,
                                c->n_silos, c->d_dslot, c->d_dflag, reinterpret_cast<uint32_t*>(c->d_cstate + 2), st, c->d_params);
    if (e) return hipfail(c, (hipError_t)e, "cache update launch");
    c->cache_ub += n;
    return ORL_OK;
}

int orl_cache_remove_device(orl_ctx* c, const orl_grain_key* d_keys, size_t n, uint8_t* d_removed, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (!c->cache_slots) return fail(c, ORL_E_STATE, "directory cache not configured (orl_cache_config)");
    if (n && (!d_keys || !d_removed)) return fail(c, ORL_E_INVALID, "null device buffer");
    if (n > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "batch %zu > max_batch %llu", n, (unsigned long long)c->s.max_batch);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    int e = launch_dir_remove(c->d_cache, c->cache_slots - 1, c->d_cclaim, c->d_cstate, d_keys, n, c->d_dslot, d_removed, st);
    if (e) return hipfail(c, (hipError_t)e, "cache remove launch");
    c->cache_tombs_ub += n;
    return ORL_OK;
}

int orl_cache_count(orl_ctx* c, uint64_t* n) {
    if (!c || !n) return ORL_E_INVALID;
    *n = 0;
    if (!c->cache_slots) return ORL_OK;
    ORL_HIP(c, hipDeviceSynchronize());
    uint64_t st[3];
    ORL_HIP(c, hipMemcpy(st, c->d_cstate, sizeof st, hipMemcpyDeviceToHost));
    *n = st[0];
    return ORL_OK;
}

// ---- f4: outbound queues, client buckets --------------------------------------------------------
int orl_outbound_queues_device(orl_ctx* c, const orl_msg_hdr* d_msgs, const uint32_t* d_route, size_t n, uint32_t n_senders,
                               uint32_t* d_queue, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (n && (!d_msgs || !d_route || !d_queue)) return fail(c, ORL_E_INVALID, "null device buffer");
    if (n_senders == 0) return fail(c, ORL_E_INVALID, "n_senders must be >= 1");
    if (n > 0xFFFFFFFFull) return fail(c, ORL_E_CAPACITY, "batch too large");
    if (int r = sync_device_state(c)) return r;
    int e = launch_outbound_queues(d_msgs, d_route, n, n_senders, c->d_silo_hash, c->d_silo_known, d_queue,
                                   stream ? stream : c->stream);
    if (e) return hipfail(c, (hipError_t)e, "outbound queues launch");
    return ORL_OK;
}

int orl_client_buckets_device(orl_ctx* c, const orl_msg_hdr* d_msgs, size_t n, uint32_t n_buckets, uint32_t* d_bucket,
                              void* stream) {
    if (!c) return ORL_E_INVALID;
    if (n && (!d_msgs || !d_bucket)) return fail(c, ORL_E_INVALID, "null device buffer");
    // above 2^30, ((key % mod) + mod) can pass int.MaxValue: the reference's checked((uint)key) then throws
    if (n_buckets == 0 || n_buckets > (1u << 30)) return fail(c, ORL_E_INVALID, "n_buckets must be in [1, 2^30]");
    if (n > 0xFFFFFFFFull) return fail(c, ORL_E_CAPACITY, "batch too large");
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    int e = launch_client_buckets(d_msgs, n, n_buckets, d_bucket, stream ? stream : c->stream);
    if (e) return hipfail(c, (hipError_t)e, "client buckets launch");
    return ORL_OK;
}

// ---- f2: wire codec ---------------------------------------------------------------------------------
int orl_silo_address_set(orl_ctx* c, uint32_t silo, const uint8_t* ip16, int32_t port, int32_t generation) {
    if (!c) return ORL_E_INVALID;
    if (silo >= 255) return fail(c, ORL_E_INVALID, "silo index %u out of range (< 255)", silo);
    if (!ip16) {
        c->silo_addr_known[silo] = 0;
        c->silo_addr_dirty = true;
        return ORL_OK;
    }
    if (port < 0 || port > 65535) return fail(c, ORL_E_INVALID, "port %d out of range", port);
    uint32_t w[6];
    std::memcpy(w, ip16, 16);
    w[4] = (uint32_t)port;
    w[5] = (uint32_t)generation;
    for (uint32_t s = 0; s < 255; ++s)
        if (s != silo && c->silo_addr_known[s] && std::memcmp(c->silo_addr[s], w, sizeof w) == 0)
            return fail(c, ORL_E_INVALID, "address already belongs to silo %u", s);
    std::memcpy(c->silo_addr[silo], w, sizeof w);
    c->silo_addr_known[silo] = 1;
    c->silo_addr_dirty = true;
    return ORL_OK;
}

int orl_decode_frames_device(orl_ctx* c, const uint8_t* d_bytes, uint64_t nbytes, const uint64_t* d_frame_offsets, size_t n,
                             uint32_t sender_override, orl_msg_hdr* d_out, uint8_t* d_status, uint32_t* d_n_bad, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (n && (!d_bytes || !d_frame_offsets || !d_out || !d_status)) return fail(c, ORL_E_INVALID, "null device buffer");
    if ((uintptr_t)d_bytes & 3u) return fail(c, ORL_E_INVALID, "frame buffer must be 4-byte aligned");
    if (sender_override > ORL_SENDER_FROM_HEADER) return fail(c, ORL_E_INVALID, "sender_override must be < 255 or 0xFF");
    if (n > 0xFFFFFFFFull) return fail(c, ORL_E_CAPACITY, "batch too large");
    if (int r = sync_device_state(c)) return r;
    int e = launch_decode_frames(d_bytes, nbytes, d_frame_offsets, n, sender_override, c->d_silo_tab, d_out, d_status,
                                 d_n_bad, c->d_decode_flag, stream ? stream : c->stream);
    if (e) return hipfail(c, (hipError_t)e, "decode frames launch");
    return ORL_OK;
}

int orl_grain_type_set(orl_ctx* c, int32_t type_code, const char* utf8, size_t len) {
    if (!c) return ORL_E_INVALID;
    if (len == 0 || !utf8) {
        c->grain_types.erase(type_code);
        c->gt_dirty = true;
        return ORL_OK;
    }
    size_t total = len;
    for (const auto& kv : c->grain_types)
        if (kv.first != type_code) total += kv.second.size();
    if (total > kGrainTypeBlob) return fail(c, ORL_E_CAPACITY, "grain type names exceed %u bytes", kGrainTypeBlob);
    if (c->grain_types.size() >= kGrainTypeSlots / 2 && !c->grain_types.count(type_code))
        return fail(c, ORL_E_CAPACITY, "more than %u grain types", kGrainTypeSlots / 2);
    c->grain_types[type_code] = std::string(utf8, len);
    c->gt_dirty = true;
    return ORL_OK;
}

int orl_stamp_frames_device(orl_ctx* c, const uint8_t* d_bytes, uint64_t nbytes, const uint64_t* d_frame_offsets, size_t n,
                            const uint32_t* d_route, const uint32_t* d_act, const orl_grain_key* d_act_keys, uint32_t n_act_keys,
                            const orl_grain_key* d_new_act_keys, uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_offsets,
                            uint64_t* d_out_total, uint8_t* d_status, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (!d_out_total) return fail(c, ORL_E_INVALID, "null total pointer");
    if (n && (!d_bytes || !d_frame_offsets || !d_route || !d_act || !d_out || !d_out_offsets || !d_status))
        return fail(c, ORL_E_INVALID, "null device buffer");
    if (n_act_keys && !d_act_keys) return fail(c, ORL_E_INVALID, "null activation key table");
    if (((uintptr_t)d_bytes & 3u) || ((uintptr_t)d_out & 3u)) return fail(c, ORL_E_INVALID, "frame buffers must be 4-byte aligned");
    if (n > 0xFFFFFFFFull) return fail(c, ORL_E_CAPACITY, "batch too large");
    if (int r = sync_device_state(c)) return r;
    if (n > c->stamp_cap) {  // scratch grows to the largest batch seen (a synchronising allocation, once)
        if (c->d_stamp_sizes) (void)hipFree(c->d_stamp_sizes);
        if (c->d_stamp_temp) (void)hipFree(c->d_stamp_temp);
        c->d_stamp_sizes = nullptr;
        c->d_stamp_temp = nullptr;
        c->stamp_cap = 0;
        const size_t tb = stamp_scan_temp_bytes(n);
        ORL_HIP(c, hipMalloc((void**)&c->d_stamp_sizes, (n + 1) * sizeof(uint64_t)));  // + the deferral flag
        ORL_HIP(c, hipMalloc(&c->d_stamp_temp, std::max<size_t>(tb, 16)));
        c->stamp_cap = n;
        c->stamp_temp_bytes = std::max<size_t>(tb, 16);
    }
    int e = launch_stamp_frames(d_bytes, nbytes, d_frame_offsets, n, d_route, d_act, d_act_keys, n_act_keys, d_new_act_keys,
                                c->d_gt, c->d_gt_blob, c->d_silo_words, c->d_stamp_sizes, c->d_stamp_temp, c->stamp_temp_bytes,
                                d_out, out_cap, d_out_offsets, d_out_total, d_status, stream ? stream : c->stream);
    if (e) return hipfail(c, (hipError_t)e, "stamp frames launch");
    return ORL_OK;
}

int orl_sync(orl_ctx* c) {
    if (!c) return ORL_E_INVALID;
    if (!c->device_mode) return ORL_OK;
    ORL_HIP(c, hipStreamSynchronize(c->stream));
    return ORL_OK;
}

int orl_bucket_device(orl_ctx* c, const uint32_t* d_act, size_t n, uint32_t* d_order, uint32_t* d_off, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    if (!d_off || (n && (!d_act || !d_order))) return fail(c, ORL_E_INVALID, "null device buffer");
    if (n > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "batch %zu > max_batch %llu", n, (unsigned long long)c->s.max_batch);
    int e = launch_bucket_acts(d_act, n, c->cfg.n_act, d_order, d_off, c->s, stream ? stream : c->stream);
    if (e) return hipfail(c, (hipError_t)e, "bucket launch");
    return ORL_OK;
}

// ---- device memory helpers for callers without a GPU runtime ----------------------------------------
int orl_device_alloc(orl_ctx* c, size_t bytes, void** out) {
    if (!c || !out) return ORL_E_INVALID;
    *out = nullptr;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    hipError_t e = hipMalloc(out, std::max<size_t>(bytes, 1));
    if (e != hipSuccess) return fail(c, ORL_E_NOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
    return ORL_OK;
}

int orl_device_free(orl_ctx* c, void* p) {
    if (!c) return ORL_E_INVALID;
    if (!p) return ORL_OK;
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    ORL_HIP(c, hipFree(p));
    return ORL_OK;
}

int orl_copy_to_device(orl_ctx* c, void* d_dst, const void* h_src, size_t bytes, void* stream) {
    if (!c || (bytes && (!d_dst || !h_src))) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    if (bytes) ORL_HIP(c, hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, stream ? (hipStream_t)stream : c->stream));
    return ORL_OK;
}

int orl_copy_to_host(orl_ctx* c, void* h_dst, const void* d_src, size_t bytes, void* stream) {
    if (!c || (bytes && (!h_dst || !d_src))) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    if (bytes) ORL_HIP(c, hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, stream ? (hipStream_t)stream : c->stream));
    return ORL_OK;
}

int orl_copy_on_device(orl_ctx* c, void* d_dst, const void* d_src, size_t bytes, void* stream) {
    if (!c || (bytes && (!d_dst || !d_src))) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    if (bytes) ORL_HIP(c, hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, stream ? (hipStream_t)stream : c->stream));
    return ORL_OK;
}

int orl_stream_sync(orl_ctx* c, void* stream) {
    if (!c) return ORL_E_INVALID;
    if (!c->device_mode) return ORL_OK;
    ORL_HIP(c, hipStreamSynchronize(stream ? (hipStream_t)stream : c->stream));
    return ORL_OK;
}

int orl_host_register(orl_ctx* c, void* p, size_t bytes) {
    if (!c || !p || !bytes) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    ORL_HIP(c, hipHostRegister(p, bytes, hipHostRegisterDefault));
    return ORL_OK;
}

int orl_host_unregister(orl_ctx* c, void* p) {
    if (!c || !p) return ORL_E_INVALID;
    ORL_HIP(c, hipHostUnregister(p));
    return ORL_OK;
}

// ---- follower graph + host-array fan-out ------------------------------------------------------------
int orl_csr_set(orl_ctx* c, const uint64_t* off, size_t n_nodes, const uint32_t* tgt, size_t n_edges) {
    if (!c || !off || (n_edges && !tgt)) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    if (off[0] != 0 || off[n_nodes] != n_edges) return fail(c, ORL_E_INVALID, "csr_off must start at 0 and end at n_edges");
    for (size_t i = 0; i < n_nodes; ++i)
        if (off[i + 1] < off[i]) return fail(c, ORL_E_INVALID, "csr_off not monotone at %zu", i);
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    ORL_HIP(c, hipDeviceSynchronize());  // a previous fan-out may still read the old graph
    (void)hipFree(c->d_csr_off); (void)hipFree(c->d_csr_tgt);
    c->d_csr_off = nullptr; c->d_csr_tgt = nullptr; c->csr_nodes = 0;
    ORL_HIP(c, hipMalloc((void**)&c->d_csr_off, (n_nodes + 1) * 8));
    ORL_HIP(c, hipMalloc((void**)&c->d_csr_tgt, std::max<size_t>(n_edges, 1) * 4));
    ORL_HIP(c, hipMemcpy(c->d_csr_off, off, (n_nodes + 1) * 8, hipMemcpyHostToDevice));
    if (n_edges) ORL_HIP(c, hipMemcpy(c->d_csr_tgt, tgt, n_edges * 4, hipMemcpyHostToDevice));
    c->csr_nodes = n_nodes;
    c->h_csr_off.assign(off, off + n_nodes + 1);
    return ORL_OK;
}

int orl_fanout_batch(orl_ctx* c, const uint32_t* pubs, const uint8_t* pub_silo, size_t n_pub, uint64_t follower_tcd,
                     uint32_t opts, uint64_t* pub_offsets, uint32_t* route, uint32_t* act, uint32_t* order, uint32_t* offsets,
                     size_t cap, uint64_t* n_out) {
    if (!c || !n_out || !pub_offsets) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "context was created without a device (device < 0)");
    if (!c->d_csr_off) return fail(c, ORL_E_STATE, "no follower graph (orl_csr_set)");
    const bool buckets = !(opts & ORL_OPT_NO_BUCKETS);
    if (n_pub && (!pubs || !pub_silo)) return fail(c, ORL_E_INVALID, "null publisher array");
    if (!route || !act || (buckets && (!order || !offsets))) return fail(c, ORL_E_INVALID, "null output array");
    // the emitted total from the host copy of the offsets: no device round trip before the launch
    uint64_t total = 0;
    for (size_t p = 0; p < n_pub; ++p) {
        if (pubs[p] >= c->csr_nodes) return fail(c, ORL_E_INVALID, "publisher %u >= %zu nodes", pubs[p], c->csr_nodes);
        total += c->h_csr_off[pubs[p] + 1] - c->h_csr_off[pubs[p]];
    }
    *n_out = total;
    if (total > cap) return fail(c, ORL_E_CAPACITY, "fan-out emits %llu > cap %zu", (unsigned long long)total, cap);
    if (total > c->s.max_batch || n_pub + 1 > c->s.max_batch) return fail(c, ORL_E_CAPACITY, "fan-out larger than max_batch");
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    const size_t in_bytes = n_pub * 5 + 16, out_words = 3 * std::max<uint64_t>(total, 1) + 1 + 2 * (n_pub + 1);
    if (int r = ensure_staging(c, in_bytes, out_words)) return r;
    uint32_t* d_pubs = reinterpret_cast<uint32_t*>(c->st_in);
    uint8_t* d_psilo = c->st_in + ((n_pub * 4 + 15) & ~size_t(15));
    uint32_t* d_route = c->st_out;
    uint32_t* d_act = d_route + total;
    uint32_t* d_order = d_act + total;
    uint64_t* d_poff = reinterpret_cast<uint64_t*>(d_order + total + (total & 1));
    hipStream_t st = c->stream;
    if (n_pub) {
        ORL_HIP(c, hipMemcpyAsync(d_pubs, pubs, n_pub * 4, hipMemcpyHostToDevice, st));
        ORL_HIP(c, hipMemcpyAsync(d_psilo, pub_silo, n_pub, hipMemcpyHostToDevice, st));
    }
    uint64_t n_dev = total;
    int r = orl_fanout_route_device(c, c->d_csr_off, c->d_csr_tgt, d_pubs, d_psilo, n_pub, follower_tcd, opts | ORL_OPT_TOTAL_GIVEN,
                                    d_poff, d_route, d_act, d_order, c->st_off, &n_dev, st);
    if (r) return r;
    if (total) {
        ORL_HIP(c, hipMemcpyAsync(route, d_route, total * 4, hipMemcpyDeviceToHost, st));
        ORL_HIP(c, hipMemcpyAsync(act, d_act, total * 4, hipMemcpyDeviceToHost, st));
        if (buckets) ORL_HIP(c, hipMemcpyAsync(order, d_order, total * 4, hipMemcpyDeviceToHost, st));
    }
    ORL_HIP(c, hipMemcpyAsync(pub_offsets, d_poff, (n_pub + 1) * 8, hipMemcpyDeviceToHost, st));
    if (buckets) ORL_HIP(c, hipMemcpyAsync(offsets, c->st_off, ((size_t)c->cfg.n_act + 2) * 4, hipMemcpyDeviceToHost, st));
    ORL_HIP(c, hipStreamSynchronize(st));
    return ORL_OK;
}

int orl_ctx_query(orl_ctx* c, uint32_t what, uint64_t* v) {
    if (!c || !v) return ORL_E_INVALID;
    switch (what) {
        case ORL_Q_DEVICE: *v = (uint64_t)(int64_t)c->cfg.device; return ORL_OK;
        case ORL_Q_N_ACT: *v = c->cfg.n_act; return ORL_OK;
        case ORL_Q_MAX_BATCH: *v = c->s.max_batch; return ORL_OK;
        case ORL_Q_WIRE_DIGEST: *v = c->hp.wire_digest; return ORL_OK;  // host state: set by orl_wire_types_set
        case ORL_Q_RANK_MODE: {
            if (!c->device_mode) return fail(c, ORL_E_STATE, "no device");
            std::lock_guard<std::mutex> lk(g_rank_mu);
            *v = (uint64_t)(int64_t)g_rank_state[c->cfg.device];
            return ORL_OK;
        }
        case ORL_Q_HOT_BATCHES:
            *v = c->s.hot_batches;
            return ORL_OK;
        case ORL_Q_HOT_KEY: {  // stage 4's hot key for the next batch (synchronises the device)
            if (!c->device_mode) return fail(c, ORL_E_STATE, "no device");
            ORL_HIP(c, hipSetDevice(c->cfg.device));
            ORL_HIP(c, hipDeviceSynchronize());
            uint32_t w = 0;
            ORL_HIP(c, hipMemcpy(&w, c->s.hot + (c->s.hot_parity & 1u), 4, hipMemcpyDeviceToHost));
            *v = w;
            return ORL_OK;
        }
        case ORL_Q_PART_ERROR: {  // the look-back state sets' error words (state[1]), read and cleared
            if (!c->device_mode) return fail(c, ORL_E_STATE, "no device");
            ORL_HIP(c, hipSetDevice(c->cfg.device));
            ORL_HIP(c, hipDeviceSynchronize());
            uint32_t any = 0;
            for (auto& L : c->s.lb) {
                uint32_t w = 0;
                ORL_HIP(c, hipMemcpy(&w, L.state + 1, 4, hipMemcpyDeviceToHost));
                if (w) ORL_HIP(c, hipMemset(L.state + 1, 0, 4));
                any |= w;
            }
            *v = any ? 1u : 0u;
            return ORL_OK;
        }
        case ORL_Q_STAGE4_ERROR: {  // stage 4's look-back error word (s4_err), read and cleared
            if (!c->device_mode) return fail(c, ORL_E_STATE, "no device");
            ORL_HIP(c, hipSetDevice(c->cfg.device));
            ORL_HIP(c, hipDeviceSynchronize());
            uint32_t w = 0;
            ORL_HIP(c, hipMemcpy(&w, c->s.s4_err, 4, hipMemcpyDeviceToHost));
            if (w) ORL_HIP(c, hipMemset(c->s.s4_err, 0, 4));
            *v = w ? 1u : 0u;
            return ORL_OK;
        }
        default: break;
    }
    if (int r = sync_device_state(c)) return r;
    switch (what) {
        case ORL_Q_PROBE_FORM:
            *v = c->probe8_valid ? 8 : c->probe_valid ? 16 : (c->probe_dev || c->probe_dev_stale) ? 17 : 32;
            return ORL_OK;
        case ORL_Q_FULL_UPLOADS: *v = c->n_full_uploads; return ORL_OK;
        case ORL_Q_SLOT_PATCHES: *v = c->n_patches; return ORL_OK;
        default: return fail(c, ORL_E_INVALID, "unknown query %u", what);
    }
}

int orl_ctx_set_rank_mode(orl_ctx* c, uint32_t mode) {
    if (!c || mode > 1) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "no device");
    std::lock_guard<std::mutex> lk(g_rank_mu);
    const int st = g_rank_state[c->cfg.device];
    if (mode == 0 && (st & 2)) return fail(c, ORL_E_STATE, "the LDS lane-order self-check failed on this device: ballot ranking only");
    ORL_HIP(c, hipSetDevice(c->cfg.device));
    ORL_HIP(c, hipDeviceSynchronize());  // kernels in flight keep the mode they started with
    ORL_HIP(c, (hipError_t)set_rank_mode(c->cfg.device, mode));
    g_rank_state[c->cfg.device] = (int)(mode | (st & 2));
    return ORL_OK;
}

int orl_set_timing(orl_ctx* c, int enable) {
    if (!c) return ORL_E_INVALID;
    if (!c->device_mode) return fail(c, ORL_E_STATE, "no device");
    if (enable && c->tev.empty()) {
        c->tev.assign(4 * (size_t)ORL_TIMING_SLOTS, nullptr);
        for (auto& e : c->tev) ORL_HIP(c, hipEventCreate(&e));
    }
    c->timing = enable != 0;
    c->tcount = 0;
    return ORL_OK;
}

int orl_timing_summary(const orl_ctx* cc, uint32_t* n_batches, float* route_ms, float* bucket_ms, float* total_ms) {
    orl_ctx* c = const_cast<orl_ctx*>(cc);
    if (!c) return ORL_E_INVALID;
    if (n_batches) *n_batches = c->tcount;
    if (c->tcount == 0) return fail(c, ORL_E_STATE, "no timed batch");
    ORL_HIP(c, hipEventSynchronize(c->tev[4 * (size_t)(c->tcount - 1) + 3]));
    double a = 0, b = 0, t = 0;
    for (uint32_t i = 0; i < c->tcount; ++i) {
        const hipEvent_t* ev = &c->tev[4 * (size_t)i];
        float x = 0, y = 0, z = 0;
        ORL_HIP(c, hipEventElapsedTime(&x, ev[1], ev[2]));
        ORL_HIP(c, hipEventElapsedTime(&y, ev[2], ev[3]));
        ORL_HIP(c, hipEventElapsedTime(&z, ev[0], ev[3]));
        a += x; b += y; t += z;
    }
    if (route_ms) *route_ms = (float)(a / c->tcount);
    if (bucket_ms) *bucket_ms = (float)(b / c->tcount);
    if (total_ms) *total_ms = (float)(t / c->tcount);
    return ORL_OK;
}

}  // extern "C"
