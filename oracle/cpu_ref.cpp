// cpu_ref.cpp — CPU restatement of the Orleans 1.1 per-message routing path.
//
// TEST INFRASTRUCTURE ONLY.  This is the parity oracle and the CPU baseline ("kind": "port") for
// bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it
// (oracle/liborleans_cpu_ref.so via ctypes).  The product (orleans_amd/, liborleans_route.so) never
// links or calls it.
//
// It restates the reference the way the silo executes it, one message at a time (paths relative to the
// randa1/orleans checkout):
//   * JenkinsHash.ComputeHash(ulong,ulong,ulong)  src/Orleans/IDs/JenkinsHash.cs:54-65,126-144
//   * JenkinsHash.ComputeHash(byte[])             src/Orleans/IDs/JenkinsHash.cs:68-115
//   * UniqueKey.GetUniformHashCode                src/Orleans/IDs/UniqueKey.cs:280-305
//   * LocalGrainDirectory.AddServer               src/OrleansRuntime/GrainDirectory/LocalGrainDirectory.cs:243-268
//   * LocalGrainDirectory.CalculateTargetSilo     ...LocalGrainDirectory.cs:439-497 (linear FindLast, as written)
//   * GrainDirectoryPartition.AddSingleActivation / LookUpGrain + IsValidSilo
//                                                 src/OrleansRuntime/GrainDirectory/GrainDirectoryPartition.cs:100-114,270-287,326-344
//   * Dispatcher.AddressMessage / SelectOrAddActivation / PreferLocal placement
//                                                 src/OrleansRuntime/Core/Dispatcher.cs:555-579,
//                                                 src/OrleansRuntime/Placement/PlacementDirectorsManager.cs:70-91,
//                                                 src/OrleansRuntime/Placement/PreferLocalPlacementDirector.cs:38-44
//   * ActivationData.EnqueueMessage FIFO          src/OrleansRuntime/Catalog/ActivationData.cs:483-514
//   * ChirperAccount.PublishMessage fan-out loop  Samples/Chirper/ChirperGrains/ChirperAccount.cs:154-157
// The directory partition is a std::unordered_map keyed by the GrainId with GetHashCode() = the
// uniform hash (GrainId.cs:196-199 → UniqueKey.GetHashCode), like the reference's Dictionary<GrainId,…>.
//
// The reference is C#/.NET and cannot be built or run here; this restatement is checked against an
// independent Python restatement (oracle/pyref.py) and the golden fixtures in tests/golden/.
// PARITY UNPINNED beyond the reference's own property test (Identifiertests.cs:284-301, byte-path
// Jenkins == u64-path Jenkins) and its shipped Chirper graph: ring ownership, directory lookup,
// placement, bucketing and fan-out have no reference golden vector.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

// JenkinsHash.Mix (JenkinsHash.cs:54-65)
inline void mix(uint32_t& a, uint32_t& b, uint32_t& c) {
    a -= b; a -= c; a ^= (c >> 13);
    b -= c; b -= a; b ^= (a << 8);
    c -= a; c -= b; c ^= (b >> 13);
    a -= b; a -= c; a ^= (c >> 12);
    b -= c; b -= a; b ^= (a << 16);
    c -= a; c -= b; c ^= (b >> 5);
    a -= b; a -= c; a ^= (c >> 3);
    b -= c; b -= a; b ^= (a << 10);
    c -= a; c -= b; c ^= (b >> 15);
}

// JenkinsHash.ComputeHash(ulong u1, ulong u2, ulong u3) (:126-144)
uint32_t hash3(uint64_t u1, uint64_t u2, uint64_t u3) {
    uint32_t a = 0x9e3779b9u, b = a, c = 0;
    a += (uint32_t)u1;
    b += (uint32_t)((u1 ^ (uint32_t)u1) >> 32);
    c += (uint32_t)u2;
    mix(a, b, c);
    a += (uint32_t)((u2 ^ (uint32_t)u2) >> 32);
    b += (uint32_t)u3;
    c += (uint32_t)((u3 ^ (uint32_t)u3) >> 32);
    mix(a, b, c);
    c += 24;
    mix(a, b, c);
    return c;
}

// JenkinsHash.ComputeHash(byte[]) (:68-115): the byte-by-byte reference form.
uint32_t hash_bytes(const uint8_t* data, size_t len) {
    uint32_t a = 0x9e3779b9u, b = a, c = 0;
    size_t i = 0;
    auto le32 = [&](size_t k) {
        return (uint32_t)data[k] | ((uint32_t)data[k + 1] << 8) | ((uint32_t)data[k + 2] << 16) | ((uint32_t)data[k + 3] << 24);
    };
    while (i + 12 <= len) {
        a += le32(i);
        b += le32(i + 4);
        c += le32(i + 8);
        i += 12;
        mix(a, b, c);
    }
    c += (uint32_t)len;
    if (i < len) a += data[i++];
    if (i < len) a += (uint32_t)data[i++] << 8;
    if (i < len) a += (uint32_t)data[i++] << 16;
    if (i < len) a += (uint32_t)data[i++] << 24;
    if (i < len) b += data[i++];
    if (i < len) b += (uint32_t)data[i++] << 8;
    if (i < len) b += (uint32_t)data[i++] << 16;
    if (i < len) b += (uint32_t)data[i++] << 24;
    if (i < len) c += (uint32_t)data[i++] << 8;
    if (i < len) c += (uint32_t)data[i++] << 16;
    if (i < len) c += (uint32_t)data[i++] << 24;
    mix(a, b, c);
    return c;
}

struct Key {
    uint64_t tcd, n0, n1;
    bool operator==(const Key& o) const { return tcd == o.tcd && n0 == o.n0 && n1 == o.n1; }
};
struct KeyHash {
    size_t operator()(const Key& k) const { return hash3(k.tcd, k.n0, k.n1); }  // GrainId.GetHashCode
};
struct Entry {
    uint32_t act;
    uint8_t silo;
};
using Partition = std::unordered_map<Key, Entry, KeyHash>;

}  // namespace

extern "C" {

// Must match include/orleans_route.h's orl_msg_hdr byte-for-byte (the oracle reads the same inputs).
struct ref_msg {
    uint64_t tcd, n0, n1;
    uint8_t sending_silo, category, flags, target_silo;
    uint32_t aux;
};

// Cluster view the routing decision depends on.
struct ref_cluster {
    uint32_t n_silos;
    uint32_t ring_n;
    int32_t ring_hash[256];   // membershipRingList order (as built by ref_ring_add)
    uint8_t ring_silo[256];
    uint8_t running[256];
    uint8_t functional[256];
    uint8_t local[256];
    uint32_t seed;            // 0xFF = none
    uint32_t policy;          // 0 prefer-local, 1 hash-spread
};

static const uint64_t kMemTcd = 2ull << 56;  // SystemGrain category, type 0
static const uint64_t kMemN0 = 0x11E0C21E01145FECull;  // Guid 01145FEC-C21E-11E0-9105-D0FB4724019B LE
static const uint64_t kMemN1 = 0x9B012447FBD00591ull;

uint32_t ref_jenkins_u64(uint64_t u1, uint64_t u2, uint64_t u3) { return hash3(u1, u2, u3); }
uint32_t ref_jenkins_bytes(const uint8_t* d, size_t n) { return hash_bytes(d, n); }

// LocalGrainDirectory.AddServer (:243-268)
int ref_ring_add(ref_cluster* cl, uint32_t silo, int32_t hash) {
    for (uint32_t i = 0; i < cl->ring_n; ++i)
        if (cl->ring_silo[i] == silo) return 0;
    if (cl->ring_n >= 256) return -1;
    int index = -1;  // FindLastIndex(s => s.hash < hash)
    for (uint32_t i = 0; i < cl->ring_n; ++i)
        if ((int64_t)cl->ring_hash[i] < (int64_t)hash) index = (int)i;
    const int at = index + 1;
    for (int i = (int)cl->ring_n; i > at; --i) {
        cl->ring_hash[i] = cl->ring_hash[i - 1];
        cl->ring_silo[i] = cl->ring_silo[i - 1];
    }
    cl->ring_hash[at] = hash;
    cl->ring_silo[at] = (uint8_t)silo;
    ++cl->ring_n;
    return 0;
}

// LocalGrainDirectory.RemoveServer list part (:270-304)
int ref_ring_remove(ref_cluster* cl, uint32_t silo) {
    uint32_t w = 0;
    for (uint32_t i = 0; i < cl->ring_n; ++i)
        if (cl->ring_silo[i] != silo) { cl->ring_hash[w] = cl->ring_hash[i]; cl->ring_silo[w] = cl->ring_silo[i]; ++w; }
    cl->ring_n = w;
    return 0;
}

// CalculateTargetSilo (:439-497).  Returns silo, 0xFF = null, 0xFE = no seed (ArgumentException).
static uint32_t calc_target_silo(const ref_cluster* cl, const Key& k, uint32_t uniform, uint32_t me, bool exclude_if_stopping) {
    if ((k.tcd >> 56) == 1) return me;  // grain.IsSystemTarget
    if (k.tcd == kMemTcd && k.n0 == kMemN0 && k.n1 == kMemN1) return cl->seed == 0xFF ? 0xFE : cl->seed;
    const int hash = (int)uniform;
    const bool running = cl->running[me] != 0;
    if (cl->ring_n == 0) return (exclude_if_stopping && !running) ? 0xFF : me;
    const bool excludeMySelf = !running && exclude_if_stopping;
    int found = -1;  // membershipRingList.FindLast(pred): scan the whole list, keep the last match
    for (uint32_t i = 0; i < cl->ring_n; ++i)
        if (cl->ring_hash[i] <= hash && (cl->ring_silo[i] != me || !excludeMySelf)) found = (int)i;
    if (found < 0) {
        uint32_t s = cl->ring_silo[cl->ring_n - 1];
        if (s == me && excludeMySelf) {
            if (cl->ring_n > 1) s = cl->ring_silo[cl->ring_n - 2]; else return 0xFF;
        }
        return s;
    }
    return cl->ring_silo[found];
}

void* ref_dir_new(void) { return new Partition(); }
void ref_dir_free(void* d) { delete static_cast<Partition*>(d); }
uint64_t ref_dir_size(void* d) { return static_cast<Partition*>(d)->size(); }

// RegisterSingleActivationAsync (LocalGrainDirectory.cs:510-544) on the activation's silo:
// owner = CalculateTargetSilo(grain) (exclude = true); owner local → AddSingleActivation (null if
// !IsValidSilo, first writer wins); status codes = ORL_INS_*.
int ref_register(const ref_cluster* cl, void* dir, const Key* keys, const uint32_t* acts, const uint8_t* silos, size_t n,
                 uint8_t* status, uint32_t* wact, uint8_t* wsilo) {
    Partition& p = *static_cast<Partition*>(dir);
    for (size_t i = 0; i < n; ++i) {
        const Key& k = keys[i];
        const uint32_t cat = (uint32_t)(k.tcd >> 56);
        uint8_t st;
        uint32_t a = 0xFFFFFFFFu;
        uint8_t s = 0xFF;
        if (cat == 6 || cat == 1) {
            st = 5;
        } else {
            const uint32_t owner = calc_target_silo(cl, k, hash3(k.tcd, k.n0, k.n1), silos[i], true);
            if (owner == 0xFF || owner == 0xFE) st = 4;
            else if (!cl->local[owner]) st = 3;
            else if (!cl->functional[silos[i]]) st = 2;
            else {
                auto it = p.find(k);
                if (it != p.end()) { st = 1; a = it->second.act; s = it->second.silo; }
                else { p.emplace(k, Entry{acts[i], silos[i]}); st = 0; a = acts[i]; s = silos[i]; }
            }
        }
        if (status) status[i] = st;
        if (wact) wact[i] = a;
        if (wsilo) wsilo[i] = s;
    }
    return 0;
}

int ref_unregister(void* dir, const Key* keys, size_t n, uint8_t* removed) {
    Partition& p = *static_cast<Partition*>(dir);
    for (size_t i = 0; i < n; ++i) {
        const size_t r = p.erase(keys[i]);
        if (removed) removed[i] = r ? 1 : 0;
    }
    return 0;
}

static inline uint32_t pack(uint32_t owner, uint32_t host, uint32_t st, uint32_t fl) {
    return (owner & 0xFF) | ((host & 0xFF) << 8) | ((st & 0xFF) << 16) | ((fl & 0xFF) << 24);
}

// Dispatcher.AddressMessage for one message (see header comment for the chain).
static uint32_t route_one(const ref_cluster* cl, const Partition& p, const ref_msg& m, bool excl, uint32_t* act) {
    *act = 0xFFFFFFFFu;
    const uint32_t me = m.sending_silo;
    if (m.flags & 1) return pack(0xFF, m.target_silo, 3, m.target_silo == me ? 2 : 0);  // IsComplete
    const Key k{m.tcd, m.n0, m.n1};
    const uint32_t cat = (uint32_t)(m.tcd >> 56);
    const uint32_t h = (m.flags & 2) ? m.aux : hash3(k.tcd, k.n0, k.n1);
    const uint32_t owner = calc_target_silo(cl, k, h, me, excl);
    if (owner == 0xFE) return pack(0xFF, 0xFF, 5, 0);
    if (owner == 0xFF) return pack(0xFF, 0xFF, 4, 0);
    if (cat == 1) return pack(owner, me, 2, 2);
    uint32_t fl = (k.tcd == kMemTcd && k.n0 == kMemN0 && k.n1 == kMemN1) ? 4u : 0u;
    if (cat == 6) return pack(owner, 0xFF, 7, fl);
    if (!cl->local[owner]) return pack(owner, 0xFF, 8, fl);
    auto it = p.find(k);  // LookUpGrain + IsValidSilo filter
    if (it != p.end() && cl->functional[it->second.silo]) {
        *act = it->second.act;
        return pack(owner, it->second.silo, 0, fl | (it->second.silo == me ? 2u : 0u));
    }
    if (cat == 4) return pack(owner, 0xFF, 6, fl);  // unregistered client
    uint32_t host = me;                           // PreferLocal
    if (cl->policy == 1) {                        // hash-spread stand-in for random placement
        uint32_t na = 0;
        for (uint32_t s = 0; s < cl->n_silos; ++s) na += cl->functional[s] ? 1 : 0;
        if (na == 0) host = 0xFF;
        else {
            uint32_t want = h % na, seen = 0;
            for (uint32_t s = 0; s < cl->n_silos; ++s)
                if (cl->functional[s]) { if (seen == want) { host = s; break; } ++seen; }
        }
    }
    return pack(owner, host, 1, fl | 1u | (host == me ? 2u : 0u));
}

int ref_route(const ref_cluster* cl, void* dir, const ref_msg* in, size_t n, uint32_t opts, uint32_t* route, uint32_t* act) {
    const Partition& p = *static_cast<Partition*>(dir);
    for (size_t i = 0; i < n; ++i) route[i] = route_one(cl, p, in[i], (opts & 1) != 0, &act[i]);
    return 0;
}

// Stable per-activation FIFO (ActivationData.EnqueueMessage): append each message to its activation's
// queue in arrival order, then lay the queues out back to back.  Bucket n_act collects every message
// without a resident activation.
int ref_bucket(const uint32_t* act, size_t n, uint32_t n_act, uint32_t* order, uint32_t* offsets) {
    std::vector<std::vector<uint32_t>> q((size_t)n_act + 1);
    for (size_t i = 0; i < n; ++i) q[act[i] < n_act ? act[i] : n_act].push_back((uint32_t)i);
    size_t pos = 0;
    for (size_t b = 0; b <= n_act; ++b) {
        offsets[b] = (uint32_t)pos;
        for (uint32_t m : q[b]) order[pos++] = m;
    }
    offsets[(size_t)n_act + 1] = (uint32_t)pos;
    return 0;
}

// The same pipeline on T host threads, for the CPU baseline: contiguous message ranges per thread
// (routing is read-only on the partition), then a stable counting sort whose per-thread histograms are
// concatenated in thread order, so the per-activation FIFO order is identical to ref_bucket's.
int ref_route_bucket_mt(const ref_cluster* cl, void* dir, const ref_msg* in, size_t n, uint32_t opts, uint32_t n_act,
                        uint32_t* route, uint32_t* act, uint32_t* order, uint32_t* offsets, int nthreads) {
    // Same outputs as ref_route_bucket (a stable counting sort by key = min(act, n_act)), computed in parallel as a
    // stable MSD split by the key's high bits followed by a counting sort of each high bucket by the low bits (one
    // thread per bucket), so the working set per thread is 2^HB + 2^(bits-HB) counters, not n_act.
    if (nthreads < 1) nthreads = 1;
    const Partition& p = *static_cast<Partition*>(dir);
    const size_t nb = (size_t)n_act + 1;  // keys 0 .. n_act
    uint32_t bits = 1;
    while (((size_t)1 << bits) < nb) ++bits;
    const uint32_t hb = bits < 12 ? bits : 12, sh = bits - hb;
    const size_t nhi = (size_t)1 << hb;
    std::vector<std::vector<uint32_t>> hist(nthreads, std::vector<uint32_t>(nhi, 0));
    auto range = [&](int t, size_t& lo, size_t& hi) { lo = n * t / nthreads; hi = n * (t + 1) / nthreads; };
    auto key_of = [&](size_t i) { return act[i] < n_act ? act[i] : n_act; };
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([&, t] {
            size_t lo, hi;
            range(t, lo, hi);
            auto& h = hist[t];
            for (size_t i = lo; i < hi; ++i) {
                route[i] = route_one(cl, p, in[i], (opts & 1) != 0, &act[i]);
                ++h[key_of(i) >> sh];
            }
        });
    for (auto& x : th) x.join();
    th.clear();
    // high-bucket-major, thread-minor exclusive scan: stable split
    std::vector<size_t> bstart(nhi + 1);
    size_t run = 0;
    for (size_t b = 0; b < nhi; ++b) {
        bstart[b] = run;
        for (int t = 0; t < nthreads; ++t) {
            const uint32_t c = hist[t][b];
            hist[t][b] = (uint32_t)run;
            run += c;
        }
    }
    bstart[nhi] = run;
    std::vector<uint32_t> tkey(n), tidx(n);
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([&, t] {
            size_t lo, hi;
            range(t, lo, hi);
            auto& h = hist[t];
            for (size_t i = lo; i < hi; ++i) {
                const uint32_t k = key_of(i);
                const uint32_t pos = h[k >> sh]++;
                tkey[pos] = k;
                tidx[pos] = (uint32_t)i;
            }
        });
    for (auto& x : th) x.join();
    th.clear();
    // each high bucket: stable counting sort by the low bits; writes its keys' offsets and its part of `order`
    std::atomic<size_t> next{0};
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([&] {
            std::vector<uint32_t> cnt((size_t)1 << sh);
            for (size_t b; (b = next.fetch_add(1)) < nhi;) {
                const size_t k0 = b << sh;
                if (k0 >= nb) continue;
                const size_t k1 = std::min(nb, (b + 1) << sh);
                std::fill(cnt.begin(), cnt.end(), 0u);
                for (size_t j = bstart[b]; j < bstart[b + 1]; ++j) ++cnt[tkey[j] - k0];
                uint32_t r = (uint32_t)bstart[b];
                for (size_t k = k0; k < k1; ++k) {
                    const uint32_t c = cnt[k - k0];
                    offsets[k] = r;
                    cnt[k - k0] = r;
                    r += c;
                }
                for (size_t j = bstart[b]; j < bstart[b + 1]; ++j) order[cnt[tkey[j] - k0]++] = tidx[j];
            }
        });
    for (auto& x : th) x.join();
    offsets[nb] = (uint32_t)n;
    return 0;
}

// Fan-out (ChirperAccount.PublishMessage :154-157): publish p expands to one message per follower in CSR
// order, follower grain = (follower_tcd, 0, id), sent from pub_silo[p].
size_t ref_fanout_expand(const uint64_t* csr_off, const uint32_t* csr_tgt, const uint32_t* pubs, const uint8_t* pub_silo,
                         size_t n_pub, uint64_t follower_tcd, ref_msg* out, size_t cap, uint64_t* pub_offsets) {
    size_t k = 0;
    for (size_t p = 0; p < n_pub; ++p) {
        if (pub_offsets) pub_offsets[p] = k;
        const uint32_t s = pubs[p];
        for (uint64_t e = csr_off[s]; e < csr_off[s + 1]; ++e) {
            if (out && k < cap) {
                ref_msg& m = out[k];
                std::memset(&m, 0, sizeof m);
                m.tcd = follower_tcd;
                m.n0 = 0;
                m.n1 = csr_tgt[e];
                m.sending_silo = pub_silo[p];
                m.category = 2;
            }
            ++k;
        }
    }
    if (pub_offsets) pub_offsets[n_pub] = k;
    return k;
}

// Destination rank of each message for the multi-GPU exchange: directory owner's rank, or my_rank for
// messages that are not directory-routed.  Stable partition order = rank-major, arrival order inside.
int ref_partition(const ref_cluster* cl, const ref_msg* in, size_t n, uint32_t opts, const uint8_t* rank_of_silo,
                  uint32_t nranks, uint32_t my_rank, uint32_t* src_index, uint64_t* counts) {
    std::vector<std::vector<uint32_t>> q(nranks);
    for (size_t i = 0; i < n; ++i) {
        const ref_msg& m = in[i];
        uint32_t d = my_rank;
        if (!(m.flags & 1) && (m.tcd >> 56) != 1) {
            const Key k{m.tcd, m.n0, m.n1};
            const uint32_t h = (m.flags & 2) ? m.aux : hash3(k.tcd, k.n0, k.n1);
            const uint32_t owner = calc_target_silo(cl, k, h, m.sending_silo, (opts & 1) != 0);
            if (owner < 0xFE) d = rank_of_silo[owner];
        }
        q[d].push_back((uint32_t)i);
    }
    size_t pos = 0;
    for (uint32_t r = 0; r < nranks; ++r) {
        counts[r] = q[r].size();
        for (uint32_t i : q[r]) src_index[pos++] = i;
    }
    return 0;
}

}  // extern "C"
