// orl_node.cpp — the silos of one GPU in a multi-GPU node: the two-hop message exchange behind the C ABI
// (SURVEY §8(b) "node-level orl_node_create", §8(e)).  Reference: OutboundMessageQueue.SendMessage's per-target-silo
// sender queues (src/OrleansRuntime/Messaging/OutboundMessageQueue.cs:113-145), the remote directory lookup
// (LocalGrainDirectory.FullLookup, LocalGrainDirectory.cs:719-765) and Dispatcher.TransportMessage (Dispatcher.cs:618-622).
//
// Per batch, every rank in lockstep (include/orleans_route.h documents the contract):
//   hop 1   per chunk: one-pass owner partition (k_part_lb) on stream P → all-gather of the per-rank counts (the host
//           needs them to size the sends) → grouped send/recv on stream X → stages 1-3 of the received chunk on stream R,
//           overlapping the next chunk's exchange;
//   hop 2   host-rank counts of the routed messages (k_host_rank_count) → all-gather → if any rank forwards: stable
//           partition of {record, route, act} by host rank (k_part_routed) → grouped send/recv;
//   host    stage 4 over the hosted messages (orl_bucket_device).
// Transports: RCCL (one process per GPU; xGMI) and LOCAL (ranks = nodes of one process, device copies + host barriers),
// the latter a one-GPU rehearsal of the exact protocol for the parity tests.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "orl_internal.h"

using namespace orl;

namespace {

constexpr uint32_t kHeadWords = ORL_NODE_HEAD_WORDS;  // layout: include/orleans_route.h (orl_node_plan_chunk)
static_assert(ORL_NODE_HEAD_WORDS == 16, "head words: counts [0, 8), status [8], form | digest [9], zero [10, 16)");
constexpr uint64_t kDigestMask = (1ull << 56) - 1;
constexpr uint32_t kDefaultTimeoutMs = 120000;  // every host wait of the exchange (orl_node_set_timeout)

// ORL_TRANSPORT_LOCAL: the ranks are node objects of one process.  All-gathers and exchanges are host barriers around
// published host words / device pointers; the data moves with device-to-device copies.
struct LocalGroup {
    uint32_t nranks = 0;
    std::mutex mu;
    std::condition_variable cv;
    uint32_t arrived = 0;
    uint64_t gen = 0;
    std::vector<std::vector<uint64_t>> words;  // per rank: its all-gather contribution
    struct Lane {
        const uint8_t* base;  // send regions of this rank: region for destination r at base + r * stride
        uint64_t stride;      // bytes
    };
    std::vector<std::vector<Lane>> lanes;      // per rank: the send regions of the current exchange
    bool broken = false;                       // a barrier timed out: the group is unusable (every barrier fails)
    // false on timeout (a rank stopped calling) or once the group is broken: the caller reports an error instead of
    // hanging.  A timeout breaks the group for every rank, so a late rank cannot pass a later barrier without the one
    // that gave up and read its stale words or freed buffers.
    bool barrier(uint32_t timeout_ms) {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return false;
        const uint64_t g = gen;
        if (++arrived == nranks) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        if (cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return gen != g || broken; }) && !broken) return true;
        broken = true;
        cv.notify_all();
        return false;
    }
};
std::mutex g_groups_mu;
std::map<std::string, std::weak_ptr<LocalGroup>> g_groups;

std::shared_ptr<LocalGroup> join_group(const uint8_t* id, uint32_t nranks) {
    std::lock_guard<std::mutex> lk(g_groups_mu);
    const std::string key(reinterpret_cast<const char*>(id), ORL_NODE_ID_BYTES);
    std::shared_ptr<LocalGroup> g = g_groups[key].lock();
    if (!g) {
        g = std::make_shared<LocalGroup>();
        g->nranks = nranks;
        g->words.assign(nranks, std::vector<uint64_t>(kHeadWords, 0));
        g->lanes.assign(nranks, {});
        g_groups[key] = g;
    }
    return g->nranks == nranks ? g : nullptr;
}

// One array moved by an exchange: rank me sends count[r] elements of `elem` bytes from send + r * stride to rank r and
// receives recv_count[r] elements from rank r, laid out back to back in source-rank order at recv.
struct Lane {
    const uint8_t* send;
    uint64_t stride;  // bytes between destination regions
    uint8_t* recv;
    uint32_t elem;
};

}  // namespace

struct orl_node {
    orl_ctx* ctx = nullptr;
    orl_node_config cfg{};
    std::string err;
    int device = 0;
    uint32_t timeout_ms = kDefaultTimeoutMs;
    bool broken = false;      // a bounded wait expired or RCCL failed: the communicator was aborted
    int stall_chunk = -1;     // ORL_NODE_INJECT_STALL: the all-gather of this chunk waits on h_stall (fault injection)
    uint32_t* h_stall = nullptr;  // pinned, device-visible release word of the injected stall
    int lb_fail = 0;          // ORL_NODE_INJECT_LB_FAIL: 1 = the hop-2 partition's, 2 = a re-partition's, 3 = stage 4's look-back "gives up"
    uint32_t n_act = 0, nr = 1, me = 0;
    uint64_t chunk_cap = 0;
    ncclComm_t comm = nullptr;
    ncclComm_t comm_h = nullptr;  // the counts all-gathers' communicator (ncclCommSplit of comm), on stream sh (round 4)
    std::shared_ptr<LocalGroup> group;
    hipStream_t sp = nullptr, sx = nullptr, sr = nullptr;
    hipStream_t sp1 = nullptr;  // hop-1 partitions alternate sp (even chunks) and sp1 (odd; round 6): a chunk's kernel tail
                                // overlaps the next chunk's start (each stream has its own look-back state in the context)
    hipStream_t sh = nullptr;  // the counts all-gathers: chunk c's runs while chunk c-1's data exchange is still on sx
    hipEvent_t ev_in = nullptr, ev_x = nullptr, ev_r = nullptr;
    hipEvent_t ev_h = nullptr;  // the hop-2 host-rank counts are written (on sh)
    hipEvent_t ev_s4 = nullptr; // the copy of the context's stage-4 error word after the last batch's stage 4 (on sr)
    uint32_t* h_s4err = nullptr;  // pinned: that copy (checked at the start of the next batch: ADVICE r5)
    bool s4_pending = false;
    hipEvent_t ev_part[2] = {nullptr, nullptr};  // the slot's partition (and heads) are complete
    hipEvent_t ev_slot[2] = {nullptr, nullptr};  // send slot released (its exchange finished)
    bool last_forward = false;  // the previous batch forwarded messages (hop 2): stage 4 then waits for the counts
    uint64_t form_word[2] = {0, 0};  // head word 9 of each send slot as last uploaded
    bool form_valid[2] = {false, false};
    uint8_t* d_ros = nullptr;
    uint8_t* d_send[2] = {nullptr, nullptr};      // hop-1 send regions: nranks x chunk_cap x 32 B per slot
    uint64_t* d_head = nullptr;                   // [2][kHeadWords]
    uint64_t* d_heads = nullptr;                  // [nranks][kHeadWords] (RCCL all-gather target)
    uint64_t* h_heads = nullptr;                  // pinned copy
    uint64_t* h_form = nullptr;                   // pinned [2]: head word 9 of each send slot (form | digest)
    uint8_t* d_recv = nullptr;                    // owned records, chunk after chunk (max_recv x 32 B)
    uint32_t* d_send_act[2] = {nullptr, nullptr}; // sender-cache act lane per send slot: nranks x chunk_cap (first cached batch)
    uint32_t* d_recv_act = nullptr;               // received act lane, max_recv (first chunk that carries one)
    uint32_t *d_route = nullptr, *d_act = nullptr, *d_order = nullptr, *d_off = nullptr;
    uint64_t* d_hcount = nullptr;                 // [8] hop-2 counts by host rank
    // hop 2 (allocated on first use)
    uint64_t f_cap = 0;
    uint8_t* d_fsend = nullptr;
    uint32_t *d_fsend_route = nullptr, *d_fsend_act = nullptr;
    uint8_t* d_frecv = nullptr;
    uint32_t *d_frecv_route = nullptr, *d_frecv_act = nullptr, *d_forder = nullptr, *d_foff = nullptr;
    uint32_t* d_fstate = nullptr;
    uint64_t* d_fcounts = nullptr;                // [ORL_NODE_MAX_CHUNKS][8] chained partition totals, then [1] u32 error word
    struct Seg {
        const void* p;
        uint64_t count;
        uint32_t width;
    };
    std::vector<Seg> segs;
    orl_msg_hdr* d_fan = nullptr;                 // expanded multicast records (orl_node_fanout_batch_device), max_batch
    // KeyExt strings of the current batch (orl_node_route_batch_keyext_device; null otherwise) and their hop-1 lanes
    const orl_ext_ref* kx_ext = nullptr;
    const uint8_t* kx_blob = nullptr;
    uint64_t kx_bytes = 0;
    orl_ext_ref* d_send_ext[2] = {nullptr, nullptr};  // nranks x chunk_cap references per slot
    uint8_t* d_send_blob[2] = {nullptr, nullptr};     // nranks x send_blob_cap bytes per slot
    uint64_t send_blob_cap = 0;
    orl_ext_ref* d_recv_ext = nullptr;                // max_recv references (the owned set's)
    uint8_t* d_recv_blob[2] = {nullptr, nullptr};     // a chunk's received strings, per slot
    uint64_t recv_blob_cap = 0;
    orl_node_stats stats{};                       // the last batch's bytes and host waits (orl_node_get_stats)
};

namespace {

int nfail(orl_node* nd, int code, const char* fmt, ...) {
    char b[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b, sizeof b, fmt, ap);
    va_end(ap);
    nd->err = b;
    return code;
}

#define NODE_HIP(nd, call)                                                                           \
    do {                                                                                             \
        hipError_t _e = (call);                                                                      \
        if (_e != hipSuccess) return nfail((nd), ORL_E_DEVICE, "%s: %s", #call, hipGetErrorString(_e)); \
    } while (0)
#define NODE_NCCL(nd, call)                                                                            \
    do {                                                                                               \
        ncclResult_t _r = (call);                                                                      \
        if (_r != ncclSuccess) return nfail((nd), ORL_E_DEVICE, "%s: %s", #call, ncclGetErrorString(_r)); \
    } while (0)
#define NODE_CTX(nd, call)                                                                              \
    do {                                                                                                \
        int _r = (call);                                                                                \
        if (_r != ORL_OK) return nfail((nd), _r, "%s: %s", #call, orl_last_error((nd)->ctx));           \
    } while (0)

// The communicator is unusable (a peer missed a deadline, RCCL reported an error, or this rank found a device fault its
// peers cannot see): abort it so RCCL kernels still waiting on peers exit (and the peers' own bounded waits see the
// error at once instead of at their deadline), break a LOCAL group the same way (every barrier of every rank fails),
// release an injected stall, and let the streams drain (bounded).  The node stays broken.
void break_node(orl_node* nd) {
    nd->broken = true;
    if (nd->comm_h) {
        (void)ncclCommAbort(nd->comm_h);
        nd->comm_h = nullptr;
    }
    if (nd->comm) {
        (void)ncclCommAbort(nd->comm);
        nd->comm = nullptr;
    }
    if (nd->group) {
        std::lock_guard<std::mutex> lk(nd->group->mu);
        nd->group->broken = true;
        nd->group->cv.notify_all();
    }
    if (nd->h_stall) __atomic_store_n(nd->h_stall, 1u, __ATOMIC_RELEASE);
}

// A host wait of the exchange, counted in the node's stats (orl_node_get_stats).
void count_wait(orl_node* nd, std::chrono::steady_clock::time_point t0) {
    nd->stats.host_wait_us += (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
    ++nd->stats.host_waits;
}

// A LOCAL-transport barrier, its wait counted in the node's stats.
bool timed_barrier(orl_node* nd, LocalGroup& g) {
    const auto t0 = std::chrono::steady_clock::now();
    const bool ok = g.barrier(nd->timeout_ms);
    count_wait(nd, t0);
    return ok;
}

// Bounded wait for stream `s` (instead of hipStreamSynchronize): polls the stream and, with RCCL, the communicator's
// asynchronous error; on an RCCL error or at the deadline the node is broken (break_node) and ORL_E_STATE returned with
// `what` and this rank's head words `d_own` (when the stream drained after the abort) in orl_node_last_error.
int wait_bounded(orl_node* nd, hipStream_t s, const char* what, int chunk, const uint64_t* d_own) {
    const auto t0 = std::chrono::steady_clock::now();
    const auto deadline = t0 + std::chrono::milliseconds(nd->timeout_ms);
    uint32_t polls = 0;
    ncclResult_t ar = ncclSuccess;
    for (;;) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) {
            count_wait(nd, t0);
            return ORL_OK;
        }
        if (q != hipErrorNotReady) return nfail(nd, ORL_E_DEVICE, "%s (chunk %d): %s", what, chunk, hipGetErrorString(q));
        ++polls;  // (both transports: the sleep backoff below applies to LOCAL rank threads too)
        if (nd->comm && (polls & 63u) == 0u) {
            if (ncclCommGetAsyncError(nd->comm, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress) break;
            if (nd->comm_h && ncclCommGetAsyncError(nd->comm_h, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress)
                break;
            ar = ncclSuccess;
        }
        if (std::chrono::steady_clock::now() > deadline) break;
        if (polls > 4096) std::this_thread::sleep_for(std::chrono::microseconds(50));
        else std::this_thread::yield();
    }
    break_node(nd);
    // the aborted communicator's kernels exit: give the stream a moment to drain before reading this rank's words
    const auto drain = std::chrono::steady_clock::now() + std::chrono::milliseconds(2000);
    bool drained = false;
    while (!(drained = hipStreamQuery(s) == hipSuccess) && std::chrono::steady_clock::now() < drain)
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    char words[256] = "unavailable (the stream did not drain)";
    uint64_t own[kHeadWords] = {};
    if (drained && d_own && hipMemcpy(own, d_own, sizeof own, hipMemcpyDeviceToHost) == hipSuccess) {
        int k = 0;
        for (uint32_t r = 0; r < nd->nr && k < (int)sizeof words - 24; ++r)
            k += snprintf(words + k, sizeof words - k, "%s%llu", r ? "," : "", (unsigned long long)own[r]);
        snprintf(words + k, sizeof words - k, " status %llu", (unsigned long long)own[8]);
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ar != ncclSuccess)
        return nfail(nd, ORL_E_STATE, "%s (chunk %d): RCCL error %s after %.0f ms; communicator aborted; rank %u head words %s",
                     what, chunk, ncclGetErrorString(ar), ms, nd->me, words);
    return nfail(nd, ORL_E_STATE, "%s (chunk %d): no completion within %u ms (a rank did not take part?); communicator aborted; "
                 "rank %u head words %s", what, chunk, nd->timeout_ms, nd->me, words);
}

// All-gather of kHeadWords u64 per rank from device `d_src` (ready once `ready` has fired) into nd->h_heads.
int allgather_heads(orl_node* nd, const uint64_t* d_src, hipEvent_t ready, int chunk) {
    // Stream sh (and with RCCL the split communicator comm_h): chunk c's counts travel while chunk c-1's data exchange
    // still runs on sx, instead of queueing behind it.  Without the split communicator (ncclCommSplit
    // failed) the all-gathers share comm and sx, as before.
    const bool split = nd->sh && (!nd->comm || nd->comm_h);
    hipStream_t hs = split ? nd->sh : nd->sx;
    NODE_HIP(nd, hipStreamWaitEvent(hs, ready, 0));
    if (nd->comm) {
        NODE_NCCL(nd, ncclAllGather(d_src, nd->d_heads, kHeadWords, ncclUint64, split ? nd->comm_h : nd->comm, hs));
        NODE_HIP(nd, hipMemcpyAsync(nd->h_heads, nd->d_heads, (size_t)nd->nr * kHeadWords * 8, hipMemcpyDeviceToHost, hs));
        if (chunk == nd->stall_chunk && nd->h_stall) {
            int e = launch_node_stall(nd->h_stall, hs);
            if (e) return nfail(nd, ORL_E_DEVICE, "stall injection: %s", hipGetErrorString((hipError_t)e));
        }
        return wait_bounded(nd, hs, chunk >= 0 ? "node counts all-gather" : "node hop-2 counts all-gather", chunk, d_src);
    }
    LocalGroup& g = *nd->group;
    NODE_HIP(nd, hipMemcpyAsync(nd->h_heads + (size_t)nd->me * kHeadWords, d_src, kHeadWords * 8, hipMemcpyDeviceToHost, hs));
    if (chunk == nd->stall_chunk && nd->h_stall) {
        int e = launch_node_stall(nd->h_stall, hs);
        if (e) return nfail(nd, ORL_E_DEVICE, "stall injection: %s", hipGetErrorString((hipError_t)e));
    }
    if (int r = wait_bounded(nd, hs, "node all-gather", chunk, d_src)) return r;
    {
        std::lock_guard<std::mutex> lk(g.mu);
        std::memcpy(g.words[nd->me].data(), nd->h_heads + (size_t)nd->me * kHeadWords, kHeadWords * 8);
    }
    if (!timed_barrier(nd, g)) {
        nd->broken = true;
        return nfail(nd, ORL_E_STATE, "node all-gather (chunk %d): a rank did not arrive within %u ms (barrier timeout)", chunk,
                     nd->timeout_ms);
    }
    {
        std::lock_guard<std::mutex> lk(g.mu);
        for (uint32_t r = 0; r < nd->nr; ++r) std::memcpy(nd->h_heads + (size_t)r * kHeadWords, g.words[r].data(), kHeadWords * 8);
    }
    if (!timed_barrier(nd, g)) {
        nd->broken = true;
        return nfail(nd, ORL_E_STATE, "node all-gather (chunk %d): a rank did not arrive within %u ms (barrier timeout)", chunk,
                     nd->timeout_ms);
    }
    return ORL_OK;
}

// Grouped send/recv of `lanes` (enqueued on nd->sx after `ready`); send[r] / recv[r] are element counts.
int exchange(orl_node* nd, const std::vector<Lane>& lanes, const uint64_t* send, const uint64_t* recv, hipEvent_t ready) {
    NODE_HIP(nd, hipStreamWaitEvent(nd->sx, ready, 0));
    const uint32_t nr = nd->nr, me = nd->me;
    std::vector<uint64_t> roff(nr + 1, 0);
    for (uint32_t r = 0; r < nr; ++r) roff[r + 1] = roff[r] + recv[r];
    for (const Lane& L : lanes)
        for (uint32_t r = 0; r < nr; ++r) nd->stats.bytes_sent[r] += send[r] * L.elem;
    if (nd->comm) {
        NODE_NCCL(nd, ncclGroupStart());
        for (const Lane& L : lanes)
            for (uint32_t r = 0; r < nr; ++r) {
                if (r == me) {
                    if (send[r])
                        NODE_HIP(nd, hipMemcpyAsync(L.recv + roff[r] * L.elem, L.send + r * L.stride, send[r] * L.elem,
                                                    hipMemcpyDeviceToDevice, nd->sx));
                    continue;
                }
                if (send[r]) NODE_NCCL(nd, ncclSend(L.send + r * L.stride, send[r] * L.elem, ncclUint8, (int)r, nd->comm, nd->sx));
                if (recv[r]) NODE_NCCL(nd, ncclRecv(L.recv + roff[r] * L.elem, recv[r] * L.elem, ncclUint8, (int)r, nd->comm, nd->sx));
            }
        NODE_NCCL(nd, ncclGroupEnd());
        return ORL_OK;
    }
    LocalGroup& g = *nd->group;
    if (int r = wait_bounded(nd, nd->sx, "node exchange: send regions", -1, nullptr)) return r;  // my send regions are complete
    {
        std::lock_guard<std::mutex> lk(g.mu);
        g.lanes[me].clear();
        for (const Lane& L : lanes) g.lanes[me].push_back(LocalGroup::Lane{L.send, L.stride});
    }
    if (!timed_barrier(nd, g)) {
        nd->broken = true;
        return nfail(nd, ORL_E_STATE, "node exchange: a rank did not arrive within %u ms (barrier timeout)", nd->timeout_ms);
    }
    std::vector<std::vector<LocalGroup::Lane>> peers;
    {
        std::lock_guard<std::mutex> lk(g.mu);
        peers = g.lanes;
    }
    for (size_t k = 0; k < lanes.size(); ++k)
        for (uint32_t r = 0; r < nr; ++r)
            if (recv[r]) {
                if (peers[r].size() != lanes.size()) return nfail(nd, ORL_E_STATE, "node exchange: ranks disagree on the lanes");
                NODE_HIP(nd, hipMemcpyAsync(lanes[k].recv + roff[r] * lanes[k].elem, peers[r][k].base + me * peers[r][k].stride,
                                            recv[r] * lanes[k].elem, hipMemcpyDeviceToDevice, nd->sx));
            }
    if (int r = wait_bounded(nd, nd->sx, "node exchange: copies", -1, nullptr)) return r;
    if (!timed_barrier(nd, g)) {  // every rank has copied out of my regions: they are free
        nd->broken = true;
        return nfail(nd, ORL_E_STATE, "node exchange: a rank did not arrive within %u ms (barrier timeout)", nd->timeout_ms);
    }
    return ORL_OK;
}

void free_node(orl_node* nd) {
    auto f = [](void* p) { if (p) (void)hipFree(p); };
    f(nd->d_ros); f(nd->d_send[0]); f(nd->d_send[1]); f(nd->d_head); f(nd->d_heads); f(nd->d_recv); f(nd->d_route); f(nd->d_act);
    f(nd->d_order); f(nd->d_off); f(nd->d_hcount); f(nd->d_fsend); f(nd->d_fsend_route); f(nd->d_fsend_act); f(nd->d_frecv);
    f(nd->d_frecv_route); f(nd->d_frecv_act); f(nd->d_forder); f(nd->d_foff); f(nd->d_fstate); f(nd->d_fcounts); f(nd->d_fan);
    f(nd->d_send_act[0]); f(nd->d_send_act[1]); f(nd->d_recv_act);
    if (nd->h_heads) (void)hipHostFree(nd->h_heads);
    if (nd->h_form) (void)hipHostFree(nd->h_form);
    if (nd->h_stall) (void)hipHostFree(nd->h_stall);
    if (nd->h_s4err) (void)hipHostFree(nd->h_s4err);
    for (int sl = 0; sl < 2; ++sl) {
        (void)hipFree(nd->d_send_ext[sl]);
        (void)hipFree(nd->d_send_blob[sl]);
        (void)hipFree(nd->d_recv_blob[sl]);
    }
    (void)hipFree(nd->d_recv_ext);
    for (hipEvent_t e : {nd->ev_in, nd->ev_part[0], nd->ev_part[1], nd->ev_x, nd->ev_r, nd->ev_h, nd->ev_slot[0], nd->ev_slot[1], nd->ev_s4})
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t s : {nd->sp, nd->sp1, nd->sx, nd->sr, nd->sh})
        if (s) (void)hipStreamDestroy(s);
    if (nd->comm_h) (void)ncclCommDestroy(nd->comm_h);
    nd->comm_h = nullptr;
    if (nd->comm) (void)ncclCommDestroy(nd->comm);
    nd->comm = nullptr;
}

// Hop-2 buffers for an owned set of up to `owned` messages (regions of that stride), grown on demand.
int ensure_hop2(orl_node* nd, uint64_t owned) {
    if (owned <= nd->f_cap && nd->d_frecv) return ORL_OK;
    NODE_HIP(nd, hipDeviceSynchronize());
    const uint64_t cap = std::max<uint64_t>(owned, 1) + (std::max<uint64_t>(owned, 1) >> 3);
    auto f = [](void*& p) { if (p) (void)hipFree(p); p = nullptr; };
    f(reinterpret_cast<void*&>(nd->d_fsend)); f(reinterpret_cast<void*&>(nd->d_fsend_route));
    f(reinterpret_cast<void*&>(nd->d_fsend_act)); f(reinterpret_cast<void*&>(nd->d_fstate));
    nd->f_cap = 0;
    NODE_HIP(nd, hipMalloc((void**)&nd->d_fsend, (size_t)nd->nr * cap * 32));
    NODE_HIP(nd, hipMalloc((void**)&nd->d_fsend_route, (size_t)nd->nr * cap * 4));
    NODE_HIP(nd, hipMalloc((void**)&nd->d_fsend_act, (size_t)nd->nr * cap * 4));
    NODE_HIP(nd, hipMalloc((void**)&nd->d_fstate, part_state_bytes(cap)));
    if (!nd->d_frecv) {
        const uint64_t m = nd->cfg.max_recv;
        NODE_HIP(nd, hipMalloc((void**)&nd->d_frecv, m * 32));
        NODE_HIP(nd, hipMalloc((void**)&nd->d_frecv_route, m * 4));
        NODE_HIP(nd, hipMalloc((void**)&nd->d_frecv_act, m * 4));
        NODE_HIP(nd, hipMalloc((void**)&nd->d_forder, m * 4));
        NODE_HIP(nd, hipMalloc((void**)&nd->d_foff, ((size_t)nd->n_act + 2) * 4));
        NODE_HIP(nd, hipMalloc((void**)&nd->d_fcounts, ORL_NODE_MAX_CHUNKS * 8 * 8 + 8));
    }
    nd->f_cap = cap;
    return ORL_OK;
}


// One u32 per rank summed over comm (on sx, bounded wait): the node's collective yes/no decisions at creation.
int allreduce_u32_sum(orl_node* nd, uint32_t v, uint32_t* sum) {
    uint32_t* d = reinterpret_cast<uint32_t*>(nd->d_hcount);  // scratch: the hop-2 counts are not in use yet
    NODE_HIP(nd, hipMemcpyAsync(d, &v, 4, hipMemcpyHostToDevice, nd->sx));
    NODE_NCCL(nd, ncclAllReduce(d, d + 1, 1, ncclUint32, ncclSum, nd->comm, nd->sx));
    if (int r = wait_bounded(nd, nd->sx, "node creation all-reduce", -3, nullptr)) return r;
    NODE_HIP(nd, hipMemcpy(sum, d + 1, 4, hipMemcpyDeviceToHost));
    NODE_HIP(nd, hipMemsetAsync(d, 0, 8, nd->sx));
    return wait_bounded(nd, nd->sx, "node creation all-reduce", -3, nullptr);
}

// The optional second communicator of the counts all-gathers (ORL_NODE_SPLIT_COMM): all ranks or none.
int setup_split_comm(orl_node* nd, bool want) {
    uint32_t n_want = 0;
    if (int r = allreduce_u32_sum(nd, want ? 1u : 0u, &n_want)) return r;
    if (n_want != 0 && n_want != nd->nr)
        return nfail(nd, ORL_E_INVALID, "ORL_NODE_SPLIT_COMM set on %u of %u ranks (every rank must use the same config)",
                     n_want, nd->nr);
    if (!n_want) return ORL_OK;
    if (ncclCommSplit(nd->comm, 0, (int)nd->me, &nd->comm_h, nullptr) != ncclSuccess) nd->comm_h = nullptr;
    uint32_t n_ok = 0;
    if (int r = allreduce_u32_sum(nd, nd->comm_h ? 1u : 0u, &n_ok)) return r;
    if (n_ok != nd->nr && nd->comm_h) {  // some rank's split failed: nobody uses the split communicator
        (void)ncclCommDestroy(nd->comm_h);
        nd->comm_h = nullptr;
    }
    return ORL_OK;
}

}  // namespace

extern "C" {

// The protocol's host decisions.  Every rank evaluates them on the same all-gathered words, so every rank reaches the
// same width, the same sizes and the same errors without another round trip.
int orl_node_plan_chunk(const uint64_t* H, uint32_t nr, uint32_t me, uint32_t written, uint64_t max_recv, uint64_t* owned_total,
                        orl_node_chunk_plan* out) {
    if (!H || !owned_total || !out || nr == 0 || nr > ORL_NODE_MAX_RANKS || me >= nr) return ORL_E_INVALID;
    if (written != 8 && written != 16 && written != 32) return ORL_E_INVALID;
    const uint64_t W = kHeadWords;
    std::memset(out, 0, sizeof *out);
    for (uint32_t r = 0; r < nr; ++r)
        if ((uint32_t)H[r * W + 8] & ORL_PART_LOOKBACK_FAILED) return ORL_E_DEVICE;
    // 8-B when every rank wrote that form with one wire-type digest and no message lacked it, 16-B when no message lacked
    // that, else 32-B headers (a rank that wrote 32-B, ORL_NODE_WIDE_ONLY, makes the chunk 32-B)
    bool all8 = true, no16 = false, no8 = false, wide = false;
    for (uint32_t r = 0; r < nr; ++r) {
        const uint32_t st = (uint32_t)H[r * W + 8];
        const uint32_t f = (uint32_t)(H[r * W + 9] >> 56);
        no16 |= (st & 1u) != 0;
        no8 |= (st & 2u) != 0;
        wide |= f == 32u;
        all8 &= f == 8u && (H[r * W + 9] & kDigestMask) == (H[0 * W + 9] & kDigestMask);
    }
    out->width = (wide || no16) ? 32u : (all8 && !no8) ? 8u : 16u;
    out->rewrite = out->width != written;
    bool ext_full = false;
    for (uint32_t r = 0; r < nr; ++r) {  // some sender addressed records from its directory cache: their handles travel too
        out->act_lane |= ((uint32_t)H[r * W + 8] & ORL_PART_CACHED) ? 1u : 0u;
        out->ext_lane |= ((uint32_t)H[r * W + 8] & ORL_PART_KEYEXT) ? 1u : 0u;  // ... KeyExt strings: their lanes travel
        ext_full |= ((uint32_t)H[r * W + 8] & ORL_PART_EXT_FULL) != 0;
    }
    for (uint32_t r = 0; r < nr; ++r) {
        out->send[r] = H[me * W + r];
        out->recv[r] = H[r * W + me];
        out->n_recv += out->recv[r];
    }
    int rc = ORL_OK;
    for (uint32_t d = 0; d < nr; ++d) {  // every rank checks every rank: all return the same error, none waits
        uint64_t in = 0;
        for (uint32_t s = 0; s < nr; ++s) in += H[s * W + d];
        owned_total[d] += in;
        if (owned_total[d] > max_recv) rc = ORL_E_CAPACITY;
    }
    if (ext_full) rc = ORL_E_CAPACITY;  // a sender's string region overflowed (every rank sees its status word)
    return rc;
}

int orl_node_plan_hop2(const uint64_t* H, uint32_t nr, uint32_t me, uint64_t n_owned, uint32_t width_mask, uint64_t max_recv,
                       orl_node_hop2_plan* out) {
    if (!H || !out || nr == 0 || nr > ORL_NODE_MAX_RANKS || me >= nr || width_mask > 7) return ORL_E_INVALID;
    const uint64_t W = kHeadWords;
    std::memset(out, 0, sizeof *out);
    for (uint32_t s = 0; s < nr; ++s)
        for (uint32_t d = 0; d < nr; ++d)
            if (s != d && H[s * W + d]) {
                out->forward = 1;
                if (s == me) out->n_forwarded += H[s * W + d];
            }
    // one record width for a forwarded set: the common width of the owned segments, or 32-B headers for a mix
    const bool w8 = width_mask & 1u, w16 = width_mask & 2u, w32 = width_mask & 4u;
    out->width = (w32 || (w8 && w16)) ? 32u : w16 ? 16u : 8u;
    if (!out->forward) {
        out->n_hosted = n_owned;
        return ORL_OK;
    }
    int rc = ORL_OK;
    for (uint32_t d = 0; d < nr; ++d) {
        uint64_t in = 0;
        for (uint32_t s = 0; s < nr; ++s) in += H[s * W + d];
        if (in > max_recv) rc = ORL_E_CAPACITY;
        if (d == me) out->n_hosted = in;
    }
    for (uint32_t r = 0; r < nr; ++r) {
        out->send[r] = H[me * W + r];
        out->recv[r] = H[r * W + me];
    }
    return rc;
}

int orl_node_unique_id(uint8_t id[ORL_NODE_ID_BYTES]) {
    if (!id) return ORL_E_INVALID;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return ORL_E_DEVICE;
    std::memcpy(id, u.internal, ORL_NODE_ID_BYTES);
    return ORL_OK;
}

const char* orl_node_last_error(const orl_node* nd) { return nd ? nd->err.c_str() : "null node"; }

int orl_node_set_timeout(orl_node* nd, uint32_t ms) {
    if (!nd || ms == 0) return ORL_E_INVALID;
    nd->timeout_ms = ms;
    return ORL_OK;
}

int orl_node_create(orl_ctx* ctx, const orl_node_config* cfg, orl_node** out) {
    if (!ctx || !cfg || !out) return ORL_E_INVALID;
    *out = nullptr;
    if (cfg->abi_version != ORL_ABI_VERSION) return ORL_E_INVALID;
    if (cfg->nranks == 0 || cfg->nranks > ORL_NODE_MAX_RANKS || cfg->rank >= cfg->nranks) return ORL_E_INVALID;
    if (cfg->transport > ORL_TRANSPORT_LOCAL || cfg->chunks == 0 || cfg->chunks > ORL_NODE_MAX_CHUNKS) return ORL_E_INVALID;
    if (cfg->max_batch == 0 || cfg->max_recv == 0 || cfg->max_recv >= (1ull << 31)) return ORL_E_INVALID;
    for (uint32_t s = 0; s < 256; ++s)
        if (cfg->rank_of_silo[s] >= cfg->nranks) return ORL_E_INVALID;
    uint64_t dev = 0, n_act = 0, mb = 0;
    if (orl_ctx_query(ctx, ORL_Q_DEVICE, &dev) || orl_ctx_query(ctx, ORL_Q_N_ACT, &n_act) ||
        orl_ctx_query(ctx, ORL_Q_MAX_BATCH, &mb))
        return ORL_E_INVALID;
    if ((int64_t)dev < 0) return ORL_E_STATE;
    orl_node* nd = new (std::nothrow) orl_node();
    if (!nd) return ORL_E_NOMEM;
    nd->ctx = ctx;
    nd->cfg = *cfg;
    nd->device = (int)(int64_t)dev;
    nd->n_act = (uint32_t)n_act;
    nd->nr = cfg->nranks;
    nd->me = cfg->rank;
    nd->chunk_cap = (cfg->max_batch + cfg->chunks - 1) / cfg->chunks;
    auto bail = [&](int code) {
        free_node(nd);
        delete nd;
        return code;
    };
    // the routing context routes one chunk's received records and buckets the owned / hosted set
    if (mb < std::max<uint64_t>(nd->chunk_cap, cfg->max_recv)) return bail(ORL_E_CAPACITY);
    if (hipSetDevice(nd->device) != hipSuccess) return bail(ORL_E_DEVICE);
    hipError_t e = hipSuccess;
    auto ok = [&](hipError_t x) { if (x != hipSuccess && e == hipSuccess) e = x; return x == hipSuccess; };
    ok(hipStreamCreateWithFlags(&nd->sp, hipStreamNonBlocking));
    ok(hipStreamCreateWithFlags(&nd->sp1, hipStreamNonBlocking));
    ok(hipStreamCreateWithFlags(&nd->sx, hipStreamNonBlocking));
    ok(hipStreamCreateWithFlags(&nd->sr, hipStreamNonBlocking));
    ok(hipStreamCreateWithFlags(&nd->sh, hipStreamNonBlocking));
    for (hipEvent_t* ev : {&nd->ev_in, &nd->ev_part[0], &nd->ev_part[1], &nd->ev_x, &nd->ev_r, &nd->ev_h, &nd->ev_slot[0], &nd->ev_slot[1],
                           &nd->ev_s4})
        ok(hipEventCreateWithFlags(ev, hipEventDisableTiming));
    const uint64_t nr = cfg->nranks, mr = cfg->max_recv;
    ok(hipMalloc((void**)&nd->d_ros, 256));
    ok(hipMemcpy(nd->d_ros, cfg->rank_of_silo, 256, hipMemcpyHostToDevice));
    for (int s = 0; s < 2; ++s) ok(hipMalloc((void**)&nd->d_send[s], nr * nd->chunk_cap * 32));
    ok(hipMalloc((void**)&nd->d_head, 2 * kHeadWords * 8));
    ok(hipMalloc((void**)&nd->d_heads, nr * kHeadWords * 8));
    ok(hipHostMalloc((void**)&nd->h_heads, nr * kHeadWords * 8, hipHostMallocDefault));
    ok(hipHostMalloc((void**)&nd->h_form, 2 * 8, hipHostMallocDefault));
    ok(hipHostMalloc((void**)&nd->h_s4err, 8, hipHostMallocDefault));
    ok(hipMalloc((void**)&nd->d_recv, mr * 32));
    ok(hipMalloc((void**)&nd->d_route, mr * 4));
    ok(hipMalloc((void**)&nd->d_act, mr * 4));
    ok(hipMalloc((void**)&nd->d_order, mr * 4));
    ok(hipMalloc((void**)&nd->d_off, ((size_t)nd->n_act + 2) * 4));
    ok(hipMalloc((void**)&nd->d_hcount, 16 * 8));
    if (e != hipSuccess) return bail(ORL_E_NOMEM);
    // head words no call writes (counts past nranks, [10, 16)) travel with the all-gathers: keep them zero
    ok(hipMemset(nd->d_head, 0, 2 * kHeadWords * 8));
    ok(hipMemset(nd->d_hcount, 0, 16 * 8));
    if (e != hipSuccess) return bail(ORL_E_DEVICE);
    for (hipEvent_t ev : {nd->ev_slot[0], nd->ev_slot[1]}) (void)hipEventRecord(ev, nd->sx);  // both slots free
    if (const char* t = getenv("ORL_NODE_TIMEOUT_MS")) {
        const long v = atol(t);
        if (v > 0) nd->timeout_ms = (uint32_t)std::min<long>(v, 0x7FFFFFFF);
    }
    if (const char* lf = getenv("ORL_NODE_INJECT_LB_FAIL"))  // fault injection on this rank only: "hop2", "rewrite", "stage4"
        nd->lb_fail = std::strcmp(lf, "hop2") == 0 ? 1 : std::strcmp(lf, "rewrite") == 0 ? 2 : std::strcmp(lf, "stage4") == 0 ? 3 : 0;
    if (const char* st = getenv("ORL_NODE_INJECT_STALL")) {  // fault injection: "<chunk>" (hop 1) or "hop2"
        nd->stall_chunk = std::strcmp(st, "hop2") == 0 ? -2 : atoi(st);
        if (!ok(hipHostMalloc((void**)&nd->h_stall, 64, hipHostMallocMapped | hipHostMallocCoherent))) return bail(ORL_E_NOMEM);
        *nd->h_stall = 0;
    }
    if (cfg->transport == ORL_TRANSPORT_RCCL) {
        ncclUniqueId u;
        std::memcpy(u.internal, cfg->group_id, ORL_NODE_ID_BYTES);
        if (ncclCommInitRank(&nd->comm, (int)nr, u, (int)cfg->rank) != ncclSuccess) {
            nd->comm = nullptr;
            return bail(ORL_E_DEVICE);
        }
        int cc = 0;
        nd->stats.comm_count = ncclCommCount(nd->comm, &cc) == ncclSuccess ? (uint32_t)cc : 0u;
        // The counts all-gathers' own communicator is opt-in (ORL_NODE_SPLIT_COMM): by default the
        // all-gathers share comm and the exchange stream sx, so no two RCCL kernels of this rank ever wait on peers at the
        // same time.  Both decisions are collective: the request is all-reduced first (ranks that disagree
        // fail creation together instead of one rank entering ncclCommSplit alone), then the split's success, so either
        // every rank uses comm_h or none does.
        if (int r = setup_split_comm(nd, (cfg->flags & ORL_NODE_SPLIT_COMM) != 0)) return bail(r);
    } else {
        nd->group = join_group(cfg->group_id, cfg->nranks);
        if (!nd->group) return bail(ORL_E_INVALID);
        nd->stats.comm_count = nd->group->nranks;
    }
    *out = nd;
    return ORL_OK;
}

int orl_node_destroy(orl_node* nd) {
    if (!nd) return ORL_E_INVALID;
    (void)hipSetDevice(nd->device);
    (void)hipDeviceSynchronize();
    free_node(nd);
    delete nd;
    return ORL_OK;
}

int orl_node_fanout_batch_device(orl_node* nd, const uint64_t* d_csr_off, const uint32_t* d_csr_tgt,
                                 const orl_grain_key* d_follower_keys, uint64_t follower_tcd, const uint32_t* d_pubs,
                                 const uint8_t* d_pub_silo, size_t n_pub, uint32_t opts, uint64_t* d_pub_offsets,
                                 uint64_t* total, orl_node_result* res, void* stream) {
    if (!nd || !res || !total) return ORL_E_INVALID;
    NODE_HIP(nd, hipSetDevice(nd->device));
    if (!nd->d_fan) NODE_HIP(nd, hipMalloc((void**)&nd->d_fan, nd->cfg.max_batch * sizeof(orl_msg_hdr)));
    NODE_CTX(nd, orl_fanout_expand_device(nd->ctx, d_csr_off, d_csr_tgt, d_follower_keys, follower_tcd, d_pubs, d_pub_silo, n_pub,
                                          opts & ORL_OPT_TOTAL_GIVEN, d_pub_offsets, nd->d_fan, nd->cfg.max_batch, total, stream));
    return orl_node_route_batch_device(nd, nd->d_fan, *total, opts & ~ORL_OPT_TOTAL_GIVEN, res, stream);
}

int orl_node_segment(const orl_node* nd, uint32_t i, const void** d_records, uint64_t* count, uint32_t* width) {
    if (!nd || i >= nd->segs.size()) return ORL_E_INVALID;
    if (d_records) *d_records = nd->segs[i].p;
    if (count) *count = nd->segs[i].count;
    if (width) *width = nd->segs[i].width;
    return ORL_OK;
}

int orl_node_get_stats(const orl_node* nd, orl_node_stats* out) {
    if (!nd || !out) return ORL_E_INVALID;
    *out = nd->stats;
    return ORL_OK;
}

int orl_node_route_batch_device(orl_node* nd, const orl_msg_hdr* d_in, size_t n, uint32_t opts, orl_node_result* res,
                                void* stream) {
    if (!nd || !res) return ORL_E_INVALID;
    {
        const uint32_t cc = nd->stats.comm_count;
        nd->stats = orl_node_stats{};
        nd->stats.comm_count = cc;
        nd->stats.exchange_mode = (nd->comm_h ? ORL_NODE_MODE_SPLIT_COMM : 0u) |
                                  (nd->sh && (!nd->comm || nd->comm_h) ? ORL_NODE_MODE_HEAD_STREAM : 0u);
        nd->stats.chunks = nd->cfg.chunks;
    }
    if (nd->broken) return nfail(nd, ORL_E_STATE, "node is broken (an earlier exchange failed; its communicator was aborted): %s",
                                 nd->err.c_str());
    if (n && !d_in) return nfail(nd, ORL_E_INVALID, "null device buffer");
    if (n > nd->cfg.max_batch) return nfail(nd, ORL_E_CAPACITY, "batch %zu > max_batch %llu", n, (unsigned long long)nd->cfg.max_batch);
    std::memset(res, 0, sizeof *res);
    if (nd->s4_pending) {  // the previous batch's stage 4 (its look-back error word, copied after it on sr)
        NODE_HIP(nd, hipSetDevice(nd->device));
        NODE_HIP(nd, hipEventSynchronize(nd->ev_s4));
        nd->s4_pending = false;
        if (*nd->h_s4err || nd->lb_fail == 3) {  // a device fault, on this rank only: its hosted order / offsets were not valid
            *nd->h_s4err = 0;
            uint64_t w = 0;
            (void)orl_ctx_query(nd->ctx, ORL_Q_STAGE4_ERROR, &w);  // reads and clears the device word
            break_node(nd);
            return nfail(nd, ORL_E_DEVICE, "the previous batch's stage 4 look-back gave up (device fault): its order / offsets "
                                           "were not valid; communicator aborted");
        }
    }
    const uint32_t nr = nd->nr, me = nd->me, K = nd->cfg.chunks;
    const uint64_t W = kHeadWords;
    const uint32_t ropts = (opts & ORL_OPT_EXCLUDE_IF_STOPPING) | ORL_OPT_NO_BUCKETS;
    hipStream_t caller = (hipStream_t)stream;
    NODE_HIP(nd, hipSetDevice(nd->device));
    NODE_HIP(nd, hipEventRecord(nd->ev_in, caller));  // the caller's batch is ready
    NODE_HIP(nd, hipStreamWaitEvent(nd->sp, nd->ev_in, 0));
    NODE_HIP(nd, hipStreamWaitEvent(nd->sp1, nd->ev_in, 0));
    auto pstream = [&](uint32_t slot) { return slot ? nd->sp1 : nd->sp; };  // chunk c's partition stream (slot c & 1)
    nd->segs.clear();
    const uint64_t cs = (n + K - 1) / K;
    uint64_t owned = 0;                       // messages received so far (this rank)
    uint64_t owned_bytes = 0;
    std::vector<uint64_t> owned_all(nr, 0);   // every rank's running receive total (capacity checks agree)
    uint64_t sent_remote = 0;
    uint32_t width_mask = 0;                  // record widths among the owned segments: bit 0 = 8, 1 = 16, 2 = 32
    // ---- hop 1 -------------------------------------------------------------------------------------------
    // Record form per chunk: every rank first writes the narrowest form it can (8-B when its context has wire types,
    // else 16-B; 32-B with ORL_NODE_WIDE_ONLY) and reports it with its wire-type digest in head word 9.  After the counts
    // all-gather every rank derives the same final form: 8-B when all ranks wrote it with one digest and no message
    // lacked it, 16-B when no message lacked that, else 32-B; a rank whose records differ re-partitions the chunk (the
    // counts do not depend on the form).
    uint64_t digest = 0;
    NODE_CTX(nd, orl_ctx_query(nd->ctx, ORL_Q_WIRE_DIGEST, &digest));
    const bool wide_only = (nd->cfg.flags & ORL_NODE_WIDE_ONLY) != 0;
    // KeyExt strings (round 6): a batch that carries them (orl_node_route_batch_keyext_device) is
    // exchanged as 32-B records with an ext-ref lane and a string lane beside them; the owner resolves the KeyExt messages
    // in its KeyExt table (a changed table is uploaded here, before anything of the batch runs, on every rank: another
    // rank's strings may arrive even when this rank sends none)
    const bool kx = nd->kx_ext != nullptr;
    NODE_CTX(nd, ctx_keyext_prepare(nd->ctx));
    const uint32_t first_form = (wide_only || kx) ? 32u : (digest ? 8u : 16u);
    if (kx) {
        const uint64_t cap = std::max<uint64_t>((nd->kx_bytes + 255) & ~uint64_t(255), 4096);
        if (!nd->d_send_ext[0] || cap > nd->send_blob_cap) {
            NODE_HIP(nd, hipDeviceSynchronize());
            for (int sl = 0; sl < 2; ++sl) {
                if (!nd->d_send_ext[sl]) NODE_HIP(nd, hipMalloc((void**)&nd->d_send_ext[sl], (size_t)nr * nd->chunk_cap * 8));
                (void)hipFree(nd->d_send_blob[sl]);
                nd->d_send_blob[sl] = nullptr;
                NODE_HIP(nd, hipMalloc((void**)&nd->d_send_blob[sl], (size_t)nr * cap));
            }
            nd->send_blob_cap = cap;
        }
    }
    // The sender's directory cache (round 5): with the context's cache populated, hop 1 sends a message whose owner is
    // remote and whose grain the cache holds straight to the rank of the cached activation, addressed (HIT | CACHED), with
    // its handle in an act lane beside the records — LocalLookup's non-owner branch (LocalGrainDirectory.cs:690-717) before
    // the FullLookup this exchange replaces (:719-765).  The lane travels with a chunk only when some rank cached a message
    // of it (ORL_PART_CACHED in the all-gathered status words: every rank agrees).
    const bool cached = ctx_cache_on(nd->ctx);
    if (cached && !nd->d_send_act[0]) {
        NODE_HIP(nd, hipDeviceSynchronize());
        for (int sl = 0; sl < 2; ++sl)
            NODE_HIP(nd, hipMalloc((void**)&nd->d_send_act[sl], (size_t)nr * nd->chunk_cap * 4));
    }
    // Partition of chunk c into send slot c & 1 (after the slot's previous exchange): per-rank counts + wire status
    // in the slot's head words.  Chunk c + 1 is partitioned before the host waits for chunk c's counts, so the
    // partition stream does not idle through the all-gather round trip.
    auto partition = [&](uint32_t c, uint32_t form) -> int {
        const uint32_t slot = c & 1u;
        const uint64_t start = std::min<uint64_t>((uint64_t)c * cs, n), len = std::min<uint64_t>(cs, n - start);
        uint64_t* head = nd->d_head + slot * kHeadWords;
        uint8_t* send = nd->d_send[slot];
        uint32_t* status = reinterpret_cast<uint32_t*>(head + 8);
        hipStream_t ps = pstream(slot);
        NODE_HIP(nd, hipStreamWaitEvent(ps, nd->ev_slot[slot], 0));  // the slot's previous exchange has finished
        // head words: [0, nr) counts and [8] status are written by the partition call itself (the counts by its last tile,
        // or zeroed for an empty chunk); [9] (form | digest) is uploaded only when it changes, so a chunk costs the
        // partition kernel and its status reset (two head writes per chunk fewer: ~10 us of small stream ops each)
        const uint64_t fw = ((uint64_t)form << 56) | (digest & kDigestMask);
        if (!nd->form_valid[slot] || nd->form_word[slot] != fw) {
            // the slot's previous head copy was consumed before its all-gather returned, so the pinned word is free
            nd->h_form[slot] = fw;
            NODE_HIP(nd, hipMemcpyAsync(head + 9, nd->h_form + slot, 8, hipMemcpyHostToDevice, ps));
            nd->form_word[slot] = fw;
            nd->form_valid[slot] = true;
        }
        KxLanes kxl{};
        if (kx && form == 32) {  // head words [10, 14): the string bytes to each destination (u32 each), the append cursors
            NODE_HIP(nd, hipMemsetAsync(head + 10, 0, 4 * 8, ps));
            kxl = KxLanes{nd->kx_ext + start, nd->kx_blob, nd->kx_bytes, nd->d_send_ext[slot], nd->d_send_blob[slot],
                          nd->send_blob_cap, reinterpret_cast<uint32_t*>(head + 10)};
        }
        NODE_CTX(nd, ctx_partition_padded(nd->ctx, d_in + start, len, opts, nd->cfg.rank_of_silo, nr, me, nd->chunk_cap, send,
                                          (int)form, head, status, ps, cached ? nd->d_send_act[slot] : nullptr,
                                          kxl.ext ? &kxl : nullptr));
        NODE_HIP(nd, hipEventRecord(nd->ev_part[slot], ps));
        return ORL_OK;
    };
    if (K > 0)
        if (int r = partition(0, first_form)) return r;
    for (uint32_t c = 0; c < K; ++c) {
        const uint32_t slot = c & 1u;
        uint64_t* head = nd->d_head + slot * kHeadWords;
        uint8_t* send = nd->d_send[slot];
        if (c + 1 < K)
            if (int r = partition(c + 1, first_form)) return r;
        if (int r = allgather_heads(nd, head, nd->ev_part[slot], (int)c)) return r;
        const uint64_t* H = nd->h_heads;
        orl_node_chunk_plan plan;
        const int pr = orl_node_plan_chunk(H, nr, me, first_form, nd->cfg.max_recv, owned_all.data(), &plan);
        if (pr == ORL_E_DEVICE) {
            for (uint32_t r = 0; r < nr; ++r)  // every rank sees every rank's status: all fail together
                if ((uint32_t)H[r * W + 8] & ORL_PART_LOOKBACK_FAILED)
                    return nfail(nd, ORL_E_DEVICE, "chunk %u: rank %u's partition look-back gave up (device fault)", c, r);
        }
        if (pr == ORL_E_CAPACITY) {
            for (uint32_t d = 0; d < nr; ++d)
                if (owned_all[d] > nd->cfg.max_recv)
                    return nfail(nd, ORL_E_CAPACITY, "rank %u receives %llu > max_recv %llu messages", d,
                                 (unsigned long long)owned_all[d], (unsigned long long)nd->cfg.max_recv);
        }
        if (pr) return nfail(nd, pr, "chunk %u: node plan failed", c);
        const uint32_t width = plan.width;
        // The rewrite runs on chunk c's own partition stream, behind chunk c's first partition: the look-back state
        // (ticket counter, epoch-tagged granules) is per stream in the context, and stream order keeps each set
        // consistent; chunk c + 1's partition, on the other stream, has a set of its own (ADVICE r3's ordering concern).
        if (plan.rewrite) {  // some rank's records do not fit the form: every rank rewrites the chunk in `width`
            if (int r = partition(c, width)) return r;
            // the rewrite's look-back is checked on this rank only (its counts are those already all-gathered)
            uint32_t st = 0;
            if (int r = wait_bounded(nd, pstream(slot), "re-partition", (int)c, nullptr)) return r;
            NODE_HIP(nd, hipMemcpy(&st, head + 8, 4, hipMemcpyDeviceToHost));
            if (nd->lb_fail == 2) st |= ORL_PART_LOOKBACK_FAILED;
            if (st & ORL_PART_LOOKBACK_FAILED) {  // only this rank sees it: abort, so the peers fail now, not at their deadline
                break_node(nd);
                return nfail(nd, ORL_E_DEVICE, "chunk %u: the %u-byte re-partition's look-back gave up (device fault); "
                             "communicator aborted", c, width);
            }
        }
        width_mask |= width == 8 ? 1u : width == 16 ? 2u : 4u;
        const uint64_t got = plan.n_recv;
        for (uint32_t r = 0; r < nr; ++r)
            if (r != me) sent_remote += plan.send[r];
        // segments start 32-B aligned, whatever the widths before them (an odd count of 8-B records, then wider ones);
        // the padding fits max_recv x 32 B: a chunk of 8- or 16-B records never fills its 32-B share
        owned_bytes = (owned_bytes + 31) & ~uint64_t(31);
        uint8_t* recv = nd->d_recv + owned_bytes;
        std::vector<Lane> lanes = {Lane{send, nd->chunk_cap * width, recv, width}};
        if (plan.act_lane) {
            if (!nd->d_recv_act) NODE_HIP(nd, hipMalloc((void**)&nd->d_recv_act, nd->cfg.max_recv * 4));
            if (!nd->d_send_act[slot]) {  // a rank without a cache sends ORL_NO_ACT for every record
                NODE_HIP(nd, hipDeviceSynchronize());
                for (int sl = 0; sl < 2; ++sl)
                    NODE_HIP(nd, hipMalloc((void**)&nd->d_send_act[sl], (size_t)nr * nd->chunk_cap * 4));
            }
            if (!cached)  // this rank wrote no act lane: ORL_NO_ACT over what it sends
                for (uint32_t r = 0; r < nr; ++r)
                    if (plan.send[r])
                        NODE_HIP(nd, hipMemsetAsync(nd->d_send_act[slot] + (size_t)r * nd->chunk_cap, 0xFF, plan.send[r] * 4, pstream(slot)));
            NODE_HIP(nd, hipEventRecord(nd->ev_part[slot], pstream(slot)));
            lanes.push_back(Lane{reinterpret_cast<uint8_t*>(nd->d_send_act[slot]), nd->chunk_cap * 4,
                                 reinterpret_cast<uint8_t*>(nd->d_recv_act + owned), 4});
        }
        uint64_t bsend[ORL_NODE_MAX_RANKS] = {0}, brecv[ORL_NODE_MAX_RANKS] = {0}, bbase[ORL_NODE_MAX_RANKS] = {0}, btot = 0;
        if (plan.ext_lane) {  // some rank's chunk carries KeyExt strings: every rank sends the ext-ref lane (+ its strings)
            if (width != 32) return nfail(nd, ORL_E_STATE, "chunk %u: KeyExt strings with %u-byte records", c, width);
            for (uint32_t r = 0; r < nr; ++r) {
                bsend[r] = (H[me * W + 10 + r / 2] >> (32 * (r & 1))) & 0xFFFFFFFFull;
                brecv[r] = (H[r * W + 10 + me / 2] >> (32 * (me & 1))) & 0xFFFFFFFFull;
                bbase[r] = btot;
                btot += brecv[r];
            }
            if (!nd->d_recv_ext || !nd->d_send_ext[slot] || btot > nd->recv_blob_cap) {
                NODE_HIP(nd, hipDeviceSynchronize());
                if (!nd->d_recv_ext) NODE_HIP(nd, hipMalloc((void**)&nd->d_recv_ext, nd->cfg.max_recv * 8));
                for (int sl = 0; sl < 2; ++sl)
                    if (!nd->d_send_ext[sl]) NODE_HIP(nd, hipMalloc((void**)&nd->d_send_ext[sl], (size_t)nr * nd->chunk_cap * 8));
                if (btot > nd->recv_blob_cap) {
                    const uint64_t cap = std::max<uint64_t>(btot + btot / 2, 4096);
                    for (int sl = 0; sl < 2; ++sl) {
                        (void)hipFree(nd->d_recv_blob[sl]);
                        nd->d_recv_blob[sl] = nullptr;
                        NODE_HIP(nd, hipMalloc((void**)&nd->d_recv_blob[sl], cap));
                    }
                    nd->recv_blob_cap = cap;
                }
            }
            if (!kx)  // this rank wrote no ext lane: {~0, ~0} (no string) over what it sends
                for (uint32_t r = 0; r < nr; ++r)
                    if (plan.send[r])
                        NODE_HIP(nd, hipMemsetAsync(nd->d_send_ext[slot] + (size_t)r * nd->chunk_cap, 0xFF, plan.send[r] * 8, pstream(slot)));
            NODE_HIP(nd, hipEventRecord(nd->ev_part[slot], pstream(slot)));
            lanes.push_back(Lane{reinterpret_cast<uint8_t*>(nd->d_send_ext[slot]), nd->chunk_cap * 8,
                                 reinterpret_cast<uint8_t*>(nd->d_recv_ext + owned), 8});
        }
        if (int r = exchange(nd, lanes, plan.send, plan.recv, nd->ev_part[slot])) return r;
        if (plan.ext_lane) {  // the strings: per-rank byte counts of their own (the head words [10, 14))
            const std::vector<Lane> blane = {Lane{kx ? nd->d_send_blob[slot] : nd->d_recv_blob[slot], kx ? nd->send_blob_cap : 0,
                                                  nd->d_recv_blob[slot], 1}};
            if (int r = exchange(nd, blane, bsend, brecv, nd->ev_part[slot])) return r;
        }
        NODE_HIP(nd, hipEventRecord(nd->ev_slot[slot], nd->sx));
        nd->segs.push_back(orl_node::Seg{recv, got, width});
        if (got) {  // stages 1-3 of the received chunk, overlapping the next chunk's exchange
            NODE_HIP(nd, hipStreamWaitEvent(nd->sr, nd->ev_slot[slot], 0));
            // (records a sender addressed from its cache: HIT | CACHED from the act lane, no probe)
            NODE_CTX(nd, ctx_route_received(nd->ctx, recv, (int)width, got, ropts, nd->d_route + owned, nd->d_act + owned,
                                            plan.act_lane ? nd->d_recv_act + owned : nullptr, nd->sr));
            if (plan.ext_lane) {  // the KeyExt messages the route left unresolved: the owner's KeyExt table, with the strings
                int e = launch_ext_rebase(nd->d_recv_ext + owned, got, nr, plan.recv, bbase, nd->sr);
                if (e) return nfail(nd, ORL_E_DEVICE, "ext rebase launch: %s", hipGetErrorString((hipError_t)e));
                NODE_CTX(nd, ctx_route_keyext_received(nd->ctx, reinterpret_cast<const orl_msg_hdr*>(recv), got, ropts,
                                                       nd->d_recv_ext + owned, nd->d_recv_blob[slot], btot, nd->d_route + owned,
                                                       nd->d_act + owned, nd->sr));
            }
        }
        owned += got;
        owned_bytes += got * width;
    }
    // ---- hop 2: does any rank host activations of messages another rank owns? -----------------------------------
    // Stage 4 over the owned set is what every batch without forwarding ends with: when the previous batch forwarded
    // nothing, launch it now on sr, right after the last chunk's route, so it runs while the hop-2 counts are taken and
    // travel.  The host-rank counts read the routed words on the all-gathers' stream sh (round 4: off the stage-4
    // stream, so stage 4 does not wait for them).  If some rank does forward after all, the owned-set result is unused
    // (the hop-2 path writes its own buffers) and costs one stage 4.
    NODE_HIP(nd, hipEventRecord(nd->ev_r, nd->sr));  // every chunk is routed
    const bool spec = !nd->last_forward;
    if (spec) NODE_CTX(nd, orl_bucket_device(nd->ctx, nd->d_act, owned, nd->d_order, nd->d_off, nd->sr));
    {
        NODE_HIP(nd, hipStreamWaitEvent(nd->sh, nd->ev_r, 0));
        int e = launch_host_rank_count(nd->d_route, owned, nd->d_ros, me, nd->d_hcount, nd->sh);
        if (e) return nfail(nd, ORL_E_DEVICE, "host rank count launch: %s", hipGetErrorString((hipError_t)e));
        NODE_HIP(nd, hipEventRecord(nd->ev_h, nd->sh));
    }
    if (int r = allgather_heads(nd, nd->d_hcount, nd->ev_h, -2)) return r;
    const uint64_t* H = nd->h_heads;
    orl_node_hop2_plan h2;
    const int pr = orl_node_plan_hop2(H, nr, me, owned, width_mask, nd->cfg.max_recv, &h2);
    if (pr == ORL_E_CAPACITY) {
        for (uint32_t d = 0; d < nr; ++d) {
            uint64_t in = 0;
            for (uint32_t s = 0; s < nr; ++s) in += H[s * W + d];
            if (in > nd->cfg.max_recv)
                return nfail(nd, ORL_E_CAPACITY, "rank %u hosts %llu > max_recv %llu messages", d, (unsigned long long)in,
                             (unsigned long long)nd->cfg.max_recv);
        }
    }
    if (pr) return nfail(nd, pr, "hop-2 plan failed");
    const bool forward = h2.forward != 0;
    res->n_owned = owned;
    res->n_forwarded = h2.n_forwarded;
    res->n_sent_remote = sent_remote;
    nd->last_forward = forward;
    if (!forward) {  // every routed message is hosted where it was routed: stage 4 over the owned set
        if (!spec) NODE_CTX(nd, orl_bucket_device(nd->ctx, nd->d_act, owned, nd->d_order, nd->d_off, nd->sr));
        res->n_hosted = owned;
        res->route = nd->d_route;
        res->act = nd->d_act;
        res->order = nd->d_order;
        res->bucket_offsets = nd->d_off;
    } else {
        const uint64_t hosted = h2.n_hosted;
        if (int r = ensure_hop2(nd, owned)) return r;
        const uint32_t wout = h2.width;
        uint32_t* d_ferr = reinterpret_cast<uint32_t*>(nd->d_fcounts + ORL_NODE_MAX_CHUNKS * 8);
        NODE_HIP(nd, hipMemsetAsync(d_ferr, 0, 4, nd->sr));
        uint64_t off = 0;
        for (size_t k = 0; k < nd->segs.size(); ++k) {  // one partition per segment, positions chained through the totals
            const orl_node::Seg& sg = nd->segs[k];
            int e = launch_part_routed(nd->d_ros, sg.p, (int)sg.width, (int)wout, nd->d_route + off, nd->d_act + off, sg.count, me,
                                       nr, nd->f_cap, nd->d_fsend, nd->d_fsend_route, nd->d_fsend_act, nd->d_fstate,
                                       k ? nd->d_fcounts + 8 * (k - 1) : nullptr, nd->d_fcounts + 8 * k,
                                       ctx_wire_tcd(nd->ctx), d_ferr, nd->sr);
            if (e) return nfail(nd, ORL_E_DEVICE, "hop-2 partition launch: %s", hipGetErrorString((hipError_t)e));
            off += sg.count;
        }
        NODE_HIP(nd, hipEventRecord(nd->ev_r, nd->sr));
        {  // the hop-2 partition's look-back error word (its state is zeroed per launch): checked before anything is sent
            uint32_t lb_err = 0;
            if (int r = wait_bounded(nd, nd->sr, "hop-2 partition", -2, nullptr)) return r;
            NODE_HIP(nd, hipMemcpy(&lb_err, d_ferr, 4, hipMemcpyDeviceToHost));
            if (nd->lb_fail == 1) lb_err = 1;
            if (lb_err) {  // only this rank sees it: abort, so the peers fail now, not at their deadline
                break_node(nd);
                return nfail(nd, ORL_E_DEVICE, "hop-2 partition look-back gave up (device fault); communicator aborted");
            }
        }
        const std::vector<Lane> lanes = {Lane{nd->d_fsend, nd->f_cap * wout, nd->d_frecv, wout},
                                         Lane{reinterpret_cast<uint8_t*>(nd->d_fsend_route), nd->f_cap * 4,
                                              reinterpret_cast<uint8_t*>(nd->d_frecv_route), 4},
                                         Lane{reinterpret_cast<uint8_t*>(nd->d_fsend_act), nd->f_cap * 4,
                                              reinterpret_cast<uint8_t*>(nd->d_frecv_act), 4}};
        if (int r = exchange(nd, lanes, h2.send, h2.recv, nd->ev_r)) return r;
        // nothing after this exchange waits on the host: bound it here, so a missing peer fails this call instead of
        // hanging the caller's stream
        if (int r = wait_bounded(nd, nd->sx, "hop-2 exchange", -2, nullptr)) return r;
        NODE_HIP(nd, hipEventRecord(nd->ev_x, nd->sx));
        NODE_HIP(nd, hipStreamWaitEvent(nd->sr, nd->ev_x, 0));
        NODE_CTX(nd, orl_bucket_device(nd->ctx, nd->d_frecv_act, hosted, nd->d_forder, nd->d_foff, nd->sr));
        nd->segs.assign(1, orl_node::Seg{nd->d_frecv, hosted, wout});
        res->hop2 = 1;
        res->n_hosted = hosted;
        res->route = nd->d_frecv_route;
        res->act = nd->d_frecv_act;
        res->order = nd->d_forder;
        res->bucket_offsets = nd->d_foff;
    }
    res->n_segments = (uint32_t)nd->segs.size();
    NODE_HIP(nd, hipEventRecord(nd->ev_r, nd->sr));
    NODE_HIP(nd, hipStreamWaitEvent(caller, nd->ev_r, 0));  // the caller's stream sees complete outputs
    // stage 4's look-back error word, copied behind the outputs (the caller does not wait for it): the next batch checks it
    NODE_HIP(nd, hipMemcpyAsync(nd->h_s4err, ctx_stage4_err(nd->ctx), 4, hipMemcpyDeviceToHost, nd->sr));
    NODE_HIP(nd, hipEventRecord(nd->ev_s4, nd->sr));
    nd->s4_pending = true;
    return ORL_OK;
}

int orl_node_route_batch_keyext_device(orl_node* nd, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const orl_ext_ref* d_ext,
                                       const uint8_t* d_blob, uint64_t blob_bytes, orl_node_result* res, void* stream) {
    if (!nd || !res) return ORL_E_INVALID;
    if (n && (!d_ext || !d_blob)) return nfail(nd, ORL_E_INVALID, "null KeyExt references or blob");
    if (blob_bytes > 0xFFFFFFFFull) return nfail(nd, ORL_E_INVALID, "KeyExt blob of %llu bytes (<= 4 GiB)", (unsigned long long)blob_bytes);
    nd->kx_ext = n ? d_ext : nullptr;
    nd->kx_blob = d_blob;
    nd->kx_bytes = blob_bytes;
    const int r = orl_node_route_batch_device(nd, d_in, n, opts, res, stream);
    nd->kx_ext = nullptr;
    nd->kx_blob = nullptr;
    nd->kx_bytes = 0;
    return r;
}

}  // extern "C"
