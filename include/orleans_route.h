/*
 * orleans_route.h — C ABI of liborleans_route.so, the MI355X batched grain-message routing engine.
 *
 * The engine replaces the per-message routing work of an Orleans 1.1 silo
 * (randa1/orleans; paths below are relative to that checkout) with a batched HIP pipeline:
 *   stage 1  GrainId uniform hash      JenkinsHash.ComputeHash(TCD,N0,N1)  src/Orleans/IDs/JenkinsHash.cs:126-144
 *   stage 2  directory ring owner      LocalGrainDirectory.CalculateTargetSilo
 *                                       src/OrleansRuntime/GrainDirectory/LocalGrainDirectory.cs:439-497
 *   stage 3  directory partition probe GrainDirectoryPartition.LookUpGrain + IsValidSilo
 *                                       src/OrleansRuntime/GrainDirectory/GrainDirectoryPartition.cs:326-344
 *            + placement of misses     PlacementDirectorsManager.SelectOrAddActivation
 *                                       src/OrleansRuntime/Placement/PlacementDirectorsManager.cs:70-91
 *   stage 4  stable per-activation FIFO ActivationData.EnqueueMessage  src/OrleansRuntime/Catalog/ActivationData.cs:483-514
 *   stage 5  multicast fan-out          ChirperAccount.PublishMessage   Samples/Chirper/ChirperGrains/ChirperAccount.cs:154-157
 *
 * The reference path has no FFI of its own (it is C#, internal interfaces only).  These entry
 * points are what a C# `NativeMethods` class ([DllImport("orleans_route")], the pattern of
 * src/Orleans/Statistics/ThreadCycleStopWatch.cs:120-128) would bind from inside
 * LocalGrainDirectory / Dispatcher / MessageCenter; see INTEGRATION.md.
 *
 * Conventions
 *  - Every function returns an int status (ORL_OK = 0, < 0 = API error; orl_last_error(ctx) explains).
 *    Nothing throws or aborts across the ABI.  Per-message outcomes are status bytes in the route word.
 *  - Caller owns every host array; the library owns all device state (ring, directory table, scratch).
 *  - `*_device` entry points take device pointers already resident in HBM and a hipStream_t (as void*);
 *    they enqueue work and return without synchronising.
 *  - A context is bound to one HIP device.  Calls on one context must not race (one submitting thread
 *    per silo context, as SURVEY §8(b) recommends); ring/table updates take effect between batches.
 *  - Silos are identified by a dense index 0..n_silos-1 (< 255); 0xFF means "null SiloAddress".
 */
#ifndef ORLEANS_ROUTE_H
#define ORLEANS_ROUTE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORL_ABI_VERSION 1u
#define ORL_MAX_SILOS 255u
#define ORL_NULL_SILO 0xFFu
#define ORL_NO_ACT 0xFFFFFFFFu
#define ORL_MAX_RING 256u

/* ---- API status codes ------------------------------------------------------------------- */
#define ORL_OK 0
#define ORL_E_INVALID (-1)   /* bad argument / unsupported key (ArgumentException analogues) */
#define ORL_E_NOMEM (-2)     /* host or device allocation failed */
#define ORL_E_DEVICE (-3)    /* HIP runtime error (message in orl_last_error) */
#define ORL_E_CAPACITY (-4)  /* batch larger than orl_config.max_batch, or directory full */
#define ORL_E_STATE (-5)     /* call not valid in the context's current state */
#define ORL_E_OVERFLOW (-6)  /* Math.Abs(int.MinValue) analogue (OutboundMessageQueue.cs:141) */

/* ---- UniqueKey categories (src/Orleans/IDs/UniqueKey.cs:41-49) ---------------------------- */
#define ORL_CAT_NONE 0u
#define ORL_CAT_SYSTEM_TARGET 1u
#define ORL_CAT_SYSTEM_GRAIN 2u
#define ORL_CAT_GRAIN 3u
#define ORL_CAT_CLIENT 4u
#define ORL_CAT_KEYEXT_GRAIN 6u

/* GrainId identity = UniqueKey {N0, N1, TypeCodeData} (UniqueKey.cs:51-54).  24 bytes.
 * Category lives in the top byte of type_code_data (UniqueKey.cs:141). */
typedef struct orl_grain_key {
    uint64_t type_code_data;
    uint64_t n0;
    uint64_t n1;
} orl_grain_key;

/* Header flags (orl_msg_hdr.flags) */
#define ORL_HDR_ADDRESS_COMPLETE 0x01u /* Message.TargetAddress.IsComplete: skip routing (Dispatcher.cs:557-558) */
#define ORL_HDR_HASH_VALID 0x02u       /* aux holds the precomputed uniform hash (KeyExt slow path, UniqueKey.cs:288-294) */

/* One message header as the routing path reads it (Message.cs:199-291): 32 bytes, SoA-friendly AoS.
 * Message order in a batch = arrival order. */
typedef struct orl_msg_hdr {
    orl_grain_key target;   /* TargetGrain */
    uint8_t sending_silo;   /* SendingSilo index == "MyAddress" of the routing silo */
    uint8_t category;       /* Message.Categories (Ping 0 / System 1 / Application 2), carried through */
    uint8_t flags;          /* ORL_HDR_* */
    uint8_t target_silo;    /* TargetSilo when ORL_HDR_ADDRESS_COMPLETE, else ignored */
    uint32_t aux;           /* precomputed uniform hash when ORL_HDR_HASH_VALID */
} orl_msg_hdr;

/* Compact 16-byte exchange record (multi-GPU wire format) for the common key shape: N0 == 0 and
 * TypeCodeData = (grain category << 56) + sign-extended 32-bit type code (UniqueKey.NewKey, UniqueKey.cs:131-152:
 * every long-key grain, GrainId.GetGrainId(int typeCode, long key), GrainId.cs:90-97).  meta packs
 * sending_silo (bits 0-7), message category (8-9), header flags (10-15; ORL_HDR_HASH_VALID not allowed:
 * the hash is recomputed), grain category (16-23) and target_silo (24-31).  Lossless: decoding gives back
 * the 32-byte orl_msg_hdr (aux = 0). */
typedef struct orl_wire_msg {
    uint64_t n1;
    uint32_t type_code_lo;  /* low 32 bits of TypeCodeData */
    uint32_t meta;
} orl_wire_msg;

/* Narrow 8-byte exchange record: the 16-byte form's content when N1 < 2^32 and the TypeCodeData is one of the
 * context's wire types (orl_wire_types_set: the node's grain classes, the same table on every rank — Orleans builds
 * one type map per cluster at silo start-up, GrainTypeManager).  meta packs sending_silo (bits 0-7), message category
 * (8-9), header flags (10-15; ORL_HDR_HASH_VALID not allowed), the wire type index (16-19; bits 20-23 zero) and
 * target_silo (24-31).  Lossless: decoding with the same table gives back the 32-byte orl_msg_hdr (N0 = 0, aux = 0). */
#define ORL_MAX_WIRE_TYPES 16u
typedef struct orl_wire8 {
    uint32_t n1;
    uint32_t meta;
} orl_wire8;

/* ---- Per-message route word ---------------------------------------------------------------
 * bits 0-7 directory owner silo, 8-15 target (host) silo, 16-23 ORL_ST_*, 24-31 ORL_RF_*      */
#define ORL_ST_HIT 0u                  /* single activation found on a functional silo */
#define ORL_ST_NEW_PLACEMENT 1u        /* miss: OnAddActivation chose the host silo (IsNewPlacement) */
#define ORL_ST_SYSTEM_TARGET 2u        /* SystemTarget: owner = routing silo (LocalGrainDirectory.cs:442-447) */
#define ORL_ST_ADDRESS_COMPLETE 3u     /* header already addressed; passed through */
#define ORL_ST_OWNER_NULL 4u           /* owner null: "Grain directory is stopping" (:471-475, :483-493) */
#define ORL_ST_NO_SEED 5u              /* membership-table grain without seed (ArgumentException :449-460) */
#define ORL_ST_CLIENT_UNREGISTERED 6u  /* client grain miss (KeyNotFoundException, PlacementDirectorsManager.cs:75-81) */
#define ORL_ST_KEYEXT_UNRESOLVED 7u    /* KeyExt grain: owner computed, partition lookup left to host */
#define ORL_ST_REMOTE_OWNER 8u         /* owner's partition not held by this context (cache/FullLookup path) */
#define ORL_ST_PAST_TOTAL 9u           /* fan-out with an overstated ORL_OPT_TOTAL_GIVEN: no message at this index */

#define ORL_RF_NEW_PLACEMENT 0x01u
#define ORL_RF_LOOPBACK 0x02u          /* target silo == sending silo (OutboundMessageQueue.cs:113-119) */
#define ORL_RF_OWNER_IS_SEED 0x04u

#define ORL_ROUTE_OWNER(r) ((uint32_t)(r) & 0xFFu)
#define ORL_ROUTE_HOST(r) (((uint32_t)(r) >> 8) & 0xFFu)
#define ORL_ROUTE_STATUS(r) (((uint32_t)(r) >> 16) & 0xFFu)
#define ORL_ROUTE_FLAGS(r) (((uint32_t)(r) >> 24) & 0xFFu)

/* Placement policy for misses (deterministic subset of the reference directors) */
#define ORL_POLICY_PREFER_LOCAL 0u  /* PreferLocalPlacementDirector.cs:38-44: the sending silo */
#define ORL_POLICY_HASH_SPREAD 1u   /* RandomPlacementDirector.cs:59-66 with hash % |active| instead of SafeRandom */

/* Route options (bit set) */
#define ORL_OPT_EXCLUDE_IF_STOPPING 0x1u /* CalculateTargetSilo(grain, excludeThisSiloIfStopping=true) */
#define ORL_OPT_NO_BUCKETS 0x2u          /* skip stage 4 (order/offsets not written) */
#define ORL_OPT_TOTAL_GIVEN 0x4u         /* fan-out: *n_out holds the exact emitted count on entry (no stream sync,
                                            so the call can be captured in a hipGraph) */

/* Directory insert outcome (orl_dir_insert_single status[]) */
#define ORL_INS_INSERTED 0u
#define ORL_INS_EXISTING 1u      /* first writer wins: winner returned (GrainInfo.AddSingleActivation :100-114) */
#define ORL_INS_INVALID_SILO 2u  /* !IsValidSilo(silo): AddSingleActivation returns null (:277-279) */
#define ORL_INS_REMOTE_OWNER 3u  /* owner partition not local: caller must forward (LocalGrainDirectory.cs:529-541) */
#define ORL_INS_OWNER_NULL 4u    /* owner null (directory stopping) */
#define ORL_INS_UNSUPPORTED 5u   /* KeyExt / SystemTarget keys are not held in the device partition */

typedef struct orl_config {
    uint32_t abi_version;      /* must be ORL_ABI_VERSION */
    int32_t device;            /* HIP device ordinal */
    uint64_t dir_capacity;     /* max directory entries; table = next_pow2(2*dir_capacity) 32-B slots */
    uint32_t n_act;            /* activation-handle space [0, n_act); buckets = n_act + 1 (last = unresolved) */
    uint32_t placement_policy; /* ORL_POLICY_* */
    uint64_t max_batch;        /* largest batch (messages, incl. fan-out output) the scratch is sized for */
} orl_config;

typedef struct orl_ctx orl_ctx;

/* ---- lifecycle ------------------------------------------------------------------------ */
int orl_ctx_create(const orl_config* cfg, orl_ctx** out);
int orl_ctx_destroy(orl_ctx* ctx);
const char* orl_last_error(const orl_ctx* ctx);
uint32_t orl_abi_version(void);

/* ---- silo table + ring (LocalGrainDirectory membership events :243-304, :390-427) ---------
 * running[i]: LocalGrainDirectory.Running of silo i (used for excludeMySelf, :478)
 * functional[i]: Membership.IsFunctionalDirectory(i) (IsValidSilo, :421-427)
 * local[i]: this context holds silo i's directory partition (its GPU hosts silo i)
 * seed: index of the Seed silo (membership-table grain owner) or ORL_NULL_SILO */
int orl_silos_set(orl_ctx* ctx, uint32_t n_silos, const uint8_t* running, const uint8_t* functional,
                  const uint8_t* local, uint32_t seed);
/* AddServer: sorted insert by signed consistent hash, before equal hashes (LocalGrainDirectory.cs:243-268) */
int orl_ring_add_server(orl_ctx* ctx, uint32_t silo, int32_t consistent_hash);
/* RemoveServer (LocalGrainDirectory.cs:270-304; list removal) */
int orl_ring_remove_server(orl_ctx* ctx, uint32_t silo);
int orl_ring_get(const orl_ctx* ctx, int32_t* hashes, uint8_t* silos, uint32_t cap, uint32_t* n_out);

/* ---- host-side identity helpers (not per message) ----------------------------------------- */
/* Utils.CalculateIdHash(text) (Utils.cs:201-220): SHA-256 of the UTF-16LE encoding of `utf8` text */
int orl_calc_id_hash(const char* utf8, size_t len, int32_t* out);
/* SiloAddress.GetConsistentHashCode (SiloAddress.cs:197-206): CalculateIdHash(endpoint + generation) */
int orl_silo_consistent_hash(const char* endpoint_utf8, int32_t generation, int32_t* out);
/* JenkinsHash.ComputeHash(byte[]) (JenkinsHash.cs:68-115) */
uint32_t orl_jenkins_bytes(const uint8_t* data, size_t len);
/* UniqueKey.GetUniformHashCode KeyExt branch (UniqueKey.cs:288-294; serialization BinaryTokenStreamWriter.cs:488-494) */
uint32_t orl_keyext_uniform_hash(const orl_grain_key* key, const char* key_ext_utf8, size_t len);

/* ---- directory partition (single activation) --------------------------------------------
 * RegisterSingleActivation → GrainDirectoryPartition.AddSingleActivation (GrainDirectoryPartition.cs:270-287).
 * Inserts are applied in array order: the first writer of a grain wins; later writers get the winner.
 * The registering silo is the activation's silo (ActivationAddress.Silo): it computes the owner with
 * CalculateTargetSilo(grain) (excludeThisSiloIfStopping = true).
 * winner_act / winner_silo / status may be NULL.  acts[i] must be < n_act. */
int orl_dir_insert_single(orl_ctx* ctx, const orl_grain_key* keys, const uint32_t* acts, const uint8_t* silos,
                          size_t n, uint32_t* winner_act, uint8_t* winner_silo, uint8_t* status);
/* RemoveGrain / RemoveActivation(force) of a single-activation grain (:290-318).  removed[i] = 1 if present. */
int orl_dir_remove(orl_ctx* ctx, const orl_grain_key* keys, size_t n, uint8_t* removed);
/* Device-resident registration / unregistration batches: same per-message outcomes as
 * orl_dir_insert_single / orl_dir_remove applied one message at a time in batch order (first writer of a
 * key wins, its activation is every later writer's winner; the first removal of a key removes it), computed
 * by kernels on the device table.  Keys, acts, silos and outputs are device arrays; nothing synchronises.
 * Out-of-range act / silo values give ORL_INS_UNSUPPORTED for that message (no host-side validation).
 * Fails with ORL_E_CAPACITY before launching if the batch could push live entries past 1/2 of the slots or
 * entries + tombstones past 7/8.  Registrations reuse tombstones (the first one on the key's chain).
 * The host mirror (orl_dir_lookup_host, orl_dir_count, the host insert/remove) is re-read from the device
 * on its next use.  Reference: LocalGrainDirectory.RegisterSingleActivationAsync / UnregisterAsync
 * (LocalGrainDirectory.cs:510-612) → GrainDirectoryPartition.AddSingleActivation / RemoveActivation
 * (GrainDirectoryPartition.cs:270-318). */
int orl_dir_insert_single_device(orl_ctx* ctx, const orl_grain_key* d_keys, const uint32_t* d_acts, const uint8_t* d_silos,
                                 size_t n, uint32_t* d_winner_act, uint8_t* d_winner_silo, uint8_t* d_status, void* stream);
int orl_dir_remove_device(orl_ctx* ctx, const orl_grain_key* d_keys, size_t n, uint8_t* d_removed, void* stream);
/* Hand-off split for a membership change (GrainDirectoryHandoffManager.ProcessSiloAddEvent,
 * GrainDirectoryHandoffManager.cs:205-250): after orl_ring_add_server, every entry whose owner under the new
 * ring, CalculateTargetSilo(grain) seen from silo `me`, is not null and not `me` (GrainDirectoryPartition.Split
 * :384-425) and whose activation silo is valid (ToListOfActivations :427-443) is written to d_keys / d_acts /
 * d_silos (device, table-slot order, at most cap entries); *d_n_out (device u64) receives the full count.
 * With ORL_SPLIT_REMOVE the emitted entries are tombstoned here (the RemoveGrain that follows a successful
 * hand-off).  The receiving silo registers them with orl_dir_insert_single_device (RegisterManySingleActivation). */
#define ORL_SPLIT_REMOVE 0x1u
int orl_dir_split_device(orl_ctx* ctx, uint32_t me, uint32_t flags, orl_grain_key* d_keys, uint32_t* d_acts, uint8_t* d_silos,
                         uint64_t cap, uint64_t* d_n_out, void* stream);
/* Merge of a partition copy (GrainDirectoryHandoffManager.ProcessSiloRemoveEvent,
 * GrainDirectoryHandoffManager.cs:141-168 → GrainDirectoryPartition.Merge, GrainDirectoryPartition.cs:366-383):
 * when a silo leaves, its successor merges the copy of the removed silo's partition it holds.  An absent grain is
 * added as is (Merge checks neither ownership nor silo validity); for a grain present on both sides GrainInfo.Merge
 * (:158-183) keeps the activation with the smaller ActivationId — UniqueKey.CompareTo order (TypeCodeData, N0, N1),
 * d_act_keys[handle] = the ActivationId key of each activation handle — and the other is reported in
 * d_dropped_act / d_dropped_silo (for Catalog.DeleteActivations on its silo; ORL_NO_ACT otherwise).  The copy is a
 * dictionary: a key repeated within the batch is ORL_MERGE_DUPLICATE after its first occurrence.  Capacity rules
 * as orl_dir_insert_single_device. */
#define ORL_MERGE_INSERTED 0u
#define ORL_MERGE_KEPT 1u         /* present; ours has the smaller ActivationId: the incoming one is dropped */
#define ORL_MERGE_REPLACED 2u     /* present; the incoming one is smaller: ours is dropped and replaced */
#define ORL_MERGE_SAME 3u         /* present with the same ActivationId */
#define ORL_MERGE_DUPLICATE 4u
#define ORL_MERGE_UNSUPPORTED 5u  /* KeyExt grain, out-of-range handle or silo */
int orl_dir_merge_device(orl_ctx* ctx, const orl_grain_key* d_keys, const uint32_t* d_acts, const uint8_t* d_silos, size_t n,
                         const orl_grain_key* d_act_keys, uint32_t n_act_keys, uint8_t* d_status, uint32_t* d_dropped_act,
                         uint8_t* d_dropped_silo, void* stream);
/* Rebuild the partition without tombstones (GrainDirectoryPartition keeps a Dictionary: no tombstones there;
 * long-running silos call this when orl_dir_insert_single_device reports ORL_E_CAPACITY with tombstones). */
int orl_dir_compact(orl_ctx* ctx);
int orl_dir_count(const orl_ctx* ctx, uint64_t* n_out);
/* Host lookup (LookUpGrain without the IsValidSilo filter): act/silo or ORL_NO_ACT/ORL_NULL_SILO */
int orl_dir_lookup_host(const orl_ctx* ctx, const orl_grain_key* keys, size_t n, uint32_t* act, uint8_t* silo);

/* ---- stage 1 alone (tests) ---------------------------------------------------------------- */
int orl_hash_batch(orl_ctx* ctx, const orl_grain_key* keys, size_t n, uint32_t* hashes_out);

/* ---- the hot path --------------------------------------------------------------------------
 * Stages 1-4 over n messages.  Outputs:
 *   route[n]            route word (owner | host<<8 | status<<16 | flags<<24)
 *   act[n]              activation handle or ORL_NO_ACT
 *   order[n]            message indices grouped by bucket, arrival order kept inside a bucket
 *   bucket_offsets[n_act+2]  bucket b holds order[offsets[b] .. offsets[b+1]); bucket n_act = unresolved
 * Host-buffer form (P/Invoke): copies in/out over PCIe and synchronises. */
int orl_route_batch(orl_ctx* ctx, const orl_msg_hdr* in, size_t n, uint32_t opts, uint32_t* route, uint32_t* act,
                    uint32_t* order, uint32_t* bucket_offsets);
/* Host-array form over 8-byte orl_wire8 records in the context's wire types (orl_wire_types_set): the narrow P/Invoke
 * call a silo makes per batch when its targets are long-key grains of known classes with 32-bit keys (the common case:
 * GrainId.GetGrainId(typeCode, long key), GrainId.cs:90-97).  PCIe carries 8 B in and 8 B out per message (+ 4 B of
 * order) instead of 32 + 8 (+ 4); outputs as orl_route_batch.  Replaces the per-message Dispatcher.AddressMessage
 * (src/OrleansRuntime/Core/Dispatcher.cs:555-579). */
int orl_route_batch_narrow(orl_ctx* ctx, const orl_wire8* in, size_t n, uint32_t opts, uint32_t* route, uint32_t* act,
                           uint32_t* order, uint32_t* bucket_offsets);
/* Device-resident form: all pointers in HBM; enqueued on `stream` (hipStream_t, NULL = default).
 * Stage 4 of a context keeps per-context state from batch to batch (the hot-key slots the tail kernel of one batch
 * writes and the next batch reads, their parity flipped by the launcher, the candidate word of the one-pass level 2,
 * the long-gap queue of the LSD offsets): every bucketing call of one context (orl_route_*_device, orl_fanout_*_device,
 * orl_bucket_device) must be enqueued on ONE stream, as the one-pass partitions must (below).  Two streams need two
 * contexts. */
int orl_route_batch_device(orl_ctx* ctx, const orl_msg_hdr* d_in, size_t n, uint32_t opts, uint32_t* d_route,
                           uint32_t* d_act, uint32_t* d_order, uint32_t* d_bucket_offsets, void* stream);

/* Stage 5 + 1-4: CSR multicast.  Publish p (account pubs[p] sending from silo pub_silo[p]) expands to
 * one send per follower csr_tgt[csr_off[pubs[p]] .. csr_off[pubs[p]+1]) in CSR order; follower grain =
 * GrainId(follower_tcd, long id) = key {follower_tcd, 0, id}.  Output message j (publisher-major) is
 * routed as in orl_route_batch_device; pub_offsets[n_pub+1] (device) maps publishes to output ranges.
 * *n_out (host) receives the number of emitted messages (this call synchronises `stream` once to read it,
 * unless opts has ORL_OPT_TOTAL_GIVEN and *n_out already holds that count).
 * Reference: ChirperAccount.PublishMessage fan-out loop (Samples/Chirper/ChirperGrains/ChirperAccount.cs:154-157),
 * ObserverSubscriptionManager.Notify (src/Orleans/Async/ObserverSubscriptionManager.cs:111-139). */
int orl_fanout_route_device(orl_ctx* ctx, const uint64_t* d_csr_off, const uint32_t* d_csr_tgt,
                            const uint32_t* d_pubs, const uint8_t* d_pub_silo, size_t n_pub, uint64_t follower_tcd,
                            uint32_t opts, uint64_t* d_pub_offsets, uint32_t* d_route, uint32_t* d_act,
                            uint32_t* d_order, uint32_t* d_bucket_offsets, uint64_t* n_out, void* stream);
/* As orl_fanout_route_device, with followers named by a device key table: follower of CSR entry j is
 * d_follower_keys[csr_tgt[j]] (any GrainId, e.g. the Guid-keyed players of Samples/Presence
 * GameGrain.UpdateGameStatus, Samples/Presence/PresenceGrains/GameGrain.cs:62-113). */
int orl_fanout_route_keys_device(orl_ctx* ctx, const uint64_t* d_csr_off, const uint32_t* d_csr_tgt,
                                 const orl_grain_key* d_follower_keys, const uint32_t* d_pubs, const uint8_t* d_pub_silo,
                                 size_t n_pub, uint32_t opts, uint64_t* d_pub_offsets, uint32_t* d_route, uint32_t* d_act,
                                 uint32_t* d_order, uint32_t* d_bucket_offsets, uint64_t* n_out, void* stream);
/* One batch of direct messages + a CSR fan-out, routed and bucketed together (one route launch, one stage-4 pass):
 * output message j < n_direct is d_direct[j] (as orl_route_batch_device); message n_direct + k is fan-out message k
 * (as orl_fanout_route_device: followers d_follower_keys[csr_tgt[...]], or GrainId(follower_tcd, csr_tgt[...]) when
 * d_follower_keys is NULL).  d_pub_offsets[n_pub+1] are absolute output positions (they start at n_direct); *n_out
 * = n_direct + emitted (with ORL_OPT_TOTAL_GIVEN it holds that total on entry, at least n_direct).  A silo tick's
 * outbound messages in one call, e.g. Samples/Presence: PresenceGrain.Heartbeat's game messages
 * (PresenceGrain.cs:42-47) + GameGrain.UpdateGameStatus's player fan-out (GameGrain.cs:62-113). */
int orl_fanout_route_mixed_device(orl_ctx* ctx, const orl_msg_hdr* d_direct, size_t n_direct, const uint64_t* d_csr_off,
                                  const uint32_t* d_csr_tgt, const orl_grain_key* d_follower_keys, uint64_t follower_tcd,
                                  const uint32_t* d_pubs, const uint8_t* d_pub_silo, size_t n_pub, uint32_t opts,
                                  uint64_t* d_pub_offsets, uint32_t* d_route, uint32_t* d_act, uint32_t* d_order,
                                  uint32_t* d_bucket_offsets, uint64_t* n_out, void* stream);

/* Stage 5 alone: the messages a batch of publishes sends, as orl_msg_hdr records in d_out (cap records), publisher-
 * major in CSR order (followers as in orl_fanout_route_mixed_device; sending silo = the publisher's, category
 * Application).  For a node whose followers' directory partitions live on other GPUs: the records go through
 * orl_node_route_batch_device (orl_node_fanout_batch_device does both).  *n_out = the emitted count (one stream sync),
 * unless ORL_OPT_TOTAL_GIVEN (then records past the real count are null, address-complete headers with target silo
 * 0xFF).  ORL_E_CAPACITY when the count exceeds cap.  Reference: ChirperAccount.PublishMessage's per-follower sends
 * (Samples/Chirper/ChirperGrains/ChirperAccount.cs:154-157), each a GrainReference call from the publisher's silo. */
int orl_fanout_expand_device(orl_ctx* ctx, const uint64_t* d_csr_off, const uint32_t* d_csr_tgt,
                             const orl_grain_key* d_follower_keys, uint64_t follower_tcd, const uint32_t* d_pubs,
                             const uint8_t* d_pub_silo, size_t n_pub, uint32_t opts, uint64_t* d_pub_offsets,
                             orl_msg_hdr* d_out, uint64_t cap, uint64_t* n_out, void* stream);

/* ---- stream / reminder rings -------------------------------------------------
 * Two ring providers route stream queues and reminders; both look CLOCKWISE (first ring point >= key):
 *   ORL_RING_CONSISTENT  ConsistentRingProvider (src/OrleansRuntime/ConsistentRing/ConsistentRingProvider.cs:
 *                        116-135, 342-379): the directory's membershipRingList (orl_ring_add_server); the
 *                        signed silo hash is compared with the uint key as a long.
 *   ORL_RING_VBUCKETS    VirtualBucketsRingProvider (VirtualBucketsRingProvider.cs:142-193, 277-313):
 *                        buckets_per_silo uniform hashes per silo (SiloAddress.GetUniformHashCodes,
 *                        SiloAddress.cs:208-230: Jenkins over IP16 | port | generation | i), lesser generation
 *                        keeps a colliding bucket, RemoveServer drops all of the silo's hashes.
 * Keys are uint32 uniform hashes (a grain's: orl_hash_batch, for reminders).  `me` + ORL_OPT_EXCLUDE_IF_STOPPING
 * give excludeMySelf (when `me` is not running). */
#define ORL_RING_CONSISTENT 0u
#define ORL_RING_VBUCKETS 1u
#define ORL_MAX_VBUCKETS_PER_SILO 64u
int orl_vring_set_buckets(orl_ctx* ctx, uint32_t buckets_per_silo);  /* default 30; only while the ring is empty */
int orl_vring_add_server(orl_ctx* ctx, uint32_t silo, const uint8_t* ip16, int32_t port, int32_t generation);
int orl_vring_remove_server(orl_ctx* ctx, uint32_t silo);
int orl_vring_get(const orl_ctx* ctx, uint32_t* hashes, uint8_t* silos, uint32_t cap, uint32_t* n_out);
int orl_ring_owner_batch_device(orl_ctx* ctx, uint32_t kind, const uint32_t* d_keys, size_t n, uint32_t me,
                                uint32_t opts, uint8_t* d_owner, void* stream);
/* Stream queue of each stream Guid (16 bytes each, Guid.ToByteArray() order): HashRingBasedStreamQueueMapper
 * .GetQueueForStream (src/Orleans/Streams/QueueAdapters/HashRingBasedStreamQueueMapper.cs:36-53,68-71,
 * src/Orleans/Runtime/HashRing.cs:95-126) with n_queues queues; d_silo (optional) = the ring owner of the
 * queue's hash under `kind` (the silo whose range holds the queue). */
int orl_stream_queue_batch_device(orl_ctx* ctx, uint32_t kind, const uint8_t* d_guids, size_t n, uint32_t n_queues,
                                  uint32_t me, uint32_t opts, uint32_t* d_queue, uint8_t* d_silo, void* stream);

/* ---- KeyExt (string-key) grains in the directory (round 5) --------------------------------------------
 * GrainDirectoryPartition holds any GrainId (GrainDirectoryPartition.cs:270-287,326-344); a KeyExt grain's identity is
 * its UniqueKey including the string extension, and its uniform hash is Jenkins over Write(UniqueKey) (UniqueKey.cs:288-
 * 294: N0, N1, TypeCodeData, int32 length, UTF-8).  The context keeps KeyExt grains in a table of their own: the 24-B key,
 * the hash and the extension bytes (a blob the library owns), first writer wins like the main partition.  A string is
 * passed as orl_ext_ref into a caller's UTF-8 blob (host or device as the call says). */
typedef struct orl_ext_ref {
    uint32_t off;  /* first byte in the blob */
    uint32_t len;  /* bytes (UTF-8, as BinaryTokenStreamWriter.Write(string) writes them) */
} orl_ext_ref;
/* RegisterSingleActivation of KeyExt grains (category ORL_CAT_KEYEXT_GRAIN; the same statuses as orl_dir_insert_single:
 * owner = the ring owner of the KeyExt hash, excludeThisSiloIfStopping; a key of another category gives
 * ORL_INS_UNSUPPORTED).  Host arrays; `blob` (blob_bytes long) holds the extensions: a reference outside it fails the call
 * with ORL_E_INVALID before anything is inserted; ORL_E_CAPACITY when the library's extension store would pass 4 GiB. */
int orl_dir_insert_keyext(orl_ctx* ctx, const orl_grain_key* keys, const orl_ext_ref* ext, const uint8_t* blob,
                          uint64_t blob_bytes, const uint32_t* acts, const uint8_t* silos, size_t n, uint32_t* winner_act,
                          uint8_t* winner_silo, uint8_t* status);
int orl_dir_remove_keyext(orl_ctx* ctx, const orl_grain_key* keys, const orl_ext_ref* ext, const uint8_t* blob,
                          uint64_t blob_bytes, size_t n, uint8_t* removed);
/* LookUpGrain of KeyExt grains on the host copy (no IsValidSilo filter; ORL_NO_ACT / ORL_NULL_SILO when absent). */
int orl_dir_lookup_keyext_host(orl_ctx* ctx, const orl_grain_key* keys, const orl_ext_ref* ext, const uint8_t* blob,
                               uint64_t blob_bytes, size_t n, uint32_t* act, uint8_t* silo);
int orl_dir_keyext_count(const orl_ctx* ctx, uint64_t* n);
/* orl_dir_insert_keyext on the device (round 6): the same statuses and winner rule (first writer of a key in the batch,
 * GrainInfo.AddSingleActivation :103-107) over device arrays, asynchronously on `stream`; the strings are read from
 * `d_blob` (blob_bytes long) and appended to the library's device store.  As orl_dir_insert_single_device: an act >=
 * n_act, a silo outside the table or a reference outside the blob gives ORL_INS_UNSUPPORTED for that message (no host
 * validation).  The device table is then the newer one: the host KeyExt calls (insert, remove, lookup, count) first
 * download it (they synchronise the device).  ORL_E_CAPACITY when the store would pass 4 GiB; a device-side overrun is
 * reported by the next host KeyExt call. */
int orl_dir_insert_keyext_device(orl_ctx* ctx, const orl_grain_key* d_keys, const orl_ext_ref* d_ext, const uint8_t* d_blob,
                                 uint64_t blob_bytes, const uint32_t* d_acts, const uint8_t* d_silos, size_t n,
                                 uint32_t* d_winner_act, uint8_t* d_winner_silo, uint8_t* d_status, void* stream);
/* orl_route_batch_device with the batch's KeyExt strings: d_ext[i] locates message i's extension in d_blob (device,
 * blob_bytes long; read only for KeyExt messages).  A KeyExt message whose header carries ORL_HDR_HASH_VALID uses that
 * hash, otherwise the kernel computes it from the bytes.  Its owner's KeyExt table is probed when the owner is local:
 * HIT (IsValidSilo-filtered), or a miss placed like any grain (PlacementDirectorsManager); a remote owner gives
 * ORL_ST_REMOTE_OWNER (the FullLookup path).  A reference outside the blob leaves ORL_ST_KEYEXT_UNRESOLVED.  Other
 * messages route exactly as in orl_route_batch_device; stage 4 follows as there. */
int orl_route_keyext_device(orl_ctx* ctx, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const orl_ext_ref* d_ext,
                            const uint8_t* d_blob, uint64_t blob_bytes, uint32_t* d_route, uint32_t* d_act, uint32_t* d_order,
                            uint32_t* d_bucket_offsets, void* stream);

/* ---- directory cache -----------------------------------------------------------
 * AdaptiveGrainDirectoryCache (src/OrleansRuntime/GrainDirectory/AdaptiveGrainDirectoryCache.cs) as a device
 * table consulted by the route kernels for grains whose directory owner is remote: LocalGrainDirectory.LocalLookup's
 * cache branch (LocalGrainDirectory.cs:691-702, GetLocalCacheData :711-717: entries on invalid silos are
 * filtered).  A hit is ORL_ST_HIT with ORL_RF_CACHED (host = the cached activation's silo); a miss stays
 * ORL_ST_REMOTE_OWNER (the FullLookup path).  Cached activations on this context's silos use its activation-handle
 * space [0, n_act) (entries outside it are dropped), so stage 4 groups messages to them like any other; an activation
 * on a silo the context does not host keeps the handle its host's catalog gave it (any value but ORL_NO_ACT: the node
 * exchange delivers such messages to the host rank, whose stage 4 buckets them; in a single context they share the
 * unresolved bucket when the handle is >= n_act).
 * AddOrUpdate: the batch's last writer of a key wins.  Remove = CACHE_INVALIDATION_HEADER handling
 * (InsideGrainClient.cs:298-308).  Expiry / size policy (the maintainer) stays with the host: remove or clear. */
#define ORL_RF_CACHED 0x08u
/* A record the sender addressed from a stale cache entry, re-addressed by the receiver's directory (orl_route_received_device,
 * the node exchange): the reference's NonExistentActivation forward with the old address in the cache-invalidation header
 * (Dispatcher.cs:138-182, 429-487).  The sender should remove the entry (orl_cache_remove_device). */
#define ORL_RF_CACHE_STALE 0x10u
int orl_cache_config(orl_ctx* ctx, uint64_t capacity);
int orl_cache_clear(orl_ctx* ctx);
int orl_cache_add_or_update_device(orl_ctx* ctx, const orl_grain_key* d_keys, const uint32_t* d_acts, const uint8_t* d_silos,
                                   size_t n, void* stream);
int orl_cache_remove_device(orl_ctx* ctx, const orl_grain_key* d_keys, size_t n, uint8_t* d_removed, void* stream);
int orl_cache_count(orl_ctx* ctx, uint64_t* n_out);

/* ---- outbound queues and client gateway buckets ------------------------------
 * Per routed message, the queue OutboundMessageQueue.SendMessage (src/OrleansRuntime/Messaging/
 * OutboundMessageQueue.cs:75-150) hands it to: ORL_OUTQ_REJECT when the route has no target (host) silo
 * (SendRejection, :100-105), ORL_OUTQ_LOOPBACK when the target is the sending silo (InboundQueue, :113-119),
 * ORL_OUTQ_PING / ORL_OUTQ_SYSTEM for those message categories, else the sender index
 * Math.Abs(TargetSilo.GetConsistentHashCode()) % n_senders (:141), or ORL_OUTQ_OVERFLOW where Math.Abs
 * throws (hash == int.MinValue; ORL_E_OVERFLOW's per-message form).  Silo consistent hashes are those given
 * to orl_ring_add_server or orl_silo_hash_set (ORL_OUTQ_UNKNOWN_SILO otherwise). */
#define ORL_OUTQ_LOOPBACK 0xFFFFFFF0u
#define ORL_OUTQ_PING 0xFFFFFFF1u
#define ORL_OUTQ_SYSTEM 0xFFFFFFF2u
#define ORL_OUTQ_REJECT 0xFFFFFFF3u
#define ORL_OUTQ_OVERFLOW 0xFFFFFFF4u
#define ORL_OUTQ_UNKNOWN_SILO 0xFFFFFFF5u
int orl_silo_hash_set(orl_ctx* ctx, uint32_t silo, int32_t consistent_hash);
int orl_outbound_queues_device(orl_ctx* ctx, const orl_msg_hdr* d_msgs, const uint32_t* d_route, size_t n,
                               uint32_t n_senders, uint32_t* d_queue, void* stream);
/* Client side: the gateway bucket of each message, TargetGrain.GetHashCode_Modulo(n_buckets)
 * (src/Orleans/Messaging/ProxiedMessageCenter.cs:222, src/Orleans/IDs/UniqueIdentifier.cs:60-66: C#'s
 * truncating % on the signed uniform hash, made non-negative), so all requests to a grain share a bucket.
 * n_buckets in [1, 2^30] (above that, (key % mod) + mod can wrap and the reference's checked cast throws). */
int orl_client_buckets_device(orl_ctx* ctx, const orl_msg_hdr* d_msgs, size_t n, uint32_t n_buckets, uint32_t* d_bucket,
                              void* stream);

/* ---- message header wire codec ------------------------------------------------
 * Received frames decoded on the device into the orl_msg_hdr records the route kernels read.  A frame is
 * Message.Serialize_Impl's output (src/Orleans/Messaging/Message.cs:915-951): int32 header length, int32 body
 * length, the header bytes of SerializationManager.SerializeMessageHeaders (SerializationManager.cs:1692-1770),
 * the body.  The caller gives each frame's byte offset (the decode offsets IncomingMessageBuffer.TryDecodeMessage
 * walks, IncomingMessageBuffer.cs:94-135); the header is parsed as DeserializeMessageHeaders does
 * (:1773-1853, BinaryTokenStreamReader.TryReadSimpleType :489-582), every value validated as the reference reader
 * validates it, and the routing fields read as the Message getters read them (Message.cs:149, 199-255, 650-666):
 *   target        TARGET_GRAIN (GrainId; a KeyExt grain also gets aux = its uniform hash, ORL_HDR_HASH_VALID)
 *   sending_silo  SENDING_SILO's index in the silo address table, or sender_override (< 255) for every frame
 *   category      CATEGORY (default Ping)
 *   flags         ORL_HDR_ADDRESS_COMPLETE when TARGET_SILO and TARGET_ACTIVATION are set (target_silo = index)
 * d_status[i] (one byte per frame) gives ORL_DEC_*; a non-OK frame's record is all zero and counts in *d_n_bad
 * (device u32, optional; the call zeroes it).  d_bytes must be 4-byte aligned; nbytes is its valid length.
 * The device decoder hands these to the host (ORL_DEC_UNSUPPORTED): SpecifiedType values (registered
 * serializers), a header dictionary nested in a header value, local-kind DateTime values (the result depends on
 * the host time zone), and a TARGET_GRAIN KeyExt that is not strict UTF-8 (its hash re-encodes the decoded
 * string).  Where the reference reader or getter throws: ORL_DEC_MALFORMED. */
#define ORL_DEC_OK 0u
#define ORL_DEC_UNSUPPORTED 1u
#define ORL_DEC_MALFORMED 2u
#define ORL_DEC_UNKNOWN_SILO 3u  /* SENDING_SILO (or TARGET_SILO of a complete address) not in the table */
#define ORL_DEC_NO_TARGET 4u     /* TargetGrain null (absent, null or not a GrainId) */
#define ORL_DEC_NO_SENDER 5u     /* SendingSilo null and no sender_override */
#define ORL_SENDER_FROM_HEADER 0xFFu
/* Silo address table: the serialized SiloAddress (16 IP bytes as BinaryTokenStreamWriter.Write(IPAddress) writes
 * them — IPv4 as 12 zero bytes + 4 — port, generation) of silo index `silo` (< 255).  ip16 NULL removes it. */
int orl_silo_address_set(orl_ctx* ctx, uint32_t silo, const uint8_t* ip16, int32_t port, int32_t generation);
int orl_decode_frames_device(orl_ctx* ctx, const uint8_t* d_bytes, uint64_t nbytes, const uint64_t* d_frame_offsets,
                             size_t n, uint32_t sender_override, orl_msg_hdr* d_out, uint8_t* d_status, uint32_t* d_n_bad,
                             void* stream);
/* Emit: the routed frames re-serialized with the placement applied — Dispatcher.AddressMessage →
 * Message.SetTargetPlacement (src/OrleansRuntime/Core/Dispatcher.cs:555-579, src/Orleans/Messaging/Message.cs:
 * 1079-1096) → Message.Serialize_Impl (:915-951).  For route status HIT the placement is
 * PlacementResult.IdentifySelection (activation d_act_keys[d_act[i]] = its ActivationId key, host silo); for
 * NEW_PLACEMENT it is SpecifyCreation (host silo, ActivationId d_new_act_keys[i] — ActivationId.NewId() is the
 * caller's —, the grain class of the target's type code from orl_grain_type_set).  The header dictionary is
 * updated as .NET's Dictionary does: PRIOR_MESSAGE_ID / PRIOR_MESSAGE_TIMES removed on a new placement or an
 * activation change (free-list slots, reused last-removed first by the keys added next), TARGET_ACTIVATION and
 * TARGET_SILO set (in place if present), and on a new placement IS_NEW_PLACEMENT = true and NEW_GRAIN_TYPE.
 * Other frames are copied unchanged (status says why).  Output frame i starts at d_out_offsets[i] (4-byte aligned,
 * back to back in frame order, padding between frames); *d_out_total = the aligned end; frames that do not fit
 * out_cap are not written (ORL_STAMP_OVERFLOW).  A frame's output never exceeds its input by more than
 * ORL_STAMP_MAX_GROWTH + the longest grain class name.  d_out 4-byte aligned; d_new_act_keys may be NULL when
 * no message is a new placement. */
#define ORL_STAMP_OK 0u
#define ORL_STAMP_COMPLETE 1u     /* TargetAddress already complete: unchanged (Dispatcher.cs:557-558) */
#define ORL_STAMP_SKIPPED 2u      /* route status other than HIT / NEW_PLACEMENT: unchanged, host path */
#define ORL_STAMP_UNSUPPORTED 3u  /* header needs the managed serializer, a string is not byte-canonical (not
                                     strict UTF-8), an unknown grain type / activation handle: unchanged */
#define ORL_STAMP_MALFORMED 4u    /* the reference throws (undecodable header; a TARGET_ACTIVATION that is not an
                                     ActivationId); an invalid frame prefix emits nothing */
#define ORL_STAMP_OVERFLOW 5u     /* past out_cap: not written */
#define ORL_STAMP_MAX_GROWTH 72u
int orl_grain_type_set(orl_ctx* ctx, int32_t type_code, const char* class_name_utf8, size_t len);  /* len 0: remove */
int orl_stamp_frames_device(orl_ctx* ctx, const uint8_t* d_bytes, uint64_t nbytes, const uint64_t* d_frame_offsets,
                            size_t n, const uint32_t* d_route, const uint32_t* d_act, const orl_grain_key* d_act_keys,
                            uint32_t n_act_keys, const orl_grain_key* d_new_act_keys, uint8_t* d_out, uint64_t out_cap,
                            uint64_t* d_out_offsets, uint64_t* d_out_total, uint8_t* d_status, void* stream);

/* ---- multi-GPU exchange support --------------------------------------------
 * Stages 1-2 + stable partition by destination rank (rank_of_silo[owner]).  Messages whose owner is
 * null / system target / complete stay on the sending rank (dest = my_rank).  Writes the partitioned
 * headers to d_out (n entries, rank-major, arrival order kept), the source index of each to
 * d_src_index, and per-rank counts to d_counts[nranks] (device, uint64). */
int orl_partition_by_owner_device(orl_ctx* ctx, const orl_msg_hdr* d_in, size_t n, uint32_t opts,
                                  const uint8_t* rank_of_silo, uint32_t nranks, uint32_t my_rank,
                                  orl_msg_hdr* d_out, uint32_t* d_src_index, uint64_t* d_counts, void* stream);
/* One-pass form for the exchange: the headers for rank r go to the padded send region
 * d_out[r * stride .. r * stride + d_counts[r]) (stride >= n; d_out holds nranks * stride headers), so
 * each region can be sent as is (grouped send/recv, RCCL over xGMI).  Same order and counts as
 * orl_partition_by_owner_device; d_src_index may be NULL (same padded layout otherwise).
 * Reference: OutboundMessageQueue.SendMessage's per-target-silo queues (OutboundMessageQueue.cs:137-145). */
int orl_partition_by_owner_padded_device(orl_ctx* ctx, const orl_msg_hdr* d_in, size_t n, uint32_t opts,
                                         const uint8_t* rank_of_silo, uint32_t nranks, uint32_t my_rank, size_t stride,
                                         orl_msg_hdr* d_out, uint32_t* d_src_index, uint64_t* d_counts, void* stream);
/* As orl_partition_by_owner_padded_device, writing 16-byte orl_wire_msg records (half the exchange
 * bytes).  *d_status (device u32) is set to 0, or to 1 if some message of the batch has no compact form
 * (then the records are invalid and the caller uses the 32-byte form for this batch); | ORL_PART_LOOKBACK_FAILED when the
 * partition's decoupled look-back gave up waiting on an earlier tile (record positions and counts invalid: a device
 * fault, not a property of the batch).
 * Every one-pass partition of a context (orl_partition_*_padded/compact/narrow_device) must be enqueued on ONE stream:
 * the look-back state is reused launch after launch (tile tickets and epochs are mirrored on the host).  A look-back
 * failure of the 32-byte form, which has no status word, is reported by orl_ctx_query(ORL_Q_PART_ERROR). */
#define ORL_PART_LOOKBACK_FAILED 0x4u
#define ORL_PART_CACHED 0x8u  /* (node hop 1) the sender's directory cache addressed some message of the chunk */
#define ORL_PART_KEYEXT 0x10u    /* (node hop 1, orl_node_route_batch_keyext_device) a KeyExt string travels with the chunk */
#define ORL_PART_EXT_FULL 0x20u  /* (node hop 1) a destination's KeyExt string region overflowed: ORL_E_CAPACITY on every rank */
int orl_partition_compact_device(orl_ctx* ctx, const orl_msg_hdr* d_in, size_t n, uint32_t opts,
                                 const uint8_t* rank_of_silo, uint32_t nranks, uint32_t my_rank, size_t stride,
                                 orl_wire_msg* d_out, uint32_t* d_src_index, uint64_t* d_counts, uint32_t* d_status,
                                 void* stream);
/* orl_route_batch_device over received compact records (the owner side of the exchange). */
int orl_route_compact_device(orl_ctx* ctx, const orl_wire_msg* d_in, size_t n, uint32_t opts, uint32_t* d_route,
                             uint32_t* d_act, uint32_t* d_order, uint32_t* d_bucket_offsets, void* stream);
/* The wire types of the 8-byte form (n <= ORL_MAX_WIRE_TYPES TypeCodeData values; n = 0 turns the form off).  Every
 * rank of a node must set the same list in the same order; the node compares a digest of it before each chunk uses
 * the 8-byte form and falls back to the 16-byte one when ranks differ. */
int orl_wire_types_set(orl_ctx* ctx, uint32_t n, const uint64_t* type_code_data);
/* As orl_partition_compact_device, writing 8-byte orl_wire8 records (a quarter of the header bytes).  *d_status (device
 * u32): bit 0 = some message has no 16-byte form, bit 1 = some message has no 8-byte form (records invalid when bit 1
 * is set: re-partition in the 16-byte form, or the 32-byte one when bit 0 is set too). */
int orl_partition_narrow_device(orl_ctx* ctx, const orl_msg_hdr* d_in, size_t n, uint32_t opts,
                                const uint8_t* rank_of_silo, uint32_t nranks, uint32_t my_rank, size_t stride,
                                orl_wire8* d_out, uint32_t* d_src_index, uint64_t* d_counts, uint32_t* d_status,
                                void* stream);
/* orl_route_batch_device over received 8-byte records, decoded with this context's wire types. */
int orl_route_narrow_device(orl_ctx* ctx, const orl_wire8* d_in, size_t n, uint32_t opts, uint32_t* d_route,
                            uint32_t* d_act, uint32_t* d_order, uint32_t* d_bucket_offsets, void* stream);
/* The node's hop-1 partition with the sender's directory cache (round 5): as orl_partition_narrow/compact_device (fmt =
 * the record width, 8 / 16 / 32), except that a message whose directory owner is on another rank and whose grain the
 * context's cache holds on a valid silo (orl_cache_add_or_update_device; LocalLookup's non-owner branch,
 * LocalGrainDirectory.cs:690-717) is addressed here — its record goes to the rank of the cached silo (rank_of_silo), with
 * that silo as the record's target silo — and d_act_out (device u32, the same padded regions as d_out: stride per rank)
 * gets its cached activation handle; every other record gets ORL_NO_ACT.  *d_status also gets ORL_PART_CACHED when a
 * message was addressed.  Without a populated cache it is the plain partition (d_act_out all ORL_NO_ACT).  Replaces
 * the non-owner silo's cache lookup + Dispatcher.AddressMessage + the send to TargetSilo (Dispatcher.cs:555-579,
 * OutboundMessageQueue.cs:113-145). */
int orl_partition_cached_device(orl_ctx* ctx, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const uint8_t* rank_of_silo,
                                uint32_t nranks, uint32_t my_rank, size_t stride, void* d_out, uint32_t fmt,
                                uint32_t* d_act_out, uint64_t* d_counts, uint32_t* d_status, void* stream);
/* Stages 1-3 of received hop-1 records (fmt 8 / 16 / 32) with their act lane: a record whose lane entry is not ORL_NO_ACT
 * was addressed by its sender's cache.  When this context holds the grain's directory partition, the record is routed by
 * the directory and keeps HIT | ORL_RF_CACHED only if the directory holds that handle on that silo; otherwise it gets the
 * directory's word | ORL_RF_CACHE_STALE (the receiving silo's NonExistentActivation forward, Dispatcher.cs:138-182).  When
 * it does not, the record gets HIT | ORL_RF_CACHED with its target silo as host and that handle, without a probe.  The
 * others are routed as orl_route_*_device do.  No stage 4 (ORL_OPT_NO_BUCKETS implied; orl_bucket_device follows over the
 * hosted set). */
int orl_route_received_device(orl_ctx* ctx, const void* d_in, uint32_t fmt, size_t n, uint32_t opts, const uint32_t* d_in_act,
                              uint32_t* d_route, uint32_t* d_act, void* stream);

/* Stage 4 alone: group already-routed messages by activation handle, FIFO inside each bucket (ActivationData.EnqueueMessage,
 * ActivationData.cs:483-514) — the receiving silo's side when the routing ran elsewhere (node hop 2).  Same outputs as
 * orl_route_batch_device's order / bucket_offsets for these handles (ORL_NO_ACT and handles >= n_act: bucket n_act). */
int orl_bucket_device(orl_ctx* ctx, const uint32_t* d_act, size_t n, uint32_t* d_order, uint32_t* d_bucket_offsets, void* stream);

/* ---- device memory for callers without a GPU runtime (the P/Invoke silo) ---------------------------------
 * A .NET host drives the *_device entry points through these: allocate HBM on the context's device, copy host arrays
 * in and out on a stream (a NULL stream is the context's own), wait.  orl_host_register page-locks a caller array once
 * (a pinned GCHandle buffer) so copies from / to it run at full PCIe rate and asynchronously.  Reference call sites:
 * the per-message managed objects these batches replace (Message header dictionary, Message.cs:90). */
int orl_device_alloc(orl_ctx* ctx, size_t bytes, void** d_out);
int orl_device_free(orl_ctx* ctx, void* d_ptr);
int orl_copy_to_device(orl_ctx* ctx, void* d_dst, const void* h_src, size_t bytes, void* stream);
int orl_copy_to_host(orl_ctx* ctx, void* h_dst, const void* d_src, size_t bytes, void* stream);
/* Device-to-device copy on `stream` (e.g. a node result's arrays into the caller's own buffers before the next batch). */
int orl_copy_on_device(orl_ctx* ctx, void* d_dst, const void* d_src, size_t bytes, void* stream);
int orl_stream_sync(orl_ctx* ctx, void* stream);
int orl_host_register(orl_ctx* ctx, void* h_ptr, size_t bytes);
int orl_host_unregister(orl_ctx* ctx, void* h_ptr);

/* ---- follower graph held by the context + host-array fan-out (SURVEY §8(b) orl_fanout_batch) -------------
 * orl_csr_set uploads a follower graph once (csr_off[n_nodes + 1], csr_tgt[n_edges]; follower of CSR entry j = the
 * long-key grain (follower_tcd, 0, csr_tgt[j])); orl_fanout_batch then expands host publisher arrays against it and
 * returns every output in host arrays (route/act/order: cap entries; pub_offsets[n_pub + 1]; bucket_offsets[n_act + 2]),
 * *n_out = the emitted count (ORL_E_CAPACITY, nothing written, when it exceeds cap).  Reference:
 * ChirperAccount.PublishMessage (Samples/Chirper/ChirperGrains/ChirperAccount.cs:154-157). */
int orl_csr_set(orl_ctx* ctx, const uint64_t* csr_off, size_t n_nodes, const uint32_t* csr_tgt, size_t n_edges);
int orl_fanout_batch(orl_ctx* ctx, const uint32_t* pubs, const uint8_t* pub_silo, size_t n_pub, uint64_t follower_tcd,
                     uint32_t opts, uint64_t* pub_offsets, uint32_t* route, uint32_t* act, uint32_t* order,
                     uint32_t* bucket_offsets, size_t cap, uint64_t* n_out);

/* ---- node: the silos of one GPU in a multi-GPU node (SURVEY §8(b) orl_node_create, §8(e)) ------------------
 * One process per GPU; a node binds a routing context (this GPU's directory partitions) to the other ranks.  Per batch
 * (orl_node_route_batch_device, called by every rank with its own local batch, in lockstep):
 *   hop 1  stages 1-2 + stable partition of the local batch by the rank of each message's directory owner (messages
 *          that need no directory stay: complete addresses, system targets, null owners), a counts all-gather, and a
 *          grouped send/recv of the per-rank regions — 8-B orl_wire8 records when every rank set the same wire types
 *          and every message of the chunk has that form, else 16-B orl_wire_msg records when they all have that form,
 *          32-B headers otherwise.  The batch is cut into `chunks` pieces: the exchange of one overlaps the
 *          routing (stages 1-3) of the previous one.  Replaces OutboundMessageQueue.SendMessage's per-target-silo
 *          sender queues (OutboundMessageQueue.cs:113-145) + the remote directory lookup (LocalGrainDirectory.cs:719-765).
 *   owner  stages 1-3 over the received records; the owned set is the received blocks in (chunk, source rank) order.
 *   hop 2  messages whose activation is hosted on another rank (route word host silo; Dispatcher.TransportMessage,
 *          Dispatcher.cs:618-622) travel on with their route word and activation handle, in owner order.  Skipped (no
 *          collective beyond one counts all-gather) when no rank has anything to forward.
 *   host   stage 4 over the hosted messages: per-activation FIFO by (source rank, source order), so per-sender order
 *          holds (a sender's messages originate on one rank).
 * transport ORL_TRANSPORT_RCCL: RCCL over xGMI (group_id = the ncclUniqueId from orl_node_unique_id on rank 0, shared out
 * of band); ORL_TRANSPORT_LOCAL: the ranks are nodes of one process (same group_id bytes), exchanging by device copies —
 * a one-GPU rehearsal of the protocol for tests.  Every rank must use the same config apart from `rank`. */
#define ORL_NODE_ID_BYTES 128u
#define ORL_TRANSPORT_RCCL 0u
#define ORL_TRANSPORT_LOCAL 1u
#define ORL_NODE_WIDE_ONLY 0x1u    /* always exchange 32-B headers */
#define ORL_NODE_SPLIT_COMM 0x2u   /* RCCL: run the counts all-gathers on a second communicator (ncclCommSplit) and stream,
                                      concurrently with the previous chunk's send/recv; off by default.  Every rank must set
                                      the same flags (checked at creation: ranks that disagree all fail with ORL_E_INVALID) */
#define ORL_NODE_MAX_RANKS 8u
#define ORL_NODE_MAX_CHUNKS 16u
typedef struct orl_node_config {
    uint32_t abi_version;
    uint32_t nranks;
    uint32_t rank;
    uint32_t transport;              /* ORL_TRANSPORT_* */
    uint8_t group_id[ORL_NODE_ID_BYTES];
    uint8_t rank_of_silo[256];       /* rank hosting each silo index */
    uint64_t max_batch;              /* messages a rank originates per batch */
    uint64_t max_recv;               /* messages a rank may own, and host, per batch */
    uint32_t chunks;                 /* 1 .. ORL_NODE_MAX_CHUNKS */
    uint32_t flags;                  /* ORL_NODE_* */
} orl_node_config;

typedef struct orl_node_result {
    uint64_t n_owned;                /* messages routed here as directory owner (hop 1 receive) */
    uint64_t n_hosted;               /* messages hosted here (bucketed here) */
    uint64_t n_forwarded;            /* of n_owned, sent on to another rank in hop 2 */
    uint64_t n_sent_remote;          /* of the local batch, sent to another rank in hop 1 */
    uint32_t hop2;                   /* 1 if hop 2 moved messages between ranks in this batch */
    uint32_t n_segments;             /* the hosted messages' records: orl_node_segment 0 .. n_segments-1, back to back */
    const uint32_t* route;           /* device [n_hosted]; valid until the next batch */
    const uint32_t* act;             /* device [n_hosted] */
    const uint32_t* order;           /* device [n_hosted]: hosted-message indices grouped per activation, FIFO */
    const uint32_t* bucket_offsets;  /* device [n_act + 2] */
} orl_node_result;

typedef struct orl_node orl_node;
int orl_node_unique_id(uint8_t id[ORL_NODE_ID_BYTES]);
int orl_node_create(orl_ctx* ctx, const orl_node_config* cfg, orl_node** out);
int orl_node_destroy(orl_node* node);
const char* orl_node_last_error(const orl_node* node);
/* Deadline of every host wait of the exchange, in ms (> 0).  Every rank should use the same value. */
int orl_node_set_timeout(orl_node* node, uint32_t ms);
/* One batch (device headers, n <= max_batch).  The outputs are complete on `stream` when the call returns (the call
 * waits on the host for each chunk's counts; the routing work may still run).
 * Failure is collective and bounded: every host wait of the exchange (the counts all-gathers, the hop-2 exchange, the
 * LOCAL transport's barriers) has a deadline (orl_node_set_timeout; default 120 s, ORL_NODE_TIMEOUT_MS overrides) and
 * RCCL's asynchronous error is polled while waiting.  A rank that misses it, or sees an RCCL error, aborts the
 * communicator (ncclCommAbort) and returns ORL_E_STATE, naming the chunk and the head words it saw in
 * orl_node_last_error; the node is then broken (every later batch returns ORL_E_STATE; destroy it and build a new one).
 * A partition look-back failure on any rank (ORL_PART_LOOKBACK_FAILED, carried in the all-gathered status words) makes
 * every rank return ORL_E_DEVICE for that chunk. */
int orl_node_route_batch_device(orl_node* node, const orl_msg_hdr* d_in, size_t n, uint32_t opts, orl_node_result* out,
                                void* stream);
/* The same with the batch's KeyExt strings (round 6): d_ext[i] locates message i's extension in d_blob (device, blob_bytes
 * long; read for KeyExt messages only), as orl_route_keyext_device takes them.  A KeyExt message without ORL_HDR_HASH_VALID
 * gets its uniform hash from the bytes at the sender (its owner is that hash's ring owner, UniqueKey.cs:288-294); the batch
 * is exchanged as 32-B records with each KeyExt message's string beside it, and the owner resolves it in its KeyExt table
 * (HIT / placement / IsValidSilo as orl_route_keyext_device: LocalGrainDirectory.cs:719-765 with the whole GrainId).  Every
 * rank calls one of the two entry points per batch; a rank without strings takes part in the string lanes of the
 * chunks another rank's strings travel in.  A KeyExt string region of a sender (max(blob_bytes, 4096) bytes per
 * destination per chunk) that overflows fails the chunk on every rank with ORL_E_CAPACITY. */
int orl_node_route_batch_keyext_device(orl_node* node, const orl_msg_hdr* d_in, size_t n, uint32_t opts, const orl_ext_ref* d_ext,
                                       const uint8_t* d_blob, uint64_t blob_bytes, orl_node_result* out, void* stream);
/* A multicast batch across the node (config 4 sharded by publisher): every rank expands its own publishes
 * (orl_fanout_expand_device into a node buffer of max_batch records) and routes the emitted messages as
 * orl_node_route_batch_device does.  *total: in = the exact emitted count with ORL_OPT_TOTAL_GIVEN, out = the count. */
int orl_node_fanout_batch_device(orl_node* node, const uint64_t* d_csr_off, const uint32_t* d_csr_tgt,
                                 const orl_grain_key* d_follower_keys, uint64_t follower_tcd, const uint32_t* d_pubs,
                                 const uint8_t* d_pub_silo, size_t n_pub, uint32_t opts, uint64_t* d_pub_offsets,
                                 uint64_t* total, orl_node_result* out, void* stream);
/* Record segment i of the last batch's hosted messages: device pointer, message count, record width (8 = orl_wire8 in
 * the context's wire types, 16 = orl_wire_msg, 32 = orl_msg_hdr).  Segments start 32-byte aligned. */
int orl_node_segment(const orl_node* node, uint32_t i, const void** d_records, uint64_t* count, uint32_t* width);
/* What the last batch of the node moved and waited for (measurement; the silo's statistics counters).  comm_count: ranks
 * of the RCCL communicator (ncclCommCount), or of the LOCAL group.  bytes_sent[r]: exchange bytes this rank sent to rank r
 * in hop 1 + hop 2 (its own share, copied locally, at r = this rank).  host_wait_us: time the host spent in the exchange's
 * bounded waits (the counts all-gathers, the LOCAL barriers, the hop-2 exchange), host_waits: how many. */
typedef struct orl_node_stats {
    uint32_t comm_count;
    uint32_t chunks;                          /* hop-1 chunks of the batch */
    uint64_t bytes_sent[ORL_NODE_MAX_RANKS];
    uint64_t host_wait_us;
    uint64_t host_waits;
    uint32_t exchange_mode;                   /* ORL_NODE_MODE_*: where the counts all-gathers run */
    uint32_t reserved;
} orl_node_stats;
#define ORL_NODE_MODE_SPLIT_COMM 0x1u  /* RCCL: on the split communicator (ORL_NODE_SPLIT_COMM) */
#define ORL_NODE_MODE_HEAD_STREAM 0x2u /* on a stream of their own (LOCAL always; RCCL only with the split communicator);
                                          otherwise queued on the exchange stream behind the previous chunk's send/recv */
int orl_node_get_stats(const orl_node* node, orl_node_stats* out);

/* The protocol's host decisions, as orl_node_route_batch_device takes them after each all-gather: exposed for hosts that
 * run the exchange over a transport of their own (orl_partition_*_padded/compact/narrow_device, the route entry points,
 * orl_bucket_device + these two), and for the multi-process CPU tests.  ORL_NODE_HEAD_WORDS u64 per rank are
 * all-gathered before each exchange.  Hop 1 (one per chunk): [0, nranks) records for each destination rank, [8] the
 * partition status word (bit 0 = a message lacks the 16-B form, bit 1 = lacks the 8-B form, ORL_PART_LOOKBACK_FAILED,
 * ORL_PART_CACHED),
 * [9] the record width the rank wrote (bits 56-63: 8 / 16 / 32) | its wire-type digest (bits 0-55, ORL_Q_WIRE_DIGEST),
 * the rest zero.  Hop 2: [0, nranks) routed messages whose activation each rank hosts (ORL_ROUTE_HOST's rank; no host:
 * the owner), the rest zero.  heads = nranks x ORL_NODE_HEAD_WORDS words in rank order. */
#define ORL_NODE_HEAD_WORDS 16u
typedef struct orl_node_chunk_plan {
    uint32_t width;                      /* every rank exchanges the chunk in this record width: 8, 16 or 32 */
    uint32_t rewrite;                    /* this rank wrote another width: partition the chunk again in `width` */
    uint64_t send[ORL_NODE_MAX_RANKS];   /* records to each rank */
    uint64_t recv[ORL_NODE_MAX_RANKS];   /* records from each rank, received back to back in rank order */
    uint64_t n_recv;
    uint32_t act_lane;                   /* some rank's directory cache addressed a record (ORL_PART_CACHED): every rank
                                            sends a u32 activation handle per record beside the records (ORL_NO_ACT: not
                                            addressed), and the receivers route addressed records without a probe */
    uint32_t ext_lane;                   /* some rank sent KeyExt strings (ORL_PART_KEYEXT; 32-B records): every rank sends an
                                            orl_ext_ref per record ({~0, ~0}: none) and its strings, head words [10, 14) =
                                            the string bytes to each rank (u32 each, rank r in word 10 + r / 2, bits
                                            32 * (r & 1)); ORL_PART_EXT_FULL on any rank gives ORL_E_CAPACITY */
} orl_node_chunk_plan;
/* written = the width this rank partitioned the chunk in; owned_total[nranks] = every rank's receive total over the
 * batch's earlier chunks (zero before chunk 0; updated).  ORL_E_CAPACITY when a rank would own more than max_recv and
 * ORL_E_DEVICE when a rank's partition look-back failed: every rank gets the same result. */
int orl_node_plan_chunk(const uint64_t* heads, uint32_t nranks, uint32_t me, uint32_t written, uint64_t max_recv,
                        uint64_t* owned_total, orl_node_chunk_plan* out);
typedef struct orl_node_hop2_plan {
    uint32_t forward;                    /* 1 if any rank forwards messages (else every rank buckets its owned set) */
    uint32_t width;                      /* record width of a forwarded set */
    uint64_t send[ORL_NODE_MAX_RANKS];   /* forwarded {record, route word, activation} to each rank (own: kept) */
    uint64_t recv[ORL_NODE_MAX_RANKS];
    uint64_t n_hosted;                   /* messages this rank buckets */
    uint64_t n_forwarded;                /* of its owned set, sent to another rank */
} orl_node_hop2_plan;
/* n_owned = this rank's owned (routed) messages; width_mask = the widths of its owned segments (bit 0 = 8, 1 = 16,
 * 2 = 32).  ORL_E_CAPACITY (on every rank) when a rank would host more than max_recv. */
int orl_node_plan_hop2(const uint64_t* heads, uint32_t nranks, uint32_t me, uint64_t n_owned, uint32_t width_mask,
                       uint64_t max_recv, orl_node_hop2_plan* out);

int orl_sync(orl_ctx* ctx);

/* ---- introspection for benchmarks / profiling ------------------------------------------------ */
/* With timing enabled, every orl_route_batch_device / orl_fanout_route*_device brackets its route kernel (stages 1-3), its bucketing
 * kernels (stage 4) and the whole call with HIP events on the submission stream (no host sync per batch;
 * up to ORL_TIMING_SLOTS batches are kept).  orl_set_timing(ctx, 1) clears the record.
 * orl_timing_summary waits for the last recorded batch and returns the per-batch averages in ms. */
/* Context state, as the next route launch sees it (pending host-side changes are uploaded first).
 *   ORL_Q_PROBE_FORM    directory form k_route probes: 8 / 16 (compact copies built by the host upload), 17 (16-B copy
 *                       rebuilt on the device after device mutations, checked by its flag), 32 (the full 32-B table)
 *   ORL_Q_FULL_UPLOADS  whole-partition uploads so far; ORL_Q_SLOT_PATCHES in-place uploads of host-changed slots */
#define ORL_Q_PROBE_FORM 1u
#define ORL_Q_FULL_UPLOADS 2u
#define ORL_Q_SLOT_PATCHES 3u
#define ORL_Q_DEVICE 4u       /* the context's HIP device ordinal */
#define ORL_Q_N_ACT 5u        /* orl_config.n_act */
#define ORL_Q_MAX_BATCH 6u    /* messages the scratch is sized for */
#define ORL_Q_RANK_MODE 7u    /* stage-4 stable ranking on this device: bit 0 = ballot match (else LDS atomics), bit 1 = the
                                 lane-order self-check failed (ballot forced) */
#define ORL_Q_WIRE_DIGEST 8u  /* FNV-1a digest of the wire types (orl_wire_types_set), 0 when the 8-B form is off */
#define ORL_Q_PART_ERROR 9u   /* 1 if a one-pass partition's look-back gave up since the last query (read and cleared;
                                 synchronises the context's device) */
#define ORL_Q_HOT_KEY 10u     /* stage 4's hot key: the activation handle (n_act = the unresolved bucket) whose messages the
                                 next batch of >= 2^20 messages places without sorting, picked from the last such batch
                                 (>= 1/32 of its messages); 0xFFFFFFFF = none.  Outputs never depend on it.  Synchronises. */
#define ORL_Q_HOT_BATCHES 11u /* batches that took stage 4's hot-key path so far (the launcher decides from a mapped host copy
                                 of the last pick, which may lag the device by the batches still queued) */
#define ORL_Q_STAGE4_ERROR 12u /* 1 if a stage-4 look-back gave up since the last query (the two-level plan's fused level 2 on
                                  a skewed batch, the LSD plan's single-sweep passes): that batch's order / offsets are not
                                  valid.  Only a device fault can cause it.  Read and cleared; synchronises the device. */
int orl_ctx_query(orl_ctx* ctx, uint32_t what, uint64_t* value);
/* Stage-4 ranking: 0 = one LDS atomic per element (its lane order is checked by a self-test per device at the first
 * context creation; ORL_RANK_MODE=ballot forces the other), 1 = ballot match.  Process-wide per device; for validation. */
int orl_ctx_set_rank_mode(orl_ctx* ctx, uint32_t mode);

#define ORL_TIMING_SLOTS 256u
int orl_set_timing(orl_ctx* ctx, int enable);
int orl_timing_summary(const orl_ctx* ctx, uint32_t* n_batches, float* route_kernel_ms, float* bucket_ms,
                       float* total_ms);

#ifdef __cplusplus
}
#endif
#endif /* ORLEANS_ROUTE_H */
