/* orl_host_demo.c — a plain C host of liborleans_route.so: the call sequence a .NET silo makes through P/Invoke
 * (INTEGRATION.md), with no Python and no GPU runtime of its own.  Test infrastructure: it links the CPU oracle
 * (oracle/liborleans_cpu_ref.so) as the checker.
 *
 *   1. context + silo table + ring from SiloAddress consistent hashes (orl_silo_consistent_hash of "10.0.0.s:11111")
 *   2. RegisterSingleActivation of 50k long-key grains (orl_dir_insert_single), type code = CalculateIdHash(class name)
 *   3. a batch of 200k headers (~9 % never registered, some complete addresses) through
 *      a. orl_route_batch on page-locked host arrays (orl_host_register),
 *      b. device buffers it allocates through the library (orl_device_alloc / orl_copy_to_device /
 *         orl_route_batch_device / orl_copy_to_host / orl_stream_sync), and
 *      c. the narrow call: the same batch as 8-byte orl_wire8 records (orl_wire_types_set with the grain class),
 *         orl_route_batch_narrow on page-locked arrays
 *   4. all three compared word for word with the oracle's route + stable bucketing of the same batch.
 *   5. KeyExt (string-key) grains (argv[1]: the golden KeyExt cases, one "tcd n0 n1 uniform hex-utf8" per line, written by
 *      tests/test_c_host.py from tests/golden/jenkins.json): their uniform hashes (orl_keyext_uniform_hash), registration
 *      (orl_dir_insert_keyext + orl_dir_lookup_keyext_host), then a batch through orl_route_keyext_device on library
 *      buffers — every registered grain HIT on its silo with its handle, the same keys with an unregistered extension
 *      placed PreferLocal, half the messages with the precomputed hash (ORL_HDR_HASH_VALID), half hashed by the kernel;
 *      owners from the oracle's ring, order / offsets from the oracle's stable bucketing.
 *
 * Build: gcc -std=c11 -O2 -I include tests/c_host/orl_host_demo.c -L orleans_amd -lorleans_route
 *        -L oracle -lorleans_cpu_ref -Wl,-rpath,<dirs> -o tools/orl_host_demo        (tests/test_c_host.py does this)
 * Exit status 0 = every word equal; it prints what differed otherwise. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "orleans_route.h"

/* the oracle's C entry points (oracle/cpu_ref.cpp) */
typedef struct ref_cluster {
    uint32_t n_silos, ring_n;
    int32_t ring_hash[256];
    uint8_t ring_silo[256], running[256], functional[256], local[256];
    uint32_t seed, policy;
} ref_cluster;
int ref_ring_add(ref_cluster* cl, uint32_t silo, int32_t hash);
void* ref_dir_new(void);
void ref_dir_free(void* d);
int ref_register(const ref_cluster* cl, void* dir, const orl_grain_key* keys, const uint32_t* acts, const uint8_t* silos,
                 size_t n, uint8_t* status, uint32_t* wact, uint8_t* wsilo);
int ref_route(const ref_cluster* cl, void* dir, const orl_msg_hdr* in, size_t n, uint32_t opts, uint32_t* route, uint32_t* act);
int ref_bucket(const uint32_t* act, size_t n, uint32_t n_act, uint32_t* order, uint32_t* offsets);

#define N_SILOS 8
#define N_GRAINS 50000
#define N_MSGS 200000

static uint64_t splitmix(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int check(orl_ctx* ctx, int rc, const char* what) {
    if (rc != ORL_OK) {
        fprintf(stderr, "%s failed: %d (%s)\n", what, rc, ctx ? orl_last_error(ctx) : "");
        exit(2);
    }
    return rc;
}

static int compare(const char* what, const uint32_t* got, const uint32_t* exp, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (got[i] != exp[i]) {
            fprintf(stderr, "%s differs at %zu: %u vs %u\n", what, i, got[i], exp[i]);
            return 1;
        }
    return 0;
}

#define MAX_KX 64

/* step 5: returns nonzero on any difference (the golden cases' file is argv[1]) */
static int keyext_step(orl_ctx* ctx, const ref_cluster* cl, const char* path) {
    FILE* f = fopen(path, "r");
    if (!f) {
        fprintf(stderr, "cannot open %s\n", path);
        return 1;
    }
    static orl_grain_key keys[2 * MAX_KX];
    static uint32_t uni[MAX_KX], acts[MAX_KX];
    static uint8_t blob[2 * MAX_KX * 512], silos[MAX_KX];
    static orl_ext_ref ext[2 * MAX_KX];
    size_t nk = 0, used = 0;
    unsigned long long tcd, n0, n1;
    unsigned u;
    char hex[1024];
    while (nk < MAX_KX && fscanf(f, "%llx %llx %llx %u %1023s", &tcd, &n0, &n1, &u, hex) == 5) {
        const size_t len = strcmp(hex, "-") == 0 ? 0 : strlen(hex) / 2;
        keys[nk].type_code_data = tcd;
        keys[nk].n0 = n0;
        keys[nk].n1 = n1;
        uni[nk] = u;
        ext[nk].off = (uint32_t)used;
        ext[nk].len = (uint32_t)len;
        for (size_t b = 0; b < len; ++b) {
            unsigned v;
            sscanf(hex + 2 * b, "%2x", &v);
            blob[used + b] = (uint8_t)v;
        }
        used += len;
        acts[nk] = 100 + (uint32_t)nk;
        silos[nk] = (uint8_t)(nk % N_SILOS);
        ++nk;
    }
    fclose(f);
    int bad = nk == 0;
    for (size_t i = 0; i < nk; ++i) {
        const uint32_t h = orl_keyext_uniform_hash(&keys[i], (const char*)blob + ext[i].off, ext[i].len);
        if (h != uni[i]) {
            fprintf(stderr, "KeyExt uniform hash %zu: %u vs golden %u\n", i, h, uni[i]);
            bad = 1;
        }
    }
    uint8_t st[MAX_KX];
    check(ctx, orl_dir_insert_keyext(ctx, keys, ext, blob, used, acts, silos, nk, NULL, NULL, st), "orl_dir_insert_keyext");
    uint32_t la[MAX_KX];
    uint8_t ls[MAX_KX];
    check(ctx, orl_dir_lookup_keyext_host(ctx, keys, ext, blob, used, nk, la, ls), "orl_dir_lookup_keyext_host");
    for (size_t i = 0; i < nk; ++i)
        if (st[i] != ORL_INS_INSERTED || la[i] != acts[i] || ls[i] != silos[i]) {
            fprintf(stderr, "KeyExt registration %zu: status %u, lookup %u / %u\n", i, st[i], la[i], ls[i]);
            bad = 1;
        }
    /* the same keys with an unregistered extension (the string + "!"): another grain */
    for (size_t i = 0; i < nk; ++i) {
        keys[nk + i] = keys[i];
        ext[nk + i].off = (uint32_t)used;
        ext[nk + i].len = ext[i].len + 1;
        memcpy(blob + used, blob + ext[i].off, ext[i].len);
        blob[used + ext[i].len] = '!';
        used += ext[i].len + 1;
    }
    const size_t m = 2 * nk;
    static orl_msg_hdr msgs[2 * MAX_KX];
    static uint32_t er[2 * MAX_KX], ea[2 * MAX_KX], eo[2 * MAX_KX], ef[N_GRAINS + 2];
    static uint32_t route[2 * MAX_KX], act[2 * MAX_KX], order[2 * MAX_KX], off[N_GRAINS + 2];
    for (size_t i = 0; i < m; ++i) {
        memset(&msgs[i], 0, sizeof msgs[i]);
        msgs[i].target = keys[i];
        msgs[i].sending_silo = (uint8_t)((i * 3) % N_SILOS);
        msgs[i].category = 2;
        if (i % 2 == 0) {  /* the precomputed hash travels with the header; the others are hashed from the bytes */
            msgs[i].flags = ORL_HDR_HASH_VALID;
            msgs[i].aux = orl_keyext_uniform_hash(&keys[i], (const char*)blob + ext[i].off, ext[i].len);
        }
    }
    /* expected: the owner is the ring owner of the KeyExt hash (the oracle's KEYEXT_UNRESOLVED word carries it) */
    static orl_msg_hdr hv[2 * MAX_KX];
    for (size_t i = 0; i < m; ++i) {
        hv[i] = msgs[i];
        hv[i].flags = ORL_HDR_HASH_VALID;
        hv[i].aux = orl_keyext_uniform_hash(&keys[i], (const char*)blob + ext[i].off, ext[i].len);
    }
    void* dir = ref_dir_new();
    ref_route(cl, dir, hv, m, 0, er, ea);
    ref_dir_free(dir);
    for (size_t i = 0; i < m; ++i) {
        const uint32_t owner = er[i] & 0xFF, me = msgs[i].sending_silo;
        if (((er[i] >> 16) & 0xFF) != ORL_ST_KEYEXT_UNRESOLVED) bad = 1;
        if (i < nk) {
            const uint32_t s = silos[i];
            er[i] = owner | (s << 8) | (ORL_ST_HIT << 16) | ((s == me ? ORL_RF_LOOPBACK : 0u) << 24);
            ea[i] = acts[i];
        } else {
            er[i] = owner | (me << 8) | (ORL_ST_NEW_PLACEMENT << 16) | ((ORL_RF_NEW_PLACEMENT | ORL_RF_LOOPBACK) << 24);
            ea[i] = ORL_NO_ACT;
        }
    }
    ref_bucket(ea, m, N_GRAINS, eo, ef);
    void *d_in, *d_ext, *d_blob, *d_route, *d_act, *d_order, *d_off;
    check(ctx, orl_device_alloc(ctx, m * sizeof *msgs, &d_in), "orl_device_alloc");
    check(ctx, orl_device_alloc(ctx, m * sizeof *ext, &d_ext), "orl_device_alloc");
    check(ctx, orl_device_alloc(ctx, used, &d_blob), "orl_device_alloc");
    check(ctx, orl_device_alloc(ctx, m * 4, &d_route), "orl_device_alloc");
    check(ctx, orl_device_alloc(ctx, m * 4, &d_act), "orl_device_alloc");
    check(ctx, orl_device_alloc(ctx, m * 4, &d_order), "orl_device_alloc");
    check(ctx, orl_device_alloc(ctx, (N_GRAINS + 2) * 4, &d_off), "orl_device_alloc");
    check(ctx, orl_copy_to_device(ctx, d_in, msgs, m * sizeof *msgs, NULL), "orl_copy_to_device");
    check(ctx, orl_copy_to_device(ctx, d_ext, ext, m * sizeof *ext, NULL), "orl_copy_to_device");
    check(ctx, orl_copy_to_device(ctx, d_blob, blob, used, NULL), "orl_copy_to_device");
    check(ctx, orl_route_keyext_device(ctx, (const orl_msg_hdr*)d_in, m, 0, (const orl_ext_ref*)d_ext, (const uint8_t*)d_blob,
                                       used, (uint32_t*)d_route, (uint32_t*)d_act, (uint32_t*)d_order, (uint32_t*)d_off, NULL),
          "orl_route_keyext_device");
    check(ctx, orl_copy_to_host(ctx, route, d_route, m * 4, NULL), "orl_copy_to_host");
    check(ctx, orl_copy_to_host(ctx, act, d_act, m * 4, NULL), "orl_copy_to_host");
    check(ctx, orl_copy_to_host(ctx, order, d_order, m * 4, NULL), "orl_copy_to_host");
    check(ctx, orl_copy_to_host(ctx, off, d_off, (N_GRAINS + 2) * 4, NULL), "orl_copy_to_host");
    check(ctx, orl_stream_sync(ctx, NULL), "orl_stream_sync");
    bad |= compare("route (KeyExt)", route, er, m) | compare("act (KeyExt)", act, ea, m) |
           compare("order (KeyExt)", order, eo, m) | compare("offsets (KeyExt)", off, ef, N_GRAINS + 2);
    void* bufs[] = {d_in, d_ext, d_blob, d_route, d_act, d_order, d_off};
    for (size_t k = 0; k < sizeof bufs / sizeof bufs[0]; ++k) check(ctx, orl_device_free(ctx, bufs[k]), "orl_device_free");
    if (!bad) printf("c host KeyExt ok: %zu golden KeyExt grains registered and %zu messages routed bit-exact\n", nk, m);
    return bad;
}

int main(int argc, char** argv) {
    orl_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.abi_version = ORL_ABI_VERSION;
    cfg.device = 0;
    cfg.dir_capacity = N_GRAINS;
    cfg.n_act = N_GRAINS;
    cfg.placement_policy = ORL_POLICY_PREFER_LOCAL;
    cfg.max_batch = N_MSGS;
    orl_ctx* ctx = NULL;
    check(NULL, orl_ctx_create(&cfg, &ctx), "orl_ctx_create");

    /* 1. silos and ring */
    ref_cluster cl;
    memset(&cl, 0, sizeof cl);
    cl.n_silos = N_SILOS;
    cl.seed = 0xFF;
    for (int s = 0; s < 256; ++s) cl.running[s] = cl.functional[s] = cl.local[s] = s < N_SILOS;
    check(ctx, orl_silos_set(ctx, N_SILOS, NULL, NULL, NULL, ORL_NULL_SILO), "orl_silos_set");
    for (uint32_t s = 0; s < N_SILOS; ++s) {
        char ep[32];
        snprintf(ep, sizeof ep, "10.0.0.%u:11111", s + 1);
        int32_t h;
        check(ctx, orl_silo_consistent_hash(ep, 1, &h), "orl_silo_consistent_hash");
        check(ctx, orl_ring_add_server(ctx, s, h), "orl_ring_add_server");
        ref_ring_add(&cl, s, h);
    }

    /* 2. registrations: GrainId(typeCode, long key), TypeCodeData = (Grain << 56) + sign-extended type code */
    const char* cls = "Orleans.Samples.Chirper.Grains.ChirperAccount";
    int32_t tc;
    check(ctx, orl_calc_id_hash(cls, strlen(cls), &tc), "orl_calc_id_hash");
    const uint64_t tcd = ((uint64_t)ORL_CAT_GRAIN << 56) + ((uint64_t)(int64_t)tc & 0x00FFFFFFFFFFFFFFull);
    orl_grain_key* keys = calloc(N_GRAINS, sizeof *keys);
    uint32_t* acts = calloc(N_GRAINS, 4);
    uint8_t* silos = calloc(N_GRAINS, 1);
    for (uint32_t i = 0; i < N_GRAINS; ++i) {
        keys[i].type_code_data = tcd;
        keys[i].n1 = i;
        acts[i] = i;
        silos[i] = (uint8_t)(i % N_SILOS);
    }
    uint8_t* st = calloc(N_GRAINS, 1);
    check(ctx, orl_dir_insert_single(ctx, keys, acts, silos, N_GRAINS, NULL, NULL, st), "orl_dir_insert_single");
    void* dir = ref_dir_new();
    ref_register(&cl, dir, keys, acts, silos, N_GRAINS, st, NULL, NULL);

    /* 3. the batch */
    orl_msg_hdr* msgs = calloc(N_MSGS, sizeof *msgs);
    uint64_t seed = 0x5EED;
    for (size_t i = 0; i < N_MSGS; ++i) {
        const uint64_t r = splitmix(&seed);
        msgs[i].target.type_code_data = tcd;
        msgs[i].target.n1 = r % (N_GRAINS + N_GRAINS / 10);  /* ~9 % never registered: placement */
        msgs[i].sending_silo = (uint8_t)((r >> 32) % N_SILOS);
        msgs[i].category = 2;
        if ((r >> 40) % 50 == 0) {  /* 2 %: complete addresses, passed through */
            msgs[i].flags = ORL_HDR_ADDRESS_COMPLETE;
            msgs[i].target_silo = (uint8_t)((r >> 48) % N_SILOS);
        }
    }
    const size_t nb = (size_t)N_GRAINS + 2;
    uint32_t *route = calloc(N_MSGS, 4), *act = calloc(N_MSGS, 4), *order = calloc(N_MSGS, 4), *off = calloc(nb, 4);
    /* a: host arrays, page-locked once (a pinned GCHandle buffer on the .NET side) */
    check(ctx, orl_host_register(ctx, msgs, N_MSGS * sizeof *msgs), "orl_host_register");
    check(ctx, orl_route_batch(ctx, msgs, N_MSGS, 0, route, act, order, off), "orl_route_batch");
    check(ctx, orl_host_unregister(ctx, msgs), "orl_host_unregister");

    /* 4. the oracle */
    uint32_t *er = calloc(N_MSGS, 4), *ea = calloc(N_MSGS, 4), *eo = calloc(N_MSGS, 4), *ef = calloc(nb, 4);
    ref_route(&cl, dir, msgs, N_MSGS, 0, er, ea);
    ref_bucket(ea, N_MSGS, N_GRAINS, eo, ef);
    int bad = compare("route (host arrays)", route, er, N_MSGS) | compare("act (host arrays)", act, ea, N_MSGS) |
              compare("order (host arrays)", order, eo, N_MSGS) | compare("offsets (host arrays)", off, ef, nb);

    /* b: device buffers allocated through the library */
    void *d_in, *d_route, *d_act, *d_order, *d_off;
    check(ctx, orl_device_alloc(ctx, N_MSGS * sizeof *msgs, &d_in), "orl_device_alloc");
    check(ctx, orl_device_alloc(ctx, N_MSGS * 4, &d_route), "orl_device_alloc");
    check(ctx, orl_device_alloc(ctx, N_MSGS * 4, &d_act), "orl_device_alloc");
    check(ctx, orl_device_alloc(ctx, N_MSGS * 4, &d_order), "orl_device_alloc");
    check(ctx, orl_device_alloc(ctx, nb * 4, &d_off), "orl_device_alloc");
    check(ctx, orl_copy_to_device(ctx, d_in, msgs, N_MSGS * sizeof *msgs, NULL), "orl_copy_to_device");
    check(ctx, orl_route_batch_device(ctx, d_in, N_MSGS, 0, d_route, d_act, d_order, d_off, NULL), "orl_route_batch_device");
    memset(route, 0, N_MSGS * 4);
    memset(order, 0, N_MSGS * 4);
    memset(off, 0, nb * 4);
    check(ctx, orl_copy_to_host(ctx, route, d_route, N_MSGS * 4, NULL), "orl_copy_to_host");
    check(ctx, orl_copy_to_host(ctx, order, d_order, N_MSGS * 4, NULL), "orl_copy_to_host");
    check(ctx, orl_copy_to_host(ctx, off, d_off, nb * 4, NULL), "orl_copy_to_host");
    check(ctx, orl_stream_sync(ctx, NULL), "orl_stream_sync");
    bad |= compare("route (device)", route, er, N_MSGS) | compare("order (device)", order, eo, N_MSGS) |
           compare("offsets (device)", off, ef, nb);
    void* bufs[] = {d_in, d_route, d_act, d_order, d_off};
    for (size_t k = 0; k < sizeof bufs / sizeof bufs[0]; ++k) check(ctx, orl_device_free(ctx, bufs[k]), "orl_device_free");

    /* c: the narrow call — {N1 low 32 bits, sending silo | category << 8 | flags << 10 | wire type << 16 | target silo
     * << 24} per message, the grain class as wire type 0 (include/orleans_route.h orl_wire8) */
    check(ctx, orl_wire_types_set(ctx, 1, &tcd), "orl_wire_types_set");
    orl_wire8* recs = calloc(N_MSGS, sizeof *recs);
    for (size_t i = 0; i < N_MSGS; ++i) {
        recs[i].n1 = (uint32_t)msgs[i].target.n1;
        recs[i].meta = (uint32_t)msgs[i].sending_silo | ((uint32_t)msgs[i].category << 8) | ((uint32_t)msgs[i].flags << 10) |
                       ((uint32_t)msgs[i].target_silo << 24);
    }
    memset(route, 0, N_MSGS * 4);
    memset(act, 0, N_MSGS * 4);
    memset(order, 0, N_MSGS * 4);
    memset(off, 0, nb * 4);
    void* pinned[] = {recs, route, act, order};
    for (size_t k = 0; k < 4; ++k)
        check(ctx, orl_host_register(ctx, pinned[k], N_MSGS * (k == 0 ? sizeof *recs : 4)), "orl_host_register");
    check(ctx, orl_route_batch_narrow(ctx, recs, N_MSGS, 0, route, act, order, off), "orl_route_batch_narrow");
    for (size_t k = 0; k < 4; ++k) check(ctx, orl_host_unregister(ctx, pinned[k]), "orl_host_unregister");
    bad |= compare("route (narrow)", route, er, N_MSGS) | compare("act (narrow)", act, ea, N_MSGS) |
           compare("order (narrow)", order, eo, N_MSGS) | compare("offsets (narrow)", off, ef, nb);
    free(recs);

    ref_dir_free(dir);
    if (argc > 1) bad |= keyext_step(ctx, &cl, argv[1]);
    check(ctx, orl_ctx_destroy(ctx), "orl_ctx_destroy");
    if (bad) return 1;
    printf("c host ok: %d messages through orl_route_batch (pinned host arrays), orl_route_batch_device "
           "(library-allocated buffers) and orl_route_batch_narrow (8-B records), bit-exact vs the oracle\n", N_MSGS);
    return 0;
}
