"""Per-rank GPU cost of the node step (config 3 split over R ranks), each kernel measured alone on one GPU.

The one-GPU rehearsal (bench.py --local-ranks) runs every rank's kernels concurrently on one device, so its per-kernel
times are not what one rank sees on its own GPU.  This lab replays one rank's share in isolation:
  1. hop 1: the rank's own 256M/R messages, owner-partitioned in `chunks` calls (k_part_lb, 8-B or 16-B records: argv[3]);
  2. routing at the owner + stage 4 at the host over everything the rank receives (every source rank's region for it,
     built here by partitioning each source's messages);
and prints milliseconds per step for the hottest rank and the rank with the median load.  Lab script, not a test.

LAB_CACHE=<entries> (round 5): every sender's directory cache holds the `entries` most frequent grains
of the Zipf stream whose directory entry another rank holds (a warm cache: the earlier lookups' results,
LocalGrainDirectory.cs:761-762; the reference's default capacity is 1M, GlobalConfiguration.cs:413,417); hop 1 then
addresses those messages at the sender (orl_partition_cached_device) and the owner routes its received records with the
act lane (orl_route_received_device: no probe for addressed ones) before stage 4 (orl_bucket_device).
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from orleans_amd import _lib as L  # noqa: E402
from orleans_amd import workloads as W  # noqa: E402
from orleans_amd.engine import GrainDirectoryEngine  # noqa: E402
from orleans_amd.node import local_silos, rank_of_silo  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main(R=8, chunks=4, width=8):
    import os
    if os.environ.get("LAB_LIB"):  # A/B: an experimental build of the library
        L.LIB_PATH = os.path.abspath(os.environ["LAB_LIB"])
    n_grains, n_total = 16_000_000, 256 << 20
    n_msgs = n_total // R
    cl = W.balanced_cluster()
    ros = rank_of_silo(cl.n_silos, R)
    keys, uni, owner, reg = W.grain_population(cl, n_grains)
    ztab = W.zipf_tables(torch, n_grains, W.SEED_C3)
    import os
    n_cache = int(os.environ.get("LAB_CACHE", "0"))
    part = GrainDirectoryEngine(n_act=1 << 24, dir_capacity=1, max_batch=n_msgs, device=0)
    W.setup_engine(part, cl)
    if n_cache:  # each grain's handle at its owner rank (W.register_population(dense_local=True) per rank)
        hnd = np.zeros(n_grains, np.uint32)
        orank = ros[owner]
        for r in range(R):
            idx = np.nonzero(reg & (orank == r))[0]
            hnd[idx] = np.arange(len(idx), dtype=np.uint32)
        zperm = ztab[1].cpu().numpy()  # Zipf rank k -> grain perm[k - 1]
        part.cache_config(n_cache)
    # every call on one torch stream (not the legacy default stream, whose handle 0 means "the context's own stream" to
    # the library), so torch's events time them and torch's copies see their results
    torch.cuda.set_stream(torch.cuda.Stream())
    st = torch.cuda.current_stream().cuda_stream
    if width == 8:
        part.set_wire_types([W.grain_tcd(cl)])
    partition = part.partition_narrow_device if width == 8 else part.partition_compact_device
    cap = n_msgs + n_msgs // 2
    d_out = torch.empty(R * cap * width, dtype=torch.uint8, device="cuda")
    d_counts = torch.zeros(R, dtype=torch.int64, device="cuda")
    d_status = torch.zeros(1, dtype=torch.int32, device="cuda")
    d_lane = torch.empty(R * cap if n_cache else 1, dtype=torch.int32, device="cuda")
    recv = [[] for _ in range(R)]
    lanes = [[] for _ in range(R)]
    part_ms = []
    two = not os.environ.get("LAB_ONE_STREAM") and chunks > 1
    st2 = torch.cuda.Stream()
    for s in range(R):
        m = W.device_messages(torch, cl, n_grains, n_msgs, W.SEED_C3, start=s * n_msgs,
                              sender_silos=local_silos(cl.n_silos, R, s), zipf=ztab)
        step = n_msgs // chunks
        if n_cache:  # rank s's warm cache: the n_cache hottest grains owned by other ranks
            mine_s = local_silos(cl.n_silos, R, s)
            W.setup_engine(part, cl, local_silos=mine_s)
            part.cache_clear()
            g = zperm[:4 * n_cache]
            g = g[reg[g] & (orank[g] != s)][:n_cache]
            kd = torch.from_numpy(np.ascontiguousarray(keys[g]).view(np.uint8)).cuda()
            part.cache_add_or_update_device(kd, torch.from_numpy(hnd[g].view(np.int32)).cuda(),
                                            torch.from_numpy(owner[g].astype(np.uint8)).cuda(), len(g), stream=st)

            def part_one(mm, k, stream=st):
                part.partition_cached_device(mm, k, ros, R, s, cap, d_out, width, d_lane, d_counts, d_status, stream=stream)
        else:
            def part_one(mm, k, stream=st):
                partition(mm, k, ros, R, s, cap, d_out, d_counts, d_status, stream=stream)

        def hop1():
            # as the node issues them: odd chunks on a second stream (round 6; LAB_ONE_STREAM=1: all on one stream)
            if two:
                st2.wait_stream(torch.cuda.current_stream())
            for c in range(chunks):
                part_one(m[c * step:], step, stream=st2.cuda_stream if (two and c & 1) else st)
            if two:
                torch.cuda.current_stream().wait_stream(st2)
        part_ms.append(timed(hop1))
        part_one(m, n_msgs)
        cnt = d_counts.cpu().numpy()
        assert int(d_status.item()) & ~L.PART_CACHED == 0, int(d_status.item())
        for r in range(R):
            recv[r].append(d_out[r * cap * width:(r * cap + int(cnt[r])) * width].clone())
            if n_cache:
                lanes[r].append(d_lane[r * cap:r * cap + int(cnt[r])].clone())
        del m
    owned = np.array([sum(x.numel() // width for x in recv[r]) for r in range(R)])
    print(f"hop 1 partition of {n_msgs >> 20}M messages in {chunks} calls: {np.median(part_ms):.3f} ms "
          f"(min {min(part_ms):.3f}, max {max(part_ms):.3f})", flush=True)
    print(f"owned per rank (M): {[round(x / 2**20, 1) for x in owned]}, max/mean {owned.max() / owned.mean():.2f}",
          flush=True)
    order = np.argsort(owned)
    which = (("hottest", int(order[-1])), ("median", int(order[R // 2])))
    if os.environ.get("LAB_ONLY"):  # e.g. LAB_ONLY=hottest under rocprofv3: one rank's kernels only
        which = tuple(w for w in which if w[0] == os.environ["LAB_ONLY"])
    for label, r in which:
        recs = torch.cat(recv[r])
        n = recs.numel() // width
        mine = local_silos(cl.n_silos, R, r)
        mask = np.zeros(cl.n_silos, np.uint8)
        mask[mine] = 1
        n_act = max(1, int((reg & mask[owner].astype(bool)).sum()))
        eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=n_act, max_batch=n, device=0)
        W.setup_engine(eng, cl, local_silos=mine)
        if width == 8:
            eng.set_wire_types([W.grain_tcd(cl)])
        W.register_population(eng, keys, owner, reg, mask, dense_local=True)
        route = torch.empty(n, dtype=torch.int32, device="cuda")
        act = torch.empty(n, dtype=torch.int32, device="cuda")
        order_o = torch.empty(n, dtype=torch.int32, device="cuda")
        offs = torch.empty(n_act + 2, dtype=torch.int32, device="cuda")
        addr = eng.address_narrow_device if width == 8 else eng.address_compact_device
        if n_cache:
            lane = torch.cat(lanes[r])
            n_addr = int((lane != -1).sum().item())

            def route_only():
                eng.route_received_device(recs, width, n, lane, route, act, stream=st)

            def route_all():
                route_only()
                eng.bucket_device(act, n, order_o, offs, stream=st)
            t_route = timed(route_only)
            t_all = timed(route_all)
            print(f"{label} rank {r}: {n_addr / max(n, 1):.3f} of the received records addressed by the senders' caches",
                  flush=True)
        else:
            t_route = timed(lambda: addr(recs, n, route, act, stream=st, opts=L.OPT_NO_BUCKETS))
            t_all = timed(lambda: addr(recs, n, route, act, order_o, offs, stream=st))
        xgmi_mb = n * (R - 1) / R * width / 1e6
        print(f"{label} rank {r}: {n / 2**20:.1f}M messages received; route {t_route:.3f} ms, route + stage 4 "
              f"{t_all:.3f} ms; n_act {n_act}; receives ~{xgmi_mb:.0f} MB over xGMI; hot key {eng.query(L.Q_HOT_KEY)}, "
              f"{eng.query(L.Q_HOT_BATCHES)} batches on the hot-key path", flush=True)
        eng.close()
        del recs
    part.close()


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
