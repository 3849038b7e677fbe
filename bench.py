#!/usr/bin/env python3
"""bench.py — routed grain messages/sec on MI355X (BASELINE.json metric), one process per GPU.

Default workload at every N (one workload along the driver's 1/2/4/8-GPU curve; BASELINE.json
configs[2], SURVEY §8(d) config 3, the batch size north_star's targets are quoted on): 8 logical silos 10.0.0.{1..8}:11111
(balanced generations), 16M ChirperAccount long-key grains all registered (activation on the directory owner), 256M
single-target messages per step in total, targets Zipf(1.1) (seed 0x5EED0003) through a seeded permutation, generated on
the device and resident in HBM before the timed region.  A step = one pass of the hot path over the batch: stages 1-4
(hash, ring owner, directory probe + placement, stable per-activation bucketing).  At N=1 the whole batch runs on one
GPU; at N>1 (torchrun) the batch is split 256M/N per GPU (strong scaling): each GPU hosts silos s*N//8 == rank and their
directory partition, originates its share from its own silos, and a step runs the node exchange behind the C ABI
(orl_node: owner partition, RCCL counts all-gather + grouped send/recv, routing at the owner, hop 2, stage 4 at the host;
SURVEY §8(e)).

Other SURVEY §8(d) workloads (measurement legs recorded under profiles/; not the driver's bench line):
  --config 1   Chirper generator graph, 1k accounts x 10 followers on one silo, every account publishes (10k messages)
  --config 2   uniform 1M grains, 64M messages per GPU (weak scaling; BASELINE configs[1], the round-1..4 headline)
  --config 4   Chirper-scale CSR: 10M accounts, power-law followers (exp 2.1, 1..1e5), 1M publishers per step
  --config 5   Presence: 100k Guid-keyed games x 8 players, 64k heartbeats per step, eager and hipGraph-replayed
  --config 6/7/8   directory mutation (f1), stream / reminder rings (f3), receive path (f2) legs

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1..8]
       python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from orleans_amd import _lib as L  # noqa: E402

if os.environ.get("LAB_LIB"):  # A/B only: an experimental build of the same library (make lab NAME=... DEFS=...)
    L.LIB_PATH = os.path.abspath(os.environ["LAB_LIB"])
L_NODE_ID_BYTES = 128

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
ROUTE_KERNEL_BYTES_PER_MSG = 72  # 32 B header + 32 B directory slot + 4 B route word + 4 B activation handle
PIPELINE_BYTES_PER_MSG = 76      # + 4 B stable position
FANOUT_BYTES_PER_MSG = 48        # 4 B CSR target + 32 B slot + 12 B outputs per emitted message
FANOUT_BYTES_PER_PUB = 40        # + 32 B header + 8 B CSR offset per publish
# config 5 (one mixed batch, Guid keys: the 32-B directory table): a direct game message reads its 32-B header and a 32-B
# slot and writes 8 B; a player message reads its 4-B CSR target, its 24-B key-table entry and a 32-B slot and writes 8 B;
# a publish reads its publisher id, silo and CSR start (4 + 1 + 8 B) and its u32 offset
PRESENCE_BYTES_DIRECT = 72
PRESENCE_BYTES_FANOUT = 68
PRESENCE_BYTES_PER_PUB = 17


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def owner_rank_counts(torch, cl, d_msgs, n, ros, world, device=0, piece=1 << 22):
    """Messages of a batch per directory-owner rank, counted by the library's own owner partition
    (orl_partition_by_owner_device: stages 1-2 + the per-rank counts of its send queues) over 4M-message pieces, with a
    throwaway context: the receive capacity (max_recv) of a node run is sized by the same code that routes."""
    from orleans_amd import workloads as W
    from orleans_amd.engine import GrainDirectoryEngine
    e = GrainDirectoryEngine(n_act=1, dir_capacity=16, max_batch=piece, device=device)
    W.setup_engine(e, cl)
    out = torch.empty((piece, 8), dtype=torch.int32, device="cuda")
    idx = torch.empty(piece, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(world, dtype=torch.int64, device="cuda")
    total = torch.zeros(world, dtype=torch.int64, device="cuda")
    # one explicit stream for the partitions AND the torch adds: torch's default stream has handle 0, which the C ABI reads
    # as "the context's own stream", and `total += cnt` would then race the partition that writes cnt
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for lo in range(0, n, piece):
            k = min(piece, n - lo)
            e.partition_by_owner_device(d_msgs[lo:lo + k], k, ros, world, 0, out, idx, cnt, stream=s.cuda_stream)
            total += cnt
    torch.cuda.synchronize()
    e.close()
    return total


class WarmCaches:
    """The bench's warm sender directory caches (--sender-cache N): rank s caches the N hottest grains of the Zipf stream
    (rank order = the workload's permutation) that are registered and owned by another rank, with the handle their owner's
    catalog registered (dense per owner rank) and the owner silo (activations live on their owners).  thresh[s] = the
    Zipf position of rank s's last cached grain, so the self-check can tell which hosted messages a sender addressed."""

    def __init__(self, zperm, reg, owner, ros, world, n):
        self.n = int(n)
        orank = ros[owner]
        self.pos = np.empty(len(zperm), np.int64)
        self.pos[zperm] = np.arange(len(zperm))
        self.orank = orank
        self.handle = np.zeros(len(owner), np.uint32)
        for r in range(world):
            idx = np.nonzero(reg & (orank == r))[0]
            self.handle[idx] = np.arange(len(idx), dtype=np.uint32)
        self.grains, self.thresh = [], []
        for s in range(world):
            z = zperm[:min(len(zperm), 2 * self.n)]
            z = z[reg[z] & (orank[z] != s)]
            while len(z) < self.n and len(z) < int((reg & (orank != s)).sum()):  # (tiny populations only)
                z = zperm[reg[zperm] & (orank[zperm] != s)]
            g = z[:self.n]
            self.grains.append(g)
            self.thresh.append(int(self.pos[g[-1]]) if len(g) else -1)

    def fill(self, torch, eng, keys, owner, s, stream):
        g = self.grains[s]
        eng.cache_config(max(self.n, 16))
        if len(g):
            eng.cache_add_or_update_device(torch.from_numpy(np.ascontiguousarray(keys[g]).view(np.uint8)).cuda(),
                                           torch.from_numpy(self.handle[g].view(np.int32)).cuda(),
                                           torch.from_numpy(owner[g].astype(np.uint8)).cuda(), len(g), stream=stream)
        torch.cuda.synchronize()

    def addressed(self, grains, senders, me):
        """Whether the sender rank of each hosted message addressed it from its cache (its owner is `me`)."""
        t = np.asarray(self.thresh, np.int64)[senders]
        return (senders != me) & (self.pos[grains] <= t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=None, choices=[1, 2, 3, 4, 5, 6, 7, 8],
                    help="6 = directory mutation leg (SURVEY §8(f) f1): device registration / unregistration batches; "
                         "7 = stream / reminder ring leg (f3); 8 = receive path leg (f2): frames -> headers -> route")
    ap.add_argument("--c5-contexts", type=int, default=1, choices=[1, 2],
                    help="config 5 split mode: routing contexts/streams per step (2: game messages and fan-out concurrently)")
    ap.add_argument("--c5-mode", default="mixed", choices=["mixed", "split"],
                    help="config 5: one orl_fanout_route_mixed_device call per step (game messages + player fan-out as "
                         "one batch), or two calls (route the game messages, then the fan-out)")
    ap.add_argument("--frames", type=int, default=4 * 1024 * 1024, help="frames per step (config 8)")
    ap.add_argument("--grains", type=int, default=None)
    ap.add_argument("--msgs", type=int, default=None,
                    help="messages per GPU per step (default: config 2 64M per GPU; config 3 256M in total, split over the GPUs)")
    ap.add_argument("--chunks", type=int, default=4, help="node exchange pipeline depth (N > 1)")
    ap.add_argument("--local-ranks", type=int, default=0,
                    help="rehearse the N-rank node exchange on ONE GPU: N ranks as threads over the in-process transport "
                         "(orl_node LOCAL); measures the protocol, not xGMI scaling")
    ap.add_argument("--host-io", choices=["pinned", "pageable", "narrow"], default=None,
                    help="config 2 at N=1: time the host-array P/Invoke call instead (orl_route_batch: 32-B headers in over "
                         "PCIe, route / act / order out; narrow = orl_route_batch_narrow: 8-B orl_wire8 records in, pinned)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--unregistered", type=float, default=0.0,
                    help="configs 2/3: fraction of the grains never registered (SURVEY §8(d) config 2's 10%% variant: "
                         "their messages miss the directory and are placed PreferLocal)")
    ap.add_argument("--sender-cache", type=int, default=0,
                    help="N > 1 (and --local-ranks), config 3: every rank's directory cache holds this many entries, warm: "
                         "the hottest grains of the Zipf stream whose directory entry another rank holds (the reference's "
                         "default cache capacity is 1M, GlobalConfiguration.cs:413,417); hop 1 then addresses those messages "
                         "at the sender (LocalGrainDirectory.cs:690-717)")
    ap.add_argument("--wire16", action="store_true",
                    help="N > 1: exchange 16-B records (no wire types) instead of the 8-B form")
    ap.add_argument("--cpu-wall", type=float, default=1.5, help="target wall seconds of the CPU baseline sample")
    ap.add_argument("--traffic-json", default=None, help="default: profiles/route_kernel_pmc[_config<N>].json")
    ap.add_argument("--check-sample", type=int, default=256 * 1024,
                    help="N > 1 (and --local-ranks): hosted messages per rank checked against the oracle after the timed "
                         "steps, on top of the size-independent checks of every hosted message (0: no oracle sample)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local_rank)
    if args.config is None:  # the headline: config 3's 256M batch at every N, so the 1/2/4/8-GPU lines share one workload
        args.config = 3
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        if args.config in (1, 5, 6, 7, 8):
            raise SystemExit("--config 1/5/6/7/8 are single-GPU measurement legs")

    if args.local_ranks and args.config == 4:
        res = run_fanout_node(args, torch, None, 0, args.local_ranks, 0, rehearsal=True)
    elif args.local_ranks:
        res = run_rehearsal(args, torch)
    elif args.config == 1:
        res = run_chirper(args, torch)
    elif args.config in (2, 3):
        res = run_single_target(args, torch, dist, rank, world, local_rank)
    elif args.config == 4:
        res = run_fanout(args, torch) if world == 1 else run_fanout_node(args, torch, dist, rank, world, local_rank)
    elif args.config == 6:
        res = run_directory(args, torch)
    elif args.config == 7:
        res = run_rings(args, torch)
    elif args.config == 8:
        res = run_wire(args, torch)
    else:
        res = run_presence(args, torch)
    if world > 1:
        dist.barrier()
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if res.get("check") not in (None, "ok"):  # a failed self-check of the hosted output fails the run (every rank)
        log(f"self-check FAILED: {res['check']}")
        sys.exit(1)


def timed_steps(args, torch, dist, world, step, sync):
    """W untimed warmup steps, then exactly K steps between barrier + synchronize; max over ranks."""
    for _ in range(args.warmup):
        step()
    sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    units = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        units += step()
    sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    return elapsed, units


def traffic_json_path(config):
    """The route kernel's PMC traffic record of a workload (scripts/make_traffic_json.py writes it)."""
    return os.path.join(ROOT, "profiles", "route_kernel_pmc.json" if config == 2 else f"route_kernel_pmc_config{config}.json")


def read_traffic(path, msgs_per_launch, world, config):
    """The route kernel's measured HBM bytes per launch (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, scripts/make_traffic_json.py)
    and where they come from, for the workload they were measured on only (the same config, all grains registered, one GPU,
    the same messages per launch); (None, None) otherwise."""
    if world != 1 or not os.path.exists(path):
        return None, None
    try:
        tj = json.load(open(path))
        if tj.get("msgs_per_launch") == msgs_per_launch and tj.get("config", 2) == config:
            src = f"{os.path.relpath(path, ROOT)}: {tj.get('method', 'rocprofv3 --pmc')}"
            if tj.get("build"):
                src += f"; measured at build {tj['build']}"
            return tj.get("hbm_bytes_per_launch"), src
    except Exception:
        return None, None
    return None, None


# ---- the node's correctness evidence (checker: after the timed steps, outside timing) ------------------------
def node_self_check(torch, eng, res, rank, cl, keys, owner, reg, local_mask, n_act, ros, expect_owned, sample, stream=None,
                    caches=None):
    """One rank's hosted output of the last timed batch: the size-independent properties of every hosted message on the
    device (orleans_amd/selfcheck.py: owner / host / status / handle per message, a permutation grouped by activation, FIFO
    inside every bucket, offsets = the count prefix), the owned count against the workload's own per-destination count,
    and the first `sample` hosted messages routed by the oracle (oracle/cpu_ref.py, the checker) bit for bit.  Returns
    the list of failures (empty: ok)."""
    from orleans_amd import selfcheck as SC
    from orleans_amd.node import narrow_records_to_headers, wire_records_to_headers
    errs = []
    if res.hop2:
        errs.append("hop 2 forwarded messages (every activation of the workload lives on its directory owner)")
    if expect_owned is not None and res.n_owned != expect_owned:
        errs.append(f"owned {res.n_owned} messages, the workload sends this rank {expect_owned}")
    d = SC.fetch_node_result(torch, eng, res, n_act, stream=stream)
    dev = d["route"].device
    owner_t = torch.as_tensor(owner.astype(np.int64), device=dev)
    handle_t = torch.as_tensor(SC.local_handles(owner, reg, local_mask), device=dev)
    ros_t = torch.as_tensor(np.asarray(ros, np.int64), device=dev)
    errs += SC.check_routes(torch, d["route"], d["act"], d["n1"], owner_t, handle_t, bool(reg.all()), ros_t, rank)
    errs += SC.check_stage4(torch, d["act"], d["order"], d["offsets"], n_act)
    k = min(int(sample), res.n_hosted)
    if k:  # the oracle replays this rank's directory partition over the first k hosted records
        from oracle import cpu_ref
        hdr, left = [], k
        for p, cnt, w in res.segments:
            take = min(cnt, left)
            if take:
                raw = eng.copy_to_host(np.zeros(take * w, np.uint8), p, stream=stream)
                hdr.append(raw.view(L.MSG_DTYPE) if w == 32 else wire_records_to_headers(raw) if w == 16 else
                           narrow_records_to_headers(raw, getattr(eng, "wire_types", ())))
                left -= take
            if not left:
                break
        hdr = np.concatenate(hdr)
        o = cpu_ref.Oracle(cl.n_silos, local=list(np.ones(cl.n_silos, np.uint8) if local_mask is None else local_mask))
        for s in range(cl.n_silos):
            o.add_server(s, int(cl.hashes[s]))
        h = SC.local_handles(owner, reg, local_mask)
        sel = np.nonzero(h >= 0)[0]
        o.register(keys[sel], h[sel].astype(np.uint32), owner[sel])
        r_ref, a_ref = o.route(hdr)
        if caches is not None:  # messages the sender addressed from its warm cache: HIT | CACHED (same host and handle)
            sent = np.asarray(ros, np.int64)[hdr["sending_silo"].astype(np.int64)]
            cached = caches.addressed(hdr["n1"].astype(np.int64), sent, rank)
            r_ref = np.where(cached, r_ref | np.uint32(L.RF_CACHED << 24), r_ref).astype(np.uint32)
        r_got = d["route"][:k].cpu().numpy().astype(np.uint32)
        a_got = d["act"][:k].cpu().numpy().astype(np.uint32)
        if not np.array_equal(r_got, r_ref):
            errs.append(f"route words differ from the oracle for {int((r_got != r_ref).sum())} of {k} sampled messages")
        if not np.array_equal(a_got, a_ref):
            errs.append(f"handles differ from the oracle for {int((a_got != a_ref).sum())} of {k} sampled messages")
    return errs


# ---- configs 2 and 3: single-target messages ---------------------------------------------------------------
def run_single_target(args, torch, dist, rank, world, local_rank):
    from orleans_amd import workloads as W
    from orleans_amd.engine import GrainDirectoryEngine
    from orleans_amd.node import GrainNode, local_silos, rank_of_silo

    zipf = args.config == 3
    n_grains = args.grains or (16_000_000 if zipf else 1_000_000)
    # config 2: 64M messages per GPU (weak scaling); config 3: 256M messages in total, 256M / N per GPU (strong)
    strong = zipf and not args.msgs
    n_total = args.msgs * world if args.msgs else (256 << 20 if zipf else (64 << 20) * world)
    n_msgs = n_total // world
    # balanced ring (silo generations, W.balanced_cluster): the reference's one-point-per-silo ring with
    # generation-1 silos gives one of 8 GPUs 2.85x the average share
    cl = W.balanced_cluster()
    ros = rank_of_silo(cl.n_silos, world)
    mine = local_silos(cl.n_silos, world, rank)
    t_setup = time.perf_counter()
    keys, uni, owner, reg = W.grain_population(cl, n_grains, 1.0 - args.unregistered)
    seed = W.SEED_C3 if zipf else W.SEED_C2
    ztab = W.zipf_tables(torch, n_grains, seed) if zipf else None
    # this rank's share of the workload's message stream, generated on the device (== the numpy generators)
    d_msgs = W.device_messages(torch, cl, n_grains, n_msgs, seed, start=rank * n_msgs,
                               sender_silos=mine if world > 1 else None, zipf=ztab)
    torch.cuda.synchronize()
    node = None
    cap = n_msgs
    local_mask = None
    n_act = n_grains
    if world > 1:
        # receive capacity: every rank's per-destination counts (the library's owner partition), summed over ranks
        # (Zipf: the hot owners get more)
        per_dest = owner_rank_counts(torch, cl, d_msgs, n_msgs, ros, world, device=local_rank)
        dist.all_reduce(per_dest)
        cap = max(n_msgs, int(per_dest.max().item()))
        cap += cap // 64 + 4096
        expect_owned = int(per_dest[rank].item())  # the self-check's owned count (every rank's messages to my silos)
    if world > 1:  # this rank's silos hold only their own partition; their catalog numbers its activations densely
        local_mask = np.zeros(cl.n_silos, np.uint8)
        local_mask[mine] = 1
        n_act = max(1, int((reg & local_mask[owner].astype(bool)).sum()))
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=n_act, max_batch=max(cap, n_msgs), device=local_rank)
    W.setup_engine(eng, cl, local_silos=mine if world > 1 else None)
    if world > 1 and not args.wire16:  # the node's grain classes: 8-B exchange records
        eng.set_wire_types([W.grain_tcd(cl)])
    n_reg = W.register_population(eng, keys, owner, reg, local_mask, dense_local=world > 1)
    del uni
    caches = None
    if world > 1 and args.sender_cache and zipf:  # warm sender directory caches (the reference's default path, f4)
        caches = WarmCaches(ztab[1].cpu().numpy(), reg, owner, ros, world, args.sender_cache)
        caches.fill(torch, eng, keys, owner, rank, torch.cuda.current_stream().cuda_stream)
    if world == 1:
        del keys
    log(f"rank {rank}/{world}: silos {[int(s) for s in mine]}, {n_reg} grains registered, {n_msgs} messages, "
        f"receive capacity {cap}" + (f", sender cache {args.sender_cache} entries" if caches else ""))
    stream = torch.cuda.current_stream().cuda_stream
    stats = {}
    if args.host_io:
        return run_host_io(args, torch, eng, cl, d_msgs, n_msgs, n_act, n_grains)
    if world == 1:
        route = torch.empty(n_msgs, dtype=torch.int32, device="cuda")
        act = torch.empty(n_msgs, dtype=torch.int32, device="cuda")
        order = torch.empty(n_msgs, dtype=torch.int32, device="cuda")
        offsets = torch.empty(n_act + 2, dtype=torch.int32, device="cuda")

        def step():
            eng.address_messages_device(d_msgs, n_msgs, route, act, order, offsets, stream=stream)
            return n_msgs
    else:
        # the node exchange behind the C ABI: owner partition, counts all-gather, grouped send/recv over RCCL, routing
        # at the owner, hop 2 when activations live elsewhere, stage 4 at the host (orl_node_route_batch_device)
        gid = torch.zeros(L_NODE_ID_BYTES, dtype=torch.uint8, device="cuda")
        if rank == 0:
            gid.copy_(torch.frombuffer(bytearray(GrainNode.unique_id()), dtype=torch.uint8))
        dist.broadcast(gid, 0)
        node = GrainNode(eng, world, rank, ros, max_batch=n_msgs, max_recv=cap, group_id=bytes(gid.cpu().numpy()),
                         chunks=args.chunks)

        def step():
            res = node.route_batch_device(d_msgs, n_msgs, stream=stream)
            stats["owned"] = stats.get("owned", 0) + res.n_owned
            stats["remote"] = stats.get("remote", 0) + res.n_sent_remote
            stats["fwd"] = stats.get("fwd", 0) + res.n_forwarded
            stats.setdefault("widths", set()).update(w for _, c, w in res.segments if c)
            xs = node.stats()
            stats["wait_us"] = stats.get("wait_us", 0) + xs["host_wait_us"]
            stats["waits"] = stats.get("waits", 0) + xs["host_waits"]
            stats["bytes_sent"] = [a + b for a, b in zip(stats.get("bytes_sent", [0] * world), xs["bytes_sent"])]
            stats["comm_count"] = xs["comm_count"]
            stats["exchange_mode"] = xs["exchange_mode"]
            stats["last"] = res
            return res.n_owned
    log(f"setup {time.perf_counter() - t_setup:.1f}s; warmup {args.warmup}")
    eng.set_timing(False)

    def sync():
        eng.sync()

    # timing events are enabled after warmup so the summary covers the timed steps only
    for _ in range(max(args.warmup, 1 if world > 1 else 0)):  # the node's first step allocates its buffers
        step()
    sync()
    torch.cuda.synchronize()
    eng.set_timing(True)
    stats.clear()
    args_w = argparse.Namespace(**{**vars(args), "warmup": 0})
    elapsed, recv_total = timed_steps(args_w, torch, dist, world, step, sync)
    nb, route_ms, bucket_ms, total_ms = eng.timing_summary()
    ms_per_step = elapsed * 1e3 / args.steps
    value = world * n_msgs * args.steps / elapsed
    # route kernel launches per step: 1 (one GPU), or one per received chunk (node)
    launches = max(1, nb // args.steps)
    per_launch_msgs = recv_total / args.steps / launches
    wire = node is not None
    rec_w = max(stats.get("widths") or {16 if wire else 32})  # the exchange record the owner's route kernel reads
    kbytes = ROUTE_KERNEL_BYTES_PER_MSG - (32 - rec_w)  # 8-B / 16-B exchange records instead of 32-B headers
    achieved = kbytes * per_launch_msgs / (route_ms * 1e-3) / 1e9
    log(f"rank {rank}: {ms_per_step:.3f} ms/step; route kernel {route_ms:.3f} ms x {launches}, bucketing {bucket_ms:.3f} ms, "
        f"call {total_ms:.3f} ms over {nb} launches")
    traffic, traffic_src = (read_traffic(args.traffic_json or traffic_json_path(args.config), per_launch_msgs, world,
                                         args.config) if not args.unregistered else (None, None))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(cl, n_grains, d_msgs, args.cpu_wall, zipf, 1.0 - args.unregistered)
    check = None
    if node is not None:  # correctness evidence of the multi-GPU run: every rank checks what it hosted (outside timing)
        t_chk = time.perf_counter()
        errs = node_self_check(torch, eng, stats["last"], rank, cl, keys, owner, reg, local_mask, n_act, ros, expect_owned,
                               args.check_sample, stream=stream, caches=caches)
        tot = torch.tensor([stats["last"].n_hosted], dtype=torch.int64, device="cuda")
        dist.all_reduce(tot)
        if int(tot.item()) != n_total:
            errs.append(f"the ranks host {int(tot.item())} messages of {n_total}")
        gathered = [None] * world
        dist.all_gather_object(gathered, errs)
        bad = [f"rank {r}: {e}" for r, es in enumerate(gathered) for e in es]
        check = "ok" if not bad else "; ".join(bad)
        log(f"rank {rank}: self-check {'ok' if not errs else errs} ({time.perf_counter() - t_chk:.1f}s)")
    if node is not None:
        node.close()
    eng.close()
    name = (f"config3: Zipf(1.1) over {n_grains / 1e6:g}M long-key grains, {n_total >> 20}M messages in total "
            f"({n_msgs >> 20}M per GPU)" if zipf else
            f"config2: uniform {n_grains // 1_000_000}M long-key grains, {n_msgs >> 20}M single-target messages per GPU")
    if args.unregistered:
        name += f", {args.unregistered:.0%} of the grains unregistered (misses placed PreferLocal)"
    name += ", 8-silo ring, stages 1-4"
    if world > 1:
        name += (", + owner partition, RCCL counts all-gather + grouped send/recv, routing at the owner, hop 2, "
                 f"stage 4 at the host (orl_node, {args.chunks} chunks)")
        if caches:
            name += (f", warm sender directory caches of {args.sender_cache} entries per rank (the hottest remote grains; "
                     "cached messages addressed at the sender)")
    out = {
        "metric": "routed grain messages/sec (node)",
        "value": value,
        "unit": "messages/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u32/u64 integer",
        "data": f"synthetic (seeded splitmix64 on the device; config {args.config} of SURVEY §8(d))",
        "config": {"workload": name, "grains": n_grains, "unregistered_frac": args.unregistered,
                   "messages_total": n_total, "messages_per_gpu": n_msgs,
                   "silos": cl.n_silos, "ring": "balanced (silo generations %s)" % W.balanced_generations(cl.n_silos),
                   "parallelism": f"directory sharded by ring range over {world} GPU(s)"},
        "roofline": {"bound": "hbm", "kernel": "k_route (stages 1-3)", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src, "bytes_per_msg": kbytes, "msgs_per_launch": per_launch_msgs, "avg_launch_ms": route_ms},
        "pipeline": {"bytes_per_msg": PIPELINE_BYTES_PER_MSG, "route_kernel_ms": route_ms,
                     "bucketing_ms": bucket_ms, "call_ms": total_ms,
                     "algorithmic_GBs": PIPELINE_BYTES_PER_MSG * value / world / 1e9,
                     "frac_of_hbm_peak": PIPELINE_BYTES_PER_MSG * value / world / 1e9 / HBM_PEAK_GBS},
        "cpu_baseline": cpu,
    }
    if stats:
        out["exchange"] = {"rank0_owned_per_step": stats["owned"] / args.steps,
                           "rank0_sent_remote_per_step": stats["remote"] / args.steps,
                           "rank0_forwarded_hop2_per_step": stats["fwd"] / args.steps,
                           "record_bytes": rec_w,
                           "rank0_xgmi_bytes_per_step": rec_w * stats["remote"] / args.steps,
                           "receive_capacity": cap,
                           "ncclCommCount": stats["comm_count"],
                           "mode": stats["exchange_mode"],
                           "rank0_bytes_sent_per_peer_per_step": [b / args.steps for b in stats["bytes_sent"]],
                           "rank0_host_wait_ms_per_step": stats["wait_us"] / 1e3 / args.steps,
                           "rank0_host_wait_ms_per_chunk": stats["wait_us"] / 1e3 / args.steps / max(1, args.chunks),
                           "rank0_host_waits_per_step": stats["waits"] / args.steps}
        out["check"] = check
        out["check_sample_per_rank"] = args.check_sample
    return out


def run_rehearsal(args, torch):
    """--local-ranks R: the multi-GPU step of configs 2 / 3 (owner partition, counts all-gather, grouped send/recv, routing
    at the owner, hop 2, stage 4 at the host) with R ranks as threads of this process on one GPU, exchanging through the
    in-process transport (device copies).  Same workload split as `torchrun --nproc-per-node R`; every rank's work shares
    the one GPU, so the time is the sum of the ranks' work, not a scaling measurement."""
    from concurrent.futures import ThreadPoolExecutor
    from orleans_amd import _lib as L
    from orleans_amd import workloads as W
    from orleans_amd.engine import GrainDirectoryEngine
    from orleans_amd.node import GrainNode, local_silos, rank_of_silo

    R = args.local_ranks
    zipf = args.config == 3
    n_grains = args.grains or (16_000_000 if zipf else 1_000_000)
    n_total = args.msgs * R if args.msgs else (256 << 20 if zipf else (64 << 20) * R)
    n_msgs = n_total // R
    cl = W.balanced_cluster()
    ros = rank_of_silo(cl.n_silos, R)
    keys, uni, owner, reg = W.grain_population(cl, n_grains, 1.0 - args.unregistered)
    seed = W.SEED_C3 if zipf else W.SEED_C2
    ztab = W.zipf_tables(torch, n_grains, seed) if zipf else None
    msgs, per_dest = [], torch.zeros(R, dtype=torch.int64, device="cuda")
    for r in range(R):
        m = W.device_messages(torch, cl, n_grains, n_msgs, seed, start=r * n_msgs, sender_silos=local_silos(cl.n_silos, R, r),
                              zipf=ztab)
        per_dest += owner_rank_counts(torch, cl, m, n_msgs, ros, R)
        msgs.append(m)
    cap = max(n_msgs, int(per_dest.max().item()))
    cap += cap // 64 + 4096
    engs, nodes, streams, masks, n_acts = [], [], [], [], []
    caches = WarmCaches(ztab[1].cpu().numpy(), reg, owner, ros, R, args.sender_cache) if (args.sender_cache and zipf) else None
    gid = b"bench-rehearsal"
    expect_owned = [int(x) for x in per_dest.cpu().numpy()]
    for r in range(R):
        mine = local_silos(cl.n_silos, R, r)
        mask = np.zeros(cl.n_silos, np.uint8)
        mask[mine] = 1
        masks.append(mask)
        n_act = max(1, int((reg & mask[owner].astype(bool)).sum()))
        n_acts.append(n_act)
        e = GrainDirectoryEngine(n_act=n_act, dir_capacity=n_act, max_batch=max(cap, n_msgs), device=0)
        W.setup_engine(e, cl, local_silos=mine)
        if not args.wire16:
            e.set_wire_types([W.grain_tcd(cl)])
        W.register_population(e, keys, owner, reg, mask, dense_local=True)
        if caches is not None:
            caches.fill(torch, e, keys, owner, r, None)
        engs.append(e)
        nodes.append(GrainNode(e, R, r, ros, max_batch=n_msgs, max_recv=cap, transport=L.TRANSPORT_LOCAL, group_id=gid,
                               chunks=args.chunks))
        streams.append(torch.cuda.Stream())
    torch.cuda.synchronize()
    stats = [dict(owned=0, remote=0, wait_us=0, waits=0) for _ in range(R)]

    def one(r):
        res = nodes[r].route_batch_device(msgs[r], n_msgs, stream=streams[r].cuda_stream)
        stats[r]["owned"] += res.n_owned
        stats[r]["remote"] += res.n_sent_remote
        xs = nodes[r].stats()
        stats[r]["wait_us"] += xs["host_wait_us"]
        stats[r]["waits"] += xs["host_waits"]
        stats[r]["bytes_sent"] = [a + b for a, b in zip(stats[r].get("bytes_sent", [0] * R), xs["bytes_sent"])]
        stats[r]["comm_count"] = xs["comm_count"]
        stats[r]["exchange_mode"] = xs["exchange_mode"]
        stats[r]["last"] = res
        streams[r].synchronize()
        return res.n_owned

    with ThreadPoolExecutor(R) as ex:
        for _ in range(max(1, args.warmup)):
            list(ex.map(one, range(R)))
        torch.cuda.synchronize()
        for st in stats:
            st.update(owned=0, remote=0, wait_us=0, waits=0, bytes_sent=[0] * R)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            list(ex.map(one, range(R)))
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    # every rank's hosted output of the last batch (outside timing): the node's correctness evidence
    t_chk = time.perf_counter()
    bad = []
    for r in range(R):
        errs = node_self_check(torch, engs[r], stats[r]["last"], r, cl, keys, owner, reg, masks[r], n_acts[r], ros,
                               expect_owned[r], args.check_sample, caches=caches)
        if errs:
            log(f"rank {r}: segments (count, width) {[(c, w) for _, c, w in stats[r]['last'].segments]}")
        bad += [f"rank {r}: {e}" for e in errs]
    if sum(st["last"].n_hosted for st in stats) != n_total:
        bad.append(f"the ranks host {sum(st['last'].n_hosted for st in stats)} messages of {n_total}")
    check = "ok" if not bad else "; ".join(bad)
    log(f"rehearsal self-check: {check} ({time.perf_counter() - t_chk:.1f}s)")
    for nd in nodes:
        nd.close()
    for e in engs:
        e.close()
    owned = [st["owned"] / args.steps for st in stats]
    log(f"rehearsal {R} ranks on one GPU: {el * 1e3 / args.steps:.2f} ms/step; owned per rank {[int(x) for x in owned]}")
    return {"metric": "routed grain messages/sec, node protocol rehearsal on ONE GPU (not a scaling number)",
            "value": n_total * args.steps / el, "unit": "messages/s", "n_gpus": 1, "local_ranks": R, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el * 1e3 / args.steps, "higher_is_better": True, "scaling": "none",
            "vs_baseline": None, "dtype": "u32/u64 integer", "data": f"synthetic (config {args.config})",
            "config": {"workload": f"config{args.config} split over {R} ranks ({n_msgs} messages each), orl_node LOCAL "
                                   f"transport, {args.chunks} chunks" + (f", warm sender directory caches of "
                                                                         f"{args.sender_cache} entries per rank"
                                                                         if caches else ""),
                       "receive_capacity": cap},
            "owned_per_rank": owned, "max_over_mean_owned": max(owned) / (sum(owned) / R),
            "sent_remote_per_rank": [st["remote"] / args.steps for st in stats],
            "exchange": {"ncclCommCount": stats[0]["comm_count"], "mode": stats[0]["exchange_mode"],
                         "bytes_sent_per_peer_per_step": [[b / args.steps for b in st["bytes_sent"]] for st in stats],
                         "host_wait_ms_per_step": [st["wait_us"] / 1e3 / args.steps for st in stats],
                         "host_wait_ms_per_chunk": [st["wait_us"] / 1e3 / args.steps / max(1, args.chunks) for st in stats],
                         "host_waits_per_step": [st["waits"] / args.steps for st in stats]},
            "check": check, "check_sample_per_rank": args.check_sample, "roofline": None, "cpu_baseline": None}


def run_host_io(args, torch, eng, cl, d_msgs, n_msgs, n_act, n_grains):
    """The host-array call a .NET silo makes (orl_route_batch): headers in host memory, outputs to host memory, PCIe
    both ways, chunked H2D / route / D2H overlap.  Not the bench headline (inputs are not HBM-resident)."""
    from orleans_amd import _lib as L
    msgs = d_msgs.cpu().numpy().reshape(-1).view(L.MSG_DTYPE)
    outs = [np.empty(n_msgs, np.uint32) for _ in range(3)] + [np.empty(n_act + 2, np.uint32)]
    narrow = args.host_io == "narrow"
    pinned = args.host_io in ("pinned", "narrow")
    rec_bytes = 8 if narrow else 32
    if narrow:  # the silo's batch as 8-B records {N1 low 32 bits, meta} with the grain class as wire type 0
        from orleans_amd import workloads as W
        eng.set_wire_types([W.grain_tcd(cl)])
        recs = np.empty((n_msgs, 2), np.uint32)
        recs[:, 0] = msgs["n1"].astype(np.uint32)
        recs[:, 1] = (msgs["sending_silo"].astype(np.uint32) | (msgs["category"].astype(np.uint32) << 8) |
                      (msgs["flags"].astype(np.uint32) << 10) | (msgs["target_silo"].astype(np.uint32) << 24))
        assert (msgs["n1"] < (1 << 32)).all() and (msgs["n0"] == 0).all()
        src = recs

        def call():
            eng.route_batch_narrow_host(recs, *outs)
    else:
        src = msgs

        def call():
            eng.route_batch_host(msgs, *outs)
    if pinned:
        for a in [src] + outs:
            eng.host_register(a)
    for _ in range(max(1, args.warmup)):
        call()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        call()
    el = time.perf_counter() - t0
    if pinned:
        for a in [src] + outs:
            eng.host_unregister(a)
    eng.close()
    pcie = n_msgs * (rec_bytes + 12) + 4 * (n_act + 2)
    log(f"host io ({args.host_io}): {el * 1e3 / args.steps:.2f} ms per {n_msgs} messages, {pcie / (el / args.steps) / 1e9:.1f} GB/s PCIe")
    return {"metric": "routed grain messages/sec (node), host arrays over PCIe", "value": n_msgs * args.steps / el,
            "unit": "messages/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u32/u64 integer", "data": "synthetic (config 2)",
            "config": {"workload": f"config2 through {'orl_route_batch_narrow' if narrow else 'orl_route_batch'} with "
                                   f"{'pinned' if pinned else 'pageable'} host arrays: {rec_bytes} B in, 12 B + offsets out per "
                                   "message over PCIe, chunked upload / route / download overlap"},
            "pcie_bytes_per_step": pcie, "pcie_bytes_per_msg": pcie / n_msgs, "pcie_GBs": pcie / (el / args.steps) / 1e9,
            "roofline": None, "cpu_baseline": None}


def cpu_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model, os.cpu_count() or 1, len(os.sched_getaffinity(0))


def cpu_baseline(cl, n_grains, d_msgs, target_wall, zipf, reg_frac=1.0):
    """The oracle (C++ restatement of the reference per-message path: linear FindLast ring scan, unordered_map partition,
    per-activation FIFO) on the host cores, as the reference's CPU path stand-in (.NET cannot run here): on the box's CPU
    share (OMP_NUM_THREADS threads, the cores this job may use), on every CPU the OS lists (a bounded sample; the threads
    then time-share the share's cores), and on 1 thread.  The reported value and `cores` are the box share's run (the
    cores this job owns); the other two are reported beside it."""
    from oracle import cpu_ref
    from orleans_amd import _lib as L
    from orleans_amd import workloads as W

    model, ncpu, navail = cpu_info()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or navail
    share = max(1, min(share, navail))
    keys, uni, owner, reg = W.grain_population(cl, n_grains, reg_frac)
    o = cpu_ref.Oracle(cl.n_silos)
    for s in range(cl.n_silos):
        o.add_server(s, int(cl.hashes[s]))
    idx = np.nonzero(reg)[0]
    o.register(keys[idx], idx.astype(np.uint32), owner[idx])
    n_all = d_msgs.shape[0]

    def host(k):
        return d_msgs[:k].cpu().numpy().reshape(-1).view(L.MSG_DTYPE)

    def timed(msgs, threads):
        t0 = time.perf_counter()
        o.route_bucket_mt(msgs, n_grains, threads)
        return time.perf_counter() - t0

    probe = host(min(n_all, 1 << 21))
    t_probe = timed(probe, share)
    # three timed repetitions of a third of the wall budget each: the value is their median, with the spread beside it
    # (one sample of a shared host's cores varied 2x between boxes)
    n_mt = int(min(n_all, max(len(probe), len(probe) * target_wall / 3 / max(t_probe, 1e-6))))
    sample = host(n_mt)
    reps = sorted(timed(sample, share) for _ in range(3))
    runs = {"share": {"threads": share, "messages": n_mt, "seconds": reps[1],
                      "spread_msgs_per_s": [n_mt / reps[2], n_mt / reps[0]]}}
    # every listed CPU (the parallel stage 4 keeps 2^12 + 2^(bits-12) counters per thread: no memory bound)
    n_cpu_threads = ncpu
    if n_cpu_threads > share:
        runs["all_cpus"] = {"threads": n_cpu_threads, "messages": n_mt, "seconds": timed(sample, n_cpu_threads)}
    n_1 = min(len(sample), 1 << 22)
    runs["one"] = {"threads": 1, "messages": n_1, "seconds": timed(sample[:n_1], 1)}
    for r in runs.values():
        r["value"] = r["messages"] / r["seconds"]
    best = runs["share"]
    log("cpu baseline: " + ", ".join(f"{k} {r['threads']} threads {r['value'] / 1e6:.1f} M msgs/s" for k, r in runs.items()) +
        f" ({model})")
    return {"value": best["value"], "unit": "messages/s", "cores": best["threads"], "kind": "port",
            "threads_share": runs["share"], "threads_all": runs.get("all_cpus"), "threads_1": runs["one"],
            "cpu_model": model, "os_cpu_count": ncpu, "sched_affinity": navail,
            "box_thread_share_env": os.environ.get("OMP_NUM_THREADS"),
            "spread": runs["share"]["spread_msgs_per_s"],
            "sample": f"first {n_mt} of the {n_all} messages of this workload"
                      f"{' (the whole batch)' if n_mt == n_all else ''}, the median of 3 timed runs on {share} threads (the "
                      f"box's CPU share; min / max in `spread`) and on "
                      f"{runs.get('all_cpus', runs['share'])['threads']} threads, the first {n_1} on 1 thread; same "
                      f"directory, stages 1-4, oracle/cpu_ref.cpp ref_route_bucket_mt"}


def cpu_step_baseline(o, make_msgs, n_act, target_wall, what):
    """The oracle's stages 1-4 (ref_route_bucket_mt) over one step's messages, made by make_msgs() (the oracle's own
    expansion for fan-out steps, timed with it), on the box's CPU share and on 1 thread."""
    from oracle import cpu_ref  # noqa: F401  (the checker; outside every timed GPU region)
    model, ncpu, navail = cpu_info()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or navail
    share = max(1, min(share, navail))
    runs = {}
    for key, threads in (("share", share), ("one", 1)):
        reps, n_done = 0, 0
        t0 = time.perf_counter()
        while True:
            msgs = make_msgs()
            o.route_bucket_mt(msgs, n_act, threads)
            reps += 1
            n_done += len(msgs)
            if time.perf_counter() - t0 > target_wall / 2:
                break
        el = time.perf_counter() - t0
        runs[key] = {"threads": threads, "messages": n_done, "seconds": el, "value": n_done / el, "steps": reps}
    log("cpu baseline: " + ", ".join(f"{k} {r['threads']} threads {r['value'] / 1e6:.2f} M msgs/s" for k, r in runs.items()))
    return {"value": runs["share"]["value"], "unit": "messages/s", "cores": share, "kind": "port", "cpu_model": model,
            "threads_share": runs["share"], "threads_1": runs["one"], "box_thread_share_env": os.environ.get("OMP_NUM_THREADS"),
            "sample": f"{runs['share']['steps']} whole steps ({what}) on {share} threads (the box's CPU share), "
                      f"{runs['one']['steps']} on 1 thread; oracle/cpu_ref.cpp expansion + ref_route_bucket_mt"}


# ---- config 1: Chirper generator graph, one silo --------------------------------------------------------------
def run_chirper(args, torch):
    """BASELINE configs[0]: the ChirperNetworkGenerator deterministic graph (1k accounts x 10 followers) on one silo,
    every account publishes once = 10k routed messages per step (fan-out + stages 1-4); the CPU leg is the oracle's
    expansion + routing + bucketing of the same step on 1 thread (the reference runs it in one silo process)."""
    from oracle import cpu_ref
    from orleans_amd import workloads as W
    from orleans_amd.engine import GrainDirectoryEngine, grain_keys_from_longs, silo_consistent_hash

    n_acc, k = 1000, 10
    src, tgt = W.chirper_graph_deterministic(n_acc, k)
    off, ftgt = W.csr_from_edges(tgt - 1, src, n_acc)  # `source follows target`: the target publishes to its followers
    tc = W.calc_id_hash(W.CHIRPER_ACCOUNT_CLASS)
    h0 = silo_consistent_hash(f"10.0.0.1:{W.PORT}", 1)
    eng = GrainDirectoryEngine(n_act=n_acc, dir_capacity=n_acc, max_batch=1 << 15, device=0)
    eng.set_silos(1)
    eng.add_server(0, h0)
    keys = grain_keys_from_longs(tc, np.arange(1, n_acc + 1, dtype=np.int64))
    eng.register_single_activation(keys, np.arange(n_acc, dtype=np.uint32), np.zeros(n_acc, np.uint8))
    tcd = (3 << 56) + (tc & 0x00FFFFFFFFFFFFFF)
    dv = "cuda"
    d_off = torch.from_numpy(off.view(np.int64)).to(dv)
    d_tgt = torch.from_numpy(ftgt.view(np.int32)).to(dv)
    pubs = np.arange(n_acc, dtype=np.uint32)
    d_pubs = torch.from_numpy(pubs.view(np.int32)).to(dv)
    d_ps = torch.zeros(n_acc, dtype=torch.uint8, device=dv)
    n = n_acc * k
    poff = torch.empty(n_acc + 1, dtype=torch.int64, device=dv)
    outs = [torch.empty(n, dtype=torch.int32, device=dv) for _ in range(3)]
    offs = torch.empty(n_acc + 2, dtype=torch.int32, device=dv)
    s = torch.cuda.Stream()

    def step():
        eng.fanout_device(d_off, d_tgt, d_pubs, d_ps, n_acc, tcd, poff, *outs, offs, stream=s.cuda_stream, total=n)

    with torch.cuda.stream(s):
        for _ in range(max(args.warmup, 2)):
            step()
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        step()
    steps = max(args.steps, 100)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        for _ in range(steps):
            g.replay()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    eng.close()
    # CPU: the oracle's per-message path over the same step (1 thread, the reference's single silo)
    o = cpu_ref.Oracle(1)
    o.add_server(0, h0)
    o.register(keys, np.arange(n_acc, dtype=np.uint32), np.zeros(n_acc, np.uint8))
    reps = 0
    t0 = time.perf_counter()
    while True:
        msgs, _ = cpu_ref.fanout_expand(off, ftgt, pubs, np.zeros(n_acc, np.uint8), tcd)
        o.route_bucket_mt(msgs, n_acc, 1)
        reps += 1
        if time.perf_counter() - t0 > args.cpu_wall:
            break
    cpu_wall = time.perf_counter() - t0
    log(f"config 1: {el * 1e6 / steps:.1f} us/step on the GPU (graph replay), {cpu_wall * 1e6 / reps:.1f} us/step on 1 CPU thread")
    return {"metric": "routed grain messages/sec (node)", "value": n * steps / el, "unit": "messages/s", "n_gpus": 1,
            "steps": steps, "warmup": args.warmup, "ms_per_step": el * 1e3 / steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32/u64 integer",
            "data": "ChirperNetworkGenerator deterministic graph (ChirperNetworkGenerator.cs:306-345)",
            "config": {"workload": "config1: Chirper 1k accounts x 10 followers on one silo, every account publishes once "
                                   "(10k routed messages per step), fan-out + stages 1-4, hipGraph replay"},
            "roofline": None,
            "cpu_baseline": {"value": n * reps / cpu_wall, "unit": "messages/s", "cores": 1, "kind": "port",
                             "cpu_model": cpu_info()[0],
                             "sample": f"{reps} whole steps (expand + route + bucket, oracle/cpu_ref.cpp) on 1 thread"}}


# ---- config 4: CSR multicast fan-out ---------------------------------------------------------------------
def run_fanout(args, torch):
    from orleans_amd import workloads as W
    from orleans_amd.engine import GrainDirectoryEngine, grain_keys_from_longs

    n_acc = args.grains or 10_000_000
    n_pub = 1_000_000
    cl = W.default_cluster()
    t_setup = time.perf_counter()
    csr_off, csr_tgt = W.powerlaw_csr(n_acc)
    keys = grain_keys_from_longs(cl.type_code, np.arange(n_acc, dtype=np.int64))
    owner = cl.owner_of(W.jenkins3_np(keys["tcd"], keys["n0"], keys["n1"]))
    # publishers per step: 1M uniformly random accounts (a fresh sample each step, pre-generated)
    n_sets = max(1, min(4, args.steps + args.warmup))
    pub_sets = [(W.stream(W.SEED_C4 ^ 0xB0B, i * n_pub, n_pub) % np.uint64(n_acc)).astype(np.uint32)
                for i in range(n_sets)]
    deg = np.diff(csr_off.astype(np.int64))
    totals = [int(deg[p].sum()) for p in pub_sets]
    cap = max(totals) + 1
    eng = GrainDirectoryEngine(n_act=n_acc, dir_capacity=n_acc, max_batch=cap, device=0)
    W.setup_engine(eng, cl)
    W.register_population(eng, keys, owner, np.ones(n_acc, bool))
    log(f"config 4: {n_acc} accounts, {len(csr_tgt)} edges, {n_pub} publishers/step, emitted {totals}")
    dev = "cuda"
    d_off = torch.from_numpy(csr_off.view(np.int64)).to(dev)
    d_tgt = torch.from_numpy(csr_tgt.view(np.int32)).to(dev)
    d_pubs = [torch.from_numpy(p.view(np.int32)).to(dev) for p in pub_sets]
    d_psilo = [torch.from_numpy(owner[p]).to(dev) for p in pub_sets]
    poff = torch.empty(n_pub + 1, dtype=torch.int64, device=dev)
    route = torch.empty(cap, dtype=torch.int32, device=dev)
    act = torch.empty(cap, dtype=torch.int32, device=dev)
    order = torch.empty(cap, dtype=torch.int32, device=dev)
    offs = torch.empty(n_acc + 2, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    k = [0]
    tcd = (3 << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)

    def step():
        i = k[0] % n_sets
        k[0] += 1
        return eng.fanout_device(d_off, d_tgt, d_pubs[i], d_psilo[i], n_pub, tcd, poff, route, act, order, offs,
                                 stream=stream, total=totals[i])
    log(f"setup {time.perf_counter() - t_setup:.1f}s")
    for _ in range(args.warmup):
        step()
    eng.sync()
    eng.set_timing(True)
    args_w = argparse.Namespace(**{**vars(args), "warmup": 0})
    elapsed, emitted = timed_steps(args_w, torch, None, 1, step, eng.sync)
    nb, route_ms, bucket_ms, total_ms = eng.timing_summary()
    eng.close()
    per_step = emitted / args.steps
    bytes_launch = FANOUT_BYTES_PER_MSG * per_step + FANOUT_BYTES_PER_PUB * n_pub
    cpu = None
    if not args.no_cpu:  # the oracle: the step's 1M publishes expanded (ref_fanout_expand) + stages 1-4, host cores
        from oracle import cpu_ref
        o = cpu_ref.Oracle(cl.n_silos)
        for s_ in range(cl.n_silos):
            o.add_server(s_, int(cl.hashes[s_]))
        o.register(keys, np.arange(n_acc, dtype=np.uint32), owner)
        cpu = cpu_step_baseline(o, lambda: cpu_ref.fanout_expand(csr_off, csr_tgt, pub_sets[0], owner[pub_sets[0]], tcd)[0],
                                n_acc, args.cpu_wall * 2, f"{n_pub} publishes -> {totals[0]} messages")
    achieved = bytes_launch / (route_ms * 1e-3) / 1e9
    log(f"config 4: {elapsed * 1e3 / args.steps:.3f} ms/step, fan-out route kernel {route_ms:.3f} ms, "
        f"bucketing {bucket_ms:.3f} ms")
    return {"metric": "routed grain messages/sec (node)", "value": emitted / elapsed, "unit": "messages/s",
            "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32/u64 integer",
            "data": "synthetic (seeded power-law CSR; config 4 of SURVEY §8(d))",
            "config": {"workload": f"config4: {n_acc} accounts, power-law followers (exp 2.1, 1..1e5), "
                                   f"{n_pub} publishers per step, fan-out + stages 1-4",
                       "edges": int(len(csr_tgt)), "emitted_per_step": per_step},
            "roofline": {"bound": "hbm", "kernel": "k_fanout_route (stage 5 + 1-3)", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "bytes_per_msg": FANOUT_BYTES_PER_MSG, "bytes_per_publish": FANOUT_BYTES_PER_PUB,
                         "avg_launch_ms": route_ms},
            "pipeline": {"route_kernel_ms": route_ms, "bucketing_ms": bucket_ms, "call_ms": total_ms},
            "cpu_baseline": cpu}


def run_fanout_node(args, torch, dist, rank, world, local_rank, rehearsal=False):
    """Config 4 sharded across GPUs: the CSR is replicated, each rank publishes for the accounts its
    silos own (1M uniformly random publishers per step in total), expands its publishes and routes the emitted messages
    across the node (orl_node_fanout_batch_device: owner partition, RCCL exchange, routing at the follower's owner,
    stage 4).  rehearsal: `world` ranks as threads of this process on one GPU (LOCAL transport), not a scaling number."""
    from concurrent.futures import ThreadPoolExecutor
    from orleans_amd import _lib as L
    from orleans_amd import workloads as W
    from orleans_amd.engine import GrainDirectoryEngine, grain_keys_from_longs
    from orleans_amd.node import GrainNode, local_silos, rank_of_silo

    n_acc = args.grains or 10_000_000
    n_pub = 1_000_000
    cl = W.balanced_cluster()
    ros = rank_of_silo(cl.n_silos, world)
    t_setup = time.perf_counter()
    csr_off, csr_tgt = W.powerlaw_csr(n_acc)
    keys = grain_keys_from_longs(cl.type_code, np.arange(n_acc, dtype=np.int64))
    owner = cl.owner_of(W.jenkins3_np(keys["tcd"], keys["n0"], keys["n1"]))
    n_sets = max(1, min(4, args.steps + args.warmup))
    pub_sets = [(W.stream(W.SEED_C4 ^ 0xB0B, i * n_pub, n_pub) % np.uint64(n_acc)).astype(np.uint32) for i in range(n_sets)]
    deg = np.diff(csr_off.astype(np.int64))
    pub_rank = [ros[owner[p.astype(np.int64)]] for p in pub_sets]
    totals = [int(deg[p].sum()) for p in pub_sets]
    ranks = list(range(world)) if rehearsal else [rank]
    # per (rank, set): publishers, their silos, emitted count; receive capacity from the followers' owner ranks
    per = {}
    recv = np.zeros(world, np.int64)
    for r in range(world):
        for i, p in enumerate(pub_sets):
            mine_p = p[pub_rank[i] == r]
            emitted = int(deg[mine_p].sum())
            per[(r, i)] = (mine_p, owner[mine_p.astype(np.int64)].astype(np.uint8), emitted)
    for i, p in enumerate(pub_sets):  # every emitted message lands at its follower's owner rank
        starts = csr_off[p.astype(np.int64)].astype(np.int64)
        lens = csr_off[p.astype(np.int64) + 1].astype(np.int64) - starts
        idx = np.repeat(starts - np.cumsum(lens) + lens, lens) + np.arange(int(lens.sum()))  # every emitted CSR entry
        recv = np.maximum(recv, np.bincount(ros[owner[csr_tgt[idx].astype(np.int64)]], minlength=world))
    max_batch = max(e for (_, _, e) in per.values()) + 1
    cap = int(recv.max())
    cap += cap // 64 + 4096
    dev = f"cuda:{local_rank}"
    d_off = torch.from_numpy(csr_off.view(np.int64)).to(dev)
    d_tgt = torch.from_numpy(csr_tgt.view(np.int32)).to(dev)
    tcd = (3 << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)
    gid = b"bench-fanout-rehearsal"
    if not rehearsal:
        g = torch.zeros(L.NODE_ID_BYTES, dtype=torch.uint8, device=dev)
        if rank == 0:
            g.copy_(torch.frombuffer(bytearray(GrainNode.unique_id()), dtype=torch.uint8))
        dist.broadcast(g, 0)
        gid = bytes(g.cpu().numpy())
    state = {}
    for r in ranks:
        mine = local_silos(cl.n_silos, world, r)
        mask = np.zeros(cl.n_silos, np.uint8)
        mask[mine] = 1
        n_act = max(1, int(mask[owner].astype(bool).sum()))
        eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=n_act, max_batch=max(cap, max_batch), device=local_rank)
        W.setup_engine(eng, cl, local_silos=mine)
        if not args.wire16:
            eng.set_wire_types([tcd])
        W.register_population(eng, keys, owner, np.ones(n_acc, bool), mask, dense_local=True)
        node = GrainNode(eng, world, r, ros, max_batch=max_batch, max_recv=cap,
                         transport=L.TRANSPORT_LOCAL if rehearsal else L.TRANSPORT_RCCL, group_id=gid, chunks=args.chunks)
        sets = [(torch.from_numpy(per[(r, i)][0].view(np.int32)).to(dev), torch.from_numpy(per[(r, i)][1]).to(dev),
                 len(per[(r, i)][0]), per[(r, i)][2]) for i in range(n_sets)]
        state[r] = dict(eng=eng, node=node, sets=sets, poff=torch.empty(n_pub + 1, dtype=torch.int64, device=dev),
                        stream=torch.cuda.Stream(device=dev))
    del keys
    log(f"config 4 node: {world} ranks{' (one-GPU rehearsal)' if rehearsal else ''}, {n_acc} accounts, {len(csr_tgt)} edges, "
        f"{n_pub} publishers/step, emitted {totals}, receive capacity {cap}; setup {time.perf_counter() - t_setup:.1f}s")
    k = [0]

    def one(r, i):
        st = state[r]
        d_pubs, d_psilo, npub, emitted = st["sets"][i]
        res = st["node"].fanout_batch_device(d_off, d_tgt, None, tcd, d_pubs, d_psilo, npub, st["poff"], total=emitted,
                                             stream=st["stream"].cuda_stream)
        st["stream"].synchronize()
        return res.n_owned

    if rehearsal:
        ex = ThreadPoolExecutor(world)

        def step():
            i = k[0] % n_sets
            k[0] += 1
            list(ex.map(lambda r: one(r, i), ranks))
            return totals[i]
    else:
        def step():
            i = k[0] % n_sets
            k[0] += 1
            one(rank, i)
            return totals[i]
    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    args_w = argparse.Namespace(**{**vars(args), "warmup": 0})
    elapsed, emitted = timed_steps(args_w, torch, None if rehearsal else dist, 1 if rehearsal else world, step,
                                   torch.cuda.synchronize)
    for st in state.values():
        st["node"].close()
        st["eng"].close()
    ms = elapsed * 1e3 / args.steps
    log(f"config 4 node: {ms:.3f} ms/step, {emitted / args.steps:.0f} emitted messages per step over {world} ranks")
    return {"metric": "routed grain messages/sec (node)" + (", node protocol rehearsal on ONE GPU (not a scaling number)"
                                                           if rehearsal else ""),
            "value": emitted / elapsed, "unit": "messages/s", "n_gpus": 1 if rehearsal else world,
            "local_ranks": world if rehearsal else None, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "none" if rehearsal else "strong", "vs_baseline": None,
            "dtype": "u32/u64 integer", "data": "synthetic (seeded power-law CSR; config 4 of SURVEY §8(d))",
            "config": {"workload": f"config4 sharded by publisher over {world} ranks: {n_acc} accounts, power-law followers, "
                                   f"{n_pub} publishers per step in total, each rank expands its own and routes the emitted "
                                   f"messages across the node (orl_node_fanout_batch_device, {args.chunks} chunks)",
                       "edges": int(len(csr_tgt)), "emitted_per_step": emitted / args.steps, "receive_capacity": cap},
            "roofline": None, "cpu_baseline": None}


# ---- leg 6: directory mutation (f1) ------------------------------------------------------------------------
def run_directory(args, torch):
    """16M ChirperAccount grains registered on the device in batches of 4M (RegisterSingleActivation with
    batch-order first-writer-wins), then 10 % unregistered and re-registered; registrations/s per batch."""
    from orleans_amd import workloads as W
    from orleans_amd.engine import GrainDirectoryEngine

    n, batch = args.grains or 16_000_000, 4 << 20
    cl = W.balanced_cluster()
    keys, uni, owner, reg = W.grain_population(cl, n)
    eng = GrainDirectoryEngine(n_act=n, dir_capacity=n, max_batch=batch, device=0)
    W.setup_engine(eng, cl)
    dev = "cuda"
    d_keys = torch.from_numpy(keys.view(np.uint8).reshape(-1, 24)).to(dev)
    d_acts = torch.arange(n, dtype=torch.int32, device=dev)
    d_silos = torch.from_numpy(owner.astype(np.uint8)).to(dev)
    d_st = torch.empty(batch, dtype=torch.uint8, device=dev)
    d_wa = torch.empty(batch, dtype=torch.int32, device=dev)
    d_ws = torch.empty(batch, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b0 in range(0, n, batch):
        m = min(batch, n - b0)
        eng.register_single_activation_device(d_keys[b0:b0 + m], d_acts[b0:b0 + m], d_silos[b0:b0 + m], m, d_st, d_wa,
                                              d_ws, stream=stream)
    torch.cuda.synchronize()
    t_ins = time.perf_counter() - t0
    assert eng.directory_count() == n
    m = n // 10
    d_rm = torch.empty(m, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b0 in range(0, m, batch):
        k = min(batch, m - b0)
        eng.unregister_device(d_keys[b0:b0 + k], k, d_rm[b0:b0 + k], stream=stream)
    for b0 in range(0, m, batch):
        k = min(batch, m - b0)
        eng.register_single_activation_device(d_keys[b0:b0 + k], d_acts[b0:b0 + k], d_silos[b0:b0 + k], k, d_st, d_wa,
                                              d_ws, stream=stream)
    torch.cuda.synchronize()
    t_churn = time.perf_counter() - t0
    assert eng.directory_count() == n
    eng.close()
    log(f"directory: {n} registrations in {t_ins * 1e3:.1f} ms; {m} removals + {m} re-registrations in "
        f"{t_churn * 1e3:.1f} ms")
    return {"metric": "directory registrations/sec", "value": n / t_ins, "unit": "registrations/s", "n_gpus": 1,
            "steps": 1, "warmup": 0, "ms_per_step": t_ins * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32/u64 integer", "data": "synthetic (config-3 population)",
            "config": {"workload": f"leg 6: {n} long-key grains registered on the device in batches of {batch}, then "
                                   f"{m} unregistered + re-registered", "table_slots": 1 << (2 * n - 1).bit_length()},
            "churn_ops_per_s": 2 * m / t_churn, "roofline": None, "cpu_baseline": None}


# ---- leg 7: stream / reminder rings (f3) -----------------------------------------------------------------
def run_rings(args, torch):
    """64M reminder keys → owning silo under the virtual-bucket ring (8 silos x 30 buckets) and the consistent
    ring, and 64M stream Guids → queue (256 queues) + pulling silo; per-kind ms and keys/s."""
    from orleans_amd import _lib as L
    from orleans_amd import workloads as W
    from orleans_amd.engine import GrainDirectoryEngine

    n = args.msgs
    cl = W.balanced_cluster()
    eng = GrainDirectoryEngine(n_act=4, dir_capacity=16, max_batch=1024, device=0)
    W.setup_engine(eng, cl)
    gens = W.balanced_generations(cl.n_silos)
    for s in range(cl.n_silos):
        eng.vring_add_server(s, bytes(12) + bytes([10, 0, 0, s + 1]), W.PORT, gens[s])
    d_keys = torch.randint(-(1 << 31), (1 << 31) - 1, (n,), dtype=torch.int32, device="cuda")
    d_guids = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device="cuda")
    d_own = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_q = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    out = {}
    for name, fn in (("vbuckets", lambda: eng.ring_owner_device(L.RING_VBUCKETS, d_keys, n, 0, d_own, stream=st)),
                     ("consistent", lambda: eng.ring_owner_device(L.RING_CONSISTENT, d_keys, n, 0, d_own, stream=st)),
                     ("stream_queue", lambda: eng.stream_queue_device(L.RING_VBUCKETS, d_guids, n, 256, 0, d_q, d_own,
                                                                      stream=st))):
        for _ in range(max(args.warmup, 1)):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        out[name] = (time.perf_counter() - t0) * 1e3 / args.steps
    eng.close()
    log("rings: " + ", ".join(f"{k} {v:.3f} ms" for k, v in out.items()) + f" per {n} keys")
    return {"metric": "ring lookups/sec", "value": n / (out["vbuckets"] * 1e-3), "unit": "keys/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": out["vbuckets"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32 integer", "data": "synthetic (random keys / Guids)",
            "config": {"workload": f"leg 7: {n} uniform-hash keys → silo (virtual-bucket ring, 8 x 30 buckets); also the "
                                   f"consistent ring and {n} stream Guids → 256 queues + pulling silo"},
            "ms": out, "roofline": {"bound": "hbm", "kernel": "k_ring_owner<VBUCKETS>",
                                    "achieved": 5.0 * n / (out["vbuckets"] * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                                    "unit": "GB/s", "frac": 5.0 * n / (out["vbuckets"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                    "traffic": None, "bytes_per_key": 5},
            "cpu_baseline": None}


def run_wire(args, torch):
    """Receive path: a receive buffer of back-to-back frames (config-2 addressing, 20% complete
    addresses, 5% KeyExt targets, bodies 0-48 B) decoded into headers on the device, then routed + bucketed."""
    from orleans_amd import _lib as L
    from orleans_amd import workloads as W
    from orleans_amd.engine import GrainDirectoryEngine

    n, n_grains = args.frames, args.grains or (1 << 24)
    cl = W.balanced_cluster()
    eng = GrainDirectoryEngine(n_act=n_grains, dir_capacity=n_grains, max_batch=n, device=0)
    W.setup_engine(eng, cl)
    W.register_silo_addresses(eng, cl)
    keys, _, owner, reg = W.grain_population(cl, n_grains, 1.0)
    W.register_population(eng, keys, owner, reg)
    t0 = time.perf_counter()
    buf, offs, exp = W.request_frames(cl, n_grains, n, complete_frac=0.2, keyext_frac=0.05)
    log(f"wire: {n} frames, {len(buf) / 2**20:.0f} MiB built in {time.perf_counter() - t0:.1f} s")
    hl = np.array([int.from_bytes(bytes(buf[int(o):int(o) + 4]), "little") for o in offs[:4096]])
    d_buf = torch.from_numpy(buf).cuda()
    d_off = torch.from_numpy(offs.view(np.int64)).cuda()
    d_hdr = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    d_st = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    d_r = torch.empty(n, dtype=torch.int32, device="cuda")
    d_a = torch.empty(n, dtype=torch.int32, device="cuda")
    d_o = torch.empty(n, dtype=torch.int32, device="cuda")
    d_f = torch.empty(n_grains + 2, dtype=torch.int32, device="cuda")
    stream = torch.cuda.Stream()  # the library launches on this stream; events are recorded on it too
    st = stream.cuda_stream

    def decode():
        eng.decode_frames_device(d_buf, len(buf), d_off, n, d_hdr, d_st, d_bad, stream=st)

    def decode_route():
        decode()
        eng.address_messages_device(d_hdr, n, d_r, d_a, d_o, d_f, stream=st)

    # emit: the routed frames re-serialized with SetTargetPlacement (ActivationId key per activation handle)
    akeys = np.zeros(n_grains, L.KEY_DTYPE)
    akeys["n0"] = np.arange(n_grains, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    akeys["n1"] = np.arange(n_grains, dtype=np.uint64)
    d_akeys = torch.from_numpy(akeys.view(np.uint8)).cuda()
    eng_types = [(cl.type_code, "Orleans.Samples.Chirper.Grains.ChirperAccount")]
    for code, name in eng_types:
        eng.set_grain_type(code, name)
    out_cap = len(buf) + n * (L.STAMP_MAX_GROWTH + 64)
    d_sout = torch.empty(out_cap, dtype=torch.uint8, device="cuda")
    d_soff = torch.empty(n, dtype=torch.int64, device="cuda")
    d_stot = torch.empty(1, dtype=torch.int64, device="cuda")
    d_sst = torch.empty(n, dtype=torch.uint8, device="cuda")

    def stamp():
        eng.stamp_frames_device(d_buf, len(buf), d_off, n, d_r, d_a, d_akeys, n_grains, None, d_sout, out_cap, d_soff,
                                d_stot, d_sst, stream=st)

    def receive_route_emit():
        decode_route()
        stamp()

    decode()
    torch.cuda.synchronize()
    assert int(d_bad.item()) == 0, "synthetic frames must decode cleanly"
    got = d_hdr[:4096].cpu().numpy().reshape(-1).view(L.MSG_DTYPE)
    for f in ("tcd", "n1", "sending_silo", "flags", "target_silo"):
        assert (got[f] == exp[f][:4096]).all(), f
    out = {}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    decode_route()
    stamp()
    torch.cuda.synchronize()
    sst = np.bincount(d_sst.cpu().numpy(), minlength=6)
    log(f"wire: stamp statuses {sst.tolist()} (OK, COMPLETE, SKIPPED, UNSUPPORTED, MALFORMED, OVERFLOW), "
        f"{int(d_stot.item()) / 2**20:.0f} MiB out")
    for name, fn in (("decode", decode), ("decode_route", decode_route), ("stamp", stamp),
                     ("decode_route_stamp", receive_route_emit)):
        for _ in range(max(args.warmup, 1)):
            fn()
        torch.cuda.synchronize()
        ev[0].record(stream)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        ev[1].record(stream)
        torch.cuda.synchronize()
        out[name] = (time.perf_counter() - t0) * 1e3 / args.steps
        out[name + "_event"] = ev[0].elapsed_time(ev[1]) / args.steps
    # algorithmic bytes per decode: the 8-byte prefix + header of every frame, its offset (8), the record (32)
    # and status (1) written; bodies are not touched
    mean_hl = float(hl.mean())
    alg = n * (8 + mean_hl + 8 + 32 + 1)
    traffic = None  # measured HBM bytes per launch (profiles/r01_leg8_decode_pmc.json), for this batch size only
    tj = os.path.join(ROOT, "profiles", "r01_leg8_decode_pmc.json")
    if os.path.exists(tj):
        rec = json.load(open(tj))
        if rec.get("frames_per_launch") == n:
            traffic = rec.get("hbm_bytes_per_launch")
    eng.close()
    cpu = None
    if not args.no_cpu:
        cpu = wire_cpu_baseline(buf, offs, cl, args.cpu_wall)
    log("wire: " + ", ".join(f"{k} {v:.3f} ms" for k, v in out.items()) + f" per {n} frames (mean header {mean_hl:.0f} B)")
    ms = out["decode_route_stamp"]
    return {"metric": "frames decoded+routed+re-serialized/sec", "value": n / (ms * 1e-3), "unit": "frames/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8/u32 integer",
            "data": "synthetic frames (request / response header dictionaries as SerializeMessageHeaders writes them)",
            "config": {"workload": f"leg 8: {n} frames -> headers (device decode) -> route + bucket -> frames "
                                   f"re-serialized with the placement (SetTargetPlacement), {n_grains} registered grains"},
            "ms": out, "decode_frames_per_s": n / (out["decode_event"] * 1e-3),
            "roofline": {"bound": "hbm", "kernel": "k_decode_frames", "achieved": alg / (out["decode_event"] * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / (out["decode_event"] * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_frame": 8 + mean_hl + 41},
            "cpu_baseline": cpu}


def wire_cpu_baseline(buf, offs, cl, target_wall):
    """oracle/wire_codec.decode_frames (pure Python, 1 core) on a bounded prefix of the same buffer."""
    from oracle import wire_codec as WC
    from orleans_amd import workloads as W
    idx = {(cl.silo_ip16(s), W.PORT, cl.gens[s]): s for s in range(cl.n_silos)}
    raw = bytes(buf[:int(offs[min(len(offs) - 1, 200_000)])])
    n = 2000
    while True:
        t0 = time.perf_counter()
        WC.decode_frames(raw, [int(o) for o in offs[:n]], idx)
        dt = time.perf_counter() - t0
        if dt > target_wall or n >= 200_000:
            break
        n = min(200_000, int(n * max(2.0, target_wall / max(dt, 1e-3))))
    return {"value": n / dt, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"first {n} frames of the same buffer through oracle/wire_codec.decode_frames (Python)"}


# ---- config 5: Presence heartbeats, small batches, hipGraph --------------------------------------------
def run_presence(args, torch):
    from orleans_amd import workloads as W
    from orleans_amd.engine import GrainDirectoryEngine

    n_games, per_game, n_hb = 100_000, 8, 64 * 1024
    log("config 5: building population")
    cl = W.default_cluster()
    pr = W.presence_population(n_games, per_game)
    n_keys = n_games * (1 + per_game)
    all_keys = np.concatenate([pr.game_keys, pr.player_keys])
    owner = cl.owner_of(W.jenkins3_np(all_keys["tcd"], all_keys["n0"], all_keys["n1"]))
    n_fan = n_hb * per_game
    mixed = args.c5_mode == "mixed"
    eng = GrainDirectoryEngine(n_act=n_keys, dir_capacity=n_keys, max_batch=n_fan + (n_hb if mixed else 0), device=0)
    W.setup_engine(eng, cl)
    W.register_population(eng, all_keys, owner, np.ones(n_keys, bool))
    # --c5-contexts 2: the game messages and the player fan-out of a step are independent, so they run concurrently on
    # two routing contexts (each with its own scratch and a copy of the partition) and two streams, forked and
    # joined inside the step; a 64k-message batch alone fills only a few dozen workgroups.
    eng2 = eng
    if args.c5_contexts > 1 and not mixed:
        eng2 = GrainDirectoryEngine(n_act=n_keys, dir_capacity=n_keys, max_batch=n_fan, device=0)
        W.setup_engine(eng2, cl)
        W.register_population(eng2, all_keys, owner, np.ones(n_keys, bool))
    n_sets = 8
    batches = [W.heartbeat_batch(pr, cl, n_hb, b) for b in range(n_sets)]
    dev = "cuda"
    d_msgs = [torch.from_numpy(m.view(np.int32).reshape(-1, 8)).to(dev) for _, m in batches]
    d_games = [torch.from_numpy(g.view(np.int32)).to(dev) for g, _ in batches]
    d_gsilo = [torch.from_numpy(owner[g.astype(np.int64)]).to(dev) for g, _ in batches]
    d_off = torch.from_numpy(pr.csr_off.view(np.int64)).to(dev)
    d_tgt = torch.from_numpy(pr.csr_tgt.view(np.int32)).to(dev)
    d_pkeys = torch.from_numpy(pr.player_keys.view(np.uint8).reshape(-1, 24)).to(dev)
    o1 = [torch.empty(n_hb, dtype=torch.int32, device=dev) for _ in range(3)]
    o2 = [torch.empty(n_fan + (n_hb if mixed else 0), dtype=torch.int32, device=dev) for _ in range(3)]
    off1 = torch.empty(n_keys + 2, dtype=torch.int32, device=dev)
    off2 = torch.empty(n_keys + 2, dtype=torch.int32, device=dev)
    poff = torch.empty(n_hb + 1, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream()
    sp = s.cuda_stream
    s2 = torch.cuda.Stream() if eng2 is not eng else s
    sp2 = s2.cuda_stream

    def one_mixed(i):
        # the step's outbound batch in one call: the 64k game messages (PresenceGrain.Heartbeat →
        # GameGrain.UpdateGameStatus) then their 8-way player fan-out (GameGrain.UpdateGameStatus →
        # PlayerGrain.JoinGame/LeaveGame), one route launch and one stage-4 pass
        eng.fanout_mixed_device(d_msgs[i], n_hb, d_off, d_tgt, d_pkeys, 0, d_games[i], d_gsilo[i], n_hb, poff,
                                o2[0], o2[1], o2[2], off2, stream=sp, total=n_hb + n_fan)

    def one(i):
        if mixed:
            return one_mixed(i)
        if s2 is not s:
            s2.wait_stream(s)  # fork
        # 1 game message per heartbeat (PresenceGrain.Heartbeat → GameGrain.UpdateGameStatus) ...
        eng.address_messages_device(d_msgs[i], n_hb, o1[0], o1[1], o1[2], off1, stream=sp)
        # ... + the 8-way player fan-out (GameGrain.UpdateGameStatus → PlayerGrain.JoinGame/LeaveGame)
        eng2.fanout_keys_device(d_off, d_tgt, d_pkeys, d_games[i], d_gsilo[i], n_hb, poff, o2[0], o2[1], o2[2], off2,
                                stream=sp2, total=n_fan)
        if s2 is not s:
            s.wait_stream(s2)  # join: the step ends on s

    per_step = n_hb + n_fan
    log("config 5: warmup")
    with torch.cuda.stream(s):
        for i in range(max(2, args.warmup)):
            one(i % n_sets)
    s.synchronize()

    # every launch and every graph replay goes to stream s (CUDAGraph.replay() runs on the current stream)
    def lat_run(fn, steps):
        lat = []
        with torch.cuda.stream(s):
            for i in range(steps):
                t0 = time.perf_counter()
                fn(i)
                s.synchronize()
                lat.append((time.perf_counter() - t0) * 1e3)
        return np.array(lat)

    def thr_run(fn, steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            for i in range(steps):
                fn(i)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    steps = max(args.steps, 20)
    lat_eager = lat_run(lambda i: one(i % n_sets), steps)
    thr_eager = thr_run(lambda i: one(i % n_sets), steps)
    # hipGraph: capture one batch per heartbeat set, replay
    log("config 5: eager done, capturing graphs")
    graphs = []
    for i in range(n_sets):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            one(i)
        graphs.append(g)
    s.synchronize()
    # the replayed graphs must produce the eager call's words (guards against an empty or stale capture)
    outs = o2 + [off2] if mixed else o1 + o2 + [off1, off2]
    for i in range(n_sets):
        for x in outs:
            x.fill_(-1)
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            graphs[i].replay()
        s.synchronize()
        rep = [x.clone() for x in outs]
        with torch.cuda.stream(s):
            one(i)
        s.synchronize()
        if not all(bool(torch.equal(a, b)) for a, b in zip(rep, outs)):
            raise RuntimeError(f"graph replay of heartbeat batch {i} differs from the eager call")
    log("config 5: graphs verified")
    lat_graph = lat_run(lambda i: graphs[i % n_sets].replay(), steps)
    thr_graph = thr_run(lambda i: graphs[i % n_sets].replay(), steps)
    # all n_sets steps in one graph (one launch per n_sets ticks: the per-launch gap amortised)
    g_all = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_all, stream=s):
        for i in range(n_sets):
            one(i)
    s.synchronize()
    reps = max(1, steps // n_sets)
    thr_graph_all = thr_run(lambda i: g_all.replay(), reps)
    # the route kernel's own time (HIP events around it on stream s), eager steps after the timed runs
    roof = None
    if mixed:
        eng.set_timing(True)
        with torch.cuda.stream(s):
            for i in range(steps):
                one(i % n_sets)
        s.synchronize()
        nb, route_ms, bucket_ms, total_ms = eng.timing_summary()
        eng.set_timing(False)
        bytes_launch = PRESENCE_BYTES_DIRECT * n_hb + PRESENCE_BYTES_FANOUT * n_fan + PRESENCE_BYTES_PER_PUB * n_hb
        achieved = bytes_launch / (route_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": "k_fanout_route (direct + fan-out, stages 5 + 1-3)", "achieved": achieved,
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                "bytes_per_launch": bytes_launch, "avg_launch_ms": route_ms, "bucketing_ms": bucket_ms, "call_ms": total_ms,
                "note": "a 590k-message step fills the chip for ~10 us per kernel: launch- and latency-bound, not HBM-bound"}
    eng.close()
    if eng2 is not eng:
        eng2.close()
    cpu = None
    if not args.no_cpu:  # the oracle over the same step: game messages + the player fan-out named by the key table
        from oracle import cpu_ref
        o = cpu_ref.Oracle(cl.n_silos)
        for s_ in range(cl.n_silos):
            o.add_server(s_, int(cl.hashes[s_]))
        o.register(all_keys, np.arange(n_keys, dtype=np.uint32), owner)
        g0, m0 = batches[0]

        def make_msgs():
            exp, _ = cpu_ref.fanout_expand(pr.csr_off, pr.csr_tgt, g0, owner[g0.astype(np.int64)], 0)
            k = pr.player_keys[exp["n1"].astype(np.int64)]
            exp["tcd"], exp["n0"], exp["n1"] = k["tcd"], k["n0"], k["n1"]
            return np.concatenate([m0, exp])
        cpu = cpu_step_baseline(o, make_msgs, n_keys, args.cpu_wall, f"{n_hb} game messages + {n_fan} player messages")
    # the step's three launch forms all do the whole step's work; the value is the fastest (named in config.timed_form).
    # A one-step graph replay pays the HIP runtime's per-graph-launch gap (~5-8 us); 8 steps per graph amortise it
    forms = {"eager": thr_eager * 1e3 / steps, "graph": thr_graph * 1e3 / steps,
             f"graph_{n_sets}_steps_per_launch": thr_graph_all * 1e3 / (reps * n_sets)}
    best = min(forms, key=forms.get)
    value = per_step / (forms[best] * 1e-3)
    log(f"config 5: eager {thr_eager * 1e3 / steps:.3f} ms/step (p50 {np.percentile(lat_eager, 50):.3f}, "
        f"p99 {np.percentile(lat_eager, 99):.3f} ms); graph {thr_graph * 1e3 / steps:.3f} ms/step "
        f"(p50 {np.percentile(lat_graph, 50):.3f}, p99 {np.percentile(lat_graph, 99):.3f} ms); "
        f"{n_sets} steps per graph {thr_graph_all * 1e3 / (reps * n_sets):.3f} ms/step")
    return {"metric": "routed grain messages/sec (node)", "value": value, "unit": "messages/s", "n_gpus": 1,
            "steps": steps, "warmup": args.warmup, "ms_per_step": forms[best], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32/u64 integer",
            "data": "synthetic (seeded Guids; config 5 of SURVEY §8(d))",
            "config": {"workload": f"config5: {n_games} Guid-keyed games x {per_game} players, {n_hb} heartbeats per "
                                   f"step = {n_hb} game + {n_fan} player messages, stages 1-5",
                       "timed_form": best, "messages_per_step": per_step, "mode": args.c5_mode,
                       "routing_contexts": 1 if mixed else args.c5_contexts},
            "latency_ms": {"eager_p50": float(np.percentile(lat_eager, 50)),
                           "eager_p99": float(np.percentile(lat_eager, 99)),
                           "graph_p50": float(np.percentile(lat_graph, 50)),
                           "graph_p99": float(np.percentile(lat_graph, 99))},
            "throughput_msgs_per_s": {k: per_step / (v * 1e-3) for k, v in forms.items()},
            "roofline": roof, "cpu_baseline": cpu}


if __name__ == "__main__":
    main()
