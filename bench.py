#!/usr/bin/env python3
"""bench.py — routed grain messages/sec on MI355X (BASELINE.json metric), one process per GPU.

Workload (BASELINE.json configs[1]): 8 logical silos 10.0.0.{1..8}:11111 gen 1,
1M ChirperAccount long-key grains all registered (activation on the directory owner), 64M single-target
messages per GPU per step, targets Uniform[0,1M) (splitmix64 seed 0x5EED0002), resident in HBM before the
timed region.  A step = one pass of the hot path over the batch: stages 1-4 (hash, ring owner, directory
probe + placement, stable per-activation bucketing).  With N GPUs (torchrun), each GPU hosts silos
s*N//8 == rank, holds their directory partition, originates 64M messages from its own silos (weak
scaling) and the step adds the owner partition + RCCL all-to-all exchange.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
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

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
ROUTE_KERNEL_BYTES_PER_MSG = 72  # 32 B header + 32 B directory slot + 4 B route word + 4 B activation handle
PIPELINE_BYTES_PER_MSG = 76      # + 4 B stable position


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--grains", type=int, default=1_000_000)
    ap.add_argument("--msgs", type=int, default=64 * 1024 * 1024, help="messages per GPU per step")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-wall", type=float, default=1.5, help="target wall seconds of the CPU baseline sample")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "route_kernel_pmc.json"))
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from orleans_amd import _lib as L
    from orleans_amd import workloads as W
    from orleans_amd.engine import GrainDirectoryEngine
    from orleans_amd.node import HipExecutor, ShardedRouter, local_silos, rank_of_silo

    n_grains, n_msgs = args.grains, args.msgs
    cl = W.default_cluster()
    ros = rank_of_silo(cl.n_silos, world)
    mine = local_silos(cl.n_silos, world, rank)
    cap = n_msgs if world == 1 else int(n_msgs * 1.25)
    t_setup = time.perf_counter()
    eng = GrainDirectoryEngine(n_act=n_grains, dir_capacity=n_grains, max_batch=cap, device=local_rank)
    W.setup_engine(eng, cl, local_silos=mine if world > 1 else None)
    keys, uni, owner, reg = W.grain_population(cl, n_grains)
    local_mask = None
    if world > 1:
        local_mask = np.zeros(cl.n_silos, np.uint8)
        local_mask[mine] = 1
    n_reg = W.register_population(eng, keys, owner, reg, local_mask)
    log(f"rank {rank}/{world}: silos {list(mine)}, {n_reg} grains registered; generating {n_msgs} messages")
    msgs = W.uniform_messages(cl, n_grains, n_msgs, seed=W.SEED_C2, start=rank * n_msgs,
                              sender_silos=mine if world > 1 else None)
    d_msgs = torch.from_numpy(msgs.view(np.int32).reshape(-1, 8)).cuda()
    stream = torch.cuda.current_stream().cuda_stream

    if world == 1:
        route = torch.empty(n_msgs, dtype=torch.int32, device="cuda")
        act = torch.empty(n_msgs, dtype=torch.int32, device="cuda")
        order = torch.empty(n_msgs, dtype=torch.int32, device="cuda")
        offsets = torch.empty(n_grains + 2, dtype=torch.int32, device="cuda")

        def step():
            eng.address_messages_device(d_msgs, n_msgs, route, act, order, offsets, stream=stream)
            return n_msgs
    else:
        router = ShardedRouter(HipExecutor(eng, cap, torch), rank, world, ros, cap, torch)

        def step():
            return router.step(d_msgs, n_msgs).n_recv
    log(f"setup {time.perf_counter() - t_setup:.1f}s; warmup {args.warmup}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    eng.set_timing(True)
    recv_total = 0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        recv_total += step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    nb, route_ms, bucket_ms, total_ms = eng.timing_summary()
    ms_per_step = elapsed * 1e3 / args.steps
    value = world * n_msgs * args.steps / elapsed
    per_launch_msgs = recv_total / args.steps
    achieved = ROUTE_KERNEL_BYTES_PER_MSG * per_launch_msgs / (route_ms * 1e-3) / 1e9
    log(f"rank {rank}: {ms_per_step:.3f} ms/step; route kernel {route_ms:.3f} ms, bucketing {bucket_ms:.3f} ms, "
        f"call {total_ms:.3f} ms over {nb} batches")

    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("msgs_per_launch") == per_launch_msgs and world == 1:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(cl, keys, owner, msgs, n_grains, args.cpu_wall)

    if world > 1:
        dist.barrier()
    if rank == 0:
        line = {
            "metric": "routed grain messages/sec (node)",
            "value": value,
            "unit": "messages/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32/u64 integer",
            "data": "synthetic (seeded splitmix64; config 2 of BASELINE.json)",
            "config": {"workload": "config2: uniform 1M long-key grains, 64M single-target messages per GPU, "
                                   "8-silo ring, stages 1-4" + (", + owner partition + RCCL all-to-all" if world > 1 else ""),
                       "grains": n_grains, "messages_per_gpu": n_msgs, "silos": cl.n_silos,
                       "parallelism": f"directory sharded by ring range over {world} GPU(s)"},
            "roofline": {"bound": "hbm", "kernel": "k_route (stages 1-3)", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_msg": ROUTE_KERNEL_BYTES_PER_MSG, "msgs_per_launch": per_launch_msgs,
                         "avg_launch_ms": route_ms},
            "pipeline": {"bytes_per_msg": PIPELINE_BYTES_PER_MSG, "route_kernel_ms": route_ms,
                         "bucketing_ms": bucket_ms, "call_ms": total_ms,
                         "algorithmic_GBs": PIPELINE_BYTES_PER_MSG * value / world / 1e9,
                         "frac_of_hbm_peak": PIPELINE_BYTES_PER_MSG * value / world / 1e9 / HBM_PEAK_GBS},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()


def cpu_baseline(cl, keys, owner, msgs, n_grains, target_wall):
    """The oracle (C++ restatement of the reference per-message path) on the host cores, on a bounded
    sample of the same workload, as the reference's CPU path stand-in (.NET cannot run here)."""
    from oracle import cpu_ref

    threads = max(1, min(16, os.cpu_count() or 1))
    o = cpu_ref.Oracle(cl.n_silos)
    for s in range(cl.n_silos):
        o.add_server(s, int(cl.hashes[s]))
    o.register(keys, np.arange(n_grains, dtype=np.uint32), owner)
    probe = msgs[: 1 << 20]
    t0 = time.perf_counter()
    o.route_bucket_mt(probe, n_grains, threads)
    t_probe = time.perf_counter() - t0
    n = int(min(len(msgs), max(len(probe), len(probe) * target_wall / max(t_probe, 1e-6))))
    sample = msgs[:n]
    t0 = time.perf_counter()
    o.route_bucket_mt(sample, n_grains, threads)
    wall = time.perf_counter() - t0
    log(f"cpu baseline: {n} messages in {wall:.2f}s on {threads} threads")
    return {"value": n / wall, "unit": "messages/s", "cores": threads, "kind": "port",
            "sample": f"first {n} of the {len(msgs)} config-2 messages (same directory, stages 1-4), "
                      f"oracle/cpu_ref.cpp ref_route_bucket_mt, {wall:.2f}s wall"}


if __name__ == "__main__":
    main()
