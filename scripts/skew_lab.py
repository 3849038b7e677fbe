#!/usr/bin/env python3
"""Stage 4 alone (orl_bucket_device) on alternating unskewed / skewed 64M-message batches.

Until round 4 the level-2 launch form followed a host hint from the previous plan: a uniform batch followed by a Zipf-hot
one had its hot bucket counted by ONE workgroup.  Since round 5 that stale case takes the fused kernel's chunked
look-back form (same launch).  This lab times each batch of a sequence of uniform, Zipf and one-key-heavy batches with HIP
events on the submission stream (no sync between batches), so the stale-hint batches show their cost next to the steady
ones.  Run it once per ORL_SEG_FUSED setting (0: the round-3 count + scan launches for every plan):

    python scripts/skew_lab.py [n_act] [n_msgs] [reps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch as t
    from orleans_amd import workloads as W
    from orleans_amd.engine import GrainDirectoryEngine
    n_act = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 64 << 20
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    eng = GrainDirectoryEngine(n_act=n_act, dir_capacity=1024, max_batch=n, device=0)
    W.setup_engine(eng, W.default_cluster())
    g = t.Generator(device="cuda")
    g.manual_seed(5)
    uni = t.randint(0, n_act, (n,), device="cuda", dtype=t.int64, generator=g).to(t.int32)
    # Zipf(1.1) ranks by inverse CDF over a 2^20-point table, scattered by a multiplicative hash
    ranks = t.arange(1, n_act + 1, device="cuda", dtype=t.float64)
    cdf = t.cumsum(ranks.pow(-1.1), 0)
    cdf /= cdf[-1].clone()
    u = t.rand(n, device="cuda", dtype=t.float64, generator=g)
    r = t.searchsorted(cdf, u).clamp_(max=n_act - 1)
    zipf = ((r * 2654435761) % n_act).to(t.int32)
    hot = uni.clone()
    hot[: n // 2] = 12345 % n_act  # one activation holds half the batch (the hot-key path picks it after this batch)
    del ranks, cdf, u, r
    order = t.empty(n, dtype=t.int32, device="cuda")
    off = t.empty(n_act + 2, dtype=t.int32, device="cuda")
    s = t.cuda.Stream()
    # the hint each batch sees is the previous plan's: uniform -> zipf is the stale case (the look-back form), zipf ->
    # zipf the steady skewed one (count + chunked scan + carry), zipf -> uniform the stale case the other way
    seq = [("uniform", uni), ("zipf stale", zipf), ("zipf", zipf), ("uniform stale", uni), ("uniform", uni),
           ("half-one-key stale", hot), ("half-one-key", hot), ("uniform stale", uni)]
    times = {}
    with t.cuda.stream(s):
        for _ in range(2):  # warm-up
            for _, a in seq:
                eng.bucket_device(a, n, order, off, stream=s.cuda_stream)
        s.synchronize()
        for _ in range(reps):
            evs = []
            for name, a in seq:
                e0, e1 = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
                e0.record(s)
                eng.bucket_device(a, n, order, off, stream=s.cuda_stream)
                e1.record(s)
                evs.append((name, e0, e1))
            s.synchronize()
            for i, (name, e0, e1) in enumerate(evs):
                times.setdefault(f"{i}:{name}", []).append(e0.elapsed_time(e1))
    mode = "fused (device-decided skew form)" if os.environ.get("ORL_SEG_FUSED", "1") != "0" else "legacy (count + scan + carry)"
    print(f"stage 4 alone, n_act {n_act}, {n} messages per batch, {mode}; median of {reps} sequences, ms per batch:")
    for k, v in times.items():
        print(f"  {k:>22}: {np.median(v):.3f}  (min {np.min(v):.3f})")
    eng.close()


if __name__ == "__main__":
    main()
