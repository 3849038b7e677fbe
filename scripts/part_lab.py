"""Hop-1 partition cost (k_part_lb) on one GPU: one rank's share of config 3 (256M / R messages), owner-partitioned
into R padded regions in `calls` launches, for 8-B / 16-B / 32-B records.  Prints ms per rank step per variant.
Lab script, not a test: python scripts/part_lab.py [R] [reps]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from orleans_amd import _lib as L  # noqa: E402
from orleans_amd import workloads as W  # noqa: E402
from orleans_amd.engine import GrainDirectoryEngine  # noqa: E402
from orleans_amd.node import local_silos, rank_of_silo  # noqa: E402


def timed(fn, reps):
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
    return float(np.median(ts)), float(min(ts))


def main(R=8, reps=7):
    import os
    if os.environ.get("LAB_LIB"):  # A/B: an experimental build of the library
        L.LIB_PATH = os.path.abspath(os.environ["LAB_LIB"])
    n_grains, n_total = 16_000_000, 256 << 20
    n_msgs = n_total // R
    cl = W.balanced_cluster()
    ros = rank_of_silo(cl.n_silos, R)
    ztab = W.zipf_tables(torch, n_grains, W.SEED_C3)
    part = GrainDirectoryEngine(n_act=1, dir_capacity=1, max_batch=n_msgs, device=0)
    W.setup_engine(part, cl)
    part.set_wire_types([W.grain_tcd(cl)])
    torch.cuda.set_stream(torch.cuda.Stream())
    st = torch.cuda.current_stream().cuda_stream
    m = W.device_messages(torch, cl, n_grains, n_msgs, W.SEED_C3, start=0, sender_silos=local_silos(cl.n_silos, R, 0),
                          zipf=ztab)
    cap = n_msgs
    d_out = torch.empty(R * cap * 32, dtype=torch.uint8, device="cuda")
    d_counts = torch.zeros(R, dtype=torch.int64, device="cuda")
    d_status = torch.zeros(1, dtype=torch.int32, device="cuda")
    fns = {8: part.partition_narrow_device, 16: part.partition_compact_device}
    for width in (8, 16):
        for calls in (1, 4):
            step = n_msgs // calls

            def run():
                for c in range(calls):
                    fns[width](m[c * step:], step, ros, R, 0, cap, d_out, d_counts, d_status, stream=st)
            med, mn = timed(run, reps)
            gbs = n_msgs * (32 + width) / (med * 1e-3) / 1e9
            print(f"width {width:2d} B, {calls} call(s) of {step >> 20}M: {med:.3f} ms (min {mn:.3f}); "
                  f"{gbs:.0f} GB/s of {32 + width} B/msg", flush=True)
    part.close()


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
