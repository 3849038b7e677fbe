"""Config 2's (LAB_C3=1: config 3's) route kernel with and without the stage-4 digit histogram (ORL_OPT_NO_BUCKETS),
for a kernel trace.

Lab script, not a test: python scripts/route_lab.py [reps]   (run under rocprofv3 --kernel-trace --stats)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from orleans_amd import _lib as L  # noqa: E402
from orleans_amd import workloads as W  # noqa: E402
from orleans_amd.engine import GrainDirectoryEngine  # noqa: E402


def main(reps=10):
    if os.environ.get("LAB_LIB"):  # A/B: an experimental build of the library (make lab)
        L.LIB_PATH = os.path.abspath(os.environ["LAB_LIB"])
    c3 = os.environ.get("LAB_C3") == "1"  # config 3's one-GPU batch: 256M messages, Zipf(1.1) over 16M grains
    n_grains, n = (16_000_000, 256 << 20) if c3 else (1_000_000, 64 << 20)
    cl = W.balanced_cluster()
    keys, uni, owner, reg = W.grain_population(cl, n_grains, 1.0)
    eng = GrainDirectoryEngine(n_act=n_grains, dir_capacity=n_grains, max_batch=n, device=0)
    W.setup_engine(eng, cl)
    W.register_population(eng, keys, owner, reg)
    ztab = W.zipf_tables(torch, n_grains, W.SEED_C3) if c3 else None
    d_msgs = W.device_messages(torch, cl, n_grains, n, W.SEED_C3 if c3 else W.SEED_C2, zipf=ztab)
    del ztab
    route, act, order = (torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(3))
    offs = torch.empty(n_grains + 2, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for name, opts in (("buckets", 0), ("no buckets", L.OPT_NO_BUCKETS)):
        for _ in range(reps):
            eng.address_messages_device(d_msgs, n, route, act, order, offs, stream=st, opts=opts)
        torch.cuda.synchronize()
        print(f"{name}: {reps} calls of {n} messages", flush=True)
    eng.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
