"""Config 3's one-GPU batch (256M messages, Zipf(1.1) over 16M grains, 24-bit handles: the LSD stage-4 plan) in two
launch forms, for a kernel trace (run under rocprofv3 --kernel-trace --stats):
  bench  the bench step: orl_route_batch_device, stages 1-4 (k_route with the fused digit histogram, then stage 4)
  split  the same step as route without buckets (k_route<0>) + orl_bucket_device over the handles, so both route
         kernels run in the same position: right after a stage 4 that streamed GBs through the caches.
Lab script, not a test: python scripts/lsd_lab.py [reps] [forms]   (LAB_LIB=...: an experimental build)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orleans_amd import _lib as L  # noqa: E402
from orleans_amd import workloads as W  # noqa: E402
from orleans_amd.engine import GrainDirectoryEngine  # noqa: E402


def main(reps=10, forms=("bench", "split")):
    if os.environ.get("LAB_LIB"):
        L.LIB_PATH = os.path.abspath(os.environ["LAB_LIB"])
    n_grains, n = 16_000_000, 256 << 20
    cl = W.balanced_cluster()
    keys, uni, owner, reg = W.grain_population(cl, n_grains, 1.0)
    eng = GrainDirectoryEngine(n_act=n_grains, dir_capacity=n_grains, max_batch=n, device=0)
    W.setup_engine(eng, cl)
    W.register_population(eng, keys, owner, reg)
    ztab = W.zipf_tables(torch, n_grains, W.SEED_C3)
    d_msgs = W.device_messages(torch, cl, n_grains, n, W.SEED_C3, zipf=ztab)
    del ztab
    route, act, order = (torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(3))
    offs = torch.empty(n_grains + 2, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for form in forms:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for i in range(reps + 2):
            if i == 2:
                ev[0].record()
            if form == "bench":
                eng.address_messages_device(d_msgs, n, route, act, order, offs, stream=st)
            else:
                eng.address_messages_device(d_msgs, n, route, act, order, offs, stream=st, opts=L.OPT_NO_BUCKETS)
                eng.bucket_device(act, n, order, offs, stream=st)
        ev[1].record()
        torch.cuda.synchronize()
        print(f"{form}: {ev[0].elapsed_time(ev[1]) / reps:.3f} ms per step ({reps} steps of {n} messages)", flush=True)
    eng.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10,
         tuple(sys.argv[2].split(",")) if len(sys.argv) > 2 else ("bench", "split"))
