"""Does routing batch i+1 overlap usefully with stage 4 of batch i?  Config 2 (1M grains, 64M messages), one GPU.

Leg A: one context, K back-to-back batches on one stream (what bench.py times).
Leg B: two contexts with the same directory, batches alternating between two streams, so one context's route
kernel (bound by random-probe fills) can run beside the other's stage 4 (bound by streaming bandwidth).
Prints ms per batch for both legs.  Lab script, not part of the product or the tests.
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from orleans_amd import workloads as W  # noqa: E402
from orleans_amd.engine import GrainDirectoryEngine  # noqa: E402


def main(k=20):
    n_grains, n_msgs = 1_000_000, 64 << 20
    cl = W.balanced_cluster()
    keys, uni, owner, reg = W.grain_population(cl, n_grains)
    d_msgs = W.device_messages(torch, cl, n_grains, n_msgs, W.SEED_C2)
    engs, outs, streams = [], [], []
    for _ in range(2):
        e = GrainDirectoryEngine(n_act=n_grains, dir_capacity=n_grains, max_batch=n_msgs, device=0)
        W.setup_engine(e, cl)
        W.register_population(e, keys, owner, reg, None)
        engs.append(e)
        outs.append([torch.empty(n_msgs, dtype=torch.int32, device="cuda") for _ in range(3)] +
                    [torch.empty(n_grains + 2, dtype=torch.int32, device="cuda")])
        streams.append(torch.cuda.Stream())

    def run(nctx):
        for i in range(k):
            j = i % nctx
            r, a, o, f = outs[j]
            engs[j].address_messages_device(d_msgs, n_msgs, r, a, o, f, stream=streams[j].cuda_stream)

    for nctx in (1, 2, 1, 2):
        run(nctx)
        torch.cuda.synchronize()
        t = time.perf_counter()
        run(nctx)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / k
        print(f"contexts={nctx}: {dt * 1e3:.3f} ms per 64M-message batch = {n_msgs / dt / 1e9:.2f} G msgs/s", flush=True)
    if not torch.equal(outs[0][2], outs[1][2]) or not torch.equal(outs[0][3], outs[1][3]):
        print("MISMATCH between contexts")
        sys.exit(1)
    for e in engs:
        e.close()


if __name__ == "__main__":
    main()
