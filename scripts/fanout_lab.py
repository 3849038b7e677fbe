"""Config 4's fan-out route kernel alone, with and without the stage-4 histogram (ORL_OPT_NO_BUCKETS), for a kernel trace.

Lab script, not a test: python scripts/fanout_lab.py [reps]   (run under rocprofv3 --kernel-trace --stats)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from orleans_amd import _lib as L  # noqa: E402
from orleans_amd import workloads as W  # noqa: E402
from orleans_amd.engine import GrainDirectoryEngine, grain_keys_from_longs  # noqa: E402


def main(reps=10):
    import os
    if os.environ.get("LAB_LIB"):  # A/B: an experimental build of the library (make lab)
        L.LIB_PATH = os.path.abspath(os.environ["LAB_LIB"])
    n_acc, n_pub = 10_000_000, 1_000_000
    cl = W.default_cluster()
    csr_off, csr_tgt = W.powerlaw_csr(n_acc)
    keys = grain_keys_from_longs(cl.type_code, np.arange(n_acc, dtype=np.int64))
    owner = cl.owner_of(W.jenkins3_np(keys["tcd"], keys["n0"], keys["n1"]))
    pubs = (W.stream(W.SEED_C4 ^ 0xB0B, 0, n_pub) % np.uint64(n_acc)).astype(np.uint32)
    total = int(np.diff(csr_off.astype(np.int64))[pubs].sum())
    eng = GrainDirectoryEngine(n_act=n_acc, dir_capacity=n_acc, max_batch=total + 1, device=0)
    W.setup_engine(eng, cl)
    W.register_population(eng, keys, owner, np.ones(n_acc, bool))
    dv = "cuda"
    d_off = torch.from_numpy(csr_off.view(np.int64)).to(dv)
    d_tgt = torch.from_numpy(csr_tgt.view(np.int32)).to(dv)
    d_pubs = torch.from_numpy(pubs.view(np.int32)).to(dv)
    d_ps = torch.from_numpy(owner[pubs]).to(dv)
    poff = torch.empty(n_pub + 1, dtype=torch.int64, device=dv)
    route, act, order = (torch.empty(total, dtype=torch.int32, device=dv) for _ in range(3))
    offs = torch.empty(n_acc + 2, dtype=torch.int32, device=dv)
    tcd = (3 << 56) + (cl.type_code & 0x00FFFFFFFFFFFFFF)
    st = torch.cuda.current_stream().cuda_stream
    for name, opts in (("buckets", 0), ("no buckets", L.OPT_NO_BUCKETS)):
        for _ in range(reps):
            eng.fanout_device(d_off, d_tgt, d_pubs, d_ps, n_pub, tcd, poff, route, act, order, offs, stream=st, opts=opts,
                              total=total)
        torch.cuda.synchronize()
        print(f"{name}: {reps} calls, {total} emitted messages each", flush=True)
    # the two-kernel form for comparison: expand to 32-B headers (k_fanout_expand), then the stream route kernel over them
    hdr = torch.empty((total, 8), dtype=torch.int32, device=dv)
    for _ in range(reps):
        eng.fanout_expand_device(d_off, d_tgt, None, tcd, d_pubs, d_ps, n_pub, poff, hdr, total, stream=st, total=total)
        eng.address_messages_device(hdr, total, route, act, order, offs, stream=st)
    torch.cuda.synchronize()
    print(f"expand + route: {reps} calls", flush=True)
    eng.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
