"""Diagnostic: bench.owner_rank_counts (library partition counts) vs the workload's owner table, config-3 workload,
8 ranks' worth of 1M-message batches on one GPU."""
import importlib.util
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
from orleans_amd import workloads as W  # noqa: E402
from orleans_amd.node import local_silos, rank_of_silo  # noqa: E402

R, n_grains, n = 8, 16_000_000, 1 << 20
cl = W.balanced_cluster()
ros = rank_of_silo(cl.n_silos, R)
keys, uni, owner, reg = W.grain_population(cl, n_grains, 1.0)
ztab = W.zipf_tables(torch, n_grains, W.SEED_C3)
d_owner = torch.as_tensor(owner.astype(np.int64), device="cuda")
d_ros = torch.as_tensor(np.asarray(ros, np.int64), device="cuda")
for r in range(2):
    m = W.device_messages(torch, cl, n_grains, n, W.SEED_C3, start=r * n, sender_silos=local_silos(cl.n_silos, R, r), zipf=ztab)
    lib = bench.owner_rank_counts(torch, cl, m, n, ros, R).cpu().numpy()
    n1 = m.view(torch.int64).view(-1, 4)[:, 2]
    ref = torch.bincount(d_ros[d_owner[n1]], minlength=R).cpu().numpy()
    print("rank", r, "lib", lib.tolist(), "owner-table", ref.tolist(), flush=True)
    for piece in (1 << 18, 1 << 22):
        print("  piece", piece, bench.owner_rank_counts(torch, cl, m, n, ros, R, piece=piece).cpu().numpy().tolist(), flush=True)
