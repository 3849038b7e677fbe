"""Size-independent checks of routed output, run on the device (torch) after a benchmark's timed steps.

What must hold for every message of a batch whatever its size, so that the multi-GPU bench and the full-size GPU tests
can check every rank's hosted output at the sizes that actually run (32M-55M messages per rank, 256M per GPU), where a
CPU oracle replay of the whole batch is out of reach.  The callers add a bounded oracle sample on top (bench.py's checker
leg, tests/); nothing here is on the routing path, and nothing here computes a routing decision: the expectations come
from the workload's definition (which grain a message targets, which silo owns it, which handle its catalog gave it).

  stage 4 (ActivationData.EnqueueMessage, ActivationData.cs:483-514): `order` is a permutation of the hosted messages,
  grouped by activation (the unresolved bucket n_act last), arrival order inside every bucket, and bucket_offsets is the
  exclusive prefix of the per-activation counts;
  stages 1-3 (LocalGrainDirectory.CalculateTargetSilo :439-497, GrainDirectoryPartition.LookUpGrain :326-344): every route
  word names the grain's directory owner, and — when every grain is registered on its owner — the owner as host, status
  HIT and the handle the owner's catalog gave the grain.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from . import _lib as L

_M32 = 0xFFFFFFFF


def _bincount(t, x, n):
    """torch.bincount in slices of 2^25 elements (one call over 256M elements raised SIGFPE inside torch's histogram kernel
    on the GPU box: DESIGN.md §5)."""
    out = t.zeros(n, dtype=t.int64, device=x.device)
    for i in range(0, x.numel(), 1 << 25):
        out += t.bincount(x[i:i + (1 << 25)], minlength=n).to(t.int64)
    return out


def fetch_node_result(t, eng, res, n_act: int, stream=None) -> dict:
    """Device copies (int64, unsigned values) of a node result's hosted arrays before the node's next batch: route, act,
    order, offsets, and each hosted message's grain id N1 decoded from its exchange record (8-B orl_wire8, 16-B
    orl_wire_msg or 32-B orl_msg_hdr, include/orleans_route.h)."""
    dev = t.device("cuda", t.cuda.current_device())

    def grab(p, words):
        x = t.empty(words, dtype=t.int32, device=dev)
        if words:
            eng.copy_on_device(x, p, 4 * words, stream=stream)
        return x

    n = res.n_hosted
    t.cuda.synchronize()  # torch's pending work is done before its freed blocks are filled from another stream
    out = {"route": grab(res.route, n), "act": grab(res.act, n), "order": grab(res.order, n),
           "offsets": grab(res.offsets, n_act + 2)}
    raws = [(grab(p, cnt * w // 4), w) for p, cnt, w in res.segments]
    # the copies run on the library's stream (stream None / torch's default stream handle 0 = the context's own stream):
    # every torch op below runs on torch's stream, so wait for the copies before the first one reads them
    t.cuda.synchronize()
    parts = []
    for raw, w in raws:
        if w == 8:
            parts.append(raw.view(-1, 2)[:, 0].to(t.int64) & _M32)
        elif w == 16:
            parts.append(raw.view(t.int64).view(-1, 2)[:, 0])
        else:
            parts.append(raw.view(t.int64).view(-1, 4)[:, 2])
    out["n1"] = t.cat(parts) if parts else t.zeros(0, dtype=t.int64, device=dev)
    t.cuda.synchronize()
    for k in ("route", "act", "order", "offsets"):
        out[k] = out[k].to(t.int64) & _M32
    return out


def check_stage4(t, act, order, offsets, n_act: int) -> List[str]:
    """Stage-4 properties of one bucketing (int64 device tensors of unsigned values)."""
    errs = []
    n = act.numel()
    key = t.clamp(act, max=n_act)
    if order.numel() != n:
        return [f"order has {order.numel()} entries for {n} messages"]
    if n and not t.equal(t.sort(order).values, t.arange(n, device=act.device)):
        errs.append("order is not a permutation of the hosted messages")
        return errs
    ks = key[order]
    if n > 1:
        d = ks[1:] - ks[:-1]
        if bool((d < 0).any()):
            errs.append(f"order is not grouped by activation ({int((d < 0).sum())} descents)")
        same = d == 0
        if bool(((order[1:] - order[:-1])[same] <= 0).any()):
            errs.append("arrival order broken inside a bucket")
    cnt = _bincount(t, key, n_act + 1)
    exp = t.zeros(n_act + 2, dtype=t.int64, device=act.device)
    exp[1:] = t.cumsum(cnt, 0)
    if not t.equal(offsets, exp):
        bad = int((offsets != exp).sum())
        errs.append(f"bucket offsets differ from the count prefix at {bad} of {n_act + 2} entries")
    return errs


def check_routes(t, route, act, n1, owner_t, handle_t, all_registered: bool, owner_rank_t=None, rank: Optional[int] = None
                 ) -> List[str]:
    """Route words and handles of hosted messages vs the workload's grains: owner_t[g] = the directory owner silo of grain
    g, handle_t[g] = the handle its owner's catalog registered (int64 device tensors); owner_rank_t[s] = the rank hosting
    silo s (node runs: every hosted message must be owned on `rank`)."""
    errs = []
    if n1.numel() != route.numel():
        return [f"{n1.numel()} hosted records for {route.numel()} route words"]
    if not route.numel():
        return errs

    def where(bad):  # count, first and last hosted index of a failing property
        i = t.nonzero(bad).flatten()
        return f"{i.numel()} messages (hosted index {int(i[0])} .. {int(i[-1])})"

    if bool((n1 >= owner_t.numel()).any()):
        return [f"a hosted record names a grain outside the population: {where(n1 >= owner_t.numel())}"]
    own = owner_t[n1]
    if not t.equal(route & 0xFF, own):
        errs.append(f"owner silo differs from the grain's ring owner for {where((route & 0xFF) != own)}")
    if owner_rank_t is not None and bool((owner_rank_t[own] != rank).any()):
        errs.append("a hosted message is owned by another rank")
    if all_registered:
        if not t.equal((route >> 8) & 0xFF, own):
            errs.append("host silo differs from the owner (every activation lives on its owner)")
        if bool((((route >> 16) & 0xFF) != L.ST_HIT).any()):
            errs.append(f"{int((((route >> 16) & 0xFF) != L.ST_HIT).sum())} registered targets did not hit the directory")
        if not t.equal(act, handle_t[n1]):
            errs.append(f"activation handle differs from the registered one for {where(act != handle_t[n1])}")
    return errs


def local_handles(owner: np.ndarray, reg: np.ndarray, local_mask: Optional[np.ndarray]) -> np.ndarray:
    """The handle W.register_population(dense_local=True) gives each grain (-1: not registered on these silos)."""
    sel = reg.copy()
    if local_mask is not None:
        sel &= local_mask[owner].astype(bool)
    h = np.full(len(owner), -1, np.int64)
    idx = np.nonzero(sel)[0]
    h[idx] = np.arange(len(idx), dtype=np.int64)
    return h
