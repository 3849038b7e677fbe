"""Stream / reminder rings: the library's host-side VirtualBucketsRingProvider state against
the oracle restatement (oracle/pyref.py), including the reference's collision and removal quirks.  The device
lookups are checked in tests/test_gpu_parity.py."""
import numpy as np

from oracle import pyref as P
from orleans_amd.engine import GrainDirectoryEngine


def _ip(i):
    return bytes(12) + bytes([10, 0, i // 256, i % 256])


def _same(eng, vr):
    hs, ss = eng.vring()
    ref = vr.sorted_list()
    assert len(hs) == len(ref)
    assert [(int(h), int(s)) for h, s in zip(hs, ss)] == ref


def test_vring_add_remove_matches_oracle():
    eng = GrainDirectoryEngine(n_act=4, dir_capacity=16, max_batch=1024, device=-1)
    eng.set_silos(40)
    vr = P.VirtualBucketsRing()
    for s in range(40):
        eng.vring_add_server(s, _ip(s + 1), 11111 + s % 2, 100 + s % 7)
        vr.add_server(s, _ip(s + 1), 11111 + s % 2, 100 + s % 7)
    _same(eng, vr)
    for s in (3, 17, 3, 39):  # removing twice is a no-op the second time
        eng.vring_remove_server(s)
        vr.remove_server(s)
        _same(eng, vr)
    eng.close()


def test_vring_collisions_generation_and_removal_quirk():
    """Bucket collisions are forced with two silo indices of the same endpoint and generation (identical hashes):
    the later AddServer takes them (an equal generation is not greater).  Removing the silo that owns nothing is
    a no-op; removing the other drops every bucket of its hashes (VirtualBucketsRingProvider.cs:170-180)."""
    eng = GrainDirectoryEngine(n_act=4, dir_capacity=16, max_batch=1024, device=-1)
    eng.set_silos(4)
    vr = P.VirtualBucketsRing(buckets_per_silo=8)
    eng.vring_set_buckets(8)
    for s, ip, gen in ((0, _ip(1), 5), (1, _ip(1), 5), (2, _ip(2), 9), (3, _ip(3), 1)):
        eng.vring_add_server(s, ip, 11111, gen)
        vr.add_server(s, ip, 11111, gen)
    _same(eng, vr)
    hs, ss = eng.vring()
    assert 0 not in ss.tolist() and 1 in ss.tolist()  # silo 1 overwrote silo 0's identical buckets
    eng.vring_remove_server(0)  # owns no bucket: nothing happens
    vr.remove_server(0)
    _same(eng, vr)
    eng.vring_remove_server(1)
    vr.remove_server(1)
    _same(eng, vr)
    assert len(eng.vring()[0]) == 16
    eng.close()


def test_queue_hashes_and_consistent_long_compare():
    """HashRingBasedStreamQueueMapper queue positions, and ConsistentRingProvider's int-vs-uint long compare:
    a key above every non-negative silo hash wraps to the most negative one."""
    assert P.stream_queue_hashes(1) == [0]
    hs = P.stream_queue_hashes(8)
    assert hs[1] == (1 << 32) // 8 + 1 and hs == sorted(hs)
    ring = P.Ring()
    for s, h in enumerate((-2_000_000_000, -5, 7, 1_500_000_000)):
        ring.add_server(s, h)
    assert P.consistent_ring_target(ring, 8, 0, False) == 3
    assert P.consistent_ring_target(ring, 0xFFFFFFF0, 0, False) == 0  # wraps to [0] (hash -2e9)
    assert P.consistent_ring_target(ring, 0, 2, True) == 3           # 7 is me (excluded) → next
