"""The device-side (torch) message generators are bit-identical to the numpy generators the parity tests use."""
import numpy as np

from orleans_amd import _lib as L
from orleans_amd import workloads as W


def test_device_generators_match_numpy():
    import torch
    cl = W.default_cluster()
    n_grains, n = 200_000, 120_001
    m = W.uniform_messages(cl, n_grains, n, seed=W.SEED_C2, start=777)
    d = W.device_messages(torch, cl, n_grains, n, W.SEED_C2, start=777, device="cpu", chunk=50_000)
    np.testing.assert_array_equal(d.numpy().reshape(-1).view(L.MSG_DTYPE), m)
    m = W.zipf_messages(cl, n_grains, n, seed=W.SEED_C3, start=12345, sender_silos=np.array([2, 5, 7], np.uint8))
    z = W.zipf_tables(torch, n_grains, device="cpu")
    d = W.device_messages(torch, cl, n_grains, n, W.SEED_C3, start=12345, sender_silos=[2, 5, 7], zipf=z, device="cpu",
                          chunk=50_000)
    np.testing.assert_array_equal(d.numpy().reshape(-1).view(L.MSG_DTYPE), m)
