"""orleans_amd — MI355X-native batched grain-message routing engine (the Orleans 1.1 routing hot path).

The product is ``liborleans_route.so`` (HIP kernels for gfx950 + C++ host, C ABI in
``include/orleans_route.h``); this package is its host-side mirror of the reference interfaces
(``engine``), synthetic workloads (``workloads``) and the multi-GPU exchange driver (``node``).
"""
from . import _lib
from .engine import (GrainDirectoryEngine, RouteResult, calc_id_hash, decode_route, grain_keys_from_guid_bytes,
                     grain_keys_from_longs, jenkins_bytes, keyext_uniform_hash, raise_for_status,
                     silo_consistent_hash, type_code_data)

__all__ = ["GrainDirectoryEngine", "RouteResult", "calc_id_hash", "decode_route", "grain_keys_from_guid_bytes",
           "grain_keys_from_longs", "jenkins_bytes", "keyext_uniform_hash", "raise_for_status",
           "silo_consistent_hash", "type_code_data", "_lib"]
