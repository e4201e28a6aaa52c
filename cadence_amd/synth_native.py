"""Full-size synthetic workloads from the native generator (libcadence_host.so, synth_native.cpp).

The config-3/5 mixed random walks and the config-4 long-tail histories of ``synth_mixed`` (same event
graph and distributions, mirroring ``common/testing/history_event_util.go``), generated and flattened
in C++ on all host threads: 1.25M mixed workflows (~52M events, the per-GPU shard of config 3) take
seconds, where the Python generator takes tens of minutes.  Returns canonical HistoryBatches with
per-event key strings (so the oracle can replay them).
"""
from __future__ import annotations

import ctypes

from . import decode
from .flatten import HistoryBatch

SEED_C3 = 0xCAD00003
SEED_C4 = 0xCAD00004
LONG_TAIL_CAPS = (32, 16, 8, 4, 4)          # synth_mixed.LONG_TAIL_CAPS: act, timer, child, rc, sig


class CSynthParams(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("n", ctypes.c_uint32), ("seed", ctypes.c_uint64),
                ("mean_len", ctypes.c_int32), ("multi_version", ctypes.c_int32),
                ("invalid_rate", ctypes.c_double), ("can_rate", ctypes.c_double),
                ("unknown_domain_rate", ctypes.c_double),
                ("min_len", ctypes.c_int32), ("max_len", ctypes.c_int32), ("run_cap", ctypes.c_int32),
                ("caps", ctypes.c_int32 * 5), ("alpha", ctypes.c_double),
                ("num_shards", ctypes.c_uint32), ("world", ctypes.c_uint32), ("rank", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


def _run(p: CSynthParams, n_threads: int) -> HistoryBatch:
    L = decode.lib()
    err = ctypes.c_int(0)
    h = L.crr_synth_histories(ctypes.byref(p), int(n_threads), ctypes.byref(err))
    if not h:
        raise RuntimeError(f"crr_synth_histories failed: {err.value}")
    return decode.batch_from_handle(L, h)


def mixed(n: int, seed: int = SEED_C3, mean_len: int = 40, multi_version: bool = False, invalid_rate: float = 0.0,
          can_rate: float = 0.0, unknown_domain_rate: float = 0.0, n_threads: int = 0, shard=None) -> HistoryBatch:
    """n mixed random-walk workflows (configs 3 / 5); defaults: every history valid.  ``shard`` =
    (num_shards, world, rank): only this rank's shards of the n-workflow workload."""
    p = CSynthParams(kind=0, n=n, seed=seed, mean_len=mean_len, multi_version=int(multi_version),
                     invalid_rate=invalid_rate, can_rate=can_rate, unknown_domain_rate=unknown_domain_rate)
    _set_shard(p, shard)
    return _run(p, n_threads)


def _set_shard(p: CSynthParams, shard):
    if shard is not None:
        p.num_shards, p.world, p.rank = (int(x) for x in shard)


def shard_of(w, num_shards: int):
    """crr_synth_shard_of over an array of workflow indices (the generator's own function)."""
    import numpy as np
    L = decode.lib()
    f = L.crr_synth_shard_of
    f.restype = ctypes.c_uint32
    f.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
    return np.array([f(int(x), int(num_shards)) for x in np.asarray(w).ravel()], np.int64)


def long_tail(n: int, seed: int = SEED_C4, max_len: int = 50_000, run_cap: int = 10_000, min_len: int = 10,
              alpha: float = 1.2, multi_version: bool = False, invalid_rate: float = 0.0, caps=LONG_TAIL_CAPS,
              n_threads: int = 0, shard=None) -> HistoryBatch:
    """n logical long-tail workflows (config 4): Zipf lengths up to max_len, continue-as-new every run_cap.
    ``shard``: as in ``mixed`` (by logical workflow: its continue-as-new runs share its workflow ID)."""
    p = CSynthParams(kind=1, n=n, seed=seed, multi_version=int(multi_version), invalid_rate=invalid_rate,
                     min_len=min_len, max_len=max_len, run_cap=run_cap, alpha=alpha)
    _set_shard(p, shard)
    for i, c in enumerate(caps or (0, 0, 0, 0, 0)):
        p.caps[i] = c
    return _run(p, n_threads)
