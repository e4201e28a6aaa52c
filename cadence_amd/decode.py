"""Persisted history blobs -> HistoryBatch, through the native decoder (libcadence_host.so).

Binds ``include/cadence_decode.h``: the thriftrw ``shared.History`` blobs that Cadence persists per
batch (``common/persistence/serializer.go:109-119``) are decoded in C++ straight into the engine's
SoA columns, skipping the ``[]*HistoryEvent`` object graph.  The result is the
canonical batch ``flatten()`` would build from the same events; ``interleave()`` it for the device.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
from typing import Iterable, List, Optional, Sequence

import numpy as np

from . import abi
from .flatten import HistoryBatch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CRR_HOST_LIB_PATH") or os.path.join(_HERE, "libcadence_host.so")
_lib = None

ERRORS = {-1: "bad argument", -2: "bad preamble (not a version-0 thriftrw blob)", -3: "truncated blob",
          -4: "unexpected thrift type", -5: "json.Unmarshal error", -6: "unknown encoding type"}


class DeserializationError(RuntimeError):
    """CadenceDeserializationError (common/persistence/serializer.go:320-333)."""

    def __init__(self, code: int, blob: int):
        super().__init__(f"DeserializeBatchEvents: {ERRORS.get(code, code)} (blob {blob})")
        self.code = code
        self.blob = blob


class CWfSource(ctypes.Structure):
    _fields_ = [("blob_begin", ctypes.c_uint32), ("blob_count", ctypes.c_uint32),
                ("init_version", ctypes.c_int64), ("now_ns", ctypes.c_int64),
                ("run_id", ctypes.c_char_p), ("branch_id", ctypes.c_char_p),
                ("final_token", ctypes.c_void_p), ("final_token_len", ctypes.c_uint32),
                ("new_run_wf", ctypes.c_int32),
                ("rebuild_last_event_id", ctypes.c_int64), ("rebuild_last_event_version", ctypes.c_int64),
                ("flags", ctypes.c_int32), ("retention_days", ctypes.c_int32)]


class CDecodedView(ctypes.Structure):
    _fields_ = [("ev", abi.CEvents), ("n_events", ctypes.c_uint64),
                ("act_side", ctypes.c_void_p), ("n_act_side", ctypes.c_uint64),
                ("start_side", ctypes.c_void_p), ("n_start_side", ctypes.c_uint64),
                ("reset_keys", ctypes.c_void_p), ("n_reset_keys", ctypes.c_uint64),
                ("arena", ctypes.c_void_p), ("n_arena", ctypes.c_uint64),
                ("wf", ctypes.c_void_p), ("n_wf", ctypes.c_uint32),
                ("table_rows", ctypes.c_uint64 * 8),
                ("key_off", ctypes.c_void_p), ("key_len", ctypes.c_void_p),
                ("key_arena", ctypes.c_void_p), ("n_key_arena", ctypes.c_uint64)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.crr_decode_histories.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.c_uint32, vp, ctypes.c_uint32,
                                           ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int64)]
        L.crr_decode_histories.restype = vp
        L.crr_decode_histories_enc.argtypes = [vp, vp, vp, ctypes.c_uint32, vp, ctypes.c_uint32, vp, ctypes.c_uint32,
                                               ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int64)]
        L.crr_decode_histories_enc.restype = vp
        L.crr_decoded_get_view.argtypes = [vp, ctypes.POINTER(CDecodedView)]
        L.crr_decoded_get_view.restype = ctypes.c_int
        L.crr_decoded_free.argtypes = [vp]
        L.crr_decoded_free.restype = None
        L.crr_synth_histories.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.crr_synth_histories.restype = vp
        _lib = L
    return _lib


@dataclasses.dataclass
class WorkflowSource:
    """One workflow's persisted batches (blobs) plus its host-injected inputs."""
    blobs: List[bytes]
    run_id: str = "run-id"
    branch_id: str = "branch-id"
    domain_failover_version: int = 0
    now_ns: int = 0
    final_token: Optional[bytes] = None
    rebuild_last_event_id: int = 0
    rebuild_last_event_version: int = 0
    new_run: Optional[int] = None        # workflow index of the CAN new-run history
    is_new_run: bool = False
    refresh_tasks: bool = False          # Rebuild's RefreshTasks after the replay
    retention_days: int = 1
    encodings: Optional[List[str]] = None   # per blob: "thriftrw" (default), "json", "" (empty), "unknown"


def _copy(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype)
    nbytes = int(n) * np.dtype(dtype).itemsize
    return np.frombuffer(ctypes.string_at(ptr, nbytes), dtype=dtype).copy()


def decode_histories(sources: Sequence[WorkflowSource], known_domains: Optional[Iterable[str]] = None,
                     n_threads: int = 0) -> HistoryBatch:
    """Decode every workflow's blobs into one canonical HistoryBatch (raises DeserializationError)."""
    L = lib()
    args = _prepare(sources, known_domains)
    return batch_from_handle(L, _decode_call(L, args, n_threads))


def time_native_decode(sources: Sequence[WorkflowSource], known_domains: Optional[Iterable[str]] = None,
                       n_threads: int = 0, min_seconds: float = 1.0) -> dict:
    """Wall time of crr_decode_histories alone (blobs already in native buffers, the Python argument
    marshalling excluded), repeated for at least ``min_seconds``: the host-ingest decode rate."""
    import time
    L = lib()
    args = _prepare(sources, known_domains)
    n_ev, reps, dt = 0, 0, 0.0
    while reps == 0 or dt < min_seconds:
        t0 = time.perf_counter()
        h = _decode_call(L, args, n_threads)
        dt += time.perf_counter() - t0
        if reps == 0:
            v = CDecodedView()
            L.crr_decoded_get_view(h, ctypes.byref(v))
            n_ev = int(v.n_events)
        L.crr_decoded_free(h)
        reps += 1
    blob_bytes = int(sum(args[1][i] for i in range(args[3])))
    return {"events": n_ev, "workflows": len(sources), "blob_bytes": blob_bytes, "reps": reps,
            "seconds_per_pass": dt / reps, "events_per_s": n_ev * reps / dt, "MB_per_s": blob_bytes * reps / dt / 1e6}


def _decode_call(L, args, n_threads: int):
    bptr, blen, benc, nb, cw, n_src, kd, nk, _keep = args
    err = ctypes.c_int(0)
    err_blob = ctypes.c_int64(-1)
    h = L.crr_decode_histories_enc(bptr, blen, benc, nb, cw, n_src, kd, nk, int(n_threads), ctypes.byref(err),
                                   ctypes.byref(err_blob))
    if not h:
        raise DeserializationError(err.value, err_blob.value)
    return h


# common.EncodingType (common/constants.go:60-67) -> CRR_ENCODING_*; EncodingTypeUnknown is the literal
# "unknow", so a blob tagged "unknown" is an unknown encoding (NewUnknownEncodingTypeError), not json
ENCODINGS = {"thriftrw": 0, "json": 1, "unknow": 2, "": 3}


def _prepare(sources: Sequence[WorkflowSource], known_domains: Optional[Iterable[str]]):
    blobs: List[bytes] = []
    encs: List[int] = []
    cw = (CWfSource * max(len(sources), 1))()
    keep = []
    for w, s in enumerate(sources):
        c = cw[w]
        c.blob_begin = len(blobs)
        c.blob_count = len(s.blobs)
        blobs.extend(s.blobs)
        for i in range(len(s.blobs)):
            e = "thriftrw" if s.encodings is None else s.encodings[i]
            encs.append(ENCODINGS.get(e, 0xFF))
        c.init_version = s.domain_failover_version
        c.now_ns = s.now_ns
        c.run_id = s.run_id.encode()
        c.branch_id = s.branch_id.encode()
        keep += [c.run_id, c.branch_id]
        if s.final_token is not None:
            buf = ctypes.create_string_buffer(s.final_token, len(s.final_token))
            keep.append(buf)
            c.final_token = ctypes.cast(buf, ctypes.c_void_p)
            c.final_token_len = len(s.final_token)
        c.new_run_wf = -1 if s.new_run is None else int(s.new_run)
        c.rebuild_last_event_id = s.rebuild_last_event_id
        c.rebuild_last_event_version = s.rebuild_last_event_version
        c.retention_days = s.retention_days
        c.flags = (abi.WF_FLAG_NEW_RUN if s.is_new_run else 0) | (abi.WF_FLAG_REFRESH_TASKS if s.refresh_tasks else 0)
    nb = len(blobs)
    bptr = (ctypes.c_void_p * max(nb, 1))()
    blen = (ctypes.c_uint64 * max(nb, 1))()
    bufs = []
    for i, b in enumerate(blobs):
        buf = ctypes.create_string_buffer(b, max(len(b), 1))
        bufs.append(buf)
        bptr[i] = ctypes.cast(buf, ctypes.c_void_p)
        blen[i] = len(b)
    if known_domains is None:
        kd, nk = None, 0xFFFFFFFF
    else:
        names = [n.encode() for n in known_domains]
        kd = (ctypes.c_char_p * max(len(names), 1))(*names)
        nk = len(names)
    benc = (ctypes.c_uint32 * max(nb, 1))(*encs) if encs else (ctypes.c_uint32 * 1)()
    return bptr, blen, benc, nb, cw, len(sources), kd, nk, (keep, bufs)


def batch_from_handle(L, h) -> HistoryBatch:
    """Copy a crr_decoded result into a canonical HistoryBatch and free it."""
    try:
        v = CDecodedView()
        L.crr_decoded_get_view(h, ctypes.byref(v))
        n = int(v.n_events)
        cols = {name: _copy(getattr(v.ev, name), n, t) for name, t in abi.EVENT_COLUMNS}
        act = _copy(v.act_side, v.n_act_side, abi.ACTIVITY_SIDE)
        start = _copy(v.start_side, v.n_start_side, abi.START_SIDE)
        rk = _copy(v.reset_keys, v.n_reset_keys, np.uint32)
        arena = _copy(v.arena, v.n_arena, np.uint8)
        wf = _copy(v.wf, v.n_wf, abi.WORKFLOW)
        batch = HistoryBatch(
            cols=cols,
            act_side=act if act.size else np.zeros(1, abi.ACTIVITY_SIDE),
            start_side=start if start.size else np.zeros(1, abi.START_SIDE),
            reset_keys=rk if rk.size else np.zeros(1, np.uint32),
            arena=arena if arena.size else np.zeros(1, np.uint8),
            wf=wf, stride=1,
            key_off=_copy(v.key_off, n, np.uint32), key_len=_copy(v.key_len, n, np.uint32),
            key_arena=_copy(v.key_arena, v.n_key_arena, np.uint8) if v.n_key_arena else np.zeros(1, np.uint8))
        for j, (name, *_rest) in enumerate(abi.TABLES):
            batch.table_rows[name] = int(v.table_rows[j])
        return batch
    finally:
        L.crr_decoded_free(h)
