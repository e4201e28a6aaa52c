"""Narrow upload format for the event columns (``crr_widen_events``, include/cadence_replay.h).

Within one workflow consecutive events differ by little (IDs and TaskIDs step by one, versions move
at failovers, refs point a few events back, timestamps advance by ms..s), so each int64 column ships
as per-event deltas along the workflow's steps at the narrowest byte width that holds every delta of
the batch; the device rebuilds the exact columns in HBM.  For the config-2 workload that is 14 B per
event instead of 49 (PCIe, not HBM, bounds a replay from host buffers).
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Dict

import numpy as np

from . import abi
from .flatten import HistoryBatch

PLAIN, UNSIGNED, DELTA, ID_MINUS = 0, 1, 2, 3
COLUMNS = ["event_id", "version", "timestamp", "task_id", "ref", "key", "aux"]


class CPackedColumn(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("width", ctypes.c_uint32), ("kind", ctypes.c_uint32)]


class CPackedEvents(ctypes.Structure):
    _fields_ = [(c, CPackedColumn) for c in COLUMNS] + [("ts_base", ctypes.c_void_p)]


@dataclasses.dataclass
class PackedEvents:
    data: Dict[str, np.ndarray]        # column -> uint8 [n_slots * width]
    width: Dict[str, int]
    kind: Dict[str, int]
    ts_base: np.ndarray                # int64 [n_wf]

    @property
    def nbytes(self) -> int:
        return int(sum(a.nbytes for a in self.data.values()) + self.ts_base.nbytes)


def _signed_width(d: np.ndarray) -> int:
    if d.size == 0:
        return 1
    lo, hi = int(d.min()), int(d.max())
    for w in range(1, 8):
        if -(1 << (8 * w - 1)) <= lo and hi < (1 << (8 * w - 1)):
            return w
    return 8


def _unsigned_width(d: np.ndarray) -> int:
    hi = int(d.max()) if d.size else 0
    for w in range(1, 8):
        if hi < (1 << (8 * w)):
            return w
    return 8


def _bytes(v: np.ndarray, w: int, n_slots: int, slots: np.ndarray) -> np.ndarray:
    full = np.zeros(n_slots, np.uint64)
    full[slots] = v.astype(np.int64).view(np.uint64) if v.dtype != np.uint64 else v
    return np.ascontiguousarray(full.view(np.uint8).reshape(n_slots, 8)[:, :w]).reshape(-1)


def event_slots(batch: HistoryBatch):
    """(workflow, step, slot, previous slot) of every real event, in workflow-major order."""
    cnt = batch.wf["ev_count"].astype(np.int64)
    st = batch.wf_strides()
    wf_idx = np.repeat(np.arange(batch.n_wf), cnt)
    step = np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    slot = batch.wf["ev_begin"].astype(np.int64)[wf_idx] + step * st[wf_idx]
    return wf_idx, step, slot, slot - st[wf_idx]


def pack_events(batch: HistoryBatch) -> PackedEvents:
    n_slots = batch.n_slots
    wf_idx, step, slot, prev = event_slots(batch)
    first = step == 0
    u = {c: np.asarray(batch.cols[c]).astype(np.int64).view(np.uint64) for c in ("event_id", "version", "timestamp",
                                                                                    "task_id", "ref")}
    ts_base = np.zeros(batch.n_wf, np.int64)
    ts_base[wf_idx[first]] = batch.cols["timestamp"][slot[first]]
    data, width, kind = {}, {}, {}
    for c in ("event_id", "version", "timestamp", "task_id"):
        v = u[c][slot]
        base = np.where(first, ts_base.view(np.uint64)[wf_idx] if c == "timestamp" else np.uint64(0),
                        u[c][np.where(first, slot, prev)])
        d = (v - base).view(np.int64)
        width[c], kind[c] = _signed_width(d), DELTA
        data[c] = _bytes(d, width[c], n_slots, slot)
    ref = u["ref"][slot].view(np.int64)
    idm = (u["event_id"][slot] - u["ref"][slot]).view(np.int64)
    wr, wi = _signed_width(ref), _signed_width(idm)
    if wi < wr:
        width["ref"], kind["ref"], data["ref"] = wi, ID_MINUS, _bytes(idm, wi, n_slots, slot)
    else:
        width["ref"], kind["ref"], data["ref"] = wr, PLAIN, _bytes(ref, wr, n_slots, slot)
    key = np.asarray(batch.cols["key"])[slot].astype(np.uint64)
    width["key"], kind["key"] = _unsigned_width(key), UNSIGNED
    data["key"] = _bytes(key, width["key"], n_slots, slot)
    aux = np.asarray(batch.cols["aux"])[slot].astype(np.int64)
    width["aux"], kind["aux"] = _signed_width(aux), PLAIN
    data["aux"] = _bytes(aux, width["aux"], n_slots, slot)
    return PackedEvents(data, width, kind, ts_base)


def unpack_events(batch: HistoryBatch, pk: PackedEvents) -> Dict[str, np.ndarray]:
    """Host restatement of crr_widen_events (test reference): the wide columns (pads zero)."""
    n_slots = batch.n_slots
    wf_idx, step, slot, _prev = event_slots(batch)
    cnt = batch.wf["ev_count"].astype(np.int64)

    def raw(c):
        w = pk.width[c]
        b = np.zeros((n_slots, 8), np.uint8)
        b[:, :w] = pk.data[c].reshape(n_slots, w)
        v = b.reshape(-1).view(np.uint64)
        if pk.kind[c] != UNSIGNED and w < 8:
            sh = np.uint64(64 - 8 * w)
            v = ((v << sh).view(np.int64) >> sh.astype(np.int64)).view(np.uint64)
        return v[slot]

    out = {}
    starts = np.cumsum(cnt) - cnt
    for c in ("event_id", "version", "timestamp", "task_id"):
        r = raw(c).copy()
        if c == "timestamp":
            r[step == 0] += pk.ts_base.view(np.uint64)[wf_idx[step == 0]]
        s = np.cumsum(r, dtype=np.uint64)          # per-workflow prefix sums (uint64 wrap)
        seg0 = np.repeat(np.where(starts > 0, s[np.maximum(starts - 1, 0)], np.uint64(0)), cnt)
        out[c] = (s - seg0).view(np.int64)
    r = raw("ref")
    out["ref"] = ((out["event_id"].view(np.uint64) - r) if pk.kind["ref"] == ID_MINUS else r).view(np.int64)
    out["key"] = raw("key").astype(np.uint32)
    out["aux"] = raw("aux").view(np.int64).astype(np.int32)
    cols = {}
    for name, t in abi.EVENT_COLUMNS:
        if name == "etype":
            continue
        a = np.zeros(n_slots, t)
        a[slot] = out[name]
        cols[name] = a
    return cols
