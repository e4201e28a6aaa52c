"""Replay outputs (host numpy images of ``crr_outputs``) and comparison helpers."""
from __future__ import annotations

import dataclasses
from typing import Dict

import numpy as np

from . import abi
from .flatten import HistoryBatch, LoadedStates, write_init


@dataclasses.dataclass
class ReplayResult:
    exec: np.ndarray                 # abi.EXEC_ROW [n_wf] in batch order
    tables: Dict[str, np.ndarray]    # name -> rows (slot-table layout of the batch)

    def live_rows(self, batch: HistoryBatch, w: int) -> Dict[str, np.ndarray]:
        r = batch.wf[w]
        out = {}
        for name, _dt, base_f, cap_f, n_f in abi.TABLES:
            n = min(int(self.exec[w][n_f]), int(r[cap_f]))
            idx = int(r[base_f]) + np.arange(n, dtype=np.int64) * int(batch.wf_strides()[w])
            out[name] = self.tables[name][idx]
        return out

    def to_loaded(self, batch: HistoryBatch, mask=None) -> LoadedStates:
        """The replayed states as loaded states for a following ApplyEvents call (canonical workflow
        order, as persisted and re-read by Load): the workflows in ``mask`` (default: status OK)."""
        ex = to_canonical_order(batch, self).copy()
        m = (ex["status"] == 0) if mask is None else np.asarray(mask, bool)
        live = _live_canonical(batch, self)
        rows = {}
        for name, _dt, _b, _c, n_f in abi.TABLES:
            if name == "tasks":
                continue
            c = np.maximum(ex[n_f].astype(np.int64), 0)
            keep = np.repeat(m, c)
            rows[name] = live[name][keep].copy()
        ex[~m] = np.zeros(1, abi.EXEC_ROW)
        ex["n_tasks"] = 0
        its = None
        if batch.interners is not None:
            its = batch.interners if batch.perm is None else [None] * batch.n_wf
            if batch.perm is not None:
                for p, c in enumerate(batch.perm):
                    its[c] = batch.interners[p]
        return LoadedStates(ex, rows, m, its)


def allocate_host(batch: HistoryBatch) -> ReplayResult:
    ex = np.zeros(max(batch.n_wf, 1), dtype=abi.EXEC_ROW)[:batch.n_wf]
    tables = {}
    for name, dt, *_ in abi.TABLES:
        rows = batch.table_rows.get(name, 0) if (name != "tasks" or batch.emit_tasks) else 0
        tables[name] = np.zeros(max(rows, 1), dtype=dt)
    write_init(batch, ex, tables)
    return ReplayResult(ex, tables)


def gather_live(batch: HistoryBatch, res: ReplayResult) -> Dict[str, np.ndarray]:
    """Concatenate every workflow's live rows in batch order (vectorised): name -> rows."""
    out = {}
    for name, _dt, base_f, cap_f, n_f in abi.TABLES:
        n = np.minimum(res.exec[n_f].astype(np.int64), batch.wf[cap_f].astype(np.int64))
        n = np.maximum(n, 0)
        tot = int(n.sum())
        if tot == 0:
            out[name] = res.tables[name][:0]
            continue
        wf_idx = np.repeat(np.arange(batch.n_wf), n)
        slot = np.arange(tot) - np.repeat(np.cumsum(n) - n, n)
        idx = batch.wf[base_f].astype(np.int64)[wf_idx] + slot * batch.wf_strides()[wf_idx]
        out[name] = res.tables[name][idx]
    return out


def to_canonical_order(batch: HistoryBatch, res: ReplayResult):
    """Exec rows reordered to canonical workflow order (for interleaved batches)."""
    if batch.perm is None:
        return res.exec
    ex = np.empty_like(res.exec)
    ex[batch.perm] = res.exec
    return ex


EXEC_COMPARE_FIELDS = [n for n in abi.EXEC_ROW.names if n != "reserved"]


def diff_results(batch_a: HistoryBatch, a: ReplayResult, batch_b: HistoryBatch, b: ReplayResult, limit=10):
    """Bit-exact comparison of two results over the same workflows (possibly different layouts).

    Returns a list of human-readable mismatch descriptions (empty == identical)."""
    msgs = []
    ea = to_canonical_order(batch_a, a)
    eb = to_canonical_order(batch_b, b)
    for f in EXEC_COMPARE_FIELDS:
        bad = np.nonzero(ea[f] != eb[f])[0]
        if bad.size:
            w = int(bad[0])
            msgs.append(f"exec.{f}: {bad.size} workflows differ, first wf {w}: {ea[f][w]} vs {eb[f][w]}")
            if len(msgs) >= limit:
                return msgs
    # live rows: gather per canonical workflow order
    la = _live_canonical(batch_a, a)
    lb = _live_canonical(batch_b, b)
    for name, *_ in abi.TABLES:
        ra, rb = la[name], lb[name]
        if ra.shape != rb.shape:
            msgs.append(f"{name}: row count {ra.shape[0]} vs {rb.shape[0]}")
            continue
        for f in ra.dtype.names:
            if f == "reserved":
                continue
            bad = np.nonzero(ra[f] != rb[f])[0]
            if bad.size:
                msgs.append(f"{name}.{f}: {bad.size} rows differ, first row {int(bad[0])}: "
                            f"{ra[f][bad[0]]} vs {rb[f][bad[0]]}")
                if len(msgs) >= limit:
                    return msgs
    return msgs


def _live_canonical(batch: HistoryBatch, res: ReplayResult):
    """Live rows concatenated in canonical workflow order."""
    if batch.perm is None:
        return gather_live(batch, res)
    # reorder workflows to canonical order, then gather
    order = np.argsort(batch.perm, kind="stable")       # canonical w -> device position
    out = {}
    for name, _dt, base_f, cap_f, n_f in abi.TABLES:
        n = np.minimum(res.exec[n_f].astype(np.int64), batch.wf[cap_f].astype(np.int64))[order]
        n = np.maximum(n, 0)
        tot = int(n.sum())
        if tot == 0:
            out[name] = res.tables[name][:0]
            continue
        wf_idx = np.repeat(order, n)
        slot = np.arange(tot) - np.repeat(np.cumsum(n) - n, n)
        idx = batch.wf[base_f].astype(np.int64)[wf_idx] + slot * batch.wf_strides()[wf_idx]
        out[name] = res.tables[name][idx]
    return out
