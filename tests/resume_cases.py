"""Shared cases for ApplyEvents onto a loaded mutable state (CRR_WF_FLAG_RESUME).

The passive-replication path (ndc/history_replicator.go:385-460) loads a persisted state
(mutableStateBuilder.Load, mutable_state_builder.go:306-349) and applies one new batch to it
(state_builder.go:73-88, :90-648).  These helpers split each history at a batch boundary, replay
the prefix from scratch, turn its rows into loaded states and replay the rest onto them.
"""
from __future__ import annotations

import dataclasses
import random
from typing import List, Tuple

import numpy as np

from cadence_amd import abi
from cadence_amd.flatten import LoadedStates, flatten
from cadence_amd.history import WorkflowHistory

KNOWN = {"domain-a", "domain-b", "parent-domain"}


def split_histories(hs: List[WorkflowHistory], seed: int, last_only: bool = False
                    ) -> Tuple[List[WorkflowHistory], List[WorkflowHistory], np.ndarray]:
    """(prefixes, suffixes, split mask): workflow w is cut after a random batch (the last batch alone
    when ``last_only``: one passive-replication task); new-run histories and single-batch histories
    are not split (they appear whole in both parts and replay from scratch in each)."""
    rng = random.Random(seed)
    pre, suf, mask = [], [], []
    for h in hs:
        nb = len(h.batches)
        if h.is_new_run or nb < 2:
            pre.append(h)
            suf.append(h)
            mask.append(False)
            continue
        k = nb - 1 if last_only else rng.randint(1, nb - 1)
        pre.append(dataclasses.replace(h, batches=h.batches[:k], final_token=None, refresh_tasks=False))
        suf.append(dataclasses.replace(h, batches=h.batches[k:]))
        mask.append(True)
    return pre, suf, np.array(mask, bool)


def loaded_from(prefix_batch, prefix_res, split_mask) -> LoadedStates:
    """Loaded states of the split workflows whose prefix replayed OK (what Load would read back)."""
    ok = prefix_res.to_loaded(prefix_batch).mask
    return prefix_res.to_loaded(prefix_batch, mask=ok & split_mask)


def load_stable(loaded: LoadedStates) -> np.ndarray:
    """Workflows whose Load reproduces the in-memory state: every live activity's ActivityID maps to
    it (Load rebuilds pendingActivityIDToEventID from the infos, mutable_state_builder.go:311-314, so a
    mapping dropped by a duplicate-ID delete comes back after a reload)."""
    n = loaded.exec.shape[0]
    c = loaded.counts("act")
    rows = loaded.rows["act"]
    wf = np.repeat(np.arange(n), c)
    unmapped = (rows["flags"] & abi.ROW_MAPPED) == 0
    bad = np.zeros(n, bool)
    np.logical_or.at(bad, wf[unmapped], True)
    return loaded.mask & ~bad


def flatten_suffix(suffixes, loaded: LoadedStates, prefix_batch):
    return flatten(suffixes, known_domains=KNOWN, loaded=loaded, interners=loaded.interners)


def compare_split_with_one_shot(one_batch, one, pre_res, suf_batch, suf, stable: np.ndarray) -> int:
    """Resumed rows == one-shot rows for the load-stable workflows whose both parts replayed OK
    (inconsistency counts are per call: prefix + suffix).  Returns how many were compared."""
    from cadence_amd.result import _live_canonical, to_canonical_order
    e1 = to_canonical_order(one_batch, one)
    e2 = to_canonical_order(suf_batch, suf)
    ep = pre_res
    sel = stable & (e1["status"] == 0) & (e2["status"] == 0)
    for f in abi.EXEC_ROW.names:
        if f in ("reserved", "inconsistencies", "n_tasks"):
            continue
        bad = np.nonzero((e1[f] != e2[f]) & sel)[0]
        assert bad.size == 0, f"exec.{f}: wf {bad[:5]}: {e1[f][bad[:5]]} vs {e2[f][bad[:5]]}"
    assert ((e1["inconsistencies"] == ep["inconsistencies"] + e2["inconsistencies"]) | ~sel).all()
    l1 = _live_canonical(one_batch, one)
    l2 = _live_canonical(suf_batch, suf)
    for name, _dt, _b, _c, n_f in abi.TABLES:
        if name == "tasks":
            continue
        k1 = np.repeat(sel, np.maximum(e1[n_f], 0))
        k2 = np.repeat(sel, np.maximum(e2[n_f], 0))
        a, b = l1[name][k1], l2[name][k2]
        assert a.shape == b.shape, name
        for f in a.dtype.names:
            if f != "reserved":
                assert (a[f] == b[f]).all(), f"{name}.{f}"
    return int(sel.sum())
