"""Batched NDC branch decisions through ``crr_ndc_prepare``.

``branchManagerImpl.prepareVersionHistory`` (``service/history/ndc/branch_manager.go:87-149``) decides,
for every incoming replication batch, which local branch of the workflow's VersionHistories it extends
(the LCA search of ``versionHistory.go:501-528``), whether a new branch must be forked, and whether the
batch is a duplicate or arrived out of order.  Here a whole batch of tasks is decided in one launch;
the persistence side of a fork (``ForkHistoryBranch`` -> new branch token) stays on the host.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import List, Sequence, Tuple

import numpy as np

from . import abi
from .abi import NDC_BRANCH, NDC_TASK, VH_ITEM

Items = List[Tuple[int, int]]   # [(event_id, version)]


@dataclasses.dataclass
class NdcTask:
    local: List[Items]            # the workflow's VersionHistories (branch items)
    current_index: int            # CurrentVersionHistoryIndex
    incoming: Items               # the replication task's VersionHistory
    first_event_id: int
    first_event_version: int


@dataclasses.dataclass
class NdcBatch:
    tasks: np.ndarray             # abi.NDC_TASK
    branches: np.ndarray          # abi.NDC_BRANCH
    items: np.ndarray             # abi.VH_ITEM
    n_out_items: int


def pack(tasks: Sequence[NdcTask]) -> NdcBatch:
    t = np.zeros(max(len(tasks), 1), abi.NDC_TASK)[: len(tasks)]
    branches, items = [], []
    out = 0
    for k, task in enumerate(tasks):
        t[k]["branch_begin"] = len(branches)
        t[k]["branch_count"] = len(task.local)
        longest = 0
        for br in task.local:
            branches.append((len(items), len(br)))
            items.extend(br)
            longest = max(longest, len(br))
        t[k]["current_index"] = task.current_index
        t[k]["incoming_begin"] = len(items)
        t[k]["incoming_count"] = len(task.incoming)
        items.extend(task.incoming)
        t[k]["out_begin"] = out
        out += longest
        t[k]["first_event_id"] = task.first_event_id
        t[k]["first_event_version"] = task.first_event_version
    return NdcBatch(tasks=t, branches=np.array(branches or [(0, 0)], abi.NDC_BRANCH),
                    items=np.array(items or [(0, 0)], abi.VH_ITEM), n_out_items=max(out, 1))


def new_branch_items(batch: NdcBatch, results: np.ndarray, out_items: np.ndarray, k: int) -> Items:
    o = int(batch.tasks[k]["out_begin"])
    n = int(results[k]["new_item_count"])
    return [(int(x["event_id"]), int(x["version"])) for x in out_items[o:o + n]]


def prepare_on_device(engine, batch: NdcBatch, stream=None):
    """crr_ndc_prepare on ``engine``'s GPU; returns (results abi.NDC_RESULT[n], out_items abi.VH_ITEM[])."""
    torch = engine.torch
    dev = engine.dev
    n = len(batch.tasks)

    def up(a):
        raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        t = torch.empty(max(raw.size, 1), dtype=torch.uint8, device=dev)
        if raw.size:
            t[: raw.size].copy_(torch.from_numpy(raw))
        return t

    T = {"tasks": up(batch.tasks), "branches": up(batch.branches), "items": up(batch.items)}
    res = torch.zeros(max(n, 1) * abi.NDC_RESULT.itemsize, dtype=torch.uint8, device=dev)
    out = torch.zeros(batch.n_out_items * abi.VH_ITEM.itemsize, dtype=torch.uint8, device=dev)
    ci = abi.CNdcInputs()
    ci.tasks, ci.branches, ci.items = T["tasks"].data_ptr(), T["branches"].data_ptr(), T["items"].data_ptr()
    ci.n_tasks = n
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    rc = engine.lib.crr_ndc_prepare(ctypes.byref(ci), ctypes.c_void_p(res.data_ptr()),
                                    ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s.cuda_stream))
    if rc != 0:
        raise RuntimeError(f"crr_ndc_prepare failed: {rc}")
    torch.cuda.synchronize(dev)
    return (res.cpu().numpy().view(abi.NDC_RESULT)[:n].copy(), out.cpu().numpy().view(abi.VH_ITEM).copy())


# ---- full-size synthetic replication tasks (config 5 benchmark) ---------------------------------------------
def version_histories(batch) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Each workflow's VersionHistory items as AddOrUpdateItem builds them over its events (one item per
    run of a version: the run's last event ID), from a canonical batch's columns: (event_id, version,
    per-workflow count)."""
    assert batch.stride == 1
    n = batch.n_wf
    cnt = batch.wf["ev_count"].astype(np.int64)
    if int(cnt.sum()) == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(n, np.int64)
    idx = np.repeat(batch.wf["ev_begin"].astype(np.int64), cnt) + (np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt))
    wf_of = np.repeat(np.arange(n), cnt)
    e = batch.cols["event_id"][idx]
    v = batch.cols["version"][idx]
    last_of_run = np.ones(idx.size, bool)
    last_of_run[:-1] = (wf_of[1:] != wf_of[:-1]) | (v[1:] != v[:-1])
    keep = last_of_run
    return e[keep].astype(np.int64), v[keep].astype(np.int64), np.bincount(wf_of[keep], minlength=n).astype(np.int64)


def tasks_from_histories(vh_e, vh_v, vh_cnt, seed: int) -> NdcBatch:
    """One replication task per workflow against its VersionHistory (vectorised): the local histories
    are the workflow's branch, plus (30 %) a second branch forked one event earlier; the incoming
    VersionHistory shares the local prefix and then -- 40 % append (its last item extended; the batch
    starts right after the local last event), 25 % a new branch (forked one event before the local
    last event, a new version run; the batch starts after the fork point), 20 % a duplicate (the batch
    was already applied), 15 % out of order (events missing before the batch: RetryTaskV2)."""
    rng = np.random.default_rng(seed)
    n = vh_cnt.size
    c = vh_cnt.astype(np.int64)
    has = c > 0
    off = np.cumsum(c) - c
    last = off + np.maximum(c - 1, 0)
    le = np.where(has, vh_e[np.minimum(last, max(vh_e.size - 1, 0))] if vh_e.size else 0, 0)
    lv = np.where(has, vh_v[np.minimum(last, max(vh_v.size - 1, 0))] if vh_v.size else 0, 0)
    prev_e = np.where(c > 1, vh_e[np.maximum(last - 1, 0)] if vh_e.size else 0, 0)
    u = rng.random(n)
    case = np.select([u < 0.40, u < 0.65, u < 0.85], [0, 1, 2], 3)            # append, new branch, dup, retry
    two = (rng.random(n) < 0.3) & has
    fork_ok = has & (le - 1 > prev_e) & (le > 1)
    case = np.where((case == 1) & ~fork_ok, 0, case)
    d = rng.integers(1, 6, n)
    # segment lengths: branch 0, branch 1, incoming
    L0 = c
    L1 = np.where(two, c, 0)
    L2 = c + (case == 1)
    tot = L0 + L1 + L2
    start = np.cumsum(tot) - tot
    N = int(tot.sum())
    e_out = np.zeros(max(N, 1), np.int64)
    v_out = np.zeros(max(N, 1), np.int64)

    def seg(begin, length, src_off):
        m = int(length.sum())
        if m == 0:
            return None
        w = np.repeat(np.arange(n), length)
        j = np.arange(m) - np.repeat(np.cumsum(length) - length, length)
        dst = np.repeat(begin, length) + j
        src = np.repeat(src_off, length) + j
        return w, j, dst, src

    # branch 0: the workflow's items
    s0 = seg(start, L0, off)
    if s0 is not None:
        w, j, dst, src = s0
        e_out[dst], v_out[dst] = vh_e[src], vh_v[src]
    # branch 1: the same, its last item one event shorter where that keeps IDs increasing
    s1 = seg(start + L0, L1, off)
    if s1 is not None:
        w, j, dst, src = s1
        e_out[dst], v_out[dst] = vh_e[src], vh_v[src]
        is_last = j == c[w] - 1
        e_out[dst[is_last & fork_ok[w]]] -= 1
    # incoming
    s2 = seg(start + L0 + L1, np.minimum(L2, c), off)
    if s2 is not None:
        w, j, dst, src = s2
        e_out[dst], v_out[dst] = vh_e[src], vh_v[src]
        is_last = j == c[w] - 1
        cw = case[w]
        e_out[dst[is_last & (cw == 0)]] += d[w[is_last & (cw == 0)]]
        e_out[dst[is_last & (cw == 1)]] -= 1
        e_out[dst[is_last & (cw == 3)]] += 10
    nb = case == 1
    if nb.any():                                      # the new version run after the fork point
        pos = start[nb] + L0[nb] + L1[nb] + c[nb]
        e_out[pos] = le[nb] + 5
        v_out[pos] = lv[nb] + 100
    first = np.select([case == 0, case == 1, case == 2], [le + 1, le, le - 2], le + 5)
    first_v = np.where(case == 1, lv + 100, lv)
    first = np.maximum(first, 1)
    # pack
    n_br = 1 + two.astype(np.int64)
    br_off = np.cumsum(n_br) - n_br
    branches = np.zeros(max(int(n_br.sum()), 1), NDC_BRANCH)
    branches["item_begin"][br_off] = start
    branches["item_count"][br_off] = L0
    b1 = br_off[two] + 1
    branches["item_begin"][b1] = (start + L0)[two]
    branches["item_count"][b1] = L1[two]
    tasks = np.zeros(n, NDC_TASK)
    tasks["branch_begin"] = br_off
    tasks["branch_count"] = n_br
    tasks["current_index"] = np.where(two & (rng.random(n) < 0.5), 1, 0)
    tasks["incoming_begin"] = start + L0 + L1
    tasks["incoming_count"] = L2
    tasks["out_begin"] = np.cumsum(c) - c
    tasks["first_event_id"] = first
    tasks["first_event_version"] = first_v
    items = np.zeros(max(N, 1), VH_ITEM)
    items["event_id"], items["version"] = e_out, v_out
    return NdcBatch(tasks=tasks, branches=branches, items=items, n_out_items=max(int(c.sum()), 1))
