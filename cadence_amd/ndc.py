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
