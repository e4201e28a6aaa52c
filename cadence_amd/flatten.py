"""Host flattening: workflow histories -> structure-of-arrays columns (``crr_inputs``).

This is the work the Go side of the cgo shim does before calling the engine (north star: "Go host
code flattens decoded HistoryEvent batches into structure-of-arrays columns").  Two layouts:

* canonical  (stride 1): events of a workflow are contiguous; slot tables likewise.
* interleaved (stride 64): workflows sorted by length, 64 per group; column index
  ``group_base + step * 64 + lane`` so that a wavefront's 64 lanes (one workflow each) read one
  contiguous 64-element run per column per step -- fully coalesced HBM loads.
"""
from __future__ import annotations

import dataclasses
from typing import Tuple, Dict, List, Optional, Sequence

import numpy as np

from . import abi
from .abi import EventType as ET
from .history import WorkflowHistory, thrift_history_branch_token

WAVE = 64


@dataclasses.dataclass
class HistoryBatch:
    """Flattened input of one crr_replay call (host numpy arrays)."""
    cols: Dict[str, np.ndarray]           # event columns, see abi.EVENT_COLUMNS
    act_side: np.ndarray                  # abi.ACTIVITY_SIDE
    start_side: np.ndarray                # abi.START_SIDE
    reset_keys: np.ndarray                # uint32
    arena: np.ndarray                     # uint8 branch-token bytes
    wf: np.ndarray                        # abi.WORKFLOW
    stride: int
    # test / oracle only: per-event key strings (never shipped to the device)
    key_off: Optional[np.ndarray] = None
    key_len: Optional[np.ndarray] = None
    key_arena: Optional[np.ndarray] = None
    # interleaved batches: device position p holds canonical workflow perm[p]
    perm: Optional[np.ndarray] = None
    # sizes of the slot tables (rows)
    table_rows: Dict[str, int] = dataclasses.field(default_factory=dict)
    # length bucketing: workflows [wave_begin, n_wf) are long histories, contiguous (stride 1),
    # replayed one per wavefront (CRR_IN_WAVE_TAIL); None: every workflow uses `stride`
    wave_begin: Optional[int] = None
    # write the transfer / timer tasks ApplyEvents generates (CRR_IN_EMIT_TASKS)
    emit_tasks: bool = False
    # config.AdvancedVisibilityWritingMode != off: RefreshTasks' search-attributes task (CRR_IN_ADVANCED_VISIBILITY)
    advanced_visibility: bool = False
    # CRR_IN_STARTED_AUX: every ActivityTaskStarted's aux is its scheduled event's act_side index, or -1
    # (interleave: the device layouts)
    started_aux: bool = False
    # CRR_IN_TIERED: (large_begin, compact_begin, compact2_begin, wide_begin, hbm_begin, big_begin) --
    # lane workflows ordered by expected live-set size (TIER_SLOTS, then HBM rows); long-tail workflows
    # no fast per-wave arena is expected to hold from big_begin on
    tiers: Optional[Tuple[int, int, int, int, int, int]] = None
    # CRR_WF_FLAG_RESUME: the loaded mutable states (batch order) the output rows start from
    init: Optional["LoadedStates"] = None
    # per-workflow key id -> string tables (batch order): (begin, count, off, len, arena), the strings of
    # loaded rows for the oracle; interners: the host's per-workflow string -> key maps (batch order)
    key_dict: Optional[Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray, np.ndarray]] = None
    interners: Optional[List[Dict[str, int]]] = None

    def wf_strides(self) -> np.ndarray:
        """Column / row stride of every workflow."""
        st = np.full(self.n_wf, self.stride, np.int64)
        if self.wave_begin is not None:
            st[self.wave_begin:] = 1
        return st

    def c_flags(self) -> int:
        resume = self.tiers is not None and self.n_wf and bool((self.wf["flags"] & abi.WF_FLAG_RESUME).any())
        return ((abi.IN_WAVE_TAIL if self.wave_begin is not None else 0) | (abi.IN_EMIT_TASKS if self.emit_tasks else 0)
                | (abi.IN_TIERED if self.tiers is not None else 0) | (abi.IN_HAS_RESUME if resume else 0)
                | (abi.IN_ADVANCED_VISIBILITY if self.advanced_visibility else 0)
                | (abi.IN_STARTED_AUX if self.started_aux else 0))

    @property
    def n_wf(self) -> int:
        return int(self.wf.shape[0])

    @property
    def n_events(self) -> int:
        return int(self.wf["ev_count"].sum())

    @property
    def n_slots(self) -> int:
        return int(self.cols["etype"].shape[0])


def _zeros_cols(n):
    return {name: np.zeros(n, dtype=t) for name, t in abi.EVENT_COLUMNS}


@dataclasses.dataclass
class LoadedStates:
    """Loaded mutable states (``mutableStateBuilder.Load``) as the engine's row images, one per workflow
    of a batch (batch order): ``exec`` rows (all zero, counts 0, for a workflow that is not resumed),
    each table's live rows concatenated in workflow order (counts = the exec rows' n_* fields) and the
    resume mask.  ``ReplayResult.to_loaded`` builds one from a replay's output."""
    exec: np.ndarray                      # abi.EXEC_ROW [n]
    rows: Dict[str, np.ndarray]           # table -> live rows, workflow-major
    mask: np.ndarray                      # bool [n]: resume this workflow
    interners: Optional[List[Dict[str, int]]] = None

    def counts(self, name: str) -> np.ndarray:
        n_f = {t[0]: t[4] for t in abi.TABLES}[name]
        return np.maximum(self.exec[n_f].astype(np.int64), 0)

    def permuted(self, perm: np.ndarray) -> "LoadedStates":
        rows = {}
        for name in self.rows:
            c = self.counts(name)
            off = np.cumsum(c) - c
            cp = c[perm]
            idx = np.repeat(off[perm], cp) + (np.arange(int(cp.sum())) - np.repeat(np.cumsum(cp) - cp, cp))
            rows[name] = self.rows[name][idx]
        its = [self.interners[i] for i in perm] if self.interners is not None else None
        return LoadedStates(self.exec[perm].copy(), rows, self.mask[perm].copy(), its)


def write_init(batch: "HistoryBatch", exec_rows: np.ndarray, tables: Dict[str, np.ndarray]):
    """Place the batch's loaded states into output buffers (host images of crr_outputs): the exec
    rows of resumed workflows and their live rows in slots 0..n-1 of their slot tables."""
    init = batch.init
    if init is None:
        return
    m = init.mask
    exec_rows[m] = init.exec[m]
    st = batch.wf_strides()
    for name, _dt, base_f, _cap_f, _n_f in abi.TABLES:
        if name not in init.rows:
            continue
        c = init.counts(name)
        tot = int(c.sum())
        if tot == 0:
            continue
        wf_idx = np.repeat(np.arange(batch.n_wf), c)
        slot = np.arange(tot) - np.repeat(np.cumsum(c) - c, c)
        idx = batch.wf[base_f].astype(np.int64)[wf_idx] + slot * st[wf_idx]
        tables[name][idx] = init.rows[name]


def key_dict_from_interners(interners: List[Dict[str, int]]):
    """(begin, count, off, len, arena) of the per-workflow key id -> string tables."""
    strs, begin, count = [], np.zeros(len(interners), np.uint32), np.zeros(len(interners), np.uint32)
    for w, ids in enumerate(interners):
        inv = [""] * len(ids)
        for k, v in ids.items():
            inv[v] = k
        begin[w] = len(strs)
        count[w] = len(inv)
        strs.extend(inv)
    enc = [x.encode() for x in strs]
    lens = np.array([len(e) for e in enc] or [0], np.uint32)
    offs = (np.cumsum(lens) - lens).astype(np.uint32)
    arena = np.frombuffer(b"".join(enc) or b"\0", np.uint8).copy()
    return begin, count, offs, lens, arena


class _Interner:
    def __init__(self, ids: Optional[Dict[str, int]] = None):
        self.ids = ids if ids is not None else {"": 0}

    def __call__(self, s) -> int:
        s = "" if s is None else str(s)
        v = self.ids.get(s)
        if v is None:
            v = len(self.ids)
            self.ids[s] = v
        return v


def _domain_status(name, known_domains) -> int:
    if not name:
        return abi.DOMAIN_NOT_SET
    if known_domains is None or name in known_domains:
        return abi.DOMAIN_RESOLVED
    return abi.DOMAIN_UNKNOWN


def flatten(histories: Sequence[WorkflowHistory], known_domains=None,
            new_run_index: Optional[Dict[int, int]] = None, loaded: Optional[LoadedStates] = None,
            interners: Optional[List[Dict[str, int]]] = None) -> HistoryBatch:
    """Flatten object histories into a canonical HistoryBatch.

    ``known_domains``: domain names the domain cache resolves (None: all resolve).
    CAN events reference their new-run history through attrs["new_run"] = workflow index.
    ``loaded``: ApplyEvents continues these loaded states (``loaded.mask``; CRR_WF_FLAG_RESUME) --
    the histories are then the new batches only; their keys are interned with ``loaded.interners``
    (or ``interners``) so they match the loaded rows' keys.
    """
    if loaded is not None and interners is None:
        interners = loaded.interners
    n_ev = sum(len(b) for h in histories for b in h.batches)
    cols = _zeros_cols(n_ev)
    key_off = np.zeros(n_ev, np.uint32)
    key_len = np.zeros(n_ev, np.uint32)
    key_arena = bytearray()
    key_cache: Dict[str, int] = {}
    act_side, start_side, reset_keys = [], [], []
    arena = bytearray()
    wf = np.zeros(len(histories), dtype=abi.WORKFLOW)
    caps = {t[3]: np.zeros(len(histories), np.int64) for t in abi.TABLES}

    def put_key_str(i, s):
        s = "" if s is None else str(s)
        off = key_cache.get(s)
        if off is None:
            off = len(key_arena)
            key_arena.extend(s.encode())
            key_cache[s] = off
        key_off[i] = off
        key_len[i] = len(s.encode())

    i = 0
    interners_out: List[Dict[str, int]] = []
    for w, h in enumerate(histories):
        intern = _Interner(interners[w] if interners is not None else None)
        interners_out.append(intern.ids)
        begin = i
        empty_at = -1
        n_act = n_timer = n_child = n_rc = n_sig = n_dtc = 0
        n_tasks = 0          # upper bound of the tasks ApplyEvents generates (task_cap)
        max_prev = 0
        vh_items = 0
        last_ver = None
        for bi, batch in enumerate(h.batches):
            if not batch:
                if empty_at < 0:
                    empty_at = i - begin
                continue
            n_tasks += 2         # the batch's timer epilogue: one activity + one user timer task at most
            for j, e in enumerate(batch):
                t = int(e.event_type)
                n_tasks += TASKS_PER_EVENT.get(t, 0)
                flags = (abi.BATCH_FIRST if j == 0 else 0) | (abi.BATCH_LAST if j == len(batch) - 1 else 0)
                cols["etype"][i] = (t & abi.ETYPE_MASK) | flags if 0 <= t < abi.EV_TYPE_COUNT else (abi.EV_PAD - 1) | flags
                cols["event_id"][i] = e.id
                cols["version"][i] = e.version
                cols["timestamp"][i] = e.timestamp
                cols["task_id"][i] = e.task_id
                if last_ver is None or e.version > last_ver:
                    vh_items += 1
                    last_ver = e.version
                ref = 0
                key = 0
                aux = 0
                ks = None
                a = e.get
                if t == ET.WorkflowExecutionStarted:
                    prev = e.attrs.get("prev_auto_reset_points", None)
                    if prev is None:
                        prev_off, prev_cnt = 0, -1
                    elif prev == "nil_points":
                        prev_off, prev_cnt = 0, -2
                    else:
                        prev_off, prev_cnt = len(reset_keys), len(prev)
                        reset_keys.extend(intern(p) for p in prev)
                        max_prev = max(max_prev, len(prev))
                    pdid = e.attrs.get("parent_workflow_domain_id")
                    pdom = a("parent_workflow_domain", "")
                    pstat = abi.DOMAIN_NOT_SET if pdid is not None else _domain_status(pdom, known_domains)
                    init = e.attrs.get("initiator")
                    start_side.append((a("task_start_to_close_timeout_seconds", 0), a("execution_start_to_close_timeout_seconds", 0),
                                       a("first_decision_task_backoff_seconds", 0),
                                       abi.INITIATOR_NIL if init is None else int(init), pstat, prev_off, prev_cnt,
                                       a("attempt", 0), a("expiration_timestamp", 0), h.refresh_jitter))
                    aux = len(start_side) - 1
                elif t == ET.DecisionTaskScheduled:
                    ref = a("attempt", 0)
                    aux = a("start_to_close_timeout_seconds", 0)
                elif t == ET.DecisionTaskStarted:
                    ref = a("scheduled_event_id", 0)
                elif t == ET.DecisionTaskCompleted:
                    ref = a("started_event_id", 0)
                    ks = a("binary_checksum", "")
                    key = intern(ks)
                    n_dtc += 1
                elif t == ET.DecisionTaskTimedOut:
                    aux = a("timeout_type", 0)
                elif t == ET.ActivityTaskScheduled:
                    ks = a("activity_id", "")
                    key = intern(ks)
                    rp = e.attrs.get("retry_policy")
                    act_side.append((a("schedule_to_start_timeout_seconds", 0), a("schedule_to_close_timeout_seconds", 0),
                                     a("start_to_close_timeout_seconds", 0), a("heartbeat_timeout_seconds", 0),
                                     1 if rp is not None else 0,
                                     (rp or {}).get("expiration_interval_in_seconds", 0) if isinstance(rp, dict) else 0,
                                     _domain_status(a("domain", ""), known_domains), 0))
                    aux = len(act_side) - 1
                    n_act += 1
                elif t in (ET.ActivityTaskStarted, ET.ActivityTaskCompleted, ET.ActivityTaskFailed,
                           ET.ActivityTaskTimedOut, ET.ActivityTaskCanceled):
                    ref = a("scheduled_event_id", 0)
                elif t == ET.ActivityTaskCancelRequested:
                    ks = a("activity_id", "")
                    key = intern(ks)
                elif t == ET.TimerStarted:
                    ks = a("timer_id", "")
                    key = intern(ks)
                    ref = a("start_to_fire_timeout_seconds", 0)
                    n_timer += 1
                elif t in (ET.TimerFired, ET.TimerCanceled):
                    ks = a("timer_id", "")
                    key = intern(ks)
                elif t == ET.StartChildWorkflowExecutionInitiated:
                    aux = _domain_status(a("domain", ""), known_domains)
                    n_child += 1
                elif t == ET.RequestCancelExternalWorkflowExecutionInitiated:
                    aux = _domain_status(a("domain", ""), known_domains)
                    n_rc += 1
                elif t == ET.SignalExternalWorkflowExecutionInitiated:
                    aux = _domain_status(a("domain", ""), known_domains)
                    n_sig += 1
                elif t in (ET.StartChildWorkflowExecutionFailed, ET.ChildWorkflowExecutionStarted,
                           ET.ChildWorkflowExecutionCompleted, ET.ChildWorkflowExecutionFailed,
                           ET.ChildWorkflowExecutionCanceled, ET.ChildWorkflowExecutionTimedOut,
                           ET.ChildWorkflowExecutionTerminated, ET.RequestCancelExternalWorkflowExecutionFailed,
                           ET.ExternalWorkflowExecutionCancelRequested, ET.SignalExternalWorkflowExecutionFailed,
                           ET.ExternalWorkflowExecutionSignaled):
                    ref = a("initiated_event_id", 0)
                elif t == ET.WorkflowExecutionContinuedAsNew:
                    nr = e.attrs.get("new_run")
                    aux = -1 if nr is None else int(nr)
                cols["ref"][i] = ref
                cols["key"][i] = key
                cols["aux"][i] = aux
                put_key_str(i, ks)
                i += 1
        n = i - begin
        if empty_at < 0 and h.batches and not h.batches[-1]:
            empty_at = n
        if not h.batches:
            empty_at = 0
        tok = thrift_history_branch_token(h.run_id, h.branch_id)
        r = wf[w]
        r["ev_begin"] = begin
        r["ev_count"] = n
        r["empty_batch_at"] = empty_at
        r["init_version"] = h.domain_failover_version
        r["now_ns"] = h.now_ns
        r["start_token_off"] = len(arena)
        r["start_token_len"] = len(tok)
        arena.extend(tok)
        if h.final_token is not None:
            r["final_token_off"] = len(arena)
            r["final_token_len"] = len(h.final_token)
            arena.extend(h.final_token)
            r["rebuild_last_event_id"] = h.rebuild_last_event_id
            r["rebuild_last_event_version"] = h.rebuild_last_event_version
        else:
            r["final_token_off"] = 0
            r["final_token_len"] = abi.NO_TOKEN
        r["flags"] = (abi.WF_FLAG_NEW_RUN if h.is_new_run else 0) | (abi.WF_FLAG_REFRESH_TASKS if h.refresh_tasks else 0)
        if loaded is not None and loaded.mask[w]:
            r["flags"] |= abi.WF_FLAG_RESUME
        caps["act_cap"][w] = n_act
        caps["timer_cap"][w] = n_timer
        caps["child_cap"][w] = n_child
        caps["rc_cap"][w] = n_rc
        caps["sig_cap"][w] = n_sig
        caps["vh_cap"][w] = vh_items
        # + RefreshTasks' search-attributes task (its other tasks fit the replay's bound)
        caps["task_cap"][w] = n_tasks + (1 if h.refresh_tasks else 0)
        r["retention_days"] = h.retention_days
        caps["rp_cap"][w] = max_prev * max(1, sum(1 for e in h.events if e.event_type == ET.WorkflowExecutionStarted)) + n_dtc
    if loaded is not None:   # the loaded rows plus this call's inserts
        for name, _dt, _b, cap_f, n_f in abi.TABLES:
            if name != "tasks":
                caps[cap_f] += np.where(loaded.mask, loaded.exec[n_f], 0).astype(np.int64)
    batch = HistoryBatch(
        cols=cols,
        act_side=np.array(act_side or [(0,) * 8], dtype=abi.ACTIVITY_SIDE),
        start_side=np.array(start_side or [(0,) * 10], dtype=abi.START_SIDE),
        reset_keys=np.array(reset_keys or [0], dtype=np.uint32),
        arena=np.frombuffer(bytes(arena) or b"\0", dtype=np.uint8).copy(),
        wf=wf, stride=1,
        key_off=key_off, key_len=key_len,
        key_arena=np.frombuffer(bytes(key_arena) or b"\0", dtype=np.uint8).copy())
    assign_canonical_tables(batch, caps)
    batch.interners = interners_out
    batch.key_dict = key_dict_from_interners(interners_out)
    if loaded is not None:
        batch.init = loaded
    return batch


def assign_canonical_tables(batch: HistoryBatch, caps: Dict[str, np.ndarray]):
    """Canonical slot-table bases: prefix sums of per-workflow capacities."""
    for name, _dt, base_f, cap_f, _n in abi.TABLES:
        c = np.maximum(caps[cap_f].astype(np.int64), 0)
        base = np.zeros_like(c)
        if c.size:
            base[1:] = np.cumsum(c)[:-1]
        batch.wf[base_f] = base
        batch.wf[cap_f] = c
        batch.table_rows[name] = int(c.sum()) if c.size else 0


# tasks the task generator adds per event type (state_builder.go:157-625): an upper bound
TASKS_PER_EVENT = {int(ET.WorkflowExecutionStarted): 3, int(ET.DecisionTaskScheduled): 1, int(ET.DecisionTaskStarted): 1,
                   int(ET.DecisionTaskTimedOut): 1, int(ET.DecisionTaskFailed): 1, int(ET.ActivityTaskScheduled): 1,
                   int(ET.StartChildWorkflowExecutionInitiated): 1,
                   int(ET.RequestCancelExternalWorkflowExecutionInitiated): 1,
                   int(ET.SignalExternalWorkflowExecutionInitiated): 1, int(ET.UpsertWorkflowSearchAttributes): 1,
                   int(ET.WorkflowExecutionCompleted): 2, int(ET.WorkflowExecutionFailed): 2,
                   int(ET.WorkflowExecutionTimedOut): 2, int(ET.WorkflowExecutionCanceled): 2,
                   int(ET.WorkflowExecutionTerminated): 2, int(ET.WorkflowExecutionContinuedAsNew): 2}

LONG_HISTORY = 256   # lane per workflow up to ~256 events, a wavefront per workflow above


def interleave(batch: HistoryBatch, wave: int = WAVE, long_threshold: Optional[int] = LONG_HISTORY,
               tiered: bool = True, big_caps: Optional[Dict[str, int]] = None) -> HistoryBatch:
    """Permute a canonical batch into the device layout.

    Workflows are sorted by event count (descending; ties by index) and packed 64 per group.
    Group g occupies ``group_len[g] * 64`` event slots; lanes shorter than the group's longest
    workflow see CRR_EV_PAD slots.  With ``long_threshold`` (length bucketing), workflows longer
    than it form a tail after the groups: contiguous events and rows (stride 1), one wavefront
    each on the device (``long_threshold=None``: every workflow lane per workflow).  CAN ``aux``
    references are remapped to device positions.  ``big_caps``: per-map live-set bounds above which a
    long workflow goes to replay_big_kernel instead of the tail kernel (default WAVE_BIG_CAPS).  ``tiered``: lane workflows are first ordered by
    the LDS tier their live sets are expected to fit (``live_set_bounds``: 1 entry per map, 2, more;
    CRR_IN_TIERED), so each segment runs with the tier that holds it instead of being retried.
    """
    assert batch.stride == 1
    n = batch.n_wf
    counts = batch.wf["ev_count"].astype(np.int64)
    order = np.lexsort((np.arange(n), -counts)).astype(np.int64)
    is_long = counts[order] > long_threshold if long_threshold is not None else np.zeros(n, bool)
    bounds = live_set_bounds(batch) if (tiered and n) else None
    tier = tier_classes(batch, bounds) if (tiered and n) else np.zeros(n, np.int64)
    if tiered and n:
        resumed = (batch.wf["flags"] & abi.WF_FLAG_RESUME) != 0
        if resumed.any():
            # a loaded state continues in a compact tier's arena (CRR_IN_HAS_RESUME) when the loaded rows
            # plus this batch's growth fit it; in the long tail it goes to the replay_big_kernel segment
            # (whose HBM-row pass continues it)
            bounds, tier = resumed_bounds(batch, bounds, resumed)
            big_tail = {k: np.where(resumed, np.iinfo(np.int32).max, v) for k, v in bounds.items()}
        else:
            big_tail = bounds
        # a short history whose live sets outgrow every compact tier joins the wave tail (one
        # wavefront, a row arena searched by 64 lanes) rather than a lane over HBM rows
        if long_threshold is not None:
            is_long |= (tier[order] == WIDE) & ~resumed[order]
        bounds = big_tail
    lanes = order[~is_long]
    longs = order[is_long]
    n_big = 0
    if tiered:
        lanes = lanes[np.argsort(tier[lanes], kind="stable")]    # by tier, then longest first
        big = np.zeros(longs.size, bool)                          # the tail: arena-sized first, then big
        for k, cap in (WAVE_BIG_CAPS if big_caps is None else big_caps).items():
            big |= bounds[k][longs] > cap
        longs = np.concatenate([longs[~big], longs[big]])
        n_big = int(big.sum())
    perm = np.concatenate([lanes, longs])                          # device pos -> canonical wf
    n_lane = int(lanes.size)
    tiers = None
    if tiered:
        lane_tier = tier[perm[:n_lane]]
        # segment boundaries on group boundaries, rounded down (a mixed group takes the larger tier)
        bnd = []
        for k in range(WIDE):
            c = int((lane_tier <= k).sum())
            b = n_lane if c == n_lane else c // wave * wave
            bnd.append(max(b, bnd[-1]) if bnd else b)
        tiers = (*bnd, n - n_big)
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    n_groups = (n_lane + wave - 1) // wave
    pos = np.arange(n_groups * wave)
    lane = pos % wave
    group = pos // wave
    cnt_sorted = np.zeros(n_groups * wave, np.int64)
    cnt_sorted[:n_lane] = counts[perm[:n_lane]]
    glen = cnt_sorted.reshape(n_groups, wave).max(axis=1)
    gbase = np.zeros(n_groups, np.int64)
    if n_groups:
        gbase[1:] = np.cumsum(glen * wave)[:-1]
    lane_slots = int((glen * wave).sum())
    tail_cnt = counts[perm[n_lane:]]
    tail_begin = lane_slots + np.concatenate([[0], np.cumsum(tail_cnt)[:-1]]).astype(np.int64)
    total_slots = lane_slots + int(tail_cnt.sum())

    dev_begin = np.empty(n, np.int64)
    dev_begin[:n_lane] = gbase[group[:n_lane]] + lane[:n_lane]
    dev_begin[n_lane:] = tail_begin
    dev_stride = np.full(n, wave, np.int64)
    dev_stride[n_lane:] = 1

    # event permutation
    cperm = counts[perm]
    src_begin = batch.wf["ev_begin"][perm].astype(np.int64)
    wf_pos = np.repeat(np.arange(n), cperm)
    step = np.arange(wf_pos.size) - np.repeat(np.cumsum(cperm) - cperm, cperm)
    src_idx = src_begin[wf_pos] + step
    dst_idx = dev_begin[wf_pos] + step * dev_stride[wf_pos]
    cols = {}
    for name, t in abi.EVENT_COLUMNS:
        c = np.zeros(total_slots, dtype=t)
        if name == "etype":
            c[:] = abi.EV_PAD | abi.BATCH_FIRST | abi.BATCH_LAST
        c[dst_idx] = batch.cols[name][src_idx]
        cols[name] = c
    # CAN new-run references -> device positions
    can = (cols["etype"] & abi.ETYPE_MASK) == ET.WorkflowExecutionContinuedAsNew
    can &= cols["aux"] >= 0
    if can.any():
        cols["aux"][can] = inv[cols["aux"][can]]
    key_off = key_len = None
    if batch.key_off is not None:
        key_off = np.zeros(total_slots, np.uint32)
        key_len = np.zeros(total_slots, np.uint32)
        key_off[dst_idx] = batch.key_off[src_idx]
        key_len[dst_idx] = batch.key_len[src_idx]

    # side records follow their events: the k-th record of lane l of group g sits at
    # side_base[g] + k * 64 + l, so a wavefront reading the same ordinal is one coalesced run
    ev_type = batch.cols["etype"][src_idx] & abi.ETYPE_MASK
    act_side = _interleave_side(batch.act_side, ev_type == ET.ActivityTaskScheduled, wf_pos, src_idx, dst_idx,
                                cols, n, n_lane, n_groups, wave, group, lane)
    start_side = _interleave_side(batch.start_side, ev_type == ET.WorkflowExecutionStarted, wf_pos, src_idx, dst_idx,
                                  cols, n, n_lane, n_groups, wave, group, lane)
    _join_started(batch, ev_type, wf_pos, step, src_idx, dst_idx, src_begin, dev_begin, dev_stride, cols)

    wf = batch.wf[perm].copy()
    wf["ev_begin"] = dev_begin
    kd = None
    if batch.key_dict is not None:
        kb, kc, ko, kl, ka = batch.key_dict
        kd = (kb[perm].copy(), kc[perm].copy(), ko, kl, ka)
    out = HistoryBatch(cols=cols, act_side=act_side, start_side=start_side,
                       reset_keys=batch.reset_keys, arena=batch.arena, wf=wf, stride=wave,
                       key_off=key_off, key_len=key_len, key_arena=batch.key_arena, perm=perm,
                       wave_begin=n_lane if long_threshold is not None else None, emit_tasks=batch.emit_tasks,
                       advanced_visibility=batch.advanced_visibility, started_aux=True, tiers=tiers, init=batch.init.permuted(perm) if batch.init is not None else None,
                       key_dict=kd, interners=[batch.interners[i] for i in perm] if batch.interners else None)
    for name, _dt, base_f, cap_f, _n in abi.TABLES:
        cap = np.zeros(n_groups * wave, np.int64)
        cap[:n_lane] = wf[cap_f][:n_lane]
        gcap = cap.reshape(n_groups, wave).max(axis=1)
        tbase = np.zeros(n_groups, np.int64)
        if n_groups:
            tbase[1:] = np.cumsum(gcap * wave)[:-1]
        lane_rows = int((gcap * wave).sum())
        tcap = np.maximum(wf[cap_f][n_lane:].astype(np.int64), 0)
        wf[base_f][:n_lane] = tbase[group[:n_lane]] + lane[:n_lane]
        wf[cap_f][:n_lane] = gcap[group[:n_lane]]
        wf[base_f][n_lane:] = lane_rows + np.concatenate([[0], np.cumsum(tcap)[:-1]]).astype(np.int64)
        out.table_rows[name] = lane_rows + int(tcap.sum())
    return out


def _interleave_side(side: np.ndarray, sel: np.ndarray, wf_pos, src_idx, dst_idx, cols, n, n_lane, n_groups, wave,
                     group, lane) -> np.ndarray:
    """Re-home the side records referenced by the selected events (wave-interleaved by ordinal) and
    point those events' ``aux`` at the new positions (``cols`` is already in device order)."""
    if not sel.any():
        return side
    w = wf_pos[sel]                      # device workflow of each referencing event (ascending)
    cnt = np.bincount(w, minlength=n).astype(np.int64)
    k = np.arange(w.size) - np.repeat(np.cumsum(cnt) - cnt, cnt)[: w.size]
    gcap = np.zeros(max(n_groups, 1), np.int64)
    if n_lane:
        np.maximum.at(gcap, group[:n_lane], cnt[:n_lane])
    gbase = np.concatenate([[0], np.cumsum(gcap * wave)[:-1]]).astype(np.int64)
    lane_rows = int((gcap * wave).sum())
    tcnt = cnt[n_lane:]
    tbase = lane_rows + np.concatenate([[0], np.cumsum(tcnt)[:-1]]).astype(np.int64)
    is_lane = w < n_lane
    new_idx = np.empty(w.size, np.int64)
    wl = w[is_lane]
    new_idx[is_lane] = gbase[group[wl]] + k[is_lane] * wave + lane[wl]
    wt = w[~is_lane]
    new_idx[~is_lane] = tbase[wt - n_lane] + k[~is_lane]
    out = np.zeros(max(lane_rows + int(tcnt.sum()), 1), side.dtype)
    dst = dst_idx[sel]
    out[new_idx] = side[cols["aux"][dst]]
    cols["aux"][dst] = new_idx.astype(np.int32)
    return out


def _join_started(batch, ev_type, wf_pos, step, src_idx, dst_idx, src_begin, dev_begin, dev_stride, cols):
    """CRR_IN_STARTED_AUX: each ActivityTaskStarted's aux becomes the (already re-homed) act_side index of its
    ActivityTaskScheduled event -- the event d = ID - ScheduledEventID steps before it in the same history, when
    that one is an ActivityTaskScheduled with ID == ScheduledEventID (IDs increase by one within a call) -- else
    -1.  The compact tiers read the scheduled event's timeouts from it (replay_kernel.hip act_started) instead of
    gathering that event's aux first (mutable_state_builder.go:2254-2276 reads the ActivityInfo the scheduled
    event built).  crr_ingest_layout writes the same (ingest_kernel.hip put_slot)."""
    st = ev_type == ET.ActivityTaskStarted
    if not st.any():
        return
    sel = np.nonzero(st)[0]
    src = src_idx[sel]
    ref = batch.cols["ref"][src].astype(np.int64)
    d = batch.cols["event_id"][src].astype(np.int64) - ref
    k = step[sel]
    ok = (d >= 1) & (d <= k)
    ks = np.where(ok, k - d, 0)
    w = wf_pos[sel]
    cand = src_begin[w] + ks                                   # canonical (stride 1) slot of the candidate
    ok &= ((batch.cols["etype"][cand] & abi.ETYPE_MASK) == ET.ActivityTaskScheduled) & \
        (batch.cols["event_id"][cand].astype(np.int64) == ref)
    dst_s = dev_begin[w] + ks * dev_stride[w]
    cols["aux"][dst_idx[sel]] = np.where(ok, cols["aux"][dst_s], -1).astype(np.int32)


def table_rows_of(batch: HistoryBatch, exec_rows: np.ndarray, tables: Dict[str, np.ndarray], w: int):
    """Live rows of workflow ``w`` (batch order) from output tables: {table: structured array}."""
    r = batch.wf[w]
    out = {}
    for name, _dt, base_f, _cap_f, n_f in abi.TABLES:
        n = int(exec_rows[w][n_f])
        n = min(n, int(r[_cap_f]))
        idx = int(r[base_f]) + np.arange(n, dtype=np.int64) * int(batch.wf_strides()[w])
        out[name] = tables[name][idx]
    return out


SMALL_TIER = {"act": 1, "timer": 1, "child": 1, "rc": 1, "sig": 1, "rp": 1}
LARGE_TIER = {"act": 2, "timer": 2, "child": 1, "rc": 1, "sig": 1, "rp": 2}   # CRR_LDS_* defaults
# replay_kernel.hip CompactTier1 / CompactTier2 (u32 event IDs, 10-bit event steps: <= 1023 events)
COMPACT1_TIER = {"act": 4, "timer": 3, "child": 2, "rc": 1, "sig": 1, "rp": 4}
COMPACT2_TIER = {"act": 8, "timer": 5, "child": 3, "rc": 3, "sig": 3, "rp": 8}
COMPACT3_TIER = {"act": 12, "timer": 8, "child": 6, "rc": 4, "sig": 4, "rp": 8}
COMPACT_MAX_EVENTS = 1023
# tier classes 0..4; WIDE: HBM rows
TIER_SLOTS = [SMALL_TIER, LARGE_TIER, COMPACT1_TIER, COMPACT2_TIER, COMPACT3_TIER]
WIDE = len(TIER_SLOTS)
COMPACT_FIRST = 2  # TIER_SLOTS index of compact tier 1


def _pair_keys(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """(a, b) int64 pairs as one 16-byte opaque key each (np.isin / np.unique compare them exactly)."""
    return np.ascontiguousarray(np.stack([a.astype(np.int64), b.astype(np.int64)], axis=1)).view("V16").ravel()


def live_set_bounds(batch: HistoryBatch) -> Dict[str, np.ndarray]:
    """Approximate peak live-set size per workflow and map (running inserts - deletes of inserted
    keys; reset points: distinct non-empty binary checksums + previous points).  Used only to pick the LDS tier: a
    workflow that outgrows its tier is replayed by the general path, so this affects speed only."""
    n = batch.n_wf
    cnt = batch.wf["ev_count"].astype(np.int64)
    step = np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    idx = np.repeat(batch.wf["ev_begin"].astype(np.int64), cnt) + step * np.repeat(batch.wf_strides(), cnt)
    t = (batch.cols["etype"][idx] & abi.ETYPE_MASK).astype(np.int64)
    wf_of = np.repeat(np.arange(n), cnt)
    out = {}
    rules = {
        "act": ([ET.ActivityTaskScheduled], [ET.ActivityTaskCompleted, ET.ActivityTaskFailed, ET.ActivityTaskTimedOut,
                                            ET.ActivityTaskCanceled]),
        "timer": ([ET.TimerStarted], [ET.TimerFired, ET.TimerCanceled]),
        "child": ([ET.StartChildWorkflowExecutionInitiated],
                  [ET.StartChildWorkflowExecutionFailed, ET.ChildWorkflowExecutionCompleted,
                   ET.ChildWorkflowExecutionFailed, ET.ChildWorkflowExecutionCanceled,
                   ET.ChildWorkflowExecutionTimedOut, ET.ChildWorkflowExecutionTerminated]),
        "rc": ([ET.RequestCancelExternalWorkflowExecutionInitiated],
               [ET.RequestCancelExternalWorkflowExecutionFailed, ET.ExternalWorkflowExecutionCancelRequested]),
        "sig": ([ET.SignalExternalWorkflowExecutionInitiated],
                [ET.SignalExternalWorkflowExecutionFailed, ET.ExternalWorkflowExecutionSignaled]),
    }
    starts = np.cumsum(cnt) - cnt
    nz = cnt > 0
    for name, (ins, dels) in rules.items():
        lut = np.zeros(64, np.int8)
        lut[[int(x) for x in ins]] = 1
        lut[[int(x) for x in dels]] = -1
        d = lut[t]
        # a delete of an entry that is not live only logs an inconsistency (Go): count a delete only
        # if its key was inserted earlier in the workflow (and, for ID-keyed maps, deleted once)
        dpos = np.nonzero(d < 0)[0]
        if dpos.size:
            ipos = np.nonzero(d > 0)[0]
            col, ins_col = ("key", "key") if name == "timer" else ("ref", "event_id")
            # (workflow, full 64-bit value) pairs, compared exactly (ingest_kernel.hip does the same)
            ik = _pair_keys(wf_of[ipos], batch.cols[ins_col][idx[ipos]])
            dk = _pair_keys(wf_of[dpos], batch.cols[col][idx[dpos]])
            valid = np.isin(dk, ik)
            if name != "timer":
                valid &= batch.cols["ref"][idx[dpos]] < batch.cols["event_id"][idx[dpos]]
                first = np.zeros(dpos.size, bool)
                first[np.unique(dk, return_index=True)[1]] = True
                valid &= first
            d = d.copy()
            d[dpos[~valid]] = 0
        if d.size == 0 or not d.any():
            out[name] = np.zeros(n, np.int64)
            continue
        cs = np.cumsum(d, dtype=np.int64)
        base = np.where(starts > 0, cs[np.maximum(starts - 1, 0)], 0)
        rel = cs - np.repeat(base, cnt)
        mx = np.zeros(n, np.int64)
        mx[nz] = np.maximum.reduceat(rel, starts[nz])
        out[name] = np.maximum(mx, 0)
    # reset points: distinct non-empty binary checksums per workflow (the replay path never evicts:
    # maxResetPoints = MaxInt32) + points carried over by the start event
    dtc_pos = np.nonzero((t == ET.DecisionTaskCompleted) & (batch.cols["key"][idx] != 0))[0]
    rp = np.zeros(n, np.int64)
    if dtc_pos.size:
        pair = (wf_of[dtc_pos].astype(np.uint64) << np.uint64(32)) | batch.cols["key"][idx[dtc_pos]].astype(np.uint64)
        rp = np.bincount((np.unique(pair) >> np.uint64(32)).astype(np.int64), minlength=n).astype(np.int64)
    prev = np.zeros(n, np.int64)
    st = t == ET.WorkflowExecutionStarted
    if st.any():
        pc = batch.start_side["prev_reset_count"][batch.cols["aux"][idx][st]].astype(np.int64)
        np.maximum.at(prev, wf_of[st], np.maximum(pc, 0))
    out["rp"] = rp + prev
    return out


# per-wave LDS arenas of the wave-per-workflow tail (replay_kernel.hip WaveTier<SmallTier>)
WAVE_SMALL_TIER = {"act": 40, "timer": 32, "child": 16, "rc": 8, "sig": 8, "rp": 24}
# replay_tail_kernel's per-wave LDS arena is WaveTier<LargeTier> (64/48/24/16/16/32 rows); a workflow that
# outgrows it is replayed again over its HBM rows in the same wavefront.  Only beyond 64 entries in some map
# does a workflow go to replay_big_kernel (whose one-wave blocks hold a 57 KB arena): measured on the config-4
# long tail, sending everything past the arena there costs more (poor occupancy) than the in-place retries.
WAVE_BIG_CAPS = {"act": 64, "timer": 64, "child": 64, "rc": 64, "sig": 64, "rp": 64}


# the event ID each table's rows are keyed by (CompactTables::load's virtual steps)
LOADED_ID = {"act": "schedule_id", "timer": "started_id", "child": "initiated_id", "rc": "initiated_id",
             "sig": "initiated_id"}
LOADED_COUNT = {"act": "n_activity", "timer": "n_timer", "child": "n_child", "rc": "n_rc", "sig": "n_signal",
                "rp": "n_reset_points"}


def resumed_bounds(batch: HistoryBatch, bounds: Dict[str, np.ndarray], resumed: np.ndarray):
    """Live-set bounds and tier classes with the loaded states counted in: a resumed workflow's bound is
    its loaded rows plus this batch's growth (deletes of loaded entries not subtracted: an upper bound).
    The compact tiers hold a loaded entry as a virtual step below vk = COMPACT_MAX_EVENTS - ev_count
    (CompactTables::load: its ID must lie in [NextEventID - vk, NextEventID)), so a resumed workflow goes
    there when its oldest live loaded ID does -- however long the history before it; CompactTables::load
    still hands anything else to the general path."""
    ex = batch.init.exec if batch.init is not None else None
    out = {}
    for m, v in bounds.items():
        add = np.maximum(ex[LOADED_COUNT[m]].astype(np.int64), 0) if ex is not None else 0
        out[m] = np.where(resumed, v + add, v)
    tier = tier_classes(batch, out)
    if ex is not None:
        nei = ex["next_event_id"].astype(np.int64)
        vk = COMPACT_MAX_EVENTS - batch.wf["ev_count"].astype(np.int64)
        oldest = nei.copy()  # no live loaded entry: nothing to place below vk
        for name, id_f in LOADED_ID.items():
            rows = batch.init.rows.get(name)
            c = batch.init.counts(name)
            if rows is None or not c.sum():
                continue
            np.minimum.at(oldest, np.repeat(np.arange(batch.n_wf), c), rows[id_f].astype(np.int64))
        tier = np.where(resumed & ((vk <= 0) | (nei - oldest > vk)), WIDE, tier)
    else:
        tier = np.where(resumed, WIDE, tier)
    # the 1- and 2-slot tiers rebuild rows from this call's events only: a resumed workflow they would
    # hold takes the smallest compact tier that does, so those segments keep their fast kernels for the
    # batch's fresh workflows (the device hands a loaded state found there to the general path)
    low = resumed & (tier < COMPACT_FIRST)
    if low.any():
        ok = _compact_ok(batch)
        cls = np.full(batch.n_wf, WIDE, np.int64)
        for k in range(WIDE - 1, COMPACT_FIRST - 1, -1):
            fit = ok.copy()
            for m, cap in TIER_SLOTS[k].items():
                fit &= out[m] <= cap
            cls = np.where(fit, k, cls)
        tier = np.where(low, cls, tier)
    return out, tier


def _compact_ok(batch: HistoryBatch) -> np.ndarray:
    """Workflows the compact encodings can take: <= COMPACT_MAX_EVENTS events, event IDs below 2^32."""
    cnt = batch.wf["ev_count"].astype(np.int64)
    ok = cnt <= COMPACT_MAX_EVENTS
    if batch.n_events:
        st = batch.wf_strides()
        idx = np.repeat(batch.wf["ev_begin"].astype(np.int64), cnt) + (
            np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt)) * np.repeat(st, cnt)
        big_id = np.zeros(batch.n_wf, bool)
        np.logical_or.at(big_id, np.repeat(np.arange(batch.n_wf), cnt), batch.cols["event_id"][idx] > 0xFFFFFFFF)
        ok &= ~big_id
    return ok


def tier_classes(batch: HistoryBatch, bounds: Optional[Dict[str, np.ndarray]] = None) -> np.ndarray:
    """Per workflow: the smallest LDS tier (TIER_SLOTS index) its live sets are expected to fit, WIDE
    (HBM rows) when none does.  The compact tiers also need <= COMPACT_MAX_EVENTS events and event IDs
    below 2^32 (their encodings; the kernel hands anything else to the general path anyway)."""
    b = live_set_bounds(batch) if bounds is None else bounds
    cls = np.full(batch.n_wf, WIDE, np.int64)
    compact_ok = _compact_ok(batch)
    for k in range(WIDE - 1, -1, -1):
        fit = np.ones(batch.n_wf, bool)
        for m, cap in TIER_SLOTS[k].items():
            fit &= b[m] <= cap
        if k >= 2:
            fit &= compact_ok
        cls = np.where(fit, k, cls)
    # the 2-slot LdsTables tier holds full rows (about 270 B per lane: 2 blocks of 4 wavefronts per CU);
    # compact tier 1 holds more entries in 176 B per lane (3 wavefronts per SIMD), so a workflow both fit
    # goes there (measured on the config-3 shard: 3.41 -> 3.20 ms); the 2-slot tier keeps the workflows
    # the compact encodings cannot take
    cls = np.where((cls == 1) & compact_ok, 2, cls)
    return cls


def fits_small_tier(batch: HistoryBatch, lanes: bool = True) -> bool:
    """Whether the 3-blocks/CU LDS tier holds every workflow's live sets (lane part: 1 entry per
    map, unless ``lanes`` is False; wave tail: the small per-wave arena)."""
    nl = batch.n_wf if batch.wave_begin is None else batch.wave_begin
    te = batch.tiers[-1] if batch.tiers is not None else batch.n_wf   # [te, n): replay_big_kernel
    if not lanes and nl == te:
        return True
    b = live_set_bounds(batch)
    lane_ok = not lanes or all(bool((b[k][:nl] <= v).all()) for k, v in SMALL_TIER.items())
    tail_ok = all(bool((b[k][nl:te] <= v).all()) for k, v in WAVE_SMALL_TIER.items())
    return lane_ok and tail_ok
