"""Host mirror of Cadence's replay interfaces over the batched MI355X engine.

The reference's interface for this path is Go:

* ``StateBuilder{ApplyEvents(domainID, requestID, workflowExecution, history, newRunHistory)
  (MutableState, error); GetMutableState() MutableState}``  (service/history/execution/state_builder.go:41-51)
* ``StateRebuilder.Rebuild(...) (MutableState, int64, error)``  (state_rebuilder.go:97-191)
* the ``MutableState`` getters replay callers read (mutable_state.go:59-239)

This module keeps those names, argument meanings and error behaviour (same error kinds and
messages; the first error aborts the workflow and leaves it partially applied, no rollback) on top
of the C ABI (``include/cadence_replay.h``) through :mod:`cadence_amd.engine`.  Work is batched: a
:class:`BatchStateBuilder` collects many workflows, replays them in one ``crr_replay`` and
materialises one :class:`MutableState` per workflow from the device rows, resolving every
string-valued field from the event that supplied it (``*_src`` provenance), exactly what the cgo
shim does on the Go side.

Fields the reference fills from ``uuid.New()`` / ``timeSource.Now()`` (child CreateRequestID,
request-cancel / signal request IDs, decision timestamps after a failure, reset-point creation time)
come from the host-injected inputs of :class:`~cadence_amd.history.WorkflowHistory` (``now_ns``)
and from ``uuid_fn`` (default: a deterministic UUID of run ID and event step).
"""
from __future__ import annotations

import dataclasses
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .abi import EventType as ET, Status
from .flatten import HistoryBatch, LoadedStates, flatten, interleave
from .history import HistoryEvent, WorkflowHistory, det_uuid, thrift_history_branch_token

EMPTY_UUID = "emptyUuid"  # common.EmptyUUID (common/constants.go:44)


# ---- errors (common/types/errors.go, common/errors) -------------------------------------------------
class CadenceError(Exception):
    """Base of the Go error kinds ApplyEvents returns."""
    go_type = "error"

    def __init__(self, message: str, status: int = 0, step: int = -1):
        super().__init__(message)
        self.message = message
        self.status = status
        self.step = step


class BadRequestError(CadenceError):
    go_type = "*types.BadRequestError"


class InternalServiceError(CadenceError):
    go_type = "*types.InternalServiceError"


class InternalFailureError(CadenceError):
    go_type = "errors.InternalFailureError"


class EntityNotExistsError(CadenceError):
    go_type = "*types.EntityNotExistsError"


class PanicError(CadenceError):
    """NewVersionHistoryItem panics in Go (versionHistory.go:37-43); surfaced as an exception."""
    go_type = "panic"


# status code -> (error class, message) with the reference's messages
_STATUS_ERRORS = {
    Status.EMPTY_HISTORY: (InternalFailureError, "encounter history size being zero"),  # state_builder.go:68, :98-100
    Status.UNKNOWN_EVENT_TYPE: (BadRequestError, "Unknown event type"),                 # :629-630
    Status.VH_LOWER_VERSION: (BadRequestError, "cannot update version history with a lower version"),
    Status.VH_EVENT_ID_NOT_INCREASING: (BadRequestError, "cannot add version history with a lower event id"),
    Status.VH_INVALID_ITEM: (PanicError, "invalid version history item event ID or version"),
    Status.VH_EMPTY: (BadRequestError, "version history is empty"),                     # versionHistory.go:303-308
    Status.INVALID_STATE_TRANSITION: (InternalServiceError, "unable to change workflow state"),
    Status.UNKNOWN_WORKFLOW_STATE: (InternalServiceError, "unknown workflow state"),
    Status.MISSING_ACTIVITY_INFO: (InternalServiceError, "unable to get activity info"),   # mutable_state_builder.go:64-65
    Status.MISSING_CHILD_INFO: (InternalServiceError, "unable to get child workflow info"),  # :66-67
    Status.DECISION_NOT_FOUND: (InternalFailureError, "unable to find decision"),          # decision_task_manager.go:211-214
    Status.DOMAIN_NOT_FOUND: (EntityNotExistsError, "Domain name not found"),
    Status.BAD_INITIATOR: (InternalServiceError, "unknown initiator"),                     # task_generator.go:269-277
    Status.TIMER_SEQUENCE: (InternalServiceError, "unable to load activity or timer"),
    Status.REBUILD_LAST_ITEM: (BadRequestError, "nDCStateRebuilder unable to rebuild mutable state"),
    Status.NEW_RUN_MISSING: (InternalServiceError, "continue-as-new new-run history missing"),
    Status.CAPACITY: (InternalServiceError, "engine slot table too small"),
}


def status_error(status: int, step: int) -> Optional[CadenceError]:
    """The Go error ApplyEvents returns for a device status code (None for CRR_OK)."""
    if status == Status.OK:
        return None
    cls, msg = _STATUS_ERRORS.get(Status(status), (InternalServiceError, f"status {status}"))
    return cls(msg, status=int(status), step=int(step))


# ---- persistence types (common/persistence/dataManagerInterfaces.go) --------------------------------
def _time(ns: int) -> Optional[int]:
    """Unix ns, or None for Go's zero time.Time{}."""
    return None if int(ns) == abi.ZERO_TIME else int(ns)


@dataclasses.dataclass
class ActivityInfo:  # persistence.ActivityInfo (dataManagerInterfaces.go:593-630)
    version: int
    schedule_id: int
    scheduled_event_batch_id: int
    scheduled_time: int
    started_id: int
    started_time: Optional[int]
    activity_id: str
    request_id: str
    domain_id: str
    schedule_to_start_timeout: int
    schedule_to_close_timeout: int
    start_to_close_timeout: int
    heartbeat_timeout: int
    cancel_requested: bool
    cancel_request_id: int
    last_heartbeat_updated_time: Optional[int]
    timer_task_status: int
    task_list: str
    has_retry_policy: bool
    last_heartbeat_timeout_visibility_in_seconds: int


@dataclasses.dataclass
class TimerInfo:  # persistence.TimerInfo
    version: int
    timer_id: str
    started_id: int
    expiry_time: int
    task_status: int


@dataclasses.dataclass
class ChildExecutionInfo:  # persistence.ChildExecutionInfo
    version: int
    initiated_id: int
    initiated_event_batch_id: int
    started_id: int
    started_workflow_id: str
    started_run_id: str
    create_request_id: str
    domain_id: str
    workflow_type_name: str
    parent_close_policy: int


@dataclasses.dataclass
class RequestCancelInfo:  # persistence.RequestCancelInfo
    version: int
    initiated_event_batch_id: int
    initiated_id: int
    cancel_request_id: str


@dataclasses.dataclass
class SignalInfo:  # persistence.SignalInfo
    version: int
    initiated_event_batch_id: int
    initiated_id: int
    signal_request_id: str
    signal_name: str
    input: bytes
    control: bytes


@dataclasses.dataclass
class VersionHistoryItem:  # persistence.VersionHistoryItem (versionHistory.go:32-46)
    event_id: int
    version: int


@dataclasses.dataclass
class VersionHistory:  # persistence.VersionHistory
    branch_token: bytes
    items: List[VersionHistoryItem]

    def get_last_item(self) -> VersionHistoryItem:  # versionHistory.go:303-313
        if not self.items:
            raise BadRequestError("version history is empty")
        return dataclasses.replace(self.items[-1])


@dataclasses.dataclass
class VersionHistories:  # persistence.VersionHistories
    current_version_history_index: int
    histories: List[VersionHistory]

    def get_current_version_history(self) -> VersionHistory:
        return self.histories[self.current_version_history_index]


@dataclasses.dataclass
class ResetPointInfo:  # types.ResetPointInfo
    binary_checksum: str
    run_id: str
    first_decision_completed_id: int
    created_time_nano: int
    resettable: bool
    from_previous_run: bool


@dataclasses.dataclass
class Checksum:  # common/checksum/defs.go: Checksum{Version, Flavor, Value}
    version: int
    flavor: int
    value: bytes


@dataclasses.dataclass
class Task:
    """A persistence.Task the task generator added (mutable_state_task_generator.go); ``kind`` is an
    abi.TaskKind.  Strings come from the event at step ``src``: the task list (decision / activity),
    the target domain / workflow (child, cancel, signal).  Cross-cluster wrapping of child / cancel /
    signal / close tasks needs cluster metadata and is left to the caller."""
    kind: int
    version: int
    visibility_timestamp: int = 0     # timer tasks
    event_id: int = 0                 # ScheduleID / InitiatedID / timer EventID
    timeout_type: int = 0             # timer / backoff type
    attempt: int = 0
    task_list: str = ""
    target_domain: str = ""
    target_workflow_id: str = ""


TRANSFER_KINDS = {abi.TaskKind.RecordWorkflowStarted, abi.TaskKind.Decision, abi.TaskKind.Activity,
                  abi.TaskKind.StartChild, abi.TaskKind.CancelExecution, abi.TaskKind.SignalExecution,
                  abi.TaskKind.UpsertSearchAttributes, abi.TaskKind.CloseExecution}


@dataclasses.dataclass
class WorkflowExecutionInfo:  # persistence.WorkflowExecutionInfo (the fields replay writes)
    domain_id: str
    workflow_id: str
    run_id: str
    state: int
    close_status: int
    next_event_id: int
    last_first_event_id: int
    last_event_task_id: int
    last_processed_event: int
    completion_event_batch_id: int
    signal_count: int
    cancel_requested: bool
    decision_version: int
    decision_schedule_id: int
    decision_started_id: int
    decision_request_id: str
    decision_timeout: int
    decision_attempt: int
    decision_started_timestamp: int
    decision_scheduled_timestamp: int
    decision_original_scheduled_timestamp: int
    start_timestamp: Optional[int]
    auto_reset_points: Optional[List[ResetPointInfo]]


class MutableState:
    """The replayed state of one workflow, with the Go getter names replay callers use."""

    def __init__(self):
        self.execution_info: Optional[WorkflowExecutionInfo] = None
        self.pending_activity_info_ids: Dict[int, ActivityInfo] = {}
        self.pending_activity_id_to_event_id: Dict[str, int] = {}
        self.pending_timer_info_ids: Dict[str, TimerInfo] = {}
        self.pending_timer_event_id_to_id: Dict[int, str] = {}
        self.pending_child_execution_info_ids: Dict[int, ChildExecutionInfo] = {}
        self.pending_request_cancel_info_ids: Dict[int, RequestCancelInfo] = {}
        self.pending_signal_info_ids: Dict[int, SignalInfo] = {}
        self.version_histories: Optional[VersionHistories] = None
        self.current_version: int = abi.EMPTY_VERSION
        self.checksum: Optional[Checksum] = None
        self.inconsistencies: int = 0
        self.transfer_tasks: List[Task] = []
        self.timer_tasks: List[Task] = []
        # what mutableStateBuilder.Load would read back (mutable_state_builder.go:306-349): the engine's row
        # images of this state, so a StateBuilder constructed on it continues it on the device
        self._loaded: Optional["_LoadedImage"] = None

    # mutable_state.go:59-239 (the subset replay callers read)
    def get_execution_info(self) -> WorkflowExecutionInfo:
        return self.execution_info

    def get_next_event_id(self) -> int:
        return self.execution_info.next_event_id

    def get_last_first_event_id(self) -> int:
        return self.execution_info.last_first_event_id

    def get_previous_started_event_id(self) -> int:
        return self.execution_info.last_processed_event

    def get_current_version(self) -> int:
        return self.current_version

    def get_version_histories(self) -> Optional[VersionHistories]:
        return self.version_histories

    def get_workflow_state_close_status(self) -> Tuple[int, int]:
        return self.execution_info.state, self.execution_info.close_status

    def is_workflow_execution_running(self) -> bool:
        return self.execution_info.state not in (abi.State.Completed,)

    def get_pending_activity_infos(self) -> Dict[int, ActivityInfo]:
        return self.pending_activity_info_ids

    def get_activity_info(self, schedule_id: int) -> Tuple[Optional[ActivityInfo], bool]:
        ai = self.pending_activity_info_ids.get(schedule_id)
        return ai, ai is not None

    def get_activity_by_activity_id(self, activity_id: str) -> Tuple[Optional[ActivityInfo], bool]:
        sid = self.pending_activity_id_to_event_id.get(activity_id)
        if sid is None:
            return None, False
        return self.get_activity_info(sid)

    def get_pending_timer_infos(self) -> Dict[str, TimerInfo]:
        return self.pending_timer_info_ids

    def get_user_timer_info(self, timer_id: str) -> Tuple[Optional[TimerInfo], bool]:
        ti = self.pending_timer_info_ids.get(timer_id)
        return ti, ti is not None

    def get_user_timer_info_by_event_id(self, started_id: int) -> Tuple[Optional[TimerInfo], bool]:
        tid = self.pending_timer_event_id_to_id.get(started_id)
        return (None, False) if tid is None else self.get_user_timer_info(tid)

    def get_pending_child_execution_infos(self) -> Dict[int, ChildExecutionInfo]:
        return self.pending_child_execution_info_ids

    def get_child_execution_info(self, initiated_id: int) -> Tuple[Optional[ChildExecutionInfo], bool]:
        ci = self.pending_child_execution_info_ids.get(initiated_id)
        return ci, ci is not None

    def get_pending_request_cancel_external_infos(self) -> Dict[int, RequestCancelInfo]:
        return self.pending_request_cancel_info_ids

    def get_pending_signal_external_infos(self) -> Dict[int, SignalInfo]:
        return self.pending_signal_info_ids

    def has_pending_decision(self) -> bool:
        return self.execution_info.decision_schedule_id != abi.EMPTY_EVENT_ID

    def has_in_flight_decision(self) -> bool:
        return self.execution_info.decision_started_id > 0

    def get_checksum(self) -> Optional[Checksum]:
        return self.checksum

    def get_transfer_tasks(self) -> List[Task]:  # mutable_state.go:226
        return self.transfer_tasks

    def get_timer_tasks(self) -> List[Task]:  # mutable_state.go:228
        return self.timer_tasks


# ---- the batched engine ---------------------------------------------------------------------------------
@dataclasses.dataclass
class _LoadedImage:
    """A replayed state as the engine reloads it: its exec row and live rows (abi row images), the
    workflow's key interner, and the events every provenance step of those rows refers to."""
    history: WorkflowHistory          # identity (IDs, branch) of the workflow
    events: List[HistoryEvent]        # every event applied so far (provenance steps index this list)
    exec_row: np.ndarray              # abi.EXEC_ROW [1]
    rows: Dict[str, np.ndarray]       # table -> live rows
    interner: Dict[str, int]


@dataclasses.dataclass
class ReplayOutcome:
    """What ApplyEvents returns for one workflow: its state, its error, and for a continue-as-new
    the new run's state (state_builder.go:587-627)."""
    mutable_state: MutableState
    error: Optional[CadenceError]
    new_run_mutable_state: Optional[MutableState] = None


def _default_uuid(run_id: str, kind: str, step: int) -> str:
    return det_uuid(run_id, kind, step)


class BatchStateBuilder:
    """Replays many workflows in one ``crr_replay`` (one MI355X) and materialises their states.

    ``known_domains`` / ``domain_ids``: the domain cache (name -> ID); a name missing from it makes
    the lookup fail with EntityNotExists at the same event as in Go.
    """

    def __init__(self, engine=None, domain_ids: Optional[Dict[str, str]] = None,
                 uuid_fn: Callable[[str, str, int], str] = _default_uuid, layout: str = "interleaved",
                 emit_tasks: bool = True):
        self.engine = engine          # None: a ReplayEngine on device 0, created at the first replay
        self.domain_ids = domain_ids
        self.uuid_fn = uuid_fn
        self.layout = layout
        self.emit_tasks = emit_tasks       # generate the transfer / timer tasks (CRR_IN_EMIT_TASKS)
        self.histories: List[WorkflowHistory] = []
        self.loaded: List[Optional[_LoadedImage]] = []
        self._outcomes: Optional[List[ReplayOutcome]] = None

    def add(self, history: WorkflowHistory, loaded: Optional[_LoadedImage] = None) -> int:
        """Stage a workflow; ``loaded``: its batches apply onto this loaded state (CRR_WF_FLAG_RESUME)."""
        self.histories.append(history)
        self.loaded.append(loaded)
        self._outcomes = None
        return len(self.histories) - 1

    def __len__(self):
        return len(self.histories)

    def invalidate(self):
        """A staged history changed: the next ``outcomes()`` replays again."""
        self._outcomes = None

    def outcomes(self) -> List[ReplayOutcome]:
        """The outcomes of the last replay, replaying first if anything was staged since."""
        if self._outcomes is None:
            self._outcomes = self.replay()
        return self._outcomes

    def replay(self) -> List[ReplayOutcome]:
        """One device replay of every staged workflow (canonical order of ``add``)."""
        known = None if self.domain_ids is None else set(self.domain_ids)
        loaded = _loaded_states(self.loaded)
        canon = flatten(self.histories, known_domains=known, loaded=loaded)
        canon.emit_tasks = self.emit_tasks
        batch = interleave(canon) if self.layout == "interleaved" else canon
        if self.engine is None:
            from .engine import ReplayEngine   # raises EngineUnavailable without the HIP library / a GPU
            self.engine = ReplayEngine(0)
        res = self.engine.replay(batch)
        # a loaded workflow's provenance steps count from its first event ever (crr_exec_row.src_next)
        all_events = [(li.events if li is not None else []) + h.events for h, li in zip(self.histories, self.loaded)]
        states = materialise(self.histories, batch, res, self.domain_ids, self.uuid_fn, all_events)
        images = res.to_loaded(batch)
        for w, h in enumerate(self.histories):
            if images.mask[w]:
                states[w][0]._loaded = _image(images, w, self.loaded[w].history if self.loaded[w] else h, all_events[w])
        out = []
        for w, h in enumerate(self.histories):
            ms, st, step = states[w]
            nr = None
            for e in h.events:
                if e.event_type == ET.WorkflowExecutionContinuedAsNew and e.attrs.get("new_run") is not None:
                    nr = states[int(e.attrs["new_run"])][0]
            out.append(ReplayOutcome(ms, status_error(st, step), nr))
        self._outcomes = out
        return out


def _loaded_states(images: Sequence[Optional[_LoadedImage]]) -> Optional[LoadedStates]:
    """The batch's loaded states (flatten's ``loaded``), or None when every workflow starts fresh."""
    if all(li is None for li in images):
        return None
    n = len(images)
    ex = np.zeros(n, abi.EXEC_ROW)
    mask = np.zeros(n, bool)
    rows = {name: [] for name, *_ in abi.TABLES if name != "tasks"}
    its = []
    for w, li in enumerate(images):
        its.append(dict(li.interner) if li is not None else None)
        if li is None:
            continue
        ex[w] = li.exec_row
        mask[w] = True
        for name in rows:
            rows[name].append(li.rows[name])
    cat = {}
    for name, dt, *_r in abi.TABLES:
        if name != "tasks":
            cat[name] = np.concatenate(rows[name]) if rows[name] else np.zeros(0, dt)
    return LoadedStates(ex, cat, mask, its)


def _image(images: LoadedStates, w: int, history: WorkflowHistory, events: List[HistoryEvent]) -> _LoadedImage:
    rows = {}
    for name, *_r in abi.TABLES:
        if name == "tasks":
            continue
        c = images.counts(name)
        off = int(c[:w].sum())
        rows[name] = images.rows[name][off:off + int(c[w])].copy()
    return _LoadedImage(history, list(events), images.exec[w:w + 1].copy(), rows,
                        dict(images.interners[w]) if images.interners is not None else {"": 0})


def _attr(e: HistoryEvent, name, default=None):
    return e.get(name, default)


def materialise(histories: Sequence[WorkflowHistory], batch: HistoryBatch, res, domain_ids=None,
                uuid_fn: Callable[[str, str, int], str] = _default_uuid, events=None):
    """Device rows -> one MutableState per workflow (canonical order): [(state, status, fail_step)].
    ``events[w]``: the events workflow w's provenance steps index (default: its history's events)."""
    n = len(histories)
    dev_of = np.arange(n) if batch.perm is None else np.argsort(batch.perm, kind="stable")
    strides = batch.wf_strides()
    out = []
    for w, h in enumerate(histories):
        d = int(dev_of[w])
        ex = res.exec[d]
        wfr = batch.wf[d]
        evs = h.events if events is None else events[w]
        rows = {}
        for name, _dt, base_f, cap_f, n_f in abi.TABLES:
            k = min(int(ex[n_f]), int(wfr[cap_f]))
            idx = int(wfr[base_f]) + np.arange(max(k, 0), dtype=np.int64) * int(strides[d])
            rows[name] = res.tables[name][idx]
        out.append((_materialise_one(h, evs, ex, rows, domain_ids, uuid_fn), int(ex["status"]), int(ex["fail_step"])))
    return out


def _domain_id(name: str, own: str, domain_ids) -> str:
    if not name:
        return own
    if domain_ids is None:
        return name
    return domain_ids.get(name, "")


def _materialise_one(h: WorkflowHistory, events: List[HistoryEvent], ex, rows, domain_ids, uuid_fn) -> MutableState:
    ms = MutableState()
    own_domain = h.domain_id
    ev = lambda s: events[s] if 0 <= s < len(events) else None  # noqa: E731
    start = ev(int(ex["start_src"]))
    dreq = int(ex["decision_request_src"])
    rps = None
    if int(ex["flags"]) & abi.EXEC_RESET_POINTS_SET:
        rps = []
        for r in rows["rp"]:
            src = ev(int(r["src"]))
            if int(r["prev_index"]) >= 0:
                p = (src.attrs.get("prev_auto_reset_points") or [])[int(r["prev_index"])]
                rps.append(ResetPointInfo(str(p), "", 0, 0, bool(int(r["flags"]) & abi.ROW_RESETTABLE), True))
            else:
                rps.append(ResetPointInfo(str(src.get("binary_checksum", "")), h.run_id,
                                          src.id, h.now_ns, bool(int(r["flags"]) & abi.ROW_RESETTABLE), False))
    ms.execution_info = WorkflowExecutionInfo(
        domain_id=own_domain, workflow_id=h.workflow_id, run_id=h.run_id,
        state=int(ex["state"]), close_status=int(ex["close_status"]),
        next_event_id=int(ex["next_event_id"]), last_first_event_id=int(ex["last_first_event_id"]),
        last_event_task_id=int(ex["last_event_task_id"]), last_processed_event=int(ex["last_processed_event"]),
        completion_event_batch_id=int(ex["completion_event_batch_id"]), signal_count=int(ex["signal_count"]),
        cancel_requested=bool(int(ex["flags"]) & abi.EXEC_CANCEL_REQUESTED),
        decision_version=int(ex["decision_version"]), decision_schedule_id=int(ex["decision_schedule_id"]),
        decision_started_id=int(ex["decision_started_id"]),
        decision_request_id=EMPTY_UUID if dreq == abi.SRC_EMPTY_UUID else str(ev(dreq).get("request_id", "")),
        decision_timeout=int(ex["decision_timeout"]), decision_attempt=int(ex["decision_attempt"]),
        decision_started_timestamp=int(ex["decision_started_ts"]),
        decision_scheduled_timestamp=int(ex["decision_scheduled_ts"]),
        decision_original_scheduled_timestamp=int(ex["decision_orig_scheduled_ts"]),
        start_timestamp=None if start is None else start.timestamp,
        auto_reset_points=rps)
    ms.current_version = int(ex["current_version"])
    ms.inconsistencies = int(ex["inconsistencies"])
    for r in rows["act"]:
        sched = ev(int(r["sched_src"]))
        started = ev(int(r["started_src"]))
        ai = ActivityInfo(
            version=int(r["version"]), schedule_id=int(r["schedule_id"]),
            scheduled_event_batch_id=int(r["scheduled_batch_id"]), scheduled_time=int(r["scheduled_time"]),
            started_id=int(r["started_id"]), started_time=_time(r["started_time"]),
            activity_id=str(sched.get("activity_id", "")),
            request_id="" if started is None else str(started.get("request_id", "")),
            domain_id=_domain_id(sched.get("domain", ""), own_domain, domain_ids),
            schedule_to_start_timeout=int(r["schedule_to_start"]), schedule_to_close_timeout=int(r["schedule_to_close"]),
            start_to_close_timeout=int(r["start_to_close"]), heartbeat_timeout=int(r["heartbeat"]),
            cancel_requested=bool(int(r["flags"]) & abi.ROW_CANCEL_REQUESTED),
            cancel_request_id=int(r["cancel_request_id"]),
            last_heartbeat_updated_time=_time(r["started_time"]),
            timer_task_status=int(r["timer_task_status"]), task_list=str(sched.get("task_list", "")),
            has_retry_policy=bool(int(r["flags"]) & abi.ROW_HAS_RETRY),
            last_heartbeat_timeout_visibility_in_seconds=int(r["last_hb_timeout_vis_s"]))
        ms.pending_activity_info_ids[ai.schedule_id] = ai
        if int(r["flags"]) & abi.ROW_MAPPED:
            ms.pending_activity_id_to_event_id[ai.activity_id] = ai.schedule_id
    for r in rows["timer"]:
        src = ev(int(r["src"]))
        ti = TimerInfo(version=int(r["version"]), timer_id=str(src.get("timer_id", "")),
                       started_id=int(r["started_id"]), expiry_time=int(r["expiry_time"]),
                       task_status=int(r["task_status"]))
        ms.pending_timer_info_ids[ti.timer_id] = ti
        ms.pending_timer_event_id_to_id[ti.started_id] = ti.timer_id
    for r in rows["child"]:
        src = ev(int(r["src"]))
        st = ev(int(r["started_src"]))
        wt = src.get("workflow_type", "")
        ci = ChildExecutionInfo(
            version=int(r["version"]), initiated_id=int(r["initiated_id"]),
            initiated_event_batch_id=int(r["initiated_batch_id"]), started_id=int(r["started_id"]),
            started_workflow_id=str(src.get("workflow_id", "")),
            started_run_id="" if st is None else str(st.get("run_id", "")),
            create_request_id=uuid_fn(h.run_id, "child", int(r["src"])),
            domain_id=_domain_id(src.get("domain", ""), own_domain, domain_ids),
            workflow_type_name=str(wt.get("name", "") if isinstance(wt, dict) else wt),
            parent_close_policy=int(src.get("parent_close_policy", 0)))
        ms.pending_child_execution_info_ids[ci.initiated_id] = ci
    for r in rows["rc"]:
        ri = RequestCancelInfo(version=int(r["version"]), initiated_event_batch_id=int(r["initiated_batch_id"]),
                               initiated_id=int(r["initiated_id"]),
                               cancel_request_id=uuid_fn(h.run_id, "cancel", int(r["src"])))
        ms.pending_request_cancel_info_ids[ri.initiated_id] = ri
    for r in rows["sig"]:
        src = ev(int(r["src"]))
        si = SignalInfo(version=int(r["version"]), initiated_event_batch_id=int(r["initiated_batch_id"]),
                        initiated_id=int(r["initiated_id"]), signal_request_id=uuid_fn(h.run_id, "signal", int(r["src"])),
                        signal_name=str(src.get("signal_name", "")), input=bytes(src.get("input", b"") or b""),
                        control=bytes(src.get("control", b"") or b""))
        ms.pending_signal_info_ids[si.initiated_id] = si
    token_src = int(ex["token_src"])
    token = b""
    if token_src == 1:
        token = thrift_history_branch_token(h.run_id, h.branch_id)
    elif token_src == 2:
        token = h.final_token
    items = [VersionHistoryItem(int(r["event_id"]), int(r["version"])) for r in rows["vh"]]
    ms.version_histories = VersionHistories(0, [VersionHistory(token, items)])
    for r in rows.get("tasks", ()):
        src = ev(int(r["src"]))
        kind = abi.TaskKind(int(r["kind"]))
        task = Task(kind=kind, version=int(r["version"]), visibility_timestamp=int(r["visibility_ts"]),
                    event_id=int(r["event_id"]), timeout_type=int(r["aux"]), attempt=int(r["attempt"]))
        if src is not None:
            if kind in (abi.TaskKind.Decision, abi.TaskKind.Activity):
                task.task_list = str(src.get("task_list", ""))
            elif kind in (abi.TaskKind.StartChild, abi.TaskKind.CancelExecution, abi.TaskKind.SignalExecution):
                task.target_domain = _domain_id(src.get("domain", ""), own_domain, domain_ids)
                task.target_workflow_id = str(src.get("workflow_id", ""))
        (ms.transfer_tasks if kind in TRANSFER_KINDS else ms.timer_tasks).append(task)
    if int(ex["flags"]) & abi.EXEC_CHECKSUM_VALID:
        ms.checksum = Checksum(version=1, flavor=1, value=int(ex["checksum"]).to_bytes(4, "big"))
    return ms


# ---- StateBuilder / StateRebuilder (state_builder.go:41-51, state_rebuilder.go:97-191) -----------------
class StateBuilder:
    """``execution.StateBuilder`` for one workflow over a :class:`BatchStateBuilder`.

    ``NewStateBuilder(shard, logger, mutableState)`` (state_builder.go:73-88): ``mutable_state`` is the
    state the events apply onto -- None for a fresh ``NewMutableStateBuilderWithVersionHistories``
    (rebuild, start-event replication), or a state a previous replay returned, i.e. what
    ``mutableStateBuilder.Load`` reads back (the passive-replication path, ndc/history_replicator.go:
    385-460): its rows are reloaded into the engine (CRR_WF_FLAG_RESUME) and only the new batches replay.

    ``apply_events`` stages a batch (the ``history`` argument of one Go ``ApplyEvents`` call); the
    device replay runs when the state is read (``get_mutable_state``) or the batch builder
    flushes, so many workflows share one launch.  Deviation from Go, by design: Go's
    ``ApplyEvents`` returns ``(MutableState, error)`` per call (state_builder.go:90-97); here the
    call returns None and the error of the first failing event of any staged call is raised by
    ``get_mutable_state`` -- the outcome is the same because replay stops at the first error in both
    (the caller aborts on it, state_rebuilder.go:221), but it surfaces at the read, not at the call.
    An empty ``history`` raises at once, as Go returns before touching state.
    """

    def __init__(self, domain_failover_version: int = 0, domain_id: str = "domain-id", workflow_id: str = "workflow-id",
                 run_id: str = "run-id", branch_id: str = "branch-id", now_ns: int = 0,
                 batch_builder: Optional[BatchStateBuilder] = None, mutable_state: Optional[MutableState] = None):
        self._bb = batch_builder if batch_builder is not None else BatchStateBuilder()
        loaded = None
        if mutable_state is not None:
            loaded = mutable_state._loaded
            if loaded is None:
                raise InternalServiceError("mutable state was not produced by a replay: no row image to load")
            o = loaded.history
            domain_id, workflow_id, run_id, branch_id = o.domain_id, o.workflow_id, o.run_id, o.branch_id
            domain_failover_version = o.domain_failover_version
        self._h = WorkflowHistory(batches=[], domain_id=domain_id, domain_failover_version=domain_failover_version,
                                  workflow_id=workflow_id, run_id=run_id, branch_id=branch_id, now_ns=now_ns)
        self._w = self._bb.add(self._h, loaded)   # staged now: every StateBuilder of a batch shares one replay
        self._new_run_w: Optional[int] = None

    def apply_events(self, domain_id: str, request_id: str, workflow_execution: Dict[str, str],
                     history: List[HistoryEvent], new_run_history: Optional[List[HistoryEvent]] = None):
        if not history:  # state_builder.go:98-100
            raise InternalFailureError("encounter history size being zero", status=int(Status.EMPTY_HISTORY))
        self._bb.invalidate()
        self._h.request_id = request_id
        if workflow_execution:
            self._h.workflow_id = workflow_execution.get("workflow_id", self._h.workflow_id)
            self._h.run_id = workflow_execution.get("run_id", self._h.run_id)
        self._h.batches.append(list(history))
        if new_run_history:
            # state_builder.go:587-627: the new run's ID is the CAN event's NewExecutionRunID
            can = [e for e in history if e.event_type == ET.WorkflowExecutionContinuedAsNew]
            new_run_id = can[-1].get("new_execution_run_id", self._h.run_id + "-new") if can else self._h.run_id + "-new"
            nr = WorkflowHistory(batches=[list(new_run_history)], domain_id=self._h.domain_id,
                                 domain_failover_version=self._h.domain_failover_version,
                                 workflow_id=self._h.workflow_id, run_id=str(new_run_id),
                                 branch_id=self._h.branch_id + "-new", now_ns=self._h.now_ns, is_new_run=True)
            self._new_run_w = self._bb.add(nr)
            for e in can:
                e.attrs["new_run"] = self._new_run_w
        return None

    def set_rebuild_target(self, token: bytes, last_event_id: int, last_event_version: int, refresh_tasks: bool = True):
        """Rebuild finalisation: SetCurrentBranchToken(token), the last-item check and (by default)
        RefreshTasks' timer-status re-selection (state_rebuilder.go:150-183)."""
        self._bb.invalidate()
        self._h.refresh_tasks = refresh_tasks
        self._h.final_token = token
        self._h.rebuild_last_event_id = last_event_id
        self._h.rebuild_last_event_version = last_event_version

    def _outcome(self) -> ReplayOutcome:
        return self._bb.outcomes()[self._w]

    def get_mutable_state(self) -> MutableState:
        o = self._outcome()
        if o.error is not None:
            raise o.error
        return o.mutable_state

    def get_new_run_mutable_state(self) -> Optional[MutableState]:
        return self._outcome().new_run_mutable_state


def rebuild(batches: Sequence[List[HistoryEvent]], target_branch_token: bytes, base_last_event_id: int,
            base_last_event_version: int, request_id: str, domain_failover_version: int = 0,
            domain_id: str = "domain-id", workflow_id: str = "workflow-id", run_id: str = "run-id",
            now_ns: int = 0, batch_builder: Optional[BatchStateBuilder] = None,
            history_sizes: Sequence[int] = ()) -> Tuple[MutableState, int]:
    """``stateRebuilderImpl.Rebuild`` (state_rebuilder.go:97-191) over one workflow's persisted
    batches: replay, ``SetCurrentBranchToken(target)``, the last-item check, ``StartTimestamp = now``.
    Returns (state, rebuilt history size = sum of the pages' blob sizes, ``history_sizes``).
    RefreshTasks' state effect -- every pending activity's / user timer's timer-task status cleared
    and the next timer of each sequence re-created -- is applied on the device
    (CRR_WF_FLAG_REFRESH_TASKS); the transfer / timer tasks it emits are not."""
    sb = StateBuilder(domain_failover_version, domain_id, workflow_id, run_id, now_ns=now_ns,
                      batch_builder=batch_builder)
    for b in batches:
        sb.apply_events(domain_id, request_id, {"workflow_id": workflow_id, "run_id": run_id}, b)
    sb.set_rebuild_target(target_branch_token, base_last_event_id, base_last_event_version)
    ms = sb.get_mutable_state()
    ms.execution_info.start_timestamp = now_ns  # state_rebuilder.go:189
    return ms, int(sum(history_sizes))
