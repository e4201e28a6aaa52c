"""Host-side history model: the subset of ``types.HistoryEvent`` the replay path reads.

Mirrors ``common/types/shared.go:3662-3710`` (HistoryEvent) and the per-type attribute getters the
state builder calls (``service/history/execution/state_builder.go:131-631``).  Attribute names are
the Go field names in snake_case.  This is the representation a caller hands to
``StateBuilder.apply_events`` / ``flatten()``; the engine itself only ever sees flattened columns.
"""
from __future__ import annotations

import base64
import dataclasses
import json
import uuid
from typing import Dict, List, Optional

from .abi import EventType


@dataclasses.dataclass
class HistoryEvent:
    event_type: int
    id: int
    version: int = 0
    timestamp: int = 0
    task_id: int = 0
    attrs: Dict = dataclasses.field(default_factory=dict)

    def get(self, name, default=None):
        v = self.attrs.get(name, default)
        return default if v is None else v


@dataclasses.dataclass
class WorkflowHistory:
    """One workflow to replay: persisted event batches plus the host-injected inputs.

    ``batches`` are the ``history`` arguments of successive ApplyEvents calls
    (state_rebuilder.go:135-148).  An empty inner list reproduces ApplyEvents' empty-history
    error (state_builder.go:98-100).
    """
    batches: List[List[HistoryEvent]]
    domain_id: str = "domain-id"
    domain_failover_version: int = 0          # initial currentVersion (mutable_state_builder.go:207)
    workflow_id: str = "workflow-id"
    run_id: str = "run-id"
    request_id: str = "request-id"            # ApplyEvents requestID -> CreateRequestID
    branch_id: str = "branch-id"              # injected uuid for NewHistoryBranchToken
    now_ns: int = 0                           # injected timeSource.Now()
    final_token: Optional[bytes] = None       # rebuild target branch token (state_rebuilder.go:150)
    rebuild_last_event_id: int = 0
    rebuild_last_event_version: int = 0
    is_new_run: bool = False                  # CAN newRunHistory replayed by the outer workflow
    refresh_tasks: bool = False               # Rebuild: RefreshTasks after the replay (state_rebuilder.go:183)
    refresh_jitter: int = 0                   # injected rand draw for RefreshTasks' decision backoff jitter
    retention_days: int = 1                   # domain retention (defaultWorkflowRetentionInDays = 1 when unknown)

    @property
    def events(self) -> List[HistoryEvent]:
        return [e for b in self.batches for e in b]


def thrift_history_branch_token(tree_id: str, branch_id: str) -> bytes:
    """NewHistoryBranchTokenByBranchID (common/persistence/dataManagerInterfaces.go:2899-2910).

    0x59 preamble + thrift binary HistoryBranch{10: TreeID, 20: BranchID, 30: Ancestors=[]}.
    """
    t = tree_id.encode()
    b = branch_id.encode()
    out = bytearray(b"\x59")
    out += b"\x0b\x00\x0a" + len(t).to_bytes(4, "big") + t
    out += b"\x0b\x00\x14" + len(b).to_bytes(4, "big") + b
    out += b"\x0f\x00\x1e\x0c" + (0).to_bytes(4, "big")
    out += b"\x00"
    return bytes(out)


def det_uuid(*parts) -> str:
    """Deterministic stand-in for uuid.New() (the reference's non-deterministic inputs are injected)."""
    return str(uuid.uuid5(uuid.NAMESPACE_URL, "/".join(str(p) for p in parts)))


# ---- Cadence JSON history (archiver testdata format) ------------------------------------------------
_JSON_ATTR = {
    "workflowExecutionStartedEventAttributes": {
        "taskStartToCloseTimeoutSeconds": "task_start_to_close_timeout_seconds",
        "executionStartToCloseTimeoutSeconds": "execution_start_to_close_timeout_seconds",
        "firstDecisionTaskBackoffSeconds": "first_decision_task_backoff_seconds",
        "initiator": "initiator", "parentWorkflowDomain": "parent_workflow_domain",
        "parentWorkflowDomainId": "parent_workflow_domain_id", "attempt": "attempt",
        "cronSchedule": "cron_schedule", "continuedExecutionRunId": "continued_execution_run_id",
        "expirationTimestamp": "expiration_timestamp", "prevAutoResetPoints": "prev_auto_reset_points",
    },
    "decisionTaskScheduledEventAttributes": {"startToCloseTimeoutSeconds": "start_to_close_timeout_seconds",
                                             "attempt": "attempt"},
    "decisionTaskStartedEventAttributes": {"scheduledEventId": "scheduled_event_id", "requestId": "request_id"},
    "decisionTaskCompletedEventAttributes": {"scheduledEventId": "scheduled_event_id",
                                             "startedEventId": "started_event_id",
                                             "binaryChecksum": "binary_checksum"},
    "decisionTaskTimedOutEventAttributes": {"timeoutType": "timeout_type"},
    "activityTaskScheduledEventAttributes": {
        "activityId": "activity_id", "domain": "domain",
        "scheduleToStartTimeoutSeconds": "schedule_to_start_timeout_seconds",
        "scheduleToCloseTimeoutSeconds": "schedule_to_close_timeout_seconds",
        "startToCloseTimeoutSeconds": "start_to_close_timeout_seconds",
        "heartbeatTimeoutSeconds": "heartbeat_timeout_seconds", "retryPolicy": "retry_policy"},
    "activityTaskStartedEventAttributes": {"scheduledEventId": "scheduled_event_id", "requestId": "request_id"},
    "activityTaskCompletedEventAttributes": {"scheduledEventId": "scheduled_event_id"},
    "activityTaskFailedEventAttributes": {"scheduledEventId": "scheduled_event_id"},
    "activityTaskTimedOutEventAttributes": {"scheduledEventId": "scheduled_event_id"},
    "activityTaskCanceledEventAttributes": {"scheduledEventId": "scheduled_event_id"},
    "activityTaskCancelRequestedEventAttributes": {"activityId": "activity_id"},
    "timerStartedEventAttributes": {"timerId": "timer_id", "startToFireTimeoutSeconds": "start_to_fire_timeout_seconds"},
    "timerFiredEventAttributes": {"timerId": "timer_id"},
    "timerCanceledEventAttributes": {"timerId": "timer_id"},
}

_TIMEOUT_NAMES = {"START_TO_CLOSE": 0, "SCHEDULE_TO_START": 1, "SCHEDULE_TO_CLOSE": 2, "HEARTBEAT": 3}


def load_json_history(path: str) -> List[HistoryEvent]:
    """Parse a Cadence JSON history (e.g. service/worker/archiver/testdata/*.json)."""
    with open(path) as f:
        raw = json.load(f)
    return events_from_json(raw)


def events_from_json(raw) -> List[HistoryEvent]:
    out = []
    for e in raw:
        et = EventType[e["eventType"]]
        attrs = {}
        for k, v in e.items():
            if not k.endswith("EventAttributes"):
                continue
            mapping = _JSON_ATTR.get(k, {})
            for jk, jv in v.items():
                name = mapping.get(jk)
                if name is None:
                    continue
                if name == "timeout_type" and isinstance(jv, str):
                    jv = _TIMEOUT_NAMES[jv]
                if name == "retry_policy" and isinstance(jv, dict):     # RetryPolicy{expirationIntervalInSeconds}
                    jv = {"expiration_interval_in_seconds": jv.get("expirationIntervalInSeconds", 0)}
                if name == "prev_auto_reset_points" and jv is not None:  # ResetPoints{points: [{binaryChecksum}]}
                    pts = jv.get("points")
                    jv = "nil_points" if pts is None else [(p or {}).get("binaryChecksum", "") for p in pts]
                attrs[name] = jv
            if k == "workflowExecutionStartedEventAttributes":
                attrs.setdefault("prev_auto_reset_points", None)
        out.append(HistoryEvent(int(et), int(e["eventId"]), int(e.get("version", 0)), int(e.get("timestamp", 0)),
                                int(e.get("taskId", 0)), attrs))
    return out


def split_batches_by_task_id(events: List[HistoryEvent]) -> List[List[HistoryEvent]]:
    """Recover persisted batches from a flat JSON history: events written in one transaction get
    consecutive task IDs (mutable_state_builder.go:736-774 assignTaskIDToEvents), so a gap in
    TaskID starts a new batch.  Used for archived histories that carry no batch boundaries."""
    batches: List[List[HistoryEvent]] = []
    prev = None
    for e in events:
        if prev is None or e.task_id != prev + 1:
            batches.append([])
        batches[-1].append(e)
        prev = e.task_id
    return batches


def branch_token_from_archival_signal(events: List[HistoryEvent], raw_json_path: str) -> bytes:
    """The archival fixture embeds a real branch token (base64) inside its first signal input."""
    with open(raw_json_path) as f:
        raw = json.load(f)
    for e in raw:
        attrs = e.get("workflowExecutionSignaledEventAttributes")
        if attrs and attrs.get("input"):
            payload = json.loads(base64.b64decode(attrs["input"]))
            if "BranchToken" in payload:
                return base64.b64decode(payload["BranchToken"])
    raise ValueError("no branch token found")
