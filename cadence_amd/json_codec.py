"""JSON-encoded history batches: serializer.SerializeBatchEvents with common.EncodingTypeJSON
(common/persistence/serializer.go:104-106, json.Marshal of []*types.HistoryEvent) for the fields the
replay reads -- the common/types JSON tags (common/types/shared.go:3662-3710 and the *EventAttributes
structs), enums by name (EventType / TimeoutType / ContinueAsNewInitiator MarshalText).  The native
decoder reads these blobs with CRR_ENCODING_JSON (cadence_amd/csrc/json_decode.cpp)."""
from __future__ import annotations

import json
from typing import Dict, List

from .abi import EventType as ET
from .history import HistoryEvent, WorkflowHistory

TIMEOUT_NAMES = ["START_TO_CLOSE", "SCHEDULE_TO_START", "SCHEDULE_TO_CLOSE", "HEARTBEAT"]
INITIATOR_NAMES = ["Decider", "RetryPolicy", "CronSchedule"]

_SCHED = (ET.ActivityTaskStarted, ET.ActivityTaskCompleted, ET.ActivityTaskFailed, ET.ActivityTaskTimedOut,
          ET.ActivityTaskCanceled)
_INIT = (ET.StartChildWorkflowExecutionFailed, ET.ChildWorkflowExecutionStarted, ET.ChildWorkflowExecutionCompleted,
         ET.ChildWorkflowExecutionFailed, ET.ChildWorkflowExecutionCanceled, ET.ChildWorkflowExecutionTimedOut,
         ET.ChildWorkflowExecutionTerminated, ET.RequestCancelExternalWorkflowExecutionFailed,
         ET.ExternalWorkflowExecutionCancelRequested, ET.SignalExternalWorkflowExecutionFailed,
         ET.ExternalWorkflowExecutionSignaled)


def attributes_key(t: int) -> str:
    n = ET(t).name
    return n[0].lower() + n[1:] + "EventAttributes"


def attributes_json(e: HistoryEvent) -> Dict:
    t, a, g = e.event_type, e.attrs, e.get
    o: Dict = {}
    if t == ET.WorkflowExecutionStarted:
        o["workflowType"] = {"name": "workflow-type"}
        if a.get("parent_workflow_domain_id") is not None:
            o["parentWorkflowDomainID"] = a["parent_workflow_domain_id"]
        if g("parent_workflow_domain", ""):
            o["parentWorkflowDomain"] = g("parent_workflow_domain")
        o["executionStartToCloseTimeoutSeconds"] = g("execution_start_to_close_timeout_seconds", 0)
        o["taskStartToCloseTimeoutSeconds"] = g("task_start_to_close_timeout_seconds", 0)
        if a.get("initiator") is not None:
            o["initiator"] = INITIATOR_NAMES[a["initiator"]] if 0 <= a["initiator"] < 3 else str(a["initiator"])
        if g("attempt", 0):
            o["attempt"] = g("attempt")
        if g("expiration_timestamp", 0):
            o["expirationTimestamp"] = g("expiration_timestamp")
        o["firstDecisionTaskBackoffSeconds"] = g("first_decision_task_backoff_seconds", 0)
        prev = a.get("prev_auto_reset_points")
        if prev == "nil_points":
            o["prevAutoResetPoints"] = {}
        elif prev is not None:
            o["prevAutoResetPoints"] = {"points": [{"binaryChecksum": p} for p in prev]}
    elif t == ET.DecisionTaskScheduled:
        o = {"taskList": {"name": "decision-tl"}, "startToCloseTimeoutSeconds": g("start_to_close_timeout_seconds", 0),
             "attempt": g("attempt", 0)}
    elif t == ET.DecisionTaskStarted:
        o = {"scheduledEventId": g("scheduled_event_id", 0), "requestId": g("request_id", "")}
    elif t == ET.DecisionTaskCompleted:
        o = {"scheduledEventId": g("scheduled_event_id", 0), "startedEventId": g("started_event_id", 0)}
        if g("binary_checksum", ""):
            o["binaryChecksum"] = g("binary_checksum")
    elif t == ET.DecisionTaskTimedOut:
        o = {"timeoutType": TIMEOUT_NAMES[g("timeout_type", 0)]}
    elif t == ET.ActivityTaskScheduled:
        o = {"activityId": g("activity_id", ""), "activityType": {"name": "activity-type"},
             "taskList": {"name": g("task_list", "activity-tl")},
             "scheduleToCloseTimeoutSeconds": g("schedule_to_close_timeout_seconds", 0),
             "scheduleToStartTimeoutSeconds": g("schedule_to_start_timeout_seconds", 0),
             "startToCloseTimeoutSeconds": g("start_to_close_timeout_seconds", 0),
             "heartbeatTimeoutSeconds": g("heartbeat_timeout_seconds", 0)}
        if g("domain", ""):
            o["domain"] = g("domain")
        rp = a.get("retry_policy")
        if rp is not None:
            o["retryPolicy"] = {"expirationIntervalInSeconds": rp.get("expiration_interval_in_seconds", 0)
                                if isinstance(rp, dict) else 0}
    elif t in _SCHED:
        o = {"scheduledEventId": g("scheduled_event_id", 0)}
    elif t == ET.ActivityTaskCancelRequested:
        o = {"activityId": g("activity_id", "")}
    elif t == ET.TimerStarted:
        o = {"timerId": g("timer_id", ""), "startToFireTimeoutSeconds": g("start_to_fire_timeout_seconds", 0)}
    elif t in (ET.TimerFired, ET.TimerCanceled):
        o = {"timerId": g("timer_id", "")}
    elif t in (ET.StartChildWorkflowExecutionInitiated, ET.RequestCancelExternalWorkflowExecutionInitiated,
               ET.SignalExternalWorkflowExecutionInitiated):
        if g("domain", ""):
            o["domain"] = g("domain")
    elif t in _INIT:
        o = {"initiatedEventId": g("initiated_event_id", 0)}
    elif t == ET.WorkflowExecutionContinuedAsNew:
        o = {"newExecutionRunId": str(g("new_execution_run_id", "new-run"))}
    return o


def event_json(e: HistoryEvent) -> Dict:
    known = e.event_type in ET._value2member_map_
    # an out-of-range type is written as its decimal text in a JSON string (UnmarshalText's
    # strconv.ParseInt fallback reads it back; Go's MarshalText would write "EventType(n)", which its
    # own UnmarshalText rejects)
    d = {"eventId": e.id, "timestamp": e.timestamp, "eventType": ET(e.event_type).name if known else str(int(e.event_type)),
         "version": e.version, "taskId": e.task_id}
    if known:
        d[attributes_key(e.event_type)] = attributes_json(e)
    return d


def serialize_batch_events_json(events: List[HistoryEvent]) -> bytes:
    return json.dumps([event_json(e) for e in events], separators=(",", ":")).encode()


def serialize_history_json(h: WorkflowHistory) -> List[bytes]:
    return [serialize_batch_events_json(b) if b else b"" for b in h.batches]
