"""thriftrw encoding of persisted history batches (the writer side of the blobs the decoder reads).

Restates ``serializerImpl.SerializeBatchEvents`` (``common/persistence/serializer.go:105-107``) for
the replay path: ``codec.ThriftRWEncoder.Encode`` (``common/codec/version0Thriftrw.go:44-61``) writes
the 0x59 preamble then the thrift binary encoding of ``shared.History{10: list<HistoryEvent>}``;
go.uber.org/thriftrw (v1.29.2, not vendored) writes a struct's set fields in ascending field-id
order and omits nil ones.  Field ids are those of ``.gen/go/shared/shared.go`` (HistoryEvent and
the *EventAttributes structs).  Used to build synthetic persisted histories for the decoder's tests
and benchmarks; the fields ApplyEvents never reads are still written (identity, inputs, task lists,
headers) so the decoder's skipping is exercised on realistic blobs.
"""
from __future__ import annotations

import random
import struct
from typing import Dict, List, Optional

from .abi import EventType as ET
from .history import HistoryEvent, WorkflowHistory

T_BOOL, T_BYTE, T_DOUBLE, T_I16, T_I32, T_I64, T_STRING, T_STRUCT, T_MAP, T_SET, T_LIST = 2, 3, 4, 6, 8, 10, 11, 12, 13, 14, 15


class W:
    """Thrift binary writer."""

    def __init__(self):
        self.b = bytearray()

    def field(self, t, fid):
        self.b += bytes([t]) + struct.pack(">h", fid)

    def i32(self, fid, v):
        self.field(T_I32, fid)
        self.b += struct.pack(">i", int(v))

    def i64(self, fid, v):
        self.field(T_I64, fid)
        self.b += struct.pack(">q", int(v))

    def string(self, fid, s):
        data = s.encode() if isinstance(s, str) else bytes(s)
        self.field(T_STRING, fid)
        self.b += struct.pack(">i", len(data)) + data

    def boolean(self, fid, v):
        self.field(T_BOOL, fid)
        self.b += bytes([1 if v else 0])

    def double(self, fid, v):
        self.field(T_DOUBLE, fid)
        self.b += struct.pack(">d", float(v))

    def struct_(self, fid, fields: List):
        """fields: list of (fid, writer_fn) already sorted, written inside a nested struct."""
        self.field(T_STRUCT, fid)
        for f in fields:
            f(self)
        self.b += b"\x00"

    def list_strings(self, fid, items):
        self.field(T_LIST, fid)
        self.b += bytes([T_STRING]) + struct.pack(">i", len(items))
        for s in items:
            d = s.encode()
            self.b += struct.pack(">i", len(d)) + d

    def map_string_binary(self, fid, m: Dict[str, bytes]):
        self.field(T_MAP, fid)
        self.b += bytes([T_STRING, T_STRING]) + struct.pack(">i", len(m))
        for k, v in m.items():
            kd = k.encode()
            self.b += struct.pack(">i", len(kd)) + kd + struct.pack(">i", len(v)) + v


def _tl(fid, name):  # TaskList{10 Name, 20 Kind}
    return (fid, lambda w: w.struct_(fid, [lambda x: x.string(10, name), lambda x: x.i32(20, 0)]))


def _wt(fid, name):
    return (fid, lambda w: w.struct_(fid, [lambda x: x.string(10, name)]))


def _s(fid, v):
    return (fid, lambda w: w.string(fid, v))


def _i32(fid, v):
    return (fid, lambda w: w.i32(fid, v))


def _i64(fid, v):
    return (fid, lambda w: w.i64(fid, v))


def _retry(fid, rp):
    def f(w):
        items = [lambda x: x.i32(10, 1), lambda x: x.double(20, 2.0), lambda x: x.i32(30, 100),
                 lambda x: x.i32(40, 5), lambda x: x.list_strings(50, ["bad-input"])]
        exp = rp.get("expiration_interval_in_seconds") if isinstance(rp, dict) else None
        if exp is not None:
            items.append(lambda x: x.i32(60, exp))
        w.struct_(fid, items)
    return (fid, f)


def _reset_points(fid, prev):  # ResetPoints{10 Points list<ResetPointInfo>}
    def f(w):
        if prev == "nil_points":
            w.struct_(fid, [])
            return
        w.field(T_STRUCT, fid)
        w.field(T_LIST, 10)
        w.b += bytes([T_STRUCT]) + struct.pack(">i", len(prev))
        for i, bc in enumerate(prev):
            w.string(10, bc)
            w.string(20, f"prev-run-{i}")
            w.i64(30, 4 + i)
            w.i64(40, 1_500_000_000_000_000_000 + i)
            w.boolean(60, True)
            w.b += b"\x00"
        w.b += b"\x00"
    return (fid, f)


# per type: attribute name -> field builder (field ids: shared.go ToWire of each *EventAttributes)
_SCHED_REF = {ET.ActivityTaskStarted: 10, ET.ActivityTaskCompleted: 20, ET.ActivityTaskFailed: 30,
              ET.ActivityTaskTimedOut: 10, ET.ActivityTaskCanceled: 30}
_INIT_REF = {ET.StartChildWorkflowExecutionFailed: 60, ET.ChildWorkflowExecutionStarted: 20,
             ET.ChildWorkflowExecutionCompleted: 50, ET.ChildWorkflowExecutionFailed: 60,
             ET.ChildWorkflowExecutionCanceled: 50, ET.ChildWorkflowExecutionTimedOut: 50,
             ET.ChildWorkflowExecutionTerminated: 40, ET.RequestCancelExternalWorkflowExecutionFailed: 50,
             ET.ExternalWorkflowExecutionCancelRequested: 10, ET.SignalExternalWorkflowExecutionFailed: 50,
             ET.ExternalWorkflowExecutionSignaled: 10}


def attribute_fields(e: HistoryEvent, rng: Optional[random.Random] = None) -> List:
    """(field id, writer) pairs of the event's attribute struct, ascending by id."""
    t = e.event_type
    a = e.attrs
    g = e.get
    f = []
    if t == ET.WorkflowExecutionStarted:
        f += [_wt(10, "workflow-type")]
        if g("parent_workflow_domain", ""):
            f.append(_s(12, g("parent_workflow_domain")))
        f += [_tl(20, "task-list"), _s(30, "input-bytes"),
              _i32(40, g("execution_start_to_close_timeout_seconds", 0)),
              _i32(50, g("task_start_to_close_timeout_seconds", 0))]
        if a.get("initiator") is not None:
            f.append(_i32(55, a["initiator"]))
        f += [_s(60, "identity"), _i32(80, g("attempt", 0))]
        if g("expiration_timestamp", 0):
            f.append(_i64(90, g("expiration_timestamp")))
        f.append(_i32(110, g("first_decision_task_backoff_seconds", 0)))
        if a.get("prev_auto_reset_points") is not None:
            f.append(_reset_points(130, a["prev_auto_reset_points"]))
    elif t == ET.DecisionTaskScheduled:
        f += [_tl(10, "decision-tl"), _i32(20, g("start_to_close_timeout_seconds", 0)), _i64(30, g("attempt", 0))]
    elif t == ET.DecisionTaskStarted:
        f += [_i64(10, g("scheduled_event_id", 0)), _s(20, "worker-identity"), _s(30, g("request_id", ""))]
    elif t == ET.DecisionTaskCompleted:
        f += [_s(10, "ctx"), _i64(20, g("scheduled_event_id", 0)), _i64(30, g("started_event_id", 0)),
              _s(40, "worker-identity")]
        if g("binary_checksum", ""):
            f.append(_s(50, g("binary_checksum")))
    elif t == ET.DecisionTaskTimedOut:
        f += [_i64(10, 0), _i64(20, 0), _i32(30, g("timeout_type", 0))]
    elif t == ET.ActivityTaskScheduled:
        f += [_s(10, g("activity_id", "")), _wt(20, "activity-type")]
        if g("domain", ""):
            f.append(_s(25, g("domain")))
        f += [_tl(30, g("task_list", "activity-tl")), _s(40, "activity-input"),
              _i32(45, g("schedule_to_close_timeout_seconds", 0)), _i32(50, g("schedule_to_start_timeout_seconds", 0)),
              _i32(55, g("start_to_close_timeout_seconds", 0)), _i32(60, g("heartbeat_timeout_seconds", 0)),
              _i64(90, 4)]
        if a.get("retry_policy") is not None:
            f.append(_retry(110, a["retry_policy"]))
    elif t in _SCHED_REF:
        fid = _SCHED_REF[t]
        f.append(_i64(fid, g("scheduled_event_id", 0)))
        if t == ET.ActivityTaskStarted:
            f += [_s(20, "worker"), _s(30, g("request_id", "")), _i32(40, 0)]
        f.sort(key=lambda x: x[0])
    elif t == ET.ActivityTaskCancelRequested:
        f += [_s(10, g("activity_id", "")), _i64(20, 4)]
    elif t == ET.TimerStarted:
        f += [_s(10, g("timer_id", "")), _i64(20, g("start_to_fire_timeout_seconds", 0)), _i64(30, 4)]
    elif t in (ET.TimerFired, ET.TimerCanceled):
        f += [_s(10, g("timer_id", "")), _i64(20, 5)]
    elif t == ET.StartChildWorkflowExecutionInitiated:
        if g("domain", ""):
            f.append(_s(10, g("domain")))
        f += [_s(20, g("workflow_id", "child-wf")), _wt(30, "child-type"), _tl(40, "child-tl"), _i32(81, 1)]
    elif t in (ET.RequestCancelExternalWorkflowExecutionInitiated, ET.SignalExternalWorkflowExecutionInitiated):
        f.append(_i64(10, 4))
        if g("domain", ""):
            f.append(_s(20, g("domain")))
        f.append((30, lambda w: w.struct_(30, [lambda x: x.string(10, "target-wf"), lambda x: x.string(20, "target-run")])))
        if t == ET.SignalExternalWorkflowExecutionInitiated:
            f += [_s(40, g("signal_name", "sig")), _s(50, "signal-input")]
    elif t in _INIT_REF:
        f.append(_i64(_INIT_REF[t], g("initiated_event_id", 0)))
    elif t == ET.WorkflowExecutionSignaled:
        f += [_s(10, "signal"), _s(20, "payload"), _s(30, "identity")]
    elif t == ET.WorkflowExecutionContinuedAsNew:
        f += [_s(10, str(g("new_execution_run_id", "new-run"))), _wt(20, "workflow-type")]
    elif t == ET.UpsertWorkflowSearchAttributes:
        f += [_i64(10, 4), (20, lambda w: w.struct_(20, [lambda x: x.map_string_binary(10, {"CustomKeywordField": b'"v"'})]))]
    elif t == ET.MarkerRecorded:
        f += [_s(10, "marker"), _s(20, "details")]
    f.sort(key=lambda x: x[0])
    return f


def encode_event(w: W, e: HistoryEvent):
    w.i64(10, e.id)
    w.i64(20, e.timestamp)
    w.i32(30, e.event_type)
    w.i64(35, e.version)
    w.i64(36, e.task_id)
    if 0 <= e.event_type <= 41:
        fid = 40 + 10 * int(e.event_type)
        w.struct_(fid, [fn for _, fn in attribute_fields(e)])
    w.b += b"\x00"


def serialize_batch_events(events: List[HistoryEvent]) -> bytes:
    """SerializeBatchEvents(events, EncodingTypeThriftRW).Data; an empty batch is an empty blob."""
    if not events:
        return b""
    w = W()
    w.b += b"\x59"                                   # preambleVersion0 (common/codec/interface.go:48)
    w.field(T_LIST, 10)                             # History.Events
    w.b += bytes([T_STRUCT]) + struct.pack(">i", len(events))
    for e in events:
        encode_event(w, e)
    w.b += b"\x00"
    return bytes(w.b)


def serialize_history(h: WorkflowHistory) -> List[bytes]:
    """One blob per persisted batch (the pages state_rebuilder.go:135-148 reads)."""
    return [serialize_batch_events(b) for b in h.batches]
