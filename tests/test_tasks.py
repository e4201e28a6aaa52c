"""Transfer / timer task emission (CRR_IN_EMIT_TASKS).

The expected sequences restate the task-generator calls of ApplyEvents (state_builder.go:157-640)
and their arguments (mutable_state_task_generator.go:143-612, timer_sequence.go:127-199), in the
order Go appends them.  CPU: the oracle.  GPU: device rows == oracle rows on every path.
"""
import pytest

from cadence_amd import abi, synth_mixed
from cadence_amd.abi import EventType as ET, TaskKind as K
from cadence_amd.flatten import flatten, interleave
from cadence_amd.history import HistoryEvent, WorkflowHistory
from cadence_amd.result import diff_results
from oracle import oracle

SEC = 1_000_000_000
NOW = 1_600_000_000 * SEC
KNOWN = {"domain-a", "domain-b", "parent-domain"}


def ev(t, i, v=12, **attrs):
    return HistoryEvent(int(t), i, v, NOW + i * SEC, 5000 + i, attrs)


def tasks_of(h, **kw):
    b = flatten([h])
    b.emit_tasks = True
    r = oracle.replay(b, 1)
    rows = r.live_rows(b, 0)["tasks"]
    return r.exec[0], [(K(int(x["kind"])), int(x["aux"]), int(x["version"]), int(x["visibility_ts"]),
                        int(x["event_id"]), int(x["attempt"]), int(x["src"])) for x in rows]


def test_activity_chain_task_sequence():
    h = WorkflowHistory(batches=[
        [ev(ET.WorkflowExecutionStarted, 1, execution_start_to_close_timeout_seconds=3600,
            task_start_to_close_timeout_seconds=10), ev(ET.DecisionTaskScheduled, 2, start_to_close_timeout_seconds=10)],
        [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
        [ev(ET.DecisionTaskCompleted, 4, started_event_id=3),
         ev(ET.ActivityTaskScheduled, 5, activity_id="a", schedule_to_start_timeout_seconds=30,
            schedule_to_close_timeout_seconds=60, start_to_close_timeout_seconds=20)],
        [ev(ET.ActivityTaskStarted, 6, scheduled_event_id=5)],
        [ev(ET.ActivityTaskCompleted, 7, scheduled_event_id=5), ev(ET.DecisionTaskScheduled, 8)],
        [ev(ET.DecisionTaskStarted, 9, scheduled_event_id=8)],
        [ev(ET.DecisionTaskCompleted, 10, started_event_id=9), ev(ET.WorkflowExecutionCompleted, 11)]],
        retention_days=7)
    ex, t = tasks_of(h)
    assert ex["status"] == 0
    ts = lambda i: NOW + i * SEC  # noqa: E731
    assert t == [
        (K.RecordWorkflowStarted, 0, 12, 0, 0, 0, 0),                      # task_generator.go:301-313
        (K.WorkflowTimeout, 0, 12, ts(1) + 3600 * SEC, 0, 0, 0),            # :143-166
        (K.Decision, 0, 12, 0, 2, 0, 1),                                    # :315-350
        (K.DecisionTimeout, 0, 12, ts(3) + 10 * SEC, 2, 0, 2),              # :352-388 (StartToClose)
        (K.Activity, 0, 12, 0, 5, 0, 4),                                    # :390-428
        # batch epilogue: ScheduleToStart (30 s) is the first activity timer (timer_sequence.go:162-199)
        (K.ActivityTimeout, abi.TimeoutType.ScheduleToStart, 12, ts(5) + 30 * SEC, 5, 0, -1),
        # started: StartToClose (20 s after start) precedes ScheduleToClose; a new timer is created
        (K.ActivityTimeout, abi.TimeoutType.StartToClose, 12, ts(6) + 20 * SEC, 5, 0, -1),
        (K.Decision, 0, 12, 0, 8, 0, 7),
        (K.DecisionTimeout, 0, 12, ts(9) + 0 * SEC, 8, 0, 8),               # DecisionTaskScheduled carried no timeout
        (K.CloseExecution, 0, 12, 0, 0, 0, 10),                             # :168-236
        (K.DeleteHistory, 0, 12, ts(11) + 7 * 86400 * SEC, 0, 0, 10),       # :238-255
    ]
    assert ex["n_tasks"] == len(t)


def test_backoff_transient_timers_and_externals():
    h = WorkflowHistory(batches=[
        [ev(ET.WorkflowExecutionStarted, 1, execution_start_to_close_timeout_seconds=100,
            first_decision_task_backoff_seconds=5, initiator=abi.INITIATOR_RETRY_POLICY, attempt=2,
            expiration_timestamp=NOW + 50 * SEC), ev(ET.DecisionTaskScheduled, 2)],
        [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
        [ev(ET.DecisionTaskFailed, 4)],                                       # transient decision (attempt 1)
        [ev(ET.DecisionTaskStarted, 5, scheduled_event_id=4)],   # transient ScheduleID = NextEventID before the batch
        [ev(ET.DecisionTaskCompleted, 6, started_event_id=5), ev(ET.TimerStarted, 7, timer_id="t",
                                                                 start_to_fire_timeout_seconds=9),
         ev(ET.StartChildWorkflowExecutionInitiated, 8), ev(ET.RequestCancelExternalWorkflowExecutionInitiated, 9),
         ev(ET.SignalExternalWorkflowExecutionInitiated, 10), ev(ET.UpsertWorkflowSearchAttributes, 11)]],
        now_ns=777)
    ex, t = tasks_of(h)
    assert ex["status"] == 0
    kinds = [x[0] for x in t]
    assert kinds == [K.RecordWorkflowStarted, K.WorkflowTimeout, K.WorkflowBackoff, K.Decision, K.DecisionTimeout,
                     K.Decision, K.DecisionTimeout, K.StartChild, K.CancelExecution, K.SignalExecution,
                     K.UpsertSearchAttributes, K.UserTimer]
    # attempt > 0: the workflow timeout is capped at the expiration time (task_generator.go:155-158)
    assert t[1][3] == NOW + 50 * SEC
    assert t[2][1] == abi.BACKOFF_RETRY and t[2][3] == NOW + SEC + 5 * SEC
    assert t[5][4] == 4 and t[5][6] == 0          # transient decision: ScheduleID = NextEventID, task list of the start
    assert t[-1][4] == 7 and t[-1][3] == NOW + 7 * SEC + 9 * SEC


def test_failure_keeps_tasks_generated_before_it():  # no rollback (state_builder.go returns mid-loop)
    h = WorkflowHistory(batches=[[ev(ET.WorkflowExecutionStarted, 1), ev(ET.DecisionTaskScheduled, 2)],
                                 [ev(ET.ActivityTaskStarted, 3, scheduled_event_id=99)]])
    ex, t = tasks_of(h)
    assert ex["status"] == abi.Status.MISSING_ACTIVITY_INFO
    assert [x[0] for x in t] == [K.RecordWorkflowStarted, K.WorkflowTimeout, K.Decision]


def test_rebuild_drops_replay_tasks():  # CloseTransactionAsSnapshot clears them (state_rebuilder.go:178-181)
    h = WorkflowHistory(batches=[[ev(ET.WorkflowExecutionStarted, 1), ev(ET.DecisionTaskScheduled, 2)]],
                        refresh_tasks=True)
    ex, t = tasks_of(h)
    assert ex["status"] == 0 and t == []


def _mixed():
    hs = synth_mixed.mixed_histories(3000, 61, multi_version=True, invalid_rate=0.2, can_rate=0.4)
    for i, h in enumerate(hs):
        h.retention_days = 1 + i % 30
    return flatten(hs, known_domains=KNOWN)


def test_tasks_identical_across_layouts():
    b = _mixed()
    b.emit_tasks = True
    want = oracle.replay(b, 2)
    assert int(want.exec["n_tasks"].sum()) > 50_000
    ib = interleave(b)
    assert ib.emit_tasks
    assert not diff_results(b, want, ib, oracle.replay(ib, 2))


@pytest.mark.gpu
def test_device_tasks_match_oracle():
    from cadence_amd.engine import ReplayEngine
    eng = ReplayEngine(0)
    b = _mixed()
    b.emit_tasks = True
    want = oracle.replay(b, 0)
    for layout in (interleave(b), interleave(b, long_threshold=None), interleave(b, long_threshold=0), b):
        got = eng.replay(layout)
        d = diff_results(layout, got, b, want)
        assert not d, "\n".join(d)
    lt = flatten(synth_mixed.long_tail_histories(80, 62, max_len=4000, run_cap=1500, multi_version=True,
                                                 caps=None), known_domains=KNOWN)
    lt.emit_tasks = True
    want = oracle.replay(lt, 0)
    got = eng.replay(interleave(lt))
    assert not diff_results(interleave(lt), got, lt, want)
