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


# ---- Rebuild's RefreshTasks (state_rebuilder.go:181-186 -> mutable_state_task_refresher.go:77-496): the
# replay's tasks are dropped (CloseTransactionAsSnapshot) and RefreshTasks' own are the task rows ----
REB_NOW = NOW + 10_000 * SEC       # the rebuild's now: RefreshTasks' startTime


def refresh_of(batches, adv=False, **kw):
    h = WorkflowHistory(batches=batches, refresh_tasks=True, now_ns=REB_NOW, retention_days=3, **kw)
    b = flatten([h], known_domains=KNOWN)
    b.emit_tasks = True
    b.advanced_visibility = adv
    r = oracle.replay(b, 1)
    rows = r.live_rows(b, 0)["tasks"]
    return r, [(K(int(x["kind"])), int(x["aux"]), int(x["version"]), int(x["visibility_ts"]),
                int(x["event_id"]), int(x["attempt"]), int(x["src"])) for x in rows]


def _start(i=1, **a):
    return ev(ET.WorkflowExecutionStarted, i, execution_start_to_close_timeout_seconds=3600,
              task_start_to_close_timeout_seconds=10, **a)


def test_refresh_scheduled_decision():
    # refreshTasksForWorkflowStart (:172-202): WorkflowTimeout from startTime = now; RecordWorkflowStarted
    # (:224-244, not closed); refreshTasksForDecision (:246-276): only scheduled -> GenerateDecisionScheduleTasks
    r, t = refresh_of([[_start(), ev(ET.DecisionTaskScheduled, 2, start_to_close_timeout_seconds=10)]])
    assert r.exec["status"][0] == 0
    assert t == [(K.WorkflowTimeout, 0, 12, REB_NOW + 3600 * SEC, 0, 0, 0),
                 (K.RecordWorkflowStarted, 0, 12, 0, 0, 0, 0),
                 (K.Decision, 0, 12, 0, 2, 0, 0)]


def test_refresh_started_decision_and_activities():
    # decision started -> GenerateDecisionStartTasks (task_generator.go:352-388); refreshTasksForActivity
    # (:278-336): a transfer task per not-started activity, then CreateNextActivityTimer; refreshTasksForTimer
    # (:338-365): CreateNextUserTimer; children not started, request-cancels, signals (:367-482)
    r, t = refresh_of([
        [_start(), ev(ET.DecisionTaskScheduled, 2, start_to_close_timeout_seconds=10)],
        [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
        [ev(ET.DecisionTaskCompleted, 4, started_event_id=3),
         ev(ET.ActivityTaskScheduled, 5, activity_id="a", schedule_to_start_timeout_seconds=30,
            schedule_to_close_timeout_seconds=60, start_to_close_timeout_seconds=20),
         ev(ET.ActivityTaskScheduled, 6, activity_id="b", schedule_to_start_timeout_seconds=40,
            schedule_to_close_timeout_seconds=90, start_to_close_timeout_seconds=20),
         ev(ET.TimerStarted, 7, timer_id="t1", start_to_fire_timeout_seconds=500),
         ev(ET.TimerStarted, 8, timer_id="t2", start_to_fire_timeout_seconds=5),
         ev(ET.StartChildWorkflowExecutionInitiated, 9, domain="domain-a"),
         ev(ET.StartChildWorkflowExecutionInitiated, 10, domain="domain-b"),
         ev(ET.RequestCancelExternalWorkflowExecutionInitiated, 11, domain="domain-a"),
         ev(ET.SignalExternalWorkflowExecutionInitiated, 12, domain="domain-b"),
         ev(ET.DecisionTaskScheduled, 13, start_to_close_timeout_seconds=15)],
        [ev(ET.ActivityTaskStarted, 14, scheduled_event_id=5), ev(ET.ChildWorkflowExecutionStarted, 15,
                                                                  initiated_event_id=9),
         ev(ET.DecisionTaskStarted, 16, scheduled_event_id=13)]], adv=True)
    assert r.exec["status"][0] == 0
    ts = lambda i: NOW + i * SEC  # noqa: E731
    assert t == [
        (K.WorkflowTimeout, 0, 12, REB_NOW + 3600 * SEC, 0, 0, 0),
        (K.RecordWorkflowStarted, 0, 12, 0, 0, 0, 0),
        (K.DecisionTimeout, abi.TimeoutType.StartToClose, 12, ts(16) + 15 * SEC, 13, 0, -1),
        (K.Activity, 0, 12, 0, 6, 0, 5),                     # activity 5 is started: no transfer task
        # the earliest activity timer after the masks are cleared: 5's StartToClose (14 + 20 s) vs 6's
        # ScheduleToStart (6 + 40 s = 46 s) -> 34 s
        (K.ActivityTimeout, abi.TimeoutType.StartToClose, 12, ts(14) + 20 * SEC, 5, 0, -1),
        (K.UserTimer, 0, 12, ts(8) + 5 * SEC, 8, 0, -1),     # t2 fires first
        (K.StartChild, 0, 12, 0, 10, 0, 9),                  # child 9 is started
        (K.CancelExecution, 0, 12, 0, 11, 0, 10),
        (K.SignalExecution, 0, 12, 0, 12, 0, 11),
        (K.UpsertSearchAttributes, 0, 12, 0, 0, 0, -1)]      # AdvancedVisibilityWritingMode on (:160-167)


def test_refresh_closed_workflow_and_delayed_decision():
    # closed: GenerateWorkflowCloseTasks from the completion event (:204-222), no RecordWorkflowStarted
    r, t = refresh_of([[_start(), ev(ET.DecisionTaskScheduled, 2)], [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
                       [ev(ET.DecisionTaskCompleted, 4, started_event_id=3), ev(ET.WorkflowExecutionCompleted, 5)]])
    assert r.exec["status"][0] == 0
    assert t == [(K.WorkflowTimeout, 0, 12, REB_NOW + 3600 * SEC, 0, 0, 0),
                 (K.CloseExecution, 0, 12, 0, 0, 0, 4),
                 (K.DeleteHistory, 0, 12, NOW + 5 * SEC + 3 * 86400 * SEC, 0, 0, 4)]
    # no decision processed or pending and a first-decision backoff: GenerateDelayedDecisionTasks
    r, t = refresh_of([[_start(first_decision_task_backoff_seconds=30, initiator=abi.INITIATOR_CRON)]])
    assert r.exec["status"][0] == 0
    assert t == [(K.WorkflowTimeout, 0, 12, REB_NOW + (3600 + 30) * SEC, 0, 0, 0),
                 (K.WorkflowBackoff, abi.BACKOFF_CRON, 12, NOW + SEC + 30 * SEC, 0, 0, 0),
                 (K.RecordWorkflowStarted, 0, 12, 0, 0, 0, 0)]
    r, t = refresh_of([[_start(first_decision_task_backoff_seconds=30, initiator=abi.INITIATOR_DECIDER)]])
    assert r.exec["status"][0] == abi.Status.BAD_INITIATOR


def test_refresh_missing_start_or_completion_event():
    # GetStartEvent (mutable_state_builder.go:1131-1157): no event with ID 1 to read
    r, _t = refresh_of([[ev(ET.DecisionTaskScheduled, 2)]])
    assert r.exec["status"][0] == abi.Status.MISSING_START_EVENT
    # GetCompletionEvent (:1085-1128) reads event NextEventID - 1 from the completion batch: a signal in a
    # later batch is not in it
    r, _t = refresh_of([[_start(), ev(ET.DecisionTaskScheduled, 2)], [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
                        [ev(ET.DecisionTaskCompleted, 4, started_event_id=3), ev(ET.WorkflowExecutionCompleted, 5)],
                        [ev(ET.WorkflowExecutionSignaled, 6)]])
    assert r.exec["status"][0] == abi.Status.MISSING_COMPLETION_EVENT


def _refresh_state_effect_histories():
    """Rebuilds whose RefreshTasks fails, with task emission on or off alike: a bad delayed-decision
    initiator (mutable_state_task_generator.go:269-277; the start event's own task generation already
    fails on it) and a missing start event
    (mutable_state_builder.go:1131-1157) with a live activity whose timer task status a failing head
    leaves as replayed (the timer refresh comes after it, mutable_state_task_refresher.go:278-336), and a
    completion event outside the completion batch (:1085-1128).  And two
    started decisions scheduled with Attempt 3 / 6: getNextDecisionTimeout's DecisionTimeout write-back
    (:352-388, :1051-1064) needs a started decision with Attempt > 1, which a replay cannot leave --
    ReplicateDecisionTaskStartedEvent is called with a nil decision and sets Attempt = 0
    (mutable_state_decision_task_manager.go:207-223) -- and RefreshTasks on a resumed state fails at
    GetStartEvent (the start event is not in the call), so the write-back is unreachable on this path."""
    act = dict(activity_id="a", schedule_to_start_timeout_seconds=30, schedule_to_close_timeout_seconds=60,
               start_to_close_timeout_seconds=20)
    hs = [
        [[_start(), ev(ET.DecisionTaskScheduled, 2, start_to_close_timeout_seconds=10, attempt=3)],
         [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)]],
        [[_start(), ev(ET.DecisionTaskScheduled, 2, start_to_close_timeout_seconds=7, attempt=6)],
         [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)]],
        [[_start(first_decision_task_backoff_seconds=30, initiator=abi.INITIATOR_DECIDER),
          ev(ET.ActivityTaskScheduled, 2, **act)]],
        [[ev(ET.DecisionTaskScheduled, 2), ev(ET.ActivityTaskScheduled, 3, **act)]],
        [[_start(), ev(ET.DecisionTaskScheduled, 2)], [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
         [ev(ET.DecisionTaskCompleted, 4, started_event_id=3), ev(ET.WorkflowExecutionCompleted, 5)],
         [ev(ET.WorkflowExecutionSignaled, 6)]],
    ]
    return [WorkflowHistory(batches=b, refresh_tasks=True, now_ns=REB_NOW, retention_days=3,
                            refresh_jitter=5 * SEC + 123 + 7 * i) for i, b in enumerate(hs)]


def test_refresh_state_effects_do_not_depend_on_emission():
    # the bad initiator already fails the replay at the start event's own GenerateDelayedDecisionTasks
    want_status = [0, 0, abi.Status.BAD_INITIATOR, abi.Status.MISSING_START_EVENT, abi.Status.MISSING_COMPLETION_EVENT]
    res, bs = {}, {}
    for emit in (False, True):
        b = bs[emit] = flatten(_refresh_state_effect_histories(), known_domains=KNOWN)
        b.emit_tasks = emit
        res[emit] = oracle.replay(b, 1)
        assert [int(s) for s in res[emit].exec["status"]] == want_status
    for f in ("decision_timeout", "decision_attempt", "status", "fail_step", "checksum", "flags"):
        assert (res[False].exec[f] == res[True].exec[f]).all(), f
    # the started decisions' Attempt is 0 after the replay, so DecisionTimeout stays the scheduled one
    assert [int(x) for x in res[False].exec["decision_attempt"][:2]] == [0, 0]
    assert [int(x) for x in res[False].exec["decision_timeout"][:2]] == [10, 7]
    # a failing head leaves the activity's timer task status as the replay's epilogue set it
    for w in (3,):
        assert int(res[False].live_rows(bs[False], w)["act"]["timer_task_status"][0]) != 0


@pytest.mark.gpu
def test_device_refresh_state_effects_match_oracle():
    from cadence_amd.engine import ReplayEngine
    eng = ReplayEngine(0)
    for emit in (False, True):
        b = flatten(_refresh_state_effect_histories() * 40, known_domains=KNOWN)
        b.emit_tasks = emit
        want = oracle.replay(b, 1)
        for layout in (interleave(b), interleave(b, long_threshold=0), b):
            layout.emit_tasks = emit
            got = eng.replay(layout)
            d = diff_results(layout, got, b, want)
            assert not d, f"emit={emit}: " + "\n".join(d)


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
