"""Known-answer cases restated from the reference's dispatch-table spec,
service/history/execution/state_builder_test.go:143-1749 (45 tests).

Each Go test hands ApplyEvents one batch holding one event (ID 130, version 1) and a mocked
MutableState / MutableStateTaskGenerator, then asserts which Replicate* call and which Generate*
calls happen with which arguments, plus, for every test (mockUpdateVersion, :128-135),
UpdateCurrentVersion(event.Version, true), GenerateActivityTimerTasks / GenerateUserTimerTasks and
SetHistoryBuilder.  Here the mock becomes a *loaded* state (CRR_WF_FLAG_RESUME, the analogue of the
mock's canned GetExecutionInfo and of the pending infos the Replicate call needs), the Replicate
call's effect is asserted on the rows it writes (mutable_state_builder.go / decision task manager,
cited per case), and the Generate* calls on the emitted task rows (CRR_IN_EMIT_TASKS).  Where a Go
mock returns an arbitrary value that the real code derives (e.g. the transient decision's
ScheduleID = NextEventID, :168-197), the derived value is expected.

Every case is replayed by the oracle (tests/test_oracle_kats.py) and by the device
(tests/test_gpu_kats.py) against the same expectations.
"""
from __future__ import annotations

import dataclasses
from typing import Callable, Dict, List, Optional

import numpy as np

from cadence_amd import abi
from cadence_amd.abi import EventType as ET, TaskKind as TK
from cadence_amd.flatten import LoadedStates, flatten
from cadence_amd.history import HistoryEvent, WorkflowHistory

SB = "service/history/execution/state_builder_test.go"
NOW = 1_700_000_000_000_000_000          # event timestamp (the tests' time.Now())
SEC = 1_000_000_000
EV_ID, VERSION = 130, 1                   # every test's event ID and version
PARENT_DOMAIN = "some random parent domain name"     # constants.TestParentDomainName
TARGET_DOMAIN = "some random target domain name"     # constants.TestTargetDomainName
KNOWN = {PARENT_DOMAIN, TARGET_DOMAIN}


def event(t, i=EV_ID, ts=NOW, v=VERSION, **attrs) -> HistoryEvent:
    return HistoryEvent(int(t), i, v, ts, 5000 + i, attrs)


# ---- the loaded state (the mock's GetExecutionInfo + the infos its Replicate call finds) ------------
@dataclasses.dataclass
class State:
    exec: Dict = dataclasses.field(default_factory=dict)
    acts: List[Dict] = dataclasses.field(default_factory=list)
    timers: List[Dict] = dataclasses.field(default_factory=list)
    children: List[Dict] = dataclasses.field(default_factory=list)
    rcs: List[Dict] = dataclasses.field(default_factory=list)
    sigs: List[Dict] = dataclasses.field(default_factory=list)
    keys: List[str] = dataclasses.field(default_factory=list)   # interned strings (ids 1..)


def running(**exec_over) -> Dict:
    """A running workflow whose next event is 130: the last batch was [129], no pending decision."""
    e = dict(state=abi.State.Running, close_status=0, next_event_id=EV_ID, last_first_event_id=EV_ID - 1,
             last_event_task_id=5000 + EV_ID - 1, last_processed_event=EV_ID - 3,
             decision_version=abi.EMPTY_VERSION, decision_schedule_id=abi.EMPTY_EVENT_ID,
             decision_started_id=abi.EMPTY_EVENT_ID, decision_attempt=0, decision_timeout=0,
             decision_request_src=abi.SRC_EMPTY_UUID, start_src=0, token_src=1, decision_start_to_close=11,
             src_next=EV_ID - 1, vh=[(EV_ID - 1, VERSION)])
    e.update(exec_over)
    return e


def act_row(schedule_id, key, started_id=abi.EMPTY_EVENT_ID, started=abi.ZERO_TIME, s2s=100, s2c=200, st2c=50,
            hb=0, tts=0, **kw):
    r = dict(schedule_id=schedule_id, version=VERSION, scheduled_batch_id=schedule_id, scheduled_time=NOW - 100 * SEC,
             started_id=started_id, started_time=started, cancel_request_id=abi.EMPTY_EVENT_ID,
             last_hb_timeout_vis_s=0, sched_src=7, started_src=-1 if started_id == abi.EMPTY_EVENT_ID else 8,
             schedule_to_start=s2s, schedule_to_close=s2c, start_to_close=st2c, heartbeat=hb, timer_task_status=tts,
             key=key, flags=abi.ROW_LIVE | abi.ROW_MAPPED, last_heartbeat_time=started)
    r.update(kw)
    return r


def loaded_states(states: List[Optional[State]]) -> LoadedStates:
    n = len(states)
    ex = np.zeros(n, abi.EXEC_ROW)
    rows = {name: [] for name, *_ in abi.TABLES if name != "tasks"}
    mask = np.zeros(n, bool)
    interners = []
    for w, s in enumerate(states):
        ids = {"": 0}
        if s is None:
            interners.append(ids)
            continue
        for k in s.keys:
            ids.setdefault(k, len(ids))
        interners.append(ids)
        mask[w] = True
        e = dict(s.exec)
        vh = e.pop("vh")
        for f, v in e.items():
            ex[f][w] = v
        for name, lst, dt, n_f in (("act", s.acts, abi.ACTIVITY_ROW, "n_activity"),
                                   ("timer", s.timers, abi.TIMER_ROW, "n_timer"),
                                   ("child", s.children, abi.CHILD_ROW, "n_child"),
                                   ("rc", s.rcs, abi.INITIATED_ROW, "n_rc"), ("sig", s.sigs, abi.INITIATED_ROW, "n_signal")):
            for d in lst:
                r = np.zeros(1, dt)
                for f, v in d.items():
                    r[f] = v
                if "flags" not in d:
                    r["flags"] = abi.ROW_LIVE
                rows[name].append(r)
            ex[n_f][w] = len(lst)
        for it in vh:
            rows["vh"].append(np.array([it], abi.VH_ITEM))
        ex["n_vh_items"][w] = len(vh)
    out = {k: (np.concatenate(v) if v else np.zeros(0, dict(((t[0], t[1]) for t in abi.TABLES))[k]))
           for k, v in rows.items()}
    return LoadedStates(ex, out, mask, interners)


# ---- cases --------------------------------------------------------------------------------------------
@dataclasses.dataclass
class Kat:
    name: str
    cite: str                                   # the Go test restated (file:line)
    batches: List[List[HistoryEvent]]           # the ApplyEvents history (one batch)
    state: Optional[State]                      # None: a fresh mutable state (the start event)
    check: Callable                             # check(exec_row, live_rows, tasks, ctx)
    new_run: Optional[List[List[HistoryEvent]]] = None   # newRunHistory (continue-as-new)
    check_new_run: Optional[Callable] = None


def tasks_of(tasks) -> List[tuple]:
    return [(int(t["kind"]), int(t["event_id"])) for t in tasks]


def expect_common(e, status=0):
    """mockUpdateVersion: UpdateCurrentVersion(event.Version, true) (+ AddOrUpdateItem(130, 1))."""
    assert int(e["status"]) == status, int(e["status"])
    if status == 0:
        assert int(e["current_version"]) == VERSION
        assert int(e["next_event_id"]) == EV_ID + 1 and int(e["last_first_event_id"]) == EV_ID   # :642-643


def vh_extended(live):
    assert [(int(x["event_id"]), int(x["version"])) for x in live["vh"]] == [(EV_ID, VERSION)]


def close_case(name, line, t, cs):
    def check(e, live, tasks, ctx):
        expect_common(e)
        assert int(e["state"]) == abi.State.Completed and int(e["close_status"]) == cs
        assert int(e["completion_event_batch_id"]) == EV_ID
        # GenerateWorkflowCloseTasks(event): the close transfer task + DeleteHistoryEventTask at
        # close time + retention (TestGlobalDomainEntry: Retention 1 day)
        assert [(int(x["kind"]), int(x["version"]), int(x["visibility_ts"])) for x in tasks] == \
            [(TK.CloseExecution, VERSION, 0), (TK.DeleteHistory, VERSION, NOW + 86400 * SEC)]
        vh_extended(live)
    return Kat(name, f"{SB}:{line}", [[event(t)]], State(exec=running()), check)


def no_task_case(name, line, batch, state, extra=None):
    def check(e, live, tasks, ctx):
        expect_common(e)
        assert tasks_of(tasks) == [], tasks_of(tasks)
        vh_extended(live)
        if extra:
            extra(e, live, ctx)
    return Kat(name, f"{SB}:{line}", [batch], state, check)


def _started_fresh(cron: bool):
    attrs = dict(parent_workflow_domain=PARENT_DOMAIN, execution_start_to_close_timeout_seconds=100,
                 task_start_to_close_timeout_seconds=11)
    if cron:   # ParentWorkflowDomainID given: no domain-cache lookup (:222 Times(0)); cron initiator + backoff
        attrs.update(parent_workflow_domain_id="deadbeef-0123-4567-890a-bcdef0123457", initiator=abi.INITIATOR_CRON,
                     first_decision_task_backoff_seconds=60)

    def check(e, live, tasks, ctx):
        assert int(e["status"]) == 0
        assert int(e["state"]) == abi.State.Created and int(e["current_version"]) == VERSION
        assert int(e["start_src"]) == 0 and int(e["token_src"]) == 1          # SetHistoryTree(runID)
        assert int(e["last_first_event_id"]) == 1 and int(e["next_event_id"]) == 2
        assert int(e["decision_schedule_id"]) == abi.EMPTY_EVENT_ID
        want = [(TK.RecordWorkflowStarted, VERSION, 0),                       # GenerateRecordWorkflowStartedTasks
                (TK.WorkflowTimeout, VERSION, NOW + (100 + (60 if cron else 0)) * SEC)]   # GenerateWorkflowStartTasks
        if cron:
            want.append((TK.WorkflowBackoff, VERSION, NOW + 60 * SEC))        # GenerateDelayedDecisionTasks
        assert [(int(x["kind"]), int(x["version"]), int(x["visibility_ts"])) for x in tasks] == want
        if cron:
            assert int(tasks[2]["aux"]) == abi.BACKOFF_CRON
        assert [(int(x["event_id"]), int(x["version"])) for x in live["vh"]] == [(1, VERSION)]
    return Kat(f"WorkflowExecutionStarted_{'WithCron' if cron else 'NoCron'}Schedule",
               f"{SB}:{189 if cron else 143}", [[event(ET.WorkflowExecutionStarted, i=1, **attrs)]], None, check)


def _can(with_new_run: bool):
    new_run = None
    if with_new_run:   # :420-466: Started, Signaled, DecisionTaskScheduled(attempt 123) in one batch
        new_run = [[event(ET.WorkflowExecutionStarted, i=1, parent_workflow_domain_id="deadbeef-0123-4567-890a-bcdef0123457",
                          parent_workflow_domain=PARENT_DOMAIN, execution_start_to_close_timeout_seconds=110,
                          task_start_to_close_timeout_seconds=11),
                    event(ET.WorkflowExecutionSignaled, i=2),
                    event(ET.DecisionTaskScheduled, i=3, start_to_close_timeout_seconds=11, attempt=123)]]

    def check(e, live, tasks, ctx):
        expect_common(e)
        # ReplicateWorkflowExecutionContinuedAsNewEvent(130, domainID, event) (mutable_state_builder.go:3366-3382)
        assert int(e["state"]) == abi.State.Completed and int(e["close_status"]) == abi.CloseStatus.ContinuedAsNew
        assert int(e["completion_event_batch_id"]) == EV_ID
        assert [int(x["kind"]) for x in tasks] == [TK.CloseExecution, TK.DeleteHistory]   # GenerateWorkflowCloseTasks

    def check_new(e, live, tasks, ctx):
        # the new run's own task generator (:485-496): started + timeout tasks, the decision schedule task
        # of event 3, then the timer epilogue (nothing pending)
        assert int(e["status"]) == 0
        assert int(e["state"]) == abi.State.Running and int(e["signal_count"]) == 1
        assert int(e["decision_schedule_id"]) == 3 and int(e["decision_attempt"]) == 123
        assert int(e["decision_timeout"]) == 11 and int(e["next_event_id"]) == 4
        assert [(int(x["kind"]), int(x["event_id"]), int(x["visibility_ts"])) for x in tasks] == \
            [(TK.RecordWorkflowStarted, 0, 0), (TK.WorkflowTimeout, 0, NOW + 110 * SEC), (TK.Decision, 3, 0)]
    name = "WorkflowExecutionContinuedAsNew" + ("" if with_new_run else "_EmptyNewRunHistory")
    return Kat(name, f"{SB}:{392 if with_new_run else 503}", [[event(ET.WorkflowExecutionContinuedAsNew)]],
               State(exec=running()), check, new_run=new_run, check_new_run=check_new if with_new_run else None)


def _decision_scheduled():
    def check(e, live, tasks, ctx):
        expect_common(e)
        # ReplicateDecisionTaskScheduledEvent(1, 130, tasklist, 11, 111, ts, ts) (decision_task_manager.go:129-166)
        assert (int(e["decision_version"]), int(e["decision_schedule_id"]), int(e["decision_started_id"])) == \
            (VERSION, EV_ID, abi.EMPTY_EVENT_ID)
        assert int(e["decision_timeout"]) == 11 and int(e["decision_attempt"]) == 111
        assert int(e["decision_scheduled_ts"]) == NOW and int(e["decision_orig_scheduled_ts"]) == NOW
        assert int(e["decision_request_src"]) == abi.SRC_EMPTY_UUID
        assert tasks_of(tasks) == [(TK.Decision, EV_ID)]                      # GenerateDecisionScheduleTasks(130)
    return Kat("DecisionTaskScheduled", f"{SB}:654",
               [[event(ET.DecisionTaskScheduled, start_to_close_timeout_seconds=11, attempt=111)]],
               State(exec=running()), check)


def _decision_started():
    st = running(decision_version=VERSION, decision_schedule_id=111, decision_timeout=11,
                 decision_scheduled_ts=NOW - SEC, decision_orig_scheduled_ts=NOW - SEC)

    def check(e, live, tasks, ctx):
        expect_common(e)
        # ReplicateDecisionTaskStartedEvent(nil, 1, 111, 130, requestID, ts): attempt forced to 0 (:223)
        assert (int(e["decision_schedule_id"]), int(e["decision_started_id"]), int(e["decision_attempt"])) == (111, EV_ID, 0)
        assert int(e["decision_started_ts"]) == NOW and int(e["decision_request_src"]) == EV_ID - 1   # RequestID of this event
        assert [(int(x["kind"]), int(x["event_id"]), int(x["visibility_ts"])) for x in tasks] == \
            [(TK.DecisionTimeout, 111, NOW + 11 * SEC)]                       # GenerateDecisionStartTasks(111)
    return Kat("DecisionTaskStarted", f"{SB}:704", [[event(ET.DecisionTaskStarted, scheduled_event_id=111)]],
               State(exec=st), check)


def _decision_failed(name, line, t, **attrs):
    st = running(decision_version=VERSION, decision_schedule_id=12, decision_started_id=28, decision_timeout=11,
                 decision_attempt=0)

    def check(e, live, tasks, ctx):
        expect_common(e)
        # Replicate{TimedOut,Failed} -> FailDecision(true) (attempt + 1); ReplicateTransientDecisionTaskScheduled
        # (:168-197): ScheduleID = NextEventID (the mock's 233 stands for it), Version = currentVersion,
        # DecisionTimeout = DecisionStartToCloseTimeout, ScheduledTimestamp = Now()
        assert int(e["decision_attempt"]) == 1
        assert (int(e["decision_schedule_id"]), int(e["decision_version"])) == (EV_ID, VERSION)
        assert int(e["decision_timeout"]) == 11 and int(e["decision_scheduled_ts"]) == ctx["now_ns"]
        assert int(e["decision_started_id"]) == abi.EMPTY_EVENT_ID
        assert tasks_of(tasks) == [(TK.Decision, EV_ID)]                      # GenerateDecisionScheduleTasks(newScheduleID)
    return Kat(name, f"{SB}:{line}", [[event(t, **attrs)]], State(exec=st), check)


def _decision_completed():
    st = running(decision_version=VERSION, decision_schedule_id=12, decision_started_id=28, decision_timeout=11)

    def extra(e, live, ctx):
        # ReplicateDecisionTaskCompletedEvent -> DeleteDecision + LastProcessedEvent = StartedEventID (:827-838)
        assert int(e["decision_schedule_id"]) == abi.EMPTY_EVENT_ID and int(e["decision_started_id"]) == abi.EMPTY_EVENT_ID
        assert int(e["last_processed_event"]) == 28 and int(e["decision_version"]) == abi.EMPTY_VERSION
    return no_task_case("DecisionTaskCompleted", 843,
                        [event(ET.DecisionTaskCompleted, scheduled_event_id=12, started_event_id=28)], State(exec=st), extra)


def _timer_started():
    def check(e, live, tasks, ctx):
        expect_common(e)
        t = live["timer"]
        assert len(t) == 1
        # ReplicateTimerStartedEvent: TimerInfo{1, "timer ID", ts + 10 s, 130, TimerTaskStatusNone}; the epilogue's
        # GenerateUserTimerTasks then creates its timer task (mockUpdateVersion)
        assert (int(t[0]["version"]), int(t[0]["started_id"]), int(t[0]["expiry_time"])) == (VERSION, EV_ID, NOW + 10 * SEC)
        assert ctx["key"](int(t[0]["key"])) == "timer ID"
        assert int(t[0]["task_status"]) == 1                                  # TimerTaskStatusCreated
        assert [(int(x["kind"]), int(x["event_id"]), int(x["visibility_ts"])) for x in tasks] == \
            [(TK.UserTimer, EV_ID, NOW + 10 * SEC)]
    return Kat("TimerStarted", f"{SB}:877",
               [[event(ET.TimerStarted, timer_id="timer ID", start_to_fire_timeout_seconds=10)]], State(exec=running()), check)


def _timer_state():
    return State(exec=running(), timers=[dict(started_id=100, version=VERSION, expiry_time=NOW + 50 * SEC, task_status=1,
                                               key=1, src=99)], keys=["timer ID"])


def _timer_deleted(e, live, ctx):
    assert len(live["timer"]) == 0 and int(e["inconsistencies"]) == 0      # DeleteUserTimer found it


def _act_state(**kw):
    return State(exec=running(), acts=[act_row(100, 1, **kw)], keys=["activity ID"])


def _activity_scheduled():
    def check(e, live, tasks, ctx):
        expect_common(e)
        a = live["act"]
        assert len(a) == 1
        a = a[0]
        # ReplicateActivityTaskScheduledEvent(130, event) -> ActivityInfo (:1029-1047 of the test)
        assert (int(a["version"]), int(a["schedule_id"]), int(a["scheduled_batch_id"])) == (VERSION, EV_ID, EV_ID)
        assert int(a["scheduled_time"]) == NOW and int(a["started_id"]) == abi.EMPTY_EVENT_ID
        assert int(a["started_time"]) == abi.ZERO_TIME and int(a["last_heartbeat_time"]) == abi.ZERO_TIME
        assert (int(a["schedule_to_start"]), int(a["schedule_to_close"]), int(a["start_to_close"]), int(a["heartbeat"])) == \
            (10, 10, 10, 10)
        assert int(a["cancel_request_id"]) == abi.EMPTY_EVENT_ID and not (int(a["flags"]) & abi.ROW_CANCEL_REQUESTED)
        assert ctx["key"](int(a["key"])) == "activity ID"
        # GenerateActivityTransferTasks(event), then GenerateActivityTimerTasks: ScheduleToStart and
        # ScheduleToClose tie at ts + 10 s; the lower timer type (ScheduleToStart) sorts first
        assert [(int(x["kind"]), int(x["event_id"]), int(x["aux"])) for x in tasks] == \
            [(TK.Activity, EV_ID, 0), (TK.ActivityTimeout, EV_ID, abi.TimeoutType.ScheduleToStart)]
        assert int(a["timer_task_status"]) == abi.TTS_SCHEDULE_TO_START
    return Kat("ActivityTaskScheduled", f"{SB}:1007",
               [[event(ET.ActivityTaskScheduled, activity_id="activity ID", schedule_to_start_timeout_seconds=10,
                       schedule_to_close_timeout_seconds=10, start_to_close_timeout_seconds=10,
                       heartbeat_timeout_seconds=10)]], State(exec=running()), check)


def _activity_started():
    def check(e, live, tasks, ctx):   # the event is 131 here (the loaded activity was scheduled as 130's predecessor)
        a = live["act"][0]
        # ReplicateActivityTaskStartedEvent (:2254-2276): Version, StartedID, RequestID, StartedTime,
        # LastHeartBeatUpdatedTime = StartedTime
        assert (int(a["version"]), int(a["started_id"]), int(a["started_time"])) == (VERSION, EV_ID + 1, NOW + 1000)
        assert int(a["last_heartbeat_time"]) == NOW + 1000 and int(a["started_src"]) == EV_ID
        # epilogue: StartToClose (50 s) is now the earliest not-yet-created timer (ScheduleToStart was)
        assert [(int(x["kind"]), int(x["aux"]), int(x["visibility_ts"])) for x in tasks] == \
            [(TK.ActivityTimeout, abi.TimeoutType.StartToClose, NOW + 1000 + 50 * SEC)]
    st = _act_state(tts=abi.TTS_SCHEDULE_TO_START)
    return Kat("ActivityTaskStarted", f"{SB}:1065",
               [[event(ET.ActivityTaskStarted, i=EV_ID + 1, ts=NOW + 1000, scheduled_event_id=100)]],
               dataclasses.replace(st, exec=running(next_event_id=EV_ID + 1, vh=[(EV_ID, VERSION)], src_next=EV_ID)),
               lambda e, live, tasks, ctx: _act_started_check(e, live, tasks, ctx, check))


def _act_started_check(e, live, tasks, ctx, check):
    assert int(e["status"]) == 0 and int(e["current_version"]) == VERSION
    assert int(e["next_event_id"]) == EV_ID + 2
    check(e, live, tasks, ctx)


def _activity_deleted(e, live, ctx):
    assert len(live["act"]) == 0 and int(e["inconsistencies"]) == 0        # DeleteActivity found it (:1310-1339)


def _activity_cancel_requested():
    def extra(e, live, ctx):
        a = live["act"][0]
        # ReplicateActivityTaskCancelRequestedEvent (:2444-2467), found by ActivityID
        assert int(a["flags"]) & abi.ROW_CANCEL_REQUESTED and int(a["cancel_request_id"]) == EV_ID
        assert int(a["version"]) == VERSION
    return no_task_case("ActivityTaskCancelRequested", 1199,
                        [event(ET.ActivityTaskCancelRequested, activity_id="activity ID")],
                        _act_state(tts=abi.TTS_SCHEDULE_TO_START), extra)


def _child_initiated():
    def check(e, live, tasks, ctx):
        expect_common(e)
        c = live["child"]
        assert len(c) == 1
        # ReplicateStartChildWorkflowExecutionInitiatedEvent(130, event, uuid) -> ChildExecutionInfo
        assert (int(c[0]["version"]), int(c[0]["initiated_id"]), int(c[0]["initiated_batch_id"]), int(c[0]["started_id"])) == \
            (VERSION, EV_ID, EV_ID, abi.EMPTY_EVENT_ID)
        assert tasks_of(tasks) == [(TK.StartChild, EV_ID)]                    # GenerateChildWorkflowTasks(event)
    return Kat("StartChildWorkflowExecutionInitiated", f"{SB}:1284",
               [[event(ET.StartChildWorkflowExecutionInitiated, domain=TARGET_DOMAIN)]], State(exec=running()), check)


def _child_state(started=False):
    return State(exec=running(), children=[dict(initiated_id=100, version=VERSION, initiated_batch_id=99,
                                                started_id=101 if started else abi.EMPTY_EVENT_ID, src=99,
                                                started_src=100 if started else -1)])


def _child_deleted(e, live, ctx):
    assert len(live["child"]) == 0 and int(e["inconsistencies"]) == 0      # DeletePendingChildExecution (:1160-1178)


def _child_started():
    def extra(e, live, ctx):
        c = live["child"][0]
        assert int(c["started_id"]) == EV_ID and int(c["started_src"]) == EV_ID - 1   # ReplicateChildWorkflowExecutionStartedEvent
    return no_task_case("ChildWorkflowExecutionStarted", 1360,
                        [event(ET.ChildWorkflowExecutionStarted, initiated_event_id=100)], _child_state(), extra)


def _initiated(name, line, t, kind, table):
    def check(e, live, tasks, ctx):
        expect_common(e)
        r = live[table]
        assert len(r) == 1
        assert (int(r[0]["version"]), int(r[0]["initiated_id"]), int(r[0]["initiated_batch_id"])) == (VERSION, EV_ID, EV_ID)
        assert tasks_of(tasks) == [(kind, EV_ID)]                             # Generate{RequestCancel,Signal}ExternalTasks
    return Kat(name, f"{SB}:{line}", [[event(t, domain=TARGET_DOMAIN)]], State(exec=running()), check)


def _init_state(table):
    row = dict(initiated_id=100, version=VERSION, initiated_batch_id=99, src=99)
    return State(exec=running(), rcs=[row] if table == "rc" else [], sigs=[row] if table == "sig" else [])


def _init_deleted(table):
    def extra(e, live, ctx):
        assert len(live[table]) == 0 and int(e["inconsistencies"]) == 0    # DeletePending{RequestCancel,Signal}
    return extra


def cases() -> List[Kat]:
    K = []
    K.append(_started_fresh(False))
    K.append(_started_fresh(True))
    for name, line, t, cs in (("WorkflowExecutionTimedOut", 243, ET.WorkflowExecutionTimedOut, abi.CloseStatus.TimedOut),
                              ("WorkflowExecutionTerminated", 273, ET.WorkflowExecutionTerminated, abi.CloseStatus.Terminated),
                              ("WorkflowExecutionFailed", 302, ET.WorkflowExecutionFailed, abi.CloseStatus.Failed),
                              ("WorkflowExecutionCompleted", 332, ET.WorkflowExecutionCompleted, abi.CloseStatus.Completed),
                              ("WorkflowExecutionCanceled", 362, ET.WorkflowExecutionCanceled, abi.CloseStatus.Canceled)):
        K.append(close_case(name, line, t, cs))
    K.append(_can(True))
    K.append(_can(False))
    K.append(no_task_case("WorkflowExecutionSignaled", 544, [event(ET.WorkflowExecutionSignaled)],
                          State(exec=running(signal_count=4)),
                          lambda e, live, ctx: _eq(int(e["signal_count"]), 5)))           # ReplicateWorkflowExecutionSignaled
    K.append(no_task_case("WorkflowExecutionCancelRequested", 571, [event(ET.WorkflowExecutionCancelRequested)],
                          State(exec=running()),
                          lambda e, live, ctx: _eq(int(e["flags"]) & abi.EXEC_CANCEL_REQUESTED, abi.EXEC_CANCEL_REQUESTED)))

    def upsert(e, live, tasks, ctx):
        expect_common(e)
        assert [(int(x["kind"]), int(x["version"])) for x in tasks] == [(TK.UpsertSearchAttributes, VERSION)]
    K.append(Kat("UpsertWorkflowSearchAttributes", f"{SB}:598", [[event(ET.UpsertWorkflowSearchAttributes)]],
                 State(exec=running()), upsert))                                           # GenerateWorkflowSearchAttrTasks
    K.append(no_task_case("MarkerRecorded", 626, [event(ET.MarkerRecorded)], State(exec=running())))
    K.append(_decision_scheduled())
    K.append(_decision_started())
    K.append(_decision_failed("DecisionTaskTimedOut", 752, ET.DecisionTaskTimedOut, timeout_type=0))
    K.append(_decision_failed("DecisionTaskFailed", 798, ET.DecisionTaskFailed))
    K.append(_decision_completed())
    K.append(_timer_started())
    K.append(no_task_case("TimerFired", 918, [event(ET.TimerFired, timer_id="timer ID")], _timer_state(), _timer_deleted))
    K.append(no_task_case("CancelTimerFailed", 948, [event(ET.CancelTimerFailed)], _timer_state()))
    K.append(no_task_case("TimerCanceled", 975, [event(ET.TimerCanceled, timer_id="timer ID")], _timer_state(),
                          _timer_deleted))
    K.append(_activity_scheduled())
    K.append(_activity_started())
    for name, line, t in (("ActivityTaskTimedOut", 1108, ET.ActivityTaskTimedOut),
                          ("ActivityTaskFailed", 1139, ET.ActivityTaskFailed),
                          ("ActivityTaskCompleted", 1169, ET.ActivityTaskCompleted),
                          ("ActivityTaskCanceled", 1252, ET.ActivityTaskCanceled)):
        K.append(no_task_case(name, line, [event(t, scheduled_event_id=100)],
                              _act_state(started_id=101, started=NOW - 50 * SEC, tts=abi.TTS_START_TO_CLOSE),
                              _activity_deleted))
    K.append(_activity_cancel_requested())
    K.append(no_task_case("RequestCancelActivityTaskFailed", 1226, [event(ET.RequestCancelActivityTaskFailed)],
                          _act_state(tts=abi.TTS_SCHEDULE_TO_START)))
    K.append(_child_initiated())
    K.append(no_task_case("StartChildWorkflowExecutionFailed", 1333,
                          [event(ET.StartChildWorkflowExecutionFailed, initiated_event_id=100)], _child_state(),
                          _child_deleted))
    K.append(_child_started())
    for name, line, t in (("ChildWorkflowExecutionTimedOut", 1387, ET.ChildWorkflowExecutionTimedOut),
                          ("ChildWorkflowExecutionTerminated", 1414, ET.ChildWorkflowExecutionTerminated),
                          ("ChildWorkflowExecutionFailed", 1441, ET.ChildWorkflowExecutionFailed),
                          ("ChildWorkflowExecutionCompleted", 1468, ET.ChildWorkflowExecutionCompleted),
                          ("ChildWorkflowExecutionCanceled", 1604, ET.ChildWorkflowExecutionCanceled)):
        K.append(no_task_case(name, line, [event(t, initiated_event_id=100)], _child_state(True), _child_deleted))
    K.append(_initiated("RequestCancelExternalWorkflowExecutionInitiated", 1497,
                        ET.RequestCancelExternalWorkflowExecutionInitiated, TK.CancelExecution, "rc"))
    K.append(no_task_case("RequestCancelExternalWorkflowExecutionFailed", 1550,
                          [event(ET.RequestCancelExternalWorkflowExecutionFailed, initiated_event_id=100)],
                          _init_state("rc"), _init_deleted("rc")))
    K.append(no_task_case("ExternalWorkflowExecutionCancelRequested", 1577,
                          [event(ET.ExternalWorkflowExecutionCancelRequested, initiated_event_id=100)],
                          _init_state("rc"), _init_deleted("rc")))
    K.append(_initiated("SignalExternalWorkflowExecutionInitiated", 1633,
                        ET.SignalExternalWorkflowExecutionInitiated, TK.SignalExecution, "sig"))
    K.append(no_task_case("SignalExternalWorkflowExecutionFailed", 1690,
                          [event(ET.SignalExternalWorkflowExecutionFailed, initiated_event_id=100)],
                          _init_state("sig"), _init_deleted("sig")))
    K.append(no_task_case("ExternalWorkflowExecutionSignaled", 1717,
                          [event(ET.ExternalWorkflowExecutionSignaled, initiated_event_id=100)],
                          _init_state("sig"), _init_deleted("sig")))
    return K


def _eq(a, b):
    assert a == b, (a, b)


NOW_INJECTED = NOW + 777                  # timeSource.Now() of every KAT workflow


def build_batch(kats: List[Kat]):
    """One canonical batch holding every case (new-run histories appended), with the loaded states and
    task emission on.  Returns (batch, index of each case's workflow, index of its new run or None)."""
    hs, states, idx, nr_idx = [], [], [], []
    for k in kats:
        idx.append(len(hs))
        hs.append(WorkflowHistory(batches=[list(b) for b in k.batches], now_ns=NOW_INJECTED, retention_days=1,
                                  run_id=f"run-{k.name}", branch_id=f"branch-{k.name}", domain_failover_version=VERSION))
        states.append(k.state)
    for i, k in enumerate(kats):
        if k.new_run is None:
            nr_idx.append(None)
            continue
        nr_idx.append(len(hs))
        can = hs[idx[i]].batches[-1][-1]
        can.attrs["new_run"] = len(hs)
        hs.append(WorkflowHistory(batches=[list(b) for b in k.new_run], now_ns=NOW_INJECTED, is_new_run=True,
                                  run_id=f"newrun-{k.name}", branch_id="nb", domain_failover_version=VERSION))
        states.append(None)
    loaded = loaded_states(states)
    b = flatten(hs, known_domains=KNOWN, loaded=loaded, interners=loaded.interners)
    b.emit_tasks = True
    return b, idx, nr_idx


def check_all(kats: List[Kat], batch, res, idx, nr_idx):
    """Run every case's expectations against a replay result of build_batch()'s batch."""
    failures = []
    for k, w, nw in zip(kats, idx, nr_idx):
        for ww, fn in ((w, k.check), (nw, k.check_new_run)):
            if ww is None or fn is None:
                continue
            e = res.exec[ww]
            live = res.live_rows(batch, ww)
            inv = {v: s for s, v in batch.interners[ww].items()}
            ctx = {"now_ns": NOW_INJECTED, "key": lambda key, inv=inv: inv.get(key)}
            try:
                fn(e, live, live["tasks"], ctx)
            except AssertionError as ex:
                failures.append(f"{k.name} ({k.cite}): {ex!r}")
    return failures


# ---- service/history/execution/timer_sequence_test.go:74-231: CreateNextUserTimer / CreateNextActivityTimer
# Each Go test hands the timer sequence a mock whose pending infos are given and whose GetCurrentVersion
# is 999.  Restated: a loaded state holding those infos, one batch [MarkerRecorded] of version 999 (so
# UpdateCurrentVersion makes currentVersion 999), whose per-batch epilogue (state_builder.go:634-640)
# runs CreateNextActivityTimer / CreateNextUserTimer.
TS = "service/history/execution/timer_sequence_test.go"
CUR = 999


def _marker_state(**kw):
    return State(exec=running(next_event_id=1000, last_first_event_id=999, src_next=999, vh=[(999, 5)]), **kw)


def _seq_act(tts, started=False, hb=1):
    st = NOW + 200_000_000 if started else abi.ZERO_TIME
    return dict(schedule_id=234, version=123, scheduled_batch_id=230, scheduled_time=NOW,
                started_id=345 if started else abi.EMPTY_EVENT_ID, started_time=st, cancel_request_id=abi.EMPTY_EVENT_ID,
                sched_src=3, started_src=4 if started else -1, schedule_to_start=10, schedule_to_close=1000,
                start_to_close=100, heartbeat=hb, timer_task_status=tts, key=1, flags=abi.ROW_LIVE | abi.ROW_MAPPED,
                attempt=12, last_heartbeat_time=abi.ZERO_TIME)


def _seq_timer(status):
    return dict(started_id=456, version=123, expiry_time=NOW + 100 * SEC, task_status=status, key=1, src=5)


def _timer_kat(name, line, state, want_tasks, after):
    def check(e, live, tasks, ctx):
        assert int(e["status"]) == 0 and int(e["current_version"]) == CUR
        got = [(int(t["kind"]), int(t["aux"]), int(t["version"]), int(t["visibility_ts"]), int(t["event_id"]),
                int(t["attempt"])) for t in tasks]
        assert got == want_tasks, got
        after(live)
    return Kat(name, f"{TS}:{line}", [[event(ET.MarkerRecorded, i=1000, v=CUR)]], state, check)


def timer_cases() -> List[Kat]:
    K = []
    K.append(_timer_kat("CreateNextUserTimer_AlreadyCreated", 74, _marker_state(timers=[_seq_timer(1)], keys=["some random timer ID"]),
                        [], lambda live: _eq(int(live["timer"][0]["task_status"]), 1)))
    # UpdateUserTimer(TaskStatus = Created) + AddTimerTasks(UserTimerTask{ExpiryTime, StartedID, currentVersion})
    K.append(_timer_kat("CreateNextUserTimer_NotCreated", 91, _marker_state(timers=[_seq_timer(0)], keys=["some random timer ID"]),
                        [(TK.UserTimer, 0, CUR, NOW + 100 * SEC, 456, 0)],
                        lambda live: _eq(int(live["timer"][0]["task_status"]), 1)))
    both = abi.TTS_SCHEDULE_TO_CLOSE | abi.TTS_SCHEDULE_TO_START
    K.append(_timer_kat("CreateNextActivityTimer_AlreadyCreated", 121,
                        _marker_state(acts=[_seq_act(both)], keys=["some random activity ID"]), [],
                        lambda live: _eq(int(live["act"][0]["timer_task_status"]), both)))
    # UpdateActivity(TimerTaskStatus = CreatedScheduleToStart) + ActivityTimeoutTask{ScheduledTime + 10 s,
    # ScheduleToStart, ScheduleID, Attempt 12, currentVersion}
    K.append(_timer_kat("CreateNextActivityTimer_NotCreated", 146,
                        _marker_state(acts=[_seq_act(0)], keys=["some random activity ID"]),
                        [(TK.ActivityTimeout, abi.TimeoutType.ScheduleToStart, CUR, NOW + 10 * SEC, 234, 12)],
                        lambda live: _eq(int(live["act"][0]["timer_task_status"]), abi.TTS_SCHEDULE_TO_START)))
    hb_vis = NOW + 200_000_000 + 1 * SEC

    def hb_after(live):
        a = live["act"][0]
        _eq(int(a["timer_task_status"]), abi.TTS_HEARTBEAT)
        _eq(int(a["last_hb_timeout_vis_s"]), hb_vis // SEC)     # LastHeartbeatTimeoutVisibilityInSeconds = .Unix()
    K.append(_timer_kat("CreateNextActivityTimer_HeartbeatTimer", 188,
                        _marker_state(acts=[_seq_act(0, started=True)], keys=["some random activity ID"]),
                        [(TK.ActivityTimeout, abi.TimeoutType.Heartbeat, CUR, hb_vis, 234, 12)], hb_after))
    # LoadAndSortActivityTimers_Multiple (:567-644): the first of the sorted sequence is activity 2345's
    # ScheduleToStart (now + 11 s, attempt 21); CreateNextActivityTimer creates exactly that one
    a1 = dict(_seq_act(0, started=True, hb=0), last_heartbeat_time=NOW + 400_000_000)
    a2 = dict(_seq_act(0, hb=6), schedule_id=2345, schedule_to_start=11, schedule_to_close=1001, start_to_close=101,
              attempt=21, key=2, last_heartbeat_time=NOW + 800_000_000)
    K.append(_timer_kat("LoadAndSortActivityTimers_Multiple_first", 567,
                        _marker_state(acts=[a1, a2], keys=["some random activity ID", "other random activity ID"]),
                        [(TK.ActivityTimeout, abi.TimeoutType.ScheduleToStart, CUR, NOW + 11 * SEC, 2345, 21)],
                        lambda live: _eq([int(a["timer_task_status"]) for a in live["act"]], [0, abi.TTS_SCHEDULE_TO_START])))
    # LoadAndSortUserTimers_Multiple (:263-302): 456 (created) sorts before 4567 -> nothing to create
    t2 = dict(started_id=4567, version=1234, expiry_time=NOW + 200 * SEC, task_status=0, key=2, src=6)
    K.append(_timer_kat("LoadAndSortUserTimers_Multiple_first", 263,
                        _marker_state(timers=[_seq_timer(1), t2], keys=["some random timer ID", "other random timer ID"]),
                        [], lambda live: _eq([int(t["task_status"]) for t in live["timer"]], [1, 0])))
    return K


# ---- service/history/execution/mutable_state_builder_test.go: transient decisions on the replay path ----
# prepareTransientDecisionCompletionFirstBatchReplicated (:634-788) replicates Started(1), DecisionTask-
# Scheduled(2), DecisionTaskStarted(3), DecisionTaskFailed, then a transient DecisionTaskScheduled(5,
# attempt 123) + DecisionTaskStarted(6).  The tests then drive the ACTIVE path (AddDecisionTask*Event,
# AddDecisionTaskScheduledEventAsHeartbeat) and assert on the history builder's transient / flushed
# events -- code the replay path never runs.  Restated here is what the replay path does with the same
# histories: the replicated failure after a failover (event version 13 > 12) schedules the transient
# decision with the new currentVersion and NextEventID (ReplicateTransientDecisionTaskScheduled,
# mutable_state_decision_task_manager.go:168-197: "the schedule ID for this decision is guaranteed to be
# wrong ... ReplicateDecisionTaskScheduledEvent will overwrite everything"), and a replicated
# DecisionTaskScheduled after it overwrites every decision field.
MSB = "service/history/execution/mutable_state_builder_test.go"


def _prepare(version=12):
    ts = NOW
    return [[event(ET.WorkflowExecutionStarted, i=1, v=version, ts=ts, execution_start_to_close_timeout_seconds=222,
                   task_start_to_close_timeout_seconds=11),
             event(ET.DecisionTaskScheduled, i=2, v=version, ts=ts, start_to_close_timeout_seconds=11, attempt=0)],
            [event(ET.DecisionTaskStarted, i=3, v=version, ts=ts, scheduled_event_id=2)],
            [event(ET.DecisionTaskFailed, i=4, v=version, ts=ts)],
            [event(ET.DecisionTaskScheduled, i=5, v=version, ts=ts, start_to_close_timeout_seconds=11, attempt=123),
             event(ET.DecisionTaskStarted, i=6, v=version, ts=ts, scheduled_event_id=5)]]


def _failover_case(name, line, t, **attrs):
    def check(e, live, tasks, ctx):
        assert int(e["status"]) == 0
        # the started transient decision had Attempt forced to 0 (:223); FailDecision(true) -> 1
        assert int(e["decision_attempt"]) == 1
        assert (int(e["decision_schedule_id"]), int(e["decision_version"])) == (7, 13)   # NextEventID, currentVersion
        assert int(e["decision_scheduled_ts"]) == ctx["now_ns"] and int(e["decision_timeout"]) == 11
        assert int(e["current_version"]) == 13 and int(e["next_event_id"]) == 8
        assert [(int(x["event_id"]), int(x["version"])) for x in live["vh"]] == [(6, 12), (7, 13)]
        assert tasks_of(tasks)[-1] == (TK.Decision, 7)
    return Kat(name, f"{MSB}:{line}", _prepare() + [[event(t, i=7, v=13, **attrs)]], None, check)


def msb_cases() -> List[Kat]:
    K = []

    def completed(e, live, tasks, ctx):   # :106-134 ReplicateDecisionCompleted after the transient completion
        assert int(e["status"]) == 0 and int(e["decision_schedule_id"]) == abi.EMPTY_EVENT_ID
        assert int(e["last_processed_event"]) == 6 and int(e["decision_attempt"]) == 0
    K.append(Kat("TransientDecisionCompletionFirstBatchReplicated_ReplicateDecisionCompleted", f"{MSB}:106",
                 _prepare() + [[event(ET.DecisionTaskCompleted, i=7, v=12, scheduled_event_id=5, started_event_id=6)]],
                 None, completed))
    K.append(_failover_case("TransientDecisionCompletionFirstBatchReplicated_FailoverDecisionTimeout", 136,
                            ET.DecisionTaskTimedOut, timeout_type=0))
    K.append(_failover_case("TransientDecisionCompletionFirstBatchReplicated_FailoverDecisionFailed", 154,
                            ET.DecisionTaskFailed))

    def sched_changed(e, live, tasks, ctx):   # :535-567: the transient decision after a failure at version 2001
        assert int(e["status"]) == 0
        assert int(e["decision_attempt"]) == 1 and int(e["decision_version"]) == 2001
        assert int(e["decision_schedule_id"]) == 7 and int(e["current_version"]) == 2001
    K.append(Kat("TransientDecisionTaskSchedule_CurrentVersionChanged", f"{MSB}:535",
                 _prepare(2000) + [[event(ET.DecisionTaskFailed, i=7, v=2001)]], None, sched_changed))

    def start_changed(e, live, tasks, ctx):   # :569-632: a replicated DecisionTaskScheduled overwrites the transient one
        assert int(e["status"]) == 0
        assert (int(e["decision_schedule_id"]), int(e["decision_attempt"]), int(e["decision_version"])) == (8, 2, 2001)
        assert int(e["decision_started_id"]) == abi.EMPTY_EVENT_ID and int(e["decision_timeout"]) == 11
    K.append(Kat("TransientDecisionTaskStart_CurrentVersionChanged", f"{MSB}:569",
                 _prepare(2000) + [[event(ET.DecisionTaskFailed, i=7, v=2000)],
                                   [event(ET.DecisionTaskScheduled, i=8, v=2001, start_to_close_timeout_seconds=11,
                                          attempt=2)]], None, start_changed))
    return K
