"""Pin the CPU restatement (oracle) to the reference's own test expectations.

Each test restates a Go unit test of the reference (file:line cited) or a known-answer vector held
in the reference's fixtures.  The oracle is test infrastructure; these tests run without a GPU.
"""
import json
import zlib

import numpy as np
import pytest

from cadence_amd import abi
from cadence_amd.abi import EventType as ET, Status
from cadence_amd.flatten import flatten, interleave
from cadence_amd.history import (HistoryEvent, WorkflowHistory, branch_token_from_archival_signal,
                                 load_json_history, split_batches_by_task_id, thrift_history_branch_token)
from cadence_amd.result import diff_results
from oracle import oracle

ARCHIVAL = "tests/golden/archival_workflow_history_v1.json"


# ---- common/persistence/versionHistory_test.go ------------------------------------------------------
def test_vh_add_or_update_version_increase():  # versionHistory_test.go:156-180
    st, items = oracle.vh_add_or_update([(3, 0), (6, 4)], 8, 5)
    assert st == 0 and items == [(3, 0), (6, 4), (8, 5)]


def test_vh_add_or_update_event_id_increase():  # :182-204
    st, items = oracle.vh_add_or_update([(3, 0), (6, 4)], 8, 4)
    assert st == 0 and items == [(3, 0), (8, 4)]


def test_vh_add_or_update_failed_lower_version():  # :206-216
    st, _ = oracle.vh_add_or_update([(3, 0), (6, 4)], 8, 3)
    assert st == Status.VH_LOWER_VERSION


def test_vh_add_or_update_failed_same_version_event_id_not_increasing():  # :218-231
    assert oracle.vh_add_or_update([(3, 0), (6, 4)], 5, 4)[0] == Status.VH_EVENT_ID_NOT_INCREASING
    assert oracle.vh_add_or_update([(3, 0), (6, 4)], 6, 4)[0] == Status.VH_EVENT_ID_NOT_INCREASING


def test_vh_add_or_update_failed_version_no_increasing():  # :233-249
    for e, v in ((6, 3), (2, 3), (7, 3)):
        assert oracle.vh_add_or_update([(3, 0), (6, 4)], e, v)[0] != 0


def test_vh_new_item_panics():  # versionHistory.go:37-43 (NewVersionHistoryItem panics)
    assert oracle.vh_add_or_update([], -1, 0)[0] == Status.VH_INVALID_ITEM
    assert oracle.vh_add_or_update([], 1, -5)[0] == Status.VH_INVALID_ITEM
    assert oracle.vh_add_or_update([], 1, abi.EMPTY_VERSION)[0] == 0


# ---- common/persistence/workflowExecutionInfo.go:45-165 (no reference unit test pins it) ----------
S, C = abi.State, abi.CloseStatus


@pytest.mark.parametrize("cur,cur_cs,new,cs,ok", [
    (S.Void, C.NONE, S.Completed, C.Failed, True),
    (S.Created, C.NONE, S.Created, C.NONE, True),
    (S.Created, C.NONE, S.Created, C.Completed, False),
    (S.Created, C.NONE, S.Running, C.NONE, True),
    (S.Created, C.NONE, S.Completed, C.Terminated, True),
    (S.Created, C.NONE, S.Completed, C.TimedOut, True),
    (S.Created, C.NONE, S.Completed, C.ContinuedAsNew, True),
    (S.Created, C.NONE, S.Completed, C.Completed, False),
    (S.Created, C.NONE, S.Zombie, C.NONE, True),
    (S.Running, C.NONE, S.Created, C.NONE, False),
    (S.Running, C.NONE, S.Running, C.NONE, True),
    (S.Running, C.NONE, S.Completed, C.Completed, True),
    (S.Running, C.NONE, S.Completed, C.NONE, False),
    (S.Running, C.NONE, S.Zombie, C.Failed, False),
    (S.Completed, C.Failed, S.Completed, C.Failed, True),
    (S.Completed, C.Failed, S.Completed, C.Completed, False),
    (S.Completed, C.Failed, S.Running, C.NONE, False),
    (S.Zombie, C.NONE, S.Zombie, C.NONE, False),        # the quirk SURVEY.md a12 keeps
    (S.Zombie, C.NONE, S.Zombie, C.Failed, True),
    (S.Zombie, C.NONE, S.Running, C.NONE, True),
    (S.Zombie, C.NONE, S.Completed, C.NONE, False),
])
def test_state_transition_matrix(cur, cur_cs, new, cs, ok):
    st, s, c = oracle.update_state(int(cur), int(cur_cs), int(new), int(cs))
    if ok:
        assert st == 0 and (s, c) == (new, cs)
    else:
        assert st == Status.INVALID_STATE_TRANSITION and (s, c) == (cur, cur_cs)


def test_state_transition_unknown_state():
    assert oracle.update_state(int(S.Corrupted), 0, int(S.Running), 0)[0] == Status.UNKNOWN_WORKFLOW_STATE
    assert oracle.update_state(int(S.Created), 0, 9, 0)[0] == Status.UNKNOWN_WORKFLOW_STATE


# ---- service/history/execution/timer_sequence_test.go: see tests/test_timer_sequence_kats.py -------------
NOW = 1_700_000_000_123_456_789
SEC = 1_000_000_000


# ---- end-to-end restatements --------------------------------------------------------------------------
def ev(t, i, v=12, ts=None, **attrs):
    return HistoryEvent(int(t), i, v, NOW + i * SEC if ts is None else ts, 5000 + i, attrs)


def test_state_rebuilder_rebuild():  # state_rebuilder_test.go:224-333 TestRebuild
    target = b"some other random branch token"
    h = WorkflowHistory(batches=[[ev(ET.WorkflowExecutionStarted, 1, task_start_to_close_timeout_seconds=233,
                                     execution_start_to_close_timeout_seconds=123)],
                                 [ev(ET.WorkflowExecutionSignaled, 2)]],
                        final_token=target, rebuild_last_event_id=2, rebuild_last_event_version=12,
                        domain_failover_version=1234)
    b = flatten([h])
    r = oracle.replay(b, 1)
    e = r.exec[0]
    assert e["status"] == 0
    live = r.live_rows(b, 0)
    assert [(int(x["event_id"]), int(x["version"])) for x in live["vh"]] == [(2, 12)]
    assert e["token_src"] == 2
    payload = oracle.payload(b, 0)
    assert target in payload
    # rebuilding to an event in the middle of a batch is rejected (state_rebuilder.go:160-176)
    h.rebuild_last_event_id = 3
    assert oracle.replay(flatten([h]), 1).exec[0]["status"] == Status.REBUILD_LAST_ITEM


def _transient_prefix():  # mutable_state_builder_test.go:634-760 prepareTransientDecisionCompletionFirstBatchReplicated
    return [[ev(ET.WorkflowExecutionStarted, 1, task_start_to_close_timeout_seconds=11,
                execution_start_to_close_timeout_seconds=222),
             ev(ET.DecisionTaskScheduled, 2, start_to_close_timeout_seconds=11, attempt=0)],
            [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
            [ev(ET.DecisionTaskFailed, 4)]]


def test_transient_decision_after_failure():  # mutable_state_decision_task_manager.go:168-197, :643-676
    now = 777
    h = WorkflowHistory(batches=_transient_prefix(), now_ns=now)
    r = oracle.replay(flatten([h]), 1).exec[0]
    assert r["decision_attempt"] == 1                      # FailDecision(true): attempt + 1
    assert r["decision_schedule_id"] == 4                  # transient: ScheduleID = NextEventID of prev batch
    assert r["decision_version"] == 12                     # currentVersion
    assert r["decision_timeout"] == 11                     # DecisionStartToCloseTimeout
    assert r["decision_scheduled_ts"] == now               # timeSource.Now()
    assert r["decision_started_id"] == abi.EMPTY_EVENT_ID
    assert r["next_event_id"] == 5


def test_transient_decision_completion_first_batch_replicated():  # mutable_state_builder_test.go:106-134
    b = _transient_prefix() + [[ev(ET.DecisionTaskScheduled, 5, start_to_close_timeout_seconds=11, attempt=123),
                                ev(ET.DecisionTaskStarted, 6, scheduled_event_id=5)],
                               [ev(ET.DecisionTaskCompleted, 7, scheduled_event_id=5, started_event_id=6)]]
    r = oracle.replay(flatten([WorkflowHistory(batches=b)]), 1).exec[0]
    assert r["status"] == 0
    assert r["decision_attempt"] == 0                      # started: attempt forced to 0 (:223)
    assert r["decision_schedule_id"] == abi.EMPTY_EVENT_ID
    assert r["last_processed_event"] == 6


def test_update_current_version_workflow_closed():  # mutable_state_builder_test.go:801-812
    b = [[ev(ET.WorkflowExecutionStarted, 1, v=5), ev(ET.DecisionTaskScheduled, 2, v=5)],
         [ev(ET.WorkflowExecutionTerminated, 3, v=7)],
         [ev(ET.MarkerRecorded, 4, v=9)]]
    r = oracle.replay(flatten([WorkflowHistory(batches=b)]), 1).exec[0]
    # closed: currentVersion = last write version (VH last item) even for a higher event version
    assert r["current_version"] == 7


def test_activity_scheduled_dispatch():  # state_builder_test.go:1007-1063 (ActivityScheduled expectations)
    b = [[ev(ET.WorkflowExecutionStarted, 1), ev(ET.DecisionTaskScheduled, 2)],
         [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
         [ev(ET.DecisionTaskCompleted, 4, started_event_id=3),
          ev(ET.ActivityTaskScheduled, 5, activity_id="a", schedule_to_start_timeout_seconds=10,
             schedule_to_close_timeout_seconds=20, start_to_close_timeout_seconds=30, heartbeat_timeout_seconds=0)]]
    bt = flatten([WorkflowHistory(batches=b)])
    r = oracle.replay(bt, 1)
    act = r.live_rows(bt, 0)["act"]
    assert len(act) == 1
    a = act[0]
    assert a["schedule_id"] == 5 and a["scheduled_batch_id"] == 4   # ScheduledEventBatchID = firstEvent.ID
    assert a["started_id"] == abi.EMPTY_EVENT_ID and a["started_time"] == abi.ZERO_TIME
    assert a["cancel_request_id"] == abi.EMPTY_EVENT_ID
    # the epilogue created the earliest timer: ScheduleToStart (10 s) before ScheduleToClose (20 s)
    assert a["timer_task_status"] == abi.TTS_SCHEDULE_TO_START
    assert r.exec[0]["last_first_event_id"] == 4 and r.exec[0]["next_event_id"] == 6


def test_duplicate_activity_id_mapping():  # mutable_state_builder.go:1310-1339 delete-by-older semantics
    b = [[ev(ET.WorkflowExecutionStarted, 1), ev(ET.DecisionTaskScheduled, 2)],
         [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
         [ev(ET.DecisionTaskCompleted, 4, started_event_id=3),
          ev(ET.ActivityTaskScheduled, 5, activity_id="dup"), ev(ET.ActivityTaskScheduled, 6, activity_id="dup")],
         [ev(ET.ActivityTaskCompleted, 7, scheduled_event_id=5)],          # removes the ID mapping of 6
         [ev(ET.ActivityTaskCancelRequested, 8, activity_id="dup")],        # no longer found: no-op
         [ev(ET.ActivityTaskCompleted, 9, scheduled_event_id=6)]]          # mapping missing: inconsistency
    bt = flatten([WorkflowHistory(batches=b)])
    r = oracle.replay(bt, 1).exec[0]
    assert r["status"] == 0 and r["n_activity"] == 0 and r["inconsistencies"] == 1


def test_unknown_event_type_and_empty_batch():
    b = [[ev(ET.WorkflowExecutionStarted, 1)], [ev(77, 2)]]
    r = oracle.replay(flatten([WorkflowHistory(batches=b)]), 1).exec[0]
    assert r["status"] == Status.UNKNOWN_EVENT_TYPE and r["fail_step"] == 1
    b = [[ev(ET.WorkflowExecutionStarted, 1)], []]
    r = oracle.replay(flatten([WorkflowHistory(batches=b)]), 1).exec[0]
    assert r["status"] == Status.EMPTY_HISTORY and r["fail_step"] == 1


# ---- thrift binary conventions: the reference's own branch-token bytes --------------------------------
def test_branch_token_kat_from_archival_fixture():
    events = load_json_history(ARCHIVAL)
    tok = branch_token_from_archival_signal(events, ARCHIVAL)
    assert len(tok) == 96
    assert tok == thrift_history_branch_token("f2b360a0-d90a-4afa-ad88-ba041fad6a42",
                                              "840307b9-9076-4ee2-82a0-45f21d61d719")


def test_checksum_crc_matches_zlib_and_layout():
    events = load_json_history(ARCHIVAL)
    h = WorkflowHistory(batches=split_batches_by_task_id(events), run_id="f2b360a0-d90a-4afa-ad88-ba041fad6a42",
                        branch_id="840307b9-9076-4ee2-82a0-45f21d61d719")
    b = flatten([h])
    r = oracle.replay(b, 1).exec[0]
    p = oracle.payload(b, 0)
    assert r["payload_len"] == len(p)
    assert zlib.crc32(p) == r["checksum"] == oracle.crc32(p)
    assert p[:4] == b"\x59\x02\x00\x0a"                    # preamble + CancelRequested field header
    # NextEventID field (24) carries 113 for the 112-event history
    i = p.index(b"\x0a\x00\x18")
    assert int.from_bytes(p[i + 3:i + 11], "big") == 113
    assert p.endswith(b"\x00\x00\x00\x00")                  # item, history, histories, payload stops


def test_archival_history_replay_summary():
    events = load_json_history(ARCHIVAL)
    h = WorkflowHistory(batches=split_batches_by_task_id(events))
    b = flatten([h])
    r = oracle.replay(b, 1)
    e = r.exec[0]
    assert e["status"] == 0 and e["state"] == abi.State.Running
    assert e["signal_count"] == 11 and e["next_event_id"] == 113
    timers = r.live_rows(b, 0)["timer"]
    assert len(timers) == 1 and timers[0]["started_id"] == 7 and timers[0]["task_status"] == 1
    assert timers[0]["expiry_time"] == 1569606123634180000 + 1296000 * SEC


def test_canonical_vs_interleaved_layout_identical():
    from cadence_amd import synth_mixed
    hs = synth_mixed.mixed_histories(500, 3, multi_version=True, invalid_rate=0.2, can_rate=0.5)
    b = flatten(hs, known_domains={"domain-a", "domain-b", "parent-domain"})
    want = oracle.replay(b, 2)
    for th in (None, 0, 40):   # all lanes, all wave tail, mixed
        ib = interleave(b, long_threshold=th)
        assert not diff_results(b, want, ib, oracle.replay(ib, 2)), th


def test_rebuild_refresh_tasks_reselects_timers():  # mutable_state_task_refresher.go:278-365 (RefreshTasks)
    # activity A (ScheduleToStart 100 s) gets its timer task in batch 3; activity B (10 s, scheduled
    # later) gets the next one in batch 4, so both carry a mask after replay.  RefreshTasks clears
    # every mask and re-creates only the earliest timer of the sequence: B's.
    b = [[ev(ET.WorkflowExecutionStarted, 1), ev(ET.DecisionTaskScheduled, 2)],
         [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
         [ev(ET.DecisionTaskCompleted, 4, started_event_id=3),
          ev(ET.ActivityTaskScheduled, 5, activity_id="A", schedule_to_start_timeout_seconds=100,
             schedule_to_close_timeout_seconds=1000),
          ev(ET.TimerStarted, 6, timer_id="t-late", start_to_fire_timeout_seconds=500),
          ev(ET.DecisionTaskScheduled, 7)],
         [ev(ET.DecisionTaskStarted, 8, scheduled_event_id=7)],
         [ev(ET.DecisionTaskCompleted, 9, started_event_id=8),
          ev(ET.ActivityTaskScheduled, 10, activity_id="B", schedule_to_start_timeout_seconds=10,
             schedule_to_close_timeout_seconds=1000),
          ev(ET.TimerStarted, 11, timer_id="t-early", start_to_fire_timeout_seconds=20)]]
    h = WorkflowHistory(batches=b)
    plain = oracle.replay(flatten([h]), 1)
    act = plain.live_rows(flatten([h]), 0)["act"]
    assert [int(a["timer_task_status"]) for a in act] == [abi.TTS_SCHEDULE_TO_START, abi.TTS_SCHEDULE_TO_START]
    tim = plain.live_rows(flatten([h]), 0)["timer"]
    assert [int(t["task_status"]) for t in tim] == [1, 1]
    h.refresh_tasks = True
    bt = flatten([h])
    r = oracle.replay(bt, 1)
    live = r.live_rows(bt, 0)
    assert [int(a["timer_task_status"]) for a in live["act"]] == [0, abi.TTS_SCHEDULE_TO_START]
    assert [int(t["task_status"]) for t in live["timer"]] == [0, 1]
    assert r.exec[0]["checksum"] == plain.exec[0]["checksum"]   # the checksum does not cover timer masks


# ---- service/history/execution/state_builder_test.go:143-1749: the dispatch table ----------------------
def test_state_builder_dispatch_table_kats():
    """All 45 state_builder_test.go cases (tests/kat_state_builder.py): one ApplyEvents batch onto the
    case's loaded state, the Replicate* effects and Generate* tasks each Go test expects."""
    import kat_state_builder as K
    kats = K.cases()
    assert len(kats) == 44            # + TestApplyEventsNewEventsNotHandled below
    batch, idx, nr = K.build_batch(kats)
    res = oracle.replay(batch, 1)
    fails = K.check_all(kats, batch, res, idx, nr)
    assert not fails, "\n".join(fails)


def test_event_type_count():  # state_builder_test.go:1744-1749 TestApplyEventsNewEventsNotHandled
    assert len(ET) == 42 == abi.EV_TYPE_COUNT


def test_mutable_state_builder_transient_decision_kats():   # mutable_state_builder_test.go:106-177, :535-632
    import kat_state_builder as K
    kats = K.msb_cases()
    batch, idx, nr = K.build_batch(kats)
    res = oracle.replay(batch, 1)
    fails = K.check_all(kats, batch, res, idx, nr)
    assert not fails, "\n".join(fails)
