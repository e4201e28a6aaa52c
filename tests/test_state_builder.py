"""The host mirror of the Go interfaces (cadence_amd.state_builder), read like the reference's tests.

Each test runs twice: against the oracle on the CPU (``engine="oracle"``, test infrastructure
standing in for the device so the host logic -- staging, materialisation, error mapping -- is
covered without a GPU) and through the HIP library on a MI355X (``engine="device"``, marked gpu).
Expectations restate the reference's unit tests (file:line cited).
"""
import pytest

from cadence_amd import abi
from cadence_amd.abi import EventType as ET, Status
from cadence_amd.history import HistoryEvent, WorkflowHistory, thrift_history_branch_token
from cadence_amd.state_builder import (BadRequestError, BatchStateBuilder, EntityNotExistsError,
                                       InternalFailureError, InternalServiceError, StateBuilder, rebuild)

SEC = 1_000_000_000
NOW = 1_600_000_000 * SEC


class OracleEngine:
    """Test stand-in for ReplayEngine: same replay(batch) -> ReplayResult contract, run by the oracle."""

    def replay(self, batch):
        from oracle import oracle
        return oracle.replay(batch, 1)


@pytest.fixture(params=["oracle", pytest.param("device", marks=pytest.mark.gpu)])
def engine(request):
    if request.param == "oracle":
        return OracleEngine()
    from cadence_amd.engine import ReplayEngine
    return ReplayEngine(0)


def ev(t, i, v=12, ts=None, **attrs):
    return HistoryEvent(int(t), i, v, NOW + i * SEC if ts is None else ts, 5000 + i, attrs)


def test_rebuild(engine):  # state_rebuilder_test.go:224-333 TestRebuild
    target = b"some other random branch token"
    batches = [[ev(ET.WorkflowExecutionStarted, 1, task_start_to_close_timeout_seconds=233,
                   execution_start_to_close_timeout_seconds=123)],
               [ev(ET.WorkflowExecutionSignaled, 2, signal_name="some random signal name")]]
    ms, size = rebuild(batches, target, 2, 12, "request-id", domain_failover_version=1234,
                       domain_id="target-domain", workflow_id="other random workflow ID", run_id="target-run",
                       now_ns=NOW + 99, batch_builder=BatchStateBuilder(engine), history_sizes=(12345, 67890))
    info = ms.get_execution_info()
    assert (info.domain_id, info.workflow_id, info.run_id) == ("target-domain", "other random workflow ID", "target-run")
    assert size == 12345 + 67890
    vh = ms.get_version_histories().get_current_version_history()
    assert vh.branch_token == target
    assert [(i.event_id, i.version) for i in vh.items] == [(2, 12)]
    assert info.start_timestamp == NOW + 99
    assert info.signal_count == 1 and ms.get_next_event_id() == 3


def test_rebuild_refreshes_timer_tasks(engine):  # state_rebuilder.go:183 RefreshTasks
    batches = [[ev(ET.WorkflowExecutionStarted, 1), ev(ET.DecisionTaskScheduled, 2)],
               [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
               [ev(ET.DecisionTaskCompleted, 4, started_event_id=3),
                ev(ET.ActivityTaskScheduled, 5, activity_id="A", schedule_to_start_timeout_seconds=100,
                   schedule_to_close_timeout_seconds=1000), ev(ET.DecisionTaskScheduled, 6)],
               [ev(ET.DecisionTaskStarted, 7, scheduled_event_id=6)],
               [ev(ET.DecisionTaskCompleted, 8, started_event_id=7),
                ev(ET.ActivityTaskScheduled, 9, activity_id="B", schedule_to_start_timeout_seconds=10,
                   schedule_to_close_timeout_seconds=1000)]]
    ms, _ = rebuild(batches, b"tok", 9, 12, "req", batch_builder=BatchStateBuilder(engine))
    status = {a.activity_id: a.timer_task_status for a in ms.get_pending_activity_infos().values()}
    assert status == {"A": 0, "B": abi.TTS_SCHEDULE_TO_START}


def test_rebuild_to_middle_of_batch_rejected(engine):  # state_rebuilder.go:160-176
    batches = [[ev(ET.WorkflowExecutionStarted, 1), ev(ET.DecisionTaskScheduled, 2)]]
    with pytest.raises(BadRequestError):
        rebuild(batches, b"tok", 1, 12, "req", batch_builder=BatchStateBuilder(engine))


def test_apply_events_empty_history():  # state_builder.go:98-100 (checked before any device work)
    sb = StateBuilder()
    with pytest.raises(InternalFailureError, match="history size being zero"):
        sb.apply_events("d", "r", {"workflow_id": "w", "run_id": "r"}, [])


def _started_decision():
    return [[ev(ET.WorkflowExecutionStarted, 1, task_start_to_close_timeout_seconds=11), ev(ET.DecisionTaskScheduled, 2)],
            [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2, request_id="decision-request")],
            [ev(ET.DecisionTaskCompleted, 4, started_event_id=3, binary_checksum="bin-1")]]


def test_activity_lifecycle(engine):  # state_builder_test.go:1007-1063, mutable_state_builder.go:2142-2276
    sb = StateBuilder(batch_builder=BatchStateBuilder(engine), domain_id="own-domain")
    for b in _started_decision():
        sb.apply_events("own-domain", "req", {}, b)
    sb.apply_events("own-domain", "req", {}, [
        ev(ET.ActivityTaskScheduled, 5, activity_id="act-1", task_list="tl", schedule_to_start_timeout_seconds=10,
           schedule_to_close_timeout_seconds=20, start_to_close_timeout_seconds=30, heartbeat_timeout_seconds=5,
           retry_policy={"expiration_interval_in_seconds": 0})])
    sb.apply_events("own-domain", "req", {}, [ev(ET.ActivityTaskStarted, 6, scheduled_event_id=5, request_id="act-req")])
    ms = sb.get_mutable_state()
    ai, ok = ms.get_activity_by_activity_id("act-1")
    assert ok and ai.schedule_id == 5 and ai.scheduled_event_batch_id == 5
    assert ai.started_id == 6 and ai.request_id == "act-req" and ai.started_time == NOW + 6 * SEC
    assert ai.last_heartbeat_updated_time == ai.started_time
    assert ai.task_list == "tl" and ai.domain_id == "own-domain" and ai.has_retry_policy
    assert (ai.schedule_to_start_timeout, ai.schedule_to_close_timeout, ai.start_to_close_timeout,
            ai.heartbeat_timeout) == (10, 20, 30, 5)
    assert ai.cancel_request_id == abi.EMPTY_EVENT_ID and not ai.cancel_requested
    # reset point for the decision's binary checksum (addBinaryCheckSumIfNotExists, :1911-1974)
    rps = ms.get_execution_info().auto_reset_points
    assert [(p.binary_checksum, p.first_decision_completed_id, p.resettable) for p in rps] == [("bin-1", 4, True)]
    assert ms.get_checksum().version == 1 and len(ms.get_checksum().value) == 4


def test_timer_child_signal_cancel_maps(engine):  # mutable_state_builder.go:3057-3081, :3417-3507, :2760-2905
    sb = StateBuilder(batch_builder=BatchStateBuilder(engine, domain_ids={"other": "other-id"}), run_id="run-x")
    for b in _started_decision():
        sb.apply_events("d", "req", {}, b)
    sb.apply_events("d", "req", {}, [
        ev(ET.TimerStarted, 5, timer_id="t1", start_to_fire_timeout_seconds=60),
        ev(ET.StartChildWorkflowExecutionInitiated, 6, domain="other", workflow_id="child-wf",
           workflow_type={"name": "child-type"}, parent_close_policy=1),
        ev(ET.RequestCancelExternalWorkflowExecutionInitiated, 7),
        ev(ET.SignalExternalWorkflowExecutionInitiated, 8, signal_name="sig", input=b"in", control=b"ctl"),
        ev(ET.DecisionTaskScheduled, 9)])
    sb.apply_events("d", "req", {}, [ev(ET.ChildWorkflowExecutionStarted, 10, initiated_event_id=6, run_id="child-run")])
    ms = sb.get_mutable_state()
    ti, ok = ms.get_user_timer_info("t1")
    assert ok and ti.started_id == 5 and ti.expiry_time == NOW + 5 * SEC + 60 * SEC
    assert ti.task_status == 1                      # the epilogue created its timer task
    assert ms.get_user_timer_info_by_event_id(5)[0] is ti
    ci, ok = ms.get_child_execution_info(6)
    assert ok and ci.started_id == 10 and ci.started_run_id == "child-run" and ci.domain_id == "other-id"
    assert ci.started_workflow_id == "child-wf" and ci.workflow_type_name == "child-type" and ci.parent_close_policy == 1
    assert ci.initiated_event_batch_id == 5 and ci.create_request_id
    assert list(ms.get_pending_request_cancel_external_infos()) == [7]
    si = ms.get_pending_signal_external_infos()[8]
    assert (si.signal_name, si.input, si.control, si.initiated_event_batch_id) == ("sig", b"in", b"ctl", 5)
    assert ms.has_pending_decision() and not ms.has_in_flight_decision()


def test_error_kinds(engine):  # ErrMissingActivityInfo (mutable_state_builder.go:64-65), domain cache
    bb = BatchStateBuilder(engine, domain_ids={"known": "k"})
    base = _started_decision()
    bb.add(WorkflowHistory(batches=base + [[ev(ET.ActivityTaskStarted, 5, scheduled_event_id=99)]]))
    bb.add(WorkflowHistory(batches=base + [[ev(ET.ActivityTaskScheduled, 5, activity_id="a", domain="unknown")]]))
    bb.add(WorkflowHistory(batches=base + [[ev(ET.WorkflowExecutionCompleted, 5)], [ev(77, 6)]]))
    bb.add(WorkflowHistory(batches=base + [[ev(ET.DecisionTaskStarted, 5, scheduled_event_id=42)]]))
    bb.add(WorkflowHistory(batches=base + [[ev(ET.ChildWorkflowExecutionStarted, 5, initiated_event_id=3)]]))
    bb.add(WorkflowHistory(batches=base + [[ev(ET.MarkerRecorded, 5, v=3)]]))
    out = bb.replay()
    assert isinstance(out[0].error, InternalServiceError) and out[0].error.status == Status.MISSING_ACTIVITY_INFO
    assert out[0].error.step == 4
    assert isinstance(out[1].error, EntityNotExistsError)
    assert isinstance(out[2].error, BadRequestError) and out[2].error.message == "Unknown event type"
    assert isinstance(out[3].error, InternalFailureError)
    assert isinstance(out[4].error, InternalServiceError) and out[4].error.status == Status.MISSING_CHILD_INFO
    assert isinstance(out[5].error, BadRequestError) and out[5].error.status == Status.VH_LOWER_VERSION
    # partially applied up to the failing event, no rollback: the completed decision stays processed
    assert out[0].mutable_state.get_previous_started_event_id() == 3


def test_continue_as_new_returns_new_run_state(engine):  # state_builder.go:587-627
    sb = StateBuilder(batch_builder=BatchStateBuilder(engine), run_id="old-run")
    for b in _started_decision():
        sb.apply_events("d", "req", {}, b)
    new_run = [ev(ET.WorkflowExecutionStarted, 1, v=12), ev(ET.DecisionTaskScheduled, 2, v=12)]
    sb.apply_events("d", "req", {}, [ev(ET.WorkflowExecutionContinuedAsNew, 5, new_execution_run_id="new-run")],
                    new_run_history=new_run)
    ms = sb.get_mutable_state()
    assert ms.get_workflow_state_close_status() == (abi.State.Completed, abi.CloseStatus.ContinuedAsNew)
    nr = sb.get_new_run_mutable_state()
    assert nr is not None and nr.get_execution_info().run_id == "new-run"
    assert nr.get_next_event_id() == 3 and nr.get_execution_info().state == abi.State.Running
    tok = nr.get_version_histories().get_current_version_history().branch_token
    assert tok == thrift_history_branch_token("new-run", "branch-id-new")


def test_transient_decision_after_failure(engine):  # mutable_state_decision_task_manager.go:168-197, :643-676
    bb = BatchStateBuilder(engine)
    bb.add(WorkflowHistory(batches=[[ev(ET.WorkflowExecutionStarted, 1, task_start_to_close_timeout_seconds=11),
                                     ev(ET.DecisionTaskScheduled, 2, start_to_close_timeout_seconds=11)],
                                    [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
                                    [ev(ET.DecisionTaskFailed, 4)]], now_ns=777))
    info = bb.replay()[0].mutable_state.get_execution_info()
    assert (info.decision_attempt, info.decision_schedule_id, info.decision_version) == (1, 4, 12)
    assert info.decision_scheduled_timestamp == 777 and info.decision_request_id == "emptyUuid"


def test_many_state_builders_share_one_replay(engine):
    """Callers keep their per-workflow ApplyEvents loop; all workflows of a batch go through one launch."""
    calls = []

    class Counting:
        def replay(self, batch):
            calls.append(batch.n_wf)
            return engine.replay(batch)

    bb = BatchStateBuilder(Counting())
    sbs = []
    for i in range(50):
        sb = StateBuilder(batch_builder=bb, run_id=f"run-{i}")
        for b in _started_decision():
            sb.apply_events("d", "req", {}, b)
        sb.apply_events("d", "req", {}, [ev(ET.WorkflowExecutionSignaled, 5 + j) for j in range(i % 4 + 1)])
        sbs.append(sb)
    states = [sb.get_mutable_state() for sb in sbs]
    assert calls == [50]
    assert [s.get_execution_info().signal_count for s in states] == [i % 4 + 1 for i in range(50)]
    assert all(s.get_execution_info().run_id == f"run-{i}" for i, s in enumerate(states))


def test_generated_tasks_materialised(engine):  # MutableState.GetTransferTasks / GetTimerTasks (mutable_state.go:226-228)
    sb = StateBuilder(batch_builder=BatchStateBuilder(engine))
    for b in _started_decision():
        sb.apply_events("d", "req", {}, b)
    sb.apply_events("d", "req", {}, [ev(ET.ActivityTaskScheduled, 5, activity_id="a", task_list="act-tl",
                                        schedule_to_start_timeout_seconds=10, schedule_to_close_timeout_seconds=20)])
    ms = sb.get_mutable_state()
    kinds = [t.kind for t in ms.get_transfer_tasks()]
    assert kinds == [abi.TaskKind.RecordWorkflowStarted, abi.TaskKind.Decision, abi.TaskKind.Activity]
    assert ms.get_transfer_tasks()[2].task_list == "act-tl" and ms.get_transfer_tasks()[2].event_id == 5
    timers = ms.get_timer_tasks()
    assert [t.kind for t in timers] == [abi.TaskKind.WorkflowTimeout, abi.TaskKind.DecisionTimeout,
                                        abi.TaskKind.ActivityTimeout]
    assert timers[-1].visibility_timestamp == NOW + 5 * SEC + 10 * SEC


def test_state_builder_continues_a_loaded_mutable_state(engine):
    """NewStateBuilder(shard, logger, mutableState) (state_builder.go:73-88) over the state a previous
    replay returned -- what mutableStateBuilder.Load reads back (mutable_state_builder.go:306-349) on the
    passive-replication path (ndc/history_replicator.go:385-460): the remaining batches applied onto it
    give the one-shot replay's state (every workflow whose activity-ID map survives a reload)."""
    import random
    from cadence_amd import synth_mixed
    hs = [h for h in synth_mixed.mixed_histories(80, 21, mean_len=40, multi_version=True) if len(h.batches) >= 2]
    rng = random.Random(5)
    one_bb, pre_bb, res_bb = (BatchStateBuilder(engine=engine) for _ in range(3))

    def builder(h, bb, **kw):
        return StateBuilder(h.domain_failover_version, h.domain_id, h.workflow_id, h.run_id, h.branch_id,
                            now_ns=h.now_ns, batch_builder=bb, **kw)

    ex = {"workflow_id": "", "run_id": ""}
    one, pre, cut = [], [], []
    for h in hs:
        ex = {"workflow_id": h.workflow_id, "run_id": h.run_id}
        k = rng.randint(1, len(h.batches) - 1)
        a, b = builder(h, one_bb), builder(h, pre_bb)
        for bt in h.batches:
            a.apply_events(h.domain_id, h.request_id, ex, bt)
        for bt in h.batches[:k]:
            b.apply_events(h.domain_id, h.request_id, ex, bt)
        one.append(a)
        pre.append(b)
        cut.append(k)
    resumed = []
    for h, b, k in zip(hs, pre, cut):
        try:
            ms = b.get_mutable_state()
        except Exception:
            resumed.append(None)
            continue
        stable = len(ms.pending_activity_id_to_event_id) == len(ms.pending_activity_info_ids)
        r = builder(h, res_bb, mutable_state=ms)
        for bt in h.batches[k:]:
            r.apply_events(h.domain_id, h.request_id, {"workflow_id": h.workflow_id, "run_id": h.run_id}, bt)
        resumed.append(r if stable else None)
    compared = 0
    for a, r in zip(one, resumed):
        if r is None:
            continue
        try:
            ma = a.get_mutable_state()
        except Exception as e:
            with pytest.raises(type(e)):
                r.get_mutable_state()
            continue
        mr = r.get_mutable_state()
        assert mr.get_checksum() == ma.get_checksum()
        assert mr.execution_info == ma.execution_info
        assert mr.get_current_version() == ma.get_current_version()
        assert mr.pending_activity_info_ids == ma.pending_activity_info_ids
        assert mr.pending_timer_info_ids == ma.pending_timer_info_ids
        assert mr.pending_child_execution_info_ids == ma.pending_child_execution_info_ids
        assert mr.pending_request_cancel_info_ids == ma.pending_request_cancel_info_ids
        assert mr.pending_signal_info_ids == ma.pending_signal_info_ids
        assert mr.version_histories == ma.version_histories
        compared += 1
    assert compared > len(hs) // 2


def test_state_builder_rejects_a_state_without_row_image():
    from cadence_amd.state_builder import MutableState
    with pytest.raises(InternalServiceError):
        StateBuilder(mutable_state=MutableState())
