"""ApplyEvents onto a loaded mutable state (CRR_WF_FLAG_RESUME), CPU side: the oracle's Load
restatement (mutable_state_builder.go:306-349) continued by the replay loop reproduces the one-shot
replay wherever Load reproduces the in-memory state, in both layouts."""
import numpy as np

from cadence_amd import abi, synth_mixed
from cadence_amd.abi import EventType as ET
from cadence_amd.flatten import flatten, interleave
from cadence_amd.history import HistoryEvent, WorkflowHistory
from cadence_amd.result import diff_results
from oracle import oracle

from resume_cases import (KNOWN, compare_split_with_one_shot, load_stable, loaded_from, split_histories)


def _split_run(hs, seed, layout=lambda b: b, last_only=False):
    one_b = flatten(hs, known_domains=KNOWN)
    one = oracle.replay(one_b, 2)
    pre, suf, mask = split_histories(hs, seed, last_only)
    pre_b = layout(flatten(pre, known_domains=KNOWN))
    pre_r = oracle.replay(pre_b, 2)
    loaded = loaded_from(pre_b, pre_r, mask)
    suf_b = layout(flatten(suf, known_domains=KNOWN, loaded=loaded))
    suf_r = oracle.replay(suf_b, 2)
    from cadence_amd.result import to_canonical_order
    return one_b, one, to_canonical_order(pre_b, pre_r), suf_b, suf_r, loaded


def test_resume_matches_one_shot_mixed():
    hs = synth_mixed.mixed_histories(600, 51, multi_version=True, invalid_rate=0.1)
    one_b, one, pre_e, suf_b, suf_r, loaded = _split_run(hs, 1)
    assert loaded.mask.sum() > 300
    stable = load_stable(loaded)
    n = compare_split_with_one_shot(one_b, one, pre_e, suf_b, suf_r, stable)
    assert n > 250
    # the resumed calls' provenance continues the prefix's: src_next covers both parts
    e = suf_r.exec
    m = loaded.mask
    assert (e["src_next"][m] == one.exec["src_next"][m]).all()


def test_resume_interleaved_layout_identical():
    hs = synth_mixed.mixed_histories(400, 52, multi_version=True, invalid_rate=0.2, can_rate=0.5)
    a = _split_run(hs, 2)
    b = _split_run(hs, 2, layout=interleave)
    assert not diff_results(a[3], a[4], b[3], b[4])


def test_resume_last_batch_only():   # one passive-replication task per workflow
    hs = synth_mixed.mixed_histories(300, 53, multi_version=True)
    one_b, one, pre_e, suf_b, suf_r, loaded = _split_run(hs, 3, last_only=True)
    assert compare_split_with_one_shot(one_b, one, pre_e, suf_b, suf_r, load_stable(loaded)) > 150


def ev(t, i, v=7, **attrs):
    return HistoryEvent(int(t), i, v, 1_700_000_000_000_000_000 + i * 1_000_000_000, 900 + i, attrs)


def test_load_remaps_duplicate_activity_ids():
    """Load rebuilds pendingActivityIDToEventID from every loaded ActivityInfo (:311-314): an activity
    whose mapping was dropped in memory by the delete of an older duplicate is mapped again after a
    reload, so a later ActivityTaskCancelRequested finds it (in memory it would not)."""
    prefix = [[ev(ET.WorkflowExecutionStarted, 1), ev(ET.DecisionTaskScheduled, 2)],
              [ev(ET.DecisionTaskStarted, 3, scheduled_event_id=2)],
              [ev(ET.DecisionTaskCompleted, 4, started_event_id=3),
               ev(ET.ActivityTaskScheduled, 5, activity_id="dup"), ev(ET.ActivityTaskScheduled, 6, activity_id="dup")],
              [ev(ET.ActivityTaskCompleted, 7, scheduled_event_id=5)]]
    tail = [[ev(ET.ActivityTaskCancelRequested, 8, activity_id="dup")]]
    h = WorkflowHistory(batches=prefix + tail)
    one = oracle.replay(flatten([h]), 1)
    b1 = flatten([WorkflowHistory(batches=prefix)])
    r1 = oracle.replay(b1, 1)
    assert int(r1.live_rows(b1, 0)["act"]["flags"][0]) & abi.ROW_MAPPED == 0     # in memory: unmapped
    loaded = r1.to_loaded(b1)
    b2 = flatten([WorkflowHistory(batches=tail)], loaded=loaded)
    r2 = oracle.replay(b2, 1)
    a_one = one.live_rows(flatten([h]), 0)["act"][0]
    a_res = r2.live_rows(b2, 0)["act"][0]
    assert not (int(a_one["flags"]) & abi.ROW_CANCEL_REQUESTED)                  # one-shot: not found
    assert int(a_res["flags"]) & abi.ROW_CANCEL_REQUESTED and a_res["cancel_request_id"] == 8
    assert r2.exec[0]["current_version"] == 7 and r2.exec[0]["src_next"] == 8


def test_resume_empty_batch_keeps_loaded_state():
    """ApplyEvents with an empty history on a loaded state (state_builder.go:98-100): error, state
    untouched, currentVersion left at Load's EmptyVersion."""
    prefix = [[ev(ET.WorkflowExecutionStarted, 1), ev(ET.DecisionTaskScheduled, 2)]]
    b1 = flatten([WorkflowHistory(batches=prefix)])
    r1 = oracle.replay(b1, 1)
    b2 = flatten([WorkflowHistory(batches=[[]])], loaded=r1.to_loaded(b1))
    r2 = oracle.replay(b2, 1).exec[0]
    assert r2["status"] == abi.Status.EMPTY_HISTORY and r2["fail_step"] == 2
    assert r2["current_version"] == abi.EMPTY_VERSION
    assert r2["next_event_id"] == 3 and r2["decision_schedule_id"] == 2


def test_resumed_tiering_follows_the_loaded_id_window():
    """A resumed workflow takes a compact tier when its live loaded IDs fit the virtual-step window
    [NextEventID - vk, NextEventID), vk = COMPACT_MAX_EVENTS - ev_count (CompactTables::load), however long
    its history: the same states shifted 5000 event IDs later keep their tiers, and a live entry older than
    the window sends its workflow to the HBM-row segment."""
    import dataclasses
    from cadence_amd import flatten as fl
    hs = synth_mixed.mixed_histories(300, 54, multi_version=True)
    pre, suf, mask = split_histories(hs, 4, last_only=True)
    pre_b = flatten(pre, known_domains=KNOWN)
    loaded = loaded_from(pre_b, oracle.replay(pre_b, 2), mask)
    suf_b = flatten(suf, known_domains=KNOWN, loaded=loaded)
    resumed = (suf_b.wf["flags"] & abi.WF_FLAG_RESUME) != 0
    bounds = fl.live_set_bounds(suf_b)
    _, base = fl.resumed_bounds(suf_b, bounds, resumed)
    with_act = resumed & (loaded.counts("act") > 0)
    assert with_act.sum() > 20 and (base[with_act] < fl.WIDE).any()
    # every loaded ID and NextEventID 5000 later: the window moves with them
    ex = loaded.exec.copy()
    ex["next_event_id"][loaded.mask] += 5000
    rows = {n: r.copy() for n, r in loaded.rows.items()}
    for n, f in fl.LOADED_ID.items():
        if n in rows and len(rows[n]):
            rows[n][f] += 5000
    shifted = dataclasses.replace(suf_b, init=dataclasses.replace(loaded, exec=ex, rows=rows))
    _, t2 = fl.resumed_bounds(shifted, bounds, resumed)
    assert (t2 == base).all()
    # one live activity older than the window
    c = loaded.counts("act")
    off = np.cumsum(c) - c
    w = int(np.nonzero(with_act & (base < fl.WIDE))[0][0])
    rows2 = {n: r.copy() for n, r in loaded.rows.items()}
    vk = fl.COMPACT_MAX_EVENTS - int(suf_b.wf["ev_count"][w])
    rows2["act"]["schedule_id"][off[w]] = int(loaded.exec["next_event_id"][w]) - vk - 1
    old = dataclasses.replace(suf_b, init=dataclasses.replace(loaded, rows=rows2))
    _, t3 = fl.resumed_bounds(old, bounds, resumed)
    assert t3[w] == fl.WIDE
    t3[w] = base[w]
    assert (t3 == base).all()
