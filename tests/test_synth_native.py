"""The native full-size workload generator (synth_native.cpp): deterministic, flattened like the
decoder / flatten.py, and replayable by the oracle with the distributions the Python generator has."""
import collections

import numpy as np

from cadence_amd import abi, synth_native
from cadence_amd.flatten import live_set_bounds
from cadence_amd.result import diff_results
from oracle import oracle


def test_deterministic_across_thread_counts():
    a = synth_native.mixed(3000, seed=5, invalid_rate=0.2, can_rate=0.5, multi_version=True, n_threads=1)
    b = synth_native.mixed(3000, seed=5, invalid_rate=0.2, can_rate=0.5, multi_version=True, n_threads=7)
    for k in a.cols:
        assert (a.cols[k] == b.cols[k]).all(), k
    assert (a.wf == b.wf).all() and (a.arena == b.arena).all() and (a.key_arena == b.key_arena).all()


def test_mixed_covers_every_outcome():
    b = synth_native.mixed(6000, seed=6, invalid_rate=0.25, can_rate=0.5, multi_version=True,
                           unknown_domain_rate=0.005)
    r = oracle.replay(b, 0)
    st = collections.Counter(int(s) for s in r.exec["status"])
    assert st[0] > 0.6 * b.n_wf and len(st) >= 10, st
    t = b.cols["etype"] & abi.ETYPE_MASK
    assert len(np.unique(t)) == abi.EV_TYPE_COUNT + 1               # every type + the unknown one
    assert (b.wf["flags"] & abi.WF_FLAG_NEW_RUN).any()
    assert (r.exec["n_vh_items"] > 1).any() and (r.exec["inconsistencies"] > 0).any()
    for name, _dt, _b, cap_f, n_f in abi.TABLES:                    # capacities bound the live sets
        assert (r.exec[n_f] <= b.wf[cap_f]).all(), name


def test_mixed_default_is_all_valid_and_sized_like_config3():
    b = synth_native.mixed(20000)
    r = oracle.replay(b, 0)
    assert (r.exec["status"] == 0).all()
    assert 38 < b.n_events / b.n_wf < 44                             # ~40 events per history
    bd = live_set_bounds(b)
    assert 2.0 < bd["act"].mean() < 3.5 and bd["timer"].max() >= 4


def test_long_tail_shape():
    b = synth_native.long_tail(300, seed=8)
    cnt = b.wf["ev_count"]
    new_run = (b.wf["flags"] & abi.WF_FLAG_NEW_RUN) != 0
    assert cnt[~new_run].max() <= 10_100 and cnt.max() > 5000         # runs cut at run_cap (+ the closing batch)
    can = ((b.cols["etype"] & abi.ETYPE_MASK) == abi.EventType.WorkflowExecutionContinuedAsNew) & (b.cols["aux"] >= 0)
    assert can.sum() == new_run.sum() > 0                             # each CAN event references its new run
    assert new_run[b.cols["aux"][can]].all()
    r = oracle.replay(b, 0)
    assert (r.exec["status"] == 0).all()
    # the walk's concurrency caps bound the maps keyed by ID; a duplicate ActivityID leaves the older
    # activity pending in the mutable state (keyed by ScheduleID) while the walk forgets it
    for f, cap in zip(("n_timer", "n_child", "n_rc", "n_signal"), synth_native.LONG_TAIL_CAPS[1:]):
        assert (r.exec[f] <= cap).all(), f
    assert r.exec["n_activity"].max() > synth_native.LONG_TAIL_CAPS[0]


def test_interleaved_oracle_matches_canonical():
    b = synth_native.mixed(2000, seed=9, invalid_rate=0.2, can_rate=0.5, multi_version=True)
    from cadence_amd.flatten import interleave
    assert not diff_results(b, oracle.replay(b, 0), interleave(b), oracle.replay(interleave(b), 0))
