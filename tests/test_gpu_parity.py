"""GPU parity: the HIP engine (through the C ABI) versus the CPU restatement, bit for bit.

Every test replays the same seeded inputs on the device and in the oracle and compares every
execution-row field, every live pending row (activity / timer / child / request-cancel / signal),
every version-history item, every reset point and the CRC32 checksum.  Integer work: bit-exact.
"""
import collections

import numpy as np
import pytest

from cadence_amd import abi, synth, synth_mixed
from cadence_amd.flatten import flatten, interleave
from cadence_amd.history import load_json_history, split_batches_by_task_id, WorkflowHistory
from cadence_amd.result import diff_results

pytestmark = pytest.mark.gpu

KNOWN = {"domain-a", "domain-b", "parent-domain"}
ARCHIVAL = "tests/golden/archival_workflow_history_v1.json"


@pytest.fixture(scope="module")
def engine():
    from cadence_amd.engine import ReplayEngine
    return ReplayEngine(0)


def _oracle():
    from oracle import oracle
    return oracle


def check(engine, batch, threads=0):
    got = engine.replay(batch)
    want = _oracle().replay(batch, threads)
    d = diff_results(batch, got, batch, want)
    assert not d, "\n".join(d)
    return got


def test_c1_activity_chain_interleaved(engine):
    b = interleave(synth.activity_chain(10_000, 3, synth.SEED_C1))
    got = check(engine, b)
    assert (got.exec["status"] == 0).all()
    assert (got.exec["state"] == abi.State.Completed).all()
    assert (got.exec["next_event_id"] == 24).all()


def test_c1_canonical_layout(engine):
    b = synth.activity_chain(2_000, 3, synth.SEED_C1)
    check(engine, b)


def test_mixed_histories_all_event_types(engine):
    hs = synth_mixed.mixed_histories(4000, 11, multi_version=True, invalid_rate=0.25, can_rate=0.5)
    b = flatten(hs, known_domains=KNOWN)
    ib = interleave(b)
    got = check(engine, ib)
    st = collections.Counter(int(s) for s in got.exec["status"])
    # the generator exercises the success path and most error kinds
    assert st[0] > 2000
    assert len(st) >= 8, st
    check(engine, b)  # canonical layout too


def test_mixed_single_version(engine):
    hs = synth_mixed.mixed_histories(3000, 12, multi_version=False, invalid_rate=0.0)
    check(engine, interleave(flatten(hs, known_domains=KNOWN)))


def test_long_histories(engine):
    hs = synth_mixed.mixed_histories(200, 13, mean_len=600, multi_version=True, invalid_rate=0.1)
    b = flatten(hs, known_domains=KNOWN)
    check(engine, interleave(b, long_threshold=None))   # lane per workflow
    ib = interleave(b)                                    # length-bucketed: a wavefront per long history
    assert ib.wave_begin < b.n_wf
    check(engine, ib)


def test_wave_per_workflow_all_event_types(engine):
    """Every workflow of the mixed set replayed one per wavefront (LDS row arenas)."""
    hs = synth_mixed.mixed_histories(3000, 21, multi_version=True, invalid_rate=0.25, can_rate=0.5)
    ib = interleave(flatten(hs, known_domains=KNOWN), long_threshold=0)
    assert ib.wave_begin == 0
    got = check(engine, ib)
    assert len(set(int(s) for s in got.exec["status"])) >= 8


def test_wave_chunks_with_failures(engine):
    """Histories of several 64-event chunks, one per wavefront, most ending in an injected error: the
    chunks after the first resolve their decision events lane-parallel and walk only the map events, so
    failures land inside such chunks (decision not found, missing activity / child, unknown domain,
    version-history checks) as well as in the per-event chunks (rare types)."""
    hs = synth_mixed.mixed_histories(1500, 23, mean_len=300, multi_version=True, invalid_rate=0.6, can_rate=0.3)
    ib = interleave(flatten(hs, known_domains=KNOWN), long_threshold=0)
    assert ib.wave_begin == 0
    got = check(engine, ib)
    st = collections.Counter(int(s) for s in got.exec["status"])
    assert st[0] > 400 and len(st) >= 8, st


def test_long_tail_continue_as_new(engine):
    """Config 4 shape: Zipf lengths, continue-as-new chains.  Unbounded random walks: live sets
    outgrow both LDS arenas, so those workflows go through the HBM-row wavefront pass."""
    hs = synth_mixed.long_tail_histories(300, 7, max_len=5000, run_cap=2000, multi_version=True, invalid_rate=0.1,
                                         caps=None)
    b = flatten(hs, known_domains=KNOWN)
    ib = interleave(b)
    got = check(engine, ib)
    assert (got.exec["status"] == 0).sum() > 0.9 * b.n_wf
    assert got.exec["n_activity"].max() > 64                # beyond the LDS arena
    assert (b.wf["flags"] & abi.WF_FLAG_NEW_RUN).any()


def test_long_tail_bounded_working_set(engine):
    """Config 4 with bounded pending sets (the per-wave LDS arenas), lanes + wavefronts mixed."""
    hs = synth_mixed.long_tail_histories(400, 8, max_len=6000, run_cap=2500, multi_version=True, invalid_rate=0.1)
    b = flatten(hs, known_domains=KNOWN)
    for th in (None, 256, 64):
        check(engine, interleave(b, long_threshold=th))


def test_archival_fixture(engine):
    ev = load_json_history(ARCHIVAL)
    h = WorkflowHistory(batches=split_batches_by_task_id(ev), run_id="f2b360a0-d90a-4afa-ad88-ba041fad6a42",
                        branch_id="840307b9-9076-4ee2-82a0-45f21d61d719", now_ns=1)
    got = check(engine, flatten([h]))
    assert got.exec["status"][0] == 0
    assert got.exec["signal_count"][0] == 11


def test_c2_full_size_bit_exact(engine):
    """Config 2 at full size (1M workflows x 29 events): every row against the oracle."""
    b = interleave(synth.activity_chain(1_000_000, 4, synth.SEED_C2))
    got = check(engine, b)
    assert (got.exec["status"] == 0).all()
    # size-independent property: recomputing checksums from the written rows reproduces them
    db = engine.upload(b)
    engine.launch(db)
    cs = engine.checksum(db)
    assert (cs == got.exec["checksum"]).all()


def test_rebuild_refresh_tasks_all_paths(engine):
    """Rebuild's RefreshTasks (CRR_WF_FLAG_REFRESH_TASKS) on half of the workflows: lane path (small and
    large LDS tiers), wavefront tail and the canonical-layout global path."""
    import random
    rng = random.Random(3)
    for hs in (synth_mixed.mixed_histories(3000, 41, multi_version=True, invalid_rate=0.1, can_rate=0.3),
               synth_mixed.long_tail_histories(60, 42, max_len=3000, run_cap=1500, multi_version=True)):
        for h in hs:
            h.refresh_tasks = rng.random() < 0.5
            h.refresh_jitter = rng.randrange(1 << 40)
        b = flatten(hs, known_domains=KNOWN)
        check(engine, interleave(b))
        check(engine, interleave(b, long_threshold=None))
        check(engine, b)
        # with task emission: RefreshTasks' own tasks (mutable_state_task_refresher.go:77-496) in the rows,
        # search-attributes task on (CRR_IN_ADVANCED_VISIBILITY)
        b.emit_tasks = True
        b.advanced_visibility = True
        for lb in (interleave(b), interleave(b, long_threshold=None), b):
            lb.emit_tasks = True
            lb.advanced_visibility = True
            check(engine, lb)


def test_decoded_blobs_replay_on_device(engine):
    """Persisted thriftrw blobs -> native decoder -> device replay, bit-exact against the oracle."""
    from cadence_amd.decode import WorkflowSource, decode_histories
    from cadence_amd.thrift_codec import serialize_history
    hs = synth_mixed.mixed_histories(2000, 43, multi_version=True, invalid_rate=0.2)
    src = [WorkflowSource(blobs=serialize_history(h), run_id=h.run_id, branch_id=h.branch_id,
                          domain_failover_version=h.domain_failover_version, now_ns=h.now_ns) for h in hs]
    check(engine, interleave(decode_histories(src, known_domains=KNOWN)))


def test_retry_routes(engine):
    """Every route of the retry pass: lane workflows that outgrow the fast tier but fit the 8-slot
    retry tier, lane workflows that outgrow that too (HBM rows, same lane), and long-tail workflows
    whose per-wave arena overflows (wavefront pass)."""
    from cadence_amd.flatten import live_set_bounds
    hs = synth_mixed.mixed_histories(3000, 31, mean_len=90, multi_version=True, invalid_rate=0.1)
    b = flatten(hs, known_domains=KNOWN)
    peak = np.max(np.stack([v for v in live_set_bounds(b).values()]), axis=0)
    assert ((peak > 2) & (peak <= 4)).sum() > 100      # retried, fit the retry tier
    assert (peak > 8).sum() > 10                       # retried, outgrow it
    check(engine, interleave(b, long_threshold=None, tiered=False))   # fast tier, then the retry pass
    tb = interleave(b, long_threshold=None)                            # tier segments: small | large | wide
    assert 0 < tb.tiers[0] <= tb.tiers[1] <= tb.tiers[2] <= tb.tiers[3] < tb.n_wf
    check(engine, tb)
    lt = flatten(synth_mixed.long_tail_histories(120, 9, max_len=3000, run_cap=1200, caps=None),
                 known_domains=KNOWN)
    check(engine, interleave(lt))
    check(engine, interleave(lt, tiered=False))


def test_measured_region_launches(engine):
    """Launches inside crr_timing_begin/_read (the bench's measured region) record one ring event
    pair each and skip the per-call phase events; the rows they leave are the oracle's."""
    import torch
    b = interleave(synth.activity_chain(4_096, 4, synth.SEED_C2))
    db = engine.upload(b)
    engine.launch(db)
    torch.cuda.synchronize()
    assert engine.last_kernel_ms()[2] > 0
    engine.timing_begin()
    for _ in range(3):
        engine.launch(db)
    assert engine.last_kernel_ms() == [-1.0, -1.0, -1.0]
    ms = engine.timing_read()
    assert len(ms) == 3 and all(m > 0 for m in ms)
    got = engine.download(db)
    want = _oracle().replay(b, 0)
    d = diff_results(b, got, b, want)
    assert not d, "\n".join(d)
    engine.launch(db)
    torch.cuda.synchronize()
    assert engine.last_kernel_ms()[2] > 0


def test_config4_long_tail_at_stated_size(engine):
    """BASELINE config 4 at its stated size: histories up to 50k events, continue-as-new every <= 10k
    (native generator), bounded and unbounded pending sets; length-bucketed (wave tail + big-arena
    segment + retry), lanes-only and untiered layouts, every row against the oracle."""
    from cadence_amd import synth_native
    for caps in (synth_native.LONG_TAIL_CAPS, None):
        b = synth_native.long_tail(400, seed=0xCAD00004, max_len=50_000, run_cap=10_000, caps=caps,
                                   multi_version=True, invalid_rate=0.05)
        assert b.wf["ev_count"].max() > 9_000 and b.n_events > 2_000_000
        check(engine, interleave(b))
        check(engine, interleave(b, tiered=False))
    check(engine, interleave(b, long_threshold=None))


def test_config3_native_mixed_shard(engine):
    """Config 3 shape from the native generator (every event type, failover versions, injected errors,
    continue-as-new), 200k workflows, tier segments, against the oracle; plus the all-valid default."""
    from cadence_amd import synth_native
    b = synth_native.mixed(200_000, seed=0xCAD00003, multi_version=True, invalid_rate=0.1, can_rate=0.3,
                           unknown_domain_rate=0.005)
    check(engine, interleave(b))
    got = check(engine, interleave(synth_native.mixed(100_000)))
    assert (got.exec["status"] == 0).all()
