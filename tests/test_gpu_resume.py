"""GPU: ApplyEvents onto loaded mutable states (CRR_WF_FLAG_RESUME) through the C ABI.

Batches 1..k of every history are replayed on the device, downloaded, re-uploaded as the loaded
states, and batches k+1..n are replayed onto them.  The device rows equal the oracle's for the same
split (every workflow, every field, bit-exact), and equal the one-shot device replay wherever Load
reproduces the in-memory state (tests/resume_cases.py).
"""
import numpy as np
import pytest

from cadence_amd import synth_mixed
from cadence_amd.flatten import flatten, interleave
from cadence_amd.result import diff_results, to_canonical_order

from resume_cases import KNOWN, compare_split_with_one_shot, load_stable, loaded_from, split_histories

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from cadence_amd.engine import ReplayEngine
    return ReplayEngine(0)


def _oracle():
    from oracle import oracle
    return oracle


def _device_split(engine, hs, seed, layout, last_only=False):
    one_b = layout(flatten(hs, known_domains=KNOWN))
    one = engine.replay(one_b)
    pre, suf, mask = split_histories(hs, seed, last_only)
    pre_b = layout(flatten(pre, known_domains=KNOWN))
    pre_r = engine.replay(pre_b)                       # device prefix -> downloaded rows
    d = diff_results(pre_b, pre_r, pre_b, _oracle().replay(pre_b, 0))
    assert not d, "\n".join(d)
    loaded = loaded_from(pre_b, pre_r, mask)           # re-uploaded as the loaded states
    suf_b = layout(flatten(suf, known_domains=KNOWN, loaded=loaded))
    suf_r = engine.replay(suf_b)
    want = _oracle().replay(suf_b, 0)                  # the oracle given the same split
    d = diff_results(suf_b, suf_r, suf_b, want)
    assert not d, "\n".join(d)
    n = compare_split_with_one_shot(one_b, one, to_canonical_order(pre_b, pre_r), suf_b, suf_r, load_stable(loaded))
    return loaded, n


@pytest.mark.parametrize("layout", ["interleaved", "canonical", "lanes_only"])
def test_resume_mixed_all_layouts(engine, layout):
    lay = {"interleaved": interleave, "canonical": lambda b: b,
           "lanes_only": lambda b: interleave(b, long_threshold=None)}[layout]
    hs = synth_mixed.mixed_histories(3000, 61, multi_version=True, invalid_rate=0.1, can_rate=0.3)
    loaded, n = _device_split(engine, hs, 5, lay)
    assert loaded.mask.sum() > 1500 and n > 1200


def test_resume_long_histories_wavefront_path(engine):
    """Long resumed histories take the long-tail segment (replay_big_kernel: HBM-row wavefront pass)."""
    hs = synth_mixed.long_tail_histories(150, 62, max_len=4000, run_cap=2000, multi_version=True, caps=None)
    loaded, n = _device_split(engine, hs, 6, interleave)
    assert n > 50


def test_resume_passive_replication_last_batch(engine):
    """One replication task per workflow: the last batch applied onto the loaded state."""
    hs = synth_mixed.mixed_histories(4000, 63, multi_version=True)
    loaded, n = _device_split(engine, hs, 7, interleave, last_only=True)
    assert n > 2500


def test_resume_old_histories_in_the_compact_window(engine):
    """Histories past the compact encodings' 1023 steps whose live loaded entries are recent resume in the
    compact tiers (the virtual-step window [NextEventID - vk, NextEventID), flatten.resumed_bounds); the
    rest take the HBM-row segment, or the general path when CompactTables::load finds an entry outside it."""
    from cadence_amd import abi
    from cadence_amd import flatten as fl
    caps = {"act": 3, "timer": 2, "child": 1, "rc": 1, "sig": 1}  # live sets a compact tier holds
    hs = synth_mixed.long_tail_histories(1000, 64, min_len=200, max_len=3000, run_cap=3000, multi_version=True,
                                         caps=caps)
    pre, suf, mask = split_histories(hs, 8, last_only=True)
    pre_b = interleave(flatten(pre, known_domains=KNOWN))
    loaded = loaded_from(pre_b, engine.replay(pre_b), mask)
    suf_b = flatten(suf, known_domains=KNOWN, loaded=loaded)
    resumed = (suf_b.wf["flags"] & abi.WF_FLAG_RESUME) != 0
    _, tier = fl.resumed_bounds(suf_b, fl.live_set_bounds(suf_b), resumed)
    old = resumed & (loaded.exec["next_event_id"] > fl.COMPACT_MAX_EVENTS)
    assert (old & (tier < fl.WIDE)).sum() > 20 and (old & (tier == fl.WIDE)).sum() > 0
    loaded2, n = _device_split(engine, hs, 8, interleave, last_only=True)
    assert n > 100   # Load-stable and equal to the one-shot replay; every workflow equals the oracle


@pytest.mark.gpu
@pytest.mark.parametrize("native", [False, True])
def test_passive_replication_in_place_matches_one_shot(native):
    """The bench's passive-replication step at test size: every workflow cut before its last batch, the
    prefix replayed, the last batches applied onto the rows left in HBM (CRR_WF_FLAG_RESUME) -- equal
    to the one-shot replay for every Load-stable workflow, checksum included, over two restored steps."""
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.flatten import interleave
    from cadence_amd.replication import PassiveReplication
    eng = ReplayEngine(0)
    if native:
        from cadence_amd import synth_native
        canon = synth_native.mixed(20000, can_rate=0.3)
    else:
        from cadence_amd import synth_mixed
        from cadence_amd.flatten import flatten
        canon = flatten(synth_mixed.mixed_histories(3000, 44, mean_len=120, multi_version=True, can_rate=0.3),
                        known_domains={"domain-a", "domain-b", "parent-domain"})
    b = interleave(canon, long_threshold=150)
    one = eng.replay(b)
    pr = PassiveReplication(eng, b)
    pr.setup()
    for _ in range(2):
        pr.restore()
        pr.step()
    v = pr.verify(one)
    assert v["mismatches"] == 0, v
    assert v["compared_workflows"] > 0.5 * v["split_workflows"] > 0, v   # the rest: failed or not Load-stable
    # every split workflow, the Load-unstable ones too, against the oracle given the same split
    vp = pr.verify_prefix_oracle(_oracle().replay, 0)     # the loaded states themselves
    assert vp["mismatches"] == 0 and vp["compared_workflows"] == b.n_wf, vp
    vo = pr.verify_oracle(_oracle().replay, 0)
    assert vo["mismatches"] == 0, vo
    assert vo["compared_workflows"] >= v["compared_workflows"], vo


def test_inconsistent_loaded_states_route_to_retry_or_capacity(engine):
    """Loaded states the compact tiers cannot continue in LDS (rows out of ID order)
    go to the general path before HBM changes and end equal to the oracle given the same rows; a state
    with more loaded rows than its slot capacity fails CRR_ERR_CAPACITY at step 0 without writing a row
    (the rest of the batch unchanged).  Neither may write outside the workflow's slots."""
    from cadence_amd import abi
    hs = synth_mixed.mixed_histories(4000, 64, multi_version=True)
    pre, suf, mask = split_histories(hs, 8, last_only=True)
    pre_b = interleave(flatten(pre, known_domains=KNOWN))
    loaded = loaded_from(pre_b, engine.replay(pre_b), mask)
    swapped = []
    for name in ("act", "timer", "child"):
        c = loaded.counts(name)
        off = np.cumsum(c) - c
        for w in np.nonzero(c >= 2)[0][:150]:   # slots 0 and 1 exchanged: rows no longer in ID order
            o = int(off[w])
            r = loaded.rows[name]
            r[[o, o + 1]] = r[[o + 1, o]]
            swapped.append(int(w))
    assert len(swapped) > 200
    suf_b = interleave(flatten(suf, known_domains=KNOWN, loaded=loaded))
    got = engine.replay(suf_b)
    want = _oracle().replay(suf_b, 0)
    d = diff_results(suf_b, got, suf_b, want)
    assert not d, "\n".join(d)
    # more loaded activities than act_cap for a few resumed workflows (the exec row's count, as uploaded)
    db = engine.upload(suf_b)
    ex = db.tensors["exec"][:suf_b.n_wf * abi.EXEC_ROW.itemsize].cpu().numpy().view(abi.EXEC_ROW).copy()
    resumed = np.nonzero((suf_b.wf["flags"] & abi.WF_FLAG_RESUME) != 0)[0]
    bad = resumed[:: max(1, resumed.size // 40)][:40]
    ex["n_activity"][bad] = suf_b.wf["act_cap"][bad] + 3
    db.tensors["exec"][:ex.nbytes].copy_(engine.torch.from_numpy(ex.view(np.uint8)))
    engine.launch(db)
    r2 = engine.download(db)
    assert (r2.exec["status"][bad] == abi.Status.CAPACITY).all()
    assert (r2.exec["fail_step"][bad] == ex["src_next"][bad]).all()
    assert (r2.exec["n_activity"][bad] == 0).all()
    keep = np.ones(suf_b.n_wf, bool)
    keep[bad] = False
    for f in ("status", "checksum", "next_event_id", "n_activity", "n_timer", "n_vh_items"):
        assert (r2.exec[f][keep] == got.exec[f][keep]).all(), f
    for name, _dt, *_ in abi.TABLES:   # only the bad workflows' own slots may differ
        if name == "tasks":
            continue
        same = r2.tables[name] == got.tables[name]
        own = np.zeros(same.shape[0], bool)
        base_f, cap_f = {t[0]: (t[2], t[3]) for t in abi.TABLES}[name]
        for w in bad:
            idx = int(suf_b.wf[base_f][w]) + np.arange(int(suf_b.wf[cap_f][w])) * int(suf_b.wf_strides()[w])
            own[idx[idx < own.size]] = True
        assert same[~own].all(), name


@pytest.mark.parametrize("gen", ["native", "python", "long"])
def test_passive_replication_from_blobs_on_device(gen):
    """Passive replication from the task's persisted bytes (replication_task.go:386-390 -> serializer.go:109-119,
    then ApplyEvents onto the loaded state): the last batches' thriftrw blobs, resident in HBM, are decoded and
    laid out on the device (crr_ingest_plan_resume / crr_ingest_layout_resume: keys interned on from the loaded
    dictionaries, the loaded descriptors continued) and replayed onto the loaded rows in place.  The laid-out
    inputs equal the host path's (replication.suffix_batch: every column, the side records each event names,
    the descriptors), and the rows equal the host path's step and the oracle's, bit for bit."""
    import dataclasses
    from cadence_amd import abi, synth_native
    from cadence_amd.blobs import encode_batch
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.replication import BlobReplication, PassiveReplication
    eng = ReplayEngine(0)
    if gen == "native":
        canon = synth_native.mixed(20000, can_rate=0.3, multi_version=True)
    elif gen == "python":
        canon = flatten(synth_mixed.mixed_histories(3000, 45, mean_len=120, multi_version=True, can_rate=0.3,
                                                    invalid_rate=0.05),
                        known_domains={"domain-a", "domain-b", "parent-domain"})
    else:   # long histories: loaded dictionaries past 64 keys take the lane-per-workflow resume pass
        canon = flatten(synth_mixed.long_tail_histories(150, 62, max_len=4000, run_cap=2000, multi_version=True, caps=None),
                        known_domains={"domain-a", "domain-b", "parent-domain"})
    b = interleave(canon, long_threshold=150)
    pr = PassiveReplication(eng, b)
    pr.setup()
    pr.restore()
    pr.step()
    host = eng.download(pr.db)
    br = BlobReplication(pr, encode_batch(canon))
    br.setup()
    for _ in range(2):
        pr.restore()
        S = br.step()
    dev = eng.download(pr.db)
    eng.torch.cuda.synchronize()
    # the inputs the device laid out against the host path's suffix batch
    sb, T = pr.suffix, br.tensors
    n_slots = int(S.n_slots)
    assert n_slots == sb.cols["etype"].size and int(S.n_events) == sb.n_events
    got = {name: T["ev_" + name][:n_slots * np.dtype(t).itemsize].cpu().numpy().view(t) for name, t in abi.EVENT_COLUMNS}
    for name, _t in abi.EVENT_COLUMNS:
        if name != "aux":
            np.testing.assert_array_equal(got[name], sb.cols[name], err_msg=name)
    from cadence_amd.abi import EventType as ET
    et = sb.cols["etype"] & abi.ETYPE_MASK
    g_side = T["act_side"][:int(S.n_act_side) * abi.ACTIVITY_SIDE.itemsize].cpu().numpy().view(abi.ACTIVITY_SIDE)
    sched = et == ET.ActivityTaskScheduled   # the side record it names
    assert sched.sum() > (3 if gen == "long" else 100)
    assert g_side[got["aux"][sched]].tobytes() == sb.act_side[sb.cols["aux"][sched]].tobytes()
    # ActivityTaskStarted joined to a scheduled event of the same new batch (rare in a last batch: the scheduled
    # one is usually in the loaded state, where the replay reads the loaded row)
    started = (et == ET.ActivityTaskStarted) & (got["aux"] >= 0)
    assert g_side[got["aux"][started]].tobytes() == sb.act_side[sb.cols["aux"][started]].tobytes()
    rest = ~np.isin(et, [ET.ActivityTaskScheduled, ET.ActivityTaskStarted, ET.WorkflowExecutionStarted])
    np.testing.assert_array_equal(got["aux"][rest], sb.cols["aux"][rest])
    g_wf = T["loaded_wf"][:b.n_wf * abi.WORKFLOW.itemsize].cpu().numpy().view(abi.WORKFLOW)   # (updated in place)
    assert g_wf.tobytes() == sb.wf.tobytes()
    # the rows: the host path's step, byte for byte
    assert dev.exec.tobytes() == host.exec.tobytes()
    for name, *_r in abi.TABLES:
        if name != "tasks":
            assert dev.tables[name].tobytes() == host.tables[name].tobytes(), name
    vo = pr.verify_oracle(_oracle().replay, 0)
    assert vo["mismatches"] == 0 and vo["compared_workflows"] > 0.5 * int(pr.split.sum()), vo


def test_resume_ingest_seed_scratch_and_bad_blobs():
    """crr_ingest_plan_resume's edges: loaded dictionaries larger than the scratch's table region report
    CRR_INGEST_SCRATCH_TOO_SMALL with the events counted right (DeviceIngest.plan then grows the scratch and the
    step's rows still equal the host path's); a task whose blob is not thriftrw fails the plan as the host
    decoder does (CadenceDeserializationError, serializer.go:320-333), naming that blob."""
    import ctypes
    from cadence_amd import abi
    from cadence_amd.blobs import BlobSet, encode_batch
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.ingest import SCRATCH_TOO_SMALL, CIngestSummary, IngestError
    from cadence_amd.replication import BlobReplication, PassiveReplication
    eng = ReplayEngine(0)
    canon = flatten(synth_mixed.long_tail_histories(150, 62, max_len=4000, run_cap=2000, multi_version=True, caps=None),
                    known_domains={"domain-a", "domain-b", "parent-domain"})
    b = interleave(canon, long_threshold=150)
    pr = PassiveReplication(eng, b)
    pr.setup()
    pr.restore()
    pr.step()
    want = eng.download(pr.db)
    br = BlobReplication(pr, encode_batch(canon))
    br.setup()
    ing, db = br.ing, br.blobs
    n_ev = br.n_events
    assert int(br.tensors["key_count"].cpu().numpy().astype(np.int64).sum()) > 4 * n_ev   # the seeds dominate the table region
    size = int(ing.lib.crr_ingest_scratch_bytes(db.c.n_blobs, db.c.n_wf, n_ev + 1))   # the events fit, the seeds not
    ing.scratch = ing.torch.zeros(size, dtype=ing.torch.uint8, device=eng.dev)
    ing.scratch_bytes = size
    S = CIngestSummary()
    s = eng.torch.cuda.current_stream(eng.dev)
    rc = ing.lib.crr_ingest_plan_resume(ctypes.byref(db.c), ctypes.byref(br.resume), ctypes.c_void_p(ing.scratch.data_ptr()),
                                        ctypes.c_size_t(size), ctypes.byref(S), ctypes.c_void_p(s.cuda_stream))
    assert rc == 0 and S.err == SCRATCH_TOO_SMALL and S.n_events == n_ev
    pr.restore()
    br.step()                                   # DeviceIngest.plan: grow and plan again
    got = eng.download(pr.db)
    assert got.exec.tobytes() == want.exec.tobytes()
    # a corrupt task payload: the first blob's preamble byte
    rb = br.blobs.blobs
    i = int(np.nonzero(rb.wf["blob_count"] > 0)[0][0])
    j = int(rb.wf["blob_begin"][i])
    bad = rb.bytes.copy()
    bad[int(rb.blob_off[j])] ^= 0xFF
    br.blobs = ing.upload(BlobSet(bytes=bad, blob_off=rb.blob_off, wf=rb.wf, strings=rb.strings))
    with pytest.raises(IngestError) as e:
        br.step()
    assert e.value.blob == j
