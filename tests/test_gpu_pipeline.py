"""Device-side live-row compaction (crr_compact_rows), the chunked host->device->host pipeline and the
device digest of the multi-GPU reduction, against the oracle and the host-side equivalents."""
import numpy as np
import pytest

from cadence_amd import abi, synth, synth_mixed
from cadence_amd.flatten import flatten, interleave
from cadence_amd.result import diff_results, gather_live

KNOWN = {"domain-a", "domain-b", "parent-domain"}


@pytest.fixture(scope="module")
def eng():
    from cadence_amd.engine import ReplayEngine
    return ReplayEngine(0)


def _mixed(n, seed, **kw):
    hs = synth_mixed.mixed_histories(n, seed, **kw)
    return flatten(hs, known_domains=KNOWN)


@pytest.mark.gpu
@pytest.mark.parametrize("emit", [False, True])
def test_compaction_matches_slot_tables(eng, emit):
    canon = _mixed(3000, 71, mean_len=90, multi_version=True, invalid_rate=0.05, can_rate=0.3)
    canon.emit_tasks = emit
    b = interleave(canon, long_threshold=120)
    b.emit_tasks = emit
    assert b.wave_begin < b.n_wf and b.tiers is not None
    db = eng.upload(b)
    eng.launch(db)
    eng.compact(db)
    cr = eng.download_compact(db)
    full = eng.download(db)
    live = gather_live(b, full)
    for t, (name, dt, _b, cap_f, n_f) in enumerate(abi.TABLES):
        if name == "tasks" and not emit:
            assert cr.offsets[t, -1] == 0
            continue
        c = np.clip(full.exec[n_f].astype(np.int64), 0, b.wf[cap_f].astype(np.int64))
        assert (cr.offsets[t] == np.concatenate([[0], np.cumsum(c)])).all(), name
        assert cr.rows[name].tobytes() == live[name].tobytes(), name
    assert cr.exec.tobytes() == full.exec.tobytes()
    assert not diff_results(b, cr.to_replay_result(b), b, full)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["interleaved", "canonical"])
def test_widen_rebuilds_columns(eng, layout):
    import torch
    from cadence_amd.wire import event_slots, pack_events
    canon = _mixed(2500, 17, mean_len=70, multi_version=True, invalid_rate=0.1, can_rate=0.3)
    b = interleave(canon, long_threshold=100) if layout == "interleaved" else canon
    db = eng.upload(b)
    for name, _t in abi.EVENT_COLUMNS:
        if name != "etype":
            db.tensors["ev_" + name].fill_(0xA5)       # garbage the widening must overwrite
    pk = pack_events(b)
    eng.attach_packed(db, pk)
    for c, a in pk.data.items():
        db.tensors["pk_" + c][:a.size].copy_(torch.from_numpy(a))
    db.tensors["pk_ts_base"].copy_(torch.from_numpy(pk.ts_base))
    eng.widen(db)
    torch.cuda.synchronize()
    _w, _s, slot, _p = event_slots(b)
    n_lane = b.wave_begin if b.wave_begin is not None else (b.n_wf if b.stride == 64 else 0)
    pad = np.zeros(b.n_slots, bool)
    if b.stride == 64 and n_lane:      # padding of live lanes (lanes past the last workflow are never read)
        lane_slots = int(b.wf["ev_begin"][n_lane]) if n_lane < b.n_wf else b.n_slots
        p = np.arange(lane_slots)
        gb = b.wf["ev_begin"][:n_lane:64].astype(np.int64)            # group bases (lane 0 of each group)
        w = (np.searchsorted(gb, p, side="right") - 1) * 64 + p % 64
        pad[:lane_slots] = ((b.cols["etype"][:lane_slots] & abi.ETYPE_MASK) == abi.EV_PAD) & (w < n_lane)
    for name, t in abi.EVENT_COLUMNS:
        if name == "etype":
            continue
        got = db.tensors["ev_" + name][:b.n_slots * np.dtype(t).itemsize].cpu().numpy().view(t)
        assert (got[slot] == b.cols[name][slot]).all(), name
        assert (got[pad] == 0).all(), name
    assert (eng.replay(b).exec["checksum"] != 0).any()


@pytest.mark.gpu
@pytest.mark.parametrize("wire", [False, True])
def test_streaming_pipeline_matches_oracle(eng, wire):
    from oracle import oracle
    from cadence_amd.pipeline import StreamingReplay
    chunks = [interleave(_mixed(1500, 90 + i, mean_len=60, multi_version=True, invalid_rate=0.05, can_rate=0.2))
              for i in range(3)]
    chunks.append(interleave(synth.activity_chain(4000, 3, synth.SEED_C2, wf_ids=np.arange(4000, 8000))))
    sr = StreamingReplay(eng, chunks, wire=wire)
    for _ in range(2):                       # a second pass reuses every buffer (outputs re-zeroed)
        st = sr.run()
    assert st["events"] == sum(c.n_events for c in chunks) and st["d2h_bytes"] > 0
    for b, cr in zip(chunks, sr.results()):
        ref = oracle.replay(b, 8)
        d = diff_results(b, cr.to_replay_result(b), b, ref)
        assert not d, d


@pytest.mark.gpu
def test_device_digest_equals_host_digest(eng):
    """Device digest == host digest on a batch with failures and continue-as-new runs (each new run is
    its own workflow row), and on a passive-replication step (ApplyEvents onto loaded states): the
    events field counts the events each call applied."""
    import torch
    from cadence_amd import dist
    b = interleave(_mixed(2000, 5, mean_len=50, invalid_rate=0.1, can_rate=0.3))
    db = eng.upload(b)
    eng.launch(db)
    keys_h = dist.device_keys(b)
    keys = torch.from_numpy(keys_h).to(eng.dev)
    d_dev = dist.digest_torch(torch, db.tensors["exec"], b.n_wf, db.tensors["wf"], keys).cpu().numpy()
    res = eng.download(db)
    assert (d_dev == dist.digest_numpy(res.exec, b.wf["ev_count"], keys_h)).all()
    assert d_dev[1] + d_dev[2] == b.n_wf and d_dev[2] > 0
    ok = res.exec["status"] == 0
    assert d_dev[0] == int(b.wf["ev_count"][ok].sum())
    assert (b.wf["flags"] & abi.WF_FLAG_NEW_RUN).any()
    # identity binding: two OK workflows' results swapped (counts and checksum sum unchanged) change it
    i, j = [int(x) for x in np.nonzero(ok & (res.exec["checksum"] != res.exec["checksum"][np.argmax(ok)]))[0][:1]] + \
           [int(np.argmax(ok))]
    row = abi.EXEC_ROW.itemsize
    ex = db.tensors["exec"]
    a, c = ex[i * row:(i + 1) * row].clone(), ex[j * row:(j + 1) * row].clone()
    ex[i * row:(i + 1) * row].copy_(c)
    ex[j * row:(j + 1) * row].copy_(a)
    d_sw = dist.digest_torch(torch, ex, b.n_wf, db.tensors["wf"], keys).cpu().numpy()
    assert (d_sw[:4] == d_dev[:4]).all() and d_sw[4] != d_dev[4]


@pytest.mark.gpu
def test_device_digest_counts_resumed_events(eng):
    import torch
    from cadence_amd import dist
    from cadence_amd.replication import PassiveReplication
    b = interleave(_mixed(1500, 9, mean_len=40))
    pr = PassiveReplication(eng, b)
    pr.setup()
    pr.restore()
    pr.step()
    n = pr.batch.n_wf
    exec_t, wf_t = pr.db.tensors["exec"], pr.db_new.tensors["wf"]     # loaded rows updated in place
    keys_h = dist.device_keys(pr.batch)
    d_dev = dist.digest_torch(torch, exec_t, n, wf_t, torch.from_numpy(keys_h).to(eng.dev)).cpu().numpy()
    res = eng.download(pr.db)
    wf = wf_t[: n * abi.WORKFLOW.itemsize].cpu().numpy().view(abi.WORKFLOW)
    assert (d_dev == dist.digest_numpy(res.exec, wf["ev_count"], keys_h)).all()
    ok = res.exec["status"] == 0
    assert d_dev[0] == int(wf["ev_count"][ok].sum()) and 0 < d_dev[0] <= pr.n_events
    # NextEventID - 1 would count the loaded prefix too
    assert d_dev[0] < int((res.exec["next_event_id"][ok] - 1).sum())


@pytest.mark.gpu
def test_fused_digest_equals_host_digest_every_path(eng):
    """The digest folded into the replay launch (crr_outputs.digest) == dist.digest_numpy of the rows, on
    every kernel that finalises workflows: the tier segments and the retry pass (mixed, interleaved), the
    wavefront tail and big kernels (long histories), the canonical-layout global kernel, task emission,
    and a passive-replication step (loaded states).  Keys bind results to identities: exchanging two OK
    workflows' keys changes it."""
    from cadence_amd import dist
    from cadence_amd.replication import PassiveReplication
    from cadence_amd.engine import fold_digest
    mixed = _mixed(3000, 11, mean_len=60, invalid_rate=0.1, can_rate=0.3)
    long = flatten(synth_mixed.long_tail_histories(60, 12, max_len=4000, run_cap=1500, multi_version=True, caps=None),
                   known_domains=KNOWN)
    cases = [("mixed", interleave(mixed)), ("lanes", interleave(mixed, long_threshold=None)), ("canonical", mixed),
             ("long", interleave(long))]
    emit = interleave(mixed)
    emit.emit_tasks = True
    cases.append(("emit", emit))
    for name, b in cases:
        db = eng.upload(b)
        keys = dist.device_keys(b)
        eng.enable_digest(db, keys)
        eng.launch(db)
        got = eng.read_digest(db)
        res = eng.download(db)
        want = dist.digest_numpy(res.exec, b.wf["ev_count"], keys)
        assert (got == want).all(), (name, got, want)
        assert got[1] + got[2] == b.n_wf, name
        eng.launch(db)   # the buffer is zeroed by each call: a second launch gives the same digest
        assert (eng.read_digest(db) == want).all(), name
    # identity binding through the keys the kernel reads
    b = cases[0][1]
    db = eng.upload(b)
    keys = dist.device_keys(b)
    eng.enable_digest(db, keys)
    eng.launch(db)
    d0 = eng.read_digest(db)
    ex = eng.download(db).exec
    ok = np.nonzero((ex["status"] == 0))[0]
    i = int(ok[0])
    j = int(ok[np.nonzero(ex["checksum"][ok] != ex["checksum"][i])[0][0]])
    k2 = keys.copy()
    k2[[i, j]] = k2[[j, i]]
    eng.enable_digest(db, k2)
    eng.launch(db)
    d1 = eng.read_digest(db)
    assert (d1[:4] == d0[:4]).all() and d1[4] != d0[4]
    # passive replication: the resumed step's digest counts this call's events
    pb = interleave(_mixed(1500, 9, mean_len=40))
    pr = PassiveReplication(eng, pb)
    pr.setup()
    keys = dist.device_keys(pr.batch)
    eng.enable_digest(pr.db_new, keys)
    pr.restore()
    pr.step()
    got = eng.read_digest(pr.db_new)
    res = eng.download(pr.db)
    wf = pr.db_new.tensors["wf"][: pb.n_wf * abi.WORKFLOW.itemsize].cpu().numpy().view(abi.WORKFLOW)
    assert (got == dist.digest_numpy(res.exec, wf["ev_count"], keys)).all()
    assert fold_digest(pr.db_new.tensors["digest"].cpu().numpy())[0] == got[0]


@pytest.mark.gpu
def test_every_launch_leaves_scratch_counters_zeroed(eng):
    """crr_replay leaves scratch[0..3] (the retry lists' counts, the retry pass's block count and the big
    segment's gate counter) zeroed after every launch -- also when nothing was handed back to the retry pass,
    whose early return then resets the gate the big blocks counted themselves into.  Valid long histories
    with unbounded live sets: a big segment beside the wave tail, every bound exact (no retries)."""
    import torch
    from oracle import oracle
    long = flatten(synth_mixed.long_tail_histories(80, 14, max_len=4000, run_cap=1500, multi_version=True,
                                                   invalid_rate=0.0, caps=None), known_domains=KNOWN)
    b = interleave(long)
    assert b.tiers is not None and b.tiers[5] < b.n_wf, "needs a big segment"
    assert b.wave_begin < b.tiers[5], "needs a wave tail beside it (the gated launch)"
    db = eng.upload(b)
    for _ in range(3):
        eng.launch(db)
        torch.cuda.synchronize()
        assert (db.tensors["scratch"][:4].cpu().numpy() == 0).all(), db.tensors["scratch"][:4].cpu().numpy()
    d = diff_results(b, eng.download(db), b, oracle.replay(b, 0))
    assert not d, d


@pytest.mark.gpu
def test_empty_batch_zeroes_the_digest(eng):
    """An empty rank (n_wf == 0) still zeroes its digest buffer: stale sums must not join the all-reduce."""
    import ctypes
    import torch
    from cadence_amd import dist
    b = interleave(_mixed(200, 3))
    db = eng.upload(b)
    eng.enable_digest(db, dist.device_keys(b))
    db.tensors["digest"].fill_(12345)
    ci = abi.CInputs()
    ctypes.memmove(ctypes.byref(ci), ctypes.byref(db.c_in), ctypes.sizeof(ci))
    ci.n_wf = 0
    s = torch.cuda.current_stream(eng.dev)
    assert eng.lib.crr_replay(ctypes.byref(ci), ctypes.byref(db.c_out), ctypes.c_void_p(s.cuda_stream)) == 0
    torch.cuda.synchronize()
    assert (db.tensors["digest"].cpu().numpy() == 0).all()


@pytest.mark.gpu
def test_live_id_sidecar_matches_rows_every_path(eng):
    """The live-ID sidecar (crr_outputs.live_ids, ABI v6) holds, for every OK workflow, the IDs of its live rows
    in slots 0..n-1 of each pending map (the checksum's lists) on every kernel path -- tier segments, retry
    pass, wavefront tail / big kernels, canonical global kernel, task emission, a passive-replication step --
    and crr_checksum reading it equals crr_checksum reading the rows and the replay's own checksums."""
    import ctypes
    import torch
    from cadence_amd.replication import PassiveReplication
    mixed = _mixed(3000, 15, mean_len=60, invalid_rate=0.1, can_rate=0.3)
    long = flatten(synth_mixed.long_tail_histories(60, 16, max_len=4000, run_cap=1500, multi_version=True, caps=None),
                   known_domains=KNOWN)
    emit = interleave(mixed)
    emit.emit_tasks = True
    cases = [("mixed", interleave(mixed)), ("lanes", interleave(mixed, long_threshold=None)), ("canonical", mixed),
             ("long", interleave(long)), ("emit", emit)]
    id_field = {"act": "schedule_id", "timer": "started_id", "child": "initiated_id", "rc": "initiated_id",
                "sig": "initiated_id"}
    counts = {"act": "n_activity", "timer": "n_timer", "child": "n_child", "rc": "n_rc", "sig": "n_signal"}
    base = {t[0]: t[2] for t in abi.TABLES}

    def check_db(name, b, db):
        res = eng.download(db)
        ok = np.nonzero(res.exec["status"] == 0)[0]
        st = b.wf_strides()
        n_ids = 0
        for t in abi.ID_TABLES:
            side = db.tensors["ids_" + t].cpu().numpy()
            rows = res.tables[t]
            for w in ok[:: max(1, ok.size // 400)]:
                n = int(res.exec[counts[t]][w])
                idx = int(b.wf[base[t]][w]) + np.arange(n, dtype=np.int64) * int(st[w])
                assert (side[idx] == rows[id_field[t]][idx]).all(), (name, t, int(w))
                n_ids += n
        # crr_checksum over the sidecar == over the rows == the replay's checksums
        with_side = eng.checksum(db)
        co = abi.COutputs()
        ctypes.memmove(ctypes.byref(co), ctypes.byref(db.c_out), ctypes.sizeof(co))
        for t in range(len(abi.ID_TABLES)):
            co.live_ids[t] = None
        out = torch.zeros(max(db.n_wf, 1), dtype=torch.int32, device=eng.dev)
        s = torch.cuda.current_stream(eng.dev)
        assert eng.lib.crr_checksum(ctypes.byref(db.c_in), ctypes.byref(co), ctypes.c_void_p(out.data_ptr()),
                                    ctypes.c_void_p(s.cuda_stream)) == 0
        rows_cs = out.cpu().numpy().view(np.uint32)[:db.n_wf]
        assert (with_side[ok] == res.exec["checksum"][ok]).all(), name
        assert (rows_cs[ok] == res.exec["checksum"][ok]).all(), name
        return n_ids

    total = 0
    for name, b in cases:
        db = eng.upload(b)
        eng.launch(db)
        total += check_db(name, b, db)
    assert total > 1000
    pb = interleave(_mixed(1500, 17, mean_len=40))
    pr = PassiveReplication(eng, pb)
    pr.setup()
    pr.restore()
    pr.step()
    check_db("passive", pr.batch, pr.db)


@pytest.mark.gpu
def test_token_crc_splice_matches_hashing_the_token():
    """crr_inputs.token_crc (ABI v7): the start token's precomputed raw CRC spliced into the checksum by a GF(2)
    shift of the register gives the same checksums -- replay and the Load verify path -- as hashing the token's
    bytes (NULL token_crc), on every kernel path, with rebuild (final) tokens and odd token lengths left to the
    bytes."""
    from cadence_amd import abi, synth, synth_native
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.flatten import interleave
    eng = ReplayEngine(0)
    batches = [interleave(synth.activity_chain(5000, 4, synth.SEED_C2, with_keys=False)),
               interleave(synth_native.mixed(20000, multi_version=True, can_rate=0.3)),
               interleave(synth_native.long_tail(30, max_len=12_000, run_cap=4_000))]
    for b in batches:
        got, want = [], []
        for tc, out in ((True, got), (False, want)):
            db = eng.upload(b, token_crc=tc)
            assert bool(db.c_in.token_crc) == tc
            eng.launch(db)
            res = eng.download(db)
            out.append(res.exec.tobytes())
            out.append(eng.checksum(db).tobytes())
        assert got == want
        ex = np.frombuffer(got[0], abi.EXEC_ROW)
        assert (ex["status"] == 0).sum() > 0.5 * b.n_wf
