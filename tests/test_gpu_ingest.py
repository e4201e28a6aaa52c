"""Device-side ingest (crr_ingest_plan / crr_ingest_layout, ingest_kernel.hip) against the host path:
the same blobs through the native decoder + flatten.interleave must give byte-identical device inputs
(columns, side records, reset keys, branch tokens, descriptors, tier boundaries, slot-table sizes, the
device order), and replaying them must give the oracle's rows."""
import numpy as np
import pytest

from cadence_amd import abi, synth, synth_mixed, synth_native
from cadence_amd.blobs import KNOWN_DOMAINS, encode_batch
from cadence_amd.decode import decode_histories
from cadence_amd.flatten import flatten, interleave
from cadence_amd.result import diff_results


@pytest.fixture(scope="module")
def eng():
    from cadence_amd.engine import ReplayEngine
    return ReplayEngine(0)


def _ingest(eng, bs, emit=False):
    from cadence_amd.ingest import DeviceIngest
    ing = DeviceIngest(eng)
    dblobs = ing.upload(bs)
    out = ing.ingest(dblobs, emit_tasks=emit)
    return ing, out


def _assert_same_inputs(got, want):
    assert got.wave_begin == want.wave_begin
    assert tuple(got.tiers) == tuple(want.tiers), (got.tiers, want.tiers)
    assert got.perm.tolist() == want.perm.tolist()
    for name, _t in abi.EVENT_COLUMNS:
        np.testing.assert_array_equal(got.cols[name], want.cols[name], err_msg=name)
    assert got.act_side.tobytes() == want.act_side.tobytes()
    assert got.start_side.tobytes() == want.start_side.tobytes()
    assert got.reset_keys.tolist() == want.reset_keys.tolist()
    assert got.arena.tobytes() == want.arena.tobytes()
    assert got.wf.tobytes() == want.wf.tobytes()
    for name, *_r in abi.TABLES:
        assert got.table_rows[name] == want.table_rows[name], name


def _host_path(bs):
    canon = decode_histories(bs.to_sources(), known_domains=KNOWN_DOMAINS)
    return canon, interleave(canon)


@pytest.mark.gpu
@pytest.mark.parametrize("gen", ["chains", "mixed", "mixed_errors", "long_tail"])
def test_device_ingest_matches_host_path(eng, gen):
    if gen == "chains":
        b = synth.activity_chain(3000, 4, synth.SEED_C2, with_keys=True, wf_ids=np.arange(3000))
    elif gen == "mixed":
        b = synth_native.mixed(6000, mean_len=45)
    elif gen == "mixed_errors":
        b = synth_native.mixed(4000, multi_version=True, invalid_rate=0.1, can_rate=0.3, unknown_domain_rate=0.2)
    else:
        b = synth_native.long_tail(40, max_len=20_000, run_cap=5_000)
    bs = encode_batch(b)
    canon, want = _host_path(bs)
    ing, out = _ingest(eng, bs)
    got = ing.to_host_batch(out)
    _assert_same_inputs(got, want)
    # and the replay of the device-laid-out inputs equals the oracle's
    from oracle import oracle
    eng.launch(out)
    res = eng.download(out)
    ref = oracle.replay(canon, 8)
    d = diff_results(want, res, canon, ref)
    assert not d, d[:3]


@pytest.mark.gpu
@pytest.mark.parametrize("gen", ["chains_59", "chains_65", "mixed_64"])
def test_device_ingest_wave_pass_boundaries(eng, gen):
    """Workflows either side of the wavefront-per-workflow pass's limit (64 events): 59- and 65-event
    activity chains, mixed histories around 64 events -- the two per-workflow kernels must agree with the
    host path byte for byte."""
    if gen == "chains_59":
        b = synth.activity_chain(2000, 9, synth.SEED_C2, with_keys=True, wf_ids=np.arange(2000))
    elif gen == "chains_65":
        b = synth.activity_chain(2000, 10, synth.SEED_C2, with_keys=True, wf_ids=np.arange(2000))
    else:
        b = synth_native.mixed(4000, mean_len=64)
    bs = encode_batch(b)
    _canon, want = _host_path(bs)
    ing, out = _ingest(eng, bs)
    _assert_same_inputs(ing.to_host_batch(out), want)


@pytest.mark.gpu
def test_device_ingest_python_histories_with_prev_reset_points(eng):
    """Python-generated histories: previous auto-reset points, unknown domains, empty batches, CAN."""
    hs = synth_mixed.mixed_histories(800, 23, multi_version=True, invalid_rate=0.3, can_rate=0.5)
    b = flatten(hs, known_domains=set(KNOWN_DOMAINS))
    bs = encode_batch(b)
    _canon, want = _host_path(bs)
    ing, out = _ingest(eng, bs)
    _assert_same_inputs(ing.to_host_batch(out), want)


@pytest.mark.gpu
def test_device_ingest_rejects_what_the_host_decoder_rejects(eng):
    """Corrupt blobs fail the plan with the host decoder's error code and the lowest failing blob."""
    from cadence_amd.decode import DeserializationError
    from cadence_amd.ingest import IngestError
    b = synth_native.mixed(200)
    for corrupt in ("preamble", "truncate", "type"):
        bs = encode_batch(b)
        i = 37
        o0, o1 = int(bs.blob_off[i]), int(bs.blob_off[i + 1])
        if corrupt == "preamble":
            bs.bytes[o0] = 0x58
        elif corrupt == "truncate":
            bs.bytes[o0 + 6] = 0x7F        # the event count: far more events than the blob holds
        else:
            bs.bytes[o0 + 1] = 0x07        # the History field's type byte: no such thrift type
        with pytest.raises(DeserializationError) as he:
            decode_histories(bs.to_sources(), known_domains=KNOWN_DOMAINS)
        with pytest.raises(IngestError) as de:
            _ingest(eng, bs)
        assert (de.value.code, de.value.blob) == (he.value.code, he.value.blob), corrupt
        del o1


@pytest.mark.gpu
def test_device_ingest_empty_and_tiny(eng):
    """A workflow with no batches, one with an empty batch, a single-event one."""
    hs = synth_mixed.mixed_histories(5, 5)
    hs[1].batches = []
    hs[2].batches.insert(1, [])
    hs[3].batches = [hs[3].batches[0][:1]]
    b = flatten(hs, known_domains=set(KNOWN_DOMAINS))
    bs = encode_batch(b)
    _canon, want = _host_path(bs)
    ing, out = _ingest(eng, bs)
    _assert_same_inputs(ing.to_host_batch(out), want)


@pytest.mark.gpu
@pytest.mark.parametrize("rate", [0.05, 0.5])
def test_device_ingest_reshaped_blobs(eng, rate):
    """Blobs in shapes thriftrw never writes (tests/thrift_tree.py: fields reversed / shuffled, the type
    after the attributes, duplicate types, lists of structs and maps of lists, leaf containers) go through
    the fast pass's deferral to the general pass and still match the host decoder byte for byte."""
    from thrift_tree import reshape_blobset
    hs = synth_mixed.mixed_histories(400, 29, multi_version=True, invalid_rate=0.2, can_rate=0.3)
    b = flatten(hs, known_domains=set(KNOWN_DOMAINS))
    for src in (encode_batch(b), encode_batch(synth_native.mixed(1500, multi_version=True, unknown_domain_rate=0.2))):
        bs = reshape_blobset(src, seed=11, rate=rate)
        _canon, want = _host_path(bs)
        ing, out = _ingest(eng, bs)
        _assert_same_inputs(ing.to_host_batch(out), want)


@pytest.mark.gpu
def test_device_ingest_scratch_too_small_then_replans(eng):
    """A plan whose scratch holds fewer events than the blobs reports CRR_INGEST_SCRATCH_TOO_SMALL (and
    decodes nothing); DeviceIngest.plan grows the scratch and plans again, matching the host path."""
    import ctypes
    from cadence_amd.ingest import SCRATCH_TOO_SMALL, CIngestSummary, DeviceIngest
    b = synth_native.mixed(700, mean_len=30)
    bs = encode_batch(b)
    _canon, want = _host_path(bs)
    ing = DeviceIngest(eng)
    db = ing.upload(bs)
    size = ing.ensure_scratch(db, 1)
    S = CIngestSummary()
    s = eng.torch.cuda.current_stream(eng.dev)
    rc = ing.lib.crr_ingest_plan(ctypes.byref(db.c), ctypes.c_void_p(ing.scratch.data_ptr()), ctypes.c_size_t(size),
                                 ctypes.byref(S), ctypes.c_void_p(s.cuda_stream))
    assert rc == 0
    assert S.err == SCRATCH_TOO_SMALL and S.n_events == want.n_events
    S2 = ing.plan(db, max_events=1)           # the grow-and-replan loop
    out = ing.layout(db, S2)
    _assert_same_inputs(ing.to_host_batch(out), want)


@pytest.mark.gpu
def test_device_ingest_reuses_scratch_across_plans(eng):
    """One DeviceIngest plans different blob sets in turn (the scratch is reused, not re-zeroed): a set
    whose reshaped blobs the fast pass defers, then a clean set, a corrupt one and the reshaped one again
    -- each equal to the host path (or failing with its error), nothing carried over from the plan
    before."""
    from thrift_tree import reshape_blobset
    from cadence_amd.decode import DeserializationError
    from cadence_amd.ingest import DeviceIngest, IngestError
    ing = DeviceIngest(eng)
    hs = synth_mixed.mixed_histories(300, 29, multi_version=True, invalid_rate=0.2, can_rate=0.3)
    reshaped = reshape_blobset(encode_batch(flatten(hs, known_domains=set(KNOWN_DOMAINS))), seed=5, rate=0.5)
    clean = encode_batch(synth_native.mixed(900, mean_len=25))
    corrupt = encode_batch(synth_native.mixed(300, mean_len=25))
    corrupt.bytes[int(corrupt.blob_off[11]) + 1] = 0x07
    for bs in (reshaped, clean, corrupt, reshaped, clean):
        try:
            _canon, want = _host_path(bs)
        except DeserializationError as he:
            with pytest.raises(IngestError) as de:
                ing.ingest(ing.upload(bs))
            assert (de.value.code, de.value.blob) == (he.code, he.blob)
            continue
        out = ing.ingest(ing.upload(bs))
        _assert_same_inputs(ing.to_host_batch(out), want)


@pytest.mark.gpu
def test_device_ingest_blobs_flush_against_the_pad(eng):
    """The blob bytes in a buffer of exactly len + CRR_INGEST_PAD bytes (the header's contract), the last
    blob ending where the padding starts."""
    from cadence_amd.ingest import INGEST_PAD, DeviceIngest
    bs = encode_batch(synth_native.mixed(400, mean_len=20))
    _canon, want = _host_path(bs)
    ing = DeviceIngest(eng)
    host = ing.host_arrays(bs)
    db = ing.upload(bs, host)
    end = int(bs.blob_off[-1])
    t = eng.torch.zeros(end + INGEST_PAD, dtype=eng.torch.uint8, device=eng.dev)
    t[:end].copy_(eng.torch.from_numpy(np.ascontiguousarray(bs.bytes[:end])))
    db.tensors["bytes"] = t
    db.c.bytes = t.data_ptr()
    out = ing.ingest(db)
    _assert_same_inputs(ing.to_host_batch(out), want)


@pytest.mark.gpu
def test_device_ingest_ids_beyond_2_40(eng):
    """Activity completions whose scheduled-event reference equals an inserted ID plus 2^40 are deletes of
    a missing entry (flatten.live_set_bounds compares exact IDs), so they must not lower the live-set
    bound on the device either: tiers and capacities stay identical to the host path."""
    import copy
    hs = synth_mixed.mixed_histories(600, 31, multi_version=False)
    hs0 = copy.deepcopy(hs)
    n_mod = 0
    for h in hs:
        for batch in h.batches:
            for e in batch:
                if e.event_type == abi.EventType.ActivityTaskCompleted and n_mod < 400:
                    e.attrs["scheduled_event_id"] = int(e.attrs["scheduled_event_id"]) + (1 << 40)
                    n_mod += 1
    assert n_mod > 50
    b = flatten(hs, known_domains=set(KNOWN_DOMAINS))
    # the exact comparison matters here: those deletes no longer lower some workflows' bounds
    from cadence_amd.flatten import live_set_bounds
    b0 = flatten(hs0, known_domains=set(KNOWN_DOMAINS))
    assert (live_set_bounds(b)["act"] > live_set_bounds(b0)["act"]).any()
    bs = encode_batch(b)
    canon, want = _host_path(bs)
    ing, out = _ingest(eng, bs)
    _assert_same_inputs(ing.to_host_batch(out), want)
    from oracle import oracle
    eng.launch(out)
    res = eng.download(out)
    d = diff_results(want, res, canon, oracle.replay(canon, 8))
    assert not d, d[:3]
