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
