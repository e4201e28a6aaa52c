"""The native thriftrw writer of synthetic persisted histories (blob_encode.cpp, benchmark / test
infrastructure) against the native decoder: decode(encode(batch)) == batch, for every generator.  The
blob -> rows benchmark and the device-ingest parity tests rely on it."""
import numpy as np
import pytest

from cadence_amd import abi, synth, synth_mixed, synth_native
from cadence_amd.blobs import KNOWN_DOMAINS, encode_batch
from cadence_amd.decode import decode_histories
from cadence_amd.flatten import flatten
from cadence_amd.thrift_codec import serialize_history

from test_decode import assert_same_batch


@pytest.mark.parametrize("gen", ["native_mixed", "python_mixed", "long_tail"])
def test_encode_then_decode_is_identity(gen):
    if gen == "native_mixed":
        b = synth_native.mixed(2000, multi_version=True, invalid_rate=0.1, can_rate=0.3, unknown_domain_rate=0.2)
    elif gen == "python_mixed":
        b = flatten(synth_mixed.mixed_histories(400, 3, multi_version=True, invalid_rate=0.25, can_rate=0.5),
                    known_domains=set(KNOWN_DOMAINS))
    else:
        b = synth_native.long_tail(12)
    bs = encode_batch(b)
    assert bs.n_wf == b.n_wf
    assert_same_batch(decode_histories(bs.to_sources(), known_domains=KNOWN_DOMAINS), b)


def test_activity_chains_round_trip():
    """Config 2's generator: every column, side record and token survives; the generator's rp_cap (1, a
    tighter bound it knows) is the only descriptor field the decoder recomputes (max_prev * starts +
    decision completions = 5)."""
    b = synth.activity_chain(300, 4, synth.SEED_C2, with_keys=True, wf_ids=np.arange(300))
    d = decode_histories(encode_batch(b).to_sources(), known_domains=KNOWN_DOMAINS)
    want = b.wf.copy()
    want["rp_cap"] = 5
    want["rp_base"] = np.arange(300) * 5
    b.wf = want
    b.table_rows["rp"] = 1500
    assert_same_batch(d, b)


def test_blobs_match_the_python_writer():
    """Same bytes as thrift_codec.serialize_history for the fields both write (a Python-generated history
    whose every string the columns carry): the native writer is the Python one, restated."""
    hs = synth_mixed.mixed_histories(60, 11)
    b = flatten(hs, known_domains=set(KNOWN_DOMAINS))
    bs = encode_batch(b)
    # blob boundaries and event counts agree (attribute bytes differ only in the request IDs the native
    # writer invents for DecisionTaskStarted / ActivityTaskStarted)
    for w, h in enumerate(hs):
        py = serialize_history(h)
        r = bs.wf[w]
        assert int(r["blob_count"]) == len(py)
        for i, pb in enumerate(py):
            nb = bs.blob(int(r["blob_begin"]) + i)
            assert nb[:9] == pb[:9]       # preamble, list header, event count


def test_split_blobs_keeps_workflows_and_new_run_links():
    """pipeline.split_blobs: chunks at workflow boundaries (never between a continue-as-new run and its
    new-run history), each with only its own strings; decoding the chunks gives the whole batch."""
    from cadence_amd.pipeline import split_blobs
    b = synth_native.mixed(3000, can_rate=0.5)
    bs = encode_batch(b)
    parts = split_blobs(bs, 5)
    assert sum(p.n_wf for p in parts) == b.n_wf
    assert sum(p.strings.size for p in parts) == bs.strings.size
    src, base = [], 0
    for p in parts:
        nr = p.wf["new_run_wf"]
        assert ((nr < 0) | (nr < p.n_wf)).all()
        for s in p.to_sources():
            if s.new_run is not None:
                s.new_run += base
            src.append(s)
        base += p.n_wf
    assert_same_batch(decode_histories(src, known_domains=KNOWN_DOMAINS), b)
