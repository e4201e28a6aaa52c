"""Native history-blob decoder (libcadence_host.so) against the Python host flattening.

The persisted form of a batch is a thriftrw-encoded ``shared.History`` behind the 0x59 preamble
(``common/persistence/serializer.go``, ``common/codec/version0Thriftrw.go``).  The decoder must turn
a workflow's blobs into exactly the columns ``flatten()`` builds from the same events.  Parity
anchors: the thrift-binary conventions are pinned by the reference's own 96-byte branch token (a
thriftrw struct behind the same preamble, in service/worker/archiver/testdata); the reference holds
no encoded history blob, so the blobs come from ``thrift_codec`` (an independent writer).
"""
import random
import struct

import numpy as np
import pytest

from cadence_amd import abi, synth_mixed
from cadence_amd.abi import EventType as ET
from cadence_amd.decode import DeserializationError, WorkflowSource, decode_histories
from cadence_amd.flatten import flatten, interleave
from cadence_amd.history import WorkflowHistory, load_json_history, split_batches_by_task_id
from cadence_amd.result import diff_results
from cadence_amd.thrift_codec import serialize_batch_events, serialize_history

KNOWN = {"domain-a", "domain-b", "parent-domain"}
ARCHIVAL = "tests/golden/archival_workflow_history_v1.json"


def sources_of(hs):
    out = []
    for h in hs:
        nr = None
        for e in h.events:
            if e.event_type == ET.WorkflowExecutionContinuedAsNew and e.attrs.get("new_run") is not None:
                nr = int(e.attrs["new_run"])
        out.append(WorkflowSource(blobs=serialize_history(h), run_id=h.run_id, branch_id=h.branch_id,
                                  domain_failover_version=h.domain_failover_version, now_ns=h.now_ns,
                                  final_token=h.final_token, rebuild_last_event_id=h.rebuild_last_event_id,
                                  rebuild_last_event_version=h.rebuild_last_event_version, new_run=nr,
                                  is_new_run=h.is_new_run, refresh_tasks=h.refresh_tasks))
    return out


def keys_of(b):
    ka = bytes(b.key_arena)
    return [ka[o:o + n] for o, n in zip(b.key_off.tolist(), b.key_len.tolist())]


def assert_same_batch(got, want):
    for name, _t in abi.EVENT_COLUMNS:
        np.testing.assert_array_equal(got.cols[name], want.cols[name], err_msg=name)
    n_act = int((want.cols["etype"] & abi.ETYPE_MASK == ET.ActivityTaskScheduled).sum())
    n_st = int((want.cols["etype"] & abi.ETYPE_MASK == ET.WorkflowExecutionStarted).sum())
    assert got.act_side[:n_act].tobytes() == want.act_side[:n_act].tobytes()
    assert got.start_side[:n_st].tobytes() == want.start_side[:n_st].tobytes()
    nrk = int(sum(max(int(c), 0) for c in want.start_side["prev_reset_count"][:n_st]))
    assert got.reset_keys[:nrk].tolist() == want.reset_keys[:nrk].tolist()
    na = int(want.wf["start_token_len"].sum() + np.where(want.wf["final_token_len"] == abi.NO_TOKEN, 0,
                                                         want.wf["final_token_len"]).sum())
    assert got.arena[:na].tobytes() == want.arena[:na].tobytes()
    assert got.wf.tobytes() == want.wf.tobytes()
    assert got.table_rows == want.table_rows
    assert keys_of(got) == keys_of(want)


def test_mixed_histories_decode_like_flatten():
    hs = synth_mixed.mixed_histories(600, 31, multi_version=True, invalid_rate=0.25, can_rate=0.5)
    want = flatten(hs, known_domains=KNOWN)
    got = decode_histories(sources_of(hs), known_domains=KNOWN)
    assert_same_batch(got, want)


def test_parallel_decode_and_all_domains_known():
    hs = synth_mixed.mixed_histories(1500, 32, multi_version=True, invalid_rate=0.1, can_rate=0.3)
    src = sources_of(hs)
    one = decode_histories(src, known_domains=None, n_threads=1)
    many = decode_histories(src, known_domains=None, n_threads=6)
    assert_same_batch(many, one)
    assert_same_batch(one, flatten(hs, known_domains=None))


def test_long_tail_and_rebuild_targets():
    hs = synth_mixed.long_tail_histories(40, 9, max_len=3000, run_cap=1200, multi_version=True, invalid_rate=0.1)
    for i, h in enumerate(hs[:10]):
        h.final_token = f"target-token-{i}".encode()
        h.rebuild_last_event_id = 7
        h.rebuild_last_event_version = 3
    assert_same_batch(decode_histories(sources_of(hs), known_domains=KNOWN), flatten(hs, known_domains=KNOWN))


def test_archival_fixture_history():
    ev = load_json_history(ARCHIVAL)
    h = WorkflowHistory(batches=split_batches_by_task_id(ev), run_id="f2b360a0-d90a-4afa-ad88-ba041fad6a42",
                        branch_id="840307b9-9076-4ee2-82a0-45f21d61d719")
    got = decode_histories(sources_of([h]))
    assert_same_batch(got, flatten([h]))
    # the start token the decoder builds is the reference's own 96-byte HistoryBranch token
    from cadence_amd.history import branch_token_from_archival_signal
    tok = branch_token_from_archival_signal(ev, ARCHIVAL)
    off, n = int(got.wf["start_token_off"][0]), int(got.wf["start_token_len"][0])
    assert got.arena[off:off + n].tobytes() == tok


def test_decoded_batch_replays_bit_exact():
    from oracle import oracle
    hs = synth_mixed.mixed_histories(400, 33, multi_version=True, invalid_rate=0.3, can_rate=0.5)
    want = flatten(hs, known_domains=KNOWN)
    got = decode_histories(sources_of(hs), known_domains=KNOWN)
    for b_got, b_want in ((got, want), (interleave(got), interleave(want))):
        assert not diff_results(b_got, oracle.replay(b_got, 2), b_want, oracle.replay(b_want, 2))


def _shuffle_fields(blob: bytes, rng: random.Random) -> bytes:
    """Re-emit every HistoryEvent of a blob with its top-level fields in random order (thrift readers
    accept any order; the attribute struct may then precede the EventType field)."""
    from cadence_amd.thrift_codec import T_LIST, T_STRUCT

    def skip(b, p, t):
        if t in (2, 3):
            return p + 1
        if t == 6:
            return p + 2
        if t == 8:
            return p + 4
        if t in (4, 10):
            return p + 8
        if t == 11:
            return p + 4 + struct.unpack(">i", b[p:p + 4])[0]
        if t == 12:
            while b[p] != 0:
                p = skip(b, p + 3, b[p])
            return p + 1
        if t == 13:
            kt, vt, n = b[p], b[p + 1], struct.unpack(">i", b[p + 2:p + 6])[0]
            p += 6
            for _ in range(n):
                p = skip(b, skip(b, p, kt), vt)
            return p
        if t in (14, 15):
            et, n = b[p], struct.unpack(">i", b[p + 1:p + 5])[0]
            p += 5
            for _ in range(n):
                p = skip(b, p, et)
            return p
        raise ValueError(t)

    assert blob[0] == 0x59 and blob[1] == T_LIST
    n = struct.unpack(">i", blob[5:9])[0]
    out = bytearray(blob[:9])
    p = 9
    for _ in range(n):
        fields = []
        while blob[p] != 0:
            q = skip(blob, p + 3, blob[p])
            fields.append(blob[p:q])
            p = q
        p += 1
        rng.shuffle(fields)
        out += b"".join(fields) + b"\x00"
    out += blob[p:]
    return bytes(out)


def test_field_order_independent():
    rng = random.Random(5)
    hs = synth_mixed.mixed_histories(200, 34, multi_version=True, invalid_rate=0.2)
    src = sources_of(hs)
    for s in src:
        s.blobs = [_shuffle_fields(b, rng) if b else b for b in s.blobs]
    assert_same_batch(decode_histories(src, known_domains=KNOWN), flatten(hs, known_domains=KNOWN))


def test_malformed_blobs_raise():
    h = synth_mixed.mixed_histories(3, 35)
    src = sources_of(h)
    good = src[1].blobs[0]
    src[1].blobs[0] = b"\x00" + good[1:]                   # not the version-0 preamble
    with pytest.raises(DeserializationError) as e:
        decode_histories(src)
    assert e.value.code == -2 and e.value.blob == len(src[0].blobs)
    src[1].blobs[0] = good[: len(good) // 2]                # truncated
    with pytest.raises(DeserializationError) as e:
        decode_histories(src)
    assert e.value.code == -3


def test_empty_batches_and_empty_workflow():
    hs = synth_mixed.mixed_histories(5, 36)
    hs[1].batches.insert(2, [])
    hs[2].batches.append([])
    hs[3].batches = []
    assert_same_batch(decode_histories(sources_of(hs)), flatten(hs))
    assert serialize_batch_events([]) == b""
