"""JSON-encoded persisted batches on the device (crr_ingest_transcode_plan / crr_ingest_transcode,
json_ingest_kernel.hip): serializer.go:321-328 decodes json / unknown / empty-encoded blobs with
json.Unmarshal.  The device rewrites them in HBM as thriftrw and the device ingest lays the batch out; the
result must be byte-identical to the host path on the same blobs (crr_decode_histories_enc, whose JSON walk
json_decode.cpp restates, + flatten.interleave), reject exactly the blobs the host rejects with the same code
and lowest blob index, and replay to the oracle's rows."""
import json

import numpy as np
import pytest

from cadence_amd import synth_mixed
from cadence_amd.blobs import KNOWN_DOMAINS, blobset_from_sources
from cadence_amd.decode import DeserializationError, WorkflowSource, decode_histories
from cadence_amd.flatten import interleave
from cadence_amd.history import events_from_json, split_batches_by_task_id
from cadence_amd.json_codec import event_json
from cadence_amd.result import diff_results
from cadence_amd.thrift_codec import serialize_history

from test_decode import ARCHIVAL
from test_decode_json import _events, json_sources
from test_gpu_ingest import _assert_same_inputs


@pytest.fixture(scope="module")
def eng():
    from cadence_amd.engine import ReplayEngine
    return ReplayEngine(0)


def _device(eng, sources, stage_bytes=None):
    """sources -> BlobSet upload -> transcode -> plan + layout; the laid-out host batch and the engine state."""
    from cadence_amd.ingest import DeviceIngest
    bs, enc = blobset_from_sources(sources)
    ing = DeviceIngest(eng)
    db = ing.upload(bs)
    tdb = ing.transcode(db, enc, stage_bytes=stage_bytes)
    out = ing.ingest(tdb)
    return ing, tdb, out


def _check(eng, sources, replay=False, stage_bytes=None):
    canon = decode_histories(sources, known_domains=KNOWN_DOMAINS)
    want = interleave(canon)
    ing, tdb, out = _device(eng, sources, stage_bytes)
    _assert_same_inputs(ing.to_host_batch(out), want)
    if replay:
        from oracle import oracle
        eng.launch(out)
        res = eng.download(out)
        ref = oracle.replay(canon, 8)
        d = diff_results(want, res, canon, ref)
        assert not d, d[:3]
    return ing, tdb


@pytest.mark.gpu
@pytest.mark.parametrize("encoding", ["json", "", "unknow"])
def test_json_histories_on_device_match_host_path(eng, encoding):
    """Python mixed histories (every event type, previous reset points, unknown domains, CAN, empty
    batches, invalid histories) persisted as JSON: layout byte-identical to the host path, rows = oracle."""
    hs = synth_mixed.mixed_histories(600 if encoding == "json" else 150, 41, multi_version=True, invalid_rate=0.2,
                                     can_rate=0.4)
    for h in hs[::7]:
        h.batches.insert(1, [])
    ing, _tdb = _check(eng, json_sources(hs, encoding), replay=encoding == "json")
    assert int(ing.last_transcode.err) == 0


@pytest.mark.gpu
def test_transcoded_blobs_decode_like_the_json(eng):
    """The transcoded bytes themselves, read back by the host thriftrw decoder, give the batch the host JSON
    decoder gives."""
    from cadence_amd.ingest import DeviceIngest
    from test_decode import assert_same_batch
    hs = synth_mixed.mixed_histories(200, 42, multi_version=True, can_rate=0.3)
    src = json_sources(hs)
    bs, enc = blobset_from_sources(src)
    ing = DeviceIngest(eng)
    tb = ing.transcoded_blobs(ing.transcode(ing.upload(bs), enc))
    assert_same_batch(decode_histories(tb.to_sources(), known_domains=KNOWN_DOMAINS),
                      decode_histories(src, known_domains=KNOWN_DOMAINS))


@pytest.mark.gpu
def test_mixed_encodings_in_one_batch_on_device(eng):
    hs = synth_mixed.mixed_histories(240, 43, multi_version=True, can_rate=0.3)
    src = json_sources(hs)
    for i, (s, h) in enumerate(zip(src, hs)):
        if i % 3 == 0:
            s.blobs, s.encodings = serialize_history(h), None
        elif i % 3 == 1 and len(s.blobs) > 1:
            tb = serialize_history(h)
            s.blobs = [tb[0]] + s.blobs[1:]
            s.encodings = ["thriftrw"] + s.encodings[1:]
    _check(eng, src, replay=True)


@pytest.mark.gpu
def test_go_json_conventions_on_device(eng):
    """Case-insensitive keys, enums by name in any case or decimal text, null as unset, unknown keys
    skipped, the last duplicate winning, escaped key and value strings (encoding/json unescapes them)."""
    evs = _events()
    raw = [event_json(e) for e in evs]
    raw[0] = {k.upper(): v for k, v in raw[0].items()}
    raw[0]["EVENTTYPE"] = "workflowexecutionstarted"
    attrs = raw[0]["WORKFLOWEXECUTIONSTARTEDEVENTATTRIBUTES"]
    attrs["initiator"] = "retrypolicy"
    attrs["somethingNew"] = {"nested": [1, 2.5e3, None, True, False, "x\\u00e9", {"a": [{}]}]}
    raw[1]["eventType"] = "+4"
    raw[1]["decisionTaskScheduledEventAttributes"]["attempt"] = None
    raw[2]["decisionTaskTimedOutEventAttributes"]["timeoutType"] = "3"
    text = json.dumps(raw).replace('"version": 7', '"version": 99, "version": 7', 1)
    # an escaped key ("eventId" is "eventId") and escaped reset-point strings (unicode, surrogate pair)
    text = text.replace('"eventId": 2', '"\\u0065ventId": 2', 1)
    text = text.replace('"bc-1"', '"bc-\\u00e9\\ud83d\\ude00\\n"', 1)
    srcs = [WorkflowSource(blobs=[text.encode()], encodings=["json"])]
    _check(eng, srcs)


@pytest.mark.gpu
@pytest.mark.parametrize("blob", [b'[{"eventId": 1.5}]', b'[{"eventId": "1"}]', b'[{"eventId": 1}', b'[null]',
                                  b'[{"eventType": "NoSuchEvent"}]', b'[{"eventId": 99999999999999999999}]',
                                  b'{"eventId": 1}', b'[{"eventId": 1}] x', b'[{"eventType": 4}]',
                                  b'[{"eventType": "EventType(99)"}]', b'[{"eventType": " 4"}]',
                                  b'[{"eventType": "4294967296"}]', b'[{"eventId": 1, "x": 1-2e}]',
                                  b'[{"eventId": 1, "x": 01}]', b'[{"eventId": 1, "x": 1.}]',
                                  b'[{"eventId": 1, "x": 1e+}]', b'[{"eventId": 1, "x": "\\q"}]',
                                  b'[{"eventId": 1, "x": fals}]',
                                  b'[{"eventId": 1, "eventType": "ActivityTaskScheduled", '
                                  b'"activityTaskScheduledEventAttributes": {"activityId": 7}}]',
                                  b'[{"eventId": 1, "x": ' + b'[' * 10001 + b']' * 10001 + b'}]',
                                  b'[{"eventId": 1, "x": ' + b'[' * 200000 + b'}]'],
                         ids=lambda b: b[:40].decode(errors="replace"))
def test_json_rejections_on_device_match_host(eng, blob):
    """Each malformed blob fails the device ingest with the host decoder's code and blob index."""
    from cadence_amd.ingest import IngestError
    src = [WorkflowSource(blobs=[json.dumps([event_json(e) for e in _events()]).encode(), blob],
                          encodings=["json", "json"])]
    with pytest.raises(DeserializationError) as he:
        decode_histories(src)
    with pytest.raises(IngestError) as de:
        _device(eng, src)
    assert (de.value.code, de.value.blob) == (he.value.code, he.value.blob) == (-5, 1)


@pytest.mark.gpu
def test_lowest_failing_blob_wins_across_encodings(eng):
    """A corrupt thriftrw blob before a rejected JSON blob: the host reports the thriftrw one (the plan's
    error); after it, the JSON one (the transcode's); an unknown encoding fails whatever its length."""
    from cadence_amd.ingest import IngestError
    good = json.dumps([event_json(e) for e in _events()]).encode()
    hs = synth_mixed.mixed_histories(4, 44)
    bad_thrift = b"\x58" + serialize_history(hs[0])[0][1:]
    for blobs, encs in (([good, bad_thrift, b"[1"], ["json", "thriftrw", "json"]),
                        ([good, b"[1", bad_thrift], ["json", "json", "thriftrw"]),
                        ([good, b"", good], ["json", "gob", "json"])):
        src = [WorkflowSource(blobs=blobs, encodings=encs)]
        with pytest.raises(DeserializationError) as he:
            decode_histories(src)
        with pytest.raises(IngestError) as de:
            _device(eng, src)
        assert (de.value.code, de.value.blob) == (he.value.code, he.value.blob)


@pytest.mark.gpu
def test_nesting_to_the_depth_limit_on_device(eng):
    """10000 levels (the batch array, the event object and 9998 in a skipped value) decode: the deep pass's
    level stack in HBM; a blob at 64..100 levels too."""
    evs = _events()
    text = json.dumps([event_json(e) for e in evs]).encode()
    srcs = []
    for d in (9998, 70, 62):
        deep = b'[' * d + b']' * d
        srcs.append(WorkflowSource(blobs=[text.replace(b'"eventId": 1,', b'"eventId": 1, "x": ' + deep + b',', 1)],
                                   encodings=["json"]))
    ing, _tdb = _check(eng, srcs)
    assert int(ing.last_transcode.n_deep) == 2


@pytest.mark.gpu
def test_empty_and_null_json_blobs_on_device(eng):
    good = json.dumps([event_json(e) for e in _events()]).encode()
    srcs = [WorkflowSource(blobs=[good, b"", b"null", b" [ ] "], encodings=["json", "json", "json", ""]),
            WorkflowSource(blobs=[], encodings=[])]
    _check(eng, srcs)


@pytest.mark.gpu
def test_archival_fixture_json_on_device(eng):
    """The reference's own types-JSON history (archiver testdata, 112 events), one JSON blob per batch."""
    raw = json.load(open(ARCHIVAL))
    batches = split_batches_by_task_id(events_from_json(raw))
    blobs, i = [], 0
    for b in batches:
        blobs.append(json.dumps(raw[i:i + len(b)]).encode())
        i += len(b)
    _check(eng, [WorkflowSource(blobs=blobs, encodings=["json"] * len(blobs))], replay=True)


@pytest.mark.gpu
def test_blobs_outgrowing_their_staging_region(eng):
    """JSON far shorter than its thriftrw form (bare event objects: every field defaulted) outgrows the
    plan's staging region and is walked again by the transcode; and a scratch with a staging area for only a
    fraction of the bytes leaves the rest unstaged -- both byte-identical to the host path."""
    good = json.dumps([event_json(e) for e in _events()]).encode()
    srcs = [WorkflowSource(blobs=[good, b"[{},{},{}]", b'[{"eventType":"TimerFired"},{"eventId":9}]', good],
                           encodings=["json"] * 4)]
    _check(eng, srcs)
    hs = synth_mixed.mixed_histories(300, 45, multi_version=True, can_rate=0.3)
    src = json_sources(hs)
    n = sum(len(b) for s in src for b in s.blobs)
    for stage in (0, n // 3):
        _check(eng, src, stage_bytes=stage)


@pytest.mark.gpu
@pytest.mark.parametrize("gen", ["mixed", "long_tail"])
def test_native_json_workloads_on_device(eng, gen):
    """The bench's JSON workloads at test size (blobs.encode_batch(json=True) over the native generators: every
    event type, unknown domains, invalid histories, CAN chains, histories past the lane limit): the device
    layout equals the host JSON path's and the rows the oracle's."""
    from cadence_amd import synth_native
    from cadence_amd.blobs import encode_batch
    if gen == "mixed":
        b = synth_native.mixed(20000, multi_version=True, invalid_rate=0.05, can_rate=0.2, unknown_domain_rate=0.1)
    else:
        b = synth_native.long_tail(30, max_len=12_000, run_cap=4_000)
    src = encode_batch(b, json=True).to_sources()
    for s in src:
        s.encodings = ["json"] * len(s.blobs)
    _check(eng, src, replay=True)


@pytest.mark.gpu
def test_attribute_objects_of_several_types(eng):
    """An event carrying attribute objects of other types before / after its own (and its own twice): the
    last occurrence of its own type's key is read, whatever came after it."""
    base = {"eventId": 2, "version": 7, "timestamp": 5, "taskId": 3}
    own = {"startToCloseTimeoutSeconds": 9, "attempt": 4}
    other = {"timeoutType": "HEARTBEAT"}
    evs = []
    for order in (("own", "other"), ("other", "own"), ("own", "other", "own2"), ("other", "other")):
        parts = [json.dumps(base)[:-1], '"eventType": "DecisionTaskScheduled"']
        for o in order:
            if o == "own":
                parts.append('"decisionTaskScheduledEventAttributes": ' + json.dumps(own))
            elif o == "own2":
                parts.append('"decisionTaskScheduledEventAttributes": ' + json.dumps({"attempt": 8}))
            else:
                parts.append('"decisionTaskTimedOutEventAttributes": ' + json.dumps(other))
        evs.append(", ".join(parts) + "}")
    blobs = ["[" + e + "]" for e in evs]
    _check(eng, [WorkflowSource(blobs=[b.encode() for b in blobs], encodings=["json"] * len(blobs))])


@pytest.mark.gpu
def test_type_errors_in_unread_occurrences(eng):
    """An attribute object of the event's own type with a type error in a read field fails the blob only when
    it is the occurrence the host reads (the last): an earlier bad one followed by a good one decodes, a good
    one followed by a bad one is rejected -- and an eventType after the attributes, or changed by a duplicate,
    reads the attributes of the final type."""
    from cadence_amd.ingest import IngestError
    good = '"activityTaskScheduledEventAttributes": {"activityId": "a1", "scheduleToCloseTimeoutSeconds": 5}'
    bad = '"activityTaskScheduledEventAttributes": {"activityId": 7}'
    head = '{"eventId": 1, "version": 1, "eventType": "ActivityTaskScheduled", '
    ok_blobs = ["[" + head + bad + ", " + good + "}]",
                '[{"eventId": 1, "version": 1, ' + good + ', "eventType": "ActivityTaskScheduled"}]',
                "[" + head + good + ', "eventType": "TimerStarted", "timerStartedEventAttributes": {"timerId": "t"}}]',
                "[" + head + good + ', "eventType": "TimerStarted"}]']
    _check(eng, [WorkflowSource(blobs=[b.encode() for b in ok_blobs], encodings=["json"] * len(ok_blobs))])
    src = [WorkflowSource(blobs=[("[" + head + good + ", " + bad + "}]").encode()], encodings=["json"])]
    with pytest.raises(DeserializationError) as he:
        decode_histories(src)
    with pytest.raises(IngestError) as de:
        _device(eng, src)
    assert (de.value.code, de.value.blob) == (he.value.code, he.value.blob)
