"""JSON-encoded history blobs (serializer.go:321-328: json / unknown / empty encodings go through
json.Unmarshal into []*types.HistoryEvent) through the native decoder (cadence_amd/csrc/json_decode.cpp)
against the host flattening of the same events.  Parity anchor held by the reference: the archival
fixture service/worker/archiver/testdata/archival_workflow_history_v1.json is that same types JSON."""
import json

import numpy as np
import pytest

from cadence_amd import synth_mixed
from cadence_amd.abi import EventType as ET
from cadence_amd.decode import DeserializationError, WorkflowSource, decode_histories
from cadence_amd.flatten import flatten
from cadence_amd.history import HistoryEvent, WorkflowHistory, events_from_json, split_batches_by_task_id
from cadence_amd.json_codec import event_json, serialize_history_json
from cadence_amd.thrift_codec import serialize_history

from test_decode import ARCHIVAL, KNOWN, assert_same_batch

SEC = 1_000_000_000


def json_sources(hs, encoding="json"):
    out = []
    for h in hs:
        nr = None
        for e in h.events:
            if e.event_type == ET.WorkflowExecutionContinuedAsNew and e.attrs.get("new_run") is not None:
                nr = int(e.attrs["new_run"])
        blobs = serialize_history_json(h)
        out.append(WorkflowSource(blobs=blobs, run_id=h.run_id, branch_id=h.branch_id,
                                  domain_failover_version=h.domain_failover_version, now_ns=h.now_ns,
                                  final_token=h.final_token, rebuild_last_event_id=h.rebuild_last_event_id,
                                  rebuild_last_event_version=h.rebuild_last_event_version, new_run=nr,
                                  is_new_run=h.is_new_run, refresh_tasks=h.refresh_tasks,
                                  encodings=[encoding] * len(blobs)))
    return out


def test_json_histories_decode_like_flatten():
    hs = synth_mixed.mixed_histories(400, 32, multi_version=True, invalid_rate=0.25, can_rate=0.5)
    assert_same_batch(decode_histories(json_sources(hs), known_domains=KNOWN), flatten(hs, known_domains=KNOWN))


@pytest.mark.parametrize("encoding", ["", "unknow"])   # EncodingTypeEmpty / Unknown ("unknow", constants.go:66)
def test_backward_compatible_encodings_decode_as_json(encoding):
    hs = synth_mixed.mixed_histories(50, 33, multi_version=True)
    assert_same_batch(decode_histories(json_sources(hs, encoding), known_domains=KNOWN), flatten(hs, known_domains=KNOWN))


def test_mixed_encodings_in_one_call():
    hs = synth_mixed.mixed_histories(120, 34, multi_version=True, can_rate=0.3)
    src = json_sources(hs)
    for i, (s, h) in enumerate(zip(src, hs)):
        if i % 3 == 0:    # thriftrw blobs for some workflows, per blob for others
            s.blobs, s.encodings = serialize_history(h), None
        elif i % 3 == 1 and len(s.blobs) > 1:
            tb = serialize_history(h)
            s.blobs = [tb[0]] + s.blobs[1:]
            s.encodings = ["thriftrw"] + s.encodings[1:]
    assert_same_batch(decode_histories(src, known_domains=KNOWN), flatten(hs, known_domains=KNOWN))


def _events():
    return [HistoryEvent(int(ET.WorkflowExecutionStarted), 1, 7, 100 * SEC, 11,
                         {"task_start_to_close_timeout_seconds": 10, "execution_start_to_close_timeout_seconds": 600,
                          "initiator": 1, "first_decision_task_backoff_seconds": 0,
                          "prev_auto_reset_points": ["bc-1", "bc-2"]}),
            HistoryEvent(int(ET.DecisionTaskScheduled), 2, 7, 101 * SEC, 12,
                         {"start_to_close_timeout_seconds": 10, "attempt": 0}),
            HistoryEvent(int(ET.DecisionTaskTimedOut), 3, 7, 102 * SEC, 13, {"timeout_type": 3})]


def test_go_json_conventions():
    """encoding/json: keys match case-insensitively, enums by name in any case or as decimal text (in
    a JSON string: UnmarshalText), null leaves a field unset, unknown keys are ignored, the last of
    duplicate keys wins."""
    evs = _events()
    raw = [event_json(e) for e in evs]
    raw[0] = {k.upper(): v for k, v in raw[0].items()}              # "EVENTID", "EVENTTYPE", ...
    raw[0]["EVENTTYPE"] = "workflowexecutionstarted"
    attrs = raw[0]["WORKFLOWEXECUTIONSTARTEDEVENTATTRIBUTES"]
    attrs["initiator"] = "retrypolicy"
    attrs["somethingNew"] = {"nested": [1, 2.5e3, None, True, "x\\u00e9"]}
    raw[1]["eventType"] = "+4"                                       # UnmarshalText: strconv.ParseInt
    raw[1]["decisionTaskScheduledEventAttributes"]["attempt"] = None   # null: stays 0
    raw[2]["decisionTaskTimedOutEventAttributes"]["timeoutType"] = "3"  # UnmarshalText's numeric fallback
    text = json.dumps(raw).replace('"version": 7', '"version": 99, "version": 7', 1)   # duplicate: last wins
    src = [WorkflowSource(blobs=[text.encode()], encodings=["json"])]
    got = decode_histories(src, known_domains=KNOWN)
    want = flatten([WorkflowHistory(batches=[evs])], known_domains=KNOWN)
    assert_same_batch(got, want)


@pytest.mark.parametrize("blob", [b'[{"eventId": 1.5}]', b'[{"eventId": "1"}]', b'[{"eventId": 1}', b'[null]',
                                  b'[{"eventType": "NoSuchEvent"}]', b'[{"eventId": 99999999999999999999}]',
                                  b'{"eventId": 1}', b'[{"eventId": 1}] x',
                                  # enums implement UnmarshalText only: a bare number is a type error, and
                                  # so is Go's own MarshalText of an out-of-range type
                                  b'[{"eventType": 4}]', b'[{"eventType": "EventType(99)"}]',
                                  b'[{"eventType": " 4"}]', b'[{"eventType": "4294967296"}]',
                                  # the JSON number grammar, inside a skipped value too
                                  b'[{"eventId": 1, "x": 1-2e}]', b'[{"eventId": 1, "x": 01}]',
                                  b'[{"eventId": 1, "x": 1.}]', b'[{"eventId": 1, "x": 1e+}]',
                                  # nesting past encoding/json's maxNestingDepth (10000)
                                  b'[{"eventId": 1, "x": ' + b'[' * 10001 + b']' * 10001 + b'}]',
                                  b'[{"eventId": 1, "x": ' + b'[' * 1000000 + b'}]'])
def test_json_errors_are_deserialization_errors(blob):
    src = [WorkflowSource(blobs=[json.dumps([event_json(e) for e in _events()]).encode(), blob],
                          encodings=["json", "json"])]
    with pytest.raises(DeserializationError) as ei:
        decode_histories(src)
    assert ei.value.code == -5 and ei.value.blob == 1


@pytest.mark.parametrize("encoding", ["gob", "unknown"])
def test_unknown_encoding_rejected(encoding):   # NewUnknownEncodingTypeError (serializer.go:326-327)
    src = [WorkflowSource(blobs=[b"[]"], encodings=[encoding])]
    with pytest.raises(DeserializationError) as ei:
        decode_histories(src)
    assert ei.value.code == -6


def test_unread_attributes_are_syntax_checked_only():
    """Documented narrowing (json_decode.h): an attributes object of another event type is checked for
    JSON syntax, not decoded into its Go struct, so a type error json.Unmarshal would report there (a
    bare-number timeoutType under decisionTaskTimedOutEventAttributes of a DecisionTaskScheduled event)
    is accepted.  Pinned so a change in either direction is deliberate."""
    blob = (b'[{"eventId": 2, "version": 7, "eventType": "DecisionTaskScheduled", '
            b'"decisionTaskTimedOutEventAttributes": {"timeoutType": 3}}]')
    got = decode_histories([WorkflowSource(blobs=[blob], encodings=["json"])])
    assert got.n_events == 1


def test_nesting_within_the_depth_limit_is_accepted():
    """A skipped value nested to exactly encoding/json's limit decodes (10000 levels with the batch
    array and the event object)."""
    evs = _events()
    text = json.dumps([event_json(e) for e in evs])
    deep = b'[' * 9998 + b']' * 9998
    blob = text.encode().replace(b'"eventId": 1,', b'"eventId": 1, "x": ' + deep + b',', 1)
    got = decode_histories([WorkflowSource(blobs=[blob], encodings=["json"])])
    assert_same_batch(got, flatten([WorkflowHistory(batches=[evs])]))


def test_empty_json_blob_is_an_empty_batch():   # DeserializeBatchEvents: len(data) == 0 -> no events
    evs = _events()
    src = [WorkflowSource(blobs=[json.dumps([event_json(e) for e in evs]).encode(), b""], encodings=["json", "json"])]
    got = decode_histories(src)
    want = flatten([WorkflowHistory(batches=[evs, []])])
    assert_same_batch(got, want)


def test_archival_fixture_json_decodes_natively():
    """The reference's own types-JSON history (archiver testdata, 112 events): each persisted batch
    re-emitted as a JSON blob of the fixture's raw event objects, decoded natively, equals the host
    reading of the same file."""
    raw = json.load(open(ARCHIVAL))
    evs = events_from_json(raw)
    batches = split_batches_by_task_id(evs)
    blobs, i = [], 0
    for b in batches:
        blobs.append(json.dumps(raw[i:i + len(b)]).encode())
        i += len(b)
    src = [WorkflowSource(blobs=blobs, encodings=["json"] * len(blobs))]
    got = decode_histories(src)
    want = flatten([WorkflowHistory(batches=batches)])
    assert_same_batch(got, want)
    assert got.n_events == 112


def test_blobset_from_sources_round_trips():
    """blobs.blobset_from_sources (the device ingest's upload layout of host-decoder inputs, any encoding)
    inverts BlobSet.to_sources: the same blobs, encodings and per-workflow inputs decode to the same batch."""
    from cadence_amd.blobs import blobset_from_sources
    from cadence_amd.decode import ENCODINGS
    hs = synth_mixed.mixed_histories(60, 35, multi_version=True, can_rate=0.3)
    src = json_sources(hs)
    src[3].blobs, src[3].encodings = serialize_history(hs[3]), None
    src[5].encodings = [""] * len(src[5].blobs)
    bs, enc = blobset_from_sources(src)
    assert bs.n_blobs == sum(len(s.blobs) for s in src) == enc.size
    back = bs.to_sources()
    names = {v: k for k, v in ENCODINGS.items()}
    k = 0
    for s in back:
        s.encodings = [names[int(e)] for e in enc[k:k + len(s.blobs)]]
        k += len(s.blobs)
    assert_same_batch(decode_histories(back, known_domains=KNOWN), decode_histories(src, known_domains=KNOWN))


@pytest.mark.parametrize("gen", ["native", "python"])
def test_native_json_encoder_decodes_back(gen):
    """blobs.encode_batch(json=True) (blob_encode.cpp: the events as common/types JSON, the bench's JSON
    workloads) read back by the host JSON decoder equals the host decoding of the thriftrw encoding."""
    from cadence_amd import synth_native
    from cadence_amd.blobs import KNOWN_DOMAINS, encode_batch
    if gen == "native":
        b = synth_native.mixed(2000, multi_version=True, invalid_rate=0.1, can_rate=0.3, unknown_domain_rate=0.2)
    else:
        b = flatten(synth_mixed.mixed_histories(300, 36, multi_version=True, invalid_rate=0.2, can_rate=0.4),
                    known_domains=set(KNOWN_DOMAINS))
    tj, tt = encode_batch(b, json=True), encode_batch(b)
    src = tj.to_sources()
    for s in src:
        s.encodings = ["json"] * len(s.blobs)
    assert_same_batch(decode_histories(src, known_domains=KNOWN_DOMAINS),
                      decode_histories(tt.to_sources(), known_domains=KNOWN_DOMAINS))
