"""CPU: the key dictionaries PassiveReplication.verify_oracle builds from the events' own key strings name
the same strings as the flattener's interners, for every key id a workflow's events carry."""
import numpy as np

from cadence_amd import synth_mixed
from cadence_amd.flatten import flatten, interleave
from cadence_amd.replication import key_dict_from_events


def _strings(kd, w):
    begin, count, off, ln, arena = kd
    b, c = int(begin[w]), int(count[w])
    return [bytes(arena[int(off[b + k]):int(off[b + k]) + int(ln[b + k])]).decode() for k in range(c)]


def test_key_dict_from_events_matches_interners():
    b = flatten(synth_mixed.mixed_histories(300, 17, multi_version=True),
                known_domains={"domain-a", "domain-b", "parent-domain"})
    for batch in (b, interleave(b, long_threshold=64)):
        kd = key_dict_from_events(batch)
        cnt = batch.wf["ev_count"].astype(np.int64)
        st = batch.wf_strides()
        for w in range(batch.n_wf):
            want, got = _strings(batch.key_dict, w), _strings(kd, w)
            x = batch.wf["ev_begin"][w] + np.arange(cnt[w]) * st[w]
            used = sorted(set(int(k) for k in batch.cols["key"][x]))
            for k in used:
                assert got[k] == want[k], (w, k)


import pytest


@pytest.mark.parametrize("gen", ["python", "native"])
def test_resume_blob_set_carries_the_last_batches(gen):
    """The replication tasks' payloads replication.resume_blob_set cuts from the whole histories' blobs decode
    (host decoder) to exactly the new events the host path applies (suffix_batch), and the seeded dictionaries
    hold the prefix's key strings in id order."""
    import dataclasses
    from cadence_amd import abi
    from cadence_amd.abi import EventType as ET
    from cadence_amd.blobs import KNOWN_DOMAINS, encode_batch
    from cadence_amd.decode import decode_histories
    from cadence_amd.replication import last_batch_cut, resume_blob_set, split_descriptors, suffix_batch
    if gen == "native":   # (the GPU test's workload: previous reset points interned by the Started events)
        from cadence_amd import synth_native
        canon = synth_native.mixed(20000, can_rate=0.3, multi_version=True)
    else:
        canon = flatten(synth_mixed.mixed_histories(800, 46, mean_len=60, multi_version=True, can_rate=0.3),
                        known_domains={"domain-a", "domain-b", "parent-domain"})
    b = interleave(canon, long_threshold=150)
    cut = last_batch_cut(b)
    pre, suf, split = split_descriptors(b, cut)
    bs, seeds = resume_blob_set(b, encode_batch(canon), cut, split, pre)
    assert bs.n_wf == b.n_wf and int(bs.wf["blob_count"].sum()) >= int(split.sum()) > 200
    dec = decode_histories(bs.to_sources(), known_domains=KNOWN_DOMAINS)
    sb = suffix_batch(b, cut, split, suf)
    cnt = sb.wf["ev_count"].astype(np.int64)
    assert dec.wf["ev_count"].astype(np.int64).tolist() == cnt.tolist()
    st = sb.wf_strides()
    wf_idx = np.repeat(np.arange(b.n_wf), cnt)
    k = np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    x = sb.wf["ev_begin"].astype(np.int64)[wf_idx] + k * st[wf_idx]
    y = dec.wf["ev_begin"].astype(np.int64)[wf_idx] + k
    for name in ("etype", "event_id", "version", "timestamp", "task_id", "ref"):
        np.testing.assert_array_equal(dec.cols[name][y], sb.cols[name][x], err_msg=name)
    # seeds + the new batch's strings, interned as the device does (WfFlattener::key_of continued from the
    # loaded dictionary) give the host path's key ids
    raw = bs.bytes.tobytes()
    keyed = (ET.DecisionTaskCompleted, ET.ActivityTaskScheduled, ET.ActivityTaskCancelRequested, ET.TimerStarted,
             ET.TimerFired, ET.TimerCanceled)
    darena = dec.key_arena.tobytes()
    checked = 0
    for p in range(b.n_wf):
        kb, kc = int(seeds["key_begin"][p]), int(seeds["key_count"][p])
        d = {raw[int(seeds["key_off"][kb + i]):int(seeds["key_off"][kb + i]) + int(seeds["key_len"][kb + i])]: i + 1
             for i in range(kc)}
        assert len(d) == kc   # distinct strings
        nxt = kc + 1
        for j in range(int(cnt[p])):
            yy, xx = int(dec.wf["ev_begin"][p]) + j, int(sb.wf["ev_begin"][p]) + j * int(st[p])
            if (dec.cols["etype"][yy] & abi.ETYPE_MASK) not in keyed or dec.key_len[yy] == 0:
                continue
            sv = darena[int(dec.key_off[yy]):int(dec.key_off[yy]) + int(dec.key_len[yy])]
            if sv not in d:
                d[sv] = nxt
                nxt += 1
            assert d[sv] == int(sb.cols["key"][xx]), (p, j)
            checked += 1
    assert checked > 200
