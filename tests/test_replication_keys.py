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
