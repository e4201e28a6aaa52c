"""flatten.live_set_bounds compares inserted and deleted IDs exactly (all 64 bits), like the device
ingest's bound table (ingest_kernel.hip)."""
import copy

from cadence_amd import abi, synth_mixed
from cadence_amd.flatten import flatten, live_set_bounds

KNOWN = {"domain-a", "domain-b", "parent-domain"}


def test_deletes_of_ids_differing_above_bit_40_do_not_count():
    hs = synth_mixed.mixed_histories(300, 31, multi_version=False)
    hs0 = copy.deepcopy(hs)
    for h in hs:
        for batch in h.batches:
            for e in batch:
                if e.event_type == abi.EventType.ActivityTaskCompleted:
                    e.attrs["scheduled_event_id"] = int(e.attrs["scheduled_event_id"]) + (1 << 40)
    b, b0 = flatten(hs, known_domains=KNOWN), flatten(hs0, known_domains=KNOWN)
    got, base = live_set_bounds(b)["act"], live_set_bounds(b0)["act"]
    # every completion became a delete of a missing entry: the bound is the number of schedules
    assert (got >= base).all() and (got > base).any()


def test_interleave_joins_started_events_to_their_scheduled_side_records():
    """CRR_IN_STARTED_AUX: after interleave, every ActivityTaskStarted whose ActivityTaskScheduled is in the same
    history (ID - ScheduledEventID steps earlier) carries that event's re-homed act_side index; the others -1.
    Checked against a plain search over the canonical batch, on lane groups and on the wavefront tail."""
    import numpy as np
    from cadence_amd.flatten import interleave
    ET = abi.EventType
    hs = synth_mixed.mixed_histories(600, 33, mean_len=80, multi_version=True, invalid_rate=0.1, can_rate=0.2)
    canon = flatten(hs, known_domains=KNOWN)
    for lt in (256, 60):
        b = interleave(canon, long_threshold=lt)
        assert b.started_aux and (b.c_flags() & abi.IN_STARTED_AUX)
        joined = missing = 0
        for p in range(b.n_wf):
            w = int(b.perm[p])
            n = int(canon.wf["ev_count"][w])
            c0 = int(canon.wf["ev_begin"][w])
            et = canon.cols["etype"][c0:c0 + n] & abi.ETYPE_MASK
            ids = canon.cols["event_id"][c0:c0 + n]
            d0, st = int(b.wf["ev_begin"][p]), int(b.wf_strides()[p])
            for k in np.nonzero(et == ET.ActivityTaskStarted)[0]:
                ref = int(canon.cols["ref"][c0 + k])
                hit = [j for j in range(k) if et[j] == ET.ActivityTaskScheduled and int(ids[j]) == ref]
                got = int(b.cols["aux"][d0 + k * st])
                if hit and int(ids[k]) - ref == k - hit[-1]:
                    want = int(b.cols["aux"][d0 + hit[-1] * st])
                    assert got == want and (b.act_side[got] == canon.act_side[canon.cols["aux"][c0 + hit[-1]]]), (p, k)
                    joined += 1
                else:
                    assert got == -1, (p, k, got)
                    missing += 1
        assert joined > 1000
