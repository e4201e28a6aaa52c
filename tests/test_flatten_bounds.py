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
