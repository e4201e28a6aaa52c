"""Narrow upload format (cadence_amd/wire.py, crr_widen_events): the host packer against its own
restatement of the device decoder, on every layout, plus extreme values."""
import numpy as np
import pytest

from cadence_amd import abi, synth, synth_mixed, synth_native
from cadence_amd.flatten import flatten, interleave
from cadence_amd.wire import pack_events, unpack_events

KNOWN = {"domain-a", "domain-b", "parent-domain"}


def _check(b):
    pk = pack_events(b)
    cols = unpack_events(b, pk)
    for name, _t in abi.EVENT_COLUMNS:
        if name == "etype":
            continue
        assert (cols[name] == b.cols[name]).all(), name
    return pk


def test_config2_is_narrow():
    b = interleave(synth.activity_chain(5000, 4, synth.SEED_C2, wf_ids=np.arange(5000)))
    pk = _check(b)
    per_event = (pk.nbytes + b.n_slots) / b.n_events        # + the etype byte
    assert per_event < 16, (pk.width, per_event)


@pytest.mark.parametrize("layout", ["canonical", "interleaved", "tail"])
def test_mixed_round_trip(layout):
    canon = flatten(synth_mixed.mixed_histories(800, 3, mean_len=80, multi_version=True, invalid_rate=0.1,
                                                can_rate=0.3), known_domains=KNOWN)
    b = canon if layout == "canonical" else interleave(canon, long_threshold=None if layout == "interleaved" else 100)
    _check(b)


def test_native_long_tail_round_trip():
    _check(interleave(synth_native.long_tail(30)))


@pytest.mark.parametrize("interleaved", [False, True])
def test_extreme_values_take_full_width(interleaved):
    b = synth.activity_chain(100, 2, 7)
    if interleaved:
        b = interleave(b)
    rng = np.random.default_rng(1)
    real = (b.cols["etype"] & abi.ETYPE_MASK) != abi.EV_PAD
    for c in ("event_id", "version", "timestamp", "task_id", "ref"):
        v = rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, size=b.n_slots, dtype=np.int64)
        b.cols[c] = np.where(real, v, 0)
    b.cols["key"] = np.where(real, rng.integers(0, 2 ** 32, size=b.n_slots, dtype=np.uint64), 0).astype(np.uint32)
    b.cols["aux"] = np.where(real, rng.integers(-2 ** 31, 2 ** 31, size=b.n_slots, dtype=np.int64), 0).astype(np.int32)
    pk = _check(b)
    assert pk.width["timestamp"] == 8 and pk.width["key"] == 4 and pk.width["aux"] == 4
