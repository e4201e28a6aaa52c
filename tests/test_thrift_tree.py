"""The test helper that re-shapes blobs (tests/thrift_tree.py): a parse / write round trip is the
identity, and re-shaped blobs decode on the host (history_decode.cpp) to the same canonical batch."""
import random

import numpy as np

from cadence_amd import synth_native
from cadence_amd.blobs import KNOWN_DOMAINS, encode_batch
from cadence_amd.decode import decode_histories

from thrift_tree import MODES, parse_blob, reshape_blob, reshape_blobset, write_blob


def test_round_trip_identity():
    bs = encode_batch(synth_native.mixed(50, mean_len=30))
    for i in range(bs.n_blobs):
        b = bs.blob(i)
        if b:
            assert write_blob(parse_blob(b)) == b


def test_reshaped_blobs_decode_to_the_same_batch():
    b = synth_native.mixed(300, mean_len=30)
    bs = encode_batch(b)
    rs = reshape_blobset(bs, seed=3, rate=0.5)
    assert rs.n_bytes > bs.n_bytes
    want = decode_histories(bs.to_sources(), known_domains=KNOWN_DOMAINS)
    got = decode_histories(rs.to_sources(), known_domains=KNOWN_DOMAINS)
    for name in want.cols:
        np.testing.assert_array_equal(got.cols[name], want.cols[name], err_msg=name)
    assert got.act_side.tobytes() == want.act_side.tobytes()
    assert got.start_side.tobytes() == want.start_side.tobytes()


def test_every_mode_applies():
    rng = random.Random(1)
    bs = encode_batch(synth_native.mixed(20, mean_len=30))
    blob = next(bs.blob(i) for i in range(bs.n_blobs) if len(bs.blob(i)) > 100)
    ev = next(f for f in parse_blob(blob) if f[1] == 10)[2][1][0]
    from thrift_tree import reshape_event
    for m in MODES:
        out = reshape_event(ev, rng, m)
        assert isinstance(out, list)
    assert reshape_blob(blob, rng, 0.0) == blob
