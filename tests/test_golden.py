"""Golden fixtures (tests/golden/*.npz, checksum_vectors.json; generator: tests/golden/make_golden.py).

The inputs are stored flattened and the expected rows with them, so these tests pin the replay
independently of the synthetic generators.  CPU: the oracle reproduces every stored row, and the
independent pure-Python checksum encoder (oracle/checksum_py.py) rebuilds every stored payload from
the stored rows.  GPU: the HIP engine reproduces every stored row and CRC, in the canonical and the
wave-interleaved layouts.  Integer work: bit-exact.
"""
import json
import os
import sys

import numpy as np
import pytest

from cadence_amd.flatten import interleave
from cadence_amd.result import diff_results

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, HERE)
from make_golden import load_case  # noqa: E402

CASES = ["c1_activity_chain", "mixed_multiversion", "mixed_rebuild", "archival"]


def _vectors():
    with open(os.path.join(HERE, "checksum_vectors.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", CASES)
def test_oracle_reproduces_golden(name):
    from oracle import oracle
    batch, want = load_case(os.path.join(HERE, f"{name}.npz"))
    got = oracle.replay(batch, 1)
    d = diff_results(batch, got, batch, want)
    assert not d, "\n".join(d)
    vec = _vectors()[name]
    assert len(vec) == batch.n_wf
    for w, v in enumerate(vec):
        assert int(got.exec["status"][w]) == v["status"] and int(got.exec["fail_step"][w]) == v["fail_step"]
        if v["status"] == 0:
            assert oracle.payload(batch, w).hex() == v["payload"]
            assert f"{int(got.exec['checksum'][w]):08x}" == v["checksum"]


@pytest.mark.parametrize("name", CASES)
def test_python_encoder_reproduces_golden_payloads(name):
    from oracle import checksum_py
    batch, want = load_case(os.path.join(HERE, f"{name}.npz"))
    n_ok = 0
    for w, v in enumerate(_vectors()[name]):
        if v["status"] != 0:
            continue
        e = want.exec[w]
        p = checksum_py.payload_from_rows(e, want.live_rows(batch, w),
                                          checksum_py.token_of(batch, w, int(e["token_src"])))
        assert p.hex() == v["payload"], f"{name}[{w}]"
        assert checksum_py.checksum_value(p).hex() == v["checksum"]
        n_ok += 1
    assert n_ok > 0


def test_golden_cases_cover_the_edges():
    """The fixtures hold what they claim: failures, multi-item VH, pending maps, rebuild tokens."""
    vec = _vectors()
    statuses = {r["status"] for rows in vec.values() for r in rows}
    assert 0 in statuses and len(statuses) >= 4          # several Go error kinds
    batch, want = load_case(os.path.join(HERE, "mixed_multiversion.npz"))
    assert (want.exec["n_vh_items"] > 1).any()
    for n in ("n_activity", "n_timer", "n_child", "n_rc", "n_signal"):
        assert (want.exec[n][want.exec["status"] == 0] > 0).any(), n
    batch, want = load_case(os.path.join(HERE, "mixed_rebuild.npz"))
    assert (want.exec["token_src"] == 2).any()
    assert np.unique(want.exec["checksum"][want.exec["status"] == 0]).size == int((want.exec["status"] == 0).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_device_reproduces_golden(name):
    from cadence_amd.engine import ReplayEngine
    eng = ReplayEngine(0)
    batch, want = load_case(os.path.join(HERE, f"{name}.npz"))
    got = eng.replay(batch)
    d = diff_results(batch, got, batch, want)
    assert not d, "\n".join(d)
    ib = interleave(batch)
    got_i = eng.replay(ib)
    d = diff_results(ib, got_i, batch, want)
    assert not d, "\n".join(d)
    for w, v in enumerate(_vectors()[name]):
        if v["status"] == 0:
            assert f"{int(got.exec['checksum'][w]):08x}" == v["checksum"]
