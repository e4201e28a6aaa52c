"""GPU: the reference's dispatch-table spec (state_builder_test.go:143-1744) and timer-sequence
creation tests (timer_sequence_test.go:74-231), restated in tests/kat_state_builder.py, replayed by the HIP engine through the C ABI -- every case's expected
Replicate* effects and Generate* tasks, in the canonical and the wave-interleaved layouts, and
bit-exact against the oracle."""
import pytest

from cadence_amd.flatten import interleave
from cadence_amd.result import diff_results

import kat_state_builder as K

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("suite", ["state_builder", "timer_sequence", "mutable_state_builder"])
@pytest.mark.parametrize("layout", ["canonical", "interleaved"])
def test_device_dispatch_table_kats(layout, suite):
    from cadence_amd.engine import ReplayEngine
    from oracle import oracle
    eng = ReplayEngine(0)
    kats = {"state_builder": K.cases, "timer_sequence": K.timer_cases, "mutable_state_builder": K.msb_cases}[suite]()
    batch, idx, nr = K.build_batch(kats)
    if layout == "interleaved":
        ib = interleave(batch)
        pos = {int(c): p for p, c in enumerate(ib.perm)}
        idx = [pos[w] for w in idx]
        nr = [None if w is None else pos[w] for w in nr]
        batch = ib
    got = eng.replay(batch)
    fails = K.check_all(kats, batch, got, idx, nr)
    assert not fails, "\n".join(fails)
    d = diff_results(batch, got, batch, oracle.replay(batch, 1))
    assert not d, "\n".join(d)
