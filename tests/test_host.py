"""Host-side logic without a GPU: C-ABI library exports, flattening, interleaving, digests."""
import ctypes
import os
import re

import numpy as np
import pytest

from cadence_amd import abi, synth, synth_mixed
from cadence_amd.flatten import flatten, interleave
from cadence_amd.history import thrift_history_branch_token

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "cadence_amd", "libcadence_replay.so")


def _declared_symbols():
    txt = "".join(open(os.path.join(ROOT, "include", h)).read() for h in ("cadence_replay.h", "cadence_ingest.h"))
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(crr_\w+)\s*\(", txt, re.M)))


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built (run __graft_entry__.build())")
def test_library_loads_and_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    syms = _declared_symbols()
    assert {"crr_replay", "crr_checksum", "crr_set_device", "crr_abi_version", "crr_sizeof",
            "crr_crc32_ieee", "crr_last_kernel_ms", "crr_release", "crr_ingest_plan", "crr_ingest_layout",
            "crr_ingest_scratch_bytes"} <= set(syms)
    for s in syms:
        assert hasattr(lib, s), s
    lib.crr_abi_version.restype = ctypes.c_int
    assert lib.crr_abi_version() == abi.ABI_VERSION
    abi.check_layout(lib)


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_release_without_device_state_is_a_no_op():
    """crr_release (teardown of the per-device launch state) is safe to call before any launch, with no
    GPU visible: there is no state, so it touches no device and returns 0; the timing read-outs then
    report nothing rather than stale values."""
    lib = ctypes.CDLL(LIB)
    lib.crr_release.restype = ctypes.c_int
    lib.crr_last_kernel_ms.restype = ctypes.c_float
    lib.crr_last_kernel_ms.argtypes = [ctypes.c_int]
    assert lib.crr_release() == 0
    assert lib.crr_release() == 0
    assert lib.crr_last_kernel_ms(1) == -1.0
    assert lib.crr_last_kernel_ms(7) == -1.0


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_library_crc32_matches_zlib():
    import zlib
    from cadence_amd.engine import crc32
    for data in (b"", b"123456789", bytes(range(256)) * 3):
        assert crc32(data) == zlib.crc32(data)
    assert crc32(b"123456789") == 0xCBF43926


def test_engine_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from cadence_amd.engine import EngineUnavailable, ReplayEngine
    with pytest.raises(EngineUnavailable):
        ReplayEngine(0)


def test_activity_chain_shape():
    b = synth.activity_chain(100, 4, 1)
    assert b.n_wf == 100 and b.n_events == 100 * 29
    t = b.cols["etype"] & abi.ETYPE_MASK
    assert (t[:29] == synth.activity_chain_template(4)[0]).all()
    # batches: first/last flags pair up
    first = (b.cols["etype"] & abi.BATCH_FIRST) != 0
    last = (b.cols["etype"] & abi.BATCH_LAST) != 0
    assert first.sum() == last.sum() == 100 * (3 + 4 * 4)
    # branch tokens are the reference's thrift layout
    tok = bytes(b.arena[:96])
    run = tok[8:44].decode()
    br = tok[51:87].decode()
    assert tok == thrift_history_branch_token(run, br)


def test_interleave_is_a_permutation():
    hs = synth_mixed.mixed_histories(300, 5, multi_version=True)
    b = flatten(hs)
    ib = interleave(b)
    assert ib.stride == 64
    # every canonical event appears exactly once at its interleaved position
    for w in range(b.n_wf):
        p = int(np.nonzero(ib.perm == w)[0][0])
        n = int(b.wf["ev_count"][w])
        src = int(b.wf["ev_begin"][w]) + np.arange(n)
        dst = int(ib.wf["ev_begin"][p]) + np.arange(n) * 64
        for name, _ in abi.EVENT_COLUMNS:
            if name == "aux":
                continue
            assert (b.cols[name][src] == ib.cols[name][dst]).all(), (w, name)
    # group-uniform bases (the fast kernel reads them as SGPRs): base - lane constant per group
    for f in ("ev_begin", "act_base", "timer_base", "child_base", "rc_base", "sig_base", "vh_base", "rp_base"):
        v = ib.wf[f].astype(np.int64) - (np.arange(ib.n_wf) % 64)
        g = np.arange(ib.n_wf) // 64
        for gi in np.unique(g):
            assert len(np.unique(v[g == gi])) == 1, f


def test_interleave_wave_tail_layout():
    """Length bucketing: histories longer than the threshold follow the lane groups, contiguous
    (stride 1) in events and rows; row ranges of all workflows are disjoint."""
    hs = synth_mixed.mixed_histories(300, 6, mean_len=60)
    b = flatten(hs)
    ib = interleave(b, long_threshold=60)
    nl = ib.wave_begin
    cnt = ib.wf["ev_count"]
    assert 0 < nl < ib.n_wf
    assert (cnt[:nl] <= 60).all() and (cnt[nl:] > 60).all()
    assert (np.diff(cnt[nl:]) <= 0).all()                          # longest first
    st = ib.wf_strides()
    assert (st[:nl] == 64).all() and (st[nl:] == 1).all()
    for w in range(nl, ib.n_wf):
        c = int(ib.perm[w])
        n = int(b.wf["ev_count"][c])
        src = int(b.wf["ev_begin"][c]) + np.arange(n)
        dst = int(ib.wf["ev_begin"][w]) + np.arange(n)
        assert (b.cols["event_id"][src] == ib.cols["event_id"][dst]).all()
    for name, _dt, base_f, cap_f, _n in abi.TABLES:
        used = np.zeros(ib.table_rows[name] + 1, np.int32)
        for w in range(ib.n_wf):
            idx = int(ib.wf[base_f][w]) + np.arange(int(ib.wf[cap_f][w])) * int(st[w])
            used[idx] += 1
        assert used.max() <= 1, name


def test_flatten_capacities_bound_live_sets():
    from oracle import oracle
    hs = synth_mixed.mixed_histories(400, 9, multi_version=True, invalid_rate=0.1)
    b = flatten(hs, known_domains={"domain-a", "domain-b", "parent-domain"})
    r = oracle.replay(b, 2)
    for name, _dt, _b, cap_f, n_f in abi.TABLES:
        assert (r.exec[n_f] <= b.wf[cap_f]).all(), name
    assert (r.exec["status"] != abi.Status.CAPACITY).all()


def test_digest_numpy_matches_torch():
    """The digest's events field is each OK workflow's ev_count (the events this call applied), not its
    NextEventID: a resumed run (passive replication) and a continue-as-new run start past event 1."""
    import torch
    from cadence_amd import dist
    rows = np.zeros(5, abi.EXEC_ROW)
    rows["status"] = [0, 0, 3, 0, 0]
    rows["checksum"] = [1, 0xFFFFFFFF, 7, 12345, 0x80000000]
    rows["next_event_id"] = [30, 24, 5, 2 ** 31 + 7, 2 ** 40 + 2]   # resumed rows: NextEventID != events + 1
    rows["inconsistencies"] = [0, 1, 0, 2, 0]
    wf = np.zeros(5, abi.WORKFLOW)
    wf["ev_count"] = [29, 23, 4, 3, 2 ** 31 - 1]
    rows["fail_step"] = [-1, -1, 2, -1, -1]
    raw = torch.from_numpy(rows.view(np.uint8).copy())
    keys = dist.workflow_keys(np.array([10, 11, 12, 2 ** 40, 7]))
    d = dist.digest_numpy(rows, wf["ev_count"], keys)
    tk = torch.from_numpy(keys.copy())
    assert (dist.digest_torch(torch, raw, 5, torch.from_numpy(wf.view(np.uint8).copy()), tk).numpy() == d).all()
    assert d[0] == 29 + 23 + 3 + 2 ** 31 - 1
    assert d[1] == 4 and d[2] == 1 and d[5] == 3


def test_digest_binds_results_to_workflow_identity():
    """Swapping two workflows' results keeps every count and the plain checksum sum, but changes the
    identity fold (and so does swapping two failures); the folds are sums, so any partition of the
    workflows over ranks reduces to the whole job's digest."""
    import torch
    from cadence_amd import dist
    rng = np.random.default_rng(3)
    n = 1000
    rows = np.zeros(n, abi.EXEC_ROW)
    rows["status"] = np.where(rng.random(n) < 0.1, 7, 0)
    rows["checksum"] = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    rows["fail_step"] = np.where(rows["status"] != 0, rng.integers(0, 50, n), -1)
    ev = rng.integers(1, 60, n)
    keys = dist.workflow_keys(rng.permutation(10 ** 6)[:n])
    d = dist.digest_numpy(rows, ev, keys)
    ok = np.nonzero(rows["status"] == 0)[0]
    bad = np.nonzero(rows["status"] != 0)[0]
    sw = rows.copy()
    sw[[ok[0], ok[1]]] = sw[[ok[1], ok[0]]]
    ev_sw = ev.copy()
    ev_sw[[ok[0], ok[1]]] = ev_sw[[ok[1], ok[0]]]
    d_sw = dist.digest_numpy(sw, ev_sw, keys)
    assert (d_sw[[0, 1, 2, 3, 5, 6]] == d[[0, 1, 2, 3, 5, 6]]).all() and d_sw[4] != d[4]
    sf = rows.copy()
    sf["fail_step"][bad[0]] += 1
    assert dist.digest_numpy(sf, ev, keys)[6] != d[6]
    # partitions reduce to the whole (wrapping int64 sums)
    part = rng.integers(0, 4, n)
    with np.errstate(over="ignore"):
        tot = sum(dist.digest_numpy(rows[part == r], ev[part == r], keys[part == r]) for r in range(4))
    assert (tot == d).all()
    raw = torch.from_numpy(rows.view(np.uint8).copy())
    wf = np.zeros(n, abi.WORKFLOW)
    wf["ev_count"] = ev
    t = dist.digest_torch(torch, raw, n, torch.from_numpy(wf.view(np.uint8).copy()), torch.from_numpy(keys.copy()))
    assert (t.numpy() == d).all()


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_replay_rejects_unaligned_tier_segments():
    """crr_replay validates CRR_IN_TIERED segment starts (multiples of 64 below the lane count)
    before any HIP call: an unaligned boundary returns -1 instead of replaying wrong rows."""
    lib = ctypes.CDLL(LIB)
    lib.crr_replay.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.crr_replay.restype = ctypes.c_int
    dummy = ctypes.c_void_p(64)          # never dereferenced: validation fails first
    ev = abi.CEvents(*([dummy.value] * len(abi.EVENT_COLUMNS)))
    ci = abi.CInputs()
    ci.ev = ev
    for f in ("act_side", "start_side", "reset_keys", "arena", "wf"):
        setattr(ci, f, dummy.value)
    ci.n_wf, ci.stride, ci.flags = 1000, 64, abi.IN_TIERED
    # every row pointer set; no digest and no live-ID sidecar (either would fail validation for its own reason)
    co = abi.COutputs(*([dummy.value] * (len(abi.COutputs._fields_) - 2)))
    for bnd in ((100, 1000, 1000, 1000, 1000), (128, 130, 1000, 1000, 1000), (3, 3, 3, 3, 3), (128, 128, 192, 200, 1000),
                (128, 128, 192, 256, 300)):
        ci.large_begin, ci.compact_begin, ci.compact2_begin, ci.wide_begin, ci.hbm_begin = bnd
        assert lib.crr_replay(ctypes.byref(ci), ctypes.byref(co), None) == -1, bnd
    ci.stride = 1                        # tier segments are a stride-64 layout only
    ci.large_begin = ci.compact_begin = ci.compact2_begin = ci.wide_begin = ci.hbm_begin = 1000
    assert lib.crr_replay(ctypes.byref(ci), ctypes.byref(co), None) == -1


HOST_LIB = os.path.join(ROOT, "cadence_amd", "libcadence_host.so")


@pytest.mark.skipif(not os.path.exists(HOST_LIB), reason="host library not built")
def test_host_library_exports_every_decode_symbol():
    txt = open(os.path.join(ROOT, "include", "cadence_decode.h")).read()
    syms = sorted(set(re.findall(r"^\w[\w\s\*]*?\b(crr_\w+)\s*\(", txt, re.M)))
    assert {"crr_decode_histories", "crr_decoded_get_view", "crr_decoded_free"} <= set(syms)
    lib = ctypes.CDLL(HOST_LIB)
    for s in syms:
        assert hasattr(lib, s), s


def test_interleave_tier_segments():
    """CRR_IN_TIERED layout: lane workflows ordered by expected tier (1 / 2 / more entries per
    map), longest first within a tier; segment boundaries on group boundaries (a mixed group is
    given the larger tier); the wave tail stays longest first."""
    from cadence_amd.flatten import tier_classes
    hs = synth_mixed.mixed_histories(1000, 33, mean_len=50)
    b = flatten(hs)
    cls = tier_classes(b)
    assert len(np.unique(cls)) >= 4
    ib = interleave(b, long_threshold=70)
    *bnd, bb = ib.tiers
    nl = ib.wave_begin
    c = cls[ib.perm[:nl]]
    assert (np.diff(c) >= 0).all()
    assert all(b % 64 == 0 or b == nl for b in bnd) and list(bnd) == sorted(bnd) and bnd[-1] <= nl
    for k, b in enumerate(bnd):      # segment k holds classes <= k (a mixed group takes the larger tier)
        assert (c[:b] <= k).all()
    assert ib.c_flags() & abi.IN_TIERED
    cnt = ib.wf["ev_count"]
    assert nl <= bb <= ib.n_wf
    assert (np.diff(cnt[nl:bb]) <= 0).all() and (np.diff(cnt[bb:]) <= 0).all()
    for k in range(6):
        seg = cnt[:nl][c == k]
        assert (np.diff(seg) <= 0).all()
    # one tier only: no segments beyond the lanes
    ic = interleave(synth.activity_chain(1000, 2, 3))
    assert ic.tiers == (ic.n_wf,) * 6
