"""NDC branch decisions: prepareVersionHistory over a batch of replication tasks.

CPU: the oracle restatement pinned to the reference's own expectations (versionHistory_test.go,
branch_manager_test.go).  GPU: crr_ndc_prepare against the oracle on random version histories, every
result field and the new branch's items bit-exact.
"""
import dataclasses
import random

import numpy as np
import pytest

from cadence_amd import abi
from cadence_amd.abi import Status
from cadence_amd.ndc import NdcTask, new_branch_items, pack, prepare_on_device
from oracle import oracle

VH1 = [(3, 0), (5, 4), (7, 6), (9, 10)]


def run(tasks):
    b = pack(tasks)
    res, out = oracle.ndc_prepare(b)
    return b, res, out


def one(task):
    b, res, out = run([task])
    return res[0], new_branch_items(b, res, out, 0)


def test_find_lca_item_return_local():  # versionHistory_test.go:319-340
    r, _ = one(NdcTask([VH1], 0, [(3, 0), (7, 4), (8, 8), (11, 12)], 12, 12))
    assert (r["lca_event_id"], r["lca_version"]) == (5, 4)


def test_find_lca_item_return_remote():  # :342-363
    r, _ = one(NdcTask([VH1], 0, [(3, 0), (5, 4), (6, 6), (11, 12)], 12, 12))
    assert (r["lca_event_id"], r["lca_version"]) == (6, 6)


def test_find_lca_item_no_lca():  # :365-384
    r, _ = one(NdcTask([VH1], 0, [(3, 1), (7, 2), (8, 3)], 9, 3))
    assert r["status"] == Status.NDC_NO_LCA


def test_lca_index_larger_event_id_wins():  # :575-604
    vh2 = [(3, 0), (5, 4), (6, 6), (11, 12)]
    r, _ = one(NdcTask([VH1, vh2], 1, [(3, 0), (5, 4), (8, 6), (11, 100)], 12, 100))
    assert r["lca_branch"] == 0 and (r["lca_event_id"], r["lca_version"]) == (7, 6)


def test_lca_index_same_event_id_shorter_wins():  # :606-634
    vh2 = [(3, 0), (5, 4), (7, 6)]
    r, _ = one(NdcTask([VH1, vh2], 0, [(3, 0), (5, 4), (8, 6), (11, 100)], 12, 100))
    assert r["lca_branch"] == 1 and (r["lca_event_id"], r["lca_version"]) == (7, 6)


@pytest.mark.parametrize("incoming,first,want_items,action", [  # DuplicateUntilLCAItem_Success :68-115
    ([(2, 0), (10, 7)], 3, [(2, 0)], abi.NDC_NEW_BRANCH),
    ([(3, 0), (5, 4), (9, 7)], 6, [(3, 0), (5, 4)], abi.NDC_NEW_BRANCH),
    ([(3, 0), (6, 4), (9, 7)], 7, [], abi.NDC_APPEND),
])
def test_duplicate_until_lca(incoming, first, want_items, action):
    r, items = one(NdcTask([[(3, 0), (6, 4)]], 0, incoming, first, 7))
    assert r["status"] == 0 and r["action"] == action
    assert items == want_items


def test_add_version_history_switches_current():  # AddVersionHistory :450-498, TestAddGetVersionHistory :543-573
    a = [(3, 0), (5, 4)]
    b = [(3, 0), (5, 4), (9, 10)]
    r, items = one(NdcTask([a, b], 0, [(3, 0), (5, 4), (8, 10), (12, 20)], 9, 20))
    assert r["status"] == 0 and r["action"] == abi.NDC_NEW_BRANCH
    assert r["branch_index"] == 2 and r["branch_changed"] == 1 and r["new_current_index"] == 2
    assert r["lca_branch"] == 1 and items == [(3, 0), (5, 4), (8, 10)]
    assert r["is_rebuilt"] == 1          # IsRebuilt :545-571: branch 1 is newer than the current one


BASE = [(10, 0), (50, 100), (100, 200), (150, 300)]


def test_prepare_appendable_no_missing_event():  # branch_manager_test.go:218-245
    r, _ = one(NdcTask([BASE], 0, BASE[:3] + [(200, 300)], 151, 300))
    assert r["status"] == 0 and r["action"] == abi.NDC_APPEND and r["branch_index"] == 0


def test_prepare_appendable_missing_event():  # :247-279 (RetryTaskV2Error)
    r, _ = one(NdcTask([BASE], 0, BASE[:3] + [(200, 300)], 152, 300))
    assert r["status"] == Status.NDC_RETRY_TASK
    assert (r["last_event_id"], r["last_version"]) == (150, 300)


def test_prepare_not_appendable_no_missing_event():  # :281-333 (fork at LCA 85 + 1, new index 1)
    local = [(10, 0), (50, 100), (95, 200), (150, 300)]
    r, items = one(NdcTask([local], 0, [(10, 0), (50, 100), (85, 200), (200, 400)], 86, 200))
    assert r["status"] == 0 and r["action"] == abi.NDC_NEW_BRANCH and r["branch_index"] == 1
    assert r["lca_branch"] == 0 and r["lca_event_id"] + 1 == 86       # ForkNodeID
    assert items == [(10, 0), (50, 100), (85, 200)]


def test_prepare_not_appendable_missing_event():  # :335-372
    local = [(10, 0), (50, 100), (95, 200), (150, 300)]
    r, _ = one(NdcTask([local], 0, [(10, 0), (50, 100), (85, 200), (200, 400)], 87, 200))
    assert r["status"] == Status.NDC_RETRY_TASK


def test_duplicate_task():  # verifyEventsOrder: incomingFirstEventID < nextEventID
    r, _ = one(NdcTask([BASE], 0, BASE[:3] + [(200, 300)], 120, 300))
    assert r["status"] == 0 and r["action"] == abi.NDC_DUPLICATE and r["branch_index"] == 0


def random_tasks(n, seed):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        # a chain of (event id, version) runs; branches diverge from it at random points
        chain, eid, ver = [], 0, rng.randint(0, 3)
        for _ in range(rng.randint(1, 6)):
            eid += rng.randint(1, 30)
            ver += rng.randint(1, 50)
            chain.append((eid, ver))

        def branch_from(ch):
            k = rng.randint(1, len(ch))
            b = [list(x) for x in ch[:k]]
            if rng.random() < 0.5:
                b[-1][0] = max(b[-2][0] + 1 if len(b) > 1 else 1, b[-1][0] - rng.randint(0, 5))
            e, v = b[-1]
            for _ in range(rng.randint(0, 3)):
                e += rng.randint(1, 20)
                v += rng.randint(1, 40)
                b.append([e, v])
            return [tuple(x) for x in b]

        local = [branch_from(chain) for _ in range(rng.randint(1, 4))]
        if rng.random() < 0.05:
            local.append([])                                         # empty branch
        incoming = branch_from(chain) if rng.random() < 0.9 else [(rng.randint(1, 9), 999)]
        if rng.random() < 0.03:
            incoming = [(5, 3), (4, 7)]                              # malformed
        last_e = incoming[-1][0] if incoming else 0
        first = last_e - rng.choice([0, 0, 1, 2, 3, 10]) + rng.choice([0, 1])
        cur = rng.randrange(len(local)) if rng.random() < 0.97 else len(local) + 1
        out.append(NdcTask(local, cur, incoming, first, incoming[-1][1] if incoming else 0))
    return out


def test_random_tasks_cover_every_outcome():
    b, res, _ = run(random_tasks(3000, 7))
    st = set(int(s) for s in res["status"])
    assert {0, Status.NDC_NO_LCA, Status.NDC_RETRY_TASK}.issubset(st)
    acts = set(int(a) for a, s in zip(res["action"], res["status"]) if s == 0)
    assert acts == {abi.NDC_APPEND, abi.NDC_NEW_BRANCH, abi.NDC_DUPLICATE}


@pytest.mark.gpu
def test_device_matches_oracle_on_random_tasks():
    from cadence_amd.engine import ReplayEngine
    eng = ReplayEngine(0)
    b = pack(random_tasks(20000, 11))
    want, want_out = oracle.ndc_prepare(b)
    got, got_out = prepare_on_device(eng, b)
    for f in abi.NDC_RESULT.names:
        bad = np.nonzero(got[f] != want[f])[0]
        assert bad.size == 0, f"{f}: {bad.size} tasks differ, first {bad[:1]}: {got[f][bad[:1]]} vs {want[f][bad[:1]]}"
    for k in range(len(b.tasks)):
        assert new_branch_items(b, got, got_out, k) == new_branch_items(b, want, want_out, k)


def _check_device(eng, b):
    want, want_out = oracle.ndc_prepare(b)
    got, got_out = prepare_on_device(eng, b)
    for f in abi.NDC_RESULT.names:
        bad = np.nonzero(got[f] != want[f])[0]
        assert bad.size == 0, f"{f}: {bad.size} tasks differ, first {bad[:1]}: {got[f][bad[:1]]} vs {want[f][bad[:1]]}"
    for k in range(len(b.tasks)):
        assert new_branch_items(b, got, got_out, k) == new_branch_items(b, want, want_out, k)
    return got


def test_empty_version_histories_are_invalid():
    r, _ = one(NdcTask([], 0, [(10, 0)], 11, 0))
    assert r["status"] == Status.NDC_BAD_INDEX and r["action"] == abi.NDC_DUPLICATE


@pytest.mark.gpu
def test_device_staged_and_unstaged_layouts():
    """The kernel stages each wavefront's span of branch descriptors and items in LDS when it fits
    (ndc.pack's contiguous layout) and reads HBM otherwise: tasks shuffled in memory (every wavefront's
    span is the whole batch), long version histories (spans past the stage), and tasks without any
    branch (invalid) give the oracle's results either way."""
    from cadence_amd.engine import ReplayEngine
    eng = ReplayEngine(0)
    tasks = random_tasks(6000, 21)
    tasks[5] = NdcTask([], 0, [(10, 0)], 11, 0)
    b = pack(tasks)
    _check_device(eng, b)
    perm = np.random.default_rng(3).permutation(len(b.tasks))
    _check_device(eng, dataclasses.replace(b, tasks=b.tasks[perm].copy()))
    longh = []
    for t in random_tasks(640, 22):   # every task's histories stretched to ~40 items: 64 tasks >> 768 items
        ext = lambda br: [(e + 1000 * i, v + 10000 * i) for i in range(8) for (e, v) in br][:40] if br else br  # noqa: E731
        longh.append(NdcTask([ext(x) for x in t.local], t.current_index, ext(t.incoming), t.first_event_id + 7000,
                             t.first_event_version))
    _check_device(eng, pack(longh))
