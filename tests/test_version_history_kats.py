"""common/persistence/versionHistory_test.go:52-680 restated on the oracle's VersionHistory functions
(oracle/ndc_ref.cpp, the same restatement crr_ndc_prepare is checked against; AddOrUpdateItem is
also the replay loop's, oracle/state_builder_ref.cpp).  FindLCAItem / FindLCAVersionHistoryIndexAndItem
/ DuplicateUntilLCAItem success / AddVersionHistory are in tests/test_ndc.py, AddOrUpdateItem in
tests/test_oracle_kats.py.  Conversion / Equals / SetBranchToken (:52-66, :145-154, :502-541) test
thrift<->internal struct copies and byte-slice equality that have no counterpart here: the engine
never converts the structs, and the branch token enters only the checksum payload (pinned by the
archival token KAT)."""
import pytest

from cadence_amd.abi import Status
from oracle import oracle as O

ITEMS = [(3, 0), (6, 4)]


@pytest.mark.parametrize("lca", [(4, 0), (2, 1), (5, 3), (7, 5), (7, 4)])
def test_duplicate_until_lca_item_failure(lca):   # :117-143 -> BadRequestError
    r, _ = O.vh_query(O.VH_DUPLICATE_UNTIL_LCA, ITEMS, *lca)
    assert r == Status.NDC_LCA_NOT_IN_BRANCH


@pytest.mark.parametrize("lca,want", [((2, 0), [(2, 0)]), ((3, 0), [(3, 0)]), ((4, 4), [(3, 0), (4, 4)]),
                                      ((6, 4), [(3, 0), (6, 4)])])
def test_duplicate_until_lca_item_success(lca, want):   # :68-115
    assert O.vh_query(O.VH_DUPLICATE_UNTIL_LCA, ITEMS, *lca) == (0, want)


def test_contains_item_true():   # :251-266: every (event, version) of each run
    prev = 0
    for e, v in ITEMS:
        for eid in range(prev + 1, e + 1):
            assert O.vh_query(O.VH_CONTAINS, ITEMS, eid, v)[0] == 1
        prev = e


@pytest.mark.parametrize("item", [(4, 0), (3, 1), (7, 4), (6, 5)])
def test_contains_item_false(item):   # :268-281
    assert O.vh_query(O.VH_CONTAINS, ITEMS, *item)[0] == 0


def test_is_lca_appendable():   # :283-317
    assert O.vh_query(O.VH_IS_LCA_APPENDABLE, ITEMS, 6, 4)[0] == 1      # _True
    assert O.vh_query(O.VH_IS_LCA_APPENDABLE, ITEMS, 6, 7)[0] == 0      # _False_VersionNotMatch
    assert O.vh_query(O.VH_IS_LCA_APPENDABLE, ITEMS, 7, 4)[0] == 0      # _False_EventIDNotMatch


def test_get_first_item():   # :386-417
    assert O.vh_query(O.VH_FIRST, [(3, 0)]) == (0, [(3, 0)])
    st, items = O.vh_query(O.VH_ADD_OR_UPDATE, [(3, 0)], 4, 0)
    assert st == 0 and O.vh_query(O.VH_FIRST, items) == (0, [(4, 0)])   # same version: the run is extended
    st, items = O.vh_query(O.VH_ADD_OR_UPDATE, items, 7, 1)
    assert st == 0 and O.vh_query(O.VH_FIRST, items) == (0, [(4, 0)])
    assert O.vh_query(O.VH_FIRST, [])[0] == Status.VH_EMPTY                 # _Failure: BadRequestError


def test_get_last_item():   # :419-451
    assert O.vh_query(O.VH_LAST, [(3, 0)]) == (0, [(3, 0)])
    st, items = O.vh_query(O.VH_ADD_OR_UPDATE, [(3, 0)], 4, 0)
    assert O.vh_query(O.VH_LAST, items) == (0, [(4, 0)])
    st, items = O.vh_query(O.VH_ADD_OR_UPDATE, items, 7, 1)
    assert O.vh_query(O.VH_LAST, items) == (0, [(7, 1)])
    assert O.vh_query(O.VH_LAST, [])[0] == Status.VH_EMPTY                  # _Failure


def test_get_event_version():   # :453-500
    items = [(3, 0), (6, 8), (8, 12)]
    for eid, v in ((1, 0), (2, 0), (3, 0), (4, 8), (5, 8), (6, 8), (7, 12), (8, 12)):
        assert O.vh_query(O.VH_EVENT_VERSION, items, eid) == (0, [(eid, v)])
    assert O.vh_query(O.VH_EVENT_VERSION, items, 0)[0] != 0                # _Failure
    assert O.vh_query(O.VH_EVENT_VERSION, items, 9)[0] != 0


def test_find_first_version_history_index_by_item():   # :636-663 (first branch that ContainsItem)
    h1 = [(3, 0), (5, 4), (7, 6)]
    h2 = [(3, 0), (5, 4), (7, 6), (9, 10)]

    def first(item):
        for i, h in enumerate((h1, h2)):
            if O.vh_query(O.VH_CONTAINS, h, *item)[0]:
                return i
        return None
    assert first((8, 10)) == 1 and first((4, 4)) == 0 and first((41, 4)) is None
