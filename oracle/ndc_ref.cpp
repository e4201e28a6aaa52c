// oracle/ndc_ref.cpp -- TEST INFRASTRUCTURE ONLY: CPU restatement of the NDC branch decision.
//
// Follows, with Go-shaped data structures (slices of items, one VersionHistories per task):
//   common/persistence/versionHistory.go  AddOrUpdateItem (:193-226), DuplicateUntilLCAItem (:142-172),
//     FindLCAItem (:248-273), IsLCAAppendable (:275-287), GetFirstItem / GetLastItem (:290-313),
//     AddVersionHistory (:450-498), FindLCAVersionHistoryIndexAndItem (:501-528), IsRebuilt (:545-571)
//   service/history/ndc/branch_manager.go  prepareVersionHistory (:87-149) without the buffered-event
//     flush, verifyEventsOrder (:199-225), createNewBranch (:227-265) up to ForkHistoryBranch
// Pinned by the reference's versionHistory_test.go and branch_manager_test.go expectations
// (tests/test_ndc.py).  Only tests/ load it (through liboracle.so).
#include <cstdint>
#include <vector>

#include "cadence_replay.h"

namespace {

using i64 = int64_t;

struct Item {
  i64 event_id, version;
  bool operator==(const Item& o) const { return event_id == o.event_id && version == o.version; }
};

struct VH {
  std::vector<Item> items;
  int add_or_update(Item it) {  // :193-226
    if (items.empty()) { items.push_back(it); return CRR_OK; }
    Item& last = items.back();
    if (it.version < last.version) return CRR_ERR_VH_LOWER_VERSION;
    if (it.event_id <= last.event_id) return CRR_ERR_VH_EVENT_ID_NOT_INCREASING;
    if (it.version > last.version) items.push_back(it);
    else last.event_id = it.event_id;
    return CRR_OK;
  }
  int last_item(Item* out) const {
    if (items.empty()) return CRR_ERR_VH_EMPTY;
    *out = items.back();
    return CRR_OK;
  }
  int first_item(Item* out) const {
    if (items.empty()) return CRR_ERR_VH_EMPTY;
    *out = items.front();
    return CRR_OK;
  }
  // ContainsItem (:228-245)
  bool contains(const Item& it) const {
    i64 prev = CRR_FIRST_EVENT_ID - 1;
    for (const Item& c : items) {
      if (it.version == c.version) {
        if (prev < it.event_id && it.event_id <= c.event_id) return true;
      } else if (it.version < c.version) {
        return false;
      }
      prev = c.event_id;
    }
    return false;
  }
  // GetEventVersion (:313-335)
  int event_version(i64 event_id, i64* out) const {
    Item last;
    int e = last_item(&last);
    if (e) return e;
    if (event_id < CRR_FIRST_EVENT_ID || event_id > last.event_id) return CRR_ERR_NDC_BAD_INDEX;
    for (const Item& c : items)
      if (event_id <= c.event_id) { *out = c.version; return CRR_OK; }
    return CRR_ERR_NDC_BAD_INDEX;
  }
  int duplicate_until_lca(const Item& lca, VH* out) const {  // :142-172
    VH v;
    for (const Item& it : items) {
      if (it.version < lca.version) {
        int e = v.add_or_update(it);
        if (e) return e;
      } else if (it.version == lca.version) {
        if (lca.event_id > it.event_id) return CRR_ERR_NDC_LCA_NOT_IN_BRANCH;
        int e = v.add_or_update(lca);
        if (e) return e;
        *out = v;
        return CRR_OK;
      } else {
        return CRR_ERR_NDC_LCA_NOT_IN_BRANCH;
      }
    }
    return CRR_ERR_NDC_LCA_NOT_IN_BRANCH;
  }
  int find_lca(const VH& remote, Item* out) const {  // :248-273
    int li = (int)items.size() - 1, ri = (int)remote.items.size() - 1;
    while (li >= 0 && ri >= 0) {
      const Item& l = items[li];
      const Item& r = remote.items[ri];
      if (l.version == r.version) {
        *out = l.event_id > r.event_id ? r : l;
        return CRR_OK;
      } else if (l.version > r.version) {
        --li;
      } else {
        --ri;
      }
    }
    return CRR_ERR_NDC_NO_LCA;
  }
};

struct VHs {
  std::vector<VH> histories;
  int current = 0;
  int find_lca_index_and_item(const VH& incoming, int* index, Item* lca) const {  // :501-528
    int vidx = 0;
    size_t vlen = 0;
    bool have = false;
    Item vitem{0, 0};
    for (size_t i = 0; i < histories.size(); ++i) {
      Item it;
      int e = histories[i].find_lca(incoming, &it);
      if (e) return e;
      if (!have || it.event_id > vitem.event_id || (it.event_id == vitem.event_id && histories[i].items.size() < vlen)) {
        vidx = (int)i;
        vlen = histories[i].items.size();
        vitem = it;
        have = true;
      }
    }
    *index = vidx;
    *lca = vitem;
    return CRR_OK;
  }
  int add(const VH& v, bool* changed, int* new_index) {  // :450-498
    Item in_first;
    int e = v.first_item(&in_first);
    if (e) return e;
    if (current < 0 || current >= (int)histories.size()) return CRR_ERR_NDC_BAD_INDEX;
    Item cur_first;
    e = histories[current].first_item(&cur_first);
    if (e) return e;
    if (in_first.version != cur_first.version) return CRR_ERR_NDC_FIRST_ITEM_MISMATCH;
    histories.push_back(v);
    *new_index = (int)histories.size() - 1;
    Item new_last, cur_last;
    e = histories.back().last_item(&new_last);
    if (e) return e;
    e = histories[current].last_item(&cur_last);
    if (e) return e;
    *changed = false;
    if (new_last.version > cur_last.version) {
      *changed = true;
      current = *new_index;
    }
    return CRR_OK;
  }
  int is_rebuilt(bool* out) const {  // :545-571
    if (current < 0 || current >= (int)histories.size()) return CRR_ERR_NDC_BAD_INDEX;
    Item cur_last;
    int e = histories[current].last_item(&cur_last);
    if (e) return e;
    for (const VH& h : histories) {
      Item l;
      e = h.last_item(&l);
      if (e) return e;
      if (l.version > cur_last.version) { *out = true; return CRR_OK; }
    }
    *out = false;
    return CRR_OK;
  }
};

// verifyEventsOrder (branch_manager.go:199-225): doContinue / duplicate / RetryTaskV2Error
int verify_events_order(const VH& local, i64 first_id, bool* do_continue, Item* last) {
  int e = local.last_item(last);
  if (e) return e;
  const i64 next = last->event_id + 1;
  if (first_id < next) { *do_continue = false; return CRR_OK; }
  if (first_id > next) return CRR_ERR_NDC_RETRY_TASK;
  *do_continue = true;
  return CRR_OK;
}

}  // namespace

// Single VersionHistory queries over caller items (restating versionHistory_test.go's unit cases):
//   op 1 DuplicateUntilLCAItem(a, b) -> status, items in out; op 2 IsLCAAppendable(a, b) -> 0/1;
//   op 3 GetFirstItem, op 4 GetLastItem -> status, item in out[0]; op 5 ContainsItem(a, b) -> 0/1;
//   op 6 GetEventVersion(a) -> status, version in out[0].version; op 7 AddOrUpdateItem(a, b) -> status, items.
// Returns the status (or the boolean), *n_out the items written to out.
extern "C" int oracle_vh_query(int op, const crr_vh_item* items, int n, int64_t a, int64_t b, crr_vh_item* out,
                               int* n_out) {
  VH v;
  for (int i = 0; i < n; ++i) v.items.push_back({items[i].event_id, items[i].version});
  *n_out = 0;
  Item it{a, b}, r{0, 0};
  switch (op) {
    case 1: {
      VH d;
      int e = v.duplicate_until_lca(it, &d);
      if (e) return e;
      for (const Item& x : d.items) out[(*n_out)++] = {x.event_id, x.version};
      return CRR_OK;
    }
    case 2: return !v.items.empty() && v.items.back() == it;  // IsLCAAppendable (:278-290)
    case 3: case 4: {
      int e = op == 3 ? v.first_item(&r) : v.last_item(&r);
      if (!e) { out[0] = {r.event_id, r.version}; *n_out = 1; }
      return e;
    }
    case 5: return v.contains(it);
    case 6: {
      i64 ver = 0;
      int e = v.event_version(a, &ver);
      if (!e) { out[0] = {a, ver}; *n_out = 1; }
      return e;
    }
    case 7: {
      if (a < 0 || (b < 0 && b != CRR_EMPTY_VERSION)) return CRR_ERR_VH_INVALID_ITEM;  // NewVersionHistoryItem
      int e = v.add_or_update(it);
      if (e) return e;
      for (const Item& x : v.items) out[(*n_out)++] = {x.event_id, x.version};
      return CRR_OK;
    }
    default: return -1;
  }
}

extern "C" int oracle_ndc_prepare(const crr_ndc_inputs* in, crr_ndc_result* results, crr_vh_item* out_items) {
  for (uint32_t k = 0; k < in->n_tasks; ++k) {
    const crr_ndc_task& t = in->tasks[k];
    VHs local;
    for (uint32_t b = 0; b < t.branch_count; ++b) {
      const crr_ndc_branch& br = in->branches[t.branch_begin + b];
      VH v;
      for (uint32_t i = 0; i < br.item_count; ++i)
        v.items.push_back(Item{in->items[br.item_begin + i].event_id, in->items[br.item_begin + i].version});
      local.histories.push_back(v);
    }
    local.current = t.current_index;
    VH incoming;
    for (uint32_t i = 0; i < t.incoming_count; ++i)
      incoming.items.push_back(Item{in->items[t.incoming_begin + i].event_id, in->items[t.incoming_begin + i].version});

    crr_ndc_result r{};
    r.status = CRR_OK;
    r.action = CRR_NDC_DUPLICATE;
    r.new_current_index = t.current_index;
    bool rebuilt = false;
    r.is_rebuilt = local.is_rebuilt(&rebuilt) == CRR_OK ? (rebuilt ? 1 : 0) : -1;

    auto finish = [&](int status) {
      r.status = status;
      if (status != CRR_OK) {
        r.action = CRR_NDC_DUPLICATE;
        r.branch_index = 0;
        r.new_item_count = 0;
        r.branch_changed = 0;
        r.new_current_index = t.current_index;
      }
      results[k] = r;
    };
    // prepareVersionHistory (branch_manager.go:87-149); a VersionHistories always holds a branch
    // (NewVersionHistories), so an empty one is invalid input
    if (t.branch_count == 0) { finish(CRR_ERR_NDC_BAD_INDEX); continue; }
    int idx = 0;
    Item lca{0, 0};
    int e = local.find_lca_index_and_item(incoming, &idx, &lca);
    if (e) { finish(e); continue; }
    r.lca_branch = idx;
    r.lca_event_id = lca.event_id;
    r.lca_version = lca.version;
    const VH& base = local.histories[idx];
    Item last{0, 0};
    bool cont = false;
    if (!base.items.empty() && base.items.back() == lca) {  // IsLCAAppendable
      e = verify_events_order(base, t.first_event_id, &cont, &last);
      r.last_event_id = last.event_id;
      r.last_version = last.version;
      if (e) { finish(e); continue; }
      r.action = cont ? CRR_NDC_APPEND : CRR_NDC_DUPLICATE;
      r.branch_index = idx;  // (doContinue, versionHistoryIndex, nil)
      finish(CRR_OK);
      continue;
    }
    VH nv;
    e = base.duplicate_until_lca(lca, &nv);
    if (e) { finish(e); continue; }
    e = verify_events_order(nv, t.first_event_id, &cont, &last);
    r.last_event_id = last.event_id;
    r.last_version = last.version;
    if (e) { finish(e); continue; }
    if (!cont) { r.action = CRR_NDC_DUPLICATE; r.branch_index = 0; finish(CRR_OK); continue; }
    // createNewBranch: ForkHistoryBranch (host) then AddVersionHistory
    bool changed = false;
    int new_index = 0;
    e = local.add(nv, &changed, &new_index);
    if (e) { finish(e); continue; }
    r.action = CRR_NDC_NEW_BRANCH;
    r.branch_index = new_index;
    r.branch_changed = changed ? 1 : 0;
    r.new_current_index = local.current;
    r.new_item_count = (int32_t)nv.items.size();
    for (size_t i = 0; i < nv.items.size(); ++i) {
      out_items[t.out_begin + i].event_id = nv.items[i].event_id;
      out_items[t.out_begin + i].version = nv.items[i].version;
    }
    finish(CRR_OK);
  }
  return 0;
}
