// ndc_kernel.hip -- batched NDC branch decisions (crr_ndc_prepare, include/cadence_replay.h).
//
// One lane per replication task.  A task's version histories are a handful of (event ID, version)
// items per branch, so every step is a short scan over HBM-resident items (L2-cached after the first
// touch); the result row and the new branch's items are the only writes.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cadence_replay.h"
#include "stream_device.h"

namespace {

using i64 = int64_t;
using i32 = int32_t;
using u32 = uint32_t;

constexpr int kBlock = 256;

struct Item {
  i64 e, v;
};
__device__ __forceinline__ Item item(const crr_vh_item* it, u32 i) { return Item{it[i].event_id, it[i].version}; }

// VersionHistory.FindLCAItem (versionHistory.go:248-273): walk both histories from the back
__device__ bool find_lca(const crr_vh_item* items, crr_ndc_branch local, u32 in_begin, u32 in_count, Item* out) {
  i32 li = (i32)local.item_count - 1, ri = (i32)in_count - 1;
  while (li >= 0 && ri >= 0) {
    const Item l = item(items, local.item_begin + li), r = item(items, in_begin + ri);
    if (l.v == r.v) {
      *out = l.e > r.e ? r : l;
      return true;
    }
    if (l.v > r.v) --li;
    else --ri;
  }
  return false;
}

__global__ void __launch_bounds__(kBlock) ndc_prepare_kernel(crr_ndc_inputs in, crr_ndc_result* res, crr_vh_item* out_items) {
  const u32 k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= in.n_tasks) return;
  const crr_ndc_task t = in.tasks[k];
  crr_ndc_result r;
  r.status = CRR_OK; r.action = CRR_NDC_DUPLICATE; r.branch_index = 0; r.lca_branch = 0;
  r.lca_event_id = 0; r.lca_version = 0; r.last_event_id = 0; r.last_version = 0;
  r.new_current_index = t.current_index; r.new_item_count = 0; r.is_rebuilt = 0; r.branch_changed = 0;

  // IsRebuilt (:545-571), reported beside the decision (-1: it would fail -- bad index or empty branch)
  const bool cur_ok = t.current_index >= 0 && (u32)t.current_index < t.branch_count &&
                      in.branches[t.branch_begin + t.current_index].item_count > 0;
  Item cur_last{0, 0};
  if (cur_ok) {
    const crr_ndc_branch cur = in.branches[t.branch_begin + t.current_index];
    cur_last = item(in.items, cur.item_begin + cur.item_count - 1);
    for (u32 b = 0; b < t.branch_count && r.is_rebuilt == 0; ++b) {  // first newer branch: true
      const crr_ndc_branch br = in.branches[t.branch_begin + b];
      if (br.item_count == 0) r.is_rebuilt = -1;
      else if (item(in.items, br.item_begin + br.item_count - 1).v > cur_last.v) r.is_rebuilt = 1;
    }
  } else {
    r.is_rebuilt = -1;
  }

  // FindLCAVersionHistoryIndexAndItem (:501-528): larger LCA event ID wins, ties to the shorter branch
  i32 idx = 0;
  u32 idx_len = 0;
  Item lca{0, 0};
  bool have = false;
  for (u32 b = 0; b < t.branch_count; ++b) {
    const crr_ndc_branch br = in.branches[t.branch_begin + b];
    Item it;
    if (!find_lca(in.items, br, t.incoming_begin, t.incoming_count, &it)) {
      r.status = CRR_ERR_NDC_NO_LCA;
      res[k] = r;
      return;
    }
    if (!have || it.e > lca.e || (it.e == lca.e && br.item_count < idx_len)) {
      idx = (i32)b; idx_len = br.item_count; lca = it; have = true;
    }
  }
  r.lca_branch = idx;
  r.lca_event_id = lca.e;
  r.lca_version = lca.v;
  const crr_ndc_branch base = in.branches[t.branch_begin + idx];
  const Item base_last = item(in.items, base.item_begin + base.item_count - 1);

  Item last;  // the last item of the branch the batch would extend
  if (base_last.e == lca.e && base_last.v == lca.v) {  // IsLCAAppendable (:275-287)
    last = base_last;
    r.branch_index = idx;
    r.action = CRR_NDC_APPEND;
  } else {
    // DuplicateUntilLCAItem (:142-172) into out_items[out_begin...], every item through
    // AddOrUpdateItem (:193-226) and its ordering errors
    u32 n = 0;
    int st = CRR_ERR_NDC_LCA_NOT_IN_BRANCH;
    Item tail{0, 0};
    auto add = [&](Item it) -> int {
      if (n > 0) {
        if (it.v < tail.v) return CRR_ERR_VH_LOWER_VERSION;
        if (it.e <= tail.e) return CRR_ERR_VH_EVENT_ID_NOT_INCREASING;
        if (it.v == tail.v) {  // same version: extend the last item
          tail.e = it.e;
          out_items[t.out_begin + n - 1].event_id = it.e;
          return CRR_OK;
        }
      }
      out_items[t.out_begin + n].event_id = it.e;
      out_items[t.out_begin + n].version = it.v;
      tail = it;
      ++n;
      return CRR_OK;
    };
    for (u32 i = 0; i < base.item_count; ++i) {
      const Item it = item(in.items, base.item_begin + i);
      if (it.v < lca.v) {
        const int e = add(it);
        if (e != CRR_OK) { st = e; break; }
      } else {
        if (it.v == lca.v && lca.e <= it.e) st = add(lca);
        break;
      }
    }
    if (st != CRR_OK) {
      r.status = st;
      r.new_item_count = 0;
      res[k] = r;
      return;
    }
    r.new_item_count = (i32)n;
    last = lca;
    r.branch_index = (i32)t.branch_count;  // AddVersionHistory appends: new index = len(Histories)
    r.action = CRR_NDC_NEW_BRANCH;
  }
  r.last_event_id = last.e;
  r.last_version = last.v;
  // verifyEventsOrder (branch_manager.go:199-225)
  const i64 next_event_id = last.e + 1;
  if (t.first_event_id < next_event_id) {  // duplicate task: (false, index, nil) appending, (false, 0, nil) forking
    if (r.action == CRR_NDC_NEW_BRANCH) r.branch_index = 0;
    r.action = CRR_NDC_DUPLICATE;
    r.new_item_count = 0;
  } else if (t.first_event_id > next_event_id) {
    r.status = CRR_ERR_NDC_RETRY_TASK;  // RetryTaskV2Error with the (last_event_id, last_version) hint
  } else if (r.action == CRR_NDC_NEW_BRANCH) {
    // AddVersionHistory (:450-498): first items must share a version; switch if the new branch is newer
    if (!(t.current_index >= 0 && (u32)t.current_index < t.branch_count)) {
      r.status = CRR_ERR_NDC_BAD_INDEX;
    } else {
      const crr_ndc_branch cur = in.branches[t.branch_begin + t.current_index];
      const Item new_first = item(out_items, t.out_begin);
      if (cur.item_count == 0) {
        r.status = CRR_ERR_VH_EMPTY;
      } else if (new_first.v != item(in.items, cur.item_begin).v) {
        r.status = CRR_ERR_NDC_FIRST_ITEM_MISMATCH;
      } else if (lca.v > item(in.items, cur.item_begin + cur.item_count - 1).v) {
        r.branch_changed = 1;
        r.new_current_index = (i32)t.branch_count;
      }
    }
  }
  if (r.status != CRR_OK) {  // prepareVersionHistory returns (false, 0, err)
    r.action = CRR_NDC_DUPLICATE;
    r.branch_index = 0;
    r.new_item_count = 0;
    r.branch_changed = 0;
    r.new_current_index = t.current_index;
  }
  res[k] = r;
}

}  // namespace

extern "C" int crr_ndc_prepare(const crr_ndc_inputs* in, crr_ndc_result* results, crr_vh_item* out_items, void* stream) {
  if (!in || (in->n_tasks && (!in->tasks || !in->branches || !in->items || !results || !out_items))) return -1;
  if (in->n_tasks == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  crr_internal::StreamDevice on_dev_(s);
  if (!on_dev_.ok) return (int)hipErrorInvalidHandle;
  hipLaunchKernelGGL(ndc_prepare_kernel, dim3((in->n_tasks + kBlock - 1) / kBlock), dim3(kBlock), 0, s, *in, results,
                     out_items);
  return (int)hipGetLastError();
}
