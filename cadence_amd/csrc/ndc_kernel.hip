// ndc_kernel.hip -- batched NDC branch decisions (crr_ndc_prepare, include/cadence_replay.h).
//
// One lane per replication task, 64 consecutive tasks per wavefront.  A task's version histories are a
// handful of (event ID, version) items per branch, read again in every phase (IsRebuilt, each branch's
// LCA walk, the duplicate copy) by lanes at different positions: read per lane from HBM, each 16-B item
// pulls its own line and the lines leave the L2 between phases (round 4: 3.0x the algorithmic bytes).
// So each wavefront first stages the span of branch descriptors and the span of items its 64 tasks use
// into LDS with coalesced 16-B loads (the spans are contiguous as ndc.pack lays a batch out; any layout
// works, a wavefront whose spans exceed the stage reads HBM instead) and walks them from LDS.  The result
// row and the new branch's items are the only writes.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cadence_replay.h"
#include "stream_device.h"

namespace {

using i64 = int64_t;
using i32 = int32_t;
using u32 = uint32_t;

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
#ifndef CRR_NDC_STAGE_ITEMS
#define CRR_NDC_STAGE_ITEMS 512
#endif
#ifndef CRR_NDC_STAGE_BRANCHES
#define CRR_NDC_STAGE_BRANCHES 256
#endif
// per wavefront: 8 KB of items, 2 KB of branch descriptors (40 KB per block, 4 blocks per CU).  Measured
// on config 5's 1M tasks (tools/prof_ndc.py): 768 items 0.132 ms, 512 items 0.118 ms, unstaged 0.144 ms
constexpr u32 kStageItems = CRR_NDC_STAGE_ITEMS;
constexpr u32 kStageBranches = CRR_NDC_STAGE_BRANCHES;

struct Item {
  i64 e, v;
};
__device__ __forceinline__ Item item(const crr_vh_item* it, u32 i) { return Item{it[i].event_id, it[i].version}; }

// the items and branch descriptors from HBM, or from the wavefront's LDS stage (array index - base)
struct GlobalSrc {
  const crr_vh_item* items;
  const crr_ndc_branch* branches;
  __device__ __forceinline__ Item at(u32 i) const { return item(items, i); }
  __device__ __forceinline__ crr_ndc_branch branch(u32 b) const { return branches[b]; }
};
struct LdsSrc {
  const crr_vh_item* items;         // LDS
  const crr_ndc_branch* branches;   // LDS
  u32 ibase, bbase;
  __device__ __forceinline__ Item at(u32 i) const { return item(items, i - ibase); }
  __device__ __forceinline__ crr_ndc_branch branch(u32 b) const { return branches[b - bbase]; }
};

// VersionHistory.FindLCAItem (versionHistory.go:248-273): walk both histories from the back
template <class SRC>
__device__ bool find_lca(const SRC& src, crr_ndc_branch local, u32 in_begin, u32 in_count, Item* out) {
  i32 li = (i32)local.item_count - 1, ri = (i32)in_count - 1;
  while (li >= 0 && ri >= 0) {
    const Item l = src.at(local.item_begin + li), r = src.at(in_begin + ri);
    if (l.v == r.v) {
      *out = l.e > r.e ? r : l;
      return true;
    }
    if (l.v > r.v) --li;
    else --ri;
  }
  return false;
}

// prepareVersionHistory (branch_manager.go:87-149) for task k
template <class SRC>
__device__ __forceinline__ void prepare_task(const SRC& src, const crr_ndc_task& t, u32 k, crr_ndc_result* res,
                                             crr_vh_item* out_items) {
  crr_ndc_result r;
  r.status = CRR_OK; r.action = CRR_NDC_DUPLICATE; r.branch_index = 0; r.lca_branch = 0;
  r.lca_event_id = 0; r.lca_version = 0; r.last_event_id = 0; r.last_version = 0;
  r.new_current_index = t.current_index; r.new_item_count = 0; r.is_rebuilt = 0; r.branch_changed = 0;

  // IsRebuilt (:545-571), reported beside the decision (-1: it would fail -- bad index or empty branch)
  const bool cur_ok = t.current_index >= 0 && (u32)t.current_index < t.branch_count &&
                      src.branch(t.branch_begin + t.current_index).item_count > 0;
  Item cur_last{0, 0};
  if (cur_ok) {
    const crr_ndc_branch cur = src.branch(t.branch_begin + t.current_index);
    cur_last = src.at(cur.item_begin + cur.item_count - 1);
    for (u32 b = 0; b < t.branch_count && r.is_rebuilt == 0; ++b) {  // first newer branch: true
      const crr_ndc_branch br = src.branch(t.branch_begin + b);
      if (br.item_count == 0) r.is_rebuilt = -1;
      else if (src.at(br.item_begin + br.item_count - 1).v > cur_last.v) r.is_rebuilt = 1;
    }
  } else {
    r.is_rebuilt = -1;
  }
  if (t.branch_count == 0) {  // a VersionHistories always holds a branch (NewVersionHistories): invalid input
    r.status = CRR_ERR_NDC_BAD_INDEX;
    res[k] = r;
    return;
  }

  // FindLCAVersionHistoryIndexAndItem (:501-528): larger LCA event ID wins, ties to the shorter branch
  i32 idx = 0;
  u32 idx_len = 0;
  Item lca{0, 0};
  bool have = false;
  for (u32 b = 0; b < t.branch_count; ++b) {
    const crr_ndc_branch br = src.branch(t.branch_begin + b);
    Item it;
    if (!find_lca(src, br, t.incoming_begin, t.incoming_count, &it)) {
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
  const crr_ndc_branch base = src.branch(t.branch_begin + idx);
  const Item base_last = src.at(base.item_begin + base.item_count - 1);

  Item last;  // the last item of the branch the batch would extend
  Item new_first{0, 0};
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
          if (n == 1) new_first.e = it.e;
          return CRR_OK;
        }
      }
      out_items[t.out_begin + n].event_id = it.e;
      out_items[t.out_begin + n].version = it.v;
      if (n == 0) new_first = it;
      tail = it;
      ++n;
      return CRR_OK;
    };
    for (u32 i = 0; i < base.item_count; ++i) {
      const Item it = src.at(base.item_begin + i);
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
    // (the new branch's first item from registers: the row just written is not read back)
    if (!(t.current_index >= 0 && (u32)t.current_index < t.branch_count)) {
      r.status = CRR_ERR_NDC_BAD_INDEX;
    } else {
      const crr_ndc_branch cur = src.branch(t.branch_begin + t.current_index);
      if (cur.item_count == 0) {
        r.status = CRR_ERR_VH_EMPTY;
      } else if (new_first.v != src.at(cur.item_begin).v) {
        r.status = CRR_ERR_NDC_FIRST_ITEM_MISMATCH;
      } else if (lca.v > src.at(cur.item_begin + cur.item_count - 1).v) {
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

// wave-wide min / max (every lane of the wavefront active)
__device__ __forceinline__ u32 wave_min(u32 v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = min(v, (u32)__shfl_xor((int)v, off, 64));
  return v;
}
__device__ __forceinline__ u32 wave_max(u32 v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = max(v, (u32)__shfl_xor((int)v, off, 64));
  return v;
}
__device__ __forceinline__ void wave_sync_lds() {  // this wavefront's LDS writes -> visible to its lanes
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ void __launch_bounds__(kBlock) ndc_prepare_kernel(crr_ndc_inputs in, crr_ndc_result* res, crr_vh_item* out_items) {
  __shared__ alignas(16) crr_vh_item s_items[kWaves][kStageItems];
  __shared__ crr_ndc_branch s_br[kWaves][kStageBranches];
  const u32 k = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool live = k < in.n_tasks;
  crr_ndc_task t{};
  if (live) t = in.tasks[k];
  // 1. the wavefront's branch descriptors [bmin, bmax)
  const u32 bmin = wave_min(live && t.branch_count ? t.branch_begin : 0xFFFFFFFFu);
  const u32 bmax = wave_max(live && t.branch_count ? t.branch_begin + t.branch_count : 0u);
  const bool br_staged = bmax <= bmin || bmax - bmin <= kStageBranches;  // uniform
  if (br_staged)
    for (u32 i = bmin + lane; i < bmax; i += 64) s_br[wv][i - bmin] = in.branches[i];
  wave_sync_lds();
  // 2. the span of items the tasks use: every local branch's and the incoming history
  u32 imin = 0xFFFFFFFFu, imax = 0;
  if (live) {
    if (t.incoming_count) {
      imin = t.incoming_begin;
      imax = t.incoming_begin + t.incoming_count;
    }
    for (u32 b = 0; b < t.branch_count; ++b) {
      const crr_ndc_branch br = br_staged ? s_br[wv][t.branch_begin + b - bmin] : in.branches[t.branch_begin + b];
      if (br.item_count) {
        imin = min(imin, br.item_begin);
        imax = max(imax, br.item_begin + br.item_count);
      }
    }
  }
  imin = wave_min(imin);
  imax = wave_max(imax);
  const bool staged = br_staged && (imax <= imin || imax - imin <= kStageItems);  // uniform
  if (staged) {  // coalesced: 16 B per lane, consecutive lanes consecutive items
    const uint4* src = reinterpret_cast<const uint4*>(in.items);
    uint4* dst = reinterpret_cast<uint4*>(&s_items[wv][0]);
    for (u32 i = imin + lane; i < imax; i += 64) dst[i - imin] = src[i];
  }
  wave_sync_lds();
  if (!live) return;
  if (staged) prepare_task(LdsSrc{&s_items[wv][0], &s_br[wv][0], imin, bmin}, t, k, res, out_items);
  else prepare_task(GlobalSrc{in.items, in.branches}, t, k, res, out_items);
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
