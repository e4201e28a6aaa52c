// compact_kernel.hip -- live-row compaction of a replay's outputs for the download.
//
// What the Go caller persists after a rebuild is the snapshot of the live state
// (mutableStateBuilder.CloseTransactionAsSnapshot, service/history/execution/mutable_state_builder.go:4033-4100:
// ActivityInfos / TimerInfos / ChildExecutionInfos / RequestCancelInfos / SignalInfos from the pending
// maps, the VersionHistories and the execution info with its reset points) -- not the engine's slot
// tables, which are sized by capacity.  This gathers each workflow's live rows (slots 0..n-1, n = its
// exec-row count clamped to its capacity; crr_replay's finalize leaves them there in ID order) into
// dense per-table buffers in workflow order, so the device->host copy carries live rows only:
//   1. count: one thread per workflow reads its counts; a wavefront prefix (shuffle-up scan) and an
//      LDS pass across the block's wavefronts give block-local prefixes;
//   2. scan: one block scans the per-block totals;
//   3. gather: the final offsets, then the rows copied as 8-byte words (the 64 lanes of a group read
//      slot j of 64 consecutive workflows: contiguous rows in the interleaved layout).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cadence_replay.h"
#include "stream_device.h"

namespace crr {
namespace {

constexpr int kT = CRR_COMPACT_TABLES;
constexpr int kCompactBlock = 256;
constexpr int kScanBlock = 1024;

struct TableDesc {
  const uint8_t* src;
  uint32_t row_bytes;
};

// count of table t for workflow w (the exec row's n_*, clamped to [0, cap]; tasks only when emitted)
__device__ __forceinline__ void counts_of(const crr_inputs& in, const crr_outputs& out, uint32_t w, int64_t c[kT]) {
  const crr_exec_row& R = out.exec[w];
  const crr_workflow& D = in.wf[w];
  const int32_t n[kT] = {R.n_activity, R.n_timer, R.n_child, R.n_rc, R.n_signal, R.n_vh_items, R.n_reset_points,
                         (in.flags & CRR_IN_EMIT_TASKS) ? R.n_tasks : 0};
  const int32_t cap[kT] = {D.act_cap, D.timer_cap, D.child_cap, D.rc_cap, D.sig_cap, D.vh_cap, D.rp_cap, D.task_cap};
#pragma unroll
  for (int t = 0; t < kT; ++t) c[t] = n[t] < 0 ? 0 : (n[t] < cap[t] ? n[t] : cap[t]);
}

// inclusive prefix over the wavefront of a per-lane value (DPP-free: shuffles up the 64 lanes)
__device__ __forceinline__ int64_t wave_inclusive(int64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

__global__ void __launch_bounds__(kCompactBlock) compact_count_kernel(crr_inputs in, crr_outputs out, int64_t* offsets,
                                                                     int64_t* block_sums, uint32_t n_blocks) {
  __shared__ int64_t wave_tot[kT][kCompactBlock / 64];
  const uint32_t w = blockIdx.x * kCompactBlock + threadIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t c[kT];
  if (w < in.n_wf) counts_of(in, out, w, c);
  else
    for (int t = 0; t < kT; ++t) c[t] = 0;
  int64_t incl[kT];
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    incl[t] = wave_inclusive(c[t]);
    if (lane == 63) wave_tot[t][wv] = incl[t];
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    int64_t before = 0, tot = 0;
    for (int k = 0; k < kCompactBlock / 64; ++k) {
      const int64_t x = wave_tot[t][k];
      before += k < wv ? x : 0;
      tot += x;
    }
    if (w < in.n_wf) offsets[(size_t)t * (in.n_wf + 1) + w] = before + incl[t] - c[t];  // block-local
    if (threadIdx.x == 0) block_sums[(size_t)t * n_blocks + blockIdx.x] = tot;
  }
}

// one block: exclusive scan of each table's block totals (in place); the grand totals -> offsets[t][n_wf]
__global__ void __launch_bounds__(kScanBlock) compact_scan_kernel(int64_t* block_sums, uint32_t n_blocks, int64_t* offsets,
                                                                  uint32_t n_wf) {
  __shared__ int64_t part[kScanBlock];
  const uint32_t per = (n_blocks + kScanBlock - 1) / kScanBlock;
  for (int t = 0; t < kT; ++t) {
    int64_t* b = block_sums + (size_t)t * n_blocks;
    const uint32_t lo = threadIdx.x * per, hi = min(lo + per, n_blocks);
    int64_t s = 0;
    for (uint32_t i = lo; i < hi; ++i) s += b[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int d = 1; d < kScanBlock; d <<= 1) {  // Hillis-Steele over the 1024 partial sums
      const int64_t o = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0;
      __syncthreads();
      part[threadIdx.x] += o;
      __syncthreads();
    }
    int64_t run = part[threadIdx.x] - s;
    for (uint32_t i = lo; i < hi; ++i) {
      const int64_t x = b[i];
      b[i] = run;
      run += x;
    }
    if (threadIdx.x == kScanBlock - 1) offsets[(size_t)t * (n_wf + 1) + n_wf] = part[kScanBlock - 1];
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kCompactBlock) compact_gather_kernel(crr_inputs in, crr_outputs out, crr_compact_out dst,
                                                                      const int64_t* block_sums, uint32_t n_blocks) {
  const uint32_t w = blockIdx.x * kCompactBlock + threadIdx.x;
  if (w >= in.n_wf) return;
  const crr_workflow& D = in.wf[w];
  const int64_t st = ((in.flags & CRR_IN_WAVE_TAIL) && w >= in.wave_begin) ? 1 : (int64_t)in.stride;
  int64_t c[kT];
  counts_of(in, out, w, c);
  const TableDesc tab[kT] = {
      {reinterpret_cast<const uint8_t*>(out.act), (uint32_t)sizeof(crr_activity_row)},
      {reinterpret_cast<const uint8_t*>(out.timer), (uint32_t)sizeof(crr_timer_row)},
      {reinterpret_cast<const uint8_t*>(out.child), (uint32_t)sizeof(crr_child_row)},
      {reinterpret_cast<const uint8_t*>(out.rc), (uint32_t)sizeof(crr_initiated_row)},
      {reinterpret_cast<const uint8_t*>(out.sig), (uint32_t)sizeof(crr_initiated_row)},
      {reinterpret_cast<const uint8_t*>(out.vh), (uint32_t)sizeof(crr_vh_item)},
      {reinterpret_cast<const uint8_t*>(out.rp), (uint32_t)sizeof(crr_reset_point_row)},
      {reinterpret_cast<const uint8_t*>(out.tasks), (uint32_t)sizeof(crr_task_row)}};
  const int64_t base[kT] = {D.act_base, D.timer_base, D.child_base, D.rc_base, D.sig_base, D.vh_base, D.rp_base, D.task_base};
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    int64_t* off = dst.offsets + (size_t)t * (in.n_wf + 1);
    const int64_t o = off[w] + block_sums[(size_t)t * n_blocks + blockIdx.x];
    off[w] = o;
    uint8_t* d = reinterpret_cast<uint8_t*>(dst.rows[t]);
    if (!d || !tab[t].src) continue;
    const uint32_t words = tab[t].row_bytes / 8;  // every row type is a multiple of 8 bytes
    for (int64_t j = 0; j < c[t]; ++j) {
      const uint64_t* s = reinterpret_cast<const uint64_t*>(tab[t].src + (size_t)(base[t] + j * st) * tab[t].row_bytes);
      uint64_t* q = reinterpret_cast<uint64_t*>(d + (size_t)(o + j) * tab[t].row_bytes);
      for (uint32_t k = 0; k < words; ++k) q[k] = s[k];
    }
  }
}

}  // namespace
}  // namespace crr

extern "C" {

size_t crr_compact_scratch_bytes(uint32_t n_wf) {
  const size_t n_blocks = (n_wf + crr::kCompactBlock - 1) / crr::kCompactBlock;
  return (n_blocks ? n_blocks : 1) * crr::kT * sizeof(int64_t);
}

int crr_compact_rows(const crr_inputs* in, const crr_outputs* out, const crr_compact_out* dst, void* stream) {
  if (!in || !out || !dst || !dst->offsets || !dst->scratch || !out->exec || !in->wf) return -1;
  if (in->stride == 0 || ((in->flags & CRR_IN_WAVE_TAIL) && in->wave_begin > in->n_wf)) return -1;
  for (int t = 0; t < CRR_COMPACT_TABLES; ++t)
    if ((uintptr_t)dst->rows[t] & 7u) return -1;  // rows are copied as 8-byte words
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  crr_internal::StreamDevice on_dev_(s);
  if (!on_dev_.ok) return (int)hipErrorInvalidHandle;
  if (in->n_wf == 0) return hipMemsetAsync(dst->offsets, 0, CRR_COMPACT_TABLES * sizeof(int64_t), s) == hipSuccess ? 0 : -2;
  const uint32_t n_blocks = (in->n_wf + crr::kCompactBlock - 1) / crr::kCompactBlock;
  int64_t* bsum = reinterpret_cast<int64_t*>(dst->scratch);
  hipLaunchKernelGGL(crr::compact_count_kernel, dim3(n_blocks), dim3(crr::kCompactBlock), 0, s, *in, *out, dst->offsets,
                     bsum, n_blocks);
  hipLaunchKernelGGL(crr::compact_scan_kernel, dim3(1), dim3(crr::kScanBlock), 0, s, bsum, n_blocks, dst->offsets, in->n_wf);
  hipLaunchKernelGGL(crr::compact_gather_kernel, dim3(n_blocks), dim3(crr::kCompactBlock), 0, s, *in, *out, *dst, bsum,
                     n_blocks);
  return (int)hipGetLastError();
}

}  // extern "C"
