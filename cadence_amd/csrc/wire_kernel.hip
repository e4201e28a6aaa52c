// wire_kernel.hip -- narrow upload format for the event columns, widened on the device.
//
// The event columns are 49 B/event wide (five int64 columns), yet within one workflow consecutive
// events differ by little: IDs and TaskIDs step by one, versions change only at failovers, refs
// point a few events back, timestamps advance by milliseconds to seconds.  Over PCIe (~50 GB/s,
// two orders below HBM) the host therefore ships each column as per-event deltas along the
// workflow's steps at the narrowest byte width (1..8) that holds every delta of the batch, and this
// kernel rebuilds the exact int64 columns in HBM (wrapping uint64 arithmetic: bit-exact for any
// input) before crr_replay reads them.  The layout is the wide one's slot for slot (same ev_begin /
// stride / wave tail), so the descriptors, side records and tables are untouched.
//   lane workflows [0, wave_begin): one thread per workflow walks its steps (the 64 lanes of a group
//     read and write one contiguous run per step) and zero-fills its padding up to the group length;
//   wave tail [wave_begin, n_wf): one wavefront per workflow, 64 steps at a time, a shuffle scan of
//     the deltas plus the carry of the previous 64.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cadence_replay.h"
#include "stream_device.h"

namespace crr {
namespace {

constexpr int kWireBlock = 256;

__device__ __forceinline__ uint64_t load_narrow(const crr_packed_column& c, int64_t i) {
  const uint8_t* p = c.data + (size_t)i * c.width;
  uint64_t v = 0;
  for (uint32_t b = 0; b < c.width; ++b) v |= (uint64_t)p[b] << (8 * b);
  if (c.kind != CRR_PACK_UNSIGNED && c.width < 8) {  // sign-extend
    const uint32_t sh = 64 - 8 * c.width;
    v = (uint64_t)((int64_t)(v << sh) >> sh);
  }
  return v;
}

struct Cols {
  uint64_t id, ver, ts, task, ref, key, aux;
};

__device__ __forceinline__ Cols load_all(const crr_packed_events& P, int64_t i) {
  return Cols{load_narrow(P.event_id, i), load_narrow(P.version, i), load_narrow(P.timestamp, i),
              load_narrow(P.task_id, i),  load_narrow(P.ref, i),     load_narrow(P.key, i),
              load_narrow(P.aux, i)};
}

// running values of the delta-coded columns; the others decode from the event alone
__device__ __forceinline__ void store(const crr_events& E, int64_t i, const crr_packed_events& P, const Cols& run,
                                      const Cols& raw) {
  int64_t* id = const_cast<int64_t*>(E.event_id);
  int64_t* ver = const_cast<int64_t*>(E.version);
  int64_t* ts = const_cast<int64_t*>(E.timestamp);
  int64_t* task = const_cast<int64_t*>(E.task_id);
  int64_t* ref = const_cast<int64_t*>(E.ref);
  uint32_t* key = const_cast<uint32_t*>(E.key);
  int32_t* aux = const_cast<int32_t*>(E.aux);
  id[i] = (int64_t)run.id;
  ver[i] = (int64_t)run.ver;
  ts[i] = (int64_t)run.ts;
  task[i] = (int64_t)run.task;
  ref[i] = P.ref.kind == CRR_PACK_ID_MINUS ? (int64_t)(run.id - raw.ref) : (int64_t)raw.ref;
  key[i] = (uint32_t)raw.key;
  aux[i] = (int32_t)(uint32_t)raw.aux;
}

__device__ __forceinline__ void zero(const crr_events& E, int64_t i) {
  const_cast<int64_t*>(E.event_id)[i] = 0;
  const_cast<int64_t*>(E.version)[i] = 0;
  const_cast<int64_t*>(E.timestamp)[i] = 0;
  const_cast<int64_t*>(E.task_id)[i] = 0;
  const_cast<int64_t*>(E.ref)[i] = 0;
  const_cast<uint32_t*>(E.key)[i] = 0;
  const_cast<int32_t*>(E.aux)[i] = 0;
}

__device__ __forceinline__ uint64_t step(const crr_packed_column& c, uint64_t prev, uint64_t raw) {
  return c.kind == CRR_PACK_DELTA ? prev + raw : raw;
}

__global__ void __launch_bounds__(kWireBlock) widen_lanes_kernel(crr_packed_events P, crr_inputs in, uint32_t n_lane) {
  const uint32_t w = blockIdx.x * kWireBlock + threadIdx.x;
  const bool live = w < n_lane;
  const crr_workflow* wfp = in.wf + (live ? w : 0);
  const int64_t begin = live ? wfp->ev_begin : 0;
  const int32_t n = live ? wfp->ev_count : 0;
  // a wavefront is one interleaved group (groups start at multiples of 64): pad to its longest member
  int32_t glen = n;
  for (int d = 32; d >= 1; d >>= 1) glen = max(glen, __shfl_xor(glen, d, 64));
  if (!live) return;
  const uint64_t ts0 = P.ts_base ? (uint64_t)P.ts_base[w] : 0;
  Cols run{0, 0, ts0, 0, 0, 0, 0};
  for (int32_t k = 0; k < glen; ++k) {
    const int64_t i = begin + (int64_t)k * in.stride;
    if (k < n) {
      const Cols raw = load_all(P, i);
      run.id = step(P.event_id, run.id, raw.id);
      run.ver = step(P.version, run.ver, raw.ver);
      run.ts = step(P.timestamp, run.ts, raw.ts);
      run.task = step(P.task_id, run.task, raw.task);
      store(in.ev, i, P, run, raw);
    } else {
      zero(in.ev, i);
    }
  }
}

__device__ __forceinline__ uint64_t wave_scan(uint64_t v) {  // inclusive prefix sum over the 64 lanes
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

__device__ __forceinline__ uint64_t scan_col(const crr_packed_column& c, uint64_t raw, uint64_t& carry) {
  if (c.kind != CRR_PACK_DELTA) return raw;
  const uint64_t s = wave_scan(raw) + carry;
  carry = __shfl(s, 63, 64);
  return s;
}

__global__ void __launch_bounds__(64) widen_tail_kernel(crr_packed_events P, crr_inputs in, uint32_t lo) {
  const uint32_t w = lo + blockIdx.x;
  if (w >= in.n_wf) return;
  const crr_workflow* wfp = in.wf + w;
  const int64_t begin = wfp->ev_begin;
  const int32_t n = wfp->ev_count;
  const int lane = threadIdx.x & 63;
  Cols carry{0, 0, P.ts_base ? (uint64_t)P.ts_base[w] : 0, 0, 0, 0, 0};
  for (int32_t c0 = 0; c0 < n; c0 += 64) {
    const int32_t k = c0 + lane;
    const bool ok = k < n;
    const int64_t i = begin + k;
    Cols raw = ok ? load_all(P, i) : Cols{0, 0, 0, 0, 0, 0, 0};
    Cols run;
    run.id = scan_col(P.event_id, raw.id, carry.id);
    run.ver = scan_col(P.version, raw.ver, carry.ver);
    run.ts = scan_col(P.timestamp, raw.ts, carry.ts);
    run.task = scan_col(P.task_id, raw.task, carry.task);
    if (ok) store(in.ev, i, P, run, raw);
  }
}

}  // namespace
}  // namespace crr

extern "C" {

int crr_widen_events(const crr_packed_events* packed, const crr_inputs* in, void* stream) {
  if (!packed || !in || !in->wf) return -1;
  const crr_packed_column* cols[7] = {&packed->event_id, &packed->version, &packed->timestamp, &packed->task_id,
                                      &packed->ref, &packed->key, &packed->aux};
  for (const crr_packed_column* c : cols) {
    if (!c->data || c->width < 1 || c->width > 8 || c->kind > CRR_PACK_ID_MINUS) return -1;
  }
  if (packed->ref.kind == CRR_PACK_DELTA || packed->key.kind == CRR_PACK_DELTA || packed->aux.kind == CRR_PACK_DELTA)
    return -1;  // ref: plain or event_id - ref; key / aux: plain
  const crr_events& e = in->ev;
  if (!e.event_id || !e.version || !e.timestamp || !e.task_id || !e.ref || !e.key || !e.aux) return -1;
  if (in->stride != 1 && in->stride != 64) return -1;
  if (in->n_wf == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  crr_internal::StreamDevice on_dev_(s);
  if (!on_dev_.ok) return (int)hipErrorInvalidHandle;
  const uint32_t n_lane = (in->flags & CRR_IN_WAVE_TAIL) ? in->wave_begin : in->n_wf;
  if (n_lane > in->n_wf) return -1;
  if (in->stride == 1 && n_lane) {  // canonical batch: every workflow one wavefront
    hipLaunchKernelGGL(crr::widen_tail_kernel, dim3(in->n_wf), dim3(64), 0, s, *packed, *in, 0u);
    return (int)hipGetLastError();
  }
  if (n_lane)
    hipLaunchKernelGGL(crr::widen_lanes_kernel, dim3((n_lane + crr::kWireBlock - 1) / crr::kWireBlock), dim3(crr::kWireBlock),
                       0, s, *packed, *in, n_lane);
  if (n_lane < in->n_wf)
    hipLaunchKernelGGL(crr::widen_tail_kernel, dim3(in->n_wf - n_lane), dim3(64), 0, s, *packed, *in, n_lane);
  return (int)hipGetLastError();
}

}  // extern "C"
