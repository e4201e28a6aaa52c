// capi.hip -- the extern "C" boundary (include/cadence_replay.h) around the replay kernels.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <mutex>

#include "cadence_replay.h"
#include "stream_device.h"

namespace crr {
template <bool WAVE_TAIL, bool EMIT>
__global__ void replay_lds_kernel(crr_inputs in, crr_outputs out, int phase, uint32_t lo, uint32_t hi);
template <bool WAVE_TAIL, bool EMIT, bool LANES = false>
__global__ void replay_lds_small_kernel(crr_inputs in, crr_outputs out, int phase, uint32_t lo, uint32_t hi);
__global__ void replay_wide_kernel(crr_inputs in, crr_outputs out, int phase, uint32_t lo, uint32_t hi);
template <bool EMIT, bool RESUME>
__global__ void replay_compact1_kernel(crr_inputs in, crr_outputs out, int phase, uint32_t lo, uint32_t hi);
template <bool EMIT, bool RESUME>
__global__ void replay_compact2_kernel(crr_inputs in, crr_outputs out, int phase, uint32_t lo, uint32_t hi);
template <bool EMIT, bool RESUME>
__global__ void replay_compact3_kernel(crr_inputs in, crr_outputs out, int phase, uint32_t lo, uint32_t hi);
__global__ void replay_big_kernel(crr_inputs in, crr_outputs out, int phase, uint32_t lo, uint32_t hi);
template <bool EMIT, bool RESUME>
__global__ void replay_tail_kernel(crr_inputs in, crr_outputs out, int phase, uint32_t lo, uint32_t hi);
__global__ void replay_global_kernel(crr_inputs in, crr_outputs out, int phase, int retry_only);
__global__ void tail_gate_kernel(const uint32_t* scratch, uint32_t need);
__global__ void replay_retry_kernel(crr_inputs in, crr_outputs out, int phase);
__global__ void checksum_kernel(crr_inputs in, crr_outputs out, uint32_t* checksums);
__global__ void token_crc_kernel(crr_inputs in, uint32_t* out);
}

namespace {

constexpr int kBlock = 256;
// side streams with the higher priority: 1 compact tier 3, 2 the big long-tail kernel, 3 compact tier 1,
// 4 compact tier 2
constexpr unsigned kSegPrioMask = 0x1E;
constexpr int kWideBlock = 256;  // replay_wide_kernel's block
constexpr unsigned kRetryGrid = 512;  // 2 blocks (one wave, 67 KB LDS arena each) per CU x 256 CUs

// Launch state is kept per HIP device, not per host thread: a cgo caller's goroutines migrate between
// OS threads, and one thread may drive several devices.  Each device's state is created on first use
// and guarded by its mutex while a call enqueues (microseconds: nothing waits on the GPU under it);
// crr_release() destroys it.  The side streams a call forks its tier segments onto are keyed by the
// caller's stream (kSideSets sets per device), so callers on different streams do not queue each
// other's segments; with more distinct caller streams than sets, the least recently used set is reused
// (still correct -- a false dependency, no more).
constexpr int kMaxDevices = 64;
constexpr int kRing = 512;   // per-launch records of a measured region (crr_timing_begin .. _read)
constexpr int kSide = 6;
constexpr int kSideSets = 4;

// n events created, or none (a partial failure destroys what it created)
bool create_events(hipEvent_t* e, int n, unsigned flags) {
  for (int i = 0; i < n; ++i) {
    if (hipEventCreateWithFlags(&e[i], flags) != hipSuccess) {
      for (int j = 0; j < i; ++j) { (void)hipEventDestroy(e[j]); e[j] = nullptr; }
      e[i] = nullptr;
      return false;
    }
  }
  return true;
}
void destroy_events(hipEvent_t* e, int n) {
  for (int i = 0; i < n; ++i) { if (e[i]) (void)hipEventDestroy(e[i]); e[i] = nullptr; }
}

// One caller stream's side streams and fork / join events.
struct SideSet {
  hipStream_t caller = nullptr;   // the stream this set serves
  unsigned long long last_use = 0;
  hipStream_t side[kSide] = {};
  hipEvent_t fork = nullptr, join[kSide] = {};
  bool ready = false;

  bool create() {
    if (ready) return true;
    // the compact tiers carry most of a mixed batch's work and tiers 2 / 3 the longest-running
    // wavefronts (their blocks hold the most LDS per lane, so the fewest fit a CU): their streams get
    // the higher priority, so their workgroups are dispatched first and the short, dense segments fill
    // the CUs around them instead of ahead of them
    int lo_prio = 0, hi_prio = 0;
    if (hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio) != hipSuccess) lo_prio = hi_prio = 0;
    int made = 0;
    for (; made < kSide; ++made) {
      const int prio = ((kSegPrioMask >> made) & 1) ? hi_prio : lo_prio;
      if (hipStreamCreateWithPriority(&side[made], hipStreamNonBlocking, prio) != hipSuccess) break;
    }
    bool ok = made == kSide && create_events(&fork, 1, hipEventDisableTiming);
    if (ok && !create_events(join, kSide, hipEventDisableTiming)) {
      destroy_events(&fork, 1);
      ok = false;
    }
    if (!ok) {
      for (int i = 0; i < made; ++i) { (void)hipStreamDestroy(side[i]); side[i] = nullptr; }
      return false;
    }
    return ready = true;
  }
  void destroy() {
    if (!ready) return;
    for (auto& x : side) { if (x) { (void)hipStreamSynchronize(x); (void)hipStreamDestroy(x); } x = nullptr; }
    destroy_events(&fork, 1);
    destroy_events(join, kSide);
    ready = false;
    caller = nullptr;
  }
};

struct DeviceState {
  std::mutex mu;
  int device = -1;
  // crr_last_kernel_ms: [0,1] phase 0, [2,3] phase 1, [4,5] the phase-1 fast-path kernel alone
  hipEvent_t ev[6] = {};
  bool valid[3] = {false, false, false};
  bool events = false;
  // measured region: a ring of event pairs around each launch's fast group, no synchronisation between
  hipEvent_t ring[2 * kRing] = {};
  int ring_n = 0;
  bool ring_on = false, ring_events = false;
  // tier segments of one phase run concurrently: side streams fork from and join back into the
  // caller's stream
  SideSet sets[kSideSets];
  unsigned long long use_clock = 0;
  // diagnostics (crr_segment_timing): when each side stream's segments of the last phase-1 group
  // finished, relative to the fork
  bool seg_on = false, seg_valid = false, seg_events = false;
  hipEvent_t seg_start = nullptr, seg_end[kSide + 1] = {};

  bool ensure_events() {
    if (!events) events = create_events(ev, 6, hipEventDefault);
    return events;
  }
  bool ensure_ring() {
    if (!ring_events) ring_events = create_events(ring, 2 * kRing, hipEventDefault);
    return ring_events;
  }
  // the side-stream set of `caller` (created on first use), or nullptr when none can be created (the
  // call then launches every segment on the caller's stream)
  SideSet* sides_for(hipStream_t caller) {
    SideSet* pick = nullptr;
    for (auto& x : sets)
      if (x.ready && x.caller == caller) pick = &x;
    if (!pick)
      for (auto& x : sets)
        if (!x.ready) { pick = &x; break; }
    if (!pick) {  // every set serves another stream: reuse the least recently used one
      pick = &sets[0];
      for (auto& x : sets)
        if (x.last_use < pick->last_use) pick = &x;
    }
    if (!pick->create()) return nullptr;
    pick->caller = caller;
    pick->last_use = ++use_clock;
    return pick;
  }
  bool ensure_seg_events() {
    if (seg_events) return true;
    if (!create_events(&seg_start, 1, hipEventDefault)) return false;
    if (!create_events(seg_end, kSide + 1, hipEventDefault)) { destroy_events(&seg_start, 1); return false; }
    return seg_events = true;
  }
  // destroys everything (the device must be current); the state can be rebuilt by a later call
  void release() {
    for (auto& x : sets) x.destroy();
    destroy_events(ev, 6);
    destroy_events(ring, 2 * kRing);
    destroy_events(&seg_start, 1);
    destroy_events(seg_end, kSide + 1);
    events = ring_events = seg_events = false;
    valid[0] = valid[1] = valid[2] = false;
    ring_n = 0;
    ring_on = seg_on = seg_valid = false;
  }
  bool any() const {
    bool s = false;
    for (auto& x : sets) s = s || x.ready;
    return s || events || ring_events || seg_events;
  }
};
DeviceState g_dev[kMaxDevices];

// The state of the current device (hipGetDevice: HIP's device selection is per host thread).
DeviceState* current_state() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
  g_dev[dev].device = dev;
  return &g_dev[dev];
}

using crr_internal::StreamDevice;

bool valid_inputs(const crr_inputs* in, const crr_outputs* out) {
  if (!in || !out) return false;
  if (in->stride == 0) return false;
  if (in->n_wf == 0) return true;
  if (!in->wf || !out->exec) return false;
  const crr_events& e = in->ev;
  if (!e.etype || !e.event_id || !e.version || !e.timestamp || !e.task_id || !e.ref || !e.key || !e.aux) return false;
  if (!in->act_side || !in->start_side || !in->reset_keys || !in->arena) return false;
  if (!out->act || !out->timer || !out->child || !out->rc || !out->sig || !out->vh || !out->rp) return false;
  if ((in->flags & CRR_IN_EMIT_TASKS) && !out->tasks) return false;
  if (in->stride == 64 && !out->scratch) return false;
  if (out->digest && !in->digest_keys) return false;
  if (out->live_ids[0])  // the sidecar: all five columns or none
    for (int t = 1; t < 5; ++t)
      if (!out->live_ids[t]) return false;
  if (in->flags & CRR_IN_WAVE_TAIL) {
    if (in->stride != 64 || in->wave_begin > in->n_wf) return false;
  }
  if (in->flags & CRR_IN_TIERED) {
    // the lane kernels keep a wavefront's geometry in SGPRs: every segment must start on a group
    // (64-workflow) boundary, or its wavefronts would straddle two groups
    const uint32_t n_lane = (in->flags & CRR_IN_WAVE_TAIL) ? in->wave_begin : in->n_wf;
    if (in->stride != 64) return false;
    for (uint32_t b : {in->large_begin, in->compact_begin, in->compact2_begin, in->wide_begin, in->hbm_begin})
      if (b < n_lane && (b & 63u)) return false;
  }
  return true;
}

// Every crr_replay leaves the retry-list counters and the big segment's gate (scratch[0..3]) zeroed; an
// error return after the fast kernels were enqueued must reset them itself (the retry pass that would have
// is not launched).
int fail_reset(const crr_outputs* out, hipStream_t s, hipError_t err) {
  if (out->scratch) (void)hipMemsetAsync(out->scratch, 0, 4 * sizeof(uint32_t), s);
  return (int)err;
}

}  // namespace

extern "C" {

int crr_abi_version(void) { return CRR_ABI_VERSION; }

size_t crr_sizeof(int which) {
  switch (which) {
    case 0: return sizeof(crr_workflow);
    case 1: return sizeof(crr_exec_row);
    case 2: return sizeof(crr_activity_row);
    case 3: return sizeof(crr_timer_row);
    case 4: return sizeof(crr_child_row);
    case 5: return sizeof(crr_initiated_row);
    case 6: return sizeof(crr_vh_item);
    case 7: return sizeof(crr_reset_point_row);
    case 8: return sizeof(crr_activity_side);
    case 9: return sizeof(crr_start_side);
    case 10: return sizeof(crr_ndc_task);
    case 11: return sizeof(crr_ndc_result);
    case 12: return sizeof(crr_task_row);
    case 13: return sizeof(crr_inputs);
    case 14: return sizeof(crr_outputs);
    default: return 0;
  }
}

int crr_set_device(int device) { return (int)hipSetDevice(device); }

int crr_segment_timing(int on) {
  DeviceState* d = current_state();
  if (!d) return -1;
  std::lock_guard<std::mutex> lk(d->mu);
  if (on && !d->ensure_seg_events()) return -1;
  d->seg_on = on != 0;
  d->seg_valid = false;
  return 0;
}

int crr_segment_ms(float* out, int n) {
  DeviceState* d = current_state();
  if (!d) return -1;
  std::lock_guard<std::mutex> lk(d->mu);
  if (!d->seg_valid || n < kSide + 1) return -1;
  for (int i = 0; i <= kSide; ++i)
    if (hipEventElapsedTime(&out[i], d->seg_start, d->seg_end[i]) != hipSuccess) return -1;
  return kSide + 1;
}

int crr_replay(const crr_inputs* in, const crr_outputs* out, void* stream) {
  if (!valid_inputs(in, out)) return -1;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (in->n_wf == 0) {
    // an empty batch still zeroes the digest (an empty rank's buffer joins the all-reduce)
    if (!out->digest) return 0;
    StreamDevice on_dev0(s);
    if (!on_dev0.ok) return (int)hipErrorInvalidHandle;
    return (int)hipMemsetAsync(out->digest, 0, CRR_DIGEST_WORDS * sizeof(int64_t), s);
  }
  StreamDevice on_dev(s);
  if (!on_dev.ok) return (int)hipErrorInvalidHandle;
  DeviceState* d = current_state();
  if (!d) return (int)hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lk(d->mu);
  // inside a crr_timing_begin region the ring's event pair is the only record: the per-call
  // phase events (crr_last_kernel_ms) would add four event packets to every measured step
  const bool timed = !d->ring_on && d->ensure_events();
  const unsigned grid = (in->n_wf + kBlock - 1) / kBlock;
  const unsigned n_lane = (in->flags & CRR_IN_WAVE_TAIL) ? in->wave_begin : in->n_wf;
  d->valid[0] = d->valid[1] = d->valid[2] = false;
  // the kernels add every workflow's contribution as it is finalised (crr_outputs.digest)
  if (out->digest && hipMemsetAsync(out->digest, 0, CRR_DIGEST_WORDS * sizeof(int64_t), s) != hipSuccess)
    return (int)hipGetLastError();
  for (int phase = 0; phase < 2; ++phase) {
    if (phase == 0 && !(in->flags & CRR_IN_HAS_NEW_RUN)) continue;
    if (timed) (void)hipEventRecord(d->ev[2 * phase], s);
    if (in->stride == 64) {
      // fast path (LDS-held tables), then one retry pass for the workflows it handed back; the
      // scratch counters are zero on entry (zero-filled by the caller, reset by the retry pass)
      const bool tail = n_lane < in->n_wf;
      const bool small = (in->flags & CRR_IN_LDS_SMALL) != 0;
      if (timed && phase == 1) (void)hipEventRecord(d->ev[4], s);
      const bool ring = phase == 1 && d->ring_on && d->ring_n < kRing;
      if (ring) (void)hipEventRecord(d->ring[2 * d->ring_n], s);
      // task emission is a separate instantiation: the plain replay loop carries none of its registers
      const bool emit = (in->flags & CRR_IN_EMIT_TASKS) != 0;
      // long-tail workflows [tail_end, n_wf) that no fast per-wave arena is expected to hold
      const uint32_t tail_end = ((in->flags & CRR_IN_TIERED) && in->big_begin >= n_lane && in->big_begin < in->n_wf)
                                    ? in->big_begin : in->n_wf;
      // one fast launch: the wave tail first (optional), then lane workflows [lo, hi)
      auto launch_fast = [&](hipStream_t s, bool small_tier, bool with_tail, uint32_t lo, uint32_t hi, bool lanes = false) {
        const unsigned wave_blocks = with_tail ? (tail_end - n_lane + kBlock / 64 - 1) / (kBlock / 64) : 0;
        const unsigned blocks = wave_blocks + (hi - lo + kBlock - 1) / kBlock;
        if (blocks == 0) return;
        const dim3 g(blocks), b(kBlock);
        if (emit) {
          if (small_tier && with_tail) hipLaunchKernelGGL((crr::replay_lds_small_kernel<true, true>), g, b, 0, s, *in, *out, phase, lo, hi);
          else if (small_tier) hipLaunchKernelGGL((crr::replay_lds_small_kernel<false, true>), g, b, 0, s, *in, *out, phase, lo, hi);
          else if (with_tail) hipLaunchKernelGGL((crr::replay_lds_kernel<true, true>), g, b, 0, s, *in, *out, phase, lo, hi);
          else hipLaunchKernelGGL((crr::replay_lds_kernel<false, true>), g, b, 0, s, *in, *out, phase, lo, hi);
        } else {
          if (small_tier && with_tail) hipLaunchKernelGGL((crr::replay_lds_small_kernel<true, false>), g, b, 0, s, *in, *out, phase, lo, hi);
          else if (small_tier && lanes) hipLaunchKernelGGL((crr::replay_lds_small_kernel<false, false, true>), g, b, 0, s, *in, *out, phase, lo, hi);
          else if (small_tier) hipLaunchKernelGGL((crr::replay_lds_small_kernel<false, false>), g, b, 0, s, *in, *out, phase, lo, hi);
          else if (with_tail) hipLaunchKernelGGL((crr::replay_lds_kernel<true, false>), g, b, 0, s, *in, *out, phase, lo, hi);
          else hipLaunchKernelGGL((crr::replay_lds_kernel<false, false>), g, b, 0, s, *in, *out, phase, lo, hi);
        }
      };
      if (in->flags & CRR_IN_TIERED) {
        // segments by expected live-set size: 1 entry per map | 2 | compact tiers 1-3 | more (HBM rows)
        auto clampb = [&](uint32_t b, uint32_t lo) { return b < lo ? lo : (b < n_lane ? b : n_lane); };
        // loaded states (CRR_IN_HAS_RESUME) continue in the compact tiers' arenas; the host places them there
        // (flatten.resumed_bounds), so the 1- and 2-slot segments keep their fast kernels for the batch's fresh
        // workflows (a loaded state found in one goes to the general path: speed only)
        const bool resume = (in->flags & CRR_IN_HAS_RESUME) != 0;
        const uint32_t lb = clampb(in->large_begin, 0), cb = clampb(in->compact_begin, lb);
        const uint32_t c2 = clampb(in->compact2_begin, cb), wb = clampb(in->wide_begin, c2);
        const uint32_t hb = clampb(in->hbm_begin, wb);
        const bool run_small = lb > 0, run_large = cb > lb, run_tail = tail && tail_end > n_lane;
        const bool run_c1 = c2 > cb, run_c2 = wb > c2, run_c3 = hb > wb, run_wide = hb < n_lane;
        const bool run_big = tail_end < in->n_wf;
        // more than one segment: the others fork onto the side streams (each launch alone leaves
        // most of the chip idle: few wavefronts, each latency-bound) and join back before the retry
        const bool many = (int)run_small + (int)run_large + (int)run_c1 + (int)run_c2 + (int)run_c3 + (int)run_wide +
                              (int)run_big + (int)run_tail > 1;
        // no side streams to be had: every segment on the caller's stream (serial, same results)
        SideSet* ss = many ? d->sides_for(s) : nullptr;
        const bool fork = ss != nullptr;
        hipStream_t s_large = fork ? ss->side[0] : s, s_wide = fork ? ss->side[1] : s, s_big = fork ? ss->side[2] : s;
        hipStream_t s_c1 = fork ? ss->side[3] : s, s_c2 = fork ? ss->side[4] : s, s_tail = fork ? ss->side[5] : s;
        const bool seg = fork && d->seg_on && phase == 1 && d->seg_events;
        if (fork) {
          if (seg) (void)hipEventRecord(d->seg_start, s);
          (void)hipEventRecord(ss->fork, s);
          for (hipStream_t x : ss->side) (void)hipStreamWaitEvent(x, ss->fork, 0);
        }
        // Launch order: the big long-tail kernel first (its 65-KB blocks fit only beside few tail wavefronts),
        // then the lane segments, the tail last.  The tail's thousands of 13-KB wavefronts fill every CU's LDS
        // as soon as they are dispatched, and a kernel queued behind them on another stream then waits for
        // tail wavefronts to finish (config 4: the big kernel finishing at 9.2 ms instead of ~5 when the tail
        // won the race); the lane segments are short, and the tail wavefronts they delay are its shortest.
        if (run_big)  // the longest histories first
          hipLaunchKernelGGL(crr::replay_big_kernel, dim3(in->n_wf - tail_end), dim3(64), 0, s_big, *in, *out, phase,
                             tail_end, in->n_wf);
        // a compact tier's launch: <EMIT, RESUME> instantiations
#define CRR_LAUNCH_COMPACT(K, lo_, hi_, strm)                                                                     \
        do {                                                                                                       \
          const dim3 g_(((hi_) - (lo_) + 63) / 64), b_(64);                                                       \
          if (emit && resume) hipLaunchKernelGGL((crr::K<true, true>), g_, b_, 0, strm, *in, *out, phase, lo_, hi_);  \
          else if (emit) hipLaunchKernelGGL((crr::K<true, false>), g_, b_, 0, strm, *in, *out, phase, lo_, hi_);      \
          else if (resume) hipLaunchKernelGGL((crr::K<false, true>), g_, b_, 0, strm, *in, *out, phase, lo_, hi_);    \
          else hipLaunchKernelGGL((crr::K<false, false>), g_, b_, 0, strm, *in, *out, phase, lo_, hi_);               \
        } while (0)
        if (run_c3) CRR_LAUNCH_COMPACT(replay_compact3_kernel, wb, hb, s_wide);
        if (run_wide)
          hipLaunchKernelGGL(crr::replay_wide_kernel, dim3((n_lane - hb + kWideBlock - 1) / kWideBlock), dim3(kWideBlock), 0,
                             s_wide, *in, *out, phase, hb, n_lane);
        if (run_c2) CRR_LAUNCH_COMPACT(replay_compact2_kernel, c2, wb, s_c2);
        if (run_c1) CRR_LAUNCH_COMPACT(replay_compact1_kernel, cb, c2, s_c1);
#undef CRR_LAUNCH_COMPACT
        launch_fast(s_large, false, false, lb, cb);
        // the 1-slot segment of a multi-segment (mixed) batch takes the divergent dispatch; a one-class
        // batch (config 2) replays in lockstep and keeps the plain switch
        launch_fast(s, true, false, 0, lb, fork);
        if (run_tail) {  // the long-history tail, one wavefront each
          // behind the big segment's blocks (tail_gate_kernel): they cannot start once tail wavefronts hold the LDS
          if (run_big && fork)
            hipLaunchKernelGGL(crr::tail_gate_kernel, dim3(1), dim3(64), 0, s_tail, out->scratch, in->n_wf - tail_end);
          const dim3 g_(tail_end - n_lane), b_(64);
          if (emit && resume) hipLaunchKernelGGL((crr::replay_tail_kernel<true, true>), g_, b_, 0, s_tail, *in, *out, phase, n_lane, tail_end);
          else if (emit) hipLaunchKernelGGL((crr::replay_tail_kernel<true, false>), g_, b_, 0, s_tail, *in, *out, phase, n_lane, tail_end);
          else if (resume) hipLaunchKernelGGL((crr::replay_tail_kernel<false, true>), g_, b_, 0, s_tail, *in, *out, phase, n_lane, tail_end);
          else hipLaunchKernelGGL((crr::replay_tail_kernel<false, false>), g_, b_, 0, s_tail, *in, *out, phase, n_lane, tail_end);
        }
        if (fork) {
          if (seg) {
            for (int i = 0; i < kSide; ++i) (void)hipEventRecord(d->seg_end[i], ss->side[i]);
            (void)hipEventRecord(d->seg_end[kSide], s);
            d->seg_valid = true;
          }
          for (int i = 0; i < kSide; ++i) {
            (void)hipEventRecord(ss->join[i], ss->side[i]);
            (void)hipStreamWaitEvent(s, ss->join[i], 0);
          }
        }
      } else {
        launch_fast(s, small, tail, 0, n_lane);
      }
      hipError_t err = hipGetLastError();
      if (err != hipSuccess) return fail_reset(out, s, err);
      if (timed && phase == 1) {
        (void)hipEventRecord(d->ev[5], s);
        d->valid[2] = true;
      }
      if (ring) {
        (void)hipEventRecord(d->ring[2 * d->ring_n + 1], s);
        ++d->ring_n;
      }
      const unsigned retry_grid = in->n_wf < kRetryGrid ? in->n_wf : kRetryGrid;
      hipLaunchKernelGGL(crr::replay_retry_kernel, dim3(retry_grid), dim3(64), 0, s, *in, *out, phase);
    } else {
      hipLaunchKernelGGL(crr::replay_global_kernel, dim3(grid), dim3(kBlock), 0, s, *in, *out, phase, 0);
    }
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return in->stride == 64 ? fail_reset(out, s, err) : (int)err;
    if (timed) {
      (void)hipEventRecord(d->ev[2 * phase + 1], s);
      d->valid[phase] = true;
    }
  }
  return 0;
}

int crr_checksum(const crr_inputs* in, const crr_outputs* out, uint32_t* checksums, void* stream) {
  if (!valid_inputs(in, out) || (!checksums && in->n_wf)) return -1;
  if (in->n_wf == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  StreamDevice on_dev(s);
  if (!on_dev.ok) return (int)hipErrorInvalidHandle;
  const unsigned grid = (in->n_wf + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(crr::checksum_kernel, dim3(grid), dim3(kBlock), 0, s, *in, *out, checksums);
  return (int)hipGetLastError();
}

int crr_token_crc(const crr_inputs* in, uint32_t* crc, void* stream) {
  if (!in || (in->n_wf && (!in->wf || !in->arena || !crc))) return -1;
  if (in->n_wf == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  StreamDevice on_dev(s);
  if (!on_dev.ok) return (int)hipErrorInvalidHandle;
  hipLaunchKernelGGL(crr::token_crc_kernel, dim3((in->n_wf + 255) / 256), dim3(256), 0, s, *in, crc);
  return (int)hipGetLastError();
}

float crr_last_kernel_ms(int which) {
  DeviceState* d = current_state();
  if (!d || which < 0 || which > 2) return -1.0f;
  std::lock_guard<std::mutex> lk(d->mu);
  if (!d->valid[which]) return -1.0f;
  float ms = -1.0f;
  if (hipEventElapsedTime(&ms, d->ev[2 * which], d->ev[2 * which + 1]) != hipSuccess) return -1.0f;
  return ms;
}

int crr_timing_begin(void) {
  DeviceState* d = current_state();
  if (!d) return -1;
  std::lock_guard<std::mutex> lk(d->mu);
  if (!d->ensure_ring()) return -1;
  d->ring_n = 0;
  d->ring_on = true;
  return 0;
}

int crr_timing_read(float* ms, int cap) {
  DeviceState* d = current_state();
  if (!d) return -1;
  std::lock_guard<std::mutex> lk(d->mu);
  d->ring_on = false;
  int n = d->ring_n < cap ? d->ring_n : cap;
  for (int i = 0; i < n; ++i) {
    if (hipEventSynchronize(d->ring[2 * i + 1]) != hipSuccess) return -1;
    if (hipEventElapsedTime(&ms[i], d->ring[2 * i], d->ring[2 * i + 1]) != hipSuccess) return -1;
  }
  return n;
}

int crr_release(void) {
  int cur = -1;
  const bool have_cur = hipGetDevice(&cur) == hipSuccess;
  int rc = 0;
  for (int i = 0; i < kMaxDevices; ++i) {
    DeviceState& d = g_dev[i];
    std::lock_guard<std::mutex> lk(d.mu);
    if (!d.any()) continue;
    if (hipSetDevice(i) != hipSuccess) { rc = -1; continue; }
    d.release();
  }
  if (have_cur) (void)hipSetDevice(cur);
  return rc;
}

uint32_t crr_crc32_ieee(const uint8_t* data, size_t len) {
  struct Table {
    uint32_t t[256];
    Table() {
      for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
        t[i] = c;
      }
    }
  };
  static const Table tab;  // thread-safe static init
  const uint32_t* table = tab.t;
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < len; ++i) c = table[(c ^ data[i]) & 0xff] ^ (c >> 8);
  return ~c;
}

}  // extern "C"
