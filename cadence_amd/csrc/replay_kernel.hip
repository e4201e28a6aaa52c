// replay_kernel.hip -- CDNA4 (gfx950) batched mutable-state replay.
//
// One lane replays one workflow (the short-history bucket): every
// workflow is an independent event-sourced state machine, so a wavefront advances 64 workflows
// in lock step.  With the wave-interleaved input layout (stride 64) each per-step column load of a
// wavefront is one contiguous 64-element run; the execution-info scalars, the version history's
// last item and the table occupancy live in VGPRs; the pending activity / timer / child /
// request-cancel / signal maps are per-workflow slot tables in HBM (interleaved the same way, so
// lanes probing slot j touch one contiguous run), reused on delete so a workflow's footprint is its
// peak concurrency.  The epilogue sorts the live rows by event ID (the order the checksum encodes)
// and streams the thriftrw checksum payload through a slicing-by-8 CRC32 whose tables sit in LDS.
//
// Control flow restates the Go path exactly as oracle/state_builder_ref.cpp does (citations there
// and inline): service/history/execution/state_builder.go:90-648, mutable_state_builder.go,
// mutable_state_decision_task_manager.go, timer_sequence.go, common/persistence/versionHistory.go,
// workflowExecutionInfo.go and execution/checksum.go.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cadence_replay.h"

namespace crr {

using i64 = int64_t;
using i32 = int32_t;
using u32 = uint32_t;
using u64 = uint64_t;

constexpr i64 kSecond = 1000000000LL;

__device__ __forceinline__ i64 wadd(i64 a, i64 b) { return (i64)((u64)a + (u64)b); }
__device__ __forceinline__ i64 add_seconds(i64 t, i64 s) { return (i64)((u64)t + (u64)s * (u64)kSecond); }
__device__ __forceinline__ i64 unix_seconds(i64 ns) {
  i64 q = ns / kSecond;
  if ((ns % kSecond) < 0) --q;
  return q;
}

// ---------------------------------------------------------------------------------------------------
// CRC32-IEEE (hash/crc32.ChecksumIEEE, common/checksum/crc.go:46), slicing-by-8 over LDS tables.
struct Crc {
  const u32* T;  // 8 x 256 in LDS
  u32 crc;
  u64 buf;
  int nbuf;
  u32 len;

  __device__ __forceinline__ void init(const u32* tables) { T = tables; crc = 0xFFFFFFFFu; buf = 0; nbuf = 0; len = 0; }
  __device__ __forceinline__ void block8(u64 b) {
    u32 lo = (u32)b ^ crc;
    u32 hi = (u32)(b >> 32);
    crc = T[7 * 256 + (lo & 0xff)] ^ T[6 * 256 + ((lo >> 8) & 0xff)] ^ T[5 * 256 + ((lo >> 16) & 0xff)] ^
          T[4 * 256 + (lo >> 24)] ^ T[3 * 256 + (hi & 0xff)] ^ T[2 * 256 + ((hi >> 8) & 0xff)] ^
          T[1 * 256 + ((hi >> 16) & 0xff)] ^ T[0 * 256 + (hi >> 24)];
  }
  // push k (1..8) bytes held in arrival order in the low bytes of d
  __device__ __forceinline__ void push(u64 d, int k) {
    len += k;
    if (k < 8) d &= ((1ull << (8 * k)) - 1ull);
    if (nbuf + k < 8) {
      buf |= d << (8 * nbuf);
      nbuf += k;
      return;
    }
    int take = 8 - nbuf;
    u64 full = nbuf ? (buf | (d << (8 * nbuf))) : d;
    block8(full);
    int rem = k - take;
    buf = rem ? (d >> (8 * take)) : 0ull;
    nbuf = rem;
  }
  __device__ __forceinline__ void u8(u32 b) { push(b & 0xff, 1); }
  __device__ __forceinline__ void be16(u32 v) { push(((v >> 8) & 0xff) | ((v & 0xff) << 8), 2); }
  __device__ __forceinline__ void be32(u32 v) { push(__builtin_bswap32(v), 4); }
  __device__ __forceinline__ void be64(i64 v) { push(__builtin_bswap64((u64)v), 8); }
  // thrift binary WriteFieldBegin: type byte + big-endian i16 id
  __device__ __forceinline__ void field(u32 type, u32 id) { push(type | (((id >> 8) & 0xff) << 8) | ((id & 0xff) << 16), 3); }
  __device__ __forceinline__ void list_i64_header(u32 id, u32 n) {  // field(TLIST,id) + (TI64, n)
    field(15, id);
    push(10u | ((u64)__builtin_bswap32(n) << 8), 5);
  }
  __device__ __forceinline__ u32 finish() {
    for (int i = 0; i < nbuf; ++i) {
      u32 b = (u32)(buf >> (8 * i)) & 0xff;
      crc = T[(crc ^ b) & 0xff] ^ (crc >> 8);
    }
    nbuf = 0;
    return ~crc;
  }
};

__device__ void build_crc_tables(u32* T) {
  // table 0: byte-wise reflected CRC32 (poly 0xEDB88320); tables 1..7: slicing-by-8 extensions
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    u32 c = (u32)i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    T[i] = c;
  }
  __syncthreads();
  for (int t = 1; t < 8; ++t) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
      u32 p = T[(t - 1) * 256 + i];
      T[t * 256 + i] = (p >> 8) ^ T[p & 0xff];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------------
// Per-lane replay state: the numeric image of WorkflowExecutionInfo plus engine bookkeeping.
struct Lane {
  // execution info (persistence.WorkflowExecutionInfo)
  i32 state, close_status;
  i64 next_event_id, last_first_event_id, last_event_task_id, last_processed_event, completion_event_batch_id;
  i64 decision_version, decision_schedule_id, decision_started_id, decision_attempt;
  i64 decision_started_ts, decision_scheduled_ts, decision_orig_scheduled_ts;
  i32 decision_timeout, decision_request_src;
  i32 signal_count;
  i32 decision_start_to_close;  // DecisionStartToCloseTimeout
  i32 start_src;
  u32 flags;                    // CRR_EXEC_CANCEL_REQUESTED | CRR_EXEC_RESET_POINTS_SET
  i64 current_version;
  i64 now_ns;
  // version history: last item in registers, earlier items in the vh table
  i64 vh_last_id, vh_last_ver;
  i32 vh_n;
  i32 token_src;
  // slot-table occupancy: live counts and high-water marks
  i32 n_act, hw_act, n_timer, hw_timer, n_child, hw_child, n_rc, hw_rc, n_sig, hw_sig, n_rp;
  i32 inconsistencies;
  i32 status, fail_step;
};

struct Ctx {
  crr_inputs in;
  crr_outputs out;
  i64 st;  // stride
  // this workflow's slot-table bases / capacities
  i64 act_base, timer_base, child_base, rc_base, sig_base, vh_base, rp_base;
  i32 act_cap, timer_cap, child_cap, rc_cap, sig_cap, vh_cap, rp_cap;
  __device__ __forceinline__ crr_activity_row* act(i32 j) const { return out.act + act_base + (i64)j * st; }
  __device__ __forceinline__ crr_timer_row* timer(i32 j) const { return out.timer + timer_base + (i64)j * st; }
  __device__ __forceinline__ crr_child_row* child(i32 j) const { return out.child + child_base + (i64)j * st; }
  __device__ __forceinline__ crr_initiated_row* rc(i32 j) const { return out.rc + rc_base + (i64)j * st; }
  __device__ __forceinline__ crr_initiated_row* sig(i32 j) const { return out.sig + sig_base + (i64)j * st; }
  __device__ __forceinline__ crr_vh_item* vh(i32 j) const { return out.vh + vh_base + (i64)j * st; }
  __device__ __forceinline__ crr_reset_point_row* rp(i32 j) const { return out.rp + rp_base + (i64)j * st; }
};

// UpdateWorkflowStateCloseStatus (common/persistence/workflowExecutionInfo.go:45-165).
// Returns CRR_OK or the error code; on success the state is updated.
__device__ __forceinline__ int update_state(Lane& L, int state, int cs) {
  bool ok;
  switch (L.state) {
    case CRR_STATE_VOID:
      ok = true;
      break;
    case CRR_STATE_CREATED:
      if (state == CRR_STATE_COMPLETED)
        ok = cs == CRR_CLOSE_TERMINATED || cs == CRR_CLOSE_TIMED_OUT || cs == CRR_CLOSE_CONTINUED_AS_NEW;
      else if (state >= CRR_STATE_CREATED && state <= CRR_STATE_ZOMBIE)
        ok = cs == CRR_CLOSE_NONE;
      else
        return CRR_ERR_UNKNOWN_WORKFLOW_STATE;
      break;
    case CRR_STATE_RUNNING:
      if (state == CRR_STATE_CREATED) ok = false;
      else if (state == CRR_STATE_COMPLETED) ok = cs != CRR_CLOSE_NONE;
      else if (state == CRR_STATE_RUNNING || state == CRR_STATE_ZOMBIE) ok = cs == CRR_CLOSE_NONE;
      else return CRR_ERR_UNKNOWN_WORKFLOW_STATE;
      break;
    case CRR_STATE_COMPLETED:
      if (state == CRR_STATE_COMPLETED) ok = cs == L.close_status;
      else if (state >= CRR_STATE_CREATED && state <= CRR_STATE_ZOMBIE) ok = false;
      else return CRR_ERR_UNKNOWN_WORKFLOW_STATE;
      break;
    case CRR_STATE_ZOMBIE:
      if (state == CRR_STATE_CREATED || state == CRR_STATE_RUNNING) ok = cs == CRR_CLOSE_NONE;
      else if (state == CRR_STATE_COMPLETED || state == CRR_STATE_ZOMBIE) ok = cs != CRR_CLOSE_NONE;
      else return CRR_ERR_UNKNOWN_WORKFLOW_STATE;
      break;
    default:
      return CRR_ERR_UNKNOWN_WORKFLOW_STATE;
  }
  if (!ok) return CRR_ERR_INVALID_STATE_TRANSITION;
  L.state = state;
  L.close_status = cs;
  return CRR_OK;
}

// UpdateDecision (mutable_state_decision_task_manager.go:697-721)
__device__ __forceinline__ void update_decision(Lane& L, i64 ver, i64 sched, i64 started, i32 req_src, i32 timeout,
                                                i64 attempt, i64 started_ts, i64 sched_ts, i64 orig_ts) {
  L.decision_version = ver;
  L.decision_schedule_id = sched;
  L.decision_started_id = started;
  L.decision_request_src = req_src;
  L.decision_timeout = timeout;
  L.decision_attempt = attempt;
  L.decision_started_ts = started_ts;
  L.decision_scheduled_ts = sched_ts;
  L.decision_orig_scheduled_ts = orig_ts;
}

// FailDecision(true) (:643-676) followed by ReplicateTransientDecisionTaskScheduled (:168-197)
__device__ __forceinline__ void fail_decision_and_transient(Lane& L) {
  update_decision(L, CRR_EMPTY_VERSION, CRR_EMPTY_EVENT_ID, CRR_EMPTY_EVENT_ID, CRR_SRC_EMPTY_UUID, 0,
                  L.decision_attempt + 1, 0, L.now_ns, 0);
  // transient: !HasPendingDecision && DecisionAttempt != 0 -- always true right after FailDecision(true)
  if (L.decision_schedule_id == CRR_EMPTY_EVENT_ID && L.decision_attempt != 0)
    update_decision(L, L.current_version, L.next_event_id, CRR_EMPTY_EVENT_ID, CRR_SRC_EMPTY_UUID,
                    L.decision_start_to_close, L.decision_attempt, 0, L.now_ns, 0);
}

// ---- slot-table primitives ---------------------------------------------------------------------------
__device__ __forceinline__ i32 find_act_by_id(const Ctx& C, const Lane& L, i64 sched) {
  for (i32 j = 0; j < L.hw_act; ++j) {
    const crr_activity_row* r = C.act(j);
    if ((r->flags & CRR_ROW_LIVE) && r->schedule_id == sched) return j;
  }
  return -1;
}
// live activity whose ActivityID mapping points at it (pendingActivityIDToEventID[key])
__device__ __forceinline__ i32 find_act_mapped(const Ctx& C, const Lane& L, u32 key) {
  for (i32 j = 0; j < L.hw_act; ++j) {
    const crr_activity_row* r = C.act(j);
    u32 f = r->flags;
    if ((f & (CRR_ROW_LIVE | CRR_ROW_MAPPED)) == (CRR_ROW_LIVE | CRR_ROW_MAPPED) && r->key == key) return j;
  }
  return -1;
}
template <class R>
__device__ __forceinline__ i32 free_slot(R* (Ctx::*row)(i32) const, const Ctx& C, i32& hw, i32 cap) {
  for (i32 j = 0; j < hw; ++j)
    if (!((C.*row)(j)->flags & CRR_ROW_LIVE)) return j;
  if (hw >= cap) return -1;
  return hw++;
}
template <class R>
__device__ __forceinline__ i32 find_initiated(R* (Ctx::*row)(i32) const, const Ctx& C, i32 hw, i64 id) {
  for (i32 j = 0; j < hw; ++j) {
    const R* r = (C.*row)(j);
    if ((r->flags & CRR_ROW_LIVE) && r->initiated_id == id) return j;
  }
  return -1;
}
__device__ __forceinline__ i32 find_timer(const Ctx& C, const Lane& L, u32 key) {
  for (i32 j = 0; j < L.hw_timer; ++j) {
    const crr_timer_row* r = C.timer(j);
    if ((r->flags & CRR_ROW_LIVE) && r->key == key) return j;
  }
  return -1;
}

// DeleteActivity (mutable_state_builder.go:1310-1339)
__device__ __forceinline__ void delete_activity(const Ctx& C, Lane& L, i64 sched) {
  i32 j = find_act_by_id(C, L, sched);
  if (j < 0) { ++L.inconsistencies; return; }
  crr_activity_row* r = C.act(j);
  u32 f = r->flags;
  u32 key = r->key;
  r->flags = f & ~(CRR_ROW_LIVE | CRR_ROW_MAPPED);
  --L.n_act;
  if (f & CRR_ROW_MAPPED) return;  // delete(pendingActivityIDToEventID, ActivityID) removed our own mapping
  i32 m = find_act_mapped(C, L, key);  // the mapping of this ActivityID points at a newer activity
  if (m >= 0) C.act(m)->flags &= ~CRR_ROW_MAPPED;
  else ++L.inconsistencies;
}

// ---- timer sequence epilogue (timer_sequence.go:127-199, :219-381, :461-493) ---------------------------
__device__ __forceinline__ bool seq_less(i64 ta, i64 ea, i32 ya, i64 tb, i64 eb, i32 yb) {
  if (ta != tb) return ta < tb;
  if (ea != eb) return ea < eb;
  return ya < yb;
}

__device__ __forceinline__ void create_next_activity_timer(const Ctx& C, Lane& L) {
  if (L.n_act == 0) return;
  bool have = false;
  i64 bt = 0, be = 0;
  i32 by = 0, bj = -1;
  bool bc = false;
  for (i32 j = 0; j < L.hw_act; ++j) {
    const crr_activity_row* r = C.act(j);
    if (!(r->flags & CRR_ROW_LIVE)) continue;
    const i64 sid = r->schedule_id;
    if (sid == CRR_EMPTY_EVENT_ID) continue;
    const i32 tts = r->timer_task_status;
    const i64 sched_t = r->scheduled_time;
    const i64 started = r->started_id;
    // ScheduleToClose
    {
      i64 t = add_seconds(sched_t, r->schedule_to_close);
      if (!have || seq_less(t, sid, CRR_TIMEOUT_SCHEDULE_TO_CLOSE, bt, be, by)) {
        have = true; bt = t; be = sid; by = CRR_TIMEOUT_SCHEDULE_TO_CLOSE; bj = j; bc = (tts & CRR_TTS_CREATED_SCHEDULE_TO_CLOSE) != 0;
      }
    }
    if (started == CRR_EMPTY_EVENT_ID) {
      i64 t = add_seconds(sched_t, r->schedule_to_start);
      if (seq_less(t, sid, CRR_TIMEOUT_SCHEDULE_TO_START, bt, be, by)) {
        bt = t; be = sid; by = CRR_TIMEOUT_SCHEDULE_TO_START; bj = j; bc = (tts & CRR_TTS_CREATED_SCHEDULE_TO_START) != 0;
      }
    } else {
      const i64 st = r->started_time;
      i64 t = add_seconds(st, r->start_to_close);
      if (seq_less(t, sid, CRR_TIMEOUT_START_TO_CLOSE, bt, be, by)) {
        bt = t; be = sid; by = CRR_TIMEOUT_START_TO_CLOSE; bj = j; bc = (tts & CRR_TTS_CREATED_START_TO_CLOSE) != 0;
      }
      const i32 hb = r->heartbeat;
      if (hb > 0) {  // LastHeartBeatUpdatedTime == StartedTime on the replay path
        i64 th = add_seconds(st, hb);
        if (seq_less(th, sid, CRR_TIMEOUT_HEARTBEAT, bt, be, by)) {
          bt = th; be = sid; by = CRR_TIMEOUT_HEARTBEAT; bj = j; bc = (tts & CRR_TTS_CREATED_HEARTBEAT) != 0;
        }
      }
    }
  }
  if (!have || bc) return;
  crr_activity_row* r = C.act(bj);
  const i32 mask = by == CRR_TIMEOUT_START_TO_CLOSE ? CRR_TTS_CREATED_START_TO_CLOSE
                 : by == CRR_TIMEOUT_SCHEDULE_TO_START ? CRR_TTS_CREATED_SCHEDULE_TO_START
                 : by == CRR_TIMEOUT_SCHEDULE_TO_CLOSE ? CRR_TTS_CREATED_SCHEDULE_TO_CLOSE
                                                       : CRR_TTS_CREATED_HEARTBEAT;
  r->timer_task_status |= mask;
  if (by == CRR_TIMEOUT_HEARTBEAT) r->last_hb_timeout_vis_s = unix_seconds(bt);
}

__device__ __forceinline__ void create_next_user_timer(const Ctx& C, Lane& L) {
  if (L.n_timer == 0) return;
  bool have = false;
  i64 bt = 0, be = 0;
  i32 bj = -1;
  for (i32 j = 0; j < L.hw_timer; ++j) {
    const crr_timer_row* r = C.timer(j);
    if (!(r->flags & CRR_ROW_LIVE)) continue;
    i64 t = r->expiry_time, e = r->started_id;
    if (!have || seq_less(t, e, 0, bt, be, 0)) { have = true; bt = t; be = e; bj = j; }
  }
  if (!have) return;
  crr_timer_row* r = C.timer(bj);
  if (r->task_status == CRR_TIMER_TASK_STATUS_CREATED) return;
  r->task_status = CRR_TIMER_TASK_STATUS_CREATED;
}

// ---- end-of-replay compaction: live rows sorted by event ID into slots 0..n-1 ---------------------------
template <class R, int WORDS>
__device__ __forceinline__ void swap_rows(R* a, R* b) {
  u64* pa = reinterpret_cast<u64*>(a);
  u64* pb = reinterpret_cast<u64*>(b);
#pragma unroll
  for (int w = 0; w < WORDS; ++w) {
    u64 x = pa[w];
    pa[w] = pb[w];
    pb[w] = x;
  }
}

template <class R, class IdOf>
__device__ __forceinline__ void compact_sort(R* (Ctx::*row)(i32) const, const Ctx& C, i32 hw, i32 n, IdOf id_of) {
  for (i32 i = 0; i < n; ++i) {
    i32 best = -1;
    i64 bid = 0;
    for (i32 j = i; j < hw; ++j) {
      const R* r = (C.*row)(j);
      if (!(r->flags & CRR_ROW_LIVE)) continue;
      i64 id = id_of(r);
      if (best < 0 || id < bid) { best = j; bid = id; }
    }
    if (best != i) swap_rows<R, sizeof(R) / 8>((C.*row)(i), (C.*row)(best));
  }
}

// generateMutableStateChecksum (checksum.go:36-114) -> GenerateCRC32 (crc.go:35-54) over
// 0x59 + MutableStateChecksumPayload.Encode (.gen/go/checksum/checksum.go:539-821).  Reads the
// numeric execution image R and the sorted live rows (slots 0..n-1) of this workflow.
__device__ __forceinline__ u32 payload_crc(const crr_exec_row& R, const Ctx& C, const crr_workflow* wfp,
                                           const uint8_t* arena, const u32* tables, u32* out_len) {
  Crc K;
  K.init(tables);
  K.u8(0x59);                                                     // preambleVersion0
  K.field(2, 10); K.u8((R.flags & CRR_EXEC_CANCEL_REQUESTED) ? 1 : 0);   // CancelRequested
  K.field(6, 15); K.be16((u32)(uint16_t)(int16_t)R.state);              // State
  K.field(10, 23); K.be64(R.last_first_event_id);
  K.field(10, 24); K.be64(R.next_event_id);
  K.field(10, 25); K.be64(R.last_processed_event);
  K.field(10, 26); K.be64((i64)R.signal_count);
  K.field(8, 35); K.be32((u32)(i32)R.decision_attempt);
  K.field(10, 36); K.be64(R.decision_version);
  K.field(10, 37); K.be64(R.decision_schedule_id);
  K.field(10, 38); K.be64(R.decision_started_id);
  K.list_i64_header(45, (u32)R.n_timer);                          // PendingTimerStartedIDs
  for (i32 i = 0; i < R.n_timer; ++i) K.be64(C.timer(i)->started_id);
  K.list_i64_header(46, (u32)R.n_activity);                       // PendingActivityScheduledIDs
  for (i32 i = 0; i < R.n_activity; ++i) K.be64(C.act(i)->schedule_id);
  K.list_i64_header(47, (u32)R.n_signal);                         // PendingSignalInitiatedIDs
  for (i32 i = 0; i < R.n_signal; ++i) K.be64(C.sig(i)->initiated_id);
  K.list_i64_header(48, (u32)R.n_rc);                             // PendingReqCancelInitiatedIDs
  for (i32 i = 0; i < R.n_rc; ++i) K.be64(C.rc(i)->initiated_id);
  K.list_i64_header(49, (u32)R.n_child);                          // PendingChildInitiatedIDs
  for (i32 i = 0; i < R.n_child; ++i) K.be64(C.child(i)->initiated_id);
  K.field(11, 55); K.be32(0);                                     // StickyTaskListName ""
  K.field(12, 56);                                                // VersionHistories (shared.go:91639)
  K.field(8, 10); K.be32(0);                                      //   CurrentVersionHistoryIndex
  K.field(15, 20); K.push(12u | ((u64)__builtin_bswap32(1u) << 8), 5);  // list<struct>, 1 history
  u32 toff = 0, tlen = 0;
  if (R.token_src == 1) { toff = wfp->start_token_off; tlen = wfp->start_token_len; }
  if (R.token_src == 2) { toff = wfp->final_token_off; tlen = wfp->final_token_len; }
  K.field(11, 10); K.be32(tlen);                                  //   VersionHistory.BranchToken (shared.go:92043)
  {
    const uint8_t* tp = arena + toff;
    u32 i = 0;
    if ((toff & 7u) == 0) {
      const u64* tw = reinterpret_cast<const u64*>(tp);
      for (; i + 8 <= tlen; i += 8) K.push(tw[i >> 3], 8);
    }
    for (; i < tlen; ++i) K.u8(tp[i]);
  }
  K.field(15, 20); K.push(12u | ((u64)__builtin_bswap32((u32)R.n_vh_items) << 8), 5);
  for (i32 i = 0; i < R.n_vh_items; ++i) {                        //   VersionHistoryItem (shared.go:92375)
    const crr_vh_item* it = C.vh(i);
    K.field(10, 10); K.be64(it->event_id);
    K.field(10, 20); K.be64(it->version);
    K.u8(0);
  }
  K.u8(0);  // VersionHistory stop
  K.u8(0);  // VersionHistories stop
  K.u8(0);  // payload stop
  *out_len = K.len;
  return K.finish();
}

// ---- the kernel ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) replay_kernel(crr_inputs in, crr_outputs out, int phase) {
  __shared__ u32 crc_tables[8 * 256];
  build_crc_tables(crc_tables);

  const u32 w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= in.n_wf) return;
  const crr_workflow* wfp = in.wf + w;
  const i32 wflags = wfp->flags;
  if (((wflags & CRR_WF_FLAG_NEW_RUN) != 0) != (phase == 0)) return;

  Ctx C;
  C.in = in;
  C.out = out;
  C.st = in.stride;
  C.act_base = wfp->act_base; C.timer_base = wfp->timer_base; C.child_base = wfp->child_base;
  C.rc_base = wfp->rc_base; C.sig_base = wfp->sig_base; C.vh_base = wfp->vh_base; C.rp_base = wfp->rp_base;
  C.act_cap = wfp->act_cap; C.timer_cap = wfp->timer_cap; C.child_cap = wfp->child_cap; C.rc_cap = wfp->rc_cap;
  C.sig_cap = wfp->sig_cap; C.vh_cap = wfp->vh_cap; C.rp_cap = wfp->rp_cap;

  const i64 ev_begin = wfp->ev_begin;
  const i32 n_ev = wfp->ev_count;
  const i32 empty_at = wfp->empty_batch_at;

  // newMutableStateBuilder (mutable_state_builder.go:174-242) + NewMutableStateBuilderWithVersionHistories (:245-254)
  Lane L;
  L.state = CRR_STATE_CREATED; L.close_status = CRR_CLOSE_NONE;
  L.next_event_id = CRR_FIRST_EVENT_ID; L.last_first_event_id = 0; L.last_event_task_id = 0;
  L.last_processed_event = CRR_EMPTY_EVENT_ID; L.completion_event_batch_id = 0;
  L.decision_version = CRR_EMPTY_VERSION; L.decision_schedule_id = CRR_EMPTY_EVENT_ID;
  L.decision_started_id = CRR_EMPTY_EVENT_ID; L.decision_attempt = 0;
  L.decision_started_ts = 0; L.decision_scheduled_ts = 0; L.decision_orig_scheduled_ts = 0;
  L.decision_timeout = 0; L.decision_request_src = CRR_SRC_EMPTY_UUID;
  L.signal_count = 0; L.decision_start_to_close = 0; L.start_src = -1; L.flags = 0;
  L.current_version = wfp->init_version;
  L.now_ns = wfp->now_ns;
  L.vh_last_id = 0; L.vh_last_ver = 0; L.vh_n = 0; L.token_src = 0;
  L.n_act = L.hw_act = L.n_timer = L.hw_timer = L.n_child = L.hw_child = 0;
  L.n_rc = L.hw_rc = L.n_sig = L.hw_sig = L.n_rp = 0;
  L.inconsistencies = 0;
  L.status = CRR_OK; L.fail_step = -1;

  const uint8_t* __restrict__ col_type = in.ev.etype;
  const int64_t* __restrict__ col_id = in.ev.event_id;
  const int64_t* __restrict__ col_ver = in.ev.version;
  const int64_t* __restrict__ col_ts = in.ev.timestamp;
  const int64_t* __restrict__ col_task = in.ev.task_id;
  const int64_t* __restrict__ col_ref = in.ev.ref;
  const uint32_t* __restrict__ col_key = in.ev.key;
  const int32_t* __restrict__ col_aux = in.ev.aux;

  i64 batch_first_id = 0;
#define FAIL(code, step) do { L.status = (code); L.fail_step = (step); goto done_events; } while (0)

  for (i32 s = 0; s < n_ev; ++s) {
    if (s == empty_at) FAIL(CRR_ERR_EMPTY_HISTORY, s);  // state_builder.go:98-100
    const i64 ix = ev_begin + (i64)s * C.st;
    const u32 et = col_type[ix];
    const i64 id = col_id[ix];
    const i64 ver = col_ver[ix];
    const i32 t = et & CRR_ETYPE_MASK;
    if (et & CRR_ETYPE_BATCH_FIRST) batch_first_id = id;  // firstEvent := history[0] (:101)

    // :112 UpdateCurrentVersion(event.Version, true) (mutable_state_builder.go:495-533)
    if (L.state == CRR_STATE_COMPLETED) {
      if (L.vh_n == 0) FAIL(CRR_ERR_VH_EMPTY, s);
      L.current_version = L.vh_last_ver;
    } else {
      L.current_version = ver;
    }
    // :123-128 AddOrUpdateItem(NewVersionHistoryItem(event.ID, event.Version)) (versionHistory.go:32-46, :193-226)
    if (id < 0 || (ver < 0 && ver != CRR_EMPTY_VERSION)) FAIL(CRR_ERR_VH_INVALID_ITEM, s);
    if (L.vh_n == 0) {
      if (C.vh_cap < 1) FAIL(CRR_ERR_CAPACITY, s);
      L.vh_last_id = id; L.vh_last_ver = ver; L.vh_n = 1;
    } else if (ver < L.vh_last_ver) {
      FAIL(CRR_ERR_VH_LOWER_VERSION, s);
    } else if (id <= L.vh_last_id) {
      FAIL(CRR_ERR_VH_EVENT_ID_NOT_INCREASING, s);
    } else if (ver > L.vh_last_ver) {
      if (L.vh_n >= C.vh_cap) FAIL(CRR_ERR_CAPACITY, s);
      crr_vh_item* it = C.vh(L.vh_n - 1);
      it->event_id = L.vh_last_id;
      it->version = L.vh_last_ver;
      L.vh_last_id = id; L.vh_last_ver = ver; ++L.vh_n;
    } else {
      L.vh_last_id = id;
    }
    L.last_event_task_id = col_task[ix];  // :129

    switch (t) {
      case CRR_EV_WORKFLOW_EXECUTION_STARTED: {  // :132-183 -> mutable_state_builder.go:1751-1829
        const crr_start_side ss = in.start_side[col_aux[ix]];
        if (ss.parent_domain_status == CRR_DOMAIN_UNKNOWN) FAIL(CRR_ERR_DOMAIN_NOT_FOUND, s);
        L.decision_start_to_close = ss.decision_start_to_close;
        L.start_src = s;
        int e = update_state(L, CRR_STATE_CREATED, CRR_CLOSE_NONE);
        if (e) FAIL(e, s);
        L.last_processed_event = CRR_EMPTY_EVENT_ID;
        L.last_first_event_id = id;
        L.decision_version = CRR_EMPTY_VERSION;
        L.decision_schedule_id = CRR_EMPTY_EVENT_ID;
        L.decision_started_id = CRR_EMPTY_EVENT_ID;
        L.decision_request_src = CRR_SRC_EMPTY_UUID;
        L.decision_timeout = 0;
        // AutoResetPoints = rolloverAutoResetPointsWithExpiringTime(PrevAutoResetPoints, ...) (:3343-3364)
        L.n_rp = 0;
        L.flags = (L.flags & ~CRR_EXEC_RESET_POINTS_SET) | (ss.prev_reset_count != -1 ? CRR_EXEC_RESET_POINTS_SET : 0u);
        for (i32 i = 0; i < ss.prev_reset_count; ++i) {
          if (L.n_rp >= C.rp_cap) FAIL(CRR_ERR_CAPACITY, s);
          crr_reset_point_row* rp = C.rp(L.n_rp++);
          rp->src = s;
          rp->prev_index = i;
          rp->key = in.reset_keys[ss.prev_reset_key_off + i];
          rp->flags = CRR_ROW_LIVE;
        }
        // GenerateDelayedDecisionTasks (mutable_state_task_generator.go:242-281)
        if (ss.first_decision_backoff > 0 && ss.initiator != CRR_INITIATOR_NIL &&
            ss.initiator != CRR_INITIATOR_RETRY_POLICY && ss.initiator != CRR_INITIATOR_CRON)
          FAIL(CRR_ERR_BAD_INITIATOR, s);
        L.token_src = 1;  // SetHistoryTree(runID) (:367-376)
        break;
      }
      case CRR_EV_DECISION_TASK_SCHEDULED: {  // :185-208 -> decision_task_manager.go:129-166
        if (L.state != CRR_STATE_ZOMBIE) {
          int e = update_state(L, CRR_STATE_RUNNING, CRR_CLOSE_NONE);
          if (e) FAIL(e, s);
        }
        const i64 ts = col_ts[ix];
        update_decision(L, ver, id, CRR_EMPTY_EVENT_ID, CRR_SRC_EMPTY_UUID, col_aux[ix], col_ref[ix], 0, ts, ts);
        break;
      }
      case CRR_EV_DECISION_TASK_STARTED: {  // :210-228 -> decision_task_manager.go:199-242
        const i64 sched = col_ref[ix];
        if (sched != L.decision_schedule_id) FAIL(CRR_ERR_DECISION_NOT_FOUND, s);
        update_decision(L, ver, sched, id, s, L.decision_timeout, 0, col_ts[ix], L.decision_scheduled_ts,
                        L.decision_orig_scheduled_ts);
        break;
      }
      case CRR_EV_DECISION_TASK_COMPLETED: {  // :230-235 -> decision_task_manager.go:244-249, :827-838
        update_decision(L, CRR_EMPTY_VERSION, CRR_EMPTY_EVENT_ID, CRR_EMPTY_EVENT_ID, CRR_SRC_EMPTY_UUID, 0, 0, 0, 0,
                        L.decision_orig_scheduled_ts);  // DeleteDecision
        L.last_processed_event = col_ref[ix];
        const u32 key = col_key[ix];
        if (key != 0) {  // addBinaryCheckSumIfNotExists (mutable_state_builder.go:1911-1974)
          bool exists = false;
          for (i32 i = 0; i < L.n_rp; ++i)
            if (C.rp(i)->key == key) { exists = true; break; }
          if (!exists) {
            if (L.n_rp >= C.rp_cap) FAIL(CRR_ERR_CAPACITY, s);
            crr_reset_point_row* rp = C.rp(L.n_rp++);
            rp->src = s;
            rp->prev_index = -1;
            rp->key = key;
            const bool resettable = L.n_child == 0 && L.n_rc == 0 && L.n_sig == 0;  // CheckResettable (:1977-1994)
            rp->flags = CRR_ROW_LIVE | (resettable ? CRR_ROW_RESETTABLE : 0u);
            L.flags |= CRR_EXEC_RESET_POINTS_SET;
          }
        }
        break;
      }
      case CRR_EV_DECISION_TASK_TIMED_OUT:  // :237-259 (StickyTaskList == "": incrementAttempt)
      case CRR_EV_DECISION_TASK_FAILED:     // :261-281
        fail_decision_and_transient(L);
        break;
      case CRR_EV_ACTIVITY_TASK_SCHEDULED: {  // :283-295 -> mutable_state_builder.go:2142-2197
        const crr_activity_side as = in.act_side[col_aux[ix]];
        if (as.domain_status == CRR_DOMAIN_UNKNOWN) FAIL(CRR_ERR_DOMAIN_NOT_FOUND, s);
        const u32 key = col_key[ix];
        // pendingActivityIDToEventID[ActivityID] = ScheduleID: the previous mapping of this ID goes away
        i32 m = find_act_mapped(C, L, key);
        if (m >= 0) C.act(m)->flags &= ~CRR_ROW_MAPPED;
        i32 j = free_slot<crr_activity_row>(&Ctx::act, C, L.hw_act, C.act_cap);
        if (j < 0) FAIL(CRR_ERR_CAPACITY, s);
        crr_activity_row* r = C.act(j);
        r->schedule_id = id;
        r->version = ver;
        r->scheduled_batch_id = batch_first_id;
        r->scheduled_time = col_ts[ix];
        r->started_id = CRR_EMPTY_EVENT_ID;
        r->started_time = CRR_ZERO_TIME;
        r->cancel_request_id = CRR_EMPTY_EVENT_ID;
        r->last_hb_timeout_vis_s = 0;
        r->sched_src = s;
        r->started_src = -1;
        r->schedule_to_start = as.schedule_to_start;
        r->schedule_to_close = as.schedule_to_close;
        r->start_to_close = as.start_to_close;
        r->heartbeat = as.heartbeat;
        r->timer_task_status = CRR_TIMER_TASK_STATUS_NONE;
        r->key = key;
        r->flags = CRR_ROW_LIVE | CRR_ROW_MAPPED | (as.has_retry_policy ? CRR_ROW_HAS_RETRY : 0u);
        ++L.n_act;
        break;
      }
      case CRR_EV_ACTIVITY_TASK_STARTED: {  // :297-302 -> :2254-2276
        i32 j = find_act_by_id(C, L, col_ref[ix]);
        if (j < 0) FAIL(CRR_ERR_MISSING_ACTIVITY_INFO, s);
        crr_activity_row* r = C.act(j);
        r->version = ver;
        r->started_id = id;
        r->started_src = s;
        r->started_time = col_ts[ix];
        break;
      }
      case CRR_EV_ACTIVITY_TASK_COMPLETED:
      case CRR_EV_ACTIVITY_TASK_FAILED:
      case CRR_EV_ACTIVITY_TASK_TIMED_OUT:
      case CRR_EV_ACTIVITY_TASK_CANCELED:  // :304-337 -> DeleteActivity
        delete_activity(C, L, col_ref[ix]);
        break;
      case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED: {  // :325-330 -> :2444-2467
        i32 j = find_act_mapped(C, L, col_key[ix]);
        if (j >= 0) {
          crr_activity_row* r = C.act(j);
          r->version = ver;
          r->flags |= CRR_ROW_CANCEL_REQUESTED;
          r->cancel_request_id = id;
        }
        break;
      }
      case CRR_EV_TIMER_STARTED: {  // :342-347 -> :3057-3081
        const u32 key = col_key[ix];
        i32 j = find_timer(C, L, key);  // pendingTimerInfoIDs[TimerID] = ti replaces a live timer
        if (j < 0) {
          j = free_slot<crr_timer_row>(&Ctx::timer, C, L.hw_timer, C.timer_cap);
          if (j < 0) FAIL(CRR_ERR_CAPACITY, s);
          ++L.n_timer;
        }
        crr_timer_row* r = C.timer(j);
        r->started_id = id;
        r->version = ver;
        r->expiry_time = add_seconds(col_ts[ix], col_ref[ix]);
        r->task_status = CRR_TIMER_TASK_STATUS_NONE;
        r->key = key;
        r->src = s;
        r->flags = CRR_ROW_LIVE;
        break;
      }
      case CRR_EV_TIMER_FIRED:
      case CRR_EV_TIMER_CANCELED: {  // :349-361 -> DeleteUserTimer (:1390-1419)
        i32 j = find_timer(C, L, col_key[ix]);
        if (j < 0) { ++L.inconsistencies; break; }
        C.timer(j)->flags = 0;
        --L.n_timer;
        break;
      }
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED: {  // :366-381 -> :3417-3453
        if (col_aux[ix] == CRR_DOMAIN_UNKNOWN) FAIL(CRR_ERR_DOMAIN_NOT_FOUND, s);
        i32 j = free_slot<crr_child_row>(&Ctx::child, C, L.hw_child, C.child_cap);
        if (j < 0) FAIL(CRR_ERR_CAPACITY, s);
        crr_child_row* r = C.child(j);
        r->initiated_id = id;
        r->version = ver;
        r->initiated_batch_id = batch_first_id;
        r->started_id = CRR_EMPTY_EVENT_ID;
        r->src = s;
        r->started_src = -1;
        r->flags = CRR_ROW_LIVE;
        ++L.n_child;
        break;
      }
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED: {  // :390-395 -> :3485-3507
        i32 j = find_initiated<crr_child_row>(&Ctx::child, C, L.hw_child, col_ref[ix]);
        if (j < 0) FAIL(CRR_ERR_MISSING_CHILD_INFO, s);
        crr_child_row* r = C.child(j);
        r->started_id = id;
        r->started_src = s;
        break;
      }
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED: {  // DeletePendingChildExecution (:1160-1178)
        i32 j = find_initiated<crr_child_row>(&Ctx::child, C, L.hw_child, col_ref[ix]);
        if (j < 0) { ++L.inconsistencies; break; }
        C.child(j)->flags = 0;
        --L.n_child;
        break;
      }
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED:
      case CRR_EV_SIGNAL_EXTERNAL_INITIATED: {  // :432-447 / :463-478 -> :2760-2779 / :2883-2905
        const bool is_rc = t == CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED;
        i32 j = is_rc ? free_slot<crr_initiated_row>(&Ctx::rc, C, L.hw_rc, C.rc_cap)
                      : free_slot<crr_initiated_row>(&Ctx::sig, C, L.hw_sig, C.sig_cap);
        if (j < 0) FAIL(CRR_ERR_CAPACITY, s);
        crr_initiated_row* r = is_rc ? C.rc(j) : C.sig(j);
        r->initiated_id = id;
        r->version = ver;
        r->initiated_batch_id = batch_first_id;
        r->src = s;
        r->flags = CRR_ROW_LIVE;
        if (is_rc) ++L.n_rc; else ++L.n_sig;
        // Generate{RequestCancel,Signal}ExternalTasks -> getTargetDomainID (task_generator.go:556-559, :604-607)
        if (col_aux[ix] == CRR_DOMAIN_UNKNOWN) FAIL(CRR_ERR_DOMAIN_NOT_FOUND, s);
        break;
      }
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED:
      case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED: {  // DeletePendingRequestCancel (:1181-1199)
        i32 j = find_initiated<crr_initiated_row>(&Ctx::rc, C, L.hw_rc, col_ref[ix]);
        if (j < 0) { ++L.inconsistencies; break; }
        C.rc(j)->flags = 0;
        --L.n_rc;
        break;
      }
      case CRR_EV_SIGNAL_EXTERNAL_FAILED:
      case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED: {  // DeletePendingSignal (:1202-1220)
        i32 j = find_initiated<crr_initiated_row>(&Ctx::sig, C, L.hw_sig, col_ref[ix]);
        if (j < 0) { ++L.inconsistencies; break; }
        C.sig(j)->flags = 0;
        --L.n_sig;
        break;
      }
      case CRR_EV_WORKFLOW_EXECUTION_SIGNALED:  // :497-502 -> :3260-3267
        L.signal_count = (i32)((u32)L.signal_count + 1u);
        break;
      case CRR_EV_WORKFLOW_EXECUTION_CANCEL_REQUESTED:  // :504-509 -> :2688-2694
        L.flags |= CRR_EXEC_CANCEL_REQUESTED;
        break;
      case CRR_EV_WORKFLOW_EXECUTION_COMPLETED:
      case CRR_EV_WORKFLOW_EXECUTION_FAILED:
      case CRR_EV_WORKFLOW_EXECUTION_TIMED_OUT:
      case CRR_EV_WORKFLOW_EXECUTION_CANCELED:
      case CRR_EV_WORKFLOW_EXECUTION_TERMINATED: {  // :517-585 -> :2561-2733, :3225-3240
        const int cs = t == CRR_EV_WORKFLOW_EXECUTION_COMPLETED ? CRR_CLOSE_COMPLETED
                     : t == CRR_EV_WORKFLOW_EXECUTION_FAILED    ? CRR_CLOSE_FAILED
                     : t == CRR_EV_WORKFLOW_EXECUTION_TIMED_OUT ? CRR_CLOSE_TIMED_OUT
                     : t == CRR_EV_WORKFLOW_EXECUTION_CANCELED  ? CRR_CLOSE_CANCELED
                                                                : CRR_CLOSE_TERMINATED;
        int e = update_state(L, CRR_STATE_COMPLETED, cs);
        if (e) FAIL(e, s);
        L.completion_event_batch_id = batch_first_id;
        break;
      }
      case CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW: {  // :587-627 -> :3366-3382
        const i32 nr = col_aux[ix];
        if (nr >= 0) {
          if ((u32)nr >= in.n_wf) FAIL(CRR_ERR_NEW_RUN_MISSING, s);
          const int nst = out.exec[nr].status;  // written by the phase-0 launch
          if (nst != CRR_OK) FAIL(nst, s);
        }
        int e = update_state(L, CRR_STATE_COMPLETED, CRR_CLOSE_CONTINUED_AS_NEW);
        if (e) FAIL(e, s);
        L.completion_event_batch_id = batch_first_id;
        break;
      }
      case CRR_EV_REQUEST_CANCEL_ACTIVITY_TASK_FAILED:  // :339-340
      case CRR_EV_CANCEL_TIMER_FAILED:                  // :363-364
      case CRR_EV_MARKER_RECORDED:                      // :494-495
      case CRR_EV_UPSERT_WORKFLOW_SEARCH_ATTRIBUTES:    // :511-515 (map merge: host materialised)
        break;
      default:  // :629-630
        FAIL(CRR_ERR_UNKNOWN_EVENT_TYPE, s);
    }

    if (et & CRR_ETYPE_BATCH_LAST) {
      // :634-640 GenerateActivityTimerTasks / GenerateUserTimerTasks
      create_next_activity_timer(C, L);
      create_next_user_timer(C, L);
      // :642-643
      L.last_first_event_id = batch_first_id;
      L.next_event_id = id + 1;
    }
  }
  if (empty_at == n_ev) FAIL(CRR_ERR_EMPTY_HISTORY, n_ev);
  // rebuild finalisation (state_rebuilder.go:150-177)
  if (wfp->final_token_len != 0xFFFFFFFFu) {
    L.token_src = 2;
    if (L.vh_n == 0) FAIL(CRR_ERR_VH_EMPTY, n_ev);
    const i64 want_id = wfp->rebuild_last_event_id, want_ver = wfp->rebuild_last_event_version;
    if (want_id < 0 || (want_ver < 0 && want_ver != CRR_EMPTY_VERSION)) FAIL(CRR_ERR_VH_INVALID_ITEM, n_ev);
    if (L.vh_last_id != want_id || L.vh_last_ver != want_ver) FAIL(CRR_ERR_REBUILD_LAST_ITEM, n_ev);
  }
done_events:
#undef FAIL

  // ---- write back: VH tail item, sorted live rows, checksum, execution row ----
  if (L.vh_n > 0) {
    crr_vh_item* it = C.vh(L.vh_n - 1);
    it->event_id = L.vh_last_id;
    it->version = L.vh_last_ver;
  }
  compact_sort<crr_activity_row>(&Ctx::act, C, L.hw_act, L.n_act, [](const crr_activity_row* r) { return r->schedule_id; });
  compact_sort<crr_timer_row>(&Ctx::timer, C, L.hw_timer, L.n_timer, [](const crr_timer_row* r) { return r->started_id; });
  compact_sort<crr_child_row>(&Ctx::child, C, L.hw_child, L.n_child, [](const crr_child_row* r) { return r->initiated_id; });
  compact_sort<crr_initiated_row>(&Ctx::rc, C, L.hw_rc, L.n_rc, [](const crr_initiated_row* r) { return r->initiated_id; });
  compact_sort<crr_initiated_row>(&Ctx::sig, C, L.hw_sig, L.n_sig, [](const crr_initiated_row* r) { return r->initiated_id; });

  crr_exec_row R;
  R.status = L.status;
  R.fail_step = L.fail_step;
  R.inconsistencies = L.inconsistencies;
  R.flags = L.flags | (L.status == CRR_OK ? CRR_EXEC_CHECKSUM_VALID : 0u);
  R.state = L.state;
  R.close_status = L.close_status;
  R.signal_count = L.signal_count;
  R.decision_timeout = L.decision_timeout;
  R.next_event_id = L.next_event_id;
  R.last_first_event_id = L.last_first_event_id;
  R.last_event_task_id = L.last_event_task_id;
  R.last_processed_event = L.last_processed_event;
  R.completion_event_batch_id = L.completion_event_batch_id;
  R.decision_version = L.decision_version;
  R.decision_schedule_id = L.decision_schedule_id;
  R.decision_started_id = L.decision_started_id;
  R.decision_attempt = L.decision_attempt;
  R.decision_started_ts = L.decision_started_ts;
  R.decision_scheduled_ts = L.decision_scheduled_ts;
  R.decision_orig_scheduled_ts = L.decision_orig_scheduled_ts;
  R.current_version = L.current_version;
  R.decision_request_src = L.decision_request_src;
  R.start_src = L.start_src;
  R.n_activity = L.n_act;
  R.n_timer = L.n_timer;
  R.n_child = L.n_child;
  R.n_rc = L.n_rc;
  R.n_signal = L.n_sig;
  R.n_vh_items = L.vh_n;
  R.n_reset_points = L.n_rp;
  R.token_src = L.token_src;
  R.checksum = 0;
  R.payload_len = 0;
  R.reserved[0] = 0;
  R.reserved[1] = 0;
  if (L.status == CRR_OK) R.checksum = payload_crc(R, C, wfp, in.arena, crc_tables, &R.payload_len);
  out.exec[w] = R;
}

// Recompute checksums from already-written rows (mutable_state_builder.go:334-348 verify path).
__global__ void __launch_bounds__(256) checksum_kernel(crr_inputs in, crr_outputs out, u32* checksums) {
  __shared__ u32 crc_tables[8 * 256];
  build_crc_tables(crc_tables);
  const u32 w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= in.n_wf) return;
  const crr_workflow* wfp = in.wf + w;
  Ctx C;
  C.in = in;
  C.out = out;
  C.st = in.stride;
  C.act_base = wfp->act_base; C.timer_base = wfp->timer_base; C.child_base = wfp->child_base;
  C.rc_base = wfp->rc_base; C.sig_base = wfp->sig_base; C.vh_base = wfp->vh_base; C.rp_base = wfp->rp_base;
  const crr_exec_row R = out.exec[w];
  u32 len = 0;
  checksums[w] = payload_crc(R, C, wfp, in.arena, crc_tables, &len);
}

}  // namespace crr
