// replay_kernel.hip -- CDNA4 (gfx950) batched mutable-state replay.
//
// One lane replays one workflow: every workflow is an independent event-sourced state machine, so
// a wavefront advances 64 workflows in lock step.
//
// Two table policies share one state-machine body (replay_body<P>):
//   * LdsTables  (fast path, wave-interleaved layout): the pending activity / timer / child /
//     request-cancel / signal maps and the reset-point keys are indexed in LDS ([slot][lane] SoA,
//     bank-conflict free).  Every lookup, the per-batch timer epilogue and the checksum's sorted ID
//     lists are served from LDS; the HBM rows of the output tables are written (never read) during
//     replay and compacted once at the end.  Group-uniform bases live in SGPRs.  A workflow whose
//     live set outgrows its LDS slots stops with CRR_INTERNAL_RETRY and is replayed again by
//   * GlobalTables (any layout, unbounded): the same maps as slot tables in the HBM output rows.
//
// The column loads of step s+1 are issued before step s is processed (software pipeline).  The
// checksum streams the thriftrw payload through a slicing-by-8 CRC32 whose tables sit in LDS.
//
// Control flow restates the Go path exactly as oracle/state_builder_ref.cpp does (citations there
// and inline): service/history/execution/state_builder.go:90-648, mutable_state_builder.go,
// mutable_state_decision_task_manager.go, timer_sequence.go, common/persistence/versionHistory.go,
// workflowExecutionInfo.go and execution/checksum.go.

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "cadence_replay.h"

// Checksums: the LdsTables kernels (config 2's) keep their CRC tables in LDS; the compact tiers and
// the tail kernel, whose occupancy is LDS-limited, read the same tables from constant memory
// (kCrcGlobal).  The compact tiers write reset-point rows to HBM at push and keep only their keys in LDS.
// (Experiment variants measured and not kept are described in DESIGN.md §4; they are not in this source.)
#ifndef CRR_LDS_ACT
#define CRR_LDS_ACT 2
#endif
#ifndef CRR_LDS_TIMER
#define CRR_LDS_TIMER 2
#endif
#ifndef CRR_LDS_CHILD
#define CRR_LDS_CHILD 1
#endif
#ifndef CRR_LDS_RC
#define CRR_LDS_RC 1
#endif
#ifndef CRR_LDS_SIG
#define CRR_LDS_SIG 1
#endif
#ifndef CRR_LDS_RP
#define CRR_LDS_RP 2
#endif

namespace crr {

using i64 = int64_t;
using i32 = int32_t;
using u32 = uint32_t;
using u64 = uint64_t;

constexpr i64 kSecond = 1000000000LL;
constexpr int kBlock = 256;
constexpr int CRR_INTERNAL_RETRY = 200;  // LDS slots exhausted: replay again with GlobalTables
constexpr u32 kScratchHeader = 64;       // scratch[0], [1] = retry list counts; lists follow the header
constexpr u32 kScratchGate = 3;          // scratch[3]: big-segment blocks resident (tail_gate_kernel)
// Retry lists: list 0 (fast path -> big-arena wavefront pass) at scratch[64 + k], list 1 (big arena ->
// HBM-row wavefront pass) at scratch[64 + n_wf + k]; scratch holds >= 2 * n_wf + 64 words.
__device__ __forceinline__ u32 retry_slot(const crr_inputs& in, int list, u32 k) {
  return kScratchHeader + (list ? in.n_wf : 0u) + k;
}

__device__ __forceinline__ i64 add_seconds(i64 t, i64 s) { return (i64)((u64)t + (u64)s * (u64)kSecond); }
__device__ __forceinline__ i64 unix_seconds(i64 ns) {  // time.Time.Unix(): floor
  i64 q = ns / kSecond;
  if ((ns % kSecond) < 0) --q;
  return q;
}
__device__ __forceinline__ i64 uniform64(i64 v) {
  u32 lo = __builtin_amdgcn_readfirstlane((u32)(u64)v);
  u32 hi = __builtin_amdgcn_readfirstlane((u32)((u64)v >> 32));
  return (i64)(((u64)hi << 32) | lo);
}
__device__ __forceinline__ i32 uniform32(i32 v) { return (i32)__builtin_amdgcn_readfirstlane((u32)v); }

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
  __device__ __forceinline__ void list_header(u32 id, u32 elem, u32 n) {  // field(TLIST,id) + (elem type, n)
    field(15, id);
    push(elem | ((u64)__builtin_bswap32(n) << 8), 5);
  }
  __device__ __forceinline__ u32 finish() {
    for (int i = 0; i < nbuf; ++i) {
      u32 b = (u32)(buf >> (8 * i)) & 0xff;
      crc = T[(crc ^ b) & 0xff] ^ (crc >> 8);
    }
    nbuf = 0;
    return ~crc;
  }
  // kSpliceBytes bytes whose raw CRC (from a zero register) is `raw`: the bytes still buffered go in first, then
  // the register advances over kSpliceBytes zero bytes -- linear in the register: r -> sum of the columns of
  // kShiftSplice its set bits select -- and the bytes' own contribution is XORed in (the update is linear
  // over GF(2) in register and data together)
  __device__ __forceinline__ void splice(u32 raw);
};

// The same slicing-by-8 tables built at compile time in constant memory, for kernels that keep no CRC
// tables in LDS (their occupancy is LDS-limited): per-lane lookups are vector loads that hit the CU's
// L1 / the L2 (8 KB), a few hundred per workflow at its end.
struct CrcTab { u32 v[8 * 256]; };
constexpr CrcTab make_crc_tab() {
  CrcTab T{};
  for (u32 i = 0; i < 256; ++i) {
    u32 c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    T.v[i] = c;
  }
  for (int t = 1; t < 8; ++t)
    for (int i = 0; i < 256; ++i) {
      const u32 p = T.v[(t - 1) * 256 + i];
      T.v[t * 256 + i] = (p >> 8) ^ T.v[p & 0xff];
    }
  return T;
}
__constant__ CrcTab kCrcGlobal = make_crc_tab();

// the splice length: NewHistoryBranchToken's 96-byte HistoryBranch (tree and branch UUIDs, no ancestors)
constexpr u32 kSpliceBytes = 96;
struct ShiftCols { u32 v[32]; };
constexpr ShiftCols make_shift_cols() {   // column i: the register 1 << i advanced over kSpliceBytes zero bytes
  const CrcTab T = make_crc_tab();
  ShiftCols c{};
  for (int i = 0; i < 32; ++i) {
    u32 r = 1u << i;
    for (u32 k = 0; k < kSpliceBytes; ++k) r = T.v[r & 0xff] ^ (r >> 8);
    c.v[i] = r;
  }
  return c;
}
__constant__ ShiftCols kShiftSplice = make_shift_cols();

__device__ __forceinline__ void Crc::splice(u32 raw) {
  for (int i = 0; i < nbuf; ++i) {
    const u32 b = (u32)(buf >> (8 * i)) & 0xff;
    crc = T[(crc ^ b) & 0xff] ^ (crc >> 8);
  }
  nbuf = 0;
  buf = 0;
  u32 r = raw;
#pragma unroll
  for (int i = 0; i < 32; ++i) r ^= kShiftSplice.v[i] & (0u - ((crc >> i) & 1u));   // the column index is uniform
  crc = r;
  len += kSpliceBytes;
}

// crr_token_crc: a lane per workflow, the raw CRC of its start token (the constant tables, through the L1)
__global__ void __launch_bounds__(256) token_crc_kernel(crr_inputs in, u32* out) {
  const u32 w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= in.n_wf) return;
  const crr_workflow* wfp = in.wf + w;
  const u32 off = wfp->start_token_off, len = wfp->start_token_len;
  Crc K;
  K.init(kCrcGlobal.v);
  K.crc = 0u;
  const uint8_t* tp = in.arena + off;
  u32 i = 0;
  if ((off & 7u) == 0) {
    const u64* tw = reinterpret_cast<const u64*>(tp);
    for (; i + 8 <= len; i += 8) K.push(tw[i >> 3], 8);
  }
  for (; i < len; ++i) K.u8(tp[i]);
  out[w] = ~K.finish();
}

// NT: the block size when the launch fixes it (no read of the dispatch packet), 0: blockDim.x
template <int NT = 0>
__device__ void build_crc_tables(u32* T) {
  const int nt = NT ? NT : (int)blockDim.x;
  // table 0: byte-wise reflected CRC32 (poly 0xEDB88320); tables 1..7: slicing-by-8 extensions
  for (int i = threadIdx.x; i < 256; i += nt) {
    u32 c = (u32)i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    T[i] = c;
  }
  __syncthreads();
  for (int t = 1; t < 8; ++t) {
    for (int i = threadIdx.x; i < 256; i += nt) {
      u32 p = T[(t - 1) * 256 + i];
      T[t * 256 + i] = (p >> 8) ^ T[p & 0xff];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------------
// Per-lane replay state: the numeric image of WorkflowExecutionInfo plus engine bookkeeping.
struct Lane {
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
  i64 vh_last_id, vh_last_ver;
  i32 vh_n;
  i32 token_src;
  i32 n_act, n_timer, n_child, n_rc, n_sig, n_rp;
  i32 inconsistencies;
  i32 status, fail_step;
  i32 n_tasks;                  // transfer / timer tasks generated (CRR_IN_EMIT_TASKS)
  i64 expiration_ns;            // executionInfo.ExpirationTime (0: unset)
  i32 src_base;                 // provenance offset of this call's steps (the resumed row's src_next; 0 fresh)
};

// Where this lane's output rows live in HBM: row(table, slot) = base + slot * stride.
struct Geo {
  crr_outputs out;
  i64 st;
  i64 act_base, timer_base, child_base, rc_base, sig_base, vh_base, rp_base;
  i32 act_cap, timer_cap, child_cap, rc_cap, sig_cap, vh_cap, rp_cap;
  i64 task_base;
  i32 task_cap;
  __device__ __forceinline__ crr_activity_row* act(i32 j) const { return out.act + act_base + (i64)j * st; }
  __device__ __forceinline__ crr_task_row* task(i32 j) const { return out.tasks + task_base + (i64)j * st; }
  __device__ __forceinline__ crr_timer_row* timer(i32 j) const { return out.timer + timer_base + (i64)j * st; }
  __device__ __forceinline__ crr_child_row* child(i32 j) const { return out.child + child_base + (i64)j * st; }
  __device__ __forceinline__ crr_initiated_row* rc(i32 j) const { return out.rc + rc_base + (i64)j * st; }
  __device__ __forceinline__ crr_initiated_row* sig(i32 j) const { return out.sig + sig_base + (i64)j * st; }
  __device__ __forceinline__ crr_vh_item* vh(i32 j) const { return out.vh + vh_base + (i64)j * st; }
  __device__ __forceinline__ crr_reset_point_row* rp(i32 j) const { return out.rp + rp_base + (i64)j * st; }
};

__device__ __forceinline__ void load_geo(Geo& G, const crr_workflow* wfp, const crr_outputs& out, i64 stride) {
  G.out = out;
  G.st = stride;
  G.act_base = wfp->act_base; G.timer_base = wfp->timer_base; G.child_base = wfp->child_base;
  G.rc_base = wfp->rc_base; G.sig_base = wfp->sig_base; G.vh_base = wfp->vh_base; G.rp_base = wfp->rp_base;
  G.act_cap = wfp->act_cap; G.timer_cap = wfp->timer_cap; G.child_cap = wfp->child_cap; G.rc_cap = wfp->rc_cap;
  G.sig_cap = wfp->sig_cap; G.vh_cap = wfp->vh_cap; G.rp_cap = wfp->rp_cap;
  G.task_base = wfp->task_base; G.task_cap = wfp->task_cap;
}

// Wave-interleaved layout: every base is group_base + lane and every capacity is the group's.
// Moving the group-uniform part to SGPRs frees ~20 VGPRs per lane.
__device__ __forceinline__ void uniformize_geo(Geo& G, i64 lane) {
  G.act_base = uniform64(G.act_base - lane) + lane;
  G.timer_base = uniform64(G.timer_base - lane) + lane;
  G.child_base = uniform64(G.child_base - lane) + lane;
  G.rc_base = uniform64(G.rc_base - lane) + lane;
  G.sig_base = uniform64(G.sig_base - lane) + lane;
  G.vh_base = uniform64(G.vh_base - lane) + lane;
  G.rp_base = uniform64(G.rp_base - lane) + lane;
  G.act_cap = uniform32(G.act_cap); G.timer_cap = uniform32(G.timer_cap); G.child_cap = uniform32(G.child_cap);
  G.rc_cap = uniform32(G.rc_cap); G.sig_cap = uniform32(G.sig_cap); G.vh_cap = uniform32(G.vh_cap);
  G.rp_cap = uniform32(G.rp_cap);
  G.task_base = uniform64(G.task_base - lane) + lane;
  G.task_cap = uniform32(G.task_cap);
}

// UpdateWorkflowStateCloseStatus (common/persistence/workflowExecutionInfo.go:45-165).
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
__device__ __forceinline__ bool fail_decision_and_transient(Lane& L, i64 now_ns) {
  update_decision(L, CRR_EMPTY_VERSION, CRR_EMPTY_EVENT_ID, CRR_EMPTY_EVENT_ID, CRR_SRC_EMPTY_UUID, 0,
                  L.decision_attempt + 1, 0, now_ns, 0);
  if (L.decision_schedule_id == CRR_EMPTY_EVENT_ID && L.decision_attempt != 0) {
    update_decision(L, L.current_version, L.next_event_id, CRR_EMPTY_EVENT_ID, CRR_SRC_EMPTY_UUID,
                    L.decision_start_to_close, L.decision_attempt, 0, now_ns, 0);
    return true;
  }
  return false;
}

// One transfer / timer task (crr_task_row) of the task generator, in the order Go adds them; the
// wavefront-per-workflow path writes it from one lane.
struct TaskSink {
  bool on;      // CRR_IN_EMIT_TASKS (uniform)
  bool writer;  // this lane writes the row
  __device__ __forceinline__ void add(Lane& L, const Geo& G, i32 kind, i32 aux, i64 version, i64 vis, i64 event_id,
                                      i32 attempt, i32 src) const {
    if (!on) return;
    if (writer && L.n_tasks < G.task_cap) {
      crr_task_row r;
      r.kind = kind; r.aux = aux; r.version = version; r.visibility_ts = vis; r.event_id = event_id;
      r.attempt = attempt; r.src = src;
      *G.task(L.n_tasks) = r;
    }
    ++L.n_tasks;
  }
};

__device__ __forceinline__ bool seq_less(i64 ta, i64 ea, i32 ya, i64 tb, i64 eb, i32 yb) {
  if (ta != tb) return ta < tb;
  if (ea != eb) return ea < eb;
  return ya < yb;
}
__device__ __forceinline__ u32 timer_mask(i32 type) {  // TimerTypeToTimerMask (timer_sequence.go:384-400)
  return type == CRR_TIMEOUT_START_TO_CLOSE ? CRR_TTS_CREATED_START_TO_CLOSE
       : type == CRR_TIMEOUT_SCHEDULE_TO_START ? CRR_TTS_CREATED_SCHEDULE_TO_START
       : type == CRR_TIMEOUT_SCHEDULE_TO_CLOSE ? CRR_TTS_CREATED_SCHEDULE_TO_CLOSE
                                               : CRR_TTS_CREATED_HEARTBEAT;
}

// Candidate timers of one pending activity (timer_sequence.go:269-381) folded into a running min.
struct BestTimer {
  bool have = false;
  i64 t = 0, e = 0;
  i32 y = 0, j = -1;
  bool created = false;
  __device__ __forceinline__ void offer(i64 tt, i64 ee, i32 yy, i32 jj, bool cc) {
    if (!have || seq_less(tt, ee, yy, t, e, y)) { have = true; t = tt; e = ee; y = yy; j = jj; created = cc; }
  }
};
// hb_t: max(StartedTime, LastHeartBeatUpdatedTime) (getActivityHeartbeatTimeout, timer_sequence.go:345-381)
__device__ __forceinline__ void activity_candidates(BestTimer& B, i32 j, i64 sid, i64 sched_t, bool started,
                                                    i64 start_t, i64 hb_t, i32 s2s, i32 s2c, i32 st2c, i32 hb, u32 tts) {
  if (sid == CRR_EMPTY_EVENT_ID) return;
  B.offer(add_seconds(sched_t, s2c), sid, CRR_TIMEOUT_SCHEDULE_TO_CLOSE, j, (tts & CRR_TTS_CREATED_SCHEDULE_TO_CLOSE) != 0);
  if (!started) {
    B.offer(add_seconds(sched_t, s2s), sid, CRR_TIMEOUT_SCHEDULE_TO_START, j, (tts & CRR_TTS_CREATED_SCHEDULE_TO_START) != 0);
  } else {
    B.offer(add_seconds(start_t, st2c), sid, CRR_TIMEOUT_START_TO_CLOSE, j, (tts & CRR_TTS_CREATED_START_TO_CLOSE) != 0);
    if (hb > 0) B.offer(add_seconds(hb_t, hb), sid, CRR_TIMEOUT_HEARTBEAT, j, (tts & CRR_TTS_CREATED_HEARTBEAT) != 0);
  }
}

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

// ===================================================================================================
// GlobalTables: pending maps as slot tables in the HBM output rows (any layout, unbounded).
// ===================================================================================================
// One event's fields.  The transitions read them through accessors: the lane path holds them in
// registers (Ev), the wavefront path reads each one out of the 64-event chunk only where a transition
// uses it (WaveEv, below).
struct Ev {
  u32 et;
  i64 id_, ver_, ts_, task_, ref_;
  u32 key_;
  i32 aux_;
  __device__ __forceinline__ i64 id() const { return id_; }
  __device__ __forceinline__ i64 ver() const { return ver_; }
  __device__ __forceinline__ i64 ts() const { return ts_; }
  __device__ __forceinline__ i64 task() const { return task_; }
  __device__ __forceinline__ i64 ref() const { return ref_; }
  __device__ __forceinline__ u32 key() const { return key_; }
  __device__ __forceinline__ i32 aux() const { return aux_; }
};

// The rows each insert writes (mutable_state_builder.go:2142-2197, :3057-3081, :3417-3453, :2760-2779, :2883-2905)
template <class EV>
__device__ __forceinline__ crr_activity_row activity_row(const EV& ev, i32 s, i64 batch_first_id,
                                                         const crr_activity_side& as) {
  crr_activity_row row;
  row.schedule_id = ev.id();
  row.version = ev.ver();
  row.scheduled_batch_id = batch_first_id;
  row.scheduled_time = ev.ts();
  row.started_id = CRR_EMPTY_EVENT_ID;
  row.started_time = CRR_ZERO_TIME;
  row.cancel_request_id = CRR_EMPTY_EVENT_ID;
  row.last_hb_timeout_vis_s = 0;
  row.sched_src = s;
  row.started_src = -1;
  row.schedule_to_start = as.schedule_to_start;
  row.schedule_to_close = as.schedule_to_close;
  row.start_to_close = as.start_to_close;
  row.heartbeat = as.heartbeat;
  row.timer_task_status = CRR_TIMER_TASK_STATUS_NONE;
  row.key = ev.key();
  row.flags = CRR_ROW_LIVE | CRR_ROW_MAPPED | (as.has_retry_policy ? CRR_ROW_HAS_RETRY : 0u);
  row.attempt = 0;
  row.last_heartbeat_time = CRR_ZERO_TIME;
  return row;
}
template <class EV>
__device__ __forceinline__ crr_timer_row timer_row(const EV& ev, i32 s) {
  crr_timer_row row;
  row.started_id = ev.id();
  row.version = ev.ver();
  row.expiry_time = add_seconds(ev.ts(), ev.ref());
  row.task_status = CRR_TIMER_TASK_STATUS_NONE;
  row.key = ev.key();
  row.src = s;
  row.flags = CRR_ROW_LIVE;
  return row;
}
template <class EV>
__device__ __forceinline__ crr_child_row child_row(const EV& ev, i32 s, i64 batch_first_id) {
  crr_child_row row;
  row.initiated_id = ev.id();
  row.version = ev.ver();
  row.initiated_batch_id = batch_first_id;
  row.started_id = CRR_EMPTY_EVENT_ID;
  row.src = s;
  row.started_src = -1;
  row.flags = CRR_ROW_LIVE;
  row.reserved = 0;
  return row;
}
template <class EV>
__device__ __forceinline__ crr_initiated_row initiated_row(const EV& ev, i32 s, i64 batch_first_id) {
  crr_initiated_row row;
  row.initiated_id = ev.id();
  row.version = ev.ver();
  row.initiated_batch_id = batch_first_id;
  row.src = s;
  row.flags = CRR_ROW_LIVE;
  return row;
}

enum : u32 {
  MOP_NONE = 0,
  MOP_ACT_INSERT, MOP_ACT_START, MOP_ACT_DELETE, MOP_ACT_CANCEL,  // ReplicateActivityTask* / DeleteActivity
  MOP_TIMER_START, MOP_TIMER_DELETE,                             // ReplicateTimerStarted / DeleteUserTimer
  MOP_CHILD_INSERT, MOP_CHILD_START, MOP_CHILD_DELETE,
  MOP_RC_INSERT, MOP_RC_DELETE, MOP_SIG_INSERT, MOP_SIG_DELETE
};
// The map operation of each event type (0: none), 4 bits per type
constexpr u32 mop_of(int t) {
  return t == CRR_EV_ACTIVITY_TASK_SCHEDULED ? MOP_ACT_INSERT
       : t == CRR_EV_ACTIVITY_TASK_STARTED ? MOP_ACT_START
       : (t == CRR_EV_ACTIVITY_TASK_COMPLETED || t == CRR_EV_ACTIVITY_TASK_FAILED || t == CRR_EV_ACTIVITY_TASK_TIMED_OUT ||
          t == CRR_EV_ACTIVITY_TASK_CANCELED) ? MOP_ACT_DELETE
       : t == CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED ? MOP_ACT_CANCEL
       : t == CRR_EV_TIMER_STARTED ? MOP_TIMER_START
       : (t == CRR_EV_TIMER_FIRED || t == CRR_EV_TIMER_CANCELED) ? MOP_TIMER_DELETE
       : t == CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED ? MOP_CHILD_INSERT
       : t == CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED ? MOP_CHILD_START
       : (t == CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED || (t >= CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED &&
          t <= CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED)) ? MOP_CHILD_DELETE
       : t == CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED ? MOP_RC_INSERT
       : (t == CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED || t == CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED) ? MOP_RC_DELETE
       : t == CRR_EV_SIGNAL_EXTERNAL_INITIATED ? MOP_SIG_INSERT
       : (t == CRR_EV_SIGNAL_EXTERNAL_FAILED || t == CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED) ? MOP_SIG_DELETE
       : MOP_NONE;
}
constexpr u64 mop_word(int w) {
  u64 v = 0;
  for (int k = 0; k < 16; ++k) v |= (u64)mop_of(16 * w + k) << (4 * k);
  return v;
}

struct GlobalTables {
  static constexpr bool kResumable = true;  // rows live in HBM: a loaded state is continued in place
  __device__ __forceinline__ static bool fits(i64) { return true; }
  i32 hw_act = 0, hw_timer = 0, hw_child = 0, hw_rc = 0, hw_sig = 0;
  // a map changed since its last batch epilogue (an unchanged one would reselect the same created
  // timer: a no-op, skipped -- each skipped pass is a scan of HBM rows)
  bool dirty_act = false, dirty_timer = false;

  template <class R>
  __device__ __forceinline__ static i32 free_slot(R* (Geo::*row)(i32) const, const Geo& G, i32& hw, i32 cap) {
    for (i32 j = 0; j < hw; ++j)
      if (!((G.*row)(j)->flags & CRR_ROW_LIVE)) return j;
    if (hw >= cap) return -1;
    return hw++;
  }
  template <class R>
  __device__ __forceinline__ static i32 find_initiated(R* (Geo::*row)(i32) const, const Geo& G, i32 hw, i64 id) {
    for (i32 j = 0; j < hw; ++j) {
      const R* r = (G.*row)(j);
      if ((r->flags & CRR_ROW_LIVE) && r->initiated_id == id) return j;
    }
    return -1;
  }
  __device__ __forceinline__ i32 find_act_by_id(const Geo& G, i64 sched) const {
    for (i32 j = 0; j < hw_act; ++j) {
      const crr_activity_row* r = G.act(j);
      if ((r->flags & CRR_ROW_LIVE) && r->schedule_id == sched) return j;
    }
    return -1;
  }
  __device__ __forceinline__ i32 find_act_mapped(const Geo& G, u32 key) const {
    for (i32 j = 0; j < hw_act; ++j) {
      const crr_activity_row* r = G.act(j);
      if ((r->flags & (CRR_ROW_LIVE | CRR_ROW_MAPPED)) == (CRR_ROW_LIVE | CRR_ROW_MAPPED) && r->key == key) return j;
    }
    return -1;
  }
  __device__ __forceinline__ i32 find_timer(const Geo& G, u32 key) const {
    for (i32 j = 0; j < hw_timer; ++j) {
      const crr_timer_row* r = G.timer(j);
      if ((r->flags & CRR_ROW_LIVE) && r->key == key) return j;
    }
    return -1;
  }

  // ReplicateActivityTaskScheduledEvent (mutable_state_builder.go:2142-2197)
  __device__ __forceinline__ int act_insert(Lane& L, const Geo& G, const crr_activity_row& row) {
    i32 m = find_act_mapped(G, row.key);  // pendingActivityIDToEventID[ActivityID] is overwritten
    if (m >= 0) G.act(m)->flags &= ~CRR_ROW_MAPPED;
    i32 j = free_slot<crr_activity_row>(&Geo::act, G, hw_act, G.act_cap);
    if (j < 0) return CRR_ERR_CAPACITY;
    *G.act(j) = row;
    ++L.n_act;
    dirty_act = true;
    return CRR_OK;
  }
  // ReplicateActivityTaskStartedEvent (:2254-2276)
  __device__ __forceinline__ int act_start(Lane& L, const Geo& G, i64 sched, i64 id, i64 ver, i32 s, i64 ts) {
    i32 j = find_act_by_id(G, sched);
    if (j < 0) return CRR_ERR_MISSING_ACTIVITY_INFO;
    crr_activity_row* r = G.act(j);
    dirty_act = true;
    r->version = ver;
    r->started_id = id;
    r->started_src = s;
    r->started_time = ts;
    r->last_heartbeat_time = ts;  // LastHeartBeatUpdatedTime = StartedTime (:2272-2273)
    return CRR_OK;
  }
  // DeleteActivity (:1310-1339)
  __device__ __forceinline__ void act_delete(Lane& L, const Geo& G, i64 sched) {
    i32 j = find_act_by_id(G, sched);
    if (j < 0) { ++L.inconsistencies; return; }
    crr_activity_row* r = G.act(j);
    u32 f = r->flags;
    u32 key = r->key;
    r->flags = f & ~(CRR_ROW_LIVE | CRR_ROW_MAPPED);
    --L.n_act;
    dirty_act = true;
    if (f & CRR_ROW_MAPPED) return;
    i32 m = find_act_mapped(G, key);
    if (m >= 0) G.act(m)->flags &= ~CRR_ROW_MAPPED;
    else ++L.inconsistencies;
  }
  // ReplicateActivityTaskCancelRequestedEvent (:2444-2467)
  __device__ __forceinline__ void act_cancel(Lane& L, const Geo& G, u32 key, i64 id, i64 ver, i32 /*s*/) {
    i32 j = find_act_mapped(G, key);
    if (j < 0) return;
    crr_activity_row* r = G.act(j);
    r->version = ver;
    r->flags |= CRR_ROW_CANCEL_REQUESTED;
    r->cancel_request_id = id;
  }
  // ReplicateTimerStartedEvent (:3057-3081)
  __device__ __forceinline__ int timer_start(Lane& L, const Geo& G, const crr_timer_row& row) {
    i32 j = find_timer(G, row.key);
    if (j < 0) {
      j = free_slot<crr_timer_row>(&Geo::timer, G, hw_timer, G.timer_cap);
      if (j < 0) return CRR_ERR_CAPACITY;
      ++L.n_timer;
    }
    *G.timer(j) = row;
    dirty_timer = true;
    return CRR_OK;
  }
  // DeleteUserTimer (:1390-1419)
  __device__ __forceinline__ void timer_delete(Lane& L, const Geo& G, u32 key) {
    i32 j = find_timer(G, key);
    if (j < 0) { ++L.inconsistencies; return; }
    G.timer(j)->flags = 0;
    --L.n_timer;
    dirty_timer = true;
  }
  // ReplicateStartChildWorkflowExecutionInitiatedEvent (:3417-3453)
  __device__ __forceinline__ int child_insert(Lane& L, const Geo& G, const crr_child_row& row) {
    i32 j = free_slot<crr_child_row>(&Geo::child, G, hw_child, G.child_cap);
    if (j < 0) return CRR_ERR_CAPACITY;
    *G.child(j) = row;
    ++L.n_child;
    return CRR_OK;
  }
  __device__ __forceinline__ int child_start(Lane& L, const Geo& G, i64 init, i64 id, i32 s) {
    i32 j = find_initiated<crr_child_row>(&Geo::child, G, hw_child, init);
    if (j < 0) return CRR_ERR_MISSING_CHILD_INFO;
    crr_child_row* r = G.child(j);
    r->started_id = id;
    r->started_src = s;
    return CRR_OK;
  }
  __device__ __forceinline__ void child_delete(Lane& L, const Geo& G, i64 init) {
    i32 j = find_initiated<crr_child_row>(&Geo::child, G, hw_child, init);
    if (j < 0) { ++L.inconsistencies; return; }
    G.child(j)->flags = 0;
    --L.n_child;
  }
  __device__ __forceinline__ int init_insert(Lane& L, const Geo& G, bool is_rc, const crr_initiated_row& row) {
    i32 j = is_rc ? free_slot<crr_initiated_row>(&Geo::rc, G, hw_rc, G.rc_cap)
                  : free_slot<crr_initiated_row>(&Geo::sig, G, hw_sig, G.sig_cap);
    if (j < 0) return CRR_ERR_CAPACITY;
    *(is_rc ? G.rc(j) : G.sig(j)) = row;
    if (is_rc) ++L.n_rc; else ++L.n_sig;
    return CRR_OK;
  }
  __device__ __forceinline__ void init_delete(Lane& L, const Geo& G, bool is_rc, i64 init) {
    i32 j = is_rc ? find_initiated<crr_initiated_row>(&Geo::rc, G, hw_rc, init)
                  : find_initiated<crr_initiated_row>(&Geo::sig, G, hw_sig, init);
    if (j < 0) { ++L.inconsistencies; return; }
    (is_rc ? G.rc(j) : G.sig(j))->flags = 0;
    if (is_rc) --L.n_rc; else --L.n_sig;
  }
  // mutableStateBuilder.Load (mutable_state_builder.go:306-349) over the loaded rows in slots 0..n-1:
  // pendingActivityIDToEventID[ActivityID] = ScheduleID for every activity (:311-314; among duplicate
  // ActivityIDs Go's map order picks one: here the latest scheduled), every row live
  __device__ __forceinline__ void load(Lane& L, const Geo& G) {
    hw_act = L.n_act; hw_timer = L.n_timer; hw_child = L.n_child; hw_rc = L.n_rc; hw_sig = L.n_sig;
    dirty_act = dirty_timer = true;  // the loaded state's timer masks are re-examined by the first epilogue
    // the ActivityID map (Load: the latest ScheduleID of each ActivityID wins): a 64-bit filter over the
    // keys finds the rows whose ActivityID may repeat; only those compare against the other rows
    u64 seen = 0, dup = 0;
    for (i32 j = 0; j < hw_act; ++j) {
      const u64 b = 1ull << (G.act(j)->key & 63u);
      dup |= seen & b;
      seen |= b;
    }
    for (i32 j = 0; j < hw_act; ++j) {
      crr_activity_row* r = G.act(j);
      const u32 key = r->key;
      const i64 sid = r->schedule_id;
      bool mapped = true;
      if (dup & (1ull << (key & 63u)))
        for (i32 k = 0; k < hw_act; ++k) {
          const crr_activity_row* o = G.act(k);
          if (k != j && o->key == key && o->schedule_id > sid) mapped = false;
        }
      r->flags = (r->flags & ~CRR_ROW_MAPPED) | CRR_ROW_LIVE | (mapped ? CRR_ROW_MAPPED : 0u);
    }
    for (i32 j = 0; j < hw_timer; ++j) G.timer(j)->flags |= CRR_ROW_LIVE;
    for (i32 j = 0; j < hw_child; ++j) G.child(j)->flags |= CRR_ROW_LIVE;
    for (i32 j = 0; j < hw_rc; ++j) G.rc(j)->flags |= CRR_ROW_LIVE;
    for (i32 j = 0; j < hw_sig; ++j) G.sig(j)->flags |= CRR_ROW_LIVE;
  }
  // reset points: rows in HBM, append-only
  __device__ __forceinline__ void rp_reset(Lane& L) { L.n_rp = 0; }
  __device__ __forceinline__ int rp_push(Lane& L, const Geo& G, const crr_reset_point_row& row) {
    if (L.n_rp >= G.rp_cap) return CRR_ERR_CAPACITY;
    *G.rp(L.n_rp++) = row;
    return CRR_OK;
  }
  __device__ __forceinline__ bool rp_has(const Lane& L, const Geo& G, u32 key) const {
    for (i32 i = 0; i < L.n_rp; ++i)
      if (G.rp(i)->key == key) return true;
    return false;
  }
  // CreateNextActivityTimer / CreateNextUserTimer (timer_sequence.go:127-199)
  __device__ __forceinline__ void epilogue(Lane& L, const Geo& G, const TaskSink& K) {
    if (L.n_act > 0 && dirty_act) {
      BestTimer B;
      for (i32 j = 0; j < hw_act; ++j) {
        const crr_activity_row* r = G.act(j);
        if (!(r->flags & CRR_ROW_LIVE)) continue;
        activity_candidates(B, j, r->schedule_id, r->scheduled_time, r->started_id != CRR_EMPTY_EVENT_ID,
                            r->started_time, max(r->started_time, r->last_heartbeat_time), r->schedule_to_start,
                            r->schedule_to_close, r->start_to_close,
                            r->heartbeat, (u32)r->timer_task_status);
      }
      if (B.have && !B.created) {
        crr_activity_row* r = G.act(B.j);
        r->timer_task_status |= timer_mask(B.y);
        if (B.y == CRR_TIMEOUT_HEARTBEAT) r->last_hb_timeout_vis_s = unix_seconds(B.t);
        K.add(L, G, CRR_TASK_ACTIVITY_TIMEOUT, B.y, L.current_version, B.t, B.e, r->attempt, -1);  // timer_sequence.go:190-196
      }
    }
    dirty_act = false;
    epilogue_timers(L, G, K);
  }
  // RefreshTasks' state effects (mutable_state_task_refresher.go:278-365)
  __device__ __forceinline__ void refresh(Lane& L, const Geo& G) {
    for (i32 j = 0; j < hw_act; ++j) G.act(j)->timer_task_status = CRR_TIMER_TASK_STATUS_NONE;
    for (i32 j = 0; j < hw_timer; ++j) G.timer(j)->task_status = CRR_TIMER_TASK_STATUS_NONE;
    dirty_act = dirty_timer = true;
    epilogue(L, G, TaskSink{false, false});
  }
  __device__ __forceinline__ void epilogue_timers(Lane& L, const Geo& G, const TaskSink& K) {
    if (L.n_timer > 0 && dirty_timer) {
      BestTimer B;
      for (i32 j = 0; j < hw_timer; ++j) {
        const crr_timer_row* r = G.timer(j);
        if (!(r->flags & CRR_ROW_LIVE)) continue;
        B.offer(r->expiry_time, r->started_id, 0, j, r->task_status == CRR_TIMER_TASK_STATUS_CREATED);
      }
      if (B.have && !B.created) {
        G.timer(B.j)->task_status = CRR_TIMER_TASK_STATUS_CREATED;
        K.add(L, G, CRR_TASK_USER_TIMER, 0, L.current_version, B.t, B.e, 0, -1);  // timer_sequence.go:151-156
      }
    }
    dirty_timer = false;
  }
  __device__ __forceinline__ bool task_writer() const { return true; }
  template <class R, class IdOf>
  __device__ __forceinline__ static void compact_sort(R* (Geo::*row)(i32) const, const Geo& G, i32 hw, i32 n, IdOf id_of) {
    // already in place (a resumed state whose map the new events did not reorder): one pass, no sort
    bool in_place = true;
    i64 prev = 0;
    for (i32 j = 0; j < hw; ++j) {
      const R* r = (G.*row)(j);
      const bool live = (r->flags & CRR_ROW_LIVE) != 0;
      const i64 id = id_of(r);
      in_place = in_place && (j < n ? live && (j == 0 || id > prev) : !live);
      prev = id;
    }
    if (in_place) return;
    for (i32 i = 0; i < n; ++i) {
      i32 best = -1;
      i64 bid = 0;
      for (i32 j = i; j < hw; ++j) {
        const R* r = (G.*row)(j);
        if (!(r->flags & CRR_ROW_LIVE)) continue;
        i64 id = id_of(r);
        if (best < 0 || id < bid) { best = j; bid = id; }
      }
      if (best != i) swap_rows<R, sizeof(R) / 8>((G.*row)(i), (G.*row)(best));
    }
  }
  // live rows sorted by event ID into slots 0..n-1
  __device__ __forceinline__ void finalize(Lane& L, const Geo& G) {
    compact_sort<crr_activity_row>(&Geo::act, G, hw_act, L.n_act, [](const crr_activity_row* r) { return r->schedule_id; });
    compact_sort<crr_timer_row>(&Geo::timer, G, hw_timer, L.n_timer, [](const crr_timer_row* r) { return r->started_id; });
    compact_sort<crr_child_row>(&Geo::child, G, hw_child, L.n_child, [](const crr_child_row* r) { return r->initiated_id; });
    compact_sort<crr_initiated_row>(&Geo::rc, G, hw_rc, L.n_rc, [](const crr_initiated_row* r) { return r->initiated_id; });
    compact_sort<crr_initiated_row>(&Geo::sig, G, hw_sig, L.n_sig, [](const crr_initiated_row* r) { return r->initiated_id; });
  }
  // sorted IDs for the checksum (after finalize)
  __device__ __forceinline__ i64 timer_id(const Geo& G, i32 i) const { return G.timer(i)->started_id; }
  __device__ __forceinline__ i64 act_id(const Geo& G, i32 i) const { return G.act(i)->schedule_id; }
  __device__ __forceinline__ i64 sig_id(const Geo& G, i32 i) const { return G.sig(i)->initiated_id; }
  __device__ __forceinline__ i64 rc_id(const Geo& G, i32 i) const { return G.rc(i)->initiated_id; }
  __device__ __forceinline__ i64 child_id(const Geo& G, i32 i) const { return G.child(i)->initiated_id; }
  __device__ __forceinline__ void retry_push(const crr_inputs&, const crr_outputs&, u32) const {}  // never retries
};

// ===================================================================================================
// LdsTables: the live pending entries are held in LDS ([slot][lane] SoA, bank-conflict free);
// HBM rows are not touched during replay.  At the end the live entries are sorted and their rows
// are rebuilt from LDS plus the source events (version / IDs / batch of the event steps recorded
// in LDS), so a workflow whose maps drain writes no pending rows at all.
// ===================================================================================================
// LDS slot tiers: workflows whose live sets fit the small tier run at 3 blocks/CU (48 KB LDS/block),
// the large tier at 2 blocks/CU (76.8 KB); anything larger falls back to GlobalTables.
template <int A, int T, int C, int R, int S, int P, int LANES_ = kBlock>
struct Tier {
  static constexpr int A_SLOTS = A, T_SLOTS = T, C_SLOTS = C, R_SLOTS = R, S_SLOTS = S, P_SLOTS = P;
  static constexpr int LANES = LANES_;  // threads of the block that share the arena
};
using SmallTier = Tier<1, 1, 1, 1, 1, 1>;
using LargeTier = Tier<CRR_LDS_ACT, CRR_LDS_TIMER, CRR_LDS_CHILD, CRR_LDS_RC, CRR_LDS_SIG, CRR_LDS_RP>;
// retry pass, lane per workflow, one wavefront per block (67 KB arena: 2 blocks/CU)
using HugeTier = Tier<8, 8, 4, 4, 4, 8, 64>;
#define CRR_TIER_SLOTS                                                                      \
  static constexpr int A_SLOTS = TIER::A_SLOTS, T_SLOTS = TIER::T_SLOTS, C_SLOTS = TIER::C_SLOTS, \
                       R_SLOTS = TIER::R_SLOTS, S_SLOTS = TIER::S_SLOTS, P_SLOTS = TIER::P_SLOTS, \
                       LANES = TIER::LANES;
// activity LDS flag bits: row bits (LIVE, MAPPED, CANCEL_REQUESTED, HAS_RETRY) + STARTED; TimerTaskStatus << 8
constexpr u32 LF_STARTED = 32u;
constexpr u32 LF_HB_VIS = 64u;  // a heartbeat timer was created: LastHeartbeatTimeoutVisibilityInSeconds set
constexpr int LF_TTS_SHIFT = 8;
constexpr u32 TF_CREATED = 2u;  // timer LDS flag: TaskStatus == TimerTaskStatusCreated
// CompactTables<TIER, true>: a loaded activity whose row image changed (MAPPED, TimerTaskStatus) and a loaded
// timer's TaskStatus as loaded -- finalize rewrites a loaded row in place only when it differs
constexpr u32 LF_DIRTY = 128u;
constexpr u32 LF_LOADED_MAPPED = 16u;   // the loaded row's persisted MAPPED bit
constexpr u32 TF_LOADED_CREATED = 4u;

template <class TIER>
struct LdsArena {
  CRR_TIER_SLOTS
  i64 a_sid[A_SLOTS][LANES];
  i64 a_sched_t[A_SLOTS][LANES];
  i64 a_start_t[A_SLOTS][LANES];
  int4 a_to[A_SLOTS][LANES];    // s2s, s2c, st2c, hb
  u32 a_key[A_SLOTS][LANES];
  u32 a_fl[A_SLOTS][LANES];
  int4 a_src[A_SLOTS][LANES];   // sched step, started step, cancel-requested step, -
  i64 t_sid[T_SLOTS][LANES];
  i64 t_exp[T_SLOTS][LANES];
  u32 t_key[T_SLOTS][LANES];
  u32 t_fl[T_SLOTS][LANES];
  i32 t_src[T_SLOTS][LANES];
  i64 c_id[C_SLOTS][LANES];
  u32 c_fl[C_SLOTS][LANES];
  int2 c_src[C_SLOTS][LANES];   // initiated step, started step
  i64 r_id[R_SLOTS][LANES];
  u32 r_fl[R_SLOTS][LANES];
  i32 r_src[R_SLOTS][LANES];
  i64 s_id[S_SLOTS][LANES];
  u32 s_fl[S_SLOTS][LANES];
  i32 s_src[S_SLOTS][LANES];
  int4 p_row[P_SLOTS][LANES];   // crr_reset_point_row
};

template <class TIER, bool LANE_DISPATCH = false>
struct LdsTables {
  // divergent wavefronts through apply_event_lanes (mixed-history segments); the one-class batches
  // (config 2) replay in lockstep and keep the plain switch, whose registers fit 3 waves per SIMD
  static constexpr bool kLaneDispatch = LANE_DISPATCH;
  CRR_TIER_SLOTS
  static constexpr bool kResumable = false;  // rows are rebuilt from this call's events: no loaded state
  __device__ __forceinline__ static bool fits(i64) { return true; }
  __device__ __forceinline__ void load(Lane&, const Geo&) {}
  using Arena = LdsArena<TIER>;
  Arena* M;
  int t;  // threadIdx.x
  const crr_inputs* in;
  i64 ev_begin;
  int list = 0;  // scratch list a workflow that outgrows the tier is handed to; < 0: the caller
                 // replays it again itself (retried)
  bool retried = false;

  __device__ __forceinline__ void init(Arena* arena, const crr_inputs* inputs, i64 begin) {
    M = arena;
    t = threadIdx.x;
    in = inputs;
    ev_begin = begin;
#pragma unroll
    for (int j = 0; j < A_SLOTS; ++j) M->a_fl[j][t] = 0;
#pragma unroll
    for (int j = 0; j < T_SLOTS; ++j) M->t_fl[j][t] = 0;
#pragma unroll
    for (int j = 0; j < C_SLOTS; ++j) M->c_fl[j][t] = 0;
#pragma unroll
    for (int j = 0; j < R_SLOTS; ++j) M->r_fl[j][t] = 0;
#pragma unroll
    for (int j = 0; j < S_SLOTS; ++j) M->s_fl[j][t] = 0;
  }
  // source-event column reads (finalize only)
  __device__ __forceinline__ i64 ix(i32 step) const { return ev_begin + (i64)step * 64; }
  __device__ __forceinline__ i64 ev_id(i32 step) const { return in->ev.event_id[ix(step)]; }
  __device__ __forceinline__ i64 ev_ver(i32 step) const { return in->ev.version[ix(step)]; }
  __device__ __forceinline__ i64 batch_first_id(i32 step) const {  // firstEvent.ID of the step's batch
    while (step > 0 && !(in->ev.etype[ix(step)] & CRR_ETYPE_BATCH_FIRST)) --step;
    return ev_id(step);
  }

  __device__ __forceinline__ i32 find_act_by_id(i64 sched) const {
    i32 hit = -1;
#pragma unroll
    for (int j = A_SLOTS - 1; j >= 0; --j)
      if ((M->a_fl[j][t] & CRR_ROW_LIVE) && M->a_sid[j][t] == sched) hit = j;
    return hit;
  }
  __device__ __forceinline__ i32 find_act_mapped(u32 key) const {
    i32 hit = -1;
#pragma unroll
    for (int j = A_SLOTS - 1; j >= 0; --j) {
      u32 f = M->a_fl[j][t];
      if ((f & (CRR_ROW_LIVE | CRR_ROW_MAPPED)) == (CRR_ROW_LIVE | CRR_ROW_MAPPED) && M->a_key[j][t] == key) hit = j;
    }
    return hit;
  }

  __device__ __forceinline__ int act_insert(Lane& L, const Geo& G, const crr_activity_row& row) {
    i32 m = find_act_mapped(row.key);
    i32 j = -1;
#pragma unroll
    for (int k = A_SLOTS - 1; k >= 0; --k)
      if (!(M->a_fl[k][t] & CRR_ROW_LIVE)) j = k;
    if (j < 0) return CRR_INTERNAL_RETRY;
    if (j >= G.act_cap) return CRR_ERR_CAPACITY;
    if (m >= 0) M->a_fl[m][t] &= ~CRR_ROW_MAPPED;
    M->a_sid[j][t] = row.schedule_id;
    M->a_sched_t[j][t] = row.scheduled_time;
    M->a_start_t[j][t] = CRR_ZERO_TIME;
    M->a_to[j][t] = make_int4(row.schedule_to_start, row.schedule_to_close, row.start_to_close, row.heartbeat);
    M->a_key[j][t] = row.key;
    M->a_fl[j][t] = row.flags;
    M->a_src[j][t] = make_int4(row.sched_src, -1, -1, 0);
    ++L.n_act;
    return CRR_OK;
  }
  __device__ __forceinline__ int act_start(Lane& L, const Geo& G, i64 sched, i64 id, i64 ver, i32 s, i64 ts) {
    i32 j = find_act_by_id(sched);
    if (j < 0) return CRR_ERR_MISSING_ACTIVITY_INFO;
    const u32 f = M->a_fl[j][t];
    // a restart after the heartbeat timer was created: LastHeartbeatTimeoutVisibilityInSeconds is no
    // longer derivable from the latest StartedTime -> let the general path replay this workflow
    if ((f & LF_STARTED) && (f & LF_HB_VIS)) return CRR_INTERNAL_RETRY;
    M->a_start_t[j][t] = ts;
    M->a_fl[j][t] = f | LF_STARTED;
    M->a_src[j][t].y = s;
    return CRR_OK;
  }
  __device__ __forceinline__ void act_delete(Lane& L, const Geo& G, i64 sched) {
    i32 j = find_act_by_id(sched);
    if (j < 0) { ++L.inconsistencies; return; }
    u32 f = M->a_fl[j][t];
    u32 key = M->a_key[j][t];
    M->a_fl[j][t] = 0;
    --L.n_act;
    if (f & CRR_ROW_MAPPED) return;
    i32 m = find_act_mapped(key);
    if (m >= 0) M->a_fl[m][t] &= ~CRR_ROW_MAPPED;
    else ++L.inconsistencies;
  }
  __device__ __forceinline__ void act_cancel(Lane& L, const Geo& G, u32 key, i64 /*id*/, i64 /*ver*/, i32 s) {
    i32 j = find_act_mapped(key);
    if (j < 0) return;
    M->a_fl[j][t] |= CRR_ROW_CANCEL_REQUESTED;
    M->a_src[j][t].z = s;
  }

  __device__ __forceinline__ i32 find_timer(u32 key) const {
    i32 hit = -1;
#pragma unroll
    for (int j = T_SLOTS - 1; j >= 0; --j)
      if ((M->t_fl[j][t] & CRR_ROW_LIVE) && M->t_key[j][t] == key) hit = j;
    return hit;
  }
  __device__ __forceinline__ int timer_start(Lane& L, const Geo& G, const crr_timer_row& row) {
    i32 j = find_timer(row.key);
    if (j < 0) {
#pragma unroll
      for (int k = T_SLOTS - 1; k >= 0; --k)
        if (!(M->t_fl[k][t] & CRR_ROW_LIVE)) j = k;
      if (j < 0) return CRR_INTERNAL_RETRY;
      if (j >= G.timer_cap) return CRR_ERR_CAPACITY;
      ++L.n_timer;
    }
    M->t_sid[j][t] = row.started_id;
    M->t_exp[j][t] = row.expiry_time;
    M->t_key[j][t] = row.key;
    M->t_fl[j][t] = CRR_ROW_LIVE;
    M->t_src[j][t] = row.src;
    return CRR_OK;
  }
  __device__ __forceinline__ void timer_delete(Lane& L, const Geo& G, u32 key) {
    i32 j = find_timer(key);
    if (j < 0) { ++L.inconsistencies; return; }
    M->t_fl[j][t] = 0;
    --L.n_timer;
  }

  template <int N>
  __device__ __forceinline__ i32 find_init(const i64 (*ids)[LANES], const u32 (*fl)[LANES], i64 id) const {
    i32 hit = -1;
#pragma unroll
    for (int j = N - 1; j >= 0; --j)
      if ((fl[j][t] & CRR_ROW_LIVE) && ids[j][t] == id) hit = j;
    return hit;
  }
  template <int N>
  __device__ __forceinline__ i32 free_init(const u32 (*fl)[LANES]) const {
    i32 hit = -1;
#pragma unroll
    for (int j = N - 1; j >= 0; --j)
      if (!(fl[j][t] & CRR_ROW_LIVE)) hit = j;
    return hit;
  }
  __device__ __forceinline__ int child_insert(Lane& L, const Geo& G, const crr_child_row& row) {
    i32 j = free_init<C_SLOTS>(M->c_fl);
    if (j < 0) return CRR_INTERNAL_RETRY;
    if (j >= G.child_cap) return CRR_ERR_CAPACITY;
    M->c_id[j][t] = row.initiated_id;
    M->c_fl[j][t] = CRR_ROW_LIVE;
    M->c_src[j][t] = make_int2(row.src, -1);
    ++L.n_child;
    return CRR_OK;
  }
  __device__ __forceinline__ int child_start(Lane& L, const Geo& G, i64 init, i64 id, i32 s) {
    i32 j = find_init<C_SLOTS>(M->c_id, M->c_fl, init);
    if (j < 0) return CRR_ERR_MISSING_CHILD_INFO;
    M->c_src[j][t].y = s;
    return CRR_OK;
  }
  __device__ __forceinline__ void child_delete(Lane& L, const Geo& G, i64 init) {
    i32 j = find_init<C_SLOTS>(M->c_id, M->c_fl, init);
    if (j < 0) { ++L.inconsistencies; return; }
    M->c_fl[j][t] = 0;
    --L.n_child;
  }
  __device__ __forceinline__ int init_insert(Lane& L, const Geo& G, bool is_rc, const crr_initiated_row& row) {
    i32 j = is_rc ? free_init<R_SLOTS>(M->r_fl) : free_init<S_SLOTS>(M->s_fl);
    if (j < 0) return CRR_INTERNAL_RETRY;
    if (j >= (is_rc ? G.rc_cap : G.sig_cap)) return CRR_ERR_CAPACITY;
    if (is_rc) { M->r_id[j][t] = row.initiated_id; M->r_fl[j][t] = CRR_ROW_LIVE; M->r_src[j][t] = row.src; ++L.n_rc; }
    else { M->s_id[j][t] = row.initiated_id; M->s_fl[j][t] = CRR_ROW_LIVE; M->s_src[j][t] = row.src; ++L.n_sig; }
    return CRR_OK;
  }
  __device__ __forceinline__ void init_delete(Lane& L, const Geo& G, bool is_rc, i64 init) {
    i32 j = is_rc ? find_init<R_SLOTS>(M->r_id, M->r_fl, init) : find_init<S_SLOTS>(M->s_id, M->s_fl, init);
    if (j < 0) { ++L.inconsistencies; return; }
    if (is_rc) { M->r_fl[j][t] = 0; --L.n_rc; }
    else { M->s_fl[j][t] = 0; --L.n_sig; }
  }
  __device__ __forceinline__ void rp_reset(Lane& L) { L.n_rp = 0; }
  __device__ __forceinline__ int rp_push(Lane& L, const Geo& G, const crr_reset_point_row& row) {
    if (L.n_rp >= P_SLOTS) return CRR_INTERNAL_RETRY;
    if (L.n_rp >= G.rp_cap) return CRR_ERR_CAPACITY;
    M->p_row[L.n_rp][t] = make_int4(row.src, row.prev_index, (i32)row.key, (i32)row.flags);
    ++L.n_rp;
    return CRR_OK;
  }
  __device__ __forceinline__ bool rp_has(const Lane& L, const Geo& G, u32 key) const {
    bool hit = false;
#pragma unroll
    for (int i = 0; i < P_SLOTS; ++i)
      if (i < L.n_rp && (u32)M->p_row[i][t].z == key) hit = true;
    return hit;
  }
  __device__ __forceinline__ void epilogue(Lane& L, const Geo& G, const TaskSink& K) {
    if (L.n_act > 0) {
      BestTimer B;
#pragma unroll
      for (int j = 0; j < A_SLOTS; ++j) {
        const u32 f = M->a_fl[j][t];
        if (!(f & CRR_ROW_LIVE)) continue;
        const int4 to = M->a_to[j][t];
        activity_candidates(B, j, M->a_sid[j][t], M->a_sched_t[j][t], (f & LF_STARTED) != 0, M->a_start_t[j][t],
                            M->a_start_t[j][t],
                            to.x, to.y, to.z, to.w, f >> LF_TTS_SHIFT);
      }
      if (B.have && !B.created) {
        M->a_fl[B.j][t] |= (timer_mask(B.y) << LF_TTS_SHIFT) | (B.y == CRR_TIMEOUT_HEARTBEAT ? LF_HB_VIS : 0u);
        K.add(L, G, CRR_TASK_ACTIVITY_TIMEOUT, B.y, L.current_version, B.t, B.e, 0, -1);
      }
    }
    if (L.n_timer > 0) {
      BestTimer B;
#pragma unroll
      for (int j = 0; j < T_SLOTS; ++j) {
        const u32 f = M->t_fl[j][t];
        if (!(f & CRR_ROW_LIVE)) continue;
        B.offer(M->t_exp[j][t], M->t_sid[j][t], 0, j, (f & TF_CREATED) != 0);
      }
      if (B.have && !B.created) {
        M->t_fl[B.j][t] |= TF_CREATED;
        K.add(L, G, CRR_TASK_USER_TIMER, 0, L.current_version, B.t, B.e, 0, -1);
      }
    }
  }
  __device__ __forceinline__ bool task_writer() const { return true; }

  // RefreshTasks' state effects (mutable_state_task_refresher.go:278-365)
  __device__ __forceinline__ void refresh(Lane& L, const Geo& G) {
#pragma unroll
    for (int j = 0; j < A_SLOTS; ++j) M->a_fl[j][t] &= ~(0xFu << LF_TTS_SHIFT);
#pragma unroll
    for (int j = 0; j < T_SLOTS; ++j) M->t_fl[j][t] &= ~TF_CREATED;
    epilogue(L, G, TaskSink{false, false});
  }

  template <int N, class SwapFn>
  __device__ __forceinline__ void sort_slots(i64 (*ids)[LANES], u32 (*fl)[LANES], i32 n, SwapFn swap_fn) {
    for (i32 i = 0; i < n; ++i) {
      i32 best = -1;
      i64 bid = 0;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        if (j < i || !(fl[j][t] & CRR_ROW_LIVE)) continue;
        const i64 id = ids[j][t];
        if (best < 0 || id < bid) { best = j; bid = id; }
      }
      if (best != i) {
        swap_fn(i, best);
        i64 x = ids[i][t]; ids[i][t] = ids[best][t]; ids[best][t] = x;
        u32 y = fl[i][t]; fl[i][t] = fl[best][t]; fl[best][t] = y;
      }
    }
  }
  template <class V>
  __device__ __forceinline__ static void swp(V& a, V& b) { V x = a; a = b; b = x; }

  // Sort the live entries by event ID (LDS) and write their rows to HBM slots 0..n-1.
  __device__ __forceinline__ void finalize(Lane& L, const Geo& G) {
    sort_slots<A_SLOTS>(M->a_sid, M->a_fl, L.n_act, [&](int i, int b) {
      swp(M->a_sched_t[i][t], M->a_sched_t[b][t]); swp(M->a_start_t[i][t], M->a_start_t[b][t]);
      swp(M->a_to[i][t], M->a_to[b][t]); swp(M->a_key[i][t], M->a_key[b][t]); swp(M->a_src[i][t], M->a_src[b][t]);
    });
    sort_slots<T_SLOTS>(M->t_sid, M->t_fl, L.n_timer, [&](int i, int b) {
      swp(M->t_exp[i][t], M->t_exp[b][t]); swp(M->t_key[i][t], M->t_key[b][t]); swp(M->t_src[i][t], M->t_src[b][t]);
    });
    sort_slots<C_SLOTS>(M->c_id, M->c_fl, L.n_child, [&](int i, int b) { swp(M->c_src[i][t], M->c_src[b][t]); });
    sort_slots<R_SLOTS>(M->r_id, M->r_fl, L.n_rc, [&](int i, int b) { swp(M->r_src[i][t], M->r_src[b][t]); });
    sort_slots<S_SLOTS>(M->s_id, M->s_fl, L.n_sig, [&](int i, int b) { swp(M->s_src[i][t], M->s_src[b][t]); });

    for (i32 i = 0; i < L.n_act; ++i) {  // ReplicateActivityTask{Scheduled,Started,CancelRequested} images
      const u32 f = M->a_fl[i][t];
      const int4 src = M->a_src[i][t];
      const int4 to = M->a_to[i][t];
      const u32 tts = (f >> LF_TTS_SHIFT) & 0xF;
      const bool started = (f & LF_STARTED) != 0;
      crr_activity_row r;
      r.schedule_id = M->a_sid[i][t];
      r.version = ev_ver(max(src.x, max(src.y, src.z)));   // last of Scheduled / Started / CancelRequested
      r.scheduled_batch_id = batch_first_id(src.x);
      r.scheduled_time = M->a_sched_t[i][t];
      r.started_id = started ? ev_id(src.y) : CRR_EMPTY_EVENT_ID;
      r.started_time = M->a_start_t[i][t];
      r.cancel_request_id = (f & CRR_ROW_CANCEL_REQUESTED) ? ev_id(src.z) : CRR_EMPTY_EVENT_ID;
      r.last_hb_timeout_vis_s = (f & LF_HB_VIS) ? unix_seconds(add_seconds(r.started_time, to.w)) : 0;
      r.sched_src = src.x;
      r.started_src = started ? src.y : -1;
      r.schedule_to_start = to.x; r.schedule_to_close = to.y; r.start_to_close = to.z; r.heartbeat = to.w;
      r.timer_task_status = (i32)tts;
      r.key = M->a_key[i][t];
      r.flags = f & (CRR_ROW_LIVE | CRR_ROW_MAPPED | CRR_ROW_CANCEL_REQUESTED | CRR_ROW_HAS_RETRY);
      r.attempt = 0;
      r.last_heartbeat_time = r.started_time;  // StartedTime (:2272-2273), Go's zero time until started
      *G.act(i) = r;
    }
    for (i32 i = 0; i < L.n_timer; ++i) {  // ReplicateTimerStartedEvent image
      const i32 src = M->t_src[i][t];
      crr_timer_row r;
      r.started_id = M->t_sid[i][t];
      r.version = ev_ver(src);
      r.expiry_time = M->t_exp[i][t];
      r.task_status = (M->t_fl[i][t] & TF_CREATED) ? CRR_TIMER_TASK_STATUS_CREATED : CRR_TIMER_TASK_STATUS_NONE;
      r.key = M->t_key[i][t];
      r.src = src;
      r.flags = CRR_ROW_LIVE;
      *G.timer(i) = r;
    }
    for (i32 i = 0; i < L.n_child; ++i) {  // ReplicateStartChildWorkflowExecutionInitiatedEvent (+ Started)
      const int2 src = M->c_src[i][t];
      crr_child_row r;
      r.initiated_id = M->c_id[i][t];
      r.version = ev_ver(src.x);
      r.initiated_batch_id = batch_first_id(src.x);
      r.started_id = src.y >= 0 ? ev_id(src.y) : CRR_EMPTY_EVENT_ID;
      r.src = src.x;
      r.started_src = src.y;
      r.flags = CRR_ROW_LIVE;
      r.reserved = 0;
      *G.child(i) = r;
    }
    for (i32 i = 0; i < L.n_rc; ++i) {
      const i32 src = M->r_src[i][t];
      crr_initiated_row r;
      r.initiated_id = M->r_id[i][t];
      r.version = ev_ver(src);
      r.initiated_batch_id = batch_first_id(src);
      r.src = src;
      r.flags = CRR_ROW_LIVE;
      *G.rc(i) = r;
    }
    for (i32 i = 0; i < L.n_sig; ++i) {
      const i32 src = M->s_src[i][t];
      crr_initiated_row r;
      r.initiated_id = M->s_id[i][t];
      r.version = ev_ver(src);
      r.initiated_batch_id = batch_first_id(src);
      r.src = src;
      r.flags = CRR_ROW_LIVE;
      *G.sig(i) = r;
    }
    for (i32 i = 0; i < L.n_rp; ++i) {
      const int4 p = M->p_row[i][t];
      crr_reset_point_row r;
      r.src = p.x;
      r.prev_index = p.y;
      r.key = (u32)p.z;
      r.flags = (u32)p.w;
      *G.rp(i) = r;
    }
  }
  __device__ __forceinline__ i64 timer_id(const Geo&, i32 i) const { return M->t_sid[i][t]; }
  __device__ __forceinline__ i64 act_id(const Geo&, i32 i) const { return M->a_sid[i][t]; }
  __device__ __forceinline__ i64 sig_id(const Geo&, i32 i) const { return M->s_id[i][t]; }
  __device__ __forceinline__ i64 rc_id(const Geo&, i32 i) const { return M->r_id[i][t]; }
  __device__ __forceinline__ i64 child_id(const Geo&, i32 i) const { return M->c_id[i][t]; }

  // Hand a workflow back to the general path: one atomic per wavefront (ballot + mbcnt prefix
  // count compacts the retrying lanes into the scratch list).
  __device__ __forceinline__ void retry_push(const crr_inputs& in, const crr_outputs& out, u32 w) {
    if (list < 0) { retried = true; return; }
    const u64 m = __builtin_amdgcn_ballot_w64(true);
    const u32 lane = threadIdx.x & 63;
    const u32 leader = (u32)__builtin_ctzll(m);
    const u32 below = __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
    u32 base = 0;
    if (lane == leader) base = atomicAdd(out.scratch + list, (u32)__builtin_popcountll(m));
    base = (u32)__shfl((int)base, (int)leader, 64);
    out.scratch[retry_slot(in, list, base + below)] = w;
  }
};

// ===================================================================================================
// CompactTables: lane per workflow with larger LDS tiers for workflows whose live sets outgrow the
// 2-slot LdsTables tier (mixed histories: several pending activities, timers, children ...).  Same
// [slot][lane] SoA layout as LdsTables at ~40 % of its bytes per slot, so 4-8 slots per map fit at
// 1-2 waves/SIMD instead of the HBM-row GlobalTables scans:
//   * event IDs as u32 and event steps as 10-bit fields (a workflow with an ID >= 2^32 or more than
//     1023 events is handed to the general path: speed only, never results);
//   * per activity only what its timer candidates need: the earliest of its candidates (the head of
//     its part of LoadAndSortActivityTimers' order, timer_sequence.go:219-381) is kept up to date
//     when the activity is scheduled or started -- the only events that change its candidate set --
//     so the per-batch epilogue compares one cached candidate per activity;
//   * everything else of a row (times, timeouts, versions, batch IDs) is re-read from the source
//     events and side records when the live rows are written at the end.
// ===================================================================================================
template <int A, int T, int C, int R, int S, int P, int LANES_ = kBlock>
struct CTier {
  static constexpr int A_SLOTS = A, T_SLOTS = T, C_SLOTS = C, R_SLOTS = R, S_SLOTS = S, P_SLOTS = P;
  static constexpr int LANES = LANES_;
};
// activity flag word: row bits (LIVE, MAPPED, CANCEL_REQUESTED, HAS_RETRY) + LF_STARTED / LF_HB_VIS,
// TimerTaskStatus << 8, the cached candidate's timer type << 12, the scheduled event's offset in its
// batch << 16 (ScheduledEventBatchID = its ID - that offset)
constexpr int CF_CAND_SHIFT = 12;
constexpr int CF_BATCH_SHIFT = 16;       // activity: 10 bits; request-cancel / signal: bits 18.. (10 bits)
constexpr int CHILD_BATCH_SHIFT = 1;     // child: bits 1-7, 127 = "walk back to the batch's first event"
constexpr u32 kChildBatchNone = 127u;
// step fields: 10 bits each
constexpr u32 kStepBits = 10, kStepMask = (1u << kStepBits) - 1u;
constexpr i32 kMaxCompactSteps = (1 << kStepBits) - 1;  // step kStepMask encodes "none"

template <class TIER>
struct CompactArena {
  CRR_TIER_SLOTS
  u32 a_key[A_SLOTS][LANES];
  u32 a_fl[A_SLOTS][LANES];
  u32 a_src[A_SLOTS][LANES];     // sched | started << 10 | cancel-requested << 20 (kStepMask: none)
  i64 a_cand[A_SLOTS][LANES];    // timestamp of the activity's earliest timer candidate
  u32 t_key[T_SLOTS][LANES];
  u32 t_fl[T_SLOTS][LANES];      // LIVE | TF_CREATED | src << 8
  i64 t_exp[T_SLOTS][LANES];
  u32 c_fl[C_SLOTS][LANES];      // LIVE | initiated src << 8 | started src << 18 (kStepMask: none)
  u32 r_fl[R_SLOTS][LANES];      // LIVE | src << 8
  u32 s_fl[S_SLOTS][LANES];
  u32 p_key[P_SLOTS][LANES];
};

// RESUME (a separate instantiation, launched when the batch holds loaded states: CRR_IN_HAS_RESUME): a
// loaded state (CRR_WF_FLAG_RESUME, mutableStateBuilder.Load) continues in the arena.  Steps become
// virtual: this call's event at local step s is v = vk + s (vk = kMaxCompactSteps - n_ev), and a loaded
// entry -- whose events precede this call -- is v = its ID - id0 < vk, id0 = NextEventID - vk, so IDs
// keep ordering by v and lookups by ID compare v exactly as for new entries.  A loaded entry keeps its
// old slot (the row in HBM stays the source of every field the arena does not hold); finalize writes the
// live rows sorted by v, so the loaded ones come first in their old order and each moves down (or stays):
// an in-place compaction that reads every old slot before anything overwrites it.  Whatever cannot be
// held this way -- a loaded ID outside [id0, id0 + vk), rows out of ID order, more loaded rows than
// slots -- goes to the general path (CRR_INTERNAL_RETRY) before anything in HBM is changed; a retry
// later in the replay first restores the one HBM word the lane loop may have overwritten (the loaded
// last version-history item).
constexpr int CF_SLOT_SHIFT = 26;        // activity: the loaded entry's old slot (4 bits)
constexpr int TF_SLOT_SHIFT = 18;        // timer: ditto
constexpr int IF_SLOT_SHIFT = 28;        // child / request-cancel / signal: ditto
template <class TIER, bool RESUME = false>
struct CompactTables {
  CRR_TIER_SLOTS
  static constexpr bool kResumable = RESUME;
  static constexpr bool kFusedMapOps = true;
  static_assert(A_SLOTS <= 16 && T_SLOTS <= 16 && C_SLOTS <= 8 && R_SLOTS <= 8 && S_SLOTS <= 8, "slot fields");
  using Arena = CompactArena<TIER>;
  Arena* M;
  int t;  // threadIdx.x
  const crr_inputs* in;
  i64 ev_begin;  // column index of virtual step v: ev_begin + v * 64
  i32 n_ev = 0;
  // RESUME: v = provenance step + vshift; loaded entries v < vk; the loaded last VH item and reset points
  i32 vshift = 0, vk = 0;
  i32 ld_vh_n = 0, ld_rp = 0;
  i64 ld_vh_id = 0, ld_vh_ver = 0;
  const crr_activity_row* ld_act = nullptr;  // slot 0 of the workflow's activity rows
  i64 ld_st = 64;                            // their slot stride
  __device__ __forceinline__ const crr_activity_row* G_act_loaded(u32 f) const {
    return ld_act + (i64)((f >> CF_SLOT_SHIFT) & 15u) * ld_st;
  }
  // No entry stores its event ID: every insert checks that its event's ID is id0 + its step (Cadence
  // assigns IDs consecutively from the first event), so an entry's ID is id0 + the step it keeps anyway,
  // and a lookup by ID compares steps.  An insert that breaks the rule hands the workflow to the general
  // path (speed only, never results).
  i64 id0 = 0;
  bool have_id0 = false;
  bool retried = false;
  // a map changed since its last batch epilogue; an unchanged map would select the same, already
  // created, timer again (a no-op), so its epilogue is skipped (as WaveTables)
  bool dirty_act = false, dirty_timer = false;

  __device__ __forceinline__ void init(Arena* arena, const crr_inputs* inputs, i64 begin, i32 n_events = 0) {
    M = arena;
    t = threadIdx.x;
    in = inputs;
    ev_begin = begin;
    n_ev = n_events;
#pragma unroll
    for (int j = 0; j < A_SLOTS; ++j) M->a_fl[j][t] = 0;
#pragma unroll
    for (int j = 0; j < T_SLOTS; ++j) M->t_fl[j][t] = 0;
#pragma unroll
    for (int j = 0; j < C_SLOTS; ++j) M->c_fl[j][t] = 0;
#pragma unroll
    for (int j = 0; j < R_SLOTS; ++j) M->r_fl[j][t] = 0;
#pragma unroll
    for (int j = 0; j < S_SLOTS; ++j) M->s_fl[j][t] = 0;
  }
  // fits the compact encodings (10-bit steps); else the general path replays it
  __device__ __forceinline__ static bool fits(i64 n_ev) { return n_ev <= kMaxCompactSteps; }
  __device__ __forceinline__ i64 ix(i32 step) const { return ev_begin + (i64)step * 64; }
  __device__ __forceinline__ i64 ev_id(i32 step) const { return in->ev.event_id[ix(step)]; }
  __device__ __forceinline__ i64 ev_ver(i32 step) const { return in->ev.version[ix(step)]; }
  __device__ __forceinline__ i64 ev_ts(i32 step) const { return in->ev.timestamp[ix(step)]; }
  __device__ __forceinline__ i64 batch_first_id(i32 step) const {
    while (step > vk && !(in->ev.etype[ix(step)] & CRR_ETYPE_BATCH_FIRST)) --step;
    return ev_id(step);
  }
  __device__ __forceinline__ static u32 step_field(u32 w, int k) { return (w >> (kStepBits * k)) & kStepMask; }
  // a virtual step as this call's provenance step (rows' *_src)
  __device__ __forceinline__ i32 prov(i32 v) const { return v - vshift; }
  // the virtual step of a loaded entry's event ID, or -1 (outside what the arena can hold)
  __device__ __forceinline__ i32 loaded_v(i64 id) const {
    const u64 d = (u64)id - (u64)id0;
    return d < (u64)vk ? (i32)d : -1;
  }

  // mutableStateBuilder.Load (mutable_state_builder.go:306-349) into the arena: every loaded row's
  // lookup fields (IDs as virtual steps, keys, flags, each activity's earliest timer candidate), all
  // issued before the first use; the ActivityID map rebuilt (:311-314: the latest ScheduleID of an
  // ActivityID wins).  Sets L.status = CRR_INTERNAL_RETRY when the state does not fit (nothing written).
  __device__ __forceinline__ void load(Lane& L, const Geo& G) {
    if constexpr (RESUME) {
      vk = kMaxCompactSteps - n_ev;
      id0 = (i64)((u64)L.next_event_id - (u64)vk);
      have_id0 = true;
      vshift = vk - L.src_base;
      ev_begin -= (i64)vk * 64;
      ld_vh_n = L.vh_n; ld_vh_id = L.vh_last_id; ld_vh_ver = L.vh_last_ver;
      ld_rp = L.n_rp;
      ld_act = G.act(0);
      ld_st = G.st;
      dirty_act = dirty_timer = true;  // the loaded timer masks are re-examined by the first epilogue
      bool ok = L.n_act <= A_SLOTS && L.n_timer <= T_SLOTS && L.n_child <= C_SLOTS && L.n_rc <= R_SLOTS &&
                L.n_sig <= S_SLOTS && L.n_rp <= P_SLOTS && vk > 0;
      if (ok) {
        // The loaded rows' reads: the first slots of every table without a branch (a slot past the loaded
        // ones reads a dummy -- the batch's first descriptor, one uniform line), so they are all in flight
        // together (one round trip for the common loaded states); the rest slot by slot.
        const void* dummy = in->wf;
        auto act_at = [&](int j) { return j < L.n_act ? G.act(j) : reinterpret_cast<const crr_activity_row*>(dummy); };
        auto timer_at = [&](int j) { return j < L.n_timer ? G.timer(j) : reinterpret_cast<const crr_timer_row*>(dummy); };
        auto child_at = [&](int j) { return j < L.n_child ? G.child(j) : reinterpret_cast<const crr_child_row*>(dummy); };
        auto rc_at = [&](int j) { return j < L.n_rc ? G.rc(j) : reinterpret_cast<const crr_initiated_row*>(dummy); };
        auto sig_at = [&](int j) { return j < L.n_sig ? G.sig(j) : reinterpret_cast<const crr_initiated_row*>(dummy); };
        auto rp_at = [&](int j) { return j < L.n_rp ? G.rp(j) : reinterpret_cast<const crr_reset_point_row*>(dummy); };
        constexpr int FA = A_SLOTS < 2 ? A_SLOTS : 2, FP = P_SLOTS < 2 ? P_SLOTS : 2;
        crr_activity_row ra[FA];
        crr_timer_row rt0 = *timer_at(0);
        crr_child_row rc0 = *child_at(0);
        const i64 rq0 = rc_at(0)->initiated_id, rs0 = sig_at(0)->initiated_id;
        u32 rpk[FP];
#pragma unroll
        for (int j = 0; j < FA; ++j) ra[j] = *act_at(j);
#pragma unroll
        for (int j = 0; j < FP; ++j) rpk[j] = rp_at(j)->key;
        // every read above is issued before any is used: pinned here, the compiler can neither sink a read
        // into its use's branch nor split a row into dependent reads
#pragma unroll
        for (int j = 0; j < FA; ++j) {
          asm volatile("" ::"v"(ra[j].schedule_id), "v"(ra[j].scheduled_time), "v"(ra[j].started_id),
                       "v"(ra[j].started_time), "v"(ra[j].last_heartbeat_time));
          asm volatile("" ::"v"(ra[j].schedule_to_start), "v"(ra[j].schedule_to_close), "v"(ra[j].start_to_close),
                       "v"(ra[j].heartbeat), "v"(ra[j].timer_task_status), "v"(ra[j].key), "v"(ra[j].flags));
        }
        asm volatile("" ::"v"(rt0.started_id), "v"(rt0.expiry_time), "v"(rt0.task_status), "v"(rt0.key),
                     "v"(rc0.initiated_id), "v"(rc0.started_id), "v"(rq0), "v"(rs0));
#pragma unroll
        for (int j = 0; j < FP; ++j) asm volatile("" ::"v"(rpk[j]));
        i32 prev = -1;
        auto put_act = [&](int j, const crr_activity_row& r) {
          const i32 v = loaded_v(r.schedule_id);
          ok = ok && v > prev && r.timer_task_status >= 0 && r.timer_task_status <= 15;
          prev = v;
          const bool started = r.started_id != CRR_EMPTY_EVENT_ID;
          i64 ct = add_seconds(r.scheduled_time, r.schedule_to_close);
          i32 cy = CRR_TIMEOUT_SCHEDULE_TO_CLOSE;
          if (!started) {
            cand_min(ct, cy, add_seconds(r.scheduled_time, r.schedule_to_start), CRR_TIMEOUT_SCHEDULE_TO_START);
          } else {
            cand_min(ct, cy, add_seconds(r.started_time, r.start_to_close), CRR_TIMEOUT_START_TO_CLOSE);
            if (r.heartbeat > 0)
              cand_min(ct, cy, add_seconds(max(r.started_time, r.last_heartbeat_time), r.heartbeat), CRR_TIMEOUT_HEARTBEAT);
          }
          M->a_key[j][t] = r.key;
          M->a_cand[j][t] = ct;
          // loaded started / cancel-requested events: any virtual step below vk (their IDs stay in the row)
          M->a_src[j][t] = (u32)(v < 0 ? 0 : v) | ((started ? 0u : kStepMask) << kStepBits) |
                           (((r.flags & CRR_ROW_CANCEL_REQUESTED) ? 0u : kStepMask) << (2 * kStepBits));
          M->a_fl[j][t] = CRR_ROW_LIVE | (r.flags & (CRR_ROW_CANCEL_REQUESTED | CRR_ROW_HAS_RETRY)) |
                          ((r.flags & CRR_ROW_MAPPED) ? LF_LOADED_MAPPED : 0u) |
                          (started ? LF_STARTED : 0u) | ((u32)r.timer_task_status << LF_TTS_SHIFT) |
                          ((u32)cy << CF_CAND_SHIFT) | ((u32)j << CF_SLOT_SHIFT);
        };
#pragma unroll
        for (int j = 0; j < FA; ++j)
          if (j < L.n_act) put_act(j, ra[j]);
        for (int j = FA; j < L.n_act; ++j) put_act(j, *G.act(j));
        prev = -1;
        auto put_timer = [&](int j, const crr_timer_row& r) {
          const i32 v = loaded_v(r.started_id);
          ok = ok && v > prev && (r.task_status == CRR_TIMER_TASK_STATUS_NONE || r.task_status == CRR_TIMER_TASK_STATUS_CREATED);
          prev = v;
          M->t_key[j][t] = r.key;
          M->t_exp[j][t] = r.expiry_time;
          M->t_fl[j][t] = CRR_ROW_LIVE |
                          (r.task_status == CRR_TIMER_TASK_STATUS_CREATED ? TF_CREATED | TF_LOADED_CREATED : 0u) |
                          ((u32)(v < 0 ? 0 : v) << 8) | ((u32)j << TF_SLOT_SHIFT);
        };
        if (L.n_timer > 0) put_timer(0, rt0);
        for (int j = 1; j < L.n_timer; ++j) put_timer(j, *G.timer(j));
        prev = -1;
        auto put_child = [&](int j, const crr_child_row& r) {
          const i32 v = loaded_v(r.initiated_id);
          ok = ok && v > prev;
          prev = v;
          const u32 sst = r.started_id != CRR_EMPTY_EVENT_ID ? 0u : kStepMask;
          M->c_fl[j][t] = CRR_ROW_LIVE | (kChildBatchNone << CHILD_BATCH_SHIFT) | ((u32)(v < 0 ? 0 : v) << 8) |
                          (sst << (8 + kStepBits)) | ((u32)j << IF_SLOT_SHIFT);
        };
        if (L.n_child > 0) put_child(0, rc0);
        for (int j = 1; j < L.n_child; ++j) put_child(j, *G.child(j));
        prev = -1;
        auto put_init = [&](u32 (*fl)[LANES], int j, i64 id) {
          const i32 v = loaded_v(id);
          ok = ok && v > prev;
          prev = v;
          fl[j][t] = CRR_ROW_LIVE | ((u32)(v < 0 ? 0 : v) << 8) | ((u32)j << IF_SLOT_SHIFT);
        };
        if (L.n_rc > 0) put_init(M->r_fl, 0, rq0);
        for (int j = 1; j < L.n_rc; ++j) put_init(M->r_fl, j, G.rc(j)->initiated_id);
        prev = -1;
        if (L.n_sig > 0) put_init(M->s_fl, 0, rs0);
        for (int j = 1; j < L.n_sig; ++j) put_init(M->s_fl, j, G.sig(j)->initiated_id);
#pragma unroll
        for (int i = 0; i < FP; ++i)
          if (i < L.n_rp) M->p_key[i][t] = rpk[i];
        for (int i = FP; i < L.n_rp; ++i) M->p_key[i][t] = G.rp(i)->key;
        // the ActivityID map: an entry is mapped unless a later-scheduled one holds the same ActivityID
#pragma unroll
        for (int j = 0; j < A_SLOTS; ++j) {
          if (j < L.n_act) {
            const u32 key = M->a_key[j][t];
            bool mapped = true;
#pragma unroll
            for (int k = j + 1; k < A_SLOTS; ++k)
              if (k < L.n_act && M->a_key[k][t] == key) mapped = false;
            const u32 f = M->a_fl[j][t];
            M->a_fl[j][t] = f | (mapped ? CRR_ROW_MAPPED : 0u) | (mapped != ((f & LF_LOADED_MAPPED) != 0) ? LF_DIRTY : 0u);
          }
        }
      }
      if (!ok) L.status = CRR_INTERNAL_RETRY;
    }
  }
  // before handing a resumed workflow back: the one loaded HBM word the lane loop may have changed
  __device__ __forceinline__ void before_retry(const Lane&, const Geo& G) const {
    if constexpr (RESUME) {
      if (ld_vh_n > 0) {
        crr_vh_item* it = G.vh(ld_vh_n - 1);
        it->event_id = ld_vh_id;
        it->version = ld_vh_ver;
      }
    }
  }
  __device__ __forceinline__ i64 id_at(u32 step) const { return (i64)((u64)id0 + step); }
  // the step an entry inserted by event ID `id` holds, or kStepMask (matches no entry)
  __device__ __forceinline__ u32 step_of(i64 id) const {
    const u64 d = (u64)id - (u64)id0;
    return (have_id0 && d < (u64)kStepMask) ? (u32)d : kStepMask;
  }
  // an insert by the event at step s: its ID must be id0 + s
  __device__ __forceinline__ bool insert_ok(i64 id, i32 s) {
    const i64 b = (i64)((u64)id - (u64)s);
    if (!have_id0) { id0 = b; have_id0 = true; return true; }
    return b == id0;
  }

  __device__ __forceinline__ i32 find_act_mapped(u32 key) const {
    i32 hit = -1;
#pragma unroll
    for (int j = A_SLOTS - 1; j >= 0; --j) {
      const u32 f = M->a_fl[j][t];
      if ((f & (CRR_ROW_LIVE | CRR_ROW_MAPPED)) == (CRR_ROW_LIVE | CRR_ROW_MAPPED) && M->a_key[j][t] == key) hit = j;
    }
    return hit;
  }
  // the earliest of an activity's timer candidates (getActivity*Timeout, timer_sequence.go:269-381);
  // candidates of one activity share its ScheduleID, so they order by (time, timer type)
  __device__ __forceinline__ static void cand_min(i64& ct, i32& cy, i64 t2, i32 y2) {
    if (t2 < ct || (t2 == ct && y2 < cy)) { ct = t2; cy = y2; }
  }

  // Map operations (apply_event runs them after its switch, every lane at once): one pass over a map's
  // slots finds the entry an operation addresses and the first free slot, then the operation's writes.
  __device__ __forceinline__ int map_op(Lane& L, const Geo& G, u32 op, const Ev& ev, i32 s, i64 bfid,
                                        const crr_activity_side& as) {
    return map_op_unified(L, G, op, ev, s + vshift, bfid, as);  // provenance step -> virtual step
  }
  // One code path for every map operation, so a divergent wavefront (lanes with different event types)
  // runs one slot scan and one write-back per step instead of one per map and operation: each lane
  // picks its map's flag and lookup words (LDS addresses), lookup value and slot count, and the
  // operations differ only in the words they write.  Same results as act_op / timer_op / child_op /
  // init_op (the per-map forms, CRR_COMPACT_UNIFIED=0).
  __device__ __forceinline__ int map_op_unified(Lane& L, const Geo& G, u32 op, const Ev& ev, i32 s, i64 bfid,
                                                const crr_activity_side& as) {
    const bool is_act = op <= MOP_ACT_CANCEL;
    const bool is_timer = op == MOP_TIMER_START || op == MOP_TIMER_DELETE;
    const bool is_child = op >= MOP_CHILD_INSERT && op <= MOP_CHILD_DELETE;
    const bool is_rc = op == MOP_RC_INSERT || op == MOP_RC_DELETE;
    const bool act_by_id = op == MOP_ACT_START || op == MOP_ACT_DELETE;
    const bool act_by_key = op == MOP_ACT_INSERT || op == MOP_ACT_CANCEL;
    const bool by_step = act_by_id || (!is_act && !is_timer);  // ScheduleID / InitiatedID lookups
    const bool insert = op == MOP_ACT_INSERT || op == MOP_TIMER_START || op == MOP_CHILD_INSERT ||
                        op == MOP_RC_INSERT || op == MOP_SIG_INSERT;
    const bool del = op == MOP_ACT_DELETE || op == MOP_TIMER_DELETE || op == MOP_CHILD_DELETE ||
                     op == MOP_RC_DELETE || op == MOP_SIG_DELETE;
    // word offsets into the arena (one index off M keeps the accesses in LDS; a select between
    // pointers would turn them into flat accesses)
    constexpr u32 kW = sizeof(u32);
    const u32 fo = (is_act ? (u32)offsetof(Arena, a_fl) : is_timer ? (u32)offsetof(Arena, t_fl)
                  : is_child ? (u32)offsetof(Arena, c_fl) : is_rc ? (u32)offsetof(Arena, r_fl) : (u32)offsetof(Arena, s_fl)) / kW + t;
    const u32 co = act_by_id ? (u32)offsetof(Arena, a_src) / kW + t : act_by_key ? (u32)offsetof(Arena, a_key) / kW + t
                 : is_timer ? (u32)offsetof(Arena, t_key) / kW + t : fo;
    u32* const W = reinterpret_cast<u32*>(M);
    u32* fl = W + fo;
    const u32* cmp = W + co;
    const i32 n = is_act ? A_SLOTS : is_timer ? T_SLOTS : is_child ? C_SLOTS : is_rc ? R_SLOTS : S_SLOTS;
    const u32 need = act_by_key ? (CRR_ROW_LIVE | CRR_ROW_MAPPED) : CRR_ROW_LIVE;
    const u32 sh = (by_step && !is_act) ? 8u : 0u;
    const u32 msk = by_step ? kStepMask : 0xFFFFFFFFu;
    // inserts of children / request-cancels / signals look nothing up (kStepMask matches no entry)
    const u32 want = by_step ? (insert ? kStepMask : step_of(ev.ref())) : ev.key();
    constexpr int kMax = A_SLOTS > T_SLOTS ? A_SLOTS : T_SLOTS;
    static_assert(kMax >= C_SLOTS && kMax >= R_SLOTS && kMax >= S_SLOTS, "activity or timer map is the largest");
    i32 hit = -1, fr = -1;
#pragma unroll
    for (int j = kMax - 1; j >= 0; --j) {
      if (j < n) {
        const u32 f = fl[j * LANES];
        const u32 v = cmp[j * LANES];
        if ((f & need) == need && ((v >> sh) & msk) == want) hit = j;
        if (!(f & CRR_ROW_LIVE)) fr = j;
      }
    }
    i32 d = 0;  // change of the map's live count
    int rc = CRR_OK;
    if (del) {
      if (hit < 0) {
        ++L.inconsistencies;
      } else {
        const u32 f = fl[hit * LANES];
        fl[hit * LANES] = 0;
        d = -1;
        if (is_act && !(f & CRR_ROW_MAPPED)) {  // DeleteActivity of an entry another one's ActivityID shadows
          const i32 m = find_act_mapped(M->a_key[hit][t]);
          if (m >= 0) M->a_fl[m][t] = (M->a_fl[m][t] & ~CRR_ROW_MAPPED) | LF_DIRTY;
          else ++L.inconsistencies;
        }
      }
    } else if (insert) {
      // TimerStarted of a live TimerID overwrites it in place (:3057-3081)
      const bool grow = !(is_timer && hit >= 0);
      const i32 j = grow ? fr : hit;
      // values, not lvalues: a conditional over the members would select their addresses and keep
      // Geo (and the output pointers in it) in scratch memory
      const i32 ca = G.act_cap, ct = G.timer_cap, cc = G.child_cap, cr = G.rc_cap, cs = G.sig_cap;
      const i32 cap = is_act ? ca : is_timer ? ct : is_child ? cc : is_rc ? cr : cs;
      if (!insert_ok(ev.id(), s) || j < 0) {
        rc = CRR_INTERNAL_RETRY;
      } else if (grow && j >= cap) {
        rc = CRR_ERR_CAPACITY;
      } else {
        // the event's offset in its batch (IDs are consecutive: insert_ok), so the rows' batch IDs need no
        // walk back over the columns at the end
        const u64 bdelta = (u64)ev.id() - (u64)bfid;
        const u32 bd = bdelta < (u64)kStepMask ? (u32)bdelta : kStepMask;
        u32 nf = CRR_ROW_LIVE | ((u32)s << 8) |
                 (is_child ? (kStepMask << (8 + kStepBits)) | ((bd < kChildBatchNone ? bd : kChildBatchNone) << CHILD_BATCH_SHIFT)
                           : (bd << (8 + kStepBits)));
        if (is_act) {
          if (hit >= 0) M->a_fl[hit][t] = (M->a_fl[hit][t] & ~CRR_ROW_MAPPED) | LF_DIRTY;
          // not started: ScheduleToClose and ScheduleToStart
          i64 ct = add_seconds(ev.ts(), as.schedule_to_close);
          i32 cy = CRR_TIMEOUT_SCHEDULE_TO_CLOSE;
          cand_min(ct, cy, add_seconds(ev.ts(), as.schedule_to_start), CRR_TIMEOUT_SCHEDULE_TO_START);
          nf = CRR_ROW_LIVE | CRR_ROW_MAPPED | (as.has_retry_policy ? CRR_ROW_HAS_RETRY : 0u) | ((u32)cy << CF_CAND_SHIFT) |
               (bd << CF_BATCH_SHIFT);
          M->a_key[j][t] = ev.key();
          M->a_src[j][t] = (u32)s | (kStepMask << kStepBits) | (kStepMask << (2 * kStepBits));
          M->a_cand[j][t] = ct;
        } else if (is_timer) {
          M->t_exp[j][t] = add_seconds(ev.ts(), ev.ref());
          M->t_key[j][t] = ev.key();
        }
        fl[j * LANES] = nf;
        d = grow ? 1 : 0;
      }
    } else if (op == MOP_ACT_START) {  // :2254-2276
      rc = CRR_ERR_MISSING_ACTIVITY_INFO;
      // the rows keep only steps: a StartedID must be id0 + its step too (else the general path)
      if (hit >= 0) rc = ev.id() != id_at((u32)s) ? CRR_INTERNAL_RETRY : act_started(hit, ev, s);
    } else if (op == MOP_CHILD_START) {  // :3485-3507
      rc = CRR_ERR_MISSING_CHILD_INFO;
      if (hit >= 0 && ev.id() != id_at((u32)s)) {
        rc = CRR_INTERNAL_RETRY;
      } else if (hit >= 0) {
        const u32 f = fl[hit * LANES];
        fl[hit * LANES] = (f & ~(kStepMask << (8 + kStepBits))) | ((u32)s << (8 + kStepBits));
        rc = CRR_OK;
      }
    } else if (hit >= 0 && ev.id() != id_at((u32)s)) {  // MOP_ACT_CANCEL: CancelRequestID = id0 + step
      rc = CRR_INTERNAL_RETRY;
    } else if (hit >= 0) {  // MOP_ACT_CANCEL (:2444-2467)
      M->a_fl[hit][t] |= CRR_ROW_CANCEL_REQUESTED;
      const u32 w = M->a_src[hit][t];
      M->a_src[hit][t] = (w & ~(kStepMask << (2 * kStepBits))) | ((u32)s << (2 * kStepBits));
    }
    dirty_act |= is_act && op != MOP_ACT_CANCEL;  // a cancel request changes no timer candidate
    dirty_timer |= is_timer;
    L.n_act += is_act ? d : 0;
    L.n_timer += is_timer ? d : 0;
    L.n_child += is_child ? d : 0;
    L.n_rc += is_rc ? d : 0;
    L.n_sig += (!is_act && !is_timer && !is_child && !is_rc) ? d : 0;
    return rc;
  }
  // ActivityTaskStarted on live entry j: its cached earliest timer candidate becomes the started set's
  __device__ __forceinline__ int act_started(i32 hit, const Ev& ev, i32 s) {
    const u32 f = M->a_fl[hit][t];
    if ((f & LF_STARTED) && (f & LF_HB_VIS)) return CRR_INTERNAL_RETRY;  // as LdsTables::act_start
    const u32 w = M->a_src[hit][t];
    const i32 ss = (i32)step_field(w, 0);
    i64 sched_t;
    i32 s2c, st2c, hb;
    if (RESUME && ss < vk) {  // a loaded activity: its row holds the scheduled event's fields
      const crr_activity_row* r = G_act_loaded(f);
      sched_t = r->scheduled_time; s2c = r->schedule_to_close; st2c = r->start_to_close; hb = r->heartbeat;
    } else {
      // the scheduled event's timeouts: through this event's own aux when the layout joined it
      // (CRR_IN_STARTED_AUX; ss is that event's step, flatten._join_started), else through the scheduled
      // event's aux -- one dependent gather less per ActivityTaskStarted
      const i64 six = ix(ss);
      const i32 pa = (in->flags & CRR_IN_STARTED_AUX) ? ev.aux() : -1;
      const crr_activity_side sa = in->act_side[pa >= 0 ? pa : in->ev.aux[six]];
      sched_t = in->ev.timestamp[six]; s2c = sa.schedule_to_close; st2c = sa.start_to_close; hb = sa.heartbeat;
    }
    i64 ct = add_seconds(sched_t, s2c);
    i32 cy = CRR_TIMEOUT_SCHEDULE_TO_CLOSE;
    cand_min(ct, cy, add_seconds(ev.ts(), st2c), CRR_TIMEOUT_START_TO_CLOSE);
    if (hb > 0) cand_min(ct, cy, add_seconds(ev.ts(), hb), CRR_TIMEOUT_HEARTBEAT);
    M->a_cand[hit][t] = ct;
    M->a_fl[hit][t] = (f & ~(3u << CF_CAND_SHIFT)) | LF_STARTED | ((u32)cy << CF_CAND_SHIFT);
    M->a_src[hit][t] = (w & ~(kStepMask << kStepBits)) | ((u32)s << kStepBits);
    return CRR_OK;
  }

  __device__ __forceinline__ void rp_reset(Lane& L) { L.n_rp = 0; }
  // Reset points are append-only (a push is final): with CRR_RP_HBM the row goes to its output slot at
  // once and only the key the later lookups compare stays in LDS (32 B per lane less in tier 2)
  __device__ __forceinline__ int rp_push(Lane& L, const Geo& G, const crr_reset_point_row& row) {
    if (L.n_rp >= P_SLOTS) return CRR_INTERNAL_RETRY;
    if (RESUME && L.n_rp < ld_rp) return CRR_INTERNAL_RETRY;  // after a reset: would overwrite a loaded row
    if (L.n_rp >= G.rp_cap) return CRR_ERR_CAPACITY;
    M->p_key[L.n_rp][t] = row.key;
    *G.rp(L.n_rp) = row;
    ++L.n_rp;
    return CRR_OK;
  }
  __device__ __forceinline__ bool rp_has(const Lane& L, const Geo& G, u32 key) const {
    bool hit = false;
#pragma unroll
    for (int i = 0; i < P_SLOTS; ++i)
      if (i < L.n_rp && M->p_key[i][t] == key) hit = true;
    return hit;
  }
  // CreateNextActivityTimer / CreateNextUserTimer (timer_sequence.go:127-199) over the cached heads
  __device__ __forceinline__ void epilogue(Lane& L, const Geo& G, const TaskSink& K) {
    // The order is (time, event ID, timer type); IDs are id0 + step, so steps order them, and each
    // activity's entry is already its own earliest candidate, so (time, step) decides -- 32-bit step
    // compares and selects, the winner's type and created bit read once afterwards.
    if (L.n_act > 0 && dirty_act) {
      bool have = false;
      i64 bt = 0;
      u32 bs = 0;
      i32 bj = 0;
#pragma unroll
      for (int j = 0; j < A_SLOTS; ++j) {
        const u32 f = M->a_fl[j][t];
        const i64 c = M->a_cand[j][t];
        const u32 st = M->a_src[j][t] & kStepMask;
        const bool better = (f & CRR_ROW_LIVE) && (!have || c < bt || (c == bt && st < bs));
        have = have || (f & CRR_ROW_LIVE);
        bt = better ? c : bt;
        bs = better ? st : bs;
        bj = better ? j : bj;
      }
      if (have) {
        const u32 f = M->a_fl[bj][t];
        const i32 y = (i32)((f >> CF_CAND_SHIFT) & 3u);
        if (!((f >> LF_TTS_SHIFT) & timer_mask(y))) {
          M->a_fl[bj][t] = f | (timer_mask(y) << LF_TTS_SHIFT) | (y == CRR_TIMEOUT_HEARTBEAT ? LF_HB_VIS : 0u) | LF_DIRTY;
          // the task carries ActivityInfo.Attempt: 0 for this call's activities, a loaded row's own
          const i32 att = (RESUME && K.on && bs < (u32)vk) ? G_act_loaded(f)->attempt : 0;
          K.add(L, G, CRR_TASK_ACTIVITY_TIMEOUT, y, L.current_version, bt, id_at(bs), att, -1);
        }
      }
    }
    dirty_act = false;
    if (L.n_timer > 0 && dirty_timer) {
      bool have = false;
      i64 bt = 0;
      u32 bs = 0;
      i32 bj = 0;
#pragma unroll
      for (int j = 0; j < T_SLOTS; ++j) {
        const u32 f = M->t_fl[j][t];
        const i64 c = M->t_exp[j][t];
        const u32 st = (f >> 8) & kStepMask;
        const bool better = (f & CRR_ROW_LIVE) && (!have || c < bt || (c == bt && st < bs));
        have = have || (f & CRR_ROW_LIVE);
        bt = better ? c : bt;
        bs = better ? st : bs;
        bj = better ? j : bj;
      }
      if (have) {
        const u32 f = M->t_fl[bj][t];
        if (!(f & TF_CREATED)) {
          M->t_fl[bj][t] = f | TF_CREATED;
          K.add(L, G, CRR_TASK_USER_TIMER, 0, L.current_version, bt, id_at(bs), 0, -1);
        }
      }
    }
    dirty_timer = false;
  }
  __device__ __forceinline__ bool task_writer() const { return true; }
  // RefreshTasks' state effects (mutable_state_task_refresher.go:278-365)
  __device__ __forceinline__ void refresh(Lane& L, const Geo& G) {
#pragma unroll
    for (int j = 0; j < A_SLOTS; ++j) M->a_fl[j][t] = (M->a_fl[j][t] & ~(0xFu << LF_TTS_SHIFT)) | LF_DIRTY;
#pragma unroll
    for (int j = 0; j < T_SLOTS; ++j) M->t_fl[j][t] &= ~TF_CREATED;
    dirty_act = dirty_timer = true;
    epilogue(L, G, TaskSink{false, false});
  }

  template <class V>
  __device__ __forceinline__ static void swp(V& a, V& b) { V x = a; a = b; b = x; }
  // selection sort of the live slots by event ID -- by step: IDs are id0 + step (slots 0..n-1 afterwards)
  template <int N, class StepFn, class SwapFn>
  __device__ __forceinline__ void sort_slots(u32 (*fl)[LANES], i32 n, StepFn step_fn, SwapFn swap_fn) {
    for (i32 i = 0; i < n; ++i) {
      i32 best = -1;
      u32 bst = 0;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        if (j < i || !(fl[j][t] & CRR_ROW_LIVE)) continue;
        const u32 st = step_fn(j);
        if (best < 0 || st < bst) { best = j; bst = st; }
      }
      if (best != i) {
        swap_fn(i, best);
        swp(fl[i][t], fl[best][t]);
      }
    }
  }
  __device__ __forceinline__ void finalize(Lane& L, const Geo& G) {
    sort_slots<A_SLOTS>(M->a_fl, L.n_act, [&](int j) { return M->a_src[j][t] & kStepMask; }, [&](int i, int b) {
      swp(M->a_key[i][t], M->a_key[b][t]); swp(M->a_src[i][t], M->a_src[b][t]);
      swp(M->a_cand[i][t], M->a_cand[b][t]);
    });
    sort_slots<T_SLOTS>(M->t_fl, L.n_timer, [&](int j) { return (M->t_fl[j][t] >> 8) & kStepMask; }, [&](int i, int b) {
      swp(M->t_exp[i][t], M->t_exp[b][t]); swp(M->t_key[i][t], M->t_key[b][t]);
    });
    sort_slots<C_SLOTS>(M->c_fl, L.n_child, [&](int j) { return (M->c_fl[j][t] >> 8) & kStepMask; }, [&](int, int) {});
    sort_slots<R_SLOTS>(M->r_fl, L.n_rc, [&](int j) { return (M->r_fl[j][t] >> 8) & kStepMask; }, [&](int, int) {});
    sort_slots<S_SLOTS>(M->s_fl, L.n_sig, [&](int j) { return (M->s_fl[j][t] >> 8) & kStepMask; }, [&](int, int) {});

    // Row fields come from the arena and the step arithmetic of consecutive IDs (an entry's event ID is
    // id0 + its step, checked when it was inserted / started / cancel-requested); the version of an event
    // from the version history (one item: every event's; else the item covering its ID).  Only the
    // activities' timestamps and side records are read back from the columns.
    for (i32 i = 0; i < L.n_act; ++i) {  // ReplicateActivityTask{Scheduled,Started,CancelRequested} images
      const u32 f = M->a_fl[i][t];
      const u32 w = M->a_src[i][t];
      const i32 ss = (i32)step_field(w, 0), st = (i32)step_field(w, 1), sc = (i32)step_field(w, 2);
      const bool started = (f & LF_STARTED) != 0, cancel = (f & CRR_ROW_CANCEL_REQUESTED) != 0;
      if (RESUME && ss < vk) {  // a loaded activity: its row, with what this call changed
        const i32 slot = (i32)((f >> CF_SLOT_SHIFT) & 15u);
        const bool new_st = started && st >= vk, new_sc = cancel && sc >= vk;
        const u32 tts = (f >> LF_TTS_SHIFT) & 0xF;
        const u32 fl = f & (CRR_ROW_LIVE | CRR_ROW_MAPPED | CRR_ROW_CANCEL_REQUESTED | CRR_ROW_HAS_RETRY);
        crr_activity_row* dst = G.act(i);
        if (slot == i && !new_st && !new_sc && !(f & LF_HB_VIS)) {  // in place: only the bookkeeping words,
          if (f & LF_DIRTY) {                                        // and only if they changed
            dst->timer_task_status = (i32)tts;
            dst->flags = fl;
          }
          continue;
        }
        crr_activity_row r = *G.act(slot);
        if (new_st) {
          r.started_id = id_at((u32)st);
          r.started_time = ev_ts(st);
          r.started_src = prov(st);
          r.last_heartbeat_time = r.started_time;
        }
        if (new_sc) r.cancel_request_id = id_at((u32)sc);
        if (new_st || new_sc) r.version = ver_of(L, G, max(new_st ? st : -1, new_sc ? sc : -1));
        if (f & LF_HB_VIS)
          r.last_hb_timeout_vis_s = unix_seconds(add_seconds(max(r.started_time, r.last_heartbeat_time), r.heartbeat));
        r.timer_task_status = (i32)tts;
        r.flags = fl;
        *dst = r;
        continue;
      }
      // the ActivityTaskScheduled event's own fields: timestamp, side record (timeouts)
      const crr_activity_side as = in->act_side[in->ev.aux[ix(ss)]];
      crr_activity_row r;
      r.schedule_id = id_at((u32)ss);
      r.version = ver_of(L, G, max(ss, max(started ? st : -1, cancel ? sc : -1)));  // last of Scheduled / Started / CancelRequested
      r.scheduled_batch_id = r.schedule_id - (i64)((f >> CF_BATCH_SHIFT) & kStepMask);
      r.scheduled_time = ev_ts(ss);
      r.started_id = started ? id_at((u32)st) : CRR_EMPTY_EVENT_ID;
      r.started_time = started ? ev_ts(st) : CRR_ZERO_TIME;
      r.cancel_request_id = cancel ? id_at((u32)sc) : CRR_EMPTY_EVENT_ID;
      r.last_hb_timeout_vis_s = (f & LF_HB_VIS) ? unix_seconds(add_seconds(r.started_time, as.heartbeat)) : 0;
      r.sched_src = prov(ss);
      r.started_src = started ? prov(st) : -1;
      r.schedule_to_start = as.schedule_to_start; r.schedule_to_close = as.schedule_to_close;
      r.start_to_close = as.start_to_close; r.heartbeat = as.heartbeat;
      r.timer_task_status = (i32)((f >> LF_TTS_SHIFT) & 0xF);
      r.key = M->a_key[i][t];
      r.flags = f & (CRR_ROW_LIVE | CRR_ROW_MAPPED | CRR_ROW_CANCEL_REQUESTED | CRR_ROW_HAS_RETRY);
      r.attempt = 0;
      r.last_heartbeat_time = r.started_time;
      *G.act(i) = r;
    }
    for (i32 i = 0; i < L.n_timer; ++i) {  // ReplicateTimerStartedEvent image
      const u32 f = M->t_fl[i][t];
      const i32 src = (i32)((f >> 8) & kStepMask);
      const i32 status = (f & TF_CREATED) ? CRR_TIMER_TASK_STATUS_CREATED : CRR_TIMER_TASK_STATUS_NONE;
      if (RESUME && src < vk) {  // a loaded timer: only its task status can have changed
        const i32 slot = (i32)((f >> TF_SLOT_SHIFT) & 15u);
        if (slot == i) {  // in place: the status word, if it changed
          if (((f & TF_CREATED) != 0) != ((f & TF_LOADED_CREATED) != 0)) G.timer(i)->task_status = status;
        } else {
          crr_timer_row r = *G.timer(slot);
          r.task_status = status;
          *G.timer(i) = r;
        }
        continue;
      }
      crr_timer_row r;
      r.started_id = id_at((u32)src);
      r.version = ver_of(L, G, src);
      r.expiry_time = M->t_exp[i][t];
      r.task_status = status;
      r.key = M->t_key[i][t];
      r.src = prov(src);
      r.flags = CRR_ROW_LIVE;
      *G.timer(i) = r;
    }
    for (i32 i = 0; i < L.n_child; ++i) {
      const u32 f = M->c_fl[i][t];
      const i32 src = (i32)((f >> 8) & kStepMask), sst = (i32)((f >> (8 + kStepBits)) & kStepMask);
      const u32 bd = (f >> CHILD_BATCH_SHIFT) & kChildBatchNone;
      const bool started = sst != (i32)kStepMask;
      if (RESUME && src < vk) {  // a loaded child: ChildWorkflowExecutionStarted may have come in this call
        const i32 slot = (i32)((f >> IF_SLOT_SHIFT) & 7u);
        const bool new_st = started && sst >= vk;
        if (slot == i && !new_st) continue;
        crr_child_row r = *G.child(slot);
        if (new_st) {
          r.started_id = id_at((u32)sst);
          r.started_src = prov(sst);
        }
        *G.child(i) = r;
        continue;
      }
      crr_child_row r;
      r.initiated_id = id_at((u32)src);
      r.version = ver_of(L, G, src);
      r.initiated_batch_id = bd != kChildBatchNone ? r.initiated_id - (i64)bd : batch_first_id(src);
      r.started_id = started ? id_at((u32)sst) : CRR_EMPTY_EVENT_ID;
      r.src = prov(src);
      r.started_src = started ? prov(sst) : -1;
      r.flags = CRR_ROW_LIVE;
      r.reserved = 0;
      *G.child(i) = r;
    }
    for (i32 i = 0; i < L.n_rc; ++i) {
      const u32 f = M->r_fl[i][t];
      const i32 src = (i32)((f >> 8) & kStepMask);
      if (RESUME && src < vk) {  // a loaded request-cancel: unchanged, moved down over the deleted ones
        const i32 slot = (i32)((f >> IF_SLOT_SHIFT) & 7u);
        if (slot != i) *G.rc(i) = *G.rc(slot);
        continue;
      }
      crr_initiated_row r;
      r.initiated_id = id_at((u32)src);
      r.version = ver_of(L, G, src);
      r.initiated_batch_id = r.initiated_id - (i64)((f >> (8 + kStepBits)) & kStepMask);
      r.src = prov(src);
      r.flags = CRR_ROW_LIVE;
      *G.rc(i) = r;
    }
    for (i32 i = 0; i < L.n_sig; ++i) {
      const u32 f = M->s_fl[i][t];
      const i32 src = (i32)((f >> 8) & kStepMask);
      if (RESUME && src < vk) {  // a loaded signal: unchanged, moved down over the deleted ones
        const i32 slot = (i32)((f >> IF_SLOT_SHIFT) & 7u);
        if (slot != i) *G.sig(i) = *G.sig(slot);
        continue;
      }
      crr_initiated_row r;
      r.initiated_id = id_at((u32)src);
      r.version = ver_of(L, G, src);
      r.initiated_batch_id = r.initiated_id - (i64)((f >> (8 + kStepBits)) & kStepMask);
      r.src = prov(src);
      r.flags = CRR_ROW_LIVE;
      *G.sig(i) = r;
    }
  }
  // the version of the event at `step`: the version history's item covering its ID (all written back to
  // the workflow's own HBM rows before finalize; one item -- a single-version history -- needs no read)
  __device__ __forceinline__ i64 ver_of(const Lane& L, const Geo& G, i32 step) const {
    if (L.vh_n <= 1) return L.vh_last_ver;
    const i64 id = id_at((u32)step);
    for (i32 j = 0; j + 1 < L.vh_n; ++j) {
      const crr_vh_item it = *G.vh(j);
      if (it.event_id >= id) return it.version;
    }
    return L.vh_last_ver;
  }
  __device__ __forceinline__ i64 timer_id(const Geo&, i32 i) const { return id_at((M->t_fl[i][t] >> 8) & kStepMask); }
  __device__ __forceinline__ i64 act_id(const Geo&, i32 i) const { return id_at(M->a_src[i][t] & kStepMask); }
  __device__ __forceinline__ i64 sig_id(const Geo&, i32 i) const { return id_at((M->s_fl[i][t] >> 8) & kStepMask); }
  __device__ __forceinline__ i64 rc_id(const Geo&, i32 i) const { return id_at((M->r_fl[i][t] >> 8) & kStepMask); }
  __device__ __forceinline__ i64 child_id(const Geo&, i32 i) const { return id_at((M->c_fl[i][t] >> 8) & kStepMask); }
  // the general path replays a workflow this tier cannot hold: list 0 of the retry pass
  __device__ __forceinline__ void retry_push(const crr_inputs& in, const crr_outputs& out, u32 w) {
    const u64 m = __builtin_amdgcn_ballot_w64(true);
    const u32 lane = threadIdx.x & 63;
    const u32 leader = (u32)__builtin_ctzll(m);
    const u32 below = __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
    u32 base = 0;
    if (lane == leader) base = atomicAdd(out.scratch, (u32)__builtin_popcountll(m));
    base = (u32)__shfl((int)base, (int)leader, 64);
    out.scratch[retry_slot(in, 0, base + below)] = w;
  }
};

// ===================================================================================================
// WaveTables: one wavefront replays one long history (length bucketing).  The
// state machine runs wave-uniform (scalar registers); the pending maps are full rows that the 64
// lanes search in parallel (one ballot per 64 slots), the per-batch timer candidates are built in
// parallel (shuffle argmin) and the live rows are ordered in parallel at the end.  Row storage:
//   * LdsRows: a per-wave LDS arena (fast path, fused into the lane kernel's launch); a live set
//     that outgrows it stops with CRR_INTERNAL_RETRY and is replayed again with
//   * HbmRows: the workflow's own output rows in HBM (bounded only by the host's capacities).
// ===================================================================================================
template <int NA, int NT, int NC, int NR, int NS, int NP>
struct WaveArena {
  static constexpr int A = NA, T = NT, C = NC, R = NR, S = NS, P = NP;
  crr_activity_row act[NA];
  crr_timer_row timer[NT];
  crr_child_row child[NC];
  crr_initiated_row rc[NR];
  crr_initiated_row sig[NS];
  crr_reset_point_row rp[NP];
  i64 ids[NA + NT + NC + NR + NS];  // sorted IDs for the checksum lists (after finalize)
};
constexpr int kWavesPerBlock = kBlock / 64;

__device__ __forceinline__ void wave_sync_lds() {  // this wave's LDS writes -> visible to all its lanes
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void wave_sync_global() {  // ... and its global-memory writes
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <class ARENA, int LIST>
struct LdsRows {
  static constexpr bool kLds = true;
  static constexpr int kList = LIST;  // scratch list a workflow that outgrows the arena is handed to
  static constexpr i32 A = ARENA::A, T = ARENA::T, C = ARENA::C, R = ARENA::R, S = ARENA::S, P = ARENA::P;
  // WaveTables::act_cand_store keeps two words per activity slot in ids[] until finalize
  static_assert(A + T + C + R + S >= 2 * A, "ids[] too small for the activity candidate cache");
  ARENA* M;
  __device__ __forceinline__ crr_activity_row& act(i32 j) const { return M->act[j]; }
  __device__ __forceinline__ crr_timer_row& timer(i32 j) const { return M->timer[j]; }
  __device__ __forceinline__ crr_child_row& child(i32 j) const { return M->child[j]; }
  __device__ __forceinline__ crr_initiated_row& rc(i32 j) const { return M->rc[j]; }
  __device__ __forceinline__ crr_initiated_row& sig(i32 j) const { return M->sig[j]; }
  __device__ __forceinline__ crr_reset_point_row& rp(i32 j) const { return M->rp[j]; }
};
struct HbmRows {
  static constexpr bool kLds = false;
  static constexpr int kList = -1;    // never outgrown
  static constexpr i32 A = 0x3fffffff, T = A, C = A, R = A, S = A, P = A;
  Geo G;
  __device__ __forceinline__ crr_activity_row& act(i32 j) const { return *G.act(j); }
  __device__ __forceinline__ crr_timer_row& timer(i32 j) const { return *G.timer(j); }
  __device__ __forceinline__ crr_child_row& child(i32 j) const { return *G.child(j); }
  __device__ __forceinline__ crr_initiated_row& rc(i32 j) const { return *G.rc(j); }
  __device__ __forceinline__ crr_initiated_row& sig(i32 j) const { return *G.sig(j); }
  __device__ __forceinline__ crr_reset_point_row& rp(i32 j) const { return *G.rp(j); }
};

template <class ST>
struct WaveTables {
  static constexpr bool kResumable = !ST::kLds;  // HbmRows continue a loaded state in place
  __device__ __forceinline__ static bool fits(i64) { return true; }
  ST S;
  i32 lane;
  i32 hw_act = 0, hw_timer = 0, hw_child = 0, hw_rc = 0, hw_sig = 0;
  bool retried = false;
  // a map changed since its last batch epilogue; an unchanged map would select the same, already
  // created, timer again (a no-op), so its epilogue is skipped
  bool dirty_act = false, dirty_timer = false;

  __device__ __forceinline__ void init() { lane = (i32)(threadIdx.x & 63); }

  // HbmRows ownership: slot j is only ever written and searched by lane j % 64, so every HBM read
  // follows that lane's own writes (single work-item ordering, no fences); a uniform read of a
  // row field takes the owner lane's value.  LDS rows are shared by the whole wave.
  // Every lane stores a shared LDS row itself: with one writer lane the compiler may forward the old
  // value to the others' later loads (per-thread reasoning: they never stored), and the lanes'
  // copies of the wave-uniform state diverge (measured: corrupted exec rows).
  __device__ __forceinline__ bool own(i32 j) const { return ST::kLds || lane == (j & 63); }
  __device__ __forceinline__ u32 bcast(i32 j, u32 v) const {
    if constexpr (ST::kLds) return v;
    else return __builtin_amdgcn_readlane(v, j & 63);
  }

  // first slot j < hw with pred(row j) (uniform), -1 if none.  The bound is made scalar (the compiler
  // cannot tell that the high-water marks are wave-uniform: a loop over a VGPR bound is compiled as a
  // divergent loop, exec masks saved and merged around every load) and every lane reads a row of the
  // block (a lane past hw reads the block's first): the predicate's loads go out together, branch-free.
  template <class Row, class F>
  __device__ __forceinline__ i32 find(Row row, i32 hw, F pred) const {
    const i32 n = uniform32(hw);
    for (i32 b = 0; b < n; b += 64) {
      const i32 j = b + lane;
      const bool hit = pred(row(j < n ? j : b));
      const u64 m = __builtin_amdgcn_ballot_w64((j < n) & hit);
      if (m) return b + (i32)__builtin_ctzll(m);
    }
    return -1;
  }
  // lowest free slot (GlobalTables::free_slot semantics); CAPACITY when `cap` rows are live,
  // INTERNAL_RETRY when the row storage is full first.  Returns the slot or a negative status.
  template <class Row>
  __device__ __forceinline__ i32 take(Row row, i32& hw, i32 store_cap, i32 cap) const {
    i32 j = find(row, hw, [](const auto& r) { return !(r.flags & CRR_ROW_LIVE); });
    if (j < 0) j = hw;
    if (j >= cap) return -CRR_ERR_CAPACITY;
    if (j >= store_cap) return -CRR_INTERNAL_RETRY;
    if (j == hw) ++hw;
    return j;
  }
  __device__ __forceinline__ auto A_() const { return [this](i32 j) -> crr_activity_row& { return S.act(j); }; }
  __device__ __forceinline__ auto T_() const { return [this](i32 j) -> crr_timer_row& { return S.timer(j); }; }
  __device__ __forceinline__ auto C_() const { return [this](i32 j) -> crr_child_row& { return S.child(j); }; }
  __device__ __forceinline__ auto R_() const { return [this](i32 j) -> crr_initiated_row& { return S.rc(j); }; }
  __device__ __forceinline__ auto S_() const { return [this](i32 j) -> crr_initiated_row& { return S.sig(j); }; }
  __device__ __forceinline__ auto P_() const { return [this](i32 j) -> crr_reset_point_row& { return S.rp(j); }; }

  // predicates with both fields read (bitwise &): a short-circuit && puts the second load behind a branch
  // and its own wait
  __device__ __forceinline__ i32 find_act_by_id(i64 sched) const {
    return find(A_(), hw_act, [&](const crr_activity_row& r) {
      return ((r.flags & CRR_ROW_LIVE) != 0) & (r.schedule_id == sched);
    });
  }
  __device__ __forceinline__ i32 find_act_mapped(u32 key) const {
    return find(A_(), hw_act, [&](const crr_activity_row& r) {
      return ((r.flags & (CRR_ROW_LIVE | CRR_ROW_MAPPED)) == (CRR_ROW_LIVE | CRR_ROW_MAPPED)) & (r.key == key);
    });
  }
  __device__ __forceinline__ i32 find_timer(u32 key) const {
    return find(T_(), hw_timer, [&](const crr_timer_row& r) { return ((r.flags & CRR_ROW_LIVE) != 0) & (r.key == key); });
  }
  template <class Row>
  __device__ __forceinline__ i32 find_initiated(Row row, i32 hw, i64 id) const {
    return find(row, hw, [&](const auto& r) { return ((r.flags & CRR_ROW_LIVE) != 0) & (r.initiated_id == id); });
  }

  // LdsRows: each activity's earliest timer candidate (timer_sequence.go:269-381 over its own timeouts),
  // kept current by what changes it -- the insert, the start, the epilogue's created mark, RefreshTasks
  // -- in the arena's ids[] (unused until finalize): the epilogue then reads one candidate per row
  // instead of recomputing every row's.  ids[j]: the time; ids[A + j]: 1 | type << 8 | created << 16.
  __device__ __forceinline__ void act_cand_store(i32 j, const crr_activity_row& r) {
    if constexpr (ST::kLds) {
      BestTimer B;
      activity_candidates(B, j, r.schedule_id, r.scheduled_time, r.started_id != CRR_EMPTY_EVENT_ID, r.started_time,
                          max(r.started_time, r.last_heartbeat_time), r.schedule_to_start, r.schedule_to_close,
                          r.start_to_close, r.heartbeat, (u32)r.timer_task_status);
      S.M->ids[j] = B.t;
      S.M->ids[ST::A + j] = B.have ? (i64)(1u | ((u32)B.y << 8) | ((B.created ? 1u : 0u) << 16)) : 0;
    }
  }
  __device__ __forceinline__ int act_insert(Lane& L, const Geo& G, const crr_activity_row& row) {
    const i32 m = find_act_mapped(row.key);
    const i32 j = take(A_(), hw_act, ST::A, G.act_cap);
    if (j < 0) return -j;
    if (m >= 0 && own(m)) S.act(m).flags &= ~CRR_ROW_MAPPED;
    if (own(j)) S.act(j) = row;
    act_cand_store(j, row);
    ++L.n_act;
    dirty_act = true;
    return CRR_OK;
  }
  __device__ __forceinline__ int act_start(Lane& L, const Geo& G, i64 sched, i64 id, i64 ver, i32 s, i64 ts) {
    const i32 j = find_act_by_id(sched);
    if (j < 0) return CRR_ERR_MISSING_ACTIVITY_INFO;
    dirty_act = true;
    if (own(j)) {
      crr_activity_row& r = S.act(j);
      r.version = ver;
      r.started_id = id;
      r.started_src = s;
      r.started_time = ts;
      r.last_heartbeat_time = ts;
      act_cand_store(j, r);
    }
    return CRR_OK;
  }
  __device__ __forceinline__ void act_delete(Lane& L, const Geo& G, i64 sched) {
    const i32 j = find_act_by_id(sched);
    if (j < 0) { ++L.inconsistencies; return; }
    const u32 f = bcast(j, S.act(j).flags);
    const u32 key = bcast(j, S.act(j).key);
    if (own(j)) S.act(j).flags = f & ~(CRR_ROW_LIVE | CRR_ROW_MAPPED);
    --L.n_act;
    dirty_act = true;
    if (f & CRR_ROW_MAPPED) return;
    const i32 m = find_act_mapped(key);
    if (m >= 0) { if (own(m)) S.act(m).flags &= ~CRR_ROW_MAPPED; }
    else ++L.inconsistencies;
  }
  __device__ __forceinline__ void act_cancel(Lane& L, const Geo& G, u32 key, i64 id, i64 ver, i32 /*s*/) {
    const i32 j = find_act_mapped(key);
    if (j < 0) return;
    if (own(j)) {
      crr_activity_row& r = S.act(j);
      r.version = ver;
      r.flags |= CRR_ROW_CANCEL_REQUESTED;
      r.cancel_request_id = id;
    }
  }
  __device__ __forceinline__ int timer_start(Lane& L, const Geo& G, const crr_timer_row& row) {
    i32 j = find_timer(row.key);
    if (j < 0) {
      j = take(T_(), hw_timer, ST::T, G.timer_cap);
      if (j < 0) return -j;
      ++L.n_timer;
    }
    if (own(j)) S.timer(j) = row;
    dirty_timer = true;
    return CRR_OK;
  }
  __device__ __forceinline__ void timer_delete(Lane& L, const Geo& G, u32 key) {
    const i32 j = find_timer(key);
    if (j < 0) { ++L.inconsistencies; return; }
    if (own(j)) S.timer(j).flags = 0;
    --L.n_timer;
    dirty_timer = true;
  }
  __device__ __forceinline__ int child_insert(Lane& L, const Geo& G, const crr_child_row& row) {
    const i32 j = take(C_(), hw_child, ST::C, G.child_cap);
    if (j < 0) return -j;
    if (own(j)) S.child(j) = row;
    ++L.n_child;
    return CRR_OK;
  }
  __device__ __forceinline__ int child_start(Lane& L, const Geo& G, i64 init, i64 id, i32 s) {
    const i32 j = find_initiated(C_(), hw_child, init);
    if (j < 0) return CRR_ERR_MISSING_CHILD_INFO;
    if (own(j)) {
      S.child(j).started_id = id;
      S.child(j).started_src = s;
    }
    return CRR_OK;
  }
  __device__ __forceinline__ void child_delete(Lane& L, const Geo& G, i64 init) {
    const i32 j = find_initiated(C_(), hw_child, init);
    if (j < 0) { ++L.inconsistencies; return; }
    if (own(j)) S.child(j).flags = 0;
    --L.n_child;
  }
  __device__ __forceinline__ int init_insert(Lane& L, const Geo& G, bool is_rc, const crr_initiated_row& row) {
    const i32 j = is_rc ? take(R_(), hw_rc, ST::R, G.rc_cap) : take(S_(), hw_sig, ST::S, G.sig_cap);
    if (j < 0) return -j;
    if (own(j)) {
      if (is_rc) S.rc(j) = row;
      else S.sig(j) = row;
    }
    if (is_rc) ++L.n_rc; else ++L.n_sig;
    return CRR_OK;
  }
  __device__ __forceinline__ void init_delete(Lane& L, const Geo& G, bool is_rc, i64 init) {
    const i32 j = is_rc ? find_initiated(R_(), hw_rc, init) : find_initiated(S_(), hw_sig, init);
    if (j < 0) { ++L.inconsistencies; return; }
    if (own(j)) {
      if (is_rc) S.rc(j).flags = 0;
      else S.sig(j).flags = 0;
    }
    if (is_rc) --L.n_rc; else --L.n_sig;
  }
  // Load over HbmRows (GlobalTables::load): lane j % 64 writes row j; the fields read across lanes (key,
  // ScheduleID) are not written here
  __device__ __forceinline__ void load(Lane& L, const Geo& G) {
    hw_act = L.n_act; hw_timer = L.n_timer; hw_child = L.n_child; hw_rc = L.n_rc; hw_sig = L.n_sig;
    dirty_act = dirty_timer = true;
    if constexpr (kResumable) {
      for (i32 j = lane; j < hw_act; j += 64) {
        crr_activity_row& r = S.act(j);
        const u32 key = r.key;
        const i64 sid = r.schedule_id;
        bool mapped = true;
        for (i32 k = 0; k < hw_act; ++k) {
          const crr_activity_row& o = S.act(k);
          if (k != j && o.key == key && o.schedule_id > sid) mapped = false;
        }
        r.flags = (r.flags & ~CRR_ROW_MAPPED) | CRR_ROW_LIVE | (mapped ? CRR_ROW_MAPPED : 0u);
      }
      for (i32 j = lane; j < hw_timer; j += 64) S.timer(j).flags |= CRR_ROW_LIVE;
      for (i32 j = lane; j < hw_child; j += 64) S.child(j).flags |= CRR_ROW_LIVE;
      for (i32 j = lane; j < hw_rc; j += 64) S.rc(j).flags |= CRR_ROW_LIVE;
      for (i32 j = lane; j < hw_sig; j += 64) S.sig(j).flags |= CRR_ROW_LIVE;
      wave_sync_global();
    }
  }
  __device__ __forceinline__ void rp_reset(Lane& L) { L.n_rp = 0; }
  __device__ __forceinline__ int rp_push(Lane& L, const Geo& G, const crr_reset_point_row& row) {
    if (L.n_rp >= G.rp_cap) return CRR_ERR_CAPACITY;
    if (L.n_rp >= ST::P) return CRR_INTERNAL_RETRY;
    if (own(L.n_rp)) S.rp(L.n_rp) = row;
    ++L.n_rp;
    return CRR_OK;
  }
  __device__ __forceinline__ bool rp_has(const Lane& L, const Geo& G, u32 key) const {
    return find(P_(), L.n_rp, [&](const crr_reset_point_row& r) { return r.key == key; }) >= 0;
  }

#ifndef CRR_WAVE_MIN_SCALAR
#define CRR_WAVE_MIN_SCALAR 2
#endif
  // argmin of the per-lane candidates across the wavefront (keys are unique: (time, eventID, type)):
  // a scalar pass with readlane over the candidate lanes -- all of them when few, else only those
  // holding the minimum timestamp (found with a shuffle tree over the timestamp alone).
  __device__ __forceinline__ static i64 readlane64(i64 v, i32 l) {
    const u32 lo = __builtin_amdgcn_readlane((u32)(u64)v, l);
    const u32 hi = __builtin_amdgcn_readlane((u32)((u64)v >> 32), l);
    return (i64)(((u64)hi << 32) | lo);
  }
  // minimum over the 64 lanes (all active), uniform: DPP steps inside each row of 16, then the
  // row broadcasts of 15 / 31 (lane 63 ends with the wave minimum) -- VALU moves, no LDS crossbar
  template <int CTRL, int ROW_MASK>
  __device__ __forceinline__ static i64 dpp_min_step(i64 v) {
    const u32 lo = (u32)(u64)v, hi = (u32)((u64)v >> 32);
    const u32 olo = (u32)__builtin_amdgcn_update_dpp((int)lo, (int)lo, CTRL, ROW_MASK, 0xF, false);
    const u32 ohi = (u32)__builtin_amdgcn_update_dpp((int)hi, (int)hi, CTRL, ROW_MASK, 0xF, false);
    const i64 o = (i64)(((u64)ohi << 32) | olo);
    return o < v ? o : v;
  }
  __device__ __forceinline__ static i64 wave_min_i64(i64 v) {
    v = dpp_min_step<0x128, 0xF>(v);  // row_ror:8
    v = dpp_min_step<0x124, 0xF>(v);  // row_ror:4
    v = dpp_min_step<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
    v = dpp_min_step<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
    v = dpp_min_step<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3
    v = dpp_min_step<0x143, 0xC>(v);  // row_bcast:31 -> rows 2, 3
    return readlane64(v, 63);
  }
  __device__ __forceinline__ static void wave_min(BestTimer& B) {
    u64 m = __builtin_amdgcn_ballot_w64(B.have);
    if (__builtin_popcountll(m) > CRR_WAVE_MIN_SCALAR) {
      // many candidates: reduce the timestamp alone (two crossbar shuffles per level), then keep only
      // the lanes holding the minimum (almost always one) for the scalar pass below
      const i64 t = wave_min_i64(B.have ? B.t : (i64)0x7fffffffffffffffLL);
      m = __builtin_amdgcn_ballot_w64(B.have && B.t == t);
    }
    {
      BestTimer R;
      while (m) {
        const i32 l = (i32)__builtin_ctzll(m);
        m &= m - 1;
        const i64 t = readlane64(B.t, l), e = readlane64(B.e, l);
        const i32 y = (i32)__builtin_amdgcn_readlane((u32)B.y, l);
        if (!R.have || seq_less(t, e, y, R.t, R.e, R.y)) {
          R.have = true; R.t = t; R.e = e; R.y = y;
          R.j = (i32)__builtin_amdgcn_readlane((u32)B.j, l);
          R.created = __builtin_amdgcn_readlane((u32)B.created, l) != 0;
        }
      }
      B = R;
    }
  }
  // CreateNextActivityTimer / CreateNextUserTimer (timer_sequence.go:127-199)
  __device__ __forceinline__ void epilogue(Lane& L, const Geo& G, const TaskSink& K) {
    if (L.n_act > 0 && dirty_act) {
      BestTimer B;
      const i32 hwa = uniform32(hw_act);
      for (i32 j = lane; j < hwa; j += 64) {
        const crr_activity_row& r = S.act(j);
        if constexpr (ST::kLds) {  // the row's flags and ID and its cached candidate, read together
          const u32 fl = r.flags;
          const i64 sid = r.schedule_id;
          const i64 w = S.M->ids[ST::A + j];
          const i64 ct = S.M->ids[j];
          if ((fl & CRR_ROW_LIVE) && (w & 1)) B.offer(ct, sid, (i32)((w >> 8) & 0xff), j, ((w >> 16) & 1) != 0);
        } else {
          if (!(r.flags & CRR_ROW_LIVE)) continue;
          activity_candidates(B, j, r.schedule_id, r.scheduled_time, r.started_id != CRR_EMPTY_EVENT_ID, r.started_time,
                              max(r.started_time, r.last_heartbeat_time),
                              r.schedule_to_start, r.schedule_to_close, r.start_to_close, r.heartbeat,
                              (u32)r.timer_task_status);
        }
      }
      wave_min(B);
      i32 attempt = 0;
      if (B.have && !B.created && own(B.j)) {
        crr_activity_row& r = S.act(B.j);
        r.timer_task_status |= timer_mask(B.y);
        if (B.y == CRR_TIMEOUT_HEARTBEAT) r.last_hb_timeout_vis_s = unix_seconds(B.t);
        attempt = r.attempt;
        if constexpr (ST::kLds) S.M->ids[ST::A + B.j] |= (i64)1 << 16;  // the row's earliest is now created
      }
      if (B.have && !B.created) K.add(L, G, CRR_TASK_ACTIVITY_TIMEOUT, B.y, L.current_version, B.t, B.e, (i32)bcast(B.j, (u32)attempt), -1);
    }
    dirty_act = false;
    if (L.n_timer > 0 && dirty_timer) {
      BestTimer B;
      const i32 hwt = uniform32(hw_timer);
      for (i32 j = lane; j < hwt; j += 64) {
        const crr_timer_row& r = S.timer(j);
        const u32 fl = r.flags;
        const i64 ex = r.expiry_time, sid = r.started_id;
        const i32 ts = r.task_status;
        if (fl & CRR_ROW_LIVE) B.offer(ex, sid, 0, j, ts == CRR_TIMER_TASK_STATUS_CREATED);
      }
      wave_min(B);
      if (B.have && !B.created && own(B.j)) S.timer(B.j).task_status = CRR_TIMER_TASK_STATUS_CREATED;
      if (B.have && !B.created) K.add(L, G, CRR_TASK_USER_TIMER, 0, L.current_version, B.t, B.e, 0, -1);
    }
    dirty_timer = false;
  }
  __device__ __forceinline__ bool task_writer() const { return lane == 0; }
  // RefreshTasks' state effects (mutable_state_task_refresher.go:278-365); each lane clears the slots
  // the epilogue's candidate loop reads with the same lane, so no cross-lane ordering is needed
  __device__ __forceinline__ void refresh(Lane& L, const Geo& G) {
    for (i32 j = lane; j < hw_act; j += 64) {
      S.act(j).timer_task_status = CRR_TIMER_TASK_STATUS_NONE;
      if constexpr (ST::kLds) S.M->ids[ST::A + j] &= ~((i64)1 << 16);
    }
    if constexpr (ST::kLds) wave_sync_lds();
    for (i32 j = lane; j < hw_timer; j += 64) S.timer(j).task_status = CRR_TIMER_TASK_STATUS_NONE;
    dirty_act = dirty_timer = true;
    epilogue(L, G, TaskSink{false, false});
  }

  // LdsRows: live rows -> HBM slots 0..n-1 in event-ID order (rank = number of smaller live IDs);
  // the sorted IDs -> ids[] for the checksum lists
  template <class R, class Row, class IdOf>
  __device__ __forceinline__ void scatter(Row row, i32 hw, i64* ids, R* (Geo::*dst)(i32) const, const Geo& G,
                                          IdOf id_of) const {
    for (i32 j = lane; j < hw; j += 64) {
      const R& r = row(j);
      if (!(r.flags & CRR_ROW_LIVE)) continue;
      const i64 id = id_of(r);
      i32 rank = 0;
      for (i32 k = 0; k < hw; ++k) rank += ((row(k).flags & CRR_ROW_LIVE) && id_of(row(k)) < id) ? 1 : 0;
      *(G.*dst)(rank) = r;
      ids[rank] = id;
    }
  }
  // HbmRows: in-place selection sort of the live rows into slots 0..n-1 (parallel argmin per slot,
  // rows swapped one 8-byte word per lane)
  template <class R, class Row, class IdOf>
  __device__ __forceinline__ void sort_in_place(Row row, i32 hw, i32 n, IdOf id_of) const {
    for (i32 i = 0; i < n; ++i) {
      wave_sync_global();
      i64 best_id = 0;
      i32 best = -1;
      for (i32 j = i + lane; j < hw; j += 64) {
        const R& r = row(j);
        if (!(r.flags & CRR_ROW_LIVE)) continue;
        const i64 id = id_of(r);
        if (best < 0 || id < best_id) { best = j; best_id = id; }
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const i32 ob = __shfl_xor(best, off, 64);
        const i64 oid = __shfl_xor((long long)best_id, off, 64);
        if (ob >= 0 && (best < 0 || oid < best_id)) { best = ob; best_id = oid; }
      }
      best = uniform32(best);
      if (best != i) {
        u64* pa = reinterpret_cast<u64*>(&row(i));
        u64* pb = reinterpret_cast<u64*>(&row(best));
        constexpr int W = (int)(sizeof(R) / 8);
        if (lane < W) {
          const u64 x = pa[lane];
          const u64 y = pb[lane];
          pa[lane] = y;
          pb[lane] = x;
        }
      }
    }
    wave_sync_global();
  }
  __device__ __forceinline__ void finalize(Lane& L, const Geo& G) {
    if constexpr (ST::kLds) {
      i64* ids = S.M->ids;
      constexpr i32 oT = ST::A, oC = oT + ST::T, oR = oC + ST::C, oS = oR + ST::R;
      scatter<crr_activity_row>(A_(), hw_act, ids, &Geo::act, G, [](const crr_activity_row& r) { return r.schedule_id; });
      scatter<crr_timer_row>(T_(), hw_timer, ids + oT, &Geo::timer, G, [](const crr_timer_row& r) { return r.started_id; });
      scatter<crr_child_row>(C_(), hw_child, ids + oC, &Geo::child, G, [](const crr_child_row& r) { return r.initiated_id; });
      scatter<crr_initiated_row>(R_(), hw_rc, ids + oR, &Geo::rc, G, [](const crr_initiated_row& r) { return r.initiated_id; });
      scatter<crr_initiated_row>(S_(), hw_sig, ids + oS, &Geo::sig, G, [](const crr_initiated_row& r) { return r.initiated_id; });
      for (i32 i = lane; i < L.n_rp; i += 64) *G.rp(i) = S.rp(i);
      wave_sync_lds();
    } else {
      sort_in_place<crr_activity_row>(A_(), hw_act, L.n_act, [](const crr_activity_row& r) { return r.schedule_id; });
      sort_in_place<crr_timer_row>(T_(), hw_timer, L.n_timer, [](const crr_timer_row& r) { return r.started_id; });
      sort_in_place<crr_child_row>(C_(), hw_child, L.n_child, [](const crr_child_row& r) { return r.initiated_id; });
      sort_in_place<crr_initiated_row>(R_(), hw_rc, L.n_rc, [](const crr_initiated_row& r) { return r.initiated_id; });
      sort_in_place<crr_initiated_row>(S_(), hw_sig, L.n_sig, [](const crr_initiated_row& r) { return r.initiated_id; });
    }
  }
  __device__ __forceinline__ i64 act_id(const Geo& G, i32 i) const {
    if constexpr (ST::kLds) return S.M->ids[i]; else return G.act(i)->schedule_id;
  }
  __device__ __forceinline__ i64 timer_id(const Geo& G, i32 i) const {
    if constexpr (ST::kLds) return S.M->ids[ST::A + i]; else return G.timer(i)->started_id;
  }
  __device__ __forceinline__ i64 child_id(const Geo& G, i32 i) const {
    if constexpr (ST::kLds) return S.M->ids[ST::A + ST::T + i]; else return G.child(i)->initiated_id;
  }
  __device__ __forceinline__ i64 rc_id(const Geo& G, i32 i) const {
    if constexpr (ST::kLds) return S.M->ids[ST::A + ST::T + ST::C + i]; else return G.rc(i)->initiated_id;
  }
  __device__ __forceinline__ i64 sig_id(const Geo& G, i32 i) const {
    if constexpr (ST::kLds) return S.M->ids[ST::A + ST::T + ST::C + ST::R + i]; else return G.sig(i)->initiated_id;
  }
  // kList < 0: the caller replays the workflow again itself (replay_retry_kernel)
  __device__ __forceinline__ void retry_push(const crr_inputs& in, const crr_outputs& out, u32 w) {
    retried = true;
    if constexpr (ST::kList >= 0) {
      if (lane == 0) {
        const u32 k = atomicAdd(out.scratch + ST::kList, 1u);
        out.scratch[retry_slot(in, ST::kList, k)] = w;
      }
    }
  }
};

// ---------------------------------------------------------------------------------------------------
// WaveRegTables: the wavefront path's pending maps (one workflow per wavefront) with their search state
// in registers.  Slot j of a map is register j / 64 of lane j % 64: each slot's key / ID, its flags and
// (activities, timers) the epilogue's candidate.  A search is a compare and a ballot per 64 slots, a free
// slot the first lane with a clear LIVE bit, and a batch epilogue a wave minimum over registers: no LDS
// round trip on the walk's critical path (WaveTables<LdsRows> searched 112-B LDS rows: 2-3 dependent
// LDS round trips per map operation).  The rows themselves stay in the LDS arena (at finalize lane j % 64
// reads row j), and the flags / timer-task bits the mirror holds are patched in when finalize writes them
// to HBM.  Every lane stores a row it changes (the same values to the same LDS address): a store by its
// owner lane alone is a branch on the lane, and the compiler then takes the whole walk -- the loop and
// everything it carries -- as divergent (exec-mask regions, its state in VGPRs).  Nothing in the walk
// branches on a per-lane value.
// fl words: bits 0-7 the row's CRR_ROW_* flags; activities: bit 8 a candidate cached, 9-11 its timeout
// type, 12 it is created, 16-19 TimerTaskStatus; timers: bit 8 TimerTaskStatusCreated.
#ifndef CRR_WAVE_REG
#define CRR_WAVE_REG 1
#endif
// register sets past the high-water mark skipped by scalar branches (big arenas: 5 activity registers)
#ifndef CRR_WAVE_SKIP
#define CRR_WAVE_SKIP 0
#endif
constexpr u32 kMirLive = CRR_ROW_LIVE, kMirMapped = CRR_ROW_MAPPED;
constexpr u32 kMirHave = 1u << 8, kMirCreated = 1u << 12, kMirTimerCreated = 1u << 8;
__device__ __forceinline__ i64 readlane_i64(i64 v, i32 l) {
  const u32 lo = __builtin_amdgcn_readlane((u32)(u64)v, l);
  const u32 hi = __builtin_amdgcn_readlane((u32)((u64)v >> 32), l);
  return (i64)(((u64)hi << 32) | lo);
}
// f(integral_constant<int, 0>), ..., f(integral_constant<int, N - 1>): the register arrays below are only ever
// indexed by such constants, so they stay in registers (a loop index -- even one the unroller removes later --
// leaves them in scratch memory)
template <class F, int... K>
__device__ __forceinline__ void each_(F&& f, std::integer_sequence<int, K...>) {
  (f(std::integral_constant<int, K>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void each(F&& f) {
  each_(f, std::make_integer_sequence<int, N>{});
}
template <class ARENA, int LIST>
struct WaveRegTables {
  static constexpr bool kResumable = false;  // a loaded state goes to the HBM-row pass
  static constexpr int kList = LIST;
  static constexpr i32 A = ARENA::A, T = ARENA::T, C = ARENA::C, R = ARENA::R, S = ARENA::S, P = ARENA::P;
  static constexpr int NA = (A + 63) / 64, NT = (T + 63) / 64, NC = (C + 63) / 64, NR = (R + 63) / 64, NS = (S + 63) / 64;
  static_assert(P <= 64, "reset-point keys: one register");
  __device__ __forceinline__ static bool fits(i64) { return true; }
  ARENA* M;
  i32 lane;
  i32 hw_act = 0, hw_timer = 0, hw_child = 0, hw_rc = 0, hw_sig = 0;  // slots ever used (wave-uniform)
  bool retried = false;
  bool dirty_act = false, dirty_timer = false;  // as WaveTables
  i64 a_id[NA], a_ct[NA];   // ScheduleID; the cached earliest timer candidate's time
  u32 a_key[NA], a_fl[NA];
  u32 t_key[NT], t_fl[NT];
  i64 t_ex[NT], t_sid[NT];  // ExpiryTime, StartedID
  i64 c_id[NC], r_id[NR], s_id[NS];
  u32 c_fl[NC], r_fl[NR], s_fl[NS];
  u32 p_key;

  __device__ __forceinline__ void init() {
    lane = (i32)(threadIdx.x & 63);
    hw_act = hw_timer = hw_child = hw_rc = hw_sig = 0;
    retried = dirty_act = dirty_timer = false;
    each<NA>([&](auto k) { a_id[k] = 0; a_ct[k] = 0; a_key[k] = 0; a_fl[k] = 0; });
    each<NT>([&](auto k) { t_key[k] = 0; t_fl[k] = 0; t_ex[k] = 0; t_sid[k] = 0; });
    each<NC>([&](auto k) { c_id[k] = 0; c_fl[k] = 0; });
    each<NR>([&](auto k) { r_id[k] = 0; r_fl[k] = 0; });
    each<NS>([&](auto k) { s_id[k] = 0; s_fl[k] = 0; });
    p_key = 0;
  }
  __device__ __forceinline__ bool task_writer() const { return lane == 0; }

  // slot j (wave-uniform) of a register array: the owner lane's value, uniform.  Register k is picked by
  // selects on the uniform j / 64, never by an indexed access (which would put the arrays in scratch)
  template <int N, class V>
  __device__ __forceinline__ static V get(const V (&a)[N], i32 j) {
    const i32 jk = j >> 6;
    V x = a[0];
#if CRR_WAVE_SKIP
    each<N>([&](auto k) { if constexpr (k > 0) { if (jk == k) x = a[k]; } });
#else
    each<N>([&](auto k) { if constexpr (k > 0) x = jk == k ? a[k] : x; });
#endif
    if constexpr (sizeof(V) == 8) return (V)readlane_i64((i64)x, j & 63);
    else return (V)__builtin_amdgcn_readlane((u32)x, j & 63);
  }
  template <int N, class V>
  __device__ __forceinline__ void put(V (&a)[N], i32 j, V v) const {
    const i32 jk = j >> 6;
    const bool me = lane == (j & 63);
#if CRR_WAVE_SKIP
    each<N>([&](auto k) { if (jk == k) a[k] = me ? v : a[k]; });
#else
    each<N>([&](auto k) { a[k] = (me & (jk == k)) ? v : a[k]; });
#endif
  }
  template <int N>
  __device__ __forceinline__ void set_bits(u32 (&a)[N], i32 j, u32 set, u32 clear) const {
    const i32 jk = j >> 6;
    const bool me = lane == (j & 63);
#if CRR_WAVE_SKIP
    each<N>([&](auto k) { if (jk == k) a[k] = me ? ((a[k] & ~clear) | set) : a[k]; });
#else
    each<N>([&](auto k) { a[k] = (me & (jk == k)) ? ((a[k] & ~clear) | set) : a[k]; });
#endif
  }
  // first slot (< hw) whose lane-predicate holds, -1 if none.  Every register's ballot is taken (no early
  // exit: a loop that can leave early may stay a loop, and index the arrays dynamically)
  template <int N, class F>
  __device__ __forceinline__ static i32 find(i32 hw, F pred) {
    const i32 n = uniform32(hw);
    i32 r = -1;
    each<N>([&](auto kk) {
      constexpr int k = N - 1 - (int)kk;
#if CRR_WAVE_SKIP
      if (64 * k < n) {
        const u64 m = __builtin_amdgcn_ballot_w64(pred(std::integral_constant<int, k>{}));
        r = m ? 64 * k + (i32)__builtin_ctzll(m) : r;
      }
#else
      const u64 m = __builtin_amdgcn_ballot_w64(pred(std::integral_constant<int, k>{})) & (64 * k < n ? ~0ull : 0ull);
      r = m ? 64 * k + (i32)__builtin_ctzll(m) : r;
#endif
    });
    return r;
  }
  // lowest free slot (GlobalTables::free_slot semantics: slots past hw are free), CAPACITY when `cap`
  // rows are live, INTERNAL_RETRY past the arena
  template <int N>
  __device__ __forceinline__ static i32 take(const u32 (&fl)[N], i32& hw, i32 store_cap, i32 cap) {
    i32 j = N * 64;
    const i32 h = uniform32(hw);
    each<N>([&](auto kk) {
      constexpr int k = N - 1 - (int)kk;
#if CRR_WAVE_SKIP
      if (64 * k <= h) {  // the first free slot is at most hw
        const u64 m = __builtin_amdgcn_ballot_w64(!(fl[k] & kMirLive));
        j = m ? 64 * k + (i32)__builtin_ctzll(m) : j;
      }
#else
      const u64 m = __builtin_amdgcn_ballot_w64(!(fl[k] & kMirLive));
      j = m ? 64 * k + (i32)__builtin_ctzll(m) : j;
#endif
    });
    if (j >= cap) return -CRR_ERR_CAPACITY;
    if (j >= store_cap) return -CRR_INTERNAL_RETRY;
    if (j >= hw) hw = j + 1;
    return j;
  }
  __device__ __forceinline__ i32 find_act_by_id(i64 sched) const {
    return find<NA>(hw_act, [&](auto k) { return ((a_fl[k] & kMirLive) != 0) & (a_id[k] == sched); });
  }
  __device__ __forceinline__ i32 find_act_mapped(u32 key) const {
    return find<NA>(hw_act, [&](auto k) { return ((a_fl[k] & (kMirLive | kMirMapped)) == (kMirLive | kMirMapped)) & (a_key[k] == key); });
  }
  // an activity's earliest timer candidate (timer_sequence.go:269-381 over its own timeouts) as fl bits 8-12
  // and its time; tts: its TimerTaskStatus
  __device__ __forceinline__ static u32 act_cand(i64& t, i64 sid, i64 sched_t, bool started, i64 start_t, i64 hb_t,
                                                  i32 s2s, i32 s2c, i32 st2c, i32 hb, u32 tts) {
    BestTimer B;
    activity_candidates(B, 0, sid, sched_t, started, start_t, hb_t, s2s, s2c, st2c, hb, tts);
    t = B.t;
    return B.have ? (kMirHave | ((u32)B.y << 9) | (B.created ? kMirCreated : 0u)) : 0u;
  }
  __device__ __forceinline__ int act_insert(Lane& L, const Geo& G, const crr_activity_row& row) {
    const i32 m = find_act_mapped(row.key);
    const i32 j = take<NA>(a_fl, hw_act, A, G.act_cap);
    if (j < 0) return -j;
    if (m >= 0) set_bits<NA>(a_fl, m, 0u, kMirMapped);
    M->act[j] = row;
    i64 ct;
    const u32 cw = act_cand(ct, row.schedule_id, row.scheduled_time, false, row.started_time, row.started_time,
                            row.schedule_to_start, row.schedule_to_close, row.start_to_close, row.heartbeat, 0u);
    put<NA>(a_id, j, row.schedule_id);
    put<NA>(a_key, j, row.key);
    put<NA>(a_ct, j, ct);
    put<NA>(a_fl, j, (row.flags & 0xffu) | cw);
    ++L.n_act;
    dirty_act = true;
    return CRR_OK;
  }
  __device__ __forceinline__ int act_start(Lane& L, const Geo& G, i64 sched, i64 id, i64 ver, i32 s, i64 ts) {
    const i32 j = find_act_by_id(sched);
    if (j < 0) return CRR_ERR_MISSING_ACTIVITY_INFO;
    dirty_act = true;
    crr_activity_row& r = M->act[j];
    const i64 sched_t = r.scheduled_time;
    const i32 s2s = r.schedule_to_start, s2c = r.schedule_to_close, st2c = r.start_to_close, hb = r.heartbeat;
    r.version = ver;
    r.started_id = id;
    r.started_src = s;
    r.started_time = ts;
    r.last_heartbeat_time = ts;
    const u32 fl = get<NA>(a_fl, j);
    i64 ct;
    const u32 cw = act_cand(ct, sched, sched_t, id != CRR_EMPTY_EVENT_ID, ts, ts, s2s, s2c, st2c, hb, (fl >> 16) & 0xffu);
    put<NA>(a_ct, j, ct);
    put<NA>(a_fl, j, (fl & ~(kMirHave | (7u << 9) | kMirCreated)) | cw);
    return CRR_OK;
  }
  __device__ __forceinline__ void act_delete(Lane& L, const Geo& G, i64 sched) {
    const i32 j = find_act_by_id(sched);
    if (j < 0) { ++L.inconsistencies; return; }
    const u32 f = get<NA>(a_fl, j);
    const u32 key = get<NA>(a_key, j);
    put<NA>(a_fl, j, 0u);
    --L.n_act;
    dirty_act = true;
    if (f & kMirMapped) return;
    const i32 m = find_act_mapped(key);
    if (m >= 0) set_bits<NA>(a_fl, m, 0u, kMirMapped);
    else ++L.inconsistencies;
  }
  __device__ __forceinline__ void act_cancel(Lane& L, const Geo& G, u32 key, i64 id, i64 ver, i32 /*s*/) {
    const i32 j = find_act_mapped(key);
    if (j < 0) return;
    crr_activity_row& r = M->act[j];
    r.version = ver;
    r.cancel_request_id = id;
    set_bits<NA>(a_fl, j, CRR_ROW_CANCEL_REQUESTED, 0u);
  }
  __device__ __forceinline__ int timer_start(Lane& L, const Geo& G, const crr_timer_row& row) {
    i32 j = find<NT>(hw_timer, [&](auto k) { return ((t_fl[k] & kMirLive) != 0) & (t_key[k] == row.key); });
    if (j < 0) {
      j = take<NT>(t_fl, hw_timer, T, G.timer_cap);
      if (j < 0) return -j;
      ++L.n_timer;
    }
    M->timer[j] = row;
    put<NT>(t_key, j, row.key);
    put<NT>(t_fl, j, row.flags & 0xffu);
    put<NT>(t_ex, j, row.expiry_time);
    put<NT>(t_sid, j, row.started_id);
    dirty_timer = true;
    return CRR_OK;
  }
  __device__ __forceinline__ void timer_delete(Lane& L, const Geo& G, u32 key) {
    const i32 j = find<NT>(hw_timer, [&](auto k) { return ((t_fl[k] & kMirLive) != 0) & (t_key[k] == key); });
    if (j < 0) { ++L.inconsistencies; return; }
    put<NT>(t_fl, j, 0u);
    --L.n_timer;
    dirty_timer = true;
  }
  __device__ __forceinline__ int child_insert(Lane& L, const Geo& G, const crr_child_row& row) {
    const i32 j = take<NC>(c_fl, hw_child, C, G.child_cap);
    if (j < 0) return -j;
    M->child[j] = row;
    put<NC>(c_id, j, row.initiated_id);
    put<NC>(c_fl, j, row.flags & 0xffu);
    ++L.n_child;
    return CRR_OK;
  }
  __device__ __forceinline__ i32 find_child(i64 init) const {
    return find<NC>(hw_child, [&](auto k) { return ((c_fl[k] & kMirLive) != 0) & (c_id[k] == init); });
  }
  __device__ __forceinline__ int child_start(Lane& L, const Geo& G, i64 init, i64 id, i32 s) {
    const i32 j = find_child(init);
    if (j < 0) return CRR_ERR_MISSING_CHILD_INFO;
    M->child[j].started_id = id;
    M->child[j].started_src = s;
    return CRR_OK;
  }
  __device__ __forceinline__ void child_delete(Lane& L, const Geo& G, i64 init) {
    const i32 j = find_child(init);
    if (j < 0) { ++L.inconsistencies; return; }
    put<NC>(c_fl, j, 0u);
    --L.n_child;
  }
  __device__ __forceinline__ int init_insert(Lane& L, const Geo& G, bool is_rc, const crr_initiated_row& row) {
    if (is_rc) {
      const i32 j = take<NR>(r_fl, hw_rc, R, G.rc_cap);
      if (j < 0) return -j;
      M->rc[j] = row;
      put<NR>(r_id, j, row.initiated_id);
      put<NR>(r_fl, j, row.flags & 0xffu);
      ++L.n_rc;
    } else {
      const i32 j = take<NS>(s_fl, hw_sig, S, G.sig_cap);
      if (j < 0) return -j;
      M->sig[j] = row;
      put<NS>(s_id, j, row.initiated_id);
      put<NS>(s_fl, j, row.flags & 0xffu);
      ++L.n_sig;
    }
    return CRR_OK;
  }
  __device__ __forceinline__ void init_delete(Lane& L, const Geo& G, bool is_rc, i64 init) {
    if (is_rc) {
      const i32 j = find<NR>(hw_rc, [&](auto k) { return ((r_fl[k] & kMirLive) != 0) & (r_id[k] == init); });
      if (j < 0) { ++L.inconsistencies; return; }
      put<NR>(r_fl, j, 0u);
      --L.n_rc;
    } else {
      const i32 j = find<NS>(hw_sig, [&](auto k) { return ((s_fl[k] & kMirLive) != 0) & (s_id[k] == init); });
      if (j < 0) { ++L.inconsistencies; return; }
      put<NS>(s_fl, j, 0u);
      --L.n_sig;
    }
  }
  __device__ __forceinline__ void rp_reset(Lane& L) { L.n_rp = 0; }
  __device__ __forceinline__ int rp_push(Lane& L, const Geo& G, const crr_reset_point_row& row) {
    if (L.n_rp >= G.rp_cap) return CRR_ERR_CAPACITY;
    if (L.n_rp >= P) return CRR_INTERNAL_RETRY;
    const i32 n = uniform32(L.n_rp);
    M->rp[n] = row;
    p_key = lane == n ? row.key : p_key;
    ++L.n_rp;
    return CRR_OK;
  }
  __device__ __forceinline__ bool rp_has(const Lane& L, const Geo& G, u32 key) const {
    return __builtin_amdgcn_ballot_w64((lane < L.n_rp) & (p_key == key)) != 0;
  }

  // argmin over candidate slots of (time, ID): the minimum time by a DPP wave minimum of the per-lane
  // minima, then the lowest ID among the slots holding it (IDs are unique among live rows); few candidates
  // take a scalar pass instead.  Returns the slot, -1 if none.
  template <int N>
  __device__ __forceinline__ static i32 argmin(const u32 (&ok)[N], const i64 (&t)[N], const i64 (&id)[N], i64& tmin) {
    u64 m[N];
    i32 cnt = 0;
    each<N>([&](auto k) { m[k] = __builtin_amdgcn_ballot_w64(ok[k] != 0); cnt += __builtin_popcountll(m[k]); });
    if (cnt == 0) return -1;
    i32 best = -1;
    i64 bt = 0, be = 0;
    if (cnt > CRR_WAVE_MIN_SCALAR) {
      i64 v = 0x7fffffffffffffffLL;
      each<N>([&](auto k) { v = (ok[k] && t[k] < v) ? t[k] : v; });
      const i64 wm = WaveTables<HbmRows>::wave_min_i64(v);
      each<N>([&](auto k) { m[k] = __builtin_amdgcn_ballot_w64(ok[k] && t[k] == wm); });
    }
    each<N>([&](auto k) {
      for (u64 x = m[k]; x; x &= x - 1) {
        const i32 l = (i32)__builtin_ctzll(x);
        const i64 tt = readlane_i64(t[k], l), ee = readlane_i64(id[k], l);
        if (best < 0 || tt < bt || (tt == bt && ee < be)) { best = 64 * k + l; bt = tt; be = ee; }
      }
    });
    tmin = bt;
    return best;
  }
  // CreateNextActivityTimer / CreateNextUserTimer (timer_sequence.go:127-199)
  __device__ __forceinline__ void epilogue(Lane& L, const Geo& G, const TaskSink& K) {
    if (L.n_act > 0 && dirty_act) {
      u32 ok[NA];
      each<NA>([&](auto k) { ok[k] = (a_fl[k] & (kMirLive | kMirHave)) == (kMirLive | kMirHave); });
      i64 t = 0;
      const i32 j = argmin<NA>(ok, a_ct, a_id, t);
      if (j >= 0) {
        const u32 fl = get<NA>(a_fl, j);
        const i32 y = (i32)((fl >> 9) & 7u);
        if (!(fl & kMirCreated)) {
          set_bits<NA>(a_fl, j, kMirCreated | (timer_mask(y) << 16), 0u);
          if (y == CRR_TIMEOUT_HEARTBEAT) M->act[j].last_hb_timeout_vis_s = unix_seconds(t);
          if (K.on) K.add(L, G, CRR_TASK_ACTIVITY_TIMEOUT, y, L.current_version, t, get<NA>(a_id, j), M->act[j].attempt, -1);
        }
      }
    }
    dirty_act = false;
    if (L.n_timer > 0 && dirty_timer) {
      u32 ok[NT];
      each<NT>([&](auto k) { ok[k] = (t_fl[k] & kMirLive) != 0; });
      i64 t = 0;
      const i32 j = argmin<NT>(ok, t_ex, t_sid, t);
      if (j >= 0 && !(get<NT>(t_fl, j) & kMirTimerCreated)) {
        set_bits<NT>(t_fl, j, kMirTimerCreated, 0u);
        K.add(L, G, CRR_TASK_USER_TIMER, 0, L.current_version, t, get<NT>(t_sid, j), 0, -1);
      }
    }
    dirty_timer = false;
  }
  // RefreshTasks' state effects (mutable_state_task_refresher.go:278-365)
  __device__ __forceinline__ void refresh(Lane& L, const Geo& G) {
    each<NA>([&](auto k) { a_fl[k] &= ~(kMirCreated | (0xffu << 16)); });
    each<NT>([&](auto k) { t_fl[k] &= ~kMirTimerCreated; });
    dirty_act = dirty_timer = true;
    epilogue(L, G, TaskSink{false, false});
  }

  // live rows -> HBM slots 0..n-1 in event-ID order (rank = number of smaller live IDs), the mirror's flags
  // patched in; the sorted IDs -> ids[] for the checksum lists
  template <int N, class Row, class Patch>
  __device__ __forceinline__ void scatter(const u32 (&fl)[N], const i64 (&id)[N], Row* rows, i64* ids,
                                          Row* (Geo::*dst)(i32) const, const Geo& G, Patch patch) const {
    i32 rank[N];
    u64 live[N];
    each<N>([&](auto k) { rank[k] = 0; live[k] = __builtin_amdgcn_ballot_w64((fl[k] & kMirLive) != 0); });
    each<N>([&](auto k2) {
      for (u64 x = live[k2]; x; x &= x - 1) {
        const i64 o = readlane_i64(id[k2], (i32)__builtin_ctzll(x));
        each<N>([&](auto k) { rank[k] += o < id[k] ? 1 : 0; });
      }
    });
    each<N>([&](auto k) {
      if ((fl[k] & kMirLive) != 0) {
        Row r = rows[64 * k + lane];
        patch(r, fl[k]);
        *(G.*dst)(rank[k]) = r;
        ids[rank[k]] = id[k];
      }
    });
  }
  __device__ __forceinline__ void finalize(Lane& L, const Geo& G) {
    i64* ids = M->ids;
    constexpr i32 oT = A, oC = oT + T, oR = oC + C, oS = oR + R;
    scatter<NA>(a_fl, a_id, M->act, ids, &Geo::act, G, [](crr_activity_row& r, u32 f) {
      r.flags = f & 0xffu;
      r.timer_task_status = (i32)((f >> 16) & 0xffu);
    });
    scatter<NT>(t_fl, t_sid, M->timer, ids + oT, &Geo::timer, G, [](crr_timer_row& r, u32 f) {
      r.flags = f & 0xffu;
      r.task_status = (f & kMirTimerCreated) ? CRR_TIMER_TASK_STATUS_CREATED : CRR_TIMER_TASK_STATUS_NONE;
    });
    scatter<NC>(c_fl, c_id, M->child, ids + oC, &Geo::child, G, [](crr_child_row& r, u32 f) { r.flags = f & 0xffu; });
    scatter<NR>(r_fl, r_id, M->rc, ids + oR, &Geo::rc, G, [](crr_initiated_row& r, u32 f) { r.flags = f & 0xffu; });
    scatter<NS>(s_fl, s_id, M->sig, ids + oS, &Geo::sig, G, [](crr_initiated_row& r, u32 f) { r.flags = f & 0xffu; });
    if (lane < L.n_rp) *G.rp(lane) = M->rp[lane];
    wave_sync_lds();
  }
  __device__ __forceinline__ i64 act_id(const Geo&, i32 i) const { return M->ids[i]; }
  __device__ __forceinline__ i64 timer_id(const Geo&, i32 i) const { return M->ids[A + i]; }
  __device__ __forceinline__ i64 child_id(const Geo&, i32 i) const { return M->ids[A + T + i]; }
  __device__ __forceinline__ i64 rc_id(const Geo&, i32 i) const { return M->ids[A + T + C + i]; }
  __device__ __forceinline__ i64 sig_id(const Geo&, i32 i) const { return M->ids[A + T + C + R + i]; }
  __device__ __forceinline__ void retry_push(const crr_inputs& in, const crr_outputs& out, u32 w) {
    retried = true;
    if constexpr (kList >= 0) {
      if (lane == 0) {
        const u32 k = atomicAdd(out.scratch + kList, 1u);
        out.scratch[retry_slot(in, kList, k)] = w;
      }
    }
  }
};

// The wavefront path's LDS-arena tables (CRR_WAVE_REG=0: the round-5 WaveTables over LDS rows, for A/B)
#if CRR_WAVE_REG
template <class ARENA, int LIST>
using WaveLds = WaveRegTables<ARENA, LIST>;
template <class ARENA, int LIST>
__device__ __forceinline__ void bind_arena(WaveRegTables<ARENA, LIST>& T, ARENA* a) { T.M = a; }
#else
template <class ARENA, int LIST>
using WaveLds = WaveTables<LdsRows<ARENA, LIST>>;
template <class ARENA, int LIST>
__device__ __forceinline__ void bind_arena(WaveTables<LdsRows<ARENA, LIST>>& T, ARENA* a) { T.S.M = a; }
#endif

// ---------------------------------------------------------------------------------------------------
// Event sources.  LaneSource: one workflow per lane, the 8 column loads of step s+1 are issued before
// step s is processed.  WaveSource: one workflow per wavefront, 64 consecutive events are loaded per
// column in one coalesced instruction (one event per lane, the next chunk one chunk ahead) and step s
// is read out of lane s % 64 into scalar registers.

// Lane per workflow: step k of this lane's workflow is column element begin + k * st.
// Loads are typed: the event type of step s+1 is fetched one step ahead of its columns, so only the
// columns that type's transition reads are fetched (per-lane predicated loads; a wavefront whose
// lanes all skip a column issues nothing for it).  TaskID is read once, for the last applied event.
namespace need {  // event types whose transition reads the column (apply_event below)
constexpr u64 bit(int t) { return 1ull << t; }
constexpr u64 kTs = bit(CRR_EV_DECISION_TASK_SCHEDULED) | bit(CRR_EV_DECISION_TASK_STARTED) |
                    bit(CRR_EV_ACTIVITY_TASK_SCHEDULED) | bit(CRR_EV_ACTIVITY_TASK_STARTED) | bit(CRR_EV_TIMER_STARTED);
constexpr u64 kRef = bit(CRR_EV_DECISION_TASK_SCHEDULED) | bit(CRR_EV_DECISION_TASK_STARTED) |
                     bit(CRR_EV_DECISION_TASK_COMPLETED) | bit(CRR_EV_ACTIVITY_TASK_STARTED) |
                     bit(CRR_EV_ACTIVITY_TASK_COMPLETED) | bit(CRR_EV_ACTIVITY_TASK_FAILED) |
                     bit(CRR_EV_ACTIVITY_TASK_TIMED_OUT) | bit(CRR_EV_ACTIVITY_TASK_CANCELED) | bit(CRR_EV_TIMER_STARTED) |
                     bit(CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED) | bit(CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED) |
                     bit(CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED) | bit(CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED) |
                     bit(CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED) | bit(CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT) |
                     bit(CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED) | bit(CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED) |
                     bit(CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED) | bit(CRR_EV_SIGNAL_EXTERNAL_FAILED) |
                     bit(CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED);
constexpr u64 kKey = bit(CRR_EV_DECISION_TASK_COMPLETED) | bit(CRR_EV_ACTIVITY_TASK_SCHEDULED) |
                     bit(CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED) | bit(CRR_EV_TIMER_STARTED) | bit(CRR_EV_TIMER_FIRED) |
                     bit(CRR_EV_TIMER_CANCELED);
constexpr u64 kAux = bit(CRR_EV_WORKFLOW_EXECUTION_STARTED) | bit(CRR_EV_DECISION_TASK_SCHEDULED) |
                     bit(CRR_EV_ACTIVITY_TASK_SCHEDULED) | bit(CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED) |
                     bit(CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW) |
                     bit(CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED) | bit(CRR_EV_SIGNAL_EXTERNAL_INITIATED);
// task emission also reads the start and close events' timestamps (workflow timeout, retention)
constexpr u64 kTsTasks = bit(CRR_EV_WORKFLOW_EXECUTION_STARTED) | bit(CRR_EV_WORKFLOW_EXECUTION_COMPLETED) |
                         bit(CRR_EV_WORKFLOW_EXECUTION_FAILED) | bit(CRR_EV_WORKFLOW_EXECUTION_TIMED_OUT) |
                         bit(CRR_EV_WORKFLOW_EXECUTION_CANCELED) | bit(CRR_EV_WORKFLOW_EXECUTION_TERMINATED) |
                         bit(CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW);
__device__ __forceinline__ bool has(u64 mask, u32 et) { return (mask >> (et & CRR_ETYPE_MASK)) & 1ull; }
}  // namespace need

struct LaneSource {
  const crr_events& E;
  i64 begin, st;
  i32 n;
  Ev nx;      // step s+1 (type and the columns it needs), in flight during step s
  u32 et_nx;  // type byte of step s+2, in flight during step s
  u64 ts_mask;   // types whose timestamp is read (uniform)
  u64 aux_mask;  // types whose aux is read (uniform): ActivityTaskStarted's too with CRR_IN_STARTED_AUX (compact tiers)
  __device__ __forceinline__ LaneSource(const crr_events& e, i64 b, i64 stride, i32 count, bool tasks, bool started_aux = false)
      : E(e), begin(b), st(stride), n(count), ts_mask(need::kTs | (tasks ? need::kTsTasks : 0ull)),
        aux_mask(need::kAux | (started_aux ? need::bit(CRR_EV_ACTIVITY_TASK_STARTED) : 0ull)) {}
  __device__ __forceinline__ i64 ix(i32 step) const { return begin + (i64)step * st; }
  __device__ __forceinline__ Ev load(i32 step, u32 et) const {
    Ev e;
    const i64 i = ix(step);
    e.et = et;
    e.id_ = E.event_id[i];
    e.ver_ = E.version[i];
    e.ts_ = need::has(ts_mask, et) ? E.timestamp[i] : 0;
    e.ref_ = need::has(need::kRef, et) ? E.ref[i] : 0;
    e.key_ = need::has(need::kKey, et) ? E.key[i] : 0u;
    e.aux_ = need::has(aux_mask, et) ? E.aux[i] : 0;
    e.task_ = 0;
    return e;
  }
  // step 0: every column with both type bytes, no load waiting on another (one round trip)
  __device__ __forceinline__ void start() {
    if (n > 0) {  // one branch: step 1's type byte (step 0's again for a one-event history) with the rest
      const i64 i = ix(0);
      nx.et = E.etype[i];
      et_nx = E.etype[ix(n > 1 ? 1 : 0)];
      nx.id_ = E.event_id[i];
      nx.ver_ = E.version[i];
      nx.ts_ = E.timestamp[i];
      nx.ref_ = E.ref[i];
      nx.key_ = E.key[i];
      nx.aux_ = E.aux[i];
      nx.task_ = 0;
    }
  }
  __device__ __forceinline__ Ev next(i32 s) {
    const Ev e = nx;
    issue(s);
    return e;
  }
  // the loads of step s + 1 (and the type byte of s + 2)
  __device__ __forceinline__ void issue(i32 s) {
    if (s + 1 < n) nx = load(s + 1, et_nx);
    if (s + 2 < n) et_nx = E.etype[ix(s + 2)];
  }
  __device__ __forceinline__ i64 task_id(i32 step) const { return E.task_id[ix(step)]; }
};

// One wavefront per workflow runs the state machine on wave-uniform values.  The workflow's events
// stream through in 64-event chunks, one event per lane (one coalesced load per column, the next chunk
// one chunk ahead).  Per chunk the version-history prologue of all 64 events runs lane-parallel
// (replay_body); the transitions then walk the chunk one event at a time and read each field out of
// its lane only where they use it (WaveEv): a MarkerRecorded reads nothing, a DecisionTaskCompleted
// two fields, instead of every event broadcasting all seven.
//   CRR_WAVE_FIELDS 0: __shfl (LDS crossbar) into VGPRs; 1: v_readlane into SGPRs; 2: v_readlane then a
//   VGPR copy.  Round 3 (config 4, alternating A/B on one box): 13.4 / 13.9 / 13.9 ms, against 15.7 ms for the
//   per-event prologue with every field broadcast.  Round 5, once the slot searches and the chunk bounds were
//   scalar: 1 is the fastest (config 4 6.05 -> 5.61 ms, the 256 longest runs alone 4.55 -> 4.24 ms; 2: no
//   gain): with the fields scalar the transitions' branches are scalar branches, not exec-masked regions.
#ifndef CRR_WAVE_FIELDS
#define CRR_WAVE_FIELDS 1
#endif
struct WaveSource {
  const crr_events& E;
  i64 begin, st;
  i32 n, lane;
  Ev cur, nxt;  // per lane: event c * 64 + lane of the current / next chunk
  __device__ __forceinline__ WaveSource(const crr_events& e, i64 b, i64 stride, i32 count)
      : E(e), begin(b), st(stride), n(uniform32(count)) {
    lane = (i32)(threadIdx.x & 63);
  }
  __device__ __forceinline__ Ev load_chunk(i32 c) const {
    Ev e;
    const i32 s = c * 64 + lane;
    const i64 ix = begin + (i64)(s < n ? s : 0) * st;
    e.et = E.etype[ix]; e.id_ = E.event_id[ix]; e.ver_ = E.version[ix]; e.ts_ = E.timestamp[ix];
    e.task_ = 0; e.ref_ = E.ref[ix]; e.key_ = E.key[ix]; e.aux_ = E.aux[ix];
    return e;
  }
  __device__ __forceinline__ i64 task_id(i32 step) const { return E.task_id[begin + (i64)step * st]; }
  __device__ __forceinline__ void start() {
    if (n > 0) cur = load_chunk(0);
  }
  // the next chunk becomes the current one
  __device__ __forceinline__ void rotate() { cur = nxt; }
  // chunk c + 1's loads, issued while chunk c is processed
  __device__ __forceinline__ void issue_next(i32 c) {
    if ((c + 1) * 64 < n) nxt = load_chunk(c + 1);
  }
};
// lane l's value of a per-lane register, wave-uniform (CRR_WAVE_FIELDS above)
__device__ __forceinline__ u32 lane_u32(u32 v, i32 l) {
#if CRR_WAVE_FIELDS == 0
  return (u32)__shfl((int)v, l, 64);
#else
  const u32 r = __builtin_amdgcn_readlane(v, l);
#if CRR_WAVE_FIELDS == 2
  u32 o;
  asm("v_mov_b32 %0, %1" : "=v"(o) : "s"(r));
  return o;
#else
  return r;
#endif
#endif
}
__device__ __forceinline__ i64 lane_i64(i64 v, i32 l) {
  const u32 lo = lane_u32((u32)(u64)v, l), hi = lane_u32((u32)((u64)v >> 32), l);
  return (i64)(((u64)hi << 32) | lo);
}
// ActivityTaskScheduled's side record (the fields the transitions read), gathered lane-parallel for the
// whole chunk before the walk: the walk's insert reads it out of its lane instead of waiting on a
// dependent HBM load per insert
struct SidePf {
  i32 s2s, s2c, st2c, hb, retry, dom;
};
// event l of the current chunk, each field read out of lane l where a transition uses it
struct WaveEv {
  const Ev& C;
  i32 l;
  u32 et;
  const SidePf* sp;
  __device__ __forceinline__ crr_activity_side act_side(const crr_inputs&) const {
    crr_activity_side a{};
    a.schedule_to_start = (i32)lane_u32((u32)sp->s2s, l);
    a.schedule_to_close = (i32)lane_u32((u32)sp->s2c, l);
    a.start_to_close = (i32)lane_u32((u32)sp->st2c, l);
    a.heartbeat = (i32)lane_u32((u32)sp->hb, l);
    a.has_retry_policy = (i32)lane_u32((u32)sp->retry, l);
    a.domain_status = (i32)lane_u32((u32)sp->dom, l);
    return a;
  }
  __device__ __forceinline__ i64 id() const { return lane_i64(C.id_, l); }
  __device__ __forceinline__ i64 ver() const { return lane_i64(C.ver_, l); }
  __device__ __forceinline__ i64 ts() const { return lane_i64(C.ts_, l); }
  __device__ __forceinline__ i64 task() const { return 0; }
  __device__ __forceinline__ i64 ref() const { return lane_i64(C.ref_, l); }
  __device__ __forceinline__ u32 key() const { return lane_u32(C.key_, l); }
  __device__ __forceinline__ i32 aux() const { return (i32)lane_u32((u32)C.aux_, l); }
};

// ---------------------------------------------------------------------------------------------------
// generateMutableStateChecksum (checksum.go:36-114) -> GenerateCRC32 (crc.go:35-54) over
// 0x59 + MutableStateChecksumPayload.Encode (.gen/go/checksum/checksum.go:539-821).
// The VersionHistory branch token the checksum covers, fetched whole before it is needed: its words
// are issued back to back (one memory round trip) instead of one dependent load per CRC block.
// Tokens are 96 bytes (NewHistoryBranchToken's thrift HistoryBranch); longer or unaligned ones take
// the byte loop for what the prefetched words do not cover.
struct TokenDesc { u32 so, sl, fo, fl; };  // crr_workflow start / final token offsets and lengths
__device__ __forceinline__ TokenDesc token_desc(const crr_workflow* wfp) {
  return TokenDesc{wfp->start_token_off, wfp->start_token_len, wfp->final_token_off, wfp->final_token_len};
}
struct TokenWords {
  static constexpr int kWords = 12;
  u64 w[kWords];
  u32 off, len, held;  // held: bytes in w (a multiple of 8)
  u32 raw;             // spliced: the start token's raw CRC (crr_inputs.token_crc), no word read
  bool spliced;
  __device__ __forceinline__ void issue(const TokenDesc& d, i32 token_src, const uint8_t* arena,
                                        const uint32_t* token_crc = nullptr, u32 wi = 0) {
    off = 0; len = 0;
    if (token_src == 1) { off = d.so; len = d.sl; }
    if (token_src == 2) { off = d.fo; len = d.fl; }
    spliced = token_src == 1 && token_crc != nullptr && len == kSpliceBytes;
    raw = spliced ? token_crc[wi] : 0u;
    held = (off & 7u) || spliced ? 0u : (len & ~7u);
    held = held < 8u * kWords ? held : 8u * kWords;
    const u64* tw = reinterpret_cast<const u64*>(arena + off);
#pragma unroll
    for (int j = 0; j < kWords; ++j) w[j] = (8u * j + 8u <= held) ? tw[j] : 0ull;
  }
};

template <class IDS>
// last_id / last_ver (have_last): the last version-history item as the replay holds it in registers (the
// row it just wrote is not read back: a store -> load round trip per workflow)
// sink (crr_outputs.live_ids, NULL or five columns): every ID the lists encode is also stored at its slot
// of the live-ID sidecar (by `sink_writer` lanes only: the wave path's lanes all compute the same payload)
__device__ __forceinline__ u32 payload_crc(const crr_exec_row& R, const IDS& ids, const Geo& G, const TokenWords& TW,
                                           const uint8_t* arena, const u32* tables, u32* out_len,
                                           bool have_last = false, i64 last_id = 0, i64 last_ver = 0,
                                           int64_t* const* sink = nullptr, bool sink_writer = false) {
  Crc K;
  K.init(tables);
  K.u8(0x59);                                                            // preambleVersion0
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
  const bool sk = sink != nullptr && sink_writer;
  auto put = [&](int t, i64 base, i32 i, i64 id) {
    if (sk) sink[t][base + (i64)i * G.st] = id;
    K.be64(id);
  };
  K.list_header(45, 10, (u32)R.n_timer);                                 // PendingTimerStartedIDs
  for (i32 i = 0; i < R.n_timer; ++i) put(1, G.timer_base, i, ids.timer_id(G, i));
  K.list_header(46, 10, (u32)R.n_activity);                              // PendingActivityScheduledIDs
  for (i32 i = 0; i < R.n_activity; ++i) put(0, G.act_base, i, ids.act_id(G, i));
  K.list_header(47, 10, (u32)R.n_signal);                                // PendingSignalInitiatedIDs
  for (i32 i = 0; i < R.n_signal; ++i) put(4, G.sig_base, i, ids.sig_id(G, i));
  K.list_header(48, 10, (u32)R.n_rc);                                    // PendingReqCancelInitiatedIDs
  for (i32 i = 0; i < R.n_rc; ++i) put(3, G.rc_base, i, ids.rc_id(G, i));
  K.list_header(49, 10, (u32)R.n_child);                                 // PendingChildInitiatedIDs
  for (i32 i = 0; i < R.n_child; ++i) put(2, G.child_base, i, ids.child_id(G, i));
  K.field(11, 55); K.be32(0);                                            // StickyTaskListName ""
  K.field(12, 56);                                                       // VersionHistories (shared.go:91639)
  K.field(8, 10); K.be32(0);                                             //   CurrentVersionHistoryIndex
  K.list_header(20, 12, 1u);                                             //   Histories: list<struct> of 1
  const u32 tlen = TW.len;
  K.field(11, 10); K.be32(tlen);                                         //   VersionHistory.BranchToken (shared.go:92043)
  if (TW.spliced) {
    K.splice(TW.raw);   // the token's precomputed contribution (crr_inputs.token_crc)
  } else {
#pragma unroll
    for (int j = 0; j < TokenWords::kWords; ++j)
      if (8u * j + 8u <= TW.held) K.push(TW.w[j], 8);
    const uint8_t* tp = arena + TW.off;
    u32 i = TW.held;
    if ((TW.off & 7u) == 0) {
      const u64* tw = reinterpret_cast<const u64*>(tp);
      for (; i + 8 <= tlen; i += 8) K.push(tw[i >> 3], 8);
    }
    for (; i < tlen; ++i) K.u8(tp[i]);
  }
  K.list_header(20, 12, (u32)R.n_vh_items);
  for (i32 i = 0; i < R.n_vh_items; ++i) {                               //   VersionHistoryItem (shared.go:92375)
    const bool reg = have_last && i == R.n_vh_items - 1;
    const i64 eid = reg ? last_id : G.vh(i)->event_id;
    const i64 ever = reg ? last_ver : G.vh(i)->version;
    K.field(10, 10); K.be64(eid);
    K.field(10, 20); K.be64(ever);
    K.u8(0);
  }
  K.u8(0);  // VersionHistory stop
  K.u8(0);  // VersionHistories stop
  K.u8(0);  // payload stop
  *out_len = K.len;
  return K.finish();
}

// ---------------------------------------------------------------------------------------------------
// GenerateWorkflowCloseTasks (task_generator.go:168-258): the close transfer task (its cross-cluster
// shape is the host's, from cluster metadata) and DeleteHistoryEventTask at close + retention
__device__ __forceinline__ void close_tasks(Lane& L, const Geo& G, const TaskSink& K, i64 ver, i64 ts, i32 s,
                                            i32 retention_days) {
  K.add(L, G, CRR_TASK_CLOSE_EXECUTION, 0, ver, 0, 0, 0, s);
  K.add(L, G, CRR_TASK_DELETE_HISTORY, 0, ver, add_seconds(ts, (i64)retention_days * 86400), 0, 0, s);
}

// Pending-map operations of the dispatch.  The 42-way switch below only decides which one an event
// performs (after the checks that precede it in Go); the operation itself runs after the switch, at
// one program point for every lane of the wavefront -- in a divergent wavefront (lane per workflow,
// mixed event types) each map's code then runs once per step instead of once per event type that
// touches it -- followed by what the transition does after it (its task, a late domain check).

// A map operation through the policy's per-operation methods (a policy may fuse them instead:
// P::kFusedMapOps, P::map_op)
template <class P, class EV>
__device__ __forceinline__ int map_op_by_method(P& T, Lane& L, const Geo& G, u32 op, const EV& ev, i32 s,
                                                i64 batch_first_id, const crr_activity_side& as) {
  switch (op) {
    case MOP_ACT_INSERT: return T.act_insert(L, G, activity_row(ev, s, batch_first_id, as));
    case MOP_ACT_START: return T.act_start(L, G, ev.ref(), ev.id(), ev.ver(), s, ev.ts());
    case MOP_ACT_DELETE: T.act_delete(L, G, ev.ref()); return CRR_OK;
    case MOP_ACT_CANCEL: T.act_cancel(L, G, ev.key(), ev.id(), ev.ver(), s); return CRR_OK;
    case MOP_TIMER_START: return T.timer_start(L, G, timer_row(ev, s));
    case MOP_TIMER_DELETE: T.timer_delete(L, G, ev.key()); return CRR_OK;
    case MOP_CHILD_INSERT: return T.child_insert(L, G, child_row(ev, s, batch_first_id));
    case MOP_CHILD_START: return T.child_start(L, G, ev.ref(), ev.id(), s);
    case MOP_CHILD_DELETE: T.child_delete(L, G, ev.ref()); return CRR_OK;
    case MOP_RC_INSERT: return T.init_insert(L, G, true, initiated_row(ev, s, batch_first_id));
    case MOP_RC_DELETE: T.init_delete(L, G, true, ev.ref()); return CRR_OK;
    case MOP_SIG_INSERT: return T.init_insert(L, G, false, initiated_row(ev, s, batch_first_id));
    case MOP_SIG_DELETE: T.init_delete(L, G, false, ev.ref()); return CRR_OK;
    default: return CRR_OK;
  }
}
template <class P, class = void>
struct FusedMapOps { static constexpr bool value = false; };
template <class P>
struct FusedMapOps<P, decltype((void)P::kFusedMapOps)> { static constexpr bool value = P::kFusedMapOps; };

// The map operation an event's transition performs, then what the transition does after it (its task,
// a late domain check).
template <class P, class EV>
__device__ __forceinline__ int map_op_and_after(Lane& L, const Geo& G, P& T, const u32 op, const EV& ev, const i32 s,
                                                const i64 batch_first_id, const crr_activity_side& as, const TaskSink& K) {
  if (op == MOP_NONE) return CRR_OK;
  int rc;
  if constexpr (FusedMapOps<P>::value) rc = T.map_op(L, G, op, ev, s, batch_first_id, as);
  else rc = map_op_by_method(T, L, G, op, ev, s, batch_first_id, as);
  if (rc) return rc;
  if (op == MOP_ACT_INSERT) {
    K.add(L, G, CRR_TASK_ACTIVITY, 0, ev.ver(), 0, ev.id(), 0, s);  // GenerateActivityTransferTasks
  } else if (op == MOP_CHILD_INSERT) {
    K.add(L, G, CRR_TASK_START_CHILD, 0, ev.ver(), 0, ev.id(), 0, s);  // GenerateChildWorkflowTasks
  } else if (op == MOP_RC_INSERT || op == MOP_SIG_INSERT) {
    // Generate{RequestCancel,Signal}ExternalTasks -> getTargetDomainID (task_generator.go:556-559, :604-607)
    if (ev.aux() == CRR_DOMAIN_UNKNOWN) return CRR_ERR_DOMAIN_NOT_FOUND;
    K.add(L, G, op == MOP_RC_INSERT ? CRR_TASK_CANCEL_EXECUTION : CRR_TASK_SIGNAL_EXECUTION, 0, ev.ver(), 0, ev.id(), 0, s);
  }
  return CRR_OK;
}

// One event of ApplyEvents' dispatch (state_builder.go:131-631); returns the Go error's status
// code (CRR_OK: applied).  `t` is a scalar when the caller found it wave-uniform.
// ActivityTaskScheduled's side record: from HBM, or from the chunk's prefetch (WaveEv::act_side)
template <class EV, class = void>
struct HasActSide { static constexpr bool value = false; };
template <class EV>
struct HasActSide<EV, decltype((void)&EV::act_side)> { static constexpr bool value = true; };
template <class EV>
__device__ __forceinline__ crr_activity_side act_side_of(const crr_inputs& in, const EV& ev) {
  if constexpr (HasActSide<EV>::value) return ev.act_side(in);
  else return in.act_side[ev.aux()];
}
template <class P, class EV>
__device__ __forceinline__ int apply_event(const crr_inputs& in, const crr_outputs& out, Lane& L, const Geo& G, P& T,
                                           const EV& ev, const i32 s, const i32 t, const i64 batch_first_id,
                                           const i64 now_ns, const TaskSink& K, const i32 retention_days) {
  const i64 id = ev.id();
  const i64 ver = ev.ver();
  u32 op = MOP_NONE;
  crr_activity_side as{};
#define FAIL(code, step) return (code)
#define CHECK(expr) do { int rc_ = (expr); if (rc_) return rc_; } while (0)
    switch (t) {
      case CRR_EV_WORKFLOW_EXECUTION_STARTED: {  // :132-183 -> mutable_state_builder.go:1751-1829
        const crr_start_side ss = in.start_side[ev.aux()];
        if (ss.parent_domain_status == CRR_DOMAIN_UNKNOWN) FAIL(CRR_ERR_DOMAIN_NOT_FOUND, s);
        L.decision_start_to_close = ss.decision_start_to_close;
        L.start_src = s;
        CHECK(update_state(L, CRR_STATE_CREATED, CRR_CLOSE_NONE));
        L.last_processed_event = CRR_EMPTY_EVENT_ID;
        L.last_first_event_id = id;
        L.decision_version = CRR_EMPTY_VERSION;
        L.decision_schedule_id = CRR_EMPTY_EVENT_ID;
        L.decision_started_id = CRR_EMPTY_EVENT_ID;
        L.decision_request_src = CRR_SRC_EMPTY_UUID;
        L.decision_timeout = 0;
        // AutoResetPoints = rolloverAutoResetPointsWithExpiringTime(PrevAutoResetPoints, ...) (:3343-3364)
        T.rp_reset(L);
        L.flags = (L.flags & ~CRR_EXEC_RESET_POINTS_SET) | (ss.prev_reset_count != -1 ? CRR_EXEC_RESET_POINTS_SET : 0u);
        for (i32 i = 0; i < ss.prev_reset_count; ++i) {
          crr_reset_point_row rp;
          rp.src = s;
          rp.prev_index = i;
          rp.key = in.reset_keys[ss.prev_reset_key_off + i];
          rp.flags = CRR_ROW_LIVE;
          CHECK(T.rp_push(L, G, rp));
        }
        if (ss.expiration_ns != 0) L.expiration_ns = ss.expiration_ns;  // (:1800-1802)
        // GenerateRecordWorkflowStartedTasks / GenerateWorkflowStartTasks (task_generator.go:143-166, :301-313)
        K.add(L, G, CRR_TASK_RECORD_WORKFLOW_STARTED, 0, ver, 0, 0, 0, s);
        if (K.on) {
          i64 vis = add_seconds(ev.ts(), (i64)ss.workflow_timeout + (i64)ss.first_decision_backoff);
          if (ss.attempt > 0 && L.expiration_ns != 0 && vis > L.expiration_ns) vis = L.expiration_ns;
          K.add(L, G, CRR_TASK_WORKFLOW_TIMEOUT, 0, ver, vis, 0, 0, s);
        }
        // GenerateDelayedDecisionTasks (mutable_state_task_generator.go:260-299)
        if (ss.first_decision_backoff > 0) {
          if (ss.initiator != CRR_INITIATOR_NIL && ss.initiator != CRR_INITIATOR_RETRY_POLICY &&
              ss.initiator != CRR_INITIATOR_CRON)
            FAIL(CRR_ERR_BAD_INITIATOR, s);
          K.add(L, G, CRR_TASK_WORKFLOW_BACKOFF, ss.initiator == CRR_INITIATOR_RETRY_POLICY ? CRR_BACKOFF_RETRY : CRR_BACKOFF_CRON,
                ver, add_seconds(ev.ts(), ss.first_decision_backoff), 0, 0, s);
        }
        L.token_src = 1;  // SetHistoryTree(runID) (:367-376)
        break;
      }
      case CRR_EV_DECISION_TASK_SCHEDULED: {  // :185-208 -> decision_task_manager.go:129-166
        if (L.state != CRR_STATE_ZOMBIE) CHECK(update_state(L, CRR_STATE_RUNNING, CRR_CLOSE_NONE));
        update_decision(L, ver, id, CRR_EMPTY_EVENT_ID, CRR_SRC_EMPTY_UUID, ev.aux(), ev.ref(), 0, ev.ts(), ev.ts());
        K.add(L, G, CRR_TASK_DECISION, 0, L.decision_version, 0, L.decision_schedule_id, 0, s);  // GenerateDecisionScheduleTasks
        break;
      }
      case CRR_EV_DECISION_TASK_STARTED: {  // :210-228 -> decision_task_manager.go:199-242
        if (ev.ref() != L.decision_schedule_id) FAIL(CRR_ERR_DECISION_NOT_FOUND, s);
        update_decision(L, ver, ev.ref(), id, s, L.decision_timeout, 0, ev.ts(), L.decision_scheduled_ts,
                        L.decision_orig_scheduled_ts);
        // GenerateDecisionStartTasks (task_generator.go:352-388)
        K.add(L, G, CRR_TASK_DECISION_TIMEOUT, CRR_TIMEOUT_START_TO_CLOSE, L.decision_version,
              add_seconds(ev.ts(), L.decision_timeout), L.decision_schedule_id, (i32)L.decision_attempt, s);
        break;
      }
      case CRR_EV_DECISION_TASK_COMPLETED: {  // :230-235 -> decision_task_manager.go:244-249, :827-838
        update_decision(L, CRR_EMPTY_VERSION, CRR_EMPTY_EVENT_ID, CRR_EMPTY_EVENT_ID, CRR_SRC_EMPTY_UUID, 0, 0, 0, 0,
                        L.decision_orig_scheduled_ts);  // DeleteDecision
        L.last_processed_event = ev.ref();
        if (ev.key() != 0 && !T.rp_has(L, G, ev.key())) {  // addBinaryCheckSumIfNotExists (:1911-1974)
          crr_reset_point_row rp;
          rp.src = s;
          rp.prev_index = -1;
          rp.key = ev.key();
          const bool resettable = L.n_child == 0 && L.n_rc == 0 && L.n_sig == 0;  // CheckResettable (:1977-1994)
          rp.flags = CRR_ROW_LIVE | (resettable ? CRR_ROW_RESETTABLE : 0u);
          CHECK(T.rp_push(L, G, rp));
          L.flags |= CRR_EXEC_RESET_POINTS_SET;
        }
        break;
      }
      case CRR_EV_DECISION_TASK_TIMED_OUT:  // :237-259 (StickyTaskList == "": incrementAttempt)
      case CRR_EV_DECISION_TASK_FAILED:     // :261-281
        if (fail_decision_and_transient(L, now_ns))  // the transient decision's schedule task (task list of the start event)
          K.add(L, G, CRR_TASK_DECISION, 0, L.decision_version, 0, L.decision_schedule_id, 0, L.start_src);
        break;
      case CRR_EV_ACTIVITY_TASK_SCHEDULED: {  // :283-295 -> mutable_state_builder.go:2142-2197
        as = act_side_of(in, ev);
        if (as.domain_status == CRR_DOMAIN_UNKNOWN) FAIL(CRR_ERR_DOMAIN_NOT_FOUND, s);
        op = MOP_ACT_INSERT;  // then GenerateActivityTransferTasks (below)
        break;
      }
      case CRR_EV_ACTIVITY_TASK_STARTED:  // :297-302 -> :2254-2276
        op = MOP_ACT_START;
        break;
      case CRR_EV_ACTIVITY_TASK_COMPLETED:
      case CRR_EV_ACTIVITY_TASK_FAILED:
      case CRR_EV_ACTIVITY_TASK_TIMED_OUT:
      case CRR_EV_ACTIVITY_TASK_CANCELED:  // :304-337 -> DeleteActivity (:1310-1339)
        op = MOP_ACT_DELETE;
        break;
      case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED:  // :325-330 -> :2444-2467
        op = MOP_ACT_CANCEL;
        break;
      case CRR_EV_TIMER_STARTED:  // :342-347 -> :3057-3081
        op = MOP_TIMER_START;
        break;
      case CRR_EV_TIMER_FIRED:
      case CRR_EV_TIMER_CANCELED:  // :349-361 -> DeleteUserTimer (:1390-1419)
        op = MOP_TIMER_DELETE;
        break;
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED:  // :366-381 -> :3417-3453
        if (ev.aux() == CRR_DOMAIN_UNKNOWN) FAIL(CRR_ERR_DOMAIN_NOT_FOUND, s);
        op = MOP_CHILD_INSERT;  // then GenerateChildWorkflowTasks (below)
        break;
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED:  // :390-395 -> :3485-3507
        op = MOP_CHILD_START;
        break;
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED:  // DeletePendingChildExecution (:1160-1178)
        op = MOP_CHILD_DELETE;
        break;
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED:  // :432-447 -> :2760-2779 (then its task, below)
        op = MOP_RC_INSERT;
        break;
      case CRR_EV_SIGNAL_EXTERNAL_INITIATED:  // :463-478 -> :2883-2905
        op = MOP_SIG_INSERT;
        break;
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED:
      case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED:  // DeletePendingRequestCancel (:1181-1199)
        op = MOP_RC_DELETE;
        break;
      case CRR_EV_SIGNAL_EXTERNAL_FAILED:
      case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED:  // DeletePendingSignal (:1202-1220)
        op = MOP_SIG_DELETE;
        break;
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
        CHECK(update_state(L, CRR_STATE_COMPLETED, cs));
        L.completion_event_batch_id = batch_first_id;
        close_tasks(L, G, K, ver, ev.ts(), s, retention_days);
        break;
      }
      case CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW: {  // :587-627 -> :3366-3382
        const i32 nr = ev.aux();
        if (nr >= 0) {
          if ((u32)nr >= in.n_wf) FAIL(CRR_ERR_NEW_RUN_MISSING, s);
          const int nst = out.exec[nr].status;  // written by the phase-0 launches
          if (nst != CRR_OK) FAIL(nst, s);
        }
        CHECK(update_state(L, CRR_STATE_COMPLETED, CRR_CLOSE_CONTINUED_AS_NEW));
        L.completion_event_batch_id = batch_first_id;
        close_tasks(L, G, K, ver, ev.ts(), s, retention_days);
        break;
      }
      case CRR_EV_REQUEST_CANCEL_ACTIVITY_TASK_FAILED:  // :339-340
      case CRR_EV_CANCEL_TIMER_FAILED:                  // :363-364
      case CRR_EV_MARKER_RECORDED:                      // :494-495
        break;
      case CRR_EV_UPSERT_WORKFLOW_SEARCH_ATTRIBUTES:    // :511-515 (map merge: host materialised)
        K.add(L, G, CRR_TASK_UPSERT_SEARCH_ATTRIBUTES, 0, L.current_version, 0, 0, 0, s);  // GenerateWorkflowSearchAttrTasks
        break;
      default:  // :629-630
        FAIL(CRR_ERR_UNKNOWN_EVENT_TYPE, s);
    }
#undef CHECK
#undef FAIL
  return map_op_and_after(L, G, T, op, ev, s, batch_first_id, as, K);
}

template <class P, class = void>
struct BeforeRetry { static constexpr bool value = false; };
template <class P>
struct BeforeRetry<P, decltype((void)&P::before_retry)> { static constexpr bool value = true; };
template <class P, class = void>
struct LaneDispatch { static constexpr bool value = true; };
template <class P>
struct LaneDispatch<P, decltype((void)P::kLaneDispatch)> { static constexpr bool value = P::kLaneDispatch; };
// types whose transition is more than a handful of field updates: the start event, the closes and
// continue-as-new (once per run each), and anything unknown
constexpr u64 kLaneRare = (1ull << CRR_EV_WORKFLOW_EXECUTION_STARTED) | (1ull << CRR_EV_WORKFLOW_EXECUTION_COMPLETED) |
                          (1ull << CRR_EV_WORKFLOW_EXECUTION_FAILED) | (1ull << CRR_EV_WORKFLOW_EXECUTION_TIMED_OUT) |
                          (1ull << CRR_EV_WORKFLOW_EXECUTION_CANCELED) | (1ull << CRR_EV_WORKFLOW_EXECUTION_TERMINATED) |
                          (1ull << CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW) | (~0ull << CRR_EV_TYPE_COUNT);

// apply_event for a wavefront whose lanes hold different event types.  The per-lane switch runs every
// case some lane needs, one exec-masked region after another, and merges the Lane fields each case
// writes at its exit (copies and mask bookkeeping: ~900 SALU + VALU per step on mixed histories).
// Here the common types are one straight-line pass: each lane's effect on the decision sub-state, the
// workflow state and the counters is a select between the old value and the new, and the map
// operation is looked up in a table; the start / close / continue-as-new events (and task emission)
// take apply_event under their lanes' mask.  Same updates, in the same order, with the same errors
// (a failing event changes nothing before its Go error, except what Go itself applies first).
template <class P>
__device__ __forceinline__ int apply_event_lanes(const crr_inputs& in, const crr_outputs& out, Lane& L, const Geo& G, P& T,
                                                 const Ev& ev, const i32 s, const i32 t, const i64 batch_first_id,
                                                 const i64 now_ns, const TaskSink& K, const i32 retention_days) {
  if (K.on || ((kLaneRare >> (t & 63)) & 1) || t >= 64)
    return apply_event(in, out, L, G, T, ev, s, t, batch_first_id, now_ns, K, retention_days);
  const bool is_ds = t == CRR_EV_DECISION_TASK_SCHEDULED, is_dt = t == CRR_EV_DECISION_TASK_STARTED;
  const bool is_dc = t == CRR_EV_DECISION_TASK_COMPLETED;
  const bool is_df = t == CRR_EV_DECISION_TASK_TIMED_OUT || t == CRR_EV_DECISION_TASK_FAILED;
  // the checks that precede any update
  int rc = CRR_OK;
  // DecisionTaskScheduled: UpdateWorkflowStateCloseStatus(Running, None) unless Zombie (:185-208)
  if (is_ds) rc = L.state == CRR_STATE_COMPLETED ? (int)CRR_ERR_INVALID_STATE_TRANSITION
                : (u32)L.state > (u32)CRR_STATE_VOID ? (int)CRR_ERR_UNKNOWN_WORKFLOW_STATE : (int)CRR_OK;
  if (is_dt && ev.ref() != L.decision_schedule_id) rc = CRR_ERR_DECISION_NOT_FOUND;  // :210-228
  crr_activity_side as{};
  if (t == CRR_EV_ACTIVITY_TASK_SCHEDULED) {  // :283-295
    as = in.act_side[ev.aux()];
    if (as.domain_status == CRR_DOMAIN_UNKNOWN) rc = CRR_ERR_DOMAIN_NOT_FOUND;
  }
  if (t == CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED && ev.aux() == CRR_DOMAIN_UNKNOWN) rc = CRR_ERR_DOMAIN_NOT_FOUND;
  if (rc) return rc;
  // the workflow state of DecisionTaskScheduled
  const bool run = is_ds && L.state != CRR_STATE_ZOMBIE;
  L.state = run ? (i32)CRR_STATE_RUNNING : L.state;
  L.close_status = run ? (i32)CRR_CLOSE_NONE : L.close_status;
  // the decision sub-state: UpdateDecision (decision_task_manager.go:697-721) with each type's arguments --
  // Scheduled (:129-166), Started (:199-242), Completed = DeleteDecision (:244-249, :827-838), TimedOut /
  // Failed = FailDecision + the transient decision (:643-676, :168-197)
  const i64 a1 = L.decision_attempt + 1;
  const bool tr = is_df && a1 != 0;  // the transient decision is scheduled
  const bool dec = is_ds || is_dt || is_dc || is_df;
  if (dec) {
    const i64 nv = (is_ds || is_dt) ? ev.ver() : tr ? L.current_version : (i64)CRR_EMPTY_VERSION;
    const i64 nsched = is_ds ? ev.id() : is_dt ? ev.ref() : tr ? L.next_event_id : (i64)CRR_EMPTY_EVENT_ID;
    const i64 nstarted = is_dt ? ev.id() : (i64)CRR_EMPTY_EVENT_ID;
    const i32 nreq = is_dt ? s : (i32)CRR_SRC_EMPTY_UUID;
    const i32 nto = is_ds ? ev.aux() : is_dt ? L.decision_timeout : tr ? L.decision_start_to_close : 0;
    const i64 natt = is_ds ? ev.ref() : is_df ? a1 : 0;
    const i64 nsts = is_dt ? ev.ts() : 0;
    const i64 nscts = is_ds ? ev.ts() : is_dt ? L.decision_scheduled_ts : is_df ? now_ns : 0;
    const i64 nots = is_ds ? ev.ts() : (is_dt || is_dc) ? L.decision_orig_scheduled_ts : 0;
    update_decision(L, nv, nsched, nstarted, nreq, nto, natt, nsts, nscts, nots);
  }
  L.last_processed_event = is_dc ? ev.ref() : L.last_processed_event;
  L.signal_count = (i32)((u32)L.signal_count + (t == CRR_EV_WORKFLOW_EXECUTION_SIGNALED ? 1u : 0u));  // :497-502
  L.flags |= t == CRR_EV_WORKFLOW_EXECUTION_CANCEL_REQUESTED ? (u32)CRR_EXEC_CANCEL_REQUESTED : 0u;  // :504-509
  if (is_dc && ev.key() != 0 && !T.rp_has(L, G, ev.key())) {  // addBinaryCheckSumIfNotExists (:1911-1974)
    crr_reset_point_row rp;
    rp.src = s;
    rp.prev_index = -1;
    rp.key = ev.key();
    const bool resettable = L.n_child == 0 && L.n_rc == 0 && L.n_sig == 0;  // CheckResettable (:1977-1994)
    rp.flags = CRR_ROW_LIVE | (resettable ? CRR_ROW_RESETTABLE : 0u);
    rc = T.rp_push(L, G, rp);
    if (rc) return rc;
    L.flags |= CRR_EXEC_RESET_POINTS_SET;
  }
  constexpr u64 w0 = mop_word(0), w1 = mop_word(1), w2 = mop_word(2);
  const u64 w = t < 16 ? w0 : t < 32 ? w1 : w2;
  const u32 op = (u32)(w >> (4 * (t & 15))) & 15u;
  return map_op_and_after(L, G, T, op, ev, s, batch_first_id, as, K);
}

// ---- RefreshTasks' tasks (mutable_state_task_refresher.go:77-496) after a Rebuild's replay ---------------
// getNextDecisionTimeout (mutable_state_task_generator.go:1051-1064), durations in ns, rand.Intn(jitterPortion)
// taken as the injected draw mod jitterPortion (crr_start_side.refresh_jitter)
__device__ __forceinline__ i64 next_decision_timeout(i64 attempt, i64 default_ns, i64 draw) {
  if (attempt <= 1) return default_ns;
  double next = attempt >= 5 ? 300e9 : 60e9 * (double)(1ll << (attempt - 2));  // 1m * 2^(attempt-2): exact
  next = next < 300e9 ? next : 300e9;                                          // capped at 5m
  i64 jp = (i64)(0.2 * next);
  if (jp < 1) jp = 1;
  next = next * 0.8 + (double)(i64)((u64)draw % (u64)jp);  // (1 - defaultJitterCoefficient): the constant 0.8
  return (i64)next;
}
// Head of RefreshTasks, before the rows are final: the start / close / record-started / decision tasks
// (refreshTasksForWorkflowStart, ...Close, ...RecordWorkflowStarted, ...Decision, :172-276).  Returns a
// Go error's status (GetStartEvent / GetCompletionEvent find nothing, a bad delayed-decision initiator).
template <class SRC>
__device__ __forceinline__ int refresh_tasks_head(const crr_inputs& in, Lane& L, const Geo& G, const TaskSink& K,
                                                  const SRC& src, i32 n_ev, i64 now_ns, i32 retention_days) {
  L.n_tasks = 0;  // CloseTransactionAsSnapshot (state_rebuilder.go:181) dropped the replay's tasks
  // GetStartEvent (mutable_state_builder.go:1131-1157): the event with ID FirstEventID, the start event
  const i32 ss = L.start_src - L.src_base;
  if (L.start_src < 0 || ss < 0 || ss >= n_ev) return CRR_ERR_MISSING_START_EVENT;
  const i64 sx = src.begin + (i64)ss * src.st;
  if (src.E.event_id[sx] != CRR_FIRST_EVENT_ID) return CRR_ERR_MISSING_START_EVENT;
  const crr_start_side sd = in.start_side[src.E.aux[sx]];
  const i64 sver = src.E.version[sx];
  // GenerateWorkflowStartTasks (task_generator.go:143-166), startTime = the rebuild's now (state_rebuilder.go:186)
  i64 vis = add_seconds(now_ns, (i64)sd.workflow_timeout + (i64)sd.first_decision_backoff);
  if (sd.attempt > 0 && L.expiration_ns != 0 && vis > L.expiration_ns) vis = L.expiration_ns;
  K.add(L, G, CRR_TASK_WORKFLOW_TIMEOUT, 0, sver, vis, 0, 0, L.start_src);
  // !HasProcessedOrPendingDecision (decision_task_manager.go:750-752): GenerateDelayedDecisionTasks (:260-299)
  if (L.decision_schedule_id == CRR_EMPTY_EVENT_ID && L.last_processed_event == CRR_EMPTY_EVENT_ID &&
      sd.first_decision_backoff > 0) {
    if (sd.initiator != CRR_INITIATOR_NIL && sd.initiator != CRR_INITIATOR_RETRY_POLICY && sd.initiator != CRR_INITIATOR_CRON)
      return CRR_ERR_BAD_INITIATOR;
    K.add(L, G, CRR_TASK_WORKFLOW_BACKOFF, sd.initiator == CRR_INITIATOR_RETRY_POLICY ? CRR_BACKOFF_RETRY : CRR_BACKOFF_CRON,
          sver, add_seconds(src.E.timestamp[sx], sd.first_decision_backoff), 0, 0, L.start_src);
  }
  if (L.close_status != CRR_CLOSE_NONE) {
    // GetCompletionEvent (mutable_state_builder.go:1085-1128): event NextEventID - 1 from the batch that
    // starts at CompletionEventBatchID -- the last event, its batch the last one
    if (L.state != CRR_STATE_COMPLETED || L.completion_event_batch_id == CRR_EMPTY_EVENT_ID || n_ev < 1 ||
        L.completion_event_batch_id != L.last_first_event_id)
      return CRR_ERR_MISSING_COMPLETION_EVENT;
    const i64 cx = src.begin + (i64)(n_ev - 1) * src.st;
    if (src.E.event_id[cx] != L.next_event_id - 1) return CRR_ERR_MISSING_COMPLETION_EVENT;
    close_tasks(L, G, K, src.E.version[cx], src.E.timestamp[cx], n_ev - 1 + L.src_base, retention_days);
  } else {  // GenerateRecordWorkflowStartedTasks (task_generator.go:301-313)
    K.add(L, G, CRR_TASK_RECORD_WORKFLOW_STARTED, 0, sver, 0, 0, 0, L.start_src);
  }
  if (L.decision_schedule_id != CRR_EMPTY_EVENT_ID) {
    if (L.decision_started_id != CRR_EMPTY_EVENT_ID) {  // GenerateDecisionStartTasks (:352-388)
      i64 stc = (i64)((u64)L.decision_timeout * (u64)kSecond);
      if (L.decision_attempt > 1) {  // the exponential decision timeout, written back (UpdateDecision)
        stc = next_decision_timeout(L.decision_attempt, (i64)((u64)L.decision_start_to_close * (u64)kSecond),
                                    sd.refresh_jitter);
        L.decision_timeout = (i32)(stc / kSecond);
      }
      K.add(L, G, CRR_TASK_DECISION_TIMEOUT, CRR_TIMEOUT_START_TO_CLOSE, L.decision_version,
            (i64)((u64)L.decision_started_ts + (u64)stc), L.decision_schedule_id, (i32)L.decision_attempt, -1);
    } else {  // GenerateDecisionScheduleTasks (:315-350): executionInfo.TaskList, the start event's
      K.add(L, G, CRR_TASK_DECISION, 0, L.decision_version, 0, L.decision_schedule_id, 0, L.start_src);
    }
  }
  return CRR_OK;
}
// The rest, from the final rows (slots 0..n-1 in event-ID order: Go ranges over the maps, an unspecified
// order): each not-started activity's transfer task, the activity timer and the user timer the refresh's
// epilogue created (the only marked activity / timer), each not-started child's, each request-cancel's and
// signal's transfer task, the search-attributes task (:278-490)
__device__ __forceinline__ void refresh_tasks_rows(const crr_inputs& in, Lane& L, const Geo& G, const TaskSink& K) {
  for (i32 i = 0; i < L.n_act; ++i) {
    const crr_activity_row* r = G.act(i);
    if (r->started_id == CRR_EMPTY_EVENT_ID) K.add(L, G, CRR_TASK_ACTIVITY, 0, r->version, 0, r->schedule_id, 0, r->sched_src);
  }
  for (i32 i = 0; i < L.n_act; ++i) {  // CreateNextActivityTimer's task (timer_sequence.go:162-199)
    const crr_activity_row* r = G.act(i);
    const u32 tts = (u32)r->timer_task_status;
    if (tts == 0) continue;
    const i32 y = (tts & CRR_TTS_CREATED_START_TO_CLOSE) ? CRR_TIMEOUT_START_TO_CLOSE
                : (tts & CRR_TTS_CREATED_SCHEDULE_TO_START) ? CRR_TIMEOUT_SCHEDULE_TO_START
                : (tts & CRR_TTS_CREATED_SCHEDULE_TO_CLOSE) ? CRR_TIMEOUT_SCHEDULE_TO_CLOSE : CRR_TIMEOUT_HEARTBEAT;
    const i64 t = y == CRR_TIMEOUT_SCHEDULE_TO_CLOSE ? add_seconds(r->scheduled_time, r->schedule_to_close)
                : y == CRR_TIMEOUT_SCHEDULE_TO_START ? add_seconds(r->scheduled_time, r->schedule_to_start)
                : y == CRR_TIMEOUT_START_TO_CLOSE ? add_seconds(r->started_time, r->start_to_close)
                : add_seconds(max(r->started_time, r->last_heartbeat_time), r->heartbeat);
    K.add(L, G, CRR_TASK_ACTIVITY_TIMEOUT, y, L.current_version, t, r->schedule_id, r->attempt, -1);
    break;
  }
  for (i32 i = 0; i < L.n_timer; ++i) {  // CreateNextUserTimer's task (:127-160)
    const crr_timer_row* r = G.timer(i);
    if (r->task_status != CRR_TIMER_TASK_STATUS_CREATED) continue;
    K.add(L, G, CRR_TASK_USER_TIMER, 0, L.current_version, r->expiry_time, r->started_id, 0, -1);
    break;
  }
  for (i32 i = 0; i < L.n_child; ++i) {  // GenerateChildWorkflowTasks (task_generator.go:449-495)
    const crr_child_row* r = G.child(i);
    if (r->started_id == CRR_EMPTY_EVENT_ID) K.add(L, G, CRR_TASK_START_CHILD, 0, r->version, 0, r->initiated_id, 0, r->src);
  }
  for (i32 i = 0; i < L.n_rc; ++i) {  // GenerateRequestCancelExternalTasks (:497-546)
    const crr_initiated_row* r = G.rc(i);
    K.add(L, G, CRR_TASK_CANCEL_EXECUTION, 0, r->version, 0, r->initiated_id, 0, r->src);
  }
  for (i32 i = 0; i < L.n_sig; ++i) {  // GenerateSignalExternalTasks (:548-597)
    const crr_initiated_row* r = G.sig(i);
    K.add(L, G, CRR_TASK_SIGNAL_EXECUTION, 0, r->version, 0, r->initiated_id, 0, r->src);
  }
  if (in.flags & CRR_IN_ADVANCED_VISIBILITY)  // refreshTasksForWorkflowSearchAttr (:484-490)
    K.add(L, G, CRR_TASK_UPSERT_SEARCH_ATTRIBUTES, 0, L.current_version, 0, 0, 0, -1);
}

// EMIT (compile time): task emission compiled in.  The fast kernels are also built without it, so
// the replay loop of a launch that does not ask for tasks carries none of its registers.
// CRC (compile time): the checksum computed here (every product launch sets it).
// Profiling aid (variant builds only, -DCRR_PHASE_PROF=1; tools/prof_replication.py --phases): wave clock at
// the phase boundaries of replay_body, summed per phase over lane 0 of every lane-path wavefront.
#ifndef CRR_PHASE_PROF
#define CRR_PHASE_PROF 0
#endif
#if CRR_PHASE_PROF
__device__ unsigned long long g_phase_prof[8];
#define CRR_PHASE(k) do { if constexpr (!std::is_same<SRC, WaveSource>::value) ph[k] = __builtin_readcyclecounter(); } while (0)
#else
#define CRR_PHASE(k) do {} while (0)
#endif
// ---- the job's digest, folded into the replay (crr_outputs.digest) -------------------
// Each finalised workflow adds its terms (cadence_replay.h) to its lane's Digest; the kernel, once every
// lane of the wavefront is back on one path, sums the wavefront's lanes (xor-shuffle tree) and lane 0 adds
// the 7 sums to the block's stripe with 64-bit atomics (8 stripes, one 128-byte line each, so a 1M-workflow
// launch's ~110k atomics spread over 56 lines).  Off (NULL) unless a caller asks for it.
struct Digest {
  i64 v[CRR_DIGEST_FIELDS] = {0, 0, 0, 0, 0, 0, 0};
  __device__ __forceinline__ void add(const crr_exec_row& R, i32 n_ev, u64 key) {
    const bool ok = R.status == CRR_OK;
    const u64 crc = (u64)(u32)R.checksum;
    const u64 fw = ((u64)(u32)R.status << 32) | (u64)(u32)R.fail_step;
    v[0] += ok ? (i64)n_ev : 0;
    v[1] += ok ? 1 : 0;
    v[2] += ok ? 0 : 1;
    v[3] += ok ? (i64)crc : 0;
    v[4] = (i64)((u64)v[4] + (ok ? (key ^ crc) : 0ull));
    v[5] += (i64)R.inconsistencies;
    v[6] = (i64)((u64)v[6] + (ok ? 0ull : (key ^ fw)));
  }
};
// The digest's pointers, read from the kernel arguments where they are used: held from the kernel's start
// they take four of the replay loop's scalar registers (config 2's kernel: 31 scalar spills and 2 vector
// ones instead of 10 and none; the digest on cost its kernel ~2 %).  Every kernel that folds a digest takes
// (crr_inputs in, crr_outputs out, ...) first; the kernel-argument segment lays them out in that order at
// their natural alignment.
constexpr size_t kKernargOut = (sizeof(crr_inputs) + alignof(crr_outputs) - 1) / alignof(crr_outputs) * alignof(crr_outputs);
// the two pointers are 8-byte fields at 8-byte-aligned offsets of structs that are 8-byte aligned, so the
// offsets above are exact; every kernel that folds a digest is checked against that signature at the end of
// this file (kDigestKernels)
static_assert(alignof(crr_inputs) == 8 && alignof(crr_outputs) == 8, "kernarg layout: 8-byte aligned ABI structs");
static_assert(offsetof(crr_inputs, digest_keys) % 8 == 0 && offsetof(crr_outputs, digest) % 8 == 0,
              "kernarg layout: digest pointers at 8-byte offsets");
static_assert(offsetof(crr_inputs, digest_keys) + 8 <= sizeof(crr_inputs) &&
                  kKernargOut + offsetof(crr_outputs, digest) + 8 <= kKernargOut + sizeof(crr_outputs),
              "kernarg layout: digest pointers inside the first two arguments");
template <class F>
struct DigestKernelSig : std::false_type {};
template <class... A>
struct DigestKernelSig<void (*)(crr_inputs, crr_outputs, A...)> : std::true_type {};
// (a volatile read of the constant segment: a scalar load at the point of use, not merged with the kernel
// start's)
typedef const __attribute__((address_space(4))) char* kernarg_ptr;
template <class T>
__device__ __forceinline__ T kernarg_late(size_t off) {
  kernarg_ptr ka = (kernarg_ptr)__builtin_amdgcn_kernarg_segment_ptr();
  return *reinterpret_cast<const volatile __attribute__((address_space(4))) T*>(ka + off);
}
__device__ __forceinline__ int64_t* digest_ptr() { return kernarg_late<int64_t*>(kKernargOut + offsetof(crr_outputs, digest)); }
__device__ __forceinline__ const uint64_t* digest_keys_ptr() {
  return kernarg_late<const uint64_t*>(offsetof(crr_inputs, digest_keys));
}
// every lane of the wavefront active (a kernel's last statement, after its per-workflow work returned)
__device__ __forceinline__ void digest_flush(const crr_outputs&, const Digest& D) {
  int64_t* const digest = digest_ptr();
  if (!digest) return;
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(digest + (blockIdx.x % CRR_DIGEST_STRIPES) * CRR_DIGEST_STRIDE);
  // (a field zero in every lane -- the failure terms of an all-OK wavefront -- is skipped; one whose lanes all
  // hold less than 2^26 is summed in 32 bits: one crossbar shuffle per level instead of two)
#pragma unroll
  for (int k = 0; k < CRR_DIGEST_FIELDS; ++k) {
    u64 x = (u64)D.v[k];
    if (__builtin_amdgcn_ballot_w64(x != 0) == 0) continue;
    if (__builtin_amdgcn_ballot_w64(x >= (1ull << 26)) == 0) {
      u32 y = (u32)x;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) y += (u32)__shfl_xor((int)y, off, 64);
      x = y;
    } else {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) x += (u64)__shfl_xor((long long)x, off, 64);
    }
    if ((threadIdx.x & 63) == 0 && x != 0) atomicAdd(dst + k, x);
  }
}

// The same over a block of kWavesPerBlock wavefronts (the LDS kernels' 256 threads): the wavefront sums meet
// in LDS and one wavefront adds the block's -- a quarter of the atomics (measured on config 2's kernel: the
// digest's atomics ~1 % of it, its reductions ~0.5-1 %, the per-workflow terms ~0.5 %).  Every thread of
// the block calls it (a kernel's last statement).
__device__ __forceinline__ void digest_flush_block(const crr_outputs&, const Digest& D) {
  int64_t* const digest = digest_ptr();
  if (!digest) return;
  __shared__ u64 part[kWavesPerBlock][CRR_DIGEST_FIELDS];
  const u32 wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < CRR_DIGEST_FIELDS; ++k) {
    u64 x = (u64)D.v[k];
    if (__builtin_amdgcn_ballot_w64(x != 0) != 0) {
      if (__builtin_amdgcn_ballot_w64(x >= (1ull << 26)) == 0) {
        u32 y = (u32)x;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) y += (u32)__shfl_xor((int)y, off, 64);
        x = y;
      } else {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) x += (u64)__shfl_xor((long long)x, off, 64);
      }
    }
    if (lane == 0) part[wv][k] = x;
  }
  __syncthreads();
  if (threadIdx.x < CRR_DIGEST_FIELDS) {
    u64 x = 0;
#pragma unroll
    for (int i = 0; i < kWavesPerBlock; ++i) x += part[i][threadIdx.x];
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(digest + (blockIdx.x % CRR_DIGEST_STRIPES) * CRR_DIGEST_STRIDE);
    if (x != 0) atomicAdd(dst + threadIdx.x, x);
  }
}

// pre_x: the workflow's exec row already read by the caller (a kernel that expects loaded states issues it
// with the descriptor, one round trip earlier), else nullptr.  dg: the lane's digest terms (nullptr: none).
template <bool EMIT, class P, class SRC>
__device__ __forceinline__ void replay_body(const crr_inputs& in, const crr_outputs& out, u32 w, const crr_workflow* wfp,
                                            const Geo& G, P& T, SRC& src, const u32* crc_tables,
                                            const crr_exec_row* pre_x = nullptr, Digest* dg = nullptr) {
#if CRR_PHASE_PROF
  u64 ph[7] = {0, 0, 0, 0, 0, 0, 0};
#endif
  CRR_PHASE(0);
  const i32 n_ev = wfp->ev_count;
  const i32 empty_at = wfp->empty_batch_at;
  const i64 now_ns = wfp->now_ns;
  // read once: a descriptor field read inside the loop is reloaded every event (stores in between may
  // alias it), and its wait drains the prefetched columns with it
  const i32 retention_days = wfp->retention_days;
  // before any column load: a wait for it would otherwise also wait for those (vmcnt counts in order);
  // pinned, so the (cache-hit) reads complete before the columns are issued
  const u32 wf_flags0 = wfp->flags;
  asm volatile("" ::"v"(wf_flags0), "v"(n_ev), "v"(empty_at));

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
  L.vh_last_id = 0; L.vh_last_ver = 0; L.vh_n = 0; L.token_src = 0;
  L.n_act = L.n_timer = L.n_child = L.n_rc = L.n_sig = L.n_rp = 0;
  L.inconsistencies = 0;
  L.status = CRR_OK; L.fail_step = -1;
  L.n_tasks = 0; L.expiration_ns = 0; L.src_base = 0;
  const TaskSink K{EMIT && (in.flags & CRR_IN_EMIT_TASKS) != 0, T.task_writer()};

  i64 batch_first_id = 0;
  i32 last_task_step = -1;
  bool task_read = false;
  TokenDesc tok{0, 0, 0, 0};  // read after the loop (failed workflows have no checksum: left zero)
#define FAIL(code, step) do { L.status = (code); L.fail_step = (step) + L.src_base; goto done_events; } while (0)
#define CHECK(expr) do { int rc_ = (expr); if (rc_) FAIL(rc_, s); } while (0)
#define CHECK_N(expr) do { int rc_ = (expr); if (rc_) FAIL(rc_, n_ev); } while (0)

  // step 0's columns in flight first: a loaded state's exec row and rows (below) are read meanwhile
  src.start();
  if (!P::fits(n_ev)) {
    L.status = CRR_INTERNAL_RETRY;  // beyond the policy's encodings (CompactTables' 10-bit steps)
    goto done_events;
  }
  if (wf_flags0 & CRR_WF_FLAG_RESUME) {
    if constexpr (P::kResumable) {
      // the loaded state (mutableStateBuilder.Load, mutable_state_builder.go:306-349) from the rows
      const crr_exec_row X = pre_x ? *pre_x : out.exec[w];
      L.state = X.state; L.close_status = X.close_status;
      L.next_event_id = X.next_event_id; L.last_first_event_id = X.last_first_event_id;
      L.last_event_task_id = X.last_event_task_id; L.last_processed_event = X.last_processed_event;
      L.completion_event_batch_id = X.completion_event_batch_id;
      L.decision_version = X.decision_version; L.decision_schedule_id = X.decision_schedule_id;
      L.decision_started_id = X.decision_started_id; L.decision_attempt = X.decision_attempt;
      L.decision_started_ts = X.decision_started_ts; L.decision_scheduled_ts = X.decision_scheduled_ts;
      L.decision_orig_scheduled_ts = X.decision_orig_scheduled_ts;
      L.decision_timeout = X.decision_timeout; L.decision_request_src = X.decision_request_src;
      L.signal_count = X.signal_count; L.decision_start_to_close = X.decision_start_to_close;
      L.start_src = X.start_src;
      L.flags = X.flags & (CRR_EXEC_CANCEL_REQUESTED | CRR_EXEC_RESET_POINTS_SET);
      L.current_version = CRR_EMPTY_VERSION;  // Load: e.currentVersion = common.EmptyVersion (:324)
      L.token_src = X.token_src;
      L.n_act = X.n_activity; L.n_timer = X.n_timer; L.n_child = X.n_child; L.n_rc = X.n_rc; L.n_sig = X.n_signal;
      L.n_rp = X.n_reset_points;
      L.vh_n = X.n_vh_items;
      L.expiration_ns = X.expiration_ns;
      L.src_base = X.src_next;
      if (L.n_act > G.act_cap || L.n_timer > G.timer_cap || L.n_child > G.child_cap || L.n_rc > G.rc_cap ||
          L.n_sig > G.sig_cap || L.n_rp > G.rp_cap || L.vh_n > G.vh_cap || L.vh_n < 0 || L.n_act < 0 ||
          L.n_timer < 0 || L.n_child < 0 || L.n_rc < 0 || L.n_sig < 0 || L.n_rp < 0) {
        L.n_act = L.n_timer = L.n_child = L.n_rc = L.n_sig = L.n_rp = L.vh_n = 0;
        FAIL(CRR_ERR_CAPACITY, 0);
      }
      if (L.vh_n > 0) {
        const crr_vh_item last = *G.vh(L.vh_n - 1);
        L.vh_last_id = last.event_id;
        L.vh_last_ver = last.version;
      }
      if constexpr (FusedMapOps<P>::value) {
        // an arena-held loaded state (compact tiers): the lines the tail reads -- the branch token the
        // checksum covers, the last event's TaskID -- fetched now, with the rows, so those reads hit the L2
        const u32 toff = L.token_src == 2 ? wfp->final_token_off : wfp->start_token_off;
        const u32 tlen = L.token_src == 2 ? wfp->final_token_len : wfp->start_token_len;
        u32 pf0 = 0, pf1 = 0;
        u64 pf2 = 0;
        if ((L.token_src == 1 || L.token_src == 2) && tlen != 0xFFFFFFFFu && tlen > 0) {
          pf0 = in.arena[toff];
          pf1 = in.arena[toff + tlen - 1];
        }
        if (n_ev > 0) pf2 = (u64)src.task_id(n_ev - 1);
        T.load(L, G);
        asm volatile("" ::"v"(pf0), "v"(pf1), "v"(pf2));
      } else {
        T.load(L, G);
      }
      if (L.status != CRR_OK) goto done_events;  // a loaded state the policy cannot hold: general path
      CRR_PHASE(1);
    } else {
      L.status = CRR_INTERNAL_RETRY;  // rows rebuilt from events cannot hold a loaded state: general path
      goto done_events;
    }
  }

  if constexpr (std::is_same<SRC, WaveSource>::value) {
    // every lane holds the same workflow: its state in scalar registers from here on (a loaded state's
    // fields come from per-lane loads, which the compiler would otherwise take as divergent)
    // Wavefront per workflow, a 64-event chunk at a time (lane l: event c0 + l).  The prologue of
    // :98-129 for every event of the chunk runs lane-parallel: each lane checks its (ID, version)
    // against its predecessor's (lane 0 against the state carried in), the version-history items it
    // closes are written at once, and the first lane whose check fails bounds the walk.  The walk
    // then runs the dispatch and the batch epilogue one event at a time.  The prologue does not read
    // the workflow state except through `completed` (UpdateCurrentVersion), which the walk applies
    // per event, and the VH_EMPTY check (only the first event of a history with no items can meet it:
    // lane 0 of the first chunk, against the loaded state).
    const i32 lane = src.lane;
    const u64 below = lane == 0 ? 0ull : (~0ull >> (64 - lane));  // lanes < this one
    // the event count read into a scalar register: loaded per lane, the compiler would take it -- and every
    // chunk bound, failure point and visit mask derived from it -- as divergent, and compile the chunk loop
    // and the walk as exec-masked loops
    const i32 n_wave = uniform32(n_ev);
    for (i32 c0 = 0; c0 < n_wave; c0 += 64) {
      if (c0) src.rotate();
      const Ev& C = src.cur;
      const i32 cnt = n_wave - c0 < 64 ? n_wave - c0 : 64;
      const bool valid = lane < cnt;
      i64 pid = __shfl_up((long long)C.id_, 1, 64), pver = __shfl_up((long long)C.ver_, 1, 64);
      if (lane == 0) { pid = L.vh_last_id; pver = L.vh_last_ver; }
      const bool first = lane == 0 && L.vh_n == 0;
      const bool grow = !first && C.ver_ > pver;
      const u64 gm = __builtin_amdgcn_ballot_w64(valid && (first || grow));
      const i32 nb = L.vh_n + __builtin_popcountll(gm & below);  // items before this event's
      // :98-100 empty batch; UpdateCurrentVersion's VH_EMPTY (mutable_state_builder.go:495-533)
      const i32 rc0 = c0 + lane == empty_at ? (i32)CRR_ERR_EMPTY_HISTORY
                      : (first && L.state == CRR_STATE_COMPLETED) ? (i32)CRR_ERR_VH_EMPTY : 0;
      // :123-128 AddOrUpdateItem(NewVersionHistoryItem(event.ID, event.Version)) (versionHistory.go:32-46, :193-226)
      const i32 vh_rc = (C.id_ < 0 || (C.ver_ < 0 && C.ver_ != CRR_EMPTY_VERSION)) ? (i32)CRR_ERR_VH_INVALID_ITEM
                        : first ? (G.vh_cap < 1 ? (i32)CRR_ERR_CAPACITY : 0)
                        : C.ver_ < pver ? (i32)CRR_ERR_VH_LOWER_VERSION
                        : C.id_ <= pid ? (i32)CRR_ERR_VH_EVENT_ID_NOT_INCREASING
                        : (grow && nb >= G.vh_cap) ? (i32)CRR_ERR_CAPACITY : 0;
      const i32 prc = !valid ? 0 : rc0 ? rc0 : vh_rc;
      const u64 em = __builtin_amdgcn_ballot_w64(prc != 0);
      const i32 lim = em ? (i32)__builtin_ctzll(em) : cnt;  // events before the first failing prologue
      if (valid && grow && lane < lim) {  // the item this event's version change closes
        crr_vh_item* it = G.vh(nb - 1);
        it->event_id = pid;
        it->version = pver;
      }
      const i32 vh_n0 = L.vh_n;
      // the version-history state after event k of the chunk (k >= 0)
#define WAVE_VH_AFTER(k)                                                                          \
      do {                                                                                        \
        L.vh_n = vh_n0 + __builtin_popcountll(gm & (~0ull >> (63 - (k))));                        \
        L.vh_last_id = lane_i64(C.id_, (k));                                                      \
        L.vh_last_ver = lane_i64(C.ver_, (k));                                                    \
      } while (0)
      const u32 tl = C.et & CRR_ETYPE_MASK;
      const bool live = valid && lane < lim;
      // the chunk's side records in flight during the lane-parallel passes below (A/B, config 4: the 256
      // longest runs 4.22-4.27 -> 4.15-4.21 ms together with the tail kernel's HBM-row copy removed; slower
      // beside it: the register pressure of both)
      SidePf SP{0, 0, 0, 0, 0, 0};
      if (valid && tl == CRR_EV_ACTIVITY_TASK_SCHEDULED) {
        const crr_activity_side* a = in.act_side + (u32)C.aux_;
        const int4 w0 = reinterpret_cast<const int4*>(a)[0], w1 = reinterpret_cast<const int4*>(a)[1];
        SP = SidePf{w0.x, w0.y, w0.z, w0.w, w1.x, w1.z};  // has_retry_policy, domain_status
      }
      src.issue_next(c0 >> 6);  // after them: a wait on a side record does not wait on the next chunk
      auto le = [](i32 k) -> u64 { return k < 0 ? 0ull : k >= 63 ? ~0ull : (2ull << k) - 1; };  // lanes <= k
      auto last_in = [](u64 m) -> i32 { return m ? 63 - (i32)__builtin_clzll(m) : -1; };
      // A chunk without the rare types (start, closes, continue-as-new, unknown) on a created or running
      // workflow, with no task emission, is `fast`: its decision events, signals, cancel requests and no-op
      // types are resolved lane-parallel, and the walk visits only the map operations, the reset points of
      // DecisionTaskCompleted and the batch ends whose epilogue has work.  Otherwise it visits every event.
      const bool fast = !K.on && (L.state == CRR_STATE_CREATED || L.state == CRR_STATE_RUNNING) &&
                        __builtin_amdgcn_ballot_w64(live && ((kLaneRare >> tl) & 1)) == 0;
      u64 vm = le(lim - 1), OPS = 0;  // lanes the walk visits; of those, the ones it applies
      i32 stop = lim;
      if (fast) {
        const bool is_ds = tl == CRR_EV_DECISION_TASK_SCHEDULED, is_dt = tl == CRR_EV_DECISION_TASK_STARTED;
        const bool is_dc = tl == CRR_EV_DECISION_TASK_COMPLETED;
        const bool is_df = tl == CRR_EV_DECISION_TASK_TIMED_OUT || tl == CRR_EV_DECISION_TASK_FAILED;
        const u64 DM = __builtin_amdgcn_ballot_w64(live && (is_ds || is_dt || is_dc || is_df));  // decision events
        const u64 DA = __builtin_amdgcn_ballot_w64(live && (is_ds || is_dt || is_dc));  // set the attempt
        const u64 BL = __builtin_amdgcn_ballot_w64(live && (C.et & CRR_ETYPE_BATCH_LAST));
        constexpr u64 mw0 = mop_word(0), mw1 = mop_word(1), mw2 = mop_word(2);
        const u32 mop = (u32)((tl < 16 ? mw0 : tl < 32 ? mw1 : mw2) >> (4 * (tl & 15))) & 15u;
        const u64 MP = __builtin_amdgcn_ballot_w64(live && mop != MOP_NONE);       // map operations
        const u64 RP = __builtin_amdgcn_ballot_w64(live && is_dc && C.key_ != 0);  // addBinaryCheckSumIfNotExists
        // FailDecision's attempt (decision_task_manager.go:643-676): the last attempt-setting decision
        // event's (Scheduled: its own; Started / Completed: 0) plus one per failure since
        const i32 u = last_in(DA & below);
        const i64 ubase = __shfl((long long)(is_ds ? C.ref_ : 0), u < 0 ? lane : u, 64);
        const i64 att = (u < 0 ? L.decision_attempt : ubase) + __builtin_popcountll(DM & below & ~le(u)) + 1;
        // NextEventID when the event is applied: the last batch end's ID + 1 (:642-643)
        const i32 bl = last_in(BL & below);
        const i64 nei = bl < 0 ? L.next_event_id : (i64)__shfl((long long)C.id_, bl < 0 ? lane : bl, 64) + 1;
        // the decision's ScheduleID after each decision event, and DecisionTaskStarted's check (:210-228)
        const i64 dsched = is_ds ? C.id_ : is_dt ? C.ref_ : (is_df && att != 0) ? nei : (i64)CRR_EMPTY_EVENT_ID;
        const i32 pr = last_in(DM & below);
        const i64 psched = (i64)__shfl((long long)dsched, pr < 0 ? lane : pr, 64);
        const u64 DF = __builtin_amdgcn_ballot_w64(live && is_dt && C.ref_ != (pr < 0 ? L.decision_schedule_id : psched));
        stop = DF ? (i32)__builtin_ctzll(DF) : lim;
        // batch ends whose epilogue has work: a map operation in the batch (or dirty maps carried in)
        const u64 seg = le(lane) & ~le(bl);
        const bool carried_dirty = T.dirty_act || T.dirty_timer;
        // DecisionTaskCompleted's reset point (addBinaryCheckSumIfNotExists, :1911-1974): a binary checksum
        // already in the list, or pushed by an earlier event of the chunk, is a no-op -- only the first
        // event of each checksum not yet listed is walked (the list only grows inside a fast chunk)
        u64 RPV = 0;
        for (u64 rpm = RP; rpm;) {
          const i32 j = (i32)__builtin_ctzll(rpm);
          const u32 key = __builtin_amdgcn_readlane(C.key_, j);
          rpm &= ~__builtin_amdgcn_ballot_w64(live && is_dc && C.key_ == key);
          if (!T.rp_has(L, G, key)) RPV |= 1ull << j;
        }
        const u64 EB = __builtin_amdgcn_ballot_w64(live && (C.et & CRR_ETYPE_BATCH_LAST) &&
                                                   ((MP & seg) != 0 || (bl < 0 && carried_dirty)));
        OPS = MP | RPV;
        vm = (OPS | EB) & le(stop - 1);
      }
      const u64 BF = __builtin_amdgcn_ballot_w64(live && (C.et & CRR_ETYPE_BATCH_FIRST));
      constexpr u64 kBatchIdTypes = (1ull << CRR_EV_ACTIVITY_TASK_SCHEDULED) |
                                    (1ull << CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED) |
                                    (1ull << CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED) |
                                    (1ull << CRR_EV_SIGNAL_EXTERNAL_INITIATED);
      // The walk.  A visited DecisionTaskCompleted runs its whole transition: its decision update is
      // overwritten by the chunk's (below), which covers it, and its reset point is the walk's part.
      i32 wfail = -1;
      int wrc = CRR_OK;
      while (vm) {
        const i32 j = (i32)__builtin_ctzll(vm);
        vm &= vm - 1;
        const i32 s = c0 + j;
        const WaveEv ev{C, j, (u32)__builtin_amdgcn_readlane(C.et, j), &SP};
        const u32 et = ev.et;
        i64 bfid = batch_first_id;
        if (!fast) {
          if (et & CRR_ETYPE_BATCH_FIRST) batch_first_id = ev.id();  // firstEvent := history[0] (:101)
          bfid = batch_first_id;
          // :112 UpdateCurrentVersion: a closed workflow keeps its version history's last version
          L.current_version = L.state == CRR_STATE_COMPLETED ? lane_i64(pver, j) : ev.ver();
          last_task_step = s;  // :129 SetLastEventTaskID(event.TaskID): read once, after the loop
        } else if (((1ull << (et & CRR_ETYPE_MASK)) & kBatchIdTypes) != 0) {
          // only the inserts record their batch's first event ID
          const i32 bf = last_in(BF & le(j));
          if (bf >= 0) bfid = lane_i64(C.id_, bf);
        }
        if (!fast || ((OPS >> j) & 1)) {
          // the status is wave-uniform (every lane replays the same workflow), and read as such: a status the
          // compiler takes as divergent makes the walk a divergent loop -- every branch of the visit an
          // exec-mask region and its loop-carried state in VGPRs
          const int rc = uniform32(apply_event(in, out, L, G, T, ev, s + L.src_base, (i32)(et & CRR_ETYPE_MASK), bfid,
                                               now_ns, K, retention_days));
          if (rc) {
            wfail = j;
            wrc = rc;
            break;
          }
        }
        if (et & CRR_ETYPE_BATCH_LAST) {
          T.epilogue(L, G, K);  // :634-640 GenerateActivityTimerTasks / GenerateUserTimerTasks
          if (!fast) {
            L.last_first_event_id = batch_first_id;  // :642-643
            L.next_event_id = ev.id() + 1;
          }
        }
      }
      if (fast) {
        // what the events [0, end) of the chunk did besides the walk (a failing DecisionTaskCompleted has
        // applied its decision update before its reset point failed)
        const i32 end = wfail >= 0 ? wfail : stop;
        const i32 dend = (wfail >= 0 && (__builtin_amdgcn_readlane(tl, wfail) == CRR_EV_DECISION_TASK_COMPLETED)) ? wfail + 1 : end;
        const bool lv = live && lane < dend;  // masks of their own, not the walk's: short live ranges
        const bool is_ds = tl == CRR_EV_DECISION_TASK_SCHEDULED, is_dt = tl == CRR_EV_DECISION_TASK_STARTED;
        const bool is_dc = tl == CRR_EV_DECISION_TASK_COMPLETED;
        const bool is_df = tl == CRR_EV_DECISION_TASK_TIMED_OUT || tl == CRR_EV_DECISION_TASK_FAILED;
        const u64 DM = __builtin_amdgcn_ballot_w64(lv && (is_ds || is_dt || is_dc || is_df));
        const u64 DS = __builtin_amdgcn_ballot_w64(lv && is_ds), DT = __builtin_amdgcn_ballot_w64(lv && is_dt);
        const u64 DC = __builtin_amdgcn_ballot_w64(lv && is_dc);
        const u64 BL = __builtin_amdgcn_ballot_w64(lv && (C.et & CRR_ETYPE_BATCH_LAST));
        const u64 E = le(end - 1);
        const i32 p = last_in(DM);
        if (p >= 0) {  // the last decision event's UpdateDecision (decision_task_manager.go:697-721)
          const i32 tp = (i32)__builtin_amdgcn_readlane(tl, p);
          auto att_at = [&](i32 x) -> i64 {  // a failed / timed-out decision's attempt
            const i32 v = last_in((DS | DT | DC) & le(x - 1));
            const i64 base = v < 0 ? L.decision_attempt : ((DS >> v) & 1) ? lane_i64(C.ref_, v) : 0;
            return base + __builtin_popcountll(DM & le(x) & ~le(v));
          };
          i64 nv, ns, nst = CRR_EMPTY_EVENT_ID, natt = 0, nsts = 0, nscts = 0, nots = 0;
          i32 nreq = CRR_SRC_EMPTY_UUID, nto = 0;
          if (tp == CRR_EV_DECISION_TASK_SCHEDULED) {  // :129-166
            nv = lane_i64(C.ver_, p); ns = lane_i64(C.id_, p); nto = (i32)lane_u32((u32)C.aux_, p);
            natt = lane_i64(C.ref_, p); nscts = lane_i64(C.ts_, p); nots = nscts;
          } else if (tp == CRR_EV_DECISION_TASK_STARTED || tp == CRR_EV_DECISION_TASK_COMPLETED) {
            // the original scheduled time: the last Scheduled (its time) or failure (0) before it
            const i32 r = last_in((DM & ~(DT | DC)) & le(p - 1));
            nots = r < 0 ? L.decision_orig_scheduled_ts : ((DS >> r) & 1) ? lane_i64(C.ts_, r) : 0;
            if (tp == CRR_EV_DECISION_TASK_STARTED) {  // :199-242
              // the timeout and scheduled time: the last decision event before it that sets them
              const i32 q = last_in(DM & ~DT & le(p - 1));
              if (q < 0) {
                nto = L.decision_timeout;
                nscts = L.decision_scheduled_ts;
              } else if ((DS >> q) & 1) {
                nto = (i32)lane_u32((u32)C.aux_, q);
                nscts = lane_i64(C.ts_, q);
              } else if ((DC >> q) & 1) {
                nto = 0;
                nscts = 0;
              } else {  // failed / timed out: the transient decision's
                nto = att_at(q) != 0 ? L.decision_start_to_close : 0;
                nscts = now_ns;
              }
              nv = lane_i64(C.ver_, p); ns = lane_i64(C.ref_, p); nst = lane_i64(C.id_, p);
              nreq = c0 + p + L.src_base; nsts = lane_i64(C.ts_, p);
            } else {  // DeleteDecision (:244-249, :827-838)
              nv = CRR_EMPTY_VERSION; ns = CRR_EMPTY_EVENT_ID;
            }
          } else {  // FailDecision + the transient decision (:643-676, :168-197)
            natt = att_at(p);
            const bool tr = natt != 0;
            const i32 b = last_in(BL & le(p - 1));
            nv = tr ? lane_i64(C.ver_, p) : (i64)CRR_EMPTY_VERSION;
            ns = !tr ? (i64)CRR_EMPTY_EVENT_ID : b < 0 ? L.next_event_id : lane_i64(C.id_, b) + 1;
            nto = tr ? L.decision_start_to_close : 0;
            nscts = now_ns;
          }
          update_decision(L, nv, ns, nst, nreq, nto, natt, nsts, nscts, nots);
        }
        const i32 q = last_in(DC);
        if (q >= 0) L.last_processed_event = lane_i64(C.ref_, q);
        if (DS & E) {  // UpdateWorkflowStateCloseStatus(Running, None) (:185-208)
          L.state = CRR_STATE_RUNNING;
          L.close_status = CRR_CLOSE_NONE;
        }
        const u64 SG = __builtin_amdgcn_ballot_w64(lv && tl == CRR_EV_WORKFLOW_EXECUTION_SIGNALED);  // :497-502
        const u64 CR = __builtin_amdgcn_ballot_w64(lv && tl == CRR_EV_WORKFLOW_EXECUTION_CANCEL_REQUESTED);
        L.signal_count = (i32)((u32)L.signal_count + (u32)__builtin_popcountll(SG & E));
        if (CR & E) L.flags |= CRR_EXEC_CANCEL_REQUESTED;  // :504-509
        const i32 b = last_in(BL & E);
        if (b >= 0) {  // :642-643
          const i32 bf = last_in(BF & le(b));
          L.last_first_event_id = bf < 0 ? batch_first_id : lane_i64(C.id_, bf);
          L.next_event_id = lane_i64(C.id_, b) + 1;
        }
        const i32 f = last_in(BF & E);
        if (f >= 0) batch_first_id = lane_i64(C.id_, f);
        const i32 k = wfail >= 0 ? wfail : stop < lim ? stop : lim - 1;  // the last event whose prologue ran
        if (k >= 0) {
          L.current_version = lane_i64(C.ver_, k);
          last_task_step = c0 + k;
        }
        if (wfail < 0 && stop < lim) {  // DecisionTaskStarted without its decision (:210-228)
          wfail = stop;
          wrc = CRR_ERR_DECISION_NOT_FOUND;
        }
      }
      if (wfail >= 0) {  // the failing event's prologue has run
        WAVE_VH_AFTER(wfail);
        FAIL(wrc, c0 + wfail);
      }
      if (lim > 0) WAVE_VH_AFTER(lim - 1);
      if (lim < cnt) {  // event c0 + lim fails its prologue; a version-history error follows UpdateCurrentVersion
        if (__builtin_amdgcn_readlane((u32)rc0, lim) == 0)
          L.current_version = L.state == CRR_STATE_COMPLETED ? lane_i64(pver, lim) : lane_i64(C.ver_, lim);
        FAIL((i32)__builtin_amdgcn_readlane((u32)prc, lim), c0 + lim);
      }
#undef WAVE_VH_AFTER
    }
  } else
  for (i32 s = 0; s < n_ev; ++s) {
    // one loop exit for the whole prologue: the checks become a select chain (no divergent branch
    // per check), and on success vh_last = (id, ver) in every case (new item, same version, first).
    const Ev ev = src.next(s);
    const u32 et = ev.et;
    const i64 id = ev.id();
    const i64 ver = ev.ver();
    const i32 t = et & CRR_ETYPE_MASK;
    if (et & CRR_ETYPE_BATCH_FIRST) batch_first_id = id;  // firstEvent := history[0] (:101)
    {
      const bool completed = L.state == CRR_STATE_COMPLETED;
      const bool first = L.vh_n == 0;
      const bool grow = !first && ver > L.vh_last_ver;
      // :98-100 empty batch; :112 UpdateCurrentVersion (mutable_state_builder.go:495-533)
      i32 rc0 = s == empty_at ? (i32)CRR_ERR_EMPTY_HISTORY : (completed && first) ? (i32)CRR_ERR_VH_EMPTY : 0;
      if (rc0 == 0) L.current_version = completed ? L.vh_last_ver : ver;
      // :123-128 AddOrUpdateItem(NewVersionHistoryItem(event.ID, event.Version)) (versionHistory.go:32-46, :193-226)
      const i32 vh_rc = (id < 0 || (ver < 0 && ver != CRR_EMPTY_VERSION)) ? (i32)CRR_ERR_VH_INVALID_ITEM
                        : first ? (G.vh_cap < 1 ? (i32)CRR_ERR_CAPACITY : 0)
                        : ver < L.vh_last_ver ? (i32)CRR_ERR_VH_LOWER_VERSION
                        : id <= L.vh_last_id ? (i32)CRR_ERR_VH_EVENT_ID_NOT_INCREASING
                        : (grow && L.vh_n >= G.vh_cap) ? (i32)CRR_ERR_CAPACITY : 0;
      rc0 = rc0 ? rc0 : vh_rc;
      if (rc0) FAIL(rc0, s);
      if (grow) {
        crr_vh_item* it = G.vh(L.vh_n - 1);
        it->event_id = L.vh_last_id;
        it->version = L.vh_last_ver;
      }
      L.vh_n += (first || grow) ? 1 : 0;
      L.vh_last_id = id;
      L.vh_last_ver = ver;
    }
    last_task_step = s;  // :129 SetLastEventTaskID(event.TaskID): read once, after the loop

    // :131-631 the 42-way dispatch.  When every active lane holds the same event type (the
    // common case: histories of one workflow type replay in lockstep) the type is wave-uniform
    // and the switch runs on a scalar register -- scalar branches, no exec-mask tree; otherwise
    // the per-lane switch.
    {
      int rc;
      const i32 tu = uniform32(t);
      const i32 ps = s + L.src_base;  // provenance step of the event (rows' *_src)
      if (__builtin_amdgcn_ballot_w64(t != tu) == 0)
        rc = apply_event(in, out, L, G, T, ev, ps, tu, batch_first_id, now_ns,
                         K, retention_days);
      else if (LaneDispatch<P>::value)
        rc = apply_event_lanes(in, out, L, G, T, ev, ps, t, batch_first_id,
                               now_ns, K, retention_days);
      else
        rc = apply_event(in, out, L, G, T, ev, ps, t, batch_first_id, now_ns,
                         K, retention_days);
      if (rc) FAIL(rc, s);
    }

    if (et & CRR_ETYPE_BATCH_LAST) {
      T.epilogue(L, G, K);  // :634-640 GenerateActivityTimerTasks / GenerateUserTimerTasks
      L.last_first_event_id = batch_first_id;  // :642-643
      L.next_event_id = id + 1;
    }
  }
  {
    // what the tail reads from HBM -- the last TaskID, the token and rebuild fields of the descriptor --
    // issued together, before the first use of any of them: one memory round trip, not a chain
    if (last_task_step >= 0) L.last_event_task_id = src.task_id(last_task_step);
    task_read = true;
    tok.so = wfp->start_token_off; tok.sl = wfp->start_token_len;
    tok.fo = wfp->final_token_off; tok.fl = wfp->final_token_len;
    const u32 final_len = tok.fl;
    const i64 want_id = wfp->rebuild_last_event_id, want_ver = wfp->rebuild_last_event_version;
    const u32 wf_flags = wfp->flags;
    if (empty_at == n_ev) FAIL(CRR_ERR_EMPTY_HISTORY, n_ev);
    if (final_len != 0xFFFFFFFFu) {  // rebuild finalisation (state_rebuilder.go:150-177)
      L.token_src = 2;
      if (L.vh_n == 0) FAIL(CRR_ERR_VH_EMPTY, n_ev);
      if (want_id < 0 || (want_ver < 0 && want_ver != CRR_EMPTY_VERSION)) FAIL(CRR_ERR_VH_INVALID_ITEM, n_ev);
      if (L.vh_last_id != want_id || L.vh_last_ver != want_ver) FAIL(CRR_ERR_REBUILD_LAST_ITEM, n_ev);
    }
    if (wf_flags & CRR_WF_FLAG_REFRESH_TASKS) {  // Rebuild's RefreshTasks (state_rebuilder.go:181-186)
      L.n_tasks = 0;    // CloseTransactionAsSnapshot drops the replay's tasks
      // with or without emission: its Go errors and the DecisionTimeout write-back are state effects (only
      // K.add is compiled out of the non-EMIT instantiations).  Before the timer refresh, as in Go
      // (mutable_state_task_refresher.go:77-170): a failing head leaves the timer task statuses as replayed.
      CHECK_N(refresh_tasks_head(in, L, G, K, src, n_ev, now_ns, retention_days));
      T.refresh(L, G);  // the state effects (the timers re-created: a task each, emitted from the rows below)
    }
  }
done_events:
  CRR_PHASE(2);
#undef CHECK
#undef CHECK_N
#undef FAIL
  if (!task_read && last_task_step >= 0) L.last_event_task_id = src.task_id(last_task_step);

  if (L.status == CRR_OK && K.on && L.n_tasks > G.task_cap) L.status = CRR_ERR_CAPACITY;
  if (L.status == CRR_INTERNAL_RETRY) {  // the GlobalTables pass replays this workflow from scratch
    if constexpr (BeforeRetry<P>::value) T.before_retry(L, G);
    out.exec[w].status = CRR_INTERNAL_RETRY;
    T.retry_push(in, out, w);
    return;
  }
  // the checksum's branch-token words go out before the row write-back, whose work hides their latency
  bool want_crc = L.status == CRR_OK;
  TokenWords TW;
  TW.issue(tok, want_crc ? L.token_src : 0, in.arena, in.token_crc, w);
  // the workflow's digest key with them: read before the loop it would be held across it (registers the
  // loop spills for), read at the add its round trip would end every wavefront
  u64 dkey = 0;
  if (dg && digest_ptr()) dkey = digest_keys_ptr()[w];
  // the wave path's items were written by the lanes of their events; the checksum reads them all
  if constexpr (std::is_same<SRC, WaveSource>::value) wave_sync_global();
  if (L.vh_n > 0) {
    crr_vh_item* it = G.vh(L.vh_n - 1);
    it->event_id = L.vh_last_id;
    it->version = L.vh_last_ver;
  }
  CRR_PHASE(3);
  T.finalize(L, G);
  CRR_PHASE(4);
  if constexpr (EMIT) {  // RefreshTasks' tasks from the final rows
    if (K.on && want_crc && (wfp->flags & CRR_WF_FLAG_REFRESH_TASKS)) {
      if constexpr (std::is_same<SRC, WaveSource>::value) wave_sync_global();
      refresh_tasks_rows(in, L, G, K);
      if (L.n_tasks > G.task_cap) {
        L.status = CRR_ERR_CAPACITY;
        L.fail_step = n_ev + L.src_base;
        want_crc = false;
      }
    }
  }

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
  R.n_tasks = L.n_tasks;
  R.decision_start_to_close = L.decision_start_to_close;
  R.expiration_ns = L.expiration_ns;
  R.src_next = L.src_base + n_ev;
  R.reserved = 0;
  if (want_crc) {
    // the live-ID sidecar (crr_outputs.live_ids) is written with the lists, by one lane of a wavefront-path replay
    int64_t* const* sink = out.live_ids[0] ? out.live_ids : nullptr;
    R.checksum = payload_crc(R, T, G, TW, in.arena, crc_tables, &R.payload_len, true, L.vh_last_id, L.vh_last_ver, sink,
                             !std::is_same<SRC, WaveSource>::value || (threadIdx.x & 63) == 0);
  }
  CRR_PHASE(5);
  out.exec[w] = R;
  // the digest's terms: one lane per workflow (the wave path's lanes all hold the same result)
  if (dg && digest_ptr() && (!std::is_same<SRC, WaveSource>::value || (threadIdx.x & 63) == 0))
    dg->add(R, n_ev, dkey);
#if CRR_PHASE_PROF
  if constexpr (!std::is_same<SRC, WaveSource>::value) {
    if ((wfp->flags & CRR_WF_FLAG_RESUME) && (threadIdx.x & 63) == 0 && ph[1] != 0) {
      atomicAdd(&g_phase_prof[0], ph[1] - ph[0]);  // prologue + load
      atomicAdd(&g_phase_prof[1], ph[2] - ph[1]);  // event loop + tail reads
      atomicAdd(&g_phase_prof[2], ph[3] - ph[2]);  // token issue, VH write
      atomicAdd(&g_phase_prof[3], ph[4] - ph[3]);  // finalize
      atomicAdd(&g_phase_prof[4], ph[5] - ph[4]);  // refresh / exec row / checksum
      atomicAdd(&g_phase_prof[5], 1ull);
    }
  }
#endif
}
#if CRR_PHASE_PROF
extern "C" int crr_phase_prof(unsigned long long* host, int reset) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase_prof), sizeof(g_phase_prof)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase_prof), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// ---- kernels ---------------------------------------------------------------------------------------
// Workflows [0, n_lane) use the batch stride (wave-interleaved: lane per workflow); workflows
// [wave_begin, n_wf) of a CRR_IN_WAVE_TAIL batch are contiguous (stride 1), one per wavefront.
__device__ __forceinline__ u32 lane_count(const crr_inputs& in) {
  return (in.flags & CRR_IN_WAVE_TAIL) ? in.wave_begin : in.n_wf;
}
__device__ __forceinline__ u32 tail_count_end(const crr_inputs& in) {
  return ((in.flags & CRR_IN_TIERED) && in.big_begin >= in.wave_begin && in.big_begin < in.n_wf) ? in.big_begin : in.n_wf;
}
__device__ __forceinline__ i64 wf_stride(const crr_inputs& in, u32 w) {
  return ((in.flags & CRR_IN_WAVE_TAIL) && w >= in.wave_begin) ? 1 : (i64)in.stride;
}

// LDS arena of a block: the lane-per-workflow [slot][lane] tables or 4 per-wave row arenas.
#ifndef CRR_SMALL_CRC  // the lane kernels' CRC tables: 0 built in LDS per block, 1 copied into LDS, 2 none
#define CRR_SMALL_CRC 0
#endif
template <class TIER> struct WaveTier;
template <> struct WaveTier<SmallTier> { using Arena = WaveArena<40, 32, 16, 8, 8, 24>; };
template <> struct WaveTier<LargeTier> { using Arena = WaveArena<64, 48, 24, 16, 16, 32>; };
template <class TIER>
union BlockArena {
  LdsArena<TIER> lane;
  typename WaveTier<TIER>::Arena wave[kWavesPerBlock];
};

// Fast path (stride 64): blocks [0, wave_blocks) replay the long-history tail one workflow per
// wavefront (dispatched first, they run longest), the remaining blocks replay lane per workflow.
template <class TIER, bool WAVE_TAIL, bool EMIT, bool LANES = false>
__device__ __forceinline__ void replay_lds(const crr_inputs& in, const crr_outputs& out, int phase, u32 lo, u32 hi,
                                           Digest& D) {
  static_assert(sizeof(typename WaveTier<TIER>::Arena) * kWavesPerBlock <= sizeof(LdsArena<TIER>),
                "per-wave arenas must fit in the lane arena");
#if CRR_SMALL_CRC == 2
  const u32* crc_tables = kCrcGlobal.v;  // gathers through the L1
#else
  __shared__ u32 crc_tables[8 * 256];
#if CRR_SMALL_CRC == 1
  {  // a copy of the constant-memory tables
    const uint4* src = reinterpret_cast<const uint4*>(kCrcGlobal.v);
    uint4* dst = reinterpret_cast<uint4*>(crc_tables);
#pragma unroll
    for (int i = 0; i < 8 * 256 / 4 / kBlock; ++i) dst[i * kBlock + threadIdx.x] = src[i * kBlock + threadIdx.x];
    __syncthreads();
  }
#else
  build_crc_tables<kBlock>(crc_tables);
#endif
#endif
  __shared__ BlockArena<TIER> arena;
  const u32 n_lane = WAVE_TAIL ? lane_count(in) : in.n_wf;
  const u32 tail_end = WAVE_TAIL ? tail_count_end(in) : in.n_wf;  // [tail_end, n_wf): replay_big_kernel
  const u32 wave_blocks = WAVE_TAIL ? (tail_end - n_lane + kWavesPerBlock - 1) / kWavesPerBlock : 0;
  if (WAVE_TAIL && blockIdx.x < wave_blocks) {
    const u32 wv = (u32)uniform32((i32)(threadIdx.x >> 6));
    const u32 w = n_lane + blockIdx.x * kWavesPerBlock + wv;
    if (w >= tail_end) return;
    const crr_workflow* wfp = in.wf + w;
    if (((wfp->flags & CRR_WF_FLAG_NEW_RUN) != 0) != (phase == 0)) return;
    Geo G;
    load_geo(G, wfp, out, 1);
    WaveLds<typename WaveTier<TIER>::Arena, 1> T;  // outgrown: the retry pass's wave list
    bind_arena(T, &arena.wave[wv]);
    T.init();

    WaveSource S(in.ev, wfp->ev_begin, 1, wfp->ev_count);
    replay_body<EMIT>(in, out, w, wfp, G, T, S, crc_tables, nullptr, &D);
    return;
  }
  const u32 w = lo + (blockIdx.x - wave_blocks) * kBlock + threadIdx.x;  // lanes [lo, hi); launched with kBlock
  if (w >= hi) return;
  const crr_workflow* wfp = in.wf + w;
  // the descriptor in one round trip: the phase test reads its flags after the geometry is loaded
  const i64 lane = threadIdx.x & 63;
  Geo G;
  load_geo(G, wfp, out, 64);
  const i64 ev_begin0 = wfp->ev_begin;
  const i32 ev_count0 = wfp->ev_count;
  const u32 wf_flags = wfp->flags;
  asm volatile("" ::"v"(ev_begin0), "v"(ev_count0), "v"(wf_flags));  // all issued before the phase test's wait
  if (((wf_flags & CRR_WF_FLAG_NEW_RUN) != 0) != (phase == 0)) return;
  uniformize_geo(G, lane);
  const i64 ev_begin = uniform64(ev_begin0 - lane) + lane;
  LdsTables<TIER, LANES> T;
  T.init(&arena.lane, &in, ev_begin);
  LaneSource S(in.ev, ev_begin, 64, wfp->ev_count, EMIT && (in.flags & CRR_IN_EMIT_TASKS) != 0);
  replay_body<EMIT>(in, out, w, wfp, G, T, S, crc_tables, nullptr, &D);
}
template <bool WAVE_TAIL, bool EMIT, bool LANES = false>
#ifndef CRR_SMALL_WAVES_PER_EU
#define CRR_SMALL_WAVES_PER_EU 3
#endif
__global__ void __launch_bounds__(kBlock, EMIT ? 2 : CRR_SMALL_WAVES_PER_EU) replay_lds_small_kernel(crr_inputs in, crr_outputs out, int phase, u32 lo, u32 hi) {
  Digest D;
  replay_lds<SmallTier, WAVE_TAIL, EMIT, LANES>(in, out, phase, lo, hi, D);
  digest_flush_block(out, D);
}
template <bool WAVE_TAIL, bool EMIT>
__global__ void __launch_bounds__(kBlock) replay_lds_kernel(crr_inputs in, crr_outputs out, int phase, u32 lo, u32 hi) {
  Digest D;
  replay_lds<LargeTier, WAVE_TAIL, EMIT>(in, out, phase, lo, hi, D);
  digest_flush_block(out, D);
}
template __global__ void replay_lds_small_kernel<false, false>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_lds_small_kernel<false, false, true>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_lds_small_kernel<true, false>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_lds_kernel<false, false>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_lds_kernel<true, false>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_lds_small_kernel<false, true>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_lds_small_kernel<true, true>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_lds_kernel<false, true>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_lds_kernel<true, true>(crr_inputs, crr_outputs, int, u32, u32);

// General path over HBM slot tables (any layout).  retry_only: replay the workflows the fast path
// handed back (scratch list), grid-striding so the launch is cheap when there are none.
__global__ void __launch_bounds__(kBlock) replay_global_kernel(crr_inputs in, crr_outputs out, int phase, int retry_only) {
  __shared__ u32 crc_tables[8 * 256];
  u32 n_items = in.n_wf;
  if (retry_only) {
    n_items = __hip_atomic_load(out.scratch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n_items == 0) return;  // uniform across the grid
  } else if (blockIdx.x * blockDim.x >= n_items) {
    return;
  }
  build_crc_tables(crc_tables);
  const u32 stride = gridDim.x * blockDim.x;
  Digest D;
  for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < n_items; i += stride) {
    const u32 w = retry_only ? out.scratch[kScratchHeader + i] : i;
    const crr_workflow* wfp = in.wf + w;
    if (((wfp->flags & CRR_WF_FLAG_NEW_RUN) != 0) != (phase == 0)) continue;
    const i64 st = wf_stride(in, w);
    Geo G;
    load_geo(G, wfp, out, st);
    GlobalTables T;
    LaneSource S(in.ev, wfp->ev_begin, st, wfp->ev_count, (in.flags & CRR_IN_EMIT_TASKS) != 0);
    replay_body<true>(in, out, w, wfp, G, T, S, crc_tables, nullptr, &D);
  }
  digest_flush(out, D);
}

// Retry pass over the workflows the fast path handed back (one launch, 64 threads per block,
// 2 blocks/CU; grid-strided, so an empty retry costs one load per block):
//   1. long-tail workflows the fast path's per-wave arenas could not hold (scratch list 1), one
//      wavefront per workflow, first with a 57 KB LDS row arena; a live set that outgrows that is
//      replayed again at once over the workflow's own HBM rows (no size limit);
//   2. lane workflows (list 0), lane per workflow again with the 8/8/4/4/4/8-slot LDS tier (gathered
//      lanes: each reads its own workflow's interleaved columns); a lane that outgrows that replays
//      its workflow again at once over its HBM rows.
// Nothing is pushed during the pass, so no block waits on another.  The last block to finish zeroes
// the list counters, so the next crr_replay needs no memset.
using BigArena = WaveArena<320, 160, 96, 64, 64, 64>;  // the retry pass's wave arena
// replay_big_kernel's: the big segment holds the histories whose live sets the host expects past the wave
// tail's arena (64 activities, 48 timers) -- in config 4 they peak at 65-71 -- so two registers per map
// (WaveRegTables) cover them; a live set past this is replayed again over the 320-slot arena, then HBM rows
#ifndef CRR_BIG_ARENA
#define CRR_BIG_ARENA 128, 128, 64, 64, 64, 64
#endif
using BigSegArena = WaveArena<CRR_BIG_ARENA>;
template <class TT, bool EMIT = true>
__device__ __forceinline__ void replay_wave_item(const crr_inputs& in, const crr_outputs& out, int phase, u32 w,
                                                 TT& T, const u32* crc_tables, Digest& D) {
  const crr_workflow* wfp = in.wf + w;
  if (((wfp->flags & CRR_WF_FLAG_NEW_RUN) != 0) != (phase == 0)) return;
  const i64 st = wf_stride(in, w);
  Geo G;
  load_geo(G, wfp, out, st);
  if constexpr (std::is_same<TT, WaveTables<HbmRows>>::value) T.S.G = G;
  T.init();
  T.hw_act = T.hw_timer = T.hw_child = T.hw_rc = T.hw_sig = 0;
  WaveSource S(in.ev, wfp->ev_begin, st, wfp->ev_count);
  replay_body<EMIT, TT, WaveSource>(in, out, w, wfp, G, T, S, crc_tables, nullptr, &D);
}
__device__ __forceinline__ void replay_lane_item(const crr_inputs& in, const crr_outputs& out, int phase, u32 w,
                                                 LdsArena<HugeTier>* arena, const u32* crc_tables, Digest& D) {
  const crr_workflow* wfp = in.wf + w;
  if (((wfp->flags & CRR_WF_FLAG_NEW_RUN) != 0) != (phase == 0)) return;
  Geo G;
  load_geo(G, wfp, out, 64);
  const bool tasks = (in.flags & CRR_IN_EMIT_TASKS) != 0;
  LdsTables<HugeTier> T;
  T.list = -1;
  T.init(arena, &in, wfp->ev_begin);
  LaneSource S(in.ev, wfp->ev_begin, 64, wfp->ev_count, tasks);
  replay_body<true>(in, out, w, wfp, G, T, S, crc_tables, nullptr, &D);
  if (T.retried) {
    GlobalTables H;
    LaneSource S2(in.ev, wfp->ev_begin, 64, wfp->ev_count, tasks);
    replay_body<true>(in, out, w, wfp, G, H, S2, crc_tables, nullptr, &D);
  }
}
// Wide segment (CRR_IN_TIERED [hbm_begin, lanes)): lane workflows whose live sets the host expects to
// outgrow the compact tiers, and loaded states (CRR_WF_FLAG_RESUME: continued in place over their rows).
// Lane per workflow over the workflows' own HBM rows (GlobalTables: no LDS, so the occupancy is the
// register-limited one; interleaved rows keep slot j of a group one coalesced run).
#ifndef CRR_WIDE_WAVES_PER_EU
#define CRR_WIDE_WAVES_PER_EU 2
#endif
__device__ __forceinline__ void replay_wide(const crr_inputs& in, const crr_outputs& out, int phase, u32 lo, u32 hi,
                                            const u32* crc_tables, Digest& D) {
  const u32 w = lo + blockIdx.x * kBlock + threadIdx.x;
  if (w >= hi) return;
  const crr_workflow* wfp = in.wf + w;
  const i64 lane = threadIdx.x & 63;
  Geo G;  // the descriptor in one round trip, as in replay_lds
  load_geo(G, wfp, out, 64);
  i64 ev_begin = wfp->ev_begin;
  const i32 ev_count0 = wfp->ev_count;
  const u32 wf_flags = wfp->flags;
  asm volatile("" ::"v"(ev_begin), "v"(ev_count0), "v"(wf_flags));
  if (((wf_flags & CRR_WF_FLAG_NEW_RUN) != 0) != (phase == 0)) return;
  if ((lo & 63u) == 0) {  // wavefront == one interleaved group: group-uniform geometry in SGPRs
    uniformize_geo(G, lane);
    ev_begin = uniform64(ev_begin - lane) + lane;
  }
  GlobalTables T;
  LaneSource S(in.ev, ev_begin, 64, wfp->ev_count, (in.flags & CRR_IN_EMIT_TASKS) != 0);
  replay_body<true>(in, out, w, wfp, G, T, S, crc_tables, nullptr, &D);
}
__global__ void __launch_bounds__(kBlock, CRR_WIDE_WAVES_PER_EU) replay_wide_kernel(crr_inputs in, crr_outputs out, int phase,
                                                                                    u32 lo, u32 hi) {
  __shared__ u32 crc_tables[8 * 256];
  build_crc_tables<kBlock>(crc_tables);
  Digest D;
  replay_wide(in, out, phase, lo, hi, crc_tables, D);
  digest_flush(out, D);
}
// Compact LDS tiers (CRR_IN_TIERED segments [compact_begin, compact2_begin), [compact2_begin,
// wide_begin) and [wide_begin, hbm_begin)): lane per workflow, 64 lanes per block; slot counts per map
// chosen by the host's live-set bounds (flatten.TIER_SLOTS).  A workflow that outgrows its tier goes to the retry pass (list 0).
using CompactTier1 = CTier<4, 3, 2, 1, 1, 4, 64>;
// tier 2 at 8 x 19.7 KB per CU (2 waves per SIMD): 5 timers (99 % of the config-3 shard's tier-2
// workflows need <= 5; the rest take tier 3)
using CompactTier2 = CTier<8, 5, 3, 3, 3, 8, 64>;
// tier 3: 29 KB per block, 5 per CU (the config-3 shard's tier-3 workflows all but ~2 % fit; the rest
// join the wave tail)
using CompactTier3 = CTier<12, 8, 6, 4, 4, 8, 64>;
// CRC tables in LDS for a compact tier's checksum (copied from the constant-memory ones at block start)
// instead of per-lane gathers from kCrcGlobal through the L1: an 8-KB table gather touches many lines per
// instruction, and with few events per workflow (a resume) the checksum is a large part of its work
// (passive replication on the config-3 shard: 1.02 -> 0.91 ms per step with the resume instantiations'
// tables in LDS, A/B on one box; their occupancy is register-limited, so the 8 KB costs no waves).  Tier 3's
// resume kernel (one wave per SIMD, few workflows) does better on the constant-memory tables: 0.885 ->
// 0.85 ms with tiers 1-2 only (round 4, A/B)
#ifndef CRR_COMPACT_LDS_CRC_MASK  // bit k: tier k+1's resume instantiation (bit 3+k: its fresh one)
#define CRR_COMPACT_LDS_CRC_MASK 3
#endif
template <int TIER_NO, bool RESUME>
struct CompactLdsCrc {
  static constexpr bool value = ((CRR_COMPACT_LDS_CRC_MASK >> ((TIER_NO - 1) + (RESUME ? 0 : 3))) & 1) != 0;
};
template <class TIER, bool EMIT, bool RESUME, int TIER_NO>
__device__ __forceinline__ void replay_compact(const crr_inputs& in, const crr_outputs& out, int phase, u32 lo, u32 hi,
                                               Digest& D) {
  __shared__ CompactArena<TIER> arena;
  const u32* crc_tables = kCrcGlobal.v;
  const u32 w = lo + blockIdx.x * 64u + threadIdx.x;
  const bool in_range = w < hi;
  const crr_workflow* wfp = in.wf + (in_range ? w : lo);
  const i64 lane = threadIdx.x & 63;
  Geo G;  // the descriptor in one round trip, as in replay_lds
  load_geo(G, wfp, out, 64);
  i64 ev_begin = wfp->ev_begin;
  const i32 ev_count0 = wfp->ev_count;
  const u32 wf_flags = wfp->flags;
  // a kernel that expects loaded states reads every exec row with its descriptor (one round trip)
  crr_exec_row X0;
  if constexpr (RESUME) X0 = out.exec[in_range ? w : lo];
  if constexpr (CompactLdsCrc<TIER_NO, RESUME>::value) {  // the tables' copy in the same round trip
    __shared__ u32 crc_lds[8 * 256];
    const uint4* src = reinterpret_cast<const uint4*>(kCrcGlobal.v);
    uint4* dst = reinterpret_cast<uint4*>(crc_lds);
#pragma unroll
    for (int i = 0; i < 8 * 256 / 4 / 64; ++i) dst[i * 64 + threadIdx.x] = src[i * 64 + threadIdx.x];
    __syncthreads();
    crc_tables = crc_lds;
  }
  if (!in_range) return;
  asm volatile("" ::"v"(ev_begin), "v"(ev_count0), "v"(wf_flags));
  if (((wf_flags & CRR_WF_FLAG_NEW_RUN) != 0) != (phase == 0)) return;
  if ((lo & 63u) == 0) {  // wavefront == one interleaved group: group-uniform geometry in SGPRs
    uniformize_geo(G, lane);
    ev_begin = uniform64(ev_begin - lane) + lane;
  }
  CompactTables<TIER, RESUME> T;
  T.init(&arena, &in, ev_begin, ev_count0);
  LaneSource S(in.ev, ev_begin, 64, wfp->ev_count, EMIT && (in.flags & CRR_IN_EMIT_TASKS) != 0,
               (in.flags & CRR_IN_STARTED_AUX) != 0);
  replay_body<EMIT, CompactTables<TIER, RESUME>, LaneSource>(in, out, w, wfp, G, T, S, crc_tables,
                                                             RESUME ? &X0 : nullptr, &D);
}
// register budgets (waves per SIMD): tier 1's 10-KB blocks would fit 15 per CU, but at 3 waves/SIMD (168
// VGPRs) its loop spills 24 VGPRs (156 B/lane of scratch); at 2 (256 VGPRs) none, and the config-3 shard
// replays 2.55-2.59 ms against 2.60-2.66 (round 5, alternated A/B on one box); tier 2's 20-KB blocks fit 8
#ifndef CRR_COMPACT1_WAVES_PER_EU
#define CRR_COMPACT1_WAVES_PER_EU 2
#endif
// the resume instantiation at 2: its loaded-row reads and in-place finalize spill at 168 VGPRs
#ifndef CRR_COMPACT1_RESUME_WAVES_PER_EU
#define CRR_COMPACT1_RESUME_WAVES_PER_EU 2
#endif
#ifndef CRR_COMPACT2_WAVES_PER_EU
#define CRR_COMPACT2_WAVES_PER_EU 2
#endif
template <bool EMIT, bool RESUME>
__global__ void __launch_bounds__(64, RESUME ? CRR_COMPACT1_RESUME_WAVES_PER_EU : CRR_COMPACT1_WAVES_PER_EU) replay_compact1_kernel(crr_inputs in, crr_outputs out, int phase, u32 lo, u32 hi) {
  Digest D;
  replay_compact<CompactTier1, EMIT, RESUME, 1>(in, out, phase, lo, hi, D);
  digest_flush(out, D);
}
template <bool EMIT, bool RESUME>
__global__ void __launch_bounds__(64, CRR_COMPACT2_WAVES_PER_EU) replay_compact2_kernel(crr_inputs in, crr_outputs out, int phase, u32 lo, u32 hi) {
  Digest D;
  replay_compact<CompactTier2, EMIT, RESUME, 2>(in, out, phase, lo, hi, D);
  digest_flush(out, D);
}
template __global__ void replay_compact1_kernel<false, false>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_compact1_kernel<true, false>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_compact2_kernel<false, false>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_compact2_kernel<true, false>(crr_inputs, crr_outputs, int, u32, u32);
// loaded states continued in the arena (CRR_IN_HAS_RESUME)
template __global__ void replay_compact1_kernel<false, true>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_compact1_kernel<true, true>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_compact2_kernel<false, true>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_compact2_kernel<true, true>(crr_inputs, crr_outputs, int, u32, u32);
// tier 3 (workflows beyond tier 2 that hold no loaded state): 55-KB blocks, 2 per CU -- a segment of a
// few hundred wavefronts, so what matters is its per-event latency (LDS, not the HBM rows' round trips)
template <bool EMIT, bool RESUME>
__global__ void __launch_bounds__(64, 1) replay_compact3_kernel(crr_inputs in, crr_outputs out, int phase, u32 lo, u32 hi) {
  Digest D;
  replay_compact<CompactTier3, EMIT, RESUME, 3>(in, out, phase, lo, hi, D);
  digest_flush(out, D);
}
template __global__ void replay_compact3_kernel<false, false>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_compact3_kernel<true, false>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_compact3_kernel<false, true>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_compact3_kernel<true, true>(crr_inputs, crr_outputs, int, u32, u32);
// Long-tail workflows the host expects to outgrow the fast kernels' per-wave arenas
// (CRR_IN_TIERED, [big_begin, n_wf)): one wavefront each with the 57 KB row arena, then HBM rows;
// launched next to the fast kernels, so the longest of them is not replayed after them.
union BigArenas {
  BigSegArena seg;
  BigArena big;
};
__global__ void __launch_bounds__(64) replay_big_kernel(crr_inputs in, crr_outputs out, int phase, u32 lo, u32 hi) {
  __shared__ u32 crc_tables[8 * 256];
  __shared__ BigArenas arena;
  // resident: counted in before anything else (tail_gate_kernel holds the tail back until every block is)
  if (threadIdx.x == 0) atomicAdd(out.scratch + kScratchGate, 1u);
  const u32 w = lo + blockIdx.x;
  if (w >= hi) return;
  build_crc_tables(crc_tables);
  Digest D;
  // two registers per map first; a live set past that is replayed again with the retry pass's 320-slot arena
  // (five registers per map), then over the HBM rows
  WaveLds<BigSegArena, -1> T;
  bind_arena(T, &arena.seg);
  replay_wave_item(in, out, phase, w, T, crc_tables, D);
  if (T.retried) {
    WaveLds<BigArena, -1> T2;
    bind_arena(T2, &arena.big);
    replay_wave_item(in, out, phase, w, T2, crc_tables, D);
    if (T2.retried) {
      WaveTables<HbmRows> H;
      replay_wave_item(in, out, phase, w, H, crc_tables, D);
    }
  }
  digest_flush(out, D);
}
// Long-history tail of a CRR_IN_TIERED batch ([wave_begin, big_begin), longest first): one wavefront
// per workflow over a 12-KB LDS row arena; a workflow that outgrows it (or resumes a loaded state) is
// replayed again over its HBM rows in the same wavefront.  The checksum reads the constant-memory CRC
// tables: without 8 KB of CRC tables in LDS 13 blocks fit a CU, so with <= 168 VGPRs the tail runs 3
// waves per SIMD -- 3072 at once, enough for config 4's tail in one round.
#ifndef CRR_TAIL_WAVES_PER_EU
#define CRR_TAIL_WAVES_PER_EU 3
#endif
// RESUME (a batch holding loaded states, CRR_IN_HAS_RESUME): a workflow the LDS arena cannot hold -- it
// outgrew it, or resumes a loaded state -- is replayed again over its HBM rows in the same wavefront.
// Otherwise such a workflow (the host's bounds route the ones expected to outgrow to the big segment) goes
// to the retry pass's wave list: without the HBM-row instantiation in the kernel the tail needs 87
// VGPRs instead of 168 with 141 VGPRs of scratch spills, and fewer scalar spills (236 vs 302).
// The big segment's blocks need 65 KB of LDS each; once the tail's thousands of 13-KB wavefronts hold the
// CUs, a big block queued behind them waits for tail wavefronts to finish (config 4: the group at 9.4 ms
// instead of 5.6 in about one launch in ten, whichever hardware queue won the dispatch race).  The tail's
// stream therefore runs this one-wavefront gate first: it returns once every big block has counted itself
// in (or after ~10 ms, a bound every wave reaches).  The counter is reset by the retry pass.
__global__ void __launch_bounds__(64) tail_gate_kernel(const u32* scratch, u32 need) {
  if (threadIdx.x != 0) return;
  const u32* counter = scratch + kScratchGate;
  for (u32 i = 0; i < (1u << 16); ++i) {  // ~10 ms at most (a poll is ~140 ns)
    if (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need) return;
    __builtin_amdgcn_s_sleep(2);
  }
}
template <bool EMIT, bool RESUME>
__global__ void __launch_bounds__(64, CRR_TAIL_WAVES_PER_EU) replay_tail_kernel(crr_inputs in, crr_outputs out, int phase,
                                                                             u32 lo, u32 hi) {
  const u32* crc_tables = kCrcGlobal.v;
  __shared__ WaveTier<LargeTier>::Arena arena;
  const u32 w = lo + blockIdx.x;
  if (w >= hi) return;
  WaveLds<WaveTier<LargeTier>::Arena, RESUME ? -1 : 1> T;
  bind_arena(T, &arena);
  Digest D;
  replay_wave_item<decltype(T), EMIT>(in, out, phase, w, T, crc_tables, D);
  if constexpr (RESUME) {
    if (T.retried) {
      WaveTables<HbmRows> H;
      replay_wave_item<WaveTables<HbmRows>, EMIT>(in, out, phase, w, H, crc_tables, D);
    }
  }
  digest_flush(out, D);
}
template __global__ void replay_tail_kernel<false, false>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_tail_kernel<true, false>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_tail_kernel<false, true>(crr_inputs, crr_outputs, int, u32, u32);
template __global__ void replay_tail_kernel<true, true>(crr_inputs, crr_outputs, int, u32, u32);
union RetryArena {
  LdsArena<HugeTier> lane;
  BigArena wave;
};
__global__ void __launch_bounds__(64) replay_retry_kernel(crr_inputs in, crr_outputs out, int phase) {
  __shared__ u32 crc_tables[8 * 256];
  __shared__ RetryArena arena;
  // counts are bounded by n_wf (each workflow is handed back at most once per launch); the clamp
  // keeps a stale or corrupted header from indexing past the lists
  const u32 n0 = min(__hip_atomic_load(out.scratch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), in.n_wf);
  const u32 n1 = min(__hip_atomic_load(out.scratch + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), in.n_wf);
  if (n0 == 0 && n1 == 0) {  // uniform across the grid: nothing was handed back
    // the big segment's gate counter still counted this phase's blocks in; no other block of this grid
    // touches it, and every big block has finished (this kernel runs after the side streams joined)
    if (blockIdx.x == 0 && threadIdx.x == 0)
      __hip_atomic_store(out.scratch + kScratchGate, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  build_crc_tables(crc_tables);
  Digest D;
  for (u32 i = blockIdx.x; i < n1; i += gridDim.x) {  // 1. long-tail workflows (they run longest)
    const u32 w = (u32)uniform32((i32)out.scratch[retry_slot(in, 1, i)]);
    if (w >= in.n_wf) continue;
    WaveLds<BigArena, -1> T;
    bind_arena(T, &arena.wave);
    replay_wave_item(in, out, phase, w, T, crc_tables, D);
    if (T.retried) {
      WaveTables<HbmRows> H;
      replay_wave_item(in, out, phase, w, H, crc_tables, D);
    }
  }
  __syncthreads();  // the lane arena reuses the wave arena's LDS
  // 2. lane workflows, spread over every block (a few handed-back lanes each when there are few:
  // the gathered loads are latency-bound, so more wavefronts beat fuller ones); blocks that did
  // fewer wave items take the first chunks
  const u32 start = (blockIdx.x + gridDim.x - (n1 % gridDim.x)) % gridDim.x;
  const u32 chunk = min(64u, (n0 + gridDim.x - 1) / gridDim.x);
  for (u32 base = start * chunk; base < n0; base += gridDim.x * chunk) {
    const u32 i = base + threadIdx.x;
    const u32 w = (threadIdx.x < chunk && i < n0) ? out.scratch[retry_slot(in, 0, i)] : in.n_wf;
    if (w < in.n_wf) replay_lane_item(in, out, phase, w, &arena.lane, crc_tables, D);
  }
  digest_flush(out, D);
  // every block has read both counts: the last one to finish resets them for the next launch
  if (threadIdx.x == 0) {
    __threadfence();
    const u32 done = atomicAdd(out.scratch + 2, 1u);
    if (done == gridDim.x - 1) {
      __hip_atomic_store(out.scratch, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(out.scratch + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(out.scratch + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(out.scratch + kScratchGate, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}



// The ID lists of a checksum from the live-ID sidecar (crr_outputs.live_ids): slot i of each column, addressed
// like the rows (base + i * stride), so a wavefront reading slot i of 64 interleaved workflows reads 512
// contiguous bytes.
struct SidecarIds {
  int64_t* const* c;
  __device__ __forceinline__ i64 act_id(const Geo& G, i32 i) const { return c[0][G.act_base + (i64)i * G.st]; }
  __device__ __forceinline__ i64 timer_id(const Geo& G, i32 i) const { return c[1][G.timer_base + (i64)i * G.st]; }
  __device__ __forceinline__ i64 child_id(const Geo& G, i32 i) const { return c[2][G.child_base + (i64)i * G.st]; }
  __device__ __forceinline__ i64 rc_id(const Geo& G, i32 i) const { return c[3][G.rc_base + (i64)i * G.st]; }
  __device__ __forceinline__ i64 sig_id(const Geo& G, i32 i) const { return c[4][G.sig_base + (i64)i * G.st]; }
};
// Recompute checksums from already-written rows (mutable_state_builder.go:334-348 verify path).
__global__ void __launch_bounds__(kBlock) checksum_kernel(crr_inputs in, crr_outputs out, u32* checksums) {
  __shared__ u32 crc_tables[8 * 256];
  build_crc_tables(crc_tables);
  const u32 w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= in.n_wf) return;
  const crr_workflow* wfp = in.wf + w;
  Geo G;
  load_geo(G, wfp, out, wf_stride(in, w));
  const crr_exec_row R = out.exec[w];
  TokenWords TW;
  TW.issue(token_desc(wfp), R.token_src, in.arena, in.token_crc, w);
  u32 len = 0;
  if (out.live_ids[0]) {  // the ID lists from the dense sidecar the replay wrote
    const SidecarIds ids{out.live_ids};
    checksums[w] = payload_crc(R, ids, G, TW, in.arena, crc_tables, &len);
  } else {                // ... or one field of each AoS row
    GlobalTables ids;
    checksums[w] = payload_crc(R, ids, G, TW, in.arena, crc_tables, &len);
  }
}

// Every kernel that folds a digest (digest_flush / digest_flush_block read the pointers from the kernel
// arguments at fixed offsets): (crr_inputs, crr_outputs, ...) must be its first two parameters.
template <class... F>
constexpr bool digest_kernels_ok(F...) { return (DigestKernelSig<F>::value && ...); }
static_assert(digest_kernels_ok(&replay_lds_small_kernel<false, false>, &replay_lds_small_kernel<false, false, true>,
                                &replay_lds_small_kernel<true, true>, &replay_lds_kernel<false, false>,
                                &replay_lds_kernel<true, true>, &replay_global_kernel, &replay_wide_kernel,
                                &replay_compact1_kernel<false, false>, &replay_compact1_kernel<true, true>,
                                &replay_compact2_kernel<false, false>, &replay_compact2_kernel<true, true>,
                                &replay_compact3_kernel<false, false>, &replay_compact3_kernel<true, true>,
                                &replay_big_kernel, &replay_tail_kernel<false, false>, &replay_tail_kernel<true, true>,
                                &replay_retry_kernel),
              "a digest-folding kernel must take (crr_inputs, crr_outputs, ...) first (kernarg_late offsets)");

}  // namespace crr
