// oracle/state_builder_ref.cpp -- TEST INFRASTRUCTURE ONLY (the parity checker / CPU baseline).
//
// A structurally faithful CPU restatement of Cadence's mutable-state replay path, written from
// the Go reference (github.com/uber/cadence @ /root/reference).  It is NOT part of the product:
// only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
//
// Parity anchoring: the Go reference cannot be compiled or run in this environment (no Go
// toolchain).  This restatement is pinned by the reference's own unit-test
// expectations restated in tests/test_oracle_kats.py (versionHistory_test.go, timer_sequence_test.go,
// state_rebuilder_test.go, mutable_state_builder_test.go transient-decision cases, the
// state_builder_test.go dispatch table) and by the thrift-binary branch-token KAT embedded in
// service/worker/archiver/testdata/archival_workflow_history_v1.json.  The checksum CRC is
// cross-checked against Python's zlib.crc32.  Exact checksum bytes have no reference golden
// vector ("checksum bytes: parity unpinned").
//
// Structure mirrors the Go code: per-workflow hash maps (Go maps), one ApplyEvents call per
// persisted batch, the same control flow and error returns, then generateMutableStateChecksum.
// Strings that the reference stores verbatim are tracked by provenance (the step of the event
// that supplied them); keys compared by string equality (ActivityID, TimerID, BinaryChecksum) are
// compared as real std::strings here, independently of the host's u32 interning.

#include "cadence_replay.h"

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

using i64 = int64_t;
using i32 = int32_t;

// Go integer arithmetic wraps; do the same without C++ signed-overflow UB.
inline i64 wadd(i64 a, i64 b) { return (i64)((uint64_t)a + (uint64_t)b); }
inline i64 wmul(i64 a, i64 b) { return (i64)((uint64_t)a * (uint64_t)b); }
constexpr i64 kSecond = 1000000000LL;
// time.Time.Unix(): seconds since epoch, floored (Go's Time.Unix for negative times floors).
inline i64 unix_seconds(i64 ns) { i64 q = ns / kSecond; if ((ns % kSecond) < 0) --q; return q; }

struct Err {
  int code = CRR_OK;
  bool ok() const { return code == CRR_OK; }
};
inline Err mk(int c) { Err e; e.code = c; return e; }

// ---- input view --------------------------------------------------------------------------------
struct KeyStrings {  // per-event key strings (ActivityID / TimerID / BinaryChecksum)
  const uint32_t* off;
  const uint32_t* len;
  const char* arena;
};

// Per-workflow key id -> string (the host interner's inverse): the strings of a loaded state's rows
// (ActivityID / TimerID / BinaryChecksum), which no event of this call carries.
struct KeyDict {
  const uint32_t* begin = nullptr;
  const uint32_t* count = nullptr;
  const uint32_t* off = nullptr;
  const uint32_t* len = nullptr;
  const char* arena = nullptr;
  bool ok() const { return begin != nullptr; }
  std::string str(uint32_t w, uint32_t key) const {
    const uint32_t i = begin[w] + key;
    return key < count[w] ? std::string(arena + off[i], len[i]) : std::string();
  }
};

// per-workflow column/row stride: the long-history tail of a CRR_IN_WAVE_TAIL batch is contiguous
inline i64 stride_of(const crr_inputs* in, const crr_workflow* wf) {
  return ((in->flags & CRR_IN_WAVE_TAIL) && (uint32_t)(wf - in->wf) >= in->wave_begin) ? 1 : (i64)in->stride;
}

// Steps are provenance steps: this call's event k is step sb + k, where sb is the resumed state's
// src_next (0 for a replay from scratch), so every *_src / fail_step value matches the engine's.
struct WfView {
  const crr_inputs* in;
  const crr_workflow* wf;
  const KeyStrings* ks;
  int sb;
  i64 idx(int step) const { return wf->ev_begin + (i64)(step - sb) * stride_of(in, wf); }
  int type(int step) const { return in->ev.etype[idx(step)] & CRR_ETYPE_MASK; }
  bool first(int step) const { return in->ev.etype[idx(step)] & CRR_ETYPE_BATCH_FIRST; }
  bool last(int step) const { return in->ev.etype[idx(step)] & CRR_ETYPE_BATCH_LAST; }
  i64 id(int s) const { return in->ev.event_id[idx(s)]; }
  i64 version(int s) const { return in->ev.version[idx(s)]; }
  i64 ts(int s) const { return in->ev.timestamp[idx(s)]; }
  i64 task_id(int s) const { return in->ev.task_id[idx(s)]; }
  i64 ref(int s) const { return in->ev.ref[idx(s)]; }
  uint32_t key(int s) const { return in->ev.key[idx(s)]; }
  i32 aux(int s) const { return in->ev.aux[idx(s)]; }
  std::string kstr(int s) const {
    i64 i = idx(s);
    return std::string(ks->arena + ks->off[i], ks->len[i]);
  }
};

// ---- persistence structs (common/persistence/dataManagerInterfaces.go:296-834) ----------------
struct ActivityInfo {
  i64 version = 0, schedule_id = 0, scheduled_batch_id = 0, scheduled_time = 0;
  i64 started_id = 0, started_time = CRR_ZERO_TIME;
  std::string activity_id;
  i32 sched_src = -1, started_src = -1;
  i32 schedule_to_start = 0, schedule_to_close = 0, start_to_close = 0, heartbeat = 0;
  bool cancel_requested = false;
  i64 cancel_request_id = 0;
  i64 last_heartbeat_updated_time = CRR_ZERO_TIME;
  i32 timer_task_status = 0;
  i32 attempt = 0;
  bool has_retry_policy = false;
  i64 last_hb_timeout_vis_s = 0;
  uint32_t key = 0;
};

struct TimerInfo {
  i64 version = 0;
  std::string timer_id;
  i64 started_id = 0, expiry_time = 0;
  i64 task_status = 0;
  i32 src = -1;
  uint32_t key = 0;
};

struct ChildExecutionInfo {
  i64 version = 0, initiated_id = 0, initiated_batch_id = 0, started_id = 0;
  i32 src = -1, started_src = -1;
};

struct InitiatedInfo {  // RequestCancelInfo / SignalInfo
  i64 version = 0, initiated_batch_id = 0, initiated_id = 0;
  i32 src = -1;
};

struct ResetPoint {
  i32 src = -1, prev_index = -1;
  std::string checksum;
  uint32_t key = 0;
  bool resettable = false;
};

struct VersionHistoryItem { i64 event_id, version; };

// persistence.VersionHistory (common/persistence/versionHistory.go)
struct VersionHistory {
  int token_src = 0;  // 0 = nil/empty token, 1 = start token, 2 = final (rebuild) token
  std::vector<VersionHistoryItem> items;

  // NewVersionHistoryItem (versionHistory.go:32-46): panics on invalid input
  static Err new_item(i64 event_id, i64 version, VersionHistoryItem* out) {
    if (event_id < 0 || (version < 0 && version != CRR_EMPTY_VERSION)) return mk(CRR_ERR_VH_INVALID_ITEM);
    out->event_id = event_id;
    out->version = version;
    return Err{};
  }
  // AddOrUpdateItem (versionHistory.go:193-226)
  Err add_or_update(const VersionHistoryItem& item) {
    if (items.empty()) { items.push_back(item); return Err{}; }
    VersionHistoryItem& last = items.back();
    if (item.version < last.version) return mk(CRR_ERR_VH_LOWER_VERSION);
    if (item.event_id <= last.event_id) return mk(CRR_ERR_VH_EVENT_ID_NOT_INCREASING);
    if (item.version > last.version) items.push_back(item);
    else last.event_id = item.event_id;
    return Err{};
  }
  // GetLastItem (versionHistory.go:303-310)
  Err last_item(VersionHistoryItem* out) const {
    if (items.empty()) return mk(CRR_ERR_VH_EMPTY);
    *out = items.back();
    return Err{};
  }
};

// persistence.WorkflowExecutionInfo numeric image
struct ExecutionInfo {
  int state = CRR_STATE_CREATED, close_status = CRR_CLOSE_NONE;
  i64 next_event_id = CRR_FIRST_EVENT_ID, last_first_event_id = 0, last_event_task_id = 0;
  i64 last_processed_event = CRR_EMPTY_EVENT_ID, completion_event_batch_id = 0;
  i64 decision_version = CRR_EMPTY_VERSION, decision_schedule_id = CRR_EMPTY_EVENT_ID;
  i64 decision_started_id = CRR_EMPTY_EVENT_ID;
  i32 decision_request_src = CRR_SRC_EMPTY_UUID;
  i32 decision_timeout = 0;
  i64 decision_attempt = 0, decision_started_ts = 0, decision_scheduled_ts = 0, decision_orig_scheduled_ts = 0;
  i32 signal_count = 0;
  bool cancel_requested = false;
  i32 decision_start_to_close_timeout = 0;  // DecisionStartToCloseTimeout
  i32 start_src = -1;
  bool auto_reset_points_set = false;       // AutoResetPoints != nil
  std::vector<ResetPoint> reset_points;     // AutoResetPoints.Points
};

// WorkflowExecutionInfo.UpdateWorkflowStateCloseStatus (common/persistence/workflowExecutionInfo.go:45-165)
Err update_workflow_state_close_status(ExecutionInfo& e, int state, int close_status) {
  auto invalid = [] { return mk(CRR_ERR_INVALID_STATE_TRANSITION); };
  switch (e.state) {
    case CRR_STATE_VOID:
      break;  // no validation
    case CRR_STATE_CREATED:
      switch (state) {
        case CRR_STATE_CREATED:
          if (close_status != CRR_CLOSE_NONE) return invalid();
          break;
        case CRR_STATE_RUNNING:
          if (close_status != CRR_CLOSE_NONE) return invalid();
          break;
        case CRR_STATE_COMPLETED:
          if (close_status != CRR_CLOSE_TERMINATED && close_status != CRR_CLOSE_TIMED_OUT &&
              close_status != CRR_CLOSE_CONTINUED_AS_NEW)
            return invalid();
          break;
        case CRR_STATE_ZOMBIE:
          if (close_status != CRR_CLOSE_NONE) return invalid();
          break;
        default:
          return mk(CRR_ERR_UNKNOWN_WORKFLOW_STATE);
      }
      break;
    case CRR_STATE_RUNNING:
      switch (state) {
        case CRR_STATE_CREATED:
          return invalid();
        case CRR_STATE_RUNNING:
          if (close_status != CRR_CLOSE_NONE) return invalid();
          break;
        case CRR_STATE_COMPLETED:
          if (close_status == CRR_CLOSE_NONE) return invalid();
          break;
        case CRR_STATE_ZOMBIE:
          if (close_status != CRR_CLOSE_NONE) return invalid();
          break;
        default:
          return mk(CRR_ERR_UNKNOWN_WORKFLOW_STATE);
      }
      break;
    case CRR_STATE_COMPLETED:
      switch (state) {
        case CRR_STATE_CREATED:
        case CRR_STATE_RUNNING:
          return invalid();
        case CRR_STATE_COMPLETED:
          if (close_status != e.close_status) return invalid();
          break;
        case CRR_STATE_ZOMBIE:
          return invalid();
        default:
          return mk(CRR_ERR_UNKNOWN_WORKFLOW_STATE);
      }
      break;
    case CRR_STATE_ZOMBIE:
      switch (state) {
        case CRR_STATE_CREATED:
        case CRR_STATE_RUNNING:
          if (close_status != CRR_CLOSE_NONE) return invalid();
          break;
        case CRR_STATE_COMPLETED:
          if (close_status == CRR_CLOSE_NONE) return invalid();
          break;
        case CRR_STATE_ZOMBIE:
          if (close_status == CRR_CLOSE_NONE) return invalid();
          break;
        default:
          return mk(CRR_ERR_UNKNOWN_WORKFLOW_STATE);
      }
      break;
    default:
      return mk(CRR_ERR_UNKNOWN_WORKFLOW_STATE);
  }
  e.state = state;
  e.close_status = close_status;
  return Err{};
}

// ---- mutableStateBuilder (service/history/execution/mutable_state_builder.go) --------------------
struct MutableState {
  // :84-110
  std::unordered_map<i64, ActivityInfo> pendingActivityInfoIDs;
  std::unordered_map<std::string, i64> pendingActivityIDToEventID;
  std::unordered_map<std::string, TimerInfo> pendingTimerInfoIDs;
  std::unordered_map<i64, std::string> pendingTimerEventIDToID;
  std::unordered_map<i64, ChildExecutionInfo> pendingChildExecutionInfoIDs;
  std::unordered_map<i64, InitiatedInfo> pendingRequestCancelInfoIDs;
  std::unordered_map<i64, InitiatedInfo> pendingSignalInfoIDs;
  ExecutionInfo exec;
  VersionHistory vh;  // NewMutableStateBuilderWithVersionHistories: one empty history (:252)
  i64 currentVersion = 0;
  i64 now_ns = 0;     // injected clock.TimeSource
  int inconsistencies = 0;
  i64 expiration_ns = 0;                 // executionInfo.ExpirationTime (0: unset)
  bool emit_tasks = false;               // CRR_IN_EMIT_TASKS
  std::vector<crr_task_row> tasks;       // AddTransferTasks / AddTimerTasks, in order
  void AddTask(int kind, int aux, i64 version, i64 vis, i64 event_id, int attempt, int src) {
    if (!emit_tasks) return;
    crr_task_row r;
    r.kind = kind; r.aux = aux; r.version = version; r.visibility_ts = vis; r.event_id = event_id;
    r.attempt = attempt; r.src = src;
    tasks.push_back(r);
  }

  // logDataInconsistency (:4720-4731)
  void log_data_inconsistency() { ++inconsistencies; }

  // UpdateCurrentVersion (:495-533), versionHistories != nil always on this path
  Err UpdateCurrentVersion(i64 version, bool forceUpdate) {
    if (exec.state == CRR_STATE_COMPLETED) {
      VersionHistoryItem last;  // GetLastWriteVersion (:566-586)
      Err e = vh.last_item(&last);
      if (!e.ok()) return e;
      currentVersion = last.version;
      return Err{};
    }
    if (!vh.items.empty()) currentVersion = vh.items.back().version;
    if (version > currentVersion || forceUpdate) currentVersion = version;
    return Err{};
  }

  // ClearStickyness (:1504-1510): sticky / client fields are "" on a replayed state.
  void ClearStickyness() {}

  // DeleteActivity (:1310-1339)
  void DeleteActivity(i64 scheduleEventID) {
    auto it = pendingActivityInfoIDs.find(scheduleEventID);
    if (it != pendingActivityInfoIDs.end()) {
      std::string aid = it->second.activity_id;
      pendingActivityInfoIDs.erase(it);
      auto jt = pendingActivityIDToEventID.find(aid);
      if (jt != pendingActivityIDToEventID.end()) pendingActivityIDToEventID.erase(jt);
      else log_data_inconsistency();
    } else {
      log_data_inconsistency();
    }
  }
  // DeleteUserTimer (:1390-1419)
  void DeleteUserTimer(const std::string& timerID) {
    auto it = pendingTimerInfoIDs.find(timerID);
    if (it != pendingTimerInfoIDs.end()) {
      i64 sid = it->second.started_id;
      pendingTimerInfoIDs.erase(it);
      auto jt = pendingTimerEventIDToID.find(sid);
      if (jt != pendingTimerEventIDToID.end()) pendingTimerEventIDToID.erase(jt);
      else log_data_inconsistency();
    } else {
      log_data_inconsistency();
    }
  }
  // DeletePendingChildExecution / DeletePendingRequestCancel / DeletePendingSignal (:1160-1220)
  template <class M>
  void delete_initiated(M& m, i64 initiatedEventID) {
    auto it = m.find(initiatedEventID);
    if (it != m.end()) m.erase(it);
    else log_data_inconsistency();
  }

  // GetActivityByActivityID (:963-973)
  ActivityInfo* GetActivityByActivityID(const std::string& aid) {
    auto it = pendingActivityIDToEventID.find(aid);
    if (it == pendingActivityIDToEventID.end()) return nullptr;
    auto jt = pendingActivityInfoIDs.find(it->second);
    return jt == pendingActivityInfoIDs.end() ? nullptr : &jt->second;
  }

  // ---- decision task manager (mutable_state_decision_task_manager.go) ----
  struct DecisionInfo {
    i64 version, schedule_id, started_id;
    i32 request_src;
    i32 timeout;
    i64 attempt, started_ts, scheduled_ts, orig_scheduled_ts;
  };
  // UpdateDecision (:697-721) -- "do not update tasklist in execution info"
  void UpdateDecision(const DecisionInfo& d) {
    exec.decision_version = d.version;
    exec.decision_schedule_id = d.schedule_id;
    exec.decision_started_id = d.started_id;
    exec.decision_request_src = d.request_src;
    exec.decision_timeout = d.timeout;
    exec.decision_attempt = d.attempt;
    exec.decision_started_ts = d.started_ts;
    exec.decision_scheduled_ts = d.scheduled_ts;
    exec.decision_orig_scheduled_ts = d.orig_scheduled_ts;
  }
  // HasPendingDecision (:723-725)
  bool HasPendingDecision() const { return exec.decision_schedule_id != CRR_EMPTY_EVENT_ID; }
  // ReplicateDecisionTaskScheduledEvent (:129-166)
  Err ReplicateDecisionTaskScheduledEvent(i64 version, i64 scheduleID, i32 startToClose, i64 attempt,
                                          i64 scheduleTs, i64 originalScheduledTs) {
    if (exec.state != CRR_STATE_ZOMBIE) {
      Err e = update_workflow_state_close_status(exec, CRR_STATE_RUNNING, CRR_CLOSE_NONE);
      if (!e.ok()) return e;
    }
    UpdateDecision({version, scheduleID, CRR_EMPTY_EVENT_ID, CRR_SRC_EMPTY_UUID, startToClose, attempt,
                    0, scheduleTs, originalScheduledTs});
    return Err{};
  }
  // ReplicateTransientDecisionTaskScheduled (:168-197); returns whether a decision was created
  bool ReplicateTransientDecisionTaskScheduled() {
    if (HasPendingDecision() || exec.decision_attempt == 0) return false;
    UpdateDecision({currentVersion, exec.next_event_id, CRR_EMPTY_EVENT_ID, CRR_SRC_EMPTY_UUID,
                    exec.decision_start_to_close_timeout, exec.decision_attempt, 0, now_ns,
                    /*OriginalScheduledTimestamp not set*/ 0});
    return true;
  }
  // ReplicateDecisionTaskStartedEvent (:199-242), decision == nil on the replay path
  Err ReplicateDecisionTaskStartedEvent(i64 version, i64 scheduleID, i64 startedID, i32 requestSrc, i64 ts) {
    // GetDecisionInfo (:755-763)
    if (scheduleID != exec.decision_schedule_id) return mk(CRR_ERR_DECISION_NOT_FOUND);
    i64 attempt = 0;  // "setting decision attempt to 0 for decision task replication"
    UpdateDecision({version, scheduleID, startedID, requestSrc, exec.decision_timeout, attempt, ts,
                    exec.decision_scheduled_ts, exec.decision_orig_scheduled_ts});
    return Err{};
  }
  // FailDecision (:643-676)
  void FailDecision(bool incrementAttempt) {
    ClearStickyness();
    DecisionInfo d{CRR_EMPTY_VERSION, CRR_EMPTY_EVENT_ID, CRR_EMPTY_EVENT_ID, CRR_SRC_EMPTY_UUID, 0, 0, 0, 0, 0};
    if (incrementAttempt) {
      d.attempt = exec.decision_attempt + 1;
      d.scheduled_ts = now_ns;
    }
    UpdateDecision(d);
  }
  // DeleteDecision (:679-694)
  void DeleteDecision() {
    UpdateDecision({CRR_EMPTY_VERSION, CRR_EMPTY_EVENT_ID, CRR_EMPTY_EVENT_ID, CRR_SRC_EMPTY_UUID, 0, 0, 0, 0,
                    exec.decision_orig_scheduled_ts});
  }
  // CheckResettable (mutable_state_builder.go:1977-1994)
  bool CheckResettable() const {
    return pendingChildExecutionInfoIDs.empty() && pendingRequestCancelInfoIDs.empty() &&
           pendingSignalInfoIDs.empty();
  }
  // addBinaryCheckSumIfNotExists (mutable_state_builder.go:1911-1974), maxResetPoints = MaxInt32
  void addBinaryCheckSumIfNotExists(const std::string& binChecksum, uint32_t key, int step) {
    if (binChecksum.empty()) return;
    for (const ResetPoint& rp : exec.reset_points) {
      // New points compare by string; points carried over from PrevAutoResetPoints compare by the
      // host's interned key (their strings live in the start event, not in the key-string arena).
      if (rp.prev_index < 0 ? rp.checksum == binChecksum : rp.key == key) return;
    }
    // len(currResetPoints) == math.MaxInt32 rotation is unreachable here
    ResetPoint rp;
    rp.src = step;
    rp.prev_index = -1;
    rp.checksum = binChecksum;
    rp.key = key;
    rp.resettable = CheckResettable();
    exec.reset_points.push_back(rp);
    exec.auto_reset_points_set = true;
    // SearchAttributes[BinaryChecksums] = json(recent checksums): string-valued, host materialised
  }
  // ReplicateDecisionTaskCompletedEvent (:244-249) -> before/afterAddDecisionTaskCompletedEvent (:827-838)
  void ReplicateDecisionTaskCompletedEvent(i64 startedEventID, const std::string& bin, uint32_t key, int step) {
    DeleteDecision();
    exec.last_processed_event = startedEventID;
    addBinaryCheckSumIfNotExists(bin, key, step);
  }
};

// ---- timer_sequence.go ------------------------------------------------------------------------------
struct TimerSequenceID {
  i64 event_id;
  i64 timestamp;
  i32 timer_type;
  bool created;
  i32 attempt;  // the activity's Attempt (0 for user timers)
};
// Less (timer_sequence.go:461-493): order by timestamp, event ID, timer type.  Sequence IDs in one
// list are pairwise distinct, so any sort yields the same first element as Go's sort.Sort.
bool seq_less(const TimerSequenceID& a, const TimerSequenceID& b) {
  if (a.timestamp != b.timestamp) return a.timestamp < b.timestamp;
  if (a.event_id != b.event_id) return a.event_id < b.event_id;
  return a.timer_type < b.timer_type;
}

inline i64 add_seconds(i64 t, i64 secs) { return wadd(t, wmul(secs, kSecond)); }  // t.Add(Duration(s)*time.Second)

// LoadAndSortActivityTimers (:219-254) with get*Timeout (:269-381)
std::vector<TimerSequenceID> LoadAndSortActivityTimers(const MutableState& ms) {
  std::vector<TimerSequenceID> v;
  v.reserve(ms.pendingActivityInfoIDs.size() * 4);
  for (const auto& kv : ms.pendingActivityInfoIDs) {
    const ActivityInfo& ai = kv.second;
    if (ai.schedule_id == CRR_EMPTY_EVENT_ID) continue;  // every getter returns nil
    // getActivityScheduleToCloseTimeout (:296-316)
    v.push_back({ai.schedule_id, add_seconds(ai.scheduled_time, ai.schedule_to_close), CRR_TIMEOUT_SCHEDULE_TO_CLOSE,
                 (ai.timer_task_status & CRR_TTS_CREATED_SCHEDULE_TO_CLOSE) > 0, ai.attempt});
    // getActivityScheduleToStartTimeout (:269-294)
    if (ai.started_id == CRR_EMPTY_EVENT_ID) {
      v.push_back({ai.schedule_id, add_seconds(ai.scheduled_time, ai.schedule_to_start), CRR_TIMEOUT_SCHEDULE_TO_START,
                   (ai.timer_task_status & CRR_TTS_CREATED_SCHEDULE_TO_START) > 0, ai.attempt});
    } else {
      // getActivityStartToCloseTimeout (:318-343)
      v.push_back({ai.schedule_id, add_seconds(ai.started_time, ai.start_to_close), CRR_TIMEOUT_START_TO_CLOSE,
                   (ai.timer_task_status & CRR_TTS_CREATED_START_TO_CLOSE) > 0, ai.attempt});
      // getActivityHeartbeatTimeout (:345-381)
      if (ai.heartbeat > 0) {
        i64 lastHeartbeat = ai.started_time;
        if (ai.last_heartbeat_updated_time > lastHeartbeat) lastHeartbeat = ai.last_heartbeat_updated_time;
        v.push_back({ai.schedule_id, add_seconds(lastHeartbeat, ai.heartbeat), CRR_TIMEOUT_HEARTBEAT,
                     (ai.timer_task_status & CRR_TTS_CREATED_HEARTBEAT) > 0, ai.attempt});
      }
    }
  }
  std::sort(v.begin(), v.end(), seq_less);
  return v;
}
// LoadAndSortUserTimers (:201-217) with getUserTimerTimeout (:256-267)
std::vector<TimerSequenceID> LoadAndSortUserTimers(const MutableState& ms) {
  std::vector<TimerSequenceID> v;
  v.reserve(ms.pendingTimerInfoIDs.size());
  for (const auto& kv : ms.pendingTimerInfoIDs) {
    const TimerInfo& ti = kv.second;
    v.push_back({ti.started_id, ti.expiry_time, CRR_TIMEOUT_START_TO_CLOSE, ti.task_status == CRR_TIMER_TASK_STATUS_CREATED, 0});
  }
  std::sort(v.begin(), v.end(), seq_less);
  return v;
}
int timer_type_to_mask(int t) {  // TimerTypeToTimerMask (:384-400)
  switch (t) {
    case CRR_TIMEOUT_START_TO_CLOSE: return CRR_TTS_CREATED_START_TO_CLOSE;
    case CRR_TIMEOUT_SCHEDULE_TO_START: return CRR_TTS_CREATED_SCHEDULE_TO_START;
    case CRR_TIMEOUT_SCHEDULE_TO_CLOSE: return CRR_TTS_CREATED_SCHEDULE_TO_CLOSE;
    default: return CRR_TTS_CREATED_HEARTBEAT;
  }
}
// CreateNextActivityTimer (:162-199)
Err CreateNextActivityTimer(MutableState& ms) {
  std::vector<TimerSequenceID> seq = LoadAndSortActivityTimers(ms);
  if (seq.empty()) return Err{};
  const TimerSequenceID& first = seq[0];
  if (first.created) return Err{};
  auto it = ms.pendingActivityInfoIDs.find(first.event_id);
  if (it == ms.pendingActivityInfoIDs.end()) return mk(CRR_ERR_TIMER_SEQUENCE);
  ActivityInfo& ai = it->second;
  ai.timer_task_status |= timer_type_to_mask(first.timer_type);
  if (first.timer_type == CRR_TIMEOUT_HEARTBEAT) ai.last_hb_timeout_vis_s = unix_seconds(first.timestamp);
  // UpdateActivity (:1292-1307) cannot fail: the info is pending.  AddTimerTasks (:190-196):
  ms.AddTask(CRR_TASK_ACTIVITY_TIMEOUT, first.timer_type, ms.currentVersion, first.timestamp, first.event_id, ai.attempt, -1);
  return Err{};
}
// CreateNextUserTimer (:127-160)
Err CreateNextUserTimer(MutableState& ms) {
  std::vector<TimerSequenceID> seq = LoadAndSortUserTimers(ms);
  if (seq.empty()) return Err{};
  const TimerSequenceID& first = seq[0];
  if (first.created) return Err{};
  // GetUserTimerInfoByEventID (:1351-1360)
  auto it = ms.pendingTimerEventIDToID.find(first.event_id);
  if (it == ms.pendingTimerEventIDToID.end()) return mk(CRR_ERR_TIMER_SEQUENCE);
  auto jt = ms.pendingTimerInfoIDs.find(it->second);
  if (jt == ms.pendingTimerInfoIDs.end()) return mk(CRR_ERR_TIMER_SEQUENCE);
  jt->second.task_status = CRR_TIMER_TASK_STATUS_CREATED;  // UpdateUserTimer (:1363-1387) succeeds
  ms.AddTask(CRR_TASK_USER_TIMER, 0, ms.currentVersion, first.timestamp, first.event_id, 0, -1);  // (:151-156)
  return Err{};
}

// GenerateWorkflowCloseTasks (task_generator.go:168-258): close transfer task + DeleteHistoryEventTask
void GenerateWorkflowCloseTasks(MutableState& ms, const WfView& v, int s) {
  ms.AddTask(CRR_TASK_CLOSE_EXECUTION, 0, v.version(s), 0, 0, 0, s);
  ms.AddTask(CRR_TASK_DELETE_HISTORY, 0, v.version(s), wadd(v.ts(s), wmul((i64)v.wf->retention_days * 86400, kSecond)),
             0, 0, s);
}

// ---- RefreshTasks (mutable_state_task_refresher.go) --------------------------------------------------
// getNextDecisionTimeout (mutable_state_task_generator.go:1051-1064) with rand.Intn(jitterPortion) taken as
// the injected draw mod jitterPortion (crr_start_side.refresh_jitter); durations in ns
i64 NextDecisionTimeout(i64 attempt, i64 default_ns, i64 draw) {
  if (attempt <= 1) return default_ns;
  // float64(defaultInitIntervalForDecisionRetry = 1m) * math.Pow(2, attempt-2), capped at 5m: exact doubles
  double next = attempt >= 5 ? 300e9 : 60e9 * (double)(1ll << (attempt - 2));
  next = next < 300e9 ? next : 300e9;                    // math.Min
  i64 jp = (i64)(0.2 * next);                            // int(defaultJitterCoefficient * nextInterval)
  if (jp < 1) jp = 1;
  next = next * 0.8 + (double)(i64)((uint64_t)draw % (uint64_t)jp);   // (1 - 0.2) is the exact constant 0.8
  return (i64)next;                                      // time.Duration(nextInterval)
}

// Each pending map in ascending event ID (Go ranges over the maps: an unspecified order).
template <class M>
std::vector<i64> sorted_keys(const M& m) {
  std::vector<i64> k;
  k.reserve(m.size());
  for (const auto& kv : m) k.push_back(kv.first);
  std::sort(k.begin(), k.end());
  return k;
}

// RefreshTasks (:77-170) on the rebuilt state; startTime = the rebuild's now (state_rebuilder.go:186)
Err RefreshTasks(const WfView& v, MutableState& ms, int n) {
  ExecutionInfo& x = ms.exec;
  // refreshTasksForWorkflowStart (:172-202): GetStartEvent reads the event with ID FirstEventID
  // (mutable_state_builder.go:1131-1157) -- here the start event this replay applied
  const int ss = x.start_src;
  if (ss < v.sb || ss >= n || v.id(ss) != CRR_FIRST_EVENT_ID) return mk(CRR_ERR_MISSING_START_EVENT);
  const crr_start_side& sd = v.in->start_side[v.aux(ss)];
  const i64 sver = v.version(ss);
  {  // GenerateWorkflowStartTasks (task_generator.go:143-166)
    i64 vis = wadd(v.wf->now_ns, wmul(wadd(sd.workflow_timeout, sd.first_decision_backoff), kSecond));
    if (sd.attempt > 0 && ms.expiration_ns != 0 && vis > ms.expiration_ns) vis = ms.expiration_ns;
    ms.AddTask(CRR_TASK_WORKFLOW_TIMEOUT, 0, sver, vis, 0, 0, ss);
  }
  // !HasProcessedOrPendingDecision (decision_task_manager.go:750-752) && backoff > 0
  const bool processed_or_pending = ms.HasPendingDecision() || x.last_processed_event != CRR_EMPTY_EVENT_ID;
  if (!processed_or_pending && sd.first_decision_backoff > 0) {  // GenerateDelayedDecisionTasks (:260-299)
    if (sd.initiator != CRR_INITIATOR_NIL && sd.initiator != CRR_INITIATOR_RETRY_POLICY && sd.initiator != CRR_INITIATOR_CRON)
      return mk(CRR_ERR_BAD_INITIATOR);
    ms.AddTask(CRR_TASK_WORKFLOW_BACKOFF, sd.initiator == CRR_INITIATOR_RETRY_POLICY ? CRR_BACKOFF_RETRY : CRR_BACKOFF_CRON,
               sver, wadd(v.ts(ss), wmul(sd.first_decision_backoff, kSecond)), 0, 0, ss);
  }
  // refreshTasksForWorkflowClose (:204-222): GetCompletionEvent (mutable_state_builder.go:1085-1128), the
  // event NextEventID - 1 read from the batch that starts at CompletionEventBatchID
  if (x.close_status != CRR_CLOSE_NONE) {
    if (x.state != CRR_STATE_COMPLETED || x.completion_event_batch_id == CRR_EMPTY_EVENT_ID)
      return mk(CRR_ERR_MISSING_COMPLETION_EVENT);
    int cs = -1;
    for (int k = n - 1; k >= v.sb && cs < 0; --k)
      if (v.id(k) == x.next_event_id - 1) cs = k;
    if (cs < 0) return mk(CRR_ERR_MISSING_COMPLETION_EVENT);
    int bf = cs;  // the first event of its batch
    while (bf > v.sb && !v.first(bf)) --bf;
    if (v.id(bf) != x.completion_event_batch_id) return mk(CRR_ERR_MISSING_COMPLETION_EVENT);
    GenerateWorkflowCloseTasks(ms, v, cs);
  } else {  // refreshTasksForRecordWorkflowStarted (:224-244)
    ms.AddTask(CRR_TASK_RECORD_WORKFLOW_STARTED, 0, sver, 0, 0, 0, ss);
  }
  // refreshTasksForDecision (:246-276)
  if (ms.HasPendingDecision()) {
    if (x.decision_started_id != CRR_EMPTY_EVENT_ID) {  // GenerateDecisionStartTasks (task_generator.go:352-388)
      i64 stc = wmul(x.decision_timeout, kSecond);
      if (x.decision_attempt > 1) {
        stc = NextDecisionTimeout(x.decision_attempt, wmul(x.decision_start_to_close_timeout, kSecond), sd.refresh_jitter);
        x.decision_timeout = (i32)(stc / kSecond);  // int32(startToCloseTimeout.Seconds()); UpdateDecision
      }
      ms.AddTask(CRR_TASK_DECISION_TIMEOUT, CRR_TIMEOUT_START_TO_CLOSE, x.decision_version,
                 wadd(x.decision_started_ts, stc), x.decision_schedule_id, (int)x.decision_attempt, -1);
    } else {  // GenerateDecisionScheduleTasks (:315-350): executionInfo.TaskList (the start event's)
      ms.AddTask(CRR_TASK_DECISION, 0, x.decision_version, 0, x.decision_schedule_id, 0, ss);
    }
  }
  // refreshTasksForActivity (:278-336): TimerTaskStatus cleared; not-started activities' transfer tasks
  for (i64 id : sorted_keys(ms.pendingActivityInfoIDs)) {
    ActivityInfo& ai = ms.pendingActivityInfoIDs[id];
    ai.timer_task_status = CRR_TIMER_TASK_STATUS_NONE;
    if (ai.started_id == CRR_EMPTY_EVENT_ID)  // GenerateActivityTransferTasks (:390-427)
      ms.AddTask(CRR_TASK_ACTIVITY, 0, ai.version, 0, ai.schedule_id, 0, ai.sched_src);
  }
  Err er = CreateNextActivityTimer(ms);
  if (!er.ok()) return er;
  // refreshTasksForTimer (:338-365)
  for (auto& kv : ms.pendingTimerInfoIDs) kv.second.task_status = CRR_TIMER_TASK_STATUS_NONE;
  er = CreateNextUserTimer(ms);
  if (!er.ok()) return er;
  // refreshTasksForChildWorkflow (:367-406): GenerateChildWorkflowTasks (task_generator.go:449-495)
  for (i64 id : sorted_keys(ms.pendingChildExecutionInfoIDs)) {
    const ChildExecutionInfo& ci = ms.pendingChildExecutionInfoIDs[id];
    if (ci.started_id == CRR_EMPTY_EVENT_ID) ms.AddTask(CRR_TASK_START_CHILD, 0, ci.version, 0, ci.initiated_id, 0, ci.src);
  }
  // refreshTasksForRequestCancelExternalWorkflow / SignalExternalWorkflow (:408-482): the initiated
  // event's version and ID (task_generator.go:497-597)
  for (i64 id : sorted_keys(ms.pendingRequestCancelInfoIDs)) {
    const InitiatedInfo& ri = ms.pendingRequestCancelInfoIDs[id];
    ms.AddTask(CRR_TASK_CANCEL_EXECUTION, 0, ri.version, 0, ri.initiated_id, 0, ri.src);
  }
  for (i64 id : sorted_keys(ms.pendingSignalInfoIDs)) {
    const InitiatedInfo& si = ms.pendingSignalInfoIDs[id];
    ms.AddTask(CRR_TASK_SIGNAL_EXECUTION, 0, si.version, 0, si.initiated_id, 0, si.src);
  }
  // refreshTasksForWorkflowSearchAttr (:484-490), AdvancedVisibilityWritingMode != off
  if (v.in->flags & CRR_IN_ADVANCED_VISIBILITY)
    ms.AddTask(CRR_TASK_UPSERT_SEARCH_ATTRIBUTES, 0, ms.currentVersion, 0, 0, 0, -1);
  return Err{};
}

// ---- the replay driver ----------------------------------------------------------------------------
struct Outcome {
  int status = CRR_OK;
  int fail_step = -1;
};

class Replayer {
 public:
  Replayer(const crr_inputs* in, const KeyStrings* ks, const Outcome* phase0)
      : in_(in), ks_(ks), phase0_(phase0) {}

  // Replays workflow `w` from a fresh NewMutableStateBuilderWithVersionHistories (:245-254), or, for a
  // CRR_WF_FLAG_RESUME workflow, from the state `ms` already holds (load_state: mutableStateBuilder.Load)
  // with provenance steps starting at `sb`.
  Outcome replay(uint32_t w, MutableState& ms, int sb = 0) {
    const crr_workflow* wf = &in_->wf[w];
    WfView v{in_, wf, ks_, sb};
    if (!(wf->flags & CRR_WF_FLAG_RESUME)) ms.currentVersion = wf->init_version;  // GetFailoverVersion() (:207)
    ms.now_ns = wf->now_ns;
    ms.emit_tasks = (in_->flags & CRR_IN_EMIT_TASKS) != 0;
    Outcome out;
    int k = sb;
    const int n = sb + wf->ev_count;
    for (;;) {
      if (k - sb == wf->empty_batch_at) {  // an ApplyEvents call with an empty batch (state_builder.go:98-100)
        out.status = CRR_ERR_EMPTY_HISTORY;
        out.fail_step = k;
        return out;
      }
      if (k >= n) break;
      int e = k;
      while (e < n - 1 && !v.last(e)) ++e;
      Outcome o = ApplyEvents(v, ms, k, e + 1);
      if (o.status != CRR_OK) return o;
      k = e + 1;
    }
    // rebuild finalisation (state_rebuilder.go:150-177) when a target branch token is supplied
    if (wf->final_token_len != 0xFFFFFFFFu) {
      ms.vh.token_src = 2;  // SetCurrentBranchToken(targetBranchToken)
      VersionHistoryItem last;
      Err er = ms.vh.last_item(&last);
      if (!er.ok()) { out.status = er.code; out.fail_step = n; return out; }
      VersionHistoryItem want;
      er = VersionHistory::new_item(wf->rebuild_last_event_id, wf->rebuild_last_event_version, &want);
      if (!er.ok()) { out.status = er.code; out.fail_step = n; return out; }
      if (last.event_id != want.event_id || last.version != want.version) {
        out.status = CRR_ERR_REBUILD_LAST_ITEM;
        out.fail_step = n;
        return out;
      }
    }
    // Rebuild: CloseTransactionAsSnapshot drops the replay's tasks, then RefreshTasks
    // (state_rebuilder.go:181-186 -> mutable_state_task_refresher.go:77-496)
    if (wf->flags & CRR_WF_FLAG_REFRESH_TASKS) {
      ms.tasks.clear();
      Err er = RefreshTasks(v, ms, n);
      if (!er.ok()) { out.status = er.code; out.fail_step = n; return out; }
    }
    return out;
  }

 private:
  static void CloseTasks(MutableState& ms, const WfView& v, int s) { GenerateWorkflowCloseTasks(ms, v, s); }

  // stateBuilderImpl.ApplyEvents (state_builder.go:90-648) for history = steps [b, e)
  Outcome ApplyEvents(const WfView& v, MutableState& ms, int b, int e) {
    Outcome out;
    auto fail = [&](int code, int step) { out.status = code; out.fail_step = step; return out; };
    const i64 firstEventID = v.id(b);
    const i64 lastEventID = v.id(e - 1);
    ms.ClearStickyness();  // :108
    for (int s = b; s < e; ++s) {
      // :112 UpdateCurrentVersion(event.Version, true)
      Err er = ms.UpdateCurrentVersion(v.version(s), true);
      if (!er.ok()) return fail(er.code, s);
      // :115-128 versionHistory.AddOrUpdateItem(NewVersionHistoryItem(event.ID, event.Version))
      VersionHistoryItem item;
      er = VersionHistory::new_item(v.id(s), v.version(s), &item);
      if (!er.ok()) return fail(er.code, s);
      er = ms.vh.add_or_update(item);
      if (!er.ok()) return fail(er.code, s);
      // :129
      ms.exec.last_event_task_id = v.task_id(s);

      const int t = v.type(s);
      switch (t) {
        case CRR_EV_WORKFLOW_EXECUTION_STARTED: {  // :132-183
          const crr_start_side& ss = in_->start_side[v.aux(s)];
          if (ss.parent_domain_status == CRR_DOMAIN_UNKNOWN) return fail(CRR_ERR_DOMAIN_NOT_FOUND, s);
          // ReplicateWorkflowExecutionStartedEvent (mutable_state_builder.go:1751-1829)
          ExecutionInfo& x = ms.exec;
          x.decision_start_to_close_timeout = ss.decision_start_to_close;
          x.start_src = s;  // CreateRequestID/DomainID/WorkflowID/RunID/TaskList/... by provenance
          er = update_workflow_state_close_status(x, CRR_STATE_CREATED, CRR_CLOSE_NONE);
          if (!er.ok()) return fail(er.code, s);
          x.last_processed_event = CRR_EMPTY_EVENT_ID;
          x.last_first_event_id = v.id(s);
          x.decision_version = CRR_EMPTY_VERSION;
          x.decision_schedule_id = CRR_EMPTY_EVENT_ID;
          x.decision_started_id = CRR_EMPTY_EVENT_ID;
          x.decision_request_src = CRR_SRC_EMPTY_UUID;
          x.decision_timeout = 0;
          // AutoResetPoints = rolloverAutoResetPointsWithExpiringTime(...) (:1813-1818, :3343-3364)
          x.reset_points.clear();
          x.auto_reset_points_set = ss.prev_reset_count != -1;
          for (int i = 0; i < ss.prev_reset_count; ++i) {
            ResetPoint rp;
            rp.src = s;
            rp.prev_index = i;
            rp.key = in_->reset_keys[ss.prev_reset_key_off + i];
            rp.resettable = false;  // provenance only: Resettable copied from the prev point by the host
            x.reset_points.push_back(rp);
          }
          // taskGenerator.GenerateRecordWorkflowStartedTasks / GenerateWorkflowStartTasks: tasks only
          if (ss.expiration_ns != 0) ms.expiration_ns = ss.expiration_ns;  // (mutable_state_builder.go:1800-1802)
          // GenerateRecordWorkflowStartedTasks (task_generator.go:301-313)
          ms.AddTask(CRR_TASK_RECORD_WORKFLOW_STARTED, 0, v.version(s), 0, 0, 0, s);
          {  // GenerateWorkflowStartTasks (:143-166), startTime = event timestamp
            i64 vis = wadd(v.ts(s), wmul(wadd(ss.workflow_timeout, ss.first_decision_backoff), kSecond));
            if (ss.attempt > 0 && ms.expiration_ns != 0 && vis > ms.expiration_ns) vis = ms.expiration_ns;
            ms.AddTask(CRR_TASK_WORKFLOW_TIMEOUT, 0, v.version(s), vis, 0, 0, s);
          }
          // GenerateDelayedDecisionTasks (mutable_state_task_generator.go:260-299)
          if (ss.first_decision_backoff > 0) {
            if (ss.initiator != CRR_INITIATOR_NIL && ss.initiator != CRR_INITIATOR_RETRY_POLICY &&
                ss.initiator != CRR_INITIATOR_CRON)
              return fail(CRR_ERR_BAD_INITIATOR, s);
            ms.AddTask(CRR_TASK_WORKFLOW_BACKOFF,
                       ss.initiator == CRR_INITIATOR_RETRY_POLICY ? CRR_BACKOFF_RETRY : CRR_BACKOFF_CRON, v.version(s),
                       wadd(v.ts(s), wmul(ss.first_decision_backoff, kSecond)), 0, 0, s);
          }
          // SetHistoryTree(runID) (:367-376): the branch token with the injected branchID
          ms.vh.token_src = 1;
          break;
        }
        case CRR_EV_DECISION_TASK_SCHEDULED: {  // :185-208
          er = ms.ReplicateDecisionTaskScheduledEvent(v.version(s), v.id(s), v.aux(s), v.ref(s), v.ts(s), v.ts(s));
          if (!er.ok()) return fail(er.code, s);
          // GenerateDecisionScheduleTasks (task_generator.go:315-350): sticky cleared, no schedule-to-start timer
          ms.AddTask(CRR_TASK_DECISION, 0, ms.exec.decision_version, 0, ms.exec.decision_schedule_id, 0, s);
          break;
        }
        case CRR_EV_DECISION_TASK_STARTED: {  // :210-228
          er = ms.ReplicateDecisionTaskStartedEvent(v.version(s), v.ref(s), v.id(s), s, v.ts(s));
          if (!er.ok()) return fail(er.code, s);
          // GenerateDecisionStartTasks (task_generator.go:352-388): Attempt == 0, no timeout override
          ms.AddTask(CRR_TASK_DECISION_TIMEOUT, CRR_TIMEOUT_START_TO_CLOSE, ms.exec.decision_version,
                     wadd(v.ts(s), wmul(ms.exec.decision_timeout, kSecond)), ms.exec.decision_schedule_id,
                     (int)ms.exec.decision_attempt, s);
          break;
        }
        case CRR_EV_DECISION_TASK_COMPLETED:  // :230-235
          ms.ReplicateDecisionTaskCompletedEvent(v.ref(s), v.kstr(s), v.key(s), s);
          break;
        case CRR_EV_DECISION_TASK_TIMED_OUT:  // :237-259
          // ReplicateDecisionTaskTimedOutEvent (:256-271): StickyTaskList == "" after ClearStickyness
          ms.FailDecision(true);
          if (ms.ReplicateTransientDecisionTaskScheduled())  // its schedule task: task list of the start event
            ms.AddTask(CRR_TASK_DECISION, 0, ms.exec.decision_version, 0, ms.exec.decision_schedule_id, 0,
                       ms.exec.start_src);
          break;
        case CRR_EV_DECISION_TASK_FAILED:  // :261-281
          ms.FailDecision(true);
          if (ms.ReplicateTransientDecisionTaskScheduled())  // its schedule task: task list of the start event
            ms.AddTask(CRR_TASK_DECISION, 0, ms.exec.decision_version, 0, ms.exec.decision_schedule_id, 0,
                       ms.exec.start_src);
          break;
        case CRR_EV_ACTIVITY_TASK_SCHEDULED: {  // :283-295 -> mutable_state_builder.go:2142-2197
          const crr_activity_side& as = in_->act_side[v.aux(s)];
          if (as.domain_status == CRR_DOMAIN_UNKNOWN) return fail(CRR_ERR_DOMAIN_NOT_FOUND, s);
          ActivityInfo ai;
          ai.version = v.version(s);
          ai.schedule_id = v.id(s);
          ai.scheduled_batch_id = firstEventID;
          ai.scheduled_time = v.ts(s);
          ai.started_id = CRR_EMPTY_EVENT_ID;
          ai.started_time = CRR_ZERO_TIME;
          ai.activity_id = v.kstr(s);
          ai.key = v.key(s);
          ai.sched_src = s;
          ai.schedule_to_start = as.schedule_to_start;
          ai.schedule_to_close = as.schedule_to_close;
          ai.start_to_close = as.start_to_close;
          ai.heartbeat = as.heartbeat;
          ai.cancel_requested = false;
          ai.cancel_request_id = CRR_EMPTY_EVENT_ID;
          ai.last_heartbeat_updated_time = CRR_ZERO_TIME;
          ai.timer_task_status = CRR_TIMER_TASK_STATUS_NONE;
          ai.has_retry_policy = as.has_retry_policy != 0;
          ms.pendingActivityInfoIDs[ai.schedule_id] = ai;
          ms.pendingActivityIDToEventID[ai.activity_id] = ai.schedule_id;
          // GenerateActivityTransferTasks (task_generator.go:390-428): ai.DomainID != "" -> no lookup
          ms.AddTask(CRR_TASK_ACTIVITY, 0, ai.version, 0, ai.schedule_id, 0, s);
          break;
        }
        case CRR_EV_ACTIVITY_TASK_STARTED: {  // :297-302 -> :2254-2276
          auto it = ms.pendingActivityInfoIDs.find(v.ref(s));
          if (it == ms.pendingActivityInfoIDs.end()) return fail(CRR_ERR_MISSING_ACTIVITY_INFO, s);
          ActivityInfo& ai = it->second;
          ai.version = v.version(s);
          ai.started_id = v.id(s);
          ai.started_src = s;  // RequestID
          ai.started_time = v.ts(s);
          ai.last_heartbeat_updated_time = ai.started_time;
          break;
        }
        case CRR_EV_ACTIVITY_TASK_COMPLETED:  // :304-309 -> :2312-2320
        case CRR_EV_ACTIVITY_TASK_FAILED:     // :311-316 -> :2354-2362
        case CRR_EV_ACTIVITY_TASK_TIMED_OUT:  // :318-323 -> :2400-2408
        case CRR_EV_ACTIVITY_TASK_CANCELED:   // :332-337 -> :2528-2536
          ms.DeleteActivity(v.ref(s));
          break;
        case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED: {  // :325-330 -> :2444-2467
          ActivityInfo* ai = ms.GetActivityByActivityID(v.kstr(s));
          if (ai == nullptr) break;
          ai->version = v.version(s);
          ai->cancel_requested = true;
          ai->cancel_request_id = v.id(s);
          break;
        }
        case CRR_EV_REQUEST_CANCEL_ACTIVITY_TASK_FAILED:  // :339-340
          break;
        case CRR_EV_TIMER_STARTED: {  // :342-347 -> :3057-3081
          TimerInfo ti;
          ti.version = v.version(s);
          ti.timer_id = v.kstr(s);
          ti.key = v.key(s);
          ti.expiry_time = add_seconds(v.ts(s), v.ref(s));
          ti.started_id = v.id(s);
          ti.task_status = CRR_TIMER_TASK_STATUS_NONE;
          ti.src = s;
          ms.pendingTimerInfoIDs[ti.timer_id] = ti;
          ms.pendingTimerEventIDToID[ti.started_id] = ti.timer_id;
          break;
        }
        case CRR_EV_TIMER_FIRED:     // :349-354 -> :3109-3117
        case CRR_EV_TIMER_CANCELED:  // :356-361 -> :3160-3168
          ms.DeleteUserTimer(v.kstr(s));
          break;
        case CRR_EV_CANCEL_TIMER_FAILED:  // :363-364
          break;
        case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED: {  // :366-381 -> :3417-3453
          if (v.aux(s) == CRR_DOMAIN_UNKNOWN) return fail(CRR_ERR_DOMAIN_NOT_FOUND, s);
          ChildExecutionInfo ci;
          ci.version = v.version(s);
          ci.initiated_id = v.id(s);
          ci.initiated_batch_id = firstEventID;
          ci.started_id = CRR_EMPTY_EVENT_ID;
          ci.src = s;  // StartedWorkflowID / WorkflowTypeName / ParentClosePolicy / CreateRequestID=uuid(s)
          ms.pendingChildExecutionInfoIDs[ci.initiated_id] = ci;
          // GenerateChildWorkflowTasks (task_generator.go:451-498): info present, domain resolved
          ms.AddTask(CRR_TASK_START_CHILD, 0, ci.version, 0, ci.initiated_id, 0, s);
          break;
        }
        case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED:      // :383-388 -> :3537-3545
        case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED:         // :397-402 -> :3590-3598
        case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED:            // :404-409 -> :3643-3651
        case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED:          // :411-416 -> :3696-3704
        case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT:         // :418-423 -> :3802-3810
        case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED:        // :425-430 -> :3749-3757
          ms.delete_initiated(ms.pendingChildExecutionInfoIDs, v.ref(s));
          break;
        case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED: {  // :390-395 -> :3485-3507
          auto it = ms.pendingChildExecutionInfoIDs.find(v.ref(s));
          if (it == ms.pendingChildExecutionInfoIDs.end()) return fail(CRR_ERR_MISSING_CHILD_INFO, s);
          it->second.started_id = v.id(s);
          it->second.started_src = s;  // StartedRunID
          break;
        }
        case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED: {  // :432-447 -> :2760-2779
          InitiatedInfo ri;
          ri.version = v.version(s);
          ri.initiated_batch_id = firstEventID;
          ri.initiated_id = v.id(s);
          ri.src = s;  // CancelRequestID = uuid(s)
          ms.pendingRequestCancelInfoIDs[ri.initiated_id] = ri;
          // GenerateRequestCancelExternalTasks -> getTargetDomainID (task_generator.go:556-559)
          if (v.aux(s) == CRR_DOMAIN_UNKNOWN) return fail(CRR_ERR_DOMAIN_NOT_FOUND, s);
          ms.AddTask(CRR_TASK_CANCEL_EXECUTION, 0, v.version(s), 0, v.id(s), 0, s);  // (:529-546)
          break;
        }
        case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED:               // :449-454 -> :2849-2856
        case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED:  // :456-461 -> :2809-2816
          ms.delete_initiated(ms.pendingRequestCancelInfoIDs, v.ref(s));
          break;
        case CRR_EV_SIGNAL_EXTERNAL_INITIATED: {  // :463-478 -> :2883-2905
          InitiatedInfo si;
          si.version = v.version(s);
          si.initiated_batch_id = firstEventID;
          si.initiated_id = v.id(s);
          si.src = s;  // SignalRequestID = uuid(s), SignalName/Input/Control from the event
          ms.pendingSignalInfoIDs[si.initiated_id] = si;
          // GenerateSignalExternalTasks -> getTargetDomainID (task_generator.go:604-607)
          if (v.aux(s) == CRR_DOMAIN_UNKNOWN) return fail(CRR_ERR_DOMAIN_NOT_FOUND, s);
          ms.AddTask(CRR_TASK_SIGNAL_EXECUTION, 0, v.version(s), 0, v.id(s), 0, s);  // (:580-597)
          break;
        }
        case CRR_EV_SIGNAL_EXTERNAL_FAILED:                 // :480-485 -> :3020-3027
        case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED:  // :487-492 -> :2979-2986
          ms.delete_initiated(ms.pendingSignalInfoIDs, v.ref(s));
          break;
        case CRR_EV_MARKER_RECORDED:  // :494-495
          break;
        case CRR_EV_WORKFLOW_EXECUTION_SIGNALED:  // :497-502 -> :3260-3267
          ms.exec.signal_count = (i32)((uint32_t)ms.exec.signal_count + 1u);
          break;
        case CRR_EV_WORKFLOW_EXECUTION_CANCEL_REQUESTED:  // :504-509 -> :2688-2694
          ms.exec.cancel_requested = true;
          break;
        case CRR_EV_UPSERT_WORKFLOW_SEARCH_ATTRIBUTES:  // :511-515 -> :2926-2948 (map merge: host materialised)
          ms.AddTask(CRR_TASK_UPSERT_SEARCH_ATTRIBUTES, 0, ms.currentVersion, 0, 0, 0, s);  // (:602-612)
          break;
        case CRR_EV_WORKFLOW_EXECUTION_COMPLETED:   // :517-529 -> :2561-2576
        case CRR_EV_WORKFLOW_EXECUTION_FAILED:      // :531-543 -> :2601-2616
        case CRR_EV_WORKFLOW_EXECUTION_TIMED_OUT:   // :545-557 -> :2640-2655
        case CRR_EV_WORKFLOW_EXECUTION_CANCELED:    // :559-571 -> :2719-2733
        case CRR_EV_WORKFLOW_EXECUTION_TERMINATED: {  // :573-585 -> :3225-3240
          int cs = t == CRR_EV_WORKFLOW_EXECUTION_COMPLETED ? CRR_CLOSE_COMPLETED
                 : t == CRR_EV_WORKFLOW_EXECUTION_FAILED    ? CRR_CLOSE_FAILED
                 : t == CRR_EV_WORKFLOW_EXECUTION_TIMED_OUT ? CRR_CLOSE_TIMED_OUT
                 : t == CRR_EV_WORKFLOW_EXECUTION_CANCELED  ? CRR_CLOSE_CANCELED
                                                            : CRR_CLOSE_TERMINATED;
          er = update_workflow_state_close_status(ms.exec, CRR_STATE_COMPLETED, cs);
          if (!er.ok()) return fail(er.code, s);
          ms.exec.completion_event_batch_id = firstEventID;
          ms.ClearStickyness();
          CloseTasks(ms, v, s);  // GenerateWorkflowCloseTasks: domain lookups resolve (host-validated)
          break;
        }
        case CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW: {  // :587-627
          int nr = v.aux(s);
          if (nr >= 0) {  // len(newRunHistory) != 0: nested replay happened in phase 0
            if ((uint32_t)nr >= in_->n_wf) return fail(CRR_ERR_NEW_RUN_MISSING, s);
            if (phase0_ && phase0_[nr].status != CRR_OK) return fail(phase0_[nr].status, s);
          }
          // ReplicateWorkflowExecutionContinuedAsNewEvent (:3366-3382)
          er = update_workflow_state_close_status(ms.exec, CRR_STATE_COMPLETED, CRR_CLOSE_CONTINUED_AS_NEW);
          if (!er.ok()) return fail(er.code, s);
          ms.exec.completion_event_batch_id = firstEventID;
          ms.ClearStickyness();
          CloseTasks(ms, v, s);
          break;
        }
        default:  // :629-630
          return fail(CRR_ERR_UNKNOWN_EVENT_TYPE, s);
      }
    }
    // :634-640 must generate the activity timer / user timer at the very end
    Err er = CreateNextActivityTimer(ms);
    if (!er.ok()) return fail(er.code, e - 1);
    er = CreateNextUserTimer(ms);
    if (!er.ok()) return fail(er.code, e - 1);
    // :642-643
    ms.exec.last_first_event_id = firstEventID;
    ms.exec.next_event_id = lastEventID + 1;
    return out;
  }

  const crr_inputs* in_;
  const KeyStrings* ks_;
  const Outcome* phase0_;
};

// ---- checksum payload (checksum.go:56-114 + thriftrw binary protocol) ------------------------------
struct Writer {
  std::vector<uint8_t> b;
  void u8(uint8_t x) { b.push_back(x); }
  void be16(uint16_t x) { u8(x >> 8); u8(x & 0xff); }
  void be32(uint32_t x) { for (int i = 3; i >= 0; --i) u8((x >> (8 * i)) & 0xff); }
  void be64(uint64_t x) { for (int i = 7; i >= 0; --i) u8((x >> (8 * i)) & 0xff); }
  void field(uint8_t type, uint16_t id) { u8(type); be16(id); }  // WriteFieldBegin
  void list_begin(uint8_t elem, uint32_t n) { u8(elem); be32(n); }  // WriteListBegin
  void stop() { u8(0); }  // WriteStructEnd
};
enum : uint8_t { TBOOL = 2, TI16 = 6, TI32 = 8, TI64 = 10, TBINARY = 11, TSTRUCT = 12, TLIST = 15 };

void build_payload(const crr_inputs* in, const crr_workflow* wf, const MutableState& ms, std::vector<uint8_t>* out) {
  Writer w;
  w.u8(0x59);  // preambleVersion0 (common/codec/interface.go:48, version0Thriftrw.go:50)
  const ExecutionInfo& x = ms.exec;
  // MutableStateChecksumPayload.Encode (.gen/go/checksum/checksum.go:539-821), field order by ID
  w.field(TBOOL, 10); w.u8(x.cancel_requested ? 1 : 0);
  w.field(TI16, 15); w.be16((uint16_t)(int16_t)x.state);
  w.field(TI64, 23); w.be64((uint64_t)x.last_first_event_id);
  w.field(TI64, 24); w.be64((uint64_t)x.next_event_id);
  w.field(TI64, 25); w.be64((uint64_t)x.last_processed_event);
  w.field(TI64, 26); w.be64((uint64_t)(i64)x.signal_count);
  w.field(TI32, 35); w.be32((uint32_t)(i32)x.decision_attempt);
  w.field(TI64, 36); w.be64((uint64_t)x.decision_version);
  w.field(TI64, 37); w.be64((uint64_t)x.decision_schedule_id);
  w.field(TI64, 38); w.be64((uint64_t)x.decision_started_id);
  std::vector<i64> timers, acts, sigs, rcs, childs;
  for (const auto& kv : ms.pendingTimerInfoIDs) timers.push_back(kv.second.started_id);
  for (const auto& kv : ms.pendingActivityInfoIDs) acts.push_back(kv.first);
  for (const auto& kv : ms.pendingSignalInfoIDs) sigs.push_back(kv.first);
  for (const auto& kv : ms.pendingRequestCancelInfoIDs) rcs.push_back(kv.first);
  for (const auto& kv : ms.pendingChildExecutionInfoIDs) childs.push_back(kv.first);
  auto emit_list = [&](uint16_t id, std::vector<i64> v) {  // common.SortInt64Slice then _List_I64_Encode
    std::sort(v.begin(), v.end());
    w.field(TLIST, id);
    w.list_begin(TI64, (uint32_t)v.size());
    for (i64 z : v) w.be64((uint64_t)z);
  };
  emit_list(45, timers);
  emit_list(46, acts);
  emit_list(47, sigs);
  emit_list(48, rcs);
  emit_list(49, childs);
  w.field(TBINARY, 55); w.be32(0);  // StickyTaskListName "" (always present)
  // VersionHistories.Encode (.gen/go/shared/shared.go:91639) via thrift.FromVersionHistories
  w.field(TSTRUCT, 56);
  w.field(TI32, 10); w.be32(0);  // CurrentVersionHistoryIndex
  w.field(TLIST, 20); w.list_begin(TSTRUCT, 1);
  {  // VersionHistory.Encode (:92043): BranchToken always non-nil after ToInternalType
    uint32_t off = 0, len = 0;
    if (ms.vh.token_src == 1) { off = wf->start_token_off; len = wf->start_token_len; }
    if (ms.vh.token_src == 2) { off = wf->final_token_off; len = wf->final_token_len; }
    w.field(TBINARY, 10); w.be32(len);
    for (uint32_t i = 0; i < len; ++i) w.u8(in->arena[off + i]);
    w.field(TLIST, 20); w.list_begin(TSTRUCT, (uint32_t)ms.vh.items.size());
    for (const auto& it : ms.vh.items) {  // VersionHistoryItem.Encode (:92375)
      w.field(TI64, 10); w.be64((uint64_t)it.event_id);
      w.field(TI64, 20); w.be64((uint64_t)it.version);
      w.stop();
    }
    w.stop();
  }
  w.stop();  // VersionHistories
  w.stop();  // payload
  *out = std::move(w.b);
}

// hash/crc32 ChecksumIEEE, bitwise reflected polynomial 0xEDB88320 (crc.go:46)
uint32_t crc32_ieee_bitwise(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  }
  return ~c;
}

// ---- row export ------------------------------------------------------------------------------------
void export_rows(const crr_inputs* in, uint32_t w, const MutableState& ms, const Outcome& oc,
                 const crr_outputs* out, int src_next) {
  const crr_workflow* wf = &in->wf[w];
  const i64 st = stride_of(in, wf);
  crr_exec_row& r = out->exec[w];
  std::memset(&r, 0, sizeof(r));
  const ExecutionInfo& x = ms.exec;
  r.status = oc.status;
  r.fail_step = oc.fail_step;
  r.inconsistencies = ms.inconsistencies;
  r.flags = (x.cancel_requested ? CRR_EXEC_CANCEL_REQUESTED : 0u) | (x.auto_reset_points_set ? CRR_EXEC_RESET_POINTS_SET : 0u);
  r.state = x.state;
  r.close_status = x.close_status;
  r.signal_count = x.signal_count;
  r.decision_timeout = x.decision_timeout;
  r.next_event_id = x.next_event_id;
  r.last_first_event_id = x.last_first_event_id;
  r.last_event_task_id = x.last_event_task_id;
  r.last_processed_event = x.last_processed_event;
  r.completion_event_batch_id = x.completion_event_batch_id;
  r.decision_version = x.decision_version;
  r.decision_schedule_id = x.decision_schedule_id;
  r.decision_started_id = x.decision_started_id;
  r.decision_attempt = x.decision_attempt;
  r.decision_started_ts = x.decision_started_ts;
  r.decision_scheduled_ts = x.decision_scheduled_ts;
  r.decision_orig_scheduled_ts = x.decision_orig_scheduled_ts;
  r.current_version = ms.currentVersion;
  r.decision_request_src = x.decision_request_src;
  r.start_src = x.start_src;
  r.token_src = ms.vh.token_src;
  r.decision_start_to_close = x.decision_start_to_close_timeout;
  r.expiration_ns = ms.expiration_ns;
  r.src_next = src_next;

  // pending activities sorted by ScheduleID
  std::vector<const ActivityInfo*> acts;
  for (const auto& kv : ms.pendingActivityInfoIDs) acts.push_back(&kv.second);
  std::sort(acts.begin(), acts.end(), [](const ActivityInfo* a, const ActivityInfo* b) { return a->schedule_id < b->schedule_id; });
  r.n_activity = (i32)acts.size();
  for (size_t i = 0; i < acts.size() && (i32)i < wf->act_cap; ++i) {
    const ActivityInfo& a = *acts[i];
    crr_activity_row& o = out->act[wf->act_base + (i64)i * st];
    std::memset(&o, 0, sizeof(o));
    o.schedule_id = a.schedule_id; o.version = a.version; o.scheduled_batch_id = a.scheduled_batch_id;
    o.scheduled_time = a.scheduled_time; o.started_id = a.started_id; o.started_time = a.started_time;
    o.cancel_request_id = a.cancel_request_id; o.last_hb_timeout_vis_s = a.last_hb_timeout_vis_s;
    o.sched_src = a.sched_src; o.started_src = a.started_src;
    o.schedule_to_start = a.schedule_to_start; o.schedule_to_close = a.schedule_to_close;
    o.start_to_close = a.start_to_close; o.heartbeat = a.heartbeat;
    o.timer_task_status = a.timer_task_status; o.key = a.key;
    o.last_heartbeat_time = a.last_heartbeat_updated_time;
    o.attempt = a.attempt;
    auto m = ms.pendingActivityIDToEventID.find(a.activity_id);
    bool mapped = m != ms.pendingActivityIDToEventID.end() && m->second == a.schedule_id;
    o.flags = CRR_ROW_LIVE | (mapped ? CRR_ROW_MAPPED : 0u) | (a.cancel_requested ? CRR_ROW_CANCEL_REQUESTED : 0u) |
              (a.has_retry_policy ? CRR_ROW_HAS_RETRY : 0u);
  }
  std::vector<const TimerInfo*> tis;
  for (const auto& kv : ms.pendingTimerInfoIDs) tis.push_back(&kv.second);
  std::sort(tis.begin(), tis.end(), [](const TimerInfo* a, const TimerInfo* b) { return a->started_id < b->started_id; });
  r.n_timer = (i32)tis.size();
  for (size_t i = 0; i < tis.size() && (i32)i < wf->timer_cap; ++i) {
    crr_timer_row& o = out->timer[wf->timer_base + (i64)i * st];
    std::memset(&o, 0, sizeof(o));
    o.started_id = tis[i]->started_id; o.version = tis[i]->version; o.expiry_time = tis[i]->expiry_time;
    o.task_status = (i32)tis[i]->task_status; o.key = tis[i]->key; o.src = tis[i]->src; o.flags = CRR_ROW_LIVE;
  }
  std::vector<const ChildExecutionInfo*> cis;
  for (const auto& kv : ms.pendingChildExecutionInfoIDs) cis.push_back(&kv.second);
  std::sort(cis.begin(), cis.end(), [](const ChildExecutionInfo* a, const ChildExecutionInfo* b) { return a->initiated_id < b->initiated_id; });
  r.n_child = (i32)cis.size();
  for (size_t i = 0; i < cis.size() && (i32)i < wf->child_cap; ++i) {
    crr_child_row& o = out->child[wf->child_base + (i64)i * st];
    std::memset(&o, 0, sizeof(o));
    o.initiated_id = cis[i]->initiated_id; o.version = cis[i]->version; o.initiated_batch_id = cis[i]->initiated_batch_id;
    o.started_id = cis[i]->started_id; o.src = cis[i]->src; o.started_src = cis[i]->started_src; o.flags = CRR_ROW_LIVE;
  }
  auto export_init = [&](const std::unordered_map<i64, InitiatedInfo>& m, crr_initiated_row* base_ptr, i64 base, i32 cap, i32* n) {
    std::vector<const InitiatedInfo*> v;
    for (const auto& kv : m) v.push_back(&kv.second);
    std::sort(v.begin(), v.end(), [](const InitiatedInfo* a, const InitiatedInfo* b) { return a->initiated_id < b->initiated_id; });
    *n = (i32)v.size();
    for (size_t i = 0; i < v.size() && (i32)i < cap; ++i) {
      crr_initiated_row& o = base_ptr[base + (i64)i * st];
      std::memset(&o, 0, sizeof(o));
      o.initiated_id = v[i]->initiated_id; o.version = v[i]->version; o.initiated_batch_id = v[i]->initiated_batch_id;
      o.src = v[i]->src; o.flags = CRR_ROW_LIVE;
    }
  };
  export_init(ms.pendingRequestCancelInfoIDs, out->rc, wf->rc_base, wf->rc_cap, &r.n_rc);
  export_init(ms.pendingSignalInfoIDs, out->sig, wf->sig_base, wf->sig_cap, &r.n_signal);
  r.n_vh_items = (i32)ms.vh.items.size();
  for (size_t i = 0; i < ms.vh.items.size() && (i32)i < wf->vh_cap; ++i) {
    crr_vh_item& o = out->vh[wf->vh_base + (i64)i * st];
    o.event_id = ms.vh.items[i].event_id;
    o.version = ms.vh.items[i].version;
  }
  r.n_tasks = (i32)ms.tasks.size();
  if (in->flags & CRR_IN_EMIT_TASKS)
    for (size_t i = 0; i < ms.tasks.size() && (i32)i < wf->task_cap; ++i) out->tasks[wf->task_base + (i64)i * st] = ms.tasks[i];
  r.n_reset_points = (i32)x.reset_points.size();
  for (size_t i = 0; i < x.reset_points.size() && (i32)i < wf->rp_cap; ++i) {
    crr_reset_point_row& o = out->rp[wf->rp_base + (i64)i * st];
    o.src = x.reset_points[i].src; o.prev_index = x.reset_points[i].prev_index; o.key = x.reset_points[i].key;
    o.flags = CRR_ROW_LIVE | (x.reset_points[i].resettable ? CRR_ROW_RESETTABLE : 0u);
  }
  bool overflow = r.n_activity > wf->act_cap || r.n_timer > wf->timer_cap || r.n_child > wf->child_cap ||
                  r.n_rc > wf->rc_cap || r.n_signal > wf->sig_cap || r.n_vh_items > wf->vh_cap ||
                  r.n_reset_points > wf->rp_cap || r.n_tasks > wf->task_cap;
  if (overflow && r.status == CRR_OK) r.status = CRR_ERR_CAPACITY;
  if (r.status == CRR_OK) {
    std::vector<uint8_t> payload;
    build_payload(in, wf, ms, &payload);
    r.checksum = crc32_ieee_bitwise(payload.data(), payload.size());
    r.payload_len = (uint32_t)payload.size();
    r.flags |= CRR_EXEC_CHECKSUM_VALID;
  }
}

// mutableStateBuilder.Load (mutable_state_builder.go:306-349) from the engine's row image of a loaded
// state (out->exec[w] and slots 0..n-1 of the workflow's tables).  Returns the provenance base (src_next).
int load_state(const crr_inputs* in, uint32_t w, const crr_outputs* out, const KeyDict& kd, MutableState& ms) {
  const crr_workflow* wf = &in->wf[w];
  const i64 st = stride_of(in, wf);
  const crr_exec_row X = out->exec[w];
  ExecutionInfo& x = ms.exec;
  x.state = X.state; x.close_status = X.close_status;
  x.next_event_id = X.next_event_id; x.last_first_event_id = X.last_first_event_id;
  x.last_event_task_id = X.last_event_task_id; x.last_processed_event = X.last_processed_event;
  x.completion_event_batch_id = X.completion_event_batch_id;
  x.decision_version = X.decision_version; x.decision_schedule_id = X.decision_schedule_id;
  x.decision_started_id = X.decision_started_id; x.decision_request_src = X.decision_request_src;
  x.decision_timeout = X.decision_timeout; x.decision_attempt = X.decision_attempt;
  x.decision_started_ts = X.decision_started_ts; x.decision_scheduled_ts = X.decision_scheduled_ts;
  x.decision_orig_scheduled_ts = X.decision_orig_scheduled_ts;
  x.signal_count = X.signal_count;
  x.cancel_requested = (X.flags & CRR_EXEC_CANCEL_REQUESTED) != 0;
  x.decision_start_to_close_timeout = X.decision_start_to_close;
  x.start_src = X.start_src;
  x.auto_reset_points_set = (X.flags & CRR_EXEC_RESET_POINTS_SET) != 0;
  ms.expiration_ns = X.expiration_ns;
  ms.currentVersion = CRR_EMPTY_VERSION;  // e.currentVersion = common.EmptyVersion (:324)
  ms.vh.token_src = X.token_src;
  for (int i = 0; i < X.n_vh_items; ++i) {
    const crr_vh_item& it = out->vh[wf->vh_base + (i64)i * st];
    ms.vh.items.push_back({it.event_id, it.version});
  }
  // e.pendingActivityInfoIDs = state.ActivityInfos; then pendingActivityIDToEventID[ActivityID] =
  // ScheduleID for every info (:311-314).  Go iterates a map: among duplicate ActivityIDs the winner is
  // arbitrary; this restatement (and the engine) let the latest scheduled one win.
  std::vector<i64> sids;
  for (int i = 0; i < X.n_activity; ++i) {
    const crr_activity_row& o = out->act[wf->act_base + (i64)i * st];
    ActivityInfo a;
    a.version = o.version; a.schedule_id = o.schedule_id; a.scheduled_batch_id = o.scheduled_batch_id;
    a.scheduled_time = o.scheduled_time; a.started_id = o.started_id; a.started_time = o.started_time;
    a.activity_id = kd.str(w, o.key); a.key = o.key;
    a.sched_src = o.sched_src; a.started_src = o.started_src;
    a.schedule_to_start = o.schedule_to_start; a.schedule_to_close = o.schedule_to_close;
    a.start_to_close = o.start_to_close; a.heartbeat = o.heartbeat;
    a.cancel_requested = (o.flags & CRR_ROW_CANCEL_REQUESTED) != 0;
    a.cancel_request_id = o.cancel_request_id;
    a.last_heartbeat_updated_time = o.last_heartbeat_time;
    a.attempt = o.attempt;
    a.timer_task_status = o.timer_task_status;
    a.has_retry_policy = (o.flags & CRR_ROW_HAS_RETRY) != 0;
    a.last_hb_timeout_vis_s = o.last_hb_timeout_vis_s;
    ms.pendingActivityInfoIDs[a.schedule_id] = a;
    sids.push_back(a.schedule_id);
  }
  std::sort(sids.begin(), sids.end());
  for (i64 sid : sids) ms.pendingActivityIDToEventID[ms.pendingActivityInfoIDs[sid].activity_id] = sid;
  for (int i = 0; i < X.n_timer; ++i) {  // e.pendingTimerInfoIDs = state.TimerInfos (+ StartedID -> TimerID)
    const crr_timer_row& o = out->timer[wf->timer_base + (i64)i * st];
    TimerInfo t;
    t.version = o.version; t.timer_id = kd.str(w, o.key); t.key = o.key;
    t.started_id = o.started_id; t.expiry_time = o.expiry_time; t.task_status = o.task_status; t.src = o.src;
    ms.pendingTimerInfoIDs[t.timer_id] = t;
    ms.pendingTimerEventIDToID[t.started_id] = t.timer_id;
  }
  for (int i = 0; i < X.n_child; ++i) {
    const crr_child_row& o = out->child[wf->child_base + (i64)i * st];
    ChildExecutionInfo c;
    c.version = o.version; c.initiated_id = o.initiated_id; c.initiated_batch_id = o.initiated_batch_id;
    c.started_id = o.started_id; c.src = o.src; c.started_src = o.started_src;
    ms.pendingChildExecutionInfoIDs[c.initiated_id] = c;
  }
  auto load_init = [&](const crr_initiated_row* rows, i64 base, int n, std::unordered_map<i64, InitiatedInfo>& m) {
    for (int i = 0; i < n; ++i) {
      const crr_initiated_row& o = rows[base + (i64)i * st];
      InitiatedInfo r;
      r.version = o.version; r.initiated_batch_id = o.initiated_batch_id; r.initiated_id = o.initiated_id; r.src = o.src;
      m[r.initiated_id] = r;
    }
  };
  load_init(out->rc, wf->rc_base, X.n_rc, ms.pendingRequestCancelInfoIDs);
  load_init(out->sig, wf->sig_base, X.n_signal, ms.pendingSignalInfoIDs);
  for (int i = 0; i < X.n_reset_points; ++i) {  // executionInfo.AutoResetPoints.Points
    const crr_reset_point_row& o = out->rp[wf->rp_base + (i64)i * st];
    ResetPoint p;
    p.src = o.src; p.prev_index = o.prev_index; p.key = o.key;
    p.checksum = o.prev_index < 0 ? kd.str(w, o.key) : std::string();
    p.resettable = (o.flags & CRR_ROW_RESETTABLE) != 0;
    x.reset_points.push_back(p);
  }
  return X.src_next;
}

struct RunCtx {
  const crr_inputs* in;
  const KeyStrings* ks;
  const KeyDict* kd;
  const crr_outputs* out;
  std::vector<Outcome>* phase0;
};

void run_range(const RunCtx& c, uint32_t lo, uint32_t hi, int phase, std::atomic<uint32_t>* next) {
  (void)lo; (void)hi;
  for (;;) {
    uint32_t w0 = next->fetch_add(256);
    if (w0 >= hi) break;
    uint32_t w1 = std::min<uint32_t>(w0 + 256, hi);
    for (uint32_t w = w0; w < w1; ++w) {
      bool is_new_run = (c.in->wf[w].flags & CRR_WF_FLAG_NEW_RUN) != 0;
      if ((phase == 0) != is_new_run) continue;
      MutableState ms;
      int sb = 0;
      if (c.in->wf[w].flags & CRR_WF_FLAG_RESUME) sb = load_state(c.in, w, c.out, *c.kd, ms);
      Replayer rep(c.in, c.ks, phase == 0 ? nullptr : c.phase0->data());
      Outcome oc = rep.replay(w, ms, sb);
      if (phase == 0) (*c.phase0)[w] = oc;
      export_rows(c.in, w, ms, oc, c.out, sb + c.in->wf[w].ev_count);
    }
  }
}

}  // namespace

extern "C" {

// Replays every workflow of `in` (host pointers) into `out` (host pointers, same row layout as the
// device engine).  key_off/key_len/key_arena give the per-event key strings.  n_threads <= 0: all.
// Workflows flagged CRR_WF_FLAG_RESUME continue the loaded state their rows in `out` hold (in place);
// dict_* give each workflow's key id -> string table for those rows (required when any resumes).
int oracle_replay2(const crr_inputs* in, const uint32_t* key_off, const uint32_t* key_len, const char* key_arena,
                   const uint32_t* dict_begin, const uint32_t* dict_count, const uint32_t* dict_off,
                   const uint32_t* dict_len, const char* dict_arena, const crr_outputs* out, int n_threads) {
  if (!in || !out) return -1;
  KeyStrings ks{key_off, key_len, key_arena};
  KeyDict kd{dict_begin, dict_count, dict_off, dict_len, dict_arena};
  for (uint32_t w = 0; w < in->n_wf; ++w)
    if ((in->wf[w].flags & CRR_WF_FLAG_RESUME) && !kd.ok()) return -2;
  std::vector<Outcome> phase0(in->n_wf);
  RunCtx c{in, &ks, &kd, out, &phase0};
  if (n_threads <= 0) n_threads = (int)std::max(1u, std::thread::hardware_concurrency());
  for (int phase = 0; phase < 2; ++phase) {
    std::atomic<uint32_t> next{0};
    if (n_threads == 1) {
      run_range(c, 0, in->n_wf, phase, &next);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < n_threads; ++t) th.emplace_back(run_range, std::cref(c), 0u, in->n_wf, phase, &next);
      for (auto& x : th) x.join();
    }
  }
  return 0;
}

int oracle_replay(const crr_inputs* in, const uint32_t* key_off, const uint32_t* key_len, const char* key_arena,
                  const crr_outputs* out, int n_threads) {
  return oracle_replay2(in, key_off, key_len, key_arena, nullptr, nullptr, nullptr, nullptr, nullptr, out, n_threads);
}

// Writes the checksum payload bytes of workflow `w` after replay (for golden-vector tests).
// Returns the payload length (bytes written up to cap), or -1.
int oracle_payload(const crr_inputs* in, const uint32_t* key_off, const uint32_t* key_len, const char* key_arena,
                   uint32_t w, uint8_t* buf, int cap) {
  if (!in || w >= in->n_wf) return -1;
  KeyStrings ks{key_off, key_len, key_arena};
  std::vector<Outcome> phase0(in->n_wf);
  // replay the new-run histories this workflow may depend on
  for (uint32_t i = 0; i < in->n_wf; ++i) {
    if (in->wf[i].flags & CRR_WF_FLAG_NEW_RUN) {
      MutableState m0;
      Replayer r0(in, &ks, nullptr);
      phase0[i] = r0.replay(i, m0);
    }
  }
  MutableState ms;
  bool nr = (in->wf[w].flags & CRR_WF_FLAG_NEW_RUN) != 0;
  Replayer rep(in, &ks, nr ? nullptr : phase0.data());
  rep.replay(w, ms);
  std::vector<uint8_t> payload;
  build_payload(in, &in->wf[w], ms, &payload);
  int n = (int)std::min<size_t>(payload.size(), (size_t)cap);
  if (buf) std::memcpy(buf, payload.data(), n);
  return (int)payload.size();
}

uint32_t oracle_crc32(const uint8_t* p, size_t n) { return crc32_ieee_bitwise(p, n); }

// ---- unit-level entry points restating reference KATs ----------------------------------------------
// VersionHistory.AddOrUpdateItem on a caller-held item list (versionHistory.go:193-226).
int oracle_vh_add_or_update(int64_t* ev_ids, int64_t* versions, int* n, int cap, int64_t event_id, int64_t version) {
  VersionHistory h;
  for (int i = 0; i < *n; ++i) h.items.push_back({ev_ids[i], versions[i]});
  VersionHistoryItem it;
  Err e = VersionHistory::new_item(event_id, version, &it);
  if (!e.ok()) return e.code;
  e = h.add_or_update(it);
  if (!e.ok()) return e.code;
  if ((int)h.items.size() > cap) return CRR_ERR_CAPACITY;
  *n = (int)h.items.size();
  for (int i = 0; i < *n; ++i) { ev_ids[i] = h.items[i].event_id; versions[i] = h.items[i].version; }
  return 0;
}

// WorkflowExecutionInfo.UpdateWorkflowStateCloseStatus (workflowExecutionInfo.go:45-165).
int oracle_update_state(int* state, int* close_status, int new_state, int new_close) {
  ExecutionInfo x;
  x.state = *state;
  x.close_status = *close_status;
  Err e = update_workflow_state_close_status(x, new_state, new_close);
  *state = x.state;
  *close_status = x.close_status;
  return e.code;
}

// LoadAndSortActivityTimers over caller rows (timer_sequence.go:219-254); returns count written.
// attempt[] receives each sequence ID's Attempt (the ActivityInfo's, getActivity*Timeout).
int oracle_activity_timer_sequence(const crr_activity_row* rows, int n, int64_t* ts, int64_t* eid, int32_t* type,
                                   int32_t* created, int32_t* attempt, int cap) {
  MutableState ms;
  for (int i = 0; i < n; ++i) {
    ActivityInfo a;
    a.schedule_id = rows[i].schedule_id; a.scheduled_time = rows[i].scheduled_time;
    a.started_id = rows[i].started_id; a.started_time = rows[i].started_time;
    a.last_heartbeat_updated_time = rows[i].last_heartbeat_time;
    a.schedule_to_start = rows[i].schedule_to_start; a.schedule_to_close = rows[i].schedule_to_close;
    a.start_to_close = rows[i].start_to_close; a.heartbeat = rows[i].heartbeat;
    a.timer_task_status = rows[i].timer_task_status;
    a.attempt = rows[i].attempt;
    ms.pendingActivityInfoIDs[a.schedule_id * 64 + i] = a;  // distinct map keys even for EmptyEventID rows
  }
  std::vector<TimerSequenceID> v = LoadAndSortActivityTimers(ms);
  int m = (int)std::min<size_t>(v.size(), (size_t)cap);
  for (int i = 0; i < m; ++i) {
    ts[i] = v[i].timestamp; eid[i] = v[i].event_id; type[i] = v[i].timer_type; created[i] = v[i].created;
    attempt[i] = v[i].attempt;
  }
  return (int)v.size();
}

// LoadAndSortUserTimers over caller rows (timer_sequence.go:201-217, getUserTimerTimeout :256-267).
int oracle_user_timer_sequence(const crr_timer_row* rows, int n, int64_t* ts, int64_t* eid, int32_t* type,
                               int32_t* created, int cap) {
  MutableState ms;
  for (int i = 0; i < n; ++i) {
    TimerInfo t;
    t.version = rows[i].version; t.started_id = rows[i].started_id; t.expiry_time = rows[i].expiry_time;
    t.task_status = rows[i].task_status; t.timer_id = std::to_string(i);
    ms.pendingTimerInfoIDs[t.timer_id] = t;
  }
  std::vector<TimerSequenceID> v = LoadAndSortUserTimers(ms);
  int m = (int)std::min<size_t>(v.size(), (size_t)cap);
  for (int i = 0; i < m; ++i) { ts[i] = v[i].timestamp; eid[i] = v[i].event_id; type[i] = v[i].timer_type; created[i] = v[i].created; }
  return (int)v.size();
}

}  // extern "C"
