// history_decode.cpp -- persisted history blobs (thriftrw) -> the replay engine's SoA columns.
//
// Host-side native code of the replay path (include/cadence_decode.h).  One pass over each blob:
// the thrift binary protocol is walked directly, the fields the state machine reads are written
// into columns / side records, everything else is skipped without materialising it.  Workflows are
// decoded in parallel chunks (std::thread), then the chunks are concatenated with offset fix-ups.
//
// Wire layout (.gen/go/shared/shared.go): HistoryEvent{10 EventId i64, 20 Timestamp i64,
// 30 EventType i32, 35 Version i64, 36 TaskId i64, 40..450 one *EventAttributes struct per type};
// thrift binary: field header = type byte + big-endian i16 id, i32/i64 big-endian, binary = be32
// length + bytes, list = element type + be32 count, struct = fields until a 0 byte.
#include "cadence_decode.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

using i64 = int64_t;
using i32 = int32_t;
using u32 = uint32_t;

enum : uint8_t { T_STOP = 0, T_BOOL = 2, T_BYTE = 3, T_DOUBLE = 4, T_I16 = 6, T_I32 = 8, T_I64 = 10,
                 T_STRING = 11, T_STRUCT = 12, T_MAP = 13, T_SET = 14, T_LIST = 15 };

struct DecodeError {
  int code;
};

// ---- thrift binary reader ---------------------------------------------------------------------------
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  void need(size_t n) const {
    if ((size_t)(end - p) < n) throw DecodeError{CRR_DECODE_TRUNCATED};
  }
  uint8_t u8() { need(1); return *p++; }
  i32 be32() {
    need(4);
    u32 v = ((u32)p[0] << 24) | ((u32)p[1] << 16) | ((u32)p[2] << 8) | p[3];
    p += 4;
    return (i32)v;
  }
  i64 be64() {
    need(8);
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
    p += 8;
    return (i64)v;
  }
  int16_t be16() {
    need(2);
    int16_t v = (int16_t)(((u32)p[0] << 8) | p[1]);
    p += 2;
    return v;
  }
  std::string str() {
    i32 n = be32();
    if (n < 0) throw DecodeError{CRR_DECODE_TRUNCATED};
    need((size_t)n);
    std::string s((const char*)p, (size_t)n);
    p += n;
    return s;
  }
  void skip(uint8_t type, int depth = 0) {
    if (depth > 64) throw DecodeError{CRR_DECODE_BAD_TYPE};
    switch (type) {
      case T_BOOL: case T_BYTE: need(1); p += 1; break;
      case T_I16: need(2); p += 2; break;
      case T_I32: need(4); p += 4; break;
      case T_DOUBLE: case T_I64: need(8); p += 8; break;
      case T_STRING: { i32 n = be32(); if (n < 0) throw DecodeError{CRR_DECODE_TRUNCATED}; need((size_t)n); p += n; break; }
      case T_STRUCT:
        for (;;) {
          uint8_t ft = u8();
          if (ft == T_STOP) break;
          be16();
          skip(ft, depth + 1);
        }
        break;
      case T_MAP: {
        uint8_t kt = u8(), vt = u8();
        i32 n = be32();
        if (n < 0) throw DecodeError{CRR_DECODE_TRUNCATED};
        for (i32 i = 0; i < n; ++i) { skip(kt, depth + 1); skip(vt, depth + 1); }
        break;
      }
      case T_SET: case T_LIST: {
        uint8_t et = u8();
        i32 n = be32();
        if (n < 0) throw DecodeError{CRR_DECODE_TRUNCATED};
        for (i32 i = 0; i < n; ++i) skip(et, depth + 1);
        break;
      }
      default: throw DecodeError{CRR_DECODE_BAD_TYPE};
    }
  }
  // typed reads of a field value; a mismatched wire type is skipped (thriftrw ignores it too)
  bool want(uint8_t got, uint8_t expect) {
    if (got == expect) return true;
    skip(got);
    return false;
  }
};

// ---- the fields one event contributes ----------------------------------------------------------------
struct Attr {
  i64 ref = 0;
  i32 aux = 0;
  std::string key;           // ActivityID / TimerID / BinaryChecksum
  bool has_key = false;
  std::string domain;        // attributes.Domain / ParentWorkflowDomain
  // ActivityTaskScheduled
  i32 s2s = 0, s2c = 0, st2c = 0, hb = 0, has_retry = 0, expiration = 0;
  // WorkflowExecutionStarted
  i32 task_s2c = 0, exec_s2c = 0, backoff = 0, initiator = CRR_INITIATOR_NIL, attempt = 0;
  i64 expiration_ts = 0;
  int prev_mode = -1;        // -1: PrevAutoResetPoints nil, -2: Points nil, 0: list
  std::vector<std::string> prev;
};

struct Event {
  i64 id = 0, ts = 0, ver = 0, task = 0;
  i32 type = 0;
  Attr a;
};

// Attribute field id (in HistoryEvent) -> event type: 40 + 10 * type for every type
// (shared.go:42000-42460: WorkflowExecutionStarted 40 ... UpsertWorkflowSearchAttributes 450).
inline int attr_type_of_field(int16_t id) {
  if (id < 40 || id > 450 || id % 10) return -1;
  return (id - 40) / 10;
}

void read_retry_policy(Reader& r, Attr& a) {  // RetryPolicy{60 ExpirationIntervalInSeconds i32}
  a.has_retry = 1;
  for (;;) {
    uint8_t ft = r.u8();
    if (ft == T_STOP) break;
    int16_t id = r.be16();
    if (id == 60 && r.want(ft, T_I32)) a.expiration = r.be32();
    else if (id != 60) r.skip(ft);
  }
}

void read_reset_points(Reader& r, Attr& a) {  // ResetPoints{10 Points list<ResetPointInfo{10 BinaryChecksum}>}
  a.prev_mode = -2;
  for (;;) {
    uint8_t ft = r.u8();
    if (ft == T_STOP) break;
    int16_t id = r.be16();
    if (id == 10 && ft == T_LIST) {
      uint8_t et = r.u8();
      i32 n = r.be32();
      if (n < 0) throw DecodeError{CRR_DECODE_TRUNCATED};
      a.prev_mode = 0;
      a.prev.clear();
      for (i32 i = 0; i < n; ++i) {
        if (et != T_STRUCT) { r.skip(et); a.prev.emplace_back(); continue; }
        std::string bc;
        for (;;) {
          uint8_t t2 = r.u8();
          if (t2 == T_STOP) break;
          int16_t id2 = r.be16();
          if (id2 == 10 && t2 == T_STRING) bc = r.str();
          else r.skip(t2);
        }
        a.prev.push_back(std::move(bc));
      }
    } else {
      r.skip(ft);
    }
  }
}

// The attribute struct of event type `t`: read the fields ApplyEvents consumes (field ids from
// shared.go's ToWire of each *EventAttributes struct), skip the rest.
void read_attributes(Reader& r, int t, Attr& a) {
  for (;;) {
    uint8_t ft = r.u8();
    if (ft == T_STOP) break;
    int16_t id = r.be16();
    bool used = true;
    switch (t) {
      case CRR_EV_WORKFLOW_EXECUTION_STARTED:
        if (id == 12 && ft == T_STRING) a.domain = r.str();                       // ParentWorkflowDomain
        else if (id == 40 && ft == T_I32) a.exec_s2c = r.be32();                  // ExecutionStartToCloseTimeoutSeconds
        else if (id == 50 && ft == T_I32) a.task_s2c = r.be32();                  // TaskStartToCloseTimeoutSeconds
        else if (id == 55 && ft == T_I32) a.initiator = r.be32();                 // Initiator
        else if (id == 80 && ft == T_I32) a.attempt = r.be32();                   // Attempt
        else if (id == 90 && ft == T_I64) a.expiration_ts = r.be64();             // ExpirationTimestamp
        else if (id == 110 && ft == T_I32) a.backoff = r.be32();                  // FirstDecisionTaskBackoffSeconds
        else if (id == 130 && ft == T_STRUCT) read_reset_points(r, a);            // PrevAutoResetPoints
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_SCHEDULED:
        if (id == 20 && ft == T_I32) a.aux = r.be32();                            // StartToCloseTimeoutSeconds
        else if (id == 30 && ft == T_I64) a.ref = r.be64();                       // Attempt
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_STARTED:
        if (id == 10 && ft == T_I64) a.ref = r.be64();                            // ScheduledEventId
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_COMPLETED:
        if (id == 30 && ft == T_I64) a.ref = r.be64();                            // StartedEventId
        else if (id == 50 && ft == T_STRING) { a.key = r.str(); a.has_key = true; }  // BinaryChecksum
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_TIMED_OUT:
        if (id == 30 && ft == T_I32) a.aux = r.be32();                            // TimeoutType
        else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_SCHEDULED:
        if (id == 10 && ft == T_STRING) { a.key = r.str(); a.has_key = true; }    // ActivityId
        else if (id == 25 && ft == T_STRING) a.domain = r.str();                  // Domain
        else if (id == 45 && ft == T_I32) a.s2c = r.be32();                       // ScheduleToCloseTimeoutSeconds
        else if (id == 50 && ft == T_I32) a.s2s = r.be32();                       // ScheduleToStartTimeoutSeconds
        else if (id == 55 && ft == T_I32) a.st2c = r.be32();                      // StartToCloseTimeoutSeconds
        else if (id == 60 && ft == T_I32) a.hb = r.be32();                        // HeartbeatTimeoutSeconds
        else if (id == 110 && ft == T_STRUCT) read_retry_policy(r, a);            // RetryPolicy
        else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_STARTED:    // ScheduledEventId: 10
      case CRR_EV_ACTIVITY_TASK_TIMED_OUT:  // 10
        if (id == 10 && ft == T_I64) a.ref = r.be64();
        else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_COMPLETED:  // 20
        if (id == 20 && ft == T_I64) a.ref = r.be64();
        else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_FAILED:     // 30
      case CRR_EV_ACTIVITY_TASK_CANCELED:   // 30
        if (id == 30 && ft == T_I64) a.ref = r.be64();
        else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED:
      case CRR_EV_TIMER_FIRED:
      case CRR_EV_TIMER_CANCELED:           // ActivityId / TimerId: 10
        if (id == 10 && ft == T_STRING) { a.key = r.str(); a.has_key = true; }
        else used = false;
        break;
      case CRR_EV_TIMER_STARTED:
        if (id == 10 && ft == T_STRING) { a.key = r.str(); a.has_key = true; }    // TimerId
        else if (id == 20 && ft == T_I64) a.ref = r.be64();                       // StartToFireTimeoutSeconds
        else used = false;
        break;
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED:                       // Domain: 10
        if (id == 10 && ft == T_STRING) a.domain = r.str();
        else used = false;
        break;
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED:
      case CRR_EV_SIGNAL_EXTERNAL_INITIATED:                                      // Domain: 20
        if (id == 20 && ft == T_STRING) a.domain = r.str();
        else used = false;
        break;
      // InitiatedEventId of the child / external-request follow-ups
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED:         // 60
        if (id == 60 && ft == T_I64) a.ref = r.be64();
        else used = false;
        break;
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED:        // 20
        if (id == 20 && ft == T_I64) a.ref = r.be64();
        else used = false;
        break;
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT:
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED:
      case CRR_EV_SIGNAL_EXTERNAL_FAILED:                  // 50
        if (id == 50 && ft == T_I64) a.ref = r.be64();
        else used = false;
        break;
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED:     // 40
        if (id == 40 && ft == T_I64) a.ref = r.be64();
        else used = false;
        break;
      case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED:
      case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED:    // 10
        if (id == 10 && ft == T_I64) a.ref = r.be64();
        else used = false;
        break;
      default:
        used = false;
    }
    if (!used) r.skip(ft);
  }
}

// HistoryEvent struct.  The attribute struct is read for the event's own type; a struct that
// arrives before field 30 (thriftrw writes ascending ids, so only in hand-made blobs) is re-read
// once the type is known.
void read_event(Reader& r, Event& e) {
  const uint8_t* attr_at = nullptr;
  int attr_t = -1;
  bool have_type = false;
  for (;;) {
    uint8_t ft = r.u8();
    if (ft == T_STOP) break;
    int16_t id = r.be16();
    if (id == 10 && ft == T_I64) e.id = r.be64();
    else if (id == 20 && ft == T_I64) e.ts = r.be64();
    else if (id == 30 && ft == T_I32) { e.type = r.be32(); have_type = true; }
    else if (id == 35 && ft == T_I64) e.ver = r.be64();
    else if (id == 36 && ft == T_I64) e.task = r.be64();
    else if (ft == T_STRUCT && attr_type_of_field(id) >= 0) {
      const int at = attr_type_of_field(id);
      if (have_type && at == e.type) {
        read_attributes(r, at, e.a);
      } else {
        if (!have_type) { attr_at = r.p; attr_t = at; }
        r.skip(ft);
      }
    } else {
      r.skip(ft);
    }
  }
  if (attr_at && attr_t == e.type) {
    Reader r2{attr_at, r.end};
    read_attributes(r2, attr_t, e.a);
  }
}

// tasks the task generator adds per event type (state_builder.go:157-625), an upper bound
constexpr int8_t kTasksPerEvent[CRR_EV_TYPE_COUNT] = {
    3, 2, 2, 2, 1, 1, 0, 1, 1, 1,   // 0 Started(+backoff) 1-3 closes 4 DTSched 5 DTStarted 6 DTCompleted 7-8 DT fail 9 ATSched
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0,   // 10-19
    0, 0, 2, 1, 0, 0, 0, 0, 2, 2,   // 22 Canceled 23 RCInitiated 28 Terminated 29 ContinuedAsNew
    1, 0, 0, 0, 0, 0, 0, 0, 1, 0,   // 30 StartChildInitiated 38 SignalInitiated
    0, 1};                          // 41 Upsert

// ---- per-chunk output --------------------------------------------------------------------------------
struct Chunk {
  std::vector<uint8_t> etype;
  std::vector<i64> id, ver, ts, task, ref;
  std::vector<u32> key;
  std::vector<i32> aux;
  std::vector<u32> key_off, key_len;
  std::string key_arena;
  std::vector<crr_activity_side> act;
  std::vector<crr_start_side> start;
  std::vector<u32> reset_keys;
  std::vector<uint8_t> arena;
  std::vector<crr_workflow> wf;
  int err = CRR_DECODE_OK;
  int64_t err_blob = -1;
};

struct Ctx {
  const uint8_t* const* blobs;
  const uint64_t* lens;
  uint32_t n_blobs;
  const crr_wf_source* wfs;
  const std::unordered_set<std::string>* known;  // null: every name resolves
};

int domain_status(const Ctx& c, const std::string& name) {
  if (name.empty()) return CRR_DOMAIN_NOT_SET;
  if (!c.known || c.known->count(name)) return CRR_DOMAIN_RESOLVED;
  return CRR_DOMAIN_UNKNOWN;
}

// NewHistoryBranchTokenByBranchID (dataManagerInterfaces.go:2899-2910): 0x59 + thrift binary
// HistoryBranch{10 TreeID string, 20 BranchID string, 30 Ancestors list<struct> = []}.
void branch_token(std::vector<uint8_t>& out, const char* tree, const char* branch) {
  auto be32 = [&](u32 v) { for (int s = 24; s >= 0; s -= 8) out.push_back((uint8_t)(v >> s)); };
  const size_t nt = tree ? strlen(tree) : 0, nb = branch ? strlen(branch) : 0;
  out.push_back(0x59);
  out.push_back(T_STRING); out.push_back(0); out.push_back(10); be32((u32)nt);
  out.insert(out.end(), tree, tree + nt);
  out.push_back(T_STRING); out.push_back(0); out.push_back(20); be32((u32)nb);
  out.insert(out.end(), branch, branch + nb);
  out.push_back(T_LIST); out.push_back(0); out.push_back(30); out.push_back(T_STRUCT); be32(0);
  out.push_back(T_STOP);
}

void decode_workflow(const Ctx& c, uint32_t w, Chunk& k) {
  const crr_wf_source& src = c.wfs[w];
  std::unordered_map<std::string, u32> intern;
  intern.emplace(std::string(), 0u);
  auto key_of = [&](const std::string& s) -> u32 {
    auto it = intern.find(s);
    if (it != intern.end()) return it->second;
    const u32 v = (u32)intern.size();
    intern.emplace(s, v);
    return v;
  };
  crr_workflow d;
  std::memset(&d, 0, sizeof(d));
  const i64 begin = (i64)k.etype.size();
  i32 empty_at = -1;
  i64 n_act = 0, n_timer = 0, n_child = 0, n_rc = 0, n_sig = 0, n_dtc = 0, n_started = 0, vh_items = 0;
  i64 max_prev = 0;
  i64 n_tasks = 0;  // upper bound of the tasks ApplyEvents generates (flatten.TASKS_PER_EVENT)
  bool have_ver = false;
  i64 last_ver = 0;
  Event e;
  for (uint32_t b = 0; b < src.blob_count; ++b) {
    const uint32_t bi = src.blob_begin + b;
    if (bi >= c.n_blobs) throw DecodeError{CRR_DECODE_BAD_ARGUMENT};
    k.err_blob = bi;
    const uint64_t len = c.lens[bi];
    i32 n_in_batch = 0;
    const i64 batch_begin = (i64)k.etype.size();
    if (len > 0) {
      Reader r{c.blobs[bi], c.blobs[bi] + len};
      if (r.u8() != 0x59) throw DecodeError{CRR_DECODE_BAD_PREAMBLE};  // version0Thriftrw.go:53-58
      // History{10 Events list<HistoryEvent>}
      for (;;) {
        uint8_t ft = r.u8();
        if (ft == T_STOP) break;
        int16_t id = r.be16();
        if (id != 10 || ft != T_LIST) { r.skip(ft); continue; }
        uint8_t et = r.u8();
        i32 n = r.be32();
        if (n < 0) throw DecodeError{CRR_DECODE_TRUNCATED};
        if (et != T_STRUCT && n > 0) throw DecodeError{CRR_DECODE_BAD_TYPE};
        for (i32 i = 0; i < n; ++i) {
          e = Event();
          read_event(r, e);
          const i32 t = e.type;
          const bool valid = t >= 0 && t < CRR_EV_TYPE_COUNT;
          k.etype.push_back((uint8_t)(valid ? t : CRR_EV_PAD - 1));
          k.id.push_back(e.id);
          k.ver.push_back(e.ver);
          k.ts.push_back(e.ts);
          k.task.push_back(e.task);
          if (!have_ver || e.ver > last_ver) { ++vh_items; last_ver = e.ver; have_ver = true; }
          n_tasks += valid ? kTasksPerEvent[t] : 0;
          i64 ref = 0;
          u32 key = 0;
          i32 aux = 0;
          const std::string* ks = nullptr;
          Attr& a = e.a;
          switch (valid ? t : -1) {
            case CRR_EV_WORKFLOW_EXECUTION_STARTED: {
              crr_start_side ss;
              std::memset(&ss, 0, sizeof(ss));
              if (a.prev_mode == -1) { ss.prev_reset_key_off = 0; ss.prev_reset_count = -1; }
              else if (a.prev_mode == -2) { ss.prev_reset_key_off = 0; ss.prev_reset_count = -2; }
              else {
                ss.prev_reset_key_off = (u32)k.reset_keys.size();
                ss.prev_reset_count = (i32)a.prev.size();
                for (const auto& p : a.prev) k.reset_keys.push_back(key_of(p));
                max_prev = std::max<i64>(max_prev, (i64)a.prev.size());
              }
              ss.decision_start_to_close = a.task_s2c;
              ss.workflow_timeout = a.exec_s2c;
              ss.first_decision_backoff = a.backoff;
              ss.initiator = a.initiator;
              ss.attempt = a.attempt;
              ss.expiration_ns = a.expiration_ts;
              // ParentWorkflowDomainID is not on the thrift wire: the name lookup (state_builder.go:137-147)
              ss.parent_domain_status = domain_status(c, a.domain);
              k.start.push_back(ss);
              aux = (i32)k.start.size() - 1;
              ++n_started;
              break;
            }
            case CRR_EV_DECISION_TASK_SCHEDULED: ref = a.ref; aux = a.aux; break;
            case CRR_EV_DECISION_TASK_STARTED: ref = a.ref; break;
            case CRR_EV_DECISION_TASK_COMPLETED: ref = a.ref; ks = &a.key; key = key_of(a.key); ++n_dtc; break;
            case CRR_EV_DECISION_TASK_TIMED_OUT: aux = a.aux; break;
            case CRR_EV_ACTIVITY_TASK_SCHEDULED: {
              ks = &a.key;
              key = key_of(a.key);
              crr_activity_side as;
              std::memset(&as, 0, sizeof(as));
              as.schedule_to_start = a.s2s; as.schedule_to_close = a.s2c; as.start_to_close = a.st2c;
              as.heartbeat = a.hb; as.has_retry_policy = a.has_retry; as.expiration_interval = a.expiration;
              as.domain_status = domain_status(c, a.domain);
              k.act.push_back(as);
              aux = (i32)k.act.size() - 1;
              ++n_act;
              break;
            }
            case CRR_EV_ACTIVITY_TASK_STARTED: case CRR_EV_ACTIVITY_TASK_COMPLETED: case CRR_EV_ACTIVITY_TASK_FAILED:
            case CRR_EV_ACTIVITY_TASK_TIMED_OUT: case CRR_EV_ACTIVITY_TASK_CANCELED:
              ref = a.ref; break;
            case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED: ks = &a.key; key = key_of(a.key); break;
            case CRR_EV_TIMER_STARTED: ks = &a.key; key = key_of(a.key); ref = a.ref; ++n_timer; break;
            case CRR_EV_TIMER_FIRED: case CRR_EV_TIMER_CANCELED: ks = &a.key; key = key_of(a.key); break;
            case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED: aux = domain_status(c, a.domain); ++n_child; break;
            case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED: aux = domain_status(c, a.domain); ++n_rc; break;
            case CRR_EV_SIGNAL_EXTERNAL_INITIATED: aux = domain_status(c, a.domain); ++n_sig; break;
            case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED:
            case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED:
            case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT:
            case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED: case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED:
            case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED: case CRR_EV_SIGNAL_EXTERNAL_FAILED:
            case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED:
              ref = a.ref; break;
            case CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW: aux = src.new_run_wf; break;
            default: break;
          }
          k.ref.push_back(ref);
          k.key.push_back(key);
          k.aux.push_back(aux);
          k.key_off.push_back((u32)k.key_arena.size());
          k.key_len.push_back(ks ? (u32)ks->size() : 0u);
          if (ks) k.key_arena.append(*ks);
          ++n_in_batch;
        }
      }
    }
    if (n_in_batch == 0) {  // an empty batch: ApplyEvents' history-size-zero error (state_builder.go:98-100)
      if (empty_at < 0) empty_at = (i32)(batch_begin - begin);
      continue;
    }
    n_tasks += 2;  // the batch's timer epilogue
    k.etype[batch_begin] |= CRR_ETYPE_BATCH_FIRST;
    k.etype.back() |= CRR_ETYPE_BATCH_LAST;
  }
  k.err_blob = -1;
  const i64 n = (i64)k.etype.size() - begin;
  if (src.blob_count == 0) empty_at = 0;
  d.ev_begin = begin;
  d.ev_count = (i32)n;
  d.empty_batch_at = empty_at;
  d.init_version = src.init_version;
  d.now_ns = src.now_ns;
  d.start_token_off = (u32)k.arena.size();
  branch_token(k.arena, src.run_id ? src.run_id : "", src.branch_id ? src.branch_id : "");
  d.start_token_len = (u32)(k.arena.size() - d.start_token_off);
  if (src.final_token) {
    d.final_token_off = (u32)k.arena.size();
    d.final_token_len = src.final_token_len;
    k.arena.insert(k.arena.end(), src.final_token, src.final_token + src.final_token_len);
    d.rebuild_last_event_id = src.rebuild_last_event_id;
    d.rebuild_last_event_version = src.rebuild_last_event_version;
  } else {
    d.final_token_off = 0;
    d.final_token_len = 0xFFFFFFFFu;
  }
  d.act_cap = (i32)n_act; d.timer_cap = (i32)n_timer; d.child_cap = (i32)n_child;
  d.rc_cap = (i32)n_rc; d.sig_cap = (i32)n_sig; d.vh_cap = (i32)vh_items;
  d.rp_cap = (i32)(max_prev * std::max<i64>(1, n_started) + n_dtc);
  d.flags = src.flags;
  d.task_cap = (i32)n_tasks;
  d.retention_days = src.retention_days;
  k.wf.push_back(d);
}

void decode_range(const Ctx& c, uint32_t w0, uint32_t w1, Chunk* k) {
  try {
    for (uint32_t w = w0; w < w1; ++w) decode_workflow(c, w, *k);
  } catch (const DecodeError& e) {
    k->err = e.code;
  } catch (...) {
    k->err = CRR_DECODE_BAD_ARGUMENT;
  }
}

template <class T>
void append(std::vector<T>& dst, const std::vector<T>& src) { dst.insert(dst.end(), src.begin(), src.end()); }

}  // namespace

struct crr_decoded {
  Chunk all;
  uint64_t table_rows[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};

extern "C" {

crr_decoded* crr_decode_histories(const uint8_t* const* blobs, const uint64_t* blob_lens, uint32_t n_blobs,
                                  const crr_wf_source* wfs, uint32_t n_wf, const char* const* known_domains,
                                  uint32_t n_known, int n_threads, int* err, int64_t* err_blob) {
  if (err) *err = CRR_DECODE_OK;
  if (err_blob) *err_blob = -1;
  if ((n_blobs && (!blobs || !blob_lens)) || (n_wf && !wfs)) {
    if (err) *err = CRR_DECODE_BAD_ARGUMENT;
    return nullptr;
  }
  std::unordered_set<std::string> known;
  const bool all_known = n_known == 0xFFFFFFFFu;
  if (!all_known)
    for (uint32_t i = 0; i < n_known; ++i) known.emplace(known_domains[i] ? known_domains[i] : "");
  Ctx c{blobs, blob_lens, n_blobs, wfs, all_known ? nullptr : &known};

  if (n_threads <= 0) n_threads = (int)std::max(1u, std::thread::hardware_concurrency());
  const uint32_t T = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)n_threads, (n_wf + 255) / 256));
  std::vector<Chunk> chunks(T);
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < T; ++t) {
    const uint32_t w0 = (uint32_t)((uint64_t)n_wf * t / T), w1 = (uint32_t)((uint64_t)n_wf * (t + 1) / T);
    if (T == 1) decode_range(c, w0, w1, &chunks[t]);
    else th.emplace_back(decode_range, std::cref(c), w0, w1, &chunks[t]);
  }
  for (auto& x : th) x.join();
  for (auto& k : chunks) {
    if (k.err != CRR_DECODE_OK) {
      if (err) *err = k.err;
      if (err_blob) *err_blob = k.err_blob;
      return nullptr;
    }
  }
  // concatenate with offset fix-ups (event indices, side-record indices, key / token / reset-key offsets)
  auto* out = new crr_decoded();
  Chunk& a = out->all;
  for (auto& k : chunks) {
    const i64 ev0 = (i64)a.etype.size();
    const i32 act0 = (i32)a.act.size(), st0 = (i32)a.start.size();
    const u32 rk0 = (u32)a.reset_keys.size(), ar0 = (u32)a.arena.size(), ka0 = (u32)a.key_arena.size();
    for (size_t i = 0; i < k.etype.size(); ++i) {
      const int t = k.etype[i] & CRR_ETYPE_MASK;
      if (t == CRR_EV_ACTIVITY_TASK_SCHEDULED) k.aux[i] += act0;
      else if (t == CRR_EV_WORKFLOW_EXECUTION_STARTED) k.aux[i] += st0;
      k.key_off[i] += ka0;
    }
    for (auto& s : k.start)
      if (s.prev_reset_count >= 0) s.prev_reset_key_off += rk0;
    for (auto& d : k.wf) {
      d.ev_begin += ev0;
      d.start_token_off += ar0;
      if (d.final_token_len != 0xFFFFFFFFu) d.final_token_off += ar0;
    }
    append(a.etype, k.etype); append(a.id, k.id); append(a.ver, k.ver); append(a.ts, k.ts);
    append(a.task, k.task); append(a.ref, k.ref); append(a.key, k.key); append(a.aux, k.aux);
    append(a.key_off, k.key_off); append(a.key_len, k.key_len); a.key_arena += k.key_arena;
    append(a.act, k.act); append(a.start, k.start); append(a.reset_keys, k.reset_keys);
    append(a.arena, k.arena); append(a.wf, k.wf);
    Chunk().etype.swap(k.etype);  // release chunk memory early
  }
  // canonical slot-table bases: prefix sums of the per-workflow capacities
  int64_t base[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (auto& d : a.wf) {
    const i32 caps[8] = {d.act_cap, d.timer_cap, d.child_cap, d.rc_cap, d.sig_cap, d.vh_cap, d.rp_cap, d.task_cap};
    int64_t* bases[8] = {&d.act_base, &d.timer_base, &d.child_base, &d.rc_base, &d.sig_base, &d.vh_base, &d.rp_base,
                         &d.task_base};
    for (int j = 0; j < 8; ++j) {
      *bases[j] = base[j];
      base[j] += std::max(caps[j], 0);
    }
  }
  for (int j = 0; j < 8; ++j) out->table_rows[j] = (uint64_t)base[j];
  return out;
}

int crr_decoded_get_view(const crr_decoded* d, crr_decoded_view* v) {
  if (!d || !v) return CRR_DECODE_BAD_ARGUMENT;
  const Chunk& a = d->all;
  v->ev.etype = a.etype.data();
  v->ev.event_id = a.id.data();
  v->ev.version = a.ver.data();
  v->ev.timestamp = a.ts.data();
  v->ev.task_id = a.task.data();
  v->ev.ref = a.ref.data();
  v->ev.key = a.key.data();
  v->ev.aux = a.aux.data();
  v->n_events = a.etype.size();
  v->act_side = a.act.data(); v->n_act_side = a.act.size();
  v->start_side = a.start.data(); v->n_start_side = a.start.size();
  v->reset_keys = a.reset_keys.data(); v->n_reset_keys = a.reset_keys.size();
  v->arena = a.arena.data(); v->n_arena = a.arena.size();
  v->wf = a.wf.data(); v->n_wf = (uint32_t)a.wf.size();
  for (int j = 0; j < 8; ++j) v->table_rows[j] = d->table_rows[j];
  v->key_off = a.key_off.data();
  v->key_len = a.key_len.data();
  v->key_arena = a.key_arena.data();
  v->n_key_arena = a.key_arena.size();
  return CRR_DECODE_OK;
}

void crr_decoded_free(crr_decoded* d) { delete d; }

}  // extern "C"
