// blob_encode.cpp -- synthetic persisted histories: a canonical flattened batch -> thriftrw blobs
// (benchmark and test infrastructure of libcadence_host.so, not part of the replay boundary).
//
// Restates cadence_amd/thrift_codec.py (serializer.SerializeBatchEvents, common/persistence/
// serializer.go:105-107: the 0x59 preamble, then shared.History{10: list<HistoryEvent>} in thrift
// binary, each struct's set fields in ascending id order as go.uber.org/thriftrw writes them) over the
// engine's columns, natively and threaded, so the full-size workloads (1M+ workflows) can be persisted
// for the blob -> rows benchmark.  The fields ApplyEvents never reads are written too (identities,
// task lists, inputs, retry policies, headers), so blobs are realistically sized and the decoders'
// skipping is exercised.  Decoding the output (crr_decode_histories, or crr_ingest_* on the device)
// gives back the input batch: strings are the per-event key strings; domain outcomes become names the
// domain cache {domain-a, domain-b, parent-domain} resolves (or not); a reset point whose binary
// checksum no event carries is named "rk-<key>".
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "cadence_decode.h"
#include "cadence_ingest.h"

namespace {

using i64 = int64_t;
using i32 = int32_t;
using u32 = uint32_t;
using u64 = uint64_t;

enum : uint8_t { T_BOOL = 2, T_DOUBLE = 4, T_I32 = 8, T_I64 = 10, T_STRING = 11, T_STRUCT = 12, T_MAP = 13, T_LIST = 15 };

struct W {
  std::string& b;
  void u8(uint8_t v) { b.push_back((char)v); }
  void be16(u32 v) { u8(v >> 8); u8(v); }
  void be32(u32 v) { u8(v >> 24); u8(v >> 16); u8(v >> 8); u8(v); }
  void be64(u64 v) { be32((u32)(v >> 32)); be32((u32)v); }
  void field(uint8_t t, u32 id) { u8(t); be16(id); }
  void i32f(u32 id, i32 v) { field(T_I32, id); be32((u32)v); }
  void i64f(u32 id, i64 v) { field(T_I64, id); be64((u64)v); }
  void str(u32 id, const char* s, size_t n) { field(T_STRING, id); be32((u32)n); b.append(s, n); }
  void str(u32 id, const std::string& s) { str(id, s.data(), s.size()); }
  void begin(u32 id) { field(T_STRUCT, id); }
  void stop() { u8(0); }
  void name_struct(u32 id, const char* name) { begin(id); str(10, name, strlen(name)); stop(); }       // WorkflowType / ActivityType
  void task_list(u32 id, const char* name) { begin(id); str(10, name, strlen(name)); i32f(20, 0); stop(); }
};

struct Inputs {
  const uint8_t* etype;
  const i64 *id, *ver, *ts, *task, *ref;
  const u32* key;
  const i32* aux;
  const crr_activity_side* act;
  const crr_start_side* start;
  const u32* reset_keys;
  const uint8_t* arena;
  const crr_workflow* wf;
  const u32 *key_off, *key_len;
  const char* key_arena;
};

struct Out {
  std::string bytes;
  std::vector<u64> blob_len;
  std::vector<crr_blob_wf> wf;
  std::string strings;
};

const char* domain_name(i32 status, bool parent) {
  if (status == CRR_DOMAIN_RESOLVED) return parent ? "parent-domain" : "domain-a";
  if (status == CRR_DOMAIN_UNKNOWN) return "unknown-domain";
  return nullptr;
}

void request_id(char out[36], u64 a, u64 b) {   // a deterministic 36-character request ID
  static const char hex[] = "0123456789abcdef";
  u64 x = a * 0x9E3779B97F4A7C15ull ^ b;
  for (int i = 0; i < 36; ++i) {
    if (i == 8 || i == 13 || i == 18 || i == 23) { out[i] = '-'; continue; }
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    out[i] = hex[(x >> 59) & 15];
  }
}

// one event (thrift_codec.encode_event / attribute_fields)
void encode_event(W& w, const Inputs& in, i64 x, u64 wf_no, const std::unordered_map<u32, std::string>& keystr) {
  const int t = in.etype[x] & CRR_ETYPE_MASK;
  const bool valid = t < CRR_EV_TYPE_COUNT;
  w.i64f(10, in.id[x]);
  w.i64f(20, in.ts[x]);
  w.i32f(30, valid ? t : 99);
  w.i64f(35, in.ver[x]);
  w.i64f(36, in.task[x]);
  if (!valid) { w.stop(); return; }
  auto key = [&]() -> std::string {
    const u32 n = in.key_len ? in.key_len[x] : 0;
    if (n) return std::string(in.key_arena + in.key_off[x], n);
    auto it = keystr.find(in.key[x]);
    return it == keystr.end() ? std::string() : it->second;
  };
  const i64 ref = in.ref[x];
  const i32 aux = in.aux[x];
  char rid[36];
  w.begin(40 + 10 * t);
  switch (t) {
    case CRR_EV_WORKFLOW_EXECUTION_STARTED: {
      const crr_start_side& s = in.start[aux];
      w.name_struct(10, "workflow-type");
      if (const char* d = domain_name(s.parent_domain_status, true)) w.str(12, d, strlen(d));
      w.task_list(20, "task-list");
      w.str(30, "input-bytes", 11);
      w.i32f(40, s.workflow_timeout);
      w.i32f(50, s.decision_start_to_close);
      if (s.initiator != CRR_INITIATOR_NIL) w.i32f(55, s.initiator);
      w.str(60, "identity", 8);
      w.i32f(80, s.attempt);
      if (s.expiration_ns) w.i64f(90, s.expiration_ns);
      w.i32f(110, s.first_decision_backoff);
      if (s.prev_reset_count == -2) {
        w.begin(130); w.stop();
      } else if (s.prev_reset_count >= 0) {
        w.begin(130);
        w.field(T_LIST, 10);
        w.u8(T_STRUCT);
        w.be32((u32)s.prev_reset_count);
        for (i32 i = 0; i < s.prev_reset_count; ++i) {
          const u32 k = in.reset_keys[s.prev_reset_key_off + i];
          auto it = keystr.find(k);
          const std::string bc = k == 0 ? std::string() : (it != keystr.end() ? it->second : "rk-" + std::to_string(k));
          w.str(10, bc);
          const std::string pr = "prev-run-" + std::to_string(i);
          w.str(20, pr);
          w.i64f(30, 4 + i);
          w.i64f(40, 1500000000000000000LL + i);
          w.field(T_BOOL, 60); w.u8(1);
          w.stop();
        }
        w.stop();
      }
      break;
    }
    case CRR_EV_DECISION_TASK_SCHEDULED:
      w.task_list(10, "decision-tl"); w.i32f(20, aux); w.i64f(30, ref);
      break;
    case CRR_EV_DECISION_TASK_STARTED:
      request_id(rid, wf_no, (u64)in.id[x]);
      w.i64f(10, ref); w.str(20, "worker-identity", 15); w.str(30, rid, 36);
      break;
    case CRR_EV_DECISION_TASK_COMPLETED: {
      w.str(10, "ctx", 3); w.i64f(20, ref - 1); w.i64f(30, ref); w.str(40, "worker-identity", 15);
      const std::string k = key();
      if (!k.empty()) w.str(50, k);
      break;
    }
    case CRR_EV_DECISION_TASK_TIMED_OUT:
      w.i64f(10, 0); w.i64f(20, 0); w.i32f(30, aux);
      break;
    case CRR_EV_ACTIVITY_TASK_SCHEDULED: {
      const crr_activity_side& a = in.act[aux];
      w.str(10, key());
      w.name_struct(20, "activity-type");
      if (const char* d = domain_name(a.domain_status, false)) w.str(25, d, strlen(d));
      w.task_list(30, "activity-tl");
      w.str(40, "activity-input", 14);
      w.i32f(45, a.schedule_to_close); w.i32f(50, a.schedule_to_start); w.i32f(55, a.start_to_close);
      w.i32f(60, a.heartbeat); w.i64f(90, 4);
      if (a.has_retry_policy) {
        w.begin(110);
        w.i32f(10, 1);
        w.field(T_DOUBLE, 20); w.be64(0x4000000000000000ull);   // 2.0
        w.i32f(30, 100); w.i32f(40, 5);
        w.field(T_LIST, 50); w.u8(T_STRING); w.be32(1); w.be32(9); w.b.append("bad-input");
        w.i32f(60, a.expiration_interval);
        w.stop();
      }
      break;
    }
    case CRR_EV_ACTIVITY_TASK_STARTED:
      request_id(rid, wf_no, (u64)in.id[x]);
      w.i64f(10, ref); w.str(20, "worker", 6); w.str(30, rid, 36); w.i32f(40, 0);
      break;
    case CRR_EV_ACTIVITY_TASK_TIMED_OUT: w.i64f(10, ref); break;
    case CRR_EV_ACTIVITY_TASK_COMPLETED: w.i64f(20, ref); break;
    case CRR_EV_ACTIVITY_TASK_FAILED: case CRR_EV_ACTIVITY_TASK_CANCELED: w.i64f(30, ref); break;
    case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED: w.str(10, key()); w.i64f(20, 4); break;
    case CRR_EV_TIMER_STARTED: w.str(10, key()); w.i64f(20, ref); w.i64f(30, 4); break;
    case CRR_EV_TIMER_FIRED: case CRR_EV_TIMER_CANCELED: w.str(10, key()); w.i64f(20, 5); break;
    case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED:
      if (const char* d = domain_name(aux, false)) w.str(10, d, strlen(d));
      w.str(20, "child-wf", 8); w.name_struct(30, "child-type"); w.task_list(40, "child-tl"); w.i32f(81, 1);
      break;
    case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED:
    case CRR_EV_SIGNAL_EXTERNAL_INITIATED:
      w.i64f(10, 4);
      if (const char* d = domain_name(aux, false)) w.str(20, d, strlen(d));
      w.begin(30); w.str(10, "target-wf", 9); w.str(20, "target-run", 10); w.stop();
      if (t == CRR_EV_SIGNAL_EXTERNAL_INITIATED) { w.str(40, "sig", 3); w.str(50, "signal-input", 12); }
      break;
    case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED: w.i64f(60, ref); break;
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED: w.i64f(20, ref); break;
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED:
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT: case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED:
    case CRR_EV_SIGNAL_EXTERNAL_FAILED:
      w.i64f(50, ref); break;
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED: w.i64f(40, ref); break;
    case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED: case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED:
      w.i64f(10, ref); break;
    case CRR_EV_WORKFLOW_EXECUTION_SIGNALED:
      w.str(10, "signal", 6); w.str(20, "payload", 7); w.str(30, "identity", 8);
      break;
    case CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW:
      w.str(10, "new-run", 7); w.name_struct(20, "workflow-type");
      break;
    case CRR_EV_UPSERT_WORKFLOW_SEARCH_ATTRIBUTES:
      w.i64f(10, 4);
      w.begin(20);
      w.field(T_MAP, 10); w.u8(T_STRING); w.u8(T_STRING); w.be32(1);
      w.be32(18); w.b.append("CustomKeywordField"); w.be32(3); w.b.append("\"v\"");
      w.stop();
      break;
    case CRR_EV_MARKER_RECORDED:
      w.str(10, "marker", 6); w.str(20, "details", 7);
      break;
    default:
      break;
  }
  w.stop();   // the attribute struct
  w.stop();   // the event
}


// ---- the same events as types JSON (json.Marshal of []*types.HistoryEvent, serializer.go:321-325) ---------
const char* const kEventTypeNames[CRR_EV_TYPE_COUNT] = {
    "WorkflowExecutionStarted", "WorkflowExecutionCompleted", "WorkflowExecutionFailed", "WorkflowExecutionTimedOut",
    "DecisionTaskScheduled", "DecisionTaskStarted", "DecisionTaskCompleted", "DecisionTaskTimedOut",
    "DecisionTaskFailed", "ActivityTaskScheduled", "ActivityTaskStarted", "ActivityTaskCompleted",
    "ActivityTaskFailed", "ActivityTaskTimedOut", "ActivityTaskCancelRequested", "RequestCancelActivityTaskFailed",
    "ActivityTaskCanceled", "TimerStarted", "TimerFired", "CancelTimerFailed", "TimerCanceled",
    "WorkflowExecutionCancelRequested", "WorkflowExecutionCanceled", "RequestCancelExternalWorkflowExecutionInitiated",
    "RequestCancelExternalWorkflowExecutionFailed", "ExternalWorkflowExecutionCancelRequested", "MarkerRecorded",
    "WorkflowExecutionSignaled", "WorkflowExecutionTerminated", "WorkflowExecutionContinuedAsNew",
    "StartChildWorkflowExecutionInitiated", "StartChildWorkflowExecutionFailed", "ChildWorkflowExecutionStarted",
    "ChildWorkflowExecutionCompleted", "ChildWorkflowExecutionFailed", "ChildWorkflowExecutionCanceled",
    "ChildWorkflowExecutionTimedOut", "ChildWorkflowExecutionTerminated", "SignalExternalWorkflowExecutionInitiated",
    "SignalExternalWorkflowExecutionFailed", "ExternalWorkflowExecutionSignaled", "UpsertWorkflowSearchAttributes"};
const char* const kTimeoutTypeNames[4] = {"START_TO_CLOSE", "SCHEDULE_TO_START", "SCHEDULE_TO_CLOSE", "HEARTBEAT"};
const char* const kInitiatorNames[3] = {"DECIDER", "RETRYPOLICY", "CRONSCHEDULE"};

struct J {   // a JSON object writer: keys in the order written
  std::string& b;
  bool first = true;
  void key(const char* k) {
    if (!first) b.push_back(',');
    first = false;
    b.push_back('"'); b.append(k); b.append("\":");
  }
  void quoted(const std::string& s) {
    b.push_back('"');
    for (char c : s) {
      if (c == '"' || c == '\\') { b.push_back('\\'); b.push_back(c); }
      else if ((unsigned char)c < 0x20) { char u[8]; snprintf(u, sizeof u, "\\u%04x", (unsigned)(unsigned char)c); b.append(u); }
      else b.push_back(c);
    }
    b.push_back('"');
  }
  void i64v(const char* k, i64 v) { key(k); b.append(std::to_string(v)); }
  void strv(const char* k, const std::string& s) { key(k); quoted(s); }
  void open(const char* k) { key(k); b.push_back('{'); first = true; }
  void close() { b.push_back('}'); first = false; }
  void name_obj(const char* k, const char* name) { open(k); strv("name", name); close(); }
  void task_list(const char* k, const char* name) { open(k); strv("name", name); strv("kind", "NORMAL"); close(); }
};

std::string enum_text(const char* const* names, int n, i32 v) {
  return v >= 0 && v < n ? std::string(names[v]) : std::to_string(v);
}

// one event (encode_event's fields, as common/types JSON tags)
void encode_event_json(std::string& b, const Inputs& in, i64 x, u64 wf_no,
                       const std::unordered_map<u32, std::string>& keystr) {
  const int t = in.etype[x] & CRR_ETYPE_MASK;
  const bool valid = t < CRR_EV_TYPE_COUNT;
  J j{b};
  b.push_back('{');
  j.i64v("eventId", in.id[x]);
  j.i64v("timestamp", in.ts[x]);
  j.key("eventType");
  j.quoted(valid ? std::string(kEventTypeNames[t]) : std::string("99"));
  j.i64v("version", in.ver[x]);
  j.i64v("taskId", in.task[x]);
  if (!valid) { b.push_back('}'); return; }
  auto key = [&]() -> std::string {
    const u32 n = in.key_len ? in.key_len[x] : 0;
    if (n) return std::string(in.key_arena + in.key_off[x], n);
    auto it = keystr.find(in.key[x]);
    return it == keystr.end() ? std::string() : it->second;
  };
  const i64 ref = in.ref[x];
  const i32 aux = in.aux[x];
  char rid[37];
  rid[36] = 0;
  std::string ak(kEventTypeNames[t]);
  ak[0] = (char)(ak[0] - 'A' + 'a');
  ak += "EventAttributes";
  j.open(ak.c_str());
  switch (t) {
    case CRR_EV_WORKFLOW_EXECUTION_STARTED: {
      const crr_start_side& s = in.start[aux];
      j.name_obj("workflowType", "workflow-type");
      if (const char* d = domain_name(s.parent_domain_status, true)) j.strv("parentWorkflowDomain", d);
      j.task_list("taskList", "task-list");
      j.strv("input", "aW5wdXQtYnl0ZXM=");
      j.i64v("executionStartToCloseTimeoutSeconds", s.workflow_timeout);
      j.i64v("taskStartToCloseTimeoutSeconds", s.decision_start_to_close);
      if (s.initiator != CRR_INITIATOR_NIL) { j.key("initiator"); j.quoted(enum_text(kInitiatorNames, 3, s.initiator)); }
      j.strv("identity", "identity");
      j.i64v("attempt", s.attempt);
      if (s.expiration_ns) j.i64v("expirationTimestamp", s.expiration_ns);
      j.i64v("firstDecisionTaskBackoffSeconds", s.first_decision_backoff);
      if (s.prev_reset_count == -2) {
        j.open("prevAutoResetPoints"); j.close();
      } else if (s.prev_reset_count >= 0) {
        j.open("prevAutoResetPoints");
        j.key("points");
        b.push_back('[');
        for (i32 i = 0; i < s.prev_reset_count; ++i) {
          const u32 k = in.reset_keys[s.prev_reset_key_off + i];
          auto it = keystr.find(k);
          const std::string bc = k == 0 ? std::string() : (it != keystr.end() ? it->second : "rk-" + std::to_string(k));
          if (i) b.push_back(',');
          J p{b};
          b.push_back('{');
          p.strv("binaryChecksum", bc);
          p.strv("runId", "prev-run-" + std::to_string(i));
          p.i64v("firstDecisionCompletedId", 4 + i);
          p.i64v("createdTimeNano", 1500000000000000000LL + i);
          p.key("resettable"); b.append("true");
          b.push_back('}');
        }
        b.push_back(']');
        j.close();
      }
      break;
    }
    case CRR_EV_DECISION_TASK_SCHEDULED:
      j.task_list("taskList", "decision-tl"); j.i64v("startToCloseTimeoutSeconds", aux); j.i64v("attempt", ref);
      break;
    case CRR_EV_DECISION_TASK_STARTED:
      request_id(rid, wf_no, (u64)in.id[x]);
      j.i64v("scheduledEventId", ref); j.strv("identity", "worker-identity"); j.strv("requestId", rid);
      break;
    case CRR_EV_DECISION_TASK_COMPLETED: {
      j.strv("executionContext", "Y3R4"); j.i64v("scheduledEventId", ref - 1); j.i64v("startedEventId", ref);
      j.strv("identity", "worker-identity");
      const std::string k = key();
      if (!k.empty()) j.strv("binaryChecksum", k);
      break;
    }
    case CRR_EV_DECISION_TASK_TIMED_OUT:
      j.i64v("scheduledEventId", 0); j.i64v("startedEventId", 0);
      j.key("timeoutType"); j.quoted(enum_text(kTimeoutTypeNames, 4, aux));
      break;
    case CRR_EV_ACTIVITY_TASK_SCHEDULED: {
      const crr_activity_side& a = in.act[aux];
      j.strv("activityId", key());
      j.name_obj("activityType", "activity-type");
      if (const char* d = domain_name(a.domain_status, false)) j.strv("domain", d);
      j.task_list("taskList", "activity-tl");
      j.strv("input", "YWN0aXZpdHktaW5wdXQ=");
      j.i64v("scheduleToCloseTimeoutSeconds", a.schedule_to_close);
      j.i64v("scheduleToStartTimeoutSeconds", a.schedule_to_start);
      j.i64v("startToCloseTimeoutSeconds", a.start_to_close);
      j.i64v("heartbeatTimeoutSeconds", a.heartbeat);
      j.i64v("decisionTaskCompletedEventId", 4);
      if (a.has_retry_policy) {
        j.open("retryPolicy");
        j.i64v("initialIntervalInSeconds", 1);
        j.key("backoffCoefficient"); b.append("2");
        j.i64v("maximumIntervalInSeconds", 100);
        j.i64v("maximumAttempts", 5);
        j.key("nonRetriableErrorReasons"); b.append("[\"bad-input\"]");
        j.i64v("expirationIntervalInSeconds", a.expiration_interval);
        j.close();
      }
      break;
    }
    case CRR_EV_ACTIVITY_TASK_STARTED:
      request_id(rid, wf_no, (u64)in.id[x]);
      j.i64v("scheduledEventId", ref); j.strv("identity", "worker"); j.strv("requestId", rid); j.i64v("attempt", 0);
      break;
    case CRR_EV_ACTIVITY_TASK_TIMED_OUT: case CRR_EV_ACTIVITY_TASK_COMPLETED: case CRR_EV_ACTIVITY_TASK_FAILED:
    case CRR_EV_ACTIVITY_TASK_CANCELED:
      j.i64v("scheduledEventId", ref);
      break;
    case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED: j.strv("activityId", key()); j.i64v("decisionTaskCompletedEventId", 4); break;
    case CRR_EV_TIMER_STARTED:
      j.strv("timerId", key()); j.i64v("startToFireTimeoutSeconds", ref); j.i64v("decisionTaskCompletedEventId", 4);
      break;
    case CRR_EV_TIMER_FIRED: case CRR_EV_TIMER_CANCELED: j.strv("timerId", key()); j.i64v("startedEventId", 5); break;
    case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED:
      if (const char* d = domain_name(aux, false)) j.strv("domain", d);
      j.strv("workflowId", "child-wf"); j.name_obj("workflowType", "child-type"); j.task_list("taskList", "child-tl");
      break;
    case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED:
    case CRR_EV_SIGNAL_EXTERNAL_INITIATED:
      j.i64v("decisionTaskCompletedEventId", 4);
      if (const char* d = domain_name(aux, false)) j.strv("domain", d);
      j.open("workflowExecution"); j.strv("workflowId", "target-wf"); j.strv("runId", "target-run"); j.close();
      if (t == CRR_EV_SIGNAL_EXTERNAL_INITIATED) { j.strv("signalName", "sig"); j.strv("input", "c2lnbmFsLWlucHV0"); }
      break;
    case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED:
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED:
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT:
    case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED: case CRR_EV_SIGNAL_EXTERNAL_FAILED:
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED: case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED:
    case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED:
      j.i64v("initiatedEventId", ref);
      break;
    case CRR_EV_WORKFLOW_EXECUTION_SIGNALED:
      j.strv("signalName", "signal"); j.strv("input", "cGF5bG9hZA=="); j.strv("identity", "identity");
      break;
    case CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW:
      j.strv("newExecutionRunId", "new-run"); j.name_obj("workflowType", "workflow-type");
      break;
    case CRR_EV_UPSERT_WORKFLOW_SEARCH_ATTRIBUTES:
      j.i64v("decisionTaskCompletedEventId", 4);
      j.open("searchAttributes"); j.key("indexedFields"); b.append("{\"CustomKeywordField\":\"InYi\"}"); j.close();
      break;
    case CRR_EV_MARKER_RECORDED:
      j.strv("markerName", "marker"); j.strv("details", "ZGV0YWlscw==");
      break;
    default:
      break;
  }
  j.close();
  b.push_back('}');
}

void encode_range(const Inputs& in, u32 w0, u32 w1, Out* o, bool json) {
  std::unordered_map<u32, std::string> keystr;
  for (u32 wi = w0; wi < w1; ++wi) {
    const crr_workflow& d = in.wf[wi];
    // key id -> string (the events' keys)
    keystr.clear();
    if (in.key_len)
      for (i32 k = 0; k < d.ev_count; ++k) {
        const i64 x = d.ev_begin + k;
        if (in.key_len[x]) keystr.emplace(in.key[x], std::string(in.key_arena + in.key_off[x], in.key_len[x]));
      }
    crr_blob_wf s;
    std::memset(&s, 0, sizeof(s));
    s.blob_begin = (u32)o->blob_len.size();   // chunk-local; fixed up on concatenation
    s.init_version = d.init_version;
    s.now_ns = d.now_ns;
    // run / branch IDs out of the start token (NewHistoryBranchTokenByBranchID's layout)
    const uint8_t* tok = in.arena + d.start_token_off;
    auto be32 = [](const uint8_t* p) { return ((u32)p[0] << 24) | ((u32)p[1] << 16) | ((u32)p[2] << 8) | p[3]; };
    const u32 nt = be32(tok + 4);
    const u32 nb = be32(tok + 8 + nt + 3);
    s.run_id_off = (u32)o->strings.size();
    s.run_id_len = nt;
    o->strings.append((const char*)tok + 8, nt);
    s.branch_id_off = (u32)o->strings.size();
    s.branch_id_len = nb;
    o->strings.append((const char*)tok + 8 + nt + 7, nb);
    if (d.final_token_len != 0xFFFFFFFFu) {
      s.final_token_off = (u32)o->strings.size();
      s.final_token_len = d.final_token_len;
      o->strings.append((const char*)in.arena + d.final_token_off, d.final_token_len);
      s.rebuild_last_event_id = d.rebuild_last_event_id;
      s.rebuild_last_event_version = d.rebuild_last_event_version;
    } else {
      s.final_token_len = 0xFFFFFFFFu;
    }
    s.new_run_wf = -1;
    s.flags = d.flags & (CRR_WF_FLAG_NEW_RUN | CRR_WF_FLAG_REFRESH_TASKS);
    s.retention_days = d.retention_days;
    // batches: BATCH_FIRST .. BATCH_LAST runs; the empty batch (if any) before step empty_batch_at
    u32 blobs = 0;
    i32 k = 0;
    auto empty_blob = [&]() { o->blob_len.push_back(0); ++blobs; };
    while (k < d.ev_count) {
      if (k == d.empty_batch_at) empty_blob();
      const size_t at = o->bytes.size();
      // count this batch's events
      i32 e = k;
      while (e < d.ev_count) {
        const bool last = in.etype[d.ev_begin + e] & CRR_ETYPE_BATCH_LAST;
        ++e;
        if (last) break;
      }
      W w{o->bytes};
      if (json) {
        o->bytes.push_back('[');
      } else {
        w.u8(0x59);
        w.field(T_LIST, 10);
        w.u8(T_STRUCT);
        w.be32((u32)(e - k));
      }
      for (i32 j = k; j < e; ++j) {
        const i64 x = d.ev_begin + j;
        if ((in.etype[x] & CRR_ETYPE_MASK) == CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW) s.new_run_wf = in.aux[x];
        if (json) {
          if (j > k) o->bytes.push_back(',');
          encode_event_json(o->bytes, in, x, wi, keystr);
        } else {
          encode_event(w, in, x, wi, keystr);
        }
      }
      if (json) o->bytes.push_back(']');
      else w.stop();
      o->blob_len.push_back(o->bytes.size() - at);
      ++blobs;
      k = e;
    }
    if (d.empty_batch_at >= 0 && d.empty_batch_at >= d.ev_count && d.ev_count > 0) empty_blob();
    s.blob_count = blobs;
    o->wf.push_back(s);
  }
}

}  // namespace

struct crr_encoded {
  std::vector<uint8_t> bytes;
  std::vector<u64> blob_off;
  std::vector<crr_blob_wf> wf;
  std::vector<uint8_t> strings;
};

extern "C" {

/* Encode a canonical batch (stride 1; host arrays as crr_inputs describes them, plus the per-event key
 * strings: key_off / key_len into key_arena, NULL if absent) into persisted blobs: thriftrw, or with json != 0
 * common/types JSON arrays of the same events (serializer.go:321-325's json encoding). */
crr_encoded* crr_encode_blobs_as(const crr_inputs* in, const uint32_t* key_off, const uint32_t* key_len,
                                 const char* key_arena, int n_threads, int json) {
  if (!in || in->stride != 1) return nullptr;
  Inputs I;
  I.etype = in->ev.etype; I.id = in->ev.event_id; I.ver = in->ev.version; I.ts = in->ev.timestamp;
  I.task = in->ev.task_id; I.ref = in->ev.ref; I.key = in->ev.key; I.aux = in->ev.aux;
  I.act = in->act_side; I.start = in->start_side; I.reset_keys = in->reset_keys; I.arena = in->arena; I.wf = in->wf;
  I.key_off = key_off; I.key_len = key_len; I.key_arena = key_arena;
  const u32 n = in->n_wf;
  if (n_threads <= 0) n_threads = (int)std::max(1u, std::thread::hardware_concurrency());
  const u32 T = std::max<u32>(1, std::min<u32>((u32)n_threads * 4, (n + 1023) / 1024));
  std::vector<Out> outs(T);
  std::vector<std::thread> th;
  for (u32 t = 0; t < T; ++t) {
    const u32 a = (u32)((u64)n * t / T), b = (u32)((u64)n * (t + 1) / T);
    th.emplace_back(encode_range, std::cref(I), a, b, &outs[t], json != 0);
    if (th.size() >= (size_t)n_threads) {
      for (auto& x : th) x.join();
      th.clear();
    }
  }
  for (auto& x : th) x.join();
  auto* r = new crr_encoded();
  size_t nbytes = 0, nblobs = 0, nstr = 0;
  for (auto& o : outs) { nbytes += o.bytes.size(); nblobs += o.blob_len.size(); nstr += o.strings.size(); }
  r->bytes.reserve(nbytes + 32);
  r->blob_off.reserve(nblobs + 1);
  r->wf.reserve(n);
  r->strings.reserve(nstr + 1);
  r->blob_off.push_back(0);
  for (auto& o : outs) {
    const u32 b0 = (u32)(r->blob_off.size() - 1);
    const u32 s0 = (u32)r->strings.size();
    for (u64 len : o.blob_len) r->blob_off.push_back(r->blob_off.back() + len);
    r->bytes.insert(r->bytes.end(), o.bytes.begin(), o.bytes.end());
    for (crr_blob_wf s : o.wf) {
      s.blob_begin += b0;
      s.run_id_off += s0;
      s.branch_id_off += s0;
      if (s.final_token_len != 0xFFFFFFFFu) s.final_token_off += s0;
      r->wf.push_back(s);
    }
    r->strings.insert(r->strings.end(), o.strings.begin(), o.strings.end());
    o = Out();
  }
  r->bytes.resize(r->bytes.size() + CRR_INGEST_PAD, 0);   // the device parser's window reads past the end
  if (r->strings.empty()) r->strings.push_back(0);
  return r;
}

/* crr_encode_blobs_as with thriftrw blobs. */
crr_encoded* crr_encode_blobs(const crr_inputs* in, const uint32_t* key_off, const uint32_t* key_len,
                              const char* key_arena, int n_threads) {
  return crr_encode_blobs_as(in, key_off, key_len, key_arena, n_threads, 0);
}

void crr_encoded_view(const crr_encoded* e, const uint8_t** bytes, uint64_t* n_bytes, const uint64_t** blob_off,
                      uint32_t* n_blobs, const crr_blob_wf** wf, uint32_t* n_wf, const uint8_t** strings,
                      uint64_t* n_strings) {
  *bytes = e->bytes.data();
  *n_bytes = e->bytes.size() - 32;
  *blob_off = e->blob_off.data();
  *n_blobs = (uint32_t)(e->blob_off.size() - 1);
  *wf = e->wf.data();
  *n_wf = (uint32_t)e->wf.size();
  *strings = e->strings.data();
  *n_strings = e->strings.size();
}

void crr_encoded_free(crr_encoded* e) { delete e; }

}  // extern "C"
