// json_decode.cpp -- JSON-encoded history batches (json.Unmarshal into []*types.HistoryEvent,
// common/persistence/serializer.go:324-325) -> the Events the flattener consumes; see json_decode.h.
#include "json_decode.h"

namespace crr_host {
namespace {

// types.EventType names in enum order (common/types/shared.go EventType, UnmarshalText: case-insensitive)
const char* const kEventTypes[CRR_EV_TYPE_COUNT] = {
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
const char* const kTimeoutTypes[] = {"START_TO_CLOSE", "SCHEDULE_TO_START", "SCHEDULE_TO_CLOSE", "HEARTBEAT"};
const char* const kInitiators[] = {"DECIDER", "RETRYPOLICY", "CRONSCHEDULE"};

// HistoryEvent's attribute key of type t: lowerCamel(type name) + "EventAttributes"
int attr_type_of_key(const std::string& k) {
  static const std::vector<std::string> keys = [] {
    std::vector<std::string> v;
    for (const char* n : kEventTypes) {
      std::string s(n);
      s[0] = (char)(s[0] - 'A' + 'a');
      v.push_back(s + "EventAttributes");
    }
    return v;
  }();
  for (int t = 0; t < CRR_EV_TYPE_COUNT; ++t)
    if (JsonReader::iequal(k, keys[t].c_str())) return t;
  return -1;
}

// an optional string field: null leaves it unset
bool opt_str(JsonReader& r, std::string& out) {
  if (r.null()) return false;
  out = r.str();
  return true;
}
template <class T>
void opt_int(JsonReader& r, T& out) {
  if (!r.null()) out = r.integer<T>();
}

void read_retry_policy(JsonReader& r, Attr& a) {  // RetryPolicy{expirationIntervalInSeconds}
  if (r.null()) return;
  a.has_retry = 1;
  r.expect('{');
  if (r.consume('}')) return;
  do {
    const std::string k = r.str();
    r.expect(':');
    if (JsonReader::iequal(k, "expirationIntervalInSeconds")) opt_int(r, a.expiration);
    else r.skip();
  } while (r.consume(','));
  r.expect('}');
}

void read_reset_points(JsonReader& r, Attr& a) {  // ResetPoints{points: [ResetPointInfo{binaryChecksum}]}
  if (r.null()) return;
  a.prev_mode = -2;
  r.expect('{');
  if (r.consume('}')) return;
  do {
    const std::string k = r.str();
    r.expect(':');
    if (!JsonReader::iequal(k, "points")) { r.skip(); continue; }
    if (r.null()) { a.prev_mode = -2; a.prev.clear(); continue; }
    a.prev_mode = 0;
    a.prev.clear();
    r.expect('[');
    if (r.consume(']')) continue;
    do {
      std::string bc;
      if (!r.null()) {
        r.expect('{');
        if (!r.consume('}')) {
          do {
            const std::string k2 = r.str();
            r.expect(':');
            if (JsonReader::iequal(k2, "binaryChecksum")) opt_str(r, bc);
            else r.skip();
          } while (r.consume(','));
          r.expect('}');
        }
      }
      a.prev.push_back(std::move(bc));
    } while (r.consume(','));
    r.expect(']');
  } while (r.consume(','));
  r.expect('}');
}

bool key_field(JsonReader& r, const std::string& k, const char* name, Attr& a) {
  if (!JsonReader::iequal(k, name)) return false;
  if (opt_str(r, a.key)) a.has_key = true;
  return true;
}
bool ref_field(JsonReader& r, const std::string& k, const char* name, Attr& a) {
  if (!JsonReader::iequal(k, name)) return false;
  opt_int(r, a.ref);
  return true;
}

// the fields of type t's attribute object that ApplyEvents consumes (same set as the thriftrw path)
void read_attributes(JsonReader& r, int t, Attr& a) {
  if (r.null()) return;
  r.expect('{');
  if (r.consume('}')) return;
  do {
    const std::string k = r.str();
    r.expect(':');
    bool used = true;
    auto is = [&](const char* n) { return JsonReader::iequal(k, n); };
    switch (t) {
      case CRR_EV_WORKFLOW_EXECUTION_STARTED:
        if (is("parentWorkflowDomain")) opt_str(r, a.domain);
        else if (is("parentWorkflowDomainID")) { std::string id; a.domain_id_set = opt_str(r, id) || a.domain_id_set; }
        else if (is("executionStartToCloseTimeoutSeconds")) opt_int(r, a.exec_s2c);
        else if (is("taskStartToCloseTimeoutSeconds")) opt_int(r, a.task_s2c);
        else if (is("initiator")) { if (!r.null()) a.initiator = r.enum_value(kInitiators, 3); }
        else if (is("attempt")) opt_int(r, a.attempt);
        else if (is("expirationTimestamp")) opt_int(r, a.expiration_ts);
        else if (is("firstDecisionTaskBackoffSeconds")) opt_int(r, a.backoff);
        else if (is("prevAutoResetPoints")) read_reset_points(r, a);
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_SCHEDULED:
        if (is("startToCloseTimeoutSeconds")) opt_int(r, a.aux);
        else if (is("attempt")) opt_int(r, a.ref);
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_STARTED:
        used = ref_field(r, k, "scheduledEventId", a);
        break;
      case CRR_EV_DECISION_TASK_COMPLETED:
        used = ref_field(r, k, "startedEventId", a) || key_field(r, k, "binaryChecksum", a);
        break;
      case CRR_EV_DECISION_TASK_TIMED_OUT:
        if (is("timeoutType")) { if (!r.null()) a.aux = r.enum_value(kTimeoutTypes, 4); }
        else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_SCHEDULED:
        if (key_field(r, k, "activityId", a)) {}
        else if (is("domain")) opt_str(r, a.domain);
        else if (is("scheduleToCloseTimeoutSeconds")) opt_int(r, a.s2c);
        else if (is("scheduleToStartTimeoutSeconds")) opt_int(r, a.s2s);
        else if (is("startToCloseTimeoutSeconds")) opt_int(r, a.st2c);
        else if (is("heartbeatTimeoutSeconds")) opt_int(r, a.hb);
        else if (is("retryPolicy")) read_retry_policy(r, a);
        else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_STARTED:
      case CRR_EV_ACTIVITY_TASK_COMPLETED:
      case CRR_EV_ACTIVITY_TASK_FAILED:
      case CRR_EV_ACTIVITY_TASK_TIMED_OUT:
      case CRR_EV_ACTIVITY_TASK_CANCELED:
        used = ref_field(r, k, "scheduledEventId", a);
        break;
      case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED:
        used = key_field(r, k, "activityId", a);
        break;
      case CRR_EV_TIMER_FIRED:
      case CRR_EV_TIMER_CANCELED:
        used = key_field(r, k, "timerId", a);
        break;
      case CRR_EV_TIMER_STARTED:
        used = key_field(r, k, "timerId", a) || ref_field(r, k, "startToFireTimeoutSeconds", a);
        break;
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED:
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED:
      case CRR_EV_SIGNAL_EXTERNAL_INITIATED:
        if (is("domain")) opt_str(r, a.domain);
        else used = false;
        break;
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED:
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED:
      case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED:
      case CRR_EV_SIGNAL_EXTERNAL_FAILED:
      case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED:
        used = ref_field(r, k, "initiatedEventId", a);
        break;
      default:
        used = false;
    }
    if (!used) r.skip();
  } while (r.consume(','));
  r.expect('}');
}

void read_event(JsonReader& r, Event& e) {
  r.expect('{');
  const char* attr_at[CRR_EV_TYPE_COUNT] = {};
  bool have_type = false;
  if (!r.consume('}')) {
    do {
      const std::string k = r.str();
      r.expect(':');
      if (JsonReader::iequal(k, "eventId")) opt_int(r, e.id);
      else if (JsonReader::iequal(k, "timestamp")) opt_int(r, e.ts);
      else if (JsonReader::iequal(k, "version")) opt_int(r, e.ver);
      else if (JsonReader::iequal(k, "taskId")) opt_int(r, e.task);
      else if (JsonReader::iequal(k, "eventType")) {
        if (!r.null()) { e.type = r.enum_value(kEventTypes, CRR_EV_TYPE_COUNT); have_type = true; }
      } else {
        const int at = attr_type_of_key(k);
        if (at >= 0) attr_at[at] = r.pos();   // the last occurrence wins; read once the type is known
        r.skip();
      }
    } while (r.consume(','));
    r.expect('}');
  }
  if (!have_type) e.type = 0;                 // a nil *EventType reads as its zero value
  if (e.type >= 0 && e.type < CRR_EV_TYPE_COUNT && attr_at[e.type]) {
    JsonReader r2(attr_at[e.type], r.pos());   // inside this event's object
    read_attributes(r2, e.type, e.a);
  }
}

}  // namespace

void json_decode_batch(const char* p, const char* end, std::vector<Event>& out) {
  JsonReader r(p, end);
  if (r.null()) { r.at_end(); return; }         // null: a nil slice, no events
  r.expect('[');
  if (!r.consume(']')) {
    do {
      if (r.null()) r.fail();                    // a nil *HistoryEvent: ApplyEvents cannot read it
      Event e;
      read_event(r, e);
      out.push_back(std::move(e));
    } while (r.consume(','));
    r.expect(']');
  }
  r.at_end();
}

}  // namespace crr_host
