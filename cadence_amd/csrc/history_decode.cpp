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
#include "host_flatten.h"
#include "json_decode.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

using namespace crr_host;

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

struct Ctx {
  const uint8_t* const* blobs;
  const uint64_t* lens;
  const uint32_t* encodings;  // null: every blob thriftrw
  uint32_t n_blobs;
  const crr_wf_source* wfs;
  const std::unordered_set<std::string>* known;  // null: every name resolves
};

void decode_workflow(const Ctx& c, uint32_t w, Chunk& k) {
  const crr_wf_source& src = c.wfs[w];
  WfFlattener f(k, c.known);
  Event e;
  for (uint32_t b = 0; b < src.blob_count; ++b) {
    const uint32_t bi = src.blob_begin + b;
    if (bi >= c.n_blobs) throw DecodeError{CRR_DECODE_BAD_ARGUMENT};
    k.err_blob = bi;
    const uint64_t len = c.lens[bi];
    const uint32_t enc = c.encodings ? c.encodings[bi] : CRR_ENCODING_THRIFTRW;
    f.batch_begin();
    if (enc > CRR_ENCODING_EMPTY) throw DecodeError{CRR_DECODE_UNKNOWN_ENCODING};
    if (len > 0 && enc != CRR_ENCODING_THRIFTRW) {   // json.Unmarshal(data, &[]*types.HistoryEvent)
      std::vector<Event> evs;
      try {
        json_decode_batch(reinterpret_cast<const char*>(c.blobs[bi]), reinterpret_cast<const char*>(c.blobs[bi]) + len, evs);
      } catch (const JsonError& je) {
        throw DecodeError{je.code};
      }
      for (Event& ev : evs) {
        ev.a.new_run = src.new_run_wf;
        f.add(ev);
      }
    } else if (len > 0) {
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
          e.a.new_run = src.new_run_wf;  // ParentWorkflowDomainID is not on the thrift wire: name lookups only
          f.add(e);
        }
      }
    }
    f.batch_end();
  }
  k.err_blob = -1;
  WfMeta m;
  m.init_version = src.init_version;
  m.now_ns = src.now_ns;
  m.run_id = src.run_id;
  m.branch_id = src.branch_id;
  m.final_token = src.final_token;
  m.final_token_len = src.final_token_len;
  m.rebuild_last_event_id = src.rebuild_last_event_id;
  m.rebuild_last_event_version = src.rebuild_last_event_version;
  m.flags = src.flags;
  m.retention_days = src.retention_days;
  f.finish(m, src.blob_count);
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

}  // namespace

extern "C" {

crr_decoded* crr_decode_histories(const uint8_t* const* blobs, const uint64_t* blob_lens, uint32_t n_blobs,
                                  const crr_wf_source* wfs, uint32_t n_wf, const char* const* known_domains,
                                  uint32_t n_known, int n_threads, int* err, int64_t* err_blob) {
  return crr_decode_histories_enc(blobs, blob_lens, nullptr, n_blobs, wfs, n_wf, known_domains, n_known, n_threads, err,
                                  err_blob);
}

crr_decoded* crr_decode_histories_enc(const uint8_t* const* blobs, const uint64_t* blob_lens,
                                      const uint32_t* blob_encodings, uint32_t n_blobs, const crr_wf_source* wfs,
                                      uint32_t n_wf, const char* const* known_domains, uint32_t n_known, int n_threads,
                                      int* err, int64_t* err_blob) {
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
  Ctx c{blobs, blob_lens, blob_encodings, n_blobs, wfs, all_known ? nullptr : &known};

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
  // concatenate with offset fix-ups and canonical slot-table bases
  auto* out = new crr_decoded();
  concat_chunks(chunks, out->all, out->table_rows);
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
