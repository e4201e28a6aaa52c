// json_ingest_kernel.hip -- JSON-encoded persisted batches in HBM -> canonical thriftrw blobs, on the GPU
// (include/cadence_ingest.h: crr_ingest_transcode_plan / crr_ingest_transcode), so the device ingest
// (ingest_kernel.hip) takes a batch whatever its blobs' encodings.
//
// serializerImpl.deserialize (common/persistence/serializer.go:312-334) decodes a DataBlob whose encoding
// is json / unknown / empty with json.Unmarshal into []*types.HistoryEvent.  The host restatement of what
// that yields for the fields ApplyEvents reads is cadence_amd/csrc/json_decode.{h,cpp} (keys matched
// case-insensitively, the last duplicate winning, null as absent, enums as names or decimal text, nesting
// past 10000 levels and any malformed value or type mismatch in a read field an error of the whole blob).
// This file restates that walk on the device and writes, per JSON blob, the thriftrw History that the
// thriftrw decoders turn into the same events: every field the JSON walk produced, with its final value,
// in thriftrw's canonical shape (0x59, then History{10: list<HistoryEvent>}; ascending field ids; the
// attribute struct of the event's own type).  Thriftrw blobs are copied as they are; a blob the walk
// rejects becomes an empty blob and the plan reports it (CRR_DECODE_BAD_JSON / _UNKNOWN_ENCODING, lowest
// index first, as crr_decode_histories_enc does).  Every string the events carry (keys, domains, reset
// points' binary checksums) is written unescaped, as encoding/json decodes it.
//
// Kernels (a lane per blob; integer / byte work, no MFMA):
//   blobs_kernel<M_PLAN>  the walk, writing the thriftrw form into the blob's staging region in the scratch
//                        (its JSON length + 64 bytes; realistic JSON shrinks ~3x) and counting its size (nesting
//                        kept in one 64-bit register: 64 levels; a deeper blob goes on the deep list, which
//                        deep_kernel<M_PLAN_DEEP> sizes with a level stack per thread in HBM, up to 10000)
//   scan                 hipCUB inclusive sum -> blob offsets of the output
//   gather_kernel        the staged blobs to their offsets (a wavefront per blob); blobs_kernel<M_WRITE> walks a
//                        blob whose form outgrew its region again into the output, deep_kernel<M_WRITE_DEEP> the
//                        deep ones
// Reads go through a 16-byte window in registers (one aligned dwordx4 per 16 bytes walked).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stddef.h>
#include <stdint.h>

#include "cadence_decode.h"
#include "cadence_ingest.h"
#include "stream_device.h"

namespace crr_json {

using i64 = int64_t;
using i32 = int32_t;
using u32 = uint32_t;
using u64 = uint64_t;
using u16 = uint16_t;
using u8 = uint8_t;
typedef u32 v4u __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;
constexpr int kMaxDepth = 10000;                       // json_decode.h JsonReader::kMaxDepth
constexpr int kDeepWords = (kMaxDepth + 2 + 63) / 64;  // one bit per level
constexpr u32 kDeepThreads = 2048;                     // threads of the deep passes (each its own stack)
constexpr u64 kNone = ~0ull;

enum : int { E_OK = 0, E_DEEP = 1, E_BAD = 2 };
// a blob's state after the plan: its thriftrw form staged (ST_OK), too large for its staging region and to be
// walked again into the output (ST_OVER), nested past 64 levels (ST_DEEP: sized and written by the deep
// passes), rejected (ST_FAILED: an empty blob)
enum : u32 { ST_OK = 0, ST_DEEP = 1, ST_FAILED = 2, ST_OVER = 3 };
constexpr u64 kStageSlack = 64;   // a blob's staging region: its own length + this (realistic JSON shrinks ~3x)
enum : u8 { T_STOP = 0, T_BOOL = 2, T_I32 = 8, T_I64 = 10, T_STRING = 11, T_STRUCT = 12, T_LIST = 15 };

// ---- name tables: ASCII-folded FNV-1a of each name, built at compile time --------------------------------
constexpr u32 fold(u32 c) { return c >= 'A' && c <= 'Z' ? c + 32 : c; }
constexpr u32 kFnv0 = 2166136261u;
constexpr u32 hstep(u32 h, u32 c) { return (h ^ fold(c)) * 16777619u; }

// every name is at most 64 bytes (the longest, RequestCancelExternalWorkflowExecutionInitiatedEventAttributes,
// is 62): its folded bytes fit 8 words, and a key is compared word for word (a longer key matches no name)
constexpr int kNameWords = 8;
template <int N, int C>
struct Names {
  char ch[C];
  u16 off[N];
  u16 len[N];
  u32 hash[N];
  u64 w[N][kNameWords];   // the folded bytes, little-endian, zero-padded
};
template <int N, int C>
constexpr Names<N, C> make_names(const char* const (&src)[N], const char* suffix) {
  Names<N, C> t{};
  int o = 0;
  for (int i = 0; i < N; ++i) {
    t.off[i] = (u16)o;
    u32 h = kFnv0;
    int n = 0;
    for (const char* s = src[i]; *s; ++s, ++n) {
      t.ch[o++] = *s; h = hstep(h, (u8)*s);
      if (n < 8 * kNameWords) t.w[i][n / 8] |= (u64)fold((u8)*s) << (8 * (n % 8));
    }
    for (const char* s = suffix; *s; ++s, ++n) {
      t.ch[o++] = *s; h = hstep(h, (u8)*s);
      if (n < 8 * kNameWords) t.w[i][n / 8] |= (u64)fold((u8)*s) << (8 * (n % 8));
    }
    t.len[i] = (u16)(n <= 8 * kNameWords ? n : 0xFFFF);   // (a longer name would never match)
    t.hash[i] = h;
  }
  return t;
}

// types.EventType names in enum order (json_decode.cpp kEventTypes); their attribute keys add "EventAttributes"
constexpr const char* kEventTypeSrc[CRR_EV_TYPE_COUNT] = {
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
constexpr const char* kTimeoutSrc[4] = {"START_TO_CLOSE", "SCHEDULE_TO_START", "SCHEDULE_TO_CLOSE", "HEARTBEAT"};
constexpr const char* kInitiatorSrc[3] = {"DECIDER", "RETRYPOLICY", "CRONSCHEDULE"};
// the JSON keys the walk reads (common/types/shared.go JSON tags)
enum Field : int {
  F_EVENT_ID, F_TIMESTAMP, F_VERSION, F_TASK_ID, F_EVENT_TYPE,
  F_PARENT_DOMAIN, F_PARENT_DOMAIN_ID, F_EXEC_S2C, F_TASK_S2C, F_INITIATOR, F_ATTEMPT, F_EXPIRATION_TS, F_BACKOFF,
  F_PREV_RESET_POINTS, F_START_TO_CLOSE, F_SCHEDULED_EVENT_ID, F_STARTED_EVENT_ID, F_BINARY_CHECKSUM,
  F_TIMEOUT_TYPE, F_ACTIVITY_ID, F_DOMAIN, F_SCHEDULE_TO_CLOSE, F_SCHEDULE_TO_START, F_HEARTBEAT, F_RETRY_POLICY,
  F_TIMER_ID, F_START_TO_FIRE, F_INITIATED_EVENT_ID, F_EXPIRATION_INTERVAL, F_POINTS, kFields
};
constexpr const char* kFieldSrc[kFields] = {
    "eventId", "timestamp", "version", "taskId", "eventType",
    "parentWorkflowDomain", "parentWorkflowDomainID", "executionStartToCloseTimeoutSeconds",
    "taskStartToCloseTimeoutSeconds", "initiator", "attempt", "expirationTimestamp", "firstDecisionTaskBackoffSeconds",
    "prevAutoResetPoints", "startToCloseTimeoutSeconds", "scheduledEventId", "startedEventId", "binaryChecksum",
    "timeoutType", "activityId", "domain", "scheduleToCloseTimeoutSeconds", "scheduleToStartTimeoutSeconds",
    "heartbeatTimeoutSeconds", "retryPolicy", "timerId", "startToFireTimeoutSeconds", "initiatedEventId",
    "expirationIntervalInSeconds", "points"};

using EvNames = Names<CRR_EV_TYPE_COUNT, 1280>;
using AttrNames = Names<CRR_EV_TYPE_COUNT, 1920>;
using FieldNames = Names<kFields, 768>;
using TimeoutNames = Names<4, 64>;
using InitNames = Names<3, 32>;
__constant__ EvNames kEvNames = make_names<CRR_EV_TYPE_COUNT, 1280>(kEventTypeSrc, "");
__constant__ AttrNames kAttrNames = make_names<CRR_EV_TYPE_COUNT, 1920>(kEventTypeSrc, "EventAttributes");
__constant__ FieldNames kFieldNames = make_names<kFields, 768>(kFieldSrc, "");
__constant__ TimeoutNames kTimeoutNames = make_names<4, 64>(kTimeoutSrc, "");
__constant__ InitNames kInitNames = make_names<3, 32>(kInitiatorSrc, "");

// ---- the reader: JsonReader (json_decode.h) over one blob [p, end) ----------------------------------------
struct SRef {      // a JSON string token: its opening quote, its decoded length, folded hash and first 64
  u64 pos;         // folded bytes (zero-padded words)
  u32 len;
  u32 hash;
  u64 h0, h1, h2, h3, h4, h5, h6, h7;
  __device__ __forceinline__ void put(u32 word, u64 v) {   // constant register indices only
    switch (word) {
      case 0: h0 = v; break; case 1: h1 = v; break; case 2: h2 = v; break; case 3: h3 = v; break;
      case 4: h4 = v; break; case 5: h5 = v; break; case 6: h6 = v; break; default: h7 = v; break;
    }
  }
};

struct JR {
  const u8* b;
  u64 p, end;
  u64 wb;          // window base (16-aligned), kNone: none
  v4u w;
  int err;         // E_*
  int depth;       // open '{' / '[' (JsonReader::level)
  u64 kinds;       // skip()'s level kinds, levels 0..63: 1 = object
  u64* deep;       // levels 64.. (the deep passes), nullptr: such a blob is deferred

  __device__ __forceinline__ void init(const u8* bytes, u64 begin, u64 e, u64* deep_stack) {
    b = bytes; p = begin; end = e; wb = kNone; err = E_OK; depth = 0; kinds = 0; deep = deep_stack;
  }
  __device__ __forceinline__ void fail() { if (err == E_OK) err = E_BAD; }
  // byte q (< end: `bytes` is readable to the 16-byte boundary past the last blob)
  __device__ __forceinline__ u32 at(u64 q) {
    const u64 a = q & ~15ull;
    if (a != wb) {
      w = *reinterpret_cast<const v4u*>(b + a);
      wb = a;
    }
    const u32 o = (u32)(q & 15);
    const u32 d = (o & 8) ? ((o & 4) ? w.w : w.z) : ((o & 4) ? w.y : w.x);
    return (d >> (8 * (o & 3))) & 0xff;
  }
  __device__ __forceinline__ static bool is_ws(u32 c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
  __device__ __forceinline__ static bool is_digit(u32 c) { return c >= '0' && c <= '9'; }
  __device__ __forceinline__ void ws() {
    while (p < end && is_ws(at(p))) ++p;
  }
  __device__ __forceinline__ int peek() {   // -1 at the end (an error)
    ws();
    if (p >= end) { fail(); return -1; }
    return (int)at(p);
  }
  __device__ __forceinline__ void level(u32 c) {
    if (c == '{' || c == '[') {
      if (++depth > kMaxDepth) fail();
    } else if (c == '}' || c == ']') {
      --depth;
    }
  }
  __device__ __forceinline__ void expect(u32 c) {
    if (err) return;
    if (peek() != (int)c) { fail(); return; }
    ++p;
    level(c);
  }
  __device__ __forceinline__ bool consume(u32 c) {
    if (err) return false;
    if (peek() != (int)c) return false;
    ++p;
    level(c);
    return true;
  }
  __device__ __forceinline__ void lit(u64 w0, u32 n) {   // the literal's n <= 8 bytes, little-endian in w0
    ws();
    if (end - p < n) { fail(); return; }
    for (u32 i = 0; i < n; ++i)
      if (at(p + i) != ((w0 >> (8 * i)) & 0xff)) { fail(); return; }
    p += n;
  }
  static constexpr u64 kNull = 0x6c6c756eull, kTrue = 0x65757274ull, kFalse = 0x65736c6166ull;
  __device__ __forceinline__ bool null() {
    if (err) return false;
    if (peek() != 'n') return false;
    lit(kNull, 4);
    return err == E_OK;
  }
  __device__ __forceinline__ void at_end() {
    ws();
    if (p != end) fail();
  }

  // -- strings: the decoded bytes one at a time (JsonReader::str) --
  struct SIt {
    u64 q;
    u32 pend;
    int np;
  };
  __device__ __forceinline__ u32 hex4(u64& q) {
    if (end - q < 4) { fail(); return 0; }
    u32 v = 0;
    for (int i = 0; i < 4; ++i) {
      const u32 c = at(q++);
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else { fail(); return 0; }
    }
    return v;
  }
  // next decoded byte; -1: the closing quote (consumed); -2: an error
  __device__ int snext(SIt& it) {
    if (it.np) {
      const int c = (int)(it.pend & 0xff);
      it.pend >>= 8;
      --it.np;
      return c;
    }
    if (err) return -2;
    if (it.q >= end) { fail(); return -2; }
    const u32 c = at(it.q++);
    if (c == '"') return -1;
    if (c < 0x20) { fail(); return -2; }
    if (c != '\\') return (int)c;
    if (it.q >= end) { fail(); return -2; }
    const u32 e = at(it.q++);
    switch (e) {
      case '"': case '\\': case '/': return (int)e;
      case 'b': return '\b';
      case 'f': return '\f';
      case 'n': return '\n';
      case 'r': return '\r';
      case 't': return '\t';
      case 'u': {
        u32 cp = hex4(it.q);
        if (err) return -2;
        if (cp >= 0xD800 && cp < 0xDC00 && end - it.q >= 6 && at(it.q) == '\\' && at(it.q + 1) == 'u') {
          const u64 save = it.q;
          it.q += 2;
          const u32 lo = hex4(it.q);
          if (err) return -2;
          if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          else { it.q = save; cp = 0xFFFD; }
        } else if (cp >= 0xD800 && cp < 0xE000) {
          cp = 0xFFFD;   // a lone surrogate: encoding/json's U+FFFD
        }
        if (cp < 0x80) return (int)cp;
        u32 first;
        if (cp < 0x800) {
          first = 0xC0 | (cp >> 6);
          it.pend = 0x80 | (cp & 0x3F); it.np = 1;
        } else if (cp < 0x10000) {
          first = 0xE0 | (cp >> 12);
          it.pend = (0x80 | ((cp >> 6) & 0x3F)) | (0x80 | (cp & 0x3F)) << 8; it.np = 2;
        } else {
          first = 0xF0 | (cp >> 18);
          it.pend = (0x80 | ((cp >> 12) & 0x3F)) | (0x80 | ((cp >> 6) & 0x3F)) << 8 | (0x80 | (cp & 0x3F)) << 16;
          it.np = 3;
        }
        return (int)first;
      }
      default: fail(); return -2;
    }
  }
  __device__ __forceinline__ SIt sit(u64 quote) const { return SIt{quote + 1, 0, 0}; }
  // a string token at the cursor: its reference, the cursor past it
  __device__ SRef str() {
    SRef k{kNone, 0, kFnv0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (err) return k;
    if (peek() != '"') { fail(); return k; }
    k.pos = p;
    SIt it = sit(p);
    u64 cur = 0;
    for (;;) {
      const int c = snext(it);
      if (c < 0) break;
      const u32 j = k.len++;
      k.hash = hstep(k.hash, (u32)c);
      if (j < 8 * kNameWords) {
        cur |= (u64)fold((u32)c) << (8 * (j & 7));
        if ((j & 7) == 7) { k.put(j >> 3, cur); cur = 0; }
      }
    }
    if ((k.len & 7) && k.len < 8 * kNameWords) k.put(k.len >> 3, cur);
    p = it.q;
    return k;
  }
  // the string at `k` equals name i of table T, ASCII case folded (JsonReader::iequal)
  // (every folded byte compared: the words hold all of a key as long as any name)
  template <class T>
  __device__ __forceinline__ bool keq(const SRef& k, const T& t, int i) {
    if (err || k.len != t.len[i] || k.hash != t.hash[i]) return false;
    const u64* w = t.w[i];
    return k.h0 == w[0] && k.h1 == w[1] && k.h2 == w[2] && k.h3 == w[3] && k.h4 == w[4] && k.h5 == w[5] &&
           k.h6 == w[6] && k.h7 == w[7];
  }
  template <class T>
  __device__ int find(const SRef& k, const T& t, int n) {
    for (int i = 0; i < n; ++i)
      if (keq(k, t, i)) return i;
    return -1;
  }

  // -- numbers --
  // a JSON integer that fits i64 / i32 (json_decode.h JsonReader::integer)
  template <bool Wide>
  __device__ i64 integer() {
    if (err) return 0;
    ws();
    bool neg = false;
    if (p < end && at(p) == '-') { neg = true; ++p; }
    if (p >= end || !is_digit(at(p))) { fail(); return 0; }
    if (at(p) == '0' && p + 1 < end && is_digit(at(p + 1))) { fail(); return 0; }
    u64 v = 0;
    while (p < end && is_digit(at(p))) {
      const u64 d = at(p++) - '0';
      if (v > (~0ull - d) / 10) { fail(); return 0; }   // >= 2^64: no integer type holds it
      v = v * 10 + d;
    }
    if (p < end) {
      const u32 c = at(p);
      if (c == '.' || c == 'e' || c == 'E') { fail(); return 0; }
    }
    const u64 lim = Wide ? (1ull << 63) : (1ull << 31);
    if (neg ? v > lim : v > lim - 1) { fail(); return 0; }
    return neg ? (i64)(0ull - v) : (i64)v;
  }
  // the JSON number grammar, syntax only (JsonReader::number)
  __device__ void number() {
    ws();
    if (p < end && at(p) == '-') ++p;
    if (p >= end || !is_digit(at(p))) { fail(); return; }
    if (at(p) == '0') ++p;
    else while (p < end && is_digit(at(p))) ++p;
    if (p < end && at(p) == '.') {
      ++p;
      if (p >= end || !is_digit(at(p))) { fail(); return; }
      while (p < end && is_digit(at(p))) ++p;
    }
    if (p < end && (at(p) == 'e' || at(p) == 'E')) {
      ++p;
      if (p < end && (at(p) == '+' || at(p) == '-')) ++p;
      if (p >= end || !is_digit(at(p))) { fail(); return; }
      while (p < end && is_digit(at(p))) ++p;
    }
    if (p < end) {
      const u32 c = at(p);
      if (is_digit(c) || c == '.' || c == '+' || c == '-' || c == 'e' || c == 'E') fail();
    }
  }
  // an enum (UnmarshalText): a JSON string holding a name of T or a decimal int32 (JsonReader::enum_value)
  template <class T>
  __device__ i32 enum_value(const T& t, int n) {
    if (err) return 0;
    if (peek() != '"') { fail(); return 0; }
    const SRef k = str();
    if (err) return 0;
    const int i = find(k, t, n);
    if (i >= 0) return i;
    SIt it = sit(k.pos);
    u32 j = 0;
    bool neg = false;
    int c = snext(it);
    if (c == '+' || c == '-') { neg = c == '-'; ++j; c = snext(it); }
    if (j == k.len) { fail(); return 0; }
    i64 v = 0;
    for (; j < k.len; ++j, c = snext(it)) {
      if (c < '0' || c > '9') { fail(); return 0; }
      v = v * 10 + (c - '0');
      if (v > ((i64)1 << 31)) { fail(); return 0; }
    }
    if (neg) v = -v;
    if (v < INT32_MIN || v > INT32_MAX) { fail(); return 0; }
    return (i32)v;
  }

  // -- skip any value (JsonReader::skip), without recursion: a kind bit per open level --
  __device__ __forceinline__ void push_kind(bool obj) {
    const int i = depth - 1;
    if (i < 64) {
      kinds = obj ? kinds | (1ull << i) : kinds & ~(1ull << i);
    } else if (deep) {
      u64& wd = deep[i / 64];
      wd = obj ? wd | (1ull << (i % 64)) : wd & ~(1ull << (i % 64));
    } else if (err == E_OK) {
      err = E_DEEP;
    }
  }
  __device__ __forceinline__ bool top_is_object() const {
    const int i = depth - 1;
    return i < 64 ? (kinds >> i) & 1 : (deep[i / 64] >> (i % 64)) & 1;
  }
  __device__ void skip() {
    const int d0 = depth;
    bool key = false;   // the next token is an object's key
    while (!err) {
      if (key) {
        (void)str();
        expect(':');
        key = false;
        continue;
      }
      const int c = peek();
      if (err) return;
      if (c == '"') {
        (void)str();
      } else if (c == '{') {
        expect('{');
        push_kind(true);
        if (err) return;
        if (!consume('}')) { key = true; continue; }
      } else if (c == '[') {
        expect('[');
        push_kind(false);
        if (err) return;
        if (!consume(']')) continue;
      } else if (c == 't') {
        lit(kTrue, 4);
      } else if (c == 'f') {
        lit(kFalse, 5);
      } else if (c == 'n') {
        lit(kNull, 4);
      } else {
        number();
      }
      // a value is done: close levels until the next value (or the starting level)
      for (;;) {
        if (err || depth == d0) return;
        const bool obj = top_is_object();
        if (consume(',')) { key = obj; break; }
        expect(obj ? '}' : ']');
      }
    }
  }
};

// ---- the attributes the walk keeps (host_flatten.h Attr, strings as their token positions) ----------------
struct Attr {
  i64 ref, expiration_ts;
  i32 aux, s2s, s2c, st2c, hb, has_retry, expiration, task_s2c, exec_s2c, backoff, initiator, attempt;
  u64 key;          // string token of the key, kNone: unset (has_key false)
  u64 domain;       // string token of the domain, kNone: unset
  bool domain_id_set;
  int prev_mode;    // -1 nil, -2 Points nil, 0 a list (the array at `points`)
  u64 points;
  __device__ __forceinline__ void clear() {
    ref = expiration_ts = 0;
    aux = s2s = s2c = st2c = hb = has_retry = expiration = task_s2c = exec_s2c = backoff = attempt = 0;
    initiator = CRR_INITIATOR_NIL;
    key = domain = points = kNone;
    domain_id_set = false;
    prev_mode = -1;
  }
};

__device__ __forceinline__ bool opt_str(JR& r, u64& pos) {
  if (r.null() || r.err) return false;
  const SRef k = r.str();
  if (r.err) return false;
  pos = k.pos;
  return true;
}
template <bool Wide, class T>
__device__ __forceinline__ void opt_int(JR& r, T& out) {
  if (!r.null() && !r.err) {
    const i64 v = r.integer<Wide>();
    if (!r.err) out = (T)v;
  }
}

// RetryPolicy{expirationIntervalInSeconds} (json_decode.cpp read_retry_policy)
__device__ void read_retry_policy(JR& r, Attr& a) {
  if (r.null() || r.err) return;
  a.has_retry = 1;
  r.expect('{');
  if (r.consume('}')) return;
  do {
    const SRef k = r.str();
    r.expect(':');
    if (r.keq(k, kFieldNames, F_EXPIRATION_INTERVAL)) opt_int<false>(r, a.expiration);
    else r.skip();
  } while (!r.err && r.consume(','));
  r.expect('}');
}

// one ResetPointInfo (null or an object): its binaryChecksum's token, kNone: "" (json_decode.cpp)
__device__ u64 read_reset_point(JR& r) {
  u64 bc = kNone;
  if (r.null() || r.err) return bc;
  r.expect('{');
  if (r.consume('}')) return bc;
  do {
    const SRef k = r.str();
    r.expect(':');
    if (r.keq(k, kFieldNames, F_BINARY_CHECKSUM)) opt_str(r, bc);
    else r.skip();
  } while (!r.err && r.consume(','));
  r.expect('}');
  return bc;
}

// ResetPoints{points: [...]} (json_decode.cpp read_reset_points): the last points array is the list
__device__ void read_reset_points(JR& r, Attr& a) {
  if (r.null() || r.err) return;
  a.prev_mode = -2;
  r.expect('{');
  if (r.consume('}')) return;
  do {
    const SRef k = r.str();
    r.expect(':');
    if (!r.keq(k, kFieldNames, F_POINTS)) { r.skip(); continue; }
    if (r.null()) { a.prev_mode = -2; a.points = kNone; continue; }
    if (r.err) break;
    a.prev_mode = 0;
    r.ws();
    a.points = r.p;
    r.expect('[');
    if (r.consume(']')) continue;
    do { (void)read_reset_point(r); } while (!r.err && r.consume(','));
    r.expect(']');
  } while (!r.err && r.consume(','));
  r.expect('}');
}

// the fields of type t's attribute object that ApplyEvents consumes (json_decode.cpp read_attributes)
__device__ void read_attributes(JR& r, int t, Attr& a) {
  if (r.null() || r.err) return;
  r.expect('{');
  if (r.consume('}')) return;
  do {
    const SRef k = r.str();
    r.expect(':');
    if (r.err) return;
    auto is = [&](int f) { return r.keq(k, kFieldNames, f); };
    bool used = true;
    switch (t) {
      case CRR_EV_WORKFLOW_EXECUTION_STARTED:
        if (is(F_PARENT_DOMAIN)) opt_str(r, a.domain);
        else if (is(F_PARENT_DOMAIN_ID)) { u64 id = kNone; if (opt_str(r, id)) a.domain_id_set = true; }
        else if (is(F_EXEC_S2C)) opt_int<false>(r, a.exec_s2c);
        else if (is(F_TASK_S2C)) opt_int<false>(r, a.task_s2c);
        else if (is(F_INITIATOR)) { if (!r.null() && !r.err) a.initiator = r.enum_value(kInitNames, 3); }
        else if (is(F_ATTEMPT)) opt_int<false>(r, a.attempt);
        else if (is(F_EXPIRATION_TS)) opt_int<true>(r, a.expiration_ts);
        else if (is(F_BACKOFF)) opt_int<false>(r, a.backoff);
        else if (is(F_PREV_RESET_POINTS)) read_reset_points(r, a);
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_SCHEDULED:
        if (is(F_START_TO_CLOSE)) opt_int<false>(r, a.aux);
        else if (is(F_ATTEMPT)) opt_int<true>(r, a.ref);
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_STARTED:
        if (is(F_SCHEDULED_EVENT_ID)) opt_int<true>(r, a.ref);
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_COMPLETED:
        if (is(F_STARTED_EVENT_ID)) opt_int<true>(r, a.ref);
        else if (is(F_BINARY_CHECKSUM)) opt_str(r, a.key);
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_TIMED_OUT:
        if (is(F_TIMEOUT_TYPE)) { if (!r.null() && !r.err) a.aux = r.enum_value(kTimeoutNames, 4); }
        else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_SCHEDULED:
        if (is(F_ACTIVITY_ID)) opt_str(r, a.key);
        else if (is(F_DOMAIN)) opt_str(r, a.domain);
        else if (is(F_SCHEDULE_TO_CLOSE)) opt_int<false>(r, a.s2c);
        else if (is(F_SCHEDULE_TO_START)) opt_int<false>(r, a.s2s);
        else if (is(F_START_TO_CLOSE)) opt_int<false>(r, a.st2c);
        else if (is(F_HEARTBEAT)) opt_int<false>(r, a.hb);
        else if (is(F_RETRY_POLICY)) read_retry_policy(r, a);
        else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_STARTED:
      case CRR_EV_ACTIVITY_TASK_COMPLETED:
      case CRR_EV_ACTIVITY_TASK_FAILED:
      case CRR_EV_ACTIVITY_TASK_TIMED_OUT:
      case CRR_EV_ACTIVITY_TASK_CANCELED:
        if (is(F_SCHEDULED_EVENT_ID)) opt_int<true>(r, a.ref);
        else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED:
        if (is(F_ACTIVITY_ID)) opt_str(r, a.key);
        else used = false;
        break;
      case CRR_EV_TIMER_FIRED:
      case CRR_EV_TIMER_CANCELED:
        if (is(F_TIMER_ID)) opt_str(r, a.key);
        else used = false;
        break;
      case CRR_EV_TIMER_STARTED:
        if (is(F_TIMER_ID)) opt_str(r, a.key);
        else if (is(F_START_TO_FIRE)) opt_int<true>(r, a.ref);
        else used = false;
        break;
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED:
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED:
      case CRR_EV_SIGNAL_EXTERNAL_INITIATED:
        if (is(F_DOMAIN)) opt_str(r, a.domain);
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
        if (is(F_INITIATED_EVENT_ID)) opt_int<true>(r, a.ref);
        else used = false;
        break;
      default:
        used = false;
    }
    if (!used) r.skip();
  } while (!r.err && r.consume(','));
  r.expect('}');
}

// ---- the thriftrw writer (W: write; else count) --------------------------------------------------------------
template <bool W>
struct TW {
  u8* o;
  u64 n;
  u64 lim;           // W: bytes past `lim` are counted, not written (the staging region's end)
  __device__ __forceinline__ void u8_(u32 v) {
    if constexpr (W) {
      if (n < lim) o[n] = (u8)v;
    }
    ++n;
  }
  __device__ __forceinline__ void be32_at(u64 at, u32 v) {
    if constexpr (W) {
      if (at + 4 <= lim) {
        o[at] = (u8)(v >> 24); o[at + 1] = (u8)(v >> 16); o[at + 2] = (u8)(v >> 8); o[at + 3] = (u8)v;
      }
    }
  }
  __device__ __forceinline__ void be32(u32 v) { be32_at(n, v); n += 4; }
  __device__ __forceinline__ void be64(u64 v) { be32((u32)(v >> 32)); be32((u32)v); }
  __device__ __forceinline__ void field(u32 t, u32 id) { u8_(t); u8_(id >> 8); u8_(id & 0xff); }
  __device__ __forceinline__ void i32f(u32 id, i32 v) { field(T_I32, id); be32((u32)v); }
  __device__ __forceinline__ void i64f(u32 id, i64 v) { field(T_I64, id); be64((u64)v); }
  // a string field from a JSON string token, unescaped; `omit_empty`: nothing for ""
  __device__ void strf(JR& r, u32 id, u64 tok, bool omit_empty) {
    u32 len = 0;
    if (tok != kNone) {
      JR::SIt it = r.sit(tok);
      while (r.snext(it) >= 0) ++len;
    }
    if (len == 0 && omit_empty) return;
    field(T_STRING, id);
    be32(len);
    if (tok == kNone) return;
    JR::SIt it = r.sit(tok);
    for (u32 j = 0; j < len; ++j) u8_((u32)r.snext(it));
  }
};

// the attribute struct of type t from the walk's final values (blob_encode.cpp / history_decode.cpp field ids)
template <bool W>
__device__ void emit_attributes(JR& r, TW<W>& w, int t, const Attr& a) {
  w.field(T_STRUCT, 40 + 10 * t);
  switch (t) {
    case CRR_EV_WORKFLOW_EXECUTION_STARTED:
      if (!a.domain_id_set) w.strf(r, 12, a.domain, true);   // ParentWorkflowDomainID given: NOT_SET
      w.i32f(40, a.exec_s2c);
      w.i32f(50, a.task_s2c);
      w.i32f(55, a.initiator);
      w.i32f(80, a.attempt);
      w.i64f(90, a.expiration_ts);
      w.i32f(110, a.backoff);
      if (a.prev_mode == -2) {
        w.field(T_STRUCT, 130);
        w.u8_(T_STOP);
      } else if (a.prev_mode == 0) {
        w.field(T_STRUCT, 130);
        w.field(T_LIST, 10);
        w.u8_(T_STRUCT);
        const u64 count_at = w.n;
        w.be32(0);
        u32 n = 0;
        JR q = r;
        q.p = a.points;
        q.depth = 0;
        q.expect('[');
        if (!q.consume(']')) {
          do {
            const u64 bc = read_reset_point(q);
            w.strf(r, 10, bc, false);
            w.u8_(T_STOP);
            ++n;
          } while (!q.err && q.consume(','));
        }
        w.be32_at(count_at, n);
        w.u8_(T_STOP);
      }
      break;
    case CRR_EV_DECISION_TASK_SCHEDULED: w.i32f(20, a.aux); w.i64f(30, a.ref); break;
    case CRR_EV_DECISION_TASK_STARTED: w.i64f(10, a.ref); break;
    case CRR_EV_DECISION_TASK_COMPLETED:
      w.i64f(30, a.ref);
      if (a.key != kNone) w.strf(r, 50, a.key, false);
      break;
    case CRR_EV_DECISION_TASK_TIMED_OUT: w.i32f(30, a.aux); break;
    case CRR_EV_ACTIVITY_TASK_SCHEDULED:
      if (a.key != kNone) w.strf(r, 10, a.key, false);
      w.strf(r, 25, a.domain, true);
      w.i32f(45, a.s2c); w.i32f(50, a.s2s); w.i32f(55, a.st2c); w.i32f(60, a.hb);
      if (a.has_retry) {
        w.field(T_STRUCT, 110);
        w.i32f(60, a.expiration);
        w.u8_(T_STOP);
      }
      break;
    case CRR_EV_ACTIVITY_TASK_STARTED: case CRR_EV_ACTIVITY_TASK_TIMED_OUT: w.i64f(10, a.ref); break;
    case CRR_EV_ACTIVITY_TASK_COMPLETED: w.i64f(20, a.ref); break;
    case CRR_EV_ACTIVITY_TASK_FAILED: case CRR_EV_ACTIVITY_TASK_CANCELED: w.i64f(30, a.ref); break;
    case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED: case CRR_EV_TIMER_FIRED: case CRR_EV_TIMER_CANCELED:
      if (a.key != kNone) w.strf(r, 10, a.key, false);
      break;
    case CRR_EV_TIMER_STARTED:
      if (a.key != kNone) w.strf(r, 10, a.key, false);
      w.i64f(20, a.ref);
      break;
    case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED: w.strf(r, 10, a.domain, true); break;
    case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED: case CRR_EV_SIGNAL_EXTERNAL_INITIATED:
      w.strf(r, 20, a.domain, true);
      break;
    case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED:
      w.i64f(60, a.ref);
      break;
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED: w.i64f(20, a.ref); break;
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED:
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT: case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED:
    case CRR_EV_SIGNAL_EXTERNAL_FAILED:
      w.i64f(50, a.ref);
      break;
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED: w.i64f(40, a.ref); break;
    case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED: case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED:
      w.i64f(10, a.ref);
      break;
    default:
      break;
  }
  w.u8_(T_STOP);
}

// one HistoryEvent object (json_decode.cpp read_event): the top-level fields, then the attribute object of
// the event's own type (the last occurrence of its key) read once the type is known
template <bool W>
__device__ void event(JR& r, TW<W>& w) {
  r.ws();
  const u64 obj = r.p;
  const int d_obj = r.depth;
  i64 id = 0, ts = 0, ver = 0, task = 0;
  i32 type = 0;
  bool have_type = false;
  // the last attribute key seen and where its value starts; `mixed`: keys of two types seen (then, unless
  // the last one is the event's type, a second pass finds the type's last occurrence)
  int attr_t = -1;
  u64 attr_at = kNone;
  bool mixed = false;
  // the event's own attributes read as they come when its type is already known (Go's marshal order puts
  // eventType first): `a` then holds the object at `a_at`, used if that is the occurrence the host reads
  Attr a;
  a.clear();
  u64 a_at = kNone;
  int a_t = -1;
  r.expect('{');
  if (!r.consume('}')) {
    do {
      const SRef k = r.str();
      r.expect(':');
      if (r.err) return;
      if (r.keq(k, kFieldNames, F_EVENT_ID)) opt_int<true>(r, id);
      else if (r.keq(k, kFieldNames, F_TIMESTAMP)) opt_int<true>(r, ts);
      else if (r.keq(k, kFieldNames, F_VERSION)) opt_int<true>(r, ver);
      else if (r.keq(k, kFieldNames, F_TASK_ID)) opt_int<true>(r, task);
      else if (r.keq(k, kFieldNames, F_EVENT_TYPE)) {
        if (!r.null() && !r.err) { type = r.enum_value(kEvNames, CRR_EV_TYPE_COUNT); have_type = true; }
      } else {
        const int t = r.find(k, kAttrNames, CRR_EV_TYPE_COUNT);
        bool read = false;
        if (t >= 0) {
          if (attr_t >= 0 && attr_t != t) mixed = true;
          attr_t = t;
          r.ws();
          attr_at = r.p;
          if (have_type && t == type) {
            const JR save = r;
            Attr ta;
            ta.clear();
            read_attributes(r, t, ta);
            if (r.err == E_DEEP) return;
            if (r.err == E_OK) {
              a = ta;
              a_at = attr_at;
              a_t = t;
              read = true;
            } else {
              r = save;   // a type error counts only if this is the occurrence read: the syntax check below
            }
          }
        }
        if (!read) r.skip();
      }
    } while (!r.err && r.consume(','));
    r.expect('}');
  }
  if (r.err) return;
  if (!have_type) type = 0;   // a nil *EventType reads as its zero value
  const u64 obj_end = r.p;
  const bool valid = type >= 0 && type < CRR_EV_TYPE_COUNT;
  if (valid) {
    // the attribute key's last occurrence: the last attribute key if it is the type's, else (keys of several
    // types seen) a second walk of the object (validated above: this walk cannot fail)
    u64 at = attr_t == type ? attr_at : kNone;
    if (attr_t != type && mixed) {
      JR q = r;
      q.p = obj;
      q.depth = d_obj;
      q.expect('{');
      if (!q.consume('}')) {
        do {
          const SRef k = q.str();
          q.expect(':');
          if (q.keq(k, kAttrNames, type)) { q.ws(); at = q.p; }
          q.skip();
        } while (!q.err && q.consume(','));
      }
    }
    if (at != kNone && !(at == a_at && a_t == type)) {
      JR q2 = r;
      q2.p = at;
      q2.end = obj_end;
      q2.depth = d_obj + 1;
      a.clear();
      read_attributes(q2, type, a);
      if (q2.err) { r.err = q2.err; return; }
    } else if (at == kNone) {
      a.clear();
    }
  }
  w.i64f(10, id);
  w.i64f(20, ts);
  w.i32f(30, type);
  w.i64f(35, ver);
  w.i64f(36, task);
  if (valid) emit_attributes(r, w, type, a);
  w.u8_(T_STOP);
}

// one blob -> thriftrw (json_decode.cpp json_decode_batch); r.err on a rejection or a deferral
template <bool W>
__device__ void transcode_json(JR& r, TW<W>& w) {
  if (r.null()) { r.at_end(); return; }   // null: a nil slice, no events (an empty blob)
  if (r.err) return;
  w.u8_(0x59);
  w.field(T_LIST, 10);
  w.u8_(T_STRUCT);
  const u64 count_at = w.n;
  w.be32(0);
  u32 n = 0;
  r.expect('[');
  if (!r.consume(']')) {
    do {
      if (r.null()) { r.fail(); return; }   // a nil *HistoryEvent: ApplyEvents cannot read it
      if (r.err) return;
      event(r, w);
      ++n;
    } while (!r.err && r.consume(','));
    r.expect(']');
  }
  r.at_end();
  w.be32_at(count_at, n);
  w.u8_(T_STOP);
}

struct Scratch {    // carved from the caller's scratch (both calls carve it the same way)
  u64* size;        // [n_blobs] the transcoded size
  u64* off;         // [n_blobs + 1] exclusive prefixes
  u32* status;      // [n_blobs] ST_*
  u64* err;         // [1] (blob << 8) | -code, min wins
  u32* n_deep;      // [1]
  u32* deep_list;   // [n_blobs]
  u64* stacks;      // [kDeepThreads][kDeepWords]
  void* scan_tmp;
  size_t scan_tmp_bytes;
  size_t bytes;     // the carve up to the staging area
  u8* stage;        // the rest of the scratch: blob i's thriftrw form at (blob_off[i] - blob_off[0]) + 64 i
  u64 stage_cap;
};

__device__ __forceinline__ void record_error(u64* err, u32 blob, int code) {
  atomicMin((unsigned long long*)err, ((u64)blob << 8) | (u64)(-code));
}

// The blob's walk, by mode:
//   M_PLAN        written into its staging region (to the region's end), sized: ST_OK / ST_OVER / ST_DEEP /
//                 ST_FAILED
//   M_PLAN_DEEP   a deep-list blob sized with the whole level stack
//   M_WRITE       an ST_OVER blob walked again into the output at its offset
//   M_WRITE_DEEP  a deep-list blob written into the output
enum Mode : int { M_PLAN, M_PLAN_DEEP, M_WRITE, M_WRITE_DEEP };
template <int M>
__device__ void one_blob(const crr_blob_batch& in, const u32* enc, const Scratch& S, u8* out, u32 bi, u64* stack) {
  constexpr bool kPlan = M == M_PLAN || M == M_PLAN_DEEP;
  const u64 b0 = in.blob_off[bi], b1 = in.blob_off[bi + 1];
  const u32 e = enc ? enc[bi] : CRR_ENCODING_THRIFTRW;
  if (M == M_WRITE && S.status[bi] != ST_OVER) return;
  if (M == M_WRITE_DEEP && S.status[bi] != ST_DEEP) return;
  if (M == M_PLAN && e > CRR_ENCODING_EMPTY) {   // NewUnknownEncodingTypeError (serializer.go:326-327), any length
    S.size[bi] = 0;
    S.status[bi] = ST_FAILED;
    record_error(S.err, bi, CRR_DECODE_UNKNOWN_ENCODING);
    return;
  }
  // the staging region (M_PLAN): blobs past the scratch's end get none
  const u64 reg = (b0 - in.blob_off[0]) + kStageSlack * bi;
  const u64 reg_len = b1 - b0 + kStageSlack;
  const u64 lim = reg + reg_len <= S.stage_cap ? reg_len : 0;
  u8* const dst = M == M_PLAN ? S.stage + reg : M == M_PLAN_DEEP ? nullptr : out + S.off[bi];
  if (e == CRR_ENCODING_THRIFTRW || b1 == b0) {   // as persisted (an empty blob: no events)
    if (M == M_PLAN) {
      S.size[bi] = b1 - b0;
      if (b1 - b0 <= lim) {
        for (u64 q = b0; q < b1; ++q) dst[q - b0] = in.bytes[q];
        S.status[bi] = ST_OK;
      } else {
        S.status[bi] = ST_OVER;
      }
    } else if (M == M_WRITE) {
      for (u64 q = b0; q < b1; ++q) dst[q - b0] = in.bytes[q];
    }
    return;
  }
  JR r;
  r.init(in.bytes, b0, b1, stack);
  if (M == M_PLAN_DEEP) {
    TW<false> w{nullptr, 0, 0};
    transcode_json(r, w);
    if (r.err) {
      S.size[bi] = 0;
      S.status[bi] = ST_FAILED;
      record_error(S.err, bi, CRR_DECODE_BAD_JSON);
    } else {
      S.size[bi] = w.n;
    }
    return;
  }
  TW<true> w{dst, 0, M == M_PLAN ? lim : ~0ull};
  transcode_json(r, w);
  if (!kPlan) return;
  if (r.err == E_DEEP) {   // nested past the register stack: the deep passes
    S.status[bi] = ST_DEEP;
    S.deep_list[atomicAdd(S.n_deep, 1u)] = bi;
    return;
  }
  if (r.err) {
    S.size[bi] = 0;
    S.status[bi] = ST_FAILED;
    record_error(S.err, bi, CRR_DECODE_BAD_JSON);
    return;
  }
  S.size[bi] = w.n;
  S.status[bi] = w.n <= lim ? ST_OK : ST_OVER;
}

template <int M>
__global__ __launch_bounds__(kBlock) void blobs_kernel(crr_blob_batch in, const u32* enc, Scratch S, u8* out) {
  const u32 bi = blockIdx.x * kBlock + threadIdx.x;
  if (bi >= in.n_blobs) return;
  one_blob<M>(in, enc, S, out, bi, nullptr);
}

// the staged blobs into the output at their offsets: a wavefront per blob, its lanes copying 8 bytes apart
__global__ __launch_bounds__(kBlock) void gather_kernel(crr_blob_batch in, Scratch S, u8* out) {
  const u32 lane = threadIdx.x & 63, nw = gridDim.x * (kBlock / 64);
  for (u32 bi = blockIdx.x * (kBlock / 64) + threadIdx.x / 64; bi < in.n_blobs; bi += nw) {
    if (S.status[bi] != ST_OK) continue;
    const u8* src = S.stage + (in.blob_off[bi] - in.blob_off[0]) + kStageSlack * bi;
    u8* dst = out + S.off[bi];
    const u64 n = S.size[bi];
    for (u64 j = lane; j < n; j += 64) dst[j] = src[j];
  }
}

// the deep list, grid-stride; each thread's level stack in HBM
template <int M>
__global__ __launch_bounds__(kBlock) void deep_kernel(crr_blob_batch in, const u32* enc, Scratch S, u8* out) {
  const u32 t = blockIdx.x * kBlock + threadIdx.x;
  const u32 n = *S.n_deep;
  u64* stack = S.stacks + (u64)t * kDeepWords;
  for (u32 i = t; i < n; i += kDeepThreads) one_blob<M>(in, enc, S, out, S.deep_list[i], stack);
}

size_t scan_tmp_bytes(uint32_t n_blobs) {
  size_t tmp = 0;
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, tmp, (const u64*)nullptr, (u64*)nullptr, (int)(n_blobs ? n_blobs : 1));
  return tmp;
}

Scratch carve(void* base, uint32_t n_blobs, size_t scratch_bytes) {
  Scratch c{};
  size_t used = 0;
  auto take = [&](size_t nb) -> void* {
    void* p = base ? static_cast<u8*>(base) + used : nullptr;
    used += (nb + 255) & ~(size_t)255;
    return p;
  };
  const u64 nb = n_blobs;
  c.size = (u64*)take(8 * (nb + 1));
  c.off = (u64*)take(8 * (nb + 1));
  c.status = (u32*)take(4 * (nb + 1));
  c.err = (u64*)take(8);
  c.n_deep = (u32*)take(4);
  c.deep_list = (u32*)take(4 * (nb + 1));
  c.stacks = (u64*)take(8ull * kDeepWords * kDeepThreads);
  c.scan_tmp_bytes = scan_tmp_bytes(n_blobs);
  c.scan_tmp = take(c.scan_tmp_bytes);
  c.bytes = used;
  c.stage = base ? static_cast<u8*>(base) + used : nullptr;
  c.stage_cap = scratch_bytes > used ? scratch_bytes - used : 0;
  return c;
}

bool valid_batch(const crr_blob_batch* in) {
  if (!in || !in->blob_off) return false;
  if (in->n_blobs && !in->bytes) return false;
  if (reinterpret_cast<uintptr_t>(in->bytes) & 15) return false;   // the 16-byte window loads
  return true;
}

}  // namespace crr_json

extern "C" {

size_t crr_ingest_transcode_scratch_bytes(uint32_t n_blobs, uint64_t n_bytes) {
  return crr_json::carve(nullptr, n_blobs, 0).bytes + n_bytes + crr_json::kStageSlack * n_blobs;
}

int crr_ingest_transcode_plan(const crr_blob_batch* in, const uint32_t* encodings, void* scratch, size_t scratch_bytes,
                              crr_transcode_summary* summary, void* stream) {
  using namespace crr_json;
  if (!valid_batch(in) || !scratch || !summary) return -1;
  const Scratch S = carve(scratch, in->n_blobs, scratch_bytes);
  if (S.bytes > scratch_bytes) return -1;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  crr_internal::StreamDevice on_dev_(s);
  if (!on_dev_.ok) return (int)hipErrorInvalidHandle;
  const u32 nb = in->n_blobs;
  hipError_t e;
  if ((e = hipMemsetAsync(S.err, 0xff, 8, s)) != hipSuccess) return (int)e;
  if ((e = hipMemsetAsync(S.n_deep, 0, 4, s)) != hipSuccess) return (int)e;
  if ((e = hipMemsetAsync(S.off, 0, 8, s)) != hipSuccess) return (int)e;
  if (nb) {
    hipLaunchKernelGGL(blobs_kernel<M_PLAN>, dim3((nb + kBlock - 1) / kBlock), dim3(kBlock), 0, s, *in, encodings,
                       S, (u8*)nullptr);
    hipLaunchKernelGGL(deep_kernel<M_PLAN_DEEP>, dim3(kDeepThreads / kBlock), dim3(kBlock), 0, s, *in, encodings, S,
                       (u8*)nullptr);
    size_t tmp = S.scan_tmp_bytes;
    if ((e = hipcub::DeviceScan::InclusiveSum(S.scan_tmp, tmp, S.size, S.off + 1, (int)nb, s)) != hipSuccess)
      return (int)e;
  }
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  u64 err = 0, total = 0;
  u32 n_deep = 0;
  if ((e = hipMemcpyAsync(&err, S.err, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
  if ((e = hipMemcpyAsync(&total, S.off + nb, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
  if ((e = hipMemcpyAsync(&n_deep, S.n_deep, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return (int)e;
  summary->err = err == ~0ull ? 0 : -(int32_t)(err & 0xff);
  summary->reserved = 0;
  summary->err_blob = err == ~0ull ? -1 : (int64_t)(err >> 8);
  summary->n_bytes = total;
  summary->n_deep = n_deep;
  summary->reserved1 = 0;
  return 0;
}

int crr_ingest_transcode(const crr_blob_batch* in, const uint32_t* encodings, void* scratch, size_t scratch_bytes,
                         const crr_transcode_summary* summary, uint8_t* out_bytes, uint64_t* out_blob_off,
                         void* stream) {
  using namespace crr_json;
  if (!valid_batch(in) || !scratch || !summary || !out_bytes || !out_blob_off) return -1;
  if (reinterpret_cast<uintptr_t>(out_bytes) & 15) return -1;
  const Scratch S = carve(scratch, in->n_blobs, scratch_bytes);
  if (S.bytes > scratch_bytes) return -1;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  crr_internal::StreamDevice on_dev_(s);
  if (!on_dev_.ok) return (int)hipErrorInvalidHandle;
  const u32 nb = in->n_blobs;
  hipError_t e;
  // the pad the ingest's window reads past the last blob
  if ((e = hipMemsetAsync(out_bytes + summary->n_bytes, 0, CRR_INGEST_PAD, s)) != hipSuccess) return (int)e;
  if (nb) {
    const u32 gather_blocks = (nb + kBlock / 64 - 1) / (kBlock / 64);
    hipLaunchKernelGGL(gather_kernel, dim3(gather_blocks < 8192 ? gather_blocks : 8192), dim3(kBlock), 0, s, *in, S,
                       out_bytes);
    hipLaunchKernelGGL(blobs_kernel<M_WRITE>, dim3((nb + kBlock - 1) / kBlock), dim3(kBlock), 0, s, *in, encodings,
                       S, out_bytes);
    hipLaunchKernelGGL(deep_kernel<M_WRITE_DEEP>, dim3(kDeepThreads / kBlock), dim3(kBlock), 0, s, *in, encodings, S,
                       out_bytes);
  }
  if ((e = hipMemcpyAsync(out_blob_off, S.off, 8ull * (nb + 1), hipMemcpyDeviceToDevice, s)) != hipSuccess)
    return (int)e;
  return (int)hipGetLastError();
}

}  // extern "C"
