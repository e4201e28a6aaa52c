// ingest_kernel.hip -- persisted thriftrw history blobs in HBM -> the replay engine's wave-interleaved,
// tiered crr_inputs, on the GPU (include/cadence_ingest.h).
//
// The host path this restates, step for step (byte-identical output, tests/test_gpu_ingest.py):
//   cadence_amd/csrc/history_decode.cpp   the thriftrw walk (read_event / read_attributes / skip)
//   cadence_amd/csrc/host_flatten.h       WfFlattener::add / batch_end / finish (columns, side records,
//                                         interned keys, capacities, branch tokens)
//   cadence_amd/flatten.py                live_set_bounds, tier_classes, interleave, _interleave_side
//
// Pipeline (crr_ingest_plan, then crr_ingest_layout once the caller has sized its buffers):
//   1 blob_head_quick_kernel / blob_head_kernel   lane per blob: the event count from the History list
//                          header (a full walk only for a blob not in thriftrw's canonical shape)
//   2 scan                 exclusive prefixes: every blob's slice of the canonical (stride-1,
//                          workflow-order) scratch columns
//   3 blob_decode_kernel   a wavefront per 64 blobs staged in LDS, a lane per blob walking it: columns,
//                          side records and key-string references (hashes, 16-byte heads) at the events'
//                          own slots; previous reset points counted; domain_resolve_kernel then looks the
//                          domain names up in the device hash set, a lane per event
//   4 reset_refs_kernel    the previous reset points' strings at their canonical reset_keys positions
//   5 wf_pass_wave_kernel  a wavefront per workflow (<= 64 events): interning by first occurrence, side-record
//                          ordinals, capacities, VH items, tasks, live-set bounds by pairwise lane compares,
//                          tier class, sort key; wf_pass_kernel, a lane per workflow with per-workflow
//                          hash tables, takes the longer ones and those with previous reset points
//   6 radix sort (hipCUB)  device order = (long, tier | big, -length, index)
//   7 geometry             per-group maxima (one wavefront per group), prefixes over groups and the
//                          tail, tier boundaries, the summary
//   layout                 interleaved columns + side records (block per group / tail workflow),
//                          descriptors, branch tokens, reset keys
// A blob whose walk finds more events than its header announced (hand-made blobs: a second events
// list) sends the plan back to a full counting walk of every blob before decoding.
//
// Parsing is integer / byte work: in the fast pass a lane walks its blob in LDS, each field header /
// integer one unaligned 8-byte ds_read; the general pass (and the header walks) read through a 32-byte
// register window over HBM (aligned dwordx4 loads, a funnel-shift extraction per value).  No MFMA.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stddef.h>
#include <stdint.h>

#include "cadence_ingest.h"
#include "cadence_decode.h"
#include "stream_device.h"

namespace crr_ingest {

using i64 = int64_t;
using i32 = int32_t;
using u32 = uint32_t;
using u64 = uint64_t;
using u8 = uint8_t;
typedef u32 v4u __attribute__((ext_vector_type(4)));

enum : u32 { T_STOP = 0, T_BOOL = 2, T_BYTE = 3, T_DOUBLE = 4, T_I16 = 6, T_I32 = 8, T_I64 = 10, T_STRING = 11,
             T_STRUCT = 12, T_MAP = 13, T_SET = 14, T_LIST = 15 };

constexpr int kBlock = 256;
constexpr i32 kLongHistory = 256;       // flatten.LONG_HISTORY
constexpr i32 kCompactMaxEvents = 1023;  // flatten.COMPACT_MAX_EVENTS
constexpr int kWide = 5;                 // flatten.WIDE
constexpr int kMaps = 6;                 // act, timer, child, rc, sig, rp
// flatten.TIER_SLOTS (act, timer, child, rc, sig, rp)
__constant__ i32 kTierSlots[5][kMaps] = {{1, 1, 1, 1, 1, 1}, {2, 2, 1, 1, 1, 2}, {4, 3, 2, 1, 1, 4},
                                         {8, 5, 3, 3, 3, 8}, {12, 8, 6, 4, 4, 8}};
__constant__ i32 kWaveSmallTier[kMaps] = {40, 32, 16, 8, 8, 24};   // flatten.WAVE_SMALL_TIER
constexpr i32 kWaveBigCap = 64;                                     // flatten.WAVE_BIG_CAPS
// host_flatten.h kTasksPerEvent
__constant__ int8_t kTasksPerEvent[CRR_EV_TYPE_COUNT] = {
    3, 2, 2, 2, 1, 1, 0, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
    0, 2, 1, 0, 0, 0, 0, 2, 2, 1, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 1};

// ---- scratch layout ------------------------------------------------------------------------------------
struct KeyRef {     // a string to intern (an event's key or a previous reset point): where, and its hash
  u64 off;          // byte offset of the string in `bytes`
  u32 len;
  u32 hash;         // str_hash of its bytes
  u64 head[2];      // its first 16 bytes, zero-padded: a string up to 16 bytes compares without a read
};
// the Points list of a start event's PrevAutoResetPoints (kept in its key slot: Started has no key)
struct PrevRef {
  u64 pos;          // first element's byte offset
  u32 n;
  u32 et;           // element type
};

struct Plan {       // pointers into the caller's scratch (carved by carve())
  u32* blob_wf;              // [n_blobs]
  u32* cnt;                  // [2][n_blobs]: events (header count), previous reset points (decode)
  u64* off;                  // [2][n_blobs + 1] exclusive prefixes
  u64* err;                  // [1] (blob << 8) | -code, min wins
  u32* flags;                // [1] bit 0: a header count was wrong (recount)
  u64* tile;                 // scan tiles
  // canonical scratch columns [max_events]
  u8* etype; i64* id; i64* ver; i64* ts; i64* task; i64* ref; u32* key; i32* aux;
  crr_activity_side* act;    // [max_events] at the ActivityTaskScheduled event's own slot
  crr_start_side* start;     // [max_events] at the WorkflowExecutionStarted event's own slot
  KeyRef* keys;              // [max_events] a keyed event's string (a Started event's PrevRef)
  KeyRef* dom_refs;          // [max_events] domain names the fast decode left to domain_resolve_kernel
                             // (aliases `table`, which only wf_pass uses, after the resolve)
  KeyRef* resets;            // [max_events] previous reset points, canonical reset_keys order
  u32* reset_ids;            // [max_events] their interned ids (= the reset_keys array)
  u64* table;                // per-workflow hash tables [8 * max_events + 64 * n_wf]
  // per workflow (canonical order)
  i32* wf_info;              // [kWfInfo][n_wf]
  u64* sort_in; u64* sort_out;     // [n_wf]
  void* sort_tmp; size_t sort_tmp_bytes;
  u32* perm; u32* inv;       // [n_wf]
  u64* arena_off;            // [n_wf + 1]
  u64* gvals;                // [kGeo][n_groups]   group maxima
  u64* tvals;                // [kGeo][n_wf]       tail values
  u64* gpre; u64* tpre;      // their exclusive prefixes
  u32* counters;             // [16]
  u32* dom_table; u32 dom_cap;
  u32 n_blobs, n_wf;
  u64 max_events;
  // resume (crr_ingest_plan_resume): device order = the batch's, keys seeded from the loaded dictionaries
  u32 resume;
  const crr_workflow* res_wf;
  const u32* key_begin; const u32* key_count; const u64* key_off; const u32* key_len;
};
// per-workflow info words (canonical index)
enum { WI_COUNT = 0, WI_EMPTY_AT, WI_ACT, WI_TIMER, WI_CHILD, WI_RC, WI_SIG, WI_VH, WI_RP, WI_TASKS, WI_STARTED,
       WI_TIER, WI_LONG, WI_BIG, kWfInfo };
// geometry values per device position: count, 8 table caps, activity / start side counts
enum { GV_LEN = 0, GV_CAP0 = 1, GV_ACT_SIDE = 9, GV_START_SIDE = 10, kGeo = 11 };
// counters
enum { C_N_LANE = 0, C_N_BIG = 1, C_TIER0 = 2 /* .. C_TIER0 + 5 */, C_SMALL_TAIL_BAD = 8, C_NEW_RUN = 9 };

__host__ __device__ inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }
constexpr size_t kDomainBytes = 64 * 1024;   // the known-domain set (<= 8192 names)
constexpr i32 kErrScratch = -100;            // CRR_INGEST_SCRATCH_TOO_SMALL

// ---- the device's string hash (interning and the known-domain set; never leaves the ingest) -------------
// Eight little-endian bytes per step (the tail zero-padded, the length in the seed), a 32-bit
// multiply per half, a final avalanche so a table's low bits see every byte.
__device__ __forceinline__ u32 str_hash_init(u32 len) { return 2166136261u ^ (len * 0x9E3779B1u); }
__device__ __forceinline__ u32 str_hash_step(u32 h, u64 v) {
  h = (h ^ (u32)v) * 16777619u;
  return (h ^ (u32)(v >> 32)) * 16777619u;
}
__device__ __forceinline__ u32 str_hash_final(u32 h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}

// ---- byte reader over one blob: a 32-byte aligned window in registers ----------------------------------
// The window holds bytes [wb, wb + 32); any read of up to 8 bytes starting in its first half is served
// from registers.  A sequential walk shifts it by 16 bytes with one dwordx4 load.  `bytes` is readable
// 32 bytes past the last blob (cadence_ingest.h).
struct Cursor { u64 p; int err; };   // where a walk ended, and how
// the general container walk (defined after Rd): a list / set / map whose header has been read
__device__ __attribute__((noinline)) Cursor skip_nested(const u8* b, u64 p, u64 end, u32 kind, u32 kt, u32 vt,
                                                        i32 n, int d0);

// The reader, in two builds: RdT<true> walks any value; RdT<false> (the decode's fast pass) has no call
// in it -- a container holding structs or containers stops the walk with kDeferGeneral, and the blob is
// decoded again by the general build (blob_decode_general_kernel).  A call would put the whole walk
// state (reader, event) in scratch memory.
constexpr int kDeferGeneral = -90;
constexpr u32 kDeferMark = 0xFFFFFFFFu;   // cnt[1][blob] of a deferred blob, until the general pass
// L: reads come from an LDS copy of the bytes [base, ...) (blob_decode_kernel stages each wavefront's
// blobs there with coalesced loads), 8 unaligned bytes per ds_read_b64 and no register window; positions
// stay offsets into `bytes`.
typedef const u8 __attribute__((address_space(3))) lds_u8;
typedef const v4u __attribute__((address_space(3))) lds_v4u;
template <bool G, bool L = false>
struct RdT {
  const u8* b;
  lds_u8* lb;        // L: the staged copy, lb[0] = bytes[base]
  u64 base;
  u64 p, end;
  u64 wb;            // window base (16-aligned), ~0: none
  v4u w0, w1;     // native vectors: HIP's uint4 struct is copied by memcpy, which keeps the reader in scratch
  int err;           // CRR_DECODE_* (0 ok)

  __device__ __forceinline__ void init(const u8* bytes, u64 begin, u64 e) {
    b = bytes; lb = nullptr; base = 0; p = begin; end = e; wb = ~0ull; err = 0;
  }
  __device__ __forceinline__ void init_staged(const u8* bytes, lds_u8* staged, u64 staged_base, u64 begin, u64 e) {
    init(bytes, begin, e);
    lb = staged; base = staged_base;
  }
  __device__ __forceinline__ v4u ld16(u64 a) const {
    if constexpr (L) return *reinterpret_cast<lds_v4u*>(lb + (u32)(a - base));
    else return *reinterpret_cast<const v4u*>(b + a);
  }
  __device__ __forceinline__ bool need(u64 n) {
    if (err) return false;
    if (end - p < n) { err = CRR_DECODE_TRUNCATED; return false; }
    return true;
  }
  // bytes q .. q+7 in memory order (little-endian u64)
  __device__ __forceinline__ u64 peek8(u64 q) {
    if constexpr (L) {   // LDS serves unaligned 8-byte reads (ds_read_b64): no window to carry
      u64 v;
      __builtin_memcpy(&v, (const void*)(lb + (u32)(q - base)), 8);
      return v;
    } else if constexpr (!G) {   // the fast pass's rare blob larger than the LDS window: unaligned loads
      u64 v;
      __builtin_memcpy(&v, b + q, 8);
      return v;
    }
    const u64 a = q & ~15ull;
    if (a != wb) {
      if (a == wb + 16) {
        w0 = w1;
      } else {
        w0 = ld16(a);
      }
      w1 = ld16(a + 16);
      wb = a;
    }
    // dwords k, k+1, k+2 of the window (k = o / 4) by two bit-selects, then the byte shift: no dynamic
    // index into the window (the compiler would spill it to scratch to index it)
    const u32 o = (u32)(q & 15);
    const bool h8 = (o & 8) != 0, h4 = (o & 4) != 0;
    const u32 a0 = h8 ? w0.z : w0.x, a1 = h8 ? w0.w : w0.y, a2 = h8 ? w1.x : w0.z, a3 = h8 ? w1.y : w0.w;
    const u32 x0 = h4 ? a1 : a0, x1 = h4 ? a2 : a1, x2 = h4 ? a3 : a2;
    const u32 lo = __builtin_amdgcn_alignbyte(x1, x0, o & 3);
    const u32 hi = __builtin_amdgcn_alignbyte(x2, x1, o & 3);
    return ((u64)hi << 32) | lo;
  }
  __device__ __forceinline__ u32 u8_() {
    if (!need(1)) return 0;
    return (u32)peek8(p++) & 0xff;
  }
  __device__ __forceinline__ i32 be16() {
    if (!need(2)) return 0;
    const u32 v = (u32)peek8(p);
    p += 2;
    return (i32)(int16_t)(((v & 0xff) << 8) | ((v >> 8) & 0xff));
  }
  __device__ __forceinline__ i32 be32() {
    if (!need(4)) return 0;
    const u32 v = (u32)peek8(p);
    p += 4;
    return (i32)__builtin_bswap32(v);
  }
  __device__ __forceinline__ i64 be64() {
    if (!need(8)) return 0;
    const u64 v = peek8(p);
    p += 8;
    return (i64)__builtin_bswap64(v);
  }
  // a struct's next field header (type byte, then big-endian i16 id); false at the stop byte or an error
  __device__ __forceinline__ bool field(u32& ft, i32& id) {
    if (!need(1)) return false;
    const u32 v = (u32)peek8(p);
    ft = v & 0xff;
    if (ft == T_STOP) { ++p; return false; }
    if (!need(3)) return false;
    id = (i32)(int16_t)(((v >> 8) & 0xff) << 8 | ((v >> 16) & 0xff));
    p += 3;
    return true;
  }
  // a thrift string: its (offset, length) in the blob bytes
  __device__ __forceinline__ void str(u64& off, u32& len) {
    const i32 n = be32();
    if (err) return;
    if (n < 0) { err = CRR_DECODE_TRUNCATED; return; }
    if (!need((u64)n)) return;
    off = p;
    len = (u32)n;
    p += (u64)n;
  }
  // a string's KeyRef (len > 0): where, its hash and its first 16 bytes, through the window
  __device__ __forceinline__ u64 head8(u64 off, u32 len) {   // bytes [off, off + min(len, 8)), zero-padded
    const u64 v = peek8(off);
    return len < 8 ? v & ((1ull << (8 * len)) - 1) : v;
  }
  __device__ __forceinline__ KeyRef key_ref(u64 off, u32 len) {
    KeyRef k;
    k.off = off; k.len = len; k.hash = 0; k.head[0] = 0; k.head[1] = 0;
    if (len == 0) return k;
    k.hash = hash(off, len);
    k.head[0] = head8(off, len);
    if (len > 8) k.head[1] = head8(off + 8, len - 8);
    return k;
  }
  // str_hash of bytes [off, off + len) through the window (the string was just walked past)
  __device__ __forceinline__ u32 hash(u64 off, u32 len) {
    u32 h = str_hash_init(len);
    for (u32 i = 0; i < len; i += 8) {
      const u64 v = peek8(off + i);
      h = str_hash_step(h, len - i < 8 ? v & ((1ull << (8 * (len - i))) - 1) : v);
    }
    return str_hash_final(h);
  }
  // skip one value of `type` (history_decode.cpp Reader::skip: a value nested deeper than 64 is
  // BAD_TYPE).  Inline: scalars, strings, structs (a count of open structs) and lists / sets / maps of
  // scalars or strings -- every skipped field of the events Cadence writes; a container holding structs
  // or containers goes out of line to skip_nested (whose level stack lives in scratch).  Nothing here
  // may take the reader's address: the walk state stays in registers.
  __device__ __forceinline__ void skip(u32 type) {
    u32 t = type;
    int open = 0;   // open structs: the value about to be skipped sits at this depth
    for (;;) {
      if (err) return;
      if (open > 64) { err = CRR_DECODE_BAD_TYPE; return; }
      if (t == T_STRUCT) ++open;
      else if (t == T_MAP || t == T_SET || t == T_LIST) skip_container(t, open);
      else skip_leaf(t);
      if (err) return;
      // the innermost open struct's next field, closing finished ones
      for (;;) {
        if (open == 0) return;
        i32 id;
        if (field(t, id)) break;
        if (err) return;
        --open;
      }
    }
  }
  __device__ __forceinline__ static bool leaf(u32 t) {
    return t == T_BOOL || t == T_BYTE || t == T_I16 || t == T_I32 || t == T_I64 || t == T_DOUBLE || t == T_STRING;
  }
  __device__ __forceinline__ void skip_leaf(u32 t) {
    switch (t) {
      case T_BOOL: case T_BYTE: if (need(1)) p += 1; break;
      case T_I16: if (need(2)) p += 2; break;
      case T_I32: if (need(4)) p += 4; break;
      case T_DOUBLE: case T_I64: if (need(8)) p += 8; break;
      case T_STRING: {
        const i32 n = be32();
        if (err) return;
        if (n < 0) { err = CRR_DECODE_TRUNCATED; return; }
        if (need((u64)n)) p += (u64)n;
        break;
      }
      default: err = CRR_DECODE_BAD_TYPE;
    }
  }
  // a list / set / map value at depth d0: its header, then its elements at depth d0 + 1 (a map's keys
  // and values alternate)
  __device__ __forceinline__ void skip_container(u32 t, int d0) {
    const u32 kt = u8_();
    const u32 vt = t == T_MAP ? u8_() : kt;
    const i32 n = be32();
    if (err) return;
    if (n < 0) { err = CRR_DECODE_TRUNCATED; return; }
    if (n == 0) return;
    if (!leaf(kt) || !leaf(vt)) {
      if constexpr (G) {
        const Cursor c = skip_nested(b, p, end, t == T_MAP ? T_MAP : T_LIST, kt, vt, n, d0);
        p = c.p;
        err = c.err;
      } else {
        err = kDeferGeneral;
      }
      return;
    }
    if (d0 + 1 > 64) { err = CRR_DECODE_BAD_TYPE; return; }
    const u64 m = t == T_MAP ? 2 * (u64)n : (u64)n;
    for (u64 i = 0; i < m && !err; ++i) skip_leaf((i & 1) ? vt : kt);
  }
  __device__ __forceinline__ bool want(u32 got, u32 expect) {   // Reader::want
    if (got == expect) return true;
    skip(got);
    return false;
  }
};
using Rd = RdT<true>;

// Rd::skip's general container walk: the value (a list / set / map whose header was just read, at depth
// d0) and everything inside it, levels on a stack (history_decode.cpp Reader::skip).  Out of line so its
// stack lives in this function's own scratch frame, not in every walk's registers.
__device__ __attribute__((noinline)) Cursor skip_nested(const u8* b, u64 p, u64 end, u32 kind, u32 kt, u32 vt,
                                                        i32 n, int d0) {
  struct Lvl { u8 kind, t1, t2, pad; i32 rem; };
  Lvl st[66];
  Rd r;
  r.init(b, p, end);
  st[0] = Lvl{(u8)kind, (u8)kt, (u8)vt, 0, kind == T_MAP ? 2 * n : n};
  int d = d0 + 1;   // depth of the next value
  u32 t = 0;
  for (;;) {
    // the next value: the innermost open level's next field / element, closing finished levels
    for (;;) {
      if (d == d0) return Cursor{r.p, r.err};
      Lvl& L = st[d - 1 - d0];
      if (L.kind == T_STRUCT) {
        i32 id;
        if (r.field(t, id)) break;
        if (r.err) return Cursor{r.p, r.err};
        --d;
        continue;
      }
      if (L.rem == 0) { --d; continue; }
      t = (L.kind == T_MAP && (L.rem & 1) == 0) ? L.t1 : L.t2;
      if (L.kind != T_MAP) t = L.t1;
      --L.rem;
      break;
    }
    if (d > 64) { r.err = CRR_DECODE_BAD_TYPE; return Cursor{r.p, r.err}; }
    switch (t) {
      case T_STRUCT: st[d - d0] = Lvl{T_STRUCT, 0, 0, 0, 0}; ++d; break;
      case T_MAP: {
        const u32 k1 = r.u8_(), v1 = r.u8_();
        const i32 m = r.be32();
        if (r.err) return Cursor{r.p, r.err};
        if (m < 0) return Cursor{r.p, CRR_DECODE_TRUNCATED};
        st[d - d0] = Lvl{T_MAP, (u8)k1, (u8)v1, 0, 2 * m};
        ++d;
        break;
      }
      case T_SET: case T_LIST: {
        const u32 et = r.u8_();
        const i32 m = r.be32();
        if (r.err) return Cursor{r.p, r.err};
        if (m < 0) return Cursor{r.p, CRR_DECODE_TRUNCATED};
        st[d - d0] = Lvl{T_LIST, (u8)et, (u8)et, 0, m};
        ++d;
        break;
      }
      default: r.skip_leaf(t);
    }
    if (r.err) return Cursor{r.p, r.err};
  }
}

// The fields of one event ApplyEvents reads (host_flatten.h Attr / Event), strings as blob references.
struct Attr {
  i64 ref;
  i32 aux;
  u64 key_off; u32 key_len;
  u64 dom_off; u32 dom_len;
  i32 s2s, s2c, st2c, hb, has_retry, expiration;
  i32 task_s2c, exec_s2c, backoff, initiator, attempt;
  i64 expiration_ts;
  i32 prev_mode;       // -1 nil, -2 Points nil, 0 list
  u64 prev_pos;        // the final Points list: first element's byte offset, count, element type
  i32 prev_n;
  u32 prev_et;
};
struct Event {
  i64 id, ts, ver, task;
  i32 type;
  Attr a;
};

__device__ __forceinline__ void attr_init(Attr& a) {
  a.ref = 0; a.aux = 0; a.key_off = 0; a.key_len = 0; a.dom_off = 0; a.dom_len = 0;
  a.s2s = a.s2c = a.st2c = a.hb = a.has_retry = a.expiration = 0;
  a.task_s2c = a.exec_s2c = a.backoff = 0; a.initiator = CRR_INITIATOR_NIL; a.attempt = 0;
  a.expiration_ts = 0; a.prev_mode = -1; a.prev_pos = 0; a.prev_n = 0; a.prev_et = 0;
}

__device__ __forceinline__ int attr_type_of_field(i32 id) {
  if (id < 40 || id > 450 || id % 10) return -1;
  return (id - 40) / 10;
}

// RetryPolicy{60 ExpirationIntervalInSeconds i32} (Reader::want: a wrong-typed field 60 is skipped)
template <bool G>
__device__ __forceinline__ void read_retry_policy(RdT<G>& r, Attr& a) {
  a.has_retry = 1;
  u32 ft;
  i32 id;
  while (r.field(ft, id)) {
    if (id == 60 && ft == T_I32) a.expiration = r.be32();
    else r.skip(ft);
  }
}

// ResetPoints{10 Points list<ResetPointInfo{10 BinaryChecksum}>}: only the final list's position is
// kept; its strings are read once the event is complete (WfFlattener::add interns them there).  Out of
// reader of its own, result by value.
struct PrevPoints { u64 p; u64 pos; i32 err, mode, n; u32 et; };
template <class R>
__device__ __forceinline__ PrevPoints walk_reset_points(R r) {
  PrevPoints o{0, 0, 0, -2, 0, 0};
  u32 ft;
  i32 id;
  while (r.field(ft, id)) {
    if (id == 10 && ft == T_LIST) {
      const u32 et = r.u8_();
      const i32 n = r.be32();
      if (r.err) break;
      if (n < 0) { r.err = CRR_DECODE_TRUNCATED; break; }
      o.mode = 0;
      o.pos = r.p;
      o.n = n;
      o.et = et;
      for (i32 i = 0; i < n && !r.err; ++i) {
        if (et != T_STRUCT) { r.skip(et); continue; }
        u32 t2;
        i32 id2;
        while (r.field(t2, id2)) {
          if (id2 == 10 && t2 == T_STRING) { u64 so; u32 sl; r.str(so, sl); }
          else r.skip(t2);
        }
      }
    } else {
      r.skip(ft);
    }
  }
  o.p = r.p;
  o.err = r.err;
  return o;
}
template <bool G>
__device__ __forceinline__ PrevPoints read_reset_points(const u8* b, u64 p, u64 end) {
  RdT<G> r;
  r.init(b, p, end);
  return walk_reset_points(r);
}

// history_decode.cpp read_attributes
template <bool G>
__device__ __forceinline__ void read_attributes(RdT<G>& r, int t, Attr& a) {
  u32 ft;
  i32 id;
  while (r.field(ft, id)) {
    bool used = true;
    switch (t) {
      case CRR_EV_WORKFLOW_EXECUTION_STARTED:
        if (id == 12 && ft == T_STRING) r.str(a.dom_off, a.dom_len);
        else if (id == 40 && ft == T_I32) a.exec_s2c = r.be32();
        else if (id == 50 && ft == T_I32) a.task_s2c = r.be32();
        else if (id == 55 && ft == T_I32) a.initiator = r.be32();
        else if (id == 80 && ft == T_I32) a.attempt = r.be32();
        else if (id == 90 && ft == T_I64) a.expiration_ts = r.be64();
        else if (id == 110 && ft == T_I32) a.backoff = r.be32();
        else if (id == 130 && ft == T_STRUCT) {
          const PrevPoints q = read_reset_points<G>(r.b, r.p, r.end);
          r.p = q.p;
          r.err = q.err;
          a.prev_mode = q.mode; a.prev_pos = q.pos; a.prev_n = q.n; a.prev_et = q.et;
        }
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_SCHEDULED:
        if (id == 20 && ft == T_I32) a.aux = r.be32();
        else if (id == 30 && ft == T_I64) a.ref = r.be64();
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_STARTED:
        if (id == 10 && ft == T_I64) a.ref = r.be64(); else used = false;
        break;
      case CRR_EV_DECISION_TASK_COMPLETED:
        if (id == 30 && ft == T_I64) a.ref = r.be64();
        else if (id == 50 && ft == T_STRING) r.str(a.key_off, a.key_len);
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_TIMED_OUT:
        if (id == 30 && ft == T_I32) a.aux = r.be32(); else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_SCHEDULED:
        if (id == 10 && ft == T_STRING) r.str(a.key_off, a.key_len);
        else if (id == 25 && ft == T_STRING) r.str(a.dom_off, a.dom_len);
        else if (id == 45 && ft == T_I32) a.s2c = r.be32();
        else if (id == 50 && ft == T_I32) a.s2s = r.be32();
        else if (id == 55 && ft == T_I32) a.st2c = r.be32();
        else if (id == 60 && ft == T_I32) a.hb = r.be32();
        else if (id == 110 && ft == T_STRUCT) read_retry_policy(r, a);
        else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_STARTED:
      case CRR_EV_ACTIVITY_TASK_TIMED_OUT:
        if (id == 10 && ft == T_I64) a.ref = r.be64(); else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_COMPLETED:
        if (id == 20 && ft == T_I64) a.ref = r.be64(); else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_FAILED:
      case CRR_EV_ACTIVITY_TASK_CANCELED:
        if (id == 30 && ft == T_I64) a.ref = r.be64(); else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED:
      case CRR_EV_TIMER_FIRED:
      case CRR_EV_TIMER_CANCELED:
        if (id == 10 && ft == T_STRING) r.str(a.key_off, a.key_len); else used = false;
        break;
      case CRR_EV_TIMER_STARTED:
        if (id == 10 && ft == T_STRING) r.str(a.key_off, a.key_len);
        else if (id == 20 && ft == T_I64) a.ref = r.be64();
        else used = false;
        break;
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED:
        if (id == 10 && ft == T_STRING) r.str(a.dom_off, a.dom_len); else used = false;
        break;
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED:
      case CRR_EV_SIGNAL_EXTERNAL_INITIATED:
        if (id == 20 && ft == T_STRING) r.str(a.dom_off, a.dom_len); else used = false;
        break;
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED:
        if (id == 60 && ft == T_I64) a.ref = r.be64(); else used = false;
        break;
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED:
        if (id == 20 && ft == T_I64) a.ref = r.be64(); else used = false;
        break;
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT:
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED:
      case CRR_EV_SIGNAL_EXTERNAL_FAILED:
        if (id == 50 && ft == T_I64) a.ref = r.be64(); else used = false;
        break;
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED:
        if (id == 40 && ft == T_I64) a.ref = r.be64(); else used = false;
        break;
      case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED:
      case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED:
        if (id == 10 && ft == T_I64) a.ref = r.be64(); else used = false;
        break;
      default:
        used = false;
    }
    if (!used) r.skip(ft);
  }
}

// history_decode.cpp read_event: an attribute struct that arrives before the type is re-read after it.
// One read_attributes site and one skip site (each is a large inline body).
template <bool G>
__device__ __forceinline__ void read_event(RdT<G>& r, Event& e) {
  e.id = e.ts = e.ver = e.task = 0;
  e.type = 0;
  attr_init(e.a);
  u64 attr_at = 0, resume = 0;
  int attr_t = -1;     // the last attribute struct seen before the type: its type (and attr_at its bytes)
  bool have_type = false, last = false;
  u32 ft;
  i32 id;
  for (;;) {
    int at = -1;
    if (!r.field(ft, id)) {
      if (r.err || attr_t < 0 || attr_t != e.type) return;
      resume = r.p;               // re-read the early attributes, then leave the reader at the stop byte
      r.p = attr_at;
      at = attr_t;
      last = true;
    } else if (id == 10 && ft == T_I64) { e.id = r.be64(); continue; }
    else if (id == 20 && ft == T_I64) { e.ts = r.be64(); continue; }
    else if (id == 30 && ft == T_I32) { e.type = r.be32(); have_type = true; continue; }
    else if (id == 35 && ft == T_I64) { e.ver = r.be64(); continue; }
    else if (id == 36 && ft == T_I64) { e.task = r.be64(); continue; }
    else {
      const int ty = ft == T_STRUCT ? attr_type_of_field(id) : -1;
      if (ty >= 0 && have_type && ty == e.type) {
        at = ty;
      } else {
        if (ty >= 0 && !have_type) { attr_at = r.p; attr_t = ty; }
        r.skip(ft);
        if (r.err) return;
        continue;
      }
    }
    read_attributes(r, at, e.a);
    if (r.err) return;
    if (last) { r.p = resume; return; }
  }
}

__device__ __forceinline__ bool keyed_type(i32 t) {
  return t == CRR_EV_DECISION_TASK_COMPLETED || t == CRR_EV_ACTIVITY_TASK_SCHEDULED ||
         t == CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED || t == CRR_EV_TIMER_STARTED || t == CRR_EV_TIMER_FIRED ||
         t == CRR_EV_TIMER_CANCELED;
}

__device__ __forceinline__ u32 str_hash_bytes(const u8* b, u64 off, u32 len) {   // (known domain names)
  u32 h = str_hash_init(len);
  for (u32 i = 0; i < len; i += 8) {
    u64 v = 0;
    for (u32 j = 0; j < 8 && i + j < len; ++j) v |= (u64)b[off + i + j] << (8 * j);
    h = str_hash_step(h, v);
  }
  return str_hash_final(h);
}

// ---- domain-cache stand-in: the known domain names as an open-addressed set -----------------------------
__device__ __forceinline__ bool bytes_equal(const u8* a, u64 ao, const u8* b, u64 bo, u32 n) {
  u32 d = 0;   // no early exit: the byte loads are independent, not a chain of round trips
  for (u32 i = 0; i < n; ++i) d |= (u32)(a[ao + i] ^ b[bo + i]);
  return d == 0;
}

__global__ void domains_build_kernel(crr_blob_batch in, u32* table, u32 cap) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= in.n_domains) return;
  u32 h = str_hash_bytes(in.strings, in.domain_off[i], in.domain_len[i]) & (cap - 1);
  for (u32 probe = 0; probe < cap; ++probe) {
    const u32 prev = atomicCAS(table + h, 0u, i + 1);
    if (prev == 0) return;
    h = (h + 1) & (cap - 1);
  }
}

// WfFlattener::domain_status
__device__ __forceinline__ i32 domain_status(const crr_blob_batch& in, const u32* table, u32 cap, u64 off, u32 len) {
  if (len == 0) return CRR_DOMAIN_NOT_SET;
  if (in.n_domains == 0xFFFFFFFFu) return CRR_DOMAIN_RESOLVED;
  if (cap == 0) return CRR_DOMAIN_UNKNOWN;
  u32 h = str_hash_bytes(in.bytes, off, len) & (cap - 1);
  for (u32 probe = 0; probe < cap; ++probe) {
    const u32 e = table[h];
    if (e == 0) return CRR_DOMAIN_UNKNOWN;
    const u32 d = e - 1;
    if (in.domain_len[d] == len && bytes_equal(in.bytes, off, in.strings, in.domain_off[d], len)) return CRR_DOMAIN_RESOLVED;
    h = (h + 1) & (cap - 1);
  }
  return CRR_DOMAIN_UNKNOWN;
}

// the same, the name's str_hash already computed (through the reader's window)
__device__ __forceinline__ i32 domain_status_h(const crr_blob_batch& in, const u32* table, u32 cap, u64 off, u32 len,
                                               u32 hash) {
  if (len == 0) return CRR_DOMAIN_NOT_SET;
  if (in.n_domains == 0xFFFFFFFFu) return CRR_DOMAIN_RESOLVED;
  if (cap == 0) return CRR_DOMAIN_UNKNOWN;
  u32 h = hash & (cap - 1);
  for (u32 probe = 0; probe < cap; ++probe) {
    const u32 e = table[h];
    if (e == 0) return CRR_DOMAIN_UNKNOWN;
    const u32 d = e - 1;
    if (in.domain_len[d] == len && bytes_equal(in.bytes, off, in.strings, in.domain_off[d], len)) return CRR_DOMAIN_RESOLVED;
    h = (h + 1) & (cap - 1);
  }
  return CRR_DOMAIN_UNKNOWN;
}

// The fast decode's domain lookups: the constant outcomes at once, a lookup in the known-domain set
// deferred (the name's reference kept at the event's slot, kDomainPending in the field) to
// domain_resolve_kernel, a lane per event -- so no walk waits on the set's round trips.
constexpr i32 kDomainPending = 0x7FFF0D0D;
template <class R>
__device__ __forceinline__ i32 domain_fast(R& r, const crr_blob_batch& in, const Plan& P, u64 x, u64 off, u32 len) {
  if (len == 0) return CRR_DOMAIN_NOT_SET;
  if (in.n_domains == 0xFFFFFFFFu) return CRR_DOMAIN_RESOLVED;
  if (P.dom_cap == 0) return CRR_DOMAIN_UNKNOWN;
  KeyRef d;
  d.off = off; d.len = len; d.hash = r.hash(off, len); d.head[0] = 0; d.head[1] = 0;
  P.dom_refs[x] = d;
  return kDomainPending;
}

// every blob decoded and the canonical scratch large enough: the later passes may read it
__device__ __forceinline__ bool plan_ok(const Plan& P) {
  const u64 NB = (u64)P.n_blobs + 1;
  return *P.err == ~0ull && *P.flags == 0 && P.off[0 * NB + P.n_blobs] <= P.max_events &&
         P.off[1 * NB + P.n_blobs] <= P.max_events;
}

__device__ __forceinline__ void record_error(u64* err, u32 blob, int code) {
  atomicMin((unsigned long long*)err, ((u64)blob << 8) | (u64)(-code));
}

// ---- 1: blob -> workflow, and each blob's event count ----------------------------------------------------
__global__ void blob_wf_kernel(crr_blob_batch in, u32* blob_wf, u64* err) {
  const u32 w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= in.n_wf) return;
  const crr_blob_wf s = in.wf[w];
  for (u32 b = 0; b < s.blob_count && s.blob_begin + b < in.n_blobs; ++b) blob_wf[s.blob_begin + b] = w;
  // the consecutive-ranges contract (cadence_ingest.h); a violation fails the plan
  const u32 expect = w == 0 ? 0u : in.wf[w - 1].blob_begin + in.wf[w - 1].blob_count;
  if (s.blob_begin != expect || (w + 1 == in.n_wf && s.blob_begin + s.blob_count != in.n_blobs))
    atomicMin((unsigned long long*)err, (u64)(-CRR_DECODE_BAD_ARGUMENT));
}

// the History struct's event lists: the whole walk, counting (the shape thriftrw does not write)
__device__ u32 count_events(Rd& r) {
  u32 n_ev = 0;
  u32 ft;
  i32 id;
  while (r.field(ft, id)) {
    if (id != 10 || ft != T_LIST) { r.skip(ft); continue; }
    const u32 et = r.u8_();
    const i32 n = r.be32();
    if (r.err) break;
    if (n < 0) { r.err = CRR_DECODE_TRUNCATED; break; }
    if (et != T_STRUCT && n > 0) { r.err = CRR_DECODE_BAD_TYPE; break; }
    for (i32 i = 0; i < n && !r.err; ++i) {
      r.skip(T_STRUCT);
      ++n_ev;
    }
  }
  return n_ev;
}

// Events per blob.  thriftrw writes History{10: list<HistoryEvent>} as its only field, so the count is
// the list header's: 0x59, 0x0F 0x00 0x0A, 0x0C, be32 n (bounded by the bytes after it: a corrupt
// count must not size the scratch; the decode finds the truncation).  Any other shape, or FULL (the
// recount after a header was wrong), walks the blob.
// blob_head_quick_kernel takes the canonical headers with two unaligned loads and leaves kHeadWalk for
// blob_head_kernel, which walks the rest (every blob when FULL).
constexpr u32 kHeadWalk = 0xFFFFFFFFu;
__global__ __launch_bounds__(kBlock) void blob_head_quick_kernel(crr_blob_batch in, Plan P) {
  const u32 bi = blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= in.n_blobs) return;
  const u64 b0 = in.blob_off[bi], b1 = in.blob_off[bi + 1];
  u32 n = 0;
  if (b1 > b0) {
    u64 h = 0;
    u32 c = 0;
    __builtin_memcpy(&h, in.bytes + b0, 8);   // readable: 32 bytes past the last blob
    __builtin_memcpy(&c, in.bytes + b0 + 5, 4);
    if ((h & 0xFFFFFFFFFFull) == 0x0C0A000F59ull && b1 - b0 >= 9) {
      const i64 cn = (i32)__builtin_bswap32(c);
      const i64 room = (i64)(b1 - b0 - 9);
      n = cn < 0 ? 0u : (u32)(cn < room ? cn : room);
    } else {
      n = kHeadWalk;
    }
  }
  P.cnt[bi] = n;
}

__global__ void blob_head_kernel(crr_blob_batch in, Plan P, int full) {
  const u32 bi = blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= in.n_blobs) return;
  if (!full && P.cnt[bi] != kHeadWalk) return;   // blob_head_quick_kernel's
  const u64 b0 = in.blob_off[bi], b1 = in.blob_off[bi + 1];
  u32 n = 0;
  if (b1 > b0) {
    Rd r;
    r.init(in.bytes, b0, b1);
    const u64 h = r.peek8(b0);
    const bool canonical = (h & 0xFFFFFFFFFFull) == 0x0C0A000F59ull && b1 - b0 >= 9;
    if (canonical && !full) {
      const i64 c = (i32)__builtin_bswap32((u32)(r.peek8(b0 + 5)));
      const i64 room = (i64)(b1 - b0 - 9);
      n = c < 0 ? 0u : (u32)(c < room ? c : room);
    } else if (r.u8_() == 0x59) {
      n = count_events(r);   // errors are the decode's to report
    }
  }
  P.cnt[bi] = n;
}

// ---- 3: the decode -----------------------------------------------------------------------------------------
// One blob, one walk: each event into its canonical slot (history_decode.cpp decode_workflow's loop,
// host_flatten.h WfFlattener::add's per-type columns); side records and key strings at the event's own
// slot (wf_pass numbers them within the workflow); a Started event's PrevAutoResetPoints list position
// in its key slot, the list's length counted per blob.
template <bool G>
__device__ __forceinline__ void decode_blob(const crr_blob_batch& in, const Plan& P, u32 bi) {
  const u64 b0 = in.blob_off[bi], b1 = in.blob_off[bi + 1];
  const u64 NB = (u64)P.n_blobs + 1;
  u64 x = P.off[0 * NB + bi];
  const u64 x_end = P.off[0 * NB + bi + 1];
  u32 n_prev = 0;
  if (b1 > b0) {
    RdT<G> r;
    r.init(in.bytes, b0, b1);
    if (r.u8_() != 0x59) { record_error(P.err, bi, CRR_DECODE_BAD_PREAMBLE); return; }  // version0Thriftrw.go:53-58
    const i32 new_run = in.wf[P.blob_wf[bi]].new_run_wf;
    const u64 x_first = x;
    Event e;
    u32 ft;
    i32 fid;
    while (r.field(ft, fid)) {
      if (fid != 10 || ft != T_LIST) { r.skip(ft); continue; }
      const u32 et = r.u8_();
      const i32 n = r.be32();
      if (r.err) break;
      if (n < 0) { r.err = CRR_DECODE_TRUNCATED; break; }
      if (et != T_STRUCT && n > 0) { r.err = CRR_DECODE_BAD_TYPE; break; }
      for (i32 i = 0; i < n; ++i) {
        read_event(r, e);
        if (r.err) break;
        if (x >= x_end) {   // more events than the header announced: the plan recounts
          atomicOr(P.flags, 1u);
          return;
        }
        const i32 t = e.type;
        const bool valid = t >= 0 && t < CRR_EV_TYPE_COUNT;
        const Attr& a = e.a;
        P.etype[x] = (u8)(valid ? t : CRR_EV_PAD - 1);
        P.id[x] = e.id; P.ver[x] = e.ver; P.ts[x] = e.ts; P.task[x] = e.task;
        i64 ref = 0;
        i32 aux = 0;
        switch (valid ? t : -1) {
          case CRR_EV_WORKFLOW_EXECUTION_STARTED: {
            crr_start_side ss;
            ss.decision_start_to_close = a.task_s2c;
            ss.workflow_timeout = a.exec_s2c;
            ss.first_decision_backoff = a.backoff;
            ss.initiator = a.initiator;
            ss.parent_domain_status = domain_status(in, P.dom_table, P.dom_cap, a.dom_off, a.dom_len);
            ss.attempt = a.attempt;
            ss.expiration_ns = a.expiration_ts;
            ss.refresh_jitter = 0;
            // prev_reset_key_off: the blob-local index of the first point until wf_pass adds the blob's
            // prefix (for an empty list too: where the next point would go, host_flatten.h)
            ss.prev_reset_key_off = n_prev;
            ss.prev_reset_count = a.prev_mode == 0 ? a.prev_n : a.prev_mode;
            if (a.prev_mode == 0) {
              PrevRef pr;
              pr.pos = a.prev_pos; pr.n = (u32)a.prev_n; pr.et = a.prev_et;
              *reinterpret_cast<PrevRef*>(P.keys + x) = pr;
              n_prev += (u32)a.prev_n;
            }
            P.start[x] = ss;
            break;
          }
          case CRR_EV_DECISION_TASK_SCHEDULED: ref = a.ref; aux = a.aux; break;
          case CRR_EV_DECISION_TASK_STARTED: ref = a.ref; break;
          case CRR_EV_DECISION_TASK_COMPLETED: ref = a.ref; break;
          case CRR_EV_DECISION_TASK_TIMED_OUT: aux = a.aux; break;
          case CRR_EV_ACTIVITY_TASK_SCHEDULED: {
            crr_activity_side as;
            as.schedule_to_start = a.s2s; as.schedule_to_close = a.s2c; as.start_to_close = a.st2c;
            as.heartbeat = a.hb; as.has_retry_policy = a.has_retry; as.expiration_interval = a.expiration;
            as.domain_status = domain_status(in, P.dom_table, P.dom_cap, a.dom_off, a.dom_len);
            as.reserved = 0;
            P.act[x] = as;
            break;
          }
          case CRR_EV_ACTIVITY_TASK_STARTED: case CRR_EV_ACTIVITY_TASK_COMPLETED: case CRR_EV_ACTIVITY_TASK_FAILED:
          case CRR_EV_ACTIVITY_TASK_TIMED_OUT: case CRR_EV_ACTIVITY_TASK_CANCELED:
            ref = a.ref; break;
          case CRR_EV_TIMER_STARTED: ref = a.ref; break;
          case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED:
          case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED:
          case CRR_EV_SIGNAL_EXTERNAL_INITIATED:
            aux = domain_status(in, P.dom_table, P.dom_cap, a.dom_off, a.dom_len);
            break;
          case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED:
          case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED:
          case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT:
          case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED: case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED:
          case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED: case CRR_EV_SIGNAL_EXTERNAL_FAILED:
          case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED:
            ref = a.ref; break;
          case CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW: aux = new_run; break;
          default: break;
        }
        if (valid && keyed_type(t)) {   // "" when the attribute is absent (key 0)
          const KeyRef kr = r.key_ref(a.key_off, a.key_len);
          P.keys[x] = kr;
        }
        P.ref[x] = ref;
        P.key[x] = 0;
        P.aux[x] = aux;
        ++x;
      }
      if (r.err) break;
    }
    if (r.err == kDeferGeneral) {   // the general pass decodes this blob again, from its start
      P.cnt[1 * (u64)P.n_blobs + bi] = kDeferMark;
      return;
    }
    if (r.err) { record_error(P.err, bi, r.err); return; }
    if (x > x_first) {   // batch boundaries
      P.etype[x_first] |= CRR_ETYPE_BATCH_FIRST;
      P.etype[x - 1] |= CRR_ETYPE_BATCH_LAST;
    }
  }
  if (x != x_end) atomicOr(P.flags, 1u);   // fewer events than the header announced: recount
  P.cnt[1 * (u64)P.n_blobs + bi] = n_prev;
}


// ---- 3a: the fast pass -------------------------------------------------------------------------------------
// thriftrw's own shape -- every struct's fields in increasing id order, an event's type before its
// attributes, no more events than the header announced -- with each value stored to its column / side
// record as it is read (defaults first, at the type), so the walk keeps only the reader and a few counters
// in registers.  Anything else (and a container of structs) defers the blob to the general pass, which
// is decode_blob<true>: the same results for these blobs, by construction the same walk.
enum : u32 { S_ID = 1, S_TS = 2, S_VER = 4, S_TASK = 8, S_REF = 16, S_AUX = 32 };

__device__ __forceinline__ bool domain_aux_type(i32 t) {
  return t == CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED || t == CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED ||
         t == CRR_EV_SIGNAL_EXTERNAL_INITIATED;
}

// the attribute fields read_attributes takes, stored where decode_blob puts them
template <class R>
__device__ __forceinline__ void fast_attributes(R& r, i32 t, const crr_blob_batch& in, const Plan& P, u64 x,
                                                u32& seen, u32& n_prev) {
  u32 ft;
  i32 id;
  i32 last = -0x10000;
  while (r.field(ft, id)) {
    if (id <= last) { r.err = kDeferGeneral; return; }
    last = id;
    bool used = true;
    switch (t) {
      case CRR_EV_WORKFLOW_EXECUTION_STARTED: {
        crr_start_side* ss = P.start + x;
        if (id == 12 && ft == T_STRING) {
          u64 o; u32 l;
          r.str(o, l);
          if (!r.err) ss->parent_domain_status = domain_fast(r, in, P, x, o, l);
        }
        else if (id == 40 && ft == T_I32) ss->workflow_timeout = r.be32();
        else if (id == 50 && ft == T_I32) ss->decision_start_to_close = r.be32();
        else if (id == 55 && ft == T_I32) ss->initiator = r.be32();
        else if (id == 80 && ft == T_I32) ss->attempt = r.be32();
        else if (id == 90 && ft == T_I64) ss->expiration_ns = r.be64();
        else if (id == 110 && ft == T_I32) ss->first_decision_backoff = r.be32();
        else if (id == 130 && ft == T_STRUCT) {
          const PrevPoints q = walk_reset_points(r);   // a copy of the reader, window included
          r.p = q.p;
          r.err = q.err;
          if (!r.err) {
            ss->prev_reset_count = q.mode == 0 ? q.n : q.mode;
            if (q.mode == 0) {
              PrevRef pr;
              pr.pos = q.pos; pr.n = (u32)q.n; pr.et = q.et;
              *reinterpret_cast<PrevRef*>(P.keys + x) = pr;
              n_prev += (u32)q.n;
            }
          }
        }
        else used = false;
        break;
      }
      case CRR_EV_DECISION_TASK_SCHEDULED:
        if (id == 20 && ft == T_I32) { P.aux[x] = r.be32(); seen |= S_AUX; }
        else if (id == 30 && ft == T_I64) { P.ref[x] = r.be64(); seen |= S_REF; }
        else used = false;
        break;
      case CRR_EV_DECISION_TASK_TIMED_OUT:
        if (id == 30 && ft == T_I32) { P.aux[x] = r.be32(); seen |= S_AUX; } else used = false;
        break;
      case CRR_EV_ACTIVITY_TASK_SCHEDULED: {
        crr_activity_side* as = P.act + x;
        if (id == 10 && ft == T_STRING) {
          u64 o; u32 l;
          r.str(o, l);
          if (!r.err) P.keys[x] = r.key_ref(o, l);
        }
        else if (id == 25 && ft == T_STRING) {
          u64 o; u32 l;
          r.str(o, l);
          if (!r.err) as->domain_status = domain_fast(r, in, P, x, o, l);
        }
        else if (id == 45 && ft == T_I32) as->schedule_to_close = r.be32();
        else if (id == 50 && ft == T_I32) as->schedule_to_start = r.be32();
        else if (id == 55 && ft == T_I32) as->start_to_close = r.be32();
        else if (id == 60 && ft == T_I32) as->heartbeat = r.be32();
        else if (id == 110 && ft == T_STRUCT) {   // RetryPolicy{60 ExpirationIntervalInSeconds}
          as->has_retry_policy = 1;
          u32 f2;
          i32 id2;
          while (r.field(f2, id2)) {
            if (id2 == 60 && f2 == T_I32) as->expiration_interval = r.be32();
            else r.skip(f2);
          }
        }
        else used = false;
        break;
      }
      case CRR_EV_DECISION_TASK_COMPLETED: case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED: case CRR_EV_TIMER_FIRED:
      case CRR_EV_TIMER_CANCELED: case CRR_EV_TIMER_STARTED: {
        const i32 key_id = t == CRR_EV_DECISION_TASK_COMPLETED ? 50 : 10;
        const i32 ref_id = t == CRR_EV_DECISION_TASK_COMPLETED ? 30 : t == CRR_EV_TIMER_STARTED ? 20 : -1;
        if (id == key_id && ft == T_STRING) {
          u64 o; u32 l;
          r.str(o, l);
          if (!r.err) P.keys[x] = r.key_ref(o, l);
        }
        else if (id == ref_id && ft == T_I64) { P.ref[x] = r.be64(); seen |= S_REF; }
        else used = false;
        break;
      }
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED:
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED:
      case CRR_EV_SIGNAL_EXTERNAL_INITIATED: {
        const i32 dom_id = t == CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED ? 10 : 20;
        if (id == dom_id && ft == T_STRING) {
          u64 o; u32 l;
          r.str(o, l);
          if (!r.err) { P.aux[x] = domain_fast(r, in, P, x, o, l); seen |= S_AUX; }
        }
        else used = false;
        break;
      }
      default: {
        // the types whose only field is the i64 reference (read_attributes' remaining cases)
        i32 ref_id = -1;
        switch (t) {
          case CRR_EV_DECISION_TASK_STARTED: case CRR_EV_ACTIVITY_TASK_STARTED: case CRR_EV_ACTIVITY_TASK_TIMED_OUT:
          case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED: case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED:
            ref_id = 10; break;
          case CRR_EV_ACTIVITY_TASK_COMPLETED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED: ref_id = 20; break;
          case CRR_EV_ACTIVITY_TASK_FAILED: case CRR_EV_ACTIVITY_TASK_CANCELED: ref_id = 30; break;
          case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED: ref_id = 40; break;
          case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED:
          case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT: case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED:
          case CRR_EV_SIGNAL_EXTERNAL_FAILED:
            ref_id = 50; break;
          case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED: ref_id = 60; break;
          default: break;
        }
        if (id == ref_id && ft == T_I64) { P.ref[x] = r.be64(); seen |= S_REF; } else used = false;
      }
    }
    if (r.err) return;
    if (!used) r.skip(ft);
    if (r.err) return;
  }
}

// one event into slot x (decode_blob's loop body for a canonical event)
template <class R>
__device__ __forceinline__ void fast_event(R& r, const crr_blob_batch& in, const Plan& P, u64 x, i32 new_run,
                                           u32& n_prev, u32 boundary) {
  u32 seen = 0;
  i32 t = -1;
  bool have_type = false;
  i32 last = -0x10000;
  u32 ft;
  i32 id;
  while (r.field(ft, id)) {
    if (id <= last) { r.err = kDeferGeneral; return; }
    last = id;
    if (id == 10 && ft == T_I64) { P.id[x] = r.be64(); seen |= S_ID; }
    else if (id == 20 && ft == T_I64) { P.ts[x] = r.be64(); seen |= S_TS; }
    else if (id == 30 && ft == T_I32) {
      t = r.be32();
      have_type = true;
      if (r.err) return;
      // the defaults of the records this type fills (attr_init's values)
      if (t == CRR_EV_WORKFLOW_EXECUTION_STARTED) {
        crr_start_side ss;
        ss.decision_start_to_close = 0; ss.workflow_timeout = 0; ss.first_decision_backoff = 0;
        ss.initiator = CRR_INITIATOR_NIL; ss.parent_domain_status = CRR_DOMAIN_NOT_SET;
        ss.prev_reset_key_off = n_prev;   // blob-local until wf_pass adds the blob's prefix
        ss.prev_reset_count = -1; ss.attempt = 0; ss.expiration_ns = 0; ss.refresh_jitter = 0;
        P.start[x] = ss;
      } else if (t == CRR_EV_ACTIVITY_TASK_SCHEDULED) {
        crr_activity_side as;
        as.schedule_to_start = 0; as.schedule_to_close = 0; as.start_to_close = 0; as.heartbeat = 0;
        as.has_retry_policy = 0; as.expiration_interval = 0; as.domain_status = CRR_DOMAIN_NOT_SET; as.reserved = 0;
        P.act[x] = as;
      }
      if (t >= 0 && t < CRR_EV_TYPE_COUNT && keyed_type(t)) {
        P.keys[x] = r.key_ref(0, 0);
      }
    }
    else if (id == 35 && ft == T_I64) { P.ver[x] = r.be64(); seen |= S_VER; }
    else if (id == 36 && ft == T_I64) { P.task[x] = r.be64(); seen |= S_TASK; }
    else {
      const int at = ft == T_STRUCT ? attr_type_of_field(id) : -1;
      if (at >= 0 && !have_type) { r.err = kDeferGeneral; return; }   // attributes before the type
      if (at >= 0 && at == t) fast_attributes(r, t, in, P, x, seen, n_prev);
      else r.skip(ft);
    }
    if (r.err) return;
  }
  if (r.err) return;
  if (!have_type) { r.err = kDeferGeneral; return; }   // the type's zero default: the general pass
  const bool valid = t >= 0 && t < CRR_EV_TYPE_COUNT;
  P.etype[x] = (u8)((valid ? t : CRR_EV_PAD - 1) | boundary);
  if (!(seen & S_ID)) P.id[x] = 0;
  if (!(seen & S_TS)) P.ts[x] = 0;
  if (!(seen & S_VER)) P.ver[x] = 0;
  if (!(seen & S_TASK)) P.task[x] = 0;
  if (!(seen & S_REF)) P.ref[x] = 0;
  if (valid && t == CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW) P.aux[x] = new_run;
  else if (!(seen & S_AUX)) P.aux[x] = 0;   // (CRR_DOMAIN_NOT_SET for a domain-aux type: also 0)
  P.key[x] = 0;
}

// The blob's slots [x, x_end) and its workflow's new_run_wf come from the caller (loaded before the
// staging).  Batch boundaries are set as the events are written: a count that was wrong sends the plan
// back to the recount and this decode runs again, so x_end is exact whenever the results are used.
template <bool L>
__device__ __forceinline__ void decode_blob_fast(const crr_blob_batch& in, const Plan& P, u32 bi, u64 b0, u64 b1,
                                                 u64 x, u64 x_end, i32 new_run, lds_u8* staged, u64 staged_base) {
  u32 n_prev = 0;
  if (b1 > b0) {
    RdT<false, L> r;
    r.init_staged(in.bytes, staged, staged_base, b0, b1);
    if (r.u8_() != 0x59) { record_error(P.err, bi, CRR_DECODE_BAD_PREAMBLE); return; }  // version0Thriftrw.go:53-58
    const u64 x_first = x;
    u32 ft;
    i32 fid;
    while (r.field(ft, fid)) {
      if (fid != 10 || ft != T_LIST) { r.skip(ft); continue; }
      const u32 et = r.u8_();
      const i32 n = r.be32();
      if (r.err) break;
      if (n < 0) { r.err = CRR_DECODE_TRUNCATED; break; }
      if (et != T_STRUCT && n > 0) { r.err = CRR_DECODE_BAD_TYPE; break; }
      for (i32 i = 0; i < n; ++i) {
        if (x >= x_end) { r.err = kDeferGeneral; break; }   // more events than announced
        fast_event(r, in, P, x, new_run, n_prev,
                   (x == x_first ? CRR_ETYPE_BATCH_FIRST : 0u) | (x + 1 == x_end ? CRR_ETYPE_BATCH_LAST : 0u));
        if (r.err) break;
        ++x;
      }
      if (r.err) break;
    }
    if (r.err == kDeferGeneral) {
      P.cnt[1 * (u64)P.n_blobs + bi] = kDeferMark;
      return;
    }
    if (r.err) { record_error(P.err, bi, r.err); return; }
  }
  if (x != x_end) atomicOr(P.flags, 1u);   // fewer events than the header announced: recount
  P.cnt[1 * (u64)P.n_blobs + bi] = n_prev;
}

// A wavefront per 64 consecutive blobs.  Their bytes are contiguous: the wavefront copies them into LDS
// with coalesced 16-byte loads (up to kStageBytes at a time), then every lane walks its own blob from
// LDS, so a walk's window loads are LDS round trips instead of a chain of dependent HBM reads.  A
// window holding only some of the blobs serves those; the rest are staged again from the first one left.
// A blob larger than the window alone is walked from HBM.
#ifndef CRR_INGEST_STAGE_KB
#define CRR_INGEST_STAGE_KB 13
#endif
constexpr u32 kStageBytes = CRR_INGEST_STAGE_KB * 1024;   // 13 KB: 12 wavefronts per CU (measured best: 10 / 16 / 20 KB slower)
__global__ __launch_bounds__(64) void blob_decode_kernel(crr_blob_batch in, Plan P) {
  __shared__ __attribute__((aligned(16))) u8 stage[kStageBytes];
  const u32 lane = threadIdx.x;
  const u32 bi = blockIdx.x * 64 + lane;
  const bool mine = bi < in.n_blobs;
  const u64 NB = (u64)P.n_blobs + 1;
  // this plan's mark, never an earlier plan's: a blob whose fast decode fails or is skipped leaves no
  // stale kDeferMark (the scratch is reused across plans) for the general pass to act on
  if (mine) P.cnt[1 * (u64)P.n_blobs + bi] = 0;
  if (P.off[0 * NB + P.n_blobs] > P.max_events) return;   // the summary reports it
  const u32 last = blockIdx.x * 64 + 64 < in.n_blobs ? blockIdx.x * 64 + 64 : in.n_blobs;
  // readable up to 32 bytes past the last blob (cadence_ingest.h): a walk's window reads end before
  // ((b1 - 1) & ~15) + 32 <= (b1 + 31) & ~15
  const u64 stage_cap = (in.blob_off[last] + 31) & ~15ull;
  const u64 b0 = mine ? in.blob_off[bi] : 0, b1 = mine ? in.blob_off[bi + 1] : 0;
  const u64 x0 = mine ? P.off[0 * NB + bi] : 0, x1 = mine ? P.off[0 * NB + bi + 1] : 0;
  const i32 new_run = mine && b1 > b0 ? in.wf[P.blob_wf[bi]].new_run_wf : 0;
  lds_u8* lb = (lds_u8*)stage;
  bool done = !mine;
  for (;;) {
    const u64 pending = __ballot(!done);
    if (pending == 0) break;
    const int f = __builtin_ctzll(pending);
    const u64 s = (u64)__shfl((long long)b0, f) & ~15ull;
    const u64 lim = s + kStageBytes < stage_cap ? s + kStageBytes : stage_cap;
    __syncthreads();   // the previous window's walks are done with it
    for (u64 o = s + 16ull * lane; o < lim; o += 64 * 16)
      *reinterpret_cast<v4u*>(stage + (o - s)) = *reinterpret_cast<const v4u*>(in.bytes + o);
    __syncthreads();
    const bool fits = !done && (b1 == b0 || (b0 >= s && ((b1 - 1) & ~15ull) + 32 <= lim));
    if (fits) {
      decode_blob_fast<true>(in, P, bi, b0, b1, x0, x1, new_run, lb, s);
      done = true;
    } else if (!done && (int)lane == f) {   // larger than the window: from HBM
      decode_blob_fast<false>(in, P, bi, b0, b1, x0, x1, new_run, lb, 0);
      done = true;
    }
  }
}

// the fast decode's deferred domain lookups (domain_fast), a lane per event; only when the plan has a
// known-domain set
__global__ __launch_bounds__(kBlock) void domain_resolve_kernel(crr_blob_batch in, Plan P) {
  const u64 NB = (u64)P.n_blobs + 1;
  const u64 n = P.off[0 * NB + P.n_blobs];
  if (n > P.max_events || *P.flags || *P.err != ~0ull) return;   // the plan reports / recounts
  const u64 n_bytes = in.blob_off[in.n_blobs];
  for (u64 x = (u64)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (u64)gridDim.x * blockDim.x) {
    const i32 t = P.etype[x] & CRR_ETYPE_MASK;
    i32* dst = t == CRR_EV_WORKFLOW_EXECUTION_STARTED ? &P.start[x].parent_domain_status
               : t == CRR_EV_ACTIVITY_TASK_SCHEDULED  ? &P.act[x].domain_status
               : domain_aux_type(t)                    ? P.aux + x
                                                       : nullptr;
    if (!dst || *dst != kDomainPending) continue;
    const KeyRef d = P.dom_refs[x];
    if (d.off > n_bytes || d.len > n_bytes - d.off) continue;   // (never: written by this plan's decode)
    *dst = domain_status_h(in, P.dom_table, P.dom_cap, d.off, d.len, d.hash);
  }
}

// the blobs the fast pass deferred (a container of structs / containers), with the general reader
__global__ __launch_bounds__(kBlock) void blob_decode_general_kernel(crr_blob_batch in, Plan P) {
  const u32 bi = blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= in.n_blobs) return;
  const u64 NB = (u64)P.n_blobs + 1;
  if (P.off[0 * NB + P.n_blobs] > P.max_events || *P.flags) return;   // reported / recounted
  if (P.cnt[1 * (u64)P.n_blobs + bi] != kDeferMark) return;
  decode_blob<true>(in, P, bi);
}

// ---- 4: previous reset points at their reset_keys positions ------------------------------------------------
__global__ void reset_refs_kernel(crr_blob_batch in, Plan P) {
  const u32 bi = blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= in.n_blobs || !plan_ok(P)) return;
  const u64 NB = (u64)P.n_blobs + 1;
  if (P.cnt[1 * (u64)P.n_blobs + bi] == 0) return;
  u64 k = P.off[1 * NB + bi];
  for (u64 x = P.off[0 * NB + bi]; x < P.off[0 * NB + bi + 1]; ++x) {
    if ((P.etype[x] & CRR_ETYPE_MASK) != CRR_EV_WORKFLOW_EXECUTION_STARTED || P.start[x].prev_reset_count <= 0) continue;
    const PrevRef pr = *reinterpret_cast<const PrevRef*>(P.keys + x);
    Rd r;
    r.init(in.bytes, pr.pos, in.blob_off[bi + 1]);
    for (u32 i = 0; i < pr.n; ++i) {   // read_reset_points: the last BinaryChecksum of each element
      u64 so = 0;
      u32 sl = 0;
      if (pr.et != T_STRUCT) {
        r.skip(pr.et);
      } else {
        u32 t2;
        i32 id2;
        while (r.field(t2, id2)) {
          if (id2 == 10 && t2 == T_STRING) r.str(so, sl);
          else r.skip(t2);
        }
      }
      P.resets[k++] = r.key_ref(so, sl);
    }
  }
}

// ---- 3: exclusive prefixes over K arrays of m u32 / u64 values (reduce, scan the tile sums, apply) --------
constexpr int kTile = 1024;
template <class T>
__global__ void scan_tiles_kernel(const T* in, u64 in_stride, u32 m, int K, u64* tile_sums, u32 n_tiles) {
  __shared__ u64 part[kBlock];
  const u32 tile = blockIdx.x, k = blockIdx.y;
  u64 s = 0;
  for (u32 i = threadIdx.x; i < kTile; i += kBlock) {
    const u64 j = (u64)tile * kTile + i;
    if (j < m) s += (u64)in[k * in_stride + j];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = kBlock / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) tile_sums[(u64)k * n_tiles + tile] = part[0];
}
// one block per array: exclusive scan of its tile sums (serial in chunks of kBlock)
__global__ void scan_tile_sums_kernel(u64* tile_sums, u32 n_tiles) {
  __shared__ u64 buf[kBlock];
  __shared__ u64 carry;
  const u32 k = blockIdx.x;
  u64* ts = tile_sums + (u64)k * n_tiles;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (u32 base = 0; base < n_tiles; base += kBlock) {
    const u32 i = base + threadIdx.x;
    const u64 v = i < n_tiles ? ts[i] : 0;
    buf[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < kBlock; o <<= 1) {   // inclusive Hillis-Steele
      const u64 add = (int)threadIdx.x >= o ? buf[threadIdx.x - o] : 0;
      __syncthreads();
      buf[threadIdx.x] += add;
      __syncthreads();
    }
    const u64 c = carry;
    if (i < n_tiles) ts[i] = c + buf[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == kBlock - 1) carry = c + buf[kBlock - 1];
    __syncthreads();
  }
}
// out[k][j] = exclusive prefix of in[k][0..j), j <= m (out has m + 1 entries per array).  A thread per 4
// consecutive values: its sum, a wave scan of the sums, the waves' totals through LDS.
template <class T>
__global__ __launch_bounds__(kBlock) void scan_apply_kernel(const T* in, u64 in_stride, u32 m, const u64* tile_sums,
                                                            u32 n_tiles, u64* out, u64 out_stride) {
  constexpr int kPer = kTile / kBlock;
  __shared__ u64 wsum[kBlock / 64];
  const u32 tile = blockIdx.x, k = blockIdx.y;
  const u32 tid = threadIdx.x, lane = tid & 63, wv = tid / 64;
  const u64 j0 = (u64)tile * kTile + (u64)tid * kPer;
  u64 v[kPer];
  u64 loc = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    v[q] = j0 + q < m ? (u64)in[k * in_stride + j0 + q] : 0;
    loc += v[q];
  }
  u64 inc = loc;
  for (u32 d = 1; d < 64; d <<= 1) {
    const u64 o = __shfl_up(inc, d);
    if (lane >= d) inc += o;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  u64 s = tile_sums[(u64)k * n_tiles + tile] + inc - loc;
  for (u32 w = 0; w < wv; ++w) s += wsum[w];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    if (j0 + q < m) out[k * out_stride + j0 + q] = s;
    s += v[q];
  }
  // the total, by the thread holding value m - 1 (values past m are 0); m == 0: tile 0's first thread
  if ((m > 0 && j0 <= m - 1 && m - 1 < j0 + kPer) || (m == 0 && tile == 0 && tid == 0)) out[k * out_stride + m] = s;
}

template <class T>
void multi_scan(const T* in, u64 in_stride, u32 m, int K, u64* tile_sums, u64* out, u64 out_stride, hipStream_t s) {
  const u32 n_tiles = (m + kTile - 1) / kTile;
  const u32 nt = n_tiles ? n_tiles : 1;
  hipLaunchKernelGGL(scan_tiles_kernel<T>, dim3(nt, K), dim3(kBlock), 0, s, in, in_stride, m, K, tile_sums, nt);
  hipLaunchKernelGGL(scan_tile_sums_kernel, dim3(K), dim3(kBlock), 0, s, tile_sums, nt);
  hipLaunchKernelGGL(scan_apply_kernel<T>, dim3(nt, K), dim3(kBlock), 0, s, in, in_stride, m, tile_sums, nt, out,
                     out_stride);
}

// ---- 5: per workflow: interning, capacities, bounds, tier, sort key --------------------------------------
// The workflow's table region: a power of two >= 2 * its entries (events, plus key strings), from a
// per-workflow prefix (no collisions across workflows).
__device__ __forceinline__ u32 pow2_at_least(u32 x) {
  u32 c = 16;
  while (c < x) c <<= 1;
  return c;
}

// 64-bit table entries.  Interning: (hash32 << 32) | (entry index + 1), the key id kept in a parallel
// word.  Bounds: (map << 40 | low 40 bits of the ID or key) + 1 in the low 43 bits, flag bits above.
constexpr u64 kInserted = 1ull << 62, kDeleteSeen = 1ull << 61;
// live-set bound table entries: the creating event's position + 1 (bits 0-32), its map (33-35), which
// of its fields holds the value (36-37); flags above
constexpr u64 kPosMask = (1ull << 33) - 1;
constexpr int kMapShift = 33, kKindShift = 36;

__device__ __forceinline__ bool same_bytes(const u8* b, u64 x, u64 y, u32 len) {
  Rd rx, ry;
  rx.init(b, x, x + len);
  ry.init(b, y, y + len);
  for (u32 i = 0; i < len; i += 8) {
    const u32 m = len - i < 8 ? len - i : 8;
    const u64 mask = m == 8 ? ~0ull : ((1ull << (8 * m)) - 1);
    if ((rx.peek8(x + i) ^ ry.peek8(y + i)) & mask) return false;
  }
  return true;
}

// the workflows wf_pass_wave_kernel takes (a wavefront per workflow): at most 64 events and 63 batches
// (their 64 offsets one load), no previous reset points to intern; wf_pass_kernel takes the rest
__device__ __forceinline__ bool wave_shaped(u32 n, u32 nr, u32 n_batches) {
  return n <= 64 && nr == 0 && n_batches < 64;
}

// the live-set map of an event type and its direction (flatten.live_set_bounds)
__device__ __forceinline__ int bound_map_of(u32 t, int& dir) {
  dir = 0;
  switch (t) {
    case CRR_EV_ACTIVITY_TASK_SCHEDULED: dir = 1; return 0;
    case CRR_EV_ACTIVITY_TASK_COMPLETED: case CRR_EV_ACTIVITY_TASK_FAILED: case CRR_EV_ACTIVITY_TASK_TIMED_OUT:
    case CRR_EV_ACTIVITY_TASK_CANCELED: dir = -1; return 0;
    case CRR_EV_TIMER_STARTED: dir = 1; return 1;
    case CRR_EV_TIMER_FIRED: case CRR_EV_TIMER_CANCELED: dir = -1; return 1;
    case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED: dir = 1; return 2;
    case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED:
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED:
    case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT: case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED:
      dir = -1; return 2;
    case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED: dir = 1; return 3;
    case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED: case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED:
      dir = -1; return 3;
    case CRR_EV_SIGNAL_EXTERNAL_INITIATED: dir = 1; return 4;
    case CRR_EV_SIGNAL_EXTERNAL_FAILED: case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED: dir = -1; return 4;
    default: return -1;
  }
}

// the per-workflow tail both passes share: tier class, counters, info words, sort key, token bytes
struct WfSummary {
  i32 n, empty_at, n_act, n_timer, n_child, n_rc, n_sig, vh, rp_cap, tasks, n_started;
  i32 bound[kMaps];
  bool compact_ok;
};
// tier_classes; returns the counter slots this workflow adds one to (bit k: counter k)
__device__ __forceinline__ u32 wf_finish(const crr_blob_batch& in, const Plan& P, u32 w, const crr_blob_wf& src,
                                         const WfSummary& S, i32* info /* [kWfInfo] */, u64& sort_key, u64& arena) {
  const i32* bound = S.bound;
  int tier = kWide;
  for (int k = kWide - 1; k >= 0; --k) {
    bool fit = true;
    for (int m = 0; m < kMaps; ++m) fit = fit && bound[m] <= kTierSlots[k][m];
    if (k >= 2) fit = fit && S.compact_ok;
    if (fit) tier = k;
  }
  if (tier == 1 && S.compact_ok) tier = 2;
  const u32 n = (u32)S.n;
  const bool is_long = (i32)n > kLongHistory || tier == kWide;
  bool big = false;
  for (int m = 0; m < kMaps; ++m) big = big || bound[m] > kWaveBigCap;
  u32 cnt = 0;
  if (is_long && !big) {
    bool small = true;
    for (int m = 0; m < kMaps; ++m) small = small && bound[m] <= kWaveSmallTier[m];
    if (!small) cnt |= 1u << C_SMALL_TAIL_BAD;
  }
  if (is_long) { if (big) cnt |= 1u << C_N_BIG; }
  else cnt |= (1u << C_N_LANE) | (1u << (C_TIER0 + tier));
  if (src.flags & CRR_WF_FLAG_NEW_RUN) cnt |= 1u << C_NEW_RUN;
  info[WI_COUNT] = (i32)n; info[WI_EMPTY_AT] = S.empty_at;
  info[WI_ACT] = S.n_act; info[WI_TIMER] = S.n_timer; info[WI_CHILD] = S.n_child;
  info[WI_RC] = S.n_rc; info[WI_SIG] = S.n_sig; info[WI_VH] = S.vh; info[WI_RP] = S.rp_cap;
  // + RefreshTasks' search-attributes task (CRR_WF_FLAG_REFRESH_TASKS: its other tasks fit the replay's bound)
  info[WI_TASKS] = S.tasks + ((src.flags & CRR_WF_FLAG_REFRESH_TASKS) ? 1 : 0); info[WI_STARTED] = S.n_started;
  info[WI_TIER] = tier; info[WI_LONG] = is_long; info[WI_BIG] = big;
  // device order (flatten.interleave): lanes by (tier, -length, index), then the long tail by (big, -length, index)
  const u64 cls = is_long ? (u64)big : (u64)tier;
  const u64 len = n < 0x1FFFFFFFu ? n : 0x1FFFFFFFu;
  sort_key = ((u64)is_long << 63) | (cls << 60) | ((0x1FFFFFFFull - len) << 31) | (u64)w;
  // the branch tokens' bytes (NewHistoryBranchTokenByBranchID) + the final token
  arena = 24ull + src.run_id_len + src.branch_id_len + (src.final_token_len != 0xFFFFFFFFu ? src.final_token_len : 0);
  return cnt;
}

__device__ __forceinline__ i32 wave_incl_sum(i32 v, u32 lane) {
  for (u32 d = 1; d < 64; d <<= 1) {
    const i32 o = __shfl_up(v, d);
    if (lane >= d) v += o;
  }
  return v;
}
__device__ __forceinline__ i32 wave_max(i32 v) {
  for (int d = 32; d >= 1; d >>= 1) { const i32 o = __shfl_xor(v, d); v = o > v ? o : v; }
  return v;
}
__device__ __forceinline__ u32 bcast_u32(u32 v, int j) { return (u32)__builtin_amdgcn_readlane((int)v, j); }
__device__ __forceinline__ u64 bcast_u64(u64 v, int j) {
  return ((u64)bcast_u32((u32)(v >> 32), j) << 32) | bcast_u32((u32)v, j);
}

// 5 (wave form): a wavefront per workflow, a lane per event (and per batch).  The same results as
// wf_pass_kernel's serial walk, by wave-wide prefix counts and pairwise compares:
//   key ids     a key's first occurrence (the lowest earlier lane with the same bytes) and its rank among
//               the first occurrences: WfFlattener::key_of's first-seen numbering
//   VH items    lanes whose version exceeds every earlier one
//   ordinals    prefix counts of Started / ActivityTaskScheduled lanes
//   bounds      each map's +1 / -1 (a delete valid as live_set_bounds decides: its key / ID inserted
//               anywhere in the workflow, ref < ID, the first delete of that ref), inclusive prefix sums,
//               their maximum
// Workflows are taken grid-stride; a wavefront's counter increments are summed in registers and added
// once at the end.
constexpr u32 kWfWaveBlock = 256;
__global__ __launch_bounds__(kWfWaveBlock) void wf_pass_wave_kernel(crr_blob_batch in, Plan P) {
  if (P.resume || !plan_ok(P)) return;   // (resume: seeded interning, wf_pass_kernel's)
  const u32 lane = threadIdx.x & 63;
  const u32 wave0 = blockIdx.x * (kWfWaveBlock / 64) + threadIdx.x / 64;
  const u32 n_waves = gridDim.x * (kWfWaveBlock / 64);
  const u64 NB = P.n_blobs + 1;
  const u64 lt = (1ull << lane) - 1;
  const u64 nw = in.n_wf;
  u32 my_count = 0;   // lane k: counter k's increments
  // the next workflow's record and batch offsets are fetched while this one is worked on
  crr_blob_wf nsrc;
  nsrc.blob_begin = 0; nsrc.blob_count = 64;
  u64 nob = 0, nrv = 0;   // lane k: the offset of batch k (events), of batches 0 and count (reset points)
  auto fetch_src = [&](u32 w) {
    if (w < in.n_wf) nsrc = in.wf[w];
  };
  auto fetch_off = [&](u32 w) {
    if (w >= in.n_wf) return;
    const u32 bb = nsrc.blob_begin, c = nsrc.blob_count;
    nob = lane <= c && c < 64 ? P.off[0 * NB + bb + lane] : 0;
    nrv = (lane == 0 || lane == c) && c < 64 ? P.off[1 * NB + bb + lane] : 0;
  };
  fetch_src(wave0);
  fetch_off(wave0);
  for (u32 w = wave0; w < in.n_wf; w += n_waves) {
    const crr_blob_wf src = nsrc;
    const u64 ob = nob, rv = nrv;
    fetch_src(w + n_waves);
    const u32 nbat = src.blob_count;
    if (nbat >= 64) { fetch_off(w + n_waves); continue; }   // wf_pass_kernel's
    const u64 e0 = (u64)__shfl((long long)ob, 0), e1 = (u64)__shfl((long long)ob, (int)nbat);
    const u64 r0 = (u64)__shfl((long long)rv, 0), r1 = (u64)__shfl((long long)rv, (int)nbat);
    const u32 n = (u32)(e1 - e0);
    if (!wave_shaped(n, (u32)(r1 - r0), nbat)) { fetch_off(w + n_waves); continue; }
    // -- batches: the first empty one, two tasks per non-empty one --
    const bool has_b = lane < nbat;
    const u64 bx0 = ob, bx1 = (u64)__shfl_down((long long)ob, 1);
    // -- events --
    const bool ev = lane < n;
    const u64 x = e0 + lane;
    const u32 t = ev ? (u32)(P.etype[x] & CRR_ETYPE_MASK) : 0xFFu;
    const i64 v = ev ? P.ver[x] : INT64_MIN;
    const i64 id = ev ? P.id[x] : 0;
    const i64 ref = ev ? P.ref[x] : 0;
    const bool keyed = ev && t < CRR_EV_TYPE_COUNT && keyed_type((i32)t);
    // every event's KeyRef slot with the columns (one round trip; a non-keyed event's is ignored)
    KeyRef kr;
    kr.off = 0; kr.len = 0; kr.hash = 0; kr.head[0] = 0; kr.head[1] = 0;
    if (ev) kr = P.keys[x];
    if (!keyed) { kr.len = 0; kr.hash = 0; }
    const bool started = t == CRR_EV_WORKFLOW_EXECUTION_STARTED;
    i32 pc = -1;
    if (started) pc = P.start[x].prev_reset_count;
    fetch_off(w + n_waves);

    const u64 empty_mask = __ballot(has_b && bx0 == bx1);
    const i32 empty_at = src.blob_count == 0 ? 0
                         : empty_mask ? (i32)((u64)__shfl((long long)bx0, __builtin_ctzll(empty_mask)) - e0) : -1;
    const i32 tasks = 2 * __popcll(__ballot(has_b && bx1 > bx0)) +
                      __shfl(wave_incl_sum(t < CRR_EV_TYPE_COUNT ? (i32)kTasksPerEvent[t] : 0, lane), 63);
    // VH items: a version above every earlier one (the first event's always)
    i64 run_max = v;
    for (u32 d = 1; d < 64; d <<= 1) {
      const i64 o = __shfl_up(run_max, d);
      if (lane >= d && o > run_max) run_max = o;
    }
    const i64 before = __shfl_up(run_max, 1);
    const i32 vh = __popcll(__ballot(ev && (lane == 0 || v > before)));
    // ordinals and counts
    const u64 m_started = __ballot(started), m_act = __ballot(t == CRR_EV_ACTIVITY_TASK_SCHEDULED);
    const u64 m_dtc = __ballot(t == CRR_EV_DECISION_TASK_COMPLETED);
    const i32 n_started = __popcll(m_started), n_act = __popcll(m_act), n_dtc = __popcll(m_dtc);
    const i32 n_timer = __popcll(__ballot(t == CRR_EV_TIMER_STARTED));
    const i32 n_child = __popcll(__ballot(t == CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED));
    const i32 n_rc = __popcll(__ballot(t == CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED));
    const i32 n_sig = __popcll(__ballot(t == CRR_EV_SIGNAL_EXTERNAL_INITIATED));
    const i32 pc_max = wave_max(pc), max_prev = pc_max > 0 ? pc_max : 0;   // 0 here: no points to intern
    if (started) {
      if (pc >= 0) P.start[x].prev_reset_key_off += (u32)r0;   // the blob-local index made global (all 0 here)
      P.aux[x] = __popcll(m_started & lt);
    }
    if (t == CRR_EV_ACTIVITY_TASK_SCHEDULED) P.aux[x] = __popcll(m_act & lt);

    // -- interning: the first occurrence of each key's bytes --
    const bool named = keyed && kr.len != 0;
    const u64 m_named = __ballot(named);
    i32 first = named ? -1 : (i32)lane;
    u32 from = 0;
    for (;;) {
      const bool pending = first < 0;
      if (!__ballot(pending)) break;
      i32 c = -1;
      for (u64 mm = m_named; mm; mm &= mm - 1) {
        const int j = __builtin_ctzll(mm);
        const u32 hj = bcast_u32(kr.hash, j), lj = bcast_u32(kr.len, j);
        if (pending && c < 0 && (u32)j >= from && (u32)j < lane && hj == kr.hash && lj == kr.len) c = j;
      }
      const int cs = c < 0 ? (int)lane : c;
      const u64 c_off = (u64)__shfl((long long)kr.off, cs);
      const u64 c_h0 = (u64)__shfl((long long)kr.head[0], cs), c_h1 = (u64)__shfl((long long)kr.head[1], cs);
      if (pending) {
        if (c < 0) first = (i32)lane;
        else if (kr.len <= 16 ? (c_h0 == kr.head[0] && c_h1 == kr.head[1]) : same_bytes(in.bytes, kr.off, c_off, kr.len))
          first = c;
        else from = (u32)c + 1;
      }
    }
    const u64 m_first = __ballot(named && first == (i32)lane);
    const u32 key = named ? 1u + (u32)__popcll(m_first & ((1ull << first) - 1)) : 0u;
    if (keyed) P.key[x] = key;

    // -- live-set bounds --
    int dir = 0;
    const int m = ev ? bound_map_of(t, dir) : -1;
    bool compact_ok = n <= (u32)kCompactMaxEvents && !__ballot(ev && id > (i64)0xFFFFFFFFll);
    const bool dtc_named = t == CRR_EV_DECISION_TASK_COMPLETED && key != 0;
    const u64 ins_val = m == 1 ? (u64)key : (u64)id;        // an insert's value
    const u64 del_val = m == 1 ? (u64)key : (u64)ref;       // what a delete looks up
    // deletes: an insert of the same map and value anywhere; an earlier delete of the same map and ref
    bool inserted = false, deleted_before = false, rp_dup = false;
    if (__ballot(dir < 0)) {
      for (u64 mm = __ballot(dir > 0); mm; mm &= mm - 1) {
        const int j = __builtin_ctzll(mm);
        const int mj = (int)bcast_u32((u32)m, j);
        const u64 ij = bcast_u64(ins_val, j);
        if (dir < 0 && mj == m && ij == del_val) inserted = true;
      }
      for (u64 mm = __ballot(dir < 0 && m != 1); mm; mm &= mm - 1) {
        const int j = __builtin_ctzll(mm);
        const int mj = (int)bcast_u32((u32)m, j);
        const u64 rj = bcast_u64(del_val, j);
        if (dir < 0 && m != 1 && mj == m && (u32)j < lane && rj == del_val) deleted_before = true;
      }
    }
    // reset points: a DecisionTaskCompleted key not seen before
    for (u64 mm = __ballot(dtc_named); mm; mm &= mm - 1) {
      const int j = __builtin_ctzll(mm);
      if (dtc_named && (u32)j < lane && bcast_u32(key, j) == key) rp_dup = true;
    }
    const bool valid = dir > 0 || (dir < 0 && (m == 1 ? inserted : inserted && ref < id && !deleted_before));
    WfSummary S;
    for (int k = 0; k < 5; ++k) {   // a map without valid deletes: its insert count, no scan
      const u64 dels = __ballot(m == k && valid && dir < 0);
      if (!dels) { S.bound[k] = __popcll(__ballot(m == k && dir > 0)); continue; }
      const i32 run = wave_incl_sum(m == k && valid ? dir : 0, lane);
      const i32 hi = wave_max(run);
      S.bound[k] = hi > 0 ? hi : 0;
    }
    S.bound[5] = __popcll(__ballot(dtc_named && !rp_dup)) + max_prev;
    S.n = (i32)n; S.empty_at = empty_at; S.n_act = n_act; S.n_timer = n_timer; S.n_child = n_child; S.n_rc = n_rc;
    S.n_sig = n_sig; S.vh = vh; S.rp_cap = max_prev * (n_started > 1 ? n_started : 1) + n_dtc; S.tasks = tasks;
    S.n_started = n_started; S.compact_ok = compact_ok;
    i32 info[kWfInfo];
    u64 sort_key, arena;
    const u32 cnt = wf_finish(in, P, w, src, S, info, sort_key, arena);
    my_count += (cnt >> lane) & 1u;
    i32 mine = 0;
#pragma unroll
    for (int k = 0; k < kWfInfo; ++k) mine = lane == (u32)k ? info[k] : mine;
    if (lane < kWfInfo) P.wf_info[lane * nw + w] = mine;
    if (lane == 0) { P.sort_in[w] = sort_key; P.arena_off[w] = arena; }
  }
  if (lane < 16 && my_count) atomicAdd(P.counters + lane, my_count);
}

__global__ void wf_pass_kernel(crr_blob_batch in, Plan P) {
  const u32 w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= in.n_wf || !plan_ok(P)) return;
  const crr_blob_wf src = in.wf[w];
  const u32 bb = src.blob_begin, be = src.blob_begin + src.blob_count;
  const u64 NB = P.n_blobs + 1;
  const u64 e0 = P.off[0 * NB + bb], e1 = P.off[0 * NB + be];
  const u64 r0 = P.off[1 * NB + bb], r1 = P.off[1 * NB + be];
  const u32 n = (u32)(e1 - e0);
  const u32 nr = (u32)(r1 - r0);
  // wf_pass_wave_kernel's.  Resuming, every workflow is this kernel's: a replication task's batch is a few
  // events, and a lane per workflow beat a wavefront per workflow with the loaded keys in lanes (config-3
  // shard, 1.25M tasks: 0.60 ms against 0.79 ms with a wavefront per workflow at once, 1.01 ms grid-stride)
  if (!P.resume && wave_shaped(n, nr, src.blob_count)) return;
  // resume: the loaded state's K keys seed the dictionary (entries n + nr + k, ids k + 1)
  const u32 K = P.resume ? P.key_count[w] : 0u, kb = P.resume ? P.key_begin[w] : 0u;
  // this workflow's scratch table: 4 * (events + reset points + seeded keys) + 64 u64 words from its own base
  const u64 tbase = 4 * e0 + 4 * r0 + 4ull * kb + 64ull * w;
  if (P.resume && tbase + 4ull * (n + nr + K) + 64 > 8 * P.max_events + 64ull * P.n_wf) {
    record_error(P.err, 0, kErrScratch);   // the seeds do not fit: the caller plans again with more
    return;
  }
  u64* tab = P.table + tbase;
  const u32 cap_i = pow2_at_least(2 * (n + nr + K) + 2);
  // resuming with a small loaded dictionary and no previous reset points: a linear search -- the loaded keys by
  // length and bytes, then this batch's earlier new keys by hash and bytes -- instead of a hash table to clear
  // and K loaded strings to hash (a replication task's batch holds a named key or two)
  const bool linear = P.resume && nr == 0 && K <= 64;
  if (!linear)
    for (u32 i = 0; i < cap_i; ++i) tab[i] = 0;
  auto seed_ref = [&](u32 k) -> KeyRef {   // (the hash through 8-byte unaligned loads: the pad follows the seeds)
    KeyRef r;
    r.off = P.key_off[kb + k]; r.len = P.key_len[kb + k];
    r.hash = 0;
    if (r.len) {
      RdT<false> rd;
      rd.init(in.bytes, r.off, r.off + r.len);
      r.hash = rd.hash(r.off, r.len);
    }
    r.head[0] = 0; r.head[1] = 0;
    return r;
  };
  // the seeds go in at the first named key (a batch without one never hashes them); the loaded strings are
  // distinct: inserted without a compare
  bool seeded = K == 0;
  auto seed_all = [&]() {
    seeded = true;
    for (u32 k = 0; k < K; ++k) {
      const KeyRef sr = seed_ref(k);
      if (sr.len == 0) continue;
      u32 slot = sr.hash & (cap_i - 1);
      while (tab[slot] != 0) slot = (slot + 1) & (cap_i - 1);
      tab[slot] = ((u64)sr.hash << 32) | (u64)(n + nr + k + 1);
    }
  };

  // One pass over the events in order: interning (WfFlattener::key_of: "" is key 0, new strings get 1, 2,
  // ... in first-seen order -- after the K loaded ones when resuming; a Started event's previous reset points
  // before anything after it), the side-record ordinals, capacities, VH items, tasks (WfFlattener::add /
  // batch_end / finish).
  // Table entries: (hash << 32) | (entry + 1), entry = event index (keys), n + reset index (resets) or
  // n + nr + loaded key index (seeds).
  u32 next_key = K + 1;
  auto intern = [&](const KeyRef& kr, u32 entry) -> u32 {
    if (kr.len == 0) return 0u;
    if (linear) {
      for (u32 k = 0; k < K; ++k)
        if (P.key_len[kb + k] == kr.len && same_bytes(in.bytes, kr.off, P.key_off[kb + k], kr.len)) return k + 1;
      for (u32 j = 0; j < entry; ++j) {   // this batch's earlier events: a new key is > K
        if (P.key[e0 + j] <= K) continue;
        const KeyRef o = P.keys[e0 + j];
        if (o.len == kr.len && o.hash == kr.hash &&
            (kr.len <= 16 ? (o.head[0] == kr.head[0] && o.head[1] == kr.head[1]) : same_bytes(in.bytes, kr.off, o.off, kr.len)))
          return P.key[e0 + j];
      }
      return next_key++;
    }
    if (!seeded) seed_all();
    u32 slot = kr.hash & (cap_i - 1);
    for (;;) {
      const u64 ent = tab[slot];
      if (ent == 0) {
        tab[slot] = ((u64)kr.hash << 32) | (u64)(entry + 1);
        return next_key++;
      }
      if ((u32)(ent >> 32) == kr.hash) {
        const u32 o = (u32)ent - 1;
        const KeyRef other = o < n ? P.keys[e0 + o] : o < n + nr ? P.resets[r0 + (o - n)] : seed_ref(o - n - nr);
        if (other.len == kr.len && same_bytes(in.bytes, kr.off, other.off, kr.len))
          return o < n ? P.key[e0 + o] : o < n + nr ? P.reset_ids[r0 + (o - n)] : o - n - nr + 1;
      }
      slot = (slot + 1) & (cap_i - 1);
    }
  };
  i32 n_act = 0, n_timer = 0, n_child = 0, n_rc = 0, n_sig = 0, n_dtc = 0, n_started = 0, vh = 0, tasks = 0;
  i32 max_prev = 0;
  i32 empty_at = -1;
  {
    bool have_ver = false;
    i64 last_ver = 0;
    u64 x = e0;
    for (u32 b = bb; b < be; ++b) {
      const u64 bx1 = P.off[0 * NB + b + 1];
      if (bx1 == x) {   // an empty batch
        if (empty_at < 0) empty_at = (i32)(x - e0);
        continue;
      }
      tasks += 2;
      const u64 rb = P.off[1 * NB + b];
      for (; x < bx1; ++x) {
        const u32 t = P.etype[x] & CRR_ETYPE_MASK;
        const i64 v = P.ver[x];
        if (!have_ver || v > last_ver) { ++vh; last_ver = v; have_ver = true; }
        if (t < CRR_EV_TYPE_COUNT) tasks += kTasksPerEvent[t];
        switch (t) {
          case CRR_EV_WORKFLOW_EXECUTION_STARTED: {
            crr_start_side& ss = P.start[x];
            const i32 pc = ss.prev_reset_count;
            if (pc >= 0) {
              const u64 g = rb + ss.prev_reset_key_off;   // the blob-local index made global
              ss.prev_reset_key_off = (u32)g;
              for (i32 k = 0; k < pc; ++k) P.reset_ids[g + k] = intern(P.resets[g + k], n + (u32)(g + k - r0));
            }
            if (pc > max_prev) max_prev = pc;
            P.aux[x] = n_started++;
            break;
          }
          case CRR_EV_DECISION_TASK_COMPLETED: ++n_dtc; P.key[x] = intern(P.keys[x], (u32)(x - e0)); break;
          case CRR_EV_ACTIVITY_TASK_SCHEDULED: P.key[x] = intern(P.keys[x], (u32)(x - e0)); P.aux[x] = n_act++; break;
          case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED: case CRR_EV_TIMER_FIRED: case CRR_EV_TIMER_CANCELED:
            P.key[x] = intern(P.keys[x], (u32)(x - e0));
            break;
          case CRR_EV_TIMER_STARTED: ++n_timer; P.key[x] = intern(P.keys[x], (u32)(x - e0)); break;
          case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED: ++n_child; break;
          case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED: ++n_rc; break;
          case CRR_EV_SIGNAL_EXTERNAL_INITIATED: ++n_sig; break;
          default: break;
        }
      }
    }
    // no batch at all: ApplyEvents' empty history (state_builder.go:98-100); resuming, nothing to apply
    if (src.blob_count == 0) empty_at = P.resume ? -1 : 0;
  }
  const i32 rp_cap = max_prev * (n_started > 1 ? n_started : 1) + n_dtc;

  // -- live-set bounds (flatten.live_set_bounds): inserts +1, deletes of inserted IDs (first delete of an
  // ID, ref < event ID) / inserted timer keys -1; the running maximum --
  i32 bound[kMaps] = {0, 0, 0, 0, 0, 0};
  bool compact_ok = n <= (u32)kCompactMaxEvents;
  if (!P.resume) {   // (resume: the tiering is the loaded layout's, no bounds to find)
    const u32 cap_b = pow2_at_least(2 * n + 2);   // <= the interning table's region
    for (u32 i = 0; i < cap_b; ++i) tab[i] = 0;
    auto map_of = [](u32 t, int& dir) -> int {
      dir = 0;
      switch (t) {
        case CRR_EV_ACTIVITY_TASK_SCHEDULED: dir = 1; return 0;
        case CRR_EV_ACTIVITY_TASK_COMPLETED: case CRR_EV_ACTIVITY_TASK_FAILED: case CRR_EV_ACTIVITY_TASK_TIMED_OUT:
        case CRR_EV_ACTIVITY_TASK_CANCELED: dir = -1; return 0;
        case CRR_EV_TIMER_STARTED: dir = 1; return 1;
        case CRR_EV_TIMER_FIRED: case CRR_EV_TIMER_CANCELED: dir = -1; return 1;
        case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED: dir = 1; return 2;
        case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED:
        case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED:
        case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT: case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED:
          dir = -1; return 2;
        case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED: dir = 1; return 3;
        case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED: case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED:
          dir = -1; return 3;
        case CRR_EV_SIGNAL_EXTERNAL_INITIATED: dir = 1; return 4;
        case CRR_EV_SIGNAL_EXTERNAL_FAILED: case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED: dir = -1; return 4;
        default: return -1;
      }
    };
    // An entry names the event that created it (its position, and which of its fields holds the value:
    // the ID, the ref or the interned key), so a lookup compares the full 64-bit value, never a truncation
    // (two IDs that differ only in high bits stay two entries, as in flatten's exact np.isin).
    enum : u32 { kById = 0, kByRef = 1, kByKey = 2 };
    auto value_of = [&](u64 ent) -> u64 {
      const u64 x = e0 + ((ent & kPosMask) - 1);
      const u32 kind = (u32)(ent >> kKindShift) & 3u;
      return kind == kById ? (u64)P.id[x] : kind == kByRef ? (u64)P.ref[x] : (u64)P.key[x];
    };
    auto find = [&](int m, u64 v, u32 kind, u64 x, bool create) -> u64* {
      u32 h = (u32)(((v ^ ((u64)m << 59)) * 0x9E3779B97F4A7C15ull) >> 32) & (cap_b - 1);
      for (;;) {
        const u64 ent = tab[h];
        if (ent == 0) {
          if (!create) return nullptr;
          tab[h] = ((u64)kind << kKindShift) | ((u64)m << kMapShift) | ((x - e0) + 1);
          return tab + h;
        }
        if ((int)((ent >> kMapShift) & 7u) == m && value_of(ent) == v) return tab + h;
        h = (h + 1) & (cap_b - 1);
      }
    };
    // inserts (np.isin is over every insert of the workflow, before or after the delete)
    for (u64 x = e0; x < e1; ++x) {
      const u32 t = P.etype[x] & CRR_ETYPE_MASK;
      if (P.id[x] > (i64)0xFFFFFFFFll) compact_ok = false;
      int dir;
      const int m = map_of(t, dir);
      if (m < 0 || dir <= 0) continue;
      const u64 v = m == 1 ? (u64)P.key[x] : (u64)P.id[x];
      *find(m, v, m == 1 ? kByKey : kById, x, true) |= kInserted;
    }
    i32 run[5] = {0, 0, 0, 0, 0};
    for (u64 x = e0; x < e1; ++x) {
      const u32 t = P.etype[x] & CRR_ETYPE_MASK;
      int dir;
      const int m = map_of(t, dir);
      if (m < 0) continue;
      if (dir < 0) {
        bool valid;
        if (m == 1) {
          u64* ent = find(1, (u64)P.key[x], kByKey, x, false);
          valid = ent && (*ent & kInserted);
        } else {
          u64* ent = find(m, (u64)P.ref[x], kByRef, x, true);   // created to carry the first-delete mark
          const bool first = !(*ent & kDeleteSeen);
          *ent |= kDeleteSeen;
          valid = (*ent & kInserted) && P.ref[x] < P.id[x] && first;
        }
        if (!valid) continue;
      }
      run[m] += dir;
      if (run[m] > bound[m]) bound[m] = run[m];
    }
    // reset points: distinct non-empty binary checksums + the most points a start event carries over
    // (the distinct count: a DecisionTaskCompleted key not seen before in this workflow)
    i32 rp = 0;
    for (u64 x = e0; x < e1; ++x) {
      if ((P.etype[x] & CRR_ETYPE_MASK) != CRR_EV_DECISION_TASK_COMPLETED || P.key[x] == 0) continue;
      u64* ent = find(5, (u64)P.key[x], kByKey, x, true);
      if (!(*ent & kInserted)) { *ent |= kInserted; ++rp; }
    }
    bound[5] = rp + (max_prev > 0 ? max_prev : 0);
  }
  WfSummary S;
  for (int m = 0; m < kMaps; ++m) S.bound[m] = bound[m];
  S.n = (i32)n; S.empty_at = empty_at; S.n_act = n_act; S.n_timer = n_timer; S.n_child = n_child; S.n_rc = n_rc;
  S.n_sig = n_sig; S.vh = vh; S.rp_cap = rp_cap; S.tasks = tasks; S.n_started = n_started; S.compact_ok = compact_ok;
  i32 info[kWfInfo];
  u64 sort_key, arena;
  const u32 cnt = wf_finish(in, P, w, src, S, info, sort_key, arena);
  for (int k = 0; k < 16; ++k)
    if ((cnt >> k) & 1u) atomicAdd(P.counters + k, 1u);
  for (int k = 0; k < kWfInfo; ++k) P.wf_info[k * (u64)in.n_wf + w] = info[k];
  P.sort_in[w] = sort_key;
  P.arena_off[w] = arena;
}

// ---- 7: geometry -------------------------------------------------------------------------------------------
__global__ void positions_kernel(Plan P, u32 n_lane) {
  const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P.n_wf) return;
  const u32 w = (u32)(P.sort_out[p] & 0x7FFFFFFFull);
  P.perm[p] = w;
  P.inv[w] = p;
  const i32* wi = P.wf_info;
  const u64 nw = P.n_wf;
  u64 v[kGeo];
  v[GV_LEN] = (u64)wi[WI_COUNT * nw + w];
  const int caps[8] = {WI_ACT, WI_TIMER, WI_CHILD, WI_RC, WI_SIG, WI_VH, WI_RP, WI_TASKS};
  for (int t = 0; t < 8; ++t) {
    const i32 c = wi[caps[t] * nw + w];
    v[GV_CAP0 + t] = c > 0 ? (u64)c : 0;
  }
  v[GV_ACT_SIDE] = (u64)wi[WI_ACT * nw + w];
  v[GV_START_SIDE] = (u64)wi[WI_STARTED * nw + w];
  if (p >= n_lane) {
    for (int k = 0; k < kGeo; ++k) P.tvals[(u64)k * nw + (p - n_lane)] = v[k];
  }
}

// one wavefront per group: the maxima of its 64 lanes (padding lanes count 0)
__global__ void group_max_kernel(Plan P, u32 n_lane, u32 n_groups) {
  const u32 g = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (g >= n_groups) return;
  const u32 lane = threadIdx.x & 63;
  const u32 p = g * 64 + lane;
  const i32* wi = P.wf_info;
  const u64 nw = P.n_wf;
  const int src[kGeo] = {WI_COUNT, WI_ACT, WI_TIMER, WI_CHILD, WI_RC, WI_SIG, WI_VH, WI_RP, WI_TASKS, WI_ACT, WI_STARTED};
  for (int k = 0; k < kGeo; ++k) {
    i32 v = 0;
    if (p < n_lane) {
      v = wi[src[k] * nw + P.perm[p]];
      if (v < 0) v = 0;
    }
    for (int o = 32; o > 0; o >>= 1) {
      const i32 x = __shfl_xor(v, o, 64);
      v = x > v ? x : v;
    }
    if (lane == 0) P.gvals[(u64)k * n_groups + g] = (u64)v * 64;
  }
}

__global__ void summary_kernel(Plan P, u32 n_lane, u32 n_groups, u32 n_tail, crr_ingest_summary* S) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const u64 NB = P.n_blobs + 1;
  S->err = 0;
  S->reserved0 = 0;
  S->err_blob = -1;
  const u64 e = *P.err;
  if (e != ~0ull) {
    S->err = -(i32)(e & 0xff);
    S->err_blob = (i64)(e >> 8);
  }
  S->n_events = P.off[0 * NB + P.n_blobs];
  if (S->err == 0 && (S->n_events > P.max_events || P.off[1 * NB + P.n_blobs] > P.max_events)) S->err = kErrScratch;
  S->n_wf = P.n_wf;
  if (S->err) return;   // nothing past the decode is valid
  auto gtot = [&](int k) { return P.gpre[(u64)k * (n_groups + 1) + n_groups]; };
  auto ttot = [&](int k) { return P.tpre[(u64)k * (n_tail + 1) + n_tail]; };
  S->n_slots = gtot(GV_LEN) + ttot(GV_LEN);
  for (int t = 0; t < 8; ++t) S->table_rows[t] = gtot(GV_CAP0 + t) + ttot(GV_CAP0 + t);
  // _interleave_side keeps the canonical array when no event references it (the 1-record placeholder)
  const u64 as = gtot(GV_ACT_SIDE) + ttot(GV_ACT_SIDE), ss = gtot(GV_START_SIDE) + ttot(GV_START_SIDE);
  S->n_act_side = as > 0 ? as : 1;
  S->n_start_side = ss > 0 ? ss : 1;
  S->n_reset_keys = P.off[1 * NB + P.n_blobs];   // (0: the caller's buffer holds flatten's [0] placeholder)
  S->arena_bytes = P.arena_off[P.n_wf];
  S->n_wf = P.n_wf;
  S->wave_begin = n_lane;
  // segment boundaries on group boundaries, rounded down (flatten.interleave)
  u32 c = 0, prev = 0;
  for (int k = 0; k < kWide; ++k) {
    c += P.counters[C_TIER0 + k];
    u32 b = (c == n_lane) ? n_lane : (c / 64) * 64;
    if (k > 0 && b < prev) b = prev;
    S->tiers[k] = b;
    prev = b;
  }
  S->tiers[5] = P.n_wf - P.counters[C_N_BIG];
  S->has_new_run = P.counters[C_NEW_RUN] ? 1u : 0u;
  S->lds_small_tail = P.counters[C_SMALL_TAIL_BAD] == 0 ? 1u : 0u;
  if (P.resume) {   // the tiering, output tables and tokens are the loaded layout's (cadence_ingest.h)
    for (int t = 0; t < 8; ++t) S->table_rows[t] = 0;
    for (int k = 0; k < 6; ++k) S->tiers[k] = 0;
    S->arena_bytes = 0;
  }
}

// resume: device position p is blob-batch workflow p (positions_kernel reads the order from sort_out)
__global__ void identity_order_kernel(Plan P) {
  const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < P.n_wf) P.sort_out[p] = p;
}

// ---- layout -----------------------------------------------------------------------------------------------
struct Dst {
  crr_events ev;
  crr_activity_side* act;
  crr_start_side* start;
  u32* reset_keys;
  u8* arena;
  crr_workflow* wf;
};

// one event (or pad) slot; side records follow their events (_interleave_side)
// x0: the workflow's first canonical slot (P.off at its first blob)
__device__ __forceinline__ void put_slot(const Plan& P, const Dst& D, u64 dst, u64 x0, i64 k, bool real,
                                         u64 side_act_base, u64 side_start_base, u64 side_stride, u32 lane) {
  u8* et = const_cast<u8*>(D.ev.etype);
  i64* id = const_cast<i64*>(D.ev.event_id);
  i64* ver = const_cast<i64*>(D.ev.version);
  i64* ts = const_cast<i64*>(D.ev.timestamp);
  i64* task = const_cast<i64*>(D.ev.task_id);
  i64* ref = const_cast<i64*>(D.ev.ref);
  u32* key = const_cast<u32*>(D.ev.key);
  i32* aux = const_cast<i32*>(D.ev.aux);
  if (!real) {
    et[dst] = (u8)(CRR_EV_PAD | CRR_ETYPE_BATCH_FIRST | CRR_ETYPE_BATCH_LAST);
    id[dst] = 0; ver[dst] = 0; ts[dst] = 0; task[dst] = 0; ref[dst] = 0; key[dst] = 0; aux[dst] = 0;
    return;
  }
  const u64 x = x0 + (u64)k;
  const u8 e = P.etype[x];
  const u32 t = e & CRR_ETYPE_MASK;
  i32 a = P.aux[x];
  if (t == CRR_EV_ACTIVITY_TASK_SCHEDULED) {   // aux: the record's ordinal in the workflow (wf_pass)
    const u64 ni = side_act_base + (u64)a * side_stride + lane;
    D.act[ni] = P.act[x];
    a = (i32)ni;
  } else if (t == CRR_EV_WORKFLOW_EXECUTION_STARTED) {
    const u64 ni = side_start_base + (u64)a * side_stride + lane;
    D.start[ni] = P.start[x];
    a = (i32)ni;
  } else if (t == CRR_EV_ACTIVITY_TASK_STARTED) {
    // CRR_IN_STARTED_AUX (flatten._join_started): the scheduled event d = ID - ScheduledEventID steps back, when
    // it is an ActivityTaskScheduled with that ID -- its side record's interleaved index; else -1
    const i64 ref = P.ref[x];
    const u64 d = (u64)P.id[x] - (u64)ref;
    a = -1;
    if (d >= 1 && d <= (u64)k) {
      const u64 xs = x - d;
      if ((P.etype[xs] & CRR_ETYPE_MASK) == CRR_EV_ACTIVITY_TASK_SCHEDULED && P.id[xs] == ref)
        a = (i32)(side_act_base + (u64)P.aux[xs] * side_stride + lane);
    }
  } else if (t == CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW && a >= 0 && (u32)a < P.n_wf) {
    a = (i32)P.inv[a];   // the new-run history's device position
  }
  et[dst] = e; id[dst] = P.id[x]; ver[dst] = P.ver[x]; ts[dst] = P.ts[x]; task[dst] = P.task[x];
  ref[dst] = P.ref[x]; key[dst] = P.key[x]; aux[dst] = a;
}

__global__ void layout_groups_kernel(crr_blob_batch in, Plan P, Dst D, u32 n_lane, u32 n_groups) {
  const u32 g = blockIdx.x;
  if (g >= n_groups) return;
  const u64 glen = P.gvals[(u64)GV_LEN * n_groups + g] / 64;   // (still the maxima: prefixes live in gpre)
  const u64 base = P.gpre[(u64)GV_LEN * (n_groups + 1) + g];
  const u64 abase = P.gpre[(u64)GV_ACT_SIDE * (n_groups + 1) + g];
  const u64 sbase = P.gpre[(u64)GV_START_SIDE * (n_groups + 1) + g];
  const u32 lane = threadIdx.x & 63;
  const u32 p = g * 64 + lane;
  const bool have = p < n_lane;
  const u32 w = have ? P.perm[p] : 0;
  const i64 cnt = have ? P.wf_info[WI_COUNT * (u64)P.n_wf + w] : 0;
  const u64 x0 = have ? P.off[in.wf[w].blob_begin] : 0;
  for (u64 k = threadIdx.x / 64; k < glen; k += blockDim.x / 64)
    put_slot(P, D, base + k * 64 + lane, x0, (i64)k, have && (i64)k < cnt, abase, sbase, 64, lane);
}

__global__ void layout_tail_kernel(crr_blob_batch in, Plan P, Dst D, u32 n_lane, u32 n_groups, u32 n_tail) {
  const u32 i = blockIdx.x;   // tail workflow
  if (i >= n_tail) return;
  const u32 p = n_lane + i;
  const u32 w = P.perm[p];
  const u64 lane_slots = P.gpre[(u64)GV_LEN * (n_groups + 1) + n_groups];
  const u64 lane_act = P.gpre[(u64)GV_ACT_SIDE * (n_groups + 1) + n_groups];
  const u64 lane_start = P.gpre[(u64)GV_START_SIDE * (n_groups + 1) + n_groups];
  const u64 base = lane_slots + P.tpre[(u64)GV_LEN * (n_tail + 1) + i];
  const u64 abase = lane_act + P.tpre[(u64)GV_ACT_SIDE * (n_tail + 1) + i];
  const u64 sbase = lane_start + P.tpre[(u64)GV_START_SIDE * (n_tail + 1) + i];
  const i64 cnt = P.wf_info[WI_COUNT * (u64)P.n_wf + w];
  const u64 x0 = P.off[in.wf[w].blob_begin];
  for (i64 k = threadIdx.x; k < cnt; k += blockDim.x) put_slot(P, D, base + k, x0, k, true, abase, sbase, 1, 0);
}

// descriptors (device order) and branch tokens (canonical order)
__global__ void layout_wf_kernel(crr_blob_batch in, Plan P, Dst D, u32 n_lane, u32 n_groups, u32 n_tail) {
  const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P.n_wf) return;
  const u32 w = P.perm[p];
  const crr_blob_wf s = in.wf[w];
  const i32* wi = P.wf_info;
  const u64 nw = P.n_wf;
  crr_workflow d;
  const bool lane_wf = p < n_lane;
  const u32 g = p / 64, lane = p & 63, ti = p - n_lane;
  auto pos = [&](int k) -> u64 {   // this workflow's base in geometry value k's space
    if (lane_wf) return P.gpre[(u64)k * (n_groups + 1) + g] + lane;
    return P.gpre[(u64)k * (n_groups + 1) + n_groups] + P.tpre[(u64)k * (n_tail + 1) + ti];
  };
  auto gcap = [&](int k, int wi_k) -> i32 {
    if (lane_wf) return (i32)(P.gvals[(u64)k * n_groups + g] / 64);
    const i32 c = wi[wi_k * nw + w];
    return c > 0 ? c : 0;
  };
  if (P.resume) {   // the loaded descriptor, continuing with the new events (replication.split_descriptors)
    if (P.res_wf == D.wf) {   // in place: only the per-call fields
      crr_workflow* o = D.wf + p;
      o->ev_begin = (i64)pos(GV_LEN);
      o->ev_count = wi[WI_COUNT * nw + w];
      o->empty_batch_at = wi[WI_EMPTY_AT * nw + w];
      o->flags |= CRR_WF_FLAG_RESUME;
      return;
    }
    d = P.res_wf[p];
    d.ev_begin = (i64)pos(GV_LEN);
    d.ev_count = wi[WI_COUNT * nw + w];
    d.empty_batch_at = wi[WI_EMPTY_AT * nw + w];
    d.flags |= CRR_WF_FLAG_RESUME;
    D.wf[p] = d;
    return;
  }
  d.ev_begin = (i64)pos(GV_LEN);
  d.ev_count = wi[WI_COUNT * nw + w];
  d.empty_batch_at = wi[WI_EMPTY_AT * nw + w];
  d.init_version = s.init_version;
  d.now_ns = s.now_ns;
  const u64 ao = P.arena_off[w];
  d.start_token_off = (u32)ao;
  d.start_token_len = 24u + s.run_id_len + s.branch_id_len;
  if (s.final_token_len != 0xFFFFFFFFu) {
    d.final_token_off = (u32)(ao + d.start_token_len);
    d.final_token_len = s.final_token_len;
    d.rebuild_last_event_id = s.rebuild_last_event_id;
    d.rebuild_last_event_version = s.rebuild_last_event_version;
  } else {
    d.final_token_off = 0;
    d.final_token_len = 0xFFFFFFFFu;
    d.rebuild_last_event_id = 0;
    d.rebuild_last_event_version = 0;
  }
  d.act_base = (i64)pos(GV_CAP0 + 0); d.act_cap = gcap(GV_CAP0 + 0, WI_ACT);
  d.timer_base = (i64)pos(GV_CAP0 + 1); d.timer_cap = gcap(GV_CAP0 + 1, WI_TIMER);
  d.child_base = (i64)pos(GV_CAP0 + 2); d.child_cap = gcap(GV_CAP0 + 2, WI_CHILD);
  d.rc_base = (i64)pos(GV_CAP0 + 3); d.rc_cap = gcap(GV_CAP0 + 3, WI_RC);
  d.sig_base = (i64)pos(GV_CAP0 + 4); d.sig_cap = gcap(GV_CAP0 + 4, WI_SIG);
  d.vh_base = (i64)pos(GV_CAP0 + 5); d.vh_cap = gcap(GV_CAP0 + 5, WI_VH);
  d.rp_base = (i64)pos(GV_CAP0 + 6); d.rp_cap = gcap(GV_CAP0 + 6, WI_RP);
  d.flags = s.flags;
  d.task_base = (i64)pos(GV_CAP0 + 7); d.task_cap = gcap(GV_CAP0 + 7, WI_TASKS);
  d.retention_days = s.retention_days;
  D.wf[p] = d;
  // branch token: 0x59 + HistoryBranch{10 TreeID, 20 BranchID, 30 Ancestors = []} (host_flatten.h branch_token)
  u8* o = D.arena + ao;
  u64 q = 0;
  auto put = [&](u32 v) { o[q++] = (u8)v; };
  auto be32 = [&](u32 v) { put(v >> 24); put(v >> 16); put(v >> 8); put(v); };
  auto copy = [&](u64 off, u32 len) {   // 8 bytes per unaligned load / store, the tail bytewise
    const u8* src = in.strings + off;
    u32 i = 0;
    for (; i + 8 <= len; i += 8) {
      u64 v;
      __builtin_memcpy(&v, src + i, 8);
      __builtin_memcpy(o + q + i, &v, 8);
    }
    for (; i < len; ++i) o[q + i] = src[i];
    q += len;
  };
  put(0x59);
  put(11); put(0); put(10); be32(s.run_id_len);
  copy(s.run_id_off, s.run_id_len);
  put(11); put(0); put(20); be32(s.branch_id_len);
  copy(s.branch_id_off, s.branch_id_len);
  put(15); put(0); put(30); put(12); be32(0);
  put(0);
  if (s.final_token_len != 0xFFFFFFFFu) copy(s.final_token_off, s.final_token_len);
}

}  // namespace crr_ingest

// ---- C ABI ----------------------------------------------------------------------------------------------------
namespace {
using namespace crr_ingest;

struct Carved {
  Plan P;
  size_t bytes;
  crr_ingest_summary* S_dev;
};

size_t sort_tmp_bytes(uint32_t n_wf) {   // hipCUB's radix-sort scratch for n_wf keys
  size_t tmp = 0;
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, (const u64*)nullptr, (u64*)nullptr, (int)(n_wf ? n_wf : 1));
  return tmp;
}

// The scratch layout for a max_events capacity; both calls carve it the same way from scratch_bytes.
Carved carve(void* scratch, uint32_t n_blobs, uint32_t n_wf, uint64_t max_events, size_t sort_tmp) {
  Carved c{};
  const uintptr_t at = reinterpret_cast<uintptr_t>(scratch);
  size_t used = 0;
  auto take = [&](size_t bytes) -> void* {
    void* p = reinterpret_cast<void*>(at + used);
    used += align_up(bytes);
    return p;
  };
  Plan& P = c.P;
  P.n_blobs = n_blobs;
  P.n_wf = n_wf;
  P.max_events = max_events;
  const u64 E = max_events ? max_events : 1;
  const u64 NB = (u64)n_blobs + 1;
  const u64 NW = n_wf ? n_wf : 1;
  P.blob_wf = (u32*)take(4 * NB);
  P.cnt = (u32*)take(4 * 2 * NB);
  P.off = (u64*)take(8 * 2 * NB);
  P.err = (u64*)take(8);
  P.flags = (u32*)take(4);
  u64 max_m = NB > NW + 1 ? NB : NW + 1;
  P.tile = (u64*)take(8 * ((max_m + kTile - 1) / kTile + 1) * kGeo);
  P.etype = (u8*)take(E);
  P.id = (i64*)take(8 * E); P.ver = (i64*)take(8 * E); P.ts = (i64*)take(8 * E); P.task = (i64*)take(8 * E);
  P.ref = (i64*)take(8 * E); P.key = (u32*)take(4 * E); P.aux = (i32*)take(4 * E);
  P.act = (crr_activity_side*)take(sizeof(crr_activity_side) * E);
  P.start = (crr_start_side*)take(sizeof(crr_start_side) * E);
  P.keys = (KeyRef*)take(sizeof(KeyRef) * E);
  P.resets = (KeyRef*)take(sizeof(KeyRef) * E);
  P.reset_ids = (u32*)take(4 * E);
  // per-workflow hash tables: a workflow of n events and r reset points uses <= 4n + 4r + 64 words
  P.table = (u64*)take(8 * (8 * E + 64 * NW));
  P.dom_refs = reinterpret_cast<KeyRef*>(P.table);   // 32 * E <= 64 * E bytes
  P.wf_info = (i32*)take(4 * kWfInfo * NW);
  P.sort_in = (u64*)take(8 * NW);
  P.sort_out = (u64*)take(8 * NW);
  P.sort_tmp_bytes = sort_tmp;
  P.sort_tmp = take(sort_tmp);
  P.perm = (u32*)take(4 * NW);
  P.inv = (u32*)take(4 * NW);
  P.arena_off = (u64*)take(8 * (NW + 1));
  const u64 NG = (NW + 63) / 64;
  P.gvals = (u64*)take(8 * kGeo * NG);
  P.tvals = (u64*)take(8 * kGeo * NW);
  P.gpre = (u64*)take(8 * kGeo * (NG + 1));
  P.tpre = (u64*)take(8 * kGeo * (NW + 1));
  P.counters = (u32*)take(4 * 16);
  c.S_dev = (crr_ingest_summary*)take(sizeof(crr_ingest_summary));
  P.dom_table = (u32*)take(kDomainBytes);
  P.dom_cap = 0;
  c.bytes = used;
  return c;
}

uint64_t max_events_of(size_t scratch_bytes, uint32_t n_blobs, uint32_t n_wf, size_t sort_tmp) {
  // the largest capacity whose carve fits (the size is monotone in it)
  uint64_t lo = 0, hi = 1;
  while (carve(nullptr, n_blobs, n_wf, hi, sort_tmp).bytes <= scratch_bytes && hi < (1ull << 40)) hi <<= 1;
  while (lo + 1 < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (carve(nullptr, n_blobs, n_wf, mid, sort_tmp).bytes <= scratch_bytes) lo = mid; else hi = mid;
  }
  return lo;
}

bool valid_batch(const crr_blob_batch* in) {
  if (!in || !in->blob_off) return false;
  if (in->n_wf && !in->wf) return false;
  if (in->n_blobs && !in->bytes) return false;
  if (reinterpret_cast<uintptr_t>(in->bytes) & 15) return false;   // the 16-byte window loads
  if (in->n_domains != 0xFFFFFFFFu && in->n_domains && (!in->domain_off || !in->domain_len || !in->strings)) return false;
  if (in->n_domains != 0xFFFFFFFFu && (size_t)in->n_domains * 2 * 4 > kDomainBytes) return false;
  if ((in->n_wf || in->n_domains) && !in->strings && in->n_wf) return false;
  if (in->n_wf >= 0x7FFFFFFFu) return false;
  return true;
}

}  // namespace

extern "C" {

size_t crr_ingest_scratch_bytes(uint32_t n_blobs, uint32_t n_wf, uint64_t max_events) {
  return carve(nullptr, n_blobs, n_wf, max_events, sort_tmp_bytes(n_wf)).bytes;
}

}  // extern "C"

namespace {
// the resume inputs into the plan (validated), or none
bool set_resume(Plan& P, const crr_blob_batch* in, const crr_ingest_resume* R) {
  P.resume = 0;
  P.res_wf = nullptr; P.key_begin = nullptr; P.key_count = nullptr; P.key_off = nullptr; P.key_len = nullptr;
  if (!R) return true;
  if (R->wave_begin > in->n_wf) return false;
  if (in->n_wf && (!R->loaded_wf || !R->key_begin || !R->key_count || !R->key_off || !R->key_len)) return false;
  P.resume = 1;
  P.res_wf = R->loaded_wf; P.key_begin = R->key_begin; P.key_count = R->key_count;
  P.key_off = R->key_off; P.key_len = R->key_len;
  return true;
}

int plan_impl(const crr_blob_batch* in, const crr_ingest_resume* R, void* scratch, size_t scratch_bytes,
              crr_ingest_summary* summary, void* stream) {
  if (!valid_batch(in) || !scratch || !summary) return -1;
  if (in->n_wf == 0 && in->n_blobs > 0) return -1;   // blobs no workflow owns
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  crr_internal::StreamDevice on_dev_(s);
  if (!on_dev_.ok) return (int)hipErrorInvalidHandle;
  const size_t stmp = sort_tmp_bytes(in->n_wf);
  const uint64_t max_events = max_events_of(scratch_bytes, in->n_blobs, in->n_wf, stmp);
  if (max_events == 0) return -1;
  Carved c = carve(scratch, in->n_blobs, in->n_wf, max_events, stmp);
  Plan P = c.P;
  if (!set_resume(P, in, R)) return -1;
  const u32 nb = in->n_blobs, nw = in->n_wf;
  const u64 NB = (u64)nb + 1;
  u32 dom_cap = 0;
  if (in->n_domains != 0xFFFFFFFFu && in->n_domains) {
    dom_cap = 16;
    while (dom_cap < 2 * in->n_domains) dom_cap <<= 1;
  }
  P.dom_cap = dom_cap;
  hipError_t e;
  if (dom_cap) {
    if ((e = hipMemsetAsync(P.dom_table, 0, 4 * (size_t)dom_cap, s)) != hipSuccess) return (int)e;
    hipLaunchKernelGGL(domains_build_kernel, dim3((in->n_domains + kBlock - 1) / kBlock), dim3(kBlock), 0, s, *in,
                       P.dom_table, dom_cap);
  }
  const unsigned gb = (nb + kBlock - 1) / kBlock, gw = (nw + kBlock - 1) / kBlock;
  // A: event counts, the decode, reset points, the per-workflow pass, the device order.  A header count
  // that was wrong (hand-made blobs) shows in `flags` at the readback below (every pass after the decode
  // skips the plan meanwhile): then all of A again, the counts from walking every blob.
  u32 n_lane = 0, flags = 0;
  u64 err = 0, n_events = 0, n_resets = 0;
  for (int full = 0; full < 2; ++full) {
    if ((e = hipMemsetAsync(P.err, 0xff, 8, s)) != hipSuccess) return (int)e;
    if ((e = hipMemsetAsync(P.flags, 0, 4, s)) != hipSuccess) return (int)e;
    if ((e = hipMemsetAsync(P.counters, 0, 4 * 16, s)) != hipSuccess) return (int)e;
    if (nw) hipLaunchKernelGGL(blob_wf_kernel, dim3(gw), dim3(kBlock), 0, s, *in, P.blob_wf, P.err);
    if (nb && !full) hipLaunchKernelGGL(blob_head_quick_kernel, dim3(gb), dim3(kBlock), 0, s, *in, P);
    if (nb) hipLaunchKernelGGL(blob_head_kernel, dim3(gb), dim3(kBlock), 0, s, *in, P, full);
    multi_scan<u32>(P.cnt, nb, nb, 1, P.tile, P.off, NB, s);
    if (nb) hipLaunchKernelGGL(blob_decode_kernel, dim3((nb + 63) / 64), dim3(64), 0, s, *in, P);
    if (nb) hipLaunchKernelGGL(blob_decode_general_kernel, dim3(gb), dim3(kBlock), 0, s, *in, P);
    if (nb && dom_cap) hipLaunchKernelGGL(domain_resolve_kernel, dim3(2048), dim3(kBlock), 0, s, *in, P);
    multi_scan<u32>(P.cnt + nb, nb, nb, 1, P.tile, P.off + NB, NB, s);   // previous reset points per blob
    if (nb) hipLaunchKernelGGL(reset_refs_kernel, dim3(gb), dim3(kBlock), 0, s, *in, P);
    if (nw) {
      const u32 blocks = (nw + kWfWaveBlock / 64 - 1) / (kWfWaveBlock / 64);
      hipLaunchKernelGGL(wf_pass_wave_kernel, dim3(blocks < 2048 ? blocks : 2048), dim3(kWfWaveBlock), 0, s, *in, P);
      hipLaunchKernelGGL(wf_pass_kernel, dim3(gw), dim3(kBlock), 0, s, *in, P);
    }
    multi_scan<u64>(P.arena_off, nw, nw, 1, P.tile, P.arena_off, (u64)nw + 1, s);
    if (nw && P.resume) {
      hipLaunchKernelGGL(identity_order_kernel, dim3(gw), dim3(kBlock), 0, s, P);
    } else if (nw) {
      size_t tmp = P.sort_tmp_bytes;
      if ((e = hipcub::DeviceRadixSort::SortKeys(P.sort_tmp, tmp, P.sort_in, P.sort_out, (int)nw, 0, 64, s)) != hipSuccess)
        return (int)e;
    }
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    // the lane / tail split sizes the geometry launches
    if ((e = hipMemcpyAsync(&n_lane, P.counters + C_N_LANE, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
    if ((e = hipMemcpyAsync(&err, P.err, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
    if ((e = hipMemcpyAsync(&n_events, P.off + nb, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
    if ((e = hipMemcpyAsync(&n_resets, P.off + NB + nb, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
    if ((e = hipMemcpyAsync(&flags, P.flags, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return (int)e;
    if (!flags) break;
  }
  if (P.resume) n_lane = R->wave_begin;   // the loaded layout's split
  const bool failed = err != ~0ull || n_lane > nw || n_events > max_events || n_resets > max_events;
  const u32 n_groups = failed ? 0 : (n_lane + 63) / 64, n_tail = failed ? 0 : nw - n_lane;
  // B: geometry and the summary (after a failed decode only the error and the counts)
  if (nw && !failed) hipLaunchKernelGGL(positions_kernel, dim3(gw), dim3(kBlock), 0, s, P, n_lane);
  if (n_groups) hipLaunchKernelGGL(group_max_kernel, dim3((n_groups + 3) / 4), dim3(256), 0, s, P, n_lane, n_groups);
  if (!failed) {
    multi_scan<u64>(P.gvals, n_groups, n_groups, kGeo, P.tile, P.gpre, (u64)n_groups + 1, s);
    multi_scan<u64>(P.tvals, nw, n_tail, kGeo, P.tile, P.tpre, (u64)n_tail + 1, s);
  }
  hipLaunchKernelGGL(summary_kernel, dim3(1), dim3(64), 0, s, P, n_lane, n_groups, n_tail, c.S_dev);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  if ((e = hipMemcpyAsync(summary, c.S_dev, sizeof(crr_ingest_summary), hipMemcpyDeviceToHost, s)) != hipSuccess)
    return (int)e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return (int)e;
  return 0;
}

int layout_impl(const crr_blob_batch* in, const crr_ingest_resume* R, void* scratch, size_t scratch_bytes,
                const crr_ingest_summary* S, const crr_inputs* dst, uint32_t* perm, void* stream) {
  if (!valid_batch(in) || !scratch || !S || !dst || S->err || S->n_wf != in->n_wf) return -1;
  if (R && S->wave_begin != R->wave_begin) return -1;
  if (!dst->wf || !dst->act_side || !dst->start_side || !dst->reset_keys || !dst->arena) return -1;
  const crr_events& ev = dst->ev;
  if (!ev.etype || !ev.event_id || !ev.version || !ev.timestamp || !ev.task_id || !ev.ref || !ev.key || !ev.aux) return -1;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  crr_internal::StreamDevice on_dev_(s);
  if (!on_dev_.ok) return (int)hipErrorInvalidHandle;
  const size_t stmp = sort_tmp_bytes(in->n_wf);
  const uint64_t max_events = max_events_of(scratch_bytes, in->n_blobs, in->n_wf, stmp);
  Carved c = carve(scratch, in->n_blobs, in->n_wf, max_events, stmp);
  Plan P = c.P;
  if (!set_resume(P, in, R)) return -1;
  const u32 nw = in->n_wf, n_lane = S->wave_begin, n_groups = (n_lane + 63) / 64, n_tail = nw - n_lane;
  Dst D;
  D.ev = ev;
  D.act = const_cast<crr_activity_side*>(dst->act_side);
  D.start = const_cast<crr_start_side*>(dst->start_side);
  D.reset_keys = const_cast<u32*>(dst->reset_keys);
  D.arena = const_cast<u8*>(dst->arena);
  D.wf = const_cast<crr_workflow*>(dst->wf);
  hipError_t e;
  // side records no event references stay zero, like flatten's zero-filled arrays
  if ((e = hipMemsetAsync(D.act, 0, S->n_act_side * sizeof(crr_activity_side), s)) != hipSuccess) return (int)e;
  if ((e = hipMemsetAsync(D.start, 0, S->n_start_side * sizeof(crr_start_side), s)) != hipSuccess) return (int)e;
  // up to 16 wavefronts per group of 64 lanes (a wavefront writes one slot row of the group per step): as many
  // as the mean group length uses -- short groups (a replication task's batch: 1-3 rows) take one or two
  const u64 lane_rows = n_groups ? S->n_slots / 64 : 0;   // (the tail counted too: an upper bound)
  u32 waves = n_groups ? (u32)((lane_rows + n_groups - 1) / n_groups) : 1;
  waves = waves < 1 ? 1 : waves > 16 ? 16 : waves;
  if (n_groups) hipLaunchKernelGGL(layout_groups_kernel, dim3(n_groups), dim3(64 * waves), 0, s, *in, P, D, n_lane, n_groups);
  if (n_tail) hipLaunchKernelGGL(layout_tail_kernel, dim3(n_tail), dim3(kBlock), 0, s, *in, P, D, n_lane, n_groups, n_tail);
  if (nw) hipLaunchKernelGGL(layout_wf_kernel, dim3((nw + kBlock - 1) / kBlock), dim3(kBlock), 0, s, *in, P, D, n_lane,
                             n_groups, n_tail);
  // reset_keys: the interned previous reset points in canonical order ([0] when there are none)
  if ((e = hipMemsetAsync(D.reset_keys, 0, 4, s)) != hipSuccess) return (int)e;
  if (S->n_reset_keys &&
      (e = hipMemcpyAsync(D.reset_keys, P.reset_ids, 4 * S->n_reset_keys, hipMemcpyDeviceToDevice, s)) != hipSuccess)
    return (int)e;
  if (perm && nw && (e = hipMemcpyAsync(perm, P.perm, 4ull * nw, hipMemcpyDeviceToDevice, s)) != hipSuccess) return (int)e;
  return (int)hipGetLastError();
}
}  // namespace

extern "C" {

int crr_ingest_plan(const crr_blob_batch* in, void* scratch, size_t scratch_bytes, crr_ingest_summary* summary,
                    void* stream) {
  return plan_impl(in, nullptr, scratch, scratch_bytes, summary, stream);
}

int crr_ingest_layout(const crr_blob_batch* in, void* scratch, size_t scratch_bytes, const crr_ingest_summary* S,
                      const crr_inputs* dst, uint32_t* perm, void* stream) {
  return layout_impl(in, nullptr, scratch, scratch_bytes, S, dst, perm, stream);
}

int crr_ingest_plan_resume(const crr_blob_batch* in, const crr_ingest_resume* resume, void* scratch,
                           size_t scratch_bytes, crr_ingest_summary* summary, void* stream) {
  if (!resume) return -1;
  return plan_impl(in, resume, scratch, scratch_bytes, summary, stream);
}

int crr_ingest_layout_resume(const crr_blob_batch* in, const crr_ingest_resume* resume, void* scratch,
                             size_t scratch_bytes, const crr_ingest_summary* S, const crr_inputs* dst, void* stream) {
  if (!resume) return -1;
  return layout_impl(in, resume, scratch, scratch_bytes, S, dst, nullptr, stream);
}

}  // extern "C"
