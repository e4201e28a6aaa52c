// host_flatten.h -- the host side's flattening of HistoryEvents into the engine's SoA input
// (crr_inputs), shared by the thriftrw decoder (history_decode.cpp) and the native synthetic
// generator (synth_native.cpp).  Private to libcadence_host.so.
//
// Per workflow: events are appended batch by batch to a Chunk (columns, side records, per-event key
// strings, branch tokens, descriptors); ActivityID / TimerID / BinaryChecksum strings are interned to
// per-workflow u32 keys (string equality preserved); slot-table capacities are exact upper bounds of
// the live sets (insert counts).  Byte-identical to cadence_amd/flatten.py on the same events.
#pragma once

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "cadence_decode.h"

namespace crr_host {

using i64 = int64_t;
using i32 = int32_t;
using u32 = uint32_t;

// ---- the fields one event contributes ----------------------------------------------------------------
struct Attr {
  i64 ref = 0;
  i32 aux = 0;
  std::string key;           // ActivityID / TimerID / BinaryChecksum
  bool has_key = false;
  std::string domain;        // attributes.Domain / ParentWorkflowDomain
  bool domain_id_set = false;  // ParentWorkflowDomainID given: no domain-cache lookup (state_builder.go:137-147)
  // ActivityTaskScheduled
  i32 s2s = 0, s2c = 0, st2c = 0, hb = 0, has_retry = 0, expiration = 0;
  // WorkflowExecutionStarted
  i32 task_s2c = 0, exec_s2c = 0, backoff = 0, initiator = CRR_INITIATOR_NIL, attempt = 0;
  i64 expiration_ts = 0;
  int prev_mode = -1;        // -1: PrevAutoResetPoints nil, -2: Points nil, 0: list
  std::vector<std::string> prev;
  i32 new_run = -1;          // WorkflowExecutionContinuedAsNew: workflow index of the new-run history
};

struct Event {
  i64 id = 0, ts = 0, ver = 0, task = 0;
  i32 type = 0;
  Attr a;
};

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

// NewHistoryBranchTokenByBranchID (dataManagerInterfaces.go:2899-2910): 0x59 + thrift binary
// HistoryBranch{10 TreeID string, 20 BranchID string, 30 Ancestors list<struct> = []}.
inline void branch_token(std::vector<uint8_t>& out, const char* tree, const char* branch) {
  auto be32 = [&](u32 v) { for (int s = 24; s >= 0; s -= 8) out.push_back((uint8_t)(v >> s)); };
  const size_t nt = tree ? strlen(tree) : 0, nb = branch ? strlen(branch) : 0;
  out.push_back(0x59);
  out.push_back(11); out.push_back(0); out.push_back(10); be32((u32)nt);
  out.insert(out.end(), tree, tree + nt);
  out.push_back(11); out.push_back(0); out.push_back(20); be32((u32)nb);
  out.insert(out.end(), branch, branch + nb);
  out.push_back(15); out.push_back(0); out.push_back(30); out.push_back(12); be32(0);
  out.push_back(0);
}

// Host-injected inputs of one workflow (crr_wf_source without the blob range).
struct WfMeta {
  i64 init_version = 0, now_ns = 0;
  const char* run_id = "";
  const char* branch_id = "";
  const uint8_t* final_token = nullptr;
  u32 final_token_len = 0;
  i64 rebuild_last_event_id = 0, rebuild_last_event_version = 0;
  i32 flags = 0, retention_days = 1;
};

// Appends one workflow's events, batch by batch, to a Chunk.
class WfFlattener {
 public:
  WfFlattener(Chunk& k, const std::unordered_set<std::string>* known) : k_(k), known_(known) {
    intern_.emplace(std::string(), 0u);
    begin_ = (i64)k_.etype.size();
  }
  int domain_status(const std::string& name) const {
    if (name.empty()) return CRR_DOMAIN_NOT_SET;
    if (!known_ || known_->count(name)) return CRR_DOMAIN_RESOLVED;
    return CRR_DOMAIN_UNKNOWN;
  }
  void batch_begin() {
    n_in_batch_ = 0;
    batch_begin_ = (i64)k_.etype.size();
  }
  void add(const Event& e) {
    const i32 t = e.type;
    const bool valid = t >= 0 && t < CRR_EV_TYPE_COUNT;
    k_.etype.push_back((uint8_t)(valid ? t : CRR_EV_PAD - 1));
    k_.id.push_back(e.id);
    k_.ver.push_back(e.ver);
    k_.ts.push_back(e.ts);
    k_.task.push_back(e.task);
    if (!have_ver_ || e.ver > last_ver_) { ++vh_items_; last_ver_ = e.ver; have_ver_ = true; }
    n_tasks_ += valid ? kTasksPerEvent[t] : 0;
    i64 ref = 0;
    u32 key = 0;
    i32 aux = 0;
    const std::string* ks = nullptr;
    const Attr& a = e.a;
    switch (valid ? t : -1) {
      case CRR_EV_WORKFLOW_EXECUTION_STARTED: {
        crr_start_side ss;
        std::memset(&ss, 0, sizeof(ss));
        if (a.prev_mode == -1) { ss.prev_reset_key_off = 0; ss.prev_reset_count = -1; }
        else if (a.prev_mode == -2) { ss.prev_reset_key_off = 0; ss.prev_reset_count = -2; }
        else {
          ss.prev_reset_key_off = (u32)k_.reset_keys.size();
          ss.prev_reset_count = (i32)a.prev.size();
          for (const auto& p : a.prev) k_.reset_keys.push_back(key_of(p));
          max_prev_ = std::max<i64>(max_prev_, (i64)a.prev.size());
        }
        ss.decision_start_to_close = a.task_s2c;
        ss.workflow_timeout = a.exec_s2c;
        ss.first_decision_backoff = a.backoff;
        ss.initiator = a.initiator;
        ss.attempt = a.attempt;
        ss.expiration_ns = a.expiration_ts;
        ss.parent_domain_status = a.domain_id_set ? CRR_DOMAIN_NOT_SET : domain_status(a.domain);
        k_.start.push_back(ss);
        aux = (i32)k_.start.size() - 1;
        ++n_started_;
        break;
      }
      case CRR_EV_DECISION_TASK_SCHEDULED: ref = a.ref; aux = a.aux; break;
      case CRR_EV_DECISION_TASK_STARTED: ref = a.ref; break;
      case CRR_EV_DECISION_TASK_COMPLETED: ref = a.ref; ks = &a.key; key = key_of(a.key); ++n_dtc_; break;
      case CRR_EV_DECISION_TASK_TIMED_OUT: aux = a.aux; break;
      case CRR_EV_ACTIVITY_TASK_SCHEDULED: {
        ks = &a.key;
        key = key_of(a.key);
        crr_activity_side as;
        std::memset(&as, 0, sizeof(as));
        as.schedule_to_start = a.s2s; as.schedule_to_close = a.s2c; as.start_to_close = a.st2c;
        as.heartbeat = a.hb; as.has_retry_policy = a.has_retry; as.expiration_interval = a.expiration;
        as.domain_status = domain_status(a.domain);
        k_.act.push_back(as);
        aux = (i32)k_.act.size() - 1;
        ++n_act_;
        break;
      }
      case CRR_EV_ACTIVITY_TASK_STARTED: case CRR_EV_ACTIVITY_TASK_COMPLETED: case CRR_EV_ACTIVITY_TASK_FAILED:
      case CRR_EV_ACTIVITY_TASK_TIMED_OUT: case CRR_EV_ACTIVITY_TASK_CANCELED:
        ref = a.ref; break;
      case CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED: ks = &a.key; key = key_of(a.key); break;
      case CRR_EV_TIMER_STARTED: ks = &a.key; key = key_of(a.key); ref = a.ref; ++n_timer_; break;
      case CRR_EV_TIMER_FIRED: case CRR_EV_TIMER_CANCELED: ks = &a.key; key = key_of(a.key); break;
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED: aux = domain_status(a.domain); ++n_child_; break;
      case CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED: aux = domain_status(a.domain); ++n_rc_; break;
      case CRR_EV_SIGNAL_EXTERNAL_INITIATED: aux = domain_status(a.domain); ++n_sig_; break;
      case CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED: case CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT:
      case CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED: case CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED:
      case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED: case CRR_EV_SIGNAL_EXTERNAL_FAILED:
      case CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED:
        ref = a.ref; break;
      case CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW: aux = a.new_run; break;
      default: break;
    }
    k_.ref.push_back(ref);
    k_.key.push_back(key);
    k_.aux.push_back(aux);
    k_.key_off.push_back((u32)k_.key_arena.size());
    k_.key_len.push_back(ks ? (u32)ks->size() : 0u);
    if (ks) k_.key_arena.append(*ks);
    ++n_in_batch_;
  }
  void batch_end() {
    if (n_in_batch_ == 0) {  // an empty batch: ApplyEvents' history-size-zero error (state_builder.go:98-100)
      if (empty_at_ < 0) empty_at_ = (i32)(batch_begin_ - begin_);
      return;
    }
    n_tasks_ += 2;  // the batch's timer epilogue
    k_.etype[batch_begin_] |= CRR_ETYPE_BATCH_FIRST;
    k_.etype.back() |= CRR_ETYPE_BATCH_LAST;
  }
  // n_batches == 0: the history itself is empty (ApplyEvents with an empty history)
  void finish(const WfMeta& m, uint32_t n_batches) {
    crr_workflow d;
    std::memset(&d, 0, sizeof(d));
    const i64 n = (i64)k_.etype.size() - begin_;
    if (n_batches == 0) empty_at_ = 0;
    d.ev_begin = begin_;
    d.ev_count = (i32)n;
    d.empty_batch_at = empty_at_;
    d.init_version = m.init_version;
    d.now_ns = m.now_ns;
    d.start_token_off = (u32)k_.arena.size();
    branch_token(k_.arena, m.run_id ? m.run_id : "", m.branch_id ? m.branch_id : "");
    d.start_token_len = (u32)(k_.arena.size() - d.start_token_off);
    if (m.final_token) {
      d.final_token_off = (u32)k_.arena.size();
      d.final_token_len = m.final_token_len;
      k_.arena.insert(k_.arena.end(), m.final_token, m.final_token + m.final_token_len);
      d.rebuild_last_event_id = m.rebuild_last_event_id;
      d.rebuild_last_event_version = m.rebuild_last_event_version;
    } else {
      d.final_token_off = 0;
      d.final_token_len = 0xFFFFFFFFu;
    }
    d.act_cap = (i32)n_act_; d.timer_cap = (i32)n_timer_; d.child_cap = (i32)n_child_;
    d.rc_cap = (i32)n_rc_; d.sig_cap = (i32)n_sig_; d.vh_cap = (i32)vh_items_;
    d.rp_cap = (i32)(max_prev_ * std::max<i64>(1, n_started_) + n_dtc_);
    d.flags = m.flags;
    // + RefreshTasks' search-attributes task (its other tasks fit the replay's bound)
    d.task_cap = (i32)n_tasks_ + ((m.flags & CRR_WF_FLAG_REFRESH_TASKS) ? 1 : 0);
    d.retention_days = m.retention_days;
    k_.wf.push_back(d);
  }

 private:
  u32 key_of(const std::string& s) {
    auto it = intern_.find(s);
    if (it != intern_.end()) return it->second;
    const u32 v = (u32)intern_.size();
    intern_.emplace(s, v);
    return v;
  }
  Chunk& k_;
  const std::unordered_set<std::string>* known_;
  std::unordered_map<std::string, u32> intern_;
  i64 begin_ = 0, batch_begin_ = 0;
  i32 empty_at_ = -1, n_in_batch_ = 0;
  i64 n_act_ = 0, n_timer_ = 0, n_child_ = 0, n_rc_ = 0, n_sig_ = 0, n_dtc_ = 0, n_started_ = 0, vh_items_ = 0;
  i64 max_prev_ = 0, n_tasks_ = 0;
  bool have_ver_ = false;
  i64 last_ver_ = 0;
};

template <class T>
void append(std::vector<T>& dst, const std::vector<T>& src) { dst.insert(dst.end(), src.begin(), src.end()); }

// Concatenates per-thread chunks (event, side-record, key / token / reset-key offsets fixed up) and
// assigns the canonical slot-table bases (prefix sums of the per-workflow capacities).
inline void concat_chunks(std::vector<Chunk>& chunks, Chunk& a, uint64_t table_rows[8]) {
  for (auto& k : chunks) {
    const i64 ev0 = (i64)a.etype.size();
    const i32 act0 = (i32)a.act.size(), st0 = (i32)a.start.size();
    const u32 rk0 = (u32)a.reset_keys.size(), ar0 = (u32)a.arena.size(), ka0 = (u32)a.key_arena.size();
    const i32 wf0 = (i32)a.wf.size();
    (void)wf0;
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
    k = Chunk();  // release chunk memory early
  }
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
  for (int j = 0; j < 8; ++j) table_rows[j] = (uint64_t)base[j];
}

}  // namespace crr_host

struct crr_decoded {
  crr_host::Chunk all;
  uint64_t table_rows[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};
