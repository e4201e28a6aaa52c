"""Profiling aid (not product code): where the wavefront path's time goes, by removing one part at a
time.  Builds variant libraries from patched copies of replay_kernel.hip (results are wrong by design;
only the kernel times are read, tools/prof_longtail.py --lib):

    python tools/wave_split.py noepi noside nowalk      ->  tools/variants/<name>.so

  noepi   the batch epilogue (timer re-selection) skipped
  noside  ActivityTaskScheduled's side record not loaded (a constant instead)
  nowalk  fast chunks visit nothing (only the lane-parallel passes run)
  bare    no chunk is walked or resolved (chunk loads, the VH prologue and the chunk bookkeeping only)
  noops   fast chunks visit their lanes but apply no map operation (visit and epilogue costs only)
  nosort  GlobalTables::finalize without its selection sorts (passive replication, tools/prof_replication.py)
  noreread  compact tiers' ActivityTaskStarted without re-reading its scheduled event (config 3)
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PATCHES = {
    "noepi": [("          T.epilogue(L, G, K);  // :634-640 GenerateActivityTimerTasks / GenerateUserTimerTasks\n"
               "          if (!fast) {",
               "          if (0) T.epilogue(L, G, K);\n          if (!fast) {")],
    "noside": [("        as = in.act_side[ev.aux()];\n        if (as.domain_status == CRR_DOMAIN_UNKNOWN) FAIL",
                "        as.domain_status = 1; as.has_retry_policy = 0; as.schedule_to_start = 10; "
                "as.schedule_to_close = 20; as.start_to_close = 10; as.heartbeat = 0;\n"
                "        if (as.domain_status == CRR_DOMAIN_UNKNOWN) FAIL")],
    "nowalk": [("        vm = (OPS | EB) & le(stop - 1);", "        vm = 0;")],
    "noops": [("        if (!fast || ((OPS >> j) & 1)) {\n          const int rc = apply_event(",
               "        if (!fast) {\n          const int rc = apply_event(")],
    "bare": [("      u64 vm = le(lim - 1), OPS = 0;", "      u64 vm = 0, OPS = 0;"),
             ("      const bool fast = !K.on &&", "      const bool fast = false && !K.on &&")],
    # lane path over HBM rows (resume / wide segment): finalize without the in-place selection sorts
    "nosort": [("    for (i32 i = 0; i < n; ++i) {\n      i32 best = -1;\n      i64 bid = 0;",
                "    for (i32 i = 0; i < 0 * n; ++i) {\n      i32 best = -1;\n      i64 bid = 0;")],
    # compact tiers: ActivityTaskStarted without the re-reads of its scheduled event (aux -> side record, time)
    "noreread": [("    const crr_activity_side sa = in->act_side[in->ev.aux[six]];\n"
                  "    i64 ct = add_seconds(in->ev.timestamp[six], sa.schedule_to_close);",
                  "    crr_activity_side sa{}; sa.schedule_to_close = 20; sa.start_to_close = 10; (void)six;\n"
                  "    i64 ct = add_seconds(ev.ts(), sa.schedule_to_close);")],
    # round 5 (config 3 traffic attribution): the compact tiers' ActivityTaskStarted without its re-read of the
    # scheduled event (aux -> side record, timestamp) ...
    "noreread2": [("      const i64 six = ix(ss);\n      const crr_activity_side sa = in->act_side[in->ev.aux[six]];\n"
                   "      sched_t = in->ev.timestamp[six]; s2c = sa.schedule_to_close; st2c = sa.start_to_close; hb = sa.heartbeat;",
                   "      (void)ss;\n      sched_t = ev.ts(); s2c = 20; st2c = 10; hb = 0;")],
    # ... and finalize building a new activity row without re-reading its scheduled / started events
    "nofinread": [("      const crr_activity_side as = in->act_side[in->ev.aux[ix(ss)]];\n      crr_activity_row r;",
                   "      crr_activity_side as{}; as.schedule_to_start = 1; as.schedule_to_close = 2; as.start_to_close = 3;\n"
                   "      crr_activity_row r;"),
                  ("      r.scheduled_time = ev_ts(ss);\n", "      r.scheduled_time = (i64)ss;\n"),
                  ("      r.started_time = started ? ev_ts(st) : CRR_ZERO_TIME;\n",
                   "      r.started_time = started ? (i64)st : CRR_ZERO_TIME;\n")],
    # passive replication in the compact tiers (CompactTables<TIER, true>), tools/prof_replication.py --lib:
    # the whole step without the checksum
    "rnocrc": [("  const bool want_crc = L.status == CRR_OK;", "  const bool want_crc = false;")],
    # resumed compact workflows stopping early (the exec row written back as loaded): after the exec-row
    # read / after the arena load -- the floor of each part of the step
    "rnop": [("      const crr_exec_row X = out.exec[w];\n",
              "      const crr_exec_row X = out.exec[w];\n"
              "      if constexpr (FusedMapOps<P>::value) { out.exec[w] = X; return; }\n")],
    "rload": [("      if (L.status != CRR_OK) goto done_events;  // a loaded state the policy cannot hold: general path\n",
               "      if (L.status != CRR_OK) goto done_events;  // a loaded state the policy cannot hold: general path\n"
               "      if constexpr (FusedMapOps<P>::value) { out.exec[w] = X; return; }\n")],
    # ... without the checksum and the finalize
    "rtail": [("  const bool want_crc = L.status == CRR_OK;", "  const bool want_crc = false;"),
              ("  T.finalize(L, G);\n\n  crr_exec_row R;", "  if (0) T.finalize(L, G);\n\n  crr_exec_row R;")],
    # ... without the finalize (no rows written)
    "rnofin": [("  T.finalize(L, G);\n\n  crr_exec_row R;", "  if (0) T.finalize(L, G);\n\n  crr_exec_row R;")],
}


def main():
    for name in sys.argv[1:]:
        s = open(os.path.join(ROOT, "cadence_amd", "csrc", "replay_kernel.hip")).read()
        for old, new in PATCHES[name]:
            if old not in s:
                raise SystemExit(f"{name}: patch point not found: {old[:60]!r}")
            s = s.replace(old, new, 1)
        d = tempfile.mkdtemp()
        p = os.path.join(d, "replay_kernel.hip")
        open(p, "w").write(s)
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build_variant.py"), name, "--src=" + p], check=True)


if __name__ == "__main__":
    main()
