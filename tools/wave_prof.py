"""Profiling aid (not product code): cycle split of the wavefront path (replay_tail_kernel, config 4).

Builds tools/variants/waveprof.so from a patched copy of replay_kernel.hip: s_memtime reads around the
parts of each 64-event chunk, summed per wavefront in scalar registers and added (lane 0) into a device
array at the end of every wavefront-path replay; crr_wave_prof() reads it.  The clocks perturb (each read
waits for the wavefront's outstanding LDS operations), so only the split is meaningful.

    python tools/wave_prof.py                # build
    python tools/prof_c4_segments.py --lib tools/variants/waveprof.so --only tail --wave-prof
Buckets (cycles summed over every wavefront-path replay, then counts):
  0 chunk loop total  1 before the walk (VH prologue, lane-parallel passes)  2 walk total  3 map-op visits
  4 other visits (reset points, events of slow chunks)  5 batch epilogues  6 after the walk
  8 chunks  9 map-op visits  10 other visits  11 epilogues  12 replays
  16 + op: cycles of the visits of map operation op (MOP_*), 32 + op: their count
  48..55 (WaveTables sub-buckets): activity epilogue candidate loads, its wave minimum, its update; the
  timer epilogue; act_insert's ActivityID lookup, its free-slot search, its row write; 56 / 57: activity /
  timer epilogue count
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WAVE = "std::is_same<SRC, WaveSource>::value"
PATCHES = [
    # the accumulators, declared with the other per-replay state
    ("  i64 batch_first_id = 0;\n  i32 last_task_step = -1;\n",
     "  i64 batch_first_id = 0;\n  i32 last_task_step = -1;\n"
     "  u64 wp_[48] = {};\n"),
    ("    for (i32 c0 = 0; c0 < n_wave; c0 += 64) {\n      if (c0) src.rotate();\n",
     "    for (i32 c0 = 0; c0 < n_wave; c0 += 64) {\n      const u64 wt0_ = __builtin_readcyclecounter();\n"
     "      if (c0) src.rotate();\n"),
    ("      i32 wfail = -1;\n      int wrc = CRR_OK;\n      while (vm) {\n",
     "      i32 wfail = -1;\n      int wrc = CRR_OK;\n      const u64 wt1_ = __builtin_readcyclecounter();\n"
     "      wp_[1] += wt1_ - wt0_; wp_[8] += 1;\n      while (vm) {\n"),
    ("        if (!fast || ((OPS >> j) & 1)) {\n          // the status is wave-uniform",
     "        const u64 wv0_ = __builtin_readcyclecounter();\n"
     "        const bool isop_ = fast && ((OPS >> j) & 1) && (et & CRR_ETYPE_MASK) != CRR_EV_DECISION_TASK_COMPLETED;\n"
     "        if (!fast || ((OPS >> j) & 1)) {\n          // the status is wave-uniform"),
    ("        if (et & CRR_ETYPE_BATCH_LAST) {\n          T.epilogue(L, G, K);  // :634-640 GenerateActivityTimerTasks / GenerateUserTimerTasks\n"
     "          if (!fast) {",
     "        const u64 wv1_ = __builtin_readcyclecounter();\n"
     "        if (isop_) { wp_[3] += wv1_ - wv0_; wp_[9] += 1; } else { wp_[4] += wv1_ - wv0_; wp_[10] += 1; }\n"
     "        { const u32 t_ = et & CRR_ETYPE_MASK; const u32 op_ = (u32)((t_ < 16 ? mop_word(0) : t_ < 32 ? mop_word(1) :"
     " mop_word(2)) >> (4 * (t_ & 15))) & 15u;\n"
     "          if (isop_) { wp_[16 + op_] += wv1_ - wv0_; wp_[32 + op_] += 1; } }\n"
     "        if (et & CRR_ETYPE_BATCH_LAST) {\n          T.epilogue(L, G, K);  // :634-640 GenerateActivityTimerTasks / GenerateUserTimerTasks\n"
     "          { const u64 wv2_ = __builtin_readcyclecounter(); wp_[5] += wv2_ - wv1_; wp_[11] += 1; }\n"
     "          if (!fast) {"),
    ("      if (fast) {\n        // what the events [0, end) of the chunk did besides the walk",
     "      const u64 wt2_ = __builtin_readcyclecounter();\n      wp_[2] += wt2_ - wt1_;\n"
     "      if (fast) {\n        // what the events [0, end) of the chunk did besides the walk"),
    ("      if (wfail >= 0) {  // the failing event's prologue has run\n        WAVE_VH_AFTER(wfail);",
     "      { const u64 wt3_ = __builtin_readcyclecounter(); wp_[6] += wt3_ - wt2_; wp_[0] += wt3_ - wt0_; }\n"
     "      if (wfail >= 0) {  // the failing event's prologue has run\n        WAVE_VH_AFTER(wfail);"),
    # WaveTables sub-buckets (wpx_): epilogue halves and act_insert's parts
    ("  bool dirty_act = false, dirty_timer = false;\n\n  __device__ __forceinline__ void init() { lane = (i32)(threadIdx.x & 63); }",
     "  bool dirty_act = false, dirty_timer = false;\n  u64 wpx_[16] = {};\n\n  __device__ __forceinline__ void init() { lane = (i32)(threadIdx.x & 63); }"),
    ("    if (L.n_act > 0 && dirty_act) {\n      BestTimer B;\n      const i32 hwa = uniform32(hw_act);",
     "    if (L.n_act > 0 && dirty_act) {\n      const u64 e0_ = __builtin_readcyclecounter();\n      BestTimer B;\n      const i32 hwa = uniform32(hw_act);"),
    ("      wave_min(B);\n      i32 attempt = 0;",
     "      const u64 e1_ = __builtin_readcyclecounter(); wpx_[0] += e1_ - e0_;\n      wave_min(B);\n"
     "      const u64 e2_ = __builtin_readcyclecounter(); wpx_[1] += e2_ - e1_; wpx_[8] += 1;\n      i32 attempt = 0;"),
    ("      if (B.have && !B.created) K.add(L, G, CRR_TASK_ACTIVITY_TIMEOUT, B.y, L.current_version, B.t, B.e, (i32)bcast(B.j, (u32)attempt), -1);\n    }",
     "      if (B.have && !B.created) K.add(L, G, CRR_TASK_ACTIVITY_TIMEOUT, B.y, L.current_version, B.t, B.e, (i32)bcast(B.j, (u32)attempt), -1);\n"
     "      wpx_[2] += __builtin_readcyclecounter() - e2_;\n    }"),
    ("    if (L.n_timer > 0 && dirty_timer) {\n      BestTimer B;\n      const i32 hwt = uniform32(hw_timer);",
     "    const u64 et0_ = __builtin_readcyclecounter();\n    const bool tdo_ = L.n_timer > 0 && dirty_timer;\n"
     "    if (L.n_timer > 0 && dirty_timer) {\n      BestTimer B;\n      const i32 hwt = uniform32(hw_timer);"),
    ("    dirty_timer = false;\n  }\n  __device__ __forceinline__ bool task_writer() const { return lane == 0; }",
     "    if (tdo_) { wpx_[3] += __builtin_readcyclecounter() - et0_; wpx_[9] += 1; }\n"
     "    dirty_timer = false;\n  }\n  __device__ __forceinline__ bool task_writer() const { return lane == 0; }"),
    ("    const i32 m = find_act_mapped(row.key);\n    const i32 j = take(A_(), hw_act, ST::A, G.act_cap);\n    if (j < 0) return -j;",
     "    const u64 i0_ = __builtin_readcyclecounter();\n    const i32 m = find_act_mapped(row.key);\n"
     "    const u64 i1_ = __builtin_readcyclecounter(); wpx_[4] += i1_ - i0_;\n"
     "    const i32 j = take(A_(), hw_act, ST::A, G.act_cap);\n"
     "    const u64 i2_ = __builtin_readcyclecounter(); wpx_[5] += i2_ - i1_;\n    if (j < 0) return -j;"),
    ("    act_cand_store(j, row);\n    ++L.n_act;\n    dirty_act = true;\n    return CRR_OK;",
     "    act_cand_store(j, row);\n    ++L.n_act;\n    dirty_act = true;\n    wpx_[6] += __builtin_readcyclecounter() - i2_;\n    return CRR_OK;"),
    # flush at the end of the replay (lane 0 of a wavefront-path replay)
    ("  out.exec[w] = R;\n",
     "  out.exec[w] = R;\n"
     "  if constexpr (" + WAVE + ") {\n"
     "    if ((threadIdx.x & 63) == 0 && wp_[8]) { wp_[12] = 1;\n"
     "      for (int q_ = 0; q_ < 48; ++q_) atomicAdd(&g_wave_prof[q_], (unsigned long long)wp_[q_]);\n"
     "      if constexpr (WaveWpx<P>::value) for (int q_ = 0; q_ < 16; ++q_) atomicAdd(&g_wave_prof[48 + q_], (unsigned long long)T.wpx_[q_]); }\n"
     "  }\n"),
    # the device array and its reader
    ("// ---- the job's digest, folded into the replay",
     "__device__ unsigned long long g_wave_prof[64];\n"
     "template <class P, class = void> struct WaveWpx { static constexpr bool value = false; };\n"
     "template <class P> struct WaveWpx<P, decltype((void)&P::wpx_)> { static constexpr bool value = true; };\n"
     "extern \"C\" int crr_wave_prof(unsigned long long* host, int reset) {\n"
     "  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wave_prof), sizeof(g_wave_prof)) != hipSuccess) return -1;\n"
     "  if (reset) { unsigned long long z[64] = {}; if (hipMemcpyToSymbol(HIP_SYMBOL(g_wave_prof), z, sizeof(z)) != hipSuccess) return -1; }\n"
     "  return 0;\n}\n"
     "// ---- the job's digest, folded into the replay"),
]


def main():
    s = open(os.path.join(ROOT, "cadence_amd", "csrc", "replay_kernel.hip")).read()
    for old, new in PATCHES:
        if old not in s:
            raise SystemExit(f"patch point not found: {old[:70]!r}")
        s = s.replace(old, new, 1)
    d = tempfile.mkdtemp()
    p = os.path.join(d, "replay_kernel.hip")
    open(p, "w").write(s)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "build_variant.py"), "waveprof", "--src=" + p], check=True)


if __name__ == "__main__":
    main()
