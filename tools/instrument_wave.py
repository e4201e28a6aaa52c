"""Profiling aid (not product code): build an instrumented copy of the replay library whose wavefront-
per-workflow path (replay_tail_kernel / replay_big_kernel) records, per workflow, its start and end
(s_memrealtime, 100 MHz) and the core cycles spent in each part of the event loop (s_memtime around
the event fetch, the version-history prologue, the dispatch and the batch epilogue).  The product
sources are patched in a temporary copy; the result is a separate .so loaded with --lib.

    python tools/instrument_wave.py build/wave_dbg.so
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def patch(src: str) -> str:
    s = src
    s = s.replace("namespace crr {\n", "namespace crr {\n__device__ unsigned long long crr_wave_dbg[8 * 65536];\n", 1)
    # per-part accumulators in replay_body (wave path only)
    s = s.replace("  const i32 retention_days = wfp->retention_days;\n",
                  "  const i32 retention_days = wfp->retention_days;\n  u64 dbg_c[4] = {0, 0, 0, 0};\n"
                  "  constexpr bool kDbg = std::is_same<SRC, WaveSource>::value;\n  u64 dbg_t = 0;\n", 1)
    s = s.replace("  src.start();\n  for (i32 s = 0; s < n_ev; ++s) {\n",
                  "  src.start();\n  if (kDbg) dbg_t = __builtin_amdgcn_s_memtime();\n"
                  "  for (i32 s = 0; s < n_ev; ++s) {\n", 1)
    s = s.replace("    const Ev ev = src.next(s);\n",
                  "    const Ev ev = src.next(s);\n    if (kDbg) { asm volatile(\"s_waitcnt lgkmcnt(0) vmcnt(0)\"); u64 t = __builtin_amdgcn_s_memtime(); dbg_c[0] += t - dbg_t; dbg_t = t; }\n", 1)
    s = s.replace("    last_task_step = s;  // :129",
                  "    if (kDbg) { u64 t = __builtin_amdgcn_s_memtime(); dbg_c[1] += t - dbg_t; dbg_t = t; }\n    last_task_step = s;  // :129", 1)
    s = s.replace("      if (rc) FAIL(rc, s);\n    }\n\n    if (et & CRR_ETYPE_BATCH_LAST) {",
                  "      if (rc) FAIL(rc, s);\n    }\n    if (kDbg) { asm volatile(\"s_waitcnt lgkmcnt(0) vmcnt(0)\"); u64 t = __builtin_amdgcn_s_memtime(); dbg_c[2] += t - dbg_t; dbg_t = t; }\n\n    if (et & CRR_ETYPE_BATCH_LAST) {", 1)
    s = s.replace("      L.next_event_id = id + 1;\n    }\n  }\n",
                  "      L.next_event_id = id + 1;\n    }\n    if (kDbg) { asm volatile(\"s_waitcnt lgkmcnt(0) vmcnt(0)\"); u64 t = __builtin_amdgcn_s_memtime(); dbg_c[3] += t - dbg_t; dbg_t = t; }\n  }\n"
                  "  if (kDbg && (threadIdx.x & 63) == 0) { unsigned long long* d = crr_wave_dbg + 8 * (w & 65535); d[3] = dbg_c[0]; d[4] = dbg_c[1]; d[5] = dbg_c[2]; d[6] = dbg_c[3]; }\n", 1)
    # start / end per workflow
    s = s.replace("  WaveSource S(in.ev, wfp->ev_begin, st, wfp->ev_count);\n  replay_body<EMIT, WaveTables<ST>, WaveSource>(in, out, w, wfp, G, T, S, crc_tables);\n",
                  "  WaveSource S(in.ev, wfp->ev_begin, st, wfp->ev_count);\n  const u64 dbg0 = __builtin_amdgcn_s_memrealtime();\n"
                  "  replay_body<EMIT, WaveTables<ST>, WaveSource>(in, out, w, wfp, G, T, S, crc_tables);\n"
                  "  if ((threadIdx.x & 63) == 0) { unsigned long long* d = crr_wave_dbg + 8 * (w & 65535); d[0] = dbg0; d[1] = __builtin_amdgcn_s_memrealtime(); d[2] = (u64)wfp->ev_count | ((u64)blockIdx.x << 32); }\n", 1)
    s += ("\nextern \"C\" int crr_wave_dbg_read(void* dst, size_t bytes) {\n"
          "  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(crr::crr_wave_dbg), bytes, 0, hipMemcpyDeviceToHost);\n}\n")
    for marker in ("crr_wave_dbg[8 * 65536]", "dbg_c[0] +=", "dbg_c[2] +=", "dbg_c[3] +=", "d[0] = dbg0"):
        if marker not in s:
            raise SystemExit(f"patch point not found: {marker}")
    return s


def main():
    out = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "build", "wave_dbg.so"))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    d = tempfile.mkdtemp()
    src = patch(open(os.path.join(ROOT, "cadence_amd", "csrc", "replay_kernel.hip")).read())
    p = os.path.join(d, "replay_kernel.hip")
    open(p, "w").write(src)
    others = [os.path.join(ROOT, "cadence_amd", "csrc", f) for f in
              ("capi.hip", "ndc_kernel.hip", "compact_kernel.hip", "wire_kernel.hip", "ingest_kernel.hip")]
    objs = [os.path.join(ROOT, "build", os.path.basename(f) + ".o") for f in others]
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-mllvm", "-amdgpu-sched-strategy=max-ilp",
             "-I", os.path.join(ROOT, "include")]
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-c", p, "-o", p + ".o"], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", p + ".o", *objs, "-o", out], check=True)
    print(out)


if __name__ == "__main__":
    main()
