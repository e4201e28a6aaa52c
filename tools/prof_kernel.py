"""Kernel-only driver for rocprofv3 / A-B timing: replays config 2 (1M x 29 events) a few times.

    python tools/prof_kernel.py [--lib path/to/lib.so] [--wf N] [--k 4] [--reps R]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=None)
    p.add_argument("--wf", type=int, default=1_000_000)
    p.add_argument("--k", type=int, default=4)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--mixed", action="store_true", help="config-3-like mixed histories instead of chains")
    p.add_argument("--native", action="store_true", help="mixed histories from the native generator (full size)")
    p.add_argument("--tiered", type=int, default=1, help="0: no tier segments (CRR_IN_TIERED off)")
    p.add_argument("--calib", action="store_true", help="first stream known byte counts (tools/calib.py)")
    p.add_argument("--segments", action="store_true", help="report when each concurrent tier segment finished")
    p.add_argument("--digest", action="store_true", help="the fused multi-GPU digest on (as bench.py's config 2)")
    p.add_argument("--no-live-ids", action="store_true", help="no live-ID sidecar (crr_outputs.live_ids)")
    p.add_argument("--no-started-aux", action="store_true", help="CRR_IN_STARTED_AUX off (A/B)")
    p.add_argument("--merge", type=int, default=0, help="tier experiment: 1 = the 2-slot segment replayed by compact "
                   "tier 1, 2 = the 1-slot segment too")
    a = p.parse_args()
    if a.calib:   # in-process (never spawn or exec from a process the profiler has put on the GPU)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import calib
        calib.run(1024, 2)
    if a.lib:
        os.environ["CRR_LIB_PATH"] = os.path.abspath(a.lib)
    import numpy as np
    import torch
    from cadence_amd import synth
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.flatten import interleave
    eng = ReplayEngine(0)
    t0 = time.time()
    if a.native:
        from cadence_amd import synth_native
        b = interleave(synth_native.mixed(a.wf), tiered=bool(a.tiered))
    elif a.mixed:
        from cadence_amd import synth_mixed
        from cadence_amd.flatten import flatten
        b = interleave(flatten(synth_mixed.mixed_histories(a.wf, 5), known_domains={"domain-a", "domain-b", "parent-domain"}),
                       tiered=bool(a.tiered))
    else:
        b = interleave(synth.activity_chain(a.wf, a.k, synth.SEED_C2, with_keys=False))
    if a.merge and b.tiers is not None:
        t = list(b.tiers)
        t[1] = t[0] if a.merge == 1 else 0   # compact_begin
        if a.merge == 2:
            t[0] = 0                          # large_begin
        b.tiers = tuple(t)
    if a.no_started_aux:   # A/B: the compact tiers gather the scheduled event's aux themselves
        b.started_aux = False
    db = eng.upload(b, live_ids=not a.no_live_ids)
    if a.digest:
        from cadence_amd import dist as cdist
        eng.enable_digest(db, cdist.device_keys(b))
    eng.launch(db)
    torch.cuda.synchronize()
    ms = []
    for _ in range(a.reps):
        eng.launch(db)
        torch.cuda.synchronize()
        ms.append(eng.last_kernel_ms()[1])
    seg = getattr(eng.lib, "crr_segment_timing", None)
    if seg is not None and a.segments:  # when each side stream's segments finished (concurrent launch)
        import ctypes
        seg(1)
        eng.launch(db)
        torch.cuda.synchronize()
        buf = (ctypes.c_float * 7)()
        eng.lib.crr_segment_ms.argtypes = [ctypes.c_void_p, ctypes.c_int]
        if eng.lib.crr_segment_ms(ctypes.addressof(buf), 7) == 7:
            print(json.dumps({"segments_end_ms": dict(zip(["large(2-slot)", "compact3+wide", "big", "compact1", "compact2",
                                                           "tail", "small(main)"], [round(x, 3) for x in buf]))}))
        seg(0)
    dbg = getattr(eng.lib, "crr_debug_cycles", None)
    if dbg is not None:  # CRR_EXP=2048 builds: per-phase wavefront cycles of the lane kernels (all launches)
        import ctypes
        buf = (ctypes.c_ulonglong * 320)()
        dbg.argtypes = [ctypes.c_void_p, ctypes.c_int]
        dbg(ctypes.addressof(buf), 320)
        names = ["1-slot", "2-slot", "compact1", "compact2", "compact3"]
        for k, nm in enumerate(names):
            v = buf[8 * k: 8 * k + 8]
            if v[5]:
                w, n = v[5], v[6]
                print(json.dumps({"tier": nm, "waves": w, "steps_per_wave": n / w,
                                  "cycles_per_wave": {"prologue": v[0] / w, "dispatch": v[1] / w, "epilogue": v[2] / w,
                                                      "loop": v[3] / w, "after_loop": v[4] / w},
                                  "cycles_per_step": {"prologue": v[0] / n, "dispatch": v[1] / n, "map_op": v[7] / n,
                                                      "epilogue": v[2] / n, "loop": v[3] / n}}))
    res = eng.download(db)
    alg = synth.algorithmic_bytes(b, res)
    med = float(np.median(ms))
    print(json.dumps({"lib": a.lib or "default", "setup_s": time.time() - t0, "tiers": b.tiers, "workflows": b.n_wf, "events": b.n_events, "kernel_ms": ms,
                      "median_ms": med, "events_per_s": b.n_events / (med * 1e-3),
                      "alg_GBs": alg / (med * 1e-3) / 1e9, "alg_bytes": alg,
                      "ok": int((res.exec["status"] == 0).sum()),
                      "checksum_xor": int(np.bitwise_xor.reduce(res.exec["checksum"].astype(np.uint64)))}))


if __name__ == "__main__":
    main()
