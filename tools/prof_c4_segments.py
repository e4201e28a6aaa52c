"""Config-4 probe: where the launch group's time goes, segment by segment.

    python tools/prof_c4_segments.py [--n 2000] [--reps 3] [--lib path.so] [--only all,tail,big,c2,...]

The config-4 batch (synth_native.long_tail, lane / wavefront threshold 256) is replayed whole, with
crr_segment_timing on (when each side stream's segments finished, relative to the fork), and then with
every segment but one emptied (its workflows' descriptors given ev_count 0, so their kernels launch and
finish at once): each segment's time alone on the GPU.  Results of the emptied runs are wrong by design;
only the times are read.  Kernel times are the phase-1 launch group (crr_last_kernel_ms).
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MOPS = ("none", "act_insert", "act_start", "act_delete", "act_cancel", "timer_start", "timer_delete", "child_insert",
        "child_start", "child_delete", "rc_insert", "rc_delete", "sig_insert", "sig_delete")
SIDE = ("large", "wide_c3", "big", "c1", "c2", "tail", "caller(small)")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=2000)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--lib", default=None)
    p.add_argument("--threshold", type=int, default=256)
    p.add_argument("--only", default="all,tail,big,c1,c2,c3,small,lanes")
    p.add_argument("--top", type=int, default=0, help="runs 'tailtop': only the N longest tail workflows")
    p.add_argument("--wave-prof", action="store_true", help="read crr_wave_prof (tools/wave_prof.py builds)")
    a = p.parse_args()
    if a.lib:
        os.environ["CRR_LIB_PATH"] = os.path.abspath(a.lib)
    import numpy as np
    import torch
    from cadence_amd import abi, synth_native
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.flatten import interleave
    eng = ReplayEngine(0)
    b = interleave(synth_native.long_tail(a.n), long_threshold=a.threshold)
    lb, cb, c2, wb, hb, big = b.tiers
    n_lane = b.wave_begin if b.wave_begin is not None else b.n_wf
    seg = {"small": (0, lb), "large": (lb, cb), "c1": (cb, c2), "c2": (c2, wb), "c3": (wb, hb), "wide": (hb, n_lane),
           "tail": (n_lane, big), "big": (big, b.n_wf)}
    seg["lanes"] = (0, n_lane)
    cnt = b.wf["ev_count"].astype(np.int64)
    info = {k: {"workflows": int(hi - lo), "events": int(cnt[lo:hi].sum()), "max_events": int(cnt[lo:hi].max()) if hi > lo else 0}
            for k, (lo, hi) in seg.items()}
    print(json.dumps({"tiers": list(b.tiers), "wave_begin": n_lane, "n_wf": b.n_wf, "segments": info}), flush=True)
    eng.lib.crr_segment_ms.argtypes = [ctypes.c_void_p, ctypes.c_int]
    wf0 = b.wf.copy()
    seg["tailtop"] = seg["tail"]
    for what in a.only.split(","):
        wf = wf0.copy()
        if what != "all":
            keep = np.zeros(b.n_wf, bool)
            if what == "tailtop":
                lo, hi = seg["tail"]
                keep[lo + np.argsort(-cnt[lo:hi], kind="stable")[:a.top]] = True
            else:
                lo, hi = seg[what]
                keep[lo:hi] = True
            keep |= (wf0["flags"] & abi.WF_FLAG_NEW_RUN) != 0   # phase 0 unchanged
            wf["ev_count"] = np.where(keep, wf0["ev_count"], 0)
            wf["empty_batch_at"] = np.where(keep, wf0["empty_batch_at"], -1)
        db = eng.upload(b)
        db.tensors["wf"][:wf.nbytes].copy_(torch.from_numpy(wf.view(np.uint8)))
        eng.lib.crr_segment_timing(1)
        wp = getattr(eng.lib, "crr_wave_prof", None) if a.wave_prof else None
        wbuf = np.zeros(64, np.uint64)
        ms, segs = [], []
        for r in range(a.reps + 1):
            db.tensors["scratch"].zero_()
            eng.launch(db)
            torch.cuda.synchronize()
            k = eng.last_kernel_ms()
            buf = (ctypes.c_float * 7)()
            got = eng.lib.crr_segment_ms(ctypes.addressof(buf), 7)
            if wp is not None:
                wp.argtypes = [ctypes.c_void_p, ctypes.c_int]
                wp(wbuf.ctypes.data, 1)   # read and reset: the last rep's split is kept
            if r:
                ms.append(k[2])
                segs.append(list(buf) if got == 7 else None)
        eng.lib.crr_segment_timing(0)
        med = float(np.median(ms))
        sm = None
        if all(s is not None for s in segs):
            sm = {n: round(float(np.median([s[i] for s in segs])), 4) for i, n in enumerate(SIDE)}
        line = {"run": what, "group_ms": ms, "median_ms": med, "segment_finish_ms": sm}
        if wp is not None:
            w = [int(x) for x in wbuf]
            cyc = {n: w[i] for i, n in enumerate(("chunk_total", "pre_walk", "walk", "map_op_visits", "other_visits",
                                                 "epilogues", "post_walk"))}
            cnts = {n: w[8 + i] for i, n in enumerate(("chunks", "map_ops", "other_visits", "epilogues", "replays"))}
            line["wave_prof"] = {"cycles": cyc, "counts": cnts,
                                 "per_chunk": {k: v / max(cnts["chunks"], 1) for k, v in cyc.items()},
                                 "per_map_op": cyc["map_op_visits"] / max(cnts["map_ops"], 1),
                                 "per_epilogue": cyc["epilogues"] / max(cnts["epilogues"], 1),
                                 "per_op": {n: {"count": w[32 + i], "cycles_each": w[16 + i] / max(w[32 + i], 1)}
                                            for i, n in enumerate(MOPS) if w[32 + i]},
                                 "wave_tables": {"act_epilogue": {"count": w[56], "cand_loads": w[48] / max(w[56], 1),
                                                                  "wave_min": w[49] / max(w[56], 1),
                                                                  "update": w[50] / max(w[56], 1)},
                                                 "timer_epilogue": {"count": w[57], "cycles_each": w[51] / max(w[57], 1)},
                                                 "act_insert": {"find_mapped": w[52] / max(w[33], 1),
                                                                "take": w[53] / max(w[33], 1),
                                                                "write": w[54] / max(w[33], 1)}}}
        print(json.dumps(line), flush=True)
        del db
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
