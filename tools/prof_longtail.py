"""Config-4 probe: long-tail histories (Zipf lengths, continue-as-new chains) replayed with and
without length bucketing; kernel time per layout and cross-layout bit-exactness.

    python tools/prof_longtail.py [--n 400] [--max-len 50000] [--run-cap 10000] [--reps 3]
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
    p.add_argument("--n", type=int, default=400, help="logical workflows (before CAN splitting)")
    p.add_argument("--max-len", type=int, default=50_000)
    p.add_argument("--run-cap", type=int, default=10_000)
    p.add_argument("--seed", type=int, default=0xCAD00004)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--thresholds", default="none,256,64")
    p.add_argument("--unbounded", action="store_true", help="unbounded pending sets (random walk)")
    p.add_argument("--lib", default=None, help="replay library to load (variant builds)")
    p.add_argument("--native", action="store_true", help="native generator (synth_native.long_tail)")
    p.add_argument("--big-caps", type=int, default=None, help="one live-set bound for every map above which a long "
                   "workflow goes to replay_big_kernel (default: the tail arena's own; huge: none)")
    a = p.parse_args()
    if a.lib:
        os.environ["CRR_LIB_PATH"] = os.path.abspath(a.lib)
    import numpy as np
    import torch
    from cadence_amd import synth_mixed
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.flatten import flatten, interleave
    from cadence_amd.result import diff_results

    t0 = time.time()
    kw = {"caps": None} if a.unbounded else {}
    if a.native:
        from cadence_amd import synth_native
        b = synth_native.long_tail(a.n, a.seed, max_len=a.max_len, run_cap=a.run_cap,
                                   caps=None if a.unbounded else synth_native.LONG_TAIL_CAPS)
    else:
        hs = synth_mixed.long_tail_histories(a.n, a.seed, max_len=a.max_len, run_cap=a.run_cap, **kw)
        b = flatten(hs, known_domains={"domain-a", "domain-b", "parent-domain"})
    gen_s = time.time() - t0
    cnt = b.wf["ev_count"]
    eng = ReplayEngine(0)
    ref = None
    for th in a.thresholds.split(","):
        thv = None if th == "none" else int(th)
        caps = None if a.big_caps is None else {k: a.big_caps for k in ("act", "timer", "child", "rc", "sig", "rp")}
        ib = interleave(b, long_threshold=thv, big_caps=caps)
        db = eng.upload(ib)
        eng.launch(db)
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            eng.launch(db)
            torch.cuda.synchronize()
            k = eng.last_kernel_ms()
            ms.append(sum(x for x in k[:2] if x > 0))   # phase 0 (new runs) + phase 1; k[2] is inside k[1]
        res = eng.download(db)
        retries = [int(x) for x in db.tensors["scratch"][:2].cpu().tolist()]
        same = None
        if ref is None:
            ref = (ib, res)
        else:
            same = not diff_results(ref[0], ref[1], ib, res)
        med = float(np.median(ms))
        print(json.dumps({"lib": a.lib, "threshold": th, "unbounded": a.unbounded, "workflows": b.n_wf, "events": int(cnt.sum()), "max_len": int(cnt.max()),
                          "wave_tail": int(b.n_wf - (ib.wave_begin if ib.wave_begin is not None else b.n_wf)), "big_caps": a.big_caps,
                          "tiers": list(ib.tiers) if ib.tiers else None,
                          "kernel_ms": ms, "median_ms": med, "events_per_s": float(cnt.sum()) / (med * 1e-3),
                          "ok": int((res.exec["status"] == 0).sum()), "same_as_first": same,
                          "retries_lane_wave": retries, "phase_ms": k,
                          "gen_s": gen_s}), flush=True)
        if ib.wave_begin is not None:
            wr = wave_records(eng, ib)
            if wr is not None:
                print(json.dumps({"threshold": th, "wave_records": wr}), flush=True)


def wave_records(eng, ib):
    """tools/instrument_wave.py builds: per wavefront-path workflow, its start / end (100 MHz realtime) and
    the core cycles of each part of the event loop; summarised over the tail (None for product builds)."""
    import ctypes
    import numpy as np
    f = getattr(eng.lib, "crr_wave_dbg_read", None)
    if f is None:
        return None
    buf = np.zeros(8 * 65536, np.uint64)
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    if f(buf.ctypes.data, buf.nbytes) != 0:
        raise RuntimeError("crr_wave_dbg_read failed")
    d = buf.reshape(65536, 8)
    lo = ib.wave_begin
    w = np.arange(lo, ib.n_wf)
    r = d[w & 65535]
    ev = (r[:, 2] & 0xFFFFFFFF).astype(np.int64)
    ok = (ev > 0) & (r[:, 1] > r[:, 0])
    r, ev, w = r[ok], ev[ok], w[ok]
    t0 = int(r[:, 0].min())
    start_us = (r[:, 0] - t0) / 100.0
    end_us = (r[:, 1] - t0) / 100.0
    dur_us = end_us - start_us
    cyc = r[:, 3:7].astype(np.float64)
    tot = cyc.sum(axis=1)
    top = np.argsort(-end_us)[:10]
    return {"workflows": int(ok.sum()), "events": int(ev.sum()), "span_us": float(end_us.max()),
            "us_per_event_median": float(np.median(dur_us / ev)), "cycles_per_event_median": float(np.median(tot / ev)),
            "start_us_max": float(start_us.max()),
            "cycle_share": {k: float(v) for k, v in zip(("fetch", "vh", "dispatch", "epilogue"), cyc.sum(axis=0) / tot.sum())},
            "critical": [{"events": int(ev[i]), "start_us": float(start_us[i]), "end_us": float(end_us[i]),
                          "us_per_event": float(dur_us[i] / ev[i]), "cycles_per_event": float(tot[i] / ev[i])} for i in top]}


if __name__ == "__main__":
    main()
