"""Device-ingest probe: persisted blobs of one chunk (config 2 activity chains or the config-3 native mixed
shape) uploaded once, then crr_ingest_plan + crr_ingest_layout timed (wall, per call) -- run it under
`rocprofv3 --kernel-trace --stats` for the per-kernel split.

    python tools/prof_ingest.py [--kind chain|mixed] [--wf 125000] [--reps 3]
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
    p.add_argument("--kind", default="chain")
    p.add_argument("--wf", type=int, default=125_000)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--lib", default=None)
    a = p.parse_args()
    if a.lib:
        os.environ["CRR_LIB_PATH"] = os.path.abspath(a.lib)
    import numpy as np
    import torch
    from cadence_amd import synth, synth_native
    from cadence_amd.blobs import encode_batch
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.ingest import DeviceIngest
    if a.kind == "chain":
        b = synth.activity_chain(a.wf, 4, synth.SEED_C2, with_keys=True, wf_ids=np.arange(a.wf))
    else:
        b = synth_native.mixed(a.wf)
    bs = encode_batch(b)
    eng = ReplayEngine(0)
    ing = DeviceIngest(eng)
    db = ing.upload(bs)
    S = ing.plan(db)
    out = ing.layout(db, S)
    torch.cuda.synchronize()
    plan_s, lay_s, rep_s = [], [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        S = ing.plan(db)
        t1 = time.perf_counter()
        ing.layout(db, S, out=out)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        eng.launch(out)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        plan_s.append(t1 - t0); lay_s.append(t2 - t1); rep_s.append(t3 - t2)
    print(json.dumps({"kind": a.kind, "workflows": bs.n_wf, "blobs": bs.n_blobs, "blob_bytes": bs.n_bytes,
                      "events": int(S.n_events), "plan_ms": [x * 1e3 for x in plan_s], "layout_ms": [x * 1e3 for x in lay_s],
                      "replay_ms": [x * 1e3 for x in rep_s],
                      "ingest_events_per_s": int(S.n_events) / (min(plan_s) + min(lay_s)),
                      "ingest_blob_GBs": bs.n_bytes / (min(plan_s) + min(lay_s)) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
