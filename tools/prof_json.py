"""Device JSON ingest probe: a workload persisted as common/types JSON blobs (blobs.encode_batch(json=True))
uploaded once, then timed per call: crr_ingest_transcode_plan + crr_ingest_transcode (JSON -> thriftrw in
HBM), crr_ingest_plan + crr_ingest_layout, the replay -- beside the same workload's thriftrw blobs through
plan + layout alone.  The replayed rows of both paths are compared (exec rows and the fused digest).  Run it
under `rocprofv3 --kernel-trace --stats` for the per-kernel split.

    python tools/prof_json.py [--kind mixed|chain] [--wf 125000] [--reps 3]
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
    p.add_argument("--kind", default="mixed")
    p.add_argument("--wf", type=int, default=125_000)
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
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
    t0 = time.perf_counter()
    bj, bt = encode_batch(b, json=True), encode_batch(b)
    enc_s = time.perf_counter() - t0
    eng = ReplayEngine(0)
    ing_j, ing_t = DeviceIngest(eng), DeviceIngest(eng)
    dj, dt = ing_j.upload(bj), ing_t.upload(bt)
    enc = torch.ones(bj.n_blobs, dtype=torch.int32, device=eng.dev)   # CRR_ENCODING_JSON
    tj = ing_j.transcode(dj, enc)
    out_j = ing_j.layout(tj, ing_j.plan(tj))
    out_t = ing_t.layout(dt, ing_t.plan(dt))
    torch.cuda.synchronize()
    res = {"transcode_ms": [], "json_ingest_ms": [], "json_total_ms": [], "thrift_ingest_ms": [], "replay_ms": []}
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tj = ing_j.transcode(dj, enc)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ing_j.layout(tj, ing_j.plan(tj), out=out_j)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ing_t.layout(dt, ing_t.plan(dt), out=out_t)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        eng.launch(out_j)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        res["transcode_ms"].append((t1 - t0) * 1e3)
        res["json_ingest_ms"].append((t2 - t1) * 1e3)
        res["json_total_ms"].append((t2 - t0) * 1e3)
        res["thrift_ingest_ms"].append((t3 - t2) * 1e3)
        res["replay_ms"].append((t4 - t3) * 1e3)
    eng.launch(out_t)
    torch.cuda.synchronize()
    same_exec = bool(torch.equal(out_j.tensors["exec"], out_t.tensors["exec"]))
    from cadence_amd import abi
    n_slots = int(ing_t.plan(dt).n_slots)    # (the buffers' slack past the slots is uninitialised)
    same_in = all(bool(torch.equal(out_j.tensors["ev_" + k][:n_slots * np.dtype(t).itemsize],
                                   out_t.tensors["ev_" + k][:n_slots * np.dtype(t).itemsize]))
                  for k, t in abi.EVENT_COLUMNS)
    S = ing_j.last_transcode
    n_ev = int(b.n_events)
    best = min(res["json_total_ms"]) / 1e3
    print(json.dumps({"kind": a.kind, "workflows": b.n_wf, "events": n_ev, "blobs": bj.n_blobs,
                      "json_bytes": bj.n_bytes, "thrift_bytes": bt.n_bytes, "transcoded_bytes": int(S.n_bytes),
                      "encode_s": enc_s, **res,
                      "json_ingest_events_per_s": n_ev / best, "json_GBs": bj.n_bytes / (min(res["transcode_ms"]) / 1e3) / 1e9,
                      "inputs_equal_thrift_path": same_in, "rows_equal_thrift_path": same_exec}), flush=True)


if __name__ == "__main__":
    main()
