"""Passive-replication probe (the bench's `passive_replication` line at its size): the config-3 shard cut
before every history's last batch, the prefix replayed once, then `--reps` steps of restore + apply the
last batches onto the loaded rows (CRR_WF_FLAG_RESUME); kernel time of each step.  Run it under
`rocprofv3 --kernel-trace --stats` to see which kernels the resume path spends its time in.

    python tools/prof_replication.py [--wf 1250000] [--reps 5]
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
    p.add_argument("--wf", type=int, default=1_250_000)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--lib", default=None, help="replay library to load (variant builds)")
    p.add_argument("--no-live-ids", action="store_true", help="no live-ID sidecar (crr_outputs.live_ids)")
    p.add_argument("--no-started-aux", action="store_true", help="CRR_IN_STARTED_AUX off (A/B)")
    p.add_argument("--hbm-rows", action="store_true", help="every lane workflow over its HBM rows (round-3 path)")
    p.add_argument("--phases", action="store_true", help="a -DCRR_PHASE_PROF=1 library: per-phase wave clocks")
    p.add_argument("--blobs", action="store_true", help="the step from the tasks' persisted blobs (BlobReplication: "
                                                          "device resume ingest + replay), wall time per step")
    a = p.parse_args()
    if a.lib:
        os.environ["CRR_LIB_PATH"] = os.path.abspath(a.lib)
    import numpy as np
    import torch
    from cadence_amd import synth_native
    from cadence_amd import dist as cdist
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.flatten import interleave
    from cadence_amd.replication import PassiveReplication

    t0 = time.time()
    canon = synth_native.mixed(a.wf, shard=(cdist.NUM_SHARDS, 1, 0))
    batch = interleave(canon, long_threshold=256)   # bench.py's N=1 shard
    batch.started_aux = not a.no_started_aux
    eng = ReplayEngine(0)
    db = eng.upload(batch)
    eng.launch(db)
    one_shot = eng.download(db)
    del db
    torch.cuda.empty_cache()
    pr = PassiveReplication(eng, batch, hbm_rows=a.hbm_rows, live_ids=not a.no_live_ids)
    pr.setup()
    setup_s = time.time() - t0
    if a.blobs:
        from cadence_amd.blobs import encode_batch
        from cadence_amd.replication import BlobReplication
        br = BlobReplication(pr, encode_batch(canon))
        br.setup()
        wall = []
        for _ in range(a.reps + 1):
            pr.restore()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            br.step()
            torch.cuda.synchronize()
            wall.append((time.perf_counter() - t1) * 1e3)
        print(json.dumps({"blobs": True, "workflows": pr.batch.n_wf, "events": br.n_events, "step_ms": wall[1:],
                          "median_ms": float(np.median(wall[1:])), "verify": pr.verify(one_shot)}), flush=True)
        return
    ms = []
    if a.phases:
        import ctypes
        buf = (ctypes.c_ulonglong * 8)()
        eng.lib.crr_phase_prof(buf, 1)
    for _ in range(a.reps + 1):
        pr.restore()
        torch.cuda.synchronize()
        eng.launch(pr.db_new)
        torch.cuda.synchronize()
        ms.append(sum(x for x in eng.last_kernel_ms()[:2] if x > 0))
    phases = None
    if a.phases:
        eng.lib.crr_phase_prof(buf, 0)
        n = max(int(buf[5]), 1)
        phases = {k: buf[i] / n for i, k in enumerate(["prologue_load", "events_tail", "token_vh", "finalize",
                                                          "exec_crc"])}
        phases["waves"] = int(buf[5])
    v = pr.verify(one_shot)
    med = float(np.median(ms[1:]))
    print(json.dumps({"hbm_rows": a.hbm_rows, "workflows": pr.batch.n_wf, "events": int(pr.n_events), "kernel_ms": ms[1:], "median_ms": med,
                      "events_per_s": pr.n_events / (med * 1e-3), "verify": v, "setup_s": setup_s, "phase_clocks_per_wave": phases}), flush=True)


if __name__ == "__main__":
    main()
