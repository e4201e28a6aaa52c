"""Config-5 probe (the bench's config5_ndc lines at their size, N = 1): the multi-version mixed histories
rebuilt onto reset branches (`--steps` replays), crr_ndc_prepare over one replication task per workflow,
crr_checksum over the replayed rows -- each through bench.py's own code, so a `rocprofv3 --pmc` pass over
this command gives the per-kernel HBM bytes of exactly the bench's workloads (tools/traffic_configs.py
names: config5_rebuild, config5_ndc_prepare, config5_checksum_verify).

    python tools/prof_config5.py [--wf 1000000] [--steps 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--wf", type=int, default=1_000_000)
    p.add_argument("--steps", type=int, default=3)
    a = p.parse_args()
    sys.argv = [sys.argv[0], "--config-steps", str(a.steps)]
    import bench
    from cadence_amd import ndc, synth_native
    from cadence_amd import dist as cdist
    from cadence_amd.flatten import interleave
    ctx = bench.Ctx(bench.parse())
    shard = (cdist.NUM_SHARDS, 1, 0)
    canon = bench.as_rebuilds(synth_native.mixed(a.wf, multi_version=True, shard=shard, seed=0xCAD00005), 0xCAD00005)
    batch = interleave(canon)
    db = ctx.eng.upload(batch)
    wall, ms = bench.timed_steps(ctx, db, a.steps, 1)
    res = ctx.eng.download(db)
    e, v, c = ndc.version_histories(canon)
    nb = ndc.tasks_from_histories(e, v, c, 0xCAD00025)
    nd = bench.ndc_line(ctx, nb)
    ck = bench.checksum_line(ctx, db, batch, res)
    print(json.dumps({"config5_rebuild": {"workflows": batch.n_wf, "events": batch.n_events, "kernel_ms": ms},
                      "config5_ndc_prepare": {"workflows": len(nb.tasks), "events": len(nb.tasks),
                                              "kernel_ms": nd["roofline"]["kernel_ms"]},
                      "config5_checksum_verify": {"workflows": batch.n_wf, "events": batch.n_events,
                                                  "kernel_ms": ck["roofline"]["kernel_ms"]}}), flush=True)


if __name__ == "__main__":
    main()
