"""The bench's blob -> rows figure alone (bench.blob_to_rows: PCIe-inclusive and device_resident) for config 2
(activity chains) or the config-3 shard (mixed): a quick probe of the device ingest end to end.

    python tools/prof_blob_rows.py [--kind chain|mixed] [--wf 1000000] [--lib path]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kind", default="chain")
    p.add_argument("--wf", type=int, default=1_000_000)
    p.add_argument("--lib", default=None)
    a = p.parse_args()
    if a.lib:
        os.environ["CRR_LIB_PATH"] = os.path.abspath(a.lib)
    import numpy as np
    sys.argv = [sys.argv[0]]
    import bench
    from cadence_amd import synth, synth_native
    from cadence_amd import dist as cdist
    ctx = bench.Ctx(bench.parse())
    if a.kind == "chain":
        canon = synth.activity_chain(a.wf, 4, synth.SEED_C2, with_keys=True, wf_ids=np.arange(a.wf))
    else:
        canon = synth_native.mixed(a.wf, shard=(cdist.NUM_SHARDS, 1, 0))
    fig = bench.blob_to_rows(ctx, canon, None, a.kind)
    fig.pop("digest", None)
    print(json.dumps(fig), flush=True)


if __name__ == "__main__":
    main()
