"""HBM bytes per replay launch group for the bench's config-3 / config-4 lines, from rocprofv3 --pmc
passes (FETCH_SIZE and WRITE_SIZE, one run each) of tools/prof_kernel.py --native (config 3) or
tools/prof_longtail.py --native (config 4).  Per replay kernel: the median over its dispatches; the group
is the sum over the replay_* kernels of one crr_replay (every tier segment, the tail, the retry pass).
FETCH_SIZE is doubled (MI355X_MICROARCH.md "HBM": gfx950 reports half of a wide read's bytes; the
replay's loads are 1-8 B per lane, calibrated at 2.0x by tools/calib_stream.hip, profiles/traffic.json),
WRITE_SIZE taken as is.

    python tools/traffic_configs.py NAME PMC_DIR --workflows N --events E [--out profiles/traffic_configs.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(root, prefixes=("replay_",), exclude=()):
    """{counter: {kernel: median over dispatches}} for the kernels whose names start with `prefixes` (and
    contain none of `exclude`)."""
    acc = collections.defaultdict(float)
    for f in sorted(glob.glob(os.path.join(root, "*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
                 .replace("crr::", "").strip())
            if not k.startswith(tuple(prefixes)) or any(x in k for x in exclude):
                continue
            acc[(r["Counter_Name"], k, f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for (c, k, _f, _d), v in acc.items():
        vals[c][k].append(v)
    return {c: {k: statistics.median(v) for k, v in ks.items()} for c, ks in vals.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("name")
    p.add_argument("root")
    p.add_argument("--workflows", type=int, required=True)
    p.add_argument("--events", type=int, required=True)
    p.add_argument("--out", default=os.path.join(ROOT, "profiles", "traffic_configs.json"))
    p.add_argument("--kernels", default="replay_", help="comma-separated kernel-name prefixes of the launch group")
    p.add_argument("--exclude", action="append", default=[], help="a name fragment to leave out (repeatable; e.g. "
                                                                  "the fresh instantiations a resume probe also dispatches)")
    a = p.parse_args()
    d = per_kernel(a.root, a.kernels.split(","), a.exclude)
    fetch = {k: 2.0 * v * 1024 for k, v in d.get("FETCH_SIZE", {}).items()}   # KB -> bytes, x2 (gfx950)
    write = {k: v * 1024 for k, v in d.get("WRITE_SIZE", {}).items()}
    if not fetch or not write:
        raise SystemExit("need FETCH_SIZE and WRITE_SIZE passes under " + a.root)
    out = json.load(open(a.out)) if os.path.exists(a.out) else {}
    out[a.name] = {"workflows": a.workflows, "events": a.events,
                   "hbm_bytes_per_launch": sum(fetch.values()) + sum(write.values()),
                   "fetch_x2_bytes": fetch, "write_bytes": write,
                   "source": os.path.relpath(a.root, ROOT)}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({a.name: out[a.name]["hbm_bytes_per_launch"]}))


if __name__ == "__main__":
    main()
