"""Turn rocprofv3 --pmc passes into calibrated HBM bytes per replay launch (profiles/traffic.json).

Each pass directory holds <name>_counter_collection.csv from one `rocprofv3 --kernel-trace --pmc ...`
run of `tools/prof_kernel.py --calib`: the calibration kernels (tools/calib_stream.hip, a known byte
count at 1/4/8-B-per-lane reads and 8-B-per-lane writes) and the replay launches of the same process.

MI355X_MICROARCH.md ("HBM"): FETCH_SIZE reports 1/2 of a 16-B/lane stream's bytes on gfx950 and other
widths are uncalibrated, so the replay kernel's FETCH_SIZE is scaled by the ratio measured on the
8-B/lane calibration read (its dominant access: 40 of 49 B per event are i64 columns), and WRITE_SIZE
by the 8-B/lane calibration write.

    python tools/traffic.py gpurun_out [--workflows N --events-per-workflow E] [--out profiles/traffic.json]
"""
import argparse
import collections
import csv
import glob
import json
import os

CALIB = {"calib_read<unsigned char>": 1, "calib_read<unsigned int>": 4, "calib_read<unsigned long>": 8,
         "calib_write<unsigned long>": 108}


def load(root):
    """{counter: {kernel: [per-dispatch values]}} over every pass directory under root."""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "*", "*counter_collection.csv"))):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("crr::", "").strip()
            per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _d, c), v in per.items():
            out[c][k].append(v)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("root")
    p.add_argument("--kernel", default="replay_lds_small_kernel<false, false, false>")
    p.add_argument("--workflows", type=int, default=1_000_000)
    p.add_argument("--events-per-workflow", type=int, default=29)
    p.add_argument("--calib-bytes", type=int, default=1 << 30)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    data = load(a.root)
    res = {"workflows": a.workflows, "events_per_workflow": a.events_per_workflow, "kernel": a.kernel}
    ratio = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        for name, kind in CALIB.items():
            v = data.get(ctr, {}).get(name)
            if v and ((ctr == "FETCH_SIZE") == (kind < 100)):
                kb = min(v)
                ratio[kind] = a.calib_bytes / (kb * 1024.0)
                res[f"calib_{ctr}_{name}"] = {"reported_KB": kb, "bytes_per_reported_byte": ratio[kind]}
    fetch = data.get("FETCH_SIZE", {}).get(a.kernel)
    write = data.get("WRITE_SIZE", {}).get(a.kernel)
    if fetch:
        res["replay_FETCH_SIZE_KB"] = sorted(fetch)
        res["read_bytes_per_launch"] = min(fetch) * 1024.0 * ratio.get(8, 1.0)
    if write:
        res["replay_WRITE_SIZE_KB"] = sorted(write)
        res["write_bytes_per_launch"] = min(write) * 1024.0 * ratio.get(108, 1.0)
    if fetch and write:
        res["hbm_bytes_per_launch"] = res["read_bytes_per_launch"] + res["write_bytes_per_launch"]
    for c in sorted(data):
        if c in ("FETCH_SIZE", "WRITE_SIZE"):
            continue
        v = data[c].get(a.kernel)
        if v:
            res.setdefault("counters", {})[c] = [min(v), max(v)]
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        open(a.out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
