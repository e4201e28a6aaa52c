"""Config-3 tier balance probe: the compact tiers run concurrently and the launch group ends with the slowest
segment (compact tier 1).  Moves the boundary between compact tiers 1 and 2 down by a fraction of tier 1's
segment (its shortest workflows then replay in tier 2's larger arena -- speed only, results unchanged), times
the launch group per shift alternately in one process, and checks the rows are byte-identical.

    python tools/prof_c3_shift.py [--wf 1250000] [--shifts 0,0.1,0.2,0.3] [--rounds 3] [--reps 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--wf", type=int, default=1_250_000)
    p.add_argument("--shifts", default="0,0.1,0.2,0.3")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--upper", action="store_true", help="shift the tier-2 / tier-3 boundary instead")
    a = p.parse_args()
    import numpy as np
    import torch
    from cadence_amd import synth_native
    from cadence_amd import dist as cdist
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.flatten import interleave
    eng = ReplayEngine(0)
    b = interleave(synth_native.mixed(a.wf, shard=(cdist.NUM_SHARDS, 1, 0)))
    db = eng.upload(b)
    ci = db.c_in
    base = (ci.compact_begin, ci.compact2_begin, ci.wide_begin)
    shifts = [float(x) for x in a.shifts.split(",")]
    ref = None
    out = {s: [] for s in shifts}
    for _ in range(a.rounds):
        for sh in shifts:
            if a.upper:
                lo, hi = base[1], base[2]
                ci.wide_begin = hi - int(sh * (hi - lo)) // 64 * 64
            else:
                lo, hi = base[0], base[1]
                ci.compact2_begin = hi - int(sh * (hi - lo)) // 64 * 64
            eng.launch(db)
            torch.cuda.synchronize()
            ms = []
            for _ in range(a.reps):
                eng.launch(db)
                torch.cuda.synchronize()
                ms.append(eng.last_kernel_ms()[1])
            res = eng.download(db)
            key = res.exec.tobytes() + b"".join(res.tables[t].tobytes() for t in ("act", "timer", "child", "rc", "sig", "vh", "rp"))
            if ref is None:
                ref = key
            out[sh].append(float(np.median(ms)))
            assert key == ref, f"rows differ at shift {sh}"
    ci.compact_begin, ci.compact2_begin, ci.wide_begin = base
    print(json.dumps({"tiers": list(b.tiers), "upper": a.upper, "median_ms_per_round": {str(k): v for k, v in out.items()},
                      "rows_identical": True}), flush=True)


if __name__ == "__main__":
    main()
