"""Diagnostics: which workflows does the fast path hand back?  Needs a library built with
-DCRR_EXP=64 (the retry pass leaves them at CRR_INTERNAL_RETRY).

    python tools/retry_diag.py --lib build/variants/lib_noretry.so [--wf N]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", required=True)
    p.add_argument("--wf", type=int, default=20000)
    p.add_argument("--longtail", action="store_true", help="config-4 long-tail histories instead of mixed")
    a = p.parse_args()
    os.environ["CRR_LIB_PATH"] = os.path.abspath(a.lib)
    import numpy as np
    from cadence_amd import synth_mixed
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.flatten import flatten, interleave, live_set_bounds, tier_classes
    if a.longtail:
        hs = synth_mixed.long_tail_histories(a.wf, 0xCAD00004, max_len=50_000, run_cap=10_000)
    else:
        hs = synth_mixed.mixed_histories(a.wf, 5)
    b = flatten(hs, known_domains={"domain-a", "domain-b", "parent-domain"})
    cls = tier_classes(b)
    bounds = live_set_bounds(b)
    eng = ReplayEngine(0)
    for tiered in (True, False):
        ib = interleave(b, tiered=tiered)
        r = eng.replay(ib)
        st = r.exec["status"]
        retried = np.nonzero(st == 200)[0]
        canon = ib.perm[retried]
        out = {"tiered": tiered, "tiers": ib.tiers, "n_retried": int(retried.size), "wave_begin": ib.wave_begin,
               "retried_len": ib.wf["ev_count"][retried][:20].tolist(),
               "by_class": np.bincount(cls[canon], minlength=3).tolist(),
               "positions_head": retried[:20].tolist()}
        if retried.size:
            out["bounds_head"] = {k: v[canon[:20]].tolist() for k, v in bounds.items()}
        print(json.dumps(out))


if __name__ == "__main__":
    main()
