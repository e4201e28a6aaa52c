"""Profiling aid: where a config-4 step's wall time goes beyond the measured launch group -- the phase-0
launch (continue-as-new new-run histories, replayed first) and the retry passes.  Per launch:
crr_last_kernel_ms [phase 0, phase 1 (all kernels), phase-1 fast group] and the synchronised wall time.

    python tools/prof_c4_phases.py [--n 2000] [--reps 10] [--lib path.so]
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
    p.add_argument("--n", type=int, default=2000)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--lib", default=None)
    a = p.parse_args()
    if a.lib:
        os.environ["CRR_LIB_PATH"] = os.path.abspath(a.lib)
    import numpy as np
    import torch
    from cadence_amd import abi, synth_native
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.flatten import interleave
    eng = ReplayEngine(0)
    b = interleave(synth_native.long_tail(a.n), long_threshold=256)
    new_run = int(((b.wf["flags"] & abi.WF_FLAG_NEW_RUN) != 0).sum())
    db = eng.upload(b)
    eng.launch(db)
    torch.cuda.synchronize()
    rows = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        eng.launch(db)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        rows.append([wall] + [float(x) for x in eng.last_kernel_ms()])
    r = np.array(rows)
    print(json.dumps({"workflows": b.n_wf, "new_run_workflows": new_run, "events": b.n_events,
                      "median_ms": {"wall": float(np.median(r[:, 0])), "phase0": float(np.median(r[:, 1])),
                                    "phase1": float(np.median(r[:, 2])), "phase1_fast_group": float(np.median(r[:, 3]))},
                      "rows": r.round(4).tolist()}), flush=True)


if __name__ == "__main__":
    main()
