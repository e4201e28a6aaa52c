"""NDC-prepare probe (A/B of library variants): the bench's config-5 replication tasks (one per workflow of
1M multi-version mixed histories, bench.ndc_line's workload) through crr_ndc_prepare, kernel time by HIP
events over --reps launches, results checked against the oracle on a sample.

    python tools/prof_ndc.py [--lib path.so] [--wf 1000000] [--reps 10]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=None)
    p.add_argument("--wf", type=int, default=1_000_000)
    p.add_argument("--reps", type=int, default=10)
    a = p.parse_args()
    if a.lib:
        os.environ["CRR_LIB_PATH"] = os.path.abspath(a.lib)
    import numpy as np
    import torch
    from cadence_amd import abi, ndc, synth_native
    from cadence_amd import dist as cdist
    from cadence_amd.engine import ReplayEngine
    from oracle import oracle
    eng = ReplayEngine(0)
    canon = synth_native.mixed(a.wf, multi_version=True, shard=(cdist.NUM_SHARDS, 1, 0), seed=0xCAD00005)
    e, v, c = ndc.version_histories(canon)
    nb = ndc.tasks_from_histories(e, v, c, 0xCAD00025)
    dev = eng.dev

    def up(x):
        raw = np.ascontiguousarray(x).view(np.uint8).reshape(-1)
        t = torch.empty(max(raw.size, 1), dtype=torch.uint8, device=dev)
        t[:raw.size].copy_(torch.from_numpy(raw))
        return t
    n = len(nb.tasks)
    T = {"tasks": up(nb.tasks), "branches": up(nb.branches), "items": up(nb.items)}
    res = torch.zeros(n * abi.NDC_RESULT.itemsize, dtype=torch.uint8, device=dev)
    out = torch.zeros(nb.n_out_items * abi.VH_ITEM.itemsize, dtype=torch.uint8, device=dev)
    ci = abi.CNdcInputs()
    ci.tasks, ci.branches, ci.items = T["tasks"].data_ptr(), T["branches"].data_ptr(), T["items"].data_ptr()
    ci.n_tasks = n
    s = torch.cuda.current_stream(dev)

    def launch():
        rc = eng.lib.crr_ndc_prepare(ctypes.byref(ci), ctypes.c_void_p(res.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                     ctypes.c_void_p(s.cuda_stream))
        assert rc == 0, rc
    launch()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
    for x, y in ev:
        x.record(s)
        launch()
        y.record(s)
    torch.cuda.synchronize()
    ms = [x.elapsed_time(y) for x, y in ev]
    got = res.cpu().numpy().view(abi.NDC_RESULT)
    m = 100_000
    want, _ = oracle.ndc_prepare(ndc.NdcBatch(tasks=nb.tasks[:m], branches=nb.branches, items=nb.items,
                                              n_out_items=nb.n_out_items))
    print(json.dumps({"lib": a.lib, "tasks": n, "kernel_ms": ms, "median_ms": float(np.median(ms)),
                      "tasks_per_s": n / (float(np.median(ms)) * 1e-3),
                      "bit_exact_sample": bool(got[:m].tobytes() == want.tobytes())}), flush=True)


if __name__ == "__main__":
    main()
