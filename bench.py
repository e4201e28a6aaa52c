"""Benchmark: history events replayed/s (+ workflows rebuilt/s, % of HBM peak) on MI355X.

One step = one crr_replay launch over this rank's whole shard of workflows (config 2 shape:
activity-chain histories of 29 events, 1M workflows per GPU), inputs resident in HBM, followed
(N > 1) by the job's one exchange: an RCCL all-reduce of counters and the checksum digest.
Weak scaling: every rank replays its own shard (shards = disjoint workflow sets, as Cadence
partitions workflows by shardID); value = events of all ranks / max-over-ranks wall time.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
PROFILE_TRAFFIC = os.path.join(ROOT, "profiles", "traffic.json")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workflows", type=int, default=1_000_000, help="workflows per GPU (config 2: 1M)")
    p.add_argument("--activities", type=int, default=4, help="activities per workflow (k=4 -> 29 events)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0, help="threads for the CPU baseline (0: os cpu share)")
    p.add_argument("--cpu-sample", type=int, default=1_000_000, help="workflows in the CPU baseline sample")
    p.add_argument("--cpu-seconds", type=float, default=2.0,
                   help="minimum wall seconds of CPU-baseline replay (x threads = CPU seconds; 2 s x 16 = 32)")
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    from cadence_amd import dist as cdist
    from cadence_amd import synth
    from cadence_amd.engine import ReplayEngine
    from cadence_amd.flatten import interleave

    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", local_rank))
    eng = ReplayEngine(local_rank)

    k = args.activities
    n_wf = args.workflows
    t0 = time.time()
    canon = synth.activity_chain(n_wf, k, synth.SEED_C2 + rank, with_keys=False)
    batch = interleave(canon)
    db = eng.upload(batch)
    gen_s = time.time() - t0
    n_events = batch.n_events
    stream = torch.cuda.current_stream()

    for _ in range(args.warmup):
        eng.launch(db, stream)
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.timing_begin()          # per-launch HIP events around the dominant kernel, on the launch stream
    t_start = time.perf_counter()
    for _ in range(args.steps):
        eng.launch(db, stream)
        if world > 1:
            d = cdist.digest_torch(torch, db.tensors["exec"], n_wf)
            cdist.all_reduce_digest(torch, dist, d)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    ms = eng.timing_read()
    if len(ms) != args.steps:
        raise RuntimeError(f"timed {len(ms)} kernel launches, expected {args.steps}")
    kernel_avg_ms = float(np.mean(ms))

    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max = float(t.item())

    res = eng.download(db)
    from cadence_amd import abi
    tier = "replay_lds_small_kernel" if db.c_in.flags & abi.IN_LDS_SMALL else "replay_lds_kernel"
    tail = bool(db.c_in.flags & abi.IN_WAVE_TAIL) and db.c_in.wave_begin < db.n_wf
    emit = bool(db.c_in.flags & abi.IN_EMIT_TASKS)
    kernel_name = f"{tier}<{str(tail).lower()}, {str(emit).lower()}>"  # <WAVE_TAIL, EMIT>, as rocprofv3 names it
    ok = bool((res.exec["status"] == 0).all())
    alg_bytes = synth.algorithmic_bytes(batch, res)
    achieved_gbs = alg_bytes / (kernel_avg_ms * 1e-3) / 1e9

    total_events = n_events * world * args.steps
    value = total_events / elapsed_max
    line = {
        "metric": "history events replayed/sec (node) + workflows rebuilt/sec; % HBM peak",
        "value": value,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic",
        "config": {"workload": "config 2: activity-chain histories (schedule/start/complete + decisions), "
                               f"{k} activities = {n_events // n_wf} events/workflow, {n_wf} workflows per GPU, "
                               "wave-interleaved SoA resident in HBM",
                   "workflows_per_gpu": n_wf, "events_per_workflow": n_events // n_wf,
                   "parallelism": f"shard-partitioned x{world} (RCCL all-reduce of counters + checksum digest)"},
        "workflows_per_s": n_wf * world * args.steps / elapsed_max,
        "all_ok": ok,
        "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": None,
                     "kernel": kernel_name, "kernel_ms": kernel_avg_ms,
                     "algorithmic_bytes_per_launch": alg_bytes},
        "setup_s": gen_s,
    }
    if os.path.exists(PROFILE_TRAFFIC):
        try:
            tr = json.load(open(PROFILE_TRAFFIC))
            if (tr.get("workflows") == n_wf and tr.get("events_per_workflow") == n_events // n_wf
                    and tr.get("kernel") == kernel_name):
                line["roofline"]["traffic"] = tr.get("hbm_bytes_per_launch")
        except Exception:
            pass

    if rank == 0 and world == 1:
        line["pcie_inclusive"] = pcie_inclusive(eng, batch, torch)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args, res, batch, k)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def pcie_inclusive(eng, batch, torch, reps=3):
    """SURVEY.md §8d's second figure: one replay with host buffers -- device allocation + H2D of the
    columns, side records and descriptors, the replay, D2H of the execution rows and the slot
    tables -- never the headline `value` (which has the inputs resident in HBM)."""
    times, parts = [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        db = eng.upload(batch)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        eng.launch(db)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        r = eng.download(db)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        times.append(t3 - t0)
        parts.append((t1 - t0, t2 - t1, t3 - t2))
        del db, r
    t = float(np.median(times))
    up, run, down = (float(np.median([p[i] for p in parts])) * 1e3 for i in range(3))
    h2d = sum(v.nbytes for v in batch.cols.values()) + batch.act_side.nbytes + batch.start_side.nbytes \
        + batch.arena.nbytes + batch.wf.nbytes
    return {"events_per_s": batch.n_events / t, "ms": t * 1e3, "h2d_bytes": int(h2d),
            "upload_ms": up, "replay_ms": run, "download_ms": down,
            "note": "pageable host buffers, allocation + upload + replay + download of exec rows and slot tables"}


def cpu_baseline(args, gpu_res, gpu_batch, k):
    """The oracle (C++ restatement of the Go stateBuilder, per-workflow hash maps) on host cores,
    over a bounded sample of the same workload; also checks the GPU rows against it."""
    from cadence_amd import synth
    from cadence_amd.result import diff_results
    from oracle import oracle
    n = min(args.cpu_sample, args.workflows)
    threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
    sample = synth.activity_chain(n, k, synth.SEED_C2, with_keys=True)
    # repeat whole passes over the sample until >= cpu_seconds of wall time (bounded CPU work)
    passes, dt, res = 0, 0.0, None
    while passes == 0 or dt < args.cpu_seconds:
        t0 = time.perf_counter()
        r = oracle.replay(sample, threads)
        dt += time.perf_counter() - t0
        res = res if res is not None else r
        passes += 1
    out = {"value": sample.n_events * passes / dt, "unit": "events/s", "cores": threads, "kind": "port",
           "sample": f"{passes} pass(es) over {n} config-2 workflows ({sample.n_events} events), seed SEED_C2, "
                     f"{threads} std::thread workers, CPU restatement of Go stateBuilder (reference not runnable)",
           "wall_s": dt, "cpu_seconds_approx": dt * threads}
    if n == args.workflows:
        d = diff_results(gpu_batch, gpu_res, sample, res)
        out["gpu_parity_bit_exact"] = not d
    return out


if __name__ == "__main__":
    main()
