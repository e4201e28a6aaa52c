"""Benchmark: history events replayed/s (+ workflows rebuilt/s, % of HBM peak) on MI355X.

Headline (``value``): BASELINE config 2 -- activity-chain histories of 29 events, 1M workflows per
GPU, inputs resident in HBM; one step = one crr_replay over this rank's shard (every workflow
rebuilt from scratch, checksum included), followed (N > 1) by the job's one exchange, an RCCL
all-reduce of the counters + checksum digest.  N ranks split ONE global workload (N x 1M workflows)
by history shard (dist.rank_workflows: shard = hash(workflow) mod 16384, shard -> rank = shard mod N),
so per-GPU work is fixed (weak scaling); value = events of all ranks / max-over-ranks wall time.

Beside it, on every rank with the same shard split and timing rules (``configs``):
  config 3 -- 1.25M mixed histories per GPU (the per-GPU shard of the 10M x 8-GPU job),
  config 4 -- long-tail histories (Zipf lengths up to 50k events, continue-as-new every 10k),
  passive replication -- the last batch of every config-3 history applied onto its loaded state,
each with its roofline and a bit-exact parity check against the oracle on a sample; and on rank 0 at
N=1: the end-to-end figure from host buffers (pinned, chunked, overlapped, compacted download), the
host-ingest rates (native decoder, flatten) and the CPU baseline (oracle on the host cores, config 2
sample and BASELINE config 1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--headline-only]
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
PROFILE_TRAFFIC_CONFIGS = os.path.join(ROOT, "profiles", "traffic_configs.json")
MAX_TIMED_STEPS = 512   # crr_timing ring size (capi.hip kRing)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workflows", type=int, default=1_000_000, help="config 2 workflows per GPU (1M)")
    p.add_argument("--activities", type=int, default=4, help="activities per workflow (k=4 -> 29 events)")
    p.add_argument("--headline-only", action="store_true", help="config 2 only (no configs 3/4, e2e, CPU)")
    p.add_argument("--config-steps", type=int, default=5, help="timed steps of the config 3 / 4 / replication lines")
    p.add_argument("--c3-workflows", type=int, default=1_250_000, help="config 3 mixed workflows per GPU")
    p.add_argument("--json-workflows", type=int, default=125_000,
                   help="workflows of the JSON-encoded device ingest line (config-3 shape, rank 0, N = 1)")
    p.add_argument("--c4-workflows", type=int, default=2000, help="config 4 logical workflows per GPU")
    p.add_argument("--c5-workflows", type=int, default=1_000_000, help="config 5 multi-version workflows per GPU")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-token-crc", action="store_true", help="hash the start tokens in the replay (A/B of crr_inputs.token_crc)")
    p.add_argument("--no-e2e", action="store_true", help="skip the host-buffer, host-ingest and blob -> rows figures")
    p.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: the CPUs this process may use)")
    p.add_argument("--cpu-sample", type=int, default=1_000_000, help="config 2 workflows in the CPU baseline sample")
    p.add_argument("--cpu-seconds", type=float, default=2.0, help="minimum wall seconds per CPU-baseline figure")
    p.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                   help="collective backend for N > 1 (nccl = RCCL; gloo: e.g. several ranks sharing one GPU)")
    p.add_argument("--device", type=int, default=-1, help="GPU of this rank (default LOCAL_RANK)")
    a = p.parse_args()
    if a.steps > MAX_TIMED_STEPS or a.config_steps > MAX_TIMED_STEPS:
        p.error(f"--steps / --config-steps: at most {MAX_TIMED_STEPS} launches are timed per region")
    if a.steps < 1:
        p.error("--steps must be >= 1")
    return a


def progress(msg):
    """A progress line on stderr (the JSON result stays the only stdout line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def host_cpus() -> int:
    """CPUs this process may run on: the cgroup CPU quota when one is set (the GPU box's per-GPU share),
    else the affinity mask."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


class Ctx:
    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.args = args
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.device = args.device if args.device >= 0 else self.local_rank
        self.backend = args.backend
        torch.cuda.set_device(self.device)
        if self.world > 1:
            if self.backend == "nccl":
                dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", self.device))
            else:
                dist.init_process_group("gloo", init_method="env://")
        from cadence_amd.engine import ReplayEngine
        self.eng = ReplayEngine(self.device)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def reduce(self, values, op="max"):
        """All-reduce a list of floats over the ranks (identity at N=1)."""
        t = self.torch.tensor(values, dtype=self.torch.float64, device="cuda" if self.backend == "nccl" else "cpu")
        if self.world > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return [float(x) for x in t.cpu()]


def timed_steps(ctx, db, steps, warmup, per_step=None, before_step=None):
    """warmup, barrier + sync, K launches (HIP-event ring around each launch's fast group), sync +
    barrier; returns (max-over-ranks wall seconds, per-launch fast-group ms)."""
    torch, eng = ctx.torch, ctx.eng
    stream = torch.cuda.current_stream()
    for _ in range(warmup):
        if before_step:
            before_step()
        eng.launch(db, stream)
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    eng.timing_begin()
    wall = 0.0
    if before_step is None:
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.launch(db, stream)
            if per_step:
                per_step()
        torch.cuda.synchronize()
        ctx.barrier()
        wall = time.perf_counter() - t0
    else:
        # each step restores its input state first (device copy, synchronised, outside the clock)
        for _ in range(steps):
            before_step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.launch(db, stream)
            torch.cuda.synchronize()
            wall += time.perf_counter() - t0
        ctx.barrier()
    ms = eng.timing_read()
    if len(ms) != steps:
        raise RuntimeError(f"timed {len(ms)} kernel launches, expected {steps}")
    return ctx.reduce([wall])[0], ms


def roofline(alg_bytes, kernel_ms, kernel, traffic=None):
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
         "traffic": traffic, "kernel": kernel, "kernel_ms": kernel_ms, "algorithmic_bytes_per_launch": int(alg_bytes)}
    if traffic:
        r["traffic_GBs"] = traffic / (kernel_ms * 1e-3) / 1e9
        r["traffic_frac"] = r["traffic_GBs"] / HBM_PEAK_GBS
    return r


# ---- config 2 (headline) -------------------------------------------------------------------------------
def config2(ctx):
    from cadence_amd import abi, synth
    from cadence_amd import dist as cdist
    from cadence_amd.flatten import interleave
    args, torch, eng = ctx.args, ctx.torch, ctx.eng
    k = args.activities
    t0 = time.time()
    ids = cdist.rank_workflows(args.workflows * ctx.world, ctx.rank, ctx.world)
    canon = synth.activity_chain(ids.size, k, synth.SEED_C2, with_keys=False, wf_ids=ids)
    batch = interleave(canon)
    db = eng.upload(batch, token_crc=not ctx.args.no_token_crc)
    # the digest is folded into every replay launch (crr_outputs.digest), bound to each device position's
    # global workflow ID; the step's exchange is then the one RCCL all-reduce of its 1-KB buffer
    eng.enable_digest(db, cdist.device_keys(batch, ids))
    setup_s = time.time() - t0
    n_wf, n_events = batch.n_wf, batch.n_events

    def exchange():
        cdist.all_reduce_digest(torch, ctx.dist, db.tensors["digest"])

    wall, ms = timed_steps(ctx, db, args.steps, args.warmup, per_step=exchange if ctx.world > 1 else None)
    kernel_avg_ms = float(np.mean(ms))
    eng.launch(db)   # the reported digest: one more launch, reduced once
    if ctx.world > 1:
        cdist.all_reduce_digest(torch, ctx.dist, db.tensors["digest"])
    digest = eng.read_digest(db)
    tot_events, tot_wf = ctx.reduce([float(n_events), float(n_wf)], op="sum")
    res = eng.download(db)
    tier = "replay_lds_small_kernel" if db.c_in.flags & abi.IN_LDS_SMALL else "replay_lds_kernel"
    tail = bool(db.c_in.flags & abi.IN_WAVE_TAIL) and db.c_in.wave_begin < db.n_wf
    emit = bool(db.c_in.flags & abi.IN_EMIT_TASKS)
    kernel_name = f"{tier}<{str(tail).lower()}, {str(emit).lower()}"  # <WAVE_TAIL, EMIT[, LANES]>, as rocprofv3 names it
    # the small tier's third parameter (divergent dispatch) is set only for multi-segment (mixed) batches
    kernel_name += ", false>" if tier == "replay_lds_small_kernel" else ">"
    alg_bytes = synth.algorithmic_bytes(batch, res, token_crc=not ctx.args.no_token_crc)
    traffic = None
    if os.path.exists(PROFILE_TRAFFIC):
        try:
            tr = json.load(open(PROFILE_TRAFFIC))
            if (tr.get("workflows") == n_wf and tr.get("events_per_workflow") == n_events // n_wf
                    and tr.get("kernel") == kernel_name):
                traffic = tr.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
    line = {
        "metric": "history events replayed/sec (node) + workflows rebuilt/sec; % HBM peak",
        "value": tot_events * args.steps / wall,
        "unit": "events/s",
        "n_gpus": ctx.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (seeded activity-chain histories, per-workflow draws)",
        "config": {"workload": "config 2: activity-chain histories (schedule/start/complete + decisions), "
                               f"{k} activities = {n_events // n_wf} events/workflow, {args.workflows} workflows per GPU "
                               f"(one {args.workflows * ctx.world}-workflow workload split by history shard), "
                               "wave-interleaved SoA resident in HBM",
                   "workflows_per_gpu": n_wf, "events_per_workflow": n_events // n_wf,
                   "parallelism": f"shard-partitioned x{ctx.world} ("
                                  f"{'RCCL' if ctx.backend == 'nccl' else 'gloo'} all-reduce of counters + checksum digest)"},
        "workflows_per_s": tot_wf * args.steps / wall,
        "all_ok": bool(digest[2] == 0 and digest[1] == tot_wf),
        "digest": [int(x) for x in digest],
        "digest_note": "folded into the replay launch (crr_outputs.digest: wave sums, 64-bit atomics into 8 striped lines); "
                       "N > 1: one RCCL all-reduce of that 1-KB buffer per step, no other kernel",
        "roofline": roofline(alg_bytes, kernel_avg_ms, kernel_name, traffic),
        "setup_s": setup_s,
    }
    return line, batch, res, db


# ---- configs 3 / 4 and passive replication ----------------------------------------------------------
FAST_GROUP = "crr_replay phase-1 launch group (tier kernels on side streams, fork to join)"


def config_traffic(name, n_wf, n_events):
    """HBM bytes per launch group of a non-headline line, from its PMC passes (tools/traffic_configs.py,
    profiles/traffic_configs.json) when they were taken on this exact workload; else None."""
    try:
        tr = json.load(open(PROFILE_TRAFFIC_CONFIGS)).get(name)
    except (OSError, ValueError):
        return None
    if tr and tr.get("workflows") == n_wf and tr.get("events") == n_events:
        return tr.get("hbm_bytes_per_launch")
    return None


def run_config(ctx, name, make_canon, workload, sample_fn, long_threshold=256, global_ids=None):
    """One non-headline line: generate this rank's shard, time `config_steps` replays (each with the fused
    digest and, N > 1, its RCCL all-reduce: BASELINE config 3's "RCCL checksum reduce"), roofline over the
    launch group, parity of the timed replays' own rows and of a sample against the oracle (rank 0)."""
    from cadence_amd import synth
    from cadence_amd.flatten import interleave
    args, torch, eng = ctx.args, ctx.torch, ctx.eng
    t0 = time.time()
    canon = make_canon()
    t1 = time.time()
    batch = interleave(canon, long_threshold=long_threshold)
    t2 = time.time()
    db = eng.upload(batch, token_crc=not ctx.args.no_token_crc)
    keys = digest_keys(ctx, batch, global_ids)
    eng.enable_digest(db, keys)
    wall, ms = timed_steps(ctx, db, args.config_steps, 1, per_step=digest_exchange(ctx, db))
    res = eng.download(db)
    dg = digest_check(ctx, db, res, batch, keys)
    tot_events, tot_wf = ctx.reduce([float(batch.n_events), float(batch.n_wf)], op="sum")
    grp_ms = float(np.mean(ms))
    out = {"workload": workload, "value": tot_events * args.config_steps / wall, "unit": "events/s",
           "ms_per_step": wall / args.config_steps * 1e3, "steps": args.config_steps,
           "workflows_per_gpu": batch.n_wf, "events_per_gpu": batch.n_events, "workflows_ok": dg["digest"][1],
           "workflows_per_s": tot_wf * args.config_steps / wall,
           "tiers": list(batch.tiers) if batch.tiers else None, "wave_tail": batch.n_wf - (batch.wave_begin or batch.n_wf),
           "digest": dg,
           "roofline": roofline(synth.algorithmic_bytes(batch, res, token_crc=not ctx.args.no_token_crc), grp_ms, FAST_GROUP,
                                config_traffic(name, batch.n_wf, batch.n_events)),
           "setup_s": {"generate": t1 - t0, "interleave": t2 - t1}}
    if ctx.rank == 0:
        out["parity_sample"] = parity_sample(ctx, sample_fn, long_threshold)
        out["parity_full"] = full_parity(ctx, batch, res, canon)
    return out, batch, res, db


def digest_keys(ctx, batch, global_ids=None):
    """Identity keys of the batch's workflows in device order: the global workflow IDs of this rank's part
    of the job (the generator's shard split, dist.rank_workflows) when they are known and match the batch,
    else rank-qualified local indices (still unique across ranks)."""
    from cadence_amd import dist as cdist
    if global_ids is None or len(global_ids) != batch.n_wf:
        global_ids = (np.int64(ctx.rank) << np.int64(40)) + np.arange(batch.n_wf, dtype=np.int64)
    return cdist.device_keys(batch, global_ids)


def digest_exchange(ctx, db):
    """The step's exchange at N > 1: the one RCCL all-reduce of the fused digest's 1-KB buffer."""
    if ctx.world == 1:
        return None
    from cadence_amd import dist as cdist
    return lambda: cdist.all_reduce_digest(ctx.torch, ctx.dist, db.tensors["digest"])


def digest_check(ctx, db, res, batch, keys):
    """The last timed step's (all-reduced) device digest against the host restatement of the same rows
    (dist.digest_numpy per rank, summed over the ranks as int64)."""
    from cadence_amd import dist as cdist
    got = ctx.eng.read_digest(db)
    want = cdist.digest_numpy(res.exec, batch.wf["ev_count"], keys)
    if ctx.world > 1:
        torch = ctx.torch
        t = torch.from_numpy(want.copy())
        if ctx.backend == "nccl":
            t = t.to(ctx.eng.dev)
        ctx.dist.all_reduce(t, op=ctx.dist.ReduceOp.SUM)
        want = t.cpu().numpy()
    return {"digest": [int(x) for x in got], "matches_host_digest": bool((got == want).all()),
            "fields": "events_ok, workflows_ok, workflows_failed, crc_sum, identity_fold, inconsistencies, failed_fold",
            "reduce": "fused into each timed replay launch" + (f"; one {'RCCL' if ctx.backend == 'nccl' else 'gloo'} "
                                                                 "all-reduce of its 1-KB buffer per timed step"
                                                                 if ctx.world > 1 else "")}


def full_parity(ctx, batch, res, canon):
    """The timed replays' own results -- every workflow of the rank's shard, every row -- against the oracle
    (outside the clock)."""
    from oracle import oracle
    from cadence_amd.result import diff_results
    t0 = time.perf_counter()
    ref = oracle.replay(canon, host_cpus())
    dt = time.perf_counter() - t0
    d = diff_results(batch, res, canon, ref)
    return {"workflows": canon.n_wf, "events": canon.n_events, "bit_exact": not d, "first_diffs": d[:3],
            "oracle_s": dt}


def parity_sample(ctx, sample_fn, long_threshold):
    from oracle import oracle
    from cadence_amd.flatten import interleave
    from cadence_amd.result import diff_results
    canon = sample_fn()
    b = interleave(canon, long_threshold=long_threshold)
    gpu = ctx.eng.replay(b)
    t0 = time.perf_counter()
    ref = oracle.replay(canon, host_cpus())
    dt = time.perf_counter() - t0
    d = diff_results(b, gpu, canon, ref)
    return {"workflows": canon.n_wf, "events": canon.n_events, "bit_exact": not d, "first_diffs": d[:3],
            "oracle_s": dt, "ok": int((gpu.exec["status"] == 0).sum())}


def passive_replication(ctx, batch, one_shot, make_canon=None):
    from cadence_amd.replication import PassiveReplication
    args, eng = ctx.args, ctx.eng
    pr = PassiveReplication(eng, batch)
    pr.setup()
    wall, ms = timed_steps(ctx, pr.db_new, args.config_steps, 1, before_step=pr.restore)
    v = pr.verify(one_shot)
    blob_path = None
    if make_canon is not None and not args.no_e2e:
        blob_path = replication_blob_path(ctx, pr, make_canon)
    tot_ev, tot_tasks = ctx.reduce([float(pr.n_events), float(v["split_workflows"])], op="sum")
    out = {"workload": "config 3 shard: the last event batch of every history applied onto its loaded mutable state "
                       "(ndc/history_replicator.go:385-460 -> StateBuilder.ApplyEvents on a Load-ed state), rows in HBM",
           "value": tot_ev * args.config_steps / wall, "unit": "events/s",
           "replication_tasks_per_s": tot_tasks * args.config_steps / wall,
           "ms_per_step": wall / args.config_steps * 1e3, "steps": args.config_steps,
           "events_per_gpu": pr.n_events, "tasks_per_gpu": v["split_workflows"],
           "vs_one_shot": v,
           "roofline": roofline(_resume_bytes(pr), float(np.mean(ms)), FAST_GROUP,   # (replication uploads splice)
                                config_traffic("passive_replication", pr.batch.n_wf, pr.n_events))}
    if blob_path is not None:
        out["blob_path"] = blob_path
    if ctx.rank == 0:   # every split workflow, the Load-unstable ones included: the oracle given the same split
        from oracle import oracle
        t0 = time.perf_counter()
        out["vs_oracle"] = pr.verify_oracle(oracle.replay, host_cpus())
        out["vs_oracle"]["oracle_s"] = time.perf_counter() - t0
        # the loaded states themselves: the whole-shard prefix replay against the oracle
        t0 = time.perf_counter()
        out["vs_oracle"]["prefix"] = pr.verify_prefix_oracle(oracle.replay, host_cpus())
        out["vs_oracle"]["prefix"]["oracle_s"] = time.perf_counter() - t0
    del pr
    return out


def replication_blob_path(ctx, pr, make_canon):
    """The same replication step from the tasks' persisted bytes: each split workflow's last batch as the
    thriftrw blob persistence stored (replication_task.go:386-390), decoded and laid out on the device onto
    the loaded states (crr_ingest_plan_resume -- its two stream syncs included -- + crr_ingest_layout_resume,
    serializer.go:109-119), then replayed onto the loaded rows in place.  `device_resident`: the blobs already
    in HBM; `pcie_inclusive`: from pinned host buffers, the H2D copies inside the clock.  Each step restores
    the loaded rows first (outside the clock); the rows after the timed steps equal the host path's step."""
    from cadence_amd import abi
    from cadence_amd.blobs import encode_batch
    from cadence_amd.replication import BlobReplication
    torch, eng, args = ctx.torch, ctx.eng, ctx.args
    t0 = time.time()
    canon = make_canon()
    bs = encode_batch(canon)
    del canon
    enc_s = time.time() - t0
    br = BlobReplication(pr, bs)
    br.setup()
    stream = torch.cuda.current_stream()
    # the host path's step: what the blob path's rows must equal
    pr.restore()
    pr.step(stream)
    want = eng.download(pr.db)
    # per task over PCIe: the blobs, their offsets and per-workflow ranges; the loaded key dictionaries (after the
    # blobs in the same buffer), the string arena and the known domains stay resident with the loaded states
    rb = br.blobs.blobs
    host = {"bytes": rb.bytes[:rb.n_bytes], "blob_off": rb.blob_off, "wf": rb.wf.view(np.uint8)}
    pinned = {k: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).pin_memory() for k, a in host.items()}
    h2d_bytes = sum(int(t.numel()) for t in pinned.values())

    def run(steps, pcie):
        wall = 0.0
        for _ in range(steps):
            pr.restore(stream)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if pcie:
                for k, t in pinned.items():
                    if t.numel():
                        br.blobs.tensors[k][:t.numel()].copy_(t, non_blocking=True)
            br.step(stream)
            torch.cuda.synchronize()
            wall += time.perf_counter() - t1
        return wall

    run(1, False)
    ctx.barrier()
    eng.timing_begin()
    wall = ctx.reduce([run(args.config_steps, False)])[0]
    ms = eng.timing_read()
    got = eng.download(pr.db)
    same = got.exec.tobytes() == want.exec.tobytes() and all(
        got.tables[t[0]].tobytes() == want.tables[t[0]].tobytes() for t in abi.TABLES if t[0] != "tasks")
    run(1, True)
    ctx.barrier()
    wall_p = ctx.reduce([run(args.config_steps, True)])[0]
    got_p = eng.download(pr.db)
    same_p = got_p.exec.tobytes() == want.exec.tobytes()
    # attribution: plan + layout alone (a sync after the layout), the rest is the replay
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.config_steps):
        S = br.ing.plan(br.blobs, stream, resume=br.resume)
        br.ing.layout_resume(br.blobs, br.resume, S, br.db.c_in, stream)
    torch.cuda.synchronize()
    ingest_ms = (time.perf_counter() - t1) / args.config_steps * 1e3
    tot_ev, tot_tasks = ctx.reduce([float(br.n_events), float(pr.split.sum())], op="sum")
    k = args.config_steps
    out = {"workload": "the replication tasks' persisted batches (one thriftrw blob per split workflow) -> device decode + "
                       "layout onto the loaded states -> ApplyEvents onto the loaded rows in place",
           "device_resident": {"events_per_s": tot_ev * k / wall, "replication_tasks_per_s": tot_tasks * k / wall,
                               "ms_per_step": wall / k * 1e3, "ingest_ms": ingest_ms,
                               "replay_kernel_ms": float(np.mean(ms)), "rows_equal_host_path": bool(same)},
           "pcie_inclusive": {"events_per_s": tot_ev * k / wall_p, "ms_per_step": wall_p / k * 1e3,
                              "h2d_bytes": h2d_bytes, "h2d_GBs": h2d_bytes * k / wall_p / 1e9,
                              "rows_equal_host_path": bool(same_p)},
           "blobs": int(rb.n_blobs), "blob_bytes": int(rb.n_bytes), "events_per_gpu": br.n_events,
           "setup_s": {"encode": enc_s}}
    del br, pinned
    torch.cuda.empty_cache()
    return out


def _resume_bytes(pr, token_crc=True):
    """Algorithmic bytes of one replication step: the new events' columns, the descriptor, the loaded
    exec row read and written, the loaded + final live rows (read, then written back), the token (its 4-byte
    precomputed CRC with crr_inputs.token_crc)."""
    from cadence_amd import abi
    b = pr.batch
    ex = pr.prefix.exec
    rows = (112 * ex["n_activity"].astype(np.int64).sum() + 40 * ex["n_timer"].astype(np.int64).sum()
            + 48 * ex["n_child"].astype(np.int64).sum() + 32 * (ex["n_rc"].astype(np.int64).sum() + ex["n_signal"].astype(np.int64).sum())
            + 16 * ex["n_vh_items"].astype(np.int64).sum() + 16 * ex["n_reset_points"].astype(np.int64).sum())
    return int(pr.n_events * abi.BYTES_PER_EVENT + b.n_wf * (abi.WORKFLOW.itemsize + 2 * abi.EXEC_ROW.itemsize
                                                             + (4 if token_crc else 96)) + 2 * rows)


# ---- config 5: NDC / XDC -----------------------------------------------------------------------------------------
def config5(ctx, n_wf, shard, global_ids=None):
    """BASELINE config 5 on this rank's shards: (a) multi-version mixed histories rebuilt onto a reset
    branch (Rebuild: the target branch token, the last-item check, RefreshTasks) -- failover versions at
    batch boundaries give 1-4 VersionHistory items; (b) crr_ndc_prepare over one replication task per
    workflow against its replayed VersionHistory (append / new branch / duplicate / out-of-order); (c)
    crr_checksum, the Load verify path, over the replayed rows.  Each with its roofline and an oracle
    parity check."""
    from cadence_amd import ndc, synth, synth_native
    from cadence_amd.flatten import interleave
    args, torch, eng = ctx.args, ctx.torch, ctx.eng
    t0 = time.time()
    canon = as_rebuilds(synth_native.mixed(n_wf * ctx.world, multi_version=True, shard=shard, seed=0xCAD00005), 0xCAD00005,
                        global_ids)
    batch = interleave(canon)
    db = eng.upload(batch, token_crc=not ctx.args.no_token_crc)
    setup = time.time() - t0
    keys = digest_keys(ctx, batch, global_ids)
    eng.enable_digest(db, keys)
    wall, ms = timed_steps(ctx, db, args.config_steps, 1, per_step=digest_exchange(ctx, db))
    res = eng.download(db)
    dg = digest_check(ctx, db, res, batch, keys)
    tot_ev, tot_wf = ctx.reduce([float(batch.n_events), float(batch.n_wf)], op="sum")
    out = {"workload": f"config 5: {n_wf} multi-version mixed histories per GPU rebuilt onto reset branches "
                       "(state_rebuilder.go:97-191: target branch token, last-item check, RefreshTasks), failover "
                       "versions at batch boundaries",
           "rebuild": {"value": tot_ev * args.config_steps / wall, "unit": "events/s",
                       "workflows_rebuilt_per_s": tot_wf * args.config_steps / wall,
                       "ms_per_step": wall / args.config_steps * 1e3, "steps": args.config_steps,
                       "events_per_gpu": batch.n_events, "workflows_per_gpu": batch.n_wf,
                       "workflows_ok": dg["digest"][1], "digest": dg,
                       "vh_items_per_workflow": float(res.exec["n_vh_items"][res.exec["status"] == 0].mean()),
                       "roofline": roofline(synth.algorithmic_bytes(batch, res, token_crc=not ctx.args.no_token_crc), float(np.mean(ms)), FAST_GROUP,
                                            config_traffic("config5_rebuild", batch.n_wf, batch.n_events)),
                       "setup_s": setup}}
    if ctx.rank == 0:
        # the timed replays' own rows, every workflow, against the oracle
        out["rebuild"]["parity_full"] = full_parity(ctx, batch, res, canon)
    # (b) NDC branch decisions
    e, v, c = ndc.version_histories(canon)
    nb = ndc.tasks_from_histories(e, v, c, 0xCAD00025 + ctx.rank)
    out["ndc_prepare"] = ndc_line(ctx, nb)
    # (c) Load verify
    out["checksum_verify"] = checksum_line(ctx, db, batch, res)
    del db
    return out


def as_rebuilds(canon, seed, global_ids=None):
    """Rebuild inputs for every workflow of a canonical batch: StateRebuilder.Rebuild replays the history
    onto a new branch whose token it installs (state_rebuilder.go:150), checks the last VersionHistory item
    against the requested (event ID, version) (:160-176; 2 % are given a mismatching one) and refreshes the
    tasks (:183).  With ``global_ids`` (the workflows' indices in the whole job) every draw is a hash of
    (seed, workflow), so a rank's part of the job equals the same workflows of the N = 1 run."""
    from cadence_amd import abi, synth
    from cadence_amd import dist as cdist
    rng = np.random.default_rng(seed)
    n = canon.n_wf
    if global_ids is not None and len(global_ids) == n:
        g = np.asarray(global_ids, np.uint64)
        with np.errstate(over="ignore"):
            h = np.stack([cdist.mix64(g * np.uint64(4) + np.uint64(seed) + np.uint64(k)) for k in range(3)], axis=1)
        raw = h[:, :2].copy().view(np.uint8).reshape(n, 16)
        tok = synth.branch_tokens(canon.arena[(canon.wf["start_token_off"].astype(np.int64)[:, None] + 8
                                               + np.arange(36)[None, :])], synth.uuid_ascii_raw(raw))
        mismatch = (h[:, 2] % np.uint64(10000)) < np.uint64(200)
        return _install_rebuilds(canon, tok, mismatch)
    tree = canon.arena[(canon.wf["start_token_off"].astype(np.int64)[:, None] + 8 + np.arange(36)[None, :])]
    tok = synth.branch_tokens(tree, synth.uuid_ascii(rng, n))
    return _install_rebuilds(canon, tok, rng.random(n) < 0.02)


def _install_rebuilds(canon, tok, mismatch):
    from cadence_amd import abi
    n = canon.n_wf
    cnt = canon.wf["ev_count"].astype(np.int64)
    last = canon.wf["ev_begin"].astype(np.int64) + np.maximum(cnt - 1, 0)
    base = canon.arena.size
    canon.arena = np.concatenate([canon.arena, tok.reshape(-1)])
    canon.wf["final_token_off"] = base + np.arange(n, dtype=np.int64) * 96
    canon.wf["final_token_len"] = 96
    ok = cnt > 0
    canon.wf["rebuild_last_event_id"] = np.where(ok, canon.cols["event_id"][last], 0) + mismatch
    canon.wf["rebuild_last_event_version"] = np.where(ok, canon.cols["version"][last], 0)
    canon.wf["flags"] |= abi.WF_FLAG_REFRESH_TASKS
    return canon


def ndc_line(ctx, nb):
    from cadence_amd import abi, ndc
    from oracle import oracle
    torch, eng, args = ctx.torch, ctx.eng, ctx.args
    dev = eng.dev
    n = len(nb.tasks)

    def up(a):
        raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        t = torch.empty(max(raw.size, 1), dtype=torch.uint8, device=dev)
        t[:raw.size].copy_(torch.from_numpy(raw))
        return t

    T = {"tasks": up(nb.tasks), "branches": up(nb.branches), "items": up(nb.items)}
    res = torch.zeros(max(n, 1) * abi.NDC_RESULT.itemsize, dtype=torch.uint8, device=dev)
    out = torch.zeros(nb.n_out_items * abi.VH_ITEM.itemsize, dtype=torch.uint8, device=dev)
    ci = abi.CNdcInputs()
    ci.tasks, ci.branches, ci.items = T["tasks"].data_ptr(), T["branches"].data_ptr(), T["items"].data_ptr()
    ci.n_tasks = n
    import ctypes
    s = torch.cuda.current_stream(dev)

    def launch():
        rc = eng.lib.crr_ndc_prepare(ctypes.byref(ci), ctypes.c_void_p(res.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                     ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"crr_ndc_prepare failed: {rc}")

    launch()
    torch.cuda.synchronize()
    ctx.barrier()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.config_steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(s)
        launch()
        b.record(s)
    torch.cuda.synchronize()
    ctx.barrier()
    wall = ctx.reduce([time.perf_counter() - t0])[0]
    k_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    got = res.cpu().numpy().view(abi.NDC_RESULT)[:n]
    tot = ctx.reduce([float(n)], op="sum")[0]
    # algorithmic bytes: the task, its branch descriptors and every item read, the result and the new
    # branch's items written
    alg = (n * (abi.NDC_TASK.itemsize + abi.NDC_RESULT.itemsize) + int(nb.tasks["branch_count"].sum()) * abi.NDC_BRANCH.itemsize
           + int(nb.branches["item_count"].sum() + nb.tasks["incoming_count"].sum()) * abi.VH_ITEM.itemsize
           + int(got["new_item_count"].clip(0).sum()) * abi.VH_ITEM.itemsize)
    line = {"workload": "one replication task per workflow against its replayed VersionHistories: prepareVersionHistory "
                        "(ndc/branch_manager.go:87-149) -- LCA, appendable / fork, DuplicateUntilLCAItem, AddVersionHistory, "
                        "verifyEventsOrder, IsRebuilt",
            "value": tot * args.config_steps / wall, "unit": "replication tasks/s", "tasks_per_gpu": n,
            "outcomes": {k: int(v) for k, v in zip(("append", "new_branch", "duplicate", "retry_task", "error"),
                                                   (((got["status"] == 0) & (got["action"] == abi.NDC_APPEND)).sum(),
                                                    ((got["status"] == 0) & (got["action"] == abi.NDC_NEW_BRANCH)).sum(),
                                                    ((got["status"] == 0) & (got["action"] == abi.NDC_DUPLICATE)).sum(),
                                                    (got["status"] == abi.Status.NDC_RETRY_TASK).sum(),
                                                    ((got["status"] != 0) & (got["status"] != abi.Status.NDC_RETRY_TASK)).sum()))},
            "roofline": roofline(alg, k_ms, "crr::ndc_prepare_kernel", config_traffic("config5_ndc_prepare", n, n))}
    if ctx.rank == 0:
        # every task of the timed launches' results (the results buffer of the last one) against the oracle
        t0 = time.perf_counter()
        want, want_items = oracle.ndc_prepare(nb)
        got_items = out.cpu().numpy().view(abi.VH_ITEM)
        nbr = np.nonzero((want["status"] == 0) & (want["action"] == abi.NDC_NEW_BRANCH))[0]
        cnt = want["new_item_count"][nbr].astype(np.int64)
        idx = (np.repeat(nb.tasks["out_begin"][nbr].astype(np.int64), cnt)
               + np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt))
        line["parity_full"] = {"tasks": n, "new_branches": int(nbr.size), "new_branch_items": int(idx.size),
                               "bit_exact": bool(got.tobytes() == want[:n].tobytes()
                                                 and got_items[idx].tobytes() == want_items[idx].tobytes()),
                               "oracle_s": time.perf_counter() - t0}
    return line


def checksum_line(ctx, db, batch, res):
    """crr_checksum (mutable_state_builder.go:334-348 -> checksum.go:45-54, the Load verify path) over the
    replayed rows, HBM-resident: every workflow's thriftrw payload rebuilt from its rows and CRC'd."""
    import ctypes
    torch, eng, args = ctx.torch, ctx.eng, ctx.args
    n = db.n_wf
    out = torch.zeros(max(n, 1), dtype=torch.int32, device=eng.dev)
    s = torch.cuda.current_stream(eng.dev)

    def launch():
        rc = eng.lib.crr_checksum(ctypes.byref(db.c_in), ctypes.byref(db.c_out), ctypes.c_void_p(out.data_ptr()),
                                  ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"crr_checksum failed: {rc}")

    launch()
    torch.cuda.synchronize()
    ctx.barrier()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.config_steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(s)
        launch()
        b.record(s)
    torch.cuda.synchronize()
    ctx.barrier()
    wall = ctx.reduce([time.perf_counter() - t0])[0]
    k_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    got = out.cpu().numpy().view(np.uint32)[:n]
    ok = res.exec["status"] == 0
    ex = res.exec
    rows = (8 * (ex["n_activity"].astype(np.int64) + ex["n_timer"] + ex["n_child"] + ex["n_rc"] + ex["n_signal"])
            + 16 * ex["n_vh_items"].astype(np.int64))[ok].sum()
    alg = int(n * (208 + 168 + 4) + int(rows) + int(np.minimum(batch.wf["start_token_len"], 4096)[ok].sum()))
    tot = ctx.reduce([float(n)], op="sum")[0]
    return {"workload": "Load verify: the mutable-state checksum recomputed from the replayed rows of every workflow",
            "value": tot * args.config_steps / wall, "unit": "workflows verified/s",
            "matches_replay_checksums": bool((got[ok] == ex["checksum"][ok]).all()), "verified": int(ok.sum()),
            "roofline": roofline(alg, k_ms, "crr::checksum_kernel",
                                 config_traffic("config5_checksum_verify", batch.n_wf, batch.n_events))}


# ---- persisted blobs -> rows (rank 0, N = 1) ---------------------------------------------------------------------
def blob_to_rows(ctx, canon, resident_digest, name, chunks=8):
    """The real input path end to end: persisted thriftrw blobs (one per ApplyEvents batch, as
    persistence returns them: serializer.go:109-119) in pinned host memory -> H2D -> device ingest
    (crr_ingest_plan + crr_ingest_layout: decode, intern, order, interleave) -> crr_replay ->
    crr_compact_rows -> D2H of the exec rows + live rows; chunked, uploads ahead of the work, two compute
    streams.  Every host and device stage is inside the clock; the blob encoding itself (what
    persistence stores) is setup.  Beside it `device_resident`: the same with the blobs already in HBM
    (ingest + replay + compaction, no PCIe)."""
    from cadence_amd import abi
    from cadence_amd import dist as cdist
    from cadence_amd.blobs import encode_batch
    from cadence_amd.pipeline import BlobStreamingReplay, split_blobs
    t0 = time.time()
    bs = encode_batch(canon)
    parts = split_blobs(bs, chunks)
    enc_s = time.time() - t0
    sr = BlobStreamingReplay(ctx.eng, parts)
    setup = time.time() - t0
    sr.run()
    runs = [sr.run() for _ in range(3)]
    med = float(np.median([r["wall_s"] for r in runs]))
    digest = np.zeros(cdist.DIGEST_LEN, np.int64)
    with np.errstate(over="ignore"):
        for cr, evc, keys in zip(sr.results(), sr.ev_counts(), sr.device_keys()):
            digest += cdist.digest_numpy(cr.exec, evc, keys)
    r0 = runs[0]
    fig = {"workload": name, "events_per_s": r0["events"] / med, "ms": med * 1e3, "events": r0["events"],
           "workflows": bs.n_wf, "blobs": bs.n_blobs, "blob_bytes": bs.n_bytes,
           "blob_bytes_per_event": bs.n_bytes / max(r0["events"], 1), "chunks": len(parts),
           "h2d_bytes": r0["h2d_bytes"], "h2d_GBs": r0["h2d_bytes"] / med / 1e9, "d2h_bytes": r0["d2h_bytes"],
           "digest": [int(x) for x in digest], "setup_s": {"encode": enc_s, "upload_plan_alloc": setup - enc_s},
           "note": "median of 3 passes; blobs in pinned host buffers as read from persistence; every stage timed"}
    if resident_digest is not None:
        fig["matches_resident_digest"] = fig["digest"] == [int(x) for x in resident_digest]
    # the bound: the uploads alone over PCIe (pinned host -> HBM, the same bytes, no compute)
    peak = sr.h2d_peak()
    fig["roofline"] = {"bound": "pcie", "achieved": fig["h2d_GBs"], "peak": peak, "unit": "GB/s",
                       "frac": fig["h2d_GBs"] / peak if peak else None,
                       "note": "peak = this pipeline's own H2D copies alone, measured in the same run"}
    # the same work with the blobs already resident in HBM: device-side stages only
    torch, eng = ctx.torch, ctx.eng
    torch.cuda.synchronize()
    tt = time.perf_counter()
    reps = 3
    for _ in range(reps):
        for i, p in enumerate(sr.parts):
            s = sr.comp[i % 2]
            S = p["ing"].plan(p["db"], s)
            out = p["out"]
            with torch.cuda.stream(s):
                for k in ["exec", "scratch"] + ["out_" + t[0] for t in abi.TABLES]:
                    out.tensors[k].zero_()
            p["ing"].layout(p["db"], S, s, out=out)
            eng.launch(out, s)
            eng.compact(out, s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - tt) / reps
    fig["device_resident"] = {"events_per_s": r0["events"] / dt, "ms": dt * 1e3,
                              "note": "blobs already in HBM: ingest (plan with its two stream syncs + layout) + replay + "
                                      "compaction per chunk, no transfers"}
    del sr
    torch.cuda.empty_cache()
    return fig


# ---- JSON-encoded persisted batches on the device (rank 0, N = 1) ------------------------------------------------
def json_ingest(ctx, n_wf, reps=3, cpu_wf=20_000):
    """Blobs persisted with the json encoding (serializer.go:321-328: json.Unmarshal into []*types.HistoryEvent),
    the config-3 shape, resident in HBM; timed per pass: crr_ingest_transcode_plan (one host sync) +
    crr_ingest_transcode (JSON -> thriftrw in HBM) + crr_ingest_plan + crr_ingest_layout + crr_replay.  Checked:
    the laid-out inputs and the replayed exec rows equal the thriftrw path's on the same workload.  Beside it
    the host JSON decoder (json_decode.cpp, crr_decode_histories_enc) on a bounded sample, all host cores."""
    from cadence_amd import dist as cdist
    from cadence_amd import synth_native
    from cadence_amd.blobs import KNOWN_DOMAINS, encode_batch
    from cadence_amd.decode import time_native_decode
    from cadence_amd.ingest import DeviceIngest
    torch, eng = ctx.torch, ctx.eng
    canon = synth_native.mixed(n_wf, shard=(cdist.NUM_SHARDS, 1, 0))
    bj, bt = encode_batch(canon, json=True), encode_batch(canon)
    ing_j, ing_t = DeviceIngest(eng), DeviceIngest(eng)
    dj, dt = ing_j.upload(bj), ing_t.upload(bt)
    enc = torch.ones(bj.n_blobs, dtype=torch.int32, device=eng.dev)     # CRR_ENCODING_JSON
    tj = ing_j.transcode(dj, enc)
    out_j = ing_j.layout(tj, ing_j.plan(tj))
    S_t = ing_t.plan(dt)
    out_t = ing_t.layout(dt, S_t)
    eng.launch(out_t)
    torch.cuda.synchronize()
    walls, tc = [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tj = ing_j.transcode(dj, enc)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ing_j.layout(tj, ing_j.plan(tj), out=out_j)
        eng.launch(out_j)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        tc.append(t1 - t0)
    from cadence_amd import abi
    n_slots = int(S_t.n_slots)    # (the buffers' slack past the slots is uninitialised)
    same_in = all(bool(torch.equal(out_j.tensors["ev_" + k][:n_slots * np.dtype(t).itemsize],
                                   out_t.tensors["ev_" + k][:n_slots * np.dtype(t).itemsize]))
                  for k, t in abi.EVENT_COLUMNS)
    same_rows = bool(torch.equal(out_j.tensors["exec"], out_t.tensors["exec"]))
    n_ev = int(canon.n_events)
    wall = float(np.median(walls))
    out = {"workload": f"config 3 shard shape: {n_wf} mixed histories persisted as common/types JSON blobs "
                       "(one per ApplyEvents batch), resident in HBM",
           "events": n_ev, "blobs": bj.n_blobs, "json_bytes": bj.n_bytes, "transcoded_bytes": int(ing_j.last_transcode.n_bytes),
           "events_per_s": n_ev / wall, "ms": wall * 1e3, "transcode_ms": float(np.median(tc)) * 1e3,
           "json_GBs": bj.n_bytes / float(np.median(tc)) / 1e9,
           "inputs_equal_thrift_path": same_in, "rows_equal_thrift_path": same_rows,
           "note": "median of passes; transcode (a lane-per-blob JSON walk staging the thriftrw form, the gather) "
                   "+ the thriftrw ingest + the replay"}
    # the transcode against HBM: the JSON read once, the thriftrw form written to the stage, read and written
    # by the gather (algorithmic bytes; the plan's host sync inside the timed span)
    out["roofline"] = roofline(bj.n_bytes + 3 * out["transcoded_bytes"], out["transcode_ms"],
                               "crr_json::blobs_kernel<M_PLAN> + gather_kernel (transcode span)")
    del dj, dt, tj, out_j, out_t, bj, bt
    torch.cuda.empty_cache()
    if not ctx.args.no_cpu_baseline:
        sj = encode_batch(synth_native.mixed(cpu_wf, shard=(cdist.NUM_SHARDS, 1, 0)), json=True).to_sources()
        for s_ in sj:
            s_.encodings = ["json"] * len(s_.blobs)
        cores = host_cpus()
        r = time_native_decode(sj, known_domains=KNOWN_DOMAINS, n_threads=cores, min_seconds=2.0)
        out["cpu_json_decode"] = {"events_per_s": r["events_per_s"], "MB_per_s": r["MB_per_s"], "cores": cores,
                                  "sample": f"{cpu_wf} workflows of the same shape, decode only (no replay)"}
        out["vs_cpu_json_decode"] = out["events_per_s"] / r["events_per_s"]
    return out


# ---- rank 0, N = 1: end to end, host ingest, CPU baseline ---------------------------------------------------
def end_to_end(ctx, n_wf, k, chunks=8):
    """Config 2 from host buffers: pinned staging, `chunks` chunks overlapped on three streams, the event
    columns in the narrow upload format widened on the device (wire.py; the 49-B/event columns
    alongside as ``columns_wide``), live rows compacted on the device; checked against the
    HBM-resident digest of the same workflows."""
    from cadence_amd import dist as cdist
    from cadence_amd import synth
    from cadence_amd.flatten import interleave
    from cadence_amd.pipeline import StreamingReplay
    bounds = np.linspace(0, n_wf, chunks + 1).astype(np.int64)
    parts = [interleave(synth.activity_chain(int(b - a), k, synth.SEED_C2, with_keys=False, wf_ids=np.arange(a, b)))
             for a, b in zip(bounds[:-1], bounds[1:])]
    out = None
    for wire in (True, False):
        t0 = time.time()
        sr = StreamingReplay(ctx.eng, parts, wire=wire)
        setup = time.time() - t0
        sr.run()                                     # warm
        runs = [sr.run() for _ in range(3)]
        med = float(np.median([r["wall_s"] for r in runs]))
        r0 = runs[0]
        digest = np.zeros(cdist.DIGEST_LEN, np.int64)
        with np.errstate(over="ignore"):
            for (a, b), cr, c in zip(zip(bounds[:-1], bounds[1:]), sr.results(), sr.chunks):
                digest += cdist.digest_numpy(cr.exec, c.batch.wf["ev_count"], cdist.device_keys(c.batch, np.arange(a, b)))
        fig = {"events_per_s": r0["events"] / med, "ms": med * 1e3, "events": r0["events"], "chunks": chunks,
               "h2d_bytes": r0["h2d_bytes"], "d2h_bytes": r0["d2h_bytes"], "h2d_bytes_per_event": r0["h2d_bytes"] / r0["events"],
               "h2d_GBs": r0["h2d_bytes"] / med / 1e9, "setup_s": setup, "digest": [int(x) for x in digest]}
        if wire:
            fig["pack_s"] = sr.pack_s
            from cadence_amd.wire import COLUMNS
            fig["widths"] = {c: int(getattr(sr.chunks[0].db.c_packed, c).width) for c in COLUMNS}
            out = fig
            out["note"] = ("host columns in pinned staging buffers (where the decoder writes them), event columns in the "
                           "narrow upload format (per-workflow deltas at the batch's narrowest byte width; host packing "
                           "time pack_s is not in the figure); per chunk: H2D, output zero-fill, crr_widen_events, replay, "
                           "crr_compact_rows, D2H of the exec rows + the live rows only; three streams overlap chunks; "
                           "median of 3 passes")
        else:
            out["columns_wide"] = fig
        del sr
        ctx.torch.cuda.empty_cache()
    return out


def host_ingest(ctx, flatten_s, flatten_events):
    """Host-side rates that feed the engine: the native thriftrw decoder (crr_decode_histories, all host
    CPUs) over encoded mixed histories, and the numpy interleave of the config-2 batch."""
    from cadence_amd import synth_mixed
    from cadence_amd.decode import WorkflowSource, time_native_decode
    from cadence_amd.thrift_codec import serialize_history
    hs = synth_mixed.mixed_histories(3000, 0xCAD00005, mean_len=40)
    src = [WorkflowSource(blobs=serialize_history(h), run_id=h.run_id, branch_id=h.branch_id, now_ns=h.now_ns,
                          domain_failover_version=h.domain_failover_version) for h in hs]
    dec = time_native_decode(src, {"domain-a", "domain-b", "parent-domain"}, n_threads=host_cpus(), min_seconds=1.0)
    dec["threads"] = host_cpus()
    return {"decode": dec, "interleave_config2": {"events_per_s": flatten_events / flatten_s, "seconds": flatten_s}}


def cpu_blob_path(ctx, threads, k):
    """The CPU doing what blob_to_rows does: persisted thriftrw blobs -> the native host decoder
    (crr_decode_histories, `threads` workers) -> the oracle's replay (`threads` workers), on a sample of
    config-2 workflows; both stages timed, the rate of the two in sequence reported."""
    from oracle import oracle
    from cadence_amd import synth
    from cadence_amd.blobs import KNOWN_DOMAINS, encode_batch
    from cadence_amd.decode import decode_histories, time_native_decode
    n = min(ctx.args.cpu_sample, 50_000)
    canon = synth.activity_chain(n, k, synth.SEED_C2, with_keys=True, wf_ids=np.arange(n))
    src = encode_batch(canon).to_sources()
    dec = time_native_decode(src, KNOWN_DOMAINS, n_threads=threads, min_seconds=ctx.args.cpu_seconds / 2)
    batch = decode_histories(src, known_domains=KNOWN_DOMAINS, n_threads=threads)
    passes, dt = 0, 0.0
    while passes == 0 or dt < ctx.args.cpu_seconds / 2:
        t0 = time.perf_counter()
        oracle.replay(batch, threads)
        dt += time.perf_counter() - t0
        passes += 1
    rep = batch.n_events * passes / dt
    both = 1.0 / (1.0 / dec["events_per_s"] + 1.0 / rep)
    return {"value": both, "unit": "events/s", "cores": threads, "kind": "port",
            "decode_events_per_s": dec["events_per_s"], "replay_events_per_s": rep,
            "sample": f"{n} config-2 workflows ({batch.n_events} events) as thriftrw blobs: native decoder "
                      f"({dec['reps']} passes) then the oracle's replay ({passes} passes), {threads} threads each"}


def cpu_baseline(ctx, gpu_res, gpu_batch, k):
    """The oracle (C++ restatement of the Go stateBuilder, per-workflow hash maps, std::thread workers)
    on this process's host CPUs: a bounded sample of config 2 (bit-compared with the GPU rows) and
    BASELINE config 1 (10k activity chains of 23 events)."""
    from oracle import oracle
    from cadence_amd import synth
    from cadence_amd.result import diff_results
    args = ctx.args
    threads = args.cpu_threads or host_cpus()

    def timed(batch):
        passes, dt, res = 0, 0.0, None
        while passes == 0 or dt < args.cpu_seconds:
            t0 = time.perf_counter()
            r = oracle.replay(batch, threads)
            dt += time.perf_counter() - t0
            res = res if res is not None else r
            passes += 1
        return passes, dt, res

    n = min(args.cpu_sample, args.workflows)
    sample = synth.activity_chain(n, k, synth.SEED_C2, with_keys=True, wf_ids=np.arange(n))
    passes, dt, res = timed(sample)
    out = {"value": sample.n_events * passes / dt, "unit": "events/s", "cores": threads, "kind": "port",
           "host_cpus_visible": os.cpu_count(),
           "sample": f"{passes} pass(es) over {n} config-2 workflows ({sample.n_events} events), {threads} std::thread "
                     "workers (this process's CPU share), CPU restatement of the Go stateBuilder (reference not runnable)",
           "wall_s": dt, "cpu_seconds_approx": dt * threads}
    if n == gpu_batch.n_wf:
        out["gpu_parity_bit_exact"] = not diff_results(gpu_batch, gpu_res, sample, res)
    out["blob_path"] = cpu_blob_path(ctx, threads, k)
    c1 = synth.activity_chain(10_000, 3, synth.SEED_C1, with_keys=True)
    p1, d1, _ = timed(c1)
    out["config1"] = {"events_per_s": c1.n_events * p1 / d1, "workflows_per_s": c1.n_wf * p1 / d1,
                      "workload": "BASELINE config 1: 10k activity-chain histories x 23 events", "passes": p1,
                      "cores": threads}
    return out


def summary(line):
    """The essentials of every line in one short object: value, roofline fraction, traffic / algorithmic
    bytes, and each parity / digest verdict."""
    def rf(x):
        r = x.get("roofline") or {}
        t, a = r.get("traffic"), r.get("algorithmic_bytes_per_launch")
        return {"frac": r.get("frac"), "kernel_ms": r.get("kernel_ms"), "traffic_x": (t / a) if (t and a) else None}

    out = {"config2": {"value": line["value"], **rf(line), "all_ok": line.get("all_ok"),
                       "parity_1M": (line.get("cpu_baseline") or {}).get("gpu_parity_bit_exact")}}
    c = line.get("configs") or {}
    for k in ("config3_mixed", "config4_long_tail"):
        if k in c:
            x = c[k]
            out[k] = {"value": x["value"], **rf(x), "digest_ok": x["digest"]["matches_host_digest"],
                      "parity_full": (x.get("parity_full") or {}).get("bit_exact"),
                      "parity_full_workflows": (x.get("parity_full") or {}).get("workflows")}
    if "passive_replication" in c:
        x = c["passive_replication"]
        vo = x.get("vs_oracle") or {}
        out["passive_replication"] = {"value": x["value"], **rf(x), "mismatches_vs_one_shot": x["vs_one_shot"].get("mismatches"),
                                      "mismatches_vs_oracle": vo.get("mismatches"),
                                      "prefix_mismatches": (vo.get("prefix") or {}).get("mismatches")}
        bp = x.get("blob_path")
        if bp:
            out["passive_replication"]["blob_path"] = {
                "device_resident_events_per_s": bp["device_resident"]["events_per_s"],
                "device_resident_ms": bp["device_resident"]["ms_per_step"],
                "pcie_inclusive_events_per_s": bp["pcie_inclusive"]["events_per_s"],
                "rows_equal_host_path": bp["device_resident"]["rows_equal_host_path"] and bp["pcie_inclusive"]["rows_equal_host_path"]}
    if "config5_ndc" in c:
        x = c["config5_ndc"]
        rb = x["rebuild"]
        out["config5_rebuild"] = {"value": rb["value"], **rf(rb), "digest_ok": rb["digest"]["matches_host_digest"],
                                  "parity_full": (rb.get("parity_full") or {}).get("bit_exact"),
                                  "parity_full_workflows": (rb.get("parity_full") or {}).get("workflows")}
        nd = x["ndc_prepare"]
        out["ndc_prepare"] = {"value": nd["value"], **rf(nd), "parity_full": (nd.get("parity_full") or {}).get("bit_exact"),
                              "parity_tasks": (nd.get("parity_full") or {}).get("tasks")}
        cv = x["checksum_verify"]
        out["checksum_verify"] = {"value": cv["value"], **rf(cv), "matches": cv["matches_replay_checksums"]}
    if "json_ingest" in line:
        x = line["json_ingest"]
        out["json_ingest"] = {"events_per_s": x["events_per_s"], "json_GBs": x["json_GBs"], "frac": x["roofline"]["frac"],
                              "rows_equal_thrift_path": x["rows_equal_thrift_path"] and x["inputs_equal_thrift_path"],
                              "vs_cpu_json_decode": x.get("vs_cpu_json_decode")}
    for k, fig in (line.get("blob_to_rows") or {}).items():
        out["blob_to_rows_" + k] = {"events_per_s": fig["events_per_s"],
                                    "device_resident": fig["device_resident"]["events_per_s"],
                                    "pcie_frac": fig["roofline"]["frac"]}
    if "cpu_baseline" in line:
        out["cpu_baseline"] = {"value": line["cpu_baseline"]["value"], "cores": line["cpu_baseline"]["cores"]}
    return out


def main():
    args = parse()
    ctx = Ctx(args)
    torch = ctx.torch
    from cadence_amd import synth_native
    from cadence_amd import dist as cdist
    line, batch2, res2, db2 = config2(ctx)
    progress("config 2 done")
    if ctx.rank == 0 and ctx.world == 1 and not args.headline_only:
        from cadence_amd.flatten import interleave
        from cadence_amd import synth
        canon = synth.activity_chain(200_000, args.activities, synth.SEED_C2, with_keys=False)
        flat_t0 = time.perf_counter()
        interleave(canon)
        flat_s, flat_ev = time.perf_counter() - flat_t0, canon.n_events
        del canon
    del db2
    torch.cuda.empty_cache()
    if not args.headline_only:
        shard = (cdist.NUM_SHARDS, ctx.world, ctx.rank)
        n3 = args.c3_workflows * ctx.world
        c3, b3, r3, db3 = run_config(
            ctx, "config3", lambda: synth_native.mixed(n3, shard=shard),
            f"config 3: {args.c3_workflows} mixed histories per GPU (timers, signals, child workflows, cancel requests; "
            f"10..70 events), the rank's history shards of one {n3}-workflow workload",
            lambda: synth_native.mixed(50_000, shard=shard),
            global_ids=cdist.rank_workflows(n3, ctx.rank, ctx.world))
        del db3
        torch.cuda.empty_cache()
        progress("config 3 done")
        pr = passive_replication(ctx, b3, r3, make_canon=lambda: synth_native.mixed(n3, shard=shard))
        progress("passive replication done")
        del b3, r3
        torch.cuda.empty_cache()
        n4 = args.c4_workflows * ctx.world
        c4, b4, r4, db4 = run_config(
            ctx, "config4", lambda: synth_native.long_tail(n4, shard=shard),
            f"config 4: {args.c4_workflows} long-tail workflows per GPU (Zipf lengths up to 50k events, continued as new "
            "every 10k: each run a workflow, a CAN's new-run history its next run's first batch), lane per workflow up "
            "to 256 events, a wavefront per longer run",
            lambda: synth_native.long_tail(60, shard=shard))
        del db4, b4, r4
        torch.cuda.empty_cache()
        progress("config 4 done")
        c5 = config5(ctx, args.c5_workflows, shard,
                     global_ids=cdist.rank_workflows(args.c5_workflows * ctx.world, ctx.rank, ctx.world))
        torch.cuda.empty_cache()
        progress("config 5 done")
        line["configs"] = {"config3_mixed": c3, "config4_long_tail": c4, "passive_replication": pr,
                           "config5_ndc": c5}
    if ctx.rank == 0 and ctx.world == 1 and not args.headline_only and not args.no_e2e:
        line["pcie_inclusive"] = end_to_end(ctx, args.workflows, args.activities)
        progress("end to end (columns) done")
        e2e = line["pcie_inclusive"]
        e2e["matches_resident_digest"] = e2e["digest"] == line["digest"] and e2e["columns_wide"]["digest"] == line["digest"]
        line["host_ingest"] = host_ingest(ctx, flat_s, flat_ev)
        from cadence_amd import synth
        c2_canon = synth.activity_chain(args.workflows, args.activities, synth.SEED_C2, with_keys=True,
                                        wf_ids=np.arange(args.workflows))
        line["blob_to_rows"] = {"config2": blob_to_rows(
            ctx, c2_canon, line["digest"],
            f"config 2 persisted: {args.workflows} activity-chain workflows, one thriftrw blob per ApplyEvents batch")}
        del c2_canon
        progress("blob -> rows config 2 done")
        c3_canon = synth_native.mixed(args.c3_workflows, shard=(cdist.NUM_SHARDS, 1, 0))
        line["blob_to_rows"]["config3_shard"] = blob_to_rows(
            ctx, c3_canon, None, f"config 3 shard persisted: {args.c3_workflows} mixed histories, one thriftrw blob per batch")
        del c3_canon
        progress("blob -> rows config 3 done")
        line["json_ingest"] = json_ingest(ctx, args.json_workflows)
        progress("JSON ingest done")
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(ctx, res2, batch2, args.activities)
        if "pcie_inclusive" in line:
            line["pcie_inclusive"]["vs_cpu_baseline"] = line["pcie_inclusive"]["events_per_s"] / line["cpu_baseline"]["value"]
        for k, fig in line.get("blob_to_rows", {}).items():
            fig["vs_cpu_baseline"] = fig["events_per_s"] / line["cpu_baseline"]["value"]
            fig["vs_cpu_blob_path"] = fig["events_per_s"] / line["cpu_baseline"]["blob_path"]["value"]
            fig["device_resident"]["vs_cpu_baseline"] = (fig["device_resident"]["events_per_s"]
                                                         / line["cpu_baseline"]["value"])
    if ctx.rank == 0:
        line["summary"] = summary(line)   # last key: the figures of every line stay in a truncated stdout tail
        print(json.dumps(line), flush=True)
    if ctx.world > 1:
        ctx.dist.destroy_process_group()


if __name__ == "__main__":
    main()
