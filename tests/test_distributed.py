"""World-size-2 gloo run of the multi-GPU path (shard partition + one digest all-reduce) on CPU."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cadence_amd import abi, synth
from cadence_amd import dist as cdist


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    # 64 shards, 8 workflows per shard; each rank replays the workflows of its shards (CPU oracle as
    # the stand-in for the device replay -- this test covers the partition + collective only)
    n_shards, per = 64, 8
    batch = synth.activity_chain(n_shards * per, 2, synth.SEED_C3)
    shard_of = np.repeat(np.arange(n_shards), per)
    mine = cdist.workflow_mask(shard_of, rank, world)
    res = oracle.replay(batch, 1)
    # the digest code the GPU ranks run (dist.digest_torch over the raw exec-row bytes), here on CPU tensors
    raw = torch.from_numpy(np.ascontiguousarray(res.exec[mine]).view(np.uint8).reshape(-1).copy())
    wfb = torch.from_numpy(np.ascontiguousarray(batch.wf[mine]).view(np.uint8).reshape(-1).copy())
    keys = cdist.workflow_keys(np.arange(batch.n_wf))            # global workflow IDs -> identity keys
    t = cdist.digest_torch(torch, raw, int(mine.sum()), wfb, torch.from_numpy(keys[mine].copy()))
    assert (t.numpy() == cdist.digest_numpy(res.exec[mine], batch.wf["ev_count"][mine], keys[mine])).all()
    # a rank that swapped two of its workflows' results (a permutation bug) must not reduce to the whole
    ok = np.nonzero(mine & (res.exec["status"] == 0))[0]
    sw = res.exec.copy()
    sw[[ok[0], ok[1]]] = sw[[ok[1], ok[0]]]
    t_sw = cdist.digest_torch(torch, torch.from_numpy(np.ascontiguousarray(sw[mine]).view(np.uint8).reshape(-1).copy()),
                              int(mine.sum()), wfb, torch.from_numpy(keys[mine].copy()))
    cdist.all_reduce_digest(torch, dist, t)
    cdist.all_reduce_digest(torch, dist, t_sw)
    q.put((rank, t.numpy().tolist(), cdist.digest_numpy(res.exec, batch.wf["ev_count"], keys).tolist(),
           t_sw.numpy().tolist()))
    dist.destroy_process_group()


def test_two_rank_shard_partition_and_digest_reduce():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    reduced = [o[1] for o in out]
    assert reduced[0] == reduced[1]
    assert reduced[0] == out[0][2]       # sum over disjoint shards == digest of the whole batch
    assert reduced[0][1] == 64 * 8        # every workflow replayed exactly once
    swapped = out[0][3]
    assert swapped[:4] == reduced[0][:4] and swapped[4] != reduced[0][4]   # identity-binding fold


def test_rank_workflows_partition_one_workload():
    """bench.py's N-rank split of one global workload: disjoint, complete, shard-consistent, and each
    rank's generated part equals the same workflows of the whole (per-workflow seeded draws)."""
    from cadence_amd import synth_native
    n, world = 4000, 4
    parts = [cdist.rank_workflows(n, r, world) for r in range(world)]
    allw = np.sort(np.concatenate(parts))
    assert (allw == np.arange(n)).all()
    sh = cdist.synthetic_shard_ids(np.arange(n))
    for r, p in enumerate(parts):
        assert (sh[p] % world == r).all()
    assert (synth_native.shard_of(np.arange(500), cdist.NUM_SHARDS) == sh[:500]).all()
    whole = synth.activity_chain(n, 2, synth.SEED_C2, wf_ids=np.arange(n), with_keys=False)
    part = synth.activity_chain(parts[1].size, 2, synth.SEED_C2, wf_ids=parts[1], with_keys=False)
    L = 17
    for c in ("event_id", "timestamp", "task_id", "ref", "key", "etype", "version"):
        assert (whole.cols[c].reshape(n, L)[parts[1]] == part.cols[c].reshape(-1, L)).all(), c
    # native generator: the rank's shards of the mixed workload, event for event
    tot = synth_native.mixed(2000)
    ps = [synth_native.mixed(2000, shard=(cdist.NUM_SHARDS, 2, r)) for r in range(2)]
    assert sum(p.n_wf for p in ps) == tot.n_wf and sum(p.n_events for p in ps) == tot.n_events


def test_shards_for_rank_partition():
    parts = [set(cdist.shards_for_rank(100, r, 8).tolist()) for r in range(8)]
    assert set().union(*parts) == set(range(100))
    assert sum(len(p) for p in parts) == 100
