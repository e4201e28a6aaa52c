"""Multi-GPU: shard-partitioned replay with one collective.

Workflows map to Cadence history shards (``common/util.go:313-316``: farm.Fingerprint32(workflowID)
% numHistoryShards; synthetic data assigns shard IDs directly) and shards map to GPUs
(``shard mod world``).  Replay has no cross-workflow dependency, so there is no data-path exchange:
each rank replays its shard set and the job's only collective is one all-reduce of an int64
digest (counts + order-independent checksum fold) -- RCCL over xGMI on the GPU path, gloo in the
CPU tests.
"""
from __future__ import annotations

import numpy as np

from . import abi

# word offsets of the digest's fields inside crr_exec_row (int32 words; next_event_id as an int64 word)
EXEC_ROW_WORDS = abi.EXEC_ROW.itemsize // 4
W_STATUS = abi.EXEC_ROW.fields["status"][1] // 4
W_INCONS = abi.EXEC_ROW.fields["inconsistencies"][1] // 4
W_CHECKSUM = abi.EXEC_ROW.fields["checksum"][1] // 4
DIGEST_LEN = 6
GOLDEN = 0x9E3779B1


NUM_SHARDS = 16384   # numHistoryShards of the synthetic workloads


def mix64(x: np.ndarray) -> np.ndarray:
    """SplitMix64 finalizer over uint64 arrays (wrapping arithmetic)."""
    x = np.asarray(x, np.uint64)
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def synthetic_shard_ids(w: np.ndarray, num_shards: int = NUM_SHARDS) -> np.ndarray:
    """History shard of synthetic workflow index w -- the stand-in for WorkflowIDToHistoryShard
    (common/util.go:313-316, farm.Fingerprint32(workflowID) % numberOfShards); the same function as
    the native generator's crr_synth_shard_of."""
    with np.errstate(over="ignore"):
        h = mix64(np.asarray(w, np.uint64) + np.uint64(0x9E3779B97F4A7C15))
    return (h % np.uint64(num_shards)).astype(np.int64)


def rank_workflows(n_global: int, rank: int, world: int, num_shards: int = NUM_SHARDS) -> np.ndarray:
    """Global indices of the workflows of a n_global-workflow workload that ``rank`` replays."""
    w = np.arange(n_global, dtype=np.int64)
    if world <= 1:
        return w
    return w[workflow_mask(synthetic_shard_ids(w, num_shards), rank, world)]


def shards_for_rank(num_shards: int, rank: int, world: int) -> np.ndarray:
    """History shards owned by ``rank``: {s : s mod world == rank}."""
    return np.arange(rank, num_shards, world, dtype=np.int64)


def workflow_mask(shard_ids: np.ndarray, rank: int, world: int) -> np.ndarray:
    return (shard_ids % world) == rank


WF_WORDS = abi.WORKFLOW.itemsize // 4
W_EV_COUNT = abi.WORKFLOW.fields["ev_count"][1] // 4


def digest_torch(torch, exec_bytes, n_wf: int, wf_bytes):
    """Device-side digest of a replayed shard from the raw exec-row and descriptor buffers (int64[6]):
    [events applied by OK workflows (each one's ev_count: the events of this call, so a resumed --
    passive-replication -- or continue-as-new run counts what it replayed, not its NextEventID), workflows
    ok, workflows failed, sum(crc of ok), sum(crc*phi mod 2^32), inconsistencies]."""
    raw = exec_bytes[: n_wf * EXEC_ROW_WORDS * 4]
    rows = raw.view(torch.int32).view(n_wf, EXEC_ROW_WORDS)
    ev = wf_bytes[: n_wf * WF_WORDS * 4].view(torch.int32).view(n_wf, WF_WORDS)[:, W_EV_COUNT].to(torch.int64)
    ok = (rows[:, W_STATUS] == 0).to(torch.int64)
    crc = rows[:, W_CHECKSUM].to(torch.int64) & 0xFFFFFFFF
    return torch.stack([
        (ev * ok).sum(),
        ok.sum(),
        n_wf - ok.sum(),
        (crc * ok).sum(),
        ((crc * GOLDEN) & 0xFFFFFFFF).sum(),
        rows[:, W_INCONS].to(torch.int64).sum(),
    ])


def digest_numpy(exec_rows: np.ndarray, ev_count: np.ndarray) -> np.ndarray:
    """Same digest from host exec rows (abi.EXEC_ROW) and the descriptors' ev_count (same order)."""
    ok = (exec_rows["status"] == 0).astype(np.int64)
    crc = exec_rows["checksum"].astype(np.int64)
    ev = np.asarray(ev_count, np.int64)
    return np.array([(ev * ok).sum(), ok.sum(), len(exec_rows) - ok.sum(), (crc * ok).sum(),
                     ((crc * GOLDEN) & 0xFFFFFFFF).sum(), exec_rows["inconsistencies"].astype(np.int64).sum()],
                    dtype=np.int64)


def all_reduce_digest(torch, dist, digest):
    """The job's one collective (RCCL all-reduce on GPU tensors, gloo on CPU)."""
    dist.all_reduce(digest, op=dist.ReduceOp.SUM)
    return digest
