"""Multi-GPU: shard-partitioned replay with one collective.

Workflows map to Cadence history shards (``common/util.go:313-316``: farm.Fingerprint32(workflowID)
% numHistoryShards; synthetic data assigns shard IDs directly) and shards map to GPUs
(``shard mod world``).  Replay has no cross-workflow dependency, so there is no data-path exchange:
each rank replays its shard set and the job's only collective is one all-reduce of an int64
digest (counts + checksum folds bound to each workflow's identity) -- RCCL over xGMI on the GPU path,
gloo in the CPU tests.
"""
from __future__ import annotations

import numpy as np

from . import abi

# word offsets of the digest's fields inside crr_exec_row (int32 words; next_event_id as an int64 word)
EXEC_ROW_WORDS = abi.EXEC_ROW.itemsize // 4
W_STATUS = abi.EXEC_ROW.fields["status"][1] // 4
W_INCONS = abi.EXEC_ROW.fields["inconsistencies"][1] // 4
W_CHECKSUM = abi.EXEC_ROW.fields["checksum"][1] // 4
W_FAIL_STEP = abi.EXEC_ROW.fields["fail_step"][1] // 4


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
DIGEST_FIELDS = ("events_ok", "workflows_ok", "workflows_failed", "crc_sum", "identity_fold", "inconsistencies",
                 "failed_fold")
DIGEST_LEN = len(DIGEST_FIELDS)


def workflow_keys(global_ids: np.ndarray) -> np.ndarray:
    """Per workflow: mix64(global workflow ID) as int64 -- the identity the digest binds each result to
    (a fold of (workflow identity, crc), so a permutation of results across workflows
    changes it, where a plain sum of checksums would not)."""
    return mix64(np.asarray(global_ids, np.uint64)).view(np.int64)


def device_keys(batch, global_ids=None) -> np.ndarray:
    """Identity keys in a batch's device order: the global workflow ID of each device position
    (``global_ids`` in canonical order; default the canonical index) through ``batch.perm``."""
    ids = np.arange(batch.n_wf, dtype=np.int64) if global_ids is None else np.asarray(global_ids, np.int64)
    if getattr(batch, "perm", None) is not None:
        ids = ids[np.asarray(batch.perm, np.int64)]
    return workflow_keys(ids)


def digest_torch(torch, exec_bytes, n_wf: int, wf_bytes, keys):
    """Device-side digest of a replayed shard from the raw exec-row and descriptor buffers and the
    workflows' identity keys (``workflow_keys`` of each device position's global workflow ID), int64[7]:
      0 events applied by OK workflows (each one's ev_count: the events of this call, so a resumed --
        passive-replication -- or continue-as-new run counts what it replayed, not its NextEventID)
      1 workflows ok, 2 workflows failed
      3 sum(crc of ok)
      4 sum over ok of key ^ crc (mod 2^64): binds every checksum to its workflow
      5 inconsistencies
      6 sum over failed of key ^ (status << 32 | fail_step) (mod 2^64): binds every failure too
    Sums wrap mod 2^64 (int64 two's complement), which the all-reduce preserves."""
    raw = exec_bytes[: n_wf * EXEC_ROW_WORDS * 4]
    rows = raw.view(torch.int32).view(n_wf, EXEC_ROW_WORDS)
    ev = wf_bytes[: n_wf * WF_WORDS * 4].view(torch.int32).view(n_wf, WF_WORDS)[:, W_EV_COUNT].to(torch.int64)
    okb = rows[:, W_STATUS] == 0
    ok = okb.to(torch.int64)
    crc = rows[:, W_CHECKSUM].to(torch.int64) & 0xFFFFFFFF
    k = keys[:n_wf]
    fail_word = ((rows[:, W_STATUS].to(torch.int64) & 0xFFFFFFFF) << 32) | (rows[:, W_FAIL_STEP].to(torch.int64) & 0xFFFFFFFF)
    zero = torch.zeros_like(k)
    return torch.stack([
        (ev * ok).sum(),
        ok.sum(),
        n_wf - ok.sum(),
        (crc * ok).sum(),
        torch.where(okb, k ^ crc, zero).sum(),
        rows[:, W_INCONS].to(torch.int64).sum(),
        torch.where(okb, zero, k ^ fail_word).sum(),
    ])


def digest_numpy(exec_rows: np.ndarray, ev_count: np.ndarray, keys: np.ndarray) -> np.ndarray:
    """Same digest from host exec rows (abi.EXEC_ROW), the descriptors' ev_count and the identity keys
    (same order)."""
    okb = exec_rows["status"] == 0
    ok = okb.astype(np.int64)
    crc = exec_rows["checksum"].astype(np.int64)
    ev = np.asarray(ev_count, np.int64)
    k = np.asarray(keys, np.int64)
    fail_word = ((exec_rows["status"].astype(np.int64) & 0xFFFFFFFF) << 32) | (exec_rows["fail_step"].astype(np.int64) & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        return np.array([(ev * ok).sum(), ok.sum(), len(exec_rows) - ok.sum(), (crc * ok).sum(),
                         np.where(okb, k ^ crc, 0).sum(dtype=np.int64),
                         exec_rows["inconsistencies"].astype(np.int64).sum(),
                         np.where(okb, 0, k ^ fail_word).sum(dtype=np.int64)], dtype=np.int64)


def all_reduce_digest(torch, dist, digest):
    """The job's one collective: RCCL all-reduce of the device tensor; under gloo (CPU tests, or several
    ranks sharing one GPU) the all-reduce runs on a host copy."""
    if dist.get_backend() == "gloo" and digest.is_cuda:
        h = digest.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM)
        digest.copy_(h)
    else:
        dist.all_reduce(digest, op=dist.ReduceOp.SUM)
    return digest
