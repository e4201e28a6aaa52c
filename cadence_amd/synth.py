"""Seeded synthetic histories, generated straight into flattened columns.

Shapes follow the reference's own history builders: the activity chain of
``service/history/testing/events_util.go`` and the event-graph rules of
``common/testing/history_event_util.go`` (decision scheduled -> started -> completed, activities
scheduled by a decision completion, closes follow starts).  No network, no datasets: synthetic.
"""
from __future__ import annotations

import numpy as np

from . import abi
from .abi import EventType as ET
from .flatten import TASKS_PER_EVENT, HistoryBatch, assign_canonical_tables

SEED_C1 = 0xCAD00001
SEED_C2 = 0xCAD00002
SEED_C3 = 0xCAD00003
BASE_TS = 1_600_000_000_000_000_000

_HEX = np.frombuffer(b"0123456789abcdef", np.uint8)


def uuid_ascii(rng: np.random.Generator, n: int) -> np.ndarray:
    """n random UUIDv4 strings as an (n, 36) uint8 ASCII array (stand-in for uuid.New())."""
    return uuid_ascii_raw(rng.integers(0, 256, size=(n, 16), dtype=np.uint8))


def uuid_ascii_raw(raw: np.ndarray) -> np.ndarray:
    """UUIDv4 strings from (n, 16) random bytes (version / variant bits set here)."""
    raw = raw.copy()
    n = raw.shape[0]
    raw[:, 6] = (raw[:, 6] & 0x0F) | 0x40
    raw[:, 8] = (raw[:, 8] & 0x3F) | 0x80
    hexd = np.empty((n, 32), np.uint8)
    hexd[:, 0::2] = _HEX[raw >> 4]
    hexd[:, 1::2] = _HEX[raw & 0x0F]
    out = np.full((n, 36), ord("-"), np.uint8)
    for dst, src, ln in ((0, 0, 8), (9, 8, 4), (14, 12, 4), (19, 16, 4), (24, 20, 12)):
        out[:, dst:dst + ln] = hexd[:, src:src + ln]
    return out


def branch_tokens(tree_ids: np.ndarray, branch_ids: np.ndarray) -> np.ndarray:
    """NewHistoryBranchTokenByBranchID for 36-char IDs, vectorised: (n, 96) uint8."""
    n = tree_ids.shape[0]
    tok = np.zeros((n, 96), np.uint8)
    tok[:, 0] = 0x59
    tok[:, 1:4] = [0x0B, 0x00, 0x0A]
    tok[:, 4:8] = [0, 0, 0, 36]
    tok[:, 8:44] = tree_ids
    tok[:, 44:47] = [0x0B, 0x00, 0x14]
    tok[:, 47:51] = [0, 0, 0, 36]
    tok[:, 51:87] = branch_ids
    tok[:, 87:91] = [0x0F, 0x00, 0x1E, 0x0C]
    tok[:, 91:95] = 0
    tok[:, 95] = 0
    return tok


def activity_chain_template(k: int):
    """Event types + batch flags of the activity-chain workflow with k activities (5 + 6k events).

    [Started, DTSched] [DTStarted] k x ([DTCompleted, ATSched] [ATStarted] [ATCompleted, DTSched]
    [DTStarted]) [DTCompleted, WFCompleted]
    """
    batches = [[ET.WorkflowExecutionStarted, ET.DecisionTaskScheduled], [ET.DecisionTaskStarted]]
    for _ in range(k):
        batches += [[ET.DecisionTaskCompleted, ET.ActivityTaskScheduled], [ET.ActivityTaskStarted],
                    [ET.ActivityTaskCompleted, ET.DecisionTaskScheduled], [ET.DecisionTaskStarted]]
    batches += [[ET.DecisionTaskCompleted, ET.WorkflowExecutionCompleted]]
    types, flags = [], []
    for b in batches:
        for j, t in enumerate(b):
            types.append(int(t))
            flags.append((abi.BATCH_FIRST if j == 0 else 0) | (abi.BATCH_LAST if j == len(b) - 1 else 0))
    return np.array(types, np.uint8), np.array(flags, np.uint8)


class _CounterDraws:
    """Per-workflow random draws: value j of stream s for workflow w is a hash of (seed, w, s, j), so a
    workflow is the same whichever subset of a workload is generated (shard partitions)."""

    def __init__(self, seed: int, wf_ids: np.ndarray):
        from .dist import mix64
        self.mix = mix64
        self.seed = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
        self.ids = np.asarray(wf_ids, np.uint64)
        self.stream = 0

    def _u64(self, m: int) -> np.ndarray:
        self.stream += 1
        with np.errstate(over="ignore"):
            x = (self.ids[:, None] * np.uint64(0x9E3779B97F4A7C15) + self.seed
                 + np.uint64(self.stream) * np.uint64(0xD1B54A32D192ED03)
                 + np.arange(m, dtype=np.uint64)[None, :] * np.uint64(0xA0761D6478BD642F))
        return self.mix(self.mix(x))

    def integers(self, lo: int, hi: int, size, dtype=np.int64):
        """size = (n_wf, m) or n_wf * m (workflow-major)."""
        n = self.ids.size
        m = (size[1] if isinstance(size, tuple) else int(size) // max(n, 1))
        v = (self._u64(m) % np.uint64(hi - lo)).astype(np.int64) + lo
        return (v if isinstance(size, tuple) else v.reshape(-1)).astype(dtype)

    def random(self, size) -> np.ndarray:
        n = self.ids.size
        m = int(size) // max(n, 1)
        return ((self._u64(m) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))).reshape(-1)


def activity_chain(n_wf: int, k: int, seed: int, version: int = 1, with_keys: bool = True,
                   now_ns: int = BASE_TS + 10 ** 15, wf_ids=None) -> HistoryBatch:
    """Config 1/2 workload: n_wf activity-chain workflows with k activities each (canonical layout).
    ``wf_ids``: the workflows' indices in a larger workload (shard partitions, dist.rank_workflows); their
    draws then depend only on (seed, index), so every rank generates exactly its part of one workload."""
    if wf_ids is not None:
        wf_ids = np.asarray(wf_ids, np.int64)
        assert wf_ids.size == n_wf
        rng = _CounterDraws(seed, wf_ids)
    else:
        wf_ids = np.arange(n_wf, dtype=np.int64)
        rng = np.random.default_rng(seed)
    types, flags = activity_chain_template(k)
    L = types.size
    N = n_wf * L
    cols = {}
    et = np.tile(types | flags, n_wf)
    cols["etype"] = et
    eid = np.tile(np.arange(1, L + 1, dtype=np.int64), n_wf)
    cols["event_id"] = eid
    cols["version"] = np.full(N, version, np.int64)
    # timestamps: start = BASE + wf * 1s, deltas U[1 ms, 10 s]
    deltas = rng.integers(1_000_000, 10_000_000_000, size=(n_wf, L), dtype=np.int64)
    deltas[:, 0] = 0
    ts = np.cumsum(deltas, axis=1) + (BASE_TS + wf_ids * 1_000_000_000)[:, None]
    cols["timestamp"] = ts.reshape(-1)
    cols["task_id"] = ((wf_ids[:, None] * L + np.arange(L, dtype=np.int64)[None, :]).reshape(-1) + 1_000_000)
    ref = np.zeros((n_wf, L), np.int64)
    aux = np.zeros((n_wf, L), np.int32)
    key = np.zeros((n_wf, L), np.uint32)
    # references inside the template (same for every workflow)
    last_dsched = last_dstart = last_asched = 0
    act_idx_in_wf = 0
    act_pos = []
    for i, t in enumerate(types):
        e = i + 1
        if t == ET.DecisionTaskScheduled:
            last_dsched = e
        elif t == ET.DecisionTaskStarted:
            ref[:, i] = last_dsched
            last_dstart = e
        elif t == ET.DecisionTaskCompleted:
            ref[:, i] = last_dstart
            key[:, i] = 1                      # interned BinaryChecksum (same build every decision)
        elif t == ET.ActivityTaskScheduled:
            last_asched = e
            key[:, i] = 2 + act_idx_in_wf      # interned ActivityID "0", "1", ...
            act_pos.append(i)
            act_idx_in_wf += 1
        elif t in (ET.ActivityTaskStarted, ET.ActivityTaskCompleted):
            ref[:, i] = last_asched
    # DecisionTaskScheduled: attempt 0, StartToCloseTimeout U{10..60}
    dpos = np.nonzero(types == ET.DecisionTaskScheduled)[0]
    aux[:, dpos] = rng.integers(10, 61, size=(n_wf, dpos.size), dtype=np.int32)
    # WorkflowExecutionStarted -> start side record per workflow
    aux[:, 0] = np.arange(n_wf, dtype=np.int32)
    start_side = np.zeros(n_wf, abi.START_SIDE)
    start_side["decision_start_to_close"] = rng.integers(10, 61, size=n_wf)
    start_side["workflow_timeout"] = rng.integers(3600, 86400, size=n_wf)
    start_side["initiator"] = abi.INITIATOR_NIL
    start_side["prev_reset_count"] = -1
    # ActivityTaskScheduled -> activity side records
    n_act = n_wf * k
    act_side = np.zeros(max(n_act, 1), abi.ACTIVITY_SIDE)
    if n_act:
        act_side["schedule_to_start"][:n_act] = rng.integers(10, 3601, size=n_act)
        act_side["schedule_to_close"][:n_act] = rng.integers(10, 3601, size=n_act)
        act_side["start_to_close"][:n_act] = rng.integers(10, 3601, size=n_act)
        hb = rng.integers(10, 61, size=n_act)
        hb[rng.random(n_act) < 0.5] = 0
        act_side["heartbeat"][:n_act] = hb
        aux[:, act_pos] = np.arange(n_act, dtype=np.int32).reshape(n_wf, k)
    cols["ref"] = ref.reshape(-1)
    cols["aux"] = aux.reshape(-1)
    cols["key"] = key.reshape(-1)
    # branch tokens
    tok = branch_tokens(uuid_ascii(rng, n_wf), uuid_ascii(rng, n_wf))
    arena = tok.reshape(-1)
    wf = np.zeros(n_wf, abi.WORKFLOW)
    wf["ev_begin"] = np.arange(n_wf, dtype=np.int64) * L
    wf["ev_count"] = L
    wf["empty_batch_at"] = -1
    wf["init_version"] = version
    wf["now_ns"] = now_ns
    wf["start_token_off"] = np.arange(n_wf, dtype=np.uint32) * 96
    wf["start_token_len"] = 96
    wf["final_token_len"] = abi.NO_TOKEN
    batch = HistoryBatch(cols=cols, act_side=act_side, start_side=start_side,
                         reset_keys=np.zeros(1, np.uint32), arena=arena, wf=wf, stride=1)
    wf["retention_days"] = 1
    n_task = sum(TASKS_PER_EVENT.get(int(t), 0) for t in types) + 2 * int((flags & abi.BATCH_LAST != 0).sum())
    caps = {"act_cap": np.full(n_wf, k), "timer_cap": np.zeros(n_wf), "child_cap": np.zeros(n_wf),
            "rc_cap": np.zeros(n_wf), "sig_cap": np.zeros(n_wf), "vh_cap": np.ones(n_wf),
            "rp_cap": np.ones(n_wf), "task_cap": np.full(n_wf, n_task)}
    assign_canonical_tables(batch, caps)
    if with_keys:
        # per-event key strings for the oracle: "bin-v1" for decisions, str(i) for activity IDs
        strs = ["", "bin-v1"] + [str(i) for i in range(k)]
        enc = [s.encode() for s in strs]
        offs = np.cumsum([0] + [len(s) for s in enc])[:-1].astype(np.uint32)
        lens = np.array([len(s) for s in enc], np.uint32)
        kk = cols["key"]
        batch.key_off = offs[kk]
        batch.key_len = lens[kk]
        batch.key_arena = np.frombuffer(b"".join(enc) or b"\0", np.uint8).copy()
    return batch


def algorithmic_bytes(batch: HistoryBatch, res=None, token_crc: bool = True) -> int:
    """Algorithmic HBM bytes of one replay launch (DESIGN.md "Roofline").

    reads : 49 B per event (8 columns) + 32 / 48 B per activity / start side record read
            + the workflow descriptor (168 B) + the branch token bytes checksummed (token_crc: a 96-byte
            start token's 4-byte precomputed CRC instead, crr_inputs.token_crc)
    writes: the execution row (192 B) + 16 B per version-history item + the live pending rows
            (activity 112, timer 40, child 48, request-cancel / signal 32, reset point 16 B)
    """
    n_ev = batch.n_events
    t = batch.cols["etype"] & abi.ETYPE_MASK
    real = t != abi.EV_PAD
    n_act_sched = int(((t == ET.ActivityTaskScheduled) & real).sum())
    n_started = int(((t == ET.WorkflowExecutionStarted) & real).sum())
    tl = np.minimum(batch.wf["start_token_len"].astype(np.int64), 4096)
    tok = int(np.where(token_crc & (tl == 96), 4, tl).sum())
    b = (n_ev * abi.BYTES_PER_EVENT + abi.ACTIVITY_SIDE.itemsize * n_act_sched + abi.START_SIDE.itemsize * n_started
         + batch.n_wf * abi.WORKFLOW.itemsize + tok)
    b += batch.n_wf * abi.EXEC_ROW.itemsize
    if res is not None:
        ex = res.exec
        b += 16 * int(ex["n_vh_items"].sum())
        b += 112 * int(ex["n_activity"].sum()) + 40 * int(ex["n_timer"].sum()) + 48 * int(ex["n_child"].sum())
        b += 32 * int(ex["n_rc"].sum() + ex["n_signal"].sum()) + 16 * int(ex["n_reset_points"].sum())
    else:
        b += 16 * batch.n_wf
    return int(b)
