"""Passive replication at scale: one new batch applied onto every workflow's loaded mutable state.

The production hot path of ``ndc/history_replicator.go:385-460`` (call at :396): the state persisted
after batches 1..k-1 is loaded (``mutableStateBuilder.Load``, mutable_state_builder.go:306-349) and
``StateBuilder.ApplyEvents`` applies batch k onto it (state_builder.go:73-88, :90-648).  On the device
the loaded state is the previous replay's output rows, left in place in HBM (slots 0..n-1 of each
workflow's regions, exactly where ``write_init`` puts a state loaded from the host), so a replication
step is one ``crr_replay`` over the new batch with CRR_WF_FLAG_RESUME.

``PassiveReplication`` cuts every workflow of an interleaved batch before its last event batch: the
prefix replays once from scratch (setup), the device output buffers are snapshotted, and each
measured step restores the snapshot (device copy, outside the timed launch) and applies the last
batches.  ``verify`` checks the result against the one-shot replay of the whole histories.
"""
from __future__ import annotations

import dataclasses
from typing import Dict

import numpy as np

from . import abi
from .engine import DeviceBatch, ReplayEngine
from .flatten import HistoryBatch
from .result import ReplayResult, gather_live


def last_batch_cut(batch: HistoryBatch) -> np.ndarray:
    """Per workflow: the step at which its last event batch starts (0 for single-batch histories)."""
    cnt = batch.wf["ev_count"].astype(np.int64)
    st = batch.wf_strides()
    tot = int(cnt.sum())
    wf_idx = np.repeat(np.arange(batch.n_wf), cnt)
    step = np.arange(tot) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    idx = batch.wf["ev_begin"].astype(np.int64)[wf_idx] + step * st[wf_idx]
    first = (batch.cols["etype"][idx] & abi.BATCH_FIRST) != 0
    cut = np.zeros(batch.n_wf, np.int64)
    np.maximum.at(cut, wf_idx[first], step[first])
    return cut


def suffix_batch(batch: HistoryBatch, cut: np.ndarray, split: np.ndarray, suf_wf: np.ndarray) -> HistoryBatch:
    """The new events alone, laid out as the host would upload them: every workflow's events from its
    cut on, re-interleaved (lane workflows: group-uniform bases, 64-wide; the wave tail contiguous),
    with the descriptors of ``suf_wf`` (table bases unchanged: the loaded rows stay where they are)."""
    n = batch.n_wf
    wave = batch.stride
    n_lane = batch.wave_begin if batch.wave_begin is not None else n
    st = batch.wf_strides()
    cnt = np.where(split, batch.wf["ev_count"].astype(np.int64) - cut, 0)
    n_groups = (n_lane + wave - 1) // wave
    pos = np.arange(n_lane)
    gcnt = np.zeros(n_groups * wave, np.int64)
    gcnt[:n_lane] = cnt[:n_lane]
    glen = gcnt.reshape(n_groups, wave).max(axis=1) if n_groups else np.zeros(0, np.int64)
    gbase = np.concatenate([[0], np.cumsum(glen * wave)[:-1]]).astype(np.int64) if n_groups else glen
    lane_slots = int((glen * wave).sum())
    begin = np.empty(n, np.int64)
    begin[:n_lane] = gbase[pos // wave] + pos % wave
    tail = cnt[n_lane:]
    begin[n_lane:] = lane_slots + np.concatenate([[0], np.cumsum(tail)[:-1]]).astype(np.int64)
    nst = np.where(np.arange(n) < n_lane, wave, 1)
    wf_idx = np.repeat(np.arange(n), cnt)
    k = np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    src = batch.wf["ev_begin"].astype(np.int64)[wf_idx] + (cut[wf_idx] + k) * st[wf_idx]
    dst = begin[wf_idx] + k * nst[wf_idx]
    total = lane_slots + int(tail.sum())
    cols = {}
    for name, t in abi.EVENT_COLUMNS:
        c = np.zeros(max(total, 1), dtype=t)
        if name == "etype":
            c[:] = abi.EV_PAD | abi.BATCH_FIRST | abi.BATCH_LAST
        c[dst] = batch.cols[name][src]
        cols[name] = c
    wf = suf_wf.copy()
    wf["ev_begin"] = begin
    wf["ev_count"] = cnt
    out = dataclasses.replace(batch, cols=cols, wf=wf, init=None, table_rows=dict(batch.table_rows))
    if batch.key_off is not None:
        out.key_off = np.zeros(max(total, 1), np.uint32)
        out.key_len = np.zeros(max(total, 1), np.uint32)
        out.key_off[dst] = batch.key_off[src]
        out.key_len[dst] = batch.key_len[src]
    return out


def split_descriptors(batch: HistoryBatch, cut: np.ndarray):
    """(prefix wf, suffix wf, split mask) descriptor arrays over the same device layout (the suffix's
    ev_begin still indexes the whole batch's columns: ``suffix_batch`` relays them out)."""
    split = (cut > 0) & ((batch.wf["flags"] & abi.WF_FLAG_NEW_RUN) == 0)
    pre = batch.wf.copy()
    suf = batch.wf.copy()
    st = batch.wf_strides()
    c = np.where(split, cut, 0)
    cnt = batch.wf["ev_count"].astype(np.int64)
    ea = batch.wf["empty_batch_at"].astype(np.int64)
    pre["ev_count"] = np.where(split, c, cnt)
    pre["empty_batch_at"] = np.where(split & (ea >= c), -1, ea)
    # the prefix is an intermediate state: no rebuild finalisation / task refresh yet
    pre["final_token_len"] = np.where(split, abi.NO_TOKEN, pre["final_token_len"])
    pre["flags"] = np.where(split, pre["flags"] & ~np.uint32(abi.WF_FLAG_REFRESH_TASKS), pre["flags"])
    suf["ev_begin"] = batch.wf["ev_begin"] + np.where(split, c * st, 0)
    suf["ev_count"] = np.where(split, cnt - c, 0)
    suf["empty_batch_at"] = np.where(split, np.where(ea >= c, ea - c, -1), -1)
    # every workflow resumes: a split one applies its last batch, the others apply nothing (their rows
    # are re-finalised unchanged)
    suf["flags"] = suf["flags"] | np.uint32(abi.WF_FLAG_RESUME)
    return pre, suf, split


@dataclasses.dataclass
class PassiveReplication:
    eng: ReplayEngine
    batch: HistoryBatch                   # interleaved, from scratch
    db: DeviceBatch = None                # the whole histories' layout: its output buffers hold the state
    db_new: DeviceBatch = None            # the new batches (suffix events), writing into db's outputs
    split: np.ndarray = None
    prefix: ReplayResult = None
    snapshot: Dict[str, object] = None
    n_events: int = 0                     # events applied per step
    hbm_rows: bool = False                # continue every lane workflow over its HBM rows (A/B only)
    pre_wf: np.ndarray = None             # the prefix replay's descriptors
    suffix: HistoryBatch = None           # the new events (the step's inputs, host copy)
    live_ids: bool = True                 # keep the live-ID sidecar (crr_outputs.live_ids)

    def setup(self):
        eng, torch, b = self.eng, self.eng.torch, self.batch
        cut = last_batch_cut(b)
        pre, suf, self.split = split_descriptors(b, cut)
        db = eng.upload(b, live_ids=self.live_ids)
        self.db = db
        wf_dev = db.tensors["wf"]
        nb = pre.nbytes
        wf_dev[:nb].copy_(torch.from_numpy(pre.view(np.uint8)))
        eng.launch(db)
        torch.cuda.synchronize(eng.dev)
        self.prefix = eng.download(db)
        self.pre_wf = pre
        sb = suffix_batch(b, cut, self.split, suf)
        self.suffix = sb
        self.n_events = sb.n_events
        dn = eng.upload(sb)
        dn.c_out = db.c_out                        # apply onto the loaded rows in place
        # the loaded states continue in the compact tiers' LDS arenas (CRR_IN_HAS_RESUME, set by the
        # batch's flags): each workflow keeps the segment of its whole history, whose live-set bound covers
        # the loaded rows plus the new batch's; hbm_rows=True instead continues every lane workflow over its
        # HBM rows (the wide GlobalTables segment) -- the round-3 path, kept for A/B measurements
        if sb.tiers is not None and self.hbm_rows:
            dn.c_in.large_begin = dn.c_in.compact_begin = dn.c_in.compact2_begin = dn.c_in.wide_begin = 0
            dn.c_in.hbm_begin = 0
            dn.c_in.flags &= ~(abi.IN_LDS_SMALL | abi.IN_HAS_RESUME)
        elif sb.tiers is not None:
            # every workflow resumes, and the 1- and 2-slot tiers rebuild rows from this call's events only:
            # their segments join compact tier 1 (whose bounds hold theirs)
            dn.c_in.large_begin = dn.c_in.compact_begin = 0
        for name, *_ in abi.TABLES:                # only db's outputs are used
            dn.tensors.pop("out_" + name, None)
        for name in abi.ID_TABLES:                 # (the live-ID sidecar too)
            dn.tensors.pop("ids_" + name, None)
        dn.tensors.pop("exec", None)
        self.db_new = dn
        self.snapshot = {k: db.tensors[k].clone() for k in self._state_keys()}
        torch.cuda.synchronize(eng.dev)

    def _state_keys(self):
        return ["exec"] + ["out_" + name for name, *_ in abi.TABLES]

    def restore(self, stream=None):
        torch = self.eng.torch
        s = stream if stream is not None else torch.cuda.current_stream(self.eng.dev)
        with torch.cuda.stream(s):
            for k in self._state_keys():
                self.db.tensors[k].copy_(self.snapshot[k], non_blocking=True)

    def step(self, stream=None):
        self.eng.launch(self.db_new, stream)

    def verify_oracle(self, replay_fn, threads: int) -> Dict[str, int]:
        """The last step's rows against the oracle given the same split (``replay_fn`` = oracle.replay: the
        suffix batch with the prefix replay's rows as its loaded states, mutableStateBuilder.Load then
        ApplyEvents) -- every split workflow whose prefix replayed OK, the Load-unstable ones included.
        Returns the counts compared and the mismatching fields."""
        b = self.batch
        ok_dev = self.prefix.exec["status"] == 0
        mask_c = np.zeros(b.n_wf, bool)
        if b.perm is None:
            mask_c[:] = ok_dev
        else:
            mask_c[b.perm] = ok_dev
        loaded = self.prefix.to_loaded(dataclasses.replace(b, wf=self.pre_wf), mask=mask_c)
        if b.perm is not None:
            loaded = loaded.permuted(b.perm)
        kd = self.suffix.key_dict if self.suffix.key_dict is not None else key_dict_from_events(b)
        ref = replay_fn(dataclasses.replace(self.suffix, init=loaded, key_dict=kd), threads)
        res = self.eng.download(self.db)
        sel = ok_dev & self.split
        bad = _compare_rows(b, res, ref, sel)
        c = np.clip(self.prefix.exec["n_activity"].astype(np.int64), 0, b.wf["act_cap"].astype(np.int64))
        live_pre = gather_live(b, self.prefix)
        unstable = np.zeros(b.n_wf, bool)
        np.logical_or.at(unstable, np.repeat(np.arange(b.n_wf), c)[(live_pre["act"]["flags"] & abi.ROW_MAPPED) == 0], True)
        return {"compared_workflows": int(sel.sum()), "load_unstable_compared": int((sel & unstable).sum()),
                "mismatches": bad}

    def verify_prefix_oracle(self, replay_fn, threads: int) -> Dict[str, int]:
        """The prefix replay (the loaded states every step starts from) against the oracle over the same
        descriptors -- every workflow, every exec field and live row -- so that ``verify_oracle`` (which
        hands the oracle the device's prefix rows as its loaded states) does not rest on the device alone."""
        b = dataclasses.replace(self.batch, wf=self.pre_wf)
        ref = replay_fn(b, threads)
        bad = _compare_rows(b, self.prefix, ref, np.ones(b.n_wf, bool))
        return {"compared_workflows": int(b.n_wf), "events": int(self.pre_wf["ev_count"].astype(np.int64).sum()),
                "mismatches": bad}

    def verify(self, one_shot: ReplayResult) -> Dict[str, int]:
        """Compare the last step's rows with the one-shot replay of the whole histories (same layout):
        every field of the exec row but the per-call counters, and every live row, for the split
        workflows whose prefix and whole replays are OK and whose loaded state is Load-stable (each
        live activity keeps its ActivityID mapping, mutable_state_builder.go:311-314)."""
        b = self.batch
        res = self.eng.download(self.db)
        ok = (self.prefix.exec["status"] == 0) & (one_shot.exec["status"] == 0) & self.split
        live_pre = gather_live(b, self.prefix)
        c = np.clip(self.prefix.exec["n_activity"].astype(np.int64), 0, b.wf["act_cap"].astype(np.int64))
        wf = np.repeat(np.arange(b.n_wf), c)
        unstable = np.zeros(b.n_wf, bool)
        np.logical_or.at(unstable, wf[(live_pre["act"]["flags"] & abi.ROW_MAPPED) == 0], True)
        sel = ok & ~unstable
        bad = _compare_rows(b, res, one_shot, sel, exact_flags=False, skip=("inconsistencies",))
        return {"compared_workflows": int(sel.sum()), "split_workflows": int(self.split.sum()),
                "resumed_ok": int((res.exec["status"] == 0).sum()), "mismatches": bad}


def resume_blob_set(b: HistoryBatch, canon_bs, cut: np.ndarray, split: np.ndarray, pre_wf: np.ndarray):
    """What passive replication receives, laid out for ``crr_ingest_plan_resume``: device position p's
    replication-task payload -- the persisted blob(s) of its last event batch (``canon_bs``: the whole
    histories of ``b``'s canonical batch, one blob per ApplyEvents batch; an empty batch at or after the cut
    comes along) -- and the loaded state's key dictionary (the strings of key ids 1..K interned by the prefix,
    ``key_dict_from_events`` over the prefix descriptors ``pre_wf``), its strings appended after the blobs.
    Workflows that are not split get no blob (they apply nothing).  Returns (BlobSet, seeds: dict of
    key_begin / key_count / key_off / key_len arrays)."""
    from .blobs import BlobSet
    n = b.n_wf
    perm = b.perm if b.perm is not None else np.arange(n)
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    src = canon_bs.wf[perm].copy()
    bc = src["blob_count"].astype(np.int64)
    bb = src["blob_begin"].astype(np.int64)
    ea = b.wf["empty_batch_at"].astype(np.int64)
    j = bc - 1 - np.where((ea >= 0) & (ea >= cut), 1, 0)
    take = np.where(split, bc - j, 0)
    tot = int(take.sum())
    blob_idx = np.repeat(bb + j, take) + (np.arange(tot) - np.repeat(np.cumsum(take) - take, take))
    bo = canon_bs.blob_off.astype(np.int64)
    lens = bo[blob_idx + 1] - bo[blob_idx]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    nbytes = int(off[-1])
    byte_src = np.repeat(bo[blob_idx], lens) + (np.arange(nbytes) - np.repeat(off[:-1], lens))
    # seeds: the dictionary the prefix interned -- ids 1..K, K the largest id its events' keys or its Started
    # events' previous reset points (interned with them, WfFlattener::add) carry; each id's string from the
    # whole history's events, or the encoder's name for an id no event names (blob_encode.cpp "rk-<id>")
    K = _prefix_key_count(b, pre_wf)
    kb, kc, ko, kl, arena = key_dict_from_events(b)
    arena = arena if arena is not None else np.zeros(0, np.uint8)
    wf_of = np.repeat(np.arange(n), K)
    kid = np.arange(int(K.sum())) - np.repeat(np.cumsum(K) - K, K) + 1
    have = kid < kc.astype(np.int64)[wf_of]
    e = np.where(have, kb.astype(np.int64)[wf_of] + kid, 0)
    s_off = np.where(have, ko[e], 0).astype(np.int64)
    s_len = np.where(have, kl[e], 0).astype(np.int64)
    missing = np.nonzero(s_len == 0)[0]
    extra = [b"rk-%d" % int(kid[i]) for i in missing]
    if extra:
        ex_len = np.array([len(x) for x in extra], np.int64)
        s_off[missing] = arena.size + np.concatenate([[0], np.cumsum(ex_len)[:-1]])
        s_len[missing] = ex_len
        arena = np.concatenate([arena, np.frombuffer(b"".join(extra), np.uint8)])
    seed_base = (nbytes + 15) // 16 * 16
    data = np.zeros(seed_base + arena.size + 32, np.uint8)
    data[:nbytes] = canon_bs.bytes[byte_src]
    data[seed_base:seed_base + arena.size] = arena
    src["blob_begin"] = (np.cumsum(take) - take).astype(np.uint32)
    src["blob_count"] = take.astype(np.uint32)
    nr = src["new_run_wf"].astype(np.int64)
    src["new_run_wf"] = np.where(nr >= 0, inv[np.clip(nr, 0, n - 1)], -1).astype(np.int32)
    bs = BlobSet(bytes=data, blob_off=off.astype(np.uint64), wf=src, strings=canon_bs.strings)
    seeds = {"key_begin": (np.cumsum(K) - K).astype(np.uint32), "key_count": K.astype(np.uint32),
             "key_off": (seed_base + s_off).astype(np.uint64), "key_len": s_len.astype(np.uint32)}
    return bs, seeds


def _prefix_key_count(b: HistoryBatch, pre_wf: np.ndarray) -> np.ndarray:
    """Per workflow: the largest key id its prefix (``pre_wf``'s events) interned -- an event's key or a
    previous reset point of a WorkflowExecutionStarted event."""
    cnt = pre_wf["ev_count"].astype(np.int64)
    st = b.wf_strides()
    wf_idx = np.repeat(np.arange(b.n_wf), cnt)
    step = np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    x = pre_wf["ev_begin"].astype(np.int64)[wf_idx] + step * st[wf_idx]
    K = np.zeros(b.n_wf, np.int64)
    np.maximum.at(K, wf_idx, b.cols["key"][x].astype(np.int64))
    started = (b.cols["etype"][x] & abi.ETYPE_MASK) == abi.EventType.WorkflowExecutionStarted
    if started.any():
        ss = b.start_side[b.cols["aux"][x[started]].astype(np.int64)]
        c = np.maximum(ss["prev_reset_count"].astype(np.int64), 0)
        w = np.repeat(wf_idx[started], c)
        j = np.repeat(ss["prev_reset_key_off"].astype(np.int64), c) + (np.arange(int(c.sum())) - np.repeat(np.cumsum(c) - c, c))
        if j.size:
            np.maximum.at(K, w, b.reset_keys[j].astype(np.int64))
    return K


@dataclasses.dataclass
class BlobReplication:
    """The same replication step from the task's persisted bytes, on the device: the last batches' blobs
    resident in HBM (as the replication task carries them, ``replication_task.go:386-390``) are decoded and
    laid out by ``crr_ingest_plan_resume`` / ``crr_ingest_layout_resume`` (``serializer.go:109-119``), then
    replayed onto the loaded rows in place -- every stage on the device, inside ``step``."""
    pr: PassiveReplication
    canon_bs: object                      # blobs.BlobSet of the whole histories (canonical order)
    ing: object = None                    # ingest.DeviceIngest
    blobs: object = None                  # ingest.DeviceBlobs: the tasks' payloads + the seeds' strings
    resume: object = None                 # ingest.CIngestResume
    db: DeviceBatch = None                # inputs written by the layout, outputs = the loaded rows
    tensors: Dict[str, object] = None
    n_events: int = 0

    def setup(self):
        from .ingest import CIngestResume, DeviceIngest
        pr, eng, torch = self.pr, self.pr.eng, self.pr.eng.torch
        b = pr.batch
        cut = last_batch_cut(b)
        bs, seeds = resume_blob_set(b, self.canon_bs, cut, pr.split, pr.pre_wf)
        self.ing = self.ing or DeviceIngest(eng)
        self.blobs = self.ing.upload(bs)
        T = {k: torch.from_numpy(np.ascontiguousarray(v)).to(eng.dev) if v.size else
             torch.zeros(1, dtype=torch.int64, device=eng.dev) for k, v in seeds.items()}
        T["loaded_wf"] = torch.from_numpy(b.wf.view(np.uint8).copy()).to(eng.dev)   # the loaded descriptors
        R = CIngestResume()
        R.loaded_wf = T["loaded_wf"].data_ptr()
        R.wave_begin = b.wave_begin if b.wave_begin is not None else b.n_wf
        for k in seeds:
            setattr(R, k, T[k].data_ptr())
        self.resume = R
        ci = abi.CInputs.from_buffer_copy(pr.db_new.c_in)   # the host path's flags and tiering
        ci.arena = pr.db.c_in.arena                          # the loaded descriptors' branch tokens
        self.db = DeviceBatch(pr.db_new.batch, T, ci, pr.db_new.c_out, eng.device)
        self.tensors = T
        S = self.ing.plan(self.blobs, resume=R)
        # the loaded descriptors are the replay's: the layout writes the new events' fields into them in place
        self.ing.allocate_inputs(S, T, ci, slack=1.05, wf_in_place=T["loaded_wf"])
        self.n_events = int(S.n_events)

    def step(self, stream=None):
        S = self.ing.plan(self.blobs, stream, resume=self.resume)
        self.ing.allocate_inputs(S, self.tensors, self.db.c_in, slack=1.05, wf_in_place=self.tensors["loaded_wf"])
        self.ing.layout_resume(self.blobs, self.resume, S, self.db.c_in, stream)
        self.pr.eng.launch(self.db, stream)
        return S


def key_dict_from_events(b: HistoryBatch):
    """Per-workflow key id -> string tables (flatten.key_dict_from_interners' format, batch order) from the
    events' own key strings: a workflow's ids are interned over its history, so every id its rows hold
    names a string some event of the history carries."""
    cnt = b.wf["ev_count"].astype(np.int64)
    st = b.wf_strides()
    wf_idx = np.repeat(np.arange(b.n_wf), cnt)
    step = np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    x = b.wf["ev_begin"].astype(np.int64)[wf_idx] + step * st[wf_idx]
    key = b.cols["key"][x].astype(np.int64)
    count = np.zeros(b.n_wf, np.int64)
    np.maximum.at(count, wf_idx, key + 1)
    count = np.maximum(count, 1)
    begin = np.cumsum(count) - count
    off = np.zeros(int(count.sum()), np.uint32)
    ln = np.zeros(int(count.sum()), np.uint32)
    has = key > 0
    slot = begin[wf_idx[has]] + key[has]
    off[slot] = b.key_off[x[has]]
    ln[slot] = b.key_len[x[has]]
    return begin.astype(np.uint32), count.astype(np.uint32), off, ln, b.key_arena


def _compare_rows(b: HistoryBatch, res: ReplayResult, want: ReplayResult, sel: np.ndarray, exact_flags=True,
                  skip=()) -> int:
    """Mismatching exec fields and live-row fields of the workflows in ``sel`` (device order; both results
    in ``b``'s layout).  exact_flags=False: a row's ActivityID-mapping bit is not compared (Load recomputes
    it; the one-shot replay never reloaded)."""
    bad = 0
    for f in abi.EXEC_ROW.names:
        if f in ("reserved", "n_tasks") or f in skip:
            continue
        bad += int(((res.exec[f] != want.exec[f]) & sel).sum())
    la, lb = gather_live(b, res), gather_live(b, want)
    for name, _dt, _b, cap_f, n_f in abi.TABLES:
        if name == "tasks":
            continue
        cap = b.wf[cap_f].astype(np.int64)     # gather_live's clamp
        ca = np.clip(res.exec[n_f].astype(np.int64), 0, cap)
        cb = np.clip(want.exec[n_f].astype(np.int64), 0, cap)
        ra, rb = la[name][np.repeat(sel, ca)], lb[name][np.repeat(sel, cb)]
        if ra.shape != rb.shape:
            bad += 1
            continue
        for fld in ra.dtype.names:
            if fld == "reserved":
                continue
            x, y = ra[fld], rb[fld]
            if fld == "flags" and not exact_flags:
                x, y = x & ~np.uint32(abi.ROW_MAPPED), y & ~np.uint32(abi.ROW_MAPPED)
            bad += int((x != y).sum())
    return bad
