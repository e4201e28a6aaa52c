"""End-to-end replay from host buffers: pinned staging, chunked and overlapped.

What a caller that holds histories in host memory pays (SURVEY.md §8d's PCIe-inclusive figure): the
columns go up from pinned staging buffers (where the native decoder / flattener writes them), the
replay and the live-row compaction (``crr_compact_rows``) run on the device, and only the exec rows
and the dense live rows come back, into pinned buffers.  Three HIP streams: uploads of chunk i+1.. run
while chunk i replays and while chunk i-1 downloads (PCIe is full duplex), so the wall time tends to
the larger of the two transfer totals rather than their sum.

Setup (untimed, once per batch shape): pinned host copies of the inputs, device buffers, pinned
output buffers.  Timed: per chunk, the uploads, zero-filling the outputs, the replay, the compaction,
the download of the exact live-row counts.  Replays from scratch only (a batch with loaded states,
CRR_WF_FLAG_RESUME, keeps its rows in the output buffers this zero-fills).
"""
from __future__ import annotations

import dataclasses
import time
from typing import Dict, List

import numpy as np

from . import abi
from .engine import COMPACT_TABLES, CompactResult, DeviceBatch, ReplayEngine
from .flatten import HistoryBatch


@dataclasses.dataclass
class _Chunk:
    batch: HistoryBatch
    db: DeviceBatch
    host_in: Dict[str, object]        # name -> pinned uint8 tensor
    dev_in: Dict[str, object]         # name -> device uint8 tensor (same bytes)
    host_exec: object
    host_off: object
    host_rows: Dict[str, object]
    host_tot: object
    totals: np.ndarray = None


def _input_arrays(batch: HistoryBatch) -> Dict[str, np.ndarray]:
    arrs = {"ev_" + name: np.asarray(batch.cols[name], dtype=t) for name, t in abi.EVENT_COLUMNS}
    arrs.update(act_side=batch.act_side, start_side=batch.start_side, reset_keys=batch.reset_keys,
                arena=np.concatenate([batch.arena, np.zeros(16, np.uint8)]), wf=batch.wf)
    return {k: np.ascontiguousarray(v).view(np.uint8).reshape(-1) for k, v in arrs.items()}


class StreamingReplay:
    """Chunked host -> device -> host replay of a list of (interleaved) batches."""

    def __init__(self, eng: ReplayEngine, chunks: List[HistoryBatch], wire: bool = False):
        """``wire``: ship the event columns in the narrow format (wire.py) and widen them on the device."""
        torch = eng.torch
        self.eng, self.torch, self.wire = eng, torch, wire
        self.chunks: List[_Chunk] = []
        self.pack_s = 0.0
        for b in chunks:
            db = eng.upload(b)                      # device buffers (inputs + outputs) and the C structs
            arrs = _input_arrays(b)
            if wire:
                from .wire import COLUMNS, pack_events
                t0 = time.perf_counter()
                pk = pack_events(b)
                self.pack_s += time.perf_counter() - t0
                eng.attach_packed(db, pk)
                for c in COLUMNS:
                    del arrs["ev_" + c]
                    arrs["pk_" + c] = pk.data[c]
                arrs["pk_ts_base"] = pk.ts_base.view(np.uint8)
            host_in, dev_in = {}, {}
            for k, a in arrs.items():
                host_in[k] = torch.from_numpy(a.copy()).pin_memory()
                dev_in[k] = db.tensors[k].view(torch.uint8)[:a.size]
            eng.compact(db)                         # allocates the dense buffers (first call)
            n = b.n_wf
            host_rows = {name: torch.empty(db.tensors["cmp_" + name].numel(), dtype=torch.uint8).pin_memory()
                         for name in COMPACT_TABLES}
            self.chunks.append(_Chunk(
                b, db, host_in, dev_in,
                torch.empty(n * abi.EXEC_ROW.itemsize, dtype=torch.uint8).pin_memory(),
                torch.empty(len(COMPACT_TABLES) * (n + 1), dtype=torch.int64).pin_memory(),
                host_rows, torch.empty(len(COMPACT_TABLES), dtype=torch.int64).pin_memory()))
        torch.cuda.synchronize(eng.dev)
        self.up = torch.cuda.Stream(eng.dev)
        self.comp = torch.cuda.Stream(eng.dev)
        self.down = torch.cuda.Stream(eng.dev)

    @property
    def n_events(self) -> int:
        return sum(c.batch.n_events for c in self.chunks)

    @property
    def h2d_bytes(self) -> int:
        return int(sum(t.numel() for c in self.chunks for t in c.host_in.values()))

    def run(self) -> Dict[str, float]:
        """One timed pass over every chunk; returns wall time and transfer volumes."""
        torch, eng = self.torch, self.eng
        torch.cuda.synchronize(eng.dev)
        t0 = time.perf_counter()
        ev_up, ev_tot = [], []
        for c in self.chunks:                                      # 1. every upload, in order
            with torch.cuda.stream(self.up):
                for k, h in c.host_in.items():
                    c.dev_in[k].copy_(h, non_blocking=True)
                e = torch.cuda.Event()
                e.record(self.up)
                ev_up.append(e)
        for c, e in zip(self.chunks, ev_up):                        # 2. replay + compaction per chunk
            self.comp.wait_event(e)
            with torch.cuda.stream(self.comp):
                T = c.db.tensors
                for k in ("exec", "scratch"):
                    T[k].zero_()
                for name, *_ in abi.TABLES:
                    T["out_" + name].zero_()
                if self.wire:
                    eng.widen(c.db, self.comp)
                eng.launch(c.db, self.comp)
                eng.compact(c.db, self.comp)
                n = c.batch.n_wf
                c.host_tot.copy_(T["cmp_offsets"].view(len(COMPACT_TABLES), n + 1)[:, n], non_blocking=True)
                et = torch.cuda.Event()
                et.record(self.comp)
                ev_tot.append(et)
        d2h = 0
        for c, et in zip(self.chunks, ev_tot):                      # 3. exact-size downloads
            et.synchronize()
            c.totals = c.host_tot.numpy().copy()
            self.down.wait_event(et)
            with torch.cuda.stream(self.down):
                T = c.db.tensors
                n = c.batch.n_wf
                c.host_exec.copy_(T["exec"][:n * abi.EXEC_ROW.itemsize], non_blocking=True)
                c.host_off.copy_(T["cmp_offsets"], non_blocking=True)
                d2h += n * abi.EXEC_ROW.itemsize + c.host_off.numel() * 8
                for t, (name, dt, *_) in enumerate(abi.TABLES):
                    nb = int(c.totals[t]) * dt.itemsize
                    if nb:
                        c.host_rows[name][:nb].copy_(T["cmp_" + name][:nb], non_blocking=True)
                        d2h += nb
        self.down.synchronize()
        wall = time.perf_counter() - t0
        return {"wall_s": wall, "events": self.n_events, "events_per_s": self.n_events / wall,
                "h2d_bytes": self.h2d_bytes, "d2h_bytes": int(d2h), "chunks": len(self.chunks)}

    def results(self) -> List[CompactResult]:
        out = []
        for c in self.chunks:
            n = c.batch.n_wf
            off = c.host_off.numpy().reshape(len(COMPACT_TABLES), n + 1).copy()
            rows = {}
            for t, (name, dt, *_) in enumerate(abi.TABLES):
                rows[name] = c.host_rows[name][:int(off[t, n]) * dt.itemsize].numpy().view(dt).copy()
            out.append(CompactResult(c.host_exec.numpy().view(abi.EXEC_ROW).copy(), off, rows))
        return out


# ---- persisted blobs -> device rows, end to end ----------------------------------------------------------------
def split_blobs(bs, chunks: int):
    """Split a BlobSet at workflow boundaries into `chunks` BlobSets (blob ranges and offsets rebased).
    Continue-as-new links (new_run_wf) must stay inside a chunk: the split moves a boundary forward
    past any workflow whose new-run history would land in the next chunk."""
    from .blobs import BlobSet
    n = bs.n_wf
    bounds = [int(x) for x in np.linspace(0, n, chunks + 1)]
    nr = bs.wf["new_run_wf"].astype(np.int64)
    for i in range(1, chunks):
        b = bounds[i]
        while 0 < b < n and ((nr[:b] >= b).any()):
            b += 1
        bounds[i] = max(b, bounds[i - 1])
    out = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        wf = bs.wf[a:b].copy()
        if b == a:
            continue
        b0 = int(wf["blob_begin"][0])
        b1 = int(wf["blob_begin"][-1] + wf["blob_count"][-1])
        o0, o1 = int(bs.blob_off[b0]), int(bs.blob_off[b1])
        wf["blob_begin"] -= b0
        wf["new_run_wf"] = np.where(wf["new_run_wf"] >= 0, wf["new_run_wf"] - a, -1)
        data = np.zeros(o1 - o0 + 32, np.uint8)
        data[:o1 - o0] = bs.bytes[o0:o1]
        # this chunk's strings only (run / branch IDs, final tokens), offsets rebased
        spans = [(wf["run_id_off"], wf["run_id_len"]), (wf["branch_id_off"], wf["branch_id_len"])]
        has_ft = wf["final_token_len"] != abi.NO_TOKEN
        spans.append((np.where(has_ft, wf["final_token_off"], 0), np.where(has_ft, wf["final_token_len"], 0)))
        lens = np.stack([ln.astype(np.int64) for _o, ln in spans], axis=1)
        new_off = (np.cumsum(lens.reshape(-1)) - lens.reshape(-1)).reshape(lens.shape)
        offs = np.stack([o.astype(np.int64) for o, _l in spans], axis=1).reshape(-1)
        fl = lens.reshape(-1)
        idx = np.repeat(offs - (np.cumsum(fl) - fl), fl) + np.arange(int(fl.sum()), dtype=np.int64)
        strings = bs.strings[idx] if idx.size else np.zeros(1, np.uint8)
        wf["run_id_off"] = new_off[:, 0]
        wf["branch_id_off"] = new_off[:, 1]
        wf["final_token_off"] = np.where(has_ft, new_off[:, 2], 0)
        out.append(BlobSet(bytes=data, blob_off=(bs.blob_off[b0:b1 + 1] - o0).astype(np.uint64), wf=wf,
                           strings=strings if strings.size else np.zeros(1, np.uint8)))
    return out


class BlobStreamingReplay:
    """Persisted blobs in host memory -> replayed rows in host memory, chunked and overlapped: per chunk
    the H2D of the blobs (pinned staging, as read from persistence), crr_ingest_plan + crr_ingest_layout
    (decode, intern, order, interleave on the device), the replay, crr_compact_rows and the D2H of the
    exec rows + live rows.  Uploads run ahead on their own stream; chunks alternate between two compute
    streams so one chunk's plan (which synchronises its stream to size the layout) overlaps the previous
    chunk's replay; downloads on a third stream."""

    def __init__(self, eng: ReplayEngine, chunks):
        from .ingest import DeviceIngest
        torch = eng.torch
        self.eng, self.torch = eng, torch
        self.parts = []
        for bs in chunks:
            ing = DeviceIngest(eng)
            host = {k: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).pin_memory()
                    for k, a in ing.host_arrays(bs).items()}
            db = ing.upload(bs, host={k: v.numpy() for k, v in host.items()})
            S = ing.plan(db)                            # sizes the scratch and the buffers once (untimed)
            out = ing.layout(db, S)
            eng.compact(out)
            n = int(S.n_wf)
            host_rows = {name: torch.empty(out.tensors["cmp_" + name].numel(), dtype=torch.uint8).pin_memory()
                         for name in COMPACT_TABLES}
            self.parts.append({"bs": bs, "ing": ing, "db": db, "host": host, "out": out, "S": S, "n": n,
                               "n_events": int(S.n_events),
                               "host_exec": torch.empty(n * abi.EXEC_ROW.itemsize, dtype=torch.uint8).pin_memory(),
                               "host_off": torch.empty(len(COMPACT_TABLES) * (n + 1), dtype=torch.int64).pin_memory(),
                               "host_rows": host_rows,
                               "host_tot": torch.empty(len(COMPACT_TABLES), dtype=torch.int64).pin_memory()})
        torch.cuda.synchronize(eng.dev)
        self.up = torch.cuda.Stream(eng.dev)
        self.comp = [torch.cuda.Stream(eng.dev), torch.cuda.Stream(eng.dev)]
        self.down = torch.cuda.Stream(eng.dev)

    @property
    def n_events(self) -> int:
        return sum(p["n_events"] for p in self.parts)

    @property
    def h2d_bytes(self) -> int:
        return int(sum(t.numel() for p in self.parts for t in p["host"].values()))

    def run(self) -> Dict[str, float]:
        torch, eng = self.torch, self.eng
        torch.cuda.synchronize(eng.dev)
        t0 = time.perf_counter()
        ev_up = []
        for p in self.parts:                                        # 1. every upload, in order
            with torch.cuda.stream(self.up):
                for k, h in p["host"].items():
                    p["db"].tensors[k][:h.numel()].copy_(h, non_blocking=True)
                e = torch.cuda.Event()
                e.record(self.up)
                ev_up.append(e)
        d2h = [0]

        def download(p, et):                                        # 3. exact-size downloads (D2H runs
            et.synchronize()                                        #    beside the remaining uploads)
            tot = p["host_tot"].numpy().copy()
            p["totals"] = tot
            self.down.wait_event(et)
            T = p["out"].tensors
            n = p["n"]
            with torch.cuda.stream(self.down):
                p["host_exec"].copy_(T["exec"][:n * abi.EXEC_ROW.itemsize], non_blocking=True)
                p["host_off"].copy_(T["cmp_offsets"], non_blocking=True)
                d2h[0] += n * abi.EXEC_ROW.itemsize + p["host_off"].numel() * 8
                for t, (name, dt, *_) in enumerate(abi.TABLES):
                    nb = int(tot[t]) * dt.itemsize
                    if nb:
                        p["host_rows"][name][:nb].copy_(T["cmp_" + name][:nb], non_blocking=True)
                        d2h[0] += nb

        queued = []                                                  # (part, totals event), not downloaded
        for i, (p, e) in enumerate(zip(self.parts, ev_up)):        # 2. ingest + replay + compaction
            s = self.comp[i % 2]
            s.wait_event(e)
            if i >= 2:                          # chunk i-2 ran on s: this plan's sync would wait for it anyway
                download(*queued.pop(0))
            S = p["ing"].plan(p["db"], s)                          # (synchronises s: the layout's sizes)
            out = p["out"]
            T = out.tensors
            with torch.cuda.stream(s):
                for k in ("exec", "scratch"):
                    T[k].zero_()
                for name, *_ in abi.TABLES:
                    T["out_" + name].zero_()
            p["ing"].layout(p["db"], S, s, out=out)
            eng.launch(out, s)
            eng.compact(out, s)
            n = p["n"]
            with torch.cuda.stream(s):
                p["host_tot"].copy_(T["cmp_offsets"].view(len(COMPACT_TABLES), n + 1)[:, n], non_blocking=True)
                et = torch.cuda.Event()
                et.record(s)
            queued.append((p, et))
        for item in queued:
            download(*item)
        self.down.synchronize()
        wall = time.perf_counter() - t0
        return {"wall_s": wall, "events": self.n_events, "events_per_s": self.n_events / wall,
                "h2d_bytes": self.h2d_bytes, "d2h_bytes": int(d2h[0]), "chunks": len(self.parts)}

    def h2d_peak(self, reps: int = 3) -> float:
        """The pinned host -> HBM copy rate of this pipeline's own uploads alone (one stream, no compute):
        the PCIe ceiling the blob -> rows figure is bound by, in GB/s (best of `reps`)."""
        torch, eng = self.torch, self.eng
        best = 0.0
        for _ in range(reps):
            torch.cuda.synchronize(eng.dev)
            t0 = time.perf_counter()
            with torch.cuda.stream(self.up):
                for p in self.parts:
                    for k, h in p["host"].items():
                        p["db"].tensors[k][:h.numel()].copy_(h, non_blocking=True)
            self.up.synchronize()
            best = max(best, self.h2d_bytes / (time.perf_counter() - t0) / 1e9)
        return best

    def results(self) -> List[CompactResult]:
        out = []
        for p in self.parts:
            n = p["n"]
            off = p["host_off"].numpy().reshape(len(COMPACT_TABLES), n + 1).copy()
            rows = {}
            for t, (name, dt, *_) in enumerate(abi.TABLES):
                rows[name] = p["host_rows"][name][:int(off[t, n]) * dt.itemsize].numpy().view(dt).copy()
            out.append(CompactResult(p["host_exec"].numpy().view(abi.EXEC_ROW).copy(), off, rows))
        return out

    def device_keys(self) -> List[np.ndarray]:
        """Per chunk, the digest identity keys in device order: each position's workflow index in the
        whole (unsplit) blob set -- the chunk's base plus the layout's perm."""
        from .dist import workflow_keys
        out, base = [], 0
        for p in self.parts:
            n = p["n"]
            perm = p["out"].tensors["perm"][:n].cpu().numpy().astype(np.int64)
            out.append(workflow_keys(base + perm))
            base += n
        return out

    def ev_counts(self) -> List[np.ndarray]:
        """Per chunk, the descriptors' ev_count in device order (for dist.digest_numpy)."""
        out = []
        for p in self.parts:
            n = p["n"]
            wf = p["out"].tensors["wf"][:n * abi.WORKFLOW.itemsize].cpu().numpy().view(abi.WORKFLOW)
            out.append(wf["ev_count"].copy())
        return out
