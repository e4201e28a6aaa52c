"""Device engine: binds ``libcadence_replay.so`` (the C ABI) and manages HBM-resident batches.

PyTorch is used only as plumbing (device allocation, streams, copies).  There is no CPU fallback:
if the HIP library is missing or no GPU is visible the engine raises.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
from typing import Dict, Optional

import numpy as np

from . import abi
from .flatten import HistoryBatch, fits_small_tier
from .result import ReplayResult

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CRR_LIB_PATH") or os.path.join(_HERE, "libcadence_replay.so")
_lib = None


class EngineUnavailable(RuntimeError):
    pass


def lib():
    """Load the HIP library (raises EngineUnavailable when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EngineUnavailable(f"{LIB_PATH} not built: run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.crr_replay.argtypes = [vp, vp, vp]
        L.crr_replay.restype = ctypes.c_int
        L.crr_checksum.argtypes = [vp, vp, vp, vp]
        L.crr_checksum.restype = ctypes.c_int
        L.crr_token_crc.argtypes = [vp, vp, vp]
        L.crr_token_crc.restype = ctypes.c_int
        L.crr_set_device.argtypes = [ctypes.c_int]
        L.crr_set_device.restype = ctypes.c_int
        L.crr_release.restype = ctypes.c_int
        L.crr_abi_version.restype = ctypes.c_int
        L.crr_crc32_ieee.argtypes = [vp, ctypes.c_size_t]
        L.crr_crc32_ieee.restype = ctypes.c_uint32
        L.crr_last_kernel_ms.argtypes = [ctypes.c_int]
        L.crr_last_kernel_ms.restype = ctypes.c_float
        L.crr_ndc_prepare.argtypes = [vp, vp, vp, vp]
        L.crr_ndc_prepare.restype = ctypes.c_int
        L.crr_timing_begin.restype = ctypes.c_int
        L.crr_timing_read.argtypes = [vp, ctypes.c_int]
        L.crr_timing_read.restype = ctypes.c_int
        L.crr_compact_rows.argtypes = [vp, vp, vp, vp]
        L.crr_compact_rows.restype = ctypes.c_int
        L.crr_compact_scratch_bytes.argtypes = [ctypes.c_uint32]
        L.crr_compact_scratch_bytes.restype = ctypes.c_size_t
        L.crr_widen_events.argtypes = [vp, vp, vp]
        L.crr_widen_events.restype = ctypes.c_int
        if L.crr_abi_version() != abi.ABI_VERSION:
            raise EngineUnavailable("ABI version mismatch")
        abi.check_layout(L)
        _lib = L
    return _lib


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise EngineUnavailable("no HIP device visible (torch.cuda.is_available() is False)")
    return torch


@dataclasses.dataclass
class DeviceBatch:
    """A HistoryBatch resident in HBM plus its output buffers."""
    batch: HistoryBatch
    tensors: Dict[str, object]
    c_in: abi.CInputs
    c_out: abi.COutputs
    device: int
    c_compact: Optional[object] = None
    c_packed: Optional[object] = None

    @property
    def n_wf(self):
        return self.batch.n_wf


def _dev_bytes(torch, arr: np.ndarray, device, pad: int = 16):
    """Copy a numpy array to a uint8 device tensor (padded so empty arrays still get an address)."""
    raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
    t = torch.empty(max(raw.size, 1) + pad, dtype=torch.uint8, device=device)
    if raw.size:
        t[:raw.size].copy_(torch.from_numpy(raw), non_blocking=False)
    return t


class ReplayEngine:
    """Batched ``StateBuilder.ApplyEvents`` on one MI355X (one process per GPU)."""

    def __init__(self, device: int = 0):
        self.torch = _torch()
        self.device = device
        self.lib = lib()
        rc = self.lib.crr_set_device(device)
        if rc != 0:
            raise EngineUnavailable(f"crr_set_device({device}) failed: {rc}")
        self.dev = self.torch.device("cuda", device)

    # -- upload ------------------------------------------------------------------------------------
    def upload(self, batch: HistoryBatch, live_ids: bool = True, token_crc: bool = True) -> DeviceBatch:
        torch = self.torch
        dev = self.dev
        T = {}
        ev = abi.CEvents()
        for name, t in abi.EVENT_COLUMNS:
            T["ev_" + name] = _dev_bytes(torch, np.asarray(batch.cols[name], dtype=t), dev)
            setattr(ev, name, T["ev_" + name].data_ptr())
        ci = abi.CInputs()
        ci.ev = ev
        # the device reads branch tokens as 8-byte words: keep the arena 8-byte padded
        arena = np.concatenate([batch.arena, np.zeros(16, np.uint8)])
        for field, arr in (("act_side", batch.act_side), ("start_side", batch.start_side),
                           ("reset_keys", batch.reset_keys), ("arena", arena), ("wf", batch.wf)):
            T[field] = _dev_bytes(torch, arr, dev)
            setattr(ci, field, T[field].data_ptr())
        ci.n_wf = batch.n_wf
        ci.stride = batch.stride
        has_new_run = bool((batch.wf["flags"] & abi.WF_FLAG_NEW_RUN).any()) if batch.n_wf else False
        ci.flags = (abi.IN_HAS_NEW_RUN if has_new_run else 0) | batch.c_flags()
        ci.wave_begin = batch.wave_begin or 0
        ci.big_begin = batch.n_wf
        if batch.tiers is not None:
            # segments by expected live-set size; LDS_SMALL then only places the wave tail
            (ci.large_begin, ci.compact_begin, ci.compact2_begin, ci.wide_begin, ci.hbm_begin,
             ci.big_begin) = batch.tiers
            if fits_small_tier(batch, lanes=False):
                ci.flags |= abi.IN_LDS_SMALL
        elif batch.stride == 64 and fits_small_tier(batch):
            ci.flags |= abi.IN_LDS_SMALL
        co = abi.COutputs()
        init_host = None
        if batch.init is not None:   # loaded states (CRR_WF_FLAG_RESUME): the rows the replay continues in place
            from .result import allocate_host
            init_host = allocate_host(batch)
        T["exec"] = torch.zeros(max(batch.n_wf, 1) * abi.EXEC_ROW.itemsize, dtype=torch.uint8, device=dev)
        if init_host is not None and batch.n_wf:
            T["exec"][:batch.n_wf * abi.EXEC_ROW.itemsize].copy_(torch.from_numpy(init_host.exec.view(np.uint8)))
        co.exec = T["exec"].data_ptr()
        for name, dt, *_ in abi.TABLES:
            rows = max(batch.table_rows.get(name, 0), 1)
            if name == "tasks" and not batch.emit_tasks:
                rows = 1   # not written without CRR_IN_EMIT_TASKS
            T["out_" + name] = torch.zeros(rows * dt.itemsize, dtype=torch.uint8, device=dev)
            if init_host is not None and name != "tasks":
                src = init_host.tables[name].view(np.uint8).reshape(-1)
                T["out_" + name][:src.size].copy_(torch.from_numpy(src))
            setattr(co, name, T["out_" + name].data_ptr())
        T["scratch"] = torch.zeros(2 * batch.n_wf + abi.SCRATCH_EXTRA_WORDS, dtype=torch.int32, device=dev)
        co.scratch = T["scratch"].data_ptr()
        if live_ids:
            # the live-ID sidecar (crr_outputs.live_ids): one int64 per row slot of each pending map, written by the
            # replay for every OK workflow and read by crr_checksum instead of the rows
            for t, name in enumerate(abi.ID_TABLES):
                T["ids_" + name] = torch.zeros(max(batch.table_rows.get(name, 0), 1), dtype=torch.int64, device=dev)
                co.live_ids[t] = T["ids_" + name].data_ptr()
        if token_crc and batch.n_wf:
            # crr_inputs.token_crc: each start token's raw CRC, computed once the arena is in HBM (a token is
            # fixed for its branch); the replay splices it into the checksum instead of hashing the token
            T["token_crc"] = torch.zeros(batch.n_wf, dtype=torch.int32, device=dev)
            ci.token_crc = T["token_crc"].data_ptr()
            s = torch.cuda.current_stream(dev)
            if self.lib.crr_token_crc(ctypes.byref(ci), ctypes.c_void_p(ci.token_crc), ctypes.c_void_p(s.cuda_stream)) != 0:
                raise RuntimeError("crr_token_crc failed")
        return DeviceBatch(batch, T, ci, co, self.device)

    # -- the fused digest (crr_outputs.digest) -------------------------------------------------------
    def enable_digest(self, db: DeviceBatch, keys: np.ndarray):
        """Every later crr_replay of ``db`` also writes its digest (dist.DIGEST_FIELDS, as stripes of partial
        sums) into ``db.tensors["digest"]``; ``keys``: each device position's identity key (dist.device_keys)."""
        torch = self.torch
        k = np.ascontiguousarray(np.asarray(keys, np.int64)[: db.n_wf])
        if k.size != db.n_wf:
            raise ValueError("one digest key per workflow")
        db.tensors["digest_keys"] = torch.from_numpy(k.copy()).to(self.dev)
        db.tensors["digest"] = torch.zeros(abi.DIGEST_WORDS, dtype=torch.int64, device=self.dev)
        db.c_in.digest_keys = db.tensors["digest_keys"].data_ptr()
        db.c_out.digest = db.tensors["digest"].data_ptr()

    def read_digest(self, db: DeviceBatch) -> np.ndarray:
        """The last launch's digest, int64[7] (its stripes summed, mod 2^64)."""
        self.torch.cuda.synchronize(self.dev)
        return fold_digest(db.tensors["digest"].cpu().numpy())

    # -- launch ------------------------------------------------------------------------------------
    def launch(self, db: DeviceBatch, stream=None):
        """Enqueue crr_replay on ``stream`` (torch stream; default: current stream)."""
        torch = self.torch
        s = stream if stream is not None else torch.cuda.current_stream(self.dev)
        rc = self.lib.crr_replay(ctypes.byref(db.c_in), ctypes.byref(db.c_out), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"crr_replay failed: {rc}")

    def last_kernel_ms(self):
        """[phase 0, phase 1 (all kernels), phase-1 fast-path kernel alone] in ms (-1: not run)."""
        return [self.lib.crr_last_kernel_ms(i) for i in range(3)]

    def timing_begin(self):
        """Start recording the fast-path kernel of every launch (HIP events on the launch stream)."""
        if self.lib.crr_timing_begin() != 0:
            raise RuntimeError("crr_timing_begin failed")

    def timing_read(self):
        """End the measured region; per-launch fast-path kernel durations in ms."""
        buf = (ctypes.c_float * 512)()
        n = self.lib.crr_timing_read(buf, 512)
        if n < 0:
            raise RuntimeError("crr_timing_read failed")
        return list(buf[:n])

    def checksum(self, db: DeviceBatch, stream=None) -> np.ndarray:
        """Recompute checksums of the replayed rows on the device (Load verify path)."""
        torch = self.torch
        s = stream if stream is not None else torch.cuda.current_stream(self.dev)
        out = torch.zeros(max(db.n_wf, 1), dtype=torch.int32, device=self.dev)
        rc = self.lib.crr_checksum(ctypes.byref(db.c_in), ctypes.byref(db.c_out), ctypes.c_void_p(out.data_ptr()),
                                   ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"crr_checksum failed: {rc}")
        torch.cuda.synchronize(self.dev)
        return out.cpu().numpy().view(np.uint32)[:db.n_wf]

    # -- download ----------------------------------------------------------------------------------
    def download(self, db: DeviceBatch) -> ReplayResult:
        self.torch.cuda.synchronize(self.dev)
        T = db.tensors
        ex = T["exec"].cpu().numpy().view(abi.EXEC_ROW)[:db.n_wf].copy()
        tables = {}
        for name, dt, *_ in abi.TABLES:
            tables[name] = T["out_" + name].cpu().numpy().view(dt)   # .cpu() is already a fresh host copy
        return ReplayResult(ex, tables)

    # -- compacted download --------------------------------------------------------------------------
    def compact(self, db: DeviceBatch, stream=None):
        """Enqueue crr_compact_rows after the replay (same stream): dense live rows on the device."""
        torch = self.torch
        s = stream if stream is not None else torch.cuda.current_stream(self.dev)
        T = db.tensors
        if "cmp_offsets" not in T:
            for name, dt, *_ in abi.TABLES:
                rows = max(db.batch.table_rows.get(name, 0), 1) if (name != "tasks" or db.batch.emit_tasks) else 1
                T["cmp_" + name] = torch.empty(rows * dt.itemsize, dtype=torch.uint8, device=self.dev)
            T["cmp_offsets"] = torch.empty(len(COMPACT_TABLES) * (db.n_wf + 1), dtype=torch.int64, device=self.dev)
            T["cmp_scratch"] = torch.empty(int(self.lib.crr_compact_scratch_bytes(db.n_wf)), dtype=torch.uint8,
                                           device=self.dev)
            co = CCompactOut()
            for i, name in enumerate(COMPACT_TABLES):
                co.rows[i] = T["cmp_" + name].data_ptr()
            co.offsets = T["cmp_offsets"].data_ptr()
            co.scratch = T["cmp_scratch"].data_ptr()
            db.c_compact = co
        rc = self.lib.crr_compact_rows(ctypes.byref(db.c_in), ctypes.byref(db.c_out), ctypes.byref(db.c_compact),
                                       ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"crr_compact_rows failed: {rc}")

    def download_compact(self, db: DeviceBatch) -> CompactResult:
        """Synchronise and copy the exec rows and the compacted live rows (exact sizes) to the host."""
        self.torch.cuda.synchronize(self.dev)
        T = db.tensors
        n = db.n_wf
        off = T["cmp_offsets"].cpu().numpy().reshape(len(COMPACT_TABLES), n + 1)
        ex = T["exec"][:n * abi.EXEC_ROW.itemsize].cpu().numpy().view(abi.EXEC_ROW).copy()
        rows = {}
        for t, (name, dt, *_) in enumerate(abi.TABLES):
            tot = int(off[t, n])
            rows[name] = T["cmp_" + name][:tot * dt.itemsize].cpu().numpy().view(dt)
        return CompactResult(ex, off, rows)

    # -- narrow upload format (wire.py) --------------------------------------------------------------
    def attach_packed(self, db: DeviceBatch, pk) -> object:
        """Device buffers for a batch's packed columns and the crr_packed_events struct over them
        (filled by the caller's copies); returns the struct."""
        from .wire import COLUMNS, CPackedEvents
        torch = self.torch
        T = db.tensors
        cp = CPackedEvents()
        for c in COLUMNS:
            a = pk.data[c]
            T["pk_" + c] = torch.empty(max(a.size, 1) + 16, dtype=torch.uint8, device=self.dev)
            col = getattr(cp, c)
            col.data = T["pk_" + c].data_ptr()
            col.width = pk.width[c]
            col.kind = pk.kind[c]
        T["pk_ts_base"] = torch.empty(max(pk.ts_base.size, 1), dtype=torch.int64, device=self.dev)
        cp.ts_base = T["pk_ts_base"].data_ptr()
        db.c_packed = cp
        return cp

    def widen(self, db: DeviceBatch, stream=None):
        """Enqueue crr_widen_events: the packed columns -> the batch's event columns in HBM."""
        s = stream if stream is not None else self.torch.cuda.current_stream(self.dev)
        rc = self.lib.crr_widen_events(ctypes.byref(db.c_packed), ctypes.byref(db.c_in), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"crr_widen_events failed: {rc}")

    def replay(self, batch: HistoryBatch) -> ReplayResult:
        db = self.upload(batch)
        self.launch(db)
        return self.download(db)


def fold_digest(raw: np.ndarray) -> np.ndarray:
    """crr_outputs.digest (CRR_DIGEST_WORDS int64: stripes of partial sums) -> the digest, int64[7]."""
    st = np.asarray(raw, np.int64).reshape(abi.DIGEST_STRIPES, abi.DIGEST_STRIDE)[:, :abi.DIGEST_FIELDS]
    with np.errstate(over="ignore"):
        return st.sum(axis=0, dtype=np.int64)


COMPACT_TABLES = [t[0] for t in abi.TABLES]   # crr_compact_out.rows order


class CCompactOut(ctypes.Structure):
    _fields_ = [("rows", ctypes.c_void_p * len(COMPACT_TABLES)), ("offsets", ctypes.c_void_p), ("scratch", ctypes.c_void_p)]


@dataclasses.dataclass
class CompactResult:
    """A replay's persisted output as downloaded by ``crr_compact_rows``: the exec rows and every
    workflow's live rows, dense per table (batch order), with per-table exclusive prefixes."""
    exec: np.ndarray                 # abi.EXEC_ROW [n_wf]
    offsets: np.ndarray              # int64 [len(COMPACT_TABLES), n_wf + 1]
    rows: Dict[str, np.ndarray]

    def to_replay_result(self, batch: HistoryBatch) -> ReplayResult:
        """Scatter the live rows back into the batch's slot-table layout (host side, for comparisons
        with ``diff_results``; slots past a workflow's count stay zero)."""
        from .result import allocate_host
        res = allocate_host(batch)
        res.exec[:] = self.exec
        st = batch.wf_strides()
        for t, (name, _dt, base_f, _c, _n) in enumerate(abi.TABLES):
            off = self.offsets[t]
            c = np.diff(off)
            tot = int(off[-1])
            if tot == 0 or name not in self.rows:
                continue
            wf_idx = np.repeat(np.arange(batch.n_wf), c)
            slot = np.arange(tot) - np.repeat(off[:-1], c)
            res.tables[name][batch.wf[base_f].astype(np.int64)[wf_idx] + slot * st[wf_idx]] = self.rows[name][:tot]
        return res


def crc32(data: bytes) -> int:
    """hash/crc32.ChecksumIEEE via the library's host helper."""
    a = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    return int(lib().crr_crc32_ieee(a.ctypes.data_as(ctypes.c_void_p), len(data)))
