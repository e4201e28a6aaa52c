"""Device-side ingest: persisted thriftrw blobs in HBM -> the replay engine's layout, on the GPU.

Binds ``include/cadence_ingest.h`` (``crr_ingest_plan`` / ``crr_ingest_layout``,
``cadence_amd/csrc/ingest_kernel.hip``).  The host uploads the blobs as persistence returned them
(``common/persistence/serializer.go:109-119``: one thriftrw ``History`` per ApplyEvents batch) plus
the per-workflow host inputs; decoding, interning, capacities, the length / live-set ordering and the
wave interleave all run on the device, and the result is a ``DeviceBatch`` ``ReplayEngine.launch``
replays -- the same bytes the host path (``decode.decode_histories`` + ``flatten.interleave``) would
have uploaded.  No CPU fallback: the HIP library must be present.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional, Sequence

import numpy as np

from . import abi
from .blobs import BLOB_WF, KNOWN_DOMAINS, BlobSet
from .engine import DeviceBatch, ReplayEngine
from .flatten import HistoryBatch


class CBlobBatch(ctypes.Structure):
    _fields_ = [("bytes", ctypes.c_void_p), ("blob_off", ctypes.c_void_p), ("n_blobs", ctypes.c_uint32),
                ("n_wf", ctypes.c_uint32), ("wf", ctypes.c_void_p), ("strings", ctypes.c_void_p),
                ("domain_off", ctypes.c_void_p), ("domain_len", ctypes.c_void_p), ("n_domains", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


class CIngestSummary(ctypes.Structure):
    _fields_ = [("err", ctypes.c_int32), ("reserved0", ctypes.c_int32), ("err_blob", ctypes.c_int64),
                ("n_events", ctypes.c_uint64), ("n_slots", ctypes.c_uint64), ("n_act_side", ctypes.c_uint64),
                ("n_start_side", ctypes.c_uint64), ("n_reset_keys", ctypes.c_uint64), ("arena_bytes", ctypes.c_uint64),
                ("table_rows", ctypes.c_uint64 * 8), ("n_wf", ctypes.c_uint32), ("wave_begin", ctypes.c_uint32),
                ("tiers", ctypes.c_uint32 * 6), ("has_new_run", ctypes.c_uint32), ("lds_small_tail", ctypes.c_uint32)]


class CTranscodeSummary(ctypes.Structure):
    """crr_transcode_summary (cadence_ingest.h): what crr_ingest_transcode_plan reports."""
    _fields_ = [("err", ctypes.c_int32), ("reserved", ctypes.c_int32), ("err_blob", ctypes.c_int64),
                ("n_bytes", ctypes.c_uint64), ("n_deep", ctypes.c_uint32), ("reserved1", ctypes.c_uint32)]


class CIngestResume(ctypes.Structure):
    """crr_ingest_resume (cadence_ingest.h): the loaded states a resume ingest continues."""
    _fields_ = [("loaded_wf", ctypes.c_void_p), ("wave_begin", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("key_begin", ctypes.c_void_p), ("key_count", ctypes.c_void_p), ("key_off", ctypes.c_void_p),
                ("key_len", ctypes.c_void_p)]


SCRATCH_TOO_SMALL = -100
# CRR_INGEST_PAD (cadence_ingest.h): blob bytes readable this far past the last blob (the parser loads the
# two 16-byte-aligned words around its cursor)
INGEST_PAD = 32


class IngestError(RuntimeError):
    """A blob the decoder rejects (CadenceDeserializationError, serializer.go:320-333), or a bad call."""

    def __init__(self, code: int, blob: int):
        from .decode import ERRORS
        super().__init__(f"device ingest: {ERRORS.get(code, code)} (blob {blob})")
        self.code = code
        self.blob = blob


def _bind(L):
    if getattr(L, "_ingest_bound", False):
        return L
    vp = ctypes.c_void_p
    L.crr_ingest_scratch_bytes.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
    L.crr_ingest_scratch_bytes.restype = ctypes.c_size_t
    L.crr_ingest_plan.argtypes = [vp, vp, ctypes.c_size_t, vp, vp]
    L.crr_ingest_plan.restype = ctypes.c_int
    L.crr_ingest_layout.argtypes = [vp, vp, ctypes.c_size_t, vp, vp, vp, vp]
    L.crr_ingest_layout.restype = ctypes.c_int
    L.crr_ingest_plan_resume.argtypes = [vp, vp, vp, ctypes.c_size_t, vp, vp]
    L.crr_ingest_plan_resume.restype = ctypes.c_int
    L.crr_ingest_layout_resume.argtypes = [vp, vp, vp, ctypes.c_size_t, vp, vp, vp]
    L.crr_ingest_layout_resume.restype = ctypes.c_int
    L.crr_ingest_transcode_scratch_bytes.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
    L.crr_ingest_transcode_scratch_bytes.restype = ctypes.c_size_t
    L.crr_ingest_transcode_plan.argtypes = [vp, vp, vp, ctypes.c_size_t, vp, vp]
    L.crr_ingest_transcode_plan.restype = ctypes.c_int
    L.crr_ingest_transcode.argtypes = [vp, vp, vp, ctypes.c_size_t, vp, vp, vp, vp]
    L.crr_ingest_transcode.restype = ctypes.c_int
    L._ingest_bound = True
    return L


@dataclasses.dataclass
class DeviceBlobs:
    """A BlobSet resident in HBM (the upload of what persistence returned) and its C view.  `pending`: a
    rejection the transcode of its JSON blobs reported, (code, blob), raised by the plan unless the plan
    finds a failing blob of a lower index (the host decoder stops at the first failing blob)."""
    blobs: BlobSet
    tensors: dict
    c: CBlobBatch
    pending: Optional[tuple] = None


@dataclasses.dataclass
class _TranscodedShape:
    """What DeviceIngest.plan reads of a transcoded batch's BlobSet."""
    n_bytes: int
    n_blobs: int
    n_wf: int


class DeviceIngest:
    """Plans and lays out blob batches on one device."""

    def __init__(self, eng: ReplayEngine, known_domains: Optional[Sequence[str]] = KNOWN_DOMAINS):
        self.eng = eng
        self.torch = eng.torch
        self.lib = _bind(eng.lib)
        self.known = None if known_domains is None else [d.encode() for d in known_domains]
        self.scratch = None
        self.scratch_bytes = 0

    # -- upload --------------------------------------------------------------------------------------------
    def host_arrays(self, bs: BlobSet):
        """The host buffers one upload copies (the strings arena gains the known domain names)."""
        strings = bs.strings
        dom_off = dom_len = np.zeros(1, np.uint32)
        if self.known is not None and self.known:
            base = strings.size
            dom_len = np.array([len(d) for d in self.known], np.uint32)
            dom_off = (base + np.concatenate([[0], np.cumsum(dom_len)[:-1]])).astype(np.uint32)
            strings = np.concatenate([strings, np.frombuffer(b"".join(self.known), np.uint8)])
        return {"bytes": bs.bytes, "blob_off": bs.blob_off, "wf": bs.wf.view(np.uint8),
                "strings": strings, "domain_off": dom_off, "domain_len": dom_len}

    def upload(self, bs: BlobSet, host=None) -> DeviceBlobs:
        torch, dev = self.torch, self.eng.dev
        arrs = host if host is not None else self.host_arrays(bs)
        T = {}
        for k, a in arrs.items():
            raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
            t = torch.empty(max(raw.size, 1) + INGEST_PAD, dtype=torch.uint8, device=dev)   # window reads past the end
            if raw.size:
                t[:raw.size].copy_(torch.from_numpy(raw) if not isinstance(a, torch.Tensor) else a)
            T[k] = t
        return DeviceBlobs(bs, T, self._c_batch(bs, T))

    def _c_batch(self, bs: BlobSet, T) -> CBlobBatch:
        c = CBlobBatch()
        c.bytes = T["bytes"].data_ptr()
        c.blob_off = T["blob_off"].data_ptr()
        c.n_blobs = bs.n_blobs
        c.n_wf = bs.n_wf
        c.wf = T["wf"].data_ptr()
        c.strings = T["strings"].data_ptr()
        c.domain_off = T["domain_off"].data_ptr()
        c.domain_len = T["domain_len"].data_ptr()
        c.n_domains = 0xFFFFFFFF if self.known is None else len(self.known)
        return c

    # -- JSON-encoded blobs: rewritten as thriftrw on the device ---------------------------------------------
    def transcode(self, db: DeviceBlobs, encodings, stream=None, stage_bytes: Optional[int] = None) -> DeviceBlobs:
        """crr_ingest_transcode_plan + crr_ingest_transcode: the batch with every json / unknown / empty-encoded
        blob rewritten in HBM as the thriftrw History the decoders read back into the same events
        (``encodings``: CRR_ENCODING_* per blob, a uint32 array or device tensor).  A rejected blob (BAD_JSON,
        UNKNOWN_ENCODING) becomes empty and is carried as ``pending`` for the plan to raise.  ``stage_bytes``:
        the blob bytes the scratch's staging area is sized for (default all of them; less: the blobs without
        room are walked again by the transcode)."""
        torch, dev = self.torch, self.eng.dev
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        L = self.lib
        nb = int(db.c.n_blobs)
        if isinstance(encodings, torch.Tensor):
            enc = encodings
        else:
            enc = torch.from_numpy(np.ascontiguousarray(encodings, np.uint32).view(np.int32)).to(dev)
        need = int(L.crr_ingest_transcode_scratch_bytes(nb, int(db.blobs.n_bytes if stage_bytes is None else stage_bytes)))
        if getattr(self, "tscratch", None) is None or self.tscratch.numel() < need:
            self.tscratch = torch.empty(need, dtype=torch.uint8, device=dev)
        size = need if stage_bytes is not None else self.tscratch.numel()
        S = CTranscodeSummary()
        vp = ctypes.c_void_p
        rc = L.crr_ingest_transcode_plan(ctypes.byref(db.c), vp(enc.data_ptr()), vp(self.tscratch.data_ptr()),
                                         ctypes.c_size_t(size), ctypes.byref(S), vp(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"crr_ingest_transcode_plan failed: {rc}")
        n_bytes = int(S.n_bytes)
        out_bytes = torch.empty(n_bytes + INGEST_PAD + 16, dtype=torch.uint8, device=dev)
        out_off = torch.empty(nb + 1, dtype=torch.int64, device=dev)
        rc = L.crr_ingest_transcode(ctypes.byref(db.c), vp(enc.data_ptr()), vp(self.tscratch.data_ptr()),
                                    ctypes.c_size_t(size), ctypes.byref(S), vp(out_bytes.data_ptr()),
                                    vp(out_off.data_ptr()), vp(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"crr_ingest_transcode failed: {rc}")
        T = dict(db.tensors)
        T["bytes"], T["blob_off"], T["encodings"] = out_bytes, out_off, enc
        c = CBlobBatch.from_buffer_copy(db.c)
        c.bytes, c.blob_off = out_bytes.data_ptr(), out_off.data_ptr()
        self.last_transcode = S
        pending = (int(S.err), int(S.err_blob)) if S.err else None
        return DeviceBlobs(_TranscodedShape(n_bytes, nb, int(db.c.n_wf)), T, c, pending)

    def transcoded_blobs(self, tdb: DeviceBlobs) -> BlobSet:
        """Download a transcoded batch as a host BlobSet (tests: the host decoder reads it back)."""
        self.torch.cuda.synchronize(self.eng.dev)
        off = tdb.tensors["blob_off"].cpu().numpy().view(np.uint64).copy()
        n = int(off[-1])
        data = np.zeros(n + INGEST_PAD, np.uint8)
        data[:n] = tdb.tensors["bytes"][:n].cpu().numpy()
        wf = tdb.tensors["wf"][:tdb.blobs.n_wf * BLOB_WF.itemsize].cpu().numpy().view(BLOB_WF).copy()
        return BlobSet(bytes=data, blob_off=off, wf=wf, strings=tdb.tensors["strings"].cpu().numpy().copy())

    # -- plan + layout ---------------------------------------------------------------------------------------
    def ensure_scratch(self, db: DeviceBlobs, max_events: int):
        need = int(self.lib.crr_ingest_scratch_bytes(db.c.n_blobs, db.c.n_wf, max_events))
        if self.scratch is None or self.scratch_bytes < need:
            self.scratch = self.torch.empty(need, dtype=self.torch.uint8, device=self.eng.dev)
            self.scratch_bytes = need
        return self.scratch_bytes

    def plan(self, db: DeviceBlobs, stream=None, max_events: Optional[int] = None,
             resume: Optional[CIngestResume] = None) -> CIngestSummary:
        """crr_ingest_plan (grows the scratch and plans again if the blobs hold more events than it fits);
        with ``resume``, crr_ingest_plan_resume (new batches onto the loaded states it names)."""
        torch = self.torch
        s = stream if stream is not None else torch.cuda.current_stream(self.eng.dev)
        cap = max_events if max_events is not None else max(4096, db.blobs.n_bytes // 40)
        while True:
            size = self.ensure_scratch(db, cap)
            S = CIngestSummary()
            if resume is None:
                rc = self.lib.crr_ingest_plan(ctypes.byref(db.c), ctypes.c_void_p(self.scratch.data_ptr()),
                                              ctypes.c_size_t(size), ctypes.byref(S), ctypes.c_void_p(s.cuda_stream))
            else:
                rc = self.lib.crr_ingest_plan_resume(ctypes.byref(db.c), ctypes.byref(resume),
                                                     ctypes.c_void_p(self.scratch.data_ptr()), ctypes.c_size_t(size),
                                                     ctypes.byref(S), ctypes.c_void_p(s.cuda_stream))
            if rc != 0:
                raise RuntimeError(f"crr_ingest_plan failed: {rc}")
            if S.err == SCRATCH_TOO_SMALL:
                cap = max(2 * cap, int(S.n_events) + 1)
                continue
            if S.err and (db.pending is None or int(S.err_blob) < db.pending[1]):
                raise IngestError(int(S.err), int(S.err_blob))
            if db.pending is not None:
                raise IngestError(*db.pending)
            return S

    def layout(self, db: DeviceBlobs, S: CIngestSummary, stream=None, emit_tasks: bool = False,
               out: Optional[DeviceBatch] = None) -> DeviceBatch:
        """crr_ingest_layout into fresh device buffers (or `out`'s, when their sizes match) and the
        output rows; returns a DeviceBatch ReplayEngine.launch replays."""
        torch, dev = self.torch, self.eng.dev
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        if out is None:
            out = self.allocate(S, emit_tasks)
        T = out.tensors
        ci = out.c_in
        perm = T["perm"]
        rc = self.lib.crr_ingest_layout(ctypes.byref(db.c), ctypes.c_void_p(self.scratch.data_ptr()),
                                        ctypes.c_size_t(self.scratch_bytes), ctypes.byref(S), ctypes.byref(ci),
                                        ctypes.c_void_p(perm.data_ptr()), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"crr_ingest_layout failed: {rc}")
        return out

    def layout_resume(self, db: DeviceBlobs, resume: CIngestResume, S: CIngestSummary, ci: abi.CInputs,
                      stream=None):
        """crr_ingest_layout_resume into the inputs ``ci`` points at (sized from ``S`` by ``allocate_inputs``):
        the new events' columns, side records, reset keys and the loaded descriptors continued."""
        s = stream if stream is not None else self.torch.cuda.current_stream(self.eng.dev)
        rc = self.lib.crr_ingest_layout_resume(ctypes.byref(db.c), ctypes.byref(resume),
                                               ctypes.c_void_p(self.scratch.data_ptr()),
                                               ctypes.c_size_t(self.scratch_bytes), ctypes.byref(S), ctypes.byref(ci),
                                               ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"crr_ingest_layout_resume failed: {rc}")

    def allocate_inputs(self, S: CIngestSummary, T: dict, ci: abi.CInputs, slack: float = 1.0, wf_in_place=None):
        """(Re)allocate the event columns, side records, reset keys and descriptors a resume layout writes
        into ``T`` (``slack`` x the summary's sizes, reused while large enough) and point ``ci`` at them;
        ``wf_in_place``: a device tensor of the loaded descriptors the layout updates in place instead."""
        torch, dev = self.torch, self.eng.dev
        need = {"ev_" + name: max(int(S.n_slots), 1) * np.dtype(t).itemsize + 16 for name, t in abi.EVENT_COLUMNS}
        need.update({"act_side": int(S.n_act_side) * abi.ACTIVITY_SIDE.itemsize + 16,
                     "start_side": int(S.n_start_side) * abi.START_SIDE.itemsize + 16,
                     "reset_keys": max(int(S.n_reset_keys), 1) * 4 + 16,
                     "wf": max(int(S.n_wf), 1) * abi.WORKFLOW.itemsize + 16})
        for k, nb in need.items():
            if k not in T or T[k].numel() < nb:
                T[k] = torch.zeros(int(nb * slack) + 16, dtype=torch.uint8, device=dev)
        for name, _t in abi.EVENT_COLUMNS:
            setattr(ci.ev, name, T["ev_" + name].data_ptr())
        for k in ("act_side", "start_side", "reset_keys", "wf"):
            setattr(ci, k, T[k].data_ptr())
        if wf_in_place is not None:
            ci.wf = wf_in_place.data_ptr()

    @staticmethod
    def input_shapes(S: CIngestSummary):
        return {"ev_slots": int(S.n_slots), "act_side": int(S.n_act_side), "start_side": int(S.n_start_side),
                "reset_keys": max(int(S.n_reset_keys), 1), "arena": int(S.arena_bytes)}

    def allocate(self, S: CIngestSummary, emit_tasks: bool = False) -> DeviceBatch:
        """Device input / output buffers for a plan's summary, and the C structs over them."""
        torch, dev = self.torch, self.eng.dev
        n = int(S.n_wf)
        T = {}
        ev = abi.CEvents()
        slots = int(S.n_slots)
        for name, t in abi.EVENT_COLUMNS:
            T["ev_" + name] = torch.empty(max(slots, 1) * np.dtype(t).itemsize + 16, dtype=torch.uint8, device=dev)
            setattr(ev, name, T["ev_" + name].data_ptr())
        ci = abi.CInputs()
        ci.ev = ev
        for field, nb in (("act_side", int(S.n_act_side) * abi.ACTIVITY_SIDE.itemsize),
                          ("start_side", int(S.n_start_side) * abi.START_SIDE.itemsize),
                          ("reset_keys", max(int(S.n_reset_keys), 1) * 4),
                          ("arena", int(S.arena_bytes) + 16),
                          ("wf", max(n, 1) * abi.WORKFLOW.itemsize)):
            T[field] = torch.zeros(max(nb, 1) + 16, dtype=torch.uint8, device=dev)
            setattr(ci, field, T[field].data_ptr())
        T["perm"] = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        ci.n_wf = n
        ci.stride = 64
        ci.wave_begin = int(S.wave_begin)
        (ci.large_begin, ci.compact_begin, ci.compact2_begin, ci.wide_begin, ci.hbm_begin, ci.big_begin) = \
            tuple(int(x) for x in S.tiers)
        # the layout joins each ActivityTaskStarted to its scheduled event's side record (CRR_IN_STARTED_AUX)
        ci.flags = (abi.IN_WAVE_TAIL | abi.IN_TIERED | abi.IN_STARTED_AUX | (abi.IN_HAS_NEW_RUN if S.has_new_run else 0)
                    | (abi.IN_LDS_SMALL if S.lds_small_tail else 0) | (abi.IN_EMIT_TASKS if emit_tasks else 0))
        co = abi.COutputs()
        T["exec"] = torch.zeros(max(n, 1) * abi.EXEC_ROW.itemsize, dtype=torch.uint8, device=dev)
        co.exec = T["exec"].data_ptr()
        table_rows = {}
        for j, (name, dt, *_r) in enumerate(abi.TABLES):
            rows = max(int(S.table_rows[j]), 1)
            table_rows[name] = int(S.table_rows[j])
            if name == "tasks" and not emit_tasks:
                rows = 1
            T["out_" + name] = torch.zeros(rows * dt.itemsize, dtype=torch.uint8, device=dev)
            setattr(co, name, T["out_" + name].data_ptr())
        T["scratch"] = torch.zeros(2 * n + abi.SCRATCH_EXTRA_WORDS, dtype=torch.int32, device=dev)
        co.scratch = T["scratch"].data_ptr()
        shell = _ShellBatch(n, emit_tasks, table_rows, int(S.wave_begin), tuple(int(x) for x in S.tiers),
                            self.input_shapes(S))
        return DeviceBatch(shell, T, ci, co, self.eng.device)

    def ingest(self, db: DeviceBlobs, stream=None, emit_tasks: bool = False) -> DeviceBatch:
        return self.layout(db, self.plan(db, stream), stream, emit_tasks)

    # -- inspection (tests) ---------------------------------------------------------------------------------
    def to_host_batch(self, out: DeviceBatch) -> HistoryBatch:
        """Download the laid-out inputs as a HistoryBatch (the host path's interleaved batch, for parity)."""
        self.torch.cuda.synchronize(self.eng.dev)
        T = out.tensors
        sh = out.batch
        n, shp = sh.n_wf, sh.shapes

        def host(key, count, dtype):
            it = np.dtype(dtype).itemsize
            return T[key][:count * it].cpu().numpy().view(dtype).copy()

        cols = {name: host("ev_" + name, shp["ev_slots"], t) for name, t in abi.EVENT_COLUMNS}
        b = HistoryBatch(cols=cols, act_side=host("act_side", shp["act_side"], abi.ACTIVITY_SIDE),
                         start_side=host("start_side", shp["start_side"], abi.START_SIDE),
                         reset_keys=host("reset_keys", shp["reset_keys"], np.uint32),
                         arena=host("arena", shp["arena"], np.uint8), wf=host("wf", n, abi.WORKFLOW), stride=64,
                         wave_begin=int(out.c_in.wave_begin), tiers=sh.tiers, emit_tasks=sh.emit_tasks,
                         perm=T["perm"][:n].cpu().numpy().astype(np.int64))
        b.table_rows = dict(sh.table_rows)
        return b


@dataclasses.dataclass
class _ShellBatch:
    """What DeviceBatch users read of its HistoryBatch when the inputs were laid out on the device."""
    _n_wf: int
    emit_tasks: bool
    table_rows: dict
    wave_begin: int
    tiers: tuple
    shapes: dict

    @property
    def n_wf(self) -> int:
        return self._n_wf
