"""Persisted history blobs at full size: a canonical HistoryBatch -> thriftrw blobs, natively.

Binds ``crr_encode_blobs`` (``cadence_amd/csrc/blob_encode.cpp``, libcadence_host.so): the
``thrift_codec.serialize_history`` encoding (``SerializeBatchEvents``, ``common/persistence/
serializer.go:105-107``) over the engine's columns, threaded, so the 1M-workflow workloads can be
persisted for the blob -> rows benchmark.  Benchmark / test infrastructure: synthetic data.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import List

import numpy as np

from . import abi, decode
from .flatten import HistoryBatch

# include/cadence_ingest.h crr_blob_wf (80 B)
BLOB_WF = np.dtype([("blob_begin", "<u4"), ("blob_count", "<u4"), ("init_version", "<i8"), ("now_ns", "<i8"),
                    ("run_id_off", "<u4"), ("run_id_len", "<u4"), ("branch_id_off", "<u4"), ("branch_id_len", "<u4"),
                    ("final_token_off", "<u4"), ("final_token_len", "<u4"), ("rebuild_last_event_id", "<i8"),
                    ("rebuild_last_event_version", "<i8"), ("new_run_wf", "<i4"), ("flags", "<i4"),
                    ("retention_days", "<i4"), ("reserved", "<i4")])
assert BLOB_WF.itemsize == 80

KNOWN_DOMAINS = ("domain-a", "domain-b", "parent-domain")   # what the encoder's names resolve against


@dataclasses.dataclass
class BlobSet:
    """Persisted batches of a set of workflows, laid out for upload: every blob concatenated (16-byte
    padded past the end), blob offsets, per-workflow ranges and host inputs, a string arena."""
    bytes: np.ndarray          # uint8 [n_bytes + 32]
    blob_off: np.ndarray       # uint64 [n_blobs + 1]
    wf: np.ndarray             # BLOB_WF [n_wf]
    strings: np.ndarray        # uint8

    @property
    def n_wf(self) -> int:
        return int(self.wf.shape[0])

    @property
    def n_blobs(self) -> int:
        return int(self.blob_off.shape[0] - 1)

    @property
    def n_bytes(self) -> int:
        return int(self.blob_off[-1])

    def blob(self, i: int) -> bytes:
        return self.bytes[int(self.blob_off[i]):int(self.blob_off[i + 1])].tobytes()

    def to_sources(self) -> List[decode.WorkflowSource]:
        """The same workflows as host-decoder inputs (decode.decode_histories)."""
        out = []
        st = self.strings.tobytes()
        for r in self.wf:
            b0, n = int(r["blob_begin"]), int(r["blob_count"])
            ft = None
            if int(r["final_token_len"]) != abi.NO_TOKEN:
                o = int(r["final_token_off"])
                ft = st[o:o + int(r["final_token_len"])]
            run = st[int(r["run_id_off"]):int(r["run_id_off"]) + int(r["run_id_len"])].decode()
            br = st[int(r["branch_id_off"]):int(r["branch_id_off"]) + int(r["branch_id_len"])].decode()
            out.append(decode.WorkflowSource(
                blobs=[self.blob(b0 + i) for i in range(n)], run_id=run, branch_id=br,
                domain_failover_version=int(r["init_version"]), now_ns=int(r["now_ns"]), final_token=ft,
                rebuild_last_event_id=int(r["rebuild_last_event_id"]),
                rebuild_last_event_version=int(r["rebuild_last_event_version"]),
                new_run=None if int(r["new_run_wf"]) < 0 else int(r["new_run_wf"]),
                is_new_run=bool(int(r["flags"]) & abi.WF_FLAG_NEW_RUN),
                refresh_tasks=bool(int(r["flags"]) & abi.WF_FLAG_REFRESH_TASKS),
                retention_days=int(r["retention_days"])))
        return out


def blobset_from_sources(sources: List[decode.WorkflowSource]):
    """Host-decoder inputs (blobs of any encoding, as persistence returned them) laid out for the device
    ingest: the BlobSet (to_sources' inverse) and each blob's CRR_ENCODING_* (uint32; an encoding name
    the serializer does not know maps to 0xFF, NewUnknownEncodingTypeError)."""
    blobs, encs, strings = [], [], bytearray()
    wf = np.zeros(len(sources), BLOB_WF)

    def put(b: bytes):
        strings.extend(b)
        return len(strings) - len(b), len(b)

    for w, s in enumerate(sources):
        r = wf[w]
        r["blob_begin"], r["blob_count"] = len(blobs), len(s.blobs)
        blobs.extend(s.blobs)
        encs.extend(decode.ENCODINGS.get("thriftrw" if s.encodings is None else e, 0xFF)
                    for e in (s.encodings or [None] * len(s.blobs)))
        r["init_version"], r["now_ns"] = s.domain_failover_version, s.now_ns
        r["run_id_off"], r["run_id_len"] = put(s.run_id.encode())
        r["branch_id_off"], r["branch_id_len"] = put(s.branch_id.encode())
        if s.final_token is None:
            r["final_token_off"], r["final_token_len"] = 0, abi.NO_TOKEN
        else:
            r["final_token_off"], r["final_token_len"] = put(bytes(s.final_token))
        r["rebuild_last_event_id"], r["rebuild_last_event_version"] = s.rebuild_last_event_id, s.rebuild_last_event_version
        r["new_run_wf"] = -1 if s.new_run is None else int(s.new_run)
        r["flags"] = (abi.WF_FLAG_NEW_RUN if s.is_new_run else 0) | (abi.WF_FLAG_REFRESH_TASKS if s.refresh_tasks else 0)
        r["retention_days"] = s.retention_days
    lens = np.array([len(b) for b in blobs], np.uint64)
    off = np.zeros(len(blobs) + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.zeros(int(off[-1]) + 32, np.uint8)
    if blobs:
        data[:int(off[-1])] = np.frombuffer(b"".join(blobs), np.uint8)
    st = np.frombuffer(bytes(strings), np.uint8).copy() if strings else np.zeros(1, np.uint8)
    return BlobSet(bytes=data, blob_off=off, wf=wf, strings=st), np.array(encs, np.uint32)


def _lib():
    L = decode.lib()
    if not getattr(L, "_encode_bound", False):
        vp = ctypes.c_void_p
        L.crr_encode_blobs.argtypes = [vp, vp, vp, vp, ctypes.c_int]
        L.crr_encode_blobs.restype = vp
        L.crr_encode_blobs_as.argtypes = [vp, vp, vp, vp, ctypes.c_int, ctypes.c_int]
        L.crr_encode_blobs_as.restype = vp
        L.crr_encoded_view.argtypes = [vp] + [vp] * 8
        L.crr_encoded_view.restype = None
        L.crr_encoded_free.argtypes = [vp]
        L.crr_encoded_free.restype = None
        L._encode_bound = True
    return L


def encode_batch(batch: HistoryBatch, n_threads: int = 0, json: bool = False) -> BlobSet:
    """Persist a canonical batch as thriftrw blobs (one per ApplyEvents batch, in order); ``json``: as
    common/types JSON blobs instead (serializer.go:321-325's json encoding; encodings ENCODINGS["json"])."""
    assert batch.stride == 1
    L = _lib()
    keep = []

    def ptr(a):
        a = np.ascontiguousarray(a)
        keep.append(a)
        return a.ctypes.data

    ci = abi.CInputs()
    for name, t in abi.EVENT_COLUMNS:
        setattr(ci.ev, name, ptr(np.asarray(batch.cols[name], t)))
    ci.act_side = ptr(batch.act_side)
    ci.start_side = ptr(batch.start_side)
    ci.reset_keys = ptr(batch.reset_keys)
    ci.arena = ptr(np.concatenate([batch.arena, np.zeros(16, np.uint8)]))
    ci.wf = ptr(batch.wf)
    ci.n_wf = batch.n_wf
    ci.stride = 1
    ko = ptr(batch.key_off) if batch.key_off is not None else None
    kl = ptr(batch.key_len) if batch.key_len is not None else None
    ka = ptr(batch.key_arena) if batch.key_arena is not None else None
    h = L.crr_encode_blobs_as(ctypes.byref(ci), ko, kl, ka, int(n_threads), int(bool(json)))
    if not h:
        raise RuntimeError("crr_encode_blobs failed")
    try:
        b, nb, bo, nbl, wf, nw, st, ns = (ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_void_p(), ctypes.c_uint32(),
                                         ctypes.c_void_p(), ctypes.c_uint32(), ctypes.c_void_p(), ctypes.c_uint64())
        L.crr_encoded_view(h, *(ctypes.byref(x) for x in (b, nb, bo, nbl, wf, nw, st, ns)))
        out = BlobSet(bytes=np.ctypeslib.as_array((ctypes.c_uint8 * (nb.value + 32)).from_address(b.value)).copy(),
                      blob_off=np.ctypeslib.as_array((ctypes.c_uint64 * (nbl.value + 1)).from_address(bo.value)).copy(),
                      wf=np.frombuffer(ctypes.string_at(wf.value, nw.value * BLOB_WF.itemsize), BLOB_WF).copy()
                      if nw.value else np.zeros(0, BLOB_WF),
                      strings=np.ctypeslib.as_array((ctypes.c_uint8 * ns.value).from_address(st.value)).copy())
    finally:
        L.crr_encoded_free(h)
    return out
