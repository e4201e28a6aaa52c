"""ctypes binding of the CPU restatement -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.  The
product path (cadence_amd.engine) never loads liboracle.so.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from cadence_amd import abi
from cadence_amd.flatten import HistoryBatch
from cadence_amd.result import ReplayResult, allocate_host

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.oracle_replay.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int]
        L.oracle_replay.restype = ctypes.c_int
        L.oracle_replay2.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int]
        L.oracle_replay2.restype = ctypes.c_int
        L.oracle_payload.argtypes = [vp, vp, vp, vp, ctypes.c_uint32, vp, ctypes.c_int]
        L.oracle_payload.restype = ctypes.c_int
        L.oracle_crc32.argtypes = [vp, ctypes.c_size_t]
        L.oracle_crc32.restype = ctypes.c_uint32
        L.oracle_vh_add_or_update.argtypes = [vp, vp, vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int64]
        L.oracle_vh_add_or_update.restype = ctypes.c_int
        L.oracle_update_state.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int]
        L.oracle_update_state.restype = ctypes.c_int
        L.oracle_activity_timer_sequence.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp, ctypes.c_int]
        L.oracle_activity_timer_sequence.restype = ctypes.c_int
        L.oracle_user_timer_sequence.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, ctypes.c_int]
        L.oracle_user_timer_sequence.restype = ctypes.c_int
        L.oracle_vh_query.argtypes = [ctypes.c_int, vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, vp, vp]
        L.oracle_vh_query.restype = ctypes.c_int
        L.oracle_ndc_prepare.argtypes = [vp, vp, vp]
        L.oracle_ndc_prepare.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class _HostInputs:
    """Keeps numpy arrays alive while ctypes holds raw pointers into them."""

    def __init__(self, batch: HistoryBatch):
        self.keep = []
        ev = abi.CEvents()
        for name, t in abi.EVENT_COLUMNS:
            a = np.ascontiguousarray(batch.cols[name], dtype=t)
            self.keep.append(a)
            setattr(ev, name, a.ctypes.data)
        ci = abi.CInputs()
        ci.ev = ev
        for field, arr in (("act_side", batch.act_side), ("start_side", batch.start_side),
                           ("reset_keys", batch.reset_keys), ("arena", batch.arena), ("wf", batch.wf)):
            a = np.ascontiguousarray(arr)
            self.keep.append(a)
            setattr(ci, field, a.ctypes.data)
        ci.n_wf = batch.n_wf
        ci.stride = batch.stride
        ci.flags = batch.c_flags()
        ci.wave_begin = batch.wave_begin or 0
        self.c = ci
        self.key_off = np.ascontiguousarray(batch.key_off, dtype=np.uint32)
        self.key_len = np.ascontiguousarray(batch.key_len, dtype=np.uint32)
        self.key_arena = np.ascontiguousarray(batch.key_arena, dtype=np.uint8)
        if self.key_off.size == 0:
            self.key_off = np.zeros(1, np.uint32)
            self.key_len = np.zeros(1, np.uint32)


def _outputs(res: ReplayResult):
    co = abi.COutputs()
    co.exec = res.exec.ctypes.data if res.exec.size else np.zeros(1, abi.EXEC_ROW).ctypes.data
    for name, *_ in abi.TABLES:
        setattr(co, name, res.tables[name].ctypes.data)
    co.scratch = None
    return co


def replay(batch: HistoryBatch, n_threads: int = 0) -> ReplayResult:
    """Replay every workflow of ``batch`` on the host (oracle)."""
    if batch.key_off is None:
        raise ValueError("oracle needs per-event key strings (batch.key_off / key_len / key_arena)")
    res = allocate_host(batch)          # loaded states (CRR_WF_FLAG_RESUME) already in place
    hi = _HostInputs(batch)
    co = _outputs(res)
    if batch.key_dict is not None:
        kd = [np.ascontiguousarray(a) for a in batch.key_dict]
        rc = lib().oracle_replay2(ctypes.byref(hi.c), _ptr(hi.key_off), _ptr(hi.key_len), _ptr(hi.key_arena),
                                  *[_ptr(a) for a in kd], ctypes.byref(co), int(n_threads))
    else:
        rc = lib().oracle_replay(ctypes.byref(hi.c), _ptr(hi.key_off), _ptr(hi.key_len), _ptr(hi.key_arena),
                                 ctypes.byref(co), int(n_threads))
    if rc != 0:
        raise RuntimeError(f"oracle_replay failed: {rc}")
    return res


def payload(batch: HistoryBatch, w: int) -> bytes:
    """Checksum payload bytes (0x59 + thrift binary) of workflow ``w`` after replay."""
    hi = _HostInputs(batch)
    n = lib().oracle_payload(ctypes.byref(hi.c), _ptr(hi.key_off), _ptr(hi.key_len), _ptr(hi.key_arena),
                             int(w), None, 0)
    buf = np.zeros(max(n, 1), np.uint8)
    lib().oracle_payload(ctypes.byref(hi.c), _ptr(hi.key_off), _ptr(hi.key_len), _ptr(hi.key_arena),
                         int(w), _ptr(buf), n)
    return buf[:n].tobytes()


def crc32(data: bytes) -> int:
    a = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    return int(lib().oracle_crc32(_ptr(a), len(data)))


def vh_add_or_update(items, event_id, version):
    """VersionHistory.AddOrUpdateItem; returns (status, new_items)."""
    cap = len(items) + 2
    ids = np.zeros(cap, np.int64)
    vers = np.zeros(cap, np.int64)
    for i, (e, v) in enumerate(items):
        ids[i], vers[i] = e, v
    n = ctypes.c_int(len(items))
    st = lib().oracle_vh_add_or_update(_ptr(ids), _ptr(vers), ctypes.byref(n), cap, int(event_id), int(version))
    return st, [(int(ids[i]), int(vers[i])) for i in range(n.value)]


def update_state(state, close, new_state, new_close):
    s = ctypes.c_int(state)
    c = ctypes.c_int(close)
    st = lib().oracle_update_state(ctypes.byref(s), ctypes.byref(c), int(new_state), int(new_close))
    return st, s.value, c.value


def activity_timer_sequence(rows: np.ndarray):
    """LoadAndSortActivityTimers over abi.ACTIVITY_ROW images (last_heartbeat_time = LastHeartBeatUpdatedTime).
    Returns [(timestamp, event_id, timer type, created, attempt)]."""
    rows = np.ascontiguousarray(rows, dtype=abi.ACTIVITY_ROW)
    cap = 4 * max(len(rows), 1)
    ts = np.zeros(cap, np.int64)
    eid = np.zeros(cap, np.int64)
    ty = np.zeros(cap, np.int32)
    cr = np.zeros(cap, np.int32)
    at = np.zeros(cap, np.int32)
    n = lib().oracle_activity_timer_sequence(_ptr(rows), len(rows), _ptr(ts), _ptr(eid), _ptr(ty), _ptr(cr), _ptr(at), cap)
    return [(int(ts[i]), int(eid[i]), int(ty[i]), bool(cr[i]), int(at[i])) for i in range(n)]


def user_timer_sequence(rows: np.ndarray):
    """LoadAndSortUserTimers over abi.TIMER_ROW images: [(timestamp, event_id, timer type, created)]."""
    rows = np.ascontiguousarray(rows, dtype=abi.TIMER_ROW)
    cap = max(len(rows), 1)
    ts = np.zeros(cap, np.int64)
    eid = np.zeros(cap, np.int64)
    ty = np.zeros(cap, np.int32)
    cr = np.zeros(cap, np.int32)
    n = lib().oracle_user_timer_sequence(_ptr(rows), len(rows), _ptr(ts), _ptr(eid), _ptr(ty), _ptr(cr), cap)
    return [(int(ts[i]), int(eid[i]), int(ty[i]), bool(cr[i])) for i in range(n)]


def ndc_prepare(batch):
    """prepareVersionHistory for every task of a cadence_amd.ndc.NdcBatch (host); (results, out_items)."""
    n = len(batch.tasks)
    tasks = np.ascontiguousarray(batch.tasks)
    branches = np.ascontiguousarray(batch.branches)
    items = np.ascontiguousarray(batch.items)
    ci = abi.CNdcInputs()
    ci.tasks, ci.branches, ci.items = tasks.ctypes.data, branches.ctypes.data, items.ctypes.data
    ci.n_tasks = n
    res = np.zeros(max(n, 1), abi.NDC_RESULT)
    out = np.zeros(batch.n_out_items, abi.VH_ITEM)
    lib().oracle_ndc_prepare(ctypes.byref(ci), _ptr(res), _ptr(out))
    return res[:n], out


VH_DUPLICATE_UNTIL_LCA, VH_IS_LCA_APPENDABLE, VH_FIRST, VH_LAST, VH_CONTAINS, VH_EVENT_VERSION, VH_ADD_OR_UPDATE = range(1, 8)


def vh_query(op, items, a=0, b=0):
    """One VersionHistory operation (versionHistory.go) on ``items`` [(event_id, version)]: (result, items out)."""
    arr = np.array([tuple(x) for x in items] or [(0, 0)], abi.VH_ITEM)
    out = np.zeros(len(items) + 2, abi.VH_ITEM)
    n = ctypes.c_int(0)
    r = lib().oracle_vh_query(int(op), _ptr(arr), len(items), int(a), int(b), _ptr(out), ctypes.byref(n))
    return r, [(int(x["event_id"]), int(x["version"])) for x in out[:n.value]]
