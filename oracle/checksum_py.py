"""TEST INFRASTRUCTURE ONLY -- an independent pure-Python restatement of the mutable-state checksum.

Second implementation of the checksum payload, written from the Go sources without looking at
the C++ oracle's or the HIP kernel's encoder, so a shared misreading of the wire format would have
to be made twice.  Only ``tests/`` and ``tests/golden/make_golden.py`` import it.

    execution/checksum.go:56-114         newMutableStateChecksumPayload: which fields are set,
                                         the five pending-ID lists sorted ascending
    common/checksum/crc.go:35-54         GenerateCRC32: payload bytes -> crc32.ChecksumIEEE,
                                         stored as 4 big-endian bytes (Version 1, Flavor 1)
    common/codec/version0Thriftrw.go:44-61, interface.go:48
                                         one preamble byte 0x59, then the thriftrw binary struct
    .gen/go/checksum/checksum.go:539-821 MutableStateChecksumPayload.Encode: field order, nil
                                         fields skipped, lists = elem type + BE i32 count
    .gen/go/shared/shared.go:91639, 92043, 92375
                                         VersionHistories / VersionHistory / VersionHistoryItem
    common/types/mapper/thrift/shared.go:5824-5876, 6706-6739
                                         From* mappers: nil slices stay nil (field omitted)

Thrift binary protocol (thriftrw ``wire``): field header = type byte + BE i16 id; stop = 0x00;
bool = 1 byte; i16/i32/i64 big-endian; binary = BE i32 length + bytes; list = elem type byte +
BE i32 count + elements; struct = fields + stop.
"""
from __future__ import annotations

import struct
import zlib
from typing import Iterable, List, Optional, Sequence, Tuple

T_BOOL, T_I16, T_I32, T_I64, T_BINARY, T_STRUCT, T_LIST = 2, 6, 8, 10, 11, 12, 15
PREAMBLE_V0_THRIFTRW = 0x59            # common/codec/interface.go:48 preambleVersion0


class _W:
    def __init__(self):
        self.b = bytearray()

    def field(self, fid: int, ftype: int):
        self.b += struct.pack(">bh", ftype, fid)

    def stop(self):
        self.b.append(0)

    def i16(self, v: int):
        self.b += struct.pack(">h", v)

    def i32(self, v: int):
        self.b += struct.pack(">i", v)

    def i64(self, v: int):
        self.b += struct.pack(">q", v)

    def binary(self, v: bytes):
        self.i32(len(v))
        self.b += v

    def list_begin(self, etype: int, n: int):
        self.b += struct.pack(">bi", etype, n)


def encode_payload(*, cancel_requested: bool, state: int, last_first_event_id: int, next_event_id: int,
                   last_processed_event_id: int, signal_count: int, decision_attempt: int,
                   decision_version: int, decision_scheduled_id: int, decision_started_id: int,
                   pending_timer_started_ids: Iterable[int], pending_activity_scheduled_ids: Iterable[int],
                   pending_signal_initiated_ids: Iterable[int], pending_req_cancel_initiated_ids: Iterable[int],
                   pending_child_initiated_ids: Iterable[int], sticky_task_list: str = "",
                   version_histories: Optional[Tuple[int, Sequence[Tuple[bytes, Sequence[Tuple[int, int]]]]]] = None
                   ) -> bytes:
    """0x59 + MutableStateChecksumPayload (checksum.go:56-114 fields, checksum.go:539-821 order).

    ``version_histories`` = (current index, [(branch token, [(event_id, version), ...]), ...]).
    CloseStatus (16), LastWriteVersion (21) and LastWriteEventID (22) are never set by
    newMutableStateChecksumPayload, so they are absent."""
    w = _W()
    w.b.append(PREAMBLE_V0_THRIFTRW)
    w.field(10, T_BOOL); w.b.append(1 if cancel_requested else 0)
    w.field(15, T_I16); w.i16(state)                       # int16(executionInfo.State)
    w.field(23, T_I64); w.i64(last_first_event_id)
    w.field(24, T_I64); w.i64(next_event_id)
    w.field(25, T_I64); w.i64(last_processed_event_id)
    w.field(26, T_I64); w.i64(signal_count)                # int64(executionInfo.SignalCount)
    w.field(35, T_I32); w.i32(decision_attempt)            # int32(executionInfo.DecisionAttempt)
    w.field(36, T_I64); w.i64(decision_version)
    w.field(37, T_I64); w.i64(decision_scheduled_id)
    w.field(38, T_I64); w.i64(decision_started_id)
    # make([]int64, 0, n) is a non-nil slice: every list is written, possibly empty
    for fid, ids in ((45, pending_timer_started_ids), (46, pending_activity_scheduled_ids),
                     (47, pending_signal_initiated_ids), (48, pending_req_cancel_initiated_ids),
                     (49, pending_child_initiated_ids)):
        ids = sorted(int(x) for x in ids)                  # common.SortInt64Slice
        w.field(fid, T_LIST); w.list_begin(T_I64, len(ids))
        for x in ids:
            w.i64(x)
    w.field(55, T_BINARY); w.binary(sticky_task_list.encode())   # StringPtr: always present
    if version_histories is not None:
        idx, hists = version_histories
        w.field(56, T_STRUCT)
        w.field(10, T_I32); w.i32(idx)                     # CurrentVersionHistoryIndex
        w.field(20, T_LIST); w.list_begin(T_STRUCT, len(hists))
        for token, items in hists:
            if token is not None:                          # BranchToken []byte: nil -> omitted
                w.field(10, T_BINARY); w.binary(bytes(token))
            if items is not None:                          # FromVersionHistoryItemArray(nil) -> nil
                w.field(20, T_LIST); w.list_begin(T_STRUCT, len(items))
                for eid, ver in items:
                    w.field(10, T_I64); w.i64(eid)
                    w.field(20, T_I64); w.i64(ver)
                    w.stop()
            w.stop()
        w.stop()
    w.stop()
    return bytes(w.b)


def crc32_ieee(data: bytes) -> int:
    """crc32.ChecksumIEEE (crc.go:46)."""
    return zlib.crc32(data) & 0xFFFFFFFF


def checksum_value(payload: bytes) -> bytes:
    """Checksum.Value: the CRC as 4 big-endian bytes (crc.go:47-53)."""
    return struct.pack(">I", crc32_ieee(payload))


def payload_from_rows(exec_row, live: dict, token: Optional[bytes]) -> bytes:
    """Payload of one replayed workflow from the engine's output rows (``abi.EXEC_ROW`` + live rows).

    ``live`` holds the workflow's live slot rows by table name (``ReplayResult.live_rows``);
    ``token`` is the branch token the engine's ``token_src`` names (None -> no VersionHistories,
    b"" -> an empty token)."""
    items: List[Tuple[int, int]] = [(int(r["event_id"]), int(r["version"])) for r in live["vh"]]
    return encode_payload(
        cancel_requested=bool(int(exec_row["flags"]) & 1),
        state=int(exec_row["state"]),
        last_first_event_id=int(exec_row["last_first_event_id"]),
        next_event_id=int(exec_row["next_event_id"]),
        last_processed_event_id=int(exec_row["last_processed_event"]),
        signal_count=int(exec_row["signal_count"]),
        decision_attempt=int(exec_row["decision_attempt"]),
        decision_version=int(exec_row["decision_version"]),
        decision_scheduled_id=int(exec_row["decision_schedule_id"]),
        decision_started_id=int(exec_row["decision_started_id"]),
        pending_timer_started_ids=[r["started_id"] for r in live["timer"]],
        pending_activity_scheduled_ids=[r["schedule_id"] for r in live["act"]],
        pending_signal_initiated_ids=[r["initiated_id"] for r in live["sig"]],
        pending_req_cancel_initiated_ids=[r["initiated_id"] for r in live["rc"]],
        pending_child_initiated_ids=[r["initiated_id"] for r in live["child"]],
        version_histories=(0, [(token if token is not None else b"", items)]),
    )


def token_of(batch, w: int, token_src: int) -> bytes:
    """Branch-token bytes named by ``token_src`` (0 nil, 1 start token, 2 rebuild target token)."""
    r = batch.wf[w]
    if token_src == 1:
        off, n = int(r["start_token_off"]), int(r["start_token_len"])
    elif token_src == 2:
        off, n = int(r["final_token_off"]), int(r["final_token_len"])
    else:
        return b""
    return bytes(batch.arena[off:off + n])
