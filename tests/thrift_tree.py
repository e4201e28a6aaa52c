"""A generic thrift-binary tree reader / writer for tests: re-shape persisted history blobs into forms
thriftrw never writes (fields out of order, the type after the attributes, duplicate fields, containers
of structs) while keeping them valid for the reference decoder (history_decode.cpp restates thriftrw's
reader, which accepts any field order).  Test infrastructure only."""
from __future__ import annotations

import random
import struct

T_BOOL, T_BYTE, T_DOUBLE, T_I16, T_I32, T_I64, T_STRING, T_STRUCT, T_MAP, T_SET, T_LIST = 2, 3, 4, 6, 8, 10, 11, 12, 13, 14, 15


class _R:
    def __init__(self, b, p=0):
        self.b, self.p = b, p

    def take(self, n):
        v = self.b[self.p:self.p + n]
        if len(v) != n:
            raise ValueError("truncated")
        self.p += n
        return v

    def value(self, t):
        if t in (T_BOOL, T_BYTE):
            return self.take(1)
        if t == T_I16:
            return self.take(2)
        if t == T_I32:
            return self.take(4)
        if t in (T_I64, T_DOUBLE):
            return self.take(8)
        if t == T_STRING:
            n = struct.unpack(">i", self.take(4))[0]
            return self.take(n)
        if t == T_STRUCT:
            fields = []
            while True:
                ft = self.take(1)[0]
                if ft == 0:
                    return fields
                fid = struct.unpack(">h", self.take(2))[0]
                fields.append([ft, fid, self.value(ft)])
        if t == T_MAP:
            kt, vt = self.take(1)[0], self.take(1)[0]
            n = struct.unpack(">i", self.take(4))[0]
            return (kt, vt, [(self.value(kt), self.value(vt)) for _ in range(n)])
        if t in (T_SET, T_LIST):
            et = self.take(1)[0]
            n = struct.unpack(">i", self.take(4))[0]
            return (et, [self.value(et) for _ in range(n)])
        raise ValueError(f"thrift type {t}")


def parse_blob(blob: bytes):
    """0x59 + History struct -> the History's field list ([type, id, value] triples)."""
    assert blob[0] == 0x59
    return _R(blob, 1).value(T_STRUCT)


def _w(out, t, v):
    if t in (T_BOOL, T_BYTE, T_I16, T_I32, T_I64, T_DOUBLE):
        out += v
    elif t == T_STRING:
        out += struct.pack(">i", len(v)) + v
    elif t == T_STRUCT:
        for ft, fid, fv in v:
            out += bytes([ft]) + struct.pack(">h", fid)
            _w(out, ft, fv)
        out.append(0)
    elif t == T_MAP:
        kt, vt, items = v
        out += bytes([kt, vt]) + struct.pack(">i", len(items))
        for k, x in items:
            _w(out, kt, k)
            _w(out, vt, x)
    else:
        et, items = v
        out += bytes([et]) + struct.pack(">i", len(items))
        for x in items:
            _w(out, et, x)


def write_blob(fields) -> bytes:
    out = bytearray([0x59])
    _w(out, T_STRUCT, fields)
    return bytes(out)


def _nested_extra(rng):
    """A field value the fast reader cannot skip inline: a list of structs / a map of lists."""
    if rng.random() < 0.5:
        return [T_LIST, 900 + rng.randrange(50),
                (T_STRUCT, [[[T_STRING, 1, b"x" * rng.randrange(5)], [T_I32, 2, b"\0\0\0\1"]]
                            for _ in range(rng.randrange(3))])]
    return [T_MAP, 950 + rng.randrange(40), (T_STRING, T_LIST, [(b"k", (T_I32, [b"\0\0\0\2"] * 2))])]


def reshape_event(ev, rng, mode):
    """One HistoryEvent's field list re-shaped by `mode`."""
    ev = [list(f) for f in ev]
    if mode == "reverse":             # attributes before the type, ids decreasing
        ev.reverse()
    elif mode == "shuffle":
        rng.shuffle(ev)
    elif mode == "dup_type":          # the type again at the end (the last one wins: the same value)
        t = [f for f in ev if f[1] == 30]
        if t:
            ev.append(list(t[0]))
    elif mode == "nested_event":      # a list of structs / map of lists among the event's fields
        ev.insert(rng.randrange(len(ev) + 1), _nested_extra(rng))
    elif mode == "nested_attr":       # ... inside the attribute struct
        for f in ev:
            if f[0] == T_STRUCT and 40 <= f[1] <= 450 and f[1] % 10 == 0:
                f[2] = [list(a) for a in f[2]]
                f[2].insert(rng.randrange(len(f[2]) + 1), _nested_extra(rng))
                break
    elif mode == "leaf_containers":   # lists / sets / maps of scalars (the fast reader's inline skip)
        ev.append([T_SET, 990, (T_I64, [b"\0" * 8] * rng.randrange(4))])
        ev.append([T_MAP, 991, (T_STRING, T_I32, [(b"a", b"\0\0\0\1")])])
    return ev


MODES = ("keep", "reverse", "shuffle", "dup_type", "nested_event", "nested_attr", "leaf_containers")


def reshape_blob(blob: bytes, rng: random.Random, rate: float = 0.3) -> bytes:
    """Re-shape a `rate` fraction of a blob's events (modes drawn from MODES)."""
    if not blob:
        return blob
    hist = parse_blob(blob)
    for f in hist:
        if f[1] == 10 and f[0] == T_LIST:
            et, evs = f[2]
            new = []
            for ev in evs:
                mode = rng.choice(MODES[1:]) if rng.random() < rate else "keep"
                new.append(reshape_event(ev, rng, mode))
            f[2] = (et, new)
    return write_blob(hist)


def reshape_blobset(bs, seed: int = 7, rate: float = 0.3):
    """A BlobSet (cadence_amd.blobs) with every blob re-shaped by reshape_blob; same workflows."""
    import dataclasses

    import numpy as np
    rng = random.Random(seed)
    blobs = [reshape_blob(bs.blob(i), rng, rate) for i in range(bs.n_blobs)]
    off = np.zeros(len(blobs) + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in blobs])
    data = np.zeros(int(off[-1]) + 32, np.uint8)
    data[:int(off[-1])] = np.frombuffer(b"".join(blobs), np.uint8)
    return dataclasses.replace(bs, bytes=data, blob_off=off)
