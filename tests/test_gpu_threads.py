"""The C ABI under a cgo-style caller: several host threads driving one device at once, each on its own
stream, and calls from a thread that never selected the device (INTEGRATION.md §4 thread model).
Every result must equal the single-threaded replay, bit for bit."""
import ctypes
import threading

import numpy as np
import pytest

from cadence_amd import synth_mixed
from cadence_amd.flatten import flatten, interleave
from cadence_amd.result import diff_results

KNOWN = {"domain-a", "domain-b", "parent-domain"}


@pytest.fixture(scope="module")
def eng():
    from cadence_amd.engine import ReplayEngine
    return ReplayEngine(0)


@pytest.mark.gpu
def test_concurrent_threads_on_one_device(eng):
    """Mixed batches fork their tier segments onto the device's side streams; four threads enqueue at
    once (the per-device mutex serialises the enqueue, not the GPU work) and each result equals the
    sequential replay of the same batch."""
    torch = eng.torch
    batches = [interleave(flatten(synth_mixed.mixed_histories(600, 40 + i, mean_len=60, can_rate=0.2),
                                  known_domains=KNOWN), long_threshold=120) for i in range(4)]
    want = [eng.replay(b) for b in batches]
    dbs = [eng.upload(b) for b in batches]
    errors = []

    def worker(i):
        try:
            s = torch.cuda.Stream(eng.dev)
            for _ in range(3):
                with torch.cuda.stream(s):
                    for k in ("exec", "scratch"):
                        dbs[i].tensors[k].zero_()
                eng.launch(dbs[i], s)
            s.synchronize()
        except Exception as e:   # noqa: BLE001 -- surfaced below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
    for b, db, w in zip(batches, dbs, want):
        got = eng.download(db)
        d = diff_results(b, got, b, w)
        assert not d, d[:3]


@pytest.mark.gpu
def test_call_from_a_thread_without_device_selection(eng):
    """A fresh thread (as a goroutine landing on a new OS thread) calls crr_replay with a stream of
    device 0 without crr_set_device: the call runs on the stream's device; crr_release afterwards tears
    the state down and a later call rebuilds it."""
    b = interleave(flatten(synth_mixed.mixed_histories(300, 77, mean_len=50), known_domains=KNOWN), long_threshold=120)
    want = eng.replay(b)
    db = eng.upload(b)
    s = eng.torch.cuda.Stream(eng.dev)
    rc = []
    t = threading.Thread(target=lambda: rc.append(eng.lib.crr_replay(ctypes.byref(db.c_in), ctypes.byref(db.c_out),
                                                                     ctypes.c_void_p(s.cuda_stream))))
    t.start()
    t.join(timeout=120)
    assert rc == [0]
    s.synchronize()
    assert not diff_results(b, eng.download(db), b, want)
    eng.torch.cuda.synchronize()
    assert eng.lib.crr_release() == 0
    assert not diff_results(b, eng.replay(b), b, want)


@pytest.mark.gpu
def test_every_stream_entry_point_from_a_fresh_thread(eng):
    """The thread model holds for every entry point that takes a stream, not only crr_replay: a fresh
    thread (no crr_set_device) runs the device ingest (plan + layout), crr_replay, crr_compact_rows,
    crr_widen_events, crr_checksum and crr_ndc_prepare on a stream of device 0; each result equals the
    same call made from the main thread."""
    import torch
    from cadence_amd import ndc
    from cadence_amd.blobs import KNOWN_DOMAINS, encode_batch
    from cadence_amd.ingest import DeviceIngest
    from cadence_amd.wire import pack_events
    from test_ndc import random_tasks
    from cadence_amd.decode import decode_histories
    bs = encode_batch(flatten(synth_mixed.mixed_histories(400, 91, mean_len=50, can_rate=0.2),
                              known_domains=set(KNOWN_DOMAINS)))
    b = interleave(decode_histories(bs.to_sources(), known_domains=KNOWN_DOMAINS))   # the host path's layout
    want = eng.replay(b)
    nb = ndc.pack(random_tasks(3000, 5))
    want_ndc, want_items = ndc.prepare_on_device(eng, nb)
    db_ref = eng.upload(b)
    eng.launch(db_ref)
    want_sums = eng.checksum(db_ref)

    got = {}
    errors = []

    def worker():
        try:
            s = torch.cuda.Stream(eng.dev)
            ing = DeviceIngest(eng)
            dblobs = ing.upload(bs)
            out = ing.layout(dblobs, ing.plan(dblobs, s), s)
            eng.launch(out, s)
            s.synchronize()
            got["ingest"] = eng.download(out)
            db = eng.upload(b)
            pk = pack_events(b)
            eng.attach_packed(db, pk)
            for c, a in pk.data.items():
                db.tensors["pk_" + c][:a.size].copy_(torch.from_numpy(a))
            db.tensors["pk_ts_base"].copy_(torch.from_numpy(pk.ts_base))
            torch.cuda.synchronize(eng.dev)
            eng.widen(db, s)
            eng.launch(db, s)
            eng.compact(db, s)
            got["sums"] = eng.checksum(db, s)
            s.synchronize()
            got["compact"] = eng.download_compact(db)
            got["ndc"] = ndc.prepare_on_device(eng, nb, s)
        except Exception as e:   # noqa: BLE001 -- surfaced below
            errors.append(e)

    t = threading.Thread(target=worker)
    t.start()
    t.join(timeout=300)
    assert not errors, errors
    assert not diff_results(b, got["compact"].to_replay_result(b), b, want)
    assert (got["sums"] == want_sums).all()
    # the device-ingested batch is in the device order of the same layout the host path builds
    assert not diff_results(b, got["ingest"], b, want)
    r, items = got["ndc"]
    assert r.tobytes() == want_ndc.tobytes() and items.tobytes() == want_items.tobytes()
