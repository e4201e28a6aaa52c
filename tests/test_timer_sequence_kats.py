"""service/history/execution/timer_sequence_test.go:74-1137 restated (34 tests).

CreateNext* (:74-231) and the heads of the *_Multiple orderings run through ApplyEvents onto loaded
states (tests/kat_state_builder.timer_cases, also replayed on the device by tests/test_gpu_kats.py);
LoadAndSort* / get*Timeout / Less (:233-1137) are checked on the oracle's LoadAndSort functions with
the exact sequence IDs each Go test expects (EventID, Timestamp, TimerType, TimerCreated, Attempt).
"""
import numpy as np
import pytest

from cadence_amd import abi
from oracle import oracle

import kat_state_builder as K

NOW = 1_700_000_000_123_456_789
SEC = 1_000_000_000
MS = 1_000_000
S2C, S2S, ST2C, HB = abi.TimeoutType.StartToClose, abi.TimeoutType.ScheduleToStart, abi.TimeoutType.ScheduleToClose, \
    abi.TimeoutType.Heartbeat
# TimerType == TimeoutType numbering: StartToClose 0, ScheduleToStart 1, ScheduleToClose 2, Heartbeat 3
START_TO_CLOSE, SCHEDULE_TO_START, SCHEDULE_TO_CLOSE = S2C, S2S, ST2C


def ai(schedule_id=234, scheduled=NOW, started_id=abi.EMPTY_EVENT_ID, started=abi.ZERO_TIME, s2s=10, s2c=1000, st2c=100,
       hb=1, last_hb=abi.ZERO_TIME, tts=0, attempt=12):
    r = np.zeros(1, abi.ACTIVITY_ROW)
    r["schedule_id"], r["scheduled_time"], r["started_id"], r["started_time"] = schedule_id, scheduled, started_id, started
    r["schedule_to_start"], r["schedule_to_close"], r["start_to_close"], r["heartbeat"] = s2s, s2c, st2c, hb
    r["last_heartbeat_time"], r["timer_task_status"], r["attempt"] = last_hb, tts, attempt
    return r


def ti(started_id=456, expiry=NOW + 100 * SEC, status=1, version=123):
    r = np.zeros(1, abi.TIMER_ROW)
    r["started_id"], r["expiry_time"], r["task_status"], r["version"] = started_id, expiry, status, version
    return r


def test_timer_engine_kats():   # :74-231 + the *_Multiple heads, through ApplyEvents onto loaded states
    kats = K.timer_cases()
    batch, idx, nr = K.build_batch(kats)
    res = oracle.replay(batch, 1)
    fails = K.check_all(kats, batch, res, idx, nr)
    assert not fails, "\n".join(fails)


# ---- LoadAndSortUserTimers / getUserTimerTimeout ----------------------------------------------------
def test_load_and_sort_user_timers_none():       # :233-239
    assert oracle.user_timer_sequence(np.zeros(0, abi.TIMER_ROW)) == []


def test_load_and_sort_user_timers_one():        # :241-261
    assert oracle.user_timer_sequence(ti()) == [(NOW + 100 * SEC, 456, START_TO_CLOSE, True)]


def test_load_and_sort_user_timers_multiple():   # :263-302
    rows = np.concatenate([ti(4567, NOW + 200 * SEC, 0, 1234), ti()])
    assert oracle.user_timer_sequence(rows) == [(NOW + 100 * SEC, 456, START_TO_CLOSE, True),
                                                (NOW + 200 * SEC, 4567, START_TO_CLOSE, False)]


def test_get_user_timer_timeout():               # :646-671
    assert oracle.user_timer_sequence(ti(status=1)) == [(NOW + 100 * SEC, 456, START_TO_CLOSE, True)]
    assert oracle.user_timer_sequence(ti(status=0)) == [(NOW + 100 * SEC, 456, START_TO_CLOSE, False)]


# ---- LoadAndSortActivityTimers ------------------------------------------------------------------------
def test_load_and_sort_activity_timers_none():   # :304-310
    assert oracle.activity_timer_sequence(np.zeros(0, abi.ACTIVITY_ROW)) == []


def test_load_and_sort_activity_timers_not_scheduled():   # :312-332
    assert oracle.activity_timer_sequence(ai(schedule_id=abi.EMPTY_EVENT_ID, scheduled=abi.ZERO_TIME)) == []


def test_load_and_sort_activity_timers_scheduled_not_started():   # :334-375
    seq = oracle.activity_timer_sequence(ai(tts=abi.TTS_SCHEDULE_TO_CLOSE | abi.TTS_SCHEDULE_TO_START))
    assert seq == [(NOW + 10 * SEC, 234, SCHEDULE_TO_START, True, 12),
                   (NOW + 1000 * SEC, 234, SCHEDULE_TO_CLOSE, True, 12)]


def test_load_and_sort_activity_timers_started_with_heartbeat():   # :377-427
    st = NOW + 200 * MS
    seq = oracle.activity_timer_sequence(ai(started_id=345, started=st,
                                            tts=abi.TTS_SCHEDULE_TO_CLOSE | abi.TTS_START_TO_CLOSE | abi.TTS_HEARTBEAT))
    assert seq == [(st + 1 * SEC, 234, HB, True, 12), (st + 100 * SEC, 234, START_TO_CLOSE, True, 12),
                   (NOW + 1000 * SEC, 234, SCHEDULE_TO_CLOSE, True, 12)]


def test_load_and_sort_activity_timers_started_without_heartbeat():   # :429-470
    st = NOW + 200 * MS
    seq = oracle.activity_timer_sequence(ai(started_id=345, started=st, hb=0,
                                            tts=abi.TTS_SCHEDULE_TO_CLOSE | abi.TTS_START_TO_CLOSE))
    assert seq == [(st + 100 * SEC, 234, START_TO_CLOSE, True, 12), (NOW + 1000 * SEC, 234, SCHEDULE_TO_CLOSE, True, 12)]


def test_load_and_sort_activity_timers_heartbeated_with_heartbeat():   # :472-522
    st, hbt = NOW + 200 * MS, NOW + 400 * MS
    seq = oracle.activity_timer_sequence(ai(started_id=345, started=st, last_hb=hbt,
                                            tts=abi.TTS_SCHEDULE_TO_CLOSE | abi.TTS_START_TO_CLOSE | abi.TTS_HEARTBEAT))
    assert seq == [(hbt + 1 * SEC, 234, HB, True, 12), (st + 100 * SEC, 234, START_TO_CLOSE, True, 12),
                   (NOW + 1000 * SEC, 234, SCHEDULE_TO_CLOSE, True, 12)]


def test_load_and_sort_activity_timers_heartbeated_without_heartbeat():   # :524-565
    st, hbt = NOW + 200 * MS, NOW + 400 * MS
    seq = oracle.activity_timer_sequence(ai(started_id=345, started=st, last_hb=hbt, hb=0,
                                            tts=abi.TTS_SCHEDULE_TO_CLOSE | abi.TTS_START_TO_CLOSE))
    assert seq == [(st + 100 * SEC, 234, START_TO_CLOSE, True, 12), (NOW + 1000 * SEC, 234, SCHEDULE_TO_CLOSE, True, 12)]


def test_load_and_sort_activity_timers_multiple():   # :567-644
    a1 = ai(started_id=345, started=NOW + 200 * MS, hb=0, last_hb=NOW + 400 * MS)
    a2 = ai(schedule_id=2345, s2s=11, s2c=1001, st2c=101, hb=6, last_hb=NOW + 800 * MS, attempt=21)
    seq = oracle.activity_timer_sequence(np.concatenate([a1, a2]))
    assert seq == [(NOW + 11 * SEC, 2345, SCHEDULE_TO_START, False, 21),
                   (NOW + 200 * MS + 100 * SEC, 234, START_TO_CLOSE, False, 12),
                   (NOW + 1000 * SEC, 234, SCHEDULE_TO_CLOSE, False, 12),
                   (NOW + 1001 * SEC, 2345, SCHEDULE_TO_CLOSE, False, 21)]


# ---- get*Timeout: each getter's contribution to the sequence --------------------------------------------
def _of(rows, ttype):
    return [s for s in oracle.activity_timer_sequence(rows) if s[2] == ttype]


@pytest.mark.parametrize("tts,created", [(abi.TTS_SCHEDULE_TO_START, True), (0, False)])
def test_get_activity_schedule_to_start(tts, created):   # :673-756
    assert _of(ai(schedule_id=abi.EMPTY_EVENT_ID, scheduled=abi.ZERO_TIME, hb=0), SCHEDULE_TO_START) == []   # NotScheduled
    assert _of(ai(hb=0, tts=tts), SCHEDULE_TO_START) == [(NOW + 10 * SEC, 234, SCHEDULE_TO_START, created, 12)]
    assert _of(ai(started_id=345, started=NOW + 200 * SEC, hb=0, tts=tts), SCHEDULE_TO_START) == []   # Started


@pytest.mark.parametrize("tts,created", [(abi.TTS_SCHEDULE_TO_CLOSE, True), (0, False)])
def test_get_activity_schedule_to_close(tts, created):   # :758-815
    assert _of(ai(schedule_id=abi.EMPTY_EVENT_ID, scheduled=abi.ZERO_TIME, hb=0), SCHEDULE_TO_CLOSE) == []
    assert _of(ai(hb=0, tts=tts), SCHEDULE_TO_CLOSE) == [(NOW + 1000 * SEC, 234, SCHEDULE_TO_CLOSE, created, 12)]


@pytest.mark.parametrize("tts,created", [(abi.TTS_START_TO_CLOSE, True), (0, False)])
def test_get_activity_start_to_close(tts, created):   # :817-874
    assert _of(ai(hb=0), START_TO_CLOSE) == []                                                    # NotStarted
    st = NOW + 200 * MS
    assert _of(ai(started_id=345, started=st, hb=0, last_hb=NOW + 400 * MS, tts=tts), START_TO_CLOSE) == \
        [(st + 100 * SEC, 234, START_TO_CLOSE, created, 12)]


@pytest.mark.parametrize("tts,created", [(abi.TTS_HEARTBEAT, True), (0, False)])
def test_get_activity_heartbeat(tts, created):   # :876-1044
    st, hbt = NOW + 200 * MS, NOW + 400 * MS
    assert _of(ai(hb=1, last_hb=hbt), HB) == []                                                    # WithHeartbeat_NotStarted
    assert _of(ai(started_id=345, started=st, hb=1, tts=tts), HB) == [(st + 1 * SEC, 234, HB, created, 12)]   # NoHeartbeat
    assert _of(ai(started_id=345, started=st, hb=1, last_hb=hbt, tts=tts), HB) == [(hbt + 1 * SEC, 234, HB, created, 12)]
    assert _of(ai(hb=0, last_hb=hbt), HB) == []                                                    # WithoutHeartbeat_*
    assert _of(ai(started_id=345, started=st, hb=0, tts=tts), HB) == []
    assert _of(ai(started_id=345, started=st, hb=0, last_hb=hbt, tts=tts), HB) == []


def test_conversion():   # :1046-1068 TimerTypeToInternal / TimerTypeToTimerMask / status constants
    assert (int(S2C), int(S2S), int(ST2C), int(HB)) == (0, 1, 2, 3)
    assert (abi.TTS_START_TO_CLOSE, abi.TTS_SCHEDULE_TO_START, abi.TTS_SCHEDULE_TO_CLOSE, abi.TTS_HEARTBEAT) == (1, 2, 4, 8)


def test_less():   # :1070-1137 TestLess_CompareTime / CompareEventID / CompareType
    # time first: an earlier Heartbeat timer of a larger event ID sorts first
    a = ai(schedule_id=124, started_id=345, started=NOW - 10 * SEC, hb=1, s2c=10_000, st2c=10_000)
    b = ai(schedule_id=123, started_id=346, started=NOW, hb=1, s2c=10_000, st2c=10_000)
    seq = oracle.activity_timer_sequence(np.concatenate([b, a]))
    assert (seq[0][1], seq[0][2]) == (124, HB)
    # same time: smaller event ID first; same time and ID: smaller timer type first
    c = ai(schedule_id=10, s2s=5, s2c=5, hb=0)
    d = ai(schedule_id=9, s2s=5, s2c=6, hb=0)
    seq = oracle.activity_timer_sequence(np.concatenate([c, d]))
    assert [(s[1], int(s[2])) for s in seq[:3]] == [(9, SCHEDULE_TO_START), (10, SCHEDULE_TO_START), (10, SCHEDULE_TO_CLOSE)]
