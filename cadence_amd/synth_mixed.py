"""Seeded random-walk histories over every event type (config 3/5 shapes + edge cases).

Mirrors the event-graph generator of ``common/testing/history_event_util.go:51-1012`` (decision
scheduled -> started -> completed/failed/timed out; decision completion emits activity / timer /
child / cancel / signal / marker / upsert events; external events arrive in their own batches
followed by a decision schedule) and adds the anomalies the reference's code paths handle:
duplicate ActivityIDs / TimerIDs, deletes of unknown IDs (data-inconsistency logging), failover
version bumps at batch boundaries (multi-item VersionHistories), transient
decisions, continue-as-new with a new-run history, and, at ``invalid_rate``, histories that end in
each error the state builder can return.
"""
from __future__ import annotations

import random
from typing import List, Optional

from .abi import EventType as ET
from .history import HistoryEvent, WorkflowHistory, det_uuid

BASE_TS = 1_600_000_000_000_000_000


class _Walk:
    def __init__(self, rng: random.Random, wf_index: int, multi_version: bool, domains):
        self.rng = rng
        self.w = wf_index
        self.eid = 0
        self.ts = BASE_TS + wf_index * 1_000_000_000
        self.version = 1 if not multi_version else rng.choice([1, 2, 10])
        self.multi_version = multi_version
        self.domains = domains
        self.batches: List[List[HistoryEvent]] = []
        self.task = 1000 + wf_index * 100000
        # mirrored state
        self.dec_sched = None
        self.dec_started = None
        self.acts = {}          # activity id -> (sched id, started)
        self.act_seq = 0
        self.timers = {}        # timer id -> started id
        self.timer_seq = 0
        self.children = {}      # initiated id -> started?
        self.rcs = set()
        self.sigs = set()
        self.closed = False
        self.attempt = 0
        self.caps = None         # optional concurrency caps {"act", "timer", "child", "rc", "sig"}

    def full(self, what: str, live) -> bool:
        return self.caps is not None and len(live) >= self.caps[what]

    def ev(self, t, **attrs) -> HistoryEvent:
        self.eid += 1
        self.ts += self.rng.randint(1_000_000, 3_000_000_000)
        self.task += 1
        return HistoryEvent(int(t), self.eid, self.version, self.ts, self.task, attrs)

    def bump_version(self):
        if self.multi_version and self.rng.random() < 0.15:
            self.version += self.rng.choice([1, 10])

    def emit(self, batch):
        self.batches.append(batch)
        self.task += self.rng.randint(2, 5)

    def domain(self):
        r = self.rng.random()
        if r < 0.7:
            return ""
        if r < 0.995:
            return self.rng.choice(self.domains[:-1])
        return self.domains[-1]          # a name the domain cache cannot resolve

    # -- event builders --
    def start(self, prev_points=None, new_run_of=None):
        b = [self.ev(ET.WorkflowExecutionStarted, task_start_to_close_timeout_seconds=self.rng.randint(5, 60),
                     execution_start_to_close_timeout_seconds=self.rng.randint(60, 86400),
                     first_decision_task_backoff_seconds=0, initiator=None,
                     parent_workflow_domain=self.rng.choice(["", "", "", "parent-domain"]),
                     prev_auto_reset_points=prev_points)]
        b.append(self.sched_decision())
        self.emit(b)

    def sched_decision(self, attempt=0):
        e = self.ev(ET.DecisionTaskScheduled, start_to_close_timeout_seconds=self.rng.randint(5, 60), attempt=attempt)
        self.dec_sched = e.id
        self.dec_started = None
        return e

    def start_decision(self):
        e = self.ev(ET.DecisionTaskStarted, scheduled_event_id=self.dec_sched, request_id=det_uuid(self.w, self.eid))
        self.dec_started = e.id
        return e

    def decision_outputs(self) -> List[HistoryEvent]:
        out = []
        for _ in range(self.rng.choice([0, 1, 1, 2, 3])):
            kind = self.rng.random()
            if kind < 0.40 and self.full("act", self.acts):
                e = self.ev(ET.MarkerRecorded)
            elif kind < 0.40:
                dup = self.acts and self.rng.random() < 0.05
                aid = self.rng.choice(list(self.acts)) if dup else str(self.act_seq)
                self.act_seq += 1
                e = self.ev(ET.ActivityTaskScheduled, activity_id=aid, domain=self.domain(),
                            schedule_to_start_timeout_seconds=self.rng.randint(1, 3600),
                            schedule_to_close_timeout_seconds=self.rng.randint(1, 3600),
                            start_to_close_timeout_seconds=self.rng.randint(1, 3600),
                            heartbeat_timeout_seconds=self.rng.choice([0, 0, self.rng.randint(1, 60)]),
                            retry_policy=({"expiration_interval_in_seconds": self.rng.randint(0, 600)}
                                          if self.rng.random() < 0.3 else None))
                self.acts[aid] = [e.id, False]
            elif kind < 0.60 and self.full("timer", self.timers):
                e = self.ev(ET.MarkerRecorded)
            elif kind < 0.60:
                dup = self.timers and self.rng.random() < 0.1
                tid = self.rng.choice(list(self.timers)) if dup else f"t{self.timer_seq}"
                self.timer_seq += 1
                e = self.ev(ET.TimerStarted, timer_id=tid, start_to_fire_timeout_seconds=self.rng.randint(1, 100000))
                self.timers[tid] = e.id
            elif kind < 0.67 and self.full("child", self.children):
                e = self.ev(ET.MarkerRecorded)
            elif kind < 0.67:
                e = self.ev(ET.StartChildWorkflowExecutionInitiated, domain=self.domain())
                self.children[e.id] = False
            elif kind < 0.72 and self.full("rc", self.rcs):
                e = self.ev(ET.MarkerRecorded)
            elif kind < 0.72:
                e = self.ev(ET.RequestCancelExternalWorkflowExecutionInitiated, domain=self.domain())
                self.rcs.add(e.id)
            elif kind < 0.77 and self.full("sig", self.sigs):
                e = self.ev(ET.MarkerRecorded)
            elif kind < 0.77:
                e = self.ev(ET.SignalExternalWorkflowExecutionInitiated, domain=self.domain())
                self.sigs.add(e.id)
            elif kind < 0.82:
                e = self.ev(ET.MarkerRecorded)
            elif kind < 0.85:
                e = self.ev(ET.UpsertWorkflowSearchAttributes)
            elif kind < 0.90 and self.acts:
                aid = self.rng.choice(list(self.acts) + ["missing-activity"])
                e = self.ev(ET.ActivityTaskCancelRequested, activity_id=aid)
            elif kind < 0.94 and self.timers:
                tid = self.rng.choice(list(self.timers))
                e = self.ev(ET.TimerCanceled, timer_id=tid)
                self.timers.pop(tid, None)
            elif kind < 0.97:
                e = self.ev(ET.CancelTimerFailed)
            else:
                e = self.ev(ET.RequestCancelActivityTaskFailed)
            out.append(e)
        return out

    def external(self) -> Optional[List[HistoryEvent]]:
        r = self.rng.random()
        if r < 0.15:
            return [self.ev(ET.WorkflowExecutionSignaled)]
        if r < 0.45 and self.acts:
            aid = self.rng.choice(list(self.acts))
            sched, started = self.acts[aid]
            if not started and self.rng.random() < 0.7:
                self.acts[aid][1] = True
                return [self.ev(ET.ActivityTaskStarted, scheduled_event_id=sched, request_id=det_uuid(self.w, "a", sched))]
            t = self.rng.choice([ET.ActivityTaskCompleted, ET.ActivityTaskCompleted, ET.ActivityTaskFailed,
                                 ET.ActivityTaskTimedOut, ET.ActivityTaskCanceled])
            self.acts.pop(aid)
            return [self.ev(t, scheduled_event_id=sched)]
        if r < 0.55 and self.timers:
            tid = self.rng.choice(list(self.timers))
            self.timers.pop(tid)
            return [self.ev(ET.TimerFired, timer_id=tid)]
        if r < 0.62 and self.children:
            cid = self.rng.choice(list(self.children))
            if not self.children[cid] and self.rng.random() < 0.6:
                self.children[cid] = True
                return [self.ev(ET.ChildWorkflowExecutionStarted, initiated_event_id=cid)]
            t = self.rng.choice([ET.ChildWorkflowExecutionCompleted, ET.ChildWorkflowExecutionFailed,
                                 ET.ChildWorkflowExecutionCanceled, ET.ChildWorkflowExecutionTimedOut,
                                 ET.ChildWorkflowExecutionTerminated, ET.StartChildWorkflowExecutionFailed])
            self.children.pop(cid)
            return [self.ev(t, initiated_event_id=cid)]
        if r < 0.67 and self.rcs:
            rid = self.rng.choice(sorted(self.rcs))
            self.rcs.discard(rid)
            t = self.rng.choice([ET.ExternalWorkflowExecutionCancelRequested, ET.RequestCancelExternalWorkflowExecutionFailed])
            return [self.ev(t, initiated_event_id=rid)]
        if r < 0.72 and self.sigs:
            sid = self.rng.choice(sorted(self.sigs))
            self.sigs.discard(sid)
            t = self.rng.choice([ET.ExternalWorkflowExecutionSignaled, ET.SignalExternalWorkflowExecutionFailed])
            return [self.ev(t, initiated_event_id=sid)]
        if r < 0.74:
            return [self.ev(ET.WorkflowExecutionCancelRequested)]
        if r < 0.76:
            # delete of an unknown initiated / scheduled ID: logged inconsistency, no error
            t = self.rng.choice([ET.ActivityTaskCompleted, ET.ChildWorkflowExecutionCompleted,
                                 ET.ExternalWorkflowExecutionSignaled, ET.ExternalWorkflowExecutionCancelRequested])
            if t == ET.ActivityTaskCompleted:
                return [self.ev(t, scheduled_event_id=999999)]
            return [self.ev(t, initiated_event_id=999999)]
        if r < 0.78:
            return [self.ev(ET.TimerFired, timer_id="no-such-timer")]
        return None


def random_workflow(rng: random.Random, w: int, target_len: int, multi_version=False, invalid=False,
                    domains=("domain-a", "domain-b", "unknown-domain"), force_close=None, caps=None) -> WorkflowHistory:
    k = _Walk(rng, w, multi_version, list(domains))
    k.caps = caps
    prev = None
    if rng.random() < 0.1:
        prev = [f"bin-{rng.randint(0, 3)}" for _ in range(rng.randint(0, 3))]
    k.start(prev_points=prev)
    binsum = f"bin-{rng.randint(0, 3)}"
    while k.eid < target_len and not k.closed:
        k.bump_version()
        if k.dec_sched is not None and k.dec_started is None:
            r = rng.random()
            if r < 0.9:
                k.emit([k.start_decision()])
            else:  # schedule-to-start timeout -> transient decision
                k.emit([k.ev(ET.DecisionTaskTimedOut, timeout_type=1)])
                k.dec_sched = None
                k.attempt += 1
            continue
        if k.dec_started is not None:
            r = rng.random()
            if r < 0.8:
                b = [k.ev(ET.DecisionTaskCompleted, scheduled_event_id=k.dec_sched, started_event_id=k.dec_started,
                          binary_checksum=rng.choice([binsum, binsum, "", f"bin-{rng.randint(0, 5)}"]))]
                k.dec_sched = k.dec_started = None
                k.attempt = 0
                b += k.decision_outputs()
                k.emit(b)
            elif r < 0.9:
                k.emit([k.ev(ET.DecisionTaskFailed)])
                k.dec_sched = k.dec_started = None
                k.attempt += 1
            else:
                k.emit([k.ev(ET.DecisionTaskTimedOut, timeout_type=0)])
                k.dec_sched = k.dec_started = None
                k.attempt += 1
            continue
        if k.attempt > 0 and rng.random() < 0.7:
            # the transient decision completes: its scheduled + started events are written together
            k.emit([k.sched_decision(attempt=k.attempt), k.start_decision()])
            continue
        ext = k.external()
        if ext is None:
            ext = [k.ev(ET.WorkflowExecutionSignaled)]
        if k.dec_sched is None and rng.random() < 0.8:
            ext.append(k.sched_decision())
        k.emit(ext)
    # close
    if force_close is not None and not k.closed:
        if k.dec_started is None:
            if k.dec_sched is None:
                k.emit([k.sched_decision()])
            k.emit([k.start_decision()])
        k.emit([k.ev(ET.DecisionTaskCompleted, scheduled_event_id=k.dec_sched, started_event_id=k.dec_started,
                     binary_checksum=binsum), k.ev(force_close)])
        k.closed = True
    if not k.closed:
        r = rng.random()
        if k.dec_started is not None and r < 0.6:
            closing = rng.choice([ET.WorkflowExecutionCompleted, ET.WorkflowExecutionFailed,
                                  ET.WorkflowExecutionCanceled, ET.WorkflowExecutionContinuedAsNew])
            b = [k.ev(ET.DecisionTaskCompleted, scheduled_event_id=k.dec_sched, started_event_id=k.dec_started,
                      binary_checksum=binsum), k.ev(closing)]
            k.emit(b)
        elif r < 0.75:
            k.emit([k.ev(rng.choice([ET.WorkflowExecutionTerminated, ET.WorkflowExecutionTimedOut]))])
        # else: left open
    if invalid:
        _inject_invalid(rng, k)
    return WorkflowHistory(batches=k.batches, domain_failover_version=rng.choice([0, 1, 5]),
                           workflow_id=f"wf-{w}", run_id=det_uuid("run", w), request_id=det_uuid("req", w),
                           branch_id=det_uuid("branch", w), now_ns=BASE_TS + 10 ** 15 + w)


def _inject_invalid(rng: random.Random, k: _Walk):
    """Append one batch that makes ApplyEvents fail in a specific way."""
    choice = rng.randrange(12)
    if choice == 0:
        k.emit([k.ev(ET.ActivityTaskStarted, scheduled_event_id=424242)])          # missing activity
    elif choice == 1:
        k.emit([k.ev(ET.ChildWorkflowExecutionStarted, initiated_event_id=424242)])  # missing child
    elif choice == 2:
        k.emit([k.ev(ET.DecisionTaskStarted, scheduled_event_id=424242)])          # decision not found
    elif choice == 3:
        k.version -= 1 if k.version > 0 else 0
        k.emit([k.ev(ET.MarkerRecorded)])                                          # lower version (maybe)
    elif choice == 4:
        e = k.ev(ET.MarkerRecorded)
        e.id = max(1, e.id - 5)                                                    # event id not increasing
        k.emit([e])
    elif choice == 5:
        e = k.ev(99)                                                               # unknown event type
        k.emit([e])
    elif choice == 6:
        k.emit([])                                                                 # empty history batch
    elif choice == 7:
        k.emit([k.ev(ET.WorkflowExecutionStarted, task_start_to_close_timeout_seconds=10)])  # Running -> Created
    elif choice == 8:
        k.emit([k.ev(ET.ActivityTaskScheduled, activity_id="x", domain="unknown-domain")])  # domain lookup
    elif choice == 9:
        e = k.ev(ET.MarkerRecorded)
        e.version = -7                                                             # invalid VH item (panic)
        k.emit([e])
    elif choice == 10:
        k.emit([k.ev(ET.WorkflowExecutionCompleted), k.ev(ET.DecisionTaskScheduled, start_to_close_timeout_seconds=5)])
    else:
        first = k.batches[0][0]                                                    # bad initiator
        first.attrs["first_decision_task_backoff_seconds"] = 5
        first.attrs["initiator"] = rng.choice([0, 7])


def mixed_histories(n: int, seed: int, mean_len: int = 40, multi_version=False, invalid_rate=0.0,
                    can_rate: float = 0.0) -> List[WorkflowHistory]:
    """n random workflows with lengths 10..2*mean_len-10 (mean ~mean_len)."""
    rng = random.Random(seed)
    out: List[WorkflowHistory] = []
    for w in range(n):
        target = rng.randint(10, max(11, 2 * mean_len - 10))
        out.append(random_workflow(rng, w, target, multi_version=multi_version, invalid=rng.random() < invalid_rate))
    if can_rate > 0:
        _attach_new_runs(rng, out, can_rate)
    return out


def _attach_new_runs(rng: random.Random, hs: List[WorkflowHistory], rate: float):
    """For closed-by-CAN workflows, append a new-run history (Started + DecisionScheduled batch)."""
    n0 = len(hs)
    for w in range(n0):
        h = hs[w]
        if not h.batches or not h.batches[-1]:
            continue
        last = h.batches[-1][-1]
        if last.event_type != ET.WorkflowExecutionContinuedAsNew or rng.random() > rate:
            continue
        nr = WorkflowHistory(batches=[[HistoryEvent(int(ET.WorkflowExecutionStarted), 1, last.version, last.timestamp + 1,
                                                    last.task_id + 1, {"task_start_to_close_timeout_seconds": 10}),
                                       HistoryEvent(int(ET.DecisionTaskScheduled), 2, last.version, last.timestamp + 2,
                                                    last.task_id + 2, {"start_to_close_timeout_seconds": 10})]],
                             domain_failover_version=h.domain_failover_version, workflow_id=h.workflow_id,
                             run_id=det_uuid("newrun", w), branch_id=det_uuid("nrbranch", w), now_ns=h.now_ns,
                             is_new_run=True)
        if rng.random() < 0.2:   # a broken new-run history: the outer CAN must fail with its error
            nr.batches[0][1].version = nr.batches[0][0].version - 1 if nr.batches[0][0].version > 0 else -5
        last.attrs["new_run"] = len(hs)
        hs.append(nr)


def zipf_lengths(rng: random.Random, n: int, alpha: float = 1.2, min_len: int = 10, max_len: int = 50_000):
    """History lengths ~ min_len * Zipf(alpha), truncated to max_len."""
    out = []
    for _ in range(n):
        u = rng.random()
        # inverse CDF of the continuous Pareto(alpha - 1) tail as a Zipf stand-in
        k = (1.0 - u) ** (-1.0 / (alpha - 1.0)) if alpha > 1.0 else 1.0 / max(1.0 - u, 1e-12)
        out.append(int(min(max_len, max(min_len, min_len * k))))
    return out


LONG_TAIL_CAPS = {"act": 32, "timer": 16, "child": 8, "rc": 4, "sig": 4}


def long_tail_histories(n: int, seed: int, alpha: float = 1.2, min_len: int = 10, max_len: int = 50_000,
                        run_cap: int = 10_000, multi_version=False, invalid_rate=0.0,
                        caps=LONG_TAIL_CAPS) -> List[WorkflowHistory]:
    """Config 4: n logical workflows with Zipf-distributed total lengths, continued-as-new every
    <= run_cap events.  Every run is its own history (replayed independently); a run closed by
    ContinuedAsNew carries the next run's first batch as its new-run history (state_builder.go:587-627).
    ``caps`` bounds the concurrently pending activities / timers / children / external requests
    (a long-running workflow keeps a bounded working set; None: unbounded random walk)."""
    rng = random.Random(seed)
    out: List[WorkflowHistory] = []
    links = []
    w = 0
    for total in zipf_lengths(rng, n, alpha, min_len, max_len):
        runs = []
        left = total
        while True:
            this = min(left, run_cap)
            left -= this
            more = left > 0
            h = random_workflow(rng, w, this, multi_version=multi_version,
                                invalid=(not more) and rng.random() < invalid_rate, domains=("domain-a", "domain-b"),
                                caps=caps,
                                force_close=ET.WorkflowExecutionContinuedAsNew if more else None)
            w += 1
            runs.append(h)
            last = h.batches[-1][-1] if h.batches and h.batches[-1] else None
            if not more or last is None or last.event_type != ET.WorkflowExecutionContinuedAsNew:
                break
        for a, b in zip(runs, runs[1:]):
            links.append((len(out) + runs.index(a), len(out) + runs.index(b)))
        out.extend(runs)
    for ia, ib in links:   # the next run's first batch is the CAN event's new-run history
        a, b = out[ia], out[ib]
        last = a.batches[-1][-1]
        nr = WorkflowHistory(batches=[[HistoryEvent(e.event_type, e.id, e.version, e.timestamp, e.task_id,
                                                    dict(e.attrs)) for e in b.batches[0]]],
                             domain_failover_version=b.domain_failover_version, workflow_id=a.workflow_id,
                             run_id=b.run_id, branch_id=det_uuid("nrbranch", ib), now_ns=a.now_ns, is_new_run=True)
        last.attrs["new_run"] = len(out)
        out.append(nr)
    return out
