"""Python image of ``include/cadence_replay.h``: constants, numpy row dtypes and ctypes structs.

Every dtype below must match the C struct byte for byte; ``check_layout()`` compares them with
``crr_sizeof()`` of the loaded library at bind time.
"""
import ctypes
import enum

import numpy as np

ABI_VERSION = 7

# common/constants.go:30-58
FIRST_EVENT_ID = 1
EMPTY_EVENT_ID = -23
EMPTY_VERSION = -24
ZERO_TIME = -(2 ** 63)          # Go time.Time{} sentinel in rows
SRC_NONE = -1
SRC_EMPTY_UUID = -2
NO_TOKEN = 0xFFFFFFFF


class EventType(enum.IntEnum):
    """types.EventType (common/types/shared.go:3272-3357)."""
    WorkflowExecutionStarted = 0
    WorkflowExecutionCompleted = 1
    WorkflowExecutionFailed = 2
    WorkflowExecutionTimedOut = 3
    DecisionTaskScheduled = 4
    DecisionTaskStarted = 5
    DecisionTaskCompleted = 6
    DecisionTaskTimedOut = 7
    DecisionTaskFailed = 8
    ActivityTaskScheduled = 9
    ActivityTaskStarted = 10
    ActivityTaskCompleted = 11
    ActivityTaskFailed = 12
    ActivityTaskTimedOut = 13
    ActivityTaskCancelRequested = 14
    RequestCancelActivityTaskFailed = 15
    ActivityTaskCanceled = 16
    TimerStarted = 17
    TimerFired = 18
    CancelTimerFailed = 19
    TimerCanceled = 20
    WorkflowExecutionCancelRequested = 21
    WorkflowExecutionCanceled = 22
    RequestCancelExternalWorkflowExecutionInitiated = 23
    RequestCancelExternalWorkflowExecutionFailed = 24
    ExternalWorkflowExecutionCancelRequested = 25
    MarkerRecorded = 26
    WorkflowExecutionSignaled = 27
    WorkflowExecutionTerminated = 28
    WorkflowExecutionContinuedAsNew = 29
    StartChildWorkflowExecutionInitiated = 30
    StartChildWorkflowExecutionFailed = 31
    ChildWorkflowExecutionStarted = 32
    ChildWorkflowExecutionCompleted = 33
    ChildWorkflowExecutionFailed = 34
    ChildWorkflowExecutionCanceled = 35
    ChildWorkflowExecutionTimedOut = 36
    ChildWorkflowExecutionTerminated = 37
    SignalExternalWorkflowExecutionInitiated = 38
    SignalExternalWorkflowExecutionFailed = 39
    ExternalWorkflowExecutionSignaled = 40
    UpsertWorkflowSearchAttributes = 41


EV_TYPE_COUNT = 42
EV_PAD = 63
ETYPE_MASK = 0x3F
BATCH_FIRST = 0x80
BATCH_LAST = 0x40


class State(enum.IntEnum):
    Created = 0
    Running = 1
    Completed = 2
    Zombie = 3
    Void = 4
    Corrupted = 5


class CloseStatus(enum.IntEnum):
    NONE = 0
    Completed = 1
    Failed = 2
    Canceled = 3
    Terminated = 4
    ContinuedAsNew = 5
    TimedOut = 6


class TimeoutType(enum.IntEnum):
    StartToClose = 0
    ScheduleToStart = 1
    ScheduleToClose = 2
    Heartbeat = 3


TTS_START_TO_CLOSE = 1
TTS_SCHEDULE_TO_START = 2
TTS_SCHEDULE_TO_CLOSE = 4
TTS_HEARTBEAT = 8

INITIATOR_NIL = -1
INITIATOR_DECIDER = 0
INITIATOR_RETRY_POLICY = 1
INITIATOR_CRON = 2

DOMAIN_NOT_SET = 0
DOMAIN_RESOLVED = 1
DOMAIN_UNKNOWN = -1


class Status(enum.IntEnum):
    OK = 0
    EMPTY_HISTORY = 1
    UNKNOWN_EVENT_TYPE = 2
    VH_LOWER_VERSION = 3
    VH_EVENT_ID_NOT_INCREASING = 4
    VH_INVALID_ITEM = 5
    VH_EMPTY = 6
    INVALID_STATE_TRANSITION = 7
    UNKNOWN_WORKFLOW_STATE = 8
    MISSING_ACTIVITY_INFO = 9
    MISSING_CHILD_INFO = 10
    DECISION_NOT_FOUND = 11
    DOMAIN_NOT_FOUND = 12
    BAD_INITIATOR = 13
    TIMER_SEQUENCE = 14
    REBUILD_LAST_ITEM = 15
    NEW_RUN_MISSING = 16
    MISSING_START_EVENT = 17          # ErrMissingWorkflowStartEvent (RefreshTasks)
    MISSING_COMPLETION_EVENT = 18     # ErrMissingWorkflowCompletionEvent (RefreshTasks)
    NDC_NO_LCA = 20
    NDC_LCA_NOT_IN_BRANCH = 21
    NDC_FIRST_ITEM_MISMATCH = 22
    NDC_RETRY_TASK = 23
    NDC_BAD_INDEX = 24
    CAPACITY = 100


EXEC_CANCEL_REQUESTED = 1
EXEC_RESET_POINTS_SET = 2
EXEC_CHECKSUM_VALID = 4

ROW_LIVE = 1
ROW_MAPPED = 2
ROW_CANCEL_REQUESTED = 4
ROW_HAS_RETRY = 8
ROW_RESETTABLE = 16

WF_FLAG_NEW_RUN = 1
WF_FLAG_REFRESH_TASKS = 2      # Rebuild's RefreshTasks state effects after the replay
WF_FLAG_RESUME = 4             # ApplyEvents onto the loaded state held in the output rows (in place)
IN_HAS_NEW_RUN = 1
IN_LDS_SMALL = 2
IN_WAVE_TAIL = 4
IN_EMIT_TASKS = 8
IN_TIERED = 16              # lane workflows ordered by expected live-set size (large_begin / wide_begin)
IN_HAS_RESUME = 32          # some workflow resumes a loaded state: the compact tiers continue it in LDS
IN_ADVANCED_VISIBILITY = 64  # RefreshTasks emits the search-attributes task
IN_STARTED_AUX = 128       # ActivityTaskStarted's aux = its scheduled event's act_side index (or -1)

# ---- numpy dtypes (byte-identical to the C structs) ------------------------------------------------
ACTIVITY_SIDE = np.dtype([
    ("schedule_to_start", "<i4"), ("schedule_to_close", "<i4"), ("start_to_close", "<i4"),
    ("heartbeat", "<i4"), ("has_retry_policy", "<i4"), ("expiration_interval", "<i4"),
    ("domain_status", "<i4"), ("reserved", "<i4")])

START_SIDE = np.dtype([
    ("decision_start_to_close", "<i4"), ("workflow_timeout", "<i4"), ("first_decision_backoff", "<i4"),
    ("initiator", "<i4"), ("parent_domain_status", "<i4"), ("prev_reset_key_off", "<u4"),
    ("prev_reset_count", "<i4"), ("attempt", "<i4"), ("expiration_ns", "<i8"), ("refresh_jitter", "<i8")])

WORKFLOW = np.dtype([
    ("ev_begin", "<i8"), ("ev_count", "<i4"), ("empty_batch_at", "<i4"),
    ("init_version", "<i8"), ("now_ns", "<i8"),
    ("start_token_off", "<u4"), ("start_token_len", "<u4"),
    ("final_token_off", "<u4"), ("final_token_len", "<u4"),
    ("rebuild_last_event_id", "<i8"), ("rebuild_last_event_version", "<i8"),
    ("act_base", "<i8"), ("timer_base", "<i8"), ("child_base", "<i8"), ("rc_base", "<i8"),
    ("sig_base", "<i8"), ("vh_base", "<i8"), ("rp_base", "<i8"),
    ("act_cap", "<i4"), ("timer_cap", "<i4"), ("child_cap", "<i4"), ("rc_cap", "<i4"),
    ("sig_cap", "<i4"), ("vh_cap", "<i4"), ("rp_cap", "<i4"), ("flags", "<i4"),
    ("task_base", "<i8"), ("task_cap", "<i4"), ("retention_days", "<i4")])

EXEC_ROW = np.dtype([
    ("status", "<i4"), ("fail_step", "<i4"), ("inconsistencies", "<i4"), ("flags", "<u4"),
    ("state", "<i4"), ("close_status", "<i4"), ("signal_count", "<i4"), ("decision_timeout", "<i4"),
    ("next_event_id", "<i8"), ("last_first_event_id", "<i8"), ("last_event_task_id", "<i8"),
    ("last_processed_event", "<i8"), ("completion_event_batch_id", "<i8"),
    ("decision_version", "<i8"), ("decision_schedule_id", "<i8"), ("decision_started_id", "<i8"),
    ("decision_attempt", "<i8"), ("decision_started_ts", "<i8"), ("decision_scheduled_ts", "<i8"),
    ("decision_orig_scheduled_ts", "<i8"), ("current_version", "<i8"),
    ("decision_request_src", "<i4"), ("start_src", "<i4"),
    ("n_activity", "<i4"), ("n_timer", "<i4"), ("n_child", "<i4"), ("n_rc", "<i4"), ("n_signal", "<i4"),
    ("n_vh_items", "<i4"), ("n_reset_points", "<i4"), ("token_src", "<i4"),
    ("checksum", "<u4"), ("payload_len", "<u4"), ("n_tasks", "<i4"), ("decision_start_to_close", "<i4"),
    ("expiration_ns", "<i8"), ("src_next", "<i4"), ("reserved", "<i4")])

ACTIVITY_ROW = np.dtype([
    ("schedule_id", "<i8"), ("version", "<i8"), ("scheduled_batch_id", "<i8"), ("scheduled_time", "<i8"),
    ("started_id", "<i8"), ("started_time", "<i8"), ("cancel_request_id", "<i8"),
    ("last_hb_timeout_vis_s", "<i8"), ("sched_src", "<i4"), ("started_src", "<i4"),
    ("schedule_to_start", "<i4"), ("schedule_to_close", "<i4"), ("start_to_close", "<i4"),
    ("heartbeat", "<i4"), ("timer_task_status", "<i4"), ("key", "<u4"), ("flags", "<u4"),
    ("attempt", "<i4"), ("last_heartbeat_time", "<i8")])

TIMER_ROW = np.dtype([
    ("started_id", "<i8"), ("version", "<i8"), ("expiry_time", "<i8"), ("task_status", "<i4"),
    ("key", "<u4"), ("src", "<i4"), ("flags", "<u4")])

CHILD_ROW = np.dtype([
    ("initiated_id", "<i8"), ("version", "<i8"), ("initiated_batch_id", "<i8"), ("started_id", "<i8"),
    ("src", "<i4"), ("started_src", "<i4"), ("flags", "<u4"), ("reserved", "<i4")])

INITIATED_ROW = np.dtype([
    ("initiated_id", "<i8"), ("version", "<i8"), ("initiated_batch_id", "<i8"), ("src", "<i4"),
    ("flags", "<u4")])

VH_ITEM = np.dtype([("event_id", "<i8"), ("version", "<i8")])

RESET_POINT_ROW = np.dtype([("src", "<i4"), ("prev_index", "<i4"), ("key", "<u4"), ("flags", "<u4")])

TASK_ROW = np.dtype([("kind", "<i4"), ("aux", "<i4"), ("version", "<i8"), ("visibility_ts", "<i8"),
                     ("event_id", "<i8"), ("attempt", "<i4"), ("src", "<i4")])


class TaskKind(enum.IntEnum):
    """crr_task_kind (transfer / timer tasks ApplyEvents generates)."""
    RecordWorkflowStarted = 1
    Decision = 2
    Activity = 3
    StartChild = 4
    CancelExecution = 5
    SignalExecution = 6
    UpsertSearchAttributes = 7
    CloseExecution = 8
    WorkflowTimeout = 16
    WorkflowBackoff = 17
    DecisionTimeout = 18
    ActivityTimeout = 19
    UserTimer = 20
    DeleteHistory = 21


BACKOFF_RETRY, BACKOFF_CRON = 0, 1

# NDC branch decisions (crr_ndc_prepare)
NDC_TASK = np.dtype([("branch_begin", "<u4"), ("branch_count", "<u4"), ("current_index", "<i4"),
                     ("incoming_begin", "<u4"), ("incoming_count", "<u4"), ("out_begin", "<u4"),
                     ("first_event_id", "<i8"), ("first_event_version", "<i8")])
NDC_BRANCH = np.dtype([("item_begin", "<u4"), ("item_count", "<u4")])
NDC_RESULT = np.dtype([("status", "<i4"), ("action", "<i4"), ("branch_index", "<i4"), ("lca_branch", "<i4"),
                       ("lca_event_id", "<i8"), ("lca_version", "<i8"), ("last_event_id", "<i8"),
                       ("last_version", "<i8"), ("new_current_index", "<i4"), ("new_item_count", "<i4"),
                       ("is_rebuilt", "<i4"), ("branch_changed", "<i4")])
NDC_APPEND, NDC_NEW_BRANCH, NDC_DUPLICATE = 0, 1, 2

SIZEOF_ORDER = [WORKFLOW, EXEC_ROW, ACTIVITY_ROW, TIMER_ROW, CHILD_ROW, INITIATED_ROW, VH_ITEM,
                RESET_POINT_ROW, ACTIVITY_SIDE, START_SIDE, NDC_TASK, NDC_RESULT, TASK_ROW]

# (name, dtype, numpy kind) of the event columns, in crr_events order
EVENT_COLUMNS = [("etype", np.uint8), ("event_id", np.int64), ("version", np.int64),
                 ("timestamp", np.int64), ("task_id", np.int64), ("ref", np.int64),
                 ("key", np.uint32), ("aux", np.int32)]
BYTES_PER_EVENT = sum(np.dtype(t).itemsize for _, t in EVENT_COLUMNS)   # 49

# output tables: (attribute, dtype, workflow base field, capacity field, exec count field)
TABLES = [("act", ACTIVITY_ROW, "act_base", "act_cap", "n_activity"),
          ("timer", TIMER_ROW, "timer_base", "timer_cap", "n_timer"),
          ("child", CHILD_ROW, "child_base", "child_cap", "n_child"),
          ("rc", INITIATED_ROW, "rc_base", "rc_cap", "n_rc"),
          ("sig", INITIATED_ROW, "sig_base", "sig_cap", "n_signal"),
          ("vh", VH_ITEM, "vh_base", "vh_cap", "n_vh_items"),
          ("rp", RESET_POINT_ROW, "rp_base", "rp_cap", "n_reset_points"),
          ("tasks", TASK_ROW, "task_base", "task_cap", "n_tasks")]   # written with IN_EMIT_TASKS only


# ---- ctypes structs -----------------------------------------------------------------------------------
class CNdcInputs(ctypes.Structure):
    _fields_ = [("tasks", ctypes.c_void_p), ("branches", ctypes.c_void_p), ("items", ctypes.c_void_p),
                ("n_tasks", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class CEvents(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name, _ in EVENT_COLUMNS]


class CInputs(ctypes.Structure):
    _fields_ = [("ev", CEvents), ("act_side", ctypes.c_void_p), ("start_side", ctypes.c_void_p),
                ("reset_keys", ctypes.c_void_p), ("arena", ctypes.c_void_p), ("wf", ctypes.c_void_p),
                ("n_wf", ctypes.c_uint32), ("stride", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("wave_begin", ctypes.c_uint32), ("large_begin", ctypes.c_uint32), ("compact_begin", ctypes.c_uint32),
                ("compact2_begin", ctypes.c_uint32), ("wide_begin", ctypes.c_uint32),
                ("big_begin", ctypes.c_uint32), ("hbm_begin", ctypes.c_uint32), ("digest_keys", ctypes.c_void_p),
                ("token_crc", ctypes.c_void_p)]


# the live-ID sidecar (crr_outputs.live_ids, ABI v6): one int64 column per pending map, addressed like its rows
ID_TABLES = ("act", "timer", "child", "rc", "sig")


class COutputs(ctypes.Structure):
    _fields_ = ([(name, ctypes.c_void_p) for name, *_ in [("exec",)] + [(t[0],) for t in TABLES] + [("scratch",), ("digest",)]]
                + [("live_ids", ctypes.c_void_p * len(ID_TABLES))])


# crr_replay's fused digest (crr_outputs.digest): stripes of partial sums (cadence_replay.h)
DIGEST_FIELDS = 7
DIGEST_STRIPES = 8
DIGEST_STRIDE = 16
DIGEST_WORDS = DIGEST_STRIPES * DIGEST_STRIDE


SCRATCH_EXTRA_WORDS = 64


def check_layout(lib):
    """Compare numpy dtype sizes with the library's sizeof() table."""
    lib.crr_sizeof.restype = ctypes.c_size_t
    lib.crr_sizeof.argtypes = [ctypes.c_int]
    for i, dt in enumerate(SIZEOF_ORDER):
        got = lib.crr_sizeof(i)
        if got != dt.itemsize:
            raise RuntimeError(f"ABI layout mismatch for struct #{i}: C {got} vs numpy {dt.itemsize}")
    for i, st in ((13, CInputs), (14, COutputs)):
        if lib.crr_sizeof(i) != ctypes.sizeof(st):
            raise RuntimeError(f"ABI layout mismatch for {st.__name__}: C {lib.crr_sizeof(i)} vs ctypes {ctypes.sizeof(st)}")
