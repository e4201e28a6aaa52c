/*
 * cadence_replay.h -- C ABI of the MI355X batched history-replay engine.
 *
 * This is the drop-in boundary for Cadence's mutable-state rebuild hot path:
 *
 *   service/history/execution/state_builder.go:41-51   StateBuilder.ApplyEvents
 *   service/history/execution/state_builder.go:90-648  stateBuilderImpl.ApplyEvents
 *   service/history/execution/mutable_state_builder.go:1751-3810  Replicate*Event
 *   service/history/execution/checksum.go:36-114       mutable-state checksum
 *
 * The reference is Go; its FFI for this path would be cgo.  Every entry point below takes
 * plain pointers and sizes (no torch / HIP-runtime types beyond an opaque stream handle) so
 * that a cgo shim can bind it one-to-one.
 *
 * Data model
 * ----------
 * A *batch* of workflows is replayed in one call.  Each workflow is a sequence of persisted
 * event batches (the unit ApplyEvents is called with; state_rebuilder.go:135-148).  Events are
 * flattened into structure-of-arrays columns (crr_events).  Event `k` of workflow `w` lives at
 * column index  wf[w].ev_begin + k * stride, where `stride` is 1 for the canonical
 * (contiguous-per-workflow) layout and 64 for the wave-interleaved layout the GPU kernel is
 * tuned for (64 workflows of similar length share one "group"; step k of all 64 is one
 * contiguous 64-element run, so every column load is fully coalesced).  Batch boundaries are
 * carried in the two high bits of the event-type byte.
 *
 * Strings never reach the device.  The host interns ActivityID / TimerID / BinaryChecksum into
 * per-workflow u32 keys (string equality preserved) and every string-valued output field is
 * returned as a *source reference* (the event step that supplied it), which the host shim
 * materialises.  Non-deterministic inputs of the reference (uuid.New(), timeSource.Now(),
 * the random branchID) are host-supplied per workflow.
 *
 * Pending activity / timer / child / request-cancel / signal maps, the version-history items
 * and the auto-reset-point list live in per-workflow slot tables ("workspace rows") addressed
 * with the same base + slot * stride rule.  After a call the first n_* slots of each table hold
 * the live rows sorted by their event ID, which is also the order the checksum encodes them in.
 */
#ifndef CADENCE_REPLAY_H_
#define CADENCE_REPLAY_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 5: status codes 17-18, CRR_IN_HAS_RESUME / CRR_IN_ADVANCED_VISIBILITY, crr_start_side.refresh_jitter,
 *    RefreshTasks' own task rows (task_cap), RefreshTasks' state effects without CRR_IN_EMIT_TASKS too,
 *    the fused digest (crr_inputs.digest_keys, crr_outputs.digest), crr_sizeof(13 / 14)
 * 6: the live-ID sidecar (crr_outputs.live_ids) */
#define CRR_ABI_VERSION 7

/* ---- constants restated from the reference ------------------------------------------------ */
/* common/constants.go:30-58 */
#define CRR_FIRST_EVENT_ID      1LL
#define CRR_EMPTY_EVENT_ID      (-23LL)
#define CRR_EMPTY_VERSION       (-24LL)
#define CRR_BUFFERED_EVENT_ID   (-123LL)
#define CRR_TRANSIENT_EVENT_ID  (-124LL)
/* Go time.Time{} (zero value) is not representable as Unix nanoseconds; rows use this sentinel. */
#define CRR_ZERO_TIME           ((int64_t)0x8000000000000000ULL)
/* "no source event" for string-valued fields; -2 = the constant common.EmptyUUID ("emptyUuid"). */
#define CRR_SRC_NONE            (-1)
#define CRR_SRC_EMPTY_UUID      (-2)

/* types.EventType, common/types/shared.go:3272-3357 (iota order). */
enum crr_event_type {
    CRR_EV_WORKFLOW_EXECUTION_STARTED = 0,
    CRR_EV_WORKFLOW_EXECUTION_COMPLETED = 1,
    CRR_EV_WORKFLOW_EXECUTION_FAILED = 2,
    CRR_EV_WORKFLOW_EXECUTION_TIMED_OUT = 3,
    CRR_EV_DECISION_TASK_SCHEDULED = 4,
    CRR_EV_DECISION_TASK_STARTED = 5,
    CRR_EV_DECISION_TASK_COMPLETED = 6,
    CRR_EV_DECISION_TASK_TIMED_OUT = 7,
    CRR_EV_DECISION_TASK_FAILED = 8,
    CRR_EV_ACTIVITY_TASK_SCHEDULED = 9,
    CRR_EV_ACTIVITY_TASK_STARTED = 10,
    CRR_EV_ACTIVITY_TASK_COMPLETED = 11,
    CRR_EV_ACTIVITY_TASK_FAILED = 12,
    CRR_EV_ACTIVITY_TASK_TIMED_OUT = 13,
    CRR_EV_ACTIVITY_TASK_CANCEL_REQUESTED = 14,
    CRR_EV_REQUEST_CANCEL_ACTIVITY_TASK_FAILED = 15,
    CRR_EV_ACTIVITY_TASK_CANCELED = 16,
    CRR_EV_TIMER_STARTED = 17,
    CRR_EV_TIMER_FIRED = 18,
    CRR_EV_CANCEL_TIMER_FAILED = 19,
    CRR_EV_TIMER_CANCELED = 20,
    CRR_EV_WORKFLOW_EXECUTION_CANCEL_REQUESTED = 21,
    CRR_EV_WORKFLOW_EXECUTION_CANCELED = 22,
    CRR_EV_REQUEST_CANCEL_EXTERNAL_INITIATED = 23,
    CRR_EV_REQUEST_CANCEL_EXTERNAL_FAILED = 24,
    CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_CANCEL_REQUESTED = 25,
    CRR_EV_MARKER_RECORDED = 26,
    CRR_EV_WORKFLOW_EXECUTION_SIGNALED = 27,
    CRR_EV_WORKFLOW_EXECUTION_TERMINATED = 28,
    CRR_EV_WORKFLOW_EXECUTION_CONTINUED_AS_NEW = 29,
    CRR_EV_START_CHILD_WORKFLOW_EXECUTION_INITIATED = 30,
    CRR_EV_START_CHILD_WORKFLOW_EXECUTION_FAILED = 31,
    CRR_EV_CHILD_WORKFLOW_EXECUTION_STARTED = 32,
    CRR_EV_CHILD_WORKFLOW_EXECUTION_COMPLETED = 33,
    CRR_EV_CHILD_WORKFLOW_EXECUTION_FAILED = 34,
    CRR_EV_CHILD_WORKFLOW_EXECUTION_CANCELED = 35,
    CRR_EV_CHILD_WORKFLOW_EXECUTION_TIMED_OUT = 36,
    CRR_EV_CHILD_WORKFLOW_EXECUTION_TERMINATED = 37,
    CRR_EV_SIGNAL_EXTERNAL_INITIATED = 38,
    CRR_EV_SIGNAL_EXTERNAL_FAILED = 39,
    CRR_EV_EXTERNAL_WORKFLOW_EXECUTION_SIGNALED = 40,
    CRR_EV_UPSERT_WORKFLOW_SEARCH_ATTRIBUTES = 41,
    CRR_EV_TYPE_COUNT = 42,
    CRR_EV_PAD = 63          /* padding slot in the interleaved layout: never replayed */
};
#define CRR_ETYPE_MASK        0x3F
#define CRR_ETYPE_BATCH_FIRST 0x80   /* event is history[0] of its ApplyEvents batch */
#define CRR_ETYPE_BATCH_LAST  0x40   /* event is history[len-1] of its ApplyEvents batch */

/* persistence.WorkflowState* / WorkflowCloseStatus*, common/persistence/dataManagerInterfaces.go:118-135 */
enum crr_workflow_state {
    CRR_STATE_CREATED = 0, CRR_STATE_RUNNING = 1, CRR_STATE_COMPLETED = 2,
    CRR_STATE_ZOMBIE = 3, CRR_STATE_VOID = 4, CRR_STATE_CORRUPTED = 5
};
enum crr_close_status {
    CRR_CLOSE_NONE = 0, CRR_CLOSE_COMPLETED = 1, CRR_CLOSE_FAILED = 2, CRR_CLOSE_CANCELED = 3,
    CRR_CLOSE_TERMINATED = 4, CRR_CLOSE_CONTINUED_AS_NEW = 5, CRR_CLOSE_TIMED_OUT = 6
};
/* types.TimeoutType, common/types/shared.go:8792-8799 == execution.TimerType */
enum crr_timeout_type {
    CRR_TIMEOUT_START_TO_CLOSE = 0, CRR_TIMEOUT_SCHEDULE_TO_START = 1,
    CRR_TIMEOUT_SCHEDULE_TO_CLOSE = 2, CRR_TIMEOUT_HEARTBEAT = 3
};
/* execution/timer_sequence.go:51-67 */
#define CRR_TIMER_TASK_STATUS_NONE     0
#define CRR_TIMER_TASK_STATUS_CREATED  1
#define CRR_TTS_CREATED_START_TO_CLOSE    1
#define CRR_TTS_CREATED_SCHEDULE_TO_START 2
#define CRR_TTS_CREATED_SCHEDULE_TO_CLOSE 4
#define CRR_TTS_CREATED_HEARTBEAT         8
/* types.ContinueAsNewInitiator, common/types/shared.go:1253-1258; -1 = nil pointer */
#define CRR_INITIATOR_NIL        (-1)
#define CRR_INITIATOR_DECIDER      0
#define CRR_INITIATOR_RETRY_POLICY 1
#define CRR_INITIATOR_CRON         2

/* Domain-cache lookups on the path resolve on the host; the device only sees the outcome. */
#define CRR_DOMAIN_NOT_SET   0   /* attribute domain name empty -> execution's own DomainID */
#define CRR_DOMAIN_RESOLVED  1   /* domain cache lookup succeeded                          */
#define CRR_DOMAIN_UNKNOWN (-1)  /* lookup fails -> EntityNotExists error from the cache   */

/* ---- per-workflow status (maps 1:1 onto the Go error returned by ApplyEvents) ------------- */
enum crr_status_code {
    CRR_OK = 0,
    CRR_ERR_EMPTY_HISTORY = 1,            /* InternalFailure  state_builder.go:98-100              */
    CRR_ERR_UNKNOWN_EVENT_TYPE = 2,       /* BadRequest       state_builder.go:629-630             */
    CRR_ERR_VH_LOWER_VERSION = 3,         /* BadRequest       versionHistory.go:204-209            */
    CRR_ERR_VH_EVENT_ID_NOT_INCREASING=4, /* BadRequest       versionHistory.go:211-216            */
    CRR_ERR_VH_INVALID_ITEM = 5,          /* panic            versionHistory.go:37-43              */
    CRR_ERR_VH_EMPTY = 6,                 /* BadRequest       versionHistory.go:303-308 (via UpdateCurrentVersion) */
    CRR_ERR_INVALID_STATE_TRANSITION = 7, /* InternalService  workflowExecutionInfo.go:45-165      */
    CRR_ERR_UNKNOWN_WORKFLOW_STATE = 8,   /* InternalService  workflowExecutionInfo.go:143-147     */
    CRR_ERR_MISSING_ACTIVITY_INFO = 9,    /* InternalService  mutable_state_builder.go:64-65       */
    CRR_ERR_MISSING_CHILD_INFO = 10,      /* InternalService  mutable_state_builder.go:66-67       */
    CRR_ERR_DECISION_NOT_FOUND = 11,      /* InternalFailure  mutable_state_decision_task_manager.go:211-214 */
    CRR_ERR_DOMAIN_NOT_FOUND = 12,        /* EntityNotExists  domain cache                         */
    CRR_ERR_BAD_INITIATOR = 13,           /* InternalService  mutable_state_task_generator.go:269-277 */
    CRR_ERR_TIMER_SEQUENCE = 14,          /* InternalService  timer_sequence.go:141-145,176-180    */
    CRR_ERR_REBUILD_LAST_ITEM = 15,       /* BadRequest       state_rebuilder.go:160-176           */
    CRR_ERR_NEW_RUN_MISSING = 16,         /* engine: CAN new-run workflow index out of range       */
    CRR_ERR_MISSING_START_EVENT = 17,     /* ErrMissingWorkflowStartEvent mutable_state_builder.go:1150-1155 (RefreshTasks) */
    CRR_ERR_MISSING_COMPLETION_EVENT = 18,/* ErrMissingWorkflowCompletionEvent :1085-1128 (RefreshTasks)      */
    /* NDC branch decisions (crr_ndc_prepare) */
    CRR_ERR_NDC_NO_LCA = 20,              /* BadRequest       versionHistory.go:270-272 "No joint point found" */
    CRR_ERR_NDC_LCA_NOT_IN_BRANCH = 21,   /* BadRequest       versionHistory.go:147-149 DuplicateUntilLCAItem  */
    CRR_ERR_NDC_FIRST_ITEM_MISMATCH = 22, /* BadRequest       versionHistory.go:474-476 AddVersionHistory      */
    CRR_ERR_NDC_RETRY_TASK = 23,          /* RetryTaskV2Error ndc/branch_manager.go:214-225 out-of-order batch */
    CRR_ERR_NDC_BAD_INDEX = 24,           /* BadRequest       versionHistory.go:442-444 invalid branch index   */
    CRR_ERR_CAPACITY = 100                /* engine: a slot table was sized too small by the host  */
};

/* ---- input ---------------------------------------------------------------------------------- */
/*
 * Event columns.  Per-type meaning of ref / key / aux (attribute getters cited):
 *   WorkflowExecutionStarted   aux = index into start side records
 *   DecisionTaskScheduled      ref = Attempt (int64), aux = StartToCloseTimeoutSeconds
 *   DecisionTaskStarted        ref = ScheduledEventID
 *   DecisionTaskCompleted      ref = StartedEventID, key = BinaryChecksum (0 == "")
 *   DecisionTaskTimedOut       aux = TimeoutType
 *   ActivityTaskScheduled      key = ActivityID, aux = index into activity side records
 *   ActivityTaskStarted / Completed / Failed / TimedOut / Canceled   ref = ScheduledEventID
 *   ActivityTaskCancelRequested key = ActivityID
 *   TimerStarted               key = TimerID, ref = StartToFireTimeoutSeconds
 *   TimerFired / TimerCanceled key = TimerID
 *   StartChildWorkflowExecutionInitiated  aux = domain status (CRR_DOMAIN_*)
 *   RequestCancelExternal...Initiated / SignalExternal...Initiated  aux = domain status
 *   child close/started, RC failed/cancel-requested, signal failed/signaled  ref = InitiatedEventID
 *   WorkflowExecutionContinuedAsNew       aux = workflow index of the new-run history (-1: none)
 */
typedef struct crr_events {
    const uint8_t*  etype;      /* crr_event_type | CRR_ETYPE_BATCH_* */
    const int64_t*  event_id;   /* HistoryEvent.ID        */
    const int64_t*  version;    /* HistoryEvent.Version   */
    const int64_t*  timestamp;  /* HistoryEvent.Timestamp (Unix ns) */
    const int64_t*  task_id;    /* HistoryEvent.TaskID    */
    const int64_t*  ref;
    const uint32_t* key;
    const int32_t*  aux;
} crr_events;

/* ActivityTaskScheduledEventAttributes fields the state machine reads (32 B). */
typedef struct crr_activity_side {
    int32_t schedule_to_start;      /* GetScheduleToStartTimeoutSeconds */
    int32_t schedule_to_close;      /* GetScheduleToCloseTimeoutSeconds */
    int32_t start_to_close;         /* GetStartToCloseTimeoutSeconds    */
    int32_t heartbeat;              /* GetHeartbeatTimeoutSeconds       */
    int32_t has_retry_policy;       /* RetryPolicy != nil               */
    int32_t expiration_interval;    /* RetryPolicy.GetExpirationIntervalInSeconds */
    int32_t domain_status;          /* CRR_DOMAIN_* for attributes.Domain */
    int32_t reserved;
} crr_activity_side;

/* WorkflowExecutionStartedEventAttributes fields the state machine reads (48 B). */
typedef struct crr_start_side {
    int32_t decision_start_to_close;   /* GetTaskStartToCloseTimeoutSeconds (DecisionStartToCloseTimeout) */
    int32_t workflow_timeout;          /* GetExecutionStartToCloseTimeoutSeconds */
    int32_t first_decision_backoff;    /* GetFirstDecisionTaskBackoffSeconds */
    int32_t initiator;                 /* CRR_INITIATOR_* */
    int32_t parent_domain_status;      /* CRR_DOMAIN_* of the ParentWorkflowDomain lookup (state_builder.go:137-147) */
    uint32_t prev_reset_key_off;       /* PrevAutoResetPoints binary checksums (keys) in crr_inputs.reset_keys */
    int32_t prev_reset_count;          /* -1 == PrevAutoResetPoints nil (or Points nil) */
    int32_t attempt;                   /* GetAttempt() (GenerateWorkflowStartTasks, task_generator.go:156) */
    int64_t expiration_ns;             /* GetExpirationTimestamp() (0: unset; mutable_state_builder.go:1800-1802) */
    int64_t refresh_jitter;            /* injected rand draw (>= 0) for RefreshTasks' decision backoff jitter:
                                          getNextDecisionTimeout's rand.Intn(jitterPortion) is taken as
                                          refresh_jitter % jitterPortion (task_generator.go:1051-1064) */
} crr_start_side;

/* Per-workflow descriptor (168 B). */
typedef struct crr_workflow {
    int64_t  ev_begin;          /* column index of step 0 */
    int32_t  ev_count;          /* number of real events */
    int32_t  empty_batch_at;    /* step index before which an empty batch sits (-1 none) */
    int64_t  init_version;      /* domainEntry.GetFailoverVersion() (mutable_state_builder.go:207) */
    int64_t  now_ns;            /* injected timeSource.Now().UnixNano() */
    uint32_t start_token_off;   /* branch token SetHistoryTree installs (state_builder.go:179-183) */
    uint32_t start_token_len;
    uint32_t final_token_off;   /* rebuild target token (state_rebuilder.go:150), len==UINT32_MAX: none */
    uint32_t final_token_len;
    int64_t  rebuild_last_event_id;       /* state_rebuilder.go:160 check, used when final token set */
    int64_t  rebuild_last_event_version;
    /* slot-table row bases (row = base + slot * stride) and capacities */
    int64_t  act_base;  int64_t timer_base; int64_t child_base; int64_t rc_base;
    int64_t  sig_base;  int64_t vh_base;    int64_t rp_base;
    int32_t  act_cap, timer_cap, child_cap, rc_cap, sig_cap, vh_cap, rp_cap;
    int32_t  flags;             /* CRR_WF_FLAG_* */
    int64_t  task_base;         /* emitted-task rows (CRR_IN_EMIT_TASKS): task_base + slot * stride */
    int32_t  task_cap;          /* rows at task_base for the tasks the replay generates; with
                                   CRR_WF_FLAG_REFRESH_TASKS they hold RefreshTasks' tasks instead, which can be one
                                   more (the search-attributes task, CRR_IN_ADVANCED_VISIBILITY): size it as the
                                   replay's upper bound + 1 (flatten.py).  Too few: CRR_ERR_CAPACITY */
    int32_t  retention_days;    /* domainEntry.GetRetentionDays (DeleteHistoryEventTask, task_generator.go:238-255) */
} crr_workflow;

#define CRR_WF_FLAG_NEW_RUN 1
/* After the replay (and the rebuild last-item check), Rebuild's RefreshTasks (state_rebuilder.go:183-186
 * -> mutable_state_task_refresher.go:77-496).  State effects, with or without CRR_IN_EMIT_TASKS: the Go
 * errors below, then every pending activity's TimerTaskStatus and user timer's TaskStatus cleared and
 * CreateNextActivityTimer / CreateNextUserTimer; a started decision with Attempt > 1 gets
 * getNextDecisionTimeout's DecisionTimeout (the jitter injected as crr_start_side.refresh_jitter; a replay
 * leaves every started decision at Attempt 0, mutable_state_decision_task_manager.go:207-223).  With CRR_IN_EMIT_TASKS the replay's own tasks are dropped
 * (CloseTransactionAsSnapshot) and the task rows hold RefreshTasks' tasks, in its order:
 *   workflow timeout (startTime = now_ns) [+ delayed decision], close tasks or record-started, the
 *   decision's schedule / start task, each pending not-started activity's transfer task, the activity
 *   timer, the user timer, each pending not-started child's, request-cancel's and signal's transfer task,
 *   the search-attributes task (CRR_IN_ADVANCED_VISIBILITY).
 * Go ranges over maps for the activity / child / request-cancel / signal groups (an unspecified order);
 * here each group is in ascending event ID.  The start event is the event with ID 1 of this call's
 * history (GetStartEvent), the close event the one with ID NextEventID - 1 in the completion batch
 * (GetCompletionEvent, read from the store); a missing one fails the call (CRR_ERR_MISSING_*_EVENT at
 * fail_step = ev_count).  The decision schedule-to-start timer follows the default dynamic config
 * (NormalDecisionScheduleToStartMaxAttempts = 0: none). */
#define CRR_WF_FLAG_REFRESH_TASKS 2
/* ApplyEvents onto a LOADED mutable state (NewStateBuilder(shard, logger, mutableState, ...) with the
 * state mutableStateBuilder.Load (mutable_state_builder.go:306-349) built from persistence; the passive
 * replication path ndc/history_replicator.go:385-460 -> stateBuilder.ApplyEvents :396).  On entry
 * out.exec[w] and slots 0..n-1 of the workflow's slot tables hold the loaded state (the image this
 * engine writes: live rows, any order); the call continues from it and rewrites them in place, as
 * ApplyEvents mutates the caller-owned MutableState.  Read from the exec row: every WorkflowExecutionInfo
 * field of the row, the n_* counts, token_src (1: the descriptor's start token is the loaded current
 * branch token), decision_start_to_close, expiration_ns and src_next (the provenance offset: step s of
 * this call is written as src_next + s).  As in Load, currentVersion starts at EmptyVersion and every
 * loaded activity is mapped by its ActivityID (duplicates: the latest scheduled one).  Capacities must
 * cover the loaded rows plus this call's inserts. */
#define CRR_WF_FLAG_RESUME 4

typedef struct crr_inputs {
    crr_events               ev;
    const crr_activity_side* act_side;
    const crr_start_side*    start_side;
    const uint32_t*          reset_keys;   /* interned binary checksums of PrevAutoResetPoints */
    const uint8_t*           arena;        /* branch-token bytes */
    const crr_workflow*      wf;
    uint32_t                 n_wf;
    uint32_t                 stride;       /* 1 (canonical) or 64 (wave-interleaved) */
    uint32_t                 flags;        /* CRR_IN_* */
    uint32_t                 wave_begin;   /* CRR_IN_WAVE_TAIL: workflows [wave_begin, n_wf) are long
                                              histories laid out contiguously (stride 1), replayed one
                                              per wavefront; [0, wave_begin) use `stride` */
    /* CRR_IN_TIERED: lane workflows [0, lanes) ordered by expected live-set size in segments replayed
       by the LDS tier that holds them (each boundary a multiple of 64 or the lane count):
         [0, large_begin)               <= 1 pending entry per map             (1-slot LDS tier)
         [large_begin, compact_begin)   <= 2 activities / timers / reset points (2-slot LDS tier)
         [compact_begin, compact2_begin) compact tier 1 (4 / 3 / 2 / 1 / 1 / 4 slots)
         [compact2_begin, wide_begin)    compact tier 2 (8 / 5 / 3 / 3 / 3 / 8 slots)
         [wide_begin, hbm_begin)         compact tier 3 (12 / 8 / 6 / 4 / 4 / 8 slots)
         [hbm_begin, lanes)              more: the workflow's own HBM rows
       (a loaded state, CRR_WF_FLAG_RESUME, belongs in a compact segment or [hbm_begin, lanes): the 1- and
       2-slot tiers rebuild rows from this call's events only and hand one to the general path)
       (hbm_begin below wide_begin, e.g. 0, reads as wide_begin: no compact tier 3 segment)
       (activity / timer / child / request-cancel / signal / reset-point slots; flatten.py) */
    uint32_t                 large_begin;
    uint32_t                 compact_begin;
    uint32_t                 compact2_begin;
    uint32_t                 wide_begin;
    uint32_t                 big_begin;    /* long-tail workflows [big_begin, n_wf) are expected to outgrow
                                              the fast kernels' per-wave arenas (replayed concurrently
                                              with the 57-KB arena); n_wf: none */
    uint32_t                 hbm_begin;
    /* The job's digest (the one collective of a multi-GPU run), folded into the replay launch:
       per workflow the identity key the digest binds its result to (e.g. a hash of the workflow ID), in batch
       order; NULL (with crr_outputs.digest NULL): no digest. */
    const uint64_t*          digest_keys;
    /* (ABI v7) Per workflow (batch order) the raw CRC of its start branch token -- the CRC-32 register after
       the token's bytes from a zero register, no final inversion: what the token contributes to the
       checksum's GenerateCRC32 (crc.go:35-54) -- as crr_token_crc writes it once the arena is in HBM (a token
       is fixed for its branch, so the caller computes it once per token).  A 96-byte start token (the
       HistoryBranch NewHistoryBranchToken writes) is then spliced into the checksum by a 32x32 GF(2) shift
       of the register instead of being read and hashed byte by byte; NULL, other lengths and final tokens
       (rebuilds): the token's bytes as before.  Results never depend on it. */
    const uint32_t*          token_crc;
} crr_inputs;

#define CRR_IN_HAS_NEW_RUN 1u   /* some workflow carries CRR_WF_FLAG_NEW_RUN: launch phase 0 */
#define CRR_IN_LDS_SMALL   2u   /* hint: live sets are small (<= 1 pending entry per map): use the
                                   3-blocks/CU LDS tier; workflows that outgrow it are replayed by
                                   the general path, so the hint affects speed only */
#define CRR_IN_WAVE_TAIL   4u   /* length bucketing (stride-64 batches only): workflows
                                   [wave_begin, n_wf) are replayed one per wavefront */
#define CRR_IN_EMIT_TASKS  8u   /* write the transfer / timer tasks ApplyEvents generates (crr_task_row) */
#define CRR_IN_TIERED     16u   /* stride-64 batches: lane workflows are ordered by expected live-set
                                   size (large_begin / wide_begin); each segment is launched with the
                                   LDS tier that holds it (1, 2 or 8 entries per map).  A hint like
                                   CRR_IN_LDS_SMALL (which it overrides): speed only, never results */
#define CRR_IN_ADVANCED_VISIBILITY 64u /* config.AdvancedVisibilityWritingMode != off: RefreshTasks also emits
                                   the search-attributes task (mutable_state_task_refresher.go:160-167) */
#define CRR_IN_STARTED_AUX 128u /* (stride-64 batches) every ActivityTaskStarted event's aux holds the act_side
                                   index of its ActivityTaskScheduled event in this call -- the event d = ID -
                                   ScheduledEventID steps before it, when that one is an ActivityTaskScheduled with
                                   ID ScheduledEventID -- or -1 (flatten.interleave, crr_ingest_layout).  The compact
                                   tiers then read the scheduled event's timeouts straight from it instead of first
                                   gathering that event's aux: a layout hint, results never depend on it */
#define CRR_IN_HAS_RESUME 32u   /* some workflow carries CRR_WF_FLAG_RESUME (CRR_IN_TIERED batches): the
                                   compact tiers (and the long-tail kernel) run the instantiations that
                                   continue loaded states.  Without it -- or for a loaded state in the 1- or
                                   2-slot segments -- the general path replays it over its HBM rows: speed
                                   only, never results */

/* ---- output rows ---------------------------------------------------------------------------- */
/* WorkflowExecutionInfo numeric image + engine status (208 B).  "step" / "*_src" values below are
 * provenance references: src_next of the resumed state (0 for a replay from scratch) + the step index
 * of the event in this call's history. */
typedef struct crr_exec_row {
    int32_t  status;                 /* crr_status_code */
    int32_t  fail_step;              /* step index of the failing event, or -1 */
    int32_t  inconsistencies;        /* logDataInconsistency() calls (mutable_state_builder.go:4720) */
    uint32_t flags;                  /* CRR_EXEC_* */
    int32_t  state, close_status;
    int32_t  signal_count;           /* int32 SignalCount */
    int32_t  decision_timeout;       /* int32 DecisionTimeout */
    int64_t  next_event_id, last_first_event_id, last_event_task_id, last_processed_event;
    int64_t  completion_event_batch_id;
    int64_t  decision_version, decision_schedule_id, decision_started_id, decision_attempt;
    int64_t  decision_started_ts, decision_scheduled_ts, decision_orig_scheduled_ts;
    int64_t  current_version;        /* in-memory currentVersion */
    int32_t  decision_request_src;   /* DecisionRequestID: step of DecisionTaskStarted, or CRR_SRC_EMPTY_UUID */
    int32_t  start_src;              /* step of the (last) WorkflowExecutionStarted event, or -1 */
    int32_t  n_activity, n_timer, n_child, n_rc, n_signal, n_vh_items, n_reset_points;
    int32_t  token_src;              /* 0: none (empty token), 1: start token, 2: final token */
    uint32_t checksum;               /* crc32.ChecksumIEEE of the thriftrw payload (crc.go:46) */
    uint32_t payload_len;            /* bytes the checksum was computed over (0x59 preamble included) */
    int32_t  n_tasks;                /* task rows written (CRR_IN_EMIT_TASKS) */
    int32_t  decision_start_to_close;/* executionInfo.DecisionStartToCloseTimeout (transient decisions) */
    int64_t  expiration_ns;          /* executionInfo.ExpirationTime, Unix ns (0: unset) */
    int32_t  src_next;               /* provenance space: the *_src / fail_step values of this row are
                                        < src_next (= the resumed row's src_next + this call's events) */
    int32_t  reserved;
} crr_exec_row;                      /* 208 B */

#define CRR_EXEC_CANCEL_REQUESTED  1u
#define CRR_EXEC_RESET_POINTS_SET  2u   /* AutoResetPoints != nil */
#define CRR_EXEC_CHECKSUM_VALID    4u

/* persistence.ActivityInfo numeric image (112 B). */
typedef struct crr_activity_row {
    int64_t  schedule_id, version, scheduled_batch_id, scheduled_time;
    int64_t  started_id, started_time;          /* started_time == CRR_ZERO_TIME until started */
    int64_t  cancel_request_id;
    int64_t  last_hb_timeout_vis_s;             /* LastHeartbeatTimeoutVisibilityInSeconds */
    int32_t  sched_src, started_src;            /* ActivityID/TaskList/... from sched_src; RequestID from started_src */
    int32_t  schedule_to_start, schedule_to_close, start_to_close, heartbeat;
    int32_t  timer_task_status;
    uint32_t key;                                /* interned ActivityID */
    uint32_t flags;                              /* CRR_ROW_* */
    int32_t  attempt;                            /* ActivityInfo.Attempt (0 on the replay path) */
    int64_t  last_heartbeat_time;                /* LastHeartBeatUpdatedTime (== started_time on replay) */
} crr_activity_row;

/* persistence.TimerInfo numeric image (40 B). */
typedef struct crr_timer_row {
    int64_t  started_id, version, expiry_time;
    int32_t  task_status;
    uint32_t key;                                /* interned TimerID */
    int32_t  src;                                /* step of TimerStarted */
    uint32_t flags;
} crr_timer_row;

/* persistence.ChildExecutionInfo numeric image (48 B). CreateRequestID = injected uuid(src). */
typedef struct crr_child_row {
    int64_t  initiated_id, version, initiated_batch_id, started_id;
    int32_t  src, started_src;
    uint32_t flags;
    int32_t  reserved;
} crr_child_row;

/* persistence.RequestCancelInfo / SignalInfo numeric image (32 B). Request IDs = injected uuid(src). */
typedef struct crr_initiated_row {
    int64_t  initiated_id, version, initiated_batch_id;
    int32_t  src;
    uint32_t flags;
} crr_initiated_row;

typedef struct crr_vh_item { int64_t event_id, version; } crr_vh_item;

/* types.ResetPointInfo provenance (16 B): a previous point from the start event or a new point. */
typedef struct crr_reset_point_row {
    int32_t  src;        /* step of DecisionTaskCompleted (new) or of WorkflowExecutionStarted (prev) */
    int32_t  prev_index; /* index into the start event's PrevAutoResetPoints, or -1 for a new point */
    uint32_t key;        /* interned binary checksum */
    uint32_t flags;      /* CRR_ROW_RESETTABLE */
} crr_reset_point_row;

#define CRR_ROW_LIVE             1u
#define CRR_ROW_MAPPED           2u   /* activity: pendingActivityIDToEventID[ActivityID] == ScheduleID */
#define CRR_ROW_CANCEL_REQUESTED 4u
#define CRR_ROW_HAS_RETRY        8u
#define CRR_ROW_RESETTABLE      16u

/* Transfer / timer tasks ApplyEvents generates, one row per task in the order
 * the Go code adds them: the task-generator calls of state_builder.go:157-625
 * (mutable_state_task_generator.go:143-612) and the per-batch timer epilogue (timer_sequence.go:127-199).
 * Strings (task list, target domain / workflow / run) come from the event at step `src`; what depends
 * on cluster metadata -- whether a child / cancel / signal task is cross-cluster
 * (isCrossClusterTask) and the shape of the close tasks (getTargetCluster / getParentCluster) --
 * is decided by the host from CRR_TASK_CLOSE_EXECUTION and the target domain. */
enum crr_task_kind {
    CRR_TASK_RECORD_WORKFLOW_STARTED = 1,   /* transfer: version = start event version            */
    CRR_TASK_DECISION = 2,                  /* transfer: event_id = ScheduleID, version = decision  */
    CRR_TASK_ACTIVITY = 3,                  /* transfer: event_id = ScheduleID                      */
    CRR_TASK_START_CHILD = 4,               /* transfer: event_id = InitiatedID                     */
    CRR_TASK_CANCEL_EXECUTION = 5,          /* transfer: event_id = InitiatedID                     */
    CRR_TASK_SIGNAL_EXECUTION = 6,          /* transfer: event_id = InitiatedID                     */
    CRR_TASK_UPSERT_SEARCH_ATTRIBUTES = 7,  /* transfer: version = current version                  */
    CRR_TASK_CLOSE_EXECUTION = 8,           /* transfer: version = close event version              */
    CRR_TASK_WORKFLOW_TIMEOUT = 16,         /* timer                                                */
    CRR_TASK_WORKFLOW_BACKOFF = 17,         /* timer: aux = WorkflowBackoffTimeoutType              */
    CRR_TASK_DECISION_TIMEOUT = 18,         /* timer: aux = TimerType, event_id = ScheduleID         */
    CRR_TASK_ACTIVITY_TIMEOUT = 19,         /* timer: aux = TimerType, event_id = ScheduleID         */
    CRR_TASK_USER_TIMER = 20,               /* timer: event_id = TimerStarted event ID              */
    CRR_TASK_DELETE_HISTORY = 21            /* timer: close timestamp + retention                   */
};
/* persistence.WorkflowBackoffTimeoutType* (dataManagerInterfaces.go) */
#define CRR_BACKOFF_RETRY 0
#define CRR_BACKOFF_CRON  1

typedef struct crr_task_row {
    int32_t kind;             /* crr_task_kind */
    int32_t aux;
    int64_t version;
    int64_t visibility_ts;    /* timer tasks (Unix ns); 0 for transfer tasks */
    int64_t event_id;
    int32_t attempt;
    int32_t src;              /* step of the event the task's strings come from (-1: none) */
} crr_task_row;               /* 40 B */

typedef struct crr_outputs {
    crr_exec_row*        exec;      /* [n_wf], indexed by workflow */
    crr_activity_row*    act;       /* slot tables, rows addressed by crr_workflow bases */
    crr_timer_row*       timer;
    crr_child_row*       child;
    crr_initiated_row*   rc;
    crr_initiated_row*   sig;
    crr_vh_item*         vh;
    crr_reset_point_row* rp;
    crr_task_row*        tasks;     /* CRR_IN_EMIT_TASKS only (else may be NULL) */
    uint32_t*            scratch;   /* engine scratch: >= 2 * n_wf + 64 words, zero-filled before the
                                       first call that uses it; every call leaves its counters zeroed */
    int64_t*             digest;    /* NULL, or CRR_DIGEST_WORDS int64 (device): this call's digest, below */
    /* ABI v6: the live-ID sidecar (NULL: not kept).  One int64 column per pending map -- 0 activity
       (ScheduleID), 1 timer (StartedID), 2 child, 3 request-cancel, 4 signal (InitiatedID) -- addressed like
       that map's rows (base + slot * stride, the crr_workflow bases), each at least as long as its row table.
       crr_replay writes, for every workflow it finalises with status CRR_OK, the IDs of slots 0..n-1 (the
       checksum's ID lists: the live rows' IDs in ascending order), so a reader of the IDs alone -- crr_checksum
       (the Load verify path) -- reads 8 dense bytes per row instead of one cache line of each AoS row.  All
       five set or none. */
    int64_t*             live_ids[5];
} crr_outputs;

/* crr_replay's digest (crr_outputs.digest, with crr_inputs.digest_keys): CRR_DIGEST_STRIPES partial sums of
 * CRR_DIGEST_FIELDS int64 fields, stripe k at digest[k * CRR_DIGEST_STRIDE]; the digest is the field-wise
 * sum over the stripes, every sum wrapping mod 2^64 (so an all-reduce SUM of the whole buffer across ranks,
 * summed over stripes afterwards, is the job's digest).  crr_replay zeroes the buffer first (an empty
 * batch, n_wf == 0, too: an empty rank's buffer is all zeros when it joins the all-reduce).  Per workflow
 * with key k, ok = (status == CRR_OK):
 *   0 ok ? ev_count : 0      1 ok      2 !ok      3 ok ? checksum : 0      4 ok ? k ^ checksum : 0
 *   5 inconsistencies        6 ok ? 0 : k ^ ((uint64)(uint32)status << 32 | (uint32)fail_step)
 * (cadence_amd/dist.py digest_numpy is the host restatement). */
#define CRR_DIGEST_FIELDS  7
#define CRR_DIGEST_STRIPES 8
#define CRR_DIGEST_STRIDE  16    /* int64 per stripe: one 128-byte line each */
#define CRR_DIGEST_WORDS   (CRR_DIGEST_STRIPES * CRR_DIGEST_STRIDE)

/* ---- NDC branch decisions ------------------------------------------------------
 * branchManagerImpl.prepareVersionHistory (service/history/ndc/branch_manager.go:87-149) for a batch
 * of replication tasks: FindLCAVersionHistoryIndexAndItem (versionHistory.go:501-528) over the local
 * VersionHistories, IsLCAAppendable (:275-287), DuplicateUntilLCAItem (:142-172), verifyEventsOrder
 * (branch_manager.go:199-225), AddVersionHistory (:450-498) for a new branch, plus IsRebuilt
 * (:545-571).  The buffered-events flush (:169-196) and ForkHistoryBranch (the new branch token)
 * stay on the host: the result names the base branch and fork point (lca_event_id + 1). */
typedef struct crr_ndc_task {
    uint32_t branch_begin;        /* local VersionHistories = branches[branch_begin, +branch_count) */
    uint32_t branch_count;
    int32_t  current_index;       /* VersionHistories.CurrentVersionHistoryIndex */
    uint32_t incoming_begin;      /* incoming VersionHistory = items[incoming_begin, +incoming_count) */
    uint32_t incoming_count;
    uint32_t out_begin;           /* new-branch items go to out_items[out_begin...] (room: the longest local branch) */
    int64_t  first_event_id;      /* the task's first event (ID, version) */
    int64_t  first_event_version;
} crr_ndc_task;

typedef struct crr_ndc_branch { uint32_t item_begin, item_count; } crr_ndc_branch;

typedef struct crr_ndc_inputs {
    const crr_ndc_task*   tasks;
    const crr_ndc_branch* branches;
    const crr_vh_item*    items;
    uint32_t              n_tasks;
    uint32_t              reserved;
} crr_ndc_inputs;

#define CRR_NDC_APPEND     0   /* doContinue, append to local branch `branch_index` */
#define CRR_NDC_NEW_BRANCH 1   /* doContinue on a new branch (index `branch_index`) forked from `lca_branch` */
#define CRR_NDC_DUPLICATE  2   /* !doContinue, no error: the batch was already applied */

typedef struct crr_ndc_result {
    int32_t status;               /* crr_status_code (CRR_OK or the error prepareVersionHistory returns) */
    int32_t action;               /* CRR_NDC_* (CRR_NDC_DUPLICATE, i.e. !doContinue, when status != CRR_OK) */
    int32_t branch_index;         /* branch the batch applies to */
    int32_t lca_branch;           /* branch holding the LCA (FindLCAVersionHistoryIndexAndItem) */
    int64_t lca_event_id, lca_version;
    int64_t last_event_id, last_version;   /* last item of the branch the order check used (RetryTaskV2 hint) */
    int32_t new_current_index;    /* CurrentVersionHistoryIndex after AddVersionHistory */
    int32_t new_item_count;       /* items of the new branch (DuplicateUntilLCAItem) at out_items[out_begin] */
    int32_t is_rebuilt;           /* IsRebuilt() of the local histories */
    int32_t branch_changed;       /* AddVersionHistory switched the current branch */
} crr_ndc_result;

/* ---- entry points ----------------------------------------------------------------------------- */
/* All pointers in crr_inputs / crr_outputs are DEVICE pointers (HBM resident).  `stream` is a
 * hipStream_t (NULL: default stream).  Returns 0 on successful launch, a negative value on an
 * invalid argument, or the positive hipError_t of a failed launch.  Per-workflow outcomes are in
 * crr_exec_row.status (first error aborts that workflow, state stays partially applied exactly as
 * the Go code leaves it -- state_builder.go returns at the first error, there is no rollback).
 *
 * Replaces: StateBuilder.ApplyEvents for a whole batch of workflows
 *           (state_builder.go:90-648, driven per batch by state_rebuilder.go:214-236 /
 *            ndc/history_replicator.go:292,396,650), plus generateMutableStateChecksum
 *           (checksum.go:36-43 via mutable_state_builder.go:4641-4651).
 * CAN new-run histories (crr_workflow.flags & CRR_WF_FLAG_NEW_RUN) are replayed in a first
 * launch, the rest in a second one, so a ContinuedAsNew event can observe its nested replay's
 * outcome (state_builder.go:587-612). */
int crr_replay(const crr_inputs* in, const crr_outputs* out, void* stream);

/* Recompute checksums of already-replayed rows (the Load verify path,
 * mutable_state_builder.go:334-348 -> checksum.go:45-54).  Writes checksums[n_wf].  With the live-ID
 * sidecar set (crr_outputs.live_ids, as the replay that wrote the rows left it) the ID lists are read from
 * it, else from the rows. */
int crr_checksum(const crr_inputs* in, const crr_outputs* out, uint32_t* checksums, void* stream);

/* crr_inputs.token_crc: the raw CRC of every workflow's start token (in->arena at start_token_off /
 * start_token_len) into crc[n_wf], on `stream`. */
int crr_token_crc(const crr_inputs* in, uint32_t* crc, void* stream);

/* Batched prepareVersionHistory over device arrays (one result per task). */
int crr_ndc_prepare(const crr_ndc_inputs* in, crr_ndc_result* results, crr_vh_item* out_items, void* stream);

/* Select the HIP device for subsequent calls from this thread (hipSetDevice: HIP's selection is per
 * host thread).
 *
 * Thread model.  Every entry point may be called from any host thread, concurrently.  A call on a
 * non-NULL stream runs on that stream's device whatever the calling thread has selected (the thread's
 * selection is restored on return), so a cgo caller whose goroutine migrates between OS threads needs
 * no runtime.LockOSThread as long as it passes its own stream; with a NULL stream the call uses the
 * thread's current device (pin the goroutine: INTEGRATION.md §4).  Launch state -- the side streams the
 * tier segments fork onto, the timing events -- is kept per device, created on first use and guarded
 * by a per-device mutex for the duration of a call's enqueue; crr_last_kernel_ms / crr_timing_* /
 * crr_segment_* report the last calls on the current device.  crr_release destroys that state. */
int crr_set_device(int device);

/* Teardown: synchronise and destroy every device's side streams and events (no call may be in flight).
 * A later call recreates what it needs.  Returns 0, or -1 if a device could not be selected. */
int crr_release(void);

/* Library / ABI version; struct sizes for binding-time layout checks. */
int crr_abi_version(void);
size_t crr_sizeof(int which);   /* 0 workflow, 1 exec row, 2 activity, 3 timer, 4 child, 5 initiated,
                                   6 vh item, 7 reset point, 8 activity side, 9 start side,
                                   10 ndc task, 11 ndc result, 12 task row, 13 crr_inputs, 14 crr_outputs */

/* Host-side CRC32-IEEE (hash/crc32.ChecksumIEEE) used by the shim's standalone verify. */
uint32_t crr_crc32_ieee(const uint8_t* data, size_t len);

/* Last launch's kernel time in milliseconds measured with HIP events on `stream`
 * (0: phase 0, new-run histories; 1: phase 1, the rest, all of its kernels; 2: the phase-1
 * fast-path (lane/wave LDS) kernel alone).  Valid after the stream has synchronised; -1 if absent. */
float crr_last_kernel_ms(int which);

/* Measured region for benchmarks: after crr_timing_begin, every crr_replay on this thread records
 * its phase-1 fast-path kernel with its own HIP event pair on the launch stream (up to 512 launches,
 * no synchronisation between launches).  crr_timing_read ends the region, waits for the events and
 * writes up to `cap` per-launch durations (ms); returns how many, or -1 on a HIP error.  Inside the
 * region crr_last_kernel_ms returns -1 (the per-call phase events are not recorded). */
int crr_timing_begin(void);
int crr_timing_read(float* ms, int cap);

/* Diagnostics: with crr_segment_timing(1), each CRR_IN_TIERED phase-1 launch group records when each
 * of its concurrent streams finished (side streams 0..5: 2-slot tier, compact tier 3 + HBM rows, big
 * tail, compact tier 1, compact tier 2, wave tail; 6: the caller's stream, 1-slot tier);
 * crr_segment_ms writes the 7 times (ms after the fork) of the last group once it completed. */
int crr_segment_timing(int on);
int crr_segment_ms(float* ms, int cap);

/* ---- live-row compaction for the download --------------------------------------------------------
 * After crr_replay (same inputs / outputs, same stream): every workflow's live rows -- slots 0..n-1 of
 * its slot-table regions, n = its exec-row count clamped to [0, capacity] -- gathered into dense
 * per-table buffers in workflow (batch) order, with each table's exclusive prefix over workflows, so a
 * caller copies to the host only the rows it persists.  Replaces the persisted-snapshot walk over the
 * pending maps (mutableStateBuilder.CloseTransactionAsSnapshot, mutable_state_builder.go:4033-4100).
 * Tables: 0 activity, 1 timer, 2 child, 3 request-cancel, 4 signal, 5 version-history items,
 * 6 reset points, 7 tasks (CRR_IN_EMIT_TASKS only).  rows[t] NULL: table t only counted.
 * Returns 0 on successful launch, -1 on an invalid argument, else the hipError_t. */
#define CRR_COMPACT_TABLES 8
typedef struct crr_compact_out {
    void*    rows[CRR_COMPACT_TABLES];  /* device, 8-byte aligned, >= the table's total live rows each */
    int64_t* offsets;                   /* device [CRR_COMPACT_TABLES][n_wf + 1]; [t][n_wf] = the total */
    void*    scratch;                   /* device, crr_compact_scratch_bytes(n_wf) bytes */
} crr_compact_out;
size_t crr_compact_scratch_bytes(uint32_t n_wf);
int crr_compact_rows(const crr_inputs* in, const crr_outputs* out, const crr_compact_out* dst, void* stream);

/* ---- narrow upload format ------------------------------------------------------------------------
 * The host may ship the event columns narrow (cadence_amd/wire.py): per column one byte width (1..8)
 * for the whole batch and an encoding; crr_widen_events rebuilds the exact crr_events columns of
 * `in` (device buffers, written) slot for slot in the same layout (in->wf, stride, wave tail), pads
 * zeroed, before crr_replay on the same stream.  The etype column is shipped as is.
 *   CRR_PACK_PLAIN     value, sign-extended
 *   CRR_PACK_UNSIGNED  value, zero-extended
 *   CRR_PACK_DELTA     value - the previous event's value of the same workflow (step 0: - 0, the
 *                      timestamp column: - ts_base[w]); uint64 wrap-around, so exact for any input
 *   CRR_PACK_ID_MINUS  (ref only) event_id - ref
 * Returns 0 on successful launch, -1 on an invalid argument, else the hipError_t.  Not part of the
 * reference interface: a transfer encoding between the host flattener and crr_replay. */
#define CRR_PACK_PLAIN    0u
#define CRR_PACK_UNSIGNED 1u
#define CRR_PACK_DELTA    2u
#define CRR_PACK_ID_MINUS 3u
typedef struct crr_packed_column {
    const uint8_t* data;     /* device: n_slots * width bytes, little-endian */
    uint32_t       width;    /* 1..8 */
    uint32_t       kind;     /* CRR_PACK_* */
} crr_packed_column;
typedef struct crr_packed_events {
    crr_packed_column event_id, version, timestamp, task_id, ref, key, aux;
    const int64_t*    ts_base;   /* device [n_wf]: the timestamp delta base (NULL: 0) */
} crr_packed_events;
int crr_widen_events(const crr_packed_events* packed, const crr_inputs* in, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CADENCE_REPLAY_H_ */
