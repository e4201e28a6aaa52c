/*
 * cadence_ingest.h -- device-side ingest: persisted thriftrw history blobs in HBM -> the replay engine's
 * wave-interleaved, tiered crr_inputs, on the GPU.
 *
 * Replaces, for a batch of workflows whose persisted batches are already in device memory (uploaded
 * as they were read from persistence), the host work before crr_replay:
 *
 *   common/persistence/serializer.go:109-119, :312-335   DeserializeBatchEvents (thriftrw blob -> events)
 *   common/codec/version0Thriftrw.go:44-61               0x59 preamble + thrift binary (go.uber.org/thriftrw v1.29.2)
 *   .gen/go/shared/shared.go:41935-42460                 HistoryEvent / *EventAttributes wire layout
 *   the cgo shim's flattening and layout: events -> SoA columns, interned
 *   ActivityID / TimerID / BinaryChecksum keys, domain-cache outcomes, slot-table capacities, the
 *   length / expected-live-set ordering and the 64-workflow wave interleave
 *
 * The result is byte-identical to the host path (crr_decode_histories, cadence_amd/flatten.interleave
 * with its default long-history threshold and tiering) on the same blobs: the same columns, side
 * records, descriptors, tier boundaries and slot-table sizes.  Only thriftrw (and empty) blobs are
 * decoded here; a batch holding json / unknown / empty-encoded blobs is first rewritten as thriftrw on
 * the device (crr_ingest_transcode_plan / crr_ingest_transcode, below).  New batches applied onto loaded states (CRR_WF_FLAG_RESUME, passive replication)
 * take crr_ingest_plan_resume / crr_ingest_layout_resume at the end of this header.
 *
 * Two calls, because the caller sizes the replay's buffers between them:
 *   crr_ingest_plan   parse every blob (twice: count, then decode into a canonical scratch layout),
 *                     intern keys, resolve domains, per-workflow capacities and live-set bounds, the
 *                     device order (radix sort) and the group geometry; writes a crr_ingest_summary
 *   crr_ingest_layout write the interleaved columns, side records, reset keys, branch tokens and
 *                     descriptors into the caller's buffers (sized from the summary)
 * Both enqueue on `stream` and return 0 on a successful launch, -1 on an invalid argument, else the
 * hipError_t.  All pointers are device pointers unless noted.
 */
#ifndef CADENCE_INGEST_H_
#define CADENCE_INGEST_H_

#include <stddef.h>
#include <stdint.h>

#include "cadence_replay.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One workflow's persisted batches and host inputs (crr_wf_source of cadence_decode.h with the strings
 * as (offset, length) into crr_blob_batch.strings).  Workflows' blob ranges are consecutive:
 * wf[0].blob_begin == 0 and wf[w + 1].blob_begin == wf[w].blob_begin + wf[w].blob_count. */
typedef struct crr_blob_wf {
    uint32_t blob_begin;
    uint32_t blob_count;
    int64_t  init_version;          /* domainEntry.GetFailoverVersion() */
    int64_t  now_ns;                /* injected timeSource.Now() */
    uint32_t run_id_off, run_id_len;        /* tree ID of the branch token */
    uint32_t branch_id_off, branch_id_len;  /* injected branch ID (state_builder.go:179-183) */
    uint32_t final_token_off;       /* rebuild target token bytes in `strings`; len UINT32_MAX: none */
    uint32_t final_token_len;
    int64_t  rebuild_last_event_id;
    int64_t  rebuild_last_event_version;
    int32_t  new_run_wf;            /* workflow index (this batch's order) of the CAN new-run history, -1 */
    int32_t  flags;                 /* CRR_WF_FLAG_NEW_RUN | CRR_WF_FLAG_REFRESH_TASKS */
    int32_t  retention_days;
    int32_t  reserved;
} crr_blob_wf;                      /* 80 B */

typedef struct crr_blob_batch {
    const uint8_t*     bytes;       /* every blob, concatenated */
    const uint64_t*    blob_off;    /* [n_blobs + 1] byte offsets into `bytes` */
    uint32_t           n_blobs;
    uint32_t           n_wf;
    const crr_blob_wf* wf;          /* [n_wf] */
    const uint8_t*     strings;     /* run / branch IDs, final tokens, known domain names */
    const uint32_t*    domain_off;  /* [n_domains] known domain names in `strings` */
    const uint32_t*    domain_len;
    uint32_t           n_domains;   /* UINT32_MAX: every name resolves */
    uint32_t           reserved;
} crr_blob_batch;

/* What the plan reports (a host struct, written by crr_ingest_plan once its work on `stream` is done:
 * the plan synchronises the stream twice, to size its own launches and to read this back). */
typedef struct crr_ingest_summary {
    int32_t  err;                   /* CRR_DECODE_* of the failing blob with the lowest index, 0: ok */
    int32_t  reserved0;
    int64_t  err_blob;              /* that blob's index, -1 */
    uint64_t n_events;              /* real events */
    uint64_t n_slots;               /* event-column slots of the layout (lane groups padded + the tail) */
    uint64_t n_act_side;            /* activity side-record slots */
    uint64_t n_start_side;          /* start side-record slots */
    uint64_t n_reset_keys;          /* previous reset points (0: allocate one entry, left 0 -- flatten's placeholder) */
    uint64_t arena_bytes;           /* branch tokens (+ final tokens) */
    uint64_t table_rows[8];         /* act, timer, child, rc, sig, vh, rp, tasks slot-table rows */
    uint32_t n_wf;
    uint32_t wave_begin;            /* lane workflows [0, wave_begin), long-history tail after */
    uint32_t tiers[6];              /* large_begin, compact_begin, compact2_begin, wide_begin, hbm_begin, big_begin */
    uint32_t has_new_run;           /* some workflow carries CRR_WF_FLAG_NEW_RUN */
    uint32_t lds_small_tail;        /* the tail [wave_begin, big_begin) fits the small per-wave arenas */
} crr_ingest_summary;

/* Device scratch the plan keeps for the layout (opaque), for a batch of at most `max_events` events
 * (a capacity the caller chooses: the plan reports CRR_INGEST_SCRATCH_TOO_SMALL in summary.err when the
 * blobs hold more, and the caller plans again with more).  Both calls take the same scratch and size. */
size_t crr_ingest_scratch_bytes(uint32_t n_blobs, uint32_t n_wf, uint64_t max_events);
#define CRR_INGEST_SCRATCH_TOO_SMALL (-100)

int crr_ingest_plan(const crr_blob_batch* in, void* scratch, size_t scratch_bytes, crr_ingest_summary* summary,
                    void* stream);

/* `dst`: device buffers sized from the summary (columns n_slots entries each; the wf descriptors
 * n_wf; act_side / start_side / reset_keys / arena their counts, arena 8-byte padded); the scalar
 * fields of *dst (n_wf, stride, flags, wave_begin, tiers) are the caller's to set from the summary; the
 * columns it writes satisfy CRR_IN_STARTED_AUX (each ActivityTaskStarted's aux joined to its scheduled event's
 * side record), so the caller may set that flag.
 * `summary_host`: the plan's summary, as read back.  Also writes perm[n_wf] (device position ->
 * workflow index of the blob batch) when perm != NULL.  For both calls `bytes` of the blob batch must be
 * 16-byte aligned and readable CRR_INGEST_PAD bytes past the end of the last blob: the parser's register
 * window loads the two 16-byte-aligned words around its cursor, so a cursor on the last byte reads up to
 * 31 bytes beyond it. */
#define CRR_INGEST_PAD 32
int crr_ingest_layout(const crr_blob_batch* in, void* scratch, size_t scratch_bytes,
                      const crr_ingest_summary* summary_host, const crr_inputs* dst, uint32_t* perm, void* stream);

/* ---- resume: a replication task's new batches onto loaded states already in HBM ------------------------
 *
 * Passive replication (service/history/ndc/replication_task.go:386-390 -> serializer.go:109-119 deserializes
 * the task's event blob; ndc/history_replicator.go:385-460 applies it, :396, onto the state
 * mutableStateBuilder.Load read back, mutable_state_builder.go:306-349).  The loaded states are the rows a
 * previous crr_replay left in its crr_outputs (slots 0..n-1 of each workflow's regions); this pair decodes
 * the new batches' blobs on the device and lays them out as the crr_inputs of a CRR_WF_FLAG_RESUME replay
 * that writes into those same outputs.
 *
 * Differences from crr_ingest_plan / _layout:
 *   order     blob-batch workflow p IS device position p of the loaded layout (no sort: the outputs are
 *             addressed by position); lanes [0, wave_begin) interleaved 64-wide, the tail contiguous
 *   keys      WfFlattener::key_of continued from the loaded state's dictionary: workflow p's loaded key k
 *             (1..key_count[p]) is the string at key_off[key_begin[p] + k - 1] (byte offset into the blob
 *             batch's `bytes`, which the caller uploads after the last blob) / key_len; a new string gets the
 *             next id in first-seen order -- the ids the one-shot layout of the whole history assigns
 *   descriptors  loaded_wf[p] (the loaded layout's descriptor: table bases / capacities, branch tokens,
 *             rebuild fields, flags) with ev_begin / ev_count / empty_batch_at of the new events and
 *             CRR_WF_FLAG_RESUME; a workflow without blobs applies nothing (ev_count 0, empty_batch_at -1)
 *   not written  the arena (the caller keeps the loaded inputs' arena: the descriptors' token offsets point
 *             into it); the summary's tiers, table_rows and arena_bytes are 0 -- the tiering is the caller's
 *             (the loaded layout's), the output tables the loaded ones
 * The new events' side records, reset keys and (CRR_IN_STARTED_AUX) started joins are written as by
 * crr_ingest_layout.  key_begin must be the exclusive prefix sum of key_count; the scratch must hold the
 * seeded keys' hash-table entries too (summary.err CRR_INGEST_SCRATCH_TOO_SMALL: plan again with more). */
typedef struct crr_ingest_resume {
    const crr_workflow* loaded_wf;  /* [n_wf] device order; may be the layout's own dst->wf (then only
                                       ev_begin / ev_count / empty_batch_at / flags are written, in place) */
    uint32_t        wave_begin;     /* the loaded layout's lane / tail split (<= n_wf) */
    uint32_t        reserved;
    const uint32_t* key_begin;      /* [n_wf] */
    const uint32_t* key_count;      /* [n_wf] */
    const uint64_t* key_off;        /* [sum key_count] into the blob batch's bytes */
    const uint32_t* key_len;        /* [sum key_count] (0: an id no string names; never matches) */
} crr_ingest_resume;

int crr_ingest_plan_resume(const crr_blob_batch* in, const crr_ingest_resume* resume, void* scratch,
                           size_t scratch_bytes, crr_ingest_summary* summary, void* stream);
int crr_ingest_layout_resume(const crr_blob_batch* in, const crr_ingest_resume* resume, void* scratch,
                             size_t scratch_bytes, const crr_ingest_summary* summary_host, const crr_inputs* dst,
                             void* stream);

/* ---- JSON-encoded batches: transcoded to thriftrw on the device ------------------------------------------
 *
 * serializerImpl.deserialize (common/persistence/serializer.go:312-334) decodes a blob whose encoding is json,
 * unknown or empty with json.Unmarshal into []*types.HistoryEvent (the host restatement:
 * cadence_amd/csrc/json_decode.h, crr_decode_histories_enc).  This pair rewrites such blobs in HBM as the
 * canonical thriftrw History the decoders read back into the same events (json_ingest_kernel.hip), so the
 * batch then goes through crr_ingest_plan / crr_ingest_layout (or the _resume pair) unchanged:
 *   crr_ingest_transcode_plan   walk every JSON blob (`encodings[i]`: CRR_ENCODING_* of blob i; NULL: all
 *                               thriftrw), stage its thriftrw form in the scratch and size it, report the
 *                               rejected blob with the lowest index (CRR_DECODE_BAD_JSON /
 *                               CRR_DECODE_UNKNOWN_ENCODING) -- synchronises the stream once to read the sizes
 *   crr_ingest_transcode        write the new blob bytes (`out_bytes`: summary.n_bytes + CRR_INGEST_PAD bytes,
 *                               16-byte aligned) and offsets (`out_blob_off`: n_blobs + 1): the staged forms
 *                               gathered; thriftrw blobs are copied as they are, a rejected blob becomes empty
 * The caller then plans the batch { out_bytes, out_blob_off, the same wf / strings / domains }; when the
 * transcode reported a rejection, the plan's own error wins if its blob index is lower (the host decoder
 * stops at the first failing blob).  Both calls take the same scratch (crr_ingest_transcode_scratch_bytes). */
typedef struct crr_transcode_summary {
    int32_t  err;                   /* CRR_DECODE_* of the rejected blob with the lowest index, 0: none */
    int32_t  reserved;
    int64_t  err_blob;              /* its index, -1 */
    uint64_t n_bytes;               /* bytes of the transcoded batch (without the pad) */
    uint32_t n_deep;                /* JSON blobs nested past 64 levels (walked with a stack in HBM) */
    uint32_t reserved1;
} crr_transcode_summary;

/* Scratch for a batch of n_blobs blobs holding n_bytes bytes: the fixed part plus a staging area (each blob's
 * length + 64 bytes) where the plan's walk leaves the thriftrw form for the transcode to gather; a smaller
 * scratch (at least the fixed part) works too -- blobs without room are walked a second time by the transcode. */
size_t crr_ingest_transcode_scratch_bytes(uint32_t n_blobs, uint64_t n_bytes);
int crr_ingest_transcode_plan(const crr_blob_batch* in, const uint32_t* encodings, void* scratch, size_t scratch_bytes,
                              crr_transcode_summary* summary, void* stream);
int crr_ingest_transcode(const crr_blob_batch* in, const uint32_t* encodings, void* scratch, size_t scratch_bytes,
                         const crr_transcode_summary* summary, uint8_t* out_bytes, uint64_t* out_blob_off,
                         void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CADENCE_INGEST_H_ */
