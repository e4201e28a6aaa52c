/*
 * cadence_decode.h -- host-side decoder: persisted history blobs -> the replay engine's SoA input.
 *
 * Replaces, for the replay path, the Go work before ApplyEvents:
 *
 *   common/persistence/serializer.go:109-119, :312-335   DeserializeBatchEvents (thriftrw blob -> []*HistoryEvent)
 *   common/codec/version0Thriftrw.go:44-61               0x59 preamble + thrift binary (go.uber.org/thriftrw v1.29.2)
 *   .gen/go/shared/shared.go:41935-42460                 HistoryEvent / *EventAttributes wire layout
 *   the cgo shim's flattening loop   events -> columns, side records, interned keys
 *
 * Each workflow is a sequence of persisted batches (one blob per ApplyEvents call, in order, as
 * state_rebuilder.go:135-148 pages them).  A blob is a thriftrw-encoded `shared.History{10: list<
 * HistoryEvent>}` behind the 0x59 preamble; an empty blob or an empty event list is an empty batch.
 * The output is a canonical (stride-1) crr_inputs image, byte-identical to what the Python host
 * flattening (cadence_amd/flatten.py) produces from the same events.
 *
 * Plain C ABI: the decoder owns its output buffers until crr_decoded_free.
 */
#ifndef CADENCE_DECODE_H_
#define CADENCE_DECODE_H_

#include <stddef.h>
#include <stdint.h>

#include "cadence_replay.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Host inputs of one workflow (the values the Go code takes from the shard, the domain cache,
 * uuid.New() and timeSource.Now()). */
typedef struct crr_wf_source {
    uint32_t       blob_begin;            /* this workflow's batches: blobs[blob_begin .. blob_begin + blob_count) */
    uint32_t       blob_count;
    int64_t        init_version;          /* domainEntry.GetFailoverVersion() (mutable_state_builder.go:207) */
    int64_t        now_ns;                /* injected timeSource.Now() */
    const char*    run_id;                /* NUL-terminated; tree ID of the branch token */
    const char*    branch_id;             /* injected uuid of NewHistoryBranchToken (state_builder.go:179-183) */
    const uint8_t* final_token;           /* rebuild target token (state_rebuilder.go:150), NULL: none */
    uint32_t       final_token_len;
    int32_t        new_run_wf;            /* workflow index of the CAN new-run history, -1: none */
    int64_t        rebuild_last_event_id;
    int64_t        rebuild_last_event_version;
    int32_t        flags;                 /* CRR_WF_FLAG_* */
    int32_t        retention_days;        /* domain retention (DeleteHistoryEventTask) */
} crr_wf_source;

/* Read-only view of a decoded batch (host pointers, valid until crr_decoded_free). */
typedef struct crr_decoded_view {
    crr_events                ev;          /* columns, n_events entries each */
    uint64_t                  n_events;
    const crr_activity_side*  act_side;    uint64_t n_act_side;
    const crr_start_side*     start_side;  uint64_t n_start_side;
    const uint32_t*           reset_keys;  uint64_t n_reset_keys;
    const uint8_t*            arena;       uint64_t n_arena;
    const crr_workflow*       wf;          uint32_t n_wf;
    uint64_t                  table_rows[8];  /* act, timer, child, rc, sig, vh, rp, tasks slot-table sizes */
    /* per-event key strings (ActivityID / TimerID / BinaryChecksum; "" otherwise), for checkers */
    const uint32_t*           key_off;
    const uint32_t*           key_len;
    const char*               key_arena;   uint64_t n_key_arena;
} crr_decoded_view;

typedef struct crr_decoded crr_decoded;

#define CRR_DECODE_OK              0
#define CRR_DECODE_BAD_ARGUMENT   -1
#define CRR_DECODE_BAD_PREAMBLE   -2   /* not a version-0 thriftrw blob (version0Thriftrw.go:53-58) */
#define CRR_DECODE_TRUNCATED      -3   /* thrift value runs past the end of the blob */
#define CRR_DECODE_BAD_TYPE       -4   /* field / element of an unexpected or unknown thrift type */
#define CRR_DECODE_BAD_JSON       -5   /* a json-encoded blob json.Unmarshal rejects (syntax or type error) */
#define CRR_DECODE_UNKNOWN_ENCODING -6 /* NewUnknownEncodingTypeError (serializer.go:326-327) */

/* DataBlob.Encoding of each blob (common.EncodingType): serializerImpl.deserialize
 * (common/persistence/serializer.go:321-328) decodes thriftrw with the thriftrw codec and json, the
 * unknown and the empty encodings with json.Unmarshal (backward compatibility); anything else fails. */
#define CRR_ENCODING_THRIFTRW 0u
#define CRR_ENCODING_JSON     1u
#define CRR_ENCODING_UNKNOWN  2u
#define CRR_ENCODING_EMPTY    3u

/* Decode every workflow's blobs.  known_domains: names the domain cache resolves (NULL with
 * n_known == UINT32_MAX: every name resolves).  n_threads <= 0: hardware concurrency.
 * Returns NULL on error with *err = CRR_DECODE_* and *err_blob = index of the offending blob
 * (the Go serializer's CadenceDeserializationError). */
crr_decoded* crr_decode_histories(const uint8_t* const* blobs, const uint64_t* blob_lens, uint32_t n_blobs,
                                  const crr_wf_source* wfs, uint32_t n_wf,
                                  const char* const* known_domains, uint32_t n_known,
                                  int n_threads, int* err, int64_t* err_blob);
/* Same, with each blob's encoding (CRR_ENCODING_*; NULL: every blob thriftrw). */
crr_decoded* crr_decode_histories_enc(const uint8_t* const* blobs, const uint64_t* blob_lens,
                                      const uint32_t* blob_encodings, uint32_t n_blobs,
                                      const crr_wf_source* wfs, uint32_t n_wf,
                                      const char* const* known_domains, uint32_t n_known,
                                      int n_threads, int* err, int64_t* err_blob);
int  crr_decoded_get_view(const crr_decoded* d, crr_decoded_view* view);
void crr_decoded_free(crr_decoded* d);

/* ---- synthetic histories (benchmark / test infrastructure, not part of the replay boundary) ---------
 * Seeded random-walk histories flattened like decoded ones (cadence_amd/csrc/synth_native.cpp):
 * CRR_SYNTH_MIXED: n workflows of 10..2*mean_len-10 events over every event type (configs 3 and 5);
 * CRR_SYNTH_LONG_TAIL: n logical workflows with Zipf(alpha) lengths in [min_len, max_len], continued
 * as new every run_cap events (each run a workflow, each CAN event's new-run history its next run's
 * first batch; config 4).  The result is freed with crr_decoded_free. */
#define CRR_SYNTH_MIXED     0
#define CRR_SYNTH_LONG_TAIL 1
typedef struct crr_synth_params {
    uint32_t kind;                 /* CRR_SYNTH_* */
    uint32_t n;
    uint64_t seed;
    int32_t  mean_len;             /* mixed */
    int32_t  multi_version;        /* failover version bumps at batch boundaries (VersionHistories items) */
    double   invalid_rate;         /* histories that end in an injected ApplyEvents error */
    double   can_rate;             /* mixed: CAN-closed histories given a new-run history */
    double   unknown_domain_rate;  /* attribute domain names the domain cache cannot resolve */
    int32_t  min_len, max_len, run_cap;   /* long tail */
    int32_t  caps[5];              /* concurrently pending activity / timer / child / rc / signal caps (<= 0: none) */
    double   alpha;                /* long tail: Zipf exponent */
    /* shard partition of one global workload: with num_shards > 0 and world > 1 only the (logical)
     * workflows w with crr_synth_shard_of(w, num_shards) % world == rank are generated, each exactly as
     * in the whole workload (per-workflow seeded); continue-as-new runs stay with their workflow */
    uint32_t num_shards, world, rank, reserved;
} crr_synth_params;

/* History shard of synthetic workflow w (stand-in for common/util.go:313-316 WorkflowIDToHistoryShard:
 * farm.Fingerprint32(workflowID) % numberOfShards; here a SplitMix64 finalizer of the workflow index). */
uint32_t crr_synth_shard_of(uint64_t w, uint32_t num_shards);

crr_decoded* crr_synth_histories(const crr_synth_params* params, int n_threads, int* err);

#ifdef __cplusplus
}
#endif
#endif /* CADENCE_DECODE_H_ */
