/*
 * mtoracle.h — C API of the CPU ORACLE (test infrastructure only).
 *
 * The oracle is a restatement of the reference merge-tree algorithm
 * (/root/reference/packages/dds/merge-tree/src) used ONLY by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
 * The product (fluidframework_amd/, libmtgpu.so) never links or calls it.
 */
#ifndef MTORACLE_H
#define MTORACLE_H
#include <stdint.h>
#include "../include/mtgpu.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct ora_doc ora_doc;

/* collaborating=1: passive observer "obs" (startOrUpdateCollaboration, MT/client.ts:1073);
 * collaborating=0: detached local document (SharedString before attach). */
ora_doc* ora_new(int collaborating);
void     ora_free(ora_doc* d);
int      ora_set_props(ora_doc* d, const mt_prop_table* props);
int      ora_set_client_names(ora_doc* d, uint32_t n, const char* const* client_json);
/* Apply run `run` of the batch (Client.applyMsg per message). Returns 0 or an
 * MT_DS_* status bitmask (the reference would have thrown). */
uint32_t ora_apply_run(ora_doc* d, const mt_op_batch* b, uint32_t run);
/* Client.applyMsg (MT/client.ts:790-850) on one ISequencedDocumentMessage given as
 * JSON text: parsed and dispatched here (GROUP, non-"op" types, markers, props),
 * independent of the hosts' batch packers.  Returns the MT_DS_* status. */
char* ora_register_info_json(ora_doc* o, const char* client_literal, const char* name_literal);
uint32_t ora_apply_msg_json(ora_doc* d, const char* json);
/* getLength(refSeq, client) for the client with long id `client_literal` (a JSON
 * string literal, e.g. "\"alice\""). */
int32_t  ora_get_length_json(ora_doc* d, int32_t ref_seq, const char* client_literal);
/* posFromRelativePos of an IRelativePosition (JSON) under that client's perspective;
 * -1 when no marker carries the id. */
int32_t  ora_rel_pos_json(ora_doc* d, int32_t ref_seq, const char* client_literal, const char* relpos_json);
/* SharedSegmentSequence.processMergeTreeMsg for the legacy format (sequence.ts:604-642):
 * applies the message and stashes it, transformed from its sequenceDelta events by
 * createOpsFromDelta (sequence.ts:58-105) when refSeq != seq - 1.  Returns the status. */
uint32_t ora_channel_process(ora_doc* d, const char* json);
/* snapshotMergeTree's catch-up messages (sequence.ts:592-602): the stash trimmed to and
 * stamped with min_seq, as JSON text (free with ora_free_buf), or NULL when empty. */
char*    ora_channel_stash_json(ora_doc* d, int32_t min_seq);
/* Delta / maintenance callbacks as records (on != 0), and the records so far as a JSON
 * array [op, kind, pos, len, b, propsBefore|null, propsAfter|null] (free with ora_free_buf). */
void     ora_delta_capture(ora_doc* d, int on);
char*    ora_delta_json(ora_doc* d);
/* Local (non-collaborating) ops, as SharedString.insertText/insertMarker/
 * annotateRange/removeText on a detached string (seq = UniversalSequenceNumber). */
int      ora_local_insert(ora_doc* d, int32_t pos, const uint16_t* text, uint32_t n,
                          int32_t marker_ref_type, int32_t prop_set);
int      ora_local_remove(ora_doc* d, int32_t start, int32_t end);
int      ora_local_annotate(ora_doc* d, int32_t start, int32_t end, int32_t prop_set, int32_t rewrite);
/* SnapshotLoader (MT/snapshotLoader.ts:39-222) on a document made with
 * ora_new(0): blobs[0] = the "header" blob, then the body chunks in
 * orderedChunkMetadata order (V1 or legacy chunks, snapshotChunks.ts:137-180);
 * the observer is "obs".  Returns the MT_DS_* status (INSERT_FAILED where the
 * reference throws, UNSUPPORTED for aliased loadBody segments / bad specs). */
int      ora_load_snapshot(ora_doc* d, uint32_t n_blobs, const char* const* blobs);
int32_t  ora_get_length(ora_doc* d, int32_t ref_seq, int32_t client); /* client -1: observer */
/* getContainingSegment under stream client `client`'s perspective at ref_seq (ref_seq < 0:
 * the local client at currentSeq, Client.getContainingSegment; client_literal non-null: the
 * client with that long id, a JSON string literal), with resolveRemoteClientPosition in
 * out16[14]; out16 in mt_seg_info order (prop_set 1 = properties defined, row -1); *json
 * (optional, ora_free_buf) = the segment's toJSONObject.  Returns found. */
int      ora_containing_segment(ora_doc* d, int32_t pos, int32_t ref_seq, int32_t client, const char* client_literal,
                                int32_t* out16, char** json);
/* Diagnostic: getLength as the sum of nodeLength over every segment (no partial lengths). */
int32_t  ora_get_length_exact(ora_doc* d, int32_t ref_seq, int32_t client);
/* The long id (JSON literal) of a short client id of the document, NULL if none. */
const char* ora_client_name(ora_doc* d, int32_t short_id);
/* Snapshot: returns a malloc'd buffer: u32 n_blobs, then per blob u64 len + bytes. */
uint8_t* ora_snapshot_v1(ora_doc* d, int32_t msn, int32_t seq, uint64_t* digest, uint64_t* total_bytes);
/* options.mergeTreeSnapshotChunkSize of the document's MergeTree (snapshotV1.ts:55; default 10000). */
void     ora_set_snapshot_chunk(ora_doc* d, double chunk_size);
/* SnapshotLegacy (MT/snapshotlegacy.ts:104-240) blobs "header"[, "body"], same packing. */
uint8_t* ora_snapshot_legacy(ora_doc* d, int32_t msn, int32_t seq, uint64_t* digest, uint64_t* total_bytes);
uint16_t* ora_get_text(ora_doc* d, uint64_t* n_units);
int32_t* ora_dump_segments(ora_doc* d, uint32_t* n_rows);  /* 12 int32 per row */
void     ora_free_buf(void* p);
/* Tree statistics: height, overlap-list pushes by short client ids >= 63, segments, blocks. */
void     ora_stats(ora_doc* d, int32_t* out4);

/* Stream generation (SURVEY.md §8(d) rules, same algorithm as mt_generate):
 * generates and applies ops_per_doc messages for document `doc`; writes the op
 * arrays (length ops_per_doc) and the payload (<= ops_per_doc*ins_len_max). */
uint32_t ora_generate_doc(const mt_gen_params* p, uint32_t doc, const mt_prop_table* props,
                          uint8_t* type, uint8_t* flags, uint16_t* client, int32_t* seq,
                          int32_t* ref_seq, int32_t* msn, int32_t* pos1, int32_t* pos2,
                          uint32_t* payload_off, uint32_t* payload_len, int32_t* prop_id,
                          uint16_t* payload, uint32_t payload_base, ora_doc** keep_doc);
/* Test support (digest manifests): the SnapshotV1 digests of documents first..first+n-1
 * generated and replayed by the oracle (ora_generate_doc's rules, global document ids), on
 * `threads` threads; pre (optional) is generated first and p continues it; ops / clients
 * (optional) are per-document counts. */
int      ora_generate_digests(const mt_gen_params* p, const mt_gen_params* pre, const mt_prop_table* props,
                              uint32_t first, uint32_t n, const uint32_t* ops, const uint32_t* clients, int threads,
                              uint64_t* digests, uint32_t* status);

/* Debug: verify partial lengths == exact leaf sums at every generated op. */
void ora_set_verify(int on);
long long ora_verify_result(long long* checks);

/* CPU baseline: replay every run of the batch on fresh documents with
 * `threads` std::threads (LPT-partitioned by op count); returns wall seconds of
 * the apply loop and optionally per-run snapshot digests (msn/seq = last op's). */
double   ora_replay_batch(const mt_op_batch* b, const mt_prop_table* props, int threads,
                          uint64_t* out_digests, uint32_t* out_status, uint64_t* out_counters);
/* The §8(d) algorithmic counters of a document in mt_doc_counters order (ops, msgs,
 * ins_units, rows_rw, depth, scoured), counted by their definitions on the oracle's own
 * object model; ora_replay_batch's out_counters (optional) holds 6 per run. */
void     ora_counters(ora_doc* d, uint64_t* out6);

#ifdef __cplusplus
}
#endif
#endif
