/*
 * mtgpu.h — C ABI of the MI355X batched merge-tree replay engine.
 *
 * This is the drop-in boundary for the data-parallel hot path of Fluid's
 * sequence DDS: server-side replay of sequenced SharedString op streams by a
 * passive observer client.  Every entry point replaces a
 * method of the reference merge-tree `Client`
 * (/root/reference/packages/dds/merge-tree/src/client.ts, cited as MT/client.ts)
 * applied to many independent documents at once:
 *
 *   mt_create / mt_destroy      one engine context per GPU (no reference analogue:
 *                               the reference holds one JS `Client` per document)
 *   mt_docs_open                `new Client(...)` + `startOrUpdateCollaboration(obs)`
 *                               MT/client.ts:78-87, :1073-1093 for n documents
 *   mt_apply_batch              `Client.applyMsg(msg)` for every message of every
 *                               document, in sequence order per document
 *                               MT/client.ts:819-841 (→ applyRemoteOp :790-817,
 *                               updateSeqNumbers :843-850)
 *   mt_update_seq               `Client.updateSeqNumbers(min, seq)` MT/client.ts:843
 *   mt_get_length               `MergeTree.getLength(refSeq, clientId)`
 *                               packages/dds/merge-tree/src/mergeTree.ts:1569
 *   mt_snapshot_v1              `Client.snapshot(...)` with newMergeTreeSnapshotFormat
 *                               (MT/client.ts:923-956 → SnapshotV1.extractSync/emit,
 *                               MT/snapshotV1.ts:98-256): per-document header and
 *                               body_i blob strings + a 64-bit digest
 *   mt_snapshot_legacy          `Client.snapshot(...)` without it (the default;
 *                               MT/client.ts:950-954 → SnapshotLegacy,
 *                               MT/snapshotlegacy.ts:104-240): header + body blobs
 *   mt_get_text                 `createTextHelper().getText(currentSeq, obs)`
 *                               MT/textSegment.ts:163-181
 *   mt_dump_segments            walkAllSegments (mergeTree.ts:2998) row dump, parity
 *   mt_load_snapshot            `SnapshotLoader.initialize` + `loadBody`
 *                               (MT/snapshotLoader.ts:39-222): reloadFromSegments
 *                               (mergeTree.ts:1185-1238) of the header chunk,
 *                               startOrUpdateCollaboration, then the body chunks
 *                               appended through insertSegments (mergeTree.ts:1974)
 *
 * Conventions: every function returns an int status (MT_OK == 0); no exception
 * crosses the ABI.  Per-document errors (the reference's `assert` throws,
 * common-utils assert.ts:12-16) are reported in a per-document status word.
 * Plain pointers and sizes only; host pointers unless a name says `_dev`.
 */
#ifndef MTGPU_H
#define MTGPU_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------- */
#define MT_OK               0
#define MT_E_INVALID        1  /* bad argument / shape                          */
#define MT_E_HIP            2  /* a HIP runtime call failed                     */
#define MT_E_OOM            3  /* a per-document pool (rows/blocks/text) is full */
#define MT_E_DOC_STATUS     4  /* a snapshot was asked of a document whose status
                                  word is set (the reference would have thrown)  */
#define MT_E_EXCHANGE       5  /* exchanged document rows fail their checksum     */
/* per-document status bits (mt_doc_status) */
#define MT_DS_ASSERT_SEQ     0x01u /* currentSeq >= seq   (MT/client.ts:482, :846) */
#define MT_DS_ASSERT_MSN     0x02u /* msn went backwards  (MT/client.ts:484, mergeTree.ts:1716) */
#define MT_DS_INSERT_FAILED  0x04u /* insert fell off the tree (mergeTree.ts:2228-2233) */
#define MT_DS_UNSUPPORTED    0x08u /* an input off the batch path: a combining op whose result
                                      is a string or would alias (MT_VAL_UNSUP), a reused
                                      marker id, a second paste of a register, ... */
#define MT_DS_OOM_ROWS       0x10u
#define MT_DS_OOM_BLOCKS     0x20u
#define MT_DS_OOM_TEXT       0x40u
#define MT_DS_OOM_PROPS      0x80u
#define MT_DS_OOM_HEAP       0x100u
#define MT_DS_OOM_WINDOW     0x200u
#define MT_DS_PROPS_TOO_MANY 0x400u
#define MT_DS_BAD_OP         0x800u /* an op record out of its batch's bounds (payload /
                                       property table), checked on the device         */
#define MT_DS_OOM_OVERLAP    0x2000u /* removedClientOverlap side list (clients >= 63) full */
#define MT_DS_THROWS         0x4000u /* an op on which the reference's Client throws: a
                                       consensus combine on a segment without the key whose
                                       defaultValue is null reads null.seq (properties.ts:
                                       41-52, TypeError); the document stops there        */
#define MT_DS_REFSEQ_BELOW_MSN 0x1000u /* refSeq < minSeq: deli nacks such ops
                                       (deli/lambda.ts:302-318); the window aggregate
                                       is exact only for refSeq >= minSeq             */

/* ---- op records (IMergeTreeOp flattened; MT/ops.ts:6-110) --------------- */
#define MT_OP_INSERT   0   /* MergeTreeDeltaType.INSERT   */
#define MT_OP_REMOVE   1   /* MergeTreeDeltaType.REMOVE   */
#define MT_OP_ANNOTATE 2   /* MergeTreeDeltaType.ANNOTATE */
#define MT_OP_NOOP     3   /* a sequenced message whose type !== "op" (or an empty
                              GROUP): only seq/msn advance (MT/client.ts:840)  */
#define MT_OP_UNSUPPORTED 4 /* an op the host found off the batch path (e.g. a
                              second marker with an id already in use): the
                              document gets MT_DS_UNSUPPORTED                    */
/* Register copy/paste (RegisterCollection, MT/mergeTree.ts:864-896; Client.copy
 * MT/client.ts:600-608).  payload_off = the register name's per-document index (the
 * host interns names); the register is keyed by (author client, name). */
#define MT_OP_CUT   5  /* remove with op.register: the range's segments are cloned into
                          the register, then removed (client.ts:347-350)              */
#define MT_OP_COPY  6  /* insert with op.register and a truthy range end: clone
                          [pos1, pos2) into the register, no insert (client.ts:425-428) */
#define MT_OP_PASTE 7  /* insert with op.register and no range end: the register's
                          segments are inserted at pos1 (client.ts:436-439, blockInsert
                          mergeTree.ts:2207-2241); an empty or unknown register is a no-op.
                          Pasting a register a second time (the reference re-links the
                          same segment objects) or one holding clones of removed
                          segments sets MT_DS_UNSUPPORTED.                              */

#define MT_OPF_END_OF_MSG 0x01u /* last member of one sequenced message: the
                                   engine runs updateSeqNumbers(msn, seq) after it.
                                   GROUP members (MT/client.ts:804-812) share seq/
                                   ref_seq/msn and only the last carries this flag */
#define MT_OPF_MARKER     0x02u /* insert of a Marker; pos2 holds refType          */
#define MT_OPF_REWRITE    0x04u /* annotate with combiningOp {name:"rewrite"}      */
#define MT_OPF_SEG_PROPS  0x08u /* insert seg has props (prop_id)                  */
#define MT_OPF_COMBINE    0x10u /* annotate with another combiningOp (Properties.combine,
                                   MT/properties.ts:24-62, through
                                   MT/segmentPropertiesManager.ts:98-103):
                                   COMBINE alone = {name:"incr"}; COMBINE|REWRITE|
                                   CONSENSUS = {name:"consensus"}; COMBINE|REWRITE =
                                   any other name (a key that holds a value keeps
                                   it).  prop_id then names a combine set (below),
                                   not the op's props.                             */
#define MT_OPF_CONSENSUS  0x02u /* on a combining annotate: the name is "consensus" */
#define MT_OPF_INCR_STRMIN 0x08u /* on an incr annotate: a truthy string / array /
                                   object minValue, which a string result compares
                                   against (properties.ts:35-38): such a result from
                                   a held value sets MT_DS_UNSUPPORTED            */
#define MT_OPF_REL1       0x20u /* pos1 is an index into rel[]: op.relativePos1
                                   (posFromRelativePos, mergeTree.ts:1949-1972)    */
#define MT_OPF_REL2       0x40u /* pos2 is an index into rel[]: op.relativePos2    */
#define MT_OPF_MARKER_ID  0x80u /* marker insert whose props carry a markerId:
                                   payload_off = the document's marker-id index   */

/*
 * One batch = per-document runs of ops, concatenated by document.
 * Run d covers ops [op_offsets[d], op_offsets[d+1]) and targets engine
 * document slot doc_ids[d].  Text payloads are UTF-16 code units
 * (JS string semantics: lengths are .length of the JS string).
 */
/* IRelativePosition (MT/ops.ts:46-61) with the marker id interned per document
 * (marker = index, -1 for an id the document never mapped). */
typedef struct mt_rel_pos {
    int32_t marker;
    int32_t before;               /* relativePos.before (truthy)                  */
    int32_t offset;               /* relativePos.offset, 0 when undefined         */
    int32_t pad;
} mt_rel_pos;

typedef struct mt_op_batch {
    uint32_t        n_runs;
    const uint32_t* doc_ids;      /* [n_runs]                                  */
    const uint32_t* op_offsets;   /* [n_runs+1]                                */
    uint32_t        n_ops;
    const uint8_t*  type;         /* [n_ops] MT_OP_*                           */
    const uint8_t*  flags;        /* [n_ops] MT_OPF_*                          */
    const uint16_t* client;       /* [n_ops] per-document client index (< 65534) */
    const int32_t*  seq;          /* [n_ops] sequenceNumber                     */
    const int32_t*  ref_seq;      /* [n_ops] referenceSequenceNumber            */
    const int32_t*  msn;          /* [n_ops] minimumSequenceNumber              */
    const int32_t*  pos1;         /* [n_ops]                                    */
    const int32_t*  pos2;         /* [n_ops] (insert marker: refType)           */
    const uint32_t* payload_off;  /* [n_ops] into payload                       */
    const uint32_t* payload_len;  /* [n_ops] UTF-16 units                       */
    const int32_t*  prop_id;      /* [n_ops] index into the prop table, -1 none */
    const uint16_t* payload;      /* UTF-16 arena                               */
    uint64_t        payload_units;
    uint32_t        n_rel;        /* relative positions referenced by REL1/REL2 */
    const mt_rel_pos* rel;        /* [n_rel]                                    */
} mt_op_batch;

/* The packed 32-byte op record the device replays (one per op member), for
 * hosts that move op streams between devices without a host round trip
 * (mt_generated_copy_dev / mt_upload_batch_dev). */
typedef struct mt_op_rec {
    uint8_t  type, flags;
    uint16_t client;
    int32_t  seq, ref_seq, msn, pos1, pos2;
    uint32_t payload_off;
    uint16_t payload_len;
    int16_t  prop_id;
} mt_op_rec;

/*
 * Host-interned property sets (the `props` of an annotate op or of an inserted
 * segment spec), already in JS Object.keys() order.  Values are interned JS
 * values: value -1 means `null` (delete the key, segmentPropertiesManager.ts:104).
 *
 * Remote combining ops.  SegmentPropertiesManager.addProperties calls
 * combine(op, previousValue, undefined, seq) for every key of the op's props
 * (segmentPropertiesManager.ts:98-103: its `newValue` is never assigned), so the op's
 * values are unused and the result depends on the key's previous value, the op's
 * name and defaultValue, and the message's seq.  The host packs such an annotate as a
 * *combine set*: the op's keys, each valued with what combine yields for a key the
 * segment does not hold (previousValue undefined):
 *   incr       defaultValue undefined / number / boolean / null -> MT_VAL_NAN (x + undefined);
 *              a string / object / array default -> the interned string String(default) +
 *              "undefined" (JS `+=`), or the minValue where a truthy string / array /
 *              object minValue compares above it (properties.ts:33-40)
 *   consensus  no defaultValue -> MT_VAL_CFRESH ({value: undefined, seq}); null ->
 *              MT_VAL_THROW (the reference throws reading null.seq); an object whose seq is
 *              -1 -> that object with seq = the message's seq (properties.ts:52-54); else the
 *              default
 *   other      no defaultValue -> MT_VAL_UNDEF; null -> MT_VAL_NULL (the key is deleted);
 *              else the default (combine's switch has no case: the default is returned)
 * A key the segment holds: incr yields NaN from a number, boolean, NaN or undefined value
 * (MT_VK_NUM), and String(value) + "undefined" from a string, array or object (the table's
 * value_incr; a fresh consensus object: incr_object), MT_VAL_UNSUP where the host left that
 * string out of the table or the op has MT_OPF_INCR_STRMIN; consensus keeps the value,
 * except that an object whose seq is -1 (MT_VK_SEQM1) is MT_VAL_UNSUP (consensus would write
 * the seq into an object every segment split from it shares); other names keep the value.
 * MT_VAL_UNSUP sets MT_DS_UNSUPPORTED on the document, MT_VAL_THROW MT_DS_THROWS.
 *
 * Stored values other than interned ids (never in an op's set): MT_VAL_NAN (JSON null,
 * never matchProperties-equal: NaN !== NaN), MT_VAL_UNDEF (the key is present with
 * value undefined: skipped by JSON.stringify, never equal) and MT_VAL_CONS(seq) (a fresh
 * consensus object: JSON {"seq":seq}, never equal since its `value` is undefined,
 * properties.ts:72-73).
 */
#define MT_VAL_NULL   (-1)
#define MT_VAL_NAN    (-2)
#define MT_VAL_UNSUP  (-3)
#define MT_VAL_CFRESH (-4)
#define MT_VAL_UNDEF  (-5)
#define MT_VAL_THROW  (-6)
#define MT_VAL_CONS_BASE (-16)                    /* MT_VAL_CONS(seq) = -16 - seq, 0 <= seq <= INT32_MAX - 16 (a larger seq: MT_DS_UNSUPPORTED) */
#define MT_VAL_CONS(seq) (MT_VAL_CONS_BASE - (seq))
#define MT_VK_NUM   0x01u   /* number or boolean: incr gives NaN                            */
#define MT_VK_SEQM1 0x02u   /* a (non-array) object whose "seq" member is the number -1     */
typedef struct mt_prop_table {
    uint32_t        n_sets;
    const uint32_t* set_off;      /* [n_sets+1] into key/value                  */
    const uint16_t* key;          /* key id per pair                            */
    const int32_t*  value;        /* value id per pair, -1 = null               */
    uint32_t        n_keys;
    const char* const* key_json;  /* [n_keys] JSON string literal (with quotes) */
    const uint32_t* key_index;    /* [n_keys] array-index value or 0xFFFFFFFF   */
    uint32_t        n_values;
    const char* const* value_json;/* [n_values] JSON text of the value          */
    const uint8_t*  value_falsy;  /* [n_values] JS falsiness (rewrite rule)     */
    const uint32_t* value_class;  /* [n_values] matchProperties() equivalence   */
    const uint8_t*  value_kind;   /* [n_values] MT_VK_* (null: every combine set
                                     is MT_DS_UNSUPPORTED)                      */
    const int32_t*  value_incr;   /* [n_values] incr of a held value (`v += undefined`,
                                     properties.ts:33-34): for a string / array / object,
                                     the id of the string String(v) + "undefined",
                                     MT_VAL_UNSUP when not interned (null: all UNSUP);
                                     ignored for MT_VK_NUM values (NaN)           */
    int32_t         incr_object;  /* the id of "[object Object]undefined" (incr of a held
                                     fresh consensus object), or MT_VAL_UNSUP; read only
                                     with value_incr                               */
} mt_prop_table;

/* Engine limits per document (pool capacities, sized from the op counts). */
typedef struct mt_limits {
    uint32_t max_docs;
    uint32_t rows_per_doc;      /* segment rows (append-only within a stream)     */
    uint32_t blocks_per_doc;    /* B-tree blocks (free-listed)                    */
    uint32_t text_per_doc;      /* UTF-16 units of the text arena                 */
    uint32_t propsets_per_doc;  /* device property-set arena entries              */
    uint32_t heap_per_doc;      /* zamboni heap entries                           */
    uint32_t window_per_doc;    /* collab-window row list                         */
    uint32_t markers_per_doc;   /* marker-id table (idToSegment); 0 = 1024        */
    uint32_t register_rows_per_doc; /* clone rows all registers hold at once; 0 = 256 */
} mt_limits;

typedef struct mt_ctx mt_ctx;

/* ---- delta callbacks as packed records (MT/mergeTreeDeltaCallback.ts) --- */
/* kind: MergeTreeDeltaType for the delta callback (MT/ops.ts:17-22), MergeTreeMaintenanceType
 * for the maintenance callback (MT/mergeTreeDeltaCallback.ts:11-23). */
#define MT_DK_INSERT     0
#define MT_DK_REMOVE     1
#define MT_DK_ANNOTATE   2
#define MT_DK_APPEND   (-1)
#define MT_DK_SPLIT    (-2)
#define MT_DK_UNLINK   (-3)
/*
 * One entry of a callback's deltaSegments, in callback order (the delta callback of an op
 * fires after its ensureIntervalBoundary SPLITs and before the zamboni APPEND/UNLINKs it
 * triggers).  pos is SequenceEvent.ranges[].position: the segment's position in the
 * observer's view (client.getPosition) evaluated when the callback fires.
 *   INSERT   seg = the new segment, len = cachedLength, a = its property set (mt_doc_pset);
 *            b = -1: the op's own seg spec; b = 0: a register paste's text clone whose text
 *            is units [pad, pad + len) of mt_delta_text; b = 1: a pasted marker of refType pad
 *            (createOpsFromDelta writes r.segment.clone().toJSONObject(), sequence.ts:83-87)
 *   REMOVE   seg = a newly removed segment (overlapping removes are not reported)
 *   ANNOTATE seg = an annotated segment, a / b = its property set before / after
 *   SPLIT    seg = the left part (len = its new length), a = the right part, b = its length
 *   APPEND   seg = prevSegment (len = its new length), a = the appended segment, b = its length
 *   UNLINK   seg = the unlinked segment
 * Segments are engine row ids, stable while the segment is linked.
 */
typedef struct mt_delta_rec {
    uint32_t op;        /* index of the op member in the batch (mt_op_batch order) */
    int32_t  kind;
    int32_t  pos, len, seg, a, b, pad;
} mt_delta_rec;

/* ---- snapshot load (MT/snapshotLoader.ts) ------------------------------- */
/* One snapshot segment, i.e. one element of a chunk's `segments` array after
 * the host's JSON.parse (IJSONSegment or IJSONSegmentWithMergeInfo,
 * MT/snapshotChunks.ts:63-76), as SnapshotLoader.specToSegment reads it
 * (MT/snapshotLoader.ts:93-124). 32 bytes. */
#define MT_LS_SEQ     0x01u   /* spec.seq present (else UniversalSequenceNumber 0)  */
#define MT_LS_CLIENT  0x02u   /* spec.client present (else NonCollabClient)         */
#define MT_LS_REMOVED 0x04u   /* spec.removedSeq/removedClient present               */
#define MT_LS_MARKER  0x08u   /* {"marker":{"refType":n}} (else a text segment)      */
typedef struct mt_load_seg {
    uint8_t  flags;           /* MT_LS_*                                              */
    uint8_t  pad0;
    uint16_t client;          /* per-document client index (MT_LS_CLIENT)            */
    int32_t  seq;             /* MT_LS_SEQ                                            */
    int32_t  removed_seq;     /* MT_LS_REMOVED                                        */
    uint16_t removed_client;  /* MT_LS_REMOVED                                        */
    int16_t  prop_id;         /* mt_set_props set of spec.props, -1: none             */
    uint32_t payload_off;     /* text: UTF-16 offset into payload                      */
    uint32_t payload_len;     /* text: UTF-16 units; marker: refType                   */
    uint32_t marker_id;       /* marker with a markerId prop: its per-document index + 1 */
    uint32_t pad1;
} mt_load_seg;
/* Per document: segments [seg_offsets[i], seg_offsets[i+1]) in chunk order
 * (header chunk first, then body_0, body_1, ...), the first header_segments[i]
 * of them from the header chunk; min_seq/seq = headerMetadata.minSequenceNumber
 * (sequenceNumber when absent) / .sequenceNumber.  The text payloads of one
 * document must be contiguous and in segment order in `payload`. */
typedef struct mt_load_batch {
    uint32_t           n_docs;
    const uint32_t*    doc_ids;          /* [n_docs] engine document slots       */
    const uint32_t*    seg_offsets;      /* [n_docs+1]                            */
    const uint32_t*    header_segments;  /* [n_docs]                              */
    const int32_t*     min_seq;          /* [n_docs]                              */
    const int32_t*     seq;              /* [n_docs]                              */
    const mt_load_seg* segs;
    const uint16_t*    payload;
    uint64_t           payload_units;
} mt_load_batch;

/* Counters the engine accumulates per document (algorithmic-byte accounting,
 * B_op = 32 + 4 L_ins + 32 (R_r + R_w) + 64 D + 64 Z). */
typedef struct mt_doc_counters {
    uint64_t ops;          /* sequenced op members applied                      */
    uint64_t msgs;         /* sequenced messages                                */
    uint64_t ins_units;    /* Σ L_ins                                          */
    uint64_t rows_rw;      /* Σ (R_r + R_w)                                    */
    uint64_t depth;        /* Σ D (one descent per op)                         */
    uint64_t scoured;      /* Σ Z                                              */
} mt_doc_counters;

int  mt_create(int device, const mt_limits* limits, mt_ctx** out);
/* As mt_create, with capacities per document (per_doc[i] for document i; its
 * max_docs field is ignored), e.g. sized from each document's op count. */
int  mt_create_docs(int device, uint32_t n_docs, const mt_limits* per_doc, mt_ctx** out);
/* HBM bytes held by the context's document pools. */
int  mt_pool_bytes(mt_ctx* ctx, uint64_t* bytes);
/* Device-side checkpoint of every document's state, and restore to it (the
 * engine's resume point: replay a stream on the same starting documents). */
int  mt_checkpoint(mt_ctx* ctx);
int  mt_restore(mt_ctx* ctx);
void mt_destroy(mt_ctx* ctx);
const char* mt_last_error(mt_ctx* ctx);

/* Open (reset) documents [first, first+n) as empty collaborating documents with
 * a passive observer (startCollaboration(obs, 0, 0), mergeTree.ts:1243). */
int  mt_docs_open(mt_ctx* ctx, uint32_t first, uint32_t n);

/* Upload the property table used by subsequent batches. */
int  mt_set_props(mt_ctx* ctx, const mt_prop_table* props);

/* Apply a host-resident batch (copies to HBM, then replays). Asynchronous on the
 * context stream; call mt_sync before reading results. */
int  mt_apply_batch(mt_ctx* ctx, const mt_op_batch* batch);

/* Upload a batch once and keep it resident; mt_replay_resident replays it on the
 * documents it names without any host->device traffic (the bench's timed path). */
int  mt_upload_batch(mt_ctx* ctx, const mt_op_batch* batch);
int  mt_replay_resident(mt_ctx* ctx);
/* Several batches applied as one (runs in part order): a host that packs on several threads
 * (the Node host's worker_threads, each packing a slice of the documents into its own columns)
 * hands its parts over as they are and the library concatenates them while it packs the op
 * records into the pinned staging buffer, on its own host threads.  Part p's indices are local
 * to it and are re-based here: payload_off of text inserts by the payload units of parts < p,
 * REL1/REL2 position indices by their relative positions, and property-set ids through
 * prop_map[p] (prop_map_len[p] entries; prop_map or prop_map[p] null: ids already global).
 * The result is the same as mt_upload_batch / mt_apply_batch of the concatenated batch. */
int  mt_upload_batch_parts(mt_ctx* ctx, uint32_t n_parts, const mt_op_batch* parts,
                           const int32_t* const* prop_map, const uint32_t* prop_map_len);
int  mt_apply_batch_parts(mt_ctx* ctx, uint32_t n_parts, const mt_op_batch* parts,
                          const int32_t* const* prop_map, const uint32_t* prop_map_len);
/* Residency of the replay.  use_lds = 2 (default): blocks and zamboni heap move
 * to LDS (9.6 KB per document, 4 waves per SIMD), rows/window/text stay in HBM,
 * and a document that outgrows the LDS blocks continues from HBM in the same
 * wave at the exact op it reached; 0: every pool in HBM; 1: rows, blocks, heap
 * and window all in LDS (finished by a second HBM launch when outgrown); 3: long
 * documents (blocks beyond LDS): zamboni heap, collab window, U set, per-block
 * corrections table and parent cache in LDS (one four-wave workgroup per CU),
 * blocks/rows/text in HBM, same in-wave hand-over (rows = window entries kept in
 * LDS, the rest stay in HBM; blocks = A/B switches, bits 1 block cache, 2 zamboni
 * prefetch, 4 corrections table, 8 parent cache: off).
 * rows/blocks/heap (0 = compiled maximum) may only lower the caps; tests use
 * small caps to force the hand-over. */
int  mt_set_residency(mt_ctx* ctx, int use_lds, int rows, int blocks, int heap);
/* Size classes under block residency (mt_set_residency 2): runs of at least big_min_ops op
 * records replay in the wide block-residency kernel (the same engine with room for 248 blocks
 * and a 254-entry zamboni heap in LDS, ~21 KB per workgroup; capture batches: the long-document
 * kernel) on a second stream launched first, concurrently with the block-residency kernel for
 * the other runs; 0 (the default) turns it off.  Results are identical either way. */
int  mt_set_size_class(mt_ctx* ctx, uint32_t big_min_ops);
/* Partitioned size classes under block residency (mt_set_residency 2): runs of at least
 * min_ops op records replay in the wide block-residency kernel (mt_set_size_class) on `cus` CUs
 * reserved for them (a CU-masked stream, the CUs spread evenly over the XCDs; capture batches:
 * the block-residency kernel, one document per SIMD), concurrently with the other runs in the
 * block-residency kernel on the remaining CUs; joined before the call returns its event.  The
 * longest documents then stay in LDS and no short run delays their start, which shortens the
 * step of a batch whose longest documents set it.  cus = 0 or min_ops = 0: off.
 * min_ops = MT_PARTITION_AUTO: chosen per resident batch by mt_plan_partition from the batch's
 * run lengths and the device's CU count (the bench default).  Results are identical whatever
 * the partition. */
#define MT_PARTITION_AUTO 0xFFFFFFFFu
int  mt_set_partition(mt_ctx* ctx, uint32_t min_ops, uint32_t cus);
/* The partition rule (host only, no context): for runs of run_ops[i] op records on a device of
 * n_cus CUs, the (min_ops, cus) whose estimated step is lowest, or (0, 0) for no partition,
 * with that estimate in *est_ms (null: not wanted).  The estimate is a model of the measured
 * kernels (DESIGN.md §3 "partition rule"): a batch's step is the larger of its throughput bound
 * (messages x per-message time / concurrent documents, 16 per CU in the block-residency
 * kernel, 7 in the wide one) and its latency bound (the longest run x one document's
 * per-message time, higher for a run that outgrows the block kernel's LDS); a partition must
 * beat no partition by 5 %. */
int  mt_plan_partition(const uint32_t* run_ops, uint32_t n_runs, uint32_t n_cus, uint32_t* min_ops, uint32_t* cus,
                       double* est_ms);
/* The partition the last replay launch used (after MT_PARTITION_AUTO: the one chosen). */
int  mt_last_partition(mt_ctx* ctx, uint32_t* min_ops, uint32_t* cus);
/* Block residency: a batch holding a run of at least min_ops op records (default 16,384)
 * replays in the kernel that continues an outgrown document in HBM in the same wave; other
 * batches in the kernel without that second engine (no scratch), an outgrown document
 * finishing in a second, all-HBM launch.  0: always the continuing kernel. */
int  mt_set_continuation(mt_ctx* ctx, uint32_t min_ops);
/* Per run of the last LDS-resident replay: the op index where it left LDS (== the run's
 * end when it finished in LDS).  Bit 31 (MT_CURSOR_DONE) set: the run continued from that
 * op in HBM in the same wave and finished there (no second launch); mask it off to read
 * the op index.  Diagnostic. */
#define MT_CURSOR_DONE 0x80000000u
int  mt_last_cursors(mt_ctx* ctx, uint32_t n_runs, uint32_t* out);
/* Milliseconds of the last replay kernel(s), timed with HIP events on the
 * context stream. */
int  mt_last_replay_ms(mt_ctx* ctx, float* ms);

/* seq[i] < 0 leaves document i's (minSeq, currentSeq) unchanged; the snapshot
 * entry points take the same convention for "snapshot at the current window". */
int  mt_update_seq(mt_ctx* ctx, uint32_t n, const uint32_t* doc_ids,
                   const int32_t* msn, const int32_t* seq);
int  mt_sync(mt_ctx* ctx);

int  mt_doc_status(mt_ctx* ctx, uint32_t n, const uint32_t* doc_ids, uint32_t* out_status);
int  mt_doc_counters_get(mt_ctx* ctx, uint32_t n, const uint32_t* doc_ids, mt_doc_counters* out);

/* Pool occupancy per document, 10 int32 each: rows high-water (rowTop), blocks
 * high-water, zamboni heap entries, window rows, text arena units in use,
 * property sets, tree height, recycled rows held, heap high-water, window
 * high-water.  Allocation is deterministic, so replaying the same stream needs
 * exactly these row/block/heap/window capacities (hosts size mt_create_docs
 * from a generation or earlier replay). */
int  mt_doc_pools(mt_ctx* ctx, uint32_t n, const uint32_t* doc_ids, int32_t* out);

/* Perspective length (refSeq, client) of each document (mergeTree.ts:1569). */
int  mt_get_length(mt_ctx* ctx, uint32_t n, const uint32_t* doc_ids,
                   const int32_t* ref_seq, const int32_t* client, int32_t* out_len);

/*
 * Position queries on the current state of replayed documents, batched (one wave per
 * document, its queries in order).  Query i asks about document doc_ids[i] at pos[i] under
 * the perspective (ref_seq[i], client[i]), client = per-document client index;
 * ref_seq[i] < 0 is the local (observer) view, (currentSeq, local client).
 *   MergeTree.getContainingSegment  MT/mergeTree.ts:1616-1627 (searchBlock :1786-1815;
 *                                   Client.getContainingSegment client.ts:1040-1043)
 *   MergeTree.resolveRemoteClientPosition  MT/mergeTree.ts:2125-2145
 * out[i].found = 0 when the segment is undefined (pos at or past the perspective length).
 * json_arena (optional): the library-owned toJSONObject text of each found segment
 * (textSegment.ts:48-54, mergeTree.ts:649-653), query i = bytes [json_off[i], json_off[i+1])
 * (empty when not found), valid until the next call.
 */
#define MT_POS_UNDEFINED INT32_MIN
typedef struct mt_seg_info {
    int32_t found;            /* 1: a segment holds pos under the perspective                   */
    int32_t offset;           /* pos minus the segment's start under the perspective             */
    int32_t obs_pos;          /* the segment's start in the local view (getPosition, :1578-1596) */
    int32_t len;              /* cachedLength                                                     */
    int32_t seq, client;      /* insertion seq; client index (-1: NonCollabClient)               */
    int32_t removed_seq;      /* INT32_MIN: undefined                                             */
    int32_t removed_client;   /* -1 when not removed                                              */
    int32_t prop_set;         /* the document's property-set id (mt_doc_pset), -1: undefined     */
    int32_t marker_ref_type;  /* -1: text segment                                                 */
    int32_t depth;            /* tree levels above the segment                                    */
    uint32_t path_lo, path_hi;/* child index per level, root first, 3 bits each (as mt_dump_segments) */
    int32_t row;              /* engine row id                                                    */
    int32_t resolved;         /* resolveRemoteClientPosition: obs_pos + offset; the local length
                                 when pos == the perspective length; else MT_POS_UNDEFINED      */
    int32_t pad;
} mt_seg_info;
int  mt_get_containing_segment(mt_ctx* ctx, uint32_t n, const uint32_t* doc_ids, const int32_t* pos,
                               const int32_t* ref_seq, const int32_t* client, mt_seg_info* out,
                               const char** json_arena, const uint64_t** json_off);
/* resolveRemoteClientPosition only: out_pos[i] = mt_seg_info.resolved of the same query. */
int  mt_resolve_remote_position(mt_ctx* ctx, uint32_t n, const uint32_t* doc_ids, const int32_t* pos,
                                const int32_t* ref_seq, const int32_t* client, int32_t* out_pos);

/* Client long-id strings (JSON literals) by per-document client index; used for
 * the snapshot's "client"/"removedClient" fields (snapshotV1.ts:229, :237). */
int  mt_set_client_names(mt_ctx* ctx, uint32_t n, const char* const* client_json);
/* Per-document client names (each Client interns its own long ids in first-seen
 * order, MT/client.ts:658-682); they override the table above for that
 * document.  n = 0 removes the override. */
int  mt_set_doc_client_names(mt_ctx* ctx, uint32_t doc_id, uint32_t n, const char* const* client_json);

/*
 * SnapshotV1 of each document: runs updateSeqNumbers(msn[i], seq[i]) first
 * (MT/client.ts:936), then extracts and serializes.  Blobs are concatenated into
 * a library-owned arena: document i owns blobs [blob_first[i], blob_first[i+1]);
 * blob j is bytes [blob_off[j], blob_off[j+1]) of *arena; blob 0 of a document is
 * "header", blob k>0 is "body_{k-1}".  digest[i] = xxh64-style digest of the
 * document's blob bytes (each blob prefixed by its length).
 */
int  mt_snapshot_v1(mt_ctx* ctx, uint32_t n, const uint32_t* doc_ids,
                    const int32_t* msn, const int32_t* seq,
                    uint64_t* out_digest,
                    const char** arena, const uint64_t** blob_off,
                    const uint32_t** blob_first);
/*
 * SnapshotLegacy of each document, the reference's default format when
 * options.newMergeTreeSnapshotFormat is unset (MT/client.ts:950-954 →
 * SnapshotLegacy.extractSync/emit, MT/snapshotlegacy.ts:104-240): after
 * updateSeqNumbers(msn[i], seq[i]), the segments at or below the MSN (removes
 * above the MSN keep their text), coalesced, in a "header" chunk of ≥ 10,000
 * characters and, if segments remain, one "body" chunk.  Same arena layout and
 * digest as mt_snapshot_v1.  The catch-up ops blob (snapshotlegacy.ts:162-172)
 * holds the caller's messages and is appended by the host.
 */
int  mt_snapshot_legacy(mt_ctx* ctx, uint32_t n, const uint32_t* doc_ids,
                        const int32_t* msn, const int32_t* seq,
                        uint64_t* out_digest,
                        const char** arena, const uint64_t** blob_off,
                        const uint32_t** blob_first);
/* options.mergeTreeSnapshotChunkSize of each document's Client (MergeTree options,
 * MT/client.ts:82-84; SnapshotV1 reads `mergeTree.options?.mergeTreeSnapshotChunkSize ??
 * SnapshotV1.chunkSize`, MT/snapshotV1.ts:55): mt_snapshot_v1 / mt_snapshot_digests close a
 * chunk once its length reaches chunk_size[i] (getSeqLengthSegs, snapshotV1.ts:70-92), and
 * mt_snapshot_legacy cuts its first ("header") chunk at it (`options?.mergeTreeSnapshotChunkSize
 * ?? sizeOfFirstChunk`, snapshotlegacy.ts:71, :109).  The value is the option after JS
 * ToNumber (the comparison `length < chunkSize`): 0 = the default 10,000;
 * MT_CHUNK_INFINITY = Infinity (one chunk); MT_CHUNK_NONE = a size no length is below (0, a
 * negative number, NaN, -Infinity: the legacy header chunk is empty and the body holds every
 * segment; SnapshotV1's chunk loop never ends on a non-empty document, so mt_snapshot_v1 /
 * mt_snapshot_digests fail with MT_E_INVALID there instead of hanging).  Lengths are integers,
 * so a positive non-integer size c acts as ceil(c).  mt_docs_open resets the documents it
 * opens to the default. */
#define MT_CHUNK_INFINITY   0xFFFFFFFFFFFFFFFFull
#define MT_CHUNK_NONE       0xFFFFFFFFFFFFFFFEull
int  mt_set_doc_snapshot_chunk(mt_ctx* ctx, uint32_t n, const uint32_t* doc_ids, const uint64_t* chunk_size);
/* Digests only (same values as mt_snapshot_v1's), for many documents: one staged
 * download, serialization spread over `threads` host threads. */
int  mt_snapshot_digests(mt_ctx* ctx, uint32_t n, const uint32_t* doc_ids, const int32_t* msn,
                         const int32_t* seq, uint64_t* out_digest, int threads);
/* Pin the two host staging buffers that mt_snapshot_* and mt_get_text download documents
 * through (double-buffered groups of documents), each at least `bytes` (0: the default group
 * budget, 384 MiB), so later calls do not pay for pinning host memory: a serving process
 * reserves once at startup.  Calls without a reservation pin on first use and grow the buffers
 * to the largest group of the call. */
int  mt_reserve_staging(mt_ctx* ctx, uint64_t bytes);
/* Observer text (UTF-16) of each document into a library-owned arena. */
int  mt_get_text(mt_ctx* ctx, uint32_t n, const uint32_t* doc_ids,
                 const uint16_t** arena, const uint64_t** off);
/* walkAllSegments order dump: per row {len, seq, client, removed_seq (INT32_MIN =
 * undefined), removed_client, overlap_mask_lo, overlap_mask_hi, prop_set(-1 none),
 * marker_ref_type(-1 text), text_off, parent_block, flags}. 12 int32 per row. */
/* SnapshotLoader (MT/snapshotLoader.ts:39-222) for each document of the batch:
 * the slot is reset, the header segments are built bottom-up into the B-tree
 * (reloadFromSegments, mergeTree.ts:1185-1238), collaboration starts at
 * (min_seq, seq) (client.ts:1073, mergeTree.ts:1243), and the body segments are
 * appended as loadBody does (snapshotLoader.ts:162-206: runs of universal
 * segments batched, others one by one, at the observer's length under
 * perspective (UniversalSequenceNumber, segment client)).  Where the reference
 * would throw ("MergeTree insert failed", mergeTree.ts:2228) the document gets
 * MT_DS_INSERT_FAILED; where its never-emptied loadBody batch would link one
 * segment object twice the document gets MT_DS_UNSUPPORTED.  Stream-ordered;
 * status words after mt_sync. */
int  mt_load_snapshot(mt_ctx* ctx, const mt_load_batch* batch);
/* The build's source hash (sha256 prefix of csrc/ + this header, __graft_entry__.source_hash):
 * lets a host prove the library it loaded was compiled from its own tree. */
const char* mt_source_hash(void);
/* Delta capture for the following batches (mt_apply_batch / mt_replay_resident): a device
 * buffer of `capacity` records (raised to one message of the largest document); 0 turns
 * capture off (the default: the replay kernels then never touch the record buffer).  A
 * batch never overflows it: before each message a document reserves the records it can
 * emit, and when a launch is full the run stops before that message, the records move to
 * the host and a further launch resumes the stopped runs, so a capture batch of any size
 * completes (mt_apply_batch is synchronous while capture is armed). */
int  mt_delta_capture(mt_ctx* ctx, uint64_t capacity);
/* The records of the last batch in callback order per document and op (sorted by op
 * index, program order within an op): a library-owned array valid until the next
 * batch.  MT_E_OOM if the batch produced more than the capacity. */
int  mt_delta_records(mt_ctx* ctx, const mt_delta_rec** out, uint64_t* n);
/* The UTF-16 text of the last batch's pasted text segments (INSERT records with b == 0 index
 * it), a library-owned array valid until the next batch; *launches (optional) = the device
 * launches the batch took. */
int  mt_delta_text(mt_ctx* ctx, const uint16_t** out, uint64_t* n, uint32_t* launches);
/* The keys and values (host-interned ids, value -1 never occurs) of property set
 * pset_id of document doc, in insertion order; returns the count in *n (<= MT_MAX_PROP_KEYS:
 * keys and values must have room for MT_MAX_PROP_KEYS entries). */
#define MT_MAX_PROP_KEYS 256   /* keys of one segment's property map (more: MT_DS_PROPS_TOO_MANY) */
int  mt_doc_pset(mt_ctx* ctx, uint32_t doc, int32_t pset_id, uint16_t* keys, int32_t* values, uint32_t* n);
int  mt_dump_segments(mt_ctx* ctx, uint32_t doc_id, int32_t** rows, uint32_t* n_rows);
void mt_free(void* p);

/* Diagnostic: per-document phase cycle counters (8 u64 each); zeros unless the
 * library was built with -DMT_PROFILE (tools/phase_profile.py). */
int  mt_prof_get(mt_ctx* ctx, uint32_t n_docs_from_0, unsigned long long* out);

/* Synthetic stream generation on the device (SURVEY.md §8(d) stream rules):
 * the engine itself acts as sequencer + observer, so every position is valid
 * under the author's (refSeq, client) perspective. */
typedef struct mt_gen_params {
    uint64_t seed;
    uint32_t n_docs;
    uint32_t ops_per_doc;        /* messages per document                        */
    uint32_t clients;            /* authoring clients per document (<= 64)        */
    uint32_t lag_max;            /* refSeq lag U[0, lag_max]                      */
    uint32_t pct_insert;         /* op mix in percent                             */
    uint32_t pct_remove;         /* (annotate = rest)                             */
    uint32_t ins_len_max;        /* insert length U[1, ins_len_max]               */
    uint32_t rem_len_max;        /* remove/annotate length U[1, rem_len_max]      */
    uint32_t n_ann_sets;         /* annotate prop sets drawn from table [0, n)    */
    uint32_t pct_rewrite;        /* annotate rewrite percentage                   */
    uint32_t doc_id_base;        /* stream of run i is seeded as document doc_id_base + i */
    uint32_t ins_len_min;        /* insert length U[max(1, ins_len_min), ins_len_max] */
    uint32_t seg_prop_sets;      /* > 0: insert k carries segment props set k % n   */
    uint32_t ins_at_end;         /* 1: every insert appends at the author's length  */
    uint32_t continue_docs;      /* 1: continue the documents' current state (no     */
                                 /*    reopen; seqs continue from currentSeq)       */
} mt_gen_params;
int  mt_generate(mt_ctx* ctx, const mt_gen_params* params);
/* As mt_generate with per-document message counts and authoring-client counts
 * (either array may be null: params->ops_per_doc / params->clients).  Runs are
 * documents 0..n_docs-1 with op offsets = prefix sums of the counts. */
int  mt_generate_docs(mt_ctx* ctx, const mt_gen_params* params, const uint32_t* ops_per_doc,
                      const uint32_t* clients_per_doc);
/* Total op records of the last generation. */
int  mt_generated_ops(mt_ctx* ctx, uint64_t* n_ops);
/* Copy the generated stream to host memory (arrays sized mt_generated_ops,
 * payload sized mt_generated_ops * ins_len_max; op i's payload starts at
 * i * ins_len_max). */
int  mt_generated_download(mt_ctx* ctx, uint8_t* type, uint8_t* flags, uint16_t* client,
                           int32_t* seq, int32_t* ref_seq, int32_t* msn, int32_t* pos1,
                           int32_t* pos2, uint32_t* payload_off, uint32_t* payload_len,
                           int32_t* prop_id, uint16_t* payload);
/* Copy the op records of generated runs [first_run, first_run + n_runs) into a
 * caller-owned device buffer (records in run order), and their payloads (op i of
 * the copy at payload_dev + i * ins_len_max; payload_off fields are left as
 * generated).  Device pointers of this context's GPU. */
int  mt_generated_copy_dev(mt_ctx* ctx, uint32_t first_run, uint32_t n_runs, mt_op_rec* rec_dev,
                           uint16_t* payload_dev);
/* Make a device-resident batch the resident batch (as mt_upload_batch, without
 * the host copy): doc_ids/op_offsets are host arrays, records and payload are
 * device buffers that the engine copies.  The records are not inspected on the
 * host, so register ops (MT_OP_CUT / COPY / PASTE) in them set MT_DS_UNSUPPORTED
 * unless a delta capture is armed; use mt_upload_batch for such streams. */
int  mt_upload_batch_dev(mt_ctx* ctx, uint32_t n_runs, const uint32_t* doc_ids, const uint32_t* op_offsets,
                         const mt_op_rec* rec_dev, const uint16_t* payload_dev, uint64_t payload_units);
/* ---- document exchange between GPUs (fluidframework_amd/shard.py) ----
 * A document travels as rows, one per op: its op record (32 B), then its payload slot of
 * L = ins_len_max UTF-16 units, so one all-to-all moves records and text together.
 * mt_generated_pack_rows: generated runs first..first+n-1 into rows_dev (device memory)
 * starting at row dst_row[i] for run first+i, and each run's 64-bit row checksum into
 * checksum[i] (host).  mt_upload_rows_dev: received rows (run r = rows op_offsets[r] ..
 * op_offsets[r+1]-1) become the resident batch for doc_ids[r], text inserts' payload_off
 * re-pointed to their slot; every run's checksum is compared with expect[r] (the sender's)
 * and MT_E_EXCHANGE returned if any differs (bad_runs[r] = 1 for those, when non-null). */
int  mt_generated_pack_rows(mt_ctx* ctx, uint32_t first_run, uint32_t n_runs, const uint64_t* dst_row,
                            void* rows_dev, uint64_t* checksum);
int  mt_upload_rows_dev(mt_ctx* ctx, uint32_t n_runs, const uint32_t* doc_ids, const uint32_t* op_offsets,
                        const void* rows_dev, uint32_t payload_stride, const uint64_t* expect, uint32_t* bad_runs);
/* Make the generated stream the resident batch (docs 0..n_docs-1). */
int  mt_generated_to_resident(mt_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* MTGPU_H */
