// mt_ctx.h — engine context (one per GPU) shared by the backends and the ABI.
#pragma once
#include <string>
#include <unordered_map>
#include <vector>
#include "mt_replay.h"
#include "mt_snapshot.h"
#include "mt_pack.h"
#include "mt_query.h"

struct mt_ctx {
    int device = 0;
    mt_limits lim{};
    MtState S{};
    MtNames names;
    std::vector<MtDocLayout> layout_h;                                     // host copy of S.layout
    uint64_t pool_bytes = 0;
    MtDocLayout tot{};                                                     // pool element totals
    // mt_checkpoint shadows (device)
    void *ck_rows = nullptr, *ck_blk = nullptr, *ck_heap = nullptr, *ck_win = nullptr, *ck_text = nullptr,
         *ck_pset = nullptr, *ck_hdr = nullptr, *ck_hold = nullptr, *ck_ovx = nullptr, *ck_mid = nullptr, *ck_reg = nullptr, *ck_regr = nullptr;
    bool ck_valid = false;
    std::unordered_map<uint32_t, std::vector<std::string>> doc_clients;   // mt_set_doc_client_names
    std::string err;
    // device op batch (resident)
    struct DevBuf { void* p = nullptr; size_t cap = 0; };
    DevBuf b_stage, b_pack_docs, b_pack_sz, b_pack_off, b_gencl, b_cursor, b_doc, b_off, b_rec, b_pay, b_pbase, b_rel, b_drec, b_dcount, b_pset_off, b_pkey, b_pval, b_pfalsy, b_pclass, b_pkind, b_tmp0, b_tmp1, b_tmp2, b_tmp3,
           b_ld_meta, b_ld_seg, b_ld_pay, b_ld_plan, b_ld_poff, b_dtext, b_resume, b_start,
           b_q, b_qgrp, b_qout, b_qat, b_qlen, b_qoff, b_qtext;   // position queries (mt_get_containing_segment)
    DevBuf b_runs, b_batch;
    // Every device buffer above, for mt_destroy (one list beside the declarations).
    std::vector<DevBuf*> dev_bufs() {
        return {&b_stage, &b_pack_docs, &b_pack_sz, &b_pack_off, &b_gencl, &b_cursor, &b_doc, &b_off, &b_rec, &b_pay, &b_pbase,
                &b_rel, &b_drec, &b_dcount, &b_pset_off, &b_pkey, &b_pval, &b_pfalsy, &b_pclass, &b_pkind, &b_tmp0, &b_tmp1,
                &b_tmp2, &b_tmp3, &b_ld_meta, &b_ld_seg, &b_ld_pay, &b_ld_plan, &b_ld_poff, &b_dtext, &b_resume, &b_start, &b_q,
                &b_qgrp, &b_qout, &b_qat, &b_qlen, &b_qoff, &b_qtext, &b_runs, &b_batch};
    }
    // options.mergeTreeSnapshotChunkSize per document (mt_set_doc_snapshot_chunk; 0 = 10,000)
    std::vector<uint64_t> snap_chunk;
    uint64_t chunk_of(uint32_t d) const { return d < snap_chunk.size() ? snap_chunk[d] : 0; }
    MtOps ops{};
    uint32_t n_runs = 0;
    std::vector<uint32_t> run_off;     // host copy of the resident batch's op offsets (n_runs + 1)
    uint64_t batch_gen = 0;            // bumped whenever a batch becomes resident
    // Size classes (mt_set_size_class): runs of at least big_min_ops op records replay in the
    // long-document kernel on stream2, concurrently with the block-residency kernel for the
    // rest; the run lists live in b_runs (long runs first), rebuilt per resident batch.
    uint32_t big_min_ops = 0;
    uint64_t runs_gen = ~0ull; uint32_t runs_min = 0, n_long = 0, n_short = 0;
    void* stream2 = nullptr; void* ev_fork = nullptr; void* ev_join = nullptr;
    // Partitioned size classes (mt_set_partition): part_cus > 0 sends the long runs to the
    // block-residency kernel on a stream masked to part_cus CUs, one document per SIMD (the
    // launch pads each workgroup's LDS to a quarter of the CU's), and the rest to the other CUs.
    uint32_t part_cus = 0, part_made = 0;
    // MT_PARTITION_AUTO: big_min_ops / part_cus chosen per resident batch (mt_plan_partition)
    bool part_auto = false; uint64_t auto_gen = ~0ull;
    // Block residency: a batch with a run of at least cont_min_ops op records replays in the
    // kernel with the in-wave HBM continuation (a long document that outgrows LDS keeps its head
    // start); other batches in the one without it (no scratch; an outgrown document finishes
    // in a second, all-HBM launch).
    uint32_t cont_min_ops = 16384, n_cont = 0, n_nocont = 0, cont_min_made = 0;
    uint64_t cont_gen = ~0ull;
    void* streamA = nullptr; void* streamB = nullptr; void* ev_joinB = nullptr;
    // mt_apply_batch / mt_upload_batch staging: two pinned host slots used alternately, each
    // with the event of its last H2D, and one device region the batch lands in
    struct Stage { void* p = nullptr; size_t cap = 0; void* ev = nullptr; };
    Stage stage[2];
    int stage_k = 0;
    void* dl_host[2] = {nullptr, nullptr}; size_t dl_cap[2] = {0, 0};   // pinned host buffers of document staging (downloads)
    uint32_t stage_epoch = 0x7E000000u;            // marks of a staging's referenced property maps
    MtGen gen{};
    uint32_t gen_docs = 0;
    std::vector<uint32_t> gen_off;     // op offsets of the generated runs
    float last_ms = 0.f;
    // LDS residency of the replay (mt_set_residency): on/off and the pool caps
    bool batch_reg = false;            // the resident batch holds register ops (FULL kernels)
    // Property maps past a wave's 64 lanes (applyPropSetWide) are built only by the FULL kernels:
    // per document, the distinct keys of every property set its ops (and loaded segments) named
    // since it was opened, until they pass MT_WAVE (doc_wide: sticky until reopened); a batch
    // holding such a document replays in the FULL kernels (batch_wide).  Host copies of the
    // property sets' keys (mt_set_props) for the scan.
    bool batch_wide = false;
    bool props_wide = false;           // the property sets name more than MT_WAVE distinct keys
    std::vector<uint32_t> h_set_off; std::vector<uint16_t> h_set_key;
    std::vector<std::vector<uint16_t>> doc_keys; std::vector<uint8_t> doc_wide;
    int use_lds = 2, lds_rows = MT_L_ROWS, lds_blks = MT_B_BLKS, lds_heap = MT_B_HEAP;
    void* stream = nullptr;
    void* ev0 = nullptr;
    void* ev1 = nullptr;
    bool ev_pending = false;
    // host-side output arenas
    std::string snap_arena;
    std::vector<uint64_t> blob_off;
    std::vector<uint32_t> blob_first;
    std::vector<uint16_t> text_arena;
    std::vector<uint64_t> text_off;
    std::string seg_json_arena;                   // mt_get_containing_segment's segment JSON
    std::vector<uint64_t> seg_json_off;
    // delta capture (mt_delta_capture / mt_delta_records)
    uint64_t delta_cap = 0, delta_tcap = 0;
    bool delta_valid = false, delta_over = false;
    std::vector<MtDeltaRec> delta_host;           // the last batch's records over all its launches
    std::vector<uint16_t> delta_text;             // pasted segments' text (INSERT records with b == 0)
    uint32_t delta_launches = 0;                  // launches the last capture batch took
};
