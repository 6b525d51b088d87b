// mt_api_impl.h — implementation of the mtgpu.h C ABI over a backend.
//
// Included by mt_engine.hip (backend HIP: pools in HBM, one wavefront per
// document on gfx950) — the product — and by tests/emu/mt_emu.cpp (backend
// EMU: host memory + host-emulated waves), which exists only so the CPU test
// suite can exercise the identical engine logic against the oracle.
//
// Required from the includer:
//   MT_FN(name)           exported symbol name
//   mtb_malloc/mtb_free   pool allocation
//   mtb_h2d/mtb_d2h/mtb_memset, mtb_sync
//   mtb_launch_replay(ctx, S, ops, gen, n_runs)
//   mtb_launch_open(ctx, S, first, n)
//   mtb_launch_update_seq(ctx, S, docs, msn, seq, n)
//   mtb_launch_get_length(ctx, S, docs, ref, cli, out, n)
//   mtb_event_start / mtb_event_stop_ms
#pragma once
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>
#include "mt_ctx.h"

static int mtb_ensure(mt_ctx* c, mt_ctx::DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return MT_OK;
    if (b.p) mtb_free(b.p);
    b.p = nullptr; b.cap = 0;
    if (mtb_malloc(&b.p, bytes) != 0) { c->err = "device allocation failed"; return MT_E_OOM; }
    b.cap = bytes;
    return MT_OK;
}

extern "C" {

const char* MT_FN(last_error)(mt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int MT_FN(create)(int device, const mt_limits* L, mt_ctx** out) {
    if (!L || !out || L->max_docs == 0) return MT_E_INVALID;
    mt_ctx* c = new mt_ctx();
    c->device = device; c->lim = *L;
    if (mtb_init(c) != 0) { *out = c; return MT_E_HIP; }
    MtState& S = c->S;
    S.maxDocs = L->max_docs;
    S.rowCap = L->rows_per_doc ? L->rows_per_doc : 4096;
    S.blkCap = L->blocks_per_doc ? L->blocks_per_doc : S.rowCap / 2 + 64;
    S.heapCap = L->heap_per_doc ? L->heap_per_doc : S.rowCap;
    S.winCap = L->window_per_doc ? L->window_per_doc : 4096;
    S.textCap = L->text_per_doc ? L->text_per_doc : S.rowCap * 8;
    S.psetCap = L->propsets_per_doc ? L->propsets_per_doc : 1024;
    S.holdCap = MT_RFL;
    const size_t D = S.maxDocs, R = (size_t)D * S.rowCap;
    void* p;
#define MT_ALLOC(field, T, count) \
    if (mtb_malloc(&p, sizeof(T) * (size_t)(count)) != 0) { c->err = "pool allocation failed: " #field; *out = c; return MT_E_OOM; } \
    S.field = (T*)p;
    MT_ALLOC(rows, MtRow, R)
    MT_ALLOC(blk, MtBlk, D * S.blkCap) MT_ALLOC(heap, MtHeapE, D * (S.heapCap + 1)) MT_ALLOC(win, int, D * S.winCap)
    MT_ALLOC(uid, int, D * S.winCap) MT_ALLOC(udelta, int, D * S.winCap) MT_ALLOC(uanc, int, D * S.winCap * MT_MAXH)
    MT_ALLOC(text, uint16_t, D * 2 * S.textCap) MT_ALLOC(pset, MtPSet, D * S.psetCap) MT_ALLOC(hdr, MtDocHdr, D)
    MT_ALLOC(hold, int, D * MT_RFL)
#undef MT_ALLOC
    mtb_memset(S.hdr, 0, sizeof(MtDocHdr) * D);
    *out = c;
    return MT_OK;
}

void MT_FN(destroy)(mt_ctx* c) {
    if (!c) return;
    MtState& S = c->S;
    void* ps[] = {S.rows, S.blk, S.heap, S.win, S.uid, S.udelta, S.uanc, S.text, S.pset, S.hdr, S.hold};
    for (void* p : ps) if (p) mtb_free(p);
    mt_ctx::DevBuf* bs[] = {&c->b_cursor, &c->b_doc, &c->b_off, &c->b_rec, &c->b_pay, &c->b_pset_off,
                            &c->b_pkey, &c->b_pval, &c->b_pfalsy, &c->b_pclass, &c->b_tmp0, &c->b_tmp1, &c->b_tmp2, &c->b_tmp3};
    for (auto* b : bs) if (b->p) mtb_free(b->p);
    mtb_fini(c);
    delete c;
}

int MT_FN(docs_open)(mt_ctx* c, uint32_t first, uint32_t n) {
    if (!c || (uint64_t)first + n > c->S.maxDocs) return MT_E_INVALID;
    if (n == 0) return MT_OK;
    return mtb_launch_open(c, first, n);
}

int MT_FN(set_props)(mt_ctx* c, const mt_prop_table* P) {
    if (!c || !P) return MT_E_INVALID;
    const uint32_t npairs = P->set_off[P->n_sets];
    int rc;
    if ((rc = mtb_ensure(c, c->b_pset_off, 4ull * (P->n_sets + 1)))) return rc;
    if ((rc = mtb_ensure(c, c->b_pkey, 2ull * npairs + 2))) return rc;
    if ((rc = mtb_ensure(c, c->b_pval, 4ull * npairs + 4))) return rc;
    if ((rc = mtb_ensure(c, c->b_pfalsy, 1ull * P->n_values + 1))) return rc;
    if ((rc = mtb_ensure(c, c->b_pclass, 4ull * P->n_values + 4))) return rc;
    mtb_h2d(c, c->b_pset_off.p, P->set_off, 4ull * (P->n_sets + 1));
    if (npairs) { mtb_h2d(c, c->b_pkey.p, P->key, 2ull * npairs); mtb_h2d(c, c->b_pval.p, P->value, 4ull * npairs); }
    if (P->n_values) { mtb_h2d(c, c->b_pfalsy.p, P->value_falsy, P->n_values); mtb_h2d(c, c->b_pclass.p, P->value_class, 4ull * P->n_values); }
    mtb_sync(c);
    c->S.p_off = (const uint32_t*)c->b_pset_off.p; c->S.p_key = (const uint16_t*)c->b_pkey.p;
    c->S.p_val = (const int32_t*)c->b_pval.p; c->S.p_falsy = (const uint8_t*)c->b_pfalsy.p;
    c->S.p_class = (const uint32_t*)c->b_pclass.p; c->S.p_nsets = P->n_sets;
    c->names.key_json.assign(P->key_json, P->key_json + P->n_keys);
    c->names.key_index.assign(P->key_index, P->key_index + P->n_keys);
    c->names.value_json.assign(P->value_json, P->value_json + P->n_values);
    c->names.value_class.assign(P->value_class, P->value_class + P->n_values);
    return MT_OK;
}

int MT_FN(set_client_names)(mt_ctx* c, uint32_t n, const char* const* cj) {
    if (!c || (n && !cj)) return MT_E_INVALID;
    c->names.client_json.assign(cj, cj + n);
    return MT_OK;
}
int MT_FN(set_doc_client_names)(mt_ctx* c, uint32_t doc, uint32_t n, const char* const* cj) {
    if (!c || doc >= c->S.maxDocs || (n && !cj)) return MT_E_INVALID;
    if (n == 0) c->doc_clients.erase(doc);
    else c->doc_clients[doc].assign(cj, cj + n);
    return MT_OK;
}

static int mt_upload_ops(mt_ctx* c, const mt_op_batch* B) {
    const size_t N = B->n_ops, R = B->n_runs;
    int rc;
    std::vector<MtOpRec> rec(N ? N : 1);
    for (size_t i = 0; i < N; i++) {
        MtOpRec& o = rec[i];
        o.type = B->type[i]; o.flags = B->flags[i]; o.client = B->client[i]; o.seq = B->seq[i]; o.ref_seq = B->ref_seq[i];
        o.msn = B->msn[i]; o.pos1 = B->pos1[i]; o.pos2 = B->pos2[i]; o.payload_off = B->payload_off[i];
        o.payload_len = (uint16_t)B->payload_len[i]; o.prop_id = (int16_t)B->prop_id[i];
    }
#define UP(buf, src, bytes) if ((rc = mtb_ensure(c, c->buf, (bytes)))) return rc; if ((bytes) && (src)) mtb_h2d(c, c->buf.p, (src), (bytes));
    UP(b_doc, B->doc_ids, 4 * R) UP(b_off, B->op_offsets, 4 * (R + 1)) UP(b_rec, rec.data(), sizeof(MtOpRec) * N)
    UP(b_pay, B->payload, 2 * B->payload_units)
#undef UP
    MtOps& o = c->ops;
    o.doc_ids = (const uint32_t*)c->b_doc.p; o.op_off = (const uint32_t*)c->b_off.p; o.rec = (MtOpRec*)c->b_rec.p;
    o.payload = (uint16_t*)c->b_pay.p; o.n_runs = B->n_runs;
    c->n_runs = B->n_runs;
    return MT_OK;
}

static int mt_check_batch(mt_ctx* c, const mt_op_batch* B) {
    if (!B || !B->op_offsets || (B->n_runs && !B->doc_ids)) { c->err = "null batch arrays"; return MT_E_INVALID; }
    if (B->op_offsets[B->n_runs] != B->n_ops) { c->err = "op_offsets[n_runs] != n_ops"; return MT_E_INVALID; }
    for (uint32_t r = 0; r < B->n_runs; r++) {
        if (B->doc_ids[r] >= c->S.maxDocs) { c->err = "doc id out of range"; return MT_E_INVALID; }
        if (B->op_offsets[r] > B->op_offsets[r + 1]) { c->err = "op_offsets not monotone"; return MT_E_INVALID; }
    }
    for (uint32_t i = 0; i < B->n_ops; i++) {
        if (B->type[i] == MT_OP_INSERT && !(B->flags[i] & MT_OPF_MARKER) &&
            (uint64_t)B->payload_off[i] + B->payload_len[i] > B->payload_units) { c->err = "payload out of range"; return MT_E_INVALID; }
        if (B->prop_id[i] >= 0 && (uint32_t)B->prop_id[i] >= c->S.p_nsets) { c->err = "prop_id out of range (mt_set_props first)"; return MT_E_INVALID; }
        if (B->prop_id[i] > 32767) { c->err = "more than 32767 property sets"; return MT_E_INVALID; }
        if (B->payload_len[i] > 65535) { c->err = "insert longer than 65535 UTF-16 units"; return MT_E_INVALID; }
    }
    return MT_OK;
}

int MT_FN(upload_batch)(mt_ctx* c, const mt_op_batch* B) {
    if (!c) return MT_E_INVALID;
    int rc = mt_check_batch(c, B);
    if (rc) return rc;
    rc = mt_upload_ops(c, B);
    mtb_sync(c);
    return rc;
}
int MT_FN(replay_resident)(mt_ctx* c) {
    if (!c || !c->ops.op_off) return MT_E_INVALID;
    int rc = mtb_ensure(c, c->b_cursor, 4ull * c->n_runs + 4);
    if (rc) return rc;
    MtGen g{}; g.enabled = 0;
    return mtb_launch_replay(c, g, c->n_runs);
}
int MT_FN(apply_batch)(mt_ctx* c, const mt_op_batch* B) {
    int rc = MT_FN(upload_batch)(c, B);
    if (rc) return rc;
    return MT_FN(replay_resident)(c);
}
int MT_FN(set_residency)(mt_ctx* c, int use_lds, int rows, int blocks, int heap) {
    if (!c || rows < 0 || blocks < 0 || heap < 0 || rows > MT_L_ROWS || blocks > MT_L_BLKS || heap > MT_L_HEAP)
        return MT_E_INVALID;
    c->use_lds = use_lds ? 1 : 0;
    c->lds_rows = rows ? rows : MT_L_ROWS; c->lds_blks = blocks ? blocks : MT_L_BLKS; c->lds_heap = heap ? heap : MT_L_HEAP;
    return MT_OK;
}
int MT_FN(last_replay_ms)(mt_ctx* c, float* ms) { if (!c || !ms) return MT_E_INVALID; *ms = c->last_ms; return MT_OK; }
int MT_FN(sync)(mt_ctx* c) { if (!c) return MT_E_INVALID; return mtb_sync(c); }

static int mt_read_hdrs(mt_ctx* c, uint32_t n, const uint32_t* docs, std::vector<MtDocHdr>& h) {
    h.resize(n);
    mtb_sync(c);
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (docs[i] >= c->S.maxDocs) return MT_E_INVALID;
        lo = docs[i] < lo ? docs[i] : lo; hi = docs[i] > hi ? docs[i] : hi;
    }
    if (n == 0) return MT_OK;
    if (n < 8) {
        for (uint32_t i = 0; i < n; i++) mtb_d2h(c, &h[i], c->S.hdr + docs[i], sizeof(MtDocHdr));
        return MT_OK;
    }
    std::vector<MtDocHdr> all((size_t)(hi - lo + 1));      // one copy of the covering header range
    mtb_d2h(c, all.data(), c->S.hdr + lo, sizeof(MtDocHdr) * all.size());
    for (uint32_t i = 0; i < n; i++) h[i] = all[docs[i] - lo];
    return MT_OK;
}
int MT_FN(doc_pools)(mt_ctx* c, uint32_t n, const uint32_t* docs, int32_t* out) {
    if (!c || (n && (!docs || !out))) return MT_E_INVALID;
    std::vector<MtDocHdr> h;
    int rc = mt_read_hdrs(c, n, docs, h);
    if (rc) return rc;
    for (uint32_t i = 0; i < n; i++) {
        int32_t* o = out + 8 * (size_t)i;
        o[0] = h[i].rowTop; o[1] = h[i].blkTop; o[2] = h[i].heapN; o[3] = h[i].winN;
        o[4] = h[i].textTop; o[5] = h[i].psetTop; o[6] = h[i].height; o[7] = h[i].rfN;
    }
    return MT_OK;
}
int MT_FN(doc_status)(mt_ctx* c, uint32_t n, const uint32_t* docs, uint32_t* out) {
    std::vector<MtDocHdr> h;
    int rc = mt_read_hdrs(c, n, docs, h);
    if (rc) return rc;
    for (uint32_t i = 0; i < n; i++) out[i] = h[i].status;
    return MT_OK;
}
int MT_FN(doc_counters_get)(mt_ctx* c, uint32_t n, const uint32_t* docs, mt_doc_counters* out) {
    std::vector<MtDocHdr> h;
    int rc = mt_read_hdrs(c, n, docs, h);
    if (rc) return rc;
    for (uint32_t i = 0; i < n; i++) {
        out[i].ops = h[i].cnt[0]; out[i].msgs = h[i].cnt[1]; out[i].ins_units = h[i].cnt[2];
        out[i].rows_rw = h[i].cnt[3]; out[i].depth = h[i].cnt[4]; out[i].scoured = h[i].cnt[5];
    }
    return MT_OK;
}

int MT_FN(update_seq)(mt_ctx* c, uint32_t n, const uint32_t* docs, const int32_t* msn, const int32_t* seq) {
    if (!c) return MT_E_INVALID;
    int rc;
    if ((rc = mtb_ensure(c, c->b_tmp0, 4ull * n))) return rc;
    if ((rc = mtb_ensure(c, c->b_tmp1, 4ull * n))) return rc;
    if ((rc = mtb_ensure(c, c->b_tmp2, 4ull * n))) return rc;
    mtb_h2d(c, c->b_tmp0.p, docs, 4ull * n); mtb_h2d(c, c->b_tmp1.p, msn, 4ull * n); mtb_h2d(c, c->b_tmp2.p, seq, 4ull * n);
    return mtb_launch_update_seq(c, (const uint32_t*)c->b_tmp0.p, (const int32_t*)c->b_tmp1.p, (const int32_t*)c->b_tmp2.p, n);
}

int MT_FN(get_length)(mt_ctx* c, uint32_t n, const uint32_t* docs, const int32_t* ref, const int32_t* cli, int32_t* out) {
    if (!c) return MT_E_INVALID;
    int rc;
    if ((rc = mtb_ensure(c, c->b_tmp0, 4ull * n))) return rc;
    if ((rc = mtb_ensure(c, c->b_tmp1, 4ull * n))) return rc;
    if ((rc = mtb_ensure(c, c->b_tmp2, 4ull * n))) return rc;
    if ((rc = mtb_ensure(c, c->b_tmp3, 4ull * n))) return rc;
    mtb_h2d(c, c->b_tmp0.p, docs, 4ull * n); mtb_h2d(c, c->b_tmp1.p, ref, 4ull * n); mtb_h2d(c, c->b_tmp2.p, cli, 4ull * n);
    rc = mtb_launch_get_length(c, (const uint32_t*)c->b_tmp0.p, (const int32_t*)c->b_tmp1.p, (const int32_t*)c->b_tmp2.p,
                               (int32_t*)c->b_tmp3.p, n);
    if (rc) return rc;
    mtb_sync(c);
    mtb_d2h(c, out, c->b_tmp3.p, 4ull * n);
    return MT_OK;
}

// Host copy of one document's state (for serialization).
struct MtHostDoc {
    MtDocHdr hdr;
    std::vector<MtRow> rows;
    std::vector<MtBlk> blk; std::vector<uint16_t> text; std::vector<MtPSet> pset;
    MtSnapView view() const {
        MtSnapView v; v.hdr = hdr; v.R = rows.data(); v.blk = blk.data(); v.text = text.data(); v.pset = pset.data();
        return v;
    }
};
static int mt_download_doc(mt_ctx* c, uint32_t d, MtHostDoc& h) {
    const MtState& S = c->S;
    mtb_d2h(c, &h.hdr, S.hdr + d, sizeof(MtDocHdr));
    const size_t R = (size_t)h.hdr.rowTop, r0 = (size_t)d * S.rowCap;
    h.rows.resize(R + 1);
    if (R) mtb_d2h(c, h.rows.data(), S.rows + r0, sizeof(MtRow) * R);
    h.blk.resize((size_t)h.hdr.blkTop + 1);
    mtb_d2h(c, h.blk.data(), S.blk + (size_t)d * S.blkCap, sizeof(MtBlk) * (size_t)h.hdr.blkTop);
    h.text.resize((size_t)h.hdr.textTop + 1);
    if (h.hdr.textTop) mtb_d2h(c, h.text.data(), S.text + ((size_t)d * 2 + (size_t)h.hdr.textHalf) * S.textCap, 2 * (size_t)h.hdr.textTop);
    h.pset.resize((size_t)h.hdr.psetTop + 1);
    if (h.hdr.psetTop) mtb_d2h(c, h.pset.data(), S.pset + (size_t)d * S.psetCap, sizeof(MtPSet) * (size_t)h.hdr.psetTop);
    return MT_OK;
}

int MT_FN(snapshot_v1)(mt_ctx* c, uint32_t n, const uint32_t* docs, const int32_t* msn, const int32_t* seq,
                       uint64_t* digest, const char** arena, const uint64_t** blob_off, const uint32_t** blob_first) {
    if (!c) return MT_E_INVALID;
    int rc = MT_FN(update_seq)(c, n, docs, msn, seq);       // Client.snapshot: updateSeqNumbers first (client.ts:936)
    if (rc) return rc;
    mtb_sync(c);
    c->snap_arena.clear(); c->blob_off.assign(1, 0); c->blob_first.assign(1, 0);
    MtHostDoc h;
    for (uint32_t i = 0; i < n; i++) {
        mt_download_doc(c, docs[i], h);
        auto dn = c->doc_clients.find(docs[i]);
        std::vector<std::string> blobs = mtsnap::snapshot_blobs(h.view(), c->names,
                                                                dn == c->doc_clients.end() ? nullptr : &dn->second);
        if (digest) digest[i] = mtsnap::blobs_digest(blobs);
        for (auto& b : blobs) { c->snap_arena += b; c->blob_off.push_back(c->snap_arena.size()); }
        c->blob_first.push_back((uint32_t)(c->blob_off.size() - 1));
    }
    if (arena) *arena = c->snap_arena.data();
    if (blob_off) *blob_off = c->blob_off.data();
    if (blob_first) *blob_first = c->blob_first.data();
    return MT_OK;
}

int MT_FN(get_text)(mt_ctx* c, uint32_t n, const uint32_t* docs, const uint16_t** arena, const uint64_t** off) {
    if (!c) return MT_E_INVALID;
    mtb_sync(c);
    c->text_arena.clear(); c->text_off.assign(1, 0);
    MtHostDoc h;
    for (uint32_t i = 0; i < n; i++) {
        mt_download_doc(c, docs[i], h);
        mtsnap::observer_text(h.view(), c->text_arena);
        c->text_off.push_back(c->text_arena.size());
    }
    if (arena) *arena = c->text_arena.data();
    if (off) *off = c->text_off.data();
    return MT_OK;
}

int MT_FN(dump_segments)(mt_ctx* c, uint32_t d, int32_t** rows, uint32_t* n_rows) {
    if (!c || d >= c->S.maxDocs) return MT_E_INVALID;
    mtb_sync(c);
    MtHostDoc h;
    mt_download_doc(c, d, h);
    std::vector<int32_t> r;
    mtsnap::dump_rows(h.view(), c->names, r);
    *n_rows = (uint32_t)(r.size() / 12);
    *rows = (int32_t*)malloc(r.size() * 4 + 4);
    if (!r.empty()) memcpy(*rows, r.data(), r.size() * 4);
    return MT_OK;
}
void MT_FN(free)(void* p) { free(p); }

// Diagnostic (MT_PROFILE builds fill it; product builds return zeros): phase cycles per doc.
int MT_FN(prof_get)(mt_ctx* c, uint32_t n, unsigned long long* out) {
    if (!c || n > c->S.maxDocs) return MT_E_INVALID;
    mtb_sync(c);
    std::vector<MtDocHdr> h(n);
    mtb_d2h(c, h.data(), c->S.hdr, sizeof(MtDocHdr) * n);
    for (uint32_t i = 0; i < n; i++) for (int k = 0; k < 8; k++) out[i * 8 + k] = h[i].prof[k];
    return MT_OK;
}

int MT_FN(generate)(mt_ctx* c, const mt_gen_params* P) {
    if (!c || !P || P->n_docs == 0 || P->n_docs > c->S.maxDocs || P->clients == 0 || P->clients > 64 ||
        P->ins_len_max == 0 || P->rem_len_max == 0 || P->n_ann_sets == 0) return MT_E_INVALID;
    if (P->pct_insert + P->pct_remove < 100 && P->n_ann_sets > c->S.p_nsets) { c->err = "annotate prop sets not uploaded"; return MT_E_INVALID; }
    const size_t N = (size_t)P->n_docs * P->ops_per_doc;
    const size_t PU = N * P->ins_len_max + 1;
    int rc;
#define AL(buf, bytes) if ((rc = mtb_ensure(c, c->buf, (bytes)))) return rc;
    AL(b_doc, 4ull * P->n_docs) AL(b_off, 4ull * (P->n_docs + 1)) AL(b_rec, sizeof(MtOpRec) * N) AL(b_pay, 2 * PU)
#undef AL
    std::vector<uint32_t> docs(P->n_docs), off(P->n_docs + 1);
    for (uint32_t i = 0; i < P->n_docs; i++) { docs[i] = i; off[i] = (uint32_t)((size_t)i * P->ops_per_doc); }
    off[P->n_docs] = (uint32_t)N;
    mtb_h2d(c, c->b_doc.p, docs.data(), 4ull * P->n_docs);
    mtb_h2d(c, c->b_off.p, off.data(), 4ull * (P->n_docs + 1));
    MtOps& o = c->ops;
    o.doc_ids = (const uint32_t*)c->b_doc.p; o.op_off = (const uint32_t*)c->b_off.p; o.rec = (MtOpRec*)c->b_rec.p;
    o.payload = (uint16_t*)c->b_pay.p; o.n_runs = P->n_docs;
    c->n_runs = P->n_docs;
    rc = MT_FN(docs_open)(c, 0, P->n_docs);
    if (rc) return rc;
    MtGen g{};
    g.seed = P->seed; g.ops = P->ops_per_doc; g.clients = P->clients; g.lag_max = P->lag_max;
    g.pct_insert = P->pct_insert; g.pct_remove = P->pct_remove; g.ins_len_max = P->ins_len_max;
    g.rem_len_max = P->rem_len_max; g.n_ann_sets = P->n_ann_sets; g.pct_rewrite = P->pct_rewrite; g.enabled = 1;
    c->gen = g; c->gen_docs = P->n_docs;
    return mtb_launch_replay(c, g, P->n_docs);
}

int MT_FN(generated_download)(mt_ctx* c, uint8_t* type, uint8_t* flags, uint16_t* client, int32_t* seq, int32_t* ref,
                              int32_t* msn, int32_t* pos1, int32_t* pos2, uint32_t* poff, uint32_t* plen, int32_t* pid,
                              uint16_t* payload) {
    if (!c || !c->gen_docs) return MT_E_INVALID;
    mtb_sync(c);
    const size_t N = (size_t)c->gen_docs * c->gen.ops;
    std::vector<MtOpRec> rec(N ? N : 1);
    mtb_d2h(c, rec.data(), c->ops.rec, sizeof(MtOpRec) * N);
    for (size_t i = 0; i < N; i++) {
        const MtOpRec& o = rec[i];
        type[i] = o.type; flags[i] = o.flags; client[i] = o.client; seq[i] = o.seq; ref[i] = o.ref_seq; msn[i] = o.msn;
        pos1[i] = o.pos1; pos2[i] = o.pos2; poff[i] = o.payload_off; plen[i] = o.payload_len; pid[i] = o.prop_id;
    }
    mtb_d2h(c, payload, c->ops.payload, 2 * (N * c->gen.ins_len_max));
    return MT_OK;
}
int MT_FN(generated_to_resident)(mt_ctx* c) {
    if (!c || !c->gen.enabled) return MT_E_INVALID;
    c->gen.enabled = 0;
    return MT_OK;
}

}  // extern "C"
