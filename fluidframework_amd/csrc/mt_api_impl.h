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
#include <algorithm>
#include <chrono>
#include <functional>
#include <thread>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>
#include "mt_ctx.h"
#include "mt_shard.h"

static int mtb_ensure(mt_ctx* c, mt_ctx::DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return MT_OK;
    if (b.p) mtb_free(b.p);
    b.p = nullptr; b.cap = 0;
    if (mtb_malloc(&b.p, bytes) != 0) { c->err = "device allocation failed"; return MT_E_OOM; }
    b.cap = bytes;
    return MT_OK;
}

// The run lists of the size classes for the resident batch (host lists uploaded once per
// batch): long runs (>= big_min_ops op records) in [0, n_long), the rest after them.
static int mt_size_class_lists(mt_ctx* c) {
    if (c->runs_gen == c->batch_gen && c->runs_min == c->big_min_ops) return MT_OK;
    const uint32_t R = c->n_runs;
    std::vector<uint32_t> lst; lst.reserve(R);
    for (uint32_t r = 0; r < R && c->run_off.size() == R + 1; r++)
        if (c->run_off[r + 1] - c->run_off[r] >= c->big_min_ops) lst.push_back(r);
    c->n_long = (uint32_t)lst.size();
    for (uint32_t r = 0; r < R && c->run_off.size() == R + 1; r++)
        if (c->run_off[r + 1] - c->run_off[r] < c->big_min_ops) lst.push_back(r);
    c->n_short = (uint32_t)lst.size() - c->n_long;
    int rc;
    if ((rc = mtb_ensure(c, c->b_runs, 4ull * lst.size() + 4))) return rc;
    if (!lst.empty()) mtb_h2d(c, c->b_runs.p, lst.data(), 4ull * lst.size());
    c->runs_gen = c->batch_gen; c->runs_min = c->big_min_ops;
    return MT_OK;
}

// The partition rule (mt_plan_partition): a model of the measured kernels.
// Per-message times of one document's wave, in microseconds: MT_PLAN_T_BLK in the block-
// residency kernel with 16 documents per CU (config 2: 153.5 ms / 10,000 messages; MT_PLAN_T_LONE
// alone), the same kernel's long document whose tree outgrows LDS and continues in HBM
// (MT_PLAN_T_CONT past about MT_PLAN_LDS_FIT messages: config 5's 1,302 ms / 65,521 messages
// unpartitioned), MT_PLAN_T_WIDE in the wide kernel with MT_PLAN_WIDE_PER_CU documents per CU
// (LDS-bound: 21.2 KB each; 1,048,576-document config 5 at 256:224, 5,338 ms for 699 M messages
// on 224 CUs) and MT_PLAN_T_WLONE its lone longest document (config 5: 887.9 ms / 65,521).
#define MT_PLAN_T_BLK   15.3
#define MT_PLAN_T_LONE  13.4
#define MT_PLAN_T_CONT  19.9
#define MT_PLAN_T_WIDE  12.0
#define MT_PLAN_WIDE_PER_CU 7
#define MT_PLAN_T_WLONE 13.5
#define MT_PLAN_LDS_FIT 10000u
struct MtPlanSide { double msgs = 0, extra = 0; uint32_t longest = 0; };
// Step estimate (microseconds) of one kernel on `cus` CUs holding `per_cu` documents each.
static double mt_plan_side(const MtPlanSide& s, double cus, double per_cu, double t_thr, double t_lone, bool cont) {
    if (s.msgs == 0) return 0;
    const double thr = (s.msgs * t_thr + (cont ? s.extra * (MT_PLAN_T_CONT - MT_PLAN_T_BLK) : 0)) / (cus * per_cu);
    const double lat = cont && s.longest > MT_PLAN_LDS_FIT
                           ? MT_PLAN_LDS_FIT * t_lone + (double)(s.longest - MT_PLAN_LDS_FIT) * MT_PLAN_T_CONT
                           : (double)s.longest * t_lone;
    return thr > lat ? thr : lat;
}
static void mt_plan_partition_impl(const uint32_t* len, uint32_t n, uint32_t ncu, uint32_t* min_ops, uint32_t* cus,
                                   double* est_us) {
    *min_ops = 0; *cus = 0;
    std::vector<uint32_t> L(len, len + n);
    std::sort(L.begin(), L.end(), std::greater<uint32_t>());
    // suffix sums over the sorted lengths: messages and continuation messages of the runs < m
    MtPlanSide all;
    for (uint32_t x : L) { all.msgs += x; all.extra += x > MT_PLAN_LDS_FIT ? x - MT_PLAN_LDS_FIT : 0; }
    all.longest = n ? L[0] : 0;
    const double off = mt_plan_side(all, ncu, 16, MT_PLAN_T_BLK, MT_PLAN_T_LONE, true);
    double best = off, bestSum = 0; uint32_t bm = 0, bk = 0;
    const uint32_t step = ncu >= 8 ? ncu / 8 : 1;                      // whole XCD shares
    for (uint32_t m = 256; m <= 32768 && ncu >= 2; m *= 2) {
        MtPlanSide A, B;
        for (uint32_t x : L) {
            MtPlanSide& s = x >= m ? A : B;
            s.msgs += x; s.extra += x > MT_PLAN_LDS_FIT ? x - MT_PLAN_LDS_FIT : 0;
            if (x > s.longest) s.longest = x;
        }
        if (A.msgs == 0) break;
        for (uint32_t k = step; k < ncu; k += step) {
            const double ta = mt_plan_side(A, k, MT_PLAN_WIDE_PER_CU, MT_PLAN_T_WIDE, MT_PLAN_T_WLONE, false);
            const double tb = mt_plan_side(B, ncu - k, 16, MT_PLAN_T_BLK, MT_PLAN_T_LONE, true);
            const double t = ta > tb ? ta : tb, sum = ta + tb;
            // the lowest step; within 1 % of it, the lowest total busy time
            if (t < best * 0.99 || (t <= best * 1.01 && bm && sum < bestSum)) { best = t < best ? t : best; bestSum = sum; bm = m; bk = k; }
        }
    }
    if (bm && best < off * 0.95) { *min_ops = bm; *cus = bk; if (est_us) *est_us = best; }
    else if (est_us) *est_us = off;
}
// MT_PARTITION_AUTO: the resident batch's partition from its run lengths (once per batch).
static void mt_auto_partition(mt_ctx* c) {
    if (!c->part_auto || c->use_lds != 2 || c->auto_gen == c->batch_gen) return;
    c->auto_gen = c->batch_gen;
    const uint32_t R = c->n_runs;
    if (c->run_off.size() != R + 1) { c->big_min_ops = 0; c->part_cus = 0; return; }
    std::vector<uint32_t> len(R);
    for (uint32_t r = 0; r < R; r++) len[r] = c->run_off[r + 1] - c->run_off[r];
    uint32_t m = 0, k = 0;
    mt_plan_partition_impl(len.data(), R, mtb_cu_count(c), &m, &k, nullptr);
    c->big_min_ops = m; c->part_cus = m ? k : 0;
}

// The continuation class of block residency for the resident batch: whether any run has at
// least cont_min_ops op records (n_cont > 0 launches the kernel with the in-wave continuation).
static int mt_cont_lists(mt_ctx* c) {
    if (c->cont_gen == c->batch_gen && c->cont_min_made == c->cont_min_ops) return MT_OK;
    const uint32_t R = c->n_runs;
    const bool ok = c->run_off.size() == R + 1;
    uint32_t nc = 0;
    for (uint32_t r = 0; r < R && ok; r++) nc += c->run_off[r + 1] - c->run_off[r] >= c->cont_min_ops;
    c->n_cont = ok ? nc : 0; c->n_nocont = ok ? R - nc : 0;
    c->cont_gen = c->batch_gen; c->cont_min_made = c->cont_min_ops;
    return MT_OK;
}

// Host loops over a batch's ops run on up to 16 threads once a batch is large enough to pay
// for them (ingest: validation and the SoA -> 32-byte record packing).
template <class F> static void mt_par_for(size_t n, F f) {
    unsigned T = std::thread::hardware_concurrency();
    T = T < 1 ? 1 : (T > 16 ? 16 : T);
    if (n < (size_t)1 << 16 || T == 1) { f((size_t)0, n, 0u); return; }
    const size_t per = (n + T - 1) / T;
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < T; t++) {
        const size_t a = per * t, b = a + per < n ? a + per : n;
        if (a < b) pool.emplace_back(f, a, b, t);
    }
    f((size_t)0, per < n ? per : n, 0u);
    for (auto& th : pool) th.join();
}

extern "C" {

const char* MT_FN(last_error)(mt_ctx* c) { return c ? c->err.c_str() : "null context"; }
#ifndef MT_SRC_HASH
#define MT_SRC_HASH "unhashed"
#endif
// The same hash behind a tag, so a build script can read it from the file's bytes without
// loading the library into its own process (dlopen caches a path's first handle).
__attribute__((used)) const char MT_FN(source_hash_tag)[] = "mt-src-hash:" MT_SRC_HASH;
const char* MT_FN(source_hash)(void) { return MT_FN(source_hash_tag) + 12; }

// Pools of every document, laid out back to back with per-document capacities.
static void mt_caps_default(mt_limits& q) {
    if (!q.rows_per_doc) q.rows_per_doc = 4096;
    if (!q.blocks_per_doc) q.blocks_per_doc = q.rows_per_doc / 2 + 64;
    if (!q.heap_per_doc) q.heap_per_doc = q.rows_per_doc;
    if (!q.window_per_doc) q.window_per_doc = 4096;
    if (!q.text_per_doc) q.text_per_doc = q.rows_per_doc * 8;
    if (!q.propsets_per_doc) q.propsets_per_doc = 1024;
    if (!q.markers_per_doc) q.markers_per_doc = 1024;
    if (!q.register_rows_per_doc) q.register_rows_per_doc = 256;
}
static int mt_create_impl(int device, uint32_t n_docs, const mt_limits* caps, bool uniform, mt_ctx** out) {
    mt_ctx* c = new mt_ctx();
    *out = c;
    c->device = device; c->lim = caps[0]; c->lim.max_docs = n_docs;
    if (mtb_init(c) != 0) return MT_E_HIP;
    MtState& S = c->S;
    S.maxDocs = n_docs;
    S.holdCap = MT_RFL;
    c->layout_h.resize(n_docs);
    MtDocLayout tot{};
    for (uint32_t d = 0; d < n_docs; d++) {
        mt_limits q = caps[uniform ? 0 : d];
        mt_caps_default(q);
        if (q.rows_per_doc > (1u << 30) || q.text_per_doc > (1u << 30) || q.window_per_doc > (1u << 26) ||
            q.register_rows_per_doc > (1u << 24)) {
            c->err = "per-document capacity too large"; return MT_E_INVALID;
        }
        MtDocLayout& y = c->layout_h[d];
        y.row = tot.row; y.blk = tot.blk; y.heap = tot.heap; y.win = tot.win; y.anc = tot.anc; y.text = tot.text; y.pset = tot.pset;
        y.mid = tot.mid; y.regr = tot.regr;
        y.rowCap = q.rows_per_doc; y.blkCap = q.blocks_per_doc; y.heapCap = q.heap_per_doc; y.winCap = q.window_per_doc;
        y.textCap = q.text_per_doc; y.psetCap = q.propsets_per_doc; y.midCap = q.markers_per_doc;
        y.regCap = q.register_rows_per_doc;
        tot.row += y.rowCap; tot.blk += y.blkCap; tot.heap += y.heapCap + 1; tot.win += y.winCap;
        tot.anc += (unsigned long long)y.winCap * MT_MAXH; tot.text += 2ull * y.textCap; tot.pset += y.psetCap;
        tot.mid += y.midCap; tot.regr += 2ull * y.regCap;
        S.rowCap = std::max(S.rowCap, y.rowCap); S.blkCap = std::max(S.blkCap, y.blkCap); S.heapCap = std::max(S.heapCap, y.heapCap);
        S.winCap = std::max(S.winCap, y.winCap); S.textCap = std::max(S.textCap, y.textCap); S.psetCap = std::max(S.psetCap, y.psetCap);
    }
    const size_t D = S.maxDocs;
    void* p;
#define MT_ALLOC(field, T, count) \
    if (mtb_malloc(&p, sizeof(T) * (size_t)(count)) != 0) { c->err = "pool allocation failed: " #field; return MT_E_OOM; } \
    S.field = (T*)p;
    MT_ALLOC(rows, MtRow, tot.row)
    MT_ALLOC(blk, MtBlk, tot.blk) MT_ALLOC(heap, MtHeapE, tot.heap) MT_ALLOC(win, int, tot.win)
    MT_ALLOC(uid, int, tot.win) MT_ALLOC(udelta, int, tot.win) MT_ALLOC(uanc, int, tot.anc)
    MT_ALLOC(text, uint16_t, tot.text) MT_ALLOC(pset, MtPSet, tot.pset) MT_ALLOC(hdr, MtDocHdr, D)
    MT_ALLOC(hold, int, D * MT_RFL) MT_ALLOC(ovx, MtOvx, D * MT_OVX_CAP) MT_ALLOC(mid, int, tot.mid)
    MT_ALLOC(reg, MtReg, D * MT_REG_CAP) MT_ALLOC(regr, int, tot.regr)
#undef MT_ALLOC
    if (mtb_malloc(&p, sizeof(MtDocLayout) * D) != 0) { c->err = "pool allocation failed: layout"; return MT_E_OOM; }
    S.layout = (const MtDocLayout*)p;
    mtb_h2d(c, p, c->layout_h.data(), sizeof(MtDocLayout) * D);
    mtb_memset(S.hdr, 0, sizeof(MtDocHdr) * D);
    c->tot = tot;
    c->pool_bytes = sizeof(MtRow) * tot.row + sizeof(MtBlk) * tot.blk + sizeof(MtHeapE) * tot.heap + 12ull * tot.win +
                    4ull * tot.anc + 2ull * tot.text + sizeof(MtPSet) * tot.pset +
                    (sizeof(MtDocHdr) + 4ull * MT_RFL + sizeof(MtDocLayout) + sizeof(MtOvx) * MT_OVX_CAP +
                     sizeof(MtReg) * MT_REG_CAP) * D + 4ull * tot.mid + 4ull * tot.regr;
    return MT_OK;
}

int MT_FN(create)(int device, const mt_limits* L, mt_ctx** out) {
    if (!L || !out || L->max_docs == 0) return MT_E_INVALID;
    return mt_create_impl(device, L->max_docs, L, true, out);
}
int MT_FN(create_docs)(int device, uint32_t n_docs, const mt_limits* per_doc, mt_ctx** out) {
    if (!per_doc || !out || n_docs == 0) return MT_E_INVALID;
    return mt_create_impl(device, n_docs, per_doc, false, out);
}
// Device-side checkpoint of every document's state (rows, blocks, heap, window,
// text, property sets, headers, recycled-row stacks): the engine's equivalent of
// a summary to resume from (SURVEY.md §5 checkpoint/resume), used by benchmarks
// that replay the same stream on the same starting state.
struct MtCkPart { void** ck; void* live; size_t bytes; };
static std::vector<MtCkPart> mt_ck_parts(mt_ctx* c) {
    const MtState& S = c->S; const MtDocLayout& t = c->tot; const size_t D = S.maxDocs;
    return {{&c->ck_rows, S.rows, sizeof(MtRow) * t.row}, {&c->ck_blk, S.blk, sizeof(MtBlk) * t.blk},
            {&c->ck_heap, S.heap, sizeof(MtHeapE) * t.heap}, {&c->ck_win, S.win, 4ull * t.win},
            {&c->ck_text, S.text, 2ull * t.text}, {&c->ck_pset, S.pset, sizeof(MtPSet) * t.pset},
            {&c->ck_hdr, S.hdr, sizeof(MtDocHdr) * D}, {&c->ck_hold, S.hold, 4ull * MT_RFL * D},
            {&c->ck_ovx, S.ovx, sizeof(MtOvx) * MT_OVX_CAP * D}, {&c->ck_mid, S.mid, 4ull * t.mid},
            {&c->ck_reg, S.reg, sizeof(MtReg) * MT_REG_CAP * D}, {&c->ck_regr, S.regr, 4ull * t.regr}};
}
int MT_FN(checkpoint)(mt_ctx* c) {
    if (!c) return MT_E_INVALID;
    int rc = mtb_sync(c);
    if (rc) return rc;
    for (auto& p : mt_ck_parts(c)) {
        if (!*p.ck && mtb_malloc(p.ck, p.bytes ? p.bytes : 16) != 0) { c->err = "checkpoint allocation failed"; return MT_E_OOM; }
        if (p.bytes) mtb_d2d(c, *p.ck, p.live, p.bytes);
    }
    c->ck_valid = true;
    return MT_OK;
}
int MT_FN(restore)(mt_ctx* c) {
    if (!c || !c->ck_valid) return MT_E_INVALID;
    int rc = mtb_sync(c);
    if (rc) return rc;
    for (auto& p : mt_ck_parts(c)) if (p.bytes) mtb_d2d(c, p.live, *p.ck, p.bytes);
    return MT_OK;
}
int MT_FN(pool_bytes)(mt_ctx* c, uint64_t* bytes) {
    if (!c || !bytes) return MT_E_INVALID;
    *bytes = c->pool_bytes;
    return MT_OK;
}

void MT_FN(destroy)(mt_ctx* c) {
    if (!c) return;
    MtState& S = c->S;
    void* ps[] = {S.rows, S.blk, S.heap, S.win, S.uid, S.udelta, S.uanc, S.text, S.pset, S.hdr, S.hold, (void*)S.layout,
                  S.ovx, S.mid, S.reg, c->ck_rows, c->ck_blk, c->ck_heap, c->ck_win, c->ck_text, c->ck_pset, c->ck_hdr,
                  c->ck_hold, c->ck_ovx, c->ck_mid, c->ck_reg, c->ck_regr, S.regr};
    for (void* p : ps) if (p) mtb_free(p);
    for (auto* b : c->dev_bufs()) if (b->p) mtb_free(b->p);
    mtb_fini(c);
    delete c;
}

int MT_FN(docs_open)(mt_ctx* c, uint32_t first, uint32_t n) {
    if (!c || (uint64_t)first + n > c->S.maxDocs) return MT_E_INVALID;
    if (n == 0) return MT_OK;
    for (uint32_t d = first; d < first + n && d < c->snap_chunk.size(); d++) c->snap_chunk[d] = 0;   // a new Client's options
    for (uint32_t d = first; d < first + n && d < c->doc_wide.size(); d++) { c->doc_wide[d] = 0; c->doc_keys[d].clear(); }
    return mtb_launch_open(c, first, n);
}
int MT_FN(set_doc_snapshot_chunk)(mt_ctx* c, uint32_t n, const uint32_t* docs, const uint64_t* chunk) {
    if (!c || (n && (!docs || !chunk))) return MT_E_INVALID;
    for (uint32_t i = 0; i < n; i++) if (docs[i] >= c->S.maxDocs) { c->err = "doc id out of range"; return MT_E_INVALID; }
    if (c->snap_chunk.size() < c->S.maxDocs) c->snap_chunk.resize(c->S.maxDocs, 0);
    for (uint32_t i = 0; i < n; i++) c->snap_chunk[docs[i]] = chunk[i];
    return MT_OK;
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
    if ((rc = mtb_ensure(c, c->b_pkind, 4ull * P->n_values + 8))) return rc;
    mtb_h2d(c, c->b_pset_off.p, P->set_off, 4ull * (P->n_sets + 1));
    if (npairs) { mtb_h2d(c, c->b_pkey.p, P->key, 2ull * npairs); mtb_h2d(c, c->b_pval.p, P->value, 4ull * npairs); }
    if (P->n_values) { mtb_h2d(c, c->b_pfalsy.p, P->value_falsy, P->n_values); mtb_h2d(c, c->b_pclass.p, P->value_class, 4ull * P->n_values); }
    // per value: what incr yields from it held, and the consensus seq -1 mark (MtState::p_vinfo);
    // element 0: incr of a fresh consensus object
    std::vector<int32_t> vinfo(P->n_values + 1);
    vinfo[0] = P->value_incr && P->incr_object >= 0 && (uint32_t)P->incr_object < P->n_values ? P->incr_object : MT_VINFO_NONE;
    for (uint32_t v = 0; P->value_kind && v < P->n_values; v++) {
        const uint8_t k = P->value_kind[v];
        const int32_t inc = P->value_incr ? P->value_incr[v] : MT_VAL_UNSUP;
        vinfo[v + 1] = (k & MT_VK_NUM) ? MT_VAL_NAN
                                       : (((inc >= 0 && (uint32_t)inc < P->n_values) ? inc : MT_VINFO_NONE) |
                                          ((k & MT_VK_SEQM1) ? MT_VINFO_SEQM1 : 0));
    }
    mtb_h2d(c, c->b_pkind.p, vinfo.data(), 4ull * vinfo.size());
    mtb_sync(c);
    c->S.p_off = (const uint32_t*)c->b_pset_off.p; c->S.p_key = (const uint16_t*)c->b_pkey.p;
    c->S.p_val = (const int32_t*)c->b_pval.p; c->S.p_falsy = (const uint8_t*)c->b_pfalsy.p;
    c->S.p_class = (const uint32_t*)c->b_pclass.p; c->S.p_nsets = P->n_sets;
    c->S.p_vinfo = (P->value_kind || !P->n_values) ? (const int32_t*)c->b_pkind.p + 1 : nullptr;
    c->h_set_off.assign(P->set_off, P->set_off + P->n_sets + 1);
    c->h_set_key.assign(P->key, P->key + npairs);
    {
        std::vector<uint16_t> ks(c->h_set_key);
        std::sort(ks.begin(), ks.end());
        const bool wide = (size_t)(std::unique(ks.begin(), ks.end()) - ks.begin()) > MT_WAVE;
        // Below MT_WAVE keys in all no document can outgrow the lanes, and batches are not
        // scanned (mt_scan_wide); when the table first passes them, the documents open now
        // have keys nobody counted: they replay in the FULL kernels until reopened.
        if (wide && !c->props_wide) {
            if (c->doc_wide.size() < c->S.maxDocs) { c->doc_wide.resize(c->S.maxDocs, 0); c->doc_keys.resize(c->S.maxDocs); }
            std::fill(c->doc_wide.begin(), c->doc_wide.end(), (uint8_t)1);
            for (auto& k : c->doc_keys) std::vector<uint16_t>().swap(k);
        }
        c->props_wide = wide;
    }
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

// Notes property set `ps` on document `doc` (mt_ctx::doc_keys); true once the document's keys
// pass a wave's lanes (its maps may then outgrow the non-FULL kernels).
static bool mt_note_set(mt_ctx* c, uint32_t doc, int ps) {
    if (ps < 0 || (size_t)ps + 1 >= c->h_set_off.size()) return false;
    if (c->doc_wide.size() < c->S.maxDocs) { c->doc_wide.resize(c->S.maxDocs, 0); c->doc_keys.resize(c->S.maxDocs); }
    if (c->doc_wide[doc]) return true;
    std::vector<uint16_t>& ks = c->doc_keys[doc];
    for (uint32_t q = c->h_set_off[ps]; q < c->h_set_off[ps + 1]; q++) {
        const uint16_t k = c->h_set_key[q];
        auto it = std::lower_bound(ks.begin(), ks.end(), k);
        if (it == ks.end() || *it != k) ks.insert(it, k);
    }
    if (ks.size() > MT_WAVE) { c->doc_wide[doc] = 1; std::vector<uint16_t>().swap(ks); return true; }
    return false;
}
// batch_wide for a batch of n_runs runs: run r's document doc(r) and its ops' property sets
// pid(i) over [op0(r), op1(r)) (sets named twice in a run are noted once).
extern "C++" {
template <class DocOf, class Op0, class Op1, class Pid>
static bool mt_scan_wide(mt_ctx* c, size_t n_runs, DocOf doc, Op0 op0, Op1 op1, Pid pid) {
    bool wide = false;
    if (!c->props_wide) return false;                 // no document can pass MT_WAVE keys
    std::vector<uint32_t> seen(c->h_set_off.size() - 1, 0);
    for (size_t r = 0; r < n_runs; r++) {
        const uint32_t d = doc(r);
        if (d < c->doc_wide.size() && c->doc_wide[d]) { wide = true; continue; }
        for (size_t i = op0(r); i < op1(r); i++) {
            const int ps = pid(i);
            if (ps < 0 || (size_t)ps >= seen.size() || seen[ps] == (uint32_t)r + 1) continue;
            seen[ps] = (uint32_t)r + 1;
            if (mt_note_set(c, d, ps)) { wide = true; break; }
        }
    }
    return wide;
}
}
// Device-built batches (the generators, the exchange: ops never seen on the host): wide when the
// property sets together could make a document wide.
static bool mt_dev_wide(const mt_ctx* c) { return c->props_wide; }

// The batch's arrays in one device region, one pinned staging copy and one asynchronous H2D
// (stream-ordered before the replay that follows; no host synchronization): doc ids, op
// offsets, the op records packed to mt_op_rec, the payload and the relative positions.  The
// caller's arrays are consumed before this returns.
static int mt_upload_ops(mt_ctx* c, const mt_op_batch* B) {
    const size_t N = B->n_ops, R = B->n_runs;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_doc = 0, o_off = al(o_doc + 4 * R), o_rec = al(o_off + 4 * (R + 1)),
                 o_pay = al(o_rec + sizeof(MtOpRec) * N), o_rel = al(o_pay + 2 * (size_t)B->payload_units),
                 total = al(o_rel + sizeof(MtRelPos) * (size_t)(B->rel ? B->n_rel : 0)) + 256;
    static_assert(sizeof(mt_rel_pos) == sizeof(MtRelPos), "relative position layout");
    int rc;
    if ((rc = mtb_ensure(c, c->b_batch, total))) return rc;
    uint8_t* h = (uint8_t*)mtb_stage_get(c, total);
    if (!h) { c->err = "pinned staging allocation failed"; return MT_E_OOM; }
    if (R) memcpy(h + o_doc, B->doc_ids, 4 * R);
    memcpy(h + o_off, B->op_offsets, 4 * (R + 1));
    MtOpRec* rec = (MtOpRec*)(h + o_rec);
    uint8_t regT[16] = {0};
    const size_t PU = (size_t)B->payload_units;
    mt_par_for(N, [&](size_t i0, size_t i1, unsigned t) {
        bool reg = false;
        for (size_t i = i0; i < i1; i++) {
            MtOpRec& o = rec[i];
            o.type = B->type[i]; o.flags = B->flags[i]; o.client = B->client[i]; o.seq = B->seq[i]; o.ref_seq = B->ref_seq[i];
            o.msn = B->msn[i]; o.pos1 = B->pos1[i]; o.pos2 = B->pos2[i]; o.payload_off = B->payload_off[i];
            o.payload_len = (uint16_t)B->payload_len[i]; o.prop_id = (int16_t)B->prop_id[i];
            reg |= B->type[i] >= MT_OP_CUT && B->type[i] <= MT_OP_PASTE;
        }
        // this thread's share of the payload (same split, in units)
        const size_t p0 = N ? PU * i0 / N : 0, p1 = N ? PU * i1 / N : PU;
        if (p1 > p0) memcpy(h + o_pay + 2 * p0, B->payload + p0, 2 * (p1 - p0));
        regT[t] = reg;
    });
    if (!N && PU) memcpy(h + o_pay, B->payload, 2 * PU);
    bool reg = false;
    for (int t = 0; t < 16; t++) reg |= regT[t] != 0;
    if (B->rel && B->n_rel) memcpy(h + o_rel, B->rel, sizeof(MtRelPos) * (size_t)B->n_rel);
    mtb_stage_send(c, c->b_batch.p, total);
    uint8_t* d = (uint8_t*)c->b_batch.p;
    MtOps& o = c->ops;
    o.doc_ids = (const uint32_t*)(d + o_doc); o.op_off = (const uint32_t*)(d + o_off); o.rec = (MtOpRec*)(d + o_rec);
    o.payload = (uint16_t*)(d + o_pay); o.n_runs = B->n_runs; o.payload_units = B->payload_units; o.pay_base = nullptr;
    o.rel = (const MtRelPos*)(d + o_rel); o.n_rel = B->rel ? B->n_rel : 0;
    c->n_runs = B->n_runs;
    c->run_off.assign(B->op_offsets, B->op_offsets + R + 1); c->batch_gen++;
    c->batch_reg = reg;
    c->batch_wide = mt_scan_wide(c, R, [&](size_t r) { return B->doc_ids[r]; }, [&](size_t r) { return B->op_offsets[r]; },
                                 [&](size_t r) { return B->op_offsets[r + 1]; }, [&](size_t i) { return B->prop_id[i]; });
    return MT_OK;
}

static int mt_check_batch(mt_ctx* c, const mt_op_batch* B) {
    if (!B || !B->op_offsets || (B->n_runs && !B->doc_ids)) { c->err = "null batch arrays"; return MT_E_INVALID; }
    if (B->op_offsets[B->n_runs] != B->n_ops) { c->err = "op_offsets[n_runs] != n_ops"; return MT_E_INVALID; }
    if (B->n_rel && !B->rel) { c->err = "n_rel without rel"; return MT_E_INVALID; }
    for (uint32_t r = 0; r < B->n_runs; r++) {
        if (B->doc_ids[r] >= c->S.maxDocs) { c->err = "doc id out of range"; return MT_E_INVALID; }
        if (B->op_offsets[r] > B->op_offsets[r + 1]) { c->err = "op_offsets not monotone"; return MT_E_INVALID; }
    }
    // per op: the first violation's message (threads check disjoint ranges; the lowest op wins)
    const char* errT[16] = {nullptr};
    size_t errI[16];
    const uint32_t nsets = c->S.p_nsets;
    mt_par_for(B->n_ops, [&](size_t i0, size_t i1, unsigned t) {
        for (size_t i = i0; i < i1; i++) {
            const char* e = nullptr;
            if (B->type[i] > MT_OP_PASTE) e = "unknown op type";
            else if (B->type[i] == MT_OP_INSERT && !(B->flags[i] & MT_OPF_MARKER) &&
                     (uint64_t)B->payload_off[i] + B->payload_len[i] > B->payload_units) e = "payload out of range";
            else if (B->prop_id[i] >= 0 && (uint32_t)B->prop_id[i] >= nsets) e = "prop_id out of range (mt_set_props first)";
            else if (B->prop_id[i] > 32767) e = "more than 32767 property sets";
            else if (B->payload_len[i] > 65535) e = "insert longer than 65535 UTF-16 units";
            else if (((B->flags[i] & MT_OPF_REL1) && (uint32_t)B->pos1[i] >= B->n_rel) ||
                     ((B->flags[i] & MT_OPF_REL2) && (uint32_t)B->pos2[i] >= B->n_rel)) e = "relative position index out of range";
            if (e) { errT[t] = e; errI[t] = i; return; }
        }
    });
    const char* e = nullptr; size_t ei = 0;
    for (int t = 0; t < 16; t++) if (errT[t] && (!e || errI[t] < ei)) { e = errT[t]; ei = errI[t]; }
    if (e) { c->err = e; return MT_E_INVALID; }
    return MT_OK;
}

int MT_FN(upload_batch)(mt_ctx* c, const mt_op_batch* B) {
    if (!c) return MT_E_INVALID;
    int rc = mt_check_batch(c, B);
    if (rc) return rc;
    return mt_upload_ops(c, B);                           // stream-ordered: no synchronization
}
// Parts concatenated into the staging layout of mt_upload_ops, re-based while packed (one pass
// over every op on the library's host threads; validation as mt_check_batch, on the re-based
// values).
static int mt_upload_parts(mt_ctx* c, uint32_t P, const mt_op_batch* parts, const int32_t* const* pmap,
                           const uint32_t* pmapLen) {
    std::vector<uint64_t> opB(P + 1, 0), payB(P + 1, 0), relB(P + 1, 0), runB(P + 1, 0);
    for (uint32_t p = 0; p < P; p++) {
        const mt_op_batch* B = &parts[p];
        if (!B->op_offsets || (B->n_runs && !B->doc_ids) || B->op_offsets[B->n_runs] != B->n_ops ||
            (B->n_rel && !B->rel) || (B->payload_units && !B->payload)) { c->err = "bad batch part"; return MT_E_INVALID; }
        for (uint32_t r = 0; r < B->n_runs; r++) {
            if (B->doc_ids[r] >= c->S.maxDocs) { c->err = "doc id out of range"; return MT_E_INVALID; }
            if (B->op_offsets[r] > B->op_offsets[r + 1]) { c->err = "op_offsets not monotone"; return MT_E_INVALID; }
        }
        opB[p + 1] = opB[p] + B->n_ops; payB[p + 1] = payB[p] + B->payload_units;
        relB[p + 1] = relB[p] + (B->rel ? B->n_rel : 0); runB[p + 1] = runB[p] + B->n_runs;
    }
    const size_t N = opB[P], R = runB[P], PU = payB[P], NR = relB[P];
    if (N >= (1ull << 32) || R >= (1ull << 32) || PU >= (1ull << 32)) { c->err = "batch parts exceed 32-bit indices"; return MT_E_INVALID; }
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_doc = 0, o_off = al(o_doc + 4 * R), o_rec = al(o_off + 4 * (R + 1)),
                 o_pay = al(o_rec + sizeof(MtOpRec) * N), o_rel = al(o_pay + 2 * PU),
                 total = al(o_rel + sizeof(MtRelPos) * NR) + 256;
    int rc;
    if ((rc = mtb_ensure(c, c->b_batch, total))) return rc;
    uint8_t* h = (uint8_t*)mtb_stage_get(c, total);
    if (!h) { c->err = "pinned staging allocation failed"; return MT_E_OOM; }
    uint32_t* docs = (uint32_t*)(h + o_doc);
    uint32_t* off = (uint32_t*)(h + o_off);
    std::vector<uint32_t> runOff(R + 1);
    off[0] = 0; runOff[0] = 0;
    for (uint32_t p = 0; p < P; p++) {
        const mt_op_batch* B = &parts[p];
        for (uint32_t r = 0; r < B->n_runs; r++) {
            docs[runB[p] + r] = B->doc_ids[r];
            off[runB[p] + r + 1] = runOff[runB[p] + r + 1] = (uint32_t)(opB[p] + B->op_offsets[r + 1]);
        }
        if (B->rel && B->n_rel) memcpy(h + o_rel + sizeof(MtRelPos) * relB[p], B->rel, sizeof(MtRelPos) * B->n_rel);
    }
    MtOpRec* rec = (MtOpRec*)(h + o_rec);
    const uint32_t nsets = c->S.p_nsets;
    const char* errT[16] = {nullptr};
    size_t errI[16];
    uint8_t regT[16] = {0};
    mt_par_for(N, [&](size_t i0, size_t i1, unsigned t) {
        bool reg = false;
        uint32_t p = (uint32_t)(std::upper_bound(opB.begin(), opB.end(), (uint64_t)i0) - opB.begin()) - 1;
        for (size_t i = i0; i < i1; i++) {
            while (i >= opB[p + 1]) p++;
            const mt_op_batch* B = &parts[p];
            const size_t j = i - opB[p];
            MtOpRec& o = rec[i];
            const uint8_t ty = B->type[j], fl = B->flags[j];
            int32_t pid = B->prop_id[j];
            const char* e = nullptr;
            if (pid >= 0 && pmap && pmap[p]) {
                if ((uint32_t)pid >= pmapLen[p]) e = "prop_id out of its part's map";
                else pid = pmap[p][pid];
            }
            const bool text = ty == MT_OP_INSERT && !(fl & MT_OPF_MARKER);
            if (ty > MT_OP_PASTE) e = "unknown op type";
            else if (text && (uint64_t)B->payload_off[j] + B->payload_len[j] > B->payload_units) e = "payload out of range";
            else if (pid >= 0 && (uint32_t)pid >= nsets) e = "prop_id out of range (mt_set_props first)";
            else if (pid > 32767) e = "more than 32767 property sets";
            else if (B->payload_len[j] > 65535) e = "insert longer than 65535 UTF-16 units";
            else if (((fl & MT_OPF_REL1) && (uint32_t)B->pos1[j] >= B->n_rel) ||
                     ((fl & MT_OPF_REL2) && (uint32_t)B->pos2[j] >= B->n_rel)) e = "relative position index out of range";
            if (e && !errT[t]) { errT[t] = e; errI[t] = i; }
            o.type = ty; o.flags = fl; o.client = B->client[j]; o.seq = B->seq[j]; o.ref_seq = B->ref_seq[j]; o.msn = B->msn[j];
            o.pos1 = B->pos1[j] + ((fl & MT_OPF_REL1) ? (int32_t)relB[p] : 0);
            o.pos2 = B->pos2[j] + ((fl & MT_OPF_REL2) ? (int32_t)relB[p] : 0);
            o.payload_off = B->payload_off[j] + (text ? (uint32_t)payB[p] : 0u);
            o.payload_len = (uint16_t)B->payload_len[j]; o.prop_id = (int16_t)pid;
            reg |= ty >= MT_OP_CUT && ty <= MT_OP_PASTE;
        }
        regT[t] = reg;
    });
    const char* e = nullptr; size_t ei = 0;
    for (int t = 0; t < 16; t++) if (errT[t] && (!e || errI[t] < ei)) { e = errT[t]; ei = errI[t]; }
    if (e) { c->err = e; return MT_E_INVALID; }
    mt_par_for(P, [&](size_t p0, size_t p1, unsigned) {           // payloads, part by part
        for (size_t p = p0; p < p1; p++)
            if (parts[p].payload_units) memcpy(h + o_pay + 2 * payB[p], parts[p].payload, 2 * parts[p].payload_units);
    });
    bool reg = false;
    for (int t = 0; t < 16; t++) reg |= regT[t] != 0;
    mtb_stage_send(c, c->b_batch.p, total);
    uint8_t* d = (uint8_t*)c->b_batch.p;
    MtOps& o = c->ops;
    o.doc_ids = (const uint32_t*)(d + o_doc); o.op_off = (const uint32_t*)(d + o_off); o.rec = (MtOpRec*)(d + o_rec);
    o.payload = (uint16_t*)(d + o_pay); o.n_runs = (uint32_t)R; o.payload_units = PU; o.pay_base = nullptr;
    o.rel = (const MtRelPos*)(d + o_rel); o.n_rel = (uint32_t)NR;
    c->n_runs = (uint32_t)R;
    c->run_off.swap(runOff); c->batch_gen++;
    c->batch_reg = reg;
    c->batch_wide = mt_scan_wide(c, R, [&](size_t r) { return docs[r]; }, [&](size_t r) { return (size_t)c->run_off[r]; },
                                 [&](size_t r) { return (size_t)c->run_off[r + 1]; }, [&](size_t i) { return (int)rec[i].prop_id; });
    return MT_OK;
}
int MT_FN(upload_batch_parts)(mt_ctx* c, uint32_t n_parts, const mt_op_batch* parts, const int32_t* const* prop_map,
                              const uint32_t* prop_map_len) {
    if (!c || (n_parts && !parts) || (prop_map && !prop_map_len)) return MT_E_INVALID;
    return mt_upload_parts(c, n_parts, parts, prop_map, prop_map_len);
}
int MT_FN(replay_resident)(mt_ctx* c);
int MT_FN(apply_batch_parts)(mt_ctx* c, uint32_t n_parts, const mt_op_batch* parts, const int32_t* const* prop_map,
                             const uint32_t* prop_map_len) {
    int rc = MT_FN(upload_batch_parts)(c, n_parts, parts, prop_map, prop_map_len);
    if (rc) return rc;
    return MT_FN(replay_resident)(c);
}
// A capture batch (mt_delta_capture armed): each launch appends records until a document
// has no headroom left for its next message (MtEngT::dReserve); that run stops there, the
// records and pasted text so far move to the host, and the next launch resumes the stopped
// runs (ops.start).  The host copies keep op order per document, so one stable sort by op
// index restores callback order (mt_delta_records).
static int mt_replay_capture(mt_ctx* c, const MtGen& g) {
    const uint32_t R = c->n_runs;
    int rc;
    if ((rc = mtb_ensure(c, c->b_resume, 4ull * R + 4))) return rc;
    if ((rc = mtb_ensure(c, c->b_start, 4ull * R + 4))) return rc;
    std::vector<uint32_t> off(R + 1), resume(R), start(R);
    if (c->run_off.size() == R + 1) off = c->run_off;
    else mtb_d2h(c, off.data(), c->ops.op_off, 4ull * (R + 1));
    for (uint32_t r = 0; r < R; r++) start[r] = off[r];
    c->delta_host.clear(); c->delta_text.clear(); c->delta_over = false; c->delta_launches = 0;
    MtOps& o = c->ops;
    o.drec = (MtDeltaRec*)c->b_drec.p; o.dcount = (unsigned long long*)c->b_dcount.p; o.dcap = c->delta_cap;
    o.dtext = (uint16_t*)c->b_dtext.p; o.dtcap = c->delta_tcap; o.resume = (uint32_t*)c->b_resume.p;
    o.start = nullptr;
    for (;;) {
        const unsigned long long zero[4] = {0, 0, 0, 0};
        mtb_h2d(c, c->b_dcount.p, zero, sizeof zero);
        if ((rc = mtb_launch_replay(c, g, R))) break;
        if ((rc = mtb_sync(c))) break;
        c->delta_launches++;
        unsigned long long cnt[4];
        mtb_d2h(c, cnt, c->b_dcount.p, sizeof cnt);
        if (cnt[MT_DC_REC] > c->delta_cap || cnt[MT_DC_TXT] > c->delta_tcap) { c->delta_over = true; break; }
        const size_t r0 = c->delta_host.size(), t0 = c->delta_text.size();
        c->delta_host.resize(r0 + cnt[MT_DC_REC]);
        if (cnt[MT_DC_REC]) mtb_d2h(c, c->delta_host.data() + r0, c->b_drec.p, sizeof(MtDeltaRec) * cnt[MT_DC_REC]);
        c->delta_text.resize(t0 + cnt[MT_DC_TXT]);
        if (cnt[MT_DC_TXT]) mtb_d2h(c, c->delta_text.data() + t0, c->b_dtext.p, 2ull * cnt[MT_DC_TXT]);
        for (size_t i = r0; i < c->delta_host.size(); i++) {      // pasted text offsets: into the batch's arena
            MtDeltaRec& q = c->delta_host[i];
            if (q.kind == MT_DK_INSERT && q.b == 0 && q.pad >= 0) q.pad += (int)t0;
        }
        mtb_d2h(c, resume.data(), c->b_resume.p, 4ull * R);
        bool done = true, progress = false;
        for (uint32_t r = 0; r < R; r++) {
            if (resume[r] < off[r + 1]) done = false;
            if (resume[r] != start[r]) progress = true;
        }
        if (done) break;
        if (!progress) { c->err = "delta capture capacity below one message's bound"; rc = MT_E_OOM; break; }
        start = resume;
        mtb_h2d(c, c->b_start.p, start.data(), 4ull * R);
        o.start = (const uint32_t*)c->b_start.p;
    }
    o.start = nullptr; o.resume = nullptr;
    c->delta_valid = false;
    return rc;
}
int MT_FN(replay_resident)(mt_ctx* c) {
    if (!c || !c->ops.op_off) return MT_E_INVALID;
    int rc = mtb_ensure(c, c->b_cursor, 4ull * c->n_runs + 4);
    if (rc) return rc;
    MtGen g{}; g.enabled = 0;
    c->delta_valid = false;
    if (c->delta_cap) return mt_replay_capture(c, g);
    c->ops.drec = nullptr; c->ops.dcount = nullptr; c->ops.dcap = 0; c->ops.dtext = nullptr; c->ops.dtcap = 0;
    c->ops.resume = nullptr; c->ops.start = nullptr;
    return mtb_launch_replay(c, g, c->n_runs);
}
int MT_FN(apply_batch)(mt_ctx* c, const mt_op_batch* B) {
    int rc = MT_FN(upload_batch)(c, B);
    if (rc) return rc;
    return MT_FN(replay_resident)(c);
}
// SnapshotLoader.loadBody's insertSegments calls as a device plan
// (MT/snapshotLoader.ts:162-206).  Universal NonCollab segments collect in a
// batch that every flush appends as one insertSegments call; the batch is never
// emptied, so a later flush re-appends already-linked segments: such a flush
// becomes one REFLUSH step (a no-op where the reference's walk falls off the
// tree, aliasing -> MT_DS_UNSUPPORTED where it would link a segment twice).
static bool mt_load_seg_ok(const mt_load_seg& g, int ms, int cs) {
    if ((g.flags & MT_LS_CLIENT) && g.client >= MT_NONCOLLAB) return false;
    if (g.flags & MT_LS_SEQ) {
        if (g.seq < 0 || g.seq > cs) return false;
        if (g.seq != 0 && g.seq <= ms) return false;     // neither universal nor in the collab window
    }
    if (g.flags & MT_LS_REMOVED) {
        if (g.removed_client >= MT_NONCOLLAB || g.removed_seq <= ms || g.removed_seq > cs) return false;
    }
    return true;
}
static void mt_load_plan(const mt_load_batch* B, uint32_t i, std::vector<MtLoadStep>& plan) {
    const uint32_t s0 = B->seg_offsets[i], s1 = B->seg_offsets[i + 1], nh = B->header_segments[i];
    const int ms = B->min_seq[i], cs = B->seq[i];
    bool ok = ms >= 0 && ms <= cs;
    for (uint32_t k = s0; k < s1 && ok; k++) ok = mt_load_seg_ok(B->segs[k], ms, cs);
    if (!ok) { plan.push_back({0, MT_LD_UNSUPPORTED, 0, 0}); return; }
    auto seglen = [&](uint32_t k) -> int {
        const mt_load_seg& g = B->segs[s0 + k];
        return (g.flags & MT_LS_MARKER) ? 1 : (int)g.payload_len;
    };
    std::vector<uint32_t> batch;
    size_t linked = 0;                                   // batch entries appended by earlier flushes
    auto flush = [&]() {
        if (batch.empty()) return;
        bool oldLinked = false;
        for (size_t j = 0; j < linked; j++) if (seglen(batch[j]) > 0) { oldLinked = true; break; }
        if (oldLinked) plan.push_back({0, batch.size() > linked ? MT_LD_REFLUSH_NEW : MT_LD_REFLUSH, MT_NONCOLLAB, 0});
        else
            for (size_t j = linked; j < batch.size(); j++)
                plan.push_back({(int)batch[j], j == linked ? MT_LD_START : MT_LD_CONT, MT_NONCOLLAB, 0});
        linked = batch.size();
    };
    for (uint32_t k = nh; k < s1 - s0; k++) {
        const mt_load_seg& g = B->segs[s0 + k];
        const int cli = (g.flags & MT_LS_CLIENT) ? (int)g.client : MT_NONCOLLAB;
        const int sq = (g.flags & MT_LS_SEQ) ? g.seq : 0;
        if (cli == MT_NONCOLLAB && sq == 0) batch.push_back(k);
        else { flush(); plan.push_back({(int)k, MT_LD_START, cli, sq}); }
    }
    flush();
}
int MT_FN(load_snapshot)(mt_ctx* c, const mt_load_batch* B) {
    if (!c || !B || !B->seg_offsets || (B->n_docs && (!B->doc_ids || !B->header_segments || !B->min_seq || !B->seq)))
        { if (c) c->err = "null load batch arrays"; return MT_E_INVALID; }
    const uint32_t n = B->n_docs;
    if (n == 0) return MT_OK;
    const uint32_t nseg = B->seg_offsets[n];
    std::vector<uint32_t> meta(5ull * n + 1);           // docs | seg_off (n+1) | nhdr | ms | cs
    std::vector<uint32_t> plan_off(n + 1, 0);
    std::vector<MtLoadStep> plan;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t s0 = B->seg_offsets[i], s1 = B->seg_offsets[i + 1];
        if (B->doc_ids[i] >= c->S.maxDocs) { c->err = "doc id out of range"; return MT_E_INVALID; }
        if (s1 < s0 || s1 > nseg || B->header_segments[i] > s1 - s0) { c->err = "bad seg_offsets/header_segments"; return MT_E_INVALID; }
        uint64_t expect = ~0ull;                          // text payloads contiguous per document
        for (uint32_t k = s0; k < s1; k++) {
            const mt_load_seg& g = B->segs[k];
            if (g.flags & MT_LS_MARKER) continue;
            if ((uint64_t)g.payload_off + g.payload_len > B->payload_units) { c->err = "payload out of range"; return MT_E_INVALID; }
            if (expect != ~0ull && g.payload_off != expect) { c->err = "document text payloads must be contiguous"; return MT_E_INVALID; }
            expect = (uint64_t)g.payload_off + g.payload_len;
        }
        for (uint32_t k = s0; k < s1; k++)
            if (B->segs[k].prop_id >= 0 && (uint32_t)B->segs[k].prop_id >= c->S.p_nsets) { c->err = "prop_id out of range (mt_set_props first)"; return MT_E_INVALID; }
        plan_off[i] = (uint32_t)plan.size();
        mt_load_plan(B, i, plan);
    }
    plan_off[n] = (uint32_t)plan.size();
    for (uint32_t i = 0; i < n; i++) {            // loaded maps count toward the documents' keys
        const uint32_t d = B->doc_ids[i];
        if (d < c->doc_wide.size()) { c->doc_wide[d] = 0; c->doc_keys[d].clear(); }
        for (uint32_t k = B->seg_offsets[i]; k < B->seg_offsets[i + 1]; k++)
            if (mt_note_set(c, d, B->segs[k].prop_id)) break;
    }
    for (uint32_t i = 0; i < n; i++) {
        meta[i] = B->doc_ids[i]; meta[n + i] = B->seg_offsets[i];
        meta[2ull * n + 1 + i] = B->header_segments[i];
        meta[3ull * n + 1 + i] = (uint32_t)B->min_seq[i]; meta[4ull * n + 1 + i] = (uint32_t)B->seq[i];
    }
    meta[2ull * n] = nseg;
    int rc;
#define UP(buf, src, bytes) if ((rc = mtb_ensure(c, c->buf, (bytes)))) return rc; if ((bytes) && (src)) mtb_h2d(c, c->buf.p, (src), (bytes));
    static_assert(sizeof(mt_load_seg) == sizeof(MtLoadSeg) && sizeof(MtLoadSeg) == 32, "load segment layout");
    UP(b_ld_meta, meta.data(), 4 * meta.size()) UP(b_ld_seg, B->segs, sizeof(MtLoadSeg) * nseg)
    UP(b_ld_pay, B->payload, 2 * B->payload_units) UP(b_ld_plan, plan.data(), sizeof(MtLoadStep) * plan.size())
    UP(b_ld_poff, plan_off.data(), 4ull * (n + 1))
#undef UP
    MtLoad L;
    const uint32_t* m = (const uint32_t*)c->b_ld_meta.p;
    L.docs = m; L.seg_off = m + n; L.nhdr = m + 2 * n + 1;
    L.ms = (const int32_t*)(m + 3 * n + 1); L.cs = (const int32_t*)(m + 4 * n + 1);
    L.segs = (const MtLoadSeg*)c->b_ld_seg.p; L.payload = (const uint16_t*)c->b_ld_pay.p;
    L.plan_off = (const uint32_t*)c->b_ld_poff.p; L.plan = (const MtLoadStep*)c->b_ld_plan.p;
    return mtb_launch_load(c, L, n);
}
int MT_FN(delta_capture)(mt_ctx* c, uint64_t capacity) {
    if (!c) return MT_E_INVALID;
    c->delta_cap = 0; c->delta_tcap = 0;
    if (capacity) {
        // one message of the largest document must fit a launch: its range (<= rowCap
        // records) plus the fixed slack; a paste's text is <= the document's text capacity
        uint64_t minr = MT_DREC_SLACK, mint = 1;
        for (const MtDocLayout& y : c->layout_h) {
            minr = std::max<uint64_t>(minr, (uint64_t)y.rowCap + MT_DREC_SLACK);
            mint = std::max<uint64_t>(mint, (uint64_t)y.textCap);
        }
        const uint64_t cap = std::max<uint64_t>(capacity, minr), tcap = std::max<uint64_t>(4 * capacity, mint);
        int rc;
        if ((rc = mtb_ensure(c, c->b_drec, sizeof(MtDeltaRec) * cap))) return rc;
        if ((rc = mtb_ensure(c, c->b_dcount, 32))) return rc;
        if ((rc = mtb_ensure(c, c->b_dtext, 2 * tcap))) return rc;
        c->delta_cap = cap; c->delta_tcap = tcap;
    }
    return MT_OK;
}
int MT_FN(delta_records)(mt_ctx* c, const mt_delta_rec** out, uint64_t* n) {
    static_assert(sizeof(mt_delta_rec) == sizeof(MtDeltaRec), "delta record layout");
    if (!c || !out || !n || !c->delta_cap) return MT_E_INVALID;
    int rc = mtb_sync(c);
    if (rc) return rc;
    if (!c->delta_valid) {
        // documents interleave in the buffer; one wave appends a document's records in
        // program order (and later launches of a run follow earlier ones), so a stable sort
        // by op index restores callback order
        std::stable_sort(c->delta_host.begin(), c->delta_host.end(),
                         [](const MtDeltaRec& x, const MtDeltaRec& y) { return x.op < y.op; });
        c->delta_valid = true;
    }
    *out = (const mt_delta_rec*)c->delta_host.data();
    *n = c->delta_host.size();
    if (c->delta_over) { c->err = "delta capture capacity exceeded"; return MT_E_OOM; }
    return MT_OK;
}
int MT_FN(delta_text)(mt_ctx* c, const uint16_t** out, uint64_t* n, uint32_t* launches) {
    if (!c || !out || !n || !c->delta_cap) return MT_E_INVALID;
    int rc = mtb_sync(c);
    if (rc) return rc;
    *out = c->delta_text.data();
    *n = c->delta_text.size();
    if (launches) *launches = c->delta_launches;
    return MT_OK;
}
int MT_FN(doc_pset)(mt_ctx* c, uint32_t doc, int32_t id, uint16_t* keys, int32_t* vals, uint32_t* n) {
    if (!c || doc >= c->S.maxDocs || !keys || !vals || !n || id < 0) return MT_E_INVALID;
    int rc = mtb_sync(c);
    if (rc) return rc;
    const MtDocLayout& y = c->layout_h[doc];
    if ((uint32_t)id >= y.psetCap) return MT_E_INVALID;
    MtPSet p[MT_PKEYS / MT_PSK];
    mtb_d2h(c, p, c->S.pset + y.pset + (size_t)id, sizeof(MtPSet));
    const uint32_t nk = p[0].n < 0 ? 0u : ((uint32_t)p[0].n > MT_PKEYS ? MT_PKEYS : (uint32_t)p[0].n);
    const uint32_t nch = nk > MT_PSK ? (nk + MT_PSK - 1) / MT_PSK : 1;
    if ((uint32_t)id + nch > y.psetCap) return MT_E_INVALID;
    if (nch > 1) mtb_d2h(c, p + 1, c->S.pset + y.pset + (size_t)id + 1, sizeof(MtPSet) * (nch - 1));
    *n = nk;
    for (uint32_t i = 0; i < nk; i++) { keys[i] = p[i >> 4].key[i & 15]; vals[i] = p[i >> 4].val[i & 15]; }
    return MT_OK;
}
int MT_FN(set_size_class)(mt_ctx* c, uint32_t big_min_ops) {
    if (!c) return MT_E_INVALID;
    c->big_min_ops = big_min_ops;
    c->part_cus = 0; c->part_auto = false;
    return MT_OK;
}
int MT_FN(set_continuation)(mt_ctx* c, uint32_t min_ops) {
    if (!c) return MT_E_INVALID;
    c->cont_min_ops = min_ops;
    return MT_OK;
}
int MT_FN(set_partition)(mt_ctx* c, uint32_t min_ops, uint32_t cus) {
    if (!c) return MT_E_INVALID;
    c->part_auto = min_ops == MT_PARTITION_AUTO;
    c->auto_gen = ~0ull;
    c->big_min_ops = c->part_auto ? 0 : min_ops;
    c->part_cus = (min_ops && !c->part_auto) ? cus : 0;
    return MT_OK;
}
int MT_FN(plan_partition)(const uint32_t* run_ops, uint32_t n, uint32_t n_cus, uint32_t* min_ops, uint32_t* cus,
                          double* est_ms) {
    if ((n && !run_ops) || !min_ops || !cus || n_cus == 0) return MT_E_INVALID;
    double us = 0;
    mt_plan_partition_impl(run_ops, n, n_cus, min_ops, cus, &us);
    if (est_ms) *est_ms = us / 1e3;
    return MT_OK;
}
int MT_FN(last_partition)(mt_ctx* c, uint32_t* min_ops, uint32_t* cus) {
    if (!c || !min_ops || !cus) return MT_E_INVALID;
    *min_ops = c->part_cus ? c->big_min_ops : 0; *cus = c->part_cus;
    return MT_OK;
}
int MT_FN(set_residency)(mt_ctx* c, int use_lds, int rows, int blocks, int heap) {
    const int maxHeap = use_lds == 3 ? MT_G_HEAP : (use_lds == 2 ? MT_B_HEAP : MT_L_HEAP);
    if (!c || use_lds < 0 || use_lds > 3 || rows < 0 || blocks < 0 || heap < 0 ||
        rows > (use_lds == 3 ? MT_G_WIN : MT_L_ROWS) ||
        blocks > (use_lds == 2 ? MT_B_BLKS : (use_lds == 3 ? 15 : MT_L_BLKS)) || heap > maxHeap)
        return MT_E_INVALID;
    c->use_lds = use_lds;
    c->lds_rows = rows ? rows : (use_lds == 3 ? MT_G_WIN : MT_L_ROWS);   // 3: window entries in LDS
    // 3: blocks = MT_BIGF_* switches (block cache, zamboni prefetch, corrections table, parent cache off; A/B)
    c->lds_blks = use_lds == 3 ? blocks : (blocks ? blocks : (use_lds == 2 ? MT_B_BLKS : MT_L_BLKS));
    c->lds_heap = heap ? heap : maxHeap;
    return MT_OK;
}
// Where each run of the last LDS-resident replay handed over to the HBM kernel
// (op index; op_offsets[run+1] = finished in LDS).  Diagnostic.
int MT_FN(last_cursors)(mt_ctx* c, uint32_t n, uint32_t* out) {
    if (!c || !out || n > c->n_runs || !c->b_cursor.p) return MT_E_INVALID;
    int rc = mtb_sync(c);
    if (rc) return rc;
    mtb_d2h(c, out, c->b_cursor.p, 4ull * n);
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
        int32_t* o = out + 10 * (size_t)i;
        o[0] = h[i].rowTop; o[1] = h[i].blkTop; o[2] = h[i].heapN; o[3] = h[i].winN;
        o[4] = h[i].textTop; o[5] = h[i].psetTop; o[6] = h[i].height; o[7] = h[i].rfN;
        o[8] = h[i].heapHW; o[9] = h[i].winHW;
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

// Position queries (mt_query.h): sorted by document (stable), one wave per document's group,
// answers back in query order; the found segments' text gathered on the device, their JSON
// written here from the text and the property-map chunks the kernel copied.
static int mt_run_queries(mt_ctx* c, uint32_t n, const uint32_t* docs, const int32_t* pos, const int32_t* ref,
                          const int32_t* cli, std::vector<MtQueryOut>& res) {
    res.assign(n, MtQueryOut{});
    if (n == 0) return MT_OK;
    for (uint32_t i = 0; i < n; i++) if (docs[i] >= c->S.maxDocs) { c->err = "query document out of range"; return MT_E_INVALID; }
    std::vector<uint32_t> ord(n);
    for (uint32_t i = 0; i < n; i++) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return docs[a] < docs[b]; });
    std::vector<MtQuery> q(n);
    std::vector<uint32_t> grp;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t i = ord[k];
        q[k].doc = docs[i]; q[k].pos = pos[i]; q[k].ref = ref ? ref[i] : -1; q[k].client = cli ? cli[i] : -1;
        if (k == 0 || docs[i] != docs[ord[k - 1]]) grp.push_back(k);
    }
    grp.push_back(n);
    const uint32_t ng = (uint32_t)grp.size() - 1;
    int rc;
    if ((rc = mtb_ensure(c, c->b_q, sizeof(MtQuery) * n))) return rc;
    if ((rc = mtb_ensure(c, c->b_qgrp, 4ull * (ng + 1)))) return rc;
    if ((rc = mtb_ensure(c, c->b_qout, sizeof(MtQueryOut) * n))) return rc;
    if ((rc = mtb_sync(c))) return rc;
    mtb_h2d(c, c->b_q.p, q.data(), sizeof(MtQuery) * n);
    mtb_h2d(c, c->b_qgrp.p, grp.data(), 4ull * (ng + 1));
    if ((rc = mtb_launch_query(c, (const MtQuery*)c->b_q.p, (const uint32_t*)c->b_qgrp.p, (MtQueryOut*)c->b_qout.p, ng))) return rc;
    if ((rc = mtb_sync(c))) return rc;
    std::vector<MtQueryOut> tmp(n);
    mtb_d2h(c, tmp.data(), c->b_qout.p, sizeof(MtQueryOut) * n);
    for (uint32_t k = 0; k < n; k++) res[ord[k]] = tmp[k];
    return MT_OK;
}

int MT_FN(get_containing_segment)(mt_ctx* c, uint32_t n, const uint32_t* docs, const int32_t* pos, const int32_t* ref,
                                  const int32_t* cli, mt_seg_info* out, const char** json_arena, const uint64_t** json_off) {
    if (!c || (n && (!docs || !pos))) return MT_E_INVALID;
    std::vector<MtQueryOut> res;
    int rc = mt_run_queries(c, n, docs, pos, ref, cli, res);
    if (rc) return rc;
    if (out) for (uint32_t i = 0; i < n; i++) out[i] = res[i].info;
    if (!json_arena) return MT_OK;
    // text of the found text segments, gathered on the device into one arena
    std::vector<unsigned long long> at, off(1, 0);
    std::vector<uint32_t> len, which;
    for (uint32_t i = 0; i < n; i++) {
        const mt_seg_info& f = res[i].info;
        if (!f.found || f.marker_ref_type >= 0 || f.len <= 0) continue;
        at.push_back(res[i].text_at); len.push_back((uint32_t)f.len); which.push_back(i);
        off.push_back(off.back() + (unsigned long long)f.len);
    }
    std::vector<uint16_t> txt(off.back());
    const uint32_t m = (uint32_t)len.size();
    if (m) {
        if ((rc = mtb_ensure(c, c->b_qat, 8ull * m))) return rc;
        if ((rc = mtb_ensure(c, c->b_qlen, 4ull * m))) return rc;
        if ((rc = mtb_ensure(c, c->b_qoff, 8ull * m))) return rc;
        if ((rc = mtb_ensure(c, c->b_qtext, 2ull * off.back()))) return rc;
        mtb_h2d(c, c->b_qat.p, at.data(), 8ull * m);
        mtb_h2d(c, c->b_qlen.p, len.data(), 4ull * m);
        mtb_h2d(c, c->b_qoff.p, off.data(), 8ull * m);
        if ((rc = mtb_launch_gather_text(c, (const unsigned long long*)c->b_qat.p, (const uint32_t*)c->b_qlen.p,
                                         (const unsigned long long*)c->b_qoff.p, (uint16_t*)c->b_qtext.p, m))) return rc;
        if ((rc = mtb_sync(c))) return rc;
        mtb_d2h(c, txt.data(), c->b_qtext.p, 2ull * off.back());
    }
    std::vector<int64_t> slot(n, -1);
    for (uint32_t k = 0; k < m; k++) slot[which[k]] = k;
    c->seg_json_arena.clear(); c->seg_json_off.assign(1, 0);
    for (uint32_t i = 0; i < n; i++) {
        const mt_seg_info& f = res[i].info;
        if (f.found) {
            const bool marker = f.marker_ref_type >= 0;
            const int64_t k = slot[i];
            std::string pj;
            if (f.prop_set >= 0) mtsnap::props_json(pj, res[i].ps, c->names);
            mtsnap::seg_json_of(c->seg_json_arena, marker, f.marker_ref_type, f.prop_set >= 0 ? &pj : nullptr,
                                k >= 0 ? txt.data() + off[k] : nullptr, k >= 0 ? (size_t)len[k] : 0);
        }
        c->seg_json_off.push_back(c->seg_json_arena.size());
    }
    *json_arena = c->seg_json_arena.data();
    if (json_off) *json_off = c->seg_json_off.data();
    return MT_OK;
}

int MT_FN(resolve_remote_position)(mt_ctx* c, uint32_t n, const uint32_t* docs, const int32_t* pos, const int32_t* ref,
                                   const int32_t* cli, int32_t* out) {
    if (!c || (n && (!docs || !pos || !out))) return MT_E_INVALID;
    std::vector<MtQueryOut> res;
    int rc = mt_run_queries(c, n, docs, pos, ref, cli, res);
    if (rc) return rc;
    for (uint32_t i = 0; i < n; i++) out[i] = res[i].info.resolved;
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
    const MtDocLayout& y = c->layout_h[d];
    mtb_d2h(c, &h.hdr, S.hdr + d, sizeof(MtDocHdr));
    const size_t R = (size_t)h.hdr.rowTop;
    h.rows.resize(R + 1);
    if (R) mtb_d2h(c, h.rows.data(), S.rows + y.row, sizeof(MtRow) * R);
    h.blk.resize((size_t)h.hdr.blkTop + 1);
    mtb_d2h(c, h.blk.data(), S.blk + y.blk, sizeof(MtBlk) * (size_t)h.hdr.blkTop);
    h.text.resize((size_t)h.hdr.textTop + 1);
    if (h.hdr.textTop) mtb_d2h(c, h.text.data(), S.text + y.text + (size_t)h.hdr.textHalf * y.textCap, 2 * (size_t)h.hdr.textTop);
    h.pset.resize((size_t)h.hdr.psetTop + 1);
    if (h.hdr.psetTop) mtb_d2h(c, h.pset.data(), S.pset + y.pset, sizeof(MtPSet) * (size_t)h.hdr.psetTop);
    return MT_OK;
}

// Gather documents' live state into host memory with two kernels and one copy
// (mt_pack.h); views[i] points into `host`.
static int mt_stage_docs(mt_ctx* c, uint32_t n, const uint32_t* docs, std::vector<MtSnapView>& views, int buf = 0) {
    views.clear();
    if (n == 0) return MT_OK;
    for (uint32_t i = 0; i < n; i++) if (docs[i] >= c->S.maxDocs) { c->err = "doc id out of range"; return MT_E_INVALID; }
    int rc;
    if ((rc = mtb_ensure(c, c->b_pack_docs, 4ull * n))) return rc;
    if ((rc = mtb_ensure(c, c->b_pack_sz, sizeof(MtPackSize) * n))) return rc;
    if ((rc = mtb_ensure(c, c->b_pack_off, 8ull * n))) return rc;
    mtb_h2d(c, c->b_pack_docs.p, docs, 4ull * n);
    const uint32_t epoch = ++c->stage_epoch;
    if ((rc = mtb_launch_pack_size(c, (const uint32_t*)c->b_pack_docs.p, (MtPackSize*)c->b_pack_sz.p, n, epoch))) return rc;
    std::vector<MtPackSize> sz(n);
    mtb_d2h(c, sz.data(), c->b_pack_sz.p, sizeof(MtPackSize) * n);
    std::vector<uint64_t> off(n + 1, 0);
    for (uint32_t i = 0; i < n; i++) off[i + 1] = off[i] + mt_pack_bytes(sz[i]);
    if ((rc = mtb_ensure(c, c->b_stage, off[n] + 16))) return rc;
    mtb_h2d(c, c->b_pack_off.p, off.data(), 8ull * n);
    if ((rc = mtb_launch_pack(c, (const uint32_t*)c->b_pack_docs.p, (const uint64_t*)c->b_pack_off.p, (uint8_t*)c->b_stage.p, n,
                              epoch))) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    if ((rc = mtb_sync(c))) return rc;
    const auto t1 = std::chrono::steady_clock::now();
    uint8_t* host = mtb_host_stage(c, off[n] + 16, buf);
    if (!host) { c->err = "pinned staging allocation failed"; return MT_E_OOM; }
    mtb_d2h(c, host, c->b_stage.p, off[n]);
    if (getenv("MT_SNAP_TIMING"))
        fprintf(stderr, "mt_stage_docs: %u docs, %.1f MB staged, pack kernel wait %.1f ms, host buffer + download %.1f ms\n", n,
                off[n] / 1e6, std::chrono::duration<double, std::milli>(t1 - t0).count(),
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
    views.resize(n);
    for (uint32_t i = 0; i < n; i++) {
        const MtStagedDoc sd = MtStagedDoc::at(host + off[i]);
        MtSnapView& v = views[i];
        v.hdr = sd.hdr; v.R = sd.R; v.blk = sd.blk; v.text = sd.text; v.pset = sd.pset;
    }
    return MT_OK;
}

// Client.snapshot asserts on the window it moves to (updateSeqNumbers, client.ts:843-850 ->
// setMinSeq, mergeTree.ts:1712-1716): a document whose status word is set after that
// (or before it) has no snapshot; the call fails instead of serializing it.
static int mt_check_staged_status(mt_ctx* c, uint32_t n, const uint32_t* docs, const std::vector<MtSnapView>& v) {
    for (uint32_t i = 0; i < n; i++)
        if (v[i].hdr.status) {
            char b[96];
            snprintf(b, sizeof b, "document %u has status 0x%x (the reference would have thrown)", docs[i], v[i].hdr.status);
            c->err = b;
            return MT_E_DOC_STATUS;
        }
    return MT_OK;
}
// Documents staged in groups of at most MT_STAGE_BUDGET bytes (estimated from their headers:
// every row, block, text unit and property set, an upper bound of the packed size), so the
// pinned download buffers stay small (pinning a multi-GB buffer costs more than the copy) and
// are reused group after group; fn(first, count, views) consumes each group while the next is
// staged; a group holds a multiple of `mult` documents (whole rounds of the emitting threads).
#define MT_STAGE_BUDGET (384ull << 20)
typedef std::function<int(uint32_t, uint32_t, const std::vector<MtSnapView>&)> MtGroupFn;
static int mt_staged_groups(mt_ctx* c, uint32_t n, const uint32_t* docs, const MtGroupFn& fn, uint32_t mult = 1,
                            bool check_status = true) {
    std::vector<MtDocHdr> h;
    int rc = mt_read_hdrs(c, n, docs, h);
    if (rc) return rc;
    const char* bs = getenv("MT_STAGE_BUDGET");             // bytes per group (tests force small groups)
    const uint64_t budget = bs ? strtoull(bs, nullptr, 10) : MT_STAGE_BUDGET;
    auto groupEnd = [&](uint32_t a) {
        uint64_t bytes = 0; uint32_t m = 0;
        while (a + m < n && m < 32768) {
            const MtDocHdr& d = h[a + m];
            const uint64_t b = 48ull * (uint64_t)(d.rowTop > 0 ? d.rowTop : 0) + 64ull * (uint64_t)(d.blkTop > 0 ? d.blkTop : 0) +
                               2ull * (uint64_t)(d.textTop > 0 ? d.textTop : 0) +
                               (uint64_t)sizeof(MtPSet) * (uint64_t)(d.psetTop > 0 ? d.psetTop : 0) + 1024;
            if (m > 0 && bytes + b > budget) break;
            bytes += b; m++;
        }
        if (a + m < n && m > mult) m -= m % mult;             // whole rounds of the emitting threads
        return a + m;
    };
    const bool timing = getenv("MT_SNAP_TIMING") != nullptr;
    // double-buffered: group g+1 is staged (device pack + download into the other pinned
    // buffer) while group g is emitted on the host threads
    std::vector<MtSnapView> cur, nxt;
    {   // both pinned buffers sized once for the call's largest group (estimates bound the packed
        // bytes): no buffer is re-pinned between groups
        uint64_t big = 0;
        for (uint32_t g = 0; g < n;) {
            const uint32_t e = groupEnd(g);
            uint64_t bytes = 0;
            for (uint32_t i = g; i < e; i++) {
                const MtDocHdr& d = h[i];
                bytes += 48ull * (uint64_t)(d.rowTop > 0 ? d.rowTop : 0) + 64ull * (uint64_t)(d.blkTop > 0 ? d.blkTop : 0) +
                         2ull * (uint64_t)(d.textTop > 0 ? d.textTop : 0) +
                         (uint64_t)sizeof(MtPSet) * (uint64_t)(d.psetTop > 0 ? d.psetTop : 0) + 1024;
            }
            if (bytes > big) big = bytes;
            g = e;
        }
        for (int buf = 0; buf < 2 && n; buf++)
            if (!mtb_host_stage(c, big + 16, buf)) { c->err = "pinned staging allocation failed"; return MT_E_OOM; }
    }
    uint32_t a = 0, b = n ? groupEnd(0) : 0;
    if (n && ((rc = mt_stage_docs(c, b - a, docs + a, cur, 0)) ||
              (check_status && (rc = mt_check_staged_status(c, b - a, docs + a, cur)))))
        return rc;
    for (int buf = 0; a < n; buf ^= 1) {
        const auto t0 = std::chrono::steady_clock::now();
        int erc = MT_OK;
        std::thread emit([&] { erc = fn(a, b - a, cur); });
        const uint32_t b2 = b < n ? groupEnd(b) : b;
        int src = MT_OK;
        if (b < n && !(src = mt_stage_docs(c, b2 - b, docs + b, nxt, buf ^ 1)) && check_status)
            src = mt_check_staged_status(c, b2 - b, docs + b, nxt);
        const auto t1 = std::chrono::steady_clock::now();
        emit.join();
        if (timing)
            fprintf(stderr, "mt_staged_groups: docs %u..%u emitted in %.1f ms beside staging the next %u in %.1f ms\n", a, b,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), b2 - b,
                    std::chrono::duration<double, std::milli>(t1 - t0).count());
        if (erc) return erc;
        if (src) return src;
        std::swap(cur, nxt);
        a = b; b = b2;
    }
    return MT_OK;
}
int MT_FN(reserve_staging)(mt_ctx* c, uint64_t bytes) {
    if (!c) return MT_E_INVALID;
    if (!bytes) bytes = MT_STAGE_BUDGET + 16;
    for (int buf = 0; buf < 2; buf++)
        if (!mtb_host_stage(c, bytes, buf)) { c->err = "pinned staging allocation failed"; return MT_E_OOM; }
    return MT_OK;
}
// SnapshotV1 of a non-empty document whose chunk size no length is below (MT_CHUNK_NONE):
// the reference's chunk loop (snapshotV1.ts:98-114) never ends; reported instead.
static std::string mt_chunk_hang_msg(uint32_t doc) {
    return "document " + std::to_string(doc) + ": mergeTreeSnapshotChunkSize is not a positive number, and "
           "SnapshotV1's chunk loop (snapshotV1.ts:98-114) never ends on a non-empty document";
}
// Client.snapshot (client.ts:923-956): SnapshotV1 or, with legacy set, SnapshotLegacy.
static int mt_snapshot_blobs(mt_ctx* c, uint32_t n, const uint32_t* docs, const int32_t* msn, const int32_t* seq,
                             uint64_t* digest, const char** arena, const uint64_t** blob_off,
                             const uint32_t** blob_first, bool legacy) {
    if (!c) return MT_E_INVALID;
    int rc = MT_FN(update_seq)(c, n, docs, msn, seq);       // Client.snapshot: updateSeqNumbers first (client.ts:936)
    if (rc) return rc;
    c->snap_arena.clear(); c->blob_off.assign(1, 0); c->blob_first.assign(1, 0);
    rc = mt_staged_groups(c, n, docs, [&](uint32_t a, uint32_t m, const std::vector<MtSnapView>& views) {
        for (uint32_t j = 0; j < m; j++) {
            const uint32_t i = a + j;
            auto dn = c->doc_clients.find(docs[i]);
            std::vector<std::string> blobs = legacy ? mtsnap::snapshot_legacy_blobs(views[j], c->names, c->chunk_of(docs[i]))
                                                    : mtsnap::snapshot_blobs(views[j], c->names,
                                                                             dn == c->doc_clients.end() ? nullptr : &dn->second,
                                                                             c->chunk_of(docs[i]));
            if (blobs.empty()) { c->err = mt_chunk_hang_msg(docs[i]); return (int)MT_E_INVALID; }
            if (digest) digest[i] = mtsnap::blobs_digest(blobs);
            for (auto& b : blobs) { c->snap_arena += b; c->blob_off.push_back(c->snap_arena.size()); }
            c->blob_first.push_back((uint32_t)(c->blob_off.size() - 1));
        }
        return (int)MT_OK;
    });
    if (rc) return rc;
    if (arena) *arena = c->snap_arena.data();
    if (blob_off) *blob_off = c->blob_off.data();
    if (blob_first) *blob_first = c->blob_first.data();
    return MT_OK;
}

int MT_FN(snapshot_v1)(mt_ctx* c, uint32_t n, const uint32_t* docs, const int32_t* msn, const int32_t* seq,
                       uint64_t* digest, const char** arena, const uint64_t** blob_off, const uint32_t** blob_first) {
    return mt_snapshot_blobs(c, n, docs, msn, seq, digest, arena, blob_off, blob_first, false);
}

int MT_FN(snapshot_legacy)(mt_ctx* c, uint32_t n, const uint32_t* docs, const int32_t* msn, const int32_t* seq,
                           uint64_t* digest, const char** arena, const uint64_t** blob_off, const uint32_t** blob_first) {
    return mt_snapshot_blobs(c, n, docs, msn, seq, digest, arena, blob_off, blob_first, true);
}

// Digests only, serialized on `threads` host threads (no blob arena).
int MT_FN(snapshot_digests)(mt_ctx* c, uint32_t n, const uint32_t* docs, const int32_t* msn, const int32_t* seq,
                            uint64_t* digest, int threads) {
    if (!c || (n && (!docs || !msn || !seq || !digest))) return MT_E_INVALID;
    int rc = MT_FN(update_seq)(c, n, docs, msn, seq);
    if (rc) return rc;
    if (threads < 1) threads = 1;
    // groups of documents (mt_staged_groups), so the staging buffers stay bounded however many
    // documents (a million Zipf documents stage ~20 GB)
    return mt_staged_groups(c, n, docs, [&](uint32_t a, uint32_t m, const std::vector<MtSnapView>& views) {
        const int th = (uint32_t)threads > m ? (int)m : threads;
        std::vector<uint32_t> hang(th, UINT32_MAX);
        auto work = [&](int t) {
            for (uint32_t i = (uint32_t)t; i < m; i += (uint32_t)th) {
                auto dn = c->doc_clients.find(docs[a + i]);
                std::vector<std::string> blobs = mtsnap::snapshot_blobs(views[i], c->names,
                                                                        dn == c->doc_clients.end() ? nullptr : &dn->second,
                                                                        c->chunk_of(docs[a + i]));
                if (blobs.empty()) { hang[t] = std::min(hang[t], a + i); continue; }
                digest[a + i] = mtsnap::blobs_digest(blobs);
            }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < th; t++) pool.emplace_back(work, t);
        work(0);
        for (auto& t : pool) t.join();
        const uint32_t h = *std::min_element(hang.begin(), hang.end());
        if (h != UINT32_MAX) { c->err = mt_chunk_hang_msg(docs[h]); return (int)MT_E_INVALID; }
        return (int)MT_OK;
    }, (uint32_t)threads);
}

int MT_FN(get_text)(mt_ctx* c, uint32_t n, const uint32_t* docs, const uint16_t** arena, const uint64_t** off) {
    if (!c) return MT_E_INVALID;
    int rc = mtb_sync(c);
    if (rc) return rc;
    for (uint32_t i = 0; i < n; i++) if (docs[i] >= c->S.maxDocs) { c->err = "doc id out of range"; return MT_E_INVALID; }
    c->text_arena.clear(); c->text_off.assign(1, 0);
    // bounded groups through the two reused pinned buffers (mt_staged_groups), documents in order;
    // a document with a status word still has its text (no status check)
    rc = mt_staged_groups(c, n, docs, [&](uint32_t, uint32_t m, const std::vector<MtSnapView>& views) {
        for (uint32_t j = 0; j < m; j++) {
            mtsnap::observer_text(views[j], c->text_arena);
            c->text_off.push_back(c->text_arena.size());
        }
        return (int)MT_OK;
    }, 1, false);
    if (rc) return rc;
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

// Stream generation with per-document op counts and client counts (null arrays:
// P->ops_per_doc / P->clients for every document).
int MT_FN(generate_docs)(mt_ctx* c, const mt_gen_params* P, const uint32_t* ops_per_doc, const uint32_t* clients_per_doc) {
    if (!c || !P || P->n_docs == 0 || P->n_docs > c->S.maxDocs || P->ins_len_max == 0 || P->rem_len_max == 0 ||
        P->n_ann_sets == 0) return MT_E_INVALID;
    if (P->pct_insert + P->pct_remove < 100 && P->n_ann_sets > c->S.p_nsets) { c->err = "annotate prop sets not uploaded"; return MT_E_INVALID; }
    if (P->ins_len_min > P->ins_len_max) { c->err = "ins_len_min > ins_len_max"; return MT_E_INVALID; }
    if (P->seg_prop_sets > c->S.p_nsets) { c->err = "segment prop sets not uploaded"; return MT_E_INVALID; }
    std::vector<uint32_t> docs(P->n_docs), off(P->n_docs + 1), cl(P->n_docs);
    off[0] = 0;
    for (uint32_t i = 0; i < P->n_docs; i++) {
        docs[i] = i;
        const uint64_t n = ops_per_doc ? ops_per_doc[i] : P->ops_per_doc;
        cl[i] = clients_per_doc ? clients_per_doc[i] : P->clients;
        if (cl[i] == 0 || cl[i] > 64) { c->err = "clients per document must be in [1, 64]"; return MT_E_INVALID; }
        if ((uint64_t)off[i] + n > 0xFFFFFFFFull) { c->err = "more than 2^32 ops in one batch"; return MT_E_INVALID; }
        off[i + 1] = (uint32_t)(off[i] + n);
    }
    const size_t N = off[P->n_docs];
    if ((uint64_t)N * P->ins_len_max >= 0xFFFFFFFFull) { c->err = "payload arena exceeds 2^32 units"; return MT_E_INVALID; }
    const size_t PU = N * P->ins_len_max + 1;
    int rc;
#define AL(buf, bytes) if ((rc = mtb_ensure(c, c->buf, (bytes)))) return rc;
    AL(b_doc, 4ull * P->n_docs) AL(b_off, 4ull * (P->n_docs + 1)) AL(b_rec, sizeof(MtOpRec) * (N + 1)) AL(b_pay, 2 * PU)
    AL(b_gencl, 4ull * P->n_docs)
#undef AL
    mtb_h2d(c, c->b_doc.p, docs.data(), 4ull * P->n_docs);
    mtb_h2d(c, c->b_off.p, off.data(), 4ull * (P->n_docs + 1));
    mtb_h2d(c, c->b_gencl.p, cl.data(), 4ull * P->n_docs);
    MtOps& o = c->ops;
    o.doc_ids = (const uint32_t*)c->b_doc.p; o.op_off = (const uint32_t*)c->b_off.p; o.rec = (MtOpRec*)c->b_rec.p;
    o.payload = (uint16_t*)c->b_pay.p; o.n_runs = P->n_docs; o.payload_units = PU; o.pay_base = nullptr;
    o.rel = nullptr; o.n_rel = 0; o.drec = nullptr; o.dcount = nullptr; o.dcap = 0;
    o.dtext = nullptr; o.dtcap = 0; o.resume = nullptr; o.start = nullptr;
    c->n_runs = P->n_docs;
    c->batch_reg = false;                     // generated streams hold no register ops
    c->batch_wide = mt_dev_wide(c);
    c->gen_off.assign(off.begin(), off.end());
    c->run_off = c->gen_off; c->batch_gen++;
    if (!P->continue_docs) {
        rc = MT_FN(docs_open)(c, 0, P->n_docs);
        if (rc) return rc;
    }
    MtGen g{};
    g.seed = P->seed; g.ops = P->ops_per_doc; g.clients = P->clients; g.lag_max = P->lag_max;
    g.pct_insert = P->pct_insert; g.pct_remove = P->pct_remove; g.ins_len_max = P->ins_len_max;
    g.rem_len_max = P->rem_len_max; g.n_ann_sets = P->n_ann_sets; g.pct_rewrite = P->pct_rewrite; g.enabled = 1;
    g.clients_per_run = (const uint32_t*)c->b_gencl.p; g.total_ops = N; g.doc_id_base = P->doc_id_base;
    g.ins_len_min = P->ins_len_min; g.seg_prop_sets = P->seg_prop_sets; g.ins_at_end = P->ins_at_end;
    c->gen = g; c->gen_docs = P->n_docs;
    return mtb_launch_replay(c, g, P->n_docs);
}
int MT_FN(generate)(mt_ctx* c, const mt_gen_params* P) {
    if (!P || P->clients == 0 || P->clients > 64) return MT_E_INVALID;
    return MT_FN(generate_docs)(c, P, nullptr, nullptr);
}
int MT_FN(generated_ops)(mt_ctx* c, uint64_t* n_ops) {
    if (!c || !n_ops || !c->gen_docs) return MT_E_INVALID;
    *n_ops = c->gen.total_ops;
    return MT_OK;
}

int MT_FN(generated_download)(mt_ctx* c, uint8_t* type, uint8_t* flags, uint16_t* client, int32_t* seq, int32_t* ref,
                              int32_t* msn, int32_t* pos1, int32_t* pos2, uint32_t* poff, uint32_t* plen, int32_t* pid,
                              uint16_t* payload) {
    if (!c || !c->gen_docs) return MT_E_INVALID;
    mtb_sync(c);
    const size_t N = c->gen.total_ops;
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
static_assert(sizeof(mt_op_rec) == sizeof(MtOpRec) && sizeof(mt_op_rec) == 32, "op record layout");
int MT_FN(generated_copy_dev)(mt_ctx* c, uint32_t first, uint32_t n, mt_op_rec* rec, uint16_t* payload) {
    if (!c || !c->gen_docs || (uint64_t)first + n > c->gen_off.size() - 1 || (n && (!rec || !payload))) return MT_E_INVALID;
    int rc = mtb_sync(c);
    if (rc) return rc;
    const uint64_t o0 = c->gen_off[first], o1 = c->gen_off[first + n];
    const uint64_t L = c->gen.ins_len_max;
    mtb_d2d(c, rec, c->ops.rec + o0, sizeof(MtOpRec) * (o1 - o0));
    mtb_d2d(c, payload, c->ops.payload + o0 * L, 2 * (o1 - o0) * L);
    return MT_OK;
}
int MT_FN(upload_batch_dev)(mt_ctx* c, uint32_t n_runs, const uint32_t* doc_ids, const uint32_t* op_offsets,
                            const mt_op_rec* rec, const uint16_t* payload, uint64_t payload_units) {
    if (!c || !op_offsets || (n_runs && !doc_ids)) return MT_E_INVALID;
    for (uint32_t r = 0; r < n_runs; r++) {
        if (doc_ids[r] >= c->S.maxDocs) { c->err = "doc id out of range"; return MT_E_INVALID; }
        if (op_offsets[r] > op_offsets[r + 1]) { c->err = "op_offsets not monotone"; return MT_E_INVALID; }
    }
    const uint64_t N = op_offsets[n_runs];
    if (N && (!rec || !payload)) return MT_E_INVALID;
    int rc;
#define UP(buf, bytes) if ((rc = mtb_ensure(c, c->buf, (bytes)))) return rc;
    UP(b_doc, 4ull * n_runs + 4) UP(b_off, 4ull * (n_runs + 1)) UP(b_rec, sizeof(MtOpRec) * N + 32) UP(b_pay, 2 * payload_units + 2)
#undef UP
    mtb_h2d(c, c->b_doc.p, doc_ids, 4ull * n_runs);
    mtb_h2d(c, c->b_off.p, op_offsets, 4ull * (n_runs + 1));
    if (N) mtb_d2d(c, c->b_rec.p, rec, sizeof(MtOpRec) * N);
    if (payload_units) mtb_d2d(c, c->b_pay.p, payload, 2 * payload_units);
    MtOps& o = c->ops;
    o.doc_ids = (const uint32_t*)c->b_doc.p; o.op_off = (const uint32_t*)c->b_off.p; o.rec = (MtOpRec*)c->b_rec.p;
    o.payload = (uint16_t*)c->b_pay.p; o.n_runs = n_runs; o.payload_units = payload_units; o.pay_base = nullptr;
    o.rel = nullptr; o.n_rel = 0;
    c->n_runs = n_runs;
    c->run_off.assign(op_offsets, op_offsets + n_runs + 1); c->batch_gen++;
    c->batch_reg = false;                     // device-built streams (shard.py) hold no register ops
    c->batch_wide = mt_dev_wide(c);
    c->gen.enabled = 0;
    return mtb_sync(c);
}
// Document exchange rows (mt_shard.h): the sender packs generated runs at their plan
// positions with per-document checksums; the receiver unpacks rows into its resident batch
// and checks every document's checksum against the sender's.
int MT_FN(generated_pack_rows)(mt_ctx* c, uint32_t first, uint32_t n, const uint64_t* dst_row, void* rows_dev,
                               uint64_t* checksum) {
    if (!c || !c->gen_docs || (uint64_t)first + n > c->gen_off.size() - 1 || (n && (!dst_row || !rows_dev || !checksum)))
        return MT_E_INVALID;
    if (c->gen.ins_len_max % 4) { c->err = "exchange rows need ins_len_max % 4 == 0"; return MT_E_INVALID; }
    if (n == 0) return MT_OK;
    int rc;
    if ((rc = mtb_sync(c))) return rc;
    if ((rc = mtb_ensure(c, c->b_tmp0, 8ull * n))) return rc;
    if ((rc = mtb_ensure(c, c->b_tmp1, 8ull * n))) return rc;
    mtb_h2d(c, c->b_tmp0.p, dst_row, 8ull * n);
    if ((rc = mtb_launch_rows(c, true, first, n, c->gen.ins_len_max, (const uint64_t*)c->b_tmp0.p, (uint64_t*)rows_dev,
                              (uint64_t*)c->b_tmp1.p))) return rc;
    if ((rc = mtb_sync(c))) return rc;
    mtb_d2h(c, checksum, c->b_tmp1.p, 8ull * n);
    return MT_OK;
}
int MT_FN(upload_rows_dev)(mt_ctx* c, uint32_t n_runs, const uint32_t* doc_ids, const uint32_t* op_offsets,
                           const void* rows_dev, uint32_t payload_stride, const uint64_t* expect, uint32_t* bad_runs) {
    if (!c || !op_offsets || (n_runs && (!doc_ids || !expect)) || payload_stride == 0 || payload_stride % 4)
        return MT_E_INVALID;
    for (uint32_t r = 0; r < n_runs; r++) {
        if (doc_ids[r] >= c->S.maxDocs) { c->err = "doc id out of range"; return MT_E_INVALID; }
        if (op_offsets[r] > op_offsets[r + 1]) { c->err = "op_offsets not monotone"; return MT_E_INVALID; }
    }
    const uint64_t N = op_offsets[n_runs], L = payload_stride;
    if (N && !rows_dev) return MT_E_INVALID;
    // payload_off is relative to the run's base (op_off[run] * L, 64-bit), so only a run's own
    // slots must stay below 2^32 units
    for (uint32_t r = 0; r < n_runs; r++)
        if ((uint64_t)(op_offsets[r + 1] - op_offsets[r]) * L >= 0xFFFFFFFFull) {
            c->err = "one document's payload slots exceed 2^32 units"; return MT_E_INVALID;
        }
    int rc;
#define UP(buf, bytes) if ((rc = mtb_ensure(c, c->buf, (bytes)))) return rc;
    UP(b_doc, 4ull * n_runs + 4) UP(b_off, 4ull * (n_runs + 1)) UP(b_rec, sizeof(MtOpRec) * N + 32) UP(b_pay, 2 * N * L + 2)
    UP(b_tmp1, 8ull * n_runs + 8) UP(b_pbase, 8ull * n_runs + 8)
#undef UP
    mtb_h2d(c, c->b_doc.p, doc_ids, 4ull * n_runs);
    mtb_h2d(c, c->b_off.p, op_offsets, 4ull * (n_runs + 1));
    {
        std::vector<unsigned long long> pbase(n_runs);
        for (uint32_t r = 0; r < n_runs; r++) pbase[r] = (unsigned long long)op_offsets[r] * L;
        if (n_runs) mtb_h2d(c, c->b_pbase.p, pbase.data(), 8ull * n_runs);
    }
    MtOps& o = c->ops;
    o.doc_ids = (const uint32_t*)c->b_doc.p; o.op_off = (const uint32_t*)c->b_off.p; o.rec = (MtOpRec*)c->b_rec.p;
    o.payload = (uint16_t*)c->b_pay.p; o.n_runs = n_runs; o.payload_units = N * L;
    o.pay_base = (const unsigned long long*)c->b_pbase.p;
    o.rel = nullptr; o.n_rel = 0;
    c->n_runs = n_runs;
    c->run_off.assign(op_offsets, op_offsets + n_runs + 1); c->batch_gen++;
    c->batch_reg = false;                     // exchanged generated streams hold no register ops
    c->batch_wide = mt_dev_wide(c);
    c->gen.enabled = 0;
    if (n_runs && (rc = mtb_launch_rows(c, false, 0, n_runs, (uint32_t)L, nullptr, (uint64_t*)rows_dev,
                                        (uint64_t*)c->b_tmp1.p))) return rc;
    if ((rc = mtb_sync(c))) return rc;
    std::vector<uint64_t> got(n_runs);
    if (n_runs) mtb_d2h(c, got.data(), c->b_tmp1.p, 8ull * n_runs);
    uint32_t bad = 0, first_bad = 0;
    for (uint32_t r = 0; r < n_runs; r++) {
        const bool b = got[r] != expect[r];
        if (bad_runs) bad_runs[r] = b ? 1u : 0u;
        if (b && !bad++) first_bad = r;
    }
    if (bad) {
        char m[128];
        snprintf(m, sizeof m, "exchange checksum mismatch on %u of %u documents (first: run %u)", bad, n_runs, first_bad);
        c->err = m;
        return MT_E_EXCHANGE;
    }
    return MT_OK;
}
int MT_FN(generated_to_resident)(mt_ctx* c) {
    if (!c || !c->gen.enabled) return MT_E_INVALID;
    c->gen.enabled = 0;
    return MT_OK;
}

}  // extern "C"
