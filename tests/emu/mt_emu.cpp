// mt_emu.cpp — TEST-ONLY host emulation of the engine (not shipped, not the product).
//
// Compiles the product's engine logic (fluidframework_amd/csrc/mt_core.h,
// mt_replay.h, mt_api_impl.h) with g++, running each document's "wavefront" as a
// host loop over emulated lanes (wave.h host branch).  CPU tests use it to check
// the exact kernel logic against the oracle without a GPU; the GPU tests then
// check the real gfx950 build (libmtgpu.so) the same way.  Exports emu_* symbols
// only, so it can never be mistaken for the product library.
#include <stdlib.h>
#include <string.h>
#include "../../fluidframework_amd/csrc/mt_ctx.h"
#include "../../fluidframework_amd/csrc/mt_shard.h"

static int mtb_init(mt_ctx*) { return 0; }
static void mtb_fini(mt_ctx* c) { for (auto& st : c->stage) free(st.p); free(c->dl_host[0]); free(c->dl_host[1]); }
static int mtb_malloc(void** p, size_t n) { *p = calloc(1, n ? n : 16); return *p ? 0 : 1; }
static void mtb_free(void* p) { free(p); }
static void mtb_memset(void* p, int v, size_t n) { memset(p, v, n); }
static void mtb_h2d(mt_ctx*, void* d, const void* s, size_t n) { memcpy(d, s, n); }
static void mtb_d2h(mt_ctx*, void* d, const void* s, size_t n) { memcpy(d, s, n); }
static void mtb_d2d(mt_ctx*, void* d, const void* s, size_t n) { memcpy(d, s, n); }
static int mtb_sync(mt_ctx*) { return MT_OK; }
static uint8_t* mtb_host_stage(mt_ctx* c, size_t n, int buf) {
    if (c->dl_cap[buf] < n) { free(c->dl_host[buf]); c->dl_host[buf] = malloc(n); c->dl_cap[buf] = c->dl_host[buf] ? n : 0; }
    return (uint8_t*)c->dl_host[buf];
}
static void* mtb_stage_get(mt_ctx* c, size_t n) {
    mt_ctx::Stage& st = c->stage[c->stage_k];
    if (st.cap < n) { free(st.p); st.p = malloc(n); st.cap = st.p ? n : 0; }
    return st.p;
}
static void mtb_stage_send(mt_ctx* c, void* dev, size_t n) { memcpy(dev, c->stage[c->stage_k].p, n); c->stage_k ^= 1; }
// FULL as on the device: the capture instantiation only while a delta buffer is armed.
// The same per-run function as the device kernels (mt_replay_doc), one run at a time.
template <bool FULL>
static void replay_runs(mt_ctx* c, uint32_t n_runs) {
    uint32_t* cursor = (uint32_t*)c->b_cursor.p;
    for (uint32_t run = 0; run < n_runs; run++) {
        MtScratch sc;
        if (c->use_lds == 3) cursor[run] = mt_replay_doc<MT_RES_BIG, FULL>(c->S, c->ops, run, &sc, c->lds_rows, c->lds_blks, c->lds_heap);
        else if (c->use_lds == 2 && c->big_min_ops && c->run_off.size() == n_runs + 1 &&
                 c->run_off[run + 1] - c->run_off[run] >= c->big_min_ops)      // size classes (mt_set_size_class)
            cursor[run] = FULL ? mt_replay_doc<MT_RES_BIG, FULL>(c->S, c->ops, run, &sc, MT_G_WIN, 0, MT_G_HEAP)
                               : mt_replay_doc<MT_RES_BLKW, FULL, true>(c->S, c->ops, run, &sc, 0, MT_BW_BLKS, MT_BW_HEAP);
        else if (c->use_lds == 2) {                       // long runs (and FULL) continue in-wave, as on the device
            bool anyLong = c->run_off.size() != n_runs + 1;
            for (uint32_t q = 0; q < n_runs && !anyLong; q++) anyLong = c->run_off[q + 1] - c->run_off[q] >= c->cont_min_ops;
            const bool cont = FULL || c->part_cus || c->big_min_ops || anyLong;
            cursor[run] = cont ? mt_replay_doc<MT_RES_BLK, FULL, true>(c->S, c->ops, run, &sc, 0, c->lds_blks, c->lds_heap)
                               : mt_replay_doc<MT_RES_BLK, FULL, false>(c->S, c->ops, run, &sc, 0, c->lds_blks, c->lds_heap);
        }
        else if (c->use_lds) cursor[run] = mt_replay_doc<MT_RES_LDS, FULL>(c->S, c->ops, run, &sc, c->lds_rows, c->lds_blks, c->lds_heap);
        else (void)mt_replay_doc<MT_RES_HBM, FULL>(c->S, c->ops, run, &sc, 0, 0, 0);
    }
    for (uint32_t run = 0; run < n_runs && (c->use_lds == 1 || (c->use_lds == 2 && !FULL)); run++) {
        MtScratch sc;
        mt_replay_doc_rest<FULL>(c->S, c->ops, run, &sc, cursor[run]);
    }
}
// Same two launches as the device (mt_engine.hip): LDS-resident pass, then the
// HBM pass resuming at each run's cursor.
static void mt_auto_partition(mt_ctx* c);
static uint32_t mtb_cu_count(mt_ctx*) { return 256; }                // an MI355X's CUs
static int mtb_launch_replay(mt_ctx* c, const MtGen& g, uint32_t n_runs) {
    if (!g.enabled) mt_auto_partition(c);
    if (g.enabled) {
        for (uint32_t run = 0; run < n_runs; run++) {
            MtScratch sc; int lastRef[64];
            const uint32_t doc = c->ops.doc_ids[run];
            MtEng e; e.bind(c->S, doc, &sc);
            mt_replay_run(e, c->ops, run, doc, &g, lastRef, c->ops.op_off[run]);
            e.store(doc);
        }
        return MT_OK;
    }
    if (c->ops.drec || c->batch_reg || c->batch_wide) replay_runs<true>(c, n_runs);
    else replay_runs<false>(c, n_runs);
    return MT_OK;
}
static int mtb_launch_open(mt_ctx* c, uint32_t first, uint32_t n) {
    for (uint32_t d = first; d < first + n; d++) { MtScratch sc; MtEng e; e.bind(c->S, d, &sc); e.open(); e.store(d); }
    return MT_OK;
}
static int mtb_launch_load(mt_ctx* c, const MtLoad& L, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        MtScratch sc; MtEng e; e.bind(c->S, L.docs[i], &sc); e.open();
        mt_load_doc(e, L, i);
        e.store(L.docs[i]);
    }
    return MT_OK;
}
static int mtb_launch_update_seq(mt_ctx* c, const uint32_t* docs, const int32_t* msn, const int32_t* seq, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        MtScratch sc; MtEng e; e.bind(c->S, docs[i], &sc);
        mt_update_seq_doc(e, msn[i], seq[i]);
        e.store(docs[i]);
    }
    return MT_OK;
}
static int mtb_launch_get_length(mt_ctx* c, const uint32_t* docs, const int32_t* ref, const int32_t* cli, int32_t* out, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        MtScratch sc; MtEng e; e.bind(c->S, docs[i], &sc);
        out[i] = e.perspectiveLengthRO(ref[i], cli[i] < 0 ? MT_NOBODY : cli[i]);
    }
    return MT_OK;
}
static int mtb_launch_query(mt_ctx* c, const MtQuery* q, const uint32_t* grp, MtQueryOut* out, uint32_t n_groups) {
    for (uint32_t g = 0; g < n_groups; g++) {
        MtScratch sc; MtEngFast e; e.bind(c->S, q[grp[g]].doc, &sc);
        mt_query_run(e, c->S, q, grp[g], grp[g + 1], out);
    }
    return MT_OK;
}
static int mtb_launch_gather_text(mt_ctx* c, const unsigned long long* at, const uint32_t* len, const unsigned long long* off,
                                  uint16_t* dst, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) memcpy(dst + off[i], c->S.text + at[i], 2ull * len[i]);
    return MT_OK;
}
static int mtb_launch_pack_size(mt_ctx* c, const uint32_t* docs, MtPackSize* out, uint32_t n, uint32_t epoch) {
    for (uint32_t i = 0; i < n; i++) { MtScratch sc; MtEng e; e.bind(c->S, docs[i], &sc); out[i] = mt_pack_size(e, epoch); }
    return MT_OK;
}
static int mtb_launch_pack(mt_ctx* c, const uint32_t* docs, const uint64_t* off, uint8_t* stage, uint32_t n, uint32_t epoch) {
    for (uint32_t i = 0; i < n; i++) { MtScratch sc; MtEng e; e.bind(c->S, docs[i], &sc); mt_pack_doc(e, stage + off[i], epoch); }
    return MT_OK;
}
static int mtb_launch_rows(mt_ctx* c, bool pack, uint32_t first, uint32_t n, uint32_t L, const uint64_t* dst, uint64_t* rows,
                           uint64_t* cs) {
    for (uint32_t i = 0; i < n; i++)
        cs[i] = pack ? mt_pack_rows_doc(c->ops, first + i, L, dst[i], (unsigned long long*)rows)
                     : mt_unpack_rows_doc(c->ops, i, L, (const unsigned long long*)rows);
    return MT_OK;
}
#define MT_FN(name) emu_##name
#include "../../fluidframework_amd/csrc/mt_api_impl.h"

// Test hook: Heap.add / Heap.get (mt_core.h heapAdd / heapGet) driven directly on document
// `doc`'s heap: ops[i] >= 0 adds {seg i, maxSeq ops[i]}, ops[i] < 0 pops; each pop writes its
// {seg, maxSeq} to out (two ints).  Returns the number of pops, or -1 on an engine status.
extern "C" int emu_test_heap(mt_ctx* c, uint32_t doc, const int32_t* ops, int n, int32_t* out) {
    MtScratch sc;
    MtEng e;
    e.bind(c->S, doc, &sc);
    int np = 0;
    for (int i = 0; i < n; i++) {
        if (ops[i] >= 0) e.heapAdd(i, ops[i]);
        else {
            const MtHeapE x = e.heapGet();
            out[2 * np] = x.seg; out[2 * np + 1] = x.maxSeq; np++;
        }
        if (e.status) return -1;
    }
    return np;
}

#if defined(MT_WTRACE)
// Write tracing (diagnostic builds only, -DMT_WTRACE; tools/write_sites.py): after every message
// of a replay the document's HBM pools are compared with a shadow copy, and every 64-byte line
// that changed is counted against its pool (rows also per field).  Under LDS residency the blocks
// and heap stay out of the pools until the run's write-back, which counts as phase 1.  A line
// rewritten by several messages counts once per message (a GPU's L2 merges such writes only while
// the line stays resident).
namespace {
mt_ctx* g_wt = nullptr;
enum { WT_ROWS, WT_BLK, WT_HEAP, WT_WIN, WT_UID, WT_UDELTA, WT_UANC, WT_TEXT, WT_PSET, WT_HDR, WT_HOLD, WT_OVX, WT_MID,
       WT_REG, WT_REGR, WT_N };
struct WtRegion { uint8_t* base; size_t bytes; };
std::vector<std::vector<uint8_t>> g_shadow(WT_N);
unsigned long long g_lines[2][WT_N], g_rowField[16], g_msgs;
WtRegion wt_region(uint32_t doc, int k) {
    const MtState& S = g_wt->S; const MtDocLayout& y = g_wt->layout_h[doc];
    switch (k) {
    case WT_ROWS: return {(uint8_t*)(S.rows + y.row), sizeof(MtRow) * y.rowCap};
    case WT_BLK: return {(uint8_t*)(S.blk + y.blk), sizeof(MtBlk) * y.blkCap};
    case WT_HEAP: return {(uint8_t*)(S.heap + y.heap), sizeof(MtHeapE) * (y.heapCap + 1)};
    case WT_WIN: return {(uint8_t*)(S.win + y.win), 4ull * y.winCap};
    case WT_UID: return {(uint8_t*)(S.uid + y.win), 4ull * y.winCap};
    case WT_UDELTA: return {(uint8_t*)(S.udelta + y.win), 4ull * y.winCap};
    case WT_UANC: return {(uint8_t*)(S.uanc + y.anc), 4ull * y.winCap * MT_MAXH};
    case WT_TEXT: return {(uint8_t*)(S.text + y.text), 4ull * y.textCap};
    case WT_PSET: return {(uint8_t*)(S.pset + y.pset), sizeof(MtPSet) * y.psetCap};
    case WT_HDR: return {(uint8_t*)(S.hdr + doc), sizeof(MtDocHdr)};
    case WT_HOLD: return {(uint8_t*)(S.hold + (size_t)doc * MT_RFL), 4ull * MT_RFL};
    case WT_OVX: return {(uint8_t*)(S.ovx + (size_t)doc * MT_OVX_CAP), sizeof(MtOvx) * MT_OVX_CAP};
    case WT_MID: return {(uint8_t*)(S.mid + y.mid), 4ull * y.midCap};
    case WT_REG: return {(uint8_t*)(S.reg + (size_t)doc * MT_REG_CAP), sizeof(MtReg) * MT_REG_CAP};
    default: return {(uint8_t*)(S.regr + y.regr), 8ull * y.regCap};
    }
}
}  // namespace
void mt_wtrace_begin(uint32_t doc) {
    if (!g_wt) return;
    // a freshly opened document: every pool but its header, block 0 and its registers (what open()
    // wrote) is free, and is poisoned, so a store rewriting what an earlier replay of the same
    // stream left there still shows as a change (tools/write_sites.py checks the digests)
    if (g_wt->S.hdr[doc].rowTop == 0)
        for (int k = 0; k < WT_N; k++) {
            if (k == WT_HDR || k == WT_REG) continue;
            const WtRegion r = wt_region(doc, k);
            const size_t skip = k == WT_BLK ? sizeof(MtBlk) : 0;
            if (r.bytes > skip) memset(r.base + skip, 0xA5, r.bytes - skip);
        }
    for (int k = 0; k < WT_N; k++) { const WtRegion r = wt_region(doc, k); g_shadow[k].assign(r.base, r.base + r.bytes); }
}
void mt_wtrace_msg(uint32_t doc, int phase) {
    if (!g_wt) return;
    if (phase == 0) g_msgs++;
    for (int k = 0; k < WT_N; k++) {
        const WtRegion r = wt_region(doc, k);
        uint8_t* sh = g_shadow[k].data();
        const uintptr_t a0 = (uintptr_t)r.base;
        for (size_t pg = 0; pg < r.bytes; pg += 4096) {           // pages first, then 64-byte lines
            const size_t pn = std::min<size_t>(4096, r.bytes - pg);
            if (!memcmp(sh + pg, r.base + pg, pn)) continue;
            for (size_t o = pg; o < pg + pn;) {
                const size_t lineEnd = std::min(pg + pn, (size_t)(((a0 + o) / 64 + 1) * 64 - a0));
                if (memcmp(sh + o, r.base + o, lineEnd - o)) {
                    g_lines[phase][k]++;
                    if (k == WT_ROWS)
                        for (size_t b = o; b < lineEnd; b += 4)
                            if (memcmp(sh + b, r.base + b, 4)) g_rowField[(b % sizeof(MtRow)) / 4]++;
                    memcpy(sh + o, r.base + o, lineEnd - o);
                }
                o = lineEnd;
            }
        }
    }
}
// on = 1: start tracing on c (counters reset); on = 0: stop and copy the counters out:
// [2][WT_N] lines (per message / at run ends), 12 row-field dword counts, messages.
extern "C" int emu_wtrace(mt_ctx* c, int on, unsigned long long* out) {
    if (on) { g_wt = c; memset(g_lines, 0, sizeof g_lines); memset(g_rowField, 0, sizeof g_rowField); g_msgs = 0; return WT_N; }
    g_wt = nullptr;
    if (out) {
        memcpy(out, g_lines, sizeof g_lines);
        memcpy(out + 2 * WT_N, g_rowField, sizeof g_rowField);
        out[2 * WT_N + 12] = g_msgs;
    }
    return WT_N;
}
#endif
