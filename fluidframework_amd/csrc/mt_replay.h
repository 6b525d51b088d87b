// mt_replay.h — Client.applyMsg for a run of one document's messages, and the
// device stream generator (SURVEY.md §8(d) stream rules; the same algorithm is
// restated in oracle/mtoracle.cpp ora_generate_doc for parity).
#pragma once
#include "mt_core.h"

struct MtRng {                                     // splitmix64
    unsigned long long s;
    MT_HD unsigned long long next() {
        unsigned long long z = (s += 0x9E3779B97F4A7C15ULL);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    MT_HD uint32_t u(uint32_t n) { return (uint32_t)(next() % (unsigned long long)n); }
};

// Synthesize message i of document `doc` from the engine's own state (the
// engine acts as sequencer + observer, so positions are valid under the
// author's perspective), writing the op record into the batch arrays.
template <class Eng>
MT_HD void mt_gen_op(Eng& e, const MtOps& ops, uint32_t i, uint32_t k, uint32_t nc,
                            const MtGen& g, MtRng& rng, int* lastRef) {
    const uint32_t a = rng.u(nc);
    const uint32_t lag = rng.u(g.lag_max + 1);
    int r = e.curSeq - (int)lag;
    if (r < lastRef[a]) r = lastRef[a];
    if (r < e.minSeq) r = e.minSeq;
    lastRef[a] = r;
    e.computeU(r, (int)a, true);
    const int L = e.perspectiveLength(r, (int)a);
    const uint32_t tsel = rng.u(100);
    int ty = tsel < g.pct_insert ? MT_OP_INSERT : (tsel < g.pct_insert + g.pct_remove ? MT_OP_REMOVE : MT_OP_ANNOTATE);
    if (L == 0) ty = MT_OP_INSERT;
    int s1 = 0, s2 = 0, pid = -1; uint32_t plen = 0; uint8_t fl = MT_OPF_END_OF_MSG;
    const uint32_t poff = (uint32_t)((size_t)i * g.ins_len_max);      // fixed stride per op record
    MtOpRec& o = ops.rec[i];
    if (ty == MT_OP_INSERT) {
        s1 = g.ins_at_end ? L : (int)rng.u((uint32_t)L + 1);
        const uint32_t lo = g.ins_len_min > 1 ? g.ins_len_min : 1;
        plen = lo + rng.u(g.ins_len_max - lo + 1);
        if (g.seg_prop_sets) { pid = (int)(k % g.seg_prop_sets); fl |= MT_OPF_SEG_PROPS; }
        for (uint32_t q = 0; q < plen; q++) {
            const uint16_t ch = (uint16_t)('a' + rng.u(26));
            ops.payload[poff + q] = ch;
        }
    } else {
        s1 = (int)rng.u((uint32_t)L);
        const uint32_t n = 1 + rng.u(g.rem_len_max);
        s2 = (s1 + (int)n < L) ? s1 + (int)n : L;
        if (ty == MT_OP_ANNOTATE) {
            pid = (int)rng.u(g.n_ann_sets);
            if (rng.u(100) < g.pct_rewrite) fl |= MT_OPF_REWRITE;
        }
    }
    int mn = lastRef[0];
    for (uint32_t c = 1; c < nc; c++) mn = lastRef[c] < mn ? lastRef[c] : mn;
    o.type = (uint8_t)ty; o.flags = fl; o.client = (uint16_t)a;
    o.seq = e.curSeq + 1; o.ref_seq = r; o.msn = mn;
    o.pos1 = s1; o.pos2 = s2; o.payload_off = poff; o.payload_len = (uint16_t)plen; o.prop_id = (int16_t)pid;
    wave_sync();
}

#if defined(MT_WTRACE) && !defined(__HIP_DEVICE_COMPILE__)
// Host-emulation diagnostic (tools/write_sites.py): the HBM lines each message dirtied, by pool.
void mt_wtrace_begin(uint32_t doc);
void mt_wtrace_msg(uint32_t doc, int phase);
#define MT_WT_BEGIN(doc) mt_wtrace_begin(doc)
#define MT_WT_MSG(doc, ph) mt_wtrace_msg(doc, ph)
#else
#define MT_WT_BEGIN(doc) ((void)0)
#define MT_WT_MSG(doc, ph) ((void)0)
#endif

// Applies ops [o0, op_off[run+1]) of the run.  With LDS pools (e.lds) it stops
// before an op that could outgrow them and returns that op's index, so the HBM
// kernel can resume there; otherwise it returns op_off[run+1].
template <class Eng>
MT_HD uint32_t mt_replay_run(Eng& e, const MtOps& ops, uint32_t run, uint32_t doc,
                                const MtGen* g, int* lastRef, uint32_t o0) {
    const uint32_t o1 = ops.op_off[run + 1];
    const unsigned long long pb = ops.pay_base ? uni64(ops.pay_base[run]) : 0ull;
    const uint16_t* payR = ops.payload + pb;                  // this run's payload (pay_base: relative offsets)
    MtRng rng; rng.s = 0;
    const uint32_t nc = g ? (g->clients_per_run ? g->clients_per_run[run] : g->clients) : 0;
    if (g) {
        rng.s = g->seed ^ (0x9E3779B97F4A7C15ULL * (unsigned long long)(g->doc_id_base + doc + 1));
        for (int c = 0; c < 64; c++) lastRef[c] = e.minSeq;   // 0 for fresh documents; continue_docs keeps MSN monotone
    }
    // Replay prefetches op i+1's record while op i runs (generation writes the
    // record at the top of each iteration, so it loads in place).
    auto wn = wave_map(8, [&](int q) MT_LAM { return (!g && o0 < o1) ? ((const int*)&ops.rec[o0])[q] : 0; });
    if (!g && Eng::kFull) { e.drec = ops.drec; e.dcount = ops.dcount; e.dcap = ops.dcap; e.dtext = ops.dtext; e.dtcap = ops.dtcap; }
    // this message's capture reservation (FULL): released after the message, or after the
    // loop when an error ends the run mid-message
    unsigned long long resR = 0, resT = 0;
#if defined(MT_EVCOUNT3) && !defined(__HIP_DEVICE_COMPILE__)
    if (e.prof[0] == 0) e.prof[0] = 1000000 - 100;          // max growth - 2 * height, offset by 1e6
    e.prof[3] = (unsigned long long)(e.blkTop - e.blkFreeN); e.prof[4] = (unsigned long long)e.height;
#endif
    for (uint32_t i = o0; i < o1; i++) {
        e.curOp = i;
        if constexpr (Eng::kLds) {
            int k = 0;                                   // a paste inserts every clone of its register
            if constexpr (Eng::kFull) {
                if (!g) {
                    const uint32_t r0 = (uint32_t)uni(((const int*)&ops.rec[i])[0]);
                    if ((int)(r0 & 0xFF) == MT_OP_PASTE) k = e.regCount((int)(r0 >> 16), uni(((const int*)&ops.rec[i])[6]));
                }
            }
            if (!e.ldsHeadroom(k)) return i;
        }
#if defined(MT_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
        const unsigned long long tg = __builtin_amdgcn_s_memtime();
        if (g) mt_gen_op(e, ops, i, i - o0, nc, *g, rng, lastRef);
        e.prof[MT_PH_GEN] += __builtin_amdgcn_s_memtime() - tg;
        const unsigned long long top = __builtin_amdgcn_s_memtime();
#else
        if (g) mt_gen_op(e, ops, i, i - o0, nc, *g, rng, lastRef);
#endif
        // one 32-byte record: lanes 0..7 hold a dword each, then broadcast
        auto w = wn;
        if (g) w = wave_map(8, [&](int q) MT_LAM { return ((const int*)&ops.rec[i])[q]; });
        else if (i + 1 < o1) wn = wave_map(8, [&](int q) MT_LAM { return ((const int*)&ops.rec[i + 1])[q]; });
        const uint32_t w0 = (uint32_t)wave_at(w, 0);
        const int ty = (int)(w0 & 0xFF);
        const uint32_t fl = (w0 >> 8) & 0xFF;
        const int c = (int)(w0 >> 16);
        const int sq = wave_at(w, 1), r = wave_at(w, 2), ms = wave_at(w, 3);
        const int p1 = wave_at(w, 4), p2 = wave_at(w, 5);
        const uint32_t poff = (uint32_t)wave_at(w, 6);
        const uint32_t w7 = (uint32_t)wave_at(w, 7);
        const int plen = (int)(w7 & 0xFFFF), pid = (int)(int16_t)(w7 >> 16);
        if (ty == MT_OP_UNSUPPORTED) { e.status |= MT_DS_UNSUPPORTED; break; }
        if constexpr (Eng::kFull) {
            if (!g && e.drec) {
                // capture headroom for this message: a range op emits at most one record per
                // character of its range (every segment it touches is visible in it), or per row
                const bool range = ty == MT_OP_REMOVE || ty == MT_OP_ANNOTATE || ty == MT_OP_CUT;
                long long k = ty == MT_OP_PASTE ? (long long)e.regCount(c, (int)poff) : 1;   // a paste: its clones
                if (range) {
                    k = (fl & (MT_OPF_REL1 | MT_OPF_REL2)) ? (long long)e.rowTop : (long long)p2 - (long long)p1;
                    if (k > (long long)e.rowTop) k = e.rowTop;
                    if (k < 0) k = 0;
                }
                resR = (unsigned long long)k + MT_DREC_SLACK;
                resT = ty == MT_OP_PASTE ? (unsigned long long)e.regTextLen(c, (int)poff) : 0ull;
                if (!e.dReserve(resR, resT)) { e.dStop = 1; return i; }
            }
        }
        if (ty != MT_OP_NOOP) {
            if (c >= MT_NONCOLLAB) e.status |= MT_DS_UNSUPPORTED;  // 0xFFFE/0xFFFF are reserved ids
            if (e.curSeq >= sq) e.status |= MT_DS_ASSERT_SEQ;       // completeAndLogOp, MT/client.ts:482
            if (e.minSeq > ms) e.status |= MT_DS_ASSERT_MSN;        // MT/client.ts:484
            if (r < e.minSeq) e.status |= MT_DS_REFSEQ_BELOW_MSN;   // nacked by deli (deli/lambda.ts:302-318)
            if (ty == MT_OP_INSERT && !(fl & MT_OPF_MARKER) && pb + (uint64_t)poff + (uint64_t)plen > ops.payload_units)
                e.status |= MT_DS_BAD_OP;
            if (e.status) break;
            const bool pre = ty == MT_OP_INSERT && !(fl & MT_OPF_MARKER) && plen <= MT_WAVE;
            const auto pay = wave_map(pre ? plen : 0, [&](int k) MT_LAM { return (int)payR[poff + (uint32_t)k]; });
            if (!(e.uValid && e.uRef == r && e.uCli == c)) e.computeU(r, c, true);
            e.mwPrefetch();                                      // long documents: warm zamboni's rows
            int q1 = p1, q2 = p2;
            if (fl & (MT_OPF_REL1 | MT_OPF_REL2)) {       // getValidOpRange (MT/client.ts:506-523)
                if ((fl & MT_OPF_REL1) && (p1 < 0 || (uint32_t)p1 >= ops.n_rel)) { e.status |= MT_DS_BAD_OP; break; }
                if ((fl & MT_OPF_REL2) && (p2 < 0 || (uint32_t)p2 >= ops.n_rel)) { e.status |= MT_DS_BAD_OP; break; }
                if (fl & MT_OPF_REL1) q1 = e.relPos(ops.rel[p1], r, c);
                if (fl & MT_OPF_REL2) q2 = e.relPos(ops.rel[p2], r, c);
                if (q1 < 0 || ((fl & MT_OPF_REL2) && q2 < 0)) { e.status |= MT_DS_UNSUPPORTED; break; }
            }
            if (ty == MT_OP_INSERT) {
                const bool marker = (fl & MT_OPF_MARKER) != 0;
                e.opInsert(q1, r, c, sq, payR + poff, plen, marker, p2, (fl & MT_OPF_SEG_PROPS) ? pid : -1,
                           (marker && (fl & MT_OPF_MARKER_ID)) ? (int)poff : -1, pay);
            } else if (ty == MT_OP_REMOVE) {
                e.opRange(MT_MAP_REMOVE, q1, q2, r, c, sq, -1, MT_PM_SET);
            } else if (ty == MT_OP_ANNOTATE) {
                e.opRange(MT_MAP_ANNOTATE, q1, q2, r, c, sq, pid, mt_prop_mode(fl));
            } else if (ty >= MT_OP_CUT && ty <= MT_OP_PASTE) {
                if constexpr (Eng::kFull) {
                    if (ty == MT_OP_PASTE) e.opPaste(q1, r, c, sq, (int)poff);
                    else {
                        e.opCopy(q1, q2, r, c, (int)poff);                   // CUT: copy, then markRangeRemoved
                        if (ty == MT_OP_CUT && !e.status) e.opRange(MT_MAP_REMOVE, q1, q2, r, c, sq, -1, MT_PM_SET);
                    }
                } else { e.status |= MT_DS_UNSUPPORTED; break; }            // launched without register support
            } else { e.status |= MT_DS_BAD_OP; break; }
            e.uValid = false;
#if defined(MT_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
            e.prof[MT_PH_OP] += __builtin_amdgcn_s_memtime() - top;
#endif
            e.c_ops += 1;
            e.c_depth += (unsigned long long)(e.height + 1);
        }
        if (fl & MT_OPF_END_OF_MSG) {                               // updateSeqNumbers, MT/client.ts:843-850
            e.c_msgs += 1;
            if (e.curSeq > sq) { e.status |= MT_DS_ASSERT_SEQ; break; }
            e.curSeq = sq;
            e.setMinSeq(ms);
            MT_WT_MSG(doc, 0);
#if defined(MT_EVCOUNT3) && !defined(__HIP_DEVICE_COMPILE__)
            {   // host emulation: blocks a message added (op and zamboni) beyond 2 * height at its start
                const int used = e.blkTop - e.blkFreeN;
                const long long g = (long long)used - (long long)e.prof[3] - 2ll * (long long)e.prof[4];
                if (g > (long long)e.prof[0] - 1000000) e.prof[0] = (unsigned long long)(g + 1000000);
                e.prof[3] = (unsigned long long)used; e.prof[4] = (unsigned long long)e.height;
            }
#endif
        }
        if (e.status) break;
        if constexpr (Eng::kFull) { if (resR) { e.dRelease(resR, resT); resR = resT = 0; } }
    }
    if constexpr (Eng::kFull) { if (resR) e.dRelease(resR, resT); }
    return o1;
}

// cursor[] flag: the run left LDS at the op index in the low bits and finished in HBM in the same
// wave (the all-HBM launch that follows skips it; mt_last_cursors reports the hand-over op).
#define MT_CUR_DONE MT_CURSOR_DONE          // include/mtgpu.h
// One document run of a replay launch (every replay kernel and the host emulation run this).
// The run starts at ops.start[run] (a capture resume) or op_off[run]; RES is the residency it
// starts in.  A document that outgrows the LDS pools continues in HBM in the same wave when
// CONT (MT_RES_BIG, and MT_RES_BLK for long runs), or else stops there and hands the rest to a
// second, all-HBM launch (the returned op index goes to cursor[]): MT_RES_LDS, and MT_RES_BLK
// for the runs shorter than the context's continuation threshold, whose kernel then carries no
// second engine and runs without scratch.  Capture launches record in ops.resume[run] where the
// run stopped for headroom (op_off[run + 1]: finished).
template <int RES, bool FULL, bool CONT = true>
MT_HD uint32_t mt_replay_doc(const MtState& S, const MtOps& ops, uint32_t run, MtScratch* sc, int l0, int l1, int l2) {
    const uint32_t doc = ops.doc_ids[run], o1 = ops.op_off[run + 1];
    const uint32_t o0 = ops.start ? ops.start[run] : ops.op_off[run];
    uint32_t cur = o0, stop = o1;
    if (o0 < o1) {
        MT_WT_BEGIN(doc);
        MtEngT<RES, FULL> e;
        e.bind(S, doc, sc);
        if constexpr (RES == MT_RES_HBM) { (void)l0; (void)l1; (void)l2; cur = mt_replay_run(e, ops, run, doc, nullptr, nullptr, o0); }
        else if (e.toLds(l0, l1, l2)) {
            cur = mt_replay_run(e, ops, run, doc, nullptr, nullptr, o0);
            e.fromLds();
        }
        const bool stopped = e.dStop != 0;
        e.store(doc);
        MT_WT_MSG(doc, 1);                                       // the write-back at the run's end
        if (stopped) { stop = cur; cur = o1; }                   // no hand-over: the host resumes it
        else if (RES != MT_RES_LDS && CONT && cur < o1) {
            // A document that outgrew LDS continues here with its pools in HBM (no second
            // launch: long documents, which outgrow it first, keep their head start).
            MtEngT<MT_RES_HBM, FULL> h;
            h.bind(S, doc, sc);
            const uint32_t c2 = mt_replay_run(h, ops, run, doc, nullptr, nullptr, cur);
            if (h.dStop) stop = c2;
            h.store(doc);
            MT_WT_MSG(doc, 1);
            cur |= MT_CUR_DONE;                              // finished here: no second launch
        }
    }
    constexpr bool handsOver = RES == MT_RES_LDS || !CONT;
    if (FULL && ops.resume && !(handsOver && cur < o1)) wave_for(1, [&](int) MT_LAM { ops.resume[run] = stop; });
    return cur;
}
// The all-HBM pass after an MT_RES_LDS or MT_RES_BLK launch: the rest of each run from its
// hand-over point.
template <bool FULL>
MT_HD void mt_replay_doc_rest(const MtState& S, const MtOps& ops, uint32_t run, MtScratch* sc, uint32_t o0) {
    const uint32_t o1 = ops.op_off[run + 1];
    if (o0 >= o1) return;
    const uint32_t doc = ops.doc_ids[run];
    MtEngT<MT_RES_HBM, FULL> e;
    e.bind(S, doc, sc);
    const uint32_t c2 = mt_replay_run(e, ops, run, doc, nullptr, nullptr, o0);
    const uint32_t stop = e.dStop ? c2 : o1;
    e.store(doc);
    if (FULL && ops.resume) wave_for(1, [&](int) MT_LAM { ops.resume[run] = stop; });
}

// Client.updateSeqNumbers(min, seq) (MT/client.ts:843-850) on one document;
// seq < 0 leaves the document's window as it is (mt_snapshot_* "current").
template <class Eng>
MT_HD void mt_update_seq_doc(Eng& e, int msn, int seq) {
    if (seq < 0) return;
    if (e.curSeq > seq) { e.status |= MT_DS_ASSERT_SEQ; return; }
    e.curSeq = seq;
    e.setMinSeq(msn);
}
