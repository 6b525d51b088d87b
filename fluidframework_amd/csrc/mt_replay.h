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
MT_HD inline void mt_gen_op(MtEng& e, const MtOps& ops, uint32_t i, uint32_t k, uint32_t doc,
                            const MtGen& g, MtRng& rng, int* lastRef) {
    const uint32_t a = rng.u(g.clients);
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
    const uint32_t poff = (uint32_t)((size_t)doc * g.ops * g.ins_len_max + (size_t)k * g.ins_len_max);
    if (ty == MT_OP_INSERT) {
        s1 = (int)rng.u((uint32_t)L + 1);
        plen = 1 + rng.u(g.ins_len_max);
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
    for (uint32_t c = 1; c < g.clients; c++) mn = lastRef[c] < mn ? lastRef[c] : mn;
    ops.type[i] = (uint8_t)ty; ops.flags[i] = fl; ops.client[i] = (uint16_t)a;
    ops.seq[i] = e.curSeq + 1; ops.ref_seq[i] = r; ops.msn[i] = mn;
    ops.pos1[i] = s1; ops.pos2[i] = s2; ops.payload_off[i] = poff; ops.payload_len[i] = plen; ops.prop_id[i] = pid;
    wave_sync();
}

MT_HD inline void mt_replay_run(MtEng& e, const MtOps& ops, uint32_t run, uint32_t doc,
                                const MtGen* g, int* lastRef) {
    const uint32_t o0 = ops.op_off[run], o1 = ops.op_off[run + 1];
    MtRng rng; rng.s = 0;
    if (g) {
        rng.s = g->seed ^ (0x9E3779B97F4A7C15ULL * (unsigned long long)(doc + 1));
        for (int c = 0; c < 64; c++) lastRef[c] = 0;
    }
    for (uint32_t i = o0; i < o1; i++) {
        if (g) mt_gen_op(e, ops, i, i - o0, doc, *g, rng, lastRef);
        const int ty = ops.type[i];
        const uint32_t fl = ops.flags[i];
        const int c = ops.client[i];
        const int sq = ops.seq[i], r = ops.ref_seq[i], ms = ops.msn[i];
        if (ty != MT_OP_NOOP) {
            if (c >= 64) e.status |= MT_DS_UNSUPPORTED;
            if (e.curSeq >= sq) e.status |= MT_DS_ASSERT_SEQ;       // completeAndLogOp, MT/client.ts:482
            if (e.minSeq > ms) e.status |= MT_DS_ASSERT_MSN;        // MT/client.ts:484
            if (e.status) break;
            if (!(e.uValid && e.uRef == r && e.uCli == c)) e.computeU(r, c, true);
            if (ty == MT_OP_INSERT) {
                const bool marker = (fl & MT_OPF_MARKER) != 0;
                e.opInsert(ops.pos1[i], r, c, sq, ops.payload + ops.payload_off[i], (int)ops.payload_len[i],
                           marker, ops.pos2[i], (fl & MT_OPF_SEG_PROPS) ? ops.prop_id[i] : -1);
            } else if (ty == MT_OP_REMOVE) {
                e.opRange(MT_MAP_REMOVE, ops.pos1[i], ops.pos2[i], r, c, sq, -1, false);
            } else if (ty == MT_OP_ANNOTATE) {
                if (fl & MT_OPF_COMBINE) { e.status |= MT_DS_UNSUPPORTED; break; }
                e.opRange(MT_MAP_ANNOTATE, ops.pos1[i], ops.pos2[i], r, c, sq, ops.prop_id[i], (fl & MT_OPF_REWRITE) != 0);
            }
            e.uValid = false;
            e.cnt[0] += 1;
            e.cnt[4] += (unsigned long long)(e.height + 1);
        }
        if (fl & MT_OPF_END_OF_MSG) {                               // updateSeqNumbers, MT/client.ts:843-850
            e.cnt[1] += 1;
            if (e.curSeq > sq) { e.status |= MT_DS_ASSERT_SEQ; break; }
            e.curSeq = sq;
            e.setMinSeq(ms);
        }
        if (e.status) break;
    }
}
