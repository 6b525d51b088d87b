// mt_query.h — position queries on replayed documents (mt_get_containing_segment):
//   MergeTree.getContainingSegment        MT/mergeTree.ts:1616-1627 (searchBlock :1786-1815)
//   MergeTree.resolveRemoteClientPosition MT/mergeTree.ts:2125-2145
//   MergeTree.getPosition                 MT/mergeTree.ts:1578-1596 (the local view)
// Batched: the host groups the queries by document, one wave takes a document's queries
// in order (the perspective's U set is reused while consecutive queries share it).  A
// query reads the document and writes only the wave's U scratch of that document.
#pragma once
#include "mt_core.h"

struct __attribute__((aligned(16))) MtQuery { uint32_t doc; int32_t pos, ref, client; };   // ref < 0: local view
// One answer: the ABI record, where the found row's text sits in the text pool, and the
// chunks of its property map (the host writes the segment's JSON from them).
struct __attribute__((aligned(16))) MtQueryOut {
    mt_seg_info info;
    unsigned long long text_at;            // element index into MtState::text (text rows)
    unsigned long long pad;
    MtPSet ps[MT_PKEYS / MT_PSK];
};
static_assert(sizeof(mt_seg_info) == 64, "mt_seg_info is 16 dwords");

template <class Eng>
MT_HD void mt_query_run(Eng& e, const MtState& S, const MtQuery* q, uint32_t q0, uint32_t q1, MtQueryOut* out) {
    for (uint32_t i = q0; i < q1; i++) {
        const int pos = uni(q[i].pos), ref = uni(q[i].ref), qc = uni(q[i].client);
        // the local view: every sequenced op applied (removals included), as (refSeq = max,
        // a client id no row carries) sees it
        const bool local = ref < 0;
        const int r = local ? 0x7FFFFFFF : ref, c = (local || qc < 0 || qc >= MT_NONCOLLAB) ? MT_NOBODY : qc;
        int off = 0, depth = 0;
        unsigned long long path = 0;
        const int s = e.containing(pos, r, c, off, depth, path);
        int f[16];
        for (int k = 0; k < 16; k++) f[k] = 0;
        unsigned long long tat = 0;
        int nch = 0, ps = -1;
        if (s >= 0) {
            const uint32_t mt = uni(e.row(s).meta);
            const bool removed = (mt & MT_M_REMOVED) != 0, marker = (mt & MT_M_MARKER) != 0;
            const int cl = (int)(mt & MT_M_CLIENT);
            const int op = e.obsPosition(s);
            ps = uni(e.row(s).props);
            f[0] = 1; f[1] = off; f[2] = op; f[3] = uni(e.row(s).len); f[4] = uni(e.row(s).seq);
            f[5] = cl == MT_NONCOLLAB ? -1 : cl;
            f[6] = removed ? uni(e.row(s).rseq) : (int)0x80000000;
            f[7] = removed ? (int)uni(e.row(s).rcl) : -1;
            f[8] = ps; f[9] = marker ? uni(e.row(s).toff) : -1;
            f[10] = depth; f[11] = (int)(uint32_t)path; f[12] = (int)(uint32_t)(path >> 32);
            f[13] = s; f[14] = op + off;
            if (!marker) tat = (unsigned long long)(e.text - S.text) + (unsigned long long)uni(e.row(s).toff);
            if (ps >= 0) { const int n = uni(e.pset[ps].n); nch = n > MT_PSK ? (n + MT_PSK - 1) / MT_PSK : 1; }
        } else {
            // resolveRemoteClientPosition's fall-through: the end of the remote view maps to the
            // end of the local one
            const int L = e.perspectiveLength(r, c);
            f[1] = -1; f[2] = -1; f[5] = -1; f[6] = (int)0x80000000; f[7] = -1; f[8] = -1; f[9] = -1; f[13] = -1;
            f[14] = pos == L ? uni(e.bk(e.root).len) : (int)0x80000000;
        }
        MtQueryOut& o = out[i];
        const auto fv = wave_map(16, [&](int k) MT_LAM { return pick16(f, k); });
        wave_for(16, [&](int k) MT_LAM { ((int*)&o.info)[k] = own(fv, k); });
        wave_for(1, [&](int) MT_LAM { o.text_at = tat; o.pad = 0; });
        // the property map's chunks, one dword per lane (28 dwords a chunk)
        constexpr int W = (int)(sizeof(MtPSet) / 4);
        for (int base = 0; base < nch * W; base += MT_WAVE) {
            const int m = (nch * W - base) < MT_WAVE ? (nch * W - base) : MT_WAVE;
            wave_for(m, [&](int k) MT_LAM { ((int*)o.ps)[base + k] = ((const int*)(e.pset + ps))[base + k]; });
        }
        wave_sync();
    }
}
