// mt_pack.h — gather documents' live state into one contiguous staging buffer
// (device side of mt_snapshot_v1 / mt_snapshot_digests / mt_get_text for many
// documents: one download instead of four copies per document).
//
// Per document, at staging offset off[i] (16-byte aligned):
//   MtDocHdr | rows[0, rowTop) | blocks[0, blkTop) | referenced psets (compacted) | live text
// Live text is compacted (as textGC does): linked text rows' slices back to back,
// with each staged row's toff rewritten to its slice; markers keep refType in toff.
#pragma once
#include "mt_core.h"

struct MtPackSize { uint32_t rows, blks, psets, text; };

MT_INLINE uint64_t mt_pack_bytes(const MtPackSize& z) {
    const uint64_t t = ((uint64_t)z.text * 2 + 15) & ~15ull;
    return sizeof(MtDocHdr) + (uint64_t)z.rows * sizeof(MtRow) + (uint64_t)z.blks * sizeof(MtBlk) +
           (uint64_t)z.psets * sizeof(MtPSet) + t;
}
MT_INLINE int mt_pset_chunks(int n) { return n > MT_PSK ? (n + MT_PSK - 1) / MT_PSK : 1; }

// Only the property maps linked rows reference are staged (the pool is append-only: an
// annotate-heavy document holds tens of maps per live row).  mt_pack_size marks each
// referenced map's first chunk with the staging epoch (MtPSet::pad[0]) and counts the marked
// maps' chunks; mt_pack_doc stages them back to back, records each one's staged index in
// pad[1] and rewrites the staged rows' ids.  (The pads are not engine state.)
template <class Eng>
MT_HD MtPackSize mt_pack_size(Eng& e, uint32_t epoch) {
    MtPackSize z; z.rows = (uint32_t)e.rowTop; z.blks = (uint32_t)e.blkTop;
    int t = 0;
    for (int base = 0; base < e.rowTop; base += MT_WAVE) {
        const int m = (e.rowTop - base) < MT_WAVE ? (e.rowTop - base) : MT_WAVE;
        t += wave_sum(wave_map(m, [&](int k) MT_LAM {
            const int s = base + k;
            const bool linked = e.R[s].parent >= 0;
            const int p = e.R[s].props;
            if (linked && p >= 0) e.pset[p].pad[0] = (int32_t)epoch;
            return (linked && !(e.R[s].meta & MT_M_MARKER)) ? e.R[s].len : 0;
        }));
    }
    z.text = (uint32_t)t;
    wave_sync();
    int np = 0;
    for (int base = 0; base < e.psetTop; base += MT_WAVE) {
        const int m = (e.psetTop - base) < MT_WAVE ? (e.psetTop - base) : MT_WAVE;
        np += wave_sum(wave_map(m, [&](int k) MT_LAM {
            const MtPSet& q = e.pset[base + k];
            return q.pad[0] == (int32_t)epoch ? mt_pset_chunks(q.n) : 0;
        }));
    }
    z.psets = (uint32_t)np;
    return z;
}

template <class Eng>
MT_HD void mt_pack_doc(Eng& e, uint8_t* dst, uint32_t epoch) {
    const int rowTop = e.rowTop, blkTop = e.blkTop, psetTop = e.psetTop;
    MtRow* rows = (MtRow*)(dst + sizeof(MtDocHdr));
    MtBlk* blks = (MtBlk*)(rows + rowTop);
    MtPSet* ps = (MtPSet*)(blks + blkTop);
    {   // header
        const int* src = (const int*)e.hdrp;
        int* d = (int*)dst;
        wave_for((int)(sizeof(MtDocHdr) / 4), [&](int k) MT_LAM { d[k] = src[k]; });
    }
    int wp = 0;                                  // referenced property maps, compacted
    for (int base = 0; base < psetTop; base += MT_WAVE) {
        const int m = (psetTop - base) < MT_WAVE ? (psetTop - base) : MT_WAVE;
        auto nc = wave_map(m, [&](int k) MT_LAM {
            const MtPSet& q = e.pset[base + k];
            return q.pad[0] == (int32_t)epoch ? mt_pset_chunks(q.n) : 0;
        });
        auto pre = wave_excl_scan(nc);
        const int tot = wave_sum(nc);
        wave_for(m, [&](int k) MT_LAM {
            const int n = own(nc, k);
            if (!n) return;
            const int o = wp + own(pre, k);
            e.pset[base + k].pad[1] = o;
            const MtQ16* src = (const MtQ16*)(e.pset + base + k);
            MtQ16* d = (MtQ16*)(ps + o);
            for (int q = 0; q < n * (int)(sizeof(MtPSet) / 16); q++) d[q] = src[q];
        });
        wp += tot;
    }
    wave_sync();
    wave_for(1, [&](int) MT_LAM { ((MtDocHdr*)dst)->psetTop = wp; });   // the staged maps' count
    uint16_t* text = (uint16_t*)(ps + wp);
    int w = 0;
    for (int base = 0; base < rowTop; base += MT_WAVE) {
        const int m = (rowTop - base) < MT_WAVE ? (rowTop - base) : MT_WAVE;
        auto ln = wave_map(m, [&](int k) MT_LAM {
            const int s = base + k;
            return (e.R[s].parent >= 0 && !(e.R[s].meta & MT_M_MARKER)) ? e.R[s].len : 0;
        });
        auto pre = wave_excl_scan(ln);
        const int tot = wave_sum(ln);
        wave_for(m, [&](int k) MT_LAM {
            const int s = base + k, l = own(ln, k);
            MtRow r = e.R[s];
            if (l > 0) {
                const int o = w + own(pre, k);
                lane_copy16(text + o, e.text + r.toff, l);
                r.toff = o; r.tcap = l;
            }
            r.props = (r.parent >= 0 && r.props >= 0) ? e.pset[r.props].pad[1] : -1;
            rows[s] = r;
        });
        w += tot;
    }
    {
        const int nq = blkTop * (int)(sizeof(MtBlk) / 16);
        const MtQ16* src = (const MtQ16*)e.blk; MtQ16* d = (MtQ16*)blks;
        for (int base = 0; base < nq; base += MT_WAVE) {
            const int m = (nq - base) < MT_WAVE ? (nq - base) : MT_WAVE;
            wave_for(m, [&](int k) MT_LAM { d[base + k] = src[base + k]; });
        }
    }
    wave_sync();
}

// Host view of one staged document.
struct MtStagedDoc {
    MtDocHdr hdr; const MtRow* R; const MtBlk* blk; const MtPSet* pset; const uint16_t* text;
    static MtStagedDoc at(const uint8_t* p) {
        MtStagedDoc v;
        v.hdr = *(const MtDocHdr*)p;
        v.R = (const MtRow*)(p + sizeof(MtDocHdr));
        v.blk = (const MtBlk*)(v.R + v.hdr.rowTop);
        v.pset = (const MtPSet*)(v.blk + v.hdr.blkTop);
        v.text = (const uint16_t*)(v.pset + v.hdr.psetTop);     // psetTop: rewritten to the staged count
        return v;
    }
};
