// mt_pack.h — gather documents' live state into one contiguous staging buffer
// (device side of mt_snapshot_v1 / mt_snapshot_digests / mt_get_text for many
// documents: one download instead of four copies per document).
//
// Per document, at staging offset off[i] (16-byte aligned):
//   MtDocHdr | rows[0, rowTop) | blocks[0, blkTop) | psets[0, psetTop) | live text
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

template <class Eng>
MT_HD MtPackSize mt_pack_size(Eng& e) {
    MtPackSize z; z.rows = (uint32_t)e.rowTop; z.blks = (uint32_t)e.blkTop; z.psets = (uint32_t)e.psetTop;
    int t = 0;
    for (int base = 0; base < e.rowTop; base += MT_WAVE) {
        const int m = (e.rowTop - base) < MT_WAVE ? (e.rowTop - base) : MT_WAVE;
        t += wave_sum(wave_map(m, [&](int k) MT_LAM {
            const int s = base + k;
            return (e.R[s].parent >= 0 && !(e.R[s].meta & MT_M_MARKER)) ? e.R[s].len : 0;
        }));
    }
    z.text = (uint32_t)t;
    return z;
}

template <class Eng>
MT_HD void mt_pack_doc(Eng& e, uint8_t* dst) {
    const int rowTop = e.rowTop, blkTop = e.blkTop, psetTop = e.psetTop;
    MtRow* rows = (MtRow*)(dst + sizeof(MtDocHdr));
    MtBlk* blks = (MtBlk*)(rows + rowTop);
    MtPSet* ps = (MtPSet*)(blks + blkTop);
    uint16_t* text = (uint16_t*)(ps + psetTop);
    {   // header
        const int* src = (const int*)e.hdrp;
        int* d = (int*)dst;
        wave_for((int)(sizeof(MtDocHdr) / 4), [&](int k) MT_LAM { d[k] = src[k]; });
    }
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
    {
        const int nq = psetTop * (int)(sizeof(MtPSet) / 16);
        const MtQ16* src = (const MtQ16*)e.pset; MtQ16* d = (MtQ16*)ps;
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
        v.text = (const uint16_t*)(v.pset + v.hdr.psetTop);
        return v;
    }
};
