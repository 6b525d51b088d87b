// mt_core.h — per-document merge-tree replay, one 64-lane wavefront per document.
//
// Restates, for the passive-observer replay path, the reference engine
// /root/reference/packages/dds/merge-tree/src (MT/ below):
//   insertSegments/blockInsert/insertingWalk  MT/mergeTree.ts:1974-2493
//   ensureIntervalBoundary/splitAt            MT/mergeTree.ts:2260, :538-582
//   markRangeRemoved/annotateRange/nodeMap    MT/mergeTree.ts:2584-2739, :2927
//   zamboniSegments/scourNode/packParent      MT/mergeTree.ts:1262-1468
//   SegmentPropertiesManager.addProperties    MT/segmentPropertiesManager.ts:38-113
//   Client.applyMsg/updateSeqNumbers          MT/client.ts:790-850
// with the exact B-tree topology (<= 8 children, 4/4 splits, packParent
// repacking, heap-ordered zamboni) because block boundaries change both the
// insert tie-break and which segments zamboni merges.
//
// What is NOT restated: PartialSequenceLengths (MT/partialLengths.ts).  It is a
// cache of perspective lengths; here a block's length under a (refSeq, client)
// perspective is computed exactly as
//      len_obs(block) + Σ_{u in U, u under block} delta_u
// where len_obs is the observer's length (all sequenced ops applied) kept per
// block, and U is the set of collab-window rows whose visibility differs
// between the observer and the perspective (delta_u = ±len_u).  The window
// list holds every row with seq > minSeq or removedSeq > minSeq; all others are
// visible identically from every valid perspective (refSeq >= minSeq).
//
// Every function below is executed by all 64 lanes of the document's wave with
// wave-uniform control flow (see wave.h); data-parallel steps use wave_map().
#pragma once
#include "wave.h"
#include "../../include/mtgpu.h"

#define MT_MAXH 16                    // max tree height (7^16 segments)
#define MT_PSK 8                      // property keys per segment (more: PROPS_TOO_MANY)
#define MT_MAXN 8                     // MaxNodesInBlock, MT/mergeTree.ts:350
#define MT_GRAN 256                   // TextSegmentGranularity, MT/mergeTree.ts:1056
#define MT_ZMAX 2                     // zamboniSegmentsMaxCount, MT/mergeTree.ts:1058
#define MT_NOREM 0x7FFFFFFF           // removedSeq "undefined"

#define MT_M_CLIENT 0x000000FFu
#define MT_M_RCLIENT 0x0000FF00u
#define MT_M_REMOVED 0x00010000u
#define MT_M_MARKER 0x00020000u
#define MT_M_INWIN 0x00040000u

struct __attribute__((aligned(16))) MtBlk {   // one 64-byte record per B-tree block
    int c[8];        // children: segment rows (height 0) or blocks
    int len;         // observer length (cachedLength, MT/mergeTree.ts:2770-2789)
    int parent;      // parent block, -1 root; next-free link when free
    int n;           // childCount
    int height;      // 0 = children are segments
    int scour;       // needsScour: -1 undefined, 0 false, 1 true
    int pad[3];
};
struct __attribute__((aligned(16))) MtPSet {  // immutable property map (insertion order)
    uint16_t key[MT_PSK];
    int32_t val[MT_PSK];
    int32_t n;
    int32_t pad[3];
};
struct MtHeapE { int seg; int maxSeq; };     // LRUSegment, MT/mergeTree.ts:915-923
struct __attribute__((aligned(16))) MtDocHdr {
    int root, height, minSeq, curSeq, rowTop, blkTop, blkFree, heapN, winN, textTop, psetTop;
    uint32_t status;
    unsigned long long cnt[6];               // mt_doc_counters order
    int textHalf;                            // which half of the doc's text arena is live
    int pad[7];
};

struct MtState {                              // device pools, doc-major
    int* seg_len; int* seg_seq; int* seg_rseq; uint32_t* seg_meta; unsigned long long* seg_ovl;
    int* seg_toff; int* seg_props; int* seg_parent; int* seg_tcap;
    MtBlk* blk; MtHeapE* heap; int* win; int* uid; int* udelta; int* uanc;
    uint16_t* text; MtPSet* pset; MtDocHdr* hdr; int* hold;   // text: 2 halves of textCap per doc
    uint32_t rowCap, blkCap, heapCap, winCap, textCap, psetCap, holdCap, maxDocs;
    // interned op property sets (mt_prop_table)
    const uint32_t* p_off; const uint16_t* p_key; const int32_t* p_val;
    const uint8_t* p_falsy; const uint32_t* p_class; uint32_t p_nsets;
};

struct MtOps {                                // device copy of an mt_op_batch
    const uint32_t* doc_ids; const uint32_t* op_off;
    uint8_t* type; uint8_t* flags; uint16_t* client; int32_t* seq; int32_t* ref_seq; int32_t* msn;
    int32_t* pos1; int32_t* pos2; uint32_t* payload_off; uint32_t* payload_len; int32_t* prop_id;
    uint16_t* payload;
    uint32_t n_runs;
};

struct MtGen {                                // device stream generator parameters
    unsigned long long seed;
    uint32_t ops, clients, lag_max, pct_insert, pct_remove, ins_len_max, rem_len_max, n_ann_sets, pct_rewrite;
    int enabled;
};

// per-wave scratch (LDS on the device)
struct MtScratch {
    int pathB[MT_MAXH + 2], pathJ[MT_MAXH + 2];
    int fB[MT_MAXH + 2], fJ[MT_MAXH + 2], fS[MT_MAXH + 2], fE[MT_MAXH + 2], fL[MT_MAXH + 2], fD[MT_MAXH + 2];
    int hold[64];
    int lastOld, lastNew;
};

MT_INLINE int pick8(const int* c, int j) {
    int v = c[0];
#pragma unroll
    for (int i = 1; i < 8; i++) v = (j == i) ? c[i] : v;
    return v;
}
MT_INLINE bool vis_rc(int seq, uint32_t meta, int rseq, unsigned long long ovl, int r, int c) {
    const int cl = (int)(meta & MT_M_CLIENT);
    if (!(cl == c || seq <= r)) return false;
    if (meta & MT_M_REMOVED) {
        const int rc = (int)((meta & MT_M_RCLIENT) >> 8);
        if (rc == c || ((ovl >> c) & 1ull) || rseq <= r) return false;
    }
    return true;
}

struct SegF { int id, len, seq, rseq, toff, props; uint32_t meta; };
struct ChildL { int len; bool tie; };
struct WinI { int id; int delta; bool live; };

enum { MT_WALK_SPLIT = 0, MT_WALK_INSERT = 1 };
enum { MT_W_OK = 0, MT_W_NOCHANGE = 1, MT_W_FAIL = 2 };
enum { MT_MAP_REMOVE = 0, MT_MAP_ANNOTATE = 1 };

struct MtEng {
    MtState S;
    // doc-local views
    int *len, *seq, *rseq, *toff, *props, *parent, *tcap, *win, *uid, *udelta, *uanc;
    uint32_t* meta; unsigned long long* ovl; MtBlk* blk; MtHeapE* heap; uint16_t* text; MtPSet* pset;
    MtScratch* sc;
    // uniform document state (MtDocHdr)
    int root, height, minSeq, curSeq, rowTop, blkTop, blkFree, heapN, winN, textTop, psetTop;
    uint32_t status;
    unsigned long long cnt[6];
    int textHalf; size_t docIdx;
    int nU; bool uValid; int uRef, uCli;

    MT_HD void bind(const MtState& st, uint32_t d, MtScratch* scratch) {
        S = st;
        const size_t r = (size_t)d * st.rowCap;
        len = st.seg_len + r; seq = st.seg_seq + r; rseq = st.seg_rseq + r; meta = st.seg_meta + r;
        ovl = st.seg_ovl + r; toff = st.seg_toff + r; props = st.seg_props + r; parent = st.seg_parent + r;
        tcap = st.seg_tcap + r;
        blk = st.blk + (size_t)d * st.blkCap; heap = st.heap + (size_t)d * (st.heapCap + 1);
        win = st.win + (size_t)d * st.winCap; uid = st.uid + (size_t)d * st.winCap;
        udelta = st.udelta + (size_t)d * st.winCap; uanc = st.uanc + (size_t)d * st.winCap * MT_MAXH;
        pset = st.pset + (size_t)d * st.psetCap; docIdx = d;
        sc = scratch;
        const MtDocHdr& h = st.hdr[d];
        root = h.root; height = h.height; minSeq = h.minSeq; curSeq = h.curSeq; rowTop = h.rowTop;
        blkTop = h.blkTop; blkFree = h.blkFree; heapN = h.heapN; winN = h.winN; textTop = h.textTop;
        psetTop = h.psetTop; status = h.status; textHalf = h.textHalf;
        text = st.text + ((size_t)d * 2 + (size_t)textHalf) * st.textCap;
        for (int i = 0; i < 6; i++) cnt[i] = h.cnt[i];
        nU = 0; uValid = false; uRef = -1; uCli = -1;
    }
    MT_HD void store(uint32_t d) {
        MtDocHdr& h = S.hdr[d];
        h.root = root; h.height = height; h.minSeq = minSeq; h.curSeq = curSeq; h.rowTop = rowTop;
        h.blkTop = blkTop; h.blkFree = blkFree; h.heapN = heapN; h.winN = winN; h.textTop = textTop;
        h.psetTop = psetTop; h.status = status; h.textHalf = textHalf;
        for (int i = 0; i < 6; i++) h.cnt[i] = cnt[i];
    }
    // Fresh empty collaborating document: root = empty block (MergeTree ctor :1105-1108,
    // startCollaboration :1243).
    MT_HD void open() {
        root = 0; height = 0; minSeq = 0; curSeq = 0; rowTop = 0; blkTop = 1; blkFree = -1;
        heapN = 0; winN = 0; textTop = 0; psetTop = 0; status = 0; textHalf = 0;
        text = S.text + docIdx * 2 * S.textCap;
        for (int i = 0; i < 6; i++) cnt[i] = 0;
        MtBlk b{}; b.len = 0; b.parent = -1; b.n = 0; b.height = 0; b.scour = -1;
        for (int i = 0; i < 8; i++) b.c[i] = -1;
        blk[0] = b;
    }

    /* ---------------------------------------------------------- pools -- */
    MT_HD int allocRow() {
        if (rowTop >= (int)S.rowCap) { status |= MT_DS_OOM_ROWS; return -1; }
        return rowTop++;
    }
    MT_HD int allocBlock() {
        if (blkFree >= 0) { int id = blkFree; blkFree = blk[id].parent; return id; }
        if (blkTop >= (int)S.blkCap) { status |= MT_DS_OOM_BLOCKS; return -1; }
        return blkTop++;
    }
    MT_HD void freeBlock(int id) { blk[id].parent = blkFree; blk[id].n = -1; blkFree = id; }
    MT_HD void winAdd(int s) {
        if (meta[s] & MT_M_INWIN) return;
        if (winN >= (int)S.winCap) { status |= MT_DS_OOM_WINDOW; return; }
        win[winN++] = s;
        meta[s] = meta[s] | MT_M_INWIN;
    }
    MT_HD SegF loadSeg(int s) const {
        SegF f; f.id = s; f.len = len[s]; f.seq = seq[s]; f.rseq = rseq[s]; f.toff = toff[s]; f.props = props[s]; f.meta = meta[s];
        return f;
    }
    MT_HD int childObsLen(int h, int id) const {
        if (h == 0) return (meta[id] & MT_M_REMOVED) ? 0 : len[id];
        return blk[id].len;
    }
    MT_HD int sumObs(const MtBlk& b) const {
        auto v = wave_map(b.n, [&](int j) { return childObsLen(b.height, pick8(b.c, j)); });
        return wave_sum(v);
    }
    MT_HD void setChildParent(int h, int id, int p) {
        if (h == 0) parent[id] = p; else blk[id].parent = p;
    }

    /* ------------------------------------- perspective window (U set) -- */
    // Scan the window list: prune settled/unlinked rows (if prune) and collect
    // U = rows whose visibility differs between the observer and (r, c).
    MT_HD void computeU(int r, int c, bool prune) {
        int newWin = 0; nU = 0;
        for (int base = 0; base < winN; base += MT_WAVE) {
            const int m = (winN - base) < MT_WAVE ? (winN - base) : MT_WAVE;
            auto wi = wave_map(m, [&](int k) {
                WinI w; w.id = win[base + k];
                const int s = w.id;
                const uint32_t mt = meta[s];
                const bool removed = (mt & MT_M_REMOVED) != 0;
                const int sq = seq[s], rs = rseq[s];
                w.live = parent[s] >= 0 && (sq > minSeq || (removed && rs > minSeq));
                const bool vr = vis_rc(sq, mt, rs, ovl[s], r, c);
                const bool vo = !removed;
                w.delta = w.live ? ((vr ? len[s] : 0) - (vo ? len[s] : 0)) : 0;
                return w;
            });
            auto live = wave_map(m, [&](int k) { return own(wi, k).live; });
            if (prune) {
                auto rk = wave_rank(live);
                const int cntLive = wave_count(live);
                wave_for(m, [&](int k) {
                    const WinI w = own(wi, k);
                    if (w.live) win[newWin + own(rk, k)] = w.id;
                    else meta[w.id] = meta[w.id] & ~MT_M_INWIN;
                });
                newWin += cntLive;
            }
            auto du = wave_map(m, [&](int k) { return own(wi, k).delta != 0; });
            auto rk2 = wave_rank(du);
            const int cntU = wave_count(du);
            const int nu0 = nU;
            wave_for(m, [&](int k) {
                if (own(du, k)) { uid[nu0 + own(rk2, k)] = own(wi, k).id; udelta[nu0 + own(rk2, k)] = own(wi, k).delta; }
            });
            nU += cntU;
        }
        if (prune) winN = newWin;
        wave_sync();
        // ancestor chains: uanc[u*MAXH + h] = block at height h above row u
        for (int base = 0; base < nU; base += MT_WAVE) {
            const int m = (nU - base) < MT_WAVE ? (nU - base) : MT_WAVE;
            const int H = height;
            wave_for(m, [&](int k) {
                int a = parent[uid[base + k]];
                for (int h = 0; h <= H; h++) {
                    uanc[(size_t)(base + k) * MT_MAXH + h] = a;
                    a = (a >= 0) ? blk[a].parent : -1;
                }
            });
        }
        wave_sync();
        uValid = true; uRef = r; uCli = c;
    }
    MT_HD int perspectiveLength(int r, int c) {
        if (!(uValid && uRef == r && uCli == c)) computeU(r, c, false);
        int s = 0;
        for (int base = 0; base < nU; base += MT_WAVE) {
            const int m = (nU - base) < MT_WAVE ? (nU - base) : MT_WAVE;
            s += wave_sum(wave_map(m, [&](int k) { return udelta[base + k]; }));
        }
        return blk[root].len + s;
    }
    // Perspective lengths of block b's children (nodeLength, MT/mergeTree.ts:1652-1692).
    MT_HD LaneArr<ChildL> childLens(const MtBlk& b, int r, int c) {
        if (b.height == 0) {
            return wave_map(b.n, [&](int j) {
                const int s = pick8(b.c, j);
                const uint32_t mt = meta[s];
                const int rs = rseq[s];
                ChildL o;
                o.len = vis_rc(seq[s], mt, rs, ovl[s], r, c) ? len[s] : 0;
                // breakTie for a leaf at pos 0 (MT/mergeTree.ts:2270-2292): false if a
                // removal the author has seen (removedSeq <= refSeq); true otherwise
                // (every row has an assigned seq on the replay path).
                o.tie = !((mt & MT_M_REMOVED) && rs <= r);
                return o;
            });
        }
        int corr[8];
#pragma unroll
        for (int j = 0; j < 8; j++) corr[j] = 0;
        const int hc = b.height - 1;
        for (int base = 0; base < nU; base += MT_WAVE) {
            const int m = (nU - base) < MT_WAVE ? (nU - base) : MT_WAVE;
            auto mk = wave_map(m, [&](int k) {
                const int a = uanc[(size_t)(base + k) * MT_MAXH + hc];
                int idx = -1;
#pragma unroll
                for (int j = 0; j < 8; j++) if (j < b.n && a == b.c[j]) idx = j;
                return idx;
            });
            auto dk = wave_map(m, [&](int k) { return udelta[base + k]; });
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (j < b.n) corr[j] += wave_sum(wave_map(m, [&](int k) { return own(mk, k) == j ? own(dk, k) : 0; }));
            }
        }
        return wave_map(b.n, [&](int j) {
            ChildL o; o.len = blk[pick8(b.c, j)].len + pick8(corr, j); o.tie = true; return o;
        });
    }

    /* ----------------------------------------------- structure edits -- */
    // Row split (BaseSegment.splitAt MT/mergeTree.ts:538-582; TextSegment
    // createSplitSegmentAt textSegment.ts:103-111): the right half copies every
    // attribute; the property map is immutable here, so both halves share it.
    MT_HD int splitRow(int s, int pos) {
        const int n = allocRow();
        if (n < 0) return -1;
        len[n] = len[s] - pos; len[s] = pos;
        seq[n] = seq[s]; rseq[n] = rseq[s]; meta[n] = meta[s] & ~MT_M_INWIN; ovl[n] = ovl[s];
        toff[n] = toff[s] + pos; props[n] = props[s]; parent[n] = parent[s];
        tcap[n] = tcap[s] - pos; tcap[s] = pos;   // each row owns [toff, toff+tcap) of the arena
        if (meta[s] & MT_M_INWIN) winAdd(n);
        return n;
    }
    // Insert `node` at child index idx of path level L, splitting full blocks
    // 4/4 upward (insertingWalk :2465-2489, split :2495-2508, updateRoot :1868).
    // `delta` = observer length added under the path (0 for a row split).
    MT_HD void insertAtPath(int L, int idx, int node, int delta) {
        for (;;) {
            const int B = sc->pathB[L];
            MtBlk b = blk[B];
            int nc[8];
#pragma unroll
            for (int i = 0; i < 8; i++) nc[i] = (i < idx) ? b.c[i] : ((i == idx) ? node : (i >= 1 ? b.c[i - 1] : -1));
            const int n1 = b.n + 1;
            setChildParent(b.height, node, B);
            if (n1 < MT_MAXN) {
#pragma unroll
                for (int i = 0; i < 8; i++) b.c[i] = (i < n1) ? nc[i] : -1;
                b.n = n1; b.len += delta;
                blk[B] = b;
                for (int l = L - 1; l >= 0; l--) blk[sc->pathB[l]].len += delta;
                return;
            }
            const int NB = allocBlock();
            if (NB < 0) return;
            MtBlk nb{};
#pragma unroll
            for (int i = 0; i < 8; i++) { nb.c[i] = (i < 4) ? nc[i + 4] : -1; b.c[i] = (i < 4) ? nc[i] : -1; }
            nb.n = 4; nb.height = b.height; nb.scour = -1; nb.parent = b.parent;
            b.n = 4;
            for (int i = 0; i < 4; i++) setChildParent(b.height, nb.c[i], NB);
            wave_sync();
            nb.len = sumObs(nb);
            b.len = sumObs(b);
            blk[NB] = nb;
            if (L == 0) {
                const int R = allocBlock();
                if (R < 0) { blk[B] = b; return; }
                MtBlk rb{};
                rb.c[0] = B; rb.c[1] = NB;
                for (int i = 2; i < 8; i++) rb.c[i] = -1;
                rb.n = 2; rb.height = b.height + 1; rb.parent = -1; rb.scour = -1; rb.len = b.len + nb.len;
                b.parent = R; blk[NB].parent = R;
                blk[B] = b; blk[R] = rb;
                root = R; height = rb.height;
                return;
            }
            blk[B] = b;
            node = NB; idx = sc->pathJ[L - 1] + 1; L = L - 1;
        }
    }
    // insertingWalk (MT/mergeTree.ts:2363-2493) for one remote op perspective.
    MT_HD int walk(int kind, int pos, int r, int c, int cand, int candLen) {
        if (!(uValid && uRef == r && uCli == c)) computeU(r, c, false);
        int B = root, L = 0, p = pos;
        for (;;) {
            const MtBlk b = blk[B];
            sc->pathB[L] = B;
            auto ch = childLens(b, r, c);
            auto lens = wave_map(b.n, [&](int j) { return own(ch, j).len; });
            auto pre = wave_excl_scan(lens);
            const int total = wave_sum(lens);
            const bool interior = b.height > 0;
            auto cond = wave_map(b.n, [&](int j) {
                const int pj = p - own(pre, j), lj = own(ch, j).len;
                if (interior) return pj <= lj;                       // breakTie: blocks always
                return pj < lj || (pj == lj && pj == 0 && own(ch, j).tie);
            });
            const int j = wave_first(cond);
            if (j >= 0) {
                const int pj = p - wave_at(pre, j);
                if (interior) { sc->pathJ[L] = j; L++; B = pick8(b.c, j); p = pj; continue; }
                const int s = pick8(b.c, j);
                if (kind == MT_WALK_SPLIT) {
                    if (pj > 0 && !(meta[s] & MT_M_MARKER)) {
                        const int n = splitRow(s, pj);
                        if (n < 0) return MT_W_FAIL;
                        insertAtPath(L, j + 1, n, 0);
                        uValid = false;
                        return MT_W_OK;
                    }
                    return MT_W_NOCHANGE;
                }
                insertAtPath(L, j, cand, candLen);           // onLeaf: candidate goes before the found row
                uValid = false;
                return MT_W_OK;
            }
            if (p - total == 0) {
                if (kind == MT_WALK_SPLIT) return MT_W_NOCHANGE;
                insertAtPath(L, b.n, cand, candLen);          // position used up at a block end: append
                uValid = false;
                return MT_W_OK;
            }
            return MT_W_FAIL;
        }
    }

    /* --------------------------------------------------------- zamboni -- */
    MT_HD void heapAdd(int s, int ms) {                       // Heap.add + fixup, collections.ts:238-251
        if (heapN + 1 > (int)S.heapCap) { status |= MT_DS_OOM_HEAP; return; }
        int k = ++heapN;
        while (k > 1) {
            const MtHeapE pe = heap[k >> 1];
            if (pe.maxSeq > ms) { heap[k] = pe; k >>= 1; } else break;
        }
        MtHeapE e; e.seg = s; e.maxSeq = ms; heap[k] = e;
    }
    MT_HD MtHeapE heapGet() {                                 // Heap.get + fixdown, collections.ts:230-268
        const MtHeapE x = heap[1];
        const MtHeapE last = heap[heapN];
        heapN--;
        if (heapN >= 1) {
            int k = 1;
            while ((k << 1) <= heapN) {
                int j = k << 1;
                MtHeapE hj = heap[j];
                if (j < heapN) { const MtHeapE hj1 = heap[j + 1]; if (hj.maxSeq > hj1.maxSeq) { j++; hj = hj1; } }
                if (last.maxSeq <= hj.maxSeq) break;
                heap[k] = hj; k = j;
            }
            heap[k] = last;
        }
        return x;
    }
    MT_HD void addToLRUSet(int s, int sq) {                   // MT/mergeTree.ts:1262-1272
        const int p = parent[s];
        if (blk[p].scour != 1 && sq > curSeq) { blk[p].scour = 1; heapAdd(s, sq); }
    }
    MT_HD bool propsMatch(int a, int b) {                      // matchProperties, MT/properties.ts:64-95
        if (a == b) return true;
        if (a < 0 || b < 0) return false;
        const int na = pset[a].n, nb = pset[b].n;
        if (na != nb) return false;
        auto ok = wave_map(na, [&](int k) {
            const uint16_t key = pset[a].key[k];
            const uint32_t ca = S.p_class[pset[a].val[k]];
            bool f = false;
            for (int i = 0; i < nb; i++) if (pset[b].key[i] == key && S.p_class[pset[b].val[i]] == ca) f = true;
            return f;
        });
        return wave_count(ok) == na;
    }
    MT_HD void copyText(int dst, int src, int n) {
        for (int base = 0; base < n; base += MT_WAVE) {
            const int m = (n - base) < MT_WAVE ? (n - base) : MT_WAVE;
            auto v = wave_map(m, [&](int k) { return (int)text[src + base + k]; });
            wave_sync();
            wave_for(m, [&](int k) { text[dst + base + k] = (uint16_t)own(v, k); });
        }
        wave_sync();
    }
    // Text-arena compaction: copy the text of every linked row into the other
    // half of the document's arena (rows are immutable slices, so garbage from
    // relocated or unlinked rows accumulates until the half is full).
    MT_HD void textGC() {
        const int other = textHalf ^ 1;
        uint16_t* dst = S.text + (docIdx * 2 + (size_t)other) * S.textCap;
        int w = 0;
        for (int base = 0; base < rowTop; base += MT_WAVE) {
            const int m = (rowTop - base) < MT_WAVE ? (rowTop - base) : MT_WAVE;
            auto ln = wave_map(m, [&](int k) {
                const int s = base + k;
                return (parent[s] >= 0 && !(meta[s] & MT_M_MARKER)) ? len[s] : 0;
            });
            auto pre = wave_excl_scan(ln);
            const int tot = wave_sum(ln);
            wave_for(m, [&](int k) {
                const int s = base + k, l = own(ln, k);
                if (l <= 0) return;
                const int o = w + own(pre, k), t0 = toff[s];
                for (int q = 0; q < l; q++) dst[o + q] = text[t0 + q];
                toff[s] = o; tcap[s] = l;
            });
            w += tot;
        }
        wave_sync();
        textHalf = other; text = dst; textTop = w;
    }
    // Reserve n units at the top of the live half (compacting first if needed).
    MT_HD int textAlloc(int n) {
        if (textTop + n > (int)S.textCap) textGC();
        if (textTop + n > (int)S.textCap) { status |= MT_DS_OOM_TEXT; return -1; }
        const int o = textTop; textTop += n; return o;
    }
    // TextSegment.append (textSegment.ts:74-85) on the arena.  A row owns
    // [toff, toff + tcap); appends fill owned space, else the row moves to a new
    // region of twice the size (amortized O(appended chars)).
    MT_HD void appendText(int pv, int s) {
        const int lp = len[pv], ls = len[s];
        if (toff[s] == toff[pv] + lp && tcap[pv] == lp) { len[pv] = lp + ls; tcap[pv] = lp + tcap[s]; return; }
        if (lp + ls <= tcap[pv]) { copyText(toff[pv] + lp, toff[s], ls); len[pv] = lp + ls; return; }
        int nc = 2 * (lp + ls); if (nc < 16) nc = 16;
        if (textTop + nc > (int)S.textCap) { textGC(); nc = lp + ls; }
        const int o = textAlloc(nc);
        if (o < 0) return;
        copyText(o, toff[pv], lp); copyText(o + lp, toff[s], ls);
        toff[pv] = o; tcap[pv] = nc; len[pv] = lp + ls;
    }
    // scourNode for a block of rows (MT/mergeTree.ts:1278-1356); kept children
    // are appended to sc->hold[*nh].
    MT_HD void scourLeaf(const MtBlk& b, int* nh) {
        auto f = wave_map(b.n, [&](int j) { return pick8(b.c, j); });
        int prev = -1, prevLen = 0, prevToff = 0, prevProps = -1; bool prevMarker = false;
        for (int k = 0; k < b.n; k++) {
            const int s = wave_at(f, k);
            const uint32_t mt = meta[s];
            cnt[5]++;
            if (mt & MT_M_REMOVED) {
                if (rseq[s] > minSeq) sc->hold[(*nh)++] = s;
                else parent[s] = -1;                               // UNLINK
                prev = -1;
            } else if (seq[s] <= minSeq) {
                const int ls = len[s];
                bool can = prev >= 0 && !prevMarker && !(mt & MT_M_MARKER) &&
                           text[prevToff + prevLen - 1] != (uint16_t)'\n' &&
                           (prevLen <= MT_GRAN || ls <= MT_GRAN) && ls > 0;
                if (can) can = propsMatch(prevProps, props[s]);
                if (can) {
                    appendText(prev, s);
                    parent[s] = -1;
                    prevLen = len[prev]; prevToff = toff[prev];
                } else {
                    sc->hold[(*nh)++] = s;
                    prev = (ls > 0) ? s : -1;
                    prevLen = ls; prevToff = toff[s]; prevProps = props[s]; prevMarker = (mt & MT_M_MARKER) != 0;
                }
            } else {
                sc->hold[(*nh)++] = s;
                prev = -1;
            }
        }
        wave_sync();
    }
    MT_HD void updatePathLens(int B) {                        // blockUpdatePathLengths(..., newStructure)
        while (B >= 0) {
            MtBlk b = blk[B];
            const int l = sumObs(b);
            blk[B].len = l;
            B = b.parent;
        }
    }
    MT_HD void packParent(int P) {                            // MT/mergeTree.ts:1359-1410
        for (;;) {
            MtBlk pb = blk[P];
            int nh = 0; int ch = 0;
            for (int i = 0; i < pb.n; i++) {
                const int cb = pick8(pb.c, i);
                const MtBlk cbk = blk[cb];
                ch = cbk.height;
                if (cbk.height == 0) scourLeaf(cbk, &nh);
                else for (int k = 0; k < cbk.n; k++) sc->hold[nh++] = pick8(cbk.c, k);
                freeBlock(cb);
            }
            int cc = nh / (MT_MAXN / 2); if (cc > MT_MAXN - 1) cc = MT_MAXN - 1; if (cc < 1) cc = 1;
            const int base = nh / cc; int extra = nh % cc; int rd = 0;
            int packed[8];
#pragma unroll
            for (int i = 0; i < 8; i++) packed[i] = -1;
            for (int ni = 0; ni < cc; ni++) {
                int cntc = base; if (extra > 0) { cntc++; extra--; }
                const int NB = allocBlock();
                if (NB < 0) return;
                MtBlk nb{};
                for (int i = 0; i < 8; i++) nb.c[i] = -1;
                for (int i = 0; i < cntc; i++) { nb.c[i] = sc->hold[rd + i]; setChildParent(ch, sc->hold[rd + i], NB); }
                rd += cntc;
                nb.n = cntc; nb.height = ch; nb.parent = P; nb.scour = -1;
                wave_sync();
                nb.len = sumObs(nb);
                blk[NB] = nb;
                for (int i = 0; i < 8; i++) if (i == ni) packed[i] = NB;
            }
#pragma unroll
            for (int i = 0; i < 8; i++) pb.c[i] = packed[i];
            pb.n = cc;
            blk[P] = pb;
            if (cc < MT_MAXN / 2 && pb.parent >= 0) { P = pb.parent; continue; }
            updatePathLens(P);
            return;
        }
    }
    MT_HD void zamboni() {                                    // MT/mergeTree.ts:1412-1468
        uValid = false;
        for (int i = 0; i < MT_ZMAX; i++) {
            if (heapN == 0 || heap[1].maxSeq > minSeq) break;
            const MtHeapE e = heapGet();
            const int p = parent[e.seg];
            if (p >= 0 && blk[p].scour != 0) {
                MtBlk b = blk[p];
                int nh = 0;
                scourLeaf(b, &nh);
                blk[p].scour = 0;
                if (nh < b.n) {
                    for (int j = 0; j < 8; j++) b.c[j] = (j < nh) ? sc->hold[j] : -1;
                    b.n = nh; b.scour = 0;
                    blk[p] = b;
                    if (nh < MT_MAXN / 2 && b.parent >= 0) packParent(b.parent);
                    else updatePathLens(p);
                }
            }
            if (status) return;
        }
    }
    MT_HD void setMinSeq(int ms) {                            // MT/mergeTree.ts:1712-1725
        if (ms > curSeq || minSeq > ms) { status |= MT_DS_ASSERT_MSN; return; }
        if (ms > minSeq) { minSeq = ms; uValid = false; zamboni(); }
    }

    /* ------------------------------------------------------ properties -- */
    // New property map = (old map or {}) updated by an op's prop set, the
    // remote addProperties rules (segmentPropertiesManager.ts:43-110): rewrite
    // first deletes keys whose new value is falsy or absent; then each key in
    // Object.keys order is deleted (null) or set (existing keys keep position).
    MT_HD int applyPropSet(int old, int opset, bool rewrite) {
        if (opset < 0 || opset >= (int)S.p_nsets) { status |= MT_DS_UNSUPPORTED; return old; }
        if (psetTop >= (int)S.psetCap) { status |= MT_DS_OOM_PROPS; return old; }
        const int id = psetTop++;
        int n = 0;
        uint16_t k[MT_PSK]; int32_t v[MT_PSK];
        for (int i = 0; i < MT_PSK; i++) { k[i] = 0; v[i] = 0; }
        if (old >= 0) {
            n = pset[old].n;
            for (int i = 0; i < MT_PSK; i++) { k[i] = pset[old].key[i]; v[i] = pset[old].val[i]; }
        }
        const uint32_t o0 = S.p_off[opset], o1 = S.p_off[opset + 1];
        if (rewrite) {
            int w = 0;
            for (int i = 0; i < MT_PSK; i++) {
                if (i >= n) break;
                bool keep = false;
                for (uint32_t q = o0; q < o1; q++) if (S.p_key[q] == k[i]) { const int32_t nv = S.p_val[q]; keep = nv >= 0 && !S.p_falsy[nv]; }
                if (keep) { k[w] = k[i]; v[w] = v[i]; w++; }
            }
            n = w;
        }
        for (uint32_t q = o0; q < o1; q++) {
            const uint16_t key = S.p_key[q]; const int32_t nv = S.p_val[q];
            int at = -1;
            for (int i = 0; i < MT_PSK; i++) if (i < n && k[i] == key) at = i;
            if (nv < 0) {
                if (at >= 0) { for (int i = at; i + 1 < MT_PSK; i++) if (i + 1 < n) { k[i] = k[i + 1]; v[i] = v[i + 1]; } n--; }
            } else if (at >= 0) v[at] = nv;
            else {
                if (n >= MT_PSK) { status |= MT_DS_PROPS_TOO_MANY; psetTop--; return old; }
                k[n] = key; v[n] = nv; n++;
            }
        }
        MtPSet ps;
        for (int i = 0; i < MT_PSK; i++) { ps.key[i] = k[i]; ps.val[i] = v[i]; }
        ps.n = n; ps.pad[0] = ps.pad[1] = ps.pad[2] = 0;
        pset[id] = ps;
        return id;
    }

    /* ----------------------------------------------------- range walks -- */
    // nodeMap over [start, end) under (r, c) with the remove / annotate leaf
    // action and post-order length maintenance (MT/mergeTree.ts:2626-2739,
    // :2584-2624, :2927-2994).  Child lengths are evaluated before the child is
    // touched, as in the reference's in-order traversal.
    MT_HD void rangeMap(int mode, int start, int end, int r, int c, int sq, int opset, bool rewrite) {
        if (!(uValid && uRef == r && uCli == c)) computeU(r, c, false);
        int L = 0;
        sc->fB[0] = root; sc->fJ[0] = 0; sc->fS[0] = start; sc->fE[0] = end; sc->fD[0] = 0;
        sc->lastOld = -2; sc->lastNew = -1;
        while (L >= 0) {
            const int B = sc->fB[L];
            const MtBlk b = blk[B];
            auto ch = childLens(b, r, c);
            auto lens = wave_map(b.n, [&](int j) { return own(ch, j).len; });
            const int j0 = sc->fJ[L];
            auto lensFrom = wave_map(b.n, [&](int j) { return j >= j0 ? own(lens, j) : 0; });
            auto pre = wave_excl_scan(lensFrom);
            const int st = sc->fS[L], en = sc->fE[L];
            auto cond = wave_map(b.n, [&](int j) {
                const int lj = own(lens, j), pj = own(pre, j);
                return j >= j0 && (en - pj) > 0 && lj > 0 && (st - pj) < lj;
            });
            if (b.height == 0) {
                const int first = wave_first(cond);
                int obsDelta = 0;
                if (first >= 0) {
                    if (mode == MT_MAP_REMOVE) {
                        auto nd = wave_map(b.n, [&](int j) {
                            if (!own(cond, j)) return 0;
                            const int s = pick8(b.c, j);
                            const uint32_t mt = meta[s];
                            if (mt & MT_M_REMOVED) {                   // overlapping remove: keep first remover
                                ovl[s] = ovl[s] | (1ull << c);
                                return 0;
                            }
                            meta[s] = (mt & ~MT_M_RCLIENT) | MT_M_REMOVED | ((uint32_t)c << 8);
                            rseq[s] = sq;
                            return len[s];
                        });
                        obsDelta = -wave_sum(nd);
                        cnt[3] += 2ull * (uint64_t)wave_count(cond);
                        wave_sync();
                        for (int j = 0; j < b.n; j++) if (wave_at(cond, j)) winAdd(pick8(b.c, j));
                    } else {
                        cnt[3] += 2ull * (uint64_t)wave_count(cond);
                        for (int j = 0; j < b.n; j++) {
                            if (!wave_at(cond, j)) continue;
                            const int s = pick8(b.c, j);
                            const int old = props[s];
                            int nw;
                            if (old == sc->lastOld) nw = sc->lastNew;
                            else { nw = applyPropSet(old, opset, rewrite); sc->lastOld = old; sc->lastNew = nw; }
                            props[s] = nw;
                        }
                    }
                    addToLRUSet(pick8(b.c, first), sq);
                }
                if (mode == MT_MAP_REMOVE) blk[B].len = b.len + obsDelta;
                sc->fD[L] += obsDelta;
                // pop
                const int d = sc->fD[L];
                L--;
                if (L >= 0) { sc->fD[L] += d; sc->fS[L] -= sc->fL[L]; sc->fE[L] -= sc->fL[L]; sc->fJ[L] += 1; }
                continue;
            }
            const int jj = wave_first(cond);
            if (jj >= 0) {
                const int pj = wave_at(pre, jj);
                sc->fS[L] = st - pj; sc->fE[L] = en - pj; sc->fJ[L] = jj; sc->fL[L] = wave_at(lens, jj);
                const int child = pick8(b.c, jj);
                L++;
                sc->fB[L] = child; sc->fJ[L] = 0; sc->fS[L] = sc->fS[L - 1]; sc->fE[L] = sc->fE[L - 1]; sc->fD[L] = 0;
                continue;
            }
            const int d = sc->fD[L];
            if (d != 0) blk[B].len = b.len + d;
            L--;
            if (L >= 0) { sc->fD[L] += d; sc->fS[L] -= sc->fL[L]; sc->fE[L] -= sc->fL[L]; sc->fJ[L] += 1; }
        }
        uValid = false;
    }

    /* -------------------------------------------------------- op apply -- */
    MT_HD void opInsert(int pos, int r, int c, int sq, const uint16_t* src, int plen, bool marker, int refType, int segProps) {
        // MergeTree.insertSegments (MT/mergeTree.ts:1974-2011)
        int w = walk(MT_WALK_SPLIT, pos, r, c, -1, 0);
        if (w == MT_W_OK) cnt[3] += 2;
        if (status) return;
        const int L = marker ? 1 : plen;
        if (L > 0) {
            const int n = allocRow();
            if (n < 0) return;
            len[n] = L; seq[n] = sq; rseq[n] = MT_NOREM;
            meta[n] = (uint32_t)c | (marker ? MT_M_MARKER : 0u);
            ovl[n] = 0ull; parent[n] = -1;
            props[n] = segProps >= 0 ? applyPropSet(-1, segProps, false) : -1;
            tcap[n] = marker ? 0 : plen;
            if (marker) toff[n] = refType;
            else {
                parent[n] = -1;                                  // not yet linked: excluded from compaction
                const int t0 = textAlloc(plen);
                if (t0 < 0) return;
                toff[n] = t0;
                for (int base = 0; base < plen; base += MT_WAVE) {
                    const int m = (plen - base) < MT_WAVE ? (plen - base) : MT_WAVE;
                    wave_for(m, [&](int k) { text[t0 + base + k] = src[base + k]; });
                }
                cnt[2] += (uint64_t)plen;
            }
            wave_sync();
            w = walk(MT_WALK_INSERT, pos, r, c, n, L);
            if (w != MT_W_OK || parent[n] < 0) { status |= MT_DS_INSERT_FAILED; return; }
            cnt[3] += 2;
            winAdd(n);
            if (sq > minSeq) addToLRUSet(n, sq);
        }
        zamboni();
    }
    MT_HD void opRange(int mode, int start, int end, int r, int c, int sq, int opset, bool rewrite) {
        int w = walk(MT_WALK_SPLIT, start, r, c, -1, 0);
        if (w == MT_W_OK) cnt[3] += 2;
        if (status) return;
        w = walk(MT_WALK_SPLIT, end, r, c, -1, 0);
        if (w == MT_W_OK) cnt[3] += 2;
        if (status) return;
        rangeMap(mode, start, end, r, c, sq, opset, rewrite);
        if (status) return;
        zamboni();
    }
};
