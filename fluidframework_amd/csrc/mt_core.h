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
#include <type_traits>
#include "wave.h"
#include "../../include/mtgpu.h"

#define MT_MAXH 16                    // max tree height (7^16 segments)
#define MT_PSK 16                     // property keys per MtPSet chunk
#define MT_PKEYS MT_MAX_PROP_KEYS      // keys of one property map (more: PROPS_TOO_MANY); up to a
                                      // wave's 64 one per lane, past that in the pool (applyPropSetWide)
#ifndef MT_PATH_RESUME
#define MT_PATH_RESUME 1              // opRange: end walk and range walk start below the root
#endif
#define MT_MAXN 8                     // MaxNodesInBlock, MT/mergeTree.ts:350
#define MT_GRAN 256                   // TextSegmentGranularity, MT/mergeTree.ts:1056
#define MT_ZMAX 2                     // zamboniSegmentsMaxCount, MT/mergeTree.ts:1058
#define MT_NOREM 0x7FFFFFFF           // removedSeq "undefined"
#define MT_RFL 128                    // recycled-row stack per document (LDS while a run executes)
// LDS-resident pools (mt_replay_lds_kernel): a document whose rows, blocks, heap
// and window fit runs entirely out of LDS; one that outgrows them mid-run is
// written back to HBM and finished by the HBM-pool kernel (exact resume).
#ifndef MT_L_ROWS
#define MT_L_ROWS 256                 // rows (and window / U-set entries)
#endif
#ifndef MT_L_BLKS
#define MT_L_BLKS 96                  // blocks (ids < 255: ancestor chains are bytes)
#endif
#ifndef MT_L_HEAP
#define MT_L_HEAP 96                  // zamboni heap entries
#endif
#define MT_L_H 8                      // ancestor-chain levels (tree height < MT_L_H - 2)
// Block residency (mt_replay_blk_kernel): only blocks and the zamboni heap move to
// LDS (rows, window and U set stay in HBM), small enough for 4 waves per SIMD.
#ifndef MT_B_BLKS
#define MT_B_BLKS 104
#endif
#ifndef MT_B_SLACK
#define MT_B_SLACK 13                 // block residency: free blocks kept beyond 2 * height before each message
#endif
#define MT_B_BT 128                   // corrections-table slots (block ids < MT_B_BLKS)
#ifndef MT_B_W
#define MT_B_W 64                     // window entries kept in LDS (the rest, if any, in HBM)
#endif
#ifndef MT_B_HEAP
#define MT_B_HEAP 94
#endif
// Wide block residency (mt_replay_blkw_kernel, MT_RES_BLKW): the same engine with room for
// the trees and heaps of long documents (~21 KB of LDS per workgroup), run for the size class
// of long runs (mt_set_size_class) beside the block-residency kernel for the rest.
#ifndef MT_BW_BLKS
#define MT_BW_BLKS 248
#endif
#ifndef MT_BW_W
#define MT_BW_W 256                   // window entries in LDS (long documents of many clients hold
#endif                                // windows of ~75 entries at 16 clients)
#ifndef MT_BW_HEAP
#define MT_BW_HEAP 254
#endif
#define MT_BW_BT 256
// Long-document residency (mt_replay_big_kernel): a document whose blocks cannot fit
// LDS (config 4: ~50k blocks) keeps its zamboni heap, collab window and the first
// MT_G_U U-set entries with their ancestor chains in LDS (~68 KB: two documents per CU),
// rows and blocks in HBM.  Meant for launches with few documents per CU.
#ifndef MT_G_U
#define MT_G_U 768
#endif
#ifndef MT_G_HEAP
#define MT_G_HEAP 2046
#endif
#ifndef MT_G_WIN
#define MT_G_WIN 2048
#endif
#define MT_G_H 12                     // ancestor-chain levels kept per U entry (tree height < MT_G_H - 2)
// Long-document residency also keeps an LDS block cache: MT_G_BC direct-mapped slots (slot =
// block id mod MT_G_BC), write-back, filled by the descents with blocks of height >= MT_G_BCH.
// A slot holding a higher block is not taken by a lower one, so the top of the tree stays
// resident and the descents, ancestor chains and path updates reach HBM only near the leaves.
// Compiled in with -DMT_G_BCACHE=1 only: measured -1 % on config 4 (upper levels already hit
// L2, and every block access then pays a tag check and flat addressing).
#ifndef MT_G_BCACHE
#define MT_G_BCACHE 0
#endif
#ifndef MT_G_BC
#define MT_G_BC (MT_G_BCACHE ? 512 : 1)
#endif
#ifndef MT_G_BCH
#define MT_G_BCH 1
#endif
#define MT_BC_EMPTY ((int)0x80000000)
// ... and runs as a workgroup of MT_G_NW waves: wave 0 applies the ops; the others take
// shares of computeU's window scan (MT_G_STG window entries staged in LDS per round) and of
// its ancestor-chain walks (mwRun / mwShare; the host emulation runs every share in turn).
#ifndef MT_G_NW
#define MT_G_NW 4
#endif
#define MT_G_STG 1024
#ifndef MT_G_MWMIN
#define MT_G_MWMIN 512                 // windows up to this many entries are scanned by wave 0 alone
#endif
#ifndef MT_G_ALLCH
#define MT_G_ALLCH 0                   // 1: ... with every chunk's rows loaded in one round trip
#endif
enum { MT_MW_EXIT = 0, MT_MW_SCAN = 1, MT_MW_CHAIN = 2, MT_MW_PREFETCH = 3 };
// Jobs alternate between two LDS slots, so wave 0 can post an asynchronous job (PREFETCH: no
// completion barrier) and write the next one while helpers still read the last.
// Runtime switches of the long-document residency (mt_set_residency(ctx, 3, rows, flags, heap)):
enum { MT_BIGF_NO_BCACHE = 1, MT_BIGF_NO_PREFETCH = 2, MT_BIGF_NO_TABLE = 4, MT_BIGF_NO_BPC = 8 };
// Per-block perspective corrections of the long-document residency: an LDS hash table
// block id -> Σ delta of the U rows under the block, built bottom-up once per U set (each
// distinct block's parent is loaded once), so a descent level looks its children up instead
// of scanning U.  Up to MT_G_HTN distinct blocks (load <= 3/4); beyond that computeU falls
// back to per-entry ancestor chains.
#ifndef MT_G_HT
#define MT_G_HT 4096
#endif
// Parent cache of the long-document residency: block id -> parent in LDS, direct-mapped, one
// dword per entry (tag = id >> MT_G_BPL in bits 20..31, parent + 1 in bits 0..19), so htBuild's
// bottom-up passes read the parents of the blocks it saw for the last U sets from LDS instead
// of HBM.  Every write of a block's parent field updates it (bpPut / bpDrop); documents with
// 2^20 blocks or more run without it.
#ifndef MT_G_BPC
#define MT_G_BPC 1
#endif
#define MT_G_BPL 11
#define MT_G_BP (1 << MT_G_BPL)
#define MT_BP_EMPTY 0xFFFFFFFFu
#define MT_G_HTN (MT_G_HT * 3 / 4)
enum { MT_RES_HBM = 0, MT_RES_LDS = 1, MT_RES_BLK = 2, MT_RES_BIG = 3, MT_RES_BLKW = 4 };
// Diagnostic builds keep per-document phase/event counters (prof[]) across binds;
// product builds never load or store them (8 SGPR pairs fewer live in the replay loop).
#if defined(MT_PROFILE) || defined(MT_PROFILE2) || defined(MT_PROFILE3) || defined(MT_PROFILE4) || defined(MT_BPC_STATS) || defined(MT_EVCOUNT3) || defined(MT_EVCOUNT) || defined(MT_EVCOUNT2)
#define MT_KEEP_PROF 1
#else
#define MT_KEEP_PROF 0
#endif

// Phase profiling (diagnostic builds only, -DMT_PROFILE): shader-clock cycles
// accumulated per phase into MtDocHdr.prof; never compiled into the product.
#if defined(MT_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
#define MT_PB(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define MT_PE(i, v) prof[i] += __builtin_amdgcn_s_memtime() - (v)
#else
#define MT_PB(v)
#define MT_PE(i, v)
#endif
// Event counters (host-emulation diagnostic builds only, -DMT_EVCOUNT): reuse prof[].
#if defined(MT_EVCOUNT)
#define MT_EV(i, v) prof[i] += (unsigned long long)(v)
#else
#define MT_EV(i, v)
#endif
// Second event set (host-emulation diagnostic builds only, -DMT_EVCOUNT2): 0 packParent,
// 1 updatePathLens levels, 2 copyText units, 3 copyText calls, 4 textGC, 5 splitRow,
// 6 zamboni calls that popped, 7 rangeMap leaf blocks.
#if defined(MT_EVCOUNT2)
#define MT_EV2(i, v) prof[i] += (unsigned long long)(v)
#else
#define MT_EV2(i, v)
#endif
// Fine-grained latency probes (device diagnostic builds only, -DMT_PROFILE2):
// 0 walk blkLoad cyc, 1 walk childLens cyc, 2 walk levels, 3 computeU cyc,
// 4 computeU calls, 5 heapGet cyc, 6 heapGet calls, 7 scourLeaf cyc.
#if defined(MT_PROFILE2) && defined(__HIP_DEVICE_COMPILE__)
#define MT_QB(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define MT_QE(i, v) prof[i] += __builtin_amdgcn_s_memtime() - (v)
#define MT_QC(i) prof[i] += 1
#else
#define MT_QB(v)
#define MT_QE(i, v)
#define MT_QC(i)
#endif
// Zamboni breakdown probes (device diagnostic builds only, -DMT_PROFILE3): 0 zamboni
// total, 1 scourLeaf, 2 appendText, 3 packParent, 4 packParent's leaf scour, 5 heapGet,
// 6 path after scour (child rewrite + pack/update), 7 pops.
#if defined(MT_PROFILE3) && defined(__HIP_DEVICE_COMPILE__)
#define MT_ZB(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define MT_ZE(i, v) prof[i] += __builtin_amdgcn_s_memtime() - (v)
#define MT_ZC(i) prof[i] += 1
#else
#define MT_ZB(v)
#define MT_ZE(i, v)
#define MT_ZC(i)
#endif
// Parent-cache statistics (host-emulation diagnostic builds only, -DMT_BPC_STATS): 0 lookups,
// 1 hits, 2 misses on an empty slot, 3 misses on another block's entry, 4 puts over another
// block's entry, 5 drops of a live entry.
#if defined(MT_BPC_STATS) && !defined(__HIP_DEVICE_COMPILE__)
#define MT_BS(i) prof[i] += 1
#else
#define MT_BS(i)
#endif
// computeU probes of the long-document residency (device diagnostic builds only, -DMT_PROFILE4):
// 0 window scan cyc, 1 htBuild cyc, 2 htBuild levels, 3 U entries, 4 window entries, 5 calls,
// 6 parent lookups, 7 parent-cache misses.
#if defined(MT_PROFILE4) && defined(__HIP_DEVICE_COMPILE__)
#define MT_UB(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define MT_UE(i, v) prof[i] += __builtin_amdgcn_s_memtime() - (v)
#define MT_UC(i, x) prof[i] += (unsigned long long)(x)
#else
#define MT_UB(v)
#define MT_UE(i, v)
#define MT_UC(i, x)
#endif
enum { MT_PH_U = 0, MT_PH_SPLIT, MT_PH_INSERT, MT_PH_RANGE, MT_PH_ZAMBONI, MT_PH_OP, MT_PH_GEN, MT_PH_TEXT };

#define MT_M_CLIENT 0x0000FFFFu        // short client id (16 bits; MT/client.ts:658-682)
#define MT_M_REMOVED 0x00010000u
#define MT_M_MARKER 0x00020000u
#define MT_M_INWIN 0x00040000u
#define MT_M_REG 0x00080000u          // a clone held by a register (not linked; its text survives compaction)
#define MT_M_NONL 0x00100000u         // the text holds no "\n" (canAppend's trailing-newline test loads nothing)
#define MT_M_HREF1 0x01000000u        // heap-entry reference count, bits 24..31 (saturating)
#define MT_M_HREF 0xFF000000u

#ifndef MT_ROW64
#define MT_ROW64 0
#endif
struct __attribute__((aligned(16))) MtRow {   // one 48-byte record per segment row
    int len;         // cachedLength (UTF-16 units; 1 for a marker)
    int seq;         // insertion seq
    int rseq;        // removedSeq (MT_NOREM = undefined)
    uint32_t meta;   // client | removedClient<<8 | REMOVED | MARKER | INWIN
    int toff;        // text arena offset (marker: refType)
    int props;       // property-set id, -1 = properties undefined
    int parent;      // leaf block, -1 = unlinked
    int tcap;        // owned text capacity at toff
    unsigned long long ovl;  // removedClientOverlap: bit c for clients c < 63; bit 63 = more in the side list
    uint32_t rcl;            // removedClientId (16 bits)
    int mid;                 // marker: its markerId's per-document index + 1 (0: none)
#if MT_ROW64
    int pad[4];              // one row per 64-byte line (a row's update dirties one line)
#endif
};
struct __attribute__((aligned(16))) MtBlk {   // one 64-byte record per B-tree block
    int c[8];        // children: segment rows (height 0) or blocks
    int len;         // observer length (cachedLength, MT/mergeTree.ts:2770-2789)
    int parent;      // parent block, -1 root; next-free link when free
    int n;           // childCount
    int height;      // 0 = children are segments
    int scour;       // needsScour: -1 undefined, 0 false, 1 true
    int pad[3];
};
// An immutable property map of n keys (insertion order) occupies ceil(n / 16) consecutive
// chunks (at least one): key i is chunk i / 16's key[i % 16]; every chunk carries n.
struct __attribute__((aligned(16))) MtPSet {
    uint16_t key[MT_PSK];
    int32_t val[MT_PSK];
    int32_t n;
    int32_t pad[3];
};
struct MtHeapE { int seg; int maxSeq; };     // LRUSegment, MT/mergeTree.ts:915-923
// removedClientOverlap entries of clients >= 63 (MT/mergeTree.ts:2563-2571), per document:
// the overlap bitmask covers clients 0..62 and its bit 63 says "look here".  An entry is
// live while its row still has the removedSeq it was written under.
struct MtOvx { int row; int rseq; int client; int pad; };
#define MT_OVX_CAP 512                         // side-list entries per document
// RegisterCollection entries (MT/mergeTree.ts:864-896) per document: the cloned segments
// of one (client, register name), as unlinked rows.  flags: 1 = holds a clone of a
// removed segment, 2 = pasted (its rows are in the tree now).
#define MT_REG_CAP 64                  // registers per document (one per lane)
// An entry's clone rows are n consecutive ids at off in the document's register row arena
// (two halves of regCap ids: copying compaction, MtEngT::regCompact).
struct MtReg { int client, name, n, flags, off, pad[3]; };
struct __attribute__((aligned(16))) MtDocHdr {
    int root, height, minSeq, curSeq, rowTop, blkTop, blkFree, heapN, winN, textTop, psetTop;
    uint32_t status;
    unsigned long long cnt[6];               // mt_doc_counters order
    int textHalf;                            // which half of the doc's text arena is live
    int rfN;                                 // recycled rows on the document's stack (hold pool)
    int blkFreeN;                            // blocks on the free list
    int heapHW, winHW;                       // high-water marks (pool sizing, mt_doc_pools)
    int ovxN;                                // overlap side-list entries
    int regTop, regHalf;                     // register row arena: used ids, live half
    int pNever;                              // a property map holding a never-equal value exists
    unsigned long long prof[8];              // MT_PROFILE builds: s_memtime cycles per phase
};

// Where one document's pools live (element offsets into the MtState pools) and
// their capacities: documents of one context may be sized differently
// (mt_create_docs), e.g. by their op counts.
struct __attribute__((aligned(16))) MtDocLayout {
    unsigned long long row, blk, heap, win, anc, text, pset, mid, regr;   // heap: cap+1 entries; text, regr: 2 halves
    uint32_t rowCap, blkCap, heapCap, winCap, textCap, psetCap, midCap, regCap;
};

struct MtState {                              // device pools, doc-major
    MtRow* rows;
    MtBlk* blk; MtHeapE* heap; int* win; int* uid; int* udelta; int* uanc;
    uint16_t* text; MtPSet* pset; MtDocHdr* hdr; int* hold;   // text: 2 halves of textCap per doc; hold: recycled-row stacks
    MtOvx* ovx;                               // overlap side lists, MT_OVX_CAP per doc
    int* mid;                                 // marker-id tables (idToSegment): row per id, -1 unmapped
    MtReg* reg;                               // register collections, MT_REG_CAP per doc
    int* regr;                                // register row arenas (MtDocLayout::regr, two halves)
    uint32_t rowCap, blkCap, heapCap, winCap, textCap, psetCap, holdCap, maxDocs;   // largest per-doc caps
    const MtDocLayout* layout;                // [maxDocs]
    // interned op property sets (mt_prop_table)
    const uint32_t* p_off; const uint16_t* p_key; const int32_t* p_val;
    const uint8_t* p_falsy; const uint32_t* p_class; uint32_t p_nsets;
    // per value: incr's result from it held (MT_VAL_NAN for a number / boolean, else the
    // interned String(v) + "undefined" in bits 0..29, MT_VINFO_NONE there when not interned)
    // and MT_VINFO_SEQM1; element -1: incr of a fresh consensus object (null: combine sets
    // unsupported); mt_set_props
    const int32_t* p_vinfo;
};
#define MT_VINFO_ID    0x3FFFFFFF
#define MT_VINFO_NONE  0x3FFFFFFF
#define MT_VINFO_SEQM1 0x40000000

struct __attribute__((aligned(16))) MtOpRec {  // one 32-byte op record (mt_op_batch member, packed)
    uint8_t type, flags; uint16_t client;
    int32_t seq, ref_seq, msn, pos1, pos2;
    uint32_t payload_off;
    uint16_t payload_len; int16_t prop_id;
};
struct MtRelPos { int marker, before, offset, pad; };   // mt_rel_pos
// One delta / maintenance callback entry (mt_delta_rec): kind, the observer-view position
// of the segment when the callback fires, its cachedLength, its row and two
// kind-specific fields (see include/mtgpu.h).
struct __attribute__((aligned(16))) MtDeltaRec { uint32_t op; int kind, pos, len, seg, a, b, pad; };
struct MtOps {                                // device copy of an mt_op_batch
    const uint32_t* doc_ids; const uint32_t* op_off;
    MtOpRec* rec;
    uint16_t* payload;
    const MtRelPos* rel; uint32_t n_rel;
    // Delta capture (null: off).  dcount[0] records appended, [1] records reserved, [2] text
    // units appended, [3] text units reserved (MT_DC_*); dtext holds pasted segments' text.
    MtDeltaRec* drec; unsigned long long* dcount; unsigned long long dcap;
    uint16_t* dtext; unsigned long long dtcap;
    uint32_t* resume;                         // capture: op index each run stopped at (op_off[run+1]: done)
    const uint32_t* start;                    // capture resume: first op of each run (null: op_off)
    uint32_t n_runs;
    uint64_t payload_units;                   // records are bounds-checked against it on the device
    // Per-run payload bases in units (null: payload_off is absolute).  An exchanged batch of a
    // million documents holds more than 2^32 payload units; its records' payload_off is then
    // relative to the run's base (mt_upload_rows_dev).
    const unsigned long long* pay_base;
};
enum { MT_DC_REC = 0, MT_DC_RECRES = 1, MT_DC_TXT = 2, MT_DC_TXTRES = 3 };
// Records one message can emit at most, beyond its own range or paste: 2 ensureIntervalBoundary
// SPLITs and two zamboni calls (the op's and setMinSeq's),
// each popping <= 2 heap entries that scour one leaf block (8) and may packParent its
// siblings (<= 8 blocks of 8).
#define MT_DREC_SLACK (2 + 2 * 2 * (8 + 64))

// Snapshot load (mt_load_snapshot): the segments of each document (mt_load_seg)
// and the host's plan of loadBody's insertSegments calls (MT/snapshotLoader.ts:162-206).
struct __attribute__((aligned(16))) MtLoadSeg {
    uint8_t flags, pad0; uint16_t client;
    int32_t seq, rseq;
    uint16_t rclient; int16_t prop;
    uint32_t poff, plen;
    uint32_t mid, pad1;                       // marker id index + 1 (0: none)
};
// One step of the body plan: START = first segment of an insertSegments call
// (ensureIntervalBoundary at the observer's length, then insert), CONT = a later
// segment of the same call (insertPos += previous cachedLength, blockInsert
// :2207-2241), REFLUSH[_NEW] = a flush of loadBody's never-emptied batch that
// would insert already-linked segments [followed by new ones], UNSUPPORTED =
// the host rejected the document (nothing is loaded).
enum { MT_LD_START = 0, MT_LD_CONT = 1, MT_LD_REFLUSH = 2, MT_LD_REFLUSH_NEW = 3, MT_LD_UNSUPPORTED = 4 };
struct MtLoadStep { int seg, kind, cli, seq; };
struct MtLoad {
    const uint32_t* docs; const uint32_t* seg_off; const uint32_t* nhdr;
    const int32_t* ms; const int32_t* cs;
    const MtLoadSeg* segs; const uint16_t* payload;
    const uint32_t* plan_off; const MtLoadStep* plan;
};
#define MT_NONCOLLAB 0xFFFE           // NonCollabClient (MT/constants.ts) in the 16-bit client field
#define MT_NOBODY 0xFFFF              // a client id no row carries (getLength's "any other client")

struct MtGen {                                // device stream generator parameters
    unsigned long long seed;
    uint32_t ops, clients, lag_max, pct_insert, pct_remove, ins_len_max, rem_len_max, n_ann_sets, pct_rewrite;
    int enabled;
    const uint32_t* clients_per_run;          // per-document authoring clients (mt_generate_docs), or null
    uint32_t doc_id_base;                     // run i is seeded as document doc_id_base + i
    uint32_t ins_len_min, seg_prop_sets, ins_at_end;
    uint64_t total_ops;                       // ops over all runs (payload stride base)
};

struct __attribute__((aligned(16))) MtQ16 { uint32_t x, y, z, w; };
// LDS home of a document's hot pools while mt_replay_lds_kernel runs it.
struct __attribute__((aligned(16))) MtLdsPools {
    MtRow rows[MT_L_ROWS];
    MtBlk blk[MT_L_BLKS];
    MtHeapE heap[MT_L_HEAP + 2];
    int win[MT_L_ROWS];
    int uid[MT_L_ROWS];
    int udelta[MT_L_ROWS];
    uint8_t uanc[MT_L_ROWS * MT_L_H];
};

// LDS home of a document's blocks and heap while mt_replay_blk_kernel (NB = MT_B_BLKS) or
// mt_replay_blkw_kernel (NB = MT_BW_BLKS) runs it.
template <int NB, int NH, int NT, int NW> struct __attribute__((aligned(16))) MtLdsBlkT {
    static_assert(NB <= NT, "block ids index the corrections table");
    MtBlk blk[NB];
    MtHeapE heap[NH + 2];
    // the window's first NW entries (the rest in HBM): computeU reads them without an HBM
    // round trip, and window appends and compaction write them here
    int win[NW];
    // Per-block perspective corrections of the current U set (Σ delta of the U rows beneath
    // each block, indexed by block id): a descent level reads its children's lengths as
    // observer length + correction instead of scanning U (no ancestor chains kept).
    int bcorr[NT];
};
using MtLdsBlk = MtLdsBlkT<MT_B_BLKS, MT_B_HEAP, MT_B_BT, MT_B_W>;
using MtLdsBlkW = MtLdsBlkT<MT_BW_BLKS, MT_BW_HEAP, MT_BW_BT, MT_BW_W>;

// LDS home of a long document's heap, window and U set while mt_replay_big_kernel runs it.
struct __attribute__((aligned(16))) MtLdsBig {
    MtHeapE heap[MT_G_HEAP + 2];
    int win[MT_G_WIN];
    int uid[MT_G_U], udelta[MT_G_U];
    int uanc[MT_G_U * MT_G_H];        // block ids (-1 = none)
    uint16_t ulist[MT_G_U];           // a descent's U entries under the current block (walk)
    MtBlk bc[MT_G_BC];                // block cache (write-back; HBM copies of cached blocks are stale)
    int btag[MT_G_BC];                // block id held by each slot, MT_BC_EMPTY if none
    // computeU's staged window entries (one round): row, delta, (parent + 1) | live << 30 | recycle << 31
    int sid[MT_G_STG], sdel[MT_G_STG], spf[MT_G_STG];
    int htk[MT_G_HT], htv[MT_G_HT];   // corrections table: block id (MT_BC_EMPTY: free), Σ delta
    uint16_t hlist[MT_G_HT];          // occupied slots in insertion (level) order
    uint32_t bpc[MT_G_BP];            // parent cache (MT_G_BPC)
    struct Job {                      // a job wave 0 posts to the workgroup (mwRun / mwPost)
        int op, r, c, r0, n, H, minSeq, heapN;
        MtRow* R; int* win; MtBlk* blk; int* uanc; uint16_t* text;
    } mw[2];
    int posted;                       // jobs wave 0 has posted (the exit job goes to slot posted & 1)
};

// per-wave scratch (LDS on the device)
struct MtScratch {
    int pathB[MT_MAXH + 2], pathJ[MT_MAXH + 2];
    int pathOff[MT_MAXH + 2], pathLen[MT_MAXH + 2];   // a walk's path blocks: perspective start, length
    int hold[64];
    int holdLen[64];                  // observer length of each held child (scourLeaves)
    uint8_t holdBlk[64];              // index (in its parent) of the block each held child was in (packParent)
    int rfree[MT_RFL];                // recycled rows (unlinked, out of the window, no heap entry)
    int corr[MT_MAXN];                // per-child perspective corrections (childLens)
};

// A row record read as 16-byte quads (one wide load per quad); may_alias keeps those accesses
// ordered with the field accesses of the same record.
struct __attribute__((aligned(16), may_alias)) MtQ16a { uint32_t x, y, z, w; };
#ifndef MT_NONL
#define MT_NONL 1                     // rows flag text without a newline (MT_M_NONL)
#endif
#ifndef MT_LEAF_ONCE
#define MT_LEAF_ONCE 1                // walk: leaf rows loaded whole once, splits from registers
#endif
#ifndef MT_GT_CH
#define MT_GT_CH 4                    // gatherText: 64-unit chunks loaded before any is stored
#endif
#ifndef MT_SCOUR_QUADS
#define MT_SCOUR_QUADS 1              // scourLeaves: rows' first two quads in two wide loads
#endif
MT_INLINE int pick16(const int* c, int j) {         // c[j] for a lane index j (no private-array indexing)
    int v = c[0];
#pragma unroll
    for (int i = 1; i < 16; i++) v = (j == i) ? c[i] : v;
    return v;
}
MT_INLINE int pick8(const int* c, int j) {
    int v = c[0];
#pragma unroll
    for (int i = 1; i < 8; i++) v = (j == i) ? c[i] : v;
    return v;
}
// Is client c in row s's removedClientOverlap?  Clients < 63 are bits of the mask; the
// rest live in the document's side list (bit 63 set), scanned only in that rare case.
// c is wave-uniform, so the c < 63 test is a scalar branch; the side-list scan runs every
// entry in every lane (no per-lane exits: see vis_rc).
MT_INLINE bool ovl_has(const MtOvx* ox, int n, unsigned long long ovl, int s, int rseq, int c) {
    if (c < 63) return ((ovl >> c) & 1ull) != 0;
    const bool more = (ovl >> 63) != 0;
    bool f = false;
    for (int i = 0; i < n; i++) {
        const MtOvx e = ox[i];
        f = f | (more & (e.row == s) & (e.client == c) & (e.rseq == rseq));
    }
    return f;
}
// nodeLength's visibility of segment row s under perspective (r, c), MT/mergeTree.ts:1652-1692.
// Evaluated without short circuits, so per-lane conditions stay lane masks instead of nested
// divergent branches: with the short-circuit form the gfx950 backend merged a caller's
// `vis ? len : 0` wrongly across those branches (removed rows whose removal the perspective
// has not seen came out as length 0; round 4, DESIGN.md §4 "Device-only INSERT_FAILED").
MT_INLINE bool vis_rc(int seq, uint32_t meta, int rseq, uint32_t rcl, unsigned long long ovl, int r, int c,
                      const MtOvx* ox, int nox, int s) {
    const int cl = (int)(meta & MT_M_CLIENT);
    const bool seen = (cl == c) | (seq <= r);
    const bool removed = (meta & MT_M_REMOVED) != 0;
    const bool gone = ((int)rcl == c) | (rseq <= r) | ovl_has(ox, nox, ovl, s, rseq, c);
    return seen & !(removed & gone);
}

struct BlkH { int len, parent, n, height, scour; };
struct ChildL { int len; bool tie; };
struct WinI { int id; int delta; int parent; bool live; bool recycle; };

enum { MT_WALK_SPLIT = 0, MT_WALK_INSERT = 1 };
enum { MT_W_OK = 0, MT_W_NOCHANGE = 1, MT_W_FAIL = 2 };
enum { MT_MAP_REMOVE = 0, MT_MAP_ANNOTATE = 1, MT_MAP_COLLECT = 2 };
// How an annotate's prop set applies (applyPropSet): plain, rewrite, or a combining op
// (MT_OPF_COMBINE: incr, MT_PM_INCR_SMIN with a string minValue; MT_OPF_COMBINE |
// MT_OPF_REWRITE: other names, with MT_OPF_CONSENSUS consensus).
enum { MT_PM_SET = 0, MT_PM_REWRITE = 1, MT_PM_INCR = 2, MT_PM_KEEP = 3, MT_PM_CONS = 4, MT_PM_INCR_SMIN = 5 };
MT_INLINE int mt_prop_mode(uint32_t fl) {
    if (!(fl & MT_OPF_COMBINE)) return (fl & MT_OPF_REWRITE) ? MT_PM_REWRITE : MT_PM_SET;
    if (fl & MT_OPF_REWRITE) return (fl & MT_OPF_CONSENSUS) ? MT_PM_CONS : MT_PM_KEEP;
    return (fl & MT_OPF_INCR_STRMIN) ? MT_PM_INCR_SMIN : MT_PM_INCR;
}

// The wave's view of one document: doc-local pool pointers and the few global
// parameters it needs (kept small: every field is wave-uniform and lives in SGPRs).
struct MtEngParams {
    uint32_t rowCap, heapCap, winCap, textCap, psetCap, p_nsets;
    uint16_t* textBase;
    const uint32_t* p_off; const uint16_t* p_key; const int32_t* p_val;
    const uint8_t* p_falsy; const uint32_t* p_class; const int32_t* p_vinfo;
};
// The LDS pools live in one file-scope __shared__ object, so every access of
// the LDS-resident engine (MtEngT<MT_RES_LDS / MT_RES_BLK>) is a ds_* instruction; the host
// emulation has one static instance (it runs one wave at a time).
#if defined(__HIP_DEVICE_COMPILE__)
__shared__ MtLdsPools mt_lds_pools_v;
#else
static MtLdsPools mt_lds_pools_v;
#endif
MT_INLINE MtLdsPools& mt_lds() { return mt_lds_pools_v; }
#if defined(__HIP_DEVICE_COMPILE__)
__shared__ MtLdsBlk mt_ldsb_v;
#else
static MtLdsBlk mt_ldsb_v;
#endif
MT_INLINE MtLdsBlk& mt_ldsb() { return mt_ldsb_v; }
#if defined(__HIP_DEVICE_COMPILE__)
__shared__ MtLdsBlkW mt_ldsbw_v;
#else
static MtLdsBlkW mt_ldsbw_v;
#endif
MT_INLINE MtLdsBlkW& mt_ldsbw() { return mt_ldsbw_v; }
#if defined(__HIP_DEVICE_COMPILE__)
__shared__ MtLdsBig mt_ldsg_v;
#else
static MtLdsBig mt_ldsg_v;
#endif
MT_INLINE MtLdsBig& mt_ldsg() { return mt_ldsg_v; }

// Cold per-document state of a bound engine: capacities, prop-table pointers, counters,
// high-water marks and LDS caps.  It lives in LDS (one instance per one-wave workgroup)
// instead of SGPRs, which the hot state fills: every field here is read or bumped a
// few times per op at most, and an SGPR spilled past the limit costs a VGPR lane.
struct MtCold {
    MtEngParams S;
    uint32_t cnt[6];
    int hw[2];
    int lcap[3];
    uint32_t gcap[4];
    int epoch, ncol, midcap;
    uint32_t op;
    MtDocHdr* hdr; int* rfhbm; MtOvx* ovx; int* midt; MtReg* regs;   // rarely dereferenced pointers
    MtBlk* blk; MtHeapE* heap; int *uid, *udelta, *uanc; MtPSet* pset;   // HBM homes (MT_RES_BLK: cold)
    int ovxn, blkfreen, texthalf, psettop;
    // delta capture (FULL instantiations): pasted-text arena, this message's record / text
    // use against its reservation, and whether the run stopped for capture headroom
    uint16_t* dtext; unsigned long long dtcap;
    uint32_t dused, tused; int dstop;
    int* regr; int regTop, regHalf, regCap;   // register row arena (this document's)
    int pcKey[4], pcVal[4];                   // newMap: property maps made from an op's set alone
    int pNever;                               // MtDocHdr::pNever
};
#if defined(__HIP_DEVICE_COMPILE__)
__shared__ MtCold mt_cold_v;
#else
static MtCold mt_cold_v;
#endif
#if defined(MT_DBG_FAIL) && defined(__HIP_DEVICE_COMPILE__)
struct MtDbg { int s, n; uint32_t op; };     // diagnostic builds: the last row split
__shared__ MtDbg mt_dbg_v;
#endif

// RES: MT_RES_HBM (every pool in HBM), MT_RES_LDS (rows, blocks, heap, window,
// U set in LDS) or MT_RES_BLK (blocks and heap in LDS).  FULL: the instantiation can
// capture delta records (mt_set_delta_capture) and apply register ops (MT_OP_CUT / COPY /
// PASTE); the replay kernels launch FULL=false unless a capture buffer is armed or the
// batch holds register ops, so the hot path carries none of that code.
template <int RES, bool FULL = true> struct MtEngT {
    static constexpr bool kFull = FULL;
    static constexpr bool LDS = RES == MT_RES_LDS;      // all hot pools in LDS
    static constexpr bool BIG = RES == MT_RES_BIG;      // heap, window, U set in LDS; blocks in HBM
    static constexpr bool BW = RES == MT_RES_BLKW;       // wide block residency (long runs)
    static constexpr bool BLKR = RES == MT_RES_BLK || BW;   // block residency, either width
    static constexpr bool BLKL = RES == MT_RES_LDS || BLKR;  // blocks + heap in LDS
    // the block-residency LDS home of this instantiation
    MT_HD auto& LB() const { if constexpr (BW) return mt_ldsbw(); else return mt_ldsb(); }
    MtEngParams& S = mt_cold_v.S;      // cold state (MtCold, LDS)
    MtDocHdr*& hdrp = mt_cold_v.hdr;
    // doc-local views
    MtRow* R;
    // Block residency keeps blocks, heap and the first U entries in LDS: their HBM homes (and
    // the property-set pool) are cold there and live in MtCold; other modes keep them in SGPRs.
    template <class T> using Home = std::conditional_t<BLKR, T&, T>;
    int* win;
    Home<int*> uid = mt_cold_v.uid; Home<int*> udelta = mt_cold_v.udelta; Home<int*> uanc = mt_cold_v.uanc;
    Home<MtBlk*> blk = mt_cold_v.blk; Home<MtHeapE*> heap = mt_cold_v.heap;
    uint16_t* text; Home<MtPSet*> pset = mt_cold_v.pset;
    MtOvx*& ovx = mt_cold_v.ovx; int& ovxN = mt_cold_v.ovxn;
    int*& midt = mt_cold_v.midt; int& midCap = mt_cold_v.midcap;   // idToSegment (MT/mergeTree.ts:1095, :1175)
    MtReg*& regs = mt_cold_v.regs;            // RegisterCollection (MT_REG_CAP entries)
    int*& regr = mt_cold_v.regr; int& regTop = mt_cold_v.regTop; int& regHalf = mt_cold_v.regHalf;
    int& regCap = mt_cold_v.regCap;
    MT_HD int& regRow(int i) const { return regr[(size_t)regHalf * regCap + i]; }
    MtDeltaRec* drec; unsigned long long* dcount; unsigned long long dcap; uint32_t& curOp = mt_cold_v.op;   // delta capture
    uint16_t*& dtext = mt_cold_v.dtext; unsigned long long& dtcap = mt_cold_v.dtcap;
    uint32_t &dUsed = mt_cold_v.dused, &tUsed = mt_cold_v.tused; int& dStop = mt_cold_v.dstop;
    MtScratch* sc;
    // pool accessors: LDS (MT_RES_LDS, MT_RES_BLK for blocks + heap) or HBM homes
    MT_HD MtRow& row(int s) const { if constexpr (LDS) return mt_lds().rows[s]; else return R[s]; }
    MT_HD MtBlk& bk(int b) const {
        if constexpr (LDS) return mt_lds().blk[b]; else if constexpr (BLKL) return LB().blk[b];
        else if constexpr (BIG && MT_G_BCACHE) {        // block cache hit: the LDS copy is the current one
            const int s = b & (MT_G_BC - 1);
            return mt_ldsg().btag[s] == b ? mt_ldsg().bc[s] : blk[b];
        } else return blk[b];
    }
    // MT_RES_BIG: install block B (its current record in lanes 0..15) in its cache slot, whose
    // tag is tg, unless the slot holds a higher live block; the evicted block is written back.
    MT_HD void bcInstall(int B, int tg, const LaneArr<int>& w, int hb) {
        if constexpr (BIG && MT_G_BCACHE) {
            if (!bcOn || hb < MT_G_BCH || tg == B) return;
            const int s = B & (MT_G_BC - 1);
            MtLdsBig& G = mt_ldsg();
            if (tg != MT_BC_EMPTY) {
                if (uni(G.bc[s].n) >= 0 && uni(G.bc[s].height) > hb) return;
                const auto old = wave_map(16, [&](int i) MT_LAM { return ((const int*)&G.bc[s])[i]; });
                wave_for(16, [&](int i) MT_LAM { ((int*)&blk[tg])[i] = own(old, i); });
            }
            wave_for(16, [&](int i) MT_LAM { ((int*)&G.bc[s])[i] = own(w, i); });
            wave_for(1, [&](int) MT_LAM { G.btag[s] = B; });
            wave_sync();
        } else { (void)B; (void)tg; (void)w; (void)hb; }
    }
    MT_HD int bcTag(int B) const {
        if constexpr (BIG && MT_G_BCACHE) return uni(mt_ldsg().btag[B & (MT_G_BC - 1)]);
        else { (void)B; return 0; }
    }
    MT_HD MtHeapE& hp(int k) const {
        if constexpr (LDS) return mt_lds().heap[k]; else if constexpr (BLKL) return LB().heap[k];
        else if constexpr (BIG) return mt_ldsg().heap[k]; else return heap[k];
    }
    // Window entry k under block residency: the first MT_B_W in LDS.  Loads and stores are made
    // in each branch (a reference to either home would be a generic pointer: flat_* accesses).
    static constexpr int kW = BW ? MT_BW_W : MT_B_W;    // window entries in LDS (block residency)
    MT_HD int winGet(int k) const {
        if constexpr (BLKR) { if (k < kW) return LB().win[k]; return win[k]; }
        else return wn(k);
    }
    MT_HD void winSet(int k, int v) const {
        if constexpr (BLKR) { if (k < kW) LB().win[k] = v; else win[k] = v; }
        else wn(k) = v;
    }
    MT_HD int& wn(int k) const {
        static_assert(!BLKR, "block residency: winGet / winSet");
        if constexpr (LDS) return mt_lds().win[k];
        else if constexpr (BIG) { if (k < lRows) return mt_ldsg().win[k]; return win[k]; }   // beyond lRows: HBM home
        else return win[k];
    }
    MT_HD int& ui(int k) const { if constexpr (LDS) return mt_lds().uid[k]; else return uid[k]; }
    MT_HD int& ud(int k) const { if constexpr (LDS) return mt_lds().udelta[k]; else return udelta[k]; }
    // MT_RES_BIG keeps the first MT_G_U U-set entries in LDS (block residency keeps no U
    // entries: the corrections table holds their sums).  U loops run per 64-entry chunk (chunks never straddle the cap), so each
    // chunk picks its home at compile time: forU calls f(std::bool_constant<inLds>, base, m).
    static constexpr bool UL = RES == MT_RES_BIG;
    static constexpr bool BT = BLKR;   // per-block corrections table (MtLdsBlkT::bcorr)
    static constexpr int UCAP = RES == MT_RES_BIG ? MT_G_U : 0;
    template <bool L> MT_HD int uiAt(int k) const {
        if constexpr (UL && L) return mt_ldsg().uid[k];
        else return ui(k);
    }
    template <bool L> MT_HD int udAt(int k) const {
        if constexpr (UL && L) return mt_ldsg().udelta[k];
        else return ud(k);
    }
    template <bool L> MT_HD void uPutAt(int k, int id, int delta) {
        if constexpr (UL && L) { mt_ldsg().uid[k] = id; mt_ldsg().udelta[k] = delta; }
        else { ui(k) = id; ud(k) = delta; }
    }
    template <bool L> MT_HD void ancPutAt(int u, int h, int a) {
        if constexpr (UL && L) {
            static_assert(BIG, "block residency keeps per-block corrections, not ancestor chains");
            mt_ldsg().uanc[u * MT_G_H + h] = a;
        } else ancPut(u, h, a);
    }
    template <bool L> MT_HD int ancGetAt(int u, int h) const {
        if constexpr (UL && L) {
            static_assert(BIG, "block residency keeps per-block corrections, not ancestor chains");
            return mt_ldsg().uanc[u * MT_G_H + h];
        } else return ancGet(u, h);
    }
    MT_HD void ancPutAny(int u, int h, int a) {
        if constexpr (UL) { if (u < UCAP) ancPutAt<true>(u, h, a); else ancPutAt<false>(u, h, a); }
        else ancPut(u, h, a);
    }
    MT_HD int ancGetAny(int u, int h) const {
        if constexpr (UL) { if (u < UCAP) return ancGetAt<true>(u, h); return ancGetAt<false>(u, h); }
        else return ancGet(u, h);
    }
    template <class F> MT_HD void forU(F f) const {
        for (int base = 0; base < nU; base += MT_WAVE) {
            const int m = (nU - base) < MT_WAVE ? (nU - base) : MT_WAVE;
            if (UL && base < UCAP) f(std::true_type{}, base, m);
            else f(std::false_type{}, base, m);
        }
    }
    // uniform document state (MtDocHdr)
    int root, height, minSeq, curSeq, rowTop, blkTop, blkFree, heapN, winN, textTop;
    int& psetTop = mt_cold_v.psettop;
    uint32_t status;
    // Counters of this bind (added into the header at store), in LDS (MtCold).
    uint32_t &c_ops = mt_cold_v.cnt[0], &c_msgs = mt_cold_v.cnt[1], &c_ins = mt_cold_v.cnt[2], &c_rows = mt_cold_v.cnt[3],
             &c_depth = mt_cold_v.cnt[4], &c_scour = mt_cold_v.cnt[5];
    unsigned long long prof[8];
    int& textHalf = mt_cold_v.texthalf; uint32_t blkCap;
    int nU; bool uValid; int uRef, uCli;
    int heapTop;                        // hp(1).maxSeq cached (INT_MAX when empty)
    int& gcEpoch = mt_cold_v.epoch;     // bumped by every text compaction
    int lastL, lastIdx; bool lastSplit; // landing spot of the last walk; did it split a block
    bool bcOn;                          // MT_RES_BIG: descents fill the LDS block cache
    bool htOk; int hlistN;              // MT_RES_BIG: the corrections table is built for U; occupied slots
    bool htOn, pfOn; int mwSeq;         // MT_RES_BIG: table / zamboni prefetch enabled; jobs posted so far
    bool bpOn;                          // MT_RES_BIG: the LDS parent cache is kept (MT_G_BPC)
    int& nCol = mt_cold_v.ncol;         // rows gathered by rangeMap(MT_MAP_COLLECT) at the register arena's tail
    int landB;                          // leaf block the last insertAtPath linked its node under
    int rfN; int*& rfHbm = mt_cold_v.rfhbm;   // recycled-row stack: depth, HBM home between runs
    int& blkFreeN = mt_cold_v.blkfreen;       // blocks on the free list
    int &heapHW = mt_cold_v.hw[0], &winHW = mt_cold_v.hw[1];   // high-water marks of heapN / winN
    // LDS residency (toLds/fromLds): LDS caps, and the HBM caps they stand in for
    static constexpr bool kLds = BLKL || BIG;           // runs check ldsHeadroom before each op
    int &lRows = mt_cold_v.lcap[0], &lBlks = mt_cold_v.lcap[1], &lHeap = mt_cold_v.lcap[2];
    uint32_t &gRowCap = mt_cold_v.gcap[0], &gBlkCap = mt_cold_v.gcap[1], &gHeapCap = mt_cold_v.gcap[2],
             &gWinCap = mt_cold_v.gcap[3];

    MT_HD void bind(const MtState& st, uint32_t d, MtScratch* scratch) {
        const MtDocLayout* Ly = st.layout + d;
        auto off = [&](const unsigned long long* p) -> size_t {
            const uint32_t* w = (const uint32_t*)p;
            return (size_t)uni(w[0]) | ((size_t)uni(w[1]) << 32);
        };
        S.rowCap = uni(Ly->rowCap); S.heapCap = uni(Ly->heapCap); S.winCap = uni(Ly->winCap); S.textCap = uni(Ly->textCap);
        S.psetCap = uni(Ly->psetCap); S.p_nsets = st.p_nsets; S.p_off = st.p_off; S.p_key = st.p_key; S.p_val = st.p_val;
        S.p_falsy = st.p_falsy; S.p_class = st.p_class; S.p_vinfo = st.p_vinfo; S.textBase = st.text + off(&Ly->text);
        blkCap = uni(Ly->blkCap); hdrp = st.hdr + d;
        R = st.rows + off(&Ly->row);
        blk = st.blk + off(&Ly->blk); heap = st.heap + off(&Ly->heap);
        const size_t wo = off(&Ly->win);
        win = st.win + wo; uid = st.uid + wo; udelta = st.udelta + wo; uanc = st.uanc + off(&Ly->anc);
        pset = st.pset + off(&Ly->pset);
        ovx = st.ovx + (size_t)d * MT_OVX_CAP;
        regs = st.reg + (size_t)d * MT_REG_CAP;
        regr = st.regr + off(&Ly->regr); regCap = (int)uni(Ly->regCap);
        midt = st.mid + off(&Ly->mid); midCap = (int)uni(Ly->midCap);
        drec = nullptr; dcount = nullptr; dcap = 0; curOp = 0;
        dtext = nullptr; dtcap = 0; dUsed = 0; tUsed = 0; dStop = 0;
        sc = scratch;
        const MtDocHdr& h = *hdrp;
        root = uni(h.root); height = uni(h.height); minSeq = uni(h.minSeq); curSeq = uni(h.curSeq); rowTop = uni(h.rowTop);
        blkTop = uni(h.blkTop); blkFree = uni(h.blkFree); heapN = uni(h.heapN); winN = uni(h.winN); textTop = uni(h.textTop);
        psetTop = uni(h.psetTop); status = uni(h.status); textHalf = uni(h.textHalf);
        text = S.textBase + (size_t)textHalf * S.textCap;
#if MT_KEEP_PROF
        for (int i = 0; i < 8; i++) prof[i] = h.prof[i];
#endif
        c_ops = c_msgs = c_ins = c_rows = c_depth = c_scour = 0;
        nU = 0; uValid = false; uRef = -1; uCli = -1;
        heapTop = heapN > 0 ? uni(heap[1].maxSeq) : 0x7FFFFFFF;     // HBM home: bind precedes toLds
        lastL = 0; lastIdx = 0; lastSplit = false; gcEpoch = 0; bcOn = false; htOk = false; hlistN = 0; htOn = pfOn = false; mwSeq = 0; bpOn = false;
        for (int i = 0; i < 4; i++) mt_cold_v.pcKey[i] = -1;
        rfHbm = st.hold + (size_t)d * MT_RFL; rfN = uni(h.rfN); blkFreeN = uni(h.blkFreeN);
        heapHW = uni(h.heapHW); winHW = uni(h.winHW); ovxN = uni(h.ovxN);
        regTop = uni(h.regTop); regHalf = uni(h.regHalf) & 1; mt_cold_v.pNever = uni(h.pNever);
        if (regTop < 0 || regTop > regCap) regTop = 0;
        if (ovxN < 0 || ovxN > MT_OVX_CAP) ovxN = 0;
        lRows = lBlks = lHeap = 0; gRowCap = gBlkCap = gHeapCap = gWinCap = 0;
        if (rfN < 0 || rfN > MT_RFL) rfN = 0;
        { const int n = rfN; const int* src = rfHbm;
          for (int base = 0; base < n; base += MT_WAVE) {
              const int m = (n - base) < MT_WAVE ? (n - base) : MT_WAVE;
              wave_for(m, [&](int k) MT_LAM { sc->rfree[base + k] = src[base + k]; });
          } }
        wave_sync();
    }
    MT_HD void store(uint32_t) {
        MtDocHdr& h = *hdrp;
        h.root = root; h.height = height; h.minSeq = minSeq; h.curSeq = curSeq; h.rowTop = rowTop;
        h.blkTop = blkTop; h.blkFree = blkFree; h.heapN = heapN; h.winN = winN; h.textTop = textTop;
        h.psetTop = psetTop; h.status = status; h.textHalf = textHalf; h.rfN = rfN; h.blkFreeN = blkFreeN;
        h.heapHW = heapHW; h.winHW = winHW; h.ovxN = ovxN; h.regTop = regTop; h.regHalf = regHalf;
        h.pNever = mt_cold_v.pNever;
        { const int n = rfN; int* dst = rfHbm;
          for (int base = 0; base < n; base += MT_WAVE) {
              const int m = (n - base) < MT_WAVE ? (n - base) : MT_WAVE;
              wave_for(m, [&](int k) MT_LAM { dst[base + k] = sc->rfree[base + k]; });
          } }
#if MT_KEEP_PROF
        for (int i = 0; i < 8; i++) h.prof[i] = prof[i];
#endif
        h.cnt[0] += c_ops; h.cnt[1] += c_msgs; h.cnt[2] += c_ins; h.cnt[3] += c_rows; h.cnt[4] += c_depth;
        h.cnt[5] += c_scour;
    }
    // Fresh empty collaborating document: root = empty block (MergeTree ctor :1105-1108,
    // startCollaboration :1243).
    MT_HD void open() {
        root = 0; height = 0; minSeq = 0; curSeq = 0; rowTop = 0; blkTop = 1; blkFree = -1;
        heapN = 0; winN = 0; textTop = 0; psetTop = 0; status = 0; textHalf = 0; heapTop = 0x7FFFFFFF; rfN = 0;
        for (int i = 0; i < 4; i++) mt_cold_v.pcKey[i] = -1;    // the memo's maps are gone with the pool
        blkFreeN = 0; heapHW = 0; winHW = 0; ovxN = 0;
        text = S.textBase;
        c_ops = c_msgs = c_ins = c_rows = c_depth = c_scour = 0;
        for (int i = 0; i < 6; i++) hdrp->cnt[i] = 0;               // store() adds this bind's counts
        for (int i = 0; i < 8; i++) prof[i] = 0;
#if !MT_KEEP_PROF
        for (int i = 0; i < 8; i++) hdrp->prof[i] = 0;
#endif
        wave_for(8, [&](int i) MT_LAM { bk(0).c[i] = -1; });
        bk(0).len = 0; bk(0).parent = -1; bk(0).n = 0; bk(0).height = 0; bk(0).scour = -1;
        bpReset();
        wave_for(MT_REG_CAP, [&](int i) MT_LAM { regs[i].client = -1; regs[i].n = 0; regs[i].flags = 0; regs[i].off = 0; });
        regTop = 0; regHalf = 0; mt_cold_v.pNever = 0;
        // idToSegment entries are not reset: an entry is read only for an id the host
        // already saw mapped in this document (mt_rel_pos.marker >= 0), and relPos
        // checks that the row still carries that id.
    }

    /* ---------------------------------------------------------- pools -- */
    // Rows are recycled once unlinked, out of the window and referenced by no
    // heap entry (nothing can reach them); the stack is LIFO so reuse stays cache-hot.
    MT_HD int allocRow() {
        if (rfN > 0) { rfN--; return uni(sc->rfree[rfN]); }
        if (rowTop >= (int)S.rowCap) { status |= MT_DS_OOM_ROWS; return -1; }
        return rowTop++;
    }
    MT_HD void freeRow(int s) { if (rfN < MT_RFL) { sc->rfree[rfN] = s; rfN++; } }
    MT_HD int allocBlock() {
        if (blkFree >= 0) { const int id = blkFree; blkFree = uni(bk(id).parent); blkFreeN--; return id; }
        if (blkTop >= (int)blkCap) { status |= MT_DS_OOM_BLOCKS; return -1; }
        return blkTop++;
    }
    MT_HD void freeBlock(int id) { bk(id).parent = blkFree; bk(id).n = -1; blkFree = id; blkFreeN++; bpDrop(id); }
    // The parent cache (MT_RES_BIG, MT_G_BPC): bpPut after every write of a block's parent field,
    // bpDrop when the field stops being a parent (free list), bpReset when block ids are reassigned.
    MT_HD static uint32_t bpPack(int b, int p) { return ((uint32_t)(b >> MT_G_BPL) << 20) | (uint32_t)(p + 1); }
    MT_HD void bpPut(int b, int p) {
        if constexpr (BIG) {
            if (MT_G_BPC && bpOn) {
                uint32_t& e = mt_ldsg().bpc[b & (MT_G_BP - 1)];
                if (e != MT_BP_EMPTY && (e >> 20) != (uint32_t)(b >> MT_G_BPL)) MT_BS(4);
                e = bpPack(b, p);
            }
        }
    }
    MT_HD void bpDrop(int b) {
        if constexpr (BIG) {
            if (MT_G_BPC && bpOn) {
                uint32_t& e = mt_ldsg().bpc[b & (MT_G_BP - 1)];
                if ((e >> 20) == (uint32_t)(b >> MT_G_BPL)) MT_BS(5);
                e = MT_BP_EMPTY;
            }
        }
    }
    MT_HD void bpReset() {
        if constexpr (BIG) {
            if (MT_G_BPC && bpOn) {
                for (int base = 0; base < MT_G_BP; base += MT_WAVE)
                    wave_for(MT_WAVE, [&](int k) MT_LAM { mt_ldsg().bpc[base + k] = MT_BP_EMPTY; });
                wave_sync();
            }
        }
    }
    // bk(b).parent, through the parent cache when it is kept (a miss fills the entry).
    MT_HD int bkParent(int b) {
        if constexpr (BIG) {
            if (MT_G_BPC && bpOn) {
                uint32_t& e = mt_ldsg().bpc[b & (MT_G_BP - 1)];
                const uint32_t v = e;
                MT_BS(0);
                if ((v >> 20) == (uint32_t)(b >> MT_G_BPL)) {
                    MT_BS(1);
#if defined(MT_BPC_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
                    if ((int)(v & 0xFFFFFu) - 1 != bk(b).parent) abort();     // host emulation: a stale entry
#endif
                    return (int)(v & 0xFFFFFu) - 1;
                }
                if (v == MT_BP_EMPTY) MT_BS(2); else MT_BS(3);
                const int p = bk(b).parent;
                e = bpPack(b, p);
                return p;
            }
        }
        return bk(b).parent;
    }

    /* ---------------------------------------------------- LDS residency -- */
    // Lane-parallel copy of n 16-byte quads.
    MT_HD static void copyQ(MtQ16* dst, const MtQ16* src, int n) {
        for (int base = 0; base < n; base += MT_WAVE) {
            const int m = (n - base) < MT_WAVE ? (n - base) : MT_WAVE;
            wave_for(m, [&](int k) MT_LAM { dst[base + k] = src[base + k]; });
        }
    }
    MT_HD static void copyI(int* dst, const int* src, int n) {
        for (int base = 0; base < n; base += MT_WAVE) {
            const int m = (n - base) < MT_WAVE ? (n - base) : MT_WAVE;
            wave_for(m, [&](int k) MT_LAM { dst[base + k] = src[base + k]; });
        }
    }
    // MT_RES_LDS: move the document's rows, blocks, heap and window into
    // the LDS pools (caps lr/lb/lh <= the MT_L_* array sizes).  False (nothing
    // moved) if they do not fit.  R/blk/heap/win keep pointing at the HBM homes.
    MT_HD bool toLds(int lr, int lb, int lh) {
        static_assert(BLKL || BIG, "LDS residency needs MtEngT<MT_RES_LDS, MT_RES_BLK or MT_RES_BIG>");
        if constexpr (BIG) {                                    // heap + window (U set is per op)
            if (lh <= 0 || lh > MT_G_HEAP) lh = MT_G_HEAP;
            if (lr <= 0 || lr > MT_G_WIN) lr = MT_G_WIN;       // window entries kept in LDS (the rest in HBM)
            if (heapN > lh || height + 3 > MT_G_H) return false;
            MtLdsBig& G = mt_ldsg();
            copyI((int*)G.heap, (const int*)heap, 2 * (heapN + 1));
            copyI(G.win, win, winN < lr ? winN : lr);
            for (int base = 0; MT_G_BCACHE && base < MT_G_BC; base += MT_WAVE)
                wave_for(MT_WAVE, [&](int k) MT_LAM { G.btag[base + k] = MT_BC_EMPTY; });
            for (int base = 0; base < MT_G_HT; base += MT_WAVE)
                wave_for(MT_WAVE, [&](int k) MT_LAM { G.htk[base + k] = MT_BC_EMPTY; G.htv[base + k] = 0; });
            htOk = false; hlistN = 0;
            bcOn = MT_G_BCACHE && !(lb & MT_BIGF_NO_BCACHE);    // lb: MT_BIGF_* switches (A/B)
            pfOn = MT_G_NW > 1 && !(lb & MT_BIGF_NO_PREFETCH);
            htOn = !(lb & MT_BIGF_NO_TABLE);
            bpOn = MT_G_BPC && !(lb & MT_BIGF_NO_BPC) && blkCap < (1u << 20);
            bpReset();
            wave_sync();
            gRowCap = S.rowCap; gBlkCap = blkCap; gHeapCap = S.heapCap; gWinCap = S.winCap;
            S.heapCap = gHeapCap < (uint32_t)lh ? gHeapCap : (uint32_t)lh;
            lRows = lr; lBlks = 0x7FFFFFFF; lHeap = lh;
            nU = 0; uValid = false;
            return true;
        }
        if constexpr (!LDS) {                                   // MT_RES_BLK / BLKW: blocks + heap only
            constexpr int kB = BW ? MT_BW_BLKS : MT_B_BLKS, kH = BW ? MT_BW_HEAP : MT_B_HEAP;
            if (lb <= 0 || lb > kB) lb = kB;
            if (lh <= 0 || lh > kH) lh = kH;
            if (blkTop > lb || heapN > lh || height + 3 > MT_L_H) return false;
            auto& B = LB();
            copyQ((MtQ16*)B.blk, (const MtQ16*)blk, blkTop * (int)(sizeof(MtBlk) / 16));
            copyI((int*)B.heap, (const int*)heap, 2 * (heapN + 1));
            copyI(B.win, win, winN < kW ? winN : kW);
            wave_sync();
            gRowCap = S.rowCap; gBlkCap = blkCap; gHeapCap = S.heapCap; gWinCap = S.winCap;
            blkCap = gBlkCap < (uint32_t)lb ? gBlkCap : (uint32_t)lb;
            S.heapCap = gHeapCap < (uint32_t)lh ? gHeapCap : (uint32_t)lh;
            lRows = 0x7FFFFFFF; lBlks = lb; lHeap = lh;
            nU = 0; uValid = false;
            return true;
        }
        if (rowTop > lr || blkTop > lb || heapN > lh || winN > lr || height + 3 > MT_L_H || lb > 255) return false;
        MtLdsPools& L = mt_lds();
        copyQ((MtQ16*)L.rows, (const MtQ16*)R, rowTop * (int)(sizeof(MtRow) / 16));
        copyQ((MtQ16*)L.blk, (const MtQ16*)blk, blkTop * (int)(sizeof(MtBlk) / 16));
        copyI((int*)L.heap, (const int*)heap, 2 * (heapN + 1));
        copyI(L.win, win, winN);
        wave_sync();
        gRowCap = S.rowCap; gBlkCap = blkCap; gHeapCap = S.heapCap; gWinCap = S.winCap;
        S.rowCap = gRowCap < (uint32_t)lr ? gRowCap : (uint32_t)lr;
        blkCap = gBlkCap < (uint32_t)lb ? gBlkCap : (uint32_t)lb;
        S.heapCap = gHeapCap < (uint32_t)lh ? gHeapCap : (uint32_t)lh;
        S.winCap = gWinCap < (uint32_t)lr ? gWinCap : (uint32_t)lr;
        lRows = lr; lBlks = lb; lHeap = lh;
        nU = 0; uValid = false;
        return true;
    }
    MT_HD void fromLds() {
        if constexpr (BIG) {
            MtLdsBig& G = mt_ldsg();
            copyI((int*)heap, (const int*)G.heap, 2 * (heapN + 1));
            copyI(win, G.win, winN < lRows ? winN : lRows);
            // write the cached blocks back (lane k: slot base + k, four 16-byte quads)
            for (int base = 0; MT_G_BCACHE && base < MT_G_BC; base += MT_WAVE) {
                wave_for(MT_WAVE, [&](int k) MT_LAM {
                    const int t = G.btag[base + k];
                    if (t != MT_BC_EMPTY) {
                        const MtQ16* src = (const MtQ16*)&G.bc[base + k];
                        MtQ16* dst = (MtQ16*)&blk[t];
                        const MtQ16 a = src[0], b = src[1], c2 = src[2], d = src[3];
                        dst[0] = a; dst[1] = b; dst[2] = c2; dst[3] = d;
                    }
                    G.btag[base + k] = MT_BC_EMPTY;
                });
            }
            bcOn = false; htOk = false; pfOn = false;
            wave_sync();
            S.heapCap = gHeapCap;
            nU = 0; uValid = false;
            return;
        }
        if constexpr (!LDS) {
            auto& B = LB();
            copyQ((MtQ16*)blk, (const MtQ16*)B.blk, blkTop * (int)(sizeof(MtBlk) / 16));
            copyI((int*)heap, (const int*)B.heap, 2 * (heapN + 1));
            copyI(win, B.win, winN < kW ? winN : kW);
            wave_sync();
            blkCap = gBlkCap; S.heapCap = gHeapCap;
            nU = 0; uValid = false;
            return;
        }
        MtLdsPools& L = mt_lds();
        copyQ((MtQ16*)R, (const MtQ16*)L.rows, rowTop * (int)(sizeof(MtRow) / 16));
        copyQ((MtQ16*)blk, (const MtQ16*)L.blk, blkTop * (int)(sizeof(MtBlk) / 16));
        copyI((int*)heap, (const int*)L.heap, 2 * (heapN + 1));
        copyI(win, L.win, winN);
        wave_sync();
        S.rowCap = gRowCap; blkCap = gBlkCap; S.heapCap = gHeapCap; S.winCap = gWinCap;
        nU = 0; uValid = false;
    }
    // Can the next op run without outgrowing the LDS pools?  Per op at most 2
    // row splits + 1 new row, 2 split cascades of height+2 blocks and packParent
    // regrowth; one heap entry per op plus one per message.  k: the further segments the op
    // inserts (a paste's clones): k rows and heap entries, and at most ceil(k / 3) + 1 more
    // blocks (a leaf split per 4 inserted rows, an interior one per 4 new blocks).
    MT_HD bool ldsHeadroom(int k = 0) const {
        const int kb = k > 0 ? (k + 2) / 3 + 1 : 0;
        if constexpr (BIG) return (lHeap - heapN) >= 4 + k && height + 3 <= MT_G_H;
        if constexpr (!BLKL) return true;
        // Block budget per message, an upper bound: the op's two cascades (two
        // split walks, or a split and an insert) allocate at most (h + 2) + (h + 3) blocks; a
        // zamboni pop's packParent chain grows the tree by at most 2 blocks in all (a level
        // re-deals its n child blocks' <= 8(n - 1) + 3 children into min(7, floor(nh / 4))
        // blocks: at most n + 2, and the chain climbs only past a level left with fewer than
        // 4 blocks, which cannot have grown), with MT_ZMAX pops in each of a message's two
        // zamboni calls: 2h + 5 + 2 * 2 * MT_ZMAX = 2h + 13.  The largest growth measured in
        // the host emulation is 2h + 2 (tools/micro/block_growth.py, MT_EVCOUNT3).
        if constexpr (!LDS) return (lBlks - blkTop + blkFreeN) >= 2 * height + MT_B_SLACK + kb && (lHeap - heapN) >= 4 + k &&
                                   height + 3 <= MT_L_H;
        return (lRows - rowTop + rfN) >= 4 + k && (lBlks - blkTop + blkFreeN) >= 6 * (height + 2) + 8 + kb &&
               (lHeap - heapN) >= 4 + k && height + 3 <= MT_L_H;
    }
    MT_HD void ancPut(int u, int h, int a) {
        if constexpr (LDS) mt_lds().uanc[u * MT_L_H + h] = (uint8_t)(a < 0 ? 255 : a);
        else uanc[(size_t)u * MT_MAXH + h] = a;
    }
    MT_HD int ancGet(int u, int h) const {
        if constexpr (LDS) { const int a = mt_lds().uanc[u * MT_L_H + h]; return a == 255 ? -1 : a; }
        else return uanc[(size_t)u * MT_MAXH + h];
    }
    MT_HD uint32_t winAddKnown(int s, uint32_t mt) {
        if (mt & MT_M_INWIN) return mt;
        if (winN >= (int)S.winCap) { status |= MT_DS_OOM_WINDOW; return mt; }
        winSet(winN++, s);
        if (winN > winHW) winHW = winN;
        row(s).meta = mt | MT_M_INWIN;
        return mt | MT_M_INWIN;
    }
    MT_HD void winAdd(int s) {
        const uint32_t mt = uni(row(s).meta);
        if (mt & MT_M_INWIN) return;
        if (winN >= (int)S.winCap) { status |= MT_DS_OOM_WINDOW; return; }
        winSet(winN++, s);
        if (winN > winHW) winHW = winN;
        row(s).meta = mt | MT_M_INWIN;
    }
    // winAdd for the rows of lanes [0, n) where sel: one meta load for all, the rows not yet
    // in the window appended in lane order (one round trip instead of one per row).
    MT_HD void winAddLanes(const LaneArr<int>& ids, const LaneArr<bool>& sel, int n) {
        if (!wave_ballot(wave_map(n, [&](int j) MT_LAM { return (bool)own(sel, j); }))) return;   // uniform skip
        auto add = wave_map(n, [&](int j) MT_LAM {
            const bool q = own(sel, j);                           // branch-free
            return (bool)(q & !(row(q ? own(ids, j) : 0).meta & MT_M_INWIN));
        });
        const int cnt = wave_count(add);
        if (!cnt) return;
        if (winN + cnt > (int)S.winCap) { status |= MT_DS_OOM_WINDOW; return; }
        const auto rk = wave_rank(add);
        const int w0 = winN;
        wave_for(n, [&](int j) MT_LAM {
            if (!own(add, j)) return;
            const int s = own(ids, j);
            winSet(w0 + own(rk, j), s);
            row(s).meta = row(s).meta | MT_M_INWIN;
        });
        winN += cnt;
        if (winN > winHW) winHW = winN;
    }
    // Scalar fields of a block (SGPRs) and its children (one per lane).
    MT_HD BlkH head(int B) const {
        BlkH h;
        h.len = uni(bk(B).len); h.parent = uni(bk(B).parent); h.n = uni(bk(B).n);
        h.height = uni(bk(B).height); h.scour = uni(bk(B).scour);
        return h;
    }
    MT_HD LaneArr<int> kids(int B, int n) const { return wave_map(n, [&](int j) MT_LAM { return bk(B).c[j]; }); }
    // Whole 64-byte block record in one transaction: lane i loads dword i;
    // children stay in lanes 0..n-1, scalar fields are broadcast to SGPRs.
    MT_HD LaneArr<int> blkLoad(int B, BlkH& h) {
        LaneArr<int> w;
        int tg = 0;
        if constexpr (BIG && MT_G_BCACHE) {               // explicit LDS / HBM load, then fill
            tg = bcTag(B);
            if (tg == B) w = wave_map(16, [&](int i) MT_LAM { return ((const int*)&mt_ldsg().bc[B & (MT_G_BC - 1)])[i]; });
            else w = wave_map(16, [&](int i) MT_LAM { return ((const int*)&blk[B])[i]; });
        } else w = wave_map(16, [&](int i) MT_LAM { return ((const int*)&bk(B))[i]; });
        h.len = wave_at(w, 8); h.parent = wave_at(w, 9); h.n = wave_at(w, 10); h.height = wave_at(w, 11); h.scour = wave_at(w, 12);
        if constexpr (BIG && MT_G_BCACHE) bcInstall(B, tg, w, h.height);
        const int n = h.n;
        return wave_map(8, [&](int j) MT_LAM { return j < n ? own(w, j) : -1; });
    }
    // Blocks in HBM: the records of all children of an interior block in one round trip
    // (lane t holds dword t&15 of child t>>4 in r0 and of child (t>>4)+4 in r1), so the
    // descent needs no separate loads for the children's lengths or the next level's block.
    MT_HD void kidsLoad(const LaneArr<int>& ch, int n, LaneArr<int>& r0, LaneArr<int>& r1) const {
        const auto c0 = wave_shfl(ch, [](int t) MT_LAM { return t >> 4; });
        const auto c1 = wave_shfl(ch, [](int t) MT_LAM { return (t >> 4) + 4; });
        r0 = wave_map(MT_WAVE, [&](int t) MT_LAM { return (t >> 4) < n ? ((const int*)&bk(own(c0, t)))[t & 15] : 0; });
        r1 = wave_map(MT_WAVE, [&](int t) MT_LAM { return (t >> 4) + 4 < n ? ((const int*)&bk(own(c1, t)))[t & 15] : 0; });
    }
    // lanes 0..7: child j's observer length (dword 8 of its record)
    MT_HD static LaneArr<int> kidsLen(const LaneArr<int>& r0, const LaneArr<int>& r1) {
        const auto a = wave_shfl(r0, [](int t) MT_LAM { return ((t & 3) << 4) + 8; });
        const auto b = wave_shfl(r1, [](int t) MT_LAM { return ((t & 3) << 4) + 8; });
        return wave_map(8, [&](int j) MT_LAM { return j < 4 ? own(a, j) : own(b, j); });
    }
    // child j's record as blkLoad returns it (j uniform)
    // (MT_RES_BIG: the child, block id b, is installed in the block cache.)
    MT_HD LaneArr<int> kidRec(const LaneArr<int>& r0, const LaneArr<int>& r1, int j, BlkH& h, int b) {
        const int o = (j & 3) << 4;
        const auto w = wave_shfl(j < 4 ? r0 : r1, [o](int t) MT_LAM { return o + (t & 15); });
        h.len = wave_at(w, 8); h.parent = wave_at(w, 9); h.n = wave_at(w, 10); h.height = wave_at(w, 11); h.scour = wave_at(w, 12);
        if constexpr (BIG && MT_G_BCACHE) { if (bcOn && h.height >= MT_G_BCH) bcInstall(b, bcTag(b), w, h.height); } else (void)b;
        const int n = h.n;
        return wave_map(8, [&](int i) MT_LAM { return i < n ? own(w, i) : -1; });
    }
    MT_HD int childObsLen(int h, int id) const {
        if (h == 0) return (row(id).meta & MT_M_REMOVED) ? 0 : row(id).len;
        return bk(id).len;
    }
    MT_HD int sumObs(int B, int n, int h) const {
        auto v = wave_map(n, [&](int j) MT_LAM { return childObsLen(h, bk(B).c[j]); });
        return wave_sum8(v);
    }
    MT_HD void setChildParent(int h, int id, int p) {
        if (h == 0) row(id).parent = p; else { bk(id).parent = p; bpPut(id, p); }
    }

    /* ------------------------------------- perspective window (U set) -- */
    // One window entry (row s) under perspective (r, c): still live in the window, recyclable,
    // and its U delta (perspective length - observer length).
    MT_HD WinI winEntry(int s, int r, int c) const {
        WinI w; w.id = s;
#if MT_SCOUR_QUADS
        // the row as three 16-byte loads (len seq rseq meta | toff props parent tcap | ovl rcl mid)
        const MtQ16a q0 = ((const MtQ16a*)&row(s))[0], q1 = ((const MtQ16a*)&row(s))[1], q2 = ((const MtQ16a*)&row(s))[2];
        const uint32_t mt = q0.w;
        const int sq = (int)q0.y, rs = (int)q0.z, ln = (int)q0.x;
        w.parent = (int)q1.z;
        const unsigned long long ovl = (unsigned long long)q2.x | ((unsigned long long)q2.y << 32);
        const uint32_t rcl = q2.z;
#else
        const uint32_t mt = row(s).meta;
        const int sq = row(s).seq, rs = row(s).rseq, ln = row(s).len;
        w.parent = row(s).parent;
        const unsigned long long ovl = row(s).ovl;
        const uint32_t rcl = row(s).rcl;
#endif
        const bool removed = (mt & MT_M_REMOVED) != 0;
        const bool linked = w.parent >= 0;
        w.live = linked && (sq > minSeq || (removed && rs > minSeq));
        w.recycle = !linked && !(mt & MT_M_HREF);
        const bool vr = vis_rc(sq, mt, rs, rcl, ovl, r, c, ovx, ovxN, s);
        const bool vo = !removed;
        w.delta = w.live ? ((vr ? ln : 0) - (vo ? ln : 0)) : 0;
        return w;
    }
    // One 64-entry chunk of the window scan, in order: compaction of live entries (prune),
    // recycled rows onto the stack, U entries with their level-0 ancestor (the leaf block).
    MT_HD void placeChunk(const LaneArr<WinI>& wi, int base, int m, bool prune, int& newWin) {
        auto live = wave_map(m, [&](int k) MT_LAM { return own(wi, k).live; });
        if (prune) {
            auto rk = wave_rank(live);
            const int cntLive = wave_count(live);
            auto rc = wave_map(m, [&](int k) MT_LAM { return own(wi, k).recycle; });
            auto rkr = wave_rank(rc);
            const int cntR = wave_count(rc), f0 = rfN;
            const int nw0 = newWin;
            wave_for(m, [&](int k) MT_LAM {
                const WinI w = own(wi, k);
                if (w.live) { if (nw0 + own(rk, k) != base + k) winSet(nw0 + own(rk, k), w.id); }
                else row(w.id).meta = row(w.id).meta & ~MT_M_INWIN;
                if (w.recycle && f0 + own(rkr, k) < MT_RFL) sc->rfree[f0 + own(rkr, k)] = w.id;
            });
            rfN = (f0 + cntR) < MT_RFL ? (f0 + cntR) : MT_RFL;
            newWin += cntLive;
        }
        auto du = wave_map(m, [&](int k) MT_LAM { return own(wi, k).delta != 0; });
        auto rk2 = wave_rank(du);
        const int cntU = wave_count(du);
        const int nu0 = nU;
        wave_for(m, [&](int k) MT_LAM {
            if (!own(du, k)) return;
            const int pos = nu0 + own(rk2, k);
            const WinI w = own(wi, k);
            if (pos < UCAP) { uPutAt<true>(pos, w.id, w.delta); ancPutAt<true>(pos, 0, w.parent); }
            else { uPutAt<false>(pos, w.id, w.delta); ancPutAt<false>(pos, 0, w.parent); }
        });
        nU += cntU;
    }
    // Ancestor chains (levels 1..H) of U entries [g0, g0 + 512) from their level-0 entries,
    // blocks in HBM (or the MT_RES_BIG block cache): the parent loads of one level are
    // independent, so a level costs one round trip for 512 entries.
    MT_HD void chainGroup(int g0, int nu, int H) {
        wave_for(MT_WAVE, [&](int k) MT_LAM {
            int a[8]; int pos[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                pos[q] = g0 + q * MT_WAVE + k;
                a[q] = pos[q] < nu ? ancGetAny(pos[q], 0) : -1;
            }
            for (int h = 1; h <= H; h++) {
#pragma unroll
                for (int q = 0; q < 8; q++) a[q] = a[q] >= 0 ? bk(a[q]).parent : -1;
#pragma unroll
                for (int q = 0; q < 8; q++) if (pos[q] < nu) ancPutAny(pos[q], h, a[q]);
            }
        });
    }
    // Multi-wave long-document residency: wave 0 posts a job to the workgroup; every wave
    // (helpers in mt_replay_big_kernel's loop) takes its share between two barriers (mwRun),
    // or the helpers alone run it while wave 0 goes on (mwPost: no completion barrier).
    MT_HD void mwPut(int op, int r, int c, int r0, int n) {
        auto& J = mt_ldsg().mw[mwSeq & 1];
        wave_for(1, [&](int) MT_LAM {
            J.op = op; J.r = r; J.c = c; J.r0 = r0; J.n = n; J.H = height; J.minSeq = minSeq; J.heapN = heapN;
            J.R = R; J.win = win; J.blk = blk; J.uanc = uanc; J.text = text;
        });
        mwSeq++;
        wave_for(1, [&](int) MT_LAM { mt_ldsg().posted = mwSeq; });
    }
    MT_HD void mwRun(int op, int r, int c, int r0, int n) {
        if constexpr (BIG) {
            mwPut(op, r, c, r0, n);
#if defined(__HIP_DEVICE_COMPILE__)
            __syncthreads();
            mwShare(0, mwSeq - 1);
            __syncthreads();
#else
            for (int w = 0; w < MT_G_NW; w++) mwShare(w, mwSeq - 1);   // host emulation: every share in turn
#endif
        } else { (void)op; (void)r; (void)c; (void)r0; (void)n; }
    }
    MT_HD void mwPost(int op) {
        if constexpr (BIG) {
            mwPut(op, 0, 0, 0, 0);
#if defined(__HIP_DEVICE_COMPILE__)
            __syncthreads();
#else
            for (int w = 1; w < MT_G_NW; w++) mwShare(w, mwSeq - 1);
#endif
        } else (void)op;
    }
    MT_HD static bool mwSync(int op) { return op != MT_MW_PREFETCH; }
    // This wave's share (wave index wv) of job number k; helpers first adopt the document's
    // pool homes and window state from it.
    MT_HD void mwShare(int wv, int k) {
        if constexpr (BIG) {
            MtLdsBig& G = mt_ldsg();
            const auto& J = G.mw[k & 1];
            const int op = uni(J.op);
            if (wv != 0) {
                R = J.R; win = J.win; blk = J.blk; uanc = J.uanc; text = J.text;
                minSeq = uni(J.minSeq);
            }
            if (op == MT_MW_SCAN) {
                const int r = uni(J.r), c = uni(J.c), r0 = uni(J.r0), n = uni(J.n);
                // chunks wv, wv + NW, ... of the round, two per step (both chunks' loads in flight)
                for (int q = wv * MT_WAVE; q < n; q += 2 * MT_G_NW * MT_WAVE) {
                    const int q2 = q + MT_G_NW * MT_WAVE;
                    const int m = (n - q) < MT_WAVE ? (n - q) : MT_WAVE;
                    const int m2 = q2 < n ? ((n - q2) < MT_WAVE ? (n - q2) : MT_WAVE) : 0;
                    const auto id1 = wave_map(m, [&](int k) MT_LAM { return winGet(r0 + q + k); });
                    const auto id2 = wave_map(m2, [&](int k) MT_LAM { return winGet(r0 + q2 + k); });
                    const auto w1 = wave_map(m, [&](int k) MT_LAM { return winEntry(own(id1, k), r, c); });
                    const auto w2 = wave_map(m2, [&](int k) MT_LAM { return winEntry(own(id2, k), r, c); });
                    auto put = [&](const LaneArr<WinI>& w, int qq, int mm) MT_LAM {
                        wave_for(mm, [&](int k) MT_LAM {
                            const WinI e = own(w, k);
                            G.sid[qq + k] = e.id; G.sdel[qq + k] = e.delta;
                            G.spf[qq + k] = (e.parent + 1) | (e.live ? 1 << 30 : 0) | (e.recycle ? (int)0x80000000 : 0);
                        });
                    };
                    put(w1, q, m);
                    put(w2, q2, m2);
                }
            } else if (op == MT_MW_CHAIN) {
                const int nu = uni(J.n), H = uni(J.H);
                for (int g0 = wv * 8 * MT_WAVE; g0 < nu; g0 += MT_G_NW * 8 * MT_WAVE) chainGroup(g0, nu, H);
            } else if (op == MT_MW_PREFETCH && wv == 1) {
                // zamboni's next pops come from the top of the heap: touch entries 1..7's rows,
                // their leaf blocks, the blocks' rows and those rows' last text unit, so wave 0's
                // scour finds them in cache (values are discarded; nothing is written)
                // (wave 0 writes these pools meanwhile: every index read is bounds-checked)
                const int hn = uni(J.heapN);
                const unsigned rc = S.rowCap, bc = gBlkCap, tc = S.textCap;
                wave_for(56, [&](int t) MT_LAM {
                    const int e = 1 + (t >> 3);
                    if (e > hn || e > (int)MT_G_HEAP) return;
                    const int sg = hp(e).seg;
                    if ((unsigned)sg >= rc) return;
                    const int p = row(sg).parent;
                    if ((unsigned)p >= bc) return;
                    const int cnt = bk(p).n, j = t & 7;
                    if (j >= cnt) return;
                    const int ch = bk(p).c[j];
                    if ((unsigned)ch >= rc) return;
                    const int tf = row(ch).toff, ln = row(ch).len;
                    const uint32_t mt = row(ch).meta;
                    int v = row(ch).seq ^ row(ch).rseq ^ row(ch).props ^ row(ch).tcap ^ (int)mt;
                    const int ix = tf + ln - 1;
                    const bool q = !(mt & MT_M_MARKER) & (ix >= 0) & ((unsigned)ix < tc);
                    const int tv = (int)text[q ? ix : 0];
                    v ^= q ? tv : 0;
                    mt_keep(v);
                });
            }
            wave_sync();
        } else { (void)wv; (void)k; }
    }
    // Posted after each op's U set: the zamboni prefetch runs beside the op's descents.
    MT_HD void mwPrefetch() {
        if constexpr (BIG) { if (pfOn && heapN > 0 && heapTop <= minSeq + 1024) mwPost(MT_MW_PREFETCH); }
    }
    // computeU of the long-document residency: the window scan in rounds of MT_G_STG entries
    // (all waves stage the entries' rows, wave 0 places them in order), then the chains.
    MT_HD void computeUmw(int r, int c, bool prune) {
        MtLdsBig& G = mt_ldsg();
        int newWin = 0; nU = 0;
        const int wN0 = winN;
        MT_UB(u0); MT_UC(4, wN0); MT_UC(5, 1);
        if (wN0 <= MT_G_MWMIN) {                    // a few chunks: wave 0 alone, no barriers
#if MT_G_ALLCH
            // every chunk's rows in one round trip (one wave per SIMD here: registers to spare),
            // then placed in order (placement writes only entries below the chunk it places)
            constexpr int NC = MT_G_MWMIN / MT_WAVE;
            LaneArr<WinI> wis[NC];
#pragma unroll
            for (int q = 0; q < NC; q++) {
                const int base = q * MT_WAVE;
                const int m = base >= wN0 ? 0 : ((wN0 - base) < MT_WAVE ? (wN0 - base) : MT_WAVE);
                const auto ids = wave_map(m, [&](int k) MT_LAM { return winGet(base + k); });
                wis[q] = wave_map(m, [&](int k) MT_LAM { return winEntry(own(ids, k), r, c); });
            }
#pragma unroll
            for (int q = 0; q < NC; q++) {
                const int base = q * MT_WAVE;
                if (base >= wN0) break;
                placeChunk(wis[q], base, (wN0 - base) < MT_WAVE ? (wN0 - base) : MT_WAVE, prune, newWin);
            }
#else
            for (int base = 0; base < wN0; base += MT_WAVE) {
                const int m = (wN0 - base) < MT_WAVE ? (wN0 - base) : MT_WAVE;
                const auto ids = wave_map(m, [&](int k) MT_LAM { return winGet(base + k); });
                const auto wi = wave_map(m, [&](int k) MT_LAM { return winEntry(own(ids, k), r, c); });
                placeChunk(wi, base, m, prune, newWin);
            }
#endif
        }
        for (int r0 = 0; wN0 > MT_G_MWMIN && r0 < wN0; r0 += MT_G_STG) {
            const int n = (wN0 - r0) < MT_G_STG ? (wN0 - r0) : MT_G_STG;
            mwRun(MT_MW_SCAN, r, c, r0, n);
            for (int q = 0; q < n; q += MT_WAVE) {
                const int m = (n - q) < MT_WAVE ? (n - q) : MT_WAVE;
                const auto wi = wave_map(m, [&](int k) MT_LAM {
                    WinI w; w.id = G.sid[q + k]; w.delta = G.sdel[q + k];
                    const int pf = G.spf[q + k];
                    w.parent = (pf & 0x3FFFFFFF) - 1; w.live = ((pf >> 30) & 1) != 0; w.recycle = pf < 0;
                    return w;
                });
                placeChunk(wi, r0 + q, m, prune, newWin);
            }
        }
        wave_sync();
        MT_UE(0, u0); MT_UC(3, nU);
        MT_UB(u1);
        htOk = false;
        if (nU > 0 && height > 0 && !(htOn && htBuild())) mwRun(MT_MW_CHAIN, r, c, 0, nU);
        MT_UE(1, u1);
        if (prune) winN = newWin;
        wave_sync();
        uValid = true; uRef = r; uCli = c;
    }
    MT_HD static unsigned htHash(int b) { return ((unsigned)b * 2654435761u) >> (32 - __builtin_ctz(MT_G_HT)); }
    // Lane-parallel insert: adds val to key's slot (claiming a free one); returns the slot and
    // whether this lane claimed it.
    MT_HD int htAdd(int key, int val, bool& won) {
        MtLdsBig& G = mt_ldsg();
        int sl = (int)htHash(key);
        won = false;
        for (;;) {
            const int old = lds_cas(&G.htk[sl], MT_BC_EMPTY, key);
            if (old == MT_BC_EMPTY) { won = true; break; }
            if (old == key) break;
            sl = (sl + 1) & (MT_G_HT - 1);
        }
        lds_add(&G.htv[sl], val);
        return sl;
    }
    MT_HD int htGet(int key) const {
        const MtLdsBig& G = mt_ldsg();
        int sl = (int)htHash(key);
        for (;;) {
            const int k = G.htk[sl];
            if (k == key) return G.htv[sl];
            if (k == MT_BC_EMPTY) return 0;
            sl = (sl + 1) & (MT_G_HT - 1);
        }
    }
    // Appends the slots lanes claimed to hlist (in lane order).
    MT_HD void htList(const LaneArr<int>& sl, const LaneArr<bool>& won, int m) {
        const auto rk = wave_rank(won);
        const int cnt = wave_count(won), h0 = hlistN;
        wave_for(m, [&](int k) MT_LAM { if (own(won, k)) mt_ldsg().hlist[h0 + own(rk, k)] = (uint16_t)own(sl, k); });
        hlistN += cnt;
    }
    // The corrections table for the current U set, bottom-up: leaf blocks get their U rows'
    // deltas, then every distinct block of one height passes its sum to its parent (root
    // excluded: no descent asks for it).  False if it would outgrow MT_G_HTN (table left
    // empty, htOk false: the caller computes ancestor chains instead).
    MT_HD bool htBuild() {
        MtLdsBig& G = mt_ldsg();
        for (int base = 0; base < hlistN; base += MT_WAVE) {               // the last U set's slots
            const int m = (hlistN - base) < MT_WAVE ? (hlistN - base) : MT_WAVE;
            wave_for(m, [&](int k) MT_LAM { const int sl = G.hlist[base + k]; G.htk[sl] = MT_BC_EMPTY; G.htv[sl] = 0; });
        }
        hlistN = 0;
        wave_sync();
        if (nU > MT_G_HTN) return false;
        forU([&](auto inL, int base, int m) MT_LAM {
            constexpr bool L = decltype(inL)::value;
            const auto a = wave_map(m, [&](int k) MT_LAM {
                bool w; const int x = htAdd(ancGetAt<L>(base + k, 0), udAt<L>(base + k), w); return w ? x : ~x;
            });
            htList(wave_map(m, [&](int k) MT_LAM { return own(a, k) >= 0 ? own(a, k) : ~own(a, k); }),
                   wave_map(m, [&](int k) MT_LAM { return own(a, k) >= 0; }), m);
        });
        wave_sync();
        int l0 = 0, l1 = hlistN;
        const int rt = root;
        for (int h = 1; h < height; h++) {                                  // blocks of height h
            if (hlistN + (l1 - l0) > MT_G_HTN) {
                for (int base = 0; base < hlistN; base += MT_WAVE) {
                    const int m = (hlistN - base) < MT_WAVE ? (hlistN - base) : MT_WAVE;
                    wave_for(m, [&](int k) MT_LAM { const int sl = G.hlist[base + k]; G.htk[sl] = MT_BC_EMPTY; G.htv[sl] = 0; });
                }
                hlistN = 0;
                wave_sync();
                return false;
            }
            for (int base = l0; base < l1; base += MT_WAVE) {
                const int m = (l1 - base) < MT_WAVE ? (l1 - base) : MT_WAVE;
                const auto ch = wave_map(m, [&](int k) MT_LAM { return (int)G.hlist[base + k]; });
#if defined(MT_PROFILE4)
                MT_UC(6, m);
                if (bpOn) MT_UC(7, wave_count(wave_map(m, [&](int k) MT_LAM {
                    const int b = G.htk[own(ch, k)];
                    return (G.bpc[b & (MT_G_BP - 1)] >> 20) != (uint32_t)(b >> MT_G_BPL);
                })));
#endif
                const auto par = wave_map(m, [&](int k) MT_LAM { return bkParent(G.htk[own(ch, k)]); });
                const auto val = wave_map(m, [&](int k) MT_LAM { return G.htv[own(ch, k)]; });
                const auto a = wave_map(m, [&](int k) MT_LAM {
                    const int p = own(par, k);
                    bool w = false; int x = 0;
                    if ((p >= 0) & (p != rt)) x = htAdd(p, own(val, k), w);
                    return w ? x : ~x;
                });
                htList(wave_map(m, [&](int k) MT_LAM { return own(a, k) >= 0 ? own(a, k) : ~own(a, k); }),
                       wave_map(m, [&](int k) MT_LAM { return own(a, k) >= 0; }), m);
            }
            wave_sync();
            l0 = l1; l1 = hlistN;
            MT_UC(2, 1);
        }
        htOk = true;
        return true;
    }
    // Scan the window list: prune settled/unlinked rows (if prune) and collect
    // U = rows whose visibility differs between the observer and (r, c).
    MT_HD void computeU(int r, int c, bool prune) {
        if constexpr (BIG && MT_G_NW > 1) {
            MT_PB(tm);
            computeUmw(r, c, prune);
            MT_PE(MT_PH_U, tm);
            return;
        }
        MT_PB(t0);
        MT_EV(0, 1); MT_EV(2, winN);
        MT_QB(q0); MT_QC(4);
        int newWin = 0; nU = 0;
        if constexpr (BT) {                               // corrections table: cleared per U set
            for (int base = 0; base < blkTop; base += MT_WAVE) {
                const int m = (blkTop - base) < MT_WAVE ? (blkTop - base) : MT_WAVE;
                wave_for(m, [&](int k) MT_LAM { LB().bcorr[base + k] = 0; });
            }
            wave_sync();
        }
        // Window rows, one 64-entry chunk at a time, software-pipelined: chunk i+1's row
        // fields are in flight while chunk i is processed, and chunk i+2's window ids behind
        // them (the window entries are distinct rows and compaction only writes entries below
        // the chunk being read, so the early reads see what in-order reads would).
        auto winIds = [&](int base) MT_LAM {
            const int m = (winN - base) < MT_WAVE ? (winN - base) : MT_WAVE;
            return wave_map(m, [&](int k) MT_LAM { return winGet(base + k); });
        };
        auto winRows = [&](const LaneArr<int>& ids, int base) MT_LAM {
            const int m = (winN - base) < MT_WAVE ? (winN - base) : MT_WAVE;
            return wave_map(m, [&](int k) MT_LAM { return winEntry(own(ids, k), r, c); });
        };
        const int wN0 = winN;
#ifndef MT_CU_PIPE
#define MT_CU_PIPE 0
#endif
#if MT_CU_PIPE
        LaneArr<WinI> wiNext{};
        LaneArr<int> idNext{};
        if (wN0 > 0) wiNext = winRows(winIds(0), 0);
        if (wN0 > MT_WAVE) idNext = winIds(MT_WAVE);
#else
        LaneArr<int> idn{};
        if (wN0 > 0) idn = winIds(0);
#endif
        for (int base = 0; base < wN0; base += MT_WAVE) {
            const int m = (wN0 - base) < MT_WAVE ? (wN0 - base) : MT_WAVE;
#if MT_CU_PIPE
            const auto wi = wiNext;
            if (base + MT_WAVE < wN0) {
                wiNext = winRows(idNext, base + MT_WAVE);
                if (base + 2 * MT_WAVE < wN0) idNext = winIds(base + 2 * MT_WAVE);
            }
#else
            // one chunk's rows at a time (the software-pipelined variant, MT_CU_PIPE, holds two
            // chunks in VGPRs and costs the hot kernel spills); the next chunk's window ids load
            // behind this chunk's rows
            const auto wi = winRows(idn, base);
            if (base + MT_WAVE < wN0) idn = winIds(base + MT_WAVE);
#endif
            auto live = wave_map(m, [&](int k) MT_LAM { return own(wi, k).live; });
            if (prune) {
                auto rk = wave_rank(live);
                const int cntLive = wave_count(live);
                auto rc = wave_map(m, [&](int k) MT_LAM { return own(wi, k).recycle; });
                auto rkr = wave_rank(rc);
                const int cntR = wave_count(rc), f0 = rfN;
                const int nw0 = newWin;
                wave_for(m, [&](int k) MT_LAM {
                    const WinI w = own(wi, k);
                    // compaction writes only entries that move (none until the first pruned one)
                    if (w.live) { if (nw0 + own(rk, k) != base + k) winSet(nw0 + own(rk, k), w.id); }
                    else row(w.id).meta = row(w.id).meta & ~MT_M_INWIN;
                    if (w.recycle && f0 + own(rkr, k) < MT_RFL) sc->rfree[f0 + own(rkr, k)] = w.id;
                });
                rfN = (f0 + cntR) < MT_RFL ? (f0 + cntR) : MT_RFL;
                newWin += cntLive;
            }
            auto du = wave_map(m, [&](int k) MT_LAM { return own(wi, k).delta != 0; });
            auto rk2 = wave_rank(du);
            const int cntU = wave_count(du);
            const int nu0 = nU;
            const int H = height;
            wave_for(m, [&](int k) MT_LAM {          // U entry: row, delta, ancestor chain
                if (!own(du, k)) return;
                const int pos = nu0 + own(rk2, k);
                const WinI w = own(wi, k);
                // blocks in LDS: the chain is walked here; in HBM: level 0 only, the rest below
                const int HH = BLKL ? H : 0;
                int a = w.parent;
                if constexpr (BT) {                       // the row's delta into every block above it
                    (void)pos;
                    for (int h = 0; (h <= HH) & (a >= 0); h++) { lds_add(&LB().bcorr[a], w.delta); a = bk(a).parent; }
                } else if constexpr (UL) {
                    if (pos < UCAP) {
                        uPutAt<true>(pos, w.id, w.delta);
                        for (int h = 0; h <= HH; h++) { ancPutAt<true>(pos, h, a); a = (a >= 0) ? bk(a).parent : -1; }
                    } else {
                        uPutAt<false>(pos, w.id, w.delta);
                        for (int h = 0; h <= HH; h++) { ancPutAt<false>(pos, h, a); a = (a >= 0) ? bk(a).parent : -1; }
                    }
                } else {
                    ui(pos) = w.id; ud(pos) = w.delta;
                    for (int h = 0; h <= HH; h++) { ancPut(pos, h, a); a = (a >= 0) ? bk(a).parent : -1; }
                }
            });
            nU += cntU;
        }
        wave_sync();
        // Blocks in HBM: ancestor chains level by level for up to eight 64-entry chunks at
        // once; the parent loads of one level are independent, so a level costs one round
        // trip for 512 entries instead of one per chunk.
        const int H = height;
        if constexpr (!BLKL) for (int g0 = 0; g0 < nU; g0 += 8 * MT_WAVE) {
            const int nu = nU;
            wave_for(MT_WAVE, [&](int k) MT_LAM {
                int a[8]; int pos[8];
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    pos[q] = g0 + q * MT_WAVE + k;
                    a[q] = pos[q] < nu ? ancGetAny(pos[q], 0) : -1;
                }
                for (int h = 1; h <= H; h++) {
#pragma unroll
                    for (int q = 0; q < 8; q++) a[q] = a[q] >= 0 ? bk(a[q]).parent : -1;
#pragma unroll
                    for (int q = 0; q < 8; q++) if (pos[q] < nu) ancPutAny(pos[q], h, a[q]);
                }
            });
        }
        if (prune) winN = newWin;
        MT_EV(1, nU);
        wave_sync();
        uValid = true; uRef = r; uCli = c;
        MT_PE(MT_PH_U, t0);
        MT_QE(3, q0);
    }
    MT_HD int perspectiveLength(int r, int c) {
        if (!(uValid && uRef == r && uCli == c)) computeU(r, c, false);
        if constexpr (BT) return uni(bk(root).len) + uni(LB().bcorr[root]);   // the root's correction: Σ delta
        int s = 0;
        forU([&](auto inL, int base, int m) MT_LAM {
            constexpr bool L = decltype(inL)::value;
            s += wave_sum(wave_map(m, [&](int k) MT_LAM { return udAt<L>(base + k); }));
        });
        return uni(bk(root).len) + s;
    }
    // perspectiveLength without touching the document's U scratch (read-only: several
    // waves may query one document at once, mt_get_length).
    MT_HD int perspectiveLengthRO(int r, int c) const {
        int s = 0;
        for (int base = 0; base < winN; base += MT_WAVE) {
            const int m = (winN - base) < MT_WAVE ? (winN - base) : MT_WAVE;
            s += wave_sum(wave_map(m, [&](int k) MT_LAM {
                const int id = winGet(base + k);
                const uint32_t mt = row(id).meta;
                const bool removed = (mt & MT_M_REMOVED) != 0;
                const int sq = row(id).seq, rs = row(id).rseq;
                const int ln = row(id).len;
                const bool live = (row(id).parent >= 0) & ((sq > minSeq) | (removed & (rs > minSeq)));
                const bool vr = vis_rc(sq, mt, rs, row(id).rcl, row(id).ovl, r, c, ovx, ovxN, id);
                return live ? (vr ? ln : 0) - (removed ? 0 : ln) : 0;     // branch-free
            }));
        }
        return uni(bk(root).len) + s;
    }
    // MergeTree.getPosition (MT/mergeTree.ts:1578-1596): the (r, c) perspective length
    // of everything before row s; an unlinked row (parent undefined) is at 0.
    MT_HD int getPosition(int s, int r, int c) {
        int B = uni(row(s).parent);
        if (B < 0) return 0;
        if (!(uValid && uRef == r && uCli == c)) computeU(r, c, false);
        int node = s, pos = 0;
        for (;;) {
            BlkH h;
            auto ch = blkLoad(B, h);
            auto cl = childLens(B, h, ch, r, c);
            const int nd = node;
            const int j = wave_first(wave_map(h.n, [&](int i) MT_LAM { return own(ch, i) == nd; }));
            pos += wave_sum8(wave_map(h.n, [&](int i) MT_LAM { return i < j ? own(cl, i).len : 0; }));
            if (h.parent < 0) return pos;
            node = B; B = h.parent;
        }
    }
    // MergeTree.getContainingSegment (MT/mergeTree.ts:1616-1627) by searchBlock (:1786-1815):
    // each block's first child whose (r, c) length exceeds what is left of pos (no tie rule;
    // a negative pos takes every block's first child, as `_pos < len` does), down to a row.
    // Returns the row and sets off = pos - its start; -1 when no child holds pos (segment
    // undefined).  depth / path: child index per level, root first, 3 bits each.
    MT_HD int containing(int pos, int r, int c, int& off, int& depth, unsigned long long& path) {
        if (!(uValid && uRef == r && uCli == c)) computeU(r, c, false);
        int B = root, p = pos;
        depth = 0; path = 0;
        for (;;) {
            BlkH h;
            auto ch = blkLoad(B, h);
            auto cl = childLens(B, h, ch, r, c);
            auto lens = wave_map(h.n, [&](int j) MT_LAM { return own(cl, j).len; });
            auto pre = wave_excl_scan8(lens);
            const int pp = p;
            const int j = wave_first(wave_map(h.n, [&](int k) MT_LAM { return pp - own(pre, k) < own(lens, k); }));
            if (j < 0) return -1;
            p -= wave_at(pre, j);
            depth++; path = (path << 3) | (unsigned long long)j;
            const int child = wave_at(ch, j);
            if (h.height == 0) { off = p; return child; }
            B = child;
        }
    }
    // posFromRelativePos (MT/mergeTree.ts:1949-1972): the marker's position under (r, c),
    // then past the marker (+ cachedLength 1 + offset) or before it (- offset).  -1: the
    // id was never mapped (getMarkerFromId undefined).  A marker whose row was unlinked
    // (or since recycled) sits at 0, as getPosition of a segment without parent does.
    MT_HD int relPos(const MtRelPos& q, int r, int c) {
        const int id = uni(q.marker);
        if (id < 0 || id >= midCap) return -1;
        const int s = uni(midt[id]);
        if (s < 0 || s >= rowTop) return 0;
        const bool live = uni(row(s).mid) == id + 1 && (uni(row(s).meta) & MT_M_MARKER);
        int pos = live ? getPosition(s, r, c) : 0;
        const int off = uni(q.offset);
        if (!uni(q.before)) pos += 1 + off; else pos -= off;
        return pos;
    }
    /* ------------------------------------------- delta / maintenance records -- */
    // Appends one record at the batch's global cursor (documents interleave; every record
    // carries its op index, and one wave appends a document's records in program order).
    MT_HD void emitDelta(int kind, int pos, int len, int seg, int a, int b, int pad = 0) {
        const unsigned long long idx = wave_atomic_add(dcount + MT_DC_REC, 1ull);
        dUsed++;
        if (idx >= dcap) return;
        MtDeltaRec q; q.op = curOp; q.kind = kind; q.pos = pos; q.len = len; q.seg = seg; q.a = a; q.b = b; q.pad = pad;
        const MtDeltaRec* qp = &q;
        wave_for(8, [&](int k) MT_LAM { ((int*)&drec[idx])[k] = ((const int*)qp)[k]; });
    }
    // Capture headroom: before each message the wave reserves the records (nr) and pasted-text
    // units (nt) the message can emit at most, so the append cursors never pass the capacity
    // however the document waves interleave.  False: this launch is full; the run stops before
    // the message and the host resumes it after draining the records.
    MT_HD bool dReserve(unsigned long long nr, unsigned long long nt) {
        const unsigned long long r0 = wave_atomic_add(dcount + MT_DC_RECRES, nr);
        const unsigned long long t0 = wave_atomic_add(dcount + MT_DC_TXTRES, nt);
        if (r0 + nr <= dcap && t0 + nt <= dtcap) { dUsed = 0; tUsed = 0; return true; }
        (void)wave_atomic_add(dcount + MT_DC_RECRES, 0ull - nr);
        (void)wave_atomic_add(dcount + MT_DC_TXTRES, 0ull - nt);
        return false;
    }
    MT_HD void dRelease(unsigned long long nr, unsigned long long nt) {   // the unused part of a reservation
        const unsigned long long ur = nr > dUsed ? nr - dUsed : 0ull, ut = nt > tUsed ? nt - tUsed : 0ull;
        if (ur) (void)wave_atomic_add(dcount + MT_DC_RECRES, 0ull - ur);
        if (ut) (void)wave_atomic_add(dcount + MT_DC_TXTRES, 0ull - ut);
    }
    // Text units a paste of register (c, name) inserts (its clones' cachedLength).
    MT_HD int regTextLen(int c, int name) {
        const int e = regFind(c, name, false);
        if (e < 0) return 0;
        const int n = uni(regs[e].n), o = uni(regs[e].off);
        int t = 0;
        for (int base = 0; base < n; base += MT_WAVE) {
            const int m = (n - base) < MT_WAVE ? (n - base) : MT_WAVE;
            t += wave_sum(wave_map(m, [&](int i) MT_LAM { return row(regRow(o + base + i)).len; }));
        }
        return t;
    }
    // Clones a paste of register (c, name) inserts.
    MT_HD int regCount(int c, int name) {
        const int e = regFind(c, name, false);
        return e < 0 ? 0 : uni(regs[e].n);
    }
    // A pasted text segment's text into the capture's text arena; returns its offset.
    MT_HD int dText(int toff, int len) {
        const unsigned long long o = wave_atomic_add(dcount + MT_DC_TXT, (unsigned long long)len);
        tUsed += (uint32_t)len;
        if (o + (unsigned long long)len > dtcap) return -2;
        for (int base = 0; base < len; base += MT_WAVE) {
            const int m = (len - base) < MT_WAVE ? (len - base) : MT_WAVE;
            wave_for(m, [&](int k) MT_LAM { dtext[o + base + k] = text[toff + base + k]; });
        }
        return (int)o;
    }
    // Observer-view position of row s (MergeTree.getPosition for the local client, whose
    // view is every sequenced op: removed rows count 0); 0 when unlinked.
    MT_HD int obsPosition(int s) {
        int B = uni(row(s).parent);
        if (B < 0) return 0;
        int node = s, pos = 0;
        bool leaf = true;
        for (;;) {
            BlkH h;
            auto ch = blkLoad(B, h);
            const bool lf = leaf;
            auto ol = wave_map(h.n, [&](int j) MT_LAM {
                const int g = own(ch, j);
                return lf ? ((row(g).meta & MT_M_REMOVED) ? 0 : row(g).len) : bk(g).len;
            });
            const int nd = node;
            const int j = wave_first(wave_map(h.n, [&](int i) MT_LAM { return own(ch, i) == nd; }));
            pos += wave_sum8(wave_map(h.n, [&](int i) MT_LAM { return i < j ? own(ol, i) : 0; }));
            if (h.parent < 0) return pos;
            node = B; B = h.parent; leaf = false;
        }
    }
    // A leaf's rows under (r, c); their meta, props and cachedLength come back from the same
    // round trip.
    MT_HD LaneArr<ChildL> leafLens(const LaneArr<int>& ch, int n, int r, int c, LaneArr<uint32_t>& lm, LaneArr<int>& lp,
                                   LaneArr<int>& lr) {
#if MT_SCOUR_QUADS
        // each row as three 16-byte loads (len seq rseq meta | toff props parent tcap | ovl rcl mid)
        const auto q0 = wave_map(n, [&](int j) MT_LAM { return ((const MtQ16a*)&row(own(ch, j)))[0]; });
        const auto q1 = wave_map(n, [&](int j) MT_LAM { return ((const MtQ16a*)&row(own(ch, j)))[1]; });
        const auto q2 = wave_map(n, [&](int j) MT_LAM { return ((const MtQ16a*)&row(own(ch, j)))[2]; });
        lm = wave_map(n, [&](int j) MT_LAM { return own(q0, j).w; });
        lp = wave_map(n, [&](int j) MT_LAM { return (int)own(q1, j).y; });
        lr = wave_map(n, [&](int j) MT_LAM { return (int)own(q0, j).x; });
        return wave_map(n, [&](int j) MT_LAM {
            const MtQ16a a = own(q0, j), x = own(q2, j);
            const uint32_t mt = a.w;
            const int rs = (int)a.z;
            const unsigned long long ovl = (unsigned long long)x.x | ((unsigned long long)x.y << 32);
            ChildL o;
            o.len = vis_rc((int)a.y, mt, rs, x.z, ovl, r, c, ovx, ovxN, own(ch, j)) ? (int)a.x : 0;
            o.tie = !((mt & MT_M_REMOVED) && rs <= r);     // breakTie (MT/mergeTree.ts:2270-2292)
            return o;
        });
#else
        lm = wave_map(n, [&](int j) MT_LAM { return row(own(ch, j)).meta; });
        lp = wave_map(n, [&](int j) MT_LAM { return row(own(ch, j)).props; });
        lr = wave_map(n, [&](int j) MT_LAM { return row(own(ch, j)).len; });
        return wave_map(n, [&](int j) MT_LAM {
            const int s = own(ch, j);
            const uint32_t mt = own(lm, j);
            const int rs = row(s).rseq;
            ChildL o;
            o.len = vis_rc(row(s).seq, mt, rs, row(s).rcl, row(s).ovl, r, c, ovx, ovxN, s) ? row(s).len : 0;
            // breakTie for a leaf at pos 0 (MT/mergeTree.ts:2270-2292): false if a
            // removal the author has seen (removedSeq <= refSeq); true otherwise
            // (every row has an assigned seq on the replay path).
            o.tie = !((mt & MT_M_REMOVED) && rs <= r);
            return o;
        });
#endif
    }
    // Perspective lengths of block B's children (nodeLength, MT/mergeTree.ts:1652-1692).
    // lsN >= 0 (MT_RES_BIG descents): only the lsN U entries listed in ulist lie under B.
    MT_HD LaneArr<ChildL> childLens(int B, const BlkH& h, const LaneArr<int>& ch, int r, int c,
                                    bool haveLen = false, const LaneArr<int>& kl = LaneArr<int>{}, int lsN = -1) {
        if (h.height == 0) {
            LaneArr<uint32_t> lm; LaneArr<int> lp, lr;
            return leafLens(ch, h.n, r, c, lm, lp, lr);
        }
        if constexpr (BT) {                              // the children's corrections from the table
            return wave_map(h.n, [&](int j) MT_LAM {
                const int b = own(ch, j);
                ChildL o; o.len = bk(b).len + LB().bcorr[b]; o.tie = true; return o;
            });
        } else return childLensU(B, h, ch, r, c, haveLen, kl, lsN);
    }
    // The U-scan form (every residency but block residency).
    MT_HD LaneArr<ChildL> childLensU(int B, const BlkH& h, const LaneArr<int>& ch, int r, int c,
                                     bool haveLen, const LaneArr<int>& kl, int lsN) {
        if constexpr (BIG) {
            if (htOk) {                                  // the children's corrections from the table
                return wave_map(h.n, [&](int j) MT_LAM {
                    const int b = own(ch, j);
                    ChildL o; o.len = (haveLen ? own(kl, j) : bk(b).len) + htGet(b); o.tie = true; return o;
                });
            }
        }
        // Each U row (one per lane) finds the child it lies under and adds its
        // delta into that child's LDS slot.
        const int hc = h.height - 1, n = h.n;
        int cid[MT_MAXN];
#pragma unroll
        for (int j = 0; j < MT_MAXN; j++) cid[j] = j < n ? wave_at(ch, j) : -2;
        wave_for(MT_MAXN, [&](int j) MT_LAM { sc->corr[j] = 0; });
        wave_sync();
        bool listed = false;
        if constexpr (BIG) {
            if (lsN >= 0) {
                listed = true;
                for (int base = 0; base < lsN; base += MT_WAVE) {
                    const int m = (lsN - base) < MT_WAVE ? (lsN - base) : MT_WAVE;
                    wave_for(m, [&](int k) MT_LAM {
                        const int u = mt_ldsg().ulist[base + k];
                        const int a = mt_ldsg().uanc[u * MT_G_H + hc];
                        int jk = -1;
#pragma unroll
                        for (int j = 0; j < MT_MAXN; j++) if (cid[j] == a) jk = j;
                        if (jk >= 0) lds_add(&sc->corr[jk], mt_ldsg().udelta[u]);
                    });
                }
            }
        }
        if (!listed) {
            forU([&](auto inL, int base, int m) MT_LAM {
                constexpr bool L = decltype(inL)::value;
                wave_for(m, [&](int k) MT_LAM {
                    const int a = ancGetAt<L>(base + k, hc);
                    int jk = -1;
#pragma unroll
                    for (int j = 0; j < MT_MAXN; j++) if (cid[j] == a) jk = j;
                    if (jk >= 0) lds_add(&sc->corr[jk], udAt<L>(base + k));
                });
            });
        }
        wave_sync();
        return wave_map(n, [&](int j) MT_LAM {
            ChildL o; o.len = (haveLen ? own(kl, j) : bk(own(ch, j)).len) + sc->corr[j]; o.tie = true; return o;
        });
    }

    // MT_RES_BIG descents: the U entries (of the list, or all when lsN < 0) whose ancestor
    // at level hc is `child`, compacted into ulist; returns their count.  A walk then
    // scans only the U rows under its current block instead of all of U at every level.
    MT_HD int narrowU(int lsN, int hc, int child) {
        const int n0 = lsN < 0 ? nU : lsN;
        int w = 0;
        for (int base = 0; base < n0; base += MT_WAVE) {
            const int m = (n0 - base) < MT_WAVE ? (n0 - base) : MT_WAVE;
            auto u = wave_map(m, [&](int k) MT_LAM { return lsN < 0 ? base + k : (int)mt_ldsg().ulist[base + k]; });
            auto keep = wave_map(m, [&](int k) MT_LAM { return mt_ldsg().uanc[own(u, k) * MT_G_H + hc] == child; });
            const auto rk = wave_rank(keep);
            const int cnt = wave_count(keep), w0 = w;
            wave_sync();                                  // in place: the chunk is read before it is rewritten
            wave_for(m, [&](int k) MT_LAM { if (own(keep, k)) mt_ldsg().ulist[w0 + own(rk, k)] = (uint16_t)own(u, k); });
            w += cnt;
        }
        wave_sync();
        return w;
    }

    /* ---------------------------------- overlap side list (clients >= 63) -- */
    // Drop entries whose row was unlinked, recycled or settled below the MSN (its
    // overlap can no longer change any perspective's view); lane-parallel compaction.
    MT_HD void ovxCompact() {
        int w = 0;
        for (int base = 0; base < ovxN; base += MT_WAVE) {
            const int m = (ovxN - base) < MT_WAVE ? (ovxN - base) : MT_WAVE;
            auto keep = wave_map(m, [&](int k) MT_LAM {
                const MtOvx e = ovx[base + k];
                return (bool)((int)(row(e.row).parent >= 0) & (int)(row(e.row).rseq == e.rseq) & (int)(e.rseq > minSeq));
            });
            auto ent = wave_map(m, [&](int k) MT_LAM { return ovx[base + k]; });
            auto rk = wave_rank(keep);
            const int cnt = wave_count(keep);
            wave_sync();
            const int w0 = w;
            wave_for(m, [&](int k) MT_LAM { if (own(keep, k)) ovx[w0 + own(rk, k)] = own(ent, k); });
            wave_sync();
            w += cnt;
        }
        ovxN = w;
    }
    MT_HD void ovxAdd(int s, int rseq, int c) {
        if (ovxN >= MT_OVX_CAP) ovxCompact();
        if (ovxN >= MT_OVX_CAP) { status |= MT_DS_OOM_OVERLAP; return; }
        MtOvx e; e.row = s; e.rseq = rseq; e.client = c; e.pad = 0;
        wave_for(1, [&](int) MT_LAM { ovx[ovxN] = e; });
        ovxN++;
    }
    // A split's right half n inherits row s's side-list entries.
    MT_HD void ovxCopy(int s, int n) {
        const int rs = uni(row(s).rseq), n0 = ovxN;
        for (int base = 0; base < n0; base += MT_WAVE) {
            const int m = (n0 - base) < MT_WAVE ? (n0 - base) : MT_WAVE;
            auto hit = wave_map(m, [&](int k) MT_LAM { const MtOvx e = ovx[base + k]; return e.row == s && e.rseq == rs; });
            auto cl = wave_map(m, [&](int k) MT_LAM { return ovx[base + k].client; });
            uint64_t b = wave_ballot(hit);
            while (b) {
                const int k = __builtin_ctzll(b); b &= b - 1;
                ovxAdd(n, rs, wave_at(cl, k));
            }
        }
    }

    /* ----------------------------------------------- structure edits -- */
    // Row split (BaseSegment.splitAt MT/mergeTree.ts:538-582; TextSegment
    // createSplitSegmentAt textSegment.ts:103-111): the right half copies every
    // attribute; the property map is immutable here, so both halves share it.
    MT_HD int splitRow(int s, int pos) {
        MT_EV2(5, 1);
        const int n = allocRow();
        if (n < 0) return -1;
#if defined(MT_DBG_FAIL) && defined(__HIP_DEVICE_COMPILE__)
        mt_dbg_v.s = s; mt_dbg_v.n = n; mt_dbg_v.op = curOp;
#endif
        const int ls = uni(row(s).len);
        const uint32_t mt = uni(row(s).meta);
        row(n).len = ls - pos; row(s).len = pos;
        const unsigned long long ov = uni64(row(s).ovl);
        row(n).seq = row(s).seq; row(n).rseq = row(s).rseq; row(n).meta = mt & ~(MT_M_INWIN | MT_M_HREF); row(n).ovl = ov;
        row(n).rcl = row(s).rcl; row(n).mid = 0;
        if (ov >> 63) ovxCopy(s, n);
        row(n).toff = row(s).toff + pos; row(n).props = row(s).props; row(n).parent = row(s).parent;
        row(n).tcap = row(s).tcap - pos; row(s).tcap = pos;   // each row owns [toff, toff+tcap) of the arena
        if (mt & MT_M_INWIN) winAddKnown(n, mt & ~(MT_M_INWIN | MT_M_HREF));   // n's meta as just written
        return n;
    }
    // splitRow with row s already loaded (lane j of lf, the walk's leaf step): the right half is
    // written by twelve lanes in one store (one dword each) and nothing of s is read again.
    // dword k of a row held in registers (k a compile-time constant after unrolling: no address
    // is taken, so the record stays in VGPRs)
    MT_HD static int rowDword(const MtRow& f, int k) {
        switch (k) {
            case 0: return f.len; case 1: return f.seq; case 2: return f.rseq; case 3: return (int)f.meta;
            case 4: return f.toff; case 5: return f.props; case 6: return f.parent; case 7: return f.tcap;
            case 8: return (int)(uint32_t)f.ovl; case 9: return (int)(uint32_t)(f.ovl >> 32);
            case 10: return (int)f.rcl; default: return f.mid;
        }
    }
    MT_HD static LaneArr<int> leafField(const LaneArr<MtRow>& lf, int j, int k) {
        (void)j;
        return wave_map(MT_WAVE, [&](int t) MT_LAM { return rowDword(own(lf, t), k); });
    }
    MT_HD int splitRowKnown(int s, int pos, const LaneArr<MtRow>& lf, int j) {
        MT_EV2(5, 1);
        const int n = allocRow();
        if (n < 0) return -1;
#if defined(MT_DBG_FAIL) && defined(__HIP_DEVICE_COMPILE__)
        mt_dbg_v.s = s; mt_dbg_v.n = n; mt_dbg_v.op = curOp;
#endif
        const uint32_t mt = (uint32_t)wave_at(leafField(lf, j, 3), j);
        const uint32_t ovh = (uint32_t)wave_at(leafField(lf, j, 9), j);
        // lane j holds row s: it writes the right half whole (three 16-byte stores)
        wave_for(MT_WAVE, [&](int t) MT_LAM {
            if (t != j) return;
            MtRow q = own(lf, t);
            q.len -= pos; q.meta &= ~(MT_M_INWIN | MT_M_HREF); q.toff += pos; q.tcap -= pos; q.mid = 0;
            row(n) = q;
        });
        row(s).len = pos; row(s).tcap = pos;                   // each row owns [toff, toff+tcap) of the arena
        if (ovh >> 31) ovxCopy(s, n);
        if (mt & MT_M_INWIN) winAddKnown(n, mt & ~(MT_M_INWIN | MT_M_HREF));   // n's meta as just written
        return n;
    }
    // Insert `node` at child index idx of path level L, splitting full blocks
    // 4/4 upward (insertingWalk :2465-2489, split :2495-2508, updateRoot :1868).
    // `delta` = observer length added under the path (0 for a row split).
    MT_HD void insertAtPath(int L, int idx, int node, int delta) {
        bool first = true;
        for (;;) {
            const int B = uni(sc->pathB[L]);
            BlkH h;
            auto cur = blkLoad(B, h);
            auto prv = wave_from8<-1>(cur);
            const int nd = node, ix = idx;
            // branch-free blend: a ?: chain here gets turned into a select of
            // closure-field addresses, which forces the closure into scratch
            auto nc = wave_map(8, [=](int i) MT_LAM {
                const int a = own(cur, i), b = own(prv, i);
                const int lt = -(int)(i < ix), eq = -(int)(i == ix);
                return (a & lt) | (nd & eq) | (b & ~(lt | eq));
            });
            const int n1 = h.n + 1;
            setChildParent(h.height, node, B);
            if (first) landB = B;
            if (n1 < MT_MAXN) {
                wave_for(8, [&](int i) MT_LAM { bk(B).c[i] = i < n1 ? own(nc, i) : -1; });
                bk(B).n = n1; bk(B).len = h.len + delta;
                // ancestors on the path: one lane per level (distinct blocks), one round trip
                if (delta != 0) wave_for(L, [&](int l) MT_LAM { const int pb = sc->pathB[l]; bk(pb).len = bk(pb).len + delta; });
                return;
            }
            lastSplit = true;
            MT_EV(6, 1);
            const int NB = allocBlock();
            if (NB < 0) return;
            auto hi = wave_from8<4>(nc);
            wave_for(8, [&](int i) MT_LAM {
                bk(NB).c[i] = i < 4 ? own(hi, i) : -1;
                bk(B).c[i] = i < 4 ? own(nc, i) : -1;
            });
            bk(NB).n = 4; bk(NB).height = h.height; bk(NB).scour = -1; bk(NB).parent = h.parent;
            bpPut(NB, h.parent);
            bk(B).n = 4;
            wave_for(4, [&](int i) MT_LAM { setChildParent(h.height, own(hi, i), NB); });
            if (first && ix >= 4) landB = NB;
            first = false;
            wave_sync();
            const int nbLen = sumObs(NB, 4, h.height), bLen = sumObs(B, 4, h.height);
            bk(NB).len = nbLen; bk(B).len = bLen;
            if (L == 0) {
                const int R = allocBlock();
                if (R < 0) return;
                wave_for(8, [&](int i) MT_LAM { bk(R).c[i] = i == 0 ? B : (i == 1 ? NB : -1); });
                bk(R).n = 2; bk(R).height = h.height + 1; bk(R).parent = -1; bk(R).scour = -1; bk(R).len = bLen + nbLen;
                bk(B).parent = R; bk(NB).parent = R;
                bpPut(R, -1); bpPut(B, R); bpPut(NB, R);
                root = R; height = h.height + 1;
                return;
            }
            node = NB; idx = uni(sc->pathJ[L - 1]) + 1; L = L - 1;
        }
    }
#if defined(MT_DBG_FAIL) && defined(__HIP_DEVICE_COMPILE__)
    // Diagnostic builds only: a walk found no position.  Prints the walk's view of the
    // block's children beside fresh (volatile, after a full wait) reloads of the same records.
    __device__ void dbgWalkFail(int kind, int B, const BlkH& h, int ch, const ChildL& cl, int pos, int p, int total, int L,
                                int r, int c) {
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        const int lane = wave_lane();
        if (lane == 0)
            printf("WALKFAIL op=%u kind=%d B=%d height=%d n=%d hlen=%d L=%d root=%d H=%d pos=%d p=%d total=%d r=%d c=%d "
                   "minSeq=%d curSeq=%d uValid=%d nU=%d lastSplit(s=%d n=%d op=%u)\n",
                   curOp, kind, B, h.height, h.n, h.len, L, root, height, pos, p, total, r, c, minSeq, curSeq, (int)uValid, nU,
                   mt_dbg_v.s, mt_dbg_v.n, mt_dbg_v.op);
        if (lane < h.n) {
            if (h.height == 0) {
                const volatile MtRow* v = (const volatile MtRow*)&row(ch);
                const int ln = v->len, sq = v->seq, rs = v->rseq, par = v->parent;
                const uint32_t mt = v->meta, rc = v->rcl;
                const unsigned long long ov = v->ovl;
                const bool vis = vis_rc(sq, mt, rs, rc, ov, r, c, ovx, ovxN, ch);
                printf("  WALKFAIL child %d row=%d used_len=%d tie=%d | fresh len=%d seq=%d rseq=%d meta=%x rcl=%u ovl=%llx "
                       "parent=%d vis=%d\n", lane, ch, cl.len, (int)cl.tie, ln, sq, rs, mt, rc, ov, par, (int)vis);
            } else {
                int corr = 0;
                if constexpr (BT) corr = LB().bcorr[ch];
                const volatile MtBlk* v = (const volatile MtBlk*)&bk(ch);
                printf("  WALKFAIL child %d blk=%d used_len=%d | bk.len=%d bcorr=%d n=%d parent=%d height=%d\n", lane, ch, cl.len,
                       v->len, corr, v->n, v->parent, v->height);
            }
        }
    }
#endif
    // insertingWalk (MT/mergeTree.ts:2363-2493) for one remote op perspective.  L0 > 0
    // resumes at level L0 of the previous walk's path (pathB/pathJ/pathOff above L0 still
    // valid, U unchanged): the root descent would pick the same children down to there.
    MT_HD int walk(int kind, int pos, int r, int c, int cand, int candLen, int L0 = 0) {
        if (!(uValid && uRef == r && uCli == c)) { computeU(r, c, false); L0 = 0; }
        int B = root, L = 0, p = pos;
        if (L0 > 0) { B = uni(sc->pathB[L0]); L = L0; p = pos - uni(sc->pathOff[L0]); }
        const bool narrow = BIG && nU <= UCAP && !htOk;   // U entries all in LDS: narrow them per level
        int lsN = -1;
        BlkH h;
        MT_QB(q0); MT_QC(2);
        auto ch = blkLoad(B, h);
        MT_QE(0, q0);
        for (;;) {
            MT_EV(5, 1);
            sc->pathB[L] = B;
            MT_QB(q1);
            // blocks in HBM: children's records (lengths + the next level's block) in one trip
            const bool kpre = !BLKL && h.height > 0;
            LaneArr<int> r0{}, r1{};
            if (kpre) kidsLoad(ch, h.n, r0, r1);
            // Leaf rows: every field in one round trip (MtRow is three 16-byte loads per lane), so a
            // split that follows needs no second load of the row (splitRowKnown).
            LaneArr<MtRow> lf{};
            LaneArr<ChildL> cl;
            if (MT_LEAF_ONCE && h.height == 0) {
                const int rr = r, cc = c;
                lf = wave_map(h.n, [&](int j) MT_LAM { return row(own(ch, j)); });
                cl = wave_map(h.n, [&](int j) MT_LAM {
                    const MtRow f = own(lf, j);
                    ChildL o;
                    o.len = vis_rc(f.seq, f.meta, f.rseq, f.rcl, f.ovl, rr, cc, ovx, ovxN, own(ch, j)) ? f.len : 0;
                    o.tie = !((f.meta & MT_M_REMOVED) && f.rseq <= rr);     // breakTie, as leafLens
                    return o;
                });
            } else cl = kpre ? childLens(B, h, ch, r, c, true, kidsLen(r0, r1), lsN) : childLens(B, h, ch, r, c);
            MT_QE(1, q1);
            auto lens = wave_map(h.n, [&](int j) MT_LAM { return own(cl, j).len; });
            auto pre = wave_excl_scan8(lens);
            const int total = wave_sum8(lens);
            sc->pathOff[L] = pos - p; sc->pathLen[L] = total;
            const bool interior = h.height > 0;
            auto cond = wave_map(h.n, [&](int j) MT_LAM {
                const int pj = p - own(pre, j), lj = own(cl, j).len;
                if (interior) return pj <= lj;                       // breakTie: blocks always
                return pj < lj || (pj == lj && pj == 0 && own(cl, j).tie);
            });
            const int j = wave_first(cond);
            if (j >= 0) {
                const int pj = p - wave_at(pre, j);
                if (interior) {
                    sc->pathJ[L] = j; L++; B = wave_at(ch, j); p = pj;
                    if (narrow && h.height > 1) lsN = narrowU(lsN, h.height - 1, B);
                    if (kpre) ch = kidRec(r0, r1, j, h, B); else ch = blkLoad(B, h);
                    continue;
                }
                const int s = wave_at(ch, j);
                lastL = L; lastSplit = false;
                if (kind == MT_WALK_SPLIT) {
                    const uint32_t sm = MT_LEAF_ONCE ? (uint32_t)wave_at(leafField(lf, j, 3), j) : uni(row(s).meta);
                    if (pj > 0 && !(sm & MT_M_MARKER)) {
                        const int n = MT_LEAF_ONCE ? splitRowKnown(s, pj, lf, j) : splitRow(s, pj);
                        if (n < 0) return MT_W_FAIL;
                        insertAtPath(L, j + 1, n, 0);
                        if (FULL && drec) {                     // SPLIT, splitLeafSegment (mergeTree.ts:2243-2258)
                            const int ps = obsPosition(s);
                            const bool rm = (uni(row(s).meta) & MT_M_REMOVED) != 0;
                            emitDelta(MT_DK_SPLIT, ps, pj, s, n, uni(row(n).len));
                            (void)rm;
                        }
                        lastIdx = j + 1;                      // an insert at pos lands before the new right half
                        // A row split keeps every row under the same ancestors unless a
                        // block split moved some: U's per-ancestor delta sums stay exact
                        // (s's delta covers both halves), so U stays valid.
                        if (lastSplit) uValid = false;
                        return MT_W_OK;
                    }
                    lastIdx = j;
                    return MT_W_NOCHANGE;
                }
                insertAtPath(L, j, cand, candLen);           // onLeaf: candidate goes before the found row
                uValid = false;
                return MT_W_OK;
            }
            if (p - total == 0) {
                lastL = L; lastIdx = h.n; lastSplit = false;
                if (kind == MT_WALK_SPLIT) return MT_W_NOCHANGE;
                insertAtPath(L, h.n, cand, candLen);          // position used up at a block end: append
                uValid = false;
                return MT_W_OK;
            }
#if defined(MT_DBG_FAIL) && defined(__HIP_DEVICE_COMPILE__)
            dbgWalkFail(kind, B, h, ch, cl, pos, p, total, L, r, c);
#endif
            return MT_W_FAIL;
        }
    }

    /* --------------------------------------------------------- zamboni -- */
    // Heap.add + fixup (collections.ts:238-251).  A heap of <= 63 entries is sifted
    // wave-parallel (lane k = slot k): one load round, a ballot, stores to the moved slots only.
    MT_HD void heapAdd(int s, int ms) {
        if (heapN + 1 > (int)S.heapCap) { status |= MT_DS_OOM_HEAP; return; }
        int k = ++heapN;
        if (heapN > heapHW) heapHW = heapN;
        if (heapN < MT_WAVE) {
            // Sift-up in one step: the parents on the path from the root to slot n hold
            // non-decreasing keys, so the entries that move down one slot (parent key > ms) are
            // the path's lowest ones; each path lane loads its parent once (no readlane chain).
            const int n = heapN, dn = 31 - __builtin_clz((unsigned)n);
            auto mv = wave_map(n + 1, [&](int c) MT_LAM {
                c = mt_opaque(c);
                const int dc = 31 - __builtin_clz((unsigned)(c | 1));
                return (bool)((int)(c >= 2) & (int)((n >> (dn - dc)) == c));
            });
            auto pms = wave_map(n + 1, [&](int c) MT_LAM { return own(mv, c) ? (int)hp(mt_opaque(c) >> 1).maxSeq : 0; });
            auto psg = wave_map(n + 1, [&](int c) MT_LAM { return own(mv, c) ? (int)hp(mt_opaque(c) >> 1).seg : 0; });
            mv = wave_map(n + 1, [&](int c) MT_LAM { return own(mv, c) && own(pms, c) > ms; });
            const int top = wave_first(mv);
            k = top < 0 ? n : top >> 1;
            wave_for(n + 1, [&](int c) MT_LAM {
                if (own(mv, c)) { hp(c).seg = own(psg, c); hp(c).maxSeq = own(pms, c); }
                if (c == k) { hp(c).seg = s; hp(c).maxSeq = ms; }
            });
            if (k == 1) heapTop = ms;
            return;
        }
        while (k > 1) {
            const int pm = uni(hp(k >> 1).maxSeq);
            if (pm > ms) { hp(k).seg = hp(k >> 1).seg; hp(k).maxSeq = pm; k >>= 1; } else break;
        }
        hp(k).seg = s; hp(k).maxSeq = ms;
        if (k == 1) heapTop = ms;
    }
    MT_HD MtHeapE heapGet() {                                 // Heap.get + fixdown, collections.ts:230-268
        MT_EV(3, 1); MT_EV(7, heapN - 1);
        if (heapN < MT_WAVE) {
            // Fix-down as a pointer chase: every slot i computes in parallel the child j(i) the
            // reference's loop would take (the left one on ties) and whether the moving last
            // entry would pass it (key > the child's); the wave then follows j from the root,
            // one readlane per level, and the slots on the path take their child's entry.
            const int N = heapN, n = N - 1;
            MtHeapE x; x.seg = uni(hp(1).seg); x.maxSeq = uni(hp(1).maxSeq);
            const int lseg = uni(hp(N).seg), lms = uni(hp(N).maxSeq);
            heapN = n;
            heapTop = 0x7FFFFFFF;
            if (n >= 1) {
                auto lm = wave_map(n + 1, [&](int i) MT_LAM { return (int)(i >= 1) & (int)(2 * i <= n) ? (int)hp(2 * mt_opaque(i)).maxSeq : 0; });
                auto rm = wave_map(n + 1, [&](int i) MT_LAM { return (int)(i >= 1) & (int)(2 * i < n) ? (int)hp(2 * mt_opaque(i) + 1).maxSeq : 0; });
                auto ls = wave_map(n + 1, [&](int i) MT_LAM { return (int)(i >= 1) & (int)(2 * i <= n) ? (int)hp(2 * mt_opaque(i)).seg : 0; });
                auto rs = wave_map(n + 1, [&](int i) MT_LAM { return (int)(i >= 1) & (int)(2 * i < n) ? (int)hp(2 * mt_opaque(i) + 1).seg : 0; });
                auto right = wave_map(n + 1, [&](int i) MT_LAM { return (bool)((int)(2 * i < n) & (int)(own(lm, i) > own(rm, i))); });
                auto cm = wave_map(n + 1, [&](int i) MT_LAM { return own(right, i) ? own(rm, i) : own(lm, i); });
                auto cs = wave_map(n + 1, [&](int i) MT_LAM { return own(right, i) ? own(rs, i) : own(ls, i); });
                auto nx = wave_map(n + 1, [&](int i) MT_LAM {
                    return (int)(i >= 1) & (int)(2 * i <= n) & (int)(own(cm, i) < lms) ? 2 * i + (int)own(right, i) : 0;
                });
                int k = 1;
                for (int t = wave_at(nx, 1); t != 0; t = wave_at(nx, t)) { MT_EV(4, 1); k = t; }
                const int dk = 31 - __builtin_clz((unsigned)k);
                wave_for(n + 1, [&](int i) MT_LAM {
                    if (i < 1 || i > k) return;
                    const int di = 31 - __builtin_clz((unsigned)i);
                    if ((k >> (dk - di)) != i) return;
                    if (i == k) { hp(i).seg = lseg; hp(i).maxSeq = lms; }
                    else { hp(i).seg = own(cs, i); hp(i).maxSeq = own(cm, i); }
                });
                heapTop = k == 1 ? lms : wave_at(cm, 1);
            }
            return x;
        }
        MtHeapE x; x.seg = uni(hp(1).seg); x.maxSeq = uni(hp(1).maxSeq);
        const int lseg = uni(hp(heapN).seg), lms = uni(hp(heapN).maxSeq);
        heapN--;
        heapTop = 0x7FFFFFFF;
        if (heapN >= 1) {
            int k = 1;
            heapTop = lms;
            while ((k << 1) <= heapN) {
                int j = k << 1;
                int hs = uni(hp(j).seg), hm = uni(hp(j).maxSeq);
                if (j < heapN) {
                    const int hm1 = uni(hp(j + 1).maxSeq);
                    if (hm > hm1) { j++; hs = uni(hp(j).seg); hm = hm1; }
                }
                if (lms <= hm) break;
                MT_EV(4, 1);
                if (k == 1) heapTop = hm;
                hp(k).seg = hs; hp(k).maxSeq = hm; k = j;
            }
            hp(k).seg = lseg; hp(k).maxSeq = lms;
        }
        return x;
    }
    MT_HD void addToLRUSet(int s, int sq) {                   // MT/mergeTree.ts:1262-1272
        if (!(sq > curSeq)) return;
        const int p = uni(row(s).parent);
        const uint32_t m = uni(row(s).meta);
        if (uni(bk(p).scour) != 1 && sq > curSeq) {
            bk(p).scour = 1;
            if ((m & MT_M_HREF) != MT_M_HREF) row(s).meta = m + MT_M_HREF1;   // saturated: never recycled
            heapAdd(s, sq);
        }
    }
    MT_HD void addToLRUSetKnown(int s, int sq, int p, uint32_t m) {
        if (!(sq > curSeq)) return;
        if (uni(bk(p).scour) != 1) {
            bk(p).scour = 1;
            if ((m & MT_M_HREF) != MT_M_HREF) row(s).meta = m + MT_M_HREF1;
            heapAdd(s, sq);
        }
    }
    MT_HD int pkey(int id, int i) const { return (int)pset[id + (i >> 4)].key[i & 15]; }
    MT_HD int pval(int id, int i) const { return pset[id + (i >> 4)].val[i & 15]; }
    // matchProperties class of a stored value: NaN, undefined and fresh consensus objects
    // (the values below 0) equal nothing, themselves included (MT_VAL_*, include/mtgpu.h).
    MT_HD uint32_t pclass(int v) const { return v >= 0 ? S.p_class[v] : 0xFFFFFFFFu; }
    // A map holding such a value matches no map, itself included (pset[id].pad[2], written
    // only while the document has one: MtCold::pNever).
    MT_HD bool pNeverMap(int a) const { return mt_cold_v.pNever && a >= 0 && uni(pset[a].pad[2]) != 0; }
    MT_HD bool propsMatch(int a, int b) {                      // matchProperties, MT/properties.ts:64-95
        if (a == b) return !pNeverMap(a);
        if (a < 0 || b < 0) return false;
        const int na = uni(pset[a].n), nb = uni(pset[b].n);
        if (na != nb) return false;
        if constexpr (FULL) {
            if (__builtin_expect(na > MT_WAVE, 0)) return propsMatchWide(a, b, na);
        } else if (na > MT_WAVE) { status |= MT_DS_PROPS_TOO_MANY; return false; }   // wide maps: FULL only
        auto ok = wave_map(na, [&](int k) MT_LAM {               // a's keys one per lane
            const int key = pkey(a, k);
            const uint32_t ca = pclass(pval(a, k));
            bool f = false;
            for (int i = 0; i < nb; i++) f |= (int)(pkey(b, i) == key) & (int)(pclass(pval(b, i)) == ca);
            return (f & (int)(ca != 0xFFFFFFFFu)) != 0;
        });
        return wave_count(ok) == na;
    }
    // ... for maps of more than 64 keys (equal counts n): a's keys in chunks of 64 lanes
    MT_HD bool propsMatchWide(int a, int b, int n) {
        for (int base = 0; base < n; base += MT_WAVE) {
            const int cnt = (n - base) < MT_WAVE ? (n - base) : MT_WAVE;
            auto ok = wave_map(cnt, [&](int k) MT_LAM {
                const int key = pkey(a, base + k);
                const uint32_t ca = pclass(pval(a, base + k));
                bool f = false;
                for (int i = 0; i < n; i++) f |= (int)(pkey(b, i) == key) & (int)(pclass(pval(b, i)) == ca);
                return (f & (int)(ca != 0xFFFFFFFFu)) != 0;
            });
            if (wave_count(ok) != cnt) return false;
        }
        return true;
    }
    // Text-arena compaction: copy the text of every linked row into the other
    // half of the document's arena (rows are immutable slices, so garbage from
    // relocated or unlinked rows accumulates until the half is full).
    MT_HD void textGC() {
        MT_EV2(4, 1);
        MT_PB(t0);
        const int other = textHalf ^ 1;
        uint16_t* dst = S.textBase + (size_t)other * S.textCap;
        int w = 0;
        for (int base = 0; base < rowTop; base += MT_WAVE) {
            const int m = (rowTop - base) < MT_WAVE ? (rowTop - base) : MT_WAVE;
            auto ln = wave_map(m, [&](int k) MT_LAM {
                const int s = base + k;
                const uint32_t mt = row(s).meta;
                const int ln = row(s).len;
                return (((row(s).parent >= 0) | ((mt & MT_M_REG) != 0)) & !(mt & MT_M_MARKER)) ? ln : 0;
            });
            auto pre = wave_excl_scan(ln);
            const int tot = wave_sum(ln);
            wave_for(m, [&](int k) MT_LAM {
                const int s = base + k, l = own(ln, k);
                if (l <= 0) return;
                const int o = w + own(pre, k), t0 = row(s).toff;
                lane_copy16(dst + o, text + t0, l);
                row(s).toff = o; row(s).tcap = l;
            });
            w += tot;
        }
        wave_sync();
        textHalf = other; text = dst; textTop = w; gcEpoch++;
        MT_PE(MT_PH_TEXT, t0);
    }
    // Reserve n units at the top of the live half (compacting first if needed).
    MT_HD int textAlloc(int n) {
        if (textTop + n > (int)S.textCap) textGC();
        if (textTop + n > (int)S.textCap) { status |= MT_DS_OOM_TEXT; return -1; }
        const int o = textTop; textTop += n; return o;
    }
    // text[dst, dst + Σ len) = the concatenation of up to 9 pieces: an optional head piece
    // (hsrc, hlen), then the text of lanes [i0, i1) of (src, len), 64 units a pass (one
    // load round trip per pass however many pieces).
    MT_HD void gatherText(int dst, int hsrc, int hlen, const LaneArr<int>& src, const LaneArr<int>& len, int i0, int i1) {
        int n = hlen;
        for (int i = i0; i < i1; i++) n += wave_at(len, i);
        MT_EV2(2, n); MT_EV2(3, 1);
        // piece of unit q: scan the (<= 9) piece prefixes, all scalar
        auto srcOf = [&](int base, int m) MT_LAM {
            auto from = wave_map(m, [&](int k) MT_LAM { const int q = base + k; return q < hlen ? hsrc + q : -1; });
            int pre = hlen;
            for (int i = i0; i < i1; i++) {
                const int ps = wave_at(src, i), pl = wave_at(len, i), p0 = pre;
                from = wave_map(m, [&](int k) MT_LAM {
                    const int q = base + k, f0 = own(from, k);
                    return (q >= p0 && q < p0 + pl) ? ps + (q - p0) : f0;
                });
                pre += pl;
            }
            return from;
        };
        // The destination never overlaps a source (a new region, or the head's slack past its
        // text), so MT_GT_CH chunks of 64 units are loaded before any is stored: one round trip
        // per MT_GT_CH * 64 units instead of one per 64.
        for (int base = 0; base < n; base += MT_GT_CH * MT_WAVE) {
            LaneArr<int> v[MT_GT_CH];
#pragma unroll
            for (int u = 0; u < MT_GT_CH; u++) {
                const int b = base + u * MT_WAVE;
                if (b >= n) break;                                   // uniform: skips the piece scan too
                const int m = (n - b) < MT_WAVE ? (n - b) : MT_WAVE;
                const auto from = srcOf(b, m);
                v[u] = wave_map(m, [&](int k) MT_LAM { return (int)text[own(from, k)]; });
            }
            wave_sync();
#pragma unroll
            for (int u = 0; u < MT_GT_CH; u++) {
                const int b = base + u * MT_WAVE;
                if (b >= n) break;
                const int m = (n - b) < MT_WAVE ? (n - b) : MT_WAVE;
                wave_for(m, [&](int k) MT_LAM { text[dst + b + k] = (uint16_t)own(v[u], k); });
            }
        }
        wave_sync();
    }
    // One zamboni merge run (TextSegment.append, textSegment.ts:74-85, applied for each
    // follower in order): head lane h takes the text of follower lanes [i0, i1).  The
    // head owns [toff, toff + tcap) of the arena: followers whose text already sits right
    // after the head's (split halves coming back together) extend it in place; the rest
    // are copied into the head's slack, or head and rest move together to a new region
    // of twice the size (amortized O(appended units)).  Returns the head's new length.
    MT_HD int mergeRun(const LaneArr<int>& f, LaneArr<int>& ft, LaneArr<int>& fc, const LaneArr<int>& fl,
                       int h, int i0, int i1) {
        MT_ZB(z2);
        const int hr = wave_at(f, h);
        int tp = wave_at(ft, h), lp = wave_at(fl, h), cp = wave_at(fc, h);
        int i = i0;
        for (; i < i1; i++) {                              // in place: no copy
            const int ts = wave_at(ft, i);
            if (!(ts == tp + lp && cp == lp)) break;
            cp = lp + wave_at(fc, i); lp += wave_at(fl, i);
        }
        if (i < i1) {
            int rest = 0;
            for (int j = i; j < i1; j++) rest += wave_at(fl, j);
            if (lp + rest <= cp) {
                gatherText(tp + lp, 0, 0, ft, fl, i, i1);
            } else {
                int nc = 2 * (lp + rest); if (nc < 16) nc = 16;
                if (textTop + nc > (int)S.textCap) {
                    // compaction moves every linked row's text (head and followers apart
                    // again, slack gone): the whole run is copied, exactly sized
                    textGC();
                    ft = wave_map(8 * MT_MAXN, [&](int t) MT_LAM { const int g = own(f, t); return g >= 0 ? row(g).toff : 0; });
                    fc = wave_map(8 * MT_MAXN, [&](int t) MT_LAM { const int g = own(f, t); return g >= 0 ? row(g).tcap : 0; });
                    tp = wave_at(ft, h); lp = wave_at(fl, h); i = i0;
                    rest = 0;
                    for (int j = i; j < i1; j++) rest += wave_at(fl, j);
                    nc = lp + rest;
                }
                const int o = textAlloc(nc);
                if (o < 0) { MT_ZE(2, z2); return lp; }
                gatherText(o, tp, lp, ft, fl, i, i1);
                tp = o; cp = nc;
            }
            lp += rest;
        }
        row(hr).len = lp; row(hr).toff = tp; row(hr).tcap = cp;
        MT_ZE(2, z2);
        return lp;
    }
    // scourNode (MT/mergeTree.ts:1278-1356) for leaf blocks blks[0..nb) (a lane array,
    // nb <= 7; lane t holds child slot t&7 of block t>>3): kept children are appended to
    // sc->hold from nh, with their observer lengths in sc->holdLen; returns the new hold
    // count.  Each block is scoured separately (prev restarts at every block).
    //
    // The reference walks the children with a `prev` cursor.  Here every decision that
    // does not depend on the walk is made lane-parallel: unlink (removed at or below the
    // MSN), held (removed above it, or inserted above it: prev resets), candidate
    // (inserted at or below it), and whether candidate k may append to the run ending at
    // k-1 (canAppend's marker / trailing "\n" / empty tests and matchProperties).  Only
    // the 256-unit granularity rule depends on the run's accumulated length; a short
    // scalar loop over the lanes in mergeable runs decides it.  Text then moves once per
    // run (mergeRun), and unlinks, frees and the hold list are lane-parallel writes.
    MT_HD int scourLeaves(const LaneArr<int>& blks, int nb, int nh) {
        const int span = 8 * nb;
        const auto bsel = wave_gather8(blks);       // block id by lane shuffle (per-block scalar arrays spilled)
        auto f = wave_map(span, [&](int t) MT_LAM {
            const int b = own(bsel, t);
            return (t & 7) < bk(b).n ? bk(b).c[t & 7] : -1;
        });
#if MT_SCOUR_QUADS
        // the fields below are the row's first two quads (len seq rseq meta | toff props parent
        // tcap): two 16-byte loads per lane instead of seven dword loads
        const auto q0 = wave_map(span, [&](int j) MT_LAM {
            const int g = own(f, j);
            return g >= 0 ? ((const MtQ16a*)&row(g))[0] : MtQ16a{0u, 0u, 0u, 0u};
        });
        const auto q1 = wave_map(span, [&](int j) MT_LAM {
            const int g = own(f, j);
            return g >= 0 ? ((const MtQ16a*)&row(g))[1] : MtQ16a{0u, 0u, 0u, 0u};
        });
        auto fl = wave_map(span, [&](int j) MT_LAM { return (int)own(q0, j).x; });
        auto fs = wave_map(span, [&](int j) MT_LAM { return (int)own(q0, j).y; });
        auto fr = wave_map(span, [&](int j) MT_LAM { return (int)own(q0, j).z; });
        auto fm = wave_map(span, [&](int j) MT_LAM { return (int)own(q0, j).w; });
        auto ft = wave_map(span, [&](int j) MT_LAM { return (int)own(q1, j).x; });
        auto fp = wave_map(span, [&](int j) MT_LAM { return (int)own(q1, j).y; });
        auto fc = wave_map(span, [&](int j) MT_LAM { return (int)own(q1, j).w; });
#else
        auto fm = wave_map(span, [&](int j) MT_LAM { const int g = own(f, j); return g >= 0 ? (int)row(g).meta : 0; });
        auto fs = wave_map(span, [&](int j) MT_LAM { const int g = own(f, j); return g >= 0 ? row(g).seq : 0; });
        auto fr = wave_map(span, [&](int j) MT_LAM { const int g = own(f, j); return g >= 0 ? row(g).rseq : 0; });
        auto fl = wave_map(span, [&](int j) MT_LAM { const int g = own(f, j); return g >= 0 ? row(g).len : 0; });
        auto fp = wave_map(span, [&](int j) MT_LAM { const int g = own(f, j); return g >= 0 ? row(g).props : 0; });
        auto ft = wave_map(span, [&](int j) MT_LAM { const int g = own(f, j); return g >= 0 ? row(g).toff : 0; });
        auto fc = wave_map(span, [&](int j) MT_LAM { const int g = own(f, j); return g >= 0 ? row(g).tcap : 0; });
#endif
        const int ms = minSeq;
        // class: 0 empty, 1 unlink, 2 held removed, 3 held above the MSN, 4 candidate
        auto cls = wave_map(span, [&](int t) MT_LAM {
            if (own(f, t) < 0) return 0;
            const uint32_t mt = (uint32_t)own(fm, t);
            if (mt & MT_M_REMOVED) return own(fr, t) <= ms ? 1 : 2;
            return own(fs, t) <= ms ? 4 : 3;
        });
        c_scour += (uint32_t)wave_count(wave_map(span, [&](int t) MT_LAM { return own(cls, t) != 0; }));
        // k may append to k-1 (same block): both candidates, both non-empty, neither a marker
        auto okPrev = wave_map(span, [&](int t) MT_LAM {
            return (own(cls, t) == 4 && own(fl, t) > 0 && !((uint32_t)own(fm, t) & MT_M_MARKER)) ? 1 : 0;
        });
        const auto okPrev1 = wave_from8<-1>(okPrev), fp1 = wave_from8<-1>(fp);
        auto pair = wave_map(span, [&](int t) MT_LAM { return ((t & 7) != 0 && own(okPrev, t) && own(okPrev1, t)) ? 1 : 0; });
        uint64_t pm = wave_ballot(wave_map(span, [&](int t) MT_LAM { return own(pair, t) != 0; }));
        uint64_t merged = 0;
        auto runLen = fl;                                // a run head's final length
        if (pm) {
            // prev's last unit (canAppend: no trailing "\n") for lanes followed by a pair
            const uint64_t needLast = pm >> 1;
            const auto need = wave_map(span, [&](int t) MT_LAM {
                return (((needLast >> t) & 1ull) != 0) & !((uint32_t)own(fm, t) & MT_M_NONL);
            });
            auto lastNL = wave_map(span, [&](int) MT_LAM { return 0; });
            if (wave_ballot(wave_map(span, [&](int t) MT_LAM { return (bool)own(need, t); })))   // uniform skip
                lastNL = wave_map(span, [&](int t) MT_LAM {              // per lane branch-free
                    const bool q = own(need, t);
                    const int last = (int)text[q ? own(ft, t) + own(fl, t) - 1 : 0];
                    return (q & (last == '\n')) ? 1 : 0;
                });
            const auto lastNL1 = wave_from8<-1>(lastNL);
            // matchProperties: equal ids match; a missing map never matches a present one;
            // two different maps compare key by key (propsMatch)
            const uint64_t slow = wave_ballot(wave_map(span, [&](int t) MT_LAM {
                const int a = own(fp1, t), b = own(fp, t);
                return ((pm >> t) & 1ull) && a != b && a >= 0 && b >= 0;
            }));
            uint64_t propOk = wave_ballot(wave_map(span, [&](int t) MT_LAM {
                const int a = own(fp1, t), b = own(fp, t);
                return a == b;
            }));
            if (mt_cold_v.pNever)                        // a shared map holding NaN / undefined
                propOk &= ~wave_ballot(wave_map(span, [&](int t) MT_LAM {
                    const int a = own(fp1, t), b = own(fp, t);
                    const bool q = (((pm >> t) & 1ull) != 0) & (a == b) & (a >= 0);
                    return (bool)(q & (pset[q ? a : 0].pad[2] != 0));
                }));
            for (uint64_t sb = slow; sb; sb &= sb - 1) {
                const int k = __builtin_ctzll(sb);
                if (propsMatch(wave_at(fp1, k), wave_at(fp, k))) propOk |= 1ull << k;
            }
            pm &= propOk & ~wave_ballot(wave_map(span, [&](int t) MT_LAM { return own(lastNL1, t) != 0; }));
            // the granularity rule: prev.len <= 256 || seg.len <= 256 on the accumulated run
            const uint64_t bigF = wave_ballot(wave_map(span, [&](int t) MT_LAM {
                return ((pm >> t) & 1ull) && own(fl, t) > MT_GRAN;
            }));
            if (!bigF) {
                // every follower is short, so every pair merges whatever the run's length: the
                // runs are the pairs' chains, and a head's length is a prefix-sum difference
                merged = pm;
                const uint64_t heads = (pm | (pm >> 1)) & ~pm;
                const auto fl0 = wave_map(MT_WAVE, [&](int t) MT_LAM { return t < span ? own(fl, t) : 0; });
                const auto S = wave_excl_scan(fl0);                      // units before lane t
                const uint64_t mg = merged;
                // S at the first lane past the run (runs end inside the span, 8 * nb <= 56 lanes)
                const auto Se = wave_shfl(S, [mg](int t) MT_LAM {
                    const uint64_t after = t < 63 ? (mg >> (t + 1)) : 0ull;
                    const int e = t + 1 + __builtin_ctzll(~after);
                    return e < 64 ? e : 63;
                });
                runLen = wave_map(span, [&](int t) MT_LAM {
                    return ((heads >> t) & 1ull) ? own(Se, t) - own(S, t) : own(fl, t);
                });
            } else {
                uint64_t walk = pm | (pm >> 1);
                int P = 0, head = -1;
                while (walk) {
                    const int k = __builtin_ctzll(walk);
                    walk &= walk - 1;
                    const int lk = wave_at(fl, k);
                    if (((pm >> k) & 1ull) && (P <= MT_GRAN || lk <= MT_GRAN)) { merged |= 1ull << k; P += lk; }
                    else {
                        if (head >= 0) runLen = wave_set(runLen, head, P);
                        head = k; P = lk;
                    }
                }
                if (head >= 0) runLen = wave_set(runLen, head, P);
            }
            // move the text, one run at a time (followers still linked: compaction keeps their text)
            for (uint64_t m = merged; m;) {
                const int i0 = __builtin_ctzll(m);
                int i1 = i0;
                while ((m >> i1) & 1ull) i1++;
                m &= ~((i1 >= 64 ? ~0ull : ((1ull << i1) - 1ull)));
                mergeRun(f, ft, fc, fl, i0 - 1, i0, i1);
                {   // the appended text may carry a newline: the head keeps the flag only if all did
                    const uint32_t hm = (uint32_t)wave_at(fm, i0 - 1);
                    if (hm & MT_M_NONL) {
                        bool all = true;
                        for (int i = i0; i < i1; i++) all = all && ((uint32_t)wave_at(fm, i) & MT_M_NONL);
                        if (!all) row(wave_at(f, i0 - 1)).meta = hm & ~MT_M_NONL;
                    }
                }
            }
        }
        if (FULL && drec) { // maintenance callbacks in child order: UNLINK (:1299-1305), APPEND (:1325-1331)
            const uint64_t unl = wave_ballot(wave_map(span, [&](int t) MT_LAM { return own(cls, t) == 1; }));
            int head = -1, acc = 0;
            for (uint64_t b = unl | merged | (merged >> 1); b; b &= b - 1) {
                const int k = __builtin_ctzll(b);
                if ((unl >> k) & 1ull) { const int g = wave_at(f, k); emitDelta(MT_DK_UNLINK, obsPosition(g), wave_at(fl, k), g, -1, -1); }
                else if ((merged >> k) & 1ull) {                   // prevSegment's length after this append
                    const int hg = wave_at(f, head), g = wave_at(f, k), lk = wave_at(fl, k);
                    acc += lk;
                    emitDelta(MT_DK_APPEND, obsPosition(hg), acc, hg, g, lk);
                } else { head = k; acc = wave_at(fl, k); }
            }
        }
        // unlinked and appended rows leave the tree; rows no heap entry or window refers
        // to go back on the recycled-row stack (in lane order)
        auto gone = wave_map(span, [&](int t) MT_LAM { return own(cls, t) == 1 || ((merged >> t) & 1ull); });
        auto freeable = wave_map(span, [&](int t) MT_LAM {
            return own(gone, t) && !((uint32_t)own(fm, t) & (MT_M_HREF | MT_M_INWIN));
        });
        const auto rkF = wave_rank(freeable);
        const int nF = wave_count(freeable), f0 = rfN;
        wave_for(span, [&](int t) MT_LAM {
            if (!own(gone, t)) return;
            row(own(f, t)).parent = -1;
            if (own(freeable, t) && f0 + own(rkF, t) < MT_RFL) sc->rfree[f0 + own(rkF, t)] = own(f, t);
        });
        rfN = (f0 + nF) < MT_RFL ? (f0 + nF) : MT_RFL;
        // kept children in order, with their observer lengths
        auto keep = wave_map(span, [&](int t) MT_LAM { return own(cls, t) >= 2 && !((merged >> t) & 1ull); });
        const auto rkK = wave_rank(keep);
        const int nK = wave_count(keep), h0 = nh;
        wave_for(span, [&](int t) MT_LAM {
            if (!own(keep, t)) return;
            const int c = own(cls, t);
            sc->hold[h0 + own(rkK, t)] = own(f, t);
            sc->holdLen[h0 + own(rkK, t)] = c == 2 ? 0 : (c == 4 ? own(runLen, t) : own(fl, t));
            sc->holdBlk[h0 + own(rkK, t)] = (uint8_t)(t >> 3);
        });
        wave_sync();
        return nh + nK;
    }
    // blockUpdatePathLengths(..., newStructure); firstLen >= 0: B's length is known.
    MT_HD void updatePathLens(int B, int firstLen = -1) {
        while (B >= 0) {
            MT_EV2(1, 1);
            const BlkH h = head(B);
            bk(B).len = firstLen >= 0 ? firstLen : sumObs(B, h.n, h.height);
            firstLen = -1;
            B = h.parent;
        }
    }
    MT_HD void packParent(int P) {                            // MT/mergeTree.ts:1359-1410
        MT_EV2(0, 1);
        for (;;) {
            BlkH ph;
            auto pch = blkLoad(P, ph);
            int nh = 0;
            const int chh = ph.height - 1;                       // children of P are blocks of this height
            if (chh == 0) { MT_ZB(z4); nh = scourLeaves(pch, ph.n, 0); MT_ZE(4, z4); }
            else {
                for (int i = 0; i < ph.n; i++) {
                    const int cb = wave_at(pch, i);
                    const int n = uni(bk(cb).n), base = nh;
                    wave_for(n, [&](int k) MT_LAM {
                        const int g = bk(cb).c[k];
                        sc->hold[base + k] = g; sc->holdLen[base + k] = bk(g).len; sc->holdBlk[base + k] = (uint8_t)i;
                    });
                    nh += n;
                }
            }
            int cc = nh / (MT_MAXN / 2); if (cc > MT_MAXN - 1) cc = MT_MAXN - 1; if (cc < 1) cc = 1;
            // New block ni < min(cc, n) is old child ni (block ids are internal: any assignment
            // gives the same tree), so a child dealt to the group of its own old block keeps its
            // parent field and is not written (about half of them); the other old children are
            // freed, and blocks beyond n come off the free list (rare).
            const int reuse = cc < ph.n ? cc : ph.n;
            const int pn = ph.n;
            for (int i = reuse; i < pn; i++) freeBlock(wave_at(pch, i));
            auto nbid = wave_shfl(pch, [=](int ni) MT_LAM { return ni < reuse ? ni : 0; });
            for (int ni = reuse; ni < cc; ni++) {            // more blocks than P had (rare)
                const int NB = allocBlock();
                if (NB < 0) return;
                nbid = wave_set(nbid, ni, NB);
            }
            wave_sync();
            // New block ni takes hold[st(ni), st(ni) + cnt(ni)): the first `extra` blocks one child
            // more than `base`.  All blocks at once: lane t writes slot t & 7 of block t >> 3 (and
            // its child's parent), then lane ni block ni's header.
            const int base = nh / cc, extra = nh % cc;
            const auto nb8 = wave_gather8(nbid);
            // the old block of each dealt child (lane t: slot t & 7 of new block t >> 3)
            const auto oi = wave_map(8 * cc, [&](int t) MT_LAM {
                const int ni = t >> 3, slot = t & 7;
                const int cnt = base + (ni < extra ? 1 : 0), st = ni * base + (ni < extra ? ni : extra);
                return slot < cnt ? (int)sc->holdBlk[st + slot] : 0;
            });
            const auto ob = wave_shfl(pch, [&](int t) MT_LAM { return own(oi, t) & 7; });
            wave_for(8 * cc, [&](int t) MT_LAM {
                const int ni = t >> 3, slot = t & 7;
                const int cnt = base + (ni < extra ? 1 : 0), st = ni * base + (ni < extra ? ni : extra);
                const int ch = slot < cnt ? sc->hold[st + slot] : -1;
                const int NB = own(nb8, t);
                bk(NB).c[slot] = ch;
                if ((int)(ch >= 0) & (int)(own(ob, t) != NB)) setChildParent(chh, ch, NB);
            });
            wave_for(cc, [&](int ni) MT_LAM {
                const int cnt = base + (ni < extra ? 1 : 0), st = ni * base + (ni < extra ? ni : extra);
                const int NB = own(nbid, ni);
                int len = 0;
                for (int k = 0; k < MT_MAXN; k++) len += k < cnt ? sc->holdLen[st + k] : 0;
                bk(NB).n = cnt; bk(NB).height = chh; bk(NB).parent = P; bk(NB).scour = -1; bk(NB).len = len;
                bpPut(NB, P);
            });
            wave_for(8, [&](int i) MT_LAM { bk(P).c[i] = i < cc ? own(nbid, i) : -1; });
            bk(P).n = cc;
            wave_sync();
            if (cc < MT_MAXN / 2 && ph.parent >= 0) { P = ph.parent; continue; }
            // The reference refreshes the path here (blockUpdatePathLengths, :1406) for its
            // partial lengths; observer lengths cannot have changed (see zamboniInner).
            return;
        }
    }
    MT_HD void zamboni() {                                    // MT/mergeTree.ts:1412-1468
        MT_PB(t0);
        MT_ZB(z0);
        zamboniInner();
        MT_ZE(0, z0);
        MT_PE(MT_PH_ZAMBONI, t0);
    }
    MT_HD void zamboniInner() {
        for (int i = 0; i < MT_ZMAX; i++) {
            if (heapN == 0 || heapTop > minSeq) break;
            uValid = false;                                   // scour/pack may restructure
            MT_EV2(6, 1);
            MT_QB(q0); MT_QC(6);
            MT_ZB(z5); MT_ZC(7);
            // the popped row's parent and meta are loaded before the sift (which touches only
            // the heap), so their round trip overlaps it
            const int s0 = uni(hp(1).seg);
            const int pv = row(s0).parent;
            const uint32_t mv = row(s0).meta;
            const MtHeapE e = heapGet();
            MT_ZE(5, z5);
            MT_QE(5, q0);
            const int p = uni(pv);
            uint32_t em = uni(mv);
            if ((em & MT_M_HREF) != MT_M_HREF) { em -= MT_M_HREF1; row(e.seg).meta = em; }
            if (p < 0 && !(em & (MT_M_HREF | MT_M_INWIN))) freeRow(e.seg);
            if (p >= 0 && uni(bk(p).scour) != 0) {
                const BlkH h = head(p);
                MT_QB(q1);
                MT_ZB(z1);
                const int nh = scourLeaves(wave_map(1, [&](int) MT_LAM { return p; }), 1, 0);
                MT_ZE(1, z1);
                MT_QE(7, q1);
                MT_ZB(z6);
                bk(p).scour = 0;
                if (nh < h.n) {
                    wave_for(8, [&](int j) MT_LAM { bk(p).c[j] = j < nh ? sc->hold[j] : -1; });
                    bk(p).n = nh;
                    wave_sync();
                    // A scour keeps every block's observer length: unlinked rows were removed
                    // (length 0 in the observer's view) and a merged run keeps its sum, so the
                    // reference's blockUpdatePathLengths (:1456-1460; it rebuilds partial
                    // lengths, which this engine does not keep) changes no observer length here.
                    if (nh < MT_MAXN / 2 && h.parent >= 0) { MT_ZB(z3); packParent(h.parent); MT_ZE(3, z3); }
                }
                MT_ZE(6, z6);
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
    // Keys live one per lane (insertion order).
    // pm: MT_PM_SET / MT_PM_REWRITE, or a combining op (MT_PM_INCR; MT_PM_KEEP for consensus
    // and other names): opset is then a combine set whose values are what combine yields
    // for a key the segment does not hold (include/mtgpu.h), and a held key's new value
    // follows from its old one (segmentPropertiesManager.ts:98-109, properties.ts:24-62).
    // combine(op, previousValue, undefined, seq) for one key: pv the held value (MT_VAL_UNDEF:
    // not held, a held undefined counts as not held), code what combine yields without one.
    // Incr of a number / boolean / NaN is NaN, of a string / array / object (a fresh consensus
    // object included) the interned String(v) + "undefined"; consensus keeps the value unless it
    // is an object whose seq is -1 (shared by every segment split from the one it was set on);
    // other names keep it.  MT_VAL_UNSUP after setting the document's status (UNSUPPORTED or
    // THROWS).
    MT_HD int combineValue(int pv, int code, int pm, int sq) {
        int nv = code;
        if (pv != MT_VAL_UNDEF) {
            const int vi = pv >= 0 ? uni(S.p_vinfo[pv]) : (pv == MT_VAL_NAN ? MT_VAL_NAN : uni(S.p_vinfo[-1]));
            if (pm == MT_PM_INCR || pm == MT_PM_INCR_SMIN) {
                const int sid = vi & MT_VINFO_ID;
                nv = vi == MT_VAL_NAN ? MT_VAL_NAN
                                      : ((vi < 0 || sid == MT_VINFO_NONE || pm == MT_PM_INCR_SMIN) ? MT_VAL_UNSUP : sid);
            } else if (pm == MT_PM_CONS) nv = (pv >= 0 && vi >= 0 && (vi & MT_VINFO_SEQM1)) ? MT_VAL_UNSUP : pv;
            else nv = pv;
        }
        if (nv == MT_VAL_CFRESH) nv = (sq >= 0 && sq <= 0x7FFFFFEF) ? MT_VAL_CONS(sq) : MT_VAL_UNSUP;   // -16 - seq fits int32
        if (nv == MT_VAL_THROW) { status |= MT_DS_THROWS; return MT_VAL_UNSUP; }
        if (nv == MT_VAL_UNSUP) status |= MT_DS_UNSUPPORTED;
        return nv;
    }
    // Whether key `key` survives a rewrite by op set [o0, o1): the set gives it a truthy value.
    MT_HD bool rewriteKeeps(int key, int o0, int o1) const {
        bool kp = false;
        for (int q = o0; q < o1; q++) if ((int)S.p_key[q] == key) { const int nv = S.p_val[q]; kp = nv >= 0 && !S.p_falsy[nv]; }
        return kp;
    }
    // applyPropSet past one key per lane (the old map and the op set together above MT_WAVE
    // keys): the new map is built in place in the pool at psetTop, chunk by chunk, and
    // committed at the end (nothing is allocated on an early return).
    MT_HD int applyPropSetWide(int old, int opset, int pm, int sq) {
        const int n0 = old >= 0 ? uni(pset[old].n) : 0;
        const int o0 = uni((int)S.p_off[opset]), o1 = uni((int)S.p_off[opset + 1]);
        const int room = (n0 + (o1 - o0)) < MT_PKEYS ? n0 + (o1 - o0) : MT_PKEYS;
        const int chCap = room > MT_PSK ? (room + MT_PSK - 1) / MT_PSK : 1;
        if (psetTop + chCap > (int)S.psetCap) { status |= MT_DS_OOM_PROPS; return old; }
        if (pm >= MT_PM_INCR && !S.p_vinfo) { status |= MT_DS_UNSUPPORTED; return old; }
        const int id = psetTop;
        int n = 0;
        for (int base = 0; base < n0; base += MT_WAVE) {          // the old map (rewrite: the kept keys)
            const int cnt = (n0 - base) < MT_WAVE ? (n0 - base) : MT_WAVE;
            const auto k = wave_map(cnt, [&](int i) MT_LAM { return pkey(old, base + i); });
            const auto v = wave_map(cnt, [&](int i) MT_LAM { return pval(old, base + i); });
            const auto keep = wave_map(cnt, [&](int i) MT_LAM { return pm != MT_PM_REWRITE || rewriteKeeps(own(k, i), o0, o1); });
            const auto rk = wave_rank(keep);
            const int m = n;
            wave_for(cnt, [&](int i) MT_LAM {
                if (own(keep, i)) { const int j = m + own(rk, i); pset[id + (j >> 4)].key[j & 15] = (uint16_t)own(k, i); pset[id + (j >> 4)].val[j & 15] = own(v, i); }
            });
            n += wave_count(keep);
        }
        wave_sync();
        for (int q = o0; q < o1; q++) {
            const int key = uni((int)S.p_key[q]);
            int nv = uni((int)S.p_val[q]);
            int at = -1;
            for (int base = 0; base < n && at < 0; base += MT_WAVE) {
                const int cnt = (n - base) < MT_WAVE ? (n - base) : MT_WAVE;
                const int f = wave_first(wave_map(cnt, [&](int i) MT_LAM { return pkey(id, base + i) == key; }));
                if (f >= 0) at = base + f;
            }
            if (pm >= MT_PM_INCR) {
                nv = combineValue(at >= 0 ? uni(pval(id, at)) : MT_VAL_UNDEF, nv, pm, sq);
                if (nv == MT_VAL_UNSUP) return old;
            }
            if (nv == MT_VAL_NULL) {
                if (at >= 0) {                                     // the keys after it move down one
                    for (int base = at; base < n - 1; base += MT_WAVE) {
                        const int cnt = (n - 1 - base) < MT_WAVE ? (n - 1 - base) : MT_WAVE;
                        const auto k = wave_map(cnt, [&](int i) MT_LAM { return pkey(id, base + i + 1); });
                        const auto v = wave_map(cnt, [&](int i) MT_LAM { return pval(id, base + i + 1); });
                        wave_sync();
                        wave_for(cnt, [&](int i) MT_LAM {
                            const int j = base + i;
                            pset[id + (j >> 4)].key[j & 15] = (uint16_t)own(k, i); pset[id + (j >> 4)].val[j & 15] = own(v, i);
                        });
                        wave_sync();
                    }
                    n--;
                }
            } else if (at >= 0) {
                wave_for(1, [&](int) MT_LAM { pset[id + (at >> 4)].val[at & 15] = nv; });
            } else {
                if (n >= MT_PKEYS) { status |= MT_DS_PROPS_TOO_MANY; return old; }
                const int j = n;
                wave_for(1, [&](int) MT_LAM { pset[id + (j >> 4)].key[j & 15] = (uint16_t)key; pset[id + (j >> 4)].val[j & 15] = nv; });
                n++;
            }
            wave_sync();
        }
        const int nch = n > MT_PSK ? (n + MT_PSK - 1) / MT_PSK : 1;
        int never = 0;
        if (pm >= MT_PM_INCR || mt_cold_v.pNever)
            for (int base = 0; base < n; base += MT_WAVE) {
                const int cnt = (n - base) < MT_WAVE ? (n - base) : MT_WAVE;
                never |= wave_ballot(wave_map(cnt, [&](int i) MT_LAM { return pval(id, base + i) < 0; })) ? 1 : 0;
            }
        if (never) mt_cold_v.pNever = 1;
        wave_for(nch * MT_PSK - n, [&](int i) MT_LAM { const int j = n + i; pset[id + (j >> 4)].key[j & 15] = 0; pset[id + (j >> 4)].val[j & 15] = 0; });
        wave_for(nch, [&](int k) MT_LAM { pset[id + k].n = n; pset[id + k].pad[2] = never; });
        wave_sync();
        psetTop += nch;
        return id;
    }
    MT_HD int applyPropSet(int old, int opset, int pm, int sq = 0) {
        if (opset < 0 || opset >= (int)S.p_nsets) { status |= MT_DS_UNSUPPORTED; return old; }
        int n = old >= 0 ? uni(pset[old].n) : 0;
        // maps past a wave's lanes are built by the FULL kernels only: the host replays a batch in
        // them once one of its documents has named more than MT_WAVE distinct keys (mt_ctx::batch_wide)
        if constexpr (FULL) {
            if (__builtin_expect(n + (uni((int)S.p_off[opset + 1]) - uni((int)S.p_off[opset])) > MT_WAVE, 0))
                return applyPropSetWide(old, opset, pm, sq);
        } else if (n > MT_WAVE) { status |= MT_DS_PROPS_TOO_MANY; return old; }
        auto kk = wave_map(n, [&](int i) MT_LAM { return pkey(old, i); });
        auto vv = wave_map(n, [&](int i) MT_LAM { return pval(old, i); });
        const int o0 = uni((int)S.p_off[opset]), o1 = uni((int)S.p_off[opset + 1]);
        if (pm == MT_PM_REWRITE && n > 0) {
            auto keep = wave_map(n, [&](int i) MT_LAM { return rewriteKeeps(own(kk, i), o0, o1); });
            auto rk = wave_rank(keep);
            const int cntk = wave_count(keep);
            // compaction through the hold scratch (free here: no scour or collect is in flight)
            wave_for(n, [&](int i) MT_LAM { if (own(keep, i)) { sc->hold[own(rk, i)] = own(kk, i); sc->holdLen[own(rk, i)] = own(vv, i); } });
            wave_sync();
            n = cntk;
            kk = wave_map(n, [&](int i) MT_LAM { return sc->hold[i]; });
            vv = wave_map(n, [&](int i) MT_LAM { return sc->holdLen[i]; });
            wave_sync();
        }
        if (pm >= MT_PM_INCR && !S.p_vinfo) { status |= MT_DS_UNSUPPORTED; return old; }
        for (int q = o0; q < o1; q++) {
            const int key = uni((int)S.p_key[q]);
            int nv = uni((int)S.p_val[q]);
            const int at = wave_first(wave_map(n, [&](int i) MT_LAM { return own(kk, i) == key; }));
            if (pm >= MT_PM_INCR) {
                nv = combineValue(at >= 0 ? wave_at(vv, at) : MT_VAL_UNDEF, nv, pm, sq);
                if (nv == MT_VAL_UNSUP) return old;
            }
            if (nv == MT_VAL_NULL) {
                if (at >= 0) {
                    auto k1 = wave_from(kk, 1), v1 = wave_from(vv, 1);
                    kk = wave_map(MT_WAVE, [&](int i) MT_LAM { const int a = own(kk, i), b = own(k1, i); return i < at ? a : b; });
                    vv = wave_map(MT_WAVE, [&](int i) MT_LAM { const int a = own(vv, i), b = own(v1, i); return i < at ? a : b; });
                    n--;
                }
            } else if (at >= 0) {
                vv = wave_map(MT_WAVE, [&](int i) MT_LAM { return i == at ? nv : own(vv, i); });
            } else {
                // FULL: n + (o1 - o0) <= MT_WAVE here; otherwise the document's keys number <= MT_WAVE
                if constexpr (!FULL) if (n >= MT_WAVE) { status |= MT_DS_PROPS_TOO_MANY; return old; }
                const int at2 = n;
                kk = wave_map(MT_WAVE, [&](int i) MT_LAM { return i == at2 ? key : own(kk, i); });
                vv = wave_map(MT_WAVE, [&](int i) MT_LAM { return i == at2 ? nv : own(vv, i); });
                n++;
            }
        }
        const int nn = n, nch = nn > MT_PSK ? (nn + MT_PSK - 1) / MT_PSK : 1;
        if (psetTop + nch > (int)S.psetCap) { status |= MT_DS_OOM_PROPS; return old; }
        const int id = psetTop;
        psetTop += nch;
        // never-equal values (NaN, undefined, fresh consensus objects; made by a combining op
        // or kept from the old map) mark the map
        const int never = (pm >= MT_PM_INCR || mt_cold_v.pNever) &&
                          wave_ballot(wave_map(nn, [&](int i) MT_LAM { return own(vv, i) < 0; })) ? 1 : 0;
        if (never) mt_cold_v.pNever = 1;
        wave_for(nch * MT_PSK, [&](int i) MT_LAM {
            pset[id + (i >> 4)].key[i & 15] = (uint16_t)(i < nn ? own(kk, i) : 0);
            pset[id + (i >> 4)].val[i & 15] = i < nn ? own(vv, i) : 0;
        });
        wave_for(nch, [&](int k) MT_LAM { pset[id + k].n = nn; pset[id + k].pad[2] = never; });
        return id;
    }

    // The property map of a new segment made from op prop set `opset` alone (TextSegment.make /
    // Marker.make -> addProperties on undefined properties).  Maps are immutable and never freed,
    // so segments made from the same set share one: a direct-mapped memo of the last maps made
    // (per bind) instead of a new map per insert.
    MT_HD int newPropMap(int opset) {
        const int k = opset & 3;
        if (mt_cold_v.pcKey[k] == opset) return mt_cold_v.pcVal[k];
        const int id = applyPropSet(-1, opset, MT_PM_SET);
        if (status) return id;
        mt_cold_v.pcKey[k] = opset; mt_cold_v.pcVal[k] = id;
        return id;
    }

    /* ----------------------------------------------------- range walks -- */
    // nodeMap over [start, end) under (r, c) with the remove / annotate leaf
    // action and post-order length maintenance (MT/mergeTree.ts:2626-2739,
    // :2584-2624, :2927-2994).  Child lengths are evaluated before the child is
    // touched, as in the reference's in-order traversal.  The frame stack lives in
    // lanes (lane L = level L: readlane/writelane, no LDS round trips): block, next
    // child, start/end relative to the block, the child's length, the observer-length
    // delta under the block and (delta capture) the block's observer-view position.
    // L0 > 0: the range lies under path block pathB[L0] of the last walks (the deepest block
    // both boundary walks passed through, tree unchanged since): the root walk would visit
    // only that branch above it, so the walk starts there and the observer-length change is
    // added to the ancestors above.  Delta capture starts at the root (observer offsets).
    MT_HD void rangeMap(int mode, int start, int end, int r, int c, int sq, int opset, int pm, int L0 = 0) {
        if (!(uValid && uRef == r && uCli == c)) { computeU(r, c, false); L0 = 0; }
        const bool rec = FULL && drec != nullptr;
        if (rec) L0 = 0;
        LaneArr<int> fB{}, fJ{}, fS{}, fE{}, fL{}, fD{}, fO{};
        const int off0 = L0 > 0 ? uni(sc->pathOff[L0]) : 0;
        fB = wave_set(fB, 0, L0 > 0 ? uni(sc->pathB[L0]) : root); fS = wave_set(fS, 0, start - off0);
        fE = wave_set(fE, 0, end - off0);
        int lastOld = -2, lastNew = -1, topD = 0;
        int L = 0;
        while (L >= 0) {
            const int B = wave_at(fB, L);
            BlkH h;
            auto ch = blkLoad(B, h);
            LaneArr<uint32_t> lm{}; LaneArr<int> lp{}, lr{};
            auto cl = h.height == 0 ? leafLens(ch, h.n, r, c, lm, lp, lr) : childLens(B, h, ch, r, c);
            auto lens = wave_map(h.n, [&](int j) MT_LAM { return own(cl, j).len; });
            const int j0 = wave_at(fJ, L);
            auto lensFrom = wave_map(h.n, [&](int j) MT_LAM { return j >= j0 ? own(lens, j) : 0; });
            auto pre = wave_excl_scan8(lensFrom);
            const int st = wave_at(fS, L), en = wave_at(fE, L);
            auto cond = wave_map(h.n, [&](int j) MT_LAM {
                const int lj = own(lens, j), pj = own(pre, j);
                return j >= j0 && (en - pj) > 0 && lj > 0 && (st - pj) < lj;
            });
            if (h.height == 0) {
                MT_EV2(7, 1);
                const int first = wave_first(cond);
                int obsDelta = 0;
                if (first >= 0) {
                    const int nact = wave_count(cond);
                    c_rows += 2ull * (uint64_t)nact;
                    if (mode == MT_MAP_COLLECT) {                      // cloneSegments' gatherSegment (:1599-1604)
                        const auto rk = wave_rank(cond);
                        const int k0 = regTop + nCol;               // into the register arena's free tail
                        wave_for(h.n, [&](int j) MT_LAM {
                            if ((int)own(cond, j) & (int)(k0 + own(rk, j) < regCap)) regRow(k0 + own(rk, j)) = own(ch, j);
                        });
                        nCol += nact;
                    } else if (mode == MT_MAP_REMOVE) {
                        auto nd = wave_map(h.n, [&](int j) MT_LAM {
                            if (!own(cond, j)) return 0;
                            const int s = own(ch, j);
                            const uint32_t mt = own(lm, j);
                            if (mt & MT_M_REMOVED) {                   // overlapping remove: keep first remover
                                row(s).ovl = row(s).ovl | (1ull << (c < 63 ? c : 63));
                                return 0;
                            }
                            row(s).meta = mt | MT_M_REMOVED;
                            row(s).rcl = (uint32_t)c;
                            row(s).rseq = sq;
                            return own(lr, j);
                        });
                        obsDelta = -wave_sum8(nd);
                        wave_sync();
                        if (c >= 63) {                                 // removedClientOverlap beyond the mask
                            const uint64_t ob = wave_ballot(wave_map(h.n, [&](int j) MT_LAM {
                                return (bool)((int)own(cond, j) & (int)(row(own(ch, j)).rseq != sq));
                            }));
                            for (uint64_t b = ob; b; b &= b - 1) {
                                const int j = __builtin_ctzll(b), s = wave_at(ch, j);
                                ovxAdd(s, uni(row(s).rseq), c);
                            }
                        }
                        winAddLanes(ch, cond, h.n);
                        if (rec) {                                     // removedSegments: newly removed only
                            const int base = wave_at(fO, L);
                            auto ol = wave_map(h.n, [&](int j) MT_LAM {
                                const int g = own(ch, j); return (row(g).meta & MT_M_REMOVED) ? 0 : row(g).len;
                            });
                            auto opre = wave_excl_scan8(ol);
                            for (uint64_t b = wave_ballot(wave_map(h.n, [&](int j) MT_LAM { return own(nd, j) > 0; })); b; b &= b - 1) {
                                const int j = __builtin_ctzll(b);
                                emitDelta(MT_DK_REMOVE, base + wave_at(opre, j), wave_at(nd, j), wave_at(ch, j), -1, -1);
                            }
                        }
                    } else {
                        LaneArr<int> opre{};
                        int base = 0;
                        if (rec) {
                            base = wave_at(fO, L);
                            auto ol = wave_map(h.n, [&](int j) MT_LAM {
                                const int g = own(ch, j); return (row(g).meta & MT_M_REMOVED) ? 0 : row(g).len;
                            });
                            opre = wave_excl_scan8(ol);
                        }
                        for (int j = 0; j < h.n; j++) {
                            if (!wave_at(cond, j)) continue;
                            const int s = wave_at(ch, j);
                            const int old = wave_at(lp, j);
                            int nw;
                            if (old == lastOld) nw = lastNew;
                            else { nw = applyPropSet(old, opset, pm, sq); lastOld = old; lastNew = nw; }
                            row(s).props = nw;
                            if (rec) emitDelta(MT_DK_ANNOTATE, base + wave_at(opre, j), uni(row(s).len), s, old, nw);
                        }
                    }
                    if (mode != MT_MAP_COLLECT) addToLRUSet(wave_at(ch, first), sq);
                }
                if (mode == MT_MAP_REMOVE) bk(B).len = h.len + obsDelta;
                const int d = wave_at(fD, L) + obsDelta;
                L--;
                if (L < 0) topD = d;
                if (L >= 0) {
                    const int fl = wave_at(fL, L);
                    fD = wave_set(fD, L, wave_at(fD, L) + d); fS = wave_set(fS, L, wave_at(fS, L) - fl);
                    fE = wave_set(fE, L, wave_at(fE, L) - fl); fJ = wave_set(fJ, L, wave_at(fJ, L) + 1);
                }
                continue;
            }
            const int jj = wave_first(cond);
            if (jj >= 0) {
                const int pj = wave_at(pre, jj);
                fS = wave_set(fS, L, st - pj); fE = wave_set(fE, L, en - pj); fJ = wave_set(fJ, L, jj);
                fL = wave_set(fL, L, wave_at(lens, jj));
                int ob = 0;
                if (rec) ob = wave_at(fO, L) + wave_sum8(wave_map(h.n, [&](int i) MT_LAM { return i < jj ? bk(own(ch, i)).len : 0; }));
                const int child = wave_at(ch, jj);
                L++;
                fB = wave_set(fB, L, child); fJ = wave_set(fJ, L, 0); fS = wave_set(fS, L, st - pj);
                fE = wave_set(fE, L, en - pj); fD = wave_set(fD, L, 0); fO = wave_set(fO, L, ob);
                continue;
            }
            const int d = wave_at(fD, L);
            if (d != 0) bk(B).len = h.len + d;
            L--;
            if (L < 0) topD = d;
            if (L >= 0) {
                const int fl = wave_at(fL, L);
                fD = wave_set(fD, L, wave_at(fD, L) + d); fS = wave_set(fS, L, wave_at(fS, L) - fl);
                fE = wave_set(fE, L, wave_at(fE, L) - fl); fJ = wave_set(fJ, L, wave_at(fJ, L) + 1);
            }
        }
        if (L0 > 0 && topD != 0) {                           // ancestors above the start block: one lane each
            const int dd = topD;
            wave_for(L0, [&](int l) MT_LAM { const int pb = sc->pathB[l]; bk(pb).len = bk(pb).len + dd; });
            wave_sync();
        }
        uValid = false;
    }
    /* -------------------------------------------------------- op apply -- */
    /* ---------------------------------------------------- snapshot load -- */
    // The header chunk (SnapshotLoader.loadHeader, MT/snapshotLoader.ts:126-160):
    // specToSegment per segment (:93-124) into rows 0..nh-1, reloadFromSegments
    // (mergeTree.ts:1185-1238: blocks of 7 children built level by level from
    // the leaves), then startCollaboration(minSeq, currentSeq) (:1243).  The
    // collab window gets every row with seq > minSeq or a removal.  Runs on a
    // freshly opened document.
    MT_HD void loadHeader(const MtLoad& Ld, uint32_t s0, int nh, int ms, int cs) {
        minSeq = ms; curSeq = cs;
        if (nh == 0) return;                                  // root stays open()'s empty block
        if (nh > (int)S.rowCap) { status |= MT_DS_OOM_ROWS; return; }
        const MtLoadSeg* G = Ld.segs + s0;
        const uint32_t pbase = uni(G[0].poff);
        int ttot = 0;
        for (int base = 0; base < nh; base += MT_WAVE) {
            const int m = (nh - base) < MT_WAVE ? (nh - base) : MT_WAVE;
            auto tl = wave_map(m, [&](int k) MT_LAM {
                const MtLoadSeg g = G[base + k];
                return (g.flags & MT_LS_MARKER) ? 0 : (int)g.plen;
            });
            ttot += wave_sum(tl);
        }
        if (ttot > (int)S.textCap) { status |= MT_DS_OOM_TEXT; return; }
        const int t0 = textTop;
        for (int base = 0; base < nh; base += MT_WAVE) {
            const int m = (nh - base) < MT_WAVE ? (nh - base) : MT_WAVE;
            wave_for(m, [&](int k) MT_LAM {
                const MtLoadSeg g = G[base + k];
                const int s = base + k;
                const bool mk = (g.flags & MT_LS_MARKER) != 0, rm = (g.flags & MT_LS_REMOVED) != 0;
                const int cl = (g.flags & MT_LS_CLIENT) ? (int)g.client : MT_NONCOLLAB;
                MtRow& w = row(s);
                w.len = mk ? 1 : (int)g.plen;
                w.seq = (g.flags & MT_LS_SEQ) ? g.seq : 0;
                w.rseq = rm ? g.rseq : MT_NOREM;
                w.meta = (uint32_t)cl | (rm ? MT_M_REMOVED : 0u) | (mk ? MT_M_MARKER : 0u);
                w.rcl = rm ? (uint32_t)g.rclient : 0u;
                w.ovl = 0ull; w.props = -1; w.parent = -1;
                w.mid = mk ? (int)g.mid : 0;
                // reloadFromSegments -> blockUpdate -> addNodeReferences maps the ids of
                // markers with localNetLength > 0 (MT/mergeTree.ts:286-297)
                if (mk && g.mid && !rm && (int)g.mid <= midCap) midt[g.mid - 1] = s;
                w.toff = mk ? (int)g.plen : t0 + (int)(g.poff - pbase);
                w.tcap = mk ? 0 : (int)g.plen;
            });
        }
        for (int base = 0; base < ttot; base += MT_WAVE) {
            const int m = (ttot - base) < MT_WAVE ? (ttot - base) : MT_WAVE;
            wave_for(m, [&](int k) MT_LAM { text[t0 + base + k] = Ld.payload[pbase + base + k]; });
        }
        textTop = t0 + ttot; rowTop = nh; c_ins += (uint64_t)ttot;
        wave_sync();
        for (int i = 0; i < nh; i++) {                        // TextSegment.make / Marker.make: addProperties(props)
            const int pid = uni((int)G[i].prop);
            if (pid >= 0) { const int ps = newPropMap(pid); row(i).props = ps; }
        }
        if (status) return;
        for (int base = 0; base < nh; base += MT_WAVE) {      // collab window
            const int m = (nh - base) < MT_WAVE ? (nh - base) : MT_WAVE;
            auto inw = wave_map(m, [&](int k) MT_LAM {
                const int s = base + k;
                return (bool)((row(s).seq > minSeq) | ((row(s).meta & MT_M_REMOVED) != 0));
            });
            const int cnt = wave_count(inw);
            if (winN + cnt > (int)S.winCap) { status |= MT_DS_OOM_WINDOW; return; }
            auto rk = wave_rank(inw);
            const int w0 = winN;
            wave_for(m, [&](int k) MT_LAM {
                if (own(inw, k)) { const int s = base + k; winSet(w0 + own(rk, k), s); row(s).meta = row(s).meta | MT_M_INWIN; }
            });
            winN += cnt;
        }
        if (winN > winHW) winHW = winN;
        // reloadFromSegments: level h groups the nodes of level h-1 seven at a time
        blkTop = 0; blkFree = -1; blkFreeN = 0;
        bpReset();                                  // nothing reads parents before the build ends
        int first = 0, count = nh, h = 0;
        for (;;) {
            const int nb = (count + MT_MAXN - 2) / (MT_MAXN - 1);
            if (blkTop + nb > (int)blkCap) { status |= MT_DS_OOM_BLOCKS; return; }
            const int b0 = blkTop; blkTop += nb;
            const int lvl = h, f0 = first, cnt = count;
            for (int base = 0; base < nb; base += MT_WAVE) {
                const int m = (nb - base) < MT_WAVE ? (nb - base) : MT_WAVE;
                wave_for(m, [&](int k) MT_LAM {
                    const int B = b0 + base + k, c0 = (base + k) * (MT_MAXN - 1);
                    const int n = (cnt - c0) < (MT_MAXN - 1) ? (cnt - c0) : (MT_MAXN - 1);
                    int len = 0;
                    for (int i = 0; i < MT_MAXN; i++) {
                        const int id = i < n ? f0 + c0 + i : -1;
                        if (id >= 0) {
                            if (lvl == 0) { row(id).parent = B; len += (row(id).meta & MT_M_REMOVED) ? 0 : row(id).len; }
                            else { bk(id).parent = B; len += bk(id).len; }
                        }
                        bk(B).c[i] = id;
                    }
                    bk(B).n = n; bk(B).len = len; bk(B).height = lvl; bk(B).parent = -1; bk(B).scour = -1;
                });
            }
            wave_sync();
            if (nb == 1) { root = b0; height = lvl; return; }
            first = b0; count = nb; h++;
        }
    }
    // One segment of a loadBody insertSegments call (mergeTree.ts:1974-2011,
    // blockInsert :2159-2242) at `pos` under perspective (UniversalSequenceNumber,
    // cli); `boundary`: first segment of the call (ensureIntervalBoundary first).
    // Returns the segment's cachedLength (0: skipped, as blockInsert skips it).
    MT_HD int loadInsert(const MtLoad& Ld, uint32_t gi, int pos, int cli, int sq, bool boundary) {
        if (boundary) { walk(MT_WALK_SPLIT, pos, 0, cli, -1, 0); if (status) return 0; }
        const MtLoadSeg* g = Ld.segs + gi;
        const uint32_t fl = uni((uint32_t)g->flags);
        const bool mk = (fl & MT_LS_MARKER) != 0, rm = (fl & MT_LS_REMOVED) != 0;
        const int plen = mk ? 0 : uni((int)g->plen);
        const int L = mk ? 1 : plen;
        if (L == 0) return 0;
        const int n = allocRow();
        if (n < 0) return 0;
        row(n).len = L; row(n).seq = sq; row(n).rseq = rm ? uni(g->rseq) : MT_NOREM;
        row(n).meta = (uint32_t)cli | (rm ? MT_M_REMOVED : 0u) | (mk ? MT_M_MARKER : 0u);
        row(n).rcl = rm ? (uint32_t)uni((int)g->rclient) : 0u;
        row(n).ovl = 0ull; row(n).parent = -1; row(n).props = -1;
        {   // insertSegments maps a marker's id before its walk (MT/mergeTree.ts:2218-2222)
            const int mi = mk ? uni((int)g->mid) : 0;
            row(n).mid = mi;
            if (mi) { if (mi > midCap) { status |= MT_DS_UNSUPPORTED; return 0; } midt[mi - 1] = n; }
        }
        row(n).tcap = plen;
        if (mk) row(n).toff = uni((int)g->plen);
        else {
            const int t0 = textAlloc(plen);
            if (t0 < 0) return 0;
            row(n).toff = t0;
            const uint16_t* src = Ld.payload + uni((int)g->poff);
            for (int base = 0; base < plen; base += MT_WAVE) {
                const int m = (plen - base) < MT_WAVE ? (plen - base) : MT_WAVE;
                wave_for(m, [&](int k) MT_LAM { text[t0 + base + k] = src[base + k]; });
            }
            c_ins += (uint64_t)plen;
        }
        const int pid = uni((int)g->prop);
        if (pid >= 0) { const int ps = newPropMap(pid); row(n).props = ps; }
        wave_sync();
        if (status) return 0;
        const int w = walk(MT_WALK_INSERT, pos, 0, cli, n, rm ? 0 : L);
        if (w != MT_W_OK || uni(row(n).parent) < 0) { status |= MT_DS_INSERT_FAILED; return 0; }
        c_rows += 2;
        if (sq > minSeq || rm) winAdd(n);
        if (sq > minSeq) addToLRUSet(n, sq);
        return L;
    }
    MT_HD void opInsert(int pos, int r, int c, int sq, const uint16_t* src, int plen, bool marker, int refType, int segProps,
                        int markerId, const LaneArr<int>& pay) {
        // MergeTree.insertSegments (MT/mergeTree.ts:1974-2011)
        MT_PB(t0);
        int w = walk(MT_WALK_SPLIT, pos, r, c, -1, 0);
        MT_PE(MT_PH_SPLIT, t0);
        if (w == MT_W_OK) c_rows += 2;
        if (status) return;
        const int L = marker ? 1 : plen;
        if (L > 0) {
            const int n = allocRow();
            if (n < 0) return;
            // payloads up to 64 units are already in lanes: flag text without a newline
            const bool nonl = MT_NONL && !marker && plen <= MT_WAVE &&
                              wave_count(wave_map(plen, [&](int k) MT_LAM { return own(pay, k) == (int)'\n'; })) == 0;
            const uint32_t m0 = (uint32_t)c | (marker ? MT_M_MARKER : 0u) | (nonl ? MT_M_NONL : 0u);
            row(n).len = L; row(n).seq = sq; row(n).rseq = MT_NOREM;
            row(n).meta = m0;
            row(n).ovl = 0ull; row(n).parent = -1; row(n).rcl = 0u;
            row(n).mid = markerId >= 0 ? markerId + 1 : 0;
            if (markerId >= 0) {                       // mapIdToSegment before the walk (MT/mergeTree.ts:2218-2222)
                if (markerId >= midCap) { status |= MT_DS_UNSUPPORTED; return; }
                midt[markerId] = n;
            }
            row(n).props = segProps >= 0 ? newPropMap(segProps) : -1;
            row(n).tcap = marker ? 0 : plen;
            if (marker) row(n).toff = refType;
            else {
                row(n).parent = -1;                                  // not yet linked: excluded from compaction
                const int t0 = textAlloc(plen);
                if (t0 < 0) return;
                row(n).toff = t0;
                if (plen <= MT_WAVE) wave_for(plen, [&](int k) MT_LAM { text[t0 + k] = (uint16_t)own(pay, k); });
                else {
                    for (int base = 0; base < plen; base += MT_WAVE) {
                        const int m = (plen - base) < MT_WAVE ? (plen - base) : MT_WAVE;
                        wave_for(m, [&](int k) MT_LAM { text[t0 + base + k] = src[base + k]; });
                    }
                }
                c_ins += (uint64_t)plen;
            }
            wave_sync();
            MT_PB(t1);
            landB = -1;
            if ((w == MT_W_OK || w == MT_W_NOCHANGE) && !lastSplit) {
                // The split walk (ensureIntervalBoundary) and the insert walk descend
                // by the same rule; with no block split in between the insert walk
                // would reach the same leaf slot: lastIdx (before the found row, at
                // the block end, or before the new right half of a split row).
                insertAtPath(lastL, lastIdx, n, L);
                uValid = false;
                w = MT_W_OK;
            } else {
                w = walk(MT_WALK_INSERT, pos, r, c, n, L);
            }
            MT_PE(MT_PH_INSERT, t1);
            if (w != MT_W_OK || landB < 0) { status |= MT_DS_INSERT_FAILED; return; }
            c_rows += 2;
            const uint32_t m1 = winAddKnown(n, m0);
            if (sq > minSeq) addToLRUSetKnown(n, sq, landB, m1);
            if (FULL && drec) emitDelta(MT_DK_INSERT, obsPosition(n), L, n, uni(row(n).props), -1, -1);   // insertSegments callback
        }
        zamboni();
    }
    /* ------------------------------------------------ register copy/paste -- */
    // The (client, name) entry of the RegisterCollection, or a free one when `alloc`;
    // -1 if absent (or the table is full).
    MT_HD int regFind(int c, int name, bool alloc) {
        auto cl = wave_map(MT_REG_CAP, [&](int i) MT_LAM { return regs[i].client; });
        auto nm = wave_map(MT_REG_CAP, [&](int i) MT_LAM { return regs[i].name; });
        const int hit = wave_first(wave_map(MT_REG_CAP, [&](int i) MT_LAM { return own(cl, i) == c && own(nm, i) == name; }));
        if (hit >= 0 || !alloc) return hit;
        return wave_first(wave_map(MT_REG_CAP, [&](int i) MT_LAM { return own(cl, i) < 0; }));
    }
    // Client.copy (MT/client.ts:600-608): cloneSegments(refSeq, client, start, end)
    // (MT/mergeTree.ts:1597-1614: every segment the range touches, whole, cloned with
    // clientId, seq, removedSeq, removedClientId and a copy of its properties,
    // MT/mergeTree.ts:476-483) replaces the register's contents.  Clones are unlinked rows
    // sharing the original's immutable text slice and property map.
    MT_HD void opCopy(int start, int end, int r, int c, int name) {
        const int e = regFind(c, name, true);
        if (e < 0) { status |= MT_DS_UNSUPPORTED; return; }          // MT_REG_CAP registers in use
        nCol = 0;
        const uint32_t cr0 = c_rows;
        rangeMap(MT_MAP_COLLECT, start, end, r, c, 0, -1, MT_PM_SET);   // sources into the arena's tail
        if (status) return;
        if (regTop + nCol > regCap) {                               // compact, then collect again
            regCompact();
            if (regTop + nCol > regCap) { status |= MT_DS_UNSUPPORTED; return; }
            nCol = 0; c_rows = cr0;                                 // (counted once)
            rangeMap(MT_MAP_COLLECT, start, end, r, c, 0, -1, MT_PM_SET);
            if (status) return;
        }
        const int n = nCol, base = regTop;
        // the clones' rows, all or none: recycled rows first (allocRow's order), then the pool top
        if (n > rfN + ((int)S.rowCap - rowTop)) { status |= MT_DS_OOM_ROWS; return; }
        const int f0 = rfN, t0 = rowTop;
        uint64_t rem = 0;
        for (int b0 = 0; b0 < n; b0 += MT_WAVE) {
            const int m = (n - b0) < MT_WAVE ? (n - b0) : MT_WAVE;
            const auto rm = wave_map(m, [&](int k) MT_LAM {
                const int i = b0 + k, s = regRow(base + i);
                const int d = i < f0 ? sc->rfree[f0 - 1 - i] : t0 + (i - f0);
                const uint32_t mt = row(s).meta;
                row(d).len = row(s).len; row(d).seq = row(s).seq; row(d).rseq = row(s).rseq;
                row(d).meta = (mt & (MT_M_CLIENT | MT_M_REMOVED | MT_M_MARKER | MT_M_NONL)) | MT_M_REG;
                row(d).rcl = row(s).rcl; row(d).props = row(s).props; row(d).mid = row(s).mid;
                row(d).toff = row(s).toff; row(d).tcap = (mt & MT_M_MARKER) ? 0 : row(s).len;
                row(d).ovl = 0ull; row(d).parent = -1;
                regRow(base + i) = d;
                return (mt & MT_M_REMOVED) != 0;
            });
            rem |= wave_ballot(rm);
        }
        rfN = n < f0 ? f0 - n : 0;
        rowTop = t0 + (n > f0 ? n - f0 : 0);
        wave_sync();
        // the entry's previous clones, unless pasted (then they are tree rows), are released
        MtReg& g = regs[e];
        const int on = uni(g.client) == c ? uni(g.n) : 0, of = uni(g.flags), oo = uni(g.off);
        if (on > 0 && !(of & 2)) {
            for (int i = 0; i < on; i++) {
                const int s = uni(regRow(oo + i));
                row(s).meta = uni(row(s).meta) & ~MT_M_REG;
                freeRow(s);
            }
        }
        const int fl = rem ? 1 : 0;
        wave_for(1, [&](int) MT_LAM { g.client = c; g.name = name; g.n = n; g.flags = fl; g.off = base; });
        regTop = base + n;
        wave_sync();
    }
    // Copying compaction of the register row arena: every entry's ids into the other half.
    MT_HD void regCompact() {
        const auto ns = wave_map(MT_REG_CAP, [&](int i) MT_LAM { return regs[i].client >= 0 ? regs[i].n : 0; });
        const auto os = wave_map(MT_REG_CAP, [&](int i) MT_LAM { return regs[i].off; });
        const int other = regHalf ^ 1;
        int* dst = regr + (size_t)other * regCap;
        int w = 0;
        for (int e = 0; e < MT_REG_CAP; e++) {
            const int n = wave_at(ns, e), o = wave_at(os, e);
            if (n <= 0) continue;
            for (int b0 = 0; b0 < n; b0 += MT_WAVE) {
                const int m = (n - b0) < MT_WAVE ? (n - b0) : MT_WAVE;
                wave_for(m, [&](int k) MT_LAM { dst[w + b0 + k] = regRow(o + b0 + k); });
            }
            const int w0 = w;
            wave_for(1, [&](int) MT_LAM { regs[e].off = w0; });
            w += n;
        }
        wave_sync();
        regHalf = other; regTop = w;
    }
    // Paste (applyInsertOp's register branch, MT/client.ts:436-444, then insertSegments
    // MT/mergeTree.ts:1974-2011 with blockInsert :2207-2241): every clone in order at
    // pos, pos + the earlier clones' cachedLength; seq and clientId become the op's.
    MT_HD void opPaste(int pos, int r, int c, int sq, int name) {
        const int e = regFind(c, name, false);
        if (e < 0) return;                                     // registerCollection.get: undefined
        MtReg& g = regs[e];
        const int n = uni(g.n), fl = uni(g.flags), o = uni(g.off);
        if (n == 0) return;                                    // no segments: the op does nothing
        if (fl & 3) { status |= MT_DS_UNSUPPORTED; return; }   // re-linked objects / removed clones
        if (walk(MT_WALK_SPLIT, pos, r, c, -1, 0) == MT_W_OK) c_rows += 2;   // ensureIntervalBoundary
        if (status) return;
        int ip = pos;
        for (int i = 0; i < n; i++) {
            const int k = uni(regRow(o + i));
            const uint32_t mt = (uni(row(k).meta) & ~(MT_M_REG | MT_M_CLIENT)) | (uint32_t)c;
            const int L = uni(row(k).len);
            row(k).meta = mt; row(k).seq = sq;
            const int mi = uni(row(k).mid);
            if ((mt & MT_M_MARKER) && mi > 0 && mi <= midCap) midt[mi - 1] = k;    // mapIdToSegment (:2218-2222)
            wave_sync();
            landB = -1;
            const int w = walk(MT_WALK_INSERT, ip, r, c, k, L);
            if (w != MT_W_OK || landB < 0) { status |= MT_DS_INSERT_FAILED; return; }
            c_rows += 2;
            const uint32_t m1 = winAddKnown(k, mt);
            if (sq > minSeq) addToLRUSetKnown(k, sq, landB, m1);
            if (FULL && drec) {   // the pasted clone's own content (createOpsFromDelta: r.segment.clone().toJSONObject())
                if (mt & MT_M_MARKER) emitDelta(MT_DK_INSERT, obsPosition(k), L, k, uni(row(k).props), 1, uni(row(k).toff));
                else {
                    const int to = dText(uni(row(k).toff), L);
                    emitDelta(MT_DK_INSERT, obsPosition(k), L, k, uni(row(k).props), 0, to);
                }
            }
            ip += L;
        }
        wave_for(1, [&](int) MT_LAM { g.flags = fl | 2; });
        wave_sync();
        zamboni();
    }
    MT_HD void opRange(int mode, int start, int end, int r, int c, int sq, int opset, int pm) {
        MT_PB(t0);
        int w = walk(MT_WALK_SPLIT, start, r, c, -1, 0);
        if (w == MT_W_OK) c_rows += 2;
        if (status) return;
        // The end boundary's walk resumes at the deepest block of the start walk's path whose
        // perspective range still holds end (tree and U unchanged unless a block split).
        // (A start past the perspective length fails at the root and leaves the path of an
        // earlier walk behind: then both walks start at the root.)
        int L0 = 0;
        if (MT_PATH_RESUME && w != MT_W_FAIL && !lastSplit && uValid && uRef == r && uCli == c) {
            for (int l = lastL; l > 0; l--) {
                if (end - uni(sc->pathOff[l]) <= uni(sc->pathLen[l])) { L0 = l; break; }
            }
        }
        w = walk(MT_WALK_SPLIT, end, r, c, -1, 0, L0);
        if (w == MT_W_OK) c_rows += 2;
        if (status) return;
        if (w == MT_W_FAIL || lastSplit || !uValid) L0 = 0;
        MT_PE(MT_PH_SPLIT, t0);
        MT_PB(t1);
        rangeMap(mode, start, end, r, c, sq, opset, pm, L0);
        MT_PE(MT_PH_RANGE, t1);
        if (status) return;
        zamboni();
    }
};
using MtEng = MtEngT<MT_RES_HBM>;
using MtEngFast = MtEngT<MT_RES_HBM, false>;

// SnapshotLoader for document i of a load batch (MT/snapshotLoader.ts:39-222) on
// a freshly opened engine document: header, collaboration start, body plan.
template <class Eng>
MT_HD void mt_load_doc(Eng& e, const MtLoad& Ld, uint32_t i) {
    const uint32_t s0 = Ld.seg_off[i], p0 = Ld.plan_off[i], p1 = Ld.plan_off[i + 1];
    if (p1 > p0 && uni(Ld.plan[p0].kind) == MT_LD_UNSUPPORTED) { e.status |= MT_DS_UNSUPPORTED; return; }
    e.loadHeader(Ld, s0, (int)Ld.nhdr[i], Ld.ms[i], Ld.cs[i]);
    int pos = 0, prevLen = 0;
    for (uint32_t k = p0; k < p1 && !e.status; k++) {
        const MtLoadStep st = Ld.plan[k];
        const int kind = uni(st.kind);
        if (kind == MT_LD_REFLUSH || kind == MT_LD_REFLUSH_NEW) {
            // The batch's first segment is already linked: the walk links it a
            // second time iff the observer length is within the NonCollab view.
            const int p = uni(e.bk(e.root).len);
            if (p <= e.perspectiveLength(0, MT_NONCOLLAB)) e.status |= MT_DS_UNSUPPORTED;
            else if (kind == MT_LD_REFLUSH_NEW) e.status |= MT_DS_INSERT_FAILED;   // a new segment falls off
            continue;
        }
        if (kind == MT_LD_UNSUPPORTED) { e.status |= MT_DS_UNSUPPORTED; break; }
        pos = kind == MT_LD_START ? uni(e.bk(e.root).len) : pos + prevLen;
        prevLen = e.loadInsert(Ld, s0 + (uint32_t)uni(st.seg), pos, uni(st.cli), uni(st.seq), kind == MT_LD_START);
        if (!e.status) e.zamboni();            // insertSegments ends with zamboniSegments (:2007-2010)
    }
}

