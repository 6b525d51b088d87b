// mt_k_replay.hip — the replay kernels of the MI355X engine, one kernel set per object.
//
// Built several times with -DMT_KSET=<n> (see __graft_entry__.build_engine): each object
// holds one group of template instantiations, so the groups compile in parallel, and
// mt_engine.hip launches them through the mtk_* functions declared in mt_kernels.h.
//   MT_KSET 0: mt_replay_blk_kernel<false, false> (the hot path: no in-wave continuation)
//   MT_KSET 1: mt_replay_blk_kernel<true, true>   5: mt_replay_blk_kernel<false, true> (long runs)
//   MT_KSET 2: mt_replay_big_kernel<false / true>  3: mt_replay_lds_kernel<false / true>
//   MT_KSET 4: the all-HBM kernels and the generator
//   MT_KSET 6: mt_replay_blkw_kernel<false, true> (the size class of long runs)
#include <hip/hip_runtime.h>
#include "mt_ctx.h"
#include "mt_kernels.h"

#ifndef MT_WAVES_PER_SIMD
#define MT_WAVES_PER_SIMD 4
#endif
// Replay: Client.applyMsg over each document's resident op run (the timed hot
// path), in two launches.  mt_replay_lds_kernel moves the document's rows,
// blocks, heap and window into LDS and runs as far as they fit (cursor[run] =
// the first op not applied); mt_replay_kernel finishes any remainder with the
// pools in HBM.
#ifndef MT_LDS_WAVES_PER_SIMD
#define MT_LDS_WAVES_PER_SIMD 1
#endif
// FULL (every replay kernel): true only while a delta-capture buffer is armed or the
// resident batch holds register ops (mt_upload_batch found MT_OP_CUT / COPY / PASTE).
// Each kernel runs one document run per one-wave workgroup (mt_replay_doc, mt_replay.h).
template <bool FULL>
__global__ __launch_bounds__(64, MT_LDS_WAVES_PER_SIMD) void mt_replay_lds_kernel(MtState S, MtOps ops, uint32_t* cursor, int lr, int lb, int lh) {
    __shared__ MtScratch sc;
    const uint32_t cur = mt_replay_doc<MT_RES_LDS, FULL>(S, ops, blockIdx.x, &sc, lr, lb, lh);
    if (__lane_id() == 0) cursor[blockIdx.x] = cur;
}
// Blocks + heap in LDS (~9.5 KB per workgroup, 4 waves per SIMD), rows/window in HBM; a
// document that outgrows LDS continues in HBM in the same wave (CONT) or stops for the
// all-HBM launch that follows.
template <bool FULL, bool CONT>
__global__ __launch_bounds__(64, MT_WAVES_PER_SIMD) void mt_replay_blk_kernel(MtState S, MtOps ops, const uint32_t* runs,
                                                                               uint32_t* cursor, int lb, int lh) {
    __shared__ MtScratch sc;
    const uint32_t run = runs ? runs[blockIdx.x] : blockIdx.x;          // size classes: a run list
    const uint32_t cur = mt_replay_doc<MT_RES_BLK, FULL, CONT>(S, ops, run, &sc, 0, lb, lh);
    if (__lane_id() == 0) cursor[run] = cur;
}
// Wide block residency (MT_RES_BLKW): the block-residency engine with room for long documents'
// trees and heaps (MT_BW_BLKS blocks, ~21 KB per workgroup), for the size class of long runs;
// continues in HBM in-wave if even that is outgrown.
template <bool FULL, bool CONT>
__global__ __launch_bounds__(64, 2) void mt_replay_blkw_kernel(MtState S, MtOps ops, const uint32_t* runs,
                                                               uint32_t* cursor) {
    __shared__ MtScratch sc;
    const uint32_t run = runs ? runs[blockIdx.x] : blockIdx.x;
    const uint32_t cur = mt_replay_doc<MT_RES_BLKW, FULL, CONT>(S, ops, run, &sc, 0, MT_BW_BLKS, MT_BW_HEAP);
    if (__lane_id() == 0) cursor[run] = cur;
}
// Long documents (MT_RES_BIG): heap, window, U set and a block cache of the tree's upper
// levels in LDS (~137 KB, one workgroup per CU), rows and the other blocks in HBM; one wave
// per SIMD at most, so the register budget is 256 VGPRs.  A document whose heap or height
// outgrows LDS continues in HBM.  lb < 0: block cache off.
// A workgroup of MT_G_NW waves per document: wave 0 replays, the others serve its posted
// computeU shares (MtEngT::mwRun / mwShare) until it posts MT_MW_EXIT; every wave reaches
// the same barriers, and wave 0 posts the exit on every path.
template <bool FULL>
__global__ __launch_bounds__(64 * MT_G_NW, 1) void mt_replay_big_kernel(MtState S, MtOps ops, const uint32_t* runs,
                                                                         uint32_t* cursor, int lw, int lb, int lh) {
    __shared__ MtScratch sc;
    const int wv = (int)(threadIdx.x >> 6);
    if (wv == 0) {
        if (__lane_id() == 0) mt_ldsg().posted = 0;
        const uint32_t run = runs ? runs[blockIdx.x] : blockIdx.x;
        const uint32_t cur = mt_replay_doc<MT_RES_BIG, FULL>(S, ops, run, &sc, lw, lb, lh);
        if (__lane_id() == 0) cursor[run] = cur;
        // the exit job goes to the slot after the last one posted
        if (__lane_id() == 0) mt_ldsg().mw[mt_ldsg().posted & 1].op = MT_MW_EXIT;
        __syncthreads();
    } else {
        MtEngT<MT_RES_BIG, FULL> h;
        for (int k = 0;; k++) {
            __syncthreads();
            const int op = __builtin_amdgcn_readfirstlane(mt_ldsg().mw[k & 1].op);
            if (op == MT_MW_EXIT) break;
            h.mwShare(wv, k);
            if (MtEngT<MT_RES_BIG, FULL>::mwSync(op)) __syncthreads();
        }
    }
}
// Every pool in HBM: whole runs, or the rest of each run after mt_replay_lds_kernel.
template <bool FULL>
__global__ __launch_bounds__(64, MT_WAVES_PER_SIMD) void mt_replay_kernel(MtState S, MtOps ops) {
    __shared__ MtScratch sc;
    (void)mt_replay_doc<MT_RES_HBM, FULL>(S, ops, blockIdx.x, &sc, 0, 0, 0);
}
// The rest of runs that outgrew LDS: usually none or a few documents, so two waves per SIMD
// (a 256-VGPR budget: no spills, no scratch) rather than the hot kernels' four.
#ifndef MT_REST_WAVES_PER_SIMD
#define MT_REST_WAVES_PER_SIMD 2
#endif
template <bool FULL>
__global__ __launch_bounds__(64, MT_REST_WAVES_PER_SIMD) void mt_replay_rest_kernel(MtState S, MtOps ops, const uint32_t* cursor) {
    __shared__ MtScratch sc;
    mt_replay_doc_rest<FULL>(S, ops, blockIdx.x, &sc, cursor[blockIdx.x]);
}
#if MT_KSET == 4
// Generation: the same engine acting as sequencer + observer, writing the op
// records it applies (a separate symbol so profiles never mix it with replay).
__global__ __launch_bounds__(64, MT_WAVES_PER_SIMD) void mt_generate_kernel(MtState S, MtOps ops, MtGen gen) {
    __shared__ MtScratch sc;
    __shared__ int lastRef[64];
    const uint32_t run = blockIdx.x;
    const uint32_t doc = ops.doc_ids[run];
    MtEng e;
    e.bind(S, doc, &sc);
    mt_replay_run(e, ops, run, doc, &gen, lastRef, ops.op_off[run]);
    e.store(doc);
}
#endif

// ------------------------------------------------------------- launchers ----
#if MT_KSET == 0
void mtk_blk_fast(hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const uint32_t* runs, uint32_t* cur, int lb,
                  int lh, uint32_t pad) {
    hipLaunchKernelGGL((mt_replay_blk_kernel<false, false>), dim3(n), dim3(64), pad, s, S, o, runs, cur, lb, lh);
}
#elif MT_KSET == 5
void mtk_blk_fast_cont(hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const uint32_t* runs, uint32_t* cur,
                       int lb, int lh, uint32_t pad) {
    hipLaunchKernelGGL((mt_replay_blk_kernel<false, true>), dim3(n), dim3(64), pad, s, S, o, runs, cur, lb, lh);
}
#elif MT_KSET == 6
#ifndef MT_BLKW_PAD_BYTES
#define MT_BLKW_PAD_BYTES 0           // diagnostic builds only: dynamic LDS per workgroup (fewer per CU)
#endif
void mtk_blkw(hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const uint32_t* runs, uint32_t* cur) {
    hipLaunchKernelGGL((mt_replay_blkw_kernel<false, true>), dim3(n), dim3(64), MT_BLKW_PAD_BYTES, s, S, o, runs, cur);
}
#elif MT_KSET == 1
void mtk_blk_full(hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const uint32_t* runs, uint32_t* cur, int lb,
                  int lh, uint32_t pad) {
    hipLaunchKernelGGL((mt_replay_blk_kernel<true, true>), dim3(n), dim3(64), pad, s, S, o, runs, cur, lb, lh);
}
#elif MT_KSET == 2
void mtk_big(bool full, hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const uint32_t* runs, uint32_t* cur,
             int lw, int lb, int lh) {
    if (full) hipLaunchKernelGGL(mt_replay_big_kernel<true>, dim3(n), dim3(64 * MT_G_NW), 0, s, S, o, runs, cur, lw, lb, lh);
    else hipLaunchKernelGGL(mt_replay_big_kernel<false>, dim3(n), dim3(64 * MT_G_NW), 0, s, S, o, runs, cur, lw, lb, lh);
}
#elif MT_KSET == 3
void mtk_lds(bool full, hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, uint32_t* cur, int lr, int lb, int lh) {
    if (full) hipLaunchKernelGGL(mt_replay_lds_kernel<true>, dim3(n), dim3(64), 0, s, S, o, cur, lr, lb, lh);
    else hipLaunchKernelGGL(mt_replay_lds_kernel<false>, dim3(n), dim3(64), 0, s, S, o, cur, lr, lb, lh);
}
#else
void mtk_hbm(bool full, hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const uint32_t* cur) {
    if (cur) {
        if (full) hipLaunchKernelGGL(mt_replay_rest_kernel<true>, dim3(n), dim3(64), 0, s, S, o, cur);
        else hipLaunchKernelGGL(mt_replay_rest_kernel<false>, dim3(n), dim3(64), 0, s, S, o, cur);
    } else if (full) hipLaunchKernelGGL(mt_replay_kernel<true>, dim3(n), dim3(64), 0, s, S, o);
    else hipLaunchKernelGGL(mt_replay_kernel<false>, dim3(n), dim3(64), 0, s, S, o);
}
void mtk_generate(hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const MtGen& g) {
    hipLaunchKernelGGL(mt_generate_kernel, dim3(n), dim3(64), 0, s, S, o, g);
}
#endif
