// mt_kernels.h — launchers of the replay kernels (mt_k_replay.hip, one object per kernel set).
#pragma once
#include <hip/hip_runtime.h>
#include "mt_core.h"

// runs: the run each workgroup replays (size classes), or null for run = blockIdx.x;
// pad: dynamic LDS bytes added to each workgroup (fewer workgroups per CU; unused by the kernel)
void mtk_blk_fast(hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const uint32_t* runs, uint32_t* cur, int lb,
                  int lh, uint32_t pad = 0);
void mtk_blk_full(hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const uint32_t* runs, uint32_t* cur, int lb,
                  int lh, uint32_t pad = 0);
// the block-residency kernel with the in-wave HBM continuation (long runs)
void mtk_blk_fast_cont(hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const uint32_t* runs, uint32_t* cur,
                       int lb, int lh, uint32_t pad = 0);
// wide block residency (MT_BW_BLKS blocks in LDS) with the in-wave continuation: long runs
void mtk_blkw(hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const uint32_t* runs, uint32_t* cur);
void mtk_big(bool full, hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const uint32_t* runs, uint32_t* cur,
             int lw, int lb, int lh);
void mtk_lds(bool full, hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, uint32_t* cur, int lr, int lb, int lh);
void mtk_hbm(bool full, hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const uint32_t* cur);
void mtk_generate(hipStream_t s, uint32_t n, const MtState& S, const MtOps& o, const MtGen& g);
