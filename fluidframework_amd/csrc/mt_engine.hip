// mt_engine.hip — MI355X (gfx950) backend of the batched merge-tree engine.
//
// One 64-lane wavefront (one workgroup) per document run: documents are
// independent, the ops inside a document are sequential.
// All per-document state lives in HBM pools (mt_core.h MtState); per-wave
// scratch (descent path, range-walk frames, scour hold list) lives in LDS.
// This is the product: there is no CPU path behind any of these entry points.
#include <hip/hip_runtime.h>
#include "mt_ctx.h"

// ------------------------------------------------------------- kernels ----
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
template <bool FULL>
__global__ __launch_bounds__(64, MT_LDS_WAVES_PER_SIMD) void mt_replay_lds_kernel(MtState S, MtOps ops, uint32_t* cursor, int lr, int lb, int lh) {
    __shared__ MtScratch sc;
    const uint32_t run = blockIdx.x;
    const uint32_t doc = ops.doc_ids[run];
    const uint32_t o0 = ops.op_off[run];
    MtEngT<MT_RES_LDS, FULL> e;
    e.bind(S, doc, &sc);
    uint32_t cur = o0;
    if (e.toLds(lr, lb, lh)) {
        cur = mt_replay_run(e, ops, run, doc, nullptr, nullptr, o0);
        e.fromLds();
    }
    cursor[run] = cur;
    e.store(doc);
}
// Blocks + heap in LDS (~9.5 KB per workgroup, 4 waves per SIMD), rows/window in HBM.
template <bool FULL>
__global__ __launch_bounds__(64, MT_WAVES_PER_SIMD) void mt_replay_blk_kernel(MtState S, MtOps ops, uint32_t* cursor, int lb, int lh) {
    __shared__ MtScratch sc;
    const uint32_t run = blockIdx.x;
    const uint32_t doc = ops.doc_ids[run];
    const uint32_t o0 = ops.op_off[run];
    MtEngT<MT_RES_BLK, FULL> e;
    e.bind(S, doc, &sc);
    uint32_t cur = o0;
    if (e.toLds(0, lb, lh)) {
        cur = mt_replay_run(e, ops, run, doc, nullptr, nullptr, o0);
        e.fromLds();
    }
    cursor[run] = cur;
    e.store(doc);
    // A document that outgrew LDS continues here with its pools in HBM (no
    // second launch: long documents, which outgrow it first, keep their head start).
    if (cur < ops.op_off[run + 1]) {
        MtEngT<MT_RES_HBM, FULL> h;
        h.bind(S, doc, &sc);
        mt_replay_run(h, ops, run, doc, nullptr, nullptr, cur);
        h.store(doc);
    }
}
// Long documents (MT_RES_BIG): heap, window and U set in LDS (~68 KB, two workgroups per
// CU), blocks and rows in HBM; one wave per SIMD at most, so the register budget is 256
// VGPRs and nothing spills.  A document whose heap or height outgrows LDS continues in HBM.
template <bool FULL>
__global__ __launch_bounds__(64, 1) void mt_replay_big_kernel(MtState S, MtOps ops, uint32_t* cursor, int lw, int lh) {
    __shared__ MtScratch sc;
    const uint32_t run = blockIdx.x;
    const uint32_t doc = ops.doc_ids[run];
    const uint32_t o0 = ops.op_off[run];
    MtEngT<MT_RES_BIG, FULL> e;
    e.bind(S, doc, &sc);
    uint32_t cur = o0;
    if (e.toLds(lw, 0, lh)) {
        cur = mt_replay_run(e, ops, run, doc, nullptr, nullptr, o0);
        e.fromLds();
    }
    cursor[run] = cur;
    e.store(doc);
    if (cur < ops.op_off[run + 1]) {
        MtEngT<MT_RES_HBM, FULL> h;
        h.bind(S, doc, &sc);
        mt_replay_run(h, ops, run, doc, nullptr, nullptr, cur);
        h.store(doc);
    }
}
template <bool FULL>
__global__ __launch_bounds__(64, MT_WAVES_PER_SIMD) void mt_replay_kernel(MtState S, MtOps ops, const uint32_t* cursor) {
    __shared__ MtScratch sc;
    const uint32_t run = blockIdx.x;
    const uint32_t o0 = cursor ? cursor[run] : ops.op_off[run];
    if (o0 >= ops.op_off[run + 1]) return;
    const uint32_t doc = ops.doc_ids[run];
    MtEngT<MT_RES_HBM, FULL> e;
    e.bind(S, doc, &sc);
    mt_replay_run(e, ops, run, doc, nullptr, nullptr, o0);
    e.store(doc);
}
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
__global__ __launch_bounds__(64) void mt_open_kernel(MtState S, uint32_t first) {
    __shared__ MtScratch sc;
    const uint32_t doc = first + blockIdx.x;
    MtEng e;
    e.bind(S, doc, &sc);
    e.open();
    e.store(doc);
}
// Snapshot load (mt_load_snapshot): one wave per document, pools in HBM.
__global__ __launch_bounds__(64) void mt_load_kernel(MtState S, MtLoad Ld) {
    __shared__ MtScratch sc;
    const uint32_t doc = Ld.docs[blockIdx.x];
    MtEng e;
    e.bind(S, doc, &sc);
    e.open();
    mt_load_doc(e, Ld, blockIdx.x);
    e.store(doc);
}
__global__ __launch_bounds__(64) void mt_update_seq_kernel(MtState S, const uint32_t* docs, const int32_t* msn, const int32_t* seq) {
    __shared__ MtScratch sc;
    const uint32_t doc = docs[blockIdx.x];
    MtEng e;
    e.bind(S, doc, &sc);
    mt_update_seq_doc(e, msn[blockIdx.x], seq[blockIdx.x]);
    e.store(doc);
}
__global__ __launch_bounds__(64) void mt_get_length_kernel(MtState S, const uint32_t* docs, const int32_t* ref, const int32_t* cli, int32_t* out) {
    __shared__ MtScratch sc;
    const uint32_t doc = docs[blockIdx.x];
    MtEng e;
    e.bind(S, doc, &sc);
    // read-only: queries of one document run in parallel workgroups
    const int l = e.perspectiveLengthRO(ref[blockIdx.x], cli[blockIdx.x] < 0 ? MT_NOBODY : cli[blockIdx.x]);
    if (__lane_id() == 0) out[blockIdx.x] = l;
}

// Staging for host-side serialization (mt_pack.h): sizes, then the packed copy.
__global__ __launch_bounds__(64) void mt_pack_size_kernel(MtState S, const uint32_t* docs, MtPackSize* out) {
    __shared__ MtScratch sc;
    MtEng e;
    e.bind(S, docs[blockIdx.x], &sc);
    const MtPackSize z = mt_pack_size(e);
    if (__lane_id() == 0) out[blockIdx.x] = z;
}
__global__ __launch_bounds__(64) void mt_pack_kernel(MtState S, const uint32_t* docs, const uint64_t* off, uint8_t* stage) {
    __shared__ MtScratch sc;
    MtEng e;
    e.bind(S, docs[blockIdx.x], &sc);
    mt_pack_doc(e, stage + off[blockIdx.x]);
}

// ----------------------------------------------------- backend plumbing ----
static int mtb_init(mt_ctx* c) {
    if (hipSetDevice(c->device) != hipSuccess) { c->err = "hipSetDevice failed"; return 1; }
    hipStream_t s; hipEvent_t a, b;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) { c->err = "hipStreamCreate failed"; return 1; }
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    c->stream = s; c->ev0 = a; c->ev1 = b;
    return 0;
}
static void mtb_fini(mt_ctx* c) {
    if (c->stream) { (void)hipStreamSynchronize((hipStream_t)c->stream); (void)hipStreamDestroy((hipStream_t)c->stream); }
    if (c->ev0) (void)hipEventDestroy((hipEvent_t)c->ev0);
    if (c->ev1) (void)hipEventDestroy((hipEvent_t)c->ev1);
}
static int mtb_malloc(void** p, size_t n) { return hipMalloc(p, n) == hipSuccess ? 0 : 1; }
static void mtb_free(void* p) { (void)hipFree(p); }
static void mtb_memset(void* p, int v, size_t n) { (void)hipMemset(p, v, n); }
static void mtb_h2d(mt_ctx* c, void* d, const void* s, size_t n) { (void)hipMemcpyAsync(d, s, n, hipMemcpyHostToDevice, (hipStream_t)c->stream); (void)hipStreamSynchronize((hipStream_t)c->stream); }
static void mtb_d2d(mt_ctx* c, void* d, const void* s, size_t n) { (void)hipMemcpyAsync(d, s, n, hipMemcpyDeviceToDevice, (hipStream_t)c->stream); (void)hipStreamSynchronize((hipStream_t)c->stream); }
static void mtb_d2h(mt_ctx* c, void* d, const void* s, size_t n) { (void)hipMemcpyAsync(d, s, n, hipMemcpyDeviceToHost, (hipStream_t)c->stream); (void)hipStreamSynchronize((hipStream_t)c->stream); }
static int mtb_sync(mt_ctx* c) {
    hipError_t e = hipStreamSynchronize((hipStream_t)c->stream);
    if (e != hipSuccess) { c->err = hipGetErrorString(e); return MT_E_HIP; }
    if (c->ev_pending) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, (hipEvent_t)c->ev0, (hipEvent_t)c->ev1) == hipSuccess) c->last_ms = ms;
        c->ev_pending = false;
    }
    (void)hipGetLastError();
    return MT_OK;
}
static int mtb_check(mt_ctx* c) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) { c->err = hipGetErrorString(e); return MT_E_HIP; }
    return MT_OK;
}
template <bool FULL>
static void launch_replay(mt_ctx* c, hipStream_t s, uint32_t n_runs) {
    if (c->use_lds == 3) {
        hipLaunchKernelGGL(mt_replay_big_kernel<FULL>, dim3(n_runs), dim3(64), 0, s, c->S, c->ops, (uint32_t*)c->b_cursor.p,
                           c->lds_rows, c->lds_heap);
    } else if (c->use_lds == 2) {
        hipLaunchKernelGGL(mt_replay_blk_kernel<FULL>, dim3(n_runs), dim3(64), 0, s, c->S, c->ops, (uint32_t*)c->b_cursor.p,
                           c->lds_blks, c->lds_heap);
    } else if (c->use_lds) {
        hipLaunchKernelGGL(mt_replay_lds_kernel<FULL>, dim3(n_runs), dim3(64), 0, s, c->S, c->ops, (uint32_t*)c->b_cursor.p,
                           c->lds_rows, c->lds_blks, c->lds_heap);
        hipLaunchKernelGGL(mt_replay_kernel<FULL>, dim3(n_runs), dim3(64), 0, s, c->S, c->ops, (const uint32_t*)c->b_cursor.p);
    } else hipLaunchKernelGGL(mt_replay_kernel<FULL>, dim3(n_runs), dim3(64), 0, s, c->S, c->ops, (const uint32_t*)nullptr);
}
static int mtb_launch_replay(mt_ctx* c, const MtGen& g, uint32_t n_runs) {
    if (n_runs == 0) return MT_OK;
    hipStream_t s = (hipStream_t)c->stream;
    (void)hipGetLastError();
    (void)hipEventRecord((hipEvent_t)c->ev0, s);
    if (g.enabled) hipLaunchKernelGGL(mt_generate_kernel, dim3(n_runs), dim3(64), 0, s, c->S, c->ops, g);
    else if (c->ops.drec || c->batch_reg) launch_replay<true>(c, s, n_runs);
    else launch_replay<false>(c, s, n_runs);
    (void)hipEventRecord((hipEvent_t)c->ev1, s);
    c->ev_pending = true;
    return mtb_check(c);
}
static int mtb_launch_open(mt_ctx* c, uint32_t first, uint32_t n) {
    (void)hipGetLastError();
    hipLaunchKernelGGL(mt_open_kernel, dim3(n), dim3(64), 0, (hipStream_t)c->stream, c->S, first);
    return mtb_check(c);
}
static int mtb_launch_load(mt_ctx* c, const MtLoad& L, uint32_t n) {
    if (!n) return MT_OK;
    (void)hipGetLastError();
    hipLaunchKernelGGL(mt_load_kernel, dim3(n), dim3(64), 0, (hipStream_t)c->stream, c->S, L);
    return mtb_check(c);
}
static int mtb_launch_update_seq(mt_ctx* c, const uint32_t* docs, const int32_t* msn, const int32_t* seq, uint32_t n) {
    if (!n) return MT_OK;
    (void)hipGetLastError();
    hipLaunchKernelGGL(mt_update_seq_kernel, dim3(n), dim3(64), 0, (hipStream_t)c->stream, c->S, docs, msn, seq);
    return mtb_check(c);
}
static int mtb_launch_get_length(mt_ctx* c, const uint32_t* docs, const int32_t* ref, const int32_t* cli, int32_t* out, uint32_t n) {
    if (!n) return MT_OK;
    (void)hipGetLastError();
    hipLaunchKernelGGL(mt_get_length_kernel, dim3(n), dim3(64), 0, (hipStream_t)c->stream, c->S, docs, ref, cli, out);
    return mtb_check(c);
}

static int mtb_launch_pack_size(mt_ctx* c, const uint32_t* docs, MtPackSize* out, uint32_t n) {
    if (!n) return MT_OK;
    (void)hipGetLastError();
    hipLaunchKernelGGL(mt_pack_size_kernel, dim3(n), dim3(64), 0, (hipStream_t)c->stream, c->S, docs, out);
    return mtb_check(c);
}
static int mtb_launch_pack(mt_ctx* c, const uint32_t* docs, const uint64_t* off, uint8_t* stage, uint32_t n) {
    if (!n) return MT_OK;
    (void)hipGetLastError();
    hipLaunchKernelGGL(mt_pack_kernel, dim3(n), dim3(64), 0, (hipStream_t)c->stream, c->S, docs, off, stage);
    return mtb_check(c);
}

#define MT_FN(name) mt_##name
#include "mt_api_impl.h"
