// mt_engine.hip — MI355X (gfx950) backend of the batched merge-tree engine.
//
// One 64-lane wavefront (one workgroup) per document run: documents are
// independent, the ops inside a document are sequential.
// All per-document state lives in HBM pools (mt_core.h MtState); per-wave
// scratch (descent path, range-walk frames, scour hold list) lives in LDS.
// This is the product: there is no CPU path behind any of these entry points.
#include <hip/hip_runtime.h>
#include "mt_ctx.h"
#include "mt_kernels.h"
#include "mt_shard.h"

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

// Position queries (mt_query.h): one wave per document group of the sorted queries.
__global__ __launch_bounds__(64) void mt_query_kernel(MtState S, const MtQuery* q, const uint32_t* grp, MtQueryOut* out) {
    __shared__ MtScratch sc;
    const uint32_t q0 = grp[blockIdx.x], q1 = grp[blockIdx.x + 1];
    MtEngFast e;
    e.bind(S, q[q0].doc, &sc);
    mt_query_run(e, S, q, q0, q1, out);
}
// Text of found segments into one arena: workgroup i copies len[i] units from text[at[i]].
__global__ __launch_bounds__(256) void mt_gather_text_kernel(const uint16_t* text, const unsigned long long* at,
                                                             const uint32_t* len, const unsigned long long* off,
                                                             uint16_t* dst) {
    const uint32_t i = blockIdx.x, n = len[i];
    const unsigned long long a = at[i], o = off[i];
    for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) dst[o + k] = text[a + k];
}

// Staging for host-side serialization (mt_pack.h): sizes, then the packed copy.
__global__ __launch_bounds__(64) void mt_pack_size_kernel(MtState S, const uint32_t* docs, MtPackSize* out, uint32_t epoch) {
    __shared__ MtScratch sc;
    MtEng e;
    e.bind(S, docs[blockIdx.x], &sc);
    const MtPackSize z = mt_pack_size(e, epoch);
    if (__lane_id() == 0) out[blockIdx.x] = z;
}
__global__ __launch_bounds__(64) void mt_pack_kernel(MtState S, const uint32_t* docs, const uint64_t* off, uint8_t* stage,
                                                     uint32_t epoch) {
    __shared__ MtScratch sc;
    MtEng e;
    e.bind(S, docs[blockIdx.x], &sc);
    mt_pack_doc(e, stage + off[blockIdx.x], epoch);
}

// Document exchange rows (mt_shard.h): one wave per document run.
__global__ __launch_bounds__(64) void mt_rows_kernel(MtOps ops, int pack, uint32_t first, uint32_t L, const uint64_t* dst,
                                                     unsigned long long* rows, uint64_t* cs) {
    const uint32_t i = blockIdx.x;
    const unsigned long long h = pack ? mt_pack_rows_doc(ops, first + i, L, dst[i], rows) : mt_unpack_rows_doc(ops, i, L, rows);
    if (__lane_id() == 0) cs[i] = h;
}

// ----------------------------------------------------- backend plumbing ----
static int mtb_init(mt_ctx* c) {
    if (hipSetDevice(c->device) != hipSuccess) { c->err = "hipSetDevice failed"; return 1; }
    hipStream_t s; hipEvent_t a, b;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) { c->err = "hipStreamCreate failed"; return 1; }
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    c->stream = s; c->ev0 = a; c->ev1 = b;
    hipStream_t s2; hipEvent_t f, j;
    if (hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) != hipSuccess) { c->err = "hipStreamCreate failed"; return 1; }
    (void)hipEventCreateWithFlags(&f, hipEventDisableTiming); (void)hipEventCreateWithFlags(&j, hipEventDisableTiming);
    c->stream2 = s2; c->ev_fork = f; c->ev_join = j;
    return 0;
}
static void mtb_fini(mt_ctx* c) {
    if (c->stream) { (void)hipStreamSynchronize((hipStream_t)c->stream); (void)hipStreamDestroy((hipStream_t)c->stream); }
    for (auto& st : c->stage) {
        if (st.ev) (void)hipEventDestroy((hipEvent_t)st.ev);
        if (st.p) (void)hipHostFree(st.p);
    }
    for (int b = 0; b < 2; b++) if (c->dl_host[b]) (void)hipHostFree(c->dl_host[b]);
    if (c->ev0) (void)hipEventDestroy((hipEvent_t)c->ev0);
    if (c->ev1) (void)hipEventDestroy((hipEvent_t)c->ev1);
    if (c->stream2) { (void)hipStreamSynchronize((hipStream_t)c->stream2); (void)hipStreamDestroy((hipStream_t)c->stream2); }
    if (c->streamA) { (void)hipStreamSynchronize((hipStream_t)c->streamA); (void)hipStreamDestroy((hipStream_t)c->streamA); }
    if (c->streamB) { (void)hipStreamSynchronize((hipStream_t)c->streamB); (void)hipStreamDestroy((hipStream_t)c->streamB); }
    if (c->ev_joinB) (void)hipEventDestroy((hipEvent_t)c->ev_joinB);
    if (c->ev_fork) (void)hipEventDestroy((hipEvent_t)c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy((hipEvent_t)c->ev_join);
}
static int mtb_malloc(void** p, size_t n) { return hipMalloc(p, n) == hipSuccess ? 0 : 1; }
static void mtb_free(void* p) { (void)hipFree(p); }
static void mtb_memset(void* p, int v, size_t n) { (void)hipMemset(p, v, n); }
static void mtb_h2d(mt_ctx* c, void* d, const void* s, size_t n) { (void)hipMemcpyAsync(d, s, n, hipMemcpyHostToDevice, (hipStream_t)c->stream); (void)hipStreamSynchronize((hipStream_t)c->stream); }
static void mtb_d2d(mt_ctx* c, void* d, const void* s, size_t n) { (void)hipMemcpyAsync(d, s, n, hipMemcpyDeviceToDevice, (hipStream_t)c->stream); (void)hipStreamSynchronize((hipStream_t)c->stream); }
static void mtb_d2h(mt_ctx* c, void* d, const void* s, size_t n) { (void)hipMemcpyAsync(d, s, n, hipMemcpyDeviceToHost, (hipStream_t)c->stream); (void)hipStreamSynchronize((hipStream_t)c->stream); }
// Pinned staging for batch uploads: the next slot, grown if needed, once its previous H2D
// is done (the slot's event); mtb_stage_send then copies it to the device asynchronously.
static void* mtb_stage_get(mt_ctx* c, size_t n) {
    mt_ctx::Stage& st = c->stage[c->stage_k];
    if (st.ev) (void)hipEventSynchronize((hipEvent_t)st.ev);
    else { hipEvent_t e; (void)hipEventCreateWithFlags(&e, hipEventDisableTiming); st.ev = e; }
    if (st.cap < n) {
        if (st.p) (void)hipHostFree(st.p);
        st.p = nullptr; st.cap = 0;
        const size_t cap = n + n / 4 + 4096;
        if (hipHostMalloc(&st.p, cap, hipHostMallocDefault) != hipSuccess) { st.p = nullptr; return nullptr; }
        st.cap = cap;
    }
    return st.p;
}
static void mtb_stage_send(mt_ctx* c, void* dev, size_t n) {
    mt_ctx::Stage& st = c->stage[c->stage_k];
    (void)hipMemcpyAsync(dev, st.p, n, hipMemcpyHostToDevice, (hipStream_t)c->stream);
    (void)hipEventRecord((hipEvent_t)st.ev, (hipStream_t)c->stream);
    c->stage_k ^= 1;
}
// Pinned host buffer the document staging downloads into (reused, grown on demand).
static uint8_t* mtb_host_stage(mt_ctx* c, size_t n, int buf) {
    if (c->dl_cap[buf] < n) {
        if (c->dl_host[buf]) (void)hipHostFree(c->dl_host[buf]);
        c->dl_host[buf] = nullptr; c->dl_cap[buf] = 0;
        const size_t cap = n + n / 4 + 4096;
        if (hipHostMalloc(&c->dl_host[buf], cap, hipHostMallocDefault) != hipSuccess) { c->dl_host[buf] = nullptr; return nullptr; }
        c->dl_cap[buf] = cap;
    }
    return (uint8_t*)c->dl_host[buf];
}
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
// The two CU-masked streams of partitioned size classes: A holds part_cus CUs spread evenly
// over the device (every k-th CU, so every XCD gives its share), B the rest.
static int mtb_partition_streams(mt_ctx* c) {
    if (c->part_made == c->part_cus && c->streamA) return 0;
    if (c->streamA) { (void)hipStreamSynchronize((hipStream_t)c->streamA); (void)hipStreamDestroy((hipStream_t)c->streamA); c->streamA = nullptr; }
    if (c->streamB) { (void)hipStreamSynchronize((hipStream_t)c->streamB); (void)hipStreamDestroy((hipStream_t)c->streamB); c->streamB = nullptr; }
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || ncu <= 0) return 1;
    const uint32_t want = c->part_cus < (uint32_t)ncu ? c->part_cus : (uint32_t)ncu - 1;
    std::vector<uint32_t> ma((ncu + 31) / 32, 0u), mb((ncu + 31) / 32, 0u);
    uint32_t got = 0;
    for (int i = 0; i < ncu; i++) {
        const bool inA = got < want && (uint64_t)i * want / (uint64_t)ncu != (uint64_t)(i + 1) * want / (uint64_t)ncu;
        if (inA) { ma[i / 32] |= 1u << (i % 32); got++; } else mb[i / 32] |= 1u << (i % 32);
    }
    hipStream_t a, b;
    if (hipExtStreamCreateWithCUMask(&a, (uint32_t)ma.size(), ma.data()) != hipSuccess) return 1;
    if (hipExtStreamCreateWithCUMask(&b, (uint32_t)mb.size(), mb.data()) != hipSuccess) { (void)hipStreamDestroy(a); return 1; }
    c->streamA = a; c->streamB = b;
    if (!c->ev_joinB) { hipEvent_t e; (void)hipEventCreateWithFlags(&e, hipEventDisableTiming); c->ev_joinB = e; }
    c->part_made = c->part_cus;
    return 0;
}
static void launch_replay(mt_ctx* c, hipStream_t s, uint32_t n_runs, bool full) {
    uint32_t* cur = (uint32_t*)c->b_cursor.p;
    if (c->use_lds == 2 && c->big_min_ops && c->n_long && c->part_cus && !mtb_partition_streams(c)) {
        // partitioned size classes: long runs on stream A's CUs in the wide block-residency
        // kernel (~21 KB of LDS, up to 7 per CU), the rest on stream B's CUs; joined.  Capture
        // batches (FULL): the block-residency kernel, one workgroup per SIMD (each padded to a
        // quarter of the CU's 160 KB of LDS: any total in (160 KB / 5, 160 KB / 4] leaves four)
        const uint32_t* runs = (const uint32_t*)c->b_runs.p;
        hipStream_t sa = (hipStream_t)c->streamA, sb = (hipStream_t)c->streamB;
        const uint32_t pad = 27u << 10;
        (void)hipEventRecord((hipEvent_t)c->ev_fork, s);
        (void)hipStreamWaitEvent(sa, (hipEvent_t)c->ev_fork, 0);
        (void)hipStreamWaitEvent(sb, (hipEvent_t)c->ev_fork, 0);
        if (full) mtk_blk_full(sa, c->n_long, c->S, c->ops, runs, cur, c->lds_blks, c->lds_heap, pad);
        else mtk_blkw(sa, c->n_long, c->S, c->ops, runs, cur);
        if (c->n_short) {
            if (full) mtk_blk_full(sb, c->n_short, c->S, c->ops, runs + c->n_long, cur, c->lds_blks, c->lds_heap);
            else mtk_blk_fast(sb, c->n_short, c->S, c->ops, runs + c->n_long, cur, c->lds_blks, c->lds_heap);
        }
        (void)hipEventRecord((hipEvent_t)c->ev_join, sa);
        (void)hipEventRecord((hipEvent_t)c->ev_joinB, sb);
        (void)hipStreamWaitEvent(s, (hipEvent_t)c->ev_join, 0);
        (void)hipStreamWaitEvent(s, (hipEvent_t)c->ev_joinB, 0);
        if (!full && c->n_short) mtk_hbm(full, s, n_runs, c->S, c->ops, cur);   // documents that outgrew LDS
        return;
    }
    if (c->use_lds == 2 && c->big_min_ops && c->n_long) {
        // size classes: long runs on stream2 in the wide block-residency kernel (launched first,
        // so the long runs take their slots before the short ones fill the CUs), the rest here,
        // joined; capture batches (FULL) take the long-document kernel
        const uint32_t* runs = (const uint32_t*)c->b_runs.p;
        hipStream_t s2 = (hipStream_t)c->stream2;
        (void)hipEventRecord((hipEvent_t)c->ev_fork, s);
        (void)hipStreamWaitEvent(s2, (hipEvent_t)c->ev_fork, 0);
        if (full) mtk_big(full, s2, c->n_long, c->S, c->ops, runs, cur, MT_G_WIN, 0, MT_G_HEAP);
        else mtk_blkw(s2, c->n_long, c->S, c->ops, runs, cur);
        if (c->n_short) {
            if (full) mtk_blk_full(s, c->n_short, c->S, c->ops, runs + c->n_long, cur, c->lds_blks, c->lds_heap);
            else mtk_blk_fast(s, c->n_short, c->S, c->ops, runs + c->n_long, cur, c->lds_blks, c->lds_heap);
        }
        (void)hipEventRecord((hipEvent_t)c->ev_join, s2);
        (void)hipStreamWaitEvent(s, (hipEvent_t)c->ev_join, 0);
        if (!full && c->n_short) mtk_hbm(full, s, n_runs, c->S, c->ops, cur);   // documents that outgrew LDS
        return;
    }
    if (c->use_lds == 3) mtk_big(full, s, n_runs, c->S, c->ops, nullptr, cur, c->lds_rows, c->lds_blks, c->lds_heap);
    else if (c->use_lds == 2) {
        if (full) mtk_blk_full(s, n_runs, c->S, c->ops, nullptr, cur, c->lds_blks, c->lds_heap);   // continues in-wave
        else if (c->n_cont == 0) {
            // no run reaches the continuation threshold: the kernel without the second engine
            mtk_blk_fast(s, n_runs, c->S, c->ops, nullptr, cur, c->lds_blks, c->lds_heap);
            mtk_hbm(full, s, n_runs, c->S, c->ops, cur);                        // documents that outgrew LDS
        } else {
            // a long run is in the batch: one launch of the kernel with the in-wave continuation
            // (the runs start in batch order, longest first under LPT; two kernels on two streams
            // let short runs take the slots first and measured slower)
            mtk_blk_fast_cont(s, n_runs, c->S, c->ops, nullptr, cur, c->lds_blks, c->lds_heap);
        }
    } else if (c->use_lds) {
        mtk_lds(full, s, n_runs, c->S, c->ops, cur, c->lds_rows, c->lds_blks, c->lds_heap);
        mtk_hbm(full, s, n_runs, c->S, c->ops, cur);
    } else mtk_hbm(full, s, n_runs, c->S, c->ops, nullptr);
}
static int mt_size_class_lists(mt_ctx* c);
static int mt_cont_lists(mt_ctx* c);
static void mt_auto_partition(mt_ctx* c);
static uint32_t mtb_cu_count(mt_ctx* c) {
    int ncu = 0;
    return hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) == hipSuccess && ncu > 0 ? (uint32_t)ncu : 256u;
}
static int mtb_launch_replay(mt_ctx* c, const MtGen& g, uint32_t n_runs) {
    if (n_runs == 0) return MT_OK;
    if (!g.enabled) mt_auto_partition(c);
    if (!g.enabled && c->use_lds == 2 && !c->big_min_ops) {
        int rc = mt_cont_lists(c);
        if (rc) return rc;
    }
    hipStream_t s = (hipStream_t)c->stream;
    if (!g.enabled && c->use_lds == 2 && c->big_min_ops) {
        int rc = mt_size_class_lists(c);
        if (rc) return rc;
    }
    (void)hipGetLastError();
    (void)hipEventRecord((hipEvent_t)c->ev0, s);
    if (g.enabled) mtk_generate(s, n_runs, c->S, c->ops, g);
    else launch_replay(c, s, n_runs, c->ops.drec || c->batch_reg || c->batch_wide);
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

static int mtb_launch_query(mt_ctx* c, const MtQuery* q, const uint32_t* grp, MtQueryOut* out, uint32_t n_groups) {
    if (!n_groups) return MT_OK;
    (void)hipGetLastError();
    hipLaunchKernelGGL(mt_query_kernel, dim3(n_groups), dim3(64), 0, (hipStream_t)c->stream, c->S, q, grp, out);
    return mtb_check(c);
}
static int mtb_launch_gather_text(mt_ctx* c, const unsigned long long* at, const uint32_t* len, const unsigned long long* off,
                                  uint16_t* dst, uint32_t n) {
    if (!n) return MT_OK;
    (void)hipGetLastError();
    hipLaunchKernelGGL(mt_gather_text_kernel, dim3(n), dim3(256), 0, (hipStream_t)c->stream, c->S.text, at, len, off, dst);
    return mtb_check(c);
}

static int mtb_launch_rows(mt_ctx* c, bool pack, uint32_t first, uint32_t n, uint32_t L, const uint64_t* dst, uint64_t* rows,
                           uint64_t* cs) {
    if (!n) return MT_OK;
    (void)hipGetLastError();
    hipLaunchKernelGGL(mt_rows_kernel, dim3(n), dim3(64), 0, (hipStream_t)c->stream, c->ops, pack ? 1 : 0, first, L, dst,
                       (unsigned long long*)rows, cs);
    return mtb_check(c);
}
static int mtb_launch_pack_size(mt_ctx* c, const uint32_t* docs, MtPackSize* out, uint32_t n, uint32_t epoch) {
    if (!n) return MT_OK;
    (void)hipGetLastError();
    hipLaunchKernelGGL(mt_pack_size_kernel, dim3(n), dim3(64), 0, (hipStream_t)c->stream, c->S, docs, out, epoch);
    return mtb_check(c);
}
static int mtb_launch_pack(mt_ctx* c, const uint32_t* docs, const uint64_t* off, uint8_t* stage, uint32_t n, uint32_t epoch) {
    if (!n) return MT_OK;
    (void)hipGetLastError();
    hipLaunchKernelGGL(mt_pack_kernel, dim3(n), dim3(64), 0, (hipStream_t)c->stream, c->S, docs, off, stage, epoch);
    return mtb_check(c);
}

#define MT_FN(name) mt_##name
#include "mt_api_impl.h"
