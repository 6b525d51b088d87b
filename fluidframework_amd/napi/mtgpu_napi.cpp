// mtgpu_napi.cpp — N-API addon over the C ABI (include/mtgpu.h).
//
// The Node/TypeScript host side of the drop-in boundary: the
// JS layer (fluidframework_amd/js/index.js) packs ISequencedDocumentMessage
// batches into the SoA op arrays of mt_op_batch and calls these functions,
// which hand typed-array memory straight to libmtgpu.so.  No compute happens
// here.  Every non-zero status is thrown as a JS Error carrying mt_last_error,
// as the reference's assert() throws (common-utils assert.ts:12-16).
// Built with g++ against /usr/include/node (no node-gyp): see __graft_entry__.
#define NAPI_VERSION 8
#include <node_api.h>

#include <math.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/mtgpu.h"

namespace {

#define NAPI_OK(call)                                                              \
    do {                                                                           \
        if ((call) != napi_ok) {                                                   \
            napi_throw_error(env, nullptr, "N-API call failed: " #call);           \
            return nullptr;                                                        \
        }                                                                          \
    } while (0)

// One JS-visible engine context.  Single-caller contract: while a syncAsync is
// pending (busy), every other call on the context throws, and destroy() is
// deferred to the worker's completion; the pending work holds a reference to
// the external, so it cannot be finalized under the worker.
struct Ctx { mt_ctx* c = nullptr; int busy = 0; bool destroy_pending = false; };

napi_value throw_rc(napi_env env, mt_ctx* c, int rc, const char* what) {
    std::string m = std::string(what) + " failed (" + std::to_string(rc) + "): " + (c ? mt_last_error(c) : "no context");
    napi_throw_error(env, nullptr, m.c_str());
    return nullptr;
}

napi_value undefined(napi_env env) { napi_value u; napi_get_undefined(env, &u); return u; }

bool get_args(napi_env env, napi_callback_info info, size_t want, napi_value* argv) {
    size_t argc = want;
    if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok || argc < want) {
        napi_throw_type_error(env, nullptr, "wrong number of arguments");
        return false;
    }
    return true;
}

mt_ctx* get_ctx(napi_env env, napi_value v) {
    void* p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p || !((Ctx*)p)->c || ((Ctx*)p)->destroy_pending) {
        napi_throw_type_error(env, nullptr, "expected an engine context (destroyed?)");
        return nullptr;
    }
    if (((Ctx*)p)->busy) {
        napi_throw_error(env, nullptr, "engine context busy: a syncAsync is pending (await it first)");
        return nullptr;
    }
    return ((Ctx*)p)->c;
}

// Typed-array view: data pointer and element count (type-checked).
template <class T> bool typed(napi_env env, napi_value v, napi_typedarray_type want, const T** data, size_t* n) {
    bool is = false;
    napi_is_typedarray(env, v, &is);
    if (!is) { napi_throw_type_error(env, nullptr, "expected a typed array"); return false; }
    napi_typedarray_type t; size_t len; void* d; napi_value ab; size_t off;
    napi_get_typedarray_info(env, v, &t, &len, &d, &ab, &off);
    if (t != want) { napi_throw_type_error(env, nullptr, "typed array has the wrong element type"); return false; }
    *data = (const T*)d; *n = len;
    return true;
}
template <class T> bool field(napi_env env, napi_value obj, const char* name, napi_typedarray_type want, const T** data, size_t* n) {
    napi_value v;
    if (napi_get_named_property(env, obj, name, &v) != napi_ok) { napi_throw_type_error(env, nullptr, name); return false; }
    if (!typed(env, v, want, data, n)) {
        std::string m = std::string("field ") + name + ": expected the documented typed array";
        napi_throw_type_error(env, nullptr, m.c_str());
        return false;
    }
    return true;
}
uint32_t u32_prop(napi_env env, napi_value obj, const char* name, uint32_t dflt) {
    napi_value v; bool has = false;
    napi_has_named_property(env, obj, name, &has);
    if (!has) return dflt;
    napi_get_named_property(env, obj, name, &v);
    uint32_t x = dflt;
    napi_get_value_uint32(env, v, &x);
    return x;
}
bool strings(napi_env env, napi_value arr, std::vector<std::string>& out) {
    bool is = false;
    napi_is_array(env, arr, &is);
    if (!is) { napi_throw_type_error(env, nullptr, "expected an array of strings"); return false; }
    uint32_t n = 0; napi_get_array_length(env, arr, &n);
    out.resize(n);
    for (uint32_t i = 0; i < n; i++) {
        napi_value e; napi_get_element(env, arr, i, &e);
        size_t len = 0;
        if (napi_get_value_string_utf8(env, e, nullptr, 0, &len) != napi_ok) { napi_throw_type_error(env, nullptr, "expected a string"); return false; }
        out[i].resize(len + 1);
        napi_get_value_string_utf8(env, e, &out[i][0], len + 1, &len);
        out[i].resize(len);
    }
    return true;
}

void ctx_finalize(napi_env, void* data, void*) {
    Ctx* x = (Ctx*)data;
    if (x->c) mt_destroy(x->c);
    delete x;
}

// create(device, limits) -> context
napi_value Create(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    int32_t dev = 0; napi_get_value_int32(env, argv[0], &dev);
    mt_limits L{};
    L.max_docs = u32_prop(env, argv[1], "maxDocs", 1);
    L.rows_per_doc = u32_prop(env, argv[1], "rowsPerDoc", 0);
    L.blocks_per_doc = u32_prop(env, argv[1], "blocksPerDoc", 0);
    L.text_per_doc = u32_prop(env, argv[1], "textPerDoc", 0);
    L.propsets_per_doc = u32_prop(env, argv[1], "propsetsPerDoc", 0);
    L.heap_per_doc = u32_prop(env, argv[1], "heapPerDoc", 0);
    L.window_per_doc = u32_prop(env, argv[1], "windowPerDoc", 0);
    L.markers_per_doc = u32_prop(env, argv[1], "markersPerDoc", 0);
    L.register_rows_per_doc = u32_prop(env, argv[1], "registerRowsPerDoc", 0);
    mt_ctx* c = nullptr;
    int rc = mt_create(dev, &L, &c);
    if (rc) { napi_value r = throw_rc(env, c, rc, "mt_create"); if (c) mt_destroy(c); return r; }
    Ctx* x = new Ctx; x->c = c;
    napi_value ext;
    NAPI_OK(napi_create_external(env, x, ctx_finalize, nullptr, &ext));
    return ext;
}

napi_value Destroy(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    void* p = nullptr;
    if (napi_get_value_external(env, argv[0], &p) == napi_ok && p && ((Ctx*)p)->c) {
        Ctx* x = (Ctx*)p;
        if (x->busy) x->destroy_pending = true;          // sync_done destroys it
        else { mt_destroy(x->c); x->c = nullptr; }
    }
    return undefined(env);
}

napi_value DocsOpen(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    uint32_t first = 0, n = 0;
    napi_get_value_uint32(env, argv[1], &first); napi_get_value_uint32(env, argv[2], &n);
    int rc = mt_docs_open(c, first, n);
    return rc ? throw_rc(env, c, rc, "mt_docs_open") : undefined(env);
}

napi_value SetResidency(napi_env env, napi_callback_info info) {
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    int32_t v[4] = {0, 0, 0, 0};
    for (int i = 0; i < 4; i++) napi_get_value_int32(env, argv[1 + i], &v[i]);
    int rc = mt_set_residency(c, v[0], v[1], v[2], v[3]);
    return rc ? throw_rc(env, c, rc, "mt_set_residency") : undefined(env);
}

// setProps(ctx, {setOff, key, value, keyJson[], keyIndex, valueJson[], valueFalsy, valueClass, valueKind,
//                valueIncr?, incrObject?})
napi_value SetProps(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    const uint32_t* off; const uint16_t* key; const int32_t* val; const uint32_t* kidx; const uint8_t* vf; const uint32_t* vc;
    size_t noff, nk, nv, nki, nvf, nvc;
    if (!field(env, argv[1], "setOff", napi_uint32_array, &off, &noff) || !field(env, argv[1], "key", napi_uint16_array, &key, &nk) ||
        !field(env, argv[1], "value", napi_int32_array, &val, &nv) || !field(env, argv[1], "keyIndex", napi_uint32_array, &kidx, &nki) ||
        !field(env, argv[1], "valueFalsy", napi_uint8_array, &vf, &nvf) || !field(env, argv[1], "valueClass", napi_uint32_array, &vc, &nvc))
        return nullptr;
    const uint8_t* vk; size_t nvk;
    if (!field(env, argv[1], "valueKind", napi_uint8_array, &vk, &nvk)) return nullptr;
    napi_value kj, vj;
    napi_get_named_property(env, argv[1], "keyJson", &kj);
    napi_get_named_property(env, argv[1], "valueJson", &vj);
    std::vector<std::string> ks, vs;
    if (!strings(env, kj, ks) || !strings(env, vj, vs)) return nullptr;
    if (noff == 0 || nk < off[noff - 1] || nv < off[noff - 1] || nki < ks.size() || nvf < vs.size() || nvc < vs.size() || nvk < vs.size()) {
        napi_throw_range_error(env, nullptr, "property table arrays are inconsistent");
        return nullptr;
    }
    std::vector<const char*> kp(ks.size() + 1), vp(vs.size() + 1);
    for (size_t i = 0; i < ks.size(); i++) kp[i] = ks[i].c_str();
    for (size_t i = 0; i < vs.size(); i++) vp[i] = vs[i].c_str();
    mt_prop_table P{};
    P.n_sets = (uint32_t)(noff - 1); P.set_off = off; P.key = key; P.value = val;
    P.n_keys = (uint32_t)ks.size(); P.key_json = kp.data(); P.key_index = kidx;
    P.n_values = (uint32_t)vs.size(); P.value_json = vp.data(); P.value_falsy = vf; P.value_class = vc; P.value_kind = vk;
    P.incr_object = MT_VAL_UNSUP;
    {   // optional: valueIncr (Int32Array, one per value) and incrObject (PropTable.incrTable)
        bool has = false;
        napi_has_named_property(env, argv[1], "valueIncr", &has);
        if (has) {
            const int32_t* vi; size_t nvi;
            if (!field(env, argv[1], "valueIncr", napi_int32_array, &vi, &nvi)) return nullptr;
            if (nvi < vs.size()) { napi_throw_range_error(env, nullptr, "valueIncr shorter than valueJson"); return nullptr; }
            P.value_incr = vi;
            napi_value io; int32_t x = MT_VAL_UNSUP;
            if (napi_get_named_property(env, argv[1], "incrObject", &io) == napi_ok) napi_get_value_int32(env, io, &x);
            P.incr_object = x;
        }
    }
    int rc = mt_set_props(c, &P);
    return rc ? throw_rc(env, c, rc, "mt_set_props") : undefined(env);
}

napi_value SetClientNames(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    std::vector<std::string> s;
    if (!strings(env, argv[1], s)) return nullptr;
    std::vector<const char*> p(s.size() + 1);
    for (size_t i = 0; i < s.size(); i++) p[i] = s[i].c_str();
    int rc = mt_set_client_names(c, (uint32_t)s.size(), p.data());
    return rc ? throw_rc(env, c, rc, "mt_set_client_names") : undefined(env);
}

napi_value SetDocClientNames(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    uint32_t doc = 0; napi_get_value_uint32(env, argv[1], &doc);
    std::vector<std::string> s;
    if (!strings(env, argv[2], s)) return nullptr;
    std::vector<const char*> p(s.size() + 1);
    for (size_t i = 0; i < s.size(); i++) p[i] = s[i].c_str();
    int rc = mt_set_doc_client_names(c, doc, (uint32_t)s.size(), p.data());
    return rc ? throw_rc(env, c, rc, "mt_set_doc_client_names") : undefined(env);
}

// setDocSnapshotChunk(ctx, docIds: Uint32Array, sizes: Float64Array): options.mergeTreeSnapshotChunkSize
// per document after ToNumber (Infinity: one chunk; sizes are rounded up, snapshotV1.ts:55, :78;
// 0, negative and NaN: no length is below it, MT_CHUNK_NONE).  New documents have the default.
napi_value SetDocSnapshotChunk(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    const uint32_t* docs; size_t nd;
    if (!typed(env, argv[1], napi_uint32_array, &docs, &nd)) return nullptr;
    const double* sz; size_t ns;
    if (!typed(env, argv[2], napi_float64_array, &sz, &ns) || ns < nd) return nullptr;
    std::vector<uint64_t> v(nd);
    for (size_t i = 0; i < nd; i++) {
        const double x = sz[i];
        v[i] = !(x > 0) ? MT_CHUNK_NONE : (x >= 1.8e19 ? MT_CHUNK_INFINITY : (uint64_t)std::ceil(x));
    }
    int rc = mt_set_doc_snapshot_chunk(c, (uint32_t)nd, docs, v.data());
    return rc ? throw_rc(env, c, rc, "mt_set_doc_snapshot_chunk") : undefined(env);
}

// reserveStaging(ctx, bytes?: number): mt_reserve_staging (pin the snapshot / text staging
// buffers once; 0 or absent: the default group budget).
napi_value ReserveStaging(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
    if (argc < 1) { napi_throw_type_error(env, nullptr, "reserveStaging(ctx, bytes?)"); return nullptr; }
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    double b = 0;
    if (argc > 1) napi_get_value_double(env, argv[1], &b);
    if (!(b >= 0)) { napi_throw_range_error(env, nullptr, "bytes must be >= 0"); return nullptr; }
    int rc = mt_reserve_staging(c, (uint64_t)b);
    return rc ? throw_rc(env, c, rc, "mt_reserve_staging") : undefined(env);
}

// A JS batch object (BatchBuilder.build / ParallelPacker parts) as an mt_op_batch over its
// typed arrays' memory; false with a pending JS exception on a malformed batch.
bool read_batch(napi_env env, napi_value obj, mt_op_batch& B) {
    B = mt_op_batch{};
    size_t nd, no, n[11], np;
    if (!field(env, obj, "docIds", napi_uint32_array, &B.doc_ids, &nd) ||
        !field(env, obj, "opOffsets", napi_uint32_array, &B.op_offsets, &no) ||
        !field(env, obj, "type", napi_uint8_array, &B.type, &n[0]) ||
        !field(env, obj, "flags", napi_uint8_array, &B.flags, &n[1]) ||
        !field(env, obj, "client", napi_uint16_array, &B.client, &n[2]) ||
        !field(env, obj, "seq", napi_int32_array, &B.seq, &n[3]) ||
        !field(env, obj, "refSeq", napi_int32_array, &B.ref_seq, &n[4]) ||
        !field(env, obj, "msn", napi_int32_array, &B.msn, &n[5]) ||
        !field(env, obj, "pos1", napi_int32_array, &B.pos1, &n[6]) ||
        !field(env, obj, "pos2", napi_int32_array, &B.pos2, &n[7]) ||
        !field(env, obj, "payloadOff", napi_uint32_array, &B.payload_off, &n[8]) ||
        !field(env, obj, "payloadLen", napi_uint32_array, &B.payload_len, &n[9]) ||
        !field(env, obj, "propId", napi_int32_array, &B.prop_id, &n[10]) ||
        !field(env, obj, "payload", napi_uint16_array, &B.payload, &np))
        return false;
    if (no != nd + 1) { napi_throw_range_error(env, nullptr, "opOffsets must have docIds.length + 1 entries"); return false; }
    B.n_runs = (uint32_t)nd;
    B.n_ops = B.op_offsets[nd];
    for (int i = 0; i < 11; i++)
        if (n[i] < B.n_ops) { napi_throw_range_error(env, nullptr, "an op array is shorter than opOffsets[n]"); return false; }
    B.payload_units = np;
    {   // optional rel: Int32Array of (marker, before, offset, pad) quads (mt_rel_pos)
        bool has = false;
        napi_has_named_property(env, obj, "rel", &has);
        if (has) {
            const int32_t* rel = nullptr; size_t nr = 0;
            if (!field(env, obj, "rel", napi_int32_array, &rel, &nr)) return false;
            B.n_rel = (uint32_t)(nr / 4); B.rel = (const mt_rel_pos*)rel;
        }
    }
    return true;
}

// applyBatch(ctx, batch): copies the batch to HBM and enqueues the replay
// (Client.applyMsg for every message of every document run).
napi_value ApplyBatch(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    mt_op_batch B;
    if (!read_batch(env, argv[1], B)) return nullptr;
    int rc = mt_apply_batch(c, &B);     // copies host arrays before returning
    return rc ? throw_rc(env, c, rc, "mt_apply_batch") : undefined(env);
}

// applyBatchParts(ctx, parts: batch[], propMaps: (Int32Array | null)[]): mt_apply_batch_parts,
// the parts of several packing threads applied as one batch without a JS-side merge
// (propMaps[p]: part p's property-set ids -> the engine table's).
napi_value ApplyBatchParts(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    bool isArr = false, isArr2 = false;
    napi_is_array(env, argv[1], &isArr); napi_is_array(env, argv[2], &isArr2);
    if (!isArr || !isArr2) { napi_throw_type_error(env, nullptr, "applyBatchParts(ctx, parts[], propMaps[])"); return nullptr; }
    uint32_t P = 0, PM = 0;
    napi_get_array_length(env, argv[1], &P); napi_get_array_length(env, argv[2], &PM);
    if (PM != P) { napi_throw_range_error(env, nullptr, "one property map per part"); return nullptr; }
    std::vector<mt_op_batch> parts(P);
    std::vector<const int32_t*> maps(P, nullptr);
    std::vector<uint32_t> mlen(P, 0);
    for (uint32_t p = 0; p < P; p++) {
        napi_value e, m;
        napi_get_element(env, argv[1], p, &e);
        if (!read_batch(env, e, parts[p])) return nullptr;
        napi_get_element(env, argv[2], p, &m);
        napi_valuetype t; napi_typeof(env, m, &t);
        if (t == napi_null || t == napi_undefined) continue;
        size_t n = 0;
        if (!typed(env, m, napi_int32_array, &maps[p], &n)) return nullptr;
        mlen[p] = (uint32_t)n;
    }
    int rc = mt_apply_batch_parts(c, P, parts.data(), maps.data(), mlen.data());   // copies before returning
    return rc ? throw_rc(env, c, rc, "mt_apply_batch_parts") : undefined(env);
}

// loadSnapshot(ctx, batch): SnapshotLoader for every document of the batch
// (segments already JSON-parsed by the JS host into 32-byte mt_load_seg records).
napi_value LoadSnapshot(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    mt_load_batch B{};
    const uint8_t* segs = nullptr;
    size_t nd, no, nh, nm, ns, nb, np;
    if (!field(env, argv[1], "docIds", napi_uint32_array, &B.doc_ids, &nd) ||
        !field(env, argv[1], "segOffsets", napi_uint32_array, &B.seg_offsets, &no) ||
        !field(env, argv[1], "headerSegments", napi_uint32_array, &B.header_segments, &nh) ||
        !field(env, argv[1], "minSeq", napi_int32_array, &B.min_seq, &nm) ||
        !field(env, argv[1], "seq", napi_int32_array, &B.seq, &ns) ||
        !field(env, argv[1], "segs", napi_uint8_array, &segs, &nb) ||
        !field(env, argv[1], "payload", napi_uint16_array, &B.payload, &np))
        return nullptr;
    if (no != nd + 1 || nh != nd || nm != nd || ns != nd) { napi_throw_range_error(env, nullptr, "per-document arrays disagree"); return nullptr; }
    if (nb < 32ull * B.seg_offsets[nd]) { napi_throw_range_error(env, nullptr, "segs shorter than 32 * segOffsets[n]"); return nullptr; }
    B.n_docs = (uint32_t)nd;
    B.segs = (const mt_load_seg*)segs;
    B.payload_units = np;
    int rc = mt_load_snapshot(c, &B);
    return rc ? throw_rc(env, c, rc, "mt_load_snapshot") : undefined(env);
}

napi_value Sync(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    int rc = mt_sync(c);
    return rc ? throw_rc(env, c, rc, "mt_sync") : undefined(env);
}

// syncAsync(ctx) -> Promise: mt_sync on a libuv worker so the event loop is not blocked.
struct SyncWork { Ctx* x; mt_ctx* c; int rc; napi_deferred d; napi_async_work w; napi_ref ref; };
void sync_exec(napi_env, void* data) { SyncWork* s = (SyncWork*)data; s->rc = mt_sync(s->c); }
void sync_done(napi_env env, napi_status, void* data) {
    SyncWork* s = (SyncWork*)data;
    std::string m = s->rc ? "mt_sync failed (" + std::to_string(s->rc) + "): " + mt_last_error(s->c) : std::string();
    s->x->busy = 0;
    if (s->x->destroy_pending) { mt_destroy(s->x->c); s->x->c = nullptr; s->x->destroy_pending = false; }
    if (s->rc == 0) napi_resolve_deferred(env, s->d, undefined(env));
    else {
        napi_value msg, err;
        napi_create_string_utf8(env, m.c_str(), m.size(), &msg);
        napi_create_error(env, nullptr, msg, &err);
        napi_reject_deferred(env, s->d, err);
    }
    napi_delete_async_work(env, s->w);
    napi_delete_reference(env, s->ref);
    delete s;
}
napi_value SyncAsync(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    void* xp = nullptr;
    napi_get_value_external(env, argv[0], &xp);
    SyncWork* s = new SyncWork{(Ctx*)xp, c, 0, nullptr, nullptr, nullptr};
    napi_value promise, name;
    NAPI_OK(napi_create_reference(env, argv[0], 1, &s->ref));     // keeps the context alive until sync_done
    s->x->busy = 1;
    NAPI_OK(napi_create_promise(env, &s->d, &promise));
    napi_create_string_utf8(env, "mt_sync", NAPI_AUTO_LENGTH, &name);
    NAPI_OK(napi_create_async_work(env, nullptr, name, sync_exec, sync_done, s, &s->w));
    NAPI_OK(napi_queue_async_work(env, s->w));
    return promise;
}

napi_value make_u32(napi_env env, const uint32_t* src, size_t n) {
    napi_value ab, ta; void* d = nullptr;
    napi_create_arraybuffer(env, 4 * n, &d, &ab);
    if (n) memcpy(d, src, 4 * n);
    napi_create_typedarray(env, napi_uint32_array, n, ab, 0, &ta);
    return ta;
}
napi_value make_i32(napi_env env, const int32_t* src, size_t n) {
    napi_value ab, ta; void* d = nullptr;
    napi_create_arraybuffer(env, 4 * n, &d, &ab);
    if (n) memcpy(d, src, 4 * n);
    napi_create_typedarray(env, napi_int32_array, n, ab, 0, &ta);
    return ta;
}

napi_value DocStatus(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    const uint32_t* docs; size_t n;
    if (!typed(env, argv[1], napi_uint32_array, &docs, &n)) return nullptr;
    std::vector<uint32_t> out(n + 1);
    int rc = mt_doc_status(c, (uint32_t)n, docs, out.data());
    return rc ? throw_rc(env, c, rc, "mt_doc_status") : make_u32(env, out.data(), n);
}

napi_value UpdateSeq(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    const uint32_t* docs; const int32_t* msn; const int32_t* seq; size_t n, n1, n2;
    if (!typed(env, argv[1], napi_uint32_array, &docs, &n) || !typed(env, argv[2], napi_int32_array, &msn, &n1) ||
        !typed(env, argv[3], napi_int32_array, &seq, &n2)) return nullptr;
    if (n1 < n || n2 < n) { napi_throw_range_error(env, nullptr, "msn/seq shorter than docs"); return nullptr; }
    int rc = mt_update_seq(c, (uint32_t)n, docs, msn, seq);
    return rc ? throw_rc(env, c, rc, "mt_update_seq") : undefined(env);
}

napi_value GetLength(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    const uint32_t* docs; const int32_t* ref; const int32_t* cli; size_t n, n1, n2;
    if (!typed(env, argv[1], napi_uint32_array, &docs, &n) || !typed(env, argv[2], napi_int32_array, &ref, &n1) ||
        !typed(env, argv[3], napi_int32_array, &cli, &n2)) return nullptr;
    if (n1 < n || n2 < n) { napi_throw_range_error(env, nullptr, "refSeq/client shorter than docs"); return nullptr; }
    std::vector<int32_t> out(n + 1);
    int rc = mt_get_length(c, (uint32_t)n, docs, ref, cli, out.data());
    return rc ? throw_rc(env, c, rc, "mt_get_length") : make_i32(env, out.data(), n);
}

// getContainingSegment(ctx, docs, pos, refSeq, client) -> {info: Int32Array (16 per query,
// mt_seg_info), json: [string | null]} (mt_get_containing_segment)
napi_value GetContainingSegment(napi_env env, napi_callback_info info) {
    napi_value argv[5];
    if (!get_args(env, info, 5, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    const uint32_t* docs; const int32_t* pos; const int32_t* ref; const int32_t* cli; size_t n, n1, n2, n3;
    if (!typed(env, argv[1], napi_uint32_array, &docs, &n) || !typed(env, argv[2], napi_int32_array, &pos, &n1) ||
        !typed(env, argv[3], napi_int32_array, &ref, &n2) || !typed(env, argv[4], napi_int32_array, &cli, &n3)) return nullptr;
    if (n1 < n || n2 < n || n3 < n) { napi_throw_range_error(env, nullptr, "pos/refSeq/client shorter than docs"); return nullptr; }
    std::vector<mt_seg_info> out(n + 1);
    const char* arena = nullptr; const uint64_t* off = nullptr;
    int rc = mt_get_containing_segment(c, (uint32_t)n, docs, pos, ref, cli, out.data(), &arena, &off);
    if (rc) return throw_rc(env, c, rc, "mt_get_containing_segment");
    napi_value o, js;
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "info", make_i32(env, (const int32_t*)out.data(), 16 * n));
    NAPI_OK(napi_create_array_with_length(env, n, &js));
    for (size_t i = 0; i < n; i++) {
        napi_value s;
        if (out[i].found) napi_create_string_utf8(env, arena + off[i], (size_t)(off[i + 1] - off[i]), &s);
        else napi_get_null(env, &s);
        napi_set_element(env, js, (uint32_t)i, s);
    }
    napi_set_named_property(env, o, "json", js);
    return o;
}

// snapshotV1(ctx, docs, msn, seq) -> [{blobs: [header, body_0, ...], digest: BigInt}]
// snapshotLegacy(ctx, docs, msn, seq) -> [{blobs: [header(, body)], digest: BigInt}]
static napi_value snapshot_blobs(napi_env env, napi_callback_info info, bool legacy) {
    napi_value argv[4];
    if (!get_args(env, info, 4, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    const uint32_t* docs; const int32_t* msn; const int32_t* seq; size_t n, n1, n2;
    if (!typed(env, argv[1], napi_uint32_array, &docs, &n) || !typed(env, argv[2], napi_int32_array, &msn, &n1) ||
        !typed(env, argv[3], napi_int32_array, &seq, &n2)) return nullptr;
    if (n1 < n || n2 < n) { napi_throw_range_error(env, nullptr, "msn/seq shorter than docs"); return nullptr; }
    std::vector<uint64_t> dig(n + 1);
    const char* arena = nullptr; const uint64_t* boff = nullptr; const uint32_t* bfirst = nullptr;
    int rc = legacy ? mt_snapshot_legacy(c, (uint32_t)n, docs, msn, seq, dig.data(), &arena, &boff, &bfirst)
                    : mt_snapshot_v1(c, (uint32_t)n, docs, msn, seq, dig.data(), &arena, &boff, &bfirst);
    if (rc) return throw_rc(env, c, rc, legacy ? "mt_snapshot_legacy" : "mt_snapshot_v1");
    napi_value out;
    NAPI_OK(napi_create_array_with_length(env, n, &out));
    for (size_t i = 0; i < n; i++) {
        napi_value o, blobs, d;
        napi_create_object(env, &o);
        const uint32_t b0 = bfirst[i], b1 = bfirst[i + 1];
        napi_create_array_with_length(env, b1 - b0, &blobs);
        for (uint32_t j = b0; j < b1; j++) {
            napi_value s;
            napi_create_string_utf8(env, arena + boff[j], (size_t)(boff[j + 1] - boff[j]), &s);
            napi_set_element(env, blobs, j - b0, s);
        }
        napi_create_bigint_uint64(env, dig[i], &d);
        napi_set_named_property(env, o, "blobs", blobs);
        napi_set_named_property(env, o, "digest", d);
        napi_set_element(env, out, (uint32_t)i, o);
    }
    return out;
}
napi_value SnapshotV1(napi_env env, napi_callback_info info) { return snapshot_blobs(env, info, false); }
napi_value SnapshotLegacy(napi_env env, napi_callback_info info) { return snapshot_blobs(env, info, true); }

// getText(ctx, docs) -> [string]: the observer's text (UTF-16 code units as-is)
napi_value GetText(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    const uint32_t* docs; size_t n;
    if (!typed(env, argv[1], napi_uint32_array, &docs, &n)) return nullptr;
    const uint16_t* arena = nullptr; const uint64_t* off = nullptr;
    int rc = mt_get_text(c, (uint32_t)n, docs, &arena, &off);
    if (rc) return throw_rc(env, c, rc, "mt_get_text");
    napi_value out;
    NAPI_OK(napi_create_array_with_length(env, n, &out));
    for (size_t i = 0; i < n; i++) {
        napi_value s;
        napi_create_string_utf16(env, (const char16_t*)(arena + off[i]), (size_t)(off[i + 1] - off[i]), &s);
        napi_set_element(env, out, (uint32_t)i, s);
    }
    return out;
}

// deltaCapture(ctx, capacity): record the delta / maintenance callbacks of later batches
napi_value DeltaCapture(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    int64_t cap = 0; napi_get_value_int64(env, argv[1], &cap);
    int rc = mt_delta_capture(c, cap > 0 ? (uint64_t)cap : 0);
    return rc ? throw_rc(env, c, rc, "mt_delta_capture") : undefined(env);
}

// deltaRecords(ctx) -> Int32Array of 8 per record (mt_delta_rec: op, kind, pos, len, seg, a, b, pad)
napi_value DeltaRecords(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    const mt_delta_rec* r = nullptr; uint64_t n = 0;
    int rc = mt_delta_records(c, &r, &n);
    if (rc) return throw_rc(env, c, rc, "mt_delta_records");
    return make_i32(env, (const int32_t*)r, (size_t)n * 8);
}

// deltaText(ctx) -> string: the UTF-16 text of the last batch's pasted text segments
// (INSERT records with b == 0 index it by pad / len), mt_delta_text
napi_value DeltaText(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    const uint16_t* t = nullptr; uint64_t n = 0;
    int rc = mt_delta_text(c, &t, &n, nullptr);
    if (rc) return throw_rc(env, c, rc, "mt_delta_text");
    napi_value s;
    NAPI_OK(napi_create_string_utf16(env, (const char16_t*)t, (size_t)n, &s));
    return s;
}

// docPset(ctx, doc, id) -> {keys: Uint32Array, values: Int32Array} (interned ids, insertion order)
napi_value DocPset(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    if (!get_args(env, info, 3, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    uint32_t doc = 0; int32_t id = -1;
    napi_get_value_uint32(env, argv[1], &doc); napi_get_value_int32(env, argv[2], &id);
    uint16_t k[MT_MAX_PROP_KEYS]; int32_t v[MT_MAX_PROP_KEYS]; uint32_t n = 0;
    int rc = mt_doc_pset(c, doc, id, k, v, &n);
    if (rc) return throw_rc(env, c, rc, "mt_doc_pset");
    uint32_t k32[MT_MAX_PROP_KEYS];
    for (uint32_t i = 0; i < n; i++) k32[i] = k[i];
    napi_value o;
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "keys", make_u32(env, k32, n));
    napi_set_named_property(env, o, "values", make_i32(env, v, n));
    return o;
}

napi_value LastError(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return nullptr;
    mt_ctx* c = get_ctx(env, argv[0]); if (!c) return nullptr;
    napi_value s;
    napi_create_string_utf8(env, mt_last_error(c), NAPI_AUTO_LENGTH, &s);
    return s;
}

const napi_property_attributes kAttr = (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable);

napi_value Init(napi_env env, napi_value exports) {
    const napi_property_descriptor props[] = {
        {"create", nullptr, Create, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"destroy", nullptr, Destroy, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"docsOpen", nullptr, DocsOpen, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"setResidency", nullptr, SetResidency, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"setProps", nullptr, SetProps, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"setClientNames", nullptr, SetClientNames, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"setDocClientNames", nullptr, SetDocClientNames, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"setDocSnapshotChunk", nullptr, SetDocSnapshotChunk, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"reserveStaging", nullptr, ReserveStaging, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"applyBatch", nullptr, ApplyBatch, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"applyBatchParts", nullptr, ApplyBatchParts, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"loadSnapshot", nullptr, LoadSnapshot, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"sync", nullptr, Sync, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"syncAsync", nullptr, SyncAsync, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"docStatus", nullptr, DocStatus, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"updateSeq", nullptr, UpdateSeq, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"getLength", nullptr, GetLength, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"getContainingSegment", nullptr, GetContainingSegment, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"snapshotV1", nullptr, SnapshotV1, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"snapshotLegacy", nullptr, SnapshotLegacy, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"getText", nullptr, GetText, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"deltaCapture", nullptr, DeltaCapture, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"deltaRecords", nullptr, DeltaRecords, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"deltaText", nullptr, DeltaText, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"docPset", nullptr, DocPset, nullptr, nullptr, nullptr, kAttr, nullptr},
        {"lastError", nullptr, LastError, nullptr, nullptr, nullptr, kAttr, nullptr},
    };
    napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
