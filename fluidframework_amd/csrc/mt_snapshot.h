// mt_snapshot.h — SnapshotV1 extraction + JSON emission from one document's
// engine state (host side of mt_snapshot_v1 / mt_get_text / mt_dump_segments).
//
// Restates Client.snapshot -> SnapshotV1.extractSync/emit
// (MT/client.ts:923-956, MT/snapshotV1.ts:70-256, MT/snapshotChunks.ts:125-149)
// for the passive-observer path: walk segments in tree order
// (walkAllSegments, mergeTree.ts:2998), elide rows removed at or below the MSN,
// greedily coalesce rows at or below the MSN (TextSegment.canAppend +
// matchProperties on clones), keep merge info for the rest, chunk at
// options.mergeTreeSnapshotChunkSize (default 10,000) characters, and serialize exactly as
// JSON.stringify does.
#pragma once
#include <limits.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <string>
#include <vector>
#include "mt_core.h"

struct MtSnapView {                  // host copy of one document's state
    MtDocHdr hdr;
    const MtRow* R;
    const MtBlk* blk; const uint16_t* text; const MtPSet* pset;
};
struct MtNames {                     // host-interned strings
    std::vector<std::string> key_json;
    std::vector<uint32_t> key_index;
    std::vector<std::string> value_json;
    std::vector<uint32_t> value_class;
    std::vector<std::string> client_json;
};

namespace mtsnap {

inline void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o.push_back((char)cp);
    else if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3F))); }
    else if (cp < 0x10000) { o.push_back((char)(0xE0 | (cp >> 12))); o.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); o.push_back((char)(0x80 | (cp & 0x3F))); }
    else { o.push_back((char)(0xF0 | (cp >> 18))); o.push_back((char)(0x80 | ((cp >> 12) & 0x3F))); o.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); o.push_back((char)(0x80 | (cp & 0x3F))); }
}
// JSON.stringify string quoting over UTF-16 code units (well-formed stringify).
inline void quote16(std::string& o, const uint16_t* s, size_t n) {
    static const char hx[] = "0123456789abcdef";
    // the plain prefix (printable ASCII other than '"' and '\\') is written byte by byte into
    // place; the general loop takes over at the first unit that needs more
    const size_t o0 = o.size();
    o.resize(o0 + n + 2);
    char* d = &o[o0];
    *d++ = '"';
    size_t i = 0;
    for (; i < n; i++) {
        const uint16_t c = s[i];
        if (c < 0x20 || c >= 0x7F || c == '"' || c == '\\') break;
        *d++ = (char)c;
    }
    if (i == n) { *d = '"'; return; }
    o.resize(o0 + 1 + i);
    for (; i < n; i++) {
        const uint16_t c = s[i];
        if (c == '"') { o += "\\\""; continue; }
        if (c == '\\') { o += "\\\\"; continue; }
        if (c < 0x20) {
            if (c == '\b') o += "\\b"; else if (c == '\f') o += "\\f"; else if (c == '\n') o += "\\n";
            else if (c == '\r') o += "\\r"; else if (c == '\t') o += "\\t";
            else { o += "\\u00"; o.push_back(hx[c >> 4]); o.push_back(hx[c & 15]); }
            continue;
        }
        if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
            put_utf8(o, 0x10000u + (((uint32_t)c - 0xD800u) << 10) + ((uint32_t)s[i + 1] - 0xDC00u));
            i++; continue;
        }
        if (c >= 0xD800 && c <= 0xDFFF) {
            o += "\\u"; o.push_back(hx[c >> 12]); o.push_back(hx[(c >> 8) & 15]); o.push_back(hx[(c >> 4) & 15]); o.push_back(hx[c & 15]);
            continue;
        }
        put_utf8(o, c);
    }
    o.push_back('"');
}
inline void put_int(std::string& o, long long v) { o += std::to_string(v); }

// A property map as JSON: array-index keys ascending, then insertion order.
// (p: the map's first chunk; key i is in chunk i / 16, MtPSet)
inline int pset_key(const MtPSet* p, int i) { return p[i >> 4].key[i & 15]; }
inline int pset_val(const MtPSet* p, int i) { return p[i >> 4].val[i & 15]; }
inline void props_json(std::string& o, const MtPSet* p, const MtNames& nm) {
    const int n = p->n < MT_PKEYS ? p->n : MT_PKEYS;
    int order[MT_PKEYS]; int m = 0;
    int idx[MT_PKEYS]; int ni = 0;
    for (int i = 0; i < n; i++) if (nm.key_index[pset_key(p, i)] != 0xFFFFFFFFu) idx[ni++] = i;
    std::sort(idx, idx + ni, [&](int a, int b) { return nm.key_index[pset_key(p, a)] < nm.key_index[pset_key(p, b)]; });
    for (int i = 0; i < ni; i++) order[m++] = idx[i];
    for (int i = 0; i < n; i++) if (nm.key_index[pset_key(p, i)] == 0xFFFFFFFFu) order[m++] = i;
    o.push_back('{');
    bool first = true;
    for (int q = 0; q < m; q++) {
        const int i = order[q], v = pset_val(p, i);
        if (v == MT_VAL_UNDEF) continue;                       // JSON.stringify skips undefined members
        if (!first) o.push_back(',');
        first = false;
        o += nm.key_json[pset_key(p, i)]; o.push_back(':');
        if (v >= 0) o += nm.value_json[v];
        else if (v <= MT_VAL_CONS_BASE) { o += "{\"seq\":"; put_int(o, (long long)MT_VAL_CONS_BASE - v); o.push_back('}'); }
        else o += "null";                                       // NaN
    }
    o.push_back('}');
}

template <class F> void walk_all(const MtSnapView& v, int B, F& f) {
    const MtBlk& b = v.blk[B];
    for (int i = 0; i < b.n; i++) {
        if (b.height == 0) f(b.c[i]);
        else walk_all(v, b.c[i], f);
    }
}

// TextSegment/Marker toJSONObject (textSegment.ts:48-54, mergeTree.ts:649-653); props: the
// property map's JSON, null when properties are undefined.
inline void seg_json_of(std::string& o, bool marker, int refType, const std::string* props, const uint16_t* txt, size_t tn) {
    if (marker) {
        o += "{\"marker\":{\"refType\":"; put_int(o, refType); o += "}";
        if (props) { o += ",\"props\":"; o += *props; }
        o += "}";
    } else if (props) {
        o += "{\"text\":"; quote16(o, txt, tn); o += ",\"props\":"; o += *props; o += "}";
    } else {
        quote16(o, txt, tn);
    }
}
// The JSON of a document's property maps, each written once (an annotate-heavy document
// repeats a few maps over thousands of segments).
struct PropsJson {
    const MtSnapView& v; const MtNames& nm;
    std::vector<std::string> js; std::vector<uint8_t> have;
    PropsJson(const MtSnapView& v_, const MtNames& nm_) : v(v_), nm(nm_), js(v_.hdr.psetTop), have(v_.hdr.psetTop, 0) {}
    const std::string* get(int ps) {
        if (ps < 0) return nullptr;
        if (ps >= (int)have.size()) { js.resize(ps + 1); have.resize(ps + 1, 0); }
        if (!have[ps]) { props_json(js[ps], v.pset + ps, nm); have[ps] = 1; }
        return &js[ps];
    }
};
// Segment JSON texts back to back, each followed by its separator (one buffer, not one
// allocation per segment; a chunk's segments are one append).
struct SegList {
    std::string buf; std::vector<size_t> off{0};
    size_t size() const { return off.size() - 1; }
    void end() { buf.push_back(','); off.push_back(buf.size()); }
    void putRange(std::string& o, size_t a, size_t n) const { if (n) o.append(buf, off[a], off[a + n] - off[a] - 1); }
    size_t bytes(size_t a, size_t n) const { return off[a + n] - off[a]; }
};
inline void seg_json(std::string& o, const MtSnapView& v, PropsJson& pj, int s, const uint16_t* txt, size_t tn) {
    seg_json_of(o, (v.R[s].meta & MT_M_MARKER) != 0, v.R[s].toff, pj.get(v.R[s].props), txt, tn);
}

// matchProperties class of a stored value; NaN, undefined and fresh consensus objects (< 0)
// equal nothing, and a map holding one (pad[2]) matches no map, itself included.
inline uint32_t value_class_of(const MtNames& nm, int v) { return v >= 0 ? nm.value_class[v] : 0xFFFFFFFFu; }
inline bool props_match(const MtSnapView& v, const MtNames& nm, int a, int b) {
    if (a == b) return a < 0 || v.pset[a].pad[2] == 0;
    if (a < 0 || b < 0) return false;
    const MtPSet* pa = v.pset + a; const MtPSet* pb = v.pset + b;
    if (pa->n != pb->n || pa->pad[2] || pb->pad[2]) return false;
    for (int i = 0; i < pa->n; i++) {
        bool f = false;
        for (int j = 0; j < pb->n; j++)
            if (pset_key(pb, j) == pset_key(pa, i) && value_class_of(nm, pset_val(pb, j)) == value_class_of(nm, pset_val(pa, i))) f = true;
        if (!f) return false;
    }
    return true;
}

// matchProperties of two staged maps, memoized by id pair (a document alternates a few maps).
struct PropsMatch {
    const MtSnapView& v; const MtNames& nm;
    long long key[16]; bool val[16];
    PropsMatch(const MtSnapView& v_, const MtNames& nm_) : v(v_), nm(nm_) { for (auto& k : key) k = -1; }
    bool operator()(int a, int b) {
        if (a == b) return a < 0 || v.pset[a].pad[2] == 0;
        if (a < 0 || b < 0) return false;
        const long long k = ((long long)a << 32) | (unsigned)b;
        const int h = (int)(((unsigned)a * 31u + (unsigned)b) & 15u);
        if (key[h] == k) return val[h];
        key[h] = k; val[h] = props_match(v, nm, a, b);
        return val[h];
    }
};
// chunk: options.mergeTreeSnapshotChunkSize (snapshotV1.ts:55; 0: SnapshotV1.chunkSize;
// MT_CHUNK_NONE: no length is below it).  Returns no blobs where the reference's chunk loop
// (snapshotV1.ts:98-114) never ends: a chunk that takes no segment while segments remain.
inline std::vector<std::string> snapshot_blobs(const MtSnapView& v, const MtNames& nm,
                                               const std::vector<std::string>* doc_clients = nullptr,
                                               uint64_t chunk = 0) {
    const unsigned long long chunkLen = chunk == MT_CHUNK_NONE ? 0ull : (chunk ? (unsigned long long)chunk : 10000ull);
    const std::vector<std::string>& cj = doc_clients ? *doc_clients : nm.client_json;
    const int minSeq = v.hdr.minSeq, curSeq = v.hdr.curSeq;
    PropsJson pj(v, nm);
    PropsMatch pm_(v, nm);
    SegList segs; std::vector<long long> lens;
    segs.buf.reserve((size_t)v.hdr.rowTop * 48); segs.off.reserve((size_t)v.hdr.rowTop + 1); lens.reserve(v.hdr.rowTop);
    int prev = -1; std::vector<uint16_t> ptext; bool pcloned = false;
    auto client = [&](int c) -> const std::string& {
        static const std::string orig = "\"original\"";
        return (c >= 0 && c < (int)cj.size()) ? cj[c] : orig;
    };
    auto pushPrev = [&]() {
        if (prev < 0) return;
        std::string& o = segs.buf;
        if (pcloned) { seg_json(o, v, pj, prev, ptext.data(), ptext.size()); lens.push_back((long long)ptext.size()); }
        else { seg_json(o, v, pj, prev, v.text + v.R[prev].toff, (size_t)v.R[prev].len); lens.push_back(v.R[prev].len); }
        segs.end();
    };
    auto extract = [&](int s) {
        const bool removed = (v.R[s].meta & MT_M_REMOVED) != 0;
        if (removed && v.R[s].rseq <= minSeq) return;                  // removed at/below the MSN: elided
        if (v.R[s].seq <= minSeq && !removed) {                         // coalesce candidates
            if (prev < 0) { prev = s; pcloned = false; return; }
            const bool pm = (v.R[prev].meta & MT_M_MARKER) != 0, sm = (v.R[s].meta & MT_M_MARKER) != 0;
            bool ok = !pm && !sm;
            if (ok) {
                const uint16_t* pt = pcloned ? ptext.data() : v.text + v.R[prev].toff;
                const size_t pl = pcloned ? ptext.size() : (size_t)v.R[prev].len;
                ok = !(pl > 0 && pt[pl - 1] == '\n') && ((long long)pl <= MT_GRAN || v.R[s].len <= MT_GRAN);
            }
            if (ok && pm_(v.R[prev].props, v.R[s].props)) {
                if (!pcloned) { ptext.assign(v.text + v.R[prev].toff, v.text + v.R[prev].toff + v.R[prev].len); pcloned = true; }
                ptext.insert(ptext.end(), v.text + v.R[s].toff, v.text + v.R[s].toff + v.R[s].len);
            } else { pushPrev(); prev = s; pcloned = false; }
            return;
        }
        pushPrev(); prev = -1; pcloned = false;
        std::string& o = segs.buf;
        o += "{\"json\":";
        const bool marker = (v.R[s].meta & MT_M_MARKER) != 0;
        seg_json(o, v, pj, s, marker ? nullptr : v.text + v.R[s].toff, marker ? 0 : (size_t)v.R[s].len);
        if (v.R[s].seq > minSeq) { o += ",\"seq\":"; put_int(o, v.R[s].seq); o += ",\"client\":"; o += client((int)(v.R[s].meta & MT_M_CLIENT)); }
        if (removed) { o += ",\"removedSeq\":"; put_int(o, v.R[s].rseq); o += ",\"removedClient\":"; o += client((int)v.R[s].rcl); }
        o += "}";
        segs.end(); lens.push_back(v.R[s].len);
    };
    walk_all(v, v.hdr.root, extract);
    pushPrev();
    struct Chunk { size_t start, count; long long length; };
    std::vector<Chunk> chunks; size_t total = 0; long long totalLen = 0;
    do {
        Chunk c{total, 0, 0};
        while ((unsigned long long)c.length < chunkLen && c.start + c.count < segs.size()) { c.length += lens[c.start + c.count]; c.count++; }
        if (c.count == 0 && total < segs.size()) return {};       // the reference loops forever here
        chunks.push_back(c); total += c.count; totalLen += c.length;
    } while (total < segs.size());
    std::vector<std::string> blobs;
    for (size_t k = 0; k < chunks.size(); k++) {
        const Chunk& c = chunks[k];
        std::string o;
        o.reserve(segs.bytes(c.start, c.count) + 256 + 16 * chunks.size());
        o += "{\"version\":\"1\",\"segmentCount\":"; put_int(o, (long long)c.count);
        o += ",\"length\":"; put_int(o, c.length); o += ",\"segments\":[";
        segs.putRange(o, c.start, c.count);
        o += "],\"startIndex\":"; put_int(o, (long long)c.start);
        if (k == 0) {
            o += ",\"headerMetadata\":{\"minSequenceNumber\":"; put_int(o, minSeq);
            o += ",\"sequenceNumber\":"; put_int(o, curSeq);
            o += ",\"orderedChunkMetadata\":[{\"id\":\"header\"}";
            for (size_t q = 1; q < chunks.size(); q++) { o += ",{\"id\":\"body_"; put_int(o, (long long)(q - 1)); o += "\"}"; }
            o += "],\"totalLength\":"; put_int(o, totalLen); o += ",\"totalSegmentCount\":"; put_int(o, (long long)total); o += "}";
        }
        o += "}";
        blobs.push_back(std::move(o));
    }
    return blobs;
}

// Client.snapshot without newMergeTreeSnapshotFormat -> SnapshotLegacy.extractSync/emit
// (MT/client.ts:950-954, MT/snapshotlegacy.ts:74-240, MT/snapshotChunks.ts:79-119,:161-180).
// mergeTree.map at (minSeq, NonCollabClient) visits exactly the rows inserted at or
// below the MSN and not removed at or below it (removes above the MSN keep their
// text); all of them coalesce greedily (canAppend + matchProperties on clones).
// Rows above the MSN are left to the catch-up ops blob, which the host appends.
// Blob 0 is "header"; blob 1, if any, is "body".  chunk: options.mergeTreeSnapshotChunkSize as
// in snapshot_blobs, the header chunk's approximate length (snapshotlegacy.ts:71, :109).
inline std::vector<std::string> snapshot_legacy_blobs(const MtSnapView& v, const MtNames& nm, uint64_t chunk = 0) {
    const int minSeq = v.hdr.minSeq;
    PropsJson pj(v, nm);
    PropsMatch pm_(v, nm);
    SegList segs; std::vector<long long> lens;
    int prev = -1; std::vector<uint16_t> ptext; bool pcloned = false;
    auto pushPrev = [&]() {
        if (prev < 0) return;
        std::string& o = segs.buf;
        const bool pm = (v.R[prev].meta & MT_M_MARKER) != 0;
        if (pcloned) { seg_json(o, v, pj, prev, ptext.data(), ptext.size()); lens.push_back((long long)ptext.size()); }
        else {
            seg_json(o, v, pj, prev, pm ? nullptr : v.text + v.R[prev].toff, pm ? 0 : (size_t)v.R[prev].len);
            lens.push_back(v.R[prev].len);
        }
        segs.end();
    };
    auto extract = [&](int s) {                                         // snapshotlegacy.ts:190-209
        const bool removed = (v.R[s].meta & MT_M_REMOVED) != 0;
        if (v.R[s].seq > minSeq || (removed && v.R[s].rseq <= minSeq)) return;
        if (prev >= 0) {
            const bool pm = (v.R[prev].meta & MT_M_MARKER) != 0, sm = (v.R[s].meta & MT_M_MARKER) != 0;
            bool ok = !pm && !sm;
            if (ok) {
                const uint16_t* pt = pcloned ? ptext.data() : v.text + v.R[prev].toff;
                const size_t pl = pcloned ? ptext.size() : (size_t)v.R[prev].len;
                ok = !(pl > 0 && pt[pl - 1] == '\n') && ((long long)pl <= MT_GRAN || v.R[s].len <= MT_GRAN);
            }
            if (ok && pm_(v.R[prev].props, v.R[s].props)) {
                if (!pcloned) { ptext.assign(v.text + v.R[prev].toff, v.text + v.R[prev].toff + v.R[prev].len); pcloned = true; }
                ptext.insert(ptext.end(), v.text + v.R[s].toff, v.text + v.R[s].toff + v.R[s].len);
                return;
            }
            pushPrev();
        }
        prev = s; pcloned = false;
    };
    walk_all(v, v.hdr.root, extract);
    pushPrev();
    long long total = 0;
    for (long long l : lens) total += l;                                // header.segmentsTotalLength (:181, :230-237)
    struct Chunk { size_t start, count; long long length; };
    auto take = [&](long long approx, size_t start) {                   // getSeqLengthSegs (:74-98)
        Chunk c{start, 0, 0};
        while (c.length < approx && c.start + c.count < segs.size()) { c.length += lens[c.start + c.count]; c.count++; }
        return c;
    };
    auto chunkStr = [&](const Chunk& c, bool header) {
        std::string o = "{\"chunkStartSegmentIndex\":"; put_int(o, (long long)c.start);
        o += ",\"chunkSegmentCount\":"; put_int(o, (long long)c.count);
        o += ",\"chunkLengthChars\":"; put_int(o, c.length);
        o += ",\"totalLengthChars\":"; put_int(o, total);
        o += ",\"totalSegmentCount\":"; put_int(o, (long long)segs.size());
        o += ",\"chunkSequenceNumber\":"; put_int(o, minSeq);
        o += ",\"segmentTexts\":[";
        o.reserve(o.size() + segs.bytes(c.start, c.count) + 256);
        segs.putRange(o, c.start, c.count);
        o += "]";
        if (header) {                                                   // buildHeaderMetadataForLegecyChunk
            o += ",\"headerMetadata\":{\"orderedChunkMetadata\":[{\"id\":\"header\"}";
            if (c.length < total) o += ",{\"id\":\"body\"}";
            o += "],\"sequenceNumber\":"; put_int(o, minSeq);          // minSequenceNumber is undefined: omitted
            o += ",\"totalLength\":"; put_int(o, total);
            o += ",\"totalSegmentCount\":"; put_int(o, (long long)segs.size()); o += "}";
        }
        o += "}";
        return o;
    };
    std::vector<std::string> blobs;
    const long long first = chunk == MT_CHUNK_NONE ? 0 : (chunk == 0 ? 10000 : (chunk >= (uint64_t)LLONG_MAX ? LLONG_MAX : (long long)chunk));
    const Chunk c1 = take(first, 0);                                   // chunkSize ?? SnapshotLegacy.sizeOfFirstChunk
    blobs.push_back(chunkStr(c1, true));
    if (c1.count < segs.size()) blobs.push_back(chunkStr(take(total, c1.count), false));
    return blobs;
}

inline uint64_t xxh64(const uint8_t* p, size_t len, uint64_t seed) {
    const uint64_t P1 = 11400714785074694791ULL, P2 = 14029467366897019727ULL, P3 = 1609587929392839161ULL,
                   P4 = 9650029242287828579ULL, P5 = 2870177450012600261ULL;
    auto rotl = [](uint64_t x, int r) { return (x << r) | (x >> (64 - r)); };
    auto rd64 = [](const uint8_t* q) { uint64_t x; memcpy(&x, q, 8); return x; };
    auto rd32 = [](const uint8_t* q) { uint32_t x; memcpy(&x, q, 4); return (uint64_t)x; };
    auto rnd = [&](uint64_t acc, uint64_t in) { acc += in * P2; acc = rotl(acc, 31); return acc * P1; };
    const uint8_t* e = p + len; uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        do { v1 = rnd(v1, rd64(p)); v2 = rnd(v2, rd64(p + 8)); v3 = rnd(v3, rd64(p + 16)); v4 = rnd(v4, rd64(p + 24)); p += 32; } while (p + 32 <= e);
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        for (uint64_t vv : {v1, v2, v3, v4}) { h ^= rnd(0, vv); h = h * P1 + P4; }
    } else h = seed + P5;
    h += (uint64_t)len;
    while (p + 8 <= e) { h ^= rnd(0, rd64(p)); h = rotl(h, 27) * P1 + P4; p += 8; }
    if (p + 4 <= e) { h ^= rd32(p) * P1; h = rotl(h, 23) * P2 + P3; p += 4; }
    while (p < e) { h ^= (*p) * P5; h = rotl(h, 11) * P1; p++; }
    h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
    return h;
}
// xxh64 fed in pieces (the same value as xxh64 of the pieces back to back).
struct Xxh64 {
    static constexpr uint64_t P1 = 11400714785074694791ULL, P2 = 14029467366897019727ULL, P3 = 1609587929392839161ULL,
                              P4 = 9650029242287828579ULL, P5 = 2870177450012600261ULL;
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1, total = 0;
    uint8_t tail[32]; size_t tn = 0;
    static uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
    static uint64_t rd64(const uint8_t* q) { uint64_t x; memcpy(&x, q, 8); return x; }
    static uint64_t rnd(uint64_t acc, uint64_t in) { acc += in * P2; acc = rotl(acc, 31); return acc * P1; }
    void stripe(const uint8_t* p) { v1 = rnd(v1, rd64(p)); v2 = rnd(v2, rd64(p + 8)); v3 = rnd(v3, rd64(p + 16)); v4 = rnd(v4, rd64(p + 24)); }
    void update(const uint8_t* p, size_t len) {
        total += len;
        if (tn) {
            const size_t k = (32 - tn) < len ? (32 - tn) : len;
            memcpy(tail + tn, p, k); tn += k; p += k; len -= k;
            if (tn < 32) return;
            stripe(tail); tn = 0;
        }
        for (; len >= 32; p += 32, len -= 32) stripe(p);
        memcpy(tail, p, len); tn = len;
    }
    uint64_t digest() const {
        uint64_t h;
        if (total >= 32) {
            h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
            for (uint64_t vv : {v1, v2, v3, v4}) { h ^= rnd(0, vv); h = h * P1 + P4; }
        } else h = P5;
        h += total;
        const uint8_t* p = tail; const uint8_t* e = tail + tn;
        while (p + 8 <= e) { h ^= rnd(0, rd64(p)); h = rotl(h, 27) * P1 + P4; p += 8; }
        if (p + 4 <= e) { uint32_t x; memcpy(&x, p, 4); h ^= (uint64_t)x * P1; h = rotl(h, 23) * P2 + P3; p += 4; }
        while (p < e) { h ^= (*p) * P5; h = rotl(h, 11) * P1; p++; }
        h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
        return h;
    }
};
// xxh64 (seed 0) of the blobs each preceded by its 8-byte little-endian length.
inline uint64_t blobs_digest(const std::vector<std::string>& blobs) {
    Xxh64 x;
    for (const auto& b : blobs) { const uint64_t n = b.size(); x.update((const uint8_t*)&n, 8); x.update((const uint8_t*)b.data(), n); }
    return x.digest();
}

inline void observer_text(const MtSnapView& v, std::vector<uint16_t>& out) {
    auto f = [&](int s) {
        if (v.R[s].meta & (MT_M_REMOVED | MT_M_MARKER)) return;
        out.insert(out.end(), v.text + v.R[s].toff, v.text + v.R[s].toff + v.R[s].len);
    };
    walk_all(v, v.hdr.root, f);
}

inline uint32_t fnv1a(const std::string& s) { uint32_t h = 2166136261u; for (unsigned char c : s) { h ^= c; h *= 16777619u; } return h; }

// 12 int32 per row, same layout as the oracle's ora_dump_segments.
inline void dump_rows(const MtSnapView& v, const MtNames& nm, std::vector<int32_t>& rows) {
    auto f = [&](int s) {
        int32_t r[12];
        const uint32_t mt = v.R[s].meta;
        r[0] = v.R[s].len; r[1] = v.R[s].seq; r[2] = (mt & MT_M_CLIENT) == MT_NONCOLLAB ? -1 : (int32_t)(mt & MT_M_CLIENT);
        const bool removed = (mt & MT_M_REMOVED) != 0;
        r[3] = removed ? v.R[s].rseq : INT32_MIN; r[4] = removed ? (int32_t)v.R[s].rcl : -1;
        r[5] = (int32_t)(v.R[s].ovl & 0xFFFFFFFFull); r[6] = (int32_t)(v.R[s].ovl >> 32);
        if (v.R[s].props >= 0) { std::string js; props_json(js, v.pset + v.R[s].props, nm); r[7] = (int32_t)(fnv1a(js) & 0x7FFFFFFF); }
        else r[7] = -1;
        r[8] = (mt & MT_M_MARKER) ? v.R[s].toff : -1;
        int ix[MT_MAXH + 2]; int depth = 0;
        int child = s; int p = v.R[s].parent; bool leafLevel = true;
        while (p >= 0) {
            const MtBlk& b = v.blk[p];
            int at = -1;
            for (int i = 0; i < b.n; i++) if (b.c[i] == child) at = i;
            ix[depth++] = at;
            child = p; p = b.parent; leafLevel = false;
        }
        (void)leafLevel;
        uint64_t path = 0;
        for (int k = depth - 1; k >= 0; k--) path = (path << 3) | (uint64_t)(ix[k] & 7);
        r[9] = depth; r[10] = (int32_t)(path & 0xFFFFFFFFull); r[11] = (int32_t)(path >> 32);
        rows.insert(rows.end(), r, r + 12);
    };
    walk_all(v, v.hdr.root, f);
}

}  // namespace mtsnap
