"use strict";
/*
 * The packing half of the Node host (no GPU addon: index.js and the ParallelPacker workers
 * both use it).  BatchBuilder restates Client.applyMsg's dispatch (packages/dds/merge-tree/
 * src/client.ts:790-841, MT/ below) into mt_op_batch columns: long client ids become
 * per-document indices, GROUP members share the message's seq, and property sets are
 * interned with JS semantics (Object.keys order, JSON.stringify text, falsiness for
 * "rewrite", matchProperties classes, MT/properties.ts:64-95).
 */
const OP_INSERT = 0, OP_REMOVE = 1, OP_ANNOTATE = 2, OP_NOOP = 3, OP_GROUP = 3, OP_UNSUPPORTED = 4;
const OP_CUT = 5, OP_COPY = 6, OP_PASTE = 7;          // register ops (include/mtgpu.h)
const F_END = 1, F_MARKER = 2, F_REWRITE = 4, F_SEG_PROPS = 8, F_COMBINE = 16, F_REL1 = 0x20, F_REL2 = 0x40,
    F_MARKER_ID = 0x80;
const MARKER_ID_KEY = "markerId";   // reservedMarkerIdKey, MT/mergeTree.ts:591
// property values other than interned ids, and value kinds (include/mtgpu.h MT_VAL_*, MT_VK_*)
const VAL_NULL = -1, VAL_NAN = -2, VAL_UNSUP = -3, VAL_CFRESH = -4, VAL_UNDEF = -5, VAL_THROW = -6, VAL_CONS_BASE = -16;
const F_CONSENSUS = 2, F_INCR_STRMIN = 8;   // on combining annotates (include/mtgpu.h)
const INCR_CHAIN_MAX = 64;                  // incr results of a held string precomputed per value
const VK_NUM = 1, VK_SEQM1 = 2;
const isNumberLike = (v) => typeof v === "number" || typeof v === "boolean";      // x + undefined is NaN
const seqMinus1 = (v) => v !== null && typeof v === "object" && !Array.isArray(v) && v.seq === -1;   // properties.ts:52
function arrayIndex(k) {
    // canonical array index (OrdinaryOwnPropertyKeys orders these first)
    if (!/^(0|[1-9][0-9]{0,9})$/.test(k)) return undefined;
    const v = Number(k);
    return v < 4294967295 ? v : undefined;
}

// matchProperties equivalence (MT/properties.ts:64-95): objects compare
// order-insensitively and recursively, primitives with ===.
function matchClassKey(v) {
    if (v !== null && typeof v === "object") {
        return "o{" + Object.keys(v).sort().map((k) => JSON.stringify(k) + ":" + matchClassKey(v[k])).join(",") + "}";
    }
    if (typeof v === "number") return "n" + String(v);
    if (typeof v === "boolean") return "b" + String(v);
    if (typeof v === "string") return "s" + JSON.stringify(v);
    return "z";
}

class PropTable {
    constructor() {
        this.keyIds = new Map(); this.keys = [];
        this.valueIds = new Map(); this.valueJson = []; this.valueFalsy = []; this.valueClass = []; this.valueKind = [];
        this.classIds = new Map();
        this.setIds = new Map(); this.sets = [];
        this.incrKeys = new Set(); this.nIncr = 0;
    }
    keyId(k) {
        let i = this.keyIds.get(k);
        if (i === undefined) { i = this.keys.length; this.keyIds.set(k, i); this.keys.push(k); }
        return i;
    }
    valueId(v) {
        if (v === null) return -1;                       // null deletes the key
        const txt = JSON.stringify(v);
        let i = this.valueIds.get(txt);
        if (i === undefined) {
            i = this.valueJson.length;
            this.valueIds.set(txt, i);
            this.valueJson.push(txt);
            this.valueFalsy.push(v ? 0 : 1);
            const ck = matchClassKey(v);
            let c = this.classIds.get(ck);
            if (c === undefined) { c = this.classIds.size; this.classIds.set(ck, c); }
            this.valueClass.push(c);
            this.valueKind.push((isNumberLike(v) ? VK_NUM : 0) | (seqMinus1(v) ? VK_SEQM1 : 0));
        }
        return i;
    }
    intern(props) {
        return this.internPairs(Object.keys(props).map((k) => [this.keyId(k), this.valueId(props[k])]));
    }
    /**
     * [combine set, flags] of a remote annotate with a combining op other than "rewrite"
     * (include/mtgpu.h): the op's keys, each valued with what combine(op, undefined, undefined,
     * seq) yields (properties.ts:24-62 via segmentPropertiesManager.ts:98-103).
     */
    internCombine(props, cop, seq) {
        const d = cop.defaultValue;
        let code, fl;
        if (cop.name === "incr") {                          // x + undefined: NaN, or String(x) + "undefined"
            const mv = cop.minValue;
            const strMin = !!mv && typeof mv === "object" || (typeof mv === "string" && mv.length > 0);
            if (d === undefined || d === null || isNumberLike(d)) code = VAL_NAN;     // NaN < minValue is false
            else {
                let r = d + undefined;                          // `_currentValue += newValue`
                if (strMin && r < mv) r = mv;                   // both strings: UTF-16 code-unit order
                code = this.valueId(r);
            }
            fl = F_COMBINE | (strMin ? F_INCR_STRMIN : 0);
            this.nIncr++;
            for (const k of Object.keys(props)) this.incrKeys.add(this.keyId(k));
        } else if (cop.name === "consensus") {              // {value: undefined, seq}; null.seq throws
            code = d === undefined ? VAL_CFRESH : (d === null ? VAL_THROW : this.valueId(seqMinus1(d) ? { ...d, seq } : d));
            fl = F_COMBINE | F_REWRITE | F_CONSENSUS;
        } else {                                            // no case in combine's switch
            code = d === undefined ? VAL_UNDEF : (d === null ? VAL_NULL : this.valueId(d));
            fl = F_COMBINE | F_REWRITE;
        }
        return [this.internPairs(Object.keys(props).map((k) => [this.keyId(k), code])), fl];
    }
    internPairs(pairs) {
        const sig = pairs.map((p) => p.join(":")).join(",");
        let i = this.setIds.get(sig);
        if (i === undefined) { i = this.sets.length; this.setIds.set(sig, i); this.sets.push(pairs); }
        return i;
    }
    /**
     * [valueIncr, incrObject] for mt_prop_table: what incr yields from each value held
     * (properties.ts:33-34, `v += undefined`): the id of that string for a string, array or
     * object that can be held under a key some incr op names (the values sets give those keys,
     * and the strings incr makes from them, INCR_CHAIN_MAX deep at most), VAL_UNSUP otherwise.
     */
    incrTable() {
        if (!this.nIncr) return [new Int32Array(Math.max(1, this.valueJson.length)).fill(VAL_UNSUP), VAL_UNSUP];
        const depthMax = Math.min(this.nIncr, INCR_CHAIN_MAX);
        const obj = this.valueId("[object Object]undefined");         // incr of a fresh consensus object
        const depth = new Map([[obj, 1]]);
        for (const s of this.sets) for (const [k, v] of s) if (this.incrKeys.has(k) && v >= 0 && !depth.has(v)) depth.set(v, 0);
        const succ = new Map();
        let frontier = [...depth.keys()];
        while (frontier.length) {
            const nxt = [];
            for (const v of frontier) {
                if (succ.has(v) || (this.valueKind[v] & VK_NUM) || depth.get(v) >= depthMax) continue;
                const w = this.valueId(JSON.parse(this.valueJson[v]) + undefined);
                succ.set(v, w);
                if (!depth.has(w)) { depth.set(w, depth.get(v) + 1); nxt.push(w); }
            }
            frontier = nxt;
        }
        const t = new Int32Array(Math.max(1, this.valueJson.length)).fill(VAL_UNSUP);
        for (const [v, w] of succ) t[v] = w;
        return [t, obj];
    }
    toNative() {
        const [valueIncr, incrObject] = this.incrTable();      // may intern strings: first
        const setOff = new Uint32Array(this.sets.length + 1);
        const key = [], value = [];
        this.sets.forEach((s, i) => { setOff[i + 1] = setOff[i] + s.length; for (const [k, v] of s) { key.push(k); value.push(v); } });
        return {
            setOff, key: Uint16Array.from(key.length ? key : [0]), value: Int32Array.from(value.length ? value : [0]),
            keyJson: this.keys.map((k) => JSON.stringify(k)),
            keyIndex: Uint32Array.from(this.keys.length ? this.keys.map((k) => { const a = arrayIndex(k); return a === undefined ? 0xFFFFFFFF : a; }) : [0]),
            valueJson: this.valueJson,
            valueFalsy: Uint8Array.from(this.valueFalsy.length ? this.valueFalsy : [0]),
            valueClass: Uint32Array.from(this.valueClass.length ? this.valueClass : [0]),
            valueKind: Uint8Array.from(this.valueKind.length ? this.valueKind : [0]),
            valueIncr, incrObject,
        };
    }
}

/** Per-document interning: long client ids (getOrAddShortClientId order, client.ts:658-682)
 * and marker ids -> the document's idToSegment table on the device (mergeTree.ts:1095). */
class ClientNames {
    constructor() { this.ids = new Map(); this.names = []; this.markerIds = new Map(); this.registerIds = new Map(); }
    /** The document's index of a register name (RegisterCollection key, with the author). */
    registerIndex(name) {
        if (!this.registerIds.has(name)) this.registerIds.set(name, this.registerIds.size);
        return this.registerIds.get(name);
    }
    index(longId) {
        let i = this.ids.get(longId);
        if (i === undefined) { i = this.names.length; this.ids.set(longId, i); this.names.push(longId); }
        return i;
    }
    /** A marker carrying this id joins the document; null for a non-string or reused id. */
    markerDefine(id) {
        if (typeof id !== "string" || this.markerIds.has(id)) return null;
        const i = this.markerIds.size;
        this.markerIds.set(id, i);
        return i;
    }
    /** getMarkerFromId: the table index, -1 when never mapped. */
    markerLookup(id) { return typeof id === "string" && this.markerIds.has(id) ? this.markerIds.get(id) : -1; }
}

// applyRemoteOp's GROUP recursion (client.ts:804-812), flattened; members share the seq
function mergeTreeMembers(contents) {
    const flat = (op) => (op && typeof op === "object") ? (op.type === OP_GROUP ? (op.ops || []).flatMap(flat) : [op]) : [];
    return flat(contents).filter((m) => m.type === OP_INSERT || m.type === OP_REMOVE || m.type === OP_ANNOTATE);
}

const COLS = [["type", Uint8Array], ["flags", Uint8Array], ["client", Uint16Array], ["seq", Int32Array],
    ["refSeq", Int32Array], ["msn", Int32Array], ["pos1", Int32Array], ["pos2", Int32Array],
    ["payloadOff", Uint32Array], ["payloadLen", Uint32Array], ["propId", Int32Array]];

/** A growable typed-array column (amortized doubling; no per-element JS objects).  shared: its
 * memory is a SharedArrayBuffer, so a worker that keeps one builder for many batches hands each
 * batch's columns to the main thread without copying, and allocates nothing per batch (new
 * ArrayBuffers count as external memory, and their growth makes V8 mark the whole heap: with
 * the documents' parsed messages held in the worker, that is most of a window's packing time). */
class Col {
    constructor(T, cap = 1024, shared = false) { this.T = T; this.shared = shared; this.a = this.alloc(cap); this.n = 0; }
    alloc(cap) { return this.shared ? new this.T(new SharedArrayBuffer(cap * this.T.BYTES_PER_ELEMENT)) : new this.T(cap); }
    grow(need) {
        let cap = this.a.length * 2;
        while (cap < need) cap *= 2;
        const b = this.alloc(cap); b.set(this.a.subarray(0, this.n)); this.a = b;
    }
    push(v) {
        if (this.n === this.a.length) this.grow(this.n + 1);
        this.a[this.n++] = v;
    }
    view() { return this.a.subarray(0, this.n); }
}

/** Packs ISequencedDocumentMessages (protocol.ts:126-166) into mt_op_batch runs, straight
 * into typed-array columns. */
class BatchBuilder {
    constructor(props, names, shared = false) {
        this.props = props; this.names = names;
        this.cols = {}; for (const [n, T] of COLS) this.cols[n] = new Col(T, 1024, shared);
        this.payload = new Col(Uint16Array, 4096, shared); this.docIds = []; this.offsets = [0]; this.rel = [];
    }
    /** Empty again, keeping the columns' memory (a worker's builder, batch after batch). */
    reset(props) {
        this.props = props;
        for (const k in this.cols) this.cols[k].n = 0;
        this.payload.n = 0; this.docIds = []; this.offsets = [0]; this.rel = [];
    }
    get nOps() { return this.cols.type.n; }
    /** op.pos{k}, or op.relativePos{k} as an index into rel (getValidOpRange, client.ts:506-523). */
    pos(op, k) {
        const v = op["pos" + k];
        if (v !== undefined) return [v, 0];
        const rp = op["relativePos" + k];
        if (!rp) return [undefined, 0];
        const idx = rp.id ? this.names.markerLookup(rp.id) : -1;
        this.rel.push([idx, rp.before ? 1 : 0, rp.offset !== undefined ? rp.offset : 0, 0]);
        return [this.rel.length - 1, k === 1 ? F_REL1 : F_REL2];
    }
    beginDoc(docId) { this.docIds.push(docId); this.offsets.push(this.offsets[this.offsets.length - 1]); }
    push(type, flags, client, seq, refSeq, msn, pos1, pos2, payloadOff, payloadLen, propId) {
        const c = this.cols;
        c.type.push(type); c.flags.push(flags); c.client.push(client); c.seq.push(seq); c.refSeq.push(refSeq);
        c.msn.push(msn); c.pos1.push(pos1 || 0); c.pos2.push(pos2 || 0); c.payloadOff.push(payloadOff);
        c.payloadLen.push(payloadLen); c.propId.push(propId);
        this.offsets[this.offsets.length - 1] += 1;
    }
    member(op, client, seq, ref, msn, last) {
        let fl = last ? F_END : 0;
        const bad = () => this.push(OP_UNSUPPORTED, fl, client, seq, ref, msn, 0, 0, 0, 0, -1);
        if (op.type === OP_INSERT) {
            const seg = op.seg;
            if (!seg && op.register) {
                // applyInsertOp's register branch (client.ts:425-444): a truthy range end copies
                // [pos1, pos2) into the register, otherwise the register is pasted at pos1
                const [pos1, rf] = this.pos(op, 1);
                if (pos1 === undefined || typeof op.register !== "string" || rf ||
                    (op.pos2 === undefined && op.relativePos2)) { bad(); return; }
                const copy = op.pos2 !== undefined && op.pos2 !== 0;
                this.push(copy ? OP_COPY : OP_PASTE, fl, client, seq, ref, msn, pos1, copy ? op.pos2 : 0,
                    this.names.registerIndex(op.register), 0, -1);
                return;
            }
            if (!seg) { this.push(OP_NOOP, fl, client, seq, ref, msn, 0, 0, 0, 0, -1); return; }   // `if (op.seg)` falsy
            const [pos1, rf] = this.pos(op, 1);
            if (pos1 === undefined) { bad(); return; }
            fl |= rf;
            let text = null, props, pos2 = 0;
            if (typeof seg === "string") text = seg;
            else if (seg.text !== undefined) { text = seg.text; props = seg.props; }
            else if (seg.marker !== undefined) { props = seg.props; fl |= F_MARKER; pos2 = seg.marker.refType || 0; }
            else throw new Error("Unrecognized IJSONSegment type");
            let pid = -1;
            if (props) {                                       // `if (props)` in TextSegment/Marker.make
                if (typeof props !== "object") throw new Error("segment props must be an object");
                pid = this.props.intern(props); fl |= F_SEG_PROPS;
            }
            let off = this.payload.n;
            if (text !== null) for (let i = 0; i < text.length; i++) this.payload.push(text.charCodeAt(i));
            if (text === null && pid >= 0 && props[MARKER_ID_KEY]) {           // Marker.getId
                const m = this.names.markerDefine(props[MARKER_ID_KEY]);
                if (m === null) { bad(); return; }
                fl |= F_MARKER_ID; off = m;
            }
            this.push(OP_INSERT, fl, client, seq, ref, msn, pos1, pos2, off, text !== null ? text.length : 0, pid);
        } else if (op.type === OP_REMOVE || op.type === OP_ANNOTATE) {
            const [pos1, f1] = this.pos(op, 1), [pos2, f2] = this.pos(op, 2);
            if (pos1 === undefined || pos2 === undefined) { bad(); return; }
            let pid = -1;
            if (op.type === OP_ANNOTATE) {
                // segmentPropertiesManager.ts:55-56: rewrite = op && op.name === "rewrite"; any other
                // truthy combiningOp combines (properties.ts:24-62)
                const cop = op.combiningOp, combine = !!cop && cop.name !== "rewrite";
                if (cop && !combine) fl |= F_REWRITE;
                if (op.props && typeof op.props === "object" && MARKER_ID_KEY in op.props) { bad(); return; }   // re-keyed marker ids
                if (combine) {
                    const [id, cfl] = this.props.internCombine(op.props, cop, seq);
                    pid = id; fl |= cfl;
                } else pid = this.props.intern(op.props);
            }
            if (op.type === OP_REMOVE && op.register) {     // cut: Client.copy, then markRangeRemoved (:347-350)
                if (typeof op.register !== "string") { bad(); return; }
                this.push(OP_CUT, fl | f1 | f2, client, seq, ref, msn, pos1, pos2, this.names.registerIndex(op.register), 0, -1);
                return;
            }
            this.push(op.type, fl | f1 | f2, client, seq, ref, msn, pos1, pos2, 0, 0, pid);
        } else {
            this.push(OP_NOOP, fl, client, seq, ref, msn, 0, 0, 0, 0, -1);
        }
    }
    /** One sequenced message (Client.applyMsg, client.ts:819-841); returns the batch op
     * index of each merge-tree member (GROUP order; [] for none). */
    addMessage(msg) {
        // getOrAddShortClientId keys a RedBlackTree with localeCompare (client.ts:73, :658)
        if (typeof msg.clientId !== "string") throw new Error("clientId must be a string on the batch path");
        const client = this.names.index(msg.clientId);
        const seq = msg.sequenceNumber, ref = msg.referenceSequenceNumber, msn = msg.minimumSequenceNumber;
        if ((msg.type === undefined ? "op" : msg.type) !== "op") {
            this.push(OP_NOOP, F_END, client, seq, ref, msn, 0, 0, 0, 0, -1);
            return [];
        }
        const c = msg.contents;
        // the common case without a GROUP: one member, no array building
        if (c && typeof c === "object" && c.type !== OP_GROUP) {
            if (c.type !== OP_INSERT && c.type !== OP_REMOVE && c.type !== OP_ANNOTATE) {
                this.push(OP_NOOP, F_END, client, seq, ref, msn, 0, 0, 0, 0, -1);
                return [];
            }
            const first = this.cols.type.n;
            this.member(c, client, seq, ref, msn, true);
            return [first];
        }
        const members = mergeTreeMembers(c);
        if (!members.length) { this.push(OP_NOOP, F_END, client, seq, ref, msn, 0, 0, 0, 0, -1); return []; }
        const first = this.cols.type.n;
        members.forEach((m, i) => this.member(m, client, seq, ref, msn, i === members.length - 1));
        return members.map((_, i) => first + i);
    }
    /** Room for n more ops in every column (one growth instead of a check per push). */
    reserve(n) {
        for (const k in this.cols) {
            const col = this.cols[k];
            if (col.n + n > col.a.length) col.grow(col.n + n);
        }
    }
    /**
     * addMessage for every message of an array (one document's ISequencedDocumentMessages as
     * SharedSegmentSequence.processCore receives them, already parsed), with the common shapes
     * packed inline: a non-GROUP "op" whose contents is an insert of a non-empty string at a
     * numeric pos1 or a remove of numeric [pos1, pos2), neither with a register.  Every other
     * message goes through addMessage.  The columns are the same as addMessage's for each.
     */
    addMessages(msgs) {
        const n = msgs.length;
        this.reserve(n);
        const cols = this.cols, names = this.names, pay = this.payload;
        let ty = cols.type.a, fl = cols.flags.a, cl = cols.client.a, sq = cols.seq.a, rf = cols.refSeq.a, ms = cols.msn.a,
            p1 = cols.pos1.a, p2 = cols.pos2.a, po = cols.payloadOff.a, pl = cols.payloadLen.a, pid = cols.propId.a;
        let o = cols.type.n, run = 0;
        const last = this.offsets.length - 1;
        for (let i = 0; i < n; i++) {
            const m = msgs[i];
            const ct = m.contents;
            let t = -1;
            if ((m.type === "op" || m.type === undefined) && typeof m.clientId === "string" && ct !== null &&
                typeof ct === "object" && ct.register === undefined && typeof ct.pos1 === "number") {
                if (ct.type === OP_INSERT && typeof ct.seg === "string" && ct.seg.length > 0) t = OP_INSERT;
                else if (ct.type === OP_REMOVE && typeof ct.pos2 === "number") t = OP_REMOVE;
            }
            if (t < 0) {                                 // the general path, then back to the columns
                for (const k in cols) cols[k].n = o;
                this.offsets[last] += run; run = 0;
                this.addMessage(m);
                this.reserve(n - i);
                o = cols.type.n;
                ty = cols.type.a; fl = cols.flags.a; cl = cols.client.a; sq = cols.seq.a; rf = cols.refSeq.a; ms = cols.msn.a;
                p1 = cols.pos1.a; p2 = cols.pos2.a; po = cols.payloadOff.a; pl = cols.payloadLen.a; pid = cols.propId.a;
                continue;
            }
            if (t === OP_INSERT) {
                const seg = ct.seg, L = seg.length;
                if (pay.n + L > pay.a.length) pay.grow(pay.n + L);
                const pa = pay.a, q = pay.n;
                for (let j = 0; j < L; j++) pa[q + j] = seg.charCodeAt(j);
                pay.n = q + L;
                po[o] = q; pl[o] = L; p2[o] = 0;
            } else {
                po[o] = 0; pl[o] = 0; p2[o] = ct.pos2 || 0;
            }
            ty[o] = t; fl[o] = F_END; p1[o] = ct.pos1 || 0; pid[o] = -1;
            cl[o] = names.index(m.clientId); sq[o] = m.sequenceNumber; rf[o] = m.referenceSequenceNumber;
            ms[o] = m.minimumSequenceNumber;
            o++; run++;
        }
        for (const k in cols) cols[k].n = o;
        this.offsets[last] += run;
    }
    build() {
        const b = { docIds: Uint32Array.from(this.docIds), opOffsets: Uint32Array.from(this.offsets),
            payload: this.payload.n ? this.payload.view() : new Uint16Array(1),
            rel: Int32Array.from(this.rel.flat()) };
        for (const [n] of COLS) b[n] = this.cols[n].view();
        return b;
    }
}


module.exports = { VAL_NULL, VAL_NAN, VAL_UNSUP, VAL_CFRESH, VAL_UNDEF, VAL_THROW, VAL_CONS_BASE, VK_NUM, VK_SEQM1,
    OP_INSERT, OP_REMOVE, OP_ANNOTATE, OP_NOOP, OP_GROUP, OP_UNSUPPORTED, OP_CUT, OP_COPY, OP_PASTE,
    F_END, F_MARKER, F_REWRITE, F_SEG_PROPS, F_COMBINE, F_REL1, F_REL2, F_MARKER_ID, MARKER_ID_KEY, arrayIndex,
    matchClassKey, PropTable, ClientNames, mergeTreeMembers, COLS, Col, BatchBuilder };
