"use strict";
/*
 * Parallel ingest for the Node host: ISequencedDocumentMessage streams (the JSON text a
 * summarizer receives per document) are parsed and packed into mt_op_batch columns by a
 * pool of worker_threads, one slice of documents per worker, and merged into one batch for
 * a single mt_apply_batch.  Each worker restates Client.applyMsg's dispatch with the same
 * BatchBuilder the main thread uses (index.js); the merge only re-bases the per-worker
 * indices: payload offsets of text inserts, relative-position indices and property-set
 * ids (each worker interns into its own PropTable, which the main thread's table absorbs).
 */
const path = require("path");
const { Worker } = require("worker_threads");

const F_MARKER = 2, F_SEG_PROPS = 8, F_REL1 = 0x20, F_REL2 = 0x40;
const OP_INSERT = 0;
const COLS = ["type", "flags", "client", "seq", "refSeq", "msn", "pos1", "pos2", "payloadOff", "payloadLen", "propId"];
const TYPES = { type: Uint8Array, flags: Uint8Array, client: Uint16Array, seq: Int32Array, refSeq: Int32Array,
    msn: Int32Array, pos1: Int32Array, pos2: Int32Array, payloadOff: Uint32Array, payloadLen: Uint32Array,
    propId: Int32Array };

class ParallelPacker {
    constructor(nWorkers) {
        this.workers = [];
        // heaps sized for documents held as parsed message objects (hundreds of MB a worker): the
        // default limits make V8 collect the old generation over and over while packing
        const resourceLimits = { maxOldGenerationSizeMb: 16384, maxYoungGenerationSizeMb: 512 };
        for (let i = 0; i < nWorkers; i++) this.workers.push(new Worker(path.join(__dirname, "pack_worker.js"), { resourceLimits }));
    }
    close() { return Promise.all(this.workers.map((w) => w.terminate())); }
    /**
     * docs: [{ id, json } | { id, file, bytes }] (the document's messages as JSON text, or
     * a file holding it that the worker reads itself); props: the
     * PropTable of the engine the batch goes to.  Resolves to { batch, names } with
     * names[i] the long client ids of docs[i] in short-id order.
     */
    /**
     * Hand each worker its share of documents (contiguous, equal counts) to hold as JSON text
     * in `windows` consecutive message windows: docs [{ id, bin }] (binary op columns,
     * pack_worker.js binToJson).  packHeld(ids, props, k) then packs window k of held documents
     * on the workers that hold them; each document's client-name table carries over from window
     * to window (resetNames() starts them again).
     */
    async prepare(docs, windows = 1, objects = false) {
        const W = this.workers.length;
        this.owner = new Map();
        const per = Math.ceil(docs.length / W);
        const jobs = [];
        for (let w = 0; w < W; w++) {
            const sl = docs.slice(w * per, (w + 1) * per);
            if (!sl.length) continue;
            for (const d of sl) this.owner.set(d.id, w);
            jobs.push(this.post(w, { prepare: sl, windows, objects }));
        }
        const r = await Promise.all(jobs);
        for (const m of r) if (m.error) throw new Error(m.error);
        return r.reduce((a, m) => a + m.bytes, 0);
    }
    async resetNames() { await Promise.all(this.workers.map((_, w) => this.post(w, { resetNames: true }))); }
    async packHeld(ids, props, win = 0) {
        const by = this.workers.map(() => []);
        for (const id of ids) by[this.owner.get(id)].push({ id, held: true, win });
        const parts = await Promise.all(by.map((l, w) => l.length ? this.post(w, { docs: l }) : null).filter((x) => x));
        const t0 = process.hrtime.bigint();
        const out = merge(parts, props);
        this.lastMergeMs = Number(process.hrtime.bigint() - t0) / 1e6;
        return out;
    }
    /**
     * packHeld without the merge: { parts, propMaps, names } for Engine.applyParts
     * (mt_apply_batch_parts re-bases and concatenates the parts on the library's host threads).
     * Each worker's property sets join `props`; propMaps[p] maps part p's set ids to the table's
     * (null when the part interned none).
     */
    async packHeldParts(ids, props, win = 0) {
        const by = this.workers.map(() => []);
        for (const id of ids) by[this.owner.get(id)].push({ id, held: true, win });
        const parts = await Promise.all(by.map((l, w) => l.length ? this.post(w, { docs: l }) : null).filter((x) => x));
        const names = [], propMaps = [];
        for (const p of parts) {
            if (p.error) throw new Error(p.error);
            propMaps.push(p.props.sets.length ? absorb(p.props, props) : null);
            for (const nm of p.names) names.push(nm);
        }
        return { parts: parts.map((p) => p.batch), propMaps, names };
    }
    post(w, msg) {
        const wk = this.workers[w];
        return new Promise((resolve, reject) => {
            const onMsg = (m) => { wk.off("error", onErr); resolve(m); };
            const onErr = (e) => { wk.off("message", onMsg); reject(e); };
            wk.once("message", onMsg);
            wk.once("error", onErr);
            wk.postMessage(msg);
        });
    }
    async pack(docs, props) {
        const W = this.workers.length;
        // contiguous slices balanced by text size (a proxy for messages)
        const size = (d) => (d.json !== undefined ? d.json.length : d.bytes || 1);
        const total = docs.reduce((a, d) => a + size(d), 0);
        const slices = [];
        let cur = [], acc = 0, k = 0;
        for (const d of docs) {
            cur.push(d); acc += size(d);
            if (acc >= (total * (k + 1)) / W && slices.length < W - 1) { slices.push(cur); cur = []; k++; }
        }
        slices.push(cur);
        const parts = await Promise.all(slices.map((sl, i) => new Promise((resolve, reject) => {
            const w = this.workers[i];
            const onMsg = (m) => { w.off("error", onErr); resolve(m); };
            const onErr = (e) => { w.off("message", onMsg); reject(e); };
            w.once("message", onMsg);
            w.once("error", onErr);
            w.postMessage({ docs: sl });
        })));
        const t0 = process.hrtime.bigint();
        const out = merge(parts, props);
        this.lastMergeMs = Number(process.hrtime.bigint() - t0) / 1e6;
        return out;
    }
}

// A worker's interned property sets as set ids of the engine's table: keys and values re-interned,
// the non-value codes of combine sets (MT_VAL_*, negative) kept as they are.
function absorb(wp, props) {
    // the keys incr ops name, and their count (PropTable.incrTable's inputs)
    for (const k of wp.incrKeys || []) props.incrKeys.add(props.keyId(wp.keys[k]));
    props.nIncr += wp.nIncr || 0;
    return Int32Array.from(wp.sets.map((pairs) => props.internPairs(pairs.map(([k, v]) =>
        [props.keyId(wp.keys[k]), v < 0 ? v : props.valueId(JSON.parse(wp.valueJson[v]))]))));
}

function merge(parts, props) {
    let nOps = 0, nPay = 0, nRel = 0, nRuns = 0;
    for (const p of parts) {
        if (p.error) throw new Error(p.error);
        nOps += p.batch.type.length; nPay += p.nPayload; nRel += p.batch.rel.length / 4; nRuns += p.batch.docIds.length;
    }
    const out = {};
    for (const c of COLS) out[c] = new TYPES[c](nOps);
    out.payload = new Uint16Array(Math.max(1, nPay));
    out.rel = new Int32Array(4 * nRel);
    out.docIds = new Uint32Array(nRuns);
    out.opOffsets = new Uint32Array(nRuns + 1);
    const names = [];
    let o = 0, pay = 0, rel = 0, run = 0;
    for (const p of parts) {
        const b = p.batch, n = b.type.length;
        for (const c of COLS) out[c].set(b[c], o);
        out.payload.set(b.payload.subarray(0, p.nPayload), pay);
        out.rel.set(b.rel, 4 * rel);
        out.docIds.set(b.docIds, run);
        for (let r = 0; r < b.docIds.length; r++) out.opOffsets[run + r + 1] = o + b.opOffsets[r + 1];
        // the worker's property sets join the engine's table; its indices are re-based
        const map = absorb(p.props, props);
        const ty = out.type, fl = out.flags, pid = out.propId, poff = out.payloadOff, p1 = out.pos1, p2 = out.pos2;
        for (let i = o; i < o + n; i++) {
            if (pid[i] >= 0) pid[i] = map[pid[i]];
            if (ty[i] === OP_INSERT && !(fl[i] & F_MARKER)) poff[i] += pay;
            if (fl[i] & F_REL1) p1[i] += rel;
            if (fl[i] & F_REL2) p2[i] += rel;
        }
        for (const nm of p.names) names.push(nm);
        o += n; pay += p.nPayload; rel += b.rel.length / 4; run += b.docIds.length;
    }
    return { batch: out, names };
}

module.exports = { ParallelPacker, merge, absorb };
