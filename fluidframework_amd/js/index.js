"use strict";
/*
 * Node host of the MI355X merge-tree engine: the TypeScript/Node side of the
 * drop-in boundary (SURVEY.md §8(b)).
 *
 * It mirrors the reference merge-tree `Client` (packages/dds/merge-tree/src/
 * client.ts, MT/ below) for the passive-observer replay path:
 *   MergeTreeClient.applyMsg(msg)            Client.applyMsg          MT/client.ts:819
 *   MergeTreeClient.updateSeqNumbers(m, s)   Client.updateSeqNumbers  MT/client.ts:843
 *   MergeTreeClient.getLength()              Client.getLength         MT/client.ts:1071
 *   MergeTreeClient.getText()                createTextHelper().getText  MT/client.ts:917
 *   MergeTreeClient.snapshot(catchUpMsgs)    Client.snapshot (SnapshotV1 / SnapshotLegacy) MT/client.ts:923
 *   MergeTreeClient.startOrUpdateCollaboration  MT/client.ts:1073
 * Messages are queued per document and applied in device batches: reads flush
 * every queued document of the group in one mt_apply_batch.  Protocol violations
 * the reference reports by throwing (assert, common-utils assert.ts:12-16) are
 * thrown here as Errors when the document's status is read.
 *
 * Packing restates Client.applyMsg's dispatch (client.ts:790-841): long client
 * ids become per-document indices, GROUP members share the message's seq, and
 * property sets are interned with JS semantics (Object.keys order, JSON.stringify
 * text, falsiness for "rewrite", matchProperties classes, MT/properties.ts:64-95).
 */
const path = require("path");

// MTGPU_NAPI: an alternate build of this addon (the tests' host-emulation build)
const addon = require(process.env.MTGPU_NAPI || path.join(__dirname, "mtgpu.node"));

const { VAL_NAN, VAL_UNDEF, VAL_CONS_BASE, OP_INSERT, OP_REMOVE, OP_ANNOTATE, OP_NOOP, OP_GROUP, OP_UNSUPPORTED, OP_CUT, OP_COPY, OP_PASTE,
    F_END, F_MARKER, F_REWRITE, F_SEG_PROPS, F_COMBINE, F_REL1, F_REL2, F_MARKER_ID, MARKER_ID_KEY, arrayIndex,
    matchClassKey, PropTable, ClientNames, mergeTreeMembers, BatchBuilder } = require("./builder.js");
const STATUS = {
    0x01: "ASSERT_SEQ", 0x02: "ASSERT_MSN", 0x04: "INSERT_FAILED", 0x08: "UNSUPPORTED",
    0x10: "OOM_ROWS", 0x20: "OOM_BLOCKS", 0x40: "OOM_TEXT", 0x80: "OOM_PROPS",
    0x100: "OOM_HEAP", 0x200: "OOM_WINDOW", 0x400: "PROPS_TOO_MANY", 0x800: "BAD_OP", 0x1000: "REFSEQ_BELOW_MSN",
    0x2000: "OOM_OVERLAP", 0x4000: "THROWS",
};
function statusNames(st) {
    return Object.keys(STATUS).filter((b) => st & Number(b)).map((b) => STATUS[b]);
}

// ---- snapshot load: the JSON half of SnapshotLoader (MT/snapshotLoader.ts) ----
const LS_SEQ = 1, LS_CLIENT = 2, LS_REMOVED = 4, LS_MARKER = 8;

/** toLatestVersion (MT/snapshotChunks.ts:137-180) of one parsed chunk. */
function latestChunk(chunk, header) {
    if (chunk.version === "1") {
        return { segments: chunk.segments, segmentCount: chunk.segmentCount,
            headerMetadata: header ? chunk.headerMetadata : undefined };
    }
    if (chunk.version === undefined) {
        let md;
        if (header) {
            md = chunk.headerMetadata;
            if (md === undefined) {
                const ids = [{ id: "header" }];
                if (chunk.chunkLengthChars < chunk.totalLengthChars) ids.push({ id: "body" });
                md = { orderedChunkMetadata: ids, minSequenceNumber: chunk.chunkMinSequenceNumber,
                    sequenceNumber: chunk.chunkSequenceNumber, totalLength: chunk.totalLengthChars,
                    totalSegmentCount: chunk.totalSegmentCount };
            }
        }
        return { segments: chunk.segmentTexts, segmentCount: chunk.chunkSegmentCount, headerMetadata: md };
    }
    throw new Error(`Unsupported chunk version: ${chunk.version}`);
}

/**
 * Parses a snapshot's blobs ({path: contents}) as SnapshotLoader.initialize does:
 * header metadata, header segments, body chunks in orderedChunkMetadata order, and
 * the catch-up ops blob (legacy format) if present (snapshotLoader.ts:39-92).
 */
function parseSnapshot(blobs) {
    const head = latestChunk(JSON.parse(blobs.header), true);
    const md = head.headerMetadata;
    if (md === undefined) throw new Error("header metadata not available");
    const out = { header: head.segments || [], body: [], seq: md.sequenceNumber,
        minSeq: md.minSequenceNumber !== undefined ? md.minSequenceNumber : md.sequenceNumber, catchupOps: [] };
    const ids = md.orderedChunkMetadata.map((c) => c.id);
    if (head.segmentCount !== md.totalSegmentCount) {
        for (const id of ids.slice(1)) {
            if (blobs[id] === undefined) throw new Error(`missing chunk ${id}`);
            for (const sp of latestChunk(JSON.parse(blobs[id]), false).segments || []) out.body.push(sp);
        }
    }
    const rest = Object.keys(blobs).filter((k) => !ids.includes(k));
    if (rest.length === 1) out.catchupOps = JSON.parse(blobs[rest[0]]);
    else if (rest.length > 1) throw new Error("Unexpected blobs in snapshot");
    return out;
}

/** Packs parsed snapshots into an mt_load_batch (32-byte mt_load_seg records). */
class LoadBuilder {
    constructor(props) {
        this.props = props; this.docIds = []; this.offsets = [0]; this.nhdr = []; this.minSeq = []; this.seq = [];
        this.recs = []; this.payload = [];
    }
    // SnapshotLoader.specToSegment (snapshotLoader.ts:93-124) over segmentFromSpec
    // (sequenceFactory.ts:31-37); null where the reference would fail.
    record(spec, names, header) {
        const merge = spec !== null && typeof spec === "object" && "json" in spec;
        const js = merge ? spec.json : spec;
        let flags = 0, text = null, refType = 0, props;
        if (typeof js === "string") text = js;
        else if (js !== null && typeof js === "object" && "text" in js) {
            if (typeof js.text !== "string") return null;
            text = js.text; props = js.props;
        } else if (js !== null && typeof js === "object" && "marker" in js) {
            refType = js.marker && js.marker.refType;
            if (!Number.isInteger(refType) || refType < 0) return null;
            flags |= LS_MARKER; props = js.props;
        } else return null;
        let pid = -1;
        if (props) {
            if (typeof props !== "object") return null;
            pid = this.props.intern(props);
        }
        let mid = 0;
        // mapped: body markers (insertSegments), header markers not removed (addNodeReferences)
        const mapped = !(merge && (spec.removedSeq !== undefined || spec.removedClient !== undefined)) || !header;
        if ((flags & LS_MARKER) && props && props[MARKER_ID_KEY] && mapped) {          // Marker.getId
            const m = names.markerDefine(props[MARKER_ID_KEY]);
            if (m === null) return null;
            mid = m + 1;
        }
        const r = { flags, client: 0, seq: 0, rseq: 0, rclient: 0, pid, poff: 0, plen: refType, mid };
        if (text !== null) {
            r.poff = this.payload.length; r.plen = text.length;
            for (let i = 0; i < text.length; i++) this.payload.push(text.charCodeAt(i));
        }
        if (merge) {
            if (spec.client !== undefined) { if (typeof spec.client !== "string") return null; r.flags |= LS_CLIENT; r.client = names.index(spec.client); }
            if (spec.seq !== undefined) { if (!Number.isInteger(spec.seq)) return null; r.flags |= LS_SEQ; r.seq = spec.seq; }
            if (spec.removedSeq !== undefined || spec.removedClient !== undefined) {
                if (!Number.isInteger(spec.removedSeq) || typeof spec.removedClient !== "string") return null;
                r.flags |= LS_REMOVED; r.rseq = spec.removedSeq; r.rclient = names.index(spec.removedClient);
            }
        }
        return r;
    }
    /** Adds one document; false if rejected (it then loads as UNSUPPORTED). */
    add(docId, snap, names) {
        const p0 = this.payload.length, recs = [];
        let ok = Number.isInteger(snap.seq) && Number.isInteger(snap.minSeq);
        const nh = snap.header.length;
        for (const [i, spec] of (ok ? snap.header.concat(snap.body) : []).entries()) {
            const r = this.record(spec, names, i < nh);
            if (r === null) { ok = false; break; }
            recs.push(r);
        }
        if (!ok) { this.payload.length = p0; recs.length = 0; }
        for (const r of recs) this.recs.push(r);
        this.docIds.push(docId); this.offsets.push(this.recs.length);
        this.nhdr.push(ok ? snap.header.length : 0);
        this.minSeq.push(ok ? snap.minSeq : -1); this.seq.push(ok ? snap.seq : 0);
        return ok;
    }
    build() {
        const buf = new ArrayBuffer(32 * Math.max(1, this.recs.length)), dv = new DataView(buf);
        this.recs.forEach((r, i) => {
            const o = 32 * i;
            dv.setUint8(o, r.flags); dv.setUint16(o + 2, r.client, true); dv.setInt32(o + 4, r.seq, true);
            dv.setInt32(o + 8, r.rseq, true); dv.setUint16(o + 12, r.rclient, true); dv.setInt16(o + 14, r.pid, true);
            dv.setUint32(o + 16, r.poff, true); dv.setUint32(o + 20, r.plen, true); dv.setUint32(o + 24, r.mid, true);
        });
        return { docIds: Uint32Array.from(this.docIds), segOffsets: Uint32Array.from(this.offsets),
            headerSegments: Uint32Array.from(this.nhdr), minSeq: Int32Array.from(this.minSeq),
            seq: Int32Array.from(this.seq), segs: new Uint8Array(buf),
            payload: Uint16Array.from(this.payload.length ? this.payload : [0]) };
    }
}

const DEFAULT_LIMITS = { rowsPerDoc: 8192, windowPerDoc: 4096, propsetsPerDoc: 8192, textPerDoc: 1 << 16, markersPerDoc: 4096 };

/** A stored property value id (mt_doc_pset) as a JS value (include/mtgpu.h MT_VAL_*). */
function decodeValue(v, valueJson) {
    if (v >= 0) return JSON.parse(valueJson[v]);
    if (v === VAL_NAN) return NaN;
    if (v === VAL_UNDEF) return undefined;
    if (v <= VAL_CONS_BASE) return { value: undefined, seq: VAL_CONS_BASE - v };
    throw new Error(`not a stored property value: ${v}`);
}

/**
 * options.mergeTreeSnapshotChunkSize as setDocSnapshotChunk takes it: null for the default
 * (`?? 10000`, snapshotV1.ts:55, snapshotlegacy.ts:71), else the number the reference's
 * `length < chunkSize` compares against (ToNumber: "300" is 300, [100] is 100, true is 1).
 * A value no length is below (0, negative, NaN) is passed on: the legacy header chunk is then
 * empty, and SnapshotV1 of a non-empty document fails at snapshot time, where the reference's
 * chunk loop never ends.
 */
function snapshotChunkOption(options) {
    const v = options ? options.mergeTreeSnapshotChunkSize : undefined;
    if (v === undefined || v === null) return null;
    return Number(v);
}

/** One engine context (one GPU) and the documents it holds. */
class Engine {
    constructor(maxDocs, limits = {}, device = 0) {
        this.maxDocs = maxDocs;
        this.h = addon.create(device, { ...DEFAULT_LIMITS, ...limits, maxDocs });
        this.props = new PropTable();
        this.uploadedSets = -1;
    }
    close() { if (this.h) { addon.destroy(this.h); this.h = null; } }
    openDocs(first, n) { addon.docsOpen(this.h, first, n); }
    setClientNames(jsonLiterals) { addon.setClientNames(this.h, jsonLiterals); }
    apply(batch) {
        if (this.uploadedSets !== this.props.sets.length) {
            addon.setProps(this.h, this.props.toNative());
            this.uploadedSets = this.props.sets.length;
        }
        addon.applyBatch(this.h, batch);
    }
    /** Several packed parts applied as one batch (mt_apply_batch_parts; ParallelPacker.packHeldParts). */
    applyParts(parts, propMaps) {
        this.uploadProps();
        addon.applyBatchParts(this.h, parts, propMaps);
    }
    uploadProps() {
        if (this.uploadedSets !== this.props.sets.length) {
            addon.setProps(this.h, this.props.toNative());
            this.uploadedSets = this.props.sets.length;
        }
    }
    loadSnapshot(batch) { this.uploadProps(); addon.loadSnapshot(this.h, batch); }
    sync() { addon.sync(this.h); }
    syncAsync() { return addon.syncAsync(this.h); }
    status(docs) { return addon.docStatus(this.h, Uint32Array.from(docs)); }
    getLength(docs, refSeq, client) { return addon.getLength(this.h, Uint32Array.from(docs), Int32Array.from(refSeq), Int32Array.from(client)); }
    /**
     * mt_get_containing_segment: per query {found, offset, obsPos, len, seq, client, removedSeq,
     * removedClient, propSet, markerRefType, depth, pathLo, pathHi, row, resolved, json}
     * (refSeq < 0: the local view; resolved === -2**31: undefined).
     */
    containingSegment(docs, pos, refSeq, client) {
        const { info, json } = addon.getContainingSegment(this.h, Uint32Array.from(docs), Int32Array.from(pos),
            Int32Array.from(refSeq), Int32Array.from(client));
        const F = ["found", "offset", "obsPos", "len", "seq", "client", "removedSeq", "removedClient", "propSet",
            "markerRefType", "depth", "pathLo", "pathHi", "row", "resolved"];
        return json.map((j, i) => {
            const o = { json: j };
            F.forEach((f, k) => { o[f] = info[16 * i + k]; });
            return o;
        });
    }
    updateSeq(docs, msn, seq) { addon.updateSeq(this.h, Uint32Array.from(docs), Int32Array.from(msn), Int32Array.from(seq)); }
    snapshot(docs, msn, seq, legacy = false) {
        return (legacy ? addon.snapshotLegacy : addon.snapshotV1)(this.h, Uint32Array.from(docs), Int32Array.from(msn),
            Int32Array.from(seq));
    }
    getText(docs) { return addon.getText(this.h, Uint32Array.from(docs)); }
    /** Record the delta / maintenance callbacks of later batches (mt_delta_capture; 0: off). */
    deltaCapture(capacity) { addon.deltaCapture(this.h, capacity); }
    /** The last batch's records: Int32Array, 8 per record (op, kind, pos, len, seg, a, b, pad). */
    deltaRecords() { return addon.deltaRecords(this.h); }
    /** The last batch's pasted text (mt_delta_text): INSERT records with b === 0 index it. */
    deltaText() { return addon.deltaText(this.h); }
    /** A document's device property set as a plain object (undefined for -1); NaN, undefined and
     * fresh consensus objects ({value: undefined, seq}, properties.ts:43-47) as the reference holds them. */
    psetObject(doc, id) {
        if (id < 0) return undefined;
        const { keys, values } = addon.docPset(this.h, doc, id);
        const o = {};
        keys.forEach((k, i) => { o[this.props.keys[k]] = decodeValue(values[i], this.props.valueJson); });
        return o;
    }
    /** options.mergeTreeSnapshotChunkSize of documents (snapshotV1.ts:55; 0: the default). */
    setSnapshotChunk(docs, sizes) { addon.setDocSnapshotChunk(this.h, Uint32Array.from(docs), Float64Array.from(sizes)); }
    /** mt_reserve_staging: pin the snapshot / text staging buffers once (0: default budget). */
    reserveStaging(bytes = 0) { addon.reserveStaging(this.h, bytes); }
}

/**
 * Drop-in subset of merge-tree `Client` for a passive observer.  All clients of
 * a group share one engine; every read flushes the group's queued messages in
 * one device batch, so thousands of documents replay together.
 */
class MergeTreeClient {
    constructor(group, docId, options) {
        this.group = group; this.docId = docId;
        this.options = options;                     // Client options (client.ts:82-84)
        this.pending = []; this.names = new ClientNames();
        this.currentSeq = 0; this.minSeq = 0; this.longClientId = undefined;
        this.deltaListener = null;                  // SequenceChannel's sequenceDelta subscription
    }
    startOrUpdateCollaboration(longClientId, minSeq = 0, currentSeq = 0) {
        this.longClientId = longClientId;
    }
    applyMsg(msg) {
        this.pending.push(msg);
        this.currentSeq = msg.sequenceNumber;
        this.minSeq = msg.minimumSequenceNumber;
    }
    getCurrentSeq() { return this.currentSeq; }
    /**
     * Client.load (client.ts:958-965) with the reference's signature: reads the snapshot
     * through an IChannelStorageService (readBlob / list, as SnapshotLoader.initialize
     * and loadBodyAndCatchupOps do, snapshotLoader.ts:39-84) and resolves to
     * { catchupOpsP }, the catch-up messages for the caller to apply.
     */
    async load(runtime, storage, serializer) {
        const text = (b) => {
            if (typeof b === "string") return b;
            if (b instanceof ArrayBuffer) return Buffer.from(b).toString("utf8");
            return Buffer.from(b.buffer, b.byteOffset, b.byteLength).toString("utf8");   // bufferToString(b, "utf8")
        };
        const blobs = { header: text(await storage.readBlob("header")) };
        for (const p of await storage.list("")) {
            if (blobs[p] === undefined) blobs[p] = text(await storage.readBlob(p));
        }
        const id = runtime && runtime.clientId !== undefined ? runtime.clientId : "snapshot";
        const { catchupOps } = this.loadBlobs(blobs, id);
        return { catchupOpsP: Promise.resolve(catchupOps) };
    }
    /**
     * SnapshotLoader over already-read blobs: `blobs` maps blob paths (header, body_0.. /
     * body, catch-up ops) to contents.  Returns { catchupOps } for the caller to apply.
     */
    loadBlobs(blobs, longClientId = "snapshot") {
        this.group.flush();
        const snap = parseSnapshot(blobs);
        const lb = new LoadBuilder(this.group.engine.props);
        lb.add(this.docId, snap, this.names);
        this.group.version++;
        addon.setDocClientNames(this.group.engine.h, this.docId, this.names.names.map((n) => JSON.stringify(n)));
        this.namesUploaded = this.names.names.length;
        this.group.engine.loadSnapshot(lb.build());
        this.group.engine.sync();
        this.checkStatus();
        this.longClientId = longClientId;
        this.minSeq = snap.minSeq; this.currentSeq = snap.seq;
        return { catchupOps: snap.catchupOps };
    }
    checkStatus() {
        const st = this.group.engine.status([this.docId])[0];
        // MT_DS_THROWS: where the reference's applyMsg throws (consensus on a null default reads
        // null.seq, properties.ts:51-52), the same TypeError
        if (st & 0x4000) throw new TypeError(`document ${this.docId}: Cannot read property 'seq' of null`);
        if (st) throw new Error(`document ${this.docId}: ${statusNames(st).join(", ")}`);
    }
    updateSeqNumbers(min, seq) {
        this.group.flush();
        this.group.version++;
        this.group.engine.updateSeq([this.docId], [min], [seq]);
        this.minSeq = min; this.currentSeq = seq;
        this.checkStatus();
    }
    getLength() {
        this.group.flush();
        this.checkStatus();
        return this.group.engine.getLength([this.docId], [0x7FFFFFFF], [-1])[0];
    }
    getText() {
        this.group.flush();
        this.checkStatus();
        return this.group.engine.getText([this.docId])[0];
    }
    // Short client ids (client.ts:658-670): the local client 0, remote clients in first-seen order.
    getOrAddShortClientId(longClientId) {
        if (this.longClientId !== undefined && longClientId === this.longClientId) return 0;
        return this.names.index(longClientId) + 1;
    }
    getShortClientId(longClientId) {
        if (this.longClientId !== undefined && longClientId === this.longClientId) return 0;
        const i = this.names.ids.get(longClientId);
        if (i === undefined) throw new Error(`unknown client ${longClientId}`);
        return i + 1;
    }
    getLongClientId(shortClientId) { return shortClientId === 0 ? this.longClientId : this.names.names[shortClientId - 1]; }
    query(pos, refSeq, shortId) {
        this.group.flush();
        this.checkStatus();
        const local = shortId === undefined || shortId === 0;
        return this.group.engine.containingSegment([this.docId], [pos], [local ? -1 : refSeq], [local ? -1 : shortId - 1])[0];
    }
    /**
     * Client.getContainingSegment (client.ts:1040-1043; MergeTree.getContainingSegment,
     * mergeTree.ts:1616-1627) in the local view: { segment, offset }.  The segment is a copy
     * (ISegment fields and toJSONObject) taken now, valid for getPosition until the document
     * next changes.
     */
    getContainingSegment(pos) {
        const q = this.query(pos, 0, undefined);
        if (!q.found) return { segment: undefined, offset: undefined };
        const j = JSON.parse(q.json);
        const shortOf = (i) => (i < 0 ? -2 : i + 1);                // NonCollabClient = -2
        const seg = {
            cachedLength: q.len, seq: q.seq, clientId: shortOf(q.client),
            removedSeq: q.removedSeq === -(2 ** 31) ? undefined : q.removedSeq,
            removedClientId: q.removedSeq === -(2 ** 31) ? undefined : shortOf(q.removedClient),
            properties: q.propSet >= 0 ? this.group.engine.psetObject(this.docId, q.propSet) : undefined,
            toJSONObject: () => j, _obsPos: q.obsPos, _version: this.group.version,
        };
        if (typeof j === "string") seg.text = j;
        else if (j.marker) seg.refType = j.marker.refType;
        else seg.text = j.text;
        return { segment: seg, offset: q.offset };
    }
    /** Client.getPosition (client.ts:306-311) of a segment copy from getContainingSegment. */
    getPosition(segment) {
        if (segment === undefined) return -1;
        if (segment._version !== this.group.version || this.pending.length) {
            throw new Error("segment copy is stale: the document changed since getContainingSegment");
        }
        return segment._obsPos;
    }
    /** MergeTree.resolveRemoteClientPosition (mergeTree.ts:2125-2145); undefined where the reference's is. */
    resolveRemoteClientPosition(remoteClientPosition, remoteClientRefSeq, remoteClientId) {
        const q = this.query(remoteClientPosition, remoteClientRefSeq, remoteClientId);
        return q.resolved === -(2 ** 31) ? undefined : q.resolved;
    }
    /**
     * Client.snapshot (client.ts:923-956) with the reference's signature: the delta
     * manager's MSN and last seq move the window (updateSeqNumbers), then the tree.
     */
    snapshot(runtime, handle, serializer, catchUpMsgs) {
        const dm = runtime.deltaManager;
        this.updateSeqNumbers(dm.minimumSequenceNumber, dm.lastSequenceNumber);
        return this.snapshotTree(catchUpMsgs, serializer, handle);
    }
    /**
     * The tree at the client's current window.  With options.newMergeTreeSnapshotFormat
     * === true: SnapshotV1 (snapshotV1.ts:98-163), header, body_0, ...; otherwise
     * SnapshotLegacy (snapshotlegacy.ts:104-175): header, body, then catchUpMsgs as
     * the catch-up blob (options.catchUpBlobName ?? "catchupOps", serializer.stringify)
     * when non-empty.
     */
    snapshotTree(catchUpMsgs, serializer, handle) {
        this.group.flush();
        this.checkStatus();
        const opts = this.options || {};
        const v1 = opts.newMergeTreeSnapshotFormat === true;
        if (v1 && catchUpMsgs !== undefined && catchUpMsgs.length !== 0) {
            throw new Error("New format should not emit catchup ops");      // client.ts:945-947
        }
        const { blobs } = this.group.engine.snapshot([this.docId], [this.minSeq], [this.currentSeq], !v1)[0];
        const entry = (path, contents) => ({ mode: "100644", path, type: "Blob", value: { contents, encoding: "utf-8" } });
        const entries = blobs.map((contents, i) => entry(i === 0 ? "header" : (v1 ? `body_${i - 1}` : "body"), contents));
        if (!v1 && catchUpMsgs !== undefined && catchUpMsgs.length > 0) {
            const name = opts.catchUpBlobName !== undefined && opts.catchUpBlobName !== null ? opts.catchUpBlobName : "catchupOps";
            entries.push(entry(name, serializer ? serializer.stringify(catchUpMsgs, handle) : JSON.stringify(catchUpMsgs)));
        }
        return { entries };
    }
}

/** Many documents on one engine: `newClient()` per document, `flush()` batches. */
class ClientGroup {
    constructor(engine) { this.engine = engine; this.clients = []; this.version = 0; }
    newClient(options) {
        const d = this.clients.length;
        if (d >= this.engine.maxDocs) throw new Error("engine document capacity exhausted");
        const cs = snapshotChunkOption(options);
        this.engine.openDocs(d, 1);
        if (cs !== null) this.engine.setSnapshotChunk([d], [cs]);
        const c = new MergeTreeClient(this, d, options);
        this.clients.push(c);
        return c;
    }
    flush() {
        const busy = this.clients.filter((c) => c.pending.length);
        if (!busy.length) return;
        const bb = new BatchBuilder(this.engine.props, null);
        const listen = [];
        for (const c of busy) {
            bb.names = c.names;
            bb.beginDoc(c.docId);
            const entries = c.pending.map((m) => [m, bb.addMessage(m)]);
            c.pending = [];
            if (c.deltaListener) listen.push([c, entries]);
            if (c.namesUploaded !== c.names.names.length) {     // snapshot "client" fields use long ids
                addon.setDocClientNames(this.engine.h, c.docId, c.names.names.map((n) => JSON.stringify(n)));
                c.namesUploaded = c.names.names.length;
            }
        }
        const batch = bb.build();
        this.version++;                                      // segment copies taken before are stale
        // Capture only around batches with a listener; the capacity is one launch's buffer
        // (a batch that emits more resumes in further launches, mt_delta_capture).
        if (listen.length) this.engine.deltaCapture(Math.max(1 << 16, 512 * listen.length + 16 * batch.type.length));
        try {
            this.engine.apply(batch);
            this.engine.sync();
            if (listen.length) this.deliver(listen);
        } finally {
            if (listen.length) this.engine.deltaCapture(0);
        }
    }
    /** Each listening client's messages with their sequenceDelta events: per op member, the
     * INSERT / REMOVE / ANNOTATE records as ranges with their property maps. */
    deliver(listen) {
        const r = this.engine.deltaRecords();
        const text = this.engine.deltaText();
        const byOp = new Map();
        for (let i = 0; i < r.length; i += 8) {
            if (r[i + 1] < 0 || r[i + 1] > 2) continue;
            if (!byOp.has(r[i])) byOp.set(r[i], []);
            byOp.get(r[i]).push(i);
        }
        for (const [c, entries] of listen) {
            c.checkStatus();
            const cache = new Map();
            const pset = (id) => {
                if (!cache.has(id)) cache.set(id, this.engine.psetObject(c.docId, id));
                return cache.get(id);
            };
            const eventsOf = (op) => (byOp.get(op) || []).map((i) => {
                const kind = r[i + 1], a = r[i + 5], b = r[i + 6], pad = r[i + 7], len = r[i + 3];
                // a register paste's clone: its own content as the engine recorded it
                let spec;
                if (kind === OP_INSERT && b === 0) spec = { text: text.substr(pad, len) };
                else if (kind === OP_INSERT && b === 1) spec = { marker: { refType: pad } };
                return { kind, pos: r[i + 2], len,
                    before: kind === OP_ANNOTATE ? pset(a) : undefined,
                    after: kind === OP_ANNOTATE ? pset(b) : (kind === OP_INSERT ? pset(a) : undefined), spec };
            });
            c.deltaListener(entries, eventsOf);
        }
    }
}

// ---- SharedSegmentSequence's merge-tree plumbing (packages/dds/sequence/src/sequence.ts) ----

/** matchProperties (MT/properties.ts:64-95). */
function matchProperties(a, b) {
    if (a) {
        if (!b) return false;
        for (const key in a) {             // eslint-disable-line guard-for-in
            if (b[key] === undefined) return false;
            else if (typeof b[key] === "object") { if (!matchProperties(a[key], b[key])) return false; }
            else if (b[key] !== a[key]) return false;
        }
        for (const key in b) if (a[key] === undefined) return false;     // eslint-disable-line guard-for-in
    } else if (b) return false;
    return true;
}

/** Object.keys of SegmentPropertiesManager.addProperties' deltas for a sequenced annotate on an
 * observer (segmentPropertiesManager.ts:67-112): under "rewrite", the keys it deletes (falsy
 * in the op) in the segment's key order, then every key of the op's props. */
function annotateDeltaKeys(op, before) {
    const deltas = {};
    const newProps = op.props || {};
    if (op.combiningOp && op.combiningOp.name === "rewrite" && before) {
        for (const key of Object.keys(before)) if (!newProps[key]) deltas[key] = null;
    }
    for (const key of Object.keys(newProps)) deltas[key] = null;
    return Object.keys(deltas);
}

/** segment.clone().toJSONObject() of an inserted segment (textSegment.ts:48-54, mergeTree.ts:649-653). */
function segmentJson(opSeg, props) {
    if (typeof opSeg === "string" || opSeg.text !== undefined) {
        const text = typeof opSeg === "string" ? opSeg : opSeg.text;
        return props ? { text, props } : text;
    }
    const o = { marker: { refType: opSeg.marker.refType } };
    if (props) o.props = props;
    return o;
}

/** createOpsFromDelta (sequence.ts:58-105) for one op's sequenceDelta event (ranges in order). */
function opsFromDelta(member, ranges) {
    const ops = [];
    for (const r of ranges) {
        if (r.kind === OP_ANNOTATE) {
            const last = ops[ops.length - 1];
            const after = r.after || {};
            const props = {};
            for (const key of annotateDeltaKeys(member, r.before)) props[key] = after[key] === undefined ? null : after[key];
            if (last && last.pos2 === r.pos && matchProperties(last.props, props)) last.pos2 += r.len;
            else ops.push({ pos1: r.pos, pos2: r.pos + r.len, props, type: OP_ANNOTATE });
        } else if (r.kind === OP_INSERT) {
            // the inserted segment's clone: the op's seg, or a pasted clone's own content
            ops.push({ pos1: r.pos, seg: segmentJson(r.spec || member.seg, r.after), type: OP_INSERT });
        } else if (r.kind === OP_REMOVE) {
            const last = ops[ops.length - 1];
            if (last && last.pos1 === r.pos) last.pos2 += r.len;
            else ops.push({ pos1: r.pos, pos2: r.pos + r.len, type: OP_REMOVE });
        }
    }
    return ops;
}

/**
 * One SharedString channel's merge-tree plumbing on a ClientGroup document (the part of
 * SharedSegmentSequence on the replay path):
 *   processCore(message)   -> processMergeTreeMsg (sequence.ts:604-642): Client.applyMsg, and
 *                             for the legacy format the stash of sequenced ops, the ones with
 *                             refSeq !== seq - 1 rebuilt from their sequenceDelta events
 *                             (the engine's delta records) with refSeq = seq - 1
 *   snapshotMergeTree(serializer) (sequence.ts:592-602) -> Client.snapshot with the stash
 *   loadCore(storage)      -> Client.load, then the catch-up ops through processMergeTreeMsg
 * `runtime` supplies options and deltaManager {minimumSequenceNumber, lastSequenceNumber}.
 * The stash's transformations resolve when the group flushes (any read).
 */
class SequenceChannel {
    constructor(group, runtime) {
        this.runtime = runtime;
        const options = (runtime && runtime.options) || {};
        this.client = group.newClient(options);
        this.client.startOrUpdateCollaboration(runtime && runtime.clientId);
        this.legacy = options.newMergeTreeSnapshotFormat !== true;
        this.messagesSinceMSNChange = [];
        if (this.legacy) this.client.deltaListener = (entries, eventsOf) => this.stash(entries, eventsOf);
    }
    processCore(message, local) {
        if (message.type !== "op") throw new Error("Sequence message not operation");     // sequence.ts:559
        this.client.applyMsg(JSON.parse(JSON.stringify(message)));      // parseHandles: the channel's own copy
    }
    stash(entries, eventsOf) {
        for (const [message, opIds] of entries) {
            let stashMessage = message;
            if (message.referenceSequenceNumber !== message.sequenceNumber - 1) {
                const ops = [];
                mergeTreeMembers(message.contents).forEach((m, i) => { ops.push(...opsFromDelta(m, eventsOf(opIds[i]))); });
                stashMessage = { ...message, referenceSequenceNumber: message.sequenceNumber - 1,
                    contents: ops.length !== 1 ? { ops, type: OP_GROUP } : ops[0] };
            }
            this.messagesSinceMSNChange.push(stashMessage);
            if (this.messagesSinceMSNChange.length > 20
                && this.messagesSinceMSNChange[20].sequenceNumber < message.minimumSequenceNumber) {
                this.processMinSequenceNumberChanged(message.minimumSequenceNumber);
            }
        }
    }
    processMinSequenceNumberChanged(minSeq) {           // sequence.ts:648-658
        let index = 0;
        for (; index < this.messagesSinceMSNChange.length; index++) {
            if (this.messagesSinceMSNChange[index].sequenceNumber > minSeq) break;
        }
        if (index !== 0) this.messagesSinceMSNChange = this.messagesSinceMSNChange.slice(index);
    }
    snapshotMergeTree(serializer, handle) {
        this.client.group.flush();
        const minSeq = this.runtime.deltaManager.minimumSequenceNumber;
        this.processMinSequenceNumberChanged(minSeq);
        this.messagesSinceMSNChange.forEach((m) => { m.minimumSequenceNumber = minSeq; });
        return this.client.snapshot(this.runtime, handle, serializer, this.messagesSinceMSNChange);
    }
    /** loadCore (sequence.ts:496-541) for the merge-tree part of the channel's storage. */
    async loadCore(storage, serializer) {
        const { catchupOpsP } = await this.client.load(this.runtime, storage, serializer);
        for (const m of await catchupOpsP) {
            const w = { minSeq: this.client.minSeq, currentSeq: this.client.currentSeq };
            if (m.minimumSequenceNumber < w.minSeq || m.referenceSequenceNumber < w.minSeq
                || m.sequenceNumber <= w.minSeq || m.sequenceNumber <= w.currentSeq) {
                throw new Error(`Invalid catchup operations in snapshot: ${JSON.stringify({
                    op: { seq: m.sequenceNumber, minSeq: m.minimumSequenceNumber, refSeq: m.referenceSequenceNumber },
                    collabWindow: { seq: w.currentSeq, minSeq: w.minSeq } })}`);
            }
            this.processCore(m, false);
        }
    }
    getText() { return this.client.getText(); }
}

module.exports = { addon, Engine, ClientGroup, MergeTreeClient, BatchBuilder, PropTable, ClientNames, statusNames,
    LoadBuilder, parseSnapshot, SequenceChannel, opsFromDelta, matchProperties };
