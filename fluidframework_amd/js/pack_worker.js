"use strict";
// One ParallelPacker worker (parallel.js): parses its documents' message JSON and packs them
// with the host's BatchBuilder into typed-array columns, returned to the main thread with
// their buffers transferred.  The worker never loads the GPU addon.
const fs = require("fs");
const { parentPort } = require("worker_threads");
const { BatchBuilder, ClientNames, PropTable } = require("./builder.js");

// A document's stream synthesized from its binary op columns (ingest benchmarking: the JSON
// text a summarizer would receive, made inside the worker that will parse it; untimed).
// File layout (little-endian int32): nOps, nPayload, then type, client, seq, refSeq, msn, pos1,
// pos2, payloadOff, payloadLen columns of nOps each, then nPayload UTF-16 units.
function binToJson(file, windows, objects = false) {
    const buf = fs.readFileSync(file);
    const i32 = new Int32Array(buf.buffer, buf.byteOffset, buf.length >> 2);
    const n = i32[0], np = i32[1];
    const col = (k) => i32.subarray(2 + k * n, 2 + (k + 1) * n);
    const [ty, cl, sq, rf, ms, p1, p2, po, pl] = [0, 1, 2, 3, 4, 5, 6, 7, 8].map(col);
    const pay = new Uint16Array(buf.buffer, buf.byteOffset + 4 * (2 + 9 * n), np);
    const out = new Array(n);
    for (let i = 0; i < n; i++) {
        const m = { clientId: "c" + cl[i], sequenceNumber: sq[i], referenceSequenceNumber: rf[i], minimumSequenceNumber: ms[i],
            type: "op" };
        if (ty[i] === 0) m.contents = { type: 0, pos1: p1[i], seg: String.fromCharCode.apply(null, pay.subarray(po[i], po[i] + pl[i])) };
        else {
            m.contents = { type: ty[i], pos1: p1[i], pos2: p2[i] };
            if (ty[i] === 2) m.contents.props = { k0: "v" };
        }
        out[i] = m;
    }
    // `windows` consecutive message windows of equal counts, one JSON text each (a stream
    // arriving over time), or (objects) the message objects themselves, as DeltaManager hands
    // them to SharedSegmentSequence.processCore already parsed
    const texts = [];
    for (let k = 0; k < windows; k++) {
        const w = out.slice(Math.floor((k * n) / windows), Math.floor(((k + 1) * n) / windows));
        texts.push(objects ? w : JSON.stringify(w));
    }
    return texts;
}
const held = new Map();            // doc id -> its stream's window JSON texts (ParallelPacker.prepare)
let shared = null;                 // the worker's builder: shared-memory columns reused batch after batch
const heldNames = new Map();       // doc id -> its ClientNames, kept across windows

parentPort.on("message", ({ docs, prepare, windows, objects, resetNames }) => {
    if (resetNames) { heldNames.clear(); parentPort.postMessage({ reset: true }); return; }
    if (prepare) {
        try {
            let bytes = 0;
            for (const d of prepare) {
                const t = binToJson(d.bin, windows || 1, !!objects);
                held.set(d.id, t);
                for (const x of t) bytes += objects ? 0 : x.length;
            }
            parentPort.postMessage({ prepared: prepare.length, bytes });
        } catch (e) {
            parentPort.postMessage({ error: String(e && e.stack || e) });
        }
        return;
    }
    try {
        const props = new PropTable();
        if (!shared) shared = new BatchBuilder(props, null, true);
        const bb = shared;
        bb.reset(props);
        const names = [];
        for (const d of docs) {
            let nm = d.held ? heldNames.get(d.id) : undefined;
            if (!nm) { nm = new ClientNames(); if (d.held) heldNames.set(d.id, nm); }
            bb.names = nm;
            bb.beginDoc(d.id);
            // a document's stream: its JSON text, or a file the worker reads itself (a worker
            // that owns its documents' streams: nothing is cloned through the main thread)
            const text = d.held ? held.get(d.id)[d.win || 0] : d.json !== undefined ? d.json : fs.readFileSync(d.file, "utf8");
            bb.addMessages(typeof text === "string" ? JSON.parse(text) : text);
            names.push(nm.names.slice());
        }
        const nPayload = bb.payload.n;
        // the columns are views of this worker's shared buffers: valid until its next batch (the
        // main thread consumes a batch, mt_apply_batch_parts copies it, before asking for another)
        const batch = bb.build();
        parentPort.postMessage({ batch, nPayload, names,
            props: { keys: props.keys, valueJson: props.valueJson, sets: props.sets, incrKeys: [...props.incrKeys],
                nIncr: props.nIncr } });
    } catch (e) {
        parentPort.postMessage({ error: String(e && e.stack || e) });
    }
});
