"use strict";
// One ParallelPacker worker (parallel.js): parses its documents' message JSON and packs them
// with the host's BatchBuilder into typed-array columns, returned to the main thread with
// their buffers transferred.  The worker never loads the GPU addon.
const fs = require("fs");
const { parentPort } = require("worker_threads");
const { BatchBuilder, ClientNames, PropTable } = require("./builder.js");

parentPort.on("message", ({ docs }) => {
    try {
        const props = new PropTable();
        const bb = new BatchBuilder(props, null);
        const names = [];
        for (const d of docs) {
            const nm = new ClientNames();
            bb.names = nm;
            bb.beginDoc(d.id);
            // a document's stream: its JSON text, or a file the worker reads itself (a worker
            // that owns its documents' streams: nothing is cloned through the main thread)
            const text = d.json !== undefined ? d.json : fs.readFileSync(d.file, "utf8");
            for (const m of JSON.parse(text)) bb.addMessage(m);
            names.push(nm.names);
        }
        const nPayload = bb.payload.n;
        const b = bb.build();
        const batch = {};
        const transfer = [];
        for (const k of Object.keys(b)) {
            batch[k] = b[k].slice();                 // own, exactly sized buffers to transfer
            transfer.push(batch[k].buffer);
        }
        parentPort.postMessage({ batch, nPayload, names,
            props: { keys: props.keys, valueJson: props.valueJson, sets: props.sets } }, transfer);
    } catch (e) {
        parentPort.postMessage({ error: String(e && e.stack || e) });
    }
});
