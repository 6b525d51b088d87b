"use strict";
// Host ingest timing for bench.py: packs ISequencedDocumentMessage lists (one list per
// document) into an mt_op_batch with the Node host's BatchBuilder, as MergeTreeClient
// flushes do, and prints {"msgs": n, "ms": t} for the packing alone (JSON parse excluded).
// usage: node pack_bench.js MESSAGES.json
const fs = require("fs");
const path = require("path");
const mt = require(path.join(__dirname, "index.js"));

const docs = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
let msgs = 0;
for (const d of docs) msgs += d.length;
const props = new mt.PropTable();
const names = docs.map(() => new mt.ClientNames());
const t0 = process.hrtime.bigint();
const bb = new mt.BatchBuilder(props, null);
docs.forEach((list, d) => {
    bb.names = names[d];
    bb.beginDoc(d);
    for (const m of list) bb.addMessage(m);
});
const batch = bb.build();
const ms = Number(process.hrtime.bigint() - t0) / 1e6;
process.stdout.write(JSON.stringify({ msgs, ms, ops: batch.type.length }) + "\n");
