"use strict";
// Test driver: the same documents' messages applied (a) as one batch packed by one BatchBuilder
// with addMessage, (b) as parts packed by several BatchBuilders, each with its own PropTable and
// addMessages (what ParallelPacker's workers do), handed to mt_apply_batch_parts with their
// property maps.  Prints both engines' texts and SnapshotV1 digests.
// usage: node parts_check.js IN.json OUT.json   (IN: {docs: [[msg...]...], parts: k})
const fs = require("fs");
const path = require("path");
const js = path.join(__dirname, "..", "..", "fluidframework_amd", "js");
const mt = require(js);
const { BatchBuilder, ClientNames, PropTable } = require(path.join(js, "builder.js"));
const { absorb } = require(path.join(js, "parallel.js"));

const [inPath, outPath] = process.argv.slice(2);
const spec = JSON.parse(fs.readFileSync(inPath, "utf8"));
const n = spec.docs.length, K = spec.parts;
const limits = { rowsPerDoc: 20000, windowPerDoc: 8192, propsetsPerDoc: 8192, textPerDoc: 1 << 18 };
const finish = (eng, namesOf) => {
    const ids = [...Array(n).keys()];
    ids.forEach((d) => mt.addon.setDocClientNames(eng.h, d, namesOf[d].map((x) => JSON.stringify(x))));
    const last = (d) => spec.docs[d][spec.docs[d].length - 1];
    const snaps = eng.snapshot(ids, ids.map((d) => last(d).minimumSequenceNumber), ids.map((d) => last(d).sequenceNumber));
    const texts = mt.addon.getText(eng.h, Uint32Array.from(ids));
    return { digests: snaps.map((s) => s.digest.toString(16)), texts };
};
// (a) one builder
const e1 = new mt.Engine(n, limits);
e1.openDocs(0, n);
const bb = new BatchBuilder(e1.props, null);
const names1 = [];
spec.docs.forEach((msgs, d) => { bb.names = new ClientNames(); bb.beginDoc(d); for (const m of msgs) bb.addMessage(m); names1.push(bb.names.names); });
e1.apply(bb.build());
e1.sync();
const a = finish(e1, names1);
// (b) K parts, documents dealt round-robin so every part interleaves with the others
const e2 = new mt.Engine(n, limits);
e2.openDocs(0, n);
const parts = [], maps = [], names2 = new Array(n);
for (let p = 0; p < K; p++) {
    const pt = new PropTable();
    const b = new BatchBuilder(pt, null);
    for (let d = p; d < n; d += K) { b.names = new ClientNames(); b.beginDoc(d); b.addMessages(spec.docs[d]); names2[d] = b.names.names; }
    parts.push(b.build());
    maps.push(pt.sets.length ? absorb(pt, e2.props) : null);
}
e2.applyParts(parts, maps);
e2.sync();
const b2 = finish(e2, names2);
fs.writeFileSync(outPath, JSON.stringify({ a, b: b2 }));
e1.close(); e2.close();
