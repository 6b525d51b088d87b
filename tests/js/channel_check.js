"use strict";
// Test driver for the Node host's SharedSegmentSequence plumbing (SequenceChannel):
// each message list is one channel's sequenced ops; the runtime mock's deltaManager
// follows the messages.  Prints each channel's snapshotMergeTree ITree (through the
// reference-signature Client.snapshot), its text, and the text of a fresh channel that
// loadCore()s the tree through an IChannelStorageService (readBlob / list / contains)
// and processes the catch-up ops.
// usage: node channel_check.js IN.json OUT.json
const fs = require("fs");
const path = require("path");
const mt = require(path.join(__dirname, "..", "..", "fluidframework_amd", "js"));

const [inPath, outPath] = process.argv.slice(2);
const spec = JSON.parse(fs.readFileSync(inPath, "utf8"));
const n = spec.channels.length;
const eng = new mt.Engine(2 * n, spec.limits || {});
const group = new mt.ClientGroup(eng);
const runtime = (id) => ({ clientId: id, options: spec.options || {},
    deltaManager: { minimumSequenceNumber: 0, lastSequenceNumber: 0 } });
const runtimes = spec.channels.map(() => runtime("observer"));
const chans = runtimes.map((rt) => new mt.SequenceChannel(group, rt));
const longest = Math.max(...spec.channels.map((c) => c.length));
for (let k = 0; k < longest; k++) {
    spec.channels.forEach((msgs, d) => {
        if (k >= msgs.length) return;
        const m = msgs[k], dm = runtimes[d].deltaManager;
        dm.minimumSequenceNumber = m.minimumSequenceNumber;
        dm.lastSequenceNumber = m.sequenceNumber;
        chans[d].processCore(m, false);
    });
    if (k % spec.flushEvery === spec.flushEvery - 1) group.flush();     // several device batches
}
const serializer = { stringify: (v) => JSON.stringify(v) };
function storageOf(tree) {          // MockStorage over an ITree (test-runtime-utils/mockStorage.ts)
    const find = (p) => tree.entries.find((e) => e.path === p);
    return {
        readBlob: async (p) => {
            const e = find(p);
            if (!e) throw new Error(`Blob does not exist: ${p}`);
            return Buffer.from(e.value.contents, "utf8");
        },
        contains: async (p) => find(p) !== undefined,
        list: async () => tree.entries.map((e) => e.path),
    };
}
(async () => {
    const out = { trees: [], texts: [], loaded: [] };
    for (const ch of chans) {
        const tree = ch.snapshotMergeTree(serializer, undefined);
        out.trees.push(tree.entries.map((e) => [e.path, e.value.contents]));
        out.texts.push(ch.getText());
        const rt = runtime("loader");
        const ch2 = new mt.SequenceChannel(group, rt);
        await ch2.loadCore(storageOf(tree), serializer);
        out.loaded.push(ch2.getText());
    }
    fs.writeFileSync(outPath, JSON.stringify(out));
    eng.close();
})().catch((e) => { console.error(e); process.exit(1); });
