"use strict";
// Test driver for the Node host (fluidframework_amd/js): replays sequenced
// message lists, one ClientGroup document per list, through MergeTreeClient
// (the Client drop-in) and prints what the parity tests compare against the
// oracle: text, length, SnapshotV1 (and SnapshotLegacy) ITree blobs and digests (optionally after
// loading a snapshot into each document).
// usage: node replay_check.js IN.json OUT.json
const fs = require("fs");
const path = require("path");
const mt = require(path.join(__dirname, "..", "..", "fluidframework_amd", "js"));

const [inPath, outPath] = process.argv.slice(2);
const spec = JSON.parse(fs.readFileSync(inPath, "utf8"));
const eng = new mt.Engine(spec.docs.length, spec.limits || {});
const group = new mt.ClientGroup(eng);
const clients = spec.docs.map(() => {
    const c = group.newClient(spec.options || { newMergeTreeSnapshotFormat: true });
    c.startOrUpdateCollaboration("observer");
    return c;
});
// optional: load a snapshot into each document first (Client.load / SnapshotLoader)
if (spec.loads) spec.loads.forEach((blobs, d) => { if (blobs) clients[d].loadBlobs(blobs); });
spec.docs.forEach((msgs, d) => { for (const m of msgs) clients[d].applyMsg(m); });
const out = { texts: [], lengths: [], blobs: [], digests: [], legacy: [] };
clients.forEach((c, d) => {
    out.texts.push(c.getText());
    out.lengths.push(c.getLength());
    out.blobs.push(c.snapshotTree().entries.map((e) => [e.path, e.value.contents]));
    if (spec.legacy) {      // the reference's default format: a Client without newMergeTreeSnapshotFormat
        const opts = c.options;
        c.options = spec.legacy.options || {};
        out.legacy.push(c.snapshotTree(spec.legacy.catchUp ? spec.legacy.catchUp[d] : undefined).entries
            .map((e) => [e.path, e.value.contents]));
        c.options = opts;
    }
});
// optional position queries [doc, pos, refSeq (< 0: local view), long client id]: through the
// Client (getContainingSegment / getPosition / resolveRemoteClientPosition) and the engine
if (spec.queries) {
    out.queries = spec.queries.map(([d, pos, ref, who]) => {
        const c = clients[d];
        const local = ref < 0;
        const known = !local && c.names.ids.has(who);
        const cli = local ? -1 : (known ? c.names.ids.get(who) : 60);
        const q = eng.containingSegment([c.docId], [pos], [ref], [cli])[0];
        const name = (i) => (i < 0 ? null : c.names.names[i]);
        const r = { ...q, client: name(q.client), removedClient: name(q.removedClient) };
        if (local) {
            const { segment, offset } = c.getContainingSegment(pos);
            r.viaClient = segment === undefined ? null : [JSON.stringify(segment.toJSONObject()), offset, c.getPosition(segment)];
        } else if (known) {
            r.viaClient = c.resolveRemoteClientPosition(pos, ref, c.getShortClientId(who));
            if (r.viaClient === undefined) r.viaClient = null;
        }
        return r;
    });
}
// digests of the Clients' own format (SnapshotLegacy without newMergeTreeSnapshotFormat)
const legacyFormat = (spec.options || { newMergeTreeSnapshotFormat: true }).newMergeTreeSnapshotFormat !== true;
const snaps = eng.snapshot(clients.map((c) => c.docId), clients.map((c) => c.minSeq), clients.map((c) => c.getCurrentSeq()),
    legacyFormat);
out.digests = snaps.map((s) => s.digest.toString(16));
fs.writeFileSync(outPath, JSON.stringify(out));
eng.close();
