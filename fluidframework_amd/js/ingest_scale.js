"use strict";
// Host ingest at full workload scale for bench.py (SURVEY.md §8(d): host packing and H2D are
// reported, not hidden).  Input: a directory of doc<i>.bin files, each one document's op columns
// (pack_worker.js binToJson).  Every worker of the pool first turns its documents into their
// message JSON text, split into WINDOWS consecutive message windows (the streams arriving over
// time; untimed), then:
//   pack_ms   parse + pack of every window of every document on the pool
//             (ParallelPacker.packHeld) + merges: the host's packing bound
//   e2e_ms    (with --gpu) messages in -> SnapshotV1 digests out through the addon: window k+1 of
//             every document is parsed and packed on the workers while the GPU uploads
//             (mt_apply_batch: pinned staging, async H2D) and replays window k of every document;
//             then one sync and SnapshotV1 of every document
// With --objects every worker holds its documents' messages as parsed objects (what DeltaManager
// hands SharedSegmentSequence.processCore; made untimed), packs them with BatchBuilder.addMessages
// and the parts go to the addon as they are (mt_apply_batch_parts concatenates them on the
// library's host threads): pack_ms is objects -> packed parts, e2e_ms objects -> digests.
// Prints one JSON line.  usage: node ingest_scale.js DIR WORKERS WINDOWS [--gpu] [--objects]
const fs = require("fs");
const path = require("path");
const { PropTable } = require(path.join(__dirname, "builder.js"));
const { ParallelPacker } = require(path.join(__dirname, "parallel.js"));

async function main() {
    const dir = process.argv[2];
    const W = Number(process.argv[3] || 16), K = Number(process.argv[4] || 8);
    const gpu = process.argv.includes("--gpu"), objects = process.argv.includes("--objects");
    const n = fs.readdirSync(dir).filter((f) => /^doc[0-9]+\.bin$/.test(f)).length;
    const docs = [];
    for (let id = 0; id < n; id++) docs.push({ id, bin: path.join(dir, `doc${id}.bin`) });
    const ids = docs.map((d) => d.id);
    const now = () => Number(process.hrtime.bigint()) / 1e6;
    const pool = new ParallelPacker(W);
    let t0 = now();
    const jsonBytes = await pool.prepare(docs, K, objects);
    const out = { docs: n, workers: W, windows: K, input: objects ? "objects" : "json", json_bytes: objects ? null : jsonBytes,
        prepare_ms: now() - t0 };
    // one window's parts of a pack (objects: unmerged parts; JSON: one merged batch)
    const packWin = async (props, k) => {
        if (!objects) { const r = await pool.packHeld(ids, props, k); return { parts: [r.batch], propMaps: [null], names: r.names }; }
        return pool.packHeldParts(ids, props, k);
    };
    await packWin(new PropTable(), 0);                                               // JIT warm-up, untimed
    await pool.resetNames();
    let msgs = 0, maxOps = 0;
    const opsOf = new Uint32Array(n);
    t0 = now();
    for (let k = 0; k < K; k++) {
        const { parts } = await packWin(new PropTable(), k);
        for (const batch of parts) {
            msgs += batch.type.length;
            for (let r = 0; r < batch.docIds.length; r++) opsOf[batch.docIds[r]] += batch.opOffsets[r + 1] - batch.opOffsets[r];
        }
    }
    out.pack_ms = now() - t0;
    out.msgs = msgs;
    out.pack_msgs_per_s = msgs / (out.pack_ms / 1e3);
    for (const v of opsOf) maxOps = Math.max(maxOps, v);
    if (gpu) {
        const mt = require(path.join(__dirname, "index.js"));
        const eng = new mt.Engine(n, { rowsPerDoc: 3 * maxOps + 64, windowPerDoc: 8192, propsetsPerDoc: 2 * maxOps + 64,
            textPerDoc: 8 * maxOps + 4096, blocksPerDoc: maxOps + 64, heapPerDoc: 2 * maxOps + 64 });
        eng.reserveStaging();
        const run = async () => {
            await pool.resetNames();
            eng.openDocs(0, n);
            const msn = new Int32Array(n), seq = new Int32Array(n);
            let applyMs = 0, packMs = 0;
            for (let k = 0; k < K; k++) {
                const tp = now();
                const { parts, propMaps, names } = await packWin(eng.props, k);   // overlaps the replay of window k-1
                packMs += now() - tp;
                let q = 0;
                for (const batch of parts) {
                    for (let r = 0; r < batch.docIds.length; r++, q++) {
                        const d = batch.docIds[r];
                        mt.addon.setDocClientNames(eng.h, d, names[q].map((x) => JSON.stringify(x)));
                        if (batch.opOffsets[r + 1] > batch.opOffsets[r]) {
                            const last = batch.opOffsets[r + 1] - 1;
                            msn[d] = batch.msn[last]; seq[d] = batch.seq[last];
                        }
                    }
                }
                const ta = now();
                // staged + enqueued: the replay runs while the next window packs
                if (objects) eng.applyParts(parts, propMaps); else eng.apply(parts[0]);
                applyMs += now() - ta;
            }
            const ts = now();
            eng.sync();
            const syncMs = now() - ts;
            const t2 = now();
            const snaps = eng.snapshot(ids, msn, seq);
            return { snaps, applyMs, packMs, syncMs, snapMs: now() - t2 };
        };
        await run();                                                                      // warm-up
        t0 = now();
        const r = await run();
        out.e2e_ms = now() - t0;
        out.e2e_msgs_per_s = out.msgs / (out.e2e_ms / 1e3);
        out.e2e_pack_ms = r.packMs; out.apply_ms = r.applyMs; out.final_sync_ms = r.syncMs; out.snapshot_ms = r.snapMs;
        let x = 0n;
        for (const s of r.snaps) x ^= s.digest;
        out.digest_xor = x.toString(16).padStart(16, "0");
        eng.close();
    }
    await pool.close();
    process.stdout.write(JSON.stringify(out) + "\n");
}

main().catch((e) => { process.stderr.write(String(e && e.stack || e) + "\n"); process.exit(1); });
