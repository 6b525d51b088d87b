"use strict";
// Host ingest timing for bench.py (SURVEY.md §8(d): host packing and H2D are reported, not
// hidden).  Input: a directory of files doc<i>.json, each one document's sequenced messages
// as JSON text (what a summarizer receives per document stream).  Prints one JSON line:
//   single_ms    parse + pack of every document on the main thread (BatchBuilder)
//   parallel_ms  the same on a pool of `workers` worker_threads (ParallelPacker) + merge
//   e2e_ms       (with --gpu) messages in -> SnapshotV1 digests out through the addon:
//                parallel parse + pack, mt_apply_batch (pinned staging, one H2D), mt_sync,
//                then snapshots (digests) of every document
// usage: node ingest_bench.js DOCS_DIR WORKERS [--gpu]
const fs = require("fs");
const path = require("path");
const { BatchBuilder, ClientNames, PropTable } = require(path.join(__dirname, "builder.js"));
const { ParallelPacker } = require(path.join(__dirname, "parallel.js"));

async function main() {
    const dir = process.argv[2];
    const n = fs.readdirSync(dir).filter((f) => /^doc[0-9]+\.json$/.test(f)).length;
    const W = Number(process.argv[3] || 8);
    const gpu = process.argv.includes("--gpu");
    const docs = [];
    for (let id = 0; id < n; id++) {
        const file = path.join(dir, `doc${id}.json`);
        docs.push({ id, file, bytes: fs.statSync(file).size });
    }
    const now = () => Number(process.hrtime.bigint()) / 1e6;

    let t0 = now();
    const bb = new BatchBuilder(new PropTable(), null);
    let msgs = 0;
    for (const d of docs) {
        bb.names = new ClientNames();
        bb.beginDoc(d.id);
        for (const m of JSON.parse(fs.readFileSync(d.file, "utf8"))) { bb.addMessage(m); msgs++; }
    }
    const single = bb.build();
    const singleMs = now() - t0;

    const pool = new ParallelPacker(W);
    await pool.pack(docs, new PropTable());                                          // worker start-up + JIT, untimed
    t0 = now();
    const par = await pool.pack(docs, new PropTable());
    const parallelMs = now() - t0;
    const same = par.batch.type.length === single.type.length &&
        ["type", "seq", "pos1", "pos2", "payloadLen"].every((k) => par.batch[k].every((v, i) => v === single[k][i]));

    const out = { msgs, ops: single.type.length, workers: W, single_ms: singleMs, parallel_ms: parallelMs,
        single_msgs_per_s: msgs / (singleMs / 1e3), parallel_msgs_per_s: msgs / (parallelMs / 1e3),
        merge_ms: pool.lastMergeMs,
        parallel_equals_single: same };
    if (gpu) {
        const mt = require(path.join(__dirname, "index.js"));
        const maxOps = Math.max(...docs.map((d, i) => single.opOffsets[i + 1] - single.opOffsets[i]));
        const eng = new mt.Engine(docs.length, { rowsPerDoc: 3 * maxOps + 64, windowPerDoc: 8192, propsetsPerDoc: 2 * maxOps + 64,
            textPerDoc: 8 * maxOps + 4096, blocksPerDoc: maxOps + 64, heapPerDoc: 2 * maxOps + 64 });
        const ids = docs.map((d) => d.id);
        const run = async () => {
            eng.openDocs(0, docs.length);
            const { batch, names } = await pool.pack(docs, eng.props);
            names.forEach((nm, i) => mt.addon.setDocClientNames(eng.h, ids[i], nm.map((n) => JSON.stringify(n))));
            eng.apply(batch);
            eng.sync();
            const last = ids.map((i) => batch.opOffsets[i + 1] - 1);
            return eng.snapshot(ids, last.map((o) => batch.msn[o]), last.map((o) => batch.seq[o]));
        };
        await run();                                                                      // warm-up
        t0 = now();
        const snaps = await run();
        out.e2e_ms = now() - t0;
        out.e2e_msgs_per_s = msgs / (out.e2e_ms / 1e3);
        let x = 0n;
        for (const s of snaps) x ^= s.digest;
        out.digest_xor = x.toString(16).padStart(16, "0");
        eng.close();
    }
    await pool.close();
    process.stdout.write(JSON.stringify(out) + "\n");
}

main().catch((e) => { process.stderr.write(String(e && e.stack || e) + "\n"); process.exit(1); });
