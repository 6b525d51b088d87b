"""The Node host (fluidframework_amd/js + the N-API addon) against the oracle.

CPU: the addon source built against the host emulation of the engine runs the
whole Node path (message packing, per-document client ids, property interning,
snapshot ITree) and must match the oracle bit for bit.  GPU: the product addon
(mtgpu.node over libmtgpu.so) does the same on the device.
"""
import json
import os
import subprocess

import pytest

from emu_lib import build_emu_napi
from js_lib import NODE, ROOT, batch_to_messages, run_node
from oracle_lib import gen_params, generate
from test_emu_parity import CONFIGS, ann_props

pytestmark = pytest.mark.skipif(NODE is None, reason="node is not installed")

EXPORTS = ["applyBatch", "applyBatchParts", "create", "deltaCapture", "deltaRecords", "deltaText", "destroy", "docPset", "docStatus", "docsOpen",
           "getContainingSegment", "getLength", "getText", "lastError",
           "loadSnapshot", "reserveStaging", "setClientNames", "setDocClientNames", "setDocSnapshotChunk", "setProps", "setResidency", "snapshotLegacy", "snapshotV1", "sync",
           "syncAsync",
           "updateSeq"]


def check(cfg, n_docs, addon, seed=31):
    props = ann_props()
    p = gen_params(seed=seed, n_docs=n_docs, **CONFIGS[cfg])
    batch, st, kept = generate(p, props, keep=True)
    assert st == [0] * n_docs
    msgs = [batch_to_messages(batch, props, d) for d in range(n_docs)]
    # The reference's default (legacy) format too: even documents pass catch-up
    # messages (their last 3), odd ones none; the blob is JSON.stringify(catchUpMsgs)
    # under catchUpBlobName (snapshotlegacy.ts:162-172).
    catch_up = [msgs[d][-3:] if d % 2 == 0 else [] for d in range(n_docs)]
    blob_name = "randomNameForCatchUpOps"     # generateSharedStrings.ts:17 renames it the same way
    queries = position_queries(batch, kept, CONFIGS[cfg]["clients"], seed)
    got = run_node(msgs, addon=addon, limits=dict(rowsPerDoc=20000, windowPerDoc=8192, propsetsPerDoc=8192,
                                                  textPerDoc=1 << 18),
                   legacy={"options": {"catchUpBlobName": blob_name}, "catchUp": catch_up}, queries=queries)
    check_queries(queries, got["queries"], kept)
    last = batch.op_offsets[1:] - 1
    for d in range(n_docs):
        od = kept[d]
        assert got["texts"][d] == od.get_text(), f"doc {d} text"
        assert got["lengths"][d] == od.get_length()
        blobs, dig = od.snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]))
        want = [("header" if i == 0 else f"body_{i - 1}", b.decode("utf-8")) for i, b in enumerate(blobs)]
        assert [tuple(x) for x in got["blobs"][d]] == want, f"doc {d} snapshot"
        assert int(got["digests"][d], 16) == dig
        lblobs, _ = od.snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]), legacy=True)
        want = [("header" if i == 0 else "body", b.decode("utf-8")) for i, b in enumerate(lblobs)]
        if catch_up[d]:
            want.append((blob_name, json.dumps(catch_up[d], separators=(",", ":"))))
        assert [tuple(x) for x in got["legacy"][d]] == want, f"doc {d} legacy snapshot"


def position_queries(batch, kept, n_clients, seed, per_doc=60):
    """[doc, pos, refSeq, "c<i>"] queries under valid perspectives (refSeq at or above the
    client's last refSeq and the MSN; -1: the local view) at the end of each stream."""
    import numpy as np
    rng = np.random.RandomState(seed)
    A, out = batch.arrays, []
    for d in range(len(batch.op_offsets) - 1):
        o0, o1 = int(batch.op_offsets[d]), int(batch.op_offsets[d + 1])
        ms, cs = int(A["msn"][o1 - 1]), int(A["seq"][o1 - 1])
        last_ref = {}
        for k in range(o0, o1):
            c = int(A["client"][k])
            last_ref[c] = max(last_ref.get(c, 0), int(A["ref_seq"][k]))
        for _ in range(per_doc):
            if rng.rand() < 0.3:
                out.append([d, int(rng.randint(-1, kept[d].get_length(cs, -1) + 2)), -1, None])
                continue
            c = int(rng.randint(0, n_clients))
            r = int(rng.randint(max(ms, last_ref.get(c, 0)), cs + 1))
            out.append([d, int(rng.randint(-1, kept[d].get_length(r, c) + 3)), r, f"c{c}"])
    return out


def check_queries(queries, got, kept):
    """Node's answers (engine record and the Client method) against the oracle's."""
    for (d, pos, ref, who), g in zip(queries, got):
        c = -1 if who is None else int(who[1:])
        want, wjs = kept[d].containing_segment(pos, ref, c)
        name = lambda i: None if i < 0 else f"c{i}"  # noqa: E731
        assert [g["found"], g["offset"], g["obsPos"], g["len"], g["seq"], g["client"], g["removedSeq"],
                g["removedClient"], g["resolved"]] == [int(want[0]), int(want[1]), int(want[2]), int(want[3]),
                                                       int(want[4]), name(int(want[5])), int(want[6]),
                                                       name(int(want[7])), int(want[14])], (d, pos, ref, who, g)
        assert g["json"] == wjs
        if who is None:
            assert g["viaClient"] == (None if wjs is None else [json.dumps(json.loads(wjs), separators=(",", ":"),
                                                                          ensure_ascii=False), int(want[1]),
                                                               int(want[2])])
        elif "viaClient" in g:
            assert g["viaClient"] == (None if int(want[14]) == -(1 << 31) else int(want[14]))


def test_product_addon_loads_and_exports():
    import __graft_entry__
    __graft_entry__.build_engine()
    path = __graft_entry__.build_napi()
    out = subprocess.run([NODE, "-e", f"console.log(JSON.stringify(Object.keys(require({json.dumps(path)})).sort()))"],
                         check=True, capture_output=True, text=True).stdout
    assert json.loads(out) == sorted(EXPORTS)


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
def test_node_host_on_emulation_matches_oracle(cfg):
    check(cfg, 3, build_emu_napi())


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["cfg1", "cfg2", "cfg3"])
def test_node_host_on_gpu_matches_oracle(cfg):
    check(cfg, 6, os.path.join(ROOT, "fluidframework_amd", "js", "mtgpu.node"))


def check_load(addon):
    """Client.load through the Node host: golden V1 files, and a collaborative
    snapshot taken mid-stream followed by the rest of the stream."""
    from test_snapshot_load import COLLAB_CASES, GOLDEN, collab_case, golden_blobs, oracle_load, sub_batch
    loads, msgs, want_text, want_blobs = [], [], [], []
    for name in GOLDEN:
        want, blobs = golden_blobs(name)
        loads.append(want)
        msgs.append([])
        od, st = oracle_load(blobs, ann_props())
        assert st == 0
        want_text.append(od.get_text())
        want_blobs.append(None)
    case = dict(COLLAB_CASES[0])
    cut = case.pop("cut")
    props, batch, snaps, blobs_l = collab_case(cut=cut, **case)
    for d in range(case["n_docs"]):
        loads.append({("header" if i == 0 else f"body_{i - 1}"): b for i, b in enumerate(blobs_l[d])})
        msgs.append(batch_to_messages(batch, props, d)[cut:])
        od, st = oracle_load(blobs_l[d], props)
        assert st == 0
        assert od.apply_run(sub_batch(batch, d, cut, case["ops"], 0), 0) == 0
        want_text.append(od.get_text())
        o = int(batch.op_offsets[d + 1]) - 1
        ob, _ = od.snapshot(int(batch.arrays["msn"][o]), int(batch.arrays["seq"][o]))
        want_blobs.append([("header" if i == 0 else f"body_{i - 1}", b.decode()) for i, b in enumerate(ob)])
    got = run_node(msgs, addon=addon, loads=loads,
                   limits=dict(rowsPerDoc=40000, windowPerDoc=8192, propsetsPerDoc=8192, textPerDoc=1 << 19,
                               blocksPerDoc=16384))
    for d in range(len(msgs)):
        assert got["texts"][d] == want_text[d], f"doc {d} text"
        if want_blobs[d] is not None:
            assert [tuple(x) for x in got["blobs"][d]] == want_blobs[d], f"doc {d} snapshot"


def test_node_host_load_on_emulation_matches_oracle():
    check_load(build_emu_napi())


@pytest.mark.gpu
def test_node_host_load_on_gpu_matches_oracle():
    check_load(os.path.join(ROOT, "fluidframework_amd", "js", "mtgpu.node"))


def check_parallel_ingest(addon, n_docs, tmp_path, cfg="cfg3", workers=3):
    """The Node ingest path (fluidframework_amd/js/ingest_bench.js): per-document JSON streams
    parsed and packed by a worker_threads pool (parallel.js) equal the single-thread packing
    column for column, and, applied through the addon, give every document the oracle's
    SnapshotV1 digest (their xor)."""
    props = ann_props()
    p = gen_params(seed=43, n_docs=n_docs, **dict(CONFIGS[cfg], ops=400))
    batch, st, kept = generate(p, props, keep=True)
    assert st == [0] * n_docs
    for d in range(n_docs):
        with open(tmp_path / f"doc{d}.json", "w") as f:
            json.dump(batch_to_messages(batch, props, d), f)
    env = dict(os.environ, MTGPU_NAPI=addon)
    r = subprocess.run([NODE, os.path.join(ROOT, "fluidframework_amd", "js", "ingest_bench.js"), str(tmp_path),
                        str(workers), "--gpu"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["parallel_equals_single"] and out["msgs"] == int(batch.op_offsets[-1])
    last = batch.op_offsets[1:] - 1
    x = 0
    for d in range(n_docs):
        x ^= kept[d].snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]))[1]
    assert out["digest_xor"] == f"{x:016x}"


def test_parallel_ingest_on_emulation(tmp_path):
    check_parallel_ingest(build_emu_napi(), 7, tmp_path)


@pytest.mark.gpu
def test_parallel_ingest_on_gpu(tmp_path):
    check_parallel_ingest(os.path.join(ROOT, "fluidframework_amd", "js", "mtgpu.node"), 16, tmp_path, workers=8)
