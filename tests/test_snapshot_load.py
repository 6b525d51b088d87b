"""Snapshot load (SnapshotLoader, MT/snapshotLoader.ts:39-222): oracle and engine.

* The reference's golden SnapshotV1 files (tests/golden/reference_snapshots_v1,
  from packages/dds/sequence/src/test/snapshots/v1) load to the text the recipes
  build and re-serialize byte-for-byte (the reference's "Snapshot rebuild" test,
  sequence/src/test/snapshotVersion.spec.ts:29-72, in observer form).
* Collaborative snapshots (collab window non-empty) taken mid-stream load
  identically in the oracle and the engine (status word, segment rows, tree
  shape), and the rest of the stream then replays on the loaded documents.
  Where the header holds the whole document the loaded replay ends with the same
  text as the uninterrupted replay.  Bodies holding window segments exercise
  loadBody's reference behaviour (insert failures, never-emptied batch).

The emulated engine runs the product's mt_core.h logic; test_gpu_parity.py
repeats the engine side on the device.
"""
import json
import os

import numpy as np
import pytest

from fluidframework_amd.batch import ClientNames, OpBatch, PropTable
from fluidframework_amd.snapshot_load import LoadBatchBuilder, load_caps, parse_snapshot
from oracle_lib import OracleDoc, gen_params, generate
from emu_lib import emu_engine
import test_oracle_golden as G

NAMES = ['"c%d"' % i for i in range(64)]
GOLDEN = ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations"]


def golden_blobs(name):
    want = G.blobs_of(name)
    order = ["header"] + sorted([k for k in want if k != "header"], key=lambda k: int(k.split("_")[1]))
    return want, [want[k] for k in order]


def stream_names(n=64):
    cn = ClientNames()
    for i in range(n):
        cn.index("c%d" % i)
    return cn


def oracle_load(blobs, props):
    d = OracleDoc(collaborating=False, props=props, names=NAMES)
    st = d.load_snapshot(blobs)
    return d, st


def engine_load(factory, snaps, props, extra_rows=0, extra_text=0):
    """Loads parsed snapshots into documents 0..n-1 of a new engine."""
    caps = load_caps(snaps, extra_rows=extra_rows, extra_text=extra_text)
    eng = factory(len(snaps), per_doc=caps)
    eng.props = props
    names = []
    bb = LoadBatchBuilder(props)
    for i, s in enumerate(snaps):
        cn = stream_names()
        bb.add(i, s, cn)
        names.append(cn)
    batch = bb.build()
    eng.upload_props(props)
    for i, cn in enumerate(names):
        eng.upload_doc_names(i, cn.json_literals())
    eng.load_snapshot(batch)
    eng.sync()
    return eng


# ---------------------------------------------------------------- golden ----
@pytest.mark.parametrize("name", GOLDEN)
def test_oracle_loads_reference_snapshot(name):
    want, blobs = golden_blobs(name)
    d, st = oracle_load(blobs, PropTable())
    assert st == 0
    ref = G.build(name)
    assert d.get_text() == ref.get_text()
    assert d.get_length() == ref.get_length()
    got, _ = d.snapshot(0, 0)
    assert [b.decode() for b in got] == blobs


@pytest.mark.parametrize("name", GOLDEN)
def test_engine_loads_reference_snapshot(name):
    check_golden(name, emu_engine)


def check_golden(name, factory):
    want, blobs = golden_blobs(name)
    props = PropTable()
    snap = parse_snapshot(want)
    eng = engine_load(factory, [snap], props)
    assert int(eng.status([0])[0]) == 0
    od, _ = oracle_load(blobs, props)
    assert eng.get_text([0])[0] == od.get_text()
    ed, odump = eng.dump(0), od.dump()
    assert ed.shape == odump.shape and (ed == odump).all()
    (eb, _), = eng.snapshot([0], [0], [0])
    assert [b.decode() for b in eb] == blobs


def golden_legacy_blobs(name):
    want = G.blobs_of(name, legacy=True)
    return want, [want[k] for k in ("header", "body") if k in want]


@pytest.mark.parametrize("name", GOLDEN)
def test_oracle_legacy_snapshot_round_trip(name):
    """Reference legacy files load (legacy chunk parsing) and re-serialize as
    SnapshotLegacy byte-for-byte."""
    want, blobs = golden_legacy_blobs(name)
    d, st = oracle_load(blobs, PropTable())
    assert st == 0
    assert d.get_text() == G.build(name).get_text()
    got, _ = d.snapshot(0, 0, legacy=True)
    assert [b.decode() for b in got] == blobs


@pytest.mark.parametrize("name", GOLDEN)
def test_engine_legacy_snapshot_round_trip(name):
    check_golden_legacy(name, emu_engine)


def check_golden_legacy(name, factory):
    want, blobs = golden_legacy_blobs(name)
    props = PropTable()
    eng = engine_load(factory, [parse_snapshot(want)], props)
    assert int(eng.status([0])[0]) == 0
    (eb, edig), = eng.snapshot([0], [0], [0], legacy=True)
    assert [b.decode() for b in eb] == blobs
    od, _ = oracle_load(blobs, props)
    assert od.snapshot(0, 0, legacy=True)[1] == edig


def test_parse_legacy_header_metadata():
    """Legacy chunks (version undefined) normalize as toLatestVersion does."""
    hdr = {"chunkStartSegmentIndex": 0, "chunkSegmentCount": 2, "chunkLengthChars": 5, "totalLengthChars": 5,
           "totalSegmentCount": 2, "chunkSequenceNumber": 7, "segmentTexts": ["abc", {"text": "de", "props": {"a": 1}}]}
    s = parse_snapshot([json.dumps(hdr)])
    assert (s.min_seq, s.seq, len(s.header), s.body) == (7, 7, 2, [])


# ------------------------------------------------------- collaborative ----
def sub_batch(batch: OpBatch, run: int, a: int, b: int, doc: int) -> OpBatch:
    o0 = int(batch.op_offsets[run])
    arrays = {k: v[o0 + a:o0 + b].copy() for k, v in batch.arrays.items()}
    return OpBatch(np.asarray([doc], np.uint32), np.asarray([0, b - a], np.uint32), arrays, batch.payload)


def collab_case(seed, n_docs, ops, cut, **kw):
    props = PropTable()
    for i in range(6):
        props.intern({f"k{i % 3}": ["x", 1, None][i % 3], f"k{(i + 1) % 3}": f"y{i}"})
    p = gen_params(seed=seed, n_docs=n_docs, ops=ops, **kw)
    batch, st, _ = generate(p, props)
    assert st == [0] * n_docs
    # replay the first `cut` ops on fresh oracle docs and snapshot there
    snaps, blobs_l = [], []
    for d in range(n_docs):
        od = OracleDoc(collaborating=True, props=props, names=NAMES)
        assert od.apply_run(sub_batch(batch, d, 0, cut, 0), 0) == 0
        o = int(batch.op_offsets[d]) + cut - 1
        blobs, _ = od.snapshot(int(batch.arrays["msn"][o]), int(batch.arrays["seq"][o]))
        blobs_l.append([b.decode() for b in blobs])
        snaps.append(parse_snapshot(blobs_l[-1]))
    return props, batch, snaps, blobs_l


COLLAB_CASES = [
    dict(seed=3, n_docs=4, ops=1200, cut=700, clients=4, lag=16, ins=60, rem=40, ins_len=8, rem_len=8),
    dict(seed=4, n_docs=3, ops=1500, cut=900, clients=8, lag=4, ins=30, rem=30, ins_len=8, rem_len=16, ann_sets=6,
         rewrite=10),
    dict(seed=5, n_docs=3, ops=2600, cut=2300, clients=3, lag=32, ins=85, rem=15, ins_len=16, rem_len=6),
]


@pytest.mark.parametrize("case", COLLAB_CASES)
def test_collab_snapshot_load_and_continue(case):
    check_collab(case, emu_engine)


def check_collab(case, factory):
    case = dict(case)
    cut = case.pop("cut")
    props, batch, snaps, blobs_l = collab_case(cut=cut, **case)
    n_docs = case["n_docs"]
    eng = engine_load(factory, snaps, props, extra_rows=4 * case["ops"], extra_text=16 * case["ops"])
    est = eng.status(range(n_docs))
    seen_body = 0
    for d in range(n_docs):
        od, ost = oracle_load(blobs_l[d], props)
        assert int(est[d]) == ost, f"doc {d} load status emu {est[d]} oracle {ost}"
        seen_body += len(snaps[d].body) > 0
        if ost:
            continue
        ed, odump = eng.dump(d), od.dump()
        assert ed.shape == odump.shape and (ed == odump).all(), f"doc {d} loaded rows"
        assert eng.get_text([d])[0] == od.get_text()
        # continue the stream on both loaded documents
        rest = sub_batch(batch, d, cut, case["ops"], d)
        ost2 = od.apply_run(sub_batch(batch, d, cut, case["ops"], 0), 0)
        eng.apply(rest)
        eng.sync()
        assert int(eng.status([d])[0]) == ost2
        if ost2:
            continue
        assert eng.get_text([d])[0] == od.get_text()
        ed, odump = eng.dump(d), od.dump()
        assert ed.shape == odump.shape and (ed == odump).all(), f"doc {d} rows after continuing"
        o = int(batch.op_offsets[d + 1]) - 1
        ms, sq = int(batch.arrays["msn"][o]), int(batch.arrays["seq"][o])
        (eb, edig), = eng.snapshot([d], [ms], [sq])
        ob, odig = od.snapshot(ms, sq)
        assert eb == ob and edig == odig
        if not snaps[d].body:
            # header-only snapshot: the loaded replay reaches the uninterrupted replay's text
            full = OracleDoc(collaborating=True, props=props, names=NAMES)
            assert full.apply_run(sub_batch(batch, d, 0, case["ops"], 0), 0) == 0
            assert od.get_text() == full.get_text()
    if case["seed"] == 5:
        assert seen_body > 0, "case meant to produce body chunks"


def test_rejected_document_is_flagged():
    props = PropTable()
    bad = {"version": "1", "segmentCount": 1, "length": 1, "startIndex": 0,
           "segments": [{"json": "a", "seq": 3, "client": "c1"}],
           "headerMetadata": {"minSequenceNumber": 5, "sequenceNumber": 9, "orderedChunkMetadata": [{"id": "header"}],
                              "totalLength": 1, "totalSegmentCount": 1}}
    snaps = [parse_snapshot([json.dumps(bad)])]
    eng = engine_load(emu_engine, snaps, props)
    assert int(eng.status([0])[0]) & 0x08          # seq in (0, minSeq]: MT_DS_UNSUPPORTED


def test_quiescent_long_snapshot_load_and_continue():
    check_quiescent(emu_engine)


def check_quiescent(factory):
    """Snapshots taken at quiescence (MSN = seq) of documents longer than one chunk:
    loadBody appends the body as one batched insertSegments call; the engine then
    keeps generating + applying ops from the loaded state, which the oracle-loaded
    documents replay identically."""
    props, batch, _, _ = collab_case(seed=5, n_docs=3, ops=2600, cut=2300, clients=3, lag=32, ins=85, rem=15,
                                     ins_len=16, rem_len=6)
    snaps, blobs_l = [], []
    for d in range(3):
        od = OracleDoc(collaborating=True, props=props, names=NAMES)
        assert od.apply_run(sub_batch(batch, d, 0, 2300, 0), 0) == 0
        sq = int(batch.arrays["seq"][int(batch.op_offsets[d]) + 2299])
        blobs, _ = od.snapshot(sq, sq)
        blobs_l.append([b.decode() for b in blobs])
        snaps.append(parse_snapshot(blobs_l[-1]))
        assert snaps[-1].body, "expected body chunks"
    eng = engine_load(factory, snaps, props, extra_rows=4000, extra_text=40000)
    assert (eng.status(range(3)) == 0).all()
    ods = []
    for d in range(3):
        od, ost = oracle_load(blobs_l[d], props)
        assert ost == 0
        ed, odump = eng.dump(d), od.dump()
        assert ed.shape == odump.shape and (ed == odump).all(), f"doc {d} loaded rows"
        ods.append(od)
    p = gen_params(seed=21, n_docs=3, ops=800, clients=5, lag=12, ins=50, rem=30, ins_len=8, rem_len=12,
                   ann_sets=6, rewrite=10)
    p.continue_docs = 1
    eng.generate(p)
    eng.sync()
    assert (eng.status(range(3)) == 0).all()
    gb = eng.generated_download()
    for d in range(3):
        assert ods[d].apply_run(gb, d) == 0
        assert eng.get_text([d])[0] == ods[d].get_text()
        ed, odump = eng.dump(d), ods[d].dump()
        assert ed.shape == odump.shape and (ed == odump).all(), f"doc {d} rows after continuing"


def _doc(header, body, ms, sq):
    """Hand-built V1 snapshot blobs (snapshotV1.ts:98-163 layout)."""
    def ln(x):
        j = x["json"] if isinstance(x, dict) and "json" in x else x
        return len(j) if isinstance(j, str) else len(j.get("text", "")) or 1
    tot = header + body
    hm = {"minSequenceNumber": ms, "sequenceNumber": sq,
          "orderedChunkMetadata": [{"id": "header"}] + ([{"id": "body_0"}] if body else []),
          "totalLength": sum(ln(x) for x in tot), "totalSegmentCount": len(tot)}
    h = {"version": "1", "segmentCount": len(header), "length": sum(ln(x) for x in header), "segments": header,
         "startIndex": 0, "headerMetadata": hm}
    out = [json.dumps(h)]
    if body:
        out.append(json.dumps({"version": "1", "segmentCount": len(body), "length": sum(ln(x) for x in body),
                               "segments": body, "startIndex": len(header)}))
    return out


X = {"json": "X", "seq": 10, "client": "c1"}
XR = {"json": "X", "seq": 10, "client": "c1", "removedSeq": 11, "removedClient": "c2"}
ZR = {"json": "ZZ", "removedSeq": 8, "removedClient": "c2"}
LOADBODY_CASES = {
    # final flush re-appends "de" (falls off the NonCollab view: no-op), then "fg" falls off: throw
    "reflush_then_new": (_doc(["abc"], ["de", X, "fg"], 5, 12), 0x04),
    # final flush only re-appends "de" and falls off the tree: a clean load
    "reflush_noop": (_doc(["abc"], ["de", X], 5, 12), 0),
    # the re-appended "de" would be linked a second time (aliased object)
    "reflush_alias": (_doc(["abc"], ["de", XR], 5, 12), 0x08),
    # a removed universal segment is visible to (0, NonCollab): "de" lands before it
    "removed_in_header": (_doc(["abc", ZR], ["de"], 5, 12), 0),
    # a window insert in the header hides from (0, NonCollab): the body batch falls off
    "window_in_header": (_doc(["abc", X], ["de"], 5, 12), 0x04),
    # markers and props through the body batch
    "markers_props": (_doc(["ab"], [{"marker": {"refType": 1}, "props": {"markerId": "m1"}},
                                    {"text": "cd", "props": {"b": True, "a": [1, 2]}}, "ef"], 3, 3), 0),
}


@pytest.mark.parametrize("name", list(LOADBODY_CASES))
def test_loadbody_reference_behaviour(name):
    check_loadbody(name, emu_engine)


def check_loadbody(name, factory):
    blobs, want = LOADBODY_CASES[name]
    props = PropTable()
    od, ost = oracle_load(blobs, props)
    assert ost == want
    eng = engine_load(factory, [parse_snapshot(blobs)], props)
    assert int(eng.status([0])[0]) == want
    if want == 0:
        assert eng.get_text([0])[0] == od.get_text()
        ed, odump = eng.dump(0), od.dump()
        assert ed.shape == odump.shape and (ed == odump).all()
        (eb, _), = eng.snapshot([0], [12], [12])
        ob, _ = od.snapshot(12, 12)
        assert eb == ob
