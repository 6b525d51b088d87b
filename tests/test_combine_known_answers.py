"""Remote combining ops and options.mergeTreeSnapshotChunkSize: known answers.

Combining ops (ICombiningOp other than "rewrite", MT/ops.ts:32-37).  A remote annotate calls
SegmentPropertiesManager.addProperties (MT/segmentPropertiesManager.ts:38-113), which for a
combining op computes `Properties.combine(combiningOp, previousValue, newValue, seq)` with a
`newValue` it never assigned (:98-103), so MT/properties.ts:24-62 always combines with
undefined:
  * incr: `x += undefined` is NaN for numbers, booleans, null and undefined; NaN is not null, so
    it is stored; JSON.stringify writes it as null; and `NaN !== NaN`, so matchProperties
    (:64-95) fails on it, which stops zamboni merges (mergeTree.ts:1306-1334) and snapshot
    coalescing (snapshotV1.ts:195-213).  For a string, array or object it is string
    concatenation: String(x) + "undefined" ("v" -> "vundefined", [1, [2, "x"]] ->
    "1,2,xundefined", {} -> "[object Object]undefined"), which a truthy string / array / object
    minValue replaces when it compares above it (:35-38);
  * consensus: a key without a value becomes {value: undefined, seq} (JSON {"seq":seq}, never
    equal: its `value` is undefined); a defaultValue whose seq is -1 gets the op's seq; any
    other held value is kept; a null defaultValue on a key without a value throws (null.seq:
    the engine's MT_DS_THROWS, a TypeError from the hosts);
  * any other name: the held value or the defaultValue (undefined included: the key is
    present with value undefined, skipped by JSON.stringify, never equal).
The expected texts below are those rules worked by hand; the oracle (oracle/mtoracle.cpp
js_combine) must produce them, and the engine must equal the oracle byte for byte.

mergeTreeSnapshotChunkSize (snapshotV1.ts:55, :70-114): SnapshotV1 closes a chunk once its
length reaches the size; sizes 100 / 1,000 / 25,000 against the oracle and the chunk rule.
"""
import json

import numpy as np
import pytest

from emu_lib import emu_engine
from fluidframework_amd.engine import ClientGroup, Engine, MergeTreeError, snapshot_chunk_option
from oracle_lib import OracleDoc

UNSUPPORTED = 0x08
THROWS = 0x4000
LIMITS = dict(rows_per_doc=8192, window_per_doc=4096, propsets_per_doc=8192, text_per_doc=1 << 16)


def msg(seq, ref, msn, contents, client="a"):
    return dict(clientId=client, sequenceNumber=seq, referenceSequenceNumber=ref, minimumSequenceNumber=msn,
                type="op", contents=contents)


def ins(pos, seg):
    return {"type": 0, "pos1": pos, "seg": seg}


def ann(p1, p2, props, cop=None):
    o = {"type": 2, "pos1": p1, "pos2": p2, "props": props}
    if cop is not None:
        o["combiningOp"] = cop
    return o


def rem(p1, p2):
    return {"type": 1, "pos1": p1, "pos2": p2}


def stream_of(ops, msn_lag=10 ** 9):
    """Messages seq 1.. of one client, refSeq = seq - 1, MSN trailing by msn_lag."""
    return [msg(i + 1, i, max(0, i - msn_lag), op) for i, op in enumerate(ops)]


def body_props(blobs):
    """The props JSON texts of every segment of a SnapshotV1, in order (None: no props)."""
    out = []
    for b in blobs:
        for s in json.loads(b)["segments"]:
            j = s["json"] if isinstance(s, dict) and "json" in s else s
            out.append(json.dumps(j.get("props"), separators=(",", ":")) if isinstance(j, dict) else None)
    return out


def props_texts(blobs):
    """The raw `"props":{...}` texts of a snapshot (as the bytes hold them: NaN is null)."""
    import re
    return re.findall(r'"props":(\{[^{}]*(?:\{[^{}]*\}[^{}]*)*\})', b"".join(blobs).decode())


# Known answers: (name, ops, expected props texts in snapshot order or expected status)
CASES = [
    # incr without a default on an absent key: NaN (JSON null)
    ("incr_absent", [ins(0, "abc"), ann(0, 3, {"k": 7}, {"name": "incr"})], ['{"k":null}']),
    # incr on held numbers and booleans, a default of 5 and a minValue: all NaN (NaN < 3 is false)
    ("incr_held", [ins(0, {"text": "ab", "props": {"x": 2, "y": True}}),
                   ann(0, 2, {"x": None, "y": 1, "z": 0}, {"name": "incr", "defaultValue": 5, "minValue": 3})],
     ['{"x":null,"y":null,"z":null}']),
    # consensus on an absent key: {value: undefined, seq: 2} -> {"seq":2}; a held value is kept
    ("consensus_fresh", [ins(0, {"text": "ab", "props": {"h": "keep"}}),
                         ann(0, 2, {"c": 1, "h": 2}, {"name": "consensus"})], ['{"h":"keep","c":{"seq":2}}']),
    # a consensus default whose seq is -1 takes the op's seq, key order kept
    ("consensus_default_seq", [ins(0, "ab"), ann(0, 2, {"c": 0}, {"name": "consensus",
                                                                  "defaultValue": {"value": 3, "seq": -1, "w": 1}})],
     ['{"c":{"value":3,"seq":2,"w":1}}']),
    ("consensus_default_plain", [ins(0, "ab"), ann(0, 2, {"c": 0}, {"name": "consensus", "defaultValue": [1, "x"]})],
     ['{"c":[1,"x"]}']),
    # another name: no case in combine's switch; no default -> the key holds undefined (omitted
    # by JSON.stringify), a null default deletes it, another default is stored
    ("other_undefined", [ins(0, {"text": "ab", "props": {"h": 1}}), ann(0, 2, {"u": 9}, {"name": "max"})],
     ['{"h":1}']),
    ("other_null_default", [ins(0, {"text": "ab", "props": {"h": 1, "d": 2}}),
                            ann(0, 2, {"d": 0, "e": 0}, {"name": "max", "defaultValue": None})], ['{"h":1,"d":2}']),
    ("other_default", [ins(0, "ab"), ann(0, 2, {"d": 0}, {"name": 5, "defaultValue": {"z": [True]}})],
     ['{"d":{"z":[true]}}']),
    # NaN maps never match: two segments annotated by one incr do not coalesce in the snapshot
    # even at the MSN, where equal plain maps do (the control case)
    ("nan_blocks_coalesce", [ins(0, "ab"), ins(2, "cd"), ann(0, 4, {"k": 1}, {"name": "incr"}),
                             ins(4, "e")], ['{"k":null}', '{"k":null}']),
    ("plain_coalesces", [ins(0, "ab"), ins(2, "cd"), ann(0, 4, {"k": 1}), ins(4, "e")], ['{"k":1}']),
    # a segment split after its incr keeps one NaN map in both halves (the engine shares the
    # map; the reference copies it): zamboni must not merge the halves back
    ("nan_split_halves", [ins(0, "abcd"), ann(0, 4, {"k": 1}, {"name": "incr"}), ins(2, "X"), rem(2, 3),
                          ins(4, "z")], ['{"k":null}', '{"k":null}']),
    ("undefined_split_halves", [ins(0, "abcd"), ann(0, 4, {"u": 1}, {"name": "other"}), ins(2, "X"), rem(2, 3),
                                ins(4, "z")], ['{}', '{}']),
    # incr of a string, array or object: string concatenation with "undefined"
    ("incr_string", [ins(0, {"text": "ab", "props": {"s": "v"}}), ann(0, 2, {"s": 1}, {"name": "incr"})],
     ['{"s":"vundefined"}']),
    ("incr_string_twice", [ins(0, {"text": "ab", "props": {"s": "v"}}), ann(0, 2, {"s": 1}, {"name": "incr"}),
                           ann(0, 1, {"s": 1}, {"name": "incr"})], ['{"s":"vundefinedundefined"}', '{"s":"vundefined"}']),
    ("incr_string_default", [ins(0, "ab"), ann(0, 2, {"s": 1}, {"name": "incr", "defaultValue": "v"})],
     ['{"s":"vundefined"}']),
    ("incr_held_object_array", [ins(0, {"text": "ab", "props": {"o": {"a": 1}, "r": [1, [2, "x"], None]}}),
                                ann(0, 2, {"o": 0, "r": 0}, {"name": "incr"})],
     ['{"o":"[object Object]undefined","r":"1,2,x,undefined"}']),
    ("incr_default_array", [ins(0, "ab"), ann(0, 2, {"a": 0}, {"name": "incr", "defaultValue": [1, 2]})],
     ['{"a":"1,2undefined"}']),
    ("incr_fresh_consensus", [ins(0, "ab"), ann(0, 2, {"c": 1}, {"name": "consensus"}),
                              ann(0, 2, {"c": 1}, {"name": "incr"})], ['{"c":"[object Object]undefined"}']),
    # a truthy string minValue above the default's result replaces it ("zzz" > "vundefined");
    # one below it does not; a number minValue never does (NaN comparison)
    ("incr_default_min_above", [ins(0, "ab"), ann(0, 2, {"s": 1}, {"name": "incr", "defaultValue": "v",
                                                                  "minValue": "zzz"})], ['{"s":"zzz"}']),
    ("incr_default_min_below", [ins(0, "ab"), ann(0, 2, {"s": 1}, {"name": "incr", "defaultValue": "v",
                                                                  "minValue": "a"})], ['{"s":"vundefined"}']),
    ("incr_default_min_number", [ins(0, "ab"), ann(0, 2, {"s": 1}, {"name": "incr", "defaultValue": "v",
                                                                   "minValue": 9})], ['{"s":"vundefined"}']),
    # another name keeps a held object whose seq is -1 (only consensus writes into it)
    ("other_held_seq_minus1", [ins(0, {"text": "ab", "props": {"c": {"seq": -1}}}), ann(0, 2, {"c": 1}, {"name": "max"})],
     ['{"c":{"seq":-1}}']),
    # the reference throws (null.seq): MT_DS_THROWS
    ("consensus_null_default", [ins(0, "ab"), ann(0, 2, {"c": 1}, {"name": "consensus", "defaultValue": None})],
     THROWS),
    # off the batch path (MT_DS_UNSUPPORTED): consensus writing into a held object whose seq is -1
    # (every segment split from it shares it), and a held string's incr result that a string
    # minValue would be compared with
    ("consensus_held_seq_minus1", [ins(0, {"text": "ab", "props": {"c": {"seq": -1}}}),
                                   ann(0, 2, {"c": 1}, {"name": "consensus"})], UNSUPPORTED),
    ("incr_held_string_min", [ins(0, {"text": "ab", "props": {"s": "v"}}),
                              ann(0, 2, {"s": 1}, {"name": "incr", "minValue": "zzz"})], UNSUPPORTED),
]


def run_engine(factory, msgs, options=None):
    g = ClientGroup(factory(1, **LIMITS))
    c = g.new_client(options or {"newMergeTreeSnapshotFormat": True})
    for m in msgs:
        c.applyMsg(m)
    g.flush()
    return g, c


@pytest.mark.parametrize("name,ops,want", CASES, ids=[c[0] for c in CASES])
def test_combine_known_answers_oracle(name, ops, want):
    """The oracle's restatement gives the hand-worked answers (MSN at the last message)."""
    msgs = stream_of(ops, msn_lag=0)
    o = OracleDoc(True)
    st = 0
    for m in msgs:
        st |= o.apply_msg(m)
    if isinstance(want, int):
        assert st & want
        return
    assert st == 0
    blobs, _ = o.snapshot(msgs[-1]["minimumSequenceNumber"], msgs[-1]["sequenceNumber"])
    assert props_texts(blobs) == want


def check_engine_case(factory, ops, want):
    msgs = stream_of(ops, msn_lag=0)
    g, _ = run_engine(factory, msgs)
    st = int(g.engine.status([0])[0])
    if isinstance(want, int):
        assert st & want, st
        return
    assert st == 0, st
    o = OracleDoc(True)
    for m in msgs:
        assert o.apply_msg(m) == 0
    ed, od = g.engine.dump(0), o.dump()
    assert ed.shape == od.shape and (ed[:, [0, 1, 3, 7, 8, 9, 10, 11]] == od[:, [0, 1, 3, 7, 8, 9, 10, 11]]).all()
    msn, seq = msgs[-1]["minimumSequenceNumber"], msgs[-1]["sequenceNumber"]
    for legacy in (True, False):
        (eb, edig), = g.engine.snapshot([0], [msn], [seq], legacy=legacy)
        ob, odig = o.snapshot(msn, seq, legacy=legacy)
        assert eb == ob and edig == odig
    assert props_texts(eb) == want                     # SnapshotV1


@pytest.mark.parametrize("name,ops,want", CASES, ids=[c[0] for c in CASES])
def test_combine_known_answers_on_emulation(name, ops, want):
    check_engine_case(emu_engine, ops, want)


@pytest.mark.gpu
@pytest.mark.parametrize("name,ops,want", CASES, ids=[c[0] for c in CASES])
def test_combine_known_answers_on_gpu(name, ops, want):
    check_engine_case(lambda n, **kw: Engine(n, device=0, **kw), ops, want)


def test_zamboni_keeps_nan_segments_apart_on_emulation():
    """The split halves of one NaN segment stay two rows after zamboni (rows, not just the
    snapshot): the reference's copies never matchProperties-match."""
    ops = CASES[[c[0] for c in CASES].index("nan_split_halves")][1]
    g, _ = run_engine(emu_engine, stream_of(ops, msn_lag=0))
    o = OracleDoc(True)
    for m in stream_of(ops, msn_lag=0):
        o.apply_msg(m)
    ed, od = g.engine.dump(0), o.dump()
    assert len(ed) == len(od)
    assert (ed[:, 0] == 2).sum() == (od[:, 0] == 2).sum() == 2     # "ab" and "cd" stay two segments


def test_packers_emit_no_unsupported_for_combining_ops():
    """incr / consensus / other names pack as combine sets (MT_OPF_COMBINE), not as
    MT_OP_UNSUPPORTED records."""
    from fluidframework_amd.batch import (MT_OP_ANNOTATE, MT_OPF_COMBINE, MT_OPF_REWRITE, MT_VAL_CFRESH, MT_VAL_NAN,
                                          MT_VAL_UNDEF, BatchBuilder, ClientNames, PropTable)
    pt = PropTable()
    bb = BatchBuilder(pt, ClientNames())
    bb.begin_doc(0)
    for i, cop in enumerate([{"name": "incr"}, {"name": "consensus"}, {"name": "max"}, True]):
        bb.add_message(msg(i + 1, i, 0, ann(0, 1, {"k": 1}, cop)))
    b = bb.build()
    assert (b.arrays["type"] == MT_OP_ANNOTATE).all()
    fl = b.arrays["flags"]
    assert fl[0] & MT_OPF_COMBINE and not fl[0] & MT_OPF_REWRITE
    assert all(f & MT_OPF_COMBINE and f & MT_OPF_REWRITE for f in fl[1:])
    codes = [pt.sets[int(p)][0][1] for p in b.arrays["prop_id"]]
    assert codes == [MT_VAL_NAN, MT_VAL_CFRESH, MT_VAL_UNDEF, MT_VAL_UNDEF]


# ---- options.mergeTreeSnapshotChunkSize -------------------------------------------------------
def chunk_doc(n_segs=600, seed=3):
    """One client's stream of n_segs appended segments of 1..60 units that never coalesce
    (alternating property maps)."""
    rng = np.random.default_rng(seed)
    ops, L = [], 0
    for i in range(n_segs):
        n = int(rng.integers(1, 61))
        ops.append(ins(L, {"text": "x" * n, "props": {"p": i % 2}}))
        L += n
    return stream_of(ops, msn_lag=0), L


@pytest.mark.parametrize("size", [100, 1000, 25000, 0.5, 99.5, "300"])
def test_snapshot_chunk_size_oracle_rule(size):
    """The oracle's chunks follow getSeqLengthSegs (snapshotV1.ts:70-92): each chunk takes
    segments until its length reaches the size; the header lists every body chunk."""
    msgs, total = chunk_doc()
    o = OracleDoc(True)
    o.set_snapshot_chunk(float(size))
    for m in msgs:
        o.apply_msg(m)
    blobs, _ = o.snapshot(msgs[-1]["minimumSequenceNumber"], msgs[-1]["sequenceNumber"])
    chunks = [json.loads(b) for b in blobs]
    sz = float(size)
    assert sum(c["length"] for c in chunks) == total
    for c in chunks[:-1]:
        lens = [len((s["json"] if "json" in s else s)["text"]) for s in c["segments"]]
        assert sum(lens) >= sz and sum(lens[:-1]) < sz
    assert len(chunks[0]["headerMetadata"]["orderedChunkMetadata"]) == len(chunks)


def check_chunk_sizes(factory):
    msgs, _ = chunk_doc()
    msn, seq = msgs[-1]["minimumSequenceNumber"], msgs[-1]["sequenceNumber"]
    for size in (100, 1000, 25000, 99.5, "300", float("inf")):
        g, c = run_engine(factory, msgs, {"newMergeTreeSnapshotFormat": True, "mergeTreeSnapshotChunkSize": size})
        o = OracleDoc(True)
        o.set_snapshot_chunk(float(size))
        for m in msgs:
            o.apply_msg(m)
        ob, odig = o.snapshot(msn, seq)
        (eb, edig), = g.engine.snapshot([0], [msn], [seq])
        assert eb == ob and edig == odig, size
        assert g.engine.snapshot_digests([0], [msn], [seq])[0] == odig
        tree = c.snapshot()
        assert [e["value"]["contents"].encode() for e in tree["entries"]] == ob
        if size == 100:
            assert len(ob) > 100
        if size == float("inf"):
            assert len(ob) == 1


def test_snapshot_chunk_sizes_on_emulation():
    check_chunk_sizes(emu_engine)


@pytest.mark.gpu
def test_snapshot_chunk_sizes_on_gpu():
    check_chunk_sizes(lambda n, **kw: Engine(n, device=0, **kw))


def test_snapshot_chunk_option_values():
    """The option as the reference's `length < chunkSize` sees it: JS ToNumber (jsjson.js_to_number)."""
    from fluidframework_amd.engine import MT_CHUNK_INFINITY, MT_CHUNK_NONE
    opt = lambda v: snapshot_chunk_option({"mergeTreeSnapshotChunkSize": v})
    assert snapshot_chunk_option(None) == 0 and snapshot_chunk_option({}) == 0
    assert opt(None) == 0                                                 # `?? SnapshotV1.chunkSize`
    assert opt(100) == 100 and opt(99.2) == 100 and opt("7") == 7 and opt(" 7 ") == 7
    assert opt(float("inf")) == MT_CHUNK_INFINITY and opt("Infinity") == MT_CHUNK_INFINITY
    assert opt(True) == 1 and opt([100]) == 100 and opt("0x10") == 16 and opt("1e3") == 1000
    for none in (0, -5, float("nan"), "abc", False, [], [1, 2], {}, "1_000", "inf", "", "-Infinity"):
        assert opt(none) == MT_CHUNK_NONE, none


def legacy_chunk_case(factory, size, n_segs=300):
    """SnapshotLegacy's header chunk is cut at the option (snapshotlegacy.ts:71, :109)."""
    from fluidframework_amd.jsjson import js_to_number
    msgs, _ = chunk_doc(n_segs)
    msn, seq = msgs[-1]["minimumSequenceNumber"], msgs[-1]["sequenceNumber"]
    opts = {"newMergeTreeSnapshotFormat": False}
    if size is not None:
        opts["mergeTreeSnapshotChunkSize"] = size
    g, c = run_engine(factory, msgs, opts)
    o = OracleDoc(True)
    if size is not None:
        o.set_snapshot_chunk(js_to_number(size))
    for m in msgs:
        o.apply_msg(m)
    ob, odig = o.snapshot(msn, seq, legacy=True)
    (eb, edig), = g.engine.snapshot([0], [msn], [seq], legacy=True)
    assert eb == ob and edig == odig, size
    tree = c.snapshot()
    assert [e["value"]["contents"].encode() for e in tree["entries"]] == ob
    return [json.loads(b) for b in ob]


LEGACY_SIZES = [None, 100, 1000, 99.5, "300", float("inf"), 0, -3, float("nan"), "abc", [250], True]


@pytest.mark.parametrize("size", LEGACY_SIZES, ids=[repr(s) for s in LEGACY_SIZES])
def test_legacy_chunk_size_on_emulation(size):
    ch = legacy_chunk_case(emu_engine, size)
    head = ch[0]
    if size in (0, -3, "abc", True) or (isinstance(size, float) and size != size):
        assert head["chunkSegmentCount"] <= (1 if size is True else 0)
        assert len(ch) == 2 and ch[1]["chunkSegmentCount"] == head["totalSegmentCount"] - head["chunkSegmentCount"]
    if size == float("inf"):
        assert len(ch) == 1


@pytest.mark.gpu
def test_legacy_chunk_size_on_gpu():
    for size in LEGACY_SIZES:
        legacy_chunk_case(lambda n, **kw: Engine(n, device=0, **kw), size)


def v1_no_length_below_case(factory):
    """SnapshotV1 with a size no length is below: the reference's chunk loop never ends on a
    non-empty document (an error here, at snapshot time, not at client creation); an empty
    document gives its one empty chunk, as the reference's do/while does."""
    msgs, _ = chunk_doc(50)
    msn, seq = msgs[-1]["minimumSequenceNumber"], msgs[-1]["sequenceNumber"]
    g, c = run_engine(factory, msgs, {"newMergeTreeSnapshotFormat": True, "mergeTreeSnapshotChunkSize": 0})
    with pytest.raises(MergeTreeError, match="chunk loop"):
        g.engine.snapshot([0], [msn], [seq])
    with pytest.raises(MergeTreeError, match="chunk loop"):
        g.engine.snapshot_digests([0], [msn], [seq])
    o = OracleDoc(True)
    o.set_snapshot_chunk(0.0)
    for m in msgs:
        o.apply_msg(m)
    with pytest.raises(RuntimeError):
        o.snapshot(msn, seq)
    g2 = ClientGroup(factory(1, **LIMITS))
    g2.new_client({"newMergeTreeSnapshotFormat": True, "mergeTreeSnapshotChunkSize": "none"})
    e = OracleDoc(True)
    e.set_snapshot_chunk(float("nan"))
    (eb, edig), = g2.engine.snapshot([0], [0], [0])
    assert (eb, edig) == e.snapshot(0, 0)


def test_v1_no_length_below_on_emulation():
    v1_no_length_below_case(emu_engine)


@pytest.mark.gpu
def test_v1_no_length_below_on_gpu():
    v1_no_length_below_case(lambda n, **kw: Engine(n, device=0, **kw))


def test_reopened_document_resets_chunk_size_on_emulation():
    """mt_docs_open gives the document a new Client's default chunk size."""
    msgs, _ = chunk_doc(200)
    eng = emu_engine(1, **LIMITS)
    eng.set_snapshot_chunk([0], [100])
    g = ClientGroup(eng)
    c = g.new_client({"newMergeTreeSnapshotFormat": True})      # opens document 0 again
    for m in msgs:
        c.applyMsg(m)
    g.flush()
    o = OracleDoc(True)
    for m in msgs:
        o.apply_msg(m)
    msn, seq = msgs[-1]["minimumSequenceNumber"], msgs[-1]["sequenceNumber"]
    assert eng.snapshot([0], [msn], [seq])[0][0] == o.snapshot(msn, seq)[0]


def check_node_chunk_and_combine(addon):
    from js_lib import run_node
    from msg_gen import stream
    msgs, _ = chunk_doc(300)
    got = run_node([msgs], addon=addon, options={"newMergeTreeSnapshotFormat": True, "mergeTreeSnapshotChunkSize": 250})
    o = OracleDoc(True)
    o.set_snapshot_chunk(250)
    for m in msgs:
        o.apply_msg(m)
    blobs, _ = o.snapshot(msgs[-1]["minimumSequenceNumber"], msgs[-1]["sequenceNumber"])
    assert [b for _, b in got["blobs"][0]] == [b.decode() for b in blobs]
    assert len(blobs) > 20
    # the reference's default format (SnapshotLegacy): its header chunk is cut at the option,
    # after ToNumber ([250] is 250; 0 leaves the header chunk empty)
    for size, num in (([250], 250.0), (0, 0.0)):
        got = run_node([msgs], addon=addon, options={"mergeTreeSnapshotChunkSize": size})
        o = OracleDoc(True)
        o.set_snapshot_chunk(num)
        for m in msgs:
            o.apply_msg(m)
        blobs, _ = o.snapshot(msgs[-1]["minimumSequenceNumber"], msgs[-1]["sequenceNumber"], legacy=True)
        assert [b for _, b in got["blobs"][0]] == [b.decode() for b in blobs], size
        assert len(blobs) == 2


def test_node_host_chunk_size_on_emulation():
    from js_lib import NODE
    from emu_lib import build_emu_napi
    if NODE is None:
        pytest.skip("node is not installed")
    check_node_chunk_and_combine(build_emu_napi())


@pytest.mark.gpu
def test_node_host_chunk_size_on_gpu():
    import os
    from js_lib import NODE, ROOT
    if NODE is None:
        pytest.skip("node is not installed")
    check_node_chunk_and_combine(os.path.join(ROOT, "fluidframework_amd", "js", "mtgpu.node"))


def consensus_null_case():
    return stream_of(dict((c[0], c[1]) for c in CASES)["consensus_null_default"], msn_lag=0)


def test_consensus_null_default_throws_a_type_error_on_emulation():
    """Where the reference's applyMsg throws (null.seq, properties.ts:51-52) the Python host
    raises a TypeError too (MT_DS_THROWS), not an "unsupported input"."""
    from fluidframework_amd.engine import ReferenceTypeError
    g, c = run_engine(emu_engine, consensus_null_case())
    assert int(g.engine.status([0])[0]) == THROWS
    with pytest.raises(TypeError, match="Cannot read property 'seq' of null"):
        c.getText()
    with pytest.raises(ReferenceTypeError):
        c.snapshot()


def test_consensus_null_default_throws_a_type_error_in_node_on_emulation(tmp_path):
    """The Node host throws the reference's TypeError."""
    import os
    import subprocess
    from js_lib import NODE, ROOT
    from emu_lib import build_emu_napi
    if NODE is None:
        pytest.skip("node is not installed")
    addon = build_emu_napi()
    script = tmp_path / "t.js"
    script.write_text(
        "const mt = require(process.argv[2]);\n"
        "const g = new mt.ClientGroup(new mt.Engine(1, {}));\n"
        "const c = g.newClient({ newMergeTreeSnapshotFormat: true });\n"
        f"for (const m of {json.dumps(consensus_null_case())}) c.applyMsg(m);\n"
        "try { c.getText(); console.log('no throw'); }\n"
        "catch (e) { console.log((e instanceof TypeError ? 'TypeError: ' : 'Error: ') + e.message); }\n")
    r = subprocess.run([NODE, str(script), os.path.join(ROOT, "fluidframework_amd", "js")], capture_output=True,
                       text=True, env=dict(os.environ, MTGPU_NAPI=addon), timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("TypeError: ") and "Cannot read property 'seq' of null" in r.stdout, r.stdout


def key_limit_case(factory):
    """A map of MT_MAX_PROP_KEYS (256) keys replays equal to the oracle (segment props past a
    wave's 64 lanes: applyPropSetWide); one key more sets MT_DS_PROPS_TOO_MANY."""
    full = {f"k{i}": i for i in range(256)}
    ops = [ins(0, {"text": "ab", "props": {f"k{i}": i for i in range(100)}}), ins(2, "cd"),
           ann(0, 4, {f"k{i}": -i for i in range(60, 256)}), ann(1, 3, {"k5": None, "k200": None}),
           ann(0, 4, {"k5": 1, "k200": 2}, {"name": "rewrite"}), ann(2, 4, full)]
    check_engine_case(factory, ops, props_texts(_oracle_blobs(ops)))
    g, _ = run_engine(factory, stream_of([ins(0, {"text": "x", "props": {**full, "one_more": 1}})], msn_lag=0))
    assert int(g.engine.status([0])[0]) & 0x400


def _oracle_blobs(ops):
    msgs = stream_of(ops, msn_lag=0)
    o = OracleDoc(True)
    for m in msgs:
        assert o.apply_msg(m) == 0
    return o.snapshot(msgs[-1]["minimumSequenceNumber"], msgs[-1]["sequenceNumber"])[0]


def test_prop_key_limit_on_emulation():
    key_limit_case(emu_engine)


@pytest.mark.gpu
def test_prop_key_limit_on_gpu():
    key_limit_case(lambda n, **kw: Engine(n, device=0, **kw))
