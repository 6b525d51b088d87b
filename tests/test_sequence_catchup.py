"""§8(f2): SharedSegmentSequence's legacy catch-up path (sequence.ts:592-658) on the engine.

For a channel's op stream (the other channels' messages leave seq gaps, so many messages
have refSeq != seq - 1), fluidframework_amd.sequence.SequenceDoc stashes every message,
transforming the ones that need it from the engine's sequenceDelta records
(createOpsFromDelta, sequence.ts:58-105), and writes SnapshotLegacy + catch-up blob.

* The whole tree equals the one computed from the ORACLE's records of the same stream
  (ora_delta_json: the oracle's own callback restatement) with the same stash rules, and
  its header/body blobs equal the oracle's SnapshotLegacy bytes.
* The property the transformation exists for (sequence.ts:612-631): loading the legacy
  snapshot and applying the catch-up messages on the oracle (SnapshotLoader +
  Client.applyMsg, its own JSON path) reproduces the document's text and length.
* createOpsFromDelta known answers written out from sequence.ts:58-105 and
  segmentPropertiesManager.ts:67-112 (remove/annotate coalescing, rewrite delta keys).
"""
import json
import os

import pytest

from emu_lib import build_emu_napi, emu_engine
from fluidframework_amd import jsjson
from fluidframework_amd import sequence as sq
from fluidframework_amd.engine import ClientGroup, Engine
from js_lib import NODE, ROOT, run_driver
from msg_gen import stream
from oracle_lib import OracleDoc
from test_message_surface import LIMITS, SURFACES

GPU = lambda n, **kw: Engine(n, device=0, **kw)  # noqa: E731


def channel_stream(seed: int, n: int, surface: str) -> list:
    """The sequenced ops of one channel: the stream's non-op messages stand for other
    channels' traffic (they reach the delta manager, not the DDS)."""
    kw = dict(SURFACES[surface])
    if kw.get("p_register"):
        # A paste's length depends on which merges zamboni made before the copy (cloneSegments
        # clones whole segments), and zamboni runs when the MSN moves: a register stream is only
        # valid for a channel that sees every MSN update the generator's observer saw.
        kw["p_nonop"] = 0.0
    msgs, _ = stream(seed, n, **kw)
    return [m for m in msgs if m["type"] == "op"]


def oracle_tree(msgs: list):
    """(oracle doc, expected catch-up blob text or None, msn, seq): the oracle's own
    processMergeTreeMsg / createOpsFromDelta / snapshotMergeTree restatement
    (ora_channel_process, oracle/mtoracle.cpp), independent of the product's transformation."""
    od = OracleDoc(True)
    for m in msgs:
        assert od.channel_process(m) == 0, m
    msn, seq = msgs[-1]["minimumSequenceNumber"], msgs[-1]["sequenceNumber"]
    return od, od.channel_stash(msn), msn, seq


def run_channels(factory, surface: str, n_docs: int = 3, n_msgs: int = 700, flush_every: int = 97):
    """Stash/blob parity on every surface; the load + catch-up replay property on those
    without relative positions: a live document resolves a relativePos against a marker
    that was removed (idToSegment keeps it), but SnapshotLegacy writes only the segments
    live at the MSN, so in the reference too an untransformed catch-up op naming a marker
    removed at or below the MSN no longer resolves after a load."""
    # Registers are not part of a snapshot either (RegisterCollection lives only in the
    # Client), so a stashed paste whose copy precedes the snapshot pastes nothing after a load.
    replay = not SURFACES[surface].get("p_relative") and not SURFACES[surface].get("p_register")
    chans = [channel_stream(17 * d + 3, n_msgs, surface) for d in range(n_docs)]
    eng = factory(n_docs, **LIMITS)
    g = ClientGroup(eng)
    docs = [sq.SequenceDoc(g) for _ in range(n_docs)]
    for k in range(max(len(c) for c in chans)):
        for d, c in zip(docs, chans):
            if k < len(c):
                d.process(c[k])
        if k % flush_every == flush_every - 1:
            g.flush()                                  # several device batches per stream
    transformed, in_stash, pastes = 0, 0, 0
    for d, msgs in zip(docs, chans):
        tree = d.snapshot()
        blobs = {e["path"]: e["value"]["contents"] for e in tree["entries"]}
        od, want, msn, seq = oracle_tree(msgs)
        moved = [m["sequenceNumber"] for m in msgs if m["referenceSequenceNumber"] != m["sequenceNumber"] - 1]
        transformed += len(moved)
        pastes += sum(1 for m in msgs if m["referenceSequenceNumber"] != m["sequenceNumber"] - 1
                      and m["sequenceNumber"] > msn and any(_is_paste(x) for x in _members(m["contents"])))
        in_stash += sum(s > msn for s in moved)
        # the stash, byte for byte (JSON.stringify order), and the legacy blobs
        assert blobs.get("catchupOps") == want
        ob, _ = od.snapshot(msn, seq, legacy=True)
        assert [blobs["header"].encode()] + ([blobs["body"].encode()] if "body" in blobs else []) == ob
        assert od.get_text() == d.getText()
        if not replay:
            continue
        # load + catch-up reproduces the document
        ld = OracleDoc(False)
        assert ld.load_snapshot([blobs["header"]] + ([blobs["body"]] if "body" in blobs else [])) == 0
        for m in json.loads(blobs.get("catchupOps", "[]")):
            assert ld.apply_msg(m) == 0, m
        # text and length, as snapshot.spec.ts:62-77 checks.  Properties are not part of
        # the guarantee: SnapshotLegacy writes each segment's *current* properties
        # (snapshotlegacy.ts:221), and createOpsFromDelta sizes an annotate range by
        # segment.cachedLength even for a segment the observer no longer sees (removed by a
        # concurrent op), so the rebuilt annotate spans visible characters the original did
        # not touch -- the engine reproduces that byte for byte (the stash check above).
        assert ld.get_text() == od.get_text() == d.getText()
        assert ld.get_length() == od.get_length()
    if SURFACES[surface].get("p_register"):
        assert pastes > 0, "no transformed register paste reached the stash"
    return transformed, in_stash


def _members(c):
    return c.get("ops", []) if c.get("type") == 3 else [c]


def _is_paste(op):        # an insert from a register (no seg, no end position: MT/client.ts:425-444)
    return op.get("type") == 0 and "register" in op and "seg" not in op and not op.get("pos2")


ALL_SURFACES = ["mixed", "groups", "markers_props", "unicode", "churn", "relative", "churn300", "registers"]


@pytest.mark.parametrize("surface", ALL_SURFACES)
def test_catchup_on_emulation(surface):
    moved, in_stash = run_channels(emu_engine, surface)
    assert moved > 300 and in_stash > 0


@pytest.mark.gpu
@pytest.mark.parametrize("surface", ALL_SURFACES)
def test_catchup_on_gpu(surface):
    moved, in_stash = run_channels(GPU, surface, n_docs=6)
    assert moved > 600 and in_stash > 0


JS_LIMITS = dict(rowsPerDoc=30000, windowPerDoc=8192, propsetsPerDoc=30000, textPerDoc=1 << 19, blocksPerDoc=16384,
                 heapPerDoc=30000)


def check_node_channels(addon, n_per_surface=2):
    """The Node host's SequenceChannel (processCore / snapshotMergeTree through the
    reference-signature Client.snapshot / loadCore through Client.load over an
    IChannelStorageService) against the oracle-derived tree, and the loaded channel's text."""
    surf = ["mixed", "markers_props", "groups", "registers", "churn300"]
    chans = [channel_stream(29 * d + i, 600, s) for i, s in enumerate(surf) for d in range(n_per_surface)]
    kinds = [s for s in surf for _ in range(n_per_surface)]
    got = run_driver("channel_check.js", {"channels": chans, "flushEvery": 89, "limits": JS_LIMITS}, addon=addon)
    for d, msgs in enumerate(chans):
        od, want, msn, seq = oracle_tree(msgs)
        blobs = dict(got["trees"][d])
        assert blobs.get("catchupOps") == want, f"channel {d} catch-up"
        ob, _ = od.snapshot(msn, seq, legacy=True)
        assert [blobs["header"].encode()] + ([blobs["body"].encode()] if "body" in blobs else []) == ob
        assert got["texts"][d] == od.get_text(), f"channel {d} text"
        if not SURFACES[kinds[d]].get("p_register"):        # registers do not survive a load
            assert got["loaded"][d] == od.get_text(), f"channel {d} loaded text"


@pytest.mark.skipif(NODE is None, reason="node is not installed")
def test_node_channel_on_emulation():
    check_node_channels(build_emu_napi())


@pytest.mark.gpu
@pytest.mark.skipif(NODE is None, reason="node is not installed")
def test_node_channel_on_gpu():
    check_node_channels(os.path.join(ROOT, "fluidframework_amd", "js", "mtgpu.node"), n_per_surface=4)


def test_python_channel_load_and_continue():
    """SequenceDoc.load (loadCore): the legacy tree loads, its catch-up ops apply through
    processMergeTreeMsg, and the channel then takes the rest of the stream."""
    msgs = channel_stream(41, 900, "mixed")
    cut = 500
    g = ClientGroup(emu_engine(2, **LIMITS))
    a = sq.SequenceDoc(g)
    for m in msgs[:cut]:
        a.process(m)
    tree = a.snapshot()
    b = sq.SequenceDoc(g, longClientId="loader")
    b.load({e["path"]: e["value"]["contents"] for e in tree["entries"]})
    for m in msgs[cut:]:
        b.process(m)
    od, want, msn, seq = oracle_tree(msgs)
    assert b.getText() == od.get_text()
    blobs = {e["path"]: e["value"]["contents"] for e in b.snapshot()["entries"]}
    assert blobs.get("catchupOps") == want


def test_new_format_keeps_no_stash():
    eng = emu_engine(1, **LIMITS)
    d = sq.SequenceDoc(ClientGroup(eng), {"newMergeTreeSnapshotFormat": True})
    for m in channel_stream(5, 200, "mixed"):
        d.process(m)
    tree = d.snapshot()
    assert d.messagesSinceMSNChange == []
    assert [e["path"] for e in tree["entries"]][0] == "header"
    assert all(not e["path"].startswith("catchup") for e in tree["entries"])


def test_non_op_message_rejected():
    d = sq.SequenceDoc(ClientGroup(emu_engine(1, **LIMITS)))
    with pytest.raises(ValueError):
        d.process(dict(clientId="a", sequenceNumber=1, referenceSequenceNumber=0, minimumSequenceNumber=0,
                       type="noop", contents=None))


# ---- createOpsFromDelta known answers (sequence.ts:58-105) -----------------------------
def R(kind, pos, ln, before=None, after=None):
    return {"kind": kind, "pos": pos, "len": ln, "before": before, "after": after}


def test_remove_ranges_coalesce_on_equal_start():
    # removed segments collapse to the position of the first: each later range starts there
    ops = sq.ops_from_delta({"type": 1, "pos1": 3, "pos2": 9}, [R(1, 3, 2), R(1, 3, 4), R(1, 5, 1)])
    assert ops == [{"pos1": 3, "pos2": 9, "type": 1}, {"pos1": 5, "pos2": 6, "type": 1}]


def test_annotate_ranges_coalesce_when_adjacent_and_matching():
    m = {"type": 2, "pos1": 0, "pos2": 9, "props": {"b": 1}}
    ops = sq.ops_from_delta(m, [R(2, 0, 2, None, {"b": 1}), R(2, 2, 3, {"x": 1}, {"x": 1, "b": 1}),
                                R(2, 6, 1, None, {"b": 1}), R(2, 7, 2, {"b": 2}, {"b": 2})])
    # values come from the segment after the op (b=2 on the last one: no match, no merge)
    assert ops == [{"pos1": 0, "pos2": 5, "props": {"b": 1}, "type": 2},
                   {"pos1": 6, "pos2": 7, "props": {"b": 1}, "type": 2},
                   {"pos1": 7, "pos2": 9, "props": {"b": 2}, "type": 2}]


def test_rewrite_delta_keys_and_values():
    # rewrite: keys the op drops (falsy in the op) first, in the segment's key order, then
    # the op's keys; integer-like keys enumerate first; dropped keys map to null
    m = {"type": 2, "pos1": 0, "pos2": 1, "props": {"z": 1, "k": 0, "5": "v"}, "combiningOp": {"name": "rewrite"}}
    ops = sq.ops_from_delta(m, [R(2, 0, 1, {"q": 1, "k": 3, "2": True, "z": 2}, {"z": 1, "k": 0, "5": "v"})])
    assert list(ops[0]["props"]) == ["2", "5", "q", "k", "z"]
    assert ops[0]["props"] == {"2": None, "5": "v", "q": None, "k": 0, "z": 1}


def test_insert_segment_json():
    assert sq.ops_from_delta({"type": 0, "pos1": 1, "seg": "ab"}, [R(0, 1, 2)]) == \
        [{"pos1": 1, "seg": "ab", "type": 0}]
    assert sq.ops_from_delta({"type": 0, "seg": {"text": "ab", "props": {}}}, [R(0, 4, 2, None, {})]) == \
        [{"pos1": 4, "seg": {"text": "ab", "props": {}}, "type": 0}]
    assert sq.ops_from_delta({"type": 0, "seg": {"marker": {"refType": 1}, "props": {"a": 1}}},
                             [R(0, 0, 1, None, {"a": 1})]) == \
        [{"pos1": 0, "seg": {"marker": {"refType": 1}, "props": {"a": 1}}, "type": 0}]


def test_transform_message_group_and_empty():
    msg = dict(clientId="a", sequenceNumber=9, referenceSequenceNumber=4, minimumSequenceNumber=2, type="op",
               contents={"type": 3, "ops": [{"type": 1, "pos1": 0, "pos2": 2}, {"type": 0, "pos1": 0, "seg": "x"}]})
    out = sq.transform_message(msg, [[], [R(0, 0, 1)]])
    assert list(out) == list(msg) and out["referenceSequenceNumber"] == 8
    assert out["contents"] == {"pos1": 0, "seg": "x", "type": 0}        # one op: not a group
    out = sq.transform_message(msg, [[], []])
    assert jsjson.stringify(out["contents"]) == '{"ops":[],"type":3}'   # createGroupOp() of nothing


def test_match_properties_restatement():
    assert sq.match_properties({"a": {"b": [1, 2]}}, {"a": {"b": [1, 2]}})
    assert not sq.match_properties({"a": {"b": [1, 2]}}, {"a": {"b": [1, 3]}})
    assert not sq.match_properties({"a": 1}, {"a": 1, "b": None})
    assert sq.match_properties(None, {}) is False and sq.match_properties({}, {}) is True
    assert sq.match_properties({"a": None}, {"a": None})
