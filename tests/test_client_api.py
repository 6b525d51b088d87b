"""The Python Client drop-in (fluidframework_amd.engine.ClientGroup /
MergeTreeClient, mirroring MT/client.ts) against the oracle, on the host
emulation (CPU) and on the device (GPU)."""
import json

import pytest

from emu_lib import emu_engine
from fluidframework_amd.engine import ClientGroup, Engine, MergeTreeError
from js_lib import batch_to_messages
from oracle_lib import gen_params, generate
from test_emu_parity import CONFIGS, ann_props

LIMITS = dict(rows_per_doc=20000, window_per_doc=8192, propsets_per_doc=8192, text_per_doc=1 << 18)


def check(factory, cfg, n_docs):
    props = ann_props()
    p = gen_params(seed=41, n_docs=n_docs, **CONFIGS[cfg])
    batch, st, kept = generate(p, props, keep=True)
    g = ClientGroup(factory(n_docs, **LIMITS))
    clients = [g.new_client({"newMergeTreeSnapshotFormat": True}) for _ in range(n_docs)]
    for d, c in enumerate(clients):
        c.startOrUpdateCollaboration("observer")
        for m in batch_to_messages(batch, props, d):
            c.applyMsg(m)
    last = batch.op_offsets[1:] - 1
    for d, c in enumerate(clients):
        od = kept[d]
        assert c.getText() == od.get_text()
        assert c.getLength() == od.get_length()
        blobs, _ = od.snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]))
        tree = c.snapshot()
        assert [e["path"] for e in tree["entries"]] == ["header"] + [f"body_{i}" for i in range(len(blobs) - 1)]
        assert [e["value"]["contents"].encode() for e in tree["entries"]] == blobs
        # The reference's default format (no newMergeTreeSnapshotFormat): SnapshotLegacy
        # plus the caller's catch-up messages (client.ts:950-954, snapshotlegacy.ts:162-172).
        c.options = None
        catch_up = batch_to_messages(batch, props, d)[-2:]
        lblobs, _ = od.snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]), legacy=True)
        tree = c.snapshot(catch_up)
        assert [e["path"] for e in tree["entries"]] == ["header", "body"][:len(lblobs)] + ["catchupOps"]
        assert [e["value"]["contents"].encode() for e in tree["entries"][:-1]] == lblobs
        assert json.loads(tree["entries"][-1]["value"]["contents"]) == catch_up


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
def test_client_group_on_emulation_matches_oracle(cfg):
    check(emu_engine, cfg, 3)


def test_client_assert_seq_raises():
    # completeAndLogOp asserts currentSeq < seq (MT/client.ts:482): the drop-in throws.
    g = ClientGroup(emu_engine(1, **LIMITS))
    c = g.new_client()
    c.applyMsg(dict(clientId="a", sequenceNumber=2, referenceSequenceNumber=0, minimumSequenceNumber=0, type="op",
                    contents={"type": 0, "pos1": 0, "seg": "ab"}))
    c.applyMsg(dict(clientId="a", sequenceNumber=2, referenceSequenceNumber=0, minimumSequenceNumber=0, type="op",
                    contents={"type": 0, "pos1": 0, "seg": "cd"}))
    with pytest.raises(MergeTreeError, match="ASSERT_SEQ"):
        c.getText()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
def test_client_group_on_gpu_matches_oracle(cfg):
    check(lambda n, **kw: Engine(n, device=0, **kw), cfg, 4)


def check_load(factory):
    """MergeTreeClient.load (Client.load / SnapshotLoader), then the rest of the stream."""
    from test_snapshot_load import COLLAB_CASES, collab_case, golden_blobs, golden_legacy_blobs, oracle_load, sub_batch
    case = dict(COLLAB_CASES[1])
    cut = case.pop("cut")
    props, batch, snaps, blobs_l = collab_case(cut=cut, **case)
    n = case["n_docs"]
    eng = factory(n + 2, rows_per_doc=40000, window_per_doc=8192, propsets_per_doc=8192, text_per_doc=1 << 19,
                  blocks_per_doc=16384)
    eng.props = props
    g = ClientGroup(eng)
    clients = [g.new_client({"newMergeTreeSnapshotFormat": True}) for _ in range(n + 1)]
    want, gblobs = golden_blobs("withAnnotations")
    assert clients[n].load(want) == {"catchupOps": []}
    od, _ = oracle_load(gblobs, props)
    assert clients[n].getText() == od.get_text()
    # the reference's legacy file of the same string: loads, and re-emits byte-for-byte
    lwant, lblobs = golden_legacy_blobs("withAnnotations")
    lc = g.new_client()
    assert lc.load(lwant) == {"catchupOps": []}
    assert lc.getText() == od.get_text()
    assert [e["value"]["contents"] for e in lc.snapshot()["entries"]] == lblobs
    for d in range(n):
        clients[d].load({("header" if i == 0 else f"body_{i - 1}"): b for i, b in enumerate(blobs_l[d])})
        for m in batch_to_messages(batch, props, d)[cut:]:
            clients[d].applyMsg(m)
    for d in range(n):
        od, st = oracle_load(blobs_l[d], props)
        assert st == 0 and od.apply_run(sub_batch(batch, d, cut, case["ops"], 0), 0) == 0
        assert clients[d].getText() == od.get_text()
        o = int(batch.op_offsets[d + 1]) - 1
        ob, _ = od.snapshot(int(batch.arrays["msn"][o]), int(batch.arrays["seq"][o]))
        assert [e["value"]["contents"].encode() for e in clients[d].snapshot()["entries"]] == ob


def test_client_load_on_emulation_matches_oracle():
    check_load(emu_engine)


@pytest.mark.gpu
def test_client_load_on_gpu_matches_oracle():
    check_load(lambda n, **kw: Engine(n, device=0, **kw))


def _msg(cid, seq, ref, msn, contents):
    return dict(clientId=cid, sequenceNumber=seq, referenceSequenceNumber=ref, minimumSequenceNumber=msn, type="op",
                contents=contents)


def _legacy_header(texts, min_seq):
    """Known-answer SnapshotLegacy header (snapshotlegacy.ts:74-98, snapshotChunks.ts:161-180)
    for a document whose snapshot fits the first chunk."""
    n = sum(len(t) for t in texts)
    return json.dumps({"chunkStartSegmentIndex": 0, "chunkSegmentCount": len(texts), "chunkLengthChars": n,
                       "totalLengthChars": n, "totalSegmentCount": len(texts), "chunkSequenceNumber": min_seq,
                       "segmentTexts": texts,
                       "headerMetadata": {"orderedChunkMetadata": [{"id": "header"}], "sequenceNumber": min_seq,
                                          "totalLength": n, "totalSegmentCount": len(texts)}},
                      separators=(",", ":"))


def check_legacy_known_answers(factory):
    """Hand-derived SnapshotLegacy bytes: an empty document; a remove above the MSN keeps its
    text and coalesces; a segment inserted above the MSN is left to the catch-up ops; once the
    MSN passes the remove, the removed text is gone and the survivors coalesce."""
    g = ClientGroup(factory(2, **LIMITS))
    empty, c = g.new_client(), g.new_client()
    assert [e["value"]["contents"] for e in empty.snapshot()["entries"]] == [_legacy_header([], 0)]
    c.applyMsg(_msg("a", 1, 0, 0, {"type": 0, "pos1": 0, "seg": "hello"}))
    c.applyMsg(_msg("b", 2, 1, 0, {"type": 0, "pos1": 5, "seg": " world"}))
    c.applyMsg(_msg("a", 3, 2, 1, {"type": 1, "pos1": 0, "pos2": 2}))
    assert c.getText() == "llo world"
    tree = c.snapshot()
    assert [e["path"] for e in tree["entries"]] == ["header"]
    assert tree["entries"][0]["value"]["contents"] == _legacy_header(["hello"], 1)
    c.updateSeqNumbers(3, 3)
    assert (c.min_seq, c.current_seq) == (3, 3)
    assert [e["value"]["contents"] for e in c.snapshot()["entries"]] == [_legacy_header(["llo world"], 3)]
    # the snapshot's own updateSeqNumbers(3, 3) must not move the MSN backwards (setMinSeq
    # asserts, mergeTree.ts:1716): the document stays readable afterwards
    assert int(c.engine.status([c.doc_id])[0]) == 0
    assert c.getText() == "llo world"
    assert c.snapshot()["entries"][0]["value"]["contents"] == _legacy_header(["llo world"], 3)


def test_legacy_known_answers_on_emulation():
    check_legacy_known_answers(emu_engine)


@pytest.mark.gpu
def test_legacy_known_answers_on_gpu():
    check_legacy_known_answers(lambda n, **kw: Engine(n, device=0, **kw))


def check_newline_blocks_append(factory):
    """TextSegment.canAppend (textSegment.ts:63-68): a segment ending in "\\n" takes no
    append, in zamboni's scour (mergeTree.ts:1278-1356) and in the snapshot's coalescing."""
    g = ClientGroup(factory(1, **LIMITS))
    c = g.new_client({"newMergeTreeSnapshotFormat": True})
    c.applyMsg(_msg("a", 1, 0, 0, {"type": 0, "pos1": 0, "seg": "ab\n"}))
    c.applyMsg(_msg("b", 2, 1, 0, {"type": 0, "pos1": 3, "seg": "cd"}))
    c.applyMsg(_msg("a", 3, 2, 0, {"type": 0, "pos1": 5, "seg": "ef"}))
    c.applyMsg(_msg("b", 4, 3, 0, {"type": 0, "pos1": 0, "seg": "x\n"}))
    c.applyMsg(_msg("a", 5, 4, 0, {"type": 0, "pos1": 2, "seg": "y"}))
    c.updateSeqNumbers(5, 5)
    assert c.getText() == "x\nyab\ncdef"
    assert [int(r[0]) for r in c.engine.dump(c.doc_id)] == [2, 4, 4]     # "x\n" | "yab\n" | "cdef"
    hdr = json.loads(c.snapshot()["entries"][0]["value"]["contents"])
    assert hdr["segments"] == ["x\n", "yab\n", "cdef"]


def test_newline_blocks_append_on_emulation():
    check_newline_blocks_append(emu_engine)


@pytest.mark.gpu
def test_newline_blocks_append_on_gpu():
    check_newline_blocks_append(lambda n, **kw: Engine(n, device=0, **kw))


def check_status_guards(factory):
    """A refSeq below the MSN (deli nacks it, deli/lambda.ts:302-318) is flagged, not
    replayed; a snapshot of a document with a status word fails (mt_snapshot_v1 returns
    MT_E_DOC_STATUS) instead of serializing it."""
    g = ClientGroup(factory(2, **LIMITS))
    a, b = g.new_client({"newMergeTreeSnapshotFormat": True}), g.new_client({"newMergeTreeSnapshotFormat": True})
    for c in (a, b):
        c.applyMsg(_msg("x", 1, 0, 0, {"type": 0, "pos1": 0, "seg": "abc"}))
        c.applyMsg(_msg("y", 2, 1, 1, {"type": 0, "pos1": 3, "seg": "def"}))
    a.applyMsg(_msg("x", 3, 0, 1, {"type": 1, "pos1": 0, "pos2": 1}))       # refSeq 0 < minSeq 1
    with pytest.raises(MergeTreeError, match="REFSEQ_BELOW_MSN"):
        a.getText()
    with pytest.raises(MergeTreeError):
        a.snapshot()
    assert b.getText() == "abcdef"                                         # other documents unaffected
    with pytest.raises(MergeTreeError, match=r"\(4\)"):
        g.engine.snapshot([a.doc_id], [1], [3])


def test_status_guards_on_emulation():
    check_status_guards(emu_engine)


@pytest.mark.gpu
def test_status_guards_on_gpu():
    check_status_guards(lambda n, **kw: Engine(n, device=0, **kw))
