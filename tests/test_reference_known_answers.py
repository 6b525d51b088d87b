"""Known answers restated from the reference's own merge-tree specs, for the passive
observer: each case is a short sequenced message list whose expected outcome (text and
the exact SnapshotV1 header bytes, or the segment structure) is written out here by
hand from the spec, and both the oracle (its own JSON path) and the engine (through the
Python `Client` drop-in) must produce it.

* properties.spec.ts:9-35 (matchProperties) — observed through coalescing: two adjacent
  segments at or below the MSN serialize as one iff their properties match
  (snapshotV1.ts:197-216, textSegment.ts:63-68).
* mergeTree.annotate.spec.ts:15-66, :485-520 — the remote cases ("remote", "remote
  only", "split remote"); and :644-677 ("sequenced local before remote") seen by an
  observer: a rewrite annotate from one client, then a plain one from another.
* snapshot.spec.ts:111-205 — MSN edge cases: segments below/above the MSN, removals above
  the MSN of segments below/above it, inserts next to removed segments, bodies past
  chunkSize; each snapshot loads back (Client.load) to the same text and length, and the
  stream continues on the loaded document.
* mergeTree.markRangeRemoved.deltaCallback.spec.ts:54-93 ("Event on Unlink") — a remove
  splits twice; once the MSN passes it zamboni unlinks the removed segment and the
  survivors on either side are not merged across it (scourNode resets prev,
  mergeTree.ts:1296-1303).
* mergeTree.insert.deltaCallback.spec.ts:35-150 and mergeTree.annotate.deltaCallback.spec.ts:
  36-153 — the countOperations tallies (delta callbacks per op, SPLIT maintenance records)
  of inserts at the start / end / middle, a marker insert, and annotates over an insertion
  or deletion the annotating client has or has not seen.
* client.walkSegments.spec.ts:22-65 — a range walk with splits visits 2 segments of 4
  characters (annotateRange's boundaries), without splits 2 whole segments of 10
  (cloneSegments, observed through a register copy and paste).
* client.getPostion.spec.ts:29-60 — event positions (Client.getPosition) of an existing, a
  removed, a moved and an about-to-be-detached segment.
* snapshotlegacy.spec.ts:14-83 — SnapshotLegacy of 10,000 (header only) and 10,010 (header
  and body) one-character segments loads back to the same length and text, twice.
"""
import json

import pytest

from emu_lib import emu_engine
from fluidframework_amd.engine import ClientGroup, Engine
from oracle_lib import OracleDoc

LIMITS = dict(rows_per_doc=40000, window_per_doc=16384, propsets_per_doc=4096, text_per_doc=1 << 18,
              blocks_per_doc=16384, heap_per_doc=40000)
GPU = lambda n, **kw: Engine(n, device=0, **kw)  # noqa: E731


def msg(cid, seq, ref, msn, contents, type="op"):
    return dict(clientId=cid, sequenceNumber=seq, referenceSequenceNumber=ref, minimumSequenceNumber=msn,
                type=type, contents=contents)


def ins(pos, seg):
    return {"type": 0, "pos1": pos, "seg": seg}


def rem(a, b):
    return {"type": 1, "pos1": a, "pos2": b}


def ann(a, b, props, rewrite=False):
    o = {"type": 2, "pos1": a, "pos2": b, "props": props}
    if rewrite:
        o["combiningOp"] = {"name": "rewrite"}
    return o


def v1_header(segments, min_seq, seq):
    """SnapshotV1 header chunk bytes (snapshotV1.ts:98-163, snapshotChunks.ts:125-149) for a
    document that fits one chunk; `segments` are already JSON-ready values."""
    length = 0
    for s in segments:
        j = s["json"] if isinstance(s, dict) and "json" in s else s
        length += len(j.encode("utf-16-le")) // 2 if isinstance(j, str) else \
            (len(j["text"].encode("utf-16-le")) // 2 if "text" in j else 1)
    hdr = {"version": "1", "segmentCount": len(segments), "length": length, "segments": segments, "startIndex": 0,
           "headerMetadata": {"minSequenceNumber": min_seq, "sequenceNumber": seq,
                              "orderedChunkMetadata": [{"id": "header"}], "totalLength": length,
                              "totalSegmentCount": len(segments)}}
    return json.dumps(hdr, separators=(",", ":"), ensure_ascii=False).encode()


def run_both(factory, msgs, load_first=None):
    """Apply `msgs` on the oracle (JSON path) and the engine; returns (oracle doc, client).
    load_first: a {path: contents} snapshot loaded into both before the messages."""
    od = OracleDoc(load_first is None)
    if load_first is not None:
        blobs = [load_first["header"]] + [load_first[k] for k in sorted(load_first) if k != "header"]
        assert od.load_snapshot(blobs) == 0
    g = ClientGroup(factory(1, **LIMITS))
    c = g.new_client({"newMergeTreeSnapshotFormat": True})
    if load_first is not None:
        c.load(load_first)
    for m in msgs:
        assert od.apply_msg(m) == 0, m
        c.applyMsg(m)
    assert c.getText() == od.get_text()
    return od, c


def header_now(od, c):
    """Both sides' SnapshotV1 header at the current window (no updateSeqNumbers)."""
    (eb, _), = c.engine.snapshot([c.doc_id], [-1], [-1])
    ob, _ = od.snapshot(c.min_seq, c.current_seq)
    assert eb == ob
    return eb[0]


# ---- properties.spec.ts:9-35 -------------------------------------------------------
MATCH = [
    ({"a": "a"}, {"a": "a"}, True),
    ({"a": "a"}, {"a": "b"}, False),
    ({"a": "a", "1": 1}, {"a": "a", "1": 1}, True),
    ({"a": "a", "1": 1}, {"a": "b", "1": 2}, False),
    ({"a": "a"}, {"b": "a"}, False),
    ({"a": "a"}, {"a": "a", "b": "b"}, False),
    ({"c": {"a": "a"}}, {"c": {"a": "a"}}, True),
    ({"c": {"a": "a"}}, {"c": {"a": "b"}}, False),
]


def check_match_properties(factory):
    for pa, pb, same in MATCH:
        msgs = [msg("x", 1, 0, 0, ins(0, {"text": "ab", "props": pa})),
                msg("x", 2, 1, 1, ins(2, {"text": "cd", "props": pb})),
                msg("x", 3, 2, 2, None, type="noop")]
        od, c = run_both(factory, msgs)
        js = lambda p: {k: p[k] for k in sorted(p, key=lambda k: (not k.isdigit(), int(k) if k.isdigit() else 0))}  # noqa
        segs = [{"text": "abcd", "props": js(pa)}] if same else \
            [{"text": "ab", "props": js(pa)}, {"text": "cd", "props": js(pb)}]
        assert header_now(od, c) == v1_header(segs, 2, 3), (pa, pb)


def test_match_properties_known_answers_on_emulation():
    check_match_properties(emu_engine)


@pytest.mark.gpu
def test_match_properties_known_answers_on_gpu():
    check_match_properties(GPU)


# ---- mergeTree.annotate.spec.ts ------------------------------------------------------
HELLO = {"header": v1_header(["hello world!"], 0, 0).decode()}


def check_annotate_remote(factory):
    # beforeEach (:27-45): "hello world!" (universal), a Tile marker inserted at
    # markerPosition 3 by the remote client at seq 1; annotate [1, 5).
    base = [msg("remote", 1, 0, 0, ins(3, {"marker": {"refType": 1}}))]
    # "remote" (:49-66) / "remote only" (:485-510)
    props = {"propertySource": "remote", "remoteProperty": 1}
    od, c = run_both(factory, base + [msg("remote", 2, 1, 0, ann(1, 5, props))], load_first=HELLO)
    marker = {"json": {"marker": {"refType": 1}, "props": props}, "seq": 1, "client": "remote"}
    assert header_now(od, c) == v1_header(["h", {"text": "el", "props": props}, marker, {"text": "l", "props": props},
                                           "o world!"], 0, 2)
    # "split remote" (:512-520): a later insert inside the annotated "el" splits it; both
    # halves keep the properties
    od, c = run_both(factory, base + [msg("remote", 2, 1, 0, ann(1, 5, props)),
                                      msg("other", 3, 2, 0, ins(2, "Z"))], load_first=HELLO)
    zz = {"json": "Z", "seq": 3, "client": "other"}
    assert header_now(od, c) == v1_header(["h", {"text": "e", "props": props}, zz, {"text": "l", "props": props}, marker,
                                           {"text": "l", "props": props}, "o world!"], 0, 3)
    # "sequenced local before remote" (:644-677) as an observer sees it: a rewrite
    # annotate {propertySource: "local"} (seq 2) then the remote one (seq 3)
    od, c = run_both(factory, base + [msg("local", 2, 1, 0, ann(1, 5, {"propertySource": "local"}, rewrite=True)),
                                      msg("remote", 3, 2, 0, ann(1, 5, props))], load_first=HELLO)
    marker = {"json": {"marker": {"refType": 1}, "props": props}, "seq": 1, "client": "remote"}
    assert header_now(od, c) == v1_header(["h", {"text": "el", "props": props}, marker, {"text": "l", "props": props},
                                           "o world!"], 0, 3)
    # rewrite after the remote annotate drops every key it does not set (:581-642 rule)
    od, c = run_both(factory, base + [msg("remote", 2, 1, 0, ann(1, 5, props)),
                                      msg("local", 3, 2, 0, ann(1, 5, {"propertySource": "local"}, rewrite=True))],
                     load_first=HELLO)
    lp = {"propertySource": "local"}
    marker = {"json": {"marker": {"refType": 1}, "props": lp}, "seq": 1, "client": "remote"}
    assert header_now(od, c) == v1_header(["h", {"text": "el", "props": lp}, marker, {"text": "l", "props": lp},
                                           "o world!"], 0, 3)


def test_annotate_remote_known_answers_on_emulation():
    check_annotate_remote(emu_engine)


@pytest.mark.gpu
def test_annotate_remote_known_answers_on_gpu():
    check_annotate_remote(GPU)


# ---- snapshot.spec.ts:111-205 ----------------------------------------------------------
class Str:
    """TestString (snapshot.spec.ts:30-109) from the observer's side: every op is a
    sequenced message of client "fakeId" (refSeq = seq - 1); increaseMsn moves the MSN
    to the op's own seq.  expect() snapshots both sides, loads each snapshot back
    (Client.load / SnapshotLoader), checks text and length, and continues on the
    loaded documents, as the spec does."""

    def __init__(self, factory):
        self.factory = factory
        self.seq = self.min_seq = 0
        self.od = OracleDoc(True)
        self.g = ClientGroup(factory(8, **LIMITS))
        self.c = self.g.new_client({"newMergeTreeSnapshotFormat": True})
        self.len = 0

    def _queue(self, op, inc):
        ref = self.seq
        self.seq += 1
        if inc:
            self.min_seq = self.seq
        m = msg("fakeId", self.seq, ref, self.min_seq, op)
        assert self.od.apply_msg(m) == 0
        self.c.applyMsg(m)

    def append(self, text, inc):
        self.insert(self.len, text, inc)

    def insert(self, pos, text, inc):
        self._queue(ins(pos, text), inc)
        self.len += len(text)

    def remove(self, a, b, inc):
        self._queue(rem(a, b), inc)
        self.len -= b - a

    def expect(self, text=None):
        if text is not None:
            assert self.c.getText() == text
        assert self.od.get_text() == self.c.getText()
        tree = self.c.snapshot()
        blobs = {e["path"]: e["value"]["contents"] for e in tree["entries"]}
        ob, _ = self.od.snapshot(self.c.min_seq, self.c.current_seq)
        assert [e["value"]["contents"].encode() for e in tree["entries"]] == ob
        od2 = OracleDoc(False)
        assert od2.load_snapshot([blobs["header"]] + [blobs[f"body_{i}"] for i in range(len(blobs) - 1)]) == 0
        c2 = self.g.new_client({"newMergeTreeSnapshotFormat": True})
        c2.load(blobs)
        assert c2.getText() == self.c.getText() == od2.get_text()
        assert c2.getLength() == self.c.getLength() == od2.get_length()
        self.od, self.c = od2, c2
        return blobs


def check_snapshot_spec(factory):
    s = Str(factory); s.append("0", True); s.expect("0")                                  # below MSN
    s = Str(factory); s.append("0", False); s.expect("0")                                 # ACKed above the MSN
    s = Str(factory); s.append("0x", False); s.remove(1, 2, False); s.expect("0")         # removal above MSN
    s = Str(factory); s.append("0x", True); s.remove(1, 2, False)                         # ... of a segment below it
    b = s.expect("0")
    assert json.loads(b["header"])["segments"] == ["0", {"json": "x", "removedSeq": 2, "removedClient": "fakeId"}]
    s.append("1", False); s.expect("01")                                                  # insert after the load
    s = Str(factory)                                                                      # relative to removed segment
    s.append("0x", False); s.append("2", False); s.remove(1, 2, False); s.insert(1, "1", False); s.append("3", False)
    s.expect("0123")
    s = Str(factory)                                                                      # ... loaded from a snapshot
    s.append("0x", False); s.append("2", False); s.remove(1, 2, False)
    s.expect("02")
    s.insert(1, "1", False); s.append("3", False); s.expect("0123")
    for inc in (True, False):                                                             # bodies past chunkSize
        s = Str(factory)
        for i in range(10000 + 10):
            s.append(str(i % 10), inc)
        b = s.expect()
        # below the MSN the appends coalesce into one segment (one chunk); above it every
        # segment carries merge info and the chunks fill to 10,000 characters
        assert len(b) == (1 if inc else 2)


def test_snapshot_spec_known_answers_on_emulation():
    check_snapshot_spec(emu_engine)


@pytest.mark.gpu
def test_snapshot_spec_known_answers_on_gpu():
    check_snapshot_spec(GPU)


# ---- mergeTree.markRangeRemoved.deltaCallback.spec.ts:54-93 --------------------------------
def check_unlink(factory):
    msgs = [msg("x", 1, 0, 0, rem(4, 6))]
    od, c = run_both(factory, msgs, load_first=HELLO)
    rows = c.engine.dump(c.doc_id)
    assert [int(r[0]) for r in rows] == [4, 2, 6]            # "hell" | "o " (removed) | "world!": two splits
    assert int(rows[1][3]) == 1
    od.apply_msg(msg("x", 2, 1, 1, None, type="noop"))       # the MSN passes the removal
    c.applyMsg(msg("x", 2, 1, 1, None, type="noop"))
    assert c.getText() == od.get_text() == "hellworld!"
    rows = c.engine.dump(c.doc_id)
    assert [int(r[0]) for r in rows] == [4, 6]               # unlinked; no merge across it
    assert (rows[:, [0, 1, 3, 9, 10, 11]] == od.dump()[:, [0, 1, 3, 9, 10, 11]]).all()


def test_unlink_known_answer_on_emulation():
    check_unlink(emu_engine)


@pytest.mark.gpu
def test_unlink_known_answer_on_gpu():
    check_unlink(GPU)


# ---- delta-callback counts (testUtils.countOperations) as a passive observer sees them ------
# The reference specs call MergeTree methods as a local client; the observer restatement has a
# remote client send the same op, so the same splits and callbacks happen in the observer's
# tree.  A delta callback counts once per op (its deltaSegments are the op's records), a
# maintenance callback once per record.
HELLO_WORLD = {"header": v1_header(["hello world"], 0, 0).decode()}
HW_CHARS = {"header": v1_header(list("hello world"), 0, 0).decode()}     # 11 one-character segments
HW_TWO = {"header": v1_header(["hello", "world"], 0, 0).decode()}       # client.walkSegments.spec.ts:16-21


def op_events(factory, load, msgs):
    """Apply msgs (one device batch each) on the engine with delta capture and on the oracle;
    both sides' records must agree; returns the per-message records [(kind, pos, len)] and
    countOperations-style counts."""
    od = OracleDoc(False)
    blobs = [load["header"]] + [load[k] for k in sorted(load) if k != "header"]
    assert od.load_snapshot(blobs) == 0
    od.delta_capture(True)
    eng = factory(1, **LIMITS)
    g = ClientGroup(eng)
    c = g.new_client({"newMergeTreeSnapshotFormat": True})
    c.load(load)
    out = []
    for m in msgs:
        od.delta_capture(False)
        od.delta_capture(True)
        assert od.apply_msg(m) == 0, m
        eng.delta_capture(1 << 16)
        c.applyMsg(m)
        g.flush()
        recs = eng.delta_records()
        eng.delta_capture(0)
        got = [(int(r["kind"]), int(r["pos"]), int(r["len"])) for r in recs]
        want = [(k, p, ln) for _, k, p, ln, *_ in od.delta_records()]
        assert got == want, (m, got, want)
        counts: dict = {}
        for k in {k for k, _, _ in got}:
            counts[k] = 1 if k >= 0 else sum(1 for x in got if x[0] == k)
        out.append((got, counts))
    assert c.getText() == od.get_text()
    return out, od, c


INSERT, REMOVE, ANNOTATE, APPEND, SPLIT, UNLINK = 0, 1, 2, -1, -2, -3


def check_insert_delta_counts(factory):
    # mergeTree.insert.deltaCallback.spec.ts:35-118 on "hello world!" (universal)
    hw = {"header": v1_header(["hello world!"], 0, 0).decode()}
    ev, _, _ = op_events(factory, hw, [msg("remote", 1, 0, 0, ins(0, "more "))])          # Insert text remote
    assert ev[0][1] == {INSERT: 1}
    ev, _, _ = op_events(factory, hw, [msg("remote", 1, 0, 0, ins(12, "more "))])         # Insert ending text
    assert ev[0][1] == {INSERT: 1}
    ev, _, _ = op_events(factory, hw, [msg("remote", 1, 0, 0, ins(4, "more "))])          # Insert middle text
    assert ev[0][1] == {INSERT: 1, SPLIT: 1}
    ev, _, _ = op_events(factory, hw, [msg("remote", 1, 0, 0, ins(4, {"marker": {"refType": 1}}))])   # Insert marker
    assert ev[0][1] == {INSERT: 1, SPLIT: 1}


def check_annotate_delta_counts(factory):
    # mergeTree.annotate.deltaCallback.spec.ts:36-153 on "hello world" (universal)
    foo = {"foo": "bar"}
    ev, _, _ = op_events(factory, HELLO_WORLD, [msg("B", 1, 0, 0, ann(4, 6, foo))])       # Event on annotation
    assert ev[0][1] == {ANNOTATE: 1, SPLIT: 2}
    # Annotate over local insertion: the annotating client's own insert is visible to it
    ev, _, _ = op_events(factory, HELLO_WORLD, [msg("B", 1, 0, 0, ins(4, "a")), msg("B", 2, 0, 0, ann(3, 8, foo))])
    assert ev[1][1] == {ANNOTATE: 1, SPLIT: 2}
    assert sum(ln for k, _, ln in ev[1][0] if k == ANNOTATE) == 5
    # Annotate over remote insertion: A's insert (seq 1) is not in B's refSeq-0 view
    ev, _, _ = op_events(factory, HELLO_WORLD, [msg("A", 1, 0, 0, ins(4, "a")), msg("B", 2, 0, 0, ann(3, 8, foo))])
    assert ev[1][1] == {ANNOTATE: 1, SPLIT: 2}
    assert sum(ln for k, _, ln in ev[1][0] if k == ANNOTATE) == 5
    # Annotate over remote deletion: A's removal (seq 1) is not in B's view either
    ev, _, _ = op_events(factory, HELLO_WORLD, [msg("A", 1, 0, 0, rem(4, 6)), msg("B", 2, 0, 0, ann(3, 8, foo))])
    assert ev[1][1] == {ANNOTATE: 1, SPLIT: 2}


def check_walk_segments(factory):
    # client.walkSegments.spec.ts:22-65 on "hello" + "world": a walk of [3, 7) visits both
    # segments (10 characters) without splitting, 2 segments of 4 characters with splitting.
    # With split (ensureIntervalBoundary at both ends, as annotateRange does):
    ev, _, _ = op_events(factory, HW_TWO, [msg("B", 1, 0, 0, ann(3, 7, {"k": 1}))])
    annot = [(p, ln) for k, p, ln in ev[0][0] if k == ANNOTATE]
    assert len(annot) == 2 and sum(ln for _, ln in annot) == 4 and ev[0][1] == {ANNOTATE: 1, SPLIT: 2}
    # Without split (mapRange, as cloneSegments' register copy does): 2 whole segments, 10 characters
    copy = msg("B", 1, 0, 0, {"type": 0, "pos1": 3, "pos2": 7, "register": "r"})
    paste = msg("B", 2, 1, 1, {"type": 0, "pos1": 0, "register": "r"})
    ev, od, c = op_events(factory, HW_TWO, [copy, paste])
    assert od.register_info("B", "r") == {"n": 2, "len": 10, "removed": 0, "pasted": 1}
    assert [(k, ln) for k, _, ln in ev[1][0] if k == INSERT] == [(INSERT, 5), (INSERT, 5)]
    assert c.getText() == "helloworldhelloworld"


def check_get_position(factory):
    # client.getPostion.spec.ts:29-60 on "hello world" as 11 one-character segments; the
    # "o" segment at 4.  SequenceDeltaEvent positions are Client.getPosition of the segment.
    ev, _, _ = op_events(factory, HW_CHARS, [msg("B", 1, 0, 0, ann(4, 5, {"k": 1}))])      # Existing Segment
    assert [(k, p) for k, p, _ in ev[0][0]] == [(ANNOTATE, 4)]
    ev, _, _ = op_events(factory, HW_CHARS, [msg("B", 1, 0, 0, rem(4, 5))])               # Deleted Segment
    assert [(k, p) for k, p, _ in ev[0][0]] == [(REMOVE, 4)]
    ev, _, _ = op_events(factory, HW_CHARS, [msg("B", 1, 0, 0, rem(3, 4)),                 # Moved Segment
                                             msg("B", 2, 1, 0, ann(3, 4, {"k": 1}))])
    assert [(k, p) for k, p, _ in ev[1][0]] == [(ANNOTATE, 3)]
    # Detached Segment: once the MSN passes the removal, zamboni scours the block: "h" takes
    # "e", "l", "l" (APPEND at 0, lengths 2, 3, 4), then unlinks "o".  The UNLINK callback
    # fires before segment.parent is cleared (mergeTree.ts:1296-1306) and getPosition walks
    # parent.children, which still holds the appended segments until the block is rebuilt,
    # so the reference names it at 4 + 1 + 1 + 1 = 7.  Afterwards it is detached: no later
    # event reaches it.
    ev, _, c = op_events(factory, HW_CHARS, [msg("B", 1, 0, 0, rem(4, 5)), msg("B", 2, 1, 1, None, type="noop"),
                                             msg("B", 3, 2, 2, ins(0, "x"))])
    assert ev[1][0][:4] == [(APPEND, 0, 2), (APPEND, 0, 3), (APPEND, 0, 4), (UNLINK, 7, 1)]
    assert all(k != UNLINK for k, _, _ in ev[2][0])
    assert c.getText() == "xhell world"


@pytest.mark.parametrize("check", [check_insert_delta_counts, check_annotate_delta_counts, check_walk_segments,
                                   check_get_position])
def test_delta_known_answers_on_emulation(check):
    check(emu_engine)


@pytest.mark.gpu
@pytest.mark.parametrize("check", [check_insert_delta_counts, check_annotate_delta_counts, check_walk_segments,
                                   check_get_position])
def test_delta_known_answers_on_gpu(check):
    check(GPU)


# ---- snapshotlegacy.spec.ts:14-83 --------------------------------------------------------
def check_snapshot_legacy(factory, n):
    """Client "0" appends `${i % 10}` with props {segment: i}, msn = seq, n times; the observer's
    SnapshotLegacy loads back to the same length and text, and again from the loaded copy."""
    msgs = [msg("0", i + 1, i, i + 1, ins(i, {"text": str(i % 10), "props": {"segment": i}})) for i in range(n)]
    lim = dict(LIMITS, propsets_per_doc=2 * n + 64)
    g = ClientGroup(factory(3, **lim))
    c0 = g.new_client()                                  # default options: SnapshotLegacy
    od = OracleDoc(True)
    for m in msgs:
        c0.applyMsg(m)
        assert od.apply_msg(m) == 0
    text, length = od.get_text(), od.get_length()
    assert c0.getText() == text and c0.getLength() == length == n
    prev_o, prev_c = od, c0
    for hop in range(2):                                  # client1 -> client2 -> client3 (:46-80)
        tree = prev_c.snapshot()
        blobs = {e["path"]: e["value"]["contents"] for e in tree["entries"]}
        ob, _ = prev_o.snapshot(n, n, legacy=True)
        assert [blobs["header"].encode()] + ([blobs["body"].encode()] if "body" in blobs else []) == ob
        assert ("body" in blobs) == (n > 10000)           # sizeOfFirstChunk (snapshotlegacy.ts:57)
        o2 = OracleDoc(False)
        assert o2.load_snapshot([blobs["header"]] + ([blobs["body"]] if "body" in blobs else [])) == 0
        c2 = g.new_client()
        c2.load(blobs)
        assert c2.getLength() == o2.get_length() == length
        assert c2.getText() == o2.get_text() == text
        prev_o, prev_c = o2, c2


@pytest.mark.parametrize("n", [10000, 10010])
def test_snapshot_legacy_known_answers_on_emulation(n):
    check_snapshot_legacy(emu_engine, n)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [10000, 10010])
def test_snapshot_legacy_known_answers_on_gpu(n):
    check_snapshot_legacy(GPU, n)


# ---- regression: rows whose removal the author has not seen (round 4) ----------------------
def check_unseen_removal_split(factory):
    """A leaf that a walk splits holds removed rows whose removal the op's author has not
    seen: they count at their full length (nodeLength, mergeTree.ts:1671-1683).  With the
    short-circuit visibility test, the gfx950 backend once merged `vis ? len : 0` wrongly for
    such rows (length 0), and the walk lost the position (INSERT_FAILED) or landed late.  B
    removes "lo " at seq 1; A, still at refSeq 0, inserts "X" at 5 of "hello world" (between
    "hello" and " "), then at 8 of its view ("wo|rld"), then removes [1, 4) of its view."""
    msgs = [msg("B", 1, 0, 0, rem(3, 6)), msg("A", 2, 0, 0, ins(5, "X")), msg("A", 3, 0, 0, ins(9, "Y")),
            msg("A", 4, 0, 0, rem(1, 4))]
    od, c = run_both(factory, msgs, load_first=HW_CHARS)
    assert c.getText() == od.get_text() == "hXwoYrld"
    header_now(od, c)


def test_unseen_removal_split_on_emulation():
    check_unseen_removal_split(emu_engine)


@pytest.mark.gpu
def test_unseen_removal_split_on_gpu():
    check_unseen_removal_split(GPU)


# ---- canAppend's trailing newline through zamboni merges (textSegment.ts:63-68) ------------
def check_newline_merge(factory):
    """"ab" takes "c\\n" (no trailing newline on "ab"), but the merged "abc\\n" must not take "d";
    "x\\ny" (newline inside, not trailing) still takes "z".  The engine flags newline-free rows
    (MT_M_NONL) and a merge clears the head's flag when a follower had a newline."""
    msgs = [msg("A", 1, 0, 0, ins(0, "ab")), msg("A", 2, 1, 1, ins(2, "c\n")), msg("A", 3, 2, 2, ins(4, "d")),
            msg("A", 4, 3, 3, ins(5, "x\ny")), msg("A", 5, 4, 4, ins(8, "z")),
            msg("A", 6, 5, 5, None, type="noop"), msg("A", 7, 6, 6, None, type="noop")]
    od, c = run_both(factory, msgs)
    assert c.getText() == "abc\ndx\nyz"
    hdr = json.loads(header_now(od, c))
    assert hdr["segments"] == ["abc\n", "dx\nyz"], hdr["segments"]


def test_newline_merge_on_emulation():
    check_newline_merge(emu_engine)


@pytest.mark.gpu
def test_newline_merge_on_gpu():
    check_newline_merge(GPU)


# ---- a range op that starts past the end of its author's view (round-3 advisor item) --------
def check_range_past_end(factory, residency):
    """A remove and an annotate whose start lies past the length in the author's view map no
    segment (mapRange finds none: the op is a no-op); the range walk's path resume must not
    reuse the previous op's path for the end then.  Under block (2) and all-HBM (0) residency."""
    def fac(n, **kw):
        e = factory(n, **kw)
        e.set_residency(residency)
        return e
    msgs = [msg("A", 1, 0, 0, ins(3, "XY")), msg("B", 2, 1, 0, rem(1, 4)),
            msg("A", 3, 2, 1, rem(20, 24)), msg("B", 4, 3, 2, ann(40, 44, {"k": 1})),
            msg("A", 5, 4, 3, rem(12, 15)), msg("B", 6, 5, 4, ins(2, "z")), msg("A", 7, 6, 5, rem(0, 2))]
    od, c = run_both(fac, msgs, load_first=HW_CHARS)
    header_now(od, c)


@pytest.mark.parametrize("residency", [2, 0])
def test_range_past_end_on_emulation(residency):
    check_range_past_end(emu_engine, residency)


@pytest.mark.gpu
@pytest.mark.parametrize("residency", [2, 0])
def test_range_past_end_on_gpu(residency):
    check_range_past_end(GPU, residency)
