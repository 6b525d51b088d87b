"""SharedSegmentSequence's merge-tree plumbing over the engine (packages/dds/sequence/src/sequence.ts).

The part of the sequence DDS that sits on the replay path for the reference's default
snapshot format (``options.newMergeTreeSnapshotFormat`` unset: SnapshotLegacy plus
catch-up ops):

* ``processMergeTreeMsg`` (sequence.ts:604-642): every sequenced op is applied through
  ``Client.applyMsg`` and stashed in ``messagesSinceMSNChange``; a message whose
  refSeq is not seq - 1 is stashed *transformed*: its contents are rebuilt from the
  ``sequenceDelta`` events it raised (``createOpsFromDelta``, sequence.ts:58-105) and
  its refSeq becomes seq - 1, so that a client loading the snapshot can apply it
  against the snapshot's state.  The events come from the engine's delta records
  (mt_delta_records, §8(f4)); the property maps they name come from the document's
  device property sets.
* the stash's GC (:636-640, ``processMinSequenceNumberChanged`` :648-658);
* ``snapshotMergeTree`` (:592-602): MSN from the delta manager, the stash's MSNs set
  to it, then ``Client.snapshot`` with the stash as catch-up messages.
"""
from __future__ import annotations

import copy
import math
from typing import Any

from . import jsjson
from .batch import _group_members

INSERT, REMOVE, ANNOTATE, GROUP = 0, 1, 2, 3


# ---- MT/properties.ts:64-95 matchProperties, restated over Python JSON values ----------
def _truthy(v) -> bool:
    return jsjson.js_truthy(v)


def _is_object_type(v) -> bool:
    return v is None or isinstance(v, (dict, list))


def _for_in_keys(v) -> list:
    if isinstance(v, dict):
        return jsjson.js_key_order(list(v.keys()))
    if isinstance(v, (list, str)):
        return [str(i) for i in range(len(v))]
    return []


_MISSING = object()


def _member(v, k):
    if isinstance(v, dict):
        x = v.get(k, _MISSING)
        return _MISSING if x is jsjson.UNDEFINED else x          # `b[key] === undefined`
    if isinstance(v, (list, str)) and k.isdigit() and int(k) < len(v) and str(int(k)) == k:
        return v[int(k)]
    return _MISSING


def _strict_eq(a, b) -> bool:
    if isinstance(a, bool) or isinstance(b, bool):
        return isinstance(a, bool) and isinstance(b, bool) and a == b
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return not (isinstance(a, float) and math.isnan(a)) and a == b
    if isinstance(a, str) and isinstance(b, str):
        return a == b
    return a is b


def match_properties(a, b) -> bool:
    if _truthy(a):
        if not _truthy(b):
            return False
        for key in _for_in_keys(a):
            bk = _member(b, key)
            if bk is _MISSING:
                return False
            if _is_object_type(bk):
                if not match_properties(_member(a, key), bk):
                    return False
            elif not _strict_eq(bk, _member(a, key)):
                return False
        for key in _for_in_keys(b):
            if _member(a, key) is _MISSING:
                return False
    elif _truthy(b):
        return False
    return True


# ---- createOpsFromDelta (sequence.ts:58-105) ------------------------------------------
def seg_json(op_seg, props) -> Any:
    """segment.clone().toJSONObject() of an inserted segment (TextSegment.toJSONObject,
    MT/textSegment.ts:48-54; Marker.toJSONObject, MT/mergeTree.ts:649-653): its text (or
    marker) and its properties after the insert (None: undefined)."""
    if isinstance(op_seg, str):
        text, marker = op_seg, None
    elif isinstance(op_seg, dict) and "text" in op_seg:
        text, marker = op_seg["text"], None
    else:
        spec = op_seg["marker"]          # refType undefined stays undefined (omitted)
        text, marker = None, ({"refType": spec["refType"]} if "refType" in spec else {})
    if marker is not None:
        return {"marker": marker, "props": props} if props is not None else {"marker": marker}
    return {"text": text, "props": props} if props is not None else text


def annotate_delta_keys(op: dict, before: dict | None) -> list:
    """Object.keys of SegmentPropertiesManager.addProperties' deltas for a remote annotate
    (segmentPropertiesManager.ts:67-112): with rewrite, the keys it deleted (in the
    segment's key order) first, then every key of the op's props."""
    new = op.get("props") or {}
    keys: list = []
    cop = op.get("combiningOp")
    if isinstance(cop, dict) and cop.get("name") == "rewrite" and before:
        keys += [k for k in jsjson.js_key_order(list(before)) if not _truthy(new.get(k))]
    keys += [k for k in jsjson.js_key_order(list(new)) if k not in keys]
    return jsjson.js_key_order(keys)


def ops_from_delta(member: dict, ranges: list) -> list:
    """createOpsFromDelta for one op's sequenceDelta event.  ranges: the event's
    deltaSegments in order, each {kind, pos, len, before, after[, spec]} (before/after: the
    segment's properties around an annotate; after: an insert's properties; spec: a pasted
    segment's content, {"text": ...} or {"marker": {"refType": n}})."""
    ops: list = []
    for r in ranges:
        if r["kind"] == ANNOTATE:
            after = r["after"] or {}
            # `r.segment.properties[key] === undefined ? null : r.segment.properties[key]`
            props = {k: (None if after.get(k, jsjson.UNDEFINED) is jsjson.UNDEFINED else after[k])
                     for k in annotate_delta_keys(member, r["before"])}
            last = ops[-1] if ops else None
            if last and last["type"] == ANNOTATE and last["pos2"] == r["pos"] and match_properties(last["props"], props):
                last["pos2"] += r["len"]
            else:
                ops.append({"pos1": r["pos"], "pos2": r["pos"] + r["len"], "props": props, "type": ANNOTATE})
        elif r["kind"] == INSERT:
            # the inserted segment's clone: the op's seg, or (a register paste has none) the
            # pasted clone's own text / marker as the engine recorded it
            spec = r.get("spec") or member["seg"]
            ops.append({"pos1": r["pos"], "seg": seg_json(spec, r["after"]), "type": INSERT})
        elif r["kind"] == REMOVE:
            last = ops[-1] if ops else None
            if last is not None and last.get("pos1") == r["pos"]:
                last["pos2"] += r["len"]
            else:
                ops.append({"pos1": r["pos"], "pos2": r["pos"] + r["len"], "type": REMOVE})
    return ops


def transform_message(message: dict, events: list) -> dict:
    """The stash entry of a message whose refSeq != seq - 1 (sequence.ts:622-631): refSeq
    becomes seq - 1 and contents the ops rebuilt from its events (one event per member)."""
    members = [m for m in _group_members(message.get("contents"))
               if m.get("type") in (INSERT, REMOVE, ANNOTATE)]
    ops: list = []
    for m, ev in zip(members, events):
        ops += ops_from_delta(m, ev)
    out = dict(message)
    out["referenceSequenceNumber"] = message["sequenceNumber"] - 1
    out["contents"] = ops[0] if len(ops) == 1 else {"ops": ops, "type": GROUP}
    return out


class SequenceDoc:
    """One SharedString's merge-tree plumbing on a ClientGroup document.

    ``process(msg)`` is processCore for a sequenced op of this DDS; the transformations
    are resolved when the group flushes (the events are device records of that batch).
    ``snapshot(min_seq)`` is snapshotMergeTree."""

    def __init__(self, group, options: dict | None = None, longClientId: str = "observer"):
        self.group = group
        self.options = options or {}
        self.client = group.new_client(self.options)
        self.client.startOrUpdateCollaboration(longClientId)
        self.legacy = self.options.get("newMergeTreeSnapshotFormat") is not True
        self.messagesSinceMSNChange: list = []
        if self.legacy:
            self.client.delta_listener = self._on_flush
        self.last_msn = 0
        self.last_seq = 0

    def process(self, raw: dict):
        """processCore -> processMergeTreeMsg for one sequenced op of this channel."""
        if raw.get("type") != "op":
            raise ValueError("Sequence message not operation")      # sequence.ts:559
        message = copy.deepcopy(raw)                      # parseHandles: the DDS works on its own copy
        self.client.applyMsg(message)
        self.last_msn = max(self.last_msn, int(message["minimumSequenceNumber"]))
        self.last_seq = int(message["sequenceNumber"])

    def observe(self, msn: int, seq: int):
        """The delta manager saw a message of another channel (MSN / last seq move)."""
        self.last_msn, self.last_seq = max(self.last_msn, int(msn)), max(self.last_seq, int(seq))

    def _on_flush(self, entries: list, events_of):
        """entries: [(message, [op index per member])]; events_of(op index) -> ranges."""
        for message, op_ids in entries:
            stash = message
            if message["referenceSequenceNumber"] != message["sequenceNumber"] - 1:
                stash = transform_message(message, [events_of(i) for i in op_ids])
            self.messagesSinceMSNChange.append(stash)
            st = self.messagesSinceMSNChange
            if len(st) > 20 and st[20]["sequenceNumber"] < message["minimumSequenceNumber"]:
                self._msn_changed(message["minimumSequenceNumber"])

    def _msn_changed(self, min_seq: int):                  # processMinSequenceNumberChanged :648-658
        st = self.messagesSinceMSNChange
        i = 0
        while i < len(st) and st[i]["sequenceNumber"] <= min_seq:
            i += 1
        if i:
            self.messagesSinceMSNChange = st[i:]

    def snapshot(self) -> dict:
        """snapshotMergeTree (sequence.ts:592-602) and Client.snapshot (client.ts:923-956):
        the delta manager's MSN and last seq move the window (updateSeqNumbers), the
        stash is trimmed and re-stamped, then the tree is written."""
        self.group.flush()
        m, s = self.last_msn, self.last_seq
        self._msn_changed(m)
        for x in self.messagesSinceMSNChange:
            x["minimumSequenceNumber"] = m
        self.client.updateSeqNumbers(m, s)
        return self.client.snapshot(self.messagesSinceMSNChange if self.legacy else None, min_seq=m, seq=s)

    def load(self, blobs: dict):
        """loadCore (sequence.ts:496-541) for the merge-tree blobs: Client.load, then the
        catch-up messages through processMergeTreeMsg after the window checks."""
        out = self.client.load(blobs)
        self.last_msn, self.last_seq = self.client.min_seq, self.client.current_seq
        for m in out["catchupOps"]:
            lo, cur = self.client.min_seq, self.client.current_seq
            if m["minimumSequenceNumber"] < lo or m["referenceSequenceNumber"] < lo or \
                    m["sequenceNumber"] <= lo or m["sequenceNumber"] <= cur:
                raise ValueError("Invalid catchup operations in snapshot: " + jsjson.stringify(
                    {"op": {"seq": m["sequenceNumber"], "minSeq": m["minimumSequenceNumber"],
                            "refSeq": m["referenceSequenceNumber"]},
                     "collabWindow": {"seq": cur, "minSeq": lo}}))
            self.process(m)
            self.client.current_seq = int(m["sequenceNumber"])

    def getText(self) -> str:
        return self.client.getText()
