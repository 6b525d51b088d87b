"""Host side of snapshot loading (mt_load_snapshot): the JSON half of SnapshotLoader.

The reference parses each chunk blob with JSON.parse and normalizes it with
toLatestVersion (MT/snapshotV1.ts:270-279, MT/snapshotChunks.ts:137-180), then
SnapshotLoader reads the header chunk's segments and metadata (loadHeader,
MT/snapshotLoader.ts:126-160) and, when the header does not hold every segment,
the body chunks in orderedChunkMetadata order (loadBody, :162-206).  This module
does that parsing and packs the segments into the mt_load_seg records the device
loader consumes; every tree operation (reloadFromSegments, startCollaboration,
the body's insertSegments calls) runs on the GPU.
"""
from __future__ import annotations

import ctypes
import json
from dataclasses import dataclass, field
from typing import Any

import numpy as np

from . import jsjson
from .batch import ClientNames, PropTable, _ptr

# mt_load_seg flags (include/mtgpu.h)
MT_LS_SEQ, MT_LS_CLIENT, MT_LS_REMOVED, MT_LS_MARKER = 0x01, 0x02, 0x04, 0x08

LOAD_SEG_DTYPE = np.dtype([("flags", np.uint8), ("pad0", np.uint8), ("client", np.uint16), ("seq", np.int32),
                           ("removed_seq", np.int32), ("removed_client", np.uint16), ("prop_id", np.int16),
                           ("payload_off", np.uint32), ("payload_len", np.uint32), ("marker_id", np.uint32),
                           ("pad1", np.uint32)])
assert LOAD_SEG_DTYPE.itemsize == 32


class MtLoadBatch(ctypes.Structure):
    _fields_ = [("n_docs", ctypes.c_uint32), ("doc_ids", ctypes.c_void_p), ("seg_offsets", ctypes.c_void_p),
                ("header_segments", ctypes.c_void_p), ("min_seq", ctypes.c_void_p), ("seq", ctypes.c_void_p),
                ("segs", ctypes.c_void_p), ("payload", ctypes.c_void_p), ("payload_units", ctypes.c_uint64)]


class SnapshotFormatError(ValueError):
    pass


@dataclass
class ParsedSnapshot:
    """One document's snapshot as SnapshotLoader sees it."""
    header: list            # segment specs of the header chunk
    body: list              # segment specs of the body chunks (empty if the header holds all)
    min_seq: int            # headerMetadata.minSequenceNumber ?? sequenceNumber
    seq: int                # headerMetadata.sequenceNumber
    total_length: int = 0
    total_segments: int = 0


def _latest(chunk: dict, header: bool) -> dict:
    """toLatestVersion (snapshotChunks.ts:137-160) + buildHeaderMetadataForLegecyChunk (:162-180)."""
    ver = chunk.get("version")
    if ver == "1":
        return {"segments": chunk.get("segments"), "segmentCount": chunk.get("segmentCount"),
                "length": chunk.get("length"), "headerMetadata": chunk.get("headerMetadata") if header else None}
    if ver is None:
        md = None
        if header:
            md = chunk.get("headerMetadata")
            if md is None:
                ids = [{"id": "header"}]
                if chunk.get("chunkLengthChars", 0) < chunk.get("totalLengthChars", 0):
                    ids.append({"id": "body"})
                md = {"orderedChunkMetadata": ids, "minSequenceNumber": chunk.get("chunkMinSequenceNumber"),
                      "sequenceNumber": chunk.get("chunkSequenceNumber"), "totalLength": chunk.get("totalLengthChars"),
                      "totalSegmentCount": chunk.get("totalSegmentCount")}
        return {"segments": chunk.get("segmentTexts"), "segmentCount": chunk.get("chunkSegmentCount"),
                "length": chunk.get("chunkLengthChars"), "headerMetadata": md}
    raise SnapshotFormatError(f"Unsupported chunk version: {ver}")


def _parse(blob) -> dict:
    if isinstance(blob, (bytes, bytearray)):
        blob = blob.decode("utf-8")
    return json.loads(blob)


def parse_snapshot(blobs: dict | list) -> ParsedSnapshot:
    """blobs: {path: contents} (an ITree's blobs) or [header, chunk1, chunk2, ...] in
    orderedChunkMetadata order."""
    get = (lambda k: blobs.get(k)) if isinstance(blobs, dict) else None
    head = _latest(_parse(blobs["header"] if get else blobs[0]), True)
    md = head["headerMetadata"]
    if md is None:
        raise SnapshotFormatError("header metadata not available")          # snapshotLoader.ts:141-143
    seq = md.get("sequenceNumber")
    ms = md.get("minSequenceNumber")
    ms = seq if ms is None else ms
    out = ParsedSnapshot(list(head["segments"] or []), [], ms, seq, md.get("totalLength") or 0,
                         md.get("totalSegmentCount") or 0)
    if head["segmentCount"] == md.get("totalSegmentCount"):                  # loadBody :170-172
        return out
    ids = [c["id"] for c in md.get("orderedChunkMetadata", [])]
    for k, cid in enumerate(ids[1:], start=1):
        raw = get(cid) if get else (blobs[k] if k < len(blobs) else None)
        if raw is None:
            raise SnapshotFormatError(f"missing chunk {cid}")
        out.body.extend(_latest(_parse(raw), False)["segments"] or [])
    return out


def _seg_record(spec: Any, props: PropTable, names: ClientNames, payload: list, header: bool = False) -> tuple | None:
    """SnapshotLoader.specToSegment (snapshotLoader.ts:93-124) over
    SharedStringFactory.segmentFromSpec (sequenceFactory.ts:31-37): the record
    fields, or None where the reference would fail."""
    merge = isinstance(spec, dict) and "json" in spec                         # hasMergeInfo, snapshotChunks.ts:74-76
    js = spec["json"] if merge else spec
    flags, p, plen, poff = 0, None, 0, 0
    if isinstance(js, str):                                                   # TextSegment.fromJSONObject
        units = jsjson.utf16_units(js)
    elif isinstance(js, dict) and "text" in js:
        if not isinstance(js["text"], str):
            return None
        units = jsjson.utf16_units(js["text"])
        p = js.get("props")
    elif isinstance(js, dict) and "marker" in js:                             # Marker.fromJSONObject
        rt = js["marker"].get("refType") if isinstance(js["marker"], dict) else None
        if not isinstance(rt, (int, float)) or isinstance(rt, bool) or int(rt) != rt or rt < 0:
            return None
        flags |= MT_LS_MARKER
        units, plen = None, int(rt)
        p = js.get("props")
    else:
        return None
    if units is not None:
        poff, plen = len(payload), len(units)
        payload.extend(units)
    pid = -1
    if p is not None and jsjson.js_truthy(p):                                 # make(..., props): addProperties
        if not isinstance(p, dict):
            return None
        pid = props.intern(p)
    mid = 0
    # mapped ids: body markers (insertSegments, mergeTree.ts:2218-2222) and header markers not
    # removed (reloadFromSegments -> addNodeReferences needs localNetLength > 0, :286-297)
    removed = merge and (spec.get("removedSeq") is not None or spec.get("removedClient") is not None)
    if flags & MT_LS_MARKER and isinstance(p, dict) and jsjson.js_truthy(p.get("markerId")) and \
            not (header and removed):                                                    # Marker.getId
        m = names.marker_define(p["markerId"])
        if m is None:
            return None                                   # duplicate or non-string id: off the batch path
        mid = m + 1
    client, seq, rseq, rcl = 0, 0, 0, 0
    if merge:
        if "client" in spec and spec["client"] is not None:
            if not isinstance(spec["client"], str):
                return None
            flags |= MT_LS_CLIENT
            client = names.index(spec["client"])
        if "seq" in spec and spec["seq"] is not None:
            flags |= MT_LS_SEQ
            seq = spec["seq"]
        rs, rc = spec.get("removedSeq"), spec.get("removedClient")
        if rs is not None or rc is not None:
            if rs is None or not isinstance(rc, str):
                return None                                                   # (the V1 writer emits both)
            flags |= MT_LS_REMOVED
            rseq, rcl = rs, names.index(rc)
        for v in (seq, rseq):
            if not isinstance(v, int) or isinstance(v, bool):
                return None
    return (flags, 0, client, seq, rseq, rcl, pid, poff, plen, mid, 0)


@dataclass
class LoadBatch:
    """A packed mt_load_batch (numpy arrays kept alive with it)."""
    doc_ids: np.ndarray
    seg_offsets: np.ndarray
    header_segments: np.ndarray
    min_seq: np.ndarray
    seq: np.ndarray
    segs: np.ndarray
    payload: np.ndarray
    _c: Any = field(default=None, repr=False)

    def to_c(self) -> MtLoadBatch:
        if self._c is None:
            self._c = MtLoadBatch(len(self.doc_ids), _ptr(self.doc_ids), _ptr(self.seg_offsets),
                                  _ptr(self.header_segments), _ptr(self.min_seq), _ptr(self.seq), _ptr(self.segs),
                                  _ptr(self.payload), int(self.payload.size))
        return self._c


class LoadBatchBuilder:
    """Packs parsed snapshots of many documents into one mt_load_batch."""

    def __init__(self, props: PropTable):
        self.props = props
        self.docs, self.offs, self.nhdr, self.ms, self.cs = [], [0], [], [], []
        self.recs: list = []
        self.payload: list = []

    def add(self, doc_id: int, snap: ParsedSnapshot, names: ClientNames) -> bool:
        """Adds one document; False if the host rejected it (it loads as MT_DS_UNSUPPORTED)."""
        p0, r0 = len(self.payload), len(self.recs)
        recs, ok = [], isinstance(snap.seq, int) and isinstance(snap.min_seq, int)
        nh0 = len(snap.header)
        for i, spec in enumerate(list(snap.header) + list(snap.body)):
            r = _seg_record(spec, self.props, names, self.payload, header=i < nh0) if ok else None
            if r is None:
                ok = False
                break
            recs.append(r)
        if not ok:                                      # min_seq < 0: the device flags MT_DS_UNSUPPORTED
            del self.payload[p0:]
            recs, nh, ms, cs = [], 0, -1, 0
        else:
            nh, ms, cs = len(snap.header), snap.min_seq, snap.seq
        self.recs.extend(recs)
        self.docs.append(doc_id)
        self.offs.append(r0 + len(recs))
        self.nhdr.append(nh)
        self.ms.append(ms)
        self.cs.append(cs)
        return ok

    def build(self) -> LoadBatch:
        segs = np.array(self.recs, dtype=LOAD_SEG_DTYPE) if self.recs else np.zeros(1, LOAD_SEG_DTYPE)
        pay = np.asarray(self.payload or [0], np.uint16)
        return LoadBatch(np.asarray(self.docs, np.uint32), np.asarray(self.offs, np.uint32),
                         np.asarray(self.nhdr, np.uint32), np.asarray(self.ms, np.int32),
                         np.asarray(self.cs, np.int32), segs, pay)


def _spec_units(x) -> int:
    js = x["json"] if isinstance(x, dict) and "json" in x else x
    if isinstance(js, str):
        return len(jsjson.utf16_units(js))
    if isinstance(js, dict) and isinstance(js.get("text"), str):
        return len(jsjson.utf16_units(js["text"]))
    return 0


def load_caps(snaps: list, extra_rows: int = 0, extra_text: int = 0) -> dict:
    """Per-document pool capacities that hold the loaded documents (+ headroom for
    the ops that follow): every segment a row (+1 per body insert for its boundary
    split), the reloadFromSegments blocks plus 4/4 splits of body inserts."""
    rows, text, blocks, props, window = [], [], [], [], []
    for s in snaps:
        segs = list(s.header) + list(s.body)
        n, units = len(segs), sum(_spec_units(x) for x in segs)
        rows.append(n + len(s.body) + 64 + extra_rows)
        text.append(2 * units + 256 + extra_text)
        blocks.append((n + len(s.body)) // 3 + 64 + extra_rows // 2)
        props.append(n + 64 + extra_rows)
        window.append(n + 64 + extra_rows)
    return dict(rows_per_doc=rows, text_per_doc=text, blocks_per_doc=blocks, propsets_per_doc=props,
                window_per_doc=window, heap_per_doc=list(rows))
