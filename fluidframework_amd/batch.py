"""Host-side packing of sequenced merge-tree messages into engine op batches.

Mirrors what the reference does per message in ``Client.applyMsg``
(packages/dds/merge-tree/src/client.ts:819-841): register the long client id,
dispatch ``msg.contents`` (IMergeTreeOp, MT/ops.ts:6-110) by type, flatten GROUP
members (client.ts:804-812, all members share the message's seq), and finish
with ``updateSeqNumbers(msg.minimumSequenceNumber, msg.sequenceNumber)``
(client.ts:840).  The result is the SoA layout of ``mt_op_batch``
(include/mtgpu.h).  Property sets and client ids are interned here so the
device only ever sees small integers.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Any

import numpy as np

from . import jsjson

MT_OP_INSERT, MT_OP_REMOVE, MT_OP_ANNOTATE, MT_OP_NOOP, MT_OP_UNSUPPORTED = 0, 1, 2, 3, 4
MT_OPF_END_OF_MSG, MT_OPF_MARKER, MT_OPF_REWRITE, MT_OPF_SEG_PROPS, MT_OPF_COMBINE = 1, 2, 4, 8, 16
MT_OPF_CONSENSUS, MT_OPF_INCR_STRMIN = 2, 8          # on combining annotates (include/mtgpu.h)
MT_OP_CUT, MT_OP_COPY, MT_OP_PASTE = 5, 6, 7      # register ops (include/mtgpu.h)
MT_OPF_REL1, MT_OPF_REL2, MT_OPF_MARKER_ID = 0x20, 0x40, 0x80
MARKER_ID_KEY = "markerId"            # reservedMarkerIdKey, MT/mergeTree.ts:591
# property values other than interned ids (include/mtgpu.h MT_VAL_*, MT_VK_*)
MT_VAL_NULL, MT_VAL_NAN, MT_VAL_UNSUP, MT_VAL_CFRESH, MT_VAL_UNDEF, MT_VAL_THROW, MT_VAL_CONS_BASE = -1, -2, -3, -4, -5, -6, -16
INCR_CHAIN_MAX = 64        # incr results of a held string precomputed per value (PropTable.to_c)
MT_VK_NUM, MT_VK_SEQM1 = 1, 2


def _is_number(v) -> bool:            # typeof v === "number" || typeof v === "boolean" (x + undefined is NaN)
    return isinstance(v, (int, float))


def _seq_minus1(v) -> bool:           # `cv.seq === -1` on a (non-array) object, properties.ts:52
    s = v.get("seq") if isinstance(v, dict) else None
    return isinstance(s, (int, float)) and not isinstance(s, bool) and s == -1


def value_kind(v) -> int:
    return (MT_VK_NUM if _is_number(v) else 0) | (MT_VK_SEQM1 if _seq_minus1(v) else 0)


def decode_value(v: int, values_json: list):
    """A stored property value id (mt_doc_pset) as a Python JSON value: interned ids through
    the table; NaN; JS undefined (jsjson.UNDEFINED); a fresh consensus object
    {value: undefined, seq} (properties.ts:43-47)."""
    import json as _json
    if v >= 0:
        return _json.loads(values_json[v])
    if v == MT_VAL_NAN:
        return float("nan")
    if v == MT_VAL_UNDEF:
        return jsjson.UNDEFINED
    if v <= MT_VAL_CONS_BASE:
        return {"value": jsjson.UNDEFINED, "seq": MT_VAL_CONS_BASE - v}
    raise ValueError(f"not a stored property value: {v}")

MT_DS_NAMES = {
    0x01: "ASSERT_SEQ", 0x02: "ASSERT_MSN", 0x04: "INSERT_FAILED", 0x08: "UNSUPPORTED",
    0x10: "OOM_ROWS", 0x20: "OOM_BLOCKS", 0x40: "OOM_TEXT", 0x80: "OOM_PROPS",
    0x100: "OOM_HEAP", 0x200: "OOM_WINDOW", 0x400: "PROPS_TOO_MANY", 0x800: "BAD_OP",
    0x1000: "REFSEQ_BELOW_MSN", 0x2000: "OOM_OVERLAP", 0x4000: "THROWS",
}


def status_names(st: int) -> list[str]:
    return [n for b, n in MT_DS_NAMES.items() if st & b]


class MtOpBatch(ctypes.Structure):
    _fields_ = [
        ("n_runs", ctypes.c_uint32), ("doc_ids", ctypes.c_void_p), ("op_offsets", ctypes.c_void_p),
        ("n_ops", ctypes.c_uint32), ("type", ctypes.c_void_p), ("flags", ctypes.c_void_p),
        ("client", ctypes.c_void_p), ("seq", ctypes.c_void_p), ("ref_seq", ctypes.c_void_p),
        ("msn", ctypes.c_void_p), ("pos1", ctypes.c_void_p), ("pos2", ctypes.c_void_p),
        ("payload_off", ctypes.c_void_p), ("payload_len", ctypes.c_void_p), ("prop_id", ctypes.c_void_p),
        ("payload", ctypes.c_void_p), ("payload_units", ctypes.c_uint64),
        ("n_rel", ctypes.c_uint32), ("rel", ctypes.c_void_p),
    ]


class MtPropTable(ctypes.Structure):
    _fields_ = [
        ("n_sets", ctypes.c_uint32), ("set_off", ctypes.c_void_p), ("key", ctypes.c_void_p),
        ("value", ctypes.c_void_p), ("n_keys", ctypes.c_uint32), ("key_json", ctypes.c_void_p),
        ("key_index", ctypes.c_void_p), ("n_values", ctypes.c_uint32), ("value_json", ctypes.c_void_p),
        ("value_falsy", ctypes.c_void_p), ("value_class", ctypes.c_void_p), ("value_kind", ctypes.c_void_p),
        ("value_incr", ctypes.c_void_p), ("incr_object", ctypes.c_int32),
    ]


class MtGenParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64 if n == "seed" else ctypes.c_uint32) for n in (
        "seed", "n_docs", "ops_per_doc", "clients", "lag_max", "pct_insert", "pct_remove",
        "ins_len_max", "rem_len_max", "n_ann_sets", "pct_rewrite", "doc_id_base", "ins_len_min", "seg_prop_sets",
        "ins_at_end", "continue_docs")]


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a is not None and a.size else 0


def _cstr_array(strs: list[str]):
    arr = (ctypes.c_char_p * max(1, len(strs)))()
    keep = [s.encode("utf-8", "surrogatepass") for s in strs]
    for i, b in enumerate(keep):
        arr[i] = b
    return arr, keep


class PropTable:
    """Interned property sets in JS ``Object.keys`` order (null = delete)."""

    def __init__(self):
        self.key_ids: dict[str, int] = {}
        self.keys: list[str] = []
        self.value_ids: dict[str, int] = {}
        self.values_json: list[str] = []
        self.values_falsy: list[int] = []
        self.values_class: list[int] = []
        self.values_kind: list[int] = []
        self._class_ids: dict[Any, int] = {}
        self.set_ids: dict[tuple, int] = {}
        self.sets: list[tuple] = []
        self._incr_keys: set[int] = set()      # keys some incr op names
        self._n_incr = 0                       # incr ops interned
        self._c = None

    def key_id(self, k: str) -> int:
        i = self.key_ids.get(k)
        if i is None:
            i = self.key_ids[k] = len(self.keys)
            self.keys.append(k)
            self._c = None
        return i

    def value_id(self, v: Any) -> int:
        if v is None:
            return -1
        txt = jsjson.stringify(v)
        i = self.value_ids.get(txt)
        if i is None:
            i = self.value_ids[txt] = len(self.values_json)
            self.values_json.append(txt)
            self.values_falsy.append(0 if jsjson.js_truthy(v) else 1)
            ck = jsjson.match_class_key(v)
            c = self._class_ids.setdefault(ck, len(self._class_ids))
            self.values_class.append(c)
            self.values_kind.append(value_kind(v))
            self._c = None
        return i

    def intern(self, props: dict) -> int:
        pairs = tuple((self.key_id(k), self.value_id(props[k])) for k in jsjson.js_key_order(list(props.keys())))
        return self._intern_pairs(pairs)

    def intern_combine(self, props: dict, cop, seq: int) -> tuple[int, int]:
        """(combine set, MT_OPF_* flags) of a remote annotate with a combining op other than
        rewrite (include/mtgpu.h): the op's keys, each valued with what
        combine(op, undefined, undefined, seq) yields (properties.ts:24-62 through
        segmentPropertiesManager.ts:98-103), i.e. for a key the segment does not hold."""
        name = cop.get("name") if isinstance(cop, dict) else None
        has_def = isinstance(cop, dict) and "defaultValue" in cop
        d = cop.get("defaultValue") if has_def else None
        if name == "incr":                  # x + undefined: NaN, or String(x) + "undefined"
            mv = cop.get("minValue")
            str_min = jsjson.js_truthy(mv) and isinstance(mv, (str, list, dict))
            if not has_def or d is None or _is_number(d):
                code = MT_VAL_NAN           # NaN < minValue is false
            else:
                r = jsjson.js_to_string(d) + "undefined"
                # `if (_currentValue < minValue)` compares two strings by UTF-16 code units
                below = str_min and jsjson.utf16_units(r) < jsjson.utf16_units(jsjson.js_to_string(mv))
                code = self.value_id(mv) if below else self.value_id(r)
            fl = MT_OPF_COMBINE | (MT_OPF_INCR_STRMIN if str_min else 0)
            self._n_incr += 1
            for k in props.keys():
                self._incr_keys.add(self.key_id(k))
        elif name == "consensus":           # {value: undefined, seq}; null.seq throws; seq -1 is set
            if not has_def:
                code = MT_VAL_CFRESH
            elif d is None:
                code = MT_VAL_THROW
            else:
                code = self.value_id({**d, "seq": seq} if _seq_minus1(d) else d)
            fl = MT_OPF_COMBINE | MT_OPF_REWRITE | MT_OPF_CONSENSUS
        else:                               # no case in combine's switch: the (default) value
            code = MT_VAL_UNDEF if not has_def else (MT_VAL_NULL if d is None else self.value_id(d))
            fl = MT_OPF_COMBINE | MT_OPF_REWRITE
        pairs = tuple((self.key_id(k), code) for k in jsjson.js_key_order(list(props.keys())))
        return self._intern_pairs(pairs), fl

    def _intern_pairs(self, pairs: tuple) -> int:
        i = self.set_ids.get(pairs)
        if i is None:
            i = self.set_ids[pairs] = len(self.sets)
            self.sets.append(pairs)
            self._c = None
        return i

    def _incr_table(self):
        """(value_incr, incr_object) for mt_prop_table: what incr yields from each value held
        (properties.ts:33-34, `v += undefined`): the id of String(v) + "undefined" for a string,
        array or object that can be held under a key some incr op names (a value some set
        gives that key, and the strings incr makes from those, INCR_CHAIN_MAX deep at most),
        MT_VAL_UNSUP for the rest; numbers and booleans give NaN on the device (MT_VK_NUM)."""
        import json as _json
        if not self._n_incr:
            return [MT_VAL_UNSUP] * len(self.values_json), MT_VAL_UNSUP
        depth_max = min(self._n_incr, INCR_CHAIN_MAX)
        obj = self.value_id("[object Object]undefined")        # incr of a fresh consensus object
        depth = {obj: 1}
        for s_ in self.sets:
            for k, v in s_:
                if k in self._incr_keys and v >= 0:
                    depth.setdefault(v, 0)
        succ = {}
        frontier = list(depth)
        while frontier:
            nxt = []
            for v in frontier:
                if v in succ or self.values_kind[v] & MT_VK_NUM or depth[v] >= depth_max:
                    continue
                w = self.value_id(jsjson.js_to_string(_json.loads(self.values_json[v])) + "undefined")
                succ[v] = w
                if w not in depth:
                    depth[w] = depth[v] + 1
                    nxt.append(w)
            frontier = nxt
        return [succ.get(v, MT_VAL_UNSUP) for v in range(len(self.values_json))], obj

    def to_c(self) -> MtPropTable:
        if self._c is not None:
            return self._c[0]
        incr, incr_obj = self._incr_table()     # may intern strings: before the arrays are built
        off = np.zeros(len(self.sets) + 1, np.uint32)
        keys, vals = [], []
        for i, s in enumerate(self.sets):
            off[i + 1] = off[i] + len(s)
            for k, v in s:
                keys.append(k)
                vals.append(v)
        keys = np.asarray(keys, np.uint16)
        vals = np.asarray(vals, np.int32)
        kj, kk = _cstr_array([jsjson.quote(k) for k in self.keys])
        kidx = np.asarray([(jsjson.array_index(k) if jsjson.array_index(k) is not None else 0xFFFFFFFF)
                           for k in self.keys] or [0], np.uint32)
        vj, vk = _cstr_array(self.values_json)
        vf = np.asarray(self.values_falsy or [0], np.uint8)
        vc = np.asarray(self.values_class or [0], np.uint32)
        vkd = np.asarray(self.values_kind or [0], np.uint8)
        vin = np.asarray(incr or [MT_VAL_UNSUP], np.int32)
        t = MtPropTable(len(self.sets), _ptr(off), _ptr(keys), _ptr(vals), len(self.keys),
                        ctypes.cast(kj, ctypes.c_void_p).value, _ptr(kidx), len(self.values_json),
                        ctypes.cast(vj, ctypes.c_void_p).value, _ptr(vf), _ptr(vc), _ptr(vkd), _ptr(vin), incr_obj)
        self._c = (t, [off, keys, vals, kj, kk, kidx, vj, vk, vf, vc, vkd, vin])
        return t


class ClientNames:
    """Per-document interning: long client ids (strings) <-> client index
    (getOrAddShortClientId order, client.ts:658-682), and marker ids <-> the index of
    the document's idToSegment table on the device (mergeTree.ts:1095, :1175)."""

    def __init__(self):
        self.ids: dict[str, int] = {}
        self.names: list[str] = []
        self.marker_ids: dict[str, int] = {}
        self.register_ids: dict[str, int] = {}

    def register_index(self, name: str) -> int:
        """The document's index of a register name (RegisterCollection key, with the author)."""
        i = self.register_ids.get(name)
        if i is None:
            i = self.register_ids[name] = len(self.register_ids)
        return i

    def marker_define(self, mid) -> int | None:
        """A marker carrying id `mid` joins the document; None if the id is not a string
        or is already in use (which marker the reference maps then depends on later block
        updates, addNodeReferences mergeTree.ts:286-297: such documents stay off the path)."""
        if not isinstance(mid, str) or mid in self.marker_ids:
            return None
        i = self.marker_ids[mid] = len(self.marker_ids)
        return i

    def marker_lookup(self, mid) -> int:
        """getMarkerFromId: the index, or -1 when no marker with that id was mapped yet."""
        return self.marker_ids.get(mid, -1) if isinstance(mid, str) else -1

    def index(self, long_id: str) -> int:
        i = self.ids.get(long_id)
        if i is None:
            i = self.ids[long_id] = len(self.names)
            self.names.append(long_id)
        return i

    def json_literals(self) -> list[str]:
        return [jsjson.quote(n) for n in self.names]


_FIELDS = [("type", np.uint8), ("flags", np.uint8), ("client", np.uint16), ("seq", np.int32),
           ("ref_seq", np.int32), ("msn", np.int32), ("pos1", np.int32), ("pos2", np.int32),
           ("payload_off", np.uint32), ("payload_len", np.uint32), ("prop_id", np.int32)]


REL_DTYPE = np.dtype([("marker", np.int32), ("before", np.int32), ("offset", np.int32), ("pad", np.int32)])


@dataclass
class OpBatch:
    """Per-document runs of flattened op members (the mt_op_batch arrays)."""
    doc_ids: np.ndarray
    op_offsets: np.ndarray
    arrays: dict
    payload: np.ndarray
    rel: np.ndarray = field(default_factory=lambda: np.zeros(0, REL_DTYPE))
    _c: Any = field(default=None, repr=False)

    @property
    def n_ops(self) -> int:
        return int(self.op_offsets[-1])

    def to_c(self) -> MtOpBatch:
        if self._c is None:
            a = self.arrays
            self._c = MtOpBatch(len(self.doc_ids), _ptr(self.doc_ids), _ptr(self.op_offsets), self.n_ops,
                                *(_ptr(a[n]) for n, _ in _FIELDS), _ptr(self.payload), int(self.payload.size),
                                len(self.rel), _ptr(self.rel))
        return self._c

    @staticmethod
    def from_arrays(doc_ids, op_offsets, payload, **arrays) -> "OpBatch":
        arrs = {n: np.ascontiguousarray(arrays[n], dtype=t) for n, t in _FIELDS}
        return OpBatch(np.ascontiguousarray(doc_ids, np.uint32), np.ascontiguousarray(op_offsets, np.uint32),
                       arrs, np.ascontiguousarray(payload, np.uint16))


def _group_members(op) -> list:
    """applyRemoteOp's GROUP recursion (client.ts:804-812), flattened in order; every
    member carries the message's seq."""
    if not isinstance(op, dict):
        return []
    if op.get("type") == 3:
        return [m for sub in (op.get("ops") or []) for m in _group_members(sub)]
    return [op]


class BatchBuilder:
    """Packs ISequencedDocumentMessage dicts (protocol.ts:126-166) per document."""

    def __init__(self, props: PropTable, names: ClientNames):
        self.props, self.names = props, names
        self.cols = {n: [] for n, _ in _FIELDS}
        self.payload: list[int] = []
        self.doc_ids: list[int] = []
        self.offsets: list[int] = [0]
        self.rel: list[tuple] = []

    def begin_doc(self, doc_id: int):
        if len(self.doc_ids) and self.offsets[-1] == len(self.cols["type"]) and len(self.doc_ids) == len(self.offsets) - 1:
            pass
        self.doc_ids.append(doc_id)
        self.offsets.append(self.offsets[-1])

    def _emit(self, **kw):
        for n, _ in _FIELDS:
            self.cols[n].append(kw.get(n, 0))
        self.offsets[-1] += 1

    def _pos(self, op: dict, k: int):
        """(value, flag) of op.pos{k}, or of op.relativePos{k} as an index into rel[]
        (getValidOpRange, client.ts:506-523: pos wins; relativePos only when pos is
        undefined).  (None, 0): neither."""
        v = op.get(f"pos{k}")
        if v is not None:
            return int(v), 0
        rp = op.get(f"relativePos{k}")
        if not rp:
            return None, 0
        mid = rp.get("id") if isinstance(rp, dict) else None
        idx = self.names.marker_lookup(mid) if jsjson.js_truthy(mid) else -1
        off = rp.get("offset")
        self.rel.append((idx, 1 if jsjson.js_truthy(rp.get("before")) else 0,
                         int(off) if isinstance(off, (int, float)) and not isinstance(off, bool) else 0, 0))
        return len(self.rel) - 1, (MT_OPF_REL1 if k == 1 else MT_OPF_REL2)

    def _member(self, op: dict, client: int, seq: int, ref: int, msn: int, last: bool):
        t = op["type"]
        fl = MT_OPF_END_OF_MSG if last else 0
        common = dict(client=client, seq=seq, ref_seq=ref, msn=msn, prop_id=-1)
        if t == MT_OP_INSERT:
            seg = op.get("seg")
            reg = op.get("register")
            if not seg and jsjson.js_truthy(reg):
                # applyInsertOp's register branch (client.ts:425-444): with a truthy range end
                # the op copies [pos1, pos2) into the register, else it pastes the register
                pos1, rf = self._pos(op, 1)
                if pos1 is None or not isinstance(reg, str) or rf or \
                        (op.get("pos2") is None and op.get("relativePos2")):
                    self._emit(type=MT_OP_UNSUPPORTED, flags=fl, **common)
                    return
                p2 = op.get("pos2")
                ty = MT_OP_COPY if (p2 is not None and p2 != 0) else MT_OP_PASTE
                self._emit(type=ty, flags=fl, pos1=pos1, pos2=int(p2) if ty == MT_OP_COPY else 0,
                           payload_off=self.names.register_index(reg), **common)
                return
            if not seg:
                # `if (op.seg)` is falsy for "" / missing: applyInsertOp returns without
                # touching the tree (client.ts:423-444); only seq/msn advance.
                self._emit(type=MT_OP_NOOP, flags=fl, **common)
                return
            pos1, rf = self._pos(op, 1)
            if pos1 is None:
                self._emit(type=MT_OP_UNSUPPORTED, flags=fl, **common)
                return
            fl |= rf
            pos2 = 0
            if isinstance(seg, str):
                text = seg
                props = None
            elif "text" in seg:
                text, props = seg["text"], seg.get("props")
            elif "marker" in seg:
                text, props = None, seg.get("props")
                fl |= MT_OPF_MARKER
                pos2 = int(seg["marker"].get("refType", 0) or 0)
            else:
                raise ValueError(f"Unrecognized IJSONSegment type: {seg!r}")
            pid = -1
            if props is not None and jsjson.js_truthy(props):     # `if (props)` in TextSegment/Marker.make
                if not isinstance(props, dict):
                    raise ValueError(f"segment props must be an object: {props!r}")
                pid = self.props.intern(props)
                fl |= MT_OPF_SEG_PROPS
            units = jsjson.utf16_units(text) if text is not None else []
            off = len(self.payload)
            self.payload.extend(units)
            if text is None and pid >= 0 and jsjson.js_truthy(props.get(MARKER_ID_KEY)):   # Marker.getId
                m = self.names.marker_define(props[MARKER_ID_KEY])
                if m is None:
                    self._emit(type=MT_OP_UNSUPPORTED, flags=fl, **common)
                    return
                fl |= MT_OPF_MARKER_ID
                off = m
            self._emit(type=t, flags=fl, pos1=pos1, pos2=pos2, payload_off=off,
                       payload_len=len(units), **{**common, "prop_id": pid})
        elif t in (MT_OP_REMOVE, MT_OP_ANNOTATE):
            reg = op.get("register") if t == MT_OP_REMOVE else None
            pos1, f1 = self._pos(op, 1)
            pos2, f2 = self._pos(op, 2)
            if pos1 is None or pos2 is None:
                self._emit(type=MT_OP_UNSUPPORTED, flags=fl, **common)
                return
            pid = -1
            if t == MT_OP_ANNOTATE:
                # segmentPropertiesManager.ts:55-56: rewrite = op && op.name === "rewrite", any other
                # truthy combiningOp combines (properties.ts:24-62)
                cop = op.get("combiningOp")
                combine = jsjson.js_truthy(cop) and not (isinstance(cop, dict) and cop.get("name") == "rewrite")
                if jsjson.js_truthy(cop) and not combine:
                    fl |= MT_OPF_REWRITE
                if isinstance(op.get("props"), dict) and MARKER_ID_KEY in op["props"]:
                    # re-keying a marker changes idToSegment only at later block updates
                    self._emit(type=MT_OP_UNSUPPORTED, flags=fl, **common)
                    return
                if combine:
                    pid, cfl = self.props.intern_combine(op["props"], cop, seq)
                    fl |= cfl
                else:
                    pid = self.props.intern(op["props"])
            if jsjson.js_truthy(reg):                   # cut: Client.copy, then markRangeRemoved (:347-350)
                if not isinstance(reg, str):
                    self._emit(type=MT_OP_UNSUPPORTED, flags=fl, **common)
                    return
                self._emit(type=MT_OP_CUT, flags=fl | f1 | f2, pos1=pos1, pos2=pos2,
                           payload_off=self.names.register_index(reg), **common)
                return
            self._emit(type=t, flags=fl | f1 | f2, pos1=pos1, pos2=pos2, **{**common, "prop_id": pid})
        else:
            self._emit(type=MT_OP_NOOP, flags=fl, **common)

    def add_message(self, msg: dict) -> list:
        """One sequenced message (Client.applyMsg semantics, client.ts:819-841).  Returns
        the batch op index of each merge-tree member (GROUP order; [] for none)."""
        if not isinstance(msg.get("clientId"), str):
            # getOrAddShortClientId keys a RedBlackTree with localeCompare (client.ts:73, :658):
            # a null id cannot be registered once the tree holds ids
            raise ValueError("clientId must be a string on the batch path")
        client = self.names.index(msg["clientId"])
        seq, ref, msn = int(msg["sequenceNumber"]), int(msg["referenceSequenceNumber"]), int(msg["minimumSequenceNumber"])
        if msg.get("type", "op") != "op":
            self._emit(type=MT_OP_NOOP, flags=MT_OPF_END_OF_MSG, client=client, seq=seq, ref_seq=ref, msn=msn, prop_id=-1)
            return []
        members = [m for m in _group_members(msg.get("contents"))
                   if m.get("type") in (MT_OP_INSERT, MT_OP_REMOVE, MT_OP_ANNOTATE)]
        if not members:
            self._emit(type=MT_OP_NOOP, flags=MT_OPF_END_OF_MSG, client=client, seq=seq, ref_seq=ref, msn=msn, prop_id=-1)
            return []
        first = len(self.cols["type"])
        for i, m in enumerate(members):
            self._member(m, client, seq, ref, msn, i == len(members) - 1)
        return list(range(first, first + len(members)))

    def build(self) -> OpBatch:
        arrays = {n: np.asarray(self.cols[n], dtype=t) for n, t in _FIELDS}
        return OpBatch(np.asarray(self.doc_ids, np.uint32), np.asarray(self.offsets, np.uint32), arrays,
                       np.asarray(self.payload or [0], np.uint16), np.array(self.rel, dtype=REL_DTYPE))


def concat_runs(a: OpBatch, b: OpBatch) -> OpBatch:
    """Per document: a's ops then b's ops (one run per document; payloads re-packed)."""
    sl = []
    for d in range(len(a.doc_ids)):
        sl.append((a, int(a.op_offsets[d]), int(a.op_offsets[d + 1]), 0))
        sl.append((b, int(b.op_offsets[d]), int(b.op_offsets[d + 1]), len(a.payload)))
    cols = {k: np.concatenate([src.arrays[k][lo:hi] for src, lo, hi, _ in sl]) for k, _ in _FIELDS}
    po = np.concatenate([src.arrays["payload_off"][lo:hi].astype(np.int64) + base for src, lo, hi, base in sl])
    pl = cols["payload_len"].astype(np.int64)
    out_off = np.concatenate(([0], np.cumsum(pl)[:-1])) if len(pl) else np.zeros(0, np.int64)
    src_pay = np.concatenate([a.payload, b.payload])
    idx = np.repeat(po - out_off, pl) + np.arange(int(pl.sum()))
    cols["payload_off"] = out_off.astype(np.uint32)
    offs = np.zeros(len(a.doc_ids) + 1, np.uint32)
    offs[1:] = np.cumsum((a.op_offsets[1:] - a.op_offsets[:-1]) + (b.op_offsets[1:] - b.op_offsets[:-1]))
    payload = src_pay[idx] if len(idx) else np.zeros(1, np.uint16)
    return OpBatch.from_arrays(a.doc_ids, offs, payload, **cols)
