"""TEST-ONLY: sequenced ISequencedDocumentMessage streams over the real message surface.

The oracle acts as the sequencer's observer: for every message it gives the author's
perspective length getLength(refSeq, author) (MT/mergeTree.ts:1569), so positions are
valid, and it applies the message through its own JSON path (ora_apply_msg_json,
restating Client.applyMsg, MT/client.ts:790-850).  The streams exercise what the
synthetic device generator does not:

* GROUP messages (MT/client.ts:804-812): 2-4 members, one seq, each member's positions
  valid after the earlier members (the author sees its own inserts and removes);
* non-"op" messages (noop/summarize/propose) that only move seq and MSN (:840);
* remote marker inserts ({"marker":{"refType":n},"props":{...}}, MT/mergeTree.ts:640-662);
* text segments with props, "props":{} (an empty but defined map), plain strings;
* text with quotes, backslashes, control characters, non-ASCII, surrogate pairs and lone
  surrogates (splits inside a pair make more of them), long inserts past the 256-unit
  append granularity, and "\\n" (canAppend, MT/textSegment.ts:63-68);
* property keys that are array indices ("0", "2", "10": enumerated first, ascending),
  falsy values (0, "", false: the rewrite rule deletes them), null (delete), nested
  objects and arrays (matchProperties recursion, MT/properties.ts:64-95), and
  rewrite-to-empty annotates ({"name":"rewrite"} with {} or all-null props);
* client churn: authors leave and new long ids join (non-ASCII ones included), so a
  document sees many more distinct clients than are active at once;
* markers carrying a markerId and ops positioned relative to them (relativePos1,
  posFromRelativePos MT/mergeTree.ts:1949-1972).

MSN follows deli (deli/lambda.ts:348-371): the minimum over connected clients' latest
refSeq; refSeq >= MSN at send time.
"""
from __future__ import annotations

import random

from oracle_lib import OracleDoc

SPECIAL = ['"', "\\", "\n", "\t", "\r", "\x01", "\x1f", "\x7f", "/", "é", "中", " ", "😀", "𝄞",
           "\ud800", "\udfff", "\udc00", " ", "<", "&"]
KEYS = ["0", "1", "2", "10", "k", "bold", "a b", "ключ", "x\"y", "4294967295", "01"]
# wide property maps (the "wide_props" surface): 45 more keys, index-like ones among them, so
# one segment's map grows well past 16 keys (56 distinct keys at most: within MT_PKEYS = 64)
WIDE_KEYS = KEYS + [f"w{i}" for i in range(36)] + ["3", "7", "11", "12", "40", "99", "100", "1000", "255"]
# very wide maps (the "very_wide_props" surface): 220 distinct keys, so one segment's map grows
# past a wave's 64 lanes (applyPropSetWide) toward MT_MAX_PROP_KEYS = 256
VERY_WIDE_KEYS = WIDE_KEYS + [f"v{i}" for i in range(164)]
VALUES = ["s", "ü", "", 0, 1, -3, 1.5, 1e21, 0.25, True, False, {"a": 1}, [1, 2], {"0": "x", "b": [True]},
          {"n": None}, "😀"]
# remote combining ops (the "combine" surface, MT/properties.ts:24-62 via
# segmentPropertiesManager.ts:98-103): "incr" works on keys whose values are numbers or booleans
# (NaN results) and strings, arrays and objects (string concatenation with "undefined");
# "consensus" and ops of other names on keys holding anything but objects whose seq is -1 (fresh
# {value: undefined, seq} objects, defaults, undefined values).  String minValues stay out of
# the streams (a held string's incr result compared with one is off the batch path).
INCR_KEYS = ["n0", "n1", "3"]
CONS_KEYS = ["v0", "v1", "7"]
NUM_VALUES = [0, 1, -2, 2.5, True, False, 1e21, 3, 4, "s", "ü😀", {"a": 1}, [1, [2, "x"]]]
INCR_DEFAULTS = [None, 0, 5, True, 2.5, "v", [1, 2], "__absent__", "__absent__"]
CONS_DEFAULTS = ["__absent__", "__absent__", 7, "x", {"a": 1}, {"value": 3, "seq": -1}, [1, 2], {"seq": 4}, False]
OTHER_DEFAULTS = ["__absent__", None, 1, "z", {"k": [1]}]


class StreamGen:
    def __init__(self, seed: int, clients: int = 4, lag: int = 12, churn: float = 0.0, p_nonop: float = 0.06,
                 p_group: float = 0.15, p_marker: float = 0.08, p_annotate: float = 0.2, p_remove: float = 0.3,
                 p_special: float = 0.25, long_every: int = 40, max_ins: int = 9, id_prefix: str = "cli",
                 max_total_clients: int | None = None, p_marker_id: float = 0.0, p_relative: float = 0.0,
                 capture: bool = False, p_register: float = 0.0, p_wide: float = 0.0, reg_names: int = 0,
                 reg_span: int = 10, p_combine: float = 0.0, p_vwide: float = 0.0):
        self.rng = random.Random(seed)
        self.lag, self.churn, self.p_nonop, self.p_group = lag, churn, p_nonop, p_group
        self.p_marker, self.p_annotate, self.p_remove, self.p_special = p_marker, p_annotate, p_remove, p_special
        self.long_every, self.max_ins = long_every, max_ins
        self.id_prefix = id_prefix
        self.max_total = max_total_clients
        self.p_marker_id, self.p_relative = p_marker_id, p_relative
        self.marker_ids: list[str] = []           # ids of markers inserted so far (idToSegment)
        self.p_register = p_register
        self.p_wide = p_wide
        # register names per client (0: REGS) and the longest copy / cut range
        self.reg_names = [f"r{i}" for i in range(reg_names)] if reg_names else self.REGS
        self.reg_span = reg_span
        self.p_combine = p_combine
        self.p_vwide = p_vwide
        self.total = 0
        self.active: dict[str, int] = {}          # long id -> latest refSeq
        for _ in range(clients):
            self._join(0)
        self.cur = 0
        self.msn = 0
        self.obs = OracleDoc(True)
        if capture:
            self.obs.delta_capture(True)
        self.msgs: list[dict] = []

    # -- clients ----------------------------------------------------------------
    def _join(self, ref: int):
        k = self.total
        self.total += 1
        nm = f"{self.id_prefix}-{k}" if k % 5 else f"ü{self.id_prefix}-{k}-😀"
        self.active[nm] = ref
        return nm

    # -- content ----------------------------------------------------------------
    def _text(self, n: int) -> str:
        r = self.rng
        out = []
        for _ in range(n):
            out.append(r.choice(SPECIAL) if r.random() < self.p_special else chr(97 + r.randrange(26)))
        return "".join(out)

    def _props(self, allow_null=True) -> dict:
        r = self.rng
        d = {}
        wide = self.p_wide > 0 and r.random() < self.p_wide     # (no draw otherwise: other surfaces keep their streams)
        vwide = self.p_vwide > 0 and r.random() < self.p_vwide
        for _ in range(r.randint(60, 140) if vwide else (r.randint(18, 45) if wide else r.randint(1, 3))):
            k = r.choice(VERY_WIDE_KEYS if vwide else (WIDE_KEYS if wide else KEYS))
            d[k] = None if (allow_null and r.random() < 0.2) else r.choice(VALUES)
        if self.p_combine and r.random() < 0.5:          # plain values on the combining ops' keys
            if r.random() < 0.5:
                d[r.choice(INCR_KEYS)] = None if (allow_null and r.random() < 0.2) else r.choice(NUM_VALUES)
            else:
                d[r.choice(CONS_KEYS)] = None if (allow_null and r.random() < 0.2) else r.choice(VALUES)
        return d

    def _combining(self) -> tuple[dict, dict]:
        """(props, combiningOp) of a remote annotate with a combining op other than rewrite."""
        r = self.rng
        x = r.random()
        if x < 0.45:
            cop, keys, defs = {"name": "incr"}, INCR_KEYS, INCR_DEFAULTS
            if r.random() < 0.3:
                cop["minValue"] = r.choice([3, 0, -1])           # NaN < minValue is false
        elif x < 0.85:
            cop, keys, defs = {"name": "consensus"}, CONS_KEYS, CONS_DEFAULTS
        else:
            cop, keys, defs = r.choice([{"name": "max"}, {"name": 5}, {}]), CONS_KEYS, OTHER_DEFAULTS
        dv = r.choice(defs)
        if dv != "__absent__":
            cop["defaultValue"] = dv
        # the op's values are unused (combine gets undefined); keys only, any values
        props = {k: r.choice(VALUES + [None]) for k in r.sample(keys, r.randint(1, 2))}
        return props, cop

    def _insert(self, L: int, k: int) -> tuple[dict, int]:
        r = self.rng
        pos = r.randint(0, L)
        if r.random() < self.p_marker:
            seg = {"marker": {"refType": r.choice([0, 1, 2, 4, 0x40])}}
            if r.random() < 0.7:
                seg["props"] = self._props(allow_null=False)
            if r.random() < self.p_marker_id:            # paragraph-marker style ids (Marker.getId)
                mid = f"m{len(self.marker_ids) + len(self.pending_ids)}-ü"
                seg["props"] = {**seg.get("props", {}), "markerId": mid}
                self.pending_ids.append(mid)
            return {"type": 0, "pos1": pos, "seg": seg}, 1
        n = r.randint(257, 300) if (self.long_every and k % self.long_every == self.long_every - 1) else \
            r.randint(1, self.max_ins)
        text = self._text(n)
        if text and text[-1] == "\ud800" and r.random() < 0.5:
            text = text[:-1] + "\n"
        units = len(text.encode("utf-16-le", "surrogatepass")) // 2
        x = r.random()
        if x < 0.6:
            seg = text
        elif x < 0.7:
            seg = {"text": text, "props": {}}
        else:
            seg = {"text": text, "props": self._props()}
        return {"type": 0, "pos1": pos, "seg": seg}, units

    def _range(self, L: int, ty: int) -> tuple[dict, int]:
        r = self.rng
        s = r.randrange(L)
        e = min(L, s + 1 + r.randrange(12))
        if ty == 1:
            return {"type": 1, "pos1": s, "pos2": e}, -(e - s)
        op = {"type": 2, "pos1": s, "pos2": e}
        if self.p_combine and r.random() < self.p_combine:
            op["props"], op["combiningOp"] = self._combining()
            return op, 0
        x = r.random()
        if x < 0.1:
            op["props"] = {}
            op["combiningOp"] = {"name": "rewrite"}
        elif x < 0.2:
            op["props"] = {k: None for k in r.sample(KEYS, 2)}
            op["combiningOp"] = {"name": "rewrite"}
        else:
            op["props"] = self._props()
            if r.random() < 0.15:
                op["combiningOp"] = {"name": "rewrite"}
        return op, 0

    REGS = ["clip", "ü-reg"]

    def _register(self, L: int) -> tuple[dict, int] | None:
        """Register ops (MT/client.ts:347-350, :425-444): cut (remove with a register), copy
        (insert with a register and a range end) and paste (insert with a register).  A paste
        is emitted only for a register the oracle holds unpasted and free of clones of
        removed segments: a second paste of one register re-links the same segment objects in
        the reference (not modelled), and pasted clones of removed segments are off the
        engine's path.  Its length change is the clones' total cachedLength."""
        r = self.rng
        name = r.choice(self.reg_names)
        x = r.random()
        if x < 0.45:
            info = self.obs.register_info(self._author, name)
            if info["n"] > 0 and not info["pasted"] and not info["removed"]:
                return {"type": 0, "pos1": r.randint(0, L), "register": name}, info["len"]
        if L == 0:
            return None
        s = r.randrange(L)
        e = min(L, s + 1 + r.randrange(self.reg_span))
        if x < 0.75:
            return {"type": 0, "pos1": s, "pos2": e, "register": name}, 0
        return {"type": 1, "pos1": s, "pos2": e, "register": name}, -(e - s)

    def _member(self, L: int, k: int) -> tuple[dict, int]:
        if self.p_register and self._first_member and self.rng.random() < self.p_register:
            got = self._register(L)
            if got is not None:
                return got
        x = self.rng.random()
        if L == 0 or x >= self.p_remove + self.p_annotate:
            op, dl = self._insert(L, k)
        else:
            op, dl = self._range(L, 1 if x < self.p_remove else 2)
        if self.marker_ids and self._first_member and self.rng.random() < self.p_relative:
            op, dl = self._relative(op, dl, L)
        return op, dl

    def _relative(self, op: dict, dl: int, L: int) -> tuple[dict, int]:
        """Re-express the op's start relative to a marker id (IRelativePosition,
        MT/ops.ts:46-61) when posFromRelativePos (computed by the oracle under the
        author's perspective) gives a valid start; first member of a message only (later
        GROUP members see the earlier members' edits)."""
        r = self.rng
        rp = {"id": r.choice(self.marker_ids)}
        if r.random() < 0.5:
            rp["before"] = True
        if r.random() < 0.5:
            rp["offset"] = r.randint(0, 3)
        p = self.obs.rel_pos_of(self._ref, self._author, rp)
        rest = {k: v for k, v in op.items() if k not in ("type", "pos1")}
        if op["type"] == 0:
            if 0 <= p <= L:
                return {"type": 0, "relativePos1": rp, **rest}, dl
            return op, dl
        if 0 <= p < op["pos2"]:
            return {"type": op["type"], "relativePos1": rp, **rest}, (-(op["pos2"] - p) if op["type"] == 1 else 0)
        return op, dl

    # -- one sequenced message ----------------------------------------------------
    def step(self) -> dict:
        r = self.rng
        k = len(self.msgs)
        if self.churn and r.random() < self.churn and len(self.active) > 1 and \
                (self.max_total is None or self.total < self.max_total):
            del self.active[r.choice(sorted(self.active))]                # leave
            self._join(self.cur)                                          # a new long id joins
        a = r.choice(sorted(self.active))
        ref = max(self.cur - r.randint(0, self.lag), self.active[a], self.msn)
        self.active[a] = ref
        msn = min(self.active.values())
        seq = self.cur + 1
        msg = dict(clientId=a, sequenceNumber=seq, referenceSequenceNumber=ref, minimumSequenceNumber=msn)
        self._author, self._ref, self.pending_ids = a, ref, []
        if r.random() < self.p_nonop:
            msg["type"] = r.choice(["noop", "summarize", "propose"])
            msg["contents"] = None
        else:
            L = self.obs.get_length_of(ref, a)
            members = []
            for i in range(r.randint(2, 4) if r.random() < self.p_group else 1):
                self._first_member = i == 0
                op, dl = self._member(L, k)
                members.append(op)
                L += dl
            msg["type"] = "op"
            msg["contents"] = members[0] if len(members) == 1 else {"type": 3, "ops": members}
        st = self.obs.apply_msg(msg)
        if st:
            raise RuntimeError(f"oracle status {st:#x} at message {k}: {msg}")
        self.cur, self.msn = seq, msn
        self.marker_ids.extend(self.pending_ids)          # mapped once the insert applied
        self.msgs.append(msg)
        return msg

    def run(self, n: int) -> list[dict]:
        for _ in range(n):
            self.step()
        return self.msgs


def stream(seed: int, n: int, **kw):
    """(messages, oracle observer after all of them)."""
    g = StreamGen(seed, **kw)
    g.run(n)
    return g.msgs, g.obs
