"""ctypes binding of the CPU oracle (oracle/mtoracle.cpp).  TEST INFRASTRUCTURE.

Used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess

import numpy as np

from fluidframework_amd.batch import MtGenParams, MtOpBatch, MtPropTable, OpBatch, PropTable

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "oracle", "mtoracle.cpp")
LIB = os.path.join(ROOT, "oracle", "_build", "libmtoracle.so")


def build_oracle(force: bool = False) -> str:
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        tmp = f"{LIB}.{os.getpid()}.tmp"  # rename into place: parallel workers never load a partial file
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", tmp, SRC])
        os.replace(tmp, LIB)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(build_oracle())
        P, I32, U32, U64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64
        L.ora_new.restype = P
        L.ora_new.argtypes = [ctypes.c_int]
        L.ora_free.argtypes = [P]
        L.ora_free_buf.argtypes = [P]
        L.ora_set_props.argtypes = [P, ctypes.POINTER(MtPropTable)]
        L.ora_set_client_names.argtypes = [P, U32, P]
        L.ora_apply_run.restype = U32
        L.ora_apply_run.argtypes = [P, ctypes.POINTER(MtOpBatch), U32]
        L.ora_local_insert.argtypes = [P, I32, P, U32, I32, I32]
        L.ora_local_remove.argtypes = [P, I32, I32]
        L.ora_local_annotate.argtypes = [P, I32, I32, I32, I32]
        L.ora_load_snapshot.restype = ctypes.c_int
        L.ora_load_snapshot.argtypes = [P, U32, P]
        L.ora_apply_msg_json.restype = U32
        L.ora_apply_msg_json.argtypes = [P, ctypes.c_char_p]
        L.ora_register_info_json.restype = P
        L.ora_register_info_json.argtypes = [P, ctypes.c_char_p, ctypes.c_char_p]
        L.ora_rel_pos_json.restype = I32
        L.ora_rel_pos_json.argtypes = [P, I32, ctypes.c_char_p, ctypes.c_char_p]
        L.ora_channel_process.restype = U32
        L.ora_channel_process.argtypes = [P, ctypes.c_char_p]
        L.ora_channel_stash_json.restype = P
        L.ora_channel_stash_json.argtypes = [P, I32]
        L.ora_delta_capture.argtypes = [P, ctypes.c_int]
        L.ora_delta_json.restype = P
        L.ora_delta_json.argtypes = [P]
        L.ora_get_length_json.restype = I32
        L.ora_get_length_json.argtypes = [P, I32, ctypes.c_char_p]
        L.ora_get_length.restype = I32
        L.ora_get_length.argtypes = [P, I32, I32]
        L.ora_snapshot_v1.restype = P
        L.ora_snapshot_v1.argtypes = [P, I32, I32, ctypes.POINTER(U64), ctypes.POINTER(U64)]
        L.ora_snapshot_legacy.restype = P
        L.ora_snapshot_legacy.argtypes = [P, I32, I32, ctypes.POINTER(U64), ctypes.POINTER(U64)]
        L.ora_get_text.restype = P
        L.ora_get_text.argtypes = [P, ctypes.POINTER(U64)]
        L.ora_dump_segments.restype = P
        L.ora_dump_segments.argtypes = [P, ctypes.POINTER(U32)]
        L.ora_stats.argtypes = [P, P]
        L.ora_generate_doc.restype = U32
        L.ora_generate_doc.argtypes = [ctypes.POINTER(MtGenParams), U32, ctypes.POINTER(MtPropTable)] + [P] * 12 + [U32, P]
        L.ora_set_verify.argtypes = [ctypes.c_int]
        L.ora_verify_result.restype = ctypes.c_longlong
        L.ora_verify_result.argtypes = [ctypes.POINTER(ctypes.c_longlong)]
        L.ora_replay_batch.restype = ctypes.c_double
        L.ora_replay_batch.argtypes = [ctypes.POINTER(MtOpBatch), ctypes.POINTER(MtPropTable), ctypes.c_int, P, P, P]
        L.ora_counters.argtypes = [P, P]
        L.ora_containing_segment.restype = ctypes.c_int
        L.ora_get_length_exact.restype = I32
        L.ora_get_length_exact.argtypes = [P, I32, I32]
        L.ora_client_name.restype = ctypes.c_char_p
        L.ora_client_name.argtypes = [P, I32]
        L.ora_containing_segment.argtypes = [P, I32, I32, I32, ctypes.c_char_p, P, ctypes.POINTER(P)]
        L.ora_set_snapshot_chunk.argtypes = [P, ctypes.c_double]
        _lib = L
    return _lib


def parse_blobs(buf: int, total: int) -> list[bytes]:
    raw = ctypes.string_at(buf, total)
    n = struct.unpack_from("<I", raw, 0)[0]
    off, out = 4, []
    for _ in range(n):
        ln = struct.unpack_from("<Q", raw, off)[0]
        off += 8
        out.append(raw[off:off + ln])
        off += ln
    return out


class OracleDoc:
    """One reference-semantics document (passive observer or detached local)."""

    def __init__(self, collaborating: bool = True, props: PropTable | None = None, names: list[str] | None = None):
        self.L = lib()
        self.h = self.L.ora_new(1 if collaborating else 0)
        self.props = props
        if props is not None:
            self.set_props(props)
        if names is not None:
            self.set_names(names)

    def __del__(self):
        try:
            if self.h:
                self.L.ora_free(self.h)
        except Exception:
            pass

    def set_props(self, props: PropTable):
        self.props = props
        self.L.ora_set_props(self.h, ctypes.byref(props.to_c()))

    def set_names(self, json_literals: list[str]):
        arr = (ctypes.c_char_p * max(1, len(json_literals)))(*[s.encode() for s in json_literals])
        self._names = arr
        self.L.ora_set_client_names(self.h, len(json_literals), ctypes.cast(arr, ctypes.c_void_p))

    def set_snapshot_chunk(self, chunk_size: float):
        """options.mergeTreeSnapshotChunkSize of the document's MergeTree (snapshotV1.ts:55)."""
        self.L.ora_set_snapshot_chunk(self.h, float(chunk_size))

    def apply_msg(self, msg: dict) -> int:
        """Client.applyMsg on the message itself (JSON; the oracle parses and dispatches it)."""
        import json
        return int(self.L.ora_apply_msg_json(self.h, json.dumps(msg, ensure_ascii=True).encode()))

    def channel_process(self, msg: dict) -> int:
        """SharedSegmentSequence.processMergeTreeMsg, legacy format (sequence.ts:604-642), on
        the oracle's own restatement: apply, then stash (transformed when refSeq != seq - 1)."""
        import json
        return int(self.L.ora_channel_process(self.h, json.dumps(msg, ensure_ascii=True).encode()))

    def channel_stash(self, min_seq: int):
        """snapshotMergeTree's catch-up messages as the JSON text of the blob (None: no blob)."""
        buf = self.L.ora_channel_stash_json(self.h, min_seq)
        if not buf:
            return None
        out = ctypes.string_at(buf).decode("utf-8")
        self.L.ora_free_buf(buf)
        return out

    def get_length_of(self, ref_seq: int, client_id: str) -> int:
        """getLength(refSeq, shortId(client_id)) under the oracle's own registration."""
        from fluidframework_amd.jsjson import quote
        return int(self.L.ora_get_length_json(self.h, ref_seq, quote(client_id).encode("utf-8", "surrogatepass")))

    def delta_capture(self, on: bool = True):
        self.L.ora_delta_capture(self.h, 1 if on else 0)

    def delta_records(self) -> list:
        """[[op, kind, pos, len, b, propsBefore, propsAfter], ...] (props as parsed JSON)."""
        import json
        buf = self.L.ora_delta_json(self.h)
        out = json.loads(ctypes.string_at(buf).decode("utf-8", "surrogatepass"))
        self.L.ora_free_buf(buf)
        return out

    def register_info(self, client_id: str, name: str) -> dict:
        """The oracle's RegisterCollection entry (client_id, name): {"n": -1} when absent, else
        {"n", "len", "removed", "pasted"}."""
        import json
        from fluidframework_amd.jsjson import quote
        buf = self.L.ora_register_info_json(self.h, quote(client_id).encode("utf-8", "surrogatepass"),
                                            quote(name).encode("utf-8", "surrogatepass"))
        out = json.loads(ctypes.string_at(buf).decode())
        self.L.ora_free_buf(buf)
        return out

    def rel_pos_of(self, ref_seq: int, client_id: str, relpos: dict) -> int:
        """posFromRelativePos under (ref_seq, client_id)'s perspective; -1: unknown id."""
        import json
        from fluidframework_amd.jsjson import quote
        return int(self.L.ora_rel_pos_json(self.h, ref_seq, quote(client_id).encode("utf-8", "surrogatepass"),
                                           json.dumps(relpos, ensure_ascii=True).encode()))

    def apply_run(self, batch: OpBatch, run: int) -> int:
        return int(self.L.ora_apply_run(self.h, ctypes.byref(batch.to_c()), run))

    # detached-string local edits (SharedString before attach)
    def insert_text(self, pos: int, text: str, props: dict | None = None):
        from fluidframework_amd.jsjson import utf16_units
        u = np.asarray(utf16_units(text) or [0], np.uint16)
        pid = self.props.intern(props) if props else -1
        if pid >= 0:
            self.set_props(self.props)
        return self.L.ora_local_insert(self.h, pos, u.ctypes.data, len(text.encode("utf-16-le", "surrogatepass")) // 2, -1, pid)

    def insert_marker(self, pos: int, ref_type: int, props: dict | None = None):
        pid = self.props.intern(props) if props else -1
        if pid >= 0:
            self.set_props(self.props)
        return self.L.ora_local_insert(self.h, pos, None, 0, ref_type, pid)

    def annotate_range(self, start: int, end: int, props: dict, rewrite: bool = False):
        pid = self.props.intern(props)
        self.set_props(self.props)
        return self.L.ora_local_annotate(self.h, start, end, pid, 1 if rewrite else 0)

    def remove_range(self, start: int, end: int):
        return self.L.ora_local_remove(self.h, start, end)

    def load_snapshot(self, blobs: list) -> int:
        """SnapshotLoader on a document made with collaborating=False: blobs[0] is
        the header blob, then the body chunks in orderedChunkMetadata order."""
        enc = [b if isinstance(b, bytes) else b.encode() for b in blobs]
        arr = (ctypes.c_char_p * len(enc))(*enc)
        return int(self.L.ora_load_snapshot(self.h, len(enc), ctypes.cast(arr, ctypes.c_void_p)))

    def get_length(self, ref_seq: int = 0, client: int = -1) -> int:
        return int(self.L.ora_get_length(self.h, ref_seq, client))

    def snapshot(self, msn: int = 0, seq: int = 0, legacy: bool = False):
        dig, tot = ctypes.c_uint64(), ctypes.c_uint64()
        fn = self.L.ora_snapshot_legacy if legacy else self.L.ora_snapshot_v1
        buf = fn(self.h, msn, seq, ctypes.byref(dig), ctypes.byref(tot))
        if not buf:
            raise RuntimeError("oracle: SnapshotV1's chunk loop never ends (chunk size no length is below)")
        blobs = parse_blobs(buf, tot.value)
        self.L.ora_free_buf(buf)
        return blobs, dig.value

    def get_text(self) -> str:
        n = ctypes.c_uint64()
        buf = self.L.ora_get_text(self.h, ctypes.byref(n))
        raw = ctypes.string_at(buf, n.value * 2)
        self.L.ora_free_buf(buf)
        return raw.decode("utf-16-le", "surrogatepass")

    def dump(self) -> np.ndarray:
        n = ctypes.c_uint32()
        buf = self.L.ora_dump_segments(self.h, ctypes.byref(n))
        a = np.frombuffer(ctypes.string_at(buf, n.value * 48), np.int32).reshape(-1, 12).copy()
        self.L.ora_free_buf(buf)
        return a

    def containing_segment(self, pos: int, ref_seq: int = -1, client: int = -1, client_id: str | None = None):
        """getContainingSegment (+ resolveRemoteClientPosition) under stream client `client`'s
        perspective at ref_seq (ref_seq < 0: the local client at currentSeq; client_id: the
        client with that long id instead): (16 int32 in mt_seg_info order, the segment's JSON
        text or None)."""
        from fluidframework_amd.jsjson import quote
        out = np.zeros(16, np.int32)
        js = ctypes.c_void_p()
        lit = quote(client_id).encode("utf-8", "surrogatepass") if client_id is not None else None
        self.L.ora_containing_segment(self.h, pos, ref_seq, client, lit, out.ctypes.data, ctypes.byref(js))
        txt = None
        if js.value:
            txt = ctypes.string_at(js.value).decode("utf-8", "surrogatepass")
            self.L.ora_free_buf(js.value)
        return out, txt

    def client_name(self, short_id: int):
        """The long id of one of the oracle's short client ids (None if none)."""
        import json
        v = self.L.ora_client_name(self.h, short_id)
        return None if v is None else json.loads(v.decode("utf-8", "surrogatepass"))

    def counters(self) -> dict:
        """The §8(d) algorithmic counters (mt_doc_counters order) by the oracle's own count."""
        out = np.zeros(6, np.uint64)
        self.L.ora_counters(self.h, out.ctypes.data)
        return dict(zip(("ops", "msgs", "ins_units", "rows_rw", "depth", "scoured"), (int(x) for x in out)))

    def stats(self):
        out = np.zeros(4, np.int32)
        self.L.ora_stats(self.h, out.ctypes.data)
        return out


def gen_params(seed=1, n_docs=1, ops=1000, clients=2, lag=8, ins=55, rem=45, ins_len=8, rem_len=16,
               ann_sets=1, rewrite=0) -> MtGenParams:
    return MtGenParams(seed, n_docs, ops, clients, lag, ins, rem, ins_len, rem_len, ann_sets, rewrite)


def generate(params: MtGenParams, props: PropTable, docs=None, keep=False, ops_per_doc=None, clients_per_doc=None,
             threads: int = 1):
    """Generate streams with the oracle as sequencer+observer; returns (OpBatch, [status], [OracleDoc]).
    ops_per_doc / clients_per_doc: per-document counts (indexed by position in docs),
    as mt_generate_docs takes them.  threads > 1: documents are generated concurrently
    (each document's stream is independent; ctypes releases the GIL)."""
    L = lib()
    docs = list(range(params.n_docs)) if docs is None else list(docs)
    if threads > 1 and len(docs) > 1:
        return _generate_threaded(params, props, docs, keep, ops_per_doc, clients_per_doc, threads)
    cols = {k: [] for k in ("type", "flags", "client", "seq", "ref_seq", "msn", "pos1", "pos2",
                            "payload_off", "payload_len", "prop_id")}
    payloads, offs, stats, kept = [], [0], [], []
    base = 0
    for j, d in enumerate(docs):
        pj = MtGenParams(*(getattr(params, f) for f, _ in MtGenParams._fields_))
        if ops_per_doc is not None:
            pj.ops_per_doc = int(ops_per_doc[j])
        if clients_per_doc is not None:
            pj.clients = int(clients_per_doc[j])
        n = pj.ops_per_doc
        a = dict(type=np.zeros(n, np.uint8), flags=np.zeros(n, np.uint8), client=np.zeros(n, np.uint16),
                 seq=np.zeros(n, np.int32), ref_seq=np.zeros(n, np.int32), msn=np.zeros(n, np.int32),
                 pos1=np.zeros(n, np.int32), pos2=np.zeros(n, np.int32), payload_off=np.zeros(n, np.uint32),
                 payload_len=np.zeros(n, np.uint32), prop_id=np.zeros(n, np.int32))
        pay = np.zeros(max(1, n * params.ins_len_max), np.uint16)
        kp = ctypes.c_void_p()
        st = L.ora_generate_doc(ctypes.byref(pj), d, ctypes.byref(props.to_c()),
                                *(a[k].ctypes.data for k in ("type", "flags", "client", "seq", "ref_seq", "msn",
                                                             "pos1", "pos2", "payload_off", "payload_len", "prop_id")),
                                pay.ctypes.data, base, ctypes.byref(kp) if keep else None)
        used = int(a["payload_len"].sum())
        payloads.append(pay[:used])
        base += used
        for k in cols:
            cols[k].append(a[k])
        offs.append(offs[-1] + n)
        stats.append(int(st))
        if keep:
            od = OracleDoc.__new__(OracleDoc)
            od.L, od.h, od.props = L, kp.value, props
            kept.append(od)
    batch = OpBatch.from_arrays(np.asarray(docs, np.uint32), np.asarray(offs, np.uint32),
                                np.concatenate(payloads) if payloads else np.zeros(1, np.uint16),
                                **{k: np.concatenate(v) for k, v in cols.items()})
    return batch, stats, kept


def _generate_threaded(params, props, docs, keep, ops_per_doc, clients_per_doc, threads):
    """generate() over a thread pool: each document generated alone (payload base 0), then
    the runs concatenated with their payload offsets rebased."""
    from concurrent.futures import ThreadPoolExecutor

    def one(j):
        return generate(params, props, docs=[docs[j]], keep=keep,
                        ops_per_doc=None if ops_per_doc is None else [ops_per_doc[j]],
                        clients_per_doc=None if clients_per_doc is None else [clients_per_doc[j]])

    with ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(one, range(len(docs))))
    bs = [p[0] for p in parts]
    pay_base = np.concatenate(([0], np.cumsum([len(b.payload) for b in bs])[:-1])).astype(np.int64)
    cols = {}
    for k in bs[0].arrays:
        cols[k] = np.concatenate([b.arrays[k] for b in bs])
    cols["payload_off"] = np.concatenate([b.arrays["payload_off"].astype(np.int64) + o
                                          for b, o in zip(bs, pay_base)]).astype(np.uint32)
    offs = np.concatenate(([0], np.cumsum([int(b.op_offsets[-1]) for b in bs]))).astype(np.uint32)
    batch = OpBatch.from_arrays(np.asarray(docs, np.uint32), offs, np.concatenate([b.payload for b in bs]), **cols)
    return batch, [p[1][0] for p in parts], [p[2][0] for p in parts] if keep else []


def replay(batch: OpBatch, props: PropTable, names: list[str] | None = None):
    """Apply every run on a fresh passive-observer document; returns docs."""
    docs = []
    for r in range(len(batch.doc_ids)):
        d = OracleDoc(True, props, names)
        st = d.apply_run(batch, r)
        docs.append((d, st))
    return docs
