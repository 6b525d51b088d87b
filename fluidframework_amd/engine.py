"""Python host of the MI355X merge-tree engine (ctypes over include/mtgpu.h).

``Engine`` owns one engine context (one GPU).  ``MergeTreeClient`` mirrors the
reference ``Client`` API for the passive-observer replay path
(packages/dds/merge-tree/src/client.ts): ``applyMsg``, ``updateSeqNumbers``,
``getLength``, ``getText``, ``snapshot``, ``getCurrentSeq`` — with the
difference that messages are queued and applied in batches on the device
(``flush``), many documents at a time.  Protocol violations that the reference
reports by throwing (common-utils assert.ts:12-16) raise ``MergeTreeError``
when the document's status is read.

The product path has no CPU fallback: if ``libmtgpu.so`` (built by
``__graft_entry__.build()``) is missing or no GPU is visible, constructing an
``Engine`` raises.
"""
from __future__ import annotations

import ctypes
import json
import os
from dataclasses import dataclass

import numpy as np

from . import jsjson
from .batch import (BatchBuilder, ClientNames, MtGenParams, MtOpBatch, MtPropTable, OpBatch, PropTable,
                    status_names)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmtgpu.so")


class MergeTreeError(RuntimeError):
    pass


class ReferenceTypeError(MergeTreeError, TypeError):
    """Where the reference's Client throws a TypeError (MT_DS_THROWS): a consensus combine on a
    segment without the key and a null defaultValue reads null.seq (properties.ts:51-52)."""


class ExchangeError(MergeTreeError):
    """Exchanged document rows whose checksum differs from the sender's (MT_E_EXCHANGE)."""

    def __init__(self, msg, bad_runs):
        super().__init__(msg)
        self.bad_runs = bad_runs


class MtLimits(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("max_docs", "rows_per_doc", "blocks_per_doc", "text_per_doc",
                                               "propsets_per_doc", "heap_per_doc", "window_per_doc",
                                               "markers_per_doc", "register_rows_per_doc")]


class MtDocCounters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("ops", "msgs", "ins_units", "rows_rw", "depth", "scoured")]


def _bind(lib, prefix: str):
    P, U32, I32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32

    def f(name, res, args):
        try:
            fn = getattr(lib, prefix + name)
        except AttributeError:      # an older build of the library (A/B runs): fails only if called
            return None
        fn.restype, fn.argtypes = res, args
        return fn

    return dict(
        create=f("create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(MtLimits), ctypes.POINTER(P)]),
        create_docs=f("create_docs", ctypes.c_int, [ctypes.c_int, U32, P, ctypes.POINTER(P)]),
        pool_bytes=f("pool_bytes", ctypes.c_int, [P, ctypes.POINTER(ctypes.c_uint64)]),
        checkpoint=f("checkpoint", ctypes.c_int, [P]),
        restore=f("restore", ctypes.c_int, [P]),
        destroy=f("destroy", None, [P]),
        last_error=f("last_error", ctypes.c_char_p, [P]),
        docs_open=f("docs_open", ctypes.c_int, [P, U32, U32]),
        doc_pools=f("doc_pools", ctypes.c_int, [P, U32, P, P]),
        set_residency=f("set_residency", ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
        set_size_class=f("set_size_class", ctypes.c_int, [P, U32]),
        set_partition=f("set_partition", ctypes.c_int, [P, U32, U32]),
        last_partition=f("last_partition", ctypes.c_int, [P, ctypes.POINTER(U32), ctypes.POINTER(U32)]),
        plan_partition=f("plan_partition", ctypes.c_int, [P, U32, U32, ctypes.POINTER(U32), ctypes.POINTER(U32),
                                                          ctypes.POINTER(ctypes.c_double)]),
        set_continuation=f("set_continuation", ctypes.c_int, [P, U32]),
        set_props=f("set_props", ctypes.c_int, [P, ctypes.POINTER(MtPropTable)]),
        set_client_names=f("set_client_names", ctypes.c_int, [P, U32, P]),
        set_doc_client_names=f("set_doc_client_names", ctypes.c_int, [P, U32, U32, P]),
        apply_batch=f("apply_batch", ctypes.c_int, [P, ctypes.POINTER(MtOpBatch)]),
        upload_batch=f("upload_batch", ctypes.c_int, [P, ctypes.POINTER(MtOpBatch)]),
        replay_resident=f("replay_resident", ctypes.c_int, [P]),
        last_cursors=f("last_cursors", ctypes.c_int, [P, U32, P]),
        last_replay_ms=f("last_replay_ms", ctypes.c_int, [P, ctypes.POINTER(ctypes.c_float)]),
        update_seq=f("update_seq", ctypes.c_int, [P, U32, P, P, P]),
        sync=f("sync", ctypes.c_int, [P]),
        doc_status=f("doc_status", ctypes.c_int, [P, U32, P, P]),
        doc_counters_get=f("doc_counters_get", ctypes.c_int, [P, U32, P, P]),
        get_length=f("get_length", ctypes.c_int, [P, U32, P, P, P, P]),
        snapshot_v1=f("snapshot_v1", ctypes.c_int, [P, U32, P, P, P, P, ctypes.POINTER(P), ctypes.POINTER(P),
                                                    ctypes.POINTER(P)]),
        snapshot_legacy=f("snapshot_legacy", ctypes.c_int, [P, U32, P, P, P, P, ctypes.POINTER(P),
                                                            ctypes.POINTER(P), ctypes.POINTER(P)]),
        snapshot_digests=f("snapshot_digests", ctypes.c_int, [P, U32, P, P, P, P, ctypes.c_int]),
        get_text=f("get_text", ctypes.c_int, [P, U32, P, ctypes.POINTER(P), ctypes.POINTER(P)]),
        dump_segments=f("dump_segments", ctypes.c_int, [P, U32, ctypes.POINTER(P), ctypes.POINTER(U32)]),
        free=f("free", None, [P]),
        generate=f("generate", ctypes.c_int, [P, ctypes.POINTER(MtGenParams)]),
        generate_docs=f("generate_docs", ctypes.c_int, [P, ctypes.POINTER(MtGenParams), P, P]),
        generated_ops=f("generated_ops", ctypes.c_int, [P, ctypes.POINTER(ctypes.c_uint64)]),
        generated_download=f("generated_download", ctypes.c_int, [P] + [P] * 12),
        generated_to_resident=f("generated_to_resident", ctypes.c_int, [P]),
        generated_copy_dev=f("generated_copy_dev", ctypes.c_int, [P, U32, U32, P, P]),
        upload_batch_dev=f("upload_batch_dev", ctypes.c_int, [P, U32, P, P, P, P, ctypes.c_uint64]),
        generated_pack_rows=f("generated_pack_rows", ctypes.c_int, [P, U32, U32, P, P, P]),
        upload_rows_dev=f("upload_rows_dev", ctypes.c_int, [P, U32, P, P, P, U32, P, P]),
        load_snapshot=f("load_snapshot", ctypes.c_int, [P, P]),
        delta_capture=f("delta_capture", ctypes.c_int, [P, ctypes.c_uint64]),
        delta_records=f("delta_records", ctypes.c_int, [P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_uint64)]),
        delta_text=f("delta_text", ctypes.c_int, [P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_uint64),
                                                  ctypes.POINTER(U32)]),
        doc_pset=f("doc_pset", ctypes.c_int, [P, U32, I32, P, P, ctypes.POINTER(U32)]),
        get_containing_segment=f("get_containing_segment", ctypes.c_int,
                                 [P, U32, P, P, P, P, P, ctypes.POINTER(P), ctypes.POINTER(P)]),
        resolve_remote_position=f("resolve_remote_position", ctypes.c_int, [P, U32, P, P, P, P, P]),
        set_doc_snapshot_chunk=f("set_doc_snapshot_chunk", ctypes.c_int, [P, U32, P, P]),
        reserve_staging=f("reserve_staging", ctypes.c_int, [P, ctypes.c_uint64]),
    )


SEG_INFO_FIELDS = ("found", "offset", "obs_pos", "len", "seq", "client", "removed_seq", "removed_client", "prop_set",
                   "marker_ref_type", "depth", "path_lo", "path_hi", "row", "resolved", "pad")
SEG_INFO_DTYPE = np.dtype([(f, np.uint32 if f.startswith("path") else np.int32) for f in SEG_INFO_FIELDS])
POS_UNDEFINED = -(1 << 31)              # MT_POS_UNDEFINED
MT_CHUNK_INFINITY = (1 << 64) - 1      # mt_set_doc_snapshot_chunk: Infinity (one chunk)
MT_CHUNK_NONE = (1 << 64) - 2          # a size no length is below (0, negative, NaN)
MT_PARTITION_AUTO = 0xFFFFFFFF         # mt_set_partition: chosen per batch (mt_plan_partition)


def plan_partition(fn: dict, run_ops, n_cus: int = 256):
    """mt_plan_partition through a bound function table (no context, no GPU call)."""
    r = _u32(run_ops)
    m, k, est = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_double()
    rc = fn["plan_partition"](r.ctypes.data if len(r) else None, len(r), int(n_cus), ctypes.byref(m), ctypes.byref(k),
                              ctypes.byref(est))
    if rc:
        raise MergeTreeError(f"mt_plan_partition failed ({rc})")
    return int(m.value), int(k.value), float(est.value)

DELTA_DTYPE = np.dtype([("op", np.uint32), ("kind", np.int32), ("pos", np.int32), ("len", np.int32),
                        ("seg", np.int32), ("a", np.int32), ("b", np.int32), ("pad", np.int32)])
DELTA_KINDS = {0: "INSERT", 1: "REMOVE", 2: "ANNOTATE", -1: "APPEND", -2: "SPLIT", -3: "UNLINK"}


def _u32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint32)


def _i32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)


class Engine:
    """One engine context on one GPU (or, for tests, the host emulation lib)."""

    def __init__(self, max_docs: int, rows_per_doc: int = 4096, blocks_per_doc: int = 0, text_per_doc: int = 0,
                 propsets_per_doc: int = 0, heap_per_doc: int = 0, window_per_doc: int = 0, device: int = 0,
                 lib_path: str | None = None, prefix: str = "mt_", per_doc: dict | None = None,
                 markers_per_doc: int = 0, register_rows_per_doc: int = 0):
        """per_doc: optional dict of per-document capacity arrays (keys rows_per_doc,
        blocks_per_doc, text_per_doc, propsets_per_doc, heap_per_doc, window_per_doc,
        markers_per_doc, register_rows_per_doc; missing keys use the scalar arguments) ->
        mt_create_docs."""
        # MTGPU_LIB: an alternate build of the same HIP engine (e.g. another occupancy target)
        path = lib_path or os.environ.get("MTGPU_LIB") or LIB_PATH
        if not os.path.exists(path):
            raise MergeTreeError(f"{path} is missing: run __graft_entry__.build() (no CPU fallback exists)")
        self.lib = ctypes.CDLL(path)
        self.fn = _bind(self.lib, prefix)
        self.max_docs = max_docs
        lim = MtLimits(max_docs, rows_per_doc, blocks_per_doc, text_per_doc, propsets_per_doc, heap_per_doc,
                       window_per_doc, markers_per_doc, register_rows_per_doc)
        h = ctypes.c_void_p()
        if per_doc:
            # one mt_limits record per document, filled column by column (a million documents)
            scal = dict(rows_per_doc=rows_per_doc, blocks_per_doc=blocks_per_doc, text_per_doc=text_per_doc,
                        propsets_per_doc=propsets_per_doc, heap_per_doc=heap_per_doc, window_per_doc=window_per_doc,
                        markers_per_doc=markers_per_doc, register_rows_per_doc=register_rows_per_doc)
            arr = np.zeros(max_docs, np.dtype([(n, np.uint32) for n, _ in MtLimits._fields_]))
            for k, v in scal.items():
                arr[k] = np.asarray(per_doc[k], np.uint32)[:max_docs] if k in per_doc else v
            rc = self.fn["create_docs"](device, max_docs, arr.ctypes.data, ctypes.byref(h))
        else:
            rc = self.fn["create"](device, ctypes.byref(lim), ctypes.byref(h))
        self.h = h
        if rc != 0:
            err = self.fn["last_error"](h).decode() if h.value else "create failed"
            raise MergeTreeError(f"mt_create failed ({rc}): {err}")
        self.props = PropTable()
        self.names = ClientNames()
        self._props_uploaded = -1

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.fn["destroy"](self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise MergeTreeError(f"{what} failed ({rc}): {self.fn['last_error'](self.h).decode()}")

    # ---- configuration ----
    def open_docs(self, first: int, n: int):
        self._check(self.fn["docs_open"](self.h, first, n), "mt_docs_open")

    def upload_props(self, props: PropTable | None = None):
        if props is not None:
            self.props = props
        self._props_c = self.props.to_c()
        self._check(self.fn["set_props"](self.h, ctypes.byref(self._props_c)), "mt_set_props")
        self._props_uploaded = len(self.props.sets)

    def upload_names(self, literals: list[str] | None = None):
        lits = literals if literals is not None else self.names.json_literals()
        arr = (ctypes.c_char_p * max(1, len(lits)))(*[s.encode() for s in lits])
        self._names_c = arr
        self._check(self.fn["set_client_names"](self.h, len(lits), ctypes.cast(arr, ctypes.c_void_p)),
                    "mt_set_client_names")

    def upload_doc_names(self, doc: int, literals: list[str]):
        """mt_set_doc_client_names: this document's long client ids by index (JSON literals)."""
        arr = (ctypes.c_char_p * max(1, len(literals)))(*[s.encode() for s in literals])
        self._check(self.fn["set_doc_client_names"](self.h, doc, len(literals), ctypes.cast(arr, ctypes.c_void_p)),
                    "mt_set_doc_client_names")

    # ---- replay ----
    def apply(self, batch: OpBatch):
        if self._props_uploaded != len(self.props.sets):
            self.upload_props()
        self._batch = batch  # keep host arrays alive until sync
        self._check(self.fn["apply_batch"](self.h, ctypes.byref(batch.to_c())), "mt_apply_batch")

    def upload(self, batch: OpBatch):
        if self._props_uploaded != len(self.props.sets):
            self.upload_props()
        self._batch = batch
        self._check(self.fn["upload_batch"](self.h, ctypes.byref(batch.to_c())), "mt_upload_batch")

    def replay_resident(self):
        self._check(self.fn["replay_resident"](self.h), "mt_replay_resident")

    def last_cursors(self, n_runs: int) -> np.ndarray:
        """mt_last_cursors: op index where each run left LDS in the last replay (bit 31 set: it
        finished in HBM in the same wave)."""
        out = np.zeros(n_runs, np.uint32)
        self._check(self.fn["last_cursors"](self.h, n_runs, out.ctypes.data), "mt_last_cursors")
        return out

    def sync(self):
        self._check(self.fn["sync"](self.h), "mt_sync")

    def last_replay_ms(self) -> float:
        v = ctypes.c_float()
        self.fn["last_replay_ms"](self.h, ctypes.byref(v))
        return float(v.value)

    def generate(self, params: MtGenParams, ops_per_doc=None, clients_per_doc=None):
        """Device stream generation (mt_generate / mt_generate_docs with per-document
        message and client counts)."""
        self._gen = params
        n = params.n_docs
        self._gen_ops = (np.full(n, params.ops_per_doc, np.uint32) if ops_per_doc is None
                         else np.ascontiguousarray(ops_per_doc, np.uint32))
        if ops_per_doc is None and clients_per_doc is None:
            self._check(self.fn["generate"](self.h, ctypes.byref(params)), "mt_generate")
            return
        o = self._gen_ops
        c = None if clients_per_doc is None else np.ascontiguousarray(clients_per_doc, np.uint32)
        self._gen_keep = (o, c)
        self._check(self.fn["generate_docs"](self.h, ctypes.byref(params), o.ctypes.data,
                                             c.ctypes.data if c is not None else None), "mt_generate_docs")

    def generated_download(self) -> OpBatch:
        p = self._gen
        v = ctypes.c_uint64()
        self._check(self.fn["generated_ops"](self.h, ctypes.byref(v)), "mt_generated_ops")
        n = int(v.value)
        a = dict(type=np.zeros(n, np.uint8), flags=np.zeros(n, np.uint8), client=np.zeros(n, np.uint16),
                 seq=np.zeros(n, np.int32), ref_seq=np.zeros(n, np.int32), msn=np.zeros(n, np.int32),
                 pos1=np.zeros(n, np.int32), pos2=np.zeros(n, np.int32), payload_off=np.zeros(n, np.uint32),
                 payload_len=np.zeros(n, np.uint32), prop_id=np.zeros(n, np.int32))
        pay = np.zeros(max(1, n * p.ins_len_max), np.uint16)
        self._check(self.fn["generated_download"](self.h, *(a[k].ctypes.data for k in (
            "type", "flags", "client", "seq", "ref_seq", "msn", "pos1", "pos2", "payload_off", "payload_len",
            "prop_id")), pay.ctypes.data), "mt_generated_download")
        offs = np.zeros(p.n_docs + 1, np.uint32)
        offs[1:] = np.cumsum(self._gen_ops, dtype=np.uint64).astype(np.uint32)
        return OpBatch.from_arrays(np.arange(p.n_docs, dtype=np.uint32), offs, pay, **a)

    def generated_copy_dev(self, first_run: int, n_runs: int, rec_ptr: int, payload_ptr: int):
        """mt_generated_copy_dev: op records / payload of generated runs into caller
        buffers (device pointers, e.g. torch tensors' data_ptr())."""
        self._check(self.fn["generated_copy_dev"](self.h, first_run, n_runs, rec_ptr, payload_ptr),
                    "mt_generated_copy_dev")

    def upload_batch_dev(self, doc_ids, op_offsets, rec_ptr: int, payload_ptr: int, payload_units: int):
        """mt_upload_batch_dev: a batch already in device memory becomes resident."""
        d, o = _u32(doc_ids), _u32(op_offsets)
        self._check(self.fn["upload_batch_dev"](self.h, len(d), d.ctypes.data, o.ctypes.data, rec_ptr, payload_ptr,
                                                int(payload_units)), "mt_upload_batch_dev")

    def generated_pack_rows(self, first_run: int, n_runs: int, dst_row, rows_ptr: int) -> np.ndarray:
        """mt_generated_pack_rows: generated runs as exchange rows (mt_op_rec + payload slot)
        at rows dst_row[i] of a device buffer; returns each run's 64-bit row checksum."""
        d = np.ascontiguousarray(dst_row, np.uint64)
        cs = np.zeros(n_runs, np.uint64)
        self._check(self.fn["generated_pack_rows"](self.h, first_run, n_runs, d.ctypes.data, rows_ptr, cs.ctypes.data),
                    "mt_generated_pack_rows")
        return cs

    def upload_rows_dev(self, doc_ids, op_offsets, rows_ptr: int, payload_stride: int, expect) -> np.ndarray:
        """mt_upload_rows_dev: received exchange rows become the resident batch; every run's
        checksum must equal the sender's (MergeTreeError otherwise).  Returns the per-run
        mismatch flags (all zero on success)."""
        d, o = _u32(doc_ids), _u32(op_offsets)
        e = np.ascontiguousarray(expect, np.uint64)
        bad = np.zeros(len(d), np.uint32)
        rc = self.fn["upload_rows_dev"](self.h, len(d), d.ctypes.data, o.ctypes.data, rows_ptr, payload_stride,
                                         e.ctypes.data, bad.ctypes.data)
        if rc == 5:                          # MT_E_EXCHANGE: the flags say which documents
            raise ExchangeError(self.fn["last_error"](self.h).decode(), bad)
        self._check(rc, "mt_upload_rows_dev")
        return bad

    def generated_to_resident(self):
        self._check(self.fn["generated_to_resident"](self.h), "mt_generated_to_resident")

    # ---- queries ----
    def status(self, docs) -> np.ndarray:
        d = _u32(docs)
        out = np.zeros(len(d), np.uint32)
        self._check(self.fn["doc_status"](self.h, len(d), d.ctypes.data, out.ctypes.data), "mt_doc_status")
        return out

    def counters(self, docs) -> dict:
        d = _u32(docs)
        out = (MtDocCounters * len(d))()
        self._check(self.fn["doc_counters_get"](self.h, len(d), d.ctypes.data, ctypes.addressof(out)),
                    "mt_doc_counters_get")
        return {f: np.array([getattr(x, f) for x in out], np.uint64) for f, _ in MtDocCounters._fields_}

    def set_residency(self, use_lds=True, rows: int = 0, blocks: int = 0, heap: int = 0):
        """mt_set_residency: 0/False HBM pools, 1/True LDS-resident, 2 blocks+heap in LDS;
        optional (lowered) LDS pool caps."""
        self._check(self.fn["set_residency"](self.h, int(use_lds), rows, blocks, heap), "mt_set_residency")

    def set_size_class(self, big_min_ops: int):
        """mt_set_size_class: under block residency, runs of at least big_min_ops op records
        replay in the long-document kernel on a second stream (0: off)."""
        self._check(self.fn["set_size_class"](self.h, int(big_min_ops)), "mt_set_size_class")

    def set_continuation(self, min_ops: int):
        """mt_set_continuation: a block-residency batch holding a run of at least min_ops op records
        continues outgrown documents in HBM in the same wave; other batches hand them to a
        second launch."""
        self._check(self.fn["set_continuation"](self.h, int(min_ops)), "mt_set_continuation")

    def set_partition(self, min_ops, cus: int = 0):
        """mt_set_partition: under block residency, runs of at least min_ops op records replay in
        the wide kernel on `cus` reserved CUs beside the rest (0: off; "auto": MT_PARTITION_AUTO,
        chosen per resident batch by mt_plan_partition)."""
        m = MT_PARTITION_AUTO if min_ops == "auto" else int(min_ops)
        self._check(self.fn["set_partition"](self.h, m, int(cus)), "mt_set_partition")

    def partition_info(self) -> dict:
        """mt_last_partition: the partition the last replay launch used."""
        m, k = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self.fn["last_partition"](self.h, ctypes.byref(m), ctypes.byref(k)), "mt_last_partition")
        return {"min_msgs": int(m.value), "cus": int(k.value)} if k.value else None

    def plan_partition(self, run_ops, n_cus: int = 256):
        """mt_plan_partition: (min_ops, cus, estimated ms) the partition rule picks for these run
        lengths ((0, 0, est) for no partition)."""
        return plan_partition(self.fn, run_ops, n_cus)

    def checkpoint(self):
        """mt_checkpoint: device copy of every document's state."""
        self._check(self.fn["checkpoint"](self.h), "mt_checkpoint")

    def restore(self):
        """mt_restore: documents back to the last checkpoint."""
        self._check(self.fn["restore"](self.h), "mt_restore")

    def pool_bytes(self) -> int:
        v = ctypes.c_uint64()
        self._check(self.fn["pool_bytes"](self.h, ctypes.byref(v)), "mt_pool_bytes")
        return int(v.value)

    def pools(self, docs) -> np.ndarray:
        """Per-document pool occupancy (mt_doc_pools): columns rowTop, blkTop, heapN,
        winN, textTop, psetTop, height, rfN, heapHW, winHW."""
        d = _u32(docs)
        out = np.zeros((len(d), 10), np.int32)
        self._check(self.fn["doc_pools"](self.h, len(d), d.ctypes.data, out.ctypes.data), "mt_doc_pools")
        return out

    def load_snapshot(self, batch):
        """mt_load_snapshot of a snapshot_load.LoadBatch (upload_props first if it interned props)."""
        self.upload_props()
        self._check(self.fn["load_snapshot"](self.h, ctypes.byref(batch.to_c())), "mt_load_snapshot")

    # ---- delta callbacks as records (include/mtgpu.h mt_delta_rec) ----
    def delta_capture(self, capacity: int):
        """Record the delta / maintenance callbacks of the following batches (0: off)."""
        self._check(self.fn["delta_capture"](self.h, int(capacity)), "mt_delta_capture")

    def delta_records(self) -> np.ndarray:
        """The last batch's records (DELTA_DTYPE), sorted by op index, callback order within an op."""
        ptr, n = ctypes.c_void_p(), ctypes.c_uint64()
        self._check(self.fn["delta_records"](self.h, ctypes.byref(ptr), ctypes.byref(n)), "mt_delta_records")
        if not n.value:
            return np.zeros(0, DELTA_DTYPE)
        return np.frombuffer(ctypes.string_at(ptr, n.value * DELTA_DTYPE.itemsize), DELTA_DTYPE).copy()

    def delta_text(self) -> tuple[np.ndarray, int]:
        """(UTF-16 units of the last batch's pasted text segments, device launches the batch took)."""
        ptr, n, launches = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_uint32()
        self._check(self.fn["delta_text"](self.h, ctypes.byref(ptr), ctypes.byref(n), ctypes.byref(launches)),
                    "mt_delta_text")
        units = np.frombuffer(ctypes.string_at(ptr, 2 * n.value), np.uint16).copy() if n.value else np.zeros(0, np.uint16)
        return units, int(launches.value)

    def doc_pset(self, doc: int, pset_id: int):
        """(key ids, value ids) of a document's device property set, insertion order."""
        k, v, n = np.zeros(256, np.uint16), np.zeros(256, np.int32), ctypes.c_uint32()   # MT_MAX_PROP_KEYS
        self._check(self.fn["doc_pset"](self.h, doc, pset_id, k.ctypes.data, v.ctypes.data, ctypes.byref(n)),
                    "mt_doc_pset")
        return k[:n.value].copy(), v[:n.value].copy()

    def pset_dict(self, doc: int, pset_id: int):
        """A device property set as a Python dict (None for -1: properties undefined); NaN,
        undefined and fresh consensus values decoded as batch.decode_value does."""
        from .batch import decode_value
        if pset_id < 0:
            return None
        keys, vals = self.doc_pset(doc, pset_id)
        return {self.props.keys[int(k)]: decode_value(int(v), self.props.values_json) for k, v in zip(keys, vals)}

    def set_snapshot_chunk(self, docs, chunk_size):
        """mt_set_doc_snapshot_chunk: options.mergeTreeSnapshotChunkSize per document (0: the
        default 10,000)."""
        d = _u32(docs)
        c = np.ascontiguousarray(chunk_size, np.uint64)
        self._check(self.fn["set_doc_snapshot_chunk"](self.h, len(d), d.ctypes.data, c.ctypes.data),
                    "mt_set_doc_snapshot_chunk")

    def reserve_staging(self, nbytes: int = 0):
        """mt_reserve_staging: pin the two host staging buffers snapshots and text reads download
        through (0: the default group budget), once, ahead of the calls that use them."""
        self._check(self.fn["reserve_staging"](self.h, int(nbytes)), "mt_reserve_staging")

    def update_seq(self, docs, msn, seq):
        d, m, s = _u32(docs), _i32(msn), _i32(seq)
        self._check(self.fn["update_seq"](self.h, len(d), d.ctypes.data, m.ctypes.data, s.ctypes.data),
                    "mt_update_seq")

    def get_length(self, docs, ref_seq, client) -> np.ndarray:
        d, r, c = _u32(docs), _i32(ref_seq), _i32(client)
        out = np.zeros(len(d), np.int32)
        self._check(self.fn["get_length"](self.h, len(d), d.ctypes.data, r.ctypes.data, c.ctypes.data,
                                          out.ctypes.data), "mt_get_length")
        return out

    def containing_segment(self, docs, pos, ref_seq=None, client=None, json: bool = True):
        """mt_get_containing_segment: getContainingSegment (MT/mergeTree.ts:1616-1627) of each
        query under (ref_seq[i], client[i]) (ref_seq < 0 or None: the local view), with
        resolveRemoteClientPosition in the `resolved` field.  Returns (SEG_INFO_DTYPE records,
        list of segment JSON texts or None when json is False / not found)."""
        d, p = _u32(docs), _i32(pos)
        n = len(d)
        r = _i32(np.full(n, -1) if ref_seq is None else ref_seq)
        c = _i32(np.full(n, -1) if client is None else client)
        out = np.zeros(n, SEG_INFO_DTYPE)
        arena, off = ctypes.c_void_p(), ctypes.c_void_p()
        self._check(self.fn["get_containing_segment"](self.h, n, d.ctypes.data, p.ctypes.data, r.ctypes.data,
                                                      c.ctypes.data, out.ctypes.data,
                                                      ctypes.byref(arena) if json else None,
                                                      ctypes.byref(off) if json else None),
                    "mt_get_containing_segment")
        texts = [None] * n
        if json:
            offs = np.ctypeslib.as_array(ctypes.cast(off, ctypes.POINTER(ctypes.c_uint64)), (n + 1,)).copy()
            raw = ctypes.string_at(arena, int(offs[-1])) if offs[-1] else b""
            texts = [raw[offs[i]:offs[i + 1]].decode("utf-8", "surrogatepass") if out["found"][i] else None
                     for i in range(n)]
        return out, texts

    def resolve_remote_position(self, docs, pos, ref_seq, client) -> np.ndarray:
        """mt_resolve_remote_position (MT/mergeTree.ts:2125-2145): local positions,
        POS_UNDEFINED where the reference returns undefined."""
        d, p, r, c = _u32(docs), _i32(pos), _i32(ref_seq), _i32(client)
        out = np.zeros(len(d), np.int32)
        self._check(self.fn["resolve_remote_position"](self.h, len(d), d.ctypes.data, p.ctypes.data, r.ctypes.data,
                                                       c.ctypes.data, out.ctypes.data), "mt_resolve_remote_position")
        return out

    def snapshot(self, docs, msn, seq, legacy: bool = False):
        """SnapshotV1 (or, with legacy, SnapshotLegacy header/body) blobs per document:
        list of (list[bytes], digest)."""
        d, m, s = _u32(docs), _i32(msn), _i32(seq)
        dig = np.zeros(len(d), np.uint64)
        arena, boff, bfirst = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        fn = "snapshot_legacy" if legacy else "snapshot_v1"
        self._check(self.fn[fn](self.h, len(d), d.ctypes.data, m.ctypes.data, s.ctypes.data,
                                dig.ctypes.data, ctypes.byref(arena), ctypes.byref(boff),
                                ctypes.byref(bfirst)), "mt_" + fn)
        first = np.ctypeslib.as_array(ctypes.cast(bfirst, ctypes.POINTER(ctypes.c_uint32)), (len(d) + 1,)).copy()
        nb = int(first[-1])
        offs = np.ctypeslib.as_array(ctypes.cast(boff, ctypes.POINTER(ctypes.c_uint64)), (nb + 1,)).copy()
        raw = ctypes.string_at(arena, int(offs[-1])) if offs[-1] else b""
        out = []
        for i in range(len(d)):
            blobs = [raw[offs[j]:offs[j + 1]] for j in range(first[i], first[i + 1])]
            out.append((blobs, int(dig[i])))
        return out

    def snapshot_digests(self, docs, msn, seq, threads: int = 8) -> np.ndarray:
        """mt_snapshot_digests: SnapshotV1 digests of many documents (one staged download,
        host serialization on `threads` threads)."""
        d, m, s = _u32(docs), _i32(msn), _i32(seq)
        out = np.zeros(len(d), np.uint64)
        self._check(self.fn["snapshot_digests"](self.h, len(d), d.ctypes.data, m.ctypes.data, s.ctypes.data,
                                                out.ctypes.data, threads), "mt_snapshot_digests")
        return out

    def get_text(self, docs) -> list[str]:
        d = _u32(docs)
        arena, off = ctypes.c_void_p(), ctypes.c_void_p()
        self._check(self.fn["get_text"](self.h, len(d), d.ctypes.data, ctypes.byref(arena), ctypes.byref(off)),
                    "mt_get_text")
        offs = np.ctypeslib.as_array(ctypes.cast(off, ctypes.POINTER(ctypes.c_uint64)), (len(d) + 1,)).copy()
        raw = ctypes.string_at(arena, int(offs[-1]) * 2) if offs[-1] else b""
        return [raw[2 * offs[i]:2 * offs[i + 1]].decode("utf-16-le", "surrogatepass") for i in range(len(d))]

    def dump(self, doc: int) -> np.ndarray:
        rows, n = ctypes.c_void_p(), ctypes.c_uint32()
        self._check(self.fn["dump_segments"](self.h, doc, ctypes.byref(rows), ctypes.byref(n)), "mt_dump_segments")
        a = np.frombuffer(ctypes.string_at(rows, n.value * 48), np.int32).reshape(-1, 12).copy()
        self.fn["free"](rows)
        return a


@dataclass
class _Pending:
    msgs: list


def catchup_ops(blobs: dict, snap) -> list:
    """The catch-up messages blob of a legacy snapshot (snapshotLoader.ts:69-92):
    the one blob that is neither the header nor a listed chunk."""
    import json as _json
    from .snapshot_load import _latest, _parse
    md = _latest(_parse(blobs["header"]), True)["headerMetadata"] or {}
    ids = {c["id"] for c in md.get("orderedChunkMetadata", [])} | {"header"}
    rest = [k for k in blobs if k not in ids]
    if len(rest) > 1:
        raise MergeTreeError("Unexpected blobs in snapshot")
    if not rest:
        return []
    raw = blobs[rest[0]]
    return _json.loads(raw.decode("utf-8") if isinstance(raw, (bytes, bytearray)) else raw)


NON_COLLAB_CLIENT = -2                  # NonCollabClient, MT/constants.ts


def snapshot_chunk_option(options: dict | None) -> int:
    """options.mergeTreeSnapshotChunkSize as mt_set_doc_snapshot_chunk takes it: 0 for the default
    (`?? 10000`, snapshotV1.ts:55, snapshotlegacy.ts:71), else the value the reference's
    `length < chunkSize` compares against, i.e. JS ToNumber of it (jsjson.js_to_number): rounded
    up (lengths are integers), MT_CHUNK_INFINITY for Infinity, MT_CHUNK_NONE when no length is
    below it (0, negative, NaN: the legacy header chunk is empty; SnapshotV1 of a non-empty
    document fails at snapshot time, where the reference's chunk loop never ends)."""
    import math
    from .jsjson import _Undefined, js_to_number
    v = (options or {}).get("mergeTreeSnapshotChunkSize")
    if v is None or isinstance(v, _Undefined):
        return 0
    x = js_to_number(v)
    if not (x > 0):
        return MT_CHUNK_NONE
    if math.isinf(x):
        return MT_CHUNK_INFINITY
    return min(int(math.ceil(x)), MT_CHUNK_NONE - 1)


class Segment:
    """A segment as Client.getContainingSegment hands it out: the ISegment fields
    (MT/mergeTree.ts:87-122) of a TextSegment or Marker, by value.  The reference hands out
    the live object; this drop-in returns a copy taken at query time, valid for getPosition
    until the document next changes (the engine's rows are reused, so no handle stays live)."""

    def __init__(self, info, js: str, client, version: int):
        self.cachedLength = int(info["len"])
        self.seq = int(info["seq"])
        self.clientId = client._short_of(int(info["client"]))
        rs = int(info["removed_seq"])
        self.removedSeq = None if rs == POS_UNDEFINED else rs
        self.removedClientId = client._short_of(int(info["removed_client"])) if self.removedSeq is not None else None
        j = json.loads(js)
        self._json = j
        # properties from the device map (NaN / undefined / consensus values as the reference
        # holds them; the JSON text has them as JSON.stringify writes them)
        props = client.engine.pset_dict(client.doc_id, int(info["prop_set"])) if int(info["prop_set"]) >= 0 else None
        if isinstance(j, str):
            self.text, self.properties = j, None
        elif "marker" in j:
            self.text, self.refType, self.properties = None, j["marker"]["refType"], props
        else:
            self.text, self.properties = j["text"], props
        self._obs_pos = int(info["obs_pos"])
        self._doc, self._version = client.doc_id, version

    def toJSONObject(self):
        return self._json


class MergeTreeClient:
    """Drop-in subset of merge-tree ``Client`` (MT/client.ts:44) for a passive observer.

    ``applyMsg`` queues; reads (``getLength``, ``getText``, ``snapshot``) flush the
    queue of every client of the engine in one device batch.
    """

    def __init__(self, engine: Engine, doc_id: int, group: "ClientGroup", options: dict | None = None):
        self.engine, self.doc_id, self.group = engine, doc_id, group
        self.options = options           # Client options (client.ts:82-84)
        self.pending: list = []
        self.names = ClientNames()       # per-document short client ids (client.ts:658-682)
        self.names_uploaded = 0
        self.current_seq = 0
        self.min_seq = 0
        self.longClientId = None
        self.delta_listener = None       # SequenceDoc's sequenceDelta subscription (sequence.py)

    def startOrUpdateCollaboration(self, longClientId, minSeq=0, currentSeq=0, branchId=0):
        self.longClientId = longClientId

    def applyMsg(self, msg: dict):
        self.pending.append(msg)

    def updateSeqNumbers(self, min_seq: int, seq: int):
        """Client.updateSeqNumbers (client.ts:843-850): the device window moves, and so
        do the host copies that snapshot() passes back to mt_update_seq."""
        self.group.flush()
        self.group.version += 1
        self.engine.update_seq([self.doc_id], [min_seq], [seq])
        self.engine.sync()
        self._raise_status()
        self.min_seq, self.current_seq = int(min_seq), int(seq)

    def _raise_status(self):
        st = int(self.engine.status([self.doc_id])[0])
        if st & 0x4000:            # MT_DS_THROWS: the reference's applyMsg throws a TypeError here
            raise ReferenceTypeError(f"document {self.doc_id}: Cannot read property 'seq' of null "
                                     "(a consensus combine on a null defaultValue, properties.ts:51-52)")
        if st:
            raise MergeTreeError(f"document {self.doc_id}: {', '.join(status_names(st))}")

    def getLength(self) -> int:
        self.group.flush()
        self._raise_status()
        return int(self.engine.get_length([self.doc_id], [0x7FFFFFFF], [-1])[0])

    def getText(self) -> str:
        self.group.flush()
        self._raise_status()
        return self.engine.get_text([self.doc_id])[0]

    def snapshot(self, catchUpMsgs: list | None = None, min_seq: int | None = None, seq: int | None = None) -> dict:
        """Client.snapshot (client.ts:923-956) as an ITree.  options
        newMergeTreeSnapshotFormat True: SnapshotV1 (snapshotV1.ts:98-163), header,
        body_0, ...; otherwise SnapshotLegacy (snapshotlegacy.ts:104-175), header,
        body, then catchUpMsgs as JSON under catchUpBlobName (default "catchupOps")."""
        self.group.flush()
        self._raise_status()
        opts = self.options or {}
        v1 = opts.get("newMergeTreeSnapshotFormat") is True
        if v1 and catchUpMsgs:
            raise MergeTreeError("New format should not emit catchup ops")      # client.ts:945-947
        m = self.min_seq if min_seq is None else min_seq
        s = self.current_seq if seq is None else seq
        blobs, _ = self.engine.snapshot([self.doc_id], [m], [s], legacy=not v1)[0]

        def entry(path, contents):
            return {"mode": "100644", "path": path, "type": "Blob", "value": {"contents": contents, "encoding": "utf-8"}}
        entries = [entry("header" if i == 0 else (f"body_{i - 1}" if v1 else "body"), b.decode("utf-8"))
                   for i, b in enumerate(blobs)]
        if not v1 and catchUpMsgs:
            name = opts.get("catchUpBlobName")
            # serializer.stringify: JSON.stringify key order and number forms
            entries.append(entry("catchupOps" if name is None else name, jsjson.stringify(catchUpMsgs)))
        return {"entries": entries}

    def getCurrentSeq(self) -> int:
        return self.current_seq

    # ---- short client ids (client.ts:658-670): the local client is 0, remote clients follow
    #      in first-seen order (the order of the reference when collaboration starts first)
    def getOrAddShortClientId(self, longClientId: str) -> int:
        if self.longClientId is not None and longClientId == self.longClientId:
            return 0
        return self.names.index(longClientId) + 1

    def getShortClientId(self, longClientId: str) -> int:
        if self.longClientId is not None and longClientId == self.longClientId:
            return 0
        if longClientId not in self.names.ids:
            raise MergeTreeError(f"unknown client {longClientId!r}")
        return self.names.ids[longClientId] + 1

    def getLongClientId(self, shortClientId: int) -> str:
        if shortClientId == 0:
            return self.longClientId
        return self.names.names[shortClientId - 1]

    def _short_of(self, index: int) -> int:
        """The engine's per-document client index as this Client's short id."""
        return NON_COLLAB_CLIENT if index < 0 else index + 1

    def _query(self, pos: int, ref_seq: int, short_id: int | None):
        self.group.flush()
        self._raise_status()
        if short_id is None or short_id == 0:
            ref, cli = -1, -1                         # the local view
        else:
            ref, cli = int(ref_seq), int(short_id) - 1
        info, js = self.engine.containing_segment([self.doc_id], [pos], [ref], [cli])
        return info[0], js[0]

    def getContainingSegment(self, pos: int) -> dict:
        """Client.getContainingSegment (client.ts:1040-1043 -> MergeTree.getContainingSegment,
        mergeTree.ts:1616-1627) under the local view: {"segment": Segment | None, "offset"}."""
        info, js = self._query(pos, 0, None)
        if not info["found"]:
            return {"segment": None, "offset": None}
        return {"segment": Segment(info, js, self, self.group.version), "offset": int(info["offset"])}

    def getPosition(self, segment: Segment) -> int:
        """Client.getPosition (client.ts:306-311): the segment's local position."""
        if segment is None:
            return -1
        if segment._doc != self.doc_id or segment._version != self.group.version or self.pending:
            raise MergeTreeError("segment copy is stale: the document changed since getContainingSegment")
        return segment._obs_pos

    def resolveRemoteClientPosition(self, remoteClientPosition: int, remoteClientRefSeq: int,
                                    remoteClientId: int):
        """MergeTree.resolveRemoteClientPosition (mergeTree.ts:2125-2145): the local position of a
        remote client's position at its refSeq; None where the reference returns undefined."""
        info, _ = self._query(remoteClientPosition, remoteClientRefSeq, remoteClientId)
        v = int(info["resolved"])
        return None if v == POS_UNDEFINED else v

    def getPropertiesAtPosition(self, pos: int):
        """Client.getPropertiesAtPosition (client.ts:1045-1057)."""
        seg = self.getContainingSegment(pos)["segment"]
        return seg.properties if seg is not None else None

    def getRangeExtentsOfPosition(self, pos: int) -> dict:
        """Client.getRangeExtentsOfPosition (client.ts:1058-1071)."""
        seg = self.getContainingSegment(pos)["segment"]
        if seg is None:
            return {"posStart": None, "posAfterEnd": None}
        return {"posStart": seg._obs_pos, "posAfterEnd": seg._obs_pos + seg.cachedLength}

    def load(self, blobs: dict, longClientId: str = "snapshot") -> dict:
        """Client.load (MT/client.ts:958) through SnapshotLoader (snapshotLoader.ts:39-222):
        `blobs` maps blob paths (header, body_0.. or body) to contents.  Returns
        {"catchupOps": [...]} (legacy catch-up blob) for the caller to apply."""
        from .snapshot_load import LoadBatchBuilder, parse_snapshot
        self.group.flush()
        chunks = {k: v for k, v in blobs.items()}
        snap = parse_snapshot(chunks)
        lb = LoadBatchBuilder(self.engine.props)
        lb.add(self.doc_id, snap, self.names)
        self.group.version += 1
        self.engine.upload_doc_names(self.doc_id, self.names.json_literals())
        self.names_uploaded = len(self.names.names)
        self.engine.load_snapshot(lb.build())
        self.engine.sync()
        self._raise_status()
        self.longClientId = longClientId
        self.min_seq, self.current_seq = snap.min_seq, snap.seq
        return {"catchupOps": catchup_ops(blobs, snap)}


class ClientGroup:
    """Many MergeTreeClients sharing one engine; flush() packs all queues into one batch."""

    def __init__(self, engine: Engine):
        self.engine = engine
        self.clients: list[MergeTreeClient] = []
        self.version = 0                 # bumped whenever any document changes (Segment copies)

    def new_client(self, options: dict | None = None) -> MergeTreeClient:
        d = len(self.clients)
        if d >= self.engine.max_docs:
            raise MergeTreeError("engine document capacity exhausted")
        cs = snapshot_chunk_option(options)
        self.engine.open_docs(d, 1)
        if cs:
            self.engine.set_snapshot_chunk([d], [cs])
        c = MergeTreeClient(self.engine, d, self, options)
        self.clients.append(c)
        return c

    def flush(self):
        busy = [c for c in self.clients if c.pending]
        if not busy:
            return
        bb = BatchBuilder(self.engine.props, None)
        listen = []
        for c in busy:
            bb.names = c.names
            bb.begin_doc(c.doc_id)
            entries = []
            for m in c.pending:
                entries.append((m, bb.add_message(m)))
                c.current_seq = int(m["sequenceNumber"])
                c.min_seq = max(c.min_seq, int(m["minimumSequenceNumber"]))
            c.pending = []
            if c.delta_listener is not None:
                listen.append((c, entries))
            if c.names_uploaded != len(c.names.names):
                self.engine.upload_doc_names(c.doc_id, c.names.json_literals())
                c.names_uploaded = len(c.names.names)
        batch = bb.build()
        self.version += 1
        self.last_batch = batch          # op indexing of delta records (Engine.delta_records)
        # Capture is armed only around batches with a listener (the other batches run the
        # kernels without capture code).  The capacity is a launch's buffer, not a bound:
        # a batch that emits more resumes in further launches (mt_delta_capture).
        if listen:
            self.engine.delta_capture(max(1 << 16, 512 * len(listen) + 16 * batch.n_ops))
        try:
            self.engine.apply(batch)
            self.engine.sync()
            if listen:
                self._deliver(listen)
        finally:
            if listen:
                self.engine.delta_capture(0)

    def _deliver(self, listen):
        """Hand each listening client its messages' sequenceDelta events: per op member,
        the INSERT/REMOVE/ANNOTATE records as ranges with their property maps."""
        recs = self.engine.delta_records()
        units, _ = self.engine.delta_text()
        by_op: dict = {}
        for r in recs:
            if 0 <= int(r["kind"]) <= 2:
                by_op.setdefault(int(r["op"]), []).append(r)
        for c, entries in listen:
            st = int(self.engine.status([c.doc_id])[0])
            if st:
                raise MergeTreeError(f"document {c.doc_id}: {', '.join(status_names(st))}")
            cache: dict = {}

            def pset(i, doc=c.doc_id, cache=cache):
                if i not in cache:
                    cache[i] = self.engine.pset_dict(doc, i)
                return cache[i]

            def events_of(op, pset=pset):
                out = []
                for r in by_op.get(op, ()):
                    k = int(r["kind"])
                    a, b, pad, ln = int(r["a"]), int(r["b"]), int(r["pad"]), int(r["len"])
                    spec = None                      # an insert of the op's own seg
                    if k == 0 and b == 0:            # a pasted text clone: its text from the device
                        spec = {"text": units[pad:pad + ln].tobytes().decode("utf-16-le", "surrogatepass")}
                    elif k == 0 and b == 1:          # a pasted marker
                        spec = {"marker": {"refType": pad}}
                    out.append({"kind": k, "pos": int(r["pos"]), "len": ln,
                                "before": pset(a) if k == 2 else None,
                                "after": pset(b) if k == 2 else (pset(a) if k == 0 else None), "spec": spec})
                return out
            c.delta_listener(entries, events_of)
