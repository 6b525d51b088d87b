"""Whole-population SnapshotV1 digest manifests of the bench workloads, made by the ORACLE on
this container's CPUs (test infrastructure: the engine is never run here).

Every document of the default seed's streams is generated and replayed by the oracle
(oracle/mtoracle.cpp ora_generate_digests: the device generator's rules, the oracle as
sequencer + observer; tests/test_gpu_parity.py pins the two generators equal) and its
SnapshotV1 digest at the final window written to tests/golden/digests/:

  config2.u64 / config3.u64 / config4.u64 / config5.u64   one little-endian uint64 per document
  config5_1m.roll.u64   the 1,048,576-document north_star run: xxh64 (seed 0) of each group of
                        1,024 consecutive documents' digests (little-endian bytes), 1,024 roll-ups
  index.json            the parameters each file was made with, its document count, XOR and sha256

bench.py compares every document's digest against these when its seed and shape match and
reports "N of N".  usage: python tools/make_digest_manifest.py [config2 config3 ...] [--threads T]
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
OUT = os.path.join(ROOT, "tests", "golden", "digests")
SEED = 20241015                    # bench.py --seed default (rank 0's streams)
ROLL = 1024


def oracle():
    from oracle_lib import lib
    L = lib()
    from fluidframework_amd.batch import MtGenParams, MtPropTable
    L.ora_generate_digests.restype = ctypes.c_int
    L.ora_generate_digests.argtypes = [ctypes.POINTER(MtGenParams), ctypes.POINTER(MtGenParams),
                                       ctypes.POINTER(MtPropTable), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    return L


def digests(p, n, threads, pre=None, ops=None, clients=None, chunk=65536, label=""):
    import bench
    from fluidframework_amd.batch import MtGenParams
    L = oracle()
    props = bench.ann_props()
    out = np.zeros(n, np.uint64)
    st = np.zeros(n, np.uint32)
    t0 = time.time()
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        o = np.ascontiguousarray(ops[a:b], np.uint32) if ops is not None else None
        c = np.ascontiguousarray(clients[a:b], np.uint32) if clients is not None else None
        d = np.zeros(b - a, np.uint64)
        s = np.zeros(b - a, np.uint32)
        L.ora_generate_digests(ctypes.byref(p), ctypes.byref(pre) if pre is not None else None,
                               ctypes.byref(props.to_c()), a, b - a, o.ctypes.data if o is not None else None,
                               c.ctypes.data if c is not None else None, threads, d.ctypes.data, s.ctypes.data)
        out[a:b], st[a:b] = d, s
        print(f"{label}: {b}/{n} documents, {time.time() - t0:.0f} s", flush=True)
    if st.any():
        raise SystemExit(f"{label}: oracle status {np.unique(st)} on {int((st != 0).sum())} documents")
    return out


def params(c, seed, n):
    from fluidframework_amd.batch import MtGenParams
    return MtGenParams(seed, n, c["ops"], c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"],
                       c["ann_sets"], c["rewrite"])


def make(name, threads):
    import bench
    from fluidframework_amd.batch import MtGenParams
    from fluidframework_amd.shard import clients_per_doc, zipf_op_counts
    if name in ("config2", "config3"):
        c = bench.CONFIGS[name]
        return digests(params(c, SEED, c["docs"]), c["docs"], threads, label=name), dict(seed=SEED, docs=c["docs"],
                                                                                         msgs_per_doc=c["ops"])
    if name == "config4":
        c = bench.CONFIGS["config4"]
        n, pre_n = c["docs"], c["prebuild"]
        pa = MtGenParams(SEED, n, pre_n, 1, 0, 100, 0, 5, 1, 1, 0)          # bench.run_config4's pre-build
        pa.ins_len_min, pa.seg_prop_sets, pa.ins_at_end = 5, 2, 1
        pb = params(c, SEED ^ 0xB, n)
        pb.continue_docs = 1
        return digests(pb, n, threads, pre=pa, chunk=threads * 4, label=name), dict(
            seed=SEED, docs=n, msgs_per_doc=c["ops"], prebuild=pre_n)
    if name in ("config5", "config5_1m"):
        c = bench.CONFIGS["config5"]
        n = c["docs"] if name == "config5" else 1048576
        ops, cl = zipf_op_counts(n, SEED), clients_per_doc(n, SEED)
        p = MtGenParams(SEED, n, 0, 2, c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"],
                        c["rewrite"])
        return digests(p, n, threads, ops=ops, clients=cl, label=name), dict(seed=SEED, docs=n,
                                                                              msgs_total=int(ops.sum()))
    raise SystemExit(f"unknown manifest {name}")


def rollups(d):
    import xxhash
    return np.array([xxhash.xxh64(d[i:i + ROLL].astype("<u8").tobytes(), seed=0).intdigest()
                     for i in range(0, len(d), ROLL)], np.uint64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="*", default=["config2", "config3", "config4", "config5"])
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    a = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    idx_path = os.path.join(OUT, "index.json")
    index = json.load(open(idx_path)) if os.path.exists(idx_path) else {}
    for name in a.names:
        t0 = time.time()
        d, meta = make(name, a.threads)
        roll = name.endswith("_1m")
        data = rollups(d) if roll else d
        fn = f"{name}.roll.u64" if roll else f"{name}.u64"
        data.astype("<u8").tofile(os.path.join(OUT, fn))
        index[name] = dict(meta, file=fn, kind=("xxh64 roll-ups of %d documents" % ROLL) if roll else "digest per document",
                           entries=int(len(data)), xor=f"{int(np.bitwise_xor.reduce(d)):016x}",
                           sha256=hashlib.sha256(data.astype("<u8").tobytes()).hexdigest(),
                           made_by="tools/make_digest_manifest.py (oracle ora_generate_digests)",
                           oracle_seconds=round(time.time() - t0, 1))
        json.dump(index, open(idx_path, "w"), indent=1, sort_keys=True)
        print(f"{name}: {len(d)} documents, xor {index[name]['xor']}, {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
