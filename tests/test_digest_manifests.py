"""The committed whole-population digest manifests (tests/golden/digests/, made by
tools/make_digest_manifest.py with the oracle) are intact and agree with the oracle on sampled
documents: bench.py's "N of N" parity is only as good as these files."""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
DIG = os.path.join(ROOT, "tests", "golden", "digests")
INDEX = json.load(open(os.path.join(DIG, "index.json")))


@pytest.mark.parametrize("name", sorted(INDEX))
def test_manifest_file_matches_index(name):
    e = INDEX[name]
    raw = open(os.path.join(DIG, e["file"]), "rb").read()
    assert len(raw) == 8 * e["entries"]
    assert hashlib.sha256(raw).hexdigest() == e["sha256"]
    if not e["file"].endswith(".roll.u64"):
        d = np.frombuffer(raw, "<u8")
        assert e["entries"] == e["docs"]
        assert f"{int(np.bitwise_xor.reduce(d)):016x}" == e["xor"]


def _oracle_digests(p, pre, first, n, ops=None, clients=None, threads=4):
    import bench
    import make_digest_manifest as m
    L = m.oracle()
    props = bench.ann_props()
    d = np.zeros(n, np.uint64)
    st = np.zeros(n, np.uint32)
    o = np.ascontiguousarray(ops, np.uint32) if ops is not None else None
    c = np.ascontiguousarray(clients, np.uint32) if clients is not None else None
    L.ora_generate_digests(ctypes.byref(p), ctypes.byref(pre) if pre is not None else None, ctypes.byref(props.to_c()),
                           first, n, o.ctypes.data if o is not None else None, c.ctypes.data if c is not None else None,
                           threads, d.ctypes.data, st.ctypes.data)
    assert not st.any()
    return d


def _manifest(name):
    return np.fromfile(os.path.join(DIG, INDEX[name]["file"]), "<u8")


@pytest.mark.parametrize("name", ["config2", "config3"])
def test_manifest_short_docs_match_oracle(name):
    import bench
    import make_digest_manifest as m
    c = bench.CONFIGS[name]
    p = m.params(c, INDEX[name]["seed"], c["docs"])
    man = _manifest(name)
    for first in (0, c["docs"] - 3):
        assert (_oracle_digests(p, None, first, 3) == man[first:first + 3]).all()


def test_manifest_config5_matches_oracle():
    import bench
    from fluidframework_amd.batch import MtGenParams
    from fluidframework_amd.shard import clients_per_doc, zipf_op_counts
    c = bench.CONFIGS["config5"]
    seed, n = INDEX["config5"]["seed"], INDEX["config5"]["docs"]
    ops, cl = zipf_op_counts(n, seed), clients_per_doc(n, seed)
    p = MtGenParams(seed, n, 0, 2, c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"], c["rewrite"])
    man = _manifest("config5")
    for first in (0, n - 64):
        got = _oracle_digests(p, None, first, 64, ops[first:first + 64], cl[first:first + 64], threads=8)
        assert (got == man[first:first + 64]).all()


def test_manifest_config5_1m_first_rollup_matches_oracle():
    import xxhash
    import bench
    from fluidframework_amd.batch import MtGenParams
    from fluidframework_amd.shard import clients_per_doc, zipf_op_counts
    c = bench.CONFIGS["config5"]
    seed, n = INDEX["config5_1m"]["seed"], INDEX["config5_1m"]["docs"]
    ops, cl = zipf_op_counts(n, seed), clients_per_doc(n, seed)
    p = MtGenParams(seed, n, 0, 2, c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"], c["rewrite"])
    d = _oracle_digests(p, None, 0, 1024, ops[:1024], cl[:1024], threads=8)
    roll = xxhash.xxh64(d.astype("<u8").tobytes(), seed=0).intdigest()
    assert roll == int(_manifest("config5_1m")[0])
