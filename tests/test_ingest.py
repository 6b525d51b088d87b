"""Ingest boundary (SURVEY §8(b) mt_apply_batch / mt_upload_batch): batches above 65,536 ops
are validated and packed into 32-byte records on several host threads.  The result must be
the single-threaded one: the same replay (digests equal to the oracle's) and, for a bad
batch, the error of the lowest offending op."""
import os

import numpy as np
import pytest

from emu_lib import emu_engine
from fluidframework_amd.batch import OpBatch
from fluidframework_amd.engine import Engine, MergeTreeError
from oracle_lib import gen_params, generate, replay
from test_emu_parity import CONFIGS, ann_props

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

NAMES = ['"c%d"' % i for i in range(64)]


def check_large_batch(factory, n_docs, ops):
    props = ann_props()
    p = gen_params(seed=5, n_docs=n_docs, **dict(CONFIGS["cfg2"], ops=ops))
    batch, st, _ = generate(p, props)
    assert st == [0] * n_docs and batch.n_ops >= 1 << 16
    eng = factory(n_docs, rows_per_doc=3 * ops + 64, window_per_doc=8192, propsets_per_doc=2 * ops + 64,
                  text_per_doc=16 * ops + 4096)
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.open_docs(0, n_docs)
    eng.apply(batch)
    eng.sync()
    assert (eng.status(range(n_docs)) == 0).all()
    last = batch.op_offsets[1:] - 1
    neg = np.full(n_docs, -1, np.int32)
    dig = eng.snapshot_digests(range(n_docs), neg, neg, threads=2)
    for d, (od, ost) in enumerate(replay(batch, props, NAMES)):
        assert ost == 0
        assert int(dig[d]) == od.snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]))[1], d


def test_large_batch_parallel_pack_on_emulation():
    check_large_batch(emu_engine, 8, 9000)


@pytest.mark.gpu
def test_large_batch_parallel_pack_on_gpu():
    check_large_batch(lambda n, **kw: Engine(n, device=0, **kw), 16, 9000)


def _bad_batch(n_ops, bad):
    """n_ops one-unit inserts in one run; `bad` maps op index -> field overrides."""
    a = dict(type=np.zeros(n_ops), flags=np.ones(n_ops), client=np.zeros(n_ops), seq=np.arange(1, n_ops + 1),
             ref_seq=np.zeros(n_ops), msn=np.zeros(n_ops), pos1=np.zeros(n_ops), pos2=np.zeros(n_ops),
             payload_off=np.zeros(n_ops), payload_len=np.ones(n_ops), prop_id=np.full(n_ops, -1))
    for i, kv in bad.items():
        for k, v in kv.items():
            a[k][i] = v
    return OpBatch.from_arrays([0], [0, n_ops], np.full(4, ord("a")), **a)


@pytest.mark.parametrize("bad,msg", [
    ({70000: dict(payload_off=9), 99000: dict(type=9)}, "payload out of range"),
    ({99000: dict(payload_off=9), 70001: dict(type=9)}, "unknown op type"),
    ({65537: dict(prop_id=3)}, "prop_id out of range"),
])
def test_large_batch_validation_reports_lowest_bad_op(bad, msg):
    eng = emu_engine(1, rows_per_doc=64, window_per_doc=64, propsets_per_doc=64, text_per_doc=64)
    eng.upload_names(NAMES)
    with pytest.raises(MergeTreeError, match=msg):
        eng.upload(_bad_batch(100000, bad))


def test_node_full_scale_ingest_packs_every_message(tmp_path):
    """js/ingest_scale.js (bench.py's full-scale Node ingest leg) on the CPU: every document's
    binary op columns become message JSON inside the workers, and the pool packs every message."""
    import json
    import shutil
    import subprocess
    import bench
    from fluidframework_amd.batch import MtGenParams
    if shutil.which("node") is None:
        pytest.skip("node is not installed")
    c = dict(bench.CONFIGS["config2"]); c["docs"] = 6; c["ops"] = 600
    eng = emu_engine(6, **bench.caps_for(c))
    eng.upload_props(bench.ann_props()); eng.upload_names(['"c%d"' % i for i in range(64)])
    eng.generate(MtGenParams(7, 6, c["ops"], c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"],
                             c["ann_sets"], c["rewrite"]))
    eng.sync()
    bench.write_doc_bins(eng.generated_download(), str(tmp_path))
    r = subprocess.run(["node", os.path.join(ROOT, "fluidframework_amd", "js", "ingest_scale.js"), str(tmp_path), "3", "4"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["docs"] == 6 and out["msgs"] == 6 * 600
    # end to end through the Node addon (built on the host emulation): the windowed pipeline's
    # SnapshotV1 digests equal a replay of the same generated streams
    from emu_lib import build_emu_napi
    addon = build_emu_napi()
    if addon is None:
        return
    env = dict(os.environ, MTGPU_NAPI=addon)
    r = subprocess.run(["node", os.path.join(ROOT, "fluidframework_amd", "js", "ingest_scale.js"), str(tmp_path), "3", "4",
                        "--gpu"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    node = json.loads(r.stdout.strip().splitlines()[-1])
    eng.generated_to_resident()
    eng.open_docs(0, 6)
    eng.replay_resident()
    eng.sync()
    neg = np.full(6, -1, np.int32)
    digs = eng.snapshot_digests(range(6), neg, neg, threads=2)
    assert node["digest_xor"] == f"{int(np.bitwise_xor.reduce(digs)):016x}"
    # --objects: the workers hold parsed message objects, pack them with addMessages and hand the
    # parts to mt_apply_batch_parts unmerged; the same digests
    r = subprocess.run(["node", os.path.join(ROOT, "fluidframework_amd", "js", "ingest_scale.js"), str(tmp_path), "3", "4",
                        "--gpu", "--objects"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    obj = json.loads(r.stdout.strip().splitlines()[-1])
    assert obj["input"] == "objects" and obj["msgs"] == 6 * 600
    assert obj["digest_xor"] == node["digest_xor"]
