"""The roofline's numerator, pinned by the oracle.

bench.py prices a launch at B_op = 32 + 4 L_ins + 32 (R_r + R_w) + 64 D + 64 Z per message,
summed from the engine's per-document counters (mt_doc_counters).  Here the oracle counts
the same quantities by their definitions on the reference's own object model
(oracle/mtoracle.cpp Tree::cnt: a row pair per ensureIntervalBoundary split, per inserted
segment and per segment a range op visits; the tree's block levels after each op member;
every segment a zamboni scourNode visits), and the engine's counters must equal them
document for document, so the algorithmic bytes are implementation-independent.
"""
import numpy as np
import pytest

from emu_lib import emu_engine
from fluidframework_amd.engine import ClientGroup, Engine
from msg_gen import stream
from oracle_lib import gen_params, generate, replay
from test_emu_parity import CONFIGS, NAMES, ann_props
from test_message_surface import LIMITS, SURFACES

KEYS = ("ops", "msgs", "ins_units", "rows_rw", "depth", "scoured")
GPU = lambda n, **kw: Engine(n, device=0, **kw)  # noqa: E731


def check_generated(factory, cfg, n_docs=4, seed=11):
    props = ann_props()
    p = gen_params(seed=seed, n_docs=n_docs, **CONFIGS[cfg])
    batch, st, _ = generate(p, props)
    assert st == [0] * n_docs
    eng = factory(n_docs, rows_per_doc=20000, window_per_doc=8192, propsets_per_doc=8192, text_per_doc=1 << 18)
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.open_docs(0, n_docs)
    eng.apply(batch)
    eng.sync()
    assert (eng.status(range(n_docs)) == 0).all()
    got = eng.counters(range(n_docs))
    for d, (od, ost) in enumerate(replay(batch, props, NAMES)):
        assert ost == 0
        want = od.counters()
        assert {k: int(got[k][d]) for k in KEYS} == want, f"doc {d}"
    return got


def check_surface(factory, surface, n_docs=3, n_msgs=900, seed=3):
    streams = [stream(seed * 97 + d, n_msgs, **SURFACES[surface]) for d in range(n_docs)]
    g = ClientGroup(factory(n_docs, **LIMITS))
    cl = [g.new_client({"newMergeTreeSnapshotFormat": True}) for _ in range(n_docs)]
    for c, (msgs, _) in zip(cl, streams):
        for m in msgs:
            c.applyMsg(m)
    g.flush()
    eng = g.engine
    assert (eng.status(range(n_docs)) == 0).all()
    got = eng.counters(range(n_docs))
    for d, (_, obs) in enumerate(streams):
        assert {k: int(got[k][d]) for k in KEYS} == obs.counters(), f"doc {d}"


@pytest.mark.parametrize("cfg", ["cfg1", "cfg2", "cfg3", "grow"])
def test_counters_match_oracle_on_emulation(cfg):
    got = check_generated(emu_engine, cfg)
    assert got["scoured"].sum() > 0 and got["depth"].sum() > got["ops"].sum()


@pytest.mark.parametrize("surface", ["groups", "markers_props", "registers", "churn300"])
def test_counters_match_oracle_on_message_surface_emulation(surface):
    check_surface(emu_engine, surface)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["cfg1", "cfg2", "cfg3", "grow"])
def test_counters_match_oracle_on_gpu(cfg):
    check_generated(GPU, cfg, n_docs=8)


@pytest.mark.gpu
@pytest.mark.parametrize("surface", ["groups", "registers"])
def test_counters_match_oracle_on_message_surface_gpu(surface):
    check_surface(GPU, surface, n_docs=6)


def test_bench_bytes_formula():
    """bench.algorithmic_bytes is the §8(d) formula over the counters."""
    import bench
    c = {k: np.array([v], np.uint64) for k, v in zip(KEYS, (5, 4, 10, 6, 9, 3))}
    assert bench.algorithmic_bytes(c) == 32 * 4 + 4 * 10 + 32 * 6 + 64 * 9 + 64 * 3
