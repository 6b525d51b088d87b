"""Engine logic (host-emulated waves) vs the oracle: bit-exact on generated streams.

The same mt_core.h logic is compiled for gfx950 in the product; tests/test_gpu_parity.py
repeats these checks on the real device.
"""
import numpy as np
import pytest

from fluidframework_amd.batch import OpBatch, PropTable
from oracle_lib import gen_params, generate, replay
from emu_lib import emu_engine

NAMES = ['"c%d"' % i for i in range(64)]


def ann_props():
    pt = PropTable()
    vals = ["s0", "s1", "s2", "s3", 1, 2, None]
    rng = np.random.RandomState(5)
    for i in range(24):
        keys = rng.choice(8, size=rng.randint(1, 4), replace=False)
        pt.intern({f"k{k}": vals[rng.randint(0, len(vals))] for k in sorted(keys)})
    return pt


CONFIGS = {
    "cfg1": dict(clients=2, lag=8, ins=55, rem=45, ins_len=8, rem_len=16, ops=1500),
    "cfg2": dict(clients=8, lag=32, ins=60, rem=40, ins_len=8, rem_len=8, ops=1500),
    "cfg3": dict(clients=8, lag=4, ins=30, rem=30, ins_len=8, rem_len=16, ops=1500, ann_sets=24, rewrite=5),
    "grow": dict(clients=4, lag=16, ins=80, rem=10, ins_len=6, rem_len=4, ops=2500, ann_sets=24, rewrite=10),
}


def compare(batch, props, n_docs, factory=None, **cap):
    eng = (factory or emu_engine)(n_docs, rows_per_doc=cap.get("rows", 20000), window_per_doc=cap.get("win", 8192),
                     propsets_per_doc=cap.get("psets", 8192), text_per_doc=cap.get("text", 1 << 18))
    if "residency" in cap:
        eng.set_residency(*cap["residency"])
    if "cont" in cap:
        eng.set_continuation(cap["cont"])
    if "reserve" in cap:
        eng.reserve_staging(cap["reserve"])
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.open_docs(0, n_docs)
    eng.apply(batch)
    eng.sync()
    st = eng.status(range(n_docs))
    assert (st == 0).all(), st
    oracle_docs = replay(batch, props, NAMES)
    last = batch.op_offsets[1:] - 1
    msn = batch.arrays["msn"][last]
    seq = batch.arrays["seq"][last]
    texts = eng.get_text(range(n_docs))
    for d in range(n_docs):
        od, ost = oracle_docs[d]
        assert ost == 0
        assert texts[d] == od.get_text(), f"doc {d} text"
        ed, odump = eng.dump(d), od.dump()
        assert ed.shape == odump.shape, f"doc {d} rows {ed.shape} vs {odump.shape}"
        bad = np.nonzero((ed != odump).any(axis=1))[0]
        assert len(bad) == 0, f"doc {d} first differing row {bad[:3]}: emu {ed[bad[0]]} oracle {odump[bad[0]]}"
    snaps = eng.snapshot(range(n_docs), msn, seq)
    digs = eng.snapshot_digests(range(n_docs), msn, seq, threads=3)
    for d in range(n_docs):
        od, _ = oracle_docs[d]
        oblobs, odig = od.snapshot(int(msn[d]), int(seq[d]))
        eblobs, edig = snaps[d]
        assert eblobs == oblobs, f"doc {d} snapshot"
        assert edig == odig
        assert int(digs[d]) == odig, f"doc {d} mt_snapshot_digests"
    # SnapshotLegacy at the same window: rows above the MSN are left out, rows
    # removed above it keep their text (snapshotlegacy.ts:177-240).
    legacy = eng.snapshot(range(n_docs), msn, seq, legacy=True)
    for d in range(n_docs):
        od, _ = oracle_docs[d]
        oblobs, odig = od.snapshot(int(msn[d]), int(seq[d]), legacy=True)
        assert legacy[d][0] == oblobs, f"doc {d} legacy snapshot"
        assert legacy[d][1] == odig
    return eng


@pytest.mark.parametrize("cfg", list(CONFIGS))
def test_emu_matches_oracle(cfg):
    props = ann_props()
    p = gen_params(seed=11, n_docs=4, **CONFIGS[cfg])
    batch, st, _ = generate(p, props)
    assert st == [0] * 4
    compare(batch, props, 4)


def test_emu_snapshots_in_staging_groups_match_oracle(monkeypatch):
    """Snapshots staged one document per group (MT_STAGE_BUDGET=1: every group is staged into
    the other pinned buffer while the last one is emitted) equal the oracle's."""
    monkeypatch.setenv("MT_STAGE_BUDGET", "1")
    props = ann_props()
    p = gen_params(seed=12, n_docs=5, **CONFIGS["cfg3"])
    batch, st, _ = generate(p, props)
    assert st == [0] * 5
    compare(batch, props, 5)


@pytest.mark.parametrize("reserve", [0, 1 << 12])
def test_emu_snapshots_after_reserved_staging_match_oracle(reserve, monkeypatch):
    """mt_reserve_staging (the default budget, or buffers smaller than a group: grown on use)
    changes nothing in the snapshots."""
    monkeypatch.setenv("MT_STAGE_BUDGET", str(1 << 16))
    props = ann_props()
    p = gen_params(seed=13, n_docs=4, **CONFIGS["cfg2"])
    batch, st, _ = generate(p, props)
    assert st == [0] * 4
    compare(batch, props, 4, reserve=reserve)


# Block-residency budget under adversarial streams: one-unit inserts build many segments and
# deep trees, 48-unit removals then unlink them in bursts (scours that leave blocks under half
# full, packParent re-dealing whole levels); with lag 0 the zamboni runs every message.  Every
# message must fit the per-message block budget (MtEngT::ldsHeadroom, 2h + 13) or hand the
# document over to HBM first: never MT_DS_OOM_BLOCKS.
ADVERSARIAL = dict(clients=2, lag=0, ins=70, rem=30, ins_len=1, rem_len=48, ops=5000)


@pytest.mark.parametrize("res", [(2, 0, 40, 12), (2, 0, 104, 94), (1, 90, 48, 24)])
def test_emu_block_budget_adversarial_matches_oracle(res):
    props = ann_props()
    p = gen_params(seed=41, n_docs=3, **ADVERSARIAL)
    batch, st, _ = generate(p, props)
    assert st == [0] * 3
    compare(batch, props, 3, residency=res)


# LDS residency hand-over: tiny LDS caps make documents leave LDS mid-run (at
# different ops, with different pools the binding one) and finish from HBM;
# (0, ...) runs the HBM-pool kernel alone.  Results must not change.
@pytest.mark.parametrize("res", [(1, 40, 40, 12), (1, 90, 48, 24), (1, 256, 96, 96), (0, 0, 0, 0),
                                 (2, 0, 40, 12), (2, 0, 104, 94), (3, 0, 0, 0), (3, 16, 0, 12), (3, 0, 7, 0), (3, 0, 4, 0)])
@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "grow"])
def test_emu_residency_handover_matches_oracle(cfg, res):
    props = ann_props()
    p = gen_params(seed=21, n_docs=3, **CONFIGS[cfg])
    batch, st, _ = generate(p, props)
    assert st == [0] * 3
    compare(batch, props, 3, residency=res)


# Block residency with tiny caps: every run in the kernel with the in-wave continuation
# (mt_set_continuation(0)) and every run in the one that hands over to a second launch.
@pytest.mark.parametrize("cont", [0, 1 << 30])
def test_emu_block_continuation_classes_match_oracle(cont):
    props = ann_props()
    p = gen_params(seed=23, n_docs=3, **CONFIGS["grow"])
    batch, st, _ = generate(p, props)
    assert st == [0] * 3
    compare(batch, props, 3, residency=(2, 0, 40, 12), cont=cont)


@pytest.mark.parametrize("cfg", ["cfg1", "cfg3"])
def test_device_generator_matches_oracle_generator(cfg):
    props = ann_props()
    p = gen_params(seed=3, n_docs=3, **CONFIGS[cfg])
    ob, _, _ = generate(p, props)
    eng = emu_engine(3, rows_per_doc=20000, window_per_doc=8192, propsets_per_doc=8192, text_per_doc=1 << 18)
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.generate(p)
    eng.sync()
    assert (eng.status(range(3)) == 0).all()
    gb = eng.generated_download()
    for k in ("type", "flags", "client", "seq", "ref_seq", "msn", "pos1", "pos2", "payload_len", "prop_id"):
        assert np.array_equal(gb.arrays[k], ob.arrays[k]), k
    # payload contents per op
    for i in range(0, gb.n_ops, 97):
        n = int(gb.arrays["payload_len"][i])
        a = gb.payload[gb.arrays["payload_off"][i]:][:n]
        b = ob.payload[ob.arrays["payload_off"][i]:][:n]
        assert np.array_equal(a, b)


def test_emu_matches_oracle_under_text_compaction_pressure():
    # A text arena barely larger than the live text forces compaction inside
    # zamboni merges (prefetched offsets must be refreshed).
    props = ann_props()
    cfg = dict(clients=4, lag=6, ins=70, rem=20, ins_len=8, rem_len=6, ops=4000, ann_sets=24, rewrite=5)
    p = gen_params(seed=17, n_docs=3, **cfg)
    batch, st, kept = generate(p, props, keep=True)
    live = max(k.get_length() for k in kept)
    compare(batch, props, 3, text=live + 600)


def split_batch(batch, k):
    """Cut every document's run into k consecutive batches at message boundaries."""
    out = [dict(doc=[], idx=[]) for _ in range(k)]
    flags = batch.arrays["flags"]
    for r, d in enumerate(batch.doc_ids):
        a, b = int(batch.op_offsets[r]), int(batch.op_offsets[r + 1])
        ends = [i + 1 for i in range(a, b) if flags[i] & 1]
        cuts = [a] + [ends[min(len(ends) - 1, (j + 1) * len(ends) // k - 1)] for j in range(k - 1)] + [b]
        for j in range(k):
            if cuts[j + 1] > cuts[j]:
                out[j]["doc"].append(d)
                out[j]["idx"].append(np.arange(cuts[j], cuts[j + 1]))
    res = []
    for o in out:
        idx = np.concatenate(o["idx"])
        offs = np.concatenate([[0], np.cumsum([len(x) for x in o["idx"]])])
        res.append(OpBatch.from_arrays(o["doc"], offs, batch.payload,
                                       **{n: batch.arrays[n][idx] for n in batch.arrays}))
    return res


def test_emu_matches_oracle_across_batches():
    # Per-document state that lives in LDS during a run (recycled-row stack)
    # must survive the run boundary: replay the same streams in 5 batches.
    props = ann_props()
    p = gen_params(seed=23, n_docs=3, **CONFIGS["cfg2"])
    batch, st, _ = generate(p, props)
    eng = emu_engine(3, rows_per_doc=20000, window_per_doc=8192, propsets_per_doc=8192, text_per_doc=1 << 18)
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.open_docs(0, 3)
    for b in split_batch(batch, 5):
        eng.apply(b)
    eng.sync()
    assert (eng.status(range(3)) == 0).all()
    oracle_docs = replay(batch, props, NAMES)
    texts = eng.get_text(range(3))
    for d in range(3):
        assert texts[d] == oracle_docs[d][0].get_text()
        assert np.array_equal(eng.dump(d), oracle_docs[d][0].dump())


STRESS = {
    "deep": dict(clients=4, lag=16, ins=92, rem=4, ins_len=3, rem_len=2, ops=6000, ann_sets=24, rewrite=10),
    "lag128": dict(clients=16, lag=128, ins=55, rem=35, ins_len=8, rem_len=12, ops=3000, ann_sets=24, rewrite=5),
    "shrink": dict(clients=8, lag=32, ins=35, rem=65, ins_len=8, rem_len=24, ops=3000),
}


@pytest.mark.parametrize("cfg", list(STRESS))
def test_emu_matches_oracle_stress(cfg):
    props = ann_props()
    p = gen_params(seed=29, n_docs=2, **STRESS[cfg])
    batch, st, _ = generate(p, props)
    assert st == [0] * 2
    compare(batch, props, 2)


def test_emu_per_document_capacities_match_oracle():
    # mt_create_docs: documents of one context with different pool sizes (sized
    # from each document's op count, as config 5's Zipf documents are).
    props = ann_props()
    p = gen_params(seed=17, n_docs=4, **CONFIGS["cfg3"])
    batch, st, _ = generate(p, props)
    n = 4
    per_doc = dict(rows_per_doc=[3000 + 500 * d for d in range(n)], window_per_doc=[2048 + 64 * d for d in range(n)],
                   text_per_doc=[40000 + 1000 * d for d in range(n)], propsets_per_doc=[4000 + 7 * d for d in range(n)])
    from fluidframework_amd.engine import Engine
    from emu_lib import build_emu
    eng = Engine(n, lib_path=build_emu(), prefix="emu_", per_doc=per_doc)
    assert eng.pool_bytes() > 0
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.open_docs(0, n)
    eng.apply(batch)
    eng.sync()
    assert (eng.status(range(n)) == 0).all()
    oracle_docs = replay(batch, props, NAMES)
    texts = eng.get_text(range(n))
    last = batch.op_offsets[1:] - 1
    snaps = eng.snapshot(range(n), batch.arrays["msn"][last], batch.arrays["seq"][last])
    for d in range(n):
        assert texts[d] == oracle_docs[d][0].get_text()
        assert np.array_equal(eng.dump(d), oracle_docs[d][0].dump())
        assert snaps[d][0] == oracle_docs[d][0].snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]))[0]


def test_emu_generator_per_document_counts_matches_oracle():
    # mt_generate_docs: skewed per-document message counts and client counts
    # (config 5's Zipf documents) produce the oracle generator's streams.
    props = ann_props()
    ops = [8, 300, 1200, 57, 2000]
    cl = [2, 16, 5, 9, 3]
    p = gen_params(seed=19, n_docs=5, **{**CONFIGS["cfg2"], "ops": 100})
    ob, st, _ = generate(p, props, ops_per_doc=ops, clients_per_doc=cl)
    assert st == [0] * 5
    eng = emu_engine(5, rows_per_doc=8192, window_per_doc=4096, propsets_per_doc=8192, text_per_doc=1 << 16)
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.generate(p, ops_per_doc=ops, clients_per_doc=cl)
    eng.sync()
    assert (eng.status(range(5)) == 0).all()
    gb = eng.generated_download()
    assert np.array_equal(gb.op_offsets, ob.op_offsets)
    for k in ("type", "flags", "client", "seq", "ref_seq", "msn", "pos1", "pos2", "payload_len", "prop_id"):
        assert np.array_equal(gb.arrays[k], ob.arrays[k]), k


# Config-2 documents (bench seed) whose full 10k-message streams once exposed a text
# compaction inside a multi-row zamboni merge run (caught by bench.py's digest parity).
BENCH_DOCS = [240, 320, 459, 490]


def bench_doc_batch(factory, docs):
    import bench
    from fluidframework_amd.batch import MtGenParams
    c = dict(bench.CONFIGS["config2"])
    props = bench.ann_props()
    out = []
    for d in docs:
        c["docs"] = 1
        g = factory(1, **bench.caps_for(c))
        g.upload_props(props)
        g.upload_names(NAMES)
        p = MtGenParams(20241015, 1, c["ops"], c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"],
                        c["ann_sets"], c["rewrite"])
        p.doc_id_base = d
        g.generate(p)
        g.sync()
        out.append(g.generated_download())
        g.close()
    return out, props


def check_bench_docs(factory):
    import bench
    from oracle_lib import OracleDoc
    c = dict(bench.CONFIGS["config2"])
    batches, props = bench_doc_batch(factory, BENCH_DOCS)
    for b in batches:
        c["docs"] = 1
        eng = factory(1, **bench.caps_for(c))
        eng.upload_props(props)
        eng.upload_names(NAMES)
        eng.open_docs(0, 1)
        eng.apply(b)
        eng.sync()
        assert eng.status([0])[0] == 0
        od = OracleDoc(True, props, NAMES)
        assert od.apply_run(b, 0) == 0
        assert eng.get_text([0])[0] == od.get_text()
        last = int(b.op_offsets[-1]) - 1
        msn, seq = int(b.arrays["msn"][last]), int(b.arrays["seq"][last])
        assert eng.snapshot([0], [msn], [seq])[0][1] == od.snapshot(msn, seq)[1]


def test_emu_bench_docs_match_oracle():
    check_bench_docs(emu_engine)


# Text arena pressure: small arenas make zamboni's merge runs compact the arena while they
# are planned (then re-planned with exactly sized regions) and reuse the spaces of split
# halves and unlinked removals (MtEngT::mergeRuns); long runs grow segments past the
# 256-unit granularity.  Results must not change.
@pytest.mark.parametrize("cfg,text,ops", [("cfg2", 4200, 3000), ("cfg3", 600, 3000), ("grow", 8000, 2500),
                                          ("cfg2", 1 << 18, 6000)])
def test_emu_text_arena_pressure_matches_oracle(cfg, text, ops):
    props = ann_props()
    c = dict(CONFIGS[cfg]); c["ops"] = ops
    p = gen_params(seed=31, n_docs=3, **c)
    batch, st, _ = generate(p, props)
    assert st == [0] * 3
    compare(batch, props, 3, text=text, residency=(2, 0, 104, 94))
