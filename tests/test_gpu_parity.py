"""HIP engine on a real MI355X vs the oracle: bit-exact text, segment/tree dump,
snapshotV1 bytes and digests; device stream generator vs oracle generator.
All calls go through the C ABI (libmtgpu.so)."""
import numpy as np
import pytest

from fluidframework_amd.engine import Engine
from oracle_lib import gen_params, generate
from test_emu_parity import CONFIGS, NAMES, ann_props, compare

pytestmark = pytest.mark.gpu


def gpu_engine(n, **kw):
    return Engine(n, device=0, **kw)


@pytest.mark.parametrize("cfg", list(CONFIGS))
def test_gpu_matches_oracle(cfg):
    props = ann_props()
    p = gen_params(seed=11, n_docs=8, **CONFIGS[cfg])
    batch, st, _ = generate(p, props)
    assert st == [0] * 8
    compare(batch, props, 8, factory=gpu_engine)


@pytest.mark.parametrize("res", [(1, 40, 40, 12), (1, 90, 48, 24), (0, 0, 0, 0), (2, 0, 40, 12), (2, 0, 0, 0),
                                 (3, 0, 0, 0), (3, 16, 0, 12)])
def test_gpu_residency_handover_matches_oracle(res):
    # Small LDS caps: documents leave LDS mid-run and mt_replay_kernel finishes
    # them from HBM at the exact op reached; (0, ...) is the HBM kernel alone.
    props = ann_props()
    p = gen_params(seed=21, n_docs=6, **CONFIGS["cfg2"])
    batch, st, _ = generate(p, props)
    assert st == [0] * 6
    compare(batch, props, 6, factory=gpu_engine, residency=res)


@pytest.mark.parametrize("cont", [0, 1 << 30])
def test_gpu_block_continuation_classes_match_oracle(cont):
    # Block residency with tiny caps: every run in the kernel with the in-wave continuation
    # (cont 0), then every run in the one without it (outgrown documents finish in the
    # all-HBM launch that follows).
    props = ann_props()
    p = gen_params(seed=23, n_docs=6, **CONFIGS["grow"])
    batch, st, _ = generate(p, props)
    assert st == [0] * 6
    compare(batch, props, 6, factory=gpu_engine, residency=(2, 0, 40, 12), cont=cont)


def test_gpu_deep_tree_matches_oracle():
    props = ann_props()
    cfg = dict(clients=8, lag=32, ins=70, rem=20, ins_len=8, rem_len=8, ops=20000, ann_sets=24, rewrite=5)
    p = gen_params(seed=99, n_docs=2, **cfg)
    batch, st, _ = generate(p, props)
    compare(batch, props, 2, factory=gpu_engine, rows=60064, win=16384, psets=80064, text=161024)


def test_gpu_many_docs_digests():
    # 256 documents in one launch: per-document digests equal the oracle's.
    props = ann_props()
    p = gen_params(seed=5, n_docs=256, **CONFIGS["cfg2"])
    batch, st, kept = generate(p, props, keep=True)
    eng = gpu_engine(256, rows_per_doc=8192, window_per_doc=4096, propsets_per_doc=4096, text_per_doc=1 << 16)
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.open_docs(0, 256)
    eng.apply(batch)
    eng.sync()
    assert (eng.status(range(256)) == 0).all()
    last = batch.op_offsets[1:] - 1
    snaps = eng.snapshot(range(256), batch.arrays["msn"][last], batch.arrays["seq"][last])
    for d in range(256):
        _, odig = kept[d].snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]))
        assert snaps[d][1] == odig, d


@pytest.mark.parametrize("cfg", ["cfg1", "cfg2", "cfg3"])
def test_gpu_generator_matches_oracle_generator(cfg):
    props = ann_props()
    p = gen_params(seed=3, n_docs=16, **CONFIGS[cfg])
    ob, _, _ = generate(p, props)
    eng = gpu_engine(16, rows_per_doc=8192, window_per_doc=4096, propsets_per_doc=8192, text_per_doc=1 << 16)
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.generate(p)
    eng.sync()
    assert (eng.status(range(16)) == 0).all()
    gb = eng.generated_download()
    for k in ("type", "flags", "client", "seq", "ref_seq", "msn", "pos1", "pos2", "payload_len", "prop_id"):
        assert np.array_equal(gb.arrays[k], ob.arrays[k]), k


def test_gpu_get_length_matches_oracle():
    props = ann_props()
    p = gen_params(seed=8, n_docs=4, **CONFIGS["cfg2"])
    batch, _, kept = generate(p, props, keep=True)
    eng = gpu_engine(4, rows_per_doc=8192, window_per_doc=4096, propsets_per_doc=4096, text_per_doc=1 << 16)
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.open_docs(0, 4)
    eng.apply(batch)
    eng.sync()
    seqs = batch.arrays["seq"][batch.op_offsets[1:] - 1]
    for c in range(8):
        for lag in (0, 5, 20):
            refs = np.maximum(seqs - lag, batch.arrays["msn"][batch.op_offsets[1:] - 1])
            got = eng.get_length(range(4), refs, [c] * 4)
            want = [kept[d].get_length(int(refs[d]), c) for d in range(4)]
            assert list(got) == want
    # many perspectives of the same documents in one call (one workgroup per query)
    q = [(d, int(max(seqs[d] - lag, batch.arrays["msn"][batch.op_offsets[d + 1] - 1])), c)
         for d in range(4) for lag in range(0, 33, 4) for c in range(8)]
    got = eng.get_length([x[0] for x in q], [x[1] for x in q], [x[2] for x in q])
    assert list(got) == [kept[d].get_length(r, c) for d, r, c in q]


def test_gpu_per_document_capacities_and_generator_counts():
    # mt_create_docs (per-document pool sizes) + mt_generate_docs (per-document
    # message and client counts): device streams equal the oracle generator's,
    # and replaying them on differently sized documents is bit-exact.
    props = ann_props()
    ops = [8, 300, 1200, 57, 2000, 640]
    cl = [2, 16, 5, 9, 3, 8]
    n = len(ops)
    p = gen_params(seed=19, n_docs=n, **{**CONFIGS["cfg2"], "ops": 100})
    ob, st, kept = generate(p, props, ops_per_doc=ops, clients_per_doc=cl, keep=True)
    assert st == [0] * n
    per_doc = dict(rows_per_doc=[3 * o + 64 for o in ops], window_per_doc=[2048] * n,
                   text_per_doc=[8 * o + 4096 for o in ops], propsets_per_doc=[64] * n, blocks_per_doc=[o + 64 for o in ops],
                   heap_per_doc=[2 * o + 64 for o in ops])
    eng = Engine(n, device=0, per_doc=per_doc)
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.generate(p, ops_per_doc=ops, clients_per_doc=cl)
    eng.sync()
    assert (eng.status(range(n)) == 0).all()
    gb = eng.generated_download()
    assert np.array_equal(gb.op_offsets, ob.op_offsets)
    for k in ("type", "flags", "client", "seq", "ref_seq", "msn", "pos1", "pos2", "payload_len", "prop_id"):
        assert np.array_equal(gb.arrays[k], ob.arrays[k]), k
    eng.generated_to_resident()
    eng.open_docs(0, n)
    eng.replay_resident()
    eng.sync()
    assert (eng.status(range(n)) == 0).all()
    last = ob.op_offsets[1:] - 1
    digs = eng.snapshot_digests(range(n), ob.arrays["msn"][last], ob.arrays["seq"][last], threads=4)
    texts = eng.get_text(range(n))
    for d in range(n):
        assert texts[d] == kept[d].get_text()
        assert int(digs[d]) == kept[d].snapshot(int(ob.arrays["msn"][last[d]]), int(ob.arrays["seq"][last[d]]))[1]


def test_gpu_bench_docs_match_oracle():
    from test_emu_parity import check_bench_docs
    check_bench_docs(gpu_engine)
