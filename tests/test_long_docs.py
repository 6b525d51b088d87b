"""Config 4 machinery on the host emulation vs the oracle: documents pre-built by
append-only inserts with alternating segment properties (no coalescing), a
device checkpoint of that state, then a deep-window stream generated on top of
it (continue_docs) and replayed from the restored checkpoint."""
import numpy as np
import pytest

from emu_lib import emu_engine
from fluidframework_amd.engine import Engine
from fluidframework_amd.batch import concat_runs as concat
from oracle_lib import gen_params, generate, replay
from test_emu_parity import NAMES, ann_props



def prebuild_params(n_docs, ops):
    p = gen_params(seed=404, n_docs=n_docs, ops=ops, clients=4, lag=0, ins=100, rem=0, ins_len=5, rem_len=1)
    p.ins_len_min, p.seg_prop_sets, p.ins_at_end = 5, 2, 1
    return p


def test_prebuild_generator_matches_oracle():
    props = ann_props()
    p = prebuild_params(3, 600)
    ob, st, kept = generate(p, props, keep=True)
    assert st == [0] * 3
    assert (ob.arrays["flags"] & 8).all() and (ob.arrays["payload_len"] == 5).all()
    eng = emu_engine(3, rows_per_doc=4096, window_per_doc=1024, propsets_per_doc=4096, text_per_doc=1 << 14)
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.generate(p)
    eng.sync()
    assert (eng.status(range(3)) == 0).all()
    gb = eng.generated_download()
    for k in ("type", "flags", "client", "seq", "ref_seq", "msn", "pos1", "pos2", "payload_len", "prop_id"):
        assert np.array_equal(gb.arrays[k], ob.arrays[k]), k
    for d in range(3):
        assert len(kept[d].dump()) == 600          # alternating props: no two neighbours coalesce
        assert np.array_equal(eng.dump(d), kept[d].dump())


def check_deep_window(factory, n, pre, ops, lag, rows, window, text, psets=8192, residency=None):
    props = ann_props()
    eng = factory(n, rows_per_doc=rows, window_per_doc=window, propsets_per_doc=psets, text_per_doc=text)
    eng.upload_props(props)
    eng.upload_names(NAMES)
    pa = prebuild_params(n, pre)
    eng.generate(pa)
    eng.sync()
    a = eng.generated_download()
    eng.checkpoint()
    pb = gen_params(seed=505, n_docs=n, ops=ops, clients=8, lag=lag, ins=60, rem=40, ins_len=8, rem_len=8)
    pb.continue_docs = 1
    eng.generate(pb)
    eng.sync()
    assert (eng.status(range(n)) == 0).all()
    b = eng.generated_download()
    assert (b.arrays["seq"][b.op_offsets[:-1]] == pre + 1).all()     # continues the pre-built documents
    neg = np.full(n, -1, np.int32)
    dig_gen = eng.snapshot_digests(range(n), neg, neg, threads=2)
    eng.restore()
    if residency is not None:
        eng.set_residency(*residency)
    eng.generated_to_resident()
    eng.replay_resident()
    eng.sync()
    assert (eng.status(range(n)) == 0).all()
    dig_replay = eng.snapshot_digests(range(n), neg, neg, threads=2)
    assert np.array_equal(dig_gen, dig_replay)
    both = concat(a, b)
    last = both.op_offsets[1:] - 1
    for d, (od, st) in enumerate(replay(both, props, NAMES)):
        assert st == 0
        assert eng.get_text([d])[0] == od.get_text()
        assert np.array_equal(eng.dump(d), od.dump())
        assert int(dig_replay[d]) == od.snapshot(int(both.arrays["msn"][last[d]]), int(both.arrays["seq"][last[d]]))[1]


# residency: (2) blk (blocks outgrow LDS: HBM continuation), (3) long-document mode with
# the compiled LDS caps, with a 64-entry LDS window (the rest in HBM) and an 8-entry heap
# cap that forces the in-wave hand-over (block cache written back mid-run), and with the
# block cache, zamboni prefetch, corrections table and parent cache off (blocks = MT_BIGF_*
# switches).
@pytest.mark.parametrize("res", [(2, 0, 0, 0), (3, 0, 0, 0), (3, 64, 0, 8), (3, 0, 7, 0), (3, 0, 8, 0)])
@pytest.mark.parametrize("lag", [64, 512])
def test_deep_window_on_checkpoint_matches_oracle(lag, res):
    check_deep_window(emu_engine, 2, 3000, 1500, lag, rows=12000, window=8192, text=1 << 16, residency=res)


@pytest.mark.gpu
@pytest.mark.parametrize("res", [(2, 0, 0, 0), (3, 0, 0, 0), (3, 64, 0, 8), (3, 0, 7, 0)])
@pytest.mark.parametrize("lag", [512, 1024])
def test_gpu_config4_downscaled_matches_oracle(lag, res):
    """SURVEY §8(c)'s config-4 down-scale on the device: 2 documents pre-built to 20k
    segments, checkpointed, then a deep-window stream (lag up to 1,024, tree height 5+)
    generated on top and replayed from the restored checkpoint."""
    check_deep_window(lambda n, **kw: Engine(n, device=0, **kw), 2, 20000, 4000, lag,
                      rows=40000, window=16384, text=1 << 18, psets=40000, residency=res)


def check_size_classes(factory, counts, big_min_ops, partition_cus=0):
    """mt_set_size_class: the longer runs of a batch go to the long-document kernel (LDS heap,
    window and U set) while the rest stay under block residency; every document must still
    match the oracle."""
    props = ann_props()
    n = len(counts)
    p = gen_params(seed=77, n_docs=n, ops=8, clients=5, lag=48, ins=60, rem=30, ins_len=8, rem_len=8, ann_sets=24,
                   rewrite=5)
    batch, st, _ = generate(p, props, ops_per_doc=counts, clients_per_doc=[5] * n)
    assert st == [0] * n
    eng = factory(n, rows_per_doc=3 * max(counts) + 64, window_per_doc=8192, propsets_per_doc=2 * max(counts) + 64,
                  text_per_doc=8 * max(counts) + 4096)
    eng.upload_props(props)
    eng.upload_names(NAMES)
    eng.set_residency(2)
    if partition_cus:
        eng.set_partition(big_min_ops, partition_cus)   # long runs on reserved CUs, one per SIMD
    else:
        eng.set_size_class(big_min_ops)
    eng.open_docs(0, n)
    eng.apply(batch)
    eng.sync()
    assert (eng.status(range(n)) == 0).all()
    last = batch.op_offsets[1:] - 1
    neg = np.full(n, -1, np.int32)
    dig = eng.snapshot_digests(range(n), neg, neg, threads=2)
    for d, (od, ost) in enumerate(replay(batch, props, NAMES)):
        assert ost == 0
        assert eng.get_text([d])[0] == od.get_text(), d
        assert np.array_equal(eng.dump(d), od.dump()), d
        assert int(dig[d]) == od.snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]))[1], d


def test_size_classes_match_oracle_on_emulation():
    check_size_classes(emu_engine, [300, 2500, 80, 1200, 40, 3000], 1000)


@pytest.mark.gpu
def test_size_classes_match_oracle_on_gpu():
    check_size_classes(lambda n, **kw: Engine(n, device=0, **kw), [300, 2500, 80, 1200, 40, 3000, 9000, 700] * 4, 1000)


def test_partition_classes_match_oracle_on_emulation():
    check_size_classes(emu_engine, [300, 2500, 80, 1200, 40, 3000], 1000, partition_cus=8)


@pytest.mark.gpu
def test_partition_classes_match_oracle_on_gpu():
    """mt_set_partition: the long runs on CU-masked stream A with padded LDS, the rest on B."""
    check_size_classes(lambda n, **kw: Engine(n, device=0, **kw), [300, 2500, 80, 1200, 40, 3000, 9000, 700] * 4, 1000,
                       partition_cus=32)
