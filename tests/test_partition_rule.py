"""The size-class partition rule (mt_plan_partition, DESIGN.md §3 "The partition rule"): a model
of the measured kernels that picks which long runs replay in the wide block-residency kernel and
on how many CUs.  Pinned here against the round-6 measurements it reproduces
(profiles/r06/partition/, profiles/r06/final/): config 5 at 131,072 documents is latency-bound
(256:192 measured at 885-890 ms), 1,048,576 documents on one GPU are throughput-bound (no
partition, 3,067 ms), config 2 has no long runs (no partition, 153.5-154 ms).  The host
emulation compiles the same mt_api_impl.h, so no GPU is needed; the product library's own
entry point (mt_plan_partition) is the same function."""
import numpy as np
import pytest

from emu_lib import emu_engine
from fluidframework_amd.batch import MtGenParams
from fluidframework_amd.engine import MergeTreeError
from fluidframework_amd.shard import clients_per_doc, generation_caps, zipf_op_counts

SEED = 20241015                    # bench.py --seed default: config 5's op counts at N = 1


@pytest.fixture(scope="module")
def eng():
    e = emu_engine(1)
    yield e
    e.close()


def test_rule_reproduces_the_measured_config5_lines(eng):
    m, k, est = eng.plan_partition(zipf_op_counts(131072, SEED), 256)
    assert (m, k) == (256, 192)                       # the bench line's partition_info
    assert abs(est - 887.0) < 0.03 * 887.0            # 885.4-889.5 ms measured
    m, k, est = eng.plan_partition(zipf_op_counts(1048576, SEED), 256)
    assert (m, k) == (0, 0)                           # partitioning loses at 1M documents
    assert abs(est - 3067.0) < 0.03 * 3067.0          # 3,066.9 ms measured
    m, k, est = eng.plan_partition(np.full(4096, 10000, np.uint32), 256)
    assert (m, k) == (0, 0) and abs(est - 153.7) < 0.03 * 153.7


def test_rule_edge_cases(eng):
    assert eng.plan_partition([], 256) == (0, 0, 0.0)
    assert eng.plan_partition([5], 256)[:2] == (0, 0)
    assert eng.plan_partition([65536] * 10, 1)[:2] == (0, 0)        # one CU: nothing to reserve
    with pytest.raises(MergeTreeError):
        eng.plan_partition([100], 0)


@pytest.mark.parametrize("seed", range(6))
def test_rule_picks_whole_xcd_shares(eng, seed):
    """Any pick is a power-of-two split length in [256, 32768] and a whole number of XCD shares
    (ncu / 8) short of the whole chip, and its estimate beats no partition by 5 %."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1000, 200000))
    ops = np.minimum(rng.zipf(1.3 + 0.1 * seed, n), 65536).astype(np.uint32) * int(rng.integers(1, 8))
    for ncu in (64, 256):
        m, k, est = eng.plan_partition(ops, ncu)
        if k:
            assert m in [256 << i for i in range(8)] and k % (ncu // 8) == 0 and 0 < k < ncu
            off = eng.plan_partition(ops[ops < 0], ncu)   # (empty: 0) sanity of the call itself
            assert off == (0, 0, 0.0) and est > 0


def test_auto_partition_replays_like_no_partition_on_emulation():
    check_auto_partition(emu_engine)


@pytest.mark.gpu
def test_auto_partition_replays_like_no_partition_on_gpu():
    from fluidframework_amd.engine import Engine
    check_auto_partition(lambda n, **kw: Engine(n, device=0, **kw))


def check_auto_partition(factory):
    """MT_PARTITION_AUTO takes the plan of the resident batch's run lengths (mt_last_partition)
    and its documents' snapshots equal those of the same batch replayed unpartitioned."""
    n = 1024
    ops = np.full(n, 100, np.uint32)
    ops[:4] = 12000                 # a latency-bound tail: runs past the block kernel's LDS (~10k)
    cl = clients_per_doc(n, 7)
    out = {}
    for mode in ("auto", 0):
        e = factory(n, per_doc=generation_caps(ops, 8))
        e.set_residency(2)
        e.upload_props(__import__("bench").ann_props())
        e.upload_names(['"c%d"' % i for i in range(64)])
        e.set_partition(mode)
        e.generate(MtGenParams(7, n, 0, 2, 32, 60, 40, 8, 8, 1, 0), ops_per_doc=ops, clients_per_doc=cl)
        e.sync()
        e.generated_to_resident()
        e.open_docs(0, n)
        e.replay_resident()
        e.sync()
        assert not e.status(range(n)).any()
        neg = np.full(n, -1, np.int32)
        out[mode] = (e.snapshot_digests(range(n), neg, neg, threads=4), e.partition_info())
        if mode == "auto":
            m, k, _ = e.plan_partition(ops, 256)
            assert (m, k) != (0, 0), "case meant to partition"
            assert out[mode][1] == {"min_msgs": m, "cus": k}
        e.close()
    assert out[0][1] is None
    assert np.array_equal(out["auto"][0], out[0][0])
