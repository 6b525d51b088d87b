"""Multi-rank document sharding (fluidframework_amd/shard.py): LPT plan,
rank-0 ingest -> all_to_all redistribution -> per-rank replay -> digest gather,
on world_size 2 with the gloo backend and the host emulation of the engine.
The gathered digests must equal the oracle's for every document and a
single-rank run's."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from fluidframework_amd.shard import clients_per_doc, lpt_assign, zipf_op_counts

NAMES = ['"c%d"' % i for i in range(64)]
GEN = dict(lag_max=32, pct_insert=60, pct_remove=40, ins_len_max=8, rem_len_max=8, n_ann_sets=1, pct_rewrite=0)


def test_zipf_counts_range_and_mean():
    c = zipf_op_counts(200000, seed=5)
    assert c.min() >= 8 and c.max() <= 65536
    assert 550 < c.mean() < 850          # truncated Zipf(1.5) on [8, 65536]: mean ~700
    assert np.array_equal(c, zipf_op_counts(200000, seed=5))
    k = clients_per_doc(1000, seed=5)
    assert k.min() >= 2 and k.max() <= 16


def test_lpt_is_deterministic_and_balanced():
    c = zipf_op_counts(5000, seed=9)
    o = lpt_assign(c, 8)
    assert np.array_equal(o, lpt_assign(c, 8))
    loads = np.bincount(o, weights=c, minlength=8)
    assert loads.max() - loads.min() <= c.max()          # LPT bound
    assert loads.max() / loads.mean() < 1.05


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, docs, counts, clients, out):
    import sys
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from emu_lib import build_emu
    from fluidframework_amd.batch import MtGenParams
    from fluidframework_amd.engine import Engine
    from fluidframework_amd.shard import build_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = build_emu()
    fac = lambda n, caps: Engine(n, lib_path=lib, prefix="emu_", per_doc=caps)
    sh = build_sharded(dist, torch.device("cpu"), fac, docs, 77, MtGenParams, GEN, names=NAMES, chunk_docs=5,
                       counts=counts, clients=clients)
    # every received document's rows matched rank 0's checksum (mt_upload_rows_dev)
    assert sh.timings["exchange_bad_docs"] == 0 and sh.timings["exchange_checked_docs"] == sh.n_docs
    sh.replay()
    sh.engine.sync()
    assert (sh.engine.status(range(sh.n_docs)) == 0).all()
    dig = sh.gather_digests(dist, torch.device("cpu"), threads=2)
    if rank == 0:
        np.save(out, dig)
    dist.barrier()
    dist.destroy_process_group()


def _run(world, docs, counts, clients, tmp_path):
    out = str(tmp_path / f"dig_{world}.npy")
    mp.start_processes(_worker, args=(world, _free_port(), docs, counts, clients, out), nprocs=world,
                       join=True, start_method="spawn")
    return np.load(out)


def test_sharded_replay_gloo_world2_matches_oracle(tmp_path):
    from oracle_lib import gen_params, generate
    from fluidframework_amd.batch import PropTable
    docs = 9
    counts = np.array([8, 40, 700, 13, 300, 1500, 64, 9, 250], np.uint32)
    clients = np.array([2, 16, 5, 9, 3, 8, 2, 4, 11], np.uint32)
    d2 = _run(2, docs, counts, clients, tmp_path)
    d1 = _run(1, docs, counts, clients, tmp_path)
    assert np.array_equal(d1, d2)
    p = gen_params(seed=77, n_docs=docs, clients=2, lag=32, ins=60, rem=40, ins_len=8, rem_len=8, ops=8)
    batch, st, kept = generate(p, PropTable(), ops_per_doc=counts, clients_per_doc=clients, keep=True)
    for d in range(docs):
        kept[d].set_names(NAMES)
    last = batch.op_offsets[1:] - 1
    want = [kept[d].snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]))[1] for d in range(docs)]
    assert [int(x) for x in d2] == want


@pytest.mark.parametrize("world", [4, 8])
def test_sharded_replay_gloo_wide_matches_oracle(world, tmp_path):
    """The 4- and 8-rank path on ~2,000 Zipf documents (sizes capped at 1,024 messages so the
    emulation finishes in seconds): the LPT split gives every rank a share, rank 0 is the only
    sender of the all_to_all_single (the other senders are empty), and the gathered digests
    come back in global document order, equal to a single rank's and to the oracle's."""
    from oracle_lib import gen_params, generate
    from fluidframework_amd.batch import PropTable
    docs = 2000
    counts = zipf_op_counts(docs, 11, hi=1024)
    clients = clients_per_doc(docs, 11)
    owner = lpt_assign(counts, world)
    assert (np.bincount(owner, minlength=world) > 0).all()
    dw = _run(world, docs, counts, clients, tmp_path)
    d1 = _run(1, docs, counts, clients, tmp_path)
    assert np.array_equal(dw, d1)
    p = gen_params(seed=77, n_docs=docs, clients=2, lag=32, ins=60, rem=40, ins_len=8, rem_len=8, ops=8)
    batch, st, kept = generate(p, PropTable(), ops_per_doc=counts, clients_per_doc=clients, keep=True,
                               threads=min(8, os.cpu_count() or 1))
    assert not any(st)
    last = batch.op_offsets[1:] - 1
    want = np.array([kept[d].snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]))[1]
                     for d in range(docs)], np.uint64)
    assert np.array_equal(dw, want)


def test_north_star_rank0_memory_fits_at_8_ranks():
    """Host-only sizing of rank 0 at N = 8 for the north_star's 1,048,576 Zipf documents:
    the send buffer of every document's exchange rows, the largest generating engine (a chunk
    of 131,072 documents with generation caps), the rows it receives and the engine for its
    own share must fit in one MI355X's 288 GB.  The pool estimate is the library's own
    (mt_pool_bytes), checked here against the emulation library on a small population."""
    from emu_lib import emu_engine
    from fluidframework_amd.shard import generation_caps, pool_bytes_estimate, rank0_peak_bytes
    small = zipf_op_counts(40, 3, hi=2048)
    caps = generation_caps(small, 8)
    eng = emu_engine(len(small), per_doc=caps)
    assert eng.pool_bytes() == pool_bytes_estimate(caps)
    ops = zipf_op_counts(1048576, 20241015)
    peak = rank0_peak_bytes(ops, world=8, ins_len=8)
    assert peak["total"] < 288e9, peak
    assert peak["send"] == int(ops.sum()) * (32 + 2 * 8)


class HostRows:
    """Exchange-row buffers in host memory (the emulation's "device" pointers)."""

    @staticmethod
    def zeros(n, w):
        return np.zeros((n, w), np.uint64)

    @staticmethod
    def ptr(a):
        return a.ctypes.data

    @staticmethod
    def corrupt(a, r, w, how):
        b = a.copy()
        if how == "bit":
            b[r, w] ^= np.uint64(1 << 17)
        else:
            b[r, :] = 0
        return b


def check_exchange_rows(factory, buf):
    """mt_generated_pack_rows / mt_upload_rows_dev: rows round-trip into a resident batch that
    replays exactly like the generated one, and any flipped bit or zeroed row of a document is
    reported for that document only (MT_E_EXCHANGE)."""
    from fluidframework_amd.batch import MtGenParams, PropTable
    from fluidframework_amd.engine import ExchangeError
    from fluidframework_amd.shard import generation_caps
    counts = np.array([30, 7, 120, 64], np.uint32)
    clients = np.array([3, 2, 9, 4], np.uint32)
    L = GEN["ins_len_max"]
    caps = generation_caps(counts, L)
    src = factory(4, per_doc=caps)
    src.upload_props(PropTable())
    src.upload_names(NAMES)
    src.generate(MtGenParams(**{**GEN, "seed": 5, "n_docs": 4, "ops_per_doc": 0, "clients": 2}),
                 ops_per_doc=counts, clients_per_doc=clients)
    src.sync()
    W = 4 + L // 4
    order = np.array([2, 0, 3, 1])                         # a plan: send order differs from generation order
    row_of = np.empty(4, np.int64)
    row_of[order] = np.concatenate(([0], np.cumsum(counts[order].astype(np.int64))[:-1]))
    rows = buf.zeros(int(counts.sum()), W)
    sums = src.generated_pack_rows(0, 4, row_of.astype(np.uint64), buf.ptr(rows))
    off = np.concatenate(([0], np.cumsum(counts[order]))).astype(np.uint32)
    dst = factory(4, per_doc={k: np.asarray(v)[order] for k, v in caps.items()})
    dst.upload_props(PropTable())
    dst.upload_names(NAMES)
    assert not dst.upload_rows_dev(range(4), off, buf.ptr(rows), L, sums[order]).any()
    dst.open_docs(0, 4)
    dst.replay_resident()
    dst.sync()
    assert (dst.status(range(4)) == 0).all()
    neg = np.full(4, -1, np.int32)
    want = src.snapshot_digests(range(4), neg, neg, threads=1)
    assert np.array_equal(dst.snapshot_digests(range(4), neg, neg, threads=1), want[order])
    for how in ("bit", "zero"):                             # corrupt the third document of the plan (doc 3)
        bad = buf.corrupt(rows, int(row_of[3]) + 5, W - 1, how)
        with pytest.raises(ExchangeError) as ei:
            dst.upload_rows_dev(range(4), off, buf.ptr(bad), L, sums[order])
        assert list(ei.value.bad_runs) == [0, 0, 1, 0]


def test_exchange_rows_checksum_catches_corruption():
    from emu_lib import emu_engine
    check_exchange_rows(emu_engine, HostRows)
