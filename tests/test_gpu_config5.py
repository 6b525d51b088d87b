"""Config 5's single-GPU path on the device (BASELINE config 5; fluidframework_amd/shard.py):
Zipf-sized documents generated on the GPU, packed into exchange rows by the HIP pack kernel
(mt_generated_pack_rows), moved by a world-size-1 all-to-all, unpacked with per-document
checksums by the HIP unpack kernel (mt_upload_rows_dev), replayed, and every SnapshotV1 digest
compared with the oracle's own generation + replay of the same documents; and the exchange's
checksum catching a flipped bit or a zeroed row on the device."""
import os

import numpy as np
import pytest

from test_shard import GEN, NAMES, check_exchange_rows

pytestmark = pytest.mark.gpu


class DevRows:
    """Exchange-row buffers in device memory (torch tensors on cuda:0)."""

    @staticmethod
    def zeros(n, w):
        import torch
        return torch.zeros((n, w), dtype=torch.int64, device="cuda:0")

    @staticmethod
    def ptr(a):
        return a.data_ptr()

    @staticmethod
    def corrupt(a, r, w, how):
        b = a.clone()
        if how == "bit":
            b[r, w] ^= 1 << 17
        else:
            b[r, :] = 0
        return b


def test_exchange_rows_checksum_catches_corruption_on_gpu():
    from fluidframework_amd.engine import Engine
    check_exchange_rows(lambda n, **kw: Engine(n, device=0, **kw), DevRows)


@pytest.mark.parametrize("docs,seed", [(2048, 11)])
def test_config5_zipf_exchange_replay_matches_oracle(docs, seed):
    import torch
    from fluidframework_amd.batch import MtGenParams, PropTable
    from fluidframework_amd.engine import Engine
    from fluidframework_amd.shard import SoloDist, build_sharded, clients_per_doc, zipf_op_counts
    from oracle_lib import generate
    counts = zipf_op_counts(docs, seed)
    clients = clients_per_doc(docs, seed)
    dev = torch.device("cuda", 0)
    fac = lambda n, caps: Engine(n, device=0, per_doc=caps)  # noqa: E731
    sh = build_sharded(SoloDist(), dev, fac, docs, seed, MtGenParams, GEN, names=NAMES, counts=counts, clients=clients)
    assert sh.timings["exchange_bad_docs"] == 0 and sh.timings["exchange_checked_docs"] == docs
    sh.replay()
    sh.engine.sync()
    assert (sh.engine.status(range(docs)) == 0).all()
    dig = sh.gather_digests(SoloDist(), dev, threads=16)
    # the oracle generates the same documents with its own generator and replays them
    p = MtGenParams(seed, docs, 0, 2, GEN["lag_max"], GEN["pct_insert"], GEN["pct_remove"], GEN["ins_len_max"],
                    GEN["rem_len_max"], GEN["n_ann_sets"], GEN["pct_rewrite"])
    batch, st, kept = generate(p, PropTable(), keep=True, ops_per_doc=counts, clients_per_doc=clients,
                               threads=min(16, os.cpu_count() or 1))
    assert not any(st)
    last = batch.op_offsets[1:] - 1
    for d in range(docs):
        kept[d].set_names(NAMES)
    want = np.array([kept[d].snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]))[1]
                     for d in range(docs)], np.uint64)
    assert int(counts.max()) > 4096                         # the Zipf tail is in the sample
    assert np.array_equal(dig, want), f"{int((dig != want).sum())} of {docs} digests differ"
