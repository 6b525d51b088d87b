"""Diagnostic: config-5 digest parity at scale.  Builds the sharded replay exactly as
bench.py does (one rank), replays once, and compares for the smallest-id documents:
(a) the digests of the full gather, (b) digests taken for those documents alone,
(c) the oracle's own generation + replay (checker).  Also the text of doc 0."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import bench
from fluidframework_amd.batch import MtGenParams
from fluidframework_amd.shard import SoloDist, build_sharded, rank_order
docs = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
c = dict(bench.CONFIGS["config5"]); seed = 20241015
gen_kw = dict(lag_max=c["lag"], pct_insert=c["ins"], pct_remove=c["rem"], ins_len_max=c["ins_len"],
              rem_len_max=c["rem_len"], n_ann_sets=c["ann_sets"], pct_rewrite=c["rewrite"])
dev = torch.device("cuda", 0)
fac = lambda n, caps: bench.Host.engine(n, 0, per_doc=caps)
sh = build_sharded(SoloDist(), dev, fac, docs, seed, MtGenParams, gen_kw, names=['"c%d"' % i for i in range(64)])
eng = sh.engine
sh.replay(); eng.sync()
print("status any", bool(eng.status(range(sh.n_docs)).any()))
digs = sh.gather_digests(SoloDist(), dev, threads=16)
k = 48
order = rank_order(sh.owner, sh.all_ops)
pos = np.empty(len(order), np.int64); pos[order] = np.arange(len(order))
neg = np.full(k, -1, np.int32)
sub = eng.snapshot_digests(pos[:k], neg, neg, threads=4)
from oracle_lib import generate
p = MtGenParams(seed, k, 0, 2, c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"], c["rewrite"])
batch, st, kept = generate(p, bench.ann_props(), docs=range(k), keep=True, ops_per_doc=sh.all_ops[:k], clients_per_doc=sh.clients_all[:k])
last = batch.op_offsets[1:] - 1
odg = np.array([kept[d].snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]))[1] for d in range(k)], np.uint64)
print("gather==sub", int((digs[:k] == sub).sum()), "sub==oracle", int((sub == odg).sum()), "gather==oracle", int((digs[:k] == odg).sum()))
t = eng.get_text([int(pos[0])])[0]
print("doc0 text eq", t == kept[0].get_text(), len(t), len(kept[0].get_text()), "ops", int(sh.all_ops[0]), "clients", int(sh.clients_all[0]))
