"""Diagnostic: config-5 exchange at scale.  Generates like shard.build_sharded, applies
its record permutation (index_select), and checks document 0's records at its LPT
position against the oracle's generator; then uploads them with upload_batch_dev into a
fresh engine and replays only that document."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import bench
from fluidframework_amd.batch import MtGenParams
from fluidframework_amd.shard import zipf_op_counts, clients_per_doc, generation_caps, rank_order, lpt_assign
N = int(sys.argv[1]); seed = 20241015; L = 8
c = dict(bench.CONFIGS["config5"])
ops = zipf_op_counts(N, seed); cli = clients_per_doc(N, seed)
eng = bench.Host.engine(N, 0, per_doc=generation_caps(ops, L))
eng.upload_names(['"c%d"' % i for i in range(64)])
p = MtGenParams(seed, N, 0, 2, c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"], c["rewrite"])
eng.generate(p, ops_per_doc=ops, clients_per_doc=cli); eng.sync()
n_total = int(ops.sum())
rec_all = torch.empty((n_total, 4), dtype=torch.int64, device="cuda"); pay_all = torch.empty((n_total, 2), dtype=torch.int64, device="cuda")
torch.cuda.synchronize(); eng.generated_copy_dev(0, N, rec_all.data_ptr(), pay_all.data_ptr()); eng.close()
owner = lpt_assign(ops, 1); order = rank_order(owner, ops)
op_off = np.zeros(N + 1, np.int64); op_off[1:] = np.cumsum(ops)
lens = ops[order].astype(np.int64); starts = op_off[order]
op_idx = np.repeat(starts - np.concatenate(([0], np.cumsum(lens)[:-1])), lens) + np.arange(int(lens.sum()))
sel = torch.from_numpy(op_idx).cuda()
rec_send = rec_all.index_select(0, sel); pay_send = pay_all.index_select(0, sel); torch.cuda.synchronize()
pos0 = int(np.nonzero(order == 0)[0][0]); loc = np.zeros(N + 1, np.int64); loc[1:] = np.cumsum(lens)
a0, a1 = int(loc[pos0]), int(loc[pos0 + 1])
got = rec_send[a0:a1].cpu().numpy().view(np.int32).reshape(-1, 8)
ref = rec_all[int(op_off[0]):int(op_off[1])].cpu().numpy().view(np.int32).reshape(-1, 8)
print("N", N, "doc0 LPT pos", pos0, "byte offset of its records", a0 * 32, "records equal after index_select", bool((got == ref).all()))
pg = pay_send[a0:a1].cpu().numpy(); pr = pay_all[int(op_off[0]):int(op_off[1])].cpu().numpy()
print("payload equal after index_select", bool((pg == pr).all()))
v_adv = pay_all[sel]; torch.cuda.synchronize()
print("payload via advanced indexing", bool((v_adv[a0:a1].cpu().numpy() == pr).all()))
v32 = pay_all.view(torch.int32).index_select(0, sel); torch.cuda.synchronize()
print("payload via int32 (n,4) index_select", bool((v32[a0:a1].cpu().numpy().view(np.int64) == pr).all()))
comb = torch.cat([rec_all, pay_all], dim=1).index_select(0, sel); torch.cuda.synchronize()
print("payload via combined (n,6) index_select", bool((comb[a0:a1, 4:].cpu().numpy() == pr).all()),
      "records", bool((comb[a0:a1, :4].cpu().numpy().view(np.int32).reshape(-1, 8) == ref).all()))
print("pay_send first mismatch rows", np.nonzero((pg != pr).any(axis=1))[0][:5], pg[:2], pr[:2])
