"""Diagnostic: is the device generation of config-5 streams at scale equal to the
oracle's generator for the first documents?  (records + payload of runs 0..47)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import bench
from fluidframework_amd.batch import MtGenParams
from fluidframework_amd.shard import zipf_op_counts, clients_per_doc, generation_caps
N = int(sys.argv[1]); k = 48; seed = 20241015
c = dict(bench.CONFIGS["config5"])
ops = zipf_op_counts(N, seed); cli = clients_per_doc(N, seed)
eng = bench.Host.engine(N, 0, per_doc=generation_caps(ops, 8))
eng.upload_names(['"c%d"' % i for i in range(64)])
p = MtGenParams(seed, N, 0, 2, c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"], c["rewrite"])
eng.generate(p, ops_per_doc=ops, clients_per_doc=cli); eng.sync()
n48 = int(ops[:k].sum())
rec = torch.zeros((n48, 4), dtype=torch.int64, device="cuda"); pay = torch.zeros((n48, 2), dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
eng.generated_copy_dev(0, k, rec.data_ptr(), pay.data_ptr()); torch.cuda.synchronize()
r = rec.cpu().numpy().view(np.int32).reshape(n48, 8)
from oracle_lib import generate
q = MtGenParams(seed, k, 0, 2, c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"], c["rewrite"])
b, st, _ = generate(q, bench.ann_props(), docs=range(k), keep=False, ops_per_doc=ops[:k], clients_per_doc=cli[:k])
a = b.arrays
print("N", N, "ops total", int(ops.sum()), "first-48 ops", n48)
print("seq eq", bool((r[:, 1] == a["seq"]).all()), "ref eq", bool((r[:, 2] == a["ref_seq"]).all()),
      "pos1 eq", bool((r[:, 4] == a["pos1"]).all()), "type eq", bool(((r[:, 0] & 0xFF) == a["type"]).all()))
poff = r[:, 6].astype(np.int64); first_bad = np.nonzero(r[:, 4] != a["pos1"])[0][:3]
print("first bad ops", first_bad, "payload_off[:4]", poff[:4])
