"""Debug aid: replay one generated document op by op on the GPU and on the host emulation,
and report the first op after which their status or row dump differ.
usage: python tools/dbg_first_divergence.py [cfg] [ops]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from emu_lib import emu_engine  # noqa: E402
from fluidframework_amd.engine import Engine  # noqa: E402
from oracle_lib import gen_params, generate  # noqa: E402
from test_emu_parity import CONFIGS, NAMES, ann_props  # noqa: E402
from test_snapshot_load import sub_batch  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg1"
n_ops = int(sys.argv[2]) if len(sys.argv) > 2 else 200
props = ann_props()
SEED = int(os.environ.get("DBG_SEED", "11"))
NDOC = int(os.environ.get("DBG_NDOC", "1"))       # stream = run DBG_RUN of an NDOC-document generation
RUN = int(os.environ.get("DBG_RUN", "0"))
p = gen_params(seed=SEED, n_docs=NDOC, **{**CONFIGS[cfg], "ops": n_ops})
batch, st, _ = generate(p, props)
engs = []
for f in (emu_engine, lambda n, **kw: Engine(n, device=0, **kw)):
    e = f(1, rows_per_doc=20000, window_per_doc=8192, propsets_per_doc=8192, text_per_doc=1 << 18)
    e.upload_props(props)
    e.upload_names(NAMES)
    e.open_docs(0, 1)
    engs.append(e)
o0 = int(batch.op_offsets[RUN])
a = {k: v[o0:] for k, v in batch.arrays.items()}
if os.environ.get("DBG_DOCS"):
    nd = int(os.environ["DBG_DOCS"])
    pm = gen_params(seed=SEED, n_docs=nd, **{**CONFIGS[cfg], "ops": n_ops})
    bm, _, _ = generate(pm, props)
    out = []
    for f in (emu_engine, lambda n, **kw: Engine(n, device=0, **kw)):
        e = f(nd, rows_per_doc=20000, window_per_doc=8192, propsets_per_doc=8192, text_per_doc=1 << 18)
        e.upload_props(props); e.upload_names(NAMES); e.open_docs(0, nd)
        e.apply(bm); e.sync()
        out.append((e.status(range(nd)), [e.dump(d) for d in range(nd)]))
    print("status emu", out[0][0], "gpu", out[1][0])
    for d in range(nd):
        de, dg = out[0][1][d], out[1][1][d]
        print("doc", d, "same" if de.shape == dg.shape and (de == dg).all() else f"DIFF {de.shape} {dg.shape}")
    sys.exit(0)
if os.environ.get("DBG_PREFIX"):
    # prefix k applied in ONE batch to fresh documents: first k whose result differs
    def run(k):
        res = []
        for f in (emu_engine, lambda n, **kw: Engine(n, device=0, **kw)):
            e = f(1, rows_per_doc=20000, window_per_doc=8192, propsets_per_doc=8192, text_per_doc=1 << 18)
            e.upload_props(props); e.upload_names(NAMES); e.open_docs(0, 1)
            if os.environ.get("DBG_RES"):
                e.set_residency(*[int(x) for x in os.environ["DBG_RES"].split(",")])
            e.apply(sub_batch(batch, RUN, 0, k, 0)); e.sync()
            res.append((int(e.status([0])[0]), e.dump(0), e.pools([0])[0]))
        (se, de, pe), (sg, dg, pg) = res
        ok = se == sg and de.shape == dg.shape and (de == dg).all() and (pe == pg).all()
        return ok, [(se, de), (sg, dg), (pe, pg)]
    lo, hi = 0, n_ops                       # run(lo) matches; find the smallest failing prefix
    if run(hi)[0]:
        print("no prefix divergence in", n_ops)
        sys.exit(0)
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if run(mid)[0]: lo = mid
        else: hi = mid
    for k in [hi]:
        ok, res = run(k)
        if not ok:
            i = k - 1
            print(f"prefix {k} differs; last op {i}: type {a['type'][i]} pos1 {a['pos1'][i]} pos2 {a['pos2'][i]} "
                  f"len {a['payload_len'][i]} seq {a['seq'][i]} ref {a['ref_seq'][i]} msn {a['msn'][i]} client {a['client'][i]}")
            (se, de), (sg, dg), (pe, pg) = res
            print("pools emu", pe.tolist(), "gpu", pg.tolist())
            print("status emu", se, "gpu", sg, "shapes", de.shape, dg.shape)
            m = min(len(de), len(dg))
            bad = np.nonzero((de[:m] != dg[:m]).any(axis=1))[0]
            print("differing rows", bad[:20])
            for r in bad[:10]:
                print(" row", r, "emu", de[r].tolist(), "gpu", dg[r].tolist())
            for j in range(max(0, i - 3), i):
                print(f"  op {j}: type {a['type'][j]} pos1 {a['pos1'][j]} pos2 {a['pos2'][j]} len {a['payload_len'][j]} "
                      f"seq {a['seq'][j]} ref {a['ref_seq'][j]} msn {a['msn'][j]} client {a['client'][j]}")
            sys.exit(1)
    print("no prefix divergence in", n_ops)
    sys.exit(0)
for i in range(n_ops):
    sb = sub_batch(batch, 0, i, i + 1, 0)
    out = []
    for e in engs:
        e.apply(sb)
        e.sync()
        out.append((int(e.status([0])[0]), e.dump(0)))
    (se, de), (sg, dg) = out
    same = se == sg and de.shape == dg.shape and (de == dg).all()
    if not same:
        print(f"op {i}: type {a['type'][i]} pos1 {a['pos1'][i]} pos2 {a['pos2'][i]} len {a['payload_len'][i]} "
              f"seq {a['seq'][i]} ref {a['ref_seq'][i]} msn {a['msn'][i]} client {a['client'][i]}")
        print("status emu", se, "gpu", sg)
        print("emu rows\n", de[:40])
        print("gpu rows\n", dg[:40])
        sys.exit(1)
print("no divergence in", n_ops, "ops")
