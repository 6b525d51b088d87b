"""Debug aid: apply the first K ops of run RUN (seed SEED, cfg2, 4 docs) as one batch with a
printf-instrumented engine (MT_DBG_PRINT builds).  usage: python tools/dbg_trace.py emu|gpu K"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from fluidframework_amd.engine import Engine  # noqa: E402
from oracle_lib import gen_params, generate  # noqa: E402
from test_emu_parity import CONFIGS, NAMES, ann_props  # noqa: E402
from test_snapshot_load import sub_batch  # noqa: E402

which, K = sys.argv[1], int(sys.argv[2])
SEED, RUN = int(os.environ.get("DBG_SEED", "41")), int(os.environ.get("DBG_RUN", "1"))
props = ann_props()
batch, _, _ = generate(gen_params(seed=SEED, n_docs=4, **{**CONFIGS["cfg2"], "ops": 1500}), props)
kw = dict(rows_per_doc=20000, window_per_doc=8192, propsets_per_doc=8192, text_per_doc=1 << 18)
if which == "emu":
    e = Engine(1, lib_path=os.path.join(ROOT, "tests", "emu", "libmtemu_dbg.so"), prefix="emu_", **kw)
else:
    e = Engine(1, lib_path=os.path.join(ROOT, "fluidframework_amd", "libmtgpu_vPRINT.so"), device=0, **kw)
e.upload_props(props)
e.upload_names(NAMES)
e.open_docs(0, 1)
e.apply(sub_batch(batch, RUN, 0, K, 0))
e.sync()
sys.stdout.flush()
print("status", e.status([0]))
