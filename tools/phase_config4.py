"""Diagnostic: phase (s_memtime) profile of config 4's measured stream on the
pre-built long documents.  MT_PROF_FLAG=MT_PROFILE|MT_PROFILE2 picks the build."""
import ctypes as C, os, subprocess, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fluidframework_amd.engine import Engine
from fluidframework_amd.batch import MtGenParams
import bench
flag = os.environ.get("MT_PROF_FLAG", "MT_PROFILE")
lib = os.path.join(ROOT, "fluidframework_amd", f"libmtgpu_{flag.lower()}.so")
if not os.path.exists(lib):                       # build here (CPU) before shipping it to a GPU run
    sys.path.insert(0, ROOT)
    import __graft_entry__
    __graft_entry__.build_engine(extra=[f"-D{flag}"], out=lib, force=True)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
pre = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
ops = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
res = sys.argv[4] if len(sys.argv) > 4 else "blk"
c = bench.CONFIGS["config4"]
rows = pre + 3 * ops + 64
eng = Engine(n, lib_path=lib, rows_per_doc=rows, blocks_per_doc=rows // 2 + 64, heap_per_doc=rows, window_per_doc=16384,
             text_per_doc=5 * pre + 8 * ops + 4096, propsets_per_doc=pre + ops + 64)
eng.upload_props(bench.ann_props()); eng.upload_names(['"c%d"' % i for i in range(64)])
pa = MtGenParams(1, n, pre, 1, 0, 100, 0, 5, 1, 1, 0); pa.ins_len_min, pa.seg_prop_sets, pa.ins_at_end = 5, 2, 1
eng.generate(pa); eng.sync(); eng.checkpoint()
pb = MtGenParams(2, n, ops, 8, 1024, 60, 40, 8, 8, 2, 0); pb.continue_docs = 1
eng.generate(pb); eng.sync(); eng.generated_to_resident(); eng.restore()
if res == "big" and os.environ.get("MT_BIG_FLAGS"):
    eng.set_residency(bench.RESIDENCY[res], 0, int(os.environ["MT_BIG_FLAGS"]), 0)   # MT_BIGF_* switches (A/B)
else:
    eng.set_residency(bench.RESIDENCY[res])
fn = eng.lib.mt_prof_get; fn.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
base = np.zeros((n, 8), np.uint64); fn(eng.h, n, base.ctypes.data)
t = time.time(); eng.replay_resident(); eng.sync(); dt = time.time() - t
raw = np.zeros((n, 8), np.uint64); fn(eng.h, n, raw.ctypes.data)
tot = (raw - base).sum(axis=0).astype(float)
names = ["computeU", "split-walks", "insert-walk", "rangeMap", "zamboni", "op-total", "gen", "textGC"]
if flag == "MT_PROFILE2":
    names = ["walk blkLoad", "walk childLens", "walk levels(n)", "computeU", "computeU(n)", "heapGet", "heapGet(n)", "scourLeaf"]
if flag == "MT_PROFILE4":
    names = ["U scan", "htBuild", "ht levels(n)", "U entries(n)", "window(n)", "computeU(n)", "parent lookups(n)",
             "parent misses(n)"]
print(f"{flag} residency={res} config4 docs={n} prebuild={pre} ops={ops} replay wall {dt*1e3:.1f} ms; per-doc mean cycles per msg:")
for i, nm in enumerate(names):
    print(f"  {nm:16s} {tot[i]/n/ops:10.0f}")
