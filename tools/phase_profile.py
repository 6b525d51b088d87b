"""Diagnostic: per-phase shader-clock shares of the replay kernel (MT_PROFILE build).

Builds fluidframework_amd/csrc/mt_engine.hip with -DMT_PROFILE into
gpurun_out/libmtgpu_prof.so (a diagnostic build, never the product) and reads the
per-document phase cycle counters after one replay of a bench workload.
"""
import ctypes, os, subprocess, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fluidframework_amd.engine import Engine
from fluidframework_amd.batch import MtGenParams
import bench

flag = os.environ.get("MT_PROF_FLAG", "MT_PROFILE")
lib = os.environ.get("MTGPU_PROF_LIB") or os.path.join(ROOT, "fluidframework_amd", f"libmtgpu_{flag.lower()}.so")
if not os.path.exists(lib):                       # build here (CPU) before shipping it to a GPU run
    sys.path.insert(0, ROOT)
    import __graft_entry__
    __graft_entry__.build_engine(extra=[f"-D{flag}"], out=lib, force=True)
cfg = sys.argv[1] if len(sys.argv) > 1 else "config2"
docs = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
c = dict(bench.CONFIGS[cfg]); c["docs"] = docs
if len(sys.argv) > 3: c["ops"] = int(sys.argv[3])
res = sys.argv[4] if len(sys.argv) > 4 else "lds"
eng = Engine(docs, lib_path=lib, **bench.caps_for(c))
eng.set_residency({"hbm": 0, "lds": 1, "blk": 2, "big": 3}[res])
eng.upload_props(bench.ann_props()); eng.upload_names(['"c%d"' % i for i in range(64)])
p = MtGenParams(7, docs, c["ops"], c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"], c["rewrite"])
eng.generate(p); eng.sync(); eng.generated_to_resident()
eng.open_docs(0, docs); t = time.time(); eng.replay_resident(); eng.sync(); dt = time.time() - t
# header layout: 12 int + 6 u64 + 8 int = 128 bytes, then prof[8]
import ctypes as C
raw = np.zeros((docs, 8), np.uint64)
hdr_size = 192
buf = (C.c_char * (hdr_size * docs))()
# read through mt_dump? use a generic host copy via a tiny helper in the lib: not exported -> use counters API + extra export
fn = eng.lib.mt_prof_get
fn.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
fn(eng.h, docs, raw.ctypes.data)
tot = raw.sum(axis=0).astype(float)
names = ["computeU", "split-walks", "insert-walk", "rangeMap", "zamboni", "op-total", "gen", "textGC"]
if flag == "MT_PROFILE3":
    names = ["zamboni", "scourLeaf", "appendText", "packParent", "pack's scour", "heapGet", "after-scour", "pops(n)"]
if flag == "MT_PROFILE2":
    names = ["walk blkLoad", "walk childLens", "walk levels(n)", "computeU", "computeU(n)", "heapGet", "heapGet(n)", "scourLeaf"]
print(f"{flag} residency={res} ops={c['ops']}")
print(f"{cfg} docs={docs} replay wall {dt*1e3:.1f} ms; per-doc mean cycles per msg:")
for i, n in enumerate(names):
    print(f"  {n:12s} {tot[i]/docs/c['ops']:10.0f} cyc/msg  ({100*tot[i]/max(tot[5],1):5.1f}% of op-total)")
