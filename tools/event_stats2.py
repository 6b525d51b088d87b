"""Diagnostic: second event set of the engine logic (host emulation, -DMT_EVCOUNT2):
packParent calls, updatePathLens levels, text copies, textGC, row splits, zamboni
pops and rangeMap leaf blocks per message.  Not part of the product."""
import os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import ctypes as C
from fluidframework_amd.engine import Engine
from fluidframework_amd.batch import MtGenParams
import bench

lib = "/tmp/libmtemu_ev2.so"
subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wno-unknown-pragmas", "-D" + os.environ.get("EVFLAG", "MT_EVCOUNT2"),
                       "-o", lib, os.path.join(ROOT, "tests", "emu", "mt_emu.cpp")])
cfg = sys.argv[1] if len(sys.argv) > 1 else "config2"
docs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
c = dict(bench.CONFIGS[cfg]); c["docs"] = docs
if len(sys.argv) > 3: c["ops"] = int(sys.argv[3])
eng = Engine(docs, lib_path=lib, prefix="emu_", **bench.caps_for(c))
eng.upload_props(bench.ann_props()); eng.upload_names(['"c%d"' % i for i in range(64)])
p = MtGenParams(7, docs, c["ops"], c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"], c["rewrite"])
eng.generate(p); eng.sync(); eng.generated_to_resident()
eng.open_docs(0, docs); eng.replay_resident(); eng.sync()
raw = np.zeros((docs, 8), np.uint64)
fn = eng.lib.emu_prof_get; fn.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
fn(eng.h, docs, raw.ctypes.data)
cnt = eng.counters(range(docs))
msgs = float(cnt["msgs"].sum()); tot = raw.sum(axis=0).astype(float)
names = ["packParent", "updatePathLens levels", "copyText units", "copyText calls", "textGC", "splitRow",
         "zamboni pops", "rangeMap leaf blocks"]
print(f"{cfg} docs={docs} msgs/doc={msgs/docs:.0f}")
for i, n in enumerate(names):
    print(f"  {n:24s} {tot[i]/msgs:8.3f} /msg")
