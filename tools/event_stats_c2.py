"""Diagnostic: per-message event counts of a short-document bench stream (config 2 / 3 shape)
on the host emulation (-DMT_EVCOUNT or EVFLAG=MT_EVCOUNT2), the same generator and seeds as
bench.py on a subset of documents.  Not the product.

usage: EVFLAG=MT_EVCOUNT2 python tools/event_stats_c2.py [config2] [docs=64] [residency=blk]
"""
import ctypes as C, os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from fluidframework_amd.engine import Engine
from fluidframework_amd.batch import MtGenParams
import bench
flag = os.environ.get("EVFLAG", "MT_EVCOUNT")
lib = f"/tmp/libmtemu_{flag.lower()}.so"
subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wno-unknown-pragmas", "-D" + flag,
                       "-o", lib, os.path.join(ROOT, "tests", "emu", "mt_emu.cpp")])
cfg = sys.argv[1] if len(sys.argv) > 1 else "config2"
docs = int(sys.argv[2]) if len(sys.argv) > 2 else 64
res = sys.argv[3] if len(sys.argv) > 3 else "blk"
c = dict(bench.CONFIGS[cfg]); c["docs"] = docs
eng = Engine(docs, lib_path=lib, prefix="emu_", **bench.caps_for(c))
eng.set_residency(bench.RESIDENCY[res])
eng.upload_props(bench.ann_props()); eng.upload_names(['"c%d"' % i for i in range(64)])
p = MtGenParams(7, docs, c["ops"], c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"],
                c["rewrite"])
eng.generate(p); eng.sync(); eng.generated_to_resident(); eng.open_docs(0, docs)
fn = eng.lib.emu_prof_get; fn.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
base = np.zeros((docs, 8), np.uint64); fn(eng.h, docs, base.ctypes.data)
eng.replay_resident(); eng.sync()
raw = np.zeros((docs, 8), np.uint64); fn(eng.h, docs, raw.ctypes.data)
msgs = float(docs * c["ops"]); tot = (raw - base).sum(axis=0).astype(float)
if flag == "MT_EVCOUNT":
    print(f"{cfg} docs={docs} res={res}: computeU/msg {tot[0]/msgs:.2f}  |U|/call {tot[1]/max(tot[0],1):.1f}  "
          f"win/call {tot[2]/max(tot[0],1):.1f}  heapGet/msg {tot[3]/msgs:.3f}  siftLevels/get {tot[4]/max(tot[3],1):.2f}  "
          f"walkLevels/msg {tot[5]/msgs:.2f}  blockSplits/msg {tot[6]/msgs:.3f}  heapN/get {tot[7]/max(tot[3],1):.0f}")
else:
    names = ["packParent", "updatePathLens levels", "copyText units", "copyText calls", "textGC", "splitRow",
             "zamboni pops", "rangeMap leaf blocks"]
    print(f"{cfg} docs={docs} res={res}: " + " ".join(f"{nm}={tot[i]/msgs:.3f}" for i, nm in enumerate(names)))
