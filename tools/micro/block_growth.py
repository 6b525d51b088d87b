"""Diagnostic (host emulation, -DMT_EVCOUNT3): the largest number of blocks one message adds
(its op and both zamboni calls) beyond 2 * height, per document, for a bench config.
usage: [LAG=..] [CLIENTS=..] python tools/micro/block_growth.py CONFIG DOCS [SEED] [OPS]"""
import ctypes as C, os, subprocess, sys
import numpy as np
ROOT=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path.insert(0, ROOT)
from fluidframework_amd.engine import Engine
from fluidframework_amd.batch import MtGenParams
import bench
lib="/tmp/libmtemu_ev3.so"
if not os.path.exists(lib):
    subprocess.check_call(["g++","-O2","-std=c++17","-fPIC","-shared","-pthread","-Wno-unknown-pragmas","-DMT_EVCOUNT3","-o",lib,os.path.join(ROOT,"tests","emu","mt_emu.cpp")])
cfg=sys.argv[1]; docs=int(sys.argv[2]); seed=int(sys.argv[3]) if len(sys.argv)>3 else 7
c=dict(bench.CONFIGS[cfg]); c["docs"]=docs
if os.environ.get("LAG"): c["lag"]=int(os.environ["LAG"])
if os.environ.get("CLIENTS"): c["clients"]=int(os.environ["CLIENTS"])
if len(sys.argv)>4: c["ops"]=int(sys.argv[4])
eng=Engine(docs, lib_path=lib, prefix="emu_", **bench.caps_for(c))
eng.set_residency(0)
eng.upload_props(bench.ann_props()); eng.upload_names(['"c%d"' % i for i in range(64)])
p=MtGenParams(seed, docs, c["ops"], c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"], c["rewrite"])
eng.generate(p); eng.sync(); eng.generated_to_resident()
eng.open_docs(0, docs); eng.replay_resident(); eng.sync()
raw=np.zeros((docs,8),np.uint64); fn=eng.lib.emu_prof_get; fn.argtypes=[C.c_void_p,C.c_uint32,C.c_void_p]; fn(eng.h,docs,raw.ctypes.data)
g=raw[:,0].astype(np.int64)-1000000
print(cfg, "docs", docs, "max per-message block growth - 2*height:", g.max(), "p99.9", np.percentile(g,99.9), "hist", np.unique(g, return_counts=True))
