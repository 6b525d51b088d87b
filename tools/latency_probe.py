"""Diagnostic: cycles per dependent step of the replay kernel (-DMT_PROFILE2 build).

Reads the fine-grained probes (walk block load, walk child lengths, computeU,
heap pop, leaf scour) after one replay of a bench workload at several document
counts (occupancy), to separate memory latency from instruction cost.
"""
import ctypes as C, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fluidframework_amd.engine import Engine
from fluidframework_amd.batch import MtGenParams
import bench

lib = os.path.join(ROOT, "fluidframework_amd", "libmtgpu_prof2.so")
cfg = sys.argv[1] if len(sys.argv) > 1 else "config2"
ops = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
for docs in [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "256,1024,4096").split(",")]:
    c = dict(bench.CONFIGS[cfg]); c["docs"] = docs; c["ops"] = ops
    eng = Engine(docs, lib_path=lib, **bench.caps_for(c))
    eng.upload_props(bench.ann_props()); eng.upload_names(['"c%d"' % i for i in range(64)])
    p = MtGenParams(7, docs, c["ops"], c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"], c["rewrite"])
    eng.generate(p); eng.sync(); eng.generated_to_resident()
    eng.open_docs(0, docs); t = time.time(); eng.replay_resident(); eng.sync(); dt = time.time() - t
    raw = np.zeros((docs, 8), np.uint64)
    fn = eng.lib.mt_prof_get; fn.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    fn(eng.h, docs, raw.ctypes.data)
    t = raw.sum(axis=0).astype(float)
    msgs = docs * ops
    print(f"{cfg} docs={docs} ops={ops}: replay {dt*1e3:.1f} ms = {dt/ops*1e6:.1f} us/msg/doc")
    print(f"  walk level: blkLoad {t[0]/t[2]:.0f} cyc, childLens {t[1]/t[2]:.0f} cyc  ({t[2]/msgs:.2f} levels/msg)")
    print(f"  computeU   {t[3]/t[4]:.0f} cyc/call ({t[4]/msgs:.2f}/msg)")
    print(f"  heapGet    {t[5]/max(t[6],1):.0f} cyc/call ({t[6]/msgs:.2f}/msg); scourLeaf {t[7]/max(t[6],1):.0f} cyc/pop")
    eng.close()
