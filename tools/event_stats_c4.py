"""Diagnostic: per-message event counts of config 4's measured stream (host emulation,
-DMT_EVCOUNT or EVFLAG=MT_EVCOUNT2 / MT_BPC_STATS), documents pre-built as bench.py does.  Not the product."""
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
n, pre, ops = 1, int(sys.argv[1]) if len(sys.argv) > 1 else 200000, int(sys.argv[2]) if len(sys.argv) > 2 else 3000
res = sys.argv[3] if len(sys.argv) > 3 else "big"
rows = pre + 3 * ops + 64
eng = Engine(n, lib_path=lib, prefix="emu_", rows_per_doc=rows, blocks_per_doc=rows // 2 + 64, heap_per_doc=rows,
             window_per_doc=16384, text_per_doc=5 * pre + 8 * ops + 4096, propsets_per_doc=pre + ops + 64)
eng.upload_props(bench.ann_props()); eng.upload_names(['"c%d"' % i for i in range(64)])
pa = MtGenParams(1, n, pre, 1, 0, 100, 0, 5, 1, 1, 0); pa.ins_len_min, pa.seg_prop_sets, pa.ins_at_end = 5, 2, 1
eng.generate(pa); eng.sync(); eng.checkpoint()
pb = MtGenParams(2, n, ops, 8, 1024, 60, 40, 8, 8, 2, 0); pb.continue_docs = 1
eng.generate(pb); eng.sync(); eng.generated_to_resident(); eng.restore()
eng.set_residency(bench.RESIDENCY[res])
fn = eng.lib.emu_prof_get; fn.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
base = np.zeros((n, 8), np.uint64); fn(eng.h, n, base.ctypes.data)
c0 = eng.counters(range(n))
eng.replay_resident(); eng.sync()
raw = np.zeros((n, 8), np.uint64); fn(eng.h, n, raw.ctypes.data)
c1 = eng.counters(range(n))
msgs = float(c1["msgs"].sum() - c0["msgs"].sum()); tot = (raw - base).sum(axis=0).astype(float)
if flag == "MT_EVCOUNT":
    print(f"config4 pre={pre} ops={ops} res={res}: computeU/msg {tot[0]/msgs:.2f}  |U|/call {tot[1]/max(tot[0],1):.1f}  "
          f"win/call {tot[2]/max(tot[0],1):.1f}  heapGet/msg {tot[3]/msgs:.3f}  siftLevels/get {tot[4]/max(tot[3],1):.2f}  "
          f"walkLevels/msg {tot[5]/msgs:.2f}  blockSplits/msg {tot[6]/msgs:.3f}  heapN/get {tot[7]/max(tot[3],1):.0f}")
elif flag == "MT_BPC_STATS":
    names = ["lookups", "hits", "miss empty", "miss other", "put evicts", "drops live"]
    print(" ".join(f"{nm}={tot[i]/msgs:.2f}" for i, nm in enumerate(names)))
else:
    names = ["packParent", "updatePathLens levels", "copyText units", "copyText calls", "textGC", "splitRow",
             "zamboni pops", "rangeMap leaf blocks"]
    print(" ".join(f"{nm}={tot[i]/msgs:.3f}" for i, nm in enumerate(names)))
