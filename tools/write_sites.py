"""Diagnostic: HBM bytes stored per message, by pool (and per row field), on the host emulation
built with -DMT_WTRACE (tests/emu/mt_emu.cpp): after every message the document's pools are
compared with a shadow copy and each 64-byte line that changed counts once for that message;
the write-back at a run's end (blocks and heap leave LDS, the header) is counted apart.  Same
generator and seeds as bench.py, on a subset of documents.  Not the product.

usage: python tools/write_sites.py [config2|config3|config5] [docs] [residency=blk] [--json OUT]
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from fluidframework_amd.batch import MtGenParams  # noqa: E402
from fluidframework_amd.engine import Engine  # noqa: E402

POOLS = ["rows", "blocks", "heap", "window", "U ids", "U deltas", "U chains", "text", "property maps", "header",
         "recycled rows", "overlap list", "marker ids", "registers", "register rows"]
ROW_FIELDS = ["len", "seq", "removedSeq", "meta", "toff", "props", "parent", "tcap", "ovl lo", "ovl hi", "rcl", "mid"]


def build():
    extra = os.environ.get("WT_FLAGS", "").split()
    lib = "/tmp/libmtemu_wtrace%s.so" % "".join(f.replace("-D", "_").replace("=", "") for f in extra)
    src = os.path.join(ROOT, "tests", "emu", "mt_emu.cpp")
    deps = [src] + [os.path.join(ROOT, "fluidframework_amd", "csrc", f) for f in os.listdir(os.path.join(ROOT, "fluidframework_amd", "csrc"))]
    if not os.path.exists(lib) or any(os.path.getmtime(lib) < os.path.getmtime(d) for d in deps):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wno-unknown-pragmas",
                               "-DMT_WTRACE"] + extra + ["-o", lib, src])
    return lib


def run(cfg="config2", docs=16, res="blk"):
    lib = build()
    c = dict(bench.CONFIGS[cfg])
    c["docs"] = docs
    if cfg == "config5":
        from fluidframework_amd.shard import clients_per_doc, generation_caps, zipf_op_counts
        ops = zipf_op_counts(docs, 20241015)
        cl = clients_per_doc(docs, 20241015)
        eng = Engine(docs, lib_path=lib, prefix="emu_", per_doc=generation_caps(ops, c["ins_len"]))
        p = MtGenParams(20241015, docs, 0, 2, c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"],
                        c["rewrite"])
        gen = lambda: eng.generate(p, ops_per_doc=ops, clients_per_doc=cl)
    else:
        eng = Engine(docs, lib_path=lib, prefix="emu_", **bench.caps_for(c))
        p = MtGenParams(20241015, docs, c["ops"], c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"],
                        c["ann_sets"], c["rewrite"])
        gen = lambda: eng.generate(p)
    eng.set_residency(bench.RESIDENCY[res])
    eng.upload_props(bench.ann_props())
    eng.upload_names(['"c%d"' % i for i in range(64)])
    gen()
    eng.sync()
    cnt = eng.counters(range(docs))
    eng.generated_to_resident()
    eng.open_docs(0, docs)
    wt = eng.lib.emu_wtrace
    wt.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    n = wt(eng.h, 1, None)
    eng.replay_resident()
    eng.sync()
    out = np.zeros(2 * n + 13, np.uint64)
    wt(eng.h, 0, out.ctypes.data)
    # the traced replay (free pools poisoned) must give the digests of a plain replay of the stream
    neg = np.full(docs, -1, np.int32)
    traced = eng.snapshot_digests(range(docs), neg, neg, threads=4)
    eng.open_docs(0, docs)
    eng.replay_resident()
    eng.sync()
    plain = eng.snapshot_digests(range(docs), neg, neg, threads=4)
    if not np.array_equal(traced, plain) or eng.status(range(docs)).any():
        raise SystemExit("traced replay differs from the plain one")
    msgs = float(out[2 * n + 12])
    per = out[:n].astype(float) * 64 / msgs
    end = out[n:2 * n].astype(float) * 64 / msgs
    fields = out[2 * n:2 * n + 12].astype(float) / msgs
    # §8(d): the rows' written part of 32 (R_r + R_w), and the inserted text (4 L_ins covers read + write)
    alg = bench.algorithmic_bytes(cnt) / msgs
    rep = {"config": cfg, "docs": docs, "residency": res, "messages": int(msgs),
           "bytes_per_msg": {POOLS[k]: round(per[k], 1) for k in range(n) if per[k] > 0},
           "bytes_per_msg_at_run_end": {POOLS[k]: round(end[k], 1) for k in range(n) if end[k] > 0},
           "row_dwords_changed_per_msg": {ROW_FIELDS[k]: round(fields[k], 2) for k in range(12)},
           "total_bytes_per_msg": round(per.sum() + end.sum(), 1),
           "algorithmic_bytes_per_msg_read_and_write": round(alg, 1)}
    eng.close()
    return rep


if __name__ == "__main__":
    a = [x for i, x in enumerate(sys.argv[1:], 1) if not x.startswith("--") and sys.argv[i - 1] != "--json"]
    rep = run(a[0] if a else "config2", int(a[1]) if len(a) > 1 else 16, a[2] if len(a) > 2 else "blk")
    print(json.dumps(rep, indent=1))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(rep, f, indent=1)
    sys.stdout.flush()
    os._exit(0)          # (the traced host-emulation build crashes in interpreter teardown; results are out)
