#!/usr/bin/env python
"""bench.py — sequenced merge-tree ops applied/sec on MI355X (BASELINE.json metric).

A "step" is one replay of the whole synthetic batch on freshly opened documents:
every document's sequenced messages are applied through the HIP engine
(Client.applyMsg semantics, packages/dds/merge-tree/src/client.ts:819) with the
op arrays already resident in HBM.  Streams are produced on the device by the
engine acting as sequencer + observer (SURVEY.md §8(d) rules), before timing.

Default workload (N=1): BASELINE.json configs[1] — 4,096 documents x 8 clients x
10,000 messages, refSeq lag U[0,32], 60/40 insert/remove (insert length U[1,8],
remove length U[1,8]).  Multi-GPU (torchrun): documents shard across ranks with
no data-path collective (weak scaling); timing = max over ranks.

JSON fields beyond the driver contract:
  roofline      algorithmic HBM bytes per launch (SURVEY.md §8(d) B_op formula,
                from the engine's per-document counters) / average replay-kernel
                time measured with HIP events on the engine's stream;
  cpu_baseline  the oracle (C++ restatement of the reference algorithm, "port")
                replaying a bounded sample of the same streams on host threads.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0
PARITY_DOCS = 8            # documents per rank the oracle replays for the N > 1 parity check
RESIDENCY = {"hbm": 0, "lds": 1, "blk": 2, "big": 3}
REPLAY_KERNEL = {"hbm": "mt_replay_kernel", "lds": "mt_replay_lds_kernel + mt_replay_kernel",
                 "blk": "mt_replay_blk_kernel", "big": "mt_replay_big_kernel"}  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md

CONFIGS = {
    # name: (docs, ops, clients, lag, ins%, rem%, ins_len, rem_len, ann_sets, rewrite%)
    "config2": dict(docs=4096, ops=10000, clients=8, lag=32, ins=60, rem=40, ins_len=8, rem_len=8, ann_sets=1, rewrite=0,
                    desc="4096 docs x 8 clients x 10k msgs, lag U[0,32], 60/40 ins/rem"),
    "config3": dict(docs=16384, ops=4000, clients=8, lag=4, ins=30, rem=30, ins_len=8, rem_len=16, ann_sets=24, rewrite=5,
                    desc="16384 docs x 8 clients x 4k msgs, lag U[0,4], 30/30/40 ins/rem/annotate, zamboni-heavy"),
    "config1": dict(docs=1, ops=10000, clients=2, lag=8, ins=55, rem=45, ins_len=8, rem_len=16, ann_sets=1, rewrite=0,
                    desc="1 doc x 2 clients x 10k msgs (reference plumbing case)"),
    # 256 long docs pre-built (untimed) by 200k 5-char appends with alternating segment props
    # (200k segments, 1M chars), then 50k measured ops with lag U[0,1024] (window ~1k)
    "config4": dict(docs=256, ops=50000, clients=8, lag=1024, ins=60, rem=40, ins_len=8, rem_len=8, ann_sets=2,
                    rewrite=0, prebuild=200000,
                    desc="256 long docs (pre-built to 200k segments / 1M chars) x 50k msgs, 8 clients, lag U[0,1024]"),
    # docs = per GPU (weak scaling; 8 GPUs = 1,048,576 docs); ops ~ Zipf(1.5) on [8, 65536], clients U[2,16]
    "config5": dict(docs=131072, ops=0, clients=0, lag=32, ins=60, rem=40, ins_len=8, rem_len=8, ann_sets=1, rewrite=0,
                    desc="Zipf(1.5)-sized docs (8..65536 msgs, clients U[2,16]), 131072 docs per GPU, rank-0 ingest, "
                         "LPT rebalance + digest gather over RCCL"),
}


class Host:
    """Where a bench run executes: the product (libmtgpu.so on the rank's GPU, RCCL for
    config 5's exchange) unless a test driver substitutes the engine factory and the
    backend (tests/bench_emu_driver.py runs the same code paths on the host emulation
    with gloo to cover the multi-rank logic on CPU; its output is never a measurement)."""
    factory = None          # (n_docs, device, **caps) -> Engine
    backend = "nccl"        # config 5's collectives
    device_type = "cuda"

    @classmethod
    def engine(cls, n, device, **kw):
        if cls.factory is not None:
            return cls.factory(n, device=device, **kw)
        from fluidframework_amd.engine import Engine
        return Engine(n, device=device, **kw)


def launch(n, argv, script=None):
    """`--gpus N` outside a torchrun environment: start N ranks, one process per GPU, with
    torch.distributed.run on 127.0.0.1 (before anything here touches a GPU) and return
    its exit code.  Every rank re-enters main() with RANK/LOCAL_RANK/WORLD_SIZE set."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(script or sys.argv[0])] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def ann_props():
    from fluidframework_amd.batch import PropTable
    pt = PropTable()
    vals = ["s0", "s1", "s2", "s3", 1, 2, None]
    rng = np.random.RandomState(5)
    for _ in range(24):
        keys = rng.choice(8, size=rng.randint(1, 4), replace=False)
        pt.intern({f"k{k}": vals[rng.randint(0, len(vals))] for k in sorted(keys)})
    return pt


def algorithmic_bytes(cnt):
    # B_op = 32 + 4 L_ins + 32 (R_r + R_w) + 64 D + 64 Z, summed over messages
    return int(32 * cnt["msgs"].sum() + 4 * cnt["ins_units"].sum() + 32 * cnt["rows_rw"].sum()
               + 64 * cnt["depth"].sum() + 64 * cnt["scoured"].sum())


def measured_traffic(cfg_name, c, kernel):
    """HBM bytes per replay launch from the committed rocprofv3 PMC passes
    (profiles/<round>/<config>_traffic.json, written by tools/traffic_from_pmc.py)
    when they were taken on this exact workload; None otherwise."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"{cfg_name}_traffic.json"))):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        if t.get("docs") == c["docs"] and t.get("msgs_per_doc") == c["ops"] and t.get("kernel") == kernel:
            best = (t["traffic_bytes"], os.path.relpath(f, ROOT))
    return best


def reserve_staging(eng):
    """Pin the snapshot staging buffers once, before the timed region (a serving process does
    this at startup); returns the milliseconds it took, reported beside the snapshot time."""
    if not eng.fn.get("reserve_staging"):
        return None
    t = time.perf_counter()
    eng.reserve_staging()
    return (time.perf_counter() - t) * 1e3


def partition_of(args, c):
    """(min_ops, cus) of --partition MIN:CUS, "auto" (the default: mt_plan_partition's rule
    applied by the library to each resident batch), None when off."""
    spec = args.partition if args.partition else c.get("partition", "auto")
    if not spec or spec == "off":
        return None
    if spec == "auto":
        return "auto"
    a, b = spec.split(":")
    return int(a), int(b)


def apply_partition(eng, args, c):
    part = partition_of(args, c)
    if args.residency == "blk" and part:
        eng.set_partition(*((part,) if part == "auto" else part))
    return part


def partition_report(eng, args, part):
    """The partition a run used: {"min_msgs", "cus", "rule"} (rule "auto" when the library
    chose it), None for none."""
    if args.residency != "blk" or not part:
        return None
    got = eng.partition_info() if eng.fn.get("last_partition") else None
    if got is None:
        return {"min_msgs": 0, "cus": 0, "rule": "auto: none"} if part == "auto" else None
    got["rule"] = "auto" if part == "auto" else "fixed"
    return got


def caps_for(c):
    ops = c["ops"]
    return dict(rows_per_doc=3 * ops + 64, blocks_per_doc=ops + 64, heap_per_doc=2 * ops + 64,
                window_per_doc=max(2048, 64 * c["lag"] + 1024), text_per_doc=ops * c["ins_len"] + 4096,
                propsets_per_doc=(2 * ops + 64) if c["ins"] + c["rem"] < 100 else 64)


def oracle_run(eng, c, params_cls, seed, n_docs, threads, ops_fn=None):
    """The first n_docs streams of the workload (regenerated by the engine: generation is
    deterministic per document) replayed by the oracle on `threads` host threads:
    (seconds, messages, SnapshotV1 digests, status words)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes
    from oracle_lib import lib as oracle
    L = oracle()
    p = params_cls(seed, n_docs, c["ops"], c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"],
                   c["rem_len"], c["ann_sets"], c["rewrite"])
    if ops_fn is None:
        eng.generate(p)
    else:
        o, k = ops_fn(n_docs)
        eng.generate(p, ops_per_doc=o, clients_per_doc=k)
    eng.sync()
    b = eng.generated_download()
    st = np.zeros(n_docs, np.uint32)
    dg = np.zeros(n_docs, np.uint64)
    oc = np.zeros((n_docs, 6), np.uint64)
    secs = L.ora_replay_batch(ctypes.byref(b.to_c()), ctypes.byref(eng.props.to_c()), threads, dg.ctypes.data,
                              st.ctypes.data, oc.ctypes.data)
    oracle_run.counters = oc              # the sample's §8(d) counters by the oracle's own count
    return secs, int(b.op_offsets[-1]), dg, st


def rank_parity(dist, bad_local, checked_local):
    """Digest parity over every rank (N > 1): each rank checked its own sample against the
    oracle; the counts are summed (gloo / RCCL all_reduce) for rank 0's line."""
    import torch
    t = torch.tensor([bad_local, checked_local], dtype=torch.int64)
    if dist is not None:
        torch_, tdist = dist
        tdist.all_reduce(t)
    return int(t[0]), int(t[1])


def parity_text(bad, checked, world, what="SnapshotV1 digests"):
    if bad == 0:
        return f"{what} == oracle on {checked} docs ({world} rank{'s' if world > 1 else ''}, each its own sample)"
    return f"DIGEST MISMATCH: {bad} of {checked} sample docs differ from the oracle"


def cpu_baseline(eng, c, params_cls, seed, target_s, threads, ops_fn=None):
    """Oracle ('port' of the reference algorithm) on a bounded sample of the same streams.
    ops_fn(n) -> (ops_per_doc, clients_per_doc) for skewed workloads (config 5)."""
    def run(n_docs):
        return oracle_run(eng, c, params_cls, seed, n_docs, threads, ops_fn)

    pilot_docs = min(c["docs"], max(threads, 16))
    t, n, dg, st = run(pilot_docs)
    docs = pilot_docs
    if t < target_s * 0.5:
        docs = int(min(c["docs"], max(pilot_docs, pilot_docs * target_s / max(t, 1e-3))))
        if docs > pilot_docs:
            t, n, dg, st = run(docs)
    out = {"value": n / t, "unit": "ops/s", "cores": threads, "kind": "port",
           "sample": f"{docs} docs ({n} msgs) of the same workload, oracle (C++ restatement of "
                     f"MT/mergeTree.ts + partialLengths.ts) on {threads} host threads, {t:.1f} s"}
    return out, dg, st


COUNTER_KEYS = ("ops", "msgs", "ins_units", "rows_rw", "depth", "scoured")


def counters_match(cnt, k):
    """The engine's per-document counters (the roofline numerator) equal the oracle's count
    of the same §8(d) quantities on the last oracle_run sample's first k documents."""
    oc = getattr(oracle_run, "counters", None)
    if oc is None or len(oc) < k:
        return False
    eng = np.stack([np.asarray(cnt[key][:k], np.uint64) for key in COUNTER_KEYS], axis=1)
    return bool(np.array_equal(eng, oc[:k]))


def digest_parity(gpu_digests, oracle_digests, oracle_status):
    """The bench line's parity field: SnapshotV1 digests of the timed replay's documents
    against the oracle's replay of the same streams (the cpu_baseline sample)."""
    k = len(oracle_digests)
    same = int((np.asarray(gpu_digests[:k], np.uint64) == oracle_digests).sum())
    if same == k and not np.asarray(oracle_status).any():
        return f"SnapshotV1 digests == oracle on {k} docs (cpu_baseline sample) + status words clean"
    return f"DIGEST MISMATCH: {k - same} of {k} sample docs differ from the oracle"


def manifest_parity(name, digs, **shape):
    """Every document's SnapshotV1 digest against the oracle-made manifest of this workload
    (tests/golden/digests, tools/make_digest_manifest.py) when one exists for this seed and
    shape: {"checked", "of", "mismatches", "manifest"} or None.  Roll-up manifests (the
    1,048,576-document run) compare xxh64 roll-ups of each 1,024 consecutive documents."""
    d = os.path.join(ROOT, "tests", "golden", "digests")
    try:
        ent = json.load(open(os.path.join(d, "index.json")))[name]
    except (OSError, ValueError, KeyError):
        return None
    if any(ent.get(k) != v for k, v in shape.items()):
        return None
    want = np.fromfile(os.path.join(d, ent["file"]), dtype="<u8")
    got = np.asarray(digs, np.uint64)
    if ent["file"].endswith(".roll.u64"):
        import xxhash
        k = int(ent["kind"].split()[3]) if "roll-ups" in ent["kind"] else 1024
        if len(got) != ent["docs"]:
            return None
        roll = np.array([xxhash.xxh64(got[i:i + k].astype("<u8").tobytes(), seed=0).intdigest()
                         for i in range(0, len(got), k)], np.uint64)
        bad_groups = np.nonzero(roll != want)[0]
        bad = int(sum(min(k, len(got) - g * k) for g in bad_groups))
        return {"checked": len(got), "of": ent["docs"], "mismatches": bad,
                "mismatch_groups": [int(g) for g in bad_groups[:16]], "manifest": f"tests/golden/digests/{ent['file']}"}
    if len(got) != len(want):
        return None
    bad = int((got != want).sum())
    return {"checked": len(got), "of": len(want), "mismatches": bad,
            "first_mismatch": int(np.nonzero(got != want)[0][0]) if bad else None,
            "manifest": f"tests/golden/digests/{ent['file']}"}


def manifest_text(m):
    if m is None:
        return ""
    if m["mismatches"] == 0:
        return f"; every document's SnapshotV1 digest == the oracle's manifest: {m['checked']} of {m['of']}"
    return f"; MANIFEST MISMATCH: {m['mismatches']} of {m['of']} documents differ from the oracle's manifest"


def run_config4(args, c, world, rank, local):
    """Config 4: long documents.  Untimed: pre-build every document by
    c['prebuild'] appends (5 chars, segment props alternating between two sets,
    so nothing coalesces), checkpoint that state, generate the measured stream
    on top of it.  A step = restore the pre-built documents (device copy) +
    replay the measured stream."""
    from fluidframework_amd.batch import MtGenParams
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        tdist.init_process_group("gloo")  # rank coordination only: replicas, no data-path collective
        dist = (torch, tdist)
    n, pre, ops = c["docs"], c["prebuild"], c["ops"]
    rows = pre + 3 * ops + 64
    eng = Host.engine(n, local, rows_per_doc=rows, blocks_per_doc=rows // 2 + 64, heap_per_doc=rows,
                 window_per_doc=16384, text_per_doc=5 * pre + c["ins_len"] * ops + 4096,
                 propsets_per_doc=pre + ops + 64)
    set_residency(eng, args)
    stage_ms = reserve_staging(eng)
    eng.upload_props(ann_props())
    eng.upload_names(['"c%d"' % i for i in range(64)])
    seed = args.seed ^ (rank * 0x9E3779B1)
    t0 = time.time()
    pa = MtGenParams(seed, n, pre, 1, 0, 100, 0, 5, 1, 1, 0)
    pa.ins_len_min, pa.seg_prop_sets, pa.ins_at_end = 5, 2, 1
    eng.generate(pa)
    eng.sync()
    if eng.status(range(n)).any():
        raise SystemExit(f"prebuild failed: {np.unique(eng.status(range(n)))}")
    cnt_a = eng.counters(range(n))
    eng.checkpoint()
    pb = MtGenParams(seed ^ 0xB, n, ops, c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"],
                     c["ann_sets"], c["rewrite"])
    pb.continue_docs = 1
    eng.generate(pb)
    eng.sync()
    if eng.status(range(n)).any():
        raise SystemExit(f"stream generation failed: {np.unique(eng.status(range(n)))}")
    cnt_b = eng.counters(range(n))
    pools = eng.pools(range(n))
    gen_s = time.time() - t0
    diff = {k: cnt_b[k] - cnt_a[k] for k in cnt_b}
    msgs = int(diff["msgs"].sum())
    bytes_per_launch = algorithmic_bytes(diff)
    eng.generated_to_resident()

    def step():
        eng.restore()
        eng.replay_resident()

    for _ in range(args.warmup):
        step()
    eng.sync()
    if dist:
        dist[1].barrier()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.steps):
        step()
        eng.sync()
        kms.append(eng.last_replay_ms())
    eng.sync()
    if dist:
        dist[1].barrier()
    dt = time.perf_counter() - t0
    if dist:
        torch, tdist = dist
        t = torch.tensor([dt], dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t.item())
    st = eng.status(range(n))
    cnt = eng.counters(range(n))
    ok = (not st.any()) and int((cnt["msgs"] - cnt_a["msgs"]).sum()) == msgs
    neg = np.full(n, -1, np.int32)
    t1 = time.perf_counter()
    digs = eng.snapshot_digests(range(n), neg, neg, threads=min(16, os.cpu_count() or 1))
    snap_ms = (time.perf_counter() - t1) * 1e3
    if world > 1:
        # every rank checks its own first documents against the oracle (untimed)
        k = min(2, n)
        _, odg, ost = cpu_baseline_config4(eng, c, pa, pb, max(1, min(16, (os.cpu_count() or 1) // world)), docs=k)
        bad_l = int((np.asarray(digs[:k], np.uint64) != odg).sum()) + int(np.asarray(ost).any()) + int(not ok)
        par_bad, par_checked = rank_parity(dist, bad_l, k)
    if rank != 0:
        return
    kern_s = float(np.mean(kms)) / 1e3
    achieved = bytes_per_launch / kern_s / 1e9 if kern_s > 0 else 0.0
    traffic = measured_traffic("config4", {"docs": n, "ops": ops}, REPLAY_KERNEL[args.residency])
    out = {
        "metric": "sequenced merge-tree ops applied/sec (whole node) + achieved HBM GB/s",
        "value": msgs * world * args.steps / dt, "unit": "ops/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int32",
        "data": "synthetic (device-generated: pre-built documents + sequenced op stream, SURVEY.md §8(d) config-4 rules)",
        "config": {"workload": f"config4: {c['desc']}", "docs_per_gpu": n, "msgs_per_doc": ops, "prebuild_appends": pre,
                   "clients": c["clients"], "lag_max": c["lag"], "tree_height_max": int(pools[:, 6].max()),
                   "rows_per_doc_max": int(pools[:, 0].max()), "window_max": int(pools[:, 9].max()),
                   "parallelism": f"doc-sharded x{world}", "residency": args.residency,
                   "step": "mt_restore (device copy of the pre-built documents) + replay"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic[0] if traffic else None,
                     "traffic_source": traffic[1] if traffic else None, "kernel": REPLAY_KERNEL[args.residency],
                     "kernel_ms": kern_s * 1e3, "bytes_per_launch": bytes_per_launch},
        "parity": "status words clean" if ok else "STATUS ERROR",
        "snapshot": {"docs": n, "ms": snap_ms, "digest_xor": f"{int(np.bitwise_xor.reduce(digs)):016x}",
                     "staging_reserve_ms": stage_ms},
        "gen_seconds": gen_s,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], odg, ost = cpu_baseline_config4(eng, c, pa, pb, min(16, os.cpu_count() or 1),
                                                             docs=min(n, args.parity_docs))
        if ok:
            out["parity"] = digest_parity(digs, odg, ost)
    elif world > 1 and ok:
        out["parity"] = parity_text(par_bad, par_checked, world)
    man = manifest_parity("config4", digs, seed=args.seed, docs=n, msgs_per_doc=ops, prebuild=pre) if ok else None
    if man is not None:
        out["parity_manifest"] = man
        out["parity"] += manifest_text(man)
    print(json.dumps(out), flush=True)


def cpu_baseline_config4(eng, c, pa, pb, threads, docs=0):
    """Oracle ('port') on one pre-built document per host thread (or `docs`): time(prebuild +
    stream) - time(prebuild), i.e. the measured stream alone, in ops/s."""
    import ctypes
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fluidframework_amd.batch import MtGenParams
    from oracle_lib import lib as oracle
    L = oracle()
    props = eng.props
    k = docs or threads
    sa = MtGenParams(*(getattr(pa, f) for f, _ in MtGenParams._fields_))
    sa.n_docs = k
    sb = MtGenParams(*(getattr(pb, f) for f, _ in MtGenParams._fields_))
    sb.n_docs = k
    eng.generate(sa)
    eng.sync()
    a = eng.generated_download()
    eng.generate(sb)
    eng.sync()
    b = eng.generated_download()
    from fluidframework_amd.batch import concat_runs
    both = concat_runs(a, b)
    st = np.zeros(k, np.uint32)
    dg = np.zeros(k, np.uint64)
    t_a = L.ora_replay_batch(ctypes.byref(a.to_c()), ctypes.byref(props.to_c()), threads, None, st.ctypes.data, None)
    t_ab = L.ora_replay_batch(ctypes.byref(both.to_c()), ctypes.byref(props.to_c()), threads, dg.ctypes.data,
                              st.ctypes.data, None)
    n_b = int(b.op_offsets[-1])
    dt = max(t_ab - t_a, 1e-6)
    return {"value": n_b / dt, "unit": "ops/s", "cores": threads, "kind": "port",
            "sample": f"{k} pre-built docs ({int(a.op_offsets[-1])} prebuild + {n_b} measured msgs), oracle (C++ "
                      f"restatement of MT/mergeTree.ts + partialLengths.ts) on {threads} host threads; "
                      f"measured-stream time = {t_ab:.1f} s - {t_a:.1f} s"}, dg, st


def run_config5(args, c, world, rank, local):
    """Config 5: Zipf-sized documents ingested on rank 0, LPT-rebalanced across the
    ranks over RCCL (one all_to_all_single of op records + payloads), replayed per
    rank, SnapshotV1 digests gathered to rank 0 (fluidframework_amd/shard.py)."""
    import torch
    from fluidframework_amd.batch import MtGenParams
    from fluidframework_amd.shard import SoloDist, build_sharded
    device = torch.device(Host.device_type, local) if Host.device_type == "cuda" else torch.device("cpu")
    if world > 1:
        import torch.distributed as tdist
        if device.type == "cuda":
            torch.cuda.set_device(local)
            tdist.init_process_group(Host.backend, device_id=device)
        else:
            tdist.init_process_group(Host.backend)
        dist = tdist
    else:
        dist = SoloDist()
    total_docs = c["docs"] * world
    gen_kw = dict(lag_max=c["lag"], pct_insert=c["ins"], pct_remove=c["rem"], ins_len_max=c["ins_len"],
                  rem_len_max=c["rem_len"], n_ann_sets=c["ann_sets"], pct_rewrite=c["rewrite"])
    names = ['"c%d"' % i for i in range(64)]
    fac = lambda n, caps: Host.engine(n, local, per_doc=caps)
    t0 = time.time()
    sh = build_sharded(dist, device, fac, total_docs, args.seed, MtGenParams, gen_kw, names=names)
    setup_s = time.time() - t0
    eng = sh.engine
    stage_ms = reserve_staging(eng)
    # corrupt exchange rows on any rank: every rank stops before replaying (no value published)
    xb = torch.tensor([int(sh.timings.get("exchange_bad_docs", 0))], dtype=torch.int64, device=device)
    if world > 1:
        dist.all_reduce(xb)
    if int(xb.item()):
        raise SystemExit(f"config5: {int(xb.item())} documents failed the exchange checksum; nothing replayed")
    set_residency(eng, args)
    big = c.get("big_min_ops", 0) if args.big_min_ops < 0 else args.big_min_ops
    if args.residency == "blk" and big:
        eng.set_size_class(big)
    part = apply_partition(eng, args, c)
    if args.cont_min >= 0:
        eng.set_continuation(args.cont_min)
    my_msgs = int(sh.ops.sum())
    for _ in range(args.warmup):
        sh.replay()
    eng.sync()
    dist.barrier()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.steps):
        sh.replay()
        eng.sync()
        kms.append(eng.last_replay_ms())
    eng.sync()
    dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    st = eng.status(range(sh.n_docs))
    cnt = eng.counters(range(sh.n_docs))
    bytes_per_launch = algorithmic_bytes(cnt)
    digs = sh.gather_digests(dist, device, threads=min(16, os.cpu_count() or 1))
    xbad = int(sh.timings.get("exchange_bad_docs", 0))
    bad = torch.tensor([int(st.any()) + int(int(cnt["msgs"].sum()) != my_msgs), xbad, sh.n_docs],
                       dtype=torch.int64, device=device)
    if world > 1:
        dist.all_reduce(bad)
        # every rank checks a sample of its own documents against the oracle (untimed)
        pb_, pc_ = config5_rank_parity(args, c, sh) if not args.no_cpu_baseline else (0, 0)
        par = torch.tensor([pb_, pc_], dtype=torch.int64, device=device)
        dist.all_reduce(par)
    if rank != 0:
        return
    total_msgs = int(sh.all_ops.sum())
    kern_s = float(np.mean(kms)) / 1e3
    achieved = bytes_per_launch / kern_s / 1e9 if kern_s > 0 else 0.0
    # the PMC passes run at N = 1 (rank 0 replays every document): per launch of that workload
    # the replay launch's kernels: partitioned size classes run the wide kernel beside the block one
    part_used = partition_report(eng, args, part)
    kname = ("mt_replay_blkw_kernel+mt_replay_blk_kernel" if part_used and part_used["cus"]
             else REPLAY_KERNEL[args.residency])
    traffic = measured_traffic("config5", {"docs": c["docs"], "ops": 0}, kname) if world == 1 else None
    out = {
        "metric": "sequenced merge-tree ops applied/sec (whole node) + achieved HBM GB/s",
        "value": total_msgs * args.steps / dt, "unit": "ops/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int32",
        "data": "synthetic (device-generated sequenced op streams, SURVEY.md §8(d) config-5 rules)",
        "config": {"workload": f"config5: {c['desc']}".replace("131072 docs per GPU", f"{c['docs']} docs per GPU"),
                   "docs_per_gpu": c["docs"], "docs_total": total_docs,
                   "msgs_total": total_msgs, "msgs_mean": total_msgs / total_docs,
                   "msgs_max": int(sh.all_ops.max()), "parallelism": f"doc-sharded x{world} (LPT)",
                   "residency": args.residency, "big_min_ops": big if args.residency == "blk" else None,
                   "partition": part_used},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic[0] if traffic else None,
                     "traffic_source": traffic[1] if traffic else None, "kernel": kname + " (rank 0)",
                     "kernel_ms": kern_s * 1e3, "bytes_per_launch": bytes_per_launch},
        "parity": "status words clean on every rank" if int(bad[0].item()) == 0 else "STATUS ERROR",
        "exchange": {"docs_checked": int(bad[2].item()), "checksum_mismatch_docs": int(bad[1].item()),
                     "note": "per-document 64-bit checksums of the exchanged rows: packed by rank 0, verified on "
                             "arrival by the owning rank (mt_generated_pack_rows / mt_upload_rows_dev)"},
        "memory": {"engine_pools_gb": eng.pool_bytes() / 1e9,
                   "exchange_buffers_peak_gb": (torch.cuda.max_memory_allocated(device) / 1e9) if device.type == "cuda" else None},
        "snapshot": {"docs": sh.n_docs, "ms": sh.timings.get("snapshot_ms"), "host_threads": min(16, os.cpu_count() or 1),
                     "staging_reserve_ms": stage_ms,
                     "note": "rank 0's mt_snapshot_digests (staged download + SnapshotV1 JSON + xxh64), before the gather"},
        "sharding": {"rebalance_ms": sh.timings.get("rebalance_ms"), "rebalance_bytes": sh.timings.get("rebalance_bytes"),
                     "digest_gather_ms": sh.timings.get("digest_ms"), "ingest_generate_s": sh.timings.get("generate_s"),
                     "setup_s": setup_s, "digest_xor": f"{int(np.bitwise_xor.reduce(digs)):016x}",
                     "docs_per_rank_max": int(np.bincount(sh.owner).max())},
    }
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline_config5(args, c, local)
        if int(bad[0].item()) == 0:
            out["parity"] = config5_parity(args, c, sh, digs)
    elif world > 1 and int(bad[0].item()) == 0 and not args.no_cpu_baseline:
        out["parity"] = parity_text(int(par[0].item()), int(par[1].item()), world) + ", all ranks clean"
    if int(bad[0].item()) == 0:
        name = "config5_1m" if total_docs == 1048576 else "config5"
        man = manifest_parity(name, digs, seed=args.seed, docs=total_docs, msgs_total=total_msgs)
        if man is not None:
            out["parity_manifest"] = man
            out["parity"] += manifest_text(man)
    if int(bad[1].item()):
        out["parity"] = f"EXCHANGE CHECKSUM MISMATCH on {int(bad[1].item())} docs; " + out["parity"]
    print(json.dumps(out), flush=True)


def run_config5_shares(args, c, local):
    """Config 5's N-rank LPT plan for c['docs'] x N documents, every rank's share replayed in turn
    on this one GPU (review item: the eight shares of north_star's 1,048,576-document plan on
    hardware without an 8-GPU node).  Each share is timed as bench's config-5 step is (warmup, then
    `steps` replays bracketed by syncs); the node step is the slowest share's.  The SnapshotV1
    digests of every share land in global document order and are checked against the manifest."""
    import torch
    from fluidframework_amd.batch import MtGenParams
    from fluidframework_amd.shard import rank_shares
    device = torch.device(Host.device_type, local) if Host.device_type == "cuda" else torch.device("cpu")
    world = args.shares
    total_docs = c["docs"] * world
    gen_kw = dict(lag_max=c["lag"], pct_insert=c["ins"], pct_remove=c["rem"], ins_len_max=c["ins_len"],
                  rem_len_max=c["rem_len"], n_ann_sets=c["ann_sets"], pct_rewrite=c["rewrite"])
    names = ['"c%d"' % i for i in range(64)]
    fac = lambda n, caps: Host.engine(n, local, per_doc=caps)
    digs = np.zeros(total_docs, np.uint64)
    shares, msgs_all, bad = [], 0, 0
    t_setup = time.time()
    for r, sh in rank_shares(device, fac, total_docs, world, args.seed, MtGenParams, gen_kw, names=names):
        eng = sh.engine
        if r == 0:
            gen_s = time.time() - t_setup
        if int(sh.timings.get("exchange_bad_docs", 0)):
            raise SystemExit(f"share {r}: {sh.timings['exchange_bad_docs']} documents failed the exchange checksum")
        set_residency(eng, args)
        part = apply_partition(eng, args, c)
        my_msgs = int(sh.ops.sum())
        msgs_all += my_msgs
        for _ in range(args.warmup):
            sh.replay()
        eng.sync()
        t0 = time.perf_counter()
        kms = []
        for _ in range(args.steps):
            sh.replay()
            eng.sync()
            kms.append(eng.last_replay_ms())
        eng.sync()
        dt = (time.perf_counter() - t0) / args.steps
        st = eng.status(range(sh.n_docs))
        cnt = eng.counters(range(sh.n_docs))
        ok = (not st.any()) and int(cnt["msgs"].sum()) == my_msgs
        bad += int(not ok)
        neg = np.full(sh.n_docs, -1, np.int32)
        digs[sh.owned] = eng.snapshot_digests(range(sh.n_docs), neg, neg, threads=min(16, os.cpu_count() or 1))
        shares.append({"rank": r, "docs": sh.n_docs, "msgs": my_msgs, "msgs_max": int(sh.ops.max()),
                       "ms_per_step": dt * 1e3, "kernel_ms": float(np.mean(kms)),
                       "exchange_bytes": sh.timings.get("rebalance_bytes"),
                       "partition": partition_report(eng, args, part),
                       "status_clean": ok})
        print(f"share {r}: {sh.n_docs} docs, {my_msgs} msgs, {dt * 1e3:.1f} ms/step", file=sys.stderr, flush=True)
    step_max = max(s_["ms_per_step"] for s_ in shares)
    out = {
        "metric": "sequenced merge-tree ops applied/sec (whole node) + achieved HBM GB/s",
        "value": msgs_all / (step_max / 1e3), "unit": "ops/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": step_max, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int32",
        "data": "synthetic (device-generated sequenced op streams, SURVEY.md §8(d) config-5 rules)",
        "kind": f"projection: the {world} ranks' LPT shares replayed one after another on one GPU; value = all "
                f"shares' messages / the slowest share's step (what an {world}-GPU node's step would be with no "
                f"exchange inside the timed region)",
        "config": {"workload": f"config5 at {total_docs} documents, N = {world} LPT plan", "docs_total": total_docs,
                   "msgs_total": msgs_all, "residency": args.residency},
        "shares": shares,
        "parity": "status words clean on every share" if bad == 0 else f"STATUS ERROR on {bad} shares",
        "setup_s": gen_s, "digest_xor": f"{int(np.bitwise_xor.reduce(digs)):016x}",
    }
    if bad == 0:
        name = "config5_1m" if total_docs == 1048576 else "config5"
        man = manifest_parity(name, digs, seed=args.seed, docs=total_docs, msgs_total=msgs_all)
        if man is not None:
            out["parity_manifest"] = man
            out["parity"] += manifest_text(man)
    print(json.dumps(out), flush=True)


def config5_parity(args, c, sh, digs):
    """Oracle replay (its own generator, same seeds and per-document counts, documents
    generated on host threads) of the smallest-id documents (--parity-docs, default 4096),
    against the digests gathered to rank 0 (checker only)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fluidframework_amd.batch import MtGenParams
    from oracle_lib import generate
    k = min(args.parity_docs or 4096, len(sh.all_ops))
    p = MtGenParams(args.seed, k, 0, 2, c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"],
                    c["rewrite"])
    cl = sh.clients_all[:k] if getattr(sh, "clients_all", None) is not None else None
    if cl is None:
        return "status words clean on every rank (no client counts for an oracle check)"
    batch, st, kept = generate(p, ann_props(), docs=range(k), keep=True, ops_per_doc=sh.all_ops[:k],
                               clients_per_doc=cl, threads=min(16, os.cpu_count() or 1))
    last = batch.op_offsets[1:] - 1
    odg = np.array([kept[d].snapshot(int(batch.arrays["msn"][last[d]]), int(batch.arrays["seq"][last[d]]))[1]
                    for d in range(k)], np.uint64)
    del kept
    return digest_parity(digs, odg, np.asarray(st)) + ", all ranks clean"


def config5_rank_parity(args, c, sh, k=16):
    """This rank's check: the oracle (its own generator, same seed and per-document counts)
    replays the k owned documents of smallest global id; their digests must equal this
    rank's (sh.local_digests, before the gather).  Returns (mismatches, checked)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fluidframework_amd.batch import MtGenParams
    from oracle_lib import generate
    loc = np.argsort(sh.owned, kind="stable")[:min(k, sh.n_docs)]
    if not len(loc):
        return 0, 0
    gids = sh.owned[loc]
    p = MtGenParams(args.seed, len(gids), 0, 2, c["lag"], c["ins"], c["rem"], c["ins_len"], c["rem_len"], c["ann_sets"],
                    c["rewrite"])
    batch, st, kept = generate(p, ann_props(), docs=gids, keep=True, ops_per_doc=sh.all_ops[gids],
                               clients_per_doc=sh.clients_all[gids])
    last = batch.op_offsets[1:] - 1
    odg = np.array([kept[j].snapshot(int(batch.arrays["msn"][last[j]]), int(batch.arrays["seq"][last[j]]))[1]
                    for j in range(len(gids))], np.uint64)
    return int((sh.local_digests[loc] != odg).sum()) + int(np.asarray(st).any()), len(gids)


def cpu_baseline_config5(args, c, local):
    """Oracle on a bounded sample of config-5 documents (same Zipf sizes)."""
    from fluidframework_amd.batch import MtGenParams
    from fluidframework_amd.shard import clients_per_doc, generation_caps, zipf_op_counts
    threads = min(16, os.cpu_count() or 1)
    n = 4000
    ops = zipf_op_counts(n, args.seed ^ 0x5A)
    cl = clients_per_doc(n, args.seed ^ 0x5A)
    eng = Host.engine(n, local, per_doc=generation_caps(ops, c["ins_len"]))
    eng.upload_props(ann_props())
    eng.upload_names(['"c%d"' % i for i in range(64)])
    cc = dict(c)
    cc["docs"] = n
    res, _, _ = cpu_baseline(eng, cc, MtGenParams, args.seed ^ 0x5A, args.cpu_seconds, threads,
                             ops_fn=lambda k: (ops[:k], cl[:k]))
    eng.close()
    return res


def batch_messages(batch, run):
    """ISequencedDocumentMessage dicts (protocol.ts:126-166) of one generated run; client i
    is "c{i}" (the ingest leg's input, built untimed)."""
    a = batch.arrays
    o0, o1 = int(batch.op_offsets[run]), int(batch.op_offsets[run + 1])
    pay = batch.payload
    out = []
    for i in range(o0, o1):
        t = int(a["type"][i])
        m = {"clientId": f"c{int(a['client'][i])}", "sequenceNumber": int(a["seq"][i]),
             "referenceSequenceNumber": int(a["ref_seq"][i]), "minimumSequenceNumber": int(a["msn"][i]), "type": "op"}
        if t == 0:
            po, pl = int(a["payload_off"][i]), int(a["payload_len"][i])
            m["contents"] = {"type": 0, "pos1": int(a["pos1"][i]), "seg": pay[po:po + pl].tobytes().decode("utf-16-le")}
        else:
            m["contents"] = {"type": t, "pos1": int(a["pos1"][i]), "pos2": int(a["pos2"][i])}
            if t == 2:
                m["contents"]["props"] = {"k0": "v"}
        out.append(m)
    return out


def ingest_leg(local, c, seed, sample_docs=64):
    """Host ingest (host packing and H2D reported, not hidden): the
    messages of `sample_docs` documents of the workload packed by the Python host
    (fluidframework_amd.batch.BatchBuilder) and by the Node host (js/index.js
    BatchBuilder), and the packed batch's upload to HBM (mt_upload_batch + sync)."""
    import shutil
    import subprocess
    import tempfile
    from fluidframework_amd.batch import BatchBuilder, ClientNames, MtGenParams, PropTable
    n = min(sample_docs, c["docs"])
    eng = Host.engine(n, local, **caps_for(dict(c, docs=n)))
    eng.upload_props(ann_props())
    eng.upload_names(['"c%d"' % i for i in range(64)])
    eng.generate(MtGenParams(seed, n, c["ops"], c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"],
                             c["rem_len"], c["ann_sets"], c["rewrite"]))
    eng.sync()
    docs = [batch_messages(eng.generated_download(), d) for d in range(n)]
    msgs = sum(len(d) for d in docs)
    t0 = time.perf_counter()
    bb = BatchBuilder(PropTable(), None)
    for d, lst in enumerate(docs):
        bb.names = ClientNames()
        bb.begin_doc(d)
        for m in lst:
            bb.add_message(m)
    batch = bb.build()
    py_s = time.perf_counter() - t0
    eng.open_docs(0, n)
    eng.sync()
    for _ in range(2):                                  # both pinned staging buffers allocated
        eng.upload(batch)
    eng.sync()
    reps = 4
    t0 = time.perf_counter()
    for _ in range(reps):                               # steady state: staging reused, no allocation
        eng.upload(batch)
    eng.sync()
    h2d_s = (time.perf_counter() - t0) / reps
    h2d_bytes = int(batch.n_ops) * 32 + int(batch.payload.nbytes)
    node = None
    exe = shutil.which("node")
    if exe:
        with tempfile.TemporaryDirectory() as td:
            for d, lst in enumerate(docs):              # one JSON stream per document
                with open(os.path.join(td, f"doc{d}.json"), "w") as f:
                    json.dump(lst, f, separators=(",", ":"))
            workers = max(1, min(16, os.cpu_count() or 1))
            cmd = [exe, os.path.join(ROOT, "fluidframework_amd", "js", "ingest_bench.js"), td, str(workers)]
            if Host.factory is None:
                cmd.append("--gpu")                     # messages in -> digests out through the addon
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
            if r.returncode == 0:
                node = json.loads(r.stdout.strip().splitlines()[-1])
            else:
                node = {"error": r.stderr[-500:]}
    eng.close()
    ok = node is not None and "error" not in node
    return {"sample": f"{n} docs x {c['ops']} msgs of the workload ({msgs} messages, one op each)",
            "python_pack_msgs_per_s": msgs / py_s,
            "node_pack_msgs_per_s": node["single_msgs_per_s"] if ok else None,
            "node_parallel_pack_msgs_per_s": node["parallel_msgs_per_s"] if ok else None,
            "node_workers": node["workers"] if ok else None,
            "node_e2e_msgs_per_s": node.get("e2e_msgs_per_s") if ok else None,
            "node": node,
            "h2d_msgs_per_s": msgs / h2d_s, "h2d_GBps": h2d_bytes / h2d_s / 1e9, "h2d_bytes": h2d_bytes,
            "note": "packers: JSON text per document -> mt_op_batch (Node: parse + pack, one thread, and a "
                    "worker_threads pool reading its own documents' streams); H2D = mt_upload_batch (validation and "
                    "record packing on up to 16 host threads into reused pinned staging, one async copy), mean of 4 "
                    "back-to-back batches + sync; node e2e = parallel parse + pack, mt_apply_batch, sync, "
                    "SnapshotV1 digests of every document; the timed replay starts from resident streams"}


def write_doc_bins(batch, td):
    """Each document's op columns as doc<i>.bin (js/pack_worker.js binToJson's layout), the
    input of js/ingest_scale.js."""
    a = batch.arrays
    off = batch.op_offsets
    pay = batch.payload
    for d in range(len(off) - 1):
        o0, o1 = int(off[d]), int(off[d + 1])
        po = a["payload_off"][o0:o1].astype(np.int64)
        pl = a["payload_len"][o0:o1].astype(np.int64)
        ins = (a["type"][o0:o1] == 0) & (pl > 0)
        p0 = int(po[ins].min()) if ins.any() else 0
        p1 = int((po + pl)[ins].max()) if ins.any() else 0
        rel = np.where(ins, po - p0, 0)
        cols = [a["type"][o0:o1], a["client"][o0:o1], a["seq"][o0:o1], a["ref_seq"][o0:o1], a["msn"][o0:o1],
                a["pos1"][o0:o1], a["pos2"][o0:o1], rel, pl]
        head = np.array([o1 - o0, p1 - p0], np.int32)
        with open(os.path.join(td, f"doc{d}.bin"), "wb") as f:
            f.write(head.tobytes())
            for col in cols:
                f.write(np.ascontiguousarray(col, np.int32).tobytes())
            f.write(np.ascontiguousarray(pay[p0:p1], np.uint16).tobytes())


def ingest_scale_leg(eng, params, c, dig_xor, windows=8, objects=False):
    """Node host ingest at the workload's full size (every document of the config): message JSON
    parsed and packed on a worker pool, then end to end through the addon with packing of message
    window k+1 (of every document) overlapped with the upload and replay of window k
    (js/ingest_scale.js).  Its SnapshotV1 digests must equal the bench's own (same messages,
    replayed from JSON).  The workload is generated again first (the CPU baseline's sample
    generation replaced it on the engine)."""
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("node")
    if not exe or Host.factory is not None:
        return None
    eng.generate(params)
    eng.sync()
    batch = eng.generated_download()
    workers = max(1, min(16, os.cpu_count() or 1))
    with tempfile.TemporaryDirectory() as td:
        t0 = time.perf_counter()
        write_doc_bins(batch, td)
        write_s = time.perf_counter() - t0
        del batch
        cmd = [exe, "--max-old-space-size=8192", os.path.join(ROOT, "fluidframework_amd", "js", "ingest_scale.js"), td,
               str(workers), str(windows), "--gpu"] + (["--objects"] if objects else [])
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        return {"error": r.stderr[-800:]}
    res = json.loads(r.stdout.strip().splitlines()[-1])
    res["digests_equal_bench"] = res.get("digest_xor") == f"{dig_xor:016x}"
    res["input_write_s"] = write_s
    if objects:
        res["note"] = (f"all {c['docs']} documents: per-document ISequencedDocumentMessage objects (already parsed, "
                       f"as SharedSegmentSequence.processCore receives them) in {windows} message windows made inside "
                       "the workers (untimed); pack_ms = BatchBuilder.addMessages of every window on the pool, parts "
                       "left unmerged; e2e_ms = pack of window k+1 of every document overlapped with "
                       "mt_apply_batch_parts (the parts concatenated and re-based on the library's host threads) "
                       "upload + replay of window k, one sync, SnapshotV1 of every document")
    else:
        res["note"] = (f"all {c['docs']} documents: per-document message JSON in {windows} message windows made "
                       "inside the workers (untimed); pack_ms = parse + pack of every window on the pool (the host "
                       "bound); e2e_ms = parse/pack of window k+1 of every document overlapped with mt_apply_batch "
                       "upload + replay of window k, one sync, SnapshotV1 of every document")
    return res


def finish_dist():
    """Every rank leaves together and tears its process group down (a rank that exits with
    its group still up can abort in the communication library's exit handlers)."""
    try:
        import torch.distributed as tdist
    except ImportError:
        return
    if tdist.is_available() and tdist.is_initialized():
        tdist.barrier()
        tdist.destroy_process_group()


def set_residency(eng, args):
    if args.residency == "big" and args.big_flags:
        eng.set_residency(RESIDENCY["big"], 0, args.big_flags, 0)  # blocks = MT_BIGF_* switches
    else:
        eng.set_residency(RESIDENCY[args.residency])


def main(argv=None):
    try:
        return _main(argv)
    finally:
        finish_dist()


def _main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="config2", choices=sorted(CONFIGS))
    ap.add_argument("--docs", type=int, default=0, help="override documents per GPU")
    ap.add_argument("--ops", type=int, default=0, help="override messages per document")
    ap.add_argument("--seed", type=int, default=20241015)
    ap.add_argument("--prebuild", type=int, default=0, help="config4: override pre-build appends per document")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-docs", type=int, default=0,
                    help="documents the oracle checks (config 4: default one per host thread; config 5: 4096)")
    ap.add_argument("--no-ingest", action="store_true", help="skip the host ingest leg (packers, H2D)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--residency", default="auto", choices=["auto", "lds", "hbm", "blk", "big"],
                    help="blk: blocks + heap in LDS, in-wave HBM continuation; big: heap + window + U set in LDS "
                         "for long documents; hbm: every pool in HBM; lds: rows/blocks/heap/window in LDS; "
                         "auto (default): big for config4, blk otherwise")
    ap.add_argument("--caps", default="", help="override pool caps, e.g. rows_per_doc=400,text_per_doc=16384")
    ap.add_argument("--big-flags", type=int, default=0,
                    help="big residency A/B switches (MT_BIGF_*): 1 block cache off, 2 zamboni prefetch off, "
                         "4 corrections table off, 8 parent cache off")
    ap.add_argument("--cont-min", type=int, default=-1,
                    help="block residency: runs of at least this many messages keep the in-wave HBM "
                         "continuation (mt_set_continuation; -1: the library default)")
    ap.add_argument("--partition", default="",
                    help="partitioned size classes under blk residency: 'auto' (default: the library's rule, "
                         "mt_plan_partition, per resident batch), 'off', or MIN_MSGS:CUS (runs of at least MIN_MSGS "
                         "messages in the wide kernel on CUS reserved CUs)")
    ap.add_argument("--big-min-ops", type=int, default=-1,
                    help="size classes under blk residency: runs of at least this many messages replay in the "
                         "long-document kernel on a second stream (0: off; default: the config's)")
    ap.add_argument("--shares", type=int, default=0,
                    help="config5: replay each rank's share of the N-rank LPT plan (docs per GPU x N documents) in "
                         "turn on this one GPU and report the slowest share's step (an N-GPU projection)")
    args = ap.parse_args(argv)
    if args.residency == "auto":
        args.residency = "big" if args.config == "config4" else "blk"

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: re-enter this script under torch.distributed.run
        raise SystemExit(launch(args.gpus, sys.argv[1:] if argv is None else argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.config == "config4":
        c = dict(CONFIGS["config4"])
        if args.docs:
            c["docs"] = args.docs
        if args.ops:
            c["ops"] = args.ops
        if args.prebuild:
            c["prebuild"] = args.prebuild
        return run_config4(args, c, world, rank, local)
    if args.config == "config5":
        c = dict(CONFIGS["config5"])
        if args.docs:
            c["docs"] = args.docs
        if args.shares:
            return run_config5_shares(args, c, local)
        return run_config5(args, c, world, rank, local)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        tdist.init_process_group("gloo")  # rank coordination only: no data-path collective (weak scaling)
        dist = (torch, tdist)

    from fluidframework_amd.batch import MtGenParams

    c = dict(CONFIGS[args.config])
    if args.docs:
        c["docs"] = args.docs
    if args.ops:
        c["ops"] = args.ops
    caps = caps_for(c)
    for kv in filter(None, args.caps.split(",")):
        k, v = kv.split("=")
        caps[k] = int(v)
    eng = Host.engine(c["docs"], local, **caps)
    set_residency(eng, args)
    stage_ms = reserve_staging(eng)
    big = c.get("big_min_ops", 0) if args.big_min_ops < 0 else args.big_min_ops
    if args.residency == "blk" and big:
        eng.set_size_class(big)
    part = apply_partition(eng, args, c) if not big else None
    if args.cont_min >= 0:
        eng.set_continuation(args.cont_min)
    eng.upload_props(ann_props())
    eng.upload_names(['"c%d"' % i for i in range(64)])
    seed = args.seed ^ (rank * 0x9E3779B1)
    params = MtGenParams(seed, c["docs"], c["ops"], c["clients"], c["lag"], c["ins"], c["rem"], c["ins_len"],
                         c["rem_len"], c["ann_sets"], c["rewrite"])
    t0 = time.time()
    eng.generate(params)
    eng.sync()
    gen_s = time.time() - t0
    st = eng.status(range(c["docs"]))
    if st.any():
        raise SystemExit(f"rank {rank}: generation failed, status {np.unique(st)}")
    cnt = eng.counters(range(c["docs"]))
    msgs = int(cnt["msgs"].sum())
    bytes_per_launch = algorithmic_bytes(cnt)
    eng.generated_to_resident()

    def step():
        eng.open_docs(0, c["docs"])
        eng.replay_resident()

    for _ in range(args.warmup):
        step()
    eng.sync()

    def barrier():
        if dist:
            dist[1].barrier()

    barrier()
    eng.sync()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.steps):
        step()
        eng.sync()
        kms.append(eng.last_replay_ms())
    eng.sync()
    barrier()
    dt = time.perf_counter() - t0
    if dist:
        torch, tdist = dist
        t = torch.tensor([dt], dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t.item())
    st = eng.status(range(c["docs"]))
    cnt2 = eng.counters(range(c["docs"]))
    handover = None
    if args.residency != "hbm":
        cur = eng.last_cursors(c["docs"]).astype(np.int64) & 0x7FFFFFFF   # high bit: finished in-wave
        ends = (np.arange(c["docs"]) + 1) * c["ops"]
        ho = np.nonzero(cur < ends)[0]
        # where each hand-over happened: the op index within its run (the rest ran from HBM)
        handover = {"docs": int(len(ho)), "at_op": [int(cur[d] - d * c["ops"]) for d in ho[:16]]}
    # SnapshotV1 of every document at its current window (reported, not timed as ops)
    t1 = time.perf_counter()
    sthreads = min(16, os.cpu_count() or 1)
    neg = np.full(c["docs"], -1, np.int32)
    digs = eng.snapshot_digests(range(c["docs"]), neg, neg, threads=sthreads) if eng.fn["snapshot_digests"] else np.zeros(1, np.uint64)
    snap_ms = (time.perf_counter() - t1) * 1e3
    dig_xor = int(np.bitwise_xor.reduce(digs)) if len(digs) else 0
    ok = (not st.any()) and int(cnt2["msgs"].sum()) == msgs
    total_msgs = msgs * world * args.steps
    value = total_msgs / dt
    kern_s = float(np.mean(kms)) / 1e3
    achieved = bytes_per_launch / kern_s / 1e9 if kern_s > 0 else 0.0
    if world > 1:
        # every rank checks its own documents against the oracle (untimed), rank 0 reports the sum
        k = min(PARITY_DOCS, c["docs"])
        _, _, odg, ost = oracle_run(eng, c, MtGenParams, seed, k, max(1, min(16, (os.cpu_count() or 1) // world)))
        bad_l = int((np.asarray(digs[:k], np.uint64) != odg).sum()) + int(np.asarray(ost).any()) + int(not ok)
        par_bad, par_checked = rank_parity(dist, bad_l, k)
    if rank != 0:
        return
    traffic = measured_traffic(args.config, c, REPLAY_KERNEL[args.residency])
    out = {
        "metric": "sequenced merge-tree ops applied/sec (whole node) + achieved HBM GB/s",
        "value": value,
        "unit": "ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (device-generated sequenced op streams, SURVEY.md §8(d) rules)",
        "config": {"workload": f"{args.config}: {c['desc']}", "docs_per_gpu": c["docs"], "msgs_per_doc": c["ops"],
                   "clients": c["clients"], "lag_max": c["lag"], "mix_ins_rem_ann": [c["ins"], c["rem"],
                                                                                   100 - c["ins"] - c["rem"]],
                   "parallelism": f"doc-sharded x{world}", "residency": args.residency,
                   "big_min_ops": big if args.residency == "blk" else None, "lds_handover_docs": handover,
                   "partition": partition_report(eng, args, part)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS,
                     "traffic": traffic[0] if traffic else None,
                     "traffic_source": traffic[1] if traffic else None,
                     "kernel": REPLAY_KERNEL[args.residency], "kernel_ms": kern_s * 1e3,
                     "bytes_per_launch": bytes_per_launch},
        "hbm_gbps_algorithmic": achieved,
        "parity": "status words clean" if ok else "STATUS ERROR",
        "snapshot": {"docs": c["docs"], "ms": snap_ms, "host_threads": sthreads, "digest_xor": f"{dig_xor:016x}",
                     "staging_reserve_ms": stage_ms,
                     "note": "mt_snapshot_digests after the timed steps: staged download + SnapshotV1 JSON + xxh64"},
        "gen_seconds": gen_s,
    }
    if world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        out["cpu_baseline"], odg, ost = cpu_baseline(eng, c, MtGenParams, seed, args.cpu_seconds, threads)
        if ok:
            out["parity"] = digest_parity(digs, odg, ost)
            out["roofline"]["bytes_pinned"] = (f"mt_doc_counters == oracle's own §8(d) count on {len(odg)} docs"
                                               if counters_match(cnt2, len(odg)) else "COUNTER MISMATCH vs oracle")
    elif world > 1 and ok:
        out["parity"] = parity_text(par_bad, par_checked, world)
    # rank 0's documents are the default seed's at any N (seed ^ rank * ...): all of them against
    # the oracle-made manifest
    man = manifest_parity(args.config, digs, seed=args.seed, docs=c["docs"], msgs_per_doc=c["ops"]) if ok else None
    if man is not None:
        out["parity_manifest"] = man
        out["parity"] += manifest_text(man)
    if world == 1 and not args.no_ingest:
        out["ingest"] = ingest_leg(local, c, seed)
        if args.config == "config2" and ok:
            out["ingest"]["node_full_scale"] = ingest_scale_leg(eng, params, c, dig_xor)
            out["ingest"]["node_objects_full_scale"] = ingest_scale_leg(eng, params, c, dig_xor, objects=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
