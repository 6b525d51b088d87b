"""Document sharding across GPUs (BASELINE config 5).

Documents are fully independent (one `Client` per DDS, packages/dds/sequence/
src/sequence.ts:131-134), so the engine shards them across ranks with no
per-op communication.  The two exchanges are the ones the north star names,
both over torch.distributed (backend "nccl" = RCCL over xGMI on ROCm; "gloo"
in the CPU tests):

1. a one-shot size-balanced redistribution: rank 0 holds every document's
   sequenced op stream (the ingest point); every rank computes the same LPT
   (longest-processing-time) plan from the broadcast op counts, and rank 0
   sends each rank its documents as exchange rows (a 32-byte op record plus the
   op's UTF-16 payload slot, csrc/mt_shard.h) in one all_to_all_single (per-link
   bound on xGMI: each destination's share travels on its own link).  The rows
   are packed at their plan positions and unpacked into the resident batch by
   the engine's own HIP kernels, and every document's 64-bit row checksum is
   compared on arrival with rank 0's (round 2 moved them with torch gathers,
   one of which returned zero rows for 16-byte rows at config-5 size);
2. the gather of per-document SnapshotV1 digests to rank 0.

Pool capacities are exact: generation runs the same deterministic engine, so
its high-water marks (mt_doc_pools) are what a replay of the same stream needs.
"""
from __future__ import annotations

import heapq
import time

import numpy as np

REC_BYTES = 32           # mt_op_rec


def zipf_op_counts(n_docs: int, seed: int, s: float = 1.5, lo: int = 8, hi: int = 65536) -> np.ndarray:
    """Messages per document ~ Zipf(s) truncated to [lo, hi] (SURVEY §8(d) config 5;
    mean ≈ 700 for the defaults), deterministic in seed."""
    k = np.arange(lo, hi + 1, dtype=np.float64)
    cdf = np.cumsum(k ** -s)
    cdf /= cdf[-1]
    u = np.random.Generator(np.random.PCG64(seed)).random(n_docs)
    return (lo + np.searchsorted(cdf, u, side="left")).astype(np.uint32)


def clients_per_doc(n_docs: int, seed: int, lo: int = 2, hi: int = 16) -> np.ndarray:
    """Authoring clients per document ~ U[lo, hi] (config 5)."""
    return np.random.Generator(np.random.PCG64(seed ^ 0xC11E)).integers(lo, hi + 1, n_docs).astype(np.uint32)


def lpt_assign(costs: np.ndarray, world: int) -> np.ndarray:
    """LPT bins: documents by decreasing cost (ties by id) each go to the least
    loaded rank (ties by rank).  Deterministic, so every rank computes the same plan."""
    order = np.lexsort((np.arange(len(costs)), -np.asarray(costs, np.int64)))
    heap = [(0, r) for r in range(world)]
    owner = np.empty(len(costs), np.int32)
    for d in order:
        load, r = heapq.heappop(heap)
        owner[d] = r
        heapq.heappush(heap, (load + int(costs[d]), r))
    return owner


def generation_caps(ops: np.ndarray, ins_len: int) -> dict:
    """Generous per-document pools for the generating context.  The window is bounded by the
    MSN's lag behind the current seq, not by the stream length; 1,048,576 Zipf documents hold
    one whose window passes 1,024 entries (a client silent for a long stretch holds the MSN)."""
    o = np.asarray(ops, np.int64)
    return dict(rows_per_doc=3 * o + 64, blocks_per_doc=o + 64, heap_per_doc=2 * o + 64,
                window_per_doc=np.minimum(2 * o + 64, 8192), text_per_doc=ins_len * o + 4096,
                propsets_per_doc=np.full(len(o), 64))


# Pool bytes per element / per document, as mt_create_impl lays them out (csrc/mt_api_impl.h):
# rows 48 B (MtRow); blocks 64 B; heap 8 B (cap + 1 entries); window + U ids + U deltas 12 B;
# ancestor chains 4 B x MT_MAXH (16) per window entry; text 2 x 2 B (two halves); property
# sets 112 B (MtPSet); marker ids 4 B; register rows 2 x 4 B; per document: header, recycled
# rows (4 x MT_RFL 128), layout, overlap side list (16 x 512), registers (32 x 64).
_DOC_FIXED = 208 + 4 * 128 + 112 + 16 * 512 + 32 * 64


def pool_bytes_estimate(caps: dict) -> int:
    """HBM bytes an engine with these per-document caps allocates (mt_pool_bytes; markers 1,024
    and register rows 256 per document unless given)."""
    c = {k: np.asarray(v, np.int64) for k, v in caps.items()}
    n = len(c["rows_per_doc"])
    mark = c.get("markers_per_doc", np.full(n, 1024))
    regr = c.get("register_rows_per_doc", np.full(n, 256))
    per = (48 * c["rows_per_doc"] + 64 * c["blocks_per_doc"] + 8 * (c["heap_per_doc"] + 1) +
           12 * c["window_per_doc"] + 4 * 16 * c["window_per_doc"] + 4 * c["text_per_doc"] +
           112 * c["propsets_per_doc"] + 4 * mark + 8 * regr + _DOC_FIXED)
    return int(per.sum())


def rank0_peak_bytes(ops: np.ndarray, world: int, ins_len: int = 8, chunk_docs: int = 131072) -> dict:
    """Rank 0's device memory peak in build_sharded + replay: the send buffer of every
    document's rows (held while generation chunks come and go), the largest generating
    engine, then the rows it receives and its own engine (generation caps: an upper bound of
    the exact replay caps)."""
    ops = np.asarray(ops, np.int64)
    send = int(ops.sum()) * (REC_BYTES + 2 * ins_len)
    gen = max(pool_bytes_estimate(generation_caps(ops[a:a + chunk_docs], ins_len))
              for a in range(0, len(ops), chunk_docs))
    owner = lpt_assign(ops, world)
    mine = ops[owner == 0]
    recv = int(mine.sum()) * (REC_BYTES + 2 * ins_len)
    own = pool_bytes_estimate(generation_caps(mine, ins_len))
    return {"send": send, "generate": gen, "recv": recv, "own_engine": own,
            "total": send + max(gen, recv + own)}


def replay_caps(pools: np.ndarray, gen_caps: dict, idx) -> np.ndarray:
    """[n, 6] caps (rows, blocks, heap, window, text, psets) from the generation's
    high-water marks (mt_doc_pools columns 0, 1, 8, 9, 5); text keeps the generation cap."""
    p = np.asarray(pools, np.int64)
    cap = np.stack([np.maximum(p[:, 0], 1), np.maximum(p[:, 1], 1), np.maximum(p[:, 8], 1), np.maximum(p[:, 9], 1),
                    np.asarray(gen_caps["text_per_doc"])[idx], np.maximum(p[:, 5], 1)], axis=1)
    return cap.astype(np.int32)


def rank_order(owner: np.ndarray, ops: np.ndarray) -> np.ndarray:
    """Documents grouped by owning rank; within a rank, largest first (so the
    longest streams start first and set less of the tail), then by id."""
    return np.lexsort((np.arange(len(ops)), -np.asarray(ops, np.int64), np.asarray(owner)))


class SoloDist:
    """The torch.distributed subset build_sharded uses, for a single process."""

    def get_world_size(self):
        return 1

    def get_rank(self):
        return 0

    def broadcast(self, t, src):
        pass

    def barrier(self):
        pass

    def all_to_all_single(self, out, inp, out_split, in_split):
        out.copy_(inp)

    def all_gather(self, outs, t):
        outs[0].copy_(t)

    def gather(self, t, gather_list=None, dst=0):
        gather_list[0].copy_(t)


CAP_KEYS = ("rows_per_doc", "blocks_per_doc", "heap_per_doc", "window_per_doc", "text_per_doc", "propsets_per_doc")


class ShardedReplay:
    """One rank's share of a sharded replay: an Engine holding its documents with
    their op streams resident, plus the plan (owner of every global document)."""

    def __init__(self, engine, owned: np.ndarray, all_ops: np.ndarray, owner: np.ndarray, timings: dict,
                 clients_all: np.ndarray | None = None):
        self.engine, self.owned, self.all_ops, self.owner, self.timings = engine, owned, all_ops, owner, timings
        self.clients_all = clients_all     # authoring clients of every global document
        self.ops = all_ops[owned]          # engine document slot i holds global document owned[i]

    @property
    def n_docs(self) -> int:
        return len(self.owned)

    def replay(self):
        # documents whose exchange rows arrived with a checksum other than rank 0's are
        # corrupt: replaying them would publish wrong results as if they were right
        bad = int(self.timings.get("exchange_bad_docs", 0))
        if bad:
            from .engine import ExchangeError
            raise ExchangeError(f"refusing to replay: {bad} of {self.n_docs} documents failed the exchange checksum",
                                np.zeros(0, np.uint32))
        self.engine.open_docs(0, self.n_docs)
        self.engine.replay_resident()

    def gather_digests(self, dist, device, threads: int = 8):
        """SnapshotV1 digests of every document at its current window, gathered to
        rank 0 in global document order (None on other ranks)."""
        import torch
        t0 = time.perf_counter()
        n = self.n_docs
        neg = np.full(n, -1, np.int32)
        dig = self.engine.snapshot_digests(range(n), neg, neg, threads=threads) if n else np.zeros(0, np.uint64)
        self.timings["snapshot_ms"] = (time.perf_counter() - t0) * 1e3     # this rank's SnapshotV1 digests
        self.local_digests = dig           # engine slot order (owned[i]): each rank's own parity sample
        world, rank = dist.get_world_size(), dist.get_rank()
        counts = np.bincount(self.owner, minlength=world)
        mx = int(counts.max()) if len(counts) else 0
        buf = torch.zeros(mx, dtype=torch.int64, device=device)
        if n:
            buf[:n] = torch.from_numpy(dig.view(np.int64)).to(device)
        # a gather to rank 0 (the only consumer), not an all-gather
        out = [torch.zeros(mx, dtype=torch.int64, device=device) for _ in range(world)] if rank == 0 else None
        dist.gather(buf, gather_list=out, dst=0)
        self.timings["digest_ms"] = (time.perf_counter() - t0) * 1e3
        if rank != 0:
            return None
        res = np.zeros(len(self.owner), np.uint64)
        order = rank_order(self.owner, self.all_ops)
        own_sorted = self.owner[order]
        for r in range(world):
            docs_r = order[own_sorted == r]
            res[docs_r] = out[r][:len(docs_r)].cpu().numpy().view(np.uint64)
        return res


class SharePlan:
    """The LPT plan every rank computes from the broadcast op counts: owner of every document,
    the send order (documents grouped by owning rank, largest first), each document's first row
    in rank 0's send buffer and each rank's op count."""

    def __init__(self, ops: np.ndarray, world: int):
        self.ops, self.world = ops, world
        self.owner = lpt_assign(ops, world)
        self.order = rank_order(self.owner, ops)
        self.row_of = np.empty(len(ops), np.int64)
        self.row_of[self.order] = np.concatenate(([0], np.cumsum(ops[self.order].astype(np.int64))[:-1]))
        self.per_rank_ops = np.array([int(ops[self.owner == r].sum()) for r in range(world)], np.int64)
        self.rank_row0 = np.concatenate(([0], np.cumsum(self.per_rank_ops)))      # rank r's rows in the send buffer

    def owned(self, rank: int) -> np.ndarray:
        """Rank `rank`'s documents in its engine's slot order (the send order)."""
        return self.order[self.owner[self.order] == rank]


def generate_send_rows(device, engine_factory, plan: SharePlan, cli: np.ndarray, seed: int, gen_params_cls,
                       gen_kw: dict, props, names, chunk_docs: int, W: int):
    """Rank 0's ingest: every document's stream generated in chunks (untimed) and packed by the
    engine straight into its plan position of the send buffer (mt_generated_pack_rows, a HIP
    kernel) with a 64-bit checksum per document.  Returns (send rows, replay caps [n, 6],
    checksums) as device tensors."""
    import torch
    ops = plan.ops
    docs_total = len(ops)
    L = int(gen_kw["ins_len_max"])
    caps_t = torch.zeros((docs_total, 6), dtype=torch.int32, device=device)
    cs_t = torch.zeros(docs_total, dtype=torch.int64, device=device)
    send = torch.empty((int(ops.sum(dtype=np.int64)), W), dtype=torch.int64, device=device)
    gcaps = generation_caps(ops, L)
    for a in range(0, docs_total, chunk_docs):
        b = min(docs_total, a + chunk_docs)
        idx = np.arange(a, b)
        eng = engine_factory(b - a, {k: np.asarray(v)[idx] for k, v in gcaps.items()})
        if props is not None:
            eng.upload_props(props)
        if names is not None:
            eng.upload_names(names)
        p = gen_params_cls(**{**gen_kw, "seed": seed, "n_docs": b - a, "ops_per_doc": 0, "clients": 2,
                              "doc_id_base": a})
        eng.generate(p, ops_per_doc=ops[idx], clients_per_doc=cli[idx])
        eng.sync()
        st = eng.status(range(b - a))
        if st.any():
            raise RuntimeError(f"generation failed for docs {a}..{b}: status {np.unique(st)}")
        caps_t[a:b] = torch.from_numpy(replay_caps(eng.pools(range(b - a)), gcaps, idx)).to(device)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        cs = eng.generated_pack_rows(0, b - a, plan.row_of[a:b].astype(np.uint64), send.data_ptr())
        cs_t[a:b] = torch.from_numpy(cs.view(np.int64)).to(device)
        eng.close()
    return send, caps_t, cs_t


def rank_engine(engine_factory, owned: np.ndarray, ops: np.ndarray, caps: np.ndarray, sums: np.ndarray, recv_ptr: int,
                L: int, props, names, tm: dict):
    """A rank's engine, sized exactly from the generation's high-water marks; the received rows
    (at device address recv_ptr) become its resident batch (mt_upload_rows_dev: unpacked by a
    HIP kernel, every document's checksum compared with rank 0's)."""
    mine = caps[owned]
    eng = engine_factory(len(owned), {k: mine[:, i] for i, k in enumerate(CAP_KEYS)})
    if props is not None:
        eng.upload_props(props)
    if names is not None:
        eng.upload_names(names)
    loc_off = np.zeros(len(owned) + 1, np.int64)
    loc_off[1:] = np.cumsum(ops[owned], dtype=np.int64)
    if loc_off[-1] >= 2 ** 32:
        raise RuntimeError("more than 2^32 ops on one rank")
    from .engine import ExchangeError
    t0 = time.perf_counter()
    try:
        eng.upload_rows_dev(np.arange(len(owned)), loc_off.astype(np.uint32), recv_ptr if loc_off[-1] else 0, L,
                            sums[owned])
        tm["exchange_bad_docs"] = 0
    except ExchangeError as e:          # reported by the caller after every rank checked its share
        tm["exchange_bad_docs"] = int(e.bad_runs.sum())
    tm["unpack_ms"] = (time.perf_counter() - t0) * 1e3
    tm["exchange_checked_docs"] = len(owned)
    return eng


def build_sharded(dist, device, engine_factory, docs_total: int, seed: int, gen_params_cls, gen_kw: dict,
                  props=None, names=None, chunk_docs: int = 131072, counts=None, clients=None) -> ShardedReplay:
    """Rank 0 generates every document's stream (the ingest point), every rank
    gets its LPT share by RCCL/gloo collectives, and each rank's engine ends up
    holding its documents with their streams resident.

    engine_factory(n_docs, per_doc_caps: dict) -> Engine;  gen_kw: MtGenParams
    fields other than seed/n_docs/ops_per_doc/clients."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    L = int(gen_kw["ins_len_max"])
    if L % 4:
        raise ValueError("ins_len_max must be a multiple of 4 (payload rows are staged as 8-byte words)")
    tm = {}
    # -- op counts / clients: known at the ingest point, broadcast to all ranks
    t0 = time.perf_counter()
    cnt_t = torch.zeros(docs_total, dtype=torch.int32, device=device)
    cli_t = torch.zeros(docs_total, dtype=torch.int32, device=device)
    if rank == 0:
        c0 = zipf_op_counts(docs_total, seed) if counts is None else np.asarray(counts, np.uint32)
        k0 = clients_per_doc(docs_total, seed) if clients is None else np.asarray(clients, np.uint32)
        cnt_t.copy_(torch.from_numpy(c0.astype(np.int32)))
        cli_t.copy_(torch.from_numpy(k0.astype(np.int32)))
    dist.broadcast(cnt_t, 0)
    dist.broadcast(cli_t, 0)
    ops = cnt_t.cpu().numpy().astype(np.uint32)
    cli = cli_t.cpu().numpy().astype(np.uint32)
    # -- the plan's send order: documents grouped by owning rank, largest first
    plan = SharePlan(ops, world)
    owner = plan.owner
    W = REC_BYTES // 8 + 2 * L // 8                  # 8-byte words per exchange row (mt_shard.h)
    per_rank_ops = plan.per_rank_ops
    my_ops = int(per_rank_ops[rank])
    tm["plan_ms"] = (time.perf_counter() - t0) * 1e3

    # -- rank 0: generate every stream (untimed ingest) into the send buffer
    if rank == 0:
        t0 = time.perf_counter()
        send, caps_t, cs_t = generate_send_rows(device, engine_factory, plan, cli, seed, gen_params_cls, gen_kw,
                                                props, names, chunk_docs, W)
        tm["generate_s"] = time.perf_counter() - t0
    else:
        caps_t = torch.zeros((docs_total, 6), dtype=torch.int32, device=device)
        cs_t = torch.zeros(docs_total, dtype=torch.int64, device=device)
    dist.broadcast(caps_t, 0)
    dist.broadcast(cs_t, 0)
    caps = caps_t.cpu().numpy()
    sums = cs_t.cpu().numpy().view(np.uint64)

    # -- redistribution: rank 0 -> every rank, one all_to_all_single of the rows
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    dist.barrier()
    t0 = time.perf_counter()
    owned = plan.owned(rank)
    if rank == 0:
        in_split = per_rank_ops.tolist()
    else:
        send = torch.empty((0, W), dtype=torch.int64, device=device)
        in_split = [0] * world
    out_split = [my_ops if r == 0 else 0 for r in range(world)]
    recv = torch.empty((my_ops, W), dtype=torch.int64, device=device)
    dist.all_to_all_single(recv, send, out_split, in_split)
    del send
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    tm["rebalance_ms"] = (time.perf_counter() - t0) * 1e3
    tm["rebalance_bytes"] = int(per_rank_ops.sum()) * (REC_BYTES + 2 * L)

    # -- this rank's engine, sized exactly; the received rows become its resident batch
    eng = rank_engine(engine_factory, owned, ops, caps, sums, recv.data_ptr() if my_ops else 0, L, props, names, tm)
    del recv
    return ShardedReplay(eng, owned, ops, owner, tm, cli)


def rank_shares(device, engine_factory, docs_total: int, world: int, seed: int, gen_params_cls, gen_kw: dict,
                props=None, names=None, chunk_docs: int = 131072):
    """Every rank's share of the N = `world` LPT plan, one after another on this one device
    (review item: all eight shares of north_star's 1,048,576-document plan on hardware without an
    8-GPU node).  This process plays rank 0 (generation into the send buffer) and then each rank in
    turn: rank r's rows are the send buffer's slice for r, exactly what all_to_all_single
    delivers to r.  Yields (r, ShardedReplay) with one engine alive at a time."""
    import torch
    L = int(gen_kw["ins_len_max"])
    ops = zipf_op_counts(docs_total, seed)
    cli = clients_per_doc(docs_total, seed)
    plan = SharePlan(ops, world)
    W = REC_BYTES // 8 + 2 * L // 8
    t0 = time.perf_counter()
    send, caps_t, cs_t = generate_send_rows(device, engine_factory, plan, cli, seed, gen_params_cls, gen_kw,
                                            props, names, chunk_docs, W)
    gen_s = time.perf_counter() - t0
    caps = caps_t.cpu().numpy()
    sums = cs_t.cpu().numpy().view(np.uint64)
    for r in range(world):
        tm = {"generate_s": gen_s, "rebalance_bytes": int(plan.per_rank_ops[r]) * (REC_BYTES + 2 * L)}
        owned = plan.owned(r)
        a, b = int(plan.rank_row0[r]), int(plan.rank_row0[r + 1])
        recv = send[a:b]
        eng = rank_engine(engine_factory, owned, ops, caps, sums, recv.data_ptr() if b > a else 0, L, props, names, tm)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        sh = ShardedReplay(eng, owned, ops, plan.owner, tm, cli)
        yield r, sh
        eng.close()
