// sanitize_driver.cpp — TEST-ONLY: the engine's host emulation (mt_emu.cpp, the product's
// engine logic compiled for the host) run under AddressSanitizer + UndefinedBehaviorSanitizer
// as a standalone executable (the sanitizer runtimes come first in its own link order; a
// Python process cannot load an ASan library properly).  Streams come from the oracle's
// generator (oracle/mtoracle.cpp ora_generate_doc), every residency mode replays them, and
// each document's SnapshotV1 digest, legacy snapshot and text must equal the oracle's.
// Build + run: tests/emu/sanitize.sh (any sanitizer report aborts with a non-zero status).
#include "mt_emu.cpp"
#include "../../oracle/mtoracle.h"

#include <stdio.h>
#include <string>
#include <vector>

struct Props {                                     // a small interned prop table (bench.ann_props-like)
    std::vector<uint32_t> off{0};
    std::vector<uint16_t> key; std::vector<int32_t> val;
    std::vector<const char*> kj{"\"k0\"", "\"k1\"", "\"k2\"", "\"3\""};
    std::vector<uint32_t> kidx{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 3};
    std::vector<std::string> vs{"\"s0\"", "\"\"", "1", "0", "{\"a\":[1,2]}", "2.5"};
    std::vector<const char*> vj;
    std::vector<uint8_t> falsy{0, 1, 0, 1, 0, 0}, kind{0, 0, 1, 1, 0, 1};
    std::vector<uint32_t> cls{0, 1, 2, 3, 4, 5};
    std::vector<int32_t> incr;                        // value_incr: String(v) + "undefined" chains
    mt_prop_table t{};
    Props() {
        for (int s = 0; s < 24; s++) {
            const int n = 1 + s % 3;
            for (int i = 0; i < n; i++) { key.push_back((uint16_t)((s + i) % 4)); val.push_back(((s * 7 + i) % 7) - 1); }
            off.push_back((uint32_t)key.size());
        }
        // combine sets (the combining-op scenario): NaN, a fresh consensus object, undefined
        for (int code : {MT_VAL_NAN, MT_VAL_CFRESH, MT_VAL_UNDEF}) {
            key.push_back(1); val.push_back(code); key.push_back(2); val.push_back(code == MT_VAL_NAN ? 0 : 4);
            off.push_back((uint32_t)key.size());
        }
        // incr of the held strings: "s0" -> "s0undefined" -> ..., "" -> "undefined" -> ..., the
        // object (and a fresh consensus object) -> "[object Object]undefined" -> ..., 40 deep
        incr.assign(vs.size(), MT_VAL_UNSUP);
        auto chain = [&](int v, std::string base) {
            for (int d = 0; d < 40; d++) {
                base += "undefined";
                const int w = (int)vs.size();
                vs.push_back("\"" + base + "\""); falsy.push_back(0); kind.push_back(0); cls.push_back((uint32_t)w);
                incr.push_back(MT_VAL_UNSUP);
                incr[v] = w; v = w;
            }
        };
        chain(0, "s0"); chain(1, ""); chain(4, "[object Object]");
        incr_object = incr[4];
        for (auto& x : vs) vj.push_back(x.c_str());
        t.n_sets = (uint32_t)off.size() - 1; t.set_off = off.data(); t.key = key.data(); t.value = val.data();
        t.n_keys = (uint32_t)kj.size(); t.key_json = kj.data(); t.key_index = kidx.data();
        t.n_values = (uint32_t)vj.size(); t.value_json = vj.data(); t.value_falsy = falsy.data(); t.value_class = cls.data();
        t.value_kind = kind.data(); t.value_incr = incr.data(); t.incr_object = incr_object;
    }
    int incr_object = MT_VAL_UNSUP;
};

// size_class: runs of at least this many messages in the wide block-residency kernel
// (mt_set_size_class; MT_RES_BLKW); combine: annotates turned into incr / consensus / other-name
// combining ops (expected digests and status words from the oracle's replay of the same batch)
struct Scenario { const char* name; uint32_t docs, ops, clients, lag, ins, rem, ins_len, rem_len, rewrite; int residency; int lds_blks; bool capture;
                  uint32_t size_class = 0; bool combine = false; };

static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { fprintf(stderr, "FAIL %s: ", sc.name); fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); fails++; } } while (0)

static void run(const Scenario& sc, Props& P) {
    mt_gen_params p{};
    p.seed = 0x5EED ^ sc.ops; p.n_docs = sc.docs; p.ops_per_doc = sc.ops; p.clients = sc.clients; p.lag_max = sc.lag;
    p.pct_insert = sc.ins; p.pct_remove = sc.rem; p.ins_len_max = sc.ins_len; p.rem_len_max = sc.rem_len;
    p.n_ann_sets = 24; p.pct_rewrite = sc.rewrite;
    const uint32_t n = sc.docs, k = sc.ops;
    std::vector<uint8_t> type(n * k), flags(n * k); std::vector<uint16_t> client(n * k), payload((size_t)n * k * sc.ins_len + 1);
    std::vector<int32_t> seq(n * k), ref(n * k), msn(n * k), p1(n * k), p2(n * k), pid(n * k);
    std::vector<uint32_t> poff(n * k), plen(n * k), off(n + 1), ids(n);
    std::vector<ora_doc*> kept(n);
    uint32_t pbase = 0;
    for (uint32_t d = 0; d < n; d++) {
        const size_t o = (size_t)d * k;
        uint32_t st = ora_generate_doc(&p, d, &P.t, &type[o], &flags[o], &client[o], &seq[o], &ref[o], &msn[o], &p1[o], &p2[o],
                                       &poff[o], &plen[o], &pid[o], &payload[pbase], pbase, &kept[d]);
        CHECK(st == 0, "oracle generation status %#x (doc %u)", st, d);
        for (uint32_t i = 0; i < k; i++) pbase += plen[o + i];
        off[d + 1] = (uint32_t)(o + k); ids[d] = d;
    }
    if (sc.size_class) {                              // ragged runs: every other document's tail cut off
        uint32_t w = 0;
        std::vector<uint32_t> noff(n + 1, 0);
        for (uint32_t d = 0; d < n; d++) {
            const uint32_t keep = d % 2 ? k / 4 : k;
            for (uint32_t i = 0; i < keep; i++) {
                const size_t a = (size_t)d * k + i;
                type[w] = type[a]; flags[w] = flags[a]; client[w] = client[a]; seq[w] = seq[a]; ref[w] = ref[a]; msn[w] = msn[a];
                p1[w] = p1[a]; p2[w] = p2[a]; poff[w] = poff[a]; plen[w] = plen[a]; pid[w] = pid[a]; w++;
            }
            noff[d + 1] = w;
        }
        off = noff;
    }
    const uint32_t NOPS = off[n];
    if (sc.combine) {                                 // a third each: incr, consensus, another name
        const int base = 24;
        for (uint32_t i = 0; i < NOPS; i++) {
            if (type[i] != MT_OP_ANNOTATE) continue;
            const uint32_t h = (seq[i] * 2654435761u) >> 28;
            if (h < 4) continue;                                               // some stay plain sets
            const int kind_ = (int)(h % 3);
            flags[i] = (uint8_t)((flags[i] & MT_OPF_END_OF_MSG) | MT_OPF_COMBINE |
                                 (kind_ ? MT_OPF_REWRITE : 0) | (kind_ == 1 ? MT_OPF_CONSENSUS : 0));
            if (h % 2) pid[i] = base + (int)(h % 3);                           // a combine set, else a plain one
        }
    }
    mt_op_batch b{};
    b.n_runs = n; b.doc_ids = ids.data(); b.op_offsets = off.data(); b.n_ops = NOPS; b.type = type.data(); b.flags = flags.data();
    b.client = client.data(); b.seq = seq.data(); b.ref_seq = ref.data(); b.msn = msn.data(); b.pos1 = p1.data(); b.pos2 = p2.data();
    b.payload_off = poff.data(); b.payload_len = plen.data(); b.prop_id = pid.data(); b.payload = payload.data(); b.payload_units = pbase;
    mt_limits L{}; L.max_docs = n; L.rows_per_doc = 3 * k + 64; L.blocks_per_doc = k + 64; L.heap_per_doc = 2 * k + 64;
    L.window_per_doc = 64 * sc.lag + 2048; L.text_per_doc = k * sc.ins_len + 4096; L.propsets_per_doc = 2 * k + 64;
    mt_ctx* c = nullptr;
    CHECK(emu_create(0, &L, &c) == MT_OK, "create");
    CHECK(emu_set_props(c, &P.t) == MT_OK, "set_props");
    std::vector<std::string> names; std::vector<const char*> np;
    for (int i = 0; i < 64; i++) names.push_back("\"c" + std::to_string(i) + "\"");
    for (auto& s : names) np.push_back(s.c_str());
    emu_set_client_names(c, 64, np.data());
    emu_set_residency(c, sc.residency, 0, sc.residency == 3 ? 0 : sc.lds_blks, 0);
    if (sc.size_class) emu_set_size_class(c, sc.size_class);
    if (sc.capture) emu_delta_capture(c, 1 << 12);
    CHECK(emu_docs_open(c, 0, n) == MT_OK, "open");
    CHECK(emu_apply_batch(c, &b) == MT_OK, "apply");
    emu_sync(c);
    std::vector<uint32_t> st(n);
    emu_doc_status(c, n, ids.data(), st.data());
    std::vector<int32_t> neg(n, -1);
    std::vector<uint64_t> dig(n);
    const char* arena; const uint64_t* boff; const uint32_t* bfirst;
    CHECK(emu_snapshot_v1(c, n, ids.data(), neg.data(), neg.data(), dig.data(), &arena, &boff, &bfirst) == MT_OK, "snapshot");
    std::vector<uint64_t> legacy(n);
    CHECK(emu_snapshot_legacy(c, n, ids.data(), neg.data(), neg.data(), legacy.data(), &arena, &boff, &bfirst) == MT_OK, "legacy");
    const uint16_t* txt; const uint64_t* toff;
    CHECK(emu_get_text(c, n, ids.data(), &txt, &toff) == MT_OK, "text");
    if (sc.size_class || sc.combine) {                // the oracle's replay of this batch
        std::vector<uint64_t> odg(n); std::vector<uint32_t> ost(n);
        ora_replay_batch(&b, &P.t, 1, odg.data(), ost.data(), nullptr);
        int combined = 0;
        for (uint32_t i = 0; i < NOPS; i++) combined += (flags[i] & MT_OPF_COMBINE) != 0;
        for (uint32_t d = 0; d < n; d++) {
            CHECK(st[d] == ost[d], "doc %u status %#x vs oracle %#x", d, st[d], ost[d]);
            CHECK(st[d] != 0 || dig[d] == odg[d], "doc %u SnapshotV1 digest vs oracle", d);
            ora_free(kept[d]);
        }
        if (sc.combine) CHECK(combined > 100, "only %d combining annotates", combined);
        uint32_t clean = 0;
        for (uint32_t d = 0; d < n; d++) clean += st[d] == 0;
        CHECK(clean == n, "%u of %u documents with a status word", n - clean, n);
        emu_destroy(c);
        fprintf(stderr, "%-28s %u docs x %u msgs (%d combining annotates): %s\n", sc.name, n, k, combined,
                fails ? "FAILED" : "ok");
        return;
    }
    for (uint32_t d = 0; d < n; d++) {
        CHECK(st[d] == 0, "doc %u status %#x", d, st[d]);
        const size_t last = (size_t)d * k + k - 1;
        uint64_t od = 0, ol = 0, tot = 0;
        ora_free_buf(ora_snapshot_v1(kept[d], msn[last], seq[last], &od, &tot));
        ora_free_buf(ora_snapshot_legacy(kept[d], msn[last], seq[last], &ol, &tot));
        CHECK(dig[d] == od, "doc %u SnapshotV1 digest %016llx vs oracle %016llx", d, (unsigned long long)dig[d], (unsigned long long)od);
        CHECK(legacy[d] == ol, "doc %u legacy digest", d);
        uint64_t nt = 0;
        uint16_t* ot = ora_get_text(kept[d], &nt);
        CHECK(nt == toff[d + 1] - toff[d] && !memcmp(ot, txt + toff[d], 2 * nt), "doc %u text", d);
        ora_free_buf(ot);
        ora_free(kept[d]);
    }
    emu_destroy(c);
    fprintf(stderr, "%-28s %u docs x %u msgs: %s\n", sc.name, n, k, fails ? "FAILED" : "ok");
}

int main() {
    Props P;
    const Scenario S[] = {
        {"config2-like blk", 6, 3000, 8, 32, 60, 40, 8, 8, 0, 2, 0, false},
        {"config3-like blk annotate", 6, 3000, 8, 4, 30, 30, 8, 16, 5, 2, 0, false},
        {"blk forced hand-over", 3, 3000, 8, 32, 60, 40, 8, 8, 0, 2, 24, false},
        {"hbm", 3, 2000, 8, 32, 55, 30, 8, 8, 5, 0, 0, false},
        {"lds forced hand-over", 3, 2000, 4, 16, 55, 30, 8, 8, 5, 1, 24, false},
        {"big long docs", 2, 12000, 8, 512, 60, 30, 8, 8, 5, 3, 0, false},
        {"capture (FULL kernels)", 3, 2000, 6, 32, 50, 30, 8, 8, 5, 2, 0, true},
        {"wide blk (size classes)", 6, 3000, 8, 32, 60, 40, 8, 8, 0, 2, 0, false, 1500, false},
        {"combining annotates", 6, 3000, 8, 8, 30, 30, 8, 16, 5, 2, 0, false, 0, true},
        {"combining annotates, wide blk", 4, 3000, 8, 8, 30, 30, 8, 16, 5, 2, 0, false, 1000, true},
    };
    for (const auto& s : S) run(s, P);
    if (fails) { fprintf(stderr, "%d checks failed\n", fails); return 1; }
    fprintf(stderr, "sanitize_driver: every scenario equal to the oracle, no sanitizer report\n");
    return 0;
}
