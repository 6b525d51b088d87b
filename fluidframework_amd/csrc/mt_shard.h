// mt_shard.h — document exchange rows for multi-GPU sharding.
//
// A document moves between GPUs as rows, one per op: its 32-byte mt_op_rec, then its
// payload slot of L UTF-16 units (the fixed stride the generator and the resident batch
// use), so one all_to_all_single moves records and text together.  The sender packs each
// document's rows at the offset the LPT plan gives it in the send buffer (no separate
// permutation pass), and both ends compute a per-document 64-bit checksum of the rows:
// the receiver unpacks them into the resident batch and flags every document whose rows
// do not sum to the sender's value, so a corrupted exchange cannot replay silently.
#pragma once
#include "mt_core.h"

MT_INLINE unsigned long long mt_mix64(unsigned long long z) {          // splitmix64 finalizer
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ULL;
    z ^= z >> 27; z *= 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
// Word k of a document's rows contributes mix(w ^ k * golden): order-insensitive to sum
// (lanes accumulate independently), sensitive to every bit and to the word's position.
MT_INLINE unsigned long long mt_row_word_hash(unsigned long long w, unsigned long long k) {
    return mt_mix64(w ^ (k * 0x9E3779B97F4A7C15ULL));
}

// Sender: run `run` of a generated batch (ops.op_off, payload at op index * L) into rows
// starting at row dst_row; returns the document's checksum (every lane holds it).
MT_HD unsigned long long mt_pack_rows_doc(const MtOps& ops, uint32_t run, uint32_t L, unsigned long long dst_row,
                                          unsigned long long* rows) {
    const unsigned long long o0 = ops.op_off[run], n = (unsigned long long)ops.op_off[run + 1] - o0;
    const unsigned long long W = 4 + L / 4;                       // 8-byte words per row
    const unsigned long long* rec = (const unsigned long long*)ops.rec;
    const unsigned long long* pay = (const unsigned long long*)ops.payload;
    unsigned long long* out = rows + dst_row * W;
    auto acc = wave_map(MT_WAVE, [&](int) MT_LAM { return 0ull; });
    for (unsigned long long base = 0; base < n * W; base += MT_WAVE) {
        const int m = (n * W - base) < MT_WAVE ? (int)(n * W - base) : MT_WAVE;
        acc = wave_map(MT_WAVE, [&](int k) MT_LAM {
            unsigned long long a = own(acc, k);
            if (k < m) {
                const unsigned long long q = base + (unsigned long long)k, j = q / W, t = q % W;
                const unsigned long long w = t < 4 ? rec[(o0 + j) * 4 + t] : pay[(o0 + j) * (L / 4) + (t - 4)];
                out[q] = w;
                a += mt_row_word_hash(w, q);
            }
            return a;
        });
    }
    return wave_sum64(acc);
}

// Receiver: rows [op_off[run], op_off[run+1]) into the resident batch (records and
// payload slots; payload_off rewritten to the op's slot relative to the run's payload base,
// op_off[run] * L, which ops.pay_base holds); returns the checksum of the rows as received.
MT_HD unsigned long long mt_unpack_rows_doc(const MtOps& ops, uint32_t run, uint32_t L, const unsigned long long* rows) {
    const unsigned long long o0 = ops.op_off[run], n = (unsigned long long)ops.op_off[run + 1] - o0;
    const unsigned long long W = 4 + L / 4;
    unsigned long long* rec = (unsigned long long*)ops.rec;
    unsigned long long* pay = (unsigned long long*)ops.payload;
    const unsigned long long* in = rows + o0 * W;
    auto acc = wave_map(MT_WAVE, [&](int) MT_LAM { return 0ull; });
    for (unsigned long long base = 0; base < n * W; base += MT_WAVE) {
        const int m = (n * W - base) < MT_WAVE ? (int)(n * W - base) : MT_WAVE;
        acc = wave_map(MT_WAVE, [&](int k) MT_LAM {
            unsigned long long a = own(acc, k);
            if (k < m) {
                const unsigned long long q = base + (unsigned long long)k, j = q / W, t = q % W;
                unsigned long long w = in[q];
                a += mt_row_word_hash(w, q);
                if (t < 4) {
                    // word 3 holds payload_off (low half) and payload_len | prop_id (high half);
                    // only a text insert's payload_off is a payload slot (markers and register
                    // ops keep their ids there)
                    if (t == 3) {
                        const unsigned long long w0 = in[j * W];
                        const uint32_t ty = (uint32_t)(w0 & 0xFF), fl = (uint32_t)((w0 >> 8) & 0xFF);
                        if (ty == MT_OP_INSERT && !(fl & MT_OPF_MARKER))
                            w = (w & 0xFFFFFFFF00000000ULL) | (unsigned long long)(uint32_t)(j * L);
                    }
                    rec[(o0 + j) * 4 + t] = w;
                } else pay[(o0 + j) * (L / 4) + (t - 4)] = w;
            }
            return a;
        });
    }
    return wave_sum64(acc);
}
