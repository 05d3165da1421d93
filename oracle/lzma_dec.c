/*
 * lzma_dec.c -- TEST INFRASTRUCTURE ONLY: LZMA-alone decoder restated from the published LZMA format
 * (the format the reference's LZCompress writes with `lzma.exe e ... -lc8 -eos`, extern.pas:202-240,
 * and its JS player reads, decoders/htmljs/lzma.js).  Used to check libANN.so's tiler_lzma_encode and
 * to read GTM files in tests.  Returns the decoded size, or -1 on a corrupt stream / -2 if out is too small.
 * `consumed` receives the compressed bytes used (header included), so concatenated streams can be walked.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "tiler_oracle.h"

typedef struct {
    const uint8_t *in;
    size_t n, pos;
    uint32_t range, code;
    int err;
} rdec;

static uint8_t rd_byte(rdec *r) {
    if (r->pos >= r->n) {
        r->err = 1;
        return 0;
    }
    return r->in[r->pos++];
}
static void rd_norm(rdec *r) {
    if (r->range < (1u << 24)) {
        r->range <<= 8;
        r->code = (r->code << 8) | rd_byte(r);
    }
}
static int rd_bit(rdec *r, uint16_t *p) {
    uint32_t bound = (r->range >> 11) * *p;
    int b;
    if (r->code < bound) {
        r->range = bound;
        *p += (uint16_t)((2048 - *p) >> 5);
        b = 0;
    } else {
        r->range -= bound;
        r->code -= bound;
        *p -= (uint16_t)(*p >> 5);
        b = 1;
    }
    rd_norm(r);
    return b;
}
static uint32_t rd_direct(rdec *r, int nb) {
    uint32_t v = 0;
    for (int i = 0; i < nb; i++) {
        r->range >>= 1;
        uint32_t t = (r->code >= r->range);
        if (t) r->code -= r->range;
        v = (v << 1) | t;
        rd_norm(r);
    }
    return v;
}
static uint32_t rd_tree(rdec *r, uint16_t *p, int nb) {
    uint32_t m = 1;
    for (int i = 0; i < nb; i++) m = (m << 1) | (uint32_t)rd_bit(r, &p[m]);
    return m - (1u << nb);
}
static uint32_t rd_tree_rev(rdec *r, uint16_t *p, int nb) {
    uint32_t m = 1, v = 0;
    for (int i = 0; i < nb; i++) {
        int b = rd_bit(r, &p[m]);
        m = (m << 1) | (uint32_t)b;
        v |= (uint32_t)b << i;
    }
    return v;
}

typedef struct {
    uint16_t choice, choice2, low[16][8], mid[16][8], high[256];
} lendec;
static void len_init(lendec *l) {
    uint16_t *p = (uint16_t *)l;
    for (size_t i = 0; i < sizeof(lendec) / 2; i++) p[i] = 1024;
}
static uint32_t len_dec(rdec *r, lendec *l, int ps) {
    if (!rd_bit(r, &l->choice)) return rd_tree(r, l->low[ps], 3);
    if (!rd_bit(r, &l->choice2)) return 8 + rd_tree(r, l->mid[ps], 3);
    return 16 + rd_tree(r, l->high, 8);
}

long or_lzma_decode(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *consumed) {
    if (n < 13) return -1;
    int props = in[0];
    if (props >= 9 * 5 * 5) return -1;
    const int lc = props % 9, lp = (props / 9) % 5, pb = props / 45;
    uint64_t usize = 0;
    for (int i = 0; i < 8; i++) usize |= (uint64_t)in[5 + i] << (8 * i);
    const int known = usize != UINT64_MAX;
    size_t lit_n = (size_t)0x300 << (lc + lp);
    uint16_t *lit = (uint16_t *)malloc(lit_n * 2);
    for (size_t i = 0; i < lit_n; i++) lit[i] = 1024;
    uint16_t is_match[12][16], is_rep[12], g0[12], g1[12], g2[12], rep0_long[12][16];
    uint16_t pos_slot[4][64], spec[128], align[16];
    lendec len_d, rep_len_d;
    for (int i = 0; i < 12; i++) {
        is_rep[i] = g0[i] = g1[i] = g2[i] = 1024;
        for (int j = 0; j < 16; j++) is_match[i][j] = rep0_long[i][j] = 1024;
    }
    for (int i = 0; i < 4; i++) for (int j = 0; j < 64; j++) pos_slot[i][j] = 1024;
    for (int i = 0; i < 128; i++) spec[i] = 1024;
    for (int i = 0; i < 16; i++) align[i] = 1024;
    len_init(&len_d);
    len_init(&rep_len_d);
    rdec r = {in, n, 13, 0xFFFFFFFFu, 0, 0};
    if (rd_byte(&r) != 0) {  /* the first range-coder byte is always 0 */
        free(lit);
        return -1;
    }
    for (int i = 0; i < 4; i++) r.code = (r.code << 8) | rd_byte(&r);
    uint32_t rep[4] = {0, 0, 0, 0};
    int state = 0;
    size_t op = 0;
    long ret = -1;
    for (;;) {
        if (known && op == usize) {
            ret = (long)op;
            break;
        }
        if (r.err) break;
        const int ps = (int)(op & ((1u << pb) - 1));
        if (!rd_bit(&r, &is_match[state][ps])) {
            const uint8_t prev = op ? out[op - 1] : 0;
            uint16_t *p = lit + 0x300 * (size_t)((((uint32_t)op & ((1u << lp) - 1)) << lc) + (prev >> (8 - lc)));
            uint32_t sym = 1;
            if (state >= 7) {
                if (op <= rep[0]) break;
                uint32_t mb = out[op - rep[0] - 1], offs = 0x100;
                while (sym < 0x100) {
                    mb <<= 1;
                    uint32_t mbit = mb & offs;
                    int b = rd_bit(&r, &p[offs + mbit + sym]);
                    sym = (sym << 1) | (uint32_t)b;
                    offs &= b ? mbit : ~mbit;
                }
            } else {
                while (sym < 0x100) sym = (sym << 1) | (uint32_t)rd_bit(&r, &p[sym]);
            }
            if (op >= cap) {
                ret = -2;
                break;
            }
            out[op++] = (uint8_t)sym;
            state = state < 4 ? 0 : state < 10 ? state - 3 : state - 6;
            continue;
        }
        uint32_t len;
        if (rd_bit(&r, &is_rep[state])) {
            if (op == 0) break;
            if (!rd_bit(&r, &g0[state])) {
                if (!rd_bit(&r, &rep0_long[state][ps])) {  /* short rep */
                    state = state < 7 ? 9 : 11;
                    if (op <= rep[0] || op >= cap) {
                        ret = op >= cap ? -2 : -1;
                        break;
                    }
                    out[op] = out[op - rep[0] - 1];
                    op++;
                    continue;
                }
            } else {
                uint32_t d;
                if (!rd_bit(&r, &g1[state])) {
                    d = rep[1];
                } else if (!rd_bit(&r, &g2[state])) {
                    d = rep[2];
                    rep[2] = rep[1];
                } else {
                    d = rep[3];
                    rep[3] = rep[2];
                    rep[2] = rep[1];
                }
                rep[1] = rep[0];
                rep[0] = d;
            }
            len = len_dec(&r, &rep_len_d, ps);
            state = state < 7 ? 8 : 11;
        } else {
            rep[3] = rep[2];
            rep[2] = rep[1];
            rep[1] = rep[0];
            len = len_dec(&r, &len_d, ps);
            state = state < 7 ? 7 : 10;
            const int ls = len < 3 ? (int)len : 3;
            const uint32_t slot = rd_tree(&r, pos_slot[ls], 6);
            uint32_t dist;
            if (slot < 4) {
                dist = slot;
            } else {
                const int footer = (int)(slot >> 1) - 1;
                dist = (2 | (slot & 1)) << footer;
                if (slot < 14) {
                    dist += rd_tree_rev(&r, spec + dist - slot - 1, footer);
                } else {
                    dist += rd_direct(&r, footer - 4) << 4;
                    dist += rd_tree_rev(&r, align, 4);
                }
            }
            if (dist == 0xFFFFFFFFu) {  /* end marker */
                ret = (r.err || (known && op != usize)) ? -1 : (long)op;
                break;
            }
            rep[0] = dist;
        }
        len += 2;
        if (op <= rep[0]) break;
        if (op + len > cap) {
            ret = -2;
            break;
        }
        for (uint32_t i = 0; i < len; i++, op++) out[op] = out[op - rep[0] - 1];
    }
    free(lit);
    if (consumed) *consumed = r.pos;
    return r.err ? -1 : ret;
}
