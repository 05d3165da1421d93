// lzma_alone.cpp -- LZMA-alone (.lzma) encoder for the GTM keyframe streams (host code in libANN.so).
//
// Replaces the reference's LZCompress (extern.pas:202-240), which writes the keyframe command stream to
// a temp file and runs the external `lzma.exe e src dst -lc8 -eos` (an LZMA SDK build that is not in the
// reference tree).  Output format (the LZMA SDK's "alone" format, read by the reference JS player's
// decodeHeader, decoders/htmljs/lzma.js:405-457): properties byte (pb * 5 + lp) * 9 + lc, dictionary
// size (u32 LE), uncompressed size (u64 LE, all ones with an end marker), then the range-coded body.
//
// The coder follows the published LZMA bitstream: 11-bit adaptive probabilities, 12-state machine,
// literals in (prev byte >> (8 - lc), pos & lp_mask) contexts (matched literals after a match), length
// coders with low/mid/high trees per pos state, 6-bit distance slots per length state + reverse trees
// + direct bits + 4 align bits, rep0..rep3 and short rep, end marker = distance 0xFFFFFFFF.  Parsing is
// greedy with one step of lazy evaluation over hash chains (3-byte hash); any valid parse decodes to the
// same bytes, so the output differs from lzma.exe's bytes but not in what a decoder returns.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "tiler_common.hpp"

namespace {

constexpr int kBits = 11, kMove = 5;
constexpr uint16_t kInit = 1 << (kBits - 1);
constexpr int kStates = 12, kPosBitsMax = 4, kLenToPosStates = 4, kAlignBits = 4;
constexpr int kEndPosModel = 14, kFullDistances = 128;
constexpr int kMinLen = 2, kMaxLen = 273;

struct RangeEnc {
    std::vector<uint8_t> out;
    uint64_t low = 0;
    uint32_t range = 0xFFFFFFFFu;
    uint8_t cache = 0;
    uint64_t cache_size = 1;

    void shift_low() {
        if ((uint32_t)low < 0xFF000000u || (low >> 32) != 0) {
            uint8_t carry = (uint8_t)(low >> 32);
            uint8_t temp = cache;
            do {
                out.push_back((uint8_t)(temp + carry));
                temp = 0xFF;
            } while (--cache_size != 0);
            cache = (uint8_t)(low >> 24);
        }
        cache_size++;
        low = (low & 0x00FFFFFFu) << 8;
    }
    void bit(uint16_t &p, int b) {
        const uint32_t bound = (range >> kBits) * p;
        if (!b) {
            range = bound;
            p += (uint16_t)(((1 << kBits) - p) >> kMove);
        } else {
            low += bound;
            range -= bound;
            p -= (uint16_t)(p >> kMove);
        }
        while (range < (1u << 24)) {
            range <<= 8;
            shift_low();
        }
    }
    void direct(uint32_t v, int n) {
        for (int i = n - 1; i >= 0; i--) {
            range >>= 1;
            if ((v >> i) & 1) low += range;
            while (range < (1u << 24)) {
                range <<= 8;
                shift_low();
            }
        }
    }
    void flush() {
        for (int i = 0; i < 5; i++) shift_low();
    }
};

// bit tree of nbits, MSB first (probs[1 .. 2^nbits - 1])
void tree(RangeEnc &rc, uint16_t *probs, int nbits, uint32_t v) {
    uint32_t m = 1;
    for (int i = nbits - 1; i >= 0; i--) {
        const int b = (v >> i) & 1;
        rc.bit(probs[m], b);
        m = (m << 1) | b;
    }
}
// reverse bit tree, LSB first
void tree_rev(RangeEnc &rc, uint16_t *probs, int nbits, uint32_t v) {
    uint32_t m = 1;
    for (int i = 0; i < nbits; i++) {
        const int b = v & 1;
        v >>= 1;
        rc.bit(probs[m], b);
        m = (m << 1) | b;
    }
}

struct LenEnc {
    uint16_t choice = kInit, choice2 = kInit;
    uint16_t low[1 << kPosBitsMax][8], mid[1 << kPosBitsMax][8], high[256];
    LenEnc() {
        for (auto &a : low) for (auto &p : a) p = kInit;
        for (auto &a : mid) for (auto &p : a) p = kInit;
        for (auto &p : high) p = kInit;
    }
    void encode(RangeEnc &rc, uint32_t len, int pos_state) {  // len >= kMinLen
        len -= kMinLen;
        if (len < 8) {
            rc.bit(choice, 0);
            tree(rc, low[pos_state], 3, len);
        } else if (len < 16) {
            rc.bit(choice, 1);
            rc.bit(choice2, 0);
            tree(rc, mid[pos_state], 3, len - 8);
        } else {
            rc.bit(choice, 1);
            rc.bit(choice2, 1);
            tree(rc, high, 8, len - 16);
        }
    }
};

struct Encoder {
    int lc, lp, pb;
    uint32_t dict;
    RangeEnc rc;
    std::vector<uint16_t> lit;
    uint16_t is_match[kStates][1 << kPosBitsMax], is_rep[kStates], is_rep_g0[kStates], is_rep_g1[kStates],
        is_rep_g2[kStates], is_rep0_long[kStates][1 << kPosBitsMax];
    uint16_t pos_slot[kLenToPosStates][64], pos_special[kFullDistances], align[1 << kAlignBits];
    LenEnc len_enc, rep_len_enc;
    int state = 0;
    uint32_t rep[4] = {0, 0, 0, 0};

    Encoder(int lc_, int lp_, int pb_, uint32_t d) : lc(lc_), lp(lp_), pb(pb_), dict(d) {
        lit.assign((size_t)0x300 << (lc + lp), kInit);
        for (auto &a : is_match) for (auto &p : a) p = kInit;
        for (auto &a : is_rep0_long) for (auto &p : a) p = kInit;
        for (int i = 0; i < kStates; i++) is_rep[i] = is_rep_g0[i] = is_rep_g1[i] = is_rep_g2[i] = kInit;
        for (auto &a : pos_slot) for (auto &p : a) p = kInit;
        for (auto &p : pos_special) p = kInit;
        for (auto &p : align) p = kInit;
    }

    void literal(const uint8_t *buf, size_t pos) {
        const int ps = (int)(pos & ((1u << pb) - 1));
        rc.bit(is_match[state][ps], 0);
        const uint8_t prev = pos ? buf[pos - 1] : 0;
        uint16_t *probs = &lit[(size_t)0x300 * ((((uint32_t)pos & ((1u << lp) - 1)) << lc) + (prev >> (8 - lc)))];
        const uint32_t sym = buf[pos];
        if (state < 7) {
            tree(rc, probs, 8, sym);
        } else {  // matched literal: the byte at rep0 steers the tree until the first differing bit
            uint32_t match_byte = buf[pos - rep[0] - 1];
            uint32_t offs = 0x100, m = 1;
            for (int i = 7; i >= 0; i--) {
                const int b = (sym >> i) & 1;
                match_byte <<= 1;
                const uint32_t match_bit = match_byte & offs;
                rc.bit(probs[offs + match_bit + m], b);
                m = (m << 1) | b;
                offs &= b ? match_bit : ~match_bit;
            }
        }
        state = state < 4 ? 0 : state < 10 ? state - 3 : state - 6;
    }

    void distance(uint32_t dist, uint32_t len) {
        const int ls = (int)(len - kMinLen < kLenToPosStates - 1 ? len - kMinLen : kLenToPosStates - 1);
        uint32_t slot;
        if (dist < 4) {
            slot = dist;
        } else {
            int nb = 31 - __builtin_clz(dist);
            slot = (uint32_t)(nb * 2) + ((dist >> (nb - 1)) & 1);
        }
        tree(rc, pos_slot[ls], 6, slot);
        if (slot >= 4) {
            const int footer = (int)(slot >> 1) - 1;
            const uint32_t base = (2 | (slot & 1)) << footer;
            const uint32_t red = dist - base;
            if (slot < kEndPosModel) {
                tree_rev(rc, pos_special + base - slot - 1, footer, red);
            } else {
                rc.direct(red >> kAlignBits, footer - kAlignBits);
                tree_rev(rc, align, kAlignBits, red & ((1u << kAlignBits) - 1));
            }
        }
    }

    void match(size_t pos, uint32_t dist, uint32_t len) {  // dist = back distance - 1
        const int ps = (int)(pos & ((1u << pb) - 1));
        rc.bit(is_match[state][ps], 1);
        rc.bit(is_rep[state], 0);
        len_enc.encode(rc, len, ps);
        distance(dist, len);
        rep[3] = rep[2];
        rep[2] = rep[1];
        rep[1] = rep[0];
        rep[0] = dist;
        state = state < 7 ? 7 : 10;
    }

    void rep_match(size_t pos, int r, uint32_t len) {
        const int ps = (int)(pos & ((1u << pb) - 1));
        rc.bit(is_match[state][ps], 1);
        rc.bit(is_rep[state], 1);
        if (r == 0) {
            rc.bit(is_rep_g0[state], 0);
            rc.bit(is_rep0_long[state][ps], 1);
        } else {
            rc.bit(is_rep_g0[state], 1);
            if (r == 1) {
                rc.bit(is_rep_g1[state], 0);
            } else {
                rc.bit(is_rep_g1[state], 1);
                rc.bit(is_rep_g2[state], r == 3);
            }
            const uint32_t d = rep[r];
            for (int i = r; i > 0; i--) rep[i] = rep[i - 1];
            rep[0] = d;
        }
        rep_len_enc.encode(rc, len, ps);
        state = state < 7 ? 8 : 11;
    }

    void short_rep(size_t pos) {
        const int ps = (int)(pos & ((1u << pb) - 1));
        rc.bit(is_match[state][ps], 1);
        rc.bit(is_rep[state], 1);
        rc.bit(is_rep_g0[state], 0);
        rc.bit(is_rep0_long[state][ps], 0);
        state = state < 7 ? 9 : 11;
    }

    void end_marker(size_t pos) {
        const int ps = (int)(pos & ((1u << pb) - 1));
        rc.bit(is_match[state][ps], 1);
        rc.bit(is_rep[state], 0);
        len_enc.encode(rc, kMinLen, ps);
        tree(rc, pos_slot[0], 6, 63);
        rc.direct((1u << 26) - 1, 26);
        tree_rev(rc, align, kAlignBits, (1u << kAlignBits) - 1);
    }
};

// hash-chain match finder over the whole input (the window is the dictionary)
struct MatchFinder {
    const uint8_t *buf;
    size_t n;
    uint32_t dict;
    std::vector<int64_t> head, prev;
    static constexpr int kHashBits = 18, kDepth = 24, kNice = 128;

    MatchFinder(const uint8_t *b, size_t nn, uint32_t d) : buf(b), n(nn), dict(d) {
        head.assign((size_t)1 << kHashBits, -1);
        prev.assign(nn ? nn : 1, -1);
    }
    uint32_t hash(size_t p) const {
        return ((uint32_t)buf[p] * 0x9E3779B1u ^ (uint32_t)buf[p + 1] * 0x85EBCA77u ^ (uint32_t)buf[p + 2] * 0xC2B2AE3Du) >>
               (32 - kHashBits);
    }
    void insert(size_t p) {
        if (p + 3 > n) return;
        const uint32_t h = hash(p);
        prev[p] = head[h];
        head[h] = (int64_t)p;
    }
    uint32_t match_len(size_t a, size_t b, uint32_t lim) const {
        uint32_t l = 0;
        while (l < lim && buf[a + l] == buf[b + l]) l++;
        return l;
    }
    // longest match at p (not yet inserted): returns len (0 if < kMinLen) and back distance - 1
    uint32_t best(size_t p, uint32_t &dist) const {
        if (p + 3 > n) return 0;
        const uint32_t lim = (uint32_t)std::min<size_t>(kMaxLen, n - p);
        uint32_t bl = 0;
        int64_t c = head[hash(p)];
        for (int d = 0; d < kDepth && c >= 0; d++, c = prev[(size_t)c]) {
            const size_t back = p - (size_t)c;
            if (back > dict) break;
            if (buf[(size_t)c + bl] != buf[p + bl]) continue;
            const uint32_t l = match_len((size_t)c, p, lim);
            if (l > bl) {
                bl = l;
                dist = (uint32_t)(back - 1);
                if (l >= kNice || l == lim) break;
            }
        }
        return bl >= (uint32_t)kMinLen ? bl : 0;
    }
};

}  // namespace

extern "C" int tiler_lzma_encode(const uint8_t *src, size_t n, int lc, int lp, int pb, uint32_t dict_size, int eos,
                                 uint8_t *dst, size_t cap, size_t *out_len) {
    if ((!src && n) || !out_len || lc < 0 || lc > 8 || lp < 0 || lp > 4 || pb < 0 || pb > 4 || dict_size < 4096) {
        tiler::set_error("tiler_lzma_encode: bad arguments (lc 0..8, lp 0..4, pb 0..4, dict >= 4096)");
        return -1;
    }
    Encoder enc(lc, lp, pb, dict_size);
    std::vector<uint8_t> hdr(13);
    hdr[0] = (uint8_t)((pb * 5 + lp) * 9 + lc);
    for (int i = 0; i < 4; i++) hdr[1 + i] = (uint8_t)(dict_size >> (8 * i));
    for (int i = 0; i < 8; i++) hdr[5 + i] = eos ? 0xFF : (uint8_t)((uint64_t)n >> (8 * i));
    MatchFinder mf(src, n, dict_size);
    size_t p = 0;
    bool have_next = false;  // the lazy look-ahead of the previous position, reused when it won
    uint32_t next_len = 0, next_dist = 0;
    while (p < n) {
        const uint32_t lim = (uint32_t)std::min<size_t>(kMaxLen, n - p);
        // rep candidates
        uint32_t rl = 0;
        int ri = -1;
        for (int r = 0; r < 4; r++) {
            const size_t back = (size_t)enc.rep[r] + 1;
            if (back > p) continue;
            const uint32_t l = mf.match_len(p - back, p, lim);
            if (l > rl) {
                rl = l;
                ri = r;
            }
        }
        uint32_t md = 0, ml;
        if (have_next) {
            ml = next_len;
            md = next_dist;
            have_next = false;
        } else {
            ml = mf.best(p, md);
        }
        if (ml >= 2 && ml <= 3 && md >= (1u << 15)) ml = 0;  // short far matches cost more than literals
        // one step of lazy evaluation: a longer match at p + 1 wins over a normal match here
        if (ml && ml < 64 && rl + 1 < ml && p + 1 < n) {
            mf.insert(p);
            uint32_t d2 = 0;
            const uint32_t l2 = mf.best(p + 1, d2);
            if (l2 > ml + 1) {
                enc.literal(src, p);
                p++;
                have_next = true;  // p + 1 is searched already (nothing was inserted since)
                next_len = l2;
                next_dist = d2;
                continue;
            }
            // keep the match at p (already inserted)
            enc.match(p, md, ml);
            for (uint32_t k = 1; k < ml; k++) mf.insert(p + k);
            p += ml;
            continue;
        }
        if (ri >= 0 && rl >= 2 && rl + 1 >= ml) {
            enc.rep_match(p, ri, rl);
            for (uint32_t k = 0; k < rl; k++) mf.insert(p + k);
            p += rl;
        } else if (ml) {
            enc.match(p, md, ml);
            for (uint32_t k = 0; k < ml; k++) mf.insert(p + k);
            p += ml;
        } else if (p > enc.rep[0] && src[p] == src[p - enc.rep[0] - 1]) {
            enc.short_rep(p);
            mf.insert(p);
            p++;
        } else {
            enc.literal(src, p);
            mf.insert(p);
            p++;
        }
    }
    if (eos) enc.end_marker(p);
    enc.rc.flush();
    const size_t total = hdr.size() + enc.rc.out.size();
    *out_len = total;
    if (!dst) return 0;  // size query
    if (cap < total) {
        tiler::set_error("tiler_lzma_encode: output buffer too small (*out_len holds the size needed)");
        return -1;
    }
    std::memcpy(dst, hdr.data(), hdr.size());
    std::memcpy(dst + hdr.size(), enc.rc.out.data(), enc.rc.out.size());
    return 0;
}
