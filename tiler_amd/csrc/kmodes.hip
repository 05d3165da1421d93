// kmodes.hip -- GlobalTiling K-Modes (TKModes, kmodes.pas:46-1060) on gfx950.
//
// Exact restatement of what the reference executes on x86-64 (asm dissimilarity kmodes.pas:316-596,
// 960-point snapshot bins, incremental modes, Delphi-LCG empty-cluster rescue), so labels and
// centroids are bit-identical to the CPU oracle (itself pinned against the reference asm).
// Byte work, no floating point: the dissimilarity is evaluated on packed dwords with v_sad_u8 (L1 of
// bytes 16..79) and a SWAR nonzero-byte count (mismatches), never reshaped into a GEMM.
//   dis = 2048 * #mismatch(80 B) + W0 + W4,  W0 = (|i8(r0-x0)| + 256|i8(r1-x1)| + S_lo) mod 2^16, ...
// Phases (ComputeKModes kmodes.pas:917-1060):
//   farthest-first init  : K rounds of {min-distance update + block argmax} / {select}   (698-776)
//   initial assignment   : all points vs K centroids, argmin ties -> last  (packed u64 atomicMin)
//   modes                : attribute histograms (atomics), first-max mode, RandInt rows for empties
//   KModesIter           : per 960-point bin: parallel assignment vs the CURRENT centroids, then one
//                          workgroup applies the bin's moves in order (MovePointCat over 80 lanes,
//                          rescue with a workgroup-parallel argmax and ordered member selection)
// Batched over GlobalTiling's palette bins (DoKModes per bin, main.pas:4195-4254, run in parallel by
// ProcThreadPool at main.pas:4339): every phase is one launch for all still-running bins -- bins sorted by
// size so the bins alive in farthest-first round j are a prefix, work lists flattened over (bin, block),
// one sequential workgroup per bin -- so launch count follows the LARGEST bin, not the sum.  A single
// ComputeKModes call is a batch of one.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <vector>


#include "kmodes.hpp"

namespace tiler {

static constexpr int KM_A = 80;     // cKModesFeatureCount (kmodes.pas:15)
static constexpr int KM_BIN = 960;  // KModesIter cBinSize (kmodes.pas:847)

__device__ __forceinline__ unsigned abs_i8(unsigned r, unsigned x) {
    const int d = (int)(int8_t)(uint8_t)(r - x);  // psubb + pabsb
    return (unsigned)(d < 0 ? -d : d);
}

__device__ __forceinline__ unsigned nz_bytes(unsigned t) {  // number of non-zero bytes of t
    const unsigned m = (((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t) & 0x80808080u;
    return __popc(m);
}

// row = list entry (centroid / member), x = item (kmodes.pas:341-412)
__device__ __forceinline__ unsigned long long km_dissim(const uint32_t *__restrict__ r, const uint32_t *__restrict__ x) {
    unsigned mism = 0, slo = 0, shi = 0;
#pragma unroll
    for (int w = 0; w < 20; w++) mism += nz_bytes(r[w] ^ x[w]);
#pragma unroll
    for (int w = 4; w < 20; w += 4) {
        slo = __builtin_amdgcn_sad_u8(r[w], x[w], slo);
        slo = __builtin_amdgcn_sad_u8(r[w + 1], x[w + 1], slo);
        shi = __builtin_amdgcn_sad_u8(r[w + 2], x[w + 2], shi);
        shi = __builtin_amdgcn_sad_u8(r[w + 3], x[w + 3], shi);
    }
    const unsigned r0 = r[0], x0 = x[0], r2 = r[2], x2 = x[2];
    const unsigned w0 = (abs_i8(r0 & 255, x0 & 255) + 256u * abs_i8((r0 >> 8) & 255, (x0 >> 8) & 255) + slo) & 0xffffu;
    const unsigned w4 = (abs_i8(r2 & 255, x2 & 255) + 256u * abs_i8((r2 >> 8) & 255, (x2 >> 8) & 255) + shi) & 0xffffu;
    return ((unsigned long long)mism << 11) + w0 + w4;
}

__device__ __forceinline__ void load_row(const uint8_t *__restrict__ p, uint32_t (&w)[20]) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const uint4 v = q[i];
        w[4 * i] = v.x;
        w[4 * i + 1] = v.y;
        w[4 * i + 2] = v.z;
        w[4 * i + 3] = v.w;
    }
}

// RandInt kmodes.pas:82-86
__device__ __forceinline__ unsigned km_randint(unsigned range, unsigned *seed) {
    *seed = *seed * 0x08088405u + 1u;
    return (unsigned)(((unsigned long long)*seed * range) >> 32);
}

struct KmState {
    const uint8_t *X;  // [n][80], rows 16-byte aligned
    int n, K, M;
    int32_t *memb;
    uint8_t *cent;      // [K][80]
    int32_t *freq;      // [K][80][M]
    int32_t *csize;     // [K]
    unsigned long long *mind;  // [n]
    uint8_t *used;             // [n]
    unsigned long long *part;  // farthest-first partial argmax [nblk]
    int32_t *center;           // [K] chosen centre rows
    unsigned long long *akey;  // [n] packed (dis << 32) | ~idx for assignments
    unsigned *seed;
    unsigned long long *cost;  // [1]
    int *moves;                // [1]
    int *err;                  // [1]
    int *dbg;                  // [8] sequential-pass counters of the bin (study hook; null in the library)
    int4 *mvl;                 // [2 * KM_BIN] this chunk's moves in order (point, to, from, 1 = first of its group)
    int *mvn;                  // [1] their count
};

// ---- the sequential part of one bin (KModesIter kmodes.pas:869-911), one workgroup of KM_SEQ_NT ----
static constexpr int KM_SEQ_NT = 512;  // 32 moves of 16 lanes (round 2: 6 of 80 lanes; 320..1024 threads: 512 best)
static constexpr int KM_SEQ_W = 16;    // lanes per move: 5 attributes per lane
static constexpr int KM_CLASH_TAB = 8192;  // buckets of the move pass's cluster-clash table (power of two; exact for K <= 8192)

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long u = __shfl_xor(v, o, 64);
        v = u > v ? u : v;
    }
    return v;
}

// MovePointCat (kmodes.pas:778-806) for one point; lane a = attribute (0..79), lane 0 also updates the
// membership and the cluster sizes.
__device__ void move_point_cat(const KmState &s, int ip, int to, int from, int a) {
    if (a < KM_A) {
        const int cur = s.X[(long)ip * KM_A + a];
        int32_t *tc = s.freq + ((long)to * KM_A + a) * s.M;
        int32_t *fc = s.freq + ((long)from * KM_A + a) * s.M;
        tc[cur]++;
        uint8_t *ct = s.cent + (long)to * KM_A + a;
        if (tc[*ct] < tc[cur]) *ct = (uint8_t)cur;
        fc[cur]--;
        uint8_t *cf = s.cent + (long)from * KM_A + a;
        if (*cf == cur) {
            int bi = -1, bv = INT32_MIN;
            for (int m = 0; m < s.M; m++)
                if (fc[m] > bv) {
                    bv = fc[m];
                    bi = m;
                }
            *cf = (uint8_t)bi;
        }
    }
    if (a == 0) {
        s.memb[ip] = to;
        s.csize[to]++;
        s.csize[from]--;
    }
}

// The same MovePointCat with W lanes per move (W divides 80 into KM_A / W attributes per lane: a = l + W k).  Every
// attribute's update touches only its own count row and mode byte, so a lane's attributes are independent: their
// loads are issued together (one dependent round trip for all of them, not one per attribute), then the stores,
// then the mode checks that read the updated counts -- each attribute sees exactly the reads and writes of the
// sequential form.
// The attribute updates of MovePointCat (kmodes.pas:778-807) for the NA attributes a = a0 + l + W k of one lane, every
// load of a kind issued together (one dependent round trip for all of them), then the stores, then the mode rules on
// the updated counts; no membership / size updates (the decision pass made them).
template <int W, int NA>
__device__ __forceinline__ void apply_point_attrs(const KmState &s, int ip, int to, int from, int a0) {
    int cur[NA], tcv[NA], fcv[NA], ctv[NA], cfv[NA];
    int32_t *tc[NA], *fc[NA];
#pragma unroll
    for (int k = 0; k < NA; k++) cur[k] = s.X[(long)ip * KM_A + a0 + W * k];
#pragma unroll
    for (int k = 0; k < NA; k++) {
        const int a = a0 + W * k;
        tc[k] = s.freq + ((long)to * KM_A + a) * s.M;
        fc[k] = s.freq + ((long)from * KM_A + a) * s.M;
        tcv[k] = tc[k][cur[k]];
        fcv[k] = fc[k][cur[k]];
        ctv[k] = s.cent[(long)to * KM_A + a];
        cfv[k] = s.cent[(long)from * KM_A + a];
    }
#pragma unroll
    for (int k = 0; k < NA; k++) {
        tc[k][cur[k]] = tcv[k] + 1;
        fc[k][cur[k]] = fcv[k] - 1;
    }
    if (s.M == 16) {
        int tct[NA];
        int4 fr[NA][4];
#pragma unroll
        for (int k = 0; k < NA; k++) {
            tct[k] = ctv[k] == cur[k] ? tcv[k] + 1 : tc[k][ctv[k]];
            if (cfv[k] == cur[k]) {
                const int4 *r4 = reinterpret_cast<const int4 *>(fc[k]);  // 64-byte rows (M = 16)
#pragma unroll
                for (int q = 0; q < 4; q++) fr[k][q] = r4[q];
            }
        }
#pragma unroll
        for (int k = 0; k < NA; k++) {
            const int a = a0 + W * k;
            if (tct[k] < tcv[k] + 1) s.cent[(long)to * KM_A + a] = (uint8_t)cur[k];
            if (cfv[k] == cur[k]) {  // GetMaxValueIndex (kmodes.pas:149-161): first maximum
                const int v[16] = {fr[k][0].x, fr[k][0].y, fr[k][0].z, fr[k][0].w, fr[k][1].x, fr[k][1].y, fr[k][1].z, fr[k][1].w,
                                   fr[k][2].x, fr[k][2].y, fr[k][2].z, fr[k][2].w, fr[k][3].x, fr[k][3].y, fr[k][3].z, fr[k][3].w};
                int bi = 0, bv = v[0];
#pragma unroll
                for (int m = 1; m < 16; m++)
                    if (v[m] > bv) {
                        bv = v[m];
                        bi = m;
                    }
                s.cent[(long)from * KM_A + a] = (uint8_t)bi;
            }
        }
    } else
#pragma unroll
    for (int k = 0; k < NA; k++) {
        const int a = a0 + W * k;
        const int tct = ctv[k] == cur[k] ? tcv[k] + 1 : tc[k][ctv[k]];
        if (tct < tcv[k] + 1) s.cent[(long)to * KM_A + a] = (uint8_t)cur[k];
        if (cfv[k] == cur[k]) {
            int bi = -1, bv = INT32_MIN;
            for (int m = 0; m < s.M; m++) {
                const int v = fc[k][m];
                if (v > bv) {
                    bv = v;
                    bi = m;
                }
            }
            s.cent[(long)from * KM_A + a] = (uint8_t)bi;
        }
    }
}

// xrow: the point's row already staged in LDS (the move pass prefetches its candidates' rows), or nullptr
template <int W>
__device__ void move_point_cat_w(const KmState &s, int ip, int to, int from, int l, const uint8_t *xrow = nullptr) {
    constexpr int NA = KM_A / W;
    static_assert(KM_A % W == 0, "W must divide the attribute count");
    int cur[NA], tcv[NA], fcv[NA], ctv[NA], cfv[NA];
    int32_t *tc[NA], *fc[NA];
#pragma unroll
    for (int k = 0; k < NA; k++) cur[k] = xrow ? xrow[l + W * k] : s.X[(long)ip * KM_A + l + W * k];
#pragma unroll
    for (int k = 0; k < NA; k++) {
        const int a = l + W * k;
        tc[k] = s.freq + ((long)to * KM_A + a) * s.M;
        fc[k] = s.freq + ((long)from * KM_A + a) * s.M;
        tcv[k] = tc[k][cur[k]];
        fcv[k] = fc[k][cur[k]];
        ctv[k] = s.cent[(long)to * KM_A + a];
        cfv[k] = s.cent[(long)from * KM_A + a];
    }
#pragma unroll
    for (int k = 0; k < NA; k++) {
        tc[k][cur[k]] = tcv[k] + 1;
        fc[k][cur[k]] = fcv[k] - 1;
    }
    if (s.M == 16) {
        // what the two mode rules read after the updates -- tc[*ct] and, where the source mode lost a count, the
        // whole updated source row (64 B) -- is loaded in ONE round trip for all NA attributes (round 2 walked the row
        // with one dependent load per value: the rule fires on most groups, ~16 round trips each)
        int tct[NA];
        int4 fr[NA][4];
#pragma unroll
        for (int k = 0; k < NA; k++) {
            tct[k] = ctv[k] == cur[k] ? tcv[k] + 1 : tc[k][ctv[k]];
            if (cfv[k] == cur[k]) {
                const int4 *r4 = reinterpret_cast<const int4 *>(fc[k]);  // 64-byte rows (M = 16)
#pragma unroll
                for (int q = 0; q < 4; q++) fr[k][q] = r4[q];
            }
        }
#pragma unroll
        for (int k = 0; k < NA; k++) {
            const int a = l + W * k;
            if (tct[k] < tcv[k] + 1) s.cent[(long)to * KM_A + a] = (uint8_t)cur[k];
            if (cfv[k] == cur[k]) {  // GetMaxValueIndex (kmodes.pas:149-161): first maximum
                const int v[16] = {fr[k][0].x, fr[k][0].y, fr[k][0].z, fr[k][0].w, fr[k][1].x, fr[k][1].y, fr[k][1].z, fr[k][1].w,
                                   fr[k][2].x, fr[k][2].y, fr[k][2].z, fr[k][2].w, fr[k][3].x, fr[k][3].y, fr[k][3].z, fr[k][3].w};
                int bi = 0, bv = v[0];
#pragma unroll
                for (int m = 1; m < 16; m++)
                    if (v[m] > bv) {
                        bv = v[m];
                        bi = m;
                    }
                s.cent[(long)from * KM_A + a] = (uint8_t)bi;
            }
        }
    } else
#pragma unroll
    for (int k = 0; k < NA; k++) {
        const int a = l + W * k;
        const int tct = ctv[k] == cur[k] ? tcv[k] + 1 : tc[k][ctv[k]];  // tc[*ct] after the increment
        if (tct < tcv[k] + 1) s.cent[(long)to * KM_A + a] = (uint8_t)cur[k];
        if (cfv[k] == cur[k]) {  // the source mode lost a count: GetMaxValueIndex (first max) over the updated row
            int bi = -1, bv = INT32_MIN;
            for (int m = 0; m < s.M; m++) {
                const int v = fc[k][m];
                if (v > bv) {
                    bv = v;
                    bi = m;
                }
            }
            s.cent[(long)from * KM_A + a] = (uint8_t)bi;
        }
    }
    if (l == 0) {
        s.memb[ip] = to;
        s.csize[to]++;
        s.csize[from]--;
    }
}

// One 960-point chunk applied in order.  The chunk's assignment keys and labels are staged in LDS, the cost
// is a parallel sum, and only the points that move are visited, in order (an ordered compaction; a rescue
// that relabels a later point of the chunk rebuilds the list from there).  MovePointCat of a point touches
// only the state of its two clusters (their counts, modes and sizes), so consecutive moves whose cluster
// pairs are pairwise disjoint commute exactly: they are applied together, KM_SEQ_G at a time, by groups of
// 80 lanes.  A move that empties its cluster (size 1 before it) runs alone and is followed by the rescue
// (GetMaxClusterMembers + a random member, kmodes.pas:886-906), exactly as the reference orders it.
// DECIDE: the decision pass -- the same move sequence (every decision reads only labels, targets and cluster sizes:
// none reads a count or a mode), with the labels and sizes updated and every move appended in order to s.mvl (group
// starts flagged) instead of applied; kmb_seq_apply then applies the attribute updates over many workgroups.
template <int NT, int W, bool DECIDE = false>
__device__ void bin_seq_body(KmState s, int p0, int p1) {
    constexpr int KM_SEQ_G = NT / W;  // moves applied concurrently (W lanes each)
    static_assert(KM_SEQ_G <= 64, "the group is chosen by one wave");
    __shared__ int sh_i[4];
    __shared__ unsigned long long sh_best[NT];
    __shared__ int sh_cnt[NT];
    __shared__ unsigned long long skey[KM_BIN];
    __shared__ int smemb[KM_BIN];
    __shared__ int slist[KM_BIN];
    __shared__ int slen;
    __shared__ int c_t[KM_SEQ_G], c_cl[KM_SEQ_G], c_old[KM_SEQ_G], c_sz[KM_SEQ_G];
    __shared__ int g_t[KM_SEQ_G], g_cl[KM_SEQ_G], g_old[KM_SEQ_G], g_k[KM_SEQ_G];
    __shared__ uint4 c_x[KM_SEQ_G * 5];  // the candidates' rows, fetched with their cluster sizes
    __shared__ int g_n, g_adv, g_single;
    int nlist = 0;  // DECIDE: moves appended (uniform)
    __shared__ int g_tab[KM_CLASH_TAB];  // cluster hash -> smallest candidate index of the group touching it (64: none)
    for (int i = threadIdx.x; i < KM_CLASH_TAB; i += NT) g_tab[i] = 64;  // (the first barrier below orders it)
    const int n = p1 - p0, tid = threadIdx.x;
    // experiment build (s.dbg): shader-clock sums of the phases (wave 0's view): staging, list builds, candidate
    // fetch, group choice, apply, rescue
    unsigned long long tm_[6] = {0, 0, 0, 0, 0, 0}, tm0 = s.dbg ? __builtin_amdgcn_s_memtime() : 0, tma = 0;
    unsigned long long cpart = 0;
    for (int t = tid; t < n; t += NT) {
        const unsigned long long k = s.akey[p0 + t];
        skey[t] = k;
        smemb[t] = s.memb[p0 + t];
        cpart += k >> 32;
    }
    sh_best[tid] = cpart;
    __syncthreads();
    if (tid < 64) {  // integer total: exact in any order
        unsigned long long c = 0;
        for (int q = tid; q < NT; q += 64) c += sh_best[q];
        c = wave_sum_u64(c);
        if (tid == 0) sh_best[0] = c;
    }
    __syncthreads();
    const unsigned long long cost = sh_best[0];
    if (s.dbg) {
        tma = __builtin_amdgcn_s_memtime();
        tm_[0] += tma - tm0;
    }
    int moves = 0, ngroups = 0, nsingle = 0, nresc = 0, nrebuild = 0;
    int from_pos = 0;
    auto target = [&](int t) { return (int)(0xFFFFFFFFu - (unsigned)(skey[t] & 0xFFFFFFFFull)); };
    for (;;) {
        // ordered list of the chunk positions >= from_pos whose best cluster differs from their label: every thread
        // flags its positions (t = from_pos + r * NT + tid), ballots rank them inside each wave, one wave scans the
        // per-(round, wave) counts (round 2: wave 0 walked contiguous segments, two dependent LDS reads per position)
        __syncthreads();
        {
            constexpr int NWV = NT / 64, MAXR = (KM_BIN + NT - 1) / NT;
            static_assert(MAXR * NWV <= 64, "one wave scans the counts");
            const int lane = tid & 63, wv = tid >> 6;
            unsigned long long bal[MAXR];
#pragma unroll
            for (int r = 0; r < MAXR; r++) {
                const int t = from_pos + r * NT + tid;
                bal[r] = __ballot(t < n && target(t) != smemb[t]);
                if (lane == 0) sh_cnt[r * NWV + wv] = __popcll(bal[r]);
            }
            __syncthreads();
            if (tid < 64) {  // exclusive scan over (round, wave) in position order
                const int c = tid < MAXR * NWV ? sh_cnt[tid] : 0;
                int incl = c;
                for (int o = 1; o < 64; o <<= 1) {
                    const int v = __shfl_up(incl, o, 64);
                    if (tid >= o) incl += v;
                }
                if (tid < MAXR * NWV) sh_cnt[NT - 64 + tid] = incl - c;
                if (tid == 63) slen = incl;
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < MAXR; r++) {
                const int t = from_pos + r * NT + tid;
                if ((bal[r] >> lane) & 1)
                    slist[sh_cnt[NT - 64 + r * NWV + wv] + __popcll(bal[r] & ((1ull << lane) - 1ull))] = t;
            }
        }
        __syncthreads();
        const int len = slen;
        if (s.dbg) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            tm_[1] += t - tma;
            tma = t;
        }
        bool rebuilt = false;
        int li = 0;
        while (li < len && !rebuilt) {
            // 1. the next KM_SEQ_G candidates of the ordered list, their clusters and the source cluster size
            if (tid < KM_SEQ_G) {
                const int k = li + tid;
                int t = -1, cl = 0, old = 0, sz = 0;
                if (k < len) {
                    t = slist[k];
                    cl = target(t);
                    old = smemb[t];
                    sz = old != cl ? s.csize[old] : 0;
                }
                c_t[tid] = t;
                c_cl[tid] = cl;
                c_old[tid] = old;
                c_sz[tid] = sz;
            }
            if (!DECIDE)
                for (int e = tid; e < KM_SEQ_G * 5; e += NT) {  // rows of the candidates (the apply step reads LDS)
                    const int k = li + e / 5;
                    if (k < len) c_x[e] = reinterpret_cast<const uint4 *>(s.X + (long)(p0 + slist[k]) * KM_A)[e % 5];
                }
            __syncthreads();
            if (s.dbg) {
                const unsigned long long t = __builtin_amdgcn_s_memtime();
                tm_[2] += t - tma;
                tma = t;
            }
            // 2. the longest prefix of them that can run together (in list order), chosen by wave 0 with ballots:
            // entries whose label already equals their target are skipped (counted in the advance), the first move
            // that empties its cluster or shares a cluster with an earlier move of the prefix ends it; a move that
            // empties its cluster at the head runs alone (then the rescue)
            if (tid < 64) {
                const int k = tid;
                const bool valid = k < KM_SEQ_G && c_t[k] >= 0;
                const int cl = valid ? c_cl[k] : -1, old = valid ? c_old[k] : -2;
                const bool mv = valid && cl != old;
                // "shares a cluster with an earlier move": every move enters the smallest index touching each of its
                // two clusters into a table indexed by cluster mod KM_CLASH_TAB (LDS atomics of one wave are applied in
                // order, before the reads below); with K > KM_CLASH_TAB a bucket shared by two clusters only ends the
                // prefix earlier (still a set of pairwise disjoint moves).  Round 2 compared each lane with every earlier one, one LDS round trip each.
                const int h1 = cl & (KM_CLASH_TAB - 1), h2 = old & (KM_CLASH_TAB - 1);
                if (mv) {
                    atomicMin(&g_tab[h1], k);
                    atomicMin(&g_tab[h2], k);
                }
                const bool clash = mv && (g_tab[h1] < k || g_tab[h2] < k);
                if (mv) {  // back to empty (after every lane's reads: one wave, in order)
                    g_tab[h1] = 64;
                    g_tab[h2] = 64;
                }
                const unsigned long long stopm = __ballot(mv && (c_sz[k < KM_SEQ_G ? k : 0] <= 1 || clash));
                const unsigned long long invm = __ballot(!valid);  // lanes >= KM_SEQ_G are invalid (none when KM_SEQ_G = 64)
                const int first_inv = invm ? __builtin_ctzll(invm) : 64;  // a full 64-candidate window: none invalid
                const int first_stop = stopm ? __builtin_ctzll(stopm) : 64;
                const int end = min(first_stop, first_inv);
                const unsigned long long below_end = end >= 64 ? ~0ull : ((1ull << end) - 1ull);
                const unsigned long long mvm = __ballot(mv) & below_end;
                const int ng = __popcll(mvm);
                if (ng == 0 && first_stop < first_inv) {  // an emptying move at the head: alone
                    if (k == first_stop) {
                        g_t[0] = c_t[k];
                        g_cl[0] = cl;
                        g_old[0] = old;
                        g_k[0] = k;
                        g_n = 1;
                        g_adv = first_stop + 1;
                        g_single = 1;
                    }
                } else {
                    if (mv && k < end) {
                        const int r = __popcll(mvm & ((1ull << k) - 1ull));
                        g_t[r] = c_t[k];
                        g_cl[r] = cl;
                        g_old[r] = old;
                        g_k[r] = k;
                    }
                    if (k == 0) {
                        g_n = ng;
                        g_adv = end;
                        g_single = 0;
                    }
                }
            }
            __syncthreads();
            if (s.dbg) {
                const unsigned long long t = __builtin_amdgcn_s_memtime();
                tm_[3] += t - tma;
                tma = t;
            }
            const int ng = g_n;
            li += g_adv;
            moves += ng;
            ngroups++;
            nsingle += g_single;
            // 3. apply them: lanes [W j, W j + W) move point j of the group
            if (DECIDE) {  // labels and sizes now (cluster-disjoint moves: no two threads touch one size), the move listed
                if (tid < ng) {
                    const int ip = p0 + g_t[tid], to = g_cl[tid], from = g_old[tid];
                    s.memb[ip] = to;
                    s.csize[to]++;
                    s.csize[from]--;
                    s.mvl[nlist + tid] = make_int4(ip, to, from, tid == 0 ? 1 : 0);
                    smemb[g_t[tid]] = to;
                }
                nlist += ng;
            } else {
                const int j = tid / W, l = tid - j * W;
                if (j < ng)
                    move_point_cat_w<W>(s, p0 + g_t[j], g_cl[j], g_old[j], l, reinterpret_cast<const uint8_t *>(c_x + g_k[j] * 5));
                if (tid < ng) smemb[g_t[tid]] = g_cl[tid];
            }
            __syncthreads();
            if (s.dbg) {
                const unsigned long long t = __builtin_amdgcn_s_memtime();
                tm_[4] += t - tma;
                tma = t;
            }
            if (!g_single) continue;
            const int t = g_t[0], old = g_old[0];
            if (s.csize[old] != 0) continue;
            nresc++;
            // GetMaxClusterMembers (kmodes.pas:631-669): largest cluster, ties -> last
            unsigned long long b = 0;
            for (int c = tid; c < s.K; c += NT) {
                const unsigned long long v = ((unsigned long long)(unsigned)s.csize[c] << 32) | (unsigned)c;
                b = v > b ? v : b;
            }
            sh_best[tid] = b;
            __syncthreads();
            if (tid < 64) {
                unsigned long long m = 0;
                for (int q = tid; q < NT; q += 64) m = max(m, sh_best[q]);
                m = wave_max_u64(m);
                if (tid == 0) sh_best[0] = m;
            }
            __syncthreads();
            const int from = (int)(sh_best[0] & 0xFFFFFFFFull);
            const int cnt = s.csize[from];
            if (tid == 0) sh_i[0] = (int)km_randint((unsigned)cnt, s.seed);
            __syncthreads();
            const int r = sh_i[0];
            // r-th member of 'from' in ascending point order (choices[RandInt(cnt)], kmodes.pas:895-902)
            const long chunk = (s.n + NT - 1) / NT;
            const long b0 = tid * chunk, b1 = min((long)s.n, b0 + chunk);
            int cm = 0;
            for (long q = b0; q < b1; q++) cm += s.memb[q] == from;
            sh_cnt[tid] = cm;
            __syncthreads();
            if (tid == 0) {
                int acc = 0, tt = 0;
                while (tt < NT && acc + sh_cnt[tt] <= r) acc += sh_cnt[tt++];
                sh_i[1] = tt;
                sh_i[2] = r - acc;
            }
            __syncthreads();
            if (tid == sh_i[1]) {
                int left = sh_i[2];
                for (long q = b0; q < b1; q++)
                    if (s.memb[q] == from && left-- == 0) {
                        sh_i[3] = (int)q;
                        break;
                    }
            }
            __syncthreads();
            const int qp = sh_i[3];
            if (DECIDE) {
                if (tid == 0) {
                    s.memb[qp] = old;
                    s.csize[old]++;
                    s.csize[from]--;
                    s.mvl[nlist] = make_int4(qp, old, from, 1);
                }
                nlist++;
            } else if (tid < KM_A) {
                move_point_cat(s, qp, old, from, tid);
            }
            if (tid == 0 && qp >= p0 && qp < p1) smemb[qp - p0] = old;
            __syncthreads();
            if (qp - p0 > t && qp < p1) {  // a later point of this chunk was relabelled: rebuild from t + 1
                from_pos = t + 1;
                rebuilt = true;
                nrebuild++;
            }
            if (s.dbg) {
                const unsigned long long tt = __builtin_amdgcn_s_memtime();
                tm_[5] += tt - tma;
                tma = tt;
            }
        }
        if (!rebuilt) break;
    }
    if (tid == 0) {
        if (DECIDE) *s.mvn = nlist;
        s.cost[0] += cost;
        s.moves[0] += moves;
        if (s.dbg) {
            atomicAdd(s.dbg + 0, ngroups);
            atomicAdd(s.dbg + 1, moves);
            atomicAdd(s.dbg + 2, nsingle);
            atomicAdd(s.dbg + 3, nresc);
            atomicAdd(s.dbg + 4, nrebuild);
            atomicMax(s.dbg + 5, ngroups);
            atomicAdd(s.dbg + 6, 1);
            unsigned long long *t64 = reinterpret_cast<unsigned long long *>(s.dbg + 8);  // [8..19]: 6 u64 clock sums
            for (int q = 0; q < 6; q++) atomicAdd(t64 + q, tm_[q]);
        }
    }
}

// ---- batched state: the single-bin KmState of bin b is a view into concatenated arrays ----
struct KmBatch {
    const uint8_t *X;             // [N][80], bins contiguous, rows 16-byte aligned
    const int32_t *boff, *koff;   // [nb+1] point / cluster offsets
    const int32_t *poff;          // [nb+1] farthest-first partial slots (blocks) per bin
    int nb, M;
    int32_t *memb;                // [N] bin-local labels
    uint8_t *cent;                // [Ktot][80]
    int32_t *freq;                // [Ktot][80][M]
    int32_t *csize;               // [Ktot]
    unsigned long long *mind;     // [N]
    uint8_t *used;                // [N]
    unsigned long long *part;     // [poff[nb]]
    int32_t *center;              // [Ktot]
    unsigned long long *akey;     // [N]
    unsigned *seed;               // [nb]
    unsigned long long *cost;     // [nb]
    int *moves, *err, *ffdone;    // [nb]
    int *dbg;                     // [nb][24] sequential-pass counters (study hook; null in the library)
    int4 *mvl;                    // [nb][2 * KM_BIN] move lists of the decision pass
    int *mvn;                     // [nb]
};

__device__ __forceinline__ KmState bin_state(const KmBatch &B, int b) {
    KmState s;
    const long p0 = B.boff[b], k0 = B.koff[b];
    s.X = B.X + p0 * KM_A;
    s.n = (int)(B.boff[b + 1] - p0);
    s.K = (int)(B.koff[b + 1] - k0);
    s.M = B.M;
    s.memb = B.memb + p0;
    s.cent = B.cent + k0 * KM_A;
    s.freq = B.freq + k0 * KM_A * B.M;
    s.csize = B.csize + k0;
    s.mind = B.mind + p0;
    s.used = B.used + p0;
    s.part = B.part + B.poff[b];
    s.center = B.center + k0;
    s.akey = B.akey + p0;
    s.seed = B.seed + b;
    s.cost = B.cost + b;
    s.moves = B.moves + b;
    s.err = B.err + b;
    s.dbg = B.dbg ? B.dbg + 24 * b : nullptr;
    s.mvl = B.mvl + (long)b * 2 * KM_BIN;
    s.mvn = B.mvn + b;
    return s;
}

__device__ __forceinline__ int bin_of(const int32_t *off, int nb, long i) {  // off[b] <= i < off[b+1]
    int lo = 0, hi = nb - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// start of a KModesIter for the bins act[blockIdx.y]: cost, moves, assignment keys
__global__ __launch_bounds__(256) void kmb_iter_reset(KmBatch B, const int *act) {
    const int r = act[blockIdx.y];
    const long p0 = B.boff[r], n = B.boff[r + 1] - p0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) B.akey[p0 + i] = ~0ull;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        B.cost[r] = 0;
        B.moves[r] = 0;
    }
}

// farthest-first start (kmodes.pas:698-710): one thread per bin
__global__ void kmb_ff_start(KmBatch B, const int32_t *start) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B.nb) return;
    KmState s = bin_state(B, b);
    const int st = start[b];
    s.center[0] = st;
    for (int a = 0; a < KM_A; a++) s.cent[a] = s.X[(long)st * KM_A + a];
    s.used[st] = 1;
}

// one farthest-first round j for every bin with K > j (a prefix of the K-sorted bins): work item =
// (bin, block of that bin); the last block of a bin to finish (counter ffdone) selects centre j + 1
struct KmFfItem {
    int bin, sub, nsub, pad;
};

__global__ __launch_bounds__(256) void kmb_ff_round(KmBatch B, const KmFfItem *items, int j) {
    __shared__ unsigned long long best[256];
    __shared__ int last;
    const KmFfItem it = items[blockIdx.x];
    KmState s = bin_state(B, it.bin);
    const int c = s.center[j];
    uint32_t item[20];
    load_row(s.X + (long)c * KM_A, item);
    unsigned long long bv = 0;
    int bi = -1;
    for (long i = (long)it.sub * 256 + threadIdx.x; i < s.n; i += (long)it.nsub * 256) {
        uint32_t row[20];
        load_row(s.X + i * KM_A, row);
        const unsigned long long d = km_dissim(row, item);
        unsigned long long m = s.mind[i];
        if (d < m) {  // cmovb: strict-less (kmodes.pas:555-558); the 'used' skip is a no-op (567)
            m = d;
            s.mind[i] = m;
        }
        if (!s.used[i] && m >= bv) {  // ascending i within a thread: '>=' keeps the last
            bv = m;
            bi = (int)i;
        }
    }
    // block reduce (value max, ties -> larger index); value fits 32 bits (dis < 2^19) unless UINT64_MAX
    const unsigned long long v32 = bv > 0xFFFFFFFFull ? 0xFFFFFFFFull : bv;
    best[threadIdx.x] = (bi < 0) ? 0ull : ((v32 << 32) | (unsigned)(bi + 1));
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) best[threadIdx.x] = max(best[threadIdx.x], best[threadIdx.x + o]);
        __syncthreads();
    }
    if (j + 1 >= s.K) return;  // last round of this bin: no selection
    if (threadIdx.x == 0) {
        s.part[it.sub] = best[0];
        __threadfence();
        last = atomicAdd(&B.ffdone[it.bin], 1) == it.nsub - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    unsigned long long bb = 0;
    for (int i = threadIdx.x; i < it.nsub; i += 256)  // device-scope loads: bypass a stale L1 line of an earlier round
        bb = max(bb, __hip_atomic_load(&s.part[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    best[threadIdx.x] = bb;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) best[threadIdx.x] = max(best[threadIdx.x], best[threadIdx.x + o]);
        __syncthreads();
    }
    const unsigned long long w = best[0];
    const int f = (w == 0) ? -1 : (int)(w & 0xFFFFFFFFull) - 1;
    if (threadIdx.x == 0) B.ffdone[it.bin] = 0;
    if (f < 0) {
        if (threadIdx.x == 0) *s.err = 1;
        return;
    }
    if (threadIdx.x < KM_A) s.cent[(long)(j + 1) * KM_A + threadIdx.x] = s.X[(long)f * KM_A + threadIdx.x];
    if (threadIdx.x == 0) {
        s.center[j + 1] = f;
        s.used[f] = 1;
    }
}

// assignment work item: points [p0, p1) of bin vs its centroids [c0, c1): akey = min(dis << 32 | ~c)
struct KmAsgItem {
    int bin, p0, p1, c0, c1, pad[3];
};

__global__ __launch_bounds__(256) void kmb_assign(KmBatch B, const KmAsgItem *items) {
    __shared__ uint4 ct[128 * 5];
    KmAsgItem it = items[blockIdx.x];
    {  // this workgroup's share of the item's centroids (gridDim.y sub-splits); ties across splits: atomicMin key
        const int per = (it.c1 - it.c0 + (int)gridDim.y - 1) / (int)gridDim.y;
        it.c0 += (int)blockIdx.y * per;
        it.c1 = min(it.c1, it.c0 + per);
        if (it.c0 >= it.c1) return;
    }
    KmState s = bin_state(B, it.bin);
    const long i = it.p0 + threadIdx.x;
    const bool valid = i < it.p1;
    uint32_t item[20];
    if (valid) load_row(s.X + i * KM_A, item);
    unsigned long long best = ~0ull;
    for (int t0 = it.c0; t0 < it.c1; t0 += 128) {
        const int cnt = min(128, it.c1 - t0);
        __syncthreads();
        for (int e = threadIdx.x; e < cnt * 5; e += 256)
            ct[e] = reinterpret_cast<const uint4 *>(s.cent + (long)t0 * KM_A)[e];
        __syncthreads();
        if (valid) {
            for (int c = 0; c < cnt; c++) {
                uint32_t row[20];
#pragma unroll
                for (int q = 0; q < 5; q++) {
                    const uint4 v = ct[c * 5 + q];
                    row[4 * q] = v.x;
                    row[4 * q + 1] = v.y;
                    row[4 * q + 2] = v.z;
                    row[4 * q + 3] = v.w;
                }
                const unsigned long long d = km_dissim(row, item);
                const unsigned long long key = (d << 32) | (0xFFFFFFFFu - (unsigned)(t0 + c));
                best = key < best ? key : best;
            }
        }
    }
    if (valid) atomicMin(&s.akey[i], best);
}

// ---- assignment with at most 16 modalities (round 3) ----
// The histograms index freq[.][.][M] by byte value, so with M <= 16 every byte of X (and of every mode) is < 16.
// Then the asm's int8 |r - x| is the plain |r - x| <= 15 and W0 / W4 never wrap (a0 + 256 a1 + S_lo <= 15 + 3,840 +
// 480 < 2^16):   dis = 2048 #mismatch + (a0 + a8) + 256 (a1 + a9) + sum_{k=16..79} |r_k - x_k|   (= km_dissim).
// A byte differs iff one of its 4 bit planes differs, so #mismatch is, per 32 bytes, the popcount of the OR of the
// 4 planes' XORs (3 words) instead of a nonzero-byte count per dword, and the L1 is one v_sad_u8 chain over bytes
// 16..79 plus two over the packed words (byte 0 | byte 8 << 8) and (byte 1 | byte 9 << 8): ~40 VALU per pair
// instead of ~155.  Prepared row, KM_PW words: [0, 16) bytes 16..79, [16, 28) planes (word 16 + 3p + k = bit p of
// bytes 32k .. 32k + 31), 28 the low word, 29 the high word, 30-31 zero.  Points are prepared once per call
// (X never changes), centroids per stage in LDS (the sequential passes change modes).
static constexpr int KM_PW = 32;
static constexpr int KM_A16_CT = 64;  // centroids per LDS stage

__device__ __forceinline__ uint32_t km_prep_word(const uint32_t *row, int w) {
    if (w < 16) return row[4 + w];
    if (w < 28) {
        const int p = (w - 16) / 3, k = (w - 16) % 3;
        uint32_t r = 0;
        for (int j = 0; j < 8 && 8 * k + j < 20; j++) {
            // bits p of the 4 bytes of dword 8k + j -> 4 consecutive bits: (b0 | b1 << 8 | b2 << 16 | b3 << 24) *
            // 0x01020408 puts b_i at bit 24 + i and nothing else in bits 24..31
            const uint32_t v = (row[8 * k + j] >> p) & 0x01010101u;
            r |= ((v * 0x01020408u) >> 24) << (4 * j);
        }
        return r;
    }
    if (w == 28) return (row[0] & 0xFFu) | ((row[2] & 0xFFu) << 8);
    if (w == 29) return ((row[0] >> 8) & 0xFFu) | (((row[2] >> 8) & 0xFFu) << 8);
    return 0;
}

__device__ __forceinline__ unsigned km_dissim16(const uint32_t *__restrict__ r, const uint32_t *__restrict__ x) {
    unsigned l1 = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) l1 = __builtin_amdgcn_sad_u8(r[w], x[w], l1);
    l1 = __builtin_amdgcn_sad_u8(r[28], x[28], l1);
    const unsigned hi = __builtin_amdgcn_sad_u8(r[29], x[29], 0u);
    unsigned mism = 0;
#pragma unroll
    for (int k = 0; k < 3; k++)
        mism += __popc((r[16 + k] ^ x[16 + k]) | (r[19 + k] ^ x[19 + k]) | (r[22 + k] ^ x[22 + k]) | (r[25 + k] ^ x[25 + k]));
    return (mism << 11) + l1 + (hi << 8);
}

// prepared point rows of the (bin-permuted) X; *bad |= 1 if some byte is >= 16
__global__ __launch_bounds__(256) void kmb_prep_points(const uint8_t *X, long N, uint4 *Xp, unsigned *bad) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < N; i += (long)gridDim.x * 256) {
        uint32_t row[20];
        load_row(X + i * KM_A, row);
        uint32_t big = 0;
#pragma unroll
        for (int d = 0; d < 20; d++) big |= row[d] & 0xF0F0F0F0u;
        if (big) atomicOr(bad, 1u);
        uint32_t o[KM_PW];
#pragma unroll
        for (int w = 0; w < KM_PW; w++) o[w] = km_prep_word(row, w);
#pragma unroll
        for (int q = 0; q < KM_PW / 4; q++) Xp[i * (KM_PW / 4) + q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    }
}

// kmb_assign with km_dissim16; inside a workgroup the argmin runs on 32-bit keys (dis << 13 | 8191 - local index:
// dis < 2^18, at most 8,192 centroids per workgroup -- host-checked), merged into the u64 key by atomicMin as before.
// G groups of 256 threads per workgroup (each one point per thread over its own slice of the item's centroids, the
// item split over gridDim.y * G slices) and PF (the next centroid's LDS row read while this one is compared) are
// experiment-build A/B forms only.  C4 assignment time (r03zk-zn, 6,423 launches): 4 slices of 256 threads 142 ms;
// 1 / 2 / 8 / 16 slices 176 / 152 / 184 / 289 ms; 2 or 4 groups per workgroup 163 / 223 ms; PF 147 ms; 2 or 4 points
// per thread (fewer waves, half / a quarter of the broadcast LDS reads per pair) 162 / 200 ms.  Neither fewer point
// re-reads nor fewer LDS reads per pair pays: the late steps (960 points x 5,035 centroids) are latency-bound waves.
template <int G, bool PF = false>
__global__ __launch_bounds__(256 * G) void kmb_assign16(KmBatch B, const KmAsgItem *items, const uint4 *__restrict__ Xp) {
    __shared__ uint4 raw[G][KM_A16_CT * 5];
    __shared__ uint4 ct[G][KM_A16_CT * (KM_PW / 4)];
    const KmAsgItem it = items[blockIdx.x];
    const int g = threadIdx.x >> 8, tid = threadIdx.x & 255;
    const int per = (it.c1 - it.c0 + (int)gridDim.y * G - 1) / ((int)gridDim.y * G);
    const int gc0 = it.c0 + ((int)blockIdx.y * G + g) * per, gc1 = min(it.c1, gc0 + per);
    if (G == 1 && gc0 >= gc1) return;
    KmState s = bin_state(B, it.bin);
    const long i = it.p0 + tid;
    const bool valid = i < it.p1 && gc0 < gc1;
    uint32_t x[KM_PW];
    if (valid) {
        const uint4 *src = Xp + ((long)B.boff[it.bin] + i) * (KM_PW / 4);
#pragma unroll
        for (int q = 0; q < KM_PW / 4; q++) {
            const uint4 v = src[q];
            x[4 * q] = v.x;
            x[4 * q + 1] = v.y;
            x[4 * q + 2] = v.z;
            x[4 * q + 3] = v.w;
        }
    }
    unsigned best = ~0u;
    for (int t = 0; t < per; t += KM_A16_CT) {  // the same trip count in every group (barriers inside)
        const int t0 = gc0 + t, cnt = max(0, min(KM_A16_CT, gc1 - t0));
        __syncthreads();
        for (int e = tid; e < cnt * 5; e += 256) raw[g][e] = reinterpret_cast<const uint4 *>(s.cent + (long)t0 * KM_A)[e];
        __syncthreads();
        for (int e = tid; e < cnt * KM_PW; e += 256)
            reinterpret_cast<uint32_t *>(ct[g])[e] =
                km_prep_word(reinterpret_cast<const uint32_t *>(raw[g] + (e / KM_PW) * 5), e % KM_PW);
        __syncthreads();
        if (valid && !PF) {
            const unsigned kb = 8191u - (unsigned)t;
            for (int c = 0; c < cnt; c++) {
                uint32_t r[KM_PW];
#pragma unroll
                for (int q = 0; q < KM_PW / 4; q++) {
                    const uint4 v = ct[g][c * (KM_PW / 4) + q];
                    r[4 * q] = v.x;
                    r[4 * q + 1] = v.y;
                    r[4 * q + 2] = v.z;
                    r[4 * q + 3] = v.w;
                }
                best = min(best, (km_dissim16(r, x) << 13) | (kb - (unsigned)c));
            }
        } else if (valid && cnt > 0) {  // PF: the next centroid's row read from LDS while this one is compared
            const unsigned kb = 8191u - (unsigned)t;
            uint4 nx[KM_PW / 4];
#pragma unroll
            for (int q = 0; q < KM_PW / 4; q++) nx[q] = ct[g][q];
            for (int c = 0; c < cnt; c++) {
                uint32_t r[KM_PW];
#pragma unroll
                for (int q = 0; q < KM_PW / 4; q++) {
                    r[4 * q] = nx[q].x;
                    r[4 * q + 1] = nx[q].y;
                    r[4 * q + 2] = nx[q].z;
                    r[4 * q + 3] = nx[q].w;
                }
                const int cn = c + 1 < cnt ? c + 1 : c;
#pragma unroll
                for (int q = 0; q < KM_PW / 4; q++) nx[q] = ct[g][cn * (KM_PW / 4) + q];
                best = min(best, (km_dissim16(r, x) << 13) | (kb - (unsigned)c));
            }
        }
    }
    if (valid) {
        const unsigned c = (unsigned)gc0 + 8191u - (best & 8191u);
        atomicMin(&s.akey[i], ((unsigned long long)(best >> 13) << 32) | (0xFFFFFFFFu - c));
    }
}

// initial labels + histograms (ComputeKModes kmodes.pas:984-1008), all points of all bins
__global__ __launch_bounds__(256) void kmb_init_hist(KmBatch B, long N) {
    for (long g = (long)blockIdx.x * 256 + threadIdx.x; g < N; g += (long)gridDim.x * 256) {
        const int b = bin_of(B.boff, B.nb, g);
        KmState s = bin_state(B, b);
        const long i = g - B.boff[b];
        const int c = (int)(0xFFFFFFFFu - (unsigned)(s.akey[i] & 0xFFFFFFFFull));
        s.memb[i] = c;
        atomicAdd(&s.csize[c], 1);
        for (int a = 0; a < KM_A; a++) atomicAdd(&s.freq[((long)c * KM_A + a) * s.M + s.X[i * KM_A + a]], 1);
    }
}

// modes (kmodes.pas:1010-1021): empty clusters take X[RandInt(n)][a] per attribute in (k, a) order
__global__ void kmb_init_modes(KmBatch B, int32_t *rand_rows) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B.nb) return;
    KmState s = bin_state(B, b);
    int32_t *rr = rand_rows + (long)B.koff[b] * KM_A;
    unsigned seed = *s.seed;
    for (int k = 0; k < s.K; k++)
        if (s.csize[k] == 0)
            for (int a = 0; a < KM_A; a++) rr[(long)k * KM_A + a] = (int)km_randint((unsigned)s.n, &seed);
    *s.seed = seed;
}

__global__ __launch_bounds__(256) void kmb_init_modes2(KmBatch B, const int32_t *rand_rows, long ktot) {
    for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < ktot * KM_A; e += (long)gridDim.x * 256) {
        const long kg = e / KM_A;
        const int a = (int)(e % KM_A);
        const int b = bin_of(B.koff, B.nb, kg);
        KmState s = bin_state(B, b);
        const long el = e - (long)B.koff[b] * KM_A;  // bin-local element (k, a)
        const int k = (int)(el / KM_A);
        if (s.csize[k] == 0) {
            s.cent[el] = s.X[(long)rand_rows[e] * KM_A + a];
        } else {
            const int32_t *f = s.freq + el * s.M;
            int bi = -1, bv = INT32_MIN;
            for (int m = 0; m < s.M; m++)
                if (f[m] > bv) {
                    bv = f[m];
                    bi = m;
                }
            s.cent[el] = (uint8_t)bi;  // GetMaxValueIndex: first max (kmodes.pas:149-161)
        }
    }
}

// each host work item (<= 64 centroids) runs as KM_ASUB workgroups of a quarter of its centroids: the late
// chunk steps hold one large bin alone, where one workgroup per item left ~1 wave per SIMD (latency-bound)
static constexpr int KM_ASUB = 4;
static constexpr int KM_A16_G = 1;  // 256-thread groups per kmb_assign16 workgroup

// one 960-point chunk of each listed bin, applied in order (KModesIter kmodes.pas:869-911)
struct KmSeqItem {
    int bin, p0, p1, pad;
};

// seq items live in the same work list as the assign items (one KmAsgItem slot each)
template <int NT, int W, bool DECIDE = false>
__global__ __launch_bounds__(NT) void kmb_seq_strided(KmBatch B, const KmAsgItem *items) {
    const KmSeqItem it = *reinterpret_cast<const KmSeqItem *>(items + blockIdx.x);
    KmState s = bin_state(B, it.bin);
    bin_seq_body<NT, W, DECIDE>(s, it.p0, it.p1);
}

// The attribute updates of one chunk's move list (kmb_seq_strided<.., true>), attributes split over NSLICE
// workgroups per bin (blockIdx.y): each applies the list in order, group after group, the moves of a group (pairwise
// cluster-disjoint) at once, one lane per (move, attribute).  Every (cluster, attribute) sees its updates in the
// reference's order; attributes are independent of each other.  Round 2 applied them on the deciding workgroup alone
// (one CU's memory traffic: ~10 us per group of ~26 moves, each touching 160 count rows).
static constexpr int KM_APPLY_SLICES = 10;
template <int NSLICE>
__global__ __launch_bounds__(32 * (KM_A / NSLICE)) void kmb_seq_apply(KmBatch B, const KmAsgItem *items) {
    constexpr int W = KM_A / NSLICE, NT = 32 * W;  // one attribute per lane, 32 moves per pass
    static_assert(KM_A % NSLICE == 0 && NT % 64 == 0, "attribute slices");
    __shared__ int gs[2 * KM_BIN + 1];  // group starts
    __shared__ int ngr;
    const KmSeqItem it = *reinterpret_cast<const KmSeqItem *>(items + blockIdx.x);
    KmState s = bin_state(B, it.bin);
    const int n = *s.mvn, tid = threadIdx.x;
    if (n == 0) return;  // uniform
    // group starts in list order: ballot ranks per wave, wave totals through LDS (one wave scans them)
    __shared__ int wtot[2 * KM_BIN / 64 + 2];
    const int nw = (n + 63) / 64;
    for (int i0 = 0; i0 < nw * 64; i0 += NT) {
        const int i = i0 + tid;
        const bool f = i < n && s.mvl[i].w != 0;
        const unsigned long long b = __ballot(f);
        if ((tid & 63) == 0 && i < nw * 64) wtot[i >> 6] = __popcll(b);
    }
    __syncthreads();
    if (tid == 0) {
        int acc = 0;
        for (int w = 0; w < nw; w++) {
            const int c = wtot[w];
            wtot[w] = acc;
            acc += c;
        }
        ngr = acc;
        gs[acc] = n;
    }
    __syncthreads();
    for (int i0 = 0; i0 < nw * 64; i0 += NT) {
        const int i = i0 + tid;
        const bool f = i < n && s.mvl[i].w != 0;
        const unsigned long long b = __ballot(f);
        if (f) gs[wtot[i >> 6] + __popcll(b & ((1ull << (tid & 63)) - 1ull))] = i;
    }
    __syncthreads();
    const int G = ngr, j = tid / W, l = tid - j * W, a0 = blockIdx.y * W + l;
    for (int g = 0; g < G; g++) {
        for (int m = gs[g] + j; m < gs[g + 1]; m += NT / W) {  // a group's moves are cluster-disjoint: any batching
            const int4 mv = s.mvl[m];
            apply_point_attrs<W, 1>(s, mv.x, mv.y, mv.z, a0);
        }
        __syncthreads();  // the next group may touch these clusters' rows
    }
}

// ---- farthest-first as ONE persistent launch (round 3) ----
// InitFarthestFirst is 5,035 rounds at C4 (the largest bin's K), each dependent on the last, and one launch per round
// cost ~40 us (20 us median, r03i trace).  Here one workgroup per CU runs every round: the items of the alive bins
// (same (bin, sub) list, points strided by KM_FF_NT), the last item of a bin to finish selects its next centre (the
// per-launch kernel's counter protocol), then a grid barrier.  The barrier is two-level -- 8 arrival counters (one
// 128-byte line each, workgroups by blockIdx % 8) -> a top counter -> 8 generation words (one per group, each polled
// by its group only) -- with
// monotonic counts inside the call (zeroed per call).  Hand-offs follow cdna_hip_programming.md Guideline 16 R1: every
// word another workgroup reads in this launch (a bin's centre index, the used flags, the per-item candidates) is
// stored AND loaded `sc1` (agent-scope atomics), drained before the counter add, so no release / acquire fence runs
// (an agent release writes back the XCD's dirty L2 lines and the acquire drops the CU's L1: r03k's first form with
// them took 56 us per round); rows and min-distances are read-only or owner-only.  cooperative_groups' grid sync (26-100 us per call on ROCm 7.2) made the r03 cooperative form slower
// than the launches it replaced.  Item u is always processed by workgroup u % G, so a point's min-distance word is
// only ever touched by one workgroup and its rows stay in that XCD's L2.  Every spin is bounded: a barrier that waits
// ~0.5 s sets *fail, every workgroup leaves, and the host reruns the rounds with the per-launch kernel (the state
// is re-initialised), so a result never depends on residency.  Same updates, same partition-independent argmax
// (value, then the largest index), so the centres are those of the per-launch rounds.
static constexpr int KM_FF_NT = 512;
static constexpr int KM_FF_SUBMAX = 512;  // farthest-first items (subs) per bin at most

// Study build only (-DTILER_KM_STAMPS, tools/ff_stamps.py; never in the shipped library): thread 0 of every workgroup
// stamps the 100 MHz real-time counter at 8 points of two windows of 64 rounds (rounds 64..127, and the 64 rounds
// from Kmax - 128 on, when only the largest bin is alive).  The stamp at "row landed" waits for the centre row.
#ifdef TILER_KM_STAMPS
__device__ unsigned long long g_km_stamps[2][64][256][8];
__device__ __forceinline__ void km_stamp(int j, int Kmax, int pt) {
    if (threadIdx.x != 0 || blockIdx.x >= 256) return;
    const int w = (j >= 64 && j < 128) ? 0 : (j >= Kmax - 128 && j < Kmax - 64) ? 1 : -1;
    if (w >= 0) g_km_stamps[w][j - (w ? Kmax - 128 : 64)][blockIdx.x][pt] = __builtin_amdgcn_s_memrealtime();
}
#define KM_STAMP(j, Kmax, pt) km_stamp(j, Kmax, pt)
#else
#define KM_STAMP(j, Kmax, pt) ((void)0)
#endif

__device__ __forceinline__ bool km_grid_sync(unsigned *bar, unsigned epoch, unsigned *fail, int Kmax = 0) {
    __shared__ int s_ok;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its sc1 stores have left (R1 drain)
    __syncthreads();
    (void)Kmax;
    if (threadIdx.x == 0) {
        KM_STAMP((int)epoch - 1, Kmax, 5);
        const int G = (int)gridDim.x, g = (int)(blockIdx.x & 7);
        const unsigned ng = (unsigned)((G - g + 7) >> 3), ngroups = (unsigned)min(G, 8);
        int ok = 1;
        // group g's generation word: its own 128-byte line, polled by that group's workgroups only
        if (__hip_atomic_fetch_add(bar + 32 * g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch * ng - 1u &&
            __hip_atomic_fetch_add(bar + 256, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch * ngroups - 1u)
            for (int x = 0; x < 8; x++) __hip_atomic_store(bar + 288 + 32 * x, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        KM_STAMP((int)epoch - 1, Kmax, 6);
        for (unsigned spins = 0; __hip_atomic_load(bar + 288 + 32 * g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch;) {
            if (__hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u || ++spins > (1u << 20)) {
                __hip_atomic_store(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        KM_STAMP((int)epoch - 1, Kmax, 7);
        s_ok = ok;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the sc1 loads below the poll
    __syncthreads();
    return s_ok != 0;
}

// The farthest-first protocol (round 3, r03zo; kmb_ff_persist2 until round 6, now kmb_ff_persist3 below): every item of round j stores its candidate
// (sc1) into the round's parity half of the part slots and arrives; after the barrier EVERY item of a bin reduces
// that bin's candidates itself (the same partition-independent maximum, so the same centre) instead of the last item
// to finish selecting and publishing it.  Gone per round: the ffdone count, the selector's candidate loads, the
// centre's sc1 publication and its load -- three dependent device-scope round trips of the ~11 on a round's
// critical path.  The slots alternate halves by round parity: round j + 1's stores cannot reach a half that a slow
// workgroup still reads for round j (it has not arrived at barrier j + 1 yet).  The used flag of a point is written
// and read only by the lane that scans it, centres and their rows for the later kernels by the bin's sub-0 item
// (plain stores: nothing in this launch reads them).

// (value, largest index) maximum of a packed u64 over the wave
__device__ __forceinline__ unsigned long long km_wave_max(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long ov = ((unsigned long long)__shfl_xor((unsigned)(v >> 32), o, 64) << 32) |
                                      (unsigned)__shfl_xor((unsigned)v, o, 64);
        v = ov > v ? ov : v;
    }
    return v;
}

// Farthest-first with WAVE work items (round 6).  Round stamps of kmb_ff_persist2 (tools/ff_stamps.py,
// profiles/r06/ff_stamps_persist2.json) put the time in the items, not the barrier: a round with only the largest bin
// alive took 7.4 us (barrier ~2.5 us of it), but rounds with every bin alive took 60 us, because each workgroup ran its
// ~13 (bin, sub) items one after another, each a dependent chain (candidate slots -> centre -> its row -> scan ->
// reduce) of ~4.6 us over only ~2 points per thread.  Here an item is one wave's: lane l of sub s owns the points
// s * 64 + l + k * nsub * 64 (the slot layout, used flags and candidate protocol of kmb_ff_persist2 per item, the
// reductions wave shuffles with no workgroup barrier), item u always on wave slot u % (8 G) -- wave u / G of workgroup
// u % G, so consecutive items sit on different CUs and a point's min-distance word stays with one lane -- so a
// workgroup's 8 waves run 8 items concurrently.  Items hold ~256 points (4 per lane, loaded together): a bin has
// min(512, n / 256) subs.  The same partition-independent maximum, so the same centres.  C4 (r06f, one box): 101 ms
// (persist2) -> 79 ms (wave items, one load at a time) -> 56 ms (slot and point loads in flight together); rounds with
// every bin alive 60 -> 21 us, with the largest bin alone 7.4 -> 7.9 us (profiles/r06/ff_stamps_*.json).  Measured and
// not kept: two items per wave carried together (256 VGPRs, 111 spilled) and ~512-point items (59.5 ms: the early
// rounds stream 80 MB of rows each and fewer, longer items lose more to latency than they save in slots).
__global__ __launch_bounds__(KM_FF_NT) void kmb_ff_persist3(KmBatch B, const KmFfItem *items, const int *ff_end,
                                                            int Kmax, unsigned *bar, unsigned *fail) {
    constexpr int NWV = KM_FF_NT / 64;
    const int lane = threadIdx.x & 63, G = (int)gridDim.x, NWS = G * NWV;
    const int ws = (int)(threadIdx.x >> 6) * G + (int)blockIdx.x;
    int alive = B.nb;
    const long half = B.poff[B.nb];
    for (int j = 0; j < Kmax; j++) {
        KM_STAMP(j, Kmax, 0);
        while (alive > 0 && B.koff[alive] - B.koff[alive - 1] <= j) alive--;
        const int nit = ff_end[alive];
        for (int u = ws; u < nit; u += NWS) {
            const KmFfItem it = items[u];
            KmState s = bin_state(B, it.bin);
            int c;
            if (j == 0) {
                c = s.center[0];  // kmb_ff_start (an earlier launch)
            } else {
                const unsigned long long *pp = s.part + ((j - 1) & 1) * half;
                unsigned long long v[KM_FF_SUBMAX / 64];  // every slot of the bin in flight at once
#pragma unroll
                for (int k = 0; k < KM_FF_SUBMAX / 64; k++)
                    v[k] = lane + 64 * k < it.nsub
                               ? __hip_atomic_load(&pp[lane + 64 * k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : 0ull;
                unsigned long long bb = 0;
#pragma unroll
                for (int k = 0; k < KM_FF_SUBMAX / 64; k++) bb = max(bb, v[k]);
                const unsigned long long w = km_wave_max(bb);
                c = (w == 0) ? -1 : (int)(w & 0xFFFFFFFFull) - 1;
                if (c < 0) {
                    if (it.sub == 0 && lane == 0) *s.err = 1;
                    c = 0;  // the call fails (host checks err); keep the rounds well-defined
                } else {
                    if (it.sub == 0) {
                        for (int a = lane; a < KM_A; a += 64) s.cent[(long)j * KM_A + a] = s.X[(long)c * KM_A + a];
                        if (lane == 0) s.center[j] = c;
                    }
                    if ((c >> 6) % it.nsub == it.sub && (c & 63) == lane) s.used[c] = 1;
                }
            }
            KM_STAMP(j, Kmax, 1);
            uint32_t item[20];
            load_row(s.X + (long)c * KM_A, item);
#ifdef TILER_KM_STAMPS
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            KM_STAMP(j, Kmax, 2);
#endif
            unsigned long long bv = 0;
            int bi = -1;
            // the lane's points 4 at a time: their rows, min-distances and used flags loaded before any is compared
            const long stride = (long)it.nsub * 64;
            for (long i0 = (long)it.sub * 64 + lane; i0 < s.n; i0 += 4 * stride) {
                uint32_t row[4][20];
                unsigned long long mv[4];
                uint8_t uf[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const long i = i0 + k * stride;
                    if (i < s.n) {
                        load_row(s.X + i * KM_A, row[k]);
                        mv[k] = s.mind[i];
                        uf[k] = s.used[i];
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const long i = i0 + k * stride;
                    if (i >= s.n) break;
                    const unsigned long long d = km_dissim(row[k], item);
                    unsigned long long m = mv[k];
                    if (d < m) {  // cmovb: strict-less (kmodes.pas:555-558)
                        m = d;
                        s.mind[i] = m;
                    }
                    if (!uf[k] && m >= bv) {  // ascending i within a lane: '>=' keeps the last
                        bv = m;
                        bi = (int)i;
                    }
                }
            }
            KM_STAMP(j, Kmax, 3);
            const unsigned long long v32 = bv > 0xFFFFFFFFull ? 0xFFFFFFFFull : bv;
            const unsigned long long best = km_wave_max(bi < 0 ? 0ull : ((v32 << 32) | (unsigned)(bi + 1)));
            KM_STAMP(j, Kmax, 4);
            if (j + 1 >= s.K) continue;  // the bin's last round: no selection (uniform)
            if (lane == 0) __hip_atomic_store(s.part + (j & 1) * half + it.sub, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (j + 1 < Kmax && !km_grid_sync(bar, (unsigned)(j + 1), fail, Kmax)) return;
    }
}

#ifdef TILER_KM_STAMPS
extern "C" int tiler_debug_km_stamps(void *out) {  // study build: the stamps of the last farthest-first launch
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_km_stamps), sizeof(g_km_stamps)) == hipSuccess ? 0 : -1;
}
#endif

// resident workgroups for kmb_ff_persist3: one per CU (0: not placeable -> per-launch rounds)
static int ff_persist_grid() {
    static const int g = [] {
        int dev = 0, ncu = 0, per = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)kmb_ff_persist3, KM_FF_NT, 0) != hipSuccess ||
            per <= 0 || ncu <= 0)
            return 0;
        return ncu;
    }();
    return g;
}

// ---- DoKModes medoid choice (main.pas:4231-4253): per cluster j with members, the member minimising
// dissim(member, centroid_j) (GetMinMatchingDissim(ToMerge, LocCentroids[j]) -> ties: last member) ----
__global__ __launch_bounds__(256) void kmb_medoid(const uint8_t *X, const int32_t *boff, const int32_t *koff, int nb,
                                                  long N, const int32_t *labels, const uint8_t *cent,
                                                  unsigned long long *best, int32_t *counts) {
    for (long g = (long)blockIdx.x * 256 + threadIdx.x; g < N; g += (long)gridDim.x * 256) {
        const int b = bin_of(boff, nb, g);
        const long i = g - boff[b];
        const long j = koff[b] + labels[g];
        uint32_t row[20], item[20];
        load_row(X + g * KM_A, row);
        load_row(cent + j * KM_A, item);
        const unsigned long long d = km_dissim(row, item);
        atomicMin(&best[j], (d << 32) | (0xFFFFFFFFu - (unsigned)i));
        atomicAdd(&counts[j], 1);
    }
}

// centroid splits of an assignment block: ~64 centroids per block, so a chunk of the largest bin alone
// still spreads over the chip (results merge by atomicMin)
__host__ __device__ inline int csplit_of(int K) {
    const int c = (K + 63) / 64;
    return c < 1 ? 1 : (c > 128 ? 128 : c);
}

// One iteration's work list, written on the device, one workgroup per chunk step c: every active bin's assignment
// items (256 points x one centroid split each, in the active order), then one seq item per bin present at the step --
// the list the host used to build and upload whenever the active set changed (up to 1.3 ms of GPU idle each time on
// C4, profiles/r06/kt_kmodes_gaps_r06o.json).  step_off[c]: the first item of step c.
static constexpr int KM_GEN_MAXB = 4096;  // active bins the generator takes (beyond: the host builds the list)
__global__ __launch_bounds__(256) void kmb_gen_items(KmBatch B, const int *act, int nact, const int *step_off,
                                                     KmAsgItem *out) {
    __shared__ int s_off[KM_GEN_MAXB + 1];
    const int c = blockIdx.x, p0 = c * KM_BIN;
    if (threadIdx.x == 0) {
        int o = 0;
        for (int j = 0; j < nact; j++) {
            const int r = act[j], n = B.boff[r + 1] - B.boff[r];
            s_off[j] = o;
            if (p0 < n) o += ((min(n - p0, KM_BIN) + 255) / 256) * csplit_of(B.koff[r + 1] - B.koff[r]);
        }
        s_off[nact] = o;
    }
    __syncthreads();
    KmAsgItem *dst = out + step_off[c];
    for (int j = 0; j < nact; j++) {
        const int cnt = s_off[j + 1] - s_off[j];
        if (cnt == 0) continue;  // bin absent at this step (uniform)
        const int r = act[j], n = B.boff[r + 1] - B.boff[r], K = B.koff[r + 1] - B.koff[r];
        const int p1 = min(n, p0 + KM_BIN), cs = csplit_of(K), per = (K + cs - 1) / cs;
        for (int e = threadIdx.x; e < cnt; e += 256) {
            const int qi = e / cs, cc = e - qi * cs, q0 = p0 + qi * 256;
            KmAsgItem it;
            it.bin = r;
            it.p0 = q0;
            it.p1 = min(p1, q0 + 256);
            it.c0 = cc * per;
            it.c1 = min(K, (cc + 1) * per);
            it.pad[0] = it.pad[1] = it.pad[2] = 0;
            dst[s_off[j] + e] = it;
        }
    }
    if (threadIdx.x == 0) {  // the seq items, in the active order
        int k = s_off[nact];
        for (int j = 0; j < nact; j++) {
            const int r = act[j], n = B.boff[r + 1] - B.boff[r];
            if (p0 >= n) continue;
            KmAsgItem it{};
            it.bin = r;  // KmSeqItem view: bin, p0, p1
            it.p0 = p0;
            it.p1 = min(n, p0 + KM_BIN);
            dst[k++] = it;
        }
    }
}

// ---- host driver ----

// counters of the last batch (tiler_kmodes_last_stats): assignment (point, centroid) pairs and dependent chunk steps
static std::atomic<long long> g_km_last_pairs{0}, g_km_last_steps{0};
static std::atomic<int> g_km_force_ff_fail{0};  // tiler_debug_kmodes_ff_fallback
void kmodes_force_ff_fallback(int on) { g_km_force_ff_fail.store(on != 0); }
void kmodes_last_stats(long long *pairs, long long *steps) {
    if (pairs) *pairs = g_km_last_pairs.load();
    if (steps) *steps = g_km_last_steps.load();
}

int kmodes_batch_dev(const uint8_t *d_X, const int32_t *h_boff, int nb, const int32_t *h_k, const int32_t *h_start,
                     int n_modalities, int32_t *d_labels, uint8_t *d_centroids, int32_t *h_iter, uint64_t *h_cost,
                     hipStream_t st) {
    if (nb <= 0 || !h_boff || !h_k || !h_start || n_modalities <= 0 || n_modalities > 256) {
        set_error("kmodes: invalid arguments (need bins, cluster counts, starts, 0 < modalities <= 256)");
        return -1;
    }
    if (((uintptr_t)d_X & 15) != 0) {
        set_error("kmodes: X must be 16-byte aligned");
        return -1;
    }
    for (int b = 0; b < nb; b++) {
        const int n = h_boff[b + 1] - h_boff[b];
        if (n <= 0 || h_k[b] <= 0 || h_k[b] > n || h_start[b] < 0 || h_start[b] >= n) {
            set_error("kmodes: invalid bin (need 0 < k <= n, 0 <= start < n)");
            return -1;
        }
    }
    // process bins in descending K (ties: size) so the bins alive in farthest-first round j are a prefix;
    // the caller's arrays stay in caller order: the permutation only renames bins inside this call
    std::vector<int> ord(nb);
    for (int b = 0; b < nb; b++) ord[b] = b;
    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return h_k[x] > h_k[y]; });
    std::vector<int32_t> koff_c(nb + 1, 0);  // caller-order cluster offsets (output layout)
    for (int b = 0; b < nb; b++) koff_c[b + 1] = koff_c[b] + h_k[b];
    std::vector<int32_t> boff(nb + 1, 0), koff(nb + 1, 0), poff(nb + 1, 0), start(nb), Kv(nb), nv(nb);
    for (int r = 0; r < nb; r++) {
        const int b = ord[r];
        nv[r] = h_boff[b + 1] - h_boff[b];
        Kv[r] = h_k[b];
        start[r] = h_start[b];
        boff[r + 1] = boff[r] + nv[r];
        koff[r + 1] = koff[r] + Kv[r];
        poff[r + 1] = poff[r] + std::min(KM_FF_SUBMAX, (nv[r] + 255) / 256);  // kmb_ff_persist3's wave items
    }
    const long N = boff[nb], Ktot = koff[nb];
    const int M = n_modalities;
    long long km_pairs = 0, km_steps = 0;  // tiler_kmodes_last_stats
    // device workspace
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    };
    const size_t o_X = carve((size_t)N * KM_A), o_boff = carve((nb + 1) * 4), o_koff = carve((nb + 1) * 4),
                 o_poff = carve((nb + 1) * 4), o_start = carve(nb * 4), o_memb = carve((size_t)N * 4),
                 o_cent = carve((size_t)Ktot * KM_A), o_freq = carve((size_t)Ktot * KM_A * M * 4),
                 o_csize = carve((size_t)Ktot * 4), o_mind = carve((size_t)N * 8), o_used = carve(N),
                 o_part = carve((size_t)poff[nb] * 16), o_center = carve((size_t)Ktot * 4), o_akey = carve((size_t)N * 8),
                 o_seed = carve(nb * 4), o_cost = carve(nb * 8), o_moves = carve(nb * 4), o_err = carve(nb * 4),
                 o_ffd = carve(nb * 4), o_rand = carve((size_t)Ktot * KM_A * 4), o_bar = carve(2304),
                 o_bad = carve(4), o_mvl = carve((size_t)nb * 2 * KM_BIN * 16), o_mvn = carve((size_t)nb * 4);
    // assignment with <= 16 modalities (kmb_assign16): prepared point rows, at most 8,192 centroids per workgroup
    bool use16 = M <= 16;
    for (int r = 0; r < nb; r++) use16 = use16 && (Kv[r] + csplit_of(Kv[r]) - 1) / csplit_of(Kv[r]) <= 8192;
    const size_t o_Xp = carve(use16 ? (size_t)N * KM_PW * 4 : 0), o_items = carve(0);
    char *buf = nullptr;
    // the largest work list: one iteration's chunk items for every bin
    size_t max_items = 0;
    for (int r = 0; r < nb; r++) {
        const int nch = (nv[r] + KM_BIN - 1) / KM_BIN;
        max_items += (size_t)nch * ((KM_BIN + 255) / 256) * csplit_of(Kv[r]) + nch;
        max_items += (size_t)((nv[r] + 255) / 256) * csplit_of(Kv[r]);
    }
    int max_steps = 0;  // chunk steps of the largest bin (the device work list's per-step offsets)
    for (int r = 0; r < nb; r++) max_steps = std::max(max_steps, (nv[r] + KM_BIN - 1) / KM_BIN);
    const size_t item_bytes = (max_items + (size_t)poff[nb] + 64) * sizeof(KmAsgItem) +
                              (size_t)(nb + 1 + max_steps) * 4 + 256;
    // farthest-first: one persistent launch for every round (kmb_ff_persist3) unless it cannot be placed
    const int g_ff = ff_persist_grid();
    TILER_HIP_CHECK(hipMalloc((void **)&buf, off + item_bytes));
    char *items = buf + o_items;
    KmBatch B;
    B.X = (const uint8_t *)(buf + o_X);
    B.boff = (const int32_t *)(buf + o_boff);
    B.koff = (const int32_t *)(buf + o_koff);
    B.poff = (const int32_t *)(buf + o_poff);
    B.nb = nb;
    B.M = M;
    B.memb = (int32_t *)(buf + o_memb);
    B.cent = (uint8_t *)(buf + o_cent);
    B.freq = (int32_t *)(buf + o_freq);
    B.csize = (int32_t *)(buf + o_csize);
    B.mind = (unsigned long long *)(buf + o_mind);
    B.used = (uint8_t *)(buf + o_used);
    B.part = (unsigned long long *)(buf + o_part);
    B.center = (int32_t *)(buf + o_center);
    B.akey = (unsigned long long *)(buf + o_akey);
    B.seed = (unsigned *)(buf + o_seed);
    B.cost = (unsigned long long *)(buf + o_cost);
    B.moves = (int *)(buf + o_moves);
    B.err = (int *)(buf + o_err);
    B.ffdone = (int *)(buf + o_ffd);
    B.mvl = (int4 *)(buf + o_mvl);
    B.mvn = (int *)(buf + o_mvn);
    B.dbg = nullptr;
    int32_t *rand_rows = (int32_t *)(buf + o_rand);
    int rc = -1;
    std::vector<char> hitems;
    auto upload_at = [&](size_t at, const void *src, size_t bytes) -> int {  // work list -> device (synchronous:
        TILER_HIP_CHECK(hipMemcpyAsync(items + at, src, bytes, hipMemcpyHostToDevice, st));  // the host buffer is reused)
        TILER_HIP_CHECK(hipStreamSynchronize(st));
        return 0;
    };
    auto upload = [&](const void *src, size_t bytes) -> int { return upload_at(0, src, bytes); };
    do {
        // permuted copy of X (bins contiguous in K order) + metadata
        for (int r = 0; r < nb; r++)
            if (hipMemcpyAsync(buf + o_X + (size_t)boff[r] * KM_A, d_X + (size_t)h_boff[ord[r]] * KM_A,
                               (size_t)nv[r] * KM_A, hipMemcpyDeviceToDevice, st) != hipSuccess)
                goto fail;
        if (hipMemcpyAsync(buf + o_boff, boff.data(), (nb + 1) * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(buf + o_koff, koff.data(), (nb + 1) * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(buf + o_poff, poff.data(), (nb + 1) * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(buf + o_start, start.data(), nb * 4, hipMemcpyHostToDevice, st) != hipSuccess)
            goto fail;
        {
            std::vector<unsigned> seeds(nb, 0x42381337u);  // ComputeKModes kmodes.pas:930, per call (= per bin)
            if (hipMemcpyAsync(B.seed, seeds.data(), nb * 4, hipMemcpyHostToDevice, st) != hipSuccess) goto fail;
            unsigned bad = 0;
            if (use16) {
                if (hipMemsetAsync(buf + o_bad, 0, 4, st) != hipSuccess) goto fail;
                hipLaunchKernelGGL(kmb_prep_points, dim3((unsigned)std::min<long>(4096, (N + 255) / 256)), dim3(256), 0, st,
                                   B.X, N, (uint4 *)(buf + o_Xp), (unsigned *)(buf + o_bad));
                if (hipGetLastError() != hipSuccess ||
                    hipMemcpyAsync(&bad, buf + o_bad, 4, hipMemcpyDeviceToHost, st) != hipSuccess)
                    goto fail;
            }
            if (hipStreamSynchronize(st) != hipSuccess) goto fail;
            use16 = use16 && bad == 0;  // a byte >= 16 (outside the declared modalities): the general kernel
        }
        // InitFarthestFirst, all bins round by round
        {
            std::vector<KmFfItem> ff;
            std::vector<int> ff_end(nb + 1, 0);  // items of bins [0, r) = ff[0, ff_end[r])
            for (int r = 0; r < nb; r++) {
                const int ns = poff[r + 1] - poff[r];
                for (int sb = 0; sb < ns; sb++) ff.push_back({r, sb, ns, 0});
                ff_end[r + 1] = (int)ff.size();
            }
            const size_t fb = ff.size() * sizeof(KmFfItem);
            {
                std::vector<char> up(fb + (nb + 1) * 4);
                memcpy(up.data(), ff.data(), fb);
                memcpy(up.data() + fb, ff_end.data(), (nb + 1) * 4);
                if (upload(up.data(), up.size())) goto fail;
            }
            auto ff_init = [&]() -> int {  // the state every farthest-first run starts from
                if (hipMemsetAsync(B.err, 0, nb * 4, st) != hipSuccess || hipMemsetAsync(B.ffdone, 0, nb * 4, st) != hipSuccess ||
                    hipMemsetAsync(B.mind, 0xff, (size_t)N * 8, st) != hipSuccess || hipMemsetAsync(B.used, 0, N, st) != hipSuccess ||
                    hipMemsetAsync(B.cent, 0xff, (size_t)Ktot * KM_A, st) != hipSuccess)
                    return -1;
                hipLaunchKernelGGL(kmb_ff_start, dim3((nb + 63) / 64), dim3(64), 0, st, B, (const int32_t *)(buf + o_start));
                return hipGetLastError() == hipSuccess ? 0 : -1;
            };
            if (ff_init()) goto fail;
            bool done = false;
            if (g_ff > 0) {
                unsigned *bar = (unsigned *)(buf + o_bar), *ffail = bar + 544;
                if (hipMemsetAsync(bar, 0, 2304, st) != hipSuccess) goto fail;  // counters, generations, fail word
                if (g_km_force_ff_fail.load() &&  // test hook: every barrier gives up at once (round 0 runs)
                    hipMemsetAsync(ffail, 0x01, 1, st) != hipSuccess)
                    goto fail;
                {
                    KTimer tm("kmodes_init", st);
                    // every item selects the centre after the barrier (r03zo: C4 122 -> 102 ms); wave items (r06)
                    hipLaunchKernelGGL(kmb_ff_persist3, dim3(g_ff), dim3(KM_FF_NT), 0, st, B, (const KmFfItem *)items,
                                       (const int *)(items + fb), Kv[0], bar, ffail);
                }
                unsigned hf = 1;
                if (hipGetLastError() != hipSuccess ||
                    hipMemcpyAsync(&hf, ffail, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                    hipStreamSynchronize(st) != hipSuccess)
                    goto fail;
                done = hf == 0;
                if (!done && ff_init()) goto fail;  // a barrier gave up: rerun the rounds one launch each
            }
            if (!done) {
                KTimer tm("kmodes_init", st);
                int alive = nb;
                for (int j = 0; j < Kv[0]; j++) {
                    while (alive > 0 && Kv[alive - 1] <= j) alive--;
                    hipLaunchKernelGGL(kmb_ff_round, dim3(ff_end[alive]), dim3(256), 0, st, B, (const KmFfItem *)items, j);
                }
            }
        }
        if (hipGetLastError() != hipSuccess) goto fail;
        // initial assignment (all points) + histograms + modes
        {
            std::vector<KmAsgItem> as;
            for (int r = 0; r < nb; r++) {
                const int cs = csplit_of(Kv[r]), per = (Kv[r] + cs - 1) / cs;
                for (int p0 = 0; p0 < nv[r]; p0 += 256)
                    for (int c = 0; c < cs; c++)
                        as.push_back({r, p0, std::min(nv[r], p0 + 256), c * per, std::min(Kv[r], (c + 1) * per), {0, 0, 0}});
            }
            for (const KmAsgItem &it : as) km_pairs += (long long)(it.p1 - it.p0) * (it.c1 - it.c0);
            if (hipMemsetAsync(B.akey, 0xff, (size_t)N * 8, st) != hipSuccess) goto fail;
            if (upload(as.data(), as.size() * sizeof(KmAsgItem))) goto fail;
            KTimer tm("kmodes_assign", st);
            if (use16)
                hipLaunchKernelGGL(kmb_assign16<KM_A16_G>, dim3((unsigned)as.size(), KM_ASUB / KM_A16_G), dim3(256 * KM_A16_G), 0, st, B,
                                   (const KmAsgItem *)items, (const uint4 *)(buf + o_Xp));
            else
                hipLaunchKernelGGL(kmb_assign, dim3((unsigned)as.size(), KM_ASUB), dim3(256), 0, st, B, (const KmAsgItem *)items);
        }
        if (hipMemsetAsync(B.csize, 0, (size_t)Ktot * 4, st) != hipSuccess ||
            hipMemsetAsync(B.freq, 0, (size_t)Ktot * KM_A * M * 4, st) != hipSuccess)
            goto fail;
        hipLaunchKernelGGL(kmb_init_hist, dim3((unsigned)std::min<long>(4096, (N + 255) / 256)), dim3(256), 0, st, B, N);
        hipLaunchKernelGGL(kmb_init_modes, dim3((nb + 63) / 64), dim3(64), 0, st, B, rand_rows);
        hipLaunchKernelGGL(kmb_init_modes2, dim3((unsigned)std::min<long>(8192, (Ktot * KM_A + 255) / 256)), dim3(256), 0,
                           st, B, (const int32_t *)rand_rows, Ktot);
        if (hipGetLastError() != hipSuccess) goto fail;
        // iterations (kmodes.pas:1023-1039), each bin until its cost stops decreasing or nothing moves
        {
            std::vector<int> active(nb);
            for (int r = 0; r < nb; r++) active[r] = r;
            std::vector<unsigned long long> best_cost(nb, ~0ull), hcost(nb);
            std::vector<int> hmoves(nb), herr(nb), iters(nb, 0);
            // the work list depends only on the active bins: an iteration whose set is unchanged (from iteration ~13
            // on at C4 only the largest bin is left) reuses the list already on the device.  Rebuilding and uploading
            // the largest bin's ~73k items took 0.5-1.1 ms of GPU idle per iteration, 21 ms per C4 call
            // (profiles/r06/kt_kmodes_gaps.json)
            std::vector<int> prev_active;
            std::vector<char> hstat(o_err + (size_t)nb * 4 - o_cost);
            std::vector<std::pair<int, int>> steps;  // (assign items, seq items) per chunk step
            size_t wb = 0;
            long long it_pairs = 0;
            while (!active.empty()) {
                if (active != prev_active && (int)active.size() <= KM_GEN_MAXB) {
                    // work list of this iteration (per chunk step c, the assign items then the seq items), written by
                    // kmb_gen_items from the active bins and the per-step offsets computed here
                    steps.clear();
                    std::vector<int> hdr(active);
                    int maxch = 0;
                    for (int r : active) maxch = std::max(maxch, (nv[r] + KM_BIN - 1) / KM_BIN);
                    size_t total = 0;
                    it_pairs = 0;
                    for (int c = 0; c < maxch; c++) {
                        int na = 0, ns = 0;
                        for (int r : active) {
                            const int p0 = c * KM_BIN;
                            if (p0 >= nv[r]) continue;
                            const int pts = std::min(nv[r] - p0, KM_BIN);
                            na += ((pts + 255) / 256) * csplit_of(Kv[r]);
                            ns++;
                            it_pairs += (long long)pts * Kv[r];  // (point, centroid) pairs the assignment evaluates
                        }
                        steps.push_back({na, ns});
                        hdr.push_back((int)total);
                        total += (size_t)na + ns;
                    }
                    wb = total * sizeof(KmAsgItem);  // the active bins follow the list (kmb_iter_reset), then the offsets
                    if (upload_at(wb, hdr.data(), hdr.size() * 4)) goto fail;
                    hipLaunchKernelGGL(kmb_gen_items, dim3((unsigned)maxch), dim3(256), 0, st, B, (const int *)(items + wb),
                                       (int)active.size(), (const int *)(items + wb) + active.size(), (KmAsgItem *)items);
                    if (hipGetLastError() != hipSuccess) goto fail;
                    prev_active = active;
                } else if (active != prev_active) {  // more bins than the generator takes: built here
                    std::vector<KmAsgItem> wl;
                    steps.clear();
                    const int qstep = 256;  // points per assignment item
                    int maxch = 0;
                    for (int r : active) maxch = std::max(maxch, (nv[r] + KM_BIN - 1) / KM_BIN);
                    for (int c = 0; c < maxch; c++) {
                        int na = 0, ns = 0;
                        for (int r : active) {
                            const int p0 = c * KM_BIN;
                            if (p0 >= nv[r]) continue;
                            const int p1 = std::min(nv[r], p0 + KM_BIN), cs = csplit_of(Kv[r]), per = (Kv[r] + cs - 1) / cs;
                            for (int q0 = p0; q0 < p1; q0 += qstep)
                                for (int cc = 0; cc < cs; cc++, na++)
                                    wl.push_back({r, q0, std::min(p1, q0 + qstep), cc * per, std::min(Kv[r], (cc + 1) * per), {0, 0, 0}});
                        }
                        for (int r : active) {
                            const int p0 = c * KM_BIN;
                            if (p0 >= nv[r]) continue;
                            KmAsgItem e{};
                            reinterpret_cast<KmSeqItem &>(e) = {r, p0, std::min(nv[r], p0 + KM_BIN), 0};
                            wl.push_back(e);
                            ns++;
                        }
                        steps.push_back({na, ns});
                    }
                    {
                        size_t q = 0;
                        it_pairs = 0;
                        for (const auto &sp : steps) {  // (point, centroid) pairs the assignment launches evaluate
                            for (int i = 0; i < sp.first; i++, q++)
                                it_pairs += (long long)(wl[q].p1 - wl[q].p0) * (wl[q].c1 - wl[q].c0);
                            q += sp.second;
                        }
                    }
                    // the work list, then the active bins (one reset launch, not three memsets per bin)
                    wb = wl.size() * sizeof(KmAsgItem);
                    hitems.resize(wb + active.size() * 4);
                    memcpy(hitems.data(), wl.data(), wb);
                    memcpy(hitems.data() + wb, active.data(), active.size() * 4);
                    if (upload(hitems.data(), hitems.size())) goto fail;
                    prev_active = active;
                }
                km_pairs += it_pairs;
                km_steps += (long long)steps.size();
                {
                    int maxn = 0;
                    for (int r : active) {
                        iters[r]++;
                        maxn = std::max(maxn, nv[r]);
                    }
                    hipLaunchKernelGGL(kmb_iter_reset, dim3((unsigned)std::min(64, (maxn + 255) / 256), (unsigned)active.size()),
                                       dim3(256), 0, st, B, (const int *)(items + wb));
                }
                {
                    size_t pos = 0;
                    for (const auto &sp : steps) {
                        {
                            KTimer tm("kmodes_assign", st);
                            if (use16)
                                hipLaunchKernelGGL(kmb_assign16<KM_A16_G>, dim3(sp.first, KM_ASUB / KM_A16_G), dim3(256 * KM_A16_G), 0, st, B,
                                                   (const KmAsgItem *)items + pos, (const uint4 *)(buf + o_Xp));
                            else
                                hipLaunchKernelGGL(kmb_assign, dim3(sp.first, KM_ASUB), dim3(256), 0, st, B,
                                                   (const KmAsgItem *)items + pos);
                        }
                        pos += sp.first;
                        // seq items are KmSeqItem views of KmAsgItem slots: stride 32 bytes
                        {
                            KTimer tm("kmodes_seq", st);
                            // the decisions (one workgroup per bin), then the attribute updates over KM_APPLY_SLICES each
                            hipLaunchKernelGGL((kmb_seq_strided<KM_SEQ_NT, KM_SEQ_W, true>), dim3(sp.second),
                                               dim3(KM_SEQ_NT), 0, st, B, (const KmAsgItem *)items + pos);
                        }
                        {
                            KTimer tm("kmodes_apply", st);
                            hipLaunchKernelGGL((kmb_seq_apply<KM_APPLY_SLICES>), dim3(sp.second, KM_APPLY_SLICES),
                                               dim3(32 * (KM_A / KM_APPLY_SLICES)), 0, st, B, (const KmAsgItem *)items + pos);
                        }
                        pos += sp.second;
                    }
                }
                if (hipGetLastError() != hipSuccess) goto fail;
                // cost, moves and err are consecutive in the workspace: one read-back per iteration
                if (hipMemcpyAsync(hstat.data(), buf + o_cost, hstat.size(), hipMemcpyDeviceToHost, st) != hipSuccess ||
                    hipStreamSynchronize(st) != hipSuccess)
                    goto fail;
                memcpy(hcost.data(), hstat.data(), nb * 8);
                memcpy(hmoves.data(), hstat.data() + (o_moves - o_cost), nb * 4);
                memcpy(herr.data(), hstat.data() + (o_err - o_cost), nb * 4);
                std::vector<int> still;
                for (int r : active) {
                    if (herr[r]) {
                        set_error("kmodes: farthest-first ran out of points (k > n)");
                        rc = -2;
                        goto fail;
                    }
                    const bool conv = (hcost[r] >= best_cost[r]) || (hmoves[r] == 0);
                    best_cost[r] = hcost[r];
                    if (!conv) still.push_back(r);
                }
                active.swap(still);
            }
            for (int r = 0; r < nb; r++) {
                if (h_iter) h_iter[ord[r]] = iters[r];
                if (h_cost) h_cost[ord[r]] = best_cost[r];
            }
        }
        // outputs in caller order: labels (bin-local) and centroids
        for (int r = 0; r < nb; r++) {
            const int b = ord[r];
            if (hipMemcpyAsync(d_labels + h_boff[b], B.memb + boff[r], (size_t)nv[r] * 4, hipMemcpyDeviceToDevice, st) !=
                    hipSuccess ||
                hipMemcpyAsync(d_centroids + (size_t)koff_c[b] * KM_A, B.cent + (size_t)koff[r] * KM_A, (size_t)Kv[r] * KM_A,
                               hipMemcpyDeviceToDevice, st) != hipSuccess)
                goto fail;
        }
        if (hipStreamSynchronize(st) != hipSuccess) goto fail;
        g_km_last_pairs.store(km_pairs);
        g_km_last_steps.store(km_steps);
        rc = 0;
    } while (0);
fail:
    if (rc == -1) set_error("kmodes: HIP failure");
    if (B.dbg) (void)hipFree(B.dbg);
    (void)hipFree(buf);
    return rc < 0 ? -1 : 0;
}

int kmodes_compute_dev(const uint8_t *d_X, int n, int k, int start_point, int n_modalities, int32_t *d_labels,
                       uint8_t *d_centroids, int *n_iter, uint64_t *cost, hipStream_t st) {
    const int32_t boff[2] = {0, n}, kk[1] = {k}, sp[1] = {start_point};
    int32_t it = 0;
    uint64_t c = 0;
    if (kmodes_batch_dev(d_X, boff, 1, kk, sp, n_modalities, d_labels, d_centroids, &it, &c, st)) return -1;
    if (n_iter) *n_iter = it;
    if (cost) *cost = c;
    return 0;
}

int kmodes_medoids_batch_dev(const uint8_t *d_X, const int32_t *h_boff, int nb, const int32_t *h_k,
                             const int32_t *d_labels, const uint8_t *d_centroids, int32_t *h_medoid, int32_t *h_counts,
                             hipStream_t st) {
    std::vector<int32_t> koff(nb + 1, 0);
    for (int b = 0; b < nb; b++) koff[b + 1] = koff[b] + h_k[b];
    const long N = h_boff[nb], K = koff[nb];
    char *buf = nullptr;
    const size_t oB = 0, oN = (size_t)K * 8, oBo = oN + (((size_t)K * 4 + 255) & ~(size_t)255), oKo = oBo + ((nb + 1) * 4 + 256);
    TILER_HIP_CHECK(hipMalloc((void **)&buf, oKo + (nb + 1) * 4 + 256));
    int rc = -1;
    do {
        if (hipMemsetAsync(buf + oB, 0xff, (size_t)K * 8, st) != hipSuccess) break;
        if (hipMemsetAsync(buf + oN, 0, (size_t)K * 4, st) != hipSuccess) break;
        if (hipMemcpyAsync(buf + oBo, h_boff, (nb + 1) * 4, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (hipMemcpyAsync(buf + oKo, koff.data(), (nb + 1) * 4, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (N > 0)
            hipLaunchKernelGGL(kmb_medoid, dim3((unsigned)std::min<long>(4096, (N + 255) / 256)), dim3(256), 0, st, d_X,
                               (const int32_t *)(buf + oBo), (const int32_t *)(buf + oKo), nb, N, d_labels, d_centroids,
                               (unsigned long long *)(buf + oB), (int32_t *)(buf + oN));
        if (hipGetLastError() != hipSuccess) break;
        std::vector<unsigned long long> b(K);
        if (hipMemcpyAsync(b.data(), buf + oB, (size_t)K * 8, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipMemcpyAsync(h_counts, buf + oN, (size_t)K * 4, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipStreamSynchronize(st) != hipSuccess) break;
        for (long j = 0; j < K; j++) h_medoid[j] = h_counts[j] > 0 ? (int32_t)(0xFFFFFFFFu - (unsigned)(b[j] & 0xFFFFFFFFull)) : -1;
        rc = 0;
    } while (0);
    if (rc) set_error("kmodes_medoids: HIP failure");
    (void)hipFree(buf);
    return rc;
}

// host-buffer entry points: stage through a private stream
template <class F>
static int with_host_batch(const uint8_t *X, long N, long K, int32_t *labels_out, uint8_t *cent_out, F run) {
    uint8_t *d_X = nullptr, *d_c = nullptr;
    int32_t *d_l = nullptr;
    hipStream_t st = nullptr;
    TILER_HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    int rc = -1;
    do {
        if (hipMalloc((void **)&d_X, (size_t)std::max(N, 1L) * KM_A) != hipSuccess) break;
        if (hipMalloc((void **)&d_c, (size_t)std::max(K, 1L) * KM_A) != hipSuccess) break;
        if (hipMalloc((void **)&d_l, (size_t)std::max(N, 1L) * 4) != hipSuccess) break;
        if (N > 0 && hipMemcpyAsync(d_X, X, (size_t)N * KM_A, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (!labels_out && !cent_out) {  // medoids: labels/centroids are inputs, results go to host in run()
            rc = run(d_X, d_l, d_c, st) ? -2 : 0;
            break;
        }
        if (run(d_X, d_l, d_c, st)) {
            rc = -2;
            break;
        }
        if (hipMemcpyAsync(labels_out, d_l, (size_t)N * 4, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipMemcpyAsync(cent_out, d_c, (size_t)K * KM_A, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipStreamSynchronize(st) != hipSuccess) break;
        rc = 0;
    } while (0);
    if (rc == -1) set_error("kmodes: HIP failure");
    (void)hipFree(d_X);
    (void)hipFree(d_c);
    (void)hipFree(d_l);
    (void)hipStreamDestroy(st);
    return rc < 0 ? -1 : 0;
}

int kmodes_batch_host(const uint8_t *X, const int32_t *boff, int nb, const int32_t *k, const int32_t *start,
                      int n_modalities, int32_t *labels, uint8_t *centroids, int32_t *n_iter, uint64_t *cost) {
    if (!X || !boff || nb <= 0 || !k || !start || !labels || !centroids) {
        set_error("kmodes: null buffer");
        return -1;
    }
    long K = 0;
    for (int b = 0; b < nb; b++) K += k[b];
    return with_host_batch(X, boff[nb], K, labels, centroids, [&](uint8_t *dX, int32_t *dl, uint8_t *dc, hipStream_t st) {
        return kmodes_batch_dev(dX, boff, nb, k, start, n_modalities, dl, dc, n_iter, cost, st);
    });
}

int kmodes_medoids_batch_host(const uint8_t *X, const int32_t *boff, int nb, const int32_t *k, const int32_t *labels,
                              const uint8_t *centroids, int32_t *medoid, int32_t *counts) {
    if (!X || !boff || nb <= 0 || !k || !labels || !centroids || !medoid || !counts) {
        set_error("kmodes_medoids: invalid arguments");
        return -1;
    }
    long K = 0;
    for (int b = 0; b < nb; b++) K += k[b];
    for (int b = 0; b < nb; b++)
        for (int i = boff[b]; i < boff[b + 1]; i++)
            if (labels[i] < 0 || labels[i] >= k[b]) {
                set_error("kmodes_medoids: label out of range");
                return -1;
            }
    return with_host_batch(X, boff[nb], K, nullptr, nullptr, [&](uint8_t *dX, int32_t *dl, uint8_t *dc, hipStream_t st) {
        TILER_HIP_CHECK(hipMemcpyAsync(dl, labels, (size_t)boff[nb] * 4, hipMemcpyHostToDevice, st));
        TILER_HIP_CHECK(hipMemcpyAsync(dc, centroids, (size_t)K * KM_A, hipMemcpyHostToDevice, st));
        return kmodes_medoids_batch_dev(dX, boff, nb, k, dl, dc, medoid, counts, st);
    });
}

int kmodes_medoids_host(const uint8_t *X, int n, const int32_t *labels, const uint8_t *centroids, int k,
                        int32_t *medoid, int32_t *counts) {
    if (n < 0 || k <= 0) {
        set_error("kmodes_medoids: invalid arguments");
        return -1;
    }
    if (n == 0) {
        for (int j = 0; j < k; j++) {
            medoid[j] = -1;
            counts[j] = 0;
        }
        return 0;
    }
    const int32_t boff[2] = {0, n}, kk[1] = {k};
    return kmodes_medoids_batch_host(X, boff, 1, kk, labels, centroids, medoid, counts);
}

int kmodes_compute_host(const uint8_t *X, int n, int nattr, int k, int start_point, int n_modalities,
                        int32_t *labels, uint8_t *centroids, int *n_iter, uint64_t *cost) {
    if (nattr != KM_A) {
        set_error("kmodes: nattr must be 80 (cKModesFeatureCount; the asm dissimilarity is 80-byte wide)");
        return -1;
    }
    if (n <= 0 || k <= 0 || k > n || start_point < 0 || start_point >= n || n_modalities <= 0 || n_modalities > 256) {
        set_error("kmodes: invalid arguments (need 0 < k <= n, 0 <= start < n, 0 < modalities <= 256)");
        return -1;
    }
    const int32_t boff[2] = {0, n}, kk[1] = {k}, sp[1] = {start_point};
    int32_t it = 0;
    uint64_t c = 0;
    if (kmodes_batch_host(X, boff, 1, kk, sp, n_modalities, labels, centroids, &it, &c)) return -1;
    if (n_iter) *n_iter = it;
    if (cost) *cost = c;
    return k;
}

}  // namespace tiler
