// orbit.hip -- mirror-orbit FrameTiling search on gfx950 (see orbit.hpp for the algebra).
//
//   orbit_eq_kernel        device check: which of the next 3 candidates equal S_m row_j bit for bit
//   (host)                 greedy grouping of consecutive candidates into orbits (base + mirror slots)
//   orbit_prep_kernel      c' = U c_base (dataset) / q' = U' q (queries): fp64 transform -> fp16 MFMA
//                          fragments + row-major fp16 + norms and rounding-error statistics
//   nn_orbit_shortlist     v_mfma_f32_32x32x16_f16, 12 k-steps = 4 isotypic blocks of 3: per (query,
//                          tile) four 48-d partial dots d_x in 4 accumulators (d_0 seeded with
//                          -||c||^2/2).  u = d_0 + |d_1| + |d_2| + |d_3| bounds the 4 mirror values
//                          q.(S_m c) - ||c||^2/2 from above; each lane keeps its L best 4-tile
//                          sub-blocks by max u (key = -2u).
//   nn_orbit_rescore       per query: re-key the kept sub-blocks from the fp16 rows, derive the exact
//                          threshold from a real reference distance, rescore every candidate whose key
//                          can reach it with the reference fp32 sequential distance, pick (dist, index).
//                          A list that may have dropped a needed entry sends the query to the generic
//                          tier-2 collect pass (nn_search.hip) with the threshold in its key domain.
#include <float.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "kdorder_dev.hpp"
#include "nn_dev.hpp"
#include "psyv_dev.hpp"
#include "orbit.hpp"
#include "orbit_map_gen.hpp"

namespace tiler {

static constexpr int OD = 192;  // descriptor dimension (cTileDCTSize, main.pas:44)
static constexpr int OS = 12;   // k-steps of 16 (4 isotypic blocks x 3)
#ifndef ORB_XBATCH
#define ORB_XBATCH 3
#endif
#ifndef ORB_RS_WAVES
#define ORB_RS_WAVES 6  // nn_orbit_rescore_kernel: waves per SIMD it is compiled for
#endif
#ifndef ORB_STG_ROWS
#define ORB_STG_ROWS 4  // nn_orbit_rescore_kernel: candidate rows staged in LDS per pass
#endif
#ifndef ORB_PR_WAVES
#define ORB_PR_WAVES 0  // nn_orbit_pairs_kernel: waves per SIMD it is compiled for (0: the compiler's choice)
#endif
#ifndef ORB_PR_UNROLL
#define ORB_PR_UNROLL 8  // nn_orbit_pairs_kernel: 16-byte load pairs in flight per lane
#endif
#ifndef ORB_DU
#define ORB_DU 4
#endif
#ifndef ORB_RS_DPP
#define ORB_RS_DPP 1  // rescore / pair pass reductions: DPP lane moves inside each row of 16, one ds_bpermute across rows
#endif
#ifndef ORB_SPLIT_TAILS
// 1: the shortlist in two query halves, the first half's rescore + pair pass on a second stream beside the second
// launch.  Measured (r06z, profiles/r06/z_split_tails_ab.txt, same box, same digest): C3 step 14.75 -> 14.61 ms, but the
// second launch absorbs the overlapped tails (shortlist 13.07 -> 13.40 ms, roofline.frac 0.458 -> 0.44) and the
// tails' own event times stop meaning their cost; a 1 % step gain does not pay for measurements that no longer
// isolate the kernels, so it stays off (an A/B switch)
#define ORB_SPLIT_TAILS 0
#endif
#ifndef ORB_PR_QUAD
#define ORB_PR_QUAD 1  // nn_orbit_pairs_kernel: the query row loaded once per quad of slot lanes, broadcast by DPP (r06o: 0.50 -> 0.42 ms)
#endif

// device copy of the transform: output coordinate o (block x = o / 48) = coef[o] * sum_t w[o][t] * v[src[o][t]]
struct OrbitMap {
    int16_t src[OD][4];
    float w[OD][4];      // +-1, 0 beyond cnt
    float cs[OD], qs[OD]; // dataset / query coefficient (cs * qs = 1 / orbit size)
    int16_t msrc[3][OD];  // mirror m = 1, 2, 3 (H, V, HV): (S_m v)[i] = msgn[m-1][i] * v[msrc[m-1][i]]
    float msgn[3][OD];
};

struct OrbitDsStat {
    unsigned long long max_n2, max_p2, max_h2, max_e2;  // double bits (non-negative)
    unsigned int bad, pad;
};

// ------------------------------------------------------------------------------------------
// host: the signed permutations of the Haar layout and the isotypic basis
// ------------------------------------------------------------------------------------------
// structure replica of WaveletGS (main.pas:2805-2840) on one 8x8 component, dx = dy = 8, depth 2
static void haar_host(const double *in, double *out) {
    double cur[64];
    memcpy(cur, in, sizeof(cur));
    const double f = 1.0 / sqrt(2.0);
    for (int dx = 8; dx >= 2; dx >>= 1) {
        double tx[64], ty[64];
        memcpy(tx, cur, sizeof(tx));
        memcpy(ty, cur, sizeof(ty));
        for (int y = 0; y < dx; y++)
            for (int x = 0; x < dx / 2; x++) {
                tx[y * 8 + x] = (cur[y * 8 + 2 * x] + cur[y * 8 + 2 * x + 1]) * f;
                tx[y * 8 + x + dx / 2] = (cur[y * 8 + 2 * x] - cur[y * 8 + 2 * x + 1]) * f;
            }
        for (int x = 0; x < dx; x++)
            for (int y = 0; y < dx / 2; y++) {
                ty[y * 8 + x] = (tx[2 * y * 8 + x] + tx[(2 * y + 1) * 8 + x]) * f;
                ty[(y + dx / 2) * 8 + x] = (tx[2 * y * 8 + x] - tx[(2 * y + 1) * 8 + x]) * f;
            }
        for (int y = 0; y < dx; y++)
            for (int x = 0; x < dx; x++) cur[y * 8 + x] = ty[y * 8 + x];
    }
    memcpy(out, cur, sizeof(cur));
}

struct SPerm {
    int src[OD];
    int sgn[OD];
};

// S = T M T^T for the pixel mirror M (T = the orthonormal 3-level Haar), rounded to a signed permutation
static bool mirror_sperm(int hm, int vm, SPerm &p) {
    static double T[64][64];  // T[i][pix]
    for (int pix = 0; pix < 64; pix++) {
        double e[64] = {0}, o[64];
        e[pix] = 1.0;
        haar_host(e, o);
        for (int i = 0; i < 64; i++) T[i][pix] = o[i];
    }
    for (int i = 0; i < 64; i++) {
        int found = -1, sg = 0;
        for (int j = 0; j < 64; j++) {
            double s = 0;
            for (int pix = 0; pix < 64; pix++) {
                const int y = pix >> 3, x = pix & 7;
                const int mp = (vm ? 7 - y : y) * 8 + (hm ? 7 - x : x);
                s += T[i][pix] * T[j][mp];
            }
            if (fabs(s) > 1e-9) {
                if (found >= 0 || fabs(fabs(s) - 1.0) > 1e-9) return false;
                found = j;
                sg = s > 0 ? 1 : -1;
            }
        }
        if (found < 0) return false;
        for (int c = 0; c < 3; c++) {
            p.src[c * 64 + i] = c * 64 + found;
            p.sgn[c * 64 + i] = sg;
        }
    }
    return true;
}

static bool build_map(OrbitMap &m) {
    SPerm g[4];
    for (int i = 0; i < OD; i++) {
        g[0].src[i] = i;
        g[0].sgn[i] = 1;
    }
    if (!mirror_sperm(1, 0, g[1]) || !mirror_sperm(0, 1, g[2])) return false;
    for (int i = 0; i < OD; i++) {  // HV = H o V: (S_H (S_V v))[i] = sH[i] sV[srcH[i]] v[srcV[srcH[i]]]
        g[3].src[i] = g[2].src[g[1].src[i]];
        g[3].sgn[i] = g[1].sgn[i] * g[2].sgn[g[1].src[i]];
    }
    memset(&m, 0, sizeof(m));
    for (int mm = 1; mm < 4; mm++)
        for (int i = 0; i < OD; i++) {
            m.msrc[mm - 1][i] = (int16_t)g[mm].src[i];
            m.msgn[mm - 1][i] = (float)g[mm].sgn[i];
        }
    int fill[4] = {0, 0, 0, 0};
    bool seen[OD] = {false};
    std::vector<int> out_src[4][48], out_w[4][48];
    int out_size[4][48];
    for (int i0 = 0; i0 < OD; i0++) {
        if (seen[i0]) continue;
        int orb[4], no = 0;
        for (int gi = 0; gi < 4; gi++) {
            const int j = g[gi].src[i0];
            bool dup = false;
            for (int t = 0; t < no; t++) dup |= orb[t] == j;
            if (!dup) orb[no++] = j;
        }
        for (int t = 0; t < no; t++) seen[orb[t]] = true;
        for (int x = 0; x < 4; x++) {
            int w[4] = {0, 0, 0, 0};
            for (int gi = 0; gi < 4; gi++) {
                const int chi = (__builtin_popcount(x & gi) & 1) ? -1 : 1;
                for (int t = 0; t < no; t++)
                    if (orb[t] == g[gi].src[i0]) w[t] += chi * g[gi].sgn[i0];
            }
            bool nz = false;
            for (int t = 0; t < no; t++) nz |= w[t] != 0;
            if (!nz) continue;
            if (fill[x] >= 48) return false;
            const int o = fill[x]++;
            out_size[x][o] = no;
            for (int t = 0; t < no; t++) {
                if (w[t] == 0) return false;
                out_src[x][o].push_back(orb[t]);
                out_w[x][o].push_back(w[t] > 0 ? 1 : -1);
            }
        }
    }
    for (int x = 0; x < 4; x++)
        if (fill[x] != 48) return false;
    // the fused query kernel reads the compile-time copy (tools/gen_orbit_map.py): it must be this map exactly
    for (int x = 0; x < 4; x++)
        for (int o = 0; o < 48; o++) {
            const int oo = x * 48 + o, no = out_size[x][o];
            if (orbitgen::CNT[oo] != no) return false;
            for (int t = 0; t < no; t++)
                if (orbitgen::SRC[oo][t] != out_src[x][o][t] || orbitgen::W[oo][t] != out_w[x][o][t]) return false;
        }
    for (int x = 0; x < 4; x++)
        for (int o = 0; o < 48; o++) {
            const int oo = x * 48 + o, no = out_size[x][o];
            for (int t = 0; t < 4; t++) {
                m.src[oo][t] = (int16_t)(t < no ? out_src[x][o][t] : 0);
                m.w[oo][t] = t < no ? (float)out_w[x][o][t] : 0.0f;
            }
            m.cs[oo] = no == 4 ? 0.5f : 1.0f;
            m.qs[oo] = no == 1 ? 1.0f : 0.5f;
            // orbit_prep_kernel stages one colour component at a time: output o of block x must read only
            // component (o % 48) / 16, i.e. k-step 3x + c holds component c
            for (int t = 0; t < no; t++)
                if (out_src[x][o][t] / 64 != o / 16) return false;
        }
    return true;
}

// ------------------------------------------------------------------------------------------
// device: orbit detection
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void orbit_eq_kernel(const float *__restrict__ rows, long n,
                                                       const OrbitMap *__restrict__ mp, uint16_t *bits) {
    const int lane = threadIdx.x & 63;
    for (long j = (long)blockIdx.x * 4 + (threadIdx.x >> 6); j < n; j += (long)gridDim.x * 4) {
        unsigned b = 0;
        for (int t = 1; t <= 3; t++) {
            if (j + t >= n) break;
            for (int m = 0; m < 3; m++) {
                bool ok = true;
                for (int i = lane; i < OD; i += 64) {  // a mismatch in any 64-dimension piece settles it
                    ok = rows[(j + t) * OD + i] == mp->msgn[m][i] * rows[j * OD + mp->msrc[m][i]];
                    if (!__all(ok)) break;
                }
                if (__all(ok)) b |= 1u << ((t - 1) * 3 + m);
            }
        }
        if (lane == 0) bits[j] = (uint16_t)b;
    }
}

// Members of a group whose rows are identical (a symmetric tile: S_m c == c) have identical exact distances to
// any query; the rescore keeps only the lowest candidate index of each identical set (the tie rule picks it
// anyway).  Bit x of dup[g] marks slot x as such a duplicate.  One wave per group.
// rep[g] holds, in 2 bits per slot, the slot of the lowest-index member with the same row (the slot itself if
// none): under ANN's tie order (kdorder_dev.hpp) the rescore picks the first-found member of each such set.
__global__ __launch_bounds__(256) void orbit_dup_kernel(const float *__restrict__ rows, const int *__restrict__ member,
                                                        long G, uint8_t *__restrict__ dup, uint8_t *__restrict__ rep) {
    const int lane = threadIdx.x & 63;
    for (long g = (long)blockIdx.x * 4 + (threadIdx.x >> 6); g < G; g += (long)gridDim.x * 4) {
        int mem[4];
#pragma unroll
        for (int x = 0; x < 4; x++) mem[x] = member[g * 4 + x];
        unsigned bits = 0, reps = 0;
#pragma unroll
        for (int x = 0; x < 4; x++) {
            int r = x;
#pragma unroll
            for (int y = 0; y < 4; y++) {
                if (y == x || mem[x] < 0 || mem[y] < 0 || mem[y] > mem[x]) continue;
                bool eq = true;
                for (int i = lane; i < OD; i += 64) eq &= rows[(long)mem[x] * OD + i] == rows[(long)mem[y] * OD + i];
                if (__all(eq)) {
                    bits |= 1u << x;
                    if (mem[y] < mem[r]) r = y;
                }
            }
            reps |= (unsigned)r << (2 * x);
        }
        if (lane == 0) {
            dup[g] = (uint8_t)bits;
            rep[g] = (uint8_t)reps;
        }
    }
}

// Bit x of mask[g]: isotypic block x of group g's fp16 c' has a nonzero value.  A mirror-symmetric tile (S_m c == c)
// has exactly-zero blocks (those odd under m), whose MFMA contributions are +-0 for every query.  One wave per group.
__global__ __launch_bounds__(256) void orbit_zmask_kernel(const _Float16 *__restrict__ rowh, long G, uint8_t *mask) {
    const int lane = threadIdx.x & 63;
    for (long g = (long)blockIdx.x * 4 + (threadIdx.x >> 6); g < G; g += (long)gridDim.x * 4) {
        unsigned m = 0;
#pragma unroll
        for (int x = 0; x < 4; x++) {
            const bool nz = lane < 48 && (float)rowh[g * OD + x * 48 + lane] != 0.0f;
            if (__any(nz)) m |= 1u << x;
        }
        if (lane == 0) mask[g] = (uint8_t)m;
    }
}

// One thread per group: the kd-tree nodes separating the group's members (ANN's visit order among them,
// kdorder_dev.hpp), i.e. the lowest common node of every present slot pair, walked from the root on positions.
__global__ __launch_bounds__(256) void orbit_gorder_kernel(KdOrder o, const int *__restrict__ member, long G,
                                                           GroupOrder *__restrict__ out, int *__restrict__ grp_of) {
    const long g = (long)blockIdx.x * 256 + threadIdx.x;
    if (g >= G) return;
    int pos[4], mem[4];
#pragma unroll
    for (int x = 0; x < 4; x++) {
        mem[x] = member[g * 4 + x];
        pos[x] = mem[x] >= 0 ? o.pos[mem[x]] : -1;
        if (mem[x] >= 0) grp_of[mem[x]] = (int)(g * 4 + x);
    }
    GroupOrder r;
    r.pad = 0;
    int nodes[3] = {-1, -1, -1}, nn = 0;
    unsigned pairs = 0;
    int pi = 0;
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = x + 1; y < 4; y++, pi++) {
            if (pos[x] < 0 || pos[y] < 0) continue;
            const int pa = min(pos[x], pos[y]), pb = max(pos[x], pos[y]);
            int s0 = 0, e0 = o.n, m = -1;
            while (e0 - s0 > o.bs) {
                const int mm = s0 + ((e0 - s0) >> 1);
                if (pb < mm) {
                    e0 = mm;
                } else if (pa >= mm) {
                    s0 = mm;
                } else {
                    m = mm;
                    break;
                }
            }
            if (m < 0) continue;  // one bucket: position order (not reached with bs = 1)
            int ni = -1;
            for (int i = 0; i < nn; i++)
                if (nodes[i] == m) ni = i;
            if (ni < 0 && nn < 3) {
                ni = nn;
                nodes[nn++] = m;
            }
            pairs |= (unsigned)(ni | ((pos[x] < m) ? 4 : 0)) << (3 * pi);
        }
    for (int i = 0; i < 3; i++) {
        r.cd[i] = (uint16_t)(nodes[i] >= 0 ? o.cd[nodes[i]] : 0);
        r.cv[i] = nodes[i] >= 0 ? o.cv[nodes[i]] : 0.0f;
    }
    r.pairs = pairs;
    out[g] = r;
}

// ANN's order of two different slots of one group (both present) for query q
// (go points into HBM: indexing the node there is a plain load, a runtime index into a register copy would
// put the struct in scratch)
__device__ __forceinline__ bool group_before(const GroupOrder *__restrict__ go, const float *__restrict__ q, int x,
                                             int y) {
    const int lo = min(x, y), hi = max(x, y);
    const int pi = lo == 0 ? hi - 1 : lo == 1 ? hi + 1 : 5;  // (0,1)(0,2)(0,3)(1,2)(1,3)(2,3)
    const unsigned code = (go->pairs >> (3 * pi)) & 7u;
    const int node = code & 3;
    const bool lo_first = (q[go->cd[node]] - go->cv[node]) < 0.0f;
    const bool low_slot_first = ((code >> 2) & 1) == (unsigned)lo_first;
    return (x == lo) == low_slot_first;
}

// ------------------------------------------------------------------------------------------
// device: transform + fp16 split (dataset rows: member != null, coefficient cs; queries: qs)
//   lane l of block b holds row b*32 + (l & 31), k = s*16 + 8*(l >> 5) + j  (A and B maps coincide)
// ------------------------------------------------------------------------------------------
struct OrbitPrepArgs {
    const float *rows;     // dataset: candidate rows [n][192]; queries: [nq][192]
    const int *member;     // dataset: [G][4] (slot 0 = base row); queries: null
    long count;            // G or nq
    const OrbitMap *mp;
    float scale;
    half8 *frag;           // [ceil(count/32)][12][64]
    _Float16 *rowh;        // [count][192] (dataset only: the query path keeps q' in the fragments; null)
    float *seed, *nc;      // dataset only
    OrbitDsStat *ds;       // dataset only
    OrbitStat *qstat;      // queries only
};

// Four waves per workgroup, one 32-row block per wave, one colour component at a time: the transform
// never mixes components (S_m permutes within each 64-value component, build_map checks it), and
// output k-step s = 3x + c holds component c's 16 outputs of isotypic block x.  So a wave stages only
// its rows' 64 values of component c in LDS (stride 65 floats: the 32 lanes of a half-wave read 32
// rows conflict-free), 8.3 KB per wave, and the 4 waves share the transform table: 16 waves per CU.
static constexpr int ORB_CS = 65;
static constexpr int ORB_PW = 4;  // waves (32-row blocks) per workgroup

__global__ __launch_bounds__(64 * ORB_PW) void orbit_prep_kernel(OrbitPrepArgs a) {
    __shared__ float srow[ORB_PW][32 * ORB_CS];
    __shared__ int16_t msrc[OD * 4];
    __shared__ float mw[OD * 4], mc[OD];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const long nblk = (a.count + 31) / 32;
    const bool dataset = a.member != nullptr;
    for (int i = tid; i < OD * 4; i += 64 * ORB_PW) {
        msrc[i] = a.mp->src[i >> 2][i & 3];
        mw[i] = a.mp->w[i >> 2][i & 3];
    }
    for (int i = tid; i < OD; i += 64 * ORB_PW) mc[i] = dataset ? a.mp->cs[i] : a.mp->qs[i];
    float *sw = srow[w];
    double t_n2 = 0.0, t_p2 = 0.0, t_h2 = 0.0, t_e2 = 0.0;  // dataset statistics over this thread's valid rows
    int t_bd = 0;
    for (long wb = blockIdx.x; wb * ORB_PW < nblk; wb += gridDim.x) {  // uniform trip count per workgroup
        const long blk = wb * ORB_PW + w;
        const long r = blk * 32 + (lane & 31);
        const bool valid = blk < nblk && r < a.count;
        // this lane's staging rows (8 float4 pieces: row rr = i / 16, piece i % 16 of the component)
        long src_row[8];
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const int rr = (lane + 64 * t) >> 4;
            const long rg = blk * 32 + rr;
            src_row[t] = (blk < nblk && rg < a.count) ? (dataset ? (long)a.member[rg * 4] : rg) : -1;
        }
        const float *row = sw + (lane & 31) * ORB_CS;
        double n2 = 0, p2 = 0, h2 = 0, e2 = 0;
        int bad = 0;
#pragma unroll 1
        for (int c = 0; c < 3; c++) {
            __syncthreads();
#pragma unroll
            for (int t = 0; t < 8; t++) {
                const int i = lane + 64 * t, rr = i >> 4, c4 = i & 15;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (src_row[t] >= 0) v = reinterpret_cast<const float4 *>(a.rows + src_row[t] * OD + c * 64)[c4];
                float *d = sw + rr * ORB_CS + c4 * 4;
                d[0] = v.x;
                d[1] = v.y;
                d[2] = v.z;
                d[3] = v.w;
            }
            __syncthreads();
            if (valid) {  // |row|^2: this half-wave lane's 32 values of the component
#pragma unroll 8
                for (int i = 0; i < 32; i++) {
                    const double orig = (double)row[32 * h + i] * (double)a.scale;
                    n2 += orig * orig;
                }
            }
#pragma unroll
            for (int x = 0; x < 4; x++) {
                const int s = 3 * x + c;
                half8 hv;
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int k = s * 16 + 8 * h + j;
                    double v = 0.0;
                    if (valid) {
#pragma unroll
                        for (int t = 0; t < 4; t++) v += (double)mw[k * 4 + t] * (double)row[(msrc[k * 4 + t] - 64 * c) & 63];  // unused terms: w = 0
                        v *= (double)mc[k] * (double)a.scale;
                    }
                    _Float16 vh = (_Float16)(float)v;
                    if (fabs((double)(float)vh) < 6.103515625e-05) vh = (_Float16)0.0f;  // no fp16 subnormal operands
                    hv[j] = vh;
                    const double dh = (double)(float)vh;
                    p2 += v * v;
                    h2 += dh * dh;
                    e2 += (v - dh) * (v - dh);
                    if (!isfinite(v) || fabs(v) > 65000.0) bad = 1;
                }
                if (blk < nblk) a.frag[(blk * OS + s) * 64 + lane] = hv;
                if (valid && a.rowh) *reinterpret_cast<half8 *>(a.rowh + r * OD + s * 16 + 8 * h) = hv;
            }
        }
        if (blk >= nblk) continue;
        n2 += __shfl_xor(n2, 32, 64);
        p2 += __shfl_xor(p2, 32, 64);
        h2 += __shfl_xor(h2, 32, 64);
        e2 += __shfl_xor(e2, 32, 64);
        bad |= __shfl_xor(bad, 32, 64);
        if (!dataset) {
            if (valid && h == 0) {
                OrbitStat q;
                q.n2 = n2;
                q.hn = sqrt(h2);
                q.en = sqrt(e2);
                q.flags = (bad || !isfinite(n2)) ? 2 : 0;
                q.pad = 0;
                a.qstat[r] = q;
            }
            continue;
        }
        if (h == 0) {
            const int rr = lane & 31;
            const int pos = ((rr >> 2) & 1) * 16 + ((rr & 3) | ((rr >> 3) << 2));
            a.seed[blk * 32 + pos] = valid ? -0.5f * (float)n2 : -INFINITY;
            if (valid) a.nc[r] = (float)n2;
        }
        if (valid) {  // this thread's running maxima (all >= 0: bit patterns order like the values)
            t_n2 = fmax(t_n2, n2);
            t_p2 = fmax(t_p2, p2);
            t_h2 = fmax(t_h2, h2);
            t_e2 = fmax(t_e2, e2);
            t_bd |= bad;
        }
    }
    if (dataset) {  // one set of atomics per workgroup (per wave and block they serialised on five words)
        __shared__ double r_d[ORB_PW][4];
        __shared__ int r_b[ORB_PW];
        const double mn = wave_max_d(t_n2), mp2 = wave_max_d(t_p2), mh = wave_max_d(t_h2), me = wave_max_d(t_e2);
        const int bd = __any(t_bd);
        if (lane == 0) {
            r_d[w][0] = mn;
            r_d[w][1] = mp2;
            r_d[w][2] = mh;
            r_d[w][3] = me;
            r_b[w] = bd;
        }
        __syncthreads();
        if (tid == 0) {
            double v[4] = {0.0, 0.0, 0.0, 0.0};
            int b = 0;
            for (int x = 0; x < ORB_PW; x++) {
                for (int y = 0; y < 4; y++) v[y] = fmax(v[y], r_d[x][y]);
                b |= r_b[x];
            }
            atomicMax(&a.ds->max_n2, (unsigned long long)__double_as_longlong(v[0]));
            atomicMax(&a.ds->max_p2, (unsigned long long)__double_as_longlong(v[1]));
            atomicMax(&a.ds->max_h2, (unsigned long long)__double_as_longlong(v[2]));
            atomicMax(&a.ds->max_e2, (unsigned long long)__double_as_longlong(v[3]));
            if (b) atomicOr(&a.ds->bad, 1u);
        }
    }
}

// ------------------------------------------------------------------------------------------
// device: the orbit shortlist.  Workgroup = NW waves x one 32-query block; the 32-tile blocks of this
// split stream through a double-buffered LDS ring (CB blocks per stage, LDS-DMA).  Accumulator element
// r of lane l holds tile row (r & 3) + 8 (r >> 2) + 4 h (h = l >> 5) of query column l & 31; sub-block
// s = r >> 2 = the 4 consecutive tiles 8 s + 4 h + 0..3.  List entry id = blk * 4 + s.
// ------------------------------------------------------------------------------------------
template <int L, int CB, int NW, int QB, int MODE>
__global__ __launch_bounds__(NW * 64, 1) void nn_orbit_shortlist_kernel(const half8 *__restrict__ cfrag,
                                                                    const float *__restrict__ cseed, int nblk,
                                                                    const half8 *__restrict__ qfrag, int nq,
                                                                    int blk_per_split, int nsplit,
                                                                    float *__restrict__ out_key,
                                                                    int *__restrict__ out_id) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int FRAG_BYTES = CB * OS * 1024;
    constexpr int BUF_BYTES = FRAG_BYTES + CB * 128;
    constexpr int NT = NW * 64;
    constexpr int PER_T = CB * OS * 64 / NT;
    static_assert((CB * OS * 64) % NT == 0, "stage must split evenly over the workgroup");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const int nqblk = (nq + 31) / 32;
    const int qb0 = (blockIdx.x * NW + w) * QB;
    const int split = blockIdx.y;
    const int b_begin = split * blk_per_split;
    const int b_end = min(nblk, b_begin + blk_per_split);

    // the wave's QB query blocks stay in registers as B fragments; each A fragment read from LDS feeds QB MFMAs
    half8 bq[QB][OS];
#pragma unroll
    for (int q = 0; q < QB; q++) {
        const long qa = min(qb0 + q, nqblk - 1);  // past the end: clamped duplicate, never written
#pragma unroll
        for (int s = 0; s < OS; s++) bq[q][s] = qfrag[(qa * OS + s) * 64 + lane];
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) before the hidden DMA starts counting
    float lk[QB][L];
    int li[QB][L];
#pragma unroll
    for (int q = 0; q < QB; q++)
#pragma unroll
        for (int i = 0; i < L; i++) {
            lk[q][i] = INFINITY;
            li[q][i] = -1;
        }

    const int nstage = (b_end > b_begin) ? (b_end - b_begin + CB - 1) / CB : 0;
    auto issue = [&](int st, int buf) {
        const int blk0 = b_begin + st * CB;
        const int nb = min(CB, b_end - blk0);
        const uint4 *src = reinterpret_cast<const uint4 *>(cfrag) + (long)blk0 * OS * 64 + w * 64 + lane;
        char *dst = smem + buf * BUF_BYTES + w * 1024;
        if (nb == CB) {
#pragma unroll
            for (int j = 0; j < PER_T; j++) glds16_asm(src + j * NT, dst + j * NT * 16);
        } else {
            const int last = nb * OS * 64 - 1 - (w * 64 + lane);
#pragma unroll
            for (int j = 0; j < PER_T; j++) glds16_asm(src + min(j * NT, last), dst + j * NT * 16);
        }
        if (w == 0 && lane < CB * 8)
            glds16_asm(reinterpret_cast<const uint4 *>(cseed) + (long)blk0 * 8 + min(lane, nb * 8 - 1),
                       smem + buf * BUF_BYTES + FRAG_BYTES);
    };

    if (nstage > 0) issue(0, 0);
    dma_drain();
    __syncthreads();
    const floatx16 zero = {0};
    for (int st = 0; st < nstage; st++) {
        const char *B = smem + (st & 1) * BUF_BYTES;
        const half8 *A = reinterpret_cast<const half8 *>(B) + lane;
        const float4 *SD = reinterpret_cast<const float4 *>(B + FRAG_BYTES) + h * 4;
        half8 a0 = A[0], a1 = A[64];
        float4 sd0 = SD[0], sd1 = SD[1], sd2 = SD[2], sd3 = SD[3];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (st + 1 < nstage) issue(st + 1, (st + 1) & 1);
#pragma unroll
        for (int cb = 0; cb < CB; cb++) {
            const int blk = b_begin + st * CB + cb;
            if (blk < b_end) {
                const floatx16 seed = {sd0.x, sd0.y, sd0.z, sd0.w, sd1.x, sd1.y, sd1.z, sd1.w,
                                       sd2.x, sd2.y, sd2.z, sd2.w, sd3.x, sd3.y, sd3.z, sd3.w};
                // p = d0 (seeded with -||c||^2/2), then p += |d_x| as each isotypic block x = 1..3 completes;
                // blocks 1 and 3 accumulate in ta, block 2 in tb (the next block's MFMAs run while p reads the last)
                floatx16 p[QB], ta[QB], tb[QB];
#pragma unroll
                for (int s = 0; s < OS; s += 2) {
                    half8 n0, n1;
                    const bool more = s + 2 < OS || cb + 1 < CB;
                    if (s + 2 < OS) {
                        n0 = A[(cb * OS + s + 2) * 64];
                        n1 = A[(cb * OS + s + 3) * 64];
                    } else if (cb + 1 < CB) {  // next block of this stage: first pair and seeds
                        n0 = A[((cb + 1) * OS) * 64];
                        n1 = A[((cb + 1) * OS + 1) * 64];
                        sd0 = SD[(cb + 1) * 8 + 0];
                        sd1 = SD[(cb + 1) * 8 + 1];
                        sd2 = SD[(cb + 1) * 8 + 2];
                        sd3 = SD[(cb + 1) * 8 + 3];
                    }
#pragma unroll
                    for (int hh = 0; hh < 2; hh++) {
                        const int ss = s + hh, x = ss / 3;
                        const half8 av = hh ? a1 : a0;
#pragma unroll
                        for (int q = 0; q < QB; q++) {
                            if (x == 0)
                                p[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bq[q][ss], ss == 0 ? seed : p[q], 0, 0, 0);
                            else if (x == 2)
                                tb[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bq[q][ss], ss % 3 == 0 ? zero : tb[q], 0, 0, 0);
                            else
                                ta[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bq[q][ss], ss % 3 == 0 ? zero : ta[q], 0, 0, 0);
                        }
                        if (MODE != 3 && x > 0 && ss % 3 == 2) {
#pragma unroll
                            for (int q = 0; q < QB; q++)
#pragma unroll
                                for (int r = 0; r < 16; r++) p[q][r] = p[q][r] + fabsf(x == 2 ? tb[q][r] : ta[q][r]);
                        }
                    }
                    if (more) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 2 * QB, 0);
                    if (more) {
                        a0 = n0;
                        a1 = n1;
                    }
                }
#pragma unroll
                for (int q = 0; q < QB; q++) {
                    if (MODE == 3) {  // timing experiment: MFMA only
                        lk[q][0] = fmaxf(lk[q][0], p[q][0] + ta[q][1] + tb[q][2]);
                        continue;
                    }
                    // p = u = d0 + |d1| + |d2| + |d3| >= every mirror value q.(S_m c) - ||c||^2/2 (key = -2u)
                    float m4[4];
#pragma unroll
                    for (int sb = 0; sb < 4; sb++)
                        m4[sb] = fmaxf(fmaxf(p[q][4 * sb], p[q][4 * sb + 1]), fmaxf(p[q][4 * sb + 2], p[q][4 * sb + 3]));
                    const float mx = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
                    if (MODE == 2) {  // timing experiment: MFMA + bound only
                        lk[q][0] = fmaxf(lk[q][0], mx);
                        continue;
                    }
                    if (__builtin_expect(__any(mx > -0.5f * lk[q][L - 1]), 0)) {
                        // insert every sub-block above the lane's current L-th entry, best first
#pragma unroll
                        for (int it = 0; it < 4; it++) {
                            float best = m4[0];
                            int bs = 0;
#pragma unroll
                            for (int sb = 1; sb < 4; sb++)
                                if (m4[sb] > best) {
                                    best = m4[sb];
                                    bs = sb;
                                }
                            const bool ins = best > -0.5f * lk[q][L - 1];
                            if (!__any(ins)) break;
                            if (ins) {
                                list_insert<L>(lk[q], li[q], -2.0f * best, blk * 4 + bs);
#pragma unroll
                                for (int sb = 0; sb < 4; sb++)
                                    if (sb == bs) m4[sb] = -INFINITY;
                            }
                        }
                    }
                }
            }
        }
        dma_drain();
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < QB; q++) {
        const int qq = (qb0 + q) * 32 + (lane & 31);
        if (qb0 + q < nqblk && qq < nq) {
            const long o = (((long)qq * nsplit + split) * 2 + h) * L;
#pragma unroll
            for (int i = 0; i < L; i++) {
                out_key[o + i] = lk[q][i];
                out_id[o + i] = li[q][i];
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// device: the orbit shortlist, software-pipelined (default).  Same contraction, bound and lists as
// nn_orbit_shortlist_kernel, but no block ends in a VALU-only tail: the bound adds of block b run beside
// its own x2/x3 MFMAs, and its last |d_3| adds, sub-block maxima and list test run beside block b+1's
// x0/x1 MFMAs.  Accumulator roles alternate between even and odd blocks so that nothing extra is live:
//     x0 -> P (seeded), x1 -> RB, x2 -> T2, x3 -> RB,   P = RA, T2 = RC on even blocks, swapped on odd,
// i.e. the previous block's P is this block's T2 (written only after the previous tail has read it).
// A list insertion for block b happens right after block b+1's front half (the branch is wave-uniform).
// ------------------------------------------------------------------------------------------
template <int L, int CB, int NW, int QB, int MODE>
__global__ __launch_bounds__(NW * 64, 1) void nn_orbit_shortlist_pipe_kernel(const half8 *__restrict__ cfrag,
                                                                         const float *__restrict__ cseed, int nblk,
                                                                         const half8 *__restrict__ qfrag, int nq,
                                                                         int blk_per_split, int nsplit,
                                                                         float *__restrict__ out_key,
                                                                         int *__restrict__ out_id, int red_end,
                                                                         const uint8_t *__restrict__ bmask,
                                                                         int flat_wg0, const uint8_t *__restrict__ bmask0,
                                                                         const int *__restrict__ flat_cnt,
                                                                         int flat_base) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int FRAG_BYTES = CB * OS * 1024;
    constexpr int BUF_BYTES = FRAG_BYTES + CB * 128;
    constexpr int NT = NW * 64;
    constexpr int PER_T = CB * OS * 64 / NT;
    static_assert((CB * OS * 64) % NT == 0, "stage must split evenly over the workgroup");
    static_assert(CB % 2 == 0, "accumulator roles alternate over pairs of blocks");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const int nqblk = (nq + 31) / 32;
    const int qb0 = (blockIdx.x * NW + w) * QB;
    const int split = blockIdx.y;
    const int b_begin = split * blk_per_split;
    const int b_end = min(nblk, b_begin + blk_per_split);

    half8 bq[QB][OS];
#pragma unroll
    for (int q = 0; q < QB; q++) {
        const long qa = min(qb0 + q, nqblk - 1);  // past the end: clamped duplicate, never written
#pragma unroll
        for (int s = 0; s < OS; s++) bq[q][s] = qfrag[(qa * OS + s) * 64 + lane];
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) before the hidden DMA starts counting
    if (NW * QB > 8 * 2 / 2 && NW == 4) {  // experiment (one wave per SIMD): the B fragments live in the AGPR file
#pragma unroll
        for (int q = 0; q < QB; q++)
#pragma unroll
            for (int s = 0; s < OS; s++) asm volatile("" : "+a"(bq[q][s]));
    }
    float lk[QB][L], th[QB];
    int li[QB][L];
#pragma unroll
    for (int q = 0; q < QB; q++) {
        th[q] = -INFINITY;  // = -lk[L-1] / 2: a sub-block enters the lane list when its bound exceeds th
#pragma unroll
        for (int i = 0; i < L; i++) {
            lk[q][i] = INFINITY;
            li[q][i] = -1;
        }
    }

    // blocks [b_begin, r_end): groups with zero isotypic blocks (orbit_build orders them first), block-serial with
    // only the nonzero k-steps; [p_begin, b_end): the pipelined full contraction
    // workgroups from flat_wg0 on hold flat query tiles only (q' block 0): every candidate block block-serially with
    // k-steps 0..2, only those streamed
    // (flat_cnt: the device count of non-flat queries -> first all-flat workgroup; flat_wg0 bounds it)
    // (flat_base: the launch's first query, when it covers a later part of the batch)
    if (flat_cnt) flat_wg0 = min(flat_wg0, (max(0, *flat_cnt - flat_base) + NW * QB * 32 - 1) / (NW * QB * 32));
    const bool flat = (int)blockIdx.x >= flat_wg0;
    const int nks = flat ? 3 : OS;
    if (flat) {
        red_end = nblk;
        bmask = bmask0;
    }
    const int r_end = max(b_begin, min(b_end, red_end));
    const int p_begin = r_end;
    auto issue_k3 = [&](int base, int end, int st, int buf) __attribute__((always_inline)) {
        // k-steps 0..2 of each block of the stage (3 x 64 16-byte pieces per block) to their usual LDS places
        const int blk0 = base + st * CB;
        const int nb = min(CB, end - blk0);
#pragma unroll
        for (int j = 0; j < (CB * 192 + NT - 1) / NT; j++) {
            const int e0 = j * NT + w * 64;  // the wave's first piece: 64-aligned, never straddles a block
            if (e0 < CB * 192) {
                const int cb = e0 / 192, r0 = e0 % 192;
                const int cbc = min(cb, nb - 1);  // past the end: a duplicate of the last block, never used
                glds16_asm(reinterpret_cast<const uint4 *>(cfrag) + (long)(blk0 + cbc) * OS * 64 + r0 + lane,
                           smem + buf * BUF_BYTES + (cb * OS * 64 + r0) * 16);
            }
        }
        if (w == 0 && lane < CB * 8)
            glds16_asm(reinterpret_cast<const uint4 *>(cseed) + (long)blk0 * 8 + min(lane, nb * 8 - 1),
                       smem + buf * BUF_BYTES + FRAG_BYTES);
    };
    auto issue_rng = [&](int base, int end, int st, int buf) __attribute__((always_inline)) {
        const int blk0 = base + st * CB;
        const int nb = min(CB, end - blk0);
        const uint4 *src = reinterpret_cast<const uint4 *>(cfrag) + (long)blk0 * OS * 64 + w * 64 + lane;
        char *dst = smem + buf * BUF_BYTES + w * 1024;
        if (nb == CB) {
#pragma unroll
            for (int j = 0; j < PER_T; j++) glds16_asm(src + j * NT, dst + j * NT * 16);
        } else {
            const int last = nb * OS * 64 - 1 - (w * 64 + lane);
#pragma unroll
            for (int j = 0; j < PER_T; j++) glds16_asm(src + min(j * NT, last), dst + j * NT * 16);
        }
        if (w == 0 && lane < CB * 8)
            glds16_asm(reinterpret_cast<const uint4 *>(cseed) + (long)blk0 * 8 + min(lane, nb * 8 - 1),
                       smem + buf * BUF_BYTES + FRAG_BYTES);
    };
    const int nstage = (b_end > p_begin) ? (b_end - p_begin + CB - 1) / CB : 0;
    auto issue = [&](int st, int buf) __attribute__((always_inline)) { issue_rng(p_begin, b_end, st, buf); };

    // list insertion of one finished block: every sub-block above the lane's current L-th entry, best first
    auto insert_block = [&](int q, float (&m4)[4], int blk) __attribute__((always_inline)) {
#pragma unroll
        for (int it = 0; it < 4; it++) {
            float best = m4[0];
            int bs = 0;
#pragma unroll
            for (int sb = 1; sb < 4; sb++)
                if (m4[sb] > best) {
                    best = m4[sb];
                    bs = sb;
                }
            const bool ins = best > th[q];
            if (!__any(ins)) break;
            if (ins) {
                list_insert<L>(lk[q], li[q], -2.0f * best, blk * 4 + bs);
#pragma unroll
                for (int sb = 0; sb < 4; sb++)
                    if (sb == bs) m4[sb] = -INFINITY;
            }
        }
        th[q] = -0.5f * lk[q][L - 1];
    };
    // sub-block maxima of a finished bound accumulator; returns the lane's max
    auto maxima = [&](const floatx16 &P, float (&m4)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int sb = 0; sb < 4; sb++) m4[sb] = fmaxf(fmaxf(P[4 * sb], P[4 * sb + 1]), fmaxf(P[4 * sb + 2], P[4 * sb + 3]));
        return fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
    };

    if (r_end > b_begin) {  // the symmetric groups' blocks (same bound, same order of adds, zero blocks skipped)
        const floatx16 zero4 = {0};
        const int nst_r = (r_end - b_begin + CB - 1) / CB;
        if (nks == 3)
            issue_k3(b_begin, r_end, 0, 0);
        else
            issue_rng(b_begin, r_end, 0, 0);
        dma_drain();
        __syncthreads();
        for (int st = 0; st < nst_r; st++) {
            const char *B = smem + (st & 1) * BUF_BYTES;
            if (st + 1 < nst_r) {
                if (nks == 3)
                    issue_k3(b_begin, r_end, st + 1, (st + 1) & 1);
                else
                    issue_rng(b_begin, r_end, st + 1, (st + 1) & 1);
            }
            const half8 *A = reinterpret_cast<const half8 *>(B) + lane;
            const float4 *SD = reinterpret_cast<const float4 *>(B + FRAG_BYTES) + h * 4;
            for (int cb = 0; cb < CB; cb++) {
                const int blk = b_begin + st * CB + cb;
                if (blk >= r_end) break;
                const unsigned act = bmask[blk];  // bit x: some group of the block has a nonzero block x
                const float4 s0 = SD[cb * 8 + 0], s1 = SD[cb * 8 + 1], s2 = SD[cb * 8 + 2], s3 = SD[cb * 8 + 3];
                const floatx16 seed = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w,
                                       s2.x, s2.y, s2.z, s2.w, s3.x, s3.y, s3.z, s3.w};
                floatx16 P[QB], T[QB];
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    const half8 av = A[(cb * OS + k) * 64];
#pragma unroll
                    for (int q = 0; q < QB; q++)
                        P[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bq[q][k], k == 0 ? seed : P[q], 0, 0, 0);
                }
#pragma unroll
                for (int x = 1; x < 4; x++) {
                    if (!((act >> x) & 1)) continue;  // uniform
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        const half8 av = A[(cb * OS + 3 * x + k) * 64];
#pragma unroll
                        for (int q = 0; q < QB; q++)
                            T[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bq[q][3 * x + k], k == 0 ? zero4 : T[q], 0, 0, 0);
                    }
#pragma unroll
                    for (int q = 0; q < QB; q++)
#pragma unroll
                        for (int r = 0; r < 16; r++) P[q][r] = P[q][r] + fabsf(T[q][r]);
                }
#pragma unroll
                for (int q = 0; q < QB; q++) {
                    float m4[4];
                    const float mx = maxima(P[q], m4);
                    if (__any(mx > th[q])) insert_block(q, m4, blk);
                }
            }
            dma_drain();
            __syncthreads();
        }
    }
    if (nstage > 0) issue(0, 0);
    dma_drain();
    __syncthreads();
    if ((MODE == 3 || MODE == 5 || MODE == 7) && w >= NW / 2) __builtin_amdgcn_s_setprio(1);  // experiment: static priority, 2nd half
    // experiment LOOSE (modes 6, 7; no longer launched: its loose keys fill the lists and send queries to the slow
    // tiers, profiles/r02s_shortlist_ab.txt): a sub-block's bound is the sum of its four per-block maxima,
    // max_t d0 + max_t |d1| + max_t |d2| + max_t |d3| >= max_t u_t (still rigorous, looser), kept in SA / SC
    constexpr bool LOOSE = MODE == 6 || MODE == 7;
    const floatx16 zero = {0};
    floatx16 RA[QB], RB[QB], RC[QB];
    float SA[QB][4], SC[QB][4];
    float dm[16];  // MODE 11 only
#pragma unroll
    for (int i = 0; i < 16; i++) dm[i] = (float)(lane + i);
#pragma unroll
    for (int q = 0; q < QB; q++) {
        RA[q] = RB[q] = RC[q] = zero;
#pragma unroll
        for (int sb = 0; sb < 4; sb++) SA[q][sb] = SC[q][sb] = -INFINITY;
    }
    int pend = -1;          // the block whose tail is pending (-1: none / not a real block)
    half8 a0, a1;           // A fragments of the next k-step pair
    float4 sd0, sd1, sd2, sd3;  // seeds of the next block

    // one block: roles P (x0, seeded), T2 (x2); RB takes x1 and x3.  On entry T2 holds the previous
    // block's bound (minus its |d_3|, which is in RB).
    auto body = [&](const half8 *A, const float4 *SD, int cb, int blk, floatx16 (&P)[QB], floatx16 (&T2)[QB],
                    float (&Sc)[QB][4], float (&Sp)[QB][4]) __attribute__((always_inline)) {
        const floatx16 seed = {sd0.x, sd0.y, sd0.z, sd0.w, sd1.x, sd1.y, sd1.z, sd1.w,
                               sd2.x, sd2.y, sd2.z, sd2.w, sd3.x, sd3.y, sd3.z, sd3.w};
        float pmx[QB];
#pragma unroll
        for (int s = 0; s < OS; s += 2) {
            half8 n0, n1;
            const bool more = s + 2 < OS || cb + 1 < CB;
            if (MODE == 14 || MODE == 15) {  // timing: no A-fragment LDS reads (the stage's first pair reused; invalid)
                n0 = a0;
                n1 = a1;
                if (s + 2 >= OS && cb + 1 < CB) {
                    sd0 = SD[(cb + 1) * 8 + 0];
                    sd1 = SD[(cb + 1) * 8 + 1];
                    sd2 = SD[(cb + 1) * 8 + 2];
                    sd3 = SD[(cb + 1) * 8 + 3];
                }
            } else if (s + 2 < OS) {
                n0 = A[(cb * OS + s + 2) * 64];
                n1 = A[(cb * OS + s + 3) * 64];
            } else if (cb + 1 < CB) {  // next block of this stage: first pair and seeds
                n0 = A[((cb + 1) * OS) * 64];
                n1 = A[((cb + 1) * OS + 1) * 64];
                sd0 = SD[(cb + 1) * 8 + 0];
                sd1 = SD[(cb + 1) * 8 + 1];
                sd2 = SD[(cb + 1) * 8 + 2];
                sd3 = SD[(cb + 1) * 8 + 3];
            }
#pragma unroll
            for (int hh = 0; hh < 2; hh++) {
                const int ss = s + hh;
                const half8 av = hh ? a1 : a0;
#pragma unroll
                for (int q = 0; q < QB; q++) {
                    if (ss < 3)
                        P[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bq[q][ss], ss == 0 ? seed : P[q], 0, 0, 0);
                    else if (ss < 6 || ss >= 9)
                        RB[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bq[q][ss], ss % 3 == 0 ? zero : RB[q], 0, 0, 0);
                    else
                        T2[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bq[q][ss], ss == 6 ? zero : T2[q], 0, 0, 0);
                }
                // the VALU beside these MFMAs, about 10 per step (each group is issued before the MFMA that
                // overwrites its input); element t of a group = accumulator element t % 16 of query block t / 16
                auto acc_abs = [&](floatx16 (&D)[QB], const floatx16 (&S)[QB], int lo, int hi) __attribute__((always_inline)) {
#pragma unroll
                    for (int t = 0; t < 16 * QB; t++)
                        if (t >= lo && t < hi) D[t / 16][t % 16] = D[t / 16][t % 16] + fabsf(S[t / 16][t % 16]);
                };
                constexpr int N3 = 16 * QB, C1 = (N3 + 2) / 3, C2 = (2 * N3 + 2) / 3;
                // LOOSE: sub-block maxima of one accumulator (|.| when AB), sub-blocks [lo, hi) of the QB * 4
                auto mx4 = [&](const floatx16 (&S)[QB], int t, bool ab) __attribute__((always_inline)) {
                    const int q = t / 4, sb = t % 4;
                    const float a = ab ? fabsf(S[q][4 * sb]) : S[q][4 * sb], b = ab ? fabsf(S[q][4 * sb + 1]) : S[q][4 * sb + 1];
                    const float c = ab ? fabsf(S[q][4 * sb + 2]) : S[q][4 * sb + 2], d = ab ? fabsf(S[q][4 * sb + 3]) : S[q][4 * sb + 3];
                    return fmaxf(fmaxf(a, b), fmaxf(c, d));
                };
                constexpr int M3 = 4 * QB, D1 = (M3 + 2) / 3, D2 = (2 * M3 + 2) / 3;
                if (LOOSE) {
                    if (ss <= 2) {  // previous block: + max |d_3| (RB) -- before step 3's MFMA writes RB
#pragma unroll
                        for (int t = 0; t < M3; t++)
                            if (t >= (ss == 0 ? 0 : ss == 1 ? D1 : D2) && t < (ss == 0 ? D1 : ss == 1 ? D2 : M3))
                                Sp[t / 4][t % 4] = Sp[t / 4][t % 4] + mx4(RB, t, true);
                    }
                    if (ss >= 3 && ss - 3 < QB) {
                        const int q = ss - 3;
                        pmx[q] = fmaxf(fmaxf(Sp[q][0], Sp[q][1]), fmaxf(Sp[q][2], Sp[q][3]));
                        asm volatile("" ::"v"(pmx[q]));
                    }
                    if (ss >= 6 && ss <= 8) {  // this block: max d0 (P) + max |d_1| (RB)
#pragma unroll
                        for (int t = 0; t < M3; t++)
                            if (t >= (ss == 6 ? 0 : ss == 7 ? D1 : D2) && t < (ss == 6 ? D1 : ss == 7 ? D2 : M3))
                                Sc[t / 4][t % 4] = mx4(P, t, false) + mx4(RB, t, true);
                    }
                    if (ss >= 10) {  // this block: + max |d_2| (T2)
#pragma unroll
                        for (int t = 0; t < M3; t++)
                            if (t >= (ss == 10 ? 0 : M3 / 2) && t < (ss == 10 ? M3 / 2 : M3))
                                Sc[t / 4][t % 4] = Sc[t / 4][t % 4] + mx4(T2, t, true);
                    }
                } else if (MODE == 11 || MODE == 12 || MODE == 14) {  // timing experiment: every MFMA chain live + (11) as many VALU adds on registers no MFMA touches (12: none)
                    const int nd = (MODE == 12 || MODE == 14) ? 0 : ss <= 2 ? 11 : ss <= 4 ? 10 : (ss >= 6 && ss <= 8) ? 11 : ss >= 10 ? 16 : 0;
#pragma unroll
                    for (int i = 0; i < nd; i++) asm volatile("v_add_f32 %0, %0, |%1|" : "+v"(dm[i & 15]) : "v"(dm[(i + 5) & 15]));
#pragma unroll
                    for (int q = 0; q < QB; q++) {  // keep every MFMA chain live (one use of each finished chain)
                        if (ss == 2) asm volatile("" ::"v"(P[q][0]));
                        if (ss == 5 || ss == 11) asm volatile("" ::"v"(RB[q][0]));
                        if (ss == 8) asm volatile("" ::"v"(T2[q][0]));
                    }
                } else if (MODE == 2) {  // timing experiment: MFMA + loads only (results invalid)
                } else if (ss <= 2)  // previous block: + |d_3| (RB) -- before step 3's MFMA writes RB
                    acc_abs(T2, RB, ss == 0 ? 0 : ss == 1 ? C1 : C2, ss == 0 ? C1 : ss == 1 ? C2 : N3);
                if (!LOOSE && MODE != 2 && (MODE < 11 || MODE == 13 || MODE == 15) && (ss == 3 || ss == 4)) {  // previous block: its max for the list test
#pragma unroll
                    for (int q = 0; q < QB; q++) {  // query blocks [0, (QB+1)/2) at step 3, the rest at step 4
                        if ((ss == 3) != (q < (QB + 1) / 2)) continue;
                        float m4[4];
                        pmx[q] = maxima(T2[q], m4);
                        // materialise here: otherwise the whole tail sinks into the (rare) insertion branch
                        // and the previous |d_3| (RB) stays live across this block's x1 MFMAs
                        asm volatile("" ::"v"(pmx[q]));
                    }
                }
                if (!LOOSE && MODE != 2 && (MODE < 11 || MODE == 13 || MODE == 15) && ss >= 6 && ss <= 8)  // this block: + |d_1| (RB, complete after step 5) -- before step 9
                    acc_abs(P, RB, ss == 6 ? 0 : ss == 7 ? C1 : C2, ss == 6 ? C1 : ss == 7 ? C2 : N3);
                if (!LOOSE && MODE != 2 && (MODE < 11 || MODE == 15) && ss >= 10)  // this block: + |d_2| (T2, complete after step 8)
                    acc_abs(P, T2, ss == 10 ? 0 : N3 / 2, ss == 10 ? N3 / 2 : N3);
                if (MODE == 13 && ss >= 9)  // experiment: the |d_2| adds in thirds over steps 9..11 (after step 9's MFMAs)
                    acc_abs(P, T2, ss == 9 ? 0 : ss == 10 ? C1 : C2, ss == 9 ? C1 : ss == 10 ? C2 : N3);
                if (MODE == 4 || MODE == 5) {  // experiment: one MFMA, then up to 6 VALU, twice per step
#pragma unroll
                    for (int g = 0; g < QB; g++) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
                    }
                }
                // program order is the schedule: nothing moves across a step (keeps each accumulator's
                // live range as written, so the role swap needs no extra registers)
                __builtin_amdgcn_sched_barrier(0);
            }
            if (more) {
                a0 = n0;
                a1 = n1;
            }
            if (s == 4 && MODE != 1 && MODE != 2 && (MODE < 11 || MODE == 13)) {
                // the previous block's list update (wave-uniform branch), then the back half
#pragma unroll
                for (int q = 0; q < QB; q++)
                    if (__builtin_expect(pend >= 0 && __any(pmx[q] > th[q]), 0)) {
                        float m4[4];
                        if (LOOSE) {
#pragma unroll
                            for (int sb = 0; sb < 4; sb++) m4[sb] = Sp[q][sb];
                        } else {
                            maxima(T2[q], m4);  // T2 still holds the previous block's bound until step 6
                        }
                        insert_block(q, m4, pend);
                    }
            }
        }
        pend = blk < b_end ? blk : -1;
    };

    for (int st = 0; st < nstage; st++) {
        const char *B = smem + (st & 1) * BUF_BYTES;
        const half8 *A = reinterpret_cast<const half8 *>(B) + lane;
        const float4 *SD = reinterpret_cast<const float4 *>(B + FRAG_BYTES) + h * 4;
        a0 = A[0];
        a1 = A[64];
        sd0 = SD[0];
        sd1 = SD[1];
        sd2 = SD[2];
        sd3 = SD[3];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (st + 1 < nstage) issue(st + 1, (st + 1) & 1);
#pragma unroll
        for (int cb = 0; cb < CB; cb += 2) {
            body(A, SD, cb, p_begin + st * CB + cb, RA, RC, SA, SC);
            body(A, SD, cb + 1, p_begin + st * CB + cb + 1, RC, RA, SC, SA);
        }
        dma_drain();
        __syncthreads();
    }
    // the last block's tail (odd position: P = RC)
    if (pend >= 0) {
#pragma unroll
        for (int q = 0; q < QB; q++) {
            float m4[4], mx;
            if (LOOSE) {
#pragma unroll
                for (int sb = 0; sb < 4; sb++)
                    m4[sb] = SC[q][sb] + fmaxf(fmaxf(fabsf(RB[q][4 * sb]), fabsf(RB[q][4 * sb + 1])),
                                               fmaxf(fabsf(RB[q][4 * sb + 2]), fabsf(RB[q][4 * sb + 3])));
                mx = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
            } else {
#pragma unroll
                for (int r = 0; r < 16; r++) RC[q][r] = RC[q][r] + fabsf(RB[q][r]);
                mx = maxima(RC[q], m4);
            }
            if (__any(mx > th[q])) insert_block(q, m4, pend);
        }
    }
#pragma unroll
    for (int q = 0; q < QB; q++) {
        const int qq = (qb0 + q) * 32 + (lane & 31);
        if (qb0 + q < nqblk && qq < nq) {
            const long o = (((long)qq * nsplit + split) * 2 + h) * L;
#pragma unroll
            for (int i = 0; i < L; i++) {
                out_key[o + i] = lk[q][i];
                out_id[o + i] = li[q][i];
            }
        }
    }
    if (MODE == 11 || MODE == 12 || MODE == 14)  // timing modes: the dummy adds stay live; the lists stay empty (as MODE 2)
#pragma unroll
        for (int i = 0; i < 16; i++) asm volatile("" ::"v"(dm[i]));
}

// ------------------------------------------------------------------------------------------
// device: orbit rescore, one wave per query
// ------------------------------------------------------------------------------------------
struct OrbitRescoreArgs {
    const float *rows, *q;          // fp32 candidate rows [n][192], query rows [nq][192]
    const _Float16 *rowh;           // fp16 c' [G][192]
    const half8 *qfrag;             // fp16 q' as MFMA B fragments [nqblk][12][64]
    const float *nc;                // [G]
    const int *member;              // [G][4]
    const uint8_t *dup;             // [G] bit x: slot x repeats a lower-index member's row
    const uint8_t *rep;             // [G] 2 bits per slot: slot of the lowest-index copy of its row
    const GroupOrder *gorder;       // [G] ANN's order inside each group (null: lowest-index tie order)
    const int *grp_of;              // [n] candidate -> g * 4 + slot
    const OrbitStat *ostat;
    const float *key;
    const int *id;
    int G, nq, L, nsplit;
    int q0;                         // first query of the launch (the launch covers [q0, nq))
    int p1;                         // entries re-keyed in the first pass (1..4)
    int *pair_cnt;                  // [nq] candidates handed to the pair pass (0: settled here or by tiers 2/3)
    int *pair_cand;                 // [nq][ORB_PSLOTS]
    double scale2;                  // scale^2
    double N, Np, Hp, Ecp;
    OrbitTail t;
};

// the reference distance (sequential fp32, every op rounded) with a short load window: the rescore
// runs one query per wave and needs occupancy more than load depth
__device__ __forceinline__ float exact_dist192_lean(const float *__restrict__ q, const float *__restrict__ c) {
    const float4 *q4 = reinterpret_cast<const float4 *>(q), *c4 = reinterpret_cast<const float4 *>(c);
    float dist = 0.0f;
#pragma unroll ORB_PR_UNROLL
    for (int i = 0; i < OD / 4; i++) {
        const float4 x = q4[i], y = c4[i];
        float t;
        t = x.x - y.x; dist = dist + t * t;
        t = x.y - y.y; dist = dist + t * t;
        t = x.z - y.z; dist = dist + t * t;
        t = x.w - y.w; dist = dist + t * t;
    }
    return dist;
}

// exact_dist192_lean for the 4 slot lanes of one query (a lane quad, every lane active): lane s loads 16-byte
// piece 4k + s of the query row and the quad broadcasts it by DPP, so each piece is requested once per quad
// instead of once per lane; the same values in the same order, so the same sum bit for bit
template <int CTRL>  // a DPP lane move (row_mask / bank_mask all rows, every lane written)
__device__ __forceinline__ int dpp_mov(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
template <int J>
__device__ __forceinline__ float quad_bcast(float v) {
    return __int_as_float(dpp_mov<J * 0x55>(__float_as_int(v)));
}
__device__ __forceinline__ float exact_dist192_quad(const float *__restrict__ q, const float *__restrict__ c, int s) {
    const float4 *q4 = reinterpret_cast<const float4 *>(q), *c4 = reinterpret_cast<const float4 *>(c);
    float dist = 0.0f;
    auto step = [&](const float4 &x, const float4 &y) __attribute__((always_inline)) {
        float t;
        t = x.x - y.x; dist = dist + t * t;
        t = x.y - y.y; dist = dist + t * t;
        t = x.z - y.z; dist = dist + t * t;
        t = x.w - y.w; dist = dist + t * t;
    };
#pragma unroll 2
    for (int k = 0; k < OD / 16; k++) {
        const float4 m = q4[4 * k + s];
        const float4 y0 = c4[4 * k], y1 = c4[4 * k + 1], y2 = c4[4 * k + 2], y3 = c4[4 * k + 3];
        step(make_float4(quad_bcast<0>(m.x), quad_bcast<0>(m.y), quad_bcast<0>(m.z), quad_bcast<0>(m.w)), y0);
        step(make_float4(quad_bcast<1>(m.x), quad_bcast<1>(m.y), quad_bcast<1>(m.z), quad_bcast<1>(m.w)), y1);
        step(make_float4(quad_bcast<2>(m.x), quad_bcast<2>(m.y), quad_bcast<2>(m.z), quad_bcast<2>(m.w)), y2);
        step(make_float4(quad_bcast<3>(m.x), quad_bcast<3>(m.y), quad_bcast<3>(m.z), quad_bcast<3>(m.w)), y3);
    }
    return dist;
}

__device__ __forceinline__ float wave_min_f(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}

static constexpr int ORB_XB = ORB_XBATCH;  // 16-byte loads in flight per lane in the re-key

// Re-key 2 list entries per half-wave: lane = (slot e, tile j, isotypic block x).  Each lane forms the 48-d partial
// dot d_x of its tile from the fp16 rows; a 2-stage Walsh-Hadamard butterfly over the 4 lanes of a tile turns
// (d_0..d_3) into the 4 mirror values V_m = sum_x chi_x(m) d_x, m = x of the lane.  Returns the candidate of
// mirror slot m (or -1) and its key ||c||^2 - 2 V_m.  `id` / `h`: the entry of this lane's slot (-1: none).
__device__ __forceinline__ int orbit_expand4(const OrbitRescoreArgs &a, long q, int id, int h, double &key) {
    typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
    const int lane = threadIdx.x & 63, j = (lane >> 2) & 3, x = lane & 3;
    const int g = (id >> 2) * 32 + 8 * (id & 3) + 4 * h + j;
    const bool gv = id >= 0 && g < a.G;
    float d = 0.0f;
    int cand = -1;
    unsigned dupb = 0;
    float ncg = 0.0f;
    if (gv) {  // fp16 products, fp32 sums (any order is inside the bound's gamma_{D+1} allowance)
        // the slot's member, the group's duplicate flags and norm travel with its fp16 row: one round trip where
        // the dependent loads after the butterfly took three more (r06q, `profiles/r06/q_rescore_ab.txt`: rescore 0.61 -> 0.55 ms)
        cand = a.member[(long)g * 4 + x];
        dupb = a.dup[g];
        ncg = a.nc[g];
        const uint4 *cr = reinterpret_cast<const uint4 *>(a.rowh + (long)g * OD + x * 48);
        // q' of block x from the MFMA B fragments: 16-byte piece t = (k-step 3x + t/2, half t%2) of query q
        const uint4 *qf = reinterpret_cast<const uint4 *>(a.qfrag) + ((q >> 5) * OS + 3 * x) * 64 + (q & 31);
#pragma unroll
        for (int t0 = 0; t0 < 6; t0 += ORB_XB) {
            uint4 cv[ORB_XB], qv[ORB_XB];
#pragma unroll
            for (int t = 0; t < ORB_XB; t++) {
                cv[t] = cr[t0 + t];
                qv[t] = qf[((t0 + t) >> 1) * 64 + 32 * ((t0 + t) & 1)];
            }
#pragma unroll
            for (int t = 0; t < ORB_XB; t++) {
                const half2_t *c2 = reinterpret_cast<const half2_t *>(&cv[t]);
                const half2_t *q2 = reinterpret_cast<const half2_t *>(&qv[t]);
#pragma unroll
                for (int u = 0; u < 4; u++) d = __builtin_amdgcn_fdot2(c2[u], q2[u], d, false);
            }
        }
    }
    float o = __shfl_xor(d, 1, 64);
    d = (x & 1) ? (o - d) : (d + o);
    o = __shfl_xor(d, 2, 64);
    d = (x & 2) ? (o - d) : (d + o);
    key = INFINITY;
    if (!gv || cand < 0 || ((dupb >> x) & 1)) return -1;
    key = (double)ncg - 2.0 * (double)d;
    return cand;  // the lowest-index copy of its row; the final pick resolves the copies (class_first)
}

// A candidate the rescore queued stands for every member of its group with an identical row (orbit_dup_kernel
// drops the others); under ANN's order the copy the kd-tree search finds first must be reported: resolved here,
// at the final pick, lane-parallel (kept out of the latency-bound rescore chain).
__device__ __forceinline__ void class_first(const OrbitRescoreArgs &a, const float *__restrict__ q, int &c, int &gs) {
    if (!a.gorder || gs < 0) return;
    const long g = gs >> 2;
    const int x = gs & 3;
    if (!a.dup[g]) return;
    const unsigned rep = a.rep[g];
    const GroupOrder *go = a.gorder + g;
    int bx = x;
    for (int y = 0; y < 4; y++) {
        const int cy = a.member[g * 4 + y];
        if (y != x && cy >= 0 && (int)((rep >> (2 * y)) & 3) == x && group_before(go, q, y, bx)) {
            bx = y;
            c = cy;
        }
    }
    gs = (int)(g * 4 + bx);
}

// ANN's order of two candidates for query q: one cached compare when they share an orbit group, the root walk
// (kdorder_dev.hpp) otherwise
__device__ __forceinline__ bool orbit_before(const OrbitRescoreArgs &a, const float *__restrict__ q, int c1, int gs1,
                                             int c2, int gs2) {
    if (a.gorder && gs1 >= 0 && gs2 >= 0 && (gs1 >> 2) == (gs2 >> 2) && c1 != c2)
        return group_before(a.gorder + (gs1 >> 2), q, gs1 & 3, gs2 & 3);
    return kd_before(a.t.ko, q, c1, c2);
}

// (dist, ANN order) minimum over a quad / half-wave: each lane holds (distance, candidate, its group code)
template <int WIDTH>
__device__ __forceinline__ void orbit_argmin(const OrbitRescoreArgs &a, const float *__restrict__ q, float &v, int &i,
                                             int &gs) {
#pragma unroll
    for (int off = WIDTH / 2; off > 0; off >>= 1) {
        float ov;
        int oi, og;
        if (WIDTH == 4 && ORB_RS_DPP) {  // the pair pass: one lane quad per query, every lane active
            ov = __int_as_float(off == 2 ? dpp_mov<0x4E>(__float_as_int(v)) : dpp_mov<0xB1>(__float_as_int(v)));
            oi = off == 2 ? dpp_mov<0x4E>(i) : dpp_mov<0xB1>(i);
            og = off == 2 ? dpp_mov<0x4E>(gs) : dpp_mov<0xB1>(gs);
        } else {
            ov = __shfl_xor(v, off, 64);
            oi = __shfl_xor(i, off, 64);
            og = __shfl_xor(gs, off, 64);
        }
        if (ov < v || (ov == v && orbit_before(a, q, oi, og, i, gs))) {
            v = ov;
            i = oi;
            gs = og;
        }
    }
}

// The rescore runs one query per HALF-wave (32 lanes): it is latency-bound (list -> re-key -> rows ->
// reference distances), so two independent chains per wave double the work in flight.  Every cross-lane
// operation below stays inside the half (xor offsets < 32, ballots masked to the half).
static constexpr int ORB_QCAP = 64;  // rescore queue per query
static constexpr int ORB_STG = ORB_STG_ROWS;  // candidate rows staged in LDS per pass
static constexpr int ORB_PSLOTS = 4; // candidates per query handed to the pair pass

// Lane moves of the half-wave reductions.  A minimum (of values, or of (value, index) pairs) is symmetric and
// associative, so any pairing that doubles the reduced span each step works: lane ^ 1 and lane ^ 2 (quad_perm), lane
// <-> 7 - lane and lane <-> 15 - lane (row half-mirror, row mirror) by DPP -- VALU lane moves, no LDS round trip --
// then lane ^ 16 by ds_bpermute.  Every lane of the half is active at each call site (the branches around them are
// uniform over the half-wave).  ORB_RS_DPP 0: five ds_bpermute steps (xor 16, 8, 4, 2, 1) as before (r06r,
// `profiles/r06/r_rescore_dpp_ab.txt`: rescore 0.540 -> 0.533 ms).
template <int STEP>  // STEP 0..4: the partner lane of the step
__device__ __forceinline__ int half_partner(int v) {
#if ORB_RS_DPP
    if (STEP == 0) return dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
    if (STEP == 1) return dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
    if (STEP == 2) return dpp_mov<0x141>(v);  // row_half_mirror: 7 - lane within 8
    if (STEP == 3) return dpp_mov<0x140>(v);  // row_mirror: 15 - lane within 16
    return __shfl_xor(v, 16, 64);
#else
    return __shfl_xor(v, 16 >> STEP, 64);
#endif
}
__device__ __forceinline__ float half_min_f(float v) {
    v = fminf(v, __int_as_float(half_partner<0>(__float_as_int(v))));
    v = fminf(v, __int_as_float(half_partner<1>(__float_as_int(v))));
    v = fminf(v, __int_as_float(half_partner<2>(__float_as_int(v))));
    v = fminf(v, __int_as_float(half_partner<3>(__float_as_int(v))));
    v = fminf(v, __int_as_float(half_partner<4>(__float_as_int(v))));
    return v;
}
template <int STEP>
__device__ __forceinline__ void half_argmin_step(float &v, int &i) {
    const float ov = __int_as_float(half_partner<STEP>(__float_as_int(v)));
    const int oi = half_partner<STEP>(i);
    const bool take = (ov < v) || (ov == v && (unsigned)oi < (unsigned)i);
    v = take ? ov : v;
    i = take ? oi : i;
}
__device__ __forceinline__ void half_argmin(float &v, int &i) {
    half_argmin_step<0>(v, i);
    half_argmin_step<1>(v, i);
    half_argmin_step<2>(v, i);
    half_argmin_step<3>(v, i);
    half_argmin_step<4>(v, i);
}
__device__ __forceinline__ unsigned half_ballot(bool p) {
    return (unsigned)(__ballot(p) >> (32 * ((threadIdx.x >> 5) & 1)));
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ORB_RS_WAVES))) void nn_orbit_rescore_kernel(OrbitRescoreArgs a) {
    const int l = threadIdx.x & 31, hq = threadIdx.x >> 5;  // lane in the half, query slot of the block
    const int hbase = threadIdx.x & 32;                     // first lane of this half in the wave
    const long q = (long)blockIdx.x * 8 + hq + a.q0;
    if (q >= a.nq) return;
    const OrbitTail &t = a.t;
    const OrbitStat st = a.ostat[q];
    const int E = a.nsplit * 2 * a.L;  // <= 32 (orbit_search limits nsplit)
    float ek = INFINITY;
    int eid = -1;
    if (l < E) {  // issued with the stat: the two loads do not wait for each other
        ek = a.key[q * E + l];
        eid = a.id[q * E + l];
    }
    if (l == 0) a.pair_cnt[q] = 0;  // the pair pass skips queries settled here or by tiers 2/3
    if (st.flags & 2) {
        if (l == 0) t.ex_list[atomicAdd(t.ex_count, 1)] = (int)q;
        return;
    }
    const int eh = (l / a.L) & 1;
    if (eid < 0) ek = INFINITY;
    const bool last = l < E && (l % a.L) == a.L - 1 && eid >= 0;
    // 1. the 2 entries with the smallest keys, re-keyed together (one round trip)
    int sel = -1;  // slot e (l >> 4) <- entry lane
    bool taken = false;
#pragma unroll
    for (int r = 0; r < 2; r++) {
        if (r >= a.p1) break;
        float v = (taken || !(ek < INFINITY)) ? INFINITY : ek;
        int who = l;
        half_argmin(v, who);
        if (v < INFINITY) {
            if (l == who) taken = true;
            if ((l >> 4) == r) sel = who;
        }
    }
    if (__shfl(sel, hbase, 64) < 0) {  // empty dataset
        if (l == 0) {
            t.out_idx[q] = -1;
            t.out_err[q] = FLT_MAX;
            if (t.m_tile) {
                t.m_tile[q] = -1;
                t.m_pal[q] = -1;
                t.m_hm[q] = 0;
                t.m_vm[q] = 0;
            }
        }
        return;
    }
    const int sl = sel < 0 ? 0 : sel;
    const int sid = __shfl(eid, hbase + sl, 64), shh = __shfl(eh, hbase + sl, 64);
    double k1;
    const int c1 = orbit_expand4(a, q, sel < 0 ? -1 : sid, shh, k1);
    float kk = c1 >= 0 ? (float)k1 : INFINITY;  // rounded: only sets a looser threshold below
    kk = half_min_f(kk);
    // 2. thresholds.  Some candidate has real key <= kk + Eo, so the winner's reference
    // distance is <= (n2 + kk + Eo)(1 + g); any candidate c that can reach it has real key <= Tr.
    const double u = 5.9604644775390625e-08;  // 2^-24
    const double g = (double)(OD + 4) * u / (1.0 - (double)(OD + 4) * u) * 1.05;
    const double gam = 2.0 * (OD + 1) * u;
    const double Eo = 1.05 * (2.0 * u * a.N * a.N + gam * (a.N * a.N + 2.0 * st.hn * a.Hp) +
                              2.0 * (st.en * a.Np + st.hn * a.Ecp)) + 1e-30;
    const double kd = (double)kk + 1e-6 * fabs((double)kk) + 1e-30;  // covers the fp32 rounding of kk
    const double Tr = (st.n2 + kd + Eo) * (1.0 + g) / (1.0 - g) - st.n2 + 1e-12 * (st.n2 + fabs(kd)) + 1e-30;
    const double Tb = Tr + Eo;
    // 3. overflow: a full lane list whose worst kept entry can still reach the threshold.  Tier 2
    // (nn_orbit_collect_kernel) re-scans every orbit against T_b in this same bound-key domain.
    if (half_ballot(last && (double)ek <= Tb)) {
        if (l == 0) {
            float tf = (float)Tb;
            if ((double)tf < Tb) tf = nextafterf(tf, INFINITY);  // an upper bound in fp32
            t.thr[q] = tf;
            const int pidx = atomicAdd(t.fb_count, 1);
            if (pidx < t.fb_max) {  // always (fb_max = nq)
                t.fb_list[pidx] = (int)q;
                t.t2_best[pidx] = ~0ull;
            } else {
                t.ex_list[atomicAdd(t.ex_count, 1)] = (int)q;
            }
        }
        return;
    }
    // 4. queue every candidate that can reach the threshold; entries beyond the first 2 that can hold
    // one are re-keyed 2 at a time; then the queue is rescored with the reference distance: candidate rows
    // are staged in LDS by the half-wave (one round trip), then one lane per candidate sums in order
    __shared__ int s_cand[8][ORB_QCAP];
    __shared__ float4 s_row[8][ORB_STG][OD / 4];
    int *sc = s_cand[hq];
    const float *qrow = a.q + q * OD;
    float bd = INFINITY;
    int bi = 0x7fffffff, bg = -1;
    int cnt = 0, nexp = 1, nres = 0;
    auto flush = [&]() {
        for (int b0 = 0; b0 < cnt; b0 += ORB_STG) {
            const int nb = min(ORB_STG, cnt - b0);
            for (int i = l; i < nb * (OD / 4); i += 32) {
                const int r = i / (OD / 4), c4 = i - r * (OD / 4);
                s_row[hq][r][c4] = reinterpret_cast<const float4 *>(a.rows + (long)sc[b0 + r] * OD)[c4];
            }
            __builtin_amdgcn_wave_barrier();
            if (l < nb) {
                const int c = sc[b0 + l];
                const float4 *q4 = reinterpret_cast<const float4 *>(qrow);
                float dist = 0.0f;
#pragma unroll ORB_DU
                for (int i = 0; i < OD / 4; i++) {
                    const float4 x = q4[i], y = s_row[hq][l][i];
                    float tt;
                    tt = x.x - y.x; dist = dist + tt * tt;
                    tt = x.y - y.y; dist = dist + tt * tt;
                    tt = x.z - y.z; dist = dist + tt * tt;
                    tt = x.w - y.w; dist = dist + tt * tt;
                }
                int cg = a.grp_of ? a.grp_of[c] : -1, cc = c;
                class_first(a, qrow, cc, cg);
                if (dist < bd || (dist == bd && orbit_before(a, qrow, cc, cg, bi, bg))) {
                    bd = dist;
                    bi = cc;
                    bg = cg;
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        nres += cnt;
        cnt = 0;
    };
    auto enqueue = [&](int c, double k) {
        const bool take = c >= 0 && k <= Tb;
        const unsigned b = half_ballot(take);
        if (take) sc[cnt + __popc(b & ((1u << l) - 1))] = c;
        cnt += __popc(b);
        __builtin_amdgcn_wave_barrier();
        if (cnt > ORB_QCAP - 32) flush();
    };
    enqueue(c1, k1);
    unsigned todo = half_ballot(!taken && eid >= 0 && (double)ek <= Tb);
    while (todo) {
        int el = -1;  // slot e <- the e-th remaining entry
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const int e = todo ? __builtin_ctz(todo) : -1;
            if (todo) todo &= todo - 1;
            if ((l >> 4) == r) el = e;
        }
        nexp++;
        const int ee = el < 0 ? 0 : el;
        const int xid = __shfl(eid, hbase + ee, 64), xh = __shfl(eh, hbase + ee, 64);
        double k;
        const int c = orbit_expand4(a, q, el < 0 ? -1 : xid, xh, k);
        enqueue(c, k);
    }
    __builtin_amdgcn_wave_barrier();
    if (nres == 0 && cnt > 0 && cnt <= ORB_PSLOTS) {
        // the usual case: a few candidates -> the reference distances run lane-parallel in the pair pass
        if (l < cnt) a.pair_cand[q * ORB_PSLOTS + l] = sc[l];
        if (l == 0) {
            a.pair_cnt[q] = cnt;
            if (t.n_expand) {
                atomicAdd(t.n_expand, nexp);
                atomicAdd(t.n_expand + 1, cnt);
            }
        }
        return;
    }
    flush();
    orbit_argmin<32>(a, qrow, bd, bi, bg);
    if (l == 0) {
        if (t.n_expand) {
            atomicAdd(t.n_expand, nexp);
            atomicAdd(t.n_expand + 1, nres);
        }
        const bool ok = bi != 0x7fffffff;
        t.out_idx[q] = ok ? bi : -1;
        t.out_err[q] = ok ? bd : FLT_MAX;
        if (t.m_tile) {
            t.m_tile[q] = ok ? t.tr_tile[bi] : -1;
            t.m_pal[q] = ok ? t.tr_pal[bi] : -1;
            const int at = ok ? t.tr_attr[bi] : 0;
            t.m_hm[q] = (at & 1) != 0;
            t.m_vm[q] = (at & 2) != 0;
        }
    }
}

// The reference distances of the rescore's queue, lane-parallel: lane = (query, slot), ORB_PSLOTS lanes per
// query; each lane sums its candidate in the reference order (sequential fp32, every op rounded), the
// query's lanes pick (distance, index) lexicographically and the first writes the tilemap item.  Running
// these 192-step chains here instead of one lane per candidate inside the half-wave rescore keeps the
// rescore's instruction stream short (it is latency-bound) and fills the lanes.  r03zr: staging the rows through LDS in
// coalesced 32-float column chunks (12 barriers, every slot's row loaded) took 1.00 ms vs 0.50 ms for this per-lane walk.
// r06o (`profiles/r06/o_pairs_ab.txt`): the query row's 16-byte pieces requested once per quad and broadcast by DPP
// (exact_dist192_quad) 0.50 -> 0.42 ms at C3, output digest unchanged; the load requests, not HBM, bound this pass.
#if ORB_PR_WAVES
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ORB_PR_WAVES))) void nn_orbit_pairs_kernel(OrbitRescoreArgs a) {
#else
__global__ __launch_bounds__(256) void nn_orbit_pairs_kernel(OrbitRescoreArgs a) {
#endif
    const long gid = (long)blockIdx.x * 256 + threadIdx.x;
    const long q = gid / ORB_PSLOTS + a.q0;
    const int s = (int)(gid % ORB_PSLOTS);
    float bd = INFINITY;
    if (q >= a.nq) return;  // whole groups: 256 % ORB_PSLOTS == 0
    const int n = a.pair_cnt[q];
    if (n == 0) return;  // uniform over the group
    int bi = 0x7fffffff, bg = -1;
#if ORB_PR_QUAD
    static_assert(ORB_PSLOTS == 4, "one lane quad per query");
    {  // every lane of the quad takes part in the broadcasts; a lane past the count re-reads slot 0's row
        const int c = a.pair_cand[q * ORB_PSLOTS + (s < n ? s : 0)];
        const float d = exact_dist192_quad(a.q + q * OD, a.rows + (long)c * OD, s);
        if (s < n) bd = d;
    }
#endif
    if (s < n) {
        int c = a.pair_cand[q * ORB_PSLOTS + s];
#if !ORB_PR_QUAD
        bd = exact_dist192_lean(a.q + q * OD, a.rows + (long)c * OD);
#endif
        if (a.grp_of) {
            bg = a.grp_of[c];
            class_first(a, a.q + q * OD, c, bg);  // same row, same distance
        }
        bi = c;
    }
    const OrbitTail &t = a.t;
    orbit_argmin<ORB_PSLOTS>(a, a.q + q * OD, bd, bi, bg);
    if (t.ko) {  // ANN's box pruning along the winner's path, with the query row still in cache
        const bool ok = kd_quad_path_ok(t.ko, a.q + q * OD, t.ko->pos[bi], t.kd_rootbox[q], bd, s);
        if (s == 0) {
            t.kd_done[q] = 1;
            if (!ok) t.kd_list[atomicAdd(t.kd_count, 1)] = (int)q;
        }
    }
    if (s == 0) {
        t.out_idx[q] = bi;
        t.out_err[q] = bd;
        if (t.m_tile) {
            t.m_tile[q] = t.tr_tile[bi];
            t.m_pal[q] = t.tr_pal[bi];
            const int at = t.tr_attr[bi];
            t.m_hm[q] = (at & 1) != 0;
            t.m_vm[q] = (at & 2) != 0;
        }
    }
}

// Tier 2 for the queries the orbit rescore could not settle (a lane list was full with its last key <= T_b): every
// orbit of the dataset is scored again with the tier-1 contraction -- the same q' fragments (the query's own
// column of its block), the same seeded d_0 and bound u = d_0 + |d_1| + |d_2| + |d_3| in fp32 -- and where the
// bound key -2u reaches T_b (rounded up to fp32 by the rescore), the four mirror keys -2 V_m, V_m = sum_x
// chi_x(m) d_x, are formed by the rescore's own butterfly and every member whose key reaches T_b is scored: its
// reference distance (sequential fp32) and its rank in ANN's visit order for this query (kd_rank) are packed into
// one u64 and min-reduced into t2_best[j] by an atomic, so (distance, ANN order) picks the winner whatever the number
// of candidates (duplicate rows included).  Any candidate that can reach the winner has real key <= T_r and so
// computed keys <= T_b, as in tier 1.  The members are queued per wave in LDS and scored
// lane-parallel, 64 at a time (the pair pass's idea), so near-tie floods keep every lane busy.  One wave = 32 tier-2
// queries (compact), workgroups split the orbit blocks; candidate fragments staged through LDS by LDS-DMA.
static constexpr int OC_CB = 2;    // orbit blocks per LDS stage
static constexpr int OC_XQ = 512;  // per-wave queue of (tier-2 slot, candidate) awaiting the exact score
struct OrbitCollectArgs {
    const half8 *cfrag;
    const float *cseed;
    int gblk;
    long G;
    const int *member;
    const half8 *qfrag;
    const int *fb_list, *fb_count;
    const float *thr;
    int blk_per_split;
    const float *rows;   // [n][192] fp32 candidate rows
    const float *q;      // [nq][192] fp32 query rows
    const KdOrder *ko;   // ANN tie order (nullptr: lowest index)
    unsigned long long *best;
};

__device__ __forceinline__ unsigned long long t2_key(float d, unsigned rank) {
    return ((unsigned long long)__float_as_uint(d) << 32) | rank;  // d >= 0: its bits order like the value
}

__global__ __launch_bounds__(256, 2) void nn_orbit_collect_kernel(OrbitCollectArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[2 * (OC_CB * OS * 1024 + OC_CB * 128)];
    __shared__ int2 xq[4][OC_XQ];
    constexpr int FRAG_BYTES = OC_CB * OS * 1024;
    constexpr int BUF_BYTES = FRAG_BYTES + OC_CB * 128;
    constexpr int PER_T = OC_CB * OS * 64 / 256;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
    const int count = *a.fb_count;  // every tier-2 query (fb_list has nq slots)
    const int b_begin = blockIdx.y * a.blk_per_split;
    const int b_end = min(a.gblk, b_begin + a.blk_per_split);
    const half8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};
    const floatx16 zero = {0};
    const unsigned long long below = (1ull << lane) - 1;
    int nx = 0;  // queue fill (wave-uniform)
    auto flush = [&]() __attribute__((always_inline)) {
        __builtin_amdgcn_wave_barrier();
        for (int e0 = 0; e0 < nx; e0 += 64) {
            const int e = e0 + lane;
            if (e < nx) {
                const int2 v = xq[w][e];
                const float *qrow = a.q + (long)a.fb_list[v.x] * OD;
                const float dist = exact_dist192_lean(qrow, a.rows + (long)v.y * OD);
                atomicMin(a.best + v.x, t2_key(dist, kd_rank(a.ko, qrow, v.y)));
            }
        }
        __builtin_amdgcn_wave_barrier();  // every lane has read its entries before the queue refills
        nx = 0;
    };
    for (int grp = blockIdx.x; grp * 128 < count; grp += gridDim.x) {
        const int j = (grp * 4 + w) * 32 + (lane & 31);
        const int q = j < count ? a.fb_list[j] : -1;
        const float t = q >= 0 ? a.thr[q] : -INFINITY;
        half8 bq[OS];
#pragma unroll
        for (int k = 0; k < OS; k++) bq[k] = q >= 0 ? a.qfrag[((long)(q >> 5) * OS + k) * 64 + (q & 31) + 32 * h] : zero8;
        const int nstage = (b_end > b_begin) ? (b_end - b_begin + OC_CB - 1) / OC_CB : 0;
        // candidate fragments + seeds straight to LDS (LDS-DMA, as the shortlist's ring)
        auto issue = [&](int st, int buf) __attribute__((always_inline)) {
            const int blk0 = b_begin + st * OC_CB;
            const int lastv = min(OC_CB, b_end - blk0) * OS * 64 - 1;
            const uint4 *src = reinterpret_cast<const uint4 *>(a.cfrag) + (long)blk0 * OS * 64;
            char *dst = smem + buf * BUF_BYTES + w * 1024;
#pragma unroll
            for (int jj = 0; jj < PER_T; jj++) glds16_asm(src + min(w * 64 + lane + jj * 256, lastv), dst + jj * 256 * 16);
            if (w == 0 && lane < OC_CB * 8)
                glds16_asm(reinterpret_cast<const uint4 *>(a.cseed) + (long)blk0 * 8 + min(lane, min(OC_CB, b_end - blk0) * 8 - 1),
                           smem + buf * BUF_BYTES + FRAG_BYTES);
        };
        __syncthreads();  // the previous group's reads of both buffers are done
        if (nstage > 0) issue(0, 0);
        dma_drain();
        __syncthreads();
        for (int st = 0; st < nstage; st++) {
            if (st + 1 < nstage) issue(st + 1, (st + 1) & 1);
            const char *B = smem + (st & 1) * BUF_BYTES;
            for (int cb = 0; cb < OC_CB; cb++) {
                const int blk = b_begin + st * OC_CB + cb;
                if (blk >= b_end) break;
                const float *sd = reinterpret_cast<const float *>(B + FRAG_BYTES) + cb * 32 + h * 16;
                floatx16 d[4];
#pragma unroll
                for (int r = 0; r < 16; r++) d[0][r] = sd[r];
                d[1] = d[2] = d[3] = zero;
#pragma unroll
                for (int k = 0; k < OS; k++) {
                    const half8 av = reinterpret_cast<const half8 *>(B)[(cb * OS + k) * 64 + lane];
                    d[k / 3] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bq[k], d[k / 3], 0, 0, 0);
                }
                unsigned pass = 0;  // element r: the orbit bound reaches T_b
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const float u = d[0][r] + fabsf(d[1][r]) + fabsf(d[2][r]) + fabsf(d[3][r]);
                    pass |= (q >= 0 && -2.0f * u <= t) ? 1u << r : 0u;
                }
                if (!__any(pass)) continue;  // the usual case (wave-uniform)
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const bool pr = (pass >> r) & 1;
                    if (!__any(pr)) continue;
                    const long g = (long)blk * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    int take = 0, m[4] = {-1, -1, -1, -1};
                    if (pr && g < a.G) {
                        const float a0 = d[0][r] + d[1][r], b0 = d[0][r] - d[1][r];
                        const float c0 = d[2][r] + d[3][r], e0 = d[2][r] - d[3][r];
                        const float V[4] = {a0 + c0, b0 + e0, a0 - c0, b0 - e0};
#pragma unroll
                        for (int x = 0; x < 4; x++) {
                            m[x] = a.member[g * 4 + x];
                            take |= (m[x] >= 0 && -2.0f * V[x] <= t) ? 1 << x : 0;
                        }
                    }
#pragma unroll
                    for (int x = 0; x < 4; x++) {  // append (j, member) in lane order
                        const bool bx = (take >> x) & 1;
                        const unsigned long long b = __ballot(bx);
                        if (bx) xq[w][nx + __popcll(b & below)] = make_int2(j, m[x]);
                        nx += __popcll(b);
                    }
                    if (nx > OC_XQ - 256) flush();  // room for the next element's <= 256 appends
                }
            }
            dma_drain();
            __syncthreads();
        }
        if (nx) flush();
    }
}

// the tier-2 winners: decode t2_best[j] -> candidate, write the outputs (kd_done stays 0: kd_verify checks them)
__global__ __launch_bounds__(256) void nn_orbit_t2_final_kernel(OrbitTail t, const float *__restrict__ qrows,
                                                                const float *__restrict__ rows) {
    const int count = *t.fb_count;
    for (long j = (long)blockIdx.x * 256 + threadIdx.x; j < count; j += (long)gridDim.x * 256) {
        const long q = t.fb_list[j];
        const unsigned long long k = t.t2_best[j];
        if (k == ~0ull) {  // nothing reached T_b: impossible for a finite query (the re-keyed entry does); exhaustive
            t.ex_list[atomicAdd(t.ex_count, 1)] = (int)q;
            continue;
        }
        const int c = kd_unrank(t.ko, qrows + q * OD, (unsigned)k);
        t.out_idx[q] = c;
        t.out_err[q] = __uint_as_float((unsigned)(k >> 32));
        if (t.m_tile) {
            t.m_tile[q] = t.tr_tile[c];
            t.m_pal[q] = t.tr_pal[c];
            const int at = t.tr_attr[c];
            t.m_hm[q] = (at & 1) != 0;
            t.m_vm[q] = (at & 2) != 0;
        }
    }
    (void)rows;
}

int orbit_tier2(NNIndex *ix, const float *d_q, const OrbitTail &tail, int nq, hipStream_t stream) {
    OrbitIndex *o = ix->orbit;
    // the tier-2 count stays on the device (no host round trip): many short candidate splits, and the x dimension
    // strides over the query groups of 128, so any count is served.  x is sized from the count the previous search
    // on this index left in the pinned h_fb_count (a heuristic only: a stale or racing value changes the grid, never
    // the result): one group per workgroup column when the count repeats (C3: ~1k tier-2 queries -> 10 columns,
    // 0.21 -> ~0.11 ms), 2 columns at least
    const int prev = ix->h_fb_count ? std::max(0, (int)((volatile int *)ix->h_fb_count)[0]) : 0;
    const int t2x_auto = std::max(2, std::min(64, (prev + prev / 4 + 127) / 128 + 1));
    const int t2x = t2x_auto;
#ifndef ORB_T2_WG
#define ORB_T2_WG 1024
#endif
    // candidate splits: about ORB_T2_WG workgroups in all (128..512 splits); r04t at C3: a fixed 512 splits (one per
    // 4 blocks) gave ~5,600 tiny workgroups, 0.152 ms -> 0.119 ms with ~1,000 (C2 0.059 -> 0.047), digests unchanged
    const int t2s = ORB_T2_WG > 0 ? std::max(128, std::min(512, ORB_T2_WG / std::max(1, std::min(t2x, (nq + 127) / 128))))
                                  : 512;
    const int nsplit = std::min(o->gblk, t2s);
    const int bps = (o->gblk + nsplit - 1) / nsplit;
    OrbitCollectArgs ca;
    ca.cfrag = (const half8 *)o->d_frag;
    ca.cseed = o->d_seed;
    ca.gblk = o->gblk;
    ca.G = o->G;
    ca.member = o->d_member;
    ca.qfrag = (const half8 *)o->qfrag;
    ca.fb_list = tail.fb_list;
    ca.fb_count = tail.fb_count;
    ca.thr = tail.thr;
    ca.blk_per_split = bps;
    ca.rows = ix->d_rows;
    ca.q = d_q;
    ca.ko = tail.ko;
    ca.best = tail.t2_best;
    {
        KTimer tm("nn_collect", stream);
        hipLaunchKernelGGL(nn_orbit_collect_kernel, dim3(std::min(t2x, (nq + 127) / 128), (o->gblk + bps - 1) / bps),
                           dim3(256), 0, stream, ca);
    }
    TILER_HIP_CHECK(hipGetLastError());
    {
        KTimer tm("nn_rescore2", stream);
        hipLaunchKernelGGL(nn_orbit_t2_final_kernel, dim3((unsigned)std::min(256, (nq + 255) / 256)), dim3(256), 0,
                           stream, tail, d_q, (const float *)ix->d_rows);
    }
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}


// ------------------------------------------------------------------------------------------
// device: FrameTiling queries in one pass (DoFrameTiling main.pas:4023-4025): RGB tile -> Haar PsyV (fp64, one
// lane per tile, psyv_dev.hpp) -> fp32 row (the exact rescoring operand) + the orbit transform q' = U' q as fp16
// MFMA B fragments + its error statistics (orbit_prep_kernel's math) + annBoxDistance to the kd-tree's box.
// The descriptors never round-trip HBM between the two steps.
// ------------------------------------------------------------------------------------------
struct FtQueryArgs {
    const int32_t *rgb;
    long n;
    int gamma;
    const double *gamma_lut;
    double haar_f, u_mul, v_mul;
    float scale;
    float *out32;        // [n][192]
    half8 *frag;         // [ceil(n/32)][12][64]
    OrbitStat *qstat;    // [n]
    const float *box;    // [2][192] or null
    float *rootbox;      // [n] when box
    int xmode;           // 0 (timing-experiment modes of round 2 lived here; results invalid when != 0)
    const int *perm;     // query i reads tile perm[i] (null: tile i)
};


// The same pass with TWO waves per 64-tile block: wave h holds input rows 4h..4h+3 of every tile (32 fp64 values per
// lane instead of 64, so the block keeps about half the registers and twice the waves per SIMD hide the loads).
// WaveletGS splits along rows with no exchange until its last level: level 1's column pairs (0,1) (2,3) | (4,5) (6,7)
// and level 2's (0,1) | (2,3) each lie in one wave; only level 3's pair of rows 0 and 1 (two values per tile) crosses,
// through LDS.  Every output element is formed by exactly the operations of haar_regs, so the rows are identical.
// After the Haar, wave 0 takes the kd root-box distance and wave 1 ||q||^2 (each a sequential sum in dimension
// order, as before); the orbit transform's 16 outputs per k-step split 8 / 8 (wave h writes fragment half h).
template <int H>
__device__ __forceinline__ void haar_half(double (&p)[32], double f, double (*xch)[64][2], int lane) {
    // slot s of p = local row s (input row 4H + s), 8 columns
#pragma unroll
    for (int s = 0; s < 4; s++) {  // level 1 rows (all 8 rows): L at x, H at x + 4
        double t[8];
#pragma unroll
        for (int x = 0; x < 4; x++) {
            const double a = p[s * 8 + 2 * x], b = p[s * 8 + 2 * x + 1];
            t[x] = (a + b) * f;
            t[x + 4] = (a - b) * f;
        }
#pragma unroll
        for (int x = 0; x < 8; x++) p[s * 8 + x] = t[x];
    }
#pragma unroll
    for (int x = 0; x < 8; x++) {  // level 1 columns: pairs (local 0,1) and (2,3) -> slots 0,1 = L (logical rows
        double t[4];               // 2H, 2H+1), slots 2,3 = H (logical rows 2H+4, 2H+5)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const double a = p[(2 * j) * 8 + x], b = p[(2 * j + 1) * 8 + x];
            t[j] = (a + b) * f;
            t[j + 2] = (a - b) * f;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) p[j * 8 + x] = t[j];
    }
#pragma unroll
    for (int s = 0; s < 2; s++) {  // level 2 rows (logical rows 2H, 2H+1 = slots 0, 1), columns 0..3
        const double a0 = p[s * 8 + 0], b0 = p[s * 8 + 1], a1 = p[s * 8 + 2], b1 = p[s * 8 + 3];
        p[s * 8 + 0] = (a0 + b0) * f;
        p[s * 8 + 1] = (a1 + b1) * f;
        p[s * 8 + 2] = (a0 - b0) * f;
        p[s * 8 + 3] = (a1 - b1) * f;
    }
#pragma unroll
    for (int x = 0; x < 4; x++) {  // level 2 columns: the pair (2H, 2H+1) -> L = logical row H (slot 0), H = row H+2 (slot 1)
        const double a = p[x], b = p[8 + x];
        p[x] = (a + b) * f;
        p[8 + x] = (a - b) * f;
    }
    // level 3 rows: logical row H (slot 0), columns 0..1
    {
        const double a = p[0], b = p[1];
        p[0] = (a + b) * f;
        p[1] = (a - b) * f;
    }
    // level 3 columns: rows 0 (wave 0) and 1 (wave 1) -> L = row 0 (wave 0), H = row 1 (wave 1)
    xch[H][lane][0] = p[0];
    xch[H][lane][1] = p[1];
    __syncthreads();
#pragma unroll
    for (int x = 0; x < 2; x++) {
        const double o = xch[1 - H][lane][x];
        p[x] = H == 0 ? (p[x] + o) * f : (o - p[x]) * f;
    }
}

// logical index (row * 8 + column) of slot value k of wave H after haar_half
template <int H>
__device__ __forceinline__ constexpr int haar_half_pos(int k) {
    const int s = k >> 3, x = k & 7;
    const int row = s >= 2 ? 2 * H + 4 + (s - 2) : (x < 4 ? (s == 0 ? H : H + 2) : 2 * H + s);
    return row * 8 + x;
}

// SM (store mode) of the kernel's outputs (rows, fragments, statistics: 1,188 B per tile, never re-read by this
// kernel): 0 plain, 1 non-temporal (`nt`: the line still stays in the XCD's L2), 2 `sc1` (the line leaves L2 once
// written), so the outputs do not evict the tile pixels from L2 between the three component passes
template <typename T>
__device__ __forceinline__ void st_out(T *p, const T &v, int sm) {
    static_assert(sizeof(T) == 16 || sizeof(T) == 4, "16- or 4-byte outputs");
    if (sm == 2) {
        if constexpr (sizeof(T) == 16) {
            typedef unsigned u4v __attribute__((ext_vector_type(4)));
            const u4v u = __builtin_bit_cast(u4v, v);
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(u) : "memory");
        } else {
            const unsigned u = __builtin_bit_cast(unsigned, v);
            asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(u) : "memory");
        }
    } else if (sm == 1) {
        __builtin_nontemporal_store(v, p);
    } else {
        *p = v;
    }
}
__device__ __forceinline__ void st_out(float4 *p, const float4 &v, int sm) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v w = {v.x, v.y, v.z, v.w};
    st_out(reinterpret_cast<f4v *>(p), w, sm);
}

template <bool FASTDIV, int H, int NT>
__device__ __forceinline__ void ft_query_half(const FtQueryArgs &a, double *lut, float *st, float *sbox,
                                              double (*xch)[64][2], double (*sred)[64]) {
    const int lane = threadIdx.x & 63;
    const long t0 = (long)blockIdx.x * 64;
    const long i = t0 + lane;
    const bool valid = i < a.n;
    const long nqblk = (a.n + 31) / 32;
    const bool has_blk = (i >> 5) < nqblk;
    const long ti = valid ? (a.perm ? (long)a.perm[i] : i) : (a.perm ? (long)a.perm[t0] : t0);
    const int4 *src = reinterpret_cast<const int4 *>(a.rgb + ti * 64) + 8 * H;
    constexpr int SM = NT;  // output store mode (st_out)
    double nb = 0, h2q[4] = {0, 0, 0, 0}, e2q[4] = {0, 0, 0, 0};  // nb: wave 0 -> (root-box, as float), wave 1 -> n2
    float rb = 0.0f;
    int bad = 0;
    const float *row = st + lane * 65;
#pragma unroll 1
    for (int c = 0; c < 3; c++) {
        double p[32];
#pragma unroll
        for (int k4 = 0; k4 < 8; k4++) {
            const int4 v = src[k4];
            const int cc[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int r = cc[e] & 0xff, g = (cc[e] >> 8) & 0xff, b = (cc[e] >> 16) & 0xff;
                const double fr = FASTDIV ? div255(r) : lut[r], fg = FASTDIV ? div255(g) : lut[g],
                             fb = FASTDIV ? div255(b) : lut[b];
                const double cy = div10000<FASTDIV>(2126.0 * fr + 7152.0 * fg + 722.0 * fb);
                p[4 * k4 + e] = c == 0 ? cy : c == 1 ? (fb - cy) * a.u_mul : (fr - cy) * a.v_mul;
            }
        }
        haar_half<H>(p, a.haar_f, xch, lane);
#pragma unroll
        for (int k = 0; k < 32; k++) st[lane * 65 + haar_half_pos<H>(k)] = (float)p[k];
        __syncthreads();
        if (H == 0 && a.box) {
#pragma unroll 4
            for (int k = 0; k < 64; k++) {  // annBoxDistance, dimension order
                const float v = row[k];
                const float lo = sbox[c * 64 + k], hi = sbox[OD + c * 64 + k];
                const float t = fmaxf(lo - v, 0.0f) + fmaxf(v - hi, 0.0f);  // lo <= hi: one term at most; + 0 exact
                rb = rb + t * t;
            }
        }
        if (H == 1 && valid) {
#pragma unroll 8
            for (int k = 0; k < 64; k++) {
                const double orig = (double)row[k] * (double)a.scale;
                nb += orig * orig;
            }
        }
        // fp32 rows: 16 lanes per tile store its 256-byte component segment, both waves
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const int pc = threadIdx.x + 128 * t, tt = pc >> 4, c4 = pc & 15;
            if (t0 + tt < a.n) {
                const float *q = st + tt * 65 + c4 * 4;
                st_out(reinterpret_cast<float4 *>(a.out32 + (t0 + tt) * OD + c * 64) + c4, make_float4(q[0], q[1], q[2], q[3]),
                       SM);
            }
        }
#pragma unroll
        for (int x = 0; x < 4; x++) {  // fully unrolled: every table word is a compile-time constant
            const int s = 3 * x + c;
            half8 hv;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const unsigned w = orbitgen::PACK[x * 16 + 8 * H + j];
                const int cnt = (int)(w >> 28);
                double v = 0.0;
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    if (t < cnt) {  // absent terms would add +0 to a v that is never -0: skipping them is exact
                        const double r = (double)row[(w >> (6 * t)) & 63];
                        v = ((w >> (24 + t)) & 1) ? v - r : v + r;
                    }
                }
                v = valid ? v * ((cnt == 1 ? 1.0 : 0.5) * (double)a.scale) : 0.0;
                _Float16 vh = (_Float16)(float)v;
                if (fabs((double)(float)vh) < 6.103515625e-05) vh = (_Float16)0.0f;  // no fp16 subnormal operands
                hv[j] = vh;
                const double dh = (double)(float)vh;
                h2q[j & 3] += dh * dh;
                e2q[j & 3] += (v - dh) * (v - dh);
                if (!isfinite(v) || fabs(v) > 65000.0) bad = 1;
                if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
            if (has_blk) st_out(a.frag + ((i >> 5) * OS + s) * 64 + (i & 31) + 32 * H, hv, SM);
            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();  // st and xch are rewritten by the next component
    }
    const double h2 = (h2q[0] + h2q[1]) + (h2q[2] + h2q[3]), e2 = (e2q[0] + e2q[1]) + (e2q[2] + e2q[3]);
    if (H == 1) {
        sred[0][lane] = h2;
        sred[1][lane] = e2;
        sred[2][lane] = nb;
        sred[3][lane] = bad ? 1.0 : 0.0;
    }
    __syncthreads();
    if (H == 0 && valid) {
        const double n2 = sred[2][lane];
        OrbitStat q;
        q.n2 = n2;
        q.hn = sqrt(h2 + sred[0][lane]);
        q.en = sqrt(e2 + sred[1][lane]);
        q.flags = (bad || sred[3][lane] != 0.0 || !isfinite(n2)) ? 2 : 0;
        q.pad = 0;
        a.qstat[i] = q;
        if (a.rootbox) st_out(a.rootbox + i, rb, SM);
    }
}

template <bool FASTDIV, int NT>
__global__ __launch_bounds__(128) void orbit_ft_query2_kernel(FtQueryArgs a) {
    __shared__ double lut[256];
    __shared__ float st[64 * 65];
    __shared__ float sbox[2 * OD];
    __shared__ double xch[2][64][2];
    __shared__ double sred[4][64];
    const double *__restrict__ glut = a.gamma_lut + 256 * (a.gamma + 1);
    for (int i = threadIdx.x; i < 256; i += 128) lut[i] = glut[i];
    if (a.box)
        for (int i = threadIdx.x; i < 2 * OD; i += 128) sbox[i] = a.box[i];
    __syncthreads();
    if (threadIdx.x < 64)
        ft_query_half<FASTDIV, 0, NT>(a, lut, st, sbox, xch, sred);
    else
        ft_query_half<FASTDIV, 1, NT>(a, lut, st, sbox, xch, sred);
}

int orbit_ft_queries(NNIndex *ix, const int32_t *d_rgb, int Q, int gamma, float *qrows, const float *box,
                     float *rootbox, hipStream_t stream, const int *perm) {
    OrbitIndex *o = ix->orbit;
    if (orbit_ensure_queries(o, Q)) return -1;
    if (gamma < -1 || gamma > 1) {
        set_error("frame tiling: gamma must be -1, 0 or 1");
        return -1;
    }
    const Luts &L = luts();
    FtQueryArgs fa;
    fa.rgb = d_rgb;
    fa.n = Q;
    fa.gamma = gamma;
    fa.gamma_lut = L.d_gamma;
    fa.haar_f = L.haar_f;
    fa.u_mul = L.u_mul;
    fa.v_mul = L.v_mul;
    fa.scale = ix->scale;
    fa.out32 = qrows;
    fa.frag = (half8 *)o->qfrag;
    fa.qstat = o->qstat;
    fa.box = box;
    fa.rootbox = rootbox;
    fa.xmode = 0;
    fa.perm = perm;
    const dim3 grid((unsigned)((Q + 63) / 64));
    KTimer tm("psyv", stream);
    // output stores non-temporal (template 1; r03g: plain 0.426 ms, nt 0.396-0.399, sc1 0.414 at C3)
    if (gamma != -1)
        hipLaunchKernelGGL((orbit_ft_query2_kernel<false, 1>), grid, dim3(128), 0, stream, fa);
    else
        hipLaunchKernelGGL((orbit_ft_query2_kernel<true, 1>), grid, dim3(128), 0, stream, fa);
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

// ------------------------------------------------------------------------------------------
// host
// ------------------------------------------------------------------------------------------
static double bits2d(unsigned long long b) {
    double v;
    memcpy(&v, &b, 8);
    return v;
}

// base = the groups' base rows rows[member[g][0]] in OrbitIndex::d_base's interleaved layout, zero past G
__global__ __launch_bounds__(256) void orbit_base_kernel(const float *__restrict__ rows, const int *__restrict__ member,
                                                         long G, float4 *__restrict__ base) {
    constexpr int W = OD / 4;
    const long total = (G + 63) / 64 * 64 * W;
    for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
        const long blk = t / (64 * W);
        const int k = (int)(t / 64 % W), l = (int)(t % 64);
        const long g = blk * 64 + l;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (g < G) v = reinterpret_cast<const float4 *>(rows)[(long)member[g * 4] * W + k];
        base[t] = v;
    }
}

void orbit_destroy(OrbitIndex *o, bool synced) {
    if (!o) return;
    if (!synced) (void)hipDeviceSynchronize();  // dfree files the blocks for reuse: nothing may still read them (hipFree's rule)
    dfree(o->d_bmask);
    dfree(o->d_bmask0);
    dfree(o->d_frag);
    dfree(o->d_rowh);
    dfree(o->d_seed);
    dfree(o->d_nc);
    dfree(o->d_member);
    dfree(o->d_dup);
    dfree(o->d_rep);
    dfree(o->d_gorder);
    dfree(o->d_grp_of);
    dfree(o->d_map);
    dfree(o->d_base);
    dfree(o->qfrag);
    dfree(o->qstat);
    dfree(o->pair_cnt);
    dfree(o->pair_cand);
    dfree(o->d_stats);
    dfree(o->key);
    dfree(o->id);
    if (o->tail_stream) stream_put(o->tail_stream);
    if (o->ev_half) (void)hipEventDestroy(o->ev_half);
    if (o->ev_tail) (void)hipEventDestroy(o->ev_tail);
    delete o;
}

int orbit_build(NNIndex *ix, hipStream_t stream) {
    if (ix->d != OD || ix->S == 0 || ix->exact_int || ix->n < 2) return 1;
    static OrbitMap hmap;
    static int map_ok = -1;
    if (map_ok < 0) map_ok = build_map(hmap) ? 1 : 0;
    if (!map_ok) return 1;
    const long n = ix->n;
    OrbitMap *d_map = nullptr;
    uint16_t *d_bits = nullptr;
    TILER_HIP_CHECK(dmalloc((void **)&d_map, sizeof(OrbitMap)));
    TILER_HIP_CHECK(hipMemcpyAsync(d_map, &hmap, sizeof(OrbitMap), hipMemcpyHostToDevice, stream));
    TILER_HIP_CHECK(dmalloc((void **)&d_bits, n * sizeof(uint16_t)));
    std::vector<uint16_t> bits(n);
    std::vector<int> member;
    // greedy grouping of rows [0, m) in index order: candidate j joins the open group (base s) in a free mirror slot
    // if row_j == S_slot row_s (checked on the device by orbit_eq_kernel); otherwise it opens a new group
    auto group = [&](long m) {
        member.clear();
        member.reserve(m + 4);
        long start = -1;
        int used = 0;
        for (long j = 0; j < m; j++) {
            bool joined = false;
            const long tt = j - start;
            if (start >= 0 && tt >= 1 && tt <= 3) {
                for (int q = 1; q <= 3 && !joined; q++)
                    if (!((used >> q) & 1) && ((bits[start] >> ((tt - 1) * 3 + q - 1)) & 1)) {
                        member[member.size() - 4 + q] = (int)j;
                        used |= 1 << q;
                        joined = true;
                    }
            }
            if (!joined) {
                member.push_back((int)j);
                member.push_back(-1);
                member.push_back(-1);
                member.push_back(-1);
                start = j;
                used = 1;
            }
        }
    };
    // A large set first checks a prefix: the candidate sets real PrepareFrameTiling builds from unrelated tiles are
    // nearly all singletons (r05: 99.7 %), and their full check read every row (0.75 ms at 387k rows) and waited for
    // it, beside the FrameTiling shortlist.  The choice only selects the kernels (both paths are exact).  r06pre
    // (profiles/r06/pre_orbit_prefix_encoder_ab.txt, same digests): whole-tileset encoder loop 9.30 -> 9.37 Mtiles/s.
    const long npre = std::min<long>(n, 16384);
    if (n > 4 * npre) {
        hipLaunchKernelGGL(orbit_eq_kernel, dim3((unsigned)((npre + 3) / 4)), dim3(256), 0, stream, ix->d_rows, npre,
                           d_map, d_bits);
        TILER_HIP_CHECK(hipGetLastError());
        TILER_HIP_CHECK(hipMemcpyAsync(bits.data(), d_bits, npre * sizeof(uint16_t), hipMemcpyDeviceToHost, stream));
        TILER_HIP_CHECK(hipStreamSynchronize(stream));
        group(npre);
        if ((long)member.size() / 4 * 20 > npre * 19) {  // >= 95 % singletons in the prefix: plain
            dfree(d_bits);
            dfree(d_map);
            return 1;
        }
    }
    hipLaunchKernelGGL(orbit_eq_kernel, dim3((unsigned)std::min<long>(8192, (n + 3) / 4)), dim3(256), 0, stream,
                       ix->d_rows, n, d_map, d_bits);
    TILER_HIP_CHECK(hipGetLastError());
    TILER_HIP_CHECK(hipMemcpyAsync(bits.data(), d_bits, n * sizeof(uint16_t), hipMemcpyDeviceToHost, stream));
    TILER_HIP_CHECK(hipStreamSynchronize(stream));
    dfree(d_bits);
    group(n);
    const long G = (long)member.size() / 4;
    if (G * 10 > n * 7) {  // < ~1.43 candidates per orbit: the generic kernels are as fast
        dfree(d_map);
        return 1;
    }
    OrbitIndex *o = new OrbitIndex();
    o->G = (int)G;
    o->gblk = (int)((G + 31) / 32);
    o->d_map = d_map;
    OrbitDsStat *d_ds = nullptr;
    TILER_HIP_CHECK(dmalloc((void **)&o->d_member, G * 4 * sizeof(int)));
    TILER_HIP_CHECK(hipMemcpyAsync(o->d_member, member.data(), G * 4 * sizeof(int), hipMemcpyHostToDevice, stream));
    TILER_HIP_CHECK(dmalloc((void **)&o->d_dup, G));
    TILER_HIP_CHECK(dmalloc((void **)&o->d_rep, G));
    hipLaunchKernelGGL(orbit_dup_kernel, dim3((unsigned)std::min<long>(8192, (G + 3) / 4)), dim3(256), 0, stream,
                       ix->d_rows, o->d_member, G, o->d_dup, o->d_rep);
    if (ix->kd) {  // ANN's order inside every group (the tree exists: nn_index_create_dev builds it first)
        TILER_HIP_CHECK(dmalloc((void **)&o->d_gorder, G * sizeof(GroupOrder)));
        TILER_HIP_CHECK(dmalloc((void **)&o->d_grp_of, n * sizeof(int)));
        TILER_HIP_CHECK(hipMemsetAsync(o->d_grp_of, 0xff, n * sizeof(int), stream));
        hipLaunchKernelGGL(orbit_gorder_kernel, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, stream, ix->kd->view(),
                           o->d_member, G, o->d_gorder, o->d_grp_of);
    }
    TILER_HIP_CHECK(hipGetLastError());
    TILER_HIP_CHECK(dmalloc(&o->d_frag, (size_t)o->gblk * OS * 1024));
    TILER_HIP_CHECK(dmalloc(&o->d_rowh, (size_t)G * OD * 2));
    TILER_HIP_CHECK(dmalloc((void **)&o->d_seed, (size_t)o->gblk * 32 * sizeof(float)));
    TILER_HIP_CHECK(dmalloc((void **)&o->d_nc, (size_t)G * sizeof(float)));
    TILER_HIP_CHECK(dmalloc((void **)&d_ds, sizeof(OrbitDsStat)));
    TILER_HIP_CHECK(hipMemsetAsync(d_ds, 0, sizeof(OrbitDsStat), stream));
    OrbitPrepArgs pa{ix->d_rows, o->d_member, G, (const OrbitMap *)d_map, ix->scale, (half8 *)o->d_frag,
                     (_Float16 *)o->d_rowh, o->d_seed, o->d_nc, d_ds, nullptr};
    hipLaunchKernelGGL(orbit_prep_kernel, dim3((unsigned)std::min<long>(4096, (o->gblk + ORB_PW - 1) / ORB_PW)),
                       dim3(64 * ORB_PW), 0, stream, pa);
    TILER_HIP_CHECK(hipGetLastError());
    OrbitDsStat ds;
    TILER_HIP_CHECK(hipMemcpyAsync(&ds, d_ds, sizeof(ds), hipMemcpyDeviceToHost, stream));
    TILER_HIP_CHECK(hipStreamSynchronize(stream));
    dfree(d_ds);
    if (ds.bad) {
        orbit_destroy(o);
        return 1;
    }
    o->N = sqrt(bits2d(ds.max_n2));
    o->Np = sqrt(bits2d(ds.max_p2));
    o->Hp = sqrt(bits2d(ds.max_h2));
    o->Ecp = sqrt(bits2d(ds.max_e2));
    o->ksteps = 12 * o->gblk;
    // Mirror-symmetric groups: an H- (V-) symmetric tile's c' is exactly zero in the isotypic blocks odd under H (V),
    // so those k-steps contribute +-0 to every query's d_x and |d_x| adds +0 to a bound that is never -0: skipping
    // them gives the same bits.  Groups are reordered (stably) so that the ones with zero blocks come first --
    // {0} only, then {0,2}, then {0,1} -- and the shortlist runs those blocks with only their nonzero k-steps.
    // Every other structure is indexed by the group number and rebuilt for the new order (member drives them all).
    {
        uint8_t *d_mask = nullptr;
        TILER_HIP_CHECK(dmalloc((void **)&d_mask, G));
        hipLaunchKernelGGL(orbit_zmask_kernel, dim3((unsigned)std::min<long>(8192, (G + 3) / 4)), dim3(256), 0, stream,
                           (const _Float16 *)o->d_rowh, G, d_mask);
        std::vector<uint8_t> mask(G);
        TILER_HIP_CHECK(hipMemcpyAsync(mask.data(), d_mask, G, hipMemcpyDeviceToHost, stream));
        TILER_HIP_CHECK(hipStreamSynchronize(stream));
        dfree(d_mask);
        auto key = [](unsigned m) { return (m & ~1u) == 0 ? 0 : (m & ~5u) == 0 ? 1 : (m & ~3u) == 0 ? 2 : 3; };
        long cnt[5] = {0, 0, 0, 0, 0};  // stable counting sort by class (4 keys)
        for (long g = 0; g < G; g++) cnt[key(mask[g]) + 1]++;
        const long nred = cnt[1] + cnt[2] + cnt[3];
        if (nred >= 64) {
            for (int k = 1; k < 5; k++) cnt[k] += cnt[k - 1];
            std::vector<int> order(G);
            for (long g = 0; g < G; g++) order[cnt[key(mask[g])]++] = (int)g;
            std::vector<int> pm((size_t)G * 4);
            for (long g = 0; g < G; g++)
                for (int x = 0; x < 4; x++) pm[g * 4 + x] = member[(size_t)order[g] * 4 + x];
            o->red_end = (int)((nred + 31) / 32);
            std::vector<uint8_t> bm(o->red_end, 0);
            for (long g = 0; g < (long)o->red_end * 32 && g < G; g++) bm[g / 32] |= mask[order[g]] | 1u;
            o->ksteps = 12 * (o->gblk - o->red_end);
            for (int b = 0; b < o->red_end; b++) o->ksteps += 3 * __builtin_popcount(bm[b]);
            TILER_HIP_CHECK(dmalloc((void **)&o->d_bmask, o->red_end));
            TILER_HIP_CHECK(hipMemcpyAsync(o->d_bmask, bm.data(), o->red_end, hipMemcpyHostToDevice, stream));
            TILER_HIP_CHECK(hipMemcpyAsync(o->d_member, pm.data(), G * 4 * sizeof(int), hipMemcpyHostToDevice, stream));
            hipLaunchKernelGGL(orbit_dup_kernel, dim3((unsigned)std::min<long>(8192, (G + 3) / 4)), dim3(256), 0, stream,
                               ix->d_rows, o->d_member, G, o->d_dup, o->d_rep);
            if (ix->kd) {
                TILER_HIP_CHECK(hipMemsetAsync(o->d_grp_of, 0xff, n * sizeof(int), stream));
                hipLaunchKernelGGL(orbit_gorder_kernel, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, stream,
                                   ix->kd->view(), o->d_member, G, o->d_gorder, o->d_grp_of);
            }
            TILER_HIP_CHECK(dmalloc((void **)&d_ds, sizeof(OrbitDsStat)));
            TILER_HIP_CHECK(hipMemsetAsync(d_ds, 0, sizeof(OrbitDsStat), stream));
            OrbitPrepArgs pb{ix->d_rows, o->d_member, G, (const OrbitMap *)d_map, ix->scale, (half8 *)o->d_frag,
                             (_Float16 *)o->d_rowh, o->d_seed, o->d_nc, d_ds, nullptr};
            hipLaunchKernelGGL(orbit_prep_kernel, dim3((unsigned)std::min<long>(4096, (o->gblk + ORB_PW - 1) / ORB_PW)),
                               dim3(64 * ORB_PW), 0, stream, pb);
            TILER_HIP_CHECK(hipGetLastError());
            TILER_HIP_CHECK(hipStreamSynchronize(stream));  // (pm, bm) stay alive until the copies are done
            dfree(d_ds);
        }
    }
    {  // the base rows in (final) group order for the small-batch orbit scan, whose mirror tables are compiled in
        bool ok = true;
        for (int m = 0; m < 3; m++)
            for (int i = 0; i < OD; i++) {
                const int c0 = (i / 64) * 64;
                ok = ok && hmap.msrc[m][i] == c0 + orbitgen::MSRC[m][i % 64] &&
                     hmap.msgn[m][i] == (orbitgen::MNEG[m][i % 64] ? -1.0f : 1.0f);
            }
        if (ok) {
            const long nb = (G + 63) / 64;
            TILER_HIP_CHECK(dmalloc((void **)&o->d_base, (size_t)nb * 64 * OD * sizeof(float)));
            hipLaunchKernelGGL(orbit_base_kernel, dim3((unsigned)std::min<long>(8192, (nb * 64 * (OD / 4) + 255) / 256)),
                               dim3(256), 0, stream, ix->d_rows, (const int *)o->d_member, G, (float4 *)o->d_base);
            TILER_HIP_CHECK(hipGetLastError());
        }
    }
    {  // block 0 only, every block: the flat query tiles' shortlist (orbit_search)
        std::vector<uint8_t> ones(o->gblk, 1);
        TILER_HIP_CHECK(dmalloc((void **)&o->d_bmask0, o->gblk));
        TILER_HIP_CHECK(hipMemcpyAsync(o->d_bmask0, ones.data(), o->gblk, hipMemcpyHostToDevice, stream));
        TILER_HIP_CHECK(hipStreamSynchronize(stream));
    }
    ix->orbit = o;
    return 0;
}

static constexpr int ORB_L = 4, ORB_CB = 4, ORB_NW = 8, ORB_QB = 2;

int orbit_ensure_queries(OrbitIndex *o, int nq) {
    if ((size_t)nq <= o->cap_q) return 0;
    const long nqblk = (nq + 31) / 32;
    if (o->qfrag || o->qstat || o->pair_cnt || o->pair_cand)  // (a first call has nothing to file: ensure_scratch)
        (void)hipDeviceSynchronize();  // the smaller buffers go back to the block cache: earlier searches must be done
    dfree(o->qfrag);
    dfree(o->qstat);
    dfree(o->pair_cnt);
    dfree(o->pair_cand);
    o->qfrag = nullptr;  // a failed allocation below leaves nothing dangling
    o->qstat = nullptr;
    o->pair_cnt = o->pair_cand = nullptr;
    o->cap_q = 0;
    TILER_HIP_CHECK(dmalloc((void **)&o->pair_cnt, (size_t)nq * sizeof(int)));
    TILER_HIP_CHECK(dmalloc((void **)&o->pair_cand, (size_t)nq * ORB_PSLOTS * sizeof(int)));
    TILER_HIP_CHECK(dmalloc(&o->qfrag, (size_t)(nqblk + 1) * OS * 1024));
    TILER_HIP_CHECK(dmalloc((void **)&o->qstat, (size_t)nq * sizeof(OrbitStat)));
    o->cap_q = nq;
    return 0;
}

int orbit_search(NNIndex *ix, const float *d_q, int nq, const OrbitTail &tail, hipStream_t stream,
                 bool queries_prepared) {
    OrbitIndex *o = ix->orbit;
    const int nqblk = (nq + 31) / 32;
    const int qpw = ORB_NW * ORB_QB;  // query blocks per workgroup (ORB_QB per wave)
    const int wgs = (nqblk + qpw - 1) / qpw;
    const int max_split = 32 / (2 * ORB_L);  // rescore: one list entry per lane of a half-wave
    // One 8-wave workgroup fills a CU (2 waves per SIMD), so a launch runs in rounds of n_cu workgroups of
    // ceil(gblk / ns) tile blocks each for ns candidate splits: pick the cheapest, preferring fewer splits (each adds
    // list entries to rescore) unless more are >= 2 % faster.  C3: 1,519 workgroups, 1 split (5.93 -> 6 rounds);
    // C2: 675 workgroups, 1 split (3 rounds of 512 blocks: 2.22 ms; 3 splits, 8 rounds of 171: 2.36 ms).
    static const int n_cu = [] {
        int dev = 0, cu = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
        return cu > 0 ? cu : 256;
    }();
    // A workgroup also pays a fixed cost of about ORB_WG_FIXED tile blocks (prologue, list start-up, epilogue: C2
    // with 3 splits ran 1.72 us per block-round against 1.26 at C3), so a round is priced as its blocks + that.
    constexpr double ORB_WG_FIXED = 64.0;
    int nsplit = 1;
    double best_t = 1e30;
    for (int ns = 1; ns <= max_split && ns <= o->gblk; ns++) {
        const double t = std::ceil((double)wgs * ns / n_cu) * (std::ceil((double)o->gblk / ns) + ORB_WG_FIXED);
        if (t < best_t * 0.98) {
            best_t = t;
            nsplit = ns;
        }
    }
    // Mixed: when the last round of whole-candidate workgroups is ragged (C2: 675 workgroups = 2.64 rounds), the
    // first R * n_cu workgroups scan every block and only the remaining ones split their blocks mix_ns ways
    // (C2: 3 rounds of 576 -> 2 x 576 + 2 x 235 block-times).  Lists keep the mix_ns stride for every query;
    // the whole-candidate part's other splits are empty entries.
    int mix_full = 0;
    {
        const int R = wgs / n_cu, rem = wgs - R * n_cu;
        for (int ns = 2; R >= 1 && rem > 0 && ns <= max_split && ns <= o->gblk; ns++) {
            const double t = R * (o->gblk + ORB_WG_FIXED) +
                             std::ceil((double)rem * ns / n_cu) * (std::ceil((double)o->gblk / ns) + ORB_WG_FIXED);
            if (t < best_t * 0.98) {
                best_t = t;
                nsplit = ns;
                mix_full = R * n_cu;
            }
        }
    }
    // Flat query tiles (from *tail.flat_cnt on, FrameTiling moves them last): their q' has only block 0, so the
    // workgroups made of them alone run the block-serial body with 3 of the 12 k-steps on every candidate block
    // (d_1..d_3 are +-0 for them: the same bounds bit for bit).  The count stays on the device: the kernel derives its
    // first all-flat workgroup from it, with any candidate split (the mixed launch is not used then).
    const int qpw_q = qpw * 32;  // queries per workgroup
    const int *flat_cnt = tail.flat_cnt;
    if (flat_cnt) mix_full = 0;
    const int bps = (o->gblk + nsplit - 1) / nsplit;
    nsplit = (o->gblk + bps - 1) / bps;
    // Two query halves (whole rounds of n_cu workgroups first): the first half's rescore and pair pass -- latency-bound
    // kernels -- run on the index's second stream while the second half's shortlist runs, instead of after it.
    int split_q = 0;
    if (ORB_SPLIT_TAILS && !mix_full && wgs >= 2 * n_cu) {
        const int wa = std::max(1, (wgs / 2 + n_cu / 2) / n_cu) * n_cu;
        if (wa < wgs && (long)wa * qpw_q < nq) {
            if (!o->tail_stream) TILER_HIP_CHECK(stream_get(&o->tail_stream));
            if (!o->ev_half) TILER_HIP_CHECK(hipEventCreateWithFlags(&o->ev_half, hipEventDisableTiming));
            if (!o->ev_tail) TILER_HIP_CHECK(hipEventCreateWithFlags(&o->ev_tail, hipEventDisableTiming));
            split_q = wa * qpw_q;
        }
    }
    if (orbit_ensure_queries(o, nq)) return -1;
    const size_t nkeys = (size_t)nq * nsplit * 2 * ORB_L;
    if (nkeys > o->cap_keys) {
        if (o->key || o->id) (void)hipDeviceSynchronize();  // (as orbit_ensure_queries)
        dfree(o->key);
        dfree(o->id);
        o->key = nullptr;
        o->id = nullptr;
        o->cap_keys = 0;
        TILER_HIP_CHECK(dmalloc((void **)&o->key, nkeys * sizeof(float)));
        TILER_HIP_CHECK(dmalloc((void **)&o->id, nkeys * sizeof(int)));
        o->cap_keys = nkeys;
    }
    if (!queries_prepared) {  // (the FrameTiling path prepares them inside its descriptor kernel, orbit_ft_queries)
        OrbitPrepArgs pa{d_q, nullptr, nq, (const OrbitMap *)o->d_map, ix->scale, (half8 *)o->qfrag,
                         nullptr, nullptr, nullptr, nullptr, o->qstat};
        KTimer tm("nn_prep", stream);
        hipLaunchKernelGGL(orbit_prep_kernel, dim3((unsigned)std::min<long>(4096, (nqblk + ORB_PW - 1) / ORB_PW)),
                           dim3(64 * ORB_PW), 0, stream, pa);
        TILER_HIP_CHECK(hipGetLastError());
    }
    {
        const size_t lds = 2 * ((size_t)ORB_CB * OS * 1024 + ORB_CB * 128);
        // one timer per launch (the query-half split makes two per search: their per-dispatch times match a trace's)
        KTimer tm(split_q > 0 ? nullptr : "nn_orbit", stream);
#define ORB_PIPE(MD)                                                                                              \
    hipLaunchKernelGGL((nn_orbit_shortlist_pipe_kernel<ORB_L, ORB_CB, ORB_NW, ORB_QB, MD>), dim3(wgs, nsplit),              \
                       dim3(ORB_NW * 64), lds, stream, (const half8 *)o->d_frag, o->d_seed, o->gblk,                   \
                       (const half8 *)o->qfrag, nq, bps, nsplit, o->key, o->id, o->red_end, o->d_bmask,                \
                       0x7fffffff, o->d_bmask0, MD == 0 ? flat_cnt : nullptr, 0)
        if (!mix_full && split_q == 0) ORB_PIPE(0);
        if (split_q > 0) {  // two launches over query halves; the end of the first one is the tails' start
            const int qb_off = split_q / 32;
            const size_t per_q = (size_t)nsplit * 2 * ORB_L;
            {
                KTimer ta("nn_orbit", stream);
                hipLaunchKernelGGL((nn_orbit_shortlist_pipe_kernel<ORB_L, ORB_CB, ORB_NW, ORB_QB, 0>),
                                   dim3(split_q / qpw_q, nsplit), dim3(ORB_NW * 64), lds, stream,
                                   (const half8 *)o->d_frag, o->d_seed, o->gblk, (const half8 *)o->qfrag, split_q, bps,
                                   nsplit, o->key, o->id, o->red_end, o->d_bmask, 0x7fffffff, o->d_bmask0, flat_cnt, 0);
            }
            TILER_HIP_CHECK(hipEventRecord(o->ev_half, stream));
            KTimer tb("nn_orbit", stream);
            hipLaunchKernelGGL((nn_orbit_shortlist_pipe_kernel<ORB_L, ORB_CB, ORB_NW, ORB_QB, 0>),
                               dim3(wgs - split_q / qpw_q, nsplit), dim3(ORB_NW * 64), lds, stream,
                               (const half8 *)o->d_frag, o->d_seed, o->gblk,
                               (const half8 *)o->qfrag + (size_t)qb_off * OS * 64, nq - split_q, bps, nsplit,
                               o->key + (size_t)split_q * per_q, o->id + (size_t)split_q * per_q, o->red_end,
                               o->d_bmask, 0x7fffffff, o->d_bmask0, flat_cnt, split_q);
        }
        if (mix_full) {
            const int qb_off = mix_full * ORB_NW * ORB_QB, q_off = qb_off * 32;  // query blocks / queries of part A
            const size_t per_q = (size_t)nsplit * 2 * ORB_L;
            const size_t na = (size_t)std::min(nq, q_off) * per_q;
            TILER_HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)o->key, 0x7f800000u, na, stream));  // +inf: empty
            TILER_HIP_CHECK(hipMemsetAsync(o->id, 0xff, na * sizeof(int), stream));
            hipLaunchKernelGGL((nn_orbit_shortlist_pipe_kernel<ORB_L, ORB_CB, ORB_NW, ORB_QB, 0>), dim3(mix_full, 1),
                               dim3(ORB_NW * 64), lds, stream, (const half8 *)o->d_frag, o->d_seed, o->gblk,
                               (const half8 *)o->qfrag, nq, o->gblk, nsplit, o->key, o->id, o->red_end, o->d_bmask,
                               0x7fffffff, o->d_bmask0, nullptr, 0);
            if (nq > q_off)
                hipLaunchKernelGGL((nn_orbit_shortlist_pipe_kernel<ORB_L, ORB_CB, ORB_NW, ORB_QB, 0>),
                                   dim3(wgs - mix_full, nsplit), dim3(ORB_NW * 64), lds, stream,
                                   (const half8 *)o->d_frag, o->d_seed, o->gblk,
                                   (const half8 *)o->qfrag + (size_t)qb_off * OS * 64, nq - q_off, bps, nsplit,
                                   o->key + (size_t)q_off * per_q, o->id + (size_t)q_off * per_q, o->red_end,
                                   o->d_bmask, 0x7fffffff, o->d_bmask0, nullptr, 0);
        }
#undef ORB_PIPE
    }
    TILER_HIP_CHECK(hipGetLastError());
    OrbitRescoreArgs ra;
    ra.rows = ix->d_rows;
    ra.q = d_q;
    ra.rowh = (const _Float16 *)o->d_rowh;
    ra.qfrag = (const half8 *)o->qfrag;
    ra.nc = o->d_nc;
    ra.member = o->d_member;
    ra.dup = o->d_dup;
    ra.rep = o->d_rep;
    ra.gorder = tail.ko ? o->d_gorder : nullptr;
    ra.grp_of = tail.ko ? o->d_grp_of : nullptr;
    ra.ostat = o->qstat;
    ra.key = o->key;
    ra.id = o->id;
    ra.G = o->G;
    ra.nq = nq;
    ra.q0 = 0;
    ra.L = ORB_L;
    ra.nsplit = nsplit;
    ra.p1 = 2;
    ra.pair_cnt = o->pair_cnt;
    ra.pair_cand = o->pair_cand;
    ra.scale2 = (double)ix->scale * (double)ix->scale;
    ra.N = o->N;
    ra.Np = o->Np;
    ra.Hp = o->Hp;
    ra.Ecp = o->Ecp;
    ra.t = tail;
    static const bool want_stats = [] {
        const char *e = getenv("TILER_ORBIT_STATS");
        return e && e[0] == '1';
    }();
    if (want_stats) {
        if (!o->d_stats) TILER_HIP_CHECK(dmalloc((void **)&o->d_stats, 2 * sizeof(int)));
        TILER_HIP_CHECK(hipMemsetAsync(o->d_stats, 0, 2 * sizeof(int), stream));
        ra.t.n_expand = o->d_stats;
    }
    // the rescore and pair pass of queries [q0, q1) on stream s
    auto tails = [&](int q0, int q1, hipStream_t s) -> int {
        OrbitRescoreArgs r = ra;
        r.q0 = q0;
        r.nq = q1;
        {
            KTimer tm("nn_rescore", s);
            hipLaunchKernelGGL(nn_orbit_rescore_kernel, dim3((unsigned)((q1 - q0 + 7) / 8)), dim3(256), 0, s, r);
        }
        TILER_HIP_CHECK(hipGetLastError());
        {
            static_assert(256 % ORB_PSLOTS == 0, "pair groups must not straddle blocks");
            KTimer tm("nn_pairs", s);
            const long lanes = (long)(q1 - q0) * ORB_PSLOTS;
            hipLaunchKernelGGL(nn_orbit_pairs_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, s, r);
        }
        TILER_HIP_CHECK(hipGetLastError());
        return 0;
    };
    if (split_q > 0) {
        TILER_HIP_CHECK(hipStreamWaitEvent(o->tail_stream, o->ev_half, 0));
        if (tails(0, split_q, o->tail_stream)) return -1;
        TILER_HIP_CHECK(hipEventRecord(o->ev_tail, o->tail_stream));
        if (tails(split_q, nq, stream)) return -1;
        TILER_HIP_CHECK(hipStreamWaitEvent(stream, o->ev_tail, 0));  // tier 2 / 3 and the caller after both halves
    } else if (tails(0, nq, stream)) {
        return -1;
    }
    if (want_stats) {
        int h[2];
        TILER_HIP_CHECK(hipMemcpyAsync(h, o->d_stats, sizeof(h), hipMemcpyDeviceToHost, stream));
        TILER_HIP_CHECK(hipStreamSynchronize(stream));
        o->last_expansions = h[0];
        o->last_rescored = h[1];
    }
    ix->last_splits = nsplit;
    ix->last_flat_dev = flat_cnt;  // flat_queries: derived from the device count when the stats are read
    ix->last_flat_nq = nq;
    ix->last_flat_qpw = qpw_q;
    ix->last_flat_wgs = wgs;
    return 0;
}

void orbit_counters(const NNIndex *ix, long long *expansions, long long *rescored) {
    const OrbitIndex *o = ix->orbit;
    *expansions = o ? o->last_expansions : 0;
    *rescored = o ? o->last_rescored : 0;
}

}  // namespace tiler
