// merge_tie_repro.hip -- standalone reproducer of the round-4/5 small-batch merge's k = 8 tie corruption
// (VERDICT r05 "what's weak" #2).  Not part of libANN.so.
//
// The kernel below is the per-lane K-list merge that nn_scan_merge_kernel<8, false> ran until round 5: each lane
// owns the splits lane, lane + 64, ... of one query's partials (each split's list sorted by (distance, ANN order)),
// and folds them into a running K-best list in registers with a shifting insertion whose comparator is kd_less --
// distance first, then on an exact tie the kd-tree visit order, a noinline walk (kdorder_dev.hpp).  The same source
// is run on the host (plain C++, same comparator) and the two lists are compared lane by lane.
//
// Inputs: 64 lanes x NS splits x K entries; distances drawn from a few values so that exact ties between entries of
// different splits of one lane are frequent; the tie order is a real KdOrder view (implicit tree over n points, bs 1)
// with random cut dimensions / values and a random query, as kd_before_tree reads it.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I tiler_amd/csrc tools/merge_tie_repro.hip \
//         -o tools/_build/merge_tie_repro [-DINLINE_WALK] [-DNO_CALL]
//   ./merge_tie_repro              -> "lanes differing: X of 64 (entries lost ..., duplicated ...)"
//
// -DINLINE_WALK: the walk force-inlined instead of noinline; -DNO_CALL: ties by index (no KdOrder, no call);
// -DFIXED: the two-phase insertion that replaced the loop (kdorder_dev.hpp kd_list_insert).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <vector>

#include "kdtree.hpp"

#pragma clang fp contract(off)

using tiler::KdOrder;

#define HC(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                              \
        }                                                                         \
    } while (0)

// ---- the tie order: kd_before_tree as kdorder_dev.hpp has it, host and device from one body ----
#if defined(INLINE_WALK)
#define WALK_ATTR __attribute__((always_inline))
#else
#define WALK_ATTR __attribute__((noinline))
#endif
static __host__ __device__ WALK_ATTR bool before_tree(const KdOrder *__restrict__ op, const float *__restrict__ q, int a,
                                                       int b) {
    const KdOrder &o = *op;
    if ((unsigned)a >= (unsigned)o.n || (unsigned)b >= (unsigned)o.n) return (unsigned)a < (unsigned)b;
    int pa = o.pos[a], pb = o.pos[b];
    const bool sw = pa > pb;
    if (sw) {
        const int t = pa;
        pa = pb;
        pb = t;
    }
    int s = 0, e = o.n;
    while (e - s > o.bs) {
        const int m = s + ((e - s) >> 1);
        if (pb < m) {
            e = m;
        } else if (pa >= m) {
            s = m;
        } else {
            const float cut_diff = q[o.cd[m]] - o.cv[m];
            return (cut_diff < 0.0f) != sw;
        }
    }
    return !sw;
}
static __host__ __device__ __forceinline__ bool before(const KdOrder *op, const float *__restrict__ q, int a, int b) {
#if defined(NO_CALL)
    return (unsigned)a < (unsigned)b;
#else
    return op ? before_tree(op, q, a, b) : (unsigned)a < (unsigned)b;
#endif
}
static __host__ __device__ __forceinline__ bool less_(const KdOrder *op, const float *__restrict__ q, float da, int a,
                                                      float db, int b) {
    return da < db || (da == db && before(op, q, a, b));
}

// ---- the round-4 merge body: one lane's running K-best over its splits (nn_search.hip, r04/r05 non-WIDE) ----
template <int K>
static __host__ __device__ __forceinline__ void lane_merge(const KdOrder *op, const float *q, int lane, int nsplit,
                                                           const float *pd, const int *pi, float (&bd)[K],
                                                           int (&bi)[K]) {
    for (int r = 0; r < K; r++) {
        bd[r] = INFINITY;
        bi[r] = 0x7fffffff;
    }
    for (int sp = lane; sp < nsplit; sp += 64)
        for (int r = 0; r < K; r++) {
            const float v = pd[(long)sp * K + r];
            const int vi = pi[(long)sp * K + r];
            if (vi == 0x7fffffff || !less_(op, q, v, vi, bd[K - 1], bi[K - 1])) break;  // the split's list is sorted
#if defined(FIXED)
            // kd_list_insert's two phases (kdorder_dev.hpp): the position first, then straight-line selects
            bool f[K];
            for (int i = 0; i < K - 1; i++) f[i] = less_(op, q, v, vi, bd[i], bi[i]);
            int p = K - 1;
            for (int i = K - 2; i >= 0; i--)
                if (f[i] && p == i + 1) p = i;
            for (int i = K - 1; i > 0; i--) {
                const bool sh = i > p;
                bd[i] = sh ? bd[i - 1] : (i == p ? v : bd[i]);
                bi[i] = sh ? bi[i - 1] : (i == p ? vi : bi[i]);
            }
            bd[0] = p == 0 ? v : bd[0];
            bi[0] = p == 0 ? vi : bi[0];
#else
            int p = K - 1;
            while (p > 0 && less_(op, q, v, vi, bd[p - 1], bi[p - 1])) {
                bd[p] = bd[p - 1];
                bi[p] = bi[p - 1];
                p--;
            }
            bd[p] = v;
            bi[p] = vi;
#endif
        }
}

template <int K>
__global__ __launch_bounds__(64) void merge_kernel(const KdOrder *op, const float *q, int nsplit, const float *pd,
                                                   const int *pi, float *od, int *oi) {
    const int lane = threadIdx.x;
    float bd[K];
    int bi[K];
    lane_merge<K>(op, q, lane, nsplit, pd, pi, bd, bi);
    for (int r = 0; r < K; r++) {
        od[lane * K + r] = bd[r];
        oi[lane * K + r] = bi[r];
    }
}

int main(int argc, char **argv) {
    constexpr int K = 8;
    const int nsplit = argc > 1 ? atoi(argv[1]) : 1024;  // 16 splits per lane, as at C3
    const int n = 1 << 16, dd = 192, nvals = argc > 2 ? atoi(argv[2]) : 6;
    const unsigned seed = argc > 3 ? (unsigned)atoi(argv[3]) : 1u;
    std::mt19937 rng(seed);
    // a KdOrder view over n points (bs 1): random leaf positions, cut dimensions and values, a random query
    std::vector<int> pos(n), pidx(n), cd(n);
    std::vector<float> cv(n), qv(dd);
    for (int i = 0; i < n; i++) pidx[i] = i;
    std::shuffle(pidx.begin(), pidx.end(), rng);
    for (int i = 0; i < n; i++) pos[pidx[i]] = i;
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    for (int i = 0; i < n; i++) {
        cd[i] = (int)(rng() % dd);
        cv[i] = U(rng);
    }
    for (auto &x : qv) x = U(rng);
    KdOrder h;
    h.n = n;
    h.bs = 1;
    h.dd = dd;
    h.pos = pos.data();
    h.pidx = pidx.data();
    h.cd = cd.data();
    h.cv = cv.data();
    // partials: each split's K entries, distinct point ids, distances from nvals values, sorted by (dist, order)
    std::vector<float> pd((size_t)nsplit * K);
    std::vector<int> pi((size_t)nsplit * K);
    std::vector<int> ids(n);
    for (int i = 0; i < n; i++) ids[i] = i;
    std::shuffle(ids.begin(), ids.end(), rng);
    int next = 0;
    for (int sp = 0; sp < nsplit; sp++) {
        std::vector<std::pair<float, int>> e(K);
        for (int r = 0; r < K; r++) e[r] = {(float)(rng() % nvals), ids[next++ % n]};
        std::sort(e.begin(), e.end(), [&](const std::pair<float, int> &x, const std::pair<float, int> &y) {
            return less_(&h, qv.data(), x.first, x.second, y.first, y.second);
        });
        for (int r = 0; r < K; r++) {
            pd[(size_t)sp * K + r] = e[r].first;
            pi[(size_t)sp * K + r] = e[r].second;
        }
    }
    // host reference
    std::vector<float> hd(64 * K);
    std::vector<int> hi(64 * K);
    for (int lane = 0; lane < 64; lane++) {
        float bd[K];
        int bi[K];
        lane_merge<K>(&h, qv.data(), lane, nsplit, pd.data(), pi.data(), bd, bi);
        for (int r = 0; r < K; r++) {
            hd[lane * K + r] = bd[r];
            hi[lane * K + r] = bi[r];
        }
    }
    // device
    int *d_pos, *d_pidx, *d_cd, *d_pi, *d_oi;
    float *d_cv, *d_q, *d_pd, *d_od;
    KdOrder *d_view;
    HC(hipMalloc(&d_pos, n * 4));
    HC(hipMalloc(&d_pidx, n * 4));
    HC(hipMalloc(&d_cd, n * 4));
    HC(hipMalloc(&d_cv, n * 4));
    HC(hipMalloc(&d_q, dd * 4));
    HC(hipMalloc(&d_pd, pd.size() * 4));
    HC(hipMalloc(&d_pi, pi.size() * 4));
    HC(hipMalloc(&d_od, 64 * K * 4));
    HC(hipMalloc(&d_oi, 64 * K * 4));
    HC(hipMalloc(&d_view, sizeof(KdOrder)));
    HC(hipMemcpy(d_pos, pos.data(), n * 4, hipMemcpyHostToDevice));
    HC(hipMemcpy(d_pidx, pidx.data(), n * 4, hipMemcpyHostToDevice));
    HC(hipMemcpy(d_cd, cd.data(), n * 4, hipMemcpyHostToDevice));
    HC(hipMemcpy(d_cv, cv.data(), n * 4, hipMemcpyHostToDevice));
    HC(hipMemcpy(d_q, qv.data(), dd * 4, hipMemcpyHostToDevice));
    HC(hipMemcpy(d_pd, pd.data(), pd.size() * 4, hipMemcpyHostToDevice));
    HC(hipMemcpy(d_pi, pi.data(), pi.size() * 4, hipMemcpyHostToDevice));
    KdOrder dv = h;
    dv.pos = d_pos;
    dv.pidx = d_pidx;
    dv.cd = d_cd;
    dv.cv = d_cv;
    HC(hipMemcpy(d_view, &dv, sizeof(KdOrder), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(merge_kernel<K>, dim3(1), dim3(64), 0, 0, d_view, d_q, nsplit, d_pd, d_pi, d_od, d_oi);
    HC(hipGetLastError());
    HC(hipDeviceSynchronize());
    std::vector<float> gd(64 * K);
    std::vector<int> gi(64 * K);
    HC(hipMemcpy(gd.data(), d_od, gd.size() * 4, hipMemcpyDeviceToHost));
    HC(hipMemcpy(gi.data(), d_oi, gi.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0, lost = 0, dup = 0, shown = 0;
    for (int lane = 0; lane < 64; lane++) {
        bool diff = false;
        for (int r = 0; r < K; r++)
            if (gi[lane * K + r] != hi[lane * K + r] || gd[lane * K + r] != hd[lane * K + r]) diff = true;
        if (!diff) continue;
        bad++;
        std::multiset<int> hs(hi.begin() + lane * K, hi.begin() + lane * K + K),
            gs(gi.begin() + lane * K, gi.begin() + lane * K + K);
        for (int x : std::set<int>(hs.begin(), hs.end())) lost += (int)hs.count(x) > (int)gs.count(x);
        for (int x : std::set<int>(gs.begin(), gs.end())) dup += gs.count(x) > 1;
        if (shown++ < 3) {
            printf("lane %d\n  host:", lane);
            for (int r = 0; r < K; r++) printf(" (%g,%d)", hd[lane * K + r], hi[lane * K + r]);
            printf("\n  gpu: ");
            for (int r = 0; r < K; r++) printf(" (%g,%d)", gd[lane * K + r], gi[lane * K + r]);
            printf("\n");
        }
    }
    printf("nsplit %d nvals %d seed %u: lanes differing: %d of 64 (host entries missing on the GPU: %d, GPU ids listed "
           "twice: %d)\n",
           nsplit, nvals, seed, bad, lost, dup);
    return bad ? 1 : 0;
}
