// kdtree.hip -- ANN 1.1.2 kd-tree (ANN_KD_STD) build over an HBM dataset + the pruning check / exact replay
// that make the MFMA search return ANN's own answer among equal distances (kdtree.hpp).
//
// Build, level by level (every node of a level at once):
//   kd_spread_kernel   one wave per chunk of <= KD_CH points of a node: per-dimension min / max (annSpread)
//   kd_select_kernel   one wave per node: reduce the chunks, spread = max - min (fp32), cut_dim = first maximum
//                      (annMaxSpread), gather the node's cut-dimension keys in pidx order
//   (host)             annMedianSplit's quickselect on each node's (key, index) pairs, bit for bit: the
//                      permutation it leaves decides which of several equal keys go LO, and so the rest of the
//                      tree; nodes of a level run on a host thread pool (the level's work is O(n))
// The rows never leave HBM: per level only the n keys (4 B each) come to the host and the new order goes back.
#include <float.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "kdorder_dev.hpp"
#include "kdtree.hpp"

namespace tiler {

static constexpr int KD_CH = 2048;  // points per spread chunk

struct KdChunk {
    int node, s, e;
};

// per-dimension min / max of pidx[s..e) (annSpread's loop: first value, then < min / > max)
__global__ __launch_bounds__(256) void kd_spread_kernel(const float *__restrict__ rows, int dd,
                                                        const int *__restrict__ pidx, const KdChunk *__restrict__ ch,
                                                        int nch, float *__restrict__ pmin, float *__restrict__ pmax) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nch) return;
    const KdChunk k = ch[c];
    for (int d0 = 0; d0 < dd; d0 += 256) {
        float mn[4], mx[4];
        {
            const float *r = rows + (long)pidx[k.s] * dd;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int d = d0 + j * 64 + lane;
                mn[j] = mx[j] = d < dd ? r[d] : 0.0f;
            }
        }
        for (int i = k.s + 1; i < k.e; i++) {
            const float *r = rows + (long)pidx[i] * dd;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int d = d0 + j * 64 + lane;
                const float v = d < dd ? r[d] : 0.0f;
                if (v < mn[j])
                    mn[j] = v;
                else if (v > mx[j])
                    mx[j] = v;
            }
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int d = d0 + j * 64 + lane;
            if (d < dd) {
                pmin[(long)c * dd + d] = mn[j];
                pmax[(long)c * dd + d] = mx[j];
            }
        }
    }
}

struct KdNodeDev {
    int s, e, c0, c1;  // positions [s, e), chunks [c0, c1)
};

// one wave per node: cut_dim = first dimension of maximum spread; keys[i] = rows[pidx[i]][cut_dim] for i in [s, e)
__global__ __launch_bounds__(256) void kd_select_kernel(const float *__restrict__ rows, int dd,
                                                        const int *__restrict__ pidx,
                                                        const KdNodeDev *__restrict__ nodes, int nn,
                                                        const float *__restrict__ pmin, const float *__restrict__ pmax,
                                                        int *__restrict__ cut_dim, float *__restrict__ keys,
                                                        float *__restrict__ box) {
    const int lane = threadIdx.x & 63;
    const int nd = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (nd >= nn) return;
    const KdNodeDev N = nodes[nd];
    float best = -INFINITY;
    int bd = 0x7fffffff;
    for (int d = lane; d < dd; d += 64) {
        float mn = pmin[(long)N.c0 * dd + d], mx = pmax[(long)N.c0 * dd + d];
        for (int c = N.c0 + 1; c < N.c1; c++) {
            mn = fminf(mn, pmin[(long)c * dd + d]);
            mx = fmaxf(mx, pmax[(long)c * dd + d]);
        }
        if (box) {  // the root node: annEnclRect
            box[d] = mn;
            box[dd + d] = mx;
        }
        const float spr = mx - mn;
        if (spr > best) {  // lane-local dims ascend: the first maximum
            best = spr;
            bd = d;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int od = __shfl_xor(bd, o, 64);
        if (ob > best || (ob == best && od < bd)) {
            best = ob;
            bd = od;
        }
    }
    // annMaxSpread: max_spr starts at 0 with max_dim 0, so an all-zero spread picks dimension 0
    const int cd = (best > 0.0f) ? bd : 0;
    if (lane == 0) cut_dim[nd] = cd;
    for (int i = N.s + lane; i < N.e; i += 64) keys[i] = rows[(long)pidx[i] * dd + cd];
}

// annMedianSplit (kd_util.cpp) on one node's (key, index) pairs, key[i] = PA(i, cut_dim): the same pivot choice,
// partition scans and swaps, then the largest low-side key moved to n_lo - 1; returns cut_val.
static float median_split_host(float *key, int *idx, int n, int n_lo) {
    auto sw = [&](int a, int b) {
        std::swap(key[a], key[b]);
        std::swap(idx[a], idx[b]);
    };
    int l = 0, r = n - 1;
    while (l < r) {
        int i = (r + l) / 2, k;
        if (key[i] > key[r]) sw(i, r);
        sw(l, i);
        const float c = key[l];
        i = l;
        k = r;
        for (;;) {
            while (key[++i] < c) {
            }
            while (key[--k] > c) {
            }
            if (i < k)
                sw(i, k);
            else
                break;
        }
        sw(l, k);
        if (k > n_lo)
            r = k - 1;
        else if (k < n_lo)
            l = k + 1;
        else
            break;
    }
    if (n_lo > 0) {
        float c = key[0];
        int k = 0;
        for (int i = 1; i < n_lo; i++)
            if (key[i] > c) {
                c = key[i];
                k = i;
            }
        sw(n_lo - 1, k);
    }
    return (float)(((double)(key[n_lo - 1] + key[n_lo])) / 2.0);
}

KdOrder KdTree::view() const {
    KdOrder o;
    o.pos = d_pos;
    o.pidx = d_pidx;
    o.cd = d_cd;
    o.cv = d_cv;
    o.lo = d_lo;
    o.hi = d_hi;
    o.box_lo = d_box;
    o.box_hi = d_box ? d_box + dd : nullptr;
    o.n = n;
    o.bs = bs;
    o.dd = dd;
    return o;
}

void kd_tree_destroy(KdTree *t) {
    if (!t) return;
    hipFree(t->d_pos);
    hipFree(t->d_pidx);
    hipFree(t->d_cd);
    hipFree(t->d_cv);
    hipFree(t->d_lo);
    hipFree(t->d_hi);
    hipFree(t->d_box);
    delete t;
}

// run f(i) for i in [0, count) on up to `threads` host threads (biggest items first: callers sort)
template <class F>
static void parallel_for(int count, int threads, F f) {
    if (count <= 1 || threads <= 1) {
        for (int i = 0; i < count; i++) f(i);
        return;
    }
    std::atomic<int> next(0);
    auto work = [&]() {
        for (int i = next.fetch_add(1); i < count; i = next.fetch_add(1)) f(i);
    };
    const int nt = std::min(threads, count);
    std::vector<std::thread> pool;
    pool.reserve(nt - 1);
    for (int t = 1; t < nt; t++) pool.emplace_back(work);
    work();
    for (auto &th : pool) th.join();
}

static int host_threads() {
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(16u, hc ? hc : 1u));
}

KdTree *kd_tree_build(const float *d_rows, int n, int dd, int bs, hipStream_t stream) {
    const auto t0 = std::chrono::steady_clock::now();
    KdTree *t = new KdTree();
    t->n = n;
    t->dd = dd;
    t->bs = std::max(1, bs);
    struct Guard {  // frees the build scratch on every exit path
        std::vector<void *> dev, host;
        ~Guard() {
            for (void *p : dev) (void)hipFree(p);
            for (void *p : host) (void)hipHostFree(p);
        }
    } g;
    auto fail = [&]() -> KdTree * {
        kd_tree_destroy(t);
        return nullptr;
    };
#define KD_CHECK(expr)                                                                     \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess) {                                                            \
            set_error(std::string("kd-tree build: ") + #expr + ": " + hipGetErrorString(_e)); \
            return fail();                                                                 \
        }                                                                                  \
    } while (0)
    const size_t nn1 = (size_t)std::max(n, 1);
    KD_CHECK(hipMalloc((void **)&t->d_pos, nn1 * 4));
    KD_CHECK(hipMalloc((void **)&t->d_pidx, nn1 * 4));
    KD_CHECK(hipMalloc((void **)&t->d_cd, nn1 * 4));
    KD_CHECK(hipMalloc((void **)&t->d_cv, nn1 * 4));
    KD_CHECK(hipMalloc((void **)&t->d_lo, nn1 * 4));
    KD_CHECK(hipMalloc((void **)&t->d_hi, nn1 * 4));
    KD_CHECK(hipMalloc((void **)&t->d_box, (size_t)2 * std::max(dd, 1) * 4));
    std::vector<int> cdv(nn1, 0);
    std::vector<float> cvv(nn1, 0.0f);
    std::vector<float> box(2 * (size_t)std::max(dd, 1), 0.0f);
    int *h_pidx = nullptr;
    float *h_keys = nullptr;
    KD_CHECK(hipHostMalloc((void **)&h_pidx, nn1 * 4, hipHostMallocDefault));
    g.host.push_back(h_pidx);
    KD_CHECK(hipHostMalloc((void **)&h_keys, nn1 * 4, hipHostMallocDefault));
    g.host.push_back(h_keys);
    for (int i = 0; i < n; i++) h_pidx[i] = i;  // SkeletonTree: pidx[i] = i
    if (n > t->bs) {
        float *d_keys = nullptr, *d_pmin = nullptr, *d_pmax = nullptr;
        int *d_cut = nullptr;
        KdChunk *d_ch = nullptr;
        KdNodeDev *d_nodes = nullptr;
        const size_t max_nodes = (size_t)n / 2 + 1;
        const size_t max_ch = (size_t)n / KD_CH + max_nodes + 1;
        KD_CHECK(hipMalloc((void **)&d_keys, nn1 * 4));
        g.dev.push_back(d_keys);
        KD_CHECK(hipMalloc((void **)&d_pmin, max_ch * dd * 4));
        g.dev.push_back(d_pmin);
        KD_CHECK(hipMalloc((void **)&d_pmax, max_ch * dd * 4));
        g.dev.push_back(d_pmax);
        KD_CHECK(hipMalloc((void **)&d_cut, max_nodes * 4));
        g.dev.push_back(d_cut);
        KD_CHECK(hipMalloc((void **)&d_ch, max_ch * sizeof(KdChunk)));
        g.dev.push_back(d_ch);
        KD_CHECK(hipMalloc((void **)&d_nodes, max_nodes * sizeof(KdNodeDev)));
        g.dev.push_back(d_nodes);
        KdChunk *h_ch = nullptr;
        KdNodeDev *h_nodes = nullptr;
        int *h_cut = nullptr;
        KD_CHECK(hipHostMalloc((void **)&h_ch, max_ch * sizeof(KdChunk), hipHostMallocDefault));
        g.host.push_back(h_ch);
        KD_CHECK(hipHostMalloc((void **)&h_nodes, max_nodes * sizeof(KdNodeDev), hipHostMallocDefault));
        g.host.push_back(h_nodes);
        KD_CHECK(hipHostMalloc((void **)&h_cut, max_nodes * 4, hipHostMallocDefault));
        g.host.push_back(h_cut);
        KD_CHECK(hipMemcpyAsync(t->d_pidx, h_pidx, (size_t)n * 4, hipMemcpyHostToDevice, stream));
        std::vector<std::pair<int, int>> level{{0, n}}, next;
        const int threads = host_threads();
        while (!level.empty()) {
            const int nn = (int)level.size();
            int nch = 0;
            for (int i = 0; i < nn; i++) {
                const int s = level[i].first, e = level[i].second;
                h_nodes[i].s = s;
                h_nodes[i].e = e;
                h_nodes[i].c0 = nch;
                for (int c = s; c < e; c += KD_CH) h_ch[nch++] = KdChunk{i, c, std::min(e, c + KD_CH)};
                h_nodes[i].c1 = nch;
            }
            KD_CHECK(hipMemcpyAsync(d_ch, h_ch, (size_t)nch * sizeof(KdChunk), hipMemcpyHostToDevice, stream));
            KD_CHECK(hipMemcpyAsync(d_nodes, h_nodes, (size_t)nn * sizeof(KdNodeDev), hipMemcpyHostToDevice, stream));
            hipLaunchKernelGGL(kd_spread_kernel, dim3((nch + 3) / 4), dim3(256), 0, stream, d_rows, dd,
                               (const int *)t->d_pidx, (const KdChunk *)d_ch, nch, d_pmin, d_pmax);
            KD_CHECK(hipGetLastError());
            hipLaunchKernelGGL(kd_select_kernel, dim3((nn + 3) / 4), dim3(256), 0, stream, d_rows, dd,
                               (const int *)t->d_pidx, (const KdNodeDev *)d_nodes, nn, (const float *)d_pmin,
                               (const float *)d_pmax, d_cut, d_keys, t->levels == 0 ? t->d_box : nullptr);
            KD_CHECK(hipGetLastError());
            KD_CHECK(hipMemcpyAsync(h_cut, d_cut, (size_t)nn * 4, hipMemcpyDeviceToHost, stream));
            KD_CHECK(hipMemcpyAsync(h_keys, d_keys, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
            KD_CHECK(hipStreamSynchronize(stream));
            // annMedianSplit per node (biggest first), recording the split node m's cut
            parallel_for(nn, threads, [&](int i) {
                const int s = level[i].first, e = level[i].second, cnt = e - s, n_lo = cnt / 2;
                const float cv = median_split_host(h_keys + s, h_pidx + s, cnt, n_lo);
                cdv[s + n_lo] = h_cut[i];
                cvv[s + n_lo] = cv;
            });
            next.clear();
            for (int i = 0; i < nn; i++) {
                const int s = level[i].first, e = level[i].second, m = s + (e - s) / 2;
                if (m - s > t->bs) next.emplace_back(s, m);
                if (e - m > t->bs) next.emplace_back(m, e);
            }
            std::stable_sort(next.begin(), next.end(), [](const std::pair<int, int> &a, const std::pair<int, int> &b) {
                return a.second - a.first > b.second - b.first;
            });
            KD_CHECK(hipMemcpyAsync(t->d_pidx, h_pidx, (size_t)n * 4, hipMemcpyHostToDevice, stream));
            level.swap(next);
            t->levels++;
        }
        KD_CHECK(hipMemcpyAsync(box.data(), t->d_box, (size_t)2 * dd * 4, hipMemcpyDeviceToHost, stream));
        KD_CHECK(hipStreamSynchronize(stream));
    } else {
        KD_CHECK(hipMemcpyAsync(t->d_pidx, h_pidx, nn1 * 4, hipMemcpyHostToDevice, stream));
    }
    // cell bounds along each node's cut dimension (rkd_tree: bnd_box.hi[cd] = cv for LO, .lo[cd] = cv for HI)
    std::vector<float> lov(nn1, 0.0f), hiv(nn1, 0.0f);
    if (n > t->bs) {
        std::vector<float> lo(box.begin(), box.begin() + dd), hi(box.begin() + dd, box.begin() + 2 * dd);
        struct Fr {
            int s, e, stage;
            float saved;
        };
        std::vector<Fr> st;
        st.push_back({0, n, 0, 0.0f});
        while (!st.empty()) {
            Fr &f = st.back();
            const int m = f.s + (f.e - f.s) / 2, cd = cdv[m];
            if (f.stage == 0) {  // enter: record cd_bnds, descend LO with hi[cd] = cv
                lov[m] = lo[cd];
                hiv[m] = hi[cd];
                f.saved = hi[cd];
                hi[cd] = cvv[m];
                f.stage = 1;
                if (m - f.s > t->bs) st.push_back({f.s, m, 0, 0.0f});
            } else if (f.stage == 1) {  // LO done: restore hi, descend HI with lo[cd] = cv
                hi[cd] = f.saved;
                f.saved = lo[cd];
                lo[cd] = cvv[m];
                f.stage = 2;
                const int s2 = m, e2 = f.e;
                if (e2 - s2 > t->bs) st.push_back({s2, e2, 0, 0.0f});
            } else {
                lo[cd] = f.saved;
                st.pop_back();
            }
        }
    }
    std::vector<int> pos(nn1, 0);
    for (int i = 0; i < n; i++) pos[h_pidx[i]] = i;
    KD_CHECK(hipMemcpyAsync(t->d_pos, pos.data(), nn1 * 4, hipMemcpyHostToDevice, stream));
    KD_CHECK(hipMemcpyAsync(t->d_cd, cdv.data(), nn1 * 4, hipMemcpyHostToDevice, stream));
    KD_CHECK(hipMemcpyAsync(t->d_cv, cvv.data(), nn1 * 4, hipMemcpyHostToDevice, stream));
    KD_CHECK(hipMemcpyAsync(t->d_lo, lov.data(), nn1 * 4, hipMemcpyHostToDevice, stream));
    KD_CHECK(hipMemcpyAsync(t->d_hi, hiv.data(), nn1 * 4, hipMemcpyHostToDevice, stream));
    KD_CHECK(hipStreamSynchronize(stream));
#undef KD_CHECK
    t->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return t;
}

int kd_tree_positions(const KdTree *t, int32_t *pos) {
    if (!t || t->n == 0) return 0;
    TILER_HIP_CHECK(hipMemcpy(pos, t->d_pos, (size_t)t->n * 4, hipMemcpyDeviceToHost));
    return 0;
}

// ------------------------------------------------------------------------------------------
// pruning check + exact replay
// ------------------------------------------------------------------------------------------
// One thread per query: ANN visits result c iff every far-child box distance on its path is below the k-th key
// current at that check.  That key is >= D_k (the final k-th distance) throughout, and > D_k while c is a tie at
// D_k not yet inserted, so box < D_k (or <= D_k for such a tie) vouches for c; otherwise -> replay.
__global__ __launch_bounds__(256) void kd_verify_kernel(KdOrder o, KdFixArgs a) {
    const long q = (long)blockIdx.x * 256 + threadIdx.x;
    if (q >= a.nq) return;
    const float *qr = a.q + q * o.dd;
    const float Dk = a.err[q * a.k + a.k - 1];
    const int i0 = a.idx[q * a.k];
    if (i0 < 0 || !(Dk < FLT_MAX)) return;  // empty dataset or fewer than k points: nothing to vouch for
    const float rb = kd_root_box(o, qr);
    bool ok = true;
    for (int j = 0; j < a.k && ok; j++) {
        const int c = a.idx[q * a.k + j];
        if ((unsigned)c >= (unsigned)o.n) {
            ok = false;
            break;
        }
        const float fb = kd_path_far_box(o, qr, o.pos[c], rb);
        const float dc = a.err[q * a.k + j];
        ok = fb < Dk || (fb <= Dk && dc == Dk);
    }
    if (!ok) a.list[atomicAdd(a.count, 1)] = (int)q;
}

// annkSearch replayed exactly (kd_search.cpp): depth-first, near child first, far child iff its box distance
// < the current k-th key (eps = 0), leaf scans with the early break, ANNmin_k insertion (equal keys keep the
// first found).  One thread per listed query; the explicit stack holds pending nodes and pending far checks.
template <int K>
__global__ __launch_bounds__(64) void kd_replay_kernel(KdOrder o, KdFixArgs a) {
    const int count = *a.count;
    for (int li = blockIdx.x * 64 + threadIdx.x; li < count; li += gridDim.x * 64) {
        const long q = a.list[li];
        const float *qr = a.q + q * o.dd;
        const int k = a.k;
        float mk[K + 1];
        int mi[K + 1];
        int cnt = 0;
        auto max_key = [&]() { return cnt == k ? mk[k - 1] : FLT_MAX; };
        // stack frames: kind 0 = visit node [s, e) with box b; kind 1 = far check of node [s, e)'s child
        struct Fr {
            int s, e, kind;
            float b;
        };
        Fr st[96];
        int sp = 0;
        st[sp++] = Fr{0, o.n, 0, kd_root_box(o, qr)};
        while (sp > 0) {
            const Fr f = st[--sp];
            if (f.kind == 0) {
                if (f.e - f.s <= o.bs) {  // ANNkd_leaf::ann_search
                    float min_dist = max_key();
                    for (int p = f.s; p < f.e; p++) {
                        const int pt = o.pidx[p];
                        const float *pp = a.rows + (long)pt * o.dd;
                        float dist = 0.0f;
                        int d;
                        for (d = 0; d < o.dd; d++) {
                            const float t = qr[d] - pp[d];
                            dist = dist + t * t;
                            if (dist > min_dist) break;
                        }
                        if (d >= o.dd) {  // ANNmin_k::insert
                            int i;
                            for (i = cnt; i > 0; i--) {
                                if (mk[i - 1] > dist) {
                                    mk[i] = mk[i - 1];
                                    mi[i] = mi[i - 1];
                                } else {
                                    break;
                                }
                            }
                            mk[i] = dist;
                            mi[i] = pt;
                            if (cnt < k) cnt++;
                            min_dist = max_key();
                        }
                    }
                    continue;
                }
                const int m = f.s + ((f.e - f.s) >> 1);
                const float cut_diff = qr[o.cd[m]] - o.cv[m];
                // near child now, far check after it returns (pushed first, popped after the near subtree)
                st[sp++] = Fr{f.s, f.e, 1, f.b};
                if (cut_diff < 0.0f)
                    st[sp++] = Fr{f.s, m, 0, f.b};
                else
                    st[sp++] = Fr{m, f.e, 0, f.b};
            } else {
                const int m = f.s + ((f.e - f.s) >> 1);
                const float qd = qr[o.cd[m]];
                const float cut_diff = qd - o.cv[m];
                const bool lo_first = cut_diff < 0.0f;
                float box_diff = lo_first ? o.lo[m] - qd : qd - o.hi[m];
                if (box_diff < 0.0f) box_diff = 0.0f;
                const float b = f.b + (cut_diff * cut_diff - box_diff * box_diff);
                if (b * 1.0f < max_key()) st[sp++] = lo_first ? Fr{m, f.e, 0, b} : Fr{f.s, m, 0, b};
            }
        }
        for (int j = 0; j < k; j++) {
            const bool ok = j < cnt;
            a.idx[q * k + j] = ok ? mi[j] : -1;
            a.err[q * k + j] = ok ? mk[j] : FLT_MAX;
        }
        if (a.m_tile) {
            const int best = cnt > 0 ? mi[0] : -1;
            a.m_tile[q] = best >= 0 ? a.tr_tile[best] : -1;
            a.m_pal[q] = best >= 0 ? a.tr_pal[best] : -1;
            const int at = best >= 0 ? a.tr_attr[best] : 0;
            a.m_hm[q] = (at & 1) != 0;
            a.m_vm[q] = (at & 2) != 0;
        }
    }
}

int kd_verify_and_replay(const KdTree *t, const KdFixArgs &a, hipStream_t stream) {
    if (!t || t->n <= t->bs || a.nq <= 0) return 0;  // a single bucket: no pruning, position order is exact
    if (a.k > 32) {
        set_error("kd replay: k > 32");
        return -1;
    }
    const KdOrder o = t->view();
    TILER_HIP_CHECK(hipMemsetAsync(a.count, 0, sizeof(int), stream));
    {
        KTimer tm("kd_verify", stream);
        hipLaunchKernelGGL(kd_verify_kernel, dim3((a.nq + 255) / 256), dim3(256), 0, stream, o, a);
    }
    TILER_HIP_CHECK(hipGetLastError());
    {
        KTimer tm("kd_replay", stream);
        const dim3 grid(64);  // grid-stride over the device-side count: no host round trip
        if (a.k <= 1)
            hipLaunchKernelGGL(kd_replay_kernel<1>, grid, dim3(64), 0, stream, o, a);
        else if (a.k <= 8)
            hipLaunchKernelGGL(kd_replay_kernel<8>, grid, dim3(64), 0, stream, o, a);
        else
            hipLaunchKernelGGL(kd_replay_kernel<32>, grid, dim3(64), 0, stream, o, a);
    }
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace tiler
