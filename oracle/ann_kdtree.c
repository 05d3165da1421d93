/*
 * ann_kdtree.c -- TEST / BASELINE INFRASTRUCTURE ONLY: the reference's CPU search for FrameTiling,
 * an ANN 1.1.2 kd-tree (ann_kdtree_create(pa, n, 192, bs = 1, ANN_KD_STD), main.pas:3961; searched with
 * ann_kdtree_search(..., eps = 0), main.pas:4027).  ANN's source is not in /root/reference (ANN.dll is a
 * Windows PE: SURVEY.md 8(a) a8, 8(c)); this restates the published ANN 1.1.2 algorithm with the
 * arithmetic recovered from the DLL:
 *   build  (kd_tree ctor, rkd_tree with kd_split = ANN_KD_STD): enclosing box of all points; at each node
 *          cut_dim = first dimension of maximum spread (max - min) over the node's points, n_lo = n / 2,
 *          quickselect so the n_lo smallest coordinates go low, cut_val = (max of low side + n_lo-th
 *          value) / 2; the node keeps the cell's bounds along cut_dim; buckets of 1 point (bs = 1).
 *   search (annkSearch, k results): box distance of q to the root box; at a split node visit the child on
 *          q's side first, then update box_dist += cut_diff^2 - box_diff^2 (fp32, ANNdist = float) and
 *          visit the far child iff box_dist * (1 + eps)^2 < the current k-th key; leaf distance = sequential
 *          fp32 sum of (q_d - p_d)^2, no FMA, break as soon as dist > the k-th key read at the leaf's start;
 *          a completed scan is inserted into ANNmin_k, which shifts only entries with a larger key (an
 *          equal distance stays behind the first found; at the k-th slot it is dropped).
 * The tie order among equal distances is therefore the tree's visit order.  libANN.so reproduces it
 * (tiler_amd/csrc/kdtree.hip); this restatement is the checker for that, pinned by the ANN 1.1.2
 * algorithm (no reference fixture exists: ANN.dll is a Windows PE).
 */
#include <float.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "tiler_oracle.h"

typedef struct {
    int cut_dim;   /* -1: leaf */
    float cut_val;
    float lo_bnd;  /* cell bounds along cut_dim */
    float hi_bnd;
    int child[2];  /* split: node ids; leaf: child[0] = first pidx position of the bucket, child[1] = its size */
} kd_node;

typedef struct {
    const float *data;
    int n, d, bs;
    kd_node *nodes;
    int nn;
    int *pidx;
    float *box_lo, *box_hi;
} kd_tree;

#define PA(i, dim) (t->data[(size_t)t->pidx[(i)] * t->d + (dim)])

static int kd_new(kd_tree *t) { return t->nn++; }

/* annMaxSpread (ANN.dll 0x1800158e0): enclosing rect, then the FIRST dimension whose spread exceeds the running
 * maximum, which starts at 0 (so all-zero spreads give dimension 0) */
static int max_spread(kd_tree *t, int *pidx, int n) {
    int best = 0;
    float best_sp = 0.0f;
    for (int dim = 0; dim < t->d; dim++) {
        float mn = t->data[(size_t)pidx[0] * t->d + dim], mx = mn;
        for (int i = 1; i < n; i++) {
            const float c = t->data[(size_t)pidx[i] * t->d + dim];
            if (c < mn) mn = c;
            if (c > mx) mx = c;
        }
        if (mx - mn > best_sp) {
            best_sp = mx - mn;
            best = dim;
        }
    }
    return best;
}

/* quickselect on pidx[0..n) by coordinate dim: afterwards the n_lo smallest sit in [0, n_lo) with
 * the largest of them at n_lo - 1, and [n_lo] holds the n_lo-th value; returns the midpoint cut. */
static float median_split(const float *data, int d, int *pidx, int n, int dim, int n_lo) {
#define C(i) (data[(size_t)pidx[(i)] * d + dim])
#define SWAP(a, b) do { int _t = pidx[(a)]; pidx[(a)] = pidx[(b)]; pidx[(b)] = _t; } while (0)
    int l = 0, r = n - 1;
    while (l < r) {
        int i = (r + l) / 2, k;
        if (C(i) > C(r)) SWAP(i, r);
        SWAP(l, i);
        const float c = C(l);
        i = l;
        k = r;
        for (;;) {
            while (C(++i) < c) {}
            while (C(--k) > c) {}
            if (i < k) SWAP(i, k);
            else break;
        }
        SWAP(l, k);
        if (k > n_lo) r = k - 1;
        else if (k < n_lo) l = k + 1;
        else break;
    }
    if (n_lo > 0) {
        float c = C(0);
        int k = 0;
        for (int i = 1; i < n_lo; i++)
            if (C(i) > c) {
                c = C(i);
                k = i;
            }
        SWAP(n_lo - 1, k);
    }
    return (C(n_lo - 1) + C(n_lo)) / 2.0f;
#undef C
#undef SWAP
}

/* rkd_tree (kd_tree.cpp): n <= bs -> a bucket leaf of pidx[0..n) (n = 0: KD_TRIVIAL, an empty leaf) */
static int kd_build(kd_tree *t, int *pidx, int n, float *lo, float *hi) {
    const int id = kd_new(t);
    kd_node *nd = &t->nodes[id];
    if (n <= t->bs) {
        nd->cut_dim = -1;
        nd->child[0] = (int)(pidx - t->pidx);
        nd->child[1] = n;
        return id;
    }
    const int cd = max_spread(t, pidx, n);
    const int n_lo = n / 2;
    const float cv = median_split(t->data, t->d, pidx, n, cd, n_lo);
    nd->cut_dim = cd;
    nd->cut_val = cv;
    nd->lo_bnd = lo[cd];
    nd->hi_bnd = hi[cd];
    const float save_hi = hi[cd];
    hi[cd] = cv;
    const int a = kd_build(t, pidx, n_lo, lo, hi);
    hi[cd] = save_hi;
    const float save_lo = lo[cd];
    lo[cd] = cv;
    const int b = kd_build(t, pidx + n_lo, n - n_lo, lo, hi);
    lo[cd] = save_lo;
    t->nodes[id].child[0] = a;
    t->nodes[id].child[1] = b;
    return id;
}

void *or_kdtree_build_bs(const float *data, int n, int d, int bs) {
    kd_tree *t = (kd_tree *)calloc(1, sizeof(kd_tree));
    t->data = data;
    t->n = n;
    t->d = d;
    t->bs = bs < 1 ? 1 : bs;
    t->nodes = (kd_node *)malloc(sizeof(kd_node) * (size_t)(2 * (n > 0 ? n : 1)));
    t->pidx = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    t->box_lo = (float *)malloc(sizeof(float) * (size_t)d);
    t->box_hi = (float *)malloc(sizeof(float) * (size_t)d);
    for (int i = 0; i < n; i++) t->pidx[i] = i;
    for (int dim = 0; dim < d; dim++) {  /* annEnclRect */
        float mn = n ? data[dim] : 0.0f, mx = mn;
        for (int i = 1; i < n; i++) {
            const float c = data[(size_t)i * d + dim];
            if (c < mn) mn = c;
            if (c > mx) mx = c;
        }
        t->box_lo[dim] = mn;
        t->box_hi[dim] = mx;
    }
    float *lo = (float *)malloc(sizeof(float) * (size_t)d), *hi = (float *)malloc(sizeof(float) * (size_t)d);
    memcpy(lo, t->box_lo, sizeof(float) * (size_t)d);
    memcpy(hi, t->box_hi, sizeof(float) * (size_t)d);
    kd_build(t, t->pidx, n, lo, hi);
    free(lo);
    free(hi);
    return t;
}

void *or_kdtree_build(const float *data, int n, int d) { return or_kdtree_build_bs(data, n, d, 1); }

static void kd_splits_walk(const kd_tree *t, int id, int s, int *cd, float *cv, float *lo, float *hi) {
    const kd_node *nd = &t->nodes[id];
    if (nd->cut_dim < 0) return;
    /* the LO subtree holds exactly n_lo = size / 2 points; its size is found from its leaves */
    int lo_size = 0;
    {
        int stack[128], sp = 0;
        stack[sp++] = nd->child[0];
        while (sp) {
            const kd_node *c = &t->nodes[stack[--sp]];
            if (c->cut_dim < 0) lo_size += c->child[1];
            else {
                stack[sp++] = c->child[0];
                stack[sp++] = c->child[1];
            }
        }
    }
    const int m = s + lo_size;
    cd[m] = nd->cut_dim;
    cv[m] = nd->cut_val;
    lo[m] = nd->lo_bnd;
    hi[m] = nd->hi_bnd;
    kd_splits_walk(t, nd->child[0], s, cd, cv, lo, hi);
    kd_splits_walk(t, nd->child[1], m, cd, cv, lo, hi);
}

/* every split node by its split position m (LO = positions [s, m)): cut dim, cut value, cell bounds [n] */
void or_kdtree_splits(void *p, int *cd, float *cv, float *lo, float *hi) {
    const kd_tree *t = (const kd_tree *)p;
    if (t->n > 0) kd_splits_walk(t, 0, 0, cd, cv, lo, hi);
}

/* leaf position of every point: pos[pidx[i]] = i (the DFS order with every LO child first) */
void or_kdtree_positions(void *p, int *pos) {
    const kd_tree *t = (const kd_tree *)p;
    for (int i = 0; i < t->n; i++) pos[t->pidx[i]] = i;
}

void or_kdtree_free(void *p) {
    kd_tree *t = (kd_tree *)p;
    if (!t) return;
    free(t->nodes);
    free(t->pidx);
    free(t->box_lo);
    free(t->box_hi);
    free(t);
}

/* annkSearch state: ANNmin_k of k entries (k + 1 slots), keys ascending, equal keys in insertion order */
typedef struct {
    const kd_tree *t;
    const float *q;
    int k, cnt;
    float mk[33];
    int mi[33];
    long visited;
} kd_query;

static float kd_max_key(const kd_query *s) { return s->cnt == s->k ? s->mk[s->k - 1] : FLT_MAX; }

/* ANNmin_k::insert: shift only the entries with key > kv, so an equal key stays behind the earlier one */
static void kd_insert(kd_query *s, float kv, int inf) {
    int i;
    for (i = s->cnt; i > 0; i--) {
        if (s->mk[i - 1] > kv) {
            s->mk[i] = s->mk[i - 1];
            s->mi[i] = s->mi[i - 1];
        } else {
            break;
        }
    }
    s->mk[i] = kv;
    s->mi[i] = inf;
    if (s->cnt < s->k) s->cnt++;
}

static void kd_search(kd_query *s, int id, float box_dist) {
    const kd_node *nd = &s->t->nodes[id];
    if (nd->cut_dim < 0) { /* ANNkd_leaf::ann_search */
        float min_dist = kd_max_key(s);
        for (int b = 0; b < nd->child[1]; b++) {
            const int j = s->t->pidx[nd->child[0] + b];
            const float *p = s->t->data + (size_t)j * s->t->d;
            float dist = 0.0f;
            int i;
            s->visited++;
            for (i = 0; i < s->t->d; i++) {
                const float t = s->q[i] - p[i];
                const float sq = t * t;
                dist = dist + sq;
                if (dist > min_dist) break;
            }
            if (i >= s->t->d) {
                kd_insert(s, dist, j);
                min_dist = kd_max_key(s);
            }
        }
        return;
    }
    const float cut_diff = s->q[nd->cut_dim] - nd->cut_val;
    if (cut_diff < 0) {
        kd_search(s, nd->child[0], box_dist);
        float box_diff = nd->lo_bnd - s->q[nd->cut_dim];
        if (box_diff < 0) box_diff = 0;
        box_dist = box_dist + (cut_diff * cut_diff - box_diff * box_diff);
        if (box_dist * 1.0f < kd_max_key(s)) kd_search(s, nd->child[1], box_dist);
    } else {
        kd_search(s, nd->child[1], box_dist);
        float box_diff = s->q[nd->cut_dim] - nd->hi_bnd;
        if (box_diff < 0) box_diff = 0;
        box_dist = box_dist + (cut_diff * cut_diff - box_diff * box_diff);
        if (box_dist * 1.0f < kd_max_key(s)) kd_search(s, nd->child[0], box_dist);
    }
}

/* annkSearch(q, k, idx, dd, eps = 0): k results ascending; missing entries -1 / FLT_MAX */
static void kd_knn(const kd_tree *t, const float *q, int k, int *idx, float *err, long *visited) {
    kd_query s;
    s.t = t;
    s.q = q;
    s.k = k;
    s.cnt = 0;
    s.visited = 0;
    if (t->n > 0) {
        float bd = 0.0f;  /* annBoxDistance */
        for (int dim = 0; dim < t->d; dim++) {
            float v = 0.0f;
            if (q[dim] < t->box_lo[dim]) v = t->box_lo[dim] - q[dim];
            else if (q[dim] > t->box_hi[dim]) v = q[dim] - t->box_hi[dim];
            bd = bd + v * v;
        }
        kd_search(&s, 0, bd);
    }
    for (int i = 0; i < k; i++) {
        idx[i] = i < s.cnt ? s.mi[i] : -1;
        if (err) err[i] = i < s.cnt ? s.mk[i] : FLT_MAX;
    }
    if (visited) *visited += s.visited;
}

static int kd_nn(const kd_tree *t, const float *q, float *err, long *visited) {
    int i;
    kd_knn(t, q, 1, &i, err, visited);
    return i;
}

typedef struct {
    const kd_tree *t;
    const float *q;
    int nq, k, tid, threads;
    int *idx;
    float *err;
    long visited;
} kd_job;

static void *kd_worker(void *p) {
    kd_job *j = (kd_job *)p;
    for (int i = j->tid; i < j->nq; i += j->threads)
        kd_knn(j->t, j->q + (size_t)i * j->t->d, j->k, j->idx + (size_t)i * j->k, j->err + (size_t)i * j->k,
               &j->visited);
    return NULL;
}

/* k <= 32 results per query: idx/err [nq][k] */
long or_kdtree_search_multi_batch(void *p, const float *q, int nq, int k, int *idx, float *err, int threads) {
    const kd_tree *t = (const kd_tree *)p;
    if (k < 1) k = 1;
    if (k > 32) k = 32;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    if (threads > nq) threads = nq > 0 ? nq : 1;
    pthread_t th[256];
    kd_job jobs[256];
    for (int i = 0; i < threads; i++) {
        jobs[i] = (kd_job){t, q, nq, k, i, threads, idx, err, 0};
        pthread_create(&th[i], NULL, kd_worker, &jobs[i]);
    }
    long visited = 0;
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        visited += jobs[i].visited;
    }
    return visited;
}

long or_kdtree_search_batch(void *p, const float *q, int nq, int *idx, float *err, int threads) {
    return or_kdtree_search_multi_batch(p, q, nq, 1, idx, err, threads);
}

/* annkPriSearch (ANN.dll 0x1800121a0; ann_kdtree_pri_search 0x180003ef0 calls it with k = 1, the caller's eps):
 * the root enters ANNpr_queue (a 1-based binary min-heap, pr_queue(n_pts) entries) with annBoxDistance; while it is
 * non-empty the minimum is extracted (inlined at 0x1800122d0) and, unless key * (1 + eps)^2 >= the current best
 * (max_key), ANNkd_split::ann_pri_search (0x180012580) descends on q's side with the same box, pushing each far child
 * with (cut_diff^2 - box_diff^2) + box, box_diff = maxss(bound difference, 0); ANNkd_leaf::ann_pri_search
 * (0x180012670) scans the bucket exactly as annkSearch's leaf does.  k = 1. */
typedef struct {
    float key;
    int node;
} pq_entry;

/* ANNpr_queue::insert (0x180008fc0): sift up while the parent's key > kv */
static void pq_insert(pq_entry *pq, int *n, float kv, int node) {
    int r = ++*n;
    while (r > 1) {
        const int p = r / 2;
        if (pq[p].key <= kv) break;
        pq[r] = pq[p];
        r = p;
    }
    pq[r].key = kv;
    pq[r].node = node;
}

/* ANNpr_queue::extr_min (0x1800122d0-0x180012364) */
static pq_entry pq_extr_min(pq_entry *pq, int *n) {
    const pq_entry top = pq[1];
    const float kn = pq[*n].key;
    (*n)--;
    int p = 1, r = 2;
    while (r <= *n) {
        if (r < *n && pq[r].key > pq[r + 1].key) r++;
        if (kn <= pq[r].key) break;
        pq[p] = pq[r];
        p = r;
        r = p << 1;
    }
    pq[p] = pq[*n + 1];
    return top;
}

static int kd_pri_nn(const kd_tree *t, const float *q, float eps, float *err, pq_entry *pq) {
    kd_query s;
    s.t = t;
    s.q = q;
    s.k = 1;
    s.cnt = 0;
    s.visited = 0;
    if (t->n > 0) {
        float max_err = eps + 1.0f;
        max_err = max_err * max_err;
        float bd = 0.0f; /* annBoxDistance */
        for (int dim = 0; dim < t->d; dim++) {
            float v = 0.0f;
            if (q[dim] < t->box_lo[dim]) v = t->box_lo[dim] - q[dim];
            else if (q[dim] > t->box_hi[dim]) v = q[dim] - t->box_hi[dim];
            bd = bd + v * v;
        }
        int hn = 0;
        pq_insert(pq, &hn, bd, 0);
        while (hn > 0) {
            const pq_entry top = pq_extr_min(pq, &hn);
            if (top.key * max_err >= kd_max_key(&s)) break;
            const float box = top.key;
            int id = top.node;
            for (;;) {
                const kd_node *nd = &t->nodes[id];
                if (nd->cut_dim < 0) { /* ANNkd_leaf::ann_pri_search */
                    float min_dist = kd_max_key(&s);
                    for (int b = 0; b < nd->child[1]; b++) {
                        const int j = t->pidx[nd->child[0] + b];
                        const float *p = t->data + (size_t)j * t->d;
                        float dist = 0.0f;
                        int i;
                        for (i = 0; i < t->d; i++) {
                            const float tt = q[i] - p[i];
                            dist = dist + tt * tt;
                            if (dist > min_dist) break;
                        }
                        if (i >= t->d) {
                            kd_insert(&s, dist, j);
                            min_dist = kd_max_key(&s);
                        }
                    }
                    break;
                }
                const float qd = q[nd->cut_dim];
                const float cut_diff = qd - nd->cut_val;
                if (cut_diff < 0) {
                    float box_diff = nd->lo_bnd - qd;
                    box_diff = box_diff > 0.0f ? box_diff : 0.0f; /* maxss */
                    pq_insert(pq, &hn, (cut_diff * cut_diff - box_diff * box_diff) + box, nd->child[1]);
                    id = nd->child[0];
                } else {
                    float box_diff = qd - nd->hi_bnd;
                    box_diff = box_diff > 0.0f ? box_diff : 0.0f;
                    pq_insert(pq, &hn, (cut_diff * cut_diff - box_diff * box_diff) + box, nd->child[0]);
                    id = nd->child[1];
                }
            }
        }
    }
    if (err) *err = s.cnt ? s.mk[0] : FLT_MAX;
    return s.cnt ? s.mi[0] : -1;
}

/* nq ann_kdtree_pri_search calls (single thread): idx/err [nq] */
void or_kdtree_pri_search_batch(void *p, const float *q, int nq, float eps, int *idx, float *err) {
    const kd_tree *t = (const kd_tree *)p;
    pq_entry *pq = (pq_entry *)malloc(((size_t)t->n + 2) * sizeof(pq_entry));
    for (int i = 0; i < nq; i++) idx[i] = kd_pri_nn(t, q + (size_t)i * t->d, eps, err + i, pq);
    free(pq);
}
