/* Study (not product, not the oracle): how much of K-Modes' per-chunk assignment an exact "touched clusters" fix-up
 * would still compute.  KModesIter (kmodes.pas:845-915) assigns each 960-point chunk against the modes as the
 * previous chunks left them.  A key computed against the modes at the iteration's start is exact for every cluster
 * whose mode bytes have not changed since; so per chunk c, with T_c = clusters whose modes changed since the start:
 *   point p with snapshot best b_p not in T_c: best = argmin over {b_p} + T_c  (min distance, ties -> highest index)
 *   point p with b_p in T_c: full argmin over all K clusters.
 * This program runs the restated K-Modes (the oracle's semantics: or_km_get_min, MovePointCat, the rescue) on one bin,
 * checks the fix-up against the full assignment at every chunk (it must be identical), and prints per iteration the
 * pairs the fix-up evaluates against the full assignment's.
 *   gcc -O2 -o /tmp/kms/study tools/km_touched_study.c oracle/liboracle.so -lpthread
 *   /tmp/kms/study X.u8 n K start */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

uint64_t or_km_dissim(const uint8_t *row, const uint8_t *item);
int or_km_get_min(const uint8_t *rows, int count, const uint8_t *item, uint64_t *best);
void or_km_update_min_distance(const uint8_t *item, const uint8_t *rows, int count, uint64_t *mindist);
uint32_t or_randint(uint32_t range, uint32_t *seed);

enum { A = 80, M = 16, BIN = 960 };
static int N, K;
static const uint8_t *X;
static int32_t *memb, *csize, *freq;
static uint8_t *cent, *snap;
static uint8_t *touched; /* [K]: mode changed since the iteration's snapshot */
static int *tlist, tn;

static int max_value_index(const int32_t *arr, int n) {
    int r = -1;
    int32_t best = INT32_MIN;
    for (int i = 0; i < n; i++)
        if (arr[i] > best) {
            best = arr[i];
            r = i;
        }
    return r;
}
static void mark(int c) {
    if (memcmp(cent + (size_t)c * A, snap + (size_t)c * A, A) != 0 && !touched[c]) {
        touched[c] = 1;
        tlist[tn++] = c;
    }
}
static void move_point_cat(int ip, int to, int from) {
    const uint8_t *pt = X + (size_t)ip * A;
    memb[ip] = to;
    csize[to]++;
    csize[from]--;
    for (int a = 0; a < A; a++) {
        int cur = pt[a];
        int32_t *tc = freq + ((size_t)to * A + a) * M, *fc = freq + ((size_t)from * A + a) * M;
        tc[cur]++;
        int ccv = cent[(size_t)to * A + a];
        if (tc[ccv] < tc[cur]) cent[(size_t)to * A + a] = (uint8_t)cur;
        fc[cur]--;
        if (cent[(size_t)from * A + a] == cur) cent[(size_t)from * A + a] = (uint8_t)max_value_index(fc, M);
    }
    mark(to);
    mark(from);
}

int main(int argc, char **argv) {
    if (argc < 5) return 2;
    N = atoi(argv[2]);
    K = atoi(argv[3]);
    const int start = atoi(argv[4]);
    uint8_t *Xb = malloc((size_t)N * A);
    FILE *f = fopen(argv[1], "rb");
    if (!f || fread(Xb, 1, (size_t)N * A, f) != (size_t)N * A) return 3;
    fclose(f);
    X = Xb;
    memb = calloc(N, 4);
    csize = calloc(K, 4);
    freq = calloc((size_t)K * A * M, 4);
    cent = malloc((size_t)K * A);
    snap = malloc((size_t)K * A);
    touched = calloc(K, 1);
    tlist = malloc(sizeof(int) * K);
    uint32_t seed = 0x42381337u;
    /* InitFarthestFirst */
    {
        uint64_t *mind = malloc(8 * (size_t)N);
        uint8_t *used = calloc(N, 1);
        memset(cent, 0xff, (size_t)K * A);
        for (int i = 0; i < N; i++) mind[i] = UINT64_MAX;
        int fp = start;
        memcpy(cent, X + (size_t)fp * A, A);
        used[fp] = 1;
        or_km_update_min_distance(X + (size_t)fp * A, X, N, mind);
        for (int c = 1; c < K; c++) {
            uint64_t mx = 0;
            fp = -1;
            for (int i = 0; i < N; i++)
                if (mind[i] >= mx && !used[i]) {
                    mx = mind[i];
                    fp = i;
                }
            memcpy(cent + (size_t)c * A, X + (size_t)fp * A, A);
            used[fp] = 1;
            or_km_update_min_distance(X + (size_t)fp * A, X, N, mind);
        }
        free(mind);
        free(used);
    }
    {
        uint64_t d;
        for (int i = 0; i < N; i++) memb[i] = or_km_get_min(cent, K, X + (size_t)i * A, &d);
        for (int i = 0; i < N; i++) csize[memb[i]]++;
        for (int i = 0; i < N; i++)
            for (int a = 0; a < A; a++) freq[((size_t)memb[i] * A + a) * M + X[(size_t)i * A + a]]++;
        for (int k = 0; k < K; k++) {
            if (csize[k] == 0)
                for (int a = 0; a < A; a++) cent[(size_t)k * A + a] = X[(size_t)or_randint((uint32_t)N, &seed) * A + a];
            else
                for (int a = 0; a < A; a++) cent[(size_t)k * A + a] = (uint8_t)max_value_index(freq + ((size_t)k * A + a) * M, M);
        }
    }
    int32_t *sb = malloc(4 * (size_t)N), *choices = malloc(4 * (size_t)N);
    uint64_t *sd = malloc(8 * (size_t)N);
    uint64_t cost = UINT64_MAX;
    long long tot_full = 0, tot_fix = 0, tot_fix_touched = 0, tot_fix_full = 0;
    for (int itr = 1;; itr++) {
        /* snapshot: every point against the modes at the iteration's start */
        memcpy(snap, cent, (size_t)K * A);
        for (int i = 0; i < N; i++) sb[i] = or_km_get_min(cent, K, X + (size_t)i * A, &sd[i]);
        for (int i = 0; i < tn; i++) touched[tlist[i]] = 0;
        tn = 0;
        int moves = 0, dirty_chunks = 0, max_t = 0;
        long long full = 0, fx_t = 0, fx_f = 0;
        uint64_t acc = 0;
        for (int b0 = 0; b0 < N; b0 += BIN) {
            const int last = (b0 + BIN < N ? b0 + BIN : N) - 1, np = last - b0 + 1;
            full += (long long)np * K;
            if (tn > 0) dirty_chunks++;
            if (tn > max_t) max_t = tn;
            int32_t clust[BIN];
            uint64_t dis[BIN];
            for (int i = b0; i <= last; i++) {
                uint64_t d;
                const int c = or_km_get_min(cent, K, X + (size_t)i * A, &d); /* the reference */
                int fc;
                uint64_t fd;
                if (!touched[sb[i]]) { /* fix-up: snapshot best + the touched clusters */
                    fc = sb[i];
                    fd = sd[i];
                    for (int t = 0; t < tn; t++) {
                        const int cc = tlist[t];
                        const uint64_t dd = or_km_dissim(cent + (size_t)cc * A, X + (size_t)i * A);
                        if (dd < fd || (dd == fd && cc > fc)) {
                            fd = dd;
                            fc = cc;
                        }
                    }
                    fx_t += tn;
                } else {
                    fc = or_km_get_min(cent, K, X + (size_t)i * A, &fd);
                    fx_f += K;
                }
                if (fc != c || fd != d) {
                    fprintf(stderr, "MISMATCH itr %d point %d: ref (%d, %llu) fix (%d, %llu)\n", itr, i, c, (unsigned long long)d, fc,
                            (unsigned long long)fd);
                    return 1;
                }
                clust[i - b0] = c;
                dis[i - b0] = d;
            }
            for (int i = b0; i <= last; i++) {
                acc += dis[i - b0];
                if (memb[i] != clust[i - b0]) {
                    moves++;
                    const int old = memb[i];
                    move_point_cat(i, clust[i - b0], old);
                    if (csize[old] == 0) {
                        int from = 0, mc = 0;
                        for (int c = 0; c < K; c++)
                            if (csize[c] >= mc) {
                                mc = csize[c];
                                from = c;
                            }
                        int cnt = 0;
                        for (int j = 0; j < N; j++)
                            if (memb[j] == from) choices[cnt++] = j;
                        const int r = choices[or_randint((uint32_t)cnt, &seed)];
                        move_point_cat(r, old, from);
                    }
                }
            }
        }
        tot_full += full;
        tot_fix_touched += fx_t;
        tot_fix_full += fx_f;
        tot_fix += fx_t + fx_f;
        printf("iter %2d moves %6d dirty_chunks %3d/%d touched_end %5d | pairs full %.3g fixup %.3g (touched %.3g + full %.3g) = %.3f\n",
               itr, moves, dirty_chunks, (N + BIN - 1) / BIN, tn, (double)full, (double)(fx_t + fx_f), (double)fx_t,
               (double)fx_f, (double)(fx_t + fx_f) / (double)full);
        fflush(stdout);
        const int conv = (acc >= cost) || (moves == 0);
        cost = acc;
        if (conv) break;
    }
    printf("total pairs: full %.4g fixup %.4g (touched %.4g, full recomputes %.4g) ratio %.3f\n", (double)tot_full,
           (double)tot_fix, (double)tot_fix_touched, (double)tot_fix_full, (double)tot_fix / (double)tot_full);
    return 0;
}
