/* Study (not product, not oracle): DLv3 pass 2 with a per-entry candidate cache, checked against the plain scans.
 *
 * The restated reduce_table3 (oracle/palette.c, quantizer.c:583-648) runs unchanged; beside it every entry i keeps
 * S_i = its two smallest (err, index) candidates of (i, tot) from its last full scan and F_i = the third smallest err
 * (a lower bound on every candidate outside S_i).  After each merge the three changed indices (c1, c2, the removed
 * last entry) leave every S_i and the two changed candidates' new values enter it when they are below F_i (what they
 * push out lowers F_i).  Each recount_next(i) the reference runs is first answered from S_i -- its smallest valid
 * entry when that is below F_i -- and that answer is compared with the scan's.  Prints hits, misses, mismatches.
 * Usage: dl3_cache_study <rgb file: uint8 r,g,b triplets> [lookup_bpc=7] [quant_to=16]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint32_t r, g, b, n; float err; int32_t cc; uint8_t rr, gg, bb; } cube3;
#ifndef M
#define M 2  /* cached candidates per entry */
#endif
typedef struct { float v[M]; int j[M]; float F; int ok; } cache_t;
static cube3 *T; static int tot; static float sq[511];
static cache_t *C;
static long long hits, misses, bad, maint_evals, maint_ins, scans;

static void setrgb(cube3 *r) { int v = (int)r->n, v2 = v >> 1; r->rr = (uint8_t)((r->r + v2) / v); r->gg = (uint8_t)((r->g + v2) / v); r->bb = (uint8_t)((r->b + v2) / v); }
static float calc_err(int c1, int c2) {
    const cube3 *a = T + c1, *b = T + c2; uint32_t P1 = a->n, P2 = b->n, P3 = P1 + P2;
    int R3 = (int)((a->r + b->r + (P3 >> 1)) / P3), G3 = (int)((a->g + b->g + (P3 >> 1)) / P3), B3 = (int)((a->b + b->b + (P3 >> 1)) / P3);
    float d1 = sq[R3 - a->rr + 255] + sq[G3 - a->gg + 255] + sq[B3 - a->bb + 255]; d1 = sqrtf(d1) * (float)P1;
    float d2 = sq[b->rr - R3 + 255] + sq[b->gg - G3 + 255] + sq[b->bb - B3 + 255]; d2 = sqrtf(d2) * (float)P2;
    return d1 + d2;
}
static int lt(float v1, int j1, float v2, int j2) { return v1 < v2 || (v1 == v2 && j1 < j2); }
/* the full scan: first minimum (the reference's), and (keep) the cache's top two + third value */
static void scan(int i, float *e, int *c, int keep) {
    float v[M + 1]; int jj[M + 1];
    for (int k = 0; k <= M; k++) { v[k] = HUGE_VALF; jj[k] = -1; }
    float err = HUGE_VALF; int c2 = 0;
    for (int j = i + 1; j < tot; j++) {
        const float cur = calc_err(i, j);
        if (cur < err) { err = cur; c2 = j; }
        if (lt(cur, j, v[M], jj[M])) {
            v[M] = cur; jj[M] = j;
            for (int k = M; k > 0 && lt(v[k], jj[k], v[k - 1], jj[k - 1]); k--) {
                float tv = v[k]; v[k] = v[k - 1]; v[k - 1] = tv; int tj = jj[k]; jj[k] = jj[k - 1]; jj[k - 1] = tj;
            }
        }
    }
    *e = err; *c = c2; scans++;
    if (!keep) return;
    for (int k = 0; k < M; k++) { C[i].v[k] = v[k]; C[i].j[k] = jj[k]; }
    C[i].F = v[M]; C[i].ok = 1;
}
static void recount_next(int i) {
    /* the cache's answer first */
    int have = 0; float av = HUGE_VALF; int aj = -1;
    if (C[i].ok) for (int s = 0; s < M; s++) if (C[i].j[s] >= 0 && lt(C[i].v[s], C[i].j[s], av, aj)) { av = C[i].v[s]; aj = C[i].j[s]; have = 1; }
    const int answer = have && av < C[i].F;
    float e; int c; scan(i, &e, &c, !answer);  /* the truth; a miss rebuilds the cache, a hit keeps it */
    if (answer) { hits++; scans--; if (!(e == av && c == aj)) bad++; } else misses++;
    T[i].err = e; T[i].cc = c;
}
static void insert(int i, float v, int j) {
    cache_t *q = C + i; maint_ins++;
    int w = -1;
    for (int s = 0; s < M && w < 0; s++) if (q->j[s] < 0) w = s;
    if (w >= 0) { q->v[w] = v; q->j[w] = j; return; }
    w = 0;  /* the worst slot */
    for (int s = 1; s < M; s++) if (lt(q->v[w], q->j[w], q->v[s], q->j[s])) w = s;
    if (lt(v, j, q->v[w], q->j[w])) { if (q->v[w] < q->F) q->F = q->v[w]; q->v[w] = v; q->j[w] = j; }
    else if (v < q->F) q->F = v;
}
static void maintain(int c1, int c2, int told) {
    for (int i = 0; i < tot; i++) {
        cache_t *q = C + i;
        if (i == c1 || (c2 != told && i == c2)) { q->ok = 0; continue; }
        if (!q->ok) continue;
        for (int s = 0; s < M; s++) if (q->j[s] == c1 || q->j[s] == c2 || q->j[s] == told) { q->j[s] = -1; q->v[s] = HUGE_VALF; }
        const int xs[2] = {c1, c2 != told ? c2 : -1};
        for (int k = 0; k < 2; k++) {
            const int x = xs[k];
            if (x <= i || x >= tot) continue;
            maint_evals++;
            const float v = calc_err(i, x);
            if (v < q->F) insert(i, v, x);
        }
    }
}
static void recount_dist(int c1) {
    recount_next(c1);
    for (int i = 0; i < c1; i++) {
        if (T[i].cc == c1) recount_next(i);
        else { const float cur = calc_err(i, c1); if (cur < T[i].err) { T[i].err = cur; T[i].cc = c1; } }
    }
}
int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s rgb.bin [bpc] [quant_to]\n", argv[0]); return 2; }
    const int bpc = argc > 2 ? atoi(argv[2]) : 7, quant_to = argc > 3 ? atoi(argv[3]) : 16;
    FILE *f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); long nb = ftell(f); fseek(f, 0, SEEK_SET);
    uint8_t *px = malloc(nb); if (fread(px, 1, nb, f) != (size_t)nb) return 1; fclose(f);
    for (int i = -255; i <= 255; i++) sq[i + 255] = (float)(i * i);
    const long lsz = 1L << (bpc * 3); const int mb = (1 << bpc) - 1;
    T = calloc(lsz, sizeof(cube3));
    for (long p = 0; p < nb / 3; p++) {
        const uint8_t *im = px + 3 * p; int r = im[0] * mb / 255, g = im[1] * mb / 255, b = im[2] * mb / 255;
        long idx = b | (g << bpc) | (r << (bpc << 1)); T[idx].r += im[0]; T[idx].g += im[1]; T[idx].b += im[2]; T[idx].n++;
    }
    tot = 0; for (long i = 0; i < lsz; i++) if (T[i].n) { setrgb(T + i); T[tot++] = T[i]; }
    const int hist = tot; C = calloc(tot + 1, sizeof(cache_t));
    int i, c1 = 0, c2 = 0;
    for (i = 0; i < tot - 1; i++) { float e; int c; scan(i, &e, &c, 1); T[i].err = e; T[i].cc = c; }
    T[i].err = HUGE_VALF; T[i].cc = tot; C[i].ok = 0;
    const long long pass1_scans = scans; scans = 0;
    while (tot > quant_to) {
        float err = HUGE_VALF;
        for (i = 0; i < tot; i++) if (T[i].err < err) { err = T[i].err; c1 = i; }
        c2 = T[c1].cc;
        T[c2].r += T[c1].r; T[c2].g += T[c1].g; T[c2].b += T[c1].b; T[c2].n += T[c1].n; setrgb(T + c2);
        tot--;
        T[c1] = T[tot]; C[c1] = C[tot];
        T[tot - 1].err = HUGE_VALF; T[tot - 1].cc = tot;
        maintain(c1, c2, tot);
        C[tot - 1].ok = 0;
        for (i = 0; i < c1; i++) if (T[i].cc == tot) T[i].cc = c1;
        for (i = c1 + 1; i < tot; i++) if (T[i].cc == tot) recount_next(i);
        recount_dist(c1);
        if (c2 != tot) recount_dist(c2);
    }
    printf("{\"colors\": %d, \"merges\": %d, \"pass1_scans\": %lld, \"recounts\": %lld, \"cache_hits\": %lld, "
           "\"cache_misses\": %lld, \"mismatches\": %lld, \"maint_calc_err\": %lld, \"maint_insertions\": %lld}\n",
           hist, hist - quant_to, pass1_scans, hits + misses, hits, misses, bad, maint_evals, maint_ins);
    return bad != 0;
}
