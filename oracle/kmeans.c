/*
 * kmeans.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * The Dither step's k-means (PrepareDitherTiles main.pas:2125-2133: yakmo_create(FPaletteCount, 1, MaxInt, 1, 0, 0,
 * 0), i.e. one restart, iterate to convergence, k-means++ initialisation, seed 0, no normalisation), written out
 * as the published algorithm because yakmo.dll is binary-only (its RNG stream and accelerated iterations are not
 * visible): parity with the DLL is unpinned.  The text the GPU product (tiler_amd/csrc/kmeans.hip) follows:
 *   distance   sum over d ascending of (x_d - c_d)^2, fp64, no contraction; ties -> lowest centroid index
 *   seeding    MT19937(seed), u = genrand_int32 / 2^32 per draw; centre 0 = point floor(u * n); centre s is
 *              drawn with probability D^2 / sum D^2: the sum over runs of L = ceil(n / 1024) points (sequential in
 *              a run, the run sums in order), the pick the first point whose running sum (runs before it, then
 *              the points of its run) exceeds u * sum; floor(u * n) when the sum is 0
 *   Lloyd      assign; stop when no label changes or after max_iter assignments; else each non-empty centroid =
 *              the mean of its members in point order summed in runs of 256 members (run sums in order) / count
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "tiler_oracle.h"

typedef struct {
    uint32_t mt[624];
    int mti;
} mt_state;

static void mt_init(mt_state *m, uint32_t s) {
    m->mt[0] = s;
    for (m->mti = 1; m->mti < 624; m->mti++)
        m->mt[m->mti] = 1812433253u * (m->mt[m->mti - 1] ^ (m->mt[m->mti - 1] >> 30)) + (uint32_t)m->mti;
}

static uint32_t mt_next(mt_state *m) {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    uint32_t y;
    if (m->mti >= 624) {
        int kk;
        for (kk = 0; kk < 624 - 397; kk++) {
            y = (m->mt[kk] & 0x80000000u) | (m->mt[kk + 1] & 0x7fffffffu);
            m->mt[kk] = m->mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; kk < 623; kk++) {
            y = (m->mt[kk] & 0x80000000u) | (m->mt[kk + 1] & 0x7fffffffu);
            m->mt[kk] = m->mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        y = (m->mt[623] & 0x80000000u) | (m->mt[0] & 0x7fffffffu);
        m->mt[623] = m->mt[396] ^ (y >> 1) ^ mag01[y & 1u];
        m->mti = 0;
    }
    y = m->mt[m->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

uint32_t or_mt19937_first(uint32_t seed) { /* known-answer hook: seed 5489 -> 3499211612 */
    mt_state m;
    mt_init(&m, seed);
    return mt_next(&m);
}

static double dist2(const double *a, const double *b, int d) {
    double acc = 0.0;
    for (int k = 0; k < d; k++) {
        const double t = a[k] - b[k];
        acc = acc + t * t;
    }
    return acc;
}

typedef struct {
    const double *X, *cent;
    long n;
    int d, k, nth, id;
    int32_t *labels;
    long changed;
} assign_job;

static void *assign_part(void *arg) {
    assign_job *j = (assign_job *)arg;
    const long b = j->n * j->id / j->nth, e = j->n * (j->id + 1) / j->nth;
    long ch = 0;
    for (long i = b; i < e; i++) {
        double best = HUGE_VAL;
        int bc = -1;
        for (int c = 0; c < j->k; c++) {
            const double v = dist2(j->X + i * j->d, j->cent + (long)c * j->d, j->d);
            if (v < best) {
                best = v;
                bc = c;
            }
        }
        if (j->labels[i] != bc) {
            j->labels[i] = bc;
            ch++;
        }
    }
    j->changed = ch;
    return NULL;
}

int or_kmeans(const double *X, long n, int d, int k, int max_iter, uint32_t seed, int32_t *labels, double *cent,
              int threads) {
    mt_state rng;
    mt_init(&rng, seed);
    double *u = (double *)malloc(sizeof(double) * (size_t)k);
    for (int s = 0; s < k; s++) u[s] = (double)mt_next(&rng) * (1.0 / 4294967296.0);
    /* k-means++ */
    long first = (long)(u[0] * (double)n);
    if (first >= n) first = n - 1;
    memcpy(cent, X + first * d, sizeof(double) * (size_t)d);
    double *mind2 = (double *)malloc(sizeof(double) * (size_t)n);
    const long L = (n + 1023) / 1024;
    for (int s = 1; s < k; s++) {
        const double *c = cent + (long)(s - 1) * d;
        for (long i = 0; i < n; i++) {
            const double v = dist2(X + i * d, c, d);
            mind2[i] = (s == 1 || v < mind2[i]) ? v : mind2[i];
        }
        double part[1024];
        for (int r = 0; r < 1024; r++) {
            double acc = 0.0;
            for (long i = (long)r * L; i < (long)(r + 1) * L && i < n; i++) acc = acc + mind2[i];
            part[r] = acc;
        }
        double S = 0.0;
        for (int r = 0; r < 1024; r++) S = S + part[r];
        long p = -1;
        if (S > 0.0) {
            const double target = u[s] * S;
            double run = 0.0;
            for (int r = 0; r < 1024 && p < 0; r++) {
                if (run + part[r] > target) {
                    const long rb = (long)r * L, re = rb + L < n ? rb + L : n;
                    double a2 = run;
                    for (long i = rb; i < re; i++) {
                        a2 = a2 + mind2[i];
                        if (a2 > target) {
                            p = i;
                            break;
                        }
                    }
                    if (p < 0) p = re - 1;
                } else
                    run = run + part[r];
            }
            if (p < 0) p = n - 1;
        } else {
            p = (long)(u[s] * (double)n);
            if (p >= n) p = n - 1;
        }
        memcpy(cent + (long)s * d, X + p * d, sizeof(double) * (size_t)d);
    }
    free(mind2);
    free(u);
    /* Lloyd */
    for (long i = 0; i < n; i++) labels[i] = -1;
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    int it = 0;
    long *cnt = (long *)malloc(sizeof(long) * (size_t)k);
    long *start = (long *)malloc(sizeof(long) * (size_t)(k + 1));
    long *members = (long *)malloc(sizeof(long) * (size_t)n);
    double *acc = (double *)malloc(sizeof(double) * (size_t)d);
    double *runacc = (double *)malloc(sizeof(double) * (size_t)d);
    while (it < max_iter) {
        pthread_t th[64];
        assign_job jobs[64];
        long changed = 0;
        for (int t = 0; t < threads; t++) {
            jobs[t] = (assign_job){X, cent, n, d, k, threads, t, labels, 0};
            if (t) pthread_create(&th[t], NULL, assign_part, &jobs[t]);
        }
        assign_part(&jobs[0]);
        for (int t = 1; t < threads; t++) pthread_join(th[t], NULL);
        for (int t = 0; t < threads; t++) changed += jobs[t].changed;
        it++;
        if (changed == 0 || it >= max_iter) break;
        memset(cnt, 0, sizeof(long) * (size_t)k);
        for (long i = 0; i < n; i++) cnt[labels[i]]++;
        start[0] = 0;
        for (int c = 0; c < k; c++) start[c + 1] = start[c] + cnt[c];
        for (int c = 0; c < k; c++) cnt[c] = start[c];
        for (long i = 0; i < n; i++) members[cnt[labels[i]]++] = i; /* point order within each cluster */
        for (int c = 0; c < k; c++) {
            const long m = start[c + 1] - start[c];
            if (m == 0) continue;
            for (int t = 0; t < d; t++) acc[t] = 0.0;
            for (long b = start[c]; b < start[c + 1]; b += 256) {
                const long e = b + 256 < start[c + 1] ? b + 256 : start[c + 1];
                for (int t = 0; t < d; t++) runacc[t] = 0.0;
                for (long i = b; i < e; i++)
                    for (int t = 0; t < d; t++) runacc[t] = runacc[t] + X[members[i] * d + t];
                for (int t = 0; t < d; t++) acc[t] = acc[t] + runacc[t];
            }
            for (int t = 0; t < d; t++) cent[(long)c * d + t] = acc[t] / (double)m;
        }
    }
    free(cnt);
    free(start);
    free(members);
    free(acc);
    free(runacc);
    return it;
}
