// dither.hip -- FinishDitherTiles' per-tile work on gfx950 (once the keyframe palettes exist):
//   DitherTile with Thomas Knoll mixing (the default, chkUseTK, main.lfm:272-282)   main.pas:1998-2055
//   or with Yliluoma mixing (chkUseTK unchecked; dither_yl_kernel below)           main.pas:1573-1826, 2055-2067
//   DeviseBestMixingPlanThomasKnoll main.pas:1828-1875, PreparePlan main.pas:1494-1526, ColorCompare 1557-1571
//   the luma sort: the reference's own QuickSort (kmodes.pas:89-136) with PlanCompareLuma (main.pas:1540-1551)
//   PrepareTileMirrors (canonical orientation) main.pas:4049-4069
// Layout: one wave per tile, one lane per pixel (y*8+x).  Each lane runs its colour's 64 error-diffusion steps
// against the tile's palette (wave-uniform, in registers), keeps its 64-entry list in LDS ([entry][lane] bytes),
// sorts it with the same QuickSort (explicit per-lane stack in LDS, larger side pending: partitions of disjoint
// ranges commute, so the visiting order does not change the result), and reads entry cDitheringMap[y*8+x].  The quadrant sums and
// the flip of PrepareTileMirrors are wave reductions and one lane permutation.
// Integer ranges: |e| <= 63*255, so |t| <= 255 + 1445 and every ColorCompare term fits int32
// (3*13*1723^2 + 32*1723^2 < 2^31): int32 arithmetic gives the reference's Int64 results exactly.
// The reference's colour cache (CountCache/ListCache) only memoises lists per colour: not needed here.
#include <string>

#include "dither.hpp"

namespace tiler {

__constant__ uint8_t c_dither_map[64] = {  // cDitheringMap main.pas:46-55
    0,  48, 12, 60, 3,  51, 15, 63, 32, 16, 44, 28, 35, 19, 47, 31, 8,  56, 4,  52, 11, 59,
    7,  55, 40, 24, 36, 20, 43, 27, 39, 23, 2,  50, 14, 62, 1,  49, 13, 61, 34, 18, 46, 30,
    33, 17, 45, 29, 10, 58, 6,  54, 9,  57, 5,  53, 42, 26, 38, 22, 41, 25, 37, 21};

constexpr int DT_WAVES = 4;       // tiles per workgroup
constexpr int DT_MAXPAL = 16;     // palette entries held in registers
constexpr int DT_STACK = 8;       // pending quicksort ranges per lane (larger side stacked: <= log2 64)

// The reference QuickSort (kmodes.pas:89-136) of this lane's list entries [0, last] ([entry][lane] bytes in LDS) by
// PlanCompareLuma: the reference's partition steps on a per-lane stack of pending ranges (disjoint ranges: the
// visiting order leaves the final array unchanged); the larger side waits, so the depth stays <= log2(last + 1)
template <class LumaOf>
__device__ __forceinline__ void lane_quicksort(uint8_t *list, uint16_t *stk, int lane, int last0, LumaOf luma_of) {
    int sp = 0;
    int first = 0, last = last0;
    for (;;) {
        while (last > first) {
            // one partition step of the reference on [first, last] (same pivot, scans and swaps)
            int i = first, j = last;
            int pp = (first + last) >> 1;
            do {
                const int lp = luma_of(list[pp * 64 + lane]);
                while (luma_of(list[i * 64 + lane]) < lp) i++;
                while (luma_of(list[j * 64 + lane]) > lp) j--;
                if (i <= j) {
                    const uint8_t t = list[j * 64 + lane];
                    list[j * 64 + lane] = list[i * 64 + lane];
                    list[i * 64 + lane] = t;
                    if (pp == i)
                        pp = j;
                    else if (pp == j)
                        pp = i;
                    i++;
                    j--;
                }
            } while (i <= j);
            // the reference sorts [first, j] then [i, last]; they are disjoint, so the order is free
            const bool hl = first < j, hr = i < last;
            if (hl && hr) {
                if (j - first > last - i) {
                    stk[(sp++) * 64 + lane] = (uint16_t)(first | (j << 8));
                    first = i;
                } else {
                    stk[(sp++) * 64 + lane] = (uint16_t)(i | (last << 8));
                    last = j;
                }
            } else if (hl) {
                last = j;
            } else if (hr) {
                first = i;
            } else {
                break;
            }
        }
        if (sp == 0) break;
        const uint16_t r = stk[(--sp) * 64 + lane];
        first = r & 0xff;
        last = r >> 8;
    }
}

// PrepareTileMirrors (main.pas:4049-4069): quadrant sums in (vf, hf) order FF, FT, TF, TT, first strict maximum;
// the tile stored in canonical orientation.  px: this lane's (pixel y*8+x) palette index; the whole wave active.
__device__ __forceinline__ void tile_mirrors_store(int px, int lane, int tile, uint8_t *__restrict__ palpix,
                                                   uint8_t *__restrict__ hm, uint8_t *__restrict__ vm) {
    const int y = lane >> 3, x = lane & 7;
    const int q = (y >= 4 ? 2 : 0) + (x >= 4 ? 1 : 0);
    int qs[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int v = q == k ? px : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        qs[k] = v;
    }
    int best = -1, bq = 0;
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (qs[k] > best) {
            best = qs[k];
            bq = k;
        }
    const int bh = bq & 1, bv = bq >> 1;
    const int src = (bv ? 7 - y : y) * 8 + (bh ? 7 - x : x);
    palpix[(long)tile * 64 + lane] = (uint8_t)__shfl(px, src, 64);
    if (lane == 0) {
        hm[tile] = (uint8_t)bh;
        vm[tile] = (uint8_t)bv;
    }
}

__global__ __launch_bounds__(64 * DT_WAVES) void dither_tk_kernel(const int32_t *__restrict__ rgb,
                                                                  const int32_t *__restrict__ pal_of,
                                                                  const int32_t *__restrict__ palettes,
                                                                  int n_palettes, int palsize, int n,
                                                                  uint8_t *__restrict__ palpix,
                                                                  uint8_t *__restrict__ hm, uint8_t *__restrict__ vm) {
    __shared__ uint8_t s_list[DT_WAVES][64 * 64];           // [entry][lane]
    __shared__ uint16_t s_stk[DT_WAVES][DT_STACK * 64];     // [depth][lane]: first | last << 8
    __shared__ int s_luma[DT_WAVES][DT_MAXPAL];             // LumaPal of the tile's palette
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int tile = blockIdx.x * DT_WAVES + w;
    if (tile >= n) return;
    const int p = pal_of[tile];
    uint8_t *list = s_list[w];
    if (p < 0 || p >= n_palettes) {  // invalid input (the host entry rejects it): defined output, no fault
        palpix[(long)tile * 64 + lane] = 0;
        if (lane == 0) hm[tile] = vm[tile] = 0;
        return;
    }
    // PreparePlan: Y2Palette r, g, b and LumaPal (wave-uniform)
    int pr[DT_MAXPAL], pg[DT_MAXPAL], pb[DT_MAXPAL], pl[DT_MAXPAL];
#pragma unroll
    for (int i = 0; i < DT_MAXPAL; i++) {
        const int c = i < palsize ? palettes[(long)p * palsize + i] : 0;
        pr[i] = c & 0xff;
        pg[i] = (c >> 8) & 0xff;
        pb[i] = (c >> 16) & 0xff;
        pl[i] = pr[i] * 2126 + pg[i] * 7152 + pb[i] * 722;
    }
    // Compare-loop constants.  With t fixed, 13*|t - p_i|^2 = 13*|t|^2 - 26*t.p_i + 13*|p_i|^2: the first term is
    // common to every i, so dropping it keeps the order and the ties of the strict-'<' scan (exact integers).
    // LumaPal_i = 10000*la_i + lb_i (0 <= lb_i < 10000), so trunc((l1 - LumaPal_i) / 10000) needs no division
    // per entry (see the loop).
    int pc[DT_MAXPAL], la[DT_MAXPAL], lb[DT_MAXPAL];
#pragma unroll
    for (int i = 0; i < DT_MAXPAL; i++) {
        pc[i] = 13 * (pr[i] * pr[i] + pg[i] * pg[i] + pb[i] * pb[i]);
        la[i] = pl[i] / 10000;
        lb[i] = pl[i] - la[i] * 10000;
    }
    if (lane < DT_MAXPAL) {
        const int c = lane < palsize ? palettes[(long)p * palsize + lane] : 0;
        s_luma[w][lane] = (c & 0xff) * 2126 + ((c >> 8) & 0xff) * 7152 + ((c >> 16) & 0xff) * 722;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    auto luma_of = [&](int v) { return s_luma[w][v]; };  // LumaPal[v] (PlanCompareLuma)
    // Distinct lumas (the usual case): every correct sort gives the same array, so entry cDitheringMap[lane] of
    // the sorted list follows from the histogram and the palette's luma order.  Equal lumas (duplicate colours,
    // or distinct colours of equal luma) make the reference QuickSort's tie order matter: exact simulation below.
    int rank = 0;
    bool tie = false;
    if (lane < palsize) {
        const int my = luma_of(lane);
        for (int j = 0; j < palsize; j++) {
            const int o = luma_of(j);
            rank += o < my ? 1 : 0;
            tie |= (o == my) && j != lane;
        }
    }
    const bool any_tie = __ballot(tie) != 0;
    // DeviseBestMixingPlanThomasKnoll for this lane's colour
    const int col = rgb[(long)tile * 64 + lane];
    const int s0 = col & 0xff, s1 = (col >> 8) & 0xff, s2 = (col >> 16) & 0xff;
    int e0 = 0, e1 = 0, e2 = 0;
    unsigned cw[DT_MAXPAL / 4] = {0, 0, 0, 0};  // list histogram, 8-bit fields: index i in word i/4, byte i%4
    for (int c = 0; c < 64; c++) {
        const int t0 = s0 + (e0 * 9) / 100, t1 = s1 + (e1 * 9) / 100, t2 = s2 + (e2 * 9) / 100;
        const int l1 = t0 * 2126 + t1 * 7152 + t2 * 722;
        // l1 = 10000*A + B with floor division (0 <= B < 10000); |t| <= 1700 keeps every product in 24 bits
        const int A = (l1 >= 0 ? l1 : l1 - 9999) / 10000, B = l1 - A * 10000;
        int least = 0x7fffffff, chosen = c & (palsize - 1);
#pragma unroll
        for (int i = 0; i < DT_MAXPAL; i++) {
            if (i < palsize) {
                const int tp = __mul24(t0, pr[i]) + __mul24(t1, pg[i]) + __mul24(t2, pb[i]);
                // trunc((l1 - LumaPal_i)/10000): floor = (A - la) - (B < lb); +1 when negative and inexact
                const int fl = (A - la[i]) - (B < lb[i] ? 1 : 0);
                const int ld = fl + ((fl < 0 && B != lb[i]) ? 1 : 0);
                const int pen = pc[i] - 26 * tp + ((ld * ld) << 5);  // ColorCompare - 13*|t|^2
                if (pen < least) {
                    least = pen;
                    chosen = i;
                }
            }
        }
        if (any_tie) list[c * 64 + lane] = (uint8_t)chosen;  // only the exact sort needs the list
        {
            const unsigned inc = 1u << (8 * (chosen & 3));
#pragma unroll
            for (int q = 0; q < DT_MAXPAL / 4; q++) cw[q] += (chosen >> 2) == q ? inc : 0u;
        }
        int cr = pr[0], cg = pg[0], cb = pb[0];
#pragma unroll
        for (int i = 1; i < DT_MAXPAL; i++)
            if (chosen == i) {
                cr = pr[i];
                cg = pg[i];
                cb = pb[i];
            }
        e0 += s0 - cr;
        e1 += s1 - cg;
        e2 += s2 - cb;
    }
    int px;
    if (!any_tie) {
        __shared__ int s_order[DT_WAVES][DT_MAXPAL];
        if (lane < palsize) s_order[w][rank] = lane;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int want = c_dither_map[lane];
        int acc = 0;
        px = 0;
        bool found = false;
        for (int r = 0; r < palsize; r++) {
            const int idx = s_order[w][r];
            unsigned word = cw[0];
#pragma unroll
            for (int q = 1; q < DT_MAXPAL / 4; q++) word = (idx >> 2) == q ? cw[q] : word;
            acc += (word >> (8 * (idx & 3))) & 0xffu;
            if (!found && acc > want) {
                px = idx;
                found = true;
            }
        }
    } else {  // QuickSort (kmodes.pas:89-136), only for palettes with equal lumas
        lane_quicksort(list, s_stk[w], lane, 63, luma_of);
        px = list[c_dither_map[lane] * 64 + lane];
    }
    tile_mirrors_store(px, lane, tile, palpix, hm, vm);
}

// DitherTile's Yliluoma branch (chkUseTK unchecked, main.pas:2055-2067): per pixel the mixing plan of
// DeviseBestMixingPlanYliluoma in the form the reference build runs -- main.pas:5 defines ASM_DBMP, so on x86-64 the
// SSE block (main.pas:1602-1752) is the algorithm: lanes (r, g, b, luma) of sum += add, add += 1 per tried count t,
// q = (gVecInv[t] * sum) mod 2^32 >> 16 (pmulld, psrld), pen = sum_k w_k (q_k - x_k)^2 mod 2^32 (psubd, pmulld,
// phaddd), w = (13, 13, 13, 32), strict '<' over (palette entry, t) in that order -- then the same luma QuickSort and
// entry (cDitheringMap * count) shr 6 of the sorted list.  One lane per pixel as the Thomas Knoll kernel; a lane's
// list (at most 2 * (mixed - 1) entries, mixed <= DY_MAXMIX) in LDS; gVecInv's rows in LDS.
constexpr int DY_MAXMIX = 64;
constexpr int DY_LIST = 2 * DY_MAXMIX;  // list entries a plan can reach (< cDitheringListLen = 256)

__global__ __launch_bounds__(64 * DT_WAVES) void dither_yl_kernel(const int32_t *__restrict__ rgb,
                                                                  const int32_t *__restrict__ pal_of,
                                                                  const int32_t *__restrict__ palettes,
                                                                  int n_palettes, int palsize, int mixed, int n,
                                                                  uint8_t *__restrict__ palpix,
                                                                  uint8_t *__restrict__ hm, uint8_t *__restrict__ vm) {
    __shared__ uint8_t s_list[DT_WAVES][DY_LIST * 64];      // [entry][lane]
    __shared__ uint16_t s_stk[DT_WAVES][DT_STACK * 64];     // [depth][lane]: first | last << 8
    __shared__ int s_luma[DT_WAVES][DT_MAXPAL];             // LumaPal of the tile's palette
    __shared__ uint32_t s_inv[DY_LIST + 1];                 // gVecInv rows: 65536 div t (main.pas:610-611)
    for (int t = threadIdx.x; t <= DY_LIST; t += blockDim.x) s_inv[t] = t ? 65536u / (uint32_t)t : 0u;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int tile = blockIdx.x * DT_WAVES + w;
    if (tile >= n) return;
    const int p = pal_of[tile];
    uint8_t *list = s_list[w];
    if (p < 0 || p >= n_palettes) {  // invalid input (the host entry rejects it): defined output, no fault
        palpix[(long)tile * 64 + lane] = 0;
        if (lane == 0) hm[tile] = vm[tile] = 0;
        return;
    }
    // PreparePlan: Y2Palette (r, g, b, LumaPal div cLumaDiv), wave-uniform
    uint32_t y0[DT_MAXPAL], y1[DT_MAXPAL], y2[DT_MAXPAL], y3[DT_MAXPAL];
#pragma unroll
    for (int i = 0; i < DT_MAXPAL; i++) {
        const int c = i < palsize ? palettes[(long)p * palsize + i] : 0;
        y0[i] = c & 0xff;
        y1[i] = (c >> 8) & 0xff;
        y2[i] = (c >> 16) & 0xff;
        y3[i] = (y0[i] * 2126u + y1[i] * 7152u + y2[i] * 722u) / 10000u;
    }
    if (lane < DT_MAXPAL) {
        const int c = lane < palsize ? palettes[(long)p * palsize + lane] : 0;
        s_luma[w][lane] = (c & 0xff) * 2126 + ((c >> 8) & 0xff) * 7152 + ((c >> 16) & 0xff) * 722;
    }
    const int col = rgb[(long)tile * 64 + lane];
    const uint32_t x0 = col & 0xff, x1 = (col >> 8) & 0xff, x2 = (col >> 16) & 0xff;
    const uint32_t x3 = (x0 * 2126u + x1 * 7152u + x2 * 722u) / 10000u;
    uint32_t so0 = 0, so1 = 0, so2 = 0, so3 = 0;
    int pc = 0;
    while (pc < mixed) {
        const int mt = pc == 0 ? 1 : pc;
        uint32_t least = 0xffffffffu;  // every pen < 2^32 beats the asm's initial 2^63 - 1: the first one is taken
        bool any = false;
        int chosen = 0, chosen_t = pc + 1;
        for (int i = 0; i < palsize; i++) {
            uint32_t s0 = so0, s1 = so1, s2 = so2, s3 = so3;
            uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
            for (int k = 0; k < DT_MAXPAL; k++)
                if (k == i) {
                    a0 = y0[k];
                    a1 = y1[k];
                    a2 = y2[k];
                    a3 = y3[k];
                }
            for (int t = pc + 1; t <= pc + mt; t++) {
                s0 += a0; s1 += a1; s2 += a2; s3 += a3;
                a0 += 1u; a1 += 1u; a2 += 1u; a3 += 1u;
                const uint32_t inv = s_inv[t];
                const uint32_t d0 = ((inv * s0) >> 16) - x0, d1 = ((inv * s1) >> 16) - x1;
                const uint32_t d2 = ((inv * s2) >> 16) - x2, d3 = ((inv * s3) >> 16) - x3;
                const uint32_t pen = (d0 * d0) * 13u + (d1 * d1) * 13u + (d2 * d2) * 13u + (d3 * d3) * 32u;
                if (!any || pen < least) {
                    any = true;
                    least = pen;
                    chosen = i;
                    chosen_t = t;
                }
            }
        }
        const int amount = min(chosen_t - pc, 256 - pc);
        for (int k = 0; k < amount; k++) list[(pc + k) * 64 + lane] = (uint8_t)chosen;
        pc += amount;
        uint32_t c0 = y0[0], c1 = y1[0], c2 = y2[0], c3 = y3[0];
#pragma unroll
        for (int k = 1; k < DT_MAXPAL; k++)
            if (k == chosen) {
                c0 = y0[k];
                c1 = y1[k];
                c2 = y2[k];
                c3 = y3[k];
            }
        so0 += c0 * (uint32_t)amount;
        so1 += c1 * (uint32_t)amount;
        so2 += c2 * (uint32_t)amount;
        so3 += c3 * (uint32_t)amount;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    auto luma_of = [&](int v) { return s_luma[w][v]; };  // LumaPal[v] (PlanCompareLuma)
    lane_quicksort(list, s_stk[w], lane, pc - 1, luma_of);
    const int px = list[((c_dither_map[lane] * pc) >> 6) * 64 + lane];
    tile_mirrors_store(px, lane, tile, palpix, hm, vm);
}

static bool dither_args_ok(int n, const void *rgb, const void *pal_of, const void *palettes, int n_palettes,
                           int palsize, int mixed, const void *palpix, const void *hm, const void *vm) {
    if (n < 0 || n_palettes <= 0 || palsize <= 0 || palsize > DT_MAXPAL ||
        (n > 0 && (!rgb || !pal_of || !palettes || !palpix || !hm || !vm))) {
        set_error("dither: invalid arguments (palette size 1..16)");
        return false;
    }
    if (mixed == 0 && (palsize & (palsize - 1))) {
        set_error("dither: invalid arguments (Thomas Knoll mixing: palette size a power of two <= 16)");
        return false;
    }
    if (mixed < 0 || mixed > DY_MAXMIX) {
        set_error("dither: Yliluoma mixed colours must be 1..64");
        return false;
    }
    return true;
}

// mixed = 0: Thomas Knoll (the default); 1..64: Yliluoma with Y2MixedColors = mixed
int dither_tiles_dev(int n, const int32_t *d_rgb, const int32_t *d_pal_of, const int32_t *d_palettes, int n_palettes,
                     int palsize, int mixed, uint8_t *d_palpix, uint8_t *d_hm, uint8_t *d_vm, hipStream_t stream) {
    if (!dither_args_ok(n, d_rgb, d_pal_of, d_palettes, n_palettes, palsize, mixed, d_palpix, d_hm, d_vm)) return -1;
    if (n == 0) return 0;
    KTimer tm("dither", stream);
    if (mixed == 0)
        hipLaunchKernelGGL(dither_tk_kernel, dim3((n + DT_WAVES - 1) / DT_WAVES), dim3(64 * DT_WAVES), 0, stream, d_rgb,
                           d_pal_of, d_palettes, n_palettes, palsize, n, d_palpix, d_hm, d_vm);
    else
        hipLaunchKernelGGL(dither_yl_kernel, dim3((n + DT_WAVES - 1) / DT_WAVES), dim3(64 * DT_WAVES), 0, stream, d_rgb,
                           d_pal_of, d_palettes, n_palettes, palsize, mixed, n, d_palpix, d_hm, d_vm);
    TILER_HIP_CHECK(hipGetLastError());
    return 0;
}

int dither_tiles_host(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes, int n_palettes,
                      int palsize, int mixed, uint8_t *palpix, uint8_t *hm, uint8_t *vm) {
    if (!dither_args_ok(n, rgb, pal_of, palettes, n_palettes, palsize, mixed, palpix, hm, vm)) return -1;
    for (int i = 0; i < n; i++)
        if (pal_of[i] < 0 || pal_of[i] >= n_palettes) {
            set_error("dither: palette index out of range");
            return -1;
        }
    if (n == 0) return 0;
    const size_t b_rgb = (size_t)n * 256, b_po = (size_t)n * 4, b_pal = (size_t)n_palettes * palsize * 4;
    const size_t b_px = (size_t)n * 64;
    char *buf = nullptr;
    TILER_HIP_CHECK(hipMalloc((void **)&buf, b_rgb + b_po + b_pal + b_px + 2 * (size_t)n + 64));
    int32_t *d_rgb = (int32_t *)buf, *d_po = (int32_t *)(buf + b_rgb), *d_pal = (int32_t *)(buf + b_rgb + b_po);
    uint8_t *d_px = (uint8_t *)(buf + b_rgb + b_po + b_pal), *d_hm = d_px + b_px, *d_vm = d_hm + n;
    hipStream_t st = nullptr;
    int rc = -1;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        (void)hipFree(buf);
        set_error("dither: stream creation failed");
        return -1;
    }
    do {
        if (hipMemcpyAsync(d_rgb, rgb, b_rgb, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (hipMemcpyAsync(d_po, pal_of, b_po, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (hipMemcpyAsync(d_pal, palettes, b_pal, hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (dither_tiles_dev(n, d_rgb, d_po, d_pal, n_palettes, palsize, mixed, d_px, d_hm, d_vm, st)) break;
        if (hipMemcpyAsync(palpix, d_px, b_px, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipMemcpyAsync(hm, d_hm, n, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipMemcpyAsync(vm, d_vm, n, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipStreamSynchronize(st) != hipSuccess) break;
        rc = 0;
    } while (0);
    if (rc) set_error(std::string("dither: HIP failure: ") + hipGetErrorString(hipGetLastError()));
    (void)hipStreamDestroy(st);
    (void)hipFree(buf);
    return rc;
}

}  // namespace tiler
