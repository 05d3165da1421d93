// tiler_common.hpp -- shared host/device helpers for libANN.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace tiler {

// thread-local last error (tiler_last_error)
void set_error(const std::string &msg);
const char *last_error();

// first-use initialisation of the device + host-computed LUTs shared by every kernel
bool ensure_init();

struct Luts {
    double *d_gamma = nullptr;  // [3][256]: row 0 = i/255.0, rows 1,2 = power(i/255, gGamma[g])
    double *d_dct = nullptr;    // [4096] gDCTLut (main.pas:615-623), computed on the host
    double *d_qmul = nullptr;   // [3][64] cDCTQuantization (main.pas:63-98) = 4/sqrt(q)
    double *d_ratio = nullptr;  // [64] cUVRatio (main.pas:3000-3009)
    double *d_lab_lin = nullptr;  // [3][256]: RGBToLAB's linearised channel of GammaCorrect rows (main.pas:2715-2721)
    double haar_f = 0.0;        // 1.0/sqrt(2.0) (main.pas:2816)
    double u_mul = 0.0;         // 0.5 / (1.0 - 722/10000)   (main.pas:2675)
    double v_mul = 0.0;         // 0.5 / (1.0 - 2126/10000)  (main.pas:2676)
};
const Luts &luts();

// Device blocks of the search indexes (devmem.hip): dmalloc hands out an idle cached block of about the size, else
// hipMalloc; dfree files the block for reuse -- the caller guarantees that no GPU work still uses it (hipFree's
// implicit device synchronisation made explicit: the destroy paths synchronise once); dfree_sync synchronises first.
hipError_t dmalloc(void **p, size_t bytes);
void dfree(void *p);
void dfree_sync(void *p);
// non-blocking streams of the current device, reused (stream_put synchronises the stream first)
hipError_t stream_get(hipStream_t *s);
void stream_put(hipStream_t s);
// 16-byte pinned host slots (per-index tier-2 counters), reused
int *pinned_slot();
void pinned_slot_free(int *p);

// Kernel timing (tiler_timing_*): RAII scope that records a HIP event pair on the launch stream.
bool timing_enabled();
struct KTimer {
    KTimer(const char *name, hipStream_t s);
    ~KTimer();
    const char *name;
    hipStream_t stream;
    void *ev_a = nullptr, *ev_b = nullptr;
};

}  // namespace tiler

#define TILER_HIP_CHECK(expr)                                                                   \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess) {                                                                 \
            tiler::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));                \
            return -1;                                                                          \
        }                                                                                       \
    } while (0)

#define TILER_HIP_CHECK_NULL(expr)                                                              \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess) {                                                                 \
            tiler::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));                \
            return nullptr;                                                                     \
        }                                                                                       \
    } while (0)
