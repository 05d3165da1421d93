// ann_api.hip -- extern "C" entry points of libANN.so (include/tiler_ann.h).
//
// The ANN.dll surface (extern.pas:63-67) plus batched / device-resident extensions.  Host-buffer
// entry points stage through a per-handle HIP stream; *_dev entry points run on the caller's
// stream with HBM pointers (the benchmarked path).  No CPU compute path exists: without a gfx950
// device every entry point fails with -1 / NULL and tiler_last_error().
#include <float.h>
#include <math.h>
#include <string.h>

#include <atomic>
#include <algorithm>
#include <chrono>
#include <thread>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/tiler_ann.h"
#include "dither.hpp"
#include "palette.hpp"
#include "prepare.hpp"
#include "kmeans.hpp"
#include "detmath.hpp"
#include "keyframes.hpp"
#include "kmodes.hpp"
#include "nn_search.hpp"
#include "orbit.hpp"
#include "psyv.hpp"
#include "smooth.hpp"

namespace tiler {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }
const char *last_error() { return g_err.c_str(); }

static std::mutex g_init_mu;
static bool g_ready = false;
static bool g_all = false;     // tiler_init(TILER_ALL_DEVICES): every visible gfx950 device bound
static int g_device = 0;       // the primary device (the only one unless g_all)
static constexpr int MAX_DEV = 64;
static bool g_bound[MAX_DEV] = {};
static Luts g_luts[MAX_DEV];
static double g_gamma[2] = {2.0, 0.6};
// live dataset bytes of the handles on each device: ann_kdtree_create places a new handle on the least loaded one
static std::mutex g_place_mu;
static long long g_dev_load[MAX_DEV] = {};

static bool bound(int d) { return d >= 0 && d < MAX_DEV && g_bound[d]; }
const Luts &luts() {  // the current device's tables (every bound device has its own copy)
    int d = -1;
    (void)hipGetDevice(&d);
    return g_luts[bound(d) ? d : g_device];
}

// ---- kernel timing --------------------------------------------------------------------------
struct TimedPair {
    std::string name;
    hipEvent_t a, b;
};
static std::mutex g_time_mu;
static std::vector<TimedPair> g_times;
static bool g_timing = false;
bool timing_enabled() { return g_timing; }
KTimer::KTimer(const char *n, hipStream_t s) : name(n), stream(s) {
    if (!g_timing || !n) return;  // a null name: no timer
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess) return;
    if (hipEventCreate(&b) != hipSuccess) {
        (void)hipEventDestroy(a);
        return;
    }
    ev_a = a;
    ev_b = b;
    (void)hipEventRecord(a, s);
}
KTimer::~KTimer() {
    if (!ev_a) return;
    (void)hipEventRecord((hipEvent_t)ev_b, stream);
    std::lock_guard<std::mutex> lk(g_time_mu);
    g_times.push_back({name, (hipEvent_t)ev_a, (hipEvent_t)ev_b});
}

// InitLuts main.pas:592-642; constants main.pas:63-98, 2675-2676, 2816, 3000-3009 -- all on the host,
// identical expressions to the CPU restatement, so device and oracle share the same bits.
static int upload_gamma_lut(Luts &L) {
    std::vector<double> g(3 * 256), lin(3 * 256);
    for (int gi = -1; gi <= 1; gi++)
        for (int i = 0; i < 256; i++) g[(gi + 1) * 256 + i] = (gi >= 0) ? pow(i / 255.0, g_gamma[gi]) : i / 255.0;
    for (int k = 0; k < 3 * 256; k++) {  // RGBToLAB main.pas:2719-2721 (FPC power = exp(2.4 * ln(.)), detmath.hpp)
        const double v = g[k];
        lin[k] = v > 0.04045 ? fpc_power_frac((v + 0.055) / 1.055, 2.4) : v / 12.92;
    }
    TILER_HIP_CHECK(hipMemcpy(L.d_gamma, g.data(), g.size() * sizeof(double), hipMemcpyHostToDevice));
    TILER_HIP_CHECK(hipMemcpy(L.d_lab_lin, lin.data(), lin.size() * sizeof(double), hipMemcpyHostToDevice));
    return 0;
}

static int build_luts(Luts &L) {
    static const int qden[3][64] = {
        {16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
         14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
         49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99},
        {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 112, 24, 26, 56, 99, 99, 99, 112, 128,
         47, 66, 99, 99, 99, 112, 128, 144, 99, 99, 99, 99, 112, 128, 144, 160, 99, 99, 99, 112, 128, 144, 160, 176,
         99, 99, 112, 128, 144, 160, 176, 192, 99, 112, 128, 144, 160, 176, 192, 208},
        {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 112, 24, 26, 56, 99, 99, 99, 112, 128,
         47, 66, 99, 99, 99, 112, 128, 144, 99, 99, 99, 99, 112, 128, 144, 160, 99, 99, 99, 112, 128, 144, 160, 176,
         99, 99, 112, 128, 144, 160, 176, 192, 99, 112, 128, 144, 160, 176, 192, 208}};
    std::vector<double> dct(4096), qm(192), ratio(64);
    int i = 0;
    for (int v = 0; v < 8; v++)
        for (int u = 0; u < 8; u++)
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) {
                    double a = (((double)x + 0.5) * (double)u) * M_PI / 16.0;
                    double b = (((double)y + 0.5) * (double)v) * M_PI / 16.0;
                    dct[i++] = cos(a) * cos(b);
                }
    for (int c = 0; c < 3; c++)
        for (int k = 0; k < 64; k++) qm[c * 64 + k] = 4.0 / sqrt((double)qden[c][k]);
    const double sh = sqrt(0.5);
    for (int v = 0; v < 8; v++)
        for (int u = 0; u < 8; u++) ratio[v * 8 + u] = (u == 0 && v == 0) ? 0.5 : ((u == 0 || v == 0) ? sh : 1.0);
    TILER_HIP_CHECK(hipMalloc((void **)&L.d_gamma, 3 * 256 * sizeof(double)));
    TILER_HIP_CHECK(hipMalloc((void **)&L.d_dct, 4096 * sizeof(double)));
    TILER_HIP_CHECK(hipMalloc((void **)&L.d_qmul, 192 * sizeof(double)));
    TILER_HIP_CHECK(hipMalloc((void **)&L.d_ratio, 64 * sizeof(double)));
    TILER_HIP_CHECK(hipMalloc((void **)&L.d_lab_lin, 3 * 256 * sizeof(double)));
    TILER_HIP_CHECK(hipMemcpy(L.d_dct, dct.data(), 4096 * sizeof(double), hipMemcpyHostToDevice));
    TILER_HIP_CHECK(hipMemcpy(L.d_qmul, qm.data(), 192 * sizeof(double), hipMemcpyHostToDevice));
    TILER_HIP_CHECK(hipMemcpy(L.d_ratio, ratio.data(), 64 * sizeof(double), hipMemcpyHostToDevice));
    L.haar_f = 1.0 / sqrt(2.0);
    L.u_mul = 0.5 / (1.0 - 722.0 / 10000.0);
    L.v_mul = 0.5 / (1.0 - 2126.0 / 10000.0);
    return upload_gamma_lut(L);
}

static int bind_device(int device) {
    hipDeviceProp_t prop;
    TILER_HIP_CHECK(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error(std::string("tiler: device ") + std::to_string(device) + " is " + prop.gcnArchName +
                  ", libANN.so is built for gfx950 only");
        return -1;
    }
    TILER_HIP_CHECK(hipSetDevice(device));
    if (build_luts(g_luts[device])) return -1;
    g_bound[device] = true;
    return 0;
}

static int init_locked(int device) {
    if (g_ready) {
        if (device == TILER_ALL_DEVICES ? g_all : (!g_all && device == g_device)) return 0;
        // already bound (explicitly, or implicitly to device 0 by an earlier call): handles, LUTs and scratch live
        // on that device (those devices), so a silent switch would run later calls on the wrong GPU
        set_error("tiler_init: the library is already bound to " +
                  (g_all ? std::string("all devices") : "device " + std::to_string(g_device)) + "; call tiler_init(" +
                  std::to_string(device) + ") before any other entry point");
        return -1;
    }
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        set_error("tiler: no HIP device visible (libANN.so runs on MI355X / gfx950 only, no CPU path)");
        return -1;
    }
    count = std::min(count, MAX_DEV);
    if (device == TILER_ALL_DEVICES) {
        // one process driving every GPU of the node (the reference encoder is one process, main.pas:972): each
        // device gets its own tables; handles are placed per device (ann_kdtree_create) and peers can copy directly
        for (int d = 0; d < count; d++)
            if (bind_device(d)) return -1;
        for (int a = 0; a < count; a++) {
            TILER_HIP_CHECK(hipSetDevice(a));
            for (int b = 0; b < count; b++) {
                int ok = 0;
                if (a != b && hipDeviceCanAccessPeer(&ok, a, b) == hipSuccess && ok) {
                    const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
                    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
                }
            }
        }
        g_all = true;
        g_device = 0;
        TILER_HIP_CHECK(hipSetDevice(0));
        g_ready = true;
        return 0;
    }
    if (device < 0 || device >= count) {
        set_error("tiler: device index out of range");
        return -1;
    }
    if (bind_device(device)) return -1;
    g_device = device;
    g_ready = true;
    return 0;
}

// Every entry point: bind on first use; the calling thread's current device is kept when the library is bound to it
// (all devices: the caller selects one with hipSetDevice, or the entry point follows its handle), else the primary.
bool ensure_init() {
    std::lock_guard<std::mutex> lk(g_init_mu);
    if (!g_ready && init_locked(0)) return false;
    int cur = -1;
    if (g_all && hipGetDevice(&cur) == hipSuccess && bound(cur)) return true;
    return hipSetDevice(g_device) == hipSuccess;
}

// the device a pointer lives on (device memory; host / unknown pointers: the current device)
static int ptr_device(const void *p) {
    int cur = g_device;
    (void)hipGetDevice(&cur);
    if (!g_all || !p) return cur;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return cur;
    }
    return (a.type == hipMemoryTypeDevice && bound(a.device)) ? a.device : cur;
}

// runs the scope on device d and restores the caller's current device afterwards
struct DevScope {
    int prev = -1;
    explicit DevScope(int d) {
        int c = -1;
        if (hipGetDevice(&c) == hipSuccess && c != d && hipSetDevice(d) == hipSuccess) prev = c;
    }
    ~DevScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// least-loaded device for a new dataset of `bytes`: the placement rule of ann_kdtree_create (ties: lowest device)
static int pick_device(const long long *load, int ndev) {
    int best = 0;
    for (int d = 1; d < ndev; d++)
        if (load[d] < load[best]) best = d;
    return best;
}
static int place_handle(long long bytes) {
    if (!g_all) return g_device;
    std::lock_guard<std::mutex> lk(g_place_mu);
    long long load[MAX_DEV];
    int map[MAX_DEV], n = 0;
    for (int d = 0; d < MAX_DEV; d++)
        if (g_bound[d]) {
            load[n] = g_dev_load[d];
            map[n++] = d;
        }
    const int d = map[pick_device(load, n)];
    g_dev_load[d] += bytes;
    return d;
}
static void unplace_handle(int dev, long long bytes) {
    std::lock_guard<std::mutex> lk(g_place_mu);
    if (dev >= 0 && dev < MAX_DEV) g_dev_load[dev] -= bytes;
}

}  // namespace tiler

using namespace tiler;

// Concurrent single-query callers of one handle (the reference's pattern: ann_kdtree_search per tile from every
// ProcThreadPool worker, main.pas:4027 / 972, and ann_kdtree_search_multi per item, main.pas:3830) are coalesced: a
// caller queues its query; the first caller that finds no batch in flight becomes the leader, takes every queued query
// of its k (callers that arrived while the previous batch ran), searches them as ONE batch and wakes each caller on its
// own slot.  Batching never changes an answer (every query's result is exact and independent of the others).  The
// leader stops once its own query is answered and hands the queue to a waiting caller.
struct CombineReq {
    const float *q = nullptr;
    int k = 1;
    int *idx = nullptr;
    float *err = nullptr;
    int rc = 0;
    bool taken = false;             // in a batch (set by its leader under Combiner::m)
    std::atomic<bool> done{false};  // answered: idx / err / rc / msg written before the release store
    std::string msg;
};
// One batch in flight: its own stream, pinned staging, device buffers and search scratch, so that several batches can be
// in flight on one handle (the second one's upload and kernels overlap the first one's; only small-batch scans run
// concurrently: they touch nothing of the index but its read-only data and the scratch swapped in for them).
struct CombineSlot {
    hipStream_t stream = nullptr;
    float *h_q = nullptr;
    int *h_res = nullptr;  // [2][cap_r / 2]: indices, then distances
    float *d_q = nullptr;
    int *d_res = nullptr;
    size_t cap_q = 0, cap_r = 0;
    SearchScratch scratch;
    bool busy = false;
};
#ifndef ANN_COMBINE_SPIN_US
#define ANN_COMBINE_SPIN_US 200  // a caller whose query is in a batch in flight spins this long before sleeping
                                 // (r06v, profiles/r06/v_percall_spin_ab.txt: C3 per-tile calls 85k -> 98k/s, 0 vs 200 us)
#endif
#ifndef ANN_COMBINE_SLOTS
#define ANN_COMBINE_SLOTS 3  // batches of one handle in flight at once (r06t, profiles/r06/t_percall_slots_ab.txt: 2 -> 3
                             // C3 per-tile calls 89k -> 95k/s, 65k-row plain handle 106k -> 120k; 4 slower)
#endif
struct Combiner {
    static constexpr int SLOTS = ANN_COMBINE_SLOTS;
    std::mutex m;
    std::condition_variable cv;
    std::deque<CombineReq *> pending;
    CombineSlot slot[SLOTS];
    long long batches = 0, calls = 0;  // counters (tiler_combine_stats)
    int max_batch = 0;
};

struct ann_kdtree {
    NNIndex *ix = nullptr;
    Combiner comb;
    hipStream_t stream = nullptr;
    float *d_q = nullptr;
    int *d_idx = nullptr;
    float *d_err = nullptr;
    size_t cap = 0;
    int32_t *d_rgb = nullptr, *d_mt = nullptr, *d_mp = nullptr;
    uint8_t *d_mh = nullptr, *d_mv = nullptr;
    size_t cap_ft = 0;
    void *d_pri = nullptr;        // kd_pri_search heap scratch (ann_kdtree_pri_search)
    size_t cap_pri = 0;
    void *d_pri_aux = nullptr;    // kd_pri_resolve scratch + the replay flags
    size_t cap_pri_aux = 0;
    PrepScratch *prep = nullptr;  // tiler_prepare_frame_tiling_dev scratch (on the global dataset's handle)
    int dev = 0;                  // the device the handle's index, stream and buffers live on
    hipEvent_t maps_ev = nullptr; // recorded after tiler_prepare_frame_tiling_dev wrote the TRTo maps (on its stream)
    hipEvent_t ready_ev = nullptr; // recorded after the rows copy and index build of ann_kdtree_create_dev_ex, on the
                                   // caller's stream when one was passed (replica_of waits for it before a peer copy)
    long long placed = 0;         // dataset bytes counted in g_dev_load[dev]
    // copies of this handle's index on other devices (tiler_kdtree_replicate, or made on first use by a device entry
    // point whose buffers live there): rows peer-copied over xGMI, the same index built there
    std::mutex rep_mu;
    ann_kdtree *rep[MAX_DEV] = {};
};

static void handle_free(ann_kdtree *t);

static int ensure_io(ann_kdtree *t, size_t nq, int d, int k) {
    const size_t need = nq * (size_t)std::max(d, k);
    if (need <= t->cap) return 0;
    hipFree(t->d_q);
    hipFree(t->d_idx);
    hipFree(t->d_err);
    TILER_HIP_CHECK(hipMalloc((void **)&t->d_q, need * sizeof(float)));
    TILER_HIP_CHECK(hipMalloc((void **)&t->d_idx, need * sizeof(int)));
    TILER_HIP_CHECK(hipMalloc((void **)&t->d_err, need * sizeof(float)));
    t->cap = need;
    return 0;
}

extern "C" {

int tiler_init(int device) {
    std::lock_guard<std::mutex> lk(g_init_mu);
    return init_locked(device);
}

int tiler_shutdown(void) { return 0; }

int tiler_timing_enable(int on) {
    g_timing = on != 0;
    return 0;
}

double tiler_timing_get(const char *kernel, int *launches) {
    std::lock_guard<std::mutex> lk(g_time_mu);
    double ms = 0.0;
    int cnt = 0;
    for (auto &p : g_times) {
        if (p.name != kernel) continue;
        float e = 0.0f;
        if (hipEventSynchronize(p.b) != hipSuccess || hipEventElapsedTime(&e, p.a, p.b) != hipSuccess) {
            set_error("tiler_timing_get: event query failed");
            return -1.0;
        }
        ms += e;
        cnt++;
    }
    if (launches) *launches = cnt;
    return ms;
}

int tiler_timing_reset(void) {
    std::lock_guard<std::mutex> lk(g_time_mu);
    for (auto &p : g_times) {
        (void)hipEventSynchronize(p.b);
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    g_times.clear();
    return 0;
}

const char *tiler_last_error(void) { return tiler::last_error(); }

int tiler_set_gamma(double g0, double g1) {
    if (!ensure_init()) return -1;
    std::lock_guard<std::mutex> lk(g_init_mu);
    g_gamma[0] = g0;
    g_gamma[1] = g1;
    for (int d = 0; d < MAX_DEV; d++)
        if (g_bound[d]) {
            DevScope ds(d);
            if (upload_gamma_lut(g_luts[d])) return -1;
        }
    return 0;
}

static bool split_ok(int bs, int split, const char *who) {
    if (bs < 1) {
        set_error(std::string(who) + ": bucket size must be >= 1");
        return false;
    }
    if (split != KD_SPLIT_STD && split != KD_SPLIT_INDEX_ORDER) {
        // the reference only ever passes ANN_KD_STD (main.pas:3779,3961); other ANN rules shape other trees
        set_error(std::string(who) + ": split rule not supported (ANN_KD_STD = 0, or 100 = ties to the lowest index)");
        return false;
    }
    return true;
}

ann_kdtree *ann_kdtree_create(float **pa, int n, int dd, int bs, int split) {
    if (!ensure_init()) return nullptr;
    if (n < 0 || dd <= 0 || (n > 0 && !pa)) {
        set_error("ann_kdtree_create: invalid arguments");
        return nullptr;
    }
    if (!split_ok(bs, split, "ann_kdtree_create")) return nullptr;
    std::vector<float> h((size_t)n * dd);
    for (int i = 0; i < n; i++) {
        if (!pa[i]) {
            set_error("ann_kdtree_create: null row pointer");
            return nullptr;
        }
        memcpy(&h[(size_t)i * dd], pa[i], sizeof(float) * dd);
    }
    // host rows: the handle goes to the least loaded bound device (one device unless tiler_init(TILER_ALL_DEVICES))
    const long long bytes = (long long)h.size() * 4;
    const int dev = place_handle(bytes);
    DevScope ds(dev);
    ann_kdtree *t = new ann_kdtree();
    t->dev = dev;
    t->placed = bytes;
    float *d_rows = nullptr;
    if (stream_get(&t->stream) != hipSuccess ||
        dmalloc((void **)&d_rows, std::max<size_t>(1, h.size()) * sizeof(float)) != hipSuccess ||
        (n > 0 && hipMemcpyAsync(d_rows, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice, t->stream) !=
                      hipSuccess)) {
        set_error("ann_kdtree_create: device allocation or copy failed");
        if (d_rows) dfree_sync(d_rows);
        handle_free(t);
        return nullptr;
    }
    t->ix = nn_index_create_dev(d_rows, n, dd, bs, split, t->stream);
    if (!t->ix) {
        handle_free(t);
        return nullptr;
    }
    return t;
}

ann_kdtree *ann_kdtree_create_dev(const float *d_rows_in, int n, int dd, void *stream) {
    return ann_kdtree_create_dev_ex(d_rows_in, n, dd, 1, KD_SPLIT_STD, stream);
}

ann_kdtree *ann_kdtree_create_dev_ex(const float *d_rows_in, int n, int dd, int bs, int split, void *stream) {
    if (!ensure_init()) return nullptr;
    if (n < 0 || dd <= 0 || (n > 0 && !d_rows_in)) {
        set_error("ann_kdtree_create_dev: invalid arguments");
        return nullptr;
    }
    if (!split_ok(bs, split, "ann_kdtree_create_dev")) return nullptr;
    const int dev = ptr_device(d_rows_in);  // device rows: the handle lives where they are
    DevScope ds(dev);
    ann_kdtree *t = new ann_kdtree();
    t->dev = dev;
    t->placed = (long long)n * dd * 4;
    {
        std::lock_guard<std::mutex> lk(g_place_mu);
        g_dev_load[dev] += t->placed;
    }
    // every failure below releases the handle (handle_free also takes its bytes back out of g_dev_load)
    float *d_rows = nullptr;
    const size_t bytes = (size_t)n * dd * sizeof(float);
    const bool ok_stream = stream_get(&t->stream) == hipSuccess;
    hipStream_t s = stream ? (hipStream_t)stream : t->stream;
    if (!ok_stream || dmalloc((void **)&d_rows, std::max<size_t>(4, bytes)) != hipSuccess ||
        (n > 0 && hipMemcpyAsync(d_rows, d_rows_in, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)) {
        set_error("ann_kdtree_create_dev: device allocation or copy failed");
        if (d_rows) dfree_sync(d_rows);
        handle_free(t);
        return nullptr;
    }
    t->ix = nn_index_create_dev(d_rows, n, dd, bs, split, s);
    if (!t->ix) {
        handle_free(t);
        return nullptr;
    }
    // the rows copy and the index build are queued on s: a replica made from another device must wait for them
    if (hipEventCreateWithFlags(&t->ready_ev, hipEventDisableTiming) != hipSuccess || hipEventRecord(t->ready_ev, s) != hipSuccess) {
        set_error("ann_kdtree_create_dev: event record failed");
        handle_free(t);
        return nullptr;
    }
    return t;
}

// release a handle (its replicas first); the caller's device is restored
static void handle_free(ann_kdtree *t) {
    if (!t) return;
    for (int d = 0; d < MAX_DEV; d++)
        if (t->rep[d]) handle_free(t->rep[d]);
    DevScope ds(t->dev);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    nn_index_destroy(t->ix);
    (void)hipFree(t->d_q);
    (void)hipFree(t->d_idx);
    (void)hipFree(t->d_err);
    (void)hipFree(t->d_rgb);
    (void)hipFree(t->d_mt);
    (void)hipFree(t->d_mp);
    (void)hipFree(t->d_mh);
    (void)hipFree(t->d_mv);
    (void)hipFree(t->d_pri);
    (void)hipFree(t->d_pri_aux);
    if (t->prep) {
        prep_scratch_free(t->prep);
        delete t->prep;
    }
    for (CombineSlot &cs : t->comb.slot) {
        if (cs.stream) (void)hipStreamSynchronize(cs.stream);
        nn_scratch_free(cs.scratch);
        (void)hipFree(cs.d_q);
        (void)hipFree(cs.d_res);
        (void)hipHostFree(cs.h_q);
        (void)hipHostFree(cs.h_res);
        stream_put(cs.stream);
    }
    if (t->maps_ev) (void)hipEventDestroy(t->maps_ev);
    if (t->ready_ev) (void)hipEventDestroy(t->ready_ev);
    stream_put(t->stream);  // (synchronised first) back to the device's pool
    unplace_handle(t->dev, t->placed);
    delete t;
}

void ann_kdtree_destroy(ann_kdtree *t) { handle_free(t); }

// the copy of t's index on device dev (t itself when it lives there), made on first use: rows (and the TRTo maps)
// peer-copied from t's device over xGMI, the index built there exactly as at create (same rows, same kd-tree)
static std::atomic<int> g_force_replicas{0};  // tiler_debug_force_replicas: copies even on the handle's own device
static ann_kdtree *replica_of(ann_kdtree *t, int dev) {
    if (!t || (t->dev == dev && !g_force_replicas.load())) return t;
    if (!bound(dev)) {
        set_error("tiler: device " + std::to_string(dev) + " is not bound (tiler_init(-1) binds every device)");
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(t->rep_mu);
    if (t->rep[dev]) return t->rep[dev];
    NNIndex *src = t->ix;
    std::lock_guard<std::mutex> ilk(src->mu);
    DevScope ds(dev);
    ann_kdtree *r = new ann_kdtree();
    r->dev = dev;
    r->placed = (long long)src->n * src->d * 4;
    {
        std::lock_guard<std::mutex> pl(g_place_mu);
        g_dev_load[dev] += r->placed;
    }
    float *d_rows = nullptr;
    const size_t bytes = (size_t)src->n * src->d * sizeof(float);
    // the source is complete before it is copied: its own stream (creates return with the index queued on it), the
    // caller's stream of a device create (ready_ev) and of the Prepare that wrote its TRTo maps (maps_ev), its searches
    if (hipStreamSynchronize(t->stream) != hipSuccess || (t->ready_ev && hipEventSynchronize(t->ready_ev) != hipSuccess) ||
        (t->maps_ev && hipEventSynchronize(t->maps_ev) != hipSuccess) ||
        (src->done_event && hipEventSynchronize(src->done_event) != hipSuccess) ||
        stream_get(&r->stream) != hipSuccess ||
        dmalloc((void **)&d_rows, std::max<size_t>(4, bytes)) != hipSuccess ||
        (bytes && hipMemcpyPeerAsync(d_rows, dev, src->d_rows, t->dev, bytes, r->stream) != hipSuccess)) {
        set_error("tiler: replica allocation or peer copy failed");
        if (d_rows) dfree_sync(d_rows);
        handle_free(r);
        return nullptr;
    }
    r->ix = nn_index_create_dev(d_rows, src->n, src->d, src->bs, src->split, r->stream);
    if (!r->ix) {
        handle_free(r);
        return nullptr;
    }
    if (src->d_tr_tile) {
        const size_t n = std::max(1, src->n);
        NNIndex *ix = r->ix;
        if (dmalloc((void **)&ix->d_tr_tile, n * 4) != hipSuccess || dmalloc((void **)&ix->d_tr_pal, n * 4) != hipSuccess ||
            dmalloc((void **)&ix->d_tr_attr, n) != hipSuccess ||
            hipMemcpyPeerAsync(ix->d_tr_tile, dev, src->d_tr_tile, t->dev, (size_t)src->n * 4, r->stream) != hipSuccess ||
            hipMemcpyPeerAsync(ix->d_tr_pal, dev, src->d_tr_pal, t->dev, (size_t)src->n * 4, r->stream) != hipSuccess ||
            hipMemcpyPeerAsync(ix->d_tr_attr, dev, src->d_tr_attr, t->dev, (size_t)src->n, r->stream) != hipSuccess) {
            set_error("tiler: replica maps copy failed");
            handle_free(r);
            return nullptr;
        }
    }
    if (hipStreamSynchronize(r->stream) != hipSuccess) {
        set_error("tiler: replica build failed");
        handle_free(r);
        return nullptr;
    }
    t->rep[dev] = r;
    return r;
}

// the handle to run a device-buffer call on: t's copy on the device of the call's buffer p
static ann_kdtree *handle_for(ann_kdtree *t, const void *p) { return g_all ? replica_of(t, ptr_device(p)) : t; }

int tiler_kdtree_replicate(ann_kdtree *t, int device) {
    if (!t || !t->ix) {
        set_error("tiler_kdtree_replicate: null handle");
        return -1;
    }
    if (!ensure_init()) return -1;
    for (int d = 0; d < MAX_DEV; d++)
        if (g_bound[d] && (device == TILER_ALL_DEVICES || device == d) && !replica_of(t, d)) return -1;
    if (device != TILER_ALL_DEVICES && !bound(device)) {
        set_error("tiler_kdtree_replicate: device not bound");
        return -1;
    }
    return 0;
}

int tiler_debug_force_replicas(int on) {
    g_force_replicas.store(on != 0);
    return 0;
}

int tiler_kdtree_device(ann_kdtree *t) {
    if (!t) {
        set_error("tiler_kdtree_device: null handle");
        return -1;
    }
    return t->dev;
}

int tiler_device_count(void) {
    if (!ensure_init()) return -1;
    int n = 0;
    for (int d = 0; d < MAX_DEV; d++) n += g_bound[d] ? 1 : 0;
    return n;
}

int tiler_placement_plan(int ndev, const int64_t *bytes, int n, int32_t *dev_out) {
    if (ndev <= 0 || ndev > MAX_DEV || n < 0 || (n > 0 && (!bytes || !dev_out))) {
        set_error("tiler_placement_plan: invalid arguments");
        return -1;
    }
    long long load[MAX_DEV] = {};
    for (int i = 0; i < n; i++) {
        const int d = pick_device(load, ndev);
        dev_out[i] = d;
        load[d] += bytes[i];
    }
    return 0;
}

ann_kdtree *tiler_prepare_frame_tiling_dev(ann_kdtree *global_ds, const int32_t *d_item_tile,
                                           const int32_t *d_item_pal, int64_t n_items, const uint8_t *d_palpix,
                                           const uint8_t *d_thm, const uint8_t *d_tvm, int n_tiles,
                                           const int32_t *d_palettes, int n_palettes, int quality, const uint8_t *near,
                                           int use_wavelets, int gamma, void *stream, tiler_prepare_info *info) {
    if (!global_ds || !global_ds->ix || (n_items > 0 && (!d_item_tile || !d_item_pal)) || !d_palpix || !d_thm ||
        !d_tvm || !d_palettes) {
        set_error("tiler_prepare_frame_tiling_dev: invalid arguments");
        return nullptr;
    }
    if (!ensure_init()) return nullptr;
    // the keyframe's handle lives where its buffers are; the global dataset's copy on that device serves its k = 8
    // preselection (peer-copied on first use when the keyframe runs on another GPU)
    const int dev = ptr_device(d_palpix);
    ann_kdtree *gds = replica_of(global_ds, dev);
    if (!gds) return nullptr;
    DevScope ds(dev);
    ann_kdtree *t = new ann_kdtree();
    t->dev = dev;
    if (stream_get(&t->stream) != hipSuccess) {
        set_error("tiler_prepare_frame_tiling_dev: stream creation failed");
        delete t;
        return nullptr;
    }
    hipStream_t s = stream ? (hipStream_t)stream : t->stream;
    long nd = 0, nc = 0;
    {
        std::lock_guard<std::mutex> lk(gds->ix->mu);  // its k = 8 search scratch and the prepare scratch
        if (!gds->prep) gds->prep = new PrepScratch();
        t->ix = prepare_frame_tiling_dev(gds->ix, *gds->prep, d_item_tile, d_item_pal, (long)n_items, d_palpix, d_thm,
                                         d_tvm, n_tiles, d_palettes, n_palettes, quality, near, use_wavelets, gamma, s,
                                         &nd, &nc);
    }
    if (!t->ix || hipEventCreateWithFlags(&t->maps_ev, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(t->maps_ev, s) != hipSuccess) {
        handle_free(t);
        return nullptr;
    }
    t->placed = (long long)nc * 192 * 4;
    {
        std::lock_guard<std::mutex> pl(g_place_mu);
        g_dev_load[dev] += t->placed;
    }
    if (info) {
        info->items = nd;
        info->candidates = nc;
    }
    return t;
}

int ann_kdtree_search_multi_batch(ann_kdtree *t, const float *q, int nq, int k, float eps, int *idxs, float *errs) {
    (void)eps;
    if (!t || !t->ix || nq < 0 || (nq > 0 && (!q || !idxs || !errs))) {
        set_error("ann_kdtree_search: invalid arguments");
        return -1;
    }
    if (k < 1 || k > 32) {
        set_error("ann_kdtree_search: k must be in 1..32");
        return -1;
    }
    if (!ensure_init()) return -1;
    DevScope ds(t->dev);
    std::lock_guard<std::mutex> lk(t->ix->mu);
    if (nq == 0) return 0;
    NNIndex *ix = t->ix;
    if (ix->n == 0) {
        for (long i = 0; i < (long)nq * k; i++) {
            idxs[i] = -1;
            errs[i] = FLT_MAX;
        }
        return 0;
    }
    if (ensure_io(t, nq, ix->d, k)) return -1;
    TILER_HIP_CHECK(hipMemcpyAsync(t->d_q, q, (size_t)nq * ix->d * sizeof(float), hipMemcpyHostToDevice, t->stream));
    if (nn_search_dev(ix, t->d_q, nq, k, t->d_idx, t->d_err, nullptr, t->stream)) return -1;
    TILER_HIP_CHECK(hipMemcpyAsync(idxs, t->d_idx, (size_t)nq * k * sizeof(int), hipMemcpyDeviceToHost, t->stream));
    TILER_HIP_CHECK(hipMemcpyAsync(errs, t->d_err, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost, t->stream));
    TILER_HIP_CHECK(hipStreamSynchronize(t->stream));
    return 0;
}

int ann_kdtree_search_batch(ann_kdtree *t, const float *q, int nq, float eps, int *idx, float *err) {
    return ann_kdtree_search_multi_batch(t, q, nq, 1, eps, idx, err);
}

static constexpr int COMBINE_MAX = 8192;  // queries per coalesced batch

// one coalesced batch: pack the queries into pinned memory, one search, unpack (the leader, outside c.m)
static int combine_run(ann_kdtree *t, CombineSlot &cs, std::vector<CombineReq *> &b, int k) {
    NNIndex *ix = t->ix;
    const int nq = (int)b.size(), d = ix->d;
    const size_t nr = (size_t)nq * k;
    DevScope ds(t->dev);
    std::unique_lock<std::mutex> lk(ix->mu);
    if (ix->n == 0) {
        for (CombineReq *r : b)
            for (int i = 0; i < k; i++) {
                r->idx[i] = -1;
                r->err[i] = FLT_MAX;
            }
        return 0;
    }
    if (!cs.stream) TILER_HIP_CHECK(stream_get(&cs.stream));
    if ((size_t)nq * d > cs.cap_q) {
        (void)hipHostFree(cs.h_q);
        (void)hipFree(cs.d_q);
        cs.h_q = nullptr;
        cs.d_q = nullptr;
        cs.cap_q = 0;
        TILER_HIP_CHECK(hipHostMalloc((void **)&cs.h_q, (size_t)nq * d * sizeof(float), hipHostMallocPortable));
        TILER_HIP_CHECK(hipMalloc((void **)&cs.d_q, (size_t)nq * d * sizeof(float)));
        cs.cap_q = (size_t)nq * d;
    }
    if (2 * nr > cs.cap_r) {  // indices then distances, one block: one copy back per batch
        (void)hipHostFree(cs.h_res);
        (void)hipFree(cs.d_res);
        cs.h_res = nullptr;
        cs.d_res = nullptr;
        cs.cap_r = 0;
        // fine-grained (coherent) pinned memory: a small-batch scan's merge kernel writes the results here itself
        TILER_HIP_CHECK(hipHostMalloc((void **)&cs.h_res, 2 * nr * sizeof(int),
                                      hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent));
        TILER_HIP_CHECK(hipMalloc((void **)&cs.d_res, 2 * nr * sizeof(int)));
        cs.cap_r = 2 * nr;
    }
    for (int j = 0; j < nq; j++) memcpy(cs.h_q + (size_t)j * d, b[j]->q, (size_t)d * sizeof(float));
    int *r_idx = cs.d_res;
    float *r_err = reinterpret_cast<float *>(cs.d_res + nr);
    TILER_HIP_CHECK(hipMemcpyAsync(cs.d_q, cs.h_q, (size_t)nq * d * sizeof(float), hipMemcpyHostToDevice, cs.stream));
    const bool small = nn_search_is_small(ix, nq, k);
    int *hd_res = nullptr;  // the device's view of h_res (a small-batch scan writes its results there: no copy back)
    TILER_HIP_CHECK(hipHostGetDevicePointer((void **)&hd_res, cs.h_res, 0));
    std::swap(ix->scratch, cs.scratch);  // this batch's scratch
    const int rc = nn_search_dev(ix, cs.d_q, nq, k, r_idx, r_err, nullptr, cs.stream, false, false,
                                 small ? hd_res : nullptr, small ? reinterpret_cast<float *>(hd_res + nr) : nullptr);
    std::swap(ix->scratch, cs.scratch);
    if (rc) return -1;
    if (!small)
        TILER_HIP_CHECK(hipMemcpyAsync(cs.h_res, cs.d_res, 2 * nr * sizeof(int), hipMemcpyDeviceToHost, cs.stream));
    // a small-batch scan is queued: the other slot may queue its batch while this one runs; any other search keeps
    // the index (its orbit / tier buffers) until it has finished
    if (small) lk.unlock();
    TILER_HIP_CHECK(hipStreamSynchronize(cs.stream));
    const float *h_err = reinterpret_cast<const float *>(cs.h_res + nr);
    for (int j = 0; j < nq; j++) {
        memcpy(b[j]->idx, cs.h_res + (size_t)j * k, (size_t)k * sizeof(int));
        memcpy(b[j]->err, h_err + (size_t)j * k, (size_t)k * sizeof(float));
    }
    return 0;
}

// Slots a handle's coalescer uses: the third pays where a small batch's scan is short (C3's 65,536 orbit base rows,
// plain handles up to ~65k rows: 89k -> 95k calls/s), and costs where each scan streams much more (262k plain rows,
// C5's 262k base rows: 16.6k -> 13.9k calls/s at C5) -- r06w, profiles/r06/w_percall_slots_c5_ab.txt
static int comb_slots(const ann_kdtree *t) {
    const NNIndex *ix = t->ix;
    const long rows = ix->orbit ? (long)ix->orbit->G : (long)ix->n;
    return rows * (long)ix->d * 4 > (96l << 20) ? std::min(2, Combiner::SLOTS) : Combiner::SLOTS;
}

static int combined_search(ann_kdtree *t, const float *q, int k, int *idx, float *err) {
    if (!t || !t->ix || !q || !idx || !err) {
        set_error("ann_kdtree_search: invalid arguments");
        return -1;
    }
    if (k < 1 || k > 32) {
        set_error("ann_kdtree_search: k must be in 1..32");
        return -1;
    }
    if (!ensure_init()) return -1;
    Combiner &c = t->comb;
    CombineReq me;
    me.q = q;
    me.k = k;
    me.idx = idx;
    me.err = err;
    std::unique_lock<std::mutex> lk(c.m);
    c.pending.push_back(&me);
    c.calls++;
    while (!me.done.load(std::memory_order_acquire)) {
        int si = -1;
        const int ns = comb_slots(t);
        for (int i = 0; i < ns && si < 0; i++)
            if (!c.slot[i].busy) si = i;
        if (si < 0 || c.pending.empty()) {  // every slot leading, or this caller's query is in a batch already
            if (me.taken && ANN_COMBINE_SPIN_US > 0) {
                // its batch is in flight (~40 us): spin on the answer for a while before sleeping -- a condition
                // variable wake-up of 16 waiting callers costs several microseconds each
                lk.unlock();
                const auto t0 = std::chrono::steady_clock::now();
                while (!me.done.load(std::memory_order_acquire) &&
                       std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(ANN_COMBINE_SPIN_US))
                    __builtin_ia32_pause();
                lk.lock();
                if (me.done.load(std::memory_order_acquire)) break;
            }
            c.cv.wait(lk);
            continue;
        }
        CombineSlot &cs = c.slot[si];
        cs.busy = true;  // lead: batches until this caller's own query is answered or nothing is left to take
        while (!me.done && !c.pending.empty()) {
            std::vector<CombineReq *> b;
            const int bk = c.pending.front()->k;
            for (auto it = c.pending.begin(); it != c.pending.end() && (int)b.size() < COMBINE_MAX;) {
                if ((*it)->k == bk) {
                    (*it)->taken = true;
                    b.push_back(*it);
                    it = c.pending.erase(it);
                } else {
                    ++it;
                }
            }
            c.batches++;
            c.max_batch = std::max(c.max_batch, (int)b.size());
            lk.unlock();
            const int rc = combine_run(t, cs, b, bk);
            const std::string msg = rc ? std::string(last_error()) : std::string();
            lk.lock();
            for (CombineReq *r : b) {
                r->rc = rc;
                r->msg = msg;
                r->done.store(true, std::memory_order_release);
            }
            c.cv.notify_all();
        }
        cs.busy = false;
        c.cv.notify_all();  // a waiting caller takes over the queue (or finds its answer)
    }
    if (me.rc) set_error(me.msg);
    return me.rc;
}

int ann_kdtree_search(ann_kdtree *t, float *q, float eps, float *err) {
    (void)eps;  // the exact answer satisfies every eps bound
    int idx = -1;
    float e = 0.0f;
    if (combined_search(t, q, 1, &idx, &e)) return -1;
    if (err) *err = e;
    return idx;
}

// annkPriSearch's answer (ann_kdtree_pri_search, extern.pas:66 -> ANN.dll 0x180003ef0, which calls annkPriSearch
// 0x1800121a0 with k = 1 and the caller's eps): the priority search replayed on the GPU (kd_pri_search), its own tie
// order and its (1 + eps)^2 termination included.  Queries in chunks that keep the heap scratch <= 1 GiB.  A handle
// without a tree (TILER_SPLIT_INDEX_ORDER) answers as ann_kdtree_search does.
int ann_kdtree_pri_search_batch(ann_kdtree *t, const float *q, int nq, float eps, int *idx, float *err) {
    if (!t || !t->ix || nq < 0 || (nq > 0 && (!q || !idx || !err))) {
        set_error("ann_kdtree_pri_search: invalid arguments");
        return -1;
    }
    if (!ensure_init()) return -1;
    if (!t->ix->kd) return ann_kdtree_search_multi_batch(t, q, nq, 1, eps, idx, err);
    DevScope ds(t->dev);
    NNIndex *ix = t->ix;
    std::lock_guard<std::mutex> lk(ix->mu);
    if (nq == 0) return 0;
    if (ix->n == 0) {
        for (int i = 0; i < nq; i++) {
            idx[i] = -1;
            err[i] = FLT_MAX;
        }
        return 0;
    }
    const size_t per = kd_pri_heap_bytes(ix->kd, 1);
    const int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)nq, ((size_t)1 << 30) / per));
    if (ensure_io(t, chunk, ix->d, 1)) return -1;
    if (per * chunk > t->cap_pri) {
        (void)hipFree(t->d_pri);
        t->d_pri = nullptr;
        t->cap_pri = 0;
        TILER_HIP_CHECK(hipMalloc(&t->d_pri, per * chunk));
        t->cap_pri = per * chunk;
    }
    // eps = 0: annkSearch's answer and the exact tie set decide almost every query (kd_pri_resolve); the rest, and
    // every query of eps > 0, replay the priority search
    const size_t aux = kd_pri_aux_bytes(chunk) + (size_t)chunk;
    if (eps == 0.0f && aux > t->cap_pri_aux) {
        (void)hipFree(t->d_pri_aux);
        t->d_pri_aux = nullptr;
        t->cap_pri_aux = 0;
        TILER_HIP_CHECK(hipMalloc(&t->d_pri_aux, aux));
        t->cap_pri_aux = aux;
    }
    for (int q0 = 0; q0 < nq; q0 += chunk) {
        const int c = std::min(chunk, nq - q0);
        TILER_HIP_CHECK(hipMemcpyAsync(t->d_q, q + (size_t)q0 * ix->d, (size_t)c * ix->d * sizeof(float),
                                       hipMemcpyHostToDevice, t->stream));
        uint8_t *flag = nullptr;
        if (eps == 0.0f) {
            flag = (uint8_t *)t->d_pri_aux + kd_pri_aux_bytes(chunk);
            if (nn_search_dev(ix, t->d_q, c, 1, t->d_idx, t->d_err, nullptr, t->stream)) return -1;
            if (kd_pri_resolve(ix->kd, ix->d_rows, t->d_q, c, t->d_err, t->d_pri_aux, t->d_idx, t->d_err, flag,
                               t->stream))
                return -1;
        }
        if (kd_pri_search(ix->kd, ix->d_rows, t->d_q, c, eps, t->d_pri, t->d_idx, t->d_err, t->stream, flag,
                          flag ? t->d_pri_aux : nullptr))
            return -1;
        TILER_HIP_CHECK(hipMemcpyAsync(idx + q0, t->d_idx, (size_t)c * sizeof(int), hipMemcpyDeviceToHost, t->stream));
        TILER_HIP_CHECK(hipMemcpyAsync(err + q0, t->d_err, (size_t)c * sizeof(float), hipMemcpyDeviceToHost, t->stream));
        TILER_HIP_CHECK(hipStreamSynchronize(t->stream));
    }
    // the heap scratch (up to 1 GiB) is not kept on the handle: several keyframe handles would each pin it
    (void)hipFree(t->d_pri);
    t->d_pri = nullptr;
    t->cap_pri = 0;
    return 0;
}

int ann_kdtree_pri_search(ann_kdtree *t, float *q, float eps, float *err) {
    int idx = -1;
    float e = 0.0f;
    if (ann_kdtree_pri_search_batch(t, q, 1, eps, &idx, &e)) return -1;
    if (err) *err = e;
    return idx;
}

int ann_kdtree_search_multi(ann_kdtree *t, int *idxs, float *errs, int cnt, float *q, float eps) {
    (void)eps;
    return combined_search(t, q, cnt, idxs, errs);
}

int tiler_set_scan_limits(int max_k1, int max_k8) {
    if (max_k1 < 0 || max_k8 < 0) {
        set_error("tiler_set_scan_limits: negative limit");
        return -1;
    }
    nn_set_scan_limits(max_k1, max_k8);
    return 0;
}

int tiler_debug_force_replay(int on) {
    nn_set_force_replay(on);
    return 0;
}

int tiler_debug_shortlist_gate(int on) {
    nn_set_shortlist_gate(on);
    return 0;
}

int tiler_combine_stats(ann_kdtree *t, int64_t *calls, int64_t *batches, int32_t *max_batch) {
    if (!t) {
        set_error("tiler_combine_stats: null handle");
        return -1;
    }
    std::lock_guard<std::mutex> lk(t->comb.m);
    if (calls) *calls = t->comb.calls;
    if (batches) *batches = t->comb.batches;
    if (max_batch) *max_batch = t->comb.max_batch;
    return 0;
}

int tiler_debug_percall_bench(ann_kdtree *t, const float *q, int nq, int k, int threads, int32_t *idx, float *err,
                              double *wall_s, double *lone_us) {
    if (!t || !t->ix || nq < 0 || (nq > 0 && (!q || !idx || !err)) || k < 1 || k > 32 || threads < 1 || threads > 256) {
        set_error("tiler_debug_percall_bench: invalid arguments");
        return -1;
    }
    const int d = t->ix->d;
    auto call = [&](int i) -> int {
        float *qi = const_cast<float *>(q + (size_t)i * d);
        if (k == 1) {
            const int r = ann_kdtree_search(t, qi, 0.0f, err + i);
            idx[i] = r;
            return r < 0 && t->ix->n > 0 ? -1 : 0;
        }
        return ann_kdtree_search_multi(t, idx + (size_t)i * k, err + (size_t)i * k, k, qi, 0.0f);
    };
    // lone calls: one caller, one query at a time (the latency of the whole per-call path)
    const int nl = std::min(nq, 64);
    std::vector<double> lat;
    for (int i = 0; i < nl; i++) {
        const auto a = std::chrono::steady_clock::now();
        if (call(i)) return -1;
        lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
    }
    std::sort(lat.begin(), lat.end());
    if (lone_us) *lone_us = lat.empty() ? 0.0 : lat[lat.size() / 2];
    // `threads` native callers on the one handle, query i on thread i % threads (a pool's workers)
    std::atomic<int> bad{0};
    std::string msg;
    std::mutex msg_mu;
    const auto a = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int w = 0; w < threads; w++)
        th.emplace_back([&, w]() {
            for (int i = w; i < nq; i += threads)
                if (call(i)) {
                    bad.store(1);
                    std::lock_guard<std::mutex> lk(msg_mu);
                    msg = last_error();
                    return;
                }
        });
    for (auto &x : th) x.join();
    if (wall_s) *wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
    if (bad.load()) {
        set_error("tiler_debug_percall_bench: " + msg);
        return -1;
    }
    return 0;
}

int ann_kdtree_search_batch_dev(ann_kdtree *t, const float *d_q, int nq, int k, int *d_idx, float *d_err,
                                void *stream) {
    if (!t || !t->ix) {
        set_error("ann_kdtree_search_batch_dev: null handle");
        return -1;
    }
    if (!ensure_init()) return -1;
    if (!(t = handle_for(t, d_q))) return -1;
    DevScope ds(t->dev);
    std::lock_guard<std::mutex> lk(t->ix->mu);
    return nn_search_dev(t->ix, d_q, nq, k, d_idx, d_err, nullptr, (hipStream_t)stream);
}

int ann_kdtree_get_stats(ann_kdtree *t, tiler_search_stats *out) {
    if (!t || !t->ix || !out) {
        set_error("ann_kdtree_get_stats: invalid arguments");
        return -1;
    }
    DevScope ds(t->dev);
    std::lock_guard<std::mutex> lk(t->ix->mu);
    // everything below was written by the last search on ITS stream (the caller's, for the _dev entry points)
    if (t->ix->done_event) TILER_HIP_CHECK(hipEventSynchronize(t->ix->done_event));
    out->queries = t->ix->last_queries;
    out->fallback_queries = t->ix->last_splits > 0 ? t->ix->h_fb_count[0] : 0;
    out->exhaustive_queries = t->ix->last_splits > 0 ? t->ix->h_fb_count[1] : t->ix->last_fallback;
    out->exact_integer = t->ix->exact_int ? 1 : 0;
    out->splits = t->ix->last_splits;
    out->orbit_groups = t->ix->orbit ? orbit_groups(t->ix) : 0;
    out->orbit_search = t->ix->last_orbit;
    out->orbit_ksteps = t->ix->orbit ? orbit_ksteps(t->ix) : 0;
    long long ne = 0, nr = 0;
    if (t->ix->orbit) orbit_counters(t->ix, &ne, &nr);
    out->orbit_expansions = ne;
    out->orbit_rescored = nr;
    out->tie_order = t->ix->kd ? 0 : 1;
    out->kd_levels = t->ix->kd ? t->ix->kd->levels : 0;
    out->kd_build_ms = t->ix->kd ? t->ix->kd->build_ms : 0.0;
    out->kd_replayed = 0;
    out->flat_queries = 0;
    if (const NNIndex *ix = t->ix; ix->last_flat_dev) {  // queries in all-flat shortlist workgroups
        int others = 0;
        TILER_HIP_CHECK(hipMemcpy(&others, ix->last_flat_dev, sizeof(int), hipMemcpyDeviceToHost));
        const long wf0 = std::min(ix->last_flat_wgs, (others + ix->last_flat_qpw - 1) / ix->last_flat_qpw);
        out->flat_queries = wf0 < ix->last_flat_wgs ? ix->last_flat_nq - wf0 * ix->last_flat_qpw : 0;
    }
    if (t->ix->kd && t->ix->scratch.kd_count) {
        int c = 0;
        TILER_HIP_CHECK(hipMemcpy(&c, t->ix->scratch.kd_count, sizeof(int), hipMemcpyDeviceToHost));
        out->kd_replayed = c;
    }
    return 0;
}

int tiler_kdtree_positions(ann_kdtree *t, int32_t *pos) {
    if (!t || !t->ix || !pos) {
        set_error("tiler_kdtree_positions: invalid arguments");
        return -1;
    }
    if (!t->ix->kd) {
        set_error("tiler_kdtree_positions: handle has no kd-tree (KD_SPLIT_INDEX_ORDER)");
        return -1;
    }
    DevScope ds(t->dev);
    std::lock_guard<std::mutex> lk(t->ix->mu);
    return kd_tree_positions(t->ix->kd, pos);
}

int tiler_psyv_batch_dev(int n, const int32_t *rgb, const uint8_t *palpix, const int32_t *tile_of,
                         const int32_t *palettes, const int32_t *pal_of, const uint8_t *flags_per, int flags, int gamma,
                         double *out64, float *out32, void *stream) {
    if (!ensure_init()) return -1;
    DevScope ds(ptr_device(rgb ? (const void *)rgb : (const void *)palpix));
    PsyvArgs a;
    a.n = n;
    a.rgb = rgb;
    a.palpix = palpix;
    a.tile_of = tile_of;
    a.palettes = palettes;
    a.pal_of = pal_of;
    a.flags_per = flags_per;
    a.flags = flags;
    a.gamma = gamma;
    a.out64 = out64;
    a.out32 = out32;
    return launch_psyv(a, (hipStream_t)stream);
}

int tiler_psyv_batch(int n, const int32_t *rgb, int n_tiles, const uint8_t *palpix, const int32_t *tile_of,
                     int n_palettes, const int32_t *palettes, const int32_t *pal_of, const uint8_t *flags_per,
                     int flags, int gamma, double *out64, float *out32) {
    if (!ensure_init()) return -1;
    if (n < 0) {
        set_error("psyv: n < 0");
        return -1;
    }
    if (n == 0) return 0;
    const bool from_pal = (flags & 1) != 0 || (flags_per != nullptr);
    std::vector<void *> bufs;
    auto up = [&](const void *h, size_t bytes) -> void * {
        if (!h || bytes == 0) return nullptr;
        void *d = nullptr;
        if (hipMalloc(&d, bytes) != hipSuccess) return nullptr;
        bufs.push_back(d);
        hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
        return d;
    };
    auto cleanup = [&]() {
        for (void *p : bufs) hipFree(p);
    };
    int32_t *d_rgb = (int32_t *)up(rgb, rgb ? (size_t)n * 64 * 4 : 0);
    uint8_t *d_pp = from_pal ? (uint8_t *)up(palpix, (size_t)std::max(n_tiles, 0) * 64) : nullptr;
    int32_t *d_to = (int32_t *)up(tile_of, tile_of ? (size_t)n * 4 : 0);
    int32_t *d_pal = from_pal ? (int32_t *)up(palettes, (size_t)std::max(n_palettes, 0) * 16 * 4) : nullptr;
    int32_t *d_po = (int32_t *)up(pal_of, pal_of ? (size_t)n * 4 : 0);
    uint8_t *d_fp = (uint8_t *)up(flags_per, flags_per ? (size_t)n : 0);
    double *d_o64 = nullptr;
    float *d_o32 = nullptr;
    if (out64 && hipMalloc((void **)&d_o64, (size_t)n * 192 * 8) == hipSuccess) bufs.push_back(d_o64);
    if (out32 && hipMalloc((void **)&d_o32, (size_t)n * 192 * 4) == hipSuccess) bufs.push_back(d_o32);
    if ((!rgb && !from_pal) || (rgb && !d_rgb) || (from_pal && (!d_pp || !d_pal)) || (out64 && !d_o64) ||
        (out32 && !d_o32)) {
        cleanup();
        set_error("psyv: missing input buffer or device allocation failed");
        return -1;
    }
    int rc = tiler_psyv_batch_dev(n, d_rgb, d_pp, d_to, d_pal, d_po, d_fp, flags, gamma, d_o64, d_o32, nullptr);
    if (rc == 0) {
        if (out64) hipMemcpy(out64, d_o64, (size_t)n * 192 * 8, hipMemcpyDeviceToHost);
        if (out32) hipMemcpy(out32, d_o32, (size_t)n * 192 * 4, hipMemcpyDeviceToHost);
        if (hipDeviceSynchronize() != hipSuccess) {
            set_error("psyv: kernel failed");
            rc = -1;
        }
    }
    cleanup();
    return rc;
}

static int set_maps_one(ann_kdtree *t, const int32_t *tr_tile, const int32_t *tr_pal, const uint8_t *tr_attr) {
    DevScope ds(t->dev);
    NNIndex *ix = t->ix;
    std::lock_guard<std::mutex> lk(ix->mu);
    const size_t n = std::max(1, ix->n);
    (void)hipDeviceSynchronize();  // a search may still read the old maps (dfree: hipFree's rule made explicit)
    dfree(ix->d_tr_tile);
    dfree(ix->d_tr_pal);
    dfree(ix->d_tr_attr);
    TILER_HIP_CHECK(dmalloc((void **)&ix->d_tr_tile, n * 4));
    TILER_HIP_CHECK(dmalloc((void **)&ix->d_tr_pal, n * 4));
    TILER_HIP_CHECK(dmalloc((void **)&ix->d_tr_attr, n));
    TILER_HIP_CHECK(hipMemcpy(ix->d_tr_tile, tr_tile, (size_t)ix->n * 4, hipMemcpyHostToDevice));
    TILER_HIP_CHECK(hipMemcpy(ix->d_tr_pal, tr_pal, (size_t)ix->n * 4, hipMemcpyHostToDevice));
    TILER_HIP_CHECK(hipMemcpy(ix->d_tr_attr, tr_attr, (size_t)ix->n, hipMemcpyHostToDevice));
    return 0;
}

int tiler_ft_set_maps(ann_kdtree *t, const int32_t *tr_tile, const int32_t *tr_pal, const uint8_t *tr_attr) {
    if (!t || !t->ix || !tr_tile || !tr_pal || !tr_attr) {
        set_error("tiler_ft_set_maps: invalid arguments");
        return -1;
    }
    if (!ensure_init()) return -1;
    if (set_maps_one(t, tr_tile, tr_pal, tr_attr)) return -1;
    std::lock_guard<std::mutex> lk(t->rep_mu);  // the copies on other devices get the same maps
    for (int d = 0; d < MAX_DEV; d++)
        if (t->rep[d] && set_maps_one(t->rep[d], tr_tile, tr_pal, tr_attr)) return -1;
    return 0;
}

int tiler_ft_get_maps(ann_kdtree *t, int32_t *tr_tile, int32_t *tr_pal, uint8_t *tr_attr) {
    if (!t || !t->ix || !tr_tile || !tr_pal || !tr_attr) {
        set_error("tiler_ft_get_maps: invalid arguments");
        return -1;
    }
    if (!t->ix->d_tr_tile) {
        set_error("tiler_ft_get_maps: the handle has no maps");
        return -1;
    }
    if (!ensure_init()) return -1;
    DevScope ds(t->dev);
    NNIndex *ix = t->ix;
    std::lock_guard<std::mutex> lk(ix->mu);
    // maps written by tiler_prepare_frame_tiling_dev on the caller's stream: wait for that work only (the other
    // streams of the device keep running); tiler_ft_set_maps copies synchronously
    if (t->maps_ev) TILER_HIP_CHECK(hipEventSynchronize(t->maps_ev));
    TILER_HIP_CHECK(hipMemcpy(tr_tile, ix->d_tr_tile, (size_t)ix->n * 4, hipMemcpyDeviceToHost));
    TILER_HIP_CHECK(hipMemcpy(tr_pal, ix->d_tr_pal, (size_t)ix->n * 4, hipMemcpyDeviceToHost));
    TILER_HIP_CHECK(hipMemcpy(tr_attr, ix->d_tr_attr, (size_t)ix->n, hipMemcpyDeviceToHost));
    return 0;
}

// FrameTiling on handle t itself (its device; the entry points pick the handle)
static int frame_tiling_on(ann_kdtree *t, const int32_t *d_rgb, int Q, int use_wavelets, int gamma, int32_t *d_tile,
                           int32_t *d_pal, uint8_t *d_hm, uint8_t *d_vm, float *d_err, void *stream) {
    if (!t->ix->d_tr_tile) {
        set_error("tiler_frame_tiling: call tiler_ft_set_maps first");
        return -1;
    }
    DevScope ds(t->dev);
    std::lock_guard<std::mutex> lk(t->ix->mu);
    if (ensure_io(t, Q, 1, 1)) return -1;
    FtMaps m{d_tile, d_pal, d_hm, d_vm};
    return nn_frame_tiling_dev(t->ix, d_rgb, Q, use_wavelets, gamma, t->d_idx, d_err, &m, (hipStream_t)stream);
}

int tiler_frame_tiling_dev(ann_kdtree *t, const int32_t *d_rgb, int Q, int use_wavelets, int gamma, int32_t *d_tile,
                           int32_t *d_pal, uint8_t *d_hm, uint8_t *d_vm, float *d_err, void *stream) {
    if (!t || !t->ix) {
        set_error("tiler_frame_tiling: null handle");
        return -1;
    }
    if (!ensure_init()) return -1;
    if (!(t = handle_for(t, d_rgb))) return -1;
    return frame_tiling_on(t, d_rgb, Q, use_wavelets, gamma, d_tile, d_pal, d_hm, d_vm, d_err, stream);
}

int tiler_frame_tiling(ann_kdtree *t, const int32_t *rgb, int Q, int use_wavelets, int gamma, int32_t *out_tile,
                       int32_t *out_pal, uint8_t *out_hm, uint8_t *out_vm, float *out_err) {
    if (!t || !t->ix || Q < 0 || (Q > 0 && (!rgb || !out_tile || !out_pal || !out_hm || !out_vm || !out_err))) {
        set_error("tiler_frame_tiling: invalid arguments");
        return -1;
    }
    if (Q == 0) return 0;
    if (!ensure_init()) return -1;
    DevScope ds(t->dev);
    if ((size_t)Q > t->cap_ft) {
        hipFree(t->d_rgb);
        hipFree(t->d_mt);
        hipFree(t->d_mp);
        hipFree(t->d_mh);
        hipFree(t->d_mv);
        TILER_HIP_CHECK(hipMalloc((void **)&t->d_rgb, (size_t)Q * 256));
        TILER_HIP_CHECK(hipMalloc((void **)&t->d_mt, (size_t)Q * 4));
        TILER_HIP_CHECK(hipMalloc((void **)&t->d_mp, (size_t)Q * 4));
        TILER_HIP_CHECK(hipMalloc((void **)&t->d_mh, (size_t)Q));
        TILER_HIP_CHECK(hipMalloc((void **)&t->d_mv, (size_t)Q));
        t->cap_ft = Q;
    }
    {
        std::lock_guard<std::mutex> lk(t->ix->mu);
        if (ensure_io(t, Q, 1, 1)) return -1;
    }
    TILER_HIP_CHECK(hipMemcpyAsync(t->d_rgb, rgb, (size_t)Q * 256, hipMemcpyHostToDevice, t->stream));
    if (frame_tiling_on(t, t->d_rgb, Q, use_wavelets, gamma, t->d_mt, t->d_mp, t->d_mh, t->d_mv, t->d_err, t->stream))
        return -1;
    TILER_HIP_CHECK(hipMemcpyAsync(out_tile, t->d_mt, (size_t)Q * 4, hipMemcpyDeviceToHost, t->stream));
    TILER_HIP_CHECK(hipMemcpyAsync(out_pal, t->d_mp, (size_t)Q * 4, hipMemcpyDeviceToHost, t->stream));
    TILER_HIP_CHECK(hipMemcpyAsync(out_hm, t->d_mh, (size_t)Q, hipMemcpyDeviceToHost, t->stream));
    TILER_HIP_CHECK(hipMemcpyAsync(out_vm, t->d_mv, (size_t)Q, hipMemcpyDeviceToHost, t->stream));
    TILER_HIP_CHECK(hipMemcpyAsync(out_err, t->d_err, (size_t)Q * 4, hipMemcpyDeviceToHost, t->stream));
    TILER_HIP_CHECK(hipStreamSynchronize(t->stream));
    return 0;
}

int tiler_smooth_keyframe(int F, int Q, int32_t *tile, int32_t *tmpidx, int32_t *pal, uint8_t *hm, uint8_t *vm,
                          uint8_t *smoothed, int T, const uint8_t *palpix, int P, const int32_t *palettes,
                          double strength) {
    if (!ensure_init()) return -1;
    return smooth_keyframe_host(F, Q, tile, tmpidx, pal, hm, vm, smoothed, T, palpix, P, palettes, strength);
}

int tiler_smooth_keyframe_dev(int F, int Q, int32_t *d_tile, int32_t *d_tmpidx, int32_t *d_pal, uint8_t *d_hm,
                              uint8_t *d_vm, uint8_t *d_smoothed, const uint8_t *d_palpix, const int32_t *d_palettes,
                              double strength, void *stream) {
    if (!ensure_init()) return -1;
    DevScope ds(ptr_device(d_tile));
    return smooth_keyframe_dev(F, Q, d_tile, d_tmpidx, d_pal, d_hm, d_vm, d_smoothed, d_palpix, d_palettes, strength,
                               (hipStream_t)stream);
}

int tiler_dither_tiles(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes, int n_palettes,
                       int palsize, uint8_t *palpix, uint8_t *hm, uint8_t *vm) {
    if (!ensure_init()) return -1;
    return dither_tiles_host(n, rgb, pal_of, palettes, n_palettes, palsize, 0, palpix, hm, vm);
}

int tiler_dither_tiles_dev(int n, const int32_t *d_rgb, const int32_t *d_pal_of, const int32_t *d_palettes,
                           int n_palettes, int palsize, uint8_t *d_palpix, uint8_t *d_hm, uint8_t *d_vm, void *stream) {
    if (!ensure_init()) return -1;
    DevScope ds(ptr_device(d_rgb));
    return dither_tiles_dev(n, d_rgb, d_pal_of, d_palettes, n_palettes, palsize, 0, d_palpix, d_hm, d_vm,
                            (hipStream_t)stream);
}

int tiler_dither_tiles_yliluoma(int n, const int32_t *rgb, const int32_t *pal_of, const int32_t *palettes,
                                int n_palettes, int palsize, int mixed_colors, uint8_t *palpix, uint8_t *hm,
                                uint8_t *vm) {
    if (!ensure_init()) return -1;
    if (mixed_colors < 1) {
        set_error("dither: Yliluoma mixed colours must be 1..64");
        return -1;
    }
    return dither_tiles_host(n, rgb, pal_of, palettes, n_palettes, palsize, mixed_colors, palpix, hm, vm);
}

int tiler_dither_tiles_yliluoma_dev(int n, const int32_t *d_rgb, const int32_t *d_pal_of, const int32_t *d_palettes,
                                    int n_palettes, int palsize, int mixed_colors, uint8_t *d_palpix, uint8_t *d_hm,
                                    uint8_t *d_vm, void *stream) {
    if (!ensure_init()) return -1;
    if (mixed_colors < 1) {
        set_error("dither: Yliluoma mixed colours must be 1..64");
        return -1;
    }
    DevScope ds(ptr_device(d_rgb));
    return dither_tiles_dev(n, d_rgb, d_pal_of, d_palettes, n_palettes, palsize, mixed_colors, d_palpix, d_hm, d_vm,
                            (hipStream_t)stream);
}

int tiler_quantize_palettes(long n_tiles, const int32_t *rgb, const int32_t *pal_of, const uint8_t *active,
                            int n_palettes, int palsize, int lookup_bpc, int32_t *palettes, int32_t *use_count,
                            int32_t *colors) {
    if (!ensure_init()) return -1;
    return quantize_palettes_host(n_tiles, rgb, pal_of, active, n_palettes, palsize, lookup_bpc, palettes, use_count,
                                  colors);
}

int tiler_quantize_palettes_dev(long n_tiles, const int32_t *d_rgb, const int32_t *d_pal_of, const uint8_t *d_active,
                                int n_palettes, int palsize, int lookup_bpc, int32_t *palettes, int32_t *use_count,
                                int32_t *colors, void *stream) {
    if (!ensure_init()) return -1;
    DevScope ds(ptr_device(d_rgb));
    return quantize_palettes_dev(n_tiles, d_rgb, d_pal_of, d_active, n_palettes, palsize, lookup_bpc, palettes,
                                 use_count, colors, (hipStream_t)stream);
}

int tiler_debug_dl3(int list_cap) {
    dl3_debug(list_cap);
    return 0;
}

int tiler_prepare_dither_tiles_dev(long n_tiles, const int32_t *d_rgb, int n_palettes, int gamma, int use_wavelets,
                                   int max_iter, uint32_t seed, int32_t *d_labels, double *d_centroids,
                                   int *iterations, void *stream) {
    if (!ensure_init()) return -1;
    DevScope ds(ptr_device(d_rgb));
    return prepare_dither_dev(n_tiles, d_rgb, n_palettes, gamma, use_wavelets, max_iter <= 0 ? 0x7fffffff : max_iter,
                              seed, d_labels, d_centroids, iterations, (hipStream_t)stream);
}

int tiler_prepare_dither_tiles(long n_tiles, const int32_t *rgb, int n_palettes, int gamma, int use_wavelets,
                               int max_iter, uint32_t seed, int32_t *labels, double *centroids, int *iterations) {
    if (!ensure_init()) return -1;
    if (n_tiles < 0 || n_palettes <= 0 || (n_tiles > 0 && (!rgb || !labels)) || !centroids) {
        set_error("prepare_dither_tiles: invalid arguments");
        return -1;
    }
    const size_t b_rgb = (size_t)n_tiles * 256, b_lab = (size_t)n_tiles * 4, b_c = (size_t)n_palettes * 192 * 8;
    char *buf = nullptr;
    TILER_HIP_CHECK(hipMalloc((void **)&buf, b_rgb + b_lab + b_c + 512));
    char *d_rgb = buf, *d_lab = buf + ((b_rgb + 255) & ~(size_t)255), *d_c = d_lab + ((b_lab + 255) & ~(size_t)255);
    hipStream_t st = nullptr;
    int rc = -1;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess) {
        do {
            if (n_tiles > 0 && hipMemcpyAsync(d_rgb, rgb, b_rgb, hipMemcpyHostToDevice, st) != hipSuccess) break;
            if (prepare_dither_dev(n_tiles, (const int32_t *)d_rgb, n_palettes, gamma, use_wavelets,
                                   max_iter <= 0 ? 0x7fffffff : max_iter, seed, (int32_t *)d_lab, (double *)d_c,
                                   iterations, st))
                break;
            if (n_tiles > 0 && hipMemcpyAsync(labels, d_lab, b_lab, hipMemcpyDeviceToHost, st) != hipSuccess) break;
            if (hipMemcpyAsync(centroids, d_c, b_c, hipMemcpyDeviceToHost, st) != hipSuccess) break;
            if (hipStreamSynchronize(st) != hipSuccess) break;
            rc = 0;
        } while (0);
        (void)hipStreamDestroy(st);
    }
    if (rc && !last_error()[0]) set_error("prepare_dither_tiles: HIP failure");
    (void)hipFree(buf);
    return rc;
}

int tiler_kmeans(const double *X, long n, int d, int k, int max_iter, uint32_t seed, int32_t *labels,
                 double *centroids, int *iterations) {
    if (!ensure_init()) return -1;
    if (n <= 0 || d <= 0 || d > 192 || k <= 0 || !X || !labels || !centroids) {
        set_error("kmeans: invalid arguments");
        return -1;
    }
    const size_t bx = (size_t)n * d * 8, bl = (size_t)n * 4, bc = (size_t)k * d * 8;
    char *buf = nullptr;
    TILER_HIP_CHECK(hipMalloc((void **)&buf, bx + bl + bc + 512));
    char *d_x = buf, *d_l = buf + ((bx + 255) & ~(size_t)255), *d_c = d_l + ((bl + 255) & ~(size_t)255);
    hipStream_t st = nullptr;
    int rc = -1;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess) {
        do {
            if (hipMemcpyAsync(d_x, X, bx, hipMemcpyHostToDevice, st) != hipSuccess) break;
            if (kmeans_dev((const double *)d_x, n, d, k, max_iter <= 0 ? 0x7fffffff : max_iter, seed, (int32_t *)d_l,
                           (double *)d_c, iterations, st))
                break;
            if (hipMemcpyAsync(labels, d_l, bl, hipMemcpyDeviceToHost, st) != hipSuccess) break;
            if (hipMemcpyAsync(centroids, d_c, bc, hipMemcpyDeviceToHost, st) != hipSuccess) break;
            if (hipStreamSynchronize(st) != hipSuccess) break;
            rc = 0;
        } while (0);
        (void)hipStreamDestroy(st);
    }
    if (rc && !last_error()[0]) set_error("kmeans: HIP failure");
    (void)hipFree(buf);
    return rc;
}

int tiler_finish_quantize_order(int n_palettes, const int32_t *use_count, int32_t *lut) {
    if (n_palettes <= 0 || !use_count || !lut) {
        set_error("finish_quantize_order: invalid arguments");
        return -1;
    }
    finish_quantize_order(use_count, n_palettes, lut);
    return 0;
}

int tiler_interframe_correlation(const int32_t *rgb, int F, int tm_w, int tm_h, double *corr) {
    if (!ensure_init()) return -1;
    return interframe_corr_host(rgb, F, tm_w, tm_h, corr);
}

int tiler_interframe_correlation_dev(const int32_t *d_rgb, int F, int tm_w, int tm_h, double *corr, void *stream) {
    if (!ensure_init()) return -1;
    DevScope ds(ptr_device(d_rgb));
    return interframe_corr_dev(d_rgb, F, tm_w, tm_h, corr, (hipStream_t)stream);
}

int tiler_find_keyframes(const double *corr, int F, int tile_map_size, int32_t *kf_of_frame) {
    return find_keyframes(corr, F, tile_map_size, kf_of_frame);
}

int tiler_kmodes_medoids(const uint8_t *X, int n, const int32_t *labels, const uint8_t *centroids, int k,
                         int32_t *medoid, int32_t *counts) {
    if (!ensure_init()) return -1;
    return kmodes_medoids_host(X, n, labels, centroids, k, medoid, counts);
}

int tiler_kmodes_compute(const uint8_t *X, int n, int nattr, int k, int start_point, int n_modalities,
                         int32_t *labels, uint8_t *centroids, int *n_iter, uint64_t *cost) {
    if (!ensure_init()) return -1;
    return kmodes_compute_host(X, n, nattr, k, start_point, n_modalities, labels, centroids, n_iter, cost);
}

int tiler_kmodes_batch(const uint8_t *X, const int32_t *bin_off, int nbins, const int32_t *k, const int32_t *start,
                       int n_modalities, int32_t *labels, uint8_t *centroids, int32_t *n_iter, uint64_t *cost) {
    if (!ensure_init()) return -1;
    return kmodes_batch_host(X, bin_off, nbins, k, start, n_modalities, labels, centroids, n_iter, cost);
}

int tiler_kmodes_batch_dev(const uint8_t *d_X, const int32_t *bin_off, int nbins, const int32_t *k,
                           const int32_t *start, int n_modalities, int32_t *d_labels, uint8_t *d_centroids,
                           int32_t *n_iter, uint64_t *cost, void *stream) {
    if (!ensure_init()) return -1;
    if (!d_X || !bin_off || !k || !start || !d_labels || !d_centroids) {
        set_error("kmodes: null buffer");
        return -1;
    }
    DevScope ds(ptr_device(d_X));
    return kmodes_batch_dev(d_X, bin_off, nbins, k, start, n_modalities, d_labels, d_centroids, n_iter, cost,
                            (hipStream_t)stream);
}

int tiler_debug_kmodes_ff_fallback(int on) {
    kmodes_force_ff_fallback(on);
    return 0;
}

int tiler_kmodes_last_stats(int64_t *assign_pairs, int64_t *chunk_steps) {
    long long p = 0, c = 0;
    kmodes_last_stats(&p, &c);
    if (assign_pairs) *assign_pairs = p;
    if (chunk_steps) *chunk_steps = c;
    return 0;
}

int tiler_kmodes_medoids_batch(const uint8_t *X, const int32_t *bin_off, int nbins, const int32_t *k,
                               const int32_t *labels, const uint8_t *centroids, int32_t *medoid, int32_t *counts) {
    if (!ensure_init()) return -1;
    return kmodes_medoids_batch_host(X, bin_off, nbins, k, labels, centroids, medoid, counts);
}

}  // extern "C"
