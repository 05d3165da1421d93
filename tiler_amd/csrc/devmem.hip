// devmem.hip -- the cache of device blocks behind every search index (round 6).
//
// The encoder makes one search index per keyframe (PrepareFrameTiling: candidate rows, MFMA fragments, kd-tree, search
// scratch; tiler_prepare_frame_tiling_dev) and destroys it after the keyframe's FrameTiling (FinishFrameTiling).  With
// hipMalloc / hipFree that is ~50 driver allocations and ~50 frees per keyframe, and every hipFree also waits for the
// whole device: bench_encoder's loop spent 7.0 ms of each 34 ms keyframe in the previous handle's destroy alone, the GPU
// idle (profiles/r06/l_encoder_loop.json, loop_ms_avg.close).  Here freed blocks stay on the device for the next index
// of about the same size (a 288 GB HBM3E device holds a keyframe's ~1 GB of index many times over).
//
// Safety is hipFree's own rule, made explicit: dfree() only files the block; the caller guarantees no GPU work still
// uses it -- the destroy paths do one hipDeviceSynchronize() first (what each hipFree did implicitly), the kd build
// frees its scratch after synchronising its stream.  A block handed out by dmalloc() is therefore idle.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "tiler_common.hpp"

namespace tiler {

namespace {
struct Block {
    size_t bytes;
    int dev;
};
constexpr int DM_MAX_DEV = 64;
constexpr size_t DM_CAP = (size_t)16 << 30;  // cached bytes per device at most (beyond: hipFree)
std::mutex g_dm_mu;
std::unordered_map<void *, Block> g_dm_live;             // every block dmalloc handed out, with its class size
std::multimap<size_t, void *> g_dm_free[DM_MAX_DEV];      // cached idle blocks by size
size_t g_dm_cached[DM_MAX_DEV] = {};

size_t dm_class(size_t bytes) {  // 256-B multiples below 1 MiB (powers of two), 2 MiB multiples above
    if (bytes <= 256) return 256;
    if (bytes < ((size_t)1 << 20)) {
        size_t c = 512;
        while (c < bytes) c <<= 1;
        return c;
    }
    const size_t g = (size_t)2 << 20;
    return (bytes + g - 1) / g * g;
}

void dm_trim_locked(int dev) {  // release every cached block of dev to the driver
    for (auto &e : g_dm_free[dev]) {
        g_dm_live.erase(e.second);
        (void)hipFree(e.second);
    }
    g_dm_free[dev].clear();
    g_dm_cached[dev] = 0;
}
}  // namespace

hipError_t dmalloc(void **p, size_t bytes) {
    *p = nullptr;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= DM_MAX_DEV) return hipMalloc(p, bytes);
    const size_t c = dm_class(bytes);
    std::lock_guard<std::mutex> lk(g_dm_mu);
    auto &fl = g_dm_free[dev];
    auto it = fl.lower_bound(c);
    if (it != fl.end() && it->first <= c + c / 4 + ((size_t)2 << 20)) {  // a cached block at most ~25 % larger
        *p = it->second;
        g_dm_cached[dev] -= it->first;
        fl.erase(it);
        return hipSuccess;
    }
    e = hipMalloc(p, c);
    if (e != hipSuccess) {  // out of memory: give the cache back to the driver and try once more
        (void)hipGetLastError();
        dm_trim_locked(dev);
        e = hipMalloc(p, c);
        if (e != hipSuccess) return e;
    }
    g_dm_live[*p] = {c, dev};
    return hipSuccess;
}

void dfree(void *p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_dm_mu);
    auto it = g_dm_live.find(p);
    if (it == g_dm_live.end()) {  // not ours (hipMalloc'd elsewhere): the driver's free
        (void)hipFree(p);
        return;
    }
    const Block b = it->second;
    if (g_dm_cached[b.dev] + b.bytes > DM_CAP) {
        g_dm_live.erase(it);
        (void)hipFree(p);
        return;
    }
    g_dm_free[b.dev].emplace(b.bytes, p);
    g_dm_cached[b.dev] += b.bytes;
}

void dfree_sync(void *p) {
    if (!p) return;
    (void)hipDeviceSynchronize();
    dfree(p);
}

// Streams and pinned count slots of the per-keyframe handles, reused the same way (a stream create / destroy pair and
// a small pinned allocation + free are further driver calls per keyframe).
namespace {
std::vector<hipStream_t> g_streams[DM_MAX_DEV];
std::vector<int *> g_slots;  // free 16-byte pinned slots
}  // namespace

hipError_t stream_get(hipStream_t *s) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    {
        std::lock_guard<std::mutex> lk(g_dm_mu);
        if (dev >= 0 && dev < DM_MAX_DEV && !g_streams[dev].empty()) {
            *s = g_streams[dev].back();
            g_streams[dev].pop_back();
            return hipSuccess;
        }
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

void stream_put(hipStream_t s) {
    if (!s) return;
    int dev = 0;
    if (hipStreamSynchronize(s) != hipSuccess || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= DM_MAX_DEV) {
        (void)hipStreamDestroy(s);
        return;
    }
    std::lock_guard<std::mutex> lk(g_dm_mu);
    if (g_streams[dev].size() >= 64) {
        (void)hipStreamDestroy(s);
        return;
    }
    g_streams[dev].push_back(s);
}

int *pinned_slot() {
    std::lock_guard<std::mutex> lk(g_dm_mu);
    if (g_slots.empty()) {  // one 64 KiB pinned page, carved into 4,096 slots (never returned)
        void *page = nullptr;
        if (hipHostMalloc(&page, 65536, hipHostMallocPortable) != hipSuccess) return nullptr;
        for (int i = 4095; i >= 0; i--) g_slots.push_back(reinterpret_cast<int *>(static_cast<char *>(page) + 16 * i));
    }
    int *p = g_slots.back();
    g_slots.pop_back();
    return p;
}

void pinned_slot_free(int *p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_dm_mu);
    g_slots.push_back(p);
}

}  // namespace tiler
